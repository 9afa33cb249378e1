"""Drop-in ``BayesianOptimizer`` for ``scripts/run_optimization.py``.

Constructor = the Bayesian7 superset signature (optimization/Bayesian7.py:202-218), so the reference driver
(scripts/run_optimization.py:116-130) constructs it unchanged and calls ``optimize()`` which returns
``(best_params[d] in physical units, best_value)`` (optimization/Bayesian7.py:729-733); the simulator duck type
``configure_geometry / run_simulation / cleanup`` (simulation/taichi.py:33,46,145) is driven unchanged.

What differs, by design: the surrogate is an exact GP on the gpx engine (fp64, one shared factorisation for the
8 outputs) instead of the batched SVGP; hyperparameters are fixed (MLL fitting: SURVEY §8f row 1).  Data flow,
CSV resume, transforms, evaluation metrics, pool-scan acquisition (variance score -> top-K -> farthest-point
sampling) and the objective/return contract follow Bayesian7.  ``acquisition="logei"|"ei"|"ucb"`` selects the
analytic improvement sweep of optimization/Bayesian.py:96-113 over a Sobol grid instead, and
``acquisition="qlogei"`` the reference's optimize_acqf on MC qLogEI (q = batch_size, L-BFGS-B restarts; acqf.py).

Surface mapping (north star fit()/predict()/acquire()):
  fit_gp_model()                 ≙ Bayesian7.fit_gp_model / Bayesian.fit_gp_model
  predict(x_orig) -> (n, 8)      ≙ Bayesian2.predict (posterior mean in physical units)
  acquire(k) -> Tensor[k, d]     ≙ Bayesian7 pool scan (:646-688) or Bayesian.optimize_acquisition_function
  optimize_acquisition_function  ≙ Bayesian.py:96-113 (returns q unit-cube candidates)
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from .engine import GPEngine, KernelParams
from .models import ExactGP
from .transforms import LogInputStandardizer, LogOutputStandardizer

OUTPUT_COLS = ["n", "eta", "sigma_y", "width", "height"]


@dataclass
class GPConfig:
    """Knobs of optimization/Bayesian7.py:30-76 that still apply, plus the fixed exact-GP hyperparameters."""

    candidates_pool_size: int = 10000     # Bayesian7.py:57
    acq_batch_size: int = 500             # Bayesian7.py:60
    acq_eval_batch_size: int = 2048       # kept for signature compatibility (the engine chunks internally)
    K_BIG_CAP: int = 8000                 # Bayesian7.py:66
    raw_samples: int = 1 << 14            # Sobol grid for the analytic improvement acquisitions
    kernel: str = "scale_linear_matern52" # Bayesian6.py:471-473 / Bayesian7.py:162-166
    lengthscale: float = 1.0
    outputscale: float = 1.0
    linear_variance: float = 0.1
    noise: float = 1e-3
    jitter_val: float = 1e-4              # Bayesian6.py GPConfig.jitter_val; retried at 1e-2 (:487)
    beta: float = 4.0
    # hyperparameters: learned each round like the reference's model fit (fit_gpytorch_mll, Bayesian.py:92-93;
    # the driven variant trains them by ELBO, Bayesian7.py:451-538) — here by exact marginal likelihood on the
    # GPU (mll.py), starting from the values above; False keeps them fixed
    fit_hyperparameters: bool = True
    prior_set: str = "none"               # "none" (ScaleKernel(Linear + Matern) of Bayesian6/7) | "dim_scaled" | "gamma"
    mll_options: Optional[dict] = None    # scipy L-BFGS-B options
    # acquisition="qlogei": optimize_acqf settings of optimization/Bayesian.py:100-112
    mc_samples: int = 512
    num_restarts: int = 10
    acqf_raw_samples: int = 1024
    batch_limit: int = 5
    maxiter: int = 200


class BayesianOptimizer:
    def __init__(
        self,
        simulator,
        bounds_list: Sequence[Sequence[float]],
        output_dir: str,
        n_initial_points: int,
        n_batches: int,
        batch_size: int,
        num_outputs: int = 8,
        svgp_threshold: int = 100,   # accepted for compatibility; the exact GP is used at every size
        resume: bool = False,
        target_total: Optional[int] = None,
        device: Optional[torch.device] = None,
        gp_config: Optional[GPConfig] = None,
        test_csv_path: Optional[str] = None,
        **kwargs,
    ):
        self.engine = kwargs.pop("engine", None)
        if self.engine is None:
            self.engine = GPEngine(device)  # HIP path; raises if libgpx.so / the GPU is missing
        self.gp_device = getattr(self.engine, "device", torch.device("cpu"))
        self.dtype = torch.float64
        self.config = gp_config or GPConfig()
        self.simulator = simulator
        self.physical_bounds = np.asarray(bounds_list, dtype=np.float64)  # (D, 2)
        self.dim = int(self.physical_bounds.shape[0])
        self.num_outputs = int(num_outputs)
        self.n_initial_points = int(n_initial_points)
        self.n_batches = int(n_batches)
        self.batch_size = int(batch_size)
        self.target_total = target_total
        self.resume = resume
        self.svgp_threshold = svgp_threshold
        self.objective_mode = str(kwargs.get("objective_mode", "min")).lower()
        self.objective_index = kwargs.get("objective_index", None)
        self.objective_weights = kwargs.get("objective_weights", None)
        self.acquisition = str(kwargs.get("acquisition", "variance")).lower()
        self.seed = kwargs.get("seed", None)
        self._rng = np.random.default_rng(self.seed)

        self.train_X = torch.empty((0, self.dim), dtype=self.dtype, device=self.gp_device)
        self.train_Y_raw = torch.empty((0, self.num_outputs), dtype=self.dtype, device=self.gp_device)
        self.test_X = None
        self.test_Y_raw = None
        self.gp_model: Optional[ExactGP] = None
        self.x_tf: Optional[LogInputStandardizer] = None
        self.y_tf: Optional[LogOutputStandardizer] = None
        self.iteration_counter = 0

        os.makedirs(output_dir, exist_ok=True)
        self.results_csv_path = os.path.join(output_dir, "optimization_results.csv")
        self.val_log_path = os.path.join(output_dir, "validation_log.csv")
        self.model_save_path = os.path.join(output_dir, "exact_gp.pt")
        self._init_data()
        if test_csv_path:
            self._load_test_set(test_csv_path)
        print(f"[BayesianOptimizer] Device: {self.gp_device} | exact GP (gpx) | outputs: {self.num_outputs}")

    # -- CSV init / resume (Bayesian7.py:268-293) --------------------------------------------------
    def _cols(self):
        return OUTPUT_COLS[: self.dim] + [f"x_{i:02d}" for i in range(1, self.num_outputs + 1)]

    def _init_data(self):
        cols = self._cols()
        if os.path.exists(self.results_csv_path) and self.resume:
            import pandas as pd

            print("[Resume] Loading existing CSV data...")
            try:
                df = pd.read_csv(self.results_csv_path)
                if not df.empty:
                    X_phys = df[cols[: self.dim]].to_numpy(dtype=np.float64)
                    Y_raw = df[cols[self.dim:]].to_numpy(dtype=np.float64)
                    b = self.physical_bounds
                    X_unit = (X_phys - b[:, 0]) / (b[:, 1] - b[:, 0])
                    self.train_X = torch.tensor(X_unit, dtype=self.dtype, device=self.gp_device)
                    self.train_Y_raw = torch.tensor(Y_raw, dtype=self.dtype, device=self.gp_device)
                    print(f"  -> Loaded {len(df)} samples.")
            except Exception as e:  # reference: print and continue fresh
                print(f"[Resume] Failed to load CSV: {e}")
        else:
            with open(self.results_csv_path, "w", encoding="utf-8") as f:
                f.write(",".join(cols) + "\n")
        if not os.path.exists(self.val_log_path):
            with open(self.val_log_path, "w", encoding="utf-8") as f:
                f.write("iteration,dataset,mse,mae,max_err,r2\n")

    def _load_test_set(self, path: str):
        if not os.path.exists(path):
            print(f"[Validation] Test CSV not found: {path}")
            return
        import pandas as pd

        df = pd.read_csv(path)
        cols = self._cols()
        df = df.dropna(subset=cols)
        b = self.physical_bounds
        X_unit = (df[cols[: self.dim]].to_numpy(dtype=np.float64) - b[:, 0]) / (b[:, 1] - b[:, 0])
        self.test_X = torch.tensor(X_unit, dtype=self.dtype, device=self.gp_device)
        self.test_Y_raw = torch.tensor(df[cols[self.dim:]].to_numpy(dtype=np.float64), dtype=self.dtype,
                                       device=self.gp_device)

    def _save_row(self, x_phys: np.ndarray, y_vals: np.ndarray):
        row = np.concatenate([x_phys, y_vals])
        with open(self.results_csv_path, "a", encoding="utf-8") as f:
            f.write(",".join([f"{v:.8f}" for v in row]) + "\n")

    # -- simulation wrapper (Bayesian7.py:330-352) --------------------------------------------------
    def run_simulation(self, params) -> Optional[np.ndarray]:
        x_unit = params.detach().cpu().numpy().flatten() if isinstance(params, torch.Tensor) else \
            np.asarray(params).flatten()
        b = self.physical_bounds
        x_phys = b[:, 0] + x_unit * (b[:, 1] - b[:, 0])
        try:
            self.simulator.configure_geometry(float(x_phys[3]), float(x_phys[4]))
            disp = self.simulator.run_simulation(float(x_phys[0]), float(x_phys[1]), float(x_phys[2]))
            if disp is None:
                return None
            disp = np.array(disp, dtype=np.float64).flatten()
            if len(disp) < self.num_outputs:
                disp = np.pad(disp, (0, self.num_outputs - len(disp)))
            return disp[: self.num_outputs]
        except Exception:
            return None

    def _scaled_to_original(self, x_unit: torch.Tensor) -> np.ndarray:
        b = self.physical_bounds
        return x_unit.detach().cpu().numpy().flatten() * (b[:, 1] - b[:, 0]) + b[:, 0]

    # -- model ---------------------------------------------------------------------------------------
    def _bounds_t(self):
        return torch.tensor(self.physical_bounds.T, dtype=self.dtype, device=self.gp_device)

    def _kernel_params(self) -> KernelParams:
        c = self.config
        return KernelParams(c.kernel, c.lengthscale, outputscale=c.outputscale, noise=c.noise,
                            linear_variance=c.linear_variance)

    def fit_gp_model(self):
        """Transforms (Bayesian7.py:363-385) + one exact posterior update on the engine for all outputs."""
        if self.train_X.shape[0] < 1:
            raise RuntimeError("Need at least one observation.")
        self.x_tf = LogInputStandardizer(self._bounds_t()).fit(self.train_X)
        self.y_tf = LogOutputStandardizer().fit(self.train_Y_raw)
        Xs = self.x_tf(self.train_X)
        Ys = self.y_tf(self.train_Y_raw)
        self.gp_model = ExactGP(Xs, Ys, self._kernel_params(), engine=self.engine,
                                jitter_schedule=(0.0, self.config.jitter_val, 1e-2))
        if self.config.fit_hyperparameters:
            self.gp_model.fit_hyperparameters(self.config.prior_set, options=self.config.mll_options)
        else:
            self.gp_model.fit()
        return self.gp_model

    def predict(self, x_orig_numpy: np.ndarray, return_var: bool = False):
        """Posterior mean of the outputs at physical-unit inputs (Bayesian2.predict, :146-174)."""
        if self.gp_model is None:
            self.fit_gp_model()
        x = torch.as_tensor(np.atleast_2d(np.asarray(x_orig_numpy, dtype=np.float64)), device=self.gp_device)
        x_unit = (x - self._bounds_t()[0]) / (self._bounds_t()[1] - self._bounds_t()[0])
        post = self.gp_model.posterior(self.x_tf(x_unit))
        y = self.y_tf.inverse_mean(post.mean)
        if return_var:
            return y.cpu().numpy(), post.variance.cpu().numpy()
        return y.cpu().numpy()

    def evaluate_model(self, X_unit: torch.Tensor, Y_true_raw: torch.Tensor, dataset_name: str = "Vali"):
        """R2 / MSE / MAE / MaxErr per output, appended to validation_log.csv (Bayesian7.py:543-592)."""
        if self.gp_model is None or X_unit is None or len(X_unit) == 0:
            return None
        post = self.gp_model.posterior(self.x_tf(X_unit))
        yp = self.y_tf.inverse_mean(post.mean).cpu().numpy()
        yt = Y_true_raw.cpu().numpy()
        rows = []
        for i in range(self.num_outputs):
            var = np.var(yt[:, i])
            ss_res = float(((yt[:, i] - yp[:, i]) ** 2).sum())
            r2 = 1.0 - ss_res / (var * len(yt)) if var > 1e-9 else 0.0
            err = np.abs(yt[:, i] - yp[:, i])
            rows.append((r2, float((err ** 2).mean()), float(err.mean()), float(err.max())))
        arr = np.array(rows)
        print(f"--- {dataset_name} Performance: mean R2={arr[:, 0].mean():.4f} MSE={arr[:, 1].mean():.4g}")
        with open(self.val_log_path, "a", encoding="utf-8") as f:
            f.write(f"{len(self.train_X)},{dataset_name},{arr[:, 1].mean():.6f},{arr[:, 2].mean():.6f},"
                    f"{arr[:, 3].max():.6f},{arr[:, 0].mean():.4f}\n")
        return arr

    # -- acquisition -----------------------------------------------------------------------------
    def _lhs(self, n: int) -> np.ndarray:
        from scipy.stats import qmc

        return qmc.LatinHypercube(d=self.dim, seed=self._rng).random(n=n)

    def _sobol(self, n: int) -> np.ndarray:
        from scipy.stats import qmc

        return qmc.Sobol(self.dim, scramble=True, seed=self._rng).random_base2(int(math.ceil(math.log2(max(n, 2)))))[:n]

    def _objective_alpha(self):
        """alpha and (y_mean, y_scale) of the scalar objective in the log-standardised space: one output
        (objective_index) or output 0."""
        t = int(self.objective_index) if self.objective_index is not None else 0
        return t

    def acquire(self, k: int) -> torch.Tensor:
        """Select k unit-cube points.  variance mode: pool scan -> top-K_big -> FPS (Bayesian7.py:646-688);
        improvement modes: analytic sweep over a Sobol grid, best k distinct scores (Bayesian.py:96-113)."""
        gp = self.gp_model
        if self.acquisition == "variance":
            pool = torch.tensor(self._lhs(self.config.candidates_pool_size), dtype=self.dtype, device=self.gp_device)
            _, _, scores = gp.engine.acquire(gp.state, self.x_tf(pool), "variance", return_scores=True)
            k_big = int(min(max(5000, 20 * k), self.config.K_BIG_CAP, self.config.candidates_pool_size))
            k_big = max(min(k_big, pool.shape[0]), k)
            _, idx_big = torch.topk(scores, k_big)
            return farthest_point_sampling(pool[idx_big], k, self._rng)
        if self.acquisition == "qlogei":
            return self._acquire_qlogei(k)
        grid = torch.tensor(self._sobol(self.config.raw_samples), dtype=self.dtype, device=self.gp_device)
        t = self._objective_alpha()
        # maximise the objective in log-standardised space; "min" mode flips the sign of the incumbent search
        Ys = self.y_tf(self.train_Y_raw)[:, t]
        sign = 1.0 if self.objective_mode == "max" else -1.0
        alpha = sign * gp.state.alpha[:, t]
        best_f = float((sign * Ys).max())
        _, _, scores = gp.engine.acquire(gp.state, self.x_tf(grid), self.acquisition, best_f=best_f,
                                         beta=self.config.beta, alpha=alpha, return_scores=True)
        k = min(k, grid.shape[0])
        _, idx = torch.topk(scores, k)
        return grid[idx]

    def _acquire_qlogei(self, k: int) -> torch.Tensor:
        """optimize_acqf on MC qLogEI with q = k jointly (optimization/Bayesian.py:96-113: 512 Sobol base samples,
        num_restarts 10, raw_samples 1024, batch_limit 5, maxiter 200), through the log-input transform, in the
        log-standardised output space (acqf.py)."""
        from .acqf import LinearMCObjective, SobolQMCNormalSampler, optimize_acqf, qLogExpectedImprovement

        gp = self.gp_model
        t = self._objective_alpha()
        sign = 1.0 if self.objective_mode == "max" else -1.0
        Ys = self.y_tf(self.train_Y_raw)[:, t]
        w = [0.0] * gp.num_outputs
        w[t] = sign
        seed = int(self._rng.integers(0, 1 << 30))
        acq = qLogExpectedImprovement(gp, best_f=float((sign * Ys).max()),
                                      sampler=SobolQMCNormalSampler(torch.Size([self.config.mc_samples]), seed),
                                      objective=LinearMCObjective(w))
        x_tf = self.x_tf

        class _OnUnitCube:  # the GP sees transformed inputs; optimize_acqf works in the unit cube
            model = gp

            def __call__(self, X):
                return acq(x_tf(X.reshape(-1, X.shape[-1])).reshape(X.shape))

        bounds = torch.stack([torch.zeros(self.dim), torch.ones(self.dim)]).to(self.dtype)
        cand, _ = optimize_acqf(_OnUnitCube(), bounds, q=k, num_restarts=self.config.num_restarts,
                                raw_samples=self.config.acqf_raw_samples,
                                options={"batch_limit": self.config.batch_limit, "maxiter": self.config.maxiter},
                                seed=seed)
        return cand.detach()

    def optimize_acquisition_function(self, gp=None) -> torch.Tensor:
        return self.acquire(self.batch_size)

    # -- objective / main loop (Bayesian7.py:597-733) ---------------------------------------------
    def _compute_objective(self, Y_raw: torch.Tensor) -> torch.Tensor:
        if Y_raw is None or Y_raw.numel() == 0:
            return torch.empty((0,), device=self.gp_device, dtype=self.dtype)
        if self.objective_weights is not None:
            w = torch.tensor(self.objective_weights, device=Y_raw.device, dtype=Y_raw.dtype).view(1, -1)
            return (Y_raw * w).sum(dim=1)
        if self.objective_index is not None:
            return Y_raw[:, int(self.objective_index)]
        return Y_raw.sum(dim=1)

    def _append(self, x_u: torch.Tensor, disp: np.ndarray):
        self.train_X = torch.cat([self.train_X, x_u.reshape(1, -1).to(self.train_X)])
        self.train_Y_raw = torch.cat([self.train_Y_raw, torch.tensor(disp, device=self.gp_device,
                                                                     dtype=self.dtype).reshape(1, -1)])
        self._save_row(self._scaled_to_original(x_u), disp)

    def optimize(self):
        assert self.target_total is not None, "target_total must be provided (e.g., 100000)"
        print("[BayesianOptimizer] Starting optimization...")
        if self.train_X.shape[0] < self.n_initial_points:
            print(f"[Init] Collecting {self.n_initial_points} LHS points...")
            for s in self._lhs(self.n_initial_points - self.train_X.shape[0]):
                x_u = torch.tensor(s, dtype=self.dtype, device=self.gp_device)
                disp = self.run_simulation(x_u)
                if disp is not None:
                    self._append(x_u, disp)
        while len(self.train_X) < self.target_total:
            self.iteration_counter += 1
            print(f"\n=== Iteration: {len(self.train_X)} samples ===")
            self.fit_gp_model()
            self.evaluate_model(self.train_X, self.train_Y_raw, "Train_Set")
            if self.test_X is not None:
                self.evaluate_model(self.test_X, self.test_Y_raw, "Test_Set")
            batch_k = min(self.config.acq_batch_size, self.batch_size, self.target_total - len(self.train_X))
            batch_X = self.acquire(batch_k)
            print(f"[Acquisition] Selected {len(batch_X)} points ({self.acquisition}).")
            new_cnt = 0
            for x_u in batch_X:
                disp = self.run_simulation(x_u)
                if disp is not None:
                    self._append(x_u, disp)
                    new_cnt += 1
            if new_cnt == 0:
                print("[Stop] No valid simulations returned in this batch.")
                break
            try:
                torch.save({"X": self.train_X.cpu(), "Y": self.train_Y_raw.cpu(),
                            "kernel": self._kernel_params().__dict__}, self.model_save_path)
            except Exception:
                pass
        print("[Done] Optimization finished.")
        if self.train_X.shape[0] == 0:
            return None, None
        obj = self._compute_objective(self.train_Y_raw)
        best_idx = int(torch.argmax(obj).item()) if self.objective_mode == "max" else int(torch.argmin(obj).item())
        return self._scaled_to_original(self.train_X[best_idx]), float(obj[best_idx].item())


def farthest_point_sampling(X: torch.Tensor, m: int, rng: Optional[np.random.Generator] = None) -> torch.Tensor:
    """Greedy farthest-point sampling (Bayesian7.py:82-106) on the tensor's device, one sync at the end."""
    n = X.shape[0]
    if m >= n:
        return X
    rng = rng or np.random.default_rng()
    idx = torch.empty(m, dtype=torch.long, device=X.device)
    first = int(rng.integers(0, n))
    idx[0] = first
    dists = torch.linalg.vector_norm(X - X[first], dim=1)
    for t in range(1, m):
        nxt = torch.argmax(dists)
        idx[t] = nxt
        dists = torch.minimum(dists, torch.linalg.vector_norm(X - X[nxt], dim=1))
    return X[idx]
