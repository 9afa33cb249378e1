"""Drop-in ``BayesianOptimizer`` for ``scripts/run_optimization.py``.

The contract with the reference's caller is kept exactly; everything behind it is this package's own design:

* constructor — the Bayesian7 superset signature (``optimization/Bayesian7.py:202-218``), so
  ``scripts/run_optimization.py:116-130`` builds it unchanged; ``optimize()`` returns ``(best_params[d] in physical
  units, best_value)`` (``Bayesian7.py:729-733``); the simulator duck type ``configure_geometry / run_simulation /
  cleanup`` (``simulation/taichi.py:33,46,145``) is driven unchanged;
* persistence — the results CSV is the run's source of truth: same columns (``n,eta,sigma_y,width,height,x_01..``),
  same ``%.8f`` rows, resume by reloading it (``Bayesian7.py:268-318``); metrics go to ``validation_log.csv``.

Behind it: the surrogate is an exact GP on the gpx engine (fp64) instead of the batched SVGP.  Its hyperparameters are
fitted by exact marginal likelihood on the GPU each round (mll.py) — one set PER OUTPUT, the reference's multi-output
SingleTaskGP (optimization/Bayesian1.py:108-116; ``GPConfig.independent_outputs``), the 8 outputs fitted in one batched
call — or held fixed and shared by the outputs (one factorisation with 8 right-hand sides, exact when the
hyperparameters are tied), in which case new observations are folded in by the bordered Cholesky
(``ExactGP.append_observations``) instead of a refit.  Acquisition modes (``acquisition=``):

* ``"variance"`` (default, Bayesian7's pool scan ``:646-688``): Latin-hypercube pool -> summed posterior variance on
  the device -> top-K on the device (``gpx_topk_f64``, deterministic ties) -> farthest-point sampling on the device
  (``gpx_fps_f64``) from a random start, as the reference's ``farthest_point_sampling`` (``:82-106``);
* ``"logei" | "ei" | "ucb"`` (the analytic forms of ``optimization/Bayesian.py:96-113``'s qLogEI at q = 1): a
  scrambled-Sobol grid scored on the device, best k by ``gpx_topk_f64``;
* ``"qlogei"`` (``Bayesian.py:100-112``): ``optimize_acqf`` on MC qLogEI; batches larger than the engine's joint
  q-batch limit (``GPX_MAX_Q``) are built greedily in chunks, each chunk conditioned on the ones before it with their
  posterior means as fantasy observations (kriging believer).

The scalar objective the improvement modes maximise is the one ``optimize()`` reports (``_scalar_objective``,
``Bayesian7.py:597-609``): the weighted sum (``objective_weights``), one output (``objective_index``) or the sum of
all outputs, negated in ``objective_mode="min"``.  The GP models log-standardised outputs (``Bayesian7.py:371-383``),
so the acquisition scores that linear combination of the modelled outputs.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _capi
from .engine import GPEngine, KernelParams
from .models import ExactGP, reference_jitter_schedule
from .transforms import LogInputStandardizer, LogOutputStandardizer

INPUT_COLUMNS = ("n", "eta", "sigma_y", "width", "height")  # simulator parameters, config/config.py order


@dataclass
class GPConfig:
    """Knobs of ``optimization/Bayesian7.py:30-76`` that still apply, plus the exact-GP hyperparameters."""

    candidates_pool_size: int = 10000     # Bayesian7.py:57
    acq_batch_size: int = 500             # Bayesian7.py:60
    acq_eval_batch_size: int = 2048       # accepted for signature compatibility (the engine chunks internally)
    K_BIG_CAP: int = 8000                 # Bayesian7.py:66
    raw_samples: int = 1 << 14            # Sobol grid of the analytic improvement modes
    kernel: str = "scale_linear_matern52" # Bayesian6.py:471-473 / Bayesian7.py:162-166
    lengthscale: float = 1.0
    outputscale: float = 1.0
    linear_variance: float = 0.1
    noise: float = 1e-3
    jitter_val: float = 1e-4              # Bayesian6.py GPConfig.jitter_val; retried at 1e-2 (:487)
    beta: float = 4.0
    # exact marginal likelihood each round (fit_gpytorch_mll, Bayesian.py:92-93; the driven variant trains by ELBO,
    # Bayesian7.py:451-538); False keeps the values above
    fit_hyperparameters: bool = True
    # with fit_hyperparameters: one hyperparameter set per output (lengthscales, outputscale, noise, constant mean), as
    # BoTorch's multi-output SingleTaskGP fits them (Bayesian1.py:108-116 [upstream]); False: one set shared by all
    independent_outputs: bool = True
    prior_set: str = "none"               # "none" (ScaleKernel(Linear + Matern) of Bayesian6/7) | "dim_scaled" | "gamma"
    mll_options: Optional[dict] = None    # scipy L-BFGS-B options
    # with fixed hyperparameters: freeze the input standardisation at the first fit and fold each round's new rows in
    # with the O(n^2 q) bordered update (gpx_append_f64) instead of refitting (Bayesian7.py:639 refits every round)
    incremental_updates: bool = True
    # Opt-in large-n policy (off by default: every round is then a full exact refit over all n points, whatever n, as
    # the reference refits its surrogate every round, Bayesian7.py:639; its svgp_threshold is accepted for
    # compatibility, Bayesian7.py:207).  With large_n_policy=True, above svgp_threshold training points (where
    # Bayesian6 switches to SVGP: optimization/Bayesian6.py:589-596, scripts/run_optimization.py:40) the drop-in keeps
    # the EXACT posterior over all points but stops paying O(n^3) per round: hyperparameters are fitted by marginal
    # likelihood on a random subsample of svgp_threshold points (drawn from an RNG of its own, so the candidate draws
    # of the run are unchanged) and then held, and each round's new rows are folded in by the bordered update
    # (O(n^2 q)).  The factor is rebuilt (and the hyperparameters refitted on a fresh subsample) whenever n has grown by
    # large_n_refit_growth since the last rebuild, or would outgrow the factor's reserved capacity.
    large_n_policy: bool = False
    large_n_refit_growth: float = 2.0
    # device memory the exact factor may take (L and W = L^{-T}: 2 n^2 doubles at capacity), as a fraction of the free
    # device memory at the rebuild; beyond it the run stops with a clear error instead of an allocator failure
    large_n_memory_fraction: float = 0.85
    # acquisition="qlogei": optimize_acqf settings of optimization/Bayesian.py:100-112
    mc_samples: int = 512
    num_restarts: int = 10
    acqf_raw_samples: int = 1024
    batch_limit: int = 5
    maxiter: int = 200


# ---- persistence -----------------------------------------------------------------------------------------------
class _ResultsTable:
    """results CSV (source of truth for resume) + validation log, in the reference's file formats."""

    def __init__(self, directory: str, dim: int, num_outputs: int):
        os.makedirs(directory, exist_ok=True)
        self.path = os.path.join(directory, "optimization_results.csv")
        self.metrics_path = os.path.join(directory, "validation_log.csv")
        self.inputs = list(INPUT_COLUMNS[:dim])
        self.outputs = [f"x_{k:02d}" for k in range(1, num_outputs + 1)]

    @property
    def columns(self) -> List[str]:
        return self.inputs + self.outputs

    def open(self, resume: bool) -> Optional[Tuple[np.ndarray, np.ndarray]]:
        """Resume: the (X_phys, Y) rows already recorded, or None.  Fresh run: a new file with the header."""
        rows = None
        if resume and os.path.exists(self.path):
            print(f"[resume] reading {self.path}")
            try:
                import pandas as pd

                table = pd.read_csv(self.path)
                if len(table):
                    rows = (table[self.inputs].to_numpy(np.float64), table[self.outputs].to_numpy(np.float64))
                    print(f"[resume] {len(table)} evaluations restored")
            except Exception as err:  # a damaged file does not stop the run: start from what the model has
                print(f"[resume] could not parse {self.path}: {err}")
        else:
            with open(self.path, "w", encoding="utf-8") as fh:
                fh.write(",".join(self.columns) + "\n")
        if not os.path.exists(self.metrics_path):
            with open(self.metrics_path, "w", encoding="utf-8") as fh:
                fh.write("iteration,dataset,mse,mae,max_err,r2\n")
        return rows

    def record(self, x_phys: np.ndarray, y: np.ndarray) -> None:
        values = np.concatenate([np.asarray(x_phys, np.float64).ravel(), np.asarray(y, np.float64).ravel()])
        with open(self.path, "a", encoding="utf-8") as fh:
            fh.write(",".join("%.8f" % v for v in values) + "\n")

    def record_metrics(self, n_train: int, name: str, per_output: np.ndarray) -> None:
        r2, mse, mae, worst = per_output[:, 0], per_output[:, 1], per_output[:, 2], per_output[:, 3]
        with open(self.metrics_path, "a", encoding="utf-8") as fh:
            fh.write(f"{n_train},{name},{mse.mean():.6f},{mae.mean():.6f},{worst.max():.6f},{r2.mean():.4f}\n")

    def read_validation(self, path: str) -> Optional[Tuple[np.ndarray, np.ndarray]]:
        if not os.path.exists(path):
            print(f"[validation] no test set at {path}")
            return None
        import pandas as pd

        table = pd.read_csv(path).dropna(subset=self.columns)
        return table[self.inputs].to_numpy(np.float64), table[self.outputs].to_numpy(np.float64)


# ---- optimizer --------------------------------------------------------------------------------------------------
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
        svgp_threshold: int = 3000,  # run_optimization.py:40's value; GPConfig.large_n_policy (opt-in) above it
        resume: bool = False,
        target_total: Optional[int] = None,
        device: Optional[torch.device] = None,
        gp_config: Optional[GPConfig] = None,
        test_csv_path: Optional[str] = None,
        **kwargs,
    ):
        engine = kwargs.pop("engine", None)
        self.engine = engine if engine is not None else GPEngine(device)  # HIP path: raises without libgpx / a GPU
        self.gp_device = getattr(self.engine, "device", torch.device("cpu"))
        self.dtype = torch.float64
        self.config = gp_config or GPConfig()
        self.simulator = simulator
        box = np.asarray(bounds_list, dtype=np.float64)
        self.physical_bounds = box
        self._lo, self._span = box[:, 0], box[:, 1] - box[:, 0]
        self.dim = box.shape[0]
        self.num_outputs = int(num_outputs)
        self.n_initial_points, self.n_batches, self.batch_size = int(n_initial_points), int(n_batches), int(batch_size)
        self.target_total, self.resume, self.svgp_threshold = target_total, resume, svgp_threshold
        self.objective_mode = str(kwargs.get("objective_mode", "min")).lower()
        self.objective_index = kwargs.get("objective_index", None)
        self.objective_weights = kwargs.get("objective_weights", None)
        self.acquisition = str(kwargs.get("acquisition", "variance")).lower()
        if self.acquisition not in ("variance", "logei", "ei", "ucb", "qlogei"):
            raise ValueError(f"unknown acquisition '{self.acquisition}'")
        self.seed = kwargs.get("seed", None)
        self._rng = np.random.default_rng(self.seed)
        # the large-n policy's hyperparameter subsamples draw from their own stream (never shift the candidate draws)
        self._subsample_rng = np.random.default_rng(None if self.seed is None else [int(self.seed), 1])

        self.table = _ResultsTable(output_dir, self.dim, self.num_outputs)
        self.results_csv_path, self.val_log_path = self.table.path, self.table.metrics_path
        self.model_save_path = os.path.join(output_dir, "exact_gp.pt")
        self.train_X = torch.empty((0, self.dim), dtype=self.dtype, device=self.gp_device)
        self.train_Y_raw = torch.empty((0, self.num_outputs), dtype=self.dtype, device=self.gp_device)
        restored = self.table.open(resume)
        if restored is not None:
            self.train_X = self._tensor(self._to_unit(restored[0]))
            self.train_Y_raw = self._tensor(restored[1])
        self.test_X = self.test_Y_raw = None
        if test_csv_path:
            held_out = self.table.read_validation(test_csv_path)
            if held_out is not None:
                self.test_X, self.test_Y_raw = self._tensor(self._to_unit(held_out[0])), self._tensor(held_out[1])
        self.gp_model: Optional[ExactGP] = None
        self._large_n_base: Optional[int] = None  # n at the last large-n rebuild
        self.x_tf: Optional[LogInputStandardizer] = None
        self.y_tf: Optional[LogOutputStandardizer] = None
        self.iteration_counter = 0
        print(f"[gpx] exact-GP surrogate on {self.gp_device}, {self.num_outputs} outputs, acquisition={self.acquisition}")

    # -- units ---------------------------------------------------------------------------------------------------
    def _tensor(self, a) -> torch.Tensor:
        return torch.as_tensor(np.asarray(a, dtype=np.float64), device=self.gp_device)

    def _to_unit(self, x_phys: np.ndarray) -> np.ndarray:
        return (np.asarray(x_phys, np.float64) - self._lo) / self._span

    def _scaled_to_original(self, x_unit) -> np.ndarray:
        u = x_unit.detach().cpu().numpy() if isinstance(x_unit, torch.Tensor) else np.asarray(x_unit)
        return self._lo + u.reshape(-1).astype(np.float64) * self._span

    def _bounds_t(self) -> torch.Tensor:
        return self._tensor(self.physical_bounds.T)

    # -- black-box evaluation ------------------------------------------------------------------------------------
    def run_simulation(self, params) -> Optional[np.ndarray]:
        """One simulator call at a unit-cube point; any failure (exception, None, out-of-range geometry) -> None, like
        the reference's wrapper (Bayesian7.py:330-352).  Width/height are the last two physical parameters."""
        x = self._scaled_to_original(params)
        try:
            self.simulator.configure_geometry(float(x[3]), float(x[4]))
            out = self.simulator.run_simulation(float(x[0]), float(x[1]), float(x[2]))
        except Exception:
            return None
        if out is None:
            return None
        out = np.asarray(out, dtype=np.float64).ravel()[: self.num_outputs]
        return np.pad(out, (0, self.num_outputs - out.size))

    def _observe(self, x_unit: torch.Tensor) -> bool:
        y = self.run_simulation(x_unit)
        if y is None:
            return False
        self.train_X = torch.cat([self.train_X, x_unit.reshape(1, -1).to(self.train_X)])
        self.train_Y_raw = torch.cat([self.train_Y_raw, self._tensor(y).reshape(1, -1)])
        self.table.record(self._scaled_to_original(x_unit), y)
        return True

    # -- surrogate -----------------------------------------------------------------------------------------------
    def _kernel_params(self) -> KernelParams:
        c = self.config
        return KernelParams(c.kernel, c.lengthscale, outputscale=c.outputscale, noise=c.noise,
                            linear_variance=c.linear_variance)

    def fit_gp_model(self):
        """Log-standardise (Bayesian7.py:363-385) and build the exact posterior for all outputs on the engine.

        A fresh fit each round (hyperparameters by marginal likelihood, or fixed), or - fixed hyperparameters,
        incremental mode - the previous round's factor extended by the rows observed since.  With
        GPConfig.large_n_policy and n > svgp_threshold (the reference's SVGP switch, Bayesian6.py:589): the large-n
        policy (GPConfig)."""
        n = self.train_X.shape[0]
        if n < 1:
            raise RuntimeError("fit_gp_model needs at least one observation")
        cfg = self.config
        self.y_tf = LogOutputStandardizer().fit(self.train_Y_raw)
        Ys = self.y_tf(self.train_Y_raw)
        if cfg.large_n_policy and n > self.svgp_threshold:
            return self._fit_large_n(n, Ys)
        self._large_n_base = None
        grow = (not cfg.fit_hyperparameters and cfg.incremental_updates and self.gp_model is not None
                and self.x_tf is not None and self.gp_model.train_X.shape[0] < n)
        if grow:
            n_old = self.gp_model.train_X.shape[0]
            self.gp_model.train_Y = Ys[:n_old]  # re-standardised targets; alpha is recomputed from all of them
            self.gp_model.append_observations(self.x_tf(self.train_X[n_old:]), Ys[n_old:])
            return self.gp_model
        self.gp_model = None  # the previous round's factor is released before the next one is allocated
        self._check_device_budget(n, n)
        self.x_tf = LogInputStandardizer(self._bounds_t()).fit(self.train_X)
        self.gp_model = ExactGP(self.x_tf(self.train_X), Ys, self._kernel_params(), engine=self.engine,
                                jitter_schedule=reference_jitter_schedule(cfg.jitter_val),
                                independent_outputs=cfg.fit_hyperparameters and cfg.independent_outputs)
        if cfg.fit_hyperparameters:
            self.gp_model.fit_hyperparameters(cfg.prior_set, options=cfg.mll_options)
        else:
            self.gp_model.fit()
        return self.gp_model

    def exact_gp_bytes(self, n: int) -> int:
        """Device bytes of the exact posterior at n training points: L and W = L^{-T} (2 padded n^2 doubles; the
        posterior sweep needs W) plus the diagonal-block inverses.  n = 100,000 (main.py:13's --evals): 160 GB, inside
        one MI355X's 288 GB; the sweep's K* chunk (<= 1 GiB) and the small vectors come on top."""
        npad = -(-int(n) // _capi.GPX_TILE) * _capi.GPX_TILE
        return 2 * npad * npad * 8 + 2 * npad * 64 * 8

    def _free_device_bytes(self) -> Optional[int]:
        """Device memory a new factor can take: the driver's free memory plus what torch's caching allocator holds
        unused (a factor released just before is still reserved there), or None off the GPU.  The cache is counted, not
        emptied: releasing it every round would send the next fit's temporaries back through hipMalloc."""
        if not (torch.cuda.is_available() and getattr(self.gp_device, "type", "cpu") == "cuda"):
            return None
        free = torch.cuda.mem_get_info(self.gp_device)[0]
        return int(free + torch.cuda.memory_reserved(self.gp_device) - torch.cuda.memory_allocated(self.gp_device))

    def _check_device_budget(self, n: int, cap: int) -> int:
        """The capacity (>= n) an exact factor can reserve within GPConfig.large_n_memory_fraction of the free device
        memory; MemoryError naming the numbers when even n does not fit."""
        free = self._free_device_bytes()
        if free is None:
            return cap
        budget = self.config.large_n_memory_fraction * free
        while cap > n and self.exact_gp_bytes(cap) > budget:
            cap = max(n, int(0.9 * cap))
        if self.exact_gp_bytes(cap) > budget:
            raise MemoryError(f"exact GP at n={n} needs {self.exact_gp_bytes(n) / 1e9:.1f} GB of device memory, "
                              f"{budget / 1e9:.1f} GB available (GPConfig.large_n_memory_fraction)")
        return cap

    def _fit_large_n(self, n: int, Ys: torch.Tensor):
        """n > svgp_threshold: exact posterior over all n points with hyperparameters from a subsample fit, new rows
        folded in by the bordered update between rebuilds (GPConfig.large_n_refit_growth)."""
        cfg = self.config
        gp = self.gp_model
        # rebuild when n has grown by large_n_refit_growth, or would outgrow the reserved capacity (the bordered update
        # would otherwise grow the buffers outside the memory budget, GPEngine.append)
        rebuild = (gp is None or self._large_n_base is None or self.x_tf is None
                   or n >= cfg.large_n_refit_growth * self._large_n_base or gp.train_X.shape[0] > n
                   or n > max(gp.capacity, gp.train_X.shape[0]))
        if not rebuild:
            n_old = gp.train_X.shape[0]
            if n_old < n:
                gp.train_Y = Ys[:n_old]
                gp.append_observations(self.x_tf(self.train_X[n_old:]), Ys[n_old:])
            return gp
        params = gp.params if gp is not None else self._kernel_params()
        self.gp_model = gp = None  # release the previous factor (2 n^2 doubles) before the rebuild allocates
        # room for the rows still to come, within the device memory budget
        cap = n if self.target_total is None else max(n, min(int(self.target_total), int(cfg.large_n_refit_growth * n)))
        cap = self._check_device_budget(n, cap)
        self.x_tf = LogInputStandardizer(self._bounds_t()).fit(self.train_X)
        Xs = self.x_tf(self.train_X)
        jit = reference_jitter_schedule(cfg.jitter_val)
        if cfg.fit_hyperparameters:
            m = int(self.svgp_threshold)
            sub = np.sort(self._subsample_rng.choice(n, size=m, replace=False))
            sub_t = torch.as_tensor(sub, device=Xs.device)
            sub_gp = ExactGP(Xs[sub_t], Ys[sub_t], params, engine=self.engine, jitter_schedule=jit,
                             independent_outputs=cfg.independent_outputs or not isinstance(params, KernelParams))
            sub_gp.fit_hyperparameters(cfg.prior_set, options=cfg.mll_options)
            params = sub_gp.params
            del sub_gp
            print(f"[gpx] n={n} > svgp_threshold={self.svgp_threshold}: hyperparameters from a {m}-point subsample")
        self.gp_model = ExactGP(Xs, Ys, params, engine=self.engine, jitter_schedule=jit, capacity=cap).fit()
        self._large_n_base = n
        return self.gp_model

    def predict(self, x_orig_numpy: np.ndarray, return_var: bool = False):
        """Posterior mean of every output at physical-unit inputs, in physical units (Bayesian2.predict, :146-174)."""
        if self.gp_model is None:
            self.fit_gp_model()
        x_unit = self._tensor(self._to_unit(np.atleast_2d(np.asarray(x_orig_numpy, np.float64))))
        post = self.gp_model.posterior(self.x_tf(x_unit))
        mean = self.y_tf.inverse_mean(post.mean).cpu().numpy()
        return (mean, post.variance.cpu().numpy()) if return_var else mean

    def evaluate_model(self, X_unit: torch.Tensor, Y_true_raw: torch.Tensor, dataset_name: str = "Vali"):
        """Per-output R2 / MSE / MAE / max error of the posterior mean (Bayesian7.py:543-592 reports the same four),
        logged to validation_log.csv; returns the (T, 4) array."""
        if self.gp_model is None or X_unit is None or len(X_unit) == 0:
            return None
        truth = Y_true_raw.cpu().numpy()
        pred = self.y_tf.inverse_mean(self.gp_model.posterior(self.x_tf(X_unit)).mean).cpu().numpy()
        resid = truth - pred
        centred = truth - truth.mean(axis=0)
        ss_tot = (centred ** 2).sum(axis=0)
        r2 = np.where(ss_tot > 1e-9 * len(truth), 1.0 - (resid ** 2).sum(axis=0) / np.maximum(ss_tot, 1e-300), 0.0)
        table = np.stack([r2, (resid ** 2).mean(axis=0), np.abs(resid).mean(axis=0), np.abs(resid).max(axis=0)], 1)
        print(f"[{dataset_name}] n={len(truth)}  R2 {table[:, 0].mean():.4f}  MSE {table[:, 1].mean():.4g}")
        if table[:, 0].mean() < 0.85 and dataset_name.lower().startswith("train"):
            print(f"[{dataset_name}] low training R2: the surrogate underfits (check noise level / hyperparameters)")
        self.table.record_metrics(len(self.train_X), dataset_name, table)
        return table

    # -- objective -----------------------------------------------------------------------------------------------
    def _scalar_objective(self, Y_raw: torch.Tensor) -> torch.Tensor:
        """What optimize() ranks observations by (Bayesian7.py:597-609)."""
        if Y_raw is None or Y_raw.numel() == 0:
            return torch.empty((0,), device=self.gp_device, dtype=self.dtype)
        return Y_raw @ self._objective_weights(Y_raw)

    _compute_objective = _scalar_objective  # the reference's name

    def _objective_weights(self, like: Optional[torch.Tensor] = None) -> torch.Tensor:
        T = self.num_outputs
        if self.objective_weights is not None:
            w = torch.as_tensor(self.objective_weights, dtype=torch.float64).reshape(-1)
            if w.numel() != T:
                raise ValueError(f"objective_weights needs {T} entries")
        elif self.objective_index is not None:
            w = torch.zeros(T, dtype=torch.float64)
            w[int(self.objective_index)] = 1.0
        else:
            w = torch.ones(T, dtype=torch.float64)
        return w.to(like.device if like is not None else self.gp_device)

    def _acq_weights(self) -> torch.Tensor:
        """Objective weights in the maximised direction (min mode negates), over the modelled outputs."""
        sign = 1.0 if self.objective_mode == "max" else -1.0
        return sign * self._objective_weights()

    def _incumbent(self, w: torch.Tensor) -> float:
        return float((self.y_tf(self.train_Y_raw) @ w.to(self.train_Y_raw)).max())

    # -- acquisition ---------------------------------------------------------------------------------------------
    def _latin_hypercube(self, n: int) -> np.ndarray:
        from scipy.stats import qmc

        return qmc.LatinHypercube(d=self.dim, seed=self._rng).random(n=n)

    def _sobol_grid(self, n: int) -> np.ndarray:
        from scipy.stats import qmc

        pts = qmc.Sobol(self.dim, scramble=True, seed=self._rng).random_base2(max(1, math.ceil(math.log2(max(n, 2)))))
        return pts[:n]

    def acquire(self, k: int) -> torch.Tensor:
        """k unit-cube points to evaluate next (mode: see the module docstring)."""
        k = int(k)
        if k < 1:
            return torch.empty((0, self.dim), dtype=self.dtype, device=self.gp_device)
        if self.acquisition == "variance":
            return self._pool_scan(k)
        if self.acquisition == "qlogei":
            return self._acquire_qlogei(k)
        return self._analytic_sweep(k)

    def _pool_scan(self, k: int) -> torch.Tensor:
        """Bayesian7.py:650-686 on the device: pool -> summed variance -> top-K_big -> FPS(k) from a random start."""
        cfg = self.config
        gp = self.gp_model
        pool = self._tensor(self._latin_hypercube(cfg.candidates_pool_size))
        if gp.independent:  # sum over the outputs of their own posterior variances, in one device sweep
            _, _, score = gp.engine.acquire_multi(gp.states, self.x_tf(pool), "variance", return_scores=True)
        else:
            # every output's variance is the shared var_std (s_t = 1 in the log-standardised space): the summed score
            # ranks like the shared variance
            _, _, score = gp.engine.acquire(gp.state, self.x_tf(pool), "variance", return_scores=True)
        k_big = min(max(5000, 20 * k), cfg.K_BIG_CAP, pool.shape[0])
        _, order = self.engine.topk(score, k_big)
        shortlist = pool[order.to(pool.device)]
        if k >= k_big:  # FPS of at least all points keeps them all (Bayesian7.py:88-89)
            return shortlist
        start = int(self._rng.integers(0, k_big))
        return shortlist[self.engine.fps(shortlist, k, start).to(pool.device)]

    def _analytic_sweep(self, k: int) -> torch.Tensor:
        """Sobol grid scored on the objective sum_t w_t f_t of the modelled outputs (ExactGP.sweep_objective: the
        combined alpha of one shared factorisation, or the multi-output sweep over independent outputs), best k by
        gpx_topk_f64."""
        gp = self.gp_model
        grid = self._tensor(self._sobol_grid(self.config.raw_samples))
        w = self._acq_weights()
        _, _, score = gp.sweep_objective(self.x_tf(grid), self.acquisition, w.tolist(), best_f=self._incumbent(w),
                                         beta=self.config.beta, return_scores=True)
        _, order = self.engine.topk(score, min(k, grid.shape[0]))
        return grid[order.to(grid.device)]

    def _acquire_qlogei(self, k: int) -> torch.Tensor:
        """optimize_acqf on MC qLogEI (Bayesian.py:96-113: 512 Sobol base samples, 10 restarts, 1024 raw samples,
        batch_limit 5, maxiter 200) in the unit cube through the log-input transform.  Chunks of at most GPX_MAX_Q
        points; after each, the model is conditioned on the chunk with its posterior mean (kriging believer)."""
        from .acqf import LinearMCObjective, SobolQMCNormalSampler, optimize_acqf, qLogExpectedImprovement

        cfg = self.config
        w = self._acq_weights()
        best_f = self._incumbent(w)
        objective = LinearMCObjective(w.cpu())
        unit_box = torch.stack([torch.zeros(self.dim), torch.ones(self.dim)]).to(self.dtype)
        x_tf = self.x_tf
        model = self.gp_model
        picked: List[torch.Tensor] = []
        remaining = k
        while remaining > 0:
            q = min(remaining, _capi.GPX_MAX_Q)
            seed = int(self._rng.integers(0, 1 << 30))
            acq = qLogExpectedImprovement(model, best_f=best_f, objective=objective,
                                          sampler=SobolQMCNormalSampler(torch.Size([cfg.mc_samples]), seed))

            class _UnitCube:  # optimize_acqf searches the unit cube; the GP sees transformed inputs
                def __init__(self, inner, m):
                    self.inner, self.model = inner, m

                def __call__(self, X):
                    return self.inner(x_tf(X.reshape(-1, X.shape[-1])).reshape(X.shape))

            cand, _ = optimize_acqf(_UnitCube(acq, model), unit_box, q=q, num_restarts=cfg.num_restarts,
                                    raw_samples=cfg.acqf_raw_samples,
                                    options={"batch_limit": cfg.batch_limit, "maxiter": cfg.maxiter}, seed=seed)
            cand = cand.detach().reshape(q, self.dim)
            picked.append(cand)
            remaining -= q
            if remaining > 0:  # condition on the chunk: fantasy observations = current posterior means
                Xf = x_tf(cand.to(self.gp_device))
                fantasy = model.posterior(Xf).mean
                model = ExactGP(torch.cat([model.train_X, Xf]), torch.cat([model.train_Y, fantasy]), model.params,
                                engine=self.engine, jitter_schedule=model.jitter_schedule).fit()
        return torch.cat(picked)

    def optimize_acquisition_function(self, gp=None) -> torch.Tensor:
        return self.acquire(self.batch_size)

    # -- main loop -----------------------------------------------------------------------------------------------
    def _initial_design(self):
        missing = self.n_initial_points - self.train_X.shape[0]
        if missing <= 0:
            return
        print(f"[init] Latin-hypercube design of {missing} points")
        for row in self._latin_hypercube(missing):
            self._observe(self._tensor(row))

    def _round(self) -> int:
        """One active-learning round: fit, report, select (Bayesian7.py:676: min(acq_batch_size, remaining) points),
        evaluate.  Returns the number of successful evaluations."""
        self.iteration_counter += 1
        print(f"\n[round {self.iteration_counter}] {len(self.train_X)} observations")
        self.fit_gp_model()
        self.evaluate_model(self.train_X, self.train_Y_raw, "Train_Set")
        if self.test_X is not None:
            self.evaluate_model(self.test_X, self.test_Y_raw, "Test_Set")
        want = min(self.config.acq_batch_size, self.target_total - len(self.train_X))
        batch = self.acquire(want)
        print(f"[round {self.iteration_counter}] {len(batch)} points selected by {self.acquisition}")
        ok = sum(self._observe(x) for x in batch)
        if ok:
            try:  # the model is recomputable from the CSV; this snapshot is a convenience
                ps = self.gp_model.params
                kernel = [dict(p.__dict__) for p in ps] if isinstance(ps, list) else dict(ps.__dict__)
                torch.save({"X": self.train_X.cpu(), "Y": self.train_Y_raw.cpu(), "kernel": kernel},
                           self.model_save_path)
            except Exception:
                pass
        return ok

    def optimize(self):
        if self.target_total is None:
            raise AssertionError("optimize() needs target_total (the total number of evaluations to reach)")
        self._initial_design()
        while len(self.train_X) < self.target_total:
            if self._round() == 0:
                print("[stop] every simulation of the round failed")
                break
        print(f"[done] {len(self.train_X)} evaluations")
        if len(self.train_X) == 0:
            return None, None
        obj = self._scalar_objective(self.train_Y_raw)
        best = int(torch.argmax(obj)) if self.objective_mode == "max" else int(torch.argmin(obj))
        return self._scaled_to_original(self.train_X[best]), float(obj[best])


def farthest_point_sampling(X: torch.Tensor, m: int, rng: Optional[np.random.Generator] = None,
                            engine: Optional[GPEngine] = None) -> torch.Tensor:
    """The m rows of X chosen by greedy farthest-point sampling from a random start (Bayesian7.py:82-106), on the
    device through gpx_fps_f64 (``engine`` defaults to one on X's device)."""
    n = X.shape[0]
    if m >= n:
        return X
    rng = rng or np.random.default_rng()
    eng = engine if engine is not None else GPEngine(X.device)
    return X[eng.fps(X, m, int(rng.integers(0, n)))]
