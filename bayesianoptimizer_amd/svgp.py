"""Driven variant (optimization/Bayesian7.py): serving a trained batched SVGP on the GPU engine, and the pool scan.

SURVEY §8a row a9 and §8f row 2.  ``scripts/run_optimization.py:4`` drives ``Bayesian7.BayesianOptimizer``, whose
acquisition (``optimization/Bayesian7.py:646-688``) is: LHS candidate pool -> per 2048-candidate chunk
``likelihood(model(x_std)).variance.sum(0)`` -> ``torch.topk(K_big)`` -> ``farthest_point_sampling(batch_k)``.  Here the
predictive, the top-k and the FPS all run in libgpx (``gpx_svgp_*``, ``gpx_topk_f64``, ``gpx_fps_f64``); the SVGP's
variational TRAINING (Adam on the ELBO, ``:451-538``) is not part of the hot path and stays out of scope
(DESIGN.md §7): a model trained by the reference is loaded from its checkpoint state dict (``batch_svgp.pt``,
``:702-707``) with ``SVGPModel.from_state_dict``.

All arithmetic is fp64 (the reference model is float32; its variational jitter, 1e-4, is kept as the default).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch

from .engine import GPEngine, KernelParams
from .transforms import LogInputStandardizer

VARIATIONAL_JITTER_F32 = 1e-4  # gpytorch settings.variational_cholesky_jitter for float32 [upstream]
NOISE_LOWER_BOUND = 1e-4       # GaussianLikelihood noise constraint GreaterThan(1e-4) [upstream]


def _softplus(x: torch.Tensor) -> torch.Tensor:
    return torch.nn.functional.softplus(x.to(torch.float64))


@dataclass
class SVGPModel:
    """Trained state of Bayesian7's BatchSVGP (``optimization/Bayesian7.py:128-178``), T tasks (outputs).

    Z: T x M x d inducing points (standardized-log input space), vmean: T x M, vchol: T x M x M
    (chol_variational_covar; its lower triangle is used), params: per task ScaleKernel(Linear + Matérn-5/2)
    hyperparameters with ConstantMean ``const_mean`` and GaussianLikelihood ``noise``."""

    Z: torch.Tensor
    vmean: torch.Tensor
    vchol: torch.Tensor
    params: List[KernelParams]
    jitter: float = VARIATIONAL_JITTER_F32

    @property
    def num_tasks(self) -> int:
        return self.Z.shape[0]

    @classmethod
    def from_state_dict(cls, model_sd: dict, likelihood_sd: Optional[dict] = None,
                        jitter: float = VARIATIONAL_JITTER_F32) -> "SVGPModel":
        """Parameters of a gpytorch BatchSVGP / GaussianLikelihood state dict (the ``{"model": ..., "likelihood":
        ...}`` checkpoint of ``optimization/Bayesian7.py:702-707``; load it with ``torch.load(path,
        weights_only=True)``).  Raw parameters go through gpytorch's default constraints [upstream]: softplus
        (Positive) for lengthscale, LinearKernel variance and outputscale; softplus + 1e-4 for the noise."""
        g = lambda k: model_sd[k].to(torch.float64)  # noqa: E731
        Z = g("variational_strategy.inducing_points")
        vmean = g("variational_strategy._variational_distribution.variational_mean")
        vchol = g("variational_strategy._variational_distribution.chol_variational_covar")
        T, M, d = Z.shape
        ls = _softplus(model_sd["covar_module.base_kernel.kernels.1.raw_lengthscale"]).reshape(T, -1)
        lv = _softplus(model_sd["covar_module.base_kernel.kernels.0.raw_variance"]).reshape(T, -1)
        os_ = _softplus(model_sd["covar_module.raw_outputscale"]).reshape(T)
        if "mean_module.raw_constant" in model_sd:
            const = g("mean_module.raw_constant").reshape(T)
        else:
            const = g("mean_module.constant").reshape(T)
        noise = torch.full((T,), NOISE_LOWER_BOUND, dtype=torch.float64)
        if likelihood_sd is not None and "noise_covar.raw_noise" in likelihood_sd:
            noise = _softplus(likelihood_sd["noise_covar.raw_noise"]).reshape(T) + NOISE_LOWER_BOUND
        params = []
        for t in range(T):
            lvt = lv[t] if lv.shape[1] == d else lv[t].expand(d)
            params.append(KernelParams("scale_linear_matern52", [float(v) for v in ls[t]], outputscale=float(os_[t]),
                                       noise=float(noise[t]), const_mean=float(const[t]),
                                       linear_variance=[float(v) for v in lvt]))
        return cls(Z=Z, vmean=vmean, vchol=vchol, params=params, jitter=jitter)


class SVGPPredictor:
    """The SVGP predictive on the engine: ``predict`` ≙ ``likelihood(model(x_std))`` mean / variance
    (``optimization/Bayesian7.py:558,668``); ``pool_scan`` ≙ the acquisition block ``:646-688``."""

    def __init__(self, model: SVGPModel, engine: Optional[GPEngine] = None,
                 input_transform: Optional[LogInputStandardizer] = None):
        self.engine = engine or GPEngine()
        self.model = model
        self.input_transform = input_transform
        self.prep = self.engine.svgp_prepare(model.params, model.Z, model.vmean, model.vchol, jitter=model.jitter)

    def _std(self, X: torch.Tensor, transformed: bool) -> torch.Tensor:
        X = X.to(device=self.engine.device, dtype=torch.float64)
        if transformed or self.input_transform is None:
            return X
        return self.input_transform(X).to(torch.float64)

    def predict(self, X: torch.Tensor, transformed: bool = False):
        """(mean, variance), each m x T, of the likelihood-wrapped predictive at X (unit cube unless
        ``transformed``)."""
        mean, var, _ = self.engine.svgp_predict(self.prep, self._std(X, transformed), want=("mean", "var"))
        return mean, var

    def uncertainty(self, X: torch.Tensor, transformed: bool = False) -> torch.Tensor:
        """Sum over tasks of the predictive variance (``pred.variance.sum(dim=0)``, ``:671``)."""
        _, _, score = self.engine.svgp_predict(self.prep, self._std(X, transformed), want=("score",))
        return score

    def pool_scan(self, cand_unit: torch.Tensor, batch_k: int, k_big_cap: int = 8000,
                  generator: Optional[torch.Generator] = None, start: Optional[int] = None):
        """Bayesian7's acquisition (``:646-688``): score the pool, keep the K_big most uncertain
        (K_big = min(max(5000, 20 batch_k), k_big_cap, pool)), then farthest-point-sample ``batch_k`` of them from a
        random start (``torch.randint``, ``:93``).  Returns (selected unit points batch_k x d, their pool indices)."""
        cand_unit = cand_unit.to(device=self.engine.device, dtype=torch.float64).contiguous()
        m = cand_unit.shape[0]
        score = self.uncertainty(cand_unit)
        k_big = int(min(max(5000, 20 * batch_k), k_big_cap, m))
        _, idx_big = self.engine.topk(score, k_big)
        cand_big = cand_unit.index_select(0, idx_big)
        if batch_k >= k_big:  # farthest_point_sampling returns its input unchanged (:89-90)
            return cand_big, idx_big
        if start is None:
            start = int(torch.randint(0, k_big, (1,), generator=generator).item())
        sel = self.engine.fps(cand_big, batch_k, start)
        return cand_big.index_select(0, sel), idx_big.index_select(0, sel)
