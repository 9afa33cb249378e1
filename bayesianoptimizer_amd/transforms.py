"""Input/output transforms of the reference, on torch tensors.

These are O(n d) elementwise host-side steps around the engine (not part of the HIP hot path):
  normalize / unnormalize            botorch.utils.transforms as used in optimization/Bayesian.py:140,
                                     optimization/Bayesian2.py:165
  Standardize                        BoTorch outcome transform (optimization/Bayesian1.py:112) [upstream]
  LogInputStandardizer               unit -> physical -> log -> standardise (optimization/Bayesian7.py:181-190,
                                     363-373; std floor 1e-6) / Bayesian6 (:445-453, floor 1e-12)
  LogOutputStandardizer              log(y + 1e-6) standardise and its inverse exp(mu*s+m)-1e-6
                                     (optimization/Bayesian7.py:371-373, 382-383, 561-562)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


def normalize(x: torch.Tensor, bounds: torch.Tensor) -> torch.Tensor:
    """bounds: (2, d) lower/upper rows (BoTorch convention)."""
    return (x - bounds[0]) / (bounds[1] - bounds[0])


def unnormalize(x: torch.Tensor, bounds: torch.Tensor) -> torch.Tensor:
    return x * (bounds[1] - bounds[0]) + bounds[0]


@dataclass
class Standardize:
    """y_std = (y - mean) / std per output, unbiased std with BoTorch's 1e-8 guard [upstream]."""

    mean: Optional[torch.Tensor] = None
    std: Optional[torch.Tensor] = None

    def fit(self, Y: torch.Tensor) -> "Standardize":
        self.mean = Y.mean(dim=0)
        std = Y.std(dim=0) if Y.shape[0] > 1 else torch.ones_like(self.mean)
        self.std = torch.where(std >= 1e-8, std, torch.ones_like(std))
        return self

    def transform(self, Y: torch.Tensor) -> torch.Tensor:
        return (Y - self.mean) / self.std

    def untransform_mean(self, mu: torch.Tensor) -> torch.Tensor:
        return self.mean + self.std * mu

    def untransform_var(self, var: torch.Tensor) -> torch.Tensor:
        return var * self.std * self.std


class LogInputStandardizer:
    """Bayesian7 input transform: x_unit -> lo + x (hi - lo) -> log(clamp 1e-6) -> (. - mean) / std."""

    def __init__(self, bounds: torch.Tensor, std_floor: float = 1e-6):
        self.bounds = bounds  # (2, d)
        self.std_floor = std_floor
        self.mean = None
        self.std = None

    def _log(self, x_unit: torch.Tensor) -> torch.Tensor:
        x_phys = unnormalize(x_unit.to(self.bounds), self.bounds)
        return torch.log(x_phys.clamp(min=1e-6))

    def fit(self, x_unit: torch.Tensor) -> "LogInputStandardizer":
        L = self._log(x_unit)
        self.mean = L.mean(dim=0, keepdim=True)
        self.std = (L.std(dim=0, keepdim=True) if L.shape[0] > 1 else torch.ones_like(self.mean)).clamp_min(
            self.std_floor)
        return self

    def __call__(self, x_unit: torch.Tensor) -> torch.Tensor:
        return (self._log(x_unit) - self.mean) / self.std


class LogOutputStandardizer:
    """Bayesian7 output transform: log(y + 1e-6) standardised per output; inverse exp(mu s + m) - 1e-6."""

    def __init__(self, std_floor: float = 1e-6, eps: float = 1e-6):
        self.std_floor = std_floor
        self.eps = eps
        self.mean = None
        self.std = None

    def fit(self, Y: torch.Tensor) -> "LogOutputStandardizer":
        L = torch.log(Y + self.eps)
        self.mean = L.mean(dim=0, keepdim=True)
        self.std = (L.std(dim=0, keepdim=True) if L.shape[0] > 1 else torch.ones_like(self.mean)).clamp_min(
            self.std_floor)
        return self

    def __call__(self, Y: torch.Tensor) -> torch.Tensor:
        return (torch.log(Y + self.eps) - self.mean) / self.std

    def inverse_mean(self, mu_std: torch.Tensor) -> torch.Tensor:
        return torch.exp(mu_std * self.std + self.mean) - self.eps
