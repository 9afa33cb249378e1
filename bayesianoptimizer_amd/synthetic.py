"""Seeded synthetic workloads of SURVEY.md §8d (shared by bench.py, tests and the smoke check).

X ~ U[0,1]^{n x d} from ``np.random.default_rng(seed)``; y = sum_j sin(6 x_j) + 0.01 N(0,1), standardised;
candidates: scrambled Sobol points (scipy.stats.qmc, seed + 1), generated on the host and uploaded once.
"""
from __future__ import annotations

import math

import numpy as np


def problem(n: int, d: int, seed: int, noise_sd: float = 0.01):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    y = np.sin(6.0 * X).sum(axis=1) + noise_sd * rng.standard_normal(n)
    sd = y.std()
    y = (y - y.mean()) / (sd if sd > 0 else 1.0)
    return X, y


def sobol(m: int, d: int, seed: int) -> np.ndarray:
    from scipy.stats import qmc

    eng = qmc.Sobol(d, scramble=True, seed=seed)
    k = int(math.ceil(math.log2(max(m, 1))))
    return eng.random_base2(k)[:m]
