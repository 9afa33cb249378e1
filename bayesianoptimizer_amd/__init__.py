"""MI355X-native exact-GP posterior engine (drop-in hot path for billbearhunter/BayesianOptimizer).

Public surface:
  GPEngine / KernelParams / GPState  — fit / posterior / acquire on device tensors via libgpx.so
  ExactGP, acquisition functions     — BoTorch-shaped wrappers (bayesianoptimizer_amd.models)
  BayesianOptimizer                  — drop-in for optimization/Bayesian7.py's constructor / optimize()
"""
from ._capi import GPXError, GPXLibraryError, GPXTimeoutError, NotPositiveDefiniteError  # noqa: F401
from .engine import GPEngine, GPState, KernelParams, botorch_default_lengthscale  # noqa: F401

__version__ = "0.1.0"
