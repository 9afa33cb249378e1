"""Stub simulator with the reference's duck type and a driver that replays run_optimization's call sequence.

The Taichi MPM simulator (simulation/taichi.py) opens a GUI and needs taichi; the stub keeps its interface:
configure_geometry(width, height) raising ValueError outside [2, 7] (taichi.py:33-44),
run_simulation(n, eta, sigma_y) -> float32[8] (taichi.py:46-62, 140-142), cleanup() (taichi.py:145-148).
"""
from __future__ import annotations

import math
import os

import numpy as np

BOUNDS = [(0.3, 1.0), (0.001, 300.0), (0.001, 400.0), (2.0, 7.0), (2.0, 7.0)]  # config/config.py


class StubSimulator:
    def __init__(self, fail_every: int = 0):
        self.width = self.height = None
        self.calls = 0
        self.fail_every = fail_every
        self.cleaned = False

    def configure_geometry(self, width, height):
        if not (2.0 <= width <= 7.0 and 2.0 <= height <= 7.0):
            raise ValueError("geometry out of range")
        self.width, self.height = width, height

    def run_simulation(self, n, eta, sigma_y):
        self.calls += 1
        if self.fail_every and self.calls % self.fail_every == 0:
            return None
        t = np.arange(1, 9, dtype=np.float64)
        base = (self.width * self.height) ** 0.5 * (1.0 - 0.5 * n) / (1.0 + 0.002 * sigma_y + 0.01 * math.log1p(eta))
        return (base * np.log1p(t) + 0.01 * t).astype(np.float32)

    def cleanup(self):
        self.cleaned = True


def run_optimization_like(optimizer_cls, total_evaluations, n_initial_points, batch_size, output_dir,
                          svgp_threshold=3000, **extra):
    """Same resume arithmetic and constructor kwargs as scripts/run_optimization.py:34-134."""
    os.makedirs(output_dir, exist_ok=True)
    csv = os.path.join(output_dir, "optimization_results.csv")
    existing = 0
    if os.path.exists(csv):
        with open(csv) as f:
            existing = max(0, sum(1 for _ in f) - 1)
    resume = existing > 0
    target_total = int(total_evaluations)
    if existing >= target_total:
        return None, None
    remaining = target_total - existing
    init = 0 if resume else min(n_initial_points, remaining)
    after = remaining - init
    n_batches = 0 if after <= 0 else math.ceil(after / batch_size)
    sim = StubSimulator()
    try:
        opt = optimizer_cls(simulator=sim, bounds_list=BOUNDS, output_dir=output_dir, n_initial_points=init,
                            n_batches=n_batches, batch_size=batch_size, svgp_threshold=svgp_threshold, resume=resume,
                            target_total=target_total, test_csv_path="validation_set.csv", **extra)
        return opt.optimize()
    finally:
        sim.cleanup()
