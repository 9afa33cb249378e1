"""Bench's SVGP driven config (Bayesian7: T = 8, M = 2048, d = 5) pool scan only, for a kernel trace: 10,000-candidate
pool -> score -> top 8000 -> FPS of 500, three times."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bayesianoptimizer_amd import GPEngine, KernelParams
from bayesianoptimizer_amd.svgp import SVGPModel, SVGPPredictor

dev = torch.device("cuda", 0)
eng = GPEngine(dev)
rng = np.random.default_rng(19)
T8, M8, d5 = 8, 2048, 5
Z = rng.standard_normal((T8, M8, d5))
vchol = np.tril(0.3 * rng.standard_normal((T8, M8, M8)) / np.sqrt(M8))
for t in range(T8):
    vchol[t][np.diag_indices(M8)] = 0.2 + 0.5 * rng.random(M8)
kps = [KernelParams("scale_linear_matern52", list(0.8 + rng.random(d5)), outputscale=0.5 + rng.random(), noise=1e-3,
                    const_mean=0.0, linear_variance=list(0.05 + 0.1 * rng.random(d5))) for _ in range(T8)]
model = SVGPModel(Z=torch.tensor(Z), vmean=torch.tensor(rng.standard_normal((T8, M8))), vchol=torch.tensor(vchol),
                  params=kps)
pred = SVGPPredictor(model, eng)
pool = torch.tensor(rng.random((10000, d5)), device=dev)
for _ in range(4):
    torch.cuda.synchronize()
    a = time.perf_counter()
    x, i = pred.pool_scan(pool, batch_k=500, start=0)
    torch.cuda.synchronize()
    b = time.perf_counter()
    pred.uncertainty(pool)
    torch.cuda.synchronize()
    print(f"pool scan {1e3 * (b - a):.2f} ms, scoring alone {1e3 * (time.perf_counter() - b):.2f} ms, first {int(i[0])}")
