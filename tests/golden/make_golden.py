"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

Run in the build container:  python tests/golden/make_golden.py [--reference /root/reference]

Fixtures are data (inputs and oracle outputs), never reference source:
  synthetic_*   seeded synthetic problems of SURVEY §8d (several kernels / dims / output counts)
  real_b6_*     the first 256 rows of the reference's results/optimization_results.csv in the exact-GP mode of
                optimization/Bayesian6.py (unit-cube X, log-standardised 8 outputs, Scale(Linear+Matern-5/2))
                scored on 512 rows of validation_set.csv
  real_b7_*     the same rows through Bayesian7's input transform (optimization/Bayesian7.py:181-190,363-385),
                RBF kernel
  results_*     the INPUTS of the reference's own results files at full size (results/optimization_results*.csv:
                physical X, 5 columns, and the 8 raw outputs, read by column position because two files name their
                outputs disp_* instead of x_*), and validation_2048 the first 2048 rows of validation_set.csv.  No
                expected outputs: tests/test_gpu_realdata.py runs the oracle on them on the GPU box's host.
                optimization_results2.csv row 2386 (1-based data row 2385) holds a corrupt field
                ("200.067 7064061164856"): that row is dropped and listed in `dropped` (the reference's own resume,
                optimization/Bayesian7.py:274-286, would fail to parse the whole file).
The reference's CSVs are read only here (at generation time); the .npz files carry the numbers.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gp_oracle as O  # noqa: E402

BOUNDS = np.array([(0.3, 1.0), (0.001, 300.0), (0.001, 400.0), (2.0, 7.0), (2.0, 7.0)])  # config/config.py:2-20
ACQS = [("ei", O.ACQ_EI), ("logei", O.ACQ_LOGEI), ("ucb", O.ACQ_UCB), ("variance", O.ACQ_VARIANCE)]


def save(name, X, Y, Xs, p: O.KernelParams, beta=4.0):
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    st = O.fit(X, Y, p)
    mu, var = O.posterior(st, Xs)
    mu = mu.reshape(Xs.shape[0], -1)
    out = dict(X=X, Y=Y, Xs=Xs, kind=p.kind, lengthscale=p.lengthscale, outputscale=p.outputscale, noise=p.noise,
               jitter=p.jitter, const_mean=p.const_mean, linear_variance=p.linear_variance, beta=beta,
               L=st.L, alpha=st.alpha.reshape(X.shape[0], -1), mu=mu, var=var)
    st0 = O.fit(X, Y[:, 0], p)
    best_f = float(Y[:, 0].max())
    out["best_f"] = best_f
    for acq, aid in ACQS:
        v, i, s = O.acquire_argmax(st0, Xs, aid, best_f=best_f, beta=beta)
        out[f"score_{acq}"] = s
        out[f"argmax_{acq}"] = i
        srt = np.sort(s[np.isfinite(s)])
        out[f"gap_{acq}"] = srt[-1] - srt[-2]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print("wrote", name, X.shape, Y.shape, Xs.shape)


def synthetic():
    for name, n, d, kind, T, seed, extra in [
        ("synthetic_rbf_n200_d4", 200, 4, O.RBF, 1, 11, {}),
        ("synthetic_matern_n256_d8", 256, 8, O.MATERN52, 1, 12, {}),
        ("synthetic_slm_n150_d5_T8", 150, 5, O.SCALE_LINEAR_MATERN52, 8, 13, {"linear_variance": 0.3}),
        ("synthetic_rbf_n129_d16", 129, 16, O.RBF, 2, 14, {"outputscale": 2.5, "const_mean": 0.3}),
        ("synthetic_rbf_n1_d3", 1, 3, O.RBF, 1, 15, {}),
    ]:
        X, y = O.synthetic_problem(n, d, seed)
        Y = np.stack([y * (1.0 + 0.25 * r) + 0.1 * r for r in range(T)], axis=1)
        Xs = O.sobol_candidates(700, d, seed + 1)
        p = O.KernelParams(kind, np.full(d, O.botorch_default_lengthscale(d)), noise=1e-4, **extra)
        save(name, X, Y, Xs, p)


def real(ref: str):
    import pandas as pd

    cols = ["n", "eta", "sigma_y", "width", "height"] + [f"x_{i:02d}" for i in range(1, 9)]
    df = pd.read_csv(os.path.join(ref, "results", "optimization_results.csv"))[cols].dropna().iloc[:256]
    dv = pd.read_csv(os.path.join(ref, "validation_set.csv"))[cols].dropna().iloc[:512]
    Xp, Yr = df[cols[:5]].to_numpy(np.float64), df[cols[5:]].to_numpy(np.float64)
    Xv = dv[cols[:5]].to_numpy(np.float64)
    lo, hi = BOUNDS[:, 0], BOUNDS[:, 1]
    Xu, Xvu = (Xp - lo) / (hi - lo), (Xv - lo) / (hi - lo)
    # Bayesian6 exact mode: log(Y + shift) standardised per output (optimization/Bayesian6.py:427-443,463-468)
    eps = max(1e-12, np.abs(Yr).max() * 1e-6)
    shift = (-Yr.min() + eps) if Yr.min() <= 0 else eps
    Yl = np.log(Yr + shift)
    Y6 = (Yl - Yl.mean(0)) / np.maximum(Yl.std(0, ddof=1), 1e-12)
    d = 5
    p6 = O.KernelParams(O.SCALE_LINEAR_MATERN52, np.full(d, 0.4), outputscale=1.5, noise=1e-4,
                        linear_variance=np.linspace(0.05, 0.45, d))
    save("real_b6_results256_val512", Xu, Y6, Xvu, p6)
    # Bayesian7 transforms (optimization/Bayesian7.py:181-190, 363-385)
    Xs7, mu_x, sd_x = O.log_standardize_inputs(Xu, BOUNDS)
    Xv7, _, _ = O.log_standardize_inputs(Xvu, BOUNDS, mu_x, sd_x)
    Yl7 = np.log(Yr + 1e-6)
    Y7 = (Yl7 - Yl7.mean(0)) / np.maximum(Yl7.std(0, ddof=1), 1e-6)
    p7 = O.KernelParams(O.RBF, np.full(d, 1.2), noise=1e-3)
    save("real_b7_results256_val512", Xs7, Y7, Xv7, p7)


RESULTS_FILES = {  # tag -> file under results/ 
    "r3000": "optimization_results.csv",
    "r3901": "optimization_results1.csv",
    "r4235": "optimization_results1012.csv",
    "r5000": "optimization_results2.csv",
    "r7740": "optimization_results1009.csv",
    "r2905": "optimization_results002.csv",     # legacy disp_1..8 header: columns are taken by position
    "r173": "optimization_results100917.csv",   # small n: below the npad = 256 fused-sweep boundary
}


def results_inputs(ref: str):
    import pandas as pd

    for tag, fname in RESULTS_FILES.items():
        df = pd.read_csv(os.path.join(ref, "results", fname))
        num = df.apply(lambda c: pd.to_numeric(c, errors="coerce")).to_numpy(np.float64)
        bad = np.flatnonzero(np.isnan(num).any(axis=1))
        num = np.delete(num, bad, axis=0)
        X, Y = num[:, :5], num[:, 5:13]
        dup = X.shape[0] - np.unique(X, axis=0).shape[0]
        np.savez_compressed(os.path.join(HERE, f"results_{tag}.npz"), X=X, Y=Y, source=np.array(fname),
                            dropped=bad.astype(np.int64), duplicate_rows=np.int64(dup))
        print("wrote", tag, fname, X.shape, "dropped", bad.tolist(), "duplicate X rows", dup)
    dv = pd.read_csv(os.path.join(ref, "validation_set.csv")).iloc[:2048].to_numpy(np.float64)
    np.savez_compressed(os.path.join(HERE, "validation_2048.npz"), X=dv[:, :5], Y=dv[:, 5:13])
    print("wrote validation_2048", dv.shape)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only-results", action="store_true", help="write only the results_* / validation fixtures")
    a = ap.parse_args()
    if not a.only_results:
        synthetic()
    if os.path.isdir(a.reference):
        if not a.only_results:
            real(a.reference)
        results_inputs(a.reference)
