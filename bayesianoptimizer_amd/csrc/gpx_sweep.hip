// Posterior / acquisition sweep over a chunk of C candidates.
// Replaces model.posterior(X) (optimization/Bayesian2.py:169-171, optimization/Bayesian6.py:615-617,688-690),
// the raw-sample sweep + argmax inside optimize_acqf (optimization/Bayesian.py:105-113) and the pool scan +
// top-k of optimization/Bayesian7.py:646-681.
//
// Per chunk, three launches:
//  1. kstar_kernel   K*[j][c] = k(x_j, xs_c) for all padded rows j (row-major npad x C, zero for j >= n),
//                    and the partial means mu_part[jb][r][c] = sum_{j in block jb} alpha[j][r] K*[j][c].
//  2. trmm_sumsq     V = L^{-1} K* = W^T K* as a triangular fp64-MFMA product (128x128 tiles, k < (I+1)*128
//                    for row tile I), never stored: each workgroup writes the column sums of V^2 over its 128
//                    rows into ss_part[I][c].  This is the n^2-flops-per-candidate term and the dominant
//                    kernel of the whole hot path.
//  3. finalize       mu = m + sum mu_part, var = k** - sum ss_part (fixed summation order: deterministic),
//                    GPyTorch/BoTorch variance floors, Standardize untransform, analytic acquisition, and a
//                    256-candidate block argmax record (max value, then lowest index; NaN never wins).
// launch_argmax_final reduces the records of the whole sweep in one workgroup.
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_trmm_asm.h"
#include <cstdlib>

namespace gpx {

// ---- acquisition math (BoTorch analytic forms [upstream], restated; oracle/gp_oracle.py mirrors them) ----
__device__ __forceinline__ double ndtr_d(double a) {  // standard normal cdf, cephes-style branches
  const double x = a * 0.70710678118654752440084436210485;
  const double z = fabs(x);
  if (z < 0.70710678118654752440084436210485) return 0.5 + 0.5 * erf(x);
  const double y = 0.5 * erfc(z);
  return (x > 0.0) ? 1.0 - y : y;
}
__device__ __forceinline__ double phi_d(double u) { return exp(-0.5 * u * u) * 0.39894228040143267793994605993438; }
__device__ __forceinline__ double ei_helper_d(double u) { return phi_d(u) + u * ndtr_d(u); }
__device__ __forceinline__ double log1mexp_d(double x) {
  return (x > -0.69314718055994530941723212145818) ? log(-expm1(x)) : log1p(-exp(x));
}
__device__ __forceinline__ double log_ei_helper_d(double u) {
  const double neg_inv_sqrt_eps = -67108864.0;  // -1/sqrt(2^-52)
  if (u > -1.0) return log(ei_helper_d(u));
  const double u_eps = fmax(u, neg_inv_sqrt_eps);
  const double w = log(erfcx(-u_eps * 0.70710678118654752440084436210485) * fabs(u_eps)) +
                   0.22579135264472743236309761494744;  // log(sqrt(pi/2))
  const double log_phi = -0.5 * u * u - 0.91893853320467274178032973640562;  // log(sqrt(2 pi))
  if (u > neg_inv_sqrt_eps) return log_phi + log1mexp_d(w);
  return log_phi - 2.0 * log(fabs(u));
}
__device__ __forceinline__ double acq_score(int kind, double mu, double var, double best_f, double beta) {
  const double sigma = sqrt(var);
  if (kind == GPX_ACQ_EI) return sigma * ei_helper_d((mu - best_f) / sigma);
  if (kind == GPX_ACQ_LOGEI) return log_ei_helper_d((mu - best_f) / sigma) + log(sigma);
  if (kind == GPX_ACQ_UCB) return mu + sqrt(beta) * sigma;
  return var;
}

// Sum of `cnt` partials spaced `stride` apart, in a fixed order: 8 independent loads in flight per group
// (a plain loop over a runtime count waited for every load before the next: 32 serial round trips).
__device__ __forceinline__ double sum_partials(const double* __restrict__ p, int cnt, int64_t stride) {
  double s = 0.0;
  int i = 0;
  for (; i + 8 <= cnt; i += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = p[(int64_t)(i + q) * stride];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; i < cnt; ++i) s += p[(int64_t)i * stride];
  return s;
}

// (value, index) order: larger value wins, equal values -> lower index; NaN already mapped to -inf.
__device__ __forceinline__ void argmax_merge(double& v, int64_t& i, double v2, int64_t i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

template <int DMAX>
__device__ __forceinline__ void load_point(const gpx_kernel_params& p, const double* __restrict__ x, bool valid,
                                           double (&xs)[DMAX], double (&xr)[DMAX]) {
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    const double v = (valid && k < p.d) ? x[k] : 0.0;
    xs[k] = (k < p.d) ? v / p.lengthscale[k] : 0.0;
    xr[k] = v;
  }
}

// ---- 1. K* and partial means ---------------------------------------------------------------------------
// KIND and ONE_RHS are compile-time so the per-element loop carries no uniform branches (kind dispatch, nrhs
// predicates); dimensions k >= d are zero in both sx/sr and xs/xr, so the distance and linear sums run over all DMAX
// without a k < d test (adding +0 leaves r2 and lv bitwise unchanged).  Rows j >= n of the last block are zero.
template <int DMAX, bool F32, int KIND, bool ONE_RHS>
__global__ void __launch_bounds__(WG) kstar_kernel(gpx_kernel_params p, int n, const double* __restrict__ X,
                                                   int64_t ldx, const double* __restrict__ alpha, int nrhs,
                                                   const double* __restrict__ Xs, int64_t ldxs, int64_t m_chunk,
                                                   int64_t C, double* __restrict__ kstar,
                                                   double* __restrict__ mu_part) {
  __shared__ double sx[NB][DMAX + 1], sr[NB][DMAX + 1], sa[NB][GPX_MAX_RHS];
  const int jb = blockIdx.y;
  const int j0 = jb * NB;
  const int d = p.d;
  for (int e = threadIdx.x; e < NB * DMAX; e += WG) {
    const int r = e / DMAX, k = e % DMAX;
    double v = 0.0;
    if (k < d && j0 + r < n) v = X[(int64_t)(j0 + r) * ldx + k];
    sx[r][k] = (k < d) ? v / p.lengthscale[k] : 0.0;
    sr[r][k] = (k < d) ? v * p.linear_variance[k] : 0.0;
  }
  for (int e = threadIdx.x; e < NB * nrhs; e += WG) {
    const int r = e / nrhs, q = e % nrhs;
    sa[r][q] = alpha[(int64_t)(j0 + r) * nrhs + q];
  }
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * WG + threadIdx.x;
  const bool valid = c < m_chunk;
  double xs[DMAX], xr[DMAX];
  load_point<DMAX>(p, Xs + (valid ? c * ldxs : 0), valid, xs, xr);
  double mu[GPX_MAX_RHS];
#pragma unroll
  for (int q = 0; q < GPX_MAX_RHS; ++q) mu[q] = 0.0;
  const int jn = n - j0 < NB ? n - j0 : NB;  // real rows of this block (<= 0 for an all-padding block)
  int j = 0;
  // four rows in flight (independent distance / exp chains; the mean accumulates in row order)
#pragma unroll 4
  for (; j < jn; ++j) {
    double lv = 0.0;
    if (KIND == GPX_KERNEL_SCALE_LINEAR_MATERN52) {
#pragma unroll
      for (int k = 0; k < DMAX; ++k) lv += sr[j][k] * xr[k];
    }
    double kv;
    if (F32) {
      float r2 = 0.0f;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) {
        const float df = (float)sx[j][k] - (float)xs[k];
        r2 += df * df;
      }
      kv = cov_from_r2_f32(KIND, p.outputscale, r2, lv);
    } else {
      double r2 = 0.0;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) {
        const double df = sx[j][k] - xs[k];
        r2 += df * df;
      }
      kv = cov_from_r2(KIND, p.outputscale, r2, lv);
    }
    kstar[(int64_t)(j0 + j) * C + c] = kv;
    if (ONE_RHS) {
      mu[0] += sa[j][0] * kv;
    } else {
#pragma unroll
      for (int q = 0; q < GPX_MAX_RHS; ++q)
        if (q < nrhs) mu[q] += sa[j][q] * kv;
    }
  }
  for (; j < NB; ++j) kstar[(int64_t)(j0 + j) * C + c] = 0.0;
  for (int q = 0; q < nrhs; ++q) mu_part[((int64_t)jb * nrhs + q) * C + c] = mu[q];
}

// fp64 K* with the distance's cross term on the matrix cores (GPyTorch's ||a||^2 + ||b||^2 - 2 a.b clamped at 0
// [upstream]; gram_mfma_kernel's arithmetic, centred by the mean of the workgroup's valid training rows).  A workgroup
// owns the 64 training rows of block jb x 256 candidates, wave w the candidates 64 w .. 64 w + 63 (four 16-column MFMA
// blocks) over the four 16-row strips.  The MFMA accumulator gives a lane rows kq + 4 r of column m of a block; before the
// stores, each group of four registers (the four column blocks of one r) is transposed across the wave's four 16-lane
// rows by two v_permlane32_swap + two v_permlane16_swap, so every store instruction writes one K* row of 64 consecutive
// candidates (512 bytes) like the difference-form kernel (an untransposed first version, four 128-byte row segments per
// instruction, ran at 3.5 vs 4.7 TB/s).  Per element: one fma, a compare and the covariance, no per-dimension VALU work.
template <int DMAX, int KIND, bool ONE_RHS>
__global__ void __launch_bounds__(WG) kstar_mfma_kernel(gpx_kernel_params p, int n, const double* __restrict__ X,
                                                        int64_t ldx, const double* __restrict__ alpha, int nrhs,
                                                        const double* __restrict__ Xs, int64_t ldxs, int64_t m_chunk,
                                                        int64_t C, double* __restrict__ kstar,
                                                        double* __restrict__ mu_part) {
  constexpr bool lin = (KIND == GPX_KERNEL_SCALE_LINEAR_MATERN52);
  constexpr int KS = DMAX / 4;
  constexpr int NRQ = ONE_RHS ? 1 : GPX_MAX_RHS;
  __shared__ double sa[NB][DMAX + 1], sb[WG][DMAX + 1], ra[lin ? NB : 1][DMAX + 1], rb[lin ? WG : 1][DMAX + 1];
  __shared__ double na[NB], nb[WG], cen[DMAX], sal[NB][NRQ];
  const int jb = blockIdx.y, j0 = jb * NB, d = p.d, t = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * WG;
  const int nv = n - j0 < NB ? n - j0 : NB;  // valid training rows of the block (<= 0: all padding)
  for (int e = t; e < NB * DMAX; e += WG) {
    const int r = e / DMAX, k = e % DMAX;
    const double v = (k < d && j0 + r < n) ? X[(int64_t)(j0 + r) * ldx + k] : 0.0;
    sa[r][k] = (k < d) ? v / p.lengthscale[k] : 0.0;
    if constexpr (lin) ra[r][k] = (k < d) ? v * p.linear_variance[k] : 0.0;
  }
  for (int e = t; e < WG * DMAX; e += WG) {
    const int r = e / DMAX, k = e % DMAX;
    const double v = (k < d && c0 + r < m_chunk) ? Xs[(c0 + r) * ldxs + k] : 0.0;
    sb[r][k] = (k < d) ? v / p.lengthscale[k] : 0.0;
    if constexpr (lin) rb[r][k] = v;
  }
  for (int e = t; e < NB * NRQ; e += WG) {
    const int r = e / NRQ, q = e % NRQ;
    sal[r][q] = (q < nrhs && j0 + r < n) ? alpha[(int64_t)(j0 + r) * nrhs + q] : 0.0;
  }
  __syncthreads();
  if (t < DMAX) {
    double s = 0.0;
    for (int r = 0; r < nv; ++r) s += sa[r][t];
    cen[t] = nv > 0 ? s / nv : 0.0;
  }
  __syncthreads();
  for (int e = t; e < NB * DMAX; e += WG) sa[e / DMAX][e % DMAX] -= cen[e % DMAX];
  for (int e = t; e < WG * DMAX; e += WG) sb[e / DMAX][e % DMAX] -= cen[e % DMAX];
  __syncthreads();
  {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) v = fma(sb[t][k], sb[t][k], v);
    nb[t] = v;
    if (t < NB) {
      double u = 0.0;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) u = fma(sa[t][k], sa[t][k], u);
      na[t] = u;
    }
  }
  __syncthreads();
  const int lane = t & 63, w = t >> 6, m = lane & 15, kq = lane >> 4;
  double mu[4][NRQ];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int q = 0; q < NRQ; ++q) mu[cb][q] = 0.0;
  double nbc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) nbc[cb] = nb[64 * w + 16 * cb + m];
#pragma unroll 1
  for (int rs = 0; rs < NB; rs += 16) {
    double kv[4][4];  // [r][cb]: row rs + kq + 4 r, candidate 64 w + 16 cb + m
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      d4 acc = {0.0, 0.0, 0.0, 0.0}, lac = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        acc = mfma16x16x4(sa[rs + m][4 * k + kq], sb[64 * w + 16 * cb + m][4 * k + kq], acc);
        if constexpr (lin) lac = mfma16x16x4(ra[rs + m][4 * k + kq], rb[64 * w + 16 * cb + m][4 * k + kq], lac);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = rs + kq + 4 * r;
        double v = cov_from_r2(KIND, p.outputscale, sqdist_expanded(na[j], nbc[cb], acc[r]), lin ? lac[r] : 0.0);
        v = j < nv ? v : 0.0;
        kv[r][cb] = v;
#pragma unroll
        for (int q = 0; q < NRQ; ++q) mu[cb][q] = fma(sal[j][q], v, mu[cb][q]);
      }
    }
    // after the transpose, register q of 16-lane row g holds row rs + q + 4 r, candidate 64 w + 16 g + m
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      transpose_rows4(kv[r]);
#pragma unroll
      for (int q = 0; q < 4; ++q) kstar[(int64_t)(j0 + rs + q + 4 * r) * C + c0 + 64 * w + lane] = kv[r][q];
    }
  }
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int q = 0; q < NRQ; ++q) {
      double v = mu[cb][q];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (kq == 0 && q < nrhs) mu_part[((int64_t)jb * nrhs + q) * C + c0 + 64 * w + 16 * cb + m] = v;
    }
}

// ---- 2. triangular product + column sums of squares ------------------------------------------------------
constexpr int TT = 128;  // trmm tile (rows of V x candidates)
using TrmmTile = MfmaTile<TT, TT, 16, true, true>;  // its accumulator layout (row_of / col_of) and LDS size
static_assert(TrmmTile::LDS_DOUBLES * 8 == trmm_asm::LDS_BYTES, "hand-placed tile uses MfmaTile's LDS image");

// kfull = 0: W upper triangular (k < (I+1)*128); kfull = 1: W is a full npad x npad matrix (the SVGP's
// W2 = L^{-T} S term, gpx_svgp.hip), k over all nI row tiles.
// With W2 (the SVGP's second product, grid.y = 2): blockIdx.y = 0 runs W2 with kfull = 1 into ss2 (the heavier,
// full-k tiles dispatched first), blockIdx.y = 1 the product given by (W, ss_part, kfull): both products of a chunk in
// one launch share its K* and one launch tail (two launches before).
__global__ void __launch_bounds__(WG) trmm_sumsq_kernel(const double* __restrict__ W, int64_t ldw,
                                                        const double* __restrict__ kstar, int64_t C, int nI, int ncb,
                                                        double* __restrict__ ss_part, int kfull,
                                                        const double* __restrict__ W2 = nullptr,
                                                        double* __restrict__ ss2 = nullptr) {
  __shared__ __attribute__((aligned(16))) double smem[TrmmTile::LDS_DOUBLES];
  if (W2 && blockIdx.y == 0) {
    W = W2;
    ss_part = ss2;
    kfull = 1;
  }
  // Candidate tiles in groups of G = 64 (every row tile of a group, heaviest first, before the next group), and inside a
  // group XCD-aware: workgroups b, b+8, ... share an XCD (dispatch is round-robin; speed only, never correctness), so
  // XCD x gets the group's candidate tiles cb = x (mod 8) and walks them row tile by row tile.  Groups keep the K*
  // panels the resident workgroups read to a quarter of the chunk at n = 4096: 7.65 vs 8.03 ms per launch (tools/
  // trmm_asm_bench.hip A4 vs A2, profiles/r05_trmm_asm_groups.log; groups of 16 / 32 / 128: 8.17 / 7.91 / 7.82 ms).
  const int b = blockIdx.x;
  int I, cb;
  constexpr int G = 64;
  if ((ncb % G) == 0) {
    const int g = b / (nI * G), bb = b % (nI * G);
    const int x = bb & 7, l = bb >> 3;
    I = nI - 1 - l / (G / 8);
    cb = g * G + 8 * (l % (G / 8)) + x;
  } else if ((ncb & 7) == 0) {
    const int x = b & 7, l = b >> 3, per = ncb >> 3;
    I = nI - 1 - l / per;
    cb = 8 * (l % per) + x;
  } else {
    I = nI - 1 - b / ncb;
    cb = b % ncb;
  }
  const double* Ab = W + (int64_t)I * TT;            // A(m=i,k) = W[k][I*128 + i]
  const double* Bb = kstar + (int64_t)cb * TT;       // B(k,n=c) = K*[k][cb*128 + c]
  // the k loop with a hand-placed instruction stream (gpx_trmm_asm.h; same MFMA sequence per accumulator as
  // MfmaTile::run, so the same bits); for the triangular W, the waves of rows 0-63 skip the diagonal tile's zero half
  trmm_asm::Tile tile;
  tile.run(Ab, ldw, Bb, C, (kfull ? nI : I + 1) * (TT / 16), smem, !kfull);
  // column sums of squares over this wave's rows, then over the lanes holding the same column
  double s[TrmmTile::WN];
#pragma unroll
  for (int j = 0; j < TrmmTile::WN; ++j) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < TrmmTile::WM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += tile.acc[i][j][r] * tile.acc[i][j][r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    s[j] = v;
  }
  // the two waves of each column half (w>>1 = 0, 1) combine through LDS (smem is free after run())
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* red = smem;
  if ((w >> 1) == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < TrmmTile::WN; ++j) red[TrmmTile::col_of(j)] = s[j];
  }
  __syncthreads();
  if ((w >> 1) == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < TrmmTile::WN; ++j) {
      const int col = TrmmTile::col_of(j);
      ss_part[(int64_t)I * C + (int64_t)cb * TT + col] = s[j] + red[col];
    }
  }
}

// ---- 1+2 fused, small n (npad <= 256) ----------------------------------------------------------
// At small n the K* round trip through HBM and the 128-row trmm tiles (whose triangle is at most two tiles deep)
// cost more than the product (profiles/r01_small_n_rates.log, n = 256: kstar 2.2 + trmm 6.4 ms per 2^22 candidates
// at 43 TF/s).  Here one wave owns 16 candidates and walks k in steps of 4: each lane evaluates K*[k][c]
// (k = k0 + lane/16, c = lane%16) straight into the B operand of v_mfma_f64_16x16x4 (no K* buffer), and the A
// operands W[k][16 ib + lane%16] of the row blocks ib >= k/16 come from L2 (W is npad^2 fp64 <= 512 KiB, shared by
// every workgroup).  The triangle is walked in 16-row blocks, so the diagonal waste is 1/16 instead of 1/2 of a
// 128-row tile.  Outputs per candidate: mu (alpha^T K* per output, no constant mean) and ss = |W^T K*|^2, in the
// layout of one mu_part / ss_part block so finalize_kernel runs unchanged with nJB = nI = 1.  The summation order differs from the
// unfused path (both are checked against the oracle at the same tolerance).
// NR = 1 (acquisition, single-output posterior) or GPX_MAX_RHS (multi-output posterior, alpha zero-padded to 8 columns
// so the mean loop has no nrhs test; mu_out[q][c] for q < nrhs).
template <int NPAD, int DMAX, int KIND, int NR>
__global__ void __launch_bounds__(WG) sweep_small_kernel(gpx_kernel_params p, int n, const double* __restrict__ X,
                                                         int64_t ldx, const double* __restrict__ alpha, int nrhs,
                                                         const double* __restrict__ W, int64_t ldw,
                                                         const double* __restrict__ Xs, int64_t ldxs, int64_t m_chunk,
                                                         int64_t C, double* __restrict__ mu_out,
                                                         double* __restrict__ ss_out) {
  constexpr int NRB = NPAD / 16;
  constexpr int KS = DMAX / 4;
  constexpr bool LIN = KIND == GPX_KERNEL_SCALE_LINEAR_MATERN52;
  // XT: the distance's cross term on MFMA (gram_mfma_kernel's arithmetic, centred by the mean of the training inputs):
  // 1.745e9 / 1.784e9 vs 1.651e9 / 1.698e9 candidates/s at n = 64 / 128, but 4.60e8 vs 5.81e8 at n = 256, where the
  // dot operands beside 16 accumulator blocks cost occupancy (tools/small_n_rates.py, profiles/r04_small_n_xterm_ab.log);
  // npad = 256 keeps the difference form.
  constexpr bool XT = NPAD <= 128;
  __shared__ double sx[NPAD][DMAX + 1], sr[LIN ? NPAD : 1][DMAX + 1], sa[NPAD][NR], sn[XT ? NPAD : 1], cen[DMAX];
  const int d = p.d, t = threadIdx.x;
  for (int e = t; e < NPAD * DMAX; e += WG) {
    const int r = e / DMAX, k = e % DMAX;
    const double v = (k < d && r < n) ? X[(int64_t)r * ldx + k] : 0.0;
    sx[r][k] = (k < d) ? v / p.lengthscale[k] : 0.0;
    if constexpr (LIN) sr[r][k] = (k < d) ? v * p.linear_variance[k] : 0.0;
  }
  for (int e = t; e < NPAD * NR; e += WG) {
    const int r = e / NR, q = e % NR;
    sa[r][q] = (r < n && q < nrhs) ? alpha[(int64_t)r * nrhs + q] : 0.0;
  }
  __syncthreads();
  if constexpr (XT) {
    if (t < DMAX) {
      double s = 0.0;
      for (int r = 0; r < n; ++r) s += sx[r][t];
      cen[t] = n > 0 ? s / n : 0.0;
    }
    __syncthreads();
    for (int e = t; e < NPAD * DMAX; e += WG) sx[e / DMAX][e % DMAX] -= cen[e % DMAX];
    __syncthreads();
    for (int r = t; r < NPAD; r += WG) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) v = fma(sx[r][k], sx[r][k], v);
      sn[r] = v;
    }
    __syncthreads();
  }
  const int lane = t & 63, w = t >> 6;
  const int kr = lane >> 4, m = lane & 15;
  const int64_t c = ((int64_t)blockIdx.x * (WG / 64) + w) * 16 + m;
  const bool valid = c < m_chunk;
  // XT: this lane's B operands of the dot (candidate m, dimensions 4 s + kr) and the candidate's squared norm; else the
  // candidate's whole point (difference form, one K* element per lane and k-step)
  double bo[XT ? KS : 1], br[XT ? KS : 1], nb = 0.0;
  double xs[XT ? 1 : DMAX], xr[XT ? 1 : DMAX];
  if constexpr (XT) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + kr;
      const double v = (valid && k < d) ? Xs[c * ldxs + k] : 0.0;
      bo[s] = (k < d) ? v / p.lengthscale[k] - cen[k] : 0.0;
      br[s] = v;
      nb = fma(bo[s], bo[s], nb);
    }
    nb += __shfl_xor(nb, 16);
    nb += __shfl_xor(nb, 32);
  } else {
    load_point<DMAX>(p, Xs + (valid ? c * ldxs : 0), valid, xs, xr);
  }
  d4 acc[NRB];
#pragma unroll
  for (int ib = 0; ib < NRB; ++ib) acc[ib] = (d4){0.0, 0.0, 0.0, 0.0};
  double mu[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) mu[q] = 0.0;
  const double* __restrict__ Wl = W + (int64_t)kr * ldw + (lane & 15);
#pragma unroll
  for (int kb = 0; kb < NRB; ++kb) {
    // XT: a.b for the 16 rows of block kb x the wave's 16 candidates; register r of the accumulator holds row
    // 16 kb + kr + 4 r of candidate m, i.e. exactly the B operand of k-step r below
    d4 dot = {0.0, 0.0, 0.0, 0.0}, lac = {0.0, 0.0, 0.0, 0.0};
    if constexpr (XT) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        dot = mfma16x16x4(sx[16 * kb + m][4 * s + kr], bo[s], dot);
        if constexpr (LIN) lac = mfma16x16x4(sr[16 * kb + m][4 * s + kr], br[s], lac);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k0 = 16 * kb + 4 * ks;
      const int j = k0 + kr;
      double kv;
      if constexpr (XT) {
        kv = cov_from_r2(KIND, p.outputscale, sqdist_expanded(sn[j], nb, dot[ks]), LIN ? lac[ks] : 0.0);
      } else {
        double r2 = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          const double df = sx[j][k] - xs[k];
          r2 += df * df;
        }
        double lv = 0.0;
        if constexpr (LIN) {
#pragma unroll
          for (int k = 0; k < DMAX; ++k) lv += sr[j][k] * xr[k];
        }
        kv = cov_from_r2(KIND, p.outputscale, r2, lv);
      }
      kv = j < n ? kv : 0.0;
#pragma unroll
      for (int q = 0; q < NR; ++q) mu[q] += sa[j][q] * kv;
#pragma unroll
      for (int ib = kb; ib < NRB; ++ib) acc[ib] = mfma16x16x4(Wl[(int64_t)k0 * ldw + 16 * ib], kv, acc[ib]);
    }
  }
  double s = 0.0;
#pragma unroll
  for (int ib = 0; ib < NRB; ++ib)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += acc[ib][r] * acc[ib][r];
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    mu[q] += __shfl_xor(mu[q], 16);
    mu[q] += __shfl_xor(mu[q], 32);
  }
  if (lane < 16 && valid) {
#pragma unroll
    for (int q = 0; q < NR; ++q)
      if (q < nrhs) mu_out[(int64_t)q * C + c] = mu[q];
    ss_out[c] = s;
  }
}

// ---- 3. finalize: posterior (mode 0) or acquisition + block argmax (mode 1) ------------------------------
struct FinalizeArgs {
  gpx_kernel_params p;
  double y_mean[GPX_MAX_RHS];
  double y_scale[GPX_MAX_RHS];
  int acq_kind;
  double best_f, beta;
  // modes 2 / 3: a linear objective sum_t w_t f_t over T independent GPs (gpx_acquire_argmax_multi_f64)
  double weight;     // mode 2: w_t of this output
  int first;         // mode 2: the first output of the chunk (overwrites the accumulators)
  double* acc_mu;    // sum_t w_t (y_mean_t + y_scale_t mu_t)                 (chunk-sized)
  double* acc_var;   // sum_t w_t^2 y_scale_t^2 max(k** - |v_t|^2, 1e-10)      (chunk-sized)
};

// mode 0: posterior (mean / variance out); 1: acquisition + 256-candidate block argmax; 2: one output of a multi-output
// objective into the accumulators; 3: acquisition + block argmax of the accumulated objective (no partials read).
// Variance floors: GPyTorch's 1e-10 per output in the standardised space, BoTorch's 1e-12 on the scored variance
// [upstream] (T = 1, w = 1: modes 2 + 3 give mode 1's value bit for bit).
__global__ void __launch_bounds__(WG) finalize_kernel(FinalizeArgs fa, int mode, const double* __restrict__ Xs,
                                                      int64_t ldxs, int64_t m_chunk, int64_t C, int nrhs, int nJB,
                                                      int nI, const double* __restrict__ mu_part,
                                                      const double* __restrict__ ss_part,
                                                      double* __restrict__ mean_out, int64_t ldmean,
                                                      double* __restrict__ var_out, double* __restrict__ scores_out,
                                                      double* __restrict__ rec_val, int64_t* __restrict__ rec_idx,
                                                      int64_t index_base) {
  const gpx_kernel_params& p = fa.p;
  const int64_t c = (int64_t)blockIdx.x * WG + threadIdx.x;
  const bool valid = c < m_chunk;
  double score = -INFINITY;
  if (valid) {
    double mu, var;
    if (mode == 3) {
      mu = fa.acc_mu[c];
      var = fmax(fa.acc_var[c], 1e-12);
    } else {
      // prior variance k(x, x)
      double kd = p.outputscale;
      if (p.kind == GPX_KERNEL_SCALE_LINEAR_MATERN52) {
        double lv = 0.0;
        for (int k = 0; k < p.d; ++k) {
          const double v = Xs[c * ldxs + k];
          lv += v * v * p.linear_variance[k];
        }
        kd = p.outputscale * (lv + 1.0);
      }
      const double ss = sum_partials(ss_part + c, nI, C);
      var = fmax(kd - ss, 1e-10);  // gpytorch min_variance (float64) [upstream]
      if (mode == 0) {
        for (int q = 0; q < nrhs; ++q) {
          double mq = sum_partials(mu_part + (int64_t)q * C + c, nJB, (int64_t)nrhs * C);
          mq += p.const_mean;
          mean_out[c * ldmean + q] = fa.y_mean[q] + fa.y_scale[q] * mq;
        }
        var_out[c] = fmax(var * (fa.y_scale[0] * fa.y_scale[0]), 1e-12);  // BoTorch min_var [upstream]
        return;
      }
      mu = sum_partials(mu_part + c, nJB, C);
      mu = fa.y_mean[0] + fa.y_scale[0] * (mu + p.const_mean);
      var = var * (fa.y_scale[0] * fa.y_scale[0]);
      if (mode == 2) {
        const double wm = fa.weight * mu, wv = (fa.weight * fa.weight) * var;
        fa.acc_mu[c] = fa.first ? wm : fa.acc_mu[c] + wm;
        fa.acc_var[c] = fa.first ? wv : fa.acc_var[c] + wv;
        return;
      }
      var = fmax(var, 1e-12);
    }
    score = acq_score(fa.acq_kind, mu, var, fa.best_f, fa.beta);
    if (scores_out) scores_out[c] = score;
    if (score != score) score = -INFINITY;
  }
  if (mode == 0 || mode == 2) return;
  // block argmax
  double bv = score;
  int64_t bi = valid ? index_base + c : INT64_MAX;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(bv, o);
    const int64_t i2 = __shfl_xor(bi, o);
    argmax_merge(bv, bi, v2, i2);
  }
  __shared__ double wv[4];
  __shared__ int64_t wi[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    wv[w] = bv;
    wi[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) argmax_merge(bv, bi, wv[q], wi[q]);
    rec_val[blockIdx.x] = bv;
    rec_idx[blockIdx.x] = bi;
  }
}

// records e = 0 .. count-1 at vals[e * stride] / idx[e * stride] (stride 1: separate arrays; 2: packed 16-byte
// (value, index) records of the cross-GPU exchange)
__global__ void __launch_bounds__(WG) argmax_final_kernel(const double* __restrict__ vals,
                                                          const int64_t* __restrict__ idx, int64_t count,
                                                          int stride, double* __restrict__ best_val,
                                                          int64_t* __restrict__ best_idx) {
  double bv = -INFINITY;
  int64_t bi = INT64_MAX;
  for (int64_t e = threadIdx.x; e < count; e += WG) {
    double v = vals[e * stride];
    if (v != v) v = -INFINITY;
    argmax_merge(bv, bi, v, idx[e * stride]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(bv, o);
    const int64_t i2 = __shfl_xor(bi, o);
    argmax_merge(bv, bi, v2, i2);
  }
  __shared__ double wv[4];
  __shared__ int64_t wi[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    wv[w] = bv;
    wi[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) argmax_merge(bv, bi, wv[q], wi[q]);
    *best_val = bv;
    *best_idx = bi;
  }
}

// ---- host side -------------------------------------------------------------------------------------------
int64_t sweep_chunk_size(int64_t npad, int64_t m) {
  // K* chunk of at most ~1 GiB, multiple of 256 candidates (tools/chunk_sweep.sh at n = 4096: 256 MiB / 8192
  // candidates -> 3.74e6, 512 MiB -> 3.78e6, 1 GiB / 32768 -> 3.81e6, 2 GiB / 65536 -> 3.73e6 candidates/s: fewer
  // launch tails and K* / finalize launches until K* outgrows what the Infinity Cache keeps warm for the trmm
  // re-reads).  The byte budget alone sets small-n chunks (tools/small_n_rates.py, 2^22 candidates: a 32768 cap
  // left n = 64 / 256 launch-bound at 3.4e8 / 2.5e8 candidates/s, 1.15e9 / 4.4e8 without it).
  int64_t cap = ((int64_t)1 << 30) / 8 / npad;
  cap = (cap / 256) * 256;
  if (cap < 256) cap = 256;
  if (cap > ((int64_t)1 << 20)) cap = (int64_t)1 << 20;
  int64_t need = ((m + 255) / 256) * 256;
  if (need < 256) need = 256;
  return need < cap ? need : cap;
}

size_t sweep_workspace_bytes(int64_t npad, int64_t nrhs, int64_t m) {
  const int64_t C = sweep_chunk_size(npad, m);
  const int64_t nrec = (m + 255) / 256 + 1;
  size_t b = 0;
  b += (size_t)npad * C * 8;                 // kstar
  b += (size_t)(npad / NB) * nrhs * C * 8;   // mu_part
  b += (size_t)(npad / TT) * C * 8;          // ss_part
  b += (size_t)nrec * 16;                    // records
  return b + 256;
}

// The fused small-n sweep covers npad <= 256, d <= 16 (1..8 outputs) and the fp64 covariance build; the rest takes
// the K* + trmm path.  An npad = 384 instance (d <= 8, 226 VGPRs, 2 waves/SIMD) measured slower than the K* + trmm path
// (2.20e8 vs 2.66e8 candidates/s at n = 384, profiles/r01_small_n_rates.log): 24 row blocks of A operands per k-step
// from L2 and half the occupancy of the npad = 256 instance.  The handle option GPX_OPT_SWEEP_FUSED = 0 forces the
// unfused path (A/B measurements, parity tests of both paths).
bool sweep_fused_ok(const Context* c, const gpx_kernel_params& p, int npad, int nrhs) {
  return c->sweep_fused && (npad == 128 || npad == 256) && p.d <= 16 && !p.cov_fp32;
}

hipError_t launch_sweep_chunk(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                              const double* W, int64_t ldw, const double* alpha, int nrhs, const double* Xs,
                              int64_t ldxs, int64_t m_chunk, const SweepBuffers& b, int mode,
                              const gpx_acq_params* a, const double* y_mean, const double* y_scale,
                              double* mean_out, int64_t ldmean, double* var_out, double* scores_out,
                              int64_t rec_offset, int64_t index_offset, const MultiOutput* mo) {
  const int64_t C = b.chunk;
  int nJB = npad / NB, nI = npad / TT;
  const int ncb = (int)((m_chunk + WG - 1) / WG);  // 256-candidate blocks actually used in this chunk
  if (sweep_fused_ok(c, p, npad, nrhs)) {
    LaunchTimer tm(c, GPX_TIMER_TRMM);
    const int nwg = (int)((m_chunk + 63) / 64);
#define GPX_SMALL_K(NP, D, K)                                                                                       \
  (nrhs == 1 ? sweep_small_kernel<NP, D, K, 1><<<nwg, WG, 0, c->stream>>>(p, n, X, ldx, alpha, nrhs, W, ldw, Xs, ldxs,  \
                                                                           m_chunk, C, b.mu_part, b.ss_part)          \
             : sweep_small_kernel<NP, D, K, GPX_MAX_RHS><<<nwg, WG, 0, c->stream>>>(                                  \
                   p, n, X, ldx, alpha, nrhs, W, ldw, Xs, ldxs, m_chunk, C, b.mu_part, b.ss_part))
#define GPX_SMALL_D(NP, D)                                                                                          \
  (p.kind == GPX_KERNEL_RBF        ? GPX_SMALL_K(NP, D, GPX_KERNEL_RBF)                                             \
   : p.kind == GPX_KERNEL_MATERN52 ? GPX_SMALL_K(NP, D, GPX_KERNEL_MATERN52)                                        \
                                   : GPX_SMALL_K(NP, D, GPX_KERNEL_SCALE_LINEAR_MATERN52))
#define GPX_SMALL(NP) (p.d <= 4 ? GPX_SMALL_D(NP, 4) : p.d <= 8 ? GPX_SMALL_D(NP, 8) : GPX_SMALL_D(NP, 16))
    if (npad == 128)
      GPX_SMALL(128);
    else
      GPX_SMALL(256);
#undef GPX_SMALL
#undef GPX_SMALL_D
#undef GPX_SMALL_K
    nJB = nI = 1;
  } else {
    {
    LaunchTimer tm(c, GPX_TIMER_KSTAR);
    dim3 g(ncb, nJB);
#define GPX_KSTAR_K(D, F, K)                                                                                     \
  (nrhs == 1 ? kstar_kernel<D, F, K, true><<<g, WG, 0, c->stream>>>(p, n, X, ldx, alpha, nrhs, Xs, ldxs, m_chunk, C, \
                                                                    b.kstar, b.mu_part)                            \
             : kstar_kernel<D, F, K, false><<<g, WG, 0, c->stream>>>(p, n, X, ldx, alpha, nrhs, Xs, ldxs, m_chunk, \
                                                                     C, b.kstar, b.mu_part))
#define GPX_KSTAR_F(D, F)                                                                                          \
  (p.kind == GPX_KERNEL_RBF        ? GPX_KSTAR_K(D, F, GPX_KERNEL_RBF)                                             \
   : p.kind == GPX_KERNEL_MATERN52 ? GPX_KSTAR_K(D, F, GPX_KERNEL_MATERN52)                                        \
                                   : GPX_KSTAR_K(D, F, GPX_KERNEL_SCALE_LINEAR_MATERN52))
#define GPX_KSTAR_M(D, K)                                                                                          \
  (nrhs == 1 ? kstar_mfma_kernel<D, K, true><<<g, WG, 0, c->stream>>>(p, n, X, ldx, alpha, nrhs, Xs, ldxs, m_chunk, C, \
                                                                      b.kstar, b.mu_part)                            \
             : kstar_mfma_kernel<D, K, false><<<g, WG, 0, c->stream>>>(p, n, X, ldx, alpha, nrhs, Xs, ldxs, m_chunk,  \
                                                                       C, b.kstar, b.mu_part))
#define GPX_KSTAR_MK(D)                                                                                            \
  (p.kind == GPX_KERNEL_RBF        ? GPX_KSTAR_M(D, GPX_KERNEL_RBF)                                                \
   : p.kind == GPX_KERNEL_MATERN52 ? GPX_KSTAR_M(D, GPX_KERNEL_MATERN52)                                           \
                                   : GPX_KSTAR_M(D, GPX_KERNEL_SCALE_LINEAR_MATERN52))
#define GPX_KSTAR(D) (p.cov_fp32 ? GPX_KSTAR_F(D, true) : GPX_KSTAR_MK(D))
    if (p.d <= 4)
      GPX_KSTAR(4);
    else if (p.d <= 8)
      GPX_KSTAR(8);
    else if (p.d <= 16)
      GPX_KSTAR(16);
    else  // d > 16: the difference form (the MFMA kernel's candidate tile would not fit 64 KB of LDS)
      p.cov_fp32 ? GPX_KSTAR_F(32, true) : GPX_KSTAR_F(32, false);
#undef GPX_KSTAR_MK
#undef GPX_KSTAR_M
#undef GPX_KSTAR
#undef GPX_KSTAR_F
#undef GPX_KSTAR_K
  }
  {
    LaunchTimer tm(c, GPX_TIMER_TRMM);
    const int ncbt = (int)((m_chunk + TT - 1) / TT);
    trmm_sumsq_kernel<<<ncbt * nI, WG, 0, c->stream>>>(W, ldw, b.kstar, C, nI, ncbt, b.ss_part, 0);
  }
  }
  {
    LaunchTimer tm(c, GPX_TIMER_ACQ);
    FinalizeArgs fa;
    fa.p = p;
    for (int q = 0; q < GPX_MAX_RHS; ++q) {
      fa.y_mean[q] = (y_mean && q < nrhs) ? y_mean[q] : 0.0;
      fa.y_scale[q] = (y_scale && q < nrhs) ? y_scale[q] : 1.0;
    }
    fa.acq_kind = a ? a->kind : 0;
    fa.best_f = a ? a->best_f : 0.0;
    fa.beta = a ? a->beta : 0.0;
    if (a) {
      fa.y_mean[0] = a->y_mean;
      fa.y_scale[0] = a->y_scale;
    }
    fa.weight = 1.0;
    fa.first = 0;
    fa.acc_mu = fa.acc_var = nullptr;
    if (mo) {  // one output of a multi-output objective: accumulate, score later (launch_multi_score)
      mode = 2;
      fa.y_mean[0] = mo->y_mean;
      fa.y_scale[0] = mo->y_scale;
      fa.weight = mo->weight;
      fa.first = mo->first;
      fa.acc_mu = mo->acc_mu;
      fa.acc_var = mo->acc_var;
    }
    finalize_kernel<<<ncb, WG, 0, c->stream>>>(fa, mode, Xs, ldxs, m_chunk, C, nrhs, nJB, nI, b.mu_part,
                                                   b.ss_part, mean_out, ldmean, var_out, scores_out,
                                                   b.rec_val + rec_offset, b.rec_idx + rec_offset,
                                                   index_offset);
  }
  return hipGetLastError();
}

hipError_t launch_multi_score(Context* c, const MultiOutput& mo, const gpx_acq_params& a, int64_t m_chunk,
                              double* scores_out, double* rec_val, int64_t* rec_idx, int64_t index_offset) {
  LaunchTimer tm(c, GPX_TIMER_ACQ);
  FinalizeArgs fa{};
  fa.acq_kind = a.kind;
  fa.best_f = a.best_f;
  fa.beta = a.beta;
  fa.acc_mu = mo.acc_mu;
  fa.acc_var = mo.acc_var;
  const int ncb = (int)((m_chunk + WG - 1) / WG);
  finalize_kernel<<<ncb, WG, 0, c->stream>>>(fa, 3, nullptr, 0, m_chunk, 0, 1, 0, 0, nullptr, nullptr, nullptr, 0,
                                             nullptr, scores_out, rec_val, rec_idx, index_offset);
  return hipGetLastError();
}

// ---- SVGP predictive: one task of Bayesian7's batched SVGP over a chunk --------------------
// mean = const + K_*Z alpha' (alpha' = L^{-T} m), var = k** - |L^{-1} k*|^2 + |S^T L^{-1} k*|^2 + noise, i.e. the
// whitened VariationalStrategy predictive k** + k*^T L^{-T} (S S^T - I) L^{-1} k* plus the GaussianLikelihood noise
// [upstream]; score (optional) accumulates sum_t var_t over the tasks (the pool-scan score, Bayesian7.py:671).
__global__ void __launch_bounds__(WG) svgp_finalize_kernel(gpx_kernel_params p, double min_var, int task,
                                                           const double* __restrict__ Xs, int64_t ldxs,
                                                           int64_t m_chunk, int64_t C, int nJB, int nI,
                                                           const double* __restrict__ mu_part,
                                                           const double* __restrict__ ss1,
                                                           const double* __restrict__ ss2,
                                                           double* __restrict__ mean_out, int64_t ldmean,
                                                           double* __restrict__ var_out, int64_t ldvar,
                                                           double* __restrict__ score) {
  const int64_t c = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (c >= m_chunk) return;
  double kd = p.outputscale;
  if (p.kind == GPX_KERNEL_SCALE_LINEAR_MATERN52) {
    double lv = 0.0;
    for (int k = 0; k < p.d; ++k) {
      const double v = Xs[c * ldxs + k];
      lv += v * v * p.linear_variance[k];
    }
    kd = p.outputscale * (lv + 1.0);
  }
  const double s1 = sum_partials(ss1 + c, nI, C);
  const double s2 = sum_partials(ss2 + c, nI, C);
  const double var = fmax(kd - s1 + s2 + p.noise, min_var);
  const double mu = sum_partials(mu_part + c, nJB, C) + p.const_mean;
  if (mean_out) mean_out[c * ldmean + task] = mu;
  if (var_out) var_out[c * ldvar + task] = var;
  if (score) score[c] = (task == 0 ? 0.0 : score[c]) + var;
}

hipError_t launch_svgp_chunk(Context* c, const gpx_kernel_params& p, double min_var, int task, int M, int Mpad,
                             const double* Z, int64_t ldz, const double* W, const double* W2, int64_t ldw,
                             const double* alpha, const double* Xs, int64_t ldxs, int64_t m_chunk,
                             const SweepBuffers& b, double* ss2, double* mean_out, int64_t ldmean, double* var_out,
                             int64_t ldvar, double* score) {
  const int64_t C = b.chunk;
  const int nJB = Mpad / NB, nI = Mpad / TT;
  const int ncb = (int)((m_chunk + WG - 1) / WG);
  {
    LaunchTimer tm(c, GPX_TIMER_KSTAR);
    dim3 g(ncb, nJB);
#define GPX_KSTAR_K(D, K) \
  kstar_kernel<D, false, K, true><<<g, WG, 0, c->stream>>>(p, M, Z, ldz, alpha, 1, Xs, ldxs, m_chunk, C, b.kstar, b.mu_part)
#define GPX_KSTAR(D)                                                                         \
  (p.kind == GPX_KERNEL_RBF        ? GPX_KSTAR_K(D, GPX_KERNEL_RBF)                          \
   : p.kind == GPX_KERNEL_MATERN52 ? GPX_KSTAR_K(D, GPX_KERNEL_MATERN52)                     \
                                   : GPX_KSTAR_K(D, GPX_KERNEL_SCALE_LINEAR_MATERN52))
    if (p.d <= 4)
      GPX_KSTAR(4);
    else if (p.d <= 8)
      GPX_KSTAR(8);
    else if (p.d <= 16)
      GPX_KSTAR(16);
    else
      GPX_KSTAR(32);
#undef GPX_KSTAR
#undef GPX_KSTAR_K
  }
  {
    LaunchTimer tm(c, GPX_TIMER_TRMM);
    const int ncbt = (int)((m_chunk + TT - 1) / TT);
    trmm_sumsq_kernel<<<dim3(ncbt * nI, 2), WG, 0, c->stream>>>(W, ldw, b.kstar, C, nI, ncbt, b.ss_part, 0, W2, ss2);
  }
  {
    LaunchTimer tm(c, GPX_TIMER_ACQ);
    svgp_finalize_kernel<<<ncb, WG, 0, c->stream>>>(p, min_var, task, Xs, ldxs, m_chunk, C, nJB, nI, b.mu_part,
                                                    b.ss_part, ss2, mean_out, ldmean, var_out, ldvar, score);
  }
  return hipGetLastError();
}

hipError_t launch_argmax_final(Context* c, const double* vals, const int64_t* idx, int64_t count, double* best_val,
                               int64_t* best_idx) {
  LaunchTimer tm(c, GPX_TIMER_ACQ);
  argmax_final_kernel<<<1, WG, 0, c->stream>>>(vals, idx, count, 1, best_val, best_idx);
  return hipGetLastError();
}

// (best_val, best_idx) -> one 16-byte record {double value; int64 index} (the send buffer of the exchange)
__global__ void record_pack_kernel(const double* __restrict__ best_val, const int64_t* __restrict__ best_idx,
                                   int64_t* __restrict__ rec) {
  if (threadIdx.x == 0) {
    rec[0] = __double_as_longlong(*best_val);
    rec[1] = *best_idx;
  }
}

hipError_t launch_record_pack(Context* c, const double* best_val, const int64_t* best_idx, int64_t* rec) {
  record_pack_kernel<<<1, 64, 0, c->stream>>>(best_val, best_idx, rec);
  return hipGetLastError();
}

hipError_t launch_argmax_records(Context* c, const int64_t* rec, int64_t count, double* best_val, int64_t* best_idx) {
  LaunchTimer tm(c, GPX_TIMER_ACQ);
  argmax_final_kernel<<<1, WG, 0, c->stream>>>(reinterpret_cast<const double*>(rec), rec + 1, count, 2, best_val,
                                               best_idx);
  return hipGetLastError();
}

}  // namespace gpx
