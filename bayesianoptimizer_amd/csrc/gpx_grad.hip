// Posterior moments of q-batches of candidates and their derivatives w.r.t. the candidate inputs: the GPU side of
// gradient-based acquisition optimisation (SURVEY §8f row 4 — optimize_acqf's L-BFGS-B restarts on qLogEI,
// optimization/Bayesian.py:100-112, optimization/Bayesian2.py:218-245; BoTorch differentiates the exact GP posterior
// with torch autograd [upstream]).  For candidates x_a (rows of Xs, consecutive q-batches) and c in a's batch:
//   mean[a]        = m + k_a^T alpha                    dmean[a][j]   = sum_i d1k(x_a, X_i)/dx_aj alpha_i
//   cov[a][c]      = k(x_a, x_c) - k_a^T K^{-1} k_c     dcov[a][j][c] = d1k(x_a, x_c)/dx_aj - sum_i d1k(x_a, X_i)/dx_aj s_ic
// with s_c = K^{-1} k_c = W (W^T k_c) (two triangular fp64-MFMA products over npad x mpad, gpx_gemm.h) and d1k the
// partial derivative in the kernel's FIRST argument.  The chain rule through the symmetric q x q covariance is then
//   dL/dx_aj = gmean[a] dmean[a][j] + sum_c (gcov[a][c] + gcov[c][a]) dcov[a][j][c]
// (bayesianoptimizer_amd/acqf.py), the diagonal included (d k(x,x) = 2 d1k(x,x) by symmetry).
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_gemm.h"

namespace gpx {

// K*[i][c] = k(X_i, Xs_c) for i < n, c < m; 0 elsewhere (npad x mpad, row length mpad).
__global__ void __launch_bounds__(WG) kstar_plain_kernel(gpx_kernel_params p, int n, int npad, int m, int mpad,
                                                         const double* __restrict__ X, int64_t ldx,
                                                         const double* __restrict__ Xs, int64_t ldxs,
                                                         double* __restrict__ Ks) {
  const int64_t e = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (e >= (int64_t)npad * mpad) return;
  const int i = (int)(e / mpad), c = (int)(e % mpad);
  double v = 0.0;
  if (i < n && c < m) {
    const bool lin = p.kind == GPX_KERNEL_SCALE_LINEAR_MATERN52;
    double r2 = 0.0, lv = 0.0;
    for (int k = 0; k < p.d; ++k) {
      const double a = X[(int64_t)i * ldx + k], b = Xs[(int64_t)c * ldxs + k];
      const double df = a / p.lengthscale[k] - b / p.lengthscale[k];
      r2 += df * df;
      if (lin) lv += a * p.linear_variance[k] * b;
    }
    v = cov_from_r2(p.kind, p.outputscale, r2, lv);
  }
  Ks[e] = v;
}

// k(a, b) and d1k(a, b)/da_j for j < d (a = the candidate, b = a training point or another candidate).
template <int DMAX>
__device__ __forceinline__ double cov_and_grad(const gpx_kernel_params& p, const double* a, const double* b,
                                               double (&g)[DMAX]) {
  double r2 = 0.0, lv = 0.0;
  const bool lin = p.kind == GPX_KERNEL_SCALE_LINEAR_MATERN52;
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    g[k] = 0.0;
    if (k < p.d) {
      const double df = b[k] / p.lengthscale[k] - a[k] / p.lengthscale[k];
      r2 += df * df;
      if (lin) lv += b[k] * p.linear_variance[k] * a[k];
    }
  }
  const double kv = cov_from_r2(p.kind, p.outputscale, r2, lv);
  // d/da_j of the stationary part = coef * (a_j - b_j) / l_j^2
  double coef;
  if (p.kind == GPX_KERNEL_RBF) {
    coef = -kv;
  } else {
    const double r = sqrt(r2);
    const double s5r = 2.23606797749978969640917366873128 * r;
    coef = -p.outputscale * (5.0 / 3.0) * (1.0 + s5r) * exp(-s5r);
  }
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    if (k < p.d) {
      const double l = p.lengthscale[k];
      g[k] = coef * (a[k] / l - b[k] / l) / l;
      if (lin) g[k] += p.outputscale * p.linear_variance[k] * b[k];
    }
  }
  return kv;
}

// Deterministic 256-thread sum of `cnt` per-thread values (wave shuffles, then the 4 wave partials in order).
template <int CNT>
__device__ __forceinline__ void block_sum(double (&v)[CNT], double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < CNT; ++q) {
    double s = v[q];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[w * CNT + q] = s;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < CNT; ++q) v[q] = ((red[q] + red[CNT + q]) + red[2 * CNT + q]) + red[3 * CNT + q];
  __syncthreads();
}

// One workgroup per (candidate a = blockIdx.y, batch member cc = blockIdx.x).
template <int DMAX>
__global__ void __launch_bounds__(WG) moments_grad_kernel(gpx_kernel_params p, int n, const double* __restrict__ X,
                                                          int64_t ldx, const double* __restrict__ alpha,
                                                          const double* __restrict__ Xs, int64_t ldxs, int q,
                                                          const double* __restrict__ S, int mpad,
                                                          double* __restrict__ mean, double* __restrict__ dmean,
                                                          double* __restrict__ cov, double* __restrict__ dcov) {
  __shared__ double red[4 * (2 * DMAX + 2)];
  const int a = blockIdx.y, cc = blockIdx.x;
  const int c = (a / q) * q + cc;  // batch member
  const int d = p.d;
  double xa[DMAX], xc[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    xa[k] = (k < d) ? Xs[(int64_t)a * ldxs + k] : 0.0;
    xc[k] = (k < d) ? Xs[(int64_t)c * ldxs + k] : 0.0;
  }
  const bool first = (cc == 0);
  // acc[0] = sum k s_ic, acc[1..d] = sum dk s_ic, acc[DMAX+1] = sum k alpha_i, acc[DMAX+2..] = sum dk alpha_i
  double acc[2 * DMAX + 2];
#pragma unroll
  for (int q2 = 0; q2 < 2 * DMAX + 2; ++q2) acc[q2] = 0.0;
  for (int i = threadIdx.x; i < n; i += WG) {
    double xi[DMAX], g[DMAX];
#pragma unroll
    for (int k = 0; k < DMAX; ++k) xi[k] = (k < d) ? X[(int64_t)i * ldx + k] : 0.0;
    const double kv = cov_and_grad<DMAX>(p, xa, xi, g);
    const double s = S[(int64_t)i * mpad + c];
    acc[0] += kv * s;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) acc[1 + k] += g[k] * s;
    if (first) {
      const double al = alpha[i];
      acc[DMAX + 1] += kv * al;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) acc[DMAX + 2 + k] += g[k] * al;
    }
  }
  block_sum<2 * DMAX + 2>(acc, red);
  if (threadIdx.x != 0) return;
  double gp[DMAX];
  const double kac = cov_and_grad<DMAX>(p, xa, xc, gp);
  cov[(int64_t)a * q + cc] = kac - acc[0];
  for (int k = 0; k < d; ++k) dcov[((int64_t)a * d + k) * q + cc] = gp[k] - acc[1 + k];
  if (first) {
    mean[a] = p.const_mean + acc[DMAX + 1];
    for (int k = 0; k < d; ++k) dmean[(int64_t)a * d + k] = acc[DMAX + 2 + k];
  }
}

size_t moments_grad_ws_doubles(int npad, int m) {
  const int mpad = ((m + NB - 1) / NB) * NB;
  const size_t blk = (size_t)npad * mpad;
  size_t p1 = gemm_split_doubles(npad, mpad, npad);
  return 3 * blk + p1 + 64;
}

hipError_t launch_moments_grad(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                               const double* W, int64_t ldw, const double* alpha, const double* Xs, int64_t ldxs,
                               int m, int q, double* mean, double* dmean, double* cov, double* dcov, double* ws) {
  const int mpad = ((m + NB - 1) / NB) * NB;
  const size_t blk = (size_t)npad * mpad;
  double* Ks = ws;
  double* V = Ks + blk;
  double* S = V + blk;
  double* P = S + blk;
  const int64_t tot = (int64_t)npad * mpad;
  kstar_plain_kernel<<<(unsigned)((tot + WG - 1) / WG), WG, 0, c->stream>>>(p, n, npad, m, mpad, X, ldx, Xs, ldxs, Ks);
  // V = W^T K*  (A(r, k) = W[k][r], nonzero for k <= r)
  hipError_t e = launch_gemm64<true, true, KR_A_LOWER>(c, npad, mpad, npad, W, ldw, Ks, mpad, nullptr, 0, V, mpad, 1.0,
                                                       0, P);
  if (e != hipSuccess) return e;
  // S = W V = K^{-1} K*  (A(r, k) = W[r][k], nonzero for k >= r)
  e = launch_gemm64<false, true, KR_A_UPPER>(c, npad, mpad, npad, W, ldw, V, mpad, nullptr, 0, S, mpad, 1.0, 0, P);
  if (e != hipSuccess) return e;
  const dim3 grid(q, m);
#define GPX_MG(D)                                                                                                    \
  moments_grad_kernel<D><<<grid, WG, 0, c->stream>>>(p, n, X, ldx, alpha, Xs, ldxs, q, S, mpad, mean, dmean, cov, \
                                                     dcov)
  if (p.d <= 4)
    GPX_MG(4);
  else if (p.d <= 8)
    GPX_MG(8);
  else if (p.d <= 16)
    GPX_MG(16);
  else
    GPX_MG(32);
#undef GPX_MG
  return hipGetLastError();
}

}  // namespace gpx
