// Gram builder: K(X,X) + (noise + jitter) I, lower 64x64 tiles of the padded matrix.
// SURVEY §8a row a3 — replaces the covar_module(X) evaluation inside GPyTorch's ExactGP path [upstream]
// (optimization/Bayesian.py:91-93, optimization/Bayesian6.py:471-484).
//
// With rb0 > 0 only the tiles of row blocks >= rb0 are built (the new rows of an incremental update).
// HBM-write-bound: each 64x64 tile is written once (32 KiB); inputs are two 64 x d slices of X staged in
// LDS (lengthscale-divided copy for the stationary part, raw copy for the linear part).  Each wave owns
// one row of the tile at a time and writes 64 consecutive doubles (512 B) per store instruction.
#include "gpx_internal.h"
#include "gpx_device.h"
#include <cstdlib>
#include <type_traits>

namespace gpx {

template <int DMAX, bool F32, int KIND>
__global__ void __launch_bounds__(WG) gram_kernel(gpx_kernel_params p, int n, int t0, const double* __restrict__ X,
                                                  int64_t ldx, double* __restrict__ K, int64_t ldk, int64_t sx,
                                                  int64_t sk, int32_t* __restrict__ info,
                                                  unsigned long long* __restrict__ zero, int64_t zero_words,
                                                  double* __restrict__ mean_out) {
  // the fit's pivot-failure word is cleared here (stream-ordered before the Cholesky) instead of by a separate
  // memset dispatch (~4.7 us at small n), and so are the words of `zero` (the triangular solve's hand-off granules,
  // gpx_fit_factor_f64): one more dispatch saved.  mean_out (per-problem parameters): the problem's constant mean, read
  // by the triangular solves of the same fit (Batch::means)
  if (blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
    if (info) info[blockIdx.y] = 0;
    if (mean_out) mean_out[blockIdx.y] = p.const_mean;
  }
  if (zero) {
    const int64_t nwg = (int64_t)gridDim.x * gridDim.y * gridDim.z;
    const int64_t wg = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    for (int64_t e = wg * WG + threadIdx.x; e < zero_words; e += nwg * WG) zero[e] = 0ull;
  }
  X += blockIdx.y * sx;  // problem of a batched fit
  K += blockIdx.y * sk;
  __shared__ double si[NB][DMAX + 1], sj[NB][DMAX + 1];    // scaled x / l
  __shared__ double ri[NB][DMAX + 1], rj[NB][DMAX + 1];    // raw x (linear kernel)
  int ti, tj;
  tri_decode(t0 + (int)blockIdx.x, ti, tj);
  const int i0 = ti * NB, j0 = tj * NB;
  const int d = p.d;
  constexpr bool lin = (KIND == GPX_KERNEL_SCALE_LINEAR_MATERN52);
  for (int e = threadIdx.x; e < NB * DMAX; e += WG) {
    int r = e / DMAX, k = e % DMAX;
    double xi = 0.0, xj = 0.0;
    if (k < d) {
      if (i0 + r < n) xi = X[(int64_t)(i0 + r) * ldx + k];
      if (j0 + r < n) xj = X[(int64_t)(j0 + r) * ldx + k];
    }
    const double l = (k < d) ? p.lengthscale[k] : 1.0;
    si[r][k] = xi / l;
    sj[r][k] = xj / l;
    ri[r][k] = xi * ((k < d) ? p.linear_variance[k] : 0.0);
    rj[r][k] = xj;
  }
  __syncthreads();
  const int c = threadIdx.x & 63;
  const int gj = j0 + c;
  double xc[DMAX], rc[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    xc[k] = sj[c][k];
    rc[k] = rj[c][k];
  }
  const double diag_add = p.noise + p.jitter;
  // gridDim.z row slices per tile (small fits: more workgroups, fewer serial exp chains per thread).  The rows of a
  // thread are processed four at a time (independent distance / exp chains in flight together: the one-row loop left
  // the kernel at 0.24 of HBM, latency-bound on the fp64 exp chain); the covariance kind is a template parameter so
  // the element loop has no uniform branches.
  const int rows = NB / gridDim.z, rbeg = blockIdx.z * rows;
  const int rw = threadIdx.x >> 6;
  for (int r0 = rbeg; r0 < rbeg + rows; r0 += 16) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + rw + 4 * u;
      const int gi = i0 + r;
      double lv = 0.0;
      if (lin) {
#pragma unroll
        for (int k = 0; k < DMAX; ++k)
          if (k < d) lv += ri[r][k] * rc[k];
      }
      if (F32) {
        float r2 = 0.0f;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          if (k < d) {
            const float df = (float)si[r][k] - (float)xc[k];
            r2 += df * df;
          }
        }
        v[u] = cov_from_r2_f32(KIND, p.outputscale, r2, lv);
      } else {
        double r2 = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          if (k < d) {
            const double df = si[r][k] - xc[k];
            r2 += df * df;
          }
        }
        v[u] = cov_from_r2(KIND, p.outputscale, r2, lv);
      }
      if (gi == gj) v[u] += diag_add;
      if (gi >= n || gj >= n) v[u] = (gi == gj) ? 1.0 : 0.0;  // identity padding
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) K[(int64_t)(i0 + r0 + rw + 4 * u) * ldk + gj] = v[u];
  }
}

// fp64 covariance build with the distance's cross term on the matrix cores (GPyTorch's own arithmetic [upstream]:
// ||a||^2 + ||b||^2 - 2 a.b on centred, lengthscale-scaled inputs, clamped at 0, exactly 0 for a point with itself).
// The difference form above spends ~2 d VALU ops and d LDS reads per element on the distance (16 + 8 at d = 8) beside
// ~22 for exp; here a.b of a 16 x 16 block is DMAX/4 v_mfma_f64_16x16x4 and the element epilogue is r2 = max(na + nb -
// 2 a.b, 0) and the covariance.  Centring: by the first row of the tile's row block (round 5; the mean of its valid rows
// before: 29.0 -> 27.7 us at n = 4096, profiles/r05_gram_ab.log), so a tile depends only on its
// own rows and columns (an appended row block reproduces a refit bit for bit) and |a|, |b| stay O(spread / lengthscale);
// the gap to the difference form is O(eps (|a|^2 + |b|^2)) per entry (bounded in tests/test_oracle.py).  The ARD linear
// term of ScaleKernel(Linear + Matern) is a second MFMA dot (raw x_i v against raw x_j).
// Wave w owns the 16-row strip(s) of the tile's rows and the 16-column blocks jb; the accumulator layout of
// v_mfma_f64_16x16x4 gives each lane rows (lane >> 4) + 4 r of column lane & 15 of a block, so a store instruction writes
// four 128-byte row segments.  Measured and not kept (profiles/r04_gram128_ab.log, r04_gram_rowstore_ab.log): whole-row
// 512-byte stores through a permlane transpose (as kstar_mfma_kernel does) 34.0 vs 28.9 us at n = 4096, and 128 x 128
// tiles 33.5 vs 29.3 us (331 vs 365 us at n = 16384); round 5, two rows of 256 B per store (column blocks paired by
// v_permlane32_swap) 28.0 vs 27.7 us (profiles/r05_gram_ab.log).
template <int DMAX, int KIND>
__global__ void __launch_bounds__(WG) gram_mfma_kernel(gpx_kernel_params p, int n, int t0, const double* __restrict__ X,
                                                       int64_t ldx, double* __restrict__ K, int64_t ldk, int64_t sx,
                                                       int64_t sk, int32_t* __restrict__ info,
                                                       unsigned long long* __restrict__ zero, int64_t zero_words,
                                                       double* __restrict__ mean_out) {
  if (blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
    if (info) info[blockIdx.y] = 0;
    if (mean_out) mean_out[blockIdx.y] = p.const_mean;
  }
  if (zero) {
    const int64_t nwg = (int64_t)gridDim.x * gridDim.y * gridDim.z;
    const int64_t wg = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    for (int64_t e = wg * WG + threadIdx.x; e < zero_words; e += nwg * WG) zero[e] = 0ull;
  }
  X += blockIdx.y * sx;
  K += blockIdx.y * sk;
  constexpr bool lin = (KIND == GPX_KERNEL_SCALE_LINEAR_MATERN52);
  constexpr int KS = DMAX / 4;  // MFMA k-steps
  // a, b: centred scaled inputs (k >= d zero); ra: raw x_i * linear variance, rb: raw x_j; na, nb: squared norms
  __shared__ double sa[NB][DMAX + 1], sb[NB][DMAX + 1], ra[lin ? NB : 1][DMAX + 1], rb[lin ? NB : 1][DMAX + 1];
  __shared__ double na[NB], nb[NB];
  int ti, tj;
  tri_decode(t0 + (int)blockIdx.x, ti, tj);
  const int i0 = ti * NB, j0 = tj * NB;
  const int d = p.d, t = threadIdx.x;
  const int nv = n - i0 < NB ? n - i0 : NB;  // valid rows of the row block (<= 0: all padding)
  // centre: the row block's first row (any common shift is exact in real arithmetic; the first row keeps |a|, |b|
  // within the block's spread as the mean does, without the mean's serial 64-row sum and two extra barriers)
  for (int e = t; e < NB * DMAX; e += WG) {
    const int r = e / DMAX, k = e % DMAX;
    double xi = 0.0, xj = 0.0, x0 = 0.0;
    if (k < d) {
      if (i0 + r < n) xi = X[(int64_t)(i0 + r) * ldx + k];
      if (j0 + r < n) xj = X[(int64_t)(j0 + r) * ldx + k];
      if (nv > 0) x0 = X[(int64_t)i0 * ldx + k];
    }
    const double c0 = (k < d) ? x0 / p.lengthscale[k] : 0.0;
    sa[r][k] = (k < d) ? xi / p.lengthscale[k] - c0 : 0.0;
    sb[r][k] = (k < d) ? xj / p.lengthscale[k] - c0 : 0.0;
    if constexpr (lin) {
      ra[r][k] = (k < d) ? xi * p.linear_variance[k] : 0.0;
      rb[r][k] = xj;
    }
  }
  __syncthreads();
  if (t < 2 * NB) {
    const int r = t & 63;
    const double(*s)[DMAX + 1] = t < NB ? sa : sb;
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) v = fma(s[r][k], s[r][k], v);
    (t < NB ? na : nb)[r] = v;
  }
  __syncthreads();
  const int lane = t & 63, w = t >> 6, m = lane & 15, kq = lane >> 4;
  const double diag_add = p.noise + p.jitter;
  // EDGE: the diagonal tiles and those holding padding rows / columns; the other (interior) tiles need neither the
  // diagonal nor the padding selects (uniform per workgroup: one branch, two copies of the loop; 28.0 -> 26.4 us at
  // n = 4096, profiles/r05_gram_ab.log)
  auto tiles = [&](auto edge_tag) {
    constexpr bool EDGE = decltype(edge_tag)::value;
    // gridDim.z row slices (small fits): the slice's 16-row strips x 4 column blocks, dealt to the waves
    const int strips = 4 / gridDim.z, s0 = blockIdx.z * strips;
    for (int b = w; b < strips * 4; b += 4) {
      const int rs = 16 * (s0 + b / 4), cs = 16 * (b % 4);
      d4 acc = {0.0, 0.0, 0.0, 0.0}, lac = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        acc = mfma16x16x4(sa[rs + m][4 * k + kq], sb[cs + m][4 * k + kq], acc);
        if constexpr (lin) lac = mfma16x16x4(ra[rs + m][4 * k + kq], rb[cs + m][4 * k + kq], lac);
      }
      const int c = cs + m, gj = j0 + c;
      double* Kc = K + (int64_t)(i0 + rs + kq) * ldk + gj;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = rs + kq + 4 * r, gi = i0 + rr;
        double r2 = sqdist_expanded(na[rr], nb[c], acc[r]);
        if (EDGE && gi == gj) r2 = 0.0;
        double v = cov_from_r2(KIND, p.outputscale, r2, lin ? lac[r] : 0.0);
        if (EDGE) {
          if (gi == gj) v += diag_add;
          if (gi >= n || gj >= n) v = (gi == gj) ? 1.0 : 0.0;  // identity padding
        }
        Kc[(int64_t)4 * r * ldk] = v;
      }
    }
  };
  if (ti == tj || i0 + NB > n || j0 + NB > n)
    tiles(std::true_type{});
  else
    tiles(std::false_type{});
}

hipError_t launch_gram(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                       double* K, int64_t ldk, const Batch& bt, int rb0, int32_t* info, void* zero,
                       size_t zero_bytes, double* mean_out) {
  LaunchTimer tm(c, GPX_TIMER_GRAM);
  const int nblk = npad / NB;
  const int t0 = rb0 * (rb0 + 1) / 2;  // tiles of the row blocks above rb0 are skipped (gpx_append_f64)
  const int tiles = (nblk * (nblk + 1) / 2 - t0) * bt.count;
  // fewer tiles than CUs: split each tile's 64 rows over 4 workgroups (n = 128: 11 -> see DESIGN_HISTORY.md); the handle option
  // GPX_OPT_GRAM_SPLIT overrides (1, 2 or 4)
  int split = tiles < 256 ? 4 : 1;
  if (c->gram_split == 1 || c->gram_split == 2 || c->gram_split == 4) split = c->gram_split;
  const dim3 grid(nblk * (nblk + 1) / 2 - t0, bt.count, split);
  auto* zp = reinterpret_cast<unsigned long long*>(zero);
  const int64_t zw = zero ? (int64_t)(zero_bytes / 8) : 0;
#define GPX_GRAM_K(D, KIND)                                                                                      \
  (p.cov_fp32 ? gram_kernel<D, true, KIND><<<grid, WG, 0, c->stream>>>(p, n, t0, X, ldx, K, ldk, bt.x, bt.k, info, zp, zw, mean_out) \
              : gram_mfma_kernel<D, KIND><<<grid, WG, 0, c->stream>>>(p, n, t0, X, ldx, K, ldk, bt.x, bt.k, info, zp, zw, \
                                                                 mean_out))
#define GPX_GRAM(D)                                                                                              \
  (p.kind == GPX_KERNEL_RBF        ? GPX_GRAM_K(D, GPX_KERNEL_RBF)                                               \
   : p.kind == GPX_KERNEL_MATERN52 ? GPX_GRAM_K(D, GPX_KERNEL_MATERN52)                                          \
                                   : GPX_GRAM_K(D, GPX_KERNEL_SCALE_LINEAR_MATERN52))
  if (p.d <= 4)
    GPX_GRAM(4);
  else if (p.d <= 8)
    GPX_GRAM(8);
  else if (p.d <= 16)
    GPX_GRAM(16);
  else
    GPX_GRAM(32);
#undef GPX_GRAM
#undef GPX_GRAM_K
  return hipGetLastError();
}

}  // namespace gpx
