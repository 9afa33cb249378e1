// Negative log marginal likelihood and its hyperparameter gradient for a fitted exact GP
// (replaces ExactMarginalLogLikelihood(...).backward() inside fit_gpytorch_mll [upstream],
// optimization/Bayesian.py:92-93, optimization/Bayesian1.py:114-115, optimization/Bayesian6.py:480-488).
//
//   -log p(Y) = sum_t [ 1/2 (y_t-m)^T alpha_t + sum_i log L_ii + n/2 log(2 pi) ]
//   d/d theta = 1/2 sum_ij (T K^{-1} - sum_t alpha_t alpha_t^T)_ij dK_ij/d theta
// for T = nrhs outputs sharing the covariance (T = 1: the SingleTaskGP objective).
//
// mll_grad_kernel: one workgroup per lower 128x128 tile (I >= J) of K^{-1} = W W^T (W = L^{-T} upper,
// row-major: W[i][k] != 0 only for k >= i, so the k loop of tile (I, J) starts at I*128).  The tile is
// accumulated on the fp64 MFMA units (same MfmaTile core as the sweep product, n^3/3 flops in total) and
// contracted in the epilogue against dK/d theta recomputed from X held in LDS, so K^{-1} never reaches HBM.
// Each workgroup writes GPX_MLL_NOUT partial sums; mll_finalize_kernel adds them in a fixed order together
// with the O(n) terms (quadratic form, log-determinant, mean gradient).
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_trmm_asm.h"
#include <algorithm>
#include <cstdlib>

namespace gpx {

namespace {

constexpr int MT = 128;  // K^{-1} tile
constexpr double SQRT5 = 2.23606797749978969640917366873128;
constexpr double LOG_2PI = 1.83787706640934548356065947281123;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace

template <int DMAX, int KIND>
__global__ void __launch_bounds__(WG) mll_grad_kernel(gpx_kernel_params p, int n, int npad,
                                                      const double* __restrict__ X, int64_t ldx,
                                                      const double* __restrict__ W, int64_t ldw,
                                                      const double* __restrict__ alpha, int nrhs, int kc,
                                                      double* __restrict__ part) {
  using Tile = MfmaTile<MT, MT, 16, false, false>;
  // Epilogue LDS: raw X rows of both tile sides, their alpha rows (<= GPX_MAX_RHS outputs), and one 128 x SW
  // slab of the K^{-1} tile.
  constexpr int SW = 16, KVP = SW + 1, XP = DMAX + 1;
  constexpr int EPI = 2 * MT * XP + 2 * MT * GPX_MAX_RHS + MT * KVP;
  constexpr int SMEM = EPI > Tile::LDS_DOUBLES ? EPI : Tile::LDS_DOUBLES;  // 73.7 KB for d <= 16
  static_assert(Tile::LDS_DOUBLES * 8 == trmm_asm::LDS_BYTES, "hand-placed tile uses MfmaTile's LDS image");
  __shared__ __attribute__((aligned(16))) double smem[SMEM];
  int I, J;
  tri_decode(blockIdx.x, I, J);
  const int i0 = I * MT, j0 = J * MT;
  // split-K: unit (tile, blockIdx.y) covers k in [i0 + y kc, min(.. + kc, npad)).  The epilogue is linear in
  // K^{-1}, so the per-unit contractions add up to the contraction of the full tile; alpha alpha^T enters in
  // chunk 0 only.  Without the split the few deepest tiles (I = 0: k over all of npad) set the critical path.
  const int kbeg = i0 + (int)blockIdx.y * kc;
  // gridDim.z = 8 (tiny grids, npad <= 256): workgroup z contracts only slab z of the tile (the MFMA product is
  // recomputed per slab, ~2 us); one workgroup over all eight slabs took 44 us at n = 128
  double* dst = part + (((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * GPX_MLL_NOUT;
  const bool all_slabs = gridDim.z == 1;
  if (kbeg >= npad) {
    for (int o = threadIdx.x; o < GPX_MLL_NOUT; o += WG) dst[o] = 0.0;
    return;
  }
  const int kend = min(kbeg + kc, npad);
  const double aa = (blockIdx.y == 0) ? 1.0 : 0.0;
  // the hand-placed k loop of gpx_trmm_asm.h (row-major operands, the Cholesky's flush tile): same MFMA sequence per
  // accumulator as MfmaTile::run, so the same bits; ends with a barrier
  trmm_asm::TileT<false, false> t;
  t.zero();
  t.run(W + (int64_t)i0 * ldw + kbeg, ldw, W + (int64_t)j0 * ldw + kbeg, ldw, (kend - kbeg) / 16, smem);

  // ---- epilogue: stage raw X rows and alpha of both tile sides in LDS
  double* xi = smem;             // [MT][XP]
  double* xj = xi + MT * XP;     // [MT][XP]
  double* ai = xj + MT * XP;                // [MT][nrhs]
  double* aj = ai + MT * GPX_MAX_RHS;       // [MT][nrhs]
  double* kv = aj + MT * GPX_MAX_RHS;       // [MT][KVP]
  const int d = p.d;
  for (int e = threadIdx.x; e < MT * DMAX; e += WG) {
    const int r = e / DMAX, k = e % DMAX;
    xi[r * XP + k] = (k < d && i0 + r < n) ? X[(int64_t)(i0 + r) * ldx + k] : 0.0;
    xj[r * XP + k] = (k < d && j0 + r < n) ? X[(int64_t)(j0 + r) * ldx + k] : 0.0;
  }
  for (int e = threadIdx.x; e < MT * nrhs; e += WG) {
    ai[e] = alpha[(int64_t)i0 * nrhs + e];
    aj[e] = alpha[(int64_t)j0 * nrhs + e];
  }
  const double tk = (double)nrhs;

  // For KIND >= 0 the kind is compile-time and, dimensions k >= d being zero in xi / xj / il, the distance loop needs
  // no k < d test (the +0 terms leave every sum bitwise unchanged): no uniform branches per element.
  // KIND < 0: the kind is read at run time (the Scale(Linear + Matern) instantiation: its extra accumulators only fit
  // two waves per SIMD in this form, 256 vs 286 VGPRs at d = 8).
  const int kind = KIND >= 0 ? KIND : p.kind;
  const bool lin = (kind == GPX_KERNEL_SCALE_LINEAR_MATERN52);
  const double s = p.outputscale;
  double il[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) il[k] = (k < d) ? 1.0 / p.lengthscale[k] : 0.0;
  double gl[DMAX], gv[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) gl[k] = gv[k] = 0.0;
  double gs = 0.0, gn = 0.0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;

  // Eight 16-column slabs: the two waves owning the slab's columns park their accumulators in LDS, then all
  // 256 threads contract the slab element by element (a rolled loop keeps register pressure flat).
#pragma unroll
  for (int sl = 0; sl < MT / SW; ++sl) {
    if (!all_slabs && sl != (int)blockIdx.z) continue;  // uniform per workgroup
    if ((w & 1) == (sl >> 2)) {
#pragma unroll
      for (int a = 0; a < Tile::WM; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) kv[Tile::row_of(a, r) * KVP + (lane & 15)] = t.acc[a][sl & 3][r];
    }
    __syncthreads();
#pragma unroll 1
    for (int e = threadIdx.x; e < MT * SW; e += WG) {
      const int ri = e / SW, cj = e % SW;
      const int gi = i0 + ri, gj = j0 + sl * SW + cj;
      if (gi >= n || gj >= n || gj > gi) continue;
      // G = (T K^{-1} - sum_t alpha_t alpha_t^T)_ij, weighted so that summing the lower triangle gives 1/2 sum_ij
      double aat = 0.0;
      for (int q = 0; q < nrhs; ++q) aat += ai[ri * nrhs + q] * aj[(sl * SW + cj) * nrhs + q];
      const double G = ((gi == gj) ? 0.5 : 1.0) * (tk * kv[ri * KVP + cj] - aa * aat);
      const double* x1 = xi + ri * XP;
      const double* x2 = xj + (sl * SW + cj) * XP;
      double q[DMAX];
      double r2 = 0.0;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) {
        q[k] = 0.0;
        if (KIND >= 0 || k < d) {
          const double df = (x1[k] - x2[k]) * il[k];
          q[k] = df * df;
          r2 += q[k];
        }
      }
      double base, kfac;  // base = dk/ds; kfac * q_k / l_k = dk/dl_k
      if (kind == GPX_KERNEL_RBF) {
        base = exp(-0.5 * r2);
        kfac = s * base;
      } else {
        const double rr = sqrt(r2);
        const double ex = exp(-SQRT5 * rr);
        base = (1.0 + SQRT5 * rr + (5.0 / 3.0) * r2) * ex;
        kfac = s * (5.0 / 3.0) * (1.0 + SQRT5 * rr) * ex;
      }
      if (lin) {
        double lv = 0.0;
#pragma unroll
        for (int k = 0; k < DMAX; ++k) {
          if (k < d) {  // kept: without it the linear kind's accumulators cost the second wave per SIMD
            const double xx = x1[k] * x2[k];
            lv += p.linear_variance[k] * xx;
            gv[k] += G * xx;
          }
        }
        base += lv;
      }
      gs += G * base;
      const double gk = G * kfac;
#pragma unroll
      for (int k = 0; k < DMAX; ++k) gl[k] += gk * q[k];
      if (gi == gj) gn += G;
    }
    __syncthreads();
  }

  // ---- workgroup reduction of the 2 + 2d partial sums (fixed order) -> part[blockIdx][GPX_MLL_NOUT]
  double* red = smem;  // [4][GPX_MLL_NOUT]
  auto put = [&](int slot, double v) {
    v = wave_sum(v);
    if (lane == 0) red[w * GPX_MLL_NOUT + slot] = v;
  };
  put(GPX_MLL_D_NOISE, gn);
  put(GPX_MLL_D_OUTPUTSCALE, gs);
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    if (k < d) {
      put(GPX_MLL_D_LENGTHSCALE + k, gl[k] * il[k]);
      if (lin) put(GPX_MLL_D_LINVAR + k, gv[k] * s);
    }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < GPX_MLL_NOUT; o += WG) {
    const bool used = o == GPX_MLL_D_NOISE || o == GPX_MLL_D_OUTPUTSCALE ||
                      (o >= GPX_MLL_D_LENGTHSCALE && o < GPX_MLL_D_LENGTHSCALE + d) ||
                      (lin && o >= GPX_MLL_D_LINVAR && o < GPX_MLL_D_LINVAR + d);
    dst[o] = used ? ((red[o] + red[GPX_MLL_NOUT + o]) + (red[2 * GPX_MLL_NOUT + o] + red[3 * GPX_MLL_NOUT + o]))
                  : 0.0;
  }
}

// Fixed-order column sums of GPX_MLL_NOUT-wide partial rows: block b adds rows [b rpb, (b+1) rpb) into out row b.
// Three 72-thread stripes read consecutive rows (coalesced 576-byte rows), then combine in LDS.
__global__ void __launch_bounds__(WG) mll_rowsum_kernel(const double* __restrict__ in, int64_t rows, int64_t rpb,
                                                        double* __restrict__ out) {
  __shared__ double acc[3][GPX_MLL_NOUT];
  const int col = threadIdx.x % GPX_MLL_NOUT, st = threadIdx.x / GPX_MLL_NOUT;
  if (st < 3) {
    const int64_t beg = (int64_t)blockIdx.x * rpb;
    const int64_t end = min(beg + rpb, rows);
    double v = 0.0;
#pragma unroll 8
    for (int64_t r = beg + st; r < end; r += 3) v += in[r * GPX_MLL_NOUT + col];
    acc[st][col] = v;
  }
  __syncthreads();
  if ((int)threadIdx.x < GPX_MLL_NOUT)
    out[(int64_t)blockIdx.x * GPX_MLL_NOUT + threadIdx.x] = (acc[0][threadIdx.x] + acc[1][threadIdx.x]) +
                                                             acc[2][threadIdx.x];
}

// Single workgroup: the O(n) terms (quadratic form, log-determinant, mean gradient) on top of the summed
// gradient row.
__global__ void __launch_bounds__(WG) mll_finalize_kernel(int n, int nrhs, const double* __restrict__ gsum,
                                                          const double* __restrict__ Y, int64_t ldy,
                                                          const double* __restrict__ L, int64_t ldl,
                                                          const double* __restrict__ alpha, double const_mean,
                                                          double* __restrict__ out) {
  __shared__ double red[WG];
  auto block_sum = [&](double v) -> double {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int h = WG / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
  };
  double q = 0.0, ld = 0.0, sa = 0.0;
  for (int i = threadIdx.x; i < n; i += WG) {
    for (int t = 0; t < nrhs; ++t) {
      const double a = alpha[(int64_t)i * nrhs + t];
      q += (Y[(int64_t)i * ldy + t] - const_mean) * a;
      sa += a;
    }
    ld += log(L[(int64_t)i * ldl + i]);
  }
  q = block_sum(q);
  ld = block_sum(ld);
  sa = block_sum(sa);
  for (int o = threadIdx.x; o < GPX_MLL_NOUT; o += WG) {
    double v = gsum[o];
    if (o == GPX_MLL_QUAD) v = 0.5 * q;
    if (o == GPX_MLL_LOGDET) v = 2.0 * ld;
    if (o == GPX_MLL_NLL) v = 0.5 * q + (double)nrhs * (ld + 0.5 * (double)n * LOG_2PI);
    if (o == GPX_MLL_D_MEAN) v = -sa;
    if (o == 6 || o == 7) v = 0.0;
    out[o] = v;
  }
}

// k-chunk of the split.  n = 4096 (round-1 probe, profiles/r01_mll_kchunk_sweep.log): kc 512 / 1024 / 2048 / npad -> 0.670 / 0.620 / 0.678 /
// 0.742 ms: a shallower chunk balances the deep tiles, but the dK epilogue runs once per unit; n = 8192
// (tools/mll_kc_sweep.sh): 512 / 1024 / 2048 -> 5.33 / 4.74 / 4.65 ms; n = 16384: 2048 / 4096 / 8192 / 16384 ->
// 28.0 / 27.1 / 26.2 / 26.1 ms (thousands of tiles balance themselves).
int mll_kchunk(int64_t npad) {
  int64_t kc = npad >= 16384 ? npad / 2 : npad / 4;
  kc = ((kc + MT - 1) / MT) * MT;
  return (int)(kc < 512 ? 512 : kc);
}

// epilogue slabs split over workgroups (gridDim.z) for the tiny grids of npad <= 256
static int mll_slab_split(int64_t npad) { return npad <= 256 ? MT / 16 : 1; }

size_t mll_workspace_bytes(int64_t npad) {
  const int64_t T = npad / MT;
  const int64_t kc = mll_kchunk(npad);
  const int64_t ny = (npad + kc - 1) / kc;
  return ((size_t)(T * (T + 1) / 2) * ny * mll_slab_split(npad) + 256 + 1) * GPX_MLL_NOUT * sizeof(double);
}

hipError_t launch_mll(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                      const double* Y, int64_t ldy, int nrhs, const double* L, int64_t ldl, const double* W,
                      int64_t ldw, const double* alpha, double* out, double* part) {
  LaunchTimer tm(c, GPX_TIMER_MLL);
  const int T = npad / MT;
  const int tiles = T * (T + 1) / 2;
  const int kc = mll_kchunk(npad);
  const dim3 grid(tiles, (npad + kc - 1) / kc, mll_slab_split(npad));
#define GPX_MLL_K(D, K) mll_grad_kernel<D, K><<<grid, WG, 0, c->stream>>>(p, n, npad, X, ldx, W, ldw, alpha, nrhs, kc, part)
#define GPX_MLL(D)                                                         \
  (p.kind == GPX_KERNEL_RBF        ? GPX_MLL_K(D, GPX_KERNEL_RBF)          \
   : p.kind == GPX_KERNEL_MATERN52 ? GPX_MLL_K(D, GPX_KERNEL_MATERN52)     \
                                   : GPX_MLL_K(D, -1))
  if (p.d <= 4)
    GPX_MLL(4);
  else if (p.d <= 8)
    GPX_MLL(8);
  else if (p.d <= 16)
    GPX_MLL(16);
  else
    GPX_MLL(32);
#undef GPX_MLL
#undef GPX_MLL_K
  const int64_t rows = (int64_t)tiles * grid.y * grid.z;
  const int64_t rpb = std::max<int64_t>(64, (rows + 255) / 256);
  const int nb = (int)((rows + rpb - 1) / rpb);
  double* stage = part + rows * GPX_MLL_NOUT;  // nb <= 256 rows
  double* gsum = stage + 256 * GPX_MLL_NOUT;
  mll_rowsum_kernel<<<nb, WG, 0, c->stream>>>(part, rows, rpb, stage);
  mll_rowsum_kernel<<<1, WG, 0, c->stream>>>(stage, nb, nb, gsum);
  mll_finalize_kernel<<<1, WG, 0, c->stream>>>(n, nrhs, gsum, Y, ldy, L, ldl, alpha, p.const_mean, out);
  return hipGetLastError();
}

}  // namespace gpx
