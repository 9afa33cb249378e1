// Driven-variant (Bayesian7) pieces of the hot path: SVGP predictive preparation and the pool-scan selection.
// SURVEY §8a row a9 / §8f row 2 — replaces gpytorch's whitened VariationalStrategy predictive [upstream] reached from
// optimization/Bayesian7.py:558,668, the torch.topk of :681 and farthest_point_sampling of :82-106,684.
//
//  * svgp_pad:   vmean -> zero-padded m (Mpad), chol_variational_covar -> S = tril(.) zero-padded (Mpad x Mpad)
//                (CholeskyVariationalDistribution masks the strict upper part [upstream]).
//  * svgp_w2:    W2 = W S with W = L_ZZ^{-T} (upper) and S (lower): 128x128 fp64-MFMA tiles over j >= max(row, col)
//                tile starts (the only non-zero products), so that var = k** - |W^T k*|^2 + |W2^T k*|^2 needs one more
//                column-sum-of-squares product per candidate (gpx_sweep.hip, trmm_sumsq with kfull = 1).
//  * topk:       stable descending radix sort (hipcub) of the scores (NaN -> -inf), first k (value, index) pairs:
//                ties keep the lower index first.
//  * fps:        greedy farthest point sampling in one workgroup: squared Euclidean distances in fp64 (same argmax as
//                the reference's torch.cdist distances up to rounding), argmax with the lowest index among ties
//                (torch.argmax), start index given by the caller (the reference draws it with torch.randint).
#include <hipcub/hipcub.hpp>
#include <climits>
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_trmm_asm.h"

namespace gpx {

__global__ void __launch_bounds__(WG) svgp_pad_kernel(int M, int Mpad, const double* __restrict__ vmean,
                                                      int64_t stride_m, const double* __restrict__ vchol, int64_t ldc,
                                                      int64_t stride_c, double* __restrict__ mpad,
                                                      double* __restrict__ spad, int64_t sdst) {
  const int t = blockIdx.y;
  const double* V = vchol + t * stride_c;
  double* S = spad + t * sdst;
  const int64_t e0 = (int64_t)blockIdx.x * WG + threadIdx.x;
  const int64_t tot = (int64_t)Mpad * Mpad;
  for (int64_t e = e0; e < tot; e += (int64_t)gridDim.x * WG) {
    const int i = (int)(e / Mpad), j = (int)(e % Mpad);
    S[e] = (i < M && j <= i) ? V[(int64_t)i * ldc + j] : 0.0;
  }
  if (e0 < Mpad) mpad[t * sdst + e0] = (e0 < M) ? vmean[t * stride_m + e0] : 0.0;
}

hipError_t launch_svgp_pad(Context* c, int ntask, int M, int Mpad, const double* vmean, int64_t stride_m,
                           const double* vchol, int64_t ldc, int64_t stride_c, double* mpad, double* spad,
                           int64_t sdst) {
  const int blocks = (int)std::min<int64_t>(((int64_t)Mpad * Mpad + WG - 1) / WG, 2048);
  svgp_pad_kernel<<<dim3(std::max(blocks, (Mpad + WG - 1) / WG), ntask), WG, 0, c->stream>>>(
      M, Mpad, vmean, stride_m, vchol, ldc, stride_c, mpad, spad, sdst);
  return hipGetLastError();
}

// W2[k][i] = sum_{j >= max(k0, i0)} W[k][j] S[j][i] for the 128x128 tile (k0, i0); W upper, S lower.
using W2Tile = MfmaTile<128, 128, 16, false, true>;  // (its accumulator layout and LDS size)
static_assert(W2Tile::LDS_DOUBLES * 8 == trmm_asm::LDS_BYTES, "hand-placed tile uses MfmaTile's LDS image");

__global__ void __launch_bounds__(WG) svgp_w2_kernel(int Mpad, const double* __restrict__ W,
                                                     const double* __restrict__ S, int64_t s_stride,
                                                     double* __restrict__ W2) {
  __shared__ __attribute__((aligned(16))) double smem[W2Tile::LDS_DOUBLES];
  const int nt = Mpad / 128;
  const int t = blockIdx.y;
  const int64_t off = (int64_t)t * Mpad * Mpad;
  S += t * s_stride;
  const int R = blockIdx.x / nt, Cc = blockIdx.x % nt;
  const int k0 = R * 128, i0 = Cc * 128;
  const int kbeg = k0 > i0 ? k0 : i0;
  // A(m, j) = W[k0 + m][j] (row-major), B(j, n) = S[j][i0 + n] (k-major), on the hand-placed k loop (gpx_trmm_asm.h:
  // the same MFMA sequence per accumulator as MfmaTile::run, so the same bits)
  trmm_asm::TileT<false, true> tile;
  tile.zero();
  tile.run(W + off + (int64_t)k0 * Mpad + kbeg, Mpad, S + i0 + (int64_t)kbeg * Mpad, Mpad, (Mpad - kbeg) / 16, smem);
  double* O = W2 + off + (int64_t)k0 * Mpad + i0;
#pragma unroll
  for (int i = 0; i < W2Tile::WM; ++i)
#pragma unroll
    for (int j = 0; j < W2Tile::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) O[(int64_t)W2Tile::row_of(i, r) * Mpad + W2Tile::col_of(j)] = tile.acc[i][j][r];
}

hipError_t launch_svgp_w2(Context* c, int ntask, int Mpad, const double* W, const double* S, int64_t s_stride,
                          double* W2) {
  const int nt = Mpad / 128;
  svgp_w2_kernel<<<dim3(nt * nt, ntask), WG, 0, c->stream>>>(Mpad, W, S, s_stride, W2);
  return hipGetLastError();
}

// ---- top-k ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(WG) topk_prep_kernel(const double* __restrict__ s, int64_t m, double* __restrict__ key,
                                                       int64_t* __restrict__ idx) {
  const int64_t e = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (e >= m) return;
  const double v = s[e];
  key[e] = (v != v) ? -INFINITY : v + 0.0;  // NaN never ranks; -0 -> +0 (radix order would split them)
  idx[e] = e;
}

__global__ void __launch_bounds__(WG) topk_copy_kernel(const double* __restrict__ key, const int64_t* __restrict__ idx,
                                                       int64_t k, int64_t* __restrict__ idx_out,
                                                       double* __restrict__ val_out) {
  const int64_t e = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (e >= k) return;
  idx_out[e] = idx[e];
  if (val_out) val_out[e] = key[e];
}

static size_t cub_sort_bytes(int64_t m) {
  size_t b = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, b, (const double*)nullptr, (double*)nullptr,
                                                     (const int64_t*)nullptr, (int64_t*)nullptr, (int)m, 0, 64,
                                                     (hipStream_t)0);
  return b;
}

size_t topk_workspace_bytes(int64_t m) {
  // keys in/out + indices in/out + sort temp storage, each 256-byte aligned
  const size_t a = ((size_t)m * 8 + 255) & ~(size_t)255;
  return 4 * a + ((cub_sort_bytes(m) + 255) & ~(size_t)255) + 256;
}

hipError_t launch_topk(Context* c, const double* scores, int64_t m, int64_t k, int64_t* idx_out, double* val_out,
                       void* ws, size_t ws_bytes) {
  const size_t a = ((size_t)m * 8 + 255) & ~(size_t)255;
  char* base = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~(uintptr_t)255);
  double* kin = reinterpret_cast<double*>(base);
  double* kout = reinterpret_cast<double*>(base + a);
  int64_t* iin = reinterpret_cast<int64_t*>(base + 2 * a);
  int64_t* iout = reinterpret_cast<int64_t*>(base + 3 * a);
  void* tmp = base + 4 * a;
  size_t tmp_bytes = cub_sort_bytes(m);
  if ((size_t)(base - reinterpret_cast<char*>(ws)) + 4 * a + tmp_bytes > ws_bytes) return hipErrorInvalidValue;
  topk_prep_kernel<<<(int)((m + WG - 1) / WG), WG, 0, c->stream>>>(scores, m, kin, iin);
  hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes, kin, kout, iin, iout, (int)m, 0, 64,
                                                             c->stream);
  if (e != hipSuccess) return e;
  topk_copy_kernel<<<(int)((k + WG - 1) / WG), WG, 0, c->stream>>>(kout, iout, k, idx_out, val_out);
  return hipGetLastError();
}

// ---- farthest point sampling ------------------------------------------------------------------------------
constexpr int FPS_WG = 1024;

template <int PPT>
__global__ void __launch_bounds__(FPS_WG) fps_kernel(const double* __restrict__ X, int64_t m, int d, int64_t ldx,
                                                     int64_t k, int64_t start, int64_t* __restrict__ idx_out) {
  __shared__ double sx[GPX_MAX_DIM];
  __shared__ double wv[FPS_WG / 64];
  __shared__ int64_t wi[FPS_WG / 64];
  __shared__ int64_t s_sel;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  double dist[PPT];
#pragma unroll
  for (int q = 0; q < PPT; ++q) dist[q] = -INFINITY;  // points beyond m never win
  int64_t sel = start;
  for (int64_t it = 0; it < k; ++it) {
    if (t == 0) idx_out[it] = sel;
    if (t < d) sx[t] = X[sel * ldx + t];
    __syncthreads();
    double bv = -INFINITY;
    int64_t bi = INT64_MAX;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int64_t p = (int64_t)q * FPS_WG + t;
      if (p < m) {
        double d2 = 0.0;
        for (int j = 0; j < d; ++j) {
          const double df = X[p * ldx + j] - sx[j];
          d2 += df * df;
        }
        dist[q] = (it == 0) ? d2 : fmin(dist[q], d2);
        if (dist[q] > bv) {  // q ascending -> p ascending within a thread: strict '>' keeps the lowest index
          bv = dist[q];
          bi = p;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(bv, o);
      const int64_t i2 = __shfl_xor(bi, o);
      if (v2 > bv || (v2 == bv && i2 < bi)) {
        bv = v2;
        bi = i2;
      }
    }
    if (lane == 0) {
      wv[w] = bv;
      wi[w] = bi;
    }
    __syncthreads();
    if (t == 0) {
      for (int q = 1; q < FPS_WG / 64; ++q)
        if (wv[q] > bv || (wv[q] == bv && wi[q] < bi)) {
          bv = wv[q];
          bi = wi[q];
        }
      s_sel = bi;
    }
    __syncthreads();
    sel = s_sel;
  }
}

// Register-resident form (d <= DM, m <= PPT * WGS; Bayesian7's case: 8000 points, d = 5): each thread keeps its
// points' coordinates in registers for the whole run, and each wave's winner publishes its coordinates with its (value,
// index), so an iteration reads no global memory (fps_kernel re-reads X and the selected point every iteration:
// ~8 us per iteration, 4.0 ms for 500 of 8000).  Same distances, same order of accumulation, same argmax and tie rule
// (largest distance, then lowest index), so the same indices.
template <int WGS, int PPT, int DM>
__global__ void __launch_bounds__(WGS) fps_reg_kernel(const double* __restrict__ X, int64_t m, int d, int64_t ldx,
                                                      int64_t k, int64_t start, int64_t* __restrict__ idx_out) {
  constexpr int NW = WGS / 64;
  __shared__ double sx[DM];
  __shared__ double wv[NW], wx[NW][DM];
  __shared__ int wi[NW];
  __shared__ int s_sel;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  double px[PPT][DM], dist[PPT];
#pragma unroll
  for (int q = 0; q < PPT; ++q) {
    const int64_t p = (int64_t)q * WGS + t;
#pragma unroll
    for (int j = 0; j < DM; ++j) px[q][j] = (p < m && j < d) ? X[p * ldx + j] : 0.0;
    dist[q] = -INFINITY;  // points beyond m never win
  }
  if (t < DM) sx[t] = t < d ? X[start * ldx + t] : 0.0;
  __syncthreads();
  int sel = (int)start;
  for (int64_t it = 0; it < k; ++it) {
    if (t == 0) idx_out[it] = sel;
    double s[DM];
#pragma unroll
    for (int j = 0; j < DM; ++j) s[j] = sx[j];
    double bv = -INFINITY;
    int bi = INT_MAX;
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int p = q * WGS + t;
      if (p < m) {
        double d2 = 0.0;
#pragma unroll
        for (int j = 0; j < DM; ++j) {
          if (j < d) {
            const double df = px[q][j] - s[j];
            d2 += df * df;
          }
        }
        dist[q] = (it == 0) ? d2 : fmin(dist[q], d2);
        if (dist[q] > bv) {  // q ascending -> p ascending within a thread: strict '>' keeps the lowest index
          bv = dist[q];
          bi = p;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double v2 = __shfl_xor(bv, o);
      const int i2 = __shfl_xor(bi, o);
      if (v2 > bv || (v2 == bv && i2 < bi)) {
        bv = v2;
        bi = i2;
      }
    }
    if (lane == 0) {
      wv[w] = bv;
      wi[w] = bi;
    }
    if (bi != INT_MAX && t == bi % WGS) {  // the wave's winner publishes its coordinates
      const int qw = bi / WGS;
#pragma unroll
      for (int q = 0; q < PPT; ++q)
        if (q == qw)
#pragma unroll
          for (int j = 0; j < DM; ++j) wx[w][j] = px[q][j];
    }
    __syncthreads();
    if (w == 0) {  // the NW wave winners: largest value, then lowest index
      double v = lane < NW ? wv[lane] : -INFINITY;
      int i = lane < NW ? wi[lane] : INT_MAX, src = lane < NW ? lane : 0;
#pragma unroll
      for (int o = NW / 2; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o);
        const int i2 = __shfl_xor(i, o), s2 = __shfl_xor(src, o);
        if (v2 > v || (v2 == v && i2 < i)) {
          v = v2;
          i = i2;
          src = s2;
        }
      }
      if (lane < DM) sx[lane] = wx[src][lane];
      if (lane == 0) s_sel = i;
    }
    __syncthreads();
    sel = s_sel;
  }
}

hipError_t launch_fps(Context* c, const double* X, int64_t m, int d, int64_t ldx, int64_t k, int64_t start,
                      int64_t* idx_out) {
  if (m <= 8 * FPS_WG && d <= 4)
    fps_reg_kernel<FPS_WG, 8, 4><<<1, FPS_WG, 0, c->stream>>>(X, m, d, ldx, k, start, idx_out);
  else if (m <= 8 * FPS_WG && d <= 5)  // 512 threads: 16 points of up to 5 coordinates per thread fit the registers
    fps_reg_kernel<512, 16, 5><<<1, 512, 0, c->stream>>>(X, m, d, ldx, k, start, idx_out);
  else if (m <= 8 * FPS_WG)
    fps_kernel<8><<<1, FPS_WG, 0, c->stream>>>(X, m, d, ldx, k, start, idx_out);
  else if (m <= 32 * FPS_WG)
    fps_kernel<32><<<1, FPS_WG, 0, c->stream>>>(X, m, d, ldx, k, start, idx_out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace gpx
