// Blocked right-looking Cholesky (lower) of the padded Gram matrix, NB = 64.
// SURVEY §8a row a4 — replaces psd_safe_cholesky in GPyTorch's exact path [upstream]; the reference's
// jitter-retry policy (optimization/Bayesian6.py:481-488) needs the failing pivot, reported in *info.
//
// Per block column k, two launches:
//  1. potrf_panel: one workgroup per block row i >= k.  Every workgroup factors and inverts the diagonal
//     block A_kk (chol_inv64, gpx_chol64.h: pivots inside one wave, MFMA for the rest); workgroup i == k
//     stores D_k = L_kk^{-1} and a copy of L_kk in the scratch half of Dinv (A_kk itself must stay intact
//     while other panel workgroups may still read it); workgroups i > k compute the panel L_ik = A_ik D_k^T
//     (64x64x64 on fp64 MFMA from LDS).
//     Re-factoring A_kk in every panel workgroup costs no extra latency and saves a launch per step.
//  2. syrk_update: trailing A_ij -= L_ik L_jk^T for all lower tiles i >= j > k on fp64 MFMA (MfmaTile);
//     one extra workgroup copies L_kk from the scratch into A_kk.
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_chol64.h"

namespace gpx {

__global__ void __launch_bounds__(WG) potrf_panel_kernel(double* __restrict__ A, int64_t lda, int k,
                                                         double* __restrict__ Dinv, int32_t* __restrict__ info) {
  if (*(volatile int32_t*)info != 0) return;  // an earlier step failed: leave the rest untouched
  __shared__ __attribute__((aligned(16))) double sA[NB * LD64];
  __shared__ __attribute__((aligned(16))) double sX[NB * LD64];
  __shared__ __attribute__((aligned(16))) double sT[NB * LD64];
  const int t = threadIdx.x;
  const int bi = k + blockIdx.x;  // block row of this workgroup
  const double* Akk = A + (int64_t)k * NB * lda + (int64_t)k * NB;
  const double* Aik = A + (int64_t)bi * NB * lda + (int64_t)k * NB;
  // panel block prefetched into registers; it is consumed after the diagonal factorisation
  double2 pre[8];
  if (blockIdx.x > 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
      pre[q] = *reinterpret_cast<const double2*>(Aik + (int64_t)r * lda + c);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    const double2 v = *reinterpret_cast<const double2*>(Akk + (int64_t)r * lda + c);
    sA[r * LD64 + c] = v.x;
    sA[r * LD64 + c + 1] = v.y;
  }
  __syncthreads();
  const int fail = chol_inv64(sA, sX, sT);
  if (blockIdx.x == 0) {
    if (t == 0 && fail >= 0) atomicCAS(info, 0, k * NB + fail + 1);
    const int nblk = gridDim.x + k;
    double* D = Dinv + (int64_t)k * NB * NB;
    double* Lkk = Dinv + (int64_t)(nblk + k) * NB * NB;  // scratch copy, moved into A by syrk_update
    for (int e = t; e < NB * NB; e += WG) {
      const int r = e >> 6, c = e & 63;
      Lkk[e] = (c <= r) ? sA[r * LD64 + c] : 0.0;
      D[e] = sX[r * LD64 + c];
    }
    return;
  }
  // Panel: L_ik = A_ik D_k^T on fp64 MFMA (each wave: one 16-row strip x 4 column blocks, K = 64)
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    sT[r * LD64 + c] = pre[q].x;
    sT[r * LD64 + c + 1] = pre[q].y;
  }
  __syncthreads();
  const int w = t >> 6, lane = t & 63;
  double* Lik = A + (int64_t)bi * NB * lda + (int64_t)k * NB;
#pragma unroll
  for (int bj = 0; bj < 4; ++bj) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = mfma_lds16<true>(acc, sT, 16 * w, 0, sX, 0, 16 * bj, (bj + 1) * 16, 1.0);  // D lower: k <= col
#pragma unroll
    for (int q = 0; q < 4; ++q)
      Lik[(int64_t)(16 * w + (lane >> 4) + 4 * q) * lda + 16 * bj + (lane & 15)] = acc[q];
  }
}

// Trailing update for block column k: tiles (i, j), k < j <= i < nblk, A_ij -= L_ik L_jk^T.
// The last workgroup of the grid copies L_kk from the Dinv scratch into A_kk.
__global__ void __launch_bounds__(WG) syrk_update_kernel(double* __restrict__ A, int64_t lda, int k, int nblk,
                                                         const double* __restrict__ Dinv,
                                                         const int32_t* __restrict__ info) {
  if (*(volatile const int32_t*)info != 0) return;
  if (blockIdx.x == gridDim.x - 1) {
    const double* src = Dinv + (int64_t)(nblk + k) * NB * NB;
    double* dst = A + (int64_t)k * NB * lda + (int64_t)k * NB;
    for (int e = threadIdx.x; e < NB * NB / 2; e += WG) {
      int r = e / (NB / 2), c2 = (e % (NB / 2)) * 2;
      *reinterpret_cast<double2*>(dst + (int64_t)r * lda + c2) = *reinterpret_cast<const double2*>(src + r * NB + c2);
    }
    return;
  }
  using Tile = MfmaTile<NB, NB, 16, false, false>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  int bi, bj;
  tri_decode(blockIdx.x, bi, bj);
  bi += k + 1;
  bj += k + 1;
  const double* Pi = A + (int64_t)bi * NB * lda + (int64_t)k * NB;  // L_ik (row-major, k contiguous)
  const double* Pj = A + (int64_t)bj * NB * lda + (int64_t)k * NB;  // L_jk
  double* C = A + (int64_t)bi * NB * lda + (int64_t)bj * NB;
  // The C tile is read into registers up front, all loads in flight at once and overlapping the MFMA loop;
  // a load-modify-store per element after the loop serialised 16 global round trips (41 us at step 0).
  double cv[Tile::WM][Tile::WN][4];
#pragma unroll
  for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
    for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[i][j][r] = C[(int64_t)Tile::row_of(i, r) * lda + Tile::col_of(j)];
  Tile tile;
  tile.run(Pi, lda, Pj, lda, 0, NB, smem);
#pragma unroll
  for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
    for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(int64_t)Tile::row_of(i, r) * lda + Tile::col_of(j)] = cv[i][j][r] - tile.acc[i][j][r];
}

hipError_t launch_potrf(Context* c, int npad, double* A, int64_t lda, double* Dinv, int32_t* info) {
  LaunchTimer tm(c, GPX_TIMER_POTRF);
  const int nblk = npad / NB;
  for (int k = 0; k < nblk; ++k) {
    potrf_panel_kernel<<<nblk - k, WG, 0, c->stream>>>(A, lda, k, Dinv, info);
    const int m = nblk - k - 1;
    syrk_update_kernel<<<m * (m + 1) / 2 + 1, WG, 0, c->stream>>>(A, lda, k, nblk, Dinv, info);
  }
  return hipGetLastError();
}

}  // namespace gpx
