// Blocked right-looking Cholesky (lower) of the padded Gram matrix, NB = 64.
// SURVEY §8a row a4 — replaces psd_safe_cholesky in GPyTorch's exact path [upstream]; the reference's
// jitter-retry policy (optimization/Bayesian6.py:481-488) needs the failing pivot, reported in *info.
//
// Per block column k, two launches:
//  1. potrf_panel: one workgroup per block row i >= k.  Every workgroup factors the diagonal block A_kk in
//     registers (4x4 elements per thread, one column published through LDS per step, 2 barriers per
//     step) while building its inverse D_k = L_kk^{-1} in the same sweep (forward substitution on the
//     identity, row j finalised at step j).  Workgroup i == k stores D_k and a copy of L_kk in the scratch
//     half of Dinv (A_kk itself must stay intact while other panel workgroups may still read it);
//     workgroups i > k compute the panel L_ik = A_ik D_k^T (64x64x64, fp64 VALU FMA from LDS).
//     Re-factoring A_kk in every panel workgroup costs no extra latency and saves a launch per step.
//  2. syrk_update: trailing A_ij -= L_ik L_jk^T for all lower tiles i >= j > k on fp64 MFMA (MfmaTile);
//     one extra workgroup copies L_kk from the scratch into A_kk.
#include "gpx_internal.h"
#include "gpx_device.h"

namespace gpx {

__global__ void __launch_bounds__(WG) potrf_panel_kernel(double* __restrict__ A, int64_t lda, int k,
                                                         double* __restrict__ Dinv, int32_t* __restrict__ info) {
  if (*(volatile int32_t*)info != 0) return;  // an earlier step failed: leave the rest untouched
  __shared__ double colbuf[NB];
  __shared__ double rowbuf[NB];
  __shared__ double pivot;
  __shared__ double sP[NB][NB + 1];   // panel block A_ik
  __shared__ double sD[NB][NB + 1];   // D_k

  const int t = threadIdx.x;
  const int tr = t >> 4, tc = t & 15;  // owns rows 4tr..4tr+3, cols 4tc..4tc+3
  const int bi = k + blockIdx.x;       // block row of this workgroup
  const double* Akk = A + (int64_t)k * NB * lda + (int64_t)k * NB;

  double a[4][4], x[4][4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const double4 v = *reinterpret_cast<const double4*>(Akk + (int64_t)(4 * tr + rr) * lda + 4 * tc);
    a[rr][0] = v.x; a[rr][1] = v.y; a[rr][2] = v.z; a[rr][3] = v.w;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) x[rr][cc] = (4 * tr + rr == 4 * tc + cc) ? 1.0 : 0.0;
  }
  // Panel block load overlaps the factorisation.
  if (blockIdx.x > 0) {
    const double* Aik = A + (int64_t)bi * NB * lda + (int64_t)k * NB;
    for (int e = t; e < NB * NB / 2; e += WG) {
      int r = e / (NB / 2), c2 = (e % (NB / 2)) * 2;
      const double2 v = *reinterpret_cast<const double2*>(Aik + (int64_t)r * lda + c2);
      sP[r][c2] = v.x;
      sP[r][c2 + 1] = v.y;
    }
  }
  bool failed_reported = false;

  for (int jb = 0; jb < NB / 4; ++jb) {
#pragma unroll
    for (int jr = 0; jr < 4; ++jr) {
      const int j = 4 * jb + jr;
      if (tr == jb && tc == jb) pivot = a[jr][jr];
      __syncthreads();
      const double pv = pivot;
      const double dj = sqrt(pv);
      const double inv_dj = 1.0 / dj;
      if (!(pv > 0.0) && t == 0 && blockIdx.x == 0 && !failed_reported) {
        atomicCAS(info, 0, k * NB + j + 1);
        failed_reported = true;
      }
      if (tc == jb) {  // owners of column j publish L(:, j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int row = 4 * tr + rr;
          double l;
          if (row > j) l = a[rr][jr] * inv_dj;
          else if (row == j) l = dj;
          else l = 0.0;
          a[rr][jr] = l;
          colbuf[row] = l;
        }
      }
      if (tr == jb) {  // owners of row j of the inverse finalise and publish it
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          x[jr][cc] *= inv_dj;
          rowbuf[4 * tc + cc] = x[jr][cc];
        }
      }
      __syncthreads();
      double lr[4], lc[4], xr[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        lr[q] = colbuf[4 * tr + q];
        lc[q] = colbuf[4 * tc + q];
        xr[q] = rowbuf[4 * tc + q];
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 4 * tr + rr;
        if (row > j) {
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            const int col = 4 * tc + cc;
            if (col > j && col <= row) a[rr][cc] -= lr[rr] * lc[cc];
            x[rr][cc] -= lr[rr] * xr[cc];
          }
        }
      }
    }
  }

  if (blockIdx.x == 0) {
    const int nblk = gridDim.x + k;
    double* D = Dinv + (int64_t)k * NB * NB;
    double* Lkk = Dinv + (int64_t)(nblk + k) * NB * NB;  // scratch copy, moved into A by syrk_update
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 4 * tr + rr;
      double4 lv, dv;
      lv.x = (4 * tc + 0 <= row) ? a[rr][0] : 0.0;
      lv.y = (4 * tc + 1 <= row) ? a[rr][1] : 0.0;
      lv.z = (4 * tc + 2 <= row) ? a[rr][2] : 0.0;
      lv.w = (4 * tc + 3 <= row) ? a[rr][3] : 0.0;
      dv.x = x[rr][0]; dv.y = x[rr][1]; dv.z = x[rr][2]; dv.w = x[rr][3];
      *reinterpret_cast<double4*>(Lkk + row * NB + 4 * tc) = lv;
      *reinterpret_cast<double4*>(D + row * NB + 4 * tc) = dv;
    }
    return;
  }
  // Panel: L_ik[r][c] = sum_q A_ik[r][q] * D[c][q]  (D lower triangular: q <= c)
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) sD[4 * tr + rr][4 * tc + cc] = x[rr][cc];
  __syncthreads();
  double acc[4][4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) acc[rr][cc] = 0.0;
  const int qmax = 4 * tc + 4;
  for (int q = 0; q < qmax; ++q) {
    double av[4], dv[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) av[rr] = sP[4 * tr + rr][q];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) dv[cc] = sD[4 * tc + cc][q];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) acc[rr][cc] += av[rr] * dv[cc];
  }
  double* Lik = A + (int64_t)bi * NB * lda + (int64_t)k * NB;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    double4 v;
    v.x = acc[rr][0]; v.y = acc[rr][1]; v.z = acc[rr][2]; v.w = acc[rr][3];
    *reinterpret_cast<double4*>(Lik + (int64_t)(4 * tr + rr) * lda + 4 * tc) = v;
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
  Tile tile;
  tile.run(Pi, lda, Pj, lda, 0, NB, smem);
  double* C = A + (int64_t)bi * NB * lda + (int64_t)bj * NB;
#pragma unroll
  for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
    for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = Tile::row_of(i, r), col = Tile::col_of(j);
        double* p = C + (int64_t)row * lda + col;
        *p = *p - tile.acc[i][j][r];
      }
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
