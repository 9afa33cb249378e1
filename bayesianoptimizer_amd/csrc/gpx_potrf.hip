// Blocked right-looking Cholesky (lower) of the padded Gram matrix, NB = 64.
// SURVEY §8a row a4 — replaces psd_safe_cholesky in GPyTorch's exact path [upstream]; the reference's
// jitter-retry policy (optimization/Bayesian6.py:481-488) needs the failing pivot, reported in *info.
//
// Per block column k, two launches:
//  1. potrf_panel: one workgroup per block row i >= k factors the tall panel [A_kk; A_ik] (128 x 64, or just
//     A_kk for i == k) in LDS: four 16-column steps, each
//        F  wave 0 factors + inverts the 16x16 pivot block in registers (chol16, gpx_chol64.h),
//        T  L_is = A_is D_ss^T for the 16-row blocks below it (fp64 MFMA),
//        U  A_ij -= L_is L_js^T for the trailing 16x16 blocks of the panel (fp64 MFMA),
//     with a one-block lookahead: wave 0 does the T and U of the next pivot block itself and goes straight on to
//     the next F (one barrier per step); waves 1-3 do the other T items, wait on an LDS counter until every T item
//     of the step is published, and do the other U items while that F runs.  Re-factoring A_kk in every workgroup
//     costs no latency and needs no extra launch; workgroup i == k stores L_kk in the scratch half of Dinv
//     (A_kk must stay intact while other workgroups may still read it), workgroups i > k store L_ik.
//  2. syrk_update: trailing A_ij -= L_ik L_jk^T for all lower tiles i >= j > k on fp64 MFMA (MfmaTile);
//     one extra workgroup copies L_kk from the scratch into A_kk.
// Finally potrf_dinv inverts every 64x64 diagonal block of L in one launch (Dinv, used by gpx_trtri_f64).
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_chol64.h"

// Optional timestamp hook for tools/potrf_bench.hip (compiled out in the library).
#ifndef GPX_PANEL_STAMP
#define GPX_PANEL_STAMP(i)
#endif

namespace gpx {

__global__ void __launch_bounds__(WG) potrf_panel_kernel(double* __restrict__ A, int64_t lda, int k,
                                                         double* __restrict__ Dinv, int32_t* __restrict__ info) {
  if (*(volatile int32_t*)info != 0) return;  // an earlier step failed: leave the rest untouched
  __shared__ __attribute__((aligned(16))) double sA[NB * LD64];      // A_kk -> L_kk
  __shared__ __attribute__((aligned(16))) double sP[NB * LD64];      // A_ik -> L_ik (i > k)
  __shared__ __attribute__((aligned(16))) double sD[2][16 * LD64];   // D_ss, double-buffered by step parity
  __shared__ int s_tdone;                                            // T items published (4 per step)
  const int t = threadIdx.x, w = t >> 6;
  const bool panel = blockIdx.x > 0;
  const int nrow = panel ? 8 : 4;  // 16-row blocks of the tall panel
  const int bi = k + blockIdx.x;
  const double* Akk = A + (int64_t)k * NB * lda + (int64_t)k * NB;
  double* Aik = A + (int64_t)bi * NB * lda + (int64_t)k * NB;
  if (t == 0) s_tdone = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    const double2 v = *reinterpret_cast<const double2*>(Akk + (int64_t)r * lda + c);
    sA[r * LD64 + c] = v.x;
    sA[r * LD64 + c + 1] = v.y;
  }
  if (panel) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
      const double2 v = *reinterpret_cast<const double2*>(Aik + (int64_t)r * lda + c);
      sP[r * LD64 + c] = v.x;
      sP[r * LD64 + c + 1] = v.y;
    }
  }
  __syncthreads();
  GPX_PANEL_STAMP(0);
  auto rows = [&](int i) -> double* { return i < 4 ? sA + 16 * i * LD64 : sP + 16 * (i - 4) * LD64; };
  // T: L_is = A_is D_ss^T (16x16x16 on MFMA, in place)
  auto tsolve = [&](int i, const double* D, int o) {
    double* R = rows(i);
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = mfma_lds16<true>(acc, R, 0, o, D, 0, 0, 16, 1.0);
    store_block16(R, 0, o, acc);
  };
  // U: A_ij -= L_is L_js^T
  auto update = [&](int i, int j, int o) {
    double* Ri = rows(i);
    d4 acc = load_block16(Ri, 0, 16 * j);
    acc = mfma_lds16<true>(acc, Ri, 0, o, rows(j), o, 0, 16, -1.0);
    store_block16(Ri, 0, 16 * j, acc);
  };
  // one increment per wave (lane 0); the release orders the wave's LDS stores before it
  auto publish = [&]() {
    if ((t & 63) == 0) __hip_atomic_fetch_add(&s_tdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  int fail = -1;
  for (int s = 0; s < 4; ++s) {
    const int o = 16 * s;
    double* D = sD[s & 1];
    if (w == 0) {
      const int f = chol16(sA, D, o);
      if (f >= 0 && fail < 0) fail = o + f;
    }
    GPX_PANEL_STAMP(1 + 3 * s);
    __syncthreads();  // publishes L_ss and D_ss
    if (w == 0) {
      // Critical path, no barrier: T and U of the next pivot block, then straight on to its F.
      if (s + 1 < nrow) tsolve(s + 1, D, o);  // at s = 3 this is the first panel row block
      publish();
      GPX_PANEL_STAMP(2 + 3 * s);
      if (s < 3) update(s + 1, s + 1, o);
    } else {
      // Waves 1-3: the remaining T items (row blocks s+2.. and the panel rows), then - once every wave's T items of
      // this step are published - the remaining U items, overlapping wave 0's next F.
      for (int i = s + 1 + w; i < nrow; i += 3) tsolve(i, D, o);
      publish();
      GPX_PANEL_STAMP(2 + 3 * s);
      while (__hip_atomic_load(&s_tdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 4 * (s + 1))
        __builtin_amdgcn_s_sleep(1);
      int e = 0;
      for (int j = s + 1; j < 4; ++j) {
        for (int i = j; i < nrow; ++i) {
          if (i == s + 1 && j == s + 1) continue;  // wave 0's lookahead item
          if (1 + e % 3 == w) update(i, j, o);
          ++e;
        }
      }
    }
    GPX_PANEL_STAMP(3 + 3 * s);
  }
  __syncthreads();
  GPX_PANEL_STAMP(13);
  if (!panel) {
    if (t == 0 && fail >= 0) atomicCAS(info, 0, k * NB + fail + 1);
    const int nblk = gridDim.x + k;
    double* Lkk = Dinv + (int64_t)(nblk + k) * NB * NB;  // scratch copy, moved into A by syrk_update
    for (int e = t; e < NB * NB; e += WG) {
      const int r = e >> 6, c = e & 63;
      Lkk[e] = (c <= r) ? sA[r * LD64 + c] : 0.0;
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    *reinterpret_cast<double2*>(Aik + (int64_t)r * lda + c) = make_double2(sP[r * LD64 + c], sP[r * LD64 + c + 1]);
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

// D_k = L_kk^{-1} for every diagonal block (one workgroup per block), into the first half of Dinv.
__global__ void __launch_bounds__(WG) potrf_dinv_kernel(const double* __restrict__ A, int64_t lda,
                                                        double* __restrict__ Dinv, const int32_t* __restrict__ info) {
  if (*(volatile const int32_t*)info != 0) return;
  __shared__ __attribute__((aligned(16))) double sL[NB * LD64];
  __shared__ __attribute__((aligned(16))) double sX[NB * LD64];
  __shared__ __attribute__((aligned(16))) double sT[NB * LD64];
  const int k = blockIdx.x, t = threadIdx.x;
  const double* Lkk = A + (int64_t)k * NB * lda + (int64_t)k * NB;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    const double2 v = *reinterpret_cast<const double2*>(Lkk + (int64_t)r * lda + c);
    sL[r * LD64 + c] = v.x;
    sL[r * LD64 + c + 1] = v.y;
  }
  __syncthreads();
  trinv64(sL, sX, sT);
  double* D = Dinv + (int64_t)k * NB * NB;
  for (int e = t; e < NB * NB; e += WG) D[e] = sX[(e >> 6) * LD64 + (e & 63)];
}

hipError_t launch_potrf(Context* c, int npad, double* A, int64_t lda, double* Dinv, int32_t* info) {
  LaunchTimer tm(c, GPX_TIMER_POTRF);
  const int nblk = npad / NB;
  for (int k = 0; k < nblk; ++k) {
    potrf_panel_kernel<<<nblk - k, WG, 0, c->stream>>>(A, lda, k, Dinv, info);
    const int m = nblk - k - 1;
    syrk_update_kernel<<<m * (m + 1) / 2 + 1, WG, 0, c->stream>>>(A, lda, k, nblk, Dinv, info);
  }
  potrf_dinv_kernel<<<nblk, WG, 0, c->stream>>>(A, lda, Dinv, info);
  return hipGetLastError();
}

}  // namespace gpx
