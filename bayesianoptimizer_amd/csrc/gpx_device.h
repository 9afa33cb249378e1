// Device-side helpers shared by the gpx kernels: covariance evaluation, triangular tile decoding and the
// fp64 MFMA tile core (v_mfma_f64_16x16x4_f64, 64-lane waves).
#pragma once
#include <hip/hip_runtime.h>
#include "gpx_internal.h"

namespace gpx {

// ---- covariance ---------------------------------------------------------------------------------
// Matches oracle/gp_oracle.py::kernel_matrix term for term: r2 is the sum over dimensions of
// ((a_k - b_k) / l_k)^2 accumulated in order k = 0..d-1, `lin` the ARD linear term.
__device__ __forceinline__ double cov_from_r2(int kind, double outputscale, double r2, double lin) {
  if (kind == GPX_KERNEL_RBF) return outputscale * exp(-0.5 * r2);
  const double r = sqrt(r2);
  const double s5r = 2.23606797749978969640917366873128 * r;  // sqrt(5) r
  const double m = (1.0 + s5r + (5.0 / 3.0) * r2) * exp(-s5r);
  if (kind == GPX_KERNEL_MATERN52) return outputscale * m;
  return outputscale * (lin + m);
}

// fp32 evaluation (gpx_kernel_params.cov_fp32, BASELINE configs[4]): r2 accumulated in fp32 from fp32-rounded
// scaled inputs, exp / sqrt / Matern polynomial in fp32, widened to fp64 before the outputscale and linear part.
__device__ __forceinline__ double cov_from_r2_f32(int kind, double outputscale, float r2, double lin) {
  if (kind == GPX_KERNEL_RBF) return outputscale * (double)expf(-0.5f * r2);
  const float r = sqrtf(r2);
  const float s5r = 2.2360679774997897f * r;
  const float m = (1.0f + s5r + (5.0f / 3.0f) * r2) * expf(-s5r);
  if (kind == GPX_KERNEL_MATERN52) return outputscale * (double)m;
  return outputscale * (lin + (double)m);
}

// Squared distance in GPyTorch's expanded form [upstream]: ||a||^2 + ||b||^2 - 2 a.b clamped at 0.  The clamp is written
// so that a NaN input stays NaN (fmax would turn it into 0: a NaN training input must still fail the Cholesky, and a NaN
// candidate must still score NaN).
__device__ __forceinline__ double sqdist_expanded(double na, double nb, double dot) {
  const double x = fma(-2.0, dot, na + nb);
  return x < 0.0 ? 0.0 : x;
}

// Exchange of the 16-lane rows of two registers (rows32: rows 2, 3 of a with rows 0, 1 of b, v_permlane32_swap; else
// the odd rows of a with the even rows of b, v_permlane16_swap), both 32-bit halves.
__device__ __forceinline__ void swap_halves(double& a, double& b, bool rows32) {
  const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
  const unsigned alo = (unsigned)ua, ahi = (unsigned)(ua >> 32), blo = (unsigned)ub, bhi = (unsigned)(ub >> 32);
  unsigned nalo, nahi, nblo, nbhi;
  if (rows32) {
    const auto l = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    nalo = l[0], nblo = l[1], nahi = h[0], nbhi = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    nalo = l[0], nblo = l[1], nahi = h[0], nbhi = h[1];
  }
  a = __longlong_as_double(((unsigned long long)nahi << 32) | nalo);
  b = __longlong_as_double(((unsigned long long)nbhi << 32) | nblo);
}
// v[q] of 16-lane row g becomes the old v[g] of row q (a 4 x 4 transpose of (lane row) x (register))
__device__ __forceinline__ void transpose_rows4(double (&v)[4]) {
  swap_halves(v[0], v[2], true);
  swap_halves(v[1], v[3], true);
  swap_halves(v[0], v[1], false);
  swap_halves(v[2], v[3], false);
}

// Linear index t over the lower triangle of an m x m block grid (row-major order of (i, j), j <= i)
// -> (i, j).
__device__ __forceinline__ void tri_decode(int t, int& i, int& j) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  i = r;
  j = t - r * (r + 1) / 2;
}

__device__ __forceinline__ d4 mfma16x16x4(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---- fp64 MFMA GEMM tile core ---------------------------------------------------------------------
// One 256-thread workgroup computes a TM x TN tile C = sum_k A(m,k) B(k,n) over k in [kbeg, kend)
// (multiples of BK).  Four waves in a 2x2 arrangement each own a (TM/2) x (TN/2) sub-tile made of
// (TM/32) x (TN/32) MFMA 16x16 blocks.
//   A_KMAJOR: A(m,k) at A[k*lda + m]  else A[m*lda + k]
//   B_KMAJOR: B(k,n) at B[k*ldb + n]  else B[n*ldb + k]
// Operands are staged global -> registers -> LDS (k-major, rows padded by 16 doubles so the two
// 16-lane halves of each ds_read_b64 group hit disjoint banks), double-buffered with one barrier per
// k-tile; the next k-tile's global loads are issued before the current tile's MFMAs.
// Accumulator layout (measured on gfx950, tools/probes/mfma_f64_probe.hip):
//   acc[i][j][r] holds C(row = wm0 + 16 i + (lane>>4) + 4 r, col = wn0 + 16 j + (lane&15)).
template <int TM, int TN, int BK, bool A_KMAJOR, bool B_KMAJOR>
struct MfmaTile {
  static constexpr int WM = TM / 32;  // MFMA blocks per wave along m
  static constexpr int WN = TN / 32;
  static constexpr int PA = TM + 16;  // padded LDS row lengths
  static constexpr int PB = TN + 16;
  static constexpr int LDS_DOUBLES = 2 * BK * (PA + PB);
  // register staging: each thread moves 2 consecutive doubles per load
  static constexpr int A_LOADS = TM * BK / (2 * WG);
  static constexpr int B_LOADS = TN * BK / (2 * WG);
  static_assert(A_LOADS >= 1 && B_LOADS >= 1, "tile too small for 256 threads");

  d4 acc[WM][WN];
  double2 ra[A_LOADS], rb[B_LOADS];

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  }

  // global -> registers for the k-tile starting at k0
  __device__ __forceinline__ void load_regs(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                            int64_t ldb, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < A_LOADS; ++q) {
      int e = (t + q * WG) * 2;  // element offset inside the BK x TM (k-major) or TM x BK tile
      if (A_KMAJOR) {
        int kk = e / TM, mm = e % TM;
        ra[q] = *reinterpret_cast<const double2*>(A + (int64_t)(k0 + kk) * lda + mm);
      } else {
        int mm = e / BK, kk = e % BK;
        ra[q] = *reinterpret_cast<const double2*>(A + (int64_t)mm * lda + k0 + kk);
      }
    }
#pragma unroll
    for (int q = 0; q < B_LOADS; ++q) {
      int e = (t + q * WG) * 2;
      if (B_KMAJOR) {
        int kk = e / TN, nn = e % TN;
        rb[q] = *reinterpret_cast<const double2*>(B + (int64_t)(k0 + kk) * ldb + nn);
      } else {
        int nn = e / BK, kk = e % BK;
        rb[q] = *reinterpret_cast<const double2*>(B + (int64_t)nn * ldb + k0 + kk);
      }
    }
  }

  // LDS column of element (m, k) of a row-major (not k-major) operand.  Its k-major transpose is written with
  // scalar ds_write_b64: a 16-lane write group holds 8 k-rows x 2 m, and with row pitch = 16 mod 32 doubles
  // all 8 k-rows land on one bank pair (8-way conflict, the MFMA loop then waits on LDS stores).  XOR-ing m
  // with (k & 14) spreads them over all 32 banks; the MFMA fragment reads (16 consecutive m of one k-row per
  // 16 lanes) only permute inside an aligned 16-block, so they stay conflict-free.
  __device__ __forceinline__ static int swz(int m, int k) { return m ^ (k & 14); }

  // registers -> LDS buffer
  __device__ __forceinline__ void store_lds(double* sA, double* sB) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < A_LOADS; ++q) {
      int e = (t + q * WG) * 2;
      if (A_KMAJOR) {
        int kk = e / TM, mm = e % TM;
        *reinterpret_cast<double2*>(sA + kk * PA + mm) = ra[q];
      } else {
        int mm = e / BK, kk = e % BK;
        const int c = swz(mm, kk);
        sA[kk * PA + c] = ra[q].x;
        sA[(kk + 1) * PA + c] = ra[q].y;
      }
    }
#pragma unroll
    for (int q = 0; q < B_LOADS; ++q) {
      int e = (t + q * WG) * 2;
      if (B_KMAJOR) {
        int kk = e / TN, nn = e % TN;
        *reinterpret_cast<double2*>(sB + kk * PB + nn) = rb[q];
      } else {
        int nn = e / BK, kk = e % BK;
        const int c = swz(nn, kk);
        sB[kk * PB + c] = rb[q].x;
        sB[(kk + 1) * PB + c] = rb[q].y;
      }
    }
  }

  __device__ __forceinline__ void frag(const double* sA, const double* sB, int ks, double* a, double* b) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int wm0 = (w >> 1) * (TM / 2);
    const int wn0 = (w & 1) * (TN / 2);
    const int kr = lane >> 4, cl = lane & 15;
    const int row = ks + kr;
    const int xa = A_KMAJOR ? 0 : (row & 14), xb = B_KMAJOR ? 0 : (row & 14);
#pragma unroll
    for (int i = 0; i < WM; ++i) a[i] = sA[row * PA + ((wm0 + 16 * i + cl) ^ xa)];
#pragma unroll
    for (int j = 0; j < WN; ++j) b[j] = sB[row * PB + ((wn0 + 16 * j + cl) ^ xb)];
  }

  __device__ __forceinline__ void mm(const double* a, const double* b) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = mfma16x16x4(a[i], b[j], acc[i][j]);
  }

  // Fragments are register double-buffered: the next k-substep's ds_reads are issued before the current
  // substep's MFMAs (+2-4 % on the sweep product, tools/trmm_bench.hip v5).
  __device__ __forceinline__ void compute(const double* sA, const double* sB) {
    static_assert(BK % 8 == 0, "BK must be a multiple of 8");
    double a0[WM], b0[WN], a1[WM], b1[WN];
    frag(sA, sB, 0, a0, b0);
#pragma unroll
    for (int ks = 0; ks < BK; ks += 8) {
      frag(sA, sB, ks + 4, a1, b1);
      mm(a0, b0);
      if (ks + 8 < BK) frag(sA, sB, ks + 8, a0, b0);
      mm(a1, b1);
    }
  }

  // The same k-tile with the MFMAs in row-block-major order (for i: for k-substep: for j): every accumulator still sees
  // its k values in ascending order (same bits), but the row block i = 0 needs only its own accumulators, so when acc is
  // seeded by loads issued in i order the first MFMAs wait for the first quarter of the seeds instead of all of them.
  __device__ __forceinline__ void compute_rows(const double* sA, const double* sB) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int wm0 = (w >> 1) * (TM / 2);
    const int wn0 = (w & 1) * (TN / 2);
    const int kr = lane >> 4, cl = lane & 15;
    double b[BK / 4][WN];
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const int row = 4 * s + kr;
      const int xb = B_KMAJOR ? 0 : (row & 14);
#pragma unroll
      for (int j = 0; j < WN; ++j) b[s][j] = sB[row * PB + ((wn0 + 16 * j + cl) ^ xb)];
    }
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        const int row = 4 * s + kr;
        const int xa = A_KMAJOR ? 0 : (row & 14);
        const double a = sA[row * PA + ((wm0 + 16 * i + cl) ^ xa)];
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = mfma16x16x4(a, b[s][j], acc[i][j]);
      }
  }

  // acc = -C (C: the TM x TN tile at Cg, row-major, leading dimension ldc): every load issued at once, so a following
  // run_acc(...) leaves acc = A B - C with no load round trip after the k loop (the caller stores -acc).
  __device__ __forceinline__ void load_neg_c(const double* __restrict__ Cg, int64_t ldc) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = -Cg[(int64_t)row_of(i, r) * ldc + col_of(j)];
  }

  // Full k loop. smem must hold LDS_DOUBLES doubles.  A/B point at the tile origin (m0 / n0 applied).
  // One loop body with swapped current/next LDS pointers: the two-branch (even/odd buffer) form made hipcc
  // rename the accumulators between branches and shuttle them through AGPR moves after dependent MFMAs
  // (48.7 vs 64.0 TF/s on the n=4096 sweep product, tools/trmm_bench.hip).
  __device__ __forceinline__ void run(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                      int64_t ldb, int kbeg, int kend, double* smem) {
    zero();
    run_acc(A, lda, B, ldb, kbeg, kend, smem);
  }

  // The same k loop accumulating onto the current acc.
  __device__ __forceinline__ void run_acc(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                          int64_t ldb, int kbeg, int kend, double* smem) {
    run_acc_after(A, lda, B, ldb, kbeg, kend, smem, [] {});
  }

  // run_acc with after_first() called once the first k-tile's global loads are issued (e.g. loads that seed acc: issued
  // behind the staging loads, so the first LDS store does not wait for them; kend > kbeg).
  // ROWS_FIRST: the first k-tile's MFMAs in row-block-major order (compute_rows), for seeds loaded by after_first.
  template <bool ROWS_FIRST = false, typename F>
  __device__ __forceinline__ void run_acc_after(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                                int64_t ldb, int kbeg, int kend, double* smem, F&& after_first) {
    if (kend <= kbeg) return;
    double* cur = smem;
    double* nxt = smem + BK * (PA + PB);
    load_regs(A, lda, B, ldb, kbeg);
    after_first();
    store_lds(cur, cur + BK * PA);
    __syncthreads();
    if constexpr (ROWS_FIRST) {
      const bool more = kbeg + BK < kend;
      if (more) load_regs(A, lda, B, ldb, kbeg + BK);
      compute_rows(cur, cur + BK * PA);
      if (more) store_lds(nxt, nxt + BK * PA);
      __syncthreads();
      double* t = cur;
      cur = nxt;
      nxt = t;
      kbeg += BK;
    }
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      const bool more = (k0 + BK) < kend;
      if (more) load_regs(A, lda, B, ldb, k0 + BK);
      compute(cur, cur + BK * PA);
      if (more) store_lds(nxt, nxt + BK * PA);
      __syncthreads();
      double* t = cur;
      cur = nxt;
      nxt = t;
    }
  }

  // The same accumulation with the last k-tile peeled: before_last() runs right before its MFMAs, when no staging loads
  // are in flight and the staging registers are dead, so an epilogue's first global loads overlap that k-tile without
  // holding registers across the loop (kend > kbeg).
  template <typename F>
  __device__ __forceinline__ void run_acc_peeled(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                                 int64_t ldb, int kbeg, int kend, double* smem, F&& before_last) {
    double* cur = smem;
    double* nxt = smem + BK * (PA + PB);
    load_regs(A, lda, B, ldb, kbeg);
    store_lds(cur, cur + BK * PA);
    __syncthreads();
    for (int k0 = kbeg; k0 + BK < kend; k0 += BK) {
      load_regs(A, lda, B, ldb, k0 + BK);
      compute(cur, cur + BK * PA);
      store_lds(nxt, nxt + BK * PA);
      __syncthreads();
      double* t = cur;
      cur = nxt;
      nxt = t;
    }
    before_last();
    compute(cur, cur + BK * PA);
    __syncthreads();
  }

  // Row / column of accumulator element (i, j, r) for this lane, relative to the tile origin.
  __device__ __forceinline__ static int row_of(int i, int r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    return (w >> 1) * (TM / 2) + 16 * i + (lane >> 4) + 4 * r;
  }
  __device__ __forceinline__ static int col_of(int j) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    return (w & 1) * (TN / 2) + 16 * j + (lane & 15);
  }
};

}  // namespace gpx
