// Latency probe of the 16x16 pivot-block factorisation (diagnostic): one wave runs chol16 (rank-1 pivots) or
// chol16_mfma (4-pivot blocks on fp64 MFMA) REPS times on the same SPD block and reports cycles per call, plus the
// max difference between the two variants' L and D = L^{-1}.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        chol16_probe.hip -o chol16_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include "gpx_internal.h"
#include "gpx_chol64.h"
using namespace gpx;

namespace gpx {
// ---- 4-pivot blocked variant on the MFMA accumulator layout ----------------------------------------------------
// The 16x16 block lives in the C/D layout of v_mfma_f64_16x16x4: lane (g = lane/16, col = lane%16) holds rows g + 4q
// (q = 0..3) of column col, i.e. register q holds block row q (rows 4q .. 4q+3).  Step k factors pivots 4k .. 4k+3:
//   1. the 4x4 diagonal block (10 values, v_readlane) is factored and inverted by every lane (uniform scalar chain:
//      four rsq pivots + ~20 dependent FMAs), D_k = L_kk^{-1};
//   2. X's block row k (X = L^{-1}, built from I by the same block row operations) becomes D_k X_k (cross-row
//      broadcasts by permlane swaps, off the factorisation chain);
//   3. the rows below get L_ik = A_ik D_k^T (the four columns of a row sit in one DPP quad: quad_perm broadcasts);
//   4. the rank-4 trailing update A -= L_k L_k^T and X -= L_k X_k are ONE v_mfma_f64_16x16x4 each: their A operand is
//      lane (kk, m) = -L[m][4k+kk] (rows <= 4k+3 zeroed), the trailing update's B operand the same register un-negated
//      (lane (kk, n) = L[n][4k+kk]) and X's B operand X's own register k (lane (kk, n) = X[4k+kk][n]).  The operand
//      register is gathered from the TRSM's lanes by ds_bpermute.
// Per pivot ~150 cycles on the chain instead of ~380 for the rank-1 elimination above (chol16), whose per-pivot row
// broadcasts dominate.
template <int M>
__device__ __forceinline__ double quad_bcast_f64(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffull), M * 0x55, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), M * 0x55, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double bpermute_f64(int src_lane, double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane * 4, (int)(u & 0xffffffffull));
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane * 4, (int)(u >> 32));
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double sel4(int i, double v0, double v1, double v2, double v3) {
  return i == 0 ? v0 : (i == 1 ? v1 : (i == 2 ? v2 : v3));
}

// sF: per step k, 32 doubles of wave-private LDS: L_kk then D_k = L_kk^{-1}, each 4x4 row-major (zeros above the
// diagonal).  Lanes fetch their lane-dependent coefficients from it (one ds_read_b128 pair) instead of selecting
// among the uniform values (v_cndmask chains were ~15 % of the first version's instructions).
template <int K>
__device__ __forceinline__ void chol16_block_step(d4& A, d4& X, int g, int col, unsigned& bad, double* sF) {
  const int lane = threadIdx.x & 63;
  // 1. the 4x4 diagonal block, uniform (v_readlane into SGPRs)
  const double a00 = readlane_f64(A[K], 4 * K), a10 = readlane_f64(A[K], 16 + 4 * K),
               a11 = readlane_f64(A[K], 16 + 4 * K + 1), a20 = readlane_f64(A[K], 32 + 4 * K),
               a21 = readlane_f64(A[K], 32 + 4 * K + 1), a22 = readlane_f64(A[K], 32 + 4 * K + 2),
               a30 = readlane_f64(A[K], 48 + 4 * K), a31 = readlane_f64(A[K], 48 + 4 * K + 1),
               a32 = readlane_f64(A[K], 48 + 4 * K + 2), a33 = readlane_f64(A[K], 48 + 4 * K + 3);
  const double r0 = pivot_rsq(a00);
  const double l00 = a00 * r0, l10 = a10 * r0, l20 = a20 * r0, l30 = a30 * r0;
  const double p1 = fma(-l10, l10, a11);
  const double r1 = pivot_rsq(p1);
  const double l11 = p1 * r1, l21 = fma(-l20, l10, a21) * r1, l31 = fma(-l30, l10, a31) * r1;
  const double p2 = fma(-l21, l21, fma(-l20, l20, a22));
  const double r2 = pivot_rsq(p2);
  const double l22 = p2 * r2, l32 = fma(-l31, l21, fma(-l30, l20, a32)) * r2;
  const double p3 = fma(-l32, l32, fma(-l31, l31, fma(-l30, l30, a33)));
  const double r3 = pivot_rsq(p3);
  const double l33 = p3 * r3;
  // failed pivots as bits 4k + i (branch-free: the values are uniform but the compiler cannot prove it)
  bad |= ((a00 > 0.0) ? 0u : 1u) << (4 * K) | ((p1 > 0.0) ? 0u : 2u) << (4 * K) | ((p2 > 0.0) ? 0u : 4u) << (4 * K) |
         ((p3 > 0.0) ? 0u : 8u) << (4 * K);
  // D_k = L_kk^{-1} (lower)
  const double d10 = -(l10 * r0) * r1, d21 = -(l21 * r1) * r2, d32 = -(l32 * r2) * r3;
  const double d20 = -fma(l21, d10, l20 * r0) * r2;
  const double d31 = -fma(l32, d21, l31 * r1) * r3;
  const double d30 = -fma(l32, d20, fma(l31, d10, l30 * r0)) * r3;
  double* F = sF + 32 * K;
  if (lane == 0) {
    double2* F2 = reinterpret_cast<double2*>(F);
    F2[0] = make_double2(l00, 0.0);
    F2[1] = make_double2(0.0, 0.0);
    F2[2] = make_double2(l10, l11);
    F2[3] = make_double2(0.0, 0.0);
    F2[4] = make_double2(l20, l21);
    F2[5] = make_double2(l22, 0.0);
    F2[6] = make_double2(l30, l31);
    F2[7] = make_double2(l32, l33);
    F2[8] = make_double2(r0, 0.0);
    F2[9] = make_double2(0.0, 0.0);
    F2[10] = make_double2(d10, r1);
    F2[11] = make_double2(0.0, 0.0);
    F2[12] = make_double2(d20, d21);
    F2[13] = make_double2(r2, 0.0);
    F2[14] = make_double2(d30, d31);
    F2[15] = make_double2(d32, r3);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): lane 0's table writes land before the wave reads them
  const double* Dk = F + 16;
  const int m = lane & 15, kk = lane >> 4;  // MFMA A/B operand coordinates of this lane
  // 2. X block row k <- D_k X_k as one MFMA: A = D_k in rows 4k..4k+3 (lane (kk, m): D_k[m - 4k][kk]), B = X_k (X's own
  //    register k), C = X with block row k cleared (its register k)
  {
    const double dop = (m >> 2) == K ? Dk[(m & 3) * 4 + kk] : 0.0;
    d4 Xc = X;
    Xc[K] = 0.0;
    X = mfma16x16x4(dop, X[K], Xc);
  }
  const int cb = col >> 2, j = col & 3;
  if constexpr (K < 3) {
    // 3. L_ik = A_ik D_k^T for the block rows i > k (lanes col = 4k + j): coefficients D_k[j][0..3]
    const double2 e01 = *reinterpret_cast<const double2*>(Dk + 4 * j);
    const double2 e23 = *reinterpret_cast<const double2*>(Dk + 4 * j + 2);
#pragma unroll
    for (int i = K + 1; i < 4; ++i) {
      const double v0 = quad_bcast_f64<0>(A[i]), v1 = quad_bcast_f64<1>(A[i]), v2 = quad_bcast_f64<2>(A[i]),
                   v3 = quad_bcast_f64<3>(A[i]);
      const double l = fma(e23.y, v3, fma(e23.x, v2, fma(e01.y, v1, e01.x * v0)));
      A[i] = cb == K ? l : A[i];
    }
    // 4. operand lane (kk, m) = L[m][4k+kk] for m > 4k+3: from lane 16 (m%4) + 4k + kk, register m/4
    const int src = 16 * (m & 3) + 4 * K + kk;
    double op = 0.0;
#pragma unroll
    for (int i = K + 1; i < 4; ++i) {
      const double v = bpermute_f64(src, A[i]);
      op = (m >> 2) == i ? v : op;
    }
    A = mfma16x16x4(-op, op, A);
    X = mfma16x16x4(-op, X[K], X);
  }
}

// Factor + invert the 16x16 SPD block at (o, o) of sA with one wave, as chol16 (same outputs, same contract); sF: 128
// doubles of LDS scratch for this wave.
template <int LDD>
__device__ __forceinline__ int chol16_mfma(double* sA, double* sD, int o, double* sF) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, col = lane & 15;
  d4 A, X;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    A[q] = sA[(o + g + 4 * q) * LD64 + o + col];
    X[q] = (g + 4 * q == col) ? 1.0 : 0.0;
  }
  unsigned bad = 0;
  chol16_block_step<0>(A, X, g, col, bad, sF);
  chol16_block_step<1>(A, X, g, col, bad, sF);
  chol16_block_step<2>(A, X, g, col, bad, sF);
  chol16_block_step<3>(A, X, g, col, bad, sF);
  const int cb = col >> 2, j = col & 3;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = g + 4 * q;
    // diagonal 4x4 blocks from the step tables, the rest from the TRSM'd registers
    const double lv = cb == q ? sF[32 * q + 4 * g + j] : A[q];
    sA[(o + r) * LD64 + o + col] = col <= r ? lv : 0.0;
    sD[r * LDD + col] = col <= r ? X[q] : 0.0;
  }
  return bad ? __builtin_ctz(bad) : -1;
}

}  // namespace gpx
// ---- cost split of the rank-1 pivot chain (timing only: V = 2 drops X = L^{-1} and the L column capture, V = 3 drops
// only the capture, V = 4 drops only X; results are not valid for V >= 2) ----
#define GPX_FMAC_REST3(J)                                                                                        \
  case J:                                                                                                        \
    asm volatile("v_fmac_f64_dpp %0, %0, %3 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %1, %1, %3 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %2, %2, %3 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"                       \
                 : "+v"(a1), "+v"(a2), "+v"(a3)                                                                  \
                 : "v"(ca));                                                                                     \
    break;
template <int J>
__device__ __forceinline__ void fmac_rest3(double& a1, double& a2, double& a3, double ca) {
  switch (J) {
    GPX_FMAC_REST3(0) GPX_FMAC_REST3(1) GPX_FMAC_REST3(2) GPX_FMAC_REST3(3) GPX_FMAC_REST3(4) GPX_FMAC_REST3(5)
    GPX_FMAC_REST3(6) GPX_FMAC_REST3(7) GPX_FMAC_REST3(8) GPX_FMAC_REST3(9) GPX_FMAC_REST3(10) GPX_FMAC_REST3(11)
    GPX_FMAC_REST3(12) GPX_FMAC_REST3(13) GPX_FMAC_REST3(14) GPX_FMAC_REST3(15)
  }
}
template <int V, int J>
__device__ __forceinline__ void pivot_var(Blk16& b, int r, int g, int& fail, double& piv, double& arj) {
  constexpr int GJ = J >> 2, QJ = J & 3;
  if (!(piv > 0.0) && fail < 0) fail = J;
  const double isq = pivot_rsq(piv);
  const double rinv = isq * isq;
  const double coef = (r > J) ? -arj * rinv : 0.0;
  if (V == 4 && g == GJ) b.l[QJ] = (r >= J) ? b.a[QJ] * isq : 0.0;
  if constexpr (J < 15) {
    constexpr int JN = J + 1, GN = JN >> 2, QN = JN & 3;
    fmac_pipe_first<J>(b.a[QN], coef);
    piv = readlane_f64(b.a[QN], JN + 16 * GN);
    arj = xrow_bcast_f64<GN>(b.a[QN]);
    if constexpr (V == 3) {
      const double coefx = (r == J) ? isq - 1.0 : coef;
      fmac_pipe_rest<J>(b.a[(QN + 1) & 3], b.a[(QN + 2) & 3], b.a[(QN + 3) & 3], b.x, coef, coefx);
    } else {
      fmac_rest3<J>(b.a[(QN + 1) & 3], b.a[(QN + 2) & 3], b.a[(QN + 3) & 3], coef);
    }
  }
}
template <int V, int... J>
__device__ __forceinline__ void pivots_var(Blk16& b, int r, int g, int& fail, std::integer_sequence<int, J...>) {
  double piv = readlane_f64(b.a[0], 0), arj = xrow_bcast_f64<0>(b.a[0]);
  (pivot_var<V, J>(b, r, g, fail, piv, arj), ...);
}
template <int V, int LDD>
__device__ __forceinline__ int chol16_var(double* sA, double* sD, int o) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  Blk16 b;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    b.a[q] = sA[(o + r) * LD64 + o + 4 * g + q];
    b.x[q] = (r == 4 * g + q) ? 1.0 : 0.0;
    b.l[q] = 0.0;
  }
  int fail = -1;
  pivots_var<V>(b, r, g, fail, std::make_integer_sequence<int, 16>{});
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * g + q;
    sA[(o + r) * LD64 + o + c] = V == 4 ? b.l[q] : b.a[q];
    sD[r * LDD + c] = b.x[q];
  }
  return fail;
}

#ifndef VARIANT
#define VARIANT ""
#endif
constexpr int LDD = 20, REPS = 64;

template <int V>
__global__ void probe(const double* A, double* L, double* D, long long* cyc) {
  __shared__ double sA[16 * LD64], sD[16 * LDD], sF[128];
  const int t = threadIdx.x;
  long long total = 0;
  int f = -1;
  for (int r = 0; r < REPS; ++r) {
    for (int e = t; e < 256; e += 64) sA[(e >> 4) * LD64 + (e & 15)] = A[e];
    __syncthreads();
    const long long c0 = __builtin_readcyclecounter();
    if (V == 0)
      f = chol16<LDD>(sA, sD, 0);
    else if (V == 1)
      f = chol16_mfma<LDD>(sA, sD, 0, sF);
    else
      f = chol16_var<V, LDD>(sA, sD, 0);
    __syncthreads();
    total += __builtin_readcyclecounter() - c0;
  }
  for (int e = t; e < 256; e += 64) {
    L[e] = sA[(e >> 4) * LD64 + (e & 15)];
    D[e] = sD[(e >> 4) * LDD + (e & 15)];
  }
  if (t == 0) cyc[0] = total / REPS, cyc[1] = f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  double hA[256];
  srand(7);
  double B[256];
  for (int i = 0; i < 256; ++i) B[i] = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = i == j ? 16.0 : 0.0;
      for (int k = 0; k < 16; ++k) s += B[i * 16 + k] * B[j * 16 + k];
      hA[i * 16 + j] = s;
    }
  double *A, *L, *D;
  long long* cyc;
  CK(hipMalloc(&A, 2048));
  CK(hipMalloc(&L, 2 * 2048));
  CK(hipMalloc(&D, 2 * 2048));
  CK(hipMalloc(&cyc, 32));
  CK(hipMemcpy(A, hA, 2048, hipMemcpyHostToDevice));
  long long hc[2][2];
  probe<0><<<1, 64>>>(A, L, D, cyc);
  CK(hipMemcpy(hc[0], cyc, 16, hipMemcpyDeviceToHost));
  probe<1><<<1, 64>>>(A, L + 256, D + 256, cyc);
  CK(hipMemcpy(hc[1], cyc, 16, hipMemcpyDeviceToHost));
  double hL[512], hD[512];
  CK(hipMemcpy(hL, L, 4096, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hD, D, 4096, hipMemcpyDeviceToHost));
  double dl = 0, dd = 0, res = 0;
  for (int i = 0; i < 256; ++i) dl = fmax(dl, fabs(hL[i] - hL[256 + i])), dd = fmax(dd, fabs(hD[i] - hD[256 + i]));
  for (int i = 0; i < 16; ++i)  // |L L^T - A|
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += hL[256 + i * 16 + k] * hL[256 + j * 16 + k];
      res = fmax(res, fabs(s - hA[i * 16 + j]));
    }
  printf("chol16 (rank-1" VARIANT "): %lld cycles/call, fail=%lld\n", hc[0][0], hc[0][1]);
  {
    long long hv[2];
    probe<2><<<1, 64>>>(A, L + 256, D + 256, cyc);
    CK(hipMemcpy(hv, cyc, 16, hipMemcpyDeviceToHost));
    printf("chol16 A-chain only (no X, no L capture): %lld cycles/call\n", hv[0]);
    probe<3><<<1, 64>>>(A, L + 256, D + 256, cyc);
    CK(hipMemcpy(hv, cyc, 16, hipMemcpyDeviceToHost));
    printf("chol16 without the L capture:            %lld cycles/call\n", hv[0]);
    probe<4><<<1, 64>>>(A, L + 256, D + 256, cyc);
    CK(hipMemcpy(hv, cyc, 16, hipMemcpyDeviceToHost));
    printf("chol16 without X:                        %lld cycles/call\n", hv[0]);
  }
  printf("chol16_mfma:     %lld cycles/call, fail=%lld\n", hc[1][0], hc[1][1]);
  printf("max|dL|=%.2e max|dD|=%.2e  mfma |LL^T-A|=%.2e\n", dl, dd, res);
  printf("CHOL16 PROBE DONE\n");
  return 0;
}
