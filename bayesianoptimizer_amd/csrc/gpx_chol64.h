// Factor + invert one 64x64 SPD diagonal block inside a 256-thread workgroup (used by potrf's panel kernel).
//
// The serial part of a Cholesky is its pivot chain, so this routine keeps every pivot inside ONE wave with no
// barrier and hands everything else to fp64 MFMA:
//   for each 16-column step s = 0..3:
//     F  (wave 0: lane r + 16 g owns row r, columns 4g..4g+3 of the 16x16 diagonal sub-block, fully unrolled):
//          16 pivots, column/row broadcasts through LDS inside the wave -> L_ss and D_ss = L_ss^{-1}
//     T  (3 waves): L_is = A_is D_ss^T for the sub-blocks below (16x16x16 MFMA from LDS)
//     U  (4 waves): A_ij -= L_is L_js^T for the trailing sub-blocks (MFMA)
//   then X = L^{-1} for the whole 64x64 by block forward substitution (X_ij = -D_ii sum_k L_ik X_kj, MFMA).
// 3 barriers per step + 6 for the inverse, instead of 2 per pivot.
//
// LDS: sA (64 x LD64) holds A on entry and L (lower; strict upper set to 0) on exit; sX (64 x LD64) receives
// L^{-1} (lower, strict upper 0); sT is a 64 x LD64 scratch.  Returns (in every thread) the 0-based failing
// pivot, or -1.
#pragma once
#include "gpx_device.h"

namespace gpx {

constexpr int LD64 = 68;  // padded row length (doubles) of the 64x64 LDS tiles

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffull), lane);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One 16x16 MFMA block product accumulated over K = 16*kb sub-blocks, operands from LDS tiles with row length
// LD64: acc += sum_t A(ra0.., ka0 + t) * B(kb0 + t, cb0..) where A is read row-major (A[row][k]) and B is read
// either row-major (B[k][col], BT=false) or as B[col][k] (BT=true, i.e. multiply by a transpose).
template <bool BT>
__device__ __forceinline__ d4 mfma_lds16(d4 acc, const double* A, int ra0, int ka0, const double* B, int kb0, int cb0,
                                         int K, double sign) {
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, kk = lane >> 4;
#pragma unroll 4
  for (int k = 0; k < K; k += 4) {
    const double a = sign * A[(ra0 + m) * LD64 + ka0 + k + kk];
    const double b = BT ? B[(cb0 + m) * LD64 + kb0 + k + kk] : B[(kb0 + k + kk) * LD64 + cb0 + m];
    acc = mfma16x16x4(a, b, acc);
  }
  return acc;
}

__device__ __forceinline__ d4 load_block16(const double* S, int r0, int c0) {
  const int lane = threadIdx.x & 63;
  d4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = S[(r0 + (lane >> 4) + 4 * q) * LD64 + c0 + (lane & 15)];
  return v;
}

__device__ __forceinline__ void store_block16(double* S, int r0, int c0, d4 v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 4; ++q) S[(r0 + (lane >> 4) + 4 * q) * LD64 + c0 + (lane & 15)] = v[q];
}

// Pivot square root and reciprocal: v_rsq_f64 refined by one Newton step (~1 ulp; the correctly rounded
// sqrt + division sequences cost ~25 dependent instructions on the pivot chain).
__device__ __forceinline__ void pivot_rsq(double piv, double& d, double& inv) {
  double y = __builtin_amdgcn_rsq(piv);
  const double h = 0.5 * piv;
  const double e = fma(-h * y, y, 0.5);
  y = fma(y, e, y);
  inv = y;
  d = piv * y;
}

// F phase: factor + invert the 16x16 block at (o, o) of sA with one whole wave; lane = r + 16 g owns row r,
// columns 4g..4g+3 of A (a[]) and of X = L^{-1} (x[], built in the same right-looking sweep).  Each pivot
// broadcasts column j of L and row j of X through two 16-double LDS slots (bc); LDS requests of one wave are
// served in order, so no barrier is needed.  L goes to sA (strict upper zeroed), X to sX.
__device__ __forceinline__ int chol16_wave(double* sA, double* sX, double* bc, int o) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  double a[4], x[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[q] = sA[(o + r) * LD64 + o + 4 * g + q];
    x[q] = (r == 4 * g + q) ? 1.0 : 0.0;
  }
  double* colbuf = bc;
  double* rowbuf = bc + 16;
  int fail = -1;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int gj = j >> 2, qj = j & 3;
    const double piv = readlane_f64(a[qj], j + 16 * gj);
    if (!(piv > 0.0) && fail < 0) fail = j;
    double d, inv;
    pivot_rsq(piv, d, inv);
    if (g == gj) {
      const double l = (r > j) ? a[qj] * inv : ((r == j) ? d : 0.0);
      a[qj] = l;
      colbuf[r] = l;
    }
    if (r == j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        x[q] *= inv;
        rowbuf[4 * g + q] = x[q];
      }
    }
    __builtin_amdgcn_wave_barrier();
    const double lr = colbuf[r];
    double lc[4], xj[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      lc[q] = colbuf[4 * g + q];
      xj[q] = rowbuf[4 * g + q];
    }
    __builtin_amdgcn_wave_barrier();
    if (r > j) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (4 * g + q > j) a[q] -= lr * lc[q];
        x[q] -= lr * xj[q];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * g + q;
    sA[(o + r) * LD64 + o + c] = (c <= r) ? a[q] : 0.0;
    sX[(o + r) * LD64 + o + c] = x[q];
  }
  return fail;
}

__device__ inline int chol_inv64(double* sA, double* sX, double* sT) {
  const int w = threadIdx.x >> 6;
  __shared__ int s_fail;
  if (threadIdx.x == 0) s_fail = -1;
  for (int s = 0; s < 4; ++s) {
    const int o = 16 * s;
    if (w == 0) {
      const int f = chol16_wave(sA, sX, sT, o);
      if ((threadIdx.x & 63) == 0 && f >= 0 && s_fail < 0) s_fail = o + f;
    }
    __syncthreads();
    // T: L_is = A_is D_ss^T (i = s+1..3), one sub-block per wave, written back in place (no other wave
    // touches block (i, s) in this phase)
    {
      const int i = s + 1 + w;
      if (i < 4) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma_lds16<true>(acc, sA, 16 * i, o, sX, o, o, 16, 1.0);  // B(k,n) = D[n][k]
        store_block16(sA, 16 * i, o, acc);
      }
    }
    __syncthreads();
    // U: A_ij -= L_is L_js^T for s < j <= i <= 3
    for (int e = w; e < 6; e += 4) {
      // enumerate the lower sub-blocks of the 3x3 trailing grid
      int ii, jj;
      if (e == 0) { ii = 1; jj = 1; } else if (e == 1) { ii = 2; jj = 1; } else if (e == 2) { ii = 2; jj = 2; }
      else if (e == 3) { ii = 3; jj = 1; } else if (e == 4) { ii = 3; jj = 2; } else { ii = 3; jj = 3; }
      const int i = s + ii, j = s + jj;
      if (i < 4 && j < 4) {
        d4 acc = load_block16(sA, 16 * i, 16 * j);
        acc = mfma_lds16<true>(acc, sA, 16 * i, o, sA, o, 16 * j, 16, -1.0);  // B(k,n) = L[j][k]
        store_block16(sA, 16 * i, 16 * j, acc);
      }
    }
    __syncthreads();
  }
  // X = L^{-1}: X_ii = D_ii (already in sX); X_ij = -D_ii * sum_{k=j}^{i-1} L_ik X_kj, by sub-diagonal.
  for (int dd = 1; dd < 4; ++dd) {
    const int nb = 4 - dd;  // blocks on this sub-diagonal
    if (w < nb) {
      const int j = w, i = w + dd;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int k = j; k < i; ++k) acc = mfma_lds16<false>(acc, sA, 16 * i, 16 * k, sX, 16 * k, 16 * j, 16, 1.0);
      store_block16(sT, 16 * i, 16 * j, acc);
    }
    __syncthreads();
    if (w < nb) {
      const int j = w, i = w + dd;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = mfma_lds16<false>(acc, sX, 16 * i, 16 * i, sT, 16 * i, 16 * j, 16, -1.0);
      store_block16(sX, 16 * i, 16 * j, acc);
    }
    __syncthreads();
  }
  // zero the strict upper 16x16 blocks of X
  for (int e = threadIdx.x; e < 64 * 64; e += WG) {
    const int rr = e >> 6, cc = e & 63;
    if ((cc >> 4) > (rr >> 4)) sX[rr * LD64 + cc] = 0.0;
  }
  __syncthreads();
  return s_fail;
}

}  // namespace gpx
