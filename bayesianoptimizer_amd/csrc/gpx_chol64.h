// In-wave building blocks of the blocked Cholesky (gpx_potrf.hip): a 16x16 pivot block factored and inverted by
// ONE wave in registers (no barrier per pivot), plus the 16x16 fp64-MFMA block products the panel kernel builds on.
//
// Register layout of a 16x16 block in a wave: lane = r + 16 g owns row r, columns 4g..4g+3.  At pivot j the pivot
// A[j][j] is one lane's register (v_readlane, uniform); every lane applies the unscaled rank-1 update
// A[r][c] -= A[r][j] A[j][c] / A[j][j] and the same row operation on X = L^{-1}, with the cross-lane operands moved
// by DPP and gfx950 permlane swaps, so only the pivot's rsq sits between two consecutive pivots.  Row j is final from
// pivot j on (its multiplier is 0), so after the last pivot the registers hold the unscaled upper factor U (row j =
// A^(j)[j][.], U[j][j] the pivot) and L = (U diag(1/sqrt(U[j][j])))^T needs no capture on the pivot chain: the panel
// scales it only where L_cc is stored (round 5: the per-pivot column capture cost 484 of 3628 cycles per block,
// profiles/r04_chol16_split.log).  LDS tiles use a padded row length LD64 (doubles).
#pragma once
#include <utility>
#include "gpx_device.h"

namespace gpx {

constexpr int LD64 = 68;  // padded row length (doubles) of the 64-wide LDS tiles

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffull), lane);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Lane J of every 16-lane row, broadcast to the whole row (v_mov_b64_dpp row_newbcast:J).
template <int J>
__device__ __forceinline__ double row_newbcast(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xf, 0xf, false);
}

// Pivot reciprocal square root: v_rsq_f64 refined by one Newton step (~1 ulp; the correctly rounded sqrt +
// division sequence costs ~25 dependent instructions on the pivot chain).
__device__ __forceinline__ double pivot_rsq(double piv) {
  double y = __builtin_amdgcn_rsq(piv);
  const double h = 0.5 * piv;
  const double e = fma(-h * y, y, 0.5);
  return fma(y, e, y);
}

struct Blk16 {
  double a[4];  // A: trailing rows updated in place; row j is final (U) once pivot j has been applied
  double x[4];  // X = L^{-1} (the factorisation's row operations applied to I)
};

// Lane J of every 16-lane row, broadcast to the whole row, as two v_mov_b32_dpp row_newbcast:J (no old value;
// the 64-bit v_mov_b64_dpp form costs an extra zeroing move and a hazard nop per value, 17 cycles per link).
template <int J>
__device__ __forceinline__ double row_bcast(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffull), 0x150 + J, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), 0x150 + J, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Lane (r + 16 G) of every 16-lane row position r, broadcast to all four rows of the wave: gfx950's
// v_permlane32_swap (rows 2,3 <-> rows 0,1 of a second copy) then v_permlane16_swap (odd <-> even rows), two VALU
// ops per 32-bit half instead of a ds_bpermute round trip through the LDS crossbar on the pivot chain.
template <int G>
__device__ __forceinline__ unsigned xrow_bcast_u32(unsigned x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // [0]: rows (0 1 0 1), [1]: rows (2 3 2 3)
  const unsigned y = (G < 2) ? r[0] : r[1];
  const auto s = __builtin_amdgcn_permlane16_swap(y, y, false, false);  // [0]: even row everywhere, [1]: odd row
  return (G % 2 == 0) ? s[0] : s[1];
}

template <int G>
__device__ __forceinline__ double xrow_bcast_f64(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = xrow_bcast_u32<G>((unsigned)(u & 0xffffffffull));
  const unsigned hi = xrow_bcast_u32<G>((unsigned)(u >> 32));
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// a[q] += ca * bcast_J(a[q]) and x[q] += cx * bcast_J(x[q]) (q = 0..3) as eight v_fmac_f64_dpp row_newbcast:J: the
// gfx90a+ 64-bit DPP form folds the row broadcast into the FMA (hipcc emits v_mov_b64_dpp + v_fmac_f64 instead, three
// instructions per value with the 32-bit halves).  The compiler's hazard recognizer does not see inside the asm, so
// the block pads the DPP read of a fresh VALU result and the next DPP / permlane read of its outputs (2 wait states
// each, as hipcc pads its own).
#define GPX_FMAC_DPP8(J)                                                                                         \
  case J:                                                                                                        \
    asm("s_nop 1\n\t"                                                                                            \
        "v_fmac_f64_dpp %0, %0, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %1, %1, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %2, %2, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %3, %3, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %4, %4, %9 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %5, %5, %9 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %6, %6, %9 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "v_fmac_f64_dpp %7, %7, %9 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                           \
        "s_nop 1"                                                                                                \
        : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3])         \
        : "v"(ca), "v"(cx));                                                                                     \
    break;
template <int J>
__device__ __forceinline__ void fmac_row_bcast8(double (&a)[4], double (&x)[4], double ca, double cx) {
  switch (J) {
    GPX_FMAC_DPP8(0) GPX_FMAC_DPP8(1) GPX_FMAC_DPP8(2) GPX_FMAC_DPP8(3) GPX_FMAC_DPP8(4) GPX_FMAC_DPP8(5)
    GPX_FMAC_DPP8(6) GPX_FMAC_DPP8(7) GPX_FMAC_DPP8(8) GPX_FMAC_DPP8(9) GPX_FMAC_DPP8(10) GPX_FMAC_DPP8(11)
    GPX_FMAC_DPP8(12) GPX_FMAC_DPP8(13) GPX_FMAC_DPP8(14) GPX_FMAC_DPP8(15)
  }
}
#undef GPX_FMAC_DPP8

// Pipelined pivot J in two asm blocks: (1) the register the next pivot reads, a[QN] (leading/trailing pads: its DPP
// source may be fresh, and v_readlane / permlane read its result next); (2) the other three a[q] and the four x[q] (their
// sources were last written a pivot earlier, >= 4 VALU instructions back; block (1) of the next pivot pads again).
// asm volatile keeps the blocks in order.
#define GPX_FMAC_PIPE(J)                                                                                         \
  case J:                                                                                                        \
    asm volatile("s_nop 1\n\t"                                                                                   \
                 "v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                  \
                 "s_nop 1"                                                                                       \
                 : "+v"(an)                                                                                      \
                 : "v"(ca));                                                                                     \
    break;
#define GPX_FMAC_REST(J)                                                                                         \
  case J:                                                                                                        \
    asm volatile("v_fmac_f64_dpp %0, %0, %7 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %1, %1, %7 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %2, %2, %7 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %3, %3, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %4, %4, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %5, %5, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"                 \
                 "v_fmac_f64_dpp %6, %6, %8 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"                       \
                 : "+v"(a1), "+v"(a2), "+v"(a3), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3])                  \
                 : "v"(ca), "v"(cx));                                                                            \
    break;
template <int J>
__device__ __forceinline__ void fmac_pipe_first(double& an, double ca) {
  switch (J) {
    GPX_FMAC_PIPE(0) GPX_FMAC_PIPE(1) GPX_FMAC_PIPE(2) GPX_FMAC_PIPE(3) GPX_FMAC_PIPE(4) GPX_FMAC_PIPE(5)
    GPX_FMAC_PIPE(6) GPX_FMAC_PIPE(7) GPX_FMAC_PIPE(8) GPX_FMAC_PIPE(9) GPX_FMAC_PIPE(10) GPX_FMAC_PIPE(11)
    GPX_FMAC_PIPE(12) GPX_FMAC_PIPE(13) GPX_FMAC_PIPE(14) GPX_FMAC_PIPE(15)
  }
}
template <int J>
__device__ __forceinline__ void fmac_pipe_rest(double& a1, double& a2, double& a3, double (&x)[4], double ca, double cx) {
  switch (J) {
    GPX_FMAC_REST(0) GPX_FMAC_REST(1) GPX_FMAC_REST(2) GPX_FMAC_REST(3) GPX_FMAC_REST(4) GPX_FMAC_REST(5)
    GPX_FMAC_REST(6) GPX_FMAC_REST(7) GPX_FMAC_REST(8) GPX_FMAC_REST(9) GPX_FMAC_REST(10) GPX_FMAC_REST(11)
    GPX_FMAC_REST(12) GPX_FMAC_REST(13) GPX_FMAC_REST(14) GPX_FMAC_REST(15)
  }
}
#undef GPX_FMAC_PIPE
#undef GPX_FMAC_REST

// chol16_pivot_fused, software-pipelined across pivots: the column register A[.][4g + (J+1)%4] that the NEXT pivot reads
// (its pivot by v_readlane, its A[r][J+1] by permlane swaps) is updated first, the next pivot's reads are issued, and
// only then the other seven row-broadcast FMAs of pivot J, so their issue overlaps the readlane -> rsq latency of pivot
// J+1.  Same operations on the same values as chol16_pivot_fused (bit-identical L and X).
template <int J>
__device__ __forceinline__ void chol16_pivot_pipe(Blk16& b, int r, int g, int& fail, double& piv, double& arj) {
  if (!(piv > 0.0) && fail < 0) fail = J;
  const double isq = pivot_rsq(piv);
  const double rinv = isq * isq;
  const double coef = (r > J) ? -arj * rinv : 0.0;
  const double coefx = (r == J) ? isq - 1.0 : coef;
  if constexpr (J < 15) {
    constexpr int JN = J + 1, GN = JN >> 2, QN = JN & 3;
    fmac_pipe_first<J>(b.a[QN], coef);
    piv = readlane_f64(b.a[QN], JN + 16 * GN);
    arj = xrow_bcast_f64<GN>(b.a[QN]);
    fmac_pipe_rest<J>(b.a[(QN + 1) & 3], b.a[(QN + 2) & 3], b.a[(QN + 3) & 3], b.x, coef, coefx);
  } else {
    fmac_row_bcast8<J>(b.a, b.x, coef, coefx);
  }
}

template <int... J>
__device__ __forceinline__ void chol16_pivots(Blk16& b, int r, int g, int& fail, std::integer_sequence<int, J...>) {
  // software-pipelined across pivots: 3632 vs 3937 cycles per 16-pivot block unpipelined (round 2, tools/chol16_probe;
  // potrf n = 4096 1.756 vs 1.767 ms); the row broadcasts folded into the FMAs: 306 vs 390 cycles per pivot
  double piv = readlane_f64(b.a[0], 0), arj = xrow_bcast_f64<0>(b.a[0]);
  (chol16_pivot_pipe<J>(b, r, g, fail, piv, arj), ...);
}

// Factor + invert a 16x16 SPD block held in registers (lane = r + 16 g: b.a[q] = A[r][4g + q]): the unscaled upper
// factor U into b.a (rows; below the diagonal: eliminated residue), L^{-1} into b.x.  Returns the 0-based failing pivot
// inside the block, or -1 (uniform).
__device__ __forceinline__ int chol16_regs(Blk16& b) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) b.x[q] = (r == 4 * g + q) ? 1.0 : 0.0;
  int fail = -1;
  chol16_pivots(b, r, g, fail, std::make_integer_sequence<int, 16>{});
  return fail;
}

// U (unscaled upper factor, rows; only its upper triangle is meaningful) into the LDS tile sA at (o, o), D = L^{-1}
// (lower, strict upper 0) into the 16x16 tile sD of row length LDD.
template <int LDD>
__device__ __forceinline__ void chol16_store(const Blk16& b, double* sA, double* sD, int o) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * g + q;
    sA[(o + r) * LD64 + o + c] = b.a[q];
    sD[r * LDD + c] = (c <= r) ? b.x[q] : 0.0;
  }
}

// L_cc[r][c] (c <= r) of a factored 64x64 diagonal tile whose 16x16 diagonal blocks hold U (chol16_store) and whose
// blocks below them hold L (the T step): the diagonal blocks give L[r][c] = U[c][r] * isq[c], with isq[c] = pivot_rsq of
// the pivot (recomputed from the same pivot, so the same isq bits as the chain's).  The stored L_cc is NOT bit-equal to a
// capture of the column operations: U's rows come from the unscaled rank-1 updates (round(a_r * rinv) * a_c is not
// bitwise symmetric with round(a_c * rinv) * a_r), while D = b.x, the T step's L_ic = A_ic D^T and the folded z use the
// column operations — the two differ at rounding level (the Dinv that potrs later forms from L_cc differs from the
// panel's D in the last bits).  Harmless for the results (tests/test_gpu_parity.py checks the factor's backward error
// ||L L^T - K|| / ||K|| at n = 4096 and 16384), and schedule-invariant: every schedule stores L_cc the same way.
// isq: 64 doubles of scratch filled by l64_isq.
__device__ __forceinline__ void l64_isq(const double* sA, double* isq) {
  const int t = threadIdx.x;
  if (t < 64) isq[t] = pivot_rsq(sA[t * LD64 + t]);
}
__device__ __forceinline__ double l64_at(const double* sA, const double* isq, int r, int c) {
  if (c > r) return 0.0;
  if ((c >> 4) == (r >> 4)) return sA[c * LD64 + r] * isq[c];
  return sA[r * LD64 + c];
}

// Factor + invert the 16x16 SPD block at (o, o) of the LDS tile sA (both triangles present, symmetric) with one
// wave: U back into sA, D = L^{-1} into sD (chol16_store).  Returns the failing pivot inside the block, or -1.
template <int LDD>
__device__ __forceinline__ int chol16(double* sA, double* sD, int o) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  Blk16 b;
#pragma unroll
  for (int q = 0; q < 4; ++q) b.a[q] = sA[(o + r) * LD64 + o + 4 * g + q];
  const int fail = chol16_regs(b);
  chol16_store<LDD>(b, sA, sD, o);
  return fail;
}

// X = L^{-1} of the lower-triangular 16x16 block at (o, o) of sL (already factored), by one wave: forward
// elimination on I with the rows of X broadcast by DPP and the multipliers read from LDS.  Written to sX at (o, o).
template <int J>
__device__ __forceinline__ void trinv16_step(double (&x)[4], const double (&lr)[16], double djinv, int r) {
  double xj[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) xj[q] = row_newbcast<J>(x[q]) * djinv;
  const double c = (r > J) ? lr[J] : 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) x[q] = (r == J) ? xj[q] : fma(-c, xj[q], x[q]);
}

template <int... J>
__device__ __forceinline__ void trinv16_steps(double (&x)[4], const double (&lr)[16], const double (&dinv)[16], int r,
                                              std::integer_sequence<int, J...>) {
  (trinv16_step<J>(x, lr, dinv[J], r), ...);
}

__device__ __forceinline__ void trinv16_dpp(const double* sL, double* sX, int o) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  double lr[16], dinv[16], x[4];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    lr[j] = sL[(o + r) * LD64 + o + j];
    dinv[j] = 1.0 / sL[(o + j) * LD64 + o + j];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) x[q] = (r == 4 * g + q) ? 1.0 : 0.0;
  trinv16_steps(x, lr, dinv, r, std::make_integer_sequence<int, 16>{});
#pragma unroll
  for (int q = 0; q < 4; ++q) sX[(o + r) * LD64 + o + 4 * g + q] = x[q];
}

// One 16x16 MFMA block product accumulated over K: acc += sign * sum_t A(ra0 + m, ka0 + t) B(kb0 + t, cb0 + n)
// with both operands in LDS tiles (row length LD64 for A, LDB for B); A is read row-major (A[row][k]) and B either row-major
// (B[k][col], BT=false) or as B[col][k] (BT=true, a multiply by a transpose).
template <bool BT, int LDB = LD64>
__device__ __forceinline__ d4 mfma_lds16(d4 acc, const double* A, int ra0, int ka0, const double* B, int kb0, int cb0,
                                         int K, double sign) {
  const int lane = threadIdx.x & 63;
  const int m = lane & 15, kk = lane >> 4;
#pragma unroll 4
  for (int k = 0; k < K; k += 4) {
    const double a = sign * A[(ra0 + m) * LD64 + ka0 + k + kk];
    const double b = BT ? B[(cb0 + m) * LDB + kb0 + k + kk] : B[(kb0 + k + kk) * LDB + cb0 + m];
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

// Inverse of a 64x64 lower-triangular L held in sL (strict upper arbitrary) into sX (lower, strict upper zero),
// 256 threads: each wave inverts one 16x16 diagonal block (trinv16_dpp), then X_ij = -X_ii sum_{k=j}^{i-1} L_ik X_kj
// by sub-diagonal on MFMA (sT: 64 x LD64 scratch).
__device__ inline void trinv64(const double* sL, double* sX, double* sT) {
  const int w = threadIdx.x >> 6;
  trinv16_dpp(sL, sX, 16 * w);
  __syncthreads();
  for (int dd = 1; dd < 4; ++dd) {
    const int nb = 4 - dd;
    if (w < nb) {
      const int j = w, i = w + dd;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int k = j; k < i; ++k) acc = mfma_lds16<false>(acc, sL, 16 * i, 16 * k, sX, 16 * k, 16 * j, 16, 1.0);
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
  for (int e = threadIdx.x; e < 64 * 64; e += WG) {
    const int rr = e >> 6, cc = e & 63;
    if ((cc >> 4) > (rr >> 4)) sX[rr * LD64 + cc] = 0.0;
  }
  __syncthreads();
}

}  // namespace gpx
