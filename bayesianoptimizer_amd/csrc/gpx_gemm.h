// Generic 64x64-tile fp64-MFMA GEMM with triangular k-ranges and deterministic split-K, shared by the incremental
// update (gpx_append.hip) and the split triangular inverse of the fit (gpx_potrf.hip).
#pragma once
#include "gpx_internal.h"
#include "gpx_device.h"

namespace gpx {

// k-range of a 64x64 output tile (rb, cb) of C = A B when one operand is upper triangular.
enum { KR_FULL = 0, KR_B_UPPER = 1, KR_A_UPPER = 2, KR_A_LOWER = 3 };

// Cout(rb, cb) = [Cin(rb, cb)] + sign * sum_k A(m, k) B(k, n) on fp64 MFMA (one 64x64 tile per workgroup).
//   A_KM: A(m, k) at A[k * lda + m] (else A[m * lda + k]);  B_KM: B(k, n) at B[k * ldb + n] (else B[n * ldb + k]).
//   lower: only tiles cb <= rb are computed.  Cin may be NULL (C = sign * A B).
// Split-K (gridDim.z > 1): the bordered update's GEMMs are thin (q' = 128 rows against K = n0 = 4096), so one
// workgroup per tile would run a 4096-long k loop on a handful of CUs; chunk z of `kchunk` k-steps instead writes
// its raw partial tile to P + z * pstride (row length ldp) and gemm_reduce_kernel sums the chunks in a fixed order.
template <bool A_KM, bool B_KM, int KR>
__global__ void __launch_bounds__(WG) gemm64_kernel(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                                    int64_t ldb, const double* __restrict__ Cin, int64_t ldcin,
                                                    double* __restrict__ Cout, int64_t ldc, int K, double sign,
                                                    int lower, int kchunk, double* __restrict__ P, int64_t ldp,
                                                    int64_t pstride) {
  using Tile = MfmaTile<NB, NB, 16, A_KM, B_KM>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  const int rb = blockIdx.y, cb = blockIdx.x;
  if (lower && cb > rb) return;
  int kbeg = 0, kend = K;
  if (KR == KR_B_UPPER) kend = min(K, (cb + 1) * NB);
  if (KR == KR_A_UPPER) kbeg = rb * NB;
  if (KR == KR_A_LOWER) kend = min(K, (rb + 1) * NB);
  const bool split = gridDim.z > 1;
  if (split) {
    const int k0 = (int)blockIdx.z * kchunk;
    kbeg = max(kbeg, k0);
    kend = min(kend, k0 + kchunk);
  }
  const double* At = A_KM ? A + rb * NB : A + (int64_t)rb * NB * lda;
  const double* Bt = B_KM ? B + cb * NB : B + (int64_t)cb * NB * ldb;
  Tile tile;
  tile.run(At, lda, Bt, ldb, kbeg, kend, smem);  // empty range: zero partial
  if (split) {
    double* Po = P + blockIdx.z * pstride + (int64_t)rb * NB * ldp + cb * NB;
#pragma unroll
    for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
      for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) Po[(int64_t)Tile::row_of(i, r) * ldp + Tile::col_of(j)] = tile.acc[i][j][r];
    return;
  }
  double* Co = Cout + (int64_t)rb * NB * ldc + cb * NB;
  const double* Ci = Cin ? Cin + (int64_t)rb * NB * ldcin + cb * NB : nullptr;
#pragma unroll
  for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
    for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = Tile::row_of(i, r), col = Tile::col_of(j);
        const double base = Ci ? Ci[(int64_t)row * ldcin + col] : 0.0;
        Co[(int64_t)row * ldc + col] = base + sign * tile.acc[i][j][r];
      }
}

// Cout = [Cin] + sign * sum_{z < nz} P_z over a rows x cols matrix (two consecutive doubles per thread); with `lower`
// only 64-tiles on or below the diagonal.
static __global__ void __launch_bounds__(WG) gemm_reduce_kernel(const double* __restrict__ P, int64_t ldp, int64_t pstride,
                                                         int nz, const double* __restrict__ Cin, int64_t ldcin,
                                                         double* __restrict__ Cout, int64_t ldc, int rows, int cols,
                                                         double sign, int lower) {
  const int64_t e = ((int64_t)blockIdx.x * WG + threadIdx.x) * 2;
  const int r = (int)(e / cols), c = (int)(e % cols);
  if (r >= rows) return;
  if (lower && (c >> 6) > (r >> 6)) return;
  double2 acc = make_double2(0.0, 0.0);
  for (int z = 0; z < nz; ++z) {
    const double2 v = *reinterpret_cast<const double2*>(P + z * pstride + (int64_t)r * ldp + c);
    acc.x += v.x;
    acc.y += v.y;
  }
  double2 out = make_double2(sign * acc.x, sign * acc.y);
  if (Cin) {
    out.x += Cin[(int64_t)r * ldcin + c];
    out.y += Cin[(int64_t)r * ldcin + c + 1];
  }
  *reinterpret_cast<double2*>(Cout + (int64_t)r * ldc + c) = out;
}

// Launch of C (rows x cols, multiples of 64) = [Cin] + sign * A B with K inner steps, split along K when the tile grid
// alone would leave the chip mostly idle.  P: split-K scratch of at least gemm_split_doubles(rows, cols, K) doubles.
constexpr int SPLIT_TARGET_WG = 1024;  // ~2 workgroups per CU on 256 CUs, twice over
inline int gemm_splits(int rows, int cols, int K) {
  const int tiles = (rows / NB) * (cols / NB);
  int s = (SPLIT_TARGET_WG + tiles - 1) / tiles;
  const int kmax = K / NB;  // at least 64 k per chunk
  s = s < 1 ? 1 : (s > kmax ? kmax : s);
  return s > 16 ? 16 : s;
}

inline size_t gemm_split_doubles(int rows, int cols, int K) {
  const int s = gemm_splits(rows, cols, K);
  return s > 1 ? (size_t)s * rows * cols : 0;
}

template <bool A_KM, bool B_KM, int KR>
inline hipError_t launch_gemm64(Context* c, int rows, int cols, int K, const double* A, int64_t lda, const double* B,
                         int64_t ldb, const double* Cin, int64_t ldcin, double* Cout, int64_t ldc, double sign,
                         int lower, double* P) {
  const int s = gemm_splits(rows, cols, K);
  if (s <= 1) {
    gemm64_kernel<A_KM, B_KM, KR><<<dim3(cols / NB, rows / NB, 1), WG, 0, c->stream>>>(
        A, lda, B, ldb, Cin, ldcin, Cout, ldc, K, sign, lower, K, nullptr, 0, 0);
    return hipGetLastError();
  }
  const int kchunk = ((K / s + NB - 1) / NB) * NB;
  const int nz = (K + kchunk - 1) / kchunk;
  const int64_t pstride = (int64_t)rows * cols;
  gemm64_kernel<A_KM, B_KM, KR><<<dim3(cols / NB, rows / NB, nz), WG, 0, c->stream>>>(
      A, lda, B, ldb, Cin, ldcin, Cout, ldc, K, sign, lower, kchunk, P, cols, pstride);
  const int64_t pairs = pstride / 2;
  gemm_reduce_kernel<<<(unsigned)((pairs + WG - 1) / WG), WG, 0, c->stream>>>(P, cols, pstride, nz, Cin, ldcin, Cout,
                                                                               ldc, rows, cols, sign, lower);
  return hipGetLastError();
}

}  // namespace gpx
