// Incremental posterior update: q new training points appended to a factored GP.
//
// The reference refits the exact GP from scratch every round after appending the new rows
// (optimization/Bayesian7.py:628-631,692-700 append, :639 refit; optimization/Bayesian.py:163-174), an
// O(n^3) update.  With the hyperparameters unchanged the leading block of the factor does not change, so the
// update is a bordered Cholesky of the new rows, O(n^2 q):
//     K = [K11 K21^T; K21 K22],  L11 = chol(K11) and W11 = L11^{-T} kept,
//     L21 = K21 W11                       (q' x n0, triangular GEMM, fp64 MFMA)
//     S   = K22 - L21 L21^T               (q' x q', lower tiles, fp64 MFMA)
//     L22 = chol(S), W22 = L22^{-T}       (the blocked potrf / trtri of gpx_potrf.hip / gpx_trtri.hip on the block)
//     W12 = -W11 (L21^T W22)              (the trtri doubling step with b1 = n0, b2 = q')
// and alpha is recomputed from the new W (two HBM GEMVs).  n0 = floor(n_old / 128) * 128: the old rows past the last
// full 128-tile (and the old identity padding) are refactored with the new ones, so every block keeps the 128-row
// alignment of a fresh fit and the result is the same factor a fresh fit of all n_new rows computes.
#include "gpx_internal.h"
#include "gpx_device.h"

namespace gpx {

// k-range of a 64x64 output tile (rb, cb) of C = A B when one operand is upper triangular.
enum { KR_FULL = 0, KR_B_UPPER = 1, KR_A_UPPER = 2 };

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
__global__ void __launch_bounds__(WG) gemm_reduce_kernel(const double* __restrict__ P, int64_t ldp, int64_t pstride,
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
hipError_t launch_gemm64(Context* c, int rows, int cols, int K, const double* A, int64_t lda, const double* B,
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

// A pivot failure inside the appended block is reported relative to it; make it global.
__global__ void info_offset_kernel(int32_t* info, int n0) {
  if (threadIdx.x == 0 && *info != 0) *info += n0;
}

// G (q x npad), T (n0 x q) and the trtri scratch of the q-block share the first region of the workspace.
inline size_t append_region_doubles(int64_t n0, int64_t q) {
  size_t a = (size_t)q * (n0 + q), b = (size_t)n0 * q, t = (size_t)q * q / 4 + 32;
  size_t m = a > b ? a : b;
  m = m > t ? m : t;
  return (m + 31) & ~(size_t)31;
}

hipError_t launch_append(Context* c, const gpx_kernel_params& p, int n_old, int n_new, const double* X, int64_t ldx,
                         double* L, int64_t ldl, double* Dinv, double* W, int64_t ldw, int32_t* info, double* ws) {
  const int npad = ((n_new + TILE - 1) / TILE) * TILE;
  const int n0 = (n_old / TILE) * TILE;
  const int q = npad - n0;               // rows refactored (multiple of 128)
  const int nb0 = n0 / NB;
  double* G = ws;                         // q x npad: Gram rows [n0, npad) (K21 | K22), row length npad
  double* P = ws + append_region_doubles(n0, q);  // split-K partials
  double* L21 = L + (int64_t)n0 * ldl;
  double* L22 = L21 + n0;
  // 1. Gram of the new rows: row gi of K lands in G row gi - n0 (n0 = 0: a full refit, straight into L).
  hipError_t e = n0 > 0 ? launch_gram(c, p, n_new, npad, X, ldx, G - (int64_t)n0 * npad, npad, Batch(), nb0)
                        : launch_gram(c, p, n_new, npad, X, ldx, L, ldl);
  if (e != hipSuccess) return e;
  if (n0 > 0) {
    // 2. L21 = K21 W11 (W11 upper: k <= column)
    e = launch_gemm64<false, true, KR_B_UPPER>(c, q, n0, n0, G, npad, W, ldw, nullptr, 0, L21, ldl, 1.0, 0, P);
    if (e != hipSuccess) return e;
    // 3. S = K22 - L21 L21^T into the lower tiles (diagonal tiles full) of L22
    e = launch_gemm64<false, false, KR_FULL>(c, q, q, n0, L21, ldl, L21, ldl, G + n0, npad, L22, ldl, -1.0, 1, P);
    if (e != hipSuccess) return e;
  }
  // 4. L22 = chol(S), W22 = L22^{-T}: the blocked kernels on the q x q block (its D_k land at Dinv block nb0 + k)
  double* Dq = Dinv + (int64_t)nb0 * NB * NB;
  e = launch_potrf(c, q, L22, ldl, Dq, info);
  if (e != hipSuccess) return e;
  if (n0 > 0) info_offset_kernel<<<1, 64, 0, c->stream>>>(info, n0);
  double* W22 = W + (int64_t)n0 * ldw + n0;
  e = launch_trtri(c, q, L22, ldl, Dq, W22, ldw, ws);
  if (e != hipSuccess) return e;
  if (n0 > 0) {
    // 5. T = L21^T W22 (n0 x q, W22 upper: k <= column), then 6. W12 = -W11 T (W11 upper: k >= row)
    double* T = ws;  // n0 x q (G is dead by now)
    e = launch_gemm64<true, true, KR_B_UPPER>(c, n0, q, q, L21, ldl, W22, ldw, nullptr, 0, T, q, 1.0, 0, P);
    if (e != hipSuccess) return e;
    e = launch_gemm64<false, true, KR_A_UPPER>(c, n0, q, n0, W, ldw, T, q, nullptr, 0, W + n0, ldw, -1.0, 0, P);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

size_t append_workspace_bytes(int64_t n_old, int64_t n_new) {
  const int64_t npad = ((n_new + TILE - 1) / TILE) * TILE;
  const int64_t n0 = (n_old / TILE) * TILE;
  const int64_t q = npad - n0;
  size_t p = 0;
  if (n0 > 0) {
    const size_t parts[4] = {gemm_split_doubles((int)q, (int)n0, (int)n0), gemm_split_doubles((int)q, (int)q, (int)n0),
                             gemm_split_doubles((int)n0, (int)q, (int)q), gemm_split_doubles((int)n0, (int)q, (int)n0)};
    for (size_t v : parts) p = v > p ? v : p;
  }
  return (append_region_doubles(n0, q) + p) * sizeof(double);
}

}  // namespace gpx
