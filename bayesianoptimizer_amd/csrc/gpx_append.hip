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
#include "gpx_gemm.h"

namespace gpx {

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
