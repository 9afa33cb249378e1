/* Plain-C use of the drop-in boundary (include/gpx.h) with no Python or torch: device buffers from hipMalloc, one
 * posterior update (gpx_fit_f64_sync) and a 4096-candidate LogEI sweep (gpx_acquire_argmax_f64), checked against a
 * small host Cholesky.  Built by __graft_entry__.build() with gcc (tools/capi_example), run by
 * tests/test_gpu_parity.py::test_c_abi_example_program.  Prints "capi example ok" on success, exit 1 otherwise. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gpx.h"

/* minimal HIP runtime surface (libamdhip64), declared here so the example needs no HIP headers */
typedef int hipError_t;
extern hipError_t hipMalloc(void** p, size_t n);
extern hipError_t hipFree(void* p);
extern hipError_t hipMemcpy(void* dst, const void* src, size_t n, int kind);
extern hipError_t hipMemset(void* p, int v, size_t n);
extern hipError_t hipDeviceSynchronize(void);
enum { H2D = 1, D2H = 2 };

#define CHECK(x)                                                                         \
  do {                                                                                   \
    gpx_status s_ = (x);                                                                 \
    if (s_ != GPX_OK) {                                                                  \
      fprintf(stderr, "%s failed: %d %s\n", #x, s_, h ? gpx_last_error(h) : "");         \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

static double rbf(const double* a, const double* b, int d, double ls) {
  double r2 = 0.0;
  for (int k = 0; k < d; ++k) {
    const double t = a[k] / ls - b[k] / ls;
    r2 += t * t;
  }
  return exp(-0.5 * r2);
}

int main(void) {
  gpx_handle h = NULL;
  const int n = 200, d = 4, m = 4096;
  const double ls = 0.6, noise = 1e-4;
  double* X = malloc(sizeof(double) * n * d);
  double* y = malloc(sizeof(double) * n);
  double* Xs = malloc(sizeof(double) * m * d);
  unsigned s = 12345u;
  for (int i = 0; i < n * d; ++i) {
    s = s * 1664525u + 1013904223u;
    X[i] = (s >> 8) / 16777216.0;
  }
  for (int i = 0; i < n; ++i) y[i] = sin(6.0 * X[i * d]) + cos(4.0 * X[i * d + 1]);
  for (int i = 0; i < m * d; ++i) {
    s = s * 1664525u + 1013904223u;
    Xs[i] = (s >> 8) / 16777216.0;
  }
  CHECK(gpx_create(0, &h));
  const int64_t npad = gpx_padded_n(n);
  size_t ws_fit = 0, ws_sweep = 0;
  CHECK(gpx_fit_workspace_size(n, 1, &ws_fit));
  CHECK(gpx_sweep_workspace_size(n, 1, m, &ws_sweep));
  double *dX, *dy, *dXs, *dK, *dW, *dDinv, *dalpha, *dbv;
  int64_t* dbi;
  int32_t* dinfo;
  void* dws;
  const size_t ws = ws_fit > ws_sweep ? ws_fit : ws_sweep;
  if (hipMalloc((void**)&dX, sizeof(double) * n * d) || hipMalloc((void**)&dy, sizeof(double) * n) ||
      hipMalloc((void**)&dXs, sizeof(double) * m * d) || hipMalloc((void**)&dK, sizeof(double) * npad * npad) ||
      hipMalloc((void**)&dW, sizeof(double) * npad * npad) ||
      hipMalloc((void**)&dDinv, sizeof(double) * 2 * (npad / 64) * 4096) ||
      hipMalloc((void**)&dalpha, sizeof(double) * npad) || hipMalloc((void**)&dbv, 8) || hipMalloc((void**)&dbi, 8) ||
      hipMalloc((void**)&dinfo, 4) || hipMalloc(&dws, ws)) {
    fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  hipMemcpy(dX, X, sizeof(double) * n * d, H2D);
  hipMemcpy(dy, y, sizeof(double) * n, H2D);
  hipMemcpy(dXs, Xs, sizeof(double) * m * d, H2D);
  gpx_kernel_params p;
  memset(&p, 0, sizeof(p));
  p.kind = GPX_KERNEL_RBF;
  p.d = d;
  for (int k = 0; k < d; ++k) p.lengthscale[k] = ls;
  p.outputscale = 1.0;
  p.noise = noise;
  int32_t info = 0;
  CHECK(gpx_fit_f64_sync(h, &p, n, dX, d, dy, 1, 1, dK, npad, dDinv, dW, npad, dalpha, dinfo, dws, ws, &info));
  double ymax = y[0];
  for (int i = 1; i < n; ++i) ymax = y[i] > ymax ? y[i] : ymax;
  gpx_acq_params a;
  memset(&a, 0, sizeof(a));
  a.kind = GPX_ACQ_LOGEI;
  a.best_f = ymax;
  a.y_scale = 1.0;
  CHECK(gpx_acquire_argmax_f64(h, &p, n, dX, d, dW, npad, dalpha, dXs, m, d, &a, 0, dbv, dbi, NULL, dws, ws));
  double bv = 0.0, alpha0 = 0.0;
  int64_t bi = -1;
  hipDeviceSynchronize();
  hipMemcpy(&bv, dbv, 8, D2H);
  hipMemcpy(&bi, dbi, 8, D2H);
  hipMemcpy(&alpha0, dalpha, 8, D2H);
  /* host check: alpha = K^{-1} y by a dense Cholesky, compared on its first entry; the argmax index is in range */
  double* K = malloc(sizeof(double) * n * n);
  double* z = malloc(sizeof(double) * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) K[i * n + j] = rbf(X + i * d, X + j * d, d, ls) + (i == j ? noise : 0.0);
  for (int j = 0; j < n; ++j) {
    for (int k = 0; k < j; ++k) K[j * n + j] -= K[j * n + k] * K[j * n + k];
    K[j * n + j] = sqrt(K[j * n + j]);
    for (int i = j + 1; i < n; ++i) {
      for (int k = 0; k < j; ++k) K[i * n + j] -= K[i * n + k] * K[j * n + k];
      K[i * n + j] /= K[j * n + j];
    }
  }
  for (int i = 0; i < n; ++i) {
    double t = y[i];
    for (int k = 0; k < i; ++k) t -= K[i * n + k] * z[k];
    z[i] = t / K[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = z[i];
    for (int k = i + 1; k < n; ++k) t -= K[k * n + i] * z[k];
    z[i] = t / K[i * n + i];
  }
  double amax = 0.0;
  for (int i = 0; i < n; ++i) amax = fabs(z[i]) > amax ? fabs(z[i]) : amax;
  const double err = fabs(alpha0 - z[0]) / amax;
  printf("alpha[0] gpu %.15e host %.15e (rel %.2e); best logEI %.6f at %lld\n", alpha0, z[0], err, bv, (long long)bi);
  if (!(err < 1e-6) || bi < 0 || bi >= m || !isfinite(bv)) return 1;
  CHECK(gpx_destroy(h));
  printf("capi example ok\n");
  return 0;
}
