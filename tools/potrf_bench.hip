// Microbenchmark + self-check of the blocked Cholesky kernels (diagnostic; includes the shipped gpx_potrf.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        potrf_bench.hip -o potrf_bench_probe
// Prints: the permlane/DPP broadcast semantics the in-wave pivot relies on, per-kernel times (panel with 1 and 64
// workgroups, syrk at step 0, diagonal inverses, full potrf) and max |L L^T - A| / max |D L_kk - I| on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>
#include "gpx_internal.h"
__device__ unsigned long long g_stamp[4][16];
__device__ unsigned g_hwid[4];
// wave-0 lane-0 timestamps of the panel phases, per wave w (lane 0): g_stamp[w][i]
#define GPX_PANEL_STAMP(i) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 1 && c == 1) { g_stamp[threadIdx.x >> 6][i] = __builtin_readcyclecounter(); if (i == 0) g_hwid[threadIdx.x >> 6] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)); } } while (0)
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"

using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void bcast_probe(double* out) {
  const int l = threadIdx.x;
  const double v = 100.0 * (l >> 4) + (l & 15);
  out[l] = row_newbcast<5>(v);
}

__global__ void f16_test(const double* A, double* L, double* X, int* fail) {
  __shared__ double sA[16 * LD64], sD[16 * LD64];

  for (int e = threadIdx.x; e < 256; e += 64) sA[(e >> 4) * LD64 + (e & 15)] = A[e];
  __syncthreads();
  const int f = chol16<LD64>(sA, sD, 0);
  __syncthreads();
  for (int e = threadIdx.x; e < 256; e += 64) { L[e] = sA[(e >> 4) * LD64 + (e & 15)]; X[e] = sD[(e >> 4) * LD64 + (e & 15)]; }
  if (threadIdx.x == 0) *fail = f;
}

int main(int argc, char** argv) {
  {
    std::vector<double> a(256), l(256), x(256);
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) a[i * 16 + j] = exp(-0.05 * (i - j) * (i - j)) + (i == j ? 0.1 : 0.0);
    double *dA, *dL, *dX; int* df;
    CK(hipMalloc(&dA, 2048)); CK(hipMalloc(&dL, 2048)); CK(hipMalloc(&dX, 2048)); CK(hipMalloc(&df, 4));
    CK(hipMemcpy(dA, a.data(), 2048, hipMemcpyHostToDevice));
    f16_test<<<1, 64>>>(dA, dL, dX, df);
    int f; CK(hipMemcpy(l.data(), dL, 2048, hipMemcpyDeviceToHost)); CK(hipMemcpy(x.data(), dX, 2048, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&f, df, 4, hipMemcpyDeviceToHost));
    std::vector<double> ref(256, 0.0);
    for (int j = 0; j < 16; ++j) {
      double s = a[j * 16 + j]; for (int k = 0; k < j; ++k) s -= ref[j * 16 + k] * ref[j * 16 + k];
      ref[j * 16 + j] = sqrt(s);
      for (int i = j + 1; i < 16; ++i) { double t = a[i * 16 + j]; for (int k = 0; k < j; ++k) t -= ref[i * 16 + k] * ref[j * 16 + k]; ref[i * 16 + j] = t / ref[j * 16 + j]; }
    }
    double el = 0, ex = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      el = std::max(el, fabs(l[i * 16 + j] - ref[i * 16 + j]));
      double s = 0; for (int k = 0; k < 16; ++k) s += x[i * 16 + k] * ref[k * 16 + j];
      ex = std::max(ex, fabs(s - (i == j)));
    }
    printf("chol16: fail=%d max|L-Lref|=%.3e max|X L - I|=%.3e\n", f, el, ex);
    if (el > 1e-12) { for (int i = 0; i < 4; ++i) { for (int j = 0; j < 6; ++j) printf(" %9.5f/%9.5f", l[i*16+j], ref[i*16+j]); printf("\n"); } }
  }
  const int n = argc > 1 ? atoi(argv[1]) : 4096, nblk = n / 64;
  {
    double* d; CK(hipMalloc(&d, 192 * 8));
    bcast_probe<<<1, 64>>>(d);
    std::vector<double> h(192); CK(hipMemcpy(h.data(), d, 192 * 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
      bad += h[l] != 100.0 * (l >> 4) + 5;
    }
    printf("broadcast probe: %s (newbcast:5 lane 33: %.0f)\n", bad ? "MISMATCH" : "ok", h[33]);
    CK(hipFree(d));
  }
  // SPD test matrix: RBF Gram of seeded points in [0,1]^8 (lengthscale 0.579) + 1e-4 I, like the bench problem
  std::vector<double> h((size_t)n * n), X((size_t)n * 8);
  srand(7);
  for (auto& v : X) v = rand() / (double)RAND_MAX;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double r2 = 0.0;
      for (int k = 0; k < 8; ++k) { const double d = (X[i * 8 + k] - X[j * 8 + k]) / 0.579; r2 += d * d; }
      h[(size_t)i * n + j] = exp(-0.5 * r2) + (i == j ? 1e-4 : 0.0);
    }
  double *A, *A0, *Dinv; int* info;
  CK(hipMalloc(&A, (size_t)n * n * 8)); CK(hipMalloc(&A0, (size_t)n * n * 8));
  CK(hipMalloc(&Dinv, (size_t)2 * nblk * 64 * 64 * 8)); CK(hipMalloc(&info, 4));
  CK(hipMemcpy(A0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto fn, int reps) {
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
      CK(hipMemset(info, 0, 4));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); fn(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end()); return t[t.size() / 2];
  };
  Context c; c.stream = 0;
  const float tp = timeit([&] { (void)launch_potrf(&c, n, A, n, Dinv, info); }, 7);
  int hinfo; CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
  std::vector<double> L((size_t)n * n), D((size_t)nblk * 4096);
  CK(hipMemcpy(L.data(), A, L.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(D.data(), Dinv, D.size() * 8, hipMemcpyDeviceToHost));
  // residual on sampled rows
  double res = 0.0;
  for (int i = 0; i < n; i += 37) {
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      for (int k = 0; k <= j; ++k) s += L[(size_t)i * n + k] * L[(size_t)j * n + k];
      res = std::max(res, fabs(s - h[(size_t)i * n + j]));
    }
  }
  double dres = 0.0;
  for (int b = 0; b < nblk; b += 7) {
    for (int r = 0; r < 64; ++r) for (int cc = 0; cc < 64; ++cc) {
      double s = 0.0;
      for (int k = 0; k < 64; ++k) s += D[(size_t)b * 4096 + r * 64 + k] * L[(size_t)(64 * b + k) * n + 64 * b + cc];
      dres = std::max(dres, fabs(s - (r == cc ? 1.0 : 0.0)));
    }
  }
  printf("n=%d full potrf: %.3f ms  info=%d  max|LL^T-A| (sampled rows)=%.3e  max|D L_kk - I|=%.3e\n", n, tp, hinfo, res, dres);
  // per-launch times of step c (after running steps 0..c-1 once): full grid, panel workgroups only
  auto time_step = [&](int c, int mode) {  // 0 full grid, 1 panel workgroups only, 2 trailing workgroups only
    CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice)); CK(hipMemset(info, 0, 4));
    for (int cc = 0; cc < c; ++cc) potrf_step_kernel<<<potrf_step_grid(cc, nblk, 1, 0), WG>>>(A, n, cc, nblk, 1, 0, Dinv, info, 0, 0, 0);
    CK(hipDeviceSynchronize());
    const int full = potrf_step_grid(c, nblk, 1, 0);
    const int grid = mode == 0 ? full : mode == 1 ? nblk - c : full - (nblk - c);
    const int first = mode == 2 ? nblk - c : 0;
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) potrf_step_kernel<<<grid, WG>>>(A, n, c, nblk, 1, 0, Dinv, info, first, 0, 0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    int hi; CK(hipMemcpy(&hi, info, 4, hipMemcpyDeviceToHost));
    return hi ? -1.0f : ms * 50.0f;
  };
  const float td = timeit([&] { for (int i = 0; i < 20; ++i) potrf_dinv_kernel<<<nblk, WG>>>(A, n, nblk, Dinv, info, 0, 0, 0); }, 5);
  for (int c : {1, 8, 16, 32, 48, nblk - 3})
    printf("step %2d: %6.2f us   panel wgs only %6.2f us   trailing wgs only %6.2f us (%d tiles)\n", c, time_step(c, 0),
           time_step(c, 1), time_step(c, 2), potrf_step_grid(c, nblk, 1, 0) - (nblk - c));
  printf("dinv: %.2f us\n", td * 50);
  CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice)); CK(hipMemset(info, 0, 4));
  potrf_step_kernel<<<potrf_step_grid(0, nblk, 1, 0), WG>>>(A, n, 0, nblk, 1, 0, Dinv, info, 0, 0, 0); CK(hipDeviceSynchronize());
  potrf_step_kernel<<<potrf_step_grid(1, nblk, 1, 0), WG>>>(A, n, 1, nblk, 1, 0, Dinv, info, 0, 0, 0); CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 3; ++rep) {
    if (rep > 0) {  // the same step again (warm instruction cache on the CUs that ran it)
      potrf_step_kernel<<<potrf_step_grid(1, nblk, 1, 0), WG>>>(A, n, 1, nblk, 1, 0, Dinv, info, 0, 0, 0);
      CK(hipDeviceSynchronize());
    }
    unsigned long long hs[4][16]; CK(hipMemcpyFromSymbol(hs, HIP_SYMBOL(g_stamp), sizeof(hs)));
    unsigned hw[4]; CK(hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_hwid), sizeof(hw)));
    printf("rep %d: wave 0 on cu %u\n", rep, (hw[0] >> 8) & 15);
    for (int w = 0; w < 1; ++w) {
      printf("wave %d stamps (cycles after load):", w);
      for (int i = 1; i <= 13; ++i) printf(" %lld", (long long)(hs[w][i] - hs[0][0]));
      printf("\n");
    }
  }
  printf("POTRF BENCH DONE\n");
  return 0;
}
