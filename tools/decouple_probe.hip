// Upper bound of a decoupled trailing update (diagnostic, timing only; includes the shipped gpx_potrf.hip): the full
// multi-launch factorisation at n = 4096 with each launch's trailing workgroups restricted to the NEAR tile columns
// (128-tile origin q0 with q0 - c < D, column-major order), i.e. what the launches would cost if a concurrent kernel
// did the far tiles.  The factor is NOT valid for D < nblk (far tiles never updated); D = 1000 is the full update in
// column-major tile order (control).  Prints the sum of launch times (hipEvents around the sequence) per D.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        decouple_probe.hip -o decouple_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "gpx_internal.h"
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// launch c: panels exactly as the library's step kernel; trailing workgroups b - tbase -> near tile (column-major)
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
near_step_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s, double* __restrict__ Dinv,
                 int32_t* __restrict__ info, int D) {
  __shared__ __attribute__((aligned(16))) double lds[STEP_LDS];
  const int b = (int)blockIdx.x;
  if (b < s.npanel) {
    if (s.split == 2 && b > 0)
      panel_role<0, 2>(A, lda, c, 1 + ((b - 1) >> 1), (b - 1) & 1, nblk, s.c0, Dinv, info, lds, PotrfFwd());
    else
      panel_role<0, 1>(A, lda, c, b, 0, nblk, s.c0, Dinv, info, lds, PotrfFwd());
    return;
  }
  if (b < s.tbase) return;
  const int M = (nblk - s.cfirst + 1) / 2, c0 = nblk - 2 * M;
  int p = b - s.tbase;
  for (int J = 0; J < M; ++J) {
    if (c0 + 2 * J - c >= D) return;
    if (p < M - J) {
      trailing_tile_at(A, lda, c, s.k0, s.cfirst, c0 + 2 * (J + p), c0 + 2 * J, lds);
      return;
    }
    p -= M - J;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, nblk = n / 64;
  std::vector<double> h((size_t)n * n), X((size_t)n * 8);
  srand(7);
  for (auto& v : X) v = rand() / (double)RAND_MAX;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double r2 = 0.0;
      for (int k = 0; k < 8; ++k) { const double d = (X[i * 8 + k] - X[j * 8 + k]) / 0.579; r2 += d * d; }
      h[(size_t)i * n + j] = exp(-0.5 * r2) + (i == j ? 1e-4 : 0.0);
    }
  double *A, *A0, *Dinv;
  int* info;
  CK(hipMalloc(&A, (size_t)n * n * 8));
  CK(hipMalloc(&A0, (size_t)n * n * 8));
  CK(hipMalloc(&Dinv, (size_t)2 * nblk * 64 * 64 * 8));
  CK(hipMalloc(&info, 4));
  CK(hipMemcpy(A0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int D, bool lib) {
    CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemset(info, 0, 4));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int c = 0; c < nblk; ++c) {
      const StepPlan s = step_plan(c, nblk, 0, c > 0 ? c - 1 : 0, c >= 1, 1, 2 * cus);
      if (lib) {
        potrf_step_kernel<0><<<s.tbase + s.ntrail, WG>>>(A, n, c, nblk, s, Dinv, info, 0, 0, 0, PotrfFwd());
      } else {
        const int M = (nblk - s.cfirst + 1) / 2, c0 = nblk - 2 * M;
        int near = 0;
        for (int J = 0; J < M && c0 + 2 * J - c < D; ++J) near += M - J;
        near_step_kernel<<<s.tbase + near, WG>>>(A, n, c, nblk, s, Dinv, info, D);
      }
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  printf("n=%d: sum of the %d step launches (ms, median of 5)\n", n, nblk);
  for (int D : {-1, 1000, 2, 3, 4, 6, 8}) {
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) t.push_back(run(D, D < 0));
    std::sort(t.begin(), t.end());
    printf("%s D=%4d: %.3f ms\n", D < 0 ? "library step kernel      " : "near-only trailing       ", D, t[2]);
  }
  printf("DECOUPLE PROBE DONE\n");
  return 0;
}
