// Launch-level split of the eager Cholesky schedule (diagnostic; includes the shipped gpx_potrf.hip): for a step c,
// the average duration of the full launch, of its panel workgroups alone and of its trailing workgroups alone
// (20 back-to-back launches each, after steps 0 .. c-1 ran once on a fresh RBF Gram matrix).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        potrf_trail_probe.hip -o potrf_trail_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_internal.h"
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, nblk = n / 64;
  const int xmap = argc > 2 ? atoi(argv[2]) : 1;  // trailing tile order (trail_tile)
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
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto plan = [&](int c) { return step_plan(c, nblk, 0, c > 0 ? c - 1 : 0, c >= 1, xmap); };
  // mode 0 full grid, 1 panel workgroups only, 2 trailing workgroups only
  auto time_step = [&](int c, int mode) {
    CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemset(info, 0, 4));
    for (int cc = 0; cc < c; ++cc) {
      const StepPlan s = plan(cc);
      potrf_step_kernel<0><<<s.tbase + s.ntrail, WG>>>(A, n, cc, nblk, s, Dinv, info, 0, 0, 0, PotrfFwd());
    }
    CK(hipDeviceSynchronize());
    const StepPlan s = plan(c);
    const int grid = mode == 0 ? s.tbase + s.ntrail : mode == 1 ? s.npanel : s.ntrail;
    const int first = mode == 2 ? s.tbase : 0;
    if (grid == 0) return 0.0f;
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) potrf_step_kernel<0><<<grid, WG>>>(A, n, c, nblk, s, Dinv, info, first, 0, 0, PotrfFwd());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 50.0f;  // us per launch
  };
  for (int c : {1, 2, 5, 10, 16, 24, 40, nblk - 3}) {
    if (c >= nblk) continue;
    const StepPlan s = plan(c);
    printf("step %2d: full %6.2f us   panel wgs only %6.2f us (%d)   trailing wgs only %6.2f us (%d tiles)\n", c,
           time_step(c, 0), time_step(c, 1), s.npanel, time_step(c, 2), s.ntrail);
  }
  printf("xmap=%d TRAIL PROBE DONE\n", xmap);
  return 0;
}
