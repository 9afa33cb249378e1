// Timeline probe of the persistent triangular solve (diagnostic; includes the shipped gpx_potrs.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        potrs_probe.hip -o potrs_probe
// Runs gpx_potrs on an identity factor (the timing does not depend on the values) and prints, per work item, the
// wall-clock stamps (100 MHz) of: item start, last block detected, after the combine barrier, before the publish,
// relative to the first item's start; then the per-hop latency (detect of item i+1's last block - publish of item i).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_internal.h"
__device__ unsigned long long g_stamp[1024][4];
__device__ unsigned long long g_cyc[1024][4];
#define GPX_POTRS_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.y == 0) { g_stamp[fwd ? K : 2 * nb - 1 - K][i] = wall_clock64(); g_cyc[fwd ? K : 2 * nb - 1 - K][i] = __builtin_readcyclecounter(); } } while (0)
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrs.hip"

using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int nrhs = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = 5;
  const int npad = (n + 127) / 128 * 128, nblk = npad / 64, nb = npad / 128;
  std::vector<double> hL((size_t)npad * npad, 0.0), hD((size_t)2 * nblk * 64 * 64, 0.0), hY((size_t)n * nrhs, 1.0);
  for (int i = 0; i < npad; ++i) hL[(size_t)i * npad + i] = 1.0;
  for (int k = 0; k < nblk; ++k)
    for (int i = 0; i < 64; ++i) hD[(size_t)k * 4096 + i * 64 + i] = 1.0;
  double *L, *D, *Y, *a;
  void* ws;
  CK(hipMalloc(&L, hL.size() * 8));
  CK(hipMalloc(&D, hD.size() * 8));
  CK(hipMalloc(&Y, hY.size() * 8));
  CK(hipMalloc(&a, (size_t)npad * nrhs * 8));
  const size_t wsb = potrs_workspace_bytes(npad, nrhs, 1);
  CK(hipMalloc(&ws, wsb));
  CK(hipMemcpy(L, hL.data(), hL.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(D, hD.data(), hD.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Y, hY.data(), hY.size() * 8, hipMemcpyHostToDevice));
  Context ctx;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, 0));
    CK(launch_potrs(&ctx, n, npad, L, npad, D, Y, nrhs, nrhs, 0.0, a, nullptr, ws));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  std::vector<double> ha((size_t)npad * nrhs);
  CK(hipMemcpy(ha.data(), a, ha.size() * 8, hipMemcpyDeviceToHost));
  double err = 0;
  for (int i = 0; i < n * nrhs; ++i) err = fmax(err, fabs(ha[i] - 1.0));
  unsigned long long st[1024][4];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st)));
  printf("n=%d nrhs=%d: potrs %.1f us (best of %d, incl. memset), %d items, max|alpha-1|=%.1e\n", n, nrhs, best * 1e3,
         reps, 2 * nb, err);
  const unsigned long long t0 = st[0][0];
  auto us = [&](unsigned long long v) { return (double)(long long)(v - t0) / 100.0; };
  double hop = 0, solve = 0, comb = 0;
  int cnt = 0;
  for (int i = 0; i < 2 * nb; ++i) {
    if (i < 12 || i >= 2 * nb - 4 || (i >= nb - 2 && i <= nb + 2))
      printf("item %3d: start %8.2f  detect %8.2f  combined %8.2f  publish %8.2f\n", i, us(st[i][0]), us(st[i][1]),
             us(st[i][2]), us(st[i][3]));
    if (i > 1 && i != nb) {
      hop += us(st[i][1]) - us(st[i - 1][3]);
      comb += us(st[i][2]) - us(st[i][1]);
      solve += us(st[i][3]) - us(st[i][2]);
      ++cnt;
    }
  }
  unsigned long long cy[1024][4];
  CK(hipMemcpyFromSymbol(cy, HIP_SYMBOL(g_cyc), sizeof(cy)));
  printf("shader clock over item 1: %.0f MHz\n", (double)(cy[1][3] - cy[1][0]) / ((double)(st[1][3] - st[1][0]) / 100.0));
  printf("per step: hop (publish -> next detect) %.2f us, detect -> combined %.2f us, solve %.2f us\n", hop / cnt,
         comb / cnt, solve / cnt);
  printf("POTRS PROBE DONE\n");
  return 0;
}
