// Timeline probe of a fit's backward solve (diagnostic; includes the shipped gpx_potrs.hip): potrs_bwd_fit_1 on an
// identity factor with z given (the timing does not depend on the values).  Per item K (chain order, nb-1 first):
// start, setup done, subtraction done (last block before alpha_{K+1}), [P items: wait for alpha_{K+1} begins, block
// detected], end; in us relative to the first item's start (100 MHz wall clock).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        potrs_fit_probe.hip -o potrs_fit_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_internal.h"
__device__ unsigned long long g_fst[1024][6];
#define GPX_POTRS_FIT_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.y == 0) g_fst[K][i] = wall_clock64(); } while (0)
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrs.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int npad = (n + 127) / 128 * 128, nblk = npad / 64, nb = npad / 128;
  std::vector<double> hL((size_t)npad * npad, 0.0), hD((size_t)2 * nblk * 64 * 64, 0.0), hz(npad, 1.0);
  for (int i = 0; i < npad; ++i) hL[(size_t)i * npad + i] = 1.0;
  for (int k = 0; k < nblk; ++k)
    for (int i = 0; i < 64; ++i) hD[(size_t)k * 4096 + i * 64 + i] = 1.0;
  double *L, *D, *z, *a;
  void* ws;
  CK(hipMalloc(&L, hL.size() * 8));
  CK(hipMalloc(&D, hD.size() * 8));
  CK(hipMalloc(&z, npad * 8));
  CK(hipMalloc(&a, (size_t)npad * 8));
  CK(hipMalloc(&ws, potrs_workspace_bytes(npad, 1, 1)));
  CK(hipMemcpy(L, hL.data(), hL.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(D, hD.data(), hD.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(z, hz.data(), npad * 8, hipMemcpyHostToDevice));
  Context ctx;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, 0));
    CK(launch_potrs(&ctx, n, npad, L, npad, D, z, 1, 1, 0.0, a, nullptr, ws, Batch(), false, z, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  std::vector<double> ha(npad);
  CK(hipMemcpy(ha.data(), a, npad * 8, hipMemcpyDeviceToHost));
  double err = 0;
  for (int i = 0; i < n; ++i) err = fmax(err, fabs(ha[i] - 1.0));
  unsigned long long st[1024][6];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_fst), sizeof(st)));
  printf("n=%d: fit backward solve %.1f us (best of 5, incl. memset), %d items, max|alpha-1|=%.1e\n", n, best * 1e3, nb,
         err);
  unsigned long long t0 = ~0ull;
  for (int K = 0; K < nb; ++K) t0 = st[K][0] < t0 ? st[K][0] : t0;
  auto us = [&](unsigned long long v) { return v ? (double)(long long)(v - t0) / 100.0 : -1.0; };
  for (int K = nb - 1; K >= 0; --K)
    printf("K %3d (d %3d): start %7.2f setup %7.2f subtracted %7.2f wait %7.2f detected %7.2f end %7.2f\n", K,
           nb - 1 - K, us(st[K][0]), us(st[K][1]), us(st[K][2]), us(st[K][3]), us(st[K][4]), us(st[K][5]));
  printf("POTRS FIT PROBE DONE\n");
  return 0;
}
