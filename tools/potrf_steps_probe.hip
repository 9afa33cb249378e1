// Per-launch timeline of the multi-launch Cholesky (diagnostic; includes the shipped gpx_potrf.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        potrf_steps_probe.hip -o potrf_steps_probe
// For every launch c (100 MHz wall clock, us): first workgroup start, last panel / trailing workgroup end, and the
// chain-critical panel workgroup (p = 1, which produces L_{c+1,c}; p = 0 for the last column): its start, end of the
// pre-update, end of each of the four in-wave pivot blocks (F), end of the factorisation, end of the store.  Summary:
// the mean gap between launch c's last end and launch c+1's first start, and the mean phase durations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "gpx_internal.h"
__device__ unsigned long long g_first[256], g_pend[256], g_tend[256];
__device__ unsigned long long g_pan[256][16];
#define GPX_STEP_STAMP(role, c, b, s)                                                                     \
  do {                                                                                                    \
    if (threadIdx.x == 0) {                                                                               \
      const unsigned long long now_ = wall_clock64();                                                     \
      if ((s) == 0) atomicMin(&g_first[c], now_);                                                        \
      else if ((role) == 0) atomicMax(&g_pend[c], now_);                                                  \
      else atomicMax(&g_tend[c], now_);                                                                   \
      if ((role) == 0 && (b) == ((c) + 1 < nblk ? 1 : 0)) g_pan[c][(s) == 0 ? 0 : 15] = now_;            \
    }                                                                                                     \
  } while (0)
#define GPX_PANEL_STAMP(i)                                                                                \
  do {                                                                                                    \
    if (threadIdx.x == 0 && p == (c + 1 < nblk ? 1 : 0) && ((i) == 0 || (i) % 3 == 1 || (i) == 13))       \
      g_pan[c][(i) == 0 ? 1 : ((i) == 13 ? 6 : 2 + (i) / 3)] = wall_clock64();                            \
    if ((threadIdx.x & 63) == 0 && threadIdx.x > 0 && p == (c + 1 < nblk ? 1 : 0) && (i) % 3 == 0 && (i) > 0 && (i) < 12) \
      atomicMax(&g_pan[c][9 + (i) / 3 - 1], wall_clock64());                                             \
  } while (0)
#define GPX_EAGER_STAMP(c, p, i)                                                                          \
  do {                                                                                                    \
    if (threadIdx.x == 0 && p == 1) g_pan[c][7 + (i)] = wall_clock64();             \
  } while (0)
namespace gpx {
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096;
  const int npad = (n + 127) / 128 * 128, nblk = npad / 64;
  std::vector<double> hA((size_t)npad * npad);
  srand(3);
  for (int i = 0; i < npad; ++i)
    for (int j = 0; j <= i; ++j) {
      const double v = i == j ? (double)npad : 0.1 * ((double)rand() / RAND_MAX - 0.5);
      hA[(size_t)i * npad + j] = hA[(size_t)j * npad + i] = v;
    }
  double *A, *Dv;
  int32_t* info;
  // argv[2]: allocation of the factored matrix (0 hipMalloc, 1 fine-grained, 3 uncached): whether the kernel-boundary
  // L2 write-back of dirty lines is what the launch gap pays
  const int amode = argc > 2 ? atoi(argv[2]) : 0;
  if (amode == 0)
    CK(hipMalloc(&A, hA.size() * 8));
  else
    CK(hipExtMallocWithFlags((void**)&A, hA.size() * 8, amode));
  CK(hipMalloc(&Dv, (size_t)2 * nblk * 4096 * 8));
  CK(hipMalloc(&info, 4));
  // argv[3]: right-hand sides of a folded forward substitution (0: the plain factorisation; 1: a fit's, NR = 1)
  const int nrhs = argc > 3 ? atoi(argv[3]) : 0;
  double *Y, *fbuf;
  CK(hipMalloc(&Y, (size_t)npad * 8 * 8));
  CK(hipMalloc(&fbuf, (size_t)2 * npad * GPX_MAX_RHS * 8));
  CK(hipMemset(Y, 0, (size_t)npad * 8 * 8));
  ForwardRhs fr;
  fr.Y = Y;
  fr.ldy = nrhs > 0 ? nrhs : 1;
  fr.nrhs = nrhs > 0 ? nrhs : 1;
  fr.n = n;
  fr.buf = fbuf;
  bool zdone = false;
  Context ctx;
  Batch bt{1, 0, 0, 0};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> ones(256, ~0ull), zeros(256, 0);
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(info, 0, 4));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_first), ones.data(), 2048));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_pend), zeros.data(), 2048));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tend), zeros.data(), 2048));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    CK(launch_potrf(&ctx, npad, A, npad, Dv, info, bt, nullptr, 0, nrhs > 0 ? &fr : nullptr, &zdone));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  int hinfo;
  CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
  std::vector<unsigned long long> f(256), pe(256), te(256), pan(256 * 16);
  CK(hipMemcpyFromSymbol(f.data(), HIP_SYMBOL(g_first), 2048));
  CK(hipMemcpyFromSymbol(pe.data(), HIP_SYMBOL(g_pend), 2048));
  CK(hipMemcpyFromSymbol(te.data(), HIP_SYMBOL(g_tend), 2048));
  CK(hipMemcpyFromSymbol(pan.data(), HIP_SYMBOL(g_pan), 256 * 16 * 8));
  printf("n=%d nblk=%d alloc=%d: potrf %.3f ms (hipEvent, incl. dinv), info=%d\n", n, nblk, amode, ms, hinfo);
  const unsigned long long t0 = f[0];
  auto us = [&](unsigned long long v) { return v ? (double)(long long)(v - t0) / 100.0 : -1.0; };
  double eload = 0, ecomp = 0;
  double uw[3] = {0, 0, 0};  // waves 1-3 done with step s's U items, relative to wave 0's end of F(s+1)
  double gap = 0, pre = 0, F[4] = {0, 0, 0, 0}, tail = 0, store = 0, wait0 = 0, trail_after = 0;
  int cnt = 0;
  printf("  c   start  panel_end trail_end | crit: start  pre   F0    F1    F2    F3   fact  store\n");
  for (int c = 0; c < nblk; ++c) {
    const unsigned long long* P = &pan[c * 16];
    const unsigned long long end = pe[c] > te[c] ? pe[c] : te[c];
    if (c < 6 || c % 8 == 0 || (c > 8 && c < 16) || (c > 96 && c < 104) || (c > 168 && c < 176) || c >= nblk - 3)
      printf("%3d %7.2f %8.2f %8.2f | %6.2f %5.2f %5.2f %5.2f %5.2f %5.2f %5.2f %5.2f\n", c, us(f[c]), us(pe[c]),
             te[c] ? us(te[c]) : -1.0, us(P[0]), (double)(P[1] - P[0]) / 100, (double)(P[2] - P[1]) / 100,
             (double)(P[3] - P[2]) / 100, (double)(P[4] - P[3]) / 100, (double)(P[5] - P[4]) / 100,
             (double)(P[6] - P[5]) / 100, (double)(P[15] - P[6]) / 100);
    if (c > 0 && c + 1 < nblk) {
      const unsigned long long pend = pe[c - 1] > te[c - 1] ? pe[c - 1] : te[c - 1];
      gap += (double)(long long)(f[c] - pend) / 100;
      wait0 += (double)(long long)(P[0] - f[c]) / 100;
      pre += (double)(P[1] - P[0]) / 100;
      eload += (double)(P[7] - P[0]) / 100;
      ecomp += (double)(P[8] - P[7]) / 100;
      for (int s = 0; s < 4; ++s) F[s] += (double)(P[2 + s] - P[1 + s]) / 100;
      tail += (double)(P[6] - P[5]) / 100;
      store += (double)(P[15] - P[6]) / 100;
      trail_after += te[c] > pe[c] ? (double)(te[c] - pe[c]) / 100 : 0.0;
      for (int s = 0; s < 3; ++s) uw[s] += (double)(long long)(P[9 + s] - P[3 + s]) / 100;
      ++cnt;
    }
    (void)end;
  }
  printf("mean over launches 1..nblk-2: launch gap %.2f us, crit-WG start after first WG %.2f, pre-update %.2f, "
         "F steps %.2f %.2f %.2f %.2f, last step tail %.2f, store %.2f, trailing beyond panels %.2f us\n",
         gap / cnt, wait0 / cnt, pre / cnt, F[0] / cnt, F[1] / cnt, F[2] / cnt, F[3] / cnt, tail / cnt, store / cnt,
         trail_after / cnt);
  printf("waves 1-3 end of U items of step s minus wave 0's end of F(s+1) (> 0: they hold the barrier): s=0 %.2f s=1 %.2f s=2 %.2f us\n",
         uw[0] / cnt, uw[1] / cnt, uw[2] / cnt);
  printf("eager pre-update split: start -> operands in LDS %.2f us, products %.2f us, stores %.2f us\n", eload / cnt,
         ecomp / cnt, (pre - eload - ecomp) / cnt);
  printf("last launch end %.2f us\n", us(pe[nblk - 1] > te[nblk - 1] ? pe[nblk - 1] : te[nblk - 1]));
  printf("STEPS PROBE DONE\n");
  return 0;
}
