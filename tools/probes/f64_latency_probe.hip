// Dependent-chain latencies (one wave, s_memtime cycles per link) of the fp64 operations on the Cholesky pivot
// chain: v_fma_f64, v_mul_f64, v_rsq_f64, v_rcp_f64, readlane -> VALU, v_mov_b64_dpp, permlane swaps, and the
// dependent v_mfma_f64_16x16x4_f64 accumulator chain.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//   -mllvm -amdgpu-mfma-vgpr-form=1 -I../../bayesianoptimizer_amd/csrc f64_latency_probe.hip -o f64_latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "gpx_chol64.h"

using namespace gpx;
constexpr int N = 256;

__global__ void probe(double* out, long long* cyc, double seed) {
  const int lane = threadIdx.x;
  double v = seed + lane * 1e-3;
  long long t0, t1;
#define CHAIN(idx, body)                                   \
  t0 = __builtin_amdgcn_s_memtime();                       \
  _Pragma("unroll 16") for (int i = 0; i < N; ++i) { body; } \
  __builtin_amdgcn_s_waitcnt(0);                            \
  out[idx * 64 + lane] = v;                                 \
  t1 = __builtin_amdgcn_s_memtime();                       \
  if (lane == 0) cyc[idx] = t1 - t0;
  CHAIN(0, v = fma(v, 0.999999, 1e-9));
  CHAIN(1, v = v * 1.0000001);
  CHAIN(2, v = __builtin_amdgcn_rsq(v));
  CHAIN(3, v = __builtin_amdgcn_rcp(v));
  CHAIN(4, v = readlane_f64(v, 5) * 1.0000001);
  CHAIN(5, v = row_newbcast<3>(v));
  CHAIN(6, v = xrow_bcast<2>(v));
  CHAIN(7, v = pivot_rsq(v));
  d4 acc = {v, v, v, v};
  const double a = v * 1e-3, b = 1e-3;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N; ++i) acc = mfma16x16x4(a, b, acc);
  out[8 * 64 + lane] = acc[0] + acc[1] + acc[2] + acc[3];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[8] = t1 - t0;
  d4 c0 = acc, c1 = acc, c2 = acc, c3 = acc;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    c0 = mfma16x16x4(a, b, c0); c1 = mfma16x16x4(a, b, c1); c2 = mfma16x16x4(a, b, c2); c3 = mfma16x16x4(a, b, c3);
  }
  out[9 * 64 + lane] = c0[0] + c1[1] + c2[2] + c3[3];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[9] = t1 - t0;
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  const long long m0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 4 * N; ++i) v = fma(v, 0.999999, 1e-9);
  out[10 * 64 + lane] = v;
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  const long long m1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { cyc[10] = m1 - m0; cyc[11] = r1 - r0; }
}

int main() {
  double* out; long long* cyc;
  hipMalloc(&out, 16 * 64 * 8);
  hipMalloc(&cyc, 16 * 8);
  for (int rep = 0; rep < 3; ++rep) probe<<<1, 64>>>(out, cyc, 1.5);
  hipDeviceSynchronize();
  long long h[16];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"v_fma_f64", "v_mul_f64", "v_rsq_f64", "v_rcp_f64", "readlane_f64+mul", "v_mov_b64_dpp newbcast",
                         "xrow_bcast (2x permlane16/32 swap)", "pivot_rsq (rsq + Newton)", "mfma_f64_16x16x4 dependent",
                         "mfma_f64_16x16x4 4 independent (per MFMA)"};
  for (int i = 0; i < 10; ++i) printf("%-42s %7.1f cyc/link\n", names[i], (double)h[i] / (i == 9 ? 4 * N : N));
  printf("clock: %.2f GHz (memtime/memrealtime*100MHz)\n", (double)h[10] / h[11] * 0.1);
  printf("F64 LATENCY PROBE DONE\n");
  return 0;
}
