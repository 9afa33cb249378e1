// Latency probe of the 16x16 pivot-block factorisation (diagnostic): one wave runs chol16 (rank-1 pivots) or
// chol16_mfma (4-pivot blocks on fp64 MFMA) REPS times on the same SPD block and reports cycles per call, plus the
// max difference between the two variants' L and D = L^{-1}.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        chol16_probe.hip -o chol16_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include "gpx_internal.h"
#include "gpx_chol64.h"
using namespace gpx;
#ifndef VARIANT
#define VARIANT ""
#endif
constexpr int LDD = 20, REPS = 64;

template <int V>
__global__ void probe(const double* A, double* L, double* D, long long* cyc) {
  __shared__ double sA[16 * LD64], sD[16 * LDD], sF[128];
  const int t = threadIdx.x;
  long long total = 0;
  int f = -1;
  for (int r = 0; r < REPS; ++r) {
    for (int e = t; e < 256; e += 64) sA[(e >> 4) * LD64 + (e & 15)] = A[e];
    __syncthreads();
    const long long c0 = __builtin_readcyclecounter();
    if (V == 0)
      f = chol16<LDD>(sA, sD, 0);
    else
      f = chol16_mfma<LDD>(sA, sD, 0, sF);
    __syncthreads();
    total += __builtin_readcyclecounter() - c0;
  }
  for (int e = t; e < 256; e += 64) {
    L[e] = sA[(e >> 4) * LD64 + (e & 15)];
    D[e] = sD[(e >> 4) * LDD + (e & 15)];
  }
  if (t == 0) cyc[0] = total / REPS, cyc[1] = f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  double hA[256];
  srand(7);
  double B[256];
  for (int i = 0; i < 256; ++i) B[i] = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = i == j ? 16.0 : 0.0;
      for (int k = 0; k < 16; ++k) s += B[i * 16 + k] * B[j * 16 + k];
      hA[i * 16 + j] = s;
    }
  double *A, *L, *D;
  long long* cyc;
  CK(hipMalloc(&A, 2048));
  CK(hipMalloc(&L, 2 * 2048));
  CK(hipMalloc(&D, 2 * 2048));
  CK(hipMalloc(&cyc, 32));
  CK(hipMemcpy(A, hA, 2048, hipMemcpyHostToDevice));
  long long hc[2][2];
  probe<0><<<1, 64>>>(A, L, D, cyc);
  CK(hipMemcpy(hc[0], cyc, 16, hipMemcpyDeviceToHost));
  probe<1><<<1, 64>>>(A, L + 256, D + 256, cyc);
  CK(hipMemcpy(hc[1], cyc, 16, hipMemcpyDeviceToHost));
  double hL[512], hD[512];
  CK(hipMemcpy(hL, L, 4096, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hD, D, 4096, hipMemcpyDeviceToHost));
  double dl = 0, dd = 0, res = 0;
  for (int i = 0; i < 256; ++i) dl = fmax(dl, fabs(hL[i] - hL[256 + i])), dd = fmax(dd, fabs(hD[i] - hD[256 + i]));
  for (int i = 0; i < 16; ++i)  // |L L^T - A|
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += hL[256 + i * 16 + k] * hL[256 + j * 16 + k];
      res = fmax(res, fabs(s - hA[i * 16 + j]));
    }
  printf("chol16 (rank-1" VARIANT "): %lld cycles/call, fail=%lld\n", hc[0][0], hc[0][1]);
  printf("chol16_mfma:     %lld cycles/call, fail=%lld\n", hc[1][0], hc[1][1]);
  printf("max|dL|=%.2e max|dD|=%.2e  mfma |LL^T-A|=%.2e\n", dl, dd, res);
  printf("CHOL16 PROBE DONE\n");
  return 0;
}
