// Flush-tile microbenchmark for the large-n Cholesky (diagnostic): one launch of every 128x128 lower tile of an
// m x m trailing matrix, C -= L_I L_J^T with K = 512 (the n = 16384 schedule flushes 8 block columns at once), as
//   F0  the step kernel's tile: row-major L panels (A[i][k]), transposed into LDS with the XOR swizzle (Tile128),
//   F1  k-major panels (a transposed copy LT[k][i] of the same columns): 16-byte LDS writes, the sweep product's tile,
// both in kernels of their own with the step kernel's occupancy (two workgroups per CU).  Prints TF/s on the 2 m^2/2 K
// useful flops, and whether F1's C equals F0's bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        flush_bench.hip -o flush_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_device.h"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <bool KM>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
flush_kernel(double* __restrict__ Cm, int64_t ldc, const double* __restrict__ L, int64_t ldl, int K) {
  using T = MfmaTile<128, 128, 16, KM, KM>;
  __shared__ __attribute__((aligned(16))) double lds[T::LDS_DOUBLES];
  int I, J;
  tri_decode((int)blockIdx.x, I, J);
  // row-major: L[i][k] (ldl = K); k-major: LT[k][i] (ldl = m)
  const double* A = KM ? L + (int64_t)I * 128 : L + (int64_t)I * 128 * ldl;
  const double* B = KM ? L + (int64_t)J * 128 : L + (int64_t)J * 128 * ldl;
  T tl;
  tl.run(A, ldl, B, ldl, 0, K, lds);
  double* C = Cm + (int64_t)I * 128 * ldc + (int64_t)J * 128;
#pragma unroll
  for (int i = 0; i < T::WM; ++i)
#pragma unroll
    for (int j = 0; j < T::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double* p = C + (int64_t)T::row_of(i, r) * ldc + T::col_of(j);
        *p = *p - tl.acc[i][j][r];
      }
}

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 15872, K = argc > 2 ? atoi(argv[2]) : 512;
  const int M = m / 128, tiles = M * (M + 1) / 2;
  std::vector<double> hL((size_t)m * K), hLT((size_t)m * K);
  srand(5);
  for (int i = 0; i < m; ++i)
    for (int k = 0; k < K; ++k) hLT[(size_t)k * m + i] = hL[(size_t)i * K + k] = rand() / (double)RAND_MAX - 0.5;
  double *C0, *C1, *L, *LT;
  CK(hipMalloc(&C0, (size_t)m * m * 8));
  CK(hipMalloc(&C1, (size_t)m * m * 8));
  CK(hipMalloc(&L, hL.size() * 8));
  CK(hipMalloc(&LT, hLT.size() * 8));
  CK(hipMemcpy(L, hL.data(), hL.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(LT, hLT.data(), hLT.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemset(C0, 0, (size_t)m * m * 8));
  CK(hipMemset(C1, 0, (size_t)m * m * 8));
  flush_kernel<false><<<tiles, WG>>>(C0, m, L, K, K);
  flush_kernel<true><<<tiles, WG>>>(C1, m, LT, m, K);
  CK(hipDeviceSynchronize());
  {
    std::vector<double> a((size_t)m * m), b((size_t)m * m);
    CK(hipMemcpy(a.data(), C0, a.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), C1, b.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t q = 0; q < a.size(); ++q) bad += a[q] != b[q];
    printf("m=%d K=%d tiles=%d: F1 vs F0 bitwise mismatches %zu\n", m, K, tiles, bad);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flops = 2.0 * 128 * 128 * (double)K * tiles;
  std::vector<float> t[2];
  for (int rep = 0; rep < 10; ++rep)
    for (int v = 0; v < 2; ++v) {
      CK(hipEventRecord(e0));
      if (v == 0)
        flush_kernel<false><<<tiles, WG>>>(C0, m, L, K, K);
      else
        flush_kernel<true><<<tiles, WG>>>(C1, m, LT, m, K);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms);
    }
  const char* names[2] = {"F0 row-major (swizzled LDS transpose)", "F1 k-major (16-byte LDS writes)"};
  for (int v = 0; v < 2; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][t[v].size() / 2];
    printf("%-40s median %.3f ms -> %.1f TF/s\n", names[v], med, flops / (med * 1e-3) / 1e12);
  }
  printf("FLUSH BENCH DONE\n");
  return 0;
}
