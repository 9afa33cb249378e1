// The sweep product's k loop at one workgroup per CU (diagnostic): the shipped trmm tile (128 x 128, BK = 16, two
// workgroups per CU) against BK = 32 (147 KB of LDS: one workgroup per CU, half the barriers per flop) and BK = 16 forced
// to one workgroup per CU, in the shipped XCD-aware heavy-first order on the n = 4096, 32768-candidate chunk.  The MFMA
// order per output is the same (k ascending), so the column sums must match bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        trmm_occ_bench.hip -o trmm_occ_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_device.h"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
constexpr int TT = 128;

template <int BK, int STAGGER = 0>
__device__ __forceinline__ void trmm_body(const double* __restrict__ W, int64_t ldw, const double* __restrict__ kstar,
                                          int64_t C, int nI, int ncb, double* __restrict__ ss_part, double* smem) {
  using Tile = MfmaTile<TT, TT, BK, true, true>;
  const int b = blockIdx.x;
  // STAGGER > 0: workgroups with bit STAGGER of b set start ~half a k-tile later (two co-resident workgroups out of step)
  if constexpr (STAGGER > 0) {
    if ((b >> STAGGER) & 1)
      __builtin_amdgcn_s_sleep(64);  // ~4096 cycles
  }
  const int x = b & 7, l = b >> 3, per = ncb >> 3;
  const int I = nI - 1 - l / per, cb = 8 * (l % per) + x;
  Tile tile;
  tile.run(W + (int64_t)I * TT, ldw, kstar + (int64_t)cb * TT, C, 0, (I + 1) * TT, smem);
  double s[Tile::WN];
#pragma unroll
  for (int j = 0; j < Tile::WN; ++j) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += tile.acc[i][j][r] * tile.acc[i][j][r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    s[j] = v;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if ((w >> 1) == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < Tile::WN; ++j) smem[Tile::col_of(j)] = s[j];
  }
  __syncthreads();
  if ((w >> 1) == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < Tile::WN; ++j)
      ss_part[(int64_t)I * C + (int64_t)cb * TT + Tile::col_of(j)] = s[j] + smem[Tile::col_of(j)];
  }
}

__global__ void __launch_bounds__(256) trmm_bk16(const double* W, int64_t ldw, const double* K, int64_t C, int nI, int ncb,
                                                 double* ss) {
  __shared__ __attribute__((aligned(16))) double smem[MfmaTile<TT, TT, 16, true, true>::LDS_DOUBLES];
  trmm_body<16>(W, ldw, K, C, nI, ncb, ss, smem);
}
template <int ST>
__global__ void __launch_bounds__(256) trmm_stagger(const double* W, int64_t ldw, const double* K, int64_t C, int nI,
                                                    int ncb, double* ss) {
  __shared__ __attribute__((aligned(16))) double smem[MfmaTile<TT, TT, 16, true, true>::LDS_DOUBLES];
  trmm_body<16, ST>(W, ldw, K, C, nI, ncb, ss, smem);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
trmm_bk32(const double* W, int64_t ldw, const double* K, int64_t C, int nI, int ncb, double* ss) {
  extern __shared__ __attribute__((aligned(16))) double dsmem[];
  trmm_body<32>(W, ldw, K, C, nI, ncb, ss, dsmem);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
trmm_bk16_occ1(const double* W, int64_t ldw, const double* K, int64_t C, int nI, int ncb, double* ss) {
  extern __shared__ __attribute__((aligned(16))) double dsmem[];  // 100 KB requested: one workgroup per CU
  trmm_body<16>(W, ldw, K, C, nI, ncb, ss, dsmem);
}

int main() {
  const int n = 4096, C = 32768, nI = n / TT, ncb = C / TT;
  double *W, *K, *ss0, *ss1;
  CK(hipMalloc(&W, (size_t)n * n * 8));
  CK(hipMalloc(&K, (size_t)n * C * 8));
  CK(hipMalloc(&ss0, (size_t)nI * C * 8));
  CK(hipMalloc(&ss1, (size_t)nI * C * 8));
  {
    std::vector<double> h((size_t)n * n);
    srand(1);
    for (int k = 0; k < n; ++k)
      for (int i = 0; i < n; ++i) h[(size_t)k * n + i] = (k <= i) ? (rand() / (double)RAND_MAX - 0.5) : 0.0;
    CK(hipMemcpy(W, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> g((size_t)n * C);
    for (auto& v : g) v = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(K, g.data(), g.size() * 8, hipMemcpyHostToDevice));
  }
  const size_t lds32 = MfmaTile<TT, TT, 32, true, true>::LDS_DOUBLES * 8, lds_occ1 = 100 * 1024;
  CK(hipFuncSetAttribute((const void*)trmm_bk32, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds32));
  CK(hipFuncSetAttribute((const void*)trmm_bk16_occ1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_occ1));
  const char* names[] = {"BK16 2 WG/CU (shipped)", "BK32 1 WG/CU", "BK16 1 WG/CU", "stagger bit 8", "stagger bit 3",
                         "stagger bit 5"};
  constexpr int NV = 6;
  auto run = [&](int v, double* out) {
    const dim3 g(ncb * nI);
    if (v == 0) trmm_bk16<<<g, 256>>>(W, n, K, C, nI, ncb, out);
    else if (v == 1) trmm_bk32<<<g, 256, lds32>>>(W, n, K, C, nI, ncb, out);
    else if (v == 2) trmm_bk16_occ1<<<g, 256, lds_occ1>>>(W, n, K, C, nI, ncb, out);
    else if (v == 3) trmm_stagger<8><<<g, 256>>>(W, n, K, C, nI, ncb, out);
    else if (v == 4) trmm_stagger<3><<<g, 256>>>(W, n, K, C, nI, ncb, out);
    else trmm_stagger<5><<<g, 256>>>(W, n, K, C, nI, ncb, out);
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  run(0, ss0);
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  std::vector<double> ref((size_t)nI * C), got((size_t)nI * C);
  CK(hipMemcpy(ref.data(), ss0, ref.size() * 8, hipMemcpyDeviceToHost));
  for (int v = 1; v < NV; ++v) {
    CK(hipMemset(ss1, 0, (size_t)nI * C * 8));
    run(v, ss1);
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    CK(hipMemcpy(got.data(), ss1, got.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t q = 0; q < ref.size(); ++q) bad += (ref[q] != got[q]);
    printf("%-24s bitwise mismatches vs shipped: %zu\n", names[v], bad);
  }
  const double flops = (double)n * n * C;
  std::vector<std::vector<float>> t(NV);
  for (int rep = 0; rep < 8; ++rep)
    for (int v = 0; v < NV; ++v) {
      CK(hipEventRecord(e0));
      run(v, ss1);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms);
    }
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][t[v].size() / 2];
    printf("%-24s median %.3f ms min %.3f ms -> %.2f TF/s (frac %.4f)\n", names[v], med, t[v][0],
           flops / (med * 1e-3) / 1e12, flops / (med * 1e-3) / 78.6e12);
  }
  printf("TRMM OCC BENCH DONE\n");
  return 0;
}
