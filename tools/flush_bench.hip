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

template <bool KM, int STAG = 0, int EPI = 0>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
flush_kernel(double* __restrict__ Cm, int64_t ldc, const double* __restrict__ L, int64_t ldl, int K) {
  using T = MfmaTile<128, 128, 16, KM, KM>;
  __shared__ __attribute__((aligned(16))) double lds[T::LDS_DOUBLES];
  // STAG > 0: the odd workgroups of the first round start STAG x ~3.4 us late, so the rounds after it are out of step
  // (every tile has the same K: the grid otherwise runs in lockstep rounds whose C loads / stores all fall together)
  if constexpr (STAG > 0) {
    if (blockIdx.x < 512 && (blockIdx.x & 1))
      for (int i = 0; i < STAG; ++i) __builtin_amdgcn_s_sleep(127);
  }
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
        if constexpr (EPI == 0) *p = *p - tl.acc[i][j][r];  // read-modify-write C (the flush)
        if constexpr (EPI == 1) *p = tl.acc[i][j][r];       // store only (timing: no C read)
        if constexpr (EPI == 2)                              // nothing stored unless impossible (timing: no C traffic)
          if (tl.acc[i][j][r] == 12345.678) *p = 0.0;
      }
}

// F5: persistent workgroups (one per slot) walking tiles b, b + grid, ...: the last k-tile of a tile issues the next
// tile's first k-tile loads and this tile's first C row group, and stores the next tile's k-tile into the idle LDS
// buffer, so the next tile starts without a load round trip and the C epilogue runs while those loads are in flight.
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
flush_persistent(double* __restrict__ Cm, int64_t ldc, const double* __restrict__ L, int64_t ldl, int K, int tiles) {
  using T = MfmaTile<128, 128, 16, false, false>;
  constexpr int BK = 16;
  __shared__ __attribute__((aligned(16))) double lds[T::LDS_DOUBLES];
  double* cur = lds;
  double* nxt = lds + BK * (T::PA + T::PB);
  int t = (int)blockIdx.x;
  if (t >= tiles) return;
  int I, J;
  tri_decode(t, I, J);
  const double* A = L + (int64_t)I * 128 * ldl;
  const double* B = L + (int64_t)J * 128 * ldl;
  T tl;
  tl.load_regs(A, ldl, B, ldl, 0);
  tl.store_lds(cur, cur + BK * T::PA);
  __syncthreads();
#pragma unroll 1
  while (true) {
    const int tn = t + (int)gridDim.x;
    const bool has_next = tn < tiles;
    int In = 0, Jn = 0;
    if (has_next) tri_decode(tn, In, Jn);
    const double* An = L + (int64_t)In * 128 * ldl;
    const double* Bn = L + (int64_t)Jn * 128 * ldl;
    double* C = Cm + (int64_t)I * 128 * ldc + (int64_t)J * 128;
    tl.zero();
#pragma unroll 1
    for (int k0 = 0; k0 + BK < K; k0 += BK) {
      tl.load_regs(A, ldl, B, ldl, k0 + BK);
      tl.compute(cur, cur + BK * T::PA);
      tl.store_lds(nxt, nxt + BK * T::PA);
      __syncthreads();
      double* x = cur;
      cur = nxt;
      nxt = x;
    }
    if (has_next) tl.load_regs(An, ldl, Bn, ldl, 0);
    double cv[T::WN][4];
    auto load_group = [&](int i) {
#pragma unroll
      for (int j = 0; j < T::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cv[j][r] = C[(int64_t)T::row_of(i, r) * ldc + T::col_of(j)];
    };
    load_group(0);
    tl.compute(cur, cur + BK * T::PA);
    if (has_next) tl.store_lds(nxt, nxt + BK * T::PA);
    __syncthreads();
    {
      double* x = cur;
      cur = nxt;
      nxt = x;
    }
#pragma unroll
    for (int i = 0; i < T::WM; ++i) {
#pragma unroll
      for (int j = 0; j < T::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) tl.acc[i][j][r] = cv[j][r] - tl.acc[i][j][r];
      if (i + 1 < T::WM) load_group(i + 1);
#pragma unroll
      for (int j = 0; j < T::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) C[(int64_t)T::row_of(i, r) * ldc + T::col_of(j)] = tl.acc[i][j][r];
    }
    if (!has_next) break;
    t = tn;
    I = In;
    J = Jn;
    A = An;
    B = Bn;
  }
}

// F7 / F8: the library's trailing tile (peeled last k-tile with C row group 0 loaded under it, group i+1 loaded before
// group i's stores) with (PF) / without an L2 prefetch of the C tile a few k-tiles before the end: each thread touches
// four of the tile's 128-byte lines with plain loads whose values feed an empty asm at the epilogue, so the loads stay
// alive, retire under the k loop's MFMAs and leave the lines in L2 for the epilogue's reads.
template <bool PF>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
flush_lib(double* __restrict__ Cm, int64_t ldc, const double* __restrict__ L, int64_t ldl, int K) {
  using T = MfmaTile<128, 128, 16, false, false>;
  constexpr int BK = 16;
  __shared__ __attribute__((aligned(16))) double lds[T::LDS_DOUBLES];
  int I, J;
  tri_decode((int)blockIdx.x, I, J);
  const double* A = L + (int64_t)I * 128 * ldl;
  const double* B = L + (int64_t)J * 128 * ldl;
  double* C = Cm + (int64_t)I * 128 * ldc + (int64_t)J * 128;
  T tl;
  tl.zero();
  double* cur = lds;
  double* nxt = lds + BK * (T::PA + T::PB);
  tl.load_regs(A, ldl, B, ldl, 0);
  tl.store_lds(cur, cur + BK * T::PA);
  __syncthreads();
  double pf[4] = {0.0, 0.0, 0.0, 0.0};
  const int t = threadIdx.x;
  for (int k0 = 0; k0 + BK < K; k0 += BK) {
    tl.load_regs(A, ldl, B, ldl, k0 + BK);
    if constexpr (PF) {
      if (k0 + 4 * BK == K) {  // three k-tiles before the end
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int line = t + q * WG;  // 1024 lines: row line / 8, 16 doubles each
          pf[q] = C[(int64_t)(line >> 3) * ldc + (line & 7) * 16];
        }
      }
    }
    tl.compute(cur, cur + BK * T::PA);
    tl.store_lds(nxt, nxt + BK * T::PA);
    __syncthreads();
    double* x = cur;
    cur = nxt;
    nxt = x;
  }
  double cv[T::WN][4];
  auto load_group = [&](int i) {
#pragma unroll
    for (int j = 0; j < T::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[j][r] = C[(int64_t)T::row_of(i, r) * ldc + T::col_of(j)];
  };
  load_group(0);
  tl.compute(cur, cur + BK * T::PA);
  if constexpr (PF) asm volatile("" ::"v"(pf[0]), "v"(pf[1]), "v"(pf[2]), "v"(pf[3]));
#pragma unroll
  for (int i = 0; i < T::WM; ++i) {
#pragma unroll
    for (int j = 0; j < T::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tl.acc[i][j][r] = cv[j][r] - tl.acc[i][j][r];
    if (i + 1 < T::WM) load_group(i + 1);
#pragma unroll
    for (int j = 0; j < T::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(int64_t)T::row_of(i, r) * ldc + T::col_of(j)] = tl.acc[i][j][r];
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
  constexpr int NV = 10;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  {  // F5 against F0, bit for bit (same MFMA order per tile)
    double* C2;
    CK(hipMalloc(&C2, (size_t)m * m * 8));
    CK(hipMemset(C2, 0, (size_t)m * m * 8));
    CK(hipMemset(C0, 0, (size_t)m * m * 8));
    flush_kernel<false><<<tiles, WG>>>(C0, m, L, K, K);
    flush_persistent<<<std::min(tiles, 2 * cus), WG>>>(C2, m, L, K, K, tiles);
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    std::vector<double> a((size_t)m * m), b((size_t)m * m);
    CK(hipMemcpy(a.data(), C0, a.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), C2, b.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t q = 0; q < a.size(); ++q) bad += a[q] != b[q];
    printf("F5 vs F0 bitwise mismatches %zu\n", bad);
    CK(hipMemset(C2, 0, (size_t)m * m * 8));
    flush_lib<true><<<tiles, WG>>>(C2, m, L, K, K);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.data(), C2, b.size() * 8, hipMemcpyDeviceToHost));
    bad = 0;
    for (size_t q = 0; q < a.size(); ++q) bad += a[q] != b[q];
    printf("F7 vs F0 bitwise mismatches %zu\n", bad);
    CK(hipFree(C2));
  }
  std::vector<float> t[NV];
  for (int rep = 0; rep < 10; ++rep)
    for (int v = 0; v < NV; ++v) {
      CK(hipEventRecord(e0));
      if (v == 0)
        flush_kernel<false><<<tiles, WG>>>(C0, m, L, K, K);
      else if (v == 1)
        flush_kernel<true><<<tiles, WG>>>(C1, m, LT, m, K);
      else if (v == 2)
        flush_kernel<false, 4><<<tiles, WG>>>(C0, m, L, K, K);
      else if (v == 3)
        flush_kernel<false, 8><<<tiles, WG>>>(C0, m, L, K, K);
      else if (v == 4)
        flush_kernel<false, 16><<<tiles, WG>>>(C0, m, L, K, K);
      else if (v == 5)
        flush_persistent<<<std::min(tiles, 2 * cus), WG>>>(C0, m, L, K, K, tiles);
      else if (v == 6)
        flush_kernel<false, 0, 1><<<tiles, WG>>>(C1, m, L, K, K);
      else if (v == 7)
        flush_kernel<false, 0, 2><<<tiles, WG>>>(C1, m, L, K, K);
      else if (v == 8)
        flush_lib<false><<<tiles, WG>>>(C0, m, L, K, K);
      else
        flush_lib<true><<<tiles, WG>>>(C0, m, L, K, K);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms);
    }
  const char* names[NV] = {"F0 row-major (swizzled LDS transpose)", "F1 k-major (16-byte LDS writes)",
                           "F0, first round staggered ~14 us", "F0, first round staggered ~27 us",
                           "F0, first round staggered ~55 us", "F5 persistent, next tile prefetched",
                           "F0 timing: C stored, not read", "F0 timing: no C traffic",
                           "F8 library epilogue", "F7 library epilogue + C prefetch"};
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][t[v].size() / 2];
    printf("%-40s median %.3f ms -> %.1f TF/s\n", names[v], med, flops / (med * 1e-3) / 1e12);
  }
  printf("FLUSH BENCH DONE\n");
  return 0;
}
