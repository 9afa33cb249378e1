// Round 5: the sweep product's k loop with a HAND-PLACED instruction stream.
// Same tile as the library's trmm_sumsq_kernel (gpx_sweep.hip): 128x128 output tile per 256-thread workgroup, 4 waves in
// 2x2 of 64x64 (4x4 v_mfma_f64_16x16x4 blocks each), BK = 16, k-major LDS tiles padded to 144 doubles, two LDS buffers,
// XCD-aware heavy-first block order, column sums of V^2.  Every accumulator sees the same MFMA sequence (k ascending in
// steps of 4, lane (kr, m) supplying A[m][k0 + kr]) as MfmaTile, so the outputs must equal the shipped kernel's bit for
// bit.  What changes is WHERE the memory instructions sit among the 64 MFMAs of a k-tile (one asm statement per
// instruction, waits counted by hand):
//   S0  fragments of substep 0 (8 ds_read_b64, issued in the previous tile's S3) -> 16 MFMAs, interleaved with the 8
//       fragment reads of S1 and, after vmcnt(0), the 8 ds_write_b128 of the NEXT k-tile into the other buffer
//   S1  16 MFMAs, interleaved with the 8 reads of S2 and the 8 buffer_load_dwordx4 of the k-tile after next
//   S2  16 MFMAs, interleaved with the 8 reads of S3;  lgkmcnt(0) + s_barrier (the next tile is in LDS for everyone,
//       and everyone is done reading this tile's buffer)
//   S3  16 MFMAs, interleaved with the 8 reads of the next tile's S0
// so the only exposed latency per k-tile is the barrier's skew; the compiler-scheduled loop waits after its last MFMA for
// the LDS writes, the barrier and the next tile's first fragment reads (gpx_sweep.hip ISA: ~400 cycles per k-tile).
// Variants: A1 the schedule above (bayesianoptimizer_amd/csrc/gpx_trmm_asm.h), A2 + waves 0-1 skipping the MFMAs of the
// diagonal 128-tile's zero 64-block.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_device.h"
#include "gpx_trmm_asm.h"

using namespace gpx;
#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int TT = 128;
using Base = MfmaTile<TT, TT, 16, true, true>;
using namespace gpx::trmm_asm;

template <int S>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
trmm_v(const double* __restrict__ W, int64_t ldw, const double* __restrict__ kstar, int64_t C, int nI, int ncb,
       double* __restrict__ ss_part) {
  __shared__ __attribute__((aligned(16))) double smem[LDS_BYTES / 8];
  int I, cb;
  if constexpr (S >= 3 && S != 5) {
    // candidate tiles in groups of G (all row tiles of a group, heaviest first, before the next group): the K* working
    // set of the resident workgroups is G panels instead of all of them
    constexpr int G = S == 3 ? 32 : S == 4 ? 64 : S == 6 ? 16 : S == 7 ? 128 : S == 8 ? 64 : 48;
    const int g = blockIdx.x / (nI * G), bb = blockIdx.x % (nI * G);
    const int x = bb & 7, l = bb >> 3, per = G >> 3;
    I = nI - 1 - l / per;
    cb = g * G + 8 * (l % per) + x;
  } else {
    const int b = blockIdx.x;
    const int x = b & 7, l = b >> 3, per = ncb >> 3;
    I = nI - 1 - l / per;
    cb = 8 * (l % per) + x;
  }
  if constexpr (S == 5 || S == 8) {
    if ((blockIdx.x >> 3) & 1) __builtin_amdgcn_s_setprio(1);
  }
  const double* Ab = W + (int64_t)I * TT;
  const double* Bb = kstar + (int64_t)cb * TT;
  d4 accv[4][4];
  if constexpr (S == 0) {
    Base tile;
    tile.run(Ab, ldw, Bb, C, 0, (I + 1) * TT, smem);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accv[i][j] = tile.acc[i][j];
  } else {
    gpx::trmm_asm::Tile tile;
    tile.run(Ab, ldw, Bb, C, (I + 1) * TT / 16, smem, S >= 2);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accv[i][j] = tile.acc[i][j];
  }
  double s[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += accv[i][j][r] * accv[i][j][r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    s[j] = v;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* red = smem;
  if ((w >> 1) == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[Base::col_of(j)] = s[j];
  }
  __syncthreads();
  if ((w >> 1) == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = Base::col_of(j);
      ss_part[(int64_t)I * C + (int64_t)cb * TT + col] = s[j] + red[col];
    }
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, C = argc > 2 ? atoi(argv[2]) : 32768, nI = n / TT, ncb = C / TT;
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
  const char* names[] = {"S0 shipped", "A1 hand-placed", "A2 + diag skip", "A3 A2 + cb groups of 32",
                         "A4 A2 + cb groups of 64", "A5 A2 + setprio half", "A6 A2 + groups of 16",
                         "A7 A2 + groups of 128", "A8 A4 + setprio half"};
  constexpr int NV = 9;
  auto run = [&](int v, double* out) {
    const dim3 g(ncb * nI);
    switch (v) {
      case 0: trmm_v<0><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 1: trmm_v<1><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 2: trmm_v<2><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 3: trmm_v<3><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 4: trmm_v<4><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 5: trmm_v<5><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 6: trmm_v<6><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 7: trmm_v<7><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      default: trmm_v<8><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
    }
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  run(0, ss0);
  CK(hipDeviceSynchronize());
  std::vector<double> ref((size_t)nI * C), got((size_t)nI * C);
  CK(hipMemcpy(ref.data(), ss0, ref.size() * 8, hipMemcpyDeviceToHost));
  for (int v = 1; v < NV; ++v) {
    CK(hipMemset(ss1, 0, (size_t)nI * C * 8));
    run(v, ss1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), ss1, got.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0, first = 0;
    for (size_t q = 0; q < ref.size(); ++q)
      if (ref[q] != got[q] && bad++ == 0) first = q;
    printf("%-20s bitwise mismatches vs S0: %zu (first at %zu: %.17g vs %.17g)\n", names[v], bad, first, ref[first],
           got[first]);
  }
  const double flops = (double)n * n * C;
  std::vector<std::vector<float>> t(NV);
  for (int rep = 0; rep < 10; ++rep)
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
    printf("%-20s median %.3f ms min %.3f ms -> %.2f TF/s (frac %.4f)\n", names[v], med, t[v][0],
           flops / (med * 1e-3) / 1e12, flops / (med * 1e-3) / 78.6e12);
  }
  printf("TRMM ASM BENCH DONE\n");
  return 0;
}
