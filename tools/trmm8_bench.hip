// Probe: the sweep product V = W^T K* (column sums of V^2) with 8 waves per 128x128 tile (2 x 4 waves of 64 x 32, acc 64
// VGPRs, up to 4 waves per SIMD at two workgroups per CU) against the shipped 4-wave tile (64 x 64 per wave, 2 waves
// per SIMD), alternating launches in one process.  Diagnostic; not part of libgpx.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_device.h"

using namespace gpx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int T = 128;

// 128 x 128 tile, NT = 64 * WMW * WNW threads, each wave (T / WMW) x (T / WNW); k-major operands staged through LDS
// (rows padded by 16 doubles), double-buffered with one barrier per k-tile, fragments register double-buffered.
template <int WMW, int WNW, int BK>
struct TileW {
  static constexpr int NT = 64 * WMW * WNW;
  static constexpr int WR = T / WMW, WC = T / WNW;   // wave sub-tile
  static constexpr int WM = WR / 16, WN = WC / 16;   // MFMA blocks per wave
  static constexpr int PA = T + 16, PB = T + 16;
  static constexpr int LDS_DOUBLES = 2 * BK * (PA + PB);
  static constexpr int LOADS = T * BK / (2 * NT);
  d4 acc[WM][WN];
  double2 ra[LOADS], rb[LOADS];
  __device__ __forceinline__ void load_regs(const double* A, int64_t lda, const double* B, int64_t ldb, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < LOADS; ++q) {
      const int e = (t + q * NT) * 2, kk = e / T, mm = e % T;
      ra[q] = *reinterpret_cast<const double2*>(A + (int64_t)(k0 + kk) * lda + mm);
      rb[q] = *reinterpret_cast<const double2*>(B + (int64_t)(k0 + kk) * ldb + mm);
    }
  }
  __device__ __forceinline__ void store_lds(double* sA, double* sB) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < LOADS; ++q) {
      const int e = (t + q * NT) * 2, kk = e / T, mm = e % T;
      *reinterpret_cast<double2*>(sA + kk * PA + mm) = ra[q];
      *reinterpret_cast<double2*>(sB + kk * PB + mm) = rb[q];
    }
  }
  __device__ __forceinline__ void frag(const double* sA, const double* sB, int ks, double* a, double* b) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm0 = (w / WNW) * WR, wn0 = (w % WNW) * WC, kr = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int i = 0; i < WM; ++i) a[i] = sA[(ks + kr) * PA + wm0 + 16 * i + cl];
#pragma unroll
    for (int j = 0; j < WN; ++j) b[j] = sB[(ks + kr) * PB + wn0 + 16 * j + cl];
  }
  __device__ __forceinline__ void mm(const double* a, const double* b) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = mfma16x16x4(a[i], b[j], acc[i][j]);
  }
  __device__ __forceinline__ void compute(const double* sA, const double* sB) {
    double a0[WM], b0[WN], a1[WM], b1[WN];
    frag(sA, sB, 0, a0, b0);
#pragma unroll
    for (int ks = 0; ks < BK; ks += 8) {
      frag(sA, sB, ks + 4, a1, b1);
      mm(a0, b0);
      if (ks + 8 < BK) frag(sA, sB, ks + 8, a0, b0);
      mm(a1, b1);
    }
  }
  __device__ __forceinline__ void run(const double* A, int64_t lda, const double* B, int64_t ldb, int kend,
                                      double* smem) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
    double* cur = smem;
    double* nxt = smem + BK * (PA + PB);
    load_regs(A, lda, B, ldb, 0);
    store_lds(cur, cur + BK * PA);
    __syncthreads();
    for (int k0 = 0; k0 < kend; k0 += BK) {
      const bool more = (k0 + BK) < kend;
      if (more) load_regs(A, lda, B, ldb, k0 + BK);
      compute(cur, cur + BK * PA);
      if (more) store_lds(nxt, nxt + BK * PA);
      __syncthreads();
      double* tt = cur;
      cur = nxt;
      nxt = tt;
    }
  }
};

// column sums of squares of the tile: per wave over its rows, then the WMW row groups through LDS
template <typename Tl>
__device__ __forceinline__ void sumsq(Tl& tile, double* smem, double* out) {
  constexpr int WNW = T / Tl::WC, WMW = T / Tl::WR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w / WNW, wc = w % WNW;
  double s[Tl::WN];
#pragma unroll
  for (int j = 0; j < Tl::WN; ++j) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < Tl::WM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += tile.acc[i][j][r] * tile.acc[i][j][r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    s[j] = v;
  }
  __syncthreads();
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < Tl::WN; ++j) smem[wr * T + wc * Tl::WC + 16 * j + lane] = s[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < T; c += Tl::NT) {
    double v = 0.0;
    for (int r = 0; r < WMW; ++r) v += smem[r * T + c];
    out[c] = v;
  }
}

template <int WMW, int WNW, int WPE>
__global__ void __launch_bounds__(64 * WMW * WNW) __attribute__((amdgpu_waves_per_eu(WPE)))
trmm_w(const double* W, int64_t ldw, const double* K, int64_t C, int nI, double* ss) {
  using Tl = TileW<WMW, WNW, 16>;
  __shared__ __attribute__((aligned(16))) double smem[Tl::LDS_DOUBLES];
  const int ncb = (int)(C / T);
  const int b = blockIdx.x;
  const int x = b & 7, l = b >> 3, per = ncb >> 3;  // the shipped XCD-aware heavy-first order
  const int I = nI - 1 - l / per, cb = 8 * (l % per) + x;
  Tl tile;
  tile.run(W + (int64_t)I * T, ldw, K + (int64_t)cb * T, C, (I + 1) * T, smem);
  sumsq(tile, smem, ss + (int64_t)I * C + (int64_t)cb * T);
}

int main() {
  const int n = 4096, nI = n / T;
  const int C = 32768;
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
  const int grid = (C / T) * nI;
  auto run = [&](int which) {
    if (which == 0) trmm_w<2, 2, 2><<<grid, 256>>>(W, n, K, C, nI, ss0);  // shipped shape: 4 waves of 64 x 64
    if (which == 1) trmm_w<2, 4, 4><<<grid, 512>>>(W, n, K, C, nI, ss1);  // 8 waves of 64 x 32
    if (which == 2) trmm_w<4, 2, 4><<<grid, 512>>>(W, n, K, C, nI, ss1);  // 8 waves of 32 x 64
    if (which == 3) trmm_w<2, 2, 2><<<grid, 256>>>(W, n, K, C, nI, ss1);  // shipped shape again
    if (which == 4) trmm_w<4, 4, 8><<<grid, 1024>>>(W, n, K, C, nI, ss1);  // 16 waves of 32 x 32
  };
  const char* names[] = {"4 waves 64x64 (old shape)", "8 waves 64x32", "8 waves 32x64", "4 waves again",
                         "16 waves 32x32"};
  const int NV = 5;
  const double flops = (double)n * n * C;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < NV; ++w) run(w);
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> t(NV);
  for (int rep = 0; rep < 5; ++rep)
    for (int w = 0; w < NV; ++w) {
      CK(hipEventRecord(e0));
      run(w);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[w].push_back(ms);
      if (w > 0 && rep == 0) {
        std::vector<double> a((size_t)nI * C), b((size_t)nI * C);
        CK(hipMemcpy(a.data(), ss0, a.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), ss1, b.size() * 8, hipMemcpyDeviceToHost));
        double md = 0;
        for (size_t q = 0; q < a.size(); ++q) md = std::max(md, std::fabs(a[q] - b[q]) / (std::fabs(a[q]) + 1e-300));
        printf("  %s: max rel diff vs shipped shape %.3e\n", names[w], md);
      }
    }
  for (int w = 0; w < NV; ++w) {
    std::sort(t[w].begin(), t[w].end());
    printf("C=%d %-30s median %.3f ms min %.3f ms -> %.2f TF/s\n", C, names[w], t[w][t[w].size() / 2], t[w][0],
           flops / (t[w][t[w].size() / 2] * 1e-3) / 1e12);
  }
  printf("TRMM8 BENCH DONE\n");
  return 0;
}
