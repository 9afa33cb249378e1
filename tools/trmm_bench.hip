// Microbenchmark of trmm_sumsq variants (V = W^T K*, column sums of V^2), interleaved in one process
// (cdna_hip_programming.md §5.4 rule 24).  W: random upper-triangular n x n, K*: random n x C.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>
#include "gpx_device.h"

using namespace gpx;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

constexpr int T128 = 128;

// Single-body k loop: current/next LDS buffers are swapped pointers instead of two duplicated branches.
template <int TM, int TN, int BK, bool AK, bool BKM>
struct Tile2 : public MfmaTile<TM, TN, BK, AK, BKM> {
  using Base = MfmaTile<TM, TN, BK, AK, BKM>;
  __device__ __forceinline__ void run(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                      int64_t ldb, int kbeg, int kend, double* smem) {
    this->zero();
    if (kend <= kbeg) return;
    double* cur = smem;
    double* nxt = smem + BK * (Base::PA + Base::PB);
    this->load_regs(A, lda, B, ldb, kbeg);
    this->store_lds(cur, cur + BK * Base::PA);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      const bool more = (k0 + BK) < kend;
      if (more) this->load_regs(A, lda, B, ldb, k0 + BK);
      this->compute(cur, cur + BK * Base::PA);
      if (more) this->store_lds(nxt, nxt + BK * Base::PA);
      __syncthreads();
      double* t = cur; cur = nxt; nxt = t;
    }
  }
};

template <class Tile>
__device__ __forceinline__ void sumsq_epilogue(Tile& tile, double* smem, double* out) {
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
    for (int j = 0; j < Tile::WN; ++j) out[Tile::col_of(j)] = s[j] + smem[Tile::col_of(j)];
  }
  __syncthreads();
}

// V0: the shipped kernel (heavy-first row tiles)
template <int BK>
__global__ void __launch_bounds__(WG) v0(const double* W, int64_t ldw, const double* K, int64_t C, int nI, double* ss) {
  using Tile = MfmaTile<T128, T128, BK, true, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  const int I = nI - 1 - blockIdx.y, cb = blockIdx.x;
  Tile tile;
  tile.run(W + (int64_t)I * T128, ldw, K + (int64_t)cb * T128, C, 0, (I + 1) * T128, smem);
  sumsq_epilogue(tile, smem, ss + (int64_t)I * C + (int64_t)cb * T128);
}

// V2: single-body tile core
template <int BK, int MINW>
__global__ void __launch_bounds__(WG, MINW) v2(const double* W, int64_t ldw, const double* K, int64_t C, int nI, double* ss) {
  using Tile = Tile2<T128, T128, BK, true, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  const int I = nI - 1 - blockIdx.y, cb = blockIdx.x;
  Tile tile;
  tile.run(W + (int64_t)I * T128, ldw, K + (int64_t)cb * T128, C, 0, (I + 1) * T128, smem);
  sumsq_epilogue(tile, smem, ss + (int64_t)I * C + (int64_t)cb * T128);
}

// V1: equal-work pairs (I, nI-1-I) per workgroup; optional XCD-aware remap so the 16 pair-WGs of a candidate
// tile share one XCD's L2.
template <int BK, bool XCD>
__global__ void __launch_bounds__(WG) v1(const double* W, int64_t ldw, const double* K, int64_t C, int nI, double* ss) {
  using Tile = MfmaTile<T128, T128, BK, true, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  const int npair = nI / 2;
  const int ncb = (int)(C / T128);
  int b = blockIdx.x;
  int p, cb;
  if (XCD) {
    const int x = b & 7, l = b >> 3;
    cb = 8 * (l / npair) + x;
    p = l % npair;
  } else {
    p = b % npair;
    cb = b / npair;
  }
  if (cb >= ncb) return;
  for (int h = 0; h < 2; ++h) {
    const int I = h == 0 ? (nI - 1 - p) : p;
    Tile tile;
    tile.run(W + (int64_t)I * T128, ldw, K + (int64_t)cb * T128, C, 0, (I + 1) * T128, smem);
    sumsq_epilogue(tile, smem, ss + (int64_t)I * C + (int64_t)cb * T128);
  }
}

int main(int argc, char** argv) {
  const int n = 4096;
  std::vector<int> Cs = {4096, 8192};
  const int nI = n / T128;
  double *W, *K, *ss0, *ss1;
  size_t Cmax = 8192;
  CK(hipMalloc(&W, (size_t)n * n * 8));
  CK(hipMalloc(&K, (size_t)n * Cmax * 8));
  CK(hipMalloc(&ss0, (size_t)nI * Cmax * 8));
  CK(hipMalloc(&ss1, (size_t)nI * Cmax * 8));
  {
    std::vector<double> h((size_t)n * n);
    srand(1);
    for (int k = 0; k < n; ++k)
      for (int i = 0; i < n; ++i) h[(size_t)k * n + i] = (k <= i) ? (rand() / (double)RAND_MAX - 0.5) : 0.0;
    CK(hipMemcpy(W, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> g((size_t)n * Cmax);
    for (auto& v : g) v = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(K, g.data(), g.size() * 8, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int C : Cs) {
    const double flops = (double)n * n * C;
    auto run = [&](int which) {
      const int ncb = C / T128;
      if (which == 0) v0<16><<<dim3(ncb, nI), WG>>>(W, n, K, C, nI, ss0);
      if (which == 1) v1<16, false><<<ncb * nI / 2, WG>>>(W, n, K, C, nI, ss1);
      if (which == 2) v1<16, true><<<ncb * nI / 2, WG>>>(W, n, K, C, nI, ss1);
      if (which == 3) v2<16, 1><<<dim3(ncb, nI), WG>>>(W, n, K, C, nI, ss1);
      if (which == 4) v2<16, 2><<<dim3(ncb, nI), WG>>>(W, n, K, C, nI, ss1);
      if (which == 5) v2<32, 1><<<dim3(ncb, nI), WG>>>(W, n, K, C, nI, ss1);
    };
    const char* names[] = {"v0 heavy-first BK16", "v1 pairs BK16", "v1 pairs+xcd BK16", "v2 single BK16", "v2 single BK16 lb2", "v2 single BK32"};
    const int NV = 6;
    std::vector<std::vector<float>> t(NV);
    for (int w = 0; w < NV; ++w) run(w);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 6; ++rep)
      for (int w = 0; w < NV; ++w) {
        CK(hipEventRecord(e0));
        run(w);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[w].push_back(ms);
        if (w > 0) {  // correctness vs v0
          std::vector<double> a((size_t)nI * C), b((size_t)nI * C);
          CK(hipMemcpy(a.data(), ss0, a.size() * 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(b.data(), ss1, b.size() * 8, hipMemcpyDeviceToHost));
          double md = 0;
          for (size_t q = 0; q < a.size(); ++q) md = std::max(md, std::fabs(a[q] - b[q]) / (std::fabs(a[q]) + 1e-300));
          if (md > 1e-12 && rep == 0) printf("  MISMATCH %s: max rel %.3e\n", names[w], md);
        }
      }
    for (int w = 0; w < NV; ++w) {
      std::sort(t[w].begin(), t[w].end());
      printf("C=%d %-22s median %.3f ms min %.3f ms -> %.2f TF/s\n", C, names[w], t[w][t[w].size() / 2], t[w][0],
             flops / (t[w][t[w].size() / 2] * 1e-3) / 1e12);
    }
  }
  printf("TRMM BENCH DONE\n");
  return 0;
}
