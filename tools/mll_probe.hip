// Probe: where does mll_grad_kernel's time go?  Interleaved timings (one process) of
//   p0  the W W^T tile product alone over the same (tile, k-chunk) grid, row-major operands (product layout)
//   p1  the same product from the transposed copy L^{-1} = W^T with k-major operands (the sweep's layout)
//   p2  the full product kernel mll_grad_kernel<8> (product + dK epilogue), kc = 512 and kc = npad
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//        -I../bayesianoptimizer_amd/csrc mll_probe.hip -o mll_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../bayesianoptimizer_amd/csrc/gpx_mll.hip"

namespace gpx {  // launch_mll is not used here; satisfy its timer references
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
using namespace gpx;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

template <bool KM>
__global__ void __launch_bounds__(WG) product_only(const double* __restrict__ W, int64_t ldw, int npad, int kc,
                                                   double* __restrict__ sink) {
  using Tile = MfmaTile<128, 128, 16, KM, KM>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  int I, J;
  tri_decode(blockIdx.x, I, J);
  const int i0 = I * 128, j0 = J * 128;
  const int kbeg = i0 + (int)blockIdx.y * kc;
  if (kbeg >= npad) return;
  const int kend = min(kbeg + kc, npad);
  Tile t;
  if (KM)
    t.run(W + i0, ldw, W + j0, ldw, kbeg, kend, smem);  // W here is the transposed copy: A(m,k) = Wt[k][i0+m]
  else
    t.run(W + (int64_t)i0 * ldw, ldw, W + (int64_t)j0 * ldw, ldw, kbeg, kend, smem);
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += t.acc[a][b][r];
  if (s == 12345.678) sink[blockIdx.x] = s;  // keep the product alive
}

int main() {
  const int n = 4096, npad = 4096, d = 8;
  const int T = npad / 128, tiles = T * (T + 1) / 2;
  double *W, *Wt, *X, *al, *part, *sink;
  CK(hipMalloc(&W, (size_t)n * n * 8));
  CK(hipMalloc(&Wt, (size_t)n * n * 8));
  CK(hipMalloc(&X, (size_t)n * d * 8));
  CK(hipMalloc(&al, (size_t)n * 8));
  CK(hipMalloc(&part, (size_t)tiles * 32 * GPX_MLL_NOUT * 8));
  CK(hipMalloc(&sink, (size_t)tiles * 8));
  {
    std::vector<double> h((size_t)n * n), ht((size_t)n * n);
    srand(1);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < n; ++k) {
        double v = (k >= i) ? (rand() / (double)RAND_MAX - 0.5) * 0.01 : 0.0;
        h[(size_t)i * n + k] = v;
        ht[(size_t)k * n + i] = v;
      }
    CK(hipMemcpy(W, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(Wt, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> x((size_t)n * d), a(n);
    for (auto& v : x) v = rand() / (double)RAND_MAX;
    for (auto& v : a) v = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(X, x.data(), x.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(al, a.data(), a.size() * 8, hipMemcpyHostToDevice));
  }
  gpx_kernel_params p{};
  p.kind = GPX_KERNEL_RBF;
  p.d = d;
  for (int k = 0; k < d; ++k) p.lengthscale[k] = 0.6;
  p.outputscale = 1.0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flops = (double)npad * npad * npad / 3.0;
  // kc sweep of the full kernel (product + epilogue) and of the product alone
  const int kcs[] = {384, 512, 768, 1024, 1536, 2048, 4096};
  for (int kc : kcs) {
    if (kc > npad) continue;
    const dim3 grid(tiles, (npad + kc - 1) / kc);
    float best[2] = {1e30f, 1e30f};
    for (int rep = 0; rep < 6; ++rep)
      for (int v = 0; v < 2; ++v) {
        auto go = [&] {
          if (v == 0) product_only<false><<<grid, WG>>>(W, npad, npad, kc, sink);
          else mll_grad_kernel<8><<<grid, WG>>>(p, n, npad, X, d, W, npad, al, 1, kc, part);
        };
        go();
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) go();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best[v] = std::min(best[v], ms / 5);
      }
    printf("kc=%5d units=%6d  product %.3f ms (%.1f TF/s)  full %.3f ms (%.1f TF/s)\n", kc, tiles * (int)grid.y,
           best[0], flops / (best[0] * 1e-3) / 1e12, best[1], flops / (best[1] * 1e-3) / 1e12);
  }
  return 0;
}
