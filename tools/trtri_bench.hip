// The triangular inverse's largest level at n = 16384 (h = 128 blocks: T = L21^T W22, W12 = -W11 T, 8192-square
// operands with one triangular factor) under two block orders (diagnostic; includes the shipped gpx_trtri.hip):
//   0  the paired-tile order shipped until round 4 (column pair cb, nt2-1-cb per workgroup, grid in (pair, row) order)
//   1  the library's order since round 4 (gpx_trtri.hip trtri_order): one tile per workgroup, heaviest k-range first,
//      XCD-aware (the sweep product's order, gpx_sweep.hip): the 8 workgroups b..b+7 that the round-robin dispatch
//      spreads over the 8 XCDs take the same heavy index and free tiles f = x (mod 8), so each XCD walks 8 free panels
// The tiles' MFMA order is the same in both, so T and W12 must match bit for bit.  Prints ms and TF/s (useful flops:
// 2 * 8192^3 / 2 per product) per variant, median of 7, alternating.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        trtri_bench.hip -o trtri_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_internal.h"
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_trtri.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int TS = 128;

// variant 0: the earlier paired-tile kernels (as shipped until round 4)
template <int TS>
__global__ void __launch_bounds__(WG) paired_t_kernel(const double* __restrict__ L, int64_t ldl,
                                                     const double* __restrict__ W, int64_t ldw,
                                                     double* __restrict__ T, int h, int nblk, int groups, int64_t sl,
                                                     int64_t sw, int64_t st) {
  using Tile = MfmaTile<TS, TS, 16, true, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  const int p = blockIdx.z % groups, prob = blockIdx.z / groups;
  L += prob * sl;
  W += prob * sw;
  T += prob * st;
  const int s1 = p * 2 * h, s2 = s1 + h;
  const int nb2 = min(2 * h, nblk - s1) - h;
  const int b1 = h * NB, b2 = nb2 * NB;
  const int nt2 = b2 / TS;
  const int rb = blockIdx.y;
  if (nb2 <= 0 || (int)blockIdx.x >= (nt2 + 1) / 2) return;
  const int64_t off1 = (int64_t)s1 * NB, off2 = (int64_t)s2 * NB;
  // T_p is b1 x b2 with row length b2; every group before the last is full (b2 = b1), so group p starts at
  // p*b1*b1 and the level's total sum_p b1*b2_p <= b1*(npad-b1) <= npad^2/4 fits the workspace.
  double* Tp = T + (int64_t)p * b1 * b1;
  for (int pass = 0; pass < 2; ++pass) {
    const int cb = pass == 0 ? (int)blockIdx.x : nt2 - 1 - (int)blockIdx.x;
    if (pass == 1 && cb == (int)blockIdx.x) break;
    const double* Ab = L + off2 * ldl + off1 + rb * TS;   // A(m=r,k=q) = L[off2+q][off1+r]
    const double* Bb = W + off2 * ldw + off2 + cb * TS;   // B(k=q,n=c) = W[off2+q][off2+c]
    Tile tile;
    tile.run(Ab, ldl, Bb, ldw, 0, (cb + 1) * TS, smem);
#pragma unroll
    for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
      for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Tp[(int64_t)(rb * TS + Tile::row_of(i, r)) * b2 + cb * TS + Tile::col_of(j)] = tile.acc[i][j][r];
  }
}

// W12 = -W11 T_p.  The k-range of tile (rb, cb) is [rb * TS, b1) (W11 upper): one workgroup takes the row pair
// rb and nt1 - 1 - rb (same balancing as trtri_t_kernel).
template <int TS>
__global__ void __launch_bounds__(WG) paired_w_kernel(double* __restrict__ W, int64_t ldw, const double* __restrict__ T,
                                                     int h, int nblk, int groups, int64_t sw, int64_t st) {
  using Tile = MfmaTile<TS, TS, 16, false, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  const int p = blockIdx.z % groups, prob = blockIdx.z / groups;
  W += prob * sw;
  T += prob * st;
  const int s1 = p * 2 * h, s2 = s1 + h;
  const int nb2 = min(2 * h, nblk - s1) - h;
  const int b1 = h * NB, b2 = nb2 * NB;
  const int nt1 = b1 / TS, nt2 = b2 / TS;
  const int cb = blockIdx.x;
  if (nb2 <= 0 || cb >= nt2 || (int)blockIdx.y >= (nt1 + 1) / 2) return;
  const int64_t off1 = (int64_t)s1 * NB, off2 = (int64_t)s2 * NB;
  const double* Bb = T + (int64_t)p * b1 * b1 + cb * TS;          // B(k=q,n=c) = T[q][c], row length b2
  for (int pass = 0; pass < 2; ++pass) {
    const int rb = pass == 0 ? (int)blockIdx.y : nt1 - 1 - (int)blockIdx.y;
    if (pass == 1 && rb == (int)blockIdx.y) break;
    const double* Ab = W + (off1 + rb * TS) * ldw + off1;           // A(m=r,k=q) = W[off1+r][off1+q]
    Tile tile;
    tile.run(Ab, ldw, Bb, b2, rb * TS, b1, smem);
    double* Wo = W + (off1 + rb * TS) * ldw + off2 + cb * TS;
#pragma unroll
    for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
      for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Wo[(int64_t)Tile::row_of(i, r) * ldw + Tile::col_of(j)] = -tile.acc[i][j][r];
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384, nblk = n / NB, h = nblk / 2, h128 = h / 2;
  const size_t nn = (size_t)n * n;
  std::vector<double> hL(nn, 0.0);
  srand(5);
  for (size_t i = 0; i < nn; ++i) hL[i] = (double)rand() / RAND_MAX - 0.5;
  double *L, *W, *W0, *T, *T2;
  CK(hipMalloc(&L, nn * 8));
  CK(hipMalloc(&W, nn * 8));
  CK(hipMalloc(&W0, nn * 8));
  CK(hipMalloc(&T, nn / 4 * 8));
  CK(hipMalloc(&T2, nn / 4 * 8));
  CK(hipMemcpy(L, hL.data(), nn * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(W0, hL.data(), nn * 8, hipMemcpyHostToDevice));  // any values: timing + bitwise comparison only
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int b2 = (nblk - h) * NB, nt1 = h * NB / TS, nt2 = b2 / TS;
  auto launch_t = [&](int v, double* To) {
    if (v == 0)
      paired_t_kernel<TS><<<dim3((h128 + 1) / 2, h128, 1), WG>>>(L, n, W, n, To, h, nblk, 1, 0, 0, 0);
    else
      trtri_t_kernel<TS, false><<<nt1 * nt2, WG>>>(L, n, W, n, To, h, nblk, 1, 0, 0, 0);
  };
  auto launch_w = [&](int v) {
    if (v == 0)
      paired_w_kernel<TS><<<dim3(h128, (h128 + 1) / 2, 1), WG>>>(W, n, T, h, nblk, 1, 0, 0);
    else
      trtri_w_kernel<TS, false><<<nt1 * nt2, WG>>>(W, n, T, h, nblk, 1, 0, 0);
  };
  auto timed = [&](auto&& f) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  // correctness: T of both variants, then W12 of both from the same T
  std::vector<double> a(nn / 4), b(nn / 4);
  CK(hipMemcpy(W, W0, nn * 8, hipMemcpyDeviceToDevice));
  timed([&] { launch_t(0, T); });
  timed([&] { launch_t(1, T2); });
  CK(hipMemcpy(a.data(), T, nn / 4 * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), T2, nn / 4 * 8, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < nn / 4; ++i) bad += a[i] != b[i];
  printf("T: bitwise mismatches variant 1 vs 0: %zu\n", bad);
  std::vector<double> wa(nn), wb(nn);
  timed([&] { launch_w(0); });
  CK(hipMemcpy(wa.data(), W, nn * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(W, W0, nn * 8, hipMemcpyDeviceToDevice));
  timed([&] { launch_w(1); });
  CK(hipMemcpy(wb.data(), W, nn * 8, hipMemcpyDeviceToHost));
  bad = 0;
  for (size_t i = 0; i < nn; ++i) bad += wa[i] != wb[i];
  printf("W: bitwise mismatches variant 1 vs 0: %zu\n", bad);
  const double flops = (double)nt1 * TS * (double)b2 * (double)b2;  // 2 * b1 * b2^2 / 2
  std::vector<float> tt[2], tw[2];
  for (int r = 0; r < 7; ++r)
    for (int v = 0; v < 2; ++v) {
      tt[v].push_back(timed([&] { launch_t(v, T); }));
      tw[v].push_back(timed([&] { launch_w(v); }));
    }
  for (int v = 0; v < 2; ++v) {
    std::sort(tt[v].begin(), tt[v].end());
    std::sort(tw[v].begin(), tw[v].end());
    printf("variant %d: T %.3f ms (%.1f TF/s)  W %.3f ms (%.1f TF/s)\n", v, tt[v][3], flops / (tt[v][3] * 1e-3) * 1e-12,
           tw[v][3], flops / (tw[v][3] * 1e-3) * 1e-12);
  }
  printf("TRTRI BENCH DONE\n");
  return 0;
}
