// Trailing-update microbenchmark of the eager Cholesky (diagnostic; includes the shipped gpx_potrf.hip): for a step c,
// the average time of the step's trailing work (column c-1 applied to every 128x128 lower tile of columns >= c+1,
// K = 64) as
//   T0  the step kernel's trailing workgroups alone (the shipped combined kernel, first_wg = tbase),
//   T1  the same trailing_role in a kernel of its own (no panel / lookahead roles: the register budget of the role alone),
//   T2  128 x 64 half tiles in a kernel of their own (twice the workgroups, half the MFMA work each),
//   T3  the 128x128 tiles of T1 in a one-workgroup-per-CU grid, each workgroup walking tiles (persistent: a CU never
//       hosts two tiles at once),
//   T4 / T5  T1's tiles with no LDS: MFMA fragments loaded straight from the L panels, 1 / 3 k-steps ahead.
// (T2 and T3 measured slower and are no longer printed: profiles/r04_trail_bench.log.)
// 20 back-to-back launches each, after steps 0 .. c-1 ran once on a fresh RBF Gram matrix.  Results are not checked
// (every variant rewrites the same tiles in place); only time is reported.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        trail_bench.hip -o trail_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_internal.h"
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
trail_only_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s) {
  __shared__ __attribute__((aligned(16))) double lds[Tile128::LDS_DOUBLES];
  trailing_role(A, lda, c, nblk, s.k0, s.cfirst, (int)blockIdx.x, s.ntrail, s.xmap, lds);
}

__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
trail_persist_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s) {
  __shared__ __attribute__((aligned(16))) double lds[Tile128::LDS_DOUBLES];
  for (int t = (int)blockIdx.x; t < s.ntrail; t += gridDim.x) {
    trailing_role(A, lda, c, nblk, s.k0, s.cfirst, t, s.ntrail, s.xmap, lds);
    __syncthreads();
  }
}

using TileH = MfmaTile<2 * NB, NB, 16, false, false>;
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
trail_half_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s) {
  __shared__ __attribute__((aligned(16))) double lds[TileH::LDS_DOUBLES];
  const int m = nblk - s.cfirst;
  const int M = (m + 1) / 2;
  const int c0 = nblk - 2 * M;
  int I, J;
  trail_tile((int)blockIdx.x >> 1, s.ntrail, M, s.xmap, I, J);
  const int half = (int)blockIdx.x & 1;
  const int r0 = c0 + 2 * I, q0 = c0 + 2 * J + half;
  const double* Li = A + (int64_t)r0 * NB * lda + (int64_t)s.k0 * NB;
  const double* Lj = A + (int64_t)q0 * NB * lda + (int64_t)s.k0 * NB;
  double* C = A + (int64_t)r0 * NB * lda + (int64_t)q0 * NB;
  TileH tl;
  double cv[TileH::WN][4];
  auto load_group = [&](int i) {
#pragma unroll
    for (int j = 0; j < TileH::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[j][r] = C[(int64_t)TileH::row_of(i, r) * lda + TileH::col_of(j)];
  };
  tl.zero();
  tl.run_acc_peeled(Li, lda, Lj, lda, 0, (c - s.k0) * NB, lds, [&] { load_group(0); });
  const rsrc_t rc = buf_rsrc(C);
#pragma unroll
  for (int i = 0; i < TileH::WM; ++i) {
#pragma unroll
    for (int j = 0; j < TileH::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tl.acc[i][j][r] = cv[j][r] - tl.acc[i][j][r];
    if (i + 1 < TileH::WM) load_group(i + 1);
#pragma unroll
    for (int j = 0; j < TileH::WN; ++j) {
      const bool colok = q0 >= s.cfirst;
      const bool k01 = colok && r0 + (TileH::row_of(i, 0) >> 6) >= q0;
      const bool k23 = colok && r0 + (TileH::row_of(i, 2) >> 6) >= q0;
      store_block_pairs_sc1<TileH>(rc, lda, i, j, tl.acc[i][j], k01, k23);
    }
  }
}

// T4: no LDS.  Every wave loads its own MFMA fragments straight from the row-major L panels (lane (m, kq) reads
// L[row m][k + kq]: four lanes cover 32 contiguous bytes of a row, a 128-byte line serves four consecutive k-steps from
// the L1), PD k-steps ahead in a register ring; no barriers; the first C row group is loaded two k-steps before the end.
template <int PD>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
trail_direct_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s) {
  constexpr int NS = PD + 1, KSTEPS = NB / 4;  // K = 64 (eager)
  const int m = nblk - s.cfirst, M = (m + 1) / 2, c0 = nblk - 2 * M;
  int I, J;
  trail_tile((int)blockIdx.x, s.ntrail, M, s.xmap, I, J);
  const int r0 = c0 + 2 * I, q0 = c0 + 2 * J;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lm = lane & 15, kq = lane >> 4;
  const int wm0 = (w >> 1) * 64, wn0 = (w & 1) * 64;
  const double* pa = A + ((int64_t)r0 * NB + wm0 + lm) * lda + (int64_t)s.k0 * NB + kq;
  const double* pb = A + ((int64_t)q0 * NB + wn0 + lm) * lda + (int64_t)s.k0 * NB + kq;
  double* C = A + (int64_t)r0 * NB * lda + (int64_t)q0 * NB;
  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  double fa[NS][4], fb[NS][4];
  auto load = [&](int st, int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[st][i] = pa[(int64_t)16 * i * lda + 4 * ks];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[st][j] = pb[(int64_t)16 * j * lda + 4 * ks];
  };
  using T = Tile128;  // same accumulator layout (4 waves of 64 x 64)
  double cv[T::WN][4];
  auto load_group = [&](int i) {
#pragma unroll
    for (int j = 0; j < T::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[j][r] = C[(int64_t)T::row_of(i, r) * lda + T::col_of(j)];
  };
#pragma unroll
  for (int st = 0; st < PD; ++st) load(st, st);
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    if (ks + PD < KSTEPS) load((ks + PD) % NS, ks + PD);
    if (ks == KSTEPS - 2) load_group(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x4(fa[ks % NS][i], fb[ks % NS][j], acc[i][j]);
  }
  const rsrc_t rc = buf_rsrc(C);
#pragma unroll
  for (int i = 0; i < T::WM; ++i) {
#pragma unroll
    for (int j = 0; j < T::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = cv[j][r] - acc[i][j][r];
    if (i + 1 < T::WM) load_group(i + 1);
#pragma unroll
    for (int j = 0; j < T::WN; ++j) {
      const int cb = q0 + (T::col_of(j) >> 6);
      const bool colok = cb >= s.cfirst;
      const bool k01 = colok && r0 + (T::row_of(i, 0) >> 6) >= cb;
      const bool k23 = colok && r0 + (T::row_of(i, 2) >> 6) >= cb;
      store_block_pairs_sc1<T>(rc, lda, i, j, acc[i][j], k01, k23);
    }
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, nblk = n / 64;
  std::vector<double> h((size_t)n * n), X((size_t)n * 8);
  srand(7);
  for (auto& v : X) v = rand() / (double)RAND_MAX;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double r2 = 0.0;
      for (int k = 0; k < 8; ++k) { const double d = (X[i * 8 + k] - X[j * 8 + k]) / 0.579; r2 += d * d; }
      h[(size_t)i * n + j] = exp(-0.5 * r2) + (i == j ? 1e-4 : 0.0);
    }
  double *A, *A0, *Dinv;
  int* info;
  CK(hipMalloc(&A, (size_t)n * n * 8));
  CK(hipMalloc(&A0, (size_t)n * n * 8));
  CK(hipMalloc(&Dinv, (size_t)2 * nblk * 64 * 64 * 8));
  CK(hipMalloc(&info, 4));
  CK(hipMemcpy(A0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto plan = [&](int c) { return step_plan(c, nblk, 0, c > 0 ? c - 1 : 0, c >= 1, 1); };
  auto time_step = [&](int c, int v) {
    CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemset(info, 0, 4));
    for (int cc = 0; cc < c; ++cc) {
      const StepPlan s = plan(cc);
      potrf_step_kernel<0><<<s.tbase + s.ntrail, WG>>>(A, n, cc, nblk, s, Dinv, info, 0, 0, 0, PotrfFwd());
    }
    CK(hipDeviceSynchronize());
    const StepPlan s = plan(c);
    if (s.ntrail == 0) return 0.0f;
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) {
      if (v == 0)
        potrf_step_kernel<0><<<s.ntrail, WG>>>(A, n, c, nblk, s, Dinv, info, s.tbase, 0, 0, PotrfFwd());
      else if (v == 1)
        trail_only_kernel<<<s.ntrail, WG>>>(A, n, c, nblk, s);
      else if (v == 2)
        trail_half_kernel<<<2 * s.ntrail, WG>>>(A, n, c, nblk, s);
      else if (v == 3)
        trail_persist_kernel<<<s.ntrail < cus ? s.ntrail : cus, WG>>>(A, n, c, nblk, s);
      else if (v == 4)
        trail_direct_kernel<1><<<s.ntrail, WG>>>(A, n, c, nblk, s);
      else
        trail_direct_kernel<3><<<s.ntrail, WG>>>(A, n, c, nblk, s);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 50.0f;  // us per launch
  };
  printf("n=%d, %d CUs; us per launch (20 back-to-back)\n", n, cus);
  // T4 / T5 against T1 on one launch of step 10 (same MFMA order per accumulator: bit for bit)
  {
    const int c = 10;
    std::vector<double> r1((size_t)n * n), r4((size_t)n * n);
    for (int v : {1, 4, 5}) {
      CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
      CK(hipMemset(info, 0, 4));
      for (int cc = 0; cc < c; ++cc) {
        const StepPlan s = plan(cc);
        potrf_step_kernel<0><<<s.tbase + s.ntrail, WG>>>(A, n, cc, nblk, s, Dinv, info, 0, 0, 0, PotrfFwd());
      }
      const StepPlan s = plan(c);
      if (v == 1) trail_only_kernel<<<s.ntrail, WG>>>(A, n, c, nblk, s);
      else if (v == 4) trail_direct_kernel<1><<<s.ntrail, WG>>>(A, n, c, nblk, s);
      else trail_direct_kernel<3><<<s.ntrail, WG>>>(A, n, c, nblk, s);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(v == 1 ? r1.data() : r4.data(), A, r1.size() * 8, hipMemcpyDeviceToHost));
      if (v != 1) {
        size_t bad = 0;
        for (size_t q = 0; q < r1.size(); ++q) bad += r1[q] != r4[q];
        printf("T%d vs T1 after one launch of step %d: %zu bitwise mismatches\n", v, c, bad);
      }
    }
  }
  for (int c : {1, 3, 5, 10, 16, 20, 24, 30, 40}) {
    if (c >= nblk) continue;
    const StepPlan s = plan(c);
    const float t0 = time_step(c, 0), t1 = time_step(c, 1), t4 = time_step(c, 4), t5 = time_step(c, 5);
    printf("step %2d (%3d tiles, %6.3f GFLOP): T0 step kernel %6.2f  T1 own kernel %6.2f  T4 direct PD=1 %6.2f  T5 direct PD=3 %6.2f\n",
           c, s.ntrail, s.ntrail * 2.0 * 128 * 128 * 64 / 1e9, t0, t1, t4, t5);
  }
  printf("TRAIL BENCH DONE\n");
  return 0;
}
