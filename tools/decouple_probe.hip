// Decoupled trailing update experiment (diagnostic; includes the shipped gpx_potrf.hip).  The eager n = 4096 schedule
// with each launch's trailing workgroups restricted to the NEAR 128-tile columns (q0 - c < D) while a persistent side
// kernel on a second stream applies the earlier columns to the FAR tiles as the panels publish them (done / ver sync
// words, bounded polls).  (1) the step launches alone with the far tiles skipped (an upper bound: the factor is not
// valid for D < nblk; D = 1000 is the full update in column-major tile order), (2) the side kernel alone with every
// column published up front (its throughput), (3) the decoupled schedule with an event after every launch.
// Result (profiles/r04_decouple_probe.log): (1) 1.04 ms vs 1.46, but (2) the side kernel reaches only 24-27 TF/s (the
// largest far tile's 58 columns are ~0.7 ms of one workgroup's serial work) and in (3) the shared CUs slow the panel
// chain: 2.42-2.49 ms, so the library does not ship it.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        decouple_probe.hip -o decouple_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "gpx_internal.h"
namespace gpx {  // timers are no-ops in this harness
LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {}
LaunchTimer::~LaunchTimer() {}
}  // namespace gpx
#include "gpx_potrf.hip"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// ---- the decoupled trailing update (the experiment; measured slower) ---------------------------------
// The flush of launch c covers only the NEAR 128-tile columns (origin q0 - c < D); a persistent side kernel on a
// second stream applies every earlier column to the FAR tiles as soon as the panels have published it, so the step
// launches on the critical path stop paying for the bulk of the trailing matrix.  Tile (r0, q0) becomes near at
// launch cn = q0 - D + 1: the side kernel owns its columns 0 .. cn - 2 (in SIDE_CHUNK-column products), the step
// launches cn, cn+1, ... one column each.  The chunking is fixed, so the factor is deterministic; it differs from the
// eager schedule's (one column per product everywhere) by rounding only.
// Sync words (zeroed on the stream before the factorisation): done[k], k < nblk = rows of column k the panel
// workgroups of launch k have stored (complete at (nblk - 1 - k) * 64); ver[(r0/2) * (nblk/2) + q0/2] = the columns the
// side kernel has applied to the tile.  Producers: write-through stores, s_waitcnt vmcnt(0), barrier, one relaxed
// agent-scope atomic (cdna_hip_programming.md §6, form R1); consumers: one lane polls, acquires, then the barrier.
constexpr int SIDE_CHUNK = 8;  // columns per side-kernel pass over a tile (K = 512)

// one lane: bounded poll until *w >= v; false on timeout or when the factorisation was aborted (info != 0)
__device__ __forceinline__ bool poll_at_least(int32_t* w, int32_t v, int32_t* info, unsigned limit) {
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v) break;
    if (spins >= limit ||
        ((spins & 63) == 63 && __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0))
      return false;
    __builtin_amdgcn_s_sleep(2);
  }
  (void)__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Near trailing workgroup `p` of launch c (tile columns in order, rows within a column): a tile that becomes near at
// this launch first waits for the side kernel's columns.
struct DPlan {
  StepPlan s;      // panels as the library's eager schedule; s.ntrail = the near tiles
  int near;        // D
  int32_t* sync;   // done[nblk], then ver[(nblk/2)^2]
  unsigned limit;
};

__device__ __forceinline__ void near_role(double* __restrict__ A, int64_t lda, int c, int nblk, const DPlan& d, int p,
                                          int32_t* __restrict__ info, double* lds) {
  const StepPlan& s = d.s;
  __shared__ int s_ok;
  const int M = (nblk - s.cfirst + 1) / 2, c0 = nblk - 2 * M;
  int J = 0;
  while (p >= M - J) {
    p -= M - J;
    ++J;
  }
  const int r0 = c0 + 2 * (J + p), q0 = c0 + 2 * J, cn = q0 - d.near + 1;
  if (c == cn && cn >= 2) {
    if (threadIdx.x == 0) {
      s_ok = poll_at_least(d.sync + nblk + (r0 >> 1) * (nblk >> 1) + (q0 >> 1), cn - 1, info, d.limit);
      if (!s_ok) atomicCAS(info, 0, (int32_t)GPX_INFO_TIMEOUT);
    }
    __syncthreads();
    if (!s_ok) return;
  }
  trailing_tile_at<2 * NB>(A, lda, c, s.k0, s.cfirst, r0, q0, lds);
}

// The far tiles (q0 >= D + 1, in q0 order, dealt round-robin to the workgroups; one workgroup per CU): pass after pass,
// the next SIDE_CHUNK columns of every owned tile, each once the panels have published its last column.
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
potrf_side_kernel(double* __restrict__ A, int64_t lda, int nblk, int D, int32_t* __restrict__ sync,
                  int32_t* __restrict__ info, unsigned limit) {
  __shared__ __attribute__((aligned(16))) double lds[Tile128::LDS_DOUBLES];
  __shared__ int s_ok;
  const int qmin = (D + 2) & ~1;  // the smallest even q0 >= D + 1
  int ntile = 0;
  for (int q0 = qmin; q0 < nblk; q0 += 2) ntile += (nblk - q0) >> 1;
#pragma unroll 1
  for (int kb = 0;; kb += SIDE_CHUNK) {
    bool any = false;
#pragma unroll 1
    for (int tix = blockIdx.x; tix < ntile; tix += gridDim.x) {
      int q0 = qmin, rem = tix;
      while (rem >= (nblk - q0) >> 1) {
        rem -= (nblk - q0) >> 1;
        q0 += 2;
      }
      const int r0 = q0 + 2 * rem, kend = q0 - D;  // this kernel's columns: 0 .. kend - 1
      if (kb >= kend) continue;
      any = true;
      const int ke = min(kb + SIDE_CHUNK, kend);
      if (threadIdx.x == 0) {
        s_ok = poll_at_least(sync + ke - 1, (nblk - ke) * NB, info, limit);
        if (!s_ok) atomicCAS(info, 0, (int32_t)GPX_INFO_TIMEOUT);
      }
      __syncthreads();
      if (!s_ok) return;
      // (A and lda opaque per tile: the tile's address arithmetic is not hoisted out of these loops, whose live-through
      // values the 128x128 accumulators leave no registers for; what still spills is saved once per kernel and
      // reloaded once per tile, one reload per k-tile of 64 MFMAs)
      double* At = A;
      int64_t ldt = lda;
      asm volatile("" : "+s"(At), "+s"(ldt));
      trailing_tile_at<2 * NB>(At, ldt, ke, kb, 0, r0, q0, lds);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_store(sync + nblk + (r0 >> 1) * (nblk >> 1) + (q0 >> 1), ke, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!any) return;
  }
}

// launch c of the decoupled schedule: the library's panels (which then publish their rows in done[c]) and the near tiles
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
dec_step_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, DPlan d, double* __restrict__ Dinv,
                int32_t* __restrict__ info) {
  if (*(volatile int32_t*)info != 0) return;
  __shared__ __attribute__((aligned(16))) double lds[STEP_LDS];
  const StepPlan& s = d.s;
  const int b = (int)blockIdx.x;
  if (b < s.npanel) {
    if (s.split == 2 && b > 0)
      panel_role<0, 2>(A, lda, c, 1 + ((b - 1) >> 1), (b - 1) & 1, nblk, s.c0, Dinv, info, lds, PotrfFwd(), s.overlap);
    else
      panel_role<0, 1>(A, lda, c, b, 0, nblk, s.c0, Dinv, info, lds, PotrfFwd(), s.overlap);
    if (b > 0) {  // L_ic stored write-through: drain, barrier, publish the rows
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(d.sync + c, s.split == 2 ? NB / 2 : NB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (b < s.tbase) return;
  near_role(A, lda, c, nblk, d, b - s.tbase, info, lds);
}

// the plan: the eager launch, its trailing grid cut to the near tile columns, the panel split decided for that grid
inline DPlan dplan(int c, int nblk, int slots, int D, int32_t* sync) {
  DPlan d;
  d.s = step_plan(c, nblk, 0, c > 0 ? c - 1 : 0, c >= 1, 1, 0);
  d.near = D;
  d.sync = sync;
  d.limit = 1u << 22;
  StepPlan& s = d.s;
  const int M = (nblk - s.cfirst + 1) / 2;
  s.ntrail = 0;
  if (c >= 1)
    for (int J = 0; J < M && nblk - 2 * M + 2 * J - c < D; ++J) s.ntrail += M - J;
  if (slots > 0 && s.npanel > 1) {
    const int np = 1 + 2 * (s.npanel - 1);
    if (((np + 7) & ~7) + s.ntrail <= slots) {
      s.split = 2;
      s.npanel = np;
    }
  }
  s.tbase = (s.npanel + 7) & ~7;
  return d;
}

// launch c: panels exactly as the library's step kernel; trailing workgroups b - tbase -> near tile (column-major)
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
near_step_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s, double* __restrict__ Dinv,
                 int32_t* __restrict__ info, int D) {
  __shared__ __attribute__((aligned(16))) double lds[STEP_LDS];
  const int b = (int)blockIdx.x;
  if (b < s.npanel) {
    if (s.split == 2 && b > 0)
      panel_role<0, 2>(A, lda, c, 1 + ((b - 1) >> 1), (b - 1) & 1, nblk, s.c0, Dinv, info, lds, PotrfFwd(), s.overlap);
    else
      panel_role<0, 1>(A, lda, c, b, 0, nblk, s.c0, Dinv, info, lds, PotrfFwd(), s.overlap);
    return;
  }
  if (b < s.tbase) return;
  const int M = (nblk - s.cfirst + 1) / 2, c0 = nblk - 2 * M;
  int p = b - s.tbase;
  for (int J = 0; J < M; ++J) {
    if (c0 + 2 * J - c >= D) return;
    if (p < M - J) {
      trailing_tile_at<2 * NB>(A, lda, c, s.k0, s.cfirst, c0 + 2 * (J + p), c0 + 2 * J, lds);
      return;
    }
    p -= M - J;
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
  auto run = [&](int D, bool lib) {
    CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
    CK(hipMemset(info, 0, 4));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int c = 0; c < nblk; ++c) {
      const StepPlan s = step_plan(c, nblk, 0, c > 0 ? c - 1 : 0, c >= 1, 1, 2 * cus);
      if (lib) {
        potrf_step_kernel<0><<<s.tbase + s.ntrail, WG>>>(A, n, c, nblk, s, Dinv, info, 0, 0, 0, PotrfFwd());
      } else {
        const int M = (nblk - s.cfirst + 1) / 2, c0 = nblk - 2 * M;
        int near = 0;
        for (int J = 0; J < M && c0 + 2 * J - c < D; ++J) near += M - J;
        near_step_kernel<<<s.tbase + near, WG>>>(A, n, c, nblk, s, Dinv, info, D);
      }
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  printf("n=%d: sum of the %d step launches (ms, median of 5)\n", n, nblk);
  for (int D : {-1, 1000, 2, 3, 4, 6, 8}) {
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) t.push_back(run(D, D < 0));
    std::sort(t.begin(), t.end());
    printf("%s D=%4d: %.3f ms\n", D < 0 ? "library step kernel      " : "near-only trailing       ", D, t[2]);
  }
  // (2) the side kernel alone, every column published up front (timing only; the factor is not valid): its throughput
  // without the step launches beside it
  const int NT = nblk / 2;
  const size_t sync_bytes = (size_t)(nblk + NT * NT) * 4;
  int32_t* sync;
  CK(hipMalloc(&sync, sync_bytes));
  hipStream_t side;
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  std::vector<int32_t> hdone(nblk);
  for (int k = 0; k < nblk; ++k) hdone[k] = (nblk - 1 - k) * NB;
  for (int D : {2, 4, 8}) {
    int ntile = 0;
    double flops = 0.0;
    for (int q0 = (D + 2) & ~1; q0 < nblk; q0 += 2) {
      ntile += (nblk - q0) / 2;
      flops += (double)((nblk - q0) / 2) * (q0 - D) * 2.0 * 128 * 128 * 64;
    }
    for (int grid : {cus, 2 * cus}) {
      std::vector<float> t;
      for (int r = 0; r < 5; ++r) {
        CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
        CK(hipMemset(info, 0, 4));
        CK(hipMemset(sync, 0, sync_bytes));
        CK(hipMemcpy(sync, hdone.data(), nblk * 4, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        potrf_side_kernel<<<std::min(grid, ntile), WG>>>(A, n, nblk, D, sync, info, 1u << 22);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      printf("side kernel alone D=%d grid %4d: %.3f ms for %d tiles, %.1f GFLOP = %.1f TF/s\n", D, std::min(grid, ntile),
             t[2], ntile, flops * 1e-9, flops / (t[2] * 1e-3) * 1e-12);
    }
  }
  // (3) the decoupled schedule as the library runs it, with an event after every step launch: per-launch durations
  // (a launch that waits for the side kernel shows it) and the side kernel's end
  std::vector<hipEvent_t> ev(nblk + 1);
  for (auto& e : ev) CK(hipEventCreate(&e));
  hipEvent_t es, fork;
  CK(hipEventCreate(&es));
  CK(hipEventCreate(&fork));
  for (int D : {2, 4, 8}) {
    std::vector<double> acc(nblk, 0.0);
    double side_end = 0.0, total = 0.0;
    const int R = 5;
    for (int r = 0; r < R; ++r) {
      CK(hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
      CK(hipMemset(info, 0, 4));
      CK(hipMemset(sync, 0, sync_bytes));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(ev[0]));
      CK(hipEventRecord(fork));
      CK(hipStreamWaitEvent(side, fork, 0));
      int ntile = 0;
      for (int q0 = (D + 2) & ~1; q0 < nblk; q0 += 2) ntile += (nblk - q0) / 2;
      potrf_side_kernel<<<std::min(cus, ntile), WG, 0, side>>>(A, n, nblk, D, sync, info, 1u << 22);
      CK(hipEventRecord(es, side));
      for (int c = 0; c < nblk; ++c) {
        const DPlan d = dplan(c, nblk, cus, D, sync);
        dec_step_kernel<<<d.s.tbase + d.s.ntrail, WG>>>(A, n, c, nblk, d, Dinv, info);
        CK(hipEventRecord(ev[c + 1]));
      }
      CK(hipDeviceSynchronize());
      CK(hipGetLastError());
      int hinfo;
      CK(hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost));
      if (hinfo != 0) printf("D=%d: info %d\n", D, hinfo);
      float ms;
      for (int c = 0; c < nblk; ++c) {
        CK(hipEventElapsedTime(&ms, ev[c], ev[c + 1]));
        acc[c] += ms / R;
      }
      CK(hipEventElapsedTime(&ms, ev[0], es));
      side_end += ms / R;
      CK(hipEventElapsedTime(&ms, ev[0], ev[nblk]));
      total += ms / R;
    }
    printf("decoupled D=%d: steps %.3f ms, side kernel ends at %.3f ms; per launch (us):", D, total, side_end);
    for (int c = 0; c < nblk; ++c) printf("%s%.0f", c % 16 ? " " : "\n  ", acc[c] * 1e3);
    printf("\n");
  }
  printf("DECOUPLE PROBE DONE\n");
  return 0;
}
