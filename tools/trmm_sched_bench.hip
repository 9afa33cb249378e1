// Round 4: the sweep product's k loop under explicit instruction schedules.
// Every variant is the library's trmm_sumsq_kernel (gpx_sweep.hip: XCD-aware heavy-first block order, 128x128 MfmaTile,
// BK = 16, column sums of V^2) with the same MFMA order, so outputs must match the shipped tile bit for bit; only the
// placement of the global loads, LDS writes and LDS fragment reads among the 64 MFMAs of a k-tile differs:
//   S0  shipped MfmaTile::run (compiler schedule)
//   S1  last k-tile peeled (branch-free body), compiler schedule
//   S2  peeled + sched_group_barrier: global loads 1 per 2 MFMAs in k-substep 0, fragment reads 1 per 4 MFMAs in
//       substeps 1-2, LDS writes of the next tile 1 per 2 MFMAs in substep 3 (Tensile SIA3-like spread)
//   S3  as S2, LDS writes spread over substeps 2-3 (1 per 4 MFMAs)
//   S4  as S2, global loads spread over substeps 0-1 (1 per 4 MFMAs)
//   S5  peeled + iglp_opt(0)
//   S6  peeled + iglp_opt(1)
//   S7  one branch-free loop body (clamped next-tile loads), compiler schedule; S8 / S9 / S10: S7 + the S3 groups /
//       iglp_opt(0) / the S2 groups
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_device.h"

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

#define SGB(mask, n) __builtin_amdgcn_sched_group_barrier(mask, n, 0)
constexpr int M_MFMA = 0x8, M_VMEM_R = 0x20, M_DS_R = 0x100, M_DS_W = 0x200;

template <int S>
__device__ __forceinline__ void schedule() {
  if constexpr (S == 2 || S == 3 || S == 4) {
    SGB(M_DS_R, 8);  // fragments of substeps 0 and 1 (ds_read2_b64 pairs)
    if constexpr (S == 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        SGB(M_MFMA, 4);
        SGB(M_VMEM_R, 1);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        SGB(M_MFMA, 2);
        SGB(M_VMEM_R, 1);
      }
      // substep 1 with substep 2's fragment reads
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        SGB(M_MFMA, 4);
        SGB(M_DS_R, 1);
      }
    }
    if constexpr (S == 3) {
      // substep 2 (its fragments for substep 3 + half the writes), substep 3 (the other writes)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        SGB(M_MFMA, 4);
        SGB(M_DS_R, 1);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        SGB(M_MFMA, 2);
        SGB(M_DS_W, 1);
      }
    } else if constexpr (S == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        SGB(M_MFMA, 4);
        SGB(M_DS_R, 1);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        SGB(M_MFMA, 2);
        SGB(M_DS_W, 1);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        SGB(M_MFMA, 4);
        SGB(M_DS_R, 1);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        SGB(M_MFMA, 2);
        SGB(M_DS_W, 1);
      }
    }
  } else if constexpr (S == 5) {
    __builtin_amdgcn_iglp_opt(0);
  } else if constexpr (S == 6) {
    __builtin_amdgcn_iglp_opt(1);
  }
}

template <int S>
struct TileS : public Base {
  // S >= 7: one branch-free loop body over every k-tile: the next tile's loads use a clamped k (the last trip re-loads its
  // own tile into the idle buffer), so loads, fragment reads, MFMAs and LDS writes share one scheduling region
  __device__ __forceinline__ void run_bf(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                         int64_t ldb, int kend, double* smem) {
    this->zero();
    double* cur = smem;
    double* nxt = smem + 16 * (PA + PB);
    this->load_regs(A, lda, B, ldb, 0);
    this->store_lds(cur, cur + 16 * PA);
    __syncthreads();
    for (int k0 = 0; k0 < kend; k0 += 16) {
      const int kn = k0 + 16 < kend ? k0 + 16 : k0;
      this->load_regs(A, lda, B, ldb, kn);
      this->compute(cur, cur + 16 * PA);
      this->store_lds(nxt, nxt + 16 * PA);
      if constexpr (S == 8) schedule<3>();
      if constexpr (S == 9) schedule<5>();
      if constexpr (S == 10) schedule<2>();
      __syncthreads();
      double* t = cur;
      cur = nxt;
      nxt = t;
    }
  }
  __device__ __forceinline__ void run_s(const double* __restrict__ A, int64_t lda, const double* __restrict__ B,
                                        int64_t ldb, int kend, double* smem) {
    this->zero();
    double* cur = smem;
    double* nxt = smem + 16 * (PA + PB);
    this->load_regs(A, lda, B, ldb, 0);
    this->store_lds(cur, cur + 16 * PA);
    __syncthreads();
    for (int k0 = 0; k0 + 16 < kend; k0 += 16) {
      this->load_regs(A, lda, B, ldb, k0 + 16);
      this->compute(cur, cur + 16 * PA);
      this->store_lds(nxt, nxt + 16 * PA);
      schedule<S>();
      __syncthreads();
      double* t = cur;
      cur = nxt;
      nxt = t;
    }
    this->compute(cur, cur + 16 * PA);
    __syncthreads();
  }
};

template <int S>
__global__ void __launch_bounds__(WG) trmm_s(const double* __restrict__ W, int64_t ldw, const double* __restrict__ kstar,
                                             int64_t C, int nI, int ncb, double* __restrict__ ss_part) {
  __shared__ __attribute__((aligned(16))) double smem[Base::LDS_DOUBLES];
  const int b = blockIdx.x;
  int I, cb;
  const int x = b & 7, l = b >> 3, per = ncb >> 3;
  I = nI - 1 - l / per;
  cb = 8 * (l % per) + x;
  const double* Ab = W + (int64_t)I * TT;
  const double* Bb = kstar + (int64_t)cb * TT;
  TileS<S> tile;
  if constexpr (S == 0)
    tile.run(Ab, ldw, Bb, C, 0, (I + 1) * TT, smem);
  else if constexpr (S >= 7)
    tile.run_bf(Ab, ldw, Bb, C, (I + 1) * TT, smem);
  else
    tile.run_s(Ab, ldw, Bb, C, (I + 1) * TT, smem);
  double s[Base::WN];
#pragma unroll
  for (int j = 0; j < Base::WN; ++j) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < Base::WM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += tile.acc[i][j][r] * tile.acc[i][j][r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    s[j] = v;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* red = smem;
  if ((w >> 1) == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < Base::WN; ++j) red[Base::col_of(j)] = s[j];
  }
  __syncthreads();
  if ((w >> 1) == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < Base::WN; ++j) {
      const int col = Base::col_of(j);
      ss_part[(int64_t)I * C + (int64_t)cb * TT + col] = s[j] + red[col];
    }
  }
}

// S11+: no LDS at all.  Every wave loads its own MFMA fragments straight from global memory (k-major operands: lanes
// m = 0..15 of a k-row read 16 consecutive doubles, so each load instruction covers four full 128-byte lines), PD
// k-steps (of 4) ahead in a register ring of PD + 1 stages; no barriers, no LDS writes or reads.  The same MFMA order per
// accumulator as the shipped tile (k ascending), so the column sums agree bit for bit.
template <int PD>
__global__ void __launch_bounds__(WG) trmm_direct(const double* __restrict__ W, int64_t ldw,
                                                  const double* __restrict__ kstar, int64_t C, int nI, int ncb,
                                                  double* __restrict__ ss_part) {
  constexpr int NS = PD + 1;
  const int b = blockIdx.x;
  const int x = b & 7, l = b >> 3, per = ncb >> 3;
  const int I = nI - 1 - l / per, cb = 8 * (l % per) + x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m = lane & 15, kq = lane >> 4;
  const double* Ab = W + (int64_t)I * TT + (w >> 1) * 64 + m + (int64_t)kq * ldw;
  const double* Bb = kstar + (int64_t)cb * TT + (w & 1) * 64 + m + (int64_t)kq * C;
  const int nsteps = (I + 1) * TT / 4;
  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  double a[NS][4], bb[NS][4];
  auto load = [&](int st, int s) {
    const int64_t ka = (int64_t)(4 * s) * ldw, kb = (int64_t)(4 * s) * C;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[st][i] = Ab[ka + 16 * i];
#pragma unroll
    for (int j = 0; j < 4; ++j) bb[st][j] = Bb[kb + 16 * j];
  };
#pragma unroll
  for (int st = 0; st < PD; ++st) load(st, st);
  for (int s0 = 0; s0 < nsteps; s0 += NS) {
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int s = s0 + st;
      const int sn = s + PD < nsteps ? s + PD : nsteps - 1;  // clamped: the tail re-loads the last step (unused)
      load((st + PD) % NS, sn);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x4(a[st][i], bb[st][j], acc[i][j]);
    }
  }
  // column sums of squares over this wave's 64 rows, then over the two row halves (as the shipped kernel)
  __shared__ double red[TT];
  double sv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += acc[i][j][r] * acc[i][j][r];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    sv[j] = v;
  }
  if ((w >> 1) == 1 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[(w & 1) * 64 + 16 * j + m] = sv[j];
  }
  __syncthreads();
  if ((w >> 1) == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = (w & 1) * 64 + 16 * j + m;
      ss_part[(int64_t)I * C + (int64_t)cb * TT + col] = sv[j] + red[col];
    }
  }
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
  const char* names[] = {"S0 shipped", "S1 peeled", "S2 sgb spread", "S3 sgb writes 2-3", "S4 sgb loads 0-1",
                         "S5 iglp_opt(0)", "S6 iglp_opt(1)", "S7 branch-free", "S8 bf + sgb S3",
                         "S9 bf + iglp(0)", "S10 bf + sgb S2", "S11 direct PD=1", "S12 direct PD=3",
                         "S13 direct PD=5"};
  constexpr int NV = 14;
  auto run = [&](int v, double* out) {
    const dim3 g(ncb * nI);
    switch (v) {
      case 0: trmm_s<0><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 1: trmm_s<1><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 2: trmm_s<2><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 3: trmm_s<3><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 4: trmm_s<4><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 5: trmm_s<5><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 6: trmm_s<6><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 7: trmm_s<7><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 8: trmm_s<8><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 9: trmm_s<9><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 10: trmm_s<10><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 11: trmm_direct<1><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      case 12: trmm_direct<3><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
      default: trmm_direct<5><<<g, WG>>>(W, n, K, C, nI, ncb, out); break;
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
    size_t bad = 0;
    for (size_t q = 0; q < ref.size(); ++q) bad += (ref[q] != got[q]);
    printf("%-20s bitwise mismatches vs S0: %zu\n", names[v], bad);
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
    printf("%-20s median %.3f ms min %.3f ms -> %.2f TF/s (frac %.4f)\n", names[v], med, t[v][0],
           flops / (med * 1e-3) / 1e12, flops / (med * 1e-3) / 78.6e12);
  }
  printf("TRMM SCHED BENCH DONE\n");
  return 0;
}
