// Round 5: the large-n Cholesky's flush tile (C -= L_I L_J^T over K = 512 for every 128 x 128 lower tile of an m x m
// trailing matrix, the n = 16384 schedule's bulk update) on the hand-placed k loop of gpx_trmm_asm.h, in the library's
// XCD-chunked 8 x 8 super-block tile order (gpx_potrf.hip trail_tile), two workgroups per CU:
//   F0  MfmaTile, row-major panels, C - acc in the epilogue (round 4's flush tile)
//   A1  trmm_asm::TileT<false, false, true>: seeded with C, subtract through the MFMA's A negation (the library's tile)
//   A2  the same on k-major panels (a transposed copy LT[k][i]): what the row-major staging costs
//   A3  A1 without the seed loads (acc from zero, C - acc after the loop): what the seeding costs
//   A4  A1 with the tile order row-major over the lower grid (no XCD chunking)
//   A5  A1 with workgroups 256..511 (the second slot of every CU in the first round) sleeping ~half a tile first, so the
//       two tiles of a CU never load / store at the same time (the stagger then persists)
//   A6  A5 with a quarter-tile sleep
//   A7  A1 with the panels read in place from a factor-shaped buffer (row stride 16384 doubles, as the library's flush
//       reads L from A), against A1's packed panels (row stride K)
//   A8  A1 storing C as the library does: write-through (sc1) 16-byte pairs (gpx_potrf.hip store_block_pairs_sc1)
// F0 / A3 must agree bit for bit, and A1 / A2 / A4 among themselves (the seeded chain rounds differently from C - acc).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -I../bayesianoptimizer_amd/csrc
//        flush_asm_bench.hip -o flush_asm_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gpx_device.h"
#include "gpx_trmm_asm.h"
using namespace gpx;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// gpx_potrf.hip trail_tile (xmap = 1)
__device__ __forceinline__ void xcd_tile(int t, int T, int M, int& I, int& J) {
  const int x = t & 7, l = t >> 3, q = T >> 3, r = T & 7;
  int p = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
  const int S = (M + 7) >> 3;
  for (int SI = 0; SI < S; ++SI) {
    const int rows = M - 8 * SI < 8 ? M - 8 * SI : 8;
    for (int SJ = 0; SJ <= SI; ++SJ) {
      const int cnt = SJ < SI ? rows * 8 : rows * (rows + 1) / 2;
      if (p < cnt) {
        if (SJ < SI) {
          I = 8 * SI + (p >> 3);
          J = 8 * SJ + (p & 7);
        } else {
          int i, j;
          tri_decode(p, i, j);
          I = 8 * SI + i;
          J = 8 * SJ + j;
        }
        return;
      }
      p -= cnt;
    }
  }
  I = J = 0;
}

// gpx_potrf.hip's write-through pair store (copied: that file is not included here)
__device__ __forceinline__ double swap_adjacent(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffull), 0xB1, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), 0xB1, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ void st2(trmm_asm::rsrc_t r, int off, double a, double b) {
  const unsigned long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = {(unsigned)x, (unsigned)(x >> 32), (unsigned)y, (unsigned)(y >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

template <int V>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
flush_v(double* __restrict__ Cm, int64_t ldc, const double* __restrict__ L, const double* __restrict__ LT, int64_t m,
        int K, int M, const double* __restrict__ LW = nullptr, int64_t ldw = 0) {
  __shared__ __attribute__((aligned(16))) double lds[trmm_asm::LDS_BYTES / 8];
  const int T = M * (M + 1) / 2;
  int I, J;
  if (V == 4)
    tri_decode((int)blockIdx.x, I, J);
  else
    xcd_tile((int)blockIdx.x, T, M, I, J);
  if ((V == 5 || V == 6) && blockIdx.x >= 256 && blockIdx.x < 512) {
    const long long t0 = wall_clock64();  // 100 MHz
    const long long wait = V == 5 ? 5000 : 2500;  // 50 / 25 us
    while (wall_clock64() - t0 < wait) __builtin_amdgcn_s_sleep(127);
  }
  double* C = Cm + (int64_t)I * 128 * ldc + (int64_t)J * 128;
  using MT = MfmaTile<128, 128, 16, false, false>;
  d4 acc[4][4];
  if constexpr (V == 0) {
    MT tl;
    tl.run(L + (int64_t)I * 128 * K, K, L + (int64_t)J * 128 * K, K, 0, K, lds);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = C[(int64_t)MT::row_of(i, r) * ldc + MT::col_of(j)] - tl.acc[i][j][r];
  } else if constexpr (V == 3) {
    trmm_asm::TileT<false, false> tl;
    tl.zero();
    tl.run(L + (int64_t)I * 128 * K, K, L + (int64_t)J * 128 * K, K, K / 16, lds);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = C[(int64_t)MT::row_of(i, r) * ldc + MT::col_of(j)] - tl.acc[i][j][r];
  } else {
    constexpr bool KM = V == 2;
    trmm_asm::TileT<KM, KM, true> tl;
    const double* A = KM ? LT + (int64_t)I * 128 : (V == 7 ? LW + (int64_t)I * 128 * ldw : L + (int64_t)I * 128 * K);
    const double* B = KM ? LT + (int64_t)J * 128 : (V == 7 ? LW + (int64_t)J * 128 * ldw : L + (int64_t)J * 128 * K);
    const int64_t ld = KM ? m : (V == 7 ? ldw : K);
    auto rc = trmm_asm::rsrc_of(C);
    tl.template run_after<false, false, 64>(A, ld, B, ld, K / 16, lds, [&] {
      const int v0 = (int)(((int64_t)MT::row_of(0, 0) * ldc + MT::col_of(0)) * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int so = (int)((int64_t)(16 * i + 4 * r) * ldc * 8);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            tl.acc[i][j][r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, v0 + 128 * j, so, 0));
        }
    });
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = tl.acc[i][j];
  }
  if constexpr (V == 8) {
    const auto rc = trmm_asm::rsrc_of(C);
    const bool even = (threadIdx.x & 1) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const d4& v = acc[i][j];
        const double x0 = swap_adjacent(even ? v[2] : v[0]);
        const double x1 = swap_adjacent(even ? v[3] : v[1]);
        const int col = MT::col_of(j) & ~1;
        const int ra = MT::row_of(i, even ? 0 : 2), rb = MT::row_of(i, even ? 1 : 3);
        st2(rc, (int)(((int64_t)ra * ldc + col) * 8), even ? v[0] : x0, even ? x0 : v[2]);
        st2(rc, (int)(((int64_t)rb * ldc + col) * 8), even ? v[1] : x1, even ? x1 : v[3]);
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(int64_t)MT::row_of(i, r) * ldc + MT::col_of(j)] = acc[i][j][r];
}

struct Bufs {
  int m, K, M, tiles;
  double *C, *C0, *L, *LT, *LW;
  int64_t ldw;
};
static Bufs make(int m, int K) {
  Bufs b{m, K, m / 128, (m / 128) * (m / 128 + 1) / 2, nullptr, nullptr, nullptr, nullptr, nullptr, 16384};
  std::vector<double> hL((size_t)m * K), hLT((size_t)m * K), hC((size_t)m * m);
  srand(5);
  for (int i = 0; i < m; ++i)
    for (int k = 0; k < K; ++k) hLT[(size_t)k * m + i] = hL[(size_t)i * K + k] = rand() / (double)RAND_MAX - 0.5;
  for (auto& v : hC) v = rand() / (double)RAND_MAX;
  CK(hipMalloc(&b.C, (size_t)m * m * 8));
  CK(hipMalloc(&b.C0, (size_t)m * m * 8));
  CK(hipMalloc(&b.L, hL.size() * 8));
  CK(hipMalloc(&b.LT, hLT.size() * 8));
  CK(hipMemcpy(b.L, hL.data(), hL.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.LT, hLT.data(), hLT.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.C0, hC.data(), hC.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&b.LW, (size_t)m * b.ldw * 8));
  CK(hipMemcpy2D(b.LW, b.ldw * 8, b.L, (size_t)K * 8, (size_t)K * 8, m, hipMemcpyDeviceToDevice));
  return b;
}
static void run(const Bufs& b, int v) {
  switch (v) {
    case 0: flush_v<0><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 1: flush_v<1><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 2: flush_v<2><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 3: flush_v<3><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 4: flush_v<4><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 5: flush_v<5><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 6: flush_v<6><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
    case 7: flush_v<7><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M, b.LW, b.ldw); break;
    default: flush_v<8><<<b.tiles, WG>>>(b.C, b.m, b.L, b.LT, b.m, b.K, b.M); break;
  }
}

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 15872, K = argc > 2 ? atoi(argv[2]) : 512;
  const char* names[] = {"F0 MfmaTile C-acc", "A1 asm seeded", "A2 asm seeded k-major", "A3 asm C-acc",
                         "A4 A1 row-major order", "A5 A1 + half-tile stagger", "A6 A1 + quarter stagger",
                         "A7 A1 panels in place", "A8 A1 write-through pairs"};
  constexpr int NV = 9;
  {  // bit-for-bit checks at a small size
    Bufs b = make(2048, K);
    const size_t mm = (size_t)b.m * b.m;
    std::vector<std::vector<double>> out(NV, std::vector<double>(mm));
    for (int v = 0; v < NV; ++v) {
      CK(hipMemcpy(b.C, b.C0, mm * 8, hipMemcpyDeviceToDevice));
      run(b, v);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(out[v].data(), b.C, mm * 8, hipMemcpyDeviceToHost));
    }
    auto diff = [&](int x, int y) {
      size_t bad = 0;
      for (size_t q = 0; q < mm; ++q) bad += out[x][q] != out[y][q];
      return bad;
    };
    printf("m=%d K=%d: mismatches F0-A3 %zu, A1-A2 %zu, A1-A4 %zu, A1-A5 %zu, A1-A6 %zu, A1-A7 %zu, A1-A8 %zu (F0-A1 %zu: the "
           "seeded chain rounds differently)\n", b.m, K, diff(0, 3), diff(1, 2), diff(1, 4), diff(1, 5), diff(1, 6),
           diff(1, 7), diff(1, 8), diff(0, 1));
  }
  Bufs b = make(m, K);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flops = 2.0 * 128 * 128 * (double)K * b.tiles;
  std::vector<float> t[NV];
  for (int rep = 0; rep < 6; ++rep)
    for (int v = 0; v < NV; ++v) {
      CK(hipMemcpy(b.C, b.C0, (size_t)m * m * 8, hipMemcpyDeviceToDevice));
      CK(hipEventRecord(e0));
      run(b, v);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms);
    }
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][t[v].size() / 2];
    printf("m=%d K=%d %-24s median %.3f ms -> %.2f TF/s (frac %.4f)\n", m, K, names[v], med,
           flops / (med * 1e-3) / 1e12, flops / (med * 1e-3) / 78.6e12);
  }
  printf("FLUSH ASM BENCH DONE\n");
  return 0;
}
