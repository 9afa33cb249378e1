// Blocked right-looking Cholesky (lower) of the padded Gram matrix, NB = 64, ONE launch per block column.
// SURVEY §8a row a4 — replaces psd_safe_cholesky in GPyTorch's exact path [upstream]; the reference's
// jitter-retry policy (optimization/Bayesian6.py:481-488) needs the failing pivot, reported in *info.
//
// Launch c (c = 0 .. nblk-1) holds two independent kinds of workgroup:
//  * panel workgroups p = 0 .. nblk-c-1 (row block i = c + p) factor block column c.  For c > 0 they first apply
//    the step-(c-1) update to exactly the tiles they need, A_cc -= L_{c,c-1} L_{c,c-1}^T and
//    A_ic -= L_{i,c-1} L_{c,c-1}^T (64x64x64 on fp64 MFMA, MfmaTile), then factor the tall panel [A_cc; A_ic]
//    (128 x 64, or A_cc alone for p = 0) in LDS in four 16-column steps:
//        F  wave 0 factors + inverts the 16x16 pivot block in registers (chol16, gpx_chol64.h),
//        T  L_is = A_is D_ss^T for the 16-row blocks below it (fp64 MFMA),
//        U  A_ij -= L_is L_js^T for the trailing 16x16 blocks of the panel (fp64 MFMA),
//    with a one-block lookahead: wave 0 does the T and U of the next pivot block itself and goes straight on to the
//    next F (one barrier per step); waves 1-3 do the other T items, wait on an LDS counter until every T item of the
//    step is published, and do the other U items while that F runs.  Where a launch's workgroups all fit the
//    co-resident slots, the first F runs on wave 0 under the other waves' pre-update MFMAs (update_eager OV).
//    Every panel workgroup re-factors A_cc (no
//    extra latency, no extra launch); p = 0 stores L_cc in the scratch half of Dinv (A_cc must stay intact while
//    the other panel workgroups read it), p > 0 store L_ic.
//  * trailing workgroups apply the step-(c-1) update to every lower tile of columns >= c+1:
//    A_ij -= L_{i,c-1} L_{j,c-1}^T on 128x128 MfmaTiles (half the HBM/L2 traffic per flop of 64x64 tiles; the
//    update is traffic-bound at 64x64: 36 us for the 2016 tiles of step 0); tiles that would run as a last, partly
//    empty round of slots run as 128x64 halves instead (StepPlan::nsplit).
// Column c+1 is thus updated by step c-1 in launch c and by step c inside the panel workgroups of launch c+1, so
// the panel factorisation (the latency-bound serial chain) overlaps the trailing update of the previous step
// instead of following it.  For large n the trailing update is flushed lazily (every g block columns, K = 64 g:
// each C tile read and written once per g columns) and lookahead workgroups bring the next panel's column up to
// date in the launch before it (StepPlan below).  potrf_dinv finally copies every L_kk from the scratch into A and inverts it (Dinv, used
// by gpx_trtri_f64).
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_chol64.h"
#include "gpx_trmm_asm.h"

// Optional timestamp hooks for tools/potrf_steps_probe.hip (compiled out in the library).
#ifndef GPX_PANEL_STAMP
#define GPX_PANEL_STAMP(i)
#endif
#ifndef GPX_STEP_STAMP
#define GPX_STEP_STAMP(role, c, b, s)
#endif
#ifndef GPX_EAGER_STAMP
#define GPX_EAGER_STAMP(c, p, i)
#endif

namespace gpx {

using Tile64 = MfmaTile<NB, NB, 16, false, false>;        // panel-side update (one 64x64 tile)
using Tile128 = MfmaTile<2 * NB, 2 * NB, 16, false, false>;  // trailing update
// LDS budget: two workgroups per CU (<= 80 KB each), so a trailing tile's loads and epilogue overlap another
// tile's MFMAs (one 128x128x64 tile alone takes ~14 us; at one workgroup per CU step 1 took 43 us for 496 tiles).
// Panel: sA, sP (64 x LD64 each) and the two D_ss buffers (16 x LDD); the Tile64 staging of the panel-side
// update aliases sP + the D buffers (both written only after the update GEMMs).
constexpr int LDD = 20;
constexpr int DBUF = 768;  // >= 2 * 16 * LDD, and sP + D buffers hold Tile64::LDS_DOUBLES
static_assert(NB * LD64 + DBUF >= Tile64::LDS_DOUBLES && DBUF >= 2 * 16 * LDD, "panel LDS aliasing");
// + the forward fold's right-hand sides of a p > 0 panel workgroup (64 x GPX_MAX_RHS, stored at the workgroup's end:
// a global store before a barrier would hold the barrier until it completes)
constexpr int PANEL_LDS = 2 * NB * LD64 + DBUF + NB * GPX_MAX_RHS;
constexpr int STEP_LDS = PANEL_LDS > Tile128::LDS_DOUBLES ? PANEL_LDS : Tile128::LDS_DOUBLES;
static_assert(STEP_LDS * 8 + 64 <= 81920, "two workgroups per CU");
// the 128 x 128 trailing tiles run the hand-placed k loop (gpx_trmm_asm.h) on the step kernel's LDS buffer
static_assert(Tile128::LDS_DOUBLES * 8 == trmm_asm::LDS_BYTES && STEP_LDS >= Tile128::LDS_DOUBLES,
              "hand-placed tile uses MfmaTile's LDS image and needs the step kernel's buffer to hold it");

// C - L_a L_b^T for a 64x64 tile into the LDS tile S (row length LD64): acc seeded with -C (its loads issued with the
// first k-tile's, no load round trip after the product), acc += L_a L_b^T over K, S = -acc.
__device__ __forceinline__ void update_to_lds(Tile64& tl, const double* __restrict__ Cg, int64_t ldc,
                                              const double* __restrict__ La, const double* __restrict__ Lb, int64_t ldl,
                                              int K, double* smem, double* S) {
  tl.load_neg_c(Cg, ldc);
  if (K == NB)
    tl.run_acc(La, ldl, Lb, ldl, 0, NB, smem);  // the eager case, on the critical path: compile-time trip count
  else
    tl.run_acc(La, ldl, Lb, ldl, 0, K, smem);
  // run_acc() ends with a barrier after its last LDS read, so S may alias the staging
#pragma unroll
  for (int i = 0; i < Tile64::WM; ++i)
#pragma unroll
    for (int j = 0; j < Tile64::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) S[Tile64::row_of(i, r) * LD64 + Tile64::col_of(j)] = -tl.acc[i][j][r];
}

// The eager pre-update (K = 64: one pending block column) of a panel workgroup: A_cc -= L_c L_c^T on the 10 lower /
// diagonal 16-blocks (the strict upper ones are never read by the factorisation) and, for p > 0, A_ic -= L_i L_c^T on
// all 16, into sA / sP.  Every global load of the step - L_c, L_i and the C seeds of the wave's blocks - is issued in one
// straight-line burst (MfmaTile's 16-k pipeline exposed a global round trip per k-tile: ~7 us for the two products
// against ~3 us of MFMA); the seeds are +C and the products subtract through the MFMA's A-operand negation (neg:[1,0,0]),
// so nothing waits on a seed before the first MFMA needs it.  Each wave owns the blocks of its lists (kPreCC / kPreIC
// below: indices into the row-major lower list kLowerBlk and A_ic blocks), each a K = 64 chain of 16 MFMAs in MfmaTile's
// k order (C - ab rounds as -(-C + ab): same results).  sA / sP double as the staging: the products are held in
// registers across a barrier.
constexpr int kLowerBlk[10][2] = {{0, 0}, {1, 0}, {1, 1}, {2, 0}, {2, 1}, {2, 2}, {3, 0}, {3, 1}, {3, 2}, {3, 3}};

__device__ __forceinline__ d4 mfma_sub(double a, double b, d4 c) {  // c - a b
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st2_sc1(rsrc_t r, int off, double a, double b) {  // 16-byte write-through store
  const unsigned long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  const u32x4_t v = {(unsigned)x, (unsigned)(x >> 32), (unsigned)y, (unsigned)(y >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
__device__ __forceinline__ double swap_adjacent_lanes(double v) {  // DPP quad_perm [1, 0, 3, 2]
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffull), 0xB1, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), 0xB1, 0xf, 0xf, false);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One 16x16 accumulator block (i, j) of an MfmaTile (rows row_of(i, r), column col_of(j)) stored write-through as 16-byte
// pairs: adjacent lanes swap halves so that the even lane holds two adjacent columns of rows r = 0, 1 and the odd lane of
// rows r = 2, 3 (sc1 stores leave no dirty line in the XCD's L2 for the kernel boundary to write back).  keep01 / keep23:
// store the even / odd lane's rows.
template <typename T>
__device__ __forceinline__ void store_block_pairs_sc1(rsrc_t rc, int64_t ld, int i, int j, const d4& v, bool keep01,
                                                      bool keep23) {
  const bool even = (threadIdx.x & 1) == 0;
  const double x0 = swap_adjacent_lanes(even ? v[2] : v[0]);
  const double x1 = swap_adjacent_lanes(even ? v[3] : v[1]);
  const int col = T::col_of(j) & ~1;
  const int ra = T::row_of(i, even ? 0 : 2), rb = T::row_of(i, even ? 1 : 3);
  if (even ? keep01 : keep23) {
    st2_sc1(rc, (int)(((int64_t)ra * ld + col) * 8), even ? v[0] : x0, even ? x0 : v[2]);
    st2_sc1(rc, (int)(((int64_t)rb * ld + col) * 8), even ? v[1] : x1, even ? x1 : v[3]);
  }
}

// The forward half of alpha's triangular solve folded into the factorisation (launch_potrf with a ForwardRhs, eager
// schedules only): z = L^{-1} (Y - mean) for NR = 1 or GPX_MAX_RHS right-hand-side columns (padded rows and columns
// >= nrhs are 0).  Row block i's running right-hand side r_i = (Y - mean)_i - sum_{k < c} L_ik z_k is kept by the panel
// workgroup of row i: in launch c >= 1 it subtracts L_{i,c-1} z_{c-1} with the L_{i,c-1} its pre-update has in LDS
// anyway, and the p = 0 workgroup (i = c) then forms z_c = L_cc^{-1} r_c block by block inside the factorisation
// (z_s = D_s r_s, r_s' -= L_s's z_s for s' > s), on wave 3, the wave with the fewest U items there.  r lives in
// global memory between launches (npad x NR), z is written once per block (npad x NR).
struct PotrfFwd {
  const double* Y = nullptr;
  int64_t ldy = 0, sy = 0;  // sy: Y stride per problem
  double* r = nullptr;      // running right-hand sides (null: no fold)
  double* z = nullptr;
  int64_t sb = 0;           // r / z stride per problem
  int nrhs = 1, n = 0;
  double mean = 0.0;
  const double* means = nullptr;  // per-problem constant means (device): mean = means[problem]
};

__device__ __forceinline__ double fwd_y(const PotrfFwd& f, int row, int rr) {
  return (row < f.n && rr < f.nrhs) ? f.Y[(int64_t)row * f.ldy + rr] - f.mean : 0.0;
}

__device__ __forceinline__ double dbl_of(unsigned lo, unsigned hi) {
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// (x_0 + x_2) + (x_1 + x_3) over the four 16-lane rows q of a wave, the same value in every row: gfx950's
// v_permlane32_swap / v_permlane16_swap (VALU) instead of two ds_bpermute round trips (measured equal inside the fold).
__device__ __forceinline__ double rowsum4(double x) {
  const unsigned long long u = __double_as_longlong(x);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)u, (unsigned)u, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
  const double y = dbl_of(lo[0], hi[0]) + dbl_of(lo[1], hi[1]);  // rows (0+2, 1+3, 0+2, 1+3)
  const unsigned long long v = __double_as_longlong(y);
  const auto lo2 = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  const auto hi2 = __builtin_amdgcn_permlane16_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
  return dbl_of(lo2[0], hi2[0]) + dbl_of(lo2[1], hi2[1]);  // even row + odd row
}

// One wave: out[rr] = sum_k M[a][k] v[k][rr] for the 16-row block M (LDS, row length ldm, KQ columns per lane
// quarter: K = 4 KQ) and v (LDS, K x NR); lane = a + 16 kq sums its quarter, the quarters are combined by two
// cross-lane exchanges in a fixed order, so every lane of row a holds the same total.
template <int NR, int KQ>
__device__ __forceinline__ void wave_matvec16(const double* M, int ldm, const double* v, double (&out)[NR]) {
  const int lane = threadIdx.x & 63, a = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) out[rr] = 0.0;
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    const int kk = kq * KQ + k;
    const double m = M[a * ldm + kk];
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) out[rr] = fma(m, v[kk * NR + rr], out[rr]);
  }
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) out[rr] = rowsum4(out[rr]);
}

// LDS stores of one lane, then reads of them by other lanes of the same wave (LDS is in order per wave; this keeps
// the compiler from moving the reads up)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Block lists per wave (OV = 0 / 1, variant V = 0 the p = 0 workgroup, 1 a panel workgroup with 64 rows of A_ic, 2 with
// 32 (SPLIT = 2)): kPreCC the wave's A_cc blocks (kLowerBlk indices, -1 ends), kPreIC its A_ic blocks {first, count}
// of the block index 4 rb + j (row block rb of the workgroup's rows, column block j), kFoldRB the right-hand-side row
// block it folds (-1: none; A_ic row blocks for p > 0, row block W of L_c for p = 0).
//  OV = 0, even split: wave W owns the A_cc blocks W, W + 4, W + 8 and a quarter of A_ic (at most 7 / 5 blocks).
//  OV = 1, overlapped: wave 0 updates only the first pivot block A_cc(0, 0) and factors it at once (chol16 in
//    registers) while waves 1-3 update the other nine A_cc blocks and A_ic (3/3/3, 9/8/8, 6/6/5 blocks), so the first
//    F step runs under the other waves' MFMAs instead of after them; wave 0 takes a fold row block in variant 1 so that
//    no wave holds two.  Wave 0 computes its block in chol16's register layout directly: lane (r, g) needs
//    A'[r][4g + q]; the MFMA leaves C[g + 4q][r] in that lane, so its A operand reads L_c's rows in the order
//    perm(m) = 4 (m % 4) + m / 4 (C[g + 4q][r] = A'[4g + q][r] = A'[r][4g + q], A' symmetric) and its seed is loaded
//    in the same order.
constexpr int kPreCC[2][3][4][5] = {
    {{{0, 4, 8, -1, -1}, {1, 5, 9, -1, -1}, {2, 6, -1, -1, -1}, {3, 7, -1, -1, -1}},
     {{0, 4, 8, -1, -1}, {1, 5, 9, -1, -1}, {2, 6, -1, -1, -1}, {3, 7, -1, -1, -1}},
     {{0, 4, 8, -1, -1}, {1, 5, 9, -1, -1}, {2, 6, -1, -1, -1}, {3, 7, -1, -1, -1}}},
    {{{0, -1, -1, -1, -1}, {1, 2, 3, -1, -1}, {4, 5, 6, -1, -1}, {7, 8, 9, -1, -1}},
     {{0, -1, -1, -1, -1}, {1, -1, -1, -1, -1}, {2, 3, 4, 5, -1}, {6, 7, 8, 9, -1}},
     {{0, -1, -1, -1, -1}, {1, 2, -1, -1, -1}, {3, 4, -1, -1, -1}, {5, 6, 7, 8, 9}}}};
constexpr int kPreIC[2][3][4][2] = {{{{0, 0}, {0, 0}, {0, 0}, {0, 0}},
                                     {{0, 4}, {4, 4}, {8, 4}, {12, 4}},
                                     {{0, 2}, {2, 2}, {4, 2}, {6, 2}}},
                                    {{{0, 0}, {0, 0}, {0, 0}, {0, 0}},
                                     {{0, 0}, {0, 8}, {8, 4}, {12, 4}},
                                     {{0, 0}, {0, 4}, {4, 4}, {0, 0}}}};
constexpr int kFoldRB[2][3][4] = {{{0, 1, 2, 3}, {0, 1, 2, 3}, {0, -1, 1, -1}},
                                  {{0, 1, 2, 3}, {1, 0, 2, 3}, {-1, 0, 1, -1}}};
constexpr int pre_count(const int* l, int n) {
  int k = 0;
  while (k < n && l[k] >= 0) ++k;
  return k;
}

template <int W, bool OV, bool PANEL, int NR, int SPLIT>
__device__ __forceinline__ void update_eager_wave(const double* __restrict__ Acc, const double* __restrict__ Aic,
                                                  const double* __restrict__ Lc, const double* __restrict__ Li,
                                                  int64_t lda, double* sA, double* sP, double* sD0, int c, int rowblk0,
                                                  const PotrfFwd& f, double* sZ, double* sR, int& fail) {
  constexpr int V = PANEL ? (SPLIT == 1 ? 1 : 2) : 0;
  constexpr bool PIV = OV && W == 0;  // this wave factors pivot block 0
  constexpr int NCC = pre_count(kPreCC[OV][V][W], 5);
  constexpr int IC0 = kPreIC[OV][V][W][0], NIC = kPreIC[OV][V][W][1];
  constexpr int RB0 = IC0 / 4, NRB = NIC > 0 ? (IC0 + NIC - 1) / 4 - RB0 + 1 : 0;  // its A_ic row blocks
  constexpr int RBF = kFoldRB[OV][V][W];
  constexpr int NRI = 8 / SPLIT;  // double2 loads of L_i per thread (64 / SPLIT rows)
  static_assert(SPLIT == 1 || SPLIT == 2, "panel split");
  const int t = threadIdx.x, lane = t & 63;
  const int g = lane >> 4, cl = lane & 15;
  double2 rl[8], ri[NRI];
  d4 acc_cc[NCC], acc_ic[NIC > 0 ? NIC : 1];
  // forward fold: z_{c-1} (-> LDS sZ) and this lane's old right-hand sides (row 16 RBF + cl of the workgroup's rows,
  // which start at global row rowblk0)
  double2 zv = make_double2(0.0, 0.0);
  double rold[NR > 0 ? NR : 1];
  if constexpr (NR > 0) {
    if (t < 32 * NR) zv = *reinterpret_cast<const double2*>(f.z + (int64_t)(c - 1) * NB * NR + 2 * t);
    if constexpr (RBF >= 0) {
      const int frow = rowblk0 + 16 * RBF + cl;
#pragma unroll
      for (int rr = 0; rr < NR; ++rr)
        rold[rr] = g != 0 ? 0.0 : (c == 1 ? fwd_y(f, frow, rr) : f.r[(int64_t)frow * NR + rr]);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, cc = e & 63;
    rl[q] = *reinterpret_cast<const double2*>(Lc + (int64_t)r * lda + cc);
    if (PANEL && q < NRI) ri[q] = *reinterpret_cast<const double2*>(Li + (int64_t)r * lda + cc);
  }
  if constexpr (PIV) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc_cc[0][q] = Acc[(int64_t)(4 * g + q) * lda + cl];  // chol16's layout
  } else {
#pragma unroll
    for (int b = 0; b < NCC; ++b) {
      const int bi = kLowerBlk[kPreCC[OV][V][W][b]][0], bj = kLowerBlk[kPreCC[OV][V][W][b]][1];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc_cc[b][q] = Acc[(int64_t)(16 * bi + g + 4 * q) * lda + 16 * bj + cl];
    }
  }
#pragma unroll
  for (int e = 0; e < NIC; ++e)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      acc_ic[e][q] = Aic[(int64_t)(16 * ((IC0 + e) >> 2) + g + 4 * q) * lda + 16 * ((IC0 + e) & 3) + cl];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, cc = e & 63;
    *reinterpret_cast<double2*>(sA + r * LD64 + cc) = rl[q];
    if (PANEL && q < NRI) *reinterpret_cast<double2*>(sP + r * LD64 + cc) = ri[q];
  }
  if constexpr (NR > 0) {
    if (t < 32 * NR) *reinterpret_cast<double2*>(sZ + 2 * t) = zv;
  }
  __syncthreads();
  GPX_EAGER_STAMP(c, rowblk0, 0);
  // k in chunks of 16: one batch of fragment reads (the four L_c row blocks serve as the B operand of every block and as
  // the A operand of the A_cc blocks; L_i's row blocks are the A_ic blocks' A operands), then the chunk's MFMAs
  const int m = lane & 15, kq = lane >> 4;
  const int mp = 4 * (m & 3) + (m >> 2);  // the pivot wave's A-operand row order
  double part[NR > 0 ? NR : 1];
#pragma unroll
  for (int rr = 0; rr < (NR > 0 ? NR : 1); ++rr) part[rr] = 0.0;
#pragma unroll
  for (int kc = 0; kc < NB; kc += 16) {
    double fc[4][4], fi[NRB > 0 ? NRB : 1][4], fp[4], ff[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) fc[jb][s] = sA[(16 * jb + m) * LD64 + kc + 4 * s + kq];
      if constexpr (PIV) fp[s] = sA[mp * LD64 + kc + 4 * s + kq];
#pragma unroll
      for (int i = 0; i < NRB; ++i) fi[i][s] = sP[(16 * (RB0 + i) + m) * LD64 + kc + 4 * s + kq];
      if constexpr (NR > 0 && RBF >= 0) ff[s] = PANEL ? sP[(16 * RBF + m) * LD64 + kc + 4 * s + kq] : fc[RBF][s];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int e = 0; e < NIC; ++e)
        acc_ic[e] = mfma_sub(fi[((IC0 + e) >> 2) - RB0][s], fc[(IC0 + e) & 3][s], acc_ic[e]);
      if constexpr (PIV) {
        acc_cc[0] = mfma_sub(fp[s], fc[0][s], acc_cc[0]);
      } else {
#pragma unroll
        for (int b = 0; b < NCC; ++b)
          acc_cc[b] = mfma_sub(fc[kLowerBlk[kPreCC[OV][V][W][b]][0]][s], fc[kLowerBlk[kPreCC[OV][V][W][b]][1]][s],
                               acc_cc[b]);
      }
      if constexpr (NR > 0 && RBF >= 0) {
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) part[rr] = fma(ff[s], sZ[(kc + 4 * s + kq) * NR + rr], part[rr]);
      }
    }
  }
  if constexpr (NR > 0 && RBF >= 0) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) part[rr] = rowsum4(part[rr]);
    if (g == 0) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) sR[(16 * RBF + cl) * NR + rr] = rold[rr] - part[rr];
    }
  }
  Blk16 bk;
  if constexpr (PIV) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bk.a[q] = acc_cc[0][q];
    fail = chol16_regs(bk);  // F of pivot block 0, under waves 1-3's MFMAs
  }
  __syncthreads();  // every wave's operand reads done: sA / sP take the results (and L_00, D_0)
  GPX_EAGER_STAMP(c, rowblk0, 1);
  if constexpr (PIV) {
    chol16_store<LDD>(bk, sA, sD0, 0);
  } else {
#pragma unroll
    for (int b = 0; b < NCC; ++b)
      store_block16(sA, 16 * kLowerBlk[kPreCC[OV][V][W][b]][0], 16 * kLowerBlk[kPreCC[OV][V][W][b]][1], acc_cc[b]);
#pragma unroll
    for (int e = 0; e < NIC; ++e) store_block16(sP, 16 * ((IC0 + e) >> 2), 16 * ((IC0 + e) & 3), acc_ic[e]);
  }
}

// OV: the overlapped lists (pivot block 0 factored on return: L_00 in sA, D_0 in sD0, fail = its failing pivot or -1)
template <bool OV, bool PANEL, int NR, int SPLIT>
__device__ __forceinline__ void update_eager(const double* __restrict__ Acc, const double* __restrict__ Aic,
                                             const double* __restrict__ Lc, const double* __restrict__ Li, int64_t lda,
                                             double* sA, double* sP, double* sD0, int c, int rowblk0,
                                             const PotrfFwd& f, double* sZ, double* sR, int& fail) {
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {  // wave-uniform: compile-time block lists per wave
    case 0: update_eager_wave<0, OV, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, sD0, c, rowblk0, f, sZ, sR, fail); break;
    case 1: update_eager_wave<1, OV, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, sD0, c, rowblk0, f, sZ, sR, fail); break;
    case 2: update_eager_wave<2, OV, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, sD0, c, rowblk0, f, sZ, sR, fail); break;
    default: update_eager_wave<3, OV, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, sD0, c, rowblk0, f, sZ, sR, fail); break;
  }
}

// Waves w = 1..3 of the p = 0 panel workgroup at pivot step s (D_s = L_ss^{-1} in D, L_s's for s' > s published in
// sA): each forms z_s = D_s r_s (the same arithmetic in every wave; wave 1 keeps it in sZall), then wave w applies
// r_{s+w} -= L_{s+w,s} z_s, so no wave carries more than two 16 x 16 products per step.
template <int NR>
__device__ __forceinline__ void fwd_pivot_step(int s, int w, const double* D, const double* sA, double* sR,
                                               double* sZs, double* sZall) {
  const int lane = threadIdx.x & 63, a = lane & 15, kq = lane >> 4;
  double part[NR];
  double* zw = sZs + (w - 1) * 16 * NR;  // this wave's copy of z_s
  wave_matvec16<NR, 4>(D, LDD, sR + 16 * s * NR, part);
  if (kq == 0) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      zw[a * NR + rr] = part[rr];
      if (w == 1) sZall[(16 * s + a) * NR + rr] = part[rr];
    }
  }
  const int s2 = s + w;
  if (s2 < 4) {
    wave_lds_sync();
    wave_matvec16<NR, 4>(sA + 16 * s2 * LD64 + 16 * s, LD64, zw, part);
    if (kq == 0) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) sR[(16 * s2 + a) * NR + rr] -= part[rr];
    }
  }
}

template <int ROWS = NB>
__device__ __forceinline__ void load_tile_lds(const double* __restrict__ G, int64_t ld, double* S) {
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < ROWS / 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    const double2 v = *reinterpret_cast<const double2*>(G + (int64_t)r * ld + c);
    S[r * LD64 + c] = v.x;
    S[r * LD64 + c + 1] = v.y;
  }
}

// Panel workgroup p of block column c (see the file comment); NR > 0: with the forward fold (PotrfFwd).  SPLIT > 1
// (p > 0): the workgroup owns rows PROWS h .. PROWS h + PROWS - 1 (PROWS = 64 / SPLIT) of row block c + p, a
// (64 + PROWS)-row tall panel, so that its pre-update MFMAs and its T / U items shrink with the split; the host picks the
// largest split whose launch still fits the co-resident slots (StepPlan::split).
template <int NR, int SPLIT>
__device__ __forceinline__ void panel_role(double* __restrict__ A, int64_t lda, int c, int p, int h, int nblk, int c0,
                                           double* __restrict__ Dinv, int32_t* __restrict__ info, double* lds,
                                           const PotrfFwd& f, bool ov) {
  constexpr int PROWS = NB / SPLIT;  // rows of A_ic this workgroup owns
  double* sA = lds;             // A_cc -> L_cc
  double* sP = sA + NB * LD64;  // A_ic -> L_ic (p > 0)
  double* sDb = sP + NB * LD64; // D_ss, double-buffered by step parity (2 x 16 x LDD)
  double* smem = sP;            // Tile64 staging of the update GEMMs (aliases sP + sDb)
  __shared__ int s_tdone;              // T items published (4 per step)
  const int t = threadIdx.x, w = t >> 6;
  const bool panel = p > 0;
  // forward fold: z_{c-1} staged in the D buffers during the pre-update; r_i of a p > 0 workgroup in the area after the
  // D buffers; for p = 0 (which never uses sP) r_c, z_s and z_c in sP
  double* sZ = sDb;
  double* sR = panel ? sDb + DBUF : sP;
  double* sZall = sP + NB * GPX_MAX_RHS;
  double* sZs = sZall + NB * GPX_MAX_RHS;  // one 16 x NR slot per wave 1..3
  static_assert(NB * GPX_MAX_RHS <= DBUF && 2 * NB * GPX_MAX_RHS + 3 * 16 * GPX_MAX_RHS <= NB * LD64, "fold LDS");
  const int nrow = panel ? 4 + PROWS / 16 : 4;  // 16-row blocks of the tall panel
  const int bi = c + p;
  const int row0 = bi * NB + PROWS * h;  // first global row of this workgroup's A_ic rows
  const double* Acc = A + (int64_t)c * NB * lda + (int64_t)c * NB;
  double* Aic = A + (int64_t)row0 * lda + (int64_t)c * NB;
  if (t == 0) s_tdone = 0;
  int fail = -1;
  bool f0 = false;  // pivot block 0 already factored by the pre-update (wave 0)
  if (c > 0) {
    // the updates of block columns c0 .. c-1 not yet applied to this column, on the two tiles this workgroup
    // factors (K = 64 (c - c0))
    const int kk = (c - c0) * NB;
    const double* Lc = A + (int64_t)c * NB * lda + (int64_t)c0 * NB;
    const double* Li = A + (int64_t)row0 * lda + (int64_t)c0 * NB;
    if (kk == NB) {
      if (ov) {
        if (panel)
          update_eager<true, true, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, sDb, c, row0, f, sZ, sR, fail);
        else
          update_eager<true, false, NR, 1>(Acc, Aic, Lc, Li, lda, sA, sP, sDb, c, c * NB, f, sZ, sR, fail);
        f0 = true;
      } else {
        if (panel)
          update_eager<false, true, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, sDb, c, row0, f, sZ, sR, fail);
        else
          update_eager<false, false, NR, 1>(Acc, Aic, Lc, Li, lda, sA, sP, sDb, c, c * NB, f, sZ, sR, fail);
      }
    } else {
      // (never split: the host splits panels only in schedules whose panels apply one column)
      // (the host folds the forward substitution only into schedules whose panels apply one column: kk == NB)
      Tile64 tl;
      update_to_lds(tl, Acc, lda, Lc, Lc, lda, kk, smem, sA);
      if (panel) {
        __syncthreads();  // smem reuse
        update_to_lds(tl, Aic, lda, Li, Lc, lda, kk, smem, sP);
      }
    }
  } else {
    load_tile_lds(Acc, lda, sA);
    if (panel) load_tile_lds<PROWS>(Aic, lda, sP);
    if constexpr (NR > 0) {
      if (!panel)
        for (int e = t; e < NB * NR; e += WG) sR[e] = fwd_y(f, e / NR, e % NR);  // r_0 = (Y - mean)_0
    }
  }
  __syncthreads();
  GPX_PANEL_STAMP(0);
  auto rows = [&](int i) -> double* { return i < 4 ? sA + 16 * i * LD64 : sP + 16 * (i - 4) * LD64; };
  // T: L_is = A_is D_ss^T (16x16x16 on MFMA, in place)
  auto tsolve = [&](int i, const double* D, int o) {
    double* R = rows(i);
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = mfma_lds16<true, LDD>(acc, R, 0, o, D, 0, 0, 16, 1.0);
    store_block16(R, 0, o, acc);
  };
  // U: A_ij -= L_is L_js^T
  auto update = [&](int i, int j, int o) {
    double* Ri = rows(i);
    d4 acc = load_block16(Ri, 0, 16 * j);
    acc = mfma_lds16<true>(acc, Ri, 0, o, rows(j), o, 0, 16, -1.0);
    store_block16(Ri, 0, 16 * j, acc);
  };
  // one increment per wave (lane 0); the release orders the wave's LDS stores before it
  auto publish = [&]() {
    if ((t & 63) == 0) __hip_atomic_fetch_add(&s_tdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  for (int s = 0; s < 4; ++s) {
    const int o = 16 * s;
    double* D = sDb + (s & 1) * 16 * LDD;
    if (w == 0 && (s > 0 || !f0)) {
      // (4-pivot blocks on v_mfma_f64_16x16x4, tools/chol16_probe.hip: correct, but measured slower inside the panel,
      // potrf 1.89 vs 1.76 ms at n = 4096: ~75 instructions per pivot and MFMA / ds_bpermute latency on the chain)
      const int f = chol16<LDD>(sA, D, o);
      if (f >= 0 && fail < 0) fail = o + f;
    }
    GPX_PANEL_STAMP(1 + 3 * s);
    if (s > 0 || !f0) __syncthreads();  // publishes L_ss and D_ss (step 0 after a pre-update: published already)
    if (w == 0) {
      // Critical path, no barrier: T and U of the next pivot block, then straight on to its F.
      if (s + 1 < nrow) tsolve(s + 1, D, o);  // at s = 3 this is the first panel row block
      publish();
      GPX_PANEL_STAMP(2 + 3 * s);
      if (s < 3) update(s + 1, s + 1, o);
    } else {
      // Waves 1-3: the remaining T items (row blocks s+2.. and the panel rows), then - once every wave's T items of
      // this step are published - the remaining U items, overlapping wave 0's next F.
      for (int i = s + 1 + w; i < nrow; i += 3) tsolve(i, D, o);
      publish();
      GPX_PANEL_STAMP(2 + 3 * s);
      while (__hip_atomic_load(&s_tdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 4 * (s + 1))
        __builtin_amdgcn_s_sleep(1);
      int e = 0;
      for (int j = s + 1; j < 4; ++j) {
        for (int i = j; i < nrow; ++i) {
          if (i == s + 1 && j == s + 1) continue;  // wave 0's lookahead item
          if (1 + e % 3 == w) update(i, j, o);
          ++e;
        }
      }
      if constexpr (NR > 0) {
        if (!panel) fwd_pivot_step<NR>(s, w, D, sA, sR, sZs, sZall);
      }
    }
    GPX_PANEL_STAMP(3 + 3 * s);
  }
  __syncthreads();
  GPX_PANEL_STAMP(13);
  if (!panel) {
    if (t == 0 && fail >= 0) atomicCAS(info, 0, c * NB + fail + 1);
    double* Lcc = Dinv + (int64_t)(nblk + c) * NB * NB;  // scratch copy, moved into A by potrf_dinv
    double* isq = sDb;  // the D buffers are free after the last step
    l64_isq(sA, isq);
    __syncthreads();
    for (int e = t; e < NB * NB; e += WG) Lcc[e] = l64_at(sA, isq, e >> 6, e & 63);
    if constexpr (NR > 0) {
      for (int e = t; e < NB * NR; e += WG) f.z[(int64_t)c * NB * NR + e] = sZall[e];
    }
    return;
  }
  const rsrc_t ra = buf_rsrc(Aic);
#pragma unroll
  for (int q = 0; q < PROWS / 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, cc = e & 63;
    st2_sc1(ra, (int)(((int64_t)r * lda + cc) * 8), sP[r * LD64 + cc], sP[r * LD64 + cc + 1]);
  }
  if constexpr (NR > 0) {
    if (c > 0)
      for (int e = t; e < PROWS * NR; e += WG) f.r[(int64_t)row0 * NR + e] = sR[e];
  }
}

// Trailing workgroup of a flush launch c: 128x128 tile `tile` of the lower triangle of block columns >= cfirst,
// A_ij -= sum_{k = k0}^{c-1} L_ik L_jk^T (K = 64 (c - k0)).  The 128-grid is aligned to the end of the matrix
// (first 64-block c0 = nblk - 2M); when it starts at block c, that block row/column is computed but not stored (it
// belongs to this launch's panel).
// Trailing workgroup t of T -> 128-tile (I, J) of the M x M lower grid.  xmap = 0: row-major tile order.  xmap = 1:
// the tiles in 8 x 8 super-block order, dealt to the XCDs in contiguous chunks (workgroups t, t+8, ... share an XCD:
// round-robin dispatch, speed only, never correctness), so an XCD's tiles read ~16 L panels through its L2 instead of
// all of them beside the C stream; the chunking is the bijective XCD swizzle of cdna_hip_programming.md section 5.
__device__ __forceinline__ void trail_tile(int t, int T, int M, int xmap, int& I, int& J) {
  if (!xmap) {
    tri_decode(t, I, J);
    return;
  }
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
  I = J = 0;  // not reached: p < T
}

// acc = -C for an MfmaTile whose origin is C (row-major, leading dimension ld) through buffer loads: the lane's row / column
// offset in one VGPR, each (i, r) row step wave-uniform (soffset) and each 16-column step an immediate, so the 64 seed loads
// need no address registers.  (16-byte pair loads + a DPP lane swap, half the load instructions, spilled 9-12 VGPRs and
// measured slower: update 1.684 vs 1.633 ms at n = 4096, profiles/r05_seed_ab.log.)
template <typename T>
__device__ __forceinline__ void load_neg_c_buf(T& tl, rsrc_t rc, int64_t ld) {
  const int v0 = (int)(((int64_t)T::row_of(0, 0) * ld + T::col_of(0)) * 8);
#pragma unroll
  for (int i = 0; i < T::WM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int so = (int)((int64_t)(16 * i + 4 * r) * ld * 8);
#pragma unroll
      for (int j = 0; j < T::WN; ++j)
        tl.acc[i][j][r] = -__builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, v0 + 128 * j, so, 0));
    }
}

// The 128 x TN tile with origin at 64-block (r0, q0): A -= sum_{k = k0}^{c-1} L_{r0..,k} L_{q0..,k}^T (TN = 128, or 64 for
// the half tiles that end a long flush, StepPlan::nsplit).
// Schedule-invariant arithmetic: the accumulator is SEEDED with -C and every product added onto it in the k order of the
// column blocks, so an element after columns k0..c-1 is the same MFMA chain whether those columns were applied one launch
// at a time (eager), all at once (a lookahead flush), by the panel's own pre-update (seeded +C with the A operand negated:
// round(C - ab) = -round(-C + ab)) or by a lookahead tile.  The factor, z and alpha are therefore bit-identical under every
// schedule, batch size and GPX_OPT_POTRF_* option (tests/test_gpu_parity.py).  (Round 4 subtracted a from-zero product in
// the epilogue, C - sum, whose rounding depended on how many columns a flush grouped.)
// The 128 x 128 tiles run the hand-placed k loop of gpx_trmm_asm.h (both operands row-major: L panels), seeded with +C and
// subtracting through the MFMA's A negation (the panel pre-update's form); the 128 x 64 halves keep MfmaTile, seeded with
// -C and stored negated.  Both give every element the same MFMA chain, so the same bits.
template <int TN>
__device__ __forceinline__ void trailing_tile_at(double* __restrict__ A, int64_t lda, int c, int k0, int cfirst, int r0,
                                                 int q0, double* lds) {
  const double* Li = A + (int64_t)r0 * NB * lda + (int64_t)k0 * NB;
  const double* Lj = A + (int64_t)q0 * NB * lda + (int64_t)k0 * NB;
  double* C = A + (int64_t)r0 * NB * lda + (int64_t)q0 * NB;
  using TileT = MfmaTile<2 * NB, TN, 16, false, false>;  // (the accumulator layout of both forms)
  const rsrc_t rc = buf_rsrc(C);
  d4 acc[TileT::WM][TileT::WN];
  if constexpr (TN == 2 * NB) {
    trmm_asm::TileT<false, false, true> tl;
    tl.template run_after<false, false, TileT::WM * TileT::WN * 4>(
        Li, lda, Lj, lda, (c - k0) * (NB / 16), lds, [&] {
          const int v0 = (int)(((int64_t)TileT::row_of(0, 0) * lda + TileT::col_of(0)) * 8);
#pragma unroll
          for (int i = 0; i < TileT::WM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int so = (int)((int64_t)(16 * i + 4 * r) * lda * 8);
#pragma unroll
              for (int j = 0; j < TileT::WN; ++j)
                tl.acc[i][j][r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, v0 + 128 * j, so, 0));
            }
        });
#pragma unroll
    for (int i = 0; i < TileT::WM; ++i)
#pragma unroll
      for (int j = 0; j < TileT::WN; ++j) acc[i][j] = tl.acc[i][j];
  } else {
    TileT tl;
    tl.template run_acc_after<true>(Li, lda, Lj, lda, 0, (c - k0) * NB, lds, [&] { load_neg_c_buf(tl, rc, lda); });
#pragma unroll
    for (int i = 0; i < TileT::WM; ++i)
#pragma unroll
      for (int j = 0; j < TileT::WN; ++j) acc[i][j] = -tl.acc[i][j];
  }
#pragma unroll
  for (int i = 0; i < TileT::WM; ++i) {
    // write-through 16-byte pairs; a 16-column pair never straddles a 64-block, and rows r = 0, 1 (even lanes) or 2, 3
    // (odd lanes) of one lane lie in one 64-row block
#pragma unroll
    for (int j = 0; j < TileT::WN; ++j) {
      const int cb = q0 + (TileT::col_of(j) >> 6);
      const bool colok = cb >= cfirst;
      const bool k01 = colok && r0 + (TileT::row_of(i, 0) >> 6) >= cb;
      const bool k23 = colok && r0 + (TileT::row_of(i, 2) >> 6) >= cb;
      store_block_pairs_sc1<TileT>(rc, lda, i, j, acc[i][j], k01, k23);
    }
  }
}

// Trailing workgroup p of a launch: tiles 0 .. ntile - nsplit - 1 whole, the last nsplit tiles as two 128 x 64 halves
// (workgroups ntile - nsplit + 2h + half).
__device__ __forceinline__ void trailing_role(double* __restrict__ A, int64_t lda, int c, int nblk, int k0, int cfirst,
                                              int p, int ntile, int nsplit, int xmap, double* lds) {
  const int M = (nblk - cfirst + 1) / 2, c0 = nblk - 2 * M;
  const int nwhole = ntile - nsplit;
  int I, J;
  if (p < nwhole) {
    trail_tile(p, ntile, M, xmap, I, J);
    trailing_tile_at<2 * NB>(A, lda, c, k0, cfirst, c0 + 2 * I, c0 + 2 * J, lds);
  } else {
    const int h = p - nwhole;
    trail_tile(nwhole + (h >> 1), ntile, M, xmap, I, J);
    trailing_tile_at<NB>(A, lda, c, k0, cfirst, c0 + 2 * I, c0 + 2 * J + (h & 1), lds);
  }
}

// Lookahead workgroup (mode 1) of launch c: tile (c+1+idx, c+1) of the next panel's column gets every pending
// update, A_i,c+1 -= sum_{k = a}^{c-1} L_ik L_{c+1,k}^T with a = the first column no flush has applied to it, so
// that the panels always apply exactly one column (K = 64 on the critical path) while the bulk of the trailing
// matrix is flushed every `lazy` launches.
__device__ __forceinline__ void lookahead_role(double* __restrict__ A, int64_t lda, int c, int a, int idx, double* lds) {
  const int i = c + 1 + idx, j = c + 1;
  const double* Li = A + (int64_t)i * NB * lda + (int64_t)a * NB;
  const double* Lj = A + (int64_t)j * NB * lda + (int64_t)a * NB;
  double* C = A + (int64_t)i * NB * lda + (int64_t)j * NB;
  Tile64 tl;
  tl.load_neg_c(C, lda);
  // K = 64 (c - a) up to 64 g in k-tiles of 16 with LA = 4 k-tiles of loads in flight (register stages st[]): a k-tile's
  // 16 MFMAs per wave (~0.4 us) cover far less than a load round trip, so MfmaTile's one-ahead prefetch left this
  // (latency-bound, few workgroups) tile waiting on every k-tile.  One barrier per k-tile, LDS double-buffered.  Same
  // MFMA order, same bits.  n = 16384 update 30.09 -> 29.95 ms, n = 8192 5.88 -> 5.84 (LA = 8: 30.15 / 5.87,
  // profiles/r04_lookahead_prefetch_ab.log).
  constexpr int LA = 4;
  const int nk = (c - a) * (NB / 16);  // a multiple of 4
  Tile64 st[LA];
  double* buf0 = lds;
  double* buf1 = lds + 16 * (Tile64::PA + Tile64::PB);
#pragma unroll
  for (int q = 0; q < LA; ++q) st[q].load_regs(Li, lda, Lj, lda, 16 * q);
  for (int k0 = 0; k0 < nk; k0 += LA) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int kt = k0 + q;
      double* cur = (q & 1) ? buf1 : buf0;
      st[q].store_lds(cur, cur + 16 * Tile64::PA);
      __syncthreads();
      if (kt + LA < nk) st[q].load_regs(Li, lda, Lj, lda, 16 * (kt + LA));
      tl.compute(cur, cur + 16 * Tile64::PA);
    }
  }
  __syncthreads();  // the last k-tile's LDS reads before the workgroup's next use of lds
  const rsrc_t rc = buf_rsrc(C);
#pragma unroll
  for (int ii = 0; ii < Tile64::WM; ++ii)
#pragma unroll
    for (int jj = 0; jj < Tile64::WN; ++jj) {
      const d4 v = -tl.acc[ii][jj];
      store_block_pairs_sc1<Tile64>(rc, lda, ii, jj, v, true, true);
    }
}

// Work split of launch c.  Flush launches (plan.flush) apply the columns k0 .. c-1 (k0 = the previous flush launch, or 0)
// to the trailing matrix.  mode 0: the panels apply the pending columns c0 = k0 .. c-1, the flush covers columns >= c+1.
// mode 1: the panels apply column c-1 only, lookahead workgroups bring column c+1 up to date (columns look_a = k0 ..
// c-1), the flush covers columns >= c+2.  The host decides which launches flush (potrf_flush_interval).
struct StepPlan {
  int npanel, nlook, ntrail, c0, look_a, cfirst, k0, flush;
  int tbase, xmap;  // first trailing workgroup (a multiple of 8 when xmap: XCD-chunked tile order), tile order
  int split;        // panel row blocks c+1.. split into 1, 2 or 4 workgroups (panel workgroup b > 0: p = 1 + (b-1) / split)
  int overlap;      // the panels' first pivot block factored under their pre-update (update_eager OV)
  int nsplit;       // the last nsplit trailing tiles run as two 128 x 64 halves each (ntrail + nsplit trailing workgroups)
};

// slots > 0: the co-resident workgroup slots a problem may fill (two per CU, shared by a batch); the panel row blocks are
// split in 2 (StepPlan::split) when the panels apply exactly one column and the split launch still fits the slots.
// split_policy (GPX_OPT_POTRF_SPLIT): -1 split where the launch fits the slots, 1 never, 3 only where it fits one
// workgroup per CU (slots / 2), so that panel workgroups do not share a CU with lookahead / trailing ones
inline StepPlan step_plan(int c, int nblk, int mode, int last_flush, bool flush, int xmap = 0, int slots = 0,
                          int split_policy = -1) {
  StepPlan s;
  s.npanel = nblk - c;
  s.split = 1;
  s.flush = flush ? 1 : 0;
  s.k0 = last_flush;
  if (mode == 0) {
    s.c0 = c > 0 ? last_flush : 0;
    s.nlook = 0;
    s.look_a = 0;
    s.cfirst = c + 1;
  } else {
    s.c0 = c > 0 ? c - 1 : 0;
    s.nlook = (c >= 1 && c + 1 < nblk) ? nblk - c - 1 : 0;
    s.look_a = last_flush;
    s.cfirst = c + 2;
  }
  const int m = nblk - s.cfirst;
  const int M = (flush && m > 0) ? (m + 1) / 2 : 0;
  s.ntrail = M * (M + 1) / 2;
  s.xmap = xmap;
  const bool eager = mode == 1 || c == 0 || c - last_flush == 1;
  if (slots > 0 && eager && s.npanel > 1 && split_policy != 1) {
    const int room = split_policy == 3 ? slots / 2 : slots;
    for (int sp = 2; sp >= 2; sp >>= 1) {  // split 4 measured slower at n = 4096 (potrf 1.48 vs 1.46 ms), equal below
      const int np = 1 + sp * (s.npanel - 1);
      const int tb = xmap ? (np + s.nlook + 7) & ~7 : np + s.nlook;
      if (tb + s.ntrail <= room) {
        s.split = sp;
        s.npanel = np;
        break;
      }
    }
  }
  s.tbase = xmap ? (s.npanel + s.nlook + 7) & ~7 : s.npanel + s.nlook;  // padding workgroups exit at once
  // the overlapped pre-update shortens the panel chain but slows launches whose trailing workgroups do not all fit
  // the co-resident slots at once (DESIGN_HISTORY.md)
  s.overlap = slots > 0 && s.tbase + s.ntrail <= slots;
  // A long flush (K >= 256) of T tiles over S slots ends with a partial round of T mod S tiles; when that remainder fills
  // at most half the slots, its tiles run as 128 x 64 halves, so the last round takes about half a tile time
  s.nsplit = 0;
  if (slots > 0 && flush && c - last_flush >= 4) {
    const int r = s.ntrail % slots;
    if (r > 0 && 2 * r <= slots) s.nsplit = r;
  } else if (slots > 0 && flush) {
    // an eager launch (K = 64) that overflows the co-resident slots by a few tiles (n = 4096, c = 1..4: 63 panels +
    // 496 tiles over 512 slots) would run them as a second round of whole tiles: halves instead
    const int over = s.tbase + s.ntrail - slots;
    if (over > 0 && 4 * over <= slots) s.nsplit = over < s.ntrail ? over : s.ntrail;
  }
  return s;
}

// NR: 0 = no forward fold, else its right-hand-side row length (one instantiation each: the fold's registers stay out
// of the plain kernel)
template <int NR>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2)))
potrf_step_kernel(double* __restrict__ A, int64_t lda, int c, int nblk, StepPlan s, double* __restrict__ Dinv,
                  int32_t* __restrict__ info, int first_wg, int64_t sa, int64_t sd, PotrfFwd f) {
  A += blockIdx.y * sa;  // problem of a batched fit
  Dinv += blockIdx.y * sd;
  info += blockIdx.y;
  if (*(volatile int32_t*)info != 0) return;  // an earlier step failed: leave the rest untouched
  __shared__ __attribute__((aligned(16))) double lds[STEP_LDS];
  const int b = first_wg + (int)blockIdx.x;
  if (b >= s.npanel + s.nlook && b < s.tbase) return;  // alignment padding of the trailing workgroups
  const int role = b < s.npanel ? 0 : (b < s.npanel + s.nlook ? 1 : 2);
  GPX_STEP_STAMP(role, c, b, 0);
  if (role == 0) {
    if constexpr (NR > 0) {
      f.Y += blockIdx.y * f.sy;
      if (f.means) f.mean = f.means[blockIdx.y];
      f.r += blockIdx.y * f.sb;
      f.z += blockIdx.y * f.sb;
    }
    if (s.split == 2 && b > 0)
      panel_role<NR, 2>(A, lda, c, 1 + ((b - 1) >> 1), (b - 1) & 1, nblk, s.c0, Dinv, info, lds, f, s.overlap);
    else
      panel_role<NR, 1>(A, lda, c, b, 0, nblk, s.c0, Dinv, info, lds, f, s.overlap);
  } else if (role == 1)
    lookahead_role(A, lda, c, s.look_a, b - s.npanel, lds);
  else
    trailing_role(A, lda, c, nblk, s.k0, s.cfirst, b - s.tbase, s.ntrail, s.nsplit, s.xmap, lds);
  GPX_STEP_STAMP(role, c, b, 1);
}

// L_kk from the scratch into A, and D_k = L_kk^{-1} into the first half of Dinv (one workgroup per block).
__global__ void __launch_bounds__(WG) potrf_dinv_kernel(double* __restrict__ A, int64_t lda, int nblk,
                                                        double* __restrict__ Dinv, const int32_t* __restrict__ info,
                                                        int64_t sa, int64_t sd, int k0, double* __restrict__ W,
                                                        int64_t ldw, int64_t sw) {
  A += blockIdx.y * sa;
  Dinv += blockIdx.y * sd;
  info += blockIdx.y;
  if (*(volatile const int32_t*)info != 0) return;
  __shared__ __attribute__((aligned(16))) double sL[NB * LD64];
  __shared__ __attribute__((aligned(16))) double sX[NB * LD64];
  __shared__ __attribute__((aligned(16))) double sT[NB * LD64];
  const int k = k0 + (int)blockIdx.x, t = threadIdx.x;
  const double* src = Dinv + (int64_t)(nblk + k) * NB * NB;
  double* Lkk = A + (int64_t)k * NB * lda + (int64_t)k * NB;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, c = e & 63;
    const double2 v = *reinterpret_cast<const double2*>(src + r * NB + c);
    *reinterpret_cast<double2*>(Lkk + (int64_t)r * lda + c) = v;
    sL[r * LD64 + c] = v.x;
    sL[r * LD64 + c + 1] = v.y;
  }
  __syncthreads();
  trinv64(sL, sX, sT);
  double* D = Dinv + (int64_t)k * NB * NB;
  for (int e = t; e < NB * NB; e += WG) D[e] = sX[(e >> 6) * LD64 + (e & 63)];
  if (W) {  // trtri_diag's work for a fit: W_kk = D_k^T, and the strictly-lower 64-block of an odd 128-tile zeroed
    W += blockIdx.y * sw;
    double* Wkk = W + (int64_t)k * NB * ldw + (int64_t)k * NB;
    for (int e = t; e < NB * NB; e += WG) Wkk[(int64_t)(e >> 6) * ldw + (e & 63)] = sX[(e & 63) * LD64 + (e >> 6)];
    if (k & 1) {
      double* Z = W + (int64_t)k * NB * ldw + (int64_t)(k - 1) * NB;
      for (int e = t; e < NB * NB; e += WG) Z[(int64_t)(e >> 6) * ldw + (e & 63)] = 0.0;
    }
  }
}

// Trailing updates are flushed every `lazy` launches (K = 64 lazy per flush): C tiles are read and written once per
// `lazy` block columns instead of every column, and the panel workgroups apply the (at most `lazy`) pending columns
// to their own tiles.  Schedule by size (tools/lazy_sweep.sh, profiles/r01_potrf_lazy_sweep*.log):
//   n = 4096:  mode 0, g = 1 -> potrf 1.73-1.75 ms (mode 1 g = 2/4: 1.81/1.94: a K = 128 flush tile is >= 14 us of
//              MFMA on one CU, longer than the ~20 us panel window once two share a CU);
//   n = 8192:  mode 1, g = 4 -> 6.34 ms (mode 0 g = 2: 6.69); round 4, with the half-tile flush tails: g = 6 5.83 ms
//              against g = 4 / 7 / 8: 5.90 / 5.96 / 5.95 (profiles/r04_lazy_interval_ab.log), while n = 6000 (94 blocks)
//              keeps g = 4 (3.165 vs 3.179 / 3.183 ms for g = 5 / 6) and n = 16384 g = 8 (30.16 vs 30.60 / 30.31 for
//              g = 6 / 10);
//   n = 16384: mode 1, g = 8 -> 31.4 ms (mode 0 g = 4: 34.4, g = 1: 46.3).
// Batched fits share the co-resident slots, so the per-launch panel chain is hidden under more trailing work and the
// eager schedule's C traffic dominates: the lookahead schedule wins (profiles/r04_batched_lazy_sweep.log, update ms,
// eager g = 1 -> mode 1 g = 4 / 6) at 64 blocks for B = 2 2.313 -> 2.186 / 2.207, B = 3 2.991 -> 2.784 / 2.792, B = 4
// 3.778 -> 3.326 / 3.287, B = 8 6.92 -> 5.56 / 5.43; at 56 blocks B = 2 1.778 -> 1.739 / 1.744, B = 4 2.747 -> 2.543 /
// 2.524; at 48 blocks B = 4 1.962 -> 1.895 / 1.863 (B = 2 1.350 -> 1.342, kept eager); at 40 and 32 blocks the eager
// schedule stays best (B = 2 / 4).  At 80–96 blocks g = 6 beats 4 / 8 for B = 2 / 4 (n = 6144 B = 4: 8.09 vs 8.34 / 8.11,
// B = 2: 4.86 vs 4.92 / 4.91; n = 5120 B = 4: 5.28 vs 5.41 / 5.30), at 128 blocks g = 8 beats 6 (B = 2: 9.28 vs 9.34,
// B = 4: 16.37 vs 16.53 ms).
// The handle options GPX_OPT_POTRF_LAZY / GPX_OPT_POTRF_MODE override.  Flushing every second launch only in the early,
// trailing-bound launches and panel-wave priority were measured neutral (DESIGN_HISTORY.md, items 14 and the prio knob)
// and are not offered.  Trailing tiles are dealt to the XCDs in 8 x 8 super-block chunks (trail_tile xmap = 1).
// Round 6 (profiles/r06_small_batched_schedule_ab.log, one process, alternating arms): batches of 8 take the lookahead
// schedule (g = 6) from 24 blocks on as well - the drop-in's 8-output fits below the SVGP threshold (n <= 3000) - :
// n = 1536 / 2048 / 2560 0.822 -> 0.767, 1.360 -> 1.248, 2.153 -> 1.908 ms (eager for the last 16 columns only from
// 40 blocks on: 2048 with it 1.262, 2560 without it 1.927); 16 blocks (n = 1024) and B = 4 at 32 blocks stay eager.
static bool batched_lookahead(int nblk, int batch) {
  return nblk <= 64 && ((batch >= 2 && nblk >= 56) || (batch >= 4 && nblk >= 48) || (batch >= 8 && nblk >= 24));
}

static int potrf_lazy(const Context* ctx, int nblk, int batch) {
  if (ctx->potrf_lazy > 0) return ctx->potrf_lazy;
  if (batched_lookahead(nblk, batch)) return batch >= 4 ? 6 : 4;
  if (batch >= 2 && nblk > 64) return nblk > 100 ? 8 : 6;
  // round 6 (profiles/r06_potrf_n16384_schedule_ab.log, one process, alternating arms): n = 16384 flushes every 12
  // columns (K = 768), eager for the last ~51: 28.11-28.16 vs 28.56-28.63 ms for 8 / the last 39 (10: 28.30-28.35, 13:
  // 28.31, 14: 28.21, 16: 28.39); n = 12288 (g = 10 / 12: 13.95 / 14.03 vs 13.98) and n = 8192 (g = 8 / 10 / 12: 5.53 /
  // 5.58 / 5.67 vs 5.54) keep theirs
  return nblk > 192 ? 12 : (nblk > 128 ? 8 : (nblk > 100 ? 6 : (nblk > 64 ? 4 : 1)));
}

static int potrf_mode(const Context* ctx, int nblk, int batch) {
  if (ctx->potrf_mode == 0 || ctx->potrf_mode == 1) return ctx->potrf_mode;
  return nblk > 64 || batched_lookahead(nblk, batch) ? 1 : 0;
}

// A single fit of 64 blocks runs its first launches (c < 25) on the lookahead schedule with a flush every 3 columns and
// switches to the eager schedule right after the flush at c = 24 (the eager launch c then applies column c - 1 to the
// panels and the trailing matrix: every column is applied exactly once).  Round 6 (profiles/r06_potrf_switch_ab.log, one
// process, alternating arms, alpha bit-identical): switch 25 / g 3 1.5472 vs 1.5666 ms for round 5's switch 9 / g 4
// (1.5542 vs 1.5670 in a second sweep; 22 / 3 1.5547, 28 / 3 1.5554, 31 / 3 1.5644, 25 / 2 1.5615, 25 / 4 1.5597,
// 25 / 6 1.5539, 33 / 2 1.5849; the same start at n = 3072 / 3584 / 5120 measured neutral or slower,
// profiles/r06_potrf_midn_schedule_ab.log): in launches 9-24 the eager schedule moved the whole trailing matrix every
// column and the panel waited on that traffic (profiles/r06_potrf_steps_4096_switch9.log: pre-update 17-22 us there,
// ~6 in the tail).
// Round 4 introduced the switch: the early launches are bound by the eager schedule's C traffic (launches 1-4: 39-42 us
// against ~17 us of panel chain, profiles/r04_potrf_launches_4096.log):
// update 1.617 -> 1.596 ms at n = 4096 (profiles/r04_potrf_hybrid_ab.log; switch at c = 5 / 9 / 13 / 17 / 25 / 33 with
// g = 4: 1.596 / 1.596-1.602 / 1.602 / 1.616 / 1.618 / 1.630 vs 1.616-1.619; g = 2 / 8 no better; the kept form 1.599 vs
// 1.616).  Smaller fits keep the eager schedule throughout: the same switch at n = 2048 / 3072 / 3584 gave 0.683 / 1.058
// / 1.325 vs 0.667 / 1.060 / 1.311 ms.
// The other way round, a single fit above 64 blocks (lookahead schedule) switches to the eager schedule for its last
// ~32 block columns (after the last flush launch before nblk - 32): there the trailing matrix is small and the eager
// launches' panel chain is the shorter one (profiles/r04_potrf_eager_tail_ab.log: n = 8192 5.832 -> 5.720 ms with the
// last 32, 5.811 -> 5.748 with 24, 5.796 -> 5.731 with 48; n = 16384 29.865 -> 29.715 with 32).
constexpr int kEagerTail = 32;
constexpr int kSwitchLazy = 3;  // the flush interval before the switch (the switch launch follows a flush launch)
// flush interval of the launches before the switch: mode 0 (eager after it) kSwitchLazy or GPX_OPT_POTRF_LAZY when the
// switch is set by option; mode 1 (lookahead before it) the schedule's own interval g
static int early_lazy(const Context* ctx, int mode, int g) {
  if (mode != 0) return g;
  return (ctx->potrf_switch >= 0 && ctx->potrf_lazy > 0) ? ctx->potrf_lazy : kSwitchLazy;
}
static int potrf_switch(const Context* ctx, int nblk, int batch, int mode, int g) {
  if (ctx->potrf_switch >= 0) {  // GPX_OPT_POTRF_SWITCH, rounded down to the launch after a flush of the early schedule
    const int ge = early_lazy(ctx, mode, g);  // (the fold needs the eager panels to apply one column)
    const int sw = ctx->potrf_switch;
    return sw <= 1 ? sw : ((sw - 1) / ge) * ge + 1;
  }
  if (ctx->potrf_mode >= 0 || ctx->potrf_lazy > 0) return 0;
  if (batch != 1) {
    // batches on the lookahead schedule finish on the eager one for their last ~16 block columns (B = 4, n = 4096:
    // 3.195 -> 3.149 ms with the switch at 49, 3.153 at 37, 3.219 at 25; profiles/r05_potrf_schedules.log): the
    // launch after the last flush at or before nblk - 16 for B >= 4 (g = 6: 49 vs 43 3.118 vs 3.135 ms in a sweep, 3.155 vs 3.165 B = 4 and 5.353 vs 5.362 B = 8 in an A/B,
    // profiles/r05_potrf_batched_switch_ab.log), one launch earlier for B = 2 (g = 4: 45; 49 measured 2.138 vs 2.133)
    if (!batched_lookahead(nblk, batch) || nblk < 40) return 0;
    return ((nblk - (batch >= 4 ? 16 : 17)) / g) * g + 1;
  }
  if (mode == 0) return nblk == 64 ? 25 : 0;
  const int tail = g >= 12 ? 48 : kEagerTail;  // (n = 16384, g = 12: the eager part from c = 205)
  if (nblk - tail < g + 1) return 0;
  return ((nblk - tail - 1) / g) * g + 1;
}

// The plan of every launch c < cend (flush launches: c >= 1 and at least one interval after the previous flush);
// launches c < sw (potrf_switch) run the lookahead schedule, the rest the eager one with a flush every launch.
template <typename F>
static void for_each_step(const Context* ctx, int nblk, int batch, int mode, int cend, int slots, F&& f) {
  const int g = potrf_lazy(ctx, nblk, batch);
  const int sw = potrf_switch(ctx, nblk, batch, mode, g);
  const int ge = early_lazy(ctx, mode, g);
  int last = 0;
  for (int c = 0; c < cend; ++c) {
    const bool early = c < sw;
    const bool flush = c >= 1 && c - last >= (early ? ge : (sw > 0 ? 1 : g));
    // flushes of K >= 384 take their tiles row-major (xmap 0): n = 16384 (K = 512) 28.78 -> 28.60 ms (the 8 x 8 XCD
    // chunks serve the shorter tiles' L2 reuse; a K = 512 chunk's 16 panels are 8 MB, twice an XCD's L2;
    // profiles/r05_flush_order_ab.log, tools/flush_asm_bench.hip A4 0.828 vs A1 0.809 of peak); K = 384: n = 8192
    // 5.673 -> 5.629 ms, B = 4 x n = 4096 3.169 -> 3.163 (profiles/r05_flush_order_384_ab.log).  The n = 4096 K = 256
    // flush (one round of 465 tiles) keeps the chunks: 87.5 vs 106 us row-major (profiles/r05_potrf_launches_4096.log)
    const int xmap = (flush && c - last >= 6) ? 0 : 1;
    f(c, step_plan(c, nblk, early ? 1 : (sw > 0 ? 0 : mode), last, flush, xmap, slots, ctx->potrf_split));
    if (flush) last = c;
  }
}

// Co-resident workgroup slots per problem (two per CU at the step kernel's LDS size, shared by the batch), or 0 when
// the device cannot be queried (no half-panel split then).
static int potrf_slots(Context* ctx, int batch) {
  if (ctx->cu_count <= 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    ctx->cu_count = cus;
  }
  return 2 * ctx->cu_count / (batch > 0 ? batch : 1);
}

static void launch_steps(Context* ctx, int nblk, double* A, int64_t lda, double* Dinv, int32_t* info, const Batch& bt,
                         int cbeg, int cend, const PotrfFwd& f = PotrfFwd()) {
  const int mode = potrf_mode(ctx, nblk, bt.count);
  for_each_step(ctx, nblk, bt.count, mode, cend, potrf_slots(ctx, bt.count), [&](int c, const StepPlan& s) {
    if (c < cbeg) return;
    const dim3 grid(s.tbase + s.ntrail + s.nsplit, bt.count);
    if (!f.r)
      potrf_step_kernel<0><<<grid, WG, 0, ctx->stream>>>(A, lda, c, nblk, s, Dinv, info, 0, bt.k, bt.dinv, f);
    else if (f.nrhs == 1)
      potrf_step_kernel<1><<<grid, WG, 0, ctx->stream>>>(A, lda, c, nblk, s, Dinv, info, 0, bt.k, bt.dinv, f);
    else
      potrf_step_kernel<GPX_MAX_RHS><<<grid, WG, 0, ctx->stream>>>(A, lda, c, nblk, s, Dinv, info, 0, bt.k, bt.dinv, f);
  });
}

static void launch_dinv(Context* ctx, int nblk, double* A, int64_t lda, double* Dinv, int32_t* info, const Batch& bt,
                        int k0, int k1, double* W = nullptr, int64_t ldw = 0) {
  potrf_dinv_kernel<<<dim3(k1 - k0, bt.count), WG, 0, ctx->stream>>>(A, lda, nblk, Dinv, info, bt.k, bt.dinv, k0, W, ldw,
                                                                      bt.w);
}

hipError_t launch_potrf(Context* ctx, int npad, double* A, int64_t lda, double* Dinv, int32_t* info, const Batch& bt,
                        double* W, int64_t ldw, const ForwardRhs* fr, bool* z_done) {
  LaunchTimer tm(ctx, GPX_TIMER_POTRF);
  const int nblk = npad / NB;
  // the trailing tiles' write-through stores address a 128-row tile through a buffer descriptor (32-bit byte offsets)
  if (lda > (int64_t(1) << 20)) return hipErrorInvalidValue;
  if (z_done) *z_done = false;
  PotrfFwd f;
  // the fold needs panels that apply exactly one pending column per launch (eager or lookahead schedules)
  // (lookahead launches always do; eager ones when they flush every launch: g = 1, or after a switch)
  const int fmode = potrf_mode(ctx, nblk, bt.count), fg = potrf_lazy(ctx, nblk, bt.count);
  if (fr && fr->Y && fr->buf && (fmode == 1 || fg == 1 || potrf_switch(ctx, nblk, bt.count, fmode, fg) > 0)) {
    const int64_t nr = rhs_row(fr->nrhs);
    f.Y = fr->Y;
    f.ldy = fr->ldy;
    f.sy = fr->sy;
    f.r = fr->buf;
    f.z = fr->buf + (int64_t)npad * nr;
    f.sb = 2 * (int64_t)npad * nr;
    f.nrhs = fr->nrhs;
    f.n = fr->n;
    f.mean = fr->mean;
    f.means = fr->means;
  }
  launch_steps(ctx, nblk, A, lda, Dinv, info, bt, 0, nblk, f);
  launch_dinv(ctx, nblk, A, lda, Dinv, info, bt, 0, nblk, W, ldw);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && z_done && f.r) *z_done = true;
  return e;
}

}  // namespace gpx
