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
//    step is published, and do the other U items while that F runs.  Every panel workgroup re-factors A_cc (no
//    extra latency, no extra launch); p = 0 stores L_cc in the scratch half of Dinv (A_cc must stay intact while
//    the other panel workgroups read it), p > 0 store L_ic.
//  * trailing workgroups apply the step-(c-1) update to every lower tile of columns >= c+1:
//    A_ij -= L_{i,c-1} L_{j,c-1}^T on 128x128 MfmaTiles (half the HBM/L2 traffic per flop of 64x64 tiles; the
//    update is traffic-bound at 64x64: 36 us for the 2016 tiles of step 0).
// Column c+1 is thus updated by step c-1 in launch c and by step c inside the panel workgroups of launch c+1, so
// the panel factorisation (the latency-bound serial chain) overlaps the trailing update of the previous step
// instead of following it.  For large n the trailing update is flushed lazily (every g block columns, K = 64 g:
// each C tile read and written once per g columns) and lookahead workgroups bring the next panel's column up to
// date in the launch before it (StepPlan below).  potrf_dinv finally copies every L_kk from the scratch into A and inverts it (Dinv, used
// by gpx_trtri_f64).
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_chol64.h"

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
// so nothing waits on a seed before the first MFMA needs it.  Wave W owns A_ic's block row W and the A_cc blocks
// W, W+4, W+8 of the row-major lower list, each a K = 64 chain of 16 MFMAs in MfmaTile's k order (C - ab rounds as
// -(-C + ab): same results).  sA / sP double as the staging: the products are held in registers across a barrier.
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

// SPLIT (p > 0 only; 1, 2 or 4): the workgroup owns 64 / SPLIT rows of A_ic (its row blocks RB = 0 .. 4 / SPLIT - 1);
// SPLIT waves share a row block, wave W updating A_ic blocks (W / SPLIT, (W % SPLIT) NIC + jj), jj < NIC = 4 / SPLIT,
// beside its A_cc blocks: at most 7 / 5 / 4 blocks per wave for SPLIT = 1 / 2 / 4.
template <int W, bool PANEL, int NR, int SPLIT>
__device__ __forceinline__ void update_eager_wave(const double* __restrict__ Acc, const double* __restrict__ Aic,
                                                  const double* __restrict__ Lc, const double* __restrict__ Li,
                                                  int64_t lda, double* sA, double* sP, int c, int rowblk0,
                                                  const PotrfFwd& f, double* sZ, double* sR) {
  constexpr int NCC = W < 2 ? 3 : 2;
  constexpr int NIC = 4 / SPLIT;                 // A_ic blocks of this wave
  constexpr int RB = W / SPLIT;                  // its A_ic row block (within the workgroup's rows)
  constexpr int JB0 = (W % SPLIT) * NIC;         // its first A_ic column block
  constexpr int NRI = 8 / SPLIT;                 // double2 loads of L_i per thread (64 / SPLIT rows)
  constexpr bool FOLD_ROWS = !PANEL || (W % SPLIT) == 0;  // waves that fold their row block's right-hand side
  const int t = threadIdx.x, lane = t & 63;
  const int g = lane >> 4, cl = lane & 15;
  double2 rl[8], ri[NRI];
  d4 acc_cc[NCC], acc_ic[NIC];
  // forward fold: z_{c-1} (-> LDS sZ) and this lane's old right-hand sides (row 16 RB + cl of the workgroup's rows,
  // which start at global row rowblk0)
  double2 zv = make_double2(0.0, 0.0);
  double rold[NR > 0 ? NR : 1];
  const int frow = rowblk0 + 16 * RB + cl;
  if constexpr (NR > 0) {
    if (t < 32 * NR) zv = *reinterpret_cast<const double2*>(f.z + (int64_t)(c - 1) * NB * NR + 2 * t);
#pragma unroll
    for (int rr = 0; rr < NR; ++rr)
      rold[rr] = (g != 0 || !FOLD_ROWS) ? 0.0 : (c == 1 ? fwd_y(f, frow, rr) : f.r[(int64_t)frow * NR + rr]);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, r = e >> 6, cc = e & 63;
    rl[q] = *reinterpret_cast<const double2*>(Lc + (int64_t)r * lda + cc);
    if (PANEL && q < NRI) ri[q] = *reinterpret_cast<const double2*>(Li + (int64_t)r * lda + cc);
  }
#pragma unroll
  for (int b = 0; b < NCC; ++b) {
    const int bi = kLowerBlk[W + 4 * b][0], bj = kLowerBlk[W + 4 * b][1];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc_cc[b][q] = Acc[(int64_t)(16 * bi + g + 4 * q) * lda + 16 * bj + cl];
  }
  if (PANEL) {
#pragma unroll
    for (int j = 0; j < NIC; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc_ic[j][q] = Aic[(int64_t)(16 * RB + g + 4 * q) * lda + 16 * (JB0 + j) + cl];
  }
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
  // the A operand of the A_cc blocks; L_i's row block W is A_ic's A operand), then the chunk's MFMAs, independent
  // across blocks
  const int m = lane & 15, kq = lane >> 4;
  // forward fold: r_i -= L_{i,c-1} z_{c-1} on the wave's 16 rows, from the L fragments the MFMAs read anyway (row block
  // W of L_i, or of L_c for p = 0): lane (m, kq) sums k = kq mod 4, its FMAs issue between the chunk's MFMAs
  double part[NR > 0 ? NR : 1];
#pragma unroll
  for (int rr = 0; rr < (NR > 0 ? NR : 1); ++rr) part[rr] = 0.0;
#pragma unroll
  for (int kc = 0; kc < NB; kc += 16) {
    double fc[4][4], fi[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) fc[jb][s] = sA[(16 * jb + m) * LD64 + kc + 4 * s + kq];
      if (PANEL) fi[s] = sP[(16 * RB + m) * LD64 + kc + 4 * s + kq];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (PANEL) {
#pragma unroll
        for (int j = 0; j < NIC; ++j) acc_ic[j] = mfma_sub(fi[s], fc[JB0 + j][s], acc_ic[j]);
      }
#pragma unroll
      for (int b = 0; b < NCC; ++b)
        acc_cc[b] = mfma_sub(fc[kLowerBlk[W + 4 * b][0]][s], fc[kLowerBlk[W + 4 * b][1]][s], acc_cc[b]);
      if constexpr (NR > 0 && FOLD_ROWS) {
        const double lv = PANEL ? fi[s] : fc[W][s];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) part[rr] = fma(lv, sZ[(kc + 4 * s + kq) * NR + rr], part[rr]);
      }
    }
  }
  if constexpr (NR > 0 && FOLD_ROWS) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) part[rr] = rowsum4(part[rr]);
    if (g == 0) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) {
        sR[(16 * RB + cl) * NR + rr] = rold[rr] - part[rr];  // stored to global memory at the workgroup's end
      }
    }
  }
  __syncthreads();  // every wave's operand reads done: sA / sP take the results
  GPX_EAGER_STAMP(c, rowblk0, 1);
#pragma unroll
  for (int b = 0; b < NCC; ++b) store_block16(sA, 16 * kLowerBlk[W + 4 * b][0], 16 * kLowerBlk[W + 4 * b][1], acc_cc[b]);
  if (PANEL) {
#pragma unroll
    for (int j = 0; j < NIC; ++j) store_block16(sP, 16 * RB, 16 * (JB0 + j), acc_ic[j]);
  }
}

template <bool PANEL, int NR, int SPLIT>
__device__ __forceinline__ void update_eager(const double* __restrict__ Acc, const double* __restrict__ Aic,
                                             const double* __restrict__ Lc, const double* __restrict__ Li, int64_t lda,
                                             double* sA, double* sP, int c, int rowblk0, const PotrfFwd& f, double* sZ,
                                             double* sR) {
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {  // wave-uniform: compile-time block lists per wave
    case 0: update_eager_wave<0, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, c, rowblk0, f, sZ, sR); break;
    case 1: update_eager_wave<1, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, c, rowblk0, f, sZ, sR); break;
    case 2: update_eager_wave<2, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, c, rowblk0, f, sZ, sR); break;
    default: update_eager_wave<3, PANEL, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, c, rowblk0, f, sZ, sR); break;
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
                                           const PotrfFwd& f, int32_t* __restrict__ done = nullptr) {
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
  if (c > 0) {
    // the updates of block columns c0 .. c-1 not yet applied to this column, on the two tiles this workgroup
    // factors (K = 64 (c - c0))
    const int kk = (c - c0) * NB;
    const double* Lc = A + (int64_t)c * NB * lda + (int64_t)c0 * NB;
    const double* Li = A + (int64_t)row0 * lda + (int64_t)c0 * NB;
    if (kk == NB) {
      if (panel)
        update_eager<true, NR, SPLIT>(Acc, Aic, Lc, Li, lda, sA, sP, c, row0, f, sZ, sR);
      else
        update_eager<false, NR, 1>(Acc, Aic, Lc, Li, lda, sA, sP, c, c * NB, f, sZ, sR);
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
  int fail = -1;
  for (int s = 0; s < 4; ++s) {
    const int o = 16 * s;
    double* D = sDb + (s & 1) * 16 * LDD;
    if (w == 0) {
      // (4-pivot blocks on v_mfma_f64_16x16x4, tools/chol16_probe.hip: correct, but measured slower inside the panel,
      // potrf 1.89 vs 1.76 ms at n = 4096: ~75 instructions per pivot and MFMA / ds_bpermute latency on the chain)
      const int f = chol16<LDD>(sA, D, o);
      if (f >= 0 && fail < 0) fail = o + f;
    }
    GPX_PANEL_STAMP(1 + 3 * s);
    __syncthreads();  // publishes L_ss and D_ss
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
    for (int e = t; e < NB * NB; e += WG) {
      const int r = e >> 6, cc = e & 63;
      Lcc[e] = (cc <= r) ? sA[r * LD64 + cc] : 0.0;
    }
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
  if (done) {  // decoupled trailing update: publish "PROWS more rows of column c" (write-through stores, drained)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) __hip_atomic_fetch_add(done + c, PROWS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// The 128x128 tile with origin at 64-block (r0, q0): A -= sum_{k = k0}^{c-1} L_{r0..,k} L_{q0..,k}^T.
__device__ __forceinline__ void trailing_tile_at(double* __restrict__ A, int64_t lda, int c, int k0, int cfirst, int r0,
                                                 int q0, double* lds) {
  const double* Li = A + (int64_t)r0 * NB * lda + (int64_t)k0 * NB;
  const double* Lj = A + (int64_t)q0 * NB * lda + (int64_t)k0 * NB;
  double* C = A + (int64_t)r0 * NB * lda + (int64_t)q0 * NB;
  Tile128 tl;
  // C - acc, stored for the 64-blocks (rb, cb) with cb >= c+1 and rb >= cb, one row group i at a time: row group 0's C
  // loads are issued before the last k-tile's MFMAs and group i+1's before group i's stores, so one load round trip is
  // exposed instead of one per group (seeding acc with -C before the product, as the 64x64 panel updates do, pushes this
  // 128x128 tile into 30 VGPR spills)
  double cv[Tile128::WN][4];
  auto load_group = [&](int i) {
#pragma unroll
    for (int j = 0; j < Tile128::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[j][r] = C[(int64_t)Tile128::row_of(i, r) * lda + Tile128::col_of(j)];
  };
  tl.zero();
  tl.run_acc_peeled(Li, lda, Lj, lda, 0, (c - k0) * NB, lds, [&] { load_group(0); });
  const rsrc_t rc = buf_rsrc(C);
#pragma unroll
  for (int i = 0; i < Tile128::WM; ++i) {
#pragma unroll
    for (int j = 0; j < Tile128::WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) tl.acc[i][j][r] = cv[j][r] - tl.acc[i][j][r];
    if (i + 1 < Tile128::WM) load_group(i + 1);
    // write-through 16-byte pairs; a 16-column pair never straddles a 64-block, and rows r = 0, 1 (even lanes) or 2, 3
    // (odd lanes) of one lane lie in one 64-row block
#pragma unroll
    for (int j = 0; j < Tile128::WN; ++j) {
      const int cb = q0 + (Tile128::col_of(j) >> 6);
      const bool colok = cb >= cfirst;
      const bool k01 = colok && r0 + (Tile128::row_of(i, 0) >> 6) >= cb;
      const bool k23 = colok && r0 + (Tile128::row_of(i, 2) >> 6) >= cb;
      store_block_pairs_sc1<Tile128>(rc, lda, i, j, tl.acc[i][j], k01, k23);
    }
  }
}

__device__ __forceinline__ void trailing_role(double* __restrict__ A, int64_t lda, int c, int nblk, int k0, int cfirst,
                                              int tile, int ntile, int xmap, double* lds) {
  const int M = (nblk - cfirst + 1) / 2, c0 = nblk - 2 * M;
  int I, J;
  trail_tile(tile, ntile, M, xmap, I, J);
  trailing_tile_at(A, lda, c, k0, cfirst, c0 + 2 * I, c0 + 2 * J, lds);
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
  tl.run_acc(Li, lda, Lj, lda, 0, (c - a) * NB, lds);
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
  int near;         // > 0: decoupled trailing update, only tile columns closer than `near` block columns (ntrail of them)
  int32_t* sync;    // decoupled trailing update: the sync words (potrf_side_kernel), else nullptr
  unsigned limit;   // their bounded polls (Context::spin_limit)
};

// slots > 0: the co-resident workgroup slots a problem may fill (two per CU, shared by a batch); the panel row blocks are
// split in 2 (StepPlan::split) when the panels apply exactly one column and the split launch still fits the slots.
inline StepPlan step_plan(int c, int nblk, int mode, int last_flush, bool flush, int xmap = 0, int slots = 0,
                          int near = 0) {
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
  s.near = 0;
  s.sync = nullptr;
  s.limit = 0;
  if (near > 0 && mode == 0 && flush && c - last_flush == 1) {
    s.near = near;
    s.ntrail = 0;
    for (int J = 0; J < M && nblk - 2 * M + 2 * J - c < near; ++J) s.ntrail += M - J;
  }
  const bool eager = mode == 1 || c == 0 || c - last_flush == 1;
  if (slots > 0 && eager && s.npanel > 1) {
    for (int sp = 2; sp >= 2; sp >>= 1) {  // split 4 measured slower at n = 4096 (potrf 1.48 vs 1.46 ms), equal below
      const int np = 1 + sp * (s.npanel - 1);
      const int tb = xmap ? (np + s.nlook + 7) & ~7 : np + s.nlook;
      if (tb + s.ntrail <= slots) {
        s.split = sp;
        s.npanel = np;
        break;
      }
    }
  }
  s.tbase = xmap ? (s.npanel + s.nlook + 7) & ~7 : s.npanel + s.nlook;  // padding workgroups exit at once
  return s;
}

// ---- decoupled trailing update (GPX_OPT_POTRF_DECOUPLE, eager schedule only) -------------------------------------
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
__device__ __forceinline__ void near_role(double* __restrict__ A, int64_t lda, int c, int nblk, const StepPlan& s, int p,
                                          int32_t* __restrict__ info, double* lds) {
  __shared__ int s_ok;
  const int M = (nblk - s.cfirst + 1) / 2, c0 = nblk - 2 * M;
  int J = 0;
  while (p >= M - J) {
    p -= M - J;
    ++J;
  }
  const int r0 = c0 + 2 * (J + p), q0 = c0 + 2 * J, cn = q0 - s.near + 1;
  if (c == cn && cn >= 2) {
    if (threadIdx.x == 0) {
      s_ok = poll_at_least(s.sync + nblk + (r0 >> 1) * (nblk >> 1) + (q0 >> 1), cn - 1, info, s.limit);
      if (!s_ok) atomicCAS(info, 0, (int32_t)GPX_INFO_TIMEOUT);
    }
    __syncthreads();
    if (!s_ok) return;
  }
  trailing_tile_at(A, lda, c, s.k0, s.cfirst, r0, q0, lds);
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
      trailing_tile_at(At, ldt, ke, kb, 0, r0, q0, lds);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_store(sync + nblk + (r0 >> 1) * (nblk >> 1) + (q0 >> 1), ke, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!any) return;
  }
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
      f.r += blockIdx.y * f.sb;
      f.z += blockIdx.y * f.sb;
    }
    if (s.split == 2 && b > 0)
      panel_role<NR, 2>(A, lda, c, 1 + ((b - 1) >> 1), (b - 1) & 1, nblk, s.c0, Dinv, info, lds, f, s.sync);
    else
      panel_role<NR, 1>(A, lda, c, b, 0, nblk, s.c0, Dinv, info, lds, f, s.sync);
  } else if (role == 1)
    lookahead_role(A, lda, c, s.look_a, b - s.npanel, lds);
  else if (s.near > 0)
    near_role(A, lda, c, nblk, s, b - s.tbase, info, lds);
  else
    trailing_role(A, lda, c, nblk, s.k0, s.cfirst, b - s.tbase, s.ntrail, s.xmap, lds);
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
//   n = 8192:  mode 1, g = 4 -> 6.34 ms (mode 0 g = 2: 6.69);
//   n = 16384: mode 1, g = 8 -> 31.4 ms (mode 0 g = 4: 34.4, g = 1: 46.3).
// The handle options GPX_OPT_POTRF_LAZY / GPX_OPT_POTRF_MODE override.  Flushing every second launch only in the early,
// trailing-bound launches and panel-wave priority were measured neutral (DESIGN.md §5, items 14 and the prio knob)
// and are not offered.  Trailing tiles are dealt to the XCDs in 8 x 8 super-block chunks (trail_tile xmap = 1).
static int potrf_lazy(const Context* ctx, int nblk) {
  if (ctx->potrf_lazy > 0) return ctx->potrf_lazy;
  return nblk > 128 ? 8 : (nblk > 64 ? 4 : 1);
}

static int potrf_mode(const Context* ctx, int nblk) {
  if (ctx->potrf_mode == 0 || ctx->potrf_mode == 1) return ctx->potrf_mode;
  return nblk > 64 ? 1 : 0;
}

// Near distance D of the decoupled trailing update (0 = off): eager schedule (mode 0, g = 1), one problem.  Off by
// size until measured faster (GPX_OPT_POTRF_DECOUPLE turns it on).
static int potrf_decouple(const Context* ctx, int nblk, int mode, int batch) {
  if (batch != 1 || mode != 0 || potrf_lazy(ctx, nblk) != 1 || ctx->potrf_decouple <= 0) return 0;
  return ctx->potrf_decouple < nblk ? ctx->potrf_decouple : 0;  // D >= nblk: every tile is near
}

// The plan of every launch c < cend (flush launches: c >= 1 and at least one interval after the previous flush).
template <typename F>
static void for_each_step(const Context* ctx, int nblk, int mode, int cend, int slots, F&& f, int near = 0) {
  const int g = potrf_lazy(ctx, nblk);
  int last = 0;
  for (int c = 0; c < cend; ++c) {
    const bool flush = c >= 1 && c - last >= g;
    f(c, step_plan(c, nblk, mode, last, flush, 1, slots, near));
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

// The decoupled update's side stream, events and sync words (created on first use, kept by the handle).
static hipError_t side_resources(Context* ctx, size_t bytes) {
  hipError_t e = hipSuccess;
  if (!ctx->side_stream) e = hipStreamCreateWithFlags(&ctx->side_stream, hipStreamNonBlocking);
  if (e == hipSuccess && !ctx->ev_fork) e = hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming);
  if (e == hipSuccess && !ctx->ev_join) e = hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming);
  if (e == hipSuccess && ctx->sync_bytes < bytes) {
    if (ctx->sync_buf) {
      e = hipStreamSynchronize(ctx->stream);  // an earlier factorisation may still use the old words
      if (e == hipSuccess) e = hipFree(ctx->sync_buf);
      ctx->sync_buf = nullptr;
      ctx->sync_bytes = 0;
    }
    if (e == hipSuccess) e = hipMalloc(&ctx->sync_buf, bytes);
    if (e == hipSuccess) ctx->sync_bytes = bytes;
  }
  return e;
}

static hipError_t launch_steps(Context* ctx, int nblk, double* A, int64_t lda, double* Dinv, int32_t* info,
                               const Batch& bt, int cbeg, int cend, const PotrfFwd& f = PotrfFwd()) {
  const int mode = potrf_mode(ctx, nblk);
  int slots = potrf_slots(ctx, bt.count);
  const int D = slots > 0 && cbeg == 0 && cend == nblk ? potrf_decouple(ctx, nblk, mode, bt.count) : 0;
  int32_t* sync = nullptr;
  if (D > 0) {
    const size_t bytes = (size_t)(nblk + (nblk / 2) * (nblk / 2)) * sizeof(int32_t);
    hipError_t e = side_resources(ctx, bytes);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->sync_buf, 0, bytes, ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev_fork, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->side_stream, ctx->ev_fork, 0);
    if (e != hipSuccess) return e;
    sync = ctx->sync_buf;
    int ntile = 0;
    for (int q0 = (D + 2) & ~1; q0 < nblk; q0 += 2) ntile += (nblk - q0) / 2;
    const int grid = ntile < slots / 2 ? ntile : slots / 2;  // one workgroup per CU
    if (grid > 0)
      potrf_side_kernel<<<grid, WG, 0, ctx->side_stream>>>(A, lda, nblk, D, sync, info, ctx->spin_limit);
    e = hipEventRecord(ctx->ev_join, ctx->side_stream);
    if (e != hipSuccess) return e;
    slots /= 2;  // the other slot of every CU is the step launches'
  }
  for_each_step(ctx, nblk, mode, cend, slots, [&](int c, StepPlan s) {
    if (c < cbeg) return;
    s.sync = sync;
    s.limit = ctx->spin_limit;
    const dim3 grid(s.tbase + s.ntrail, bt.count);
    if (!f.r)
      potrf_step_kernel<0><<<grid, WG, 0, ctx->stream>>>(A, lda, c, nblk, s, Dinv, info, 0, bt.k, bt.dinv, f);
    else if (f.nrhs == 1)
      potrf_step_kernel<1><<<grid, WG, 0, ctx->stream>>>(A, lda, c, nblk, s, Dinv, info, 0, bt.k, bt.dinv, f);
    else
      potrf_step_kernel<GPX_MAX_RHS><<<grid, WG, 0, ctx->stream>>>(A, lda, c, nblk, s, Dinv, info, 0, bt.k, bt.dinv, f);
  }, D);
  return D > 0 ? hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0) : hipSuccess;
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
  if (fr && fr->Y && fr->buf && (potrf_mode(ctx, nblk) == 1 || potrf_lazy(ctx, nblk) == 1)) {
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
  }
  const hipError_t es = launch_steps(ctx, nblk, A, lda, Dinv, info, bt, 0, nblk, f);
  if (es != hipSuccess) return es;
  launch_dinv(ctx, nblk, A, lda, Dinv, info, bt, 0, nblk, W, ldw);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && z_done && f.r) *z_done = true;
  return e;
}

}  // namespace gpx
