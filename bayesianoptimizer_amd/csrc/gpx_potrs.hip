// alpha = K^{-1} (Y - m) from the Cholesky factor alone (LAPACK potrs): forward L z = b, then backward L^T alpha = z,
// in ONE persistent launch whose workgroups hand 128-row blocks of z / alpha to each other.
// SURVEY §8a row a5 (GPyTorch's mean_cache [upstream], reached from optimization/Bayesian.py:89-94): the posterior
// update of SURVEY §8d (Gram + Cholesky + alpha) no longer forms W = L^{-T} (n^3/3 more flops, 0.61 ms at n = 4096);
// W is built by gpx_trtri_f64 only when a sweep, a posterior or a gradient needs it.
//
// Work items: forward block K = 0 .. nb-1, then backward block K = nb-1 .. 0 (nb = npad / 128).  Workgroup g of a
// problem (G <= nb workgroups, the grid sized to be co-resident) owns blocks g, g + G, ... in BOTH directions and runs
// its forward items in ascending block order, then its backward items in descending order.  A forward item waits only
// on forward items of smaller blocks and a backward item only on backward items of larger blocks (and its own forward
// result), so the smallest pending forward item and, once every forward item is done, the largest pending backward
// item can always proceed: no deadlock.  Every workgroup streams nb - 1 tiles in all (block K: K tiles forward,
// nb - 1 - K backward); the former item-index order (item i on workgroup i mod G) gave workgroup nb-1 both 31-tile items
// at n = 4096 and made the backward solve wait on its tile stream (`profiles/r02_potrs_timeline.log`: 130 us backward
// against 90 us forward).
//   forward K:  v = b_K - sum_{J<K} L_KJ z_J, each 128x128 tile L_KJ loaded into registers BEFORE its z_J is waited
//               for; then z_K = L_KK^{-1} v with potrf's 64-block inverses: z_a = D_a v_a, v_b -= L_ba z_a,
//               z_b = D_b v_b.
//   backward K: v = z_K - sum_{J>K} L_JK^T alpha_J; alpha_b = D_b^T v_b, v_a -= L_ba^T alpha_b, alpha_a = D_a^T v_a.
// Every accumulation runs in a fixed order (J ascending forward, descending backward; fixed lane reductions), so the
// result does not depend on timing or placement, and a batched solve equals single solves bit for bit.
//
// Hand-off (cdna_hip_programming.md §6 Guideline 16, form R2 — the data is the flag): every double of a published
// block travels as two naturally aligned 8-byte {tag, 32-bit half} granules, each written by ONE agent-scope atomic
// (sc1) store; one consumer wave re-reads the block's granules with agent-scope atomic loads until every tag equals
// the phase's epoch (1 = z, 2 = alpha).  The granule buffer is zeroed by a memset before the launch.  Spins are
// bounded: a solve that stops making progress sets the timeout word, every waiter then gives up and the items it
// owned write NaN into alpha.
#include "gpx_internal.h"
#include "gpx_device.h"

// Optional timestamp hook for tools/potrs_probe.hip (compiled out in the library).
#ifndef GPX_POTRS_STAMP
#define GPX_POTRS_STAMP(i)
#endif
#ifndef GPX_POTRS_FIT_STAMP
#define GPX_POTRS_FIT_STAMP(i)
#endif

namespace gpx {

namespace {

constexpr int SB = 128;       // rows per hand-off block
constexpr int LDT = NB + 1;   // LDS row length of the 64x64 diagonal tiles

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// One wave: wait until all 256*NR granules of a block carry `epoch`, then write their 32-bit halves into dst
// (SB x NR doubles, row-major; wave-private, so no workgroup barrier is needed before the wave reads it back).
// Every wave of a consumer sweeps for itself.  The abort word is read only every 64th failed pass (its sc1 load would
// otherwise double each poll's round trip).  Returns false on timeout / abort.
template <int NR>
__device__ __forceinline__ bool sweep_block(gu64* g, unsigned epoch, double* dst, gu32* abort_word, unsigned limit) {
  constexpr int PER = 4 * NR;  // granules per lane: SB * NR * 2 / 64
  const int lane = threadIdx.x & 63;
  unsigned long long x[PER];
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      x[k] = __hip_atomic_load(g + lane + 64 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok &= (unsigned)(x[k] >> 32) == epoch;
    }
    if (__all(ok)) break;
    if (spins >= limit ||
        ((spins & 63) == 63 && __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
      if (lane == 0) __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  unsigned* d32 = reinterpret_cast<unsigned*>(dst);
#pragma unroll
  for (int k = 0; k < PER; ++k) d32[lane + 64 * k] = (unsigned)x[k];  // granule gi = element gi/2, half gi%2
  return true;
}

template <int NR>
__device__ __forceinline__ void publish_block(gu64* g, unsigned epoch, const double* src) {
  const unsigned* s32 = reinterpret_cast<const unsigned*>(src);
  for (int gi = threadIdx.x; gi < SB * NR * 2; gi += WG)
    __hip_atomic_store(g + gi, ((unsigned long long)epoch << 32) | s32[gi], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Lane exchanges inside groups of 8 lanes by DPP (VALU, no LDS round trip like __shfl_xor's ds_bpermute):
// xor 1 / xor 2 by quad_perm, xor 4 by row_shl:4 into banks 0/2 and row_shr:4 into banks 1/3.
template <int CTRL, int BANKS>
__device__ __forceinline__ unsigned dpp_u32(unsigned old, unsigned x) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, 0xf, BANKS, false);
}
template <int X>
__device__ __forceinline__ double xor_lane(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  unsigned rlo, rhi;
  if constexpr (X == 1) {
    rlo = dpp_u32<0xB1, 0xf>(0u, lo);
    rhi = dpp_u32<0xB1, 0xf>(0u, hi);
  } else if constexpr (X == 2) {
    rlo = dpp_u32<0x4E, 0xf>(0u, lo);
    rhi = dpp_u32<0x4E, 0xf>(0u, hi);
  } else {
    static_assert(X == 4, "xor 1, 2 or 4");
    rlo = dpp_u32<0x114, 0xA>(dpp_u32<0x104, 0x5>(0u, lo), lo);
    rhi = dpp_u32<0x114, 0xA>(dpp_u32<0x104, 0x5>(0u, hi), hi);
  }
  return __longlong_as_double(((unsigned long long)rhi << 32) | rlo);
}

// 64x64 tile of a row-major global matrix into LDS (row length LDT)
__device__ __forceinline__ void tile_to_lds(const double* __restrict__ G, int64_t ld, double* S) {
  for (int e = threadIdx.x; e < NB * NB / 2; e += WG) {
    const int r = (2 * e) >> 6, c = (2 * e) & 63;
    const double2 v = *reinterpret_cast<const double2*>(G + (int64_t)r * ld + c);
    S[r * LDT + c] = v.x;
    S[r * LDT + c + 1] = v.y;
  }
}

// out (64 x NR) = M x (TRANS: M^T x), or out -= ... (SUB); M in LDS (row length LDT), x / out in LDS (row-major,
// NR per row).  Thread (i = t/4, q = t%4) sums j in [16q, 16q+16), the four partials are combined by lane shuffles.
template <int NR, bool TRANS, bool SUB>
__device__ __forceinline__ void gemv64(double* out, const double* M, const double* x) {
  const int t = threadIdx.x, i = t >> 2, q = t & 3;
  double p[NR];
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) p[rr] = 0.0;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) {
    const int j = 16 * q + jj;
    const double m = TRANS ? M[j * LDT + i] : M[i * LDT + j];
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) p[rr] = fma(m, x[j * NR + rr], p[rr]);
  }
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) {
    p[rr] += __shfl_xor(p[rr], 1);
    p[rr] += __shfl_xor(p[rr], 2);
  }
  if (q == 0) {
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) out[i * NR + rr] = SUB ? out[i * NR + rr] - p[rr] : p[rr];
  }
}

// NR = 8: the diagonal block is solved in three 64-steps (D_a, L_ba, D_b from LDS).
template <int NR>
struct SolveLds {
  double Da[NB * LDT], Db[NB * LDT], Lba[NB * LDT];
  double zw[WG / 64][SB * NR];  // wave-private copy of the block being consumed
  double vs[SB * NR];           // right-hand side / working vector
  double os[SB * NR];           // the block being produced
};

// NR = 1: the whole 128x128 inverse D_KK = L_KK^{-1} = [D_a 0; -D_b L_ba D_a  D_b] is formed at the start of the item
// (before anything is waited for), so the step on the chain is ONE matrix-vector product.
constexpr int LDK = SB + 4;  // LDS row length of D_KK
struct SolveLds1 {
  double Dk[SB * LDK];
  double zw[WG / 64][SB];  // wave-private copy of the block being consumed
  double vs[SB];
};

// C(64x64) = sign * A(64x64) B(64x64), operands in LDS (row lengths LDA / LDB), fp64 MFMA 16x16x4: wave w computes the
// 32x32 quadrant (w/2, w%2).  A lower triangular (A_LOW) / B lower triangular (B_LOW) bound the k range per block.
// Result in registers: acc[i][j][r] = C(32 (w/2) + 16 i + lane/16 + 4 r, 32 (w%2) + 16 j + lane%16).
template <int LDA, int LDB, bool A_LOW, bool B_LOW>
__device__ __forceinline__ void mfma64_lds(d4 (&acc)[2][2], const double* A, const double* B, double sign) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = 32 * (w >> 1), n0 = 32 * (w & 1);
  const int l16 = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
      // k range with a non-zero product: B lower -> k >= first column of the block; A lower -> k <= last row
      const int kb = B_LOW ? n0 + 16 * j : 0;
      const int ke = A_LOW ? m0 + 16 * i + 16 : NB;
      for (int k = kb; k < ke; k += 4) {
        const double a = sign * A[(m0 + 16 * i + l16) * LDA + k + kk];
        const double b = B[(k + kk) * LDB + n0 + 16 * j + l16];
        acc[i][j] = mfma16x16x4(a, b, acc[i][j]);
      }
    }
}

template <int LDC>
__device__ __forceinline__ void store_quadrants(double* C, const d4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = 32 * (w >> 1), n0 = 32 * (w & 1);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(m0 + 16 * i + (lane >> 4) + 4 * r) * LDC + n0 + 16 * j + (lane & 15)] = acc[i][j][r];
}

// D_KK of chain block K into s.Dk: D_a, D_b and L_ba staged in its blocks, T = L_ba D_a parked in the (zero) upper
// block, then the lower-left block = -D_b T.
__device__ __forceinline__ void form_block_inverse(SolveLds1& s, const double* __restrict__ Dinv,
                                                   const double* __restrict__ L, int64_t ldl, int K) {
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)K * SB;
  const double* Da = Dinv + (int64_t)(2 * K) * NB * NB;
  const double* Db = Dinv + (int64_t)(2 * K + 1) * NB * NB;
  const double* Lba = L + (r0 + NB) * ldl + r0;
  for (int e = t; e < NB * NB / 2; e += WG) {
    const int r = (2 * e) >> 6, c = (2 * e) & 63;
    const double2 a = *reinterpret_cast<const double2*>(Da + r * NB + c);
    const double2 b = *reinterpret_cast<const double2*>(Db + r * NB + c);
    const double2 l = *reinterpret_cast<const double2*>(Lba + (int64_t)r * ldl + c);
    s.Dk[r * LDK + c] = a.x;
    s.Dk[r * LDK + c + 1] = a.y;
    s.Dk[(NB + r) * LDK + NB + c] = b.x;
    s.Dk[(NB + r) * LDK + NB + c + 1] = b.y;
    s.Dk[r * LDK + NB + c] = l.x;  // L_ba parked in the upper-right block
    s.Dk[r * LDK + NB + c + 1] = l.y;
  }
  __syncthreads();
  d4 acc[2][2];
  mfma64_lds<LDK, LDK, false, true>(acc, s.Dk + NB, s.Dk, 1.0);  // T = L_ba D_a (D_a lower)
  __syncthreads();
  store_quadrants<LDK>(s.Dk + NB, acc);
  __syncthreads();
  mfma64_lds<LDK, LDK, true, false>(acc, s.Dk + NB * LDK + NB, s.Dk + NB, -1.0);  // -D_b T (D_b lower)
  __syncthreads();
  store_quadrants<LDK>(s.Dk + NB * LDK, acc);
  for (int e = t; e < NB * NB; e += WG) s.Dk[(e >> 6) * LDK + NB + (e & 63)] = 0.0;
  __syncthreads();
}

// Off-diagonal tile of one consumed block, 64 doubles per thread.
//  forward  (tile L_KJ, rows of block K x columns of block J): thread t owns rows rq + 32k (rq = t/8, k < 4) and the
//           column pairs 16 c2 + 2 g (g = t%8, c2 < 8): a load instruction reads 8 x 16 B = one whole 128-B line per row;
//  backward (tile L_JK, rows of block J x columns of block K): thread t owns column t/2 of block K and rows
//           64 (t%2) .. +63 of block J (two 256-B runs per instruction).
struct TileRegs {
  double2 v[32];
};

__device__ __forceinline__ void load_tile_fwd(TileRegs& R, const double* __restrict__ L, int64_t ldl, int64_t r0,
                                              int64_t c0) {
  const int t = threadIdx.x, g = t & 7, rq = t >> 3;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c2 = 0; c2 < 8; ++c2)
      R.v[8 * k + c2] = *reinterpret_cast<const double2*>(L + (r0 + rq + 32 * k) * ldl + c0 + 16 * c2 + 2 * g);
}

__device__ __forceinline__ void load_tile_bwd(TileRegs& R, const double* __restrict__ L, int64_t ldl, int64_t r0,
                                              int64_t c0) {
  const int t = threadIdx.x, c = t >> 1, h = t & 1;
  const double* src = L + (r0 + NB * h) * ldl + c0 + c;
#pragma unroll
  for (int i = 0; i < 32; ++i) R.v[i] = make_double2(src[(int64_t)(2 * i) * ldl], src[(int64_t)(2 * i + 1) * ldl]);
}

template <int NR>
__device__ __forceinline__ void fma_fwd(double (&acc)[4][NR], const TileRegs& R, const double* z) {
  const int g = threadIdx.x & 7;
  if constexpr (NR == 1) {
    // the thread's 16 z entries as 8 16-byte LDS reads issued back to back, then the FMAs
    double2 zz[8];
#pragma unroll
    for (int c2 = 0; c2 < 8; ++c2) zz[c2] = *reinterpret_cast<const double2*>(z + 16 * c2 + 2 * g);
#pragma unroll
    for (int c2 = 0; c2 < 8; ++c2)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc[k][0] = fma(R.v[8 * k + c2].y, zz[c2].y, fma(R.v[8 * k + c2].x, zz[c2].x, acc[k][0]));
    return;
  }
#pragma unroll
  for (int c2 = 0; c2 < 8; ++c2) {
    const int c = 16 * c2 + 2 * g;
    double z0[NR], z1[NR];
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      z0[rr] = z[c * NR + rr];
      z1[rr] = z[(c + 1) * NR + rr];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int rr = 0; rr < NR; ++rr)
        acc[k][rr] = fma(R.v[8 * k + c2].y, z1[rr], fma(R.v[8 * k + c2].x, z0[rr], acc[k][rr]));
  }
}

template <int NR>
__device__ __forceinline__ void fma_bwd(double (&acc)[4][NR], const TileRegs& R, const double* a) {
  const int h = threadIdx.x & 1;
  if constexpr (NR == 1) {
    // the 64 alpha entries of this half as 16-byte LDS reads (same address across the lanes of a half: broadcast),
    // two independent accumulation chains
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int i0 = 0; i0 < 32; i0 += 8) {
      double2 aa[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) aa[i] = *reinterpret_cast<const double2*>(a + NB * h + 2 * (i0 + i));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s0 = fma(R.v[i0 + i].x, aa[i].x, s0);
        s1 = fma(R.v[i0 + i].y, aa[i].y, s1);
      }
    }
    acc[0][0] += s0 + s1;
    return;
  }
#pragma unroll
  for (int i = 0; i < 32; ++i)
#pragma unroll
    for (int rr = 0; rr < NR; ++rr)
      acc[0][rr] = fma(R.v[i].y, a[(NB * h + 2 * i + 1) * NR + rr], fma(R.v[i].x, a[(NB * h + 2 * i) * NR + rr],
                                                                          acc[0][rr]));
}

}  // namespace

// Single right-hand side, standalone solve (forward + backward): D_KK formed up front, one product on the chain, the
// block published from registers.  A fit's backward half is potrs_bwd_fit_1.
__device__ void potrs_items_1(int n, int npad, const double* __restrict__ L, int64_t ldl,
                              const double* __restrict__ Dinv, const double* __restrict__ Y, int64_t ldy,
                              double const_mean, double* __restrict__ alpha, gu64* gz, gu64* ga, gu32* abort_word,
                              unsigned limit, SolveLds1& s, int& s_abort) {
  const int t = threadIdx.x, w = t >> 6;
  const int nb = npad / SB;
  const int G = gridDim.x;
  // blocks g, g + G, ... of this workgroup: forward ascending, then backward descending (see the file comment)
  const int nown = (nb - (int)blockIdx.x + G - 1) / G;
  for (int step = 0; step < 2 * nown; ++step) {
    const bool fwd = step < nown;
    const int K = (int)blockIdx.x + (fwd ? step : 2 * nown - 1 - step) * G;
    const int64_t r0 = (int64_t)K * SB;
    const int jcount = fwd ? K : nb - 1 - K;
    GPX_POTRS_STAMP(0);
    auto jblk = [&](int jj) { return fwd ? jj : nb - 1 - jj; };
    TileRegs ta, tb;
    auto load_tile = [&](TileRegs& R, int jj) {
      if (fwd)
        load_tile_fwd(R, L, ldl, r0, (int64_t)jblk(jj) * SB);
      else
        load_tile_bwd(R, L, ldl, (int64_t)jblk(jj) * SB, r0);
    };
    if (jcount > 0) load_tile(ta, 0);  // in flight while D_KK is formed
    // the first backward item is the block of the last forward item: its D_KK is still in LDS
    if (fwd || step != nown) form_block_inverse(s, Dinv, L, ldl, K);
    if (fwd) {
      if (t < SB) s.vs[t] = (r0 + t < n) ? Y[(r0 + t) * ldy] - const_mean : 0.0;
    } else if (w == 0) {
      if (!sweep_block<1>(gz + r0 * 2, 1u, s.vs, abort_word, limit) && (t & 63) == 0) s_abort = 1;
    }
    double acc[4][1];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k][0] = 0.0;
    // every wave polls the block it needs into its own LDS copy (no workgroup barrier in the loop)
    double* zw = s.zw[w];
    auto consume = [&](const TileRegs& R, int jj) {
      if (!sweep_block<1>((fwd ? gz : ga) + (int64_t)jblk(jj) * SB * 2, fwd ? 1u : 2u, zw, abort_word, limit) &&
          (t & 63) == 0)
        s_abort = 1;
      GPX_POTRS_STAMP(1);
      if (fwd)
        fma_fwd<1>(acc, R, zw);
      else
        fma_bwd<1>(acc, R, zw);
    };
    // no workgroup barrier in this loop; the next tile is loaded while the current one's block is waited for
    for (int jj = 0; jj < jcount; jj += 2) {
      const bool two = jj + 1 < jcount;
      if (two) load_tile(tb, jj + 1);
      consume(ta, jj);
      if (!two) break;
      if (jj + 2 < jcount) load_tile(ta, jj + 2);
      consume(tb, jj + 1);
    }
    // v = b - sum (right-hand side in s.vs), one barrier, then z = D_KK v (forward) / alpha = D_KK^T v (backward)
    if (fwd) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[k][0] += xor_lane<1>(acc[k][0]);
        acc[k][0] += xor_lane<2>(acc[k][0]);
        acc[k][0] += xor_lane<4>(acc[k][0]);
      }
    } else {
      acc[0][0] += xor_lane<1>(acc[0][0]);
    }
    __syncthreads();  // s.vs (right-hand side) complete
    if (fwd) {
      if ((t & 7) == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) s.vs[(t >> 3) + 32 * k] -= acc[k][0];
      }
    } else if ((t & 1) == 0) {
      s.vs[t >> 1] -= acc[0][0];
    }
    __syncthreads();
    GPX_POTRS_STAMP(2);
    const bool aborted = s_abort != 0;  // uniform; sticky for the rest of the launch
    if (fwd) {
      const int g = t & 7, rq = t >> 3;
      // LDS reads batched ahead of the FMAs (8 x 16 B per row, the thread's 16 v entries once)
      double2 vv[8];
#pragma unroll
      for (int c2 = 0; c2 < 8; ++c2) vv[c2] = *reinterpret_cast<const double2*>(s.vs + 16 * c2 + 2 * g);
      double z[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        double2 d[8];
#pragma unroll
        for (int c2 = 0; c2 < 8; ++c2)
          d[c2] = *reinterpret_cast<const double2*>(s.Dk + (rq + 32 * k) * LDK + 16 * c2 + 2 * g);
        double z0 = 0.0, z1 = 0.0;
#pragma unroll
        for (int c2 = 0; c2 < 8; ++c2) {
          z0 = fma(d[c2].x, vv[c2].x, z0);
          z1 = fma(d[c2].y, vv[c2].y, z1);
        }
        z[k] = z0 + z1;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z[k] += xor_lane<1>(z[k]);
        z[k] += xor_lane<2>(z[k]);
        z[k] += xor_lane<4>(z[k]);
        if (aborted) z[k] = __builtin_nan("");
      }
      GPX_POTRS_STAMP(3);
      if (g < 2) {  // lanes 0 / 1 of a row publish its low / high half
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const unsigned long long u = __double_as_longlong(z[k]);
          __hip_atomic_store(gz + (r0 + rq + 32 * k) * 2 + g, (1ull << 32) | (g ? (u >> 32) : (u & 0xffffffffull)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else {
      const int c = t >> 1, h = t & 1;
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int i0 = 0; i0 < NB; i0 += 16) {
        double dd[16];
        double2 vv[8];
#pragma unroll
        for (int i = 0; i < 16; ++i) dd[i] = s.Dk[(NB * h + i0 + i) * LDK + c];
#pragma unroll
        for (int i = 0; i < 8; ++i) vv[i] = *reinterpret_cast<const double2*>(s.vs + NB * h + i0 + 2 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a0 = fma(dd[2 * i], vv[i].x, a0);
          a1 = fma(dd[2 * i + 1], vv[i].y, a1);
        }
      }
      double a = a0 + a1;
      a += xor_lane<1>(a);
      if (aborted) a = __builtin_nan("");
      GPX_POTRS_STAMP(3);
      const unsigned long long u = __double_as_longlong(a);
      __hip_atomic_store(ga + (r0 + c) * 2 + h, (2ull << 32) | (h ? (u >> 32) : (u & 0xffffffffull)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (h == 0) alpha[r0 + c] = (r0 + c < n || aborted) ? a : 0.0;
    }
    __syncthreads();  // LDS reuse by the next item
  }
}

// ---- the backward half of a fit (zin: z from the factorisation's folded forward substitution), one right-hand side --
// alpha_K = D_KK^T (z_K - sum_{J>K} L_JK^T alpha_J) for K = nb-1 .. 0, the chain running through alpha_{K+1}.  Every
// item starts at launch time (one item per workgroup up to n = 32768), so how it prepares depends on how soon the chain
// reaches it (d = nb - 1 - K hops after its start):
//   d < BWD_TRIPLE  no setup: D_a, D_b and L_ba staged in LDS, and after the last subtraction alpha_b = D_b^T v_b,
//                   v_a -= L_ba^T alpha_b, alpha_a = D_a^T v_a (three 64 x 64 products): the chain starts ~5 us after the
//                   launch instead of after the ~10 us of forming D_KK (tools/potrs_fit_probe.hip);
//   else            the 128 x 128 inverse D_KK formed at the start (form_block_inverse): one product after the last
//                   subtraction (potrs_items_1's backward item, with its two register tiles).
// Measured and not kept (profiles/r04_potrs_fit_timeline.log): precomputing P = L_{K+1,K} D_KK so that the step on the
// chain becomes alpha_K = u - P^T alpha_{K+1} (u = D_KK^T (z_K - sum_{J>K+1} ...)) - P costs ~30 us of setup, and u then
// depends on alpha_{K+2}, so two hops took ~9 us instead of ~6.
constexpr int BWD_TRIPLE = 3;

__device__ void potrs_bwd_fit_1(int n, int npad, const double* __restrict__ L, int64_t ldl,
                                const double* __restrict__ Dinv, double* __restrict__ alpha, gu64* ga,
                                gu32* abort_word, unsigned limit, SolveLds1& s, int& s_abort,
                                const double* __restrict__ zin) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int nb = npad / SB;
  const int G = gridDim.x;
  const int nown = (nb - (int)blockIdx.x + G - 1) / G;
  double* zw = s.zw[w];
  for (int step = 0; step < nown; ++step) {
    const int K = (int)blockIdx.x + (nown - 1 - step) * G;  // descending
    const int64_t r0 = (int64_t)K * SB;
    const int jcount = nb - 1 - K;
    const bool triple = nb - 1 - K < BWD_TRIPLE;
    GPX_POTRS_FIT_STAMP(0);
    TileRegs ta, tb;
    auto load_tile = [&](TileRegs& R, int jj) { load_tile_bwd(R, L, ldl, (int64_t)(nb - 1 - jj) * SB, r0); };
    if (jcount > 0) load_tile(ta, 0);  // in flight during the setup
    double* Da = s.Dk;  // triple: D_a, D_b, L_ba (row length LDT) and the produced block
    double* Db = Da + NB * LDT;
    double* Lba = Db + NB * LDT;
    double* os = Lba + NB * LDT;
    if (triple) {
      tile_to_lds(Dinv + (int64_t)(2 * K) * NB * NB, NB, Da);
      tile_to_lds(Dinv + (int64_t)(2 * K + 1) * NB * NB, NB, Db);
      tile_to_lds(L + (r0 + NB) * ldl + r0, ldl, Lba);
    } else {
      form_block_inverse(s, Dinv, L, ldl, K);
    }
    if (t < SB) s.vs[t] = zin[r0 + t];
    GPX_POTRS_FIT_STAMP(1);
    double acc[4][1] = {{0.0}, {0.0}, {0.0}, {0.0}};
    auto consume = [&](const TileRegs& R, int jj) {
      if (!sweep_block<1>(ga + (int64_t)(nb - 1 - jj) * SB * 2, 2u, zw, abort_word, limit) && lane == 0) s_abort = 1;
      fma_bwd<1>(acc, R, zw);
    };
    for (int jj = 0; jj < jcount; jj += 2) {  // the next tile loads while the current one's block is awaited
      const bool two = jj + 1 < jcount;
      if (two) load_tile(tb, jj + 1);
      consume(ta, jj);
      if (!two) break;
      if (jj + 2 < jcount) load_tile(ta, jj + 2);
      consume(tb, jj + 1);
    }
    acc[0][0] += xor_lane<1>(acc[0][0]);
    GPX_POTRS_FIT_STAMP(2);
    __syncthreads();  // s.vs, the staged blocks and every wave's abort flag
    if ((t & 1) == 0) s.vs[t >> 1] -= acc[0][0];
    __syncthreads();
    const bool aborted = s_abort != 0;
    if (triple) {
      gemv64<1, true, false>(os + NB, Db, s.vs + NB);
      __syncthreads();
      gemv64<1, true, true>(s.vs, Lba, os + NB);
      __syncthreads();
      gemv64<1, true, false>(os, Da, s.vs);
      __syncthreads();
      if (aborted && t < SB) os[t] = __builtin_nan("");
      __syncthreads();
      publish_block<1>(ga + r0 * 2, 2u, os);
      if (t < SB) alpha[r0 + t] = (r0 + t < n || aborted) ? os[t] : 0.0;
    } else {
      // alpha_K = D_KK^T v: thread (c, h) sums rows 64 h .. 64 h + 63 of column c (four independent chains)
      const int c = t >> 1, h = t & 1;
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int i0 = 0; i0 < NB; i0 += 16) {
        double dd[16];
        double2 vv[8];
#pragma unroll
        for (int i = 0; i < 16; ++i) dd[i] = s.Dk[(NB * h + i0 + i) * LDK + c];
#pragma unroll
        for (int i = 0; i < 8; ++i) vv[i] = *reinterpret_cast<const double2*>(s.vs + NB * h + i0 + 2 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          a4[(2 * i) & 3] = fma(dd[2 * i], vv[i].x, a4[(2 * i) & 3]);
          a4[(2 * i + 1) & 3] = fma(dd[2 * i + 1], vv[i].y, a4[(2 * i + 1) & 3]);
        }
      }
      double a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      a += xor_lane<1>(a);
      if (aborted) a = __builtin_nan("");
      const unsigned long long u = __double_as_longlong(a);
      __hip_atomic_store(ga + (r0 + c) * 2 + h, (2ull << 32) | (h ? (u >> 32) : (u & 0xffffffffull)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      if (h == 0) alpha[r0 + c] = (r0 + c < n || aborted) ? a : 0.0;
    }
    GPX_POTRS_FIT_STAMP(5);
    __syncthreads();  // LDS reuse by the next item
  }
}

template <int NR>
__device__ void potrs_items(int n, int npad, const double* __restrict__ L, int64_t ldl, const double* __restrict__ Dinv,
                            const double* __restrict__ Y, int64_t ldy, int nrhs, double const_mean,
                            double* __restrict__ alpha, gu64* gz, gu64* ga, gu32* abort_word, unsigned limit,
                            SolveLds<NR>& s, int& s_abort, const double* __restrict__ zin) {
  const int t = threadIdx.x, w = t >> 6;
  double* zw = s.zw[w];
  const int nb = npad / SB;
  const int G = gridDim.x;
  // blocks g, g + G, ... of this workgroup: forward ascending, then backward descending (see the file comment)
  const int nown = (nb - (int)blockIdx.x + G - 1) / G;
  for (int step = zin ? nown : 0; step < 2 * nown; ++step) {
    const bool fwd = step < nown;
    const int K = (int)blockIdx.x + (fwd ? step : 2 * nown - 1 - step) * G;
    const int64_t r0 = (int64_t)K * SB;
    const int jcount = fwd ? K : nb - 1 - K;
    auto jblk = [&](int jj) { return fwd ? jj : nb - 1 - jj; };
    TileRegs ta;
    auto load_tile = [&](TileRegs& R, int jj) {
      if (fwd)
        load_tile_fwd(R, L, ldl, r0, (int64_t)jblk(jj) * SB);
      else
        load_tile_bwd(R, L, ldl, (int64_t)jblk(jj) * SB, r0);
    };
    if (jcount > 0) load_tile(ta, 0);
    // diagonal 128-block: D_a, D_b (potrf's inverses of the 64-blocks) and L_ba
    if (fwd || step != nown || zin) {  // the first backward item reuses the last forward item's diagonal block
      tile_to_lds(Dinv + (int64_t)(2 * K) * NB * NB, NB, s.Da);
      tile_to_lds(Dinv + (int64_t)(2 * K + 1) * NB * NB, NB, s.Db);
      tile_to_lds(L + (r0 + NB) * ldl + r0, ldl, s.Lba);
    }
    if (fwd) {
      for (int e = t; e < SB * NR; e += WG) {
        const int row = e / NR, rr = e % NR;
        const int64_t gi = r0 + row;
        s.vs[e] = (rr < nrhs && gi < n) ? Y[gi * ldy + rr] - const_mean : 0.0;
      }
    } else if (zin) {
      for (int e = t; e < SB * NR; e += WG) s.vs[e] = zin[r0 * NR + e];
    } else if (w == 0) {
      if (!sweep_block<NR>(gz + r0 * NR * 2, 1u, s.vs, abort_word, limit) && (t & 63) == 0) s_abort = 1;
    }
    double acc[4][NR];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) acc[k][rr] = 0.0;
    // one register tile (the sweep's 4 NR granules per lane and 4 NR accumulators leave no room for a second one)
    for (int jj = 0; jj < jcount; ++jj) {
      if (jj > 0) load_tile(ta, jj);
      if (!sweep_block<NR>((fwd ? gz : ga) + (int64_t)jblk(jj) * SB * NR * 2, fwd ? 1u : 2u, zw, abort_word, limit) &&
          (t & 63) == 0)
        s_abort = 1;
      if (fwd)
        fma_fwd<NR>(acc, ta, zw);
      else
        fma_bwd<NR>(acc, ta, zw);
    }
    __syncthreads();  // staged diagonal block, right-hand side and the abort flag of every wave's sweeps
    const bool aborted = s_abort != 0;
    if (fwd) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
          acc[k][rr] += __shfl_xor(acc[k][rr], 1);
          acc[k][rr] += __shfl_xor(acc[k][rr], 2);
          acc[k][rr] += __shfl_xor(acc[k][rr], 4);
        }
      if ((t & 7) == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int rr = 0; rr < NR; ++rr) s.vs[((t >> 3) + 32 * k) * NR + rr] -= acc[k][rr];
      }
    } else {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) acc[0][rr] += __shfl_xor(acc[0][rr], 1);
      if ((t & 1) == 0) {
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) s.vs[(t >> 1) * NR + rr] -= acc[0][rr];
      }
    }
    __syncthreads();
    if (fwd) {
      gemv64<NR, false, false>(s.os, s.Da, s.vs);
      __syncthreads();
      gemv64<NR, false, true>(s.vs + NB * NR, s.Lba, s.os);
      __syncthreads();
      gemv64<NR, false, false>(s.os + NB * NR, s.Db, s.vs + NB * NR);
    } else {
      gemv64<NR, true, false>(s.os + NB * NR, s.Db, s.vs + NB * NR);
      __syncthreads();
      gemv64<NR, true, true>(s.vs, s.Lba, s.os + NB * NR);
      __syncthreads();
      gemv64<NR, true, false>(s.os, s.Da, s.vs);
    }
    __syncthreads();
    if (aborted) {
      for (int e = t; e < SB * NR; e += WG) s.os[e] = __builtin_nan("");
      __syncthreads();
    }
    publish_block<NR>((fwd ? gz : ga) + r0 * NR * 2, fwd ? 1u : 2u, s.os);
    if (!fwd) {
      for (int e = t; e < SB * nrhs; e += WG) {
        const int row = e / nrhs, rr = e % nrhs;
        alpha[(r0 + row) * nrhs + rr] = (r0 + row < n || aborted) ? s.os[row * NR + rr] : 0.0;
      }
    }
    __syncthreads();  // LDS reuse by the next item
  }
}

template <int NR>
__global__ void __launch_bounds__(WG) potrs_kernel(int n, int npad, const double* __restrict__ L, int64_t ldl,
                                                   const double* __restrict__ Dinv, const double* __restrict__ Y,
                                                   int64_t ldy, int nrhs, double const_mean, double* __restrict__ alpha,
                                                   int32_t* __restrict__ info, unsigned long long* granules,
                                                   unsigned* abort_ptr, int64_t sl, int64_t sd, int64_t sy, int64_t sa,
                                                   int64_t sg, unsigned limit, const double* __restrict__ zin,
                                                   int64_t sz, const double* __restrict__ means) {
  const int prob = blockIdx.y;
  if (means) const_mean = means[prob];  // per-problem kernel parameters (Batch::means)
  if (zin) zin += prob * sz;
  L += prob * sl;
  Dinv += prob * sd;
  Y += prob * sy;
  alpha += prob * sa;
  gu64* gz = (gu64*)(granules + prob * sg);  // forward blocks (epoch 1)
  gu64* ga = gz + (int64_t)npad * NR * 2;     // backward blocks (epoch 2)
  gu32* abort_word = (gu32*)(abort_ptr + prob);
  if (info && *(volatile int32_t*)(info + prob) != 0) return;  // failed factor: nothing to solve (uniform per problem)
  __shared__ int s_abort;
  if (threadIdx.x == 0) s_abort = 0;
  if constexpr (NR == 1) {
    __shared__ __attribute__((aligned(16))) SolveLds1 s;
    __syncthreads();
    if (zin)
      potrs_bwd_fit_1(n, npad, L, ldl, Dinv, alpha, ga, abort_word, limit, s, s_abort, zin);
    else
      potrs_items_1(n, npad, L, ldl, Dinv, Y, ldy, const_mean, alpha, gz, ga, abort_word, limit, s, s_abort);
  } else {
    __shared__ __attribute__((aligned(16))) SolveLds<NR> s;
    __syncthreads();
    potrs_items<NR>(n, npad, L, ldl, Dinv, Y, ldy, nrhs, const_mean, alpha, gz, ga, abort_word, limit, s, s_abort,
                    zin);
  }
  // a timed-out hand-off: alpha holds NaN; the problem's pivot word reports it (GPX_INFO_TIMEOUT), so a caller that
  // checks info never mistakes the NaN scores for a result
  __syncthreads();
  if (threadIdx.x == 0 && s_abort && info) atomicCAS(info + prob, 0, (int32_t)GPX_INFO_TIMEOUT);
}

size_t potrs_granule_bytes(int64_t npad, int64_t nrhs) {
  const int64_t nr = nrhs == 1 ? 1 : GPX_MAX_RHS;
  return (size_t)(2 * npad * nr * 2) * sizeof(unsigned long long);
}

size_t potrs_clear_bytes(int64_t npad, int64_t nrhs, int64_t batch) {
  return ((potrs_granule_bytes(npad, nrhs) * batch + 4 * (size_t)batch) + 15) & ~(size_t)15;
}

hipError_t launch_potrs(Context* c, int n, int npad, const double* L, int64_t ldl, const double* Dinv,
                        const double* Y, int64_t ldy, int nrhs, double const_mean, double* alpha,
                        int32_t* info, void* ws, const Batch& bt, bool ws_cleared, const double* z, int64_t sz) {
  LaunchTimer tm(c, GPX_TIMER_ALPHA);
  const int nb = npad / SB;
  // granules of every problem, then one abort word per problem; zeroed as ONE block from the workspace start (by the
  // fit's Gram launch, or here)
  const size_t gbytes = potrs_granule_bytes(npad, nrhs);
  auto* granules = reinterpret_cast<unsigned long long*>(ws);
  auto* abort_word = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) + gbytes * bt.count);
  if (!ws_cleared) {
    hipError_t e = hipMemsetAsync(ws, 0, potrs_clear_bytes(npad, nrhs, bt.count), c->stream);
    if (e != hipSuccess) return e;
  }
  // co-resident grid: one workgroup per CU (124 / 135 KB of LDS at NR = 8 / 1), split over the batch
  if (c->cu_count <= 0) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    c->cu_count = cus;
  }
  int G = c->cu_count / bt.count;
  if (G < 1) G = 1;
  if (G > nb) G = nb;
  const int64_t sg = (int64_t)(gbytes / sizeof(unsigned long long));
  if (nrhs == 1)
    potrs_kernel<1><<<dim3(G, bt.count), WG, 0, c->stream>>>(n, npad, L, ldl, Dinv, Y, ldy, nrhs, const_mean, alpha,
                                                             info, granules, abort_word, bt.k, bt.dinv, bt.y,
                                                             bt.alpha, sg, c->spin_limit, z, sz, bt.means);
  else
    potrs_kernel<GPX_MAX_RHS><<<dim3(G, bt.count), WG, 0, c->stream>>>(n, npad, L, ldl, Dinv, Y, ldy, nrhs,
                                                                       const_mean, alpha, info, granules, abort_word,
                                                                       bt.k, bt.dinv, bt.y, bt.alpha, sg, c->spin_limit,
                                                                       z, sz, bt.means);
  return hipGetLastError();
}

size_t potrs_forward_offset(int64_t npad, int64_t nrhs, int64_t batch) {
  return (potrs_clear_bytes(npad, nrhs, batch) + 255) & ~(size_t)255;
}

size_t potrs_workspace_bytes(int64_t npad, int64_t nrhs, int64_t batch) {
  return potrs_forward_offset(npad, nrhs, batch) + (size_t)(2 * npad * rhs_row((int)nrhs)) * 8 * batch + 64;
}

}  // namespace gpx
