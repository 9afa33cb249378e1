// Persistent dataflow Cholesky (lower, NB = 64) for npad <= 4096: ONE launch per factorisation (per batch).
// DIAGNOSTIC PROBE BUILD ONLY (tools/dag_probe.hip): measured slower than the library's multi-launch schedule at every
// size, so it is not part of libgpx.
// SURVEY §8a row a4 (psd_safe_cholesky in GPyTorch's exact path [upstream], reached from
// optimization/Bayesian.py:89-94); the failing pivot is reported in *info for the jitter retry of
// optimization/Bayesian6.py:481-488.
//
// Why: the multi-launch schedule (gpx_potrf.hip) runs one launch per block column, and every launch lasts as long as its
// slowest workgroup: at n = 4096 the first ~22 launches are bound by the trailing update (2-3x the ~20 us panel chain)
// and every launch pays a kernel boundary (3.3-3.9 us).  Here the work is a dataflow graph inside one launch:
//  * the CHAIN workgroup (blockIdx.x == 0) owns the critical path.  Step c: wait until tiles (c, c-1) and (c, c) hold
//    every update of columns < c-1, L_{c,c-1} = A_{c,c-1} D_{c-1}^T (D_{c-1} = L_{c-1,c-1}^{-1} is still in its LDS),
//    A_cc -= L_{c,c-1} L_{c,c-1}^T, then factor A_cc in LDS (four 16-pivot in-wave blocks, gpx_chol64.h) while the other
//    waves build the full inverse D_c = L_cc^{-1} block row by block row.  L and D leave as write-through stores.
//  * POOL workgroups take tasks from a host-scheduled list (one atomic ticket per task):
//      FR(i, k)        L_ik = A_ik D_k^T, then A_{i,k+1} -= L_ik L_{k+1,k}^T     (the next panel column, row i)
//      U64(i, j, k0, k1)   A_ij -= sum_{k0 <= k < k1} L_ik L_jk^T  on one 64x64 block
//      U128(I, J, k0, k1)  the same on the 128x128 tile of blocks (2I, 2I+1) x (2J, 2J+1)
//    Column j receives stage j-1 from FR (the chain for the diagonal block), stage j-2 from U64 "next column" tasks,
//    and (odd j) stage j-3 from U64 as well; every earlier stage comes from U128 tiles of the 128-column pair j/2, whose
//    stages are aggregated into K = 64 g products while the pair is far from the front (each C tile read and written
//    once per g columns instead of every column).
//  Dependencies are per-block version counters (stages applied), per-row counters of published L_ik and the chain's
//  progress word.  Hand-offs follow cdna_hip_programming.md §6 Guideline 16 in its sc1 form (MI355X_MICROARCH.md
//  § visibility, valid-forms table row 1): every handed-off byte is stored with an sc1 (write-through) store, every
//  storing wave drains (s_waitcnt vmcnt(0)), a workgroup barrier, then ONE lane stores the counter; the consumer's one
//  wave polls with sc1 loads, a barrier, then EVERY load of handed-off bytes is an sc1 buffer load; one workgroup per
//  CU (LDS > 80 KB).  Spins are bounded; an abort word (pivot failure or timeout) makes every waiter give up.
//  The task order is a host simulation's start order (a topological order of the graph), so a task only waits on the
//  chain or on tasks earlier in the list: with the chain resident and any number of resident pool workgroups the graph
//  drains.  The arithmetic of every task is fixed (the schedule decides who runs it, never how), so the factor does not
//  depend on timing or placement and a batched factorisation equals single ones bit for bit.
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_chol64.h"
#include <algorithm>
#include <climits>
#include <cmath>
#include <map>
#include <memory>
#include <vector>

// Optional timestamp hooks for tools/dag_probe.hip (compiled out in the library).
#ifndef GPX_DAG_STAMP
#define GPX_DAG_STAMP(kind, a, b, s)
#endif
#ifndef GPX_DAG_TASK_STAMP
#define GPX_DAG_TASK_STAMP(idx, s)
#endif

namespace gpx {
// entry points of this probe build (not part of libgpx)
int potrf_dag_workers(Context* c, int npad, int batch);
hipError_t launch_potrf_dag(Context* c, int npad, double* A, int64_t lda, double* Dinv, int32_t* info,
                            const Batch& bt, double* W, int64_t ldw, const ForwardRhs* fr = nullptr);
void potrf_dag_release(Context* c);

namespace dag {

constexpr int LD = LD64;              // LDS row length of a 64x64 tile (doubles)
constexpr int TILE_D = NB * LD;       // doubles per LDS tile
constexpr int HDR = 16;               // sync words before the per-row counters
enum { W_CHAIN = 0, W_ABORT = 1, W_TICKET = 2 };  // tickets: W_TICKET + list (0 critical, 1 front, 2 bulk)
enum { T_FR = 1, T_U64 = 2, T_U128 = 3 };

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kSC1 = 16;  // aux operand of the buffer intrinsics: sc1

__device__ __forceinline__ rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double2 ld2(rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSC1);
  return make_double2(__longlong_as_double(((unsigned long long)v.y << 32) | v.x),
                      __longlong_as_double(((unsigned long long)v.w << 32) | v.z));
}
__device__ __forceinline__ double ld1(rsrc_t r, int off) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSC1);
  return __longlong_as_double(((unsigned long long)v.y << 32) | v.x);
}
__device__ __forceinline__ void st2(rsrc_t r, int off, double a, double b) {
  const unsigned long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  const u32x4 v = {(unsigned)x, (unsigned)(x >> 32), (unsigned)y, (unsigned)(y >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSC1);
}
__device__ __forceinline__ void st1(rsrc_t r, int off, double a) {
  const unsigned long long x = __double_as_longlong(a);
  const u32x2 v = {(unsigned)x, (unsigned)(x >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, kSC1);
}

struct Sync {
  int* w;
  int nblk;
  __device__ int* chain() const { return w + W_CHAIN; }
  __device__ int* abort_word() const { return w + W_ABORT; }
  __device__ int* ticket(int which) const { return w + W_TICKET + which; }
  __device__ int* lrow(int i) const { return w + HDR + i; }
  __device__ int* ver(int i, int j) const { return w + HDR + nblk + i * nblk + j; }
};

__host__ __device__ inline int sync_words(int nblk) { return (HDR + nblk + nblk * nblk + 3) & ~3; }

// One wave polls: lane l waits for *mine >= want (mine == nullptr: satisfied).  Returns false once the abort word is set
// (or this wave sets it after `limit` spins: timeout).
__device__ __forceinline__ bool wave_wait(const Sync& s, const int* mine, int want, unsigned limit) {
  const int lane = threadIdx.x & 63;
  for (unsigned spins = 0;; ++spins) {
    const bool ok = !mine || __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
    if (__all(ok)) return true;
    if (spins >= limit) {
      if (lane == 0) __hip_atomic_store(s.abort_word(), 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if ((spins & 63) == 63 && __hip_atomic_load(s.abort_word(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
      return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// Workgroup wait: wave 0 polls, every wave leaves through the same barrier (uniform result).  After it, handed-off
// bytes are read with sc1 loads only.
__device__ __forceinline__ bool wg_wait(const Sync& s, const int* mine, int want, unsigned limit) {
  int ok = 1;
  if (threadIdx.x < 64) ok = wave_wait(s, mine, want, limit) ? 1 : 0;
  return __syncthreads_and(ok) != 0;
}

// Every storing wave drains its sc1 stores, a barrier, then lanes 0 .. nw-1 of wave 0 store their word.
__device__ __forceinline__ void wg_publish(int* word, int value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && word) __hip_atomic_store(word, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 64x64 tile (row-major, leading dimension ld) -> LDS (row length LD), sc1 loads, all issued before the LDS writes.
__device__ __forceinline__ void tile_in(const double* G, int64_t ld, double* S) {
  const rsrc_t r = rsrc(G);
  const int t = threadIdx.x;
  double2 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, rr = e >> 6, cc = e & 63;
    v[q] = ld2(r, (int)(((int64_t)rr * ld + cc) * 8));
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, rr = e >> 6, cc = e & 63;
    S[rr * LD + cc] = v[q].x;
    S[rr * LD + cc + 1] = v[q].y;
  }
}

// LDS tile -> global (sc1); LOWER: 16-blocks above the block diagonal stored as zeros.
template <bool LOWER>
__device__ __forceinline__ void tile_out(const double* S, double* G, int64_t ld) {
  const rsrc_t r = rsrc(G);
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = (t + q * WG) * 2, rr = e >> 6, cc = e & 63;
    double a = S[rr * LD + cc], b = S[rr * LD + cc + 1];
    if (LOWER && (cc >> 4) > (rr >> 4)) a = b = 0.0;
    st2(r, (int)(((int64_t)rr * ld + cc) * 8), a, b);
  }
}

// Block row w (16 rows) of R = S D^T, D lower triangular (64x64 in LDS): acc[bj] = R(16w.., 16bj..).  The four
// accumulation chains are interleaved per k-step (they share the A operand), so consecutive MFMAs are independent.
__device__ __forceinline__ void rowblock_times_lower_t(d4 (&acc)[4], const double* S, const double* D, int w) {
  const int lane = threadIdx.x & 63, m = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int bj = 0; bj < 4; ++bj) acc[bj] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const double a = S[(16 * w + m) * LD + 4 * ks + kk];
#pragma unroll
    for (int bj = 0; bj < 4; ++bj)
      if (ks < 4 * (bj + 1)) acc[bj] = mfma16x16x4(a, D[(16 * bj + m) * LD + 4 * ks + kk], acc[bj]);
  }
}

// Block row w of C - R Q^T (64x64 operands in LDS, full K = 64), four chains interleaved: acc[bj] = C(16w.., 16bj..)
// - sum_k R(16w + ., k) Q(16bj + ., k).
__device__ __forceinline__ void rowblock_sub_abt(d4 (&acc)[4], const double* C, const double* R, const double* Q, int w) {
  const int lane = threadIdx.x & 63, m = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int bj = 0; bj < 4; ++bj) acc[bj] = load_block16(C, 16 * w, 16 * bj);
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const double a = -R[(16 * w + m) * LD + 4 * ks + kk];
#pragma unroll
    for (int bj = 0; bj < 4; ++bj) acc[bj] = mfma16x16x4(a, Q[(16 * bj + m) * LD + 4 * ks + kk], acc[bj]);
  }
}

// Blocks (I0,J0), (I1,J1), (I2,J2) of A -= L L^T (K = 64, L in LDS), three chains interleaved.
template <int I0, int J0, int I1, int J1, int I2, int J2>
__device__ __forceinline__ void syrk3(double* sA, const double* L) {
  const int lane = threadIdx.x & 63, m = lane & 15, kk = lane >> 4;
  d4 c0 = load_block16(sA, 16 * I0, 16 * J0), c1 = load_block16(sA, 16 * I1, 16 * J1),
     c2 = load_block16(sA, 16 * I2, 16 * J2);
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 4 * ks + kk;
    c0 = mfma16x16x4(-L[(16 * I0 + m) * LD + k], L[(16 * J0 + m) * LD + k], c0);
    c1 = mfma16x16x4(-L[(16 * I1 + m) * LD + k], L[(16 * J1 + m) * LD + k], c1);
    c2 = mfma16x16x4(-L[(16 * I2 + m) * LD + k], L[(16 * J2 + m) * LD + k], c2);
  }
  store_block16(sA, 16 * I0, 16 * J0, c0);
  store_block16(sA, 16 * I1, 16 * J1, c1);
  store_block16(sA, 16 * I2, 16 * J2, c2);
}

template <int I0, int J0>
__device__ __forceinline__ void syrk1(double* sA, const double* L) {
  const int lane = threadIdx.x & 63, m = lane & 15, kk = lane >> 4;
  d4 c0 = load_block16(sA, 16 * I0, 16 * J0);
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 4 * ks + kk;
    c0 = mfma16x16x4(-L[(16 * I0 + m) * LD + k], L[(16 * J0 + m) * LD + k], c0);
  }
  store_block16(sA, 16 * I0, 16 * J0, c0);
}

// A -= L L^T on the ten lower / diagonal 16-blocks of a 64x64 tile (both in LDS), three blocks per wave at most
__device__ __forceinline__ void syrk_lower(double* sA, const double* L, int w) {
  if (w == 0) syrk3<0, 0, 1, 0, 1, 1>(sA, L);
  else if (w == 1) syrk3<2, 0, 2, 1, 2, 2>(sA, L);
  else if (w == 2) syrk3<3, 0, 3, 1, 3, 2>(sA, L);
  else syrk1<3, 3>(sA, L);
}

// acc (block row w of a 64x64 result, acc layout) -> global tile G (sc1, 8-byte stores) and, optionally, LDS S.
__device__ __forceinline__ void rowblock_out(const d4 (&acc)[4], int w, double* G, int64_t ld, double* S) {
  const rsrc_t r = rsrc(G);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int bj = 0; bj < 4; ++bj)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * w + (lane >> 4) + 4 * q, col = 16 * bj + (lane & 15);
      if (G) st1(r, (int)(((int64_t)row * ld + col) * 8), acc[bj][q]);
      if (S) S[row * LD + col] = acc[bj][q];
    }
}

// Rows 0..15 of an LDS tile -> global (sc1), by waves 1-3 (the chain's S row of wave 0)
__device__ __forceinline__ void rows16_out(const double* S, double* G, int64_t ld) {
  const rsrc_t r = rsrc(G);
  for (int e = threadIdx.x - 64; e < 16 * 32; e += WG - 64) {
    const int row = e >> 5, col = 2 * (e & 31);
    st2(r, (int)(((int64_t)row * ld + col) * 8), S[row * LD + col], S[row * LD + col + 1]);
  }
}

// ---- forward substitution folded into the factorisation -----------------------------------------------------------
// z = L^{-1} b, b = Y - mean (0 on padded rows / right-hand sides), block row by block row: y_i = b_i - sum_{k<i} L_ik z_k
// accumulates in stage order (FR(i, k) applies stage k right after its L_ik, before it publishes anything that lets
// stage k+1 of row i start; the chain applies stage c-1 of row c after its S), and z_c = D_c y_c.  The triangular solve
// then runs its backward half only (gpx_potrs.hip).  Right-hand sides are rows of NR doubles (NR = 1, or GPX_MAX_RHS).
struct Fwd {
  const double* Y;  // nullptr: no forward substitution in this launch
  int64_t ldy, sy, sf;  // sy: Y stride per problem; sf: yb / zb stride per problem
  int nrhs, n, nr;
  double mean;
  double* yb;  // running right-hand sides, npad x nr (written and read in this launch: sc1)
  double* zb;  // z, npad x nr
  // this problem's arrays (read from the kernel arguments where they are used: no registers held across the tasks)
  __device__ const double* y_in() const { return Y + (int64_t)blockIdx.y * sy; }
  __device__ double* ybuf() const { return yb + (int64_t)blockIdx.y * sf; }
  __device__ double* zbuf() const { return zb + (int64_t)blockIdx.y * sf; }
};

__device__ __forceinline__ double rhs_b(const Fwd& f, int row, int rr) {
  return (row < f.n && rr < f.nrhs) ? f.y_in()[(int64_t)row * f.ldy + rr] - f.mean : 0.0;
}

// The 16-row layout of a wave: lane = 4 i + q (row i of the block, quarter q of the 64 columns).  The lane's own
// right-hand sides after the reduction: NR = 1: q = 0 holds rr 0; NR = 8: lane q holds rr 2q and 2q+1.
template <int NR>
__device__ __forceinline__ int own_rr(int q, int e) {
  return NR == 1 ? ((q == 0 && e == 0) ? 0 : -1) : 2 * q + e;
}

// The lane's two sums of own_rr of row i of a 16-row block, sum_j M(i, j) x(j, rr) (M rows in LDS with row stride LD,
// x in LDS as 64 x NR): lane (i, q) sums j in [16q, 16q + 16) (LOWER: only column blocks q <= rowblk), then the four
// partials of a row are combined by a reduce-scatter over lanes q ^ 2 and q ^ 1 (NR = 8) or two xor shuffles (NR = 1):
// every sum in one fixed order, without indexing registers by lane.
template <int NR, bool LOWER>
__device__ __forceinline__ void gemv16(double (&out)[2], const double* M, const double* x, int rowblk) {
  const int lane = threadIdx.x & 63, i = lane >> 2, q = lane & 3;
  double p[NR];
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) p[rr] = 0.0;
  if (!LOWER || q <= rowblk) {
#pragma unroll 4
    for (int jj = 0; jj < 16; ++jj) {
      const int j = 16 * q + jj;
      const double m = M[i * LD + j];
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) p[rr] = fma(m, x[j * NR + rr], p[rr]);
    }
  }
  if constexpr (NR == 1) {
    p[0] += __shfl_xor(p[0], 1);
    p[0] += __shfl_xor(p[0], 2);
    out[0] = p[0];
    out[1] = 0.0;
  } else {
    static_assert(NR == 8, "one or eight right-hand sides");
    const bool hi2 = (q & 2) != 0, hi1 = (q & 1) != 0;
    double a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double keep = hi2 ? p[j + 4] : p[j], send = hi2 ? p[j] : p[j + 4];
      a[j] = keep + __shfl_xor(send, 2);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const double keep = hi1 ? a[j + 2] : a[j], send = hi1 ? a[j] : a[j + 2];
      out[j] = keep + __shfl_xor(send, 1);
    }
  }
}

// The lane's two y values of row `row` (global): from b on the row's first stage, else from yb (sc1)
template <int NR>
__device__ __forceinline__ void load_y(const Fwd& f, int row, bool first, double (&y)[2]) {
  const int q = threadIdx.x & 3;
  const rsrc_t r = rsrc(f.ybuf());
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int rr = own_rr<NR>(q, e);
    y[e] = 0.0;
    if (rr >= 0) y[e] = first ? rhs_b(f, row, rr) : ld1(r, (int)(((int64_t)row * NR + rr) * 8));
  }
}

// y -= L z on the wave's 16 rows (L rows in LDS), the result into yb (sc1) or LDS (ys: 64 x NR, row i0 + i)
template <int NR>
__device__ __forceinline__ void fwd_rows16(const Fwd& f, const double* Lrows, const double* zs, double (&y)[2], int row,
                                           double* ys, int i0) {
  const int lane = threadIdx.x & 63, i = lane >> 2, q = lane & 3;
  double p[2];
  gemv16<NR, false>(p, Lrows, zs, 0);
  const rsrc_t r = rsrc(f.ybuf());
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int rr = own_rr<NR>(q, e);
    if (rr < 0) continue;
    const double v = y[e] - p[e];
    if (ys)
      ys[(i0 + i) * NR + rr] = v;
    else
      st1(r, (int)(((int64_t)row * NR + rr) * 8), v);
  }
}

// z rows of 16-row block rb of chain block c: z = D y (D in LDS, y in LDS 64 x NR) -> zs (LDS) and zb (sc1)
template <int NR>
__device__ __forceinline__ void z_rows16(const Fwd& f, const double* D, const double* ys, int c, int rb, double* zs) {
  const int lane = threadIdx.x & 63, i = lane >> 2, q = lane & 3;
  double p[2];
  gemv16<NR, true>(p, D + 16 * rb * LD, ys, rb);
  const rsrc_t r = rsrc(f.zbuf());
  const int row = 16 * rb + i;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int rr = own_rr<NR>(q, e);
    if (rr < 0) continue;
    const double v = p[e];
    if (zs) zs[row * NR + rr] = v;
    st1(r, (int)(((int64_t)(c * NB + row) * NR + rr) * 8), v);
  }
}

// ---- one step of the chain ---------------------------------------------------------------------------------------
// In: sA = A_cc and (c > 0) sB = A_{c,c-1}, both holding every update of columns < c-1; sX = D_{c-1}.
//  (c > 0) S: every wave computes its block row of L_{c,c-1} = A_{c,c-1} D_{c-1}^T into sB and global memory (sc1).
//      Wave 0 then applies A_00 -= L_0 L_0^T (its own rows only) and goes straight into the first pivot block; waves
//      1-3 wait for the four L block rows (LDS counter) and apply the nine other blocks of A_cc -= L L^T while it runs.
//  Pivot block s (0..3): wave 0 factors + inverts block (s, s) in registers (chol16), then - without a barrier - the
//      T and U items of block row s+1 and the next pivot block; waves 1-3 do the other T items (L_is = A_is D_ss^T),
//      the U items (A_ij -= L_is L_js^T) and block row s of the inverse, X_sj = -D_ss sum_{k=j}^{s-1} L_sk X_kj.
//  After pivot blocks 1 and 2, waves 1-3 look (one poll) whether the next step's tiles (c+1, c) and (c+1, c+1) are
//      final through column c-1 and, once they are, load them into sB / sN (the 64 x 128 strip, one third per wave).
// Out: sA = L_cc (lower 16-blocks), sX = D_c.  Returns the failing pivot 0..63 or -1, uniform; *pref == 3: prefetched.
struct ChainShared {
  int cnt, srow, fail, pref, prefdone, pub, zcnt;
};

__device__ __forceinline__ void prefetch_share(const double* strip, int64_t ld, double* sB, double* sN, int w) {
  const int lane = threadIdx.x & 63;
  const rsrc_t r = rsrc(strip);
  const int col = 2 * lane;  // 0 .. 126 over the 128 columns of the strip
  double* dst = col < NB ? sB : sN;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    double2 v[11];
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      const int row = (w - 1) + 3 * (11 * half + q);
      if (row < NB) v[q] = ld2(r, (int)(((int64_t)row * ld + col) * 8));
    }
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      const int row = (w - 1) + 3 * (11 * half + q);
      if (row < NB) {
        dst[row * LD + (col & 63)] = v[q].x;
        dst[row * LD + (col & 63) + 1] = v[q].y;
      }
    }
  }
}

// Output of the previous step by waves 1-3 (one third of the rows each): L_pp (its lower 16-blocks, zeros above)
// and D_p into global memory (sc1), and - for a fit that forms W - W_pp = D_p^T (plain stores: W is not read in the
// launch) with the strictly lower 64-block of an odd 128-tile zeroed.
__device__ __forceinline__ void store_prev(const double* sL, const double* sD, double* Lg, int64_t lda, double* Dg,
                                           double* W, int64_t ldw, int p, int w) {
  const int lane = threadIdx.x & 63;
  const rsrc_t rl = rsrc(Lg), rd = rsrc(Dg);
  const int col = 2 * (lane & 31);
  for (int row = (w - 1) * 2 + (lane >> 5); row < NB; row += 6) {
    double a = sL[row * LD + col], b = sL[row * LD + col + 1];
    if ((col >> 4) > (row >> 4)) a = b = 0.0;
    st2(rl, (int)(((int64_t)row * lda + col) * 8), a, b);
    double x = sD[row * LD + col], y = sD[row * LD + col + 1];
    if ((col >> 4) > (row >> 4)) x = y = 0.0;
    st2(rd, (int)(((int64_t)row * NB + col) * 8), x, y);
  }
  if (W) {
    double* Wpp = W + (int64_t)p * NB * ldw + (int64_t)p * NB;
    for (int e = threadIdx.x - 64; e < NB * NB; e += WG - 64) {
      const int r = e >> 6, cc = e & 63;
      Wpp[(int64_t)r * ldw + cc] = ((r >> 4) > (cc >> 4)) ? 0.0 : sD[cc * LD + r];
    }
    if (p & 1) {
      double* Z = W + (int64_t)p * NB * ldw + (int64_t)(p - 1) * NB;
      for (int e = threadIdx.x - 64; e < NB * NB; e += WG - 64) Z[(int64_t)(e >> 6) * ldw + (e & 63)] = 0.0;
    }
  }
}

__device__ __forceinline__ int chain_step(const Sync& s, int c, int nblk, double* A, int64_t lda, double* Dinv,
                                          double* W, int64_t ldw, double* sA, double* sB, double* sX, double* sN,
                                          ChainShared& sh, const Fwd& fw, double* fl) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  auto dblk = [&](int q) { return sX + 16 * q * LD + 16 * q; };
  auto tsolve = [&](int i, int q) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    acc = mfma_lds16<true, LD>(acc, sA, 16 * i, 16 * q, dblk(q), 0, 0, 16, 1.0);
    store_block16(sA, 16 * i, 16 * q, acc);
  };
  auto update = [&](int i, int j, int q) {
    d4 acc = load_block16(sA, 16 * i, 16 * j);
    acc = mfma_lds16<true>(acc, sA, 16 * i, 16 * q, sA, 16 * q, 16 * j, 16, -1.0);
    store_block16(sA, 16 * i, 16 * j, acc);
  };
  // sum_{k=j}^{q-1} L_qk X_kj (acc layout), and X_qj = -D_qq P: the accumulator register r of P is the B operand of
  // k-step r (rows 4r + lane/16)
  auto xpart = [&](int q, int j) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int k = j; k < q; ++k) acc = mfma_lds16<false>(acc, sA, 16 * q, 16 * k, sX, 16 * k, 16 * j, 16, 1.0);
    return acc;
  };
  auto xfinish = [&](int q, int j, const d4& acc) {
    const int m = lane & 15, kk = lane >> 4;
    d4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) x = mfma16x16x4(-dblk(q)[m * LD + 4 * r + kk], acc[r], x);
    store_block16(sX, 16 * q, 16 * j, x);
  };
  auto lds_add = [&](int* word) {
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(word, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(old);
  };
  auto lds_wait = [&](int* word, int want) {
    while (__hip_atomic_load(word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < want) __builtin_amdgcn_s_sleep(1);
  };
  const bool has_next = c + 1 < nblk;
  const double* strip = A + (int64_t)(c + 1) * NB * lda + (int64_t)c * NB;  // tiles (c+1, c) | (c+1, c+1)
  bool my_pref = false;
  auto try_prefetch = [&]() {  // waves 1-3 only
    if (!has_next || my_pref) return;
    if (w == 1 && __hip_atomic_load(&sh.pref, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      const int* mine = lane == 0 ? s.ver(c + 1, c) : (lane == 1 ? s.ver(c + 1, c + 1) : nullptr);
      const bool ok = !mine || __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= c;
      if (__all(ok) && lane == 0) __hip_atomic_store(&sh.pref, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (__hip_atomic_load(&sh.pref, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 1) {
      prefetch_share(strip, lda, sB, sN, w);
      my_pref = true;
      lds_add(&sh.prefdone);
    }
  };
  if (t == 0) {
    sh.cnt = 0;
    sh.srow = 0;
    sh.fail = -1;
    sh.pref = 0;
    sh.prefdone = 0;
    sh.pub = 0;
    sh.zcnt = 0;
  }
  __syncthreads();
  // forward substitution: y blocks of waves 1-3 (wave 1: 16-row blocks 0 and 1, waves 2 / 3: block 2 / 3), the running
  // y of the previous / this block in fl (two alternating 64 x NR buffers), z_{c-1} in fl + 2 * 64 * NR
  const bool fwd = fw.Y != nullptr;
  const int yb0 = w == 1 ? 0 : w, ynb = w == 1 ? 2 : 1;
  double yold[2][2];
  double* yprev = fl + ((c + 1) & 1) * NB * GPX_MAX_RHS;
  double* ycur = fl + (c & 1) * NB * GPX_MAX_RHS;
  double* zp = fl + 2 * NB * GPX_MAX_RHS;
  if (c > 0) {
    if (fwd && w > 0) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (b >= ynb) break;
        const int row = c * NB + 16 * (yb0 + b) + (lane >> 2);
        if (fw.nr == 1)
          load_y<1>(fw, row, c == 1, yold[b]);
        else
          load_y<GPX_MAX_RHS>(fw, row, c == 1, yold[b]);
      }
    }
    if (fwd && w >= 2) {
      // z_{c-1} = D_{c-1} y_{c-1} (before chol16 overwrites sX: counted in srow below)
      for (int rb = 2 * (w - 2); rb < 2 * (w - 2) + 2; ++rb) {
        if (fw.nr == 1)
          z_rows16<1>(fw, sX, yprev, c - 1, rb, zp);
        else
          z_rows16<GPX_MAX_RHS>(fw, sX, yprev, c - 1, rb, zp);
      }
      lds_add(&sh.zcnt);
    }
    if (w > 0) {
      // the previous step's L_{c-1,c-1} (in sN) and D_{c-1} (in sX) leave while wave 0 starts this step; the last of
      // waves 1-3 to drain them publishes chain word 2c (D_{c-1} readable: the stage c-1 tasks of the pool start)
      store_prev(sN, sX, A + (int64_t)(c - 1) * NB * lda + (int64_t)(c - 1) * NB, lda,
                 Dinv + (int64_t)(c - 1) * NB * NB, W, ldw, c - 1, w);
    }
    d4 acc[4];
    double* Lrow = A + (int64_t)c * NB * lda + (int64_t)(c - 1) * NB;
    rowblock_times_lower_t(acc, sB, sX, w);  // reads only this wave's rows of sB
    rowblock_out(acc, w, w ? Lrow : nullptr, lda, sB);  // wave 0's rows leave through waves 1-3 below
    GPX_DAG_STAMP(0, c, 0, 1);
    lds_add(&sh.srow);
    if (w == 0) {
      d4 u = load_block16(sA, 0, 0);
      u = mfma_lds16<true>(u, sB, 0, 0, sB, 0, 0, NB, -1.0);
      store_block16(sA, 0, 0, u);
      lds_wait(&sh.srow, 4);  // every wave's S reads of D_{c-1} (and stores of it) are done before chol16 overwrites sX
      GPX_DAG_STAMP(0, c, 0, 2);
    } else {
      // L_{c,c-1} and D_{c-1} leave before the factorisation starts: the last of waves 1-3 to drain publishes chain
      // word 2c+1 (the pool's stage c-1 tasks and the critical task's column c both start from it)
      lds_wait(&sh.srow, 4);
      rows16_out(sB, Lrow, lda);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lds_add(&sh.pub) == 2 && lane == 0)
        __hip_atomic_store(s.chain(), 2 * c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 1) syrk3<1, 0, 2, 1, 3, 1>(sA, sB);
      else if (w == 2) syrk3<1, 1, 2, 2, 3, 2>(sA, sB);
      else syrk3<2, 0, 3, 0, 3, 3>(sA, sB);
      if (fwd) {  // y_c -= L_{c,c-1} z_{c-1} into LDS (z_c = D_c y_c leaves in the next step)
        lds_wait(&sh.zcnt, 2);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if (b >= ynb) break;
          const int rb = yb0 + b;
          if (fw.nr == 1)
            fwd_rows16<1>(fw, sB + 16 * rb * LD, zp, yold[b], 0, ycur, 16 * rb);
          else
            fwd_rows16<GPX_MAX_RHS>(fw, sB + 16 * rb * LD, zp, yold[b], 0, ycur, 16 * rb);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // L_{c,c-1} drained before the first barrier (published after it)
  }
  int fail = -1;
  d4 ptail = {0.0, 0.0, 0.0, 0.0};  // waves 1-3: sum_{k=j}^{2} L_3k X_kj of their block X_3j (j = w - 1), from q = 2
  for (int q = 0; q < 4; ++q) {
    if (w == 0) {
      const int f = chol16<LD>(sA, dblk(q), 16 * q);
      if (f >= 0 && fail < 0) fail = 16 * q + f;
    }
    __syncthreads();  // L_qq, D_qq (q = 0: also A_cc -= L L^T and the stores of L_{c,c-1})
    GPX_DAG_STAMP(0, c, 0, 3 + q);
    if (w == 0) {
      if (q < 3) tsolve(q + 1, q);
      lds_add(&sh.cnt);
      if (q < 3) update(q + 1, q + 1, q);
    } else {
      for (int i = q + 1 + w; i < 4; i += 3) tsolve(i, q);
      lds_add(&sh.cnt);
      lds_wait(&sh.cnt, 4 * (q + 1));
      int e = 0;
      for (int j = q + 1; j < 4; ++j)
        for (int i = j; i < 4; ++i) {
          if (i == q + 1 && j == q + 1) continue;  // wave 0's lookahead item
          if (1 + e % 3 == w) update(i, j, q);
          ++e;
        }
      if (q < 3) {
        for (int j = 0; j < q; ++j)
          if (1 + j % 3 == w) xfinish(q, j, xpart(q, j));
      }
      if (q == 2) {
        // block row 3 of the inverse up to its last factor: X_3j = -D_33 P_3j with P_3j = sum_{k=j}^{2} L_3k X_kj.
        // Wave w takes j = w - 1: X_20 / X_21 are this wave's own step-2 items (wave 1 / 2), L_32 is wave 0's
        // lookahead item (published before the counter above reached 12).
        ptail = xpart(3, w - 1);
      } else if (q == 3) {
        xfinish(3, w - 1, ptail);
      }
      if (q >= 1) try_prefetch();
    }
  }
  if (t == 0) sh.fail = fail;
  __syncthreads();
  GPX_DAG_STAMP(0, c, 0, 7);
  return sh.fail;
}

// ---- tile GEMM tasks from global memory (sc1 operand loads) -------------------------------------------------------
template <int TM>
struct DagTile : MfmaTile<TM, TM, 16, false, false> {
  using Base = MfmaTile<TM, TM, 16, false, false>;
  // operands: rows of A (rsrc at the tile's first row) x k, rows of B x k; element (m, k) at m * ld + k
  __device__ __forceinline__ void load_sc1(rsrc_t a, rsrc_t b, int64_t ld, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < Base::A_LOADS; ++q) {
      const int e = (t + q * WG) * 2, mm = e / 16, kk = e % 16;
      this->ra[q] = ld2(a, (int)(((int64_t)mm * ld + k0 + kk) * 8));
    }
#pragma unroll
    for (int q = 0; q < Base::B_LOADS; ++q) {
      const int e = (t + q * WG) * 2, nn = e / 16, kk = e % 16;
      this->rb[q] = ld2(b, (int)(((int64_t)nn * ld + k0 + kk) * 8));
    }
  }
  __device__ __forceinline__ void load_neg_c_sc1(rsrc_t c, int64_t ld) {
#pragma unroll
    for (int i = 0; i < Base::WM; ++i)
#pragma unroll
      for (int j = 0; j < Base::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          this->acc[i][j][r] = -ld1(c, (int)(((int64_t)Base::row_of(i, r) * ld + Base::col_of(j)) * 8));
  }
  __device__ __forceinline__ void run_acc_sc1(rsrc_t a, rsrc_t b, int64_t ld, int kbeg, int kend, double* smem) {
    double* cur = smem;
    double* nxt = smem + 16 * (Base::PA + Base::PB);
    load_sc1(a, b, ld, kbeg);
    this->store_lds(cur, cur + 16 * Base::PA);
    __syncthreads();
    for (int k0 = kbeg; k0 < kend; k0 += 16) {
      const bool more = (k0 + 16) < kend;
      if (more) load_sc1(a, b, ld, k0 + 16);
      this->compute(cur, cur + 16 * Base::PA);
      if (more) this->store_lds(nxt, nxt + 16 * Base::PA);
      __syncthreads();
      double* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
  }
  // C - A B^T = -acc, stored (sc1) where the element's global 16-block is on or below the block diagonal
  __device__ __forceinline__ void store_lower(rsrc_t c, int64_t ld, int row0, int col0) {
#pragma unroll
    for (int i = 0; i < Base::WM; ++i)
#pragma unroll
      for (int j = 0; j < Base::WN; ++j) {
        const int col = Base::col_of(j);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = Base::row_of(i, r);
          if (((row0 + row) >> 4) >= ((col0 + col) >> 4))
            st1(c, (int)(((int64_t)row * ld + col) * 8), -this->acc[i][j][r]);
        }
      }
  }
};

// ---- roles ---------------------------------------------------------------------------------------------------------
struct Args {
  double* A;
  int64_t lda;
  int nblk;
  double* Dinv;
  int32_t* info;
  double* W;
  int64_t ldw;
  int* sync;
  int64_t sa, sd, sw, ss;  // per-problem strides (A, Dinv, W in doubles; sync in ints)
  const unsigned long long* tasks;  // critical [0, lend[0]), front [lend[0], lend[1]), bulk [lend[1], lend[2])
  int lend[3];
  int wend[2];  // workers: blockIdx.x in [1, wend[0]) critical, [wend[0], wend[1]) front, the rest bulk
  unsigned spin_limit;
  Fwd fw;  // forward substitution (fw.Y == nullptr: none)
};

__device__ void chain_role(const Args& g, double* A, double* Dinv, double* W, int32_t* info, const Sync& s,
                           double* lds, const Fwd& fw, double* fl) {
  double* sA = lds;
  double* sB = lds + TILE_D;
  double* sX = lds + 2 * TILE_D;
  double* sN = lds + 3 * TILE_D;
  __shared__ ChainShared sh;
  const int t = threadIdx.x;
  const int64_t lda = g.lda;
  const int nblk = g.nblk;
  auto blk = [&](int i, int j) { return A + (int64_t)i * NB * lda + (int64_t)j * NB; };
  tile_in(blk(0, 0), lda, sA);
  if (fw.Y)  // y_0 = b_0
    for (int e = t; e < NB * fw.nr; e += WG) fl[e] = rhs_b(fw, e / fw.nr, e % fw.nr);
  __syncthreads();
  for (int c = 0; c < nblk; ++c) {
    GPX_DAG_STAMP(0, c, 0, 0);
    const int f = chain_step(s, c, nblk, A, lda, Dinv, W, g.ldw, sA, sB, sX, sN, sh, fw, fl);
    if (f >= 0) {
      if (t == 0) {
        atomicCAS(info, 0, c * NB + f + 1);
        __hip_atomic_store(s.abort_word(), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
    if (c + 1 == nblk) {  // the last factor and inverse (earlier ones leave during the next step)
      if (fw.Y && (t >> 6) >= 2) {  // and the last z
        const int w = t >> 6;
        for (int rb = 2 * (w - 2); rb < 2 * (w - 2) + 2; ++rb) {
          if (fw.nr == 1)
            z_rows16<1>(fw, sX, fl + (c & 1) * NB * GPX_MAX_RHS, c, rb, nullptr);
          else
            z_rows16<GPX_MAX_RHS>(fw, sX, fl + (c & 1) * NB * GPX_MAX_RHS, c, rb, nullptr);
        }
      }
      tile_out<true>(sA, blk(c, c), lda);
      tile_out<true>(sX, Dinv + (int64_t)c * NB * NB, NB);
      if (W) {
        double* Wcc = W + (int64_t)c * NB * g.ldw + (int64_t)c * NB;
        for (int e = t; e < NB * NB; e += WG) {
          const int r = e >> 6, cc = e & 63;
          Wcc[(int64_t)r * g.ldw + cc] = ((r >> 4) > (cc >> 4)) ? 0.0 : sX[cc * LD + r];
        }
        if (c & 1) {
          double* Z = W + (int64_t)c * NB * g.ldw + (int64_t)(c - 1) * NB;
          for (int e = t; e < NB * NB; e += WG) Z[(int64_t)(e >> 6) * g.ldw + (e & 63)] = 0.0;
        }
      }
      wg_publish(t == 0 ? s.chain() : nullptr, 2 * c + 2);
      GPX_DAG_STAMP(0, c, 0, 8);
      break;
    }
    GPX_DAG_STAMP(0, c, 0, 8);
    if (sh.prefdone < 3) {  // the next tiles were not final during the factorisation: wait, then load them
      const int lane = t & 63;
      const int* mine = lane == 0 ? s.ver(c + 1, c) : (lane == 1 ? s.ver(c + 1, c + 1) : nullptr);
      if (!wg_wait(s, mine, c, g.spin_limit)) break;
      tile_in(blk(c + 1, c), lda, sB);
      tile_in(blk(c + 1, c + 1), lda, sN);
    }
    __syncthreads();
    GPX_DAG_STAMP(0, c, 0, 9);
    double* tmp = sA;  // sA (L_cc, stored during the next step) becomes the next prefetch target
    sA = sN;
    sN = tmp;
  }
}

// The front columns of stage k: k+1, k+2, k+3, and k+4 when k is odd, so that the 128-column pair J = {2J, 2J+1} leaves
// the bulk tiles after stage 2J-4 and its stages 2J-3 .. 2J-1 (2J) are FR column updates - among them the diagonal
// blocks' stage 2J-3, which the critical task FR(2J, 2J-2) would otherwise wait for at the end of a 128x128 bulk tile.
constexpr int kMaxFront = 4;
__host__ __device__ inline int front_cols(int k, int nblk, int (&cols)[kMaxFront]) {
  int n = 0;
  for (int j = k + 1; j <= k + 4 && j < nblk; ++j)
    if (j < k + 4 || (k & 1)) cols[n++] = j;
  return n;
}

// The first stage a bulk tile of column pair J no longer receives.
__host__ __device__ inline int bulk_limit(int J) { return 2 * J - 3; }

// The order in which FR(i, k) updates its front blocks (j <= i): the critical task FR(k+2, k) the diagonal block and
// then column k+1; the others column k+1 (L_{k+1,k} comes first, from the chain), the diagonal block, the rest.
__host__ __device__ inline int fr_order(int i, int k, int nblk, int (&order)[kMaxFront]) {
  int cols[kMaxFront];
  const int nc = front_cols(k, nblk, cols);
  int n = 0;
  if (i == k + 2) {
    order[n++] = k + 2;
    order[n++] = k + 1;
    return n;
  }
  for (int q = 0; q < nc; ++q)
    if (cols[q] == k + 1 && cols[q] < i) order[n++] = cols[q];
  for (int q = 0; q < nc; ++q)
    if (cols[q] == i) order[n++] = cols[q];
  for (int q = 0; q < nc; ++q)
    if (cols[q] != k + 1 && cols[q] < i) order[n++] = cols[q];
  return n;
}

// FR's stage of the forward substitution: z_k into LDS and the lane's y values of row block i (after the wait for D_k,
// which z_k travels with), then y_i -= L_ik z_k on the wave's rows into yb, before FR publishes L_ik.
__device__ __forceinline__ void fr_forward_load(const Fwd& fw, int i, int k, double (&yo)[2], double* zs) {
  if (!fw.Y) return;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int row = i * NB + 16 * w + (lane >> 2);
  if (fw.nr == 1)
    load_y<1>(fw, row, k == 0, yo);
  else
    load_y<GPX_MAX_RHS>(fw, row, k == 0, yo);
  const rsrc_t r = rsrc(fw.zbuf() + (int64_t)k * NB * fw.nr);
  for (int e = t; e < NB * fw.nr; e += WG) zs[e] = ld1(r, e * 8);
}

__device__ __forceinline__ void fr_forward_apply(const Fwd& fw, int i, const double* sL, const double* zs,
                                                 double (&yo)[2]) {
  if (!fw.Y) return;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int row = i * NB + 16 * w + (lane >> 2);
  if (fw.nr == 1)
    fwd_rows16<1>(fw, sL + 16 * w * LD, zs, yo, row, nullptr, 0);
  else
    fwd_rows16<GPX_MAX_RHS>(fw, sL + 16 * w * LD, zs, yo, row, nullptr, 0);
}

// FR(i, k): L_ik = A_ik D_k^T (published as soon as it is stored), then row i of stage k on the front columns j <= i:
// the diagonal block first when i is one of them (A_ii -= L_ik L_ik^T needs no other task), then A_ij -= L_ik L_jk^T
// with L_{k+1,k} from the chain and L_{k+2,k} / L_{k+3,k} from FR(k+2, k) / FR(k+3, k).  One task per row and stage
// (L_ik stays in LDS for every product), so the chain's next tiles (c+1, c) and (c+1, c+1) come from ONE task,
// FR(c+1, c-1): one hand-off on the cycle chain -> pool -> chain.
__device__ bool task_fr(const Args& g, double* A, double* Dinv, const Sync& s, int i, int k, double* lds, int idx,
                        const Fwd& fw, double* zs) {
  double* sA = lds;
  double* sB = lds + TILE_D;
  double* sX = lds + 2 * TILE_D;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int64_t lda = g.lda;
  auto blk = [&](int a, int b) { return A + (int64_t)a * NB * lda + (int64_t)b * NB; };
  {
    // lane 0: D_k published; lane 1: A_ik final through column k-1 (the front blocks are waited for one by one below)
    const int* mine = lane == 0 ? s.chain() : (lane == 1 ? s.ver(i, k) : nullptr);
    if (!wg_wait(s, mine, lane == 0 ? 2 * k + 2 : k, g.spin_limit)) return false;
  }
  GPX_DAG_TASK_STAMP(idx, 2);
  double yo[2];
  fr_forward_load(fw, i, k, yo, zs);
  tile_in(blk(i, k), lda, sA);
  tile_in(Dinv + (int64_t)k * NB * NB, NB, sX);
  __syncthreads();
  d4 acc[4];
  rowblock_times_lower_t(acc, sA, sX, w);
  rowblock_out(acc, w, blk(i, k), lda, sA);
  fr_forward_apply(fw, i, sA, zs, yo);
  wg_publish(t == 0 ? s.lrow(i) : nullptr, k + 1);
  GPX_DAG_TASK_STAMP(idx, 3);
  // front blocks in the order the chain needs them: column k+1 (the chain's next tile (k+2, k+1) when i = k+2), the
  // diagonal block, then the others.  Each waits for its own version (the bulk tile of a column pair entering the
  // front lands late in its stage) and, off the diagonal, for L_jk.
  int order[kMaxFront];
  const int nord = fr_order(i, k, g.nblk, order);
  for (int q = 0; q < nord; ++q) {
    const int j = order[q];
    {
      const int* mine = lane == 0 ? s.ver(i, j)
                        : (lane == 1 && j != i) ? (j == k + 1 ? s.chain() : s.lrow(j)) : nullptr;
      const int want = lane == 0 ? k : (j == k + 1 ? 2 * k + 3 : k + 1);
      if (!wg_wait(s, mine, want, g.spin_limit)) return false;
    }
    tile_in(blk(i, j), lda, sB);
    if (j == i) {
      __syncthreads();
      syrk_lower(sB, sA, w);
      __syncthreads();
      tile_out<true>(sB, blk(i, i), lda);
    } else {
      tile_in(blk(j, k), lda, sX);
      __syncthreads();
      rowblock_sub_abt(acc, sB, sA, sX, w);
      rowblock_out(acc, w, blk(i, j), lda, nullptr);
    }
    wg_publish(t == 0 ? s.ver(i, j) : nullptr, k + 1);
  }
  GPX_DAG_TASK_STAMP(idx, 4);
  return true;
}

// FR(k+2, k), the critical task (the chain's step k+2 starts from its two front blocks): the same arithmetic as task_fr,
// with every operand that does not come from the chain loaded BEFORE the chain's hand-offs, so that only D_k and
// L_{k+1,k} are on the cycle chain -> task -> chain.  A_ik (-> L_ik), A_ii and A_{i,k+1} stay in LDS; D_k and then
// L_{k+1,k} take the fourth tile.  The diagonal block first (it needs nothing from the chain beyond D_k).
__device__ bool task_fr_crit(const Args& g, double* A, double* Dinv, const Sync& s, int k, double* lds, int idx,
                             const Fwd& fw, double* zs) {
  double* sL = lds;               // A_ik -> L_ik
  double* sC = lds + TILE_D;      // A_{i,k+1}
  double* sD = lds + 2 * TILE_D;  // D_k, then L_{k+1,k}
  double* sG = lds + 3 * TILE_D;  // A_ii
  const int i = k + 2;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int64_t lda = g.lda;
  auto blk = [&](int a, int b) { return A + (int64_t)a * NB * lda + (int64_t)b * NB; };
  {
    const int* mine = lane == 0 ? s.ver(i, k) : (lane == 1 ? s.ver(i, k + 1) : (lane == 2 ? s.ver(i, i) : nullptr));
    if (!wg_wait(s, mine, k, g.spin_limit)) return false;
  }
  tile_in(blk(i, k), lda, sL);
  tile_in(blk(i, k + 1), lda, sC);
  tile_in(blk(i, i), lda, sG);
  {
    const int* mine = lane == 0 ? s.chain() : nullptr;
    if (!wg_wait(s, mine, 2 * k + 2, g.spin_limit)) return false;
  }
  GPX_DAG_TASK_STAMP(idx, 2);
  double yo[2];
  fr_forward_load(fw, i, k, yo, zs);
  tile_in(Dinv + (int64_t)k * NB * NB, NB, sD);
  __syncthreads();
  d4 acc[4];
  rowblock_times_lower_t(acc, sL, sD, w);
  rowblock_out(acc, w, blk(i, k), lda, sL);
  fr_forward_apply(fw, i, sL, zs, yo);
  wg_publish(t == 0 ? s.lrow(i) : nullptr, k + 1);
  GPX_DAG_TASK_STAMP(idx, 3);
  syrk_lower(sG, sL, w);
  __syncthreads();
  tile_out<true>(sG, blk(i, i), lda);
  wg_publish(t == 0 ? s.ver(i, i) : nullptr, k + 1);
  {
    const int* mine = lane == 0 ? s.chain() : nullptr;
    if (!wg_wait(s, mine, 2 * k + 3, g.spin_limit)) return false;
  }
  tile_in(blk(k + 1, k), lda, sD);
  __syncthreads();
  rowblock_sub_abt(acc, sC, sL, sD, w);
  rowblock_out(acc, w, blk(i, k + 1), lda, nullptr);
  wg_publish(t == 0 ? s.ver(i, k + 1) : nullptr, k + 1);
  GPX_DAG_TASK_STAMP(idx, 4);
  return true;
}

// A_ij -= sum_{k0 <= k < k1} L_ik L_jk^T on a 64x64 block (T = 64) or the 128x128 tile of blocks (2i.., 2j..) (T = 128)
template <int T>
__device__ bool task_update(const Args& g, double* A, const Sync& s, int i, int j, int k0, int k1, double* lds,
                            int idx) {
  constexpr int R = T / NB;  // 64-blocks per tile side
  const int lane = threadIdx.x & 63;
  const int64_t lda = g.lda;
  const int rb = R * i, cb = R * j;  // first 64-block row / column
  {
    // lanes 0 .. 2R-1: L rows published through stage k1-1; lanes 2R ..: the tile's blocks at version k0
    const int* mine = nullptr;
    int want = k1;
    if (lane < R) mine = s.lrow(rb + lane);
    else if (lane < 2 * R) mine = s.lrow(cb + lane - R);
    else if (lane < 2 * R + R * R) {
      const int q = lane - 2 * R, bi = rb + q / R, bj = cb + q % R;
      if (bi >= bj) mine = s.ver(bi, bj);
      want = k0;
    }
    if (!wg_wait(s, mine, want, g.spin_limit)) return false;
  }
  GPX_DAG_TASK_STAMP(idx, 2);
  const rsrc_t ra = rsrc(A + (int64_t)rb * NB * lda), rbv = rsrc(A + (int64_t)cb * NB * lda);
  const rsrc_t rc = rsrc(A + (int64_t)rb * NB * lda + (int64_t)cb * NB);
  DagTile<T> tl;
  tl.load_neg_c_sc1(rc, lda);
  tl.run_acc_sc1(ra, rbv, lda, k0 * NB, k1 * NB, lds);
  tl.store_lower(rc, lda, rb * NB, cb * NB);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < R * R) {
    const int bi = rb + threadIdx.x / R, bj = cb + threadIdx.x % R;
    if (bi >= bj) __hip_atomic_store(s.ver(bi, bj), k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

__device__ void pool_role(const Args& g, double* A, double* Dinv, const Sync& s, double* lds, const Fwd& fw,
                          double* zs) {
  __shared__ int s_ticket;
  // the critical and front workers take their own list, then join the bulk list
  int which = (int)blockIdx.x < g.wend[0] ? 0 : ((int)blockIdx.x < g.wend[1] ? 1 : 2);
  for (;;) {
    if (threadIdx.x == 0)
      s_ticket = __hip_atomic_fetch_add(s.ticket(which), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    int idx = s_ticket;
    __syncthreads();
    idx += which ? g.lend[which - 1] : 0;
    if (idx >= g.lend[which]) {
      if (which == 2) return;
      which = 2;
      continue;
    }
    const unsigned long long code = g.tasks[idx];
    const int type = (int)(code & 0xff), a = (int)((code >> 8) & 0xff), b = (int)((code >> 16) & 0xff),
              k0 = (int)((code >> 24) & 0xff), k1 = (int)((code >> 32) & 0xff);
    GPX_DAG_TASK_STAMP(idx, 0);
    bool ok;
    if (type == T_FR)
      ok = a == b + 2 ? task_fr_crit(g, A, Dinv, s, b, lds, idx, fw, zs) : task_fr(g, A, Dinv, s, a, b, lds, idx, fw, zs);
    else if (type == T_U64)
      ok = task_update<64>(g, A, s, a, b, k0, k1, lds, idx);
    else
      ok = task_update<128>(g, A, s, a, b, k0, k1, lds, idx);
    GPX_DAG_TASK_STAMP(idx, 1);
    if (!ok) return;
    __syncthreads();  // LDS reuse by the next task
  }
}

// LDS: four 64x64 tiles (the chain's A_cc, L / A_{c,c-1}, D and the next A_cc; a task's operands); > 80 KB, so one
// workgroup per CU.
constexpr int LDS_DOUBLES = 4 * TILE_D;
static_assert(LDS_DOUBLES >= DagTile<128>::LDS_DOUBLES, "U128 staging fits the task LDS");
static_assert(LDS_DOUBLES * 8 > 80 * 1024, "one workgroup per CU");

__global__ void __launch_bounds__(WG, 1) potrf_dag_kernel(Args g) {
  const int prob = blockIdx.y;
  double* A = g.A + prob * g.sa;
  double* Dinv = g.Dinv + prob * g.sd;
  double* W = g.W ? g.W + prob * g.sw : nullptr;
  int32_t* info = g.info + prob;
  const Sync s{g.sync + prob * g.ss, g.nblk};
  const Fwd& fw = g.fw;
  __shared__ __attribute__((aligned(16))) double lds[LDS_DOUBLES];
  __shared__ __attribute__((aligned(16))) double fl[3 * NB * GPX_MAX_RHS];  // forward substitution vectors
  if (blockIdx.x == 0)
    chain_role(g, A, Dinv, W, info, s, lds, fw, fl);
  else
    pool_role(g, A, Dinv, s, lds, fw, fl);
  // a timed-out wait leaves the abort word at 2: every workgroup that saw it reports the distinct failure code
  if (threadIdx.x == 0 && __hip_atomic_load(s.abort_word(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2)
    atomicCAS(info, 0, (int32_t)GPX_INFO_TIMEOUT);
}

// ---- host: the task lists -----------------------------------------------------------------------------------------
// Two lists: the FRONT (FR and the U64 column tasks, in stage order) for F dedicated front workers, so that the tasks
// the chain waits on never queue behind long bulk tiles, and the BULK (U128 tiles) for the other workers (front workers
// join it once the front list is exhausted).  The bulk order is the start order of a discrete-time simulation with
// measured task durations (microseconds on MI355X at n = 4096, tools/dag_probe): a free bulk worker takes the ready
// tile with the least slack (deadline = the chain reaching the stage at which its 128-column pair leaves the bulk,
// minus its remaining work), with every released stage up to kMaxChunk at once, and only when at least kMinChunk
// stages are released or its slack is short.  F is the simulated best of a few splits.  Any start order of the graph
// is a topological order, which is all the device relies on (tools/dag_plan_check.hip: every list drains under a
// worst-case in-order executor, for any number of workers).
struct Plan {
  std::vector<unsigned long long> list;  // critical tasks, front tasks, bulk tasks
  int lend[3] = {0, 0, 0};                // list ends
  int crit_workers = 0, front_workers = 0;
  unsigned long long* dev = nullptr;
  double sim_us = 0.0;
  std::vector<double> sim_chain;  // simulated start of each chain step (diagnostics)
  std::vector<double> sim_crit;   // critical FR(k+2, k): taken, tiles final, L_ik published, done, then the
                                  // times its three tiles became final (diagnostics)
  double sim_busy_front = 0.0, sim_busy_bulk = 0.0;  // worker-microseconds busy
};

static unsigned long long encode(int type, int a, int b, int k0, int k1) {
  return (unsigned long long)type | ((unsigned long long)a << 8) | ((unsigned long long)b << 16) |
         ((unsigned long long)k0 << 24) | ((unsigned long long)k1 << 32);
}

struct SimCost {
  double chain = 16.0;    // one chain step
  double chain_s = 3.0;   // step start -> L_{c,c-1} published
  double hop = 2.0;       // publish -> visible to a polling workgroup
  double fr_s = 5.0;      // FR: start -> L_ik published
  double fr_u = 3.0;      // FR: one front block (tile load + 64x64x64 product + store + publish)
  double crit_pre = 3.0;  // critical FR: its three tiles loaded before the chain's hand-off
  double crit_s = 3.5;    // critical FR: D_k visible -> L_ik published (D_k load, product, store)
  double crit_u = 2.5;    // critical FR: one front block from LDS operands (+ the L_{k+1,k} load for the column)
  double u64(int K) const { return 4.0 + 2.0 * K; }
  double u128(int K) const { return 6.0 + 10.0 * K; }
};

static Plan simulate(int nblk, int P, int F) {
  const SimCost cost;
  const int kMinChunk = 4, kMaxChunk = 8;
  const double dt = 0.25, INF = 1e30;
  Plan plan;
  const int CW = nblk >= 3 ? std::min(3, std::max(1, P - F - 1)) : 0;  // critical workers
  plan.crit_workers = CW;
  plan.front_workers = F;
  const int M = nblk / 2;
  std::vector<double> verT((size_t)nblk * nblk * (nblk + 1), INF), lrowT((size_t)nblk * (nblk + 1), INF),
      chainT(2 * nblk + 2, INF);
  auto VT = [&](int i, int j, int v) -> double& { return verT[((size_t)i * nblk + j) * (nblk + 1) + v]; };
  auto LT = [&](int i, int v) -> double& { return lrowT[(size_t)i * (nblk + 1) + v]; };
  for (int i = 0; i < nblk; ++i) {
    LT(i, 0) = 0.0;
    for (int j = 0; j <= i; ++j) VT(i, j, 0) = 0.0;
  }
  chainT[0] = 0.0;
  // the critical list: FR(k+2, k), the only front task the chain's next step waits on; the front list: the others
  struct FTask { int type, i, j, k; };
  std::vector<FTask> crit, front;
  for (int k = 0; k + 2 < nblk; ++k) {
    crit.push_back({T_FR, k + 2, k, k});
    for (int i = k + 3; i < nblk; ++i) front.push_back({T_FR, i, k, k});
  }
  for (const FTask& f : crit) plan.list.push_back(encode(T_FR, f.i, f.k, 0, 0));
  plan.lend[0] = (int)plan.list.size();
  for (const FTask& f : front) plan.list.push_back(encode(T_FR, f.i, f.k, 0, 0));
  plan.lend[1] = (int)plan.list.size();
  std::vector<FTask> lists[2] = {crit, front};
  size_t lnext[2] = {0, 0};
  plan.sim_crit.assign(7 * crit.size(), -1.0);
  // bulk units: the 128x128 tiles (I, J), I > J, and the three 64-blocks of each diagonal tile (J, J) - the diagonal
  // blocks' last bulk stages gate the critical task two steps later, and a U64 lands in a fraction of a U128's time
  struct BTile { int T, a, b, J, v; bool busy; };
  std::vector<BTile> tiles;
  for (int J = 2; J < M; ++J) {
    tiles.push_back({64, 2 * J, 2 * J, J, 0, false});
    tiles.push_back({64, 2 * J + 1, 2 * J, J, 0, false});
    tiles.push_back({64, 2 * J + 1, 2 * J + 1, J, 0, false});
    for (int I = J + 1; I < M; ++I) tiles.push_back({128, I, J, J, 0, false});
  }
  size_t bulk_left = tiles.size();
  int cstep = 0;
  double cfree = 0.0;
  // cls: 0 critical, 1 front, 2 bulk; held: the FR task the worker holds (index into lists[cls], -1: none); phase 0:
  // waiting to start, 1 + q: front block q of its order next; tcur: when the task's previous phase ends
  struct Worker { double free; int held; int cls; int phase; double tcur, pre; };
  std::vector<Worker> wk(P);
  for (int p = 0; p < P; ++p) wk[p] = {0.0, -1, p < CW ? 0 : (p < CW + F ? 1 : 2), 0, 0.0, -1.0};
  struct Ev { double t; int kind, a, b, v; };  // kind 0 chain word, 1 lrow, 2 version, 3 tile free
  std::vector<Ev> evs;
  auto front_ready = [&](const FTask& f, double now) {
    return chainT[2 * f.k + 2] <= now && VT(f.i, f.k, f.k) <= now;
  };
  double now = 0.0;
  for (long guard = 0; guard < 8000000; ++guard, now += dt) {
    for (size_t e = 0; e < evs.size();) {
      const Ev x = evs[e];
      if (x.t > now) {
        ++e;
        continue;
      }
      if (x.kind == 0) chainT[x.v] = std::min(chainT[x.v], x.t);
      else if (x.kind == 1) LT(x.a, x.v) = std::min(LT(x.a, x.v), x.t);
      else if (x.kind == 2) VT(x.a, x.b, x.v) = std::min(VT(x.a, x.b, x.v), x.t);
      else tiles[x.a].busy = false;
      evs[e] = evs.back();
      evs.pop_back();
    }
    if (cstep < nblk && cfree <= now &&
        (cstep == 0 || (VT(cstep, cstep - 1, cstep - 1) <= now && VT(cstep, cstep, cstep - 1) <= now))) {
      if (cstep) evs.push_back({now + cost.chain_s + cost.hop, 0, 0, 0, 2 * cstep + 1});
      cfree = now + cost.chain;
      evs.push_back({cfree + cost.hop, 0, 0, 0, 2 * cstep + 2});
      plan.sim_chain.push_back(now);
      ++cstep;
    }
    {
      int busy_b = 0, busy_f = 0;
      for (const Worker& w : wk)
        if (w.free > now) (w.cls < 2 ? busy_f : busy_b)++;
      plan.sim_busy_front += busy_f * dt;
      plan.sim_busy_bulk += busy_b * dt;
    }
    bool front_busy = false;
    std::vector<int> idle;
    for (int p = 0; p < P; ++p) {
      Worker& w = wk[p];
      if (w.free > now) {
        front_busy = front_busy || w.cls < 2;
        continue;
      }
      if (w.cls < 2 && w.held < 0) {
        if (lnext[w.cls] < lists[w.cls].size()) {
          w.held = (int)lnext[w.cls]++;
          w.phase = 0;
          w.pre = -1.0;
          if (w.cls == 0) plan.sim_crit[7 * w.held] = now;
        } else {
          w.cls = 2;  // joins the bulk
        }
      }
      if (w.held >= 0) {
        front_busy = true;
        const FTask& f = lists[w.cls][w.held];
        const bool crit = f.i == f.k + 2;
        if (w.phase == 0) {
          if (crit) {
            // its three tiles first (from the moment they are final), then D_k
            if (w.pre < 0.0) {
              if (VT(f.i, f.k, f.k) > now || VT(f.i, f.k + 1, f.k) > now || VT(f.i, f.i, f.k) > now) continue;
              w.pre = now + cost.crit_pre;
              plan.sim_crit[7 * w.held + 1] = now;
              plan.sim_crit[7 * w.held + 4] = VT(f.i, f.k, f.k);
              plan.sim_crit[7 * w.held + 5] = VT(f.i, f.k + 1, f.k);
              plan.sim_crit[7 * w.held + 6] = VT(f.i, f.i, f.k);
            }
            if (chainT[2 * f.k + 2] > now) continue;
            w.tcur = std::max(w.pre, chainT[2 * f.k + 2]) + cost.crit_s;
            plan.sim_crit[7 * w.held + 2] = w.tcur;
          } else {
            if (!front_ready(f, now)) continue;
            w.tcur = now + cost.fr_s;
          }
          evs.push_back({w.tcur + cost.hop, 1, f.i, 0, f.k + 1});
          w.phase = 1;
        }
        // the front blocks in fr_order, each once its version (and L block) is known; the task holds the worker
        // meanwhile, as on the device
        int order[kMaxFront];
        const int nord = fr_order(f.i, f.k, nblk, order);
        while (w.phase - 1 < nord) {
          const int j = order[w.phase - 1];
          double ready = crit ? 0.0 : VT(f.i, j, f.k);
          if (j != f.i) ready = std::max(ready, j == f.k + 1 ? chainT[2 * f.k + 3] : LT(j, f.k + 1));
          if (ready > now) break;  // not visible yet (or not even scheduled)
          w.tcur = std::max(w.tcur, ready) + (crit ? cost.crit_u : cost.fr_u);
          evs.push_back({w.tcur + cost.hop, 2, f.i, j, f.k + 1});
          ++w.phase;
        }
        if (w.phase - 1 < nord) continue;
        if (crit && w.cls == 0) plan.sim_crit[7 * w.held + 3] = w.tcur;
        w.free = w.tcur;
        w.held = -1;
        continue;
      }
      idle.push_back(p);
    }
    if (cstep >= nblk && lnext[0] >= crit.size() && lnext[1] >= front.size() && !front_busy && bulk_left == 0) break;
    if (idle.empty() || bulk_left == 0) continue;
    struct Cand { double slack; int q, K; };
    std::vector<Cand> cands;
    for (size_t q = 0; q < tiles.size(); ++q) {
      const BTile& b = tiles[q];
      const int limit = bulk_limit(b.J);
      if (b.busy || b.v >= limit) continue;
      int rel = limit;
      int rows[4] = {b.a, b.b, b.a, b.b};
      if (b.T == 128) rows[0] = 2 * b.a, rows[1] = 2 * b.a + 1, rows[2] = 2 * b.b, rows[3] = 2 * b.b + 1;
      for (int r : rows) {
        int v = b.v;
        while (v < rel && LT(r, v + 1) <= now) ++v;
        rel = std::min(rel, v);
      }
      const int avail = rel - b.v;
      if (avail <= 0) continue;
      const double deadline = cfree + (double)(limit - cstep) * cost.chain;
      const int remaining = limit - b.v;
      const int kc = std::min(remaining, kMaxChunk);
      const double rem_t = std::ceil((double)remaining / kMaxChunk) * (b.T == 128 ? cost.u128(kc) : cost.u64(kc));
      const double slack = deadline - now - rem_t;
      if (avail < kMinChunk && rel < limit && slack > 2 * cost.chain) continue;
      cands.push_back({slack, (int)q, std::min(avail, kMaxChunk)});
    }
    std::sort(cands.begin(), cands.end(), [](const Cand& x, const Cand& y) {
      return x.slack < y.slack || (x.slack == y.slack && x.q < y.q);
    });
    size_t ni = 0;
    for (const Cand& cd : cands) {
      if (ni >= idle.size()) break;
      Worker& w = wk[idle[ni++]];
      BTile& b = tiles[cd.q];
      plan.list.push_back(encode(b.T == 128 ? T_U128 : T_U64, b.a, b.b, b.v, b.v + cd.K));
      const double end = now + (b.T == 128 ? cost.u128(cd.K) : cost.u64(cd.K));
      b.v += cd.K;
      if (b.T == 128) {
        for (int bi : {2 * b.a, 2 * b.a + 1})
          for (int bj : {2 * b.b, 2 * b.b + 1}) evs.push_back({end + cost.hop, 2, bi, bj, b.v});
      } else {
        evs.push_back({end + cost.hop, 2, b.a, b.b, b.v});
      }
      b.busy = true;
      evs.push_back({end, 3, cd.q, 0, 0});
      if (b.v >= bulk_limit(b.J)) --bulk_left;
      w.free = end;
    }
  }
  plan.lend[2] = (int)plan.list.size();
  plan.sim_us = std::max(now, cfree);
  return plan;
}

static Plan build_plan(int nblk, int P) {
  Plan best;
  best.sim_us = 1e30;
  for (int div : {8, 6, 4, 3}) {
    const int F = std::max(1, std::min(nblk, P / div));
    if (F + 3 > P) continue;
    Plan p = simulate(nblk, P, F);
    if (p.sim_us < best.sim_us) best = std::move(p);
  }
  return best;
}

// one plan per (nblk, workers) per handle
struct Cache {
  std::map<std::pair<int, int>, std::unique_ptr<Plan>> plans;
};

}  // namespace dag

size_t potrf_dag_sync_bytes(int npad, int batch) { return (size_t)dag::sync_words(npad / NB) * 4 * batch; }

void potrf_dag_release(Context* c) {
  auto* cache = reinterpret_cast<dag::Cache*>(c->dag_cache);
  if (cache) {
    for (auto& kv : cache->plans)
      if (kv.second->dev) (void)hipFree(kv.second->dev);
    delete cache;
  }
  c->dag_cache = nullptr;
  if (c->dag_sync) (void)hipFree(c->dag_sync);
  c->dag_sync = nullptr;
  c->dag_sync_bytes = 0;
}

// Workgroups per problem: one per CU, split evenly over the batch; 0 = the DAG schedule does not apply.
int potrf_dag_workers(Context* c, int npad, int batch) {
  const int nblk = npad / NB;
  if (nblk < 2 || nblk > 64) return 0;
  if (c->cu_count <= 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    c->cu_count = cus;
  }
  const int per = c->cu_count / batch;
  return per >= 8 ? per : 0;
}

hipError_t launch_potrf_dag(Context* c, int npad, double* A, int64_t lda, double* Dinv, int32_t* info,
                            const Batch& bt, double* W, int64_t ldw, const ForwardRhs* fr) {
  const int nblk = npad / NB;
  const int G = potrf_dag_workers(c, npad, bt.count);
  if (!G) return hipErrorInvalidValue;
  auto* cache = reinterpret_cast<dag::Cache*>(c->dag_cache);
  if (!cache) {
    cache = new dag::Cache();
    c->dag_cache = cache;
  }
  auto key = std::make_pair(nblk, G - 1);
  auto it = cache->plans.find(key);
  if (it == cache->plans.end()) {
    std::unique_ptr<dag::Plan> p(new dag::Plan(dag::build_plan(nblk, G - 1)));
    const size_t bytes = p->list.size() * sizeof(unsigned long long);
    if (bytes) {
      hipError_t e = hipMalloc(&p->dev, bytes);
      if (e != hipSuccess) return e;
      e = hipMemcpy(p->dev, p->list.data(), bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) return e;
    }
    it = cache->plans.emplace(key, std::move(p)).first;
  }
  const dag::Plan& plan = *it->second;
  const size_t sbytes = potrf_dag_sync_bytes(npad, bt.count);
  if (c->dag_sync_bytes < sbytes) {
    if (c->dag_sync) (void)hipFree(c->dag_sync);
    c->dag_sync = nullptr;
    c->dag_sync_bytes = 0;
    hipError_t e = hipMalloc(&c->dag_sync, sbytes);
    if (e != hipSuccess) return e;
    c->dag_sync_bytes = sbytes;
  }
  hipError_t e = hipMemsetAsync(c->dag_sync, 0, sbytes, c->stream);
  if (e != hipSuccess) return e;
  dag::Args g;
  g.A = A;
  g.lda = lda;
  g.nblk = nblk;
  g.Dinv = Dinv;
  g.info = info;
  g.W = W;
  g.ldw = ldw;
  g.sync = reinterpret_cast<int*>(c->dag_sync);
  g.sa = bt.k;
  g.sd = bt.dinv;
  g.sw = bt.w;
  g.ss = dag::sync_words(nblk);
  g.tasks = plan.dev;
  for (int q = 0; q < 3; ++q) g.lend[q] = plan.lend[q];
  g.wend[0] = 1 + plan.crit_workers;
  g.wend[1] = 1 + plan.crit_workers + plan.front_workers;
  g.spin_limit = c->spin_limit;
  g.fw = dag::Fwd{nullptr, 0, 0, 0, 0, 0, 1, 0.0, nullptr, nullptr};
  if (fr && fr->Y) {
    const int nr = rhs_row(fr->nrhs);
    g.fw = dag::Fwd{fr->Y, fr->ldy, fr->sy, 2 * (int64_t)npad * nr, fr->nrhs, fr->n, nr, fr->mean, fr->buf,
                    fr->buf + (int64_t)npad * nr};
  }
  dag::potrf_dag_kernel<<<dim3(G, bt.count), WG, 0, c->stream>>>(g);
  return hipGetLastError();
}

}  // namespace gpx
