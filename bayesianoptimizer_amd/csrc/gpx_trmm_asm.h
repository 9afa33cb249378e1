// The sweep product's 128 x 128 fp64 MFMA tile with a HAND-PLACED k loop (round 5).
//
// Same tile as MfmaTile<128, 128, 16, true, true>: 256 threads, 4 waves in 2 x 2 of 64 x 64 (4 x 4 v_mfma_f64_16x16x4
// blocks each), BK = 16, k-major LDS tiles padded to 144 doubles, two LDS buffers, global -> register -> LDS staging.
// Every accumulator sees the same MFMA sequence as MfmaTile (k ascending in steps of 4, lane (kr, m) supplying
// A[m][k0 + kr] and B[k0 + kr][n]), so results are bit-identical to it (tools/trmm_asm_bench.hip checks that).  What
// differs is the instruction stream: one asm statement per instruction, in this order per k-tile (per wave, 64 MFMAs):
//   S0  16 MFMAs on the substep-0 fragments (read during the previous tile's S3), after MFMA e: the e-th fragment read of
//       S1 (e < 8); vmcnt(0) after MFMA 7, then the 8 ds_write_b128 of the NEXT k-tile (staged in registers) into the
//       other LDS buffer
//   S1  16 MFMAs; the 8 fragment reads of S2, the 8 buffer_load_dwordx4 of the k-tile AFTER next into the registers
//   S2  16 MFMAs; the 8 fragment reads of S3;  lgkmcnt(0) + s_barrier: the next tile is in LDS for every wave, and every
//       wave is done reading this tile's buffer
//   S3  16 MFMAs; the 8 fragment reads of the next tile's S0
// so per k-tile the only exposed latency is the barrier's skew.  hipcc's schedule of the same loop (MfmaTile::run) waits
// after its last MFMA for the LDS writes, the barrier and the next tile's first fragment reads; probe
// (tools/trmm_asm_bench.hip, n = 4096, 32768 candidates, profiles/r05_trmm_asm_bench.log): 7.83 vs 8.29 ms = 0.893 vs
// 0.844 of the 78.6 TF/s fp64 peak.
//
// Register discipline (cdna_hip_programming.md §5.7): fragment and staging registers are "=v" outputs of their load
// statements and are named "+v" by the wait statement that completes them, so hipcc never reads, moves or reuses them
// in between; every memory operation of the loop is in asm (hipcc counts none of them, and emits no wait of its own in
// the loop).  WAR distances: a fragment register is overwritten by a read issued at least one MFMA after the last MFMA
// reading it (operands are read at issue; LDS data returns >= 64 cycles later); the staging registers are reloaded one
// substep after their ds_writes.  After the loop 24 wait states separate the last MFMA from VALU reads of acc.
#pragma once
#include "gpx_internal.h"

namespace gpx {
namespace trmm_asm {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef double v2d __attribute__((ext_vector_type(2)));  // HIP's double2 is a struct: not an asm register operand

__device__ __forceinline__ rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// c += a b, or with NEG c -= a b (the A operand's neg modifier: round(c - ab) = -round(-c + ab), so a tile seeded with +C
// computes exactly what one seeded with -C and stored negated does)
template <bool NEG = false>
__device__ __forceinline__ void mfma_a(d4& c, double a, double b) {
  if constexpr (NEG)
    asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0 neg:[1,0,0]" : "+v"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
template <int OFF>
__device__ __forceinline__ void dsr(double& d, unsigned addr) {
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
template <int OFF>
__device__ __forceinline__ void dsw(unsigned addr, const v2d& v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF));
}
__device__ __forceinline__ void bld(v2d& d, unsigned voff, rsrc_t r, unsigned soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff));
}
template <int OFF>
__device__ __forceinline__ void bld8(double& d, unsigned voff, rsrc_t r, unsigned soff) {
  asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen offset:%4" : "=v"(d) : "v"(voff), "s"(r), "s"(soff), "i"(OFF));
}
template <int OFF>
__device__ __forceinline__ void dsw8(unsigned addr, double v) {
  asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(addr), "v"(v), "i"(OFF));
}

// LDS geometry (bytes): buffer b at b * BUF, A (k-major, pitch 144 doubles) at +0, B at +SB_OFF
constexpr int PITCH = 144 * 8;
constexpr int SB_OFF = 16 * PITCH;
constexpr int BUF = 2 * SB_OFF;
constexpr int LDS_BYTES = 2 * BUF;  // 73728: two workgroups per CU

struct Frag {
  double a[4], b[4];
};

template <int N>
__device__ __forceinline__ void wait_lgkm(Frag& f) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.a[2]), "+v"(f.a[3]), "+v"(f.b[0]), "+v"(f.b[1]), "+v"(f.b[2]),
                 "+v"(f.b[3])
               : "i"(N));
}

// One operand tile (128 x 16 per k-tile) of the product: its global -> register staging, its LDS image (k-major, the
// layout MfmaTile builds: a k-major operand copied row for row, a row-major one transposed with the XOR swizzle
// m ^ (k & 14) of MfmaTile::swz) and its fragment reads.
//   KM (k-major, X(m, k) = G[k * ld + m]): 4 buffer_load_dwordx4 (k-row t/64 + 4q, elements 2 (t % 64) .. + 1), 4
//       ds_write_b128; fragment reads from one base address.
//   !KM (row-major, X(m, k) = G[m * ld + k]): 8 buffer_load_dwordx2 (row t/8 + 32q, elements k = 2 (t % 8) and + 1:
//       MfmaTile's 16-byte load split in halves, because an asm operand cannot name half of a register quad), 8
//       ds_write_b64 into k-rows kk, kk + 1 at column m ^ kk; fragment reads from one base address per k-substep (the
//       swizzle makes the lane's column depend on the substep through (4 S) & 12).
template <bool KM>
struct Operand {
  v2d rk[4];     // KM staging
  double rr[8];  // !KM staging: rr[2q], rr[2q + 1] = elements (t/8 + 32q, kk), (.., kk + 1)
  unsigned voff, soff_q;  // global byte offset of this thread's first element; the q-th load adds q * soff_q
  unsigned wbase;         // LDS write base (buffer 0)
  unsigned rbase[4];      // LDS fragment read base (buffer 0) per k-substep (KM: all equal)
  static constexpr int NLOAD = KM ? 4 : 8;
  static constexpr int NWRITE = KM ? 4 : 8;

  // region: byte offset of this operand's tile inside a buffer; w0: the wave's first row (wm0 or wn0)
  __device__ __forceinline__ void init(unsigned lds0, int region, int w0, int64_t ld) {
    const int t = threadIdx.x, lane = t & 63, kr = lane >> 4, m = lane & 15;
    if constexpr (KM) {
      voff = (unsigned)(((int64_t)(t >> 6) * ld + 2 * (t & 63)) * 8);
      soff_q = (unsigned)(4 * ld * 8);
      wbase = lds0 + region + (unsigned)(((t >> 6) * 144 + 2 * (t & 63)) * 8);
#pragma unroll
      for (int s = 0; s < 4; ++s) rbase[s] = lds0 + region + (unsigned)((kr * 144 + w0 + m) * 8);
    } else {
      const int kk = 2 * (t & 7);
      voff = (unsigned)(((int64_t)(t >> 3) * ld + kk) * 8);
      soff_q = (unsigned)(32 * ld * 8);
      wbase = lds0 + region + (unsigned)((kk * 144 + ((t >> 3) ^ kk)) * 8);
#pragma unroll
      for (int s = 0; s < 4; ++s)
        rbase[s] = lds0 + region + (unsigned)((kr * 144 + w0 + (m ^ (kr & 2) ^ ((4 * s) & 12))) * 8);
    }
  }
  // the q-th global load of a k-tile whose descriptor is r
  __device__ __forceinline__ void load(rsrc_t r, int q) {
    if constexpr (KM)
      bld(rk[q], voff, r, soff_q * (unsigned)q);
    else if (q & 1)
      bld8<8>(rr[q], voff, r, soff_q * (unsigned)(q >> 1));
    else
      bld8<0>(rr[q], voff, r, soff_q * (unsigned)(q >> 1));
  }
  // the q-th LDS write of the staged k-tile into buffer BB
  template <int BB>
  __device__ __forceinline__ void write(int q) {
    if constexpr (KM) {
      switch (q) {
        case 0: dsw<BB * BUF + 0 * 4 * PITCH>(wbase, rk[0]); break;
        case 1: dsw<BB * BUF + 1 * 4 * PITCH>(wbase, rk[1]); break;
        case 2: dsw<BB * BUF + 2 * 4 * PITCH>(wbase, rk[2]); break;
        default: dsw<BB * BUF + 3 * 4 * PITCH>(wbase, rk[3]); break;
      }
    } else {
      switch (q) {  // element (row t/8 + 32 (q/2), k = kk + (q & 1)): LDS k-row kk + (q & 1), column (t/8 ^ kk) + 32 (q/2)
        case 0: dsw8<BB * BUF + 0 * 256>(wbase, rr[0]); break;
        case 1: dsw8<BB * BUF + PITCH + 0 * 256>(wbase, rr[1]); break;
        case 2: dsw8<BB * BUF + 1 * 256>(wbase, rr[2]); break;
        case 3: dsw8<BB * BUF + PITCH + 1 * 256>(wbase, rr[3]); break;
        case 4: dsw8<BB * BUF + 2 * 256>(wbase, rr[4]); break;
        case 5: dsw8<BB * BUF + PITCH + 2 * 256>(wbase, rr[5]); break;
        case 6: dsw8<BB * BUF + 3 * 256>(wbase, rr[6]); break;
        default: dsw8<BB * BUF + PITCH + 3 * 256>(wbase, rr[7]); break;
      }
    }
  }
  // fragment i of substep S from buffer BB: X[4 S + kr][w0 + 16 i + m] (swizzled for !KM)
  template <int BB, int S>
  __device__ __forceinline__ void frag(double& d, int i) {
    constexpr int base = BB * BUF + 4 * S * PITCH;
    switch (i) {
      case 0: dsr<base + 0 * 128>(d, rbase[S]); break;
      case 1: dsr<base + 1 * 128>(d, rbase[S]); break;
      case 2: dsr<base + 2 * 128>(d, rbase[S]); break;
      default: dsr<base + 3 * 128>(d, rbase[S]); break;
    }
  }
  // descriptor based at k-tile kt
  __device__ __forceinline__ rsrc_t at(const double* G, int64_t ld, int kt) const {
    return rsrc_of(KM ? G + (int64_t)kt * 16 * ld : G + (int64_t)kt * 16);
  }
};

// s_waitcnt vmcnt(N) completing the staged k-tile (N: younger loads that may stay in flight, e.g. accumulator seeds)
template <int N, bool AKM, bool BKM>
__device__ __forceinline__ void wait_vm(Operand<AKM>& A, Operand<BKM>& B) {
  if constexpr (AKM && BKM)
    asm volatile("s_waitcnt vmcnt(%8)"
                 : "+v"(A.rk[0]), "+v"(A.rk[1]), "+v"(A.rk[2]), "+v"(A.rk[3]), "+v"(B.rk[0]), "+v"(B.rk[1]),
                   "+v"(B.rk[2]), "+v"(B.rk[3])
                 : "i"(N));
  else if constexpr (!AKM && BKM)
    asm volatile("s_waitcnt vmcnt(%12)"
                 : "+v"(A.rr[0]), "+v"(A.rr[1]), "+v"(A.rr[2]), "+v"(A.rr[3]), "+v"(A.rr[4]), "+v"(A.rr[5]),
                   "+v"(A.rr[6]), "+v"(A.rr[7]), "+v"(B.rk[0]), "+v"(B.rk[1]), "+v"(B.rk[2]), "+v"(B.rk[3])
                 : "i"(N));
  else if constexpr (AKM && !BKM)
    asm volatile("s_waitcnt vmcnt(%12)"
                 : "+v"(A.rk[0]), "+v"(A.rk[1]), "+v"(A.rk[2]), "+v"(A.rk[3]), "+v"(B.rr[0]), "+v"(B.rr[1]),
                   "+v"(B.rr[2]), "+v"(B.rr[3]), "+v"(B.rr[4]), "+v"(B.rr[5]), "+v"(B.rr[6]), "+v"(B.rr[7])
                 : "i"(N));
  else
    asm volatile("s_waitcnt vmcnt(%16)"
                 : "+v"(A.rr[0]), "+v"(A.rr[1]), "+v"(A.rr[2]), "+v"(A.rr[3]), "+v"(A.rr[4]), "+v"(A.rr[5]),
                   "+v"(A.rr[6]), "+v"(A.rr[7]), "+v"(B.rr[0]), "+v"(B.rr[1]), "+v"(B.rr[2]), "+v"(B.rr[3]),
                   "+v"(B.rr[4]), "+v"(B.rr[5]), "+v"(B.rr[6]), "+v"(B.rr[7])
                 : "i"(N));
}
template <bool AKM, bool BKM>
__device__ __forceinline__ void wait_vm0(Operand<AKM>& A, Operand<BKM>& B) {
  wait_vm<0>(A, B);
}

// The 128 x 128 tile.  AKM / BKM: A(m, k) / B(k, n) k-major (A(m, k) = Ag[k lda + m], B(k, n) = Bg[k ldb + n]) or
// row-major (A(m, k) = Ag[m lda + k], B(k, n) = Bg[n ldb + k]).
template <bool AKM, bool BKM, bool NEG = false>
struct TileT {
  d4 acc[4][4];  // acc[i][j][r]: row (w >> 1) * 64 + 16 i + (lane >> 4) + 4 r, column (w & 1) * 64 + 16 j + (lane & 15)
  Frag f0, f1;
  Operand<AKM> A;
  Operand<BKM> B;
  static constexpr int NL = Operand<AKM>::NLOAD + Operand<BKM>::NLOAD;    // global loads per k-tile (8 / 12 / 16)
  static constexpr int NW = Operand<AKM>::NWRITE + Operand<BKM>::NWRITE;  // LDS writes per k-tile

  __device__ __forceinline__ void mm(const Frag& f, int e) {
    mfma_a<NEG>(acc[e >> 2][e & 3], f.a[e >> 2], f.b[e & 3]);
  }

  __device__ __forceinline__ void gload(rsrc_t rA, rsrc_t rB, int q) {
    if (q < Operand<AKM>::NLOAD)
      A.load(rA, q);
    else
      B.load(rB, q - Operand<AKM>::NLOAD);
  }
  template <int BB>
  __device__ __forceinline__ void lwrite(int q) {
    if (q < Operand<AKM>::NWRITE)
      A.template write<BB>(q);
    else
      B.template write<BB>(q - Operand<AKM>::NWRITE);
  }
  // the 8 fragment reads of substep S: a[0], b[0], a[1], b[1], ...
  template <int BB, int S>
  __device__ __forceinline__ void read_frag(Frag& f, int q) {
    if (q & 1)
      B.template frag<BB, S>(f.b[q >> 1], q >> 1);
    else
      A.template frag<BB, S>(f.a[q >> 1], q >> 1);
  }

  // One k-tile from LDS buffer CUR (see the file comment).  NEXT: a following k-tile exists (staged in the operands'
  // registers: written to the other buffer during S0, its substep-0 fragments read during S3); NEXT2: the tile after it
  // exists (its global loads issued during S1 from descriptors rA / rB).  skip (wave-uniform, 0-4): the wave's first
  // `skip` 16-row blocks have all-zero operand rows in this k-tile (a triangular operand's diagonal), so their MFMAs are
  // left out (4: the same memory traffic without any MFMA).
  template <int CUR, bool NEXT, bool NEXT2>
  __device__ __forceinline__ void ktile(rsrc_t rA, rsrc_t rB, int skip = 0) {
    constexpr int NXT = CUR ^ 1;
    wait_lgkm<0>(f0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if ((e >> 2) >= skip) mm(f0, e);
      if (e < 8) read_frag<CUR, 1>(f1, e);
      if (NEXT) {
        if (e == 7) wait_vm0(A, B);
        if (e >= 8)
#pragma unroll
          for (int q = (e - 8) * NW / 8; q < (e - 7) * NW / 8; ++q) lwrite<NXT>(q);
      }
    }
    if (NEXT)
      wait_lgkm<(NW < 15 ? NW : 15)>(f1);  // the 8 reads of S1 are older than the NW writes (lgkmcnt is 4 bits)
    else
      wait_lgkm<0>(f1);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if ((e >> 2) >= skip) mm(f1, e);
      if (e < 8) read_frag<CUR, 2>(f0, e);
      if (NEXT2)
#pragma unroll
        for (int q = e * NL / 16; q < (e + 1) * NL / 16; ++q) gload(rA, rB, q);
    }
    wait_lgkm<0>(f0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if ((e >> 2) >= skip) mm(f0, e);
      if (e < 8) read_frag<CUR, 3>(f1, e);
    }
    wait_lgkm<0>(f1);
    if (NEXT) asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if ((e >> 2) >= skip) mm(f1, e);
      if (NEXT && e < 8) read_frag<NXT, 0>(f0, e);
    }
  }

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  }

  // acc += A B over nk k-tiles of 16 (nk even, >= 2; >= 8 with skip_tail, >= 4 + 2 with skip_head), on acc as it is
  // (zero() first for a plain product).  Rows must be 16-byte aligned (k-major) / 8-byte (row-major), and byte offsets
  // inside one k-tile of an operand must fit 31 bits (the descriptors are rebased every k-tile).
  // skip_head / skip_tail (wave-uniform): this wave's operand fragments are all zero in the first / last 4 k-tiles
  // (a triangular operand's diagonal 128-tile), so it skips those MFMAs (acc + 0 = acc: the same bits for finite
  // operands).  HEAD / TAIL: compile the peeled k-tiles that honour them.  smem: LDS_BYTES, 16-byte aligned.
  template <bool HEAD = false, bool TAIL = false>
  __device__ void run(const double* __restrict__ Ag, int64_t lda, const double* __restrict__ Bg, int64_t ldb, int nk,
                      double* smem, bool skip_head = false, bool skip_tail = false) {
    run_after<HEAD, TAIL, 0>(Ag, lda, Bg, ldb, nk, smem, [] {}, skip_head, skip_tail);
  }

  // run() with after_first() called right after the first k-tile's global loads: NSEED loads it issues (hipcc-counted
  // builtins seeding acc) stay in flight through the prologue; hipcc waits for them before the first MFMA that reads
  // the accumulator they fill (in-order vmcnt: the younger asm loads only make its waits more conservative).
  template <bool HEAD, bool TAIL, int NSEED, typename F>
  __device__ void run_after(const double* __restrict__ Ag, int64_t lda, const double* __restrict__ Bg, int64_t ldb,
                            int nk, double* smem, F&& after_first, bool skip_head = false, bool skip_tail = false) {
    const int w = threadIdx.x >> 6;
    const unsigned lds0 = (unsigned)(uintptr_t)smem;  // the low 32 bits of a shared pointer are its LDS address
    A.init(lds0, 0, (w >> 1) * 64, lda);
    B.init(lds0, SB_OFF, (w & 1) * 64, ldb);
    // prologue: k-tile 0 -> LDS buffer 0, k-tile 1 -> registers, substep-0 fragments of tile 0
#pragma unroll
    for (int q = 0; q < NL; ++q) gload(A.at(Ag, lda, 0), B.at(Bg, ldb, 0), q);
    after_first();
    wait_vm<(NSEED < 63 ? NSEED : 63)>(A, B);  // (vmcnt is 6 bits)
#pragma unroll
    for (int q = 0; q < NW; ++q) lwrite<0>(q);
#pragma unroll
    for (int q = 0; q < NL; ++q) gload(A.at(Ag, lda, 1), B.at(Bg, ldb, 1), q);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int q = 0; q < 8; ++q) read_frag<0, 0>(f0, q);
    auto dA = [&](int kt) { return A.at(Ag, lda, kt); };
    auto dB = [&](int kt) { return B.at(Bg, ldb, kt); };
    int k = 0;
    if (HEAD) {  // tiles 0-3 (their tiles after next exist: nk >= 6)
      ktile<0, true, true>(dA(2), dB(2), skip_head ? 4 : 0);
      ktile<1, true, true>(dA(3), dB(3), skip_head ? 4 : 0);
      ktile<0, true, true>(dA(4), dB(4), skip_head ? 4 : 0);
      ktile<1, true, true>(dA(5), dB(5), skip_head ? 4 : 0);
      k = 4;
    }
    const int kmain = TAIL ? nk - 4 : nk - 2;  // tiles [k, kmain) in the pair loop, each with a tile after next
    for (; k < kmain; k += 2) {
      ktile<0, true, true>(dA(k + 2), dB(k + 2));
      ktile<1, true, true>(dA(k + 3), dB(k + 3));
    }
    if (TAIL) {
      ktile<0, true, true>(dA(nk - 2), dB(nk - 2), skip_tail ? 4 : 0);
      ktile<1, true, true>(dA(nk - 1), dB(nk - 1), skip_tail ? 4 : 0);
    }
    ktile<0, true, false>(dA(0), dB(0), (TAIL && skip_tail) ? 4 : 0);
    ktile<1, false, false>(dA(0), dB(0), (TAIL && skip_tail) ? 4 : 0);
    // the last MFMAs' results are read by VALU code next: 24 wait states (cdna_hip_programming.md §5.7 item 2)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // run() for an upper-triangular A block row (A(m, k) = 0 for k > m + 128 (nk / 8 - 1)), nk a multiple of 8: the last
  // 8 k-tiles are the diagonal 128-block, local k-tile j = 0..7, in which the waves of rows 0-63 skip their row blocks
  // i < j (all of them for j >= 4) and the waves of rows 64-127 their row blocks i < j - 4.
  __device__ void run_tri(const double* __restrict__ Ag, int64_t lda, const double* __restrict__ Bg, int64_t ldb, int nk,
                          double* smem) {
    const int w = threadIdx.x >> 6;
    const int lo = __builtin_amdgcn_readfirstlane(w >> 1) == 0 ? 0 : 4;  // 4: rows 64-127
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    A.init(lds0, 0, (w >> 1) * 64, lda);
    B.init(lds0, SB_OFF, (w & 1) * 64, ldb);
#pragma unroll
    for (int q = 0; q < NL; ++q) gload(A.at(Ag, lda, 0), B.at(Bg, ldb, 0), q);
    wait_vm<0>(A, B);
#pragma unroll
    for (int q = 0; q < NW; ++q) lwrite<0>(q);
#pragma unroll
    for (int q = 0; q < NL; ++q) gload(A.at(Ag, lda, 1), B.at(Bg, ldb, 1), q);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int q = 0; q < 8; ++q) read_frag<0, 0>(f0, q);
    auto dA = [&](int kt) { return A.at(Ag, lda, kt); };
    auto dB = [&](int kt) { return B.at(Bg, ldb, kt); };
    // the wave's zero row blocks in local k-tile j: min(max(j - lo, 0), 4)
    auto sk = [&](int j) { const int v = j - lo; return v < 0 ? 0 : (v > 4 ? 4 : v); };
    const int kd = nk - 8;  // first k-tile of the diagonal block
    for (int k = 0; k < kd; k += 2) {
      ktile<0, true, true>(dA(k + 2), dB(k + 2));
      ktile<1, true, true>(dA(k + 3), dB(k + 3));
    }
    ktile<0, true, true>(dA(kd + 2), dB(kd + 2), sk(0));
    ktile<1, true, true>(dA(kd + 3), dB(kd + 3), sk(1));
    ktile<0, true, true>(dA(kd + 4), dB(kd + 4), sk(2));
    ktile<1, true, true>(dA(kd + 5), dB(kd + 5), sk(3));
    ktile<0, true, true>(dA(kd + 6), dB(kd + 6), sk(4));
    ktile<1, true, true>(dA(kd + 7), dB(kd + 7), sk(5));
    ktile<0, true, false>(dA(0), dB(0), sk(6));
    ktile<1, false, false>(dA(0), dB(0), sk(7));
    // the last MFMAs' results are read by VALU code next: 24 wait states (cdna_hip_programming.md §5.7 item 2)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
};

// The sweep product's tile: both operands k-major; for the triangular W (zero_tail: nk a multiple of 8) the zero 16 x 16
// blocks of the diagonal 128-block are skipped (run_tri: the waves of rows 0-63 / 64-127 form 10 / 26 of their 32 row-block
// x k-tile products there, against 16 / 32 when only the zero 64-block was skipped).
struct Tile : TileT<true, true> {
  __device__ void run(const double* __restrict__ Ag, int64_t lda, const double* __restrict__ Bg, int64_t ldb, int nk,
                      double* smem, bool zero_tail) {
    zero();
    if (zero_tail)
      TileT<true, true>::run_tri(Ag, lda, Bg, ldb, nk, smem);
    else
      TileT<true, true>::run<false, false>(Ag, lda, Bg, ldb, nk, smem);
  }
};

}  // namespace trmm_asm
}  // namespace gpx
