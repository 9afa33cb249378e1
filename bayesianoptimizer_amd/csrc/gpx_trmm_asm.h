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

__device__ __forceinline__ void mfma_a(d4& c, double a, double b) {
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

// LDS geometry (bytes): buffer b at b * BUF, A (k-major, pitch 144 doubles) at +0, B at +SB_OFF
constexpr int PITCH = 144 * 8;
constexpr int SB_OFF = 16 * PITCH;
constexpr int BUF = 2 * SB_OFF;
constexpr int LDS_BYTES = 2 * BUF;  // 73728: two workgroups per CU

struct Frag {
  double a[4], b[4];
};

// the q-th of the 8 fragment reads of substep S (k-rows 4S..4S+3) of buffer BB: a[i] = A[kr][wm0 + 16 i + m],
// b[j] = B[kr][wn0 + 16 j + m]
template <int BB, int S>
__device__ __forceinline__ void read_frag(Frag& f, unsigned ra, unsigned rb, int q) {
  constexpr int base = BB * BUF + 4 * S * PITCH;
  switch (q) {
    case 0: dsr<base + 0 * 128>(f.a[0], ra); break;
    case 1: dsr<base + 0 * 128>(f.b[0], rb); break;
    case 2: dsr<base + 1 * 128>(f.a[1], ra); break;
    case 3: dsr<base + 1 * 128>(f.b[1], rb); break;
    case 4: dsr<base + 2 * 128>(f.a[2], ra); break;
    case 5: dsr<base + 2 * 128>(f.b[2], rb); break;
    case 6: dsr<base + 3 * 128>(f.a[3], ra); break;
    default: dsr<base + 3 * 128>(f.b[3], rb); break;
  }
}

template <int N>
__device__ __forceinline__ void wait_lgkm(Frag& f) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.a[2]), "+v"(f.a[3]), "+v"(f.b[0]), "+v"(f.b[1]), "+v"(f.b[2]),
                 "+v"(f.b[3])
               : "i"(N));
}
__device__ __forceinline__ void wait_vm0(v2d (&r)[8]) {
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]));
}

struct Tile {
  d4 acc[4][4];  // acc[i][j][r]: row (w >> 1) * 64 + 16 i + (lane >> 4) + 4 r, column (w & 1) * 64 + 16 j + (lane & 15)
  Frag f0, f1;
  v2d r[8];          // staged k-tile: r[0..3] A k-rows t/64 + 4q, r[4..7] B k-rows
  unsigned vga, vgb;  // global byte offsets of this thread's first A / B element of a k-tile
  unsigned ra, rb;    // LDS fragment read bases (buffer 0)
  unsigned wa, wb;    // LDS write bases (buffer 0)

  __device__ __forceinline__ void mm(const Frag& f, int e) { mfma_a(acc[e >> 2][e & 3], f.a[e >> 2], f.b[e & 3]); }

  __device__ __forceinline__ void gload(rsrc_t A, rsrc_t B, unsigned sa, unsigned sb, int q) {
    if (q < 4)
      bld(r[q], vga, A, sa * (unsigned)q);
    else
      bld(r[q], vgb, B, sb * (unsigned)(q - 4));
  }
  template <int BB>
  __device__ __forceinline__ void lwrite(int q) {
    constexpr int o = BB * BUF;
    switch (q) {
      case 0: dsw<o + 0 * 4 * PITCH>(wa, r[0]); break;
      case 1: dsw<o + 1 * 4 * PITCH>(wa, r[1]); break;
      case 2: dsw<o + 2 * 4 * PITCH>(wa, r[2]); break;
      case 3: dsw<o + 3 * 4 * PITCH>(wa, r[3]); break;
      case 4: dsw<o + 0 * 4 * PITCH>(wb, r[4]); break;
      case 5: dsw<o + 1 * 4 * PITCH>(wb, r[5]); break;
      case 6: dsw<o + 2 * 4 * PITCH>(wb, r[6]); break;
      default: dsw<o + 3 * 4 * PITCH>(wb, r[7]); break;
    }
  }

  // One k-tile from LDS buffer CUR.  NEXT: a following k-tile exists (staged in r[]: written to the other buffer during
  // S0, its substep-0 fragments read during S3); NEXT2: the tile after it exists (loaded into r[] during S1; rA / rB
  // are descriptors based at its first k-row).  MM = false (wave-uniform): the same memory traffic without the MFMAs (a
  // wave whose A rows are all zero in this k-tile: W's strictly lower 64-block of a diagonal 128-tile).
  template <int CUR, bool NEXT, bool NEXT2>
  __device__ __forceinline__ void ktile(rsrc_t rA, rsrc_t rB, unsigned sa, unsigned sb, bool MM = true) {
    constexpr int NXT = CUR ^ 1;
    wait_lgkm<0>(f0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (MM) mm(f0, e);
      if (e < 8) read_frag<CUR, 1>(f1, ra, rb, e);
      if (NEXT) {
        if (e == 7) wait_vm0(r);
        if (e >= 8) lwrite<NXT>(e - 8);
      }
    }
    if (NEXT)
      wait_lgkm<8>(f1);  // the 8 reads of S1 are older than the 8 writes
    else
      wait_lgkm<0>(f1);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (MM) mm(f1, e);
      if (e < 8) read_frag<CUR, 2>(f0, ra, rb, e);
      if (NEXT2 && e >= 8) gload(rA, rB, sa, sb, e - 8);
    }
    wait_lgkm<0>(f0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (MM) mm(f0, e);
      if (e < 8) read_frag<CUR, 3>(f1, ra, rb, e);
    }
    wait_lgkm<0>(f1);
    if (NEXT) asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (MM) mm(f1, e);
      if (NEXT && e < 8) read_frag<NXT, 0>(f0, ra, rb, e);
    }
  }

  // acc = A B over nk k-tiles of 16 (nk even, >= 8 when zero_tail, else >= 2), A(m, k) = Ag[k * lda + m],
  // B(k, n) = Bg[k * ldb + n] (both k-major, 16-byte aligned rows).  zero_tail: A's rows 0..63 are zero in the last 4
  // k-tiles (the triangular W's diagonal 128-tile), so waves 0-1 skip those MFMAs (acc + 0 = acc: the same bits for
  // finite operands).  smem: LDS_BYTES, 16-byte aligned.  Byte offsets inside one operand must fit 32 bits per k-tile
  // row group (the descriptors are rebased every k-tile).
  __device__ void run(const double* __restrict__ Ag, int64_t lda, const double* __restrict__ Bg, int64_t ldb, int nk,
                      double* smem, bool zero_tail) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int kr = lane >> 4, m = lane & 15;
    const int wm0 = (w >> 1) * 64, wn0 = (w & 1) * 64;
    const unsigned lds0 = (unsigned)(uintptr_t)smem;  // the low 32 bits of a shared pointer are its LDS address
    ra = lds0 + (unsigned)((kr * 144 + wm0 + m) * 8);
    rb = lds0 + SB_OFF + (unsigned)((kr * 144 + wn0 + m) * 8);
    wa = lds0 + (unsigned)(((t >> 6) * 144 + 2 * (t & 63)) * 8);
    wb = wa + SB_OFF;
    vga = (unsigned)(((int64_t)(t >> 6) * lda + 2 * (t & 63)) * 8);
    vgb = (unsigned)(((int64_t)(t >> 6) * ldb + 2 * (t & 63)) * 8);
    const unsigned sa = (unsigned)(4 * lda * 8), sb = (unsigned)(4 * ldb * 8);
    const bool skip = zero_tail && __builtin_amdgcn_readfirstlane(w >> 1) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
    // prologue: k-tile 0 -> LDS buffer 0, k-tile 1 -> r[], substep-0 fragments of tile 0
#pragma unroll
    for (int q = 0; q < 8; ++q) gload(rsrc_of(Ag), rsrc_of(Bg), sa, sb, q);
    wait_vm0(r);
#pragma unroll
    for (int q = 0; q < 8; ++q) lwrite<0>(q);
#pragma unroll
    for (int q = 0; q < 8; ++q) gload(rsrc_of(Ag + 16 * lda), rsrc_of(Bg + 16 * ldb), sa, sb, q);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int q = 0; q < 8; ++q) read_frag<0, 0>(f0, ra, rb, q);
    auto dA = [&](int kt) { return rsrc_of(Ag + (int64_t)kt * 16 * lda); };
    auto dB = [&](int kt) { return rsrc_of(Bg + (int64_t)kt * 16 * ldb); };
    const int kmain = zero_tail ? nk - 4 : nk - 2;  // tiles [0, kmain) in the pair loop, each with a tile after next
    for (int k = 0; k < kmain; k += 2) {
      ktile<0, true, true>(dA(k + 2), dB(k + 2), sa, sb);
      ktile<1, true, true>(dA(k + 3), dB(k + 3), sa, sb);
    }
    if (zero_tail) {
      ktile<0, true, true>(dA(nk - 2), dB(nk - 2), sa, sb, !skip);
      ktile<1, true, true>(dA(nk - 1), dB(nk - 1), sa, sb, !skip);
    }
    ktile<0, true, false>(dA(0), dB(0), sa, sb, !skip);
    ktile<1, false, false>(dA(0), dB(0), sa, sb, !skip);
    // the last MFMAs' results are read by VALU code next: 24 wait states (cdna_hip_programming.md §5.7 item 2)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
};

}  // namespace trmm_asm
}  // namespace gpx
