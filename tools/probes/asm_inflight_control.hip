// Positive control for bayesianoptimizer_amd/csrc/check_asm_inflight.py (tests/test_build_checks.py; never run).
// The hand-placed k loop of gpx_trmm_asm.h with a RUNTIME choice between two continuations after its prologue: the
// prologue's fragment reads are still in flight at the branch, and hipcc copies their registers (v_mov before the
// s_waitcnt) to reconcile the two paths' allocations.  That is the round-6 TRTRI bug the build check exists for; the
// checker must report this kernel.
#include "gpx_trmm_asm.h"
using namespace gpx;
using namespace gpx::trmm_asm;
__global__ void __launch_bounds__(256) asm_inflight_control(const double* Ag, long lda, const double* Bg, long ldb,
                                                            int nk, double* out) {
  __shared__ __attribute__((aligned(16))) double smem[LDS_BYTES / 8];
  TileT<false, true> t;
  t.zero();
  const int w = threadIdx.x >> 6;
  const unsigned lds0 = (unsigned)(uintptr_t)smem;
  t.A.init(lds0, 0, (w >> 1) * 64, lda);
  t.B.init(lds0, SB_OFF, (w & 1) * 64, ldb);
  auto dA = [&](int kt) { return t.A.at(Ag, lda, kt); };
  auto dB = [&](int kt) { return t.B.at(Bg, ldb, kt); };
#pragma unroll
  for (int q = 0; q < TileT<false, true>::NL; ++q) t.gload(dA(0), dB(0), q);
  wait_vm<0>(t.A, t.B);
#pragma unroll
  for (int q = 0; q < TileT<false, true>::NW; ++q) t.lwrite<0>(q);
#pragma unroll
  for (int q = 0; q < TileT<false, true>::NL; ++q) t.gload(dA(1), dB(1), q);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int q = 0; q < 8; ++q) t.read_frag<0, 0>(t.f0, q);
  if (nk > 8) {
    t.ktile<0, true, true>(dA(2), dB(2), 1);
    t.ktile<1, true, true>(dA(3), dB(3), 2);
    for (int k = 2; k < nk - 2; k += 2) {
      t.ktile<0, true, true>(dA(k + 2), dB(k + 2));
      t.ktile<1, true, true>(dA(k + 3), dB(k + 3));
    }
    t.ktile<0, true, false>(dA(0), dB(0));
    t.ktile<1, false, false>(dA(0), dB(0));
  } else {
    t.ktile<0, true, false>(dA(0), dB(0), 3);
    t.ktile<1, false, false>(dA(0), dB(0), 4);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __syncthreads();
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 4; ++r) out[threadIdx.x * 64 + i * 16 + j * 4 + r] = t.acc[i][j][r];
}
