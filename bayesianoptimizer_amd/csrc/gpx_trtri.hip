// Triangular inverse W = L^{-T} (upper, row-major) and alpha = K^{-1}(y - m) = W W^T (y - m).
// alpha is GPyTorch's mean_cache [upstream]; W turns every later solve L^{-1} k* of
// the posterior/acquisition sweep into an independent triangular product (gpx_sweep.hip).
//
// TRTRI by recursive doubling over the 64x64 diagonal inverses D_k produced by potrf:
//   level 0: W_kk = D_k^T, and the 64x64 block below the diagonal inside every 128-tile is zeroed;
//   level l: for groups of 2h blocks (h = 2^(l-1)), with first half (off1, b1) and second half (off2, b2):
//       T   = L21^T W22          (b1 x b2; W22 upper: k <= c)
//       W12 = -W11 T             (b1 x b2; W11 upper: k >= r)
//   two MFMA launches per level, all groups of a level batched in blockIdx.z: 1 + 2*ceil(log2(nblk))
//   launches in total.  Works for any even number of 64-blocks (the last group may be partial).
#include "gpx_internal.h"
#include "gpx_device.h"
#include "gpx_trmm_asm.h"

namespace gpx {

__global__ void __launch_bounds__(WG) trtri_diag_kernel(const double* __restrict__ Dinv, double* __restrict__ W,
                                                        int64_t ldw, int64_t sd, int64_t sw) {
  Dinv += blockIdx.y * sd;  // problem of a batched fit
  W += blockIdx.y * sw;
  const int b = blockIdx.x;
  const double* D = Dinv + (int64_t)b * NB * NB;
  double* Wbb = W + (int64_t)b * NB * ldw + (int64_t)b * NB;
  for (int e = threadIdx.x; e < NB * NB; e += WG) {
    const int r = e / NB, c = e % NB;
    Wbb[(int64_t)r * ldw + c] = D[c * NB + r];  // transpose: W_bb = D_b^T
  }
  if (b & 1) {  // zero the strictly-lower 64x64 block of this 128-tile
    double* Z = W + (int64_t)b * NB * ldw + (int64_t)(b - 1) * NB;
    for (int e = threadIdx.x; e < NB * NB; e += WG) Z[(int64_t)(e / NB) * ldw + (e % NB)] = 0.0;
  }
}

// Block order of the 128-tile levels (large n): one output tile per workgroup, heaviest k-range first (no long tile
// left running alone at the end of a level), XCD-aware when the free index spans a multiple of 8 tiles: the
// round-robin dispatch puts workgroups b, b+8, ... on one XCD, so XCD x takes the free tiles f = x (mod 8) and walks the
// heavy index down, its resident workgroups sharing 8 free-operand panels through one L2 (the sweep product's order,
// gpx_sweep.hip).  n = 16384, last level: T 9.24 -> 8.08 ms, W12 9.55 -> 8.68 ms against the paired order
// (tools/trtri_bench.hip, profiles/r04_trtri_order_bench.log; same tiles, bit-identical); the whole inverse
// 25.7 -> 23.6 ms.  The 64-tile levels keep the paired order (PAIRED: a workgroup takes the k-ranges of tile pair
// (x, nt - 1 - x), so every workgroup does the same work; the XCD order measured 0.72 vs 0.66 ms at n = 4096).
// nH / nF: tile counts of a full group; tiles past a partial last group exit.  The groups of a level share one grid
// dimension with the heavy index outermost (round 5): every group's heaviest tiles start first, instead of group
// g + 1's heaviest tiles waiting behind group g's light ones (n = 16384, levels h = 32 / 64: 4 / 2 groups).
__device__ __forceinline__ void trtri_order(int b, int nH, int nF, int groups, bool heavy_high, int& H, int& F,
                                            int& g) {
  int q;
  if ((nF & 7) == 0) {
    const int l = b >> 3, per = nF >> 3;
    q = l / (per * groups);
    const int rem = l % (per * groups);
    g = rem / per;
    F = 8 * (rem % per) + (b & 7);
  } else {
    q = b / (nF * groups);
    const int rem = b % (nF * groups);
    g = rem / nF;
    F = rem % nF;
  }
  H = heavy_high ? nH - 1 - q : q;
}

// T_p = L21^T W22 for group p of level with half-size h blocks (TS x TS output tiles; TS = 64, or 128 for the big
// levels of large n).  blockIdx.z = group + groups * problem.  The k-range of tile (rb, cb) is (cb + 1) * TS (W22
// upper; its 128-aligned diagonal tiles have the strictly-lower 64-block zeroed by trtri_diag).  PAIRED: grid
// (pairs, rows), column pair cb, nt2 - 1 - cb; else grid nt1^2, trtri_order with heavy index cb.
template <int TS, bool PAIRED>
__global__ void __launch_bounds__(WG) trtri_t_kernel(const double* __restrict__ L, int64_t ldl,
                                                     const double* __restrict__ W, int64_t ldw,
                                                     double* __restrict__ T, int h, int nblk, int groups, int64_t sl,
                                                     int64_t sw, int64_t st) {
  using Tile = MfmaTile<TS, TS, 16, true, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  // PAIRED: group and problem in blockIdx.z; else the group is decoded from blockIdx.x (trtri_order), problem = z
  int p = PAIRED ? (int)(blockIdx.z % groups) : 0, ocb = 0, orb = 0;
  const int prob = PAIRED ? (int)(blockIdx.z / groups) : (int)blockIdx.z;
  if constexpr (!PAIRED) {
    const int h1 = h * NB / TS;
    trtri_order(blockIdx.x, h1, h1, groups, true, ocb, orb, p);
  }
  L += prob * sl;
  W += prob * sw;
  T += prob * st;
  const int s1 = p * 2 * h, s2 = s1 + h;
  const int nb2 = min(2 * h, nblk - s1) - h;
  if (nb2 <= 0) return;
  const int b1 = h * NB, b2 = nb2 * NB;
  const int nt2 = b2 / TS;
  const int64_t off1 = (int64_t)s1 * NB, off2 = (int64_t)s2 * NB;
  // T_p is b1 x b2 with row length b2; every group before the last is full (b2 = b1), so group p starts at
  // p*b1*b1 and the level's total sum_p b1*b2_p <= b1*(npad-b1) <= npad^2/4 fits the workspace.
  double* Tp = T + (int64_t)p * b1 * b1;
  auto tile_at = [&](int rb, int cb) {
    const double* Ab = L + off2 * ldl + off1 + rb * TS;  // A(m=r,k=q) = L[off2+q][off1+r]
    const double* Bb = W + off2 * ldw + off2 + cb * TS;  // B(k=q,n=c) = W[off2+q][off2+c]
    d4 acc[Tile::WM][Tile::WN];
    if constexpr (TS == 128) {
      // the hand-placed k loop (gpx_trmm_asm.h, same bits as MfmaTile::run); B = W22's diagonal 128-tile is zero in its
      // last 64 k-rows for the left 64 columns, so those waves skip the last 4 k-tiles' MFMAs
      trmm_asm::TileT<true, true> tile;
      tile.zero();
      const bool skip = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 1) == 0;
      tile.template run<false, true>(Ab, ldl, Bb, ldw, (cb + 1) * (TS / 16), smem, false, skip);
#pragma unroll
      for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
        for (int j = 0; j < Tile::WN; ++j) acc[i][j] = tile.acc[i][j];
    } else {
      Tile tile;
      tile.run(Ab, ldl, Bb, ldw, 0, (cb + 1) * TS, smem);
#pragma unroll
      for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
        for (int j = 0; j < Tile::WN; ++j) acc[i][j] = tile.acc[i][j];
    }
#pragma unroll
    for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
      for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Tp[(int64_t)(rb * TS + Tile::row_of(i, r)) * b2 + cb * TS + Tile::col_of(j)] = acc[i][j][r];
  };
  if constexpr (PAIRED) {
    const int rb = blockIdx.y, x = blockIdx.x;
    if (x >= (nt2 + 1) / 2) return;
    tile_at(rb, x);
    if (nt2 - 1 - x != x) {  // (run() ends with a barrier after its last LDS read)
      tile_at(rb, nt2 - 1 - x);
    }
  } else {
    if (ocb < nt2) tile_at(orb, ocb);
  }
}

// W12 = -W11 T_p.  The k-range of tile (rb, cb) is [rb * TS, b1) (W11 upper).  PAIRED: grid (cols, pairs), row pair
// rb, nt1 - 1 - rb; else grid nt1^2, trtri_order with heavy index rb (lightest last).
template <int TS, bool PAIRED>
__global__ void __launch_bounds__(WG) trtri_w_kernel(double* __restrict__ W, int64_t ldw, const double* __restrict__ T,
                                                     int h, int nblk, int groups, int64_t sw, int64_t st) {
  using Tile = MfmaTile<TS, TS, 16, false, true>;
  __shared__ __attribute__((aligned(16))) double smem[Tile::LDS_DOUBLES];
  int p = PAIRED ? (int)(blockIdx.z % groups) : 0, orb = 0, ocb = 0;
  const int prob = PAIRED ? (int)(blockIdx.z / groups) : (int)blockIdx.z;
  if constexpr (!PAIRED) {
    const int h1 = h * NB / TS;
    trtri_order(blockIdx.x, h1, h1, groups, false, orb, ocb, p);
  }
  W += prob * sw;
  T += prob * st;
  const int s1 = p * 2 * h, s2 = s1 + h;
  const int nb2 = min(2 * h, nblk - s1) - h;
  if (nb2 <= 0) return;
  const int b1 = h * NB, b2 = nb2 * NB;
  const int nt1 = b1 / TS, nt2 = b2 / TS;
  const int64_t off1 = (int64_t)s1 * NB, off2 = (int64_t)s2 * NB;
  auto tile_at = [&](int rb, int cb) {
    const double* Bb = T + (int64_t)p * b1 * b1 + cb * TS;  // B(k=q,n=c) = T[q][c], row length b2
    const double* Ab = W + (off1 + rb * TS) * ldw + off1;   // A(m=r,k=q) = W[off1+r][off1+q]
    d4 acc[Tile::WM][Tile::WN];
    if constexpr (TS == 128) {
      // the hand-placed k loop from k = rb * TS (A row-major: W11 read along its rows); A = W11's diagonal 128-tile is
      // zero in its first 64 k-columns for the lower 64 rows, so those waves skip the first 4 k-tiles' MFMAs
      trmm_asm::TileT<false, true> tile;
      tile.zero();
      const bool skip = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7) == 1;
      tile.template run<true, false>(Ab + rb * TS, ldw, Bb + (int64_t)rb * TS * b2, b2, (b1 - rb * TS) / 16, smem, skip,
                                     false);
#pragma unroll
      for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
        for (int j = 0; j < Tile::WN; ++j) acc[i][j] = tile.acc[i][j];
    } else {
      Tile tile;
      tile.run(Ab, ldw, Bb, b2, rb * TS, b1, smem);
#pragma unroll
      for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
        for (int j = 0; j < Tile::WN; ++j) acc[i][j] = tile.acc[i][j];
    }
    double* Wo = W + (off1 + rb * TS) * ldw + off2 + cb * TS;
#pragma unroll
    for (int i = 0; i < Tile::WM; ++i)
#pragma unroll
      for (int j = 0; j < Tile::WN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) Wo[(int64_t)Tile::row_of(i, r) * ldw + Tile::col_of(j)] = -acc[i][j][r];
  };
  if constexpr (PAIRED) {
    const int cb = blockIdx.x, y = blockIdx.y;
    if (cb >= nt2 || y >= (nt1 + 1) / 2) return;
    tile_at(y, cb);
    if (nt1 - 1 - y != y) {  // (run() ends with a barrier after its last LDS read)
      tile_at(nt1 - 1 - y, cb);
    }
  } else {
    if (ocb < nt2) tile_at(orb, ocb);
  }
}

hipError_t launch_trtri(Context* c, int npad, const double* L, int64_t ldl, const double* Dinv, double* W,
                        int64_t ldw, double* T, const Batch& bt, bool diag_done) {
  LaunchTimer tm(c, GPX_TIMER_TRTRI);
  const int nblk = npad / NB;
  if (!diag_done) trtri_diag_kernel<<<dim3(nblk, bt.count), WG, 0, c->stream>>>(Dinv, W, ldw, bt.dinv, bt.w);
  for (int h = 1; h < nblk; h *= 2) {
    const int groups = (nblk + 2 * h - 1) / (2 * h);
    // 128x128 tiles (half the operand traffic per flop) once a level still fills the chip with them: >= ~1024 tiles
    // per problem (n = 16384: levels h >= 32; n = 8192: the last level; n <= 4096: never).  Decided per
    // problem size, not batch count, so a batched fit stays bit-identical to single fits.
    const int h128 = h / 2;
    if (h >= 2 && (int64_t)groups * h128 * ((h128 + 1) / 2) >= 512) {
      const dim3 grid(h128 * h128 * groups, 1, bt.count);
      trtri_t_kernel<128, false><<<grid, WG, 0, c->stream>>>(L, ldl, W, ldw, T, h, nblk, groups, bt.k, bt.w, bt.ws);
      trtri_w_kernel<128, false><<<grid, WG, 0, c->stream>>>(W, ldw, T, h, nblk, groups, bt.w, bt.ws);
      continue;
    }
    const int hp = (h + 1) / 2;  // paired tiles
    trtri_t_kernel<NB, true><<<dim3(hp, h, groups * bt.count), WG, 0, c->stream>>>(L, ldl, W, ldw, T, h, nblk, groups,
                                                                                   bt.k, bt.w, bt.ws);
    trtri_w_kernel<NB, true><<<dim3(h, hp, groups * bt.count), WG, 0, c->stream>>>(W, ldw, T, h, nblk, groups, bt.w,
                                                                                   bt.ws);
  }
  return hipGetLastError();
}

// ---- alpha -----------------------------------------------------------------------------------------
constexpr int AK = 128;  // k-chunk of the z = W^T y pass

// zpart[kc][i][r] = sum_{k in chunk kc, k <= i} W[k][i] * ytil[k][r]
__global__ void __launch_bounds__(WG) alpha_z_kernel(int n, int npad, const double* __restrict__ W, int64_t ldw,
                                                     const double* __restrict__ Y, int64_t ldy, int nrhs,
                                                     double const_mean, double* __restrict__ zpart, int64_t sw,
                                                     int64_t sy, int64_t sws, const double* __restrict__ means) {
  if (means) const_mean = means[blockIdx.z];  // per-problem kernel parameters (Batch::means)
  W += blockIdx.z * sw;  // problem of a batched fit
  Y += blockIdx.z * sy;
  zpart += blockIdx.z * sws;
  __shared__ double ys[AK + 16][GPX_MAX_RHS];  // zero rows past the chunk: the last 16-group reads up to AK + 15
  const int i = blockIdx.x * WG + threadIdx.x;
  const int kc = blockIdx.y;
  const int k0 = kc * AK;
  if (k0 > blockIdx.x * WG + WG - 1) return;  // whole chunk below every column of this block: unused
  for (int e = threadIdx.x; e < (AK + 16) * GPX_MAX_RHS; e += WG) {
    const int kk = e / GPX_MAX_RHS, r = e % GPX_MAX_RHS;
    const int k = k0 + kk;
    ys[kk][r] = (kk < AK && r < nrhs && k < n) ? (Y[(int64_t)k * ldy + r] - const_mean) : 0.0;
  }
  __syncthreads();
  double acc[GPX_MAX_RHS];
#pragma unroll
  for (int r = 0; r < GPX_MAX_RHS; ++r) acc[r] = 0.0;
  if (i < npad) {
    const int kend = min(k0 + AK, i + 1);
    // Branch-free groups of 16: clamped (always in-bounds) W loads, masked to 0 past the column's last row, so the
    // loads issue together and no per-element branch splits the loop (the per-element `if` form spent 17-23 us in
    // branches and waits at n = 128).  Accumulation order per output is k ascending, as before; the masked tail
    // adds +0.0.
    for (int k = k0; k < kend; k += 16) {
      double wv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int kq = min(k + q, kend - 1);
        const double v = W[(int64_t)kq * ldw + i];
        wv[q] = (k + q < kend) ? v : 0.0;
      }
      if (nrhs == 1) {
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[0] += wv[q] * ys[k + q - k0][0];
      } else {
#pragma unroll
        for (int r = 0; r < GPX_MAX_RHS; ++r)
          if (r < nrhs) {
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[r] += wv[q] * ys[k + q - k0][r];
          }
      }
    }
    for (int r = 0; r < nrhs; ++r) zpart[((int64_t)kc * npad + i) * nrhs + r] = acc[r];
  }
}

// z[i][r] = sum over valid chunks
__global__ void __launch_bounds__(WG) alpha_zsum_kernel(int npad, int nrhs, const double* __restrict__ zpart,
                                                        double* __restrict__ z, int64_t sws) {
  zpart += blockIdx.y * sws;
  z += blockIdx.y * sws;
  const int e = blockIdx.x * WG + threadIdx.x;
  if (e >= npad * nrhs) return;
  const int i = e / nrhs;
  double s = 0.0;
  for (int kc = 0; kc * AK <= i; ++kc) s += zpart[(int64_t)kc * npad * nrhs + e];
  z[e] = s;
}

// alpha[k][r] = sum_{i >= k} W[k][i] z[i][r]; one wave per row k.
__global__ void __launch_bounds__(WG) alpha_w_kernel(int n, int npad, const double* __restrict__ W, int64_t ldw,
                                                     const double* __restrict__ z, int nrhs, double* __restrict__ alpha,
                                                     int64_t sw, int64_t sws, int64_t sa, int zfold = 0) {
  W += blockIdx.y * sw;
  z += blockIdx.y * sws;
  alpha += blockIdx.y * sa;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= npad) return;
  double acc[GPX_MAX_RHS];
#pragma unroll
  for (int r = 0; r < GPX_MAX_RHS; ++r) acc[r] = 0.0;
  for (int i = k + lane; i < npad; i += 64) {
    const double w = W[(int64_t)k * ldw + i];
#pragma unroll
    for (int r = 0; r < GPX_MAX_RHS; ++r) {
      if (r < nrhs) {
        double zi;
        if (zfold) {  // z = the zpart chunk sums, in alpha_zsum_kernel's order (small npad: one dispatch fewer)
          zi = 0.0;
          for (int kc = 0; kc * AK <= i; ++kc) zi += z[(int64_t)kc * npad * nrhs + (int64_t)i * nrhs + r];
        } else {
          zi = z[(int64_t)i * nrhs + r];
        }
        acc[r] += w * zi;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < GPX_MAX_RHS; ++r) {
    if (r < nrhs) {
      double v = acc[r];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) alpha[(int64_t)k * nrhs + r] = (k < n) ? v : 0.0;
    }
  }
}

hipError_t launch_alpha(Context* c, int n, int npad, const double* W, int64_t ldw, const double* Y, int64_t ldy,
                        int nrhs, double const_mean, double* alpha, double* zpart, double* z, const Batch& bt) {
  LaunchTimer tm(c, GPX_TIMER_ALPHA);
  dim3 g1((npad + WG - 1) / WG, npad / AK, bt.count);
  alpha_z_kernel<<<g1, WG, 0, c->stream>>>(n, npad, W, ldw, Y, ldy, nrhs, const_mean, zpart, bt.w, bt.y, bt.ws,
                                              bt.means);
  if (npad <= 4 * AK) {  // <= 4 chunks: alpha_w sums them itself (z entries re-read per row, from L2)
    alpha_w_kernel<<<dim3((npad + 3) / 4, bt.count), WG, 0, c->stream>>>(n, npad, W, ldw, zpart, nrhs, alpha, bt.w,
                                                                          bt.ws, bt.alpha, 1);
    return hipGetLastError();
  }
  alpha_zsum_kernel<<<dim3((npad * nrhs + WG - 1) / WG, bt.count), WG, 0, c->stream>>>(npad, nrhs, zpart, z, bt.ws);
  alpha_w_kernel<<<dim3((npad + 3) / 4, bt.count), WG, 0, c->stream>>>(n, npad, W, ldw, z, nrhs, alpha, bt.w, bt.ws,
                                                                        bt.alpha);
  return hipGetLastError();
}

// out = W z for an upper-triangular W and one right-hand side of npad entries (the SVGP's alpha' = L^{-T} m),
// batched over problems with strides bt.w (W), bt.y (z), bt.alpha (out).
hipError_t launch_trmv_upper(Context* c, int npad, const double* W, int64_t ldw, const double* z, double* out,
                             const Batch& bt) {
  alpha_w_kernel<<<dim3((npad + 3) / 4, bt.count), WG, 0, c->stream>>>(npad, npad, W, ldw, z, 1, out, bt.w, bt.y,
                                                                        bt.alpha);
  return hipGetLastError();
}

}  // namespace gpx
