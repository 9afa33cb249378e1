// Internal declarations shared by the gpx HIP translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <string>
#include <vector>
#include "../../include/gpx.h"

namespace gpx {

constexpr int NB = 64;              // Cholesky / TRTRI block (64x64 diagonal blocks)
constexpr int TILE = GPX_TILE;      // padding granule and sweep tile (128)
constexpr int WG = 256;             // threads per workgroup (4 waves of 64)

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- context -----------------------------------------------------------------------------------
struct PendingTimer {
  int timer;
  hipEvent_t start, stop;
};

struct Context {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string last_error;
  int32_t timing_mask = 0;
  double timer_ms[GPX_TIMER_COUNT] = {0};
  int64_t timer_launches[GPX_TIMER_COUNT] = {0};
  std::vector<PendingTimer> pending;
  std::vector<hipEvent_t> free_events;
  int cu_count = 0;  // CUs of the device (queried once: persistent solve grid, Cholesky slot budget)
  // bounded spins of the in-launch hand-offs (potrs): passes before a waiter gives up and reports a timeout
  unsigned spin_limit = 1u << 22;
  // options (include/gpx.h GPX_OPT_*; set by gpx_set_option or GPX_OPTIONS at gpx_create)
  int sweep_fused = 1;     // fused small-n sweep where it applies
  int gram_split = 0;      // 0 by size, else workgroups per Gram tile
  int potrf_lazy = 0;      // multi-launch flush interval, 0 by size
  int potrf_mode = -1;     // multi-launch panel mode, -1 by size
  int potrf_switch = -1;   // launch at which a single fit switches schedule (gpx_potrf.hip potrf_switch), -1 by size
  int potrf_split = -1;    // panel split policy (gpx_potrf.hip step_plan): -1 fits the slots, 1 never, 3 one per CU
};

// Scoped device switch of one C ABI call: makes the handle's device current and restores the caller's current device
// on exit, so a call on an engine of device k never moves the caller's (e.g. torch's) current device.
struct DeviceScope {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceScope(int device) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != device) {
      err = hipSetDevice(device);
      if (err != hipSuccess) prev = -1;
    } else {
      prev = -1;  // nothing to restore
    }
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

// Scoped timer: records a start event on construction and a stop event on destruction when the
// timer's bit is set in the context's mask.
struct LaunchTimer {
  Context* c;
  int timer;
  hipEvent_t s = nullptr, e = nullptr;
  LaunchTimer(Context* ctx, int t);
  ~LaunchTimer();
};

// ---- batched fits -------------------------------------------------------------------------------
// `count` independent problems of the same n / d / kernel parameters (restarts or seeds, BASELINE configs[3]) run in
// the same launches: the problem index is one more grid dimension and every array of problem b starts at
// base + b * stride (element strides; a workspace slice of `ws` doubles per problem).  count = 1: a single fit.
// Read-only inputs (x, y) may use any stride >= 0 (0: every problem reads the same X, e.g. the T outputs of one
// multi-output model; y = 1 with ldy = T: output column b of one n x T target matrix).  means (device, optional): per-problem
// constant means written by the fit's Gram launches when the problems carry their own kernel parameters
// (gpx_fit_*_batched_params_f64); the triangular solves then read means[b] instead of their scalar const_mean.
struct Batch {
  int count = 1;
  int64_t x = 0, y = 0, k = 0, dinv = 0, w = 0, alpha = 0, ws = 0;
  const double* means = nullptr;
};

// ---- launch wrappers (defined in the .hip files) -------------------------------------------------
// zero / zero_bytes (optional, a multiple of 8): a buffer the Gram launch clears besides (the next launches' flags)
// mean_out (optional): mean_out[b] = p.const_mean for each problem b of the launch (Batch::means of the solves)
hipError_t launch_gram(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                       double* K, int64_t ldk, const Batch& bt = Batch(), int rb0 = 0, int32_t* info = nullptr,
                       void* zero = nullptr, size_t zero_bytes = 0, double* mean_out = nullptr);
// The forward half of alpha's triangular solve folded into the dataflow Cholesky: z = L^{-1} (Y - mean), with the
// padded rows and right-hand sides >= nrhs at 0.  buf (per problem, stride 2 npad nr doubles): the running right-hand
// sides (npad x nr), then z (npad x nr); nr = 1 for one right-hand side, else GPX_MAX_RHS (potrs' layout).
struct ForwardRhs {
  const double* Y = nullptr;
  int64_t ldy = 0, sy = 0;  // sy: Y stride per problem
  int nrhs = 1, n = 0;
  double mean = 0.0;
  const double* means = nullptr;  // per-problem means (device), overriding `mean` (Batch::means)
  double* buf = nullptr;
};
inline int rhs_row(int nrhs) { return nrhs == 1 ? 1 : GPX_MAX_RHS; }
// W (optional): the Dinv pass also writes W's diagonal blocks D_k^T (what trtri_diag would), so a fit that follows
// with launch_trtri(..., diag_done = true) saves one dispatch.  fr (optional): fold the forward substitution into the
// factorisation where the dataflow schedule runs; *z_done tells whether it did (z = buf + npad nr per problem).
hipError_t launch_potrf(Context* c, int npad, double* A, int64_t lda, double* Dinv, int32_t* info,
                        const Batch& bt = Batch(), double* W = nullptr, int64_t ldw = 0,
                        const ForwardRhs* fr = nullptr, bool* z_done = nullptr);
hipError_t launch_trtri(Context* c, int npad, const double* L, int64_t ldl, const double* Dinv, double* W,
                        int64_t ldw, double* T, const Batch& bt = Batch(), bool diag_done = false);
hipError_t launch_alpha(Context* c, int n, int npad, const double* W, int64_t ldw, const double* Y, int64_t ldy,
                        int nrhs, double const_mean, double* alpha, double* zpart, double* z,
                        const Batch& bt = Batch());
// alpha from L + Dinv by forward/backward triangular solves (gpx_potrs.hip); ws: potrs_workspace_bytes, zeroed by
// the launch itself (its hand-off granules)
size_t potrs_workspace_bytes(int64_t npad, int64_t nrhs, int64_t batch);
// ws_cleared: the granule block (potrs_clear_bytes) was already zeroed on the stream (by launch_gram in a fit)
size_t potrs_clear_bytes(int64_t npad, int64_t nrhs, int64_t batch);
// byte offset in the potrs workspace of the ForwardRhs buffer (2 npad nr doubles per problem)
size_t potrs_forward_offset(int64_t npad, int64_t nrhs, int64_t batch);
// z (optional): z = L^{-1} (Y - mean) from the factorisation (ForwardRhs; per problem at z + b * sz): the backward half
// only
hipError_t launch_potrs(Context* c, int n, int npad, const double* L, int64_t ldl, const double* Dinv,
                        const double* Y, int64_t ldy, int nrhs, double const_mean, double* alpha,
                        int32_t* info, void* ws, const Batch& bt = Batch(), bool ws_cleared = false,
                        const double* z = nullptr, int64_t sz = 0);

struct SweepBuffers {
  double* kstar;     // npad x C
  double* mu_part;   // (npad/64) x nrhs x C
  double* ss_part;   // (npad/128) x C
  double* rec_val;   // records (one per 256-candidate block over the whole sweep)
  int64_t* rec_idx;
  int64_t chunk;     // C
};
// One output t of a linear objective sum_t w_t f_t over independent GPs (gpx_acquire_argmax_multi_f64): the chunk's
// posterior of output t, untransformed by (y_mean, y_scale), weighted into chunk-sized accumulators.
struct MultiOutput {
  double weight = 1.0, y_mean = 0.0, y_scale = 1.0;
  int first = 1;
  double* acc_mu = nullptr;
  double* acc_var = nullptr;
};
// mode 0: posterior (write mean/var); mode 1: acquisition (records + optional scores); mo != nullptr: accumulate one
// output of a multi-output objective instead (mode ignored), scored afterwards by launch_multi_score
hipError_t launch_sweep_chunk(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                              const double* W, int64_t ldw, const double* alpha, int nrhs, const double* Xs,
                              int64_t ldxs, int64_t m_chunk, const SweepBuffers& b, int mode,
                              const gpx_acq_params* a, const double* y_mean, const double* y_scale,
                              double* mean_out, int64_t ldmean, double* var_out, double* scores_out,
                              int64_t rec_offset, int64_t index_offset, const MultiOutput* mo = nullptr);
hipError_t launch_multi_score(Context* c, const MultiOutput& mo, const gpx_acq_params& a, int64_t m_chunk,
                              double* scores_out, double* rec_val, int64_t* rec_idx, int64_t index_offset);
hipError_t launch_argmax_final(Context* c, const double* vals, const int64_t* idx, int64_t count, double* best_val,
                               int64_t* best_idx);
// the cross-GPU exchange (gpx_comm.cpp): pack the device record into {double value; int64 index}, and reduce
// `count` such packed records
hipError_t launch_record_pack(Context* c, const double* best_val, const int64_t* best_idx, int64_t* rec);
hipError_t launch_argmax_records(Context* c, const int64_t* rec, int64_t count, double* best_val, int64_t* best_idx);

// SVGP predictive of one task over a chunk (gpx_sweep.hip); ss2: (Mpad/128) x C partials of the full W2 product.
hipError_t launch_svgp_chunk(Context* c, const gpx_kernel_params& p, double min_var, int task, int M, int Mpad,
                             const double* Z, int64_t ldz, const double* W, const double* W2, int64_t ldw,
                             const double* alpha, const double* Xs, int64_t ldxs, int64_t m_chunk,
                             const SweepBuffers& b, double* ss2, double* mean_out, int64_t ldmean, double* var_out,
                             int64_t ldvar, double* score);
// SVGP preparation helpers (gpx_svgp.hip)
hipError_t launch_svgp_pad(Context* c, int ntask, int M, int Mpad, const double* vmean, int64_t stride_m,
                           const double* vchol, int64_t ldc, int64_t stride_c, double* mpad, double* spad,
                           int64_t sdst);
hipError_t launch_trmv_upper(Context* c, int npad, const double* W, int64_t ldw, const double* z, double* out,
                             const Batch& bt);
hipError_t launch_svgp_w2(Context* c, int ntask, int Mpad, const double* W, const double* S, int64_t s_stride,
                          double* W2);
size_t topk_workspace_bytes(int64_t m);
hipError_t launch_topk(Context* c, const double* scores, int64_t m, int64_t k, int64_t* idx_out, double* val_out,
                       void* ws, size_t ws_bytes);
hipError_t launch_fps(Context* c, const double* X, int64_t m, int d, int64_t ldx, int64_t k, int64_t start,
                      int64_t* idx_out);

hipError_t launch_append(Context* c, const gpx_kernel_params& p, int n_old, int n_new, const double* X, int64_t ldx,
                         double* L, int64_t ldl, double* Dinv, double* W, int64_t ldw, int32_t* info, double* ws);
size_t append_workspace_bytes(int64_t n_old, int64_t n_new);

size_t moments_grad_ws_doubles(int npad, int m);
hipError_t launch_moments_grad(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                               const double* W, int64_t ldw, const double* alpha, const double* Xs, int64_t ldxs,
                               int m, int q, double* mean, double* dmean, double* cov, double* dcov, double* ws);

size_t mll_workspace_bytes(int64_t npad);
hipError_t launch_mll(Context* c, const gpx_kernel_params& p, int n, int npad, const double* X, int64_t ldx,
                      const double* Y, int64_t ldy, int nrhs, const double* L, int64_t ldl, const double* W,
                      int64_t ldw, const double* alpha, double* out, double* part);

int64_t sweep_chunk_size(int64_t npad, int64_t m);
size_t sweep_workspace_bytes(int64_t npad, int64_t nrhs, int64_t m);

}  // namespace gpx
