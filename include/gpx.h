/*
 * gpx.h — C ABI of the MI355X-native exact-GP posterior engine (libgpx.so).
 *
 * This is the drop-in boundary for the hot path of billbearhunter/BayesianOptimizer.  In the reference
 * the path runs inside BoTorch/GPyTorch (not vendored); each entry point below names the reference call
 * site whose arithmetic it replaces.  Python binds it with ctypes (bayesianoptimizer_amd/_capi.py); see
 * INTEGRATION.md for the binding stub a maintainer adds to the reference.
 *
 * Conventions
 *  - Every array pointer is a DEVICE pointer owned by the caller (PyTorch tensors serve as containers).
 *    Host pointers are only the parameter structs and the out-scalars named *_host.
 *  - All matrices are row-major fp64 with an explicit leading dimension (in elements).
 *  - Training size n is padded internally to gpx_padded_n(n) (a multiple of GPX_TILE); padded rows of K are
 *    the identity, so L, L^{-1} and alpha are exact block extensions of the unpadded ones.  Buffers named
 *    "padded" must have gpx_padded_n(n) rows/cols.
 *  - Calls are asynchronous on the handle's stream (gpx_set_stream) and never allocate device memory;
 *    scratch comes from the caller's workspace (size from the *_workspace_size queries).
 *  - Errors: return a gpx_status; gpx_last_error(h) gives a message.  NOT_PD is reported through a device
 *    int32 `info` (0 = OK, > 0 failing pivot + 1, LAPACK potrf convention) so the fit stays asynchronous;
 *    gpx_fit_f64_sync reads it back and returns GPX_NOT_PD, like the reference's jitter-retry path
 *    (optimization/Bayesian6.py:481-488) expects an exception.  info = GPX_INFO_TIMEOUT (negative) means an
 *    in-launch hand-off of the factorisation or of the triangular solve gave up after its bounded spin
 *    (gpx_fit_f64_sync: GPX_TIMEOUT); the factor / alpha are then invalid.
 */
#ifndef GPX_H
#define GPX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPX_MAX_DIM 32
#define GPX_MAX_RHS 8
#define GPX_TILE 128
#define GPX_MAX_LD (1 << 20)            /* leading dimension limit of the matrix arguments (K, L, W) */
#define GPX_MAX_Q 32                    /* q-batch size of gpx_moments_grad_f64 */
#define GPX_MAX_GRAD_CANDIDATES 16384  /* candidates per gpx_moments_grad_f64 call */

typedef struct gpx_context* gpx_handle;
typedef struct gpx_comm_s* gpx_comm;   /* RCCL communicator of the cross-GPU record exchange */
#define GPX_COMM_ID_BYTES 128          /* ncclUniqueId */
typedef int32_t gpx_status;

enum {
  GPX_OK = 0,
  GPX_NOT_PD = 1,
  GPX_INVALID_ARG = 2,
  GPX_HIP_ERROR = 3,
  GPX_RCCL_ERROR = 4,
  GPX_TIMEOUT = 5 /* a persistent launch's hand-off timed out (device info = GPX_INFO_TIMEOUT) */
};
#define GPX_INFO_TIMEOUT ((int32_t)0x80000000)

/* Covariance modules used by the reference.
 * RBF: BoTorch SingleTaskGP default (optimization/Bayesian.py:91, Bayesian1.py:109) [upstream]
 * MATERN52: MaternKernel(nu=2.5) (config 3 of BASELINE.json)
 * SCALE_LINEAR_MATERN52: ScaleKernel(LinearKernel + MaternKernel(2.5)) (optimization/Bayesian6.py:471-473,
 *                        optimization/Bayesian7.py:162-166) */
enum { GPX_KERNEL_RBF = 0, GPX_KERNEL_MATERN52 = 1, GPX_KERNEL_SCALE_LINEAR_MATERN52 = 2 };

/* Acquisition scores (maximised). EI/LOGEI/UCB: BoTorch analytic forms [upstream] of the qLogEI call
 * (optimization/Bayesian.py:100-101); VARIANCE: the pool-scan score of optimization/Bayesian7.py:671. */
enum { GPX_ACQ_EI = 0, GPX_ACQ_LOGEI = 1, GPX_ACQ_UCB = 2, GPX_ACQ_VARIANCE = 3 };

/* Timers kept by gpx_timing_* (one per kernel family; gpx_timing_enable takes a bitmask of 1<<timer). */
enum {
  GPX_TIMER_GRAM = 0,
  GPX_TIMER_POTRF = 1,
  GPX_TIMER_TRTRI = 2,
  GPX_TIMER_ALPHA = 3,
  GPX_TIMER_KSTAR = 4,
  GPX_TIMER_TRMM = 5,
  GPX_TIMER_ACQ = 6,
  GPX_TIMER_MLL = 7,
  GPX_TIMER_COUNT = 8
};

/* Layout of the gpx_mll_grad_f64 output vector (GPX_MLL_NOUT doubles).  Gradients are of the negative log
 * marginal likelihood w.r.t. the natural (constrained) hyperparameters of gpx_kernel_params. */
enum {
  GPX_MLL_NLL = 0,            /* -log p(y) = QUAD + LOGDET/2 + n/2 log(2 pi) */
  GPX_MLL_QUAD = 1,           /* (y - m)^T K^{-1} (y - m) / 2 */
  GPX_MLL_LOGDET = 2,         /* log |K| = 2 sum log L_ii */
  GPX_MLL_D_NOISE = 3,
  GPX_MLL_D_OUTPUTSCALE = 4,
  GPX_MLL_D_MEAN = 5,
  GPX_MLL_D_LENGTHSCALE = 8,  /* GPX_MAX_DIM entries */
  GPX_MLL_D_LINVAR = 40,      /* GPX_MAX_DIM entries (SCALE_LINEAR_MATERN52 only) */
  GPX_MLL_NOUT = 72
};

typedef struct {
  int32_t kind;                          /* GPX_KERNEL_* */
  int32_t d;                             /* input dimension, 1..GPX_MAX_DIM */
  double lengthscale[GPX_MAX_DIM];       /* ARD lengthscales (Matérn / RBF part) */
  double linear_variance[GPX_MAX_DIM];   /* ARD LinearKernel variances (SCALE_LINEAR_MATERN52 only) */
  double outputscale;                    /* ScaleKernel s^2 (1.0 for BoTorch>=0.12 RBF default) */
  double noise;                          /* GaussianLikelihood noise sigma^2 */
  double jitter;                         /* extra diagonal (gpytorch.settings.cholesky_jitter) */
  double const_mean;                     /* ConstantMean */
  int32_t cov_fp32;                      /* 1: evaluate distances / exp / Matérn polynomial in fp32 (BASELINE
                                            configs[4] mixed-precision build), widen to fp64 before the fp64
                                            factorisation and sweep; 0: fp64 throughout */
  int32_t reserved;                      /* must be 0 */
} gpx_kernel_params;

typedef struct {
  int32_t kind;     /* GPX_ACQ_* */
  int32_t reserved; /* must be 0 */
  double best_f;    /* incumbent, in untransformed units (optimization/Bayesian.py:98) */
  double beta;      /* UCB beta */
  double y_mean;    /* Standardize untransform: mu_out = y_mean + y_scale * mu */
  double y_scale;   /*                          var_out = y_scale^2 * var       */
} gpx_acq_params;

/* ---- library / handle ---------------------------------------------------------------------------- */
const char* gpx_version(void);
gpx_status gpx_create(int32_t device, gpx_handle* out);
gpx_status gpx_destroy(gpx_handle h);
/* stream: a hipStream_t passed as void* (NULL = default stream). */
gpx_status gpx_set_stream(gpx_handle h, void* stream);
const char* gpx_last_error(gpx_handle h);
int64_t gpx_padded_n(int64_t n);
/* sizeof(gpx_kernel_params) (560) and sizeof(gpx_acq_params) (40) as compiled into the library: a binding checks its
 * own struct definitions against these once at load time.  Every entry point taking a
 * gpx_kernel_params also rejects cov_fp32 outside {0, 1} and reserved != 0 with GPX_INVALID_ARG. */
size_t gpx_kernel_params_size(void);
size_t gpx_acq_params_size(void);

/* Per-handle options (tuning and diagnostics; every default is the measured best).  gpx_create reads the environment
 * variable GPX_OPTIONS once ("name=value,name=value", names as below in lower case without the prefix, e.g.
 * "sweep_fused=0,potrf_mode=1"; an unknown name is reported on stderr and ignored); nothing else in the library reads
 * the environment.  The numbers are stable ABI: a removed option keeps its slot as GPX_OPT_RESERVED_n, which
 * gpx_set_option / gpx_get_option reject with GPX_INVALID_ARG.  The Cholesky schedule options (potrf_*) and gram_split
 * change no result bit: the schedules are arithmetic-invariant (any schedule that folds the forward substitution - every
 * default, and every potrf_mode 1 or potrf_lazy 1 setting - gives the same L, z and alpha; potrf_mode 0 with
 * potrf_lazy > 1 runs the forward substitution as a separate solve, so only alpha's rounding differs there).
 * sweep_fused = 0 takes the K* + trmm path at padded n <= 256, which sums in a different order: its results agree with
 * the fused path to the parity tolerance, not bit for bit.
 *  GPX_OPT_RESERVED_0      (was GPX_OPT_POTRF_SCHEDULE, removed in 0.4)
 *  GPX_OPT_SPIN_LIMIT      polls before an in-launch hand-off (the triangular solve's) gives up and
 *                          reports GPX_INFO_TIMEOUT (default 4194304; 0 = give up at the first unmet poll: tests)
 *  GPX_OPT_SWEEP_FUSED     1 (default) the fused small-n sweep where it applies (padded n <= 256), 0 the K* + trmm path
 *  GPX_OPT_GRAM_SPLIT      0 by size (default), else 1, 2 or 4 workgroups per 64x64 Gram tile
 *  GPX_OPT_POTRF_LAZY      multi-launch schedule: 0 by size and batch (default), else flush the trailing update every g columns
 *  GPX_OPT_POTRF_MODE      multi-launch schedule: -1 by size and batch (default), 0 eager panels, 1 lookahead panels
 *  GPX_OPT_POTRF_SWITCH    multi-launch schedule: -1 by size and batch (default), 0 no switch, k > 0: launches < k on
 *                          the lookahead schedule (flush every potrf_lazy, default 3 / by size), the rest eager (rounded
 *                          down to the launch after a flush)
 *  GPX_OPT_POTRF_SPLIT     panel row blocks per workgroup: -1 (default) split in 2 where the launch still fits the
 *                          co-resident slots, 1 never split, 3 split only where the split launch fits one workgroup per CU */
enum {
  GPX_OPT_RESERVED_0 = 0,
  GPX_OPT_SPIN_LIMIT = 1,
  GPX_OPT_SWEEP_FUSED = 2,
  GPX_OPT_GRAM_SPLIT = 3,
  GPX_OPT_POTRF_LAZY = 4,
  GPX_OPT_POTRF_MODE = 5,
  GPX_OPT_POTRF_SWITCH = 6,
  GPX_OPT_POTRF_SPLIT = 7,
  GPX_OPT_COUNT = 8
};
gpx_status gpx_set_option(gpx_handle h, int32_t option, int64_t value);
gpx_status gpx_get_option(gpx_handle h, int32_t option, int64_t* value_host);

/* ---- fit = posterior update ----------------------------------------------- */
/* Gram K(X,X)+(noise+jitter)I into the lower triangle of the padded K (replaces the covar_module(X) +
 * likelihood evaluation inside ExactMarginalLogLikelihood / ExactGP prediction strategy [upstream],
 * reached from optimization/Bayesian.py:91-93 and optimization/Bayesian6.py:476-484). */
gpx_status gpx_gram_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                        double* K, int64_t ldk);

/* In-place blocked lower Cholesky of the padded matrix (replaces psd_safe_cholesky [upstream];
 * jitter policy optimization/Bayesian6.py:483,487).  Dinv (2 * padded_n/64 * 64*64 doubles) receives the
 * inverses of the 64x64 diagonal blocks in its first half; the second half is scratch.  Only the lower
 * triangle of A is defined afterwards.  info: device int32, 0 or pivot+1. */
gpx_status gpx_potrf_f64(gpx_handle h, int64_t n, double* A, int64_t lda, double* Dinv, int32_t* info);

/* W = L^{-T} (upper triangular, row-major, i.e. W[k][i] = (L^{-1})[i][k]; strict lower part zeroed).
 * Needs the Dinv of gpx_potrf_f64.  Used by alpha and the candidate sweep. */
gpx_status gpx_trtri_workspace_size(int64_t n, size_t* bytes);
gpx_status gpx_trtri_f64(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv, double* W,
                         int64_t ldw, void* ws, size_t ws_bytes);

/* The same for `batch` factors at fixed element strides (the W of gpx_fit_factor_batched_f64's problems before their
 * sweeps), in the same launches. */
gpx_status gpx_trtri_batched_workspace_size(int64_t n, int64_t batch, size_t* bytes);
gpx_status gpx_trtri_batched_f64(gpx_handle h, int64_t batch, int64_t n, const double* L, int64_t ldl, int64_t stride_l,
                                 const double* Dinv, int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w,
                                 void* ws, size_t ws_bytes);

/* alpha = K^{-1} (Y - const_mean) = W W^T (Y - m) for nrhs <= GPX_MAX_RHS right-hand sides.  Y: n x nrhs
 * row-major with leading dim ldy; alpha: contiguous padded_n x nrhs (rows >= n are set to 0).
 * Replaces the ExactGP mean_cache [upstream]. */
gpx_status gpx_alpha_workspace_size(int64_t n, int64_t nrhs, size_t* bytes);
gpx_status gpx_alpha_f64(gpx_handle h, int64_t n, const double* W, int64_t ldw, const double* Y, int64_t ldy,
                         int64_t nrhs, double const_mean, double* alpha, void* ws, size_t ws_bytes);

/* One full posterior update: Gram + Cholesky + L^{-T} + alpha.  K (padded, in/out: holds L afterwards),
 * W, Dinv, alpha as above.  Asynchronous; *info (device) reports NOT_PD. */
gpx_status gpx_fit_workspace_size(int64_t n, int64_t nrhs, size_t* bytes);
gpx_status gpx_fit_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                       const double* Y, int64_t ldy, int64_t nrhs, double* K, int64_t ldk, double* Dinv,
                       double* W, int64_t ldw, double* alpha, int32_t* info, void* ws, size_t ws_bytes);
/* Same, then synchronises the stream and returns GPX_NOT_PD with *info_host = pivot+1 on failure. */
gpx_status gpx_fit_f64_sync(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                            const double* Y, int64_t ldy, int64_t nrhs, double* K, int64_t ldk, double* Dinv,
                            double* W, int64_t ldw, double* alpha, int32_t* info, void* ws, size_t ws_bytes,
                            int32_t* info_host);

/* alpha = K^{-1} (Y - const_mean) from the factor alone (LAPACK potrs): forward L z = Y - m, backward L^T alpha = z,
 * with L and Dinv as gpx_potrf_f64 left them (no W needed).  Y: n x nrhs (leading dim ldy), alpha: contiguous
 * padded_n x nrhs (rows >= n are 0).  info (device, nullable): the factor's pivot word — a failed factor (non-zero)
 * leaves alpha untouched; a solve whose in-launch hand-off times out writes GPX_INFO_TIMEOUT into it (and NaN into
 * alpha).  One launch; its workgroups hand 128-row blocks of z / alpha to each other inside it (deterministic: fixed
 * accumulation order).  Replaces the ExactGP mean_cache [upstream]. */
gpx_status gpx_potrs_workspace_size(int64_t n, int64_t nrhs, size_t* bytes);
gpx_status gpx_potrs_f64(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv, const double* Y,
                         int64_t ldy, int64_t nrhs, double const_mean, double* alpha, int32_t* info, void* ws,
                         size_t ws_bytes);

/* The posterior update as SURVEY §8d defines it — Gram + Cholesky + alpha — WITHOUT the explicit inverse: alpha by
 * gpx_potrs_f64.  K (padded, in/out: holds L afterwards), Dinv, alpha, info as in gpx_fit_f64.  Everything the fit
 * caches for prediction is then ready except W = L^{-T}, which gpx_trtri_f64(L, Dinv) builds when a sweep, a posterior,
 * an MLL gradient or an append needs it (the inverse costs as much as the factorisation; an update that is followed
 * by more updates before the next sweep never pays it). */
gpx_status gpx_fit_factor_workspace_size(int64_t n, int64_t nrhs, size_t* bytes);
gpx_status gpx_fit_factor_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                              const double* Y, int64_t ldy, int64_t nrhs, double* K, int64_t ldk, double* Dinv,
                              double* alpha, int32_t* info, void* ws, size_t ws_bytes);

/* Batched posterior updates: `batch` independent problems of the same n, d and kernel parameters (restarts /
 * seeds: BASELINE configs[3], the per-batch `info` of the SURVEY §8b proposal) in the SAME launches, the problem
 * index being one more grid dimension.  Every array of problem b starts at base + b * stride_* (element strides;
 * outputs K / Dinv / W / alpha >= one problem; the read-only X and Y any stride >= 0: X stride 0 = one X shared by
 * every problem, Y stride 1 with ldy = batch = column b of an n x batch target matrix); info: device int32[batch],
 * each 0 or that problem's failing pivot + 1.  Results are identical bit for
 * bit to `batch` calls of gpx_fit_f64 with the default options, although the batch may take a different Cholesky
 * schedule (every schedule computes each factor entry by the same MFMA chain, gpx_potrf.hip trailing_tile_at), so a
 * problem's result does not depend on how many problems share its GPU.  The Cholesky is a latency-bound chain of nblk dependent launches, so a batch of B
 * costs far less than B fits (replaces the per-restart fits of optimize_acqf / fit_gpytorch_mll restarts [upstream]). */
gpx_status gpx_fit_batched_workspace_size(int64_t n, int64_t nrhs, int64_t batch, size_t* bytes);
gpx_status gpx_fit_batched_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n, const double* X,
                               int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy, int64_t stride_y,
                               int64_t nrhs, double* K, int64_t ldk, int64_t stride_k, double* Dinv,
                               int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w, double* alpha,
                               int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes);
/* The same without W (gpx_fit_factor_f64 per problem, bit-identical to it). */
gpx_status gpx_fit_factor_batched_workspace_size(int64_t n, int64_t nrhs, int64_t batch, size_t* bytes);
gpx_status gpx_fit_factor_batched_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n,
                                      const double* X, int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy,
                                      int64_t stride_y, int64_t nrhs, double* K, int64_t ldk, int64_t stride_k,
                                      double* Dinv, int64_t stride_dinv, double* alpha, int64_t stride_alpha,
                                      int32_t* info, void* ws, size_t ws_bytes);

/* The same with ONE PARAMETER SET PER PROBLEM: p points to `batch` parameter structs of the same d (any kind, lengthscales,
 * outputscale, linear variances, noise, jitter and constant mean).  This is the reference's multi-output SingleTaskGP
 * (optimization/Bayesian1.py:108-116: SingleTaskGP(X, Y[n, 8], Standardize(m=8)), a batch of 8 independent GPs on one X,
 * each with its own lengthscales, outputscale, noise and ConstantMean [upstream]; optimization/Bayesian6.py:474-478
 * shares the covariance module, but its likelihood noise and mean are still per output): X stride 0, Y stride 1 with
 * ldy = batch and nrhs = 1.  The covariance of each problem is built with its own parameters (one Gram launch per
 * problem when they differ), the Cholesky and the solves run once over all problems; a problem's result is bit for bit
 * the single fit with its parameters.  Workspace sizes as for the shared-parameter entry points. */
gpx_status gpx_fit_batched_params_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n,
                                      const double* X, int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy,
                                      int64_t stride_y, int64_t nrhs, double* K, int64_t ldk, int64_t stride_k,
                                      double* Dinv, int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w,
                                      double* alpha, int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes);
gpx_status gpx_fit_factor_batched_params_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n,
                                             const double* X, int64_t ldx, int64_t stride_x, const double* Y,
                                             int64_t ldy, int64_t stride_y, int64_t nrhs, double* K, int64_t ldk,
                                             int64_t stride_k, double* Dinv, int64_t stride_dinv, double* alpha,
                                             int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes);

/* Incremental posterior update: rows n_old .. n_new-1 of X / Y appended to a GP whose L, Dinv and W
 * hold a successful fit (gpx_fit_f64 or an earlier append) of the first n_old rows with the SAME kernel parameters.
 * The reference appends the new observations and refits from scratch every round (optimization/Bayesian7.py:628-631,
 * 692-700 then :639; optimization/Bayesian.py:163-174); with the hyperparameters unchanged the leading block of the
 * factor is unchanged, so this bordered update costs O(n^2 q) (q = n_new - n_old) instead of O(n^3) and produces the
 * factor, W and alpha a fresh gpx_fit_f64 of all n_new rows would (rows past the last full 128-tile of the old fit
 * are refactored).  L / W must have leading dims >= gpx_padded_n(n_new) (allocate with spare capacity), Dinv room
 * for 2 * gpx_padded_n(n_new)/64 blocks, alpha gpx_padded_n(n_new) x nrhs.  Y holds all n_new targets (alpha is
 * recomputed, so a re-standardised Y is fine).  info: device int32, 0 or global failing pivot + 1. */
gpx_status gpx_append_workspace_size(int64_t n_old, int64_t n_new, int64_t nrhs, size_t* bytes);
gpx_status gpx_append_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n_old, int64_t n_new, const double* X,
                          int64_t ldx, const double* Y, int64_t ldy, int64_t nrhs, double* L, int64_t ldl,
                          double* Dinv, double* W, int64_t ldw, double* alpha, int32_t* info, void* ws,
                          size_t ws_bytes);

/* ---- posterior / acquisition ---------------------------------------------- */
/* Posterior at m points Xs (m x d, ld ldxs): mean (m x nrhs, ld ldmean) and variance (m), untransformed
 * by (y_mean[r], y_scale[r]) per output r (host arrays of nrhs; NULL = identity).  Replaces
 * model.posterior(X).mean/.variance (optimization/Bayesian2.py:169-171, optimization/Bayesian6.py:615-617).
 * var_out is the variance of output 0's untransform (all outputs share the factor). */
gpx_status gpx_sweep_workspace_size(int64_t n, int64_t nrhs, int64_t m, size_t* bytes);
gpx_status gpx_posterior_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                             const double* W, int64_t ldw, const double* alpha, int64_t nrhs, const double* Xs,
                             int64_t m, int64_t ldxs, const double* y_mean_host, const double* y_scale_host,
                             double* mean_out, int64_t ldmean, double* var_out, void* ws, size_t ws_bytes);

/* Candidate sweep: score m candidates with an analytic acquisition on the posterior whose mean uses the
 * padded_n vector `alpha` (one output column of gpx_alpha_f64, or a weighted combination of columns for a
 * linear objective) and reduce to (best value, lowest index among ties); reported indices are
 * index_offset + local index (candidate shards on several GPUs).  best_val/best_idx are device scalars; scores_out
 * (device, m) is optional (NULL = not written).  Replaces the raw-sample sweep + argmax of optimize_acqf
 * (optimization/Bayesian.py:105-113) and the pool scan + topk of optimization/Bayesian7.py:646-681. */
gpx_status gpx_acquire_argmax_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X,
                                  int64_t ldx, const double* W, int64_t ldw, const double* alpha,
                                  const double* Xs, int64_t m, int64_t ldxs, const gpx_acq_params* a,
                                  int64_t index_offset, double* best_val, int64_t* best_idx,
                                  double* scores_out, void* ws, size_t ws_bytes);

/* Candidate sweep of a LINEAR OBJECTIVE over T independent GPs on the same training inputs X (the outputs of the batched
 * fits above, or of separate fits / appends of the same n): f = sum_t w_t (y_mean[t] + y_scale[t] g_t) with g_t the
 * posterior of output t: its own p[t], W_host[t] (device pointer to its W = L^{-T}, leading dim ldw_host[t]) and
 * alpha_host[t] (device pointer to its padded_n alpha column); W_host / ldw_host / alpha_host are host arrays of T.  So mean = sum_t w_t (y_mean[t] +
 * y_scale[t] mu_t) and, the outputs being independent, variance = sum_t w_t^2 y_scale[t]^2 var_t (each var_t floored at
 * 1e-10 in its standardised space, the sum at 1e-12: GPyTorch's / BoTorch's floors [upstream]).  Scored with a's kind /
 * best_f / beta (a->y_mean, a->y_scale are not used: the per-output y_mean_host / y_scale_host are, NULL = 0 / 1) and
 * reduced like gpx_acquire_argmax_f64.  VARIANCE with w_t = 1 is the variance-sum pool-scan score of
 * optimization/Bayesian7.py:671 over independent outputs; EI / LogEI / UCB with weights the scalarised objective of a
 * multi-output model (optimization/Bayesian1.py:119-140's mean-of-8 objective, analytic form).  T = 1, w = 1 gives
 * gpx_acquire_argmax_f64's scores bit for bit. */
gpx_status gpx_sweep_multi_workspace_size(int64_t n, int64_t m, size_t* bytes);
gpx_status gpx_acquire_argmax_multi_f64(gpx_handle h, const gpx_kernel_params* p, int64_t T, int64_t n, const double* X,
                                        int64_t ldx, const double* const* W_host, const int64_t* ldw_host,
                                        const double* const* alpha_host, const double* weights_host,
                                        const double* y_mean_host, const double* y_scale_host, const double* Xs,
                                        int64_t m, int64_t ldxs, const gpx_acq_params* a, int64_t index_offset,
                                        double* best_val, int64_t* best_idx, double* scores_out, void* ws,
                                        size_t ws_bytes);

/* Deterministic (value, index) reduction of `count` device records: max value, then lowest index; NaN
 * never wins.  Used after the cross-GPU all-gather of per-rank records. */
gpx_status gpx_argmax_combine_f64(gpx_handle h, const double* vals, const int64_t* idx, int64_t count,
                                  double* best_val, int64_t* best_idx);

/* ---- gradients for acquisition optimisation ---------------------------------------------- */
/* Posterior moments of m candidates Xs (m x d) grouped in consecutive q-batches (m/q batches of q points: restarts of
 * optimize_acqf x its q, optimization/Bayesian.py:105-112, optimization/Bayesian2.py:240-245) and their derivatives
 * w.r.t. the candidates, for the L-BFGS-B refinement that BoTorch drives with torch autograd [upstream].  In the
 * engine's (standardised) units, with alpha one padded_n column and c ranging over a's batch:
 *   mean[a]   = const_mean + k_a^T alpha                 dmean[a*d + j]       = d mean[a] / d x_aj
 *   cov[a*q + c'] = k(x_a, x_c) - k_a^T K^{-1} k_c     dcov[(a*d + j)*q + c'] = d1 k(x_a, x_c)/dx_aj - d k_a/dx_aj^T K^{-1} k_c
 * (c = batch start + c'; d1 = derivative in the first argument only, so that the gradient of a function L of the batch
 * covariance is dL/dx_aj = sum_c' (G[a][c] + G[c][a]) dcov[(a*d+j)*q + c'] with G = dL/dcov).  K^{-1} k_c = W (W^T k_c)
 * on fp64 MFMA; the q-batch posterior covariance is noise-free (add noise for observation noise).  All outputs are
 * device arrays; deterministic. */
gpx_status gpx_moments_grad_workspace_size(int64_t n, int64_t m, size_t* bytes);
gpx_status gpx_moments_grad_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                                const double* W, int64_t ldw, const double* alpha, const double* Xs, int64_t m,
                                int64_t q, int64_t ldxs, double* mean, double* dmean, double* cov, double* dcov,
                                void* ws, size_t ws_bytes);

/* ---- cross-GPU selection exchange (SURVEY §8b gpx_allreduce_argmax, §8e) ------------------------------------------ */
/* One process per GPU.  Rank 0 creates the communicator id (gpx_comm_unique_id), the host side broadcasts its
 * GPX_COMM_ID_BYTES bytes (e.g. over torch.distributed), every rank calls gpx_comm_init (collective).
 * gpx_allreduce_argmax replaces every rank's device (best_val, best_idx) record by the global best: the record is
 * packed into one 16-byte {fp64 value, int64 index} on the device, ONE RCCL all-gather of those 16 bytes per rank runs
 * over xGMI, then the argmax_combine kernel (max value, lowest global index, NaN never wins) on the handle's stream —
 * RCCL has no MAXLOC.  Three stream operations per exchange; no host synchronisation.  Replaces the final best-candidate selection across the
 * independent restarts/shards (BASELINE configs[3]). */
gpx_status gpx_comm_unique_id(uint8_t* id_out);
gpx_status gpx_comm_init(gpx_handle h, const uint8_t* id, int32_t nranks, int32_t rank, gpx_comm* out);
gpx_status gpx_comm_destroy(gpx_comm c);
gpx_status gpx_allreduce_argmax_workspace_size(gpx_comm c, size_t* bytes);
gpx_status gpx_allreduce_argmax(gpx_handle h, gpx_comm c, double* best_val, int64_t* best_idx, void* ws,
                                size_t ws_bytes);

/* ---- marginal likelihood -------------------------------------------------------- */
/* Negative log marginal likelihood of a fitted exact GP with T = nrhs outputs sharing the covariance (T = 1:
 * the SingleTaskGP objective) and its gradient w.r.t. the shared hyperparameters:
 *   -log p(Y) = sum_t [ (y_t - m)^T alpha_t / 2 ] + T (sum log L_ii + n/2 log 2 pi)
 *   d/d theta = 1/2 sum_ij (T K^{-1} - sum_t alpha_t alpha_t^T)_ij dK_ij/d theta,   d/dm = -sum_t sum_i alpha_ti,
 * with K^{-1} = W W^T formed tile by tile on the MFMA units and contracted against dK/d theta recomputed
 * from X inside the same kernel (K^{-1} is never stored).  Inputs are the outputs of gpx_fit_f64: L (the
 * factored K), W, alpha (contiguous padded_n x nrhs), and the targets Y (n x nrhs, leading dim ldy) the fit
 * used.  out: device array of GPX_MLL_NOUT doubles (layout above; QUAD and LOGDET are the totals over the
 * outputs and one log|K|; the covariance is differentiated in fp64 regardless of cov_fp32).  Deterministic
 * (fixed reduction order).  Replaces ExactMarginalLogLikelihood(...).backward() inside fit_gpytorch_mll
 * [upstream] (optimization/Bayesian.py:92-93, optimization/Bayesian1.py:114-115, optimization/Bayesian6.py:480-488). */
gpx_status gpx_mll_workspace_size(int64_t n, size_t* bytes);
/* (the batched form is below) */
gpx_status gpx_mll_grad_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                            const double* Y, int64_t ldy, int64_t nrhs, const double* L, int64_t ldl,
                            const double* W, int64_t ldw, const double* alpha, double* out, void* ws,
                            size_t ws_bytes);

/* The same for `batch` independent problems with one parameter set each (the fits of gpx_fit_batched_params_f64):
 * problem b's X, Y, L, W, alpha at base + b * stride_* (X / Y strides >= 0, as in the batched fit), its output vector at
 * out + b * GPX_MLL_NOUT.  The reference's multi-output fit_gpytorch_mll minimises the SUM of the per-output losses
 * (optimization/Bayesian1.py:114-115 [upstream]); the host side (mll.py) sums them.  Workspace: gpx_mll_workspace_size. */
gpx_status gpx_mll_grad_batched_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n, const double* X,
                                    int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy, int64_t stride_y,
                                    int64_t nrhs, const double* L, int64_t ldl, int64_t stride_l, const double* W,
                                    int64_t ldw, int64_t stride_w, const double* alpha, int64_t stride_alpha,
                                    double* out, void* ws, size_t ws_bytes);

/* ---- SVGP predictive + pool-scan selection: the driven variant ---------------- */
/* optimization/Bayesian7.py's BatchSVGP (ntask outputs, each with its own ScaleKernel(Linear + Matérn-5/2)
 * hyperparameters p[t], ConstantMean p[t].const_mean and GaussianLikelihood noise p[t].noise) served from its trained
 * variational state: inducing points Z (ntask x M x d), variational mean m (ntask x M) and chol_variational_covar
 * (ntask x M x M, only its lower triangle is used, like CholeskyVariationalDistribution [upstream]).
 *
 * gpx_svgp_prepare_f64 (once per trained model) factors K_ZZ + jitter I per task (gpytorch's VariationalStrategy
 * jitter: 1e-4 for the reference's float32 model [upstream]) and stores per task, in padded Mpad x Mpad blocks
 * (Mpad = gpx_padded_n(M)): W = L_ZZ^{-T}, W2 = W S, and alpha' = W m (Mpad entries).  info: int32[ntask].
 * gpx_svgp_predict_f64 evaluates the whitened predictive of every task at m points Xs (already input-transformed,
 * Bayesian7.py:181-190): mean = const + k*^T alpha', var = max(k** - |W^T k*|^2 + |W2^T k*|^2 + noise, min_var)
 * (= likelihood(model(x)).variance, Bayesian7.py:558,668) into mean_out / var_out (m x ntask, NULL = skip) and
 * score_out[m] = sum over tasks of var (the pool-scan uncertainty score, Bayesian7.py:671; NULL = skip). */
gpx_status gpx_svgp_prepare_workspace_size(int64_t M, int64_t ntask, size_t* bytes);
gpx_status gpx_svgp_prepare_f64(gpx_handle h, const gpx_kernel_params* p, int64_t ntask, int64_t M, double jitter,
                                const double* Z, int64_t ldz, int64_t stride_z, const double* vmean,
                                int64_t stride_m, const double* vchol, int64_t ldc, int64_t stride_c, double* W,
                                double* W2, double* alpha, int32_t* info, void* ws, size_t ws_bytes);
gpx_status gpx_svgp_predict_workspace_size(int64_t M, int64_t m, size_t* bytes);
gpx_status gpx_svgp_predict_f64(gpx_handle h, const gpx_kernel_params* p, int64_t ntask, int64_t M, const double* Z,
                                int64_t ldz, int64_t stride_z, const double* W, const double* W2, const double* alpha,
                                const double* Xs, int64_t m, int64_t ldxs, double min_var, double* mean_out,
                                int64_t ldmean, double* var_out, int64_t ldvar, double* score_out, void* ws,
                                size_t ws_bytes);

/* The k largest scores in descending order (replaces torch.topk, Bayesian7.py:681): stable, so equal scores keep
 * the lower index first; NaN ranks last.  idx_out: int64[k], val_out: double[k] (NULL = skip). */
gpx_status gpx_topk_workspace_size(int64_t m, size_t* bytes);
gpx_status gpx_topk_f64(gpx_handle h, const double* scores, int64_t m, int64_t k, int64_t* idx_out, double* val_out,
                        void* ws, size_t ws_bytes);

/* Greedy farthest point sampling of k of the m points X (m <= 32768), starting at index `start` (the reference
 * draws it with torch.randint): farthest_point_sampling of Bayesian7.py:82-106.  Squared Euclidean distances in
 * fp64, argmax with the lowest index among ties (torch.argmax).  idx_out: int64[k], the selection order. */
gpx_status gpx_fps_f64(gpx_handle h, const double* X, int64_t m, int64_t d, int64_t ldx, int64_t k, int64_t start,
                       int64_t* idx_out);

/* ---- instrumentation ------------------------------------------------------------------------------ */
/* For every timer whose bit is set in `mask`, each launch of that kernel family is bracketed by hipEvents
 * on the handle's stream; totals are read with gpx_timing_query (synchronises the stream). mask 0 = off. */
gpx_status gpx_timing_enable(gpx_handle h, int32_t mask);
gpx_status gpx_timing_reset(gpx_handle h);
gpx_status gpx_timing_query(gpx_handle h, int32_t timer, double* total_ms_host, int64_t* launches_host);

#ifdef __cplusplus
}
#endif
#endif /* GPX_H */
