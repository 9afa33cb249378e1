// The C ABI of libgpx.so (include/gpx.h): argument validation, workspace carving, chunk loop and timers.
// Every exported symbol is extern "C" with plain pointers; no torch types cross this boundary.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include "gpx_internal.h"

using gpx::Context;

namespace {

// GPX_SOURCE_SHA256: sha256 over csrc/* and include/gpx.h (the Makefile stamps it; tests/test_capi.py recomputes it from
// the working tree, so a stale or foreign libgpx.so is caught)
#ifndef GPX_SOURCE_SHA256
#define GPX_SOURCE_SHA256 "unstamped"
#endif
constexpr const char* kVersion = "gpx 0.5.0 (gfx950, fp64 MFMA) src " GPX_SOURCE_SHA256;

gpx_status fail(Context* c, gpx_status st, const std::string& msg) {
  if (c) c->last_error = msg;
  return st;
}

gpx_status hip_check(Context* c, hipError_t e, const char* where) {
  if (e == hipSuccess) return GPX_OK;
  return fail(c, GPX_HIP_ERROR, std::string(where) + ": " + hipGetErrorString(e));
}


int64_t padded(int64_t n) { return ((n + GPX_TILE - 1) / GPX_TILE) * GPX_TILE; }

gpx_status check_params(Context* c, const gpx_kernel_params* p) {
  if (!p) return fail(c, GPX_INVALID_ARG, "kernel params pointer is NULL");
  if (p->kind < GPX_KERNEL_RBF || p->kind > GPX_KERNEL_SCALE_LINEAR_MATERN52)
    return fail(c, GPX_INVALID_ARG, "unknown kernel kind " + std::to_string(p->kind));
  if (p->d < 1 || p->d > GPX_MAX_DIM)
    return fail(c, GPX_INVALID_ARG, "input dimension d=" + std::to_string(p->d) + " outside [1, 32]");
  for (int k = 0; k < p->d; ++k)
    if (!(p->lengthscale[k] > 0.0) || !std::isfinite(p->lengthscale[k]))
      return fail(c, GPX_INVALID_ARG, "lengthscale[" + std::to_string(k) + "] must be positive and finite");
  if (!(p->outputscale >= 0.0) || !(p->noise >= 0.0) || !(p->jitter >= 0.0))
    return fail(c, GPX_INVALID_ARG, "outputscale/noise/jitter must be non-negative");
  // The trailing int32 pair is part of the contract: a caller whose struct definition stops before it (552 instead of
  // gpx_kernel_params_size() bytes) would hand over whatever follows its struct in memory, and a stray non-zero
  // cov_fp32 would silently switch the covariance build to fp32.  Anything but {0, 1} / 0 is rejected.
  if (p->cov_fp32 != 0 && p->cov_fp32 != 1)
    return fail(c, GPX_INVALID_ARG, "cov_fp32 must be 0 or 1 (got " + std::to_string(p->cov_fp32) +
                                        "; is the caller's gpx_kernel_params " + std::to_string(sizeof(gpx_kernel_params)) +
                                        " bytes?)");
  if (p->reserved != 0) return fail(c, GPX_INVALID_ARG, "gpx_kernel_params.reserved must be 0");
  return GPX_OK;
}

gpx_status check_n(Context* c, int64_t n) {
  if (n < 1 || n > (int64_t)1 << 20) return fail(c, GPX_INVALID_ARG, "n must be in [1, 2^20]");
  return GPX_OK;
}

gpx_status check_ld(Context* c, int64_t ld, int64_t minimum, const char* name, bool even) {
  if (ld < minimum) return fail(c, GPX_INVALID_ARG, std::string(name) + " leading dimension too small");
  if (even && (ld & 1)) return fail(c, GPX_INVALID_ARG, std::string(name) + " leading dimension must be even");
  // the matrix kernels address 128-row tiles through buffer descriptors with 32-bit byte offsets
  if (even && ld > GPX_MAX_LD)
    return fail(c, GPX_INVALID_ARG, std::string(name) + " leading dimension above GPX_MAX_LD (2^20)");
  return GPX_OK;
}

#define GPX_TRY(expr)               \
  do {                              \
    gpx_status _st = (expr);        \
    if (_st != GPX_OK) return _st;  \
  } while (0)

// Makes the handle's device current for the rest of the calling entry point and restores the caller's device on return.
#define GPX_USE_DEVICE(c)                                  \
  gpx::DeviceScope _gpx_dev((c)->device);                  \
  if (_gpx_dev.err != hipSuccess) return hip_check((c), _gpx_dev.err, "hipSetDevice")

#define GPX_NONNULL(c, ptr) \
  do { if (!(ptr)) return fail((c), GPX_INVALID_ARG, #ptr " is NULL"); } while (0)

size_t trtri_ws(int64_t npad) { return (size_t)npad * npad / 4 * 8 + 256; }
size_t alpha_ws(int64_t npad, int64_t nrhs) { return ((size_t)(npad / 128) + 1) * npad * nrhs * 8 + 512; }

double* align256(void* p) {
  uintptr_t u = reinterpret_cast<uintptr_t>(p);
  u = (u + 255) & ~(uintptr_t)255;
  return reinterpret_cast<double*>(u);
}

}  // namespace

namespace gpx {

LaunchTimer::LaunchTimer(Context* ctx, int t) : c(ctx), timer(t) {
  if (!(c->timing_mask & (1 << t))) return;
  auto take = [&]() {
    hipEvent_t ev;
    if (!c->free_events.empty()) {
      ev = c->free_events.back();
      c->free_events.pop_back();
    } else if (hipEventCreate(&ev) != hipSuccess) {
      return (hipEvent_t) nullptr;
    }
    return ev;
  };
  s = take();
  e = take();
  if (s) (void)hipEventRecord(s, c->stream);
}

LaunchTimer::~LaunchTimer() {
  if (!s || !e) return;
  (void)hipEventRecord(e, c->stream);
  c->pending.push_back({timer, s, e});
}

}  // namespace gpx

extern "C" {

const char* gpx_version(void) { return kVersion; }

int64_t gpx_padded_n(int64_t n) { return padded(n); }

size_t gpx_kernel_params_size(void) { return sizeof(gpx_kernel_params); }

size_t gpx_acq_params_size(void) { return sizeof(gpx_acq_params); }

static void apply_env_options(Context* c);

gpx_status gpx_create(int32_t device, gpx_handle* out) {
  if (!out) return GPX_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return GPX_HIP_ERROR;
  if (device < 0 || device >= count) return GPX_INVALID_ARG;
  Context* c = new (std::nothrow) Context();
  if (!c) return GPX_HIP_ERROR;
  c->device = device;
  apply_env_options(c);
  {
    gpx::DeviceScope dev(device);  // the device must be selectable; the caller's current device is left as it was
    if (dev.err != hipSuccess) {
      delete c;
      return GPX_HIP_ERROR;
    }
  }
  *out = reinterpret_cast<gpx_handle>(c);
  return GPX_OK;
}

gpx_status gpx_destroy(gpx_handle h) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  (void)hipStreamSynchronize(c->stream);
  for (auto& pt : c->pending) {
    (void)hipEventDestroy(pt.start);
    (void)hipEventDestroy(pt.stop);
  }
  for (auto ev : c->free_events) (void)hipEventDestroy(ev);
  delete c;
  return GPX_OK;
}

gpx_status gpx_set_stream(gpx_handle h, void* stream) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  c->stream = reinterpret_cast<hipStream_t>(stream);
  return GPX_OK;
}

static gpx_status set_option(Context* c, int32_t option, int64_t v) {
  switch (option) {
    case GPX_OPT_SPIN_LIMIT:
      if (v < 0 || v > 0x7fffffff) return fail(c, GPX_INVALID_ARG, "spin_limit must be in [0, 2^31)");
      c->spin_limit = (unsigned)v;
      return GPX_OK;
    case GPX_OPT_SWEEP_FUSED:
      if (v != 0 && v != 1) return fail(c, GPX_INVALID_ARG, "sweep_fused must be 0 or 1");
      c->sweep_fused = (int)v;
      return GPX_OK;
    case GPX_OPT_GRAM_SPLIT:
      if (v != 0 && v != 1 && v != 2 && v != 4) return fail(c, GPX_INVALID_ARG, "gram_split must be 0, 1, 2 or 4");
      c->gram_split = (int)v;
      return GPX_OK;
    case GPX_OPT_POTRF_LAZY:
      if (v < 0 || v > 16) return fail(c, GPX_INVALID_ARG, "potrf_lazy must be in [0, 16]");
      c->potrf_lazy = (int)v;
      return GPX_OK;
    case GPX_OPT_POTRF_MODE:
      if (v < -1 || v > 1) return fail(c, GPX_INVALID_ARG, "potrf_mode must be -1, 0 or 1");
      c->potrf_mode = (int)v;
      return GPX_OK;
    case GPX_OPT_POTRF_SWITCH:
      if (v < -1 || v > 16384) return fail(c, GPX_INVALID_ARG, "potrf_switch must be in [-1, 16384]");
      c->potrf_switch = (int)v;
      return GPX_OK;
    case GPX_OPT_POTRF_SPLIT:
      if (v != -1 && v != 1 && v != 3) return fail(c, GPX_INVALID_ARG, "potrf_split must be -1, 1 or 3");
      c->potrf_split = (int)v;
      return GPX_OK;
    default:
      return fail(c, GPX_INVALID_ARG, "unknown option " + std::to_string(option));
  }
}

static int option_by_name(const std::string& name) {
  // index = GPX_OPT_* number; slot 0 is reserved (the removed potrf_schedule) and has no name
  static const char* names[GPX_OPT_COUNT] = {"", "spin_limit", "sweep_fused", "gram_split", "potrf_lazy", "potrf_mode",
                                               "potrf_switch", "potrf_split"};
  for (int i = 1; i < GPX_OPT_COUNT; ++i)
    if (name == names[i]) return i;
  return -1;
}

// GPX_OPTIONS="name=value,...": the library's only read of the environment (tuning / A-B tools)
static void apply_env_options(Context* c) {
  const char* e = std::getenv("GPX_OPTIONS");
  if (!e) return;
  std::string all(e);
  size_t pos = 0;
  while (pos < all.size()) {
    size_t end = all.find(',', pos);
    if (end == std::string::npos) end = all.size();
    const std::string item = all.substr(pos, end - pos);
    const size_t eq = item.find('=');
    if (eq != std::string::npos) {
      const int opt = option_by_name(item.substr(0, eq));
      if (opt >= 0) {
        if (set_option(c, opt, std::atoll(item.c_str() + eq + 1)) != GPX_OK)
          std::fprintf(stderr, "gpx: GPX_OPTIONS: %s (ignored)\n", c->last_error.c_str());
      } else {
        std::fprintf(stderr, "gpx: GPX_OPTIONS: unknown option '%s' (ignored)\n", item.substr(0, eq).c_str());
      }
    } else if (!item.empty()) {
      std::fprintf(stderr, "gpx: GPX_OPTIONS: '%s' is not name=value (ignored)\n", item.c_str());
    }
    pos = end + 1;
  }
  c->last_error.clear();
}

gpx_status gpx_set_option(gpx_handle h, int32_t option, int64_t value) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  return set_option(c, option, value);
}

gpx_status gpx_get_option(gpx_handle h, int32_t option, int64_t* value_host) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_NONNULL(c, value_host);
  switch (option) {
    case GPX_OPT_SPIN_LIMIT: *value_host = c->spin_limit; return GPX_OK;
    case GPX_OPT_SWEEP_FUSED: *value_host = c->sweep_fused; return GPX_OK;
    case GPX_OPT_GRAM_SPLIT: *value_host = c->gram_split; return GPX_OK;
    case GPX_OPT_POTRF_LAZY: *value_host = c->potrf_lazy; return GPX_OK;
    case GPX_OPT_POTRF_MODE: *value_host = c->potrf_mode; return GPX_OK;
    case GPX_OPT_POTRF_SWITCH: *value_host = c->potrf_switch; return GPX_OK;
    case GPX_OPT_POTRF_SPLIT: *value_host = c->potrf_split; return GPX_OK;
    default: return fail(c, GPX_INVALID_ARG, "unknown option " + std::to_string(option));
  }
}

const char* gpx_last_error(gpx_handle h) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return "invalid handle";
  return c->last_error.c_str();
}

// gram_impl clears *info (when given) inside the gram kernel: the fit needs no separate memset dispatch
static gpx_status gram_impl(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                            double* K, int64_t ldk, int32_t* info, void* zero = nullptr, size_t zero_bytes = 0) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_params(c, p));
  GPX_TRY(check_n(c, n));
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, K);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldk, npad, "K", true));
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_gram(c, *p, (int)n, (int)npad, X, ldx, K, ldk, gpx::Batch(), 0, info, zero, zero_bytes),
                   "gram");
}

gpx_status gpx_gram_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                        double* K, int64_t ldk) {
  return gram_impl(h, p, n, X, ldx, K, ldk, nullptr);
}

static gpx_status potrf_impl(gpx_handle h, int64_t n, double* A, int64_t lda, double* Dinv, int32_t* info,
                             bool clear_info, double* W = nullptr, int64_t ldw = 0,
                             const gpx::ForwardRhs* fr = nullptr, bool* z_done = nullptr) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_n(c, n));
  GPX_NONNULL(c, A);
  GPX_NONNULL(c, Dinv);
  GPX_NONNULL(c, info);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, lda, npad, "A", true));
  GPX_USE_DEVICE(c);
  if (clear_info) GPX_TRY(hip_check(c, hipMemsetAsync(info, 0, sizeof(int32_t), c->stream), "memset info"));
  return hip_check(c, gpx::launch_potrf(c, (int)npad, A, lda, Dinv, info, gpx::Batch(), W, ldw, fr, z_done), "potrf");
}

gpx_status gpx_potrf_f64(gpx_handle h, int64_t n, double* A, int64_t lda, double* Dinv, int32_t* info) {
  return potrf_impl(h, n, A, lda, Dinv, info, true);
}

gpx_status gpx_trtri_workspace_size(int64_t n, size_t* bytes) {
  if (!bytes || n < 1) return GPX_INVALID_ARG;
  *bytes = trtri_ws(padded(n));
  return GPX_OK;
}

static gpx_status trtri_impl(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv, double* W,
                             int64_t ldw, void* ws, size_t ws_bytes, bool diag_done) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_n(c, n));
  GPX_NONNULL(c, L);
  GPX_NONNULL(c, Dinv);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldl, npad, "L", true));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  if (ws_bytes < trtri_ws(npad)) return fail(c, GPX_INVALID_ARG, "trtri workspace too small");
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_trtri(c, (int)npad, L, ldl, Dinv, W, ldw, align256(ws), gpx::Batch(), diag_done),
                   "trtri");
}

gpx_status gpx_trtri_f64(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv, double* W,
                         int64_t ldw, void* ws, size_t ws_bytes) {
  return trtri_impl(h, n, L, ldl, Dinv, W, ldw, ws, ws_bytes, false);
}

gpx_status gpx_trtri_batched_workspace_size(int64_t n, int64_t batch, size_t* bytes) {
  if (!bytes || n < 1 || batch < 1 || batch > 65535) return GPX_INVALID_ARG;
  *bytes = ((trtri_ws(padded(n)) + 255) & ~(size_t)255) * (size_t)batch + 256;
  return GPX_OK;
}

gpx_status gpx_trtri_batched_f64(gpx_handle h, int64_t batch, int64_t n, const double* L, int64_t ldl, int64_t stride_l,
                                 const double* Dinv, int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w,
                                 void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_n(c, n));
  if (batch < 1 || batch > 65535) return fail(c, GPX_INVALID_ARG, "batch must be in [1, 65535]");
  GPX_NONNULL(c, L);
  GPX_NONNULL(c, Dinv);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldl, npad, "L", true));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  if (batch > 1) {
    if (stride_l < npad * ldl || stride_w < npad * ldw || stride_dinv < 2 * (npad / gpx::NB) * gpx::NB * gpx::NB)
      return fail(c, GPX_INVALID_ARG, "batch strides smaller than one problem");
    if ((stride_l | stride_w | stride_dinv) & 1) return fail(c, GPX_INVALID_ARG, "L/W/Dinv strides must be even");
  }
  size_t need = 0;
  GPX_TRY(gpx_trtri_batched_workspace_size(n, batch, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "batched trtri workspace too small");
  GPX_USE_DEVICE(c);
  gpx::Batch bt;
  bt.count = (int)batch;
  bt.k = stride_l;
  bt.dinv = stride_dinv;
  bt.w = stride_w;
  bt.ws = (int64_t)(((trtri_ws(npad) + 255) & ~(size_t)255) / sizeof(double));
  return hip_check(c, gpx::launch_trtri(c, (int)npad, L, ldl, Dinv, W, ldw, align256(ws), bt, false), "trtri");
}

gpx_status gpx_alpha_workspace_size(int64_t n, int64_t nrhs, size_t* bytes) {
  if (!bytes || n < 1 || nrhs < 1 || nrhs > GPX_MAX_RHS) return GPX_INVALID_ARG;
  *bytes = alpha_ws(padded(n), nrhs);
  return GPX_OK;
}

gpx_status gpx_alpha_f64(gpx_handle h, int64_t n, const double* W, int64_t ldw, const double* Y, int64_t ldy,
                         int64_t nrhs, double const_mean, double* alpha, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_n(c, n));
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, Y);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  if (ws_bytes < alpha_ws(npad, nrhs)) return fail(c, GPX_INVALID_ARG, "alpha workspace too small");
  GPX_USE_DEVICE(c);
  double* zpart = align256(ws);
  double* z = zpart + (size_t)(npad / 128) * npad * nrhs;
  return hip_check(c, gpx::launch_alpha(c, (int)n, (int)npad, W, ldw, Y, ldy, (int)nrhs, const_mean, alpha, zpart, z),
                   "alpha");
}

gpx_status gpx_fit_workspace_size(int64_t n, int64_t nrhs, size_t* bytes) {
  if (!bytes || n < 1 || nrhs < 1 || nrhs > GPX_MAX_RHS) return GPX_INVALID_ARG;
  const int64_t npad = padded(n);
  size_t a = trtri_ws(npad), b = alpha_ws(npad, nrhs);
  *bytes = a > b ? a : b;
  return GPX_OK;
}

gpx_status gpx_fit_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                       const double* Y, int64_t ldy, int64_t nrhs, double* K, int64_t ldk, double* Dinv, double* W,
                       int64_t ldw, double* alpha, int32_t* info, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  size_t need = 0;
  if (gpx_fit_workspace_size(n, nrhs, &need) != GPX_OK)
    return fail(c, GPX_INVALID_ARG, "invalid n / nrhs for fit");
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "fit workspace too small");
  if (!info) return fail(c, GPX_INVALID_ARG, "info is NULL");
  GPX_TRY(gram_impl(h, p, n, X, ldx, K, ldk, info));
  if (!W) return fail(c, GPX_INVALID_ARG, "W is NULL");
  // W's leading dimension is validated before the Dinv pass writes W's diagonal blocks
  GPX_TRY(check_ld(c, ldw, padded(n), "W", true));
  GPX_TRY(potrf_impl(h, n, K, ldk, Dinv, info, false, W, ldw));
  GPX_TRY(trtri_impl(h, n, K, ldk, Dinv, W, ldw, ws, ws_bytes, true));
  return gpx_alpha_f64(h, n, W, ldw, Y, ldy, nrhs, p->const_mean, alpha, ws, ws_bytes);
}

gpx_status gpx_fit_f64_sync(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                            const double* Y, int64_t ldy, int64_t nrhs, double* K, int64_t ldk, double* Dinv,
                            double* W, int64_t ldw, double* alpha, int32_t* info, void* ws, size_t ws_bytes,
                            int32_t* info_host) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(gpx_fit_f64(h, p, n, X, ldx, Y, ldy, nrhs, K, ldk, Dinv, W, ldw, alpha, info, ws, ws_bytes));
  int32_t hinfo = 0;
  GPX_TRY(hip_check(c, hipMemcpyAsync(&hinfo, info, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream), "info D2H"));
  GPX_TRY(hip_check(c, hipStreamSynchronize(c->stream), "sync"));
  if (info_host) *info_host = hinfo;
  if (hinfo == GPX_INFO_TIMEOUT)
    return fail(c, GPX_TIMEOUT, "an in-launch hand-off of the factorisation timed out (spin limit)");
  if (hinfo != 0)
    return fail(c, GPX_NOT_PD, "Gram matrix not positive definite at pivot " + std::to_string(hinfo - 1));
  return GPX_OK;
}

gpx_status gpx_potrs_workspace_size(int64_t n, int64_t nrhs, size_t* bytes) {
  if (!bytes || n < 1 || nrhs < 1 || nrhs > GPX_MAX_RHS) return GPX_INVALID_ARG;
  *bytes = gpx::potrs_workspace_bytes(padded(n), nrhs, 1) + 256;
  return GPX_OK;
}

static gpx_status potrs_impl(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv,
                             const double* Y, int64_t ldy, int64_t nrhs, double const_mean, double* alpha,
                             int32_t* info, void* ws, size_t ws_bytes, bool ws_cleared, const double* z = nullptr);

gpx_status gpx_potrs_f64(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv, const double* Y,
                         int64_t ldy, int64_t nrhs, double const_mean, double* alpha, int32_t* info, void* ws,
                         size_t ws_bytes) {
  return potrs_impl(h, n, L, ldl, Dinv, Y, ldy, nrhs, const_mean, alpha, info, ws, ws_bytes, false);
}

static gpx_status potrs_impl(gpx_handle h, int64_t n, const double* L, int64_t ldl, const double* Dinv,
                             const double* Y, int64_t ldy, int64_t nrhs, double const_mean, double* alpha,
                             int32_t* info, void* ws, size_t ws_bytes, bool ws_cleared, const double* z) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_n(c, n));
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  GPX_NONNULL(c, L);
  GPX_NONNULL(c, Dinv);
  GPX_NONNULL(c, Y);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldl, npad, "L", true));
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  size_t need = 0;
  GPX_TRY(gpx_potrs_workspace_size(n, nrhs, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "potrs workspace too small");
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_potrs(c, (int)n, (int)npad, L, ldl, Dinv, Y, ldy, (int)nrhs, const_mean, alpha, info,
                                        align256(ws), gpx::Batch(), ws_cleared, z),
                   "potrs");
}

gpx_status gpx_fit_factor_workspace_size(int64_t n, int64_t nrhs, size_t* bytes) {
  return gpx_potrs_workspace_size(n, nrhs, bytes);
}

gpx_status gpx_fit_factor_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                              const double* Y, int64_t ldy, int64_t nrhs, double* K, int64_t ldk, double* Dinv,
                              double* alpha, int32_t* info, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  size_t need = 0;
  if (gpx_fit_factor_workspace_size(n, nrhs, &need) != GPX_OK)
    return fail(c, GPX_INVALID_ARG, "invalid n / nrhs for fit");
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "fit workspace too small");
  if (!info) return fail(c, GPX_INVALID_ARG, "info is NULL");
  if (!ws) return fail(c, GPX_INVALID_ARG, "ws is NULL");
  GPX_NONNULL(c, Y);
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  // the Gram launch also clears the triangular solve's hand-off granules (no memset dispatch)
  const int64_t npad = padded(n);
  GPX_TRY(gram_impl(h, p, n, X, ldx, K, ldk, info, align256(ws), gpx::potrs_clear_bytes(npad, nrhs, 1)));
  // the dataflow Cholesky also runs the forward substitution; the solve is then its backward half
  gpx::ForwardRhs fr;
  fr.Y = Y;
  fr.ldy = ldy;
  fr.nrhs = (int)nrhs;
  fr.n = (int)n;
  fr.mean = p->const_mean;
  fr.buf = reinterpret_cast<double*>(reinterpret_cast<char*>(align256(ws)) + gpx::potrs_forward_offset(npad, nrhs, 1));
  bool z_done = false;
  GPX_TRY(potrf_impl(h, n, K, ldk, Dinv, info, false, nullptr, 0, &fr, &z_done));
  return potrs_impl(h, n, K, ldk, Dinv, Y, ldy, nrhs, p->const_mean, alpha, info, ws, ws_bytes, true,
                    z_done ? fr.buf + npad * gpx::rhs_row((int)nrhs) : nullptr);
}

gpx_status gpx_append_workspace_size(int64_t n_old, int64_t n_new, int64_t nrhs, size_t* bytes) {
  if (!bytes || n_old < 1 || n_new <= n_old || nrhs < 1 || nrhs > GPX_MAX_RHS) return GPX_INVALID_ARG;
  size_t a = gpx::append_workspace_bytes(n_old, n_new), b = alpha_ws(padded(n_new), nrhs);
  *bytes = (a > b ? a : b) + 256;
  return GPX_OK;
}

gpx_status gpx_append_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n_old, int64_t n_new, const double* X,
                          int64_t ldx, const double* Y, int64_t ldy, int64_t nrhs, double* L, int64_t ldl,
                          double* Dinv, double* W, int64_t ldw, double* alpha, int32_t* info, void* ws,
                          size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_params(c, p));
  GPX_TRY(check_n(c, n_new));
  if (n_old < 1 || n_new <= n_old) return fail(c, GPX_INVALID_ARG, "append needs 1 <= n_old < n_new");
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, Y);
  GPX_NONNULL(c, L);
  GPX_NONNULL(c, Dinv);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, info);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n_new);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  GPX_TRY(check_ld(c, ldl, npad, "L", true));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  size_t need = 0;
  GPX_TRY(gpx_append_workspace_size(n_old, n_new, nrhs, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "append workspace too small");
  GPX_USE_DEVICE(c);
  double* base = align256(ws);
  GPX_TRY(hip_check(c, hipMemsetAsync(info, 0, sizeof(int32_t), c->stream), "memset info"));
  GPX_TRY(hip_check(c, gpx::launch_append(c, *p, (int)n_old, (int)n_new, X, ldx, L, ldl, Dinv, W, ldw, info, base),
                    "append"));
  double* zpart = base;
  double* z = zpart + (size_t)(npad / 128) * npad * nrhs;
  return hip_check(c, gpx::launch_alpha(c, (int)n_new, (int)npad, W, ldw, Y, ldy, (int)nrhs, p->const_mean, alpha,
                                        zpart, z),
                   "alpha");
}

static size_t fit_slice_bytes(int64_t npad, int64_t nrhs) {
  size_t a = trtri_ws(npad), b = alpha_ws(npad, nrhs);
  return ((a > b ? a : b) + 255) & ~(size_t)255;
}

// Bytes at the end of a batched fit's workspace for the per-problem constant means (Batch::means) of a fit whose
// problems carry their own kernel parameters.
static size_t means_bytes(int64_t batch) { return ((size_t)batch * 8 + 255) & ~(size_t)255; }

gpx_status gpx_fit_batched_workspace_size(int64_t n, int64_t nrhs, int64_t batch, size_t* bytes) {
  if (!bytes || n < 1 || nrhs < 1 || nrhs > GPX_MAX_RHS || batch < 1 || batch > 65535) return GPX_INVALID_ARG;
  *bytes = fit_slice_bytes(padded(n), nrhs) * (size_t)batch + means_bytes(batch) + 256;
  return GPX_OK;
}

gpx_status gpx_fit_factor_batched_workspace_size(int64_t n, int64_t nrhs, int64_t batch, size_t* bytes) {
  if (!bytes || n < 1 || nrhs < 1 || nrhs > GPX_MAX_RHS || batch < 1 || batch > 65535) return GPX_INVALID_ARG;
  *bytes = ((gpx::potrs_workspace_bytes(padded(n), nrhs, batch) + 255) & ~(size_t)255) + means_bytes(batch) + 256;
  return GPX_OK;
}

// Batched posterior updates; W == nullptr: factor + triangular solves only (gpx_fit_factor_batched_f64).  p points to
// one gpx_kernel_params (pstep = 0: shared by every problem) or to `batch` of them (pstep = 1, the
// gpx_fit_*_batched_params_f64 entry points).  Per-problem parameters that differ are served by one Gram launch per
// problem (its covariance parameters as kernel arguments; each launch fills the GPU from n ~ 1000 on) which also writes
// the problem's constant mean into the workspace for the solves; the Cholesky, the forward / backward solves and the
// inverse stay ONE set of launches over all problems (the latency-bound chain is what batching amortises).
static gpx_status fit_batched_impl(gpx_handle h, const gpx_kernel_params* p, int64_t pstep, int64_t batch, int64_t n,
                                   const double* X, int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy,
                                   int64_t stride_y, int64_t nrhs, double* K, int64_t ldk, int64_t stride_k,
                                   double* Dinv, int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w,
                                   double* alpha, int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  const bool inverse = W != nullptr;
  if (batch < 1 || batch > 65535) return fail(c, GPX_INVALID_ARG, "batch must be in [1, 65535]");
  GPX_NONNULL(c, p);
  bool shared = true;
  for (int64_t b = 0; b < (pstep ? batch : 1); ++b) {
    const gpx_status st = check_params(c, p + b);
    if (st != GPX_OK) return fail(c, st, "problem " + std::to_string(b) + ": " + c->last_error);
    if (p[b].d != p[0].d)
      return fail(c, GPX_INVALID_ARG, "every problem of a batched fit needs the same input dimension d");
    if (b > 0 && std::memcmp(p + b, p, sizeof(gpx_kernel_params)) != 0) shared = false;
  }
  GPX_TRY(check_n(c, n));
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, Y);
  GPX_NONNULL(c, K);
  GPX_NONNULL(c, Dinv);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, info);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  GPX_TRY(check_ld(c, ldk, npad, "K", true));
  if (inverse) GPX_TRY(check_ld(c, ldw, npad, "W", true));
  const int64_t nblk = npad / gpx::NB;
  if (batch > 1) {
    // outputs must not overlap (a stride of 0 would make the problems race on the same output); the read-only inputs
    // may be shared (stride 0: one X for the T outputs of a multi-output model) or interleaved (Y stride 1, ldy = T:
    // output column b of an n x T target matrix)
    if (stride_x < 0 || stride_y < 0) return fail(c, GPX_INVALID_ARG, "X / Y strides must be >= 0");
    if (stride_k < npad * ldk || (inverse && stride_w < npad * ldw) || stride_dinv < 2 * nblk * gpx::NB * gpx::NB ||
        stride_alpha < npad * nrhs)
      return fail(c, GPX_INVALID_ARG, "batch strides smaller than one problem");
    if ((stride_k | (inverse ? stride_w : 0) | stride_dinv) & 1)
      return fail(c, GPX_INVALID_ARG, "K/W/Dinv strides must be even");
  }
  size_t need = 0;
  if (inverse)
    GPX_TRY(gpx_fit_batched_workspace_size(n, nrhs, batch, &need));
  else
    GPX_TRY(gpx_fit_factor_batched_workspace_size(n, nrhs, batch, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "batched fit workspace too small");
  GPX_USE_DEVICE(c);
  gpx::Batch bt;
  bt.count = (int)batch;
  bt.x = stride_x;
  bt.y = stride_y;
  bt.k = stride_k;
  bt.dinv = stride_dinv;
  bt.w = stride_w;
  bt.alpha = stride_alpha;
  bt.ws = (int64_t)(fit_slice_bytes(npad, nrhs) / sizeof(double));
  double* slice = align256(ws);
  // per-problem constant means after the solves' part of the workspace
  const size_t solve_bytes = inverse ? fit_slice_bytes(npad, nrhs) * (size_t)batch
                                     : ((gpx::potrs_workspace_bytes(npad, nrhs, batch) + 255) & ~(size_t)255);
  double* means = shared ? nullptr : reinterpret_cast<double*>(reinterpret_cast<char*>(slice) + solve_bytes);
  bt.means = means;
  // the gram kernel clears info[0 .. batch) before the Cholesky (no separate memset dispatch), and in a factor-only fit
  // the triangular solve's hand-off granules of every problem
  void* zero = inverse ? nullptr : slice;
  const size_t zero_bytes = inverse ? 0 : gpx::potrs_clear_bytes(npad, nrhs, batch);
  if (shared) {
    GPX_TRY(hip_check(c, gpx::launch_gram(c, *p, (int)n, (int)npad, X, ldx, K, ldk, bt, 0, info, zero, zero_bytes),
                      "gram"));
  } else {
    for (int64_t b = 0; b < batch; ++b)
      GPX_TRY(hip_check(c, gpx::launch_gram(c, p[b], (int)n, (int)npad, X + b * stride_x, ldx, K + b * stride_k, ldk,
                                            gpx::Batch(), 0, info + b, b == 0 ? zero : nullptr, b == 0 ? zero_bytes : 0,
                                            means + b),
                        "gram"));
  }
  if (!inverse) {
    // factor + forward substitution (dataflow schedule), then the backward half of the solve
    gpx::ForwardRhs fr;
    fr.Y = Y;
    fr.ldy = ldy;
    fr.sy = stride_y;
    fr.nrhs = (int)nrhs;
    fr.n = (int)n;
    fr.mean = p->const_mean;
    fr.means = means;
    fr.buf = reinterpret_cast<double*>(reinterpret_cast<char*>(slice) + gpx::potrs_forward_offset(npad, nrhs, batch));
    bool z_done = false;
    GPX_TRY(hip_check(c, gpx::launch_potrf(c, (int)npad, K, ldk, Dinv, info, bt, nullptr, 0, &fr, &z_done), "potrf"));
    const int64_t nr = gpx::rhs_row((int)nrhs);
    return hip_check(c, gpx::launch_potrs(c, (int)n, (int)npad, K, ldk, Dinv, Y, ldy, (int)nrhs, p->const_mean, alpha,
                                          info, slice, bt, true, z_done ? fr.buf + npad * nr : nullptr, 2 * npad * nr),
                     "potrs");
  }
  GPX_TRY(hip_check(c, gpx::launch_potrf(c, (int)npad, K, ldk, Dinv, info, bt, W, ldw), "potrf"));
  GPX_TRY(hip_check(c, gpx::launch_trtri(c, (int)npad, K, ldk, Dinv, W, ldw, slice, bt, true), "trtri"));
  double* zpart = slice;
  double* z = zpart + (size_t)(npad / 128) * npad * nrhs;
  return hip_check(c, gpx::launch_alpha(c, (int)n, (int)npad, W, ldw, Y, ldy, (int)nrhs, p->const_mean, alpha, zpart, z,
                                        bt),
                   "alpha");
}

gpx_status gpx_fit_batched_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n, const double* X,
                               int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy, int64_t stride_y,
                               int64_t nrhs, double* K, int64_t ldk, int64_t stride_k, double* Dinv,
                               int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w, double* alpha,
                               int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_NONNULL(c, W);
  return fit_batched_impl(h, p, 0, batch, n, X, ldx, stride_x, Y, ldy, stride_y, nrhs, K, ldk, stride_k, Dinv,
                          stride_dinv, W, ldw, stride_w, alpha, stride_alpha, info, ws, ws_bytes);
}

gpx_status gpx_fit_factor_batched_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n,
                                      const double* X, int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy,
                                      int64_t stride_y, int64_t nrhs, double* K, int64_t ldk, int64_t stride_k,
                                      double* Dinv, int64_t stride_dinv, double* alpha, int64_t stride_alpha,
                                      int32_t* info, void* ws, size_t ws_bytes) {
  return fit_batched_impl(h, p, 0, batch, n, X, ldx, stride_x, Y, ldy, stride_y, nrhs, K, ldk, stride_k, Dinv,
                          stride_dinv, nullptr, 0, 0, alpha, stride_alpha, info, ws, ws_bytes);
}

gpx_status gpx_fit_batched_params_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n,
                                      const double* X, int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy,
                                      int64_t stride_y, int64_t nrhs, double* K, int64_t ldk, int64_t stride_k,
                                      double* Dinv, int64_t stride_dinv, double* W, int64_t ldw, int64_t stride_w,
                                      double* alpha, int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_NONNULL(c, W);
  return fit_batched_impl(h, p, 1, batch, n, X, ldx, stride_x, Y, ldy, stride_y, nrhs, K, ldk, stride_k, Dinv,
                          stride_dinv, W, ldw, stride_w, alpha, stride_alpha, info, ws, ws_bytes);
}

gpx_status gpx_fit_factor_batched_params_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n,
                                             const double* X, int64_t ldx, int64_t stride_x, const double* Y,
                                             int64_t ldy, int64_t stride_y, int64_t nrhs, double* K, int64_t ldk,
                                             int64_t stride_k, double* Dinv, int64_t stride_dinv, double* alpha,
                                             int64_t stride_alpha, int32_t* info, void* ws, size_t ws_bytes) {
  return fit_batched_impl(h, p, 1, batch, n, X, ldx, stride_x, Y, ldy, stride_y, nrhs, K, ldk, stride_k, Dinv,
                          stride_dinv, nullptr, 0, 0, alpha, stride_alpha, info, ws, ws_bytes);
}

gpx_status gpx_mll_workspace_size(int64_t n, size_t* bytes) {
  if (!bytes || n < 1 || n > ((int64_t)1 << 20)) return GPX_INVALID_ARG;
  *bytes = gpx::mll_workspace_bytes(padded(n)) + 256;
  return GPX_OK;
}

gpx_status gpx_mll_grad_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                            const double* Y, int64_t ldy, int64_t nrhs, const double* L, int64_t ldl,
                            const double* W, int64_t ldw, const double* alpha, double* out, void* ws,
                            size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_params(c, p));
  GPX_TRY(check_n(c, n));
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, Y);
  GPX_NONNULL(c, L);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, out);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldl, npad, "L", false));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  if (ws_bytes < gpx::mll_workspace_bytes(npad) + 256) return fail(c, GPX_INVALID_ARG, "mll workspace too small");
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_mll(c, *p, (int)n, (int)npad, X, ldx, Y, ldy, (int)nrhs, L, ldl, W, ldw, alpha, out,
                                      align256(ws)), "mll");
}

// T independent problems (one gpx_kernel_params each): the fitted state of problem b at base + b * stride_*, out at
// out + b * GPX_MLL_NOUT.  One gradient pass per problem on the stream, the workspace of gpx_mll_workspace_size reused by
// each (the pass fills the GPU from n ~ 1000 on; the per-problem parameters enter the contraction's dK/dtheta epilogue).
gpx_status gpx_mll_grad_batched_f64(gpx_handle h, const gpx_kernel_params* p, int64_t batch, int64_t n, const double* X,
                                    int64_t ldx, int64_t stride_x, const double* Y, int64_t ldy, int64_t stride_y,
                                    int64_t nrhs, const double* L, int64_t ldl, int64_t stride_l, const double* W,
                                    int64_t ldw, int64_t stride_w, const double* alpha, int64_t stride_alpha,
                                    double* out, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  if (batch < 1 || batch > 65535) return fail(c, GPX_INVALID_ARG, "batch must be in [1, 65535]");
  GPX_NONNULL(c, p);
  for (int64_t b = 0; b < batch; ++b) {
    const gpx_status st = check_params(c, p + b);
    if (st != GPX_OK) return fail(c, st, "problem " + std::to_string(b) + ": " + c->last_error);
  }
  GPX_TRY(check_n(c, n));
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, Y);
  GPX_NONNULL(c, L);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, out);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  for (int64_t b = 0; b < batch; ++b) GPX_TRY(check_ld(c, ldx, p[b].d, "X", false));
  GPX_TRY(check_ld(c, ldl, npad, "L", false));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  GPX_TRY(check_ld(c, ldy, nrhs, "Y", false));
  if (batch > 1 && (stride_x < 0 || stride_y < 0 || stride_l < npad * ldl || stride_w < npad * ldw ||
                    stride_alpha < npad * nrhs))
    return fail(c, GPX_INVALID_ARG, "batch strides smaller than one problem (X / Y: >= 0)");
  if (ws_bytes < gpx::mll_workspace_bytes(npad) + 256) return fail(c, GPX_INVALID_ARG, "mll workspace too small");
  GPX_USE_DEVICE(c);
  for (int64_t b = 0; b < batch; ++b)
    GPX_TRY(hip_check(c, gpx::launch_mll(c, p[b], (int)n, (int)npad, X + b * stride_x, ldx, Y + b * stride_y, ldy,
                                         (int)nrhs, L + b * stride_l, ldl, W + b * stride_w, ldw, alpha + b * stride_alpha,
                                         out + b * GPX_MLL_NOUT, align256(ws)),
                      "mll"));
  return GPX_OK;
}

gpx_status gpx_moments_grad_workspace_size(int64_t n, int64_t m, size_t* bytes) {
  if (!bytes || n < 1 || m < 1 || m > GPX_MAX_GRAD_CANDIDATES) return GPX_INVALID_ARG;
  *bytes = gpx::moments_grad_ws_doubles((int)padded(n), (int)m) * sizeof(double) + 256;
  return GPX_OK;
}

gpx_status gpx_moments_grad_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                                const double* W, int64_t ldw, const double* alpha, const double* Xs, int64_t m,
                                int64_t q, int64_t ldxs, double* mean, double* dmean, double* cov, double* dcov,
                                void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_params(c, p));
  GPX_TRY(check_n(c, n));
  if (m < 1 || m > GPX_MAX_GRAD_CANDIDATES) return fail(c, GPX_INVALID_ARG, "m must be in [1, GPX_MAX_GRAD_CANDIDATES]");
  if (q < 1 || q > GPX_MAX_Q || m % q != 0) return fail(c, GPX_INVALID_ARG, "q must be in [1, GPX_MAX_Q] and divide m");
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, Xs);
  GPX_NONNULL(c, mean);
  GPX_NONNULL(c, dmean);
  GPX_NONNULL(c, cov);
  GPX_NONNULL(c, dcov);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  GPX_TRY(check_ld(c, ldxs, p->d, "Xs", false));
  size_t need = 0;
  GPX_TRY(gpx_moments_grad_workspace_size(n, m, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "moments_grad workspace too small");
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_moments_grad(c, *p, (int)n, (int)npad, X, ldx, W, ldw, alpha, Xs, ldxs, (int)m,
                                               (int)q, mean, dmean, cov, dcov, align256(ws)),
                   "moments_grad");
}

gpx_status gpx_sweep_workspace_size(int64_t n, int64_t nrhs, int64_t m, size_t* bytes) {
  if (!bytes || n < 1 || m < 1 || nrhs < 1 || nrhs > GPX_MAX_RHS) return GPX_INVALID_ARG;
  *bytes = gpx::sweep_workspace_bytes(padded(n), nrhs, m);
  return GPX_OK;
}

static gpx_status carve_sweep(Context* c, int64_t npad, int64_t nrhs, int64_t m, void* ws, size_t ws_bytes,
                              gpx::SweepBuffers* b) {
  if (!ws) return fail(c, GPX_INVALID_ARG, "sweep workspace is NULL");
  if (ws_bytes < gpx::sweep_workspace_bytes(npad, nrhs, m)) return fail(c, GPX_INVALID_ARG, "sweep workspace too small");
  const int64_t C = gpx::sweep_chunk_size(npad, m);
  double* base = align256(ws);
  b->chunk = C;
  b->kstar = base;
  b->mu_part = b->kstar + (size_t)npad * C;
  b->ss_part = b->mu_part + (size_t)(npad / gpx::NB) * nrhs * C;
  b->rec_val = b->ss_part + (size_t)(npad / 128) * C;
  const int64_t nrec = (m + 255) / 256 + 1;
  b->rec_idx = reinterpret_cast<int64_t*>(b->rec_val + nrec);
  return GPX_OK;
}

gpx_status gpx_posterior_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                             const double* W, int64_t ldw, const double* alpha, int64_t nrhs, const double* Xs,
                             int64_t m, int64_t ldxs, const double* y_mean_host, const double* y_scale_host,
                             double* mean_out, int64_t ldmean, double* var_out, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_params(c, p));
  GPX_TRY(check_n(c, n));
  if (nrhs < 1 || nrhs > GPX_MAX_RHS) return fail(c, GPX_INVALID_ARG, "nrhs must be in [1, 8]");
  if (m < 1) return fail(c, GPX_INVALID_ARG, "m must be >= 1");
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, Xs);
  GPX_NONNULL(c, mean_out);
  GPX_NONNULL(c, var_out);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  GPX_TRY(check_ld(c, ldxs, p->d, "Xs", false));
  GPX_TRY(check_ld(c, ldmean, nrhs, "mean", false));
  gpx::SweepBuffers b;
  GPX_TRY(carve_sweep(c, npad, nrhs, m, ws, ws_bytes, &b));
  GPX_USE_DEVICE(c);
  for (int64_t s = 0; s < m; s += b.chunk) {
    const int64_t mc = (m - s) < b.chunk ? (m - s) : b.chunk;
    GPX_TRY(hip_check(c,
                      gpx::launch_sweep_chunk(c, *p, (int)n, (int)npad, X, ldx, W, ldw, alpha, (int)nrhs, Xs + s * ldxs,
                                              ldxs, mc, b, 0, nullptr, y_mean_host, y_scale_host,
                                              mean_out + s * ldmean, ldmean, var_out + s, nullptr, 0, 0),
                      "posterior"));
  }
  return GPX_OK;
}

gpx_status gpx_acquire_argmax_f64(gpx_handle h, const gpx_kernel_params* p, int64_t n, const double* X, int64_t ldx,
                                  const double* W, int64_t ldw, const double* alpha, const double* Xs, int64_t m,
                                  int64_t ldxs, const gpx_acq_params* a, int64_t index_offset, double* best_val,
                                  int64_t* best_idx, double* scores_out, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_params(c, p));
  GPX_TRY(check_n(c, n));
  if (m < 1) return fail(c, GPX_INVALID_ARG, "m must be >= 1");
  if (!a) return fail(c, GPX_INVALID_ARG, "acquisition params pointer is NULL");
  if (a->kind < GPX_ACQ_EI || a->kind > GPX_ACQ_VARIANCE) return fail(c, GPX_INVALID_ARG, "unknown acquisition kind");
  if (a->reserved != 0) return fail(c, GPX_INVALID_ARG, "gpx_acq_params.reserved must be 0");
  if (!(a->y_scale > 0.0)) return fail(c, GPX_INVALID_ARG, "y_scale must be positive");
  if (a->kind == GPX_ACQ_UCB && !(a->beta >= 0.0)) return fail(c, GPX_INVALID_ARG, "UCB beta must be >= 0");
  if (index_offset < 0) return fail(c, GPX_INVALID_ARG, "index_offset must be >= 0");
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, Xs);
  GPX_NONNULL(c, best_val);
  GPX_NONNULL(c, best_idx);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldw, npad, "W", true));
  GPX_TRY(check_ld(c, ldxs, p->d, "Xs", false));
  gpx::SweepBuffers b;
  GPX_TRY(carve_sweep(c, npad, 1, m, ws, ws_bytes, &b));
  GPX_USE_DEVICE(c);
  int64_t rec = 0;
  for (int64_t s = 0; s < m; s += b.chunk) {
    const int64_t mc = (m - s) < b.chunk ? (m - s) : b.chunk;
    GPX_TRY(hip_check(c,
                      gpx::launch_sweep_chunk(c, *p, (int)n, (int)npad, X, ldx, W, ldw, alpha, 1, Xs + s * ldxs, ldxs,
                                              mc, b, 1, a, nullptr, nullptr, nullptr, 0, nullptr,
                                              scores_out ? scores_out + s : nullptr, rec, index_offset + s),
                      "acquire"));
    rec += (mc + 255) / 256;
  }
  return hip_check(c, gpx::launch_argmax_final(c, b.rec_val, b.rec_idx, rec, best_val, best_idx), "argmax");
}

gpx_status gpx_sweep_multi_workspace_size(int64_t n, int64_t m, size_t* bytes) {
  if (!bytes || n < 1 || m < 1) return GPX_INVALID_ARG;
  const int64_t npad = padded(n);
  *bytes = ((gpx::sweep_workspace_bytes(npad, 1, m) + 255) & ~(size_t)255) +
           2 * (size_t)gpx::sweep_chunk_size(npad, m) * sizeof(double) + 256;
  return GPX_OK;
}

gpx_status gpx_acquire_argmax_multi_f64(gpx_handle h, const gpx_kernel_params* p, int64_t T, int64_t n, const double* X,
                                        int64_t ldx, const double* const* W_host, const int64_t* ldw_host,
                                        const double* const* alpha_host, const double* weights_host,
                                        const double* y_mean_host, const double* y_scale_host, const double* Xs,
                                        int64_t m, int64_t ldxs, const gpx_acq_params* a, int64_t index_offset,
                                        double* best_val, int64_t* best_idx, double* scores_out, void* ws,
                                        size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  if (T < 1 || T > 64) return fail(c, GPX_INVALID_ARG, "T (outputs) must be in [1, 64]");
  GPX_NONNULL(c, p);
  GPX_NONNULL(c, weights_host);
  for (int64_t t = 0; t < T; ++t) {
    const gpx_status st = check_params(c, p + t);
    if (st != GPX_OK) return fail(c, st, "output " + std::to_string(t) + ": " + c->last_error);
    if (p[t].d != p[0].d) return fail(c, GPX_INVALID_ARG, "every output needs the same input dimension d");
    if (!std::isfinite(weights_host[t])) return fail(c, GPX_INVALID_ARG, "objective weights must be finite");
    if (y_scale_host && !(y_scale_host[t] > 0.0)) return fail(c, GPX_INVALID_ARG, "y_scale must be positive");
  }
  GPX_TRY(check_n(c, n));
  if (m < 1) return fail(c, GPX_INVALID_ARG, "m must be >= 1");
  if (!a) return fail(c, GPX_INVALID_ARG, "acquisition params pointer is NULL");
  if (a->kind < GPX_ACQ_EI || a->kind > GPX_ACQ_VARIANCE) return fail(c, GPX_INVALID_ARG, "unknown acquisition kind");
  if (a->reserved != 0) return fail(c, GPX_INVALID_ARG, "gpx_acq_params.reserved must be 0");
  if (a->kind == GPX_ACQ_UCB && !(a->beta >= 0.0)) return fail(c, GPX_INVALID_ARG, "UCB beta must be >= 0");
  if (index_offset < 0) return fail(c, GPX_INVALID_ARG, "index_offset must be >= 0");
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, W_host);
  GPX_NONNULL(c, ldw_host);
  GPX_NONNULL(c, alpha_host);
  GPX_NONNULL(c, Xs);
  GPX_NONNULL(c, best_val);
  GPX_NONNULL(c, best_idx);
  GPX_NONNULL(c, ws);
  const int64_t npad = padded(n);
  GPX_TRY(check_ld(c, ldx, p->d, "X", false));
  GPX_TRY(check_ld(c, ldxs, p->d, "Xs", false));
  for (int64_t t = 0; t < T; ++t) {
    if (!W_host[t] || !alpha_host[t]) return fail(c, GPX_INVALID_ARG, "W / alpha of output " + std::to_string(t) + " is NULL");
    GPX_TRY(check_ld(c, ldw_host[t], npad, "W", true));
  }
  size_t need = 0;
  GPX_TRY(gpx_sweep_multi_workspace_size(n, m, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "multi-output sweep workspace too small");
  gpx::SweepBuffers b;
  const size_t sweep_bytes = (gpx::sweep_workspace_bytes(npad, 1, m) + 255) & ~(size_t)255;
  GPX_TRY(carve_sweep(c, npad, 1, m, ws, sweep_bytes, &b));
  GPX_USE_DEVICE(c);
  gpx::MultiOutput mo;
  mo.acc_mu = reinterpret_cast<double*>(reinterpret_cast<char*>(align256(ws)) + sweep_bytes);
  mo.acc_var = mo.acc_mu + b.chunk;
  int64_t rec = 0;
  for (int64_t s = 0; s < m; s += b.chunk) {
    const int64_t mc = (m - s) < b.chunk ? (m - s) : b.chunk;
    for (int64_t t = 0; t < T; ++t) {
      mo.weight = weights_host[t];
      mo.y_mean = y_mean_host ? y_mean_host[t] : 0.0;
      mo.y_scale = y_scale_host ? y_scale_host[t] : 1.0;
      mo.first = t == 0;
      GPX_TRY(hip_check(c,
                        gpx::launch_sweep_chunk(c, p[t], (int)n, (int)npad, X, ldx, W_host[t], ldw_host[t],
                                                alpha_host[t], 1, Xs + s * ldxs, ldxs, mc, b, 1, a, nullptr,
                                                nullptr, nullptr, 0, nullptr, nullptr, 0, 0, &mo),
                        "acquire (multi-output)"));
    }
    GPX_TRY(hip_check(c, gpx::launch_multi_score(c, mo, *a, mc, scores_out ? scores_out + s : nullptr, b.rec_val + rec,
                                                 b.rec_idx + rec, index_offset + s),
                      "acquire (multi-output score)"));
    rec += (mc + 255) / 256;
  }
  return hip_check(c, gpx::launch_argmax_final(c, b.rec_val, b.rec_idx, rec, best_val, best_idx), "argmax");
}

gpx_status gpx_argmax_combine_f64(gpx_handle h, const double* vals, const int64_t* idx, int64_t count,
                                  double* best_val, int64_t* best_idx) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  if (count < 1) return fail(c, GPX_INVALID_ARG, "count must be >= 1");
  GPX_NONNULL(c, vals);
  GPX_NONNULL(c, idx);
  GPX_NONNULL(c, best_val);
  GPX_NONNULL(c, best_idx);
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_argmax_final(c, vals, idx, count, best_val, best_idx), "argmax_combine");
}

// ---- SVGP predictive + pool-scan selection --------------------------------------
namespace {
struct SvgpPrepLayout {
  size_t L, dinv, slice, spad, mpad, total;  // byte offsets / sizes per task (256-aligned)
};
size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }
SvgpPrepLayout svgp_prep_layout(int64_t Mpad) {
  SvgpPrepLayout l;
  const size_t L = al256((size_t)Mpad * Mpad * 8);
  const size_t D = al256((size_t)2 * (Mpad / gpx::NB) * gpx::NB * gpx::NB * 8);
  const size_t fs = al256(trtri_ws(Mpad) > alpha_ws(Mpad, 1) ? trtri_ws(Mpad) : alpha_ws(Mpad, 1));
  l.L = 0;
  l.dinv = L;
  l.slice = L + D;
  l.spad = L + D + fs;
  l.mpad = l.spad + L;
  l.total = l.mpad + al256((size_t)Mpad * 8);
  return l;
}
gpx_status check_svgp(Context* c, const gpx_kernel_params* p, int64_t ntask, int64_t M) {
  if (ntask < 1 || ntask > 64) return fail(c, GPX_INVALID_ARG, "ntask must be in [1, 64]");
  if (M < 1 || M > 65536) return fail(c, GPX_INVALID_ARG, "number of inducing points must be in [1, 65536]");
  if (!p) return fail(c, GPX_INVALID_ARG, "kernel params pointer is NULL");
  for (int64_t t = 0; t < ntask; ++t) {
    GPX_TRY(check_params(c, p + t));
    if (p[t].d != p[0].d) return fail(c, GPX_INVALID_ARG, "all tasks must share the input dimension");
  }
  return GPX_OK;
}
}  // namespace

gpx_status gpx_svgp_prepare_workspace_size(int64_t M, int64_t ntask, size_t* bytes) {
  if (!bytes || M < 1 || ntask < 1) return GPX_INVALID_ARG;
  *bytes = svgp_prep_layout(padded(M)).total * (size_t)ntask + 256;
  return GPX_OK;
}

gpx_status gpx_svgp_prepare_f64(gpx_handle h, const gpx_kernel_params* p, int64_t ntask, int64_t M, double jitter,
                                const double* Z, int64_t ldz, int64_t stride_z, const double* vmean,
                                int64_t stride_m, const double* vchol, int64_t ldc, int64_t stride_c, double* W,
                                double* W2, double* alpha, int32_t* info, void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_svgp(c, p, ntask, M));
  GPX_NONNULL(c, Z);
  GPX_NONNULL(c, vmean);
  GPX_NONNULL(c, vchol);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, W2);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, info);
  GPX_NONNULL(c, ws);
  if (!(jitter >= 0.0)) return fail(c, GPX_INVALID_ARG, "jitter must be non-negative");
  GPX_TRY(check_ld(c, ldz, p[0].d, "Z", false));
  GPX_TRY(check_ld(c, ldc, M, "chol_variational_covar", false));
  if (ntask > 1 && (stride_z < M * ldz || stride_m < M || stride_c < M * ldc))
    return fail(c, GPX_INVALID_ARG, "task strides smaller than one task");
  const int64_t Mpad = padded(M);
  size_t need = 0;
  GPX_TRY(gpx_svgp_prepare_workspace_size(M, ntask, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "svgp prepare workspace too small");
  GPX_USE_DEVICE(c);
  const SvgpPrepLayout lay = svgp_prep_layout(Mpad);
  char* base = reinterpret_cast<char*>(align256(ws));
  auto at = [&](int64_t t, size_t off) { return reinterpret_cast<double*>(base + lay.total * t + off); };
  const int64_t tstride = (int64_t)(lay.total / sizeof(double));  // elements between tasks in the workspace
  GPX_TRY(hip_check(c, hipMemsetAsync(info, 0, sizeof(int32_t) * ntask, c->stream), "memset info"));
  // K_ZZ + jitter I per task (the hyperparameters differ per task; the likelihood noise is not part of K_ZZ)
  for (int64_t t = 0; t < ntask; ++t) {
    gpx_kernel_params q = p[t];
    q.noise = 0.0;
    q.jitter = jitter;
    GPX_TRY(hip_check(c, gpx::launch_gram(c, q, (int)M, (int)Mpad, Z + t * stride_z, ldz, at(t, lay.L), Mpad), "gram"));
  }
  gpx::Batch bt;
  bt.count = (int)ntask;
  bt.k = tstride;
  bt.dinv = tstride;
  bt.ws = tstride;
  bt.w = Mpad * Mpad;
  GPX_TRY(hip_check(c, gpx::launch_potrf(c, (int)Mpad, at(0, lay.L), Mpad, at(0, lay.dinv), info, bt), "potrf"));
  GPX_TRY(hip_check(c, gpx::launch_trtri(c, (int)Mpad, at(0, lay.L), Mpad, at(0, lay.dinv), W, Mpad, at(0, lay.slice),
                                         bt),
                    "trtri"));
  // zero-padded m and S = tril(chol) in the workspace, then alpha' = W m and W2 = W S
  GPX_TRY(hip_check(c, gpx::launch_svgp_pad(c, (int)ntask, (int)M, (int)Mpad, vmean, stride_m, vchol, ldc, stride_c,
                                            at(0, lay.mpad), at(0, lay.spad), tstride),
                    "svgp pad"));
  gpx::Batch tv;
  tv.count = (int)ntask;
  tv.w = Mpad * Mpad;
  tv.y = tstride;
  tv.alpha = Mpad;
  GPX_TRY(hip_check(c, gpx::launch_trmv_upper(c, (int)Mpad, W, Mpad, at(0, lay.mpad), alpha, tv), "alpha'"));
  return hip_check(c, gpx::launch_svgp_w2(c, (int)ntask, (int)Mpad, W, at(0, lay.spad), tstride, W2), "svgp W2");
}

gpx_status gpx_svgp_predict_workspace_size(int64_t M, int64_t m, size_t* bytes) {
  if (!bytes || M < 1 || m < 1) return GPX_INVALID_ARG;
  const int64_t Mpad = padded(M);
  const int64_t C = gpx::sweep_chunk_size(Mpad, m);
  *bytes = gpx::sweep_workspace_bytes(Mpad, 1, m) + (size_t)(Mpad / 128) * C * 8 + 512;
  return GPX_OK;
}

gpx_status gpx_svgp_predict_f64(gpx_handle h, const gpx_kernel_params* p, int64_t ntask, int64_t M, const double* Z,
                                int64_t ldz, int64_t stride_z, const double* W, const double* W2, const double* alpha,
                                const double* Xs, int64_t m, int64_t ldxs, double min_var, double* mean_out,
                                int64_t ldmean, double* var_out, int64_t ldvar, double* score_out, void* ws,
                                size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_TRY(check_svgp(c, p, ntask, M));
  GPX_NONNULL(c, Z);
  GPX_NONNULL(c, W);
  GPX_NONNULL(c, W2);
  GPX_NONNULL(c, alpha);
  GPX_NONNULL(c, Xs);
  GPX_NONNULL(c, ws);
  if (m < 1) return fail(c, GPX_INVALID_ARG, "m must be >= 1");
  if (!mean_out && !var_out && !score_out) return fail(c, GPX_INVALID_ARG, "no output requested");
  if (!(min_var >= 0.0)) return fail(c, GPX_INVALID_ARG, "min_var must be non-negative");
  GPX_TRY(check_ld(c, ldz, p[0].d, "Z", false));
  GPX_TRY(check_ld(c, ldxs, p[0].d, "Xs", false));
  if (mean_out) GPX_TRY(check_ld(c, ldmean, ntask, "mean", false));
  if (var_out) GPX_TRY(check_ld(c, ldvar, ntask, "var", false));
  if (ntask > 1 && stride_z < M * ldz) return fail(c, GPX_INVALID_ARG, "task stride of Z smaller than one task");
  const int64_t Mpad = padded(M);
  size_t need = 0;
  GPX_TRY(gpx_svgp_predict_workspace_size(M, m, &need));
  if (ws_bytes < need) return fail(c, GPX_INVALID_ARG, "svgp predict workspace too small");
  gpx::SweepBuffers b;
  GPX_TRY(carve_sweep(c, Mpad, 1, m, ws, ws_bytes, &b));
  double* ss2 = reinterpret_cast<double*>(((uintptr_t)(b.rec_idx + (m + 255) / 256 + 1) + 255) & ~(uintptr_t)255);
  GPX_USE_DEVICE(c);
  for (int64_t s = 0; s < m; s += b.chunk) {
    const int64_t mc = (m - s) < b.chunk ? (m - s) : b.chunk;
    for (int64_t t = 0; t < ntask; ++t) {
      GPX_TRY(hip_check(c,
                        gpx::launch_svgp_chunk(c, p[t], min_var, (int)t, (int)M, (int)Mpad, Z + t * stride_z, ldz,
                                               W + t * Mpad * Mpad, W2 + t * Mpad * Mpad, Mpad, alpha + t * Mpad,
                                               Xs + s * ldxs, ldxs, mc, b, ss2, mean_out ? mean_out + s * ldmean : nullptr,
                                               ldmean, var_out ? var_out + s * ldvar : nullptr, ldvar,
                                               score_out ? score_out + s : nullptr),
                        "svgp predict"));
    }
  }
  return GPX_OK;
}

gpx_status gpx_topk_workspace_size(int64_t m, size_t* bytes) {
  if (!bytes || m < 1 || m > ((int64_t)1 << 30)) return GPX_INVALID_ARG;
  *bytes = gpx::topk_workspace_bytes(m);
  return GPX_OK;
}

gpx_status gpx_topk_f64(gpx_handle h, const double* scores, int64_t m, int64_t k, int64_t* idx_out, double* val_out,
                        void* ws, size_t ws_bytes) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_NONNULL(c, scores);
  GPX_NONNULL(c, idx_out);
  GPX_NONNULL(c, ws);
  if (m < 1 || m > ((int64_t)1 << 30)) return fail(c, GPX_INVALID_ARG, "m must be in [1, 2^30]");
  if (k < 1 || k > m) return fail(c, GPX_INVALID_ARG, "k must be in [1, m]");
  if (ws_bytes < gpx::topk_workspace_bytes(m)) return fail(c, GPX_INVALID_ARG, "topk workspace too small");
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_topk(c, scores, m, k, idx_out, val_out, ws, ws_bytes), "topk");
}

gpx_status gpx_fps_f64(gpx_handle h, const double* X, int64_t m, int64_t d, int64_t ldx, int64_t k, int64_t start,
                       int64_t* idx_out) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  GPX_NONNULL(c, X);
  GPX_NONNULL(c, idx_out);
  if (m < 1 || m > 32 * 1024) return fail(c, GPX_INVALID_ARG, "fps supports 1 <= m <= 32768 points");
  if (d < 1 || d > GPX_MAX_DIM) return fail(c, GPX_INVALID_ARG, "d must be in [1, 32]");
  if (k < 1 || k > m) return fail(c, GPX_INVALID_ARG, "k must be in [1, m]");
  if (start < 0 || start >= m) return fail(c, GPX_INVALID_ARG, "start index outside [0, m)");
  GPX_TRY(check_ld(c, ldx, d, "X", false));
  GPX_USE_DEVICE(c);
  return hip_check(c, gpx::launch_fps(c, X, m, (int)d, ldx, k, start, idx_out), "fps");
}

gpx_status gpx_timing_enable(gpx_handle h, int32_t mask) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  c->timing_mask = mask;
  return GPX_OK;
}

gpx_status gpx_timing_reset(gpx_handle h) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  if (!c->pending.empty()) (void)hipStreamSynchronize(c->stream);
  for (auto& pt : c->pending) {
    c->free_events.push_back(pt.start);
    c->free_events.push_back(pt.stop);
  }
  c->pending.clear();
  for (int t = 0; t < GPX_TIMER_COUNT; ++t) {
    c->timer_ms[t] = 0.0;
    c->timer_launches[t] = 0;
  }
  return GPX_OK;
}

gpx_status gpx_timing_query(gpx_handle h, int32_t timer, double* total_ms_host, int64_t* launches_host) {
  Context* c = reinterpret_cast<Context*>(h);
  if (!c) return GPX_INVALID_ARG;
  if (timer < 0 || timer >= GPX_TIMER_COUNT) return fail(c, GPX_INVALID_ARG, "unknown timer");
  if (!c->pending.empty()) {
    GPX_TRY(hip_check(c, hipStreamSynchronize(c->stream), "timing sync"));
    for (auto& pt : c->pending) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, pt.start, pt.stop) == hipSuccess) {
        c->timer_ms[pt.timer] += ms;
        c->timer_launches[pt.timer] += 1;
      }
      c->free_events.push_back(pt.start);
      c->free_events.push_back(pt.stop);
    }
    c->pending.clear();
  }
  if (total_ms_host) *total_ms_host = c->timer_ms[timer];
  if (launches_host) *launches_host = c->timer_launches[timer];
  return GPX_OK;
}

}  // extern "C"
