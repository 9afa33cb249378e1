// Cross-GPU exchange of the selection records over RCCL (SURVEY §8b `gpx_allreduce_argmax`, §8e): one process per
// GPU, every rank holds a (fp64 value, int64 global index) record; an RCCL all-gather of the 16-byte records over
// xGMI, then the deterministic argmax_combine kernel (max value, lowest index among ties, NaN never wins) on the
// handle's stream.  RCCL has no MAXLOC reduction, hence gather + local combine (every rank computes the same result).
// The communicator is bootstrapped from an ncclUniqueId that rank 0 creates and the host side broadcasts (the
// Python binding uses torch.distributed for that: bayesianoptimizer_amd/dist.py, RCCLArgmaxExchange).
#include <rccl/rccl.h>
#include <cstring>
#include <string>
#include "gpx_internal.h"

struct gpx_comm_s {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
};

namespace {
gpx_status rccl_fail(gpx::Context* c, ncclResult_t r, const char* where) {
  if (c) c->last_error = std::string(where) + ": " + ncclGetErrorString(r);
  return GPX_RCCL_ERROR;
}
}  // namespace

extern "C" {

gpx_status gpx_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return GPX_INVALID_ARG;
  static_assert(sizeof(ncclUniqueId) == GPX_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return GPX_RCCL_ERROR;
  memcpy(id_out, &id, sizeof(id));
  return GPX_OK;
}

gpx_status gpx_comm_init(gpx_handle h, const uint8_t* id, int32_t nranks, int32_t rank, gpx_comm* out) {
  gpx::Context* c = reinterpret_cast<gpx::Context*>(h);
  if (!c || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return GPX_INVALID_ARG;
  *out = nullptr;
  gpx::DeviceScope dev(c->device);  // RCCL binds the communicator to the current device
  if (dev.err != hipSuccess) return GPX_HIP_ERROR;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  gpx_comm cm = new gpx_comm_s();
  const ncclResult_t r = ncclCommInitRank(&cm->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete cm;
    return rccl_fail(c, r, "ncclCommInitRank");
  }
  cm->nranks = nranks;
  cm->rank = rank;
  *out = cm;
  return GPX_OK;
}

gpx_status gpx_comm_destroy(gpx_comm cm) {
  if (!cm) return GPX_INVALID_ARG;
  const ncclResult_t r = ncclCommDestroy(cm->comm);
  delete cm;
  return r == ncclSuccess ? GPX_OK : GPX_RCCL_ERROR;
}

// workspace: the 16-byte send record, then the nranks gathered records (256-aligned)
static size_t exchange_ws_bytes(int nranks) { return 256 + 256 + (size_t)nranks * 16; }

gpx_status gpx_allreduce_argmax_workspace_size(gpx_comm cm, size_t* bytes) {
  if (!cm || !bytes) return GPX_INVALID_ARG;
  *bytes = exchange_ws_bytes(cm->nranks);
  return GPX_OK;
}

gpx_status gpx_allreduce_argmax(gpx_handle h, gpx_comm cm, double* best_val, int64_t* best_idx, void* ws,
                                size_t ws_bytes) {
  gpx::Context* c = reinterpret_cast<gpx::Context*>(h);
  if (!c || !cm) return GPX_INVALID_ARG;
  if (!best_val || !best_idx || !ws) {
    c->last_error = "best_val / best_idx / ws is NULL";
    return GPX_INVALID_ARG;
  }
  if (ws_bytes < exchange_ws_bytes(cm->nranks)) {
    c->last_error = "allreduce_argmax workspace too small";
    return GPX_INVALID_ARG;
  }
  gpx::DeviceScope dev(c->device);
  if (dev.err != hipSuccess) {
    c->last_error = "hipSetDevice failed";
    return GPX_HIP_ERROR;
  }
  // one record {fp64 value, int64 index} per rank, ONE all-gather of 16 bytes each, then the deterministic combine
  uintptr_t u = (reinterpret_cast<uintptr_t>(ws) + 255) & ~(uintptr_t)255;
  int64_t* send = reinterpret_cast<int64_t*>(u);
  int64_t* recv = send + 32;  // 256 bytes further
  hipError_t e = gpx::launch_record_pack(c, best_val, best_idx, send);
  if (e != hipSuccess) {
    c->last_error = std::string("record_pack: ") + hipGetErrorString(e);
    return GPX_HIP_ERROR;
  }
  const ncclResult_t r = ncclAllGather(send, recv, 2, ncclInt64, cm->comm, c->stream);
  if (r != ncclSuccess) return rccl_fail(c, r, "ncclAllGather");
  e = gpx::launch_argmax_records(c, recv, cm->nranks, best_val, best_idx);
  if (e != hipSuccess) {
    c->last_error = std::string("argmax_combine: ") + hipGetErrorString(e);
    return GPX_HIP_ERROR;
  }
  return GPX_OK;
}

}  // extern "C"
