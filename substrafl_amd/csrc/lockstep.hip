// lockstep.hip -- native executor of the client-sharded lockstep schedules (substrafl_amd/lockstep.py)
// over RCCL, behind the C ABI of include/fedagg.h (fedagg_comm_*, fedagg_lockstep_execute).
//
// The Python schedule builder computes, once per (M, K, G, rank), every run (one chain-kernel
// launch over a client block) and every point-to-point message of every exchange group; this
// file issues them: for t = 0, 1, ...
//   group t  on the communicator's stream, after the compute stream's work so far (step t - 1):
//            ncclGroupStart; the group's ncclSend / ncclRecv; ncclGroupEnd
//   step t   on the caller's (compute) stream, after group t - 1: the runs' chain kernels
// then the optional in-place ncclReduce of the numel == 1 product workspace onto the root.
// ONE host thread, ONE communicator, and group t of every rank pairs only with group t of its
// peers -- deadlock-free whatever the hardware queues interleave (lockstep.py's module docstring).
// Two HIP streams per rank: the caller's and the communicator's (<= GPU_MAX_HW_QUEUES = 4).
//
// RCCL is loaded at run time (dlopen): the process's already-loaded librccl when there is one
// (torch bundles its own), else ROCm's -- so a process never holds two RCCL instances.

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fedagg.h"

namespace {

thread_local char g_lerr[512] = "";

int lfail(int code, const char* msg, const char* detail = "") {
  snprintf(g_lerr, sizeof(g_lerr), "%s%s", msg, detail);
  return code;
}

struct Rccl {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclReduce) Reduce = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

int rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl.h) return FEDAGG_OK;
  const char* p = (path && *path) ? path : "librccl.so.1";
  void* h = dlopen(p, RTLD_NOW | RTLD_NOLOAD);  // the instance already in the process, if any
  if (!h) h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
  if (!h) return lfail(FEDAGG_EINVAL, "fedagg_comm: cannot load RCCL: ", dlerror());
  Rccl r;
  r.h = h;
#define SYM(f)                                                                        \
  r.f = reinterpret_cast<decltype(r.f)>(dlsym(h, "nccl" #f));                         \
  if (!r.f) return lfail(FEDAGG_EINVAL, "fedagg_comm: RCCL lacks nccl", #f);
  SYM(GetUniqueId) SYM(CommInitRank) SYM(CommDestroy) SYM(CommAbort) SYM(CommGetAsyncError) SYM(GroupStart)
  SYM(GroupEnd) SYM(Send) SYM(Recv) SYM(Reduce) SYM(GetErrorString)
#undef SYM
  g_rccl = r;
  return FEDAGG_OK;
}

int nccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return FEDAGG_OK;
  snprintf(g_lerr, sizeof(g_lerr), "%s: %s", what, g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "RCCL error");
  return FEDAGG_EHIP;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return FEDAGG_OK;
  snprintf(g_lerr, sizeof(g_lerr), "%s: %s", what, hipGetErrorString(e));
  return FEDAGG_EHIP;
}

ncclDataType_t nccl_type(int kind) {
  switch (kind) {
    case FEDAGG_F16: return ncclFloat16;
    case FEDAGG_F64: return ncclFloat64;
    default: return ncclFloat32;
  }
}

}  // namespace

struct fedagg_comm {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, nranks = 0;
  hipStream_t stream = nullptr;  // the communicator's stream
  std::vector<hipEvent_t> ev;    // per exchange group (grown on demand, reused across executions)
  hipEvent_t ev_compute = nullptr;
};

extern "C" {

const char* fedagg_comm_last_error(void) { return g_lerr; }

int fedagg_comm_unique_id(const char* rccl_path, void* id_out) {
  if (!id_out) return lfail(FEDAGG_EINVAL, "fedagg_comm_unique_id: NULL output");
  int rc = rccl_load(rccl_path);
  if (rc) return rc;
  ncclUniqueId id;
  rc = nccl_check(g_rccl.GetUniqueId(&id), "ncclGetUniqueId");
  if (rc) return rc;
  memcpy(id_out, &id, sizeof(id));
  return FEDAGG_OK;
}

int fedagg_comm_create(const char* rccl_path, int nranks, int rank, const void* unique_id, int device,
                       fedagg_comm** out) {
  if (!out || !unique_id || nranks < 1 || rank < 0 || rank >= nranks)
    return lfail(FEDAGG_EINVAL, "fedagg_comm_create: invalid argument");
  *out = nullptr;
  int rc = rccl_load(rccl_path);
  if (rc) return rc;
  if ((rc = hip_check(hipSetDevice(device), "hipSetDevice"))) return rc;
  fedagg_comm* c = new fedagg_comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  if ((rc = hip_check(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate")) ||
      (rc = hip_check(hipEventCreateWithFlags(&c->ev_compute, hipEventDisableTiming), "hipEventCreate")) ||
      (rc = nccl_check(g_rccl.CommInitRank(&c->comm, nranks, id, rank), "ncclCommInitRank"))) {
    if (c->ev_compute) (void)hipEventDestroy(c->ev_compute);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return rc;
  }
  *out = c;
  return FEDAGG_OK;
}

int fedagg_comm_destroy(fedagg_comm* c) {
  if (!c) return FEDAGG_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  int rc = c->comm ? nccl_check(g_rccl.CommDestroy(c->comm), "ncclCommDestroy") : FEDAGG_OK;
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->ev_compute);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return rc;
}

int fedagg_comm_abort(fedagg_comm* c) {
  if (!c || !c->comm) return FEDAGG_OK;
  int rc = nccl_check(g_rccl.CommAbort(c->comm), "ncclCommAbort");
  c->comm = nullptr;
  return rc;
}

int fedagg_comm_async_error(fedagg_comm* c) {
  if (!c || !c->comm) return lfail(FEDAGG_EINVAL, "fedagg_comm_async_error: no communicator");
  ncclResult_t st = ncclSuccess;
  int rc = nccl_check(g_rccl.CommGetAsyncError(c->comm, &st), "ncclCommGetAsyncError");
  if (rc) return rc;
  return nccl_check(st, "RCCL asynchronous error");
}

int fedagg_lockstep_execute(fedagg_comm* c, const fedagg_lockstep_run* runs, int nruns,
                            const fedagg_lockstep_msg* msgs, int nmsgs, int ngroups, void* ws, uint64_t ws_count,
                            int ws_kind, int root, void* stream) {
  if (!c || !c->comm || ngroups < 0 || nruns < 0 || nmsgs < 0 || (nruns && !runs) || (nmsgs && !msgs))
    return lfail(FEDAGG_EINVAL, "fedagg_lockstep_execute: invalid argument");
  hipStream_t s = (hipStream_t)stream;
  int rc;
  while ((int)c->ev.size() < ngroups) {
    hipEvent_t e;
    if ((rc = hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate"))) return rc;
    c->ev.push_back(e);
  }
  int ri = 0, mi = 0;
  for (int t = 0; t < ngroups; ++t) {
    // group t: after the compute stream's work so far (everything up to step t - 1)
    if (mi < nmsgs && msgs[mi].group == t) {
      if ((rc = hip_check(hipEventRecord(c->ev_compute, s), "hipEventRecord")) ||
          (rc = hip_check(hipStreamWaitEvent(c->stream, c->ev_compute, 0), "hipStreamWaitEvent")))
        return rc;
      if ((rc = nccl_check(g_rccl.GroupStart(), "ncclGroupStart"))) return rc;
      for (; mi < nmsgs && msgs[mi].group == t; ++mi) {
        const fedagg_lockstep_msg& m = msgs[mi];
        const ncclDataType_t dt = nccl_type(m.kind);
        rc = m.send ? nccl_check(g_rccl.Send(m.buf, m.count, dt, m.peer, c->comm, c->stream), "ncclSend")
                    : nccl_check(g_rccl.Recv(m.buf, m.count, dt, m.peer, c->comm, c->stream), "ncclRecv");
        if (rc) {
          (void)g_rccl.GroupEnd();
          return rc;
        }
      }
      if ((rc = nccl_check(g_rccl.GroupEnd(), "ncclGroupEnd"))) return rc;
      if ((rc = hip_check(hipEventRecord(c->ev[t], c->stream), "hipEventRecord"))) return rc;
    } else if ((rc = hip_check(hipEventRecord(c->ev[t], c->stream), "hipEventRecord"))) {
      return rc;  // an empty group still orders the streams like a group
    }
    if (mi < nmsgs && msgs[mi].group < t)
      return lfail(FEDAGG_EINVAL, "fedagg_lockstep_execute: messages must be sorted by group");
    // step t: after group t - 1 (the inputs of step t)
    if (t > 0 && (rc = hip_check(hipStreamWaitEvent(s, c->ev[t - 1], 0), "hipStreamWaitEvent"))) return rc;
    for (; ri < nruns && runs[ri].step == t; ++ri) {
      const fedagg_lockstep_run& r = runs[ri];
      if (r.K <= 0) return lfail(FEDAGG_EINVAL, "fedagg_lockstep_execute: a run needs >= 1 client");
      switch (r.op) {
        case FEDAGG_RUN_FEDAVG:
          if (r.kind == FEDAGG_F32)
            rc = fedagg_fedavg_chain_f32((const float* const*)r.x, (const float*)r.w, r.K, r.n, r.seed,
                                         (float*)r.acc, s);
          else if (r.kind == FEDAGG_BF16)
            rc = fedagg_fedavg_chain_bf16((const uint16_t* const*)r.x, (const float*)r.w, r.K, r.n, r.seed,
                                          (float*)r.acc, s);
          else if (r.kind == FEDAGG_F64)
            rc = fedagg_fedavg_chain_f64((const double* const*)r.x, (const double*)r.w, r.K, r.n, r.seed,
                                         (double*)r.acc, s);
          else
            rc = fedagg_fedavg_chain_f16((const uint16_t* const*)r.x, (const uint16_t*)r.w, r.K, r.n, r.seed,
                                         (uint16_t*)r.acc, s);
          break;
        case FEDAGG_RUN_FEDAVG_TILED:
          if (r.kind == FEDAGG_F32)
            rc = fedagg_fedavg_chain_tiled_f32((const float*)r.x[0], (const float*)r.w, r.K, r.n, r.tile_vectors,
                                               r.seed, (float*)r.acc, s);
          else
            rc = fedagg_fedavg_chain_tiled_bf16((const uint16_t*)r.x[0], (const float*)r.w, r.K, r.n,
                                                r.tile_vectors, r.seed, (float*)r.acc, s);
          break;
        case FEDAGG_RUN_SCAFFOLD:
          if (r.kind == FEDAGG_F32)
            rc = fedagg_scaffold_chain_f32((const float* const*)r.x, (const float* const*)r.x2, (const float*)r.c,
                                           (const double*)r.w, r.K, r.n, r.seed, r.finish, r.lr, (double*)r.acc,
                                           (double*)r.acc2, s);
          else
            rc = fedagg_scaffold_chain_f64((const double* const*)r.x, (const double* const*)r.x2,
                                           (const double*)r.c, (const double*)r.w, r.K, r.n, r.seed, r.finish, r.lr,
                                           (double*)r.acc, (double*)r.acc2, s);
          break;
        default:
          return lfail(FEDAGG_EINVAL, "fedagg_lockstep_execute: unknown run op");
      }
      if (rc) return lfail(rc, "fedagg_lockstep_execute: run failed: ", fedagg_last_error());
    }
  }
  if (ri != nruns || mi != nmsgs)
    return lfail(FEDAGG_EINVAL, "fedagg_lockstep_execute: runs / messages beyond the last group or unsorted");
  if (ngroups > 0 && (rc = hip_check(hipStreamWaitEvent(s, c->ev[ngroups - 1], 0), "hipStreamWaitEvent")))
    return rc;
  if (ws && ws_count) {  // numel == 1 products: summed onto the root (exact: x + 0; one rank: a copy)
    if ((rc = hip_check(hipEventRecord(c->ev_compute, s), "hipEventRecord")) ||
        (rc = hip_check(hipStreamWaitEvent(c->stream, c->ev_compute, 0), "hipStreamWaitEvent")) ||
        (rc = nccl_check(g_rccl.Reduce(ws, ws, ws_count, nccl_type(ws_kind), ncclSum, root, c->comm, c->stream),
                         "ncclReduce")) ||
        (rc = hip_check(hipEventRecord(c->ev_compute, c->stream), "hipEventRecord")) ||
        (rc = hip_check(hipStreamWaitEvent(s, c->ev_compute, 0), "hipStreamWaitEvent")))
      return rc;
  }
  return FEDAGG_OK;
}

}  // extern "C"
