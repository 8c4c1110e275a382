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
  decltype(&ncclCommCount) CommCount = nullptr;
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
  SYM(GroupEnd) SYM(Send) SYM(Recv) SYM(Reduce) SYM(GetErrorString) SYM(CommCount)
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

// One run of a schedule on stream s (the chain-kernel entry points of fedagg.hip).
int run_one(const fedagg_lockstep_run& r, hipStream_t s) {
  if (r.K <= 0) return lfail(FEDAGG_EINVAL, "lockstep: a run needs >= 1 client");
  int rc = FEDAGG_OK;
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
    case FEDAGG_RUN_FEDAVG_PUSH: {  // output: mapped peer memory; input accumulator: acc2 (NULL: seed / acc)
      const float* in = r.acc2 ? (const float*)r.acc2 : (r.seed ? nullptr : (const float*)r.acc);
      if (r.kind == FEDAGG_F32)
        rc = fedagg_fedavg_chain_push_f32((const float* const*)r.x, (const float*)r.w, r.K, r.n, in, (float*)r.acc, s);
      else if (r.kind == FEDAGG_BF16)
        rc = fedagg_fedavg_chain_push_bf16((const uint16_t* const*)r.x, (const float*)r.w, r.K, r.n, in,
                                           (float*)r.acc, s);
      else
        return lfail(FEDAGG_EINVAL, "lockstep: push runs are fp32 or bf16 (fp32 accumulators)");
      break;
    }
    case FEDAGG_RUN_SCAFFOLD_PUSH_DELTA:
    case FEDAGG_RUN_SCAFFOLD_PUSH_CV: {  // one bucket: x = its K rows; acc = output, acc2 = input
      const int ph = r.op == FEDAGG_RUN_SCAFFOLD_PUSH_CV;
      const double* in = r.acc2 ? (const double*)r.acc2 : (r.seed ? nullptr : (const double*)r.acc);
      if (r.kind == FEDAGG_F32)
        rc = fedagg_scaffold_chain_push_f32((const float* const*)r.x, (const double*)r.w, r.K, r.n, ph,
                                            (const float*)r.c, r.lr, r.finish, in, (double*)r.acc, s);
      else if (r.kind == FEDAGG_F64)
        rc = fedagg_scaffold_chain_push_f64((const double* const*)r.x, (const double*)r.w, r.K, r.n, ph,
                                            (const double*)r.c, r.lr, r.finish, in, (double*)r.acc, s);
      else
        return lfail(FEDAGG_EINVAL, "lockstep: Scaffold push runs take fp32 or fp64 buckets (fp64 accumulators)");
      break;
    }
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
      return lfail(FEDAGG_EINVAL, "lockstep: unknown run op");
  }
  return rc ? lfail(rc, "lockstep: run failed: ", fedagg_last_error()) : FEDAGG_OK;
}


// ---- push executor (fedagg_push_execute): progress counters in a node-shared host page ----
constexpr int PUSH_MAX_WAITS = 32;  // counters / tags one wait kernel polls (one lane each)
constexpr int PUSH_MAX_TAGS = 16;   // landing tags one signal kernel writes (one lane each)
constexpr uint64_t PUSH_TAG_ERR = 1ull << 32;   // err word: a landing tag (not a counter) timed out
constexpr uint64_t PUSH_PEER_ERR = 1ull << 33;  // err word: gave up because rank (low bits - 1) failed
struct PushWaitArgs {
  uint32_t n;
  uint32_t idx[PUSH_MAX_WAITS];
  uint64_t val[PUSH_MAX_WAITS];
  const uint64_t* tag[PUSH_MAX_WAITS];
};
struct PushSignalArgs {
  uint32_t n;
  uint64_t* tag[PUSH_MAX_TAGS];
};

__device__ __forceinline__ uint64_t ld_acquire_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The first rank whose err word is set (its wait gave up: the call's result is void everywhere),
// or -1.  errs: the nranks err words of the node-shared page.
__device__ __forceinline__ int push_failed_rank(const uint64_t* errs, uint32_t nranks) {
  for (uint32_t j = 0; j < nranks; ++j)
    if (ld_acquire_sys(errs + j)) return (int)j;
  return -1;
}

// Lane i polls progress[idx[i]] until it reaches val[i] (system-scope acquire: what the producer
// released before its signal is visible to the kernels after this one); then, for a landing tag,
// its tag word until it holds this call's generation `gen` -- a tag still missing when the counter
// was already there is the ordering gap between the PCIe counter and the xGMI data: counted in
// *late and waited out.  A wait that exceeds `timeout` ticks gives up and records idx + 1 (+
// PUSH_TAG_ERR for a tag) in *err.  Fail fast: a wait also gives up as soon as ANY rank's err word
// is set (a peer's or an earlier wait of this rank: the call's result is void), recording
// PUSH_PEER_ERR + that rank + 1 when the cause is another rank's, so a dead or slow peer costs
// the group one timeout, not one per wait.  The err words are scanned every PUSH_ERR_SCAN_EVERY
// polls and not on entry (on the error-free path a wait whose counter is already there
// reads no err word at all -- the entry scan of nranks uncached host-page words cost ~9 us per step,
// profiles/r06f_push_overhead_probe.jsonl; a failure is still seen within tens of microseconds).
// Every lane reaches the end (the late count is a wave ballot).
constexpr uint32_t PUSH_ERR_SCAN_EVERY = 16;

__global__ void __launch_bounds__(64) push_wait_kernel(const uint64_t* progress, PushWaitArgs a, uint64_t gen,
                                                       uint64_t timeout, uint64_t* err, uint64_t* late,
                                                       const uint64_t* errs, uint32_t nranks, uint32_t rank) {
  const uint32_t i = threadIdx.x;
  bool was_late = false;
  if (i < a.n) {
    const uint64_t t0 = wall_clock64();
    int peer = -1;      // the first failed rank, once a scan has seen one
    uint64_t code = 0;  // this lane's own failure
    const uint64_t* tag = a.tag[i];
    bool counter_done = false;
    uint32_t polls = 0;
    while (peer < 0 && !code) {
      if (!counter_done) {
        if (ld_acquire_sys(progress + a.idx[i]) >= a.val[i]) {
          counter_done = true;
          if (!tag) break;
          if (ld_acquire_sys(tag) >= gen) break;
          was_late = true;
          continue;
        }
      } else if (ld_acquire_sys(tag) >= gen) {
        break;
      }
      if (wall_clock64() - t0 > timeout) code = (uint64_t)a.idx[i] + 1 + (counter_done ? PUSH_TAG_ERR : 0);
      else {
        __builtin_amdgcn_s_sleep(16);
        if (++polls % PUSH_ERR_SCAN_EVERY == 0) peer = push_failed_rank(errs, nranks);
      }
    }
    if (code) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (peer >= 0 && (uint32_t)peer != rank &&
             !__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
      __hip_atomic_store(err, PUSH_PEER_ERR + (uint64_t)peer + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint64_t m = __ballot(was_late);
  if (i == 0 && m) {  // only this rank's wait kernels (one stream, in order) write its late word
    const uint64_t v = __hip_atomic_load(late, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(late, v + (uint64_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// After everything before it on the stream (the step's push runs, whose peer stores are
// system-scope write-through stores each wave waited to be acknowledged before retiring -- no
// release fence there): the landing tags of the consumers this step pushed to (peer HBM, the
// data's own path), then a release, then progress[idx] = value (the node-shared host page).
__global__ void __launch_bounds__(64) push_signal_kernel(uint64_t* progress, uint32_t idx, uint64_t value,
                                                         PushSignalArgs t, uint64_t gen) {
  const uint32_t i = threadIdx.x;
  if (i < t.n) __hip_atomic_store(t.tag[i], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // the wave's tag stores performed before the counter
  if (i == 0) __hip_atomic_store(progress + idx, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// dst[0, n) = src[0, n) (4-byte words) with ordinary vector stores: a copy into a peer's mapped
// memory that stays in the stream's order (a runtime copy into imported memory need not), ended
// by a system-scope release like the push runs.
__global__ void __launch_bounds__(256) push_copy_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                        uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) dst[i] = src[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// Root: ws[i] = stage[0][i] + ... + stage[G-1][i] in rank order (one owner per column, the
// others +0.0: exact).  T: fp32 (FedAvg's products) or fp64 (Scaffold's).
template <typename T>
__global__ void __launch_bounds__(256) push_stage_sum_kernel(T* __restrict__ ws, const T* __restrict__ stage, int G,
                                                             uint64_t n) {
#pragma clang fp contract(off)
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    T a = stage[i];
    for (int g = 1; g < G; ++g) a = a + stage[(uint64_t)g * n + i];
    ws[i] = a;
  }
}

int push_signal(uint64_t* progress, int rank, uint64_t value, const fedagg_push_tag* tags, int& ti, int ntags,
                int step, uint64_t gen, hipStream_t s) {
  PushSignalArgs a;
  memset(&a, 0, sizeof(a));
  for (; ti < ntags && tags[ti].step == step; ++ti) {
    if (a.n >= (uint32_t)PUSH_MAX_TAGS) return lfail(FEDAGG_EINVAL, "fedagg_push_execute: > 16 landing tags a step");
    a.tag[a.n++] = tags[ti].tag;
  }
  hipLaunchKernelGGL(push_signal_kernel, dim3(1), dim3(64), 0, s, progress, (uint32_t)rank, value, a, gen);
  return hip_check(hipGetLastError(), "push_signal_kernel");
}

int push_copy(void* dst, const void* src, uint64_t bytes, hipStream_t s) {
  if (bytes % 4) return lfail(FEDAGG_EINVAL, "push: copies are whole 4-byte words");
  const uint64_t words = bytes / 4;
  if (!words) return FEDAGG_OK;
  const uint64_t g = (words + 255) / 256;
  hipLaunchKernelGGL(push_copy_kernel, dim3((unsigned)(g < 2048 ? g : 2048)), dim3(256), 0, s, (uint32_t*)dst,
                     (const uint32_t*)src, words);
  return hip_check(hipGetLastError(), "push_copy_kernel");
}

int push_waits(const fedagg_push_wait* waits, int& wi, int nwaits, int step, uint64_t* progress, uint64_t base,
               uint64_t timeout, uint64_t* err, uint64_t* late, int nranks, int rank, hipStream_t s) {
  while (wi < nwaits && waits[wi].step == step) {
    PushWaitArgs a;
    memset(&a, 0, sizeof(a));
    for (; wi < nwaits && waits[wi].step == step && a.n < PUSH_MAX_WAITS; ++wi) {
      const int64_t v = (int64_t)base + waits[wi].value;
      if (v <= 0 && !waits[wi].tag) continue;  // the counters start at 0
      a.idx[a.n] = (uint32_t)waits[wi].rank;
      a.val[a.n] = (uint64_t)(v > 0 ? v : 0);
      a.tag[a.n] = waits[wi].tag;
      ++a.n;
    }
    if (!a.n) continue;
    hipLaunchKernelGGL(push_wait_kernel, dim3(1), dim3(64), 0, s, (const uint64_t*)progress, a, base + 1, timeout, err,
                       late, (const uint64_t*)progress + nranks, (uint32_t)nranks, (uint32_t)rank);
    int rc = hip_check(hipGetLastError(), "push_wait_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
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

int fedagg_comm_count(fedagg_comm* c, int* count_out) {
  if (!c || !c->comm || !count_out) return lfail(FEDAGG_EINVAL, "fedagg_comm_count: invalid argument");
  return nccl_check(g_rccl.CommCount(c->comm, count_out), "ncclCommCount");
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
      if ((rc = run_one(runs[ri], s))) return rc;
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


// ---- push executor ----
int fedagg_ipc_get(const void* ptr, void* handle_out, uint64_t* offset_out) {
  if (!ptr || !handle_out || !offset_out) return lfail(FEDAGG_EINVAL, "fedagg_ipc_get: NULL argument");
  static_assert(sizeof(hipIpcMemHandle_t) <= FEDAGG_IPC_HANDLE_BYTES, "IPC handle size");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  int rc;
  if ((rc = hip_check(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr), "hipMemGetAddressRange"))) return rc;
  hipIpcMemHandle_t h;
  if ((rc = hip_check(hipIpcGetMemHandle(&h, (void*)base), "hipIpcGetMemHandle"))) return rc;
  memset(handle_out, 0, FEDAGG_IPC_HANDLE_BYTES);
  memcpy(handle_out, &h, sizeof(h));
  *offset_out = (uint64_t)((const char*)ptr - (const char*)base);
  return FEDAGG_OK;
}

int fedagg_ipc_open(const void* handle, void** base_out) {
  if (!handle || !base_out) return lfail(FEDAGG_EINVAL, "fedagg_ipc_open: NULL argument");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hip_check(hipIpcOpenMemHandle(base_out, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
}

int fedagg_ipc_close(void* base) { return base ? hip_check(hipIpcCloseMemHandle(base), "hipIpcCloseMemHandle") : 0; }

int fedagg_host_map(void* host, uint64_t bytes, void** dev_out) {
  if (!host || !bytes || !dev_out) return lfail(FEDAGG_EINVAL, "fedagg_host_map: invalid argument");
  int rc;
  if ((rc = hip_check(hipHostRegister(host, bytes, hipHostRegisterMapped), "hipHostRegister"))) return rc;
  return hip_check(hipHostGetDevicePointer(dev_out, host, 0), "hipHostGetDevicePointer");
}

int fedagg_host_unmap(void* host) { return host ? hip_check(hipHostUnregister(host), "hipHostUnregister") : 0; }

int fedagg_device_alloc_uncached(uint64_t bytes, void** out) {
  if (!out || !bytes) return lfail(FEDAGG_EINVAL, "fedagg_device_alloc_uncached: invalid argument");
  *out = nullptr;
  int rc;
  if ((rc = hip_check(hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags"))) return rc;
  return hip_check(hipMemset(*out, 0, bytes), "hipMemset");
}

int fedagg_device_free(void* p) { return p ? hip_check(hipFree(p), "hipFree") : 0; }

#if FEDAGG_TUNING
int fedagg_copy_async(void* dst, const void* src, uint64_t bytes, void* stream) {
  if (!bytes) return FEDAGG_OK;
  if (!dst || !src) return lfail(FEDAGG_EINVAL, "fedagg_copy_async: NULL argument");
  return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream), "hipMemcpyAsync");
}
#endif

int fedagg_wall_clock_hz(uint64_t* hz_out) {
  if (!hz_out) return lfail(FEDAGG_EINVAL, "fedagg_wall_clock_hz: NULL output");
  int dev = 0, khz = 0, rc;
  if ((rc = hip_check(hipGetDevice(&dev), "hipGetDevice")) ||
      (rc = hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev), "hipDeviceGetAttribute")))
    return rc;
  *hz_out = (uint64_t)khz * 1000ull;
  return FEDAGG_OK;
}

int fedagg_push_execute(const fedagg_lockstep_run* runs, int nruns, const fedagg_push_wait* waits, int nwaits,
                        const fedagg_push_tag* tags, int ntags,
                        int nsteps, uint64_t* progress, int rank, int nranks, uint64_t base, uint64_t timeout_ticks,
                        const void* ws_src, void* ws_dst, uint64_t ws_bytes, int ws_kind, const void* ws_stage,
                        const fedagg_push_copy* copies, int ncopies, void* const* aux_streams, int naux,
                        void* stream) {
  if (nruns < 0 || nwaits < 0 || ntags < 0 || nsteps < 0 || (nruns && !runs) || (nwaits && !waits) ||
      (ntags && !tags) || !progress || nranks < 1 ||
      rank < 0 || rank >= nranks || (ws_bytes && (!ws_src || !ws_dst)) || naux < 0 || naux > 7 ||
      (naux && !aux_streams) || ncopies < 0 || (ncopies && !copies) ||
      (ws_bytes && ws_kind != FEDAGG_F32 && ws_kind != FEDAGG_F64) ||
      (ws_bytes % (ws_kind == FEDAGG_F64 ? 8 : 4)))
    return lfail(FEDAGG_EINVAL, "fedagg_push_execute: invalid argument");
  for (int i = 0; i < ncopies; ++i)
    if (!copies[i].dst || !copies[i].src) return lfail(FEDAGG_EINVAL, "fedagg_push_execute: NULL landing copy");
  for (int i = 0; i < nwaits; ++i)
    if (waits[i].rank < 0 || waits[i].rank >= nranks || waits[i].step < 0 || waits[i].step > nsteps ||
        (i && waits[i].step < waits[i - 1].step))
      return lfail(FEDAGG_EINVAL, "fedagg_push_execute: waits out of range or unsorted");
  for (int i = 0; i < nruns; ++i)
    if ((runs[i].op != FEDAGG_RUN_FEDAVG && runs[i].op != FEDAGG_RUN_FEDAVG_PUSH &&
         runs[i].op != FEDAGG_RUN_SCAFFOLD_PUSH_DELTA && runs[i].op != FEDAGG_RUN_SCAFFOLD_PUSH_CV) ||
        runs[i].step < 0 || runs[i].step >= nsteps || (i && runs[i].step < runs[i - 1].step))
      return lfail(FEDAGG_EINVAL, "fedagg_push_execute: runs must be row push runs sorted by step");
  for (int i = 0; i < ntags; ++i)
    if (!tags[i].tag || tags[i].step < 0 || tags[i].step >= nsteps || (i && tags[i].step < tags[i - 1].step))
      return lfail(FEDAGG_EINVAL, "fedagg_push_execute: tags out of range or unsorted");
  hipStream_t s = (hipStream_t)stream;
  uint64_t* err = progress + nranks + rank;
  uint64_t* late = progress + 2 * nranks + rank;
  const uint64_t gen = base + 1;  // this call's generation: its entry value, unique and > 0
  int rc, ti = 0;
  // base + 1: this rank entered the call -- everything its stream held before (a refill of the
  // output, the previous call's reads of its slots) is done, so peers may write into its buffers
  if ((rc = push_signal(progress, rank, base + 1, tags, ti, 0, -1, gen, s))) return rc;
  // a step's launches (one per consumer: each writes over its own xGMI link) spread over the
  // caller's stream and the aux streams, forked from and joined back into the caller's stream
  // fork / join events: kept for the thread's lifetime (per device), never destroyed while a
  // wait the GPU has not run yet may still name them; re-recording one is safe (a wait takes the
  // record current when it is enqueued)
  static thread_local hipEvent_t ev_pool[16][8];
  static thread_local bool ev_made[16];
  int dev = 0;
  if ((rc = hip_check(hipGetDevice(&dev), "hipGetDevice"))) return rc;
  if (dev < 0 || dev >= 16) return lfail(FEDAGG_EINVAL, "fedagg_push_execute: device index beyond 15");
  if (!ev_made[dev]) {
    for (int i = 0; i < 8; ++i)
      if ((rc = hip_check(hipEventCreateWithFlags(&ev_pool[dev][i], hipEventDisableTiming), "hipEventCreate")))
        return rc;
    ev_made[dev] = true;
  }
  hipEvent_t* ev = ev_pool[dev];
  int ri = 0, wi = 0;
  for (int t = 0; t < nsteps; ++t) {
    if ((rc = push_waits(waits, wi, nwaits, t, progress, base, timeout_ticks, err, late, nranks, rank, s))) return rc;
    if (t == 0 && ws_bytes &&  // after step 0's waits, which include the root's entry
        (rc = push_copy(ws_dst, ws_src, ws_bytes, s)))
      return rc;
    int r0 = ri;
    while (ri < nruns && runs[ri].step == t) ++ri;
    const int nlaunch = ri - r0, used = nlaunch - 1 < naux ? nlaunch - 1 : naux;
    if (used > 0) {  // fork: the aux streams start after the waits above
      if ((rc = hip_check(hipEventRecord(ev[0], s), "hipEventRecord"))) return rc;
      for (int a = 0; a < used; ++a)
        if ((rc = hip_check(hipStreamWaitEvent((hipStream_t)aux_streams[a], ev[0], 0), "hipStreamWaitEvent")))
          return rc;
    }
    for (int i = 0; i < nlaunch; ++i) {
      hipStream_t si = (used > 0 && i % (used + 1)) ? (hipStream_t)aux_streams[i % (used + 1) - 1] : s;
      if ((rc = run_one(runs[r0 + i], si))) return rc;
    }
    for (int a = 0; a < used; ++a)  // join: the step's signal after every launch of it
      if ((rc = hip_check(hipEventRecord(ev[1 + a], (hipStream_t)aux_streams[a]), "hipEventRecord")) ||
          (rc = hip_check(hipStreamWaitEvent(s, ev[1 + a], 0), "hipStreamWaitEvent")))
        return rc;
    // step t done: its consumers' landing tags, then base + t + 2
    if ((rc = push_signal(progress, rank, base + t + 2, tags, ti, ntags, t, gen, s))) return rc;
  }
  if ((rc = push_waits(waits, wi, nwaits, nsteps, progress, base, timeout_ticks, err, late, nranks, rank, s)))
    return rc;
  if (ti != ntags || wi != nwaits) return lfail(FEDAGG_EINVAL, "fedagg_push_execute: tags / waits beyond the last step");
  // root, once every rank's last step is in: the finished pieces others pushed, into the output;
  // the numel == 1 staging rows, summed into this rank's workspace
  for (int i = 0; i < ncopies; ++i)
    if ((rc = push_copy(copies[i].dst, copies[i].src, copies[i].bytes, s))) return rc;
  if (ws_stage && ws_bytes) {
    const uint64_t n = ws_bytes / (ws_kind == FEDAGG_F64 ? 8 : 4), g = (n + 255) / 256;
    const dim3 grid((unsigned)(g < 1024 ? g : 1024));
    if (ws_kind == FEDAGG_F64)
      hipLaunchKernelGGL(push_stage_sum_kernel<double>, grid, dim3(256), 0, s, (double*)ws_src,
                         (const double*)ws_stage, nranks, n);
    else
      hipLaunchKernelGGL(push_stage_sum_kernel<float>, grid, dim3(256), 0, s, (float*)ws_src, (const float*)ws_stage,
                         nranks, n);
    if ((rc = hip_check(hipGetLastError(), "push_stage_sum_kernel"))) return rc;
  }
  return FEDAGG_OK;
}

}  // extern "C"
