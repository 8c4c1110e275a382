// thread_rccl.hip -- TEST INFRASTRUCTURE: a stand-in for the part of RCCL's API that the native
// lockstep executor (substrafl_amd/csrc/lockstep.hip) dlopens, with the ranks of a communicator as
// THREADS of one process on one GPU.  RCCL itself refuses two ranks on one GPU ("Duplicate GPU
// detected"), so this is how the executor's multi-rank path -- the run / message tables of every
// rank, the cross-stream event order, the slot reuse, the numel == 1 workspace reduce -- runs for
// real on the one-GPU test box (tests/test_native_executor_threads.py).  Never part of the product.
//
// Semantics kept from RCCL: a send completes on the sender's stream only after the receiver has
// consumed the data (like RCCL's blocking P2P kernels), a receive completes on the receiver's stream
// once the data is in place, the messages of a group are matched per (peer, direction) in issue
// order, ncclReduce(sum) lands on the root in rank order.  What differs: ncclGroupEnd blocks the
// HOST until every peer of the group has issued the matching group (RCCL blocks on the GPU), which
// is deadlock-free for the lockstep schedules for the same reason RCCL is (every rank issues its
// groups in order).  Data moves with device-to-device copies on the receiver's stream.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

struct Posted {  // one send, as its receiver sees it
  const void* buf = nullptr;
  size_t bytes = 0;
  hipEvent_t ready = nullptr;  // recorded on the sender's stream: the data is there
  hipEvent_t done = nullptr;   // recorded on the receiver's stream: the data has been copied out
  bool consumed = false;
};

struct World {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  // (src, dst, seq) -> the posted send
  std::map<std::tuple<int, int, uint64_t>, std::shared_ptr<Posted>> box;
  // collective reduces, by sequence number: the ranks' buffers and ready events
  struct Red {
    std::vector<const void*> buf;
    std::vector<hipEvent_t> ready;
    int posted = 0;
    hipEvent_t done = nullptr;
  };
  std::map<uint64_t, std::shared_ptr<Red>> red;
  std::vector<hipEvent_t> events;  // every event made for this world (freed with it)
  int alive = 0;
};

std::mutex g_mu;
std::map<uint64_t, std::shared_ptr<World>> g_worlds;
uint64_t g_next_id = 1;

struct Op {
  bool send;
  void* buf;
  size_t bytes;
  int peer;
  hipStream_t stream;
};

hipEvent_t new_event(World& w) {  // NOT under w.mu: no HIP call is ever made holding the world's lock
  hipEvent_t e = nullptr;
  (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  std::lock_guard<std::mutex> lk(w.mu);
  w.events.push_back(e);
  return e;
}

template <typename T>
__global__ void add_kernel(T* __restrict__ dst, const T* __restrict__ src, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = dst[i] + src[i];
}

__global__ void add_half_kernel(_Float16* __restrict__ dst, const _Float16* __restrict__ src, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (_Float16)((float)dst[i] + (float)src[i]);
}

bool launch_add(void* dst, const void* src, size_t count, ncclDataType_t t, hipStream_t s) {
  if (!count) return true;
  const unsigned blocks = (unsigned)((count + 255) / 256);
  switch (t) {
    case ncclFloat32:
      hipLaunchKernelGGL(add_kernel<float>, dim3(blocks), dim3(256), 0, s, (float*)dst, (const float*)src, count);
      return true;
    case ncclFloat64:
      hipLaunchKernelGGL(add_kernel<double>, dim3(blocks), dim3(256), 0, s, (double*)dst, (const double*)src, count);
      return true;
    case ncclFloat16:
      hipLaunchKernelGGL(add_half_kernel, dim3(blocks), dim3(256), 0, s, (_Float16*)dst, (const _Float16*)src, count);
      return true;
    default:
      return false;
  }
}

}  // namespace

struct ncclComm {
  std::shared_ptr<World> w;
  int rank = 0;
  std::vector<uint64_t> sent, recvd;  // per peer: messages issued so far (the matching sequence)
  uint64_t reduces = 0;
  std::vector<Op> ops;                // the open group
};

namespace {

thread_local int t_depth = 0;                   // ncclGroupStart nesting on this thread
thread_local ncclComm* t_group_comm = nullptr;  // the communicator of the open group

constexpr auto kWait = std::chrono::seconds(20);  // a peer that has not posted by then never will

// One group: post every send (its data-ready event recorded on the sender's stream), then serve
// every receive (wait for the matching post, copy on the receiver's stream after the data-ready
// event, record the consumed event), then make each send's stream wait for its consumed event.
// HIP calls are made outside the world's lock, so a HIP call that blocks cannot stall other ranks'
// posting.
ncclResult_t run_group(ncclComm* c) {
  World& w = *c->w;
  static const bool trace = getenv("THREAD_RCCL_TRACE") != nullptr;
  if (trace) {
    fprintf(stderr, "[thread_rccl] rank %d group:", c->rank);
    for (const Op& o : c->ops) fprintf(stderr, " %s%d:%zu", o.send ? "s" : "r", o.peer, o.bytes);
    fprintf(stderr, "\n");
  }
  std::vector<std::pair<Op, std::shared_ptr<Posted>>> sends;
  for (const Op& o : c->ops) {
    if (!o.send) continue;
    auto p = std::make_shared<Posted>();
    p->buf = o.buf;
    p->bytes = o.bytes;
    p->ready = new_event(w);
    if (hipEventRecord(p->ready, o.stream) != hipSuccess) return ncclUnhandledCudaError;
    {
      std::lock_guard<std::mutex> lk(w.mu);
      w.box[{c->rank, o.peer, c->sent[o.peer]++}] = p;
    }
    w.cv.notify_all();
    sends.emplace_back(o, p);
  }
  for (const Op& o : c->ops) {
    if (o.send) continue;
    const auto key = std::make_tuple(o.peer, c->rank, c->recvd[o.peer]++);
    std::shared_ptr<Posted> p;
    {
      std::unique_lock<std::mutex> lk(w.mu);
      if (!w.cv.wait_for(lk, kWait, [&] { return w.box.count(key) > 0; }))
        return ncclSystemError;  // the peer never issued its group: a schedule bug
      p = w.box[key];
      w.box.erase(key);
    }
    if (p->bytes != o.bytes) return ncclInvalidUsage;  // mismatched message sizes
    hipEvent_t done = new_event(w);
    if (hipStreamWaitEvent(o.stream, p->ready, 0) != hipSuccess ||
        hipMemcpyAsync(o.buf, p->buf, o.bytes, hipMemcpyDeviceToDevice, o.stream) != hipSuccess ||
        hipEventRecord(done, o.stream) != hipSuccess)
      return ncclUnhandledCudaError;
    {
      std::lock_guard<std::mutex> lk(w.mu);
      p->done = done;
      p->consumed = true;
    }
    w.cv.notify_all();
  }
  for (auto& sp : sends) {  // a send completes once its data has been copied out
    const std::shared_ptr<Posted>& p = sp.second;
    {
      std::unique_lock<std::mutex> lk(w.mu);
      if (!w.cv.wait_for(lk, kWait, [&] { return p->consumed; })) return ncclSystemError;
    }
    if (hipStreamWaitEvent(sp.first.stream, p->done, 0) != hipSuccess) return ncclUnhandledCudaError;
  }
  c->ops.clear();
  return ncclSuccess;
}

}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error";
    case ncclSystemError: return "thread_rccl: a peer never issued the matching operation (timeout)";
    case ncclInvalidUsage: return "thread_rccl: invalid usage (mismatched message sizes or arguments)";
    case ncclUnhandledCudaError: return "thread_rccl: HIP call failed";
    default: return "thread_rccl: error";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(g_mu);
  memset(id, 0, sizeof(*id));
  const uint64_t v = g_next_id++;
  memcpy(id->internal, &v, sizeof(v));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  uint64_t key;
  memcpy(&key, id.internal, sizeof(key));
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto& slot = g_worlds[key];
    if (!slot) {
      slot = std::make_shared<World>();
      slot->n = nranks;
    }
    if (slot->n != nranks) return ncclInvalidUsage;
    w = slot;
    w->alive++;
  }
  auto* c = new ncclComm();
  c->w = w;
  c->rank = rank;
  c->sent.assign(nranks, 0);
  c->recvd.assign(nranks, 0);
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  std::shared_ptr<World> w = c->w;
  delete c;
  std::lock_guard<std::mutex> lk(g_mu);
  if (--w->alive == 0) {
    (void)hipDeviceSynchronize();
    for (hipEvent_t e : w->events) (void)hipEventDestroy(e);
    w->events.clear();
    for (auto it = g_worlds.begin(); it != g_worlds.end();)
      it = (it->second == w) ? g_worlds.erase(it) : std::next(it);
  }
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) { return ncclCommDestroy(c); }

ncclResult_t ncclCommCount(const ncclComm_t c, int* count) {
  if (!c || !count) return ncclInvalidArgument;
  *count = (int)c->sent.size();  // one entry per rank of the world
  return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t, ncclResult_t* st) {
  if (st) *st = ncclSuccess;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  t_depth++;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth > 0) return ncclSuccess;
  ncclComm* c = t_group_comm;
  t_group_comm = nullptr;
  return c ? run_group(c) : ncclSuccess;  // an empty group completes at once
}

namespace {
ncclResult_t p2p(bool send, const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c,
                 hipStream_t s) {
  if (!c || peer < 0 || peer >= c->w->n) return ncclInvalidArgument;
  c->ops.push_back(Op{send, const_cast<void*>(buf), count * type_size(t), peer, s});
  if (t_depth == 0) return run_group(c);
  if (t_group_comm && t_group_comm != c) return ncclInvalidUsage;  // one communicator per group here
  t_group_comm = c;
  return ncclSuccess;
}
}  // namespace

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  return p2p(true, buf, count, t, peer, c, s);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  return p2p(false, buf, count, t, peer, c, s);
}

ncclResult_t ncclReduce(const void* sendbuf, void* recvbuf, size_t count, ncclDataType_t t, ncclRedOp_t op, int root,
                        ncclComm_t c, hipStream_t s) {
  if (!c || op != ncclSum || root < 0 || root >= c->w->n) return ncclInvalidArgument;
  World& w = *c->w;
  const uint64_t seq = c->reduces++;
  hipEvent_t ready = new_event(w);
  if (hipEventRecord(ready, s) != hipSuccess) return ncclUnhandledCudaError;
  std::shared_ptr<World::Red> r;
  {
    std::lock_guard<std::mutex> lk(w.mu);
    auto& slot = w.red[seq];
    if (!slot) {
      slot = std::make_shared<World::Red>();
      slot->buf.assign(w.n, nullptr);
      slot->ready.assign(w.n, nullptr);
    }
    r = slot;
    r->buf[c->rank] = sendbuf;
    r->ready[c->rank] = ready;
    r->posted++;
  }
  w.cv.notify_all();
  if (c->rank == root) {
    {
      std::unique_lock<std::mutex> lk(w.mu);
      if (!w.cv.wait_for(lk, kWait, [&] { return r->posted == w.n; })) return ncclSystemError;
    }
    if (sendbuf != recvbuf &&
        hipMemcpyAsync(recvbuf, sendbuf, count * type_size(t), hipMemcpyDeviceToDevice, s) != hipSuccess)
      return ncclUnhandledCudaError;
    for (int q = 0; q < w.n; ++q) {  // rank order
      if (q == root) continue;
      if (hipStreamWaitEvent(s, r->ready[q], 0) != hipSuccess || !launch_add(recvbuf, r->buf[q], count, t, s))
        return ncclUnhandledCudaError;
    }
    hipEvent_t done = new_event(w);
    if (hipEventRecord(done, s) != hipSuccess) return ncclUnhandledCudaError;
    {
      std::lock_guard<std::mutex> lk(w.mu);
      r->done = done;
    }
    w.cv.notify_all();
    return ncclSuccess;
  }
  hipEvent_t done = nullptr;
  {
    std::unique_lock<std::mutex> lk(w.mu);
    if (!w.cv.wait_for(lk, kWait, [&] { return r->done != nullptr; })) return ncclSystemError;
    done = r->done;
  }
  return hipStreamWaitEvent(s, done, 0) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

}  // extern "C"
