// session.hip -- native host runtime of the aggregation engine: one GPU, one HIP stream,
// grow-only HBM buffers, a pinned staging ring and a worker pool that packs the clients'
// host arrays into the ring while earlier chunks are already on the PCIe link.
//
// Why native: an aggregate task is one short-lived process (remote/register/register.py:96-121)
// that receives K host pickles.  Doing the pack + H2D + D2H plumbing here (instead of through
// PyTorch) keeps torch's CUDA context creation off the task's critical path and overlaps the
// host memcpy with the DMA, which a Python loop cannot do without holding the GIL per chunk.
//
// Data path of fedagg_session_stage (one call per bucket):
//   client k's row = its layer arrays back to back (segments); the row is cut into chunks of
//   `chunk_bytes`; chunk u is packed by a worker into pinned slot u % R, then the main thread
//   enqueues hipMemcpyAsync(slot -> HBM row k) on the session stream and records the slot's
//   event; a slot is reused only after its event completed.  W workers, R >= W slots.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <sys/syscall.h>
#include <unistd.h>

#include "fedagg.h"
#include "host_pool.h"

// defined in fedagg.hip
extern "C" const char* fedagg_last_error(void);
namespace fedagg_internal {
void set_error(const char* msg);
}

using fedagg_host::Pool;
using fedagg_host::Ring;

namespace {

int hip_fail(const char* what, hipError_t e) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
  fedagg_internal::set_error(buf);
  return FEDAGG_EHIP;
}

#define HIP_TRY(call)                                     \
  do {                                                    \
    hipError_t e_ = (call);                               \
    if (e_ != hipSuccess) return hip_fail(#call, e_);     \
  } while (0)

}  // namespace

struct fedagg_session {
  int device = 0;
  hipStream_t stream = nullptr;
  // second H2D queue: staging alternates its chunks over `stream` and `xstream`, so one chunk's
  // copy is set up while the other's is on the link (4 MiB pinned chunks: 49 GB/s on one queue,
  // 56 GB/s over two on MI355X, profiles/r01_h2d_probe.log); the tail of a stage joins `stream`
  hipStream_t xstream = nullptr;
  hipEvent_t join_ev = nullptr;
  int copy_streams = 2;
  int threads = 8;
  uint64_t chunk_bytes = 4ull << 20;  // 4 MiB: same staging rate as 16 MiB, a third of the cold ring cost
  int slots = 12;
  void* ring_base = nullptr;  // one pinned block: slot i at ring_base + i * chunk_bytes, so
                              // adjacent slots can take one larger DMA (fetch super-chunks)
  Ring ring;
  std::vector<hipEvent_t> ring_ev;
  void* dbuf[FEDAGG_SESSION_BUFFERS] = {};
  uint64_t dbytes[FEDAGG_SESSION_BUFFERS] = {};
  hipEvent_t tev[FEDAGG_SESSION_EVENTS] = {};  // timing events (fedagg_session_event_*)
  Pool* pool = nullptr;
  double last_stage_s = 0, last_fetch_s = 0;
  uint64_t fail_copy_after = 0;  // test knob: the n-th copy of the session fails (0 = never)
  uint64_t copies = 0;
  std::vector<int> cpus;  // fedagg_session_affinity: the pack workers' and the ring's CPUs (empty: any)
  // start-up phases, seconds (fedagg_session_phases): create's HIP runtime init + device, its
  // streams / events; warm's pinned ring, worker pool, HBM buffers, code-object load
  double phase[FEDAGG_SESSION_PHASES] = {};

  int ensure_ring() {
    if (ring.size() == slots && ring.chunk_bytes == chunk_bytes) return FEDAGG_OK;
    release_ring();
    ring.slot.assign(slots, nullptr);
    ring_ev.assign(slots, nullptr);
    ring.used.assign(slots, false);
    ring.chunk_bytes = chunk_bytes;
    hipError_t e;
    if (cpus.empty()) {
      e = hipHostMalloc(&ring_base, (size_t)slots * chunk_bytes, hipHostMallocDefault);
    } else {
      // allocated under the user's NUMA policy (hipHostMallocNumaUser) by a thread bound to the
      // session's CPUs: the default local policy puts the pinned pages on their node
      e = hipErrorUnknown;
      std::thread t([&] {
        (void)hipSetDevice(device);  // the new thread's current device: this session's GPU
        if (fedagg_host::bind_thread(cpus))
          e = hipHostMalloc(&ring_base, (size_t)slots * chunk_bytes, hipHostMallocNumaUser);
        else
          e = hipHostMalloc(&ring_base, (size_t)slots * chunk_bytes, hipHostMallocDefault);
      });
      t.join();
    }
    if (e != hipSuccess) {
      ring_base = nullptr;
      release_ring();
      return hip_fail("hipHostMalloc(staging ring)", e);
    }
    for (int i = 0; i < slots; ++i) {
      ring.slot[i] = static_cast<char*>(ring_base) + (size_t)i * chunk_bytes;
      if ((e = hipEventCreateWithFlags(&ring_ev[i], hipEventDisableTiming)) != hipSuccess) {
        ring_ev[i] = nullptr;
        release_ring();
        return hip_fail("hipEventCreate(staging ring)", e);
      }
    }
    return FEDAGG_OK;
  }
  void release_ring() {
    for (size_t i = 0; i < ring_ev.size(); ++i) {
      if (ring_ev[i]) {
        (void)hipEventSynchronize(ring_ev[i]);
        (void)hipEventDestroy(ring_ev[i]);
      }
    }
    if (ring_base) (void)hipHostFree(ring_base);
    ring_base = nullptr;
    ring.slot.clear();
    ring.used.clear();
    ring.chunk_bytes = 0;
    ring_ev.clear();
  }
  std::mutex pool_m;  // workers() may be reached from a compare-only check beside a stage call
  Pool& workers() {
    std::lock_guard<std::mutex> g(pool_m);
    if (!pool || pool->size() != threads || pool->cpus() != cpus) {
      delete pool;
      pool = new Pool(threads, cpus);
    }
    return *pool;
  }
};

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The copy engine of host_pool.h's pipelines on HIP: queue 0 = the session stream, queue 1 = the
// second H2D queue; one event per ring slot.
struct HipEngine {
  fedagg_session* s;
  bool injected() { return s->fail_copy_after && ++s->copies >= s->fail_copy_after; }
  int h2d(int q, void* d, const void* h, uint64_t n) {
    if (injected()) return hip_fail("hipMemcpyAsync(H2D) [injected by the fail_copy_after knob]", hipErrorUnknown);
    hipError_t e = hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, q ? s->xstream : s->stream);
    return e == hipSuccess ? FEDAGG_OK : hip_fail("hipMemcpyAsync(H2D)", e);
  }
  int h2d_2d(int q, void* d, uint64_t dpitch, const void* h, uint64_t spitch, uint64_t width, uint64_t height) {
    if (injected()) return hip_fail("hipMemcpy2DAsync(H2D) [injected by the fail_copy_after knob]", hipErrorUnknown);
    hipError_t e = hipMemcpy2DAsync(d, dpitch, h, spitch, width, height, hipMemcpyHostToDevice,
                                    q ? s->xstream : s->stream);
    return e == hipSuccess ? FEDAGG_OK : hip_fail("hipMemcpy2DAsync(H2D)", e);
  }
  int d2h(void* h, const void* d, uint64_t n) {
    if (injected()) return hip_fail("hipMemcpyAsync(D2H) [injected by the fail_copy_after knob]", hipErrorUnknown);
    hipError_t e = hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s->stream);
    return e == hipSuccess ? FEDAGG_OK : hip_fail("hipMemcpyAsync(D2H)", e);
  }
  int mark(int slot, int q) {
    hipError_t e = hipEventRecord(s->ring_ev[slot], q ? s->xstream : s->stream);
    return e == hipSuccess ? FEDAGG_OK : hip_fail("hipEventRecord(ring)", e);
  }
  void wait(int slot) { (void)hipEventSynchronize(s->ring_ev[slot]); }
};

}  // namespace

extern "C" {

fedagg_session* fedagg_session_create(int device) {
  const double t0 = now_s();
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);  // the process's first HIP call initialises the runtime
  if (e != hipSuccess || n <= 0) {
    hip_fail("fedagg_session_create: no HIP device", e == hipSuccess ? hipErrorNoDevice : e);
    return nullptr;
  }
  if (device < 0 || device >= n) {
    fedagg_internal::set_error("fedagg_session_create: device index out of range");
    return nullptr;
  }
  if ((e = hipSetDevice(device)) != hipSuccess) {
    hip_fail("hipSetDevice", e);
    return nullptr;
  }
  auto* s = new fedagg_session();
  s->device = device;
  const double t1 = now_s();
  s->phase[0] = t1 - t0;
  if ((e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&s->xstream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&s->join_ev, hipEventDisableTiming)) != hipSuccess) {
    hip_fail("fedagg_session_create: stream/event", e);
    if (s->xstream) (void)hipStreamDestroy(s->xstream);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return nullptr;
  }
  s->phase[1] = now_s() - t1;
  return s;
}

void fedagg_session_destroy(fedagg_session* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  (void)hipStreamSynchronize(s->stream);
  (void)hipStreamSynchronize(s->xstream);
  s->release_ring();
  for (int i = 0; i < FEDAGG_SESSION_BUFFERS; ++i)
    if (s->dbuf[i]) (void)hipFree(s->dbuf[i]);
  for (int i = 0; i < FEDAGG_SESSION_EVENTS; ++i)
    if (s->tev[i]) (void)hipEventDestroy(s->tev[i]);
  (void)hipEventDestroy(s->join_ev);
  (void)hipStreamDestroy(s->xstream);
  (void)hipStreamDestroy(s->stream);
  delete s->pool;
  delete s;
}

void* fedagg_session_stream(fedagg_session* s) { return s ? (void*)s->stream : nullptr; }

int fedagg_session_set(fedagg_session* s, const char* key, long long value) {
  if (!s || !key) return FEDAGG_EINVAL;
  if (!strcmp(key, "threads") && value >= 1 && value <= 256) {
    s->threads = (int)value;
    if (s->slots < s->threads + 2) {
      s->release_ring();
      s->slots = s->threads + 2;
    }
  } else if (!strcmp(key, "chunk_bytes") && value >= (1 << 16)) {
    s->release_ring();
    s->chunk_bytes = (uint64_t)value;
  } else if (!strcmp(key, "copy_streams") && (value == 1 || value == 2)) {
    s->copy_streams = (int)value;
  } else if (!strcmp(key, "slots") && value >= 2 && value <= 1024) {
    s->release_ring();
    s->slots = (int)std::max<long long>(value, s->threads + 1);
  } else if (!strcmp(key, "fail_copy_after") && value >= 0) {  // tests: error paths of stage/fetch
    s->fail_copy_after = (uint64_t)value;
    s->copies = 0;
  } else {
    fedagg_internal::set_error("fedagg_session_set: unknown key or bad value");
    return FEDAGG_EINVAL;
  }
  return FEDAGG_OK;
}

int fedagg_session_affinity(fedagg_session* s, const int* cpus, int ncpus) {
  if (!s || ncpus < 0 || (ncpus && !cpus)) {
    fedagg_internal::set_error("fedagg_session_affinity: invalid argument");
    return FEDAGG_EINVAL;
  }
  std::vector<int> v(cpus, cpus + ncpus);
  for (int c : v)
    if (c < 0 || c >= CPU_SETSIZE) {
      fedagg_internal::set_error("fedagg_session_affinity: CPU index out of range");
      return FEDAGG_EINVAL;
    }
  // workers() compares s->cpus under pool_m (a compare-only check may run beside this call): swap
  // them under the same lock; the ring is released on the session's device, the caller's restored
  std::lock_guard<std::mutex> g(s->pool_m);
  if (v != s->cpus) {
    int caller = -1;
    (void)hipGetDevice(&caller);
    (void)hipSetDevice(s->device);
    s->release_ring();  // re-allocated on the new CPUs' node at the next stage / fetch
    s->cpus = std::move(v);
    if (caller >= 0) (void)hipSetDevice(caller);
  }
  return FEDAGG_OK;
}

int fedagg_session_ring_node(fedagg_session* s) {
  if (!s || !s->ring_base) return -1;
  int node = -1;
  // get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR): the node of the page holding the address
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, s->ring_base, 3UL) != 0) return -1;
  return node;
}

int fedagg_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 13) {
    fedagg_internal::set_error("fedagg_device_pci_bus_id: buffer too small");
    return FEDAGG_EINVAL;
  }
  hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
  return e == hipSuccess ? FEDAGG_OK : hip_fail("hipDeviceGetPCIBusId", e);
}

int fedagg_session_buffer(fedagg_session* s, int slot, uint64_t bytes, void** d_ptr) {
  if (!s || slot < 0 || slot >= FEDAGG_SESSION_BUFFERS || !d_ptr) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  if (s->dbytes[slot] < bytes) {
    if (s->dbuf[slot]) {
      HIP_TRY(hipStreamSynchronize(s->stream));
      HIP_TRY(hipFree(s->dbuf[slot]));
      s->dbuf[slot] = nullptr;
      s->dbytes[slot] = 0;
    }
    HIP_TRY(hipMalloc(&s->dbuf[slot], bytes));
    s->dbytes[slot] = bytes;
  }
  *d_ptr = s->dbuf[slot];
  return FEDAGG_OK;
}

int fedagg_session_warm(fedagg_session* s, const uint64_t* slot_bytes, int nslots) {
  if (!s || nslots < 0 || nslots > FEDAGG_SESSION_BUFFERS || (nslots > 0 && !slot_bytes)) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  double t = now_s();
  int rc = s->ensure_ring();
  if (rc) return rc;
  s->phase[2] = now_s() - t;
  t = now_s();
  (void)s->workers();
  s->phase[3] = now_s() - t;
  t = now_s();
  void* probe = nullptr;
  for (int i = 0; i < nslots; ++i) {
    if (!slot_bytes[i]) continue;
    void* d = nullptr;
    rc = fedagg_session_buffer(s, i, slot_bytes[i], &d);
    if (rc) return rc;
    if (!probe && slot_bytes[i] >= 4096) probe = d;
  }
  if (!probe) {
    rc = fedagg_session_buffer(s, FEDAGG_SESSION_BUFFERS - 1, 4096, &probe);
    if (rc) return rc;
  }
  s->phase[4] = now_s() - t;
  t = now_s();
  // one tiny launch loads the kernels' code object now rather than at the first aggregation
  HIP_TRY(hipMemsetAsync(probe, 0, 4096, s->stream));
  rc = fedagg_read_probe_f32(static_cast<const float*>(probe), 512, static_cast<float*>(probe) + 512, 1,
                             (void*)s->stream);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->stream));
  s->phase[5] = now_s() - t;
  return FEDAGG_OK;
}

int fedagg_session_stage(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg,
                         const void* const* h_seg, const uint64_t* seg_bytes) {
  if (nseg < 0 || (nseg > 0 && !seg_bytes)) return FEDAGG_EINVAL;
  uint64_t row = 0;
  for (int i = 0; i < nseg; ++i) row += seg_bytes[i];
  return fedagg_session_stage_range(s, d_dst, ld_bytes, K, nseg, h_seg, seg_bytes, 0, row);
}

namespace {

// shared argument checks and set-up of the staging entry points; returns the row length in bytes
int stage_prepare(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg, const void* const* h_seg,
                  const uint64_t* seg_bytes, uint64_t byte_lo, uint64_t byte_hi, uint64_t* row_out) {
  if (!s || !d_dst || K <= 0 || nseg < 0 || (nseg > 0 && (!h_seg || !seg_bytes)) || byte_hi < byte_lo)
    return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  int rc = s->ensure_ring();
  if (rc) return rc;
  uint64_t full = 0;
  for (int i = 0; i < nseg; ++i) full += seg_bytes[i];
  if (byte_hi > full) {
    fedagg_internal::set_error("fedagg_session_stage_range: byte range beyond the row");
    return FEDAGG_EINVAL;
  }
  const uint64_t row = byte_hi - byte_lo;  // bytes [byte_lo, byte_hi) of every client's row
  if (row > ld_bytes) {
    fedagg_internal::set_error("fedagg_session_stage: segments exceed the row stride");
    return FEDAGG_EINVAL;
  }
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < nseg; ++i)
      if (!h_seg[(size_t)k * nseg + i] && seg_bytes[i]) {
        fedagg_internal::set_error("fedagg_session_stage: NULL host segment");
        return FEDAGG_EINVAL;
      }
  *row_out = row;
  return FEDAGG_OK;
}

// run(engine, two_queues) between the joins of the two copy queues
}  // namespace
}  // extern "C"
namespace {
template <class Run>
int stage_run_with(fedagg_session* s, Run run) {
  const double t0 = now_s();
  const bool two = s->copy_streams > 1;
  if (two) {  // the second queue starts after everything already enqueued on the session stream
    HIP_TRY(hipEventRecord(s->join_ev, s->stream));
    HIP_TRY(hipStreamWaitEvent(s->xstream, s->join_ev, 0));
  }
  HipEngine eng{s};
  int rc = run(eng, two);
  if (two) {  // work enqueued on the session stream after this call sees every staged byte
    hipError_t e = hipEventRecord(s->join_ev, s->xstream);
    if (e == hipSuccess) e = hipStreamWaitEvent(s->stream, s->join_ev, 0);
    if (e != hipSuccess && !rc) rc = hip_fail("fedagg_session_stage: join of the copy queues", e);
  }
  s->last_stage_s = now_s() - t0;
  return rc;
}

int stage_run(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg, const void* const* h_seg,
              const uint64_t* seg_bytes, uint64_t byte_lo, uint64_t row, int check_esz, uint64_t* mismatches) {
  return stage_run_with(s, [&](HipEngine& eng, bool two) {
    return fedagg_host::stage_pipeline(eng, s->workers(), s->ring, h_seg, seg_bytes, nseg, K, byte_lo, row,
                                       static_cast<char*>(d_dst), ld_bytes, two, check_esz, mismatches);
  });
}

}  // namespace

extern "C" {

int fedagg_session_stage_range(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg,
                               const void* const* h_seg, const uint64_t* seg_bytes, uint64_t byte_lo,
                               uint64_t byte_hi) {
  uint64_t row = 0;
  int rc = stage_prepare(s, d_dst, ld_bytes, K, nseg, h_seg, seg_bytes, byte_lo, byte_hi, &row);
  if (rc) return rc;
  return stage_run(s, d_dst, ld_bytes, K, nseg, h_seg, seg_bytes, byte_lo, row, 0, nullptr);
}

int fedagg_session_stage_tiled(fedagg_session* s, void* d_dst, uint64_t tile_bytes, int K, int nseg,
                               const void* const* h_seg, const uint64_t* seg_bytes) {
  if (nseg < 0 || (nseg > 0 && !seg_bytes)) return FEDAGG_EINVAL;
  uint64_t full = 0, row = 0;
  for (int i = 0; i < nseg; ++i) full += seg_bytes[i];
  int rc = stage_prepare(s, d_dst, full, K, nseg, h_seg, seg_bytes, 0, full, &row);
  if (rc) return rc;
  if (!tile_bytes || tile_bytes % 16 || tile_bytes > s->chunk_bytes) {
    fedagg_internal::set_error("fedagg_session_stage_tiled: tile_bytes must be a multiple of 16 and <= chunk_bytes");
    return FEDAGG_EINVAL;
  }
  return stage_run_with(s, [&](HipEngine& eng, bool two) {
    return fedagg_host::stage_tiled_pipeline(eng, s->workers(), s->ring, h_seg, seg_bytes, nseg, K, row, tile_bytes,
                                             static_cast<char*>(d_dst), two);
  });
}

int fedagg_session_stage_tiled_row(fedagg_session* s, void* d_dst, uint64_t tile_bytes, int K, int k, int nseg,
                                   const void* const* h_seg, const uint64_t* seg_bytes) {
  if (nseg < 0 || (nseg > 0 && !seg_bytes)) return FEDAGG_EINVAL;
  if (K <= 0 || k < 0 || k >= K) {
    fedagg_internal::set_error("fedagg_session_stage_tiled_row: need 0 <= k < K");
    return FEDAGG_EINVAL;
  }
  uint64_t full = 0, row = 0;
  for (int i = 0; i < nseg; ++i) full += seg_bytes[i];
  int rc = stage_prepare(s, d_dst, full, 1, nseg, h_seg, seg_bytes, 0, full, &row);
  if (rc) return rc;
  if (!tile_bytes || tile_bytes % 16 || tile_bytes > s->chunk_bytes) {
    fedagg_internal::set_error("fedagg_session_stage_tiled_row: tile_bytes must be a multiple of 16 and <= chunk_bytes");
    return FEDAGG_EINVAL;
  }
  return stage_run_with(s, [&](HipEngine& eng, bool two) {
    return fedagg_host::stage_row_tiled_pipeline(eng, s->workers(), s->ring, h_seg, seg_bytes, nseg, row, tile_bytes,
                                                 K, k, static_cast<char*>(d_dst), two);
  });
}

int fedagg_session_stage_check(fedagg_session* s, void* d_dst, int K, int nseg, const void* const* h_seg,
                               const uint64_t* seg_bytes, uint64_t byte_lo, uint64_t byte_hi, int kind,
                               uint64_t* mismatches) {
  if (!mismatches || (kind != FEDAGG_F32 && kind != FEDAGG_F64)) {
    fedagg_internal::set_error("fedagg_session_stage_check: kind must be FEDAGG_F32 or FEDAGG_F64");
    return FEDAGG_EINVAL;
  }
  const int esz = kind == FEDAGG_F64 ? 8 : 4;
  for (int i = 0; i < nseg && seg_bytes; ++i)
    if (seg_bytes[i] % esz) {
      fedagg_internal::set_error("fedagg_session_stage_check: segment not a whole number of elements");
      return FEDAGG_EINVAL;
    }
  if (byte_lo % esz || byte_hi % esz) {
    fedagg_internal::set_error("fedagg_session_stage_check: byte range not element-aligned");
    return FEDAGG_EINVAL;
  }
  *mismatches = 0;
  if (!d_dst) {  // compare only: no HIP call, no ring -- safe beside a stage call on the same session
    if (!s || K <= 0 || nseg < 0 || (nseg > 0 && (!h_seg || !seg_bytes)) || byte_hi < byte_lo) return FEDAGG_EINVAL;
    uint64_t full = 0;
    for (int i = 0; i < nseg; ++i) full += seg_bytes[i];
    for (int k = 0; k < K; ++k)
      for (int i = 0; i < nseg; ++i)
        if (!h_seg[(size_t)k * nseg + i] && seg_bytes[i]) {
          fedagg_internal::set_error("fedagg_session_stage_check: NULL host segment");
          return FEDAGG_EINVAL;
        }
    if (byte_hi > full) {
      fedagg_internal::set_error("fedagg_session_stage_check: byte range beyond the row");
      return FEDAGG_EINVAL;
    }
    *mismatches = fedagg_host::check_rows(s->workers(), h_seg, seg_bytes, nseg, K, byte_lo, byte_hi - byte_lo, esz);
    return FEDAGG_OK;
  }
  uint64_t row = 0;
  int rc = stage_prepare(s, d_dst, byte_hi - byte_lo, K, nseg, h_seg, seg_bytes, byte_lo, byte_hi, &row);
  if (rc) return rc;
  return stage_run(s, d_dst, row, K, nseg, h_seg, seg_bytes, byte_lo, row, esz, mismatches);
}

int fedagg_session_fetch(fedagg_session* s, const void* d_src, void* h_dst, uint64_t bytes) {
  if (!s || !d_src || (!h_dst && bytes)) return FEDAGG_EINVAL;
  const double t0 = now_s();
  HIP_TRY(hipSetDevice(s->device));
  int rc = s->ensure_ring();
  if (rc) return rc;
  // D2H in super-chunks of adjacent slots (16 MiB copies run at 55 GB/s where 4 MiB ones reach
  // 49, profiles/r01_h2d_probe.log), copied out of the ring by the workers (host_pool.h)
  HipEngine eng{s};
  rc = fedagg_host::fetch_pipeline(eng, s->workers(), s->ring, static_cast<const char*>(d_src),
                                   static_cast<char*>(h_dst), bytes);
  s->last_fetch_s = now_s() - t0;
  return rc;
}

int fedagg_session_event_record(fedagg_session* s, int ev) {
  if (!s || ev < 0 || ev >= FEDAGG_SESSION_EVENTS) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  if (!s->tev[ev]) HIP_TRY(hipEventCreate(&s->tev[ev]));
  HIP_TRY(hipEventRecord(s->tev[ev], s->stream));
  return FEDAGG_OK;
}

int fedagg_session_event_elapsed(fedagg_session* s, int ev0, int ev1, float* ms) {
  if (!s || !ms || ev0 < 0 || ev1 < 0 || ev0 >= FEDAGG_SESSION_EVENTS || ev1 >= FEDAGG_SESSION_EVENTS ||
      !s->tev[ev0] || !s->tev[ev1])
    return FEDAGG_EINVAL;
  HIP_TRY(hipEventSynchronize(s->tev[ev1]));
  HIP_TRY(hipEventElapsedTime(ms, s->tev[ev0], s->tev[ev1]));
  return FEDAGG_OK;
}

int fedagg_session_activate(fedagg_session* s) {
  if (!s) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  return FEDAGG_OK;
}

int fedagg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int fedagg_device_get(int* device_out) {
  if (!device_out) return FEDAGG_EINVAL;
  HIP_TRY(hipGetDevice(device_out));
  return FEDAGG_OK;
}

int fedagg_device_set(int device) {
  HIP_TRY(hipSetDevice(device));
  return FEDAGG_OK;
}

int fedagg_device_memory(int device, uint64_t* free_bytes, uint64_t* total_bytes) {
  if (!free_bytes || !total_bytes) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(device));
  size_t f = 0, t = 0;
  HIP_TRY(hipMemGetInfo(&f, &t));
  *free_bytes = f;
  *total_bytes = t;
  return FEDAGG_OK;
}

int fedagg_session_memset(fedagg_session* s, void* d, int value, uint64_t bytes) {
  if (!s || !d) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(hipMemsetAsync(d, value, bytes, s->stream));
  return FEDAGG_OK;
}

int fedagg_session_copy_d2d(fedagg_session* s, void* d_dst, const void* d_src, uint64_t bytes) {
  if (!s || (bytes && (!d_dst || !d_src))) return FEDAGG_EINVAL;
  if (!bytes) return FEDAGG_OK;
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, s->stream));
  return FEDAGG_OK;
}

int fedagg_session_sync(fedagg_session* s) {
  if (!s) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(hipStreamSynchronize(s->stream));
  return FEDAGG_OK;
}

int fedagg_session_phases(fedagg_session* s, double* out, int n) {
  if (!s || n < 0 || (n && !out)) return FEDAGG_EINVAL;
  for (int i = 0; i < n && i < FEDAGG_SESSION_PHASES; ++i) out[i] = s->phase[i];
  return FEDAGG_OK;
}

int fedagg_session_timing(fedagg_session* s, double* stage_s, double* fetch_s) {
  if (!s) return FEDAGG_EINVAL;
  if (stage_s) *stage_s = s->last_stage_s;
  if (fetch_s) *fetch_s = s->last_fetch_s;
  return FEDAGG_OK;
}

}  // extern "C"
