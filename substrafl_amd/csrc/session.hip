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

#include "fedagg.h"
#include "host_pool.h"

// defined in fedagg.hip
extern "C" const char* fedagg_last_error(void);
namespace fedagg_internal {
void set_error(const char* msg);
}

using fedagg_host::Done;
using fedagg_host::gather_range;
using fedagg_host::Pool;

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
  std::vector<void*> ring;
  std::vector<hipEvent_t> ring_ev;
  std::vector<bool> ring_used;
  void* dbuf[FEDAGG_SESSION_BUFFERS] = {};
  uint64_t dbytes[FEDAGG_SESSION_BUFFERS] = {};
  Pool* pool = nullptr;
  double last_stage_s = 0, last_fetch_s = 0;

  int ensure_ring() {
    if ((int)ring.size() == slots) return FEDAGG_OK;
    release_ring();
    ring.assign(slots, nullptr);
    ring_ev.assign(slots, nullptr);
    ring_used.assign(slots, false);
    HIP_TRY(hipHostMalloc(&ring_base, (size_t)slots * chunk_bytes, hipHostMallocDefault));
    for (int i = 0; i < slots; ++i) {
      ring[i] = static_cast<char*>(ring_base) + (size_t)i * chunk_bytes;
      HIP_TRY(hipEventCreateWithFlags(&ring_ev[i], hipEventDisableTiming));
    }
    return FEDAGG_OK;
  }
  void release_ring() {
    for (size_t i = 0; i < ring.size(); ++i) {
      if (ring_ev[i]) {
        (void)hipEventSynchronize(ring_ev[i]);
        (void)hipEventDestroy(ring_ev[i]);
      }
    }
    if (ring_base) (void)hipHostFree(ring_base);
    ring_base = nullptr;
    ring.clear();
    ring_ev.clear();
    ring_used.clear();
  }
  Pool& workers() {
    if (!pool || pool->size() != threads) {
      delete pool;
      pool = new Pool(threads);
    }
    return *pool;
  }
};

namespace {


double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

fedagg_session* fedagg_session_create(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
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
  if ((e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&s->xstream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&s->join_ev, hipEventDisableTiming)) != hipSuccess) {
    hip_fail("fedagg_session_create: stream/event", e);
    if (s->xstream) (void)hipStreamDestroy(s->xstream);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return nullptr;
  }
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
  } else {
    fedagg_internal::set_error("fedagg_session_set: unknown key or bad value");
    return FEDAGG_EINVAL;
  }
  return FEDAGG_OK;
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
  int rc = s->ensure_ring();
  if (rc) return rc;
  (void)s->workers();
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
  // one tiny launch loads the kernels' code object now rather than at the first aggregation
  HIP_TRY(hipMemsetAsync(probe, 0, 4096, s->stream));
  rc = fedagg_read_probe_f32(static_cast<const float*>(probe), 512, static_cast<float*>(probe) + 512, 1,
                             (void*)s->stream);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s->stream));
  return FEDAGG_OK;
}

int fedagg_session_stage(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg,
                         const void* const* h_seg, const uint64_t* seg_bytes) {
  if (nseg < 0 || (nseg > 0 && !seg_bytes)) return FEDAGG_EINVAL;
  uint64_t row = 0;
  for (int i = 0; i < nseg; ++i) row += seg_bytes[i];
  return fedagg_session_stage_range(s, d_dst, ld_bytes, K, nseg, h_seg, seg_bytes, 0, row);
}

int fedagg_session_stage_range(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg,
                               const void* const* h_seg, const uint64_t* seg_bytes, uint64_t byte_lo,
                               uint64_t byte_hi) {
  if (!s || !d_dst || K <= 0 || nseg < 0 || (nseg > 0 && (!h_seg || !seg_bytes)) || byte_hi < byte_lo)
    return FEDAGG_EINVAL;
  const double t0 = now_s();
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
  const uint64_t cb = s->chunk_bytes;
  const uint64_t per_row = row ? (row + cb - 1) / cb : 0;
  const uint64_t units = per_row * (uint64_t)K;
  const int R = (int)s->ring.size();
  Pool& pool = s->workers();
  const bool two = s->copy_streams > 1 && units > 1;
  if (two) {  // the second queue starts after everything already enqueued on the session stream
    HIP_TRY(hipEventRecord(s->join_ev, s->stream));
    HIP_TRY(hipStreamWaitEvent(s->xstream, s->join_ev, 0));
  }
  std::vector<Done> done(units ? std::min<uint64_t>(units, (uint64_t)R) : 1);
  // In-order window: unit u lives in slot u % R.  R-1 packs run ahead of the copy being
  // enqueued; a slot is refilled only after the copy that read it completed, while the next
  // copy is already in flight, so the link never waits on the main thread.
  uint64_t next_submit = 0;
  auto submit = [&](uint64_t u) {
    const int slot = (int)(u % R);
    if (s->ring_used[slot]) (void)hipEventSynchronize(s->ring_ev[slot]);  // H2D of unit u-R done
    s->ring_used[slot] = false;
    Done& d = done[slot];
    d.done = false;
    const int k = (int)(u / per_row);
    const uint64_t a = (u % per_row) * cb, b = std::min(row, a + cb);
    const void* const* segs = h_seg + (size_t)k * nseg;
    char* dst = static_cast<char*>(s->ring[slot]);
    pool.submit([=, &d] {
      gather_range(segs, seg_bytes, nseg, byte_lo + a, byte_lo + b, dst);
      d.set();
    });
  };
  for (; next_submit < units && next_submit + 1 < (uint64_t)R; ++next_submit) submit(next_submit);
  for (uint64_t u = 0; u < units; ++u) {
    const int slot = (int)(u % R);
    done[slot].wait();
    const int k = (int)(u / per_row);
    const uint64_t a = (u % per_row) * cb, b = std::min(row, a + cb);
    char* dst = static_cast<char*>(d_dst) + (uint64_t)k * ld_bytes + a;
    hipStream_t q = (two && (u & 1)) ? s->xstream : s->stream;
    HIP_TRY(hipMemcpyAsync(dst, s->ring[slot], b - a, hipMemcpyHostToDevice, q));
    HIP_TRY(hipEventRecord(s->ring_ev[slot], q));
    s->ring_used[slot] = true;
    if (next_submit < units) submit(next_submit++);
  }
  if (two) {  // work enqueued on the session stream after this call sees every staged byte
    HIP_TRY(hipEventRecord(s->join_ev, s->xstream));
    HIP_TRY(hipStreamWaitEvent(s->stream, s->join_ev, 0));
  }
  s->last_stage_s = now_s() - t0;
  return FEDAGG_OK;
}

int fedagg_session_fetch(fedagg_session* s, const void* d_src, void* h_dst, uint64_t bytes) {
  if (!s || !d_src || (!h_dst && bytes)) return FEDAGG_EINVAL;
  const double t0 = now_s();
  HIP_TRY(hipSetDevice(s->device));
  int rc = s->ensure_ring();
  if (rc) return rc;
  const uint64_t cb = s->chunk_bytes;
  const int R = (int)s->ring.size();
  // D2H in super-chunks of G adjacent slots (one DMA of G * chunk_bytes: 16 MiB copies run at
  // 55 GB/s where 4 MiB ones reach 49, profiles/r01_h2d_probe.log); each slot of a super-chunk is
  // then copied out by its own worker once the DMA's event completes.  Groups rotate over the ring.
  const int G = std::max(1, std::min(4, R / 2));
  const int NG = R / G;
  const uint64_t sb = cb * (uint64_t)G;
  const uint64_t units = (bytes + sb - 1) / sb;
  Pool& pool = s->workers();
  std::vector<Done> done(R);
  std::vector<bool> pending(R, false);
  for (uint64_t u = 0; u < units; ++u) {
    const int g0 = (int)(u % (uint64_t)NG) * G;  // first slot of this group
    for (int i = 0; i < G; ++i)
      if (pending[g0 + i]) done[g0 + i].wait();
    const uint64_t a = u * sb, b = std::min(bytes, a + sb);
    HIP_TRY(hipMemcpyAsync(s->ring[g0], static_cast<const char*>(d_src) + a, b - a, hipMemcpyDeviceToHost,
                           s->stream));
    HIP_TRY(hipEventRecord(s->ring_ev[g0], s->stream));
    hipEvent_t ev = s->ring_ev[g0];
    for (int i = 0; i < G; ++i) {
      const uint64_t pa = a + (uint64_t)i * cb;
      if (pa >= b) break;
      const uint64_t pb = std::min(b, pa + cb);
      const int slot = g0 + i;
      s->ring_used[slot] = i == 0;
      done[slot].done = false;
      pending[slot] = true;
      char* src = static_cast<char*>(s->ring[slot]);
      char* dst = static_cast<char*>(h_dst) + pa;
      Done* d = &done[slot];
      pool.submit([=] {
        (void)hipEventSynchronize(ev);
        memcpy(dst, src, pb - pa);
        d->set();
      });
    }
  }
  for (int i = 0; i < R; ++i)
    if (pending[i]) done[i].wait();
  s->last_fetch_s = now_s() - t0;
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

int fedagg_session_sync(fedagg_session* s) {
  if (!s) return FEDAGG_EINVAL;
  HIP_TRY(hipSetDevice(s->device));
  HIP_TRY(hipStreamSynchronize(s->stream));
  return FEDAGG_OK;
}

int fedagg_session_timing(fedagg_session* s, double* stage_s, double* fetch_s) {
  if (!s) return FEDAGG_EINVAL;
  if (stage_s) *stage_s = s->last_stage_s;
  if (fetch_s) *fetch_s = s->last_fetch_s;
  return FEDAGG_OK;
}

}  // extern "C"
