// host_pool.h -- the host-only half of the session runtime (session.hip): the pack worker pool,
// the per-chunk completion flag and the segment-range gather.  Plain C++17, no HIP, so that
// tests/c/host_pool_test.cpp builds it with g++ under ThreadSanitizer and AddressSanitizer
// (tests/test_host_sanitizers.py, SURVEY.md §5 "race detection").
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

namespace fedagg_host {

// Bind the calling thread to `cpus` (none: leave it as it is); false if the kernel refused.
inline bool bind_thread(const std::vector<int>& cpus) {
  if (cpus.empty()) return true;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

class Pool {
 public:
  // n workers; with `cpus`, each binds itself to those CPUs before taking work (a GPU's pack
  // workers on that GPU's NUMA node, next to its pinned ring: multi_device.host_placement)
  explicit Pool(int n, std::vector<int> cpus = {}) : cpus_(std::move(cpus)) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  int size() const { return (int)th_.size(); }
  const std::vector<int>& cpus() const { return cpus_; }

 private:
  void run() {
    bind_thread(cpus_);  // best effort: a refused mask leaves the worker where the OS put it
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  const std::vector<int> cpus_;  // before th_: the workers read it as they start
  std::vector<std::thread> th_;
  std::deque<std::function<void()>> q_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

// completion flag for one packed chunk.  set() notifies while it still holds the mutex: the
// waiter may return -- and destroy the flag -- as soon as it can observe done == true, so
// nothing of the flag may be touched after the mutex is released (ThreadSanitizer caught the
// notify-after-unlock form racing with ~Done in tests/c/host_pool_test.cpp).
struct Done {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  void set() {
    std::lock_guard<std::mutex> g(m);
    done = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [this] { return done; });
  }
};

// Copy bytes [a, b) of the concatenation of segments (ptr[i], len[i]) into dst.
inline void gather_range(const void* const* ptr, const uint64_t* len, int nseg, uint64_t a, uint64_t b, char* dst) {
  uint64_t off = 0;
  for (int i = 0; i < nseg && off < b; ++i) {
    const uint64_t s0 = off, s1 = off + len[i];
    off = s1;
    const uint64_t lo = std::max(a, s0), hi = std::min(b, s1);
    if (lo >= hi) continue;
    memcpy(dst + (lo - a), static_cast<const char*>(ptr[i]) + (lo - s0), hi - lo);
  }
}

// Value-equality mismatches of n elements (T = float or double): equal when x == r or both are
// NaN, so +0 == -0 and NaN == NaN, as np.testing.assert_array_equal (scaffold.py:193-196).
template <typename T>
inline uint64_t count_value_mismatch(const char* x, const char* r, uint64_t n) {
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) {
    T a, b;
    memcpy(&a, x + i * sizeof(T), sizeof(T));
    memcpy(&b, r + i * sizeof(T), sizeof(T));
    bad += !((a == b) || (a != a && b != b));
  }
  return bad;
}

// Mismatching elements (size esz: 4 = float, 8 = double) between bytes [a, b) of two rows given
// as segment lists of the same lengths.  Byte-identical stretches are skipped with memcmp; only
// a differing 4 KiB block is compared by value.  Segment and range bounds are element-aligned.
inline uint64_t count_mismatch_range(const void* const* x, const void* const* ref, const uint64_t* len, int nseg,
                                     uint64_t a, uint64_t b, int esz) {
  uint64_t off = 0, bad = 0;
  for (int i = 0; i < nseg && off < b; ++i) {
    const uint64_t s0 = off, s1 = off + len[i];
    off = s1;
    const uint64_t lo = std::max(a, s0), hi = std::min(b, s1);
    if (lo >= hi) continue;
    const char* px = static_cast<const char*>(x[i]) + (lo - s0);
    const char* pr = static_cast<const char*>(ref[i]) + (lo - s0);
    if (px == pr) continue;  // the very same array (simulation mode hands every client one c)
    for (uint64_t u = 0; u < hi - lo; u += 4096) {
      const uint64_t n = std::min<uint64_t>(4096, hi - lo - u);
      if (!memcmp(px + u, pr + u, n)) continue;
      bad += esz == 8 ? count_value_mismatch<double>(px + u, pr + u, n / 8)
                      : count_value_mismatch<float>(px + u, pr + u, n / 4);
    }
  }
  return bad;
}

// ------------------------------------------------------------------------------------------
// The staging and fetch pipelines of the session (session.hip), written against a copy engine
// so that the same code runs on HIP in the library and on a fake DMA thread with injected
// failures under ThreadSanitizer / AddressSanitizer (tests/c/host_pool_test.cpp).  Eng provides
//   int  h2d(int q, void* d_dst, const void* h_src, uint64_t n)  enqueue a copy on queue q (0/1)
//   int  d2h(void* h_dst, const void* d_src, uint64_t n)          enqueue a copy on queue 0
//   int  mark(int slot, int q)     record slot's completion event after queue q's copies
//   void wait(int slot)            block until slot's last recorded event completed
// and returns 0 or a negative error code from each enqueueing call.  On an error the pipelines
// stop submitting, wait for every pack / copy-out task already handed to the pool (those hold
// pointers into this call's flags and the caller's buffers), and only then return the code.
// ------------------------------------------------------------------------------------------
struct Ring {
  std::vector<void*> slot;     // R pinned chunks of chunk_bytes
  std::vector<bool> used;      // a copy reading / writing the slot may still be in flight
  uint64_t chunk_bytes = 0;
  int size() const { return (int)slot.size(); }
};

// Value check of bytes [byte_lo, byte_lo + row) of rows 1..K-1 against row 0 (esz-byte elements),
// in 1 MiB pieces of the row on the pool; returns the number of mismatching elements.  Touches
// nothing but the pool and the caller's segments, so it may run beside a staging call.
inline uint64_t check_rows(Pool& pool, const void* const* h_seg, const uint64_t* seg_bytes, int nseg, int K,
                           uint64_t byte_lo, uint64_t row, int esz) {
  const uint64_t piece = 1ull << 20;
  const uint64_t npieces = (K >= 2 && row) ? (row + piece - 1) / piece : 0;
  std::atomic<uint64_t> bad{0};
  std::vector<Done> cdone(npieces ? npieces : 1);
  for (uint64_t p = 0; p < npieces; ++p) {
    const uint64_t a = byte_lo + p * piece, b = byte_lo + std::min(row, (p + 1) * piece);
    Done* d = &cdone[p];
    pool.submit([=, &bad] {
      uint64_t n = 0;
      for (int k = 1; k < K; ++k) n += count_mismatch_range(h_seg + (size_t)k * nseg, h_seg, seg_bytes, nseg, a, b, esz);
      bad.fetch_add(n, std::memory_order_relaxed);
      d->set();
    });
  }
  for (uint64_t p = 0; p < npieces; ++p) cdone[p].wait();
  return bad.load();
}

// The staging ring: `units` pieces, unit u packed by a worker into ring slot u % R
// (pack(u, slot) on the pool) and copied to the device by the calling thread (copy(u, slot, q):
// enqueue the unit's copies from the slot on queue q, alternating over two queues with two_queues;
// returns 0 or an error code).
// In-order window: R-1 packs run ahead of the copy being enqueued; a slot is refilled only after
// the copy that read it completed, while the next copy is already in flight, so the link never
// waits on the enqueueing thread.  On an error the packs already submitted are waited for (they
// read the caller's segments and write the ring) before the code is returned.
template <class Eng, class Pack, class Copy>
int ring_stage(Eng& eng, Pool& pool, Ring& ring, uint64_t units, bool two_queues, Pack pack, Copy copy) {
  const int R = ring.size();
  const bool two = two_queues && units > 1;
  std::vector<Done> done(units ? std::min<uint64_t>(units, (uint64_t)R) : 1);
  std::vector<bool> pending(done.size(), false);
  int rc = 0;
  uint64_t next_submit = 0;
  auto submit = [&](uint64_t u) {
    const int slot = (int)(u % R);
    if (ring.used[slot]) eng.wait(slot);  // the copy of unit u - R is done
    ring.used[slot] = false;
    Done& d = done[slot];
    d.done = false;
    pending[slot] = true;
    char* dst = static_cast<char*>(ring.slot[slot]);
    pool.submit([=, &d] {
      pack(u, dst);
      d.set();
    });
  };
  for (; next_submit < units && next_submit + 1 < (uint64_t)R; ++next_submit) submit(next_submit);
  for (uint64_t u = 0; u < units && !rc; ++u) {
    const int slot = (int)(u % R);
    done[slot].wait();
    pending[slot] = false;
    const int q = (two && (u & 1)) ? 1 : 0;
    rc = copy(u, static_cast<const char*>(ring.slot[slot]), q);
    if (!rc) rc = eng.mark(slot, q);
    if (!rc) ring.used[slot] = true;
    if (!rc && next_submit < units) submit(next_submit++);
  }
  for (size_t i = 0; i < done.size(); ++i)  // packs still running read the caller's segments
    if (pending[i]) done[i].wait();
  return rc;
}

// K rows of nseg host segments -> d_dst + k * ld_bytes, bytes [byte_lo, byte_lo + row) of each
// row.  check_esz > 0: only row 0 is staged, rows 1..K-1 are compared with it by value on the
// host (mismatching elements added to *mismatches) -- the server-control-variate check of
// scaffold.py:193-196 done while the bytes are in host memory anyway, one copy over PCIe.
template <class Eng>
int stage_pipeline(Eng& eng, Pool& pool, Ring& ring, const void* const* h_seg, const uint64_t* seg_bytes, int nseg,
                   int K, uint64_t byte_lo, uint64_t row, char* d_dst, uint64_t ld_bytes, bool two_queues,
                   int check_esz = 0, uint64_t* mismatches = nullptr) {
  const uint64_t cb = ring.chunk_bytes;
  const int Ks = check_esz ? 1 : K;
  const uint64_t per_row = row ? (row + cb - 1) / cb : 0;  // unit u: chunk u % per_row of row u / per_row
  const int rc = ring_stage(
      eng, pool, ring, per_row * (uint64_t)Ks, two_queues,
      [=](uint64_t u, char* dst) {
        const uint64_t a = (u % per_row) * cb, b = std::min(row, a + cb);
        gather_range(h_seg + (size_t)(u / per_row) * nseg, seg_bytes, nseg, byte_lo + a, byte_lo + b, dst);
      },
      [&, per_row, cb](uint64_t u, const char* slot, int q) {
        const uint64_t a = (u % per_row) * cb;
        return eng.h2d(q, d_dst + (u / per_row) * ld_bytes + a, slot, std::min(row, a + cb) - a);
      });
  if (rc || !check_esz || K < 2) return rc;
  const uint64_t bad = check_rows(pool, h_seg, seg_bytes, nseg, K, byte_lo, row, check_esz);
  if (mismatches) *mismatches += bad;
  return 0;
}

// K rows of nseg host segments (row bytes each) -> the tile-interleaved layout of
// fedagg_fedavg_tiled_*: tile t of row k (bytes [t * tb, (t + 1) * tb)) at d_dst + (t * K + k) * tb.
// The destination is one run of (tile, row) blocks, so a unit is a run of whole blocks gathered
// from the K rows into one pinned slot and ONE contiguous copy; the pad of a row's last, partial
// tile is not written on the host (the kernels never read it).  tb <= the ring's chunk_bytes.
template <class Eng>
int stage_tiled_pipeline(Eng& eng, Pool& pool, Ring& ring, const void* const* h_seg, const uint64_t* seg_bytes,
                         int nseg, int K, uint64_t row, uint64_t tb, char* d_dst, bool two_queues) {
  if (!tb || tb > ring.chunk_bytes) return -1;
  const uint64_t tiles = row ? (row + tb - 1) / tb : 0;
  const uint64_t blocks = tiles * (uint64_t)K, bpu = ring.chunk_bytes / tb;
  return ring_stage(
      eng, pool, ring, (blocks + bpu - 1) / bpu, two_queues,
      [=](uint64_t u, char* dst) {
        const uint64_t j1 = std::min(blocks, (u + 1) * bpu);
        for (uint64_t j = u * bpu; j < j1; ++j) {
          const uint64_t t = j / (uint64_t)K, a = t * tb, b = std::min(row, a + tb);
          gather_range(h_seg + (size_t)(j % (uint64_t)K) * nseg, seg_bytes, nseg, a, b, dst + (j - u * bpu) * tb);
        }
      },
      [&, blocks, bpu](uint64_t u, const char* slot, int q) {
        return eng.h2d(q, d_dst + u * bpu * tb, slot, (std::min(blocks, (u + 1) * bpu) - u * bpu) * tb);
      });
}

// ONE row (client k of K) into the tile-interleaved layout, as its bytes arrive (engine.ingest):
// each unit is a run of whole tiles of the row, packed contiguous into a pinned slot and copied
// with ONE 2-D copy whose rows are the tiles (width tb, source pitch tb, destination pitch K * tb,
// first destination d_dst + (t0 * K + k) * tb).  Eng::h2d_2d(q, d, dpitch, h, spitch, width, height).
template <class Eng>
int stage_row_tiled_pipeline(Eng& eng, Pool& pool, Ring& ring, const void* const* h_seg, const uint64_t* seg_bytes,
                             int nseg, uint64_t row, uint64_t tb, int K, int k, char* d_dst, bool two_queues) {
  if (!tb || tb > ring.chunk_bytes || K <= 0 || k < 0 || k >= K) return -1;
  const uint64_t tiles = row ? (row + tb - 1) / tb : 0, tpu = ring.chunk_bytes / tb;
  return ring_stage(
      eng, pool, ring, (tiles + tpu - 1) / tpu, two_queues,
      [=](uint64_t u, char* dst) {
        const uint64_t a = u * tpu * tb;
        gather_range(h_seg, seg_bytes, nseg, a, std::min(row, a + tpu * tb), dst);
      },
      [&, tiles, tpu](uint64_t u, const char* slot, int q) {
        const uint64_t t0 = u * tpu, n = std::min(tiles, t0 + tpu) - t0;
        return eng.h2d_2d(q, d_dst + (t0 * (uint64_t)K + (uint64_t)k) * tb, (uint64_t)K * tb, slot, tb, tb, n);
      });
}

// bytes from d_src into host h_dst through the ring: D2H in super-chunks of G adjacent slots
// (one DMA of G * chunk_bytes), each slot of a super-chunk copied out by its own worker once the
// DMA's event completed.  Groups rotate over the ring.
template <class Eng>
int fetch_pipeline(Eng& eng, Pool& pool, Ring& ring, const char* d_src, char* h_dst, uint64_t bytes) {
  const uint64_t cb = ring.chunk_bytes;
  const int R = ring.size();
  const int G = std::max(1, std::min(4, R / 2));
  const int NG = R / G;
  const uint64_t sb = cb * (uint64_t)G;
  const uint64_t units = (bytes + sb - 1) / sb;
  std::vector<Done> done(R);
  std::vector<bool> pending(R, false);
  int rc = 0;
  for (uint64_t u = 0; u < units && !rc; ++u) {
    const int g0 = (int)(u % (uint64_t)NG) * G;  // first slot of this group
    for (int i = 0; i < G; ++i)
      if (pending[g0 + i]) {
        done[g0 + i].wait();
        pending[g0 + i] = false;
      }
    // (a staging copy still reading a slot is ordered before this D2H on queue 0: stage joins
    // its second queue into queue 0 before returning)
    const uint64_t a = u * sb, b = std::min(bytes, a + sb);
    rc = eng.d2h(ring.slot[g0], d_src + a, b - a);
    if (!rc) rc = eng.mark(g0, 0);
    if (rc) break;
    for (int i = 0; i < G; ++i) ring.used[g0 + i] = i == 0;
    for (int i = 0; i < G; ++i) {
      const uint64_t pa = a + (uint64_t)i * cb;
      if (pa >= b) break;
      const uint64_t pb = std::min(b, pa + cb);
      const int slot = g0 + i;
      done[slot].done = false;
      pending[slot] = true;
      const char* src = static_cast<const char*>(ring.slot[slot]);
      char* dst = h_dst + pa;
      Done* d = &done[slot];
      pool.submit([=, &eng] {
        eng.wait(g0);
        memcpy(dst, src, pb - pa);
        d->set();
      });
    }
  }
  for (int i = 0; i < R; ++i)  // copy-out tasks write the caller's buffer
    if (pending[i]) done[i].wait();
  return rc;
}

}  // namespace fedagg_host
