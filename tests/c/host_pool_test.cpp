// Host-side runtime pieces of libfedagg (substrafl_amd/csrc/host_pool.h) under g++ sanitizers:
// gather_range against a byte-wise reference over random segment lists and ranges, and the
// worker pool + completion flags driven the way fedagg_session_stage / _fetch drive them
// (a ring of R slots, flags reused per slot, the flag vector destroyed as soon as the last
// wait returns).  Built and run by tests/test_host_sanitizers.py with -fsanitize=thread and
// with -fsanitize=address,undefined.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "host_pool.h"

using fedagg_host::Done;
using fedagg_host::gather_range;
using fedagg_host::Pool;
using fedagg_host::Ring;

static int check_gather(std::mt19937_64& rng) {
  const int nseg = (int)(rng() % 9);
  std::vector<std::vector<char>> segs(nseg);
  std::vector<const void*> ptr(nseg);
  std::vector<uint64_t> len(nseg);
  std::vector<char> cat;
  for (int i = 0; i < nseg; ++i) {
    segs[i].resize(rng() % 300);  // empty segments included
    for (auto& c : segs[i]) c = (char)rng();
    ptr[i] = segs[i].data();
    len[i] = segs[i].size();
    cat.insert(cat.end(), segs[i].begin(), segs[i].end());
  }
  const uint64_t total = cat.size();
  const uint64_t a = total ? rng() % (total + 1) : 0;
  const uint64_t b = a + (total - a ? rng() % (total - a + 1) : 0);
  std::vector<char> dst(b - a + 1, 0x5a);
  gather_range(ptr.data(), len.data(), nseg, a, b, dst.data());
  for (uint64_t i = a; i < b; ++i)
    if (dst[i - a] != cat[i]) return 1;
  return dst[b - a] == 0x5a ? 0 : 1;  // nothing written past the range
}

// The staging pipeline's shape: unit u is packed by a worker into slot u % R; the "copy" of unit u
// (here: a memcpy out of the slot) starts only after its flag is set; a slot is refilled only
// after the copy that read it.  Returns the number of wrong output bytes.
static long pipeline(Pool& pool, int R, int units, int unit_bytes, std::mt19937_64& rng) {
  std::vector<char> src((size_t)units * unit_bytes), out(src.size(), 0);
  for (auto& c : src) c = (char)rng();
  std::vector<std::vector<char>> ring(R, std::vector<char>(unit_bytes));
  {
    std::vector<Done> done(R);
    int next = 0;
    auto submit = [&](int u) {
      Done& d = done[u % R];
      d.done = false;
      char* slot = ring[u % R].data();
      const char* s = src.data() + (size_t)u * unit_bytes;
      pool.submit([=, &d] {
        memcpy(slot, s, unit_bytes);
        d.set();
      });
    };
    for (; next < units && next + 1 < R; ++next) submit(next);
    for (int u = 0; u < units; ++u) {
      done[u % R].wait();
      memcpy(out.data() + (size_t)u * unit_bytes, ring[u % R].data(), unit_bytes);
      if (next < units) submit(next++);
    }
  }  // flags destroyed right after the last wait: set() must not touch them after releasing
  long bad = 0;
  for (size_t i = 0; i < src.size(); ++i) bad += src[i] != out[i];
  return bad;
}

// ------------------------------------------------------------------------------------------
// The session's real staging / fetch pipelines (fedagg_host::stage_pipeline / fetch_pipeline)
// over a fake copy engine: one "DMA" thread executes the enqueued copies in order, slot events
// complete when the DMA passed them, and the n-th copy can be made to fail (the HIP error path:
// ADVICE r01 -- pending pack / copy-out tasks must be drained before the call returns).
// ------------------------------------------------------------------------------------------
struct FakeDma {
  struct Job {
    char* dst;
    const char* src;
    uint64_t n;
    uint64_t seq;
  };
  std::mutex m;
  std::condition_variable cv;
  std::deque<Job> q;
  uint64_t enq = 0, doneseq = 0;
  std::vector<uint64_t> ev;  // per slot: sequence number the slot's event waits for
  bool stop = false;
  uint64_t fail_at = 0, calls = 0;
  std::thread th;
  explicit FakeDma(int slots) : ev(slots, 0) {
    th = std::thread([this] {
      for (;;) {
        Job j;
        {
          std::unique_lock<std::mutex> l(m);
          cv.wait(l, [this] { return stop || !q.empty(); });
          if (q.empty()) return;
          j = q.front();
          q.pop_front();
        }
        memcpy(j.dst, j.src, j.n);
        std::lock_guard<std::mutex> g(m);
        doneseq = j.seq;
        cv.notify_all();
      }
    });
  }
  ~FakeDma() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
  int copy(void* d, const void* s, uint64_t n) {
    if (fail_at && ++calls >= fail_at) return -2;
    std::lock_guard<std::mutex> g(m);
    q.push_back({static_cast<char*>(d), static_cast<const char*>(s), n, ++enq});
    cv.notify_all();
    return 0;
  }
  int h2d(int, void* d, const void* s, uint64_t n) { return copy(d, s, n); }
  int h2d_2d(int, void* d, uint64_t dpitch, const void* s, uint64_t spitch, uint64_t w, uint64_t h) {
    for (uint64_t i = 0; i < h; ++i) {
      const int rc = copy(static_cast<char*>(d) + i * dpitch, static_cast<const char*>(s) + i * spitch, w);
      if (rc) return rc;
    }
    return 0;
  }
  int d2h(void* h, const void* d, uint64_t n) { return copy(h, d, n); }
  int mark(int slot, int) {
    std::lock_guard<std::mutex> g(m);
    ev[slot] = enq;
    return 0;
  }
  void wait(int slot) {
    std::unique_lock<std::mutex> l(m);
    const uint64_t want = ev[slot];
    cv.wait(l, [&] { return doneseq >= want; });
  }
  void drain() {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [&] { return doneseq >= enq; });
  }
};

// K client rows of random segments staged through a ring into a "device" buffer and fetched
// back; with fail_at, the fail_at-th copy fails and the call must return the error cleanly.
static int staging_round_trip(Pool& pool, std::mt19937_64& rng, uint64_t fail_at, bool check) {
  const int K = 1 + (int)(rng() % 6), nseg = 1 + (int)(rng() % 5), R = pool.size() + 2 + (int)(rng() % 3);
  const uint64_t cb = 64 * (1 + rng() % 8);  // small chunks: many units
  std::vector<uint64_t> len(nseg);
  uint64_t row = 0;
  for (auto& l : len) row += (l = 4 * (rng() % 200));  // whole floats
  std::vector<std::vector<std::vector<float>>> data(K, std::vector<std::vector<float>>(nseg));
  std::vector<const void*> segs((size_t)K * nseg);
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < nseg; ++i) {
      auto& v = data[k][i];
      v.resize(len[i] / 4);
      for (auto& f : v) f = (float)(int)(rng() % 7) - 3.0f;
      if (check && k > 0 && rng() % 2) v = data[0][i];  // mostly identical copies of c
      if (check && k > 0 && !v.empty() && rng() % 3 == 0) v[0] = -v[0] + 1.0f;
      segs[(size_t)k * nseg + i] = v.data();
    }
  std::vector<char> ring_mem((size_t)R * cb);
  Ring ring;
  ring.chunk_bytes = cb;
  for (int i = 0; i < R; ++i) ring.slot.push_back(ring_mem.data() + (size_t)i * cb);
  ring.used.assign(R, false);
  const uint64_t ld = row + 16;
  std::vector<char> dev((size_t)K * ld, 0), back(dev.size(), 0);
  FakeDma dma(R);
  dma.fail_at = fail_at;
  uint64_t mism = 0;
  int rc = fedagg_host::stage_pipeline(dma, pool, ring, segs.data(), len.data(), nseg, K, 0, row, dev.data(), ld,
                                       true, check ? 4 : 0, &mism);
  dma.drain();
  if (fail_at) {
    const uint64_t units = (row ? (row + cb - 1) / cb : 0) * (check ? 1 : K);
    return (fail_at <= units) == (rc != 0) ? 0 : 1;  // an error exactly when the failing copy was reached
  }
  if (rc) return 1;
  if (check) {  // row 0 staged, the mismatch count is the value comparison of the others
    uint64_t want = 0;
    for (int k = 1; k < K; ++k)
      for (int i = 0; i < nseg; ++i)
        for (size_t e = 0; e < data[k][i].size(); ++e) want += data[k][i][e] != data[0][i][e];
    if (want != mism) return 1;
  }
  for (int k = 0; k < (check ? 1 : K); ++k) {
    uint64_t off = 0;
    for (int i = 0; i < nseg; ++i) {
      if (len[i] && memcmp(dev.data() + (size_t)k * ld + off, data[k][i].data(), len[i])) return 1;
      off += len[i];
    }
  }
  rc = fedagg_host::fetch_pipeline(dma, pool, ring, dev.data(), back.data(), dev.size());
  dma.drain();
  if (rc) return 1;
  return memcmp(back.data(), dev.data(), dev.size()) ? 1 : 0;
}

// The tile-interleaved staging (fedagg_session_stage_tiled): K rows of random segments -> tile t
// of row k at block t * K + k; every row byte lands where the layout puts it; with fail_at, the
// fail_at-th copy fails and the call returns the error after its packs drained.
static int tiled_round_trip(Pool& pool, std::mt19937_64& rng, uint64_t fail_at) {
  const int K = 1 + (int)(rng() % 7), nseg = 1 + (int)(rng() % 4), R = pool.size() + 2 + (int)(rng() % 3);
  const uint64_t tb = 16 * (1 + rng() % 8), cb = tb * (1 + rng() % 5);
  std::vector<uint64_t> len(nseg);
  uint64_t row = 0;
  for (auto& l : len) row += (l = 4 * (rng() % 150));
  std::vector<std::vector<std::vector<char>>> data(K, std::vector<std::vector<char>>(nseg));
  std::vector<const void*> segs((size_t)K * nseg);
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < nseg; ++i) {
      data[k][i].resize(len[i]);
      for (auto& c : data[k][i]) c = (char)rng();
      segs[(size_t)k * nseg + i] = data[k][i].data();
    }
  std::vector<char> ring_mem((size_t)R * cb);
  Ring ring;
  ring.chunk_bytes = cb;
  for (int i = 0; i < R; ++i) ring.slot.push_back(ring_mem.data() + (size_t)i * cb);
  ring.used.assign(R, false);
  const uint64_t tiles = (row + tb - 1) / tb;
  std::vector<char> dev((size_t)(tiles * K * tb) + 1, 0);
  FakeDma dma(R);
  dma.fail_at = fail_at;
  const bool per_row = rng() % 2 == 0;  // all rows at once, or one row at a time (engine.ingest)
  int rc = 0;
  if (per_row) {
    for (int k = 0; k < K && !rc; ++k)
      rc = fedagg_host::stage_row_tiled_pipeline(dma, pool, ring, segs.data() + (size_t)k * nseg, len.data(), nseg, row,
                                                 tb, K, k, dev.data(), true);
  } else {
    rc = fedagg_host::stage_tiled_pipeline(dma, pool, ring, segs.data(), len.data(), nseg, K, row, tb, dev.data(),
                                           true);
  }
  dma.drain();
  if (fail_at) {
    const uint64_t bpu = cb / tb;  // per_row: one 2-D copy per unit, one fake copy per tile
    const uint64_t copies = per_row ? tiles * K : (tiles * K + bpu - 1) / bpu;
    return (fail_at <= copies) == (rc != 0) ? 0 : 1;
  }
  if (rc) return 1;
  for (int k = 0; k < K; ++k) {
    std::vector<char> flat;
    for (int i = 0; i < nseg; ++i) flat.insert(flat.end(), data[k][i].begin(), data[k][i].end());
    for (uint64_t b = 0; b < row; ++b)
      if (dev[(size_t)(((b / tb) * K + k) * tb + b % tb)] != flat[b]) return 1;
  }
  return dev.back() == 0 ? 0 : 1;  // nothing written past the layout
}

static int fetch_with_failure(Pool& pool, std::mt19937_64& rng) {
  const int R = pool.size() + 2;
  const uint64_t cb = 256;
  std::vector<char> ring_mem((size_t)R * cb);
  Ring ring;
  ring.chunk_bytes = cb;
  for (int i = 0; i < R; ++i) ring.slot.push_back(ring_mem.data() + (size_t)i * cb);
  ring.used.assign(R, false);
  const uint64_t bytes = 1 + rng() % 20000;
  std::vector<char> dev(bytes), host(bytes);
  for (auto& c : dev) c = (char)rng();
  FakeDma dma(R);
  dma.fail_at = 1 + rng() % 6;
  int rc = fedagg_host::fetch_pipeline(dma, pool, ring, dev.data(), host.data(), bytes);
  dma.drain();
  const int G = std::max(1, std::min(4, R / 2));
  const uint64_t units = (bytes + cb * G - 1) / (cb * G);
  return (dma.fail_at <= units) == (rc != 0) ? 0 : 1;
}

// check_rows (the compare-only Scaffold c check) from several threads while a staging pipeline
// runs on the same pool -- the ingest path of engine.py does exactly this.
static int concurrent_checks(Pool& pool, std::mt19937_64& rng) {
  const int nseg = 3, K = 2;
  std::vector<std::vector<float>> ref(nseg), x(nseg);
  std::vector<uint64_t> len(nseg);
  for (int i = 0; i < nseg; ++i) {
    ref[i].resize(50000 + rng() % 400000);
    for (auto& f : ref[i]) f = (float)(int)(rng() % 1000);
    x[i] = ref[i];
    len[i] = ref[i].size() * 4;
  }
  x[1][17] += 1.0f;
  x[2][x[2].size() - 1] = -x[2][x[2].size() - 1] + 0.5f;
  std::vector<const void*> segs;
  for (int i = 0; i < nseg; ++i) segs.push_back(ref[i].data());
  for (int i = 0; i < nseg; ++i) segs.push_back(x[i].data());
  uint64_t row = 0;
  for (auto l : len) row += l;
  std::vector<uint64_t> got(4, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] { got[t] = fedagg_host::check_rows(pool, segs.data(), len.data(), nseg, K, 0, row, 4); });
  const int bad = staging_round_trip(pool, rng, 0, false);
  for (auto& t : th) t.join();
  for (auto g : got)
    if (g != 2) return 1;
  return bad;
}

int main() {
  std::mt19937_64 rng(20241016);
  for (int t = 0; t < 4000; ++t)
    if (check_gather(rng)) {
      fprintf(stderr, "gather_range mismatch (trial %d)\n", t);
      return 1;
    }
  for (int threads : {1, 3, 8}) {
    Pool pool(threads);
    for (int rep = 0; rep < 60; ++rep) {
      const int R = threads + 2 + (int)(rng() % 3);
      const long bad = pipeline(pool, R, 1 + (int)(rng() % 40), 64 + (int)(rng() % 4096), rng);
      if (bad) {
        fprintf(stderr, "pipeline: %ld wrong bytes (threads %d, rep %d)\n", bad, threads, rep);
        return 1;
      }
    }
  }
  for (int threads : {1, 4}) {
    Pool pool(threads);
    for (int rep = 0; rep < 80; ++rep) {
      const bool check = rep % 2 == 1;
      const uint64_t fail_at = rep % 3 == 2 ? 1 + rng() % 12 : 0;
      if (staging_round_trip(pool, rng, fail_at, check)) {
        fprintf(stderr, "stage/fetch pipeline failed (threads %d, rep %d, fail_at %llu)\n", threads, rep,
                (unsigned long long)fail_at);
        return 1;
      }
      if (tiled_round_trip(pool, rng, rep % 4 == 3 ? 1 + rng() % 10 : 0)) {
        fprintf(stderr, "tiled stage pipeline failed (threads %d, rep %d)\n", threads, rep);
        return 1;
      }
      if (fetch_with_failure(pool, rng)) {
        fprintf(stderr, "fetch pipeline error path failed (threads %d, rep %d)\n", threads, rep);
        return 1;
      }
    }
  }
  {
    Pool pool(4);
    for (int rep = 0; rep < 20; ++rep)
      if (concurrent_checks(pool, rng)) {
        fprintf(stderr, "concurrent check_rows failed (rep %d)\n", rep);
        return 1;
      }
  }
  printf("host_pool_test: ok\n");
  return 0;
}
