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
  printf("host_pool_test: ok\n");
  return 0;
}
