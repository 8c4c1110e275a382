// host_pack_probe.cpp -- the host side of MultiDeviceEngine's ingress without the GPUs
// (VERDICT r04 "Next 4"): P concurrent stage pipelines (one per GPU of a node), each with its
// own worker pool of T threads and its own staging ring, pack K client rows of B bytes each
// through host_pool.h's stage_pipeline -- the very code session.hip runs -- with a copy engine
// that completes every "H2D" at once (no DMA, no GPU).  What it measures is the host's pack
// ceiling: memcpy from the clients' arrays into the rings, which the 8 PCIe links of a node must
// not out-run.  Optional --bind: pipeline p's workers on CPUs [p*T, (p+1)*T) (a stand-in for the
// per-GPU NUMA binding; the 1-GPU box grants 16 CPUs, so P x T <= 16 there).
//
//   g++ -O3 -std=c++17 -pthread -I substrafl_amd/csrc tools/host_pack_probe.cpp -o tools/_host_pack_probe
//   tools/_host_pack_probe --configs 1x1,1x2,1x4,1x8,1x16,2x8,4x4,8x2 --mib-per-pipeline 2048
//
// Prints one JSON line per (P, T): aggregate GB/s of packed bytes, best of --reps.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "host_pool.h"

using namespace fedagg_host;

namespace {

struct NoDma {  // every copy "completes" when enqueued: the pack alone is timed
  int h2d(int, void*, const void*, uint64_t) { return 0; }
  int mark(int, int) { return 0; }
  void wait(int) {}
};

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct Pipeline {
  std::vector<std::vector<char>> rows;  // K client rows (one segment each)
  std::vector<const void*> seg;
  std::vector<uint64_t> seg_bytes;
  Ring ring;
  std::vector<char> ring_mem;
  Pool* pool = nullptr;
};

}  // namespace

int main(int argc, char** argv) {
  std::string configs = "1x1,1x2,1x4,1x8,1x16,2x8,4x4,8x2";
  uint64_t mib = 2048, chunk = 4ull << 20;
  int K = 8, reps = 3;
  bool bind = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--configs" && i + 1 < argc) configs = argv[++i];
    else if (a == "--mib-per-pipeline" && i + 1 < argc) mib = strtoull(argv[++i], nullptr, 10);
    else if (a == "--clients" && i + 1 < argc) K = atoi(argv[++i]);
    else if (a == "--reps" && i + 1 < argc) reps = atoi(argv[++i]);
    else if (a == "--bind") bind = true;
  }
  size_t pos = 0;
  while (pos < configs.size()) {
    size_t end = configs.find(',', pos);
    std::string c = configs.substr(pos, end == std::string::npos ? std::string::npos : end - pos);
    pos = end == std::string::npos ? configs.size() : end + 1;
    const int P = atoi(c.c_str()), T = atoi(c.substr(c.find('x') + 1).c_str());
    if (P < 1 || T < 1) continue;
    const uint64_t row = (mib << 20) / (uint64_t)K;
    std::vector<Pipeline> pipes(P);
    for (int p = 0; p < P; ++p) {
      Pipeline& pl = pipes[p];
      pl.rows.assign(K, std::vector<char>(row));
      for (auto& r : pl.rows) memset(r.data(), 1 + p, row);  // faulted in, like unpickled arrays
      for (auto& r : pl.rows) {
        pl.seg.push_back(r.data());
        pl.seg_bytes.push_back(row);
      }
      const int R = T + 2;
      pl.ring_mem.assign((size_t)R * chunk, 0);
      for (int s = 0; s < R; ++s) pl.ring.slot.push_back(pl.ring_mem.data() + (size_t)s * chunk);
      pl.ring.used.assign(R, false);
      pl.ring.chunk_bytes = chunk;
      std::vector<int> cpus;
      if (bind)
        for (int t = 0; t < T; ++t) cpus.push_back(p * T + t);
      pl.pool = new Pool(T, cpus);
    }
    double best = 0;
    for (int r = 0; r < reps; ++r) {
      std::vector<std::thread> th;
      const double t0 = now();
      for (int p = 0; p < P; ++p)
        th.emplace_back([&, p] {
          NoDma eng;
          Pipeline& pl = pipes[p];
          stage_pipeline(eng, *pl.pool, pl.ring, pl.seg.data(), pl.seg_bytes.data(), 1, K, 0, row, nullptr, 0,
                         false);
        });
      for (auto& t : th) t.join();
      const double dt = now() - t0;
      const double gbs = (double)P * K * row / dt / 1e9;
      if (gbs > best) best = gbs;
    }
    printf("{\"pipelines\": %d, \"threads_per_pipeline\": %d, \"threads\": %d, \"bytes_per_pipeline\": %llu, "
           "\"chunk_bytes\": %llu, \"bind\": %s, \"pack_GBps\": %.2f, \"pack_GBps_per_pipeline\": %.2f}\n",
           P, T, P * T, (unsigned long long)((uint64_t)K * row), (unsigned long long)chunk, bind ? "true" : "false",
           best, best / P);
    fflush(stdout);
    for (auto& pl : pipes) delete pl.pool;
  }
  return 0;
}
