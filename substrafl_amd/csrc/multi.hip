// multi.hip -- one process, several GPUs: the parameter-range FedAvg of an aggregate task in ONE
// C call (SURVEY.md §8(b) "fa_multi_init / fa_reduce_sharded_*", §8(e) primary partitioning).
//
// A Substra aggregate task is one OS process (remote/register/register.py:96 runs one
// function.py), so a host that wants the node's GPUs drives them from one process.  The Python
// drop-in does that in substrafl_amd/multi_device.py (MultiDeviceEngine); this is the same plan for
// a host in another language, without Python:
//   * the flat bucket range [0, M) is cut into one contiguous, 512-element-aligned shard per
//     device (sharding.shard_bounds);
//   * one thread and one private session per shard (repeated device indices get their own
//     sessions, so a one-GPU box exercises the sharded path), its pack workers and pinned ring
//     placed on the GPU's NUMA node (multi_device.host_placement);
//   * the thread streams its shard through its GPU in sub-ranges sized to the free HBM
//     (out-of-core past 288 GB): stage bytes [lo, hi) of every client's row over the GPU's own
//     PCIe link (fedagg_session_stage_range), run the bucket kernel with the client order and the
//     numel == 1 patch of the elements it owns, fetch its slice straight into the caller's output.
// Every output element is computed by the single-GPU kernel's arithmetic, so the result is bit-
// identical to fedagg_fedavg_* over the whole range and to the reference (fed_avg.py:217-222): no
// collective, no re-association.

#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fedagg.h"

namespace fedagg_internal {
void set_error(const char* msg);
}

namespace {

constexpr uint64_t kShardAlign = 512;     // elements: every shard row starts 256-B aligned (sharding.SHARD_ALIGN)
constexpr uint64_t kRowAlignBytes = 256;  // row stride of a staged [K, ld] bucket (layout.ROW_ALIGN_BYTES)
constexpr double kHeadroom = 0.85;        // share of free HBM one sub-range may take (multi_device.HBM_HEADROOM)
constexpr int kPackThreadsCap = 32;       // pack workers per GPU past which staging stops scaling
enum { kSlotBucket = 0, kSlotOut = 1, kSlotWs = 2 };

int fail(const std::string& msg) {
  fedagg_internal::set_error(msg.c_str());
  return FEDAGG_EINVAL;
}

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const std::string& text) {
  std::vector<int> out;
  size_t i = 0;
  while (i < text.size()) {
    size_t j = text.find(',', i);
    if (j == std::string::npos) j = text.size();
    std::string part = text.substr(i, j - i);
    while (!part.empty() && isspace((unsigned char)part.back())) part.pop_back();
    if (!part.empty()) {
      int a = 0, b = 0;
      if (sscanf(part.c_str(), "%d-%d", &a, &b) == 2)
        for (int c = a; c <= b; ++c) out.push_back(c);
      else if (sscanf(part.c_str(), "%d", &a) == 1)
        out.push_back(a);
    }
    i = j + 1;
  }
  return out;
}

std::string read_file(const std::string& path) {
  std::string s;
  if (FILE* f = fopen(path.c_str(), "r")) {
    char buf[4096];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, n);
    fclose(f);
  }
  return s;
}

// NUMA node of a GPU (sysfs numa_node of its PCI function), -1 when unknown
int gpu_numa_node(int device) {
  char bus[64] = {};
  if (fedagg_device_pci_bus_id(device, bus, sizeof(bus)) != FEDAGG_OK) return -1;
  for (char* p = bus; *p; ++p) *p = (char)tolower((unsigned char)*p);
  std::string t = read_file(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
  int node = -1;
  if (t.empty() || sscanf(t.c_str(), "%d", &node) != 1) return -1;
  return node;
}

std::vector<int> allowed_cpus() {
  std::vector<int> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return out;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

uint64_t row_ld(uint64_t n, uint64_t esz) {  // multi_device._ld
  const uint64_t per_row = std::max<uint64_t>(1, kRowAlignBytes / esz);
  return std::max(per_row, (n + per_row - 1) / per_row * per_row);
}

struct Shard {
  int device = 0;
  fedagg_session* s = nullptr;
  int numa_node = -1;
  int threads = 0;
  std::vector<int> cpus;
  uint64_t held[3] = {0, 0, 0};  // bytes of the session buffer slots this engine grew
  // the last call
  uint64_t lo = 0, hi = 0;
  int ranges = 0;
  double stage_s = 0, kernel_fetch_s = 0;
};

}  // namespace

struct fedagg_multi {
  std::vector<Shard> shards;
  uint64_t max_shard_bytes = 0;  // 0: kHeadroom of the device's free HBM
  std::mutex m;                  // one aggregation at a time per engine
};

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int shard_buffer(Shard& sh, int slot, uint64_t bytes, void** d) {
  int rc = fedagg_session_buffer(sh.s, slot, bytes, d);
  if (rc == FEDAGG_OK) sh.held[slot] = std::max(sh.held[slot], bytes);
  return rc;
}

// HBM one sub-range of shard g may take: its free HBM plus the buffers the call reuses
int shard_budget(fedagg_multi* m, Shard& sh, uint64_t* budget) {
  if (m->max_shard_bytes) {
    *budget = m->max_shard_bytes;
    return FEDAGG_OK;
  }
  uint64_t free_b = 0, total_b = 0;
  int rc = fedagg_device_memory(sh.device, &free_b, &total_b);
  if (rc) return rc;
  *budget = (uint64_t)((double)(free_b + sh.held[0] + sh.held[1] + sh.held[2]) * kHeadroom);
  return FEDAGG_OK;
}

template <class T>
struct KernelOf;
template <>
struct KernelOf<float> {
  static int run(const float* const* rows, const void* w, int K, uint64_t n, const uint64_t* idx, int P, void* ws,
                 void* out, void* stream) {
    return fedagg_fedavg_f32(rows, static_cast<const float*>(w), K, n, idx, P, ws, static_cast<float*>(out), stream);
  }
};
template <>
struct KernelOf<double> {
  static int run(const double* const* rows, const void* w, int K, uint64_t n, const uint64_t* idx, int P, void* ws,
                 void* out, void* stream) {
    return fedagg_fedavg_f64(rows, static_cast<const double*>(w), K, n, idx, P, ws, static_cast<double*>(out),
                             stream);
  }
};

template <>
struct KernelOf<uint16_t> {  // fp16 buckets (bit patterns), fp16 weights and output: NumPy's half loops
  static int run(const uint16_t* const* rows, const void* w, int K, uint64_t n, const uint64_t* idx, int P, void* ws,
                 void* out, void* stream) {
    return fedagg_fedavg_f16(rows, static_cast<const uint16_t*>(w), K, n, idx, P, ws, static_cast<uint16_t*>(out),
                             stream);
  }
};

// One shard: its sub-ranges through its GPU, in order.
template <class T>
int run_shard(fedagg_multi* m, Shard& sh, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
              const void* h_w, const std::vector<uint64_t>& idx, T* h_out, size_t ws_bytes) {
  const uint64_t esz = sizeof(T);
  sh.ranges = 0;
  sh.stage_s = sh.kernel_fetch_s = 0;
  if (sh.hi <= sh.lo) return FEDAGG_OK;
  int rc = fedagg_session_activate(sh.s);
  if (rc) return rc;
  uint64_t budget = 0;
  if ((rc = shard_budget(m, sh, &budget))) return rc;
  uint64_t cap = std::max<uint64_t>(kShardAlign, budget / ((uint64_t)(K + 1) * esz));
  const uint64_t step = std::max(kShardAlign, cap / kShardAlign * kShardAlign);  // multi_device._split
  std::vector<const T*> rows(K);
  std::vector<uint64_t> pw;
  for (uint64_t lo = sh.lo; lo < sh.hi; lo += step) {
    const uint64_t hi = std::min(sh.hi, lo + step), n = hi - lo, ld = row_ld(n, esz);
    const double t0 = now_s();
    void *d_bucket = nullptr, *d_out = nullptr, *d_ws = nullptr;
    if ((rc = shard_buffer(sh, kSlotBucket, (uint64_t)K * ld * esz, &d_bucket))) return rc;
    if ((rc = fedagg_session_stage_range(sh.s, d_bucket, ld * esz, K, nseg, h_seg, seg_bytes, lo * esz, hi * esz)))
      return rc;
    const double t1 = now_s();
    if ((rc = shard_buffer(sh, kSlotOut, ld * esz, &d_out))) return rc;
    if ((rc = shard_buffer(sh, kSlotWs, ws_bytes, &d_ws))) return rc;
    pw.clear();
    for (uint64_t i : idx)
      if (i >= lo && i < hi) pw.push_back(i - lo);
    for (int k = 0; k < K; ++k)
      rows[k] = reinterpret_cast<const T*>(static_cast<const char*>(d_bucket) + (uint64_t)k * ld * esz);
    if ((rc = KernelOf<T>::run(rows.data(), h_w, K, n, pw.empty() ? nullptr : pw.data(), (int)pw.size(), d_ws, d_out,
                               fedagg_session_stream(sh.s))))
      return rc;
    if ((rc = fedagg_session_fetch(sh.s, d_out, h_out + lo, n * esz))) return rc;
    sh.stage_s += t1 - t0;
    sh.kernel_fetch_s += now_s() - t1;
    ++sh.ranges;
  }
  return FEDAGG_OK;
}

template <class T>
int multi_fedavg(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                 const void* h_w, const uint64_t* h_idx, int P, T* h_out, const char* name) {
  if (!m || K <= 0 || nseg < 0 || (nseg > 0 && (!h_seg || !seg_bytes)) || !h_w || P < 0 || (P > 0 && !h_idx) ||
      !h_out)
    return fail(std::string(name) + ": invalid argument");
  uint64_t row = 0;
  for (int i = 0; i < nseg; ++i) {
    if (seg_bytes[i] % sizeof(T)) return fail(std::string(name) + ": segment not a whole number of elements");
    row += seg_bytes[i];
  }
  const uint64_t M = row / sizeof(T);
  std::vector<uint64_t> idx(h_idx, h_idx + P);
  for (uint64_t i : idx)
    if (i >= M) return fail(std::string(name) + ": numel == 1 index out of range");
  if (M == 0) return FEDAGG_OK;
  std::lock_guard<std::mutex> g(m->m);
  int caller = -1;
  (void)hipGetDevice(&caller);
  // shard_bounds(M, G): equal, 512-element-multiple chunks; the last shards may get less or nothing
  const uint64_t G = m->shards.size();
  uint64_t chunk = (M + G - 1) / G;
  chunk = (chunk + kShardAlign - 1) / kShardAlign * kShardAlign;
  for (uint64_t gi = 0; gi < G; ++gi) {
    m->shards[gi].lo = std::min(M, gi * chunk);
    m->shards[gi].hi = std::min(M, (gi + 1) * chunk);
  }
  const size_t ws_bytes = fedagg_pairwise_ws_bytes(K, std::max(1, P), 8);
  std::vector<int> rcs(G, FEDAGG_OK);
  std::vector<std::string> errs(G);
  std::vector<std::thread> th;
  int spawn_rc = FEDAGG_OK;
  try {
    for (uint64_t gi = 0; gi < G; ++gi)
      th.emplace_back([&, gi] {
        rcs[gi] = run_shard<T>(m, m->shards[gi], K, nseg, h_seg, seg_bytes, h_w, idx, h_out, ws_bytes);
        if (rcs[gi]) errs[gi] = fedagg_last_error();  // the error text is per thread: carry it back
      });
  } catch (const std::exception& e) {  // no thread for a shard: the started ones finish, the call fails
    spawn_rc = FEDAGG_EINVAL;
    errs.assign(G, std::string("cannot start a shard thread: ") + e.what());
  }
  for (auto& t : th) t.join();
  if (spawn_rc) {
    if (caller >= 0) (void)hipSetDevice(caller);
    return fail(std::string(name) + ": " + errs[0]);
  }
  if (caller >= 0) (void)hipSetDevice(caller);  // the caller's later work stays on its own device
  for (uint64_t gi = 0; gi < G; ++gi)
    if (rcs[gi]) {
      char buf[640];
      snprintf(buf, sizeof(buf), "%s: shard %d (device %d): %s", name, (int)gi, m->shards[gi].device, errs[gi].c_str());
      fedagg_internal::set_error(buf);
      return rcs[gi];
    }
  return FEDAGG_OK;
}

}  // namespace

extern "C" {

fedagg_multi* fedagg_multi_create(int ndev, const int* devs, int pack_threads) {
  if (ndev <= 0 || !devs || pack_threads < 0 || pack_threads > 256) {
    fail("fedagg_multi_create: need ndev >= 1 device indices and 0 <= pack_threads <= 256");
    return nullptr;
  }
  int caller = -1;
  (void)hipGetDevice(&caller);
  auto* m = new (std::nothrow) fedagg_multi();
  if (!m) {
    fail("fedagg_multi_create: out of host memory");
    return nullptr;
  }
  const std::vector<int> allowed = allowed_cpus();
  const int per = pack_threads ? pack_threads
                               : std::max(2, std::min(kPackThreadsCap, (int)allowed.size() / ndev));
  for (int g = 0; g < ndev; ++g) {
    Shard sh;
    sh.device = devs[g];
    sh.s = fedagg_session_create(devs[g]);  // a private session: its buffers, ring and workers
    if (!sh.s) {
      std::string e = fedagg_last_error();
      for (auto& o : m->shards) fedagg_session_destroy(o.s);
      delete m;
      if (caller >= 0) (void)hipSetDevice(caller);
      fail("fedagg_multi_create: device " + std::to_string(devs[g]) + ": " + e);
      return nullptr;
    }
    sh.threads = per;
    sh.numa_node = gpu_numa_node(devs[g]);
    if (sh.numa_node >= 0) {  // the allowed CPUs of the GPU's node (multi_device.node_cpus)
      std::vector<int> node = parse_cpulist(
          read_file("/sys/devices/system/node/node" + std::to_string(sh.numa_node) + "/cpulist"));
      for (int c : node)
        if (std::find(allowed.begin(), allowed.end(), c) != allowed.end()) sh.cpus.push_back(c);
    }
    int rc = fedagg_session_set(sh.s, "threads", per);
    if (!rc) rc = fedagg_session_affinity(sh.s, sh.cpus.data(), (int)sh.cpus.size());
    if (rc) {
      std::string e = fedagg_last_error();
      fedagg_session_destroy(sh.s);
      for (auto& o : m->shards) fedagg_session_destroy(o.s);
      delete m;
      if (caller >= 0) (void)hipSetDevice(caller);
      fail("fedagg_multi_create: placement of device " + std::to_string(devs[g]) + ": " + e);
      return nullptr;
    }
    m->shards.push_back(std::move(sh));
  }
  if (caller >= 0) (void)hipSetDevice(caller);
  return m;
}

void fedagg_multi_destroy(fedagg_multi* m) {
  if (!m) return;
  int caller = -1;
  (void)hipGetDevice(&caller);
  {
    std::lock_guard<std::mutex> g(m->m);
    for (auto& sh : m->shards) fedagg_session_destroy(sh.s);
  }
  if (caller >= 0) (void)hipSetDevice(caller);
  delete m;
}

int fedagg_multi_set(fedagg_multi* m, const char* key, long long value) {
  if (!m || !key) return fail("fedagg_multi_set: invalid argument");
  std::lock_guard<std::mutex> g(m->m);
  if (!strcmp(key, "max_shard_bytes") && value >= 0) {
    m->max_shard_bytes = (uint64_t)value;
    return FEDAGG_OK;
  }
  if (!strcmp(key, "threads") && value >= 1 && value <= 256) {
    for (auto& sh : m->shards) {
      int rc = fedagg_session_set(sh.s, "threads", value);
      if (rc) return rc;
      sh.threads = (int)value;
    }
    return FEDAGG_OK;
  }
  return fail("fedagg_multi_set: unknown key or bad value");
}

int fedagg_multi_fedavg_f32(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                            const float* h_w, const uint64_t* h_idx, int P, float* h_out) {
  return multi_fedavg<float>(m, K, nseg, h_seg, seg_bytes, h_w, h_idx, P, h_out, "fedagg_multi_fedavg_f32");
}

int fedagg_multi_fedavg_f64(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                            const double* h_w, const uint64_t* h_idx, int P, double* h_out) {
  return multi_fedavg<double>(m, K, nseg, h_seg, seg_bytes, h_w, h_idx, P, h_out, "fedagg_multi_fedavg_f64");
}

int fedagg_multi_fedavg_f16(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                            const uint16_t* h_w, const uint64_t* h_idx, int P, uint16_t* h_out) {
  return multi_fedavg<uint16_t>(m, K, nseg, h_seg, seg_bytes, h_w, h_idx, P, h_out, "fedagg_multi_fedavg_f16");
}

int fedagg_multi_shard_info(fedagg_multi* m, int g, int* device, int* numa_node, int* threads, int* ncpus,
                            uint64_t* lo, uint64_t* hi, int* ranges) {
  if (!m || g < 0 || g >= (int)m->shards.size()) return fail("fedagg_multi_shard_info: no such shard");
  std::lock_guard<std::mutex> lk(m->m);
  const Shard& sh = m->shards[g];
  if (device) *device = sh.device;
  if (numa_node) *numa_node = sh.numa_node;
  if (threads) *threads = sh.threads;
  if (ncpus) *ncpus = (int)sh.cpus.size();
  if (lo) *lo = sh.lo;
  if (hi) *hi = sh.hi;
  if (ranges) *ranges = sh.ranges;
  return FEDAGG_OK;
}

}  // extern "C"
