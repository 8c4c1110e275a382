// Stream-priority probe: does a small copy kernel on a second stream (the shape of an RCCL P2P
// kernel: a few workgroups moving a message) get CUs while the client-shard chain kernel fills
// the chip, and does a high-priority stream (hipStreamCreateWithPriority) change that?
//
// The chain kernel is the product's own (fedagg_fedavg_chain_f32, 64 clients x N elements, rows),
// launched on the compute stream; ~200 us later the copy kernel (W workgroups x 256 threads,
// 16-B vectors, B bytes) is launched on the "communicator" stream.  Reported per configuration
// (median over the trials): the copy's latency from its stream's start event to its end event,
// the chain kernel's time, and both alone.  A copy that waits for the chain kernel to drain shows
// a latency near the chain kernel's remaining time; one that gets CUs shows about its own time.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/priority_probe.hip -Iinclude \
//          -Lsubstrafl_amd -lfedagg -Wl,-rpath,'$ORIGIN/../substrafl_amd' -o tools/_priority_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "fedagg.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct alignas(16) v4 {
  unsigned x, y, z, w;
};

__global__ void __launch_bounds__(256) copy_kernel(const v4* __restrict__ src, v4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) dst[i] = src[i];
}

static float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int K = 64;
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (16ull << 20);  // elements per client
  const size_t bytes = argc > 2 ? strtoull(argv[2], nullptr, 10) : (32ull << 20);  // copy message
  const int wgs = argc > 3 ? atoi(argv[3]) : 16;
  const int trials = 15;
  const int delay_us = 200;
  float* rows;
  float* acc;
  v4 *src, *dst;
  CK(hipMalloc((void**)&rows, K * n * sizeof(float)));
  CK(hipMalloc((void**)&acc, n * sizeof(float)));
  CK(hipMalloc((void**)&src, bytes));
  CK(hipMalloc((void**)&dst, bytes));
  CK(hipMemset(rows, 0, K * n * sizeof(float)));
  CK(hipMemset(src, 1, bytes));
  std::vector<const float*> ptrs(K);
  std::vector<float> w(K, 1.0f / K);
  for (int k = 0; k < K; ++k) ptrs[k] = rows + k * n;
  int lo, hi;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t sc, sn, sh;
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&sn, hipStreamNonBlocking, lo));
  CK(hipStreamCreateWithPriority(&sh, hipStreamNonBlocking, hi));
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  const size_t nv = bytes / 16;
  auto chain = [&](hipStream_t s) {
    int rc = fedagg_fedavg_chain_f32(ptrs.data(), w.data(), K, n, 1, acc, s);
    if (rc) {
      fprintf(stderr, "chain: %s\n", fedagg_last_error());
      exit(1);
    }
  };
  auto copy = [&](hipStream_t s) { copy_kernel<<<wgs, 256, 0, s>>>(src, dst, nv); };
  // warm-up
  for (int i = 0; i < 3; ++i) {
    chain(sc);
    copy(sn);
    copy(sh);
  }
  CK(hipDeviceSynchronize());
  std::vector<float> chain_alone, copy_alone;
  for (int i = 0; i < trials; ++i) {
    CK(hipEventRecord(a0, sc));
    chain(sc);
    CK(hipEventRecord(a1, sc));
    CK(hipEventSynchronize(a1));
    float ms;
    CK(hipEventElapsedTime(&ms, a0, a1));
    chain_alone.push_back(ms);
    CK(hipEventRecord(b0, sn));
    copy(sn);
    CK(hipEventRecord(b1, sn));
    CK(hipEventSynchronize(b1));
    CK(hipEventElapsedTime(&ms, b0, b1));
    copy_alone.push_back(ms);
  }
  printf("{\"elements_per_client\": %llu, \"clients\": %d, \"copy_bytes\": %zu, \"copy_workgroups\": %d, "
         "\"priority_range\": [%d, %d], \"chain_alone_ms\": %.4f, \"copy_alone_ms\": %.4f}\n",
         (unsigned long long)n, K, bytes, wgs, lo, hi, median(chain_alone), median(copy_alone));
  for (int cfg = 0; cfg < 2; ++cfg) {
    hipStream_t s2 = cfg ? sh : sn;
    std::vector<float> lat, chain_t, start_off;
    for (int i = 0; i < trials; ++i) {
      CK(hipEventRecord(a0, sc));
      chain(sc);
      CK(hipEventRecord(a1, sc));
      std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
      CK(hipEventRecord(b0, s2));
      copy(s2);
      CK(hipEventRecord(b1, s2));
      CK(hipDeviceSynchronize());
      float l, c, o;
      CK(hipEventElapsedTime(&l, b0, b1));
      CK(hipEventElapsedTime(&c, a0, a1));
      CK(hipEventElapsedTime(&o, a0, b0));
      lat.push_back(l);
      chain_t.push_back(c);
      start_off.push_back(o);
    }
    printf("{\"copy_stream\": \"%s\", \"copy_latency_ms\": %.4f, \"copy_latency_max_ms\": %.4f, "
           "\"copy_start_after_chain_start_ms\": %.4f, \"chain_ms\": %.4f}\n",
           cfg ? "high priority" : "normal priority", median(lat), *std::max_element(lat.begin(), lat.end()),
           median(start_off), median(chain_t));
  }
  CK(hipFree(rows));
  CK(hipFree(acc));
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
