// Compute / exchange overlap probe for the lockstep executor (csrc/lockstep.hip) on ONE GPU.
//
// The executor issues, per step t: on the communicator's stream, after an event of the compute
// stream (step t - 1 done), the exchange group t (RCCL P2P kernels: a few workgroups per peer,
// link-rate bound); on the compute stream, after group t - 1's event, step t's chain kernel
// (64 clients x n elements).  The schedule's efficiency rests on group t's kernels running WHILE
// step t's chain kernel runs.  A probe question the 8-GPU node cannot be asked in isolation:
// does a small kernel on the second stream get CUs while the chain kernel fills the chip?
//
// Stand-in for the exchange: a copy kernel of W workgroups moving B bytes (a few workgroups move
// a message at roughly one xGMI link's rate).  Configurations, S steps each (median of trials):
//   compute_only   the S chain launches back to back
//   copy_only      the S copy launches back to back
//   lockstep       the executor's issue pattern (events both ways, as lockstep.hip)
//   lockstep_hi    the same with the communicator stream at the greatest priority
//   lockstep_mask  compute stream CU-masked to exclude R CUs, communicator stream on those R CUs
//   lockstep_cap   the chain kernel's grid capped (fedagg_tune grid_cap) so CUs keep free slots
// overlap = (compute_only + copy_only - lockstep) / min(compute_only, copy_only): 1 = full overlap.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/overlap_probe.hip -Iinclude \
//          -Lsubstrafl_amd -lfedagg -Wl,-rpath,'$ORIGIN/../substrafl_amd' -o tools/_overlap_probe
// Usage: tools/_overlap_probe [n_elements_per_client] [copy_bytes] [copy_workgroups] [steps] [reserved_cus]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 3900000ull;
  const size_t bytes = argc > 2 ? strtoull(argv[2], nullptr, 10) : (16ull << 20);
  const int wgs = argc > 3 ? atoi(argv[3]) : 4;
  const int S = argc > 4 ? atoi(argv[4]) : 32;
  const int reserved = argc > 5 ? atoi(argv[5]) : 8;
  const int trials = 7;
  float *rows, *acc;
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
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  int lo, hi;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t sc, sx, sx_hi, sc_m, sx_m;
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sx, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&sx_hi, hipStreamNonBlocking, hi));
  // CU masks: the communicator keeps `reserved` CUs spread evenly over the mask's bit range
  const int words = (ncu + 31) / 32;
  std::vector<uint32_t> mc(words, 0), mx(words, 0);
  const int stride = reserved > 0 ? ncu / reserved : ncu + 1;
  for (int i = 0; i < ncu; ++i) {
    const bool comm = reserved > 0 && (i % stride) == 0 && i / stride < reserved;
    (comm ? mx : mc)[i / 32] |= 1u << (i % 32);
  }
  CK(hipExtStreamCreateWithCUMask(&sc_m, words, mc.data()));
  CK(hipExtStreamCreateWithCUMask(&sx_m, words, mx.data()));
  std::vector<hipEvent_t> evc(S + 1), evx(S + 1);
  for (int i = 0; i <= S; ++i) {
    CK(hipEventCreateWithFlags(&evc[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evx[i], hipEventDisableTiming));
  }
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const size_t nv = bytes / 16;
  auto chain = [&](hipStream_t s) {
    if (fedagg_fedavg_chain_f32(ptrs.data(), w.data(), K, n, 1, acc, s)) {
      fprintf(stderr, "chain: %s\n", fedagg_last_error());
      exit(1);
    }
  };
  auto copy = [&](hipStream_t s) { copy_kernel<<<wgs, 256, 0, s>>>(src, dst, nv); };
  auto timed = [&](hipStream_t s, auto body) {
    std::vector<float> v;
    for (int r = 0; r < trials + 1; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, s));
      body();
      CK(hipEventRecord(t1, s));
      CK(hipDeviceSynchronize());
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      if (r) v.push_back(ms);  // the first is a warm-up
    }
    return median(v);
  };
  auto lockstep = [&](hipStream_t c, hipStream_t x) {
    // as csrc/lockstep.hip: group t after the compute stream's work so far; step t after group t - 1
    for (int t = 0; t <= S; ++t) {
      CK(hipEventRecord(evc[t], c));
      CK(hipStreamWaitEvent(x, evc[t], 0));
      if (t < S) copy(x);
      CK(hipEventRecord(evx[t], x));
      if (t > 0) CK(hipStreamWaitEvent(c, evx[t - 1], 0));
      if (t < S) chain(c);
    }
    CK(hipStreamWaitEvent(c, evx[S], 0));
  };
  const float tc = timed(sc, [&] { for (int t = 0; t < S; ++t) chain(sc); });
  const float tx = timed(sx, [&] { for (int t = 0; t < S; ++t) copy(sx); });
  const float tcm = timed(sc_m, [&] { for (int t = 0; t < S; ++t) chain(sc_m); });
  const float txm = timed(sx_m, [&] { for (int t = 0; t < S; ++t) copy(sx_m); });
  auto ov = [&](float t, float a, float b) { return (a + b - t) / std::min(a, b); };
  printf("{\"clients\": %d, \"elements_per_client\": %llu, \"copy_bytes\": %zu, \"copy_workgroups\": %d, "
         "\"steps\": %d, \"cus\": %d, \"reserved_cus\": %d, \"compute_only_ms\": %.4f, \"copy_only_ms\": %.4f, "
         "\"compute_only_masked_ms\": %.4f, \"copy_only_masked_ms\": %.4f}\n",
         K, (unsigned long long)n, bytes, wgs, S, ncu, reserved, tc, tx, tcm, txm);
  const float a = timed(sc, [&] { lockstep(sc, sx); });
  printf("{\"config\": \"lockstep\", \"ms\": %.4f, \"overlap\": %.3f}\n", a, ov(a, tc, tx));
  const float b = timed(sc, [&] { lockstep(sc, sx_hi); });
  printf("{\"config\": \"lockstep_hi\", \"ms\": %.4f, \"overlap\": %.3f}\n", b, ov(b, tc, tx));
  const float m = timed(sc_m, [&] { lockstep(sc_m, sx_m); });
  printf("{\"config\": \"lockstep_mask\", \"ms\": %.4f, \"overlap_vs_unmasked\": %.3f}\n", m, ov(m, tc, tx));
  for (int cap : {ncu, 2 * ncu}) {
    fedagg_tune("grid_cap", cap);
    const float tcc = timed(sc, [&] { for (int t = 0; t < S; ++t) chain(sc); });
    const float g = timed(sc, [&] { lockstep(sc, sx); });
    printf("{\"config\": \"lockstep_cap\", \"grid_cap\": %d, \"compute_only_ms\": %.4f, \"ms\": %.4f, "
           "\"overlap_vs_uncapped\": %.3f}\n", cap, tcc, g, ov(g, tc, tx));
  }
  fedagg_tune("grid_cap", 0);
  CK(hipFree(rows));
  CK(hipFree(acc));
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
