// alloc_probe.hip -- does C5's kernel time depend on WHICH 90 GB allocation it reads?
// (VERDICT r05 "Next 2"; tools/c5_step_probe.py found a second, newly allocated C5 buffer in the
// same process 2.1 % slower for all its launches while the first stayed at its time.)
//
// One process, the C5 product launch (fedagg_fedavg_tiled_bf16, 128 clients x 350M, tile 4096,
// 89.6 GB of bf16 in + 1.4 GB fp32 out) over buffers allocated one after another:
//   A  hipMalloc, the process's first big allocation
//   B  hipMalloc while A is held (the c5_step_probe "fresh" case)
//   A' A again (is A still at its time?)
//   -- A and B freed --
//   C  hipExtMallocWithFlags(hipDeviceMallocContiguous): physically contiguous, the largest
//      page-table fragments the driver can map (skipped when the driver refuses it)
//   D  hipMalloc after the frees
// Each buffer is filled with the same hashed bf16 values by a kernel, one untimed launch, then
// `launches` launches timed one by one with events; the outputs are checked bit-equal across the
// buffers.  One JSON line per buffer on stdout.
//   hipcc --offload-arch=gfx950 -O3 -Iinclude tools/alloc_probe.hip -Lsubstrafl_amd -lfedagg \
//         -Wl,-rpath,'$ORIGIN/../substrafl_amd' -o tools/_alloc_probe
//   tools/_alloc_probe [launches=30] [settle_s=8]
// settle_s: idle after each hipFree before the next allocation, so the driver's background clear
// of the freed VRAM (~38 GB/s) is over before the next buffer is timed (0: as round 6's
// first run, whose C and D buffers were timed inside the clear of A and B).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>

#include "fedagg.h"

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

static const int K = 128;
static const uint64_t M = 350000000ull;
static const uint64_t TV = 4096;  // FEDAGG_TILE_VECTORS_BF16
static const uint64_t L = 8;      // bf16 per 16-B vector

__global__ void fill_kernel(uint16_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
    uint32_t h = (uint32_t)(i * 2654435761ull) ^ (uint32_t)(i >> 29);
    h = (h ^ (h >> 15)) * 2246822519u;
    h ^= h >> 13;
    p[i] = (uint16_t)(0x3c00u + (h & 0x7ffu) - 0x400u);  // bf16 bit patterns of moderate values
  }
}

struct Res {
  double mean, median, mn, mx, first;
  uint64_t crc;
};

static Res run(const uint16_t* base, float* out, float* h_out, const float* w, int launches, hipStream_t s) {
  std::vector<hipEvent_t> ev(2 * (launches + 1));
  for (auto& e : ev) CHECK(hipEventCreate(&e));
  for (int i = 0; i <= launches; ++i) {
    CHECK(hipEventRecord(ev[2 * i], s));
    int rc = fedagg_fedavg_tiled_bf16(base, w, K, M, TV, nullptr, 0, nullptr, out, (void*)s);
    if (rc) {
      fprintf(stderr, "fedavg_tiled_bf16: %s\n", fedagg_last_error());
      exit(2);
    }
    CHECK(hipEventRecord(ev[2 * i + 1], s));
  }
  CHECK(hipStreamSynchronize(s));
  std::vector<double> ms;
  float first = 0;
  CHECK(hipEventElapsedTime(&first, ev[0], ev[1]));
  for (int i = 1; i <= launches; ++i) {
    float t = 0;
    CHECK(hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
    ms.push_back(t);
  }
  for (auto& e : ev) CHECK(hipEventDestroy(e));
  std::vector<double> srt = ms;
  std::sort(srt.begin(), srt.end());
  double sum = 0;
  for (double v : ms) sum += v;
  CHECK(hipMemcpy(h_out, out, M * sizeof(float), hipMemcpyDeviceToHost));
  uint64_t crc = 1469598103934665603ull;
  const uint32_t* u = reinterpret_cast<const uint32_t*>(h_out);
  for (uint64_t i = 0; i < M; i += 97) crc = (crc ^ u[i]) * 1099511628211ull;
  return Res{sum / ms.size(), srt[srt.size() / 2], srt.front(), srt.back(), first, crc};
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 30;
  const double settle_s = argc > 2 ? atof(argv[2]) : 8.0;
  auto settle = [&] {
    if (settle_s > 0) usleep((useconds_t)(settle_s * 1e6));
  };
  const uint64_t nvec = (M + L - 1) / L;
  const uint64_t elems = (nvec + TV - 1) / TV * K * TV * L;
  const uint64_t bytes = elems * sizeof(uint16_t);
  hipStream_t s;
  CHECK(hipSetDevice(0));
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float w[K];
  for (int k = 0; k < K; ++k) w[k] = 1.0f / (float)K;
  float* out = nullptr;
  CHECK(hipMalloc(&out, M * sizeof(float)));
  std::vector<float> h_out(M);
  auto measure = [&](const char* name, uint16_t* p, double alloc_s) {
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, s, p, elems);
    CHECK(hipStreamSynchronize(s));
    Res r = run(p, out, h_out.data(), w, launches, s);
    size_t f = 0, t = 0;
    CHECK(hipMemGetInfo(&f, &t));
    printf("{\"buffer\": \"%s\", \"bytes\": %llu, \"alloc_s\": %.3f, \"first_ms\": %.4f, \"launches\": %d, "
           "\"ms_mean\": %.4f, \"ms_median\": %.4f, \"ms_min\": %.4f, \"ms_max\": %.4f, \"TBps_median\": %.4f, "
           "\"frac_of_8TBps\": %.4f, \"free_GiB_after\": %.1f, \"crc\": \"%016llx\"}\n",
           name, (unsigned long long)bytes, alloc_s, r.first, launches, r.mean, r.median, r.mn, r.mx,
           (K * M * 2.0 + M * 4.0) / (r.median * 1e-3) / 1e12, (K * M * 2.0 + M * 4.0) / (r.median * 1e-3) / 8e12,
           f / 1073741824.0, (unsigned long long)r.crc);
    fflush(stdout);
  };
  auto now = [] {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
  };
  uint16_t *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
  settle();  // and any clear a previous process left
  double t0 = now();
  CHECK(hipMalloc(&a, bytes));
  measure("A hipMalloc (first)", a, now() - t0);
  t0 = now();
  CHECK(hipMalloc(&b, bytes));
  measure("B hipMalloc (second, A held)", b, now() - t0);
  measure("A again", a, 0.0);
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  settle();
  t0 = now();
  hipError_t e = hipExtMallocWithFlags((void**)&c, bytes, hipDeviceMallocContiguous);
  if (e == hipSuccess) {
    measure("C hipExtMallocWithFlags(contiguous)", c, now() - t0);
    CHECK(hipFree(c));
    settle();
  } else {
    printf("{\"buffer\": \"C hipExtMallocWithFlags(contiguous)\", \"refused\": \"%s\"}\n", hipGetErrorString(e));
    (void)hipGetLastError();
  }
  t0 = now();
  CHECK(hipMalloc(&d, bytes));
  measure("D hipMalloc (after the frees)", d, now() - t0);
  CHECK(hipFree(d));
  CHECK(hipFree(out));
  return 0;
}
