// C3 layout experiment: FedAvg over K = 64 fp32 client buckets of M = 125M in the
// production [K, M] row layout (64 read streams) against a tile-interleaved [tiles, K, tile]
// layout (each workgroup reads ONE contiguous K x tile region), with the C3 kernel's tile (16
// vectors x 512 threads, clients in pairs, nt loads, nt 16-B stores), with and without the
// output.  Timing only: both layouts run the same arithmetic over the same buffer.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/c3_layout_probe.hip -o tools/_c3_layout_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int K, bool INTER, bool WRITE, int VPT, int BLK, int U>
__global__ void __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(BLK >= 512 && VPT * U <= 32 ? 2 : 1)))
fa(const f32x4* __restrict__ x, const float* __restrict__ w, uint64_t nvec, f32x4* __restrict__ out) {
#pragma clang fp contract(off)
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  const uint64_t t = blockIdx.x;
  if ((t + 1) * T > nvec) return;
  f32x4 acc[VPT];
#pragma unroll
  for (int n = 0; n < VPT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += U) {
    f32x4 r[U][VPT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f32x4* base = INTER ? x + (t * K + k0 + u) * T : x + (uint64_t)(k0 + u) * nvec + t * T;
#pragma unroll
      for (int n = 0; n < VPT; ++n) r[u][n] = __builtin_nontemporal_load(base + n * BLK + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wk = w[k0 + u];
#pragma unroll
      for (int n = 0; n < VPT; ++n) acc[n] = acc[n] + r[u][n] * wk;
    }
  }
  if (WRITE) {
#pragma unroll
    for (int n = 0; n < VPT; ++n) __builtin_nontemporal_store(acc[n], out + t * T + n * BLK + threadIdx.x);
  } else {
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < VPT; ++n) s += acc[n].x + acc[n].y + acc[n].z + acc[n].w;
    if (s == 1234.5f) out[0] = acc[0];
  }
}

template <int K, bool INTER, bool WRITE, int VPT, int BLK, int U>
void run(const char* name, const f32x4* x, const float* w, uint64_t nvec, f32x4* out) {
  const unsigned grid = (unsigned)(nvec / ((uint64_t)VPT * BLK));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((fa<K, INTER, WRITE, VPT, BLK, U>), dim3(grid), dim3(BLK), 0, 0, x, w, nvec, out);
  CK(hipDeviceSynchronize());
  float best = 1e30f, tot = 0.f;
  const int reps = 10;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((fa<K, INTER, WRITE, VPT, BLK, U>), dim3(grid), dim3(BLK), 0, 0, x, w, nvec, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
    tot += ms;
  }
  CK(hipGetLastError());
  const double bytes = (double)grid * VPT * BLK * 16.0 * (K + (WRITE ? 1 : 0));
  printf("{\"K\": %d, \"pattern\": \"%s\", \"vpt\": %d, \"block\": %d, \"u\": %d, \"write\": %d, \"us_best\": %.1f, \"us_mean\": %.1f, "
         "\"GBps_best\": %.1f}\n",
         K, name, VPT, BLK, U, (int)WRITE, best * 1e3, tot / reps * 1e3, bytes / (best * 1e-3) / 1e9);
  fflush(stdout);
}

template <int K>
void sweep(uint64_t m_req, bool full) {
  const uint64_t M = m_req / (16 * 512 * 4) * (16 * 512 * 4);  // whole tiles of every shape
  const uint64_t nvec = M / 4;
  f32x4 *x, *out;
  float* w;
  CK(hipMalloc(&x, (uint64_t)K * M * 4));
  CK(hipMalloc(&out, M * 4));
  CK(hipMalloc(&w, K * 4));
  CK(hipMemset(x, 0, (uint64_t)K * M * 4));
  float hw[K];
  for (int k = 0; k < K; ++k) hw[k] = 1.0f / K;
  CK(hipMemcpy(w, hw, sizeof hw, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    run<K, false, true, 16, 512, 2>("rows", x, w, nvec, out);
    run<K, true, true, 16, 512, 2>("interleaved", x, w, nvec, out);
    run<K, false, false, 16, 512, 2>("rows", x, w, nvec, out);
    if (!full) continue;
    run<K, true, false, 16, 512, 2>("interleaved", x, w, nvec, out);
    run<K, false, true, 8, 256, 4>("rows", x, w, nvec, out);
    run<K, true, true, 8, 256, 4>("interleaved", x, w, nvec, out);
    run<K, false, true, 4, 256, 4>("rows", x, w, nvec, out);
    run<K, true, true, 4, 256, 4>("interleaved", x, w, nvec, out);
  }
  CK(hipFree(x));
  CK(hipFree(out));
  CK(hipFree(w));
}

// 128 x 175M fp32 rows (C5's streams and footprint): bytes per stream per workgroup step
template <int K>
void tiles(uint64_t m_req) {
  const uint64_t M = m_req / (32 * 1024 * 4) * (32 * 1024 * 4);
  const uint64_t nvec = M / 4;
  f32x4 *x, *out;
  float* w;
  CK(hipMalloc(&x, (uint64_t)K * M * 4));
  CK(hipMalloc(&out, M * 4));
  CK(hipMalloc(&w, K * 4));
  CK(hipMemset(x, 0, (uint64_t)K * M * 4));
  float hw[K];
  for (int k = 0; k < K; ++k) hw[k] = 1.0f / K;
  CK(hipMemcpy(w, hw, sizeof hw, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    run<K, false, true, 16, 512, 2>("rows 128K/stream", x, w, nvec, out);
    run<K, false, true, 32, 512, 1>("rows 256K/stream", x, w, nvec, out);
    run<K, false, true, 16, 1024, 1>("rows 256K/stream", x, w, nvec, out);
    run<K, false, true, 8, 1024, 2>("rows 128K/stream", x, w, nvec, out);
    run<K, false, true, 32, 256, 1>("rows 128K/stream", x, w, nvec, out);
    run<K, false, true, 8, 256, 4>("rows 32K/stream", x, w, nvec, out);
    run<K, false, true, 4, 256, 8>("rows 16K/stream", x, w, nvec, out);
  }
  CK(hipFree(x));
  CK(hipFree(out));
  CK(hipFree(w));
}

// no argument: the C3 shape (64 x 125M, every tile); "c5": 64 x 125M and 128 x 175M fp32 (the C5
// footprint, 89.6 GB, with C5's 128 client streams) side by side; "tiles": tile shapes at 128 x 175M;
// "kscan": 8, 16 and 32 clients
int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "";
  if (mode[0] == 't') {
    tiles<128>(175000000ull);
    return 0;
  }
  if (mode[0] == 'k') {  // "kscan": rows vs interleaved at 8, 16 and 32 clients (~16 GB each)
    sweep<8>(500000000ull, false);
    sweep<16>(250000000ull, false);
    sweep<32>(125000000ull, false);
    return 0;
  }
  const bool c5 = mode[0] == 'c' && mode[1] == '5';
  sweep<64>(125000000ull, !c5);
  if (c5) sweep<128>(175000000ull, false);
  return 0;
}
