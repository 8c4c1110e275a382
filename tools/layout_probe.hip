// Layout experiment: FedAvg over K = 8 fp32 client buckets in the
// production [K, M] layout (8 read streams) against a tile-interleaved [tiles, K, tile] layout
// (one read stream).  Same arithmetic, same tile walk; only the client addresses differ.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/layout_probe.hip -o tools/_layout_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 256;
constexpr int K = 8;

template <bool INTER, int VPT>
__global__ void __launch_bounds__(BLOCK) fa(const f32x4* __restrict__ x, const float* __restrict__ w,
                                            uint64_t nvec, f32x4* __restrict__ out) {
#pragma clang fp contract(off)
  const uint64_t tile = (uint64_t)VPT * BLOCK;
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[k];
  for (uint64_t t = blockIdx.x; t * tile + tile <= nvec; t += gridDim.x) {
    f32x4 acc[VPT];
#pragma unroll
    for (int n = 0; n < VPT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += 4) {
      f32x4 r[4][VPT];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int n = 0; n < VPT; ++n) {
          const uint64_t inner = (uint64_t)n * BLOCK + threadIdx.x;
          const uint64_t off = INTER ? (t * K + k0 + u) * tile + inner : (uint64_t)(k0 + u) * nvec + t * tile + inner;
          r[u][n] = __builtin_nontemporal_load(x + off);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int n = 0; n < VPT; ++n) {
          const f32x4 p = r[u][n] * wk[k0 + u];
          acc[n] = acc[n] + p;
        }
    }
#pragma unroll
    for (int n = 0; n < VPT; ++n) __builtin_nontemporal_store(acc[n], out + t * tile + (uint64_t)n * BLOCK + threadIdx.x);
  }
}

template <bool INTER, int VPT>
static float run(const f32x4* x, const float* w, uint64_t nvec, f32x4* out, int grid, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((fa<INTER, VPT>), dim3(grid), dim3(BLOCK), 0, 0, x, w, nvec, out);
  std::vector<float> ms(reps);
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((fa<INTER, VPT>), dim3(grid), dim3(BLOCK), 0, 0, x, w, nvec, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms[i], a, b));
  }
  std::sort(ms.begin(), ms.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms[reps / 2];
}

int main(int argc, char** argv) {
  const uint64_t M = argc > 1 ? strtoull(argv[1], nullptr, 10) : 25000000ull;
  const int VPT = 4;
  const uint64_t tile = (uint64_t)VPT * BLOCK;
  const uint64_t nvec = (M / 4) / tile * tile;  // whole tiles only
  const uint64_t ntiles = nvec / tile;
  f32x4 *x, *out, *out2;
  float* w;
  CK(hipMalloc(&x, K * nvec * 16));
  CK(hipMalloc(&out, nvec * 16));
  CK(hipMalloc(&out2, nvec * 16));
  CK(hipMalloc(&w, K * 4));
  std::vector<float> hw(K);
  for (int k = 0; k < K; ++k) hw[k] = (k + 1) / 36.0f;
  CK(hipMemcpy(w, hw.data(), K * 4, hipMemcpyHostToDevice));
  // fill: values depend on (client, element) only, so both layouts hold the same clients
  {
    std::vector<float> h(nvec * 4);
    for (int k = 0; k < K; ++k) {
      for (uint64_t i = 0; i < nvec * 4; ++i) h[i] = (float)((i * 2654435761ull + k * 40503ull) % 1000003) * 1e-3f;
      CK(hipMemcpy(x + k * nvec, h.data(), nvec * 16, hipMemcpyHostToDevice));  // [K, M] first
    }
  }
  const double bytes = (double)(K + 1) * nvec * 16;
  int grids[] = {(int)ntiles, 4096, 8192, 2048};
  for (int g : grids) {
    float t = run<false, 4>(x, w, nvec, out, g, 21);
    printf("{\"layout\": \"rows\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", g, t * 1e3, bytes / (t * 1e-3) / 1e9);
  }
  // re-lay the same clients tile-interleaved: x2[(t*K + k)*tile + i] = x[k*nvec + t*tile + i]
  f32x4* x2;
  CK(hipMalloc(&x2, K * nvec * 16));
  CK(hipMemcpy2D(x2, K * tile * 16, x, tile * 16, tile * 16, 1, hipMemcpyDeviceToDevice));  // warm the API
  for (int k = 0; k < K; ++k)
    CK(hipMemcpy2D(x2 + k * tile, K * tile * 16, x + k * nvec, tile * 16, tile * 16, ntiles, hipMemcpyDeviceToDevice));
  for (int g : grids) {
    float t = run<true, 4>(x2, w, nvec, out2, g, 21);
    printf("{\"layout\": \"interleaved\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", g, t * 1e3, bytes / (t * 1e-3) / 1e9);
  }
  std::vector<float> a(nvec * 4), b(nvec * 4);
  CK(hipMemcpy(a.data(), out, nvec * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), out2, nvec * 16, hipMemcpyDeviceToHost));
  uint64_t diff = 0;
  for (uint64_t i = 0; i < nvec * 4; ++i) diff += memcmp(&a[i], &b[i], 4) != 0;
  printf("{\"same_results\": %s, \"M\": %llu}\n", diff ? "false" : "true", (unsigned long long)(nvec * 4));
  return diff ? 1 : 0;
}
