// Memory-pattern ceiling of the Scaffold bucket kernel: the same tile walk as
// scaffold_kernel's 4 x 4 shape (a workgroup step = 4 x 256 contiguous 16-B vectors per stream,
// clients in groups of 4, delta and control-variate streams interleaved, c read last, two 32-B
// outputs per input vector) with the fp64 arithmetic replaced by one integer xor per word, so the
// only cost left is the HBM traffic pattern.  Runs the pattern with and without the writes, and
// the FedAvg C2 pattern (8 streams, 16-B outputs) for comparison.
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_mix_probe.hip -o tools/_stream_mix_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 256;
constexpr int VPT = 4;
constexpr int SU = 4;

// B buckets of K client rows each (row stride nvec vectors), plus C extra single streams read
// last; W = output vectors written per input vector and bucket (0: none, 1: 16 B, 2: 32 B).
template <int K, int B, int C, int W, bool INTER = false>
__global__ void __launch_bounds__(BLOCK) pattern(const u32x4* __restrict__ x, const u32x4* __restrict__ c,
                                                 uint64_t nvec, u32x4* __restrict__ out) {
  const uint64_t tile = (uint64_t)VPT * BLOCK;
  const uint64_t t = blockIdx.x;
  if ((t + 1) * tile > nvec) return;
  u32x4 acc[B][VPT];
#pragma unroll
  for (int b = 0; b < B; ++b)
#pragma unroll
    for (int n = 0; n < VPT; ++n) acc[b][n] = u32x4{0, 0, 0, 0};
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += SU) {
    u32x4 r[B][SU][VPT];
#pragma unroll
    for (int u = 0; u < SU; ++u)
#pragma unroll
      for (int n = 0; n < VPT; ++n)
#pragma unroll
        for (int b = 0; b < B; ++b)
          r[b][u][n] = __builtin_nontemporal_load(
              x + (INTER ? (t * (B * K) + (uint64_t)b * K + k0 + u) * tile   // tile-major: the B*K client
                         : ((uint64_t)b * K + k0 + u) * nvec + t * tile) +  // tiles of one step adjacent
              (uint64_t)n * BLOCK + threadIdx.x);
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int u = 0; u < SU; ++u)
#pragma unroll
        for (int n = 0; n < VPT; ++n) acc[b][n] ^= r[b][u][n];
  }
#pragma unroll
  for (int i = 0; i < C; ++i)
#pragma unroll
    for (int n = 0; n < VPT; ++n)
      acc[B - 1][n] ^= __builtin_nontemporal_load(c + (uint64_t)i * nvec + t * tile + (uint64_t)n * BLOCK + threadIdx.x);
  if constexpr (W > 0) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave0 = t * tile + (threadIdx.x - lane);
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int n = 0; n < VPT; ++n) {
        // W x 16 B per lane, each store instruction writing 1 KiB contiguous per wave
        u32x4* o = out + ((uint64_t)b * nvec + wave0 + (uint64_t)n * BLOCK) * W;
#pragma unroll
        for (int s = 0; s < W; ++s) __builtin_nontemporal_store(acc[b][n] + s, o + s * 64 + lane);
      }
  } else {
    unsigned v = 0;
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int n = 0; n < VPT; ++n) v ^= acc[b][n][0] ^ acc[b][n][3];
    if (v == 0x9e3779b9u) out[threadIdx.x] = acc[0][0];  // keep the loads
  }
}

template <int K, int B, int C, int W, bool INTER = false>
static void run(const char* name, const u32x4* x, const u32x4* c, uint64_t nvec, u32x4* out) {
  const int grid = (int)(nvec / (VPT * BLOCK));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((pattern<K, B, C, W, INTER>), dim3(grid), dim3(BLOCK), 0, 0, x, c, nvec, out);
  std::vector<float> ms(15);
  for (auto& m : ms) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((pattern<K, B, C, W, INTER>), dim3(grid), dim3(BLOCK), 0, 0, x, c, nvec, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&m, a, b));
  }
  std::sort(ms.begin(), ms.end());
  const double bytes = ((double)B * K + C + (double)B * W) * nvec * 16;
  printf("{\"pattern\": \"%s\", \"read_streams\": %d, \"write_bytes_per_vector\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
         name, B * K + C, B * W * 16, ms[7] * 1e3, bytes / (ms[7] * 1e-3) / 1e9);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const uint64_t M = argc > 1 ? strtoull(argv[1], nullptr, 10) : 25000000ull;  // fp32 elements per row
  const uint64_t tile = (uint64_t)VPT * BLOCK;
  const uint64_t nvec = (M / 4) / tile * tile;
  u32x4 *x, *c, *out;
  CK(hipMalloc(&x, 2 * 16 * nvec * 16));
  CK(hipMalloc(&c, nvec * 16));
  CK(hipMalloc(&out, 2 * 2 * nvec * 16));
  CK(hipMemset(x, 1, 2 * 16 * nvec * 16));
  CK(hipMemset(c, 2, nvec * 16));
  run<16, 2, 1, 2>("scaffold 16 clients: 33 streams, 2 x 32-B outputs", x, c, nvec, out);
  run<16, 2, 1, 0>("scaffold 16 clients, reads only", x, c, nvec, out);
  run<16, 2, 1, 1>("scaffold 16 clients, 2 x 16-B outputs", x, c, nvec, out);
  run<32, 1, 1, 2>("33 streams one bucket, 1 x 32-B output", x, c, nvec, out);
  run<8, 1, 0, 1>("fedavg 8 clients: 8 streams, 16-B output", x, c, nvec, out);
  run<8, 1, 0, 0>("fedavg 8 clients, reads only", x, c, nvec, out);
  run<32, 1, 0, 1>("fedavg 32 clients, 16-B output", x, c, nvec, out);
  // tile-major layout (the K client tiles of one workgroup step adjacent in memory: one stream)
  run<16, 2, 1, 2, true>("tile-major scaffold 16 clients, 2 x 32-B outputs", x, c, nvec, out);
  run<16, 2, 1, 0, true>("tile-major scaffold 16 clients, reads only", x, c, nvec, out);
  run<8, 1, 0, 1, true>("tile-major fedavg 8 clients, 16-B output", x, c, nvec, out);
  return 0;
}
