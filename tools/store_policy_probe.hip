// Store / load cache-policy probe: the Scaffold C4 memory pattern of
// tools/stream_mix_probe.hip (33 non-temporal read streams, two 32-B outputs per input vector)
// and the FedAvg C2 pattern (8 streams, one 16-B output), with the output stores issued as
// buffer stores under every combination of the gfx950 cache-policy bits (aux: 1 = sc0,
// 2 = nt, 16 = sc1), against the __builtin_nontemporal_store form the kernels use.  Writes
// are the part of the mix that costs (a marginal ~3.5 TB/s); this asks whether a policy other
// than nt drains them more cheaply.  `load` mode does the same for the client loads (buffer
// loads per client row under each policy, against __builtin_nontemporal_load).
// Usage: _store_policy_probe [M] [load | c3]
// Build: hipcc --offload-arch=gfx950 -O3 tools/store_policy_probe.hip -o tools/_store_policy_probe
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

// B buckets of K client rows, C single streams read last, W output vectors per input vector and
// bucket; AUX < 0: __builtin_nontemporal_store, else a buffer store with that cache policy.
template <int LAUX>
__device__ __forceinline__ u32x4 ld(const u32x4* row, uint64_t i) {
  if constexpr (LAUX < 0) {
    return __builtin_nontemporal_load(row + i);
  } else {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(row), 0, 0x7FFFFFFF, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, LAUX);
  }
}

template <int K, int B, int C, int W, int AUX, int LAUX = -1>
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
          r[b][u][n] = ld<LAUX>(x + ((uint64_t)b * K + k0 + u) * nvec, t * tile + (uint64_t)n * BLOCK + threadIdx.x);
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
      acc[B - 1][n] ^= ld<LAUX>(c + (uint64_t)i * nvec, t * tile + (uint64_t)n * BLOCK + threadIdx.x);
  if constexpr (W == 0) {
    unsigned v = 0;
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int n = 0; n < VPT; ++n) v ^= acc[b][n][0] ^ acc[b][n][3];
    if (v == 0x9e3779b9u) out[threadIdx.x] = acc[0][0];  // keep the loads
    return;
  }
  const int lane = threadIdx.x & 63;
  const uint64_t wave0 = t * tile + (threadIdx.x - lane);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
  for (int b = 0; b < B; ++b)
#pragma unroll
    for (int n = 0; n < VPT; ++n) {
      const uint64_t o = ((uint64_t)b * nvec + wave0 + (uint64_t)n * BLOCK) * W;  // vectors
#pragma unroll
      for (int s = 0; s < W; ++s) {
        if constexpr (AUX < 0) {
          __builtin_nontemporal_store(acc[b][n] + s, out + o + s * 64 + lane);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(acc[b][n] + s, rs, (int)((o + s * 64 + lane) * 16), 0, AUX);
        }
      }
    }
}

template <int K, int B, int C, int W, int AUX, int LAUX = -1>
static void run(const char* name, const u32x4* x, const u32x4* c, uint64_t nvec, u32x4* out) {
  const int grid = (int)(nvec / (VPT * BLOCK));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((pattern<K, B, C, W, AUX, LAUX>), dim3(grid), dim3(BLOCK), 0, 0, x, c, nvec, out);
  std::vector<float> ms(15);
  for (auto& m : ms) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((pattern<K, B, C, W, AUX, LAUX>), dim3(grid), dim3(BLOCK), 0, 0, x, c, nvec, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&m, a, b));
  }
  std::sort(ms.begin(), ms.end());
  const double bytes = ((double)B * K + C + (double)B * W) * nvec * 16;
  printf("{\"pattern\": \"%s\", \"aux\": %d, \"load_aux\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, AUX, LAUX,
         ms[7] * 1e3,
         bytes / (ms[7] * 1e-3) / 1e9);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

template <int AUX>
static void both(const u32x4* x, const u32x4* c, uint64_t nvec, u32x4* out) {
  run<16, 2, 1, 2, AUX>("scaffold 16 clients, 2 x 32-B outputs", x, c, nvec, out);
  run<8, 1, 0, 1, AUX>("fedavg 8 clients, 16-B output", x, c, nvec, out);
}

template <int LAUX>
static void loads(const u32x4* x, const u32x4* c, uint64_t nvec, u32x4* out) {
  run<16, 2, 1, 2, -1, LAUX>("scaffold 16 clients, 2 x 32-B outputs", x, c, nvec, out);
  run<8, 1, 0, 1, 16, LAUX>("fedavg 8 clients, 16-B output (sc1)", x, c, nvec, out);
  run<8, 1, 0, 0, 16, LAUX>("fedavg 8 clients, reads only", x, c, nvec, out);
  run<32, 1, 0, 0, 16, LAUX>("32 clients, reads only", x, c, nvec, out);
}

// C3's pattern: 64 client streams, one 16-B output (or none), M fp32 per row.
static int c3_mode(uint64_t M) {
  const uint64_t tile = (uint64_t)VPT * BLOCK;
  const uint64_t nvec = (M / 4) / tile * tile;
  if (nvec * 16 >= 0x7FFFFFFFull) {
    fprintf(stderr, "output exceeds the 32-bit buffer offset range\n");
    return 2;
  }
  u32x4 *x, *c, *out;
  CK(hipMalloc(&x, 64 * nvec * 16));
  CK(hipMalloc(&c, 16));
  CK(hipMalloc(&out, nvec * 16));
  CK(hipMemset(x, 1, 64 * nvec * 16));
  for (int rep = 0; rep < 2; ++rep) {
    run<64, 1, 0, 0, -1>("64 clients, reads only", x, c, nvec, out);
    run<64, 1, 0, 1, -1>("64 clients, 16-B output (nt)", x, c, nvec, out);
    run<64, 1, 0, 1, 16>("64 clients, 16-B output (sc1)", x, c, nvec, out);
    run<32, 1, 0, 0, -1>("32 clients, reads only", x, c, nvec, out);
    run<32, 1, 0, 1, -1>("32 clients, 16-B output (nt)", x, c, nvec, out);
  }
  CK(hipFree(x));
  CK(hipFree(c));
  CK(hipFree(out));
  return 0;
}

int main(int argc, char** argv) {
  const bool load_mode = argc > 2 && argv[2][0] == 'l';
  const uint64_t M = argc > 1 ? strtoull(argv[1], nullptr, 10) : 25000000ull;  // fp32 elements per row
  if (argc > 2 && argv[2][0] == 'c') return c3_mode(M);
  const uint64_t tile = (uint64_t)VPT * BLOCK;
  const uint64_t nvec = (M / 4) / tile * tile;
  if (2 * 2 * nvec * 16 >= 0x7FFFFFFFull) {
    fprintf(stderr, "output exceeds the 32-bit buffer offset range\n");
    return 2;
  }
  u32x4 *x, *c, *out;
  CK(hipMalloc(&x, 2 * 16 * nvec * 16));
  CK(hipMalloc(&c, nvec * 16));
  CK(hipMalloc(&out, 2 * 2 * nvec * 16));
  CK(hipMemset(x, 1, 2 * 16 * nvec * 16));
  CK(hipMemset(c, 2, nvec * 16));
  for (int rep = 0; rep < 2 && load_mode; ++rep) {
    loads<-1>(x, c, nvec, out);
    loads<0>(x, c, nvec, out);
    loads<2>(x, c, nvec, out);
    loads<1>(x, c, nvec, out);
    loads<16>(x, c, nvec, out);
    loads<17>(x, c, nvec, out);
    loads<3>(x, c, nvec, out);
    loads<18>(x, c, nvec, out);
    loads<19>(x, c, nvec, out);
  }
  for (int rep = 0; rep < 2 && !load_mode; ++rep) {
    both<-1>(x, c, nvec, out);
    both<0>(x, c, nvec, out);
    both<2>(x, c, nvec, out);
    both<1>(x, c, nvec, out);
    both<16>(x, c, nvec, out);
    both<17>(x, c, nvec, out);
    both<3>(x, c, nvec, out);
    both<18>(x, c, nvec, out);
    both<19>(x, c, nvec, out);
  }
  CK(hipFree(x));
  CK(hipFree(c));
  CK(hipFree(out));
  return 0;
}
