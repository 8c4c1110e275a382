// C4 layout experiment (DESIGN.md §9.2 / §9.3b "next"): Scaffold's one-bucket launch pair over
// K = 16 fp32 client buckets of M = 25M (delta bucket, then control variate bucket + c), fp64
// products / sums / outputs, in the production [K, M] row layout (16 read streams per launch)
// against a tile-interleaved [tiles, K, tile] layout (each workgroup reads ONE contiguous K x tile
// region), with the production tile (8 vectors x 256 threads, clients in groups of 4, nt loads,
// nt stores coalesced through LDS) and larger ones, with and without the outputs.  Timing only:
// both layouts run the same arithmetic over the same bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/scaffold_layout_probe.hip -o tools/_scaffold_layout_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int K = 16;

// one wave's 64 lanes x 32 B of fp64 results, stored as two fully coalesced 1 KiB rows
template <bool NTS>
__device__ __forceinline__ void store32(f64x2* wave_dst, f64x2 lo, f64x2 hi, f64x2* lds) {
  const int lane = threadIdx.x & 63;
  lds[2 * lane] = lo;
  lds[2 * lane + 1] = hi;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const f64x2 a = lds[lane], b = lds[64 + lane];
  if (NTS) {
    __builtin_nontemporal_store(a, wave_dst + lane);
    __builtin_nontemporal_store(b, wave_dst + 64 + lane);
  } else {
    wave_dst[lane] = a;
    wave_dst[64 + lane] = b;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// PH 0: out = lr * sum_k w_k x_k; PH 1: out = sum_k w_k x_k + c (client order, fp64)
template <bool INTER, bool WRITE, int PH, int VPT, int BLK, int SU, bool NTS = true>
__global__ void __launch_bounds__(BLK)
sc(const f32x4* __restrict__ x, const double* __restrict__ w, const f32x4* __restrict__ c, double lr,
   uint64_t nvec, double* __restrict__ out, uint64_t pitch) {
#pragma clang fp contract(off)
  __shared__ f64x2 stage[BLK / 64][128];
  f64x2* lds = stage[threadIdx.x / 64];
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  const uint64_t ntiles = nvec / T;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    double acc[VPT][4];
#pragma unroll
    for (int n = 0; n < VPT; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[n][j] = 0.0;
    for (int k0 = 0; k0 < K; k0 += SU) {
      f32x4 r[SU][VPT];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const f32x4* base = INTER ? x + (t * K + k0 + u) * T : x + (uint64_t)(k0 + u) * pitch + t * T;
#pragma unroll
        for (int n = 0; n < VPT; ++n) r[u][n] = __builtin_nontemporal_load(base + n * BLK + threadIdx.x);
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const double wk = w[k0 + u];
#pragma unroll
        for (int n = 0; n < VPT; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double p = wk * (double)r[u][n][j];
            acc[n][j] = acc[n][j] + p;
          }
      }
    }
#pragma unroll
    for (int n = 0; n < VPT; ++n) {
      if (PH == 1) {
        const f32x4 cv = __builtin_nontemporal_load(c + t * T + n * BLK + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[n][j] = acc[n][j] + (double)cv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[n][j] = lr * acc[n][j];
      }
    }
    if (WRITE) {
#pragma unroll
      for (int n = 0; n < VPT; ++n) {
        const uint64_t v0 = t * T + n * BLK + (threadIdx.x & ~63u);
        store32<NTS>(reinterpret_cast<f64x2*>(out + v0 * 4), f64x2{acc[n][0], acc[n][1]}, f64x2{acc[n][2], acc[n][3]},
                lds);
      }
    } else {
      double s = 0.0;
#pragma unroll
      for (int n = 0; n < VPT; ++n) s += acc[n][0] + acc[n][1] + acc[n][2] + acc[n][3];
      if (s == 1234.5) out[0] = s;
    }
  }
}

struct Bufs {
  f32x4 *d_rows, *cv_rows, *d_int, *cv_int, *c;
  double *w, *dout, *cout;
  uint64_t nvec;
};

// chunks > 1 (rows only): the pair launched per parameter chunk (outputs of one chunk ~ 400 MB /
// chunks), delta and control-variate launch of each chunk back to back
template <bool INTER, bool WRITE, int VPT, int BLK, int SU, bool NTS = true>
void run(const char* name, const Bufs& b, int grid_cap, int reps, int chunks = 1) {
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  const uint64_t ntiles = b.nvec / T;
  const uint64_t ctiles = (ntiles + chunks - 1) / chunks;
  const int grid = (int)std::min<uint64_t>(ctiles, grid_cap > 0 ? (uint64_t)grid_cap : ctiles);
  const f32x4* xd = INTER ? b.d_int : b.d_rows;
  const f32x4* xc = INTER ? b.cv_int : b.cv_rows;
  auto pair = [&]() {
    for (int ch = 0; ch < chunks; ++ch) {
      const uint64_t t0 = ch * ctiles, nt = std::min(ctiles, ntiles - t0), o = t0 * T;
      sc<INTER, WRITE, 0, VPT, BLK, SU, NTS><<<grid, BLK>>>(xd + o, b.w, b.c + o, 0.5, nt * T, b.dout + o * 4, b.nvec);
      sc<INTER, WRITE, 1, VPT, BLK, SU, NTS><<<grid, BLK>>>(xc + o, b.w, b.c + o, 0.5, nt * T, b.cout + o * 4, b.nvec);
    }
  };
  for (int i = 0; i < 3; ++i) pair();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(e0));
    pair();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float m;
    CK(hipEventElapsedTime(&m, e0, e1));
    ms.push_back(m);
  }
  std::sort(ms.begin(), ms.end());
  const double used = (double)ntiles * T * 16;  // bytes per client bucket actually walked
  const double bytes = 2 * K * used + used + (WRITE ? 2 * 2 * used : 0);
  printf("%-44s grid %6d  median %8.1f us  min %8.1f us  %6.3f TB/s (median)\n", name, grid, ms[reps / 2] * 1e3,
         ms[0] * 1e3, bytes / (ms[reps / 2] * 1e-3) / 1e12);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const uint64_t M = argc > 1 ? strtoull(argv[1], nullptr, 10) : 25000000ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 30;
  Bufs b;
  b.nvec = M / 4;
  const uint64_t bucket = (uint64_t)K * b.nvec * 16;
  CK(hipMalloc(&b.d_rows, bucket));
  CK(hipMalloc(&b.cv_rows, bucket));
  CK(hipMalloc(&b.d_int, bucket));
  CK(hipMalloc(&b.cv_int, bucket));
  CK(hipMalloc(&b.c, b.nvec * 16));
  CK(hipMalloc(&b.w, K * 8));
  CK(hipMalloc(&b.dout, b.nvec * 32));
  CK(hipMalloc(&b.cout, b.nvec * 32));
  CK(hipMemset(b.d_rows, 0x3c, bucket));
  CK(hipMemset(b.cv_rows, 0x3d, bucket));
  CK(hipMemset(b.d_int, 0x3c, bucket));
  CK(hipMemset(b.cv_int, 0x3d, bucket));
  CK(hipMemset(b.c, 0x3e, b.nvec * 16));
  std::vector<double> w(K, 1.0 / K);
  CK(hipMemcpy(b.w, w.data(), K * 8, hipMemcpyHostToDevice));
  printf("scaffold one-bucket launch pair, K=%d fp32 clients x M=%llu, fp64 out (%.2f GB algorithmic)\n", K,
         (unsigned long long)M, (2.0 * K * M * 4 + M * 4 + 2.0 * M * 8) / 1e9);
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d\n", pass);
    run<false, true, 8, 256, 4>("rows   8x256 su4 (production tile) +out", b, 0, reps);
    run<false, true, 8, 256, 4, false>("rows   8x256 su4 +out plain stores", b, 0, reps);
    run<false, false, 8, 256, 4>("rows   8x256 su4 reads only", b, 0, reps);
    run<true, true, 8, 256, 4>("inter  8x256 su4 +out", b, 0, reps);
    run<true, true, 16, 256, 2>("inter 16x256 su2 +out", b, 0, reps);
    run<true, true, 16, 256, 2, false>("inter 16x256 su2 +out plain stores", b, 0, reps);
    run<false, true, 16, 256, 2>("rows  16x256 su2 +out", b, 0, reps);
    run<false, true, 8, 256, 4, false>("rows   8x256 su4 +out plain, 2 chunks", b, 0, reps, 2);
    run<false, true, 8, 256, 4, false>("rows   8x256 su4 +out plain, 4 chunks", b, 0, reps, 4);
    run<false, true, 8, 256, 4>("rows   8x256 su4 +out nt, 4 chunks", b, 0, reps, 4);
    run<false, true, 8, 256, 4, false>("rows   8x256 su4 +out plain, 8 chunks", b, 0, reps, 8);
  }
  return 0;
}
