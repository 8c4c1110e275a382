// C4 write-burst experiment (VERDICT r03 "Next 4"): Scaffold's one-bucket launch
// pair (K = 16 fp32 client buckets of M = 25M, fp64 products / sums / outputs; the delta bucket
// then the control-variate bucket + c) at 0.815 of 8 TB/s, 92 % of the read ceiling, PMC traffic
// 1.0002x the algorithmic bytes: the 0.4 GB of fp64 outputs cost ~3 read-bytes each in HBM
// read/write turnarounds.  The one lever not tried: fewer, larger write bursts per workgroup.
// Here each workgroup walks TILES consecutive tiles (VPT x 256 vectors per client stream each),
// keeps their fp64 outputs in LDS, and only after its reads writes them out as ONE contiguous
// burst of TILES x VPT x 8 KiB with every thread of the workgroup storing 16-B vectors -- against
// the production walk (one 8 x 256 tile per workgroup step, clients in groups of 4, nt loads, the
// outputs of each wave stored as two coalesced 1 KiB rows right after its tile).  Same arithmetic
// and bytes; the outputs of every variant are compared with the production walk's bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/scaffold_burst_probe.hip -o tools/_scaffold_burst_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int K = 16;
constexpr int BLK = 256;

// acc[n][:] = sum_k w_k x_k (fp64, client order) for this thread's VPT vectors of tile t, then
// PH 0: * lr; PH 1: + c
template <int PH, int VPT, int SU>
__device__ __forceinline__ void tile_sum(const f32x4* __restrict__ x, const double* __restrict__ w,
                                         const f32x4* __restrict__ c, double lr, uint64_t pitch, uint64_t t,
                                         double (&acc)[VPT][4]) {
#pragma clang fp contract(off)
  constexpr uint64_t T = (uint64_t)VPT * BLK;
#pragma unroll
  for (int n = 0; n < VPT; ++n)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[n][j] = 0.0;
  for (int k0 = 0; k0 < K; k0 += SU) {
    f32x4 r[SU][VPT];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const f32x4* base = x + (uint64_t)(k0 + u) * pitch + t * T;
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
}

// production walk: the outputs of each wave as two coalesced 1 KiB rows right after its tile
template <int PH, int VPT, int SU>
__global__ void __launch_bounds__(BLK) sc_tile(const f32x4* __restrict__ x, const double* __restrict__ w,
                                               const f32x4* __restrict__ c, double lr, uint64_t ntiles,
                                               uint64_t pitch, double* __restrict__ out) {
  __shared__ f64x2 stage[BLK / 64][128];
  f64x2* lds = stage[threadIdx.x / 64];
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  const int lane = threadIdx.x & 63;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    double acc[VPT][4];
    tile_sum<PH, VPT, SU>(x, w, c, lr, pitch, t, acc);
#pragma unroll
    for (int n = 0; n < VPT; ++n) {
      f64x2* dst = reinterpret_cast<f64x2*>(out + (t * T + n * BLK + (threadIdx.x & ~63u)) * 4);
      lds[2 * lane] = f64x2{acc[n][0], acc[n][1]};
      lds[2 * lane + 1] = f64x2{acc[n][2], acc[n][3]};
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_nontemporal_store(lds[lane], dst + lane);
      __builtin_nontemporal_store(lds[64 + lane], dst + 64 + lane);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// burst walk: TILES consecutive tiles per workgroup, their outputs kept in LDS, then one
// contiguous burst of TILES * VPT * 8 KiB stored by the whole workgroup (16 B per thread per store)
template <int PH, int VPT, int SU, int TILES>
__global__ void __launch_bounds__(BLK) sc_burst(const f32x4* __restrict__ x, const double* __restrict__ w,
                                                const f32x4* __restrict__ c, double lr, uint64_t ntiles,
                                                uint64_t pitch, double* __restrict__ out) {
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  constexpr int NV = TILES * VPT * BLK * 2;  // f64x2 of one burst
  __shared__ f64x2 buf[NV];
  const uint64_t ngroups = (ntiles + TILES - 1) / TILES;
  for (uint64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint64_t t0 = g * TILES;
    const int nt = (int)std::min<uint64_t>(TILES, ntiles - t0);
    for (int i = 0; i < nt; ++i) {
      double acc[VPT][4];
      tile_sum<PH, VPT, SU>(x, w, c, lr, pitch, t0 + i, acc);
#pragma unroll
      for (int n = 0; n < VPT; ++n) {
        const int v = i * (int)T + n * BLK + threadIdx.x;  // vector index within the burst
        buf[2 * v] = f64x2{acc[n][0], acc[n][1]};
        buf[2 * v + 1] = f64x2{acc[n][2], acc[n][3]};
      }
    }
    __syncthreads();
    f64x2* dst = reinterpret_cast<f64x2*>(out + t0 * T * 4);
    const int nv = nt * (int)T * 2;
    for (int i = threadIdx.x; i < nv; i += BLK) __builtin_nontemporal_store(buf[i], dst + i);
    __syncthreads();  // the buffer is refilled by the next group
  }
}

struct Bufs {
  f32x4 *d, *cv, *c;
  double *w, *dout, *cout, *dref, *cref;
  uint64_t nvec;
};

template <typename L>
double timed(L pair, int reps) {
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
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms[reps / 2];
}

bool same(const double* a, const double* b, uint64_t n) {
  std::vector<double> ha(n), hb(n);
  CK(hipMemcpy(ha.data(), a, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), b, n * 8, hipMemcpyDeviceToHost));
  return memcmp(ha.data(), hb.data(), n * 8) == 0;
}

template <int VPT, int SU>
double run_tile(const Bufs& b, uint64_t used_vec, int reps, double* dout, double* cout) {
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  const uint64_t ntiles = used_vec / T;
  const int grid = (int)ntiles;
  auto pair = [&]() {
    sc_tile<0, VPT, SU><<<grid, BLK>>>(b.d, b.w, b.c, 0.5, ntiles, b.nvec, dout);
    sc_tile<1, VPT, SU><<<grid, BLK>>>(b.cv, b.w, b.c, 0.5, ntiles, b.nvec, cout);
  };
  return timed(pair, reps);
}

template <int VPT, int SU, int TILES>
double run_burst(const Bufs& b, uint64_t used_vec, int reps, double* dout, double* cout) {
  constexpr uint64_t T = (uint64_t)VPT * BLK;
  const uint64_t ntiles = used_vec / T;
  const int grid = (int)((ntiles + TILES - 1) / TILES);
  auto pair = [&]() {
    sc_burst<0, VPT, SU, TILES><<<grid, BLK>>>(b.d, b.w, b.c, 0.5, ntiles, b.nvec, dout);
    sc_burst<1, VPT, SU, TILES><<<grid, BLK>>>(b.cv, b.w, b.c, 0.5, ntiles, b.nvec, cout);
  };
  return timed(pair, reps);
}

int main(int argc, char** argv) {
  const uint64_t M = argc > 1 ? strtoull(argv[1], nullptr, 10) : 25000000ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 30;
  Bufs b;
  b.nvec = M / 4;
  const uint64_t bucket = (uint64_t)K * b.nvec * 16;
  CK(hipMalloc(&b.d, bucket));
  CK(hipMalloc(&b.cv, bucket));
  CK(hipMalloc(&b.c, b.nvec * 16));
  CK(hipMalloc(&b.w, K * 8));
  CK(hipMalloc(&b.dout, b.nvec * 32));
  CK(hipMalloc(&b.cout, b.nvec * 32));
  CK(hipMalloc(&b.dref, b.nvec * 32));
  CK(hipMalloc(&b.cref, b.nvec * 32));
  {  // distinct values per client and element (bit patterns of small floats)
    std::vector<float> h(b.nvec * 4);
    for (int k = 0; k < K; ++k) {
      for (uint64_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761ull + k * 97ull) % 10007) * 1e-3f - 5.0f;
      CK(hipMemcpy(reinterpret_cast<float*>(b.d) + k * h.size(), h.data(), h.size() * 4, hipMemcpyHostToDevice));
      for (auto& v : h) v = -0.5f * v;
      CK(hipMemcpy(reinterpret_cast<float*>(b.cv) + k * h.size(), h.data(), h.size() * 4, hipMemcpyHostToDevice));
    }
    CK(hipMemcpy(b.c, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  std::vector<double> w(K);
  for (int k = 0; k < K; ++k) w[k] = (k + 1.0) / (K * (K + 1) / 2.0);
  CK(hipMemcpy(b.w, w.data(), K * 8, hipMemcpyHostToDevice));
  // every variant walks the same whole tiles: the largest tile's multiple (32 KiB x 8 per stream)
  const uint64_t unit = (uint64_t)8 * BLK * 8;
  const uint64_t used = b.nvec / unit * unit;
  const double bytes = (2.0 * K * used + used) * 16 + 2.0 * used * 32;
  printf("scaffold one-bucket launch pair, K=%d fp32 clients x %llu of M=%llu, fp64 out (%.3f GB algorithmic)\n", K,
         (unsigned long long)(used * 4), (unsigned long long)M, bytes / 1e9);
  auto report = [&](const char* name, double ms, bool ok) {
    printf("%-58s median %8.1f us  %6.3f TB/s  %s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12,
           ok ? "bit-identical" : "MISMATCH");
  };
  for (int pass = 0; pass < 2; ++pass) {
    printf("-- pass %d\n", pass);
    double ms = run_tile<8, 4>(b, used, reps, b.dref, b.cref);
    report("production: 8x256 tile su4, wave rows after each tile", ms, true);
    ms = run_burst<8, 4, 1>(b, used, reps, b.dout, b.cout);
    report("burst  8x256 su4, 1 tile  ->  64 KiB burst (64 KiB LDS)", ms,
           same(b.dout, b.dref, used * 4) && same(b.cout, b.cref, used * 4));
    ms = run_burst<4, 4, 2>(b, used, reps, b.dout, b.cout);
    report("burst  4x256 su4, 2 tiles ->  64 KiB burst (64 KiB LDS)", ms,
           same(b.dout, b.dref, used * 4) && same(b.cout, b.cref, used * 4));
    ms = run_burst<4, 4, 4>(b, used, reps, b.dout, b.cout);
    report("burst  4x256 su4, 4 tiles -> 128 KiB burst (128 KiB LDS)", ms,
           same(b.dout, b.dref, used * 4) && same(b.cout, b.cref, used * 4));
    ms = run_burst<8, 4, 2>(b, used, reps, b.dout, b.cout);
    report("burst  8x256 su4, 2 tiles -> 128 KiB burst (128 KiB LDS)", ms,
           same(b.dout, b.dref, used * 4) && same(b.cout, b.cref, used * 4));
    ms = run_burst<2, 8, 8>(b, used, reps, b.dout, b.cout);
    report("burst  2x256 su8, 8 tiles -> 128 KiB burst (128 KiB LDS)", ms,
           same(b.dout, b.dref, used * 4) && same(b.cout, b.cref, used * 4));
    ms = run_burst<2, 8, 4>(b, used, reps, b.dout, b.cout);
    report("burst  2x256 su8, 4 tiles ->  64 KiB burst (64 KiB LDS)", ms,
           same(b.dout, b.dref, used * 4) && same(b.cout, b.cref, used * 4));
  }
  return 0;
}
