// fedagg.hip -- hand-written gfx950 (MI355X / CDNA4) kernels for SubstraFL's aggregation
// hot path, behind the C ABI declared in include/fedagg.h.
//
// The path is element-wise and HBM-bound (0.5 FLOP per input byte for fp32 FedAvg), so
// the design is a pure streaming one -- no MFMA, no LDS staging of the client streams:
//   * one thread owns one 16-byte vector of the flat bucket (4 fp32 / 8 bf16 / 2 fp64 /
//     8 fp16 elements) and walks the K clients IN LIST ORDER, which is the order the
//     reference's np.sum(list, axis=0) adds them (fed_avg.py:221-222);
//   * the client loop is unrolled by FA_UNROLL with all loads issued before the dependent
//     add chain, so every lane keeps FA_UNROLL x 16 B in flight (the HBM latency cover);
//   * client pointers and weights live in the kernel-argument segment (scalar loads,
//     no device-side table, graph-capturable); clients beyond FEDAGG_KCHUNK continue
//     from the partial sum already in `out`, which is exact because the accumulator
//     type is the stored type;
//   * grid-stride over the bucket with a launch of a few thousand 256-thread
//     workgroups (>> 256 CUs; blocks are dealt round-robin over the 8 XCDs and have no
//     reuse to localise, so no XCD remap is needed here).
// Bit parity with NumPy requires every product and sum to be rounded separately: the
// file is compiled with -ffp-contract=off AND every kernel body carries
// `#pragma clang fp contract(off)` (hipcc otherwise emits v_fmac_f32 for acc + x*w).

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "fedagg.h"

#define FA_BLOCK 256
#define FA_UNROLL 8

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, const char* a = "", long long b = 0) {
  snprintf(g_err, sizeof(g_err), fmt, a, b);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return FEDAGG_EHIP;
  }
  return FEDAGG_OK;
}

// Launch shape (tunable through fedagg_set_launch; defaults measured on MI355X).
int g_grid_cap = 4096;   // workgroups per launch before grid-striding
int g_nontemporal = 1;   // client streams are read once: non-temporal loads

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------
// element types: storage type TIn, product/accumulate type TP, output storage TOut
// ------------------------------------------------------------------------------------
struct F32 {
  using In = float;
  using P = float;
  using Out = float;
  static constexpr int L = 4;  // elements per 16-byte vector
  __device__ static P cvt(In v) { return v; }
  __device__ static void unpack(u32x4 r, P* o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __uint_as_float(r[j]);
  }
  __device__ static Out out(P v) { return v; }
  __device__ static P in_out(Out v) { return v; }
};
struct BF16 {
  using In = uint16_t;
  using P = float;
  using Out = float;
  static constexpr int L = 8;
  __device__ static P cvt(In v) { return __uint_as_float(((uint32_t)v) << 16); }  // exact upcast
  __device__ static void unpack(u32x4 r, P* o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = __uint_as_float(r[j] << 16);
      o[2 * j + 1] = __uint_as_float(r[j] & 0xFFFF0000u);
    }
  }
  __device__ static Out out(P v) { return v; }
  __device__ static P in_out(Out v) { return v; }
};
struct F64 {
  using In = double;
  using P = double;
  using Out = double;
  static constexpr int L = 2;
  __device__ static P cvt(In v) { return v; }
  __device__ static void unpack(u32x4 r, P* o) {
    o[0] = __hiloint2double((int)r[1], (int)r[0]);
    o[1] = __hiloint2double((int)r[3], (int)r[2]);
  }
  __device__ static Out out(P v) { return v; }
  __device__ static P in_out(Out v) { return v; }
};
struct F16 {
  using In = uint16_t;  // fp16 bit pattern
  using P = _Float16;
  using Out = uint16_t;
  static constexpr int L = 8;
  __device__ static P bits(uint16_t b) {
    P h;
    __builtin_memcpy(&h, &b, 2);
    return h;
  }
  __device__ static P cvt(In v) { return bits(v); }
  __device__ static void unpack(u32x4 r, P* o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = bits((uint16_t)(r[j] & 0xFFFFu));
      o[2 * j + 1] = bits((uint16_t)(r[j] >> 16));
    }
  }
  __device__ static Out out(P v) {
    uint16_t b;
    __builtin_memcpy(&b, &v, 2);
    return b;
  }
  __device__ static P in_out(Out v) { return bits(v); }
};

template <typename E, int KC>
struct FaArgs {
  const typename E::In* x[KC];
  typename E::P w[KC];
};

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else
    return *reinterpret_cast<const u32x4*>(p);
}

// out[v*L .. v*L+L) for one 16-byte vector of Out elements of width L.
template <typename E>
__device__ __forceinline__ void store_vec(typename E::Out* out, uint64_t v, const typename E::P* acc) {
  typename E::Out o[E::L];
#pragma unroll
  for (int j = 0; j < E::L; ++j) o[j] = E::out(acc[j]);
  constexpr int bytes = E::L * sizeof(typename E::Out);
  static_assert(bytes % 16 == 0, "output vector must be whole 16-byte stores");
  const u32x4* src = reinterpret_cast<const u32x4*>(o);
  u32x4* dst = reinterpret_cast<u32x4*>(out + v * E::L);
#pragma unroll
  for (int s = 0; s < bytes / 16; ++s) dst[s] = src[s];
}

template <typename E>
__device__ __forceinline__ void load_vec(const typename E::Out* out, uint64_t v, typename E::P* acc) {
  typename E::Out o[E::L];
  constexpr int bytes = E::L * sizeof(typename E::Out);
  const u32x4* src = reinterpret_cast<const u32x4*>(out + v * E::L);
  u32x4* dst = reinterpret_cast<u32x4*>(o);
#pragma unroll
  for (int s = 0; s < bytes / 16; ++s) dst[s] = src[s];
#pragma unroll
  for (int j = 0; j < E::L; ++j) acc[j] = E::in_out(o[j]);
}

// ------------------------------------------------------------------------------------
// FedAvg bucket kernel (fed_avg.py:217-222)
// ------------------------------------------------------------------------------------
template <typename E, int KC, bool NT>
__global__ void __launch_bounds__(FA_BLOCK)
    fedavg_kernel(const FaArgs<E, KC> a, const int K, const int first, const uint64_t nvec, const uint64_t M,
                  typename E::Out* __restrict__ out) {
#pragma clang fp contract(off)
  using P = typename E::P;
  constexpr int L = E::L;
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  const uint64_t gid = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x;

  for (uint64_t v = gid; v < nvec; v += stride) {
    P acc[L];
    if (first) {
#pragma unroll
      for (int j = 0; j < L; ++j) acc[j] = P(0.0f);  // NumPy seeds add.reduce with +0.0
    } else {
      load_vec<E>(out, v, acc);
    }
    int k = 0;
    for (; k + FA_UNROLL <= K; k += FA_UNROLL) {
      u32x4 raw[FA_UNROLL];
#pragma unroll
      for (int u = 0; u < FA_UNROLL; ++u) raw[u] = ld16<NT>(a.x[k + u] + v * L);
#pragma unroll
      for (int u = 0; u < FA_UNROLL; ++u) {
        P xs[L];
        E::unpack(raw[u], xs);
        const P w = a.w[k + u];
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const P p = xs[j] * w;  // fl(x_k * w_k)
          acc[j] = acc[j] + p;    // fl(acc + p), client order
        }
      }
    }
    for (; k < K; ++k) {
      const u32x4 raw = ld16<NT>(a.x[k] + v * L);
      P xs[L];
      E::unpack(raw, xs);
      const P w = a.w[k];
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const P p = xs[j] * w;
        acc[j] = acc[j] + p;
      }
    }
    store_vec<E>(out, v, acc);
  }

  // Scalar remainder (M % L elements, or everything when a pointer is not 16-B aligned).
  for (uint64_t i = nvec * L + gid; i < M; i += stride) {
    P acc = first ? P(0.0f) : E::in_out(out[i]);
    for (int k = 0; k < K; ++k) {
      const P p = E::cvt(a.x[k][i]) * a.w[k];
      acc = acc + p;
    }
    out[i] = E::out(acc);
  }
}

// ------------------------------------------------------------------------------------
// Scaffold two-bucket kernel (scaffold.py:204-295), fp64 products and sums
// ------------------------------------------------------------------------------------
template <typename TIn, int KC>
struct ScArgs {
  const TIn* d[KC];
  const TIn* cv[KC];
  double w[KC];
};

template <typename TIn>
__device__ __forceinline__ void unpack_d(u32x4 r, double* o) {
  if constexpr (sizeof(TIn) == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (double)__uint_as_float(r[j]);
  } else {
    o[0] = __hiloint2double((int)r[1], (int)r[0]);
    o[1] = __hiloint2double((int)r[3], (int)r[2]);
  }
}

template <typename TIn, int KC, bool NT>
__global__ void __launch_bounds__(FA_BLOCK)
    scaffold_kernel(const ScArgs<TIn, KC> a, const int K, const int first, const int last,
                    const TIn* __restrict__ c, const double lr, const uint64_t nvec, const uint64_t M,
                    double* __restrict__ dout, double* __restrict__ cout) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  constexpr int SU = FA_UNROLL / 2;  // two streams per client
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  const uint64_t gid = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x;

  for (uint64_t v = gid; v < nvec; v += stride) {
    double ad[L], ac[L];
    if (first) {
#pragma unroll
      for (int j = 0; j < L; ++j) ad[j] = ac[j] = 0.0;
    } else {
#pragma unroll
      for (int j = 0; j < L; ++j) {
        ad[j] = dout[v * L + j];
        ac[j] = cout[v * L + j];
      }
    }
    int k = 0;
    for (; k + SU <= K; k += SU) {
      u32x4 rd[SU], rc[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        rd[u] = ld16<NT>(a.d[k + u] + v * L);
        rc[u] = ld16<NT>(a.cv[k + u] + v * L);
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        double xd[L], xc[L];
        unpack_d<TIn>(rd[u], xd);
        unpack_d<TIn>(rc[u], xc);
        const double w = a.w[k + u];
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const double pd = w * xd[j];
          const double pc = w * xc[j];
          ad[j] = ad[j] + pd;
          ac[j] = ac[j] + pc;
        }
      }
    }
    for (; k < K; ++k) {
      double xd[L], xc[L];
      unpack_d<TIn>(ld16<NT>(a.d[k] + v * L), xd);
      unpack_d<TIn>(ld16<NT>(a.cv[k] + v * L), xc);
      const double w = a.w[k];
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const double pd = w * xd[j];
        const double pc = w * xc[j];
        ad[j] = ad[j] + pd;
        ac[j] = ac[j] + pc;
      }
    }
    if (last) {
      double xcc[L];
      unpack_d<TIn>(ld16<NT>(c + v * L), xcc);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        ac[j] = ac[j] + xcc[j];  // server c appended LAST (scaffold.py:262-263)
        ad[j] = lr * ad[j];      // aggregation_lr * sum (scaffold.py:293)
      }
    }
    f64x2* dd = reinterpret_cast<f64x2*>(dout + v * L);
    f64x2* cc = reinterpret_cast<f64x2*>(cout + v * L);
#pragma unroll
    for (int s = 0; s < L / 2; ++s) {
      f64x2 t0 = {ad[2 * s], ad[2 * s + 1]};
      f64x2 t1 = {ac[2 * s], ac[2 * s + 1]};
      dd[s] = t0;
      cc[s] = t1;
    }
  }
  for (uint64_t i = nvec * L + gid; i < M; i += stride) {
    double ad = first ? 0.0 : dout[i];
    double ac = first ? 0.0 : cout[i];
    for (int k = 0; k < K; ++k) {
      const double pd = a.w[k] * (double)a.d[k][i];
      const double pc = a.w[k] * (double)a.cv[k][i];
      ad = ad + pd;
      ac = ac + pc;
    }
    if (last) {
      ac = ac + (double)c[i];
      ad = lr * ad;
    }
    dout[i] = ad;
    cout[i] = ac;
  }
}

// ------------------------------------------------------------------------------------
// NumPy pairwise summation for numel == 1 tensors
// ------------------------------------------------------------------------------------
struct IdxArgs {
  uint64_t idx[FEDAGG_MAX_PAIRWISE];
};

// Stage 1: ws[p * stride + kbase + k] = fl(x_k[idx_p] * w_k), written in the
// accumulation type of the pairwise sum (fp32 for fp16 inputs: HALF_pairwise_sum).
template <typename E, int KC, typename TW>
__global__ void __launch_bounds__(FA_BLOCK)
    pairwise_gather_kernel(const FaArgs<E, KC> a, const int Kc, const int kbase, const IdxArgs ix, const int P,
                           const int64_t stride, TW* __restrict__ ws) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * FA_BLOCK + threadIdx.x;
  if (t >= P * Kc) return;
  const int p = t / Kc, k = t % Kc;
  const typename E::P prod = E::cvt(a.x[k][ix.idx[p]]) * a.w[k];
  ws[p * stride + kbase + k] = (TW)prod;
}

template <typename TIn, int KC>
__global__ void __launch_bounds__(FA_BLOCK)
    scaffold_gather_kernel(const ScArgs<TIn, KC> a, const int Kc, const int kbase, const IdxArgs ix, const int P,
                           const int64_t K, double* __restrict__ ws_d, double* __restrict__ ws_c) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * FA_BLOCK + threadIdx.x;
  if (t >= P * Kc) return;
  const int p = t / Kc, k = t % Kc;
  const uint64_t i = ix.idx[p];
  ws_d[p * K + kbase + k] = a.w[k] * (double)a.d[k][i];
  ws_c[p * (K + 1) + kbase + k] = a.w[k] * (double)a.cv[k][i];
}

template <typename T>
__device__ T pw_leaf(const T* a, int64_t n) {
#pragma clang fp contract(off)
  if (n < 8) {
    T res = T(-0.0);
    for (int64_t i = 0; i < n; ++i) res = res + a[i];
    return res;
  }
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
  }
  T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + a[i];
  return res;
}

// Iterative form of NumPy's recursive pairwise_sum (blocks of <= 128, split at n/2
// rounded down to a multiple of 8).
template <typename T>
__device__ T pw_sum(const T* a, int64_t n) {
#pragma clang fp contract(off)
  int64_t lo[64], nn[64];
  T left[64];
  int stage[64];
  int sp = 0;
  lo[0] = 0;
  nn[0] = n;
  stage[0] = 0;
  T ret = T(0);
  for (;;) {
    // descend
    while (nn[sp] > 128) {
      int64_t n2 = nn[sp] / 2;
      n2 -= n2 % 8;
      stage[sp] = 1;
      lo[sp + 1] = lo[sp];
      nn[sp + 1] = n2;
      stage[sp + 1] = 0;
      ++sp;
    }
    ret = pw_leaf(a + lo[sp], nn[sp]);
    // ascend
    bool done = true;
    while (sp > 0) {
      --sp;
      if (stage[sp] == 1) {
        left[sp] = ret;
        stage[sp] = 2;
        int64_t n2 = nn[sp] / 2;
        n2 -= n2 % 8;
        lo[sp + 1] = lo[sp] + n2;
        nn[sp + 1] = nn[sp] - n2;
        stage[sp + 1] = 0;
        ++sp;
        done = false;
        break;
      }
      ret = left[sp] + ret;
    }
    if (done) return ret;
  }
}

// Stage 2: out[idx_p] = (+0.0 + pairwise(ws[p])) (times lr for Scaffold's delta).
template <typename TW, typename E>
__global__ void pairwise_tree_kernel(const TW* __restrict__ ws, const int64_t n, const IdxArgs ix, const int P,
                                     typename E::Out* __restrict__ out) {
#pragma clang fp contract(off)
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const TW s = TW(0.0f) + pw_sum(ws + p * n, n);
  out[ix.idx[p]] = E::out((typename E::P)s);
}

__global__ void scaffold_tree_kernel(const double* __restrict__ ws_d, const double* __restrict__ ws_c,
                                     const int64_t K, const IdxArgs ix, const int P, const double lr,
                                     double* __restrict__ dout, double* __restrict__ cout) {
#pragma clang fp contract(off)
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const double sd = 0.0 + pw_sum(ws_d + p * K, K);
  const double sc = 0.0 + pw_sum(ws_c + p * (K + 1), K + 1);
  dout[ix.idx[p]] = lr * sd;
  cout[ix.idx[p]] = sc;
}

__global__ void scaffold_c_tail_kernel(const float* c32, const double* c64, const IdxArgs ix, const int P,
                                       const int64_t K, double* __restrict__ ws_c) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  ws_c[p * (K + 1) + K] = c32 ? (double)c32[ix.idx[p]] : c64[ix.idx[p]];
}

// ------------------------------------------------------------------------------------
// Scaffold server-control-variate equality check (scaffold.py:193-196)
// ------------------------------------------------------------------------------------
template <typename T, int KC>
struct EqArgs {
  const T* x[KC];
};

template <typename T, int KC>
__global__ void __launch_bounds__(FA_BLOCK)
    equal_count_kernel(const EqArgs<T, KC> a, const int K, const T* __restrict__ ref, const uint64_t M,
                       unsigned long long* __restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  unsigned long long bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; i < M; i += stride) {
    const T r = ref[i];
    for (int k = 0; k < K; ++k) {
      const T v = a.x[k][i];
      bad += !((v == r) || (v != v && r != r));
    }
  }
  // wave reduction, then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(cnt, bad);
}

// ------------------------------------------------------------------------------------
// read-stream probe
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(FA_BLOCK) read_probe_kernel(const float* __restrict__ x, uint64_t nvec,
                                                              float* __restrict__ sink) {
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  for (uint64_t v = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; v < nvec; v += stride) {
    u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x) + v);
    s.x += __uint_as_float(r.x);
    s.y += __uint_as_float(r.y);
    s.z += __uint_as_float(r.z);
    s.w += __uint_as_float(r.w);
  }
  float t = s.x + s.y + s.z + s.w;
  for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
  if (threadIdx.x == 0) sink[blockIdx.x] = t;
}

// ------------------------------------------------------------------------------------
// host-side launch helpers
// ------------------------------------------------------------------------------------
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline unsigned grid_for(uint64_t work) {
  uint64_t g = (work + FA_BLOCK - 1) / FA_BLOCK;
  if (g < 1) g = 1;
  if (g > (uint64_t)g_grid_cap) g = (uint64_t)g_grid_cap;
  return (unsigned)g;
}

template <typename E>
int fedavg_launch(const typename E::In* const* x, const typename E::P* w, int K, uint64_t M,
                  typename E::Out* out, hipStream_t s) {
  if (K <= 0) return fail(FEDAGG_EINVAL, "fedavg: K must be > 0 (got %s%lld)", "", K);
  if (!x || !w || !out) return fail(FEDAGG_EINVAL, "fedavg: NULL argument%s%lld", "", 0);
  if (M == 0) return FEDAGG_OK;
  bool vec = aligned16(out);
  for (int k = 0; k < K && vec; ++k) {
    if (!x[k]) return fail(FEDAGG_EINVAL, "fedavg: client pointer %s%lld is NULL", "", k);
    vec = aligned16(x[k]);
  }
  const uint64_t nvec = vec ? M / E::L : 0;
  const unsigned grid = grid_for(nvec ? nvec : M);
  for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK) {
    const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
    FaArgs<E, FEDAGG_KCHUNK> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) {
      if (!x[k0 + k]) return fail(FEDAGG_EINVAL, "fedavg: client pointer %s%lld is NULL", "", k0 + k);
      a.x[k] = x[k0 + k];
      a.w[k] = w[k0 + k];
    }
    if (g_nontemporal)
      hipLaunchKernelGGL((fedavg_kernel<E, FEDAGG_KCHUNK, true>), dim3(grid), dim3(FA_BLOCK), 0, s, a, kc,
                         k0 == 0 ? 1 : 0, nvec, M, out);
    else
      hipLaunchKernelGGL((fedavg_kernel<E, FEDAGG_KCHUNK, false>), dim3(grid), dim3(FA_BLOCK), 0, s, a, kc,
                         k0 == 0 ? 1 : 0, nvec, M, out);
    int rc = check_launch("fedavg_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

template <typename E, typename TW>
int fedavg_pairwise_launch(const typename E::In* const* x, const typename E::P* w, int K, const uint64_t* idx, int P,
                           void* ws, typename E::Out* out, hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (K <= 0 || P < 0 || !x || !w || !idx || !ws || !out)
    return fail(FEDAGG_EINVAL, "fedavg_pairwise: invalid argument%s%lld", "", 0);
  TW* wsT = static_cast<TW*>(ws);
  for (int p0 = 0; p0 < P; p0 += FEDAGG_MAX_PAIRWISE) {
    const int pc = (P - p0) < FEDAGG_MAX_PAIRWISE ? (P - p0) : FEDAGG_MAX_PAIRWISE;
    IdxArgs ix;
    memset(&ix, 0, sizeof(ix));
    for (int p = 0; p < pc; ++p) ix.idx[p] = idx[p0 + p];
    for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK) {
      const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
      FaArgs<E, FEDAGG_KCHUNK> a;
      memset(&a, 0, sizeof(a));
      for (int k = 0; k < kc; ++k) {
        a.x[k] = x[k0 + k];
        a.w[k] = w[k0 + k];
      }
      const unsigned g = (unsigned)((pc * kc + FA_BLOCK - 1) / FA_BLOCK);
      hipLaunchKernelGGL((pairwise_gather_kernel<E, FEDAGG_KCHUNK, TW>), dim3(g), dim3(FA_BLOCK), 0, s, a, kc, k0,
                         ix, pc, (int64_t)K, wsT);
      int rc = check_launch("pairwise_gather_kernel");
      if (rc) return rc;
    }
    hipLaunchKernelGGL((pairwise_tree_kernel<TW, E>), dim3(1), dim3(64), 0, s, wsT, (int64_t)K, ix, pc, out);
    int rc = check_launch("pairwise_tree_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

template <typename TIn>
int scaffold_launch(const TIn* const* d, const TIn* const* cv, const TIn* c, const double* w, int K, uint64_t M,
                    double lr, double* dout, double* cout, hipStream_t s) {
  if (K <= 0) return fail(FEDAGG_EINVAL, "scaffold: K must be > 0 (got %s%lld)", "", K);
  if (!d || !cv || !c || !w || !dout || !cout) return fail(FEDAGG_EINVAL, "scaffold: NULL argument%s%lld", "", 0);
  if (M == 0) return FEDAGG_OK;
  bool vec = aligned16(c) && aligned16(dout) && aligned16(cout);
  for (int k = 0; k < K && vec; ++k) {
    if (!d[k] || !cv[k]) return fail(FEDAGG_EINVAL, "scaffold: client pointer %s%lld is NULL", "", k);
    vec = aligned16(d[k]) && aligned16(cv[k]);
  }
  constexpr int L = 16 / sizeof(TIn);
  const uint64_t nvec = vec ? M / L : 0;
  const unsigned grid = grid_for(nvec ? nvec : M);
  for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK_SCAFFOLD) {
    const int kc = (K - k0) < FEDAGG_KCHUNK_SCAFFOLD ? (K - k0) : FEDAGG_KCHUNK_SCAFFOLD;
    ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) {
      if (!d[k0 + k] || !cv[k0 + k])
        return fail(FEDAGG_EINVAL, "scaffold: client pointer %s%lld is NULL", "", k0 + k);
      a.d[k] = d[k0 + k];
      a.cv[k] = cv[k0 + k];
      a.w[k] = w[k0 + k];
    }
    const int first = k0 == 0, last = (k0 + kc) == K;
    if (g_nontemporal)
      hipLaunchKernelGGL((scaffold_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, true>), dim3(grid), dim3(FA_BLOCK), 0, s, a,
                         kc, first, last, c, lr, nvec, M, dout, cout);
    else
      hipLaunchKernelGGL((scaffold_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, false>), dim3(grid), dim3(FA_BLOCK), 0, s,
                         a, kc, first, last, c, lr, nvec, M, dout, cout);
    int rc = check_launch("scaffold_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

template <typename TIn>
int scaffold_pairwise_launch(const TIn* const* d, const TIn* const* cv, const TIn* c, const double* w, int K,
                             const uint64_t* idx, int P, double lr, void* ws, double* dout, double* cout,
                             hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (K <= 0 || P < 0 || !d || !cv || !c || !w || !idx || !ws || !dout || !cout)
    return fail(FEDAGG_EINVAL, "scaffold_pairwise: invalid argument%s%lld", "", 0);
  double* ws_d = static_cast<double*>(ws);
  double* ws_c = ws_d + (size_t)FEDAGG_MAX_PAIRWISE * K;
  for (int p0 = 0; p0 < P; p0 += FEDAGG_MAX_PAIRWISE) {
    const int pc = (P - p0) < FEDAGG_MAX_PAIRWISE ? (P - p0) : FEDAGG_MAX_PAIRWISE;
    IdxArgs ix;
    memset(&ix, 0, sizeof(ix));
    for (int p = 0; p < pc; ++p) ix.idx[p] = idx[p0 + p];
    for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK_SCAFFOLD) {
      const int kc = (K - k0) < FEDAGG_KCHUNK_SCAFFOLD ? (K - k0) : FEDAGG_KCHUNK_SCAFFOLD;
      ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD> a;
      memset(&a, 0, sizeof(a));
      for (int k = 0; k < kc; ++k) {
        a.d[k] = d[k0 + k];
        a.cv[k] = cv[k0 + k];
        a.w[k] = w[k0 + k];
      }
      const unsigned g = (unsigned)((pc * kc + FA_BLOCK - 1) / FA_BLOCK);
      hipLaunchKernelGGL((scaffold_gather_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD>), dim3(g), dim3(FA_BLOCK), 0, s, a,
                         kc, k0, ix, pc, (int64_t)K, ws_d, ws_c);
      int rc = check_launch("scaffold_gather_kernel");
      if (rc) return rc;
    }
    const float* c32 = sizeof(TIn) == 4 ? reinterpret_cast<const float*>(c) : nullptr;
    const double* c64 = sizeof(TIn) == 8 ? reinterpret_cast<const double*>(c) : nullptr;
    hipLaunchKernelGGL(scaffold_c_tail_kernel, dim3(1), dim3(64), 0, s, c32, c64, ix, pc, (int64_t)K, ws_c);
    hipLaunchKernelGGL(scaffold_tree_kernel, dim3(1), dim3(64), 0, s, ws_d, ws_c, (int64_t)K, ix, pc, lr, dout,
                       cout);
    int rc = check_launch("scaffold_tree_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

template <typename T>
int equal_launch(const T* const* x, int K, uint64_t M, unsigned long long* cnt, hipStream_t s) {
  if (K <= 0 || !x || !cnt) return fail(FEDAGG_EINVAL, "equal_count: invalid argument%s%lld", "", 0);
  if (M == 0 || K == 1) return FEDAGG_OK;
  const unsigned grid = grid_for(M);
  for (int k0 = 1; k0 < K; k0 += FEDAGG_KCHUNK) {
    const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
    EqArgs<T, FEDAGG_KCHUNK> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) a.x[k] = x[k0 + k];
    hipLaunchKernelGGL((equal_count_kernel<T, FEDAGG_KCHUNK>), dim3(grid), dim3(FA_BLOCK), 0, s, a, kc, x[0], M,
                       cnt);
    int rc = check_launch("equal_count_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

}  // namespace

// ======================================================================================
// C ABI
// ======================================================================================
extern "C" {

int fedagg_abi_version(void) { return FEDAGG_ABI_VERSION; }
const char* fedagg_last_error(void) { return g_err; }

int fedagg_set_launch(int grid_cap, int nontemporal) {
  if (grid_cap > 0) g_grid_cap = grid_cap;
  if (nontemporal >= 0) g_nontemporal = nontemporal ? 1 : 0;
  return FEDAGG_OK;
}

int fedagg_fedavg_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M, float* d_out,
                      void* stream) {
  return fedavg_launch<F32>(d_clients, h_w, K, M, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M, float* d_out,
                       void* stream) {
  return fedavg_launch<BF16>(d_clients, h_w, K, M, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_f64(const double* const* d_clients, const double* h_w, int K, uint64_t M, double* d_out,
                      void* stream) {
  return fedavg_launch<F64>(d_clients, h_w, K, M, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, uint64_t M, uint16_t* d_out,
                      void* stream) {
  if (!h_w) return fail(FEDAGG_EINVAL, "fedavg_f16: NULL weights%s%lld", "", 0);
  _Float16 w[FEDAGG_KCHUNK];
  // weights travel as fp16 bit patterns; reinterpret in chunks
  if (K <= 0) return fail(FEDAGG_EINVAL, "fedavg_f16: K must be > 0 (got %s%lld)", "", K);
  // fedavg_launch reads w[k] for k < K; build a contiguous _Float16 copy
  _Float16* wf = K <= FEDAGG_KCHUNK ? w : new _Float16[K];
  memcpy(wf, h_w, sizeof(uint16_t) * (size_t)K);
  int rc = fedavg_launch<F16>(d_clients, wf, K, M, d_out, (hipStream_t)stream);
  if (wf != w) delete[] wf;
  return rc;
}

size_t fedagg_pairwise_ws_bytes(int K, int P, int elem_bytes) {
  (void)P;
  if (K <= 0) return 0;
  // per launch chunk: up to FEDAGG_MAX_PAIRWISE segments x (K + 1) terms, two buckets
  return (size_t)2 * FEDAGG_MAX_PAIRWISE * (size_t)(K + 1) * (size_t)(elem_bytes < 8 ? 8 : elem_bytes);
}

int fedagg_fedavg_pairwise_f32(const float* const* d_clients, const float* h_w, int K, const uint64_t* h_idx, int P,
                               void* d_ws, float* d_out, void* stream) {
  return fedavg_pairwise_launch<F32, float>(d_clients, h_w, K, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_pairwise_bf16(const uint16_t* const* d_clients, const float* h_w, int K, const uint64_t* h_idx,
                                int P, void* d_ws, float* d_out, void* stream) {
  return fedavg_pairwise_launch<BF16, float>(d_clients, h_w, K, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_pairwise_f64(const double* const* d_clients, const double* h_w, int K, const uint64_t* h_idx, int P,
                               void* d_ws, double* d_out, void* stream) {
  return fedavg_pairwise_launch<F64, double>(d_clients, h_w, K, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_pairwise_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, const uint64_t* h_idx,
                               int P, void* d_ws, uint16_t* d_out, void* stream) {
  if (K <= 0 || !h_w) return fail(FEDAGG_EINVAL, "fedavg_pairwise_f16: invalid argument%s%lld", "", 0);
  _Float16* wf = new _Float16[K];
  memcpy(wf, h_w, sizeof(uint16_t) * (size_t)K);
  int rc = fedavg_pairwise_launch<F16, float>(d_clients, wf, K, h_idx, P, d_ws, d_out, (hipStream_t)stream);
  delete[] wf;
  return rc;
}

int fedagg_scaffold_f32(const float* const* d_delta, const float* const* d_cv, const float* d_c, const double* h_w,
                        int K, uint64_t M, double lr, double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_launch<float>(d_delta, d_cv, d_c, h_w, K, M, lr, d_delta_out, d_c_out, (hipStream_t)stream);
}
int fedagg_scaffold_f64(const double* const* d_delta, const double* const* d_cv, const double* d_c,
                        const double* h_w, int K, uint64_t M, double lr, double* d_delta_out, double* d_c_out,
                        void* stream) {
  return scaffold_launch<double>(d_delta, d_cv, d_c, h_w, K, M, lr, d_delta_out, d_c_out, (hipStream_t)stream);
}
int fedagg_scaffold_pairwise_f32(const float* const* d_delta, const float* const* d_cv, const float* d_c,
                                 const double* h_w, int K, const uint64_t* h_idx, int P, double lr, void* d_ws,
                                 double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_pairwise_launch<float>(d_delta, d_cv, d_c, h_w, K, h_idx, P, lr, d_ws, d_delta_out, d_c_out,
                                         (hipStream_t)stream);
}
int fedagg_scaffold_pairwise_f64(const double* const* d_delta, const double* const* d_cv, const double* d_c,
                                 const double* h_w, int K, const uint64_t* h_idx, int P, double lr, void* d_ws,
                                 double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_pairwise_launch<double>(d_delta, d_cv, d_c, h_w, K, h_idx, P, lr, d_ws, d_delta_out, d_c_out,
                                          (hipStream_t)stream);
}

int fedagg_equal_count_f32(const float* const* d_copies, int K, uint64_t M, unsigned long long* d_mismatches,
                           void* stream) {
  return equal_launch<float>(d_copies, K, M, d_mismatches, (hipStream_t)stream);
}
int fedagg_equal_count_f64(const double* const* d_copies, int K, uint64_t M, unsigned long long* d_mismatches,
                           void* stream) {
  return equal_launch<double>(d_copies, K, M, d_mismatches, (hipStream_t)stream);
}

int fedagg_read_probe_f32(const float* d_x, uint64_t M, float* d_sink, int grid, void* stream) {
  if (!d_x || !d_sink || grid <= 0 || !aligned16(d_x))
    return fail(FEDAGG_EINVAL, "read_probe: invalid argument%s%lld", "", 0);
  hipLaunchKernelGGL(read_probe_kernel, dim3(grid), dim3(FA_BLOCK), 0, (hipStream_t)stream, d_x, M / 4, d_sink);
  return check_launch("read_probe_kernel");
}

}  // extern "C"
