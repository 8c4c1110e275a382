// fedagg.hip -- hand-written gfx950 (MI355X / CDNA4) kernels for SubstraFL's aggregation
// hot path, behind the C ABI declared in include/fedagg.h.
//
// The path is element-wise and HBM-bound (0.5 FLOP per input byte for fp32 FedAvg), so
// the design is a pure streaming one -- no MFMA, no LDS staging of the client streams:
//   * one thread owns one 16-byte vector of the flat bucket (4 fp32 / 8 bf16 / 2 fp64 /
//     8 fp16 elements) and walks the K clients IN LIST ORDER, which is the order the
//     reference's np.sum(list, axis=0) adds them (fed_avg.py:221-222);
//   * the client loop is unrolled by FA_UNROLL with all loads issued before the dependent
//     add chain, so every lane keeps FA_UNROLL x 16 B (x VPT vectors) in flight;
//   * client pointers and weights live in the kernel-argument segment (scalar loads,
//     no device-side table, graph-capturable); clients beyond FEDAGG_KCHUNK continue
//     from the partial sum already in `out`, which is exact because the accumulator
//     type is the stored type;
//   * numel == 1 tensors (NumPy pairwise order) are patched inside the
//     same launch by the thread that owns their vector, computing the pairwise tree from the
//     client pointers directly (single-chunk launches, <= FEDAGG_FUSED_PAIRWISE indices);
//     larger cases fall back to the separate gather + tree kernels;
//   * grid-stride over the bucket with a launch of a few thousand 256-thread workgroups
//     (>> 256 CUs; blocks are dealt round-robin over the 8 XCDs and have no reuse to
//     localise, so no XCD remap is needed here).
// Bit parity with NumPy requires every product and sum to be rounded separately: the
// file is compiled with -ffp-contract=off AND every kernel body carries
// `#pragma clang fp contract(off)` (hipcc otherwise emits v_fmac_f32 for acc + x*w).

#include <hip/hip_runtime.h>

#include <type_traits>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <vector>

#include "fedagg.h"

// FEDAGG_TUNING=1 (`__graft_entry__.build(tuning=True)`, tools/): every launch variant the
// experiment knobs of fedagg_tune select is instantiated -- the shapes, load paths, occupancy caps
// and walks DESIGN.md records as measured and not kept.  The product library (the default) holds
// only the shapes the default dispatch selects (shape_for, the Scaffold launch plan, the tiled
// kernels) and refuses the experiment knobs.
#ifndef FEDAGG_TUNING
#define FEDAGG_TUNING 0
#endif

#define FA_BLOCK 256
#define FA_UNROLL 8

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, long long b = 0) {
  snprintf(g_err, sizeof(g_err), fmt, b);
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

// Launch shape (fedagg_tune); defaults are the values measured best on MI355X.
int g_grid_cap = 0;     // workgroups per launch before grid-striding (0: one step per workgroup)
int g_nt_load = 1;      // client streams are read once: non-temporal loads
int g_nt_store = 1;     // non-temporal output stores (-1: auto, on from NT_STORE_MIN_K clients)
int g_vpt = 0;          // 16-byte vectors per thread per step (0: auto, see shape_for)
int g_unroll = 8;       // clients per load group (ignored when vpt is auto)
int g_pipe = 0;         // software-pipelined client groups
int g_tile = 1;         // a workgroup step covers VPT*256 contiguous vectors
int g_fuse_pw = 1;      // patch numel==1 tensors inside the bucket launch
int g_sc_vpt = 0;       // Scaffold: 16-byte vectors per thread per step (1/2/4/8; 0: auto, sc_shape_for)
int g_sc_unroll = 4;    // Scaffold: clients per load group (2/4/8, with an explicit sc_vpt)
[[maybe_unused]] int g_sc_split = 0;     // Scaffold: phase-split walk (all delta streams, then all control-variate streams)
int g_buf = 0;          // FedAvg: buffer-descriptor client loads (8/16-KiB tiles, fp32/bf16)
int g_fa_occ = 0;       // FedAvg: register-capped occupancy variants (0: off; 2-4 with the 8/16-KiB shapes)
int g_sc_buf = 0;       // Scaffold: buffer-descriptor client loads (fp32 inputs, 4- and 8-vector tiles)
int g_sc_bsplit = 0;    // Scaffold: bucket-split workgroup pairs (delta / control variate per workgroup)
int g_flat_vec = 1;     // 16-B (4-element) client flat ops when every operand is fp32
int g_eq_vec = 1;       // vectorised c-equality check (16-B loads) when every copy is 16-B aligned
int g_sc_pipe = 0;      // Scaffold: software-pipelined client groups (next group's loads before this group's adds)
int g_tpb = 1;          // consecutive tiles per workgroup (1: one step per workgroup)
[[maybe_unused]] int g_sc_cpf = 0;       // Scaffold 4 x 4 tile: c loaded with the last client group
[[maybe_unused]] int g_sc_occ = 0;       // Scaffold 4 x 4 tile: register-capped build (waves per SIMD, 0 = uncapped)
[[maybe_unused]] int g_sc_blk = 256;     // Scaffold 4 x 4 tile: threads per workgroup (256 or 512)
int g_sc_2l = -1;       // Scaffold: one bucket at a time (-1 auto: from SC_2L_MIN_K clients; 1 / 2 / 0)
[[maybe_unused]] int g_sc_sc1 = 0;       // Scaffold 4 x 4 tiles: write-through (sc1) output stores
int g_tiled_few = 0;    // recommend the tile-interleaved layout below 32 fp32 clients too (fedagg_tune "tiled_few";
                        // 8 x 25M: 134.5 vs 134.4 us on rows, profiles/r02_layout_c2_*.json -- no gain)
int g_st_sc1 = -1;      // FedAvg: write-through (sc1) output stores (-1: auto, below SC1_MAX_K clients)
int g_fa_blk = 0;       // FedAvg fp32/bf16 global-load tiles: threads per workgroup (0 auto, 256, 512)
int g_xcd = 0;          // XCD-contiguous tile order (blocks sharing an XCD take adjacent tiles)
// Push runs (fedagg_fedavg_chain_push_f32): the accumulator is a peer GPU's memory mapped over
// xGMI.  Their output stores are system-scope write-through stores (st16<3>: sc0 sc1) and every
// wave waits for their acknowledgements before it retires (s_waitcnt vmcnt(0)), so the stores are
// performed at system scope before the executor's tag / counter writes that follow the launch.
// (A per-wave system-scope release fence -- buffer_wbl2 sc0 sc1 -- does the same for stores that
// sit in this GPU's L2, which these never do; it cost 26-204 % of the run's time on one MI355X,
// profiles/r04_push_overhead.jsonl, for nothing the write-through stores do not already give.)
thread_local int g_rel_sys = 0;
// Push runs: the input accumulator (this rank's slot, fp32 for f32 and bf16 buckets) when the
// output is elsewhere (a peer's slot); the first client chunk reads it instead of `out`.
thread_local const void* g_acc_in = nullptr;
constexpr int NT_STORE_MIN_K = 16;
// Output stores as device-scope write-through (sc1) instead of non-temporal: 8 x 25M fp32 133.6
// vs 140.0 us, fp16 71.5 vs 75.0, fp64 280 vs 298; from 32 clients the output is <= 3 % of the
// bytes and it is neutral (64 x 125M fp32 +0.4 %, 128 x 350M bf16 -0.6 %; profiles/r02_sc1_*.log)
constexpr int SC1_MAX_K = 32;
// Scaffold one bucket at a time (two launches, K streams in flight instead of 2K + 1), 8 x 4
// tiles: 16 x 25M fp32 571 vs 594 us for the fused 4 x 4 walk, 32 x 25M 1.032 vs 1.087 ms,
// 64 x 25M 1.949 vs 2.013 ms; 8 x 100M ties (1.467 ms either way), so the fused walk stays
// below 16 clients for fp32 inputs; fp64 inputs take the pipelined one-bucket tiles at any K
// (profiles/r02_sc2l_*.log)
constexpr int SC_2L_MIN_K = 16;

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------
// element types: storage type In, product/accumulate type P, output storage Out,
// pairwise-sum accumulation type W (NumPy's HALF_pairwise_sum sums in fp32)
// ------------------------------------------------------------------------------------
struct F32 {
  using In = float;
  using P = float;
  using Out = float;
  using W = float;
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
  using W = float;
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
  using W = double;
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
  using W = float;
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

// numel == 1 element indices patched inside the bucket launch
struct PwArgs {
  uint64_t idx[FEDAGG_FUSED_PAIRWISE];
  int n;
};

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  else
    return *reinterpret_cast<const u32x4*>(p);
}

// Store policy SP: 0 plain, 1 non-temporal, 2 device-scope write-through (sc1) as a buffer store
// based at the first active lane's address (callers' lanes store at ascending addresses within
// one wave, so every lane offset is a small non-negative 32-bit number), 3 the same store at system
// scope (sc0 sc1: written through to memory -- a peer GPU's over xGMI -- and acknowledged from
// there; the push executor's runs, which then wait for their acknowledgements before retiring).
template <int SP>
__device__ __forceinline__ void st16(void* p, u32x4 v) {
  if constexpr (SP == 2 || SP == 3) {
    const uint64_t addr = reinterpret_cast<uint64_t>(p);
    // readfirstlane returns int: widen through unsigned (a sign-extended low word would corrupt
    // the high address bits)
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(addr >> 32));
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)addr);
    const uint64_t base = ((uint64_t)hi << 32) | (uint64_t)lo;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(addr - base), 0, SP == 3 ? 17 : 16);  // sc0 = 1, sc1 = 16
  } else if constexpr (SP == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  } else {
    *reinterpret_cast<u32x4*>(p) = v;
  }
}

// out[v*L .. v*L+L) for one 16-byte input vector (L Out elements: 16 or 32 bytes).
template <typename E, int NTS>
__device__ __forceinline__ void store_vec(typename E::Out* out, uint64_t v, const typename E::P* acc) {
  typename E::Out o[E::L];
#pragma unroll
  for (int j = 0; j < E::L; ++j) o[j] = E::out(acc[j]);
  constexpr int bytes = E::L * sizeof(typename E::Out);
  static_assert(bytes % 16 == 0, "output vector must be whole 16-byte stores");
  const u32x4* src = reinterpret_cast<const u32x4*>(o);
#pragma unroll
  for (int s = 0; s < bytes / 16; ++s) st16<NTS>(reinterpret_cast<u32x4*>(out + v * E::L) + s, src[s]);
}

// A wave's 64 lanes each own 32 contiguous output bytes (bf16->fp32 FedAvg, fp32->fp64
// Scaffold) of one 2 KiB run.  Stored directly, every store instruction would write 16 B per
// lane at a 32-B stride (half of each 64-B line per instruction: PMC WRITE_SIZE showed 1.36x
// the written bytes).  Transposing through 2 KiB of LDS turns them into two fully coalesced
// 1 KiB store instructions.  Requires all 64 lanes active (callers check wave-uniformly).
template <int NTS>
__device__ __forceinline__ void store32_coalesced(void* wave_dst, u32x4 lo, u32x4 hi, u32x4* lds_wave) {
  const int lane = threadIdx.x & 63;
  lds_wave[2 * lane] = lo;
  lds_wave[2 * lane + 1] = hi;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const u32x4 a = lds_wave[lane];
  const u32x4 b = lds_wave[64 + lane];
  st16<NTS>(reinterpret_cast<u32x4*>(wave_dst) + lane, a);
  st16<NTS>(reinterpret_cast<u32x4*>(wave_dst) + 64 + lane, b);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // WAR before the buffer is reused
  __builtin_amdgcn_wave_barrier();
}

template <typename E, int NTS>
__device__ __forceinline__ void store_vec_wave(typename E::Out* out, uint64_t v, const typename E::P* acc,
                                               bool wave_full, u32x4* lds_wave) {
  constexpr int bytes = E::L * sizeof(typename E::Out);
  if constexpr (bytes == 32) {
    if (wave_full) {
      typename E::Out o[E::L];
#pragma unroll
      for (int j = 0; j < E::L; ++j) o[j] = E::out(acc[j]);
      const u32x4* src = reinterpret_cast<const u32x4*>(o);
      const uint64_t v0 = v - (threadIdx.x & 63);
      store32_coalesced<NTS>(out + v0 * E::L, src[0], src[1], lds_wave);
      return;
    }
  }
  store_vec<E, NTS>(out, v, acc);
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
// NumPy pairwise summation (loops_utils.h.src pairwise_sum, PW_BLOCKSIZE 128), on a
// generator get(i) of the n terms.  n <= 128: one leaf.
// ------------------------------------------------------------------------------------
template <typename T, typename G>
__device__ __forceinline__ T pw_leaf(const G& get, int64_t lo, int64_t n) {
#pragma clang fp contract(off)
  if (n < 8) {
    T res = T(-0.0);
    for (int64_t i = 0; i < n; ++i) res = res + get(lo + i);
    return res;
  }
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = get(lo + j);
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + get(lo + i + j);
  }
  T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + get(lo + i);
  return res;
}

// Iterative form of the recursive split (n > 128: split at n/2 rounded down to a multiple of 8).
template <typename T, typename G>
__device__ T pw_sum(const G& get, int64_t n) {
#pragma clang fp contract(off)
  if (n <= 128) return pw_leaf<T>(get, 0, n);
  int64_t lo[64], nn[64];
  T left[64];
  int stage[64];
  int sp = 0;
  lo[0] = 0;
  nn[0] = n;
  stage[0] = 0;
  T ret = T(0);
  for (;;) {
    while (nn[sp] > 128) {  // descend into left halves
      int64_t n2 = nn[sp] / 2;
      n2 -= n2 % 8;
      stage[sp] = 1;
      lo[sp + 1] = lo[sp];
      nn[sp + 1] = n2;
      stage[sp + 1] = 0;
      ++sp;
    }
    ret = pw_leaf<T>(get, lo[sp], nn[sp]);
    bool done = true;
    while (sp > 0) {  // ascend: left done -> start right; right done -> combine
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

// Tile-interleaved client buckets (fedagg_fedavg_tiled_*): the K clients' tiles of TV 16-B
// vectors alternate in HBM -- tile t of client k at vector (t * K + k) * TV -- so a workgroup
// reads ONE contiguous K x TV region per step instead of K regions a row apart.  With the
// per-client base base_k = base + k * TV, client k's vector v is at (v / TV) * pitch + v % TV of
// base_k, pitch = K * TV.  TV = 0: the [K, ld] row layout (identity).
template <int TV>
__device__ __forceinline__ uint64_t in_vec(uint64_t v, uint64_t pitch) {
  if constexpr (TV == 0) return v;
  else return (v / TV) * pitch + v % TV;
}
template <int TV, int L>
__device__ __forceinline__ uint64_t in_elem(uint64_t e, uint64_t pitch) {
  if constexpr (TV == 0) return e;
  else return in_vec<TV>(e / L, pitch) * L + e % L;
}

// Fused numel==1 patch: +0.0 + pairwise over the K products of element e (e: the element's
// index in the client's bucket storage, see in_elem).
template <typename E, int KC>
__device__ __forceinline__ typename E::P fedavg_pairwise_elem(const FaArgs<E, KC>& a, int K, uint64_t e) {
#pragma clang fp contract(off)
  using W = typename E::W;
  auto get = [&](int64_t k) -> W { return (W)(E::cvt(a.x[k][e]) * a.w[k]); };
  const W s = W(0.0f) + pw_leaf<W>(get, 0, K);
  return (typename E::P)s;
}

// Tile order.  The dispatcher deals blocks round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// "Workgroup dispatch"), so with the identity order the blocks resident on one XCD are spread
// over 8x the address span of the grid's in-flight window, in every client stream.  remap = 1
// gives the blocks of one `b % 8` group a contiguous run of tiles (bijective for any grid size),
// so each XCD streams one compact window per client.  Speed only: any order is correct.
__device__ __forceinline__ uint64_t tile_of_block(const int remap) {
  const uint32_t b = blockIdx.x, G = gridDim.x;
  if (!remap || G < 16) return b;
  const uint32_t q = G / 8, r = G % 8, x = b % 8, i = b / 8;
  return (uint64_t)(x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// it-th tile of this block: the grid-stride order above (tpb == 1), or tpb consecutive tiles
// per block (tpb > 1; the caller divides the grid by tpb).  Speed only.
__device__ __forceinline__ bool block_tile(const int remap, const int tpb, const uint64_t it, uint64_t* t) {
  if (tpb > 1) {
    if (it >= (uint64_t)tpb) return false;
    *t = (uint64_t)blockIdx.x * tpb + it;
  } else {
    *t = tile_of_block(remap) + it * gridDim.x;
  }
  return true;
}

// ------------------------------------------------------------------------------------
// FedAvg bucket kernel (fed_avg.py:217-222)
// ------------------------------------------------------------------------------------
// One group of U clients for N vectors: products and in-order adds.
template <typename E, int N, int U>
__device__ __forceinline__ void fedavg_accumulate(const u32x4 (&raw)[N][U], const typename E::P* w,
                                                  typename E::P (*acc)[E::L]) {
#pragma clang fp contract(off)
  using P = typename E::P;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const P wu = w[u];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      P xs[E::L];
      E::unpack(raw[n][u], xs);
#pragma unroll
      for (int j = 0; j < E::L; ++j) {
        const P p = xs[j] * wu;       // fl(x_k * w_k)
        acc[n][j] = acc[n][j] + p;    // fl(acc + p), client order
      }
    }
  }
}

// BUF: raw buffer loads through one descriptor per client based at this workgroup's tile (byte
// offset tb, scalar): every load addresses with the same 32-bit lane offset plus a scalar n*4 KiB,
// instead of one 64-bit VGPR address per (client, vector).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* row, uint64_t tb) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(static_cast<const char*>(row)) + tb, 0, 0x7FFFFFFF,
                                           0x00020000);
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16_buf(__amdgpu_buffer_rsrc_t r, int n) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(threadIdx.x * 16u), n * FA_BLOCK * 16, NT ? 2 : 0);
}

template <typename E, int KC, bool NT, int N, int U, bool BUF = false>
__device__ __forceinline__ void fedavg_load_group(const FaArgs<E, KC>& a, int k, const uint64_t* v,
                                                  u32x4 (&raw)[N][U], uint64_t tb = 0) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (BUF) {
      const __amdgpu_buffer_rsrc_t r = tile_rsrc(a.x[k + u], tb);
#pragma unroll
      for (int n = 0; n < N; ++n) raw[n][u] = ld16_buf<NT>(r, n);
    } else {
#pragma unroll
      for (int n = 0; n < N; ++n) raw[n][u] = ld16<NT>(a.x[k + u] + v[n] * E::L);
    }
  }
}

// acc[n][:] = sum over the K clients (in order) for the N 16-byte vectors v[n] (output
// indices; vin[n]: where those vectors sit in the client buckets, == v[n] in the row layout).
// PIPE: the loads of client group g+1 are issued before the adds of group g (two register
// buffers), so a wave keeps 2*U*N loads in flight across the add chain.
template <typename E, int KC, bool NT, int N, int U, bool PIPE, bool BUF = false>
__device__ __forceinline__ void fedavg_vectors(const FaArgs<E, KC>& a, const int K, const int first,
                                               const uint64_t* v, const uint64_t* vin, typename E::P (*acc)[E::L],
                                               const typename E::Out* out, const uint64_t tb = 0) {
#pragma clang fp contract(off)
  using P = typename E::P;
  constexpr int L = E::L;
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if (first) {
#pragma unroll
      for (int j = 0; j < L; ++j) acc[n][j] = P(0.0f);  // NumPy seeds add.reduce with +0.0
    } else {
      load_vec<E>(out, v[n], acc[n]);
    }
  }
  int k = 0;
  if constexpr (PIPE) {
    if (K >= U) {
      u32x4 ra[N][U], rb[N][U];
      fedavg_load_group<E, KC, NT, N, U>(a, 0, vin, ra);
      for (;;) {
        const bool mb = k + 2 * U <= K;
        if (mb) fedavg_load_group<E, KC, NT, N, U>(a, k + U, vin, rb);
        fedavg_accumulate<E, N, U>(ra, a.w + k, acc);
        k += U;
        if (!mb) break;
        const bool ma = k + 2 * U <= K;
        if (ma) fedavg_load_group<E, KC, NT, N, U>(a, k + U, vin, ra);
        fedavg_accumulate<E, N, U>(rb, a.w + k, acc);
        k += U;
        if (!ma) break;
      }
    }
  } else {
    for (; k + U <= K; k += U) {
      u32x4 raw[N][U];
      fedavg_load_group<E, KC, NT, N, U, BUF>(a, k, vin, raw, tb);
      fedavg_accumulate<E, N, U>(raw, a.w + k, acc);
    }
  }
  for (; k < K; ++k) {
    const P w = a.w[k];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      P xs[L];
      if constexpr (BUF) E::unpack(ld16_buf<NT>(tile_rsrc(a.x[k], tb), n), xs);
      else E::unpack(ld16<NT>(a.x[k] + vin[n] * L), xs);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const P p = xs[j] * w;
        acc[n][j] = acc[n][j] + p;
      }
    }
  }
}

// numel==1 patch for the N vectors v[] of this thread: one call site of the pairwise tree
// (the owner vector is found first) keeps the unrolled kernel body small.
template <typename E, int KC, int N, int TV = 0>
__device__ __forceinline__ void patch_pairwise(const FaArgs<E, KC>& a, const PwArgs& pw, const int K,
                                               const uint64_t* v, typename E::P (*acc)[E::L],
                                               const uint64_t pitch = 0) {
  constexpr int L = E::L;
  for (int p = 0; p < pw.n; ++p) {
    const uint64_t e = pw.idx[p];
    int owner = -1;
#pragma unroll
    for (int n = 0; n < N; ++n)
      if (e / L == v[n]) owner = n;
    if (owner >= 0) {
      const typename E::P val = fedavg_pairwise_elem<E, KC>(a, K, in_elem<TV, L>(e, pitch));
      const int j = (int)(e % L);
#pragma unroll
      for (int n = 0; n < N; ++n)
#pragma unroll
        for (int jj = 0; jj < L; ++jj)
          if (n == owner && jj == j) acc[n][jj] = val;
    }
  }
}

// Variant knobs (fedagg_tune): NT/NTS non-temporal loads/stores; VPT vectors per thread per
// step; U clients per load group; PIPE software-pipelined client groups; TILE: a workgroup owns
// VPT*256 CONTIGUOUS vectors per step (a wave reads VPT KiB contiguous per client) instead of
// VPT grid-strided vectors.
// OCC (fedagg_tune "fa_occ"): minimum waves per SIMD the register allocation must allow
// (amdgpu_waves_per_eu; 1 = no constraint beyond the launch bound).
// BLK (fedagg_tune "fa_blk"): threads per workgroup of the global-load tiles; 512 gives a
// workgroup step the footprint of the 256-thread tile with twice the vectors per thread, at half
// the registers per thread.
// TV (fedagg_fedavg_tiled_*): the client buckets are tile-interleaved with tiles of TV = VPT*BLK
// vectors and `pitch` = K * TV (in_vec above); 0: the [K, ld] row layout.
template <typename E, int KC, bool NT, int NTS, int VPT, int U, bool PIPE, bool TILE, int OCC = 1, bool BUF = false,
          int BLK = FA_BLOCK, int TV = 0>
__global__ void __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(OCC)))
    fedavg_kernel(const FaArgs<E, KC> a, const PwArgs pw, const int K, const int first, const uint64_t nvec,
                  const uint64_t M, typename E::Out* __restrict__ out, const int remap, const int tpb,
                  const uint64_t pitch, const int rel, const typename E::Out* in) {
#pragma clang fp contract(off)
  using P = typename E::P;
  constexpr int L = E::L;
  // first == 0: where the running accumulator is read -- a separate input only in the push runs'
  // instantiations (NTS 3), so every other kernel compiles exactly as before
  const typename E::Out* acc_src = (NTS == 3 && in) ? in : out;
  static_assert(!BUF || BLK == FA_BLOCK, "buffer-descriptor tiles assume 256-thread workgroups");
  static_assert(TV == 0 || (TILE && !PIPE && TV == VPT * BLK), "tile-interleaved buckets: one tile per workgroup step");
  const uint64_t stride = (uint64_t)gridDim.x * BLK;
  const uint64_t gid = (uint64_t)blockIdx.x * BLK + threadIdx.x;

  if constexpr (TILE) {
    constexpr bool WIDE = E::L * sizeof(typename E::Out) == 32;
    __shared__ u32x4 stage[WIDE ? BLK / 64 : 1][128];
    u32x4* lds_wave = stage[WIDE ? threadIdx.x / 64 : 0];
    const uint64_t tile = (uint64_t)VPT * BLK;
    uint64_t t;
    for (uint64_t it = 0; block_tile(remap, tpb, it, &t) && t * tile < nvec; ++it) {
      const uint64_t base = t * tile + threadIdx.x;
      // wave-uniform: every lane of this wave has all VPT vectors in range
      const bool wave_full = (base - (threadIdx.x & 63)) + 63 + (VPT - 1) * BLK < nvec;
      if (base + (VPT - 1) * BLK < nvec) {
        uint64_t v[VPT], vin[VPT];
#pragma unroll
        for (int n = 0; n < VPT; ++n) {
          v[n] = base + n * BLK;
          vin[n] = TV ? t * pitch + n * BLK + threadIdx.x : v[n];
        }
        P acc[VPT][L];
        fedavg_vectors<E, KC, NT, VPT, U, PIPE, BUF>(a, K, first, v, vin, acc, acc_src, (TV ? t * pitch : t * tile) * 16);
        if (pw.n) patch_pairwise<E, KC, VPT, TV>(a, pw, K, v, acc, pitch);
#pragma unroll
        for (int n = 0; n < VPT; ++n) store_vec_wave<E, NTS>(out, v[n], acc[n], wave_full, lds_wave);
      } else {
        for (uint64_t v0 = base; v0 < nvec; v0 += BLK) {
          P acc[1][L];
          const uint64_t vi0 = in_vec<TV>(v0, pitch);
          fedavg_vectors<E, KC, NT, 1, U, PIPE>(a, K, first, &v0, &vi0, acc, acc_src);
          if (pw.n) patch_pairwise<E, KC, 1, TV>(a, pw, K, &v0, acc, pitch);
          store_vec<E, NTS>(out, v0, acc[0]);
        }
      }
    }
  } else {
    uint64_t v0 = gid;
    if constexpr (VPT > 1) {
      for (; v0 + (VPT - 1) * stride < nvec; v0 += VPT * stride) {
        uint64_t v[VPT];
#pragma unroll
        for (int n = 0; n < VPT; ++n) v[n] = v0 + n * stride;
        P acc[VPT][L];
        fedavg_vectors<E, KC, NT, VPT, U, PIPE>(a, K, first, v, v, acc, acc_src);
        if (pw.n) patch_pairwise<E, KC, VPT>(a, pw, K, v, acc);
#pragma unroll
        for (int n = 0; n < VPT; ++n) store_vec<E, NTS>(out, v[n], acc[n]);
      }
    }
    for (; v0 < nvec; v0 += stride) {
      P acc[1][L];
      fedavg_vectors<E, KC, NT, 1, U, PIPE>(a, K, first, &v0, &v0, acc, acc_src);
      if (pw.n) patch_pairwise<E, KC, 1>(a, pw, K, &v0, acc);
      store_vec<E, NTS>(out, v0, acc[0]);
    }
  }

  // Scalar remainder (M % L elements, or everything when a pointer is not 16-B aligned).
  for (uint64_t i = nvec * L + gid; i < M; i += stride) {
    P acc = first ? P(0.0f) : E::in_out(acc_src[i]);
    const uint64_t ii = in_elem<TV, L>(i, pitch);
    for (int k = 0; k < K; ++k) {
      const P p = E::cvt(a.x[k][ii]) * a.w[k];
      acc = acc + p;
    }
    for (int p = 0; p < pw.n; ++p)
      if (pw.idx[p] == i) acc = fedavg_pairwise_elem<E, KC>(a, K, ii);
    if constexpr (NTS == 3 && std::is_same<typename E::Out, float>::value)  // push runs: system scope too
      __hip_atomic_store(out + i, E::out(acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      out[i] = E::out(acc);
  }
  if (rel) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // push runs: this wave's sc0 sc1 stores acknowledged
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

// Fused numel==1 patch for Scaffold: delta = lr*(0 + pw_K(w*d)), c' = 0 + pw_{K+1}(w*cv, c)
template <typename TIn, int KC>
__device__ __forceinline__ void scaffold_pairwise_elem(const ScArgs<TIn, KC>& a, int K, const TIn* c, double lr,
                                                    uint64_t e, double* dval, double* cval) {
#pragma clang fp contract(off)
  auto gd = [&](int64_t k) -> double { return a.w[k] * (double)a.d[k][e]; };
  auto gc = [&](int64_t k) -> double { return k < K ? a.w[k] * (double)a.cv[k][e] : (double)c[e]; };
  const double sd = 0.0 + pw_leaf<double>(gd, 0, K);
  *dval = lr * sd;
  *cval = 0.0 + pw_leaf<double>(gc, 0, K + 1);
}

// Loads of one group of SU clients, both buckets, for the N vectors v[].
template <typename TIn, int KC, bool NT, int N, int SU, bool BUF = false>
__device__ __forceinline__ void scaffold_load_group(const ScArgs<TIn, KC>& a, const int k, const uint64_t* v,
                                                    u32x4 (&rd)[N][SU], u32x4 (&rc)[N][SU], uint64_t tb = 0) {
  constexpr int L = 16 / sizeof(TIn);
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    if constexpr (BUF) {  // buffer descriptors based at the tile (see fedavg_load_group)
      const __amdgpu_buffer_rsrc_t r_d = tile_rsrc(a.d[k + u], tb), r_c = tile_rsrc(a.cv[k + u], tb);
#pragma unroll
      for (int n = 0; n < N; ++n) {
        rd[n][u] = ld16_buf<NT>(r_d, n);
        rc[n][u] = ld16_buf<NT>(r_c, n);
      }
    } else {
#pragma unroll
      for (int n = 0; n < N; ++n) {
        rd[n][u] = ld16<NT>(a.d[k + u] + v[n] * L);
        rc[n][u] = ld16<NT>(a.cv[k + u] + v[n] * L);
      }
    }
  }
}

// fp64 products and in-order adds of one loaded group (scaffold.py:262,293: w_k * x_k summed in
// list order).
template <typename TIn, int N, int SU>
__device__ __forceinline__ void scaffold_accumulate(const u32x4 (&rd)[N][SU], const u32x4 (&rc)[N][SU],
                                                    const double* w, double (*ad)[16 / sizeof(TIn)],
                                                    double (*ac)[16 / sizeof(TIn)]) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const double wu = w[u];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      double xd[L], xc[L];
      unpack_d<TIn>(rd[n][u], xd);
      unpack_d<TIn>(rc[n][u], xc);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const double pd = wu * xd[j];
        const double pc = wu * xc[j];
        ad[n][j] = ad[n][j] + pd;
        ac[n][j] = ac[n][j] + pc;
      }
    }
  }
}

// N 16-byte vectors of both buckets: in-order fp64 sums over the K clients, then (last chunk)
// + c and * lr, the fused numel==1 patch, and the fp64 stores.  PIPE: software-pipelined groups.
// CPF: the server c vectors of the last chunk are loaded together with the last client group's
// loads instead of after the client walk (one dependent HBM round trip less per tile).
template <typename TIn, int KC, bool NT, int NTS, int N, int SU, bool PIPE = false, bool BUF = false,
          bool CPF = false>
__device__ __forceinline__ void scaffold_vectors(const ScArgs<TIn, KC>& a, const PwArgs& pw, const int K,
                                                 const int first, const int last, const TIn* __restrict__ c,
                                                 const double lr, const uint64_t* v, double* __restrict__ dout,
                                                 double* __restrict__ cout, bool wave_full, u32x4* lds_wave,
                                                 const uint64_t tb = 0) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  double ad[N][L], ac[N][L];
#pragma unroll
  for (int n = 0; n < N; ++n) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      ad[n][j] = first ? 0.0 : dout[v[n] * L + j];
      ac[n][j] = first ? 0.0 : cout[v[n] * L + j];
    }
  }
  int k = 0;
  u32x4 craw[CPF ? N : 1];
  bool pre_c = false;
  if constexpr (PIPE) {
    // the next group's loads are issued before this group's fp64 products and adds
    if (K >= SU) {
      u32x4 da[N][SU], ca[N][SU], db[N][SU], cb[N][SU];
      scaffold_load_group<TIn, KC, NT, N, SU>(a, 0, v, da, ca);
      for (;;) {
        const bool mb = k + 2 * SU <= K;
        if (mb) scaffold_load_group<TIn, KC, NT, N, SU>(a, k + SU, v, db, cb);
        scaffold_accumulate<TIn, N, SU>(da, ca, a.w + k, ad, ac);
        k += SU;
        if (!mb) break;
        const bool ma = k + 2 * SU <= K;
        if (ma) scaffold_load_group<TIn, KC, NT, N, SU>(a, k + SU, v, da, ca);
        scaffold_accumulate<TIn, N, SU>(db, cb, a.w + k, ad, ac);
        k += SU;
        if (!ma) break;
      }
    }
  } else {
    for (; k + SU <= K; k += SU) {
      u32x4 rd[N][SU], rc[N][SU];
      if constexpr (CPF) {
        if (last && k + SU == K && !pre_c) {
#pragma unroll
          for (int n = 0; n < N; ++n) craw[n] = ld16<NT>(c + v[n] * L);
          pre_c = true;
        }
      }
      scaffold_load_group<TIn, KC, NT, N, SU, BUF>(a, k, v, rd, rc, tb);
      scaffold_accumulate<TIn, N, SU>(rd, rc, a.w + k, ad, ac);
    }
  }
  for (; k < K; ++k) {
    const double w = a.w[k];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      double xd[L], xc[L];
      if constexpr (BUF) {
        unpack_d<TIn>(ld16_buf<NT>(tile_rsrc(a.d[k], tb), n), xd);
        unpack_d<TIn>(ld16_buf<NT>(tile_rsrc(a.cv[k], tb), n), xc);
      } else {
        unpack_d<TIn>(ld16<NT>(a.d[k] + v[n] * L), xd);
        unpack_d<TIn>(ld16<NT>(a.cv[k] + v[n] * L), xc);
      }
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const double pd = w * xd[j];
        const double pc = w * xc[j];
        ad[n][j] = ad[n][j] + pd;
        ac[n][j] = ac[n][j] + pc;
      }
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if (last) {
      double xcc[L];
      if constexpr (CPF) unpack_d<TIn>(pre_c ? craw[n] : ld16<NT>(c + v[n] * L), xcc);
      else unpack_d<TIn>(ld16<NT>(c + v[n] * L), xcc);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        ac[n][j] = ac[n][j] + xcc[j];  // server c appended LAST (scaffold.py:262-263)
        ad[n][j] = lr * ad[n][j];      // aggregation_lr * sum (scaffold.py:293)
      }
    }
  }
  for (int p = 0; p < pw.n; ++p) {  // numel==1 patch (fused launches are single-chunk: first & last)
    const uint64_t e = pw.idx[p];
    int owner = -1;
#pragma unroll
    for (int n = 0; n < N; ++n)
      if (e / L == v[n]) owner = n;
    if (owner >= 0) {
      double dv, cvv;
      scaffold_pairwise_elem<TIn, KC>(a, K, c, lr, e, &dv, &cvv);
      const int j = (int)(e % L);
#pragma unroll
      for (int n = 0; n < N; ++n)
#pragma unroll
        for (int jj = 0; jj < L; ++jj)
          if (n == owner && jj == j) {
            ad[n][jj] = dv;
            ac[n][jj] = cvv;
          }
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if constexpr (L == 4) {
      if (wave_full) {  // fp32 in -> 32 B of fp64 out per lane: coalesce through LDS
        const uint64_t v0 = v[n] - (threadIdx.x & 63);
        const f64x2 d0 = {ad[n][0], ad[n][1]}, d1 = {ad[n][2], ad[n][3]};
        const f64x2 c0 = {ac[n][0], ac[n][1]}, c1 = {ac[n][2], ac[n][3]};
        store32_coalesced<NTS>(dout + v0 * L, __builtin_bit_cast(u32x4, d0), __builtin_bit_cast(u32x4, d1), lds_wave);
        store32_coalesced<NTS>(cout + v0 * L, __builtin_bit_cast(u32x4, c0), __builtin_bit_cast(u32x4, c1), lds_wave);
        continue;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < L / 2; ++s2) {
      f64x2 t0 = {ad[n][2 * s2], ad[n][2 * s2 + 1]};
      f64x2 t1 = {ac[n][2 * s2], ac[n][2 * s2 + 1]};
      st16<NTS>(reinterpret_cast<f64x2*>(dout + v[n] * L) + s2, __builtin_bit_cast(u32x4, t0));
      st16<NTS>(reinterpret_cast<f64x2*>(cout + v[n] * L) + s2, __builtin_bit_cast(u32x4, t1));
    }
  }
}

// Phase-split variant (fedagg_tune "sc_split"): the same per-element arithmetic, but the
// thread streams all K delta vectors first (and stores the delta result), then all K control
// variate vectors: half the concurrent streams and half the live accumulators of the fused
// walk, so a wave can own twice the contiguous bytes per stream.
template <typename TIn, int KC, bool NT, int N, int SU, int PH>
__device__ __forceinline__ void scaffold_phase_load(const ScArgs<TIn, KC>& a, const int k, const uint64_t* v,
                                                    u32x4 (&r)[N][SU]) {
  constexpr int L = 16 / sizeof(TIn);
#pragma unroll
  for (int u = 0; u < SU; ++u)
#pragma unroll
    for (int n = 0; n < N; ++n) {
      if constexpr (PH == 0) r[n][u] = ld16<NT>(a.d[k + u] + v[n] * L);
      else r[n][u] = ld16<NT>(a.cv[k + u] + v[n] * L);
    }
}

template <typename TIn, int KC, int N, int SU>
__device__ __forceinline__ void scaffold_phase_add(const ScArgs<TIn, KC>& a, const int k, const u32x4 (&r)[N][SU],
                                                   double (&acc)[N][16 / sizeof(TIn)]) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const double w = a.w[k + u];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      double x[L];
      unpack_d<TIn>(r[n][u], x);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const double p = w * x[j];
        acc[n][j] = acc[n][j] + p;
      }
    }
  }
}

// PIPE: the next client group's loads are issued before this group's fp64 products and adds.
// SEPIN (push runs only, scaffold_push_kernel): the running accumulator is read from `in`
// instead of `out`; every other instantiation compiles exactly as before.
template <typename TIn, int KC, bool NT, int NTS, int N, int SU, int PH, bool PIPE = false, bool SEPIN = false>
__device__ __forceinline__ void scaffold_phase(const ScArgs<TIn, KC>& a, const PwArgs& pw, const int K,
                                               const int first, const int last, const TIn* __restrict__ c,
                                               const double lr, const uint64_t* v, double* __restrict__ out,
                                               bool wave_full, u32x4* lds_wave, const double* in = nullptr) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  double acc[N][L];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int j = 0; j < L; ++j) {
      if constexpr (SEPIN)
        acc[n][j] = first ? 0.0 : in[v[n] * L + j];
      else
        acc[n][j] = first ? 0.0 : out[v[n] * L + j];
    }
  int k = 0;
  if constexpr (PIPE) {
    if (K >= SU) {
      u32x4 ra[N][SU], rb[N][SU];
      scaffold_phase_load<TIn, KC, NT, N, SU, PH>(a, 0, v, ra);
      for (;;) {
        const bool mb = k + 2 * SU <= K;
        if (mb) scaffold_phase_load<TIn, KC, NT, N, SU, PH>(a, k + SU, v, rb);
        scaffold_phase_add<TIn, KC, N, SU>(a, k, ra, acc);
        k += SU;
        if (!mb) break;
        const bool ma = k + 2 * SU <= K;
        if (ma) scaffold_phase_load<TIn, KC, NT, N, SU, PH>(a, k + SU, v, ra);
        scaffold_phase_add<TIn, KC, N, SU>(a, k, rb, acc);
        k += SU;
        if (!ma) break;
      }
    }
  } else {
    for (; k + SU <= K; k += SU) {
      u32x4 r[N][SU];
      scaffold_phase_load<TIn, KC, NT, N, SU, PH>(a, k, v, r);
      scaffold_phase_add<TIn, KC, N, SU>(a, k, r, acc);
    }
  }
  for (; k < K; ++k) {
    const double w = a.w[k];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      double x[L];
      if constexpr (PH == 0) unpack_d<TIn>(ld16<NT>(a.d[k] + v[n] * L), x);
      else unpack_d<TIn>(ld16<NT>(a.cv[k] + v[n] * L), x);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const double p = w * x[j];
        acc[n][j] = acc[n][j] + p;
      }
    }
  }
  if (last) {
#pragma unroll
    for (int n = 0; n < N; ++n) {
      if constexpr (PH == 0) {
#pragma unroll
        for (int j = 0; j < L; ++j) acc[n][j] = lr * acc[n][j];  // scaffold.py:293
      } else {
        double xc[L];
        unpack_d<TIn>(ld16<NT>(c + v[n] * L), xc);
#pragma unroll
        for (int j = 0; j < L; ++j) acc[n][j] = acc[n][j] + xc[j];  // c last (scaffold.py:262-263)
      }
    }
  }
  for (int p = 0; p < pw.n; ++p) {
    const uint64_t e = pw.idx[p];
    int owner = -1;
#pragma unroll
    for (int n = 0; n < N; ++n)
      if (e / L == v[n]) owner = n;
    if (owner >= 0) {
      double dv, cvv;
      scaffold_pairwise_elem<TIn, KC>(a, K, c, lr, e, &dv, &cvv);
      const int j = (int)(e % L);
#pragma unroll
      for (int n = 0; n < N; ++n)
#pragma unroll
        for (int jj = 0; jj < L; ++jj)
          if (n == owner && jj == j) acc[n][jj] = PH == 0 ? dv : cvv;
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if constexpr (L == 4) {
      if (wave_full) {
        const uint64_t v0 = v[n] - (threadIdx.x & 63);
        const f64x2 t0 = {acc[n][0], acc[n][1]}, t1 = {acc[n][2], acc[n][3]};
        store32_coalesced<NTS>(out + v0 * L, __builtin_bit_cast(u32x4, t0), __builtin_bit_cast(u32x4, t1), lds_wave);
        continue;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < L / 2; ++s2) {
      f64x2 t = {acc[n][2 * s2], acc[n][2 * s2 + 1]};
      st16<NTS>(reinterpret_cast<f64x2*>(out + v[n] * L) + s2, __builtin_bit_cast(u32x4, t));
    }
  }
}

template <typename TIn, int KC, bool NT, int NTS, int N, int SU>
__device__ __forceinline__ void scaffold_vectors_split(const ScArgs<TIn, KC>& a, const PwArgs& pw, const int K,
                                                       const int first, const int last, const TIn* __restrict__ c,
                                                       const double lr, const uint64_t* v, double* __restrict__ dout,
                                                       double* __restrict__ cout, bool wave_full, u32x4* lds_wave) {
  scaffold_phase<TIn, KC, NT, NTS, N, SU, 0>(a, pw, K, first, last, c, lr, v, dout, wave_full, lds_wave);
  scaffold_phase<TIn, KC, NT, NTS, N, SU, 1>(a, pw, K, first, last, c, lr, v, cout, wave_full, lds_wave);
}

// Same tiling as fedavg_kernel: a workgroup step covers VPT*BLK contiguous vectors.
// OCC (fedagg_tune "sc_occ"): minimum waves per SIMD for the register allocation; BLK
// ("sc_blk"): threads per workgroup (256, or 512: 32 KiB per stream per workgroup step at VPT 4);
// CPF ("sc_cpf"): c loaded with the last client group.
template <typename TIn, int KC, bool NT, int NTS, int VPT, int SU, bool SPLIT, bool PIPE = false, bool BUF = false,
          bool CPF = false, int OCC = 1, int BLK = FA_BLOCK>
__global__ void __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(OCC)))
    scaffold_kernel(const ScArgs<TIn, KC> a, const PwArgs pw, const int K, const int first, const int last,
                    const TIn* __restrict__ c, const double lr, const uint64_t nvec, const uint64_t M,
                    double* __restrict__ dout, double* __restrict__ cout, const int remap, const int tpb) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  static_assert(!BUF || BLK == FA_BLOCK, "buffer-descriptor tiles assume 256-thread workgroups");
  const uint64_t stride = (uint64_t)gridDim.x * BLK;
  const uint64_t gid = (uint64_t)blockIdx.x * BLK + threadIdx.x;
  __shared__ u32x4 stage[BLK / 64][128];
  u32x4* lds_wave = stage[threadIdx.x / 64];
  const uint64_t tile = (uint64_t)VPT * BLK;
  uint64_t t;
  for (uint64_t it = 0; block_tile(remap, tpb, it, &t) && t * tile < nvec; ++it) {
    const uint64_t base = t * tile + threadIdx.x;
    const bool wave_full = (base - (threadIdx.x & 63)) + 63 + (VPT - 1) * BLK < nvec;
    if (base + (VPT - 1) * BLK < nvec) {
      uint64_t v[VPT];
#pragma unroll
      for (int n = 0; n < VPT; ++n) v[n] = base + n * BLK;
      if constexpr (SPLIT)
        scaffold_vectors_split<TIn, KC, NT, NTS, VPT, SU>(a, pw, K, first, last, c, lr, v, dout, cout, wave_full,
                                                           lds_wave);
      else
        scaffold_vectors<TIn, KC, NT, NTS, VPT, SU, PIPE, BUF, CPF>(a, pw, K, first, last, c, lr, v, dout, cout,
                                                                     wave_full, lds_wave, t * tile * 16);
    } else {
      for (uint64_t v0 = base; v0 < nvec; v0 += BLK)
        scaffold_vectors<TIn, KC, NT, NTS, 1, SU>(a, pw, K, first, last, c, lr, &v0, dout, cout, false, lds_wave);
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
    for (int p = 0; p < pw.n; ++p)
      if (pw.idx[p] == i) scaffold_pairwise_elem<TIn, KC>(a, K, c, lr, i, &ad, &ac);
    dout[i] = ad;
    cout[i] = ac;
  }
}

// Bucket-split variant (fedagg_tune "sc_bsplit"): workgroup pairs (2t, 2t+1) own the same tile,
// the even one streams the K delta rows, the odd one the K control-variate rows (+ c).  A thread
// then holds one bucket's loads and accumulators (half the registers of the fused walk), so the
// launch can give a wave 8 KiB per stream like the FedAvg kernel, while both buckets stay in
// flight chip-wide at once (unlike sc_split, which walks them one after the other per thread).
// Same per-element arithmetic and order as scaffold_kernel.  Vector path only (16-B aligned
// operands, nvec = M / L); the grid is even.
template <typename TIn, int KC, bool NT, int NTS, int VPT, int SU>
__global__ void __launch_bounds__(FA_BLOCK)
    scaffold_bsplit_kernel(const ScArgs<TIn, KC> a, const PwArgs pw, const int K, const int first, const int last,
                           const TIn* __restrict__ c, const double lr, const uint64_t nvec, const uint64_t M,
                           double* __restrict__ dout, double* __restrict__ cout) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  __shared__ u32x4 stage[FA_BLOCK / 64][128];
  u32x4* lds_wave = stage[threadIdx.x / 64];
  const int ph = blockIdx.x & 1;
  const uint64_t pairs = gridDim.x / 2, pb = blockIdx.x >> 1;
  const uint64_t tile = (uint64_t)VPT * FA_BLOCK;
  for (uint64_t t = pb; t * tile < nvec; t += pairs) {
    const uint64_t base = t * tile + threadIdx.x;
    const bool wave_full = (base - (threadIdx.x & 63)) + 63 + (VPT - 1) * FA_BLOCK < nvec;
    if (base + (VPT - 1) * FA_BLOCK < nvec) {
      uint64_t v[VPT];
#pragma unroll
      for (int n = 0; n < VPT; ++n) v[n] = base + n * FA_BLOCK;
      if (ph == 0)
        scaffold_phase<TIn, KC, NT, NTS, VPT, SU, 0>(a, pw, K, first, last, c, lr, v, dout, wave_full, lds_wave);
      else
        scaffold_phase<TIn, KC, NT, NTS, VPT, SU, 1>(a, pw, K, first, last, c, lr, v, cout, wave_full, lds_wave);
    } else {
      for (uint64_t v0 = base; v0 < nvec; v0 += FA_BLOCK) {
        if (ph == 0)
          scaffold_phase<TIn, KC, NT, NTS, 1, SU, 0>(a, pw, K, first, last, c, lr, &v0, dout, false, lds_wave);
        else
          scaffold_phase<TIn, KC, NT, NTS, 1, SU, 1>(a, pw, K, first, last, c, lr, &v0, cout, false, lds_wave);
      }
    }
  }
  // scalar remainder (M % L elements): the even workgroups, both buckets
  if (ph) return;
  for (uint64_t i = nvec * L + pb * FA_BLOCK + threadIdx.x; i < M; i += pairs * FA_BLOCK) {
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
    for (int p = 0; p < pw.n; ++p)
      if (pw.idx[p] == i) scaffold_pairwise_elem<TIn, KC>(a, K, c, lr, i, &ad, &ac);
    dout[i] = ad;
    cout[i] = ac;
  }
}

// One-bucket launches (fedagg_tune "sc_2l"): the grid walks ONE of the two buckets at a time --
// phase 0: the K delta rows into dout (lr applied after the sum), phase 1: the K control-variate
// rows plus c into cout.  The two sums are independent, so the bytes and the per-element
// arithmetic are those of scaffold_kernel; what changes is that only K (or K + 1) client streams
// are in flight at a time instead of 2K + 1.  PH 0 / 1: one launch per phase (the host launches
// 0 then 1); PH 2: one launch whose first half of workgroups runs phase 0 and second half phase
// 1 (the dispatcher starts workgroups in index order, so the phases overlap only at the seam).
template <typename TIn, int KC, bool NT, int NTS, int VPT, int SU, int P, bool PIPE>
__device__ __forceinline__ void scaffold_bucket_walk(const ScArgs<TIn, KC>& a, const PwArgs& pw, const int K,
                                                     const int first, const int last, const TIn* __restrict__ c,
                                                     const double lr, const uint64_t nvec, const uint64_t M,
                                                     double* __restrict__ out, const uint64_t lb,
                                                     const uint64_t nblk, u32x4* lds_wave) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  const uint64_t tile = (uint64_t)VPT * FA_BLOCK;
  for (uint64_t t = lb; t * tile < nvec; t += nblk) {
    const uint64_t base = t * tile + threadIdx.x;
    const bool wave_full = (base - (threadIdx.x & 63)) + 63 + (VPT - 1) * FA_BLOCK < nvec;
    if (base + (VPT - 1) * FA_BLOCK < nvec) {
      uint64_t v[VPT];
#pragma unroll
      for (int n = 0; n < VPT; ++n) v[n] = base + n * FA_BLOCK;
      scaffold_phase<TIn, KC, NT, NTS, VPT, SU, P, PIPE>(a, pw, K, first, last, c, lr, v, out, wave_full, lds_wave);
    } else {
      for (uint64_t v0 = base; v0 < nvec; v0 += FA_BLOCK)
        scaffold_phase<TIn, KC, NT, NTS, 1, SU, P>(a, pw, K, first, last, c, lr, &v0, out, false, lds_wave);
    }
  }
  for (uint64_t i = nvec * L + lb * FA_BLOCK + threadIdx.x; i < M; i += nblk * FA_BLOCK) {  // scalar remainder
    double acc = first ? 0.0 : out[i];
    for (int k = 0; k < K; ++k) {
      const double p = a.w[k] * (double)(P == 0 ? a.d[k][i] : a.cv[k][i]);
      acc = acc + p;
    }
    if (last) acc = P == 0 ? lr * acc : acc + (double)c[i];
    for (int p = 0; p < pw.n; ++p)
      if (pw.idx[p] == i) {
        double dv, cvv;
        scaffold_pairwise_elem<TIn, KC>(a, K, c, lr, i, &dv, &cvv);
        acc = P == 0 ? dv : cvv;
      }
    out[i] = acc;
  }
}

template <typename TIn, int KC, bool NT, int NTS, int VPT, int SU, int PH, bool PIPE = false>
__global__ void __launch_bounds__(FA_BLOCK)
    scaffold_bucket_kernel(const ScArgs<TIn, KC> a, const PwArgs pw, const int K, const int first, const int last,
                           const TIn* __restrict__ c, const double lr, const uint64_t nvec, const uint64_t M,
                           double* __restrict__ dout, double* __restrict__ cout) {
  __shared__ u32x4 stage[FA_BLOCK / 64][128];
  u32x4* lds_wave = stage[threadIdx.x / 64];
  if constexpr (PH == 2) {
    const uint64_t half = gridDim.x / 2;
    if (blockIdx.x < half)
      scaffold_bucket_walk<TIn, KC, NT, NTS, VPT, SU, 0, PIPE>(a, pw, K, first, last, c, lr, nvec, M, dout, blockIdx.x,
                                                          half, lds_wave);
    else
      scaffold_bucket_walk<TIn, KC, NT, NTS, VPT, SU, 1, PIPE>(a, pw, K, first, last, c, lr, nvec, M, cout,
                                                          blockIdx.x - half, half, lds_wave);
  } else {
    scaffold_bucket_walk<TIn, KC, NT, NTS, VPT, SU, PH, PIPE>(a, pw, K, first, last, c, lr, nvec, M, PH == 0 ? dout : cout,
                                                         blockIdx.x, gridDim.x, lds_wave);
  }
}

// Push runs of the client-sharded Scaffold schedules (fedagg_scaffold_chain_push_*): ONE bucket
// of a client block -- PH 0 the delta rows (x lr at the finish), PH 1 the control-variate rows
// (+ c at the finish) -- continuing the fp64 accumulator `in` (this rank's slot, or the output
// itself for a later client chunk; first: from +0.0) into `out`, a peer's mapped slot or the
// root's output, with system-scope write-through stores (st16<3>); every wave waits for their
// acknowledgements before it retires.  Per-element arithmetic and order: scaffold_bucket_walk's
// (scaffold.py:262-263, 293).  SEP: the accumulator is read from `in` (a chain's first client
// chunk continuing a slot); otherwise from `out` (later chunks; `in` unused).
template <typename TIn, int VPT, int SU, int PH, bool PIPE, bool SEP>
__global__ void __launch_bounds__(FA_BLOCK)
    scaffold_push_kernel(const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD> a, const int K, const int first, const int last,
                         const TIn* __restrict__ c, const double lr, const uint64_t nvec, const uint64_t M,
                         const double* __restrict__ in, double* __restrict__ out) {
#pragma clang fp contract(off)
  constexpr int L = 16 / sizeof(TIn);
  __shared__ u32x4 stage[FA_BLOCK / 64][128];
  u32x4* lds_wave = stage[threadIdx.x / 64];
  PwArgs pw;  // chain runs carry no numel == 1 patch (the schedule's products / finish do)
  pw.n = 0;
  const uint64_t tile = (uint64_t)VPT * FA_BLOCK;
  for (uint64_t t = blockIdx.x; t * tile < nvec; t += gridDim.x) {
    const uint64_t base = t * tile + threadIdx.x;
    const bool wave_full = (base - (threadIdx.x & 63)) + 63 + (VPT - 1) * FA_BLOCK < nvec;
    if (base + (VPT - 1) * FA_BLOCK < nvec) {
      uint64_t v[VPT];
#pragma unroll
      for (int n = 0; n < VPT; ++n) v[n] = base + n * FA_BLOCK;
      scaffold_phase<TIn, FEDAGG_KCHUNK_SCAFFOLD, true, 3, VPT, SU, PH, PIPE, SEP>(a, pw, K, first, last, c, lr, v, out,
                                                                                  wave_full, lds_wave, in);
    } else {
      for (uint64_t v0 = base; v0 < nvec; v0 += FA_BLOCK)
        scaffold_phase<TIn, FEDAGG_KCHUNK_SCAFFOLD, true, 3, 1, SU, PH, false, SEP>(a, pw, K, first, last, c, lr, &v0,
                                                                                  out, false, lds_wave, in);
    }
  }
  for (uint64_t i = nvec * L + (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; i < M;
       i += (uint64_t)gridDim.x * FA_BLOCK) {  // scalar remainder
    double acc = first ? 0.0 : (SEP ? in[i] : out[i]);
    for (int k = 0; k < K; ++k) {
      const double p = a.w[k] * (double)(PH == 0 ? a.d[k][i] : a.cv[k][i]);
      acc = acc + p;
    }
    if (last) acc = PH == 0 ? lr * acc : acc + (double)c[i];
    __hip_atomic_store(out + i, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc0 sc1 stores acknowledged
}

// ------------------------------------------------------------------------------------
// Separate numel==1 path (K > one chunk, or more indices than fit the kernel arguments)
// ------------------------------------------------------------------------------------
struct IdxArgs {
  uint64_t idx[FEDAGG_MAX_PAIRWISE];
};

// Stage 1: ws[p * stride + kbase + k] = fl(x_k[idx_p] * w_k), in the pairwise-sum type W.
template <typename E, int KC>
__global__ void __launch_bounds__(FA_BLOCK)
    pairwise_gather_kernel(const FaArgs<E, KC> a, const int Kc, const int kbase, const IdxArgs ix, const int P,
                           const int64_t stride, typename E::W* __restrict__ ws) {
#pragma clang fp contract(off)
  const int t = blockIdx.x * FA_BLOCK + threadIdx.x;
  if (t >= P * Kc) return;
  const int p = t / Kc, k = t % Kc;
  const typename E::P prod = E::cvt(a.x[k][ix.idx[p]]) * a.w[k];
  ws[p * stride + kbase + k] = (typename E::W)prod;
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

// Stage 2: out[idx_p] = (+0.0 + pairwise(ws[p * stride .. p * stride + n)))
template <typename E>
__global__ void pairwise_tree_kernel(const typename E::W* __restrict__ ws, const int64_t n, const int64_t stride,
                                     const IdxArgs ix, const int P, typename E::Out* __restrict__ out) {
#pragma clang fp contract(off)
  using W = typename E::W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const W* row = ws + p * stride;
  auto get = [&](int64_t i) -> W { return row[i]; };
  const W s = W(0.0f) + pw_sum<W>(get, n);
  out[ix.idx[p]] = E::out((typename E::P)s);
}

template <typename TIn>
__global__ void scaffold_tree_kernel(const double* __restrict__ ws_d, double* __restrict__ ws_c, const TIn* c,
                                     const int64_t K, const IdxArgs ix, const int P, const double lr,
                                     double* __restrict__ dout, double* __restrict__ cout) {
#pragma clang fp contract(off)
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const double* rd = ws_d + p * K;
  double* rc = ws_c + p * (K + 1);
  rc[K] = (double)c[ix.idx[p]];  // server c is the last term (scaffold.py:262)
  auto gd = [&](int64_t i) -> double { return rd[i]; };
  auto gc = [&](int64_t i) -> double { return rc[i]; };
  const double sd = 0.0 + pw_sum<double>(gd, K);
  const double sc = 0.0 + pw_sum<double>(gc, K + 1);
  dout[ix.idx[p]] = lr * sd;
  cout[ix.idx[p]] = sc;
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
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(cnt, bad);
}

// Vectorised form (16-B loads, contiguous tiles of VPT*256 vectors per workgroup step, client
// copies in groups of 4), used when every pointer is 16-B aligned.  Same per-element test.
template <typename T>
__device__ __forceinline__ unsigned eq_mismatches(u32x4 x, u32x4 r) {
  constexpr int L = 16 / sizeof(T);
  T xv[L], rv[L];
  __builtin_memcpy(xv, &x, 16);
  __builtin_memcpy(rv, &r, 16);
  unsigned bad = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) bad += !((xv[j] == rv[j]) || (xv[j] != xv[j] && rv[j] != rv[j]));
  return bad;
}

template <typename T, int KC, int VPT>
__global__ void __launch_bounds__(FA_BLOCK)
    equal_count_vec_kernel(const EqArgs<T, KC> a, const int K, const T* __restrict__ ref, const uint64_t nvec,
                           const uint64_t M, unsigned long long* __restrict__ cnt) {
  constexpr int L = 16 / sizeof(T);
  constexpr int U = 4;
  unsigned long long bad = 0;
  const uint64_t tile = (uint64_t)VPT * FA_BLOCK;
  for (uint64_t base = (uint64_t)blockIdx.x * tile + threadIdx.x; base < nvec; base += (uint64_t)gridDim.x * tile) {
    u32x4 r[VPT];
    bool in[VPT];
#pragma unroll
    for (int n = 0; n < VPT; ++n) {
      in[n] = base + (uint64_t)n * FA_BLOCK < nvec;
      if (in[n]) r[n] = ld16<true>(ref + (base + (uint64_t)n * FA_BLOCK) * L);
    }
    int k = 0;
    for (; k + U <= K; k += U) {
      u32x4 x[VPT][U];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int n = 0; n < VPT; ++n)
          if (in[n]) x[n][u] = ld16<true>(a.x[k + u] + (base + (uint64_t)n * FA_BLOCK) * L);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int n = 0; n < VPT; ++n)
          if (in[n]) bad += eq_mismatches<T>(x[n][u], r[n]);
    }
    for (; k < K; ++k)
#pragma unroll
      for (int n = 0; n < VPT; ++n)
        if (in[n]) bad += eq_mismatches<T>(ld16<true>(a.x[k] + (base + (uint64_t)n * FA_BLOCK) * L), r[n]);
  }
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  for (uint64_t i = nvec * L + (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; i < M; i += stride) {
    const T rr = ref[i];
    for (int k = 0; k < K; ++k) {
      const T v = a.x[k][i];
      bad += !((v == rr) || (v != v && rr != rr));
    }
  }
  for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(cnt, bad);
}

// ------------------------------------------------------------------------------------
// dtype plumbing on the device (exact widening casts; per-client pre-scaling for layers whose
// clients do not share one dtype) -- NumPy semantics: int/bool -> float64 is the C cast
// (round to nearest), float widening is exact, x * w is computed in x's own float type.
// ------------------------------------------------------------------------------------
template <typename TI>
__device__ __forceinline__ double ld_as_double(const void* p, uint64_t i) {
  return (double)static_cast<const TI*>(p)[i];
}

__device__ double load_kind(const void* p, int kind, uint64_t i) {
  switch (kind) {
    case FEDAGG_F16: return (double)static_cast<const _Float16*>(p)[i];
    case FEDAGG_F32: return (double)static_cast<const float*>(p)[i];
    case FEDAGG_F64: return static_cast<const double*>(p)[i];
    case FEDAGG_I8: return ld_as_double<int8_t>(p, i);
    case FEDAGG_I16: return ld_as_double<int16_t>(p, i);
    case FEDAGG_I32: return ld_as_double<int32_t>(p, i);
    case FEDAGG_I64: return ld_as_double<int64_t>(p, i);
    case FEDAGG_U8: return ld_as_double<uint8_t>(p, i);
    case FEDAGG_U16: return ld_as_double<uint16_t>(p, i);
    case FEDAGG_U32: return ld_as_double<uint32_t>(p, i);
    case FEDAGG_U64: return ld_as_double<uint64_t>(p, i);
    case FEDAGG_BOOL: return static_cast<const uint8_t*>(p)[i] ? 1.0 : 0.0;
    default: return 0.0;
  }
}

__global__ void __launch_bounds__(FA_BLOCK)
    cast_kernel(const void* __restrict__ in, int in_kind, void* __restrict__ out, int out_kind, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; i < n; i += stride) {
    if (in_kind == FEDAGG_I64 || in_kind == FEDAGG_U64) {
      // 64-bit integers: convert straight to the output type (one rounding, like NumPy)
      if (out_kind == FEDAGG_F64)
        static_cast<double*>(out)[i] = in_kind == FEDAGG_I64 ? (double)static_cast<const int64_t*>(in)[i]
                                                            : (double)static_cast<const uint64_t*>(in)[i];
      else
        static_cast<float*>(out)[i] = in_kind == FEDAGG_I64 ? (float)static_cast<const int64_t*>(in)[i]
                                                           : (float)static_cast<const uint64_t*>(in)[i];
      continue;
    }
    const double v = load_kind(in, in_kind, i);  // exact for every other supported input
    if (out_kind == FEDAGG_F64)
      static_cast<double*>(out)[i] = v;
    else if (out_kind == FEDAGG_F32)
      static_cast<float*>(out)[i] = (float)v;
    else
      static_cast<_Float16*>(out)[i] = (_Float16)v;
  }
}

__global__ void __launch_bounds__(FA_BLOCK)
    scale_cast_kernel(const void* __restrict__ in, int in_kind, double w, void* __restrict__ out, int out_kind,
                      uint64_t n) {
#pragma clang fp contract(off)
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; i < n; i += stride) {
    double p;
    if (in_kind == FEDAGG_F16)
      p = (double)(static_cast<const _Float16*>(in)[i] * (_Float16)w);
    else if (in_kind == FEDAGG_F32)
      p = (double)(static_cast<const float*>(in)[i] * (float)w);
    else
      p = static_cast<const double*>(in)[i] * w;
    if (out_kind == FEDAGG_F64)
      static_cast<double*>(out)[i] = p;
    else if (out_kind == FEDAGG_F32)
      static_cast<float*>(out)[i] = (float)p;
    else
      static_cast<_Float16*>(out)[i] = (_Float16)p;
  }
}

// ------------------------------------------------------------------------------------
// Client-side flat-bucket ops: the producer / consumer of the
// buckets, i.e. weight_manager's per-layer torch loops (weight_manager.py:103-238) done as one
// launch over up to SEG_GROUP layers.  Workgroup b serves layer l with
// block_start[l] <= b < block_start[l+1], elements [(b - block_start[l]) * SEG_CHUNK, ...).
// Semantics follow the reference's torch ops bit for bit:
//   weighted_sum_parameters (:182-212): Python sum() from int 0 over param * coeff, i.e.
//     acc = fl(0 + fl(x_0 * fl32(c_0))); acc = fl(acc + fl(x_i * fl32(c_i)))  (-0 becomes +0)
//   increment_parameters (:103-137):  w = fl(w + fl(fl32(mult) * u))
//   get_parameters / set_parameters: plain copies.
// ------------------------------------------------------------------------------------
#define SEG_GROUP 32
#define SEG_CHUNK 8192  // elements per workgroup

struct SegArgs {
  const void* p[FEDAGG_FLAT_MAX_LISTS][SEG_GROUP];  // list-major layer pointers
  uint64_t n[SEG_GROUP];
  uint64_t flat_off[SEG_GROUP];
  uint32_t block_start[SEG_GROUP + 1];
  double coeff[FEDAGG_FLAT_MAX_LISTS];
  uint32_t f64;  // bit j: list j is fp64; bit 31: the flat bucket is fp64
  int nl, nlists;
};

__device__ __forceinline__ int seg_of_block(const SegArgs& a, uint32_t b) {
  int l = 0;
  while (l + 1 < a.nl && a.block_start[l + 1] <= b) ++l;  // scalar, <= SEG_GROUP steps
  return l;
}

// torch's ``tensor * python_float``: fp32 tensors compute in fp32 with the scalar rounded to
// fp32, fp64 tensors in fp64.  Returned in double (exact for the fp32 product).
__device__ __forceinline__ double seg_product(const void* p, uint64_t i, bool is64, double c) {
#pragma clang fp contract(off)
  if (is64) return static_cast<const double*>(p)[i] * c;
  return (double)(static_cast<const float*>(p)[i] * (float)c);
}

// op 0: gather (flat = p0), 1: scatter (p0 = flat), 2: wsum (flat = sum() of p_j * c_j),
// 3: increment (p0 = p0 + c0 * flat).  Layers and flat are fp32 or fp64 per SegArgs::f64;
// mixed fp32/fp64 operands follow torch's promotion (the op runs in fp64 once either side is).
template <int OP>
__global__ void __launch_bounds__(FA_BLOCK) flat_seg_kernel(const SegArgs a, void* __restrict__ flat) {
#pragma clang fp contract(off)
  const int l = seg_of_block(a, blockIdx.x);
  const uint64_t base = (uint64_t)(blockIdx.x - a.block_start[l]) * SEG_CHUNK;
  const uint64_t n = a.n[l];
  const bool flat64 = (a.f64 >> 31) & 1u;
  float* f32 = static_cast<float*>(flat) + a.flat_off[l];
  double* f64 = static_cast<double*>(flat) + a.flat_off[l];
  for (uint64_t i = base + threadIdx.x; i < base + SEG_CHUNK && i < n; i += FA_BLOCK) {
    if constexpr (OP == 0) {
      if (flat64) f64[i] = static_cast<const double*>(a.p[0][l])[i];
      else f32[i] = static_cast<const float*>(a.p[0][l])[i];
    } else if constexpr (OP == 1) {
      if (flat64) const_cast<double*>(static_cast<const double*>(a.p[0][l]))[i] = f64[i];
      else const_cast<float*>(static_cast<const float*>(a.p[0][l]))[i] = f32[i];
    } else if constexpr (OP == 2) {
      // Python sum() from int 0: 0 + p_0 (-0 becomes +0), then acc + p_j in the promoted type
      bool acc64 = a.f64 & 1u;
      double acc = seg_product(a.p[0][l], i, acc64, a.coeff[0]);
      acc = acc64 ? 0.0 + acc : (double)(0.0f + (float)acc);
      for (int j = 1; j < a.nlists; ++j) {
        const bool is64 = (a.f64 >> j) & 1u;
        const double t = seg_product(a.p[j][l], i, is64, a.coeff[j]);
        acc64 = acc64 || is64;
        acc = acc64 ? acc + t : (double)((float)acc + (float)t);
      }
      if (flat64) f64[i] = acc;
      else f32[i] = (float)acc;
    } else {
      // w += m * u with w fp32: u fp32 -> fl32(w + fl32(fl32(m) * u)); u fp64 -> fl32(w + fl64(m * u))
      float* w = const_cast<float*>(static_cast<const float*>(a.p[0][l]));
      if (flat64) {
        const double t = a.coeff[0] * f64[i];
        w[i] = (float)((double)w[i] + t);
      } else {
        const float t = (float)a.coeff[0] * f32[i];
        w[i] = w[i] + t;
      }
    }
  }
}

// All-fp32 form of flat_seg_kernel: 16-B accesses (4 elements per lane).  Layer tensors are
// 16-B aligned, but a layer's slice of the flat bucket starts wherever the previous layers end,
// so the accesses are declared 4-B aligned: gfx950 serves unaligned dwordx4 loads and stores,
// a wave still touches one contiguous KiB (plus at most one extra line).  Same per-element
// arithmetic as the scalar kernel's fp32 branches.
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));

template <int OP>
__global__ void __launch_bounds__(FA_BLOCK) flat_seg_vec_kernel(const SegArgs a, float* __restrict__ flat) {
#pragma clang fp contract(off)
  const int l = seg_of_block(a, blockIdx.x);
  const uint64_t base = (uint64_t)(blockIdx.x - a.block_start[l]) * SEG_CHUNK;
  const uint64_t n = a.n[l];
  const uint64_t end = base + SEG_CHUNK < n ? base + SEG_CHUNK : n;
  float* f = flat + a.flat_off[l];
  float cf[FEDAGG_FLAT_MAX_LISTS];
#pragma unroll
  for (int j = 0; j < FEDAGG_FLAT_MAX_LISTS; ++j) cf[j] = (float)a.coeff[j];  // torch rounds the scalar
  for (uint64_t i = base + 4 * (uint64_t)threadIdx.x; i < end; i += 4 * (uint64_t)FA_BLOCK) {
    if (i + 4 <= end) {
      if constexpr (OP == 0) {
        *reinterpret_cast<f32x4u*>(f + i) = *reinterpret_cast<const f32x4u*>(static_cast<const float*>(a.p[0][l]) + i);
      } else if constexpr (OP == 1) {
        *reinterpret_cast<f32x4u*>(const_cast<float*>(static_cast<const float*>(a.p[0][l])) + i) =
            *reinterpret_cast<const f32x4u*>(f + i);
      } else if constexpr (OP == 2) {
        const f32x4u t0 = *reinterpret_cast<const f32x4u*>(static_cast<const float*>(a.p[0][l]) + i) * cf[0];
        f32x4u acc = f32x4u(0.0f) + t0;  // Python sum() starts from int 0
        for (int j = 1; j < a.nlists; ++j) {
          const f32x4u t = *reinterpret_cast<const f32x4u*>(static_cast<const float*>(a.p[j][l]) + i) * cf[j];
          acc = acc + t;
        }
        *reinterpret_cast<f32x4u*>(f + i) = acc;
      } else {
        float* w = const_cast<float*>(static_cast<const float*>(a.p[0][l])) + i;
        const f32x4u t = cf[0] * *reinterpret_cast<const f32x4u*>(f + i);
        *reinterpret_cast<f32x4u*>(w) = *reinterpret_cast<const f32x4u*>(w) + t;
      }
    } else {
      for (uint64_t e = i; e < end; ++e) {
        if constexpr (OP == 0) {
          f[e] = static_cast<const float*>(a.p[0][l])[e];
        } else if constexpr (OP == 1) {
          const_cast<float*>(static_cast<const float*>(a.p[0][l]))[e] = f[e];
        } else if constexpr (OP == 2) {
          float acc = 0.0f + static_cast<const float*>(a.p[0][l])[e] * cf[0];
          for (int j = 1; j < a.nlists; ++j) {
            const float t = static_cast<const float*>(a.p[j][l])[e] * cf[j];
            acc = acc + t;
          }
          f[e] = acc;
        } else {
          float* w = const_cast<float*>(static_cast<const float*>(a.p[0][l]));
          const float t = cf[0] * f[e];
          w[e] = w[e] + t;
        }
      }
    }
  }
}

template <int OP>
int flat_seg_launch(const void* const* ptrs, const int* kinds, int nlists, const double* coeffs,
                    const uint64_t* numel, int L, void* flat, int flat_kind, hipStream_t s) {
  if (L < 0 || nlists < 1 || nlists > FEDAGG_FLAT_MAX_LISTS || (L > 0 && (!ptrs || !numel || !flat)))
    return fail(FEDAGG_EINVAL, "flat op: invalid argument (L=%lld)", L);
  if (flat_kind != FEDAGG_F32 && flat_kind != FEDAGG_F64)
    return fail(FEDAGG_EINVAL, "flat op: the flat bucket must be fp32 or fp64 (kind %lld)", flat_kind);
  uint32_t mask = flat_kind == FEDAGG_F64 ? (1u << 31) : 0u;
  bool any64 = false;
  for (int j = 0; j < nlists; ++j) {
    const int k = kinds ? kinds[j] : FEDAGG_F32;
    if (k != FEDAGG_F32 && k != FEDAGG_F64) return fail(FEDAGG_EINVAL, "flat op: list %lld is not fp32/fp64", j);
    if (k == FEDAGG_F64) mask |= 1u << j, any64 = true;
  }
  // operand kinds each op supports (the Python layer routes everything else to torch)
  if ((OP == 0 || OP == 1) && any64 != (flat_kind == FEDAGG_F64))
    return fail(FEDAGG_EINVAL, "flat copy: layer and flat kinds differ");
  if (OP == 2 && any64 != (flat_kind == FEDAGG_F64))
    return fail(FEDAGG_EINVAL, "flat wsum: the result kind must be the promoted kind of the lists");
  if (OP == 3 && any64) return fail(FEDAGG_EINVAL, "flat increment: parameters must be fp32");
  uint64_t off = 0;
  for (int l0 = 0; l0 < L; l0 += SEG_GROUP) {
    const int nl = (L - l0) < SEG_GROUP ? (L - l0) : SEG_GROUP;
    SegArgs a;
    memset(&a, 0, sizeof(a));
    a.nl = nl;
    a.nlists = nlists;
    a.f64 = mask;
    for (int j = 0; j < nlists; ++j) a.coeff[j] = coeffs ? coeffs[j] : 1.0;
    uint64_t blocks = 0;
    for (int l = 0; l < nl; ++l) {
      for (int j = 0; j < nlists; ++j) {
        a.p[j][l] = ptrs[(size_t)j * L + l0 + l];
        if (!a.p[j][l] && numel[l0 + l]) return fail(FEDAGG_EINVAL, "flat op: NULL layer pointer %lld", l0 + l);
      }
      a.n[l] = numel[l0 + l];
      a.flat_off[l] = off;
      a.block_start[l] = (uint32_t)blocks;
      off += numel[l0 + l];
      blocks += (numel[l0 + l] + SEG_CHUNK - 1) / SEG_CHUNK;
    }
    a.block_start[nl] = (uint32_t)blocks;
    if (blocks == 0) continue;
    if (mask == 0 && g_flat_vec)
      hipLaunchKernelGGL((flat_seg_vec_kernel<OP>), dim3((unsigned)blocks), dim3(FA_BLOCK), 0, s, a,
                         static_cast<float*>(flat));
    else
      hipLaunchKernelGGL((flat_seg_kernel<OP>), dim3((unsigned)blocks), dim3(FA_BLOCK), 0, s, a, flat);
    int rc = check_launch("flat_seg_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

// ------------------------------------------------------------------------------------
// read-stream probe (same 16-B non-temporal load path as the bucket kernels)
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(FA_BLOCK) read_probe_kernel(const float* __restrict__ x, uint64_t nvec,
                                                              float* __restrict__ sink) {
  const uint64_t stride = (uint64_t)gridDim.x * FA_BLOCK;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (uint64_t v = (uint64_t)blockIdx.x * FA_BLOCK + threadIdx.x; v < nvec; v += stride) {
    u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x) + v);
    s0 += __uint_as_float(r.x);
    s1 += __uint_as_float(r.y);
    s2 += __uint_as_float(r.z);
    s3 += __uint_as_float(r.w);
  }
  float t = s0 + s1 + s2 + s3;
  for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
  if (threadIdx.x == 0) sink[blockIdx.x] = t;
}

// The bucket kernels' own walk with one stream: one workgroup per tile of VPT x 256 contiguous
// 16-B vectors, all VPT nt loads issued before use (tools/hbm_ceiling_probe.hip: the fastest
// read pattern found, 7.1-7.2 TB/s over 32 GiB).  The sink is written only on an impossible fold
// value, so it needs one float and adds no traffic.
template <int VPT>
__global__ void __launch_bounds__(FA_BLOCK) read_probe_tile_kernel(const u32x4* __restrict__ x, uint64_t nvec,
                                                                   float* __restrict__ sink) {
  const uint64_t base = (uint64_t)blockIdx.x * VPT * FA_BLOCK + threadIdx.x;
  unsigned f = 0;
  if (base + (uint64_t)(VPT - 1) * FA_BLOCK < nvec) {
    u32x4 r[VPT];
#pragma unroll
    for (int n = 0; n < VPT; ++n) r[n] = __builtin_nontemporal_load(x + base + (uint64_t)n * FA_BLOCK);
#pragma unroll
    for (int n = 0; n < VPT; ++n) f ^= r[n].x ^ r[n].y ^ r[n].z ^ r[n].w;
  } else {
    for (uint64_t v = base; v < nvec; v += FA_BLOCK) f ^= x[v].x ^ x[v].y ^ x[v].z ^ x[v].w;
  }
  if (f == 0x9e3779b9u) sink[0] = __uint_as_float(f);
}

// ------------------------------------------------------------------------------------
// host-side launch helpers
// ------------------------------------------------------------------------------------
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline unsigned grid_for(uint64_t work) {
  uint64_t g = (work + FA_BLOCK - 1) / FA_BLOCK;
  if (g < 1) g = 1;
  if (g_grid_cap > 0 && g > (uint64_t)g_grid_cap) g = (uint64_t)g_grid_cap;
  return (unsigned)g;
}

template <typename E, bool NT, int NTS, int VPT, int U, bool PIPE, bool TILE, int OCC = 1, bool BUF = false,
          int BLK = FA_BLOCK, bool INTER = false>
void launch_fedavg_variant(unsigned grid, hipStream_t s, const FaArgs<E, FEDAGG_KCHUNK>& a, const PwArgs& pw,
                           int kc, int first, uint64_t nvec, uint64_t M, typename E::Out* out, uint64_t pitch = 0) {
  if (BLK != FA_BLOCK) grid = (grid + BLK / FA_BLOCK - 1) / (BLK / FA_BLOCK);  // the caller sized it for 256
  hipLaunchKernelGGL((fedavg_kernel<E, FEDAGG_KCHUNK, NT, NTS, VPT, U, PIPE, TILE, OCC, BUF, BLK, INTER ? VPT * BLK : 0>),
                     dim3(grid), dim3(BLK), 0, s, a, pw, kc, first, nvec, M, out, g_xcd, g_tpb, pitch, g_rel_sys,
                     static_cast<const typename E::Out*>(g_acc_in));
}

// Shape family (fedagg_tune "vpt" / "unroll" / "tile" / "pipe"), instantiated for every element
// type: contiguous tiles of VPT*256 vectors per workgroup step with U-client load groups, the
// grid-strided single-vector shape, and the pipelined variant; each with plain or
// non-temporal output stores.  Client loads are non-temporal unless nt_load = 0 (one shape).
// Measured on MI355X (tools/tune_fedavg.py, profiles/r01_tune_*.log, r01_vpt16_*.log): 8 KiB per
// wave per client (vpt 8) with 4-client load groups is best at 8 clients (8 x 25M fp32: 6.5 TB/s;
// 16 KiB loses 11 %: half the workgroups); from 32 clients on, 16 KiB per wave per client with
// 2-client groups wins (32 x 125M: +3 %, 64 x 125M fp32: 6.79 vs 6.65 TB/s, 128 x 350M bf16: +1 %);
// 16 clients tie.  Box-to-box spread is ~3 %.
struct Shape {
  int vpt, unroll;
  bool pipe;
  int occ;  // > 1: the register-capped (amdgpu_waves_per_eu) build of the 8/16-KiB tile
  bool buf;  // buffer-descriptor client loads
  int blk = FA_BLOCK;  // threads per workgroup (global-load tiles without pipelining)
};
template <typename E>
inline Shape shape_for(int K, uint64_t nvec) {
  const int blk = g_fa_blk ? g_fa_blk : FA_BLOCK;
  if (g_vpt > 0) return {g_vpt, g_unroll, g_pipe != 0, g_fa_occ, g_buf != 0, blk};
  // fp64: the adds of a client group take long enough that the HBM idles unless the next
  // group's loads are already in flight (software-pipelined tiles: 8 x 25M fp64 6.0 vs 5.1 TB/s,
  // 64 x 62.5M 6.1 vs 4.9; profiles/r01_tune2_f64_*.log)
  if constexpr (std::is_same<E, F64>::value) return Shape{4, 4, true, 0};
  // many client streams over a SHORT bucket (the runs of the client-sharded schedules, relay
  // chunks): a tile small enough for the grid to cover the CUs twice over -- 64 x 2M fp32: 7.10
  // TB/s with 4 x 4 against 5.59 with 8 x 4 (244 workgroups); 64 x 1M: 6.80 with 2 x 8 against
  // 3.29; 64 x 0.5M: 6.44 against 1.84 (profiles/r03e_small_runs_probe.log)
  if constexpr (std::is_same<E, F32>::value || std::is_same<E, BF16>::value) {
    if (K >= 32 && nvec < (uint64_t)384 * 1024) return Shape{2, 8, false, 0, false, blk};
    if (K >= 32 && nvec < (uint64_t)768 * 1024) return Shape{4, 4, false, 0, false, blk};
  }
  // many client streams over a large bucket: 16 KiB per wave per stream (fewer DRAM row
  // switches; 64 x 125M fp32 +2 %, 128 x 350M bf16 +1 %, 64 x 125M fp16 +1 %), as long as the
  // grid stays >> 256 CUs
  if (K >= 32 && nvec >= (uint64_t)16 * FA_BLOCK * 2048) {
    // bf16: client pairs with buffer-descriptor loads (128 x 350M: 12.64 vs 12.96 ms with global
    // loads, 64 x 125M: -7.7 %; profiles/r01_buf2_*.log; slower for fp32, r01_buf_c{2,3}.log);
    // fp32: client pairs in 512-thread workgroups (253 VGPRs under the 512-thread launch bound,
    // 2 waves per SIMD, no spill): 64 x 125M 4.68 vs 4.79 ms for the 256-thread build capped to 2
    // waves, 0.3-1.4 % on five other K >= 32 shapes, never slower (profiles/r02_blk*.log); the
    // 256-thread build uncapped takes 257 registers and runs 1 wave (-1.4 %, r01_occ_c3.log)
    if constexpr (std::is_same<E, BF16>::value) return Shape{16, 2, false, g_fa_occ, true, blk};
    if constexpr (std::is_same<E, F32>::value)
      return Shape{16, 2, false, g_fa_occ > 1 ? g_fa_occ : 2, false, g_fa_blk ? g_fa_blk : 2 * FA_BLOCK};
    return Shape{16, 2, false, g_fa_occ, false, blk};
  }
  if constexpr (std::is_same<E, F16>::value) return Shape{4, 4, false, 0, g_buf != 0};  // 8 x 25M: +5 % over 8 KiB
  return Shape{8, 4, false, g_fa_occ, g_buf != 0, blk};
}

template <typename E, int NTS>
void launch_fedavg_shape(unsigned grid, hipStream_t s, const FaArgs<E, FEDAGG_KCHUNK>& a, const PwArgs& pw, int kc,
                         int first, uint64_t nvec, uint64_t M, typename E::Out* out, Shape sh) {
#define FA_ARGS grid, s, a, pw, kc, first, nvec, M, out
#if !FEDAGG_TUNING
  // product: the shapes shape_for returns under the default knobs (sc1 or nt output stores)
  if constexpr (std::is_same<E, F64>::value) {
    return launch_fedavg_variant<E, true, NTS, 4, 4, true, true>(FA_ARGS);  // pipelined 4 x 4
  } else if constexpr (std::is_same<E, F16>::value) {
    if (sh.vpt >= 16) return launch_fedavg_variant<E, true, NTS, 16, 2, false, true>(FA_ARGS);
    return launch_fedavg_variant<E, true, NTS, 4, 4, false, true>(FA_ARGS);
  } else {
    if (sh.vpt >= 16) {
      if constexpr (std::is_same<E, BF16>::value)  // client pairs over buffer descriptors
        return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, true>(FA_ARGS);
      else  // client pairs in 512-thread workgroups
        return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, false, 512>(FA_ARGS);
    }
    if (sh.vpt <= 2) return launch_fedavg_variant<E, true, NTS, 2, 8, false, true>(FA_ARGS);  // short buckets
    if (sh.vpt <= 4) return launch_fedavg_variant<E, true, NTS, 4, 4, false, true>(FA_ARGS);
    return launch_fedavg_variant<E, true, NTS, 8, 4, false, true>(FA_ARGS);
  }
#else
  if constexpr (NTS == 2 || NTS == 3) {  // write-through (sc1 / sc0 sc1) output stores: the auto shapes and their neighbours only
    if (sh.pipe) {
      if (sh.vpt >= 8) return launch_fedavg_variant<E, true, NTS, 8, 2, true, true>(FA_ARGS);
      return launch_fedavg_variant<E, true, NTS, 4, 4, true, true>(FA_ARGS);
    }
    if constexpr (std::is_same<E, F32>::value || std::is_same<E, BF16>::value) {
      if (sh.vpt >= 16 && sh.blk > FA_BLOCK && !sh.buf)
        return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, false, 512>(FA_ARGS);
      if (sh.vpt >= 16 && sh.buf) return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, true>(FA_ARGS);
      if (sh.vpt >= 16 && sh.occ > 1) return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 2>(FA_ARGS);
    }
    if (sh.vpt >= 16) return launch_fedavg_variant<E, true, NTS, 16, 2, false, true>(FA_ARGS);
    if (sh.vpt >= 8) return launch_fedavg_variant<E, true, NTS, 8, 4, false, true>(FA_ARGS);
    return launch_fedavg_variant<E, true, NTS, 4, 4, false, true>(FA_ARGS);
  } else {
  if (!g_nt_load) return launch_fedavg_variant<E, false, NTS, 1, 8, false, false>(FA_ARGS);
  if (g_tile) {
    if (sh.pipe) {  // contiguous tiles with the next client group's loads issued before this group's adds
      if (sh.vpt >= 8) return launch_fedavg_variant<E, true, NTS, 8, 2, true, true>(FA_ARGS);
      return launch_fedavg_variant<E, true, NTS, 4, 4, true, true>(FA_ARGS);
    }
    if constexpr (NTS == 1 && std::is_same<E, F16>::value) {
      if (sh.buf && !sh.pipe) {  // fp16: buffer-descriptor loads, uncapped builds only
        if (sh.vpt >= 16) {
          if (sh.unroll <= 1) return launch_fedavg_variant<E, true, NTS, 16, 1, false, true, 1, true>(FA_ARGS);
          return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, true>(FA_ARGS);
        }
        if (sh.vpt >= 8 && sh.unroll > 2) return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 1, true>(FA_ARGS);
        if (sh.vpt >= 4 && sh.unroll >= 4) return launch_fedavg_variant<E, true, NTS, 4, 4, false, true, 1, true>(FA_ARGS);
      }
    }
    if constexpr (NTS == 1 && (std::is_same<E, F32>::value || std::is_same<E, BF16>::value)) {
      if constexpr (std::is_same<E, F32>::value) {
        if (sh.blk > 2 * FA_BLOCK && !sh.buf && !sh.pipe) {  // 1024-thread workgroups (experiment)
          if (sh.vpt >= 8) return launch_fedavg_variant<E, true, NTS, 8, 2, false, true, 1, false, 1024>(FA_ARGS);
          return launch_fedavg_variant<E, true, NTS, 4, 4, false, true, 1, false, 1024>(FA_ARGS);
        }
      }
      if (sh.blk > FA_BLOCK && !sh.buf && !sh.pipe) {  // 512-thread workgroups
        if (sh.vpt >= 16) return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, false, 512>(FA_ARGS);
        if (sh.vpt >= 8 && sh.unroll <= 2) return launch_fedavg_variant<E, true, NTS, 8, 2, false, true, 1, false, 512>(FA_ARGS);
        if (sh.vpt >= 8) return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 1, false, 512>(FA_ARGS);
        return launch_fedavg_variant<E, true, NTS, 4, 4, false, true, 1, false, 512>(FA_ARGS);
      }
      if (sh.buf && !sh.pipe) {  // buffer-descriptor loads (one lane offset for every client stream)
        if (sh.vpt >= 16) {
          if (sh.unroll <= 1) {
            if (sh.occ > 1) return launch_fedavg_variant<E, true, NTS, 16, 1, false, true, 2, true>(FA_ARGS);
            return launch_fedavg_variant<E, true, NTS, 16, 1, false, true, 1, true>(FA_ARGS);
          }
          if (sh.occ > 1) return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 2, true>(FA_ARGS);
          return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 1, true>(FA_ARGS);
        }
        if (sh.vpt >= 8 && sh.unroll > 2) {
          if (sh.occ >= 4) return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 4, true>(FA_ARGS);
          if (sh.occ == 3) return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 3, true>(FA_ARGS);
          return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 1, true>(FA_ARGS);
        }
      }
      if (sh.occ > 1) {  // register-capped occupancy variants of the 8- and 16-KiB shapes
        if (sh.vpt >= 16) {
          if (sh.unroll <= 1) {
            if (sh.occ <= 2) return launch_fedavg_variant<E, true, NTS, 16, 1, false, true, 2>(FA_ARGS);
            return launch_fedavg_variant<E, true, NTS, 16, 1, false, true, 3>(FA_ARGS);
          }
          return launch_fedavg_variant<E, true, NTS, 16, 2, false, true, 2>(FA_ARGS);
        }
        if (sh.vpt >= 8 && sh.unroll > 2) {
          if (sh.occ >= 4) return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 4>(FA_ARGS);
          return launch_fedavg_variant<E, true, NTS, 8, 4, false, true, 3>(FA_ARGS);
        }
      }
    }
    if (sh.vpt >= 16) {  // 16 KiB per wave per client stream
      if (sh.unroll <= 1) return launch_fedavg_variant<E, true, NTS, 16, 1, false, true>(FA_ARGS);
      return launch_fedavg_variant<E, true, NTS, 16, 2, false, true>(FA_ARGS);
    }
    if (sh.vpt >= 8) {
      if (sh.unroll <= 2) return launch_fedavg_variant<E, true, NTS, 8, 2, false, true>(FA_ARGS);
      return launch_fedavg_variant<E, true, NTS, 8, 4, false, true>(FA_ARGS);
    }
    if (sh.vpt >= 4) {
      if (sh.unroll <= 4) return launch_fedavg_variant<E, true, NTS, 4, 4, false, true>(FA_ARGS);
      return launch_fedavg_variant<E, true, NTS, 4, 8, false, true>(FA_ARGS);
    }
    if (sh.vpt >= 2) return launch_fedavg_variant<E, true, NTS, 2, 8, false, true>(FA_ARGS);
  }
  if (g_pipe) return launch_fedavg_variant<E, true, NTS, 1, 8, true, false>(FA_ARGS);
  if (sh.vpt >= 2) return launch_fedavg_variant<E, true, NTS, 2, 8, false, false>(FA_ARGS);
  if (sh.unroll >= 16) return launch_fedavg_variant<E, true, NTS, 1, 16, false, false>(FA_ARGS);
  if (sh.unroll <= 4) return launch_fedavg_variant<E, true, NTS, 1, 4, false, false>(FA_ARGS);
  return launch_fedavg_variant<E, true, NTS, 1, 8, false, false>(FA_ARGS);
  }
#endif
#undef FA_ARGS
}

template <typename E>
void launch_fedavg(unsigned grid, hipStream_t s, const FaArgs<E, FEDAGG_KCHUNK>& a, const PwArgs& pw, int kc,
                   int first, uint64_t nvec, uint64_t M, typename E::Out* out, bool nts, bool sc1, Shape sh) {
  if constexpr (std::is_same<E, F32>::value || std::is_same<E, BF16>::value) {
    if (g_rel_sys) return launch_fedavg_shape<E, 3>(grid, s, a, pw, kc, first, nvec, M, out, sh);  // push runs
  }
#if FEDAGG_TUNING
  if (nts && sc1 && g_nt_load && g_tile)
    launch_fedavg_shape<E, 2>(grid, s, a, pw, kc, first, nvec, M, out, sh);
  else if (nts)
    launch_fedavg_shape<E, 1>(grid, s, a, pw, kc, first, nvec, M, out, sh);
  else
    launch_fedavg_shape<E, 0>(grid, s, a, pw, kc, first, nvec, M, out, sh);
#else
  (void)nts;  // non-temporal loads and stores are fixed in the product build
  if (sc1)
    launch_fedavg_shape<E, 2>(grid, s, a, pw, kc, first, nvec, M, out, sh);
  else
    launch_fedavg_shape<E, 1>(grid, s, a, pw, kc, first, nvec, M, out, sh);
#endif
}

// idx_in (tile-interleaved buckets): where each numel==1 element sits in the client buckets
// (NULL: at its output index, the row layout).
template <typename E>
int fedavg_pairwise_launch(const typename E::In* const* x, const typename E::P* w, int K, const uint64_t* idx, int P,
                           void* ws, typename E::Out* out, hipStream_t s, const uint64_t* idx_in = nullptr) {
  if (P == 0) return FEDAGG_OK;
  if (K <= 0 || P < 0 || !x || !w || !idx || !ws || !out)
    return fail(FEDAGG_EINVAL, "fedavg_pairwise: invalid argument (K=%lld)", K);
  using W = typename E::W;
  W* wsT = static_cast<W*>(ws);
  for (int p0 = 0; p0 < P; p0 += FEDAGG_MAX_PAIRWISE) {
    const int pc = (P - p0) < FEDAGG_MAX_PAIRWISE ? (P - p0) : FEDAGG_MAX_PAIRWISE;
    IdxArgs ix, ixin;
    memset(&ix, 0, sizeof(ix));
    for (int p = 0; p < pc; ++p) ix.idx[p] = idx[p0 + p];
    ixin = ix;
    if (idx_in)
      for (int p = 0; p < pc; ++p) ixin.idx[p] = idx_in[p0 + p];
    for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK) {
      const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
      FaArgs<E, FEDAGG_KCHUNK> a;
      memset(&a, 0, sizeof(a));
      for (int k = 0; k < kc; ++k) {
        a.x[k] = x[k0 + k];
        a.w[k] = w[k0 + k];
      }
      const unsigned g = (unsigned)((pc * kc + FA_BLOCK - 1) / FA_BLOCK);
      hipLaunchKernelGGL((pairwise_gather_kernel<E, FEDAGG_KCHUNK>), dim3(g), dim3(FA_BLOCK), 0, s, a, kc, k0, ixin,
                         pc, (int64_t)K, wsT);
      int rc = check_launch("pairwise_gather_kernel");
      if (rc) return rc;
    }
    hipLaunchKernelGGL((pairwise_tree_kernel<E>), dim3(1), dim3(64), 0, s, (const W*)wsT, (int64_t)K, (int64_t)K, ix,
                       pc, out);
    int rc = check_launch("pairwise_tree_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

// Products of a client block at the numel==1 indices, for a pairwise tree over clients held by
// several launches (or ranks): ws[p * stride + kbase + k] = fl(x_k[idx_p] * w_k) in type W.
template <typename E>
int pairwise_products_launch(const typename E::In* const* x, const typename E::P* w, int K, const uint64_t* idx,
                             int P, int64_t stride, int kbase, typename E::W* ws, hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (K <= 0 || P < 0 || !x || !w || !idx || !ws || kbase < 0 || stride < (int64_t)kbase + K)
    return fail(FEDAGG_EINVAL, "pairwise_products: invalid argument (K=%lld)", K);
  for (int k = 0; k < K; ++k)
    if (!x[k]) return fail(FEDAGG_EINVAL, "pairwise_products: client pointer %lld is NULL", k);
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
      hipLaunchKernelGGL((pairwise_gather_kernel<E, FEDAGG_KCHUNK>), dim3(g), dim3(FA_BLOCK), 0, s, a, kc, kbase + k0,
                         ix, pc, stride, ws + (int64_t)p0 * stride);
      int rc = check_launch("pairwise_gather_kernel");
      if (rc) return rc;
    }
  }
  return FEDAGG_OK;
}

// out[idx_p] = +0.0 + pairwise(ws[p * stride .. p * stride + n)) for p < P.
template <typename E>
int pairwise_finish_launch(const typename E::W* ws, int64_t n, int64_t stride, const uint64_t* idx, int P,
                           typename E::Out* out, hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (n <= 0 || P < 0 || stride < n || !ws || !idx || !out)
    return fail(FEDAGG_EINVAL, "pairwise_finish: invalid argument (n=%lld)", n);
  for (int p0 = 0; p0 < P; p0 += FEDAGG_MAX_PAIRWISE) {
    const int pc = (P - p0) < FEDAGG_MAX_PAIRWISE ? (P - p0) : FEDAGG_MAX_PAIRWISE;
    IdxArgs ix;
    memset(&ix, 0, sizeof(ix));
    for (int p = 0; p < pc; ++p) ix.idx[p] = idx[p0 + p];
    hipLaunchKernelGGL((pairwise_tree_kernel<E>), dim3(1), dim3(64), 0, s, ws + (int64_t)p0 * stride, n, stride, ix,
                       pc, out);
    int rc = check_launch("pairwise_tree_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

// seed = false: the accumulator starts from d_out (a partial sum over the clients before this
// block, e.g. received from the previous rank of a client-sharded chain) instead of +0.0.
template <typename E>
int fedavg_launch(const typename E::In* const* x, const typename E::P* w, int K, uint64_t M, const uint64_t* idx,
                  int P, void* ws, typename E::Out* out, hipStream_t s, bool seed = true) {
  if (K <= 0) return fail(FEDAGG_EINVAL, "fedavg: K must be > 0 (got %lld)", K);
  if (!x || !w || !out) return fail(FEDAGG_EINVAL, "fedavg: NULL argument");
  if (P < 0 || (P > 0 && !idx)) return fail(FEDAGG_EINVAL, "fedavg: bad pairwise index list (P=%lld)", P);
  for (int p = 0; p < P; ++p)
    if (idx[p] >= M) return fail(FEDAGG_EINVAL, "fedavg: pairwise index %lld out of range", (long long)idx[p]);
  if (M == 0) return FEDAGG_OK;
  bool vec = aligned16(out);
  for (int k = 0; k < K; ++k) {
    if (!x[k]) return fail(FEDAGG_EINVAL, "fedavg: client pointer %lld is NULL", k);
    vec = vec && aligned16(x[k]);
  }
  const bool fuse = g_fuse_pw && P <= FEDAGG_FUSED_PAIRWISE && K <= FEDAGG_KCHUNK;
  if (P > 0 && !fuse && !ws) return fail(FEDAGG_EINVAL, "fedavg: workspace needed for %lld pairwise segments", P);
  const uint64_t nvec = vec ? M / E::L : 0;
  const Shape sh = shape_for<E>(K, nvec);
  const uint64_t per_thread = (g_tile && g_nt_load) ? (uint64_t)sh.vpt : 1;
  unsigned grid = grid_for(nvec ? (nvec + per_thread - 1) / per_thread : M);
  if (g_tpb > 1 && g_tile && nvec)  // every tile exactly once: no grid cap with tpb
    grid = (unsigned)(((nvec + per_thread - 1) / per_thread + g_tpb - 1) / g_tpb);
  for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK) {
    const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
    FaArgs<E, FEDAGG_KCHUNK> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) {
      a.x[k] = x[k0 + k];
      a.w[k] = w[k0 + k];
    }
    PwArgs pw;
    memset(&pw, 0, sizeof(pw));
    if (fuse) {
      pw.n = P;
      for (int p = 0; p < P; ++p) pw.idx[p] = idx[p];
    }
    const bool nts = g_nt_store < 0 ? K >= NT_STORE_MIN_K : g_nt_store != 0;
    const bool sc1 = g_st_sc1 < 0 ? K < SC1_MAX_K : g_st_sc1 != 0;
    launch_fedavg<E>(grid, s, a, pw, kc, (k0 == 0 && seed) ? 1 : 0, nvec, M, out, nts, sc1, sh);
    g_acc_in = nullptr;  // later chunks continue from out
    int rc = check_launch("fedavg_kernel");
    if (rc) return rc;
  }
  if (P > 0 && !fuse) return fedavg_pairwise_launch<E>(x, w, K, idx, P, ws, out, s);
  return FEDAGG_OK;
}

// Tile-interleaved buckets (fedagg_fedavg_tiled_*): the tiled kernels walk the same tiles as the
// row-layout auto shapes -- fp32: 16 vectors x 512 threads from 32 clients over large buckets
// (FEDAGG_TILE_VECTORS_F32), 8 x 256 with write-through stores below 32 clients
// (FEDAGG_TILE_VECTORS_F32_FEW); bf16: 16 x 256 with buffer loads.  The layout is recommended
// (fedagg_fedavg_tile_vectors_*) where the row-layout auto shape is that very tile; the tiled
// entry points take any K and M with one of those tiles.
template <typename E>
bool tiled_tile_ok(uint64_t tv) {
  if constexpr (std::is_same<E, F32>::value) return tv == FEDAGG_TILE_VECTORS_F32 || tv == FEDAGG_TILE_VECTORS_F32_FEW;
  if constexpr (std::is_same<E, BF16>::value) return tv == FEDAGG_TILE_VECTORS_BF16;
  return false;
}

template <typename E>
uint64_t tiled_tile_vectors(int K, uint64_t M) {
  if (K <= 0 || !g_nt_load || !g_tile || g_vpt > 0 || g_tpb > 1) return 0;
  const uint64_t nvec = M / E::L;
  const Shape sh = shape_for<E>(K, nvec);
  if (sh.pipe) return 0;
  if constexpr (std::is_same<E, F32>::value) {
    if (sh.vpt == 16 && sh.unroll == 2 && sh.blk == 2 * FA_BLOCK && !sh.buf) return FEDAGG_TILE_VECTORS_F32;
    // the few-client tile with its write-through stores, over >= 1024 workgroup tiles
    const bool sc1 = g_st_sc1 < 0 ? K < SC1_MAX_K : g_st_sc1 != 0;
    const bool nts = g_nt_store < 0 ? K >= NT_STORE_MIN_K : g_nt_store != 0;
    if (g_tiled_few && sh.vpt == 8 && sh.unroll == 4 && sh.blk == FA_BLOCK && !sh.buf && sh.occ <= 1 && sc1 && nts &&
        nvec >= (uint64_t)FEDAGG_TILE_VECTORS_F32_FEW * 1024)
      return FEDAGG_TILE_VECTORS_F32_FEW;
    return 0;
  }
  if constexpr (std::is_same<E, BF16>::value)
    return sh.vpt == 16 && sh.unroll == 2 && sh.buf && sh.occ <= 1 ? FEDAGG_TILE_VECTORS_BF16 : 0;
  return 0;
}

template <typename E>
int fedavg_tiled_launch(const typename E::In* base, const typename E::P* w, int K, uint64_t M, uint64_t tv,
                        const uint64_t* idx, int P, void* ws, typename E::Out* out, hipStream_t s, bool seed = true) {
  if (K <= 0) return fail(FEDAGG_EINVAL, "fedavg_tiled: K must be > 0 (got %lld)", K);
  if (!base || !w || !out) return fail(FEDAGG_EINVAL, "fedavg_tiled: NULL argument");
  if (!aligned16(base) || !aligned16(out)) return fail(FEDAGG_EINVAL, "fedavg_tiled: buffers must be 16-B aligned");
  if (!tiled_tile_ok<E>(tv))
    return fail(FEDAGG_EINVAL, "fedavg_tiled: the tile must be one of FEDAGG_TILE_VECTORS_* (got %lld vectors)",
                (long long)tv);
  if (P < 0 || (P > 0 && !idx)) return fail(FEDAGG_EINVAL, "fedavg_tiled: bad pairwise index list (P=%lld)", P);
  for (int p = 0; p < P; ++p)
    if (idx[p] >= M) return fail(FEDAGG_EINVAL, "fedavg_tiled: pairwise index %lld out of range", (long long)idx[p]);
  const bool fuse = g_fuse_pw && P <= FEDAGG_FUSED_PAIRWISE && K <= FEDAGG_KCHUNK;
  if (P > 0 && !fuse && !ws) return fail(FEDAGG_EINVAL, "fedavg_tiled: workspace needed for %lld pairwise segments", P);
  constexpr int L = E::L;
  const uint64_t nvec = M / L, pitch = (uint64_t)K * tv;
  const uint64_t vpt = tv == FEDAGG_TILE_VECTORS_F32_FEW ? 8 : 16;
  const unsigned grid = grid_for((nvec + vpt - 1) / vpt);
  std::vector<const typename E::In*> x(K);
  for (int k = 0; k < K; ++k) x[k] = base + (uint64_t)k * tv * L;
  for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK) {
    const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
    FaArgs<E, FEDAGG_KCHUNK> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) {
      a.x[k] = x[k0 + k];
      a.w[k] = w[k0 + k];
    }
    PwArgs pw;
    memset(&pw, 0, sizeof(pw));
    if (fuse) {
      pw.n = P;
      for (int p = 0; p < P; ++p) pw.idx[p] = idx[p];
    }
    const int first = (k0 == 0 && seed) ? 1 : 0;
    if constexpr (std::is_same<E, F32>::value) {
      if (tv == FEDAGG_TILE_VECTORS_F32_FEW)  // 8 x 256 tile, write-through (sc1) stores
        launch_fedavg_variant<E, true, 2, 8, 4, false, true, 1, false, FA_BLOCK, true>(grid, s, a, pw, kc, first, nvec,
                                                                                      M, out, pitch);
      else
        launch_fedavg_variant<E, true, 1, 16, 2, false, true, 1, false, 2 * FA_BLOCK, true>(grid, s, a, pw, kc, first,
                                                                                            nvec, M, out, pitch);
    } else
      launch_fedavg_variant<E, true, 1, 16, 2, false, true, 1, true, FA_BLOCK, true>(grid, s, a, pw, kc, first, nvec,
                                                                                    M, out, pitch);
    int rc = check_launch("fedavg_kernel (tiled)");
    if (rc) return rc;
  }
  if (P > 0 && !fuse) {
    std::vector<uint64_t> in(P);
    for (int p = 0; p < P; ++p) {
      const uint64_t v = idx[p] / L;
      in[p] = ((v / tv) * pitch + v % tv) * L + idx[p] % L;
    }
    return fedavg_pairwise_launch<E>(x.data(), w, K, idx, P, ws, out, s, in.data());
  }
  return FEDAGG_OK;
}

template <typename TIn>
int scaffold_pairwise_launch(const TIn* const* d, const TIn* const* cv, const TIn* c, const double* w, int K,
                             const uint64_t* idx, int P, double lr, void* ws, double* dout, double* cout,
                             hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (K <= 0 || P < 0 || !d || !cv || !c || !w || !idx || !ws || !dout || !cout)
    return fail(FEDAGG_EINVAL, "scaffold_pairwise: invalid argument (K=%lld)", K);
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
    hipLaunchKernelGGL((scaffold_tree_kernel<TIn>), dim3(1), dim3(64), 0, s, (const double*)ws_d, ws_c, c,
                       (int64_t)K, ix, pc, lr, dout, cout);
    int rc = check_launch("scaffold_tree_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

// Client-block products for a Scaffold pairwise tree held by several launches / ranks.  ws layout:
// delta terms [P][Ktot] doubles, then control-variate terms [P][Ktot + 1] (the last column is c,
// written by the finish step); this block's clients go to columns kbase .. kbase + K - 1.
template <typename TIn>
int scaffold_products_launch(const TIn* const* d, const TIn* const* cv, const double* w, int K, int kbase, int Ktot,
                             const uint64_t* idx, int P, double* ws, hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (K <= 0 || P < 0 || !d || !cv || !w || !idx || !ws || kbase < 0 || kbase + K > Ktot)
    return fail(FEDAGG_EINVAL, "scaffold_products: invalid argument (K=%lld)", K);
  for (int k = 0; k < K; ++k)
    if (!d[k] || !cv[k]) return fail(FEDAGG_EINVAL, "scaffold_products: client pointer %lld is NULL", k);
  double* ws_d = ws;
  double* ws_c = ws + (size_t)P * Ktot;
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
                         kc, kbase + k0, ix, pc, (int64_t)Ktot, ws_d + (size_t)p0 * Ktot,
                         ws_c + (size_t)p0 * (Ktot + 1));
      int rc = check_launch("scaffold_gather_kernel");
      if (rc) return rc;
    }
  }
  return FEDAGG_OK;
}

// dout[idx_p] = lr * (0 + pairwise(delta terms)), cout[idx_p] = 0 + pairwise(cv terms, c last).
template <typename TIn>
int scaffold_finish_launch(double* ws, int Ktot, const TIn* c, const uint64_t* idx, int P, double lr, double* dout,
                           double* cout, hipStream_t s) {
  if (P == 0) return FEDAGG_OK;
  if (Ktot <= 0 || P < 0 || !ws || !c || !idx || !dout || !cout)
    return fail(FEDAGG_EINVAL, "scaffold_finish: invalid argument (K=%lld)", Ktot);
  double* ws_d = ws;
  double* ws_c = ws + (size_t)P * Ktot;
  for (int p0 = 0; p0 < P; p0 += FEDAGG_MAX_PAIRWISE) {
    const int pc = (P - p0) < FEDAGG_MAX_PAIRWISE ? (P - p0) : FEDAGG_MAX_PAIRWISE;
    IdxArgs ix;
    memset(&ix, 0, sizeof(ix));
    for (int p = 0; p < pc; ++p) ix.idx[p] = idx[p0 + p];
    hipLaunchKernelGGL((scaffold_tree_kernel<TIn>), dim3(1), dim3(64), 0, s, (const double*)(ws_d + (size_t)p0 * Ktot),
                       ws_c + (size_t)p0 * (Ktot + 1), c, (int64_t)Ktot, ix, pc, lr, dout, cout);
    int rc = check_launch("scaffold_tree_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

template <typename TIn, bool NT, int NTS, int VPT, int SU, bool SPLIT = false, bool PIPE = false, bool BUF = false,
          bool CPF = false, int OCC = 1, int BLK = FA_BLOCK>
void launch_scaffold_variant(unsigned grid, hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a,
                             const PwArgs& pw, int kc, int first, int last, const TIn* c, double lr, uint64_t nvec,
                             uint64_t M, double* dout, double* cout) {
  if (BLK != FA_BLOCK) grid = (grid + BLK / FA_BLOCK - 1) / (BLK / FA_BLOCK);  // the caller sized it for 256
  hipLaunchKernelGGL((scaffold_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, NT, NTS, VPT, SU, SPLIT, PIPE, BUF, CPF, OCC, BLK>),
                     dim3(grid), dim3(BLK), 0, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout, g_xcd, g_tpb);
}

// Scaffold shapes (fedagg_tune "sc_vpt" / "sc_unroll"; nt_load / nt_store shared with FedAvg).

#if FEDAGG_TUNING
template <typename TIn, int VPT, int SU>
void launch_scaffold_bsplit_variant(unsigned grid, hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a,
                                    const PwArgs& pw, int kc, int first, int last, const TIn* c, double lr,
                                    uint64_t nvec, uint64_t M, double* dout, double* cout) {
  hipLaunchKernelGGL((scaffold_bsplit_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, true, true, VPT, SU>), dim3(grid),
                     dim3(FA_BLOCK), 0, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout);
}

// Bucket-split shapes (sc_vpt x sc_unroll); grid = 2 x the tile count (even).
template <typename TIn>
void launch_scaffold_bsplit(unsigned grid, hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a,
                            const PwArgs& pw, int kc, int first, int last, const TIn* c, double lr, uint64_t nvec,
                            uint64_t M, double* dout, double* cout, const int sv, const int su) {
#define SC_ARGS grid, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout
  if (sv >= 8) {
    if (su >= 4) return launch_scaffold_bsplit_variant<TIn, 8, 4>(SC_ARGS);
    return launch_scaffold_bsplit_variant<TIn, 8, 2>(SC_ARGS);
  }
  if (sv >= 4) {
    if (su >= 8) return launch_scaffold_bsplit_variant<TIn, 4, 8>(SC_ARGS);
    return launch_scaffold_bsplit_variant<TIn, 4, 4>(SC_ARGS);
  }
  return launch_scaffold_bsplit_variant<TIn, 2, 8>(SC_ARGS);
#undef SC_ARGS
}

#endif

// Does a Scaffold call walk one bucket per launch (scaffold_bucket_kernel x 2) or both at once?
inline bool scaffold_one_bucket(int K, size_t in_bytes, uint64_t nvec) {
  const bool bsplit = g_sc_bsplit && nvec && g_nt_load && g_nt_store != 0;
  return g_nt_load && (g_sc_2l < 0 ? ((K >= SC_2L_MIN_K || in_bytes == 8) && nvec && !bsplit && g_sc_vpt <= 0)
                                   : g_sc_2l != 0);
}

template <typename TIn, int NTS, int VPT, int SU, bool PIPE = false>
void launch_scaffold_2l_variant(hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a, const PwArgs& pw,
                                int kc, int first, int last, const TIn* c, double lr, uint64_t nvec, uint64_t M,
                                double* dout, double* cout) {
  const unsigned grid = grid_for(nvec ? (nvec + VPT - 1) / VPT : M);
  if (g_sc_2l == 2) {  // one launch, phase-ordered halves
    hipLaunchKernelGGL((scaffold_bucket_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, true, NTS, VPT, SU, 2, PIPE>), dim3(2 * grid),
                       dim3(FA_BLOCK), 0, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout);
    return;
  }
  hipLaunchKernelGGL((scaffold_bucket_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, true, NTS, VPT, SU, 0, PIPE>), dim3(grid),
                     dim3(FA_BLOCK), 0, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout);
  hipLaunchKernelGGL((scaffold_bucket_kernel<TIn, FEDAGG_KCHUNK_SCAFFOLD, true, NTS, VPT, SU, 1, PIPE>), dim3(grid),
                     dim3(FA_BLOCK), 0, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout);
}

#if FEDAGG_TUNING
// One-bucket launch pairs (sc_2l): 4 x 4, 8 x 4, 8 x 2 and 16 x 2 tiles with nt or write-through
// (sc_sc1) stores; plain stores for the 4 x 4 tile only.
template <typename TIn, int NTS>
void launch_scaffold_2l_shape(hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a, const PwArgs& pw, int kc,
                              int first, int last, const TIn* c, double lr, uint64_t nvec, uint64_t M, double* dout,
                              double* cout, const int sv, const int su, const bool pipe) {
#define SC2_ARGS s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout
  if constexpr (NTS == 0) {
    return launch_scaffold_2l_variant<TIn, 0, 4, 4>(SC2_ARGS);
  } else {
    if (pipe) {  // pipelined client groups
      if (sv >= 8) return launch_scaffold_2l_variant<TIn, NTS, 8, 2, true>(SC2_ARGS);
      if (su >= 4) return launch_scaffold_2l_variant<TIn, NTS, 4, 4, true>(SC2_ARGS);
      return launch_scaffold_2l_variant<TIn, NTS, 4, 2, true>(SC2_ARGS);
    }
    if (sv >= 16) {
      if (su <= 1) return launch_scaffold_2l_variant<TIn, NTS, 16, 1>(SC2_ARGS);
      return launch_scaffold_2l_variant<TIn, NTS, 16, 2>(SC2_ARGS);
    }
    if (sv >= 8 && su <= 2) return launch_scaffold_2l_variant<TIn, NTS, 8, 2>(SC2_ARGS);
    if (sv >= 8) return launch_scaffold_2l_variant<TIn, NTS, 8, 4>(SC2_ARGS);
    if (su >= 8) return launch_scaffold_2l_variant<TIn, NTS, 4, 8>(SC2_ARGS);
    return launch_scaffold_2l_variant<TIn, NTS, 4, 4>(SC2_ARGS);
  }
#undef SC2_ARGS
}

#endif

template <typename TIn>
void launch_scaffold_2l(hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a, const PwArgs& pw, int kc,
                        int first, int last, const TIn* c, double lr, uint64_t nvec, uint64_t M, double* dout,
                        double* cout, const int sv, const int su, const bool pipe) {
#if !FEDAGG_TUNING
  // product: fp32 8 x 4 tiles, fp64 pipelined 4 x 2 tiles, nt stores
  (void)sv;
  (void)su;
  (void)pipe;
  if constexpr (sizeof(TIn) == 4)
    launch_scaffold_2l_variant<TIn, 1, 8, 4>(s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout);
  else
    launch_scaffold_2l_variant<TIn, 1, 4, 2, true>(s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout);
#else
  if (g_nt_store == 0)
    launch_scaffold_2l_shape<TIn, 0>(s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout, sv, su, pipe);
  else if (g_sc_sc1)
    launch_scaffold_2l_shape<TIn, 2>(s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout, sv, su, pipe);
  else
    launch_scaffold_2l_shape<TIn, 1>(s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout, sv, su, pipe);
#endif
}

template <typename TIn>
void launch_scaffold(unsigned grid, hipStream_t s, const ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD>& a, const PwArgs& pw,
                     int kc, int first, int last, const TIn* c, double lr, uint64_t nvec, uint64_t M, double* dout,
                     double* cout, const int sv, const int su, const bool buf) {
#define SC_ARGS grid, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout
#if !FEDAGG_TUNING
  // product: 4 x 4 global loads below 32 clients; from 32, fp32 8 x 4 over buffer descriptors,
  // fp64 8 x 2 (the scalar tail of unaligned buckets runs in the same kernels)
  (void)su;
  (void)buf;
  if constexpr (sizeof(TIn) == 4) {
    if (sv >= 8) return launch_scaffold_variant<TIn, true, true, 8, 4, false, false, true>(SC_ARGS);
  } else {
    if (sv >= 8) return launch_scaffold_variant<TIn, true, true, 8, 2>(SC_ARGS);
  }
  return launch_scaffold_variant<TIn, true, true, 4, 4>(SC_ARGS);
#else
  const bool nts = g_nt_store != 0;
  if (!g_nt_load) return launch_scaffold_variant<TIn, false, false, 1, 4>(SC_ARGS);
  if (buf && nts && !g_sc_split && !g_sc_pipe && sizeof(TIn) == 4) {  // buffer-descriptor loads
    if (sv >= 8) {
      if (su >= 4) return launch_scaffold_variant<TIn, true, true, 8, 4, false, false, true>(SC_ARGS);
      return launch_scaffold_variant<TIn, true, true, 8, 2, false, false, true>(SC_ARGS);
    }
    if (sv >= 4) {
      if (su <= 2) return launch_scaffold_variant<TIn, true, true, 4, 2, false, false, true>(SC_ARGS);
      if (g_sc_sc1) return launch_scaffold_variant<TIn, true, 2, 4, 4, false, false, true>(SC_ARGS);
      return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, true>(SC_ARGS);
    }
  }
  if (g_sc_pipe && nts && !g_sc_split) {  // software-pipelined client groups
    if (sv >= 4) return launch_scaffold_variant<TIn, true, true, 4, 2, false, true>(SC_ARGS);
    return launch_scaffold_variant<TIn, true, true, 2, 4, false, true>(SC_ARGS);
  }
  if (g_sc_split && nts) {  // phase-split walk (nt stores)
    if (sv >= 8) {
      if (su <= 2) return launch_scaffold_variant<TIn, true, true, 8, 2, true>(SC_ARGS);
      return launch_scaffold_variant<TIn, true, true, 8, 4, true>(SC_ARGS);
    }
    if (su >= 8) return launch_scaffold_variant<TIn, true, true, 4, 8, true>(SC_ARGS);
    return launch_scaffold_variant<TIn, true, true, 4, 4, true>(SC_ARGS);
  }
  if (sv >= 8) {
    if (su >= 2 && nts) return launch_scaffold_variant<TIn, true, true, 8, 2>(SC_ARGS);
    if (nts) return launch_scaffold_variant<TIn, true, true, 8, 1>(SC_ARGS);
    return launch_scaffold_variant<TIn, true, false, 8, 1>(SC_ARGS);
  }
  if (sv >= 4) {
    if (su <= 2) {
      if (nts) return launch_scaffold_variant<TIn, true, true, 4, 2>(SC_ARGS);
      return launch_scaffold_variant<TIn, true, false, 4, 2>(SC_ARGS);
    }
    if (nts && (g_sc_cpf || g_sc_occ > 1 || g_sc_blk > FA_BLOCK)) {  // 4 x 4 experiments (fedagg_tune)
      const int v = (g_sc_cpf ? 1 : 0) | (g_sc_occ > 1 ? 2 : 0) | (g_sc_blk > FA_BLOCK ? 4 : 0);
      switch (v) {
        case 1: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, true>(SC_ARGS);
        case 2: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, false, 4>(SC_ARGS);
        case 3: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, true, 4>(SC_ARGS);
        case 4: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, false, 1, 512>(SC_ARGS);
        case 5: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, true, 1, 512>(SC_ARGS);
        case 6: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, false, 2, 512>(SC_ARGS);
        default: return launch_scaffold_variant<TIn, true, true, 4, 4, false, false, false, true, 2, 512>(SC_ARGS);
      }
    }
    if (nts && g_sc_sc1) return launch_scaffold_variant<TIn, true, 2, 4, 4>(SC_ARGS);  // write-through stores
    if (nts) return launch_scaffold_variant<TIn, true, true, 4, 4>(SC_ARGS);
    return launch_scaffold_variant<TIn, true, false, 4, 4>(SC_ARGS);
  }
  if (sv >= 2) {
    if (su <= 2) {
      if (nts) return launch_scaffold_variant<TIn, true, true, 2, 2>(SC_ARGS);
      return launch_scaffold_variant<TIn, true, false, 2, 2>(SC_ARGS);
    }
    if (su >= 8 && nts) return launch_scaffold_variant<TIn, true, true, 2, 8>(SC_ARGS);
    if (nts) return launch_scaffold_variant<TIn, true, true, 2, 4>(SC_ARGS);
    return launch_scaffold_variant<TIn, true, false, 2, 4>(SC_ARGS);
  }
  if (su >= 8 && nts) return launch_scaffold_variant<TIn, true, true, 1, 8>(SC_ARGS);
  if (nts) return launch_scaffold_variant<TIn, true, true, 1, 4>(SC_ARGS);
  return launch_scaffold_variant<TIn, true, false, 1, 4>(SC_ARGS);
#endif
#undef SC_ARGS
}

// seed = false: both accumulators start from d_dout / d_cout (partial sums of the clients before
// this block); finish = false: the sums are left as they are (no + c, no lr), c is not read.
template <typename TIn>
int scaffold_launch(const TIn* const* d, const TIn* const* cv, const TIn* c, const double* w, int K, uint64_t M,
                    const uint64_t* idx, int P, void* ws, double lr, double* dout, double* cout, hipStream_t s,
                    bool seed = true, bool finish = true) {
  if (K <= 0) return fail(FEDAGG_EINVAL, "scaffold: K must be > 0 (got %lld)", K);
  if (!d || !cv || (finish && !c) || !w || !dout || !cout) return fail(FEDAGG_EINVAL, "scaffold: NULL argument");
  if (P < 0 || (P > 0 && !idx)) return fail(FEDAGG_EINVAL, "scaffold: bad pairwise index list (P=%lld)", P);
  if (P > 0 && !(seed && finish)) return fail(FEDAGG_EINVAL, "scaffold: pairwise patch needs a whole chain (P=%lld)", P);
  for (int p = 0; p < P; ++p)
    if (idx[p] >= M) return fail(FEDAGG_EINVAL, "scaffold: pairwise index %lld out of range", (long long)idx[p]);
  if (M == 0) return FEDAGG_OK;
  bool vec = (!finish || aligned16(c)) && aligned16(dout) && aligned16(cout);
  for (int k = 0; k < K; ++k) {
    if (!d[k] || !cv[k]) return fail(FEDAGG_EINVAL, "scaffold: client pointer %lld is NULL", k);
    vec = vec && aligned16(d[k]) && aligned16(cv[k]);
  }
  const bool fuse = g_fuse_pw && P <= FEDAGG_FUSED_PAIRWISE && K <= FEDAGG_KCHUNK_SCAFFOLD;
  if (P > 0 && !fuse && !ws) return fail(FEDAGG_EINVAL, "scaffold: workspace needed for %lld pairwise segments", P);
  constexpr int L = 16 / sizeof(TIn);
  const uint64_t nvec = vec ? M / L : 0;
  // launch shape: from 32 clients on (fp32 inputs), 8 vectors x 4-client groups over buffer
  // descriptors (252 VGPRs, 2 waves/SIMD; 64 x 25M 2.00 vs 2.04 ms for 8 x 2 global loads,
  // 48 x 12M 763 vs > 789 us, 32 x 25M 1.113 vs 1.120 ms; profiles/r01_scbuf2_*.log), 4 x 4 global
  // loads below (16 x 25M: 6.23 vs 6.16 TB/s for 8 x 2; profiles/r01_tune3_*.log)
  const bool wide = K >= 32;
  const int sv = g_sc_vpt > 0 ? g_sc_vpt : (wide ? 8 : 4);
  const int su = g_sc_vpt > 0 ? g_sc_unroll : (wide ? (sizeof(TIn) == 4 ? 4 : 2) : 4);
  const bool buf = g_sc_vpt > 0 ? g_sc_buf != 0 : (wide && sizeof(TIn) == 4);
  const uint64_t per_thread = g_nt_load ? (uint64_t)sv : 1;
  unsigned grid = grid_for(nvec ? (nvec + per_thread - 1) / per_thread : M);
  // bucket-split pairs: vector path with nt loads/stores only (the tail is in-kernel)
  const bool bsplit = g_sc_bsplit && nvec && g_nt_load && g_nt_store != 0;
  const bool two = scaffold_one_bucket(K, sizeof(TIn), nvec);
  if (bsplit) grid *= 2;
  else if (g_tpb > 1 && nvec)  // every tile exactly once: no grid cap with tpb
    grid = (unsigned)(((nvec + per_thread - 1) / per_thread + g_tpb - 1) / g_tpb);
  for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK_SCAFFOLD) {
    const int kc = (K - k0) < FEDAGG_KCHUNK_SCAFFOLD ? (K - k0) : FEDAGG_KCHUNK_SCAFFOLD;
    ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) {
      a.d[k] = d[k0 + k];
      a.cv[k] = cv[k0 + k];
      a.w[k] = w[k0 + k];
    }
    PwArgs pw;
    memset(&pw, 0, sizeof(pw));
    if (fuse) {
      pw.n = P;
      for (int p = 0; p < P; ++p) pw.idx[p] = idx[p];
    }
    const int first = k0 == 0 && seed, last = (k0 + kc) == K && finish;
    // fp64 inputs: software-pipelined 4 x 2 tiles (16 x 25M: 1.178 ms, against 1.409 fused, 1.340
    // for the best unpipelined one-bucket tile; the fp32 one-bucket tiles lose 11-20 % pipelined)
    if (two)
      launch_scaffold_2l<TIn>(s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout,
                              g_sc_vpt > 0 ? g_sc_vpt : (sizeof(TIn) == 4 ? 8 : 4),
                              g_sc_vpt > 0 ? g_sc_unroll : (sizeof(TIn) == 4 ? 4 : 2),
                              g_sc_vpt > 0 ? g_sc_pipe != 0 : sizeof(TIn) == 8);
#if FEDAGG_TUNING
    else if (bsplit)
      launch_scaffold_bsplit<TIn>(grid, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout, sv, su);
#endif
    else
      launch_scaffold<TIn>(grid, s, a, pw, kc, first, last, c, lr, nvec, M, dout, cout, sv, su, buf);
    int rc = check_launch("scaffold_kernel");
    if (rc) return rc;
  }
  if (P > 0 && !fuse) return scaffold_pairwise_launch<TIn>(d, cv, c, w, K, idx, P, lr, ws, dout, cout, s);
  return FEDAGG_OK;
}

template <typename T>
int equal_launch(const T* const* x, int K, uint64_t M, unsigned long long* cnt, hipStream_t s) {
  if (K <= 0 || !x || !cnt) return fail(FEDAGG_EINVAL, "equal_count: invalid argument (K=%lld)", K);
  if (M == 0 || K == 1) return FEDAGG_OK;
  bool vec = g_eq_vec != 0;
  for (int k = 0; k < K; ++k) {
    if (!x[k]) return fail(FEDAGG_EINVAL, "equal_count: client pointer %lld is NULL", k);
    vec = vec && aligned16(x[k]);
  }
  constexpr int EQ_VPT = 4;
  const uint64_t nvec = vec ? M / (16 / sizeof(T)) : 0;
  const unsigned grid = vec ? grid_for((nvec + EQ_VPT - 1) / EQ_VPT) : grid_for(M);
  for (int k0 = 1; k0 < K; k0 += FEDAGG_KCHUNK) {
    const int kc = (K - k0) < FEDAGG_KCHUNK ? (K - k0) : FEDAGG_KCHUNK;
    EqArgs<T, FEDAGG_KCHUNK> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) a.x[k] = x[k0 + k];
    if (vec)
      hipLaunchKernelGGL((equal_count_vec_kernel<T, FEDAGG_KCHUNK, EQ_VPT>), dim3(grid), dim3(FA_BLOCK), 0, s, a, kc,
                         x[0], nvec, M, cnt);
    else
      hipLaunchKernelGGL((equal_count_kernel<T, FEDAGG_KCHUNK>), dim3(grid), dim3(FA_BLOCK), 0, s, a, kc, x[0], M,
                         cnt);
    int rc = check_launch("equal_count_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}

template <typename T>
const T* cptr(const void* p) {
  return static_cast<const T*>(p);
}

}  // namespace

namespace fedagg_internal {
void set_error(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }
}  // namespace fedagg_internal

// ======================================================================================
// C ABI
// ======================================================================================
extern "C" {

int fedagg_abi_version(void) { return FEDAGG_ABI_VERSION; }

int fedagg_scaffold_launches(int K, int in_elem_bytes, uint64_t M, int aligned) {
  if (K <= 0 || (in_elem_bytes != 4 && in_elem_bytes != 8))
    return fail(FEDAGG_EINVAL, "scaffold_launches: bad K or element bytes (K=%lld; element bytes must be 4 or 8)",
                (long long)K);
  const uint64_t nvec = aligned ? M / (16 / (uint64_t)in_elem_bytes) : 0;
  return scaffold_one_bucket(K, (size_t)in_elem_bytes, nvec) ? 2 : 1;
}
const char* fedagg_last_error(void) { return g_err; }

int fedagg_tune(const char* key, long long value) {
  if (!key) return fail(FEDAGG_EINVAL, "fedagg_tune: NULL key");
  // knobs of the product build: they choose among the shapes it holds
  if (!strcmp(key, "grid_cap")) g_grid_cap = (int)value;
  else if (!strcmp(key, "fuse_pairwise")) g_fuse_pw = value ? 1 : 0;
  else if (!strcmp(key, "eq_vec")) g_eq_vec = value ? 1 : 0;
  else if (!strcmp(key, "flat_vec")) g_flat_vec = value ? 1 : 0;
  else if (!strcmp(key, "st_sc1")) g_st_sc1 = value < 0 ? -1 : (value ? 1 : 0);
  else if (!strcmp(key, "tiled_few")) g_tiled_few = value ? 1 : 0;
  else if (!strcmp(key, "sc_2l") && value <= 1) g_sc_2l = value < 0 ? -1 : (value == 0 ? 0 : 1);
#if FEDAGG_TUNING
  // experiment knobs (measured, not kept: DESIGN.md §5, §8, §9)
  else if (!strcmp(key, "sc_2l")) g_sc_2l = 2;
  else if (!strcmp(key, "nt_load")) g_nt_load = value ? 1 : 0;
  else if (!strcmp(key, "nt_store")) g_nt_store = value < 0 ? -1 : (value ? 1 : 0);
  else if (!strcmp(key, "vpt"))
    g_vpt = value <= 0 ? 0 : value >= 16 ? 16 : value >= 8 ? 8 : (value >= 4 ? 4 : (value >= 2 ? 2 : 1));
  else if (!strcmp(key, "unroll"))
    g_unroll = value >= 16 ? 16 : (value <= 1 ? 1 : value <= 2 ? 2 : (value <= 4 ? 4 : 8));
  else if (!strcmp(key, "pipe")) g_pipe = value ? 1 : 0;
  else if (!strcmp(key, "tile")) g_tile = value ? 1 : 0;
  else if (!strcmp(key, "sc_vpt")) g_sc_vpt = value <= 0 ? 0 : value >= 8 ? 8 : (value >= 4 ? 4 : (value >= 2 ? 2 : 1));
  else if (!strcmp(key, "sc_unroll")) g_sc_unroll = value <= 1 ? 1 : value <= 2 ? 2 : (value >= 8 ? 8 : 4);
  else if (!strcmp(key, "sc_split")) g_sc_split = value ? 1 : 0;
  else if (!strcmp(key, "sc_buf")) g_sc_buf = value ? 1 : 0;
  else if (!strcmp(key, "sc_bsplit")) g_sc_bsplit = value ? 1 : 0;
  else if (!strcmp(key, "buf")) g_buf = value ? 1 : 0;
  else if (!strcmp(key, "fa_occ")) g_fa_occ = value <= 1 ? 0 : (value >= 4 ? 4 : (int)value);
  else if (!strcmp(key, "xcd")) g_xcd = value ? 1 : 0;
  else if (!strcmp(key, "sc_pipe")) g_sc_pipe = value ? 1 : 0;
  else if (!strcmp(key, "tpb")) g_tpb = value < 1 ? 1 : (value > 64 ? 64 : (int)value);
  else if (!strcmp(key, "sc_cpf")) g_sc_cpf = value ? 1 : 0;
  else if (!strcmp(key, "sc_occ")) g_sc_occ = value <= 1 ? 0 : (int)value;
  else if (!strcmp(key, "sc_blk")) g_sc_blk = value >= 512 ? 512 : 256;
  else if (!strcmp(key, "sc_sc1")) g_sc_sc1 = value ? 1 : 0;
  else if (!strcmp(key, "fa_blk")) g_fa_blk = value <= 0 ? 0 : (value >= 1024 ? 1024 : (value >= 512 ? 512 : 256));
#endif
  else return fail(FEDAGG_EINVAL, "fedagg_tune: unknown key, or an experiment knob of a FEDAGG_TUNING build");
  return FEDAGG_OK;
}

int fedagg_tuning_build(void) { return FEDAGG_TUNING; }

size_t fedagg_pairwise_ws_bytes(int K, int P, int elem_bytes) {
  (void)P;
  (void)elem_bytes;
  if (K <= 0) return 0;
  // per launch chunk: up to FEDAGG_MAX_PAIRWISE segments x (K + 1) terms, two buckets, 8-B terms
  return (size_t)2 * FEDAGG_MAX_PAIRWISE * (size_t)(K + 1) * 8;
}

int fedagg_fedavg_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M, const uint64_t* h_idx,
                      int P, void* d_ws, float* d_out, void* stream) {
  return fedavg_launch<F32>(d_clients, h_w, K, M, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M, const uint64_t* h_idx,
                       int P, void* d_ws, float* d_out, void* stream) {
  return fedavg_launch<BF16>(d_clients, h_w, K, M, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
uint64_t fedagg_fedavg_tile_vectors_f32(int K, uint64_t M) { return tiled_tile_vectors<F32>(K, M); }
uint64_t fedagg_fedavg_tile_vectors_bf16(int K, uint64_t M) { return tiled_tile_vectors<BF16>(K, M); }
int fedagg_fedavg_tiled_f32(const float* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                            const uint64_t* h_idx, int P, void* d_ws, float* d_out, void* stream) {
  return fedavg_tiled_launch<F32>(d_base, h_w, K, M, tile_vectors, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_tiled_bf16(const uint16_t* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                             const uint64_t* h_idx, int P, void* d_ws, float* d_out, void* stream) {
  return fedavg_tiled_launch<BF16>(d_base, h_w, K, M, tile_vectors, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_f64(const double* const* d_clients, const double* h_w, int K, uint64_t M, const uint64_t* h_idx,
                      int P, void* d_ws, double* d_out, void* stream) {
  return fedavg_launch<F64>(d_clients, h_w, K, M, h_idx, P, d_ws, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, uint64_t M,
                      const uint64_t* h_idx, int P, void* d_ws, uint16_t* d_out, void* stream) {
  if (!h_w || K <= 0) return fail(FEDAGG_EINVAL, "fedavg_f16: invalid weights (K=%lld)", K);
  // weights travel as fp16 bit patterns: same bytes as _Float16
  return fedavg_launch<F16>(d_clients, reinterpret_cast<const _Float16*>(h_w), K, M, h_idx, P, d_ws, d_out,
                            (hipStream_t)stream);
}

int fedagg_scaffold_f32(const float* const* d_delta, const float* const* d_cv, const float* d_c, const double* h_w,
                        int K, uint64_t M, const uint64_t* h_idx, int P, void* d_ws, double lr, double* d_delta_out,
                        double* d_c_out, void* stream) {
  return scaffold_launch<float>(d_delta, d_cv, d_c, h_w, K, M, h_idx, P, d_ws, lr, d_delta_out, d_c_out,
                                (hipStream_t)stream);
}
int fedagg_scaffold_f64(const double* const* d_delta, const double* const* d_cv, const double* d_c,
                        const double* h_w, int K, uint64_t M, const uint64_t* h_idx, int P, void* d_ws, double lr,
                        double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_launch<double>(d_delta, d_cv, d_c, h_w, K, M, h_idx, P, d_ws, lr, d_delta_out, d_c_out,
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

int fedagg_flat_gather_f32(const float* const* d_layers, const uint64_t* numel, int L, float* d_flat,
                           void* stream) {
  return flat_seg_launch<0>(reinterpret_cast<const void* const*>(d_layers), nullptr, 1, nullptr, numel, L, d_flat,
                            FEDAGG_F32, (hipStream_t)stream);
}
int fedagg_flat_scatter_f32(float* const* d_layers, const uint64_t* numel, int L, const float* d_flat, void* stream) {
  return flat_seg_launch<1>(reinterpret_cast<const void* const*>(d_layers), nullptr, 1, nullptr, numel, L,
                            const_cast<float*>(d_flat), FEDAGG_F32, (hipStream_t)stream);
}
int fedagg_flat_wsum_f32(const float* const* d_layers, int nlists, const double* coeffs, const uint64_t* numel, int L,
                         float* d_flat, void* stream) {
  return flat_seg_launch<2>(reinterpret_cast<const void* const*>(d_layers), nullptr, nlists, coeffs, numel, L, d_flat,
                            FEDAGG_F32, (hipStream_t)stream);
}
int fedagg_flat_increment_f32(float* const* d_layers, const uint64_t* numel, int L, const float* d_flat,
                              double multiplier, void* stream) {
  return flat_seg_launch<3>(reinterpret_cast<const void* const*>(d_layers), nullptr, 1, &multiplier, numel, L,
                            const_cast<float*>(d_flat), FEDAGG_F32, (hipStream_t)stream);
}
int fedagg_flat_gather(const void* const* d_layers, int kind, const uint64_t* numel, int L, void* d_flat,
                       void* stream) {
  return flat_seg_launch<0>(d_layers, &kind, 1, nullptr, numel, L, d_flat, kind, (hipStream_t)stream);
}
int fedagg_flat_wsum(const void* const* d_layers, const int* kinds, int nlists, const double* coeffs,
                     const uint64_t* numel, int L, void* d_flat, int flat_kind, void* stream) {
  return flat_seg_launch<2>(d_layers, kinds, nlists, coeffs, numel, L, d_flat, flat_kind, (hipStream_t)stream);
}
int fedagg_flat_increment(float* const* d_layers, const uint64_t* numel, int L, const void* d_flat, int flat_kind,
                          double multiplier, void* stream) {
  return flat_seg_launch<3>(reinterpret_cast<const void* const*>(d_layers), nullptr, 1, &multiplier, numel, L,
                            const_cast<void*>(d_flat), flat_kind, (hipStream_t)stream);
}

static bool is_float_kind(int k) { return k == FEDAGG_F16 || k == FEDAGG_F32 || k == FEDAGG_F64; }

int fedagg_cast(const void* d_in, int in_kind, void* d_out, int out_kind, uint64_t n, void* stream) {
  if (!d_in || !d_out || in_kind < 0 || in_kind > FEDAGG_BOOL || !is_float_kind(out_kind))
    return fail(FEDAGG_EINVAL, "fedagg_cast: unsupported kinds (out %lld)", out_kind);
  if (n == 0) return FEDAGG_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(FA_BLOCK), 0, (hipStream_t)stream, d_in, in_kind, d_out,
                     out_kind, n);
  return check_launch("cast_kernel");
}

int fedagg_scale_cast(const void* d_in, int in_kind, double w, void* d_out, int out_kind, uint64_t n, void* stream) {
  if (!d_in || !d_out || !is_float_kind(in_kind) || !is_float_kind(out_kind))
    return fail(FEDAGG_EINVAL, "fedagg_scale_cast: float kinds only (in %lld)", in_kind);
  if (n == 0) return FEDAGG_OK;
  hipLaunchKernelGGL(scale_cast_kernel, dim3(grid_for(n)), dim3(FA_BLOCK), 0, (hipStream_t)stream, d_in, in_kind, w,
                     d_out, out_kind, n);
  return check_launch("scale_cast_kernel");
}

// ---- client-sharded building blocks (chain / partial sums / split pairwise trees) ----
int fedagg_fedavg_chain_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M, int seed,
                            float* d_out, void* stream) {
  return fedavg_launch<F32>(d_clients, h_w, K, M, nullptr, 0, nullptr, d_out, (hipStream_t)stream, seed != 0);
}
// Push runs: d_in (this rank's accumulator slot, fp32; NULL = start from +0.0) continued by the
// block's clients in order, written to d_out (a peer's mapped slot or the root's output) with
// system-scope write-through stores, every wave waiting for their acknowledgements.
extern "C++" template <typename E>
int fedavg_push_launch(const typename E::In* const* d_clients, const typename E::P* h_w, int K, uint64_t M,
                       const float* d_in, float* d_out, hipStream_t s) {
  if (d_in && (!aligned16(d_in) || !aligned16(d_out)))
    return fail(FEDAGG_EINVAL, "fedavg_chain_push: accumulators must be 16-B aligned (K=%lld)", K);
  g_rel_sys = 1;
  g_acc_in = d_in;
  const int rc = fedavg_launch<E>(d_clients, h_w, K, M, nullptr, 0, nullptr, d_out, s, d_in == nullptr);
  g_rel_sys = 0;
  g_acc_in = nullptr;
  return rc;
}
int fedagg_fedavg_chain_push_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M,
                                 const float* d_in, float* d_out, void* stream) {
  return fedavg_push_launch<F32>(d_clients, h_w, K, M, d_in, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_chain_push_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M,
                                  const float* d_in, float* d_out, void* stream) {
  return fedavg_push_launch<BF16>(d_clients, h_w, K, M, d_in, d_out, (hipStream_t)stream);
}
int fedagg_fedavg_chain_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M, int seed,
                             float* d_out, void* stream) {
  return fedavg_launch<BF16>(d_clients, h_w, K, M, nullptr, 0, nullptr, d_out, (hipStream_t)stream, seed != 0);
}
int fedagg_fedavg_chain_f64(const double* const* d_clients, const double* h_w, int K, uint64_t M, int seed,
                            double* d_out, void* stream) {
  return fedavg_launch<F64>(d_clients, h_w, K, M, nullptr, 0, nullptr, d_out, (hipStream_t)stream, seed != 0);
}
int fedagg_fedavg_chain_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, uint64_t M, int seed,
                            uint16_t* d_out, void* stream) {
  if (!h_w || K <= 0) return fail(FEDAGG_EINVAL, "fedavg_chain_f16: invalid weights (K=%lld)", K);
  return fedavg_launch<F16>(d_clients, reinterpret_cast<const _Float16*>(h_w), K, M, nullptr, 0, nullptr, d_out,
                            (hipStream_t)stream, seed != 0);
}

int fedagg_fedavg_chain_tiled_f32(const float* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                                  int seed, float* d_out, void* stream) {
  return fedavg_tiled_launch<F32>(d_base, h_w, K, M, tile_vectors, nullptr, 0, nullptr, d_out, (hipStream_t)stream,
                                  seed != 0);
}
int fedagg_fedavg_chain_tiled_bf16(const uint16_t* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                                   int seed, float* d_out, void* stream) {
  return fedavg_tiled_launch<BF16>(d_base, h_w, K, M, tile_vectors, nullptr, 0, nullptr, d_out, (hipStream_t)stream,
                                   seed != 0);
}

int fedagg_pairwise_products_f32(const float* const* d_clients, const float* h_w, int K, const uint64_t* h_idx,
                                 int P, int64_t stride, int kbase, float* d_ws, void* stream) {
  return pairwise_products_launch<F32>(d_clients, h_w, K, h_idx, P, stride, kbase, d_ws, (hipStream_t)stream);
}
int fedagg_pairwise_products_bf16(const uint16_t* const* d_clients, const float* h_w, int K, const uint64_t* h_idx,
                                  int P, int64_t stride, int kbase, float* d_ws, void* stream) {
  return pairwise_products_launch<BF16>(d_clients, h_w, K, h_idx, P, stride, kbase, d_ws, (hipStream_t)stream);
}
int fedagg_pairwise_products_f64(const double* const* d_clients, const double* h_w, int K, const uint64_t* h_idx,
                                 int P, int64_t stride, int kbase, double* d_ws, void* stream) {
  return pairwise_products_launch<F64>(d_clients, h_w, K, h_idx, P, stride, kbase, d_ws, (hipStream_t)stream);
}
int fedagg_pairwise_products_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, const uint64_t* h_idx,
                                 int P, int64_t stride, int kbase, float* d_ws, void* stream) {
  if (!h_w || K <= 0) return fail(FEDAGG_EINVAL, "pairwise_products_f16: invalid weights (K=%lld)", K);
  return pairwise_products_launch<F16>(d_clients, reinterpret_cast<const _Float16*>(h_w), K, h_idx, P, stride, kbase,
                                       d_ws, (hipStream_t)stream);
}
int fedagg_pairwise_finish_f32(const float* d_ws, int64_t n, int64_t stride, const uint64_t* h_idx, int P,
                               float* d_out, void* stream) {
  return pairwise_finish_launch<F32>(d_ws, n, stride, h_idx, P, d_out, (hipStream_t)stream);
}
int fedagg_pairwise_finish_f64(const double* d_ws, int64_t n, int64_t stride, const uint64_t* h_idx, int P,
                               double* d_out, void* stream) {
  return pairwise_finish_launch<F64>(d_ws, n, stride, h_idx, P, d_out, (hipStream_t)stream);
}
int fedagg_pairwise_finish_f16(const float* d_ws, int64_t n, int64_t stride, const uint64_t* h_idx, int P,
                               uint16_t* d_out, void* stream) {
  return pairwise_finish_launch<F16>(d_ws, n, stride, h_idx, P, d_out, (hipStream_t)stream);
}

int fedagg_scaffold_chain_f32(const float* const* d_delta, const float* const* d_cv, const float* d_c,
                              const double* h_w, int K, uint64_t M, int seed, int finish, double lr,
                              double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_launch<float>(d_delta, d_cv, d_c, h_w, K, M, nullptr, 0, nullptr, lr, d_delta_out, d_c_out,
                                (hipStream_t)stream, seed != 0, finish != 0);
}
int fedagg_scaffold_chain_f64(const double* const* d_delta, const double* const* d_cv, const double* d_c,
                              const double* h_w, int K, uint64_t M, int seed, int finish, double lr,
                              double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_launch<double>(d_delta, d_cv, d_c, h_w, K, M, nullptr, 0, nullptr, lr, d_delta_out, d_c_out,
                                 (hipStream_t)stream, seed != 0, finish != 0);
}
// Scaffold push runs: one bucket (phase 0: delta, phase 1: control variate) of a client block,
// d_in (this rank's fp64 accumulator slot; NULL = from +0.0) continued by the block's K rows into
// d_out (a peer's mapped slot or the root's output); finish: x lr (phase 0) or + d_c (phase 1).
// The tiles of the product's one-bucket launches (fp32 8 x 4, fp64 pipelined 4 x 2).
extern "C++" template <typename TIn>
int scaffold_push_launch(const TIn* const* d_rows, const double* h_w, int K, uint64_t M, int phase, const TIn* d_c,
                         double lr, int finish, const double* d_in, double* d_out, hipStream_t s) {
  if (K <= 0 || !d_rows || !h_w || !d_out || (phase != 0 && phase != 1) || (finish && phase == 1 && !d_c))
    return fail(FEDAGG_EINVAL, "scaffold_chain_push: invalid argument (K=%lld)", K);
  if (M == 0) return FEDAGG_OK;
  bool vec = aligned16(d_out) && (!d_in || aligned16(d_in)) && (!(finish && phase == 1) || aligned16(d_c));
  for (int k = 0; k < K; ++k) {
    if (!d_rows[k]) return fail(FEDAGG_EINVAL, "scaffold_chain_push: client pointer %lld is NULL", k);
    vec = vec && aligned16(d_rows[k]);
  }
  constexpr int L = 16 / sizeof(TIn);
  constexpr int VPT = sizeof(TIn) == 4 ? 8 : 4, SU = sizeof(TIn) == 4 ? 4 : 2;
  constexpr bool PIPE = sizeof(TIn) == 8;
  const uint64_t nvec = vec ? M / L : 0;
  const unsigned grid = grid_for(nvec ? (nvec + VPT - 1) / VPT : M);
  for (int k0 = 0; k0 < K; k0 += FEDAGG_KCHUNK_SCAFFOLD) {
    const int kc = (K - k0) < FEDAGG_KCHUNK_SCAFFOLD ? (K - k0) : FEDAGG_KCHUNK_SCAFFOLD;
    ScArgs<TIn, FEDAGG_KCHUNK_SCAFFOLD> a;
    memset(&a, 0, sizeof(a));
    for (int k = 0; k < kc; ++k) {
      a.d[k] = d_rows[k0 + k];
      a.cv[k] = d_rows[k0 + k];
      a.w[k] = h_w[k0 + k];
    }
    const int first = k0 == 0 && !d_in, last = (k0 + kc) == K && finish;
    const bool sep = k0 == 0 && d_in;  // later chunks continue the output itself
#define SCP(PH, SEP)                                                                                            \
  hipLaunchKernelGGL((scaffold_push_kernel<TIn, VPT, SU, PH, PIPE, SEP>), dim3(grid), dim3(FA_BLOCK), 0, s, a, kc, \
                     first, last, d_c, lr, nvec, M, d_in, d_out)
    if (phase == 0) {
      if (sep) SCP(0, true);
      else SCP(0, false);
    } else {
      if (sep) SCP(1, true);
      else SCP(1, false);
    }
#undef SCP
    const int rc = check_launch("scaffold_push_kernel");
    if (rc) return rc;
  }
  return FEDAGG_OK;
}
int fedagg_scaffold_chain_push_f32(const float* const* d_rows, const double* h_w, int K, uint64_t M, int phase,
                                   const float* d_c, double lr, int finish, const double* d_in, double* d_out,
                                   void* stream) {
  return scaffold_push_launch<float>(d_rows, h_w, K, M, phase, d_c, lr, finish, d_in, d_out, (hipStream_t)stream);
}
int fedagg_scaffold_chain_push_f64(const double* const* d_rows, const double* h_w, int K, uint64_t M, int phase,
                                   const double* d_c, double lr, int finish, const double* d_in, double* d_out,
                                   void* stream) {
  return scaffold_push_launch<double>(d_rows, h_w, K, M, phase, d_c, lr, finish, d_in, d_out, (hipStream_t)stream);
}
int fedagg_scaffold_products_f32(const float* const* d_delta, const float* const* d_cv, const double* h_w, int K,
                                 int kbase, int Ktot, const uint64_t* h_idx, int P, double* d_ws, void* stream) {
  return scaffold_products_launch<float>(d_delta, d_cv, h_w, K, kbase, Ktot, h_idx, P, d_ws, (hipStream_t)stream);
}
int fedagg_scaffold_products_f64(const double* const* d_delta, const double* const* d_cv, const double* h_w, int K,
                                 int kbase, int Ktot, const uint64_t* h_idx, int P, double* d_ws, void* stream) {
  return scaffold_products_launch<double>(d_delta, d_cv, h_w, K, kbase, Ktot, h_idx, P, d_ws, (hipStream_t)stream);
}
int fedagg_scaffold_finish_f32(double* d_ws, int Ktot, const float* d_c, const uint64_t* h_idx, int P, double lr,
                               double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_finish_launch<float>(d_ws, Ktot, d_c, h_idx, P, lr, d_delta_out, d_c_out, (hipStream_t)stream);
}
int fedagg_scaffold_finish_f64(double* d_ws, int Ktot, const double* d_c, const uint64_t* h_idx, int P, double lr,
                               double* d_delta_out, double* d_c_out, void* stream) {
  return scaffold_finish_launch<double>(d_ws, Ktot, d_c, h_idx, P, lr, d_delta_out, d_c_out, (hipStream_t)stream);
}

int fedagg_read_probe_f32(const float* d_x, uint64_t M, float* d_sink, int grid, void* stream) {
  if (!d_x || !d_sink || grid <= 0 || !aligned16(d_x)) return fail(FEDAGG_EINVAL, "read_probe: invalid argument");
  hipLaunchKernelGGL(read_probe_kernel, dim3(grid), dim3(FA_BLOCK), 0, (hipStream_t)stream, d_x, M / 4, d_sink);
  return check_launch("read_probe_kernel");
}

int fedagg_read_probe_tile_f32(const float* d_x, uint64_t M, float* d_sink, int vpt, void* stream) {
  if (!d_x || !d_sink || !aligned16(d_x) || M < 4 || (vpt != 4 && vpt != 8 && vpt != 16))
    return fail(FEDAGG_EINVAL, "read_probe_tile: invalid argument");
  const uint64_t nvec = M / 4, tile = (uint64_t)vpt * FA_BLOCK, grid = (nvec + tile - 1) / tile;
  if (grid > 0x7fffffffull) return fail(FEDAGG_EINVAL, "read_probe_tile: buffer too large");
  hipStream_t s = (hipStream_t)stream;
  if (vpt == 4) hipLaunchKernelGGL(read_probe_tile_kernel<4>, dim3(grid), dim3(FA_BLOCK), 0, s, (const u32x4*)d_x, nvec, d_sink);
  if (vpt == 8) hipLaunchKernelGGL(read_probe_tile_kernel<8>, dim3(grid), dim3(FA_BLOCK), 0, s, (const u32x4*)d_x, nvec, d_sink);
  if (vpt == 16) hipLaunchKernelGGL(read_probe_tile_kernel<16>, dim3(grid), dim3(FA_BLOCK), 0, s, (const u32x4*)d_x, nvec, d_sink);
  return check_launch("read_probe_tile_kernel");
}

}  // extern "C"
