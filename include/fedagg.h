/*
 * fedagg.h -- C ABI of the MI355X (gfx950) aggregation engine for SubstraFL's
 * federated-strategy hot path.
 *
 * The reference has no native code: its hot path is NumPy called from Python
 * (SURVEY.md §2.3).  Each entry point below replaces one arithmetic step of the
 * reference and names the lines it replaces.  The Python host side
 * (substrafl_amd/_native.py, ctypes) is what binds them; INTEGRATION.md shows the
 * binding a SubstraFL maintainer would add.
 *
 * Conventions
 *   - All pointers named d_* are device (HBM) pointers owned by the caller.
 *   - Pointer tables (const T* const* d_clients) and weight vectors (h_w*) are
 *     HOST arrays of K entries; the library copies them into kernel arguments
 *     (chunks of FEDAGG_KCHUNK clients), so nothing is allocated and every call is
 *     capturable into a hipGraph.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream).  Every call is
 *     asynchronous on that stream.
 *   - Return value: 0 on success, a negative FEDAGG_E* code otherwise;
 *     fedagg_last_error() gives the message of the calling thread's last failure.
 *   - Arithmetic is bit-exact with the reference NumPy path (no FMA contraction,
 *     client order preserved, IEEE round-to-nearest-even, denormals kept).
 */
#ifndef FEDAGG_H
#define FEDAGG_H

#include <stddef.h>
#include <stdint.h>

/* 1 when building the tuning library (__graft_entry__.build(tuning=True)); the product is 0 */
#ifndef FEDAGG_TUNING
#define FEDAGG_TUNING 0
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define FEDAGG_ABI_VERSION 17
#define FEDAGG_KCHUNK 128          /* clients per launch for FedAvg (kernel-argument table)      */
#define FEDAGG_KCHUNK_SCAFFOLD 64  /* clients per launch for Scaffold (two tables)               */
#define FEDAGG_FUSED_PAIRWISE 16   /* numel==1 segments patched inside the bucket launch         */
#define FEDAGG_MAX_PAIRWISE 64     /* numel==1 segments per launch of the separate pairwise path */

enum {
  FEDAGG_OK = 0,
  FEDAGG_EINVAL = -1, /* bad argument (K <= 0, NULL pointer, index out of range, ...) */
  FEDAGG_EHIP = -2,   /* a HIP runtime call failed                                    */
};

int fedagg_abi_version(void);
const char* fedagg_last_error(void);
/* Process-wide launch knobs (defaults are the values measured best on MI355X).  The product
 * library takes the knobs that choose among the shapes it holds:
 *   "grid_cap"      workgroups per launch before the kernels grid-stride (<= 0: no cap)
 *   "fuse_pairwise" patch numel==1 tensors inside the bucket launch (0/1)
 *   "eq_vec"        16-B loads in the c-equality check (0/1)      "flat_vec"  16-B client flat ops (0/1)
 *   "st_sc1"        FedAvg output stores as write-through (sc1) stores (-1 auto: below 32 clients)
 *   "sc_2l"         Scaffold: 1 = one bucket per launch, 0 = both buckets in one walk, -1 = auto
 *   "tiled_few"     recommend tile-interleaved buckets below 32 fp32 clients too (0/1)
 * A library built with -DFEDAGG_TUNING=1 (fedagg_tuning_build() == 1) also instantiates every
 * variant DESIGN.md records as measured and not kept, selected by the experiment knobs "nt_load",
 * "nt_store", "vpt", "unroll", "pipe", "tile", "xcd", "tpb", "buf", "fa_occ", "fa_blk", "sc_vpt",
 * "sc_unroll", "sc_split", "sc_bsplit", "sc_buf", "sc_pipe", "sc_cpf", "sc_occ", "sc_blk",
 * "sc_sc1" and "sc_2l" = 2; the product library refuses them.
 * Returns FEDAGG_EINVAL for an unknown (or, in the product library, an experiment) key. */
int fedagg_tune(const char* key, long long value);
/* 1 in a FEDAGG_TUNING build (every experiment variant instantiated), 0 in the product library. */
int fedagg_tuning_build(void);

/* Workspace for the separate numel==1 path, needed only when it cannot be fused
 * (K > FEDAGG_KCHUNK (FedAvg) / FEDAGG_KCHUNK_SCAFFOLD (Scaffold), or P > FEDAGG_FUSED_PAIRWISE). */
size_t fedagg_pairwise_ws_bytes(int K, int P, int elem_bytes);

/* ---------------------------------------------------------------------------
 * FedAvg bucket reduction.
 * Replaces substrafl/strategies/fed_avg.py:217-222
 *     states = [x_k * (n_k / n) for k]; np.sum(states, axis=0)
 * for every element of a flat bucket of M elements:
 *     acc = +0.0;  for k in 0..K-1 (list order):  acc = fl(acc + fl(x_k[i] * w_k))
 * where h_w[k] = fl(n_k / n) (computed by the caller in double and rounded to the
 * product type, fed_avg.py:221).
 * numel == 1 tensors: np.sum(list, axis=0) reduces those along the contiguous axis, i.e.
 *     out = +0.0 + pairwise_sum(p_0 .. p_{K-1})
 * with NumPy's 8-accumulator / 128-block pairwise tree.  h_idx lists
 * the P flat indices of such elements (may be NULL when P == 0); d_ws is a device workspace
 * of fedagg_pairwise_ws_bytes() bytes, only read when the patch cannot be fused (may be NULL
 * otherwise).
 * -------------------------------------------------------------------------*/
int fedagg_fedavg_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M, const uint64_t* h_idx,
                      int P, void* d_ws, float* d_out, void* stream);
/* bf16 client buckets, fp32 product/accumulate/output: bit-identical to the reference
 * run on the exact fp32 upcast (the reference itself cannot carry bf16:
 * torch_fed_avg_algo.py:229 `.numpy()` raises on BFloat16). */
int fedagg_fedavg_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M, const uint64_t* h_idx,
                       int P, void* d_ws, float* d_out, void* stream);
/* Tile-interleaved buckets (same arithmetic, same results, another HBM layout).  With the row
 * layout above the K client streams of a workgroup step lie a bucket row apart; interleaving
 * the clients' tiles -- tile t of client k at 16-B vector (t * K + k) * T of d_base, every tile
 * T vectors, the last one padded -- makes a workgroup step read one contiguous K x T region
 * (64 x 125M fp32: 1.7 %, 128 x 175M: 3 % faster in tools/c3_layout_probe.hip).  Element i of
 * client k: vector v = i / L (L = 4 fp32, 8 bf16), at ((v / T) * K + k) * T + v % T, lane i % L.
 * T is one of the tiles the tiled kernels walk (FEDAGG_TILE_VECTORS_*: the tiles of the row
 * layout's kernels from 32 clients over large buckets, and below 32 fp32 clients); any K and M
 * are accepted.  The layout is recommended
 * where fedagg_fedavg_tile_vectors_*(K, M) returns T (0: keep the row layout, whose kernel for
 * that shape walks another tile).  Buffer: ceil(ceil(M / L) / T) * K * T * 16 bytes. */
#define FEDAGG_TILE_VECTORS_F32 8192  /* 16 vectors x 512 threads: 128 KiB of fp32 per client */
#define FEDAGG_TILE_VECTORS_F32_FEW 2048 /* 8 x 256 (the row layout's tile below 32 clients): 32 KiB */
#define FEDAGG_TILE_VECTORS_BF16 4096 /* 16 vectors x 256 threads: 64 KiB of bf16 per client  */
uint64_t fedagg_fedavg_tile_vectors_f32(int K, uint64_t M);
uint64_t fedagg_fedavg_tile_vectors_bf16(int K, uint64_t M);
int fedagg_fedavg_tiled_f32(const float* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                            const uint64_t* h_idx, int P, void* d_ws, float* d_out, void* stream);
int fedagg_fedavg_tiled_bf16(const uint16_t* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                             const uint64_t* h_idx, int P, void* d_ws, float* d_out, void* stream);
/* fp64 buckets (also integer layers after an exact cast: x_int * python_float is a
 * float64 ufunc loop in NumPy). */
int fedagg_fedavg_f64(const double* const* d_clients, const double* h_w, int K, uint64_t M, const uint64_t* h_idx,
                      int P, void* d_ws, double* d_out, void* stream);
/* fp16 buckets: NumPy's half loops round every multiply and add to fp16 (an fp32
 * intermediate is innocuous for + and *, 24 >= 2*11+2); its HALF_pairwise_sum adds in
 * fp32 and rounds once.  h_w holds fp16 bit patterns. */
int fedagg_fedavg_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, uint64_t M,
                      const uint64_t* h_idx, int P, void* d_ws, uint16_t* d_out, void* stream);

/* ---------------------------------------------------------------------------
 * Scaffold two-bucket reduction, fp64 (NumPy 2 / NEP 50: the float64 client weights
 * are strong scalars, scaffold.py:319-320, so every product and sum is fp64).
 * Replaces scaffold.py:262-263 (control variate: sum_k w_k*cv_k, then + c LAST) and
 * scaffold.py:293 (delta: lr * sum_k w_k*delta_k):
 *     d_delta_out[i] = lr * (+0.0 + sum_seq_k fl64(w_k * delta_k[i]))
 *     d_c_out[i]     =       +0.0 + sum_seq_k fl64(w_k * cv_k[i]) + c[i]
 * h_w[k] = double(n_k) / double(n).  Inputs fp32 (_f32) or fp64 (_f64).  numel == 1
 * elements (h_idx): pairwise over the K (delta) and K + 1 (cv, c last) fp64 terms.
 * -------------------------------------------------------------------------*/
int fedagg_scaffold_f32(const float* const* d_delta, const float* const* d_cv, const float* d_c, const double* h_w,
                        int K, uint64_t M, const uint64_t* h_idx, int P, void* d_ws, double lr, double* d_delta_out,
                        double* d_c_out, void* stream);
int fedagg_scaffold_f64(const double* const* d_delta, const double* const* d_cv, const double* d_c,
                        const double* h_w, int K, uint64_t M, const uint64_t* h_idx, int P, void* d_ws, double lr,
                        double* d_delta_out, double* d_c_out, void* stream);
/* Kernel launches per chunk of <= 64 clients that fedagg_scaffold_* makes under the current
 * tuning: 1 (scaffold_kernel, both buckets in one walk) or 2 (scaffold_bucket_kernel, the delta
 * bucket then the control-variate bucket); in_elem_bytes 4 or 8, aligned = every operand 16-B
 * aligned.  For profilers and benchmarks that attribute kernel time; < 0 on bad arguments. */
int fedagg_scaffold_launches(int K, int in_elem_bytes, uint64_t M, int aligned);

/* ---------------------------------------------------------------------------
 * Scaffold server-control-variate check, scaffold.py:193-196
 *     np.testing.assert_array_equal(c_0, c_k)  for every client k
 * Value equality (+0.0 == -0.0, NaN == NaN).  Adds the number of mismatching
 * elements over all copies to *d_mismatches (a device uint64 the caller zeroes).
 * -------------------------------------------------------------------------*/
int fedagg_equal_count_f32(const float* const* d_copies, int K, uint64_t M, unsigned long long* d_mismatches,
                           void* stream);
int fedagg_equal_count_f64(const double* const* d_copies, int K, uint64_t M, unsigned long long* d_mismatches,
                           void* stream);

/* ---------------------------------------------------------------------------
 * Client-sharded building blocks (sharding.py).  The K clients are
 * cut into contiguous blocks, each block's buckets live on one GPU; the reference's
 * sequential client sum (fed_avg.py:221-222, scaffold.py:262-263,293) is then either
 *   - CHAINED: block b continues the accumulator of blocks 0..b-1 (received from the
 *     previous rank over xGMI) -- bit-identical to one pass, or
 *   - re-associated: every block sums from +0.0, the partial sums are combined on the
 *     root (RCCL reduce, or a gather + rank-order sum) -- a few ulp off the reference.
 * The numel==1 elements (NumPy pairwise order over ALL K products) cannot be chained:
 * every block writes its products into columns kbase.. of a [P][stride] workspace, the
 * root reduces the workspaces and runs the tree.
 *
 * fedavg_chain: acc = seed ? +0.0 : d_out[i];  acc = fl(acc + fl(x_k[i] * h_w[k])) for the K
 *   clients of this block, in order; d_out[i] = acc (no numel==1 patch; h_w are the GLOBAL
 *   weights fl(n_k / n)).  bf16 buckets accumulate into fp32 d_out, fp16 weights as bits.
 * -------------------------------------------------------------------------*/
int fedagg_fedavg_chain_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M, int seed,
                            float* d_out, void* stream);
/* The push executor's chain runs (FEDAGG_RUN_FEDAVG_PUSH): d_out = fl-continued d_in (this rank's
 * fp32 accumulator slot; NULL: start from +0.0) + the block's clients in order (fed_avg.py:221-222),
 * where d_out may be a peer GPU's memory mapped over xGMI.  Outputs are stored with system-scope
 * write-through stores and every wave waits for their acknowledgements, so the stores are performed
 * at system scope before the executor's tag / counter writes that follow the launch.  bf16 buckets
 * accumulate in fp32 like fedagg_fedavg_chain_bf16.  d_in / d_out 16-B aligned. */
int fedagg_fedavg_chain_push_f32(const float* const* d_clients, const float* h_w, int K, uint64_t M,
                                 const float* d_in, float* d_out, void* stream);
int fedagg_fedavg_chain_push_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M,
                                  const float* d_in, float* d_out, void* stream);
int fedagg_fedavg_chain_bf16(const uint16_t* const* d_clients, const float* h_w, int K, uint64_t M, int seed,
                             float* d_out, void* stream);
/* The push executor's Scaffold runs (FEDAGG_RUN_SCAFFOLD_PUSH_DELTA / _CV): ONE bucket of a client
 * block -- phase 0 the K delta rows, phase 1 the K control-variate rows -- d_out = the fp64
 * accumulator d_in (this rank's slot; NULL: start from +0.0) continued by fl(h_w[k] * x_k) in
 * client order; finish: phase 0 then multiplies by lr (scaffold.py:293), phase 1 adds d_c
 * (scaffold.py:262-263).  The arithmetic of fedagg_scaffold_chain_*'s two sums, one bucket at a
 * time; the stores as fedagg_fedavg_chain_push_* (system scope, acknowledged before the wave
 * retires).  d_rows / d_in / d_out / d_c 16-B aligned for the vector path. */
int fedagg_scaffold_chain_push_f32(const float* const* d_rows, const double* h_w, int K, uint64_t M, int phase,
                                   const float* d_c, double lr, int finish, const double* d_in, double* d_out,
                                   void* stream);
int fedagg_scaffold_chain_push_f64(const double* const* d_rows, const double* h_w, int K, uint64_t M, int phase,
                                   const double* d_c, double lr, int finish, const double* d_in, double* d_out,
                                   void* stream);
int fedagg_fedavg_chain_f64(const double* const* d_clients, const double* h_w, int K, uint64_t M, int seed,
                            double* d_out, void* stream);
int fedagg_fedavg_chain_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, uint64_t M, int seed,
                            uint16_t* d_out, void* stream);
/* The same over a tile-interleaved block (the layout of fedagg_fedavg_tiled_*: tile t of client k
 * at 16-B vector (t * K + k) * tile_vectors of d_base): a rank's client block in the client-sharded
 * schedules, where each block holds >= 32 clients (the weak form holds C3's 64 per rank). */
int fedagg_fedavg_chain_tiled_f32(const float* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                                  int seed, float* d_out, void* stream);
int fedagg_fedavg_chain_tiled_bf16(const uint16_t* d_base, const float* h_w, int K, uint64_t M, uint64_t tile_vectors,
                                   int seed, float* d_out, void* stream);
/* d_ws[p * stride + kbase + k] = fl(x_k[h_idx[p]] * h_w[k]) in the pairwise-sum type (fp32 for
 * f32/bf16/f16 -- NumPy's HALF_pairwise_sum adds in fp32 -- fp64 for f64). */
int fedagg_pairwise_products_f32(const float* const* d_clients, const float* h_w, int K, const uint64_t* h_idx,
                                 int P, int64_t stride, int kbase, float* d_ws, void* stream);
int fedagg_pairwise_products_bf16(const uint16_t* const* d_clients, const float* h_w, int K, const uint64_t* h_idx,
                                  int P, int64_t stride, int kbase, float* d_ws, void* stream);
int fedagg_pairwise_products_f64(const double* const* d_clients, const double* h_w, int K, const uint64_t* h_idx,
                                 int P, int64_t stride, int kbase, double* d_ws, void* stream);
int fedagg_pairwise_products_f16(const uint16_t* const* d_clients, const uint16_t* h_w, int K, const uint64_t* h_idx,
                                 int P, int64_t stride, int kbase, float* d_ws, void* stream);
/* d_out[h_idx[p]] = +0.0 + pairwise_sum(d_ws[p * stride .. p * stride + n)) (fed_avg.py:222 on a
 * numel == 1 tensor).  _f32 also serves bf16 buckets (fp32 output). */
int fedagg_pairwise_finish_f32(const float* d_ws, int64_t n, int64_t stride, const uint64_t* h_idx, int P,
                               float* d_out, void* stream);
int fedagg_pairwise_finish_f64(const double* d_ws, int64_t n, int64_t stride, const uint64_t* h_idx, int P,
                               double* d_out, void* stream);
int fedagg_pairwise_finish_f16(const float* d_ws, int64_t n, int64_t stride, const uint64_t* h_idx, int P,
                               uint16_t* d_out, void* stream);
/* Scaffold (fp64): seed ? +0.0 : d_*_out as the accumulators; finish = 1 on the LAST block only:
 * then + c (scaffold.py:262-263) and * lr (scaffold.py:293), d_c read; finish = 0: plain sums,
 * d_c may be NULL. */
int fedagg_scaffold_chain_f32(const float* const* d_delta, const float* const* d_cv, const float* d_c,
                              const double* h_w, int K, uint64_t M, int seed, int finish, double lr,
                              double* d_delta_out, double* d_c_out, void* stream);
int fedagg_scaffold_chain_f64(const double* const* d_delta, const double* const* d_cv, const double* d_c,
                              const double* h_w, int K, uint64_t M, int seed, int finish, double lr,
                              double* d_delta_out, double* d_c_out, void* stream);
/* Scaffold numel==1 workspace: P * (2 * Ktot + 1) doubles = delta terms [P][Ktot], then
 * control-variate terms [P][Ktot + 1] (column Ktot = c, written by _finish). */
int fedagg_scaffold_products_f32(const float* const* d_delta, const float* const* d_cv, const double* h_w, int K,
                                 int kbase, int Ktot, const uint64_t* h_idx, int P, double* d_ws, void* stream);
int fedagg_scaffold_products_f64(const double* const* d_delta, const double* const* d_cv, const double* h_w, int K,
                                 int kbase, int Ktot, const uint64_t* h_idx, int P, double* d_ws, void* stream);
int fedagg_scaffold_finish_f32(double* d_ws, int Ktot, const float* d_c, const uint64_t* h_idx, int P, double lr,
                               double* d_delta_out, double* d_c_out, void* stream);
int fedagg_scaffold_finish_f64(double* d_ws, int Ktot, const double* d_c, const uint64_t* h_idx, int P, double lr,
                               double* d_delta_out, double* d_c_out, void* stream);

/* ---------------------------------------------------------------------------
 * Native executor of the client-sharded lockstep schedules (substrafl_amd/lockstep.py,
 * DESIGN.md §6).  The schedule -- every run (one chain launch over a client block) and every
 * point-to-point message of every exchange group -- is computed once on the host; this issues it
 * from ONE thread on ONE RCCL communicator: for t = 0, 1, ...: exchange group t on the
 * communicator's stream after the caller's stream so far (ncclGroupStart / Send / Recv / End),
 * then step t's runs on the caller's stream after group t - 1; finally the in-place ncclReduce
 * of the numel == 1 product workspace onto the root.  Group t of every rank pairs only with group
 * t of its peers, so the schedule cannot deadlock.  Replaces the per-element client loop of
 * fed_avg.py:221-222 / scaffold.py:262-263,293 across GPUs (the reference has no multi-GPU path).
 * RCCL is dlopen'ed from rccl_path (NULL: "librccl.so.1"), reusing an instance already loaded.
 * -------------------------------------------------------------------------*/
enum { FEDAGG_BF16 = 12 };  /* kind of a run over bf16 buckets (fp32 accumulators)              */
enum { FEDAGG_RUN_FEDAVG = 0, FEDAGG_RUN_FEDAVG_TILED = 1, FEDAGG_RUN_SCAFFOLD = 2,
       FEDAGG_RUN_FEDAVG_PUSH = 3 /* FedAvg run (f32 / bf16) storing into mapped peer memory (push
                                     executor): acc = the output, acc2 = the input accumulator (NULL:
                                     seed ? +0.0 : acc) */,
       FEDAGG_RUN_SCAFFOLD_PUSH_DELTA = 4, /* Scaffold push run (f32 / f64 buckets, fp64 accumulators):
                                              x = the block's K delta rows, acc / acc2 as
                                              FEDAGG_RUN_FEDAVG_PUSH; finish: x lr */
       FEDAGG_RUN_SCAFFOLD_PUSH_CV = 5     /* the same over the K control-variate rows; finish: + c */ };
typedef struct fedagg_lockstep_run {
  int32_t step;              /* the step it runs at (runs sorted by step)                        */
  int32_t op;                /* FEDAGG_RUN_*                                                     */
  int32_t kind;              /* FEDAGG_F32 / FEDAGG_BF16 / FEDAGG_F64 / FEDAGG_F16 (Scaffold: F32/F64) */
  int32_t K;                 /* clients of the block (>= 1)                                      */
  int32_t seed, finish;      /* seed: start from +0.0; finish (Scaffold): + c, then * lr         */
  uint64_t n;                /* elements                                                         */
  uint64_t tile_vectors;     /* FEDAGG_RUN_FEDAVG_TILED: the tile                                */
  const void* const* x;      /* K client pointers (tiled: x[0] = the run's tile-interleaved bucket) */
  const void* const* x2;     /* Scaffold: the K control-variate pointers                         */
  const void* w;             /* K weights: float (f32/bf16), double (f64, Scaffold), fp16 bits   */
  const void* c;             /* Scaffold, finish: c of these elements                            */
  double lr;                 /* Scaffold: aggregation_lr                                         */
  void* acc;                 /* accumulator (Scaffold: the delta sum)                            */
  void* acc2;                /* Scaffold: the control-variate sum                                */
} fedagg_lockstep_run;
typedef struct fedagg_lockstep_msg {
  int32_t group;             /* exchange group (messages sorted by group)                        */
  int32_t send;              /* 1 send, 0 receive                                                */
  int32_t peer;              /* rank of the communicator                                         */
  int32_t kind;              /* element kind: FEDAGG_F32 / FEDAGG_F64 / FEDAGG_F16               */
  void* buf;
  uint64_t count;
} fedagg_lockstep_msg;
typedef struct fedagg_comm fedagg_comm;
/* rank 0 of the group: a fresh RCCL unique id (128 bytes) to hand to every rank */
int fedagg_comm_unique_id(const char* rccl_path, void* id_out);
/* every rank at once (collective): the communicator of `nranks` ranks on GPU `device` */
int fedagg_comm_create(const char* rccl_path, int nranks, int rank, const void* unique_id, int device,
                       fedagg_comm** out);
int fedagg_comm_destroy(fedagg_comm* comm);
/* ncclCommAbort (a watchdog's way out of a stuck exchange) */
int fedagg_comm_abort(fedagg_comm* comm);
/* ncclCommCount: the ranks RCCL itself counts in the communicator (the N > 1 bench line reports it) */
int fedagg_comm_count(fedagg_comm* comm, int* count_out);
/* 0, or FEDAGG_EHIP if RCCL reports an asynchronous error on the communicator */
int fedagg_comm_async_error(fedagg_comm* comm);
const char* fedagg_comm_last_error(void);
/* Enqueue the whole schedule (asynchronous on `stream` and the communicator's stream; the
 * caller's stream waits for everything at the end).  ws / ws_count / ws_kind: the numel == 1
 * product workspace, reduced in place onto `root` (NULL / 0: none). */
int fedagg_lockstep_execute(fedagg_comm* comm, const fedagg_lockstep_run* runs, int nruns,
                            const fedagg_lockstep_msg* msgs, int nmsgs, int ngroups, void* ws, uint64_t ws_count,
                            int ws_kind, int root, void* stream);

/* ---------------------------------------------------------------------------
 * Push executor of the same schedules (substrafl_amd/push.py, DESIGN.md §6 "Push"): no exchange
 * kernels.  Each run's chain kernel writes its accumulator straight into the consumer's slot (or
 * the root's output) through an IPC mapping over xGMI, continuing the input accumulator it reads
 * from this rank's own slot (fedagg_fedavg_chain_push_{f32,bf16}, fedagg_scaffold_chain_push_*).  Cross-process
 * order: one monotonic progress counter per rank in a node-shared host page; a call publishes
 * base + 1 on entry (the rank's earlier stream work is done: peers may write into its buffers),
 * then before step t a one-lane wait kernel polls the counters the step needs and after it a
 * one-lane signal kernel publishes base + t + 2 (system-scope release); the next call's base is
 * base + nsteps + 1.  Every wait points to a strictly earlier step
 * of another rank, so no hardware-queue mapping can deadlock it; a wait that exceeds
 * `timeout_ticks` (wall-clock ticks) gives up and records the counter index + 1 in
 * progress[nranks + rank] (+ 2^32 when it was a landing tag; the host checks it).
 * Landing tags: the counters travel to host memory over PCIe while the data a step pushed travels
 * over xGMI into the consumer's HBM, so a counter is no proof that the data landed.  After step t a
 * rank's signal kernel also writes the call's generation (base + 1) into one tag word per consumer
 * it pushed to at step t -- in the consumer's own (uncached) HBM, over the same link as the data,
 * after the step's runs each ended with a system-scope release -- and a consumer waits for the tag
 * of every push it reads, after the producer's counter; a tag found missing once the counter was
 * there is counted in progress[2 * nranks + rank] (the ordering gap, measured), and waited for.
 * Replaces the per-element client loop of fed_avg.py:221-222 across GPUs, like
 * fedagg_lockstep_execute.
 * -------------------------------------------------------------------------*/
#define FEDAGG_IPC_HANDLE_BYTES 64
/* IPC handle of the allocation holding `ptr`, and ptr's byte offset in it */
int fedagg_ipc_get(const void* ptr, void* handle_out, uint64_t* offset_out);
/* map another process's allocation (hipIpcOpenMemHandle, peer access enabled lazily) */
int fedagg_ipc_open(const void* handle, void** base_out);
int fedagg_ipc_close(void* base);
/* page-locked, device-mapped view of host memory (a node-shared page of progress counters) */
int fedagg_host_map(void* host, uint64_t bytes, void** dev_out);
int fedagg_host_unmap(void* host);
/* device memory no L2 caches (hipDeviceMallocUncached), zeroed: the push executor's landing
 * buffers, written by peers, read by this GPU's kernels without stale cache lines */
int fedagg_device_alloc_uncached(uint64_t bytes, void** out);
int fedagg_device_free(void* p);
#if FEDAGG_TUNING
/* FEDAGG_TUNING build only (the product library does not export it): device-to-device runtime
 * copy on `stream` (the same HIP runtime as the caller's streams), for tools/push_tail_probe.py.
 * No product path uses it, and none reads peer-written memory with it. */
int fedagg_copy_async(void* dst, const void* src, uint64_t bytes, void* stream);
#endif
/* wall-clock ticks per second of the device timer the wait kernels use */
int fedagg_wall_clock_hz(uint64_t* hz_out);
typedef struct fedagg_push_wait {
  int32_t step;              /* waited before this step's runs (nsteps: after the last step)     */
  int32_t rank;              /* whose progress counter                                           */
  int64_t value;             /* counter >= base + value (<= 0: nothing to wait for)              */
  const uint64_t* tag;       /* NULL, or this rank's landing tag of the producer's push: after the
                                counter, wait for *tag >= base + 1                               */
} fedagg_push_wait;
typedef struct fedagg_push_tag {
  int32_t step;              /* written after this step's runs (tags sorted by step)             */
  int32_t reserved;
  uint64_t* tag;             /* a consumer's landing tag (mapped peer memory): *tag = base + 1   */
} fedagg_push_tag;
typedef struct fedagg_push_copy {
  void* dst;                 /* the root's output                                                */
  const void* src;           /* its landing buffer (what other ranks pushed)                     */
  uint64_t bytes;            /* a multiple of 4                                                  */
} fedagg_push_copy;
/* runs: FEDAGG_RUN_FEDAVG / FEDAGG_RUN_FEDAVG_PUSH (acc: a mapped peer address; f32 or bf16) or
 * FEDAGG_RUN_SCAFFOLD_PUSH_DELTA / _CV (f32 or f64 buckets) sorted by step;
 * waits sorted by step; tags: the landing tags this rank writes, sorted by step (<= 16 a step);
 * ws_src / ws_dst / ws_bytes: the numel == 1 products (ws_kind FEDAGG_F32 for FedAvg, FEDAGG_F64
 * for Scaffold) copied to this rank's staging row on the root after step 0's waits (0 bytes:
 * none); ws_stage (root only, else NULL): the nranks staging rows, summed in rank order into
 * ws_src after the last waits.  copies (root only): the finished pieces other ranks pushed,
 * copied from the landing buffers into the outputs after the last waits.  A step's launches (one
 * per consumer and bucket, each writing over its own link) are spread round-robin over `stream`
 * and the `naux` (<= 7) aux streams, forked from and joined back into `stream` around the step.
 * Asynchronous on `stream`. */
int fedagg_push_execute(const fedagg_lockstep_run* runs, int nruns, const fedagg_push_wait* waits, int nwaits,
                        const fedagg_push_tag* tags, int ntags,
                        int nsteps, uint64_t* progress, int rank, int nranks, uint64_t base, uint64_t timeout_ticks,
                        const void* ws_src, void* ws_dst, uint64_t ws_bytes, int ws_kind, const void* ws_stage,
                        const fedagg_push_copy* copies, int ncopies, void* const* aux_streams, int naux,
                        void* stream);

/* ---------------------------------------------------------------------------
 * Client-side flat-bucket ops (the producer / consumer of the buckets, SURVEY.md §8(a)
 * a5-a7).  A model's L parameter tensors (device pointers d_layers[l], numel[l] fp32 elements
 * each, in weight_manager.model_parameters order, weight_manager.py:53-76) map onto one flat
 * bucket (layers back to back).  One launch per 32 layers instead of one torch op per layer.
 *   gather:    flat = concat(layers)                       get_parameters  (weight_manager.py:79-100)
 *   scatter:   layers = split(flat)                        set_parameters  (:215-238)
 *   wsum:      flat = sum() of layers_j * coeffs[j]         weighted_sum_parameters (:182-212),
 *              Python sum() order from int 0: acc = fl(0 + fl(x_0*fl32(c_0))), acc = fl(acc + fl(x_j*fl32(c_j)));
 *              d_layers is list-major [nlists][L], nlists <= FEDAGG_FLAT_MAX_LISTS
 *              (subtract_parameters :140-158 = coeffs {1,-1}; add_parameters :161-179 = {1,1};
 *              Scaffold's control-variate update torch_scaffold_algo.py:451-458 = {-1, -1/(lr*n)})
 *   increment: layers += fl32(multiplier) * flat           increment_parameters (:103-137)
 * -------------------------------------------------------------------------*/
#define FEDAGG_FLAT_MAX_LISTS 4
int fedagg_flat_gather_f32(const float* const* d_layers, const uint64_t* numel, int L, float* d_flat, void* stream);
int fedagg_flat_scatter_f32(float* const* d_layers, const uint64_t* numel, int L, const float* d_flat, void* stream);
int fedagg_flat_wsum_f32(const float* const* d_layers, int nlists, const double* coeffs, const uint64_t* numel, int L,
                         float* d_flat, void* stream);
int fedagg_flat_increment_f32(float* const* d_layers, const uint64_t* numel, int L, const float* d_flat,
                              double multiplier, void* stream);
/* Kind-generic forms (kinds FEDAGG_F32 / FEDAGG_F64, enum below) for Scaffold's client side,
 * where the server control variate arrives as fp64 (scaffold.py:262-263 outputs fp64) and torch
 * promotes (torch_scaffold_algo.py:256-268 increment with fp64 delta_variate, :424-427, :451-462):
 *   wsum:      kinds[j] per list; d_flat has the promoted kind (fp64 if any list is fp64).
 *              p_j = fl_j(x * c_j) in list j's kind (c rounded to fp32 for fp32 lists);
 *              acc = 0 + p_0, then acc = acc + p_j in the promoted kind of (acc, p_j).
 *   increment: fp32 parameters += multiplier * flat; an fp64 flat runs in fp64:
 *              w = fl32(fl64(w) + fl64(m * u)).
 *   gather:    layers of one kind into a flat bucket of that kind. */
int fedagg_flat_gather(const void* const* d_layers, int kind, const uint64_t* numel, int L, void* d_flat,
                       void* stream);
int fedagg_flat_wsum(const void* const* d_layers, const int* kinds, int nlists, const double* coeffs,
                     const uint64_t* numel, int L, void* d_flat, int flat_kind, void* stream);
int fedagg_flat_increment(float* const* d_layers, const uint64_t* numel, int L, const void* d_flat, int flat_kind,
                          double multiplier, void* stream);

/* ---------------------------------------------------------------------------
 * dtype plumbing (device side, NumPy semantics).  Kinds: */
enum {
  FEDAGG_F16 = 0, FEDAGG_F32 = 1, FEDAGG_F64 = 2,
  FEDAGG_I8 = 3, FEDAGG_I16 = 4, FEDAGG_I32 = 5, FEDAGG_I64 = 6,
  FEDAGG_U8 = 7, FEDAGG_U16 = 8, FEDAGG_U32 = 9, FEDAGG_U64 = 10, FEDAGG_BOOL = 11,
};
/* out[i] = (out_kind) in[i]: integer/bool -> float as NumPy's astype (round to nearest),
 * float widening exact.  Used for integer layers (x_int * python_float is a float64 loop). */
int fedagg_cast(const void* d_in, int in_kind, void* d_out, int out_kind, uint64_t n, void* stream);
/* out[i] = (out_kind) fl_in(in[i] * fl_in(w)): one client's product in its own float type,
 * then widened -- a layer whose clients carry different dtypes (fed_avg.py:221-222 stacks the
 * per-client products, then promotes). */
int fedagg_scale_cast(const void* d_in, int in_kind, double w, void* d_out, int out_kind, uint64_t n, void* stream);

/* ---------------------------------------------------------------------------
 * Measurement helper: streams M floats (16-B non-temporal loads, the load path of the
 * bucket kernels) and writes one float per workgroup to d_sink.  Gives the read-stream
 * ceiling the roofline fraction is also quoted against.
 * -------------------------------------------------------------------------*/
int fedagg_read_probe_f32(const float* d_x, uint64_t M, float* d_sink, int grid, void* stream);
/* The same, in the bucket kernels' tile walk: one workgroup per tile of vpt x 256 contiguous 16-B
 * vectors (vpt 4, 8 or 16), every load of a thread in flight at once; d_sink needs one float
 * (written only on an impossible value).  The read ceiling is the best of both probes. */
int fedagg_read_probe_tile_f32(const float* d_x, uint64_t M, float* d_sink, int vpt, void* stream);

/* ---------------------------------------------------------------------------
 * Host runtime ("session"): one GPU, one HIP stream, grow-only HBM buffers, a pinned
 * staging ring and a worker pool.  It replaces the plumbing around the reference's hot path
 * (shared states arrive as host pickles, substratools_methods.py:54-66, and the result is
 * pickled back, :82-86) without PyTorch on the task's critical path.
 * -------------------------------------------------------------------------*/
#define FEDAGG_SESSION_BUFFERS 16
#define FEDAGG_SESSION_EVENTS 8
typedef struct fedagg_session fedagg_session;
/* NULL on failure (no device, ...): see fedagg_last_error(). */
fedagg_session* fedagg_session_create(int device);
void fedagg_session_destroy(fedagg_session* s);
/* the session's hipStream_t, to pass as `stream` to the kernel entry points */
void* fedagg_session_stream(fedagg_session* s);
/* knobs: "threads" (pack workers), "chunk_bytes" (pinned slot size), "slots" (ring length),
 * "copy_streams" (1 or 2 H2D queues for staging; default 2), "fail_copy_after" (tests: the n-th
 * copy enqueued from now on fails with FEDAGG_EHIP; 0 = never) */
int fedagg_session_set(fedagg_session* s, const char* key, long long value);
/* Host placement (multi_device.host_placement): the session's pack workers bind to `cpus`
 * (ncpus == 0: no binding), and its pinned staging ring is allocated by a thread bound to them
 * under the user's NUMA policy (hipHostMallocNumaUser), so the ring lands on their node --
 * the GPU's own NUMA node.  Takes effect at the next stage / fetch (the ring is re-allocated). */
int fedagg_session_affinity(fedagg_session* s, const int* cpus, int ncpus);
/* NUMA node of the page holding the session's pinned ring (get_mempolicy), -1 if unknown or the
 * ring is not allocated yet */
int fedagg_session_ring_node(fedagg_session* s);
/* hipDeviceGetPCIBusId: "dddd:bb:dd.f" of `device` into buf (len >= 13), for the NUMA node
 * lookup in /sys/bus/pci/devices/<id>/numa_node */
int fedagg_device_pci_bus_id(int device, char* buf, int len);
/* grow-only device buffer number `slot` (0..FEDAGG_SESSION_BUFFERS-1) of at least `bytes` */
int fedagg_session_buffer(fedagg_session* s, int slot, uint64_t bytes, void** d_ptr);
/* Prepare everything the first aggregation would otherwise pay for, so a one-shot task process
 * can do it while it is still unpickling its inputs (on another thread): the pinned staging ring,
 * the worker pool, HBM buffers slot i of slot_bytes[i] bytes (0: skip), and the kernels' code
 * object (one tiny launch).  Returns when done. */
int fedagg_session_warm(fedagg_session* s, const uint64_t* slot_bytes, int nslots);
/* Pack K host rows into HBM: row k = concatenation of the nseg host segments
 * h_seg[k*nseg + i] (seg_bytes[i] bytes each), written at d_dst + k*ld_bytes.  Host memory
 * may be pageable; the copies are pipelined through the pinned ring and enqueued on the
 * session stream (the host segments may be released once the call returns). */
int fedagg_session_stage(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg,
                         const void* const* h_seg, const uint64_t* seg_bytes);
/* Same, for bytes [byte_lo, byte_hi) of every client's row only (a parameter-range shard,
 * SURVEY.md §8(e)): written at d_dst + k*ld_bytes.  fedagg_session_stage is the full range. */
int fedagg_session_stage_range(fedagg_session* s, void* d_dst, uint64_t ld_bytes, int K, int nseg,
                               const void* const* h_seg, const uint64_t* seg_bytes, uint64_t byte_lo,
                               uint64_t byte_hi);
/* K rows of host segments in the tile-interleaved layout of fedagg_fedavg_tiled_*: tile t of row k
 * (row bytes [t * tile_bytes, (t + 1) * tile_bytes)) lands at d_dst + (t * K + k) * tile_bytes;
 * the K rows' tiles are gathered into each pinned chunk on the workers, so every H2D copy is one
 * contiguous run of blocks.  tile_bytes: FEDAGG_TILE_VECTORS_* x 16 (a multiple of 16, at most the
 * session's chunk_bytes); d_dst holds ceil(row / tile_bytes) * K * tile_bytes bytes. */
int fedagg_session_stage_tiled(fedagg_session* s, void* d_dst, uint64_t tile_bytes, int K, int nseg,
                               const void* const* h_seg, const uint64_t* seg_bytes);
/* ONE row (client k of K; nseg host segments) into the same tile-interleaved layout: its tile t
 * lands at d_dst + (t * K + k) * tile_bytes, one strided 2-D H2D copy per pinned chunk -- the
 * per-client staging of an ingest, where the clients arrive one by one (engine.ingest). */
int fedagg_session_stage_tiled_row(fedagg_session* s, void* d_dst, uint64_t tile_bytes, int K, int k, int nseg,
                                   const void* const* h_seg, const uint64_t* seg_bytes);
/* Scaffold's server-control-variate check on the host, during staging (scaffold.py:193-196,
 * np.testing.assert_array_equal(c_0, c_k)): K clients' c rows (nseg host segments each, as
 * fedagg_session_stage); ONE copy -- bytes [byte_lo, byte_hi) of row 0 -- is staged to d_dst, the
 * same bytes of rows 1..K-1 are compared with it by value on the pack workers (+0 == -0,
 * NaN == NaN; byte-identical stretches skipped) and the number of mismatching elements is written
 * to *mismatches.  kind: FEDAGG_F32 or FEDAGG_F64 (every segment of that element type; the range
 * element-aligned).  Replaces K-1 PCIe copies plus the device check (fedagg_equal_count_*).
 * d_dst may be NULL: compare only (rows already staged, e.g. while the inputs are still loading). */
int fedagg_session_stage_check(fedagg_session* s, void* d_dst, int K, int nseg, const void* const* h_seg,
                               const uint64_t* seg_bytes, uint64_t byte_lo, uint64_t byte_hi, int kind,
                               uint64_t* mismatches);
/* Make the session's GPU the calling thread's current device (kernel entry points launch on
 * the current device: a thread driving several sessions calls this before each one's launches). */
int fedagg_session_activate(fedagg_session* s);
/* number of visible GPUs (0 when none or on error) */
int fedagg_device_count(void);
/* the calling thread's current HIP device, and setting it: the session calls bind their device
 * to the calling thread, so the engine's entry points restore the caller's device on return
 * (engine.serialized) -- a multi-device aggregation must not leave the caller's later work (its
 * training, in simulate_experiment) on the last GPU it drove */
int fedagg_device_get(int* device_out);
int fedagg_device_set(int device);
/* hipMemGetInfo of `device`: free and total HBM bytes (sizing of out-of-core shards). */
int fedagg_device_memory(int device, uint64_t* free_bytes, uint64_t* total_bytes);
/* Copy `bytes` from HBM into (pageable) host memory; returns when the data is in h_dst. */
int fedagg_session_fetch(fedagg_session* s, const void* d_src, void* h_dst, uint64_t bytes);
int fedagg_session_memset(fedagg_session* s, void* d, int value, uint64_t bytes);
/* Copy `bytes` between two allocations of the session's GPU, ordered on its stream (the device
 * hand-off of simulation mode, substrafl_amd/handoff.py: a client's exported bucket into the
 * aggregator's [K, ld] rows, the aggregator's output into a client's update bucket, instead of a
 * D2H + H2D round trip; replaces the H2D of `torch.from_numpy(x).to(device)`,
 * torch_fed_avg_algo.py:189-194, and the staging of fed_avg.py:217-222's inputs). */
int fedagg_session_copy_d2d(fedagg_session* s, void* d_dst, const void* d_src, uint64_t bytes);
int fedagg_session_sync(fedagg_session* s);
/* timing events on the session stream (0 <= ev < FEDAGG_SESSION_EVENTS): record, and the time
 * between two recorded events in ms (waits for ev1) -- per-shard kernel time of the one-process
 * multi-GPU engine (bench.py --engine multi-device) */
int fedagg_session_event_record(fedagg_session* s, int ev);
int fedagg_session_event_elapsed(fedagg_session* s, int ev0, int ev1, float* ms);
/* wall time of the last stage / fetch call, seconds */
int fedagg_session_timing(fedagg_session* s, double* stage_s, double* fetch_s);
/* Start-up phases of the session, seconds, into out[0 .. min(n, FEDAGG_SESSION_PHASES)): 0 the HIP
 * runtime's initialisation and the device (fedagg_session_create's first calls: the whole runtime
 * start-up when it is the process's first HIP call), 1 its streams and events, then
 * fedagg_session_warm's 2 pinned staging ring (hipHostMalloc, on the NUMA node of the session's
 * CPUs), 3 worker pool, 4 HBM buffers, 5 code-object load (the first kernel launch, synchronised);
 * 0.0 for a phase that has not run.  The task process's start-up attribution
 * (remote/substratools_methods.py:94-118: the prewarm overlapped with the unpickling). */
#define FEDAGG_SESSION_PHASES 6
int fedagg_session_phases(fedagg_session* s, double* out, int n);

/* ---------------------------------------------------------------------------
 * One process, several GPUs (csrc/multi.hip): the parameter-range FedAvg of an aggregate task in
 * one call -- the plan of substrafl_amd/multi_device.py (MultiDeviceEngine) for a host in any
 * language (SURVEY.md §8(b) "fa_multi_init / fa_reduce_sharded_*", §8(e) primary partitioning).
 * A Substra aggregate task is one OS process (remote/register/register.py:96), so a host that
 * wants the node's GPUs drives them from one process.  Replaces fed_avg.py:217-222 over host
 * buckets, bit-identical to fedagg_fedavg_* over the whole range (no collective):
 *   - [0, M) is cut into one contiguous 512-element-aligned shard per device (equal chunks, the
 *     last shards may get less or nothing);
 *   - one thread and one private session per shard (a repeated device index gets its own, so a
 *     one-GPU box exercises the sharded path), its `pack_threads` pack workers (0: the CPUs this
 *     process may use / ndev, 2..32) and pinned ring bound to the GPU's NUMA node;
 *   - each shard streams through its GPU in sub-ranges sized to 85 % of its free HBM (or the
 *     "max_shard_bytes" knob): stage bytes [lo, hi) of every row (fedagg_session_stage_range),
 *     the bucket kernel with the numel == 1 patch of the elements it owns, fetch into h_out.
 * Rows: K clients x nseg host segments each (h_seg[k * nseg + i], seg_bytes[i] bytes; pageable
 * host memory, as fedagg_session_stage), M = sum(seg_bytes) / element size; h_w the K weights
 * fl(n_k / n); h_idx the P flat indices of numel == 1 tensors; h_out M elements of host memory.
 * Blocking: returns when h_out holds the result; the caller's current device is unchanged.  One
 * call at a time per object (calls on one object serialise). */
typedef struct fedagg_multi fedagg_multi;
fedagg_multi* fedagg_multi_create(int ndev, const int* devs, int pack_threads);
void fedagg_multi_destroy(fedagg_multi* m);
/* knobs: "max_shard_bytes" (HBM one sub-range may take; 0 = 85 % of free HBM), "threads" */
int fedagg_multi_set(fedagg_multi* m, const char* key, long long value);
int fedagg_multi_fedavg_f32(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                            const float* h_w, const uint64_t* h_idx, int P, float* h_out);
int fedagg_multi_fedavg_f64(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                            const double* h_w, const uint64_t* h_idx, int P, double* h_out);
/* fp16 buckets: h_w and h_out hold fp16 bit patterns (fedagg_fedavg_f16's semantics, NumPy's half loops) */
int fedagg_multi_fedavg_f16(fedagg_multi* m, int K, int nseg, const void* const* h_seg, const uint64_t* seg_bytes,
                            const uint16_t* h_w, const uint64_t* h_idx, int P, uint16_t* h_out);
/* shard g: its device, the GPU's NUMA node (-1 unknown), pack workers, CPUs they are bound to, and
 * of the last call its element range [lo, hi) and the sub-ranges it streamed (any pointer NULL) */
int fedagg_multi_shard_info(fedagg_multi* m, int g, int* device, int* numa_node, int* threads, int* ncpus,
                            uint64_t* lo, uint64_t* hi, int* ranges);

#ifdef __cplusplus
}
#endif
#endif /* FEDAGG_H */
