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

#ifdef __cplusplus
extern "C" {
#endif

#define FEDAGG_ABI_VERSION 2
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
/* Process-wide launch knobs (defaults are the values measured best on MI355X):
 *   "grid_cap"      workgroups per launch before the kernels grid-stride (<= 0: no cap)
 *   "nt_load"       non-temporal client loads (0/1)      "nt_store"  non-temporal output stores
 *   "vpt"           16-B vectors per thread per step (0 = auto by K, 1/2/4/8)
 *   "unroll"        clients per load group (2/4/8/16, with an explicit vpt)
 *   "tile"          a workgroup step covers vpt*256 contiguous vectors (0/1)
 *   "pipe"          software-pipelined client groups (0/1, vpt 1 only)
 *   "fuse_pairwise" patch numel==1 tensors inside the bucket launch (0/1)
 *   "sc_vpt"        Scaffold: 16-B vectors per thread per step (1/2/4/8)
 *   "sc_unroll"     Scaffold: clients per load group (2/4)
 * Returns FEDAGG_EINVAL for an unknown key. */
int fedagg_tune(const char* key, long long value);

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
 * Measurement helper: streams M floats (16-B non-temporal loads, the load path of the
 * bucket kernels) and writes one float per workgroup to d_sink.  Gives the read-stream
 * ceiling the roofline fraction is also quoted against.
 * -------------------------------------------------------------------------*/
int fedagg_read_probe_f32(const float* d_x, uint64_t M, float* d_sink, int grid, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FEDAGG_H */
