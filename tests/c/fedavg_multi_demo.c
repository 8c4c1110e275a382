/* The one-call multi-device entry from plain C (no HIP headers, no Python): fedagg_multi_* over
 * `devs` (default {0, 0}: two shards on one GPU, each with its own session) against the
 * single-device path (fedagg_session_stage + fedagg_fedavg_f32 over the whole range), bit for bit,
 * and against the reference order on the host for the numel >= 2 elements (fed_avg.py:217-222:
 * acc = +0.0; acc = fl(acc + fl(x_k * w_k))).  Layers of ragged sizes with a (1,)-shaped one in the
 * middle (NumPy's pairwise order over the K products, K >= 8 here); a small "max_shard_bytes" makes
 * every shard stream through its GPU in several sub-ranges (the out-of-core path).
 * Usage: fedavg_multi_demo [dev0 dev1 ...]
 * Build: gcc -O2 -ffp-contract=off -Iinclude tests/c/fedavg_multi_demo.c -Lsubstrafl_amd -lfedagg */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fedagg.h"

#define K 10
#define NSEG 4
static const uint64_t numel[NSEG] = {70001, 1, 100000, 30003}; /* M = 200005; the (1,) layer at 70001 */

static uint32_t lcg(uint32_t* s) { return *s = *s * 1664525u + 1013904223u; }

int main(int argc, char** argv) {
  int devs[16] = {0, 0};
  int ndev = 2;
  if (argc > 1) {
    ndev = argc - 1 > 16 ? 16 : argc - 1;
    for (int g = 0; g < ndev; ++g) devs[g] = atoi(argv[g + 1]);
  }
  uint64_t M = 0, seg_bytes[NSEG];
  for (int i = 0; i < NSEG; ++i) {
    M += numel[i];
    seg_bytes[i] = numel[i] * sizeof(float);
  }
  float* layers[K][NSEG];
  const void* seg[K * NSEG];
  uint32_t seed = 777u;
  long long n[K], n_all = 0;
  for (int k = 0; k < K; ++k) {
    n[k] = 1 + (long long)(lcg(&seed) % 5000u);
    n_all += n[k];
    for (int i = 0; i < NSEG; ++i) {
      layers[k][i] = malloc(seg_bytes[i]);
      for (uint64_t e = 0; e < numel[i]; ++e) layers[k][i][e] = ((float)(int32_t)lcg(&seed)) * 1e-9f;
      seg[k * NSEG + i] = layers[k][i];
    }
  }
  float w[K];
  for (int k = 0; k < K; ++k) w[k] = (float)((double)n[k] / (double)n_all); /* fl32(n_k / n) */
  uint64_t idx[1] = {numel[0]};

  /* the single-device call over the whole range */
  float* single = calloc(M, sizeof(float));
  float* multi = calloc(M, sizeof(float));
  fedagg_session* s = fedagg_session_create(devs[0]);
  if (!s) {
    fprintf(stderr, "session: %s\n", fedagg_last_error());
    return 2;
  }
  const uint64_t ld = (M + 63) / 64 * 64;
  void *d_rows = NULL, *d_out = NULL, *d_ws = NULL;
  if (fedagg_session_buffer(s, 0, K * ld * sizeof(float), &d_rows) ||
      fedagg_session_buffer(s, 1, ld * sizeof(float), &d_out) ||
      fedagg_session_buffer(s, 2, fedagg_pairwise_ws_bytes(K, 1, 8), &d_ws) ||
      fedagg_session_stage(s, d_rows, ld * sizeof(float), K, NSEG, seg, seg_bytes)) {
    fprintf(stderr, "stage: %s\n", fedagg_last_error());
    return 2;
  }
  const float* rows[K];
  for (int k = 0; k < K; ++k) rows[k] = (const float*)((const char*)d_rows + k * ld * sizeof(float));
  if (fedagg_fedavg_f32(rows, w, K, M, idx, 1, d_ws, (float*)d_out, fedagg_session_stream(s)) ||
      fedagg_session_fetch(s, d_out, single, sizeof(float) * M)) {
    fprintf(stderr, "fedavg: %s\n", fedagg_last_error());
    return 2;
  }
  fedagg_session_destroy(s);

  /* the one-call multi-device path */
  fedagg_multi* m = fedagg_multi_create(ndev, devs, 0);
  if (!m) {
    fprintf(stderr, "multi_create: %s\n", fedagg_last_error());
    return 2;
  }
  /* (K + 1) x 4 B per element: ~24 K elements per sub-range, several per shard */
  if (fedagg_multi_set(m, "max_shard_bytes", 1 << 20) ||
      fedagg_multi_fedavg_f32(m, K, NSEG, seg, seg_bytes, w, idx, 1, multi)) {
    fprintf(stderr, "multi_fedavg: %s\n", fedagg_last_error());
    return 2;
  }
  int ranges_total = 0, shards_used = 0;
  for (int g = 0; g < ndev; ++g) {
    int dev = -1, node = -2, threads = 0, ncpus = 0, ranges = 0;
    uint64_t lo = 0, hi = 0;
    if (fedagg_multi_shard_info(m, g, &dev, &node, &threads, &ncpus, &lo, &hi, &ranges)) {
      fprintf(stderr, "shard_info: %s\n", fedagg_last_error());
      return 2;
    }
    printf("shard %d: device %d numa %d threads %d cpus %d range [%llu, %llu) sub-ranges %d\n", g, dev, node, threads,
           ncpus, (unsigned long long)lo, (unsigned long long)hi, ranges);
    ranges_total += ranges;
    shards_used += hi > lo;
  }
  /* a second call on the same object (grow-only buffers reused): the same bits */
  float* again = calloc(M, sizeof(float));
  if (fedagg_multi_set(m, "max_shard_bytes", 0) || fedagg_multi_fedavg_f32(m, K, NSEG, seg, seg_bytes, w, idx, 1, again)) {
    fprintf(stderr, "multi_fedavg (2): %s\n", fedagg_last_error());
    return 2;
  }
  /* fp64 buckets through the same object: the f64 entry against the single-device f64 kernel */
  int bad64 = 0;
  {
    double* l64[K][NSEG];
    const void* seg64[K * NSEG];
    uint64_t bytes64[NSEG];
    for (int i = 0; i < NSEG; ++i) bytes64[i] = numel[i] * sizeof(double);
    for (int k = 0; k < K; ++k)
      for (int i = 0; i < NSEG; ++i) {
        l64[k][i] = malloc(bytes64[i]);
        for (uint64_t e = 0; e < numel[i]; ++e) l64[k][i][e] = (double)layers[k][i][e] * 1.000000119;
        seg64[k * NSEG + i] = l64[k][i];
      }
    double w64[K];
    for (int k = 0; k < K; ++k) w64[k] = (double)n[k] / (double)n_all;
    double* multi64 = calloc(M, sizeof(double));
    double* single64 = calloc(M, sizeof(double));
    if (fedagg_multi_fedavg_f64(m, K, NSEG, seg64, bytes64, w64, idx, 1, multi64)) {
      fprintf(stderr, "multi_fedavg_f64: %s\n", fedagg_last_error());
      return 2;
    }
    fedagg_session* s64 = fedagg_session_create(devs[0]);
    const uint64_t ld64 = (M + 31) / 32 * 32;
    void *r64 = NULL, *o64 = NULL, *w64s = NULL;
    if (!s64 || fedagg_session_buffer(s64, 0, K * ld64 * sizeof(double), &r64) ||
        fedagg_session_buffer(s64, 1, ld64 * sizeof(double), &o64) ||
        fedagg_session_buffer(s64, 2, fedagg_pairwise_ws_bytes(K, 1, 8), &w64s) ||
        fedagg_session_stage(s64, r64, ld64 * sizeof(double), K, NSEG, seg64, bytes64)) {
      fprintf(stderr, "stage f64: %s\n", fedagg_last_error());
      return 2;
    }
    const double* rows64[K];
    for (int k = 0; k < K; ++k) rows64[k] = (const double*)((const char*)r64 + k * ld64 * sizeof(double));
    if (fedagg_fedavg_f64(rows64, w64, K, M, idx, 1, w64s, (double*)o64, fedagg_session_stream(s64)) ||
        fedagg_session_fetch(s64, o64, single64, sizeof(double) * M)) {
      fprintf(stderr, "fedavg_f64: %s\n", fedagg_last_error());
      return 2;
    }
    fedagg_session_destroy(s64);
    for (uint64_t e = 0; e < M; ++e) bad64 += memcmp(&multi64[e], &single64[e], sizeof(double)) != 0;
  }
  fedagg_multi_destroy(m);
  /* a device that does not exist: no object, the error names it */
  int nodev[1] = {4096};
  fedagg_multi* none = fedagg_multi_create(1, nodev, 0);
  const int refused = none == NULL && strstr(fedagg_last_error(), "device 4096") != NULL;
  if (none) fedagg_multi_destroy(none);

  int bad = 0, bad_again = 0, bad_ref = 0;
  for (uint64_t e = 0; e < M; ++e) {
    bad += memcmp(&multi[e], &single[e], sizeof(float)) != 0;
    bad_again += memcmp(&again[e], &single[e], sizeof(float)) != 0;
  }
  uint64_t base = 0;
  for (int i = 0; i < NSEG; ++i) {
    if (numel[i] >= 2)
      for (uint64_t e = 0; e < numel[i]; ++e) {
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) {
          float p = layers[k][i][e] * w[k];
          acc = acc + p;
        }
        bad_ref += memcmp(&acc, &single[base + e], sizeof(float)) != 0;
      }
    base += numel[i];
  }
  printf("fedavg_multi_demo: K=%d M=%llu shards=%d used=%d sub_ranges=%d mismatches=%d again=%d vs_reference_order=%d "
         "f64=%d bad_device_refused=%d (abi %d)\n",
         K, (unsigned long long)M, ndev, shards_used, ranges_total, bad, bad_again, bad_ref, bad64, refused,
         fedagg_abi_version());
  return (bad || bad_again || bad_ref || bad64 || !refused || ranges_total <= ndev) ? 1 : 0;
}
