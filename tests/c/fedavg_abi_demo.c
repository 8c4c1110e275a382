/* The drop-in boundary from plain C (no HIP headers, no Python): what a binding from another
 * language does.  Stages K host buckets through the native session, runs fedagg_fedavg_f32 and
 * checks every element bit for bit against the reference order (fed_avg.py:217-222 under NumPy
 * 2: acc = +0.0; acc = fl(acc + fl(x_k * w_k)) for numel >= 2; +0.0 + pairwise_sum for the
 * numel == 1 element, which for K < 8 is the sequential sum seeded with -0.0).
 * Build: gcc -O2 -ffp-contract=off -Iinclude tests/c/fedavg_abi_demo.c -Lsubstrafl_amd -lfedagg */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fedagg.h"

#define K 5
#define M 1001 /* one 1000-element layer, then a (1,)-shaped layer at flat index 1000 */
#define LD 1024

static uint32_t lcg(uint32_t* s) { return *s = *s * 1664525u + 1013904223u; }

int main(void) {
  static float x[K][LD];
  static float out[LD];
  static float ref[M];
  uint32_t seed = 12345u;
  long long n[K], n_all = 0;
  for (int k = 0; k < K; ++k) {
    n[k] = 1 + (long long)(lcg(&seed) % 5000u);
    n_all += n[k];
    for (int i = 0; i < LD; ++i) x[k][i] = ((float)(int32_t)lcg(&seed)) * 1e-9f;
  }
  float w[K];
  for (int k = 0; k < K; ++k) w[k] = (float)((double)n[k] / (double)n_all); /* fl32(n_k / n) */

  for (int i = 0; i < M - 1; ++i) {
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) {
      float p = x[k][i] * w[k];
      acc = acc + p;
    }
    ref[i] = acc;
  }
  {
    float pw = -0.0f;
    for (int k = 0; k < K; ++k) {
      float p = x[k][M - 1] * w[k];
      pw = pw + p;
    }
    ref[M - 1] = 0.0f + pw;
  }

  fedagg_session* s = fedagg_session_create(0);
  if (!s) {
    fprintf(stderr, "session: %s\n", fedagg_last_error());
    return 2;
  }
  void *d_rows = NULL, *d_out = NULL;
  if (fedagg_session_buffer(s, 0, sizeof(x), &d_rows) || fedagg_session_buffer(s, 1, sizeof(out), &d_out)) {
    fprintf(stderr, "buffer: %s\n", fedagg_last_error());
    return 2;
  }
  const void* seg[K];
  uint64_t seg_bytes[1] = {sizeof(x[0])};
  for (int k = 0; k < K; ++k) seg[k] = x[k];
  if (fedagg_session_stage(s, d_rows, sizeof(x[0]), K, 1, seg, seg_bytes)) {
    fprintf(stderr, "stage: %s\n", fedagg_last_error());
    return 2;
  }
  const float* rows[K];
  for (int k = 0; k < K; ++k) rows[k] = (const float*)((const char*)d_rows + k * sizeof(x[0]));
  uint64_t idx[1] = {M - 1};
  if (fedagg_fedavg_f32(rows, w, K, M, idx, 1, NULL, (float*)d_out, fedagg_session_stream(s)) ||
      fedagg_session_fetch(s, d_out, out, sizeof(float) * M)) {
    fprintf(stderr, "fedavg: %s\n", fedagg_last_error());
    return 2;
  }
  int bad = 0;
  for (int i = 0; i < M; ++i) bad += memcmp(&out[i], &ref[i], sizeof(float)) != 0;
  fedagg_session_destroy(s);
  printf("fedavg_abi_demo: K=%d M=%d mismatches=%d (abi %d)\n", K, M, bad, fedagg_abi_version());
  return bad ? 1 : 0;
}
