/*
 * c_client.c — a plain C caller of the drop-in boundary (include/shelfi.h), no Python:
 * the round the reference's CKKS class runs (ckks.cpp:25-59 keygen, :61-104 encrypt,
 * :264-320 computeWeightedAverage, :170-213 decrypt), as a C/C++ aggregator (or a cgo /
 * JNI stub over the same symbols) would drive it.
 *
 *   c_client CRYPTODIR      (writes PALISADE key files there; prints "C CLIENT OK")
 *
 * Checks, with BASELINE config 2's parameters (N = 2^15, L = 4, batch 16384):
 *  1. keygen writes the three cereal files; a second context loads them (loadCryptoParams);
 *  2. 4 learners encrypt 3 ciphertexts' worth of values (blob and PALISADE wire formats);
 *  3. the weighted average decrypts, in the second context, to the plain weighted sum
 *     within 1e-7 (exact decode) and 1e-6 (flooded decode, the default);
 *  4. error paths: weight/learner mismatch in size, a non-finite weight, a truncated blob.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shelfi.h"

#define CHECK(call)                                                                      \
  do {                                                                                   \
    int rc_ = (call);                                                                    \
    if (rc_ != SHELFI_OK) {                                                              \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,          \
              shelfi_last_error());                                                      \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

enum { C = 4, BATCH = 16384, N_VALUES = 3 * BATCH - 1000 };

static double max_err(const double* a, const double* b, size_t n) {
  double m = 0.0;
  for (size_t i = 0; i < n; ++i) {
    const double d = fabs(a[i] - b[i]);
    if (!(d <= m)) m = d;  /* also propagates NaN */
  }
  return m;
}

static int round_trip(shelfi_ctx* enc_ctx, shelfi_ctx* dec_ctx, int palisade_wire, double** x,
                      const float* w, const double* expect) {
  uint8_t* blobs[C];
  size_t lens[C];
  CHECK(shelfi_set_wire_format(enc_ctx, palisade_wire));
  for (int c = 0; c < C; ++c) CHECK(shelfi_encrypt(enc_ctx, x[c], N_VALUES, &blobs[c], &lens[c]));
  uint8_t* agg = NULL;
  size_t agg_len = 0;
  CHECK(shelfi_weighted_average(dec_ctx, (const uint8_t* const*)blobs, lens, w, C, &agg, &agg_len));
  double* out = (double*)malloc(sizeof(double) * N_VALUES);
  CHECK(shelfi_set_decode_noise(dec_ctx, 0, 1.0));
  CHECK(shelfi_decrypt(dec_ctx, agg, agg_len, N_VALUES, out));
  const double e_exact = max_err(out, expect, N_VALUES);
  CHECK(shelfi_set_decode_noise(dec_ctx, 1, 1.0));
  CHECK(shelfi_decrypt(dec_ctx, agg, agg_len, N_VALUES, out));
  const double e_flood = max_err(out, expect, N_VALUES);
  int log_error = -1;
  CHECK(shelfi_decode_log_error(dec_ctx, &log_error));
  printf("%s wire: %zu-byte aggregate, max|dec - plain| exact %.3g, flooded %.3g (logError %d)\n",
         palisade_wire ? "PALISADE" : "blob", agg_len, e_exact, e_flood, log_error);
  int ok = e_exact < 1e-7 && e_flood < 1e-6 && log_error >= 0;
  /* error paths: a truncated aggregate, a non-finite weight */
  if (shelfi_decrypt(dec_ctx, agg, agg_len / 2, N_VALUES, out) != SHELFI_ERR_FORMAT) ok = 0;
  float bad[C];
  memcpy(bad, w, sizeof(bad));
  bad[1] = NAN;
  uint8_t* agg2 = NULL;
  size_t agg2_len = 0;
  if (shelfi_weighted_average(dec_ctx, (const uint8_t* const*)blobs, lens, bad, C, &agg2, &agg2_len) !=
      SHELFI_ERR_RANGE)
    ok = 0;
  shelfi_free(agg2);
  free(out);
  shelfi_free(agg);
  for (int c = 0; c < C; ++c) shelfi_free(blobs[c]);
  return ok;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s CRYPTODIR\n", argv[0]);
    return 2;
  }
  char dir[4096];
  snprintf(dir, sizeof(dir), "%s/", argv[1]);
  if (shelfi_abi_version() != SHELFI_ABI_VERSION) {
    fprintf(stderr, "ABI version mismatch\n");
    return 1;
  }
  /* the generating side: keygen writes the reference's three files */
  shelfi_ctx* a = NULL;
  CHECK(shelfi_ctx_create(0, 4, 52, 60, BATCH, 0, &a));
  CHECK(shelfi_set_seed(a, 7));
  CHECK(shelfi_keygen(a, dir));
  /* the aggregating side: another context that only loads the files */
  shelfi_ctx* b = NULL;
  CHECK(shelfi_ctx_create(0, 4, 52, 60, BATCH, 0, &b));
  CHECK(shelfi_load(b, dir));
  shelfi_info ia, ib;
  CHECK(shelfi_ctx_info(a, &ia));
  CHECK(shelfi_ctx_info(b, &ib));
  if (ia.ring_dim != 32768 || ia.num_towers != 4 || ia.key_id != ib.key_id || !ib.palisade_keys) {
    fprintf(stderr, "loaded context differs: N %u L %u key ids %llx %llx palisade %d\n", ia.ring_dim,
            ia.num_towers, (unsigned long long)ia.key_id, (unsigned long long)ib.key_id, ib.palisade_keys);
    return 1;
  }
  /* learner vectors and the plain FedAvg (float32 weights, ckks.cpp:287) */
  double* x[C];
  double* expect = (double*)calloc(N_VALUES, sizeof(double));
  const float w[C] = {0.4f, 0.3f, 0.2f, 0.1f};
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int c = 0; c < C; ++c) {
    x[c] = (double*)malloc(sizeof(double) * N_VALUES);
    for (size_t i = 0; i < N_VALUES; ++i) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      x[c][i] = (double)(float)((double)(s >> 11) * 0x1.0p-53 * 2.0 - 1.0);
      expect[i] += (double)w[c] * x[c][i];
    }
  }
  int ok = round_trip(a, b, 0, x, w, expect) && round_trip(a, b, 1, x, w, expect);
  /* ckks.cpp:265-268: a weight/learner size mismatch is an argument error at this level */
  uint8_t* none = NULL;
  size_t none_len = 0;
  if (shelfi_weighted_average(b, NULL, NULL, w, C, &none, &none_len) != SHELFI_ERR_ARG) ok = 0;
  for (int c = 0; c < C; ++c) free(x[c]);
  free(expect);
  shelfi_ctx_destroy(b);
  shelfi_ctx_destroy(a);
  puts(ok ? "C CLIENT OK" : "C CLIENT FAILED");
  return ok ? 0 : 1;
}
