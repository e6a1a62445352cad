/* Third-party CPU baseline for bench.py (not the product, not the oracle):
 * the reference's row pipeline built on OpenSSL 3's secp256k1 arithmetic
 * (NID_secp256k1, EC_POINT_mul / EC_POINT_add, EVP SHA-256), on std pthreads.
 *
 * The north star names libsecp256k1 as the CPU baseline; it is absent from
 * the image, and SURVEY.md §8(d) names OpenSSL's EC as the fallback, labelled
 * as such.  It is also an arithmetic independent of both the oracle and the
 * product: tests/test_cpu_openssl.py checks its values against the golden
 * stage KATs (the reference's own scripts' numbers) and its flags against the
 * SQL cases and the random-row fixture.
 *
 * Per row (src/cudasp_gpu.cu pipeline):
 *   S = d·T                                   (a7, variable base)
 *   ser = (0x02 | (S.y & 1)) ‖ BE(S.x) ‖ 00000000   (a8, :236-284)
 *   t = SHA256(H(tag) ‖ H(tag) ‖ ser), tag "BIP0352/SharedSecret"  (a9)
 *   P0 = t·G with t the BE digest, not reduced mod n (a10, a11)
 *   F = P0 + B; v = int64 of the top 8 BE bytes of F.x; then F + L_j (a12)
 * A row matches if v, or a label sum's v, is in its outputs list.
 *
 * Keys off the curve are refused (-2).  Rows whose tweak OpenSSL refuses (not on the curve) or whose sums hit the
 * point at infinity get flag 0 and are counted in the return value; the
 * reference gives such rows whatever its formulas produce, so this baseline
 * is only meant for valid, generic inputs (bench's synthetic tables).
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t* scan;
  const uint8_t* spend;
  const uint8_t* labels;
  uint32_t label_count;
  const uint8_t* tweaks;
  uint32_t n;
  const int64_t* outputs;
  const uint32_t* offs;
  const uint32_t* lens;
  uint8_t* flags;      /* scan: per-row flag */
  uint8_t* sx;         /* values: 32 B BE S.x per row (may be NULL) */
  uint8_t* t;          /* values: 32 B BE digest per row (may be NULL) */
  int64_t* values;     /* values: n x (1 + label_count) (may be NULL) */
  uint32_t next;       /* next row block (atomic) */
  uint32_t refused;    /* rows refused (atomic) */
  int error;
} job_t;

enum { BLOCK = 64 };

static int set_point(const EC_GROUP* g, EC_POINT* p, const uint8_t le64[64], BN_CTX* ctx) {
  BIGNUM* x = BN_lebin2bn(le64, 32, NULL);
  BIGNUM* y = BN_lebin2bn(le64 + 32, 32, NULL);
  const int ok = x && y && EC_POINT_set_affine_coordinates(g, p, x, y, ctx) == 1;
  BN_free(x);
  BN_free(y);
  return ok;
}

/* v of a point: the signed int64 of the top 8 big-endian bytes of x */
static int x_top64(const EC_GROUP* g, const EC_POINT* p, BIGNUM* x, BN_CTX* ctx, int64_t* v) {
  uint8_t be[32];
  if (EC_POINT_is_at_infinity(g, p)) return 0;
  if (EC_POINT_get_affine_coordinates(g, p, x, NULL, ctx) != 1) return 0;
  if (BN_bn2binpad(x, be, 32) != 32) return 0;
  uint64_t u = 0;
  for (int i = 0; i < 8; i++) u = (u << 8) | be[i];
  *v = (int64_t)u;
  return 1;
}

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  EC_GROUP* g = EC_GROUP_new_by_curve_name(NID_secp256k1);
  BN_CTX* ctx = BN_CTX_new();
  EVP_MD_CTX* mid = EVP_MD_CTX_new();
  EVP_MD_CTX* h = EVP_MD_CTX_new();
  const uint32_t nl = j->label_count;
  EC_POINT *T = NULL, *S = NULL, *P0 = NULL, *F = NULL, *B = NULL, *FL = NULL;
  EC_POINT** L = NULL;
  BIGNUM *d = NULL, *tb = NULL, *x = NULL, *y = NULL;
  int ok = g && ctx && mid && h;
  if (ok) {
    T = EC_POINT_new(g);
    S = EC_POINT_new(g);
    P0 = EC_POINT_new(g);
    F = EC_POINT_new(g);
    B = EC_POINT_new(g);
    FL = EC_POINT_new(g);
    L = (EC_POINT**)calloc(nl ? nl : 1, sizeof(EC_POINT*));
    d = BN_lebin2bn(j->scan, 32, NULL);
    tb = BN_new();
    x = BN_new();
    y = BN_new();
    ok = T && S && P0 && F && B && FL && L && d && tb && x && y;
  }
  /* the fixed base's precomputation, as libsecp256k1's ecmult_gen context */
  ok = ok && EC_GROUP_precompute_mult(g, ctx) == 1;
  /* the spend and label keys: OpenSSL holds only points on the curve */
  int keys_ok = ok && set_point(g, B, j->spend, ctx);
  for (uint32_t k = 0; keys_ok && k < nl; k++) {
    L[k] = EC_POINT_new(g);
    keys_ok = L[k] && set_point(g, L[k], j->labels + 64 * (size_t)k, ctx);
  }
  if (ok && !keys_ok) {
    __atomic_store_n(&j->error, 2, __ATOMIC_RELAXED);
    ERR_clear_error();
    ok = 0;
  }
  /* the constant first block H(tag) ‖ H(tag) as a SHA-256 midstate */
  uint8_t tag[32];
  unsigned int tl = 0;
  ok = ok && EVP_Digest("BIP0352/SharedSecret", 20, tag, &tl, EVP_sha256(), NULL) == 1;
  ok = ok && EVP_DigestInit_ex(mid, EVP_sha256(), NULL) == 1 && EVP_DigestUpdate(mid, tag, 32) == 1 &&
       EVP_DigestUpdate(mid, tag, 32) == 1;
  if (!ok && !__atomic_load_n(&j->error, __ATOMIC_RELAXED)) {
    __atomic_store_n(&j->error, 1, __ATOMIC_RELAXED);
    ERR_print_errors_fp(stderr);
  }
  while (ok) {
    const uint32_t r0 = __atomic_fetch_add(&j->next, BLOCK, __ATOMIC_RELAXED);
    if (r0 >= j->n) break;
    const uint32_t r1 = r0 + BLOCK < j->n ? r0 + BLOCK : j->n;
    for (uint32_t r = r0; r < r1; r++) {
      int64_t* vals = j->values ? j->values + (size_t)r * (1 + nl) : NULL;
      if (j->flags) j->flags[r] = 0;
      uint8_t ser[37], be[32], dig[32];
      int good = set_point(g, T, j->tweaks + 64 * (size_t)r, ctx) && EC_POINT_mul(g, S, NULL, T, d, ctx) == 1 &&
                 !EC_POINT_is_at_infinity(g, S) && EC_POINT_get_affine_coordinates(g, S, x, y, ctx) == 1 &&
                 BN_bn2binpad(x, be, 32) == 32;
      if (good) {
        ser[0] = (uint8_t)(0x02 | BN_is_odd(y));
        memcpy(ser + 1, be, 32);
        memset(ser + 33, 0, 4);
        unsigned int dl = 0;
        good = EVP_MD_CTX_copy_ex(h, mid) == 1 && EVP_DigestUpdate(h, ser, 37) == 1 &&
               EVP_DigestFinal_ex(h, dig, &dl) == 1 && BN_bin2bn(dig, 32, tb) != NULL &&
               EC_POINT_mul(g, P0, tb, NULL, NULL, ctx) == 1 && EC_POINT_add(g, F, P0, B, ctx) == 1;
        if (j->sx) memcpy(j->sx + 32 * (size_t)r, be, 32);
        if (j->t) memcpy(j->t + 32 * (size_t)r, dig, 32);
      }
      int64_t v = 0;
      good = good && x_top64(g, F, x, ctx, &v);
      if (!good) {
        __atomic_fetch_add(&j->refused, 1, __ATOMIC_RELAXED);
        continue;
      }
      if (vals) vals[0] = v;
      const int64_t* outs = j->outputs ? j->outputs + j->offs[r] : NULL;
      const uint32_t len = j->outputs ? j->lens[r] : 0;
      int hit = 0;
      for (uint32_t k = 0; k < len && !hit; k++) hit = outs[k] == v;
      /* labels in list order, breaking on the first hit (:157-170) unless
       * every value is wanted */
      for (uint32_t k = 0; k < nl && (!hit || vals); k++) {
        int64_t vl = 0;
        if (EC_POINT_add(g, FL, F, L[k], ctx) != 1 || !x_top64(g, FL, x, ctx, &vl)) {
          if (vals) vals[1 + k] = 0;
          continue;
        }
        if (vals) vals[1 + k] = vl;
        for (uint32_t q = 0; q < len && !hit; q++) hit = outs[q] == vl;
      }
      if (j->flags) j->flags[r] = (uint8_t)hit;
    }
  }
  if (L)
    for (uint32_t k = 0; k < nl; k++) EC_POINT_free(L[k]);
  free(L);
  EC_POINT_free(T);
  EC_POINT_free(S);
  EC_POINT_free(P0);
  EC_POINT_free(F);
  EC_POINT_free(B);
  EC_POINT_free(FL);
  BN_free(d);
  BN_free(tb);
  BN_free(x);
  BN_free(y);
  EVP_MD_CTX_free(mid);
  EVP_MD_CTX_free(h);
  BN_CTX_free(ctx);
  EC_GROUP_free(g);
  return NULL;
}

static int run(job_t* j, int threads) {
  if (threads <= 0) threads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  if (!th) return -1;
  int started = 1;
  for (; started < threads; started++)
    if (pthread_create(&th[started], NULL, worker, j) != 0) break;  /* fewer threads: still correct */
  worker(j);
  for (int i = 1; i < started; i++) pthread_join(th[i], NULL);
  free(th);
  return j->error ? -j->error : (int)j->refused;
}

/* Flags of n rows (tweaks: n x 64-byte LE x‖y; outputs CSR), the reference's
 * semantics.  Returns the number of rows refused (>= 0), -2 when the spend
 * key or a label key is not on the curve (OpenSSL cannot hold it; the
 * reference's formulas run on such keys regardless, e.g. the big-endian G of
 * test/sql/cudasp.test:72), or -1 on another OpenSSL error. */
int cudasp_cpu_openssl_scan(const uint8_t scan[32], const uint8_t spend[64], const uint8_t* label_keys,
                            uint32_t label_count, const uint8_t* tweaks, uint32_t n, const int64_t* outputs,
                            const uint32_t* offs, const uint32_t* lens, uint8_t* flags, int threads) {
  job_t j;
  memset(&j, 0, sizeof j);
  j.scan = scan;
  j.spend = spend;
  j.labels = label_keys;
  j.label_count = label_count;
  j.tweaks = tweaks;
  j.n = n;
  j.outputs = outputs;
  j.offs = offs;
  j.lens = lens;
  j.flags = flags;
  return run(&j, threads);
}

/* Per-stage values of n rows: S.x (32 B BE), the tagged hash t (32 B), and
 * v of F and of every F + L_j (n x (1 + label_count) int64). */
int cudasp_cpu_openssl_values(const uint8_t scan[32], const uint8_t spend[64], const uint8_t* label_keys,
                              uint32_t label_count, const uint8_t* tweaks, uint32_t n, uint8_t* sx, uint8_t* t,
                              int64_t* values, int threads) {
  job_t j;
  memset(&j, 0, sizeof j);
  j.scan = scan;
  j.spend = spend;
  j.labels = label_keys;
  j.label_count = label_count;
  j.tweaks = tweaks;
  j.n = n;
  j.sx = sx;
  j.t = t;
  j.values = values;
  return run(&j, threads);
}
