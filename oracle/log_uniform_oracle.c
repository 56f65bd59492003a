/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's native log-uniform sampler, used by
 * tests/ and bench.py's cpu_baseline leg as the checker.  The product path
 * (graph-transformer_amd/csrc/log_uniform_sampler.cpp) never links this file.
 *
 * Reference being restated (all paths under /root/reference/U2GNN_pytorch/log_uniform/):
 *   Log_Uniform_Sampler.cpp:10-16  ctor: prob[i] = (log(i+2)-log(i+1))/log(N+1), stored as float
 *   Log_Uniform_Sampler.cpp:23-32  expected_count: -expm1(num_tries*log1p(-prob[i])) as float
 *   Log_Uniform_Sampler.cpp:57-71  sample: draw x~U[0,1), v = lround(exp(x*log N)) - 1,
 *                                  insert into a set until `size` distinct values; count draws
 *   Log_Uniform_Sampler.h:14      engine = std::default_random_engine seeded 1111
 *                                  (libstdc++: minstd_rand0, a=16807, m=2^31-1)
 *   Log_Uniform_Sampler.h:15      std::uniform_real_distribution<double>(0,1), which in libstdc++
 *                                  is generate_canonical<double,53>: two engine draws per double.
 *
 * Parity pin: tests/test_oracle_sampler.py checks this file against sample sets
 * produced by the reference's own C++ compiled from /root/reference
 * (oracle/build_ref_sampler.sh -> oracle/_ref/), stored in tests/golden/.
 *
 * The set is returned SORTED (the reference returns unordered_set iteration order;
 * only the set matters to the loss up to float summation order).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t n;          /* range_max */
    uint64_t state;     /* minstd_rand0 state */
    float *prob;
} lus_oracle;

static uint64_t minstd_next(lus_oracle *s) {
    s->state = (s->state * 16807ULL) % 2147483647ULL;
    return s->state;
}

/* libstdc++ generate_canonical<double, 53>(minstd_rand0): r = max-min+1 = 2^31-2,
 * floor(log2 r) = 30 -> k = ceil(53/30) = 2 draws. tmp is kept as double and
 * multiplied by the long-double r (bits/random.tcc). */
static double canonical(lus_oracle *s) {
    const long double r = 2147483646.0L;
    double sum = 0.0, tmp = 1.0;
    for (int k = 0; k < 2; ++k) {
        sum += (double)(minstd_next(s) - 1ULL) * tmp;
        tmp = (double)((long double)tmp * r);
    }
    double ret = sum / tmp;
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}

void *lus_oracle_create(int64_t n, uint32_t seed) {
    lus_oracle *s = (lus_oracle *)calloc(1, sizeof(lus_oracle));
    s->n = n;
    uint64_t st = seed % 2147483647ULL;
    s->state = st == 0 ? 1 : st;
    s->prob = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i)
        s->prob[i] = (float)((log((double)(i + 2)) - log((double)(i + 1))) / log((double)(n + 1)));
    return s;
}

void lus_oracle_destroy(void *h) {
    lus_oracle *s = (lus_oracle *)h;
    if (!s) return;
    free(s->prob);
    free(s);
}

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* Returns 0 on success, -1 if size > n (the reference would loop forever).
 * out: `size` distinct ids, sorted ascending. */
int lus_oracle_sample(void *h, int64_t size, int64_t *out, int32_t *num_tries) {
    lus_oracle *s = (lus_oracle *)h;
    if (size > s->n || size < 0) return -1;
    /* membership by a byte map over [0, n) — values are always in range because
     * x < 1 => exp(x log n) < n => lround(..) <= n => v <= n-1, and x >= 0 => v >= 0. */
    unsigned char *seen = (unsigned char *)calloc((size_t)s->n + 1, 1);
    int64_t got = 0;
    int32_t tries = 0;
    const double log_n = log((double)s->n);
    while (got != size) {
        tries += 1;
        double x = canonical(s);
        long v = lround(exp(x * log_n)) - 1;
        if (!seen[v]) { seen[v] = 1; out[got++] = v; }
    }
    free(seen);
    qsort(out, (size_t)size, sizeof(int64_t), cmp_i64);
    *num_tries = tries;
    return 0;
}

void lus_oracle_expected_count(void *h, int32_t num_tries, const int64_t *ids, int64_t n, float *out) {
    lus_oracle *s = (lus_oracle *)h;
    for (int64_t i = 0; i < n; ++i)
        out[i] = (float)(-expm1((double)num_tries * log1p(-(double)s->prob[ids[i]])));
}

float lus_oracle_probability(void *h, int64_t idx) {
    return ((lus_oracle *)h)->prob[idx];
}
