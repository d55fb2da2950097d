/*
 * oracle_selftest.c -- driver of the CPU oracle for sanitizer builds (TEST INFRASTRUCTURE ONLY).
 *
 * `make -C oracle asan` compiles splink_oracle.c into this one translation unit with
 * -fsanitize=address,undefined (no OpenMP: the pragmas fall away, the arithmetic is the same) and
 * tests/test_oracle_sanitize.py feeds it the golden string pairs, long / surrogate / empty strings
 * and small EM problems.  Every value is printed exactly (%a) so the test can compare it with the
 * reference's fixtures and with the -O2 OpenMP library the other tests use.
 *
 * Input (whitespace-separated integers / hex or decimal doubles), any number of sections:
 *   S n            then n pairs: la a[la] lb b[lb] (UTF-16 units)  ca ca[..] cb cb[..] (code points)
 *                  -> per pair: "jw lev"
 *   G K R P link   then per column: kind nlev t0 t1 t2; per column, R rows: valid n16 u16[n16] n32 u32[n32];
 *                  then P pairs: l r  -> P lines of K gammas (link = 1 runs the two-table branch)
 *   E K P lam one_minus  then nlev[K], m[ΣL], u[ΣL], gammas[P][K]
 *                  -> stats, log-likelihood (sum, count), P scores, bayes of the first min(P, 4) scores
 */
#include "splink_oracle.c"

#include <stdio.h>

static int64_t rd_i(void)
{
    long long v = 0;
    if (scanf("%lld", &v) != 1) { fprintf(stderr, "selftest: bad integer\n"); exit(2); }
    return (int64_t)v;
}

static double rd_d(void)
{
    char buf[128];
    if (scanf("%127s", buf) != 1) { fprintf(stderr, "selftest: bad double\n"); exit(2); }
    return strtod(buf, NULL);
}

/* exact-size heap copies, so the sanitizer sees every out-of-bounds read of the oracle */
static uint16_t *rd_u16(int64_t n)
{
    uint16_t *p = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; i++) p[i] = (uint16_t)rd_i();
    return p;
}

static uint32_t *rd_u32(int64_t n)
{
    uint32_t *p = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; i++) p[i] = (uint32_t)rd_i();
    return p;
}

static void strings(void)
{
    const int64_t n = rd_i();
    for (int64_t i = 0; i < n; i++) {
        const int64_t la = rd_i();
        uint16_t *a = rd_u16(la);
        const int64_t lb = rd_i();
        uint16_t *b = rd_u16(lb);
        const int64_t ca = rd_i();
        uint32_t *x = rd_u32(ca);
        const int64_t cb = rd_i();
        uint32_t *y = rd_u32(cb);
        printf("%a %lld\n", orc_jaro_winkler_u16(a, la, b, lb), (long long)orc_levenshtein_u32(x, ca, y, cb));
        free(a);
        free(b);
        free(x);
        free(y);
    }
}

static void gammas(void)
{
    const int K = (int)rd_i();
    const int64_t R = rd_i(), P = rd_i();
    const int link = (int)rd_i();
    int kinds[64], nlev[64];
    double thr[64 * 3];
    for (int k = 0; k < K; k++) {
        kinds[k] = (int)rd_i();
        nlev[k] = (int)rd_i();
        for (int t = 0; t < 3; t++) thr[3 * k + t] = rd_d();
    }
    orc_strcol cols[64], cols_r[64];
    for (int k = 0; k < K; k++) {
        /* two passes would need the input twice: grow the unit arrays as the rows arrive */
        int64_t cap16 = 16, cap32 = 16, n16 = 0, n32 = 0;
        uint16_t *u16 = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)cap16);
        uint32_t *u32 = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)cap32);
        int64_t *off16 = (int64_t *)malloc(sizeof(int64_t) * (size_t)(R + 1));
        int64_t *off32 = (int64_t *)malloc(sizeof(int64_t) * (size_t)(R + 1));
        uint8_t *valid = (uint8_t *)malloc((size_t)(R > 0 ? R : 1));
        for (int64_t r = 0; r < R; r++) {
            valid[r] = (uint8_t)rd_i();
            off16[r] = n16;
            const int64_t l16 = rd_i();
            if (n16 + l16 > cap16) { cap16 = 2 * (n16 + l16); u16 = (uint16_t *)realloc(u16, sizeof(uint16_t) * (size_t)cap16); }
            for (int64_t i = 0; i < l16; i++) u16[n16++] = (uint16_t)rd_i();
            off32[r] = n32;
            const int64_t l32 = rd_i();
            if (n32 + l32 > cap32) { cap32 = 2 * (n32 + l32); u32 = (uint32_t *)realloc(u32, sizeof(uint32_t) * (size_t)cap32); }
            for (int64_t i = 0; i < l32; i++) u32[n32++] = (uint32_t)rd_i();
        }
        off16[R] = n16;
        off32[R] = n32;
        cols[k].u16 = u16;
        cols[k].off16 = off16;
        cols[k].u32 = u32;
        cols[k].off32 = off32;
        cols[k].valid = valid;
        cols_r[k] = cols[k];
    }
    int32_t *pl = (int32_t *)calloc((size_t)(P > 0 ? P : 1), sizeof(int32_t));
    int32_t *pr = (int32_t *)calloc((size_t)(P > 0 ? P : 1), sizeof(int32_t));
    for (int64_t p = 0; p < P; p++) {
        pl[p] = (int32_t)rd_i();
        pr[p] = (int32_t)rd_i();
    }
    int8_t *out = (int8_t *)malloc((size_t)(P * K > 0 ? P * K : 1));
    orc_gammas(K, kinds, nlev, thr, cols, link ? cols_r : cols, P, pl, pr, out);
    for (int64_t p = 0; p < P; p++) {
        for (int k = 0; k < K; k++) printf(k ? " %d" : "%d", out[p * K + k]);
        printf("\n");
    }
    for (int k = 0; k < K; k++) {
        free((void *)cols[k].u16);
        free((void *)cols[k].off16);
        free((void *)cols[k].u32);
        free((void *)cols[k].off32);
        free((void *)cols[k].valid);
    }
    free(pl);
    free(pr);
    free(out);
}

static void em(void)
{
    const int K = (int)rd_i();
    const int64_t P = rd_i();
    const double lam = rd_d(), one_minus = rd_d();
    int nlev[64], tot = 0, slots = 0;
    for (int k = 0; k < K; k++) {
        nlev[k] = (int)rd_i();
        tot += nlev[k];
        slots += nlev[k] + 1;
    }
    double *m = (double *)malloc(sizeof(double) * (size_t)tot), *u = (double *)malloc(sizeof(double) * (size_t)tot);
    for (int i = 0; i < tot; i++) m[i] = rd_d();
    for (int i = 0; i < tot; i++) u[i] = rd_d();
    int8_t *g = (int8_t *)malloc((size_t)(P * K > 0 ? P * K : 1));
    for (int64_t i = 0; i < P * K; i++) g[i] = (int8_t)rd_i();
    const int n_stats = 3 + 4 * slots;
    double *stats = (double *)malloc(sizeof(double) * (size_t)n_stats);
    orc_em_stats(K, nlev, P, g, lam, one_minus, m, u, stats, 0);
    for (int i = 0; i < n_stats; i++) printf(i ? " %a" : "%a", stats[i]);
    printf("\n");
    double ll[2];
    orc_log_likelihood(K, nlev, P, g, lam, one_minus, m, u, ll);
    printf("%a %a\n", ll[0], ll[1]);
    double *mp = (double *)malloc(sizeof(double) * (size_t)(P > 0 ? P : 1));
    orc_score(K, nlev, P, g, lam, one_minus, m, u, mp);
    for (int64_t p = 0; p < P; p++) printf(p ? " %a" : "%a", mp[p]);
    printf("\n");
    const int nb = P < 4 ? (int)P : 4;
    printf("%a\n", nb > 0 ? orc_bayes(nb, mp) : 0.0);
    free(m);
    free(u);
    free(g);
    free(stats);
    free(mp);
}

int main(void)
{
    char sec[8];
    while (scanf("%7s", sec) == 1) {
        if (sec[0] == 'S') strings();
        else if (sec[0] == 'G') gammas();
        else if (sec[0] == 'E') em();
        else { fprintf(stderr, "selftest: unknown section %s\n", sec); return 2; }
        fflush(stdout);
    }
    return 0;
}
