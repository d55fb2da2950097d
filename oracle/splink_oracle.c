/*
 * splink_oracle.c -- CPU restatement of splink's comparison + EM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product: it
 * is loaded only by tests/, __graft_entry__.smoke() (as the checker) and
 * bench.py's cpu_baseline leg.  The product (splink_amd/, libsplink_hip.so)
 * never links or calls it.
 *
 * Parity pins: the JSON fixtures in tests/golden/, generated from the reference itself
 * (tests/golden/make_golden.py drives /root/reference/splink's SQL generators
 * through sqlite with Spark-semantics UDFs).  Jaro-Winkler exactness beyond the
 * reference's own level expectations (tests/test_spark.py:355-419) rests on the
 * commons-text 1.4 bytecode restatement in SURVEY.md §2.3.
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------- */
/* Jaro-Winkler: commons-text 1.4 JaroWinklerDistance.apply / matches, as     */
/* wrapped by the jar's uk.gov.moj.dash.linkage.JaroWinklerSimilarity.call    */
/* (called from case_statements.py:84,95-96,106-108,250).     */
/* Operates on UTF-16 code units.                                            */
/* ------------------------------------------------------------------------- */
double orc_jaro_winkler_u16(const uint16_t *first, int64_t lf, const uint16_t *second, int64_t ls)
{
    const uint16_t *mx, *mn;
    int64_t lmx, lmn;
    if (lf > ls) { mx = first; lmx = lf; mn = second; lmn = ls; }
    else { mx = second; lmx = ls; mn = first; lmn = lf; }
    int64_t range = lmx / 2 - 1;
    if (range < 0) range = 0;

    int64_t stack_idx[256];
    unsigned char stack_flag[256];
    int64_t *idx = lmn <= 256 ? stack_idx : (int64_t *)malloc(sizeof(int64_t) * (size_t)lmn);
    unsigned char *flag = lmx <= 256 ? stack_flag : (unsigned char *)malloc((size_t)lmx);
    memset(flag, 0, (size_t)lmx);
    int64_t m = 0;
    for (int64_t mi = 0; mi < lmn; mi++) {
        idx[mi] = -1;
        uint16_t c = mn[mi];
        int64_t lo = mi - range > 0 ? mi - range : 0;
        int64_t hi = mi + range + 1 < lmx ? mi + range + 1 : lmx;
        for (int64_t xi = lo; xi < hi; xi++) {
            if (!flag[xi] && c == mx[xi]) { idx[mi] = xi; flag[xi] = 1; m++; break; }
        }
    }
    /* transpositions: k-th matched char of min (min order) vs k-th flagged char of max */
    int64_t t = 0, xi = 0;
    for (int64_t mi = 0; mi < lmn; mi++) {
        if (idx[mi] < 0) continue;
        while (!flag[xi]) xi++;
        if (mn[mi] != mx[xi]) t++;
        xi++;
    }
    int64_t prefix = 0;
    for (int64_t mi = 0; mi < lmn; mi++) {
        if (first[mi] == second[mi]) prefix++;
        else break;
    }
    if (idx != stack_idx) free(idx);
    if (flag != stack_flag) free(flag);
    if (m == 0) return 0.0;
    double md = (double)m;
    double j = ((md / (double)lf + md / (double)ls) + (md - (double)(t / 2)) / md) / 3.0;
    if (j < 0.7) return j;
    double w = 1.0 / (double)lmx;
    if (w > 0.1) w = 0.1;
    return j + (w * (double)prefix) * (1.0 - j);
}

/* ------------------------------------------------------------------------- */
/* Levenshtein: Spark UTF8String.levenshteinDistance (unit costs, code points),*/
/* called from case_statements.py:121,133,135.                                */
/* ------------------------------------------------------------------------- */
int64_t orc_levenshtein_u32(const uint32_t *s, int64_t ls, const uint32_t *t, int64_t lt)
{
    if (ls == 0) return lt;
    if (lt == 0) return ls;
    int64_t stack_row[257] = {0};
    int64_t *row = lt + 1 <= 257 ? stack_row : (int64_t *)malloc(sizeof(int64_t) * (size_t)(lt + 1));
    for (int64_t j = 0; j <= lt; j++) row[j] = j;
    for (int64_t i = 1; i <= ls; i++) {
        int64_t diag = row[0];
        row[0] = i;
        for (int64_t j = 1; j <= lt; j++) {
            int64_t up = row[j];
            int64_t best = diag + (s[i - 1] != t[j - 1]);
            if (up + 1 < best) best = up + 1;
            if (row[j - 1] + 1 < best) best = row[j - 1] + 1;
            row[j] = best;
            diag = up;
        }
    }
    int64_t r = row[lt];
    if (row != stack_row) free(row);
    return r;
}

/* ------------------------------------------------------------------------- */
/* Column programs for the standard comparison templates                      */
/* (case_statements.py:62-141).  Used for the config workloads and the CPU    */
/* baseline; arbitrary CASE expressions are checked by oracle/oracle.py.     */
/* ------------------------------------------------------------------------- */
enum { ORC_EQ = 0, ORC_JW = 1, ORC_LEV = 2 };

typedef struct {
    const uint16_t *u16; const int64_t *off16;   /* UTF-16 code units */
    const uint32_t *u32; const int64_t *off32;   /* code points */
    const uint8_t *valid;
} orc_strcol;

static int eq_u16(const orc_strcol *c, int64_t a, int64_t b)
{
    int64_t la = c->off16[a + 1] - c->off16[a], lb = c->off16[b + 1] - c->off16[b];
    if (la != lb) return 0;
    return memcmp(c->u16 + c->off16[a], c->u16 + c->off16[b], (size_t)la * 2) == 0;
}

/*
 * gamma for one pair and one template column.
 *   EQ  (strict_equality_2, :62-71):            null -1 | equal 1 | 0
 *   JW  (jaro_2/3/4, :81-113):                  null -1 | jw > t[0] -> L-1 | > t[1] -> L-2 | ... | 0
 *   LEV (levenshtein_3/4, :117-141):            null -1 | equal L-1 | ratio <= t[0] -> L-2 | ... | 0
 */
static int gamma_one(int kind, int nlev, const double *thr, const orc_strcol *c, int64_t a, int64_t b)
{
    if (!c->valid[a] || !c->valid[b]) return -1;
    if (kind == ORC_EQ) return eq_u16(c, a, b) ? 1 : 0;
    if (kind == ORC_JW) {
        double jw = orc_jaro_winkler_u16(c->u16 + c->off16[a], c->off16[a + 1] - c->off16[a],
                                         c->u16 + c->off16[b], c->off16[b + 1] - c->off16[b]);
        for (int i = 0; i < nlev - 1; i++)
            if (jw > thr[i]) return nlev - 1 - i;
        return 0;
    }
    /* LEV */
    if (eq_u16(c, a, b)) return nlev - 1;
    int64_t la = c->off32[a + 1] - c->off32[a], lb = c->off32[b + 1] - c->off32[b];
    double den = ((double)la + (double)lb) / 2.0;
    if (den == 0.0) return 0; /* NULL ratio: falls through to else */
    double lev = (double)orc_levenshtein_u32(c->u32 + c->off32[a], la, c->u32 + c->off32[b], lb);
    double ratio = lev / den;
    for (int i = 0; i < nlev - 2; i++)
        if (ratio <= thr[i]) return nlev - 2 - i;
    return 0;
}

int orc_gammas(int K, const int *kinds, const int *nlev, const double *thr /* K x 3 */,
               const orc_strcol *cols_l, const orc_strcol *cols_r, int64_t P,
               const int32_t *pl, const int32_t *pr, int8_t *out /* P x K */)
{
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t p = 0; p < P; p++) {
        for (int k = 0; k < K; k++) {
            /* both sides index the same column layout; for dedupe cols_l == cols_r */
            const orc_strcol *cl = &cols_l[k], *cr = &cols_r[k];
            int g;
            if (cl == cr) {
                g = gamma_one(kinds[k], nlev[k], thr + 3 * k, cl, pl[p], pr[p]);
            } else {
                /* link_only: build a two-table view */
                if (!cl->valid[pl[p]] || !cr->valid[pr[p]]) { g = -1; }
                else {
                    const uint16_t *a = cl->u16 + cl->off16[pl[p]], *b = cr->u16 + cr->off16[pr[p]];
                    int64_t la = cl->off16[pl[p] + 1] - cl->off16[pl[p]], lb = cr->off16[pr[p] + 1] - cr->off16[pr[p]];
                    int eq = la == lb && memcmp(a, b, (size_t)la * 2) == 0;
                    if (kinds[k] == ORC_EQ) g = eq;
                    else if (kinds[k] == ORC_JW) {
                        double jw = orc_jaro_winkler_u16(a, la, b, lb);
                        g = 0;
                        for (int i = 0; i < nlev[k] - 1; i++)
                            if (jw > thr[3 * k + i]) { g = nlev[k] - 1 - i; break; }
                    } else if (eq) g = nlev[k] - 1;
                    else {
                        int64_t ca = cl->off32[pl[p] + 1] - cl->off32[pl[p]], cb = cr->off32[pr[p] + 1] - cr->off32[pr[p]];
                        double den = ((double)ca + (double)cb) / 2.0;
                        g = 0;
                        if (den != 0.0) {
                            double ratio = (double)orc_levenshtein_u32(cl->u32 + cl->off32[pl[p]], ca,
                                                                       cr->u32 + cr->off32[pr[p]], cb) / den;
                            for (int i = 0; i < nlev[k] - 2; i++)
                                if (ratio <= thr[3 * k + i]) { g = nlev[k] - 2 - i; break; }
                        }
                    }
                }
            }
            out[p * K + k] = (int8_t)g;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* E-step (expectation_step.py:167-185, :196-221) and the M-step sufficient   */
/* statistics (maximisation_step.py:41-90).                                   */
/*                                                                           */
/* m/u arrive already quantised the way the reference renders them           */
/* (`cast({p:.35f} as double)`, expectation_step.py:212); lambda and one_minus */
/* are the doubles of `cast({λ} as double)` / `cast({1-λ} as double)`         */
/* (:173-176).  mp = (λ·m1·…·mK) / ((λ·m1·…·mK) + ((1-λ)·u1·…·uK)), products   */
/* left-associative, γ = -1 -> 1.0; a zero denominator makes mp NULL.        */
/*                                                                           */
/* stats layout (doubles):                                                   */
/*   [0] Σ mp (non-null)   [1] rows   [2] non-null rows                       */
/*   then per column k, per level v in -1..L_k-1 (offset lvl_off[k] + v + 1): */
/*   4 values: rows, non-null rows, Σ mp, Σ (1 - mp)                          */
/* ------------------------------------------------------------------------- */
static inline int mp_one(int K, const int8_t *g, const int *lvl_off, double lambda, double one_minus,
                         const double *m, const double *u, double *mp)
{
    double num = lambda, den = one_minus;
    for (int k = 0; k < K; k++) {
        int v = g[k];
        num = num * (v < 0 ? 1.0 : m[lvl_off[k] - k + v]);
    }
    for (int k = 0; k < K; k++) {
        int v = g[k];
        den = den * (v < 0 ? 1.0 : u[lvl_off[k] - k + v]);
    }
    double d = num + den;
    if (d == 0.0) return 0;
    *mp = num / d;
    return 1;
}

/* lvl_off[k] = Σ_{j<k} (L_j + 1): slot of (k, -1); m/u are flattened [Σ L_k] so m index = lvl_off[k]-k+v */
/* Sums over up to billions of pairs: each thread keeps Neumaier-compensated partial sums and the
 * partials are combined in thread order, so the statistics are accurate to a few ulps whatever P and
 * the thread count (a plain running sum drifts by ~1e-9 relative past 1e9 terms, enough to move a
 * float32-cast m / u by an ulp and fail a 1e-9 comparison against an exact evaluation). */
static inline void neu_add(double *s, double *c, double x)
{
    double t = *s + x;
    if (fabs(*s) >= fabs(x)) *c += (*s - t) + x;
    else *c += (x - t) + *s;
    *s = t;
}

/* weight (optional, NULL = 1 per row): rows of `gam` stand for that many pairs each (distinct comparison
 * vectors with their counts, orc_pattern_hist), each term entering the sums as weight x value. */
static int em_stats_impl(int K, const int *nlev, int64_t P, const int8_t *gam, const int64_t *weight, double lambda,
                         double one_minus, const double *m, const double *u, double *stats)
{
    int lvl_off[64];
    int n_slots = 0;
    for (int k = 0; k < K; k++) { lvl_off[k] = n_slots; n_slots += nlev[k] + 1; }
    int n_stats = 3 + 4 * n_slots;
    memset(stats, 0, sizeof(double) * (size_t)n_stats);
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#endif
    double *part = (double *)calloc((size_t)nt * 2 * (size_t)n_stats, sizeof(double));  /* [thread][sum | comp] */
#pragma omp parallel
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        double *loc = part + (size_t)tid * 2 * (size_t)n_stats, *cmp = loc + n_stats;
#pragma omp for schedule(static)
        for (int64_t p = 0; p < P; p++) {
            const int8_t *g = gam + p * K;
            const double w = weight ? (double)weight[p] : 1.0;
            double mp = 0.0;
            int ok = mp_one(K, g, lvl_off, lambda, one_minus, m, u, &mp);
            loc[1] += w;  /* counts stay exact in doubles (< 2^53) */
            if (ok) { neu_add(&loc[0], &cmp[0], w * mp); loc[2] += w; }
            for (int k = 0; k < K; k++) {
                const int o = 3 + 4 * (lvl_off[k] + g[k] + 1);
                loc[o] += w;
                if (ok) {
                    loc[o + 1] += w;
                    neu_add(&loc[o + 2], &cmp[o + 2], w * mp);
                    neu_add(&loc[o + 3], &cmp[o + 3], w * (1.0 - mp));
                }
            }
        }
    }
    for (int i = 0; i < n_stats; i++) {
        double s = 0.0, c = 0.0;
        for (int t = 0; t < nt; t++) {
            const double *loc = part + (size_t)t * 2 * (size_t)n_stats;
            neu_add(&s, &c, loc[i]);
            neu_add(&s, &c, loc[n_stats + i]);
        }
        stats[i] = s + c;
    }
    free(part);
    return n_stats;
}

int orc_em_stats(int K, const int *nlev, int64_t P, const int8_t *gam, double lambda, double one_minus,
                 const double *m, const double *u, double *stats, int n_threads_hint)
{
    (void)n_threads_hint;
    return em_stats_impl(K, nlev, P, gam, NULL, lambda, one_minus, m, u, stats);
}

/* The same statistics from distinct comparison vectors and their pair counts. */
int orc_em_stats_weighted(int K, const int *nlev, int64_t n, const int8_t *gam, const int64_t *count,
                          double lambda, double one_minus, const double *m, const double *u, double *stats)
{
    return em_stats_impl(K, nlev, n, gam, count, lambda, one_minus, m, u, stats);
}

/* Mixed-radix pattern index of each comparison vector, code = Σ_k (γ_k + 1) · Π_{j<k} (L_j + 1) (the
 * packing the device uses; computed here from the γ columns alone), and its histogram (hist may be NULL;
 * out may be NULL).  hist is ADDED to (callers accumulate chunks). */
void orc_pattern_codes(int K, const int *nlev, int64_t P, const int8_t *gam, int64_t n_pat, int32_t *out,
                       int64_t *hist)
{
    int64_t stride[64];
    int64_t s = 1;
    for (int k = 0; k < K; k++) { stride[k] = s; s *= nlev[k] + 1; }
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#endif
    int64_t *part = hist ? (int64_t *)calloc((size_t)nt * (size_t)n_pat, sizeof(int64_t)) : NULL;
#pragma omp parallel
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        int64_t *h = part ? part + (size_t)tid * (size_t)n_pat : NULL;
#pragma omp for schedule(static)
        for (int64_t p = 0; p < P; p++) {
            const int8_t *g = gam + p * K;
            int64_t c = 0;
            for (int k = 0; k < K; k++) c += (int64_t)(g[k] + 1) * stride[k];
            if (out) out[p] = (int32_t)c;
            if (h) h[c] += 1;
        }
    }
    if (part) {
        for (int t = 0; t < nt; t++)
            for (int64_t i = 0; i < n_pat; i++) hist[i] += part[(size_t)t * (size_t)n_pat + i];
        free(part);
    }
}

/* Log-likelihood of the parameters (expectation_step.py:224-272): Σ over pairs of
 * ln(λ·Πm + (1-λ)·Πu), Spark's ln giving NULL (skipped by sum) for arguments <= 0.
 * out[0] = the sum, out[1] = the number of non-NULL terms. */
void orc_log_likelihood(int K, const int *nlev, int64_t P, const int8_t *gam, double lambda, double one_minus,
                        const double *m, const double *u, double *out)
{
    int lvl_off[64];
    int n_slots = 0;
    for (int k = 0; k < K; k++) { lvl_off[k] = n_slots; n_slots += nlev[k] + 1; }
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#endif
    double *part = (double *)calloc((size_t)nt * 3, sizeof(double));  /* [thread][sum, comp, count] */
#pragma omp parallel
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        double *q = part + 3 * (size_t)tid;
#pragma omp for schedule(static)
        for (int64_t p = 0; p < P; p++) {
            const int8_t *g = gam + p * K;
            double num = lambda, den = one_minus;
            for (int k = 0; k < K; k++) num = num * (g[k] < 0 ? 1.0 : m[lvl_off[k] - k + g[k]]);
            for (int k = 0; k < K; k++) den = den * (g[k] < 0 ? 1.0 : u[lvl_off[k] - k + g[k]]);
            const double d = num + den;
            if (d > 0.0) { neu_add(&q[0], &q[1], log(d)); q[2] += 1.0; }
        }
    }
    double s = 0.0, c = 0.0, cnt = 0.0;  /* compensated, in thread order */
    for (int t = 0; t < nt; t++) {
        neu_add(&s, &c, part[3 * t]);
        neu_add(&s, &c, part[3 * t + 1]);
        cnt += part[3 * t + 2];
    }
    free(part);
    out[0] = s + c;
    out[1] = cnt;
}

/* Final scoring pass: mp per pair (NaN where the reference yields NULL). */
void orc_score(int K, const int *nlev, int64_t P, const int8_t *gam, double lambda, double one_minus,
               const double *m, const double *u, double *mp_out)
{
    int lvl_off[64];
    int n_slots = 0;
    for (int k = 0; k < K; k++) { lvl_off[k] = n_slots; n_slots += nlev[k] + 1; }
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < P; p++) {
        double mp;
        mp_out[p] = mp_one(K, gam + p * K, lvl_off, lambda, one_minus, m, u, &mp) ? mp : NAN;
    }
}

/* bayes(p1..pn) = Πp / (Πp + Π(1-p))  (term_frequencies.py:21-46) */
double orc_bayes(int n, const double *p)
{
    double a = p[0], b = 1.0 - p[0];
    for (int i = 1; i < n; i++) { a = a * p[i]; }
    for (int i = 1; i < n; i++) { b = b * (1.0 - p[i]); }
    return a / (a + b);
}
