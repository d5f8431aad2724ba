/*
 * rlib.c -- restated third-party numerics the reference calls (TEST INFRASTRUCTURE ONLY).
 *
 *  R RNG       : set.seed -> RNG_Init (50 LCG scrambles, 625 LCG fills, mti = 624),
 *                MT_genrand (MT19937 + tempering, * 2^-32), fixup() into (0,1).
 *                Pinned: tests/golden/r_runif_kat.json (R's runif outputs for seeds 1/42/123).
 *  Rcpp sample : sugar/functions/sample.h  EmpiricalSample, FixupProb, SampleReplace
 *                (+ R's revsort heapsort); Walker alias (>200 significant categories)
 *                is NOT restated -> ORC_E_WALKER.  Parity unpinned (no reference tests).
 *  nmath       : rbeta (Cheng 1978 algorithms BB / BC as in R's rbeta.c).
 *                qbeta(0.1, a, b) only feeds the branch test at hg:359, so it is restated
 *                as the equivalent pbeta(x; a, b) > 0.1 (continued fraction).  Unpinned.
 *  GSL         : gsl_sf_hyperg_2F1_e for a,b,c >= 0, 0 <= x < 0.995 (hyperg_2F1_series),
 *                the only branch the reference reaches (x = (m-1)/m or u(m-1)/(1+u(m-1))).
 */
#include "oracle.h"
#include <math.h>
#include <float.h>
#include <string.h>
#include <stdlib.h>

/* ------------------------------------------------------------------ R RNG */
#define MT_N 624
#define MT_M 397
#define MATRIX_A   0x9908b0dfU
#define UPPER_MASK 0x80000000U
#define LOWER_MASK 0x7fffffffU
#define TEMPERING_MASK_B 0x9d2c5680U
#define TEMPERING_MASK_C 0xefc60000U
static const double i2_32m1 = 2.328306437080797e-10; /* 1/(2^32 - 1) */

void orc_rng_set_seed(orc_rng* r, uint32_t seed) {
    /* RNG_Init: initial scrambling, then fill i_seed[0..624] (dummy[0] is mti) */
    for (int j = 0; j < 50; j++) seed = (69069U * seed + 1U);
    uint32_t fill[625];
    for (int j = 0; j < 625; j++) { seed = (69069U * seed + 1U); fill[j] = seed; }
    for (int j = 0; j < 624; j++) r->mt[j] = fill[j + 1];
    r->mti = 624;  /* FixupSeeds(kind, initial=1): dummy[0] = 624 */
}

static void mt_sgenrand(orc_rng* r, uint32_t seed) {
    for (int i = 0; i < MT_N; i++) {
        r->mt[i] = seed & 0xffff0000U;
        seed = 69069U * seed + 1U;
        r->mt[i] |= (seed & 0xffff0000U) >> 16;
        seed = 69069U * seed + 1U;
    }
    r->mti = MT_N;
}

static double mt_genrand(orc_rng* r) {
    static const uint32_t mag01[2] = {0x0U, MATRIX_A};
    uint32_t y;
    if (r->mti >= MT_N) {
        int kk;
        if (r->mti == MT_N + 1) mt_sgenrand(r, 4357);
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (r->mt[kk] & UPPER_MASK) | (r->mt[kk + 1] & LOWER_MASK);
            r->mt[kk] = r->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (r->mt[kk] & UPPER_MASK) | (r->mt[kk + 1] & LOWER_MASK);
            r->mt[kk] = r->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1];
        }
        y = (r->mt[MT_N - 1] & UPPER_MASK) | (r->mt[0] & LOWER_MASK);
        r->mt[MT_N - 1] = r->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1];
        r->mti = 0;
    }
    y = r->mt[r->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & TEMPERING_MASK_B;
    y ^= (y << 15) & TEMPERING_MASK_C;
    y ^= (y >> 18);
    return ((double)y * 2.3283064365386963e-10);
}

double orc_unif_rand(orc_rng* r) {
    double x = mt_genrand(r);
    if (x <= 0.0) return 0.5 * i2_32m1;
    if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
    return x;
}

void orc_rng_export(const orc_rng* r, int32_t out[625]) {
    out[0] = r->mti;
    for (int i = 0; i < 624; i++) out[i + 1] = (int32_t)r->mt[i];
}
void orc_rng_import(orc_rng* r, const int32_t in[625]) {
    r->mti = in[0];
    for (int i = 0; i < 624; i++) r->mt[i] = (uint32_t)in[i + 1];
}

/* --------------------------------------------------------- Rcpp sample() */
/* R src/main/sort.c revsort: sort a[] descending by heapsort, permuting ib[] alongside. */
void orc_revsort(double* a, int* ib, int n) {
    int l, j, ir, i;
    double ra;
    int ii;
    if (n <= 1) return;
    a--; ib--;
    l = (n >> 1) + 1;
    ir = n;
    for (;;) {
        if (l > 1) {
            l = l - 1;
            ra = a[l];
            ii = ib[l];
        } else {
            ra = a[ir];
            ii = ib[ir];
            a[ir] = a[1];
            ib[ir] = ib[1];
            if (--ir == 1) {
                a[1] = ra;
                ib[1] = ii;
                return;
            }
        }
        i = l;
        j = l << 1;
        while (j <= ir) {
            if (j < ir && a[j] > a[j + 1]) ++j;
            if (ra > a[j]) {
                a[i] = a[j];
                ib[i] = ib[j];
                j += (i = j);
            } else
                j = ir + 1;
        }
        a[i] = ra;
        ib[i] = ii;
    }
}

/* Walker's alias draw (Rcpp sugar sample.h WalkerSample, restated from R src/main/random.c
 * walker_ProbSampleReplace): the table over the FixupProb-normalised p, then one uniform:
 * rU = unif_rand() * n, k = (int) rU, pick k if rU < q[k] + k else its alias a[k].
 * HL holds the entries with q < 1 from the front and the others from the back.  R leaves
 * a[] uninitialised for entries the loop never assigns (they keep q >= 1 in exact
 * arithmetic); here they alias themselves. */
static int walker_pick(const double* p, int n, double u, int* HL, double* q, int* a) {
    int h = -1, l = n;
    for (int i = 0; i < n; i++) {
        q[i] = p[i] * n;
        a[i] = i;
        if (q[i] < 1.) HL[++h] = i; else HL[--l] = i;
    }
    if (h >= 0 && l < n) {
        for (int k = 0; k < n - 1; k++) {
            const int i = HL[k], j = HL[l];
            a[i] = j;
            q[j] += q[i] - 1;
            if (q[j] < 1.) l++;
            if (l >= n) break;
        }
    }
    for (int i = 0; i < n; i++) q[i] += i;
    const double rU = u * n;
    const int k = (int)rU;
    return rU < q[k] ? k : a[k];
}

/* sample(x, 1, TRUE, probs): FixupProb -> (Walker if >200) -> SampleReplace.
 * Returns the 0-based position into x.  probs is not modified (Rcpp clones it). */
static int sample_prob1_impl(orc_rng* r, double rU_given, const double* probs, int n, int* out_index);

int orc_sample_prob1(orc_rng* r, const double* probs, int n, int* out_index) {
    return sample_prob1_impl(r, 0.0, probs, n, out_index);
}

/* The same draw with its uniform given (the optimised oracle draws a sweep's uniforms
 * ahead; FixupProb's failures return before the uniform would be consumed). */
int orc_sample_prob1_u(const double* probs, int n, double rU, int* out_index) {
    return sample_prob1_impl(NULL, rU, probs, n, out_index);
}

static int sample_prob1_impl(orc_rng* r, double rU_given, const double* probs, int n, int* out_index) {
    double  pbuf[256];
    int     permbuf[256];
    double* p = n <= 256 ? pbuf : (double*)malloc(sizeof(double) * (size_t)n);
    int*    perm = n <= 256 ? permbuf : (int*)malloc(sizeof(int) * (size_t)n);
    int st = ORC_OK;
    if (!p || !perm) { st = ORC_E_ARG; goto done; }
    memcpy(p, probs, sizeof(double) * (size_t)n);
    /* FixupProb (Rcpp sample.h, adapted from R random.c) */
    {
        double sum = 0.0;
        int npos = 0;
        for (int i = 0; i < n; i++) {
            if (!isfinite(p[i])) { st = ORC_E_PROB; goto done; }
            if (p[i] < 0) { st = ORC_E_PROB; goto done; }
            if (p[i] > 0) { npos++; sum += p[i]; }
        }
        if (npos == 0) { st = ORC_E_PROB; goto done; }
        for (int i = 0; i < n; i++) p[i] /= sum;
    }
    {
        int nc = 0;
        for (int i = 0; i < n; i++) nc += (n * p[i] > 0.1);
        if (nc > 200) {                                   /* Walker alias (> 200 categories) */
            int* HL = (int*)malloc(sizeof(int) * (size_t)n);
            int* a = (int*)malloc(sizeof(int) * (size_t)n);
            double* q = (double*)malloc(sizeof(double) * (size_t)n);
            if (!HL || !a || !q) st = ORC_E_ARG;
            else *out_index = walker_pick(p, n, r ? orc_unif_rand(r) : rU_given, HL, q, a);
            free(HL); free(a); free(q);
            goto done;
        }
    }
    /* SampleReplace, k = 1 */
    {
        int nm1 = n - 1, j;
        for (int i = 0; i < n; i++) perm[i] = i + 1;
        orc_revsort(p, perm, n);
        for (int i = 1; i < n; i++) p[i] += p[i - 1];
        double rU = r ? orc_unif_rand(r) : rU_given;
        for (j = 0; j < nm1; j++)
            if (rU <= p[j]) break;
        *out_index = perm[j] - 1;
    }
done:
    if (p != pbuf) free(p);
    if (perm != permbuf) free(perm);
    return st;
}

/* sample(n, 1, replace) with one_based = true: EmpiricalSample, size < 2 path. */
int orc_sample_int1(orc_rng* r, int n) { return (int)(n * orc_unif_rand(r) + 1); }

/* ----------------------------------------------------------------- nmath */
#define expmax (DBL_MAX_EXP * M_LN2)

/* R nmath rbeta.c (Cheng 1978, algorithms BB and BC).  The static parameter cache of
 * the original only avoids recomputation; it does not change results. */
double orc_rbeta(orc_rng* rng, double aa, double bb) {
    if (isnan(aa) || isnan(bb) || aa < 0. || bb < 0.) return NAN;
    if (!isfinite(aa) && !isfinite(bb)) return 0.5;
    if (aa == 0. && bb == 0.) return (orc_unif_rand(rng) < 0.5) ? 0. : 1.;
    if (!isfinite(aa) || bb == 0.) return 1.0;
    if (!isfinite(bb) || aa == 0.) return 0.0;

    double a, b, alpha;
    double r, s, t, u1, u2, v, w, y, z;
    double beta, gamma, delta, k1, k2;

    a = fmin(aa, bb);
    b = fmax(aa, bb);
    alpha = a + b;

#define v_w_from__u1_bet(AA)             \
    v = beta * log(u1 / (1.0 - u1));     \
    if (v <= expmax) {                   \
        w = AA * exp(v);                 \
        if (!isfinite(w)) w = DBL_MAX;   \
    } else                               \
        w = DBL_MAX

    if (a <= 1.0) { /* Algorithm BC */
        beta = 1.0 / a;
        delta = 1.0 + b - a;
        k1 = delta * (0.0138889 + 0.0416667 * a) / (b * beta - 0.777778);
        k2 = 0.25 + (0.5 + 0.25 / delta) * a;
        for (;;) {
            u1 = orc_unif_rand(rng);
            u2 = orc_unif_rand(rng);
            if (u1 < 0.5) {
                y = u1 * u2;
                z = u1 * y;
                if (0.25 * u2 + z - y >= k1) continue;
            } else {
                z = u1 * u1 * u2;
                if (z <= 0.25) {
                    v_w_from__u1_bet(b);
                    break;
                }
                if (z >= k2) continue;
            }
            v_w_from__u1_bet(b);
            if (alpha * (log(alpha / (a + w)) + v) - 1.3862944 >= log(z)) break;
        }
        return (aa == a) ? a / (a + w) : w / (a + w);
    } else { /* Algorithm BB */
        beta = sqrt((alpha - 2.0) / (2.0 * a * b - alpha));
        gamma = a + 1.0 / beta;
        do {
            u1 = orc_unif_rand(rng);
            u2 = orc_unif_rand(rng);
            v_w_from__u1_bet(a);
            z = u1 * u1 * u2;
            r = gamma * v - 1.3862944;
            s = a + r - w;
            if (s + 2.609438 >= 5.0 * z) break;
            t = log(z);
            if (s > t) break;
        } while (r + alpha * log(alpha / (b + w)) < t);
        return (aa != a) ? b / (b + w) : w / (b + w);
    }
#undef v_w_from__u1_bet
}

/* Regularized incomplete beta I_x(a,b): modified Lentz continued fraction. */
static double betacf(double a, double b, double x) {
    const double FPMIN = 1e-300, EPS = 1e-16;
    double qab = a + b, qap = a + 1.0, qam = a - 1.0;
    double c = 1.0, d = 1.0 - qab * x / qap;
    if (fabs(d) < FPMIN) d = FPMIN;
    d = 1.0 / d;
    double h = d;
    for (int m = 1; m <= 200000; m++) {
        int m2 = 2 * m;
        double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
        d = 1.0 + aa * d; if (fabs(d) < FPMIN) d = FPMIN;
        c = 1.0 + aa / c; if (fabs(c) < FPMIN) c = FPMIN;
        d = 1.0 / d; h *= d * c;
        aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
        d = 1.0 + aa * d; if (fabs(d) < FPMIN) d = FPMIN;
        c = 1.0 + aa / c; if (fabs(c) < FPMIN) c = FPMIN;
        d = 1.0 / d;
        double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < EPS) break;
    }
    return h;
}

double orc_pbeta(double x, double a, double b) {
    if (x <= 0.0) return 0.0;
    if (x >= 1.0) return 1.0;
    double lbt = lgamma(a + b) - lgamma(a) - lgamma(b) + a * log(x) + b * log1p(-x);
    if (x < (a + 1.0) / (a + b + 2.0)) return exp(lbt) * betacf(a, b, x) / a;
    return 1.0 - exp(lbt) * betacf(b, a, 1.0 - x) / b;
}

/* hg:359 test R::qbeta(0.1, a, b, 1, 0) < x, restated as pbeta(x; a, b) > 0.1. */
int orc_qbeta01_lt(double a, double b, double x) {
    if (isnan(a) || isnan(b) || a < 0 || b < 0) return 0;   /* qbeta -> NaN: comparison false */
    if (b == 0) return 0;                                   /* all mass at 1: qbeta = 1        */
    if (a == 0) return x > 0;                               /* all mass at 0                   */
    return orc_pbeta(x, a, b) > 0.1;
}

/* ------------------------------------------------------------------- GSL */
#define GSL_SUCCESS   0
#define GSL_EMAXITER  11
#define GSL_EDOM      1
#define GSL_EUNIMPL   24
#define GSL_DBL_EPS   2.2204460492503131e-16
#define LOC_EPS       (1000.0 * GSL_DBL_EPS)

static int hyperg_2F1_series(double a, double b, double c, double x, double* val) {
    double sum_pos = 1.0, sum_neg = 0.0, del_pos = 1.0, del_neg = 0.0, del = 1.0, k = 0.0;
    int i = 0;
    if (fabs(c) < GSL_DBL_EPS) return GSL_EUNIMPL;  /* not reachable from the reference */
    do {
        if (++i > 30000) { *val = sum_pos - sum_neg; return GSL_EMAXITER; }
        del *= (a + k) * (b + k) * x / ((c + k) * (k + 1.0));
        if (del > 0.0) {
            del_pos = del;
            sum_pos += del;
        } else if (del == 0.0) {
            del_pos = 0.0;
            del_neg = 0.0;
            break;
        } else {
            del_neg = -del;
            sum_neg -= del;
        }
        k += 1.0;
    } while (fabs((del_pos + del_neg) / (sum_pos - sum_neg)) > GSL_DBL_EPS);
    *val = sum_pos - sum_neg;
    return GSL_SUCCESS;
}

int orc_hyperg_2F1(double a, double b, double c, double x, double* val) {
    const double d = c - a - b;
    *val = 0.0;
    if (x < -1.0 || 1.0 <= x) return GSL_EDOM;
    if (fabs(c - b) < LOC_EPS || fabs(c - a) < LOC_EPS) {   /* pow_omx(x, d) */
        double ln_omx = log(1.0 - x);
        *val = exp(d * ln_omx);
        return GSL_SUCCESS;
    }
    if (a >= 0.0 && b >= 0.0 && c >= 0.0 && x >= 0.0 && x < 0.995)
        return hyperg_2F1_series(a, b, c, x, val);
    return GSL_EUNIMPL;
}

/* Extension (hdpm HDPM_OPT_HIG_LOGSPACE; not the reference): log 2F1.  The reference's
 * series first (a finite value keeps its bits through log); on overflow or maxiter the
 * positive series again with the partial sum rescaled by 2^-960 past 2^960, 10^7 terms. */
static double log2f1_a1_upper(double A, double C, double x) {
    /* 2F1(A, 1; C; x) = (C-1) x^(1-C) (1-x)^(C-A-1) B_x(C-1, A-C+1), upper-tail form */
    double p = C - 1.0, q = A - C + 1.0;
    double lbeta = lgamma(p) + lgamma(q) - lgamma(p + q);
    double lt = q * log1p(-x) + p * log(x) - log(q) + log(betacf(q, p, 1.0 - x)) - lbeta;
    return log(p) - p * log(x) - q * log1p(-x) + lbeta + log1p(-exp(lt));
}

int orc_log_hyperg_2F1(double a, double b, double c, double x, double* lval) {
    double L = NAN;
    if ((a == 1.0 || b == 1.0) && x > 0.0 && x < 1.0) {
        double A = b == 1.0 ? a : b, p = c - 1.0, q = A - c + 1.0;
        if (p > 0.0 && q > 0.0 && x >= (p + 1.0) / (p + q + 2.0)) {
            L = log2f1_a1_upper(A, c, x);
            if (L > 712.0) { *lval = L; return GSL_SUCCESS; }  /* the plain series overflows */
        }
    }
    double plain;
    int st = orc_hyperg_2F1(a, b, c, x, &plain);
    *lval = NAN;
    if (st == GSL_SUCCESS && isfinite(plain)) {
        *lval = log(plain);
        return st;
    }
    if (st != GSL_SUCCESS && st != GSL_EMAXITER) return st;
    if (isfinite(L)) { *lval = L; return GSL_SUCCESS; }
    if (fabs(c - b) < LOC_EPS || fabs(c - a) < LOC_EPS) {
        *lval = (c - a - b) * log(1.0 - x);
        return GSL_SUCCESS;
    }
    double sum = 1.0, del = 1.0, k = 0.0, scale = 0.0;
    int i = 0;
    do {
        if (++i > 10000000) { *lval = log(sum) + scale * M_LN2; return GSL_EMAXITER; }
        del *= (a + k) * (b + k) * x / ((c + k) * (k + 1.0));
        if (del == 0.0) break;
        sum += del;
        if (sum > 0x1p960) {
            sum *= 0x1p-960;
            del *= 0x1p-960;
            scale += 960.0;
        }
        k += 1.0;
    } while (fabs(del / sum) > GSL_DBL_EPS);
    *lval = scale == 0.0 ? log(sum) : log(sum) + scale * M_LN2;
    return GSL_SUCCESS;
}
