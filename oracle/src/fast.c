/*
 * fast.c -- the optimised CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * the same arithmetic and the same draws as the incremental-count
 * restatement in model.c (orc_sample_allocation with counts), so every label, parameter
 * and stream position is bit-identical to it; what changes is where the work is done:
 *   - a cluster's per-attribute dhamming values depend on the data only through x == c
 *     (cf:355-377), so each cluster gets a table of its two values per attribute, evaluated
 *     with the same call, and a point's log-likelihood is the same j-ordered running sum
 *     of table entries (n8:47-49, 84-89);
 *   - a sweep's m + 1 uniforms per point sit at fixed stream positions (n8:65-69, 99-102),
 *     so the sweep's uniforms are drawn ahead, and the log-likelihoods of every point
 *     against the clusters present at the sweep start and against its m latent picks are
 *     computed in parallel (OpenMP) before the serial scan;
 *   - the scan (n8:95-159) runs on one core with incremental counts; a cluster created or
 *     replaced during the sweep (cases 3 and 4) gets its table when it appears and its
 *     log-likelihoods of the following points in parallel chunks of growing length.
 * This is what lets the oracle check the HIP path at the BASELINE sizes (C5: N = 1M), and
 * it is the "optimised CPU" baseline of BASELINE.md.
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define DATA(A, i, j) ((A)->data[(size_t)(j) * (size_t)(A)->n + (size_t)(i)])

static int g_threads = 0;
void orc_set_threads(int n) { g_threads = n; }
static int threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}

uint8_t* orc_codes_rowmajor(const orc_aux* A) {
    uint8_t* x = (uint8_t*)malloc((size_t)A->n * (size_t)A->d + 1);
    if (!x) return NULL;
    const int nt = threads();
    (void)nt;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int i = 0; i < A->n; i++)
        for (int j = 0; j < A->d; j++) x[(size_t)i * A->d + j] = (uint8_t)(int)DATA(A, i, j);
    return x;
}

/* tab[2j] = dhamming on a match, tab[2j + 1] on a mismatch (cf:355-377, same call) */
void orc_cluster_table(const orc_aux* A, const double* sig, double* tab) {
    for (int j = 0; j < A->d; j++) {
        tab[2 * j] = orc_dhamming(1, 1, sig[j], A->attrisize[j]);
        tab[2 * j + 1] = orc_dhamming(0, 1, sig[j], A->attrisize[j]);
    }
}

/* sum_j dhamming(x_j, cen_j, ...) in j order from the table (n8:47-49) */
double orc_row_ll_table(const uint8_t* x, const double* cen, const double* tab, int d) {
    double ll = 0.0;
    for (int j = 0; j < d; j++) ll += tab[2 * j + ((int)x[j] != (int)cen[j])];
    return ll;
}

/* Rcpp sample(cls, 1, TRUE, probs) (n8:99-102), as orc_sample_prob1_u, with one shortcut:
 * when the largest normalised probability is unique and the uniform is <= it, revsort puts it
 * first and the cumulative compare stops there, so the draw is its index without sorting. */
static int sample_prob1_fast(const double* probs, int n, double rU, int* out_index) {
    double sum = 0.0;
    int npos = 0;
    for (int i = 0; i < n; i++) {
        if (!isfinite(probs[i]) || probs[i] < 0) return orc_sample_prob1_u(probs, n, rU, out_index);
        if (probs[i] > 0) { npos++; sum += probs[i]; }
    }
    if (npos == 0) return orc_sample_prob1_u(probs, n, rU, out_index);
    double pmax = -1.0;
    int amax = -1, ties = 0, nc = 0;
    for (int i = 0; i < n; i++) {
        const double p = probs[i] / sum;                       /* FixupProb */
        nc += (n * p > 0.1);
        if (p > pmax) { pmax = p; amax = i; ties = 1; }
        else if (p == pmax) ties++;
    }
    if (nc > 200 || ties != 1 || !(rU <= pmax)) return orc_sample_prob1_u(probs, n, rU, out_index);
    *out_index = amax;
    return ORC_OK;
}

typedef struct {
    int cap;
    double* tab;   /* [cap][2d] */
    int* src;      /* label -> cluster of the sweep start whose parameters it holds, or -1 */
    double** col;  /* label with src -1: its log-likelihoods of the sweep's points
                      [col_lo, col_hi), computed ahead of the scan in parallel chunks */
    int* col_lo;
    int* col_hi;
    int* chunk;    /* next chunk length (doubles per refill: a short-lived label costs little) */
} label_tabs;

static int tabs_reserve(label_tabs* T, int need, int d) {
    if (need <= T->cap) return ORC_OK;
    int nc = T->cap ? T->cap : 16;
    while (nc < need) nc *= 2;
    double* nt = (double*)realloc(T->tab, sizeof(double) * (size_t)nc * 2 * d);
    if (!nt) return ORC_E_ARG;
    T->tab = nt;
    int* ns = (int*)realloc(T->src, sizeof(int) * (size_t)nc);
    if (!ns) return ORC_E_ARG;
    T->src = ns;
    double** ncol = (double**)realloc(T->col, sizeof(double*) * (size_t)nc);
    if (!ncol) return ORC_E_ARG;
    for (int k = T->cap; k < nc; k++) ncol[k] = NULL;
    T->col = ncol;
    int* a = (int*)realloc(T->col_lo, sizeof(int) * (size_t)nc);
    if (!a) return ORC_E_ARG;
    T->col_lo = a;
    a = (int*)realloc(T->col_hi, sizeof(int) * (size_t)nc);
    if (!a) return ORC_E_ARG;
    T->col_hi = a;
    a = (int*)realloc(T->chunk, sizeof(int) * (size_t)nc);
    if (!a) return ORC_E_ARG;
    T->chunk = a;
    T->cap = nc;
    return ORC_OK;
}

/* label c took new parameters at scan position q: its table; its log-likelihoods come in
 * chunks from the next point on (label_ll) */
static int label_fresh(label_tabs* T, const orc_aux* A, const orc_state* s, int c, int np, int q) {
    const int d = A->d;
    orc_cluster_table(A, s->sigma + (size_t)c * d, T->tab + (size_t)c * 2 * d);
    T->src[c] = -1;
    if (!T->col[c]) T->col[c] = (double*)malloc(sizeof(double) * (size_t)np);
    if (!T->col[c]) return ORC_E_ARG;
    T->col_lo[c] = T->col_hi[c] = q + 1;
    T->chunk[c] = 256;
    return ORC_OK;
}

/* the same j-ordered sum the scan would form for point q against label c (src -1), from a
 * chunk computed ahead in parallel */
static double label_ll(label_tabs* T, const orc_aux* A, const orc_state* s, int c, int first, int np, int q) {
    if (q >= T->col_hi[c]) {
        const int d = A->d;
        const int lo = q, hi = q + T->chunk[c] < np ? q + T->chunk[c] : np;
        if (T->chunk[c] < (1 << 16)) T->chunk[c] *= 2;
        double* col = T->col[c];
        const double* cen = s->center + (size_t)c * d;
        const double* tab = T->tab + (size_t)c * 2 * d;
        const uint8_t* X = A->codes;
        const int nt = (int64_t)(hi - lo) * d > 200000 ? threads() : 1;
        (void)nt;
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int p = lo; p < hi; p++) col[p] = orc_row_ll_table(X + (size_t)(first + p) * d, cen, tab, d);
        T->col_lo[c] = lo;
        T->col_hi[c] = hi;
    }
    return T->col[c][q];
}

/* n8:10-160 for points first .. first+count-1 (count < 0: to the end), counts[] maintained
 * as in orc_sample_allocation.  A->codes is required. */
int orc_neal8_sweep_opt(const orc_aux* A, orc_state* s, int m, const orc_pool* pool, orc_rng* r,
                        int* counts, int first, int count) {
    const int n = A->n, d = A->d;
    const uint8_t* X = A->codes;
    if (!X || !counts || m < 1) return ORC_E_ARG;
    const int last = count < 0 ? n : first + count;
    const int np = last - first;
    if (np <= 0) return ORC_OK;
    const int K0 = s->total_cls;
    const int64_t P = pool->P;
    const int nt = threads();
    (void)nt;
    int st = ORC_OK;
    size_t used = 0;                               /* uniforms consumed by the scan */
    label_tabs T = {0, NULL, NULL, NULL, NULL, NULL, NULL};
    double* U = (double*)malloc(sizeof(double) * (size_t)np * (m + 1));
    double* LE = (double*)malloc(sizeof(double) * ((size_t)np * (K0 > 0 ? K0 : 1)));
    double* LL = (double*)malloc(sizeof(double) * (size_t)np * m);
    int64_t* pick = (int64_t*)malloc(sizeof(int64_t) * (size_t)np * m);
    double* probs = NULL;
    double* logn = NULL;
    /* during the scan c_i holds cluster ids that survive relabelling: label = raw2lab[id];
     * case 2's "relabel every k-1 to old_cls" (n8:126-133) becomes one map update */
    int* raw2lab = (int*)malloc(sizeof(int) * ((size_t)K0 + np + 1));
    int* lab2raw = (int*)malloc(sizeof(int) * ((size_t)K0 + np + 1));
    int next_raw = K0;
    if (!U || !LE || !LL || !pick || !raw2lab || !lab2raw || tabs_reserve(&T, K0 + 1, d)) {
        st = ORC_E_ARG;
        goto out;
    }
    for (int k = 0; k < K0; k++) raw2lab[k] = lab2raw[k] = k;

    /* the sweep's uniforms, drawn ahead from a copy of the stream: m picks then the
     * categorical, per point */
    {
        orc_rng r2 = *r;
        for (size_t q = 0; q < (size_t)np * (m + 1); q++) U[q] = orc_unif_rand(&r2);
    }
    for (int k = 0; k < K0; k++) {
        orc_cluster_table(A, s->sigma + (size_t)k * d, T.tab + (size_t)k * 2 * d);
        T.src[k] = k;
    }
    /* parallel: every point against the sweep-start clusters and its m latent picks */
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int q = 0; q < np; q++) {
        const int i = first + q;
        const uint8_t* xi = X + (size_t)i * d;
        for (int k = 0; k < K0; k++)
            LE[(size_t)q * K0 + k] = orc_row_ll_table(xi, s->center + (size_t)k * d, T.tab + (size_t)k * 2 * d, d);
        for (int l = 0; l < m; l++) {
            const int64_t e = (int)((double)P * U[(size_t)q * (m + 1) + l] + 1) - 1;   /* n8:66 */
            pick[(size_t)q * m + l] = e;
            const double* pc = pool->center + (size_t)e * d;
            const double* ps = pool->sigma + (size_t)e * d;
            double ll = 0.0;
            for (int j = 0; j < d; j++) ll += orc_dhamming((int)xi[j], (int)pc[j], ps[j], A->attrisize[j]);
            LL[(size_t)q * m + l] = ll;
        }
    }

    /* serial scan: n8:29-159 with incremental counts */
    logn = (double*)malloc(sizeof(double) * ((size_t)n + 2));
    if (!logn) { st = ORC_E_ARG; goto out; }
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int c = 0; c <= n + 1; c++) logn[c] = log((double)c);
    const double log_factor = log(A->gamma / m);
    int pcap = 0;
    for (int q = 0; q < np && !st; q++) {
        const int i = first + q;
        const int own = raw2lab[s->c_i[i]];
        const int k = s->total_cls;
        const int own_size = counts[own];
        const int k_minus = own_size == 1 ? k - 1 : k;
        if (k + m > pcap) {
            pcap = 2 * (k + m);
            double* np2 = (double*)realloc(probs, sizeof(double) * (size_t)pcap);
            if (!np2) { st = ORC_E_ARG; break; }
            probs = np2;
        }
        double ll_own = 0.0;
        for (int c = 0; c < k; c++) {                                   /* n8:40-56 */
            const double ll = T.src[c] >= 0 ? LE[(size_t)q * K0 + T.src[c]] : label_ll(&T, A, s, c, first, np, q);
            if (c == own) ll_own = ll;
            const int nz = counts[c] - (own == c);
            probs[c] = nz != 0 ? logn[nz] + ll : -INFINITY;             /* logn[k] = log((double)k) */
        }
        used += m;                                                      /* n8:65-69 */
        for (int l = 0; l < m; l++)                                     /* n8:72-92 */
            probs[k + l] = log_factor + ((l == 0 && k_minus < k) ? ll_own : LL[(size_t)q * m + l]);
        {                                                               /* n8:95-96 */
            double mx = probs[0];
            for (int c = 1; c < k + m; c++) if (probs[c] > mx) mx = probs[c];
            for (int c = 0; c < k + m; c++) probs[c] = exp(probs[c] - mx);
            double sum = 0.0;
            for (int c = 0; c < k + m; c++) sum += probs[c];
            for (int c = 0; c < k + m; c++) probs[c] = probs[c] / sum;
        }
        int new_cls;
        st = sample_prob1_fast(probs, k + m, U[(size_t)q * (m + 1) + m], &new_cls);     /* n8:99-102 */
        if (st) break;
        used += 1;
        const int old_cls = own;
        if (own_size != 1 && new_cls < k) {                             /* case 1 (n8:107-112) */
            s->c_i[i] = lab2raw[new_cls];
            counts[old_cls]--; counts[new_cls]++;
        } else if (new_cls < k && own_size == 1) {                      /* case 2 (n8:114-137) */
            s->c_i[i] = lab2raw[new_cls];
            memmove(s->center + (size_t)old_cls * d, s->center + (size_t)(k - 1) * d, sizeof(double) * d);
            memmove(s->sigma + (size_t)old_cls * d, s->sigma + (size_t)(k - 1) * d, sizeof(double) * d);
            if (old_cls != k - 1) {
                memmove(T.tab + (size_t)old_cls * 2 * d, T.tab + (size_t)(k - 1) * 2 * d, sizeof(double) * 2 * d);
                T.src[old_cls] = T.src[k - 1];
                double* t = T.col[old_cls];
                T.col[old_cls] = T.col[k - 1];
                T.col[k - 1] = t;
                T.col_lo[old_cls] = T.col_lo[k - 1];
                T.col_hi[old_cls] = T.col_hi[k - 1];
                T.chunk[old_cls] = T.chunk[k - 1];
            }
            s->ncent -= 1;
            s->total_cls = k - 1;
            counts[old_cls]--; counts[new_cls]++;
            if (old_cls != k - 1) {
                const int r = lab2raw[k - 1];                             /* relabel k-1 -> old_cls */
                raw2lab[r] = old_cls;
                lab2raw[old_cls] = r;
                counts[old_cls] += counts[k - 1];
                counts[k - 1] = 0;
            } else {
                for (int p = 0; p < n; p++) s->c_i[p] = raw2lab[s->c_i[p]];
                for (int r = 0; r < next_raw; r++) raw2lab[r] = r < k ? r : 0;
                for (int r = 0; r < k; r++) lab2raw[r] = r;
                st = orc_validate_state(s);
            }
        } else if (new_cls >= k && own_size != 1) {                     /* case 3 (n8:139-149) */
            const int64_t e = pick[(size_t)q * m + (new_cls - k)];
            raw2lab[next_raw] = k;
            lab2raw[k] = next_raw;
            s->c_i[i] = next_raw++;
            if (s->ncent >= s->cap || tabs_reserve(&T, k + 1, d)) { st = ORC_E_ARG; break; }
            memcpy(s->center + (size_t)s->ncent * d, pool->center + (size_t)e * d, sizeof(double) * d);
            memcpy(s->sigma + (size_t)s->ncent * d, pool->sigma + (size_t)e * d, sizeof(double) * d);
            if (label_fresh(&T, A, s, k, np, q)) { st = ORC_E_ARG; break; }
            s->ncent += 1;
            s->total_cls += 1;
            counts[old_cls]--; counts[k] = 1;
        } else {                                                         /* case 4 (n8:151-158) */
            const int l = new_cls - k;
            if (!(l == 0 && k_minus < k)) {      /* not the singleton's own parameters */
                const int64_t e = pick[(size_t)q * m + l];
                memcpy(s->center + (size_t)old_cls * d, pool->center + (size_t)e * d, sizeof(double) * d);
                memcpy(s->sigma + (size_t)old_cls * d, pool->sigma + (size_t)e * d, sizeof(double) * d);
                if (label_fresh(&T, A, s, old_cls, np, q)) { st = ORC_E_ARG; break; }
            }
        }
    }
out:
    if (raw2lab) {
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int p = 0; p < n; p++) s->c_i[p] = raw2lab[s->c_i[p]];
    }
    for (size_t q = 0; q < used; q++) (void)orc_unif_rand(r);      /* the stream as drawn */
    for (int k = 0; k < T.cap; k++) free(T.col[k]);
    free(U); free(LE); free(LL); free(pick); free(probs); free(logn); free(raw2lab); free(lab2raw); free(T.tab); free(T.src); free(T.col); free(T.col_lo); free(T.col_hi); free(T.chunk);
    return st;
}

/* compute_loglikelihood (cf:379-401): the same running sum over points then attributes,
 * its terms from the cluster tables. */
double orc_compute_loglikelihood_opt(const orc_aux* A, const orc_state* s) {
    const int d = A->d, K = s->total_cls;
    double* tab = (double*)malloc(sizeof(double) * (size_t)(K > 0 ? K : 1) * 2 * d);
    if (!tab || !A->codes) { free(tab); return NAN; }
    for (int k = 0; k < K; k++) orc_cluster_table(A, s->sigma + (size_t)k * d, tab + (size_t)k * 2 * d);
    double ll = 0.0;
    for (int i = 0; i < A->n; i++) {
        const int c = s->c_i[i];
        const uint8_t* x = A->codes + (size_t)i * d;
        const double* cen = s->center + (size_t)c * d;
        const double* t = tab + (size_t)c * 2 * d;
        for (int j = 0; j < d; j++) ll += t[2 * j + ((int)x[j] != (int)cen[j])];
    }
    free(tab);
    return ll;
}
