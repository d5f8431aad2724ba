/*
 * ffi.c -- flat ctypes entry points into the oracle (TEST INFRASTRUCTURE ONLY).
 * State is passed as caller-owned arrays; `data` is column-major n x d doubles
 * (Rcpp::NumericMatrix layout), centers/sigma are row-per-cluster K x d doubles.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

void orc_ffi_set_seed(uint32_t seed, int32_t* state625) {
    orc_rng r;
    orc_rng_set_seed(&r, seed);
    orc_rng_export(&r, state625);
}

void orc_ffi_runif(int32_t* state625, int64_t n, double* out) {
    orc_rng r;
    orc_rng_import(&r, state625);
    for (int64_t i = 0; i < n; i++) out[i] = orc_unif_rand(&r);
    orc_rng_export(&r, state625);
}

void orc_ffi_rbeta(int32_t* state625, double a, double b, int n, double* out) {
    orc_rng r;
    orc_rng_import(&r, state625);
    for (int i = 0; i < n; i++) out[i] = orc_rbeta(&r, a, b);
    orc_rng_export(&r, state625);
}

int orc_ffi_rhig(int32_t* state625, double v, double w, double m, int n, double* out) {
    orc_rng r;
    orc_rng_import(&r, state625);
    int err = ORC_OK;
    for (int i = 0; i < n && !err; i++) out[i] = orc_rhig1(&r, v, w, m, &err);
    orc_rng_export(&r, state625);
    return err;
}

int orc_ffi_sample_prob1(int32_t* state625, const double* probs, int n, int* out_index) {
    orc_rng r;
    orc_rng_import(&r, state625);
    int st = orc_sample_prob1(&r, probs, n, out_index);
    orc_rng_export(&r, state625);
    return st;
}

double orc_ffi_norm_const2(double d, double c, double m, int* err) {
    *err = ORC_OK;
    return orc_norm_const2(d, c, m, err);
}

void orc_ffi_set_hig_logspace(int on) { orc_set_hig_logspace(on); }

int orc_ffi_qbeta01_lt(double a, double b, double x) { return orc_qbeta01_lt(a, b, x); }
double orc_ffi_pbeta(double x, double a, double b) { return orc_pbeta(x, a, b); }
double orc_ffi_dhamming(int x, int c, double s, int m) { return orc_dhamming(x, c, s, m); }

/* L[i*K + k] = sum_j dhamming(x_ij, center_kj, sigma_kj, m_j) in j order (n8:47-49),
 * H[i*K + k] = #{j : x_ij != center_kj}. */
void orc_ffi_loglik_matrix(const double* data, int n, int d, const int* attrisize,
                           const double* centers, const double* sigma, int K, double* L, int* H) {
    for (int i = 0; i < n; i++)
        for (int k = 0; k < K; k++) {
            double ll = 0.0;
            int h = 0;
            for (int j = 0; j < d; j++) {
                int x = (int)data[(size_t)j * n + i];
                int c = (int)centers[(size_t)k * d + j];
                ll += orc_dhamming(x, c, sigma[(size_t)k * d + j], attrisize[j]);
                h += (x != c);
            }
            if (L) L[(size_t)i * K + k] = ll;
            if (H) H[(size_t)i * K + k] = h;
        }
}

static int load_state(orc_state* s, int n, int d, int cap, const int* c_i, int K,
                      const double* centers, const double* sigma) {
    int st = orc_state_alloc(s, n, d, cap);
    if (st) return st;
    memcpy(s->c_i, c_i, sizeof(int) * (size_t)n);
    memcpy(s->center, centers, sizeof(double) * (size_t)K * d);
    memcpy(s->sigma, sigma, sizeof(double) * (size_t)K * d);
    s->total_cls = K;
    s->ncent = K;
    return ORC_OK;
}

static void store_state(const orc_state* s, int* c_i, int* K, double* centers, double* sigma) {
    memcpy(c_i, s->c_i, sizeof(int) * (size_t)s->n);
    memcpy(centers, s->center, sizeof(double) * (size_t)s->ncent * s->d);
    memcpy(sigma, s->sigma, sizeof(double) * (size_t)s->ncent * s->d);
    *K = s->total_cls;
}

/* One Neal-8 sweep = n calls of sample_allocation in index order (la:95-99); no update_phi.
 * centers/sigma must hold cap rows.  fast: 0 faithful, 1 incremental counts. */
int orc_ffi_neal8_sweep(const double* data, int n, int d, const int* attrisize, double gamma,
                        const double* v, const double* w, int* c_i, int* K, double* centers,
                        double* sigma, int cap, int m, const double* pool_center,
                        const double* pool_sigma, int64_t P, int32_t* state625, int fast,
                        int first, int count) {
    orc_aux A = {n, d, data, attrisize, gamma, v, w, NULL};
    orc_state s;
    int st = load_state(&s, n, d, cap, c_i, *K, centers, sigma);
    if (st) return st;
    orc_pool pool = {P, d, (double*)pool_center, (double*)pool_sigma};
    orc_rng r;
    orc_rng_import(&r, state625);
    int* counts = NULL;
    uint8_t* codes = NULL;
    if (fast) {
        counts = (int*)calloc((size_t)cap + 1, sizeof(int));
        for (int i = 0; i < n; i++) counts[s.c_i[i]]++;
    }
    if (fast >= 2) {
        codes = orc_codes_rowmajor(&A);
        A.codes = codes;
        st = orc_neal8_sweep_opt(&A, &s, m, &pool, &r, counts, first, count);
    } else {
        int last = count < 0 ? n : first + count;
        for (int i = first; i < last && !st; i++) st = orc_sample_allocation(i, &A, &s, m, &pool, &r, counts);
    }
    orc_rng_export(&r, state625);
    store_state(&s, c_i, K, centers, sigma);
    free(counts);
    free(codes);
    orc_state_free(&s);
    return st;
}

int orc_ffi_update_phi(const double* data, int n, int d, const int* attrisize, const double* v,
                       const double* w, const int* c_i, int K, double* centers, double* sigma,
                       const int* idx, int nidx, int32_t* state625) {
    orc_aux A = {n, d, data, attrisize, 0.0, v, w};
    orc_state s;
    int st = load_state(&s, n, d, K > 0 ? K : 1, c_i, K, centers, sigma);
    if (st) return st;
    orc_rng r;
    orc_rng_import(&r, state625);
    st = orc_update_phi(&r, &A, &s, idx, nidx);
    orc_rng_export(&r, state625);
    memcpy(centers, s.center, sizeof(double) * (size_t)K * d);
    memcpy(sigma, s.sigma, sizeof(double) * (size_t)K * d);
    orc_state_free(&s);
    return st;
}

double orc_ffi_compute_loglikelihood(const double* data, int n, int d, const int* attrisize,
                                     const int* c_i, int K, const double* centers, const double* sigma) {
    orc_aux A = {n, d, data, attrisize, 0.0, NULL, NULL, NULL};
    orc_state s;
    if (load_state(&s, n, d, K > 0 ? K : 1, c_i, K, centers, sigma)) return 0.0;
    double ll = orc_compute_loglikelihood(&A, &s);
    orc_state_free(&s);
    return ll;
}

/* the same sum from the cluster tables (fast.c): bit-identical, without N D exp/log */
double orc_ffi_compute_loglikelihood_opt(const double* data, int n, int d, const int* attrisize,
                                         const int* c_i, int K, const double* centers, const double* sigma) {
    orc_aux A = {n, d, data, attrisize, 0.0, NULL, NULL, NULL};
    orc_state s;
    if (load_state(&s, n, d, K > 0 ? K : 1, c_i, K, centers, sigma)) return 0.0;
    uint8_t* codes = orc_codes_rowmajor(&A);
    A.codes = codes;
    double ll = orc_compute_loglikelihood_opt(&A, &s);
    free(codes);
    orc_state_free(&s);
    return ll;
}

void orc_ffi_set_threads(int nthreads) { orc_set_threads(nthreads); }

int orc_ffi_pool_generate(const int* attrisize, int d, const double* v, const double* w, int64_t P,
                          double* pool_center, double* pool_sigma, int32_t* state625) {
    orc_aux A = {0, d, NULL, attrisize, 0.0, v, w};
    orc_pool pool = {P, d, pool_center, pool_sigma};
    orc_rng r;
    orc_rng_import(&r, state625);
    int st = orc_pool_generate(&r, &A, &pool);
    orc_rng_export(&r, state625);
    return st;
}

int orc_ffi_restricted_gibbs(const double* data, int n, int d, const int* attrisize, const double* v,
                             const double* w, const int* S, int nS, int* c_i, int K, double* centers,
                             double* sigma, int i1, int i2, int t, int32_t* state625, int fast) {
    orc_aux A = {n, d, data, attrisize, 0.0, v, w, NULL};
    orc_state s;
    int st = load_state(&s, n, d, K, c_i, K, centers, sigma);
    if (st) return st;
    uint8_t* codes = fast >= 2 ? orc_codes_rowmajor(&A) : NULL;
    A.codes = codes;
    orc_rng r;
    orc_rng_import(&r, state625);
    st = orc_restricted_gibbs(S, nS, &s, i1, i2, &A, t, &r, fast);
    free(codes);
    orc_rng_export(&r, state625);
    int Kout;
    store_state(&s, c_i, &Kout, centers, sigma);
    orc_state_free(&s);
    return st;
}

double orc_ffi_logprobgs_c_i(const double* data, int n, int d, const int* attrisize,
                             const int* gs_c, const double* gs_center, const double* gs_sigma, int gsK,
                             const int* g_c, const int* S, int nS, int i1, int i2) {
    orc_aux A = {n, d, data, attrisize, 0.0, NULL, NULL};
    orc_state gs, g;
    load_state(&gs, n, d, gsK, gs_c, gsK, gs_center, gs_sigma);
    load_state(&g, n, d, gsK, g_c, gsK, gs_center, gs_sigma);
    double out = orc_logprobgs_c_i(&gs, &g, &A, S, nS, i1, i2);
    orc_state_free(&gs);
    orc_state_free(&g);
    return out;
}

int orc_ffi_split_and_merge(const double* data, int n, int d, const int* attrisize, double gamma,
                            const double* v, const double* w, int* c_i, int* K, double* centers,
                            double* sigma, int cap, int t, int r, int idx_1_sm, int32_t* state625,
                            int fast, int* accepted) {
    orc_aux A = {n, d, data, attrisize, gamma, v, w, NULL};
    orc_state s;
    int st = load_state(&s, n, d, cap, c_i, *K, centers, sigma);
    if (st) return st;
    uint8_t* codes = fast >= 2 ? orc_codes_rowmajor(&A) : NULL;
    A.codes = codes;
    orc_rng rng;
    orc_rng_import(&rng, state625);
    st = orc_split_and_merge(&s, &A, t, r, idx_1_sm, &rng, fast, accepted);
    free(codes);
    orc_rng_export(&rng, state625);
    store_state(&s, c_i, K, centers, sigma);
    orc_state_free(&s);
    return st;
}
