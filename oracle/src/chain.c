/*
 * chain.c -- run_markov_chain driver of code/launcher.cpp (TEST INFRASTRUCTURE ONLY),
 * plus flat ctypes entry points used by tests/ and bench.py's cpu_baseline leg.
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* la:6-174 */
int orc_run_markov_chain(const double* data, int n, int d, const int* attrisize, double gamma,
                         const double* v, const double* w, const orc_chain_params* p,
                         const int* c_i_init, int32_t* rng_state, int* out_total_cls, int* out_c_i,
                         double* out_loglik, int* out_accepted, int* final_ass) {
    orc_aux A = {n, d, data, attrisize, gamma, v, w, NULL};
    uint8_t* codes = p->fast >= 2 ? orc_codes_rowmajor(&A) : NULL;   /* optimised oracle */
    A.codes = codes;
    orc_rng rng;
    orc_rng_import(&rng, rng_state);
    orc_state s;
    int st = orc_state_alloc(&s, n, d, n + 2);
    if (st) return st;
    orc_pool pool = {0, d, NULL, NULL};
    int* counts = NULL;
    /* la:30-43 initial assignment */
    s.total_cls = p->L;
    if (c_i_init) {
        int mn = c_i_init[0];
        for (int i = 1; i < n; i++) if (c_i_init[i] < mn) mn = c_i_init[i];
        for (int i = 0; i < n; i++) s.c_i[i] = c_i_init[i] - mn;
        s.total_cls = orc_unique_count(s.c_i, n, -1);
    } else {
        for (int i = 0; i < n; i++) s.c_i[i] = (int)(p->L * orc_unif_rand(&rng) + 1) - 1;
    }
    if (s.total_cls > s.cap) { st = ORC_E_ARG; goto out; }
    /* la:46-48: all centers, then all sigmas */
    for (int c = 0; c < s.total_cls && !st; c++)
        st = orc_sample_center_1_cluster(&rng, &A, NULL, s.center + (size_t)c * d);
    for (int c = 0; c < s.total_cls && !st; c++)
        st = orc_sample_sigma_1_cluster(&rng, &A, v, w, s.sigma + (size_t)c * d);
    if (st) goto out;
    s.ncent = s.total_cls;
    st = orc_update_phi(&rng, &A, &s, NULL, 0);   /* la:51 */
    if (st) goto out;
    /* la:67-77 latent pool */
    pool.P = (int64_t)n * p->m * p->thinning;
    pool.center = (double*)malloc(sizeof(double) * (size_t)pool.P * d);
    pool.sigma = (double*)malloc(sizeof(double) * (size_t)pool.P * d);
    if (!pool.center || !pool.sigma) { st = ORC_E_ARG; goto out; }
    st = orc_pool_generate(&rng, &A, &pool);
    if (st) goto out;
    if (p->fast) counts = (int*)calloc((size_t)n + 2, sizeof(int));

    int idx_1_sm = 0;
    const int total = (p->iterations + p->burnin) * p->thinning;
    for (int iter = 0; iter < total; ++iter) {
        int accepted = 0;
        if (p->neal8 && iter % p->n8_step_size == 0) {   /* la:94-103 */
            if (p->fast) {
                st = orc_validate_state(&s);
                if (st) goto out;
                memset(counts, 0, sizeof(int) * ((size_t)n + 2));
                for (int i = 0; i < n; i++) counts[s.c_i[i]]++;
            }
            if (p->fast >= 2) {
                st = orc_neal8_sweep_opt(&A, &s, p->m, &pool, &rng, counts, 0, -1);
                if (st) goto out;
            } else {
                for (int i = 0; i < n; i++) {
                    st = orc_sample_allocation(i, &A, &s, p->m, &pool, &rng, counts);
                    if (st) goto out;
                }
            }
            st = orc_update_phi(&rng, &A, &s, NULL, 0);
            if (st) goto out;
        }
        if (p->split_merge && iter % p->sam_step_size == 0) {   /* la:111-115 */
            st = orc_split_and_merge(&s, &A, p->t, p->r, idx_1_sm, &rng, p->fast, &accepted);
            if (st) goto out;
            idx_1_sm = (idx_1_sm + 1) % n;
        }
        if (iter % 1000 == 0) {                                 /* la:123-129 */
            st = orc_pool_generate(&rng, &A, &pool);
            if (st) goto out;
        }
        const int rec = iter >= p->thinning * p->burnin && iter % p->thinning == 0;
        double ll = 0.0;
        if (rec || !p->fast)                                    /* la:132 */
            ll = p->fast >= 2 ? orc_compute_loglikelihood_opt(&A, &s) : orc_compute_loglikelihood(&A, &s);
        if (rec) {
            int at = iter / p->thinning - p->burnin;
            if (out_total_cls) out_total_cls[at] = s.total_cls;
            if (out_c_i) memcpy(out_c_i + (size_t)at * n, s.c_i, sizeof(int) * (size_t)n);
            if (out_loglik) out_loglik[at] = ll;
            if (out_accepted) out_accepted[at] = accepted;
        }
    }
    if (final_ass) memcpy(final_ass, s.c_i, sizeof(int) * (size_t)n);
out:
    orc_rng_export(&rng, rng_state);
    free(pool.center); free(pool.sigma); free(counts); free(codes);
    orc_state_free(&s);
    return st;
}
