/*
 * split_merge.c -- split-merge move of code/split_merge.cpp (TEST INFRASTRUCTURE ONLY).
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define DATA(A, i, j) ((A)->data[(size_t)(j) * (size_t)(A)->n + (size_t)(i)])

static int count_eq(const int* c, int n, int v) {
    int s = 0;
    for (int i = 0; i < n; i++) s += (c[i] == v);
    return s;
}

static double row_ll(const orc_aux* A, int i, const double* cen, const double* sig) {
    double h = 0.0;
    for (int j = 0; j < A->d; j++)
        h += orc_dhamming((int)DATA(A, i, j), (int)cen[j], sig[j], A->attrisize[j]);
    return h;
}

/* fast >= 2 with A->codes (the optimised oracle, fast.c): the same sums from the two
 * clusters' dhamming tables (bit-identical terms in the same order) */
static int g_tables = 0;
typedef struct { double* t[2]; } two_tabs;
static int tabs_on(const orc_aux* A) { return g_tables && A->codes; }
static void two_tabs_make(two_tabs* T, const orc_aux* A, const double* s0, const double* s1) {
    T->t[0] = (double*)malloc(sizeof(double) * 2 * (size_t)A->d);
    T->t[1] = (double*)malloc(sizeof(double) * 2 * (size_t)A->d);
    orc_cluster_table(A, s0, T->t[0]);
    orc_cluster_table(A, s1, T->t[1]);
}
static void two_tabs_free(two_tabs* T) { free(T->t[0]); free(T->t[1]); }
static double row_ll_k(const orc_aux* A, const two_tabs* T, int k, int i, const double* cen, const double* sig) {
    if (T->t[0]) return orc_row_ll_table(A->codes + (size_t)i * A->d, cen, T->t[k], A->d);
    return row_ll(A, i, cen, sig);
}

/* sm:6-18 logdensity_hig */
static double logdensity_hig(double sigmaj, double v, double w, double m, int* err) {
    double K = orc_norm_const2(w, v, m, err);
    return K - (v + w) * log(1 + exp(-1 / sigmaj) * (m - 1)) - (w + 1) / sigmaj - 2 * log(sigmaj);
}

/* sm:20-94 logprobgs_phi */
static double logprobgs_phi(const orc_state* gs, const orc_state* g, const orc_aux* A, int idx, int* err) {
    const int d = A->d;
    int c = gs->c_i[idx];
    int* members = (int*)malloc(sizeof(int) * (size_t)A->n);
    int nm = 0;
    for (int i = 0; i < A->n; i++) if (gs->c_i[i] == c) members[nm++] = i;
    const double* gsig = g->sigma + (size_t)g->c_i[idx] * d;
    double log_center_prob = 0;
    const double* cstar = gs->center + (size_t)c * d;
    for (int j = 0; j < d; j++) {
        /* compute_prob_centers column j (cf:480-505) */
        const int m_j = A->attrisize[j];
        double z[256];
        for (int l = 0; l < m_j; l++) z[l] = 0.0;
        for (int q = 0; q < nm; q++) {
            int value = (int)DATA(A, members[q], j);
            if (value >= 1 && value <= m_j) z[value - 1]++;
        }
        for (int l = 0; l < m_j; l++) z[l] = (-((double)nm - z[l])) / gsig[j];
        double mx = z[0];
        for (int l = 1; l < m_j; l++) if (z[l] > mx) mx = z[l];
        for (int l = 0; l < m_j; l++) z[l] = exp(z[l] - mx);
        double sum = 0.0;
        for (int l = 0; l < m_j; l++) sum += z[l];
        for (int l = 0; l < m_j; l++) z[l] = z[l] / sum;
        log_center_prob += log(z[(int)cstar[j] - 1]);
    }
    double log_sigma_prob = 0;
    const double* gss = gs->sigma + (size_t)c * d;
    for (int j = 0; j < d; j++) {
        double sumdelta = 0.0;
        for (int q = 0; q < nm; q++) if (DATA(A, members[q], j) == cstar[j]) sumdelta++;
        double new_v = A->v[j] + sumdelta;
        double new_w = A->w[j] + nm - sumdelta;
        log_sigma_prob += logdensity_hig(gss[j], new_v, new_w, A->attrisize[j], err);
    }
    free(members);
    return log_center_prob + log_sigma_prob;
}

/* sm:96-161 logprobgs_c_i */
double orc_logprobgs_c_i(const orc_state* gs, const orc_state* g, const orc_aux* A,
                         const int* S, int nS, int i1, int i2) {
    const int d = A->d;
    double logpgs = 0;
    int c1 = g->c_i[i1], c2 = g->c_i[i2];
    int n1 = count_eq(g->c_i, A->n, c1), n2 = count_eq(g->c_i, A->n, c2);
    two_tabs T = {{NULL, NULL}};
    if (tabs_on(A)) two_tabs_make(&T, A, gs->sigma + (size_t)c1 * d, gs->sigma + (size_t)c2 * d);
    for (int q = 0; q < nS; q++) {
        int s = S[q];
        double probs[2];
        for (int k = 0; k < 2; k++) {
            int cls = k == 0 ? c1 : c2;
            double H = row_ll_k(A, &T, k, s, gs->center + (size_t)cls * d, gs->sigma + (size_t)cls * d);
            int n = (k == 0 ? n1 : n2) - (g->c_i[s] == cls);
            probs[k] = log((double)n) + H;
        }
        double mx = probs[0];
        if (probs[1] > mx) mx = probs[1];
        probs[0] = exp(probs[0] - mx);
        probs[1] = exp(probs[1] - mx);
        double sum = 0.0;
        sum += probs[0]; sum += probs[1];
        probs[0] = probs[0] / sum;
        probs[1] = probs[1] / sum;
        int cur = gs->c_i[s] == c1 ? 0 : 1;
        logpgs += log(probs[cur]);
    }
    two_tabs_free(&T);
    return logpgs;
}

/* sm:163-225 split_restricted_gibbs_sampler.  fast: counts of c1/c2 tracked incrementally. */
int orc_restricted_gibbs(const int* S, int nS, orc_state* s, int i1, int i2, const orc_aux* A,
                         int t, orc_rng* r, int fast) {
    const int d = A->d;
    int c1 = s->c_i[i1], c2 = s->c_i[i2];
    g_tables = fast >= 2;
    for (int iter = 0; iter < t; ++iter) {
        int n1 = 0, n2 = 0;
        if (fast) { n1 = count_eq(s->c_i, A->n, c1); n2 = count_eq(s->c_i, A->n, c2); }
        two_tabs T = {{NULL, NULL}};
        if (fast >= 2 && A->codes) two_tabs_make(&T, A, s->sigma + (size_t)c1 * d, s->sigma + (size_t)c2 * d);
        for (int q = 0; q < nS; q++) {
            int sp = S[q];
            double probs[2];
            for (int k = 0; k < 2; k++) {
                int cls = k == 0 ? c1 : c2;
                double H = row_ll_k(A, &T, k, sp, s->center + (size_t)cls * d, s->sigma + (size_t)cls * d);
                int n = fast ? (k == 0 ? n1 : n2) - (s->c_i[sp] == cls)
                             : count_eq(s->c_i, A->n, cls) - (s->c_i[sp] == cls);
                probs[k] = log((double)n) + H;
            }
            double mx = probs[0];
            if (probs[1] > mx) mx = probs[1];
            probs[0] = exp(probs[0] - mx);
            probs[1] = exp(probs[1] - mx);
            double sum = 0.0;
            sum += probs[0]; sum += probs[1];
            probs[0] = probs[0] / sum;
            probs[1] = probs[1] / sum;
            int pick;
            int st = orc_sample_prob1(r, probs, 2, &pick);
            if (st) { two_tabs_free(&T); return st; }
            int newc = pick == 0 ? c1 : c2;
            if (fast && newc != s->c_i[sp]) {
                if (s->c_i[sp] == c1) { n1--; n2++; } else { n2--; n1++; }
            }
            s->c_i[sp] = newc;
        }
        two_tabs_free(&T);
        int idx[2] = {c1, c2};
        int st = orc_update_phi(r, A, s, idx, 2);
        if (st) return st;
        st = orc_validate_state(s);
        if (st) return st;
    }
    return ORC_OK;
}

/* sm:393-417 loglikelihood_hamming */
static double loglikelihood_hamming(const orc_state* s, int c, const orc_aux* A) {
    double ll = 0.0;
    const double* cen = s->center + (size_t)c * A->d;
    const double* sig = s->sigma + (size_t)c * A->d;
    if (tabs_on(A)) {
        double* t = (double*)malloc(sizeof(double) * 2 * (size_t)A->d);
        orc_cluster_table(A, sig, t);
        for (int i = 0; i < A->n; i++)
            if (s->c_i[i] == c) {
                const uint8_t* x = A->codes + (size_t)i * A->d;
                for (int j = 0; j < A->d; j++) ll += t[2 * j + ((int)x[j] != (int)cen[j])];
            }
        free(t);
        return ll;
    }
    for (int i = 0; i < A->n; i++)
        if (s->c_i[i] == c)
            for (int j = 0; j < A->d; j++)
                ll += orc_dhamming((int)DATA(A, i, j), (int)cen[j], sig[j], A->attrisize[j]);
    return ll;
}

/* sm:419-436 priors */
static double priors(const orc_state* s, int c, const orc_aux* A, int* err) {
    const double* sig = s->sigma + (size_t)c * A->d;
    double priorg = 0;
    for (int j = 0; j < A->d; j++) {
        priorg -= log((double)A->attrisize[j]);
        priorg += logdensity_hig(sig[j], A->v[j], A->w[j], A->attrisize[j], err);
    }
    return priorg;
}

static double min0(double x) { return (x < 0.0) ? x : 0.0; }   /* std::min(0.0, x) */

/* sm:438-487 split_acc_prob */
static double split_acc_prob(const orc_state* sp, const orc_state* st, const orc_state* sl,
                             const orc_state* ml, const int* S, int nS, int i1, int i2,
                             const orc_aux* A, int* err) {
    double alpha = A->gamma;
    double log_prior = 0.0, log_likelihood = 0.0, log_proposal = 0.0;
    log_prior += log(alpha);
    log_prior += lgamma((double)count_eq(sp->c_i, A->n, sp->c_i[i1]));
    log_prior += lgamma((double)count_eq(sp->c_i, A->n, sp->c_i[i2]));
    log_prior += priors(sp, sp->c_i[i1], A, err);
    log_prior += priors(sp, sp->c_i[i2], A, err);
    log_prior -= lgamma((double)count_eq(st->c_i, A->n, st->c_i[i1]));
    log_prior -= priors(st, st->c_i[i1], A, err);
    log_likelihood += loglikelihood_hamming(sp, sp->c_i[i1], A);
    log_likelihood += loglikelihood_hamming(sp, sp->c_i[i2], A);
    log_likelihood -= loglikelihood_hamming(st, st->c_i[i1], A);
    log_proposal += logprobgs_phi(st, ml, A, i1, err);
    log_proposal -= logprobgs_phi(sp, sl, A, i1, err);
    log_proposal -= logprobgs_phi(sp, sl, A, i2, err);
    log_proposal -= orc_logprobgs_c_i(sp, sl, A, S, nS, i1, i2);
    return min0(log_prior + log_likelihood + log_proposal);
}

/* sm:489-540 merge_acc_prob */
static double merge_acc_prob(const orc_state* sm, const orc_state* st, const orc_state* sl,
                             const orc_state* ml, const int* S, int nS, int i1, int i2,
                             const orc_aux* A, int* err) {
    double alpha = A->gamma;
    double log_prior = 0.0, log_likelihood = 0.0, log_proposal = 0.0;
    log_prior += lgamma((double)count_eq(sm->c_i, A->n, sm->c_i[i1]));
    log_prior += priors(sm, sm->c_i[i1], A, err);
    log_prior -= log(alpha);
    log_prior -= lgamma((double)count_eq(st->c_i, A->n, st->c_i[i1]));
    log_prior -= lgamma((double)count_eq(st->c_i, A->n, st->c_i[i2]));
    log_prior -= priors(st, st->c_i[i1], A, err);
    log_prior -= priors(st, st->c_i[i2], A, err);
    log_likelihood += loglikelihood_hamming(sm, sm->c_i[i2], A);
    log_likelihood -= loglikelihood_hamming(st, st->c_i[i1], A);
    log_likelihood -= loglikelihood_hamming(st, st->c_i[i2], A);
    log_proposal += logprobgs_phi(st, sl, A, i1, err);
    log_proposal += logprobgs_phi(st, sl, A, i2, err);
    log_proposal += orc_logprobgs_c_i(st, sl, A, S, nS, i1, i2);
    log_proposal -= logprobgs_phi(sm, ml, A, i2, err);
    return min0(log_prior + log_likelihood + log_proposal);
}

/* sm:303-352 split_launch_state */
static int split_launch_state(const int* S, int nS, const orc_state* st, int i1, int i2, int t,
                              const orc_aux* A, orc_state* sl, orc_rng* r, int fast) {
    const int d = A->d;
    int e = orc_state_copy(sl, st);
    if (e) return e;
    if (st->c_i[i1] == st->c_i[i2]) {
        sl->c_i[i1] = st->total_cls;
        if (sl->ncent + 1 > sl->cap) return ORC_E_ARG;
        e = orc_sample_center_1_cluster(r, A, NULL, sl->center + (size_t)sl->ncent * d);
        if (e) return e;
        e = orc_sample_sigma_1_cluster(r, A, A->v, A->w, sl->sigma + (size_t)sl->ncent * d);
        if (e) return e;
        sl->ncent++;
        sl->total_cls++;
    } else {
        e = orc_sample_center_1_cluster(r, A, NULL, sl->center + (size_t)st->c_i[i1] * d);
        if (e) return e;
        e = orc_sample_sigma_1_cluster(r, A, A->v, A->w, sl->sigma + (size_t)st->c_i[i1] * d);
        if (e) return e;
    }
    e = orc_sample_center_1_cluster(r, A, NULL, sl->center + (size_t)st->c_i[i2] * d);
    if (e) return e;
    e = orc_sample_sigma_1_cluster(r, A, A->v, A->w, sl->sigma + (size_t)st->c_i[i2] * d);
    if (e) return e;
    {
        int ref[2] = {sl->c_i[i1], sl->c_i[i2]};
        for (int q = 0; q < nS; q++) sl->c_i[S[q]] = ref[(int)(2 * orc_unif_rand(r))];
    }
    e = orc_restricted_gibbs(S, nS, sl, i1, i2, A, t, r, fast);
    if (e) return e;
    return orc_validate_state(sl);
}

/* sm:354-391 merge_launch_state */
static int merge_launch_state(const int* S, int nS, const orc_state* st, int i1, int i2, int rr,
                              const orc_aux* A, orc_state* ml, orc_rng* r) {
    const int d = A->d;
    int e = orc_state_copy(ml, st);
    if (e) return e;
    if (ml->c_i[i1] != ml->c_i[i2]) {
        ml->c_i[i1] = ml->c_i[i2];
        for (int q = 0; q < nS; q++) ml->c_i[S[q]] = ml->c_i[i2];
    }
    e = orc_sample_center_1_cluster(r, A, NULL, ml->center + (size_t)ml->c_i[i2] * d);
    if (e) return e;
    e = orc_sample_sigma_1_cluster(r, A, A->v, A->w, ml->sigma + (size_t)ml->c_i[i2] * d);
    if (e) return e;
    e = orc_clean_var(ml, ml, A);
    if (e) return e;
    for (int iter = 0; iter < rr; ++iter) {
        int idx = ml->c_i[i2];
        e = orc_update_phi(r, A, ml, &idx, 1);
        if (e) return e;
    }
    return orc_validate_state(ml);
}

/* sm:542-598 split_and_merge (with select_observations_random, sm:263-301) */
int orc_split_and_merge(orc_state* s, const orc_aux* A, int t, int rr, int idx_1_sm,
                        orc_rng* rng, int fast, int* accepted) {
    const int n = A->n;
    int i1 = idx_1_sm, i2;
    (void)i1;
    *accepted = 0;
    g_tables = fast >= 2;
    /* sample(seq(0, n-1), 2, FALSE): EmpiricalSample without replacement */
    {
        int nn = n;
        int j = (int)(nn * orc_unif_rand(rng));
        int x_j = j;                       /* x = 0..n-1 initially */
        i1 = x_j;
        /* x[j] = x[--nn]: position j now holds n-1 */
        --nn;
        int j2 = (int)(nn * orc_unif_rand(rng));
        i2 = (j2 == j) ? n - 1 : j2;
    }
    int* S = (int*)malloc(sizeof(int) * (size_t)n);
    int nS = 0;
    for (int i = 0; i < n; ++i) {
        if (i == i1 || i == i2) continue;
        if (s->c_i[i] == s->c_i[i1] || s->c_i[i] == s->c_i[i2]) S[nS++] = i;
    }
    orc_state sl, ml, ss;
    int e = orc_state_alloc(&sl, n, A->d, s->cap);
    e |= orc_state_alloc(&ml, n, A->d, s->cap);
    e |= orc_state_alloc(&ss, n, A->d, s->cap);
    if (e) { e = ORC_E_ARG; goto out; }
    e = split_launch_state(S, nS, s, i1, i2, t, A, &sl, rng, fast);
    if (e) goto out;
    e = merge_launch_state(S, nS, s, i1, i2, rr, A, &ml, rng);
    if (e) goto out;
    double acpt;
    int gerr = ORC_OK;
    if (s->c_i[i1] == s->c_i[i2]) {
        orc_state_copy(&ss, &sl);
        e = orc_restricted_gibbs(S, nS, &ss, i1, i2, A, 1, rng, fast);
        if (e) goto out;
        acpt = split_acc_prob(&ss, s, &sl, &ml, S, nS, i1, i2, A, &gerr);
    } else {
        orc_state_copy(&ss, &ml);
        int idx = ss.c_i[i2];
        e = orc_update_phi(rng, A, &ss, &idx, 1);
        if (e) goto out;
        acpt = merge_acc_prob(&ss, s, &sl, &ml, S, nS, i1, i2, A, &gerr);
    }
    if (gerr) { e = gerr; goto out; }
    e = orc_validate_state(&ss);
    if (e) goto out;
    if (log(orc_unif_rand(rng)) < acpt) {
        e = orc_clean_var(s, &ss, A);
        if (e) goto out;
        e = orc_validate_state(s);
        *accepted = 1;
    }
out:
    orc_state_free(&sl); orc_state_free(&ml); orc_state_free(&ss);
    free(S);
    return e;
}
