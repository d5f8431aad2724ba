/*
 * oracle.h -- CPU restatement of the reference sampler (TEST INFRASTRUCTURE ONLY).
 *
 * This directory is the parity oracle for the hdpm MI355X path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product library (split_and_merge_gibbs_sampling_amd/csrc) never links it.
 *
 * It restates, in plain C, the algorithm of Filippo-Galli/Split_and_merge_Gibbs_sampling
 * (code/ *.cpp, snapshot 2025-04-18) together with the third-party numerics the
 * reference calls but does not vendor:
 *   - R's Mersenne-Twister unif_rand + set.seed scrambling       (R src/main/RNG.c)
 *   - Rcpp sugar sample(): EmpiricalSample / FixupProb / SampleReplace + R revsort
 *   - R nmath rbeta (Cheng 1978 BB/BC) and a pbeta-based qbeta(0.1,..) branch test
 *   - GSL gsl_sf_hyperg_2F1_e, positive-series branch (hyperg_2F1_series)
 * Parity status: R's RNG stream is pinned by R's known runif() outputs
 * (tests/golden/r_runif_kat.json).  Everything else is "parity unpinned":
 * the reference needs R + Rcpp + GSL, none of which exist in this image, so it
 * cannot be built or run here ("Oracle").
 *
 * Every function cites the reference file:line it follows.  Abbreviations:
 *   cf = code/common_functions.cpp, n8 = code/neal8.cpp, sm = code/split_merge.cpp,
 *   hg = code/hyperg.cpp, la = code/launcher.cpp.
 */
#ifndef HDPM_ORACLE_H
#define HDPM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (mirror the reference's failure modes) ---- */
#define ORC_OK            0
#define ORC_E_VALIDATE    1   /* validate_state -> Rcpp::stop (cf:146-172)            */
#define ORC_E_GSL         2   /* norm_const2 throw std::runtime_error (hg:38-45)        */
#define ORC_E_PROB        3   /* FixupProb stop(): NA / negative / too few positive      */
#define ORC_E_WALKER      4   /* (no longer returned: Walker alias sampling is restated)  */
#define ORC_E_ARG         5   /* bad argument / allocation failure                       */

/* ---- R MT19937 (R src/main/RNG.c: MT_genrand, RNG_Init, fixup) ---- */
typedef struct {
    int32_t  mti;        /* dummy[0] in R: position inside mt[]                  */
    uint32_t mt[624];
} orc_rng;

void   orc_rng_set_seed(orc_rng* r, uint32_t seed);    /* set.seed(seed), kind = MT   */
double orc_unif_rand(orc_rng* r);                      /* unif_rand() incl. fixup      */
void   orc_rng_export(const orc_rng* r, int32_t out[625]);
void   orc_rng_import(orc_rng* r, const int32_t in[625]);

/* ---- Rcpp sugar sample() pieces ---- */
void orc_revsort(double* a, int* ib, int n);                         /* R sort.c revsort */
int  orc_sample_prob1(orc_rng* r, const double* probs, int n, int* out_index); /* sample(x,1,TRUE,p) -> 0-based index */
int  orc_sample_int1(orc_rng* r, int n);                             /* sample(n,1,..)[0] (1-based value) */

/* ---- R nmath ---- */
double orc_rbeta(orc_rng* r, double aa, double bb);
double orc_pbeta(double x, double a, double b);
int    orc_qbeta01_lt(double a, double b, double x);  /* qbeta(0.1,a,b,1,0) < x */

/* ---- GSL 2F1 (positive series) + HIG numerics (hg) ---- */
int    orc_hyperg_2F1(double a, double b, double c, double x, double* val); /* GSL status */
double orc_norm_const2(double d, double c, double m, int* err);            /* hg:11-48  */
double orc_hyperg2(double a, double b, double c, double x);                /* hg:51-78  */
double orc_lF_conK2(double u, double d, double c, double m, double lK);    /* hg:183-217 */
double orc_bisec_hyper2(double d, double c, double m, double Omega, int* err); /* hg:221-287 */
double orc_rhig1(orc_rng* r, double v, double w, double m, int* err);      /* hg:346-378, n=1 */
/* extension mirrored from hdpm (HDPM_OPT_HIG_LOGSPACE), not the reference: */
int    orc_log_hyperg_2F1(double a, double b, double c, double x, double* lval);
void   orc_set_hig_logspace(int on);

/* ---- model ---- */
double orc_dhamming(int x, int c, double s, int attrisize);               /* cf:355-377 */

typedef struct {
    int n, d;
    const double* data;      /* column-major n x d, like Rcpp::NumericMatrix   */
    const int*    attrisize; /* d                                               */
    double gamma;
    const double* v;         /* d */
    const double* w;         /* d */
    const uint8_t* codes;    /* optional: the same data as row-major n x d uint8 codes
                                (the optimised paths of fast.c; NULL elsewhere)    */
} orc_aux;

typedef struct {
    int  n, d, cap;
    int* c_i;                /* n labels                                        */
    int  total_cls;
    int  ncent;              /* length of center/sigma lists                     */
    double* center;          /* cap x d (row per cluster)                        */
    double* sigma;           /* cap x d                                          */
} orc_state;

typedef struct {
    int64_t P;               /* number of pool entries (n*m*thinning, la:67)     */
    int d;
    double* center;          /* P x d */
    double* sigma;           /* P x d */
} orc_pool;

int  orc_state_alloc(orc_state* s, int n, int d, int cap);
void orc_state_free(orc_state* s);
int  orc_state_copy(orc_state* dst, const orc_state* src);   /* internal_state deep clone (cfh:38-61) */

int    orc_validate_state(const orc_state* s);
int    orc_unique_count(const int* c_i, int n, int skip);    /* unique_classes(_without_index).length() */
int    orc_sample_center_1_cluster(orc_rng* r, const orc_aux* A, const double* const* probs, double* out);
int    orc_sample_sigma_1_cluster(orc_rng* r, const orc_aux* A, const double* v, const double* w, double* out);
int    orc_update_phi(orc_rng* r, const orc_aux* A, orc_state* s, const int* idx, int nidx);  /* cf:511-591 */
double orc_compute_loglikelihood(const orc_aux* A, const orc_state* s);                     /* cf:379-401 */
int    orc_clean_var(orc_state* upd, const orc_state* cur, const orc_aux* A);               /* cf:296-353 */

/* Neal-8 (n8:10-160).  counts==NULL -> reference-faithful O(N) bookkeeping;
 * counts!=NULL -> incremental per-label counts (same arithmetic, same draws). */
int orc_sample_allocation(int idx, const orc_aux* A, orc_state* s, int m, const orc_pool* pool,
                          orc_rng* r, int* counts);
int orc_pool_generate(orc_rng* r, const orc_aux* A, orc_pool* pool);   /* la:74-77 / la:124-128 */

/* ---- optimised oracle (fast.c): same arithmetic and draws, bit-identical results ---- */
void    orc_set_threads(int n);                       /* OpenMP threads (0: default)      */
uint8_t* orc_codes_rowmajor(const orc_aux* A);       /* malloc'd n x d codes              */
void    orc_cluster_table(const orc_aux* A, const double* sig, double* tab);   /* [d][2] */
double  orc_row_ll_table(const uint8_t* x, const double* cen, const double* tab, int d);
int     orc_neal8_sweep_opt(const orc_aux* A, orc_state* s, int m, const orc_pool* pool, orc_rng* r,
                            int* counts, int first, int count);
double  orc_compute_loglikelihood_opt(const orc_aux* A, const orc_state* s);
int     orc_sample_prob1_u(const double* probs, int n, double rU, int* out_index); /* given uniform */

/* split-merge (sm) */
int orc_restricted_gibbs(const int* S, int nS, orc_state* s, int i1, int i2, const orc_aux* A,
                         int t, orc_rng* r, int fast);                            /* sm:163-225 */
double orc_logprobgs_c_i(const orc_state* gs, const orc_state* g, const orc_aux* A,
                         const int* S, int nS, int i1, int i2);                   /* sm:96-161 */
int orc_split_and_merge(orc_state* s, const orc_aux* A, int t, int r, int idx_1_sm,
                        orc_rng* rng, int fast, int* accepted);                   /* sm:542-598 */

/* ---- flat entry points for ctypes (tests / bench cpu_baseline) ---- */
typedef struct {
    int verbose, m, iterations, L, burnin, t, r;
    int neal8, split_merge, n8_step_size, sam_step_size, thinning;
    int fast;                 /* 0 = reference-faithful bookkeeping, 1 = incremental counts */
} orc_chain_params;

/* run_markov_chain (la:6-174).  c_i_init may be NULL (random init with L labels).
 * Outputs (caller-allocated, `iterations` rows):
 *   out_total_cls[it], out_c_i[it*n], out_loglik[it], out_accepted[it]; final_ass[n].
 * rng_state: 625 int32 in/out (R .Random.seed without the kind word). */
int orc_run_markov_chain(const double* data_colmajor, int n, int d, const int* attrisize,
                         double gamma, const double* v, const double* w,
                         const orc_chain_params* p, const int* c_i_init, int32_t* rng_state,
                         int* out_total_cls, int* out_c_i, double* out_loglik, int* out_accepted,
                         int* final_ass);

#ifdef __cplusplus
}
#endif
#endif
