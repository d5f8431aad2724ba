/*
 * hdpm.h -- C ABI of the MI355X-native Neal-8 / split-merge reassignment engine.
 *
 * Drop-in boundary for the hot path of Filippo-Galli/Split_and_merge_Gibbs_sampling.
 * The reference exposes this path as in-process C++ calls behind one Rcpp export; each
 * entry point below names the reference interface it replaces.  An Rcpp adapter that
 * keeps the reference's R-facing signature is given in INTEGRATION.md.
 *
 * Conventions
 *   - The caller owns every host buffer; the context owns device memory.
 *   - Every call returns an int status (HDPM_OK = 0); hdpm_last_error() describes it.
 *     No C++ exception crosses this boundary.
 *   - One context per host thread per GPU.  The library never calls the R API.
 *   - The R random stream (Mersenne-Twister, the 625 words of .Random.seed after the
 *     kind word) lives in the context and is consumed in the reference's order; it can
 *     be set and read back explicitly.
 *   - Categorical data are codes 1..m_j (the reference's NumericMatrix values).
 *     `codes` is row-major N x D uint8; `centers` are K x D doubles (integer-valued, as
 *     the reference's NumericVector centers), `sigma` K x D doubles.
 */
#ifndef HDPM_H
#define HDPM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDPM_OK          0
#define HDPM_E_VALIDATE  1  /* validate_state failed -> Rcpp::stop in the reference      */
#define HDPM_E_GSL       2  /* norm_const2 threw (GSL 2F1 overflow)                         */
#define HDPM_E_PROB      3  /* FixupProb stop(): no positive / non-finite probability      */
#define HDPM_E_WALKER    4  /* Walker alias table (Rcpp sample, > 200 categories) failed  */
#define HDPM_E_ARG       5  /* invalid argument or capacity                                 */
#define HDPM_E_DEVICE    6  /* HIP runtime error                                            */
#define HDPM_E_NODEVICE  7  /* no usable gfx950 device                                      */

typedef struct hdpm_ctx hdpm_ctx;

/* Parameters of run_markov_chain (code/launcher.cpp:7-14), same names and meaning. */
typedef struct {
    int32_t verbose, m, iterations, L, burnin, t, r;
    int32_t neal8, split_merge, n8_step_size, sam_step_size, thinning;
} hdpm_chain_params;

/* Per-context counters (cumulative since hdpm_ctx_create or hdpm_reset_stats). */
typedef struct {
    int64_t sweeps, rounds, restarts, exact_points, moves, checked_rounds, prepass_points;
    double  t_prepass_ms, t_resolve_ms, t_stats_ms, t_host_phi_ms, t_rng_ms, t_loglik_ms, t_exact_ms;
    /* latent pool generation (la:74-77, 124-128): calls, entries, wall time, and for the
     * device generator its phases: stream slice, attempt tables, host walk, values */
    int64_t pool_calls, pool_entries, pool_device_calls;
    double  t_pool_ms, t_pool_mt_ms, t_pool_accept_ms, t_pool_parse_ms, t_pool_values_ms;
    /* update_phi speculated while the device sweeps: passes run, and clusters whose
     * speculative draws were kept (the sweep left them untouched) */
    int64_t phi_spec_runs, phi_spec_clusters;
    /* prepass launches timed with HIP events (every 8th; t_prepass_ms covers these) and
     * their points */
    int64_t prepass_timed, prepass_timed_points;
    /* device random-stream windows generated: all, and those started from the host state
     * (a window that did not cover the next draws) */
    int64_t rng_windows, rng_windows_fresh;
    /* points the prepass could not prove "stay" (exact rows built for them) */
    int64_t listed_points;
    /* split-merge moves (sm:542-598): count, wall time, and its parts: restricted scans
     * on the device (upload + kernels + wait), update_phi draws, acceptance terms */
    int64_t sm_moves;
    double  t_sm_ms, t_sm_scan_ms, t_sm_phi_ms, t_sm_terms_ms;
    /* update_phi on the device (csrc/phi.hip): updates committed there, and updates it
     * handed back to the host (a case it does not restate: Walker, rhig's bisection path, a
     * drift outside its window, ...); the status of the last one (PhiStatus, 0 = ok) */
    int64_t phi_device_calls, phi_device_fallbacks, phi_device_last_status;
    /* update stream slices found in a copy made an iteration ahead, and such copies made */
    int64_t phi_lookahead_hits, phi_lookahead_copies;
    /* next sweeps enqueued before the iteration's update was joined, and those that ran;
     * go decisions refused because the wait kernel's limit was near (the sweep ran
     * unpipelined), and enqueued sweeps gated off on the device and re-run from point 0 */
    int64_t pipe_enqueued, pipe_runs, pipe_refused, pipe_recovered;
    /* device update_phi by composition trees (every pick fixed), and tree-mode updates re-run
     * by the per-start-drift walks (a pick depended on the uniform) */
    int64_t phi_tree_calls, phi_tree_retries;
    /* device pool generations whose entry starts fell back to the sequential host walk (the
     * segment parse's chain left a window: an entry longer than mean + 14 sd; or debug bit 28) */
    int64_t pool_walk_fallbacks;
    /* update_phi speculated on the device beside the sweep (phi_mode device): launched, and
     * committed as the iteration's update (the sweep moved no point) */
    int64_t phi_dspec_launched, phi_dspec_used;
    /* resolver launches by the device-wide fixed-point resolver (k_resolve_fpg) */
    int64_t fpg_launches;
    /* split-merge update_phi calls (sm:221, 387, 584) run on the device */
    int64_t phi_sm_device_calls;
    /* bit s set: a device update_phi was handed back with PhiStatus s (bit 15: the status was
     * ok but the stream position could not be adopted) */
    int64_t phi_fallback_status_mask;
    /* split-merge device updates re-run with a wider drift window (the drift left the first) */
    int64_t phi_sm_window_retries;
    /* k_resolve_fpg launches that gave up at a grid barrier (a workgroup not resident within the
     * limit, HDPM_OPT_FPG_WAIT_US) and were continued from their first undecided point by the
     * one-workgroup resolver */
    int64_t fpg_aborts;
    /* exact-row launches by the mass kernels: a wave per point (k_exact_rows_mass) and a thread
     * per point (k_exact_rows_lanes) */
    int64_t exact_mass_launches, exact_lanes_launches;
    /* launches that listed every point (a context's first launch, or more than half the points
     * expected uncertain: a chain far from convergence) */
    int64_t dense_launches;
    /* split-merge restricted scans walked on many CUs (k_sm_scan_wide), and those that gave up
     * (grid not resident) and ran on one workgroup */
    int64_t sm_wide_scans, sm_wide_fallbacks;
    /* device update_phi calls enqueued on the fast path (csrc/phi.hip launch_phi2: every pick
     * fixed, no copies), and those of them handed to the general kernels or the host */
    int64_t phi_fast_calls, phi_fast_handbacks;
    /* recorded iterations' labels (hdpm_iterations_record, la:145): taken from the host mirror
     * with the sweep's move log applied (12 B per moved point), and downloaded whole (N words) */
    int64_t labels_mirrored, labels_downloaded;
    /* device updates whose stream state came back with their outputs (k_phi2_values copies the
     * block of the position after the draws; no state copy to wait for) */
    int64_t phi_state_direct;
    /* chained device updates (the next iteration's, enqueued behind the current speculation
     * before it ran): launched, committed, and dropped at the go (the update before them was not
     * the one committed) */
    int64_t phi_chain_launched, phi_chain_used, phi_chain_dropped;
    /* sweeps enqueued ahead that the device started itself (k_pipe_wait's own go behind a
     * completed device update, no host round trip), and goes the host could not follow (the
     * chain state is then undefined and the context reports an error; never expected) */
    int64_t pipe_auto, pipe_desync;
    /* restricted Gibbs samplers run as one device chain (every scan, its table update and its
     * update_phi({c1, c2}) enqueued together, sm:163-225): chains, scans run in them, and chains
     * the host continued from their first unfinished scan or update (an update the device handed
     * back, a draw outside the stream window) */
    int64_t sm_chain_runs, sm_chain_scans, sm_chain_resumes;
} hdpm_stats;

int         hdpm_device_count(void);
int         hdpm_ctx_create(int32_t device, hdpm_ctx** out);
void        hdpm_ctx_destroy(hdpm_ctx* ctx);
const char* hdpm_last_error(const hdpm_ctx* ctx);

/* aux_data (code/common_functions.hpp:65-72): data, n, attrisize, gamma, v, w. */
int hdpm_set_data(hdpm_ctx* ctx, const uint8_t* codes, int32_t n, int32_t d, const int32_t* attrisize,
                  double gamma, const double* v, const double* w);

/* R RNG: set.seed(seed) semantics, or the 625-word state (mti, mt[624]). */
int hdpm_rng_set_seed(hdpm_ctx* ctx, uint32_t seed);
int hdpm_rng_set_state(hdpm_ctx* ctx, const int32_t* state625);
int hdpm_rng_get_state(const hdpm_ctx* ctx, int32_t* state625);

/* internal_state (code/common_functions.hpp:32-63): c_i (labels 0..K-1), centers, sigma. */
int hdpm_set_state(hdpm_ctx* ctx, const int32_t* c_i, int32_t K, const double* centers, const double* sigma);
int hdpm_get_state(hdpm_ctx* ctx, int32_t* c_i, int32_t* K, double* centers, double* sigma, int32_t cap);

/* Latent-parameter pool (code/launcher.cpp:67-77): P entries of (center, sigma). */
int hdpm_set_pool(hdpm_ctx* ctx, const double* centers, const double* sigma, int64_t P);
int hdpm_get_pool(hdpm_ctx* ctx, double* centers, double* sigma, int64_t P);
/* Draw P prior entries from the context stream exactly as la:74-77 / la:124-128. */
int hdpm_generate_pool(hdpm_ctx* ctx, int64_t P);

/* One Neal-8 sweep: N calls of sample_allocation (code/neal8.hpp:4-5, neal8.cpp:10-160)
 * in index order, i.e. the loop code/launcher.cpp:95-99.  Consumes m+1 uniforms/point. */
int hdpm_neal8_sweep(hdpm_ctx* ctx, int32_t m);

/* update_phi (code/common_functions.hpp:113, .cpp:511-591); idx == NULL -> all clusters. */
int hdpm_update_phi(hdpm_ctx* ctx, const int32_t* cluster_indexes, int32_t n_idx);

/* compute_loglikelihood (code/common_functions.hpp:105, .cpp:379-401). */
int hdpm_compute_loglikelihood(hdpm_ctx* ctx, double* out);

/* The N x K log-likelihood matrix and integer Hamming counts against the current
 * clusters (code/neal8.cpp:40-50 inner loop), L[i*K+k], H[i*K+k]. */
int hdpm_loglik_matrix(hdpm_ctx* ctx, double* L, int32_t* H);

/* split_restricted_gibbs_sampler (code/split_merge.hpp:13, .cpp:163-225) on the state. */
int hdpm_restricted_gibbs(hdpm_ctx* ctx, const int32_t* S, int32_t nS, int32_t i1, int32_t i2, int32_t t);

/* logprobgs_c_i (code/split_merge.hpp:11, .cpp:96-161): gamma_star = context state,
 * gamma = launch labels g_c_i. */
int hdpm_logprobgs_c_i(hdpm_ctx* ctx, const int32_t* g_c_i, const int32_t* S, int32_t nS, int32_t i1,
                       int32_t i2, double* out);

/* split_and_merge (code/split_merge.hpp:217-219, .cpp:542-598). */
int hdpm_split_and_merge(hdpm_ctx* ctx, int32_t t, int32_t r, int32_t idx_1_sm, int32_t* accepted);

/* run_markov_chain (code/launcher.cpp:6-174).  c_i_init may be NULL (random init with L
 * labels).  Output buffers (any may be NULL): out_total_cls[iterations],
 * out_c_i[iterations * n], out_loglik[iterations], out_accepted[iterations], final_ass[n];
 * out_time_s = wall seconds of the sampling loop (results$time). */
int hdpm_run_markov_chain(hdpm_ctx* ctx, const hdpm_chain_params* p, const int32_t* c_i_init,
                          int32_t* out_total_cls, int32_t* out_c_i, double* out_loglik,
                          int32_t* out_accepted, int32_t* final_ass, double* out_time_s);

/* The two halves of run_markov_chain, for callers that drive the loop themselves:
 * hdpm_init_chain = la:27-77 (initial labels, centers, sigmas, update_phi, latent pool of
 * n*m*thinning entries); hdpm_iteration = one pass of the loop body la:85-132 for
 * iteration `iter` (Neal-8 sweep + update_phi, split-merge, pool regeneration when
 * iter % 1000 == 0, compute_loglikelihood).  idx_1_sm is carried by the caller. */
int hdpm_init_chain(hdpm_ctx* ctx, const hdpm_chain_params* p, const int32_t* c_i_init);
int hdpm_iteration(hdpm_ctx* ctx, const hdpm_chain_params* p, int32_t iter, int32_t* idx_1_sm,
                   int32_t* accepted, double* loglik);
/* `count` consecutive iterations iter0 .. iter0+count-1 (accepted / loglik: count entries
 * each, may be NULL).  Same chain as calling hdpm_iteration for each; between two
 * iterations of the batch the next sweep is launched on the device before this call's
 * host work for the current one is done (the loop of la:85-154 without R in between). */
int hdpm_iterations(hdpm_ctx* ctx, const hdpm_chain_params* p, int32_t iter0, int32_t count, int32_t* idx_1_sm,
                    int32_t* accepted, double* loglik);

/* hdpm_iterations with the saved iterations recorded (la:139-153, the R driver's sampling phase):
 * iteration iter is saved when iter >= thinning * burnin and iter % thinning == 0; the s-th saved
 * iteration of this call writes total_cls[s] (K), c_i[s * n .. s * n + n) (its labels; may be
 * NULL), and appends its K x d centers and sigmas (doubles, as hdpm_get_state) to the context's
 * record, taken with hdpm_record_take.  *nsaved: saved iterations of this call.  Unlike
 * hdpm_get_state between hdpm_iteration calls, nothing is dropped: the next sweep stays
 * pipelined, and a label vector comes from the host's mirror of the labels (kept across sweeps
 * without moves, updated from the sweep's move log otherwise) instead of an N-word download. */
int hdpm_iterations_record(hdpm_ctx* ctx, const hdpm_chain_params* p, int32_t iter0, int32_t count, int32_t* idx_1_sm,
                           int32_t* accepted, double* loglik, int32_t* total_cls, int32_t* c_i, int32_t* nsaved);
/* The recorded centers / sigmas (rows of d doubles, in saved-iteration order) appended since the
 * last take: *nrows is their number; with centers and sigmas non-NULL (nrows rows each) they are
 * copied out and the record is cleared. */
int hdpm_record_take(hdpm_ctx* ctx, double* centers, double* sigmas, int64_t* nrows);

/* Diagnostics / testing. */
/* Draw `count` raw 32-bit MT outputs (MT_genrand before scaling) on the device and advance
 * the context stream past them (same values as `count` host draws). */
int hdpm_rng_fill_device(hdpm_ctx* ctx, int64_t count, uint32_t* out);
int hdpm_get_stats(const hdpm_ctx* ctx, hdpm_stats* out);
int hdpm_reset_stats(hdpm_ctx* ctx);
/* Testing / diagnostics.  mode bit 0: evaluate every point on the exact path (no
 * certainty shortcut); bit 1: print per-phase timings to stderr; bit 2: compute the
 * log-likelihood with the per-point kernel (no regrouping into match counts); bit 3: no
 * snapshot speculation (the resolver decides every uncertain point itself); bit 4: recount
 * the frequency tables every update_phi (no incremental move log); bit 5: accumulate a host
 * timeline of hdpm_iteration (printed to stderr when the context is destroyed); bit 6:
 * generate latent pools with the sequential host generator instead of the device one; bit 7:
 * no speculative update_phi during the sweep; bit 8: no next sweep prepared at the end of
 * an iteration; bit 9: HIP events around every kernel of every launch (per-kernel times);
 * bit 10: the prepass gathers full bound records for latent picks (no pool-entry heads);
 * bit 11: exact rows one wave per point (no workgroup-per-point LDS staging); bit 12: no
 * block mode in the resolver (uncertain points decided one by one); bit 13: block mode for
 * every resolver launch (not only after a launch that listed kResolveBlkMin points); bit 14:
 * wide layouts take the generic prepass (one thread per point) instead of k_prepass_wide; bit 15:
 * the prepared next sweep is launched before the speculative update_phi is started; bit 16:
 * restricted scans of >= 4096 points draw their uniforms on the host (not from the device
 * generator windows); bit 17: a sweep prepared at the end of hdpm_iterations does not start
 * its prepass on the device; bit 18: the prepass certifies "stay" by the margin only (not by
 * the draw's uniform, kernels.hip stay_by_uniform); bit 19: update_phi on the host (the job
 * speculated during the sweep) even when the device update is selected (HDPM_OPT_PHI_DEVICE
 * or HDPM_PHI=device; csrc/phi.hip); bit 20: no lookahead copy of the next update's stream
 * slice (it is copied when the next sweep's draws are reserved); bit 21: the iteration
 * commits the new tables and computes the log-likelihood before it prepares the next sweep
 * (by default the next speculative update_phi is started first); bit 22: no next sweep
 * enqueued while the iteration's update is drawn (gated on the device, k_pipe_wait); bit 23:
 * the one-wave resolvers (LIST mode, block mode after many exact decisions) instead of the
 * fixed-point resolver k_resolve_fp (which bits 0, 12 and 13 also turn off); bit 24: with the
 * fixed-point resolver too, a launch after one that decided many points itself lists every
 * point (no certification by the draw's uniform), as the one-wave resolvers always do; bit 25:
 * the fixed-point resolver for every launch it fits (by default a launch after one that listed
 * fewer than 64 points -- a converged chain -- takes the one-wave LIST resolver); bit 26: the
 * fixed-point resolver's first round starts every point from "stay" instead of its snapshot
 * draw's outcome; bit 27: the device update_phi resolves its drifts by the per-start-drift walks
 * (k_phi_cwalk) instead of the composition trees (k_phi_tree); bit 28: the device pool generator's
 * entry starts by the sequential host walk instead of the segment parse (k_pool_seg*);
 * bit 29: the fixed-point resolver on one workgroup (k_resolve_fp) even after a launch that
 * listed many points (by default those take the device-wide k_resolve_fpg); bit 30: k_resolve_fpg
 * for every fixed-point launch (testing: also the launches with few listed points). */
int hdpm_set_debug(hdpm_ctx* ctx, int32_t mode);
/* The prepass's pool-entry heads, P entries of wb*Ws + 2 words padded to a power of two
 * (Ws <= 4) or to a multiple of 8 words (wide layouts) (csrc/kernels.hpp "Pool-entry heads",
 * head_stride); HDPM_E_ARG when the data's layout has none (Ws > 32, i.e. d > 2048, or rows
 * of more than 64 words: wb * Ws > 64). */
int hdpm_get_pool_heads(hdpm_ctx* ctx, uint64_t* out, int64_t P);
/* Options.  HDPM_OPT_HIG_LOGSPACE (value != 0): an extension beyond the reference -- the
 * HIG normalising constant's 2F1 series (norm_const2, hg:11-48, and lF_conK2, hg:183-217)
 * is summed with a rescaled partial sum, so clusters of thousands of members get a finite
 * log-density where GSL's double series overflows and the reference throws
 * (HDPM_E_GSL); 10^7 series terms instead of 30000.  Wherever the reference's series stays
 * finite within 30000 terms the values are bit-identical.  Default 0 (reference
 * semantics). */
#define HDPM_OPT_HIG_LOGSPACE 1
/* HDPM_OPT_PHI_DEVICE: where update_phi runs.  0: the host job speculated during the sweep;
 * 1: the device (csrc/phi.hip: center draws, rhig's beta-path sigma draws resolved over
 * acceptance masks by composition tables, tables and bound records; the fast path launch_phi2
 * first when every pick is fixed, else the general kernels); 2: the device's general kernels
 * only; 3 (default): automatic -- the device for the chain's update_phi of at least 4096
 * (cluster, attribute) items, where the host job's serial draws outlast the sweep, the host job
 * otherwise and for split-merge's updates.  Cases the device does not restate fall back to the
 * host.  Same chain either way.  HDPM_PHI=host|device|device-general|auto in the environment
 * sets the default. */
#define HDPM_OPT_PHI_DEVICE 2
/* HDPM_OPT_PIPE_WAIT_US (testing): the limit, in microseconds, after which the wait kernel of
 * a sweep enqueued ahead gives up and gates the sweep off (default 2 s).  A positive value
 * also makes the host refuse a go given after a quarter of the limit; a negative value sets
 * the limit to -value without that check, so the device-side gate-off (and the engine's
 * recovery from it: the sweep re-run ungated, same chain) can be exercised. */
#define HDPM_OPT_PIPE_WAIT_US 3
/* HDPM_OPT_FPG_WAIT_US: the limit, in microseconds, after which a grid barrier of the device-wide
 * resolver (k_resolve_fpg) gives up (default 2 s).  A launch that gives up has committed
 * exactly the windows before the barrier; it ends as a restart there and the engine continues
 * with the one-workgroup resolver (same chain; hdpm_stats.fpg_aborts counts these). */
#define HDPM_OPT_FPG_WAIT_US 4
/* HDPM_OPT_FPG_FAIL_AT (testing): workgroup 0 of every k_resolve_fpg launch gives up at its
 * value-th grid barrier (0: never), to exercise that recovery deterministically. */
#define HDPM_OPT_FPG_FAIL_AT 5
/* HDPM_OPT_EXACT_KERNEL (testing): the exact-rows kernel of launches with many listed points:
 * 0 automatic (default), 1 a wave per point (k_exact_rows_mass), 2 a thread per point with
 * compare / select (k_exact_rows_lanes), 3 a thread per point with level-indexed tables
 * (k_exact_rows_lv) -- where the state fits it.  Same chain either way. */
#define HDPM_OPT_EXACT_KERNEL 6
/* HDPM_OPT_LAT_NEGLIGIBLE (testing): the margin (>= 40, default 40) below the best cluster under
 * which a latent entry kept as a head bound by the exact rows counts as probability 0 in a draw;
 * above it the draw computes the latent's exact sum.  A large value sends every such latent to
 * the exact sum (the fallback path).  Same chain either way. */
#define HDPM_OPT_LAT_NEGLIGIBLE 7
/* HDPM_OPT_SM_WIDE_WAIT_US (testing): the grid-barrier limit of the split-merge scan on many CUs
 * (default 50000 us); a scan that gives up writes nothing and is walked on one workgroup
 * (hdpm_stats.sm_wide_fallbacks).  0 gives up at the first barrier, unconditionally; values above
 * 1e9 us are an argument error.  Same chain either way. */
#define HDPM_OPT_SM_WIDE_WAIT_US 8
/* HDPM_OPT_SM_CHAIN: the restricted Gibbs sampler of a split-merge move (sm:163-225, its t scans
 * and update_phi({c1, c2}) calls) as one device chain where it applies (1; also HDPM_SM_CHAIN=1
 * in the environment) or scan by scan with the host between them (0, the default: measured
 * faster at C3 and C4).  Testing:
 * 2 + 3k turns the chain off at scan k (the host continues from there), 3 + 3k / 4 + 3k hand the
 * scan's update of the lower / larger label back.  Same chain either way (hdpm_stats.sm_chain_*). */
#define HDPM_OPT_SM_CHAIN 9
int hdpm_set_option(hdpm_ctx* ctx, int32_t option, double value);
/* The current value of an option (the same units as hdpm_set_option; HDPM_OPT_PHI_DEVICE
 * reads 1 when update_phi runs on the device, which may be the default). */
int hdpm_get_option(hdpm_ctx* ctx, int32_t option, double* value);
/* Posterior analysis (realdata_analysis/zoo_simulator.R:193-236, 339-344; mcclust /
 * mcclust.ext).  hdpm_psm_build: the posterior similarity matrix of M saved label vectors
 * c_trace[M x N] (results$c_i, labels 0..254) -- comp.psm(C) -- kept on the device as
 * co-clustering counts (psm = count / M).  hdpm_psm_rows: rows row0 .. row0+nrows-1 of psm
 * (N doubles each).  hdpm_psm_vi_lb: VI.lb(cls, psm) of ncand candidate partitions
 * cls[ncand x N] (the lower bound of the posterior expected variation of information that
 * minVI minimises). */
int hdpm_psm_build(hdpm_ctx* ctx, const int32_t* c_trace, int32_t M, int32_t N);
int hdpm_psm_rows(hdpm_ctx* ctx, int32_t row0, int32_t nrows, double* out);
int hdpm_psm_vi_lb(hdpm_ctx* ctx, const int32_t* cls, int32_t ncand, double* out);
/* Testing: one draw on the device from log-weights logw[E] (E <= 256) and the uniform rU --
 * the n8:95-102 categorical draw (two_way = 0; *pick = the 0-based index, or -status) or the
 * sm:204-215 two-way draw (two_way = 1, E = 2) -- with the engine's exp, glibc's algorithm
 * (ocml = 0), or the device libm's (ocml = 1: what the engine used before; shows the ulp
 * differences the glibc replica removes). */
int hdpm_debug_draw(hdpm_ctx* ctx, const double* logw, int32_t E, double rU, int32_t two_way, int32_t ocml,
                    int32_t* pick);
/* Testing: exp (fn = 0) or log (fn = 1) of x[n] on the device, glibc's algorithm (ocml = 0)
 * or the device libm's (ocml = 1). */
int hdpm_debug_math(hdpm_ctx* ctx, const double* x, int64_t n, int32_t fn, int32_t ocml, double* out);
/* Block until every kernel and copy the context has queued is done, a prepared next
 * sweep's prefix (scratch outputs only) included; the prepared sweep stays prepared. */
int hdpm_synchronize(hdpm_ctx* ctx);
/* Drop a prepared next sweep (the one the last hdpm_iterations / hdpm_iteration call set up:
 * its prepass possibly queued on the device, its speculative update_phi on the host pool):
 * the job is joined and the stream rewound, so the next iteration does all of its own work
 * (bench.py calls it between the warmup and the timed window).  Any other state-changing
 * call does the same implicitly. */
int hdpm_drop_prepared(hdpm_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* HDPM_H */
