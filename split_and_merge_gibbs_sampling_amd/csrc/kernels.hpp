// kernels.hpp -- argument blocks shared by the host runtime and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include <cstdio>
#include <cstdlib>

namespace hdpm {

// Diagnosis (HDPM_SYNC_EACH=1): every kernel launch of the engine is followed by a stream
// synchronisation and its name and status on stderr, so a device fault is pinned on the
// kernel that raised it (the next launch would otherwise report it).
inline bool sync_each() {
  static const bool on = [] {
    const char* e = std::getenv("HDPM_SYNC_EACH");
    return e && std::atoi(e) == 1;
  }();
  return on;
}
inline void sync_report(const char* name, hipStream_t s) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  std::fprintf(stderr, "[sync] %s: %s\n", name, hipGetErrorString(e));
}
#define HDPM_LAUNCH(kern, grid, block, lds, strm, ...)                       \
  do {                                                                      \
    hipLaunchKernelGGL(kern, grid, block, lds, strm, __VA_ARGS__);          \
    if (::hdpm::sync_each()) ::hdpm::sync_report(#kern, strm);              \
  } while (0)

constexpr int kBlock = 256;        // prepass points per workgroup (4 waves)
constexpr int kWave = 64;

// Byte-packed categorical rows, tiled for coalesced 16-B-per-lane loads:
//   byte (i, j) lives at ((i/64 * nq + j/16) * 64 + i%64) * 16 + j%16
// so one wave reading chunk q of its 64 points touches 1 KiB contiguous.
__host__ __device__ inline int64_t tiled_offset(int64_t i, int j, int nq) {
  return (((i >> 6) * nq + (j >> 4)) * 64 + (i & 63)) * 16 + (j & 15);
}

// Per-entry parameter tables: codes[e][dp] (dp = 16*nq, zero padded) and
// tab[e][d][2] = {dhamming on match, dhamming on mismatch} (host glibc values).
struct ParamTables {
  const uint8_t* codes;
  const double* tab;
};

// Bit-sliced codes.  A row's categorical codes (code - 1, `wb` bits) are stored as wb
// bit-planes of Ws 64-bit words each (bit j % 64 of word j / 64 of plane b = bit b of
// attribute j's code; Ws = words per plane, padded to 2 or 4 when d <= 256 so kernels can
// keep a row in registers).  The mismatch mask of a point x and a center c is then
// M = OR_b (x_b ^ c_b), one bit per attribute.
__host__ __device__ inline int plane_words(int d) {
  const int wd = (d + 63) / 64;
  return wd <= 2 ? 2 : wd <= 4 ? 4 : wd;
}

// Bound data per parameter entry (cluster slot or pool entry), `bw` u64 words:
//   [0, wb*Ws)              the center's bit-sliced codes
//   [wb*Ws, (wb+kQ)*Ws)     kQ penalty bit-planes: bit b of q_j = floor(|d_j| / delta),
//                           d_j = dhamming(match) - dhamming(mismatch)
//   then, as doubles: A = sum_j dhamming(match), delta, dmin = min_j |d_j|,
//                     scale = sum_j max(|match_j|, |mismatch_j|).
// For a point with mismatch mask M:  H = popc(M), Sq = sum_b 2^b popc(M & plane_b), and
//   A - delta (Sq + H) <= ll <= A - delta Sq     (planes: precise)
//   ll <= A - dmin H                              (codes only: crude)
// up to rounding, covered by kBoundEps * (1 + scale) (a sum of d terms has error below
// d 2^-53 scale).  bw is even, so records are 16-B aligned for vector loads.
constexpr int kQ = 4;
constexpr double kBoundEps = 1e-9;

__host__ __device__ inline int bound_words(int wb, int Ws) { return (wb + kQ) * Ws + 4; }

// Pool-entry heads: what the prepass gathers for a latent pick, wb*Ws + 2 words padded to
// a power of two (64 B at C5 instead of the 128-B bound record; a random gather costs
// one memory request per aligned head, measured: 64-B heads 76 us, 48-B packed heads 85 us,
// 128-B records 85 us per C5 prepass) --
//   [0, wb*Ws)   the center's bit-sliced codes (as in the bound record)
//   then four floats: A_up = A + kBoundEps (1 + scale) rounded up, and rounded down dmin,
//   S_a = S(h_a), S_b = S(h_b), where S(h) is the sum of the h smallest d_j.
// A mismatch set of H attributes costs at least S(H) >= S(h) + (H - h) dmin for H >= h
// (the H smallest d_j include the h smallest, and every further one is >= dmin), so
//   ll <= A_up - max(dmin H, S_a + (H - h_a) dmin [H >= h_a], S_b + (H - h_b) dmin [H >= h_b]).
// A latent center is uniform over the levels, so H has mean mu = sum_j (1 - 1/m_j) and
// variance s2 = sum_j (1 - 1/m_j) / m_j whatever the point; h_a = mu - 4 s, h_b = mu - 1.25 s
// (tools/latent_bound_study.py: at C5 the bound leaves 6e-5 of the picks uncertain; those
// lanes gather the full record).  Used for the templated prepass layouts (Ws == 2, or
// Ws == 4 with wb <= 4: the head padded to a power of two words) and the wide prepass
// (k_prepass_wide: padded to a multiple of 8 words, 64 B; 448 B at C4 instead of the
// 864-B record).
constexpr __host__ __device__ inline int head_words(int wb, int Ws) { return wb * Ws + 2; }
constexpr __host__ __device__ inline bool templ_fits(int wb, int Ws) { return Ws == 2 || (Ws == 4 && wb <= 4); }
// Wide layouts: one 16-lane group per point (a lane per plane word, Ws <= 32 so at most two
// words per lane), the workgroup's 64-point row tile staged in LDS ((wb Ws + 1) words per
// point) and the next tile prefetched in registers (wb Ws <= 64: 4 words per thread).
constexpr int kWideRowMax = 64;
constexpr __host__ __device__ inline bool wide_fits(int wb, int Ws) {
  return !templ_fits(wb, Ws) && Ws <= 32 && wb * Ws <= kWideRowMax;
}
constexpr __host__ __device__ inline int head_stride(int wb, int Ws) {
  if (!templ_fits(wb, Ws)) return (head_words(wb, Ws) + 7) / 8 * 8;
  int s = 4;
  while (s < head_words(wb, Ws)) s *= 2;
  return s;
}
__host__ __device__ inline bool head_fits(int wb, int Ws) { return templ_fits(wb, Ws) || wide_fits(wb, Ws); }

// Rows, tiled: word q of point i at ((i/64) * W + q) * 64 + i%64 (W words per row).
__host__ __device__ inline int64_t packed_offset(int64_t i, int q, int W) {
  return ((i >> 6) * W + q) * 64 + (i & 63);
}

struct PrepassArgs {
  const uint8_t* codes_t;
  int n, d, nq;
  const int* c;              // slot of each point
  const int* counts;         // points per slot (current)
  const int* slot_of_label;  // K entries
  int K;
  int S;                     // slots (columns) at this snapshot
  ParamTables slots;
  ParamTables pool;
  const uint64_t* xbs;       // bit-sliced rows (tiled), wb * Ws words per row
  int Ws, wb;                // words per bit-plane, bits per attribute
  const uint64_t* slot_bnd;  // [slot][bw]
  const uint64_t* pool_bnd;  // [entry][bw]
  const uint64_t* pool_head; // [entry][head_words] (head_fits), or nullptr: full records only
  int head_ha, head_hb;      // the heads' h_a, h_b
  int bw;
  uint64_t* csum;           // per label: its slot's record, logn[count], slot id (bw + 2 words)
  int64_t P;
  const uint32_t* raw;       // R MT raw outputs, (m+1) per point
  int m;
  const double* logn;        // logn[k] = log(k) (glibc), k = 0..n+1
  double logfac;             // log(gamma / m)
  double thresh;             // certainty threshold incl. 2 * drift budget
  double dmax2;              // 2 * drift budget (stay_by_uniform), +inf: margins only
  double* L;                 // exact rows of the uncertain points: L[rowpos * (S + m) + e]
  int* rowpos;               // per point: its row in L, or -1 (certain at the snapshot)
  double* margin;            // per point: lower bound on the own-cluster margin, or -inf
  int* list;                 // per block: ordered uncertain points
  int* cnt;                  // per block: number of uncertain points
  int* dense;                // all uncertain rows in index order (k_list_scan)
  int* dense_total;          // their number
  int* spec;                 // per dense-list position: the draw in the snapshot state (or -1)
  double* spec_rad;          // per dense-list position: log-weight drift under which it holds
  int4* rq;                  // per dense-list position: {row, point, slot, categorical draw}
  int p0;
  int exact_wave;            // 1: exact rows one wave per point (no workgroup staging)
  int wide;                  // 1: wide layouts take k_prepass_wide (0: the generic kernel)
  int* zero;                 // k_cluster_summary clears this word first (the sweep's move count), or nullptr
  int* wide_ctr;             // [2] k_prepass_wide's chunk counter, k_exact_rows_mass's point counter
                             // (cleared by k_cluster_summary)
  int exact_grid;            // the exact-rows grid (0: from the launch size); workgroups loop over the list
  int* boff;                 // [list blocks] offsets of the blocks' rows in the dense list (exact_scan)
  int exact_scan;            // 1: the dense list by k_list_scan before the exact rows (many listed
                             // points: every workgroup then reads its rows, no per-point block walk)
  int nlb, lblock;           // list blocks of this launch and their points (k_exact_rows_wg's own list scan)
  int mmax;                  // levels of the widest attribute (k_exact_rows_lv's level-indexed tables)
  int spec_lv;               // 1: snapshot draws may come from k_snap_draws behind k_exact_rows_lv
  int dense_direct;          // 1: every point listed by k_dense_list (no prepass, no list scan)
  int exact_pref;            // testing (HDPM_OPT_EXACT_KERNEL): 0 auto, 1 k_exact_rows_mass, 2 _lanes, 3 _lv
  double thresh_ref;         // the prepass's margin threshold (k_snap_draws counts the points it would list)
  double dmax2_ref;          // ... and its drift allowance of the uniform test (+inf: margins only)
  // latent bounds (k_exact_rows_lv with lbound): a latent entry whose head bound puts it at
  // least kLatMargin below the point's best cluster gets that bound in its L column instead of
  // the exact sum, and bit u of lmask[row] set (readers: kernels.hip latent_value_fix)
  int lbound;
  unsigned int* lmask;       // [row] bounded latent columns (nullptr: none)
  double lat_negl;           // a bounded latent counts as -inf this far below the best cluster (kLatNegligible)
  // pipelined iterations (engine.cpp iterations_pipelined): the kernels run only while *gate
  // is set, and read the sweep's draws from *raw_ptr (a position found on the device)
  const int* gate;
  const uint32_t* const* raw_ptr;
  // k_prepass_wide's persistent grid: workgroups per CU (0: as many as fit).  Fewer leave room
  // on every CU for the device update_phi beside the sweep (engine.cpp wide_per_cu).
  int wide_per_cu = 0;
};

// A latent entry kept as a head bound counts as probability 0 this far below the best
// cluster (kernels.hip latent_fix; the default of PrepassArgs / ResolveArgs::lat_negl)
constexpr double kLatNegligible = 40.0;

// A sweep's kernels in a pipeline read `raw` from the device (pipe_gate); false: skip.
// The gate word is read with a vector load, so the compiler takes its value as divergent and
// guards the rest by the exec mask alone -- without a branch around a block this short -- and
// the scalar load of *raw_ptr then ran with every lane off: a closed gate with raw_ptr null
// (the gated-off warm launches) faulted on address 0.  The gate is made
// wave-uniform (readfirstlane), so a closed gate branches around the load.
__device__ __forceinline__ bool gate_closed(const int* gate) {
  return gate && __builtin_amdgcn_readfirstlane(*(volatile const int*)gate) == 0;
}
template <class A>
__device__ __forceinline__ bool pipe_gate(A& a) {
  if (!a.gate) return true;
  const int g = __builtin_amdgcn_readfirstlane(*(volatile const int*)a.gate);
  if (g == 0) return false;
  a.raw = *a.raw_ptr;
  return true;
}

// A sweep enqueued before the host knows whether it may run (k_pipe_wait): the host writes
// its slot (host-coherent memory) once the previous iteration is decided -- flag 1 go (with
// the sweep's draws), 2 abort -- and the wait kernel turns it into the gate the sweep's
// kernels read (pipe_gate): go, and the previous sweep completed in its one launch without
// a move.  status: the flag seen (3: none within the time limit; 4: the device's own go).
//
// Device-side go (PipeAuto, the device update_phi's chained pipeline): the host authorises it
// when it enqueues the sweep (the iteration after this one runs a Neal-8 sweep with the
// speculated update); the wait kernel -- behind the speculated update's completion in stream
// order -- then gives the go itself when the previous sweep completed in one launch without a
// move and the update completed (its chain word), its draws in the window `win_*` after the
// update's end, and tells the host (dev 1, raw_dev); otherwise it writes dev 2 and waits for
// the host's flag as before.  The host follows a device go (pipe_go) and never releases it.
constexpr int kPipeOff = 10;   // ResolveCtl::status of an enqueued sweep that was gated off
struct PipeSlot {
  int flag;
  int dev;                     // written by k_pipe_wait with PipeAuto: 1 went, 2 waits for flag
  const uint32_t* raw;
  const uint32_t* raw_dev;     // the sweep's draws, when dev == 1
};
struct PhiChain;
struct PipeAuto {
  const PhiChain* chain;       // the update whose tables the sweep scatters
  const uint32_t* win_raw;
  int64_t win_start, win_count;
  int64_t sweep_len;           // N (m + 1)
  int on;
};
struct PipeGate {
  int gate;
  int status;
  const uint32_t* raw;
};

// The resolver of a pipelined sweep (ResolveArgs::dry) stops with this status before its
// first decision that would change the state; nothing has changed then.
constexpr int kDryStop = 9;

// The resolver runs in block mode (csrc/kernels.hip, k_resolve_blk) when in the previous
// launch at least this many uncertain points needed a decision of their own (their
// snapshot draws no longer held).
constexpr int kResolveBlkMin = 256;

// Control block written by the resolver.
struct ResolveCtl {
  int next;       // first point not yet decided (n when the sweep is complete)
  int status;     // 0 ok, else hdpm::Status
  int restart;    // 1 if stopped to recompute columns after a new slot
  int K;
  int nslots;
  int moves;
  int exact;      // decisions computed in the resolver (not taken from the snapshot draws)
  int checked;    // 1 if the drift budget was exceeded (checked mode)
  int listed;     // points the prepass left uncertain (exact rows built) in this launch
  int aborted;    // 1: k_resolve_fpg gave up at a grid barrier (a workgroup not resident in time);
                  // the state is consistent at `next` (restart there, with k_resolve_fp)
  int uncertain;  // dense launches: listed points the prepass's margin test would have listed
                  // (k_snap_draws' count), or -1
};

struct ResolveArgs {
  int n, d, dp, m;
  int64_t P;
  int* c;
  int* counts;
  int* slot_of_label;
  int* label_of_slot;
  int* slot_src;             // pool entry a dynamic slot was created from (-1: original)
  uint8_t* slot_codes;
  double* slot_tab;
  ParamTables pool;
  const uint32_t* raw;
  const double* logn;
  double logfac;
  const double* L;           // rows of uncertain points, S + m entries each
  const int* rowpos;
  uint64_t* slot_bnd;
  const uint64_t* pool_bnd;
  int bw;
  int S;                     // slots at the snapshot (L columns 0..S-1; latents at S + l)
  const double* margin;
  const int* list;
  const int* dense;          // uncertain rows in index order
  const int* dense_total;
  const int* spec;           // per dense-list position: the snapshot draw (k_exact_rows), or -1
  const double* spec_rad;    // its radius (decide_values)
  const int4* rq;            // per dense-list position: {row, point, slot, categorical draw}
  int nblocks;
  int p0;
  double T;                  // certainty threshold without drift
  double dmax;               // drift budget used by the prepass
  int scap;                  // slot capacity (device arrays, summary stride)
  int lcap;                  // slot capacity of the resolver's LDS state (>= nslots + 2)
  int K;
  int nslots;
  ResolveCtl* ctl;
  int* summary;              // at exit: [label -> slot: scap][count per slot: scap][pool source per slot: scap]
  int force_exact;           // testing: evaluate every point on the exact path
  // move log for the incremental sufficient statistics (nullptr: not kept):
  // mlog[3q .. 3q+2] = (point, from slot, to slot); *mcount entries so far this sweep
  int* mlog;
  int* mcount;
  unsigned int* freq;        // per-slot freq [slot][d][mmax] (new slots are zeroed here)
  int fstride;               // d * mmax
  long long* prof;           // diagnostics: resolver phase times (s_memrealtime ticks) or nullptr
  int blocks;                // 1: block mode (k_resolve_blk; needs K + m <= 64, nslots <= 64)
  const int* gate;           // as PrepassArgs
  const uint32_t* const* raw_ptr;
  int dry;                   // 1: stop (kDryStop) at the first decision that is not "stay"
  int fp;                    // 1: fixed-point resolver (k_resolve_fp; needs K + m <= 64, lcap <= 64)
  int debug_fp;              // bit 0: its first round starts from "stay" (not the snapshot draws' outcomes)
  // device-wide fixed-point resolver (k_resolve_fpg, fpg > 1 workgroups, one resident per CU):
  // fpg_buf = fpg_words(fpg) ints of cross-workgroup scratch, its kFpgBarWords barrier words zeroed by the host
  int fpg;
  int* fpg_buf;
  const int* uncertain;      // dense launches: k_snap_draws' count of would-be-listed points (or nullptr)
  const unsigned int* lmask; // [row] latent columns of L holding head bounds, not exact sums (or nullptr)
  const uint8_t* codes_t;    // the data (tiled codes): exact latent sums for bounded columns
  int nq;
  double lat_negl;           // as PrepassArgs::lat_negl
  int all_listed;            // 1: every point of [p0, n) listed (k_dense_list): nothing to re-test
  long long fpg_limit;       // a grid barrier gives up after this many wall_clock64 ticks (100 MHz)
  int fpg_fail;              // testing: workgroup 0 gives up at its fpg_fail-th grid barrier (0: never)
};
// Cross-workgroup scratch of k_resolve_fpg (G workgroups), in ints: barrier [0, 96), state mirror
// [96, 96 + 8 + 3 * 64 + 16), then per workgroup: stop and changed (two parities each), fail,
// moves, fresh; per workgroup and slot: round deltas (two parities), committed deltas; then per
// workgroup (doubles): drift.
constexpr int kFpgSlots = 64;
constexpr int kFpgState = 8;
constexpr int kFpgPerWg = 8;
constexpr int kFpgBarWords = 96;   // barrier words (the 64-bit barrier word at 0, then padding)
constexpr int kFpgZeroWords = kFpgBarWords + kFpgState + 16;   // zeroed before every launch (barrier, state mirror)
__host__ __device__ inline size_t fpg_words(int G) {
  return (size_t)kFpgBarWords + kFpgState + 3 * kFpgSlots + 16 + (size_t)G * kFpgPerWg + (size_t)3 * G * kFpgSlots +
         (size_t)2 * G + 16;
}

// Cluster parameter upload: one staging buffer, scattered on the device.
//   [codes: nent * dp bytes][tab: nent * 2d doubles][bnd: nent * bw words][counts: nent ints][slot: nent ints]
// (offsets rounded up to 16 B).  full == 1: entries are labels 0..nent-1, and the slot maps are
// reset to the identity with the given counts; full == 0: entry r goes to slot[r] only.
struct UploadLayout {
  size_t off_codes, off_tab, off_bnd, off_counts, off_slot, bytes;
};
__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline UploadLayout upload_layout(int nent, int dp, int d, int bw) {
  UploadLayout L;
  L.off_codes = 0;
  L.off_tab = align16((size_t)nent * dp);
  L.off_bnd = align16(L.off_tab + (size_t)nent * 2 * d * 8);
  L.off_counts = align16(L.off_bnd + (size_t)nent * bw * 8);
  L.off_slot = align16(L.off_counts + (size_t)nent * 4);
  L.bytes = align16(L.off_slot + (size_t)nent * 4);
  return L;
}

struct HistArgs {
  const uint8_t* codes_t;
  int n, d, nq;
  const int* label;          // label per point
  const unsigned char* mask; // per label: include (nullptr = all)
  int K, mmax;
  unsigned int* freq;        // [K][d][mmax]
  // packed path (k_hist_packed): rows in `wb`-bit fields, labels sliced KC per grid row
  const uint64_t* xpk;
  int W, wb;
  int KC;                    // labels per slice (LDS counters KC * mmax * d)
  int tiles_per_block;
  unsigned int* partial;     // [slice][block][KC * mmax * d]
};

struct LoglikArgs {
  const uint8_t* codes_t;
  int n, d, nq;
  const int* label;
  ParamTables cl;            // per label tables
  double* partial;           // per block (hi, lo) pairs
};

}  // namespace hdpm

namespace hdpm {

// Restricted Gibbs scan over S (code/split_merge.cpp:163-225) and logprobgs_c_i (96-161).
// The device chain of a restricted Gibbs sampler (split_merge.inl sm_chain): scan k's gate,
// draws and cluster sizes, written by k_sm_link from the update before it (kernels with a
// link read them there instead of their arguments and do nothing when ok == 0).
struct SmLink {
  const uint32_t* raw;       // the scan's nS draws (inside the stream window)
  int ok;                    // 1: the scan runs (the update before it completed, its draws in the window)
  int n1, n2;                // sizes of c_i_1, c_i_2 before the scan
};

// Frequency table of a point list (k_sm_freq): out[j * mmax + x_ij - 1] += 1 over the points
// list[q] with side[q] == want (side == nullptr: every point), and the extra points (>= 0).
struct SmFreqArgs {
  const uint8_t* codes_t;
  int n, d, nq, mmax;
  const int* list;
  int nlist;
  const int* side;
  int want;
  int extra[2];
  // side_prev != nullptr: the change of the want-side table since side_prev (points now on
  // `want` count +1, points that left it -1, two's complement in the u32 counters; no extras)
  const int* side_prev;
  uint32_t* out;             // [d][mmax], zeroed by the launcher (unless prezeroed)
  int prezeroed;
  const SmLink* link;        // device chain: nothing counted unless link->ok (nullptr: always)
};

struct SmArgs {
  const uint8_t* codes_t;
  int n, d, nq;
  const int* S;              // point indices, scan order
  int nS;
  ParamTables two;           // tables of the two clusters (entry 0 = c_i_1, entry 1 = c_i_2)
  double* ll;                // [2][nS]
  int* side;                 // in/out: 0 -> c_i_1, 1 -> c_i_2, per S position
  const int* side_ref;       // launch-state side (logprobgs_c_i), per S position
  const uint32_t* raw;       // nS raw draws (scan)
  const double* logn;
  int n1, n2;                // current (scan) or launch (logprobgs) cluster sizes
  int* out_counts;           // [2] final sizes after the scan
  double* out;               // logprobgs partial (hi, lo) per block
  int* cert;                 // scan: per S position, [3][2] certified count bands (k_sm_cert)
  int* side_prev;            // k_sm_cert copies the sides before the scan here (nullptr: no copy)
  int cert_in_ll;            // k_sm_ll_lds computes the certified bands too (no k_sm_cert launch)
  int* wide_buf;             // k_sm_scan_wide: [0] arrivals, [1] gave up, [2] rounds, [3] pad, [4, 4 + 2G) deltas
  long long wide_limit;      // its barrier waits give up after this many wall_clock64 ticks
  uint32_t* zero;            // zeroed by k_sm_ll_lds (zero_n words): the table k_sm_freq fills next
  int zero_n;
  const SmLink* link;        // device chain: raw, n1, n2 from the link; nothing runs unless link->ok
};

}  // namespace hdpm

namespace hdpm {

// update_phi (code/common_functions.cpp:511-591) on the device (csrc/phi.hip).  T clusters
// (ascending labels) each draw d centers, then d sigmas (rhig, hyperg.cpp:346-378), from one
// slice of the R stream.  The sigma draws consume 2 uniforms per rbeta attempt, so where a
// draw starts depends on every earlier rejection: item k (cluster t = k / d, attribute
// j = k % d) starts at its nominal position t*3d + d + 2j plus a drift delta >= 0.
// k_phi_masks evaluates every candidate's acceptance at every drift of a window around the
// expected drift (bit masks, all items in parallel); k_phi_walk resolves the drifts in
// stream order over the masks (one wave, fixed-point rounds of 64 items); k_phi_values
// computes sigmas, dhamming tables, bound records and the regrouped log-likelihood terms.
// Anything the device does not restate (Walker tables, the bisection path of rhig, an
// ambiguous pbeta branch test, a drift outside its window, a short stream slice) sets a
// status and nothing is committed: the host runs the update itself.
struct PhiCand {             // rbeta setup of one (cluster, attribute, center level)
  int kind;                  // 2 = BC, 3 = BB (RBeta::Kind); 0: inactive; 1: bisection path
  int pad;
  double aa, a, b, alpha, beta, gamma, k1, k2, thr, m;   // as PoolClass
};

struct PhiArgs {
  int T, d, dp, mmax, sumatt, wb, Ws, bw;
  const int* lab;            // [T] label of cluster t (ascending)
  const int* cnt;            // [T] its size
  const unsigned* freq;      // [label][d][mmax]
  const double* sig_in;      // [T][d] current sigma (cf:498 uses it in the center probabilities)
  const int32_t* att;        // [d] m_j
  const int* aoff;           // [d + 1] prefix sums of m_j
  const double* v;           // [d]
  const double* w;           // [d]
  const uint64_t* gtab;      // glibc exp table then log table (512 words)
  const uint32_t* raw;       // the stream slice from the update's first draw
  int64_t nraw;              // its length
  // scratch
  double* cum;               // [T][sumatt] cumulative probabilities in revsort order
  uint8_t* perm;             // [T][sumatt] level (0-based) of each sorted position
  uint8_t* det;              // [T][d] deterministic pick + 1, or 0 (depends on the uniform)
  PhiCand* cand;             // [T][sumatt] per center level
  int* act;                  // active candidates: [0] count, then (t * sumatt + aoff[j] + l) entries
  int64_t nact_cap;
  uint64_t* mask;            // [T * sumatt][nw] acceptance bits per drift (candidates of uniform-dependent picks)
  uint64_t* maskd;           // [T * d][nw] the same for items whose pick does not depend on the uniform
  uint8_t* ikind;            // [T][d] such an item's candidate kind (0: the pick depends on the uniform)
  int wpb;                   // waves per workgroup of k_phi_cwalk / k_phi_values
  int groups;                // k_phi_cwalk workgroups per cluster
  // pipelined iterations: raw from *raw_ptr (k_phi_locate), skipped unless *gate; the
  // chain writes the next sweep's start position *pos_out = *pos_in + sweep_len + draws
  const uint32_t* const* raw_ptr;
  const int* gate;
  const int64_t* pos_in;
  int64_t* pos_out;
  int64_t sweep_len;
  int nw;                    // words per candidate
  double rate, sdev;         // expected drift per item and its sd per sqrt(item): window model
  uint8_t* pick;             // [T][d] drawn center level (0-based)
  int64_t* apos;             // [T][d] position of the accepted attempt (relative to raw)
  int* status;               // [0] status (0 ok), [1] first failing item, [2..3] consumption (int64)
  // outputs
  uint8_t* stage;            // UploadLayout(T, dp, d, bw) staging (entry t -> slot `slot_of[t]`)
  const int* slot_of;        // [T] slot of each entry, or nullptr (slot = label)
  double* sig_out;           // [T][d] new sigmas
  double* ll;                // [T][2] regrouped log-likelihood (hi, lo) of each cluster
  // speculative cluster walks (k_phi_cwalk): cluster t's start drift is one of
  // phi_clo(t) + c, c < Wc; F[t][c] = its end drift (-1: the walk left its windows)
  double* lg;                // [span] log(u / (1 - u)) of each stream position
  double* lzz;               // [span] log(u_p * u_p * u_(p+1))
  int64_t span;
  int* F;                    // [T * S][Wc]
  int Wc;
  int L, S;                  // walk segments: items [s L, (s + 1) L) of a cluster, S per cluster
  int64_t* dts;              // [T] the start drift of each cluster (k_phi_chain)
  // composition trees (k_phi_tree, k_phi_tree_top, k_phi_values2; used when tree != nullptr):
  // every item whose pick does not depend on the uniform is a function of the drift, f(delta) =
  // delta + 2 (attempts rejected from delta on); a node of the tree is the composition of the
  // functions of its items, tabulated over the tW start drifts phi_lo(first item) + c as the
  // extra uniforms it consumes (uint16, kPhiBad: outside the windows).  Level 0 nodes are
  // blocks of 4 items, a level-l node the composition of its two level-(l - 1) children;
  // cluster t's tables start at tree + t * tpc * tW (level l at phi_loff(tnb, l)).
  uint16_t* tree;
  int tW;                    // start drifts per table (64 (nw - 1): a lookup reads two mask words)
  int tnb;                   // level-0 blocks per cluster, ceil(d / 4)
  int tSB, tS;               // blocks per k_phi_tree workgroup (power of two), workgroups per cluster
  int tpc;                   // tables per cluster
  int tRootLds;              // (unused: the roots are always staged in LDS)
  int* tnd;                  // [T] cluster t has a pick that depends on the uniform: walked per start
                             // drift (k_phi_cwalk) into its root table, then from its drift (one wave)
  // fast path (launch_phi2: k_phi2_group -> k_phi2_tree -> k_phi2_values), every pick fixed:
  // groups of gs consecutive items of a cluster (G per cluster), each tabulated over tW start
  // drifts by the workgroup that computes its masks; inputs and outputs may live in coherent
  // host memory (no copies); status words tagged with the call's generation (no memset)
  int gs, G;
  uint16_t* gtab2;           // [T * G][tW] group tables
  uint16_t* roots;           // [T][tW] cluster tables
  int* ctr;                  // [2] last-workgroup counters ([1]: k_phi2_values; self-resetting)
  int gen;                   // status generation: status[0] = gen << 4 | code belongs to this call
  int* status_host;          // [4] status (code, -, consumption int64) written by the last k_phi2_values workgroup
  unsigned long long* tdbg;  // testing (HDPM_PHI_TIMING): wall-clock marks of the fast path's phases, or nullptr
  int* lab_dev;              // [2T] device copy of lab then cnt, written by k_phi2_group for k_phi2_values
  // the stream state after the update (fast path): the 624 words of the block that holds the
  // position after its draws, then that position's index in the block (0: not copied -- the
  // block is not inside [raw - raw_back, raw + nraw)); written before status_host, or nullptr
  uint32_t* state_host;
  int mti_pos;               // the index in its block (1..624) of the update's first position
  int64_t raw_back;          // words of the stream window before `raw`
  // chained updates (fast path): an update enqueued behind the previous one before that one
  // ran.  With chain_in set, its first draw is at chain_in->end + sweep_len (the previous
  // update's end, then the sweep between them) inside the window (win_raw, win_start, win_count,
  // win_mti0: raw, nraw, raw_back and mti_pos are derived on the device), its labels, counts and
  // sigmas are the previous update's (lab / cnt / sig_in point at its lab_dev and sig_dev), and
  // it runs only if the previous update completed (else status kPhiOff, nothing computed).
  const struct PhiChain* chain_in;
  struct PhiChain* chain_out;  // this update's end position and completion, or nullptr
  int64_t pos0;              // absolute stream position of the first draw (chain_in: set on the device)
  const uint32_t* win_raw;
  int64_t win_start, win_count;
  int win_mti0;
  double* sig_dev;           // [T][d] device copy of sig_out (a chained successor's sig_in), or nullptr
};
// Written by the last k_phi2_values workgroup of an update with chain_out.
struct PhiChain {
  int64_t end;               // absolute stream position after the update's draws
  int ok;                    // 1: completed (status 0), 0: not
  int pad;
};
// Device chain of a restricted Gibbs sampler (split_merge.inl sm_chain), per scan k:
// k_sm_link: scan k's link from the update before it (`prev`: its end position and completion,
// or the chain's seed word), the link's own chain word for the update after the scan (same
// end, ok = the link's: that update's first draw follows the scan's nS), and the two
// clusters' tables from the previous scan's updates' staging in side order (entry 0 = c_i_1).
// (update_phi({c1, c2}) runs as two one-cluster updates in ascending label order, the second
// chained behind the first: each starts at drift 0, so its center picks are fixed by its
// first d uniforms and the fast path never hands back for a pick that depends on them)
struct SmLinkArgs {
  const PhiChain* prev;
  const int* counts_in;      // sizes after the previous scan, or nullptr: n1, n2
  int n1, n2, nS;
  const uint32_t* win_raw;   // the stream window holding the chain's draws
  int64_t win_start, win_count;
  SmLink* link;
  PhiChain* chain;
  const uint8_t* stage[2];   // the previous scan's updates' UploadLayout(1, dp, d, bw) staging by
                             // ascending label, or nullptr (the tables stay)
  int dp, d, bw, swap;       // swap: c_i_1 has the larger label
  uint8_t* two_codes;        // [2][dp]
  double* two_tab;           // [2][2 d]
};
// k_sm_tabs: after scan k's k_sm_freq (delta: the change of c_i_1's table), both tables in
// ascending label order (F[a1] = c_i_1's += delta, F[1 - a1] = fm - F[a1]) and the update's
// labels and sizes (lab_cnt = {0, 1, size of F[0], size of F[1]}: the first update reads label
// lab_cnt[0] and size lab_cnt[2], the second lab_cnt[1] and lab_cnt[3]).
struct SmTabsArgs {
  const SmLink* link;
  const uint32_t* delta;
  const uint32_t* fm;        // [d][mmax] the table of S + {i1, i2}
  uint32_t* F;               // [2][d][mmax]
  int a1, nt;                // index of c_i_1's table, d * mmax
  const int* counts;         // [2] sizes after the scan (c_i_1, c_i_2)
  int* lab_cnt;              // [4]
};

// Level sizes of a composition tree over nb >= 1 level-0 blocks.
__host__ __device__ inline int phi_lcount(int nb, int l) { return ((nb - 1) >> l) + 1; }
__host__ __device__ inline int phi_loff(int nb, int l) {
  int o = 0;
  for (int i = 0; i < l; ++i) o += phi_lcount(nb, i);
  return o;
}
__host__ __device__ inline int phi_ltop(int nb) {
  int l = 0;
  while (phi_lcount(nb, l) > 1) ++l;
  return l;
}
constexpr uint16_t kPhiBad = 0xFFFF;

// Drift windows of the device update_phi (phi.hip).  Extra uniforms per sigma draw: mean
// rate, sd sdev; after k draws the drift is rate k +- kPhiSd sdev sqrt(k).
constexpr double kPhiSd = 7.0;
__host__ __device__ inline int64_t phi_lo(int64_t k, double rate, double sdev) {
  const double c = rate * (double)k - kPhiSd * sdev * sqrt((double)k) - 16.0;
  return c <= 0.0 ? 0 : (int64_t)c;
}
__host__ __device__ inline int64_t phi_hi(int64_t k, double rate, double sdev) {
  return (int64_t)(rate * (double)k + kPhiSd * sdev * sqrt((double)k)) + 80;
}

// Windows of the device stream a pipelined iteration may read (engine.cpp RngWindow).
struct PipeWin {
  const uint32_t* raw;
  int64_t start, count;
};

// k_phi_locate: the update's slice after the sweep from *pos_in; k_pipe_check: the commit
// decision of an iteration and the next sweep's slice.
struct PipeArgs {
  int* gate;                 // the pipeline runs while set
  int* commit_ok;            // this iteration's tables go to the slots (k_scatter_clusters gate)
  const ResolveCtl* ctl;     // the sweep's resolver control block
  int* phi_status;           // the update's status words [4] (status, -, consumption int64)
  const double* ll;          // the update's log-likelihood pairs [T][2]
  int T, n;
  const int64_t* pos_in;     // the sweep's start position
  const int64_t* pos_next;   // the next sweep's start position (the update's chain)
  int64_t sweep_len;         // N (m + 1)
  int64_t need;              // k_phi_locate: stream words the update may read
  PipeWin win[2];
  const uint32_t** raw_out;  // k_phi_locate: the update's slice; k_pipe_check: the next sweep's
  int* act;                  // k_phi_locate clears the candidate count
  int64_t* rec;              // k_pipe_check: [0] 1 committed / 2 not run / 3 stopped, [1] ctl status,
                             // [2] log-likelihood bits, [3] next position, [4] phi status, [5] window stop
};

// kPhiNonDet: a center pick depends on the uniform (the composition trees need fixed picks);
// the update is re-run with the per-start-drift walks (k_phi_cwalk)
enum PhiStatus { kPhiOk = 0, kPhiWalker = 1, kPhiBisect = 2, kPhiAmbig = 3, kPhiWindow = 4, kPhiShort = 5,
                 kPhiProb = 6, kPhiInactive = 7, kPhiCap = 8, kPhiNonDet = 9,
                 kPhiOff = 10 /* chained update whose predecessor did not complete: not run */ };

// R's Mersenne-Twister stream on the device (one workgroup, one twist per barrier).
// Output r >= 0 continues the host state (X_0, mti0): the first 624 - mti0 outputs temper
// X_0[mti0..623]; then block b >= 1 tempers X_b = twist^b(X_0).  Every X_b is exported so
// the host can adopt the state at any later position.
struct MtGenArgs {
  const uint32_t* init;   // X_0 (624 words)
  int mti0;
  int64_t count;
  uint32_t* out;          // count raw outputs
  uint32_t* arrays;       // X_b for b >= export_from (index b - 1); earlier blocks not stored
  int nblocks;
  int export_from;
  // multi-workgroup generation (k_mt_gen_multi): workgroup g starts at block g * bpg from
  // the jump polynomial jpoly[g] (z^(624 * bpg * g - 1) mod phi, 312 words each)
  const uint64_t* jpoly;
  const uint32_t* jidx;   // set-bit positions of jpoly[g]: jidx[joff[g] .. joff[g + 1])
  const int* joff;
  int bpg;
  int G;
};

}  // namespace hdpm
