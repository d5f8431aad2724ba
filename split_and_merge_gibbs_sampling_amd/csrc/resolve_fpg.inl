// resolve_fpg.inl -- the device-wide fixed-point resolver (included by kernels.hip after
// k_resolve_fp, whose helpers it uses).
//
// k_resolve_fp walks the dense list of listed points in chunks of kFpThreads positions on one
// workgroup: a chunk's outcomes are the fixed point of "every point draws in the state its
// predecessors' outcomes leave" (code/neal8.cpp:40-160 in index order), reached by rounds that
// redraw the points behind the first changed outcome.  k_resolve_fpg runs G such chunks at
// once, one workgroup each (a window of G kFpThreads positions, workgroups resident together:
// one per CU), and makes the fixed point the window's: every round each workgroup publishes
// the net count change per slot of its chunk's movers and the position of its first stop;
// after a grid barrier each workgroup forms its chunk's start counts (the committed counts plus
// the changes of the chunks before it, up to the window's first stop), redraws the points
// whose state changed, and publishes whether an outcome changed; the window has converged when
// no outcome changed in a round.  Point k's state depends only on points < k, so the fixed
// point is the sequential walk whatever the guesses; a count change of one point moves the
// others' log-weights by ~1/n, so a round changes few outcomes and windows settle in a few
// rounds.  Then, in lockstep: the drift after each position (prefix maximum across the
// chunks), the unlisted points re-tested (a failure truncates the window there and restarts the
// launch, as in k_resolve_fp), the commit (labels, move log by atomic positions, counts: every
// workgroup applies the window's total change to its own copy of the state), and the window's
// first stop processed by the serial path (RCtx::process) on the workgroup that holds it, which
// publishes the state for the others.  Every barrier gives up after 2 s (every wave exits; the
// launch then reports a resolver failure).
namespace fpg {

// scratch layout (kernels.hpp fpg_words)
struct Lay {
  int* bar;      // [0] arrivals, [32] generation, [64] abort: separate 128-B lines, so the spinning
                 // loads of the generation do not contend with the arrivals' atomics
  int* ms;       // state mirror: K, nslots, status, restart, next, nstruct, exact, moves, go, nlog, checked
  int* sol;
  int* los;
  int* cnt;
  int* stop;     // [2][G] first stop (chunk position) or kFpThreads, by round parity
  int* chg;      // [2][G] an outcome changed in the round before
  int* fail;     // [G] first failing unlisted point or INT_MAX
  int* mov;      // [G] committed moves
  int* fresh;    // [G] committed own draws
  int* dr;       // [2][G][64] round deltas per slot, by round parity
  int* dc;       // [G][64] committed deltas per slot
  double* sd;    // [G] drift maximum over the chunk's movers
  double* md;    // state mirror: dnow, dvmax
};
__device__ __forceinline__ Lay lay(int* b, int G) {
  Lay L;
  L.bar = b;
  L.ms = b + kFpgBarWords;
  L.sol = b + kFpgBarWords + kFpgState + 16;
  L.los = L.sol + kFpgSlots;
  L.cnt = L.los + kFpgSlots;
  int* q = L.cnt + kFpgSlots;
  L.stop = q;                  // [0, 2G)
  L.chg = q + 2 * G;           // [2G, 4G)
  L.fail = q + 4 * G;
  L.mov = q + 5 * G;
  L.fresh = q + 6 * G;
  q += kFpgPerWg * G;
  L.dr = q;
  L.dc = q + 2 * G * kFpgSlots;
  q += 3 * G * kFpgSlots;
  q += ((uintptr_t)q & 7) ? 1 : 0;
  L.sd = reinterpret_cast<double*>(q);
  L.md = L.sd + G;
  return L;
}

// loads of other workgroups' data: agent-scope atomics (coherent at L2, not a stale L1 line)
__device__ __forceinline__ int ald(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double aldd(const double* p) {
  const unsigned long long u =
      __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double((long long)u);
}

// Grid barrier, all or nothing: either every workgroup passes it or none does.  One 64-bit
// word (zeroed by the host before the launch): generation in the high half, a poison bit and
// the arrival count in the low half.  The last arrival advances the generation (count back to
// 0); a workgroup that waited `limit` ticks (or is told to give up: `fail`, testing) poisons the
// word, by compare-and-swap, only while the generation is unchanged and not every workgroup has
// arrived, so no barrier is both passed and poisoned.  A poisoned word stays poisoned: every
// later arrival sees it and gives up too.  False: this barrier (and the launch) gave up -- the
// caller then knows that no workgroup got past it.
constexpr unsigned long long kBarPoison = 1ull << 31;
constexpr unsigned long long kBarCount = kBarPoison - 1;
__device__ __forceinline__ bool sync(const Lay& L, int G, int* flag, long long limit, bool fail) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    int ab = 0;
    unsigned long long* const w = reinterpret_cast<unsigned long long*>(L.bar);
    auto give_up = [&](unsigned gen) -> int {   // 1: poisoned (or found poisoned), 0: the barrier passed
      unsigned long long cur = __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      for (;;) {
        if ((unsigned)(cur >> 32) != gen) return 0;
        if (cur & kBarPoison) return 1;
        if ((cur & kBarCount) >= (unsigned long long)G) return -1;   // completing: wait for the generation
        if (__hip_atomic_compare_exchange_strong(w, &cur, cur | kBarPoison, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          return 1;
      }
    };
    if (fail) {
      // this workgroup never arrives, so the barrier can neither pass nor be completing
      const unsigned long long cur = __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      (void)give_up((unsigned)(cur >> 32));
      ab = 1;
    } else {
      const unsigned long long old = __hip_atomic_fetch_add(w, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned gen = (unsigned)(old >> 32);
      if (old & kBarPoison) {
        ab = 1;
      } else if ((old & kBarCount) + 1 == (unsigned long long)G) {
        __hip_atomic_fetch_add(w, (1ull << 32) - (unsigned long long)G, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const long long t0 = wall_clock64();
        // (relaxed polls, one acquire fence after: an agent-scope acquire load invalidates the
        // XCD's L2 -- per poll, it cost every workgroup of the XCD its cached data)
        for (int spin = 0;; ++spin) {
          const unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(v >> 32) != gen) break;
          if (v & kBarPoison) { ab = 1; break; }
          if ((spin & 31) == 31 && wall_clock64() - t0 > limit) {
            const int r = give_up(gen);
            if (r > 0) { ab = 1; break; }
            if (r == 0) break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
    }
    __threadfence();
    *flag = ab;
  }
  __syncthreads();
  return *flag == 0;
}

// sum over workgroups h < hi of v[h * 64 + s] for s = lane, by all waves (independent loads),
// into out[64] (LDS); red: LDS [kFpWaves][64]
__device__ __forceinline__ void prefix_slots(const int* v, int hi, int* red, int* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // eight loads in flight per lane before they are added (a loop of load-then-add waited for
  // every L2 round trip: ~32 of them per round for the last workgroup of a 256-wide window)
  int acc = 0;
  for (int h0 = wv; h0 < hi; h0 += 8 * kFpWaves) {
    int x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int h = h0 + k * kFpWaves;
      x[k] = h < hi ? ald(v + (size_t)h * kFpgSlots + lane) : 0;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += x[k];
  }
  red[wv * kWave + lane] = acc;
  __syncthreads();
  if (wv == 0) {
    int t = 0;
    for (int w = 0; w < kFpWaves; ++w) t += red[w * kWave + lane];
    out[lane] = t;
  }
  __syncthreads();
}

// one wave: reductions over workgroups h < n of per-workgroup values (64 independent loads at
// a time)
__device__ __forceinline__ double wave_max_over(const double* v, int n, double init) {
  const int lane = threadIdx.x & 63;
  double m = init;
  for (int h0 = 0; h0 < n; h0 += 4 * kWave) {
    double x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = h0 + k * kWave + lane < n ? aldd(v + h0 + k * kWave + lane) : init;
#pragma unroll
    for (int k = 0; k < 4; ++k) m = fmax(m, x[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  return m;
}
__device__ __forceinline__ int wave_min_over(const int* v, int n, int init) {
  const int lane = threadIdx.x & 63;
  int m = init;
  for (int h0 = 0; h0 < n; h0 += 4 * kWave) {
    int x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = h0 + k * kWave + lane < n ? ald(v + h0 + k * kWave + lane) : init;
#pragma unroll
    for (int k = 0; k < 4; ++k) m = min(m, x[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
  return m;
}
__device__ __forceinline__ int wave_sum_over(const int* v, int n) {
  const int lane = threadIdx.x & 63;
  int m = 0;
  for (int h0 = 0; h0 < n; h0 += 4 * kWave) {
    int x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = h0 + k * kWave + lane < n ? ald(v + h0 + k * kWave + lane) : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) m += x[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o);
  return m;
}

}  // namespace fpg

// LDS of k_resolve_fpg beyond k_resolve_fp's: start counts (this and the last round), the
// reduction scratch, the window's flags
struct FpgShared {
  int sc[kWave], sc_prev[kWave], add[kWave];
  int red[kFpWaves * kWave];
  int flag, gs, gs_prev, conv, u, ufirst, nm, nf, flag2, pad2;
  double dch, dwin;
};

__host__ __device__ inline size_t resolve_fpg_lds_bytes(int lcap, int m) {
  return ((resolve_fp_lds_bytes(lcap, m) + 15) & ~(size_t)15) + sizeof(FpgShared);
}

template <int EM>
__global__ __launch_bounds__(kFpThreads) void k_resolve_fpg(ResolveArgs a) {
  if (!pipe_gate(a)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = gridDim.x, g = blockIdx.x;
  const unsigned long long below = (1ull << lane) - 1ull;
  RState st;
  resolve_layout(a, st, smem, false);
  RShared& S = *st.sh;
  FpShared* F = (FpShared*)(smem + ((resolve_lds_bytes(a.lcap, a.m, 0, 0) + 15) & ~(size_t)15));
  FpgShared* X = (FpgShared*)(smem + ((resolve_fp_lds_bytes(a.lcap, a.m) + 15) & ~(size_t)15));
  const fpg::Lay L = fpg::lay(a.fpg_buf, G);
  long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // debug bit 1 profile (workgroup 0): [2] ticks in grid barriers, [3] in the rounds, [4] in
  // the drift / re-test / commit phase; tsub[0] windows
  const bool prof = a.prof != nullptr && g == 0;
  if (prof) tp[0] = wall_clock64();
  int nwin = 0;
  int nbar = 0;      // grid barriers so far (the same sequence on every workgroup)
  auto bar = [&]() -> bool {
    const long long t = prof ? wall_clock64() : 0;
    ++nbar;
    const bool r = fpg::sync(L, G, &X->flag, a.fpg_limit, g == 0 && nbar == a.fpg_fail);
    if (prof) tp[2] += wall_clock64() - t;
    return r;
  };
  if (tid == 0) { F->nlog = a.mcount ? *a.mcount : 0; F->go = 1; F->iters = 0; X->gs_prev = G; }
  for (int e = tid; e < 256; e += kFpThreads) F->etab[e] = devtab::kGlibcExpTab[e];
  resolve_init(a, st);
  const int total = *a.dense_total;
  const int ncol = a.S + a.m;
  const int nsl = S.nslots;
  const int WIN = G * kFpThreads;
  int64_t vfrom = a.p0;
  bool go = true, ok = true;
  int q0 = 0;
  int qs = 0;            // dense-list position of the last window's stop
  bool stopped = false;  // the launch gave up at the barrier behind a stop (of workgroup gs_stop)
  int gs_stop = -1;
  // the state the stopping workgroup published (L.ms, L.sol / los / cnt, L.md), taken over
  auto adopt = [&]() {
    if (wv == 0) {
      const int c = fpg::ald(L.cnt + lane);
      if (lane < st.lcap) {
        st.sol[lane] = fpg::ald(L.sol + lane);
        st.los[lane] = fpg::ald(L.los + lane);
        if (c != st.cnt[lane]) {
          st.cnt[lane] = c;
          st.l1[lane] = fp_logn(a, c);
          st.l0[lane] = fp_logn(a, c - 1);
        }
      }
      if (lane == 0) {
        const int* m = L.ms;
        S.K = fpg::ald(m + 0); S.nslots = fpg::ald(m + 1); S.status = fpg::ald(m + 2);
        S.restart = fpg::ald(m + 3); S.next = fpg::ald(m + 4); S.nstruct = fpg::ald(m + 5);
        S.exact = fpg::ald(m + 6); S.moves = fpg::ald(m + 7); F->go = fpg::ald(m + 8);
        F->nlog = fpg::ald(m + 9); S.checked = fpg::ald(m + 10);
        S.dnow = fpg::aldd(L.md + 0);
        S.dvmax = fpg::aldd(L.md + 1);
      }
    }
    __syncthreads();
  };
  if (prof) tp[1] = wall_clock64();
  while (q0 < total && go && ok) {
    ++nwin;
    const long long tw0 = prof ? wall_clock64() : 0;
    const int cq = q0 + g * kFpThreads;
    const int nc = max(0, min(kFpThreads, total - cq));
    const bool in = tid < nc;
    const int4 r = in ? gld(a.rq + cq + tid) : make_int4(0, 0, 0, 0);
    const int own = r.z;
    const int sp = (in && a.spec) ? gld(a.spec + cq + tid) : -1;
    const double sr = (in && a.spec) ? gld(a.spec_rad + cq + tid) : 0.0;
    // (the categorical uniform: fp_draw_at reads it from the record)
    F->pi[tid] = in ? r.y : INT_MAX;
    const int K = S.K, E = K + a.m;
    const bool struct0 = S.nstruct == 0;
    int cls = 0, tgt = own, pick = -1, co = 0, ct = 0;
    if (in && struct0 && sp >= 0 && !(a.debug_fp & 1)) {
      const bool single0 = st.cnt[own] == 1;
      if (sp < K) {
        const int s2 = st.sol[sp];
        if (!single0) { cls = s2 != own ? 1 : 0; tgt = s2; }
        else cls = 2;
      } else {
        cls = (single0 && sp == K) ? 0 : 2;
      }
    }
    bool fresh = false;
    int chg = -1, fs = nc, gs = G;
    bool conv = false;
    int lastchg = 1, pb = 0;
    if (tid == 0) X->gs_prev = G;
    if (wv == 0) X->sc_prev[lane] = INT_MIN;
    // One grid barrier per round: a round publishes its outcomes' count changes and stops
    // together with whether the evaluation before changed an outcome, into the buffers of its
    // parity (a workgroup still reading the last round's reads the other parity); the window has
    // converged when, after a barrier, no workgroup's last evaluation changed an outcome.
    for (int it = 0; it <= WIN + 2; ++it) {
      pb = it & 1;
      int* const Lstop = L.stop + pb * G;
      int* const Lchg = L.chg + pb * G;
      int* const Ldr = L.dr + (size_t)pb * G * kFpgSlots;
      // (1) this chunk's first stop and its movers' net change per slot, published
      const unsigned long long sbal = __ballot(in && cls == 2);
      if (lane == 0) F->wstop[wv] = sbal ? wv * kWave + __ffsll((long long)sbal) - 1 : kFpThreads;
      F->wd[wv][lane] = 0;
      __syncthreads();
      int fsl = nc;
      for (int w = 0; w < kFpWaves; ++w) fsl = min(fsl, F->wstop[w]);
      const bool mover0 = in && cls == 1 && tid < fsl;
      if (mover0) {
        atomicAdd(&F->wd[wv][own], -1);
        atomicAdd(&F->wd[wv][tgt], 1);
      }
      __syncthreads();
      if (wv == 0) {
        int t = 0;
        for (int w = 0; w < kFpWaves; ++w) t += F->wd[w][lane];
        Ldr[(size_t)g * kFpgSlots + lane] = t;
        if (lane == 0) {
          Lstop[g] = fsl < nc ? fsl : kFpThreads;
          Lchg[g] = lastchg;
        }
      }
      if (!(ok = bar())) break;
      // converged when no outcome of the window changed in the last evaluation
      if (it > 0) {
        if (wv == 0) {
          bool any = false;
          for (int h0 = 0; h0 < G && !any; h0 += kWave) {
            const int h = h0 + lane;
            any = __ballot(h < G && fpg::ald(Lchg + h) != 0) != 0ull;
          }
          if (lane == 0) X->flag2 = any ? 0 : 1;
        }
        __syncthreads();
        if (X->flag2) { conv = true; break; }
      }
      // (2) the window's first stopping chunk; this chunk's start counts
      if (wv == 0) {
        int f = G;
        for (int h0 = 0; h0 < G; h0 += kWave) {
          const int h = h0 + lane;
          const unsigned long long b = __ballot(h < G && fpg::ald(Lstop + h) < kFpThreads);
          if (b) { f = h0 + __ffsll((long long)b) - 1; break; }
        }
        if (lane == 0) X->gs = f;
      }
      fpg::prefix_slots(Ldr, g, X->red, X->add);
      gs = X->gs;
      const bool active = g <= gs && nc > 0;
      fs = g < gs ? nc : (g == gs ? fsl : 0);
      // start counts changed (or the chunk was idle): every point draws again
      bool restart_all = false;
      if (wv == 0) {
        const int c0 = (lane < nsl ? st.cnt[lane] : 0) + X->add[lane];
        const bool diff = c0 != X->sc_prev[lane];
        X->sc[lane] = c0;
        X->sc_prev[lane] = c0;
        const unsigned long long db = __ballot(diff);
        if (lane == 0) X->conv = db ? 1 : 0;
      }
      __syncthreads();
      if (X->conv || g > X->gs_prev) restart_all = true;
      if (restart_all) chg = -1;
      const bool mover = in && cls == 1 && tid < fs;
      // counts at each wave's first point (lane = slot)
      if (wv == 0) {
        int c = X->sc[lane];
        for (int w = 0; w < kFpWaves; ++w) {
          F->wc[w][lane] = c;
          c += F->wd[w][lane];
        }
      }
      __syncthreads();
      // (3) per wave: the movers per slot it touches (ballot masks)
      F->bin[wv][lane] = 0ull;
      F->bout[wv][lane] = 0ull;
      unsigned long long touch = mover ? ((1ull << own) | (1ull << tgt)) : 0ull;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) touch |= __shfl_xor(touch, o);
      for (unsigned long long t = touch; t; t &= t - 1) {
        const int sl = __ffsll((long long)t) - 1;
        const unsigned long long bi = __ballot(mover && tgt == sl), bo = __ballot(mover && own == sl);
        if (lane == 0) { F->bin[wv][sl] = bi; F->bout[wv][sl] = bo; }
      }
      wave_sync();
      auto corr = [&](int sl) -> int {
        return __popcll(F->bin[wv][sl] & below) - __popcll(F->bout[wv][sl] & below);
      };
      // (4) redraw behind the first changed outcome (k_resolve_fp's evaluation)
      bool changed = false;
      bool ev2 = false, need = false;
      int cnow2 = 0;
      const bool evl = active && in && tid > chg && tid <= fs;
      const double wdb = (struct0 && a.spec) ? fp_wave_drift_bound(a, st, F->wc[wv], F->bin[wv], F->bout[wv], nsl)
                                             : INFINITY;
      if (evl && struct0 && sp >= 0 && wdb < sr) {
        // every entry's drift is below this point's radius: its snapshot draw holds
        const int cnow = F->wc[wv][own] + corr(own);
        const bool single = cnow == 1;
        const int np = sp;
        fresh = false;
        int ncl = 2, nt = own;
        if (np < K) {
          const int s2 = st.sol[np];
          if (!single) { ncl = s2 != own ? 1 : 0; nt = s2; }
        } else if (single && np == K) {
          ncl = 0;
        }
        const int ctn = F->wc[wv][nt] + corr(nt);
        changed = ncl != cls || (ncl == 1 && nt != tgt);
        cls = ncl;
        tgt = nt;
        pick = np;
        co = cnow;
        ct = ctn;
      } else if (evl) {
        ev2 = true;
        cnow2 = F->wc[wv][own] + corr(own);
        // the snapshot draw holds while every log-count term drifted less than its radius
        bool take_spec = false;
        if (struct0 && sp >= 0) {
          const double drift = fp_lane_drift<EM>(st, F->wc[wv], corr, own, cnow2, K);
          take_spec = drift == 0.0 || drift < sr;
        }
        need = !take_spec;
      }
      // the draws of this round, compacted into dense waves (kernels.hip fp_draws_compacted)
      const int dpk = fp_draws_compacted<EM>(a, st, F, need, cq, K, E, ncol);
      if (ev2) {
        const int cnow = cnow2;
        const bool single = cnow == 1;
        const int np = need ? dpk : sp;
        fresh = need;
        int ncl = 2, nt = own;
        if (np >= 0) {
          if (np < K) {
            const int s2 = st.sol[np];
            if (!single) { ncl = s2 != own ? 1 : 0; nt = s2; }
          } else if (single && np == K) {
            ncl = 0;
          }
        }
        const int ctn = F->wc[wv][nt] + corr(nt);
        changed = ncl != cls || (ncl == 1 && nt != tgt);
        cls = ncl;
        tgt = nt;
        pick = np;
        co = cnow;
        ct = ctn;
      }
      const unsigned long long cbal = __ballot(changed);
      if (lane == 0) F->wchg[wv] = cbal ? wv * kWave + __ffsll((long long)cbal) - 1 : kFpThreads;
      __syncthreads();
      int c2 = kFpThreads;
      for (int w = 0; w < kFpWaves; ++w) c2 = min(c2, F->wchg[w]);
      if (tid == 0) {
        F->iters++;
        X->gs_prev = gs;
      }
      lastchg = c2 < kFpThreads ? 1 : 0;
      chg = c2 < kFpThreads ? c2 : nc;
      __syncthreads();              // (X->gs_prev, F->wchg before the next round rewrites them)
    }
    const long long tw1 = prof ? wall_clock64() : 0;
    if (prof) tp[3] += tw1 - tw0;
    if (!ok) break;
    if (!conv) {       // cannot happen (at most WIN + 1 rounds); stop loudly
      if (tid == 0) { S.status = 5; S.next = F->pi[0]; }
      go = false;
      break;
    }
    const bool active = g <= gs && nc > 0;
    // ---- the drift after each position: within the chunk, then across the chunks before it
    // (a dense launch lists every point: nothing to re-test, so neither phase runs)
    const bool mv = active && in && cls == 1 && tid < fs;
    double dwin = S.dnow;
    int ufirst = INT_MAX;
    if (!a.all_listed) {
    double sd = mv ? fmax(slot_drift_at(a, st, own, co - 1), slot_drift_at(a, st, tgt, ct + 1)) : 0.0;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const double x = __shfl_up(sd, o);
      if (lane >= o) sd = fmax(sd, x);
    }
    if (lane == kWave - 1) F->wsd[wv] = sd;
    if (wv == 0) F->cmo[lane] = 0;
    __syncthreads();
    if (mv) atomicAdd(&F->cmo[own], 1);
    if (tid == 0) {
      double m2 = 0.0;
      for (int w = 0; w < kFpWaves; ++w) m2 = fmax(m2, F->wsd[w]);
      L.sd[g] = m2;
    }
    if (!(ok = bar())) break;
    // the drift at this chunk's start and over the window (every chunk up to the stop)
    if (wv == 0) {
      const double x = fpg::wave_max_over(L.sd, min(g, gs + 1), S.dnow);
      const double y = fpg::wave_max_over(L.sd, min(G, gs + 1), S.dnow);
      if (lane == 0) { X->dch = x; X->dwin = y; }
    }
    __syncthreads();
    const double dch = X->dch;
    dwin = X->dwin;
    double dpre = dch;
    for (int w = 0; w < wv; ++w) dpre = fmax(dpre, F->wsd[w]);
    F->dnl[tid] = fmax(sd, dpre);
    __syncthreads();
    if (wv == 0) {
      int mn = F->wc[0][lane];
      for (int w = 1; w < kFpWaves; ++w) mn = min(mn, F->wc[w][lane]);
      F->cmin[lane] = mn - F->cmo[lane];
    }
    __syncthreads();
    // ---- unlisted points between this chunk's listed ones (before its stop), re-tested
    if (tid == 0) X->u = INT_MAX;
    __syncthreads();
    if (active) {
      const int64_t lo = g == 0 ? vfrom : (int64_t)gld(a.rq + cq - 1).y + 1;
      const int64_t hi = fs < nc ? F->pi[fs] : F->pi[nc - 1];
      const double dtop = fs > 0 ? F->dnl[fs - 1] : dch;
      if (dtop > a.dmax && hi > lo) {
        const int64_t u = fp_verify(a, st, F, fs, dch, lo, hi, F->cmin);
        if (u < hi && tid == 0) X->u = (int)u;
      }
    }
    __syncthreads();
    if (tid == 0) L.fail[g] = X->u;
    if (!(ok = bar())) break;
    if (wv == 0) {
      const int x = fpg::wave_min_over(L.fail, min(G, gs + 1), INT_MAX);
      if (lane == 0) X->ufirst = x;
    }
    __syncthreads();
    ufirst = X->ufirst;
    if (dwin > a.dmax && tid == 0) S.checked = 1;
    }
    // ---- commit the positions before the first stop and before the first failing point: the
    // count changes are published first, the labels and the move log written only after the
    // barrier, so a launch that gives up at that barrier has committed nothing of this window
    int kc = active ? fs : 0;
    if (ufirst != INT_MAX)
      while (kc > 0 && F->pi[kc - 1] >= ufirst) --kc;
    const bool cm = mv && tid < kc;
    const unsigned long long mmc = __ballot(cm);
    const unsigned long long fbal = __ballot(active && in && tid < kc && fresh);
    if (lane == 0) { F->wmov[wv] = __popcll(mmc); F->wfresh[wv] = __popcll(fbal); }
    if (wv == 0) F->wd[0][lane] = 0;
    __syncthreads();
    if (cm) {
      atomicAdd(&F->wd[0][own], -1);
      atomicAdd(&F->wd[0][tgt], 1);
    }
    __syncthreads();
    if (wv == 0) {
      L.dc[(size_t)g * kFpgSlots + lane] = F->wd[0][lane];
      if (lane == 0) {
        int nm = 0, nf = 0;
        for (int w = 0; w < kFpWaves; ++w) { nm += F->wmov[w]; nf += F->wfresh[w]; }
        L.mov[g] = nm;
        L.fresh[g] = nf;
      }
    }
    if (tid == fs && active && fs < nc) {
      F->stop_rq = r;
      F->stop_pick = pick;
      F->stop_fresh = fresh ? 1 : 0;
    }
    if (!(ok = bar())) break;
    // labels and the move log (positions: the window's log starts at F->nlog, this chunk's
    // after the moves of the chunks before it -- the order k_resolve_fp would log them in)
    if (wv == 0) {
      const int before = fpg::wave_sum_over(L.mov, g);
      if (lane == 0) X->red[0] = F->nlog + before;
    }
    __syncthreads();
    const int lbase = X->red[0];
    __syncthreads();             // (prefix_slots below reuses red)
    if (cm) {
      a.c[r.y] = tgt;
      if (a.mlog) {
        int q = lbase + __popcll(mmc & below);
        for (int w = 0; w < wv; ++w) q += F->wmov[w];
        a.mlog[3 * q] = r.y;
        a.mlog[3 * q + 1] = own;
        a.mlog[3 * q + 2] = tgt;
      }
    }
    // ---- every workgroup applies the window's committed changes to its copy of the state
    fpg::prefix_slots(L.dc, min(G, gs + 1), X->red, X->add);
    if (wv == 0) {
      double cd = 0.0;
      if (lane < nsl) {
        const int dl = X->add[lane];
        if (dl != 0) {
          const int c = st.cnt[lane] + dl;
          st.cnt[lane] = c;
          st.l1[lane] = fp_logn(a, c);
          st.l0[lane] = fp_logn(a, c - 1);
        }
        cd = count_drift(st, a.logn, lane);
      }
      cd = wave_max(cd);
      const int nm = fpg::wave_sum_over(L.mov, min(G, gs + 1));
      const int nf = fpg::wave_sum_over(L.fresh, min(G, gs + 1));
      if (lane == 0) {
        S.moves += nm;
        S.exact += nf;
        S.dnow = fmax(S.dnow, dwin);
        S.dvmax = fmax(S.dvmax, cd);
        if (a.mlog) F->nlog += nm;
      }
    }
    __syncthreads();
    if (ufirst != INT_MAX) {
      // a re-tested point is no longer certain: the launch restarts there
      if (tid == 0) { S.restart = 1; S.next = ufirst; S.checked = 1; }
      go = false;
      break;
    }
    if (gs < G) {
      // ---- the window's first stop: the serial path on the workgroup that holds it, in the
      // committed state; it publishes the state for the others (tagged with the window, last)
      qs = q0 + gs * kFpThreads + fpg::ald(L.stop + pb * G + gs);
      gs_stop = gs;
      if (g == gs) {
        if (wv == 0) fp_stop(a);
        __syncthreads();
        if (wv == 0) {
          L.sol[lane] = st.sol[lane];
          L.los[lane] = st.los[lane];
          L.cnt[lane] = st.cnt[lane];
          if (lane == 0) {
            int* m = L.ms;
            m[0] = S.K; m[1] = S.nslots; m[2] = S.status; m[3] = S.restart; m[4] = S.next; m[5] = S.nstruct;
            m[6] = S.exact; m[7] = S.moves; m[8] = F->go; m[9] = F->nlog; m[10] = S.checked;
            L.md[0] = S.dnow;
            L.md[1] = S.dvmax;
          }
          __threadfence();
          if (lane == 0) __hip_atomic_store(L.ms + 11, nwin, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (!(ok = bar())) { stopped = true; break; }
      if (g != gs) adopt();
      go = F->go != 0;
      vfrom = (int64_t)gld(a.rq + qs).y + 1;
      q0 = qs + 1;
    } else {
      const int qe = min(total, q0 + WIN);
      vfrom = (int64_t)gld(a.rq + qe - 1).y + 1;
      q0 = qe;
    }
    if (prof) tp[4] += wall_clock64() - tw1;
    __syncthreads();
  }
  if (g != 0) return;
  if (!ok) {
    // A barrier gave up (a workgroup was not resident in time, or fpg_fail): no workgroup got past
    // it, so the committed state is the one at a window boundary -- before this window's commit
    // (workgroup 0's copy of the state is that state), or after its stop, which the stopping
    // workgroup published before the barrier.  The launch ends as a restart at the first point
    // not decided; the host runs that restart with the one-workgroup resolver.
    bool known = true;
    if (stopped && gs_stop != 0) {
      if (wv == 0) {
        const long long t0 = wall_clock64();
        int tag = 0;
        while ((tag = __hip_atomic_load(L.ms + 11, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != nwin &&
               wall_clock64() - t0 < a.fpg_limit)
          __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lane == 0) X->flag = tag == nwin ? 1 : 0;
      }
      __syncthreads();
      known = X->flag != 0;
      if (known) adopt();
    }
    if (tid == 0) {
      if (!known) {
        S.status = 5;              // the stopping workgroup never published: a resolver failure
        S.next = (int)a.p0;
      } else {
        S.aborted = 1;
        if (!(stopped && !F->go)) {
          // (a stop that ended the launch itself keeps its own restart / status)
          S.restart = 1;
          S.next = (int)(stopped ? (int64_t)gld(a.rq + qs).y + 1 : vfrom);
        }
      }
    }
    __syncthreads();
  }
  // the unlisted points after the last listed one (one workgroup, as k_resolve_fp)
  if (ok && go && S.status == 0 && !S.restart && S.dnow > a.dmax) (void)fp_verify(a, st, F, 0, S.dnow, vfrom, a.n, st.cnt);
  if (tid == 0) { tp[5] = F->iters; S.tsub[0] = nwin; S.tsub[1] = total; }
  resolve_finish(a, st, F->nlog, tp, a.prof != nullptr);
}
