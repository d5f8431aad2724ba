// split_merge.inl -- split-merge move (code/split_merge.cpp) on the hdpm runtime.
// Included by engine.cpp.  The orchestration (launch states, acceptance ratio, clean_var)
// runs on the host with the reference's draw order; the restricted Gibbs scan
// (sm:163-225) and the logprobgs_c_i sum (sm:96-161) run on the device.
#pragma once

namespace hdpm {

hipError_t launch_sm_ll(const SmArgs& a, hipStream_t s);
hipError_t launch_sm_scan(const SmArgs& a, hipStream_t s);
hipError_t launch_sm_lpgs(const SmArgs& a, hipStream_t s);
hipError_t launch_sm_freq(const SmFreqArgs& a, hipStream_t s);
bool sm_ll_lds_fits(int d, int nq);
int sm_scan_wide_grid(int nS);
hipError_t launch_sm_scan_wide(const SmArgs& a, int G, hipStream_t s);
hipError_t launch_sm_link(const SmLinkArgs& a, hipStream_t s);
hipError_t launch_sm_tabs(const SmTabsArgs& a, hipStream_t s);
hipError_t launch_phi2(const PhiArgs& a, hipStream_t s, hipEvent_t before_values);

// HDPM_SM_WIDE=0: the one-workgroup restricted scan only (A/B of k_sm_scan_wide, the default:
// 13.5 against 80 us per C4 scan, profiles/r05/split_merge/wide/)
static bool sm_wide_on() {
  static const bool on = [] {
    const char* e = std::getenv("HDPM_SM_WIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// A host copy of internal_state (cfh:32-63): labels, parameters, sizes.
struct HState {
  std::vector<int32_t> c;
  int K = 0;
  std::vector<uint8_t> center;  // K x d
  std::vector<double> sigma;    // K x d
  std::vector<int32_t> counts;  // K
};

static SmWork& smwork(Ctx* c) { return c->sm; }

static void ctx_to_hstate(Ctx* c, HState& s) {
  c->download_labels();
  s.c = c->h_c;
  s.K = c->K;
  s.center = c->h_center;
  s.sigma = c->h_sigma;
  s.counts = c->h_counts;
}

static void hstate_to_ctx(Ctx* c, const HState& s) {
  c->h_c = s.c;
  c->K = s.K;
  c->h_center = s.center;
  c->h_sigma = s.sigma;
  c->h_counts = s.counts;
  c->upload_labels();
  c->upload_clusters();
}

// validate_state (cf:146-172) on a host state.
static int hvalidate(const HState& s) {
  int mx = -1;
  for (int x : s.c) mx = std::max(mx, x);
  std::vector<char> seen(mx + 2, 0);
  int u = 0;
  for (int x : s.c)
    if (x >= 0 && !seen[x]) { seen[x] = 1; u++; }
  return u == s.K ? kOk : kValidate;
}

// Per-attribute dhamming values for a parameter row (host glibc, as the device tables).
static void row_tables(const Ctx* c, const uint8_t* cen, const double* sig, std::vector<double>& tab) {
  tab.resize(2 * c->d);
  for (int j = 0; j < c->d; ++j) dhamming_pair(sig[j], c->att[j], &tab[2 * j], &tab[2 * j + 1]);
  (void)cen;
}

// Adds the wall time of its scope to a stats field.
struct SmTimer {
  double& acc;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit SmTimer(double& a) : acc(a) {}
  ~SmTimer() { acc += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
};

// Frequency tables of one cluster (f[j * mmax + l] = members with code l + 1 at attribute j,
// integer-valued doubles) and its size.  The split-merge move touches only the members M =
// S + {i1, i2} of c(i1) and c(i2) (sm:263-301), so every table it needs is a subset of M's;
// they are built once per move and updated by the points a restricted scan moves, instead of
// the reference's O(N D) membership scan per update_phi / logprobgs_phi call.  Counts are
// exact in doubles, so the tables equal the reference's freq bit for bit.
struct Freq {
  std::vector<double> f;
  int nn = 0;
};

// Table of the members q of M with s.c[q] == k (k < 0: all of M); attribute ranges on the
// host pool for wide rows.
static void freq_over(const Ctx* c, const HState& s, const std::vector<int>& M, int k, Freq& F) {
  F.f.assign((size_t)c->d * c->mmax, 0.0);
  std::vector<int> mem;
  mem.reserve(M.size());
  for (int q : M)
    if (k < 0 || s.c[q] == k) mem.push_back(q);
  F.nn = (int)mem.size();
  const int64_t work = (int64_t)mem.size() * c->d;
  const int chunk = 32;
  const int nchunk = (c->d + chunk - 1) / chunk;
  auto run = [&](int ch) {
    const int j0 = ch * chunk, j1 = std::min(c->d, j0 + chunk);
    double* f = F.f.data();
    for (int q : mem) {
      const uint8_t* x = &c->codes[(size_t)q * c->d];
      for (int j = j0; j < j1; ++j) f[(size_t)j * c->mmax + (x[j] - 1)] += 1.0;
    }
  };
  if (work >= (1 << 18) && nchunk > 1) pool_for(nchunk, run, 1);
  else for (int ch = 0; ch < nchunk; ++ch) run(ch);
}

// Rows `to1` move from F2 to F1 and rows `to2` from F1 to F2 (attribute ranges on the host
// pool when there are many).
static void freq_move(const Ctx* c, Freq& F1, Freq& F2, const std::vector<int>& to1, const std::vector<int>& to2) {
  const int64_t work = (int64_t)(to1.size() + to2.size()) * c->d;
  const int chunk = 32;
  const int nchunk = (c->d + chunk - 1) / chunk;
  auto run = [&](int ch) {
    const int j0 = ch * chunk, j1 = std::min(c->d, j0 + chunk);
    double* f1 = F1.f.data();
    double* f2 = F2.f.data();
    for (int i : to1) {
      const uint8_t* x = &c->codes[(size_t)i * c->d];
      for (int j = j0; j < j1; ++j) {
        const size_t o = (size_t)j * c->mmax + (x[j] - 1);
        f1[o] += 1.0;
        f2[o] -= 1.0;
      }
    }
    for (int i : to2) {
      const uint8_t* x = &c->codes[(size_t)i * c->d];
      for (int j = j0; j < j1; ++j) {
        const size_t o = (size_t)j * c->mmax + (x[j] - 1);
        f2[o] += 1.0;
        f1[o] -= 1.0;
      }
    }
  };
  if (work >= (1 << 18) && nchunk > 1) pool_for(nchunk, run, 1);
  else for (int ch = 0; ch < nchunk; ++ch) run(ch);
  F1.nn += (int)to1.size() - (int)to2.size();
  F2.nn += (int)to2.size() - (int)to1.size();
}

// Tables of the two clusters that split M in s: rows labelled k1 into F1, the others into
// F2, in one pass (attribute ranges on the host pool).
static void freq_split(const Ctx* c, const HState& s, const std::vector<int>& M, int k1, Freq& F1, Freq& F2) {
  F1.f.assign((size_t)c->d * c->mmax, 0.0);
  F2.f.assign((size_t)c->d * c->mmax, 0.0);
  int n1 = 0;
  for (int q : M) n1 += s.c[q] == k1;
  F1.nn = n1;
  F2.nn = (int)M.size() - n1;
  const int chunk = 32;
  const int nchunk = (c->d + chunk - 1) / chunk;
  auto run = [&](int ch) {
    const int j0 = ch * chunk, j1 = std::min(c->d, j0 + chunk);
    for (int q : M) {
      double* f = (s.c[q] == k1 ? F1 : F2).f.data();
      const uint8_t* x = &c->codes[(size_t)q * c->d];
      for (int j = j0; j < j1; ++j) f[(size_t)j * c->mmax + (x[j] - 1)] += 1.0;
    }
  };
  if ((int64_t)M.size() * c->d >= (1 << 18) && nchunk > 1) pool_for(nchunk, run, 1);
  else for (int ch = 0; ch < nchunk; ++ch) run(ch);
}

static void freq_plus(const Freq& A, const Freq& B, Freq& out) {
  out.f.resize(A.f.size());
  for (size_t i = 0; i < A.f.size(); ++i) out.f[i] = A.f[i] + B.f[i];
  out.nn = A.nn + B.nn;
}

static void freq_minus(const Freq& A, const Freq& B, Freq& out) {
  out.f.resize(A.f.size());
  for (size_t i = 0; i < A.f.size(); ++i) out.f[i] = A.f[i] - B.f[i];
  out.nn = A.nn - B.nn;
}

// update_phi (cf:511-591) of one cluster k of s whose table is F.
// The center probabilities of every attribute are computed first (on the host pool for wide
// rows; each attribute's values come from the same expressions), then drawn in attribute
// order, then the sigmas (Ctx::sample_sigma_wide).
static int hupdate_phi_one(Ctx* c, HState& s, int k, const Freq& F) {
  if (F.nn == 0) return kOk;
  SmTimer tm(c->stats.t_sm_phi_ms);
  const int mm = c->mmax;
  std::vector<double> prob((size_t)c->d * mm), cum((size_t)c->d * mm), nv(c->d), nw(c->d);
  std::vector<int> perm((size_t)c->d * mm), pst(c->d);
  const double nn = (double)F.nn;
  uint8_t* cen = &s.center[(size_t)k * c->d];
  double* sig = &s.sigma[(size_t)k * c->d];
  auto probs = [&](int j) {    // cf:496-503
    const int mj = c->att[j];
    const double* f = &F.f[(size_t)j * mm];
    double* pr = &prob[(size_t)j * mm];
    for (int l = 0; l < mj; ++l) pr[l] = (-(nn - f[l])) / sig[j];
    double mx = pr[0];
    for (int l = 1; l < mj; ++l) if (pr[l] > mx) mx = pr[l];
    for (int l = 0; l < mj; ++l) pr[l] = std::exp(pr[l] - mx);
    double sum = 0.0;
    for (int l = 0; l < mj; ++l) sum += pr[l];
    for (int l = 0; l < mj; ++l) pr[l] = pr[l] / sum;
    // sample(1:m_j, 1, TRUE, prob) up to its uniform: FixupProb, revsort, cumulative sums
    pst[j] = sample_prob1_prep(pr, mj, &cum[(size_t)j * mm], &perm[(size_t)j * mm]);
  };
  if (c->d >= 128) pool_for(c->d, probs, 16);
  else for (int j = 0; j < c->d; ++j) probs(j);
  c->rng_sync();
  for (int j = 0; j < c->d; ++j) {
    if (pst[j] < 0) return -pst[j];           // validation precedes the draw
    const int pick = sample_prob1_pick(&cum[(size_t)j * mm], &perm[(size_t)j * mm], c->att[j], c->rng.unif(), pst[j]);
    cen[j] = (uint8_t)(pick + 1);
  }
  for (int j = 0; j < c->d; ++j) {
    const double sumdelta = F.f[(size_t)j * c->mmax + (cen[j] - 1)];
    nw[j] = c->w[j] + nn - sumdelta;
    nv[j] = c->v[j] + sumdelta;
  }
  return c->sample_sigma_wide(nv.data(), nw.data(), sig);
}

// update_phi (cf:511-591) of clusters ks[0..nk) (ascending labels: the order of the
// reference's cluster mask) for wide rows, through the engine's update_phi pipeline
// (Ctx::pj_*, the Neal-8 path's): the stream slice is generated ahead with its logits on the
// host pool, phase A (center probabilities, revsort, rhig branch and rbeta constants of the
// likely center) runs per attribute on the pool, phase B draws in reference order with
// speculative first rbeta attempts, phase C solves the bisections.  Same expressions and
// draws as hupdate_phi_one; one pool job per call instead of two pool passes and serial
// log / exp per rbeta attempt.
static int hupdate_phi_job(Ctx* c, HState& s, const int* ks, const Freq* const* Fs, int nk) {
  SmTimer tm(c->stats.t_sm_phi_ms);
  const int d = c->d, mm = c->mmax;
  std::vector<unsigned> fq((size_t)nk * d * mm);
  std::vector<int> cnt(nk);
  std::vector<uint8_t> cen((size_t)nk * d);
  std::vector<double> sig((size_t)nk * d);
  std::vector<int> touched;
  for (int t = 0; t < nk; ++t) {
    const Freq& F = *Fs[t];
    cnt[t] = F.nn;
    for (size_t e = 0; e < (size_t)d * mm; ++e) fq[(size_t)t * d * mm + e] = (unsigned)F.f[e];
    std::memcpy(&cen[(size_t)t * d], &s.center[(size_t)ks[t] * d], d);
    std::memcpy(&sig[(size_t)t * d], &s.sigma[(size_t)ks[t] * d], (size_t)d * 8);
    if (F.nn > 0) touched.push_back(t);
  }
  if (touched.empty()) return kOk;
  SmWork& W = smwork(c);
  c->rng_sync();
  StreamAhead& sa = c->phi_stream;
  if (W.phi_prefetch <= 0) W.phi_prefetch = (int64_t)4 * nk * d + 1024;
  if (!c->fill_stream_from(W.phi_prefetch)) {
    // an unseeded stream: the one-pass path
    for (int t = 0; t < nk; ++t) {
      const int st = hupdate_phi_one(c, s, ks[t], *Fs[t]);
      if (st) return st;
    }
    return kOk;
  }
  sa.used = 0;
  HostPool::get().run(sa.n, 1024, [&](int64_t a0, int64_t a1) { sa.logits(a0, a1); });
  sa.avail = INT64_MAX;
  sa.wait_avail = nullptr;
  sa.live = &c->rng;
  c->pj_setup(touched, 0, cnt.data(), fq.data(), cen.data(), sig.data(), UploadLayout{}, false, nullptr, false);
  c->pj.sig_in = sig.data();
  c->pj.stage = false;
  c->pj_launch();
  const int berr = c->pj_finish();
  const int gsl_t = c->pj.gsl.load();
  sa.finish();
  W.phi_prefetch = std::max<int64_t>((int64_t)nk * d + 1024, sa.used + sa.used / 4 + 512);
  sa.n = 0;
  if (berr) return berr;
  if (gsl_t >= 0) return kGsl;
  for (int t : touched) {
    std::memcpy(&s.center[(size_t)ks[t] * d], &cen[(size_t)t * d], d);
    std::memcpy(&s.sigma[(size_t)ks[t] * d], &sig[(size_t)t * d], (size_t)d * 8);
  }
  return kOk;
}

// update_phi (cf:511-591) of clusters ks[0..nk) (ascending labels) on the device
// (Ctx::device_update_phi_sm, csrc/phi.hip): -1 when it does not apply (the host job runs).
static int dupdate_phi_sm(Ctx* c, HState& s, const int* ks, const Freq* const* Fs, int nk) {
  if (c->phi_mode == 0 || c->phi_mode == 3) return -1;    // (automatic mode: the host job)
  SmTimer tm(c->stats.t_sm_phi_ms);
  const int d = c->d, mm = c->mmax;
  std::vector<int> idx;
  for (int t = 0; t < nk; ++t)
    if (Fs[t]->nn > 0) idx.push_back(t);
  const int T = (int)idx.size();
  if (T == 0) return kOk;
  std::vector<unsigned> fq((size_t)T * d * mm);
  std::vector<int> cnt(T);
  std::vector<double> sg((size_t)T * d), so((size_t)T * d);
  std::vector<uint8_t> cen((size_t)T * d);
  for (int q = 0; q < T; ++q) {
    const Freq& F = *Fs[idx[q]];
    cnt[q] = F.nn;
    for (size_t e = 0; e < (size_t)d * mm; ++e) fq[(size_t)q * d * mm + e] = (unsigned)F.f[e];
    std::memcpy(&sg[(size_t)q * d], &s.sigma[(size_t)ks[idx[q]] * d], (size_t)d * 8);
  }
  const int st = c->device_update_phi_sm(T, cnt.data(), fq.data(), sg.data(), cen.data(), so.data());
  if (st != kOk) return -1;
  for (int q = 0; q < T; ++q) {
    std::memcpy(&s.center[(size_t)ks[idx[q]] * d], &cen[(size_t)q * d], d);
    std::memcpy(&s.sigma[(size_t)ks[idx[q]] * d], &so[(size_t)q * d], (size_t)d * 8);
  }
  return kOk;
}

// update_phi of {ka, kb} in the reference's order (ascending label; a repeated label once)
static int hupdate_phi_pair(Ctx* c, HState& s, int ka, const Freq& Fa, int kb, const Freq& Fb) {
  {
    // on the device when update_phi is placed there (HDPM_OPT_PHI_DEVICE)
    const int ks[2] = {std::min(ka, kb), std::max(ka, kb)};
    const Freq* fs[2] = {ka <= kb ? &Fa : &Fb, ka <= kb ? &Fb : &Fa};
    if (dupdate_phi_sm(c, s, ks, fs, ka == kb ? 1 : 2) == kOk) return kOk;
  }
  if (c->d < 128 || (c->debug & 128)) {
    int st = ka <= kb ? hupdate_phi_one(c, s, ka, Fa) : hupdate_phi_one(c, s, kb, Fb);
    if (st) return st;
    if (ka != kb) st = ka < kb ? hupdate_phi_one(c, s, kb, Fb) : hupdate_phi_one(c, s, ka, Fa);
    return st;
  }
  if (ka == kb) return hupdate_phi_job(c, s, &ka, std::array<const Freq*, 1>{&Fa}.data(), 1);
  const int ks[2] = {std::min(ka, kb), std::max(ka, kb)};
  const Freq* fs[2] = {ka < kb ? &Fa : &Fb, ka < kb ? &Fb : &Fa};
  return hupdate_phi_job(c, s, ks, fs, 2);
}

static void hrecount(const Ctx* c, HState& s) {
  s.counts.assign(s.K, 0);
  for (int i = 0; i < c->n; ++i)
    if (s.c[i] >= 0 && s.c[i] < s.K) s.counts[s.c[i]]++;
}

// Device: exact lls of the S points against clusters (k1, k2) of state s.
// The pinned staging buffers are reused by the next call only after a stream wait (every
// caller synchronizes before it returns).
static void sm_upload_two(Ctx* c, SmWork& W, const HState& s, int k1, int k2) {
  const size_t nc = 2 * (size_t)c->dp, nt = 4 * (size_t)c->d;
  W.h_two_codes.ensure(nc);
  W.h_two_tab.ensure(nt);
  uint8_t* cc = W.h_two_codes.p;
  double* tt = W.h_two_tab.p;
  std::memset(cc, 0, nc);
  if (c->d >= 128) {
    // wide rows: the two clusters' dhamming pairs (an exp and a log each) on the host pool
    const int d = c->d;
    const uint8_t* c1 = &s.center[(size_t)k1 * d];
    const uint8_t* c2 = &s.center[(size_t)k2 * d];
    const double* s1 = &s.sigma[(size_t)k1 * d];
    const double* s2 = &s.sigma[(size_t)k2 * d];
    pool_for(2 * d, [&](int q) {
      const int e = q / d, j = q - e * d;
      cc[e * c->dp + j] = (e ? c2 : c1)[j];
      dhamming_pair((e ? s2 : s1)[j], c->att[j], &tt[2 * d * e + 2 * j], &tt[2 * d * e + 2 * j + 1]);
    }, 64);
  } else {
    c->tables_for(&s.center[(size_t)k1 * c->d], &s.sigma[(size_t)k1 * c->d], cc, tt);
    c->tables_for(&s.center[(size_t)k2 * c->d], &s.sigma[(size_t)k2 * c->d], cc + c->dp, tt + 2 * c->d);
  }
  W.d_two_codes.ensure(nc);
  W.d_two_tab.ensure(nt);
  HIPCHK(hipMemcpyAsync(W.d_two_codes.p, cc, nc, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(W.d_two_tab.p, tt, nt * 8, hipMemcpyHostToDevice, c->stream));
}

static SmArgs sm_args(Ctx* c, SmWork& W, int nS) {
  SmArgs a;
  a.codes_t = c->d_codes_t.p; a.n = c->n; a.d = c->d; a.nq = c->nq;
  a.S = W.d_S.p; a.nS = nS;
  a.two = ParamTables{W.d_two_codes.p, W.d_two_tab.p};
  a.ll = W.d_ll.p; a.side = W.d_side.p; a.side_ref = W.d_side_ref.p; a.raw = W.d_raw.p;
  a.logn = c->d_logn.p; a.n1 = 0; a.n2 = 0; a.out_counts = W.d_counts2.p; a.out = W.d_out.p;
  a.cert = W.d_cert.p;
  a.side_prev = nullptr;
  a.cert_in_ll = 0;
  a.zero = nullptr;
  a.zero_n = 0;
  a.wide_buf = nullptr;
  a.wide_limit = 0;
  a.link = nullptr;
  return a;
}

static void sm_upload_S(Ctx* c, SmWork& W, const std::vector<int>& S) {
  const size_t nS = S.size();
  W.d_S.ensure(std::max<size_t>(nS, 1));
  W.d_side.ensure(std::max<size_t>(nS, 1));
  W.d_side_ref.ensure(std::max<size_t>(nS, 1));
  W.d_ll.ensure(std::max<size_t>(2 * nS, 2));
  W.d_raw.ensure(std::max<size_t>(nS, 1));
  W.d_cert.ensure(std::max<size_t>(6 * nS, 6));
  W.d_counts2.ensure(2);
  W.d_out.ensure(std::max<size_t>(2 * ((nS + kBlock - 1) / kBlock), 2));
  if (nS) HIPCHK(hipMemcpyAsync(W.d_S.p, S.data(), nS * 4, hipMemcpyHostToDevice, c->stream));
}

// Table of the points of S (uploaded, W.d_S) on side `want` of the device sides (or all of
// them: side = nullptr) plus the points e0, e1 (>= 0), counted on the device (k_sm_freq): one
// launch and one table download instead of a host pass over |S| D codes.  With side_prev,
// F is updated instead by the points whose side differs from side_prev (+1 onto `want`, -1
// off it): after a scan only the points it moved are counted.
static void sm_freq_device(Ctx* c, SmWork& W, int nS, const int* side, int want, int e0, int e1, Freq& F,
                           const int* side_prev = nullptr, bool prezeroed = false) {
  const size_t nt = (size_t)c->d * c->mmax;
  W.d_freq.ensure(nt);
  W.h_freq.ensure(nt);
  SmFreqArgs a;
  a.codes_t = c->d_codes_t.p; a.n = c->n; a.d = c->d; a.nq = c->nq; a.mmax = c->mmax;
  a.list = W.d_S.p; a.nlist = nS; a.side = side; a.want = want;
  a.extra[0] = e0; a.extra[1] = e1;
  a.side_prev = side_prev;
  a.out = W.d_freq.p;
  a.prezeroed = prezeroed ? 1 : 0;
  a.link = nullptr;
  HIPCHK(launch_sm_freq(a, c->stream));
  HIPCHK(hipMemcpyAsync(W.h_freq.p, W.d_freq.p, nt * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int32_t* h = (const int32_t*)W.h_freq.p;
  int nn = 0;
  // every counted point has a code in 1..m_0 at attribute 0, so row 0 sums to the point count:
  // this relies on Ctx::set_data rejecting code 0 ("codes must lie in 1..attrisize[j]") and on
  // k_sm_freq counting every code >= 1.  If codes ever admit 0 (NA), count the points here.
  for (int l = 0; l < c->mmax; ++l) nn += h[l];
  if (side_prev) {
    for (size_t e = 0; e < nt; ++e) F.f[e] += (double)h[e];
    F.nn += nn;
  } else {
    F.f.resize(nt);
    for (size_t e = 0; e < nt; ++e) F.f[e] = (double)h[e];
    F.nn = nn;
  }
}


// sm:163-225's t scans, each followed by update_phi({c1, c2}) (sm:221), as one device chain
// when the move's tables live on the device.  Per scan k: k_sm_link (the scan's draws after the
// previous update's end, its sizes, the previous updates' tables in side order) -> k_sm_ll_lds
// -> k_sm_scan_wide / k_sm_scan -> k_sm_freq (the points the scan moved) -> k_sm_tabs (both
// tables, the updates' sizes) -> update_phi({c1, c2}) as two fast one-cluster device updates in
// ascending label order (launch_phi2, chained: the first draws after the scan's nS, the second
// after the first; inputs on the device).  Each one-cluster update starts at drift 0, so its
// center picks are fixed by its first d uniforms (k_phi2_group) -- a two-cluster update's second
// cluster starts at an unknown drift, and a freshly split cluster's picks depend on it.  No host
// step between scans: the sides, tables, chain words and the last updates' outputs come down
// once.  An update the device hands back (or a scan whose draws would leave the stream window)
// turns every later step off, so the device holds the state after the last complete step and
// the host continues from there: *next_iter, and *at_phi = 1 when that iteration's scan ran (both
// updates to do), 2 when its first update completed too (the larger label's update to do).
// -1: not applicable (nothing changed, nothing enqueued).
static int sm_chain(Ctx* c, SmWork& W, const std::vector<int>& S, HState& s, int i1, int i2, int t, Freq& F1,
                    Freq& F2, const Freq& FM, int* next_iter, int* at_phi) {
  *next_iter = 0;
  *at_phi = 0;
  const int c1 = s.c[i1], c2 = s.c[i2];
  const int nS = (int)S.size(), d = c->d, mm = c->mmax;
  if (c->sm_chain_mode == 0 || t < 1 || t > 64 || nS < 1 || c1 == c2) return -1;
  if (c->phi_mode == 0 || (c->debug & (524288 | 64 | 65536)) || d > 2048 || !Ctx::glibc_selfcheck()) return -1;
  if (!sm_ll_lds_fits(d, c->nq)) return -1;
  bool fast = false;
  const Ctx::PhiPlan pf = c->fast_plan(1, true, 16, &fast);
  if (!fast) return -1;
  c->rng_sync();
  const uint64_t P0 = c->rng.pos;
  RngWindow* Wn = c->window_at(P0, (int64_t)t * (nS + 2 * pf.need));
  if (!Wn || !c->can_adopt(*Wn, P0)) return -1;
  SmTimer tm(c->stats.t_sm_scan_ms);
  c->dspec_drain();                                 // phd's scratch is the chain's now
  hipStream_t st = c->stream;
  auto& phd = c->phd;
  const size_t nt = (size_t)d * mm;
  const int a1 = c1 < c2 ? 0 : 1;                   // c_i_1's place in ascending label order
  const int klab[2] = {std::min(c1, c2), std::max(c1, c2)};
  const int Gw = sm_wide_on() ? sm_scan_wide_grid(nS) : 0;
  const size_t wstride = 4 + 2 * (size_t)std::max(Gw, 1);
  const size_t stage_b = align16(upload_layout(1, c->dp, d, c->bw).bytes);
  size_t o_pick, o_sig, o_ll, obytes;
  Ctx::phi_out_layout(1, d, &o_pick, &o_sig, &o_ll, &obytes);
  const size_t o_state = align16(obytes), out_b = align16(o_state + 625 * 4 + 64);
  const int nu = 2 * t;                             // updates: scan k's are 2k (lower label), 2k + 1
  const int tc = std::max(t, 16);                   // (sized once for the usual t: no reallocation)
  W.d_links.ensure(tc);
  W.d_chain.ensure(1 + 3 * (size_t)tc);
  W.d_F.ensure(2 * nt);
  W.d_FM.ensure(nt);
  W.d_labcnt.ensure(4 * (size_t)tc);
  W.d_labdev.ensure(4 * (size_t)tc);
  W.d_stage.ensure(stage_b * 2 * tc);
  W.d_sig.ensure((size_t)(tc + 1) * 2 * d);
  W.h_cout.ensure(out_b * 2 * tc, hipHostMallocCoherent);
  W.d_wide.ensure(wstride * tc);
  W.d_side_prev.ensure(std::max(nS, 1));
  W.d_freq.ensure(nt);
  W.h_side.ensure(std::max(nS, 1));
  // inputs: both tables and the table of S + {i1, i2} (counts, exact in u32), both sigma rows,
  // the seed chain word (the first scan's draws start at P0)
  const size_t o_fm = align16(2 * nt * 4), o_sg = align16(o_fm + nt * 4), o_seed = align16(o_sg + 2 * (size_t)d * 8),
               in_b = o_seed + sizeof(PhiChain);
  W.h_cin.ensure(in_b + 64);
  {
    uint32_t* hf = (uint32_t*)W.h_cin.p;
    for (size_t e = 0; e < nt; ++e) {
      hf[a1 * nt + e] = (uint32_t)F1.f[e];
      hf[(1 - a1) * nt + e] = (uint32_t)F2.f[e];
      ((uint32_t*)(W.h_cin.p + o_fm))[e] = (uint32_t)FM.f[e];
    }
    double* hs = (double*)(W.h_cin.p + o_sg);
    std::memcpy(hs + (size_t)a1 * d, &s.sigma[(size_t)c1 * d], (size_t)d * 8);
    std::memcpy(hs + (size_t)(1 - a1) * d, &s.sigma[(size_t)c2 * d], (size_t)d * 8);
    PhiChain seed{(int64_t)P0, 1, 0};
    std::memcpy(W.h_cin.p + o_seed, &seed, sizeof(seed));
  }
  HIPCHK(hipMemcpyAsync(W.d_F.p, W.h_cin.p, 2 * nt * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(W.d_FM.p, W.h_cin.p + o_fm, nt * 4, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(W.d_sig.p, W.h_cin.p + o_sg, 2 * (size_t)d * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(W.d_chain.p, W.h_cin.p + o_seed, sizeof(PhiChain), hipMemcpyHostToDevice, st));
  sm_upload_two(c, W, s, c1, c2);                   // the first scan's tables (later ones: k_sm_link)
  HIPCHK(hipStreamWaitEvent(st, Wn->done, 0));
  if (phd.last_s && phd.last_s != st) HIPCHK(hipStreamWaitEvent(st, phd.ev_last, 0));
  if (!phd.ev_last) HIPCHK(hipEventCreateWithFlags(&phd.ev_last, hipEventDisableTiming));
  if (!phd.status.p) {
    phd.status.ensure(4);
    HIPCHK(hipMemsetAsync(phd.status.p, 0, 16, st));
  }
  if (!phd.ctr.p) {
    phd.ctr.ensure(2);
    HIPCHK(hipMemsetAsync(phd.ctr.p, 0, 2 * sizeof(int), st));
  }
  phd.gtab2.ensure((size_t)pf.G * pf.tW);
  phd.roots.ensure((size_t)pf.tW);
  // chain words: [0] the seed, then per scan k the link's (1 + 3k) and its updates' (2 + 3k, 3 + 3k)
  auto link_w = [](int k) { return 1 + 3 * k; };
  auto upd_w = [](int u) { return 2 + 3 * (u >> 1) + (u & 1); };
  c->mark("sm.chain_in");
  for (int k = 0; k < t; ++k) {
    SmLink* lk = W.d_links.p + k;
    SmLinkArgs la{};
    la.prev = W.d_chain.p + (k == 0 ? 0 : upd_w(2 * k - 1));
    la.counts_in = k == 0 ? nullptr : W.d_counts2.p;
    la.n1 = F1.nn;
    la.n2 = F2.nn;
    la.nS = nS;
    la.win_raw = Wn->raw.p;
    la.win_start = (int64_t)Wn->start_pos;
    la.win_count = c->sm_chain_mode == 2 + 3 * k ? 0 : Wn->count;   // (testing: this scan off)
    la.link = lk;
    la.chain = W.d_chain.p + link_w(k);
    for (int e = 0; e < 2; ++e) la.stage[e] = k == 0 ? nullptr : W.d_stage.p + stage_b * (2 * (k - 1) + e);
    la.dp = c->dp;
    la.d = d;
    la.bw = c->bw;
    la.swap = a1;
    la.two_codes = W.d_two_codes.p;
    la.two_tab = W.d_two_tab.p;
    HIPCHK(launch_sm_link(la, st));
    SmArgs a = sm_args(c, W, nS);
    a.raw = nullptr;
    a.link = lk;
    a.side_prev = W.d_side_prev.p;
    a.cert_in_ll = 1;
    a.zero = W.d_freq.p;
    a.zero_n = (int)nt;
    HIPCHK(launch_sm_ll(a, st));
    if (Gw) {
      a.wide_buf = W.d_wide.p + wstride * k;
      a.wide_limit = c->sm_wide_ticks;
      HIPCHK(launch_sm_scan_wide(a, Gw, st));
    }
    HIPCHK(launch_sm_scan(a, st));
    SmFreqArgs fa{};
    fa.codes_t = c->d_codes_t.p; fa.n = c->n; fa.d = d; fa.nq = c->nq; fa.mmax = mm;
    fa.list = W.d_S.p; fa.nlist = nS; fa.side = W.d_side.p; fa.want = 0;
    fa.extra[0] = -1; fa.extra[1] = -1;
    fa.side_prev = W.d_side_prev.p;
    fa.out = W.d_freq.p;
    fa.prezeroed = 1;
    fa.link = lk;
    HIPCHK(launch_sm_freq(fa, st));
    SmTabsArgs ta{lk, W.d_freq.p, W.d_FM.p, W.d_F.p, a1, (int)nt, W.d_counts2.p, W.d_labcnt.p + 4 * k};
    HIPCHK(launch_sm_tabs(ta, st));
    // the scan's update_phi({c1, c2}): the lower label's update behind the link (its first draw
    // after the scan's nS), the larger label's behind it
    for (int e = 0; e < 2; ++e) {
      const int u = 2 * k + e;
      PhiArgs pa = c->phi_args(pf);
      pa.freq = W.d_F.p;
      pa.lab = W.d_labcnt.p + 4 * k + e;
      pa.cnt = W.d_labcnt.p + 4 * k + 2 + e;
      pa.sig_in = W.d_sig.p + ((size_t)k * 2 + e) * d;
      pa.chain_in = W.d_chain.p + (e == 0 ? link_w(k) : upd_w(u - 1));
      pa.chain_out = W.d_chain.p + upd_w(u);
      pa.win_raw = Wn->raw.p;
      pa.win_start = (int64_t)Wn->start_pos;
      pa.win_count = c->sm_chain_mode == 3 + 3 * k + e ? 0 : Wn->count;   // (testing: this update off)
      pa.win_mti0 = Wn->mti0;
      pa.sweep_len = e == 0 ? nS : 0;
      pa.raw = nullptr; pa.nraw = 0; pa.raw_back = 0; pa.mti_pos = 0; pa.pos0 = 0;
      pa.status = phd.status.p;
      pa.stage = W.d_stage.p + stage_b * u;
      pa.lab_dev = W.d_labdev.p + 4 * k + 2 * e;
      pa.sig_dev = W.d_sig.p + ((size_t)(k + 1) * 2 + e) * d;
      uint8_t* ho = W.h_cout.p + out_b * u;
      ((volatile int*)ho)[0] = -1;
      pa.pick = ho + o_pick;
      pa.sig_out = (double*)(ho + o_sig);
      pa.ll = (double*)(ho + o_ll);
      pa.status_host = (int*)ho;
      pa.state_host = (uint32_t*)(ho + o_state);
      pa.state_host[624] = 0;
      if (++phd.gen >= (1 << 26)) {                 // generations only grow: restart from 1
        HIPCHK(hipStreamSynchronize(st));
        HIPCHK(hipMemsetAsync(phd.status.p, 0, 16, st));
        phd.gen = 1;
      }
      pa.gs = pf.gs; pa.G = pf.G; pa.gtab2 = phd.gtab2.p; pa.roots = phd.roots.p; pa.ctr = phd.ctr.p;
      pa.gen = phd.gen;
      pa.tree = nullptr;
      pa.lg = nullptr;
      pa.lzz = nullptr;
      pa.tdbg = nullptr;
      HIPCHK(launch_phi2(pa, st, nullptr));
      phd.fast_calls++;
      c->stats.phi_fast_calls++;
    }
  }
  HIPCHK(hipEventRecord(phd.ev_last, st));
  phd.last_s = st;
  c->phd_release(st);
  // the results down once: the sides, both tables, the chain words, the wide scans' flags
  const int ncw = 1 + 3 * t;
  const size_t o_cw = align16(2 * nt * 4), o_wd = align16(o_cw + (size_t)ncw * sizeof(PhiChain)),
               back_b = o_wd + wstride * t * 4;
  W.h_cback.ensure(back_b + 64);
  HIPCHK(hipMemcpyAsync(W.h_side.p, W.d_side.p, (size_t)nS * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(W.h_cback.p, W.d_F.p, 2 * nt * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(W.h_cback.p + o_cw, W.d_chain.p, (size_t)ncw * sizeof(PhiChain), hipMemcpyDeviceToHost, st));
  if (Gw) HIPCHK(hipMemcpyAsync(W.h_cback.p + o_wd, W.d_wide.p, wstride * t * 4, hipMemcpyDeviceToHost, st));
  if (!W.ev_chain) HIPCHK(hipEventCreateWithFlags(&W.ev_chain, hipEventDisableTiming));
  HIPCHK(hipEventRecord(W.ev_chain, st));
  c->mark("sm.chain_enqueued");
  {
    // (a blocking wait's wake-up costs tens of microseconds: poll, then block after 2 s)
    const auto t0 = std::chrono::steady_clock::now();
    for (int polls = 0;; ++polls) {
      const hipError_t q = hipEventQuery(W.ev_chain);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) HIPCHK(q);
      HostPool::spin_pause();
      if ((polls & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        HIPCHK(hipEventSynchronize(W.ev_chain));
        break;
      }
    }
  }
  c->mark("sm.chain_done");
  const PhiChain* cw = (const PhiChain*)(W.h_cback.p + o_cw);
  const uint32_t* hF = (const uint32_t*)W.h_cback.p;
  auto ustat = [&](int u) { return ((const int*)(W.h_cout.p + out_b * u))[0]; };
  // the first update that did not complete (nu: none)
  int uf = nu;
  for (int u = 0; u < nu; ++u)
    if (ustat(u) != kPhiOk || cw[upd_w(u)].ok != 1) {
      uf = u;
      break;
    }
  const int kf = uf >> 1;                                   // its scan
  const bool scan_kf = uf < nu && cw[link_w(kf)].ok == 1;   // that scan ran
  const int ran = kf + (scan_kf ? 1 : 0);                   // scans run
  if (Gw)
    for (int k = 0; k < ran; ++k) {
      c->stats.sm_wide_scans++;
      if (((const int*)(W.h_cback.p + o_wd))[wstride * k + 1] != 0) c->stats.sm_wide_fallbacks++;
    }
  // the state after the last complete step: sides, tables, sizes
  if (ran > 0) {
    const int* hs = W.h_side.p;
    for (int q = 0; q < nS; ++q) s.c[S[q]] = hs[q] == 0 ? c1 : c2;
    for (int e2 = 0; e2 < 2; ++e2) {
      Freq& F = (e2 == 0) ? F1 : F2;
      const uint32_t* src = hF + (size_t)(e2 == 0 ? a1 : 1 - a1) * nt;
      for (size_t e = 0; e < nt; ++e) F.f[e] = (double)src[e];
      int nn = 0;
      for (int l = 0; l < mm; ++l) nn += (int)src[l];
      F.nn = nn;
    }
    s.counts[c1] = F1.nn;
    s.counts[c2] = F2.nn;
  }
  // the parameters of the updates that completed (each cluster's last)
  for (int u = 0; u < uf; ++u) {
    int64_t cons = 0;
    std::memcpy(&cons, W.h_cout.p + out_b * u + 8, 8);
    Ctx::PhiDevice::adapt(phd.p_rej_sm, cons - 3 * (int64_t)d, d, 0.9);
  }
  for (int e = 0; e < 2; ++e) {
    int u = uf - 1;
    while (u >= 0 && (u & 1) != e) --u;
    if (u < 0) continue;
    const uint8_t* ho = W.h_cout.p + out_b * u;
    const uint8_t* pk = ho + o_pick;
    const int k = klab[e];
    for (int j = 0; j < d; ++j) s.center[(size_t)k * d + j] = (uint8_t)(pk[j] + 1);
    std::memcpy(&s.sigma[(size_t)k * d], ho + o_sig, (size_t)d * 8);
  }
  c->stats.phi_device_calls += uf;
  c->stats.phi_sm_device_calls += uf;
  c->stats.sm_chain_runs++;
  c->stats.sm_chain_scans += ran;
  if (uf == nu) {
    // the host stream after the last update's draws (its state came back with its outputs)
    const uint8_t* ho = W.h_cout.p + out_b * (nu - 1);
    c->adopt_after_phi(*Wn, (uint64_t)cw[upd_w(nu - 1)].end, (const uint32_t*)(ho + o_state));
    *next_iter = t;
    return kOk;
  }
  // continue on the host from the first unfinished step
  c->stats.sm_chain_resumes++;
  const int stk = ustat(uf);
  if (scan_kf && stk != kPhiOff && stk != kPhiOk) {
    c->stats.phi_fallback_status_mask |= (int64_t)1 << std::min(std::max(stk, 0), 14);
    c->stats.phi_fast_handbacks++;
    if (stk == kPhiShort || stk == kPhiWindow) Ctx::PhiDevice::widen(phd.p_rej_sm, 0.9);
  }
  if (std::getenv("HDPM_PHI_TRACE"))
    std::fprintf(stderr, "[sm chain] t %d nS %d: scan %d %s (update status %d)\n", t, nS, kf,
                 !scan_kf ? "off" : (uf & 1) ? "ran, second update handed back" : "ran, update handed back", stk);
  uint64_t pos;
  if (!scan_kf) pos = (uint64_t)cw[kf == 0 ? 0 : upd_w(2 * kf - 1)].end;
  else if ((uf & 1) == 0) pos = (uint64_t)cw[link_w(kf)].end + (uint64_t)nS;
  else pos = (uint64_t)cw[upd_w(uf - 1)].end;
  c->adopt_state_at(*Wn, pos);
  c->rng_sync();
  *next_iter = kf;
  *at_phi = !scan_kf ? 0 : (uf & 1) ? 2 : 1;
  return kOk;
}

// sm:163-225 on host state s with the scan on the device.  F1 / F2: the tables of s.c[i1]
// and s.c[i2] on entry, kept current (points the scan moves change sides).  The members of
// both clusters are S + {i1, i2}, so their sizes come from the tables, neither can empty
// (i1, i2 never move) and validate_state (sm:222) cannot fail.
// members_are_S: the two clusters hold exactly S + {i1, i2} (the split-merge move; the C ABI
// entry point takes any S).  Then the tables come from the device (sm_freq_device): F1 / F2
// empty on entry are counted there (the split launch state), and after every scan F1 is
// recounted from the device sides and F2 = (F1 + F2 on entry) - F1; the sides come down once,
// after the last scan.
static int restricted_gibbs(Ctx* c, const std::vector<int>& S, HState& s, int i1, int i2, int t, Freq& F1,
                            Freq& F2, bool members_are_S) {
  SmWork& W = smwork(c);
  const int c1 = s.c[i1], c2 = s.c[i2];
  const int nS = (int)S.size();
  sm_upload_S(c, W, S);
  std::vector<int> side(nS), to1, to2;   // sides before the current scan
  // pinned staging: draws up, sides down (each iteration ends with a stream wait)
  W.h_side.ensure(std::max(nS, 1));
  W.h_raw.ensure(std::max(nS, 1));
  int* hs = W.h_side.p;
  uint32_t* raw = W.h_raw.p;
  for (int q = 0; q < nS; ++q) side[q] = (s.c[S[q]] == c1) ? 0 : 1;
  const bool dev_tables = members_are_S && c1 != c2 && c->mmax * 16 * 4 <= 64 * 1024;
  if (!dev_tables && F1.f.empty()) {
    std::vector<int> M(S);
    M.push_back(i1);
    M.push_back(i2);
    std::sort(M.begin(), M.end());
    freq_split(c, s, M, c1, F1, F2);
  }
  Freq FM;                                      // the table of S + {i1, i2} (dev_tables)
  if (dev_tables) {
    std::memcpy(hs, side.data(), (size_t)nS * 4);
    if (nS) HIPCHK(hipMemcpyAsync(W.d_side.p, hs, (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
    if (F1.f.empty()) {
      sm_freq_device(c, W, nS, nullptr, 0, i1, i2, FM);
      sm_freq_device(c, W, nS, W.d_side.p, 0, i1, -1, F1);
      freq_minus(FM, F1, F2);
    } else {
      freq_plus(F1, F2, FM);
    }
  }
  // large scans take their |S| draws from the device windows (no host generation and copy;
  // the host stream adopts the state after them); debug bit 16 draws them on the host
  const bool dev_draws = nS >= 4096 && !(c->debug & 65536);
  // the whole sampler as one device chain where it applies (sm_chain); the host continues
  // from the first step the chain did not finish
  int iter0 = 0, at_phi = 0;
  if (dev_tables && sm_chain(c, W, S, s, i1, i2, t, F1, F2, FM, &iter0, &at_phi) == kOk) {
    c->mark("sm.chain");
    if (iter0 == t) return kOk;
  }
  for (int iter = iter0; iter < t; ++iter) {
    if (at_phi && iter == iter0) {
      // the chain's scan ran, its update_phi({c1, c2}) did not (1) or only the lower label's
      // did (2): the rest here
      int st;
      if (at_phi == 2) {
        const int kh = std::max(c1, c2);
        const Freq& Fh = kh == c1 ? F1 : F2;
        st = hupdate_phi_pair(c, s, kh, Fh, kh, Fh);
      } else {
        st = hupdate_phi_pair(c, s, c1, F1, c2, F2);
      }
      c->mark("sm.phi");
      if (st) return st;
      continue;
    }
    const uint32_t* d_raw = nullptr;
    if (dev_draws) {
      c->rng_sync();
      c->mark("sm.sync");
      d_raw = c->device_draws(nS);
    } else {
      c->rng.raw_block(raw, nS);
    }
    c->mark("sm.draws");
    // c1 == c2 (only through the C ABI): every draw picks the same label, so only the
    // draws are consumed
    if (nS && c1 != c2) {
      SmTimer tm(c->stats.t_sm_scan_ms);
      sm_upload_two(c, W, s, c1, c2);
      c->mark("sm.upload");
      // later scans start from the sides the previous scan left on the device
      if (iter == 0 && !dev_tables) {
        std::memcpy(hs, side.data(), (size_t)nS * 4);
        HIPCHK(hipMemcpyAsync(W.d_side.p, hs, (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
      }
      if (!d_raw) HIPCHK(hipMemcpyAsync(W.d_raw.p, raw, (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
      SmArgs a = sm_args(c, W, nS);
      if (d_raw) a.raw = d_raw;
      a.n1 = F1.nn; a.n2 = F2.nn;
      // one launch fewer: the certified bands and the delta table's zeroing in k_sm_ll_lds
      const bool fused = dev_tables && sm_ll_lds_fits(c->d, c->nq);
      if (dev_tables) {
        W.d_side_prev.ensure(std::max(nS, 1));
        W.d_freq.ensure((size_t)c->d * c->mmax);
        a.side_prev = W.d_side_prev.p;
        if (fused) {
          a.cert_in_ll = 1;
          a.zero = W.d_freq.p;
          a.zero_n = c->d * c->mmax;
        }
      }
      HIPCHK(launch_sm_ll(a, c->stream));
      // the walk on many CUs when the move's tables come from the device (k_sm_scan_wide; it
      // gives up, writing nothing, if its grid is not resident -- then k_sm_scan runs)
      const int Gw = (dev_tables && fused && sm_wide_on()) ? sm_scan_wide_grid(nS) : 0;
      if (Gw) {
        W.d_wide.ensure(4 + 2 * (size_t)Gw);
        W.h_wide.ensure(4);
        a.wide_buf = W.d_wide.p;
        a.wide_limit = c->sm_wide_ticks;          // 50 ms of the 100 MHz clock by default
        HIPCHK(launch_sm_scan_wide(a, Gw, c->stream));
        HIPCHK(hipMemcpyAsync(W.h_wide.p, W.d_wide.p, 16, hipMemcpyDeviceToHost, c->stream));
      }
      // (behind the wide scan, k_sm_scan returns at once unless it gave up: then it restores
      // the pre-scan sides and walks -- no host round trip either way)
      HIPCHK(launch_sm_scan(a, c->stream));
      if (dev_tables) {
        sm_freq_device(c, W, nS, W.d_side.p, 0, -1, -1, F1, W.d_side_prev.p, fused);
        if (Gw) {
          c->stats.sm_wide_scans++;
          if (W.h_wide.p[1] != 0) c->stats.sm_wide_fallbacks++;
        }
        freq_minus(FM, F1, F2);
        c->mark("sm.device");
        if (iter + 1 == t) {
          // the state's labels after the last scan
          HIPCHK(hipMemcpyAsync(hs, W.d_side.p, (size_t)nS * 4, hipMemcpyDeviceToHost, c->stream));
          HIPCHK(hipStreamSynchronize(c->stream));
          for (int q = 0; q < nS; ++q) s.c[S[q]] = hs[q] == 0 ? c1 : c2;
        }
        c->mark("sm.sides");
        s.counts[c1] = F1.nn;
        s.counts[c2] = F2.nn;
        const int st = hupdate_phi_pair(c, s, c1, F1, c2, F2);
        c->mark("sm.phi");
        if (st) return st;
        continue;
      }
      HIPCHK(hipMemcpyAsync(hs, W.d_side.p, (size_t)nS * 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      c->mark("sm.device");
      to1.clear();
      to2.clear();
      for (int q = 0; q < nS; ++q) {
        if (hs[q] == side[q]) continue;
        side[q] = hs[q];
        const int i = S[q];
        s.c[i] = side[q] == 0 ? c1 : c2;
        (side[q] == 0 ? to1 : to2).push_back(i);
      }
      c->mark("sm.sides");
      if (members_are_S && 4 * (to1.size() + to2.size()) > (size_t)nS) {
        // many moves (the first scan of a random split): rebuilding c1's table from its
        // rows costs |c1| D, moving them 2 (moves) D
        Freq tot;
        freq_plus(F1, F2, tot);
        std::vector<int> rows1;
        rows1.reserve(F1.nn + to1.size());
        rows1.push_back(i1);
        for (int q = 0; q < nS; ++q)
          if (side[q] == 0) rows1.push_back(S[q]);
        freq_over(c, s, rows1, -1, F1);
        freq_minus(tot, F1, F2);
      } else {
        freq_move(c, F1, F2, to1, to2);
      }
      c->mark("sm.freq");
    }
    s.counts[c1] = F1.nn;
    s.counts[c2] = F2.nn;
    // sm:221 update_phi({c1, c2}): the mask visits clusters in ascending index order, a
    // repeated index once (c1 == c2 only through the restricted-Gibbs C ABI)
    const int st = hupdate_phi_pair(c, s, c1, F1, c2, F2);
    c->mark("sm.phi");
    if (st) return st;
  }
  return kOk;
}

// sm:96-161, gamma_star = gs, gamma = g (launch).  Device terms, compensated sum.
// n1, n2: sizes of g's clusters c(i1), c(i2).
static double logprobgs_c_i(Ctx* c, const HState& gs, const HState& g, const std::vector<int>& S, int i1,
                            int i2, int n1, int n2) {
  SmWork& W = smwork(c);
  const int c1 = g.c[i1], c2 = g.c[i2];
  const int nS = (int)S.size();
  if (nS == 0) return 0.0;
  sm_upload_S(c, W, S);
  std::vector<int> side(nS), sref(nS);
  for (int q = 0; q < nS; ++q) {
    side[q] = gs.c[S[q]] == c1 ? 0 : 1;
    sref[q] = g.c[S[q]] == c1 ? 0 : (g.c[S[q]] == c2 ? 1 : 2);
  }
  sm_upload_two(c, W, gs, c1, c2);
  HIPCHK(hipMemcpyAsync(W.d_side.p, side.data(), (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(W.d_side_ref.p, sref.data(), (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
  SmArgs a = sm_args(c, W, nS);
  a.n1 = n1; a.n2 = n2;
  HIPCHK(launch_sm_ll(a, c->stream));
  HIPCHK(launch_sm_lpgs(a, c->stream));
  const int nb = (nS + kBlock - 1) / kBlock;
  W.h_out.resize(2 * nb);
  HIPCHK(hipMemcpyAsync(W.h_out.data(), W.d_out.p, W.h_out.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  double hi = 0.0, lo = 0.0;
  for (int b = 0; b < nb; ++b) {
    const double x = W.h_out[2 * b];
    const double s = hi + x, bb = s - hi;
    lo += (hi - (s - bb)) + (x - bb) + W.h_out[2 * b + 1];
    hi = s;
  }
  return hi + lo;
}

// sm:6-18
static double logdensity_hig_k(double K, double sigmaj, double vv, double ww, double m) {
  return K - (vv + ww) * std::log(1 + std::exp(-1 / sigmaj) * (m - 1)) - (ww + 1) / sigmaj - 2 * std::log(sigmaj);
}
static double logdensity_hig(double sigmaj, double vv, double ww, double m, int* err, bool logspace) {
  double K = norm_const2(ww, vv, m, err, logspace);
  return logdensity_hig_k(K, sigmaj, vv, ww, m);
}

// sm:20-94
// Per-attribute terms on the host pool for wide rows; the sums keep attribute order.
template <class F>
static void per_attribute(const Ctx* c, F f) {
  if (c->d >= 128) pool_for(c->d, f, 16);
  else for (int j = 0; j < c->d; ++j) f(j);
}

// F: the table of gs's cluster c(idx).
static double logprobgs_phi(Ctx* c, const HState& gs, const HState& g, int idx, const Freq& F, int* err) {
  const int k = gs.c[idx];
  const std::vector<double>& f = F.f;
  const int nm = F.nn;
  const double* gsig = &g.sigma[(size_t)g.c[idx] * c->d];
  const uint8_t* cstar = &gs.center[(size_t)k * c->d];
  const double* gss = &gs.sigma[(size_t)k * c->d];
  std::vector<double> lc(c->d), ls(c->d);
  std::vector<int> er(c->d, 0);
  per_attribute(c, [&](int j) {
    const int mj = c->att[j];
    double z[256];
    for (int l = 0; l < mj; ++l) z[l] = (-((double)nm - f[(size_t)j * c->mmax + l])) / gsig[j];
    double mx = z[0];
    for (int l = 1; l < mj; ++l) if (z[l] > mx) mx = z[l];
    for (int l = 0; l < mj; ++l) z[l] = std::exp(z[l] - mx);
    double sum = 0.0;
    for (int l = 0; l < mj; ++l) sum += z[l];
    for (int l = 0; l < mj; ++l) z[l] = z[l] / sum;
    lc[j] = std::log(z[cstar[j] - 1]);
    const double sumdelta = f[(size_t)j * c->mmax + (cstar[j] - 1)];
    const double new_v = c->v[j] + sumdelta;
    const double new_w = c->w[j] + nm - sumdelta;
    int e = 0;
    ls[j] = logdensity_hig(gss[j], new_v, new_w, c->att[j], &e, c->hig_log);
    er[j] = e;
  });
  double log_center_prob = 0, log_sigma_prob = 0;
  for (int j = 0; j < c->d; ++j) log_center_prob += lc[j];
  for (int j = 0; j < c->d; ++j) {
    log_sigma_prob += ls[j];
    if (er[j]) *err = er[j];
  }
  return log_center_prob + log_sigma_prob;
}

// sm:393-417 from the cluster's table: per attribute f matches and nn - f mismatches of its
// two dhamming values, summed with a compensated (Neumaier) sum.  The reference adds the N_k D
// terms one by one; this regrouping agrees with it to its own rounding (~1e-13 relative at
// 10^6 terms) and only enters the acceptance test log(u) < ratio (sm:591).
static double loglikelihood_hamming(Ctx* c, const HState& s, int k, const Freq& F) {
  std::vector<double> tab;
  row_tables(c, &s.center[(size_t)k * c->d], &s.sigma[(size_t)k * c->d], tab);
  const uint8_t* cen = &s.center[(size_t)k * c->d];
  double hi = 0.0, lo = 0.0;
  auto add = [&](double x) {
    const double t = hi + x;
    lo += std::fabs(hi) >= std::fabs(x) ? (hi - t) + x : (x - t) + hi;
    hi = t;
  };
  for (int j = 0; j < c->d; ++j) {
    const double fm = F.f[(size_t)j * c->mmax + (cen[j] - 1)];
    add(fm * tab[2 * j]);
    add(((double)F.nn - fm) * tab[2 * j + 1]);
  }
  return hi + lo;
}

// sm:419-436.  Its normalising constants norm_const2(w_j, v_j, m_j) depend on the
// hyperparameters and attribute sizes only: computed once (SmWork::prior_nc) and reused by
// every move.
static double priors(Ctx* c, const HState& s, int k, int* err) {
  SmWork& W = smwork(c);
  const int d = c->d;
  // keyed on every input of norm_const2: v, w, the attribute sizes m_j and the 2F1 mode (a
  // second set_data with the same v / w but other m_j must not reuse the constants)
  if (W.prior_log != (int)c->hig_log || W.prior_v != c->v || W.prior_w != c->w || W.prior_att != c->att ||
      (int)W.prior_nc.size() != d) {
    W.prior_nc.assign(d, 0.0);
    W.prior_err.assign(d, 0);
    per_attribute(c, [&](int j) {
      int e = 0;
      W.prior_nc[j] = norm_const2(c->w[j], c->v[j], c->att[j], &e, c->hig_log);
      W.prior_err[j] = e;
    });
    W.prior_v = c->v;
    W.prior_w = c->w;
    W.prior_att = c->att;
    W.prior_log = (int)c->hig_log;
  }
  const double* sig = &s.sigma[(size_t)k * d];
  std::vector<double> ld(d);
  per_attribute(c, [&](int j) { ld[j] = logdensity_hig_k(W.prior_nc[j], sig[j], c->v[j], c->w[j], c->att[j]); });
  double priorg = 0;
  for (int j = 0; j < d; ++j) {
    priorg -= std::log((double)c->att[j]);
    priorg += ld[j];
    if (W.prior_err[j]) *err = W.prior_err[j];
  }
  return priorg;
}

static double min0(double x) { return (x < 0.0) ? x : 0.0; }

// validate_state (cf:146-172) on a state whose counts are exact (labels in [0, K), counts[k]
// its members): the distinct labels are then the non-empty clusters -- O(K) instead of two
// passes over N.  Every state of the move keeps its counts exact (recount_delta, the
// restricted scans' table sizes, clean_var).
static int hvalidate_counted(const HState& s) {
  int u = 0;
  for (int k = 0; k < s.K; ++k) u += s.counts[k] > 0;
  return u == s.K ? kOk : kValidate;
}

// Counts of `to` from the exact counts of `from`, the two states differing only at the points
// of M (the move's members): O(|M|) instead of a pass over N.
static void recount_delta(const HState& from, HState& to, const std::vector<int>& M) {
  to.counts = from.counts;
  to.counts.resize(to.K, 0);
  for (int q : M) {
    to.counts[from.c[q]]--;
    to.counts[to.c[q]]++;
  }
}

// cf:296-353 clean_var(updated, current, unique(current.c_i)) for a `cur` with exact counts
// (labels in [0, cur.K)): unique(c_i) is its non-empty clusters in ascending order, and the
// labels are rewritten only when the reference's map moves one (a cluster at or above the new
// K); otherwise `upd` takes them as they are.  `upd` may be `cur` (every read of cur precedes
// the write that could change it).
static int clean_var(Ctx* c, HState& upd, const HState& cur) {
  std::vector<int> existing;
  for (int l = 0; l < cur.K; ++l)
    if (cur.counts[l] > 0) existing.push_back(l);
  const int maxl = existing.empty() ? 0 : existing.back();
  const int num = (int)existing.size();
  std::vector<int> map(maxl + 1, -1);
  for (int i = 0; i < num; ++i) {
    int idx_temp = 0;
    if (existing[i] < num) map[existing[i]] = existing[i];
    else {
      while (idx_temp <= maxl && map[idx_temp] != -1 && idx_temp < num) idx_temp++;
      map[existing[i]] = idx_temp;
    }
  }
  std::vector<uint8_t> nc((size_t)num * c->d, 0);
  std::vector<double> ns((size_t)num * c->d, 0.0);
  std::vector<int32_t> cnt(num, 0);
  bool ident = true;
  for (int i = 0; i < num; ++i) {
    const int dst = map[existing[i]];
    ident = ident && dst == existing[i];
    std::memcpy(&nc[(size_t)dst * c->d], &cur.center[(size_t)existing[i] * c->d], c->d);
    std::memcpy(&ns[(size_t)dst * c->d], &cur.sigma[(size_t)existing[i] * c->d], (size_t)c->d * 8);
    cnt[dst] = cur.counts[existing[i]];
  }
  if (!ident) {
    upd.c.resize(cur.c.size());
    for (size_t i = 0; i < cur.c.size(); ++i) upd.c[i] = map[cur.c[i]];   // every label exists
  } else if (&upd != &cur) {
    upd.c = cur.c;
  }
  upd.center = std::move(nc);
  upd.sigma = std::move(ns);
  upd.counts = std::move(cnt);
  upd.K = num;
  return hvalidate_counted(upd);
}

static void push_cluster(Ctx* c, HState& s) {
  s.center.resize((size_t)(s.K + 1) * c->d);
  s.sigma.resize((size_t)(s.K + 1) * c->d);
}

// sm:542-598
int Ctx::split_and_merge(int t, int r, int idx_1_sm, int* accepted) {
  rng_sync();
  if (!have_state) { err = "no state"; return kArg; }
  (void)idx_1_sm;  // overwritten by select_observations_random (sm:278), as in the reference
  *accepted = 0;
  HState st;
  ctx_to_hstate(this, st);
  // every host index below is a label < K (the state's arrays are K x d): refuse a state
  // that breaks this rather than write outside them
  for (int x : st.c)
    if (x < 0 || x >= st.K) { err = "State validation failed: label outside 0..K-1"; return kValidate; }
  if (n < 2) { err = "split_and_merge needs at least two observations"; return kArg; }
  if ((int)st.counts.size() != st.K) hrecount(this, st);   // (the move keeps counts exact from here)
  // sm:263-301 select_observations_random: sample(0..n-1, 2, FALSE)
  int i1, i2;
  {
    int nn = n;
    const int j = (int)(nn * rng.unif());
    i1 = j;
    --nn;
    const int j2 = (int)(nn * rng.unif());
    i2 = (j2 == j) ? n - 1 : j2;
  }
  std::vector<int> S, M;               // M: S + {i1, i2}, ascending
  for (int i = 0; i < n; ++i) {
    if (st.c[i] != st.c[i1] && st.c[i] != st.c[i2]) continue;
    M.push_back(i);
    if (i != i1 && i != i2) S.push_back(i);
  }
  Freq FM;                             // every cluster below that holds i1 or i2 is within M
  int e;
  // sm:303-352 split_launch_state
  HState sl = st;
  if (st.c[i1] == st.c[i2]) {
    sl.c[i1] = st.K;
    push_cluster(this, sl);
    sample_center_uniform(&sl.center[(size_t)sl.K * d]);
    e = sample_sigma_wide(v.data(), w.data(),&sl.sigma[(size_t)sl.K * d]);
    if (e) { err = "rhig failed"; return e; }
    sl.K++;
  } else {
    sample_center_uniform(&sl.center[(size_t)st.c[i1] * d]);
    e = sample_sigma_wide(v.data(), w.data(),&sl.sigma[(size_t)st.c[i1] * d]);
    if (e) { err = "rhig failed"; return e; }
  }
  sample_center_uniform(&sl.center[(size_t)st.c[i2] * d]);
  e = sample_sigma_wide(v.data(), w.data(),&sl.sigma[(size_t)st.c[i2] * d]);
  if (e) { err = "rhig failed"; return e; }
  {
    const int ref[2] = {sl.c[i1], sl.c[i2]};
    for (int q : S) sl.c[q] = ref[(int)(2 * rng.unif())];
  }
  recount_delta(st, sl, M);
  Freq F1, F2;                         // tables of sl.c[i1], sl.c[i2] (they split M)
  // (counted by restricted_gibbs: on the device from the launch sides)
  e = restricted_gibbs(this, S, sl, i1, i2, t, F1, F2, true);
  freq_plus(F1, F2, FM);
  mark("sm.split_state");
  if (e) { err = "split launch state failed"; return e; }
  e = hvalidate_counted(sl);
  if (e) { err = "State validation failed: split_launch_state"; return e; }
  const int n1_sl = F1.nn, n2_sl = F2.nn;
  // sm:354-391 merge_launch_state
  HState ml = st;
  if (ml.c[i1] != ml.c[i2]) {
    ml.c[i1] = ml.c[i2];
    for (int q : S) ml.c[q] = ml.c[i2];
    recount_delta(st, ml, M);
  }
  sample_center_uniform(&ml.center[(size_t)ml.c[i2] * d]);
  e = sample_sigma_wide(v.data(), w.data(),&ml.sigma[(size_t)ml.c[i2] * d]);
  if (e) { err = "rhig failed"; return e; }
  e = clean_var(this, ml, ml);
  if (e) { err = "State validation failed: clean_var"; return e; }
  for (int iter = 0; iter < r; ++iter) {
    e = hupdate_phi_pair(this, ml, ml.c[i2], FM, ml.c[i2], FM);
    if (e) { err = "update_phi failed"; return e; }
  }
  e = hvalidate_counted(ml);
  if (e) { err = "State validation failed: merge_launch_state"; return e; }
  mark("sm.merge_state");
  // proposal
  HState ss;
  double acpt;
  int gerr = kOk;
  const double alpha = gamma;
  if (st.c[i1] == st.c[i2]) {
    ss = sl;
    e = restricted_gibbs(this, S, ss, i1, i2, 1, F1, F2, true);    // F1, F2 now ss's tables
    if (e) { err = "restricted gibbs failed"; return e; }
    // sm:438-487 (st.c[i1]'s members are all of M)
    SmTimer tm(stats.t_sm_terms_ms);
    mark("sm.t0");
    double log_prior = 0.0, log_likelihood = 0.0, log_proposal = 0.0;
    log_prior += std::log(alpha);
    log_prior += std::lgamma((double)F1.nn);
    log_prior += std::lgamma((double)F2.nn);
    log_prior += priors(this, ss, ss.c[i1], &gerr);
    log_prior += priors(this, ss, ss.c[i2], &gerr);
    log_prior -= std::lgamma((double)FM.nn);
    log_prior -= priors(this, st, st.c[i1], &gerr);
    mark("sm.t.priors");
    log_likelihood += loglikelihood_hamming(this, ss, ss.c[i1], F1);
    log_likelihood += loglikelihood_hamming(this, ss, ss.c[i2], F2);
    log_likelihood -= loglikelihood_hamming(this, st, st.c[i1], FM);
    mark("sm.t.ll");
    log_proposal += logprobgs_phi(this, st, ml, i1, FM, &gerr);
    log_proposal -= logprobgs_phi(this, ss, sl, i1, F1, &gerr);
    log_proposal -= logprobgs_phi(this, ss, sl, i2, F2, &gerr);
    mark("sm.t.lpphi");
    log_proposal -= logprobgs_c_i(this, ss, sl, S, i1, i2, n1_sl, n2_sl);
    mark("sm.t.lpci");
    acpt = min0(log_prior + log_likelihood + log_proposal);
  } else {
    ss = ml;
    e = hupdate_phi_pair(this, ss, ss.c[i2], FM, ss.c[i2], FM);
    if (e) { err = "update_phi failed"; return e; }
    // sm:489-540 (ss's merged cluster is M; st's two clusters split M)
    SmTimer tm(stats.t_sm_terms_ms);
    mark("sm.t0");
    Freq S1, S2;
    if (!S.empty() && mmax * 16 * 4 <= 64 * 1024) {
      // st's c(i1) within M counted on the device from st's sides of S (a host pass over
      // |M| D codes took ~0.6 ms at C4)
      SmWork& W = smwork(this);
      const int nS = (int)S.size();
      sm_upload_S(this, W, S);
      W.h_side.ensure(nS);
      W.d_side_prev.ensure(nS);
      for (int q = 0; q < nS; ++q) W.h_side.p[q] = st.c[S[q]] == st.c[i1] ? 0 : 1;
      HIPCHK(hipMemcpyAsync(W.d_side_prev.p, W.h_side.p, (size_t)nS * 4, hipMemcpyHostToDevice, stream));
      sm_freq_device(this, W, nS, W.d_side_prev.p, 0, i1, st.c[i2] == st.c[i1] ? i2 : -1, S1);
    } else {
      freq_over(this, st, M, st.c[i1], S1);
    }
    freq_minus(FM, S1, S2);
    mark("sm.t.freq");
    double log_prior = 0.0, log_likelihood = 0.0, log_proposal = 0.0;
    log_prior += std::lgamma((double)FM.nn);
    log_prior += priors(this, ss, ss.c[i1], &gerr);
    log_prior -= std::log(alpha);
    log_prior -= std::lgamma((double)S1.nn);
    log_prior -= std::lgamma((double)S2.nn);
    log_prior -= priors(this, st, st.c[i1], &gerr);
    log_prior -= priors(this, st, st.c[i2], &gerr);
    mark("sm.t.priors");
    log_likelihood += loglikelihood_hamming(this, ss, ss.c[i2], FM);
    log_likelihood -= loglikelihood_hamming(this, st, st.c[i1], S1);
    log_likelihood -= loglikelihood_hamming(this, st, st.c[i2], S2);
    mark("sm.t.ll");
    log_proposal += logprobgs_phi(this, st, sl, i1, S1, &gerr);
    log_proposal += logprobgs_phi(this, st, sl, i2, S2, &gerr);
    log_proposal += logprobgs_c_i(this, st, sl, S, i1, i2, n1_sl, n2_sl);
    log_proposal -= logprobgs_phi(this, ss, ml, i2, FM, &gerr);
    mark("sm.t.lp");
    acpt = min0(log_prior + log_likelihood + log_proposal);
  }
  if (gerr) { err = "norm_const2 - hypergeometric diverging with infinity"; return gerr; }
  e = hvalidate_counted(ss);
  if (e) { err = "State validation failed: split_and_merge - state_star"; return e; }
  if (std::log(rng.unif()) < acpt) {   // sm:591
    HState ns = st;
    e = clean_var(this, ns, ss);
    if (e) { err = "State validation failed: clean_var"; return e; }
    hstate_to_ctx(this, ns);
    *accepted = 1;
  }
  return kOk;
}

// C-ABI helpers operating on the context state.
int sm_restricted_gibbs_device(Ctx* c, const int32_t* S, int32_t nS, int32_t i1, int32_t i2, int32_t t) {
  c->rng_sync();
  if (!c->have_state) { c->err = "no state"; return kArg; }
  HState s;
  ctx_to_hstate(c, s);
  std::vector<int> SS(S, S + nS), all(c->n);
  for (int i = 0; i < c->n; ++i) all[i] = i;
  Freq F1, F2;                         // the clusters may hold points outside S here
  freq_over(c, s, all, s.c[i1], F1);
  freq_over(c, s, all, s.c[i2], F2);
  int st = restricted_gibbs(c, SS, s, i1, i2, t, F1, F2, false);
  if (st) { c->err = "restricted gibbs failed"; return st; }
  st = hvalidate(s);
  if (st) { c->err = "State validation failed: restricted gibbs"; return st; }
  hstate_to_ctx(c, s);
  return kOk;
}

int sm_logprobgs_c_i_api(Ctx* c, const int32_t* g_c_i, const int32_t* S, int32_t nS, int32_t i1, int32_t i2,
                         double* out) {
  if (!c->have_state) { c->err = "no state"; return kArg; }
  HState gs, g;
  ctx_to_hstate(c, gs);
  g = gs;
  g.c.assign(g_c_i, g_c_i + c->n);
  std::vector<int> SS(S, S + nS);
  int n1 = 0, n2 = 0;
  for (int i = 0; i < c->n; ++i) { n1 += (g.c[i] == g.c[i1]); n2 += (g.c[i] == g.c[i2]); }
  *out = logprobgs_c_i(c, gs, g, SS, i1, i2, n1, n2);
  return kOk;
}

}  // namespace hdpm
