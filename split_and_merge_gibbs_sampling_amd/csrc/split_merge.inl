// split_merge.inl -- split-merge move (code/split_merge.cpp) on the hdpm runtime.
// Included by engine.cpp.  The orchestration (launch states, acceptance ratio, clean_var)
// runs on the host with the reference's draw order; the restricted Gibbs scan
// (sm:163-225) and the logprobgs_c_i sum (sm:96-161) run on the device.
#pragma once

namespace hdpm {

hipError_t launch_sm_ll(const SmArgs& a, hipStream_t s);
hipError_t launch_sm_scan(const SmArgs& a, double T, hipStream_t s);
hipError_t launch_sm_lpgs(const SmArgs& a, hipStream_t s);

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

// freq of one cluster over its members (host): f[j][l]
static void host_freq(const Ctx* c, const HState& s, int k, std::vector<double>& f, int& nn) {
  f.assign((size_t)c->d * c->mmax, 0.0);
  nn = 0;
  for (int i = 0; i < c->n; ++i) {
    if (s.c[i] != k) continue;
    nn++;
    const uint8_t* x = &c->codes[(size_t)i * c->d];
    for (int j = 0; j < c->d; ++j) f[(size_t)j * c->mmax + (x[j] - 1)] += 1.0;
  }
}

// update_phi (cf:511-591) on a host state for the clusters in idx (ascending order).
static int hupdate_phi(Ctx* c, HState& s, std::vector<int> idx) {
  std::vector<char> mask(s.K, 0);
  for (int k : idx)
    if (k >= 0 && k < s.K) mask[k] = 1;
  std::vector<double> f, prob(c->mmax), nv(c->d), nw(c->d);
  for (int i = 0; i < s.K; ++i) {
    if (!mask[i]) continue;
    int nn;
    host_freq(c, s, i, f, nn);
    if (nn == 0) continue;
    uint8_t* cen = &s.center[(size_t)i * c->d];
    double* sig = &s.sigma[(size_t)i * c->d];
    for (int j = 0; j < c->d; ++j) {
      const int mj = c->att[j];
      for (int l = 0; l < mj; ++l) prob[l] = (-((double)nn - f[(size_t)j * c->mmax + l])) / sig[j];
      double mx = prob[0];
      for (int l = 1; l < mj; ++l) if (prob[l] > mx) mx = prob[l];
      for (int l = 0; l < mj; ++l) prob[l] = std::exp(prob[l] - mx);
      double sum = 0.0;
      for (int l = 0; l < mj; ++l) sum += prob[l];
      for (int l = 0; l < mj; ++l) prob[l] = prob[l] / sum;
      int pick = sample_prob1(c->rng, prob.data(), mj, c->sp, c->sperm);
      if (pick < 0) return -pick;
      cen[j] = (uint8_t)(pick + 1);
    }
    for (int j = 0; j < c->d; ++j) {
      const double sumdelta = f[(size_t)j * c->mmax + (cen[j] - 1)];
      nw[j] = c->w[j] + nn - sumdelta;
      nv[j] = c->v[j] + sumdelta;
    }
    int st = c->sample_sigma(nv.data(), nw.data(), sig);
    if (st) return st;
  }
  return kOk;
}

static void hrecount(const Ctx* c, HState& s) {
  s.counts.assign(s.K, 0);
  for (int i = 0; i < c->n; ++i)
    if (s.c[i] >= 0 && s.c[i] < s.K) s.counts[s.c[i]]++;
}

// Device: exact lls of the S points against clusters (k1, k2) of state s.
static void sm_upload_two(Ctx* c, SmWork& W, const HState& s, int k1, int k2) {
  std::vector<uint8_t> cc(2 * (size_t)c->dp, 0);
  std::vector<double> tt(4 * (size_t)c->d);
  c->tables_for(&s.center[(size_t)k1 * c->d], &s.sigma[(size_t)k1 * c->d], cc.data(), tt.data());
  c->tables_for(&s.center[(size_t)k2 * c->d], &s.sigma[(size_t)k2 * c->d], cc.data() + c->dp, tt.data() + 2 * c->d);
  W.d_two_codes.ensure(cc.size());
  W.d_two_tab.ensure(tt.size());
  HIPCHK(hipMemcpyAsync(W.d_two_codes.p, cc.data(), cc.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(W.d_two_tab.p, tt.data(), tt.size() * 8, hipMemcpyHostToDevice, c->stream));
}

static SmArgs sm_args(Ctx* c, SmWork& W, int nS) {
  SmArgs a;
  a.codes_t = c->d_codes_t.p; a.n = c->n; a.d = c->d; a.nq = c->nq;
  a.S = W.d_S.p; a.nS = nS;
  a.two = ParamTables{W.d_two_codes.p, W.d_two_tab.p};
  a.ll = W.d_ll.p; a.side = W.d_side.p; a.side_ref = W.d_side_ref.p; a.raw = W.d_raw.p;
  a.logn = c->d_logn.p; a.n1 = 0; a.n2 = 0; a.out_counts = W.d_counts2.p; a.out = W.d_out.p;
  return a;
}

static void sm_upload_S(Ctx* c, SmWork& W, const std::vector<int>& S) {
  const size_t nS = S.size();
  W.d_S.ensure(std::max<size_t>(nS, 1));
  W.d_side.ensure(std::max<size_t>(nS, 1));
  W.d_side_ref.ensure(std::max<size_t>(nS, 1));
  W.d_ll.ensure(std::max<size_t>(2 * nS, 2));
  W.d_raw.ensure(std::max<size_t>(nS, 1));
  W.d_counts2.ensure(2);
  W.d_out.ensure(std::max<size_t>(2 * ((nS + kBlock - 1) / kBlock), 2));
  if (nS) HIPCHK(hipMemcpyAsync(W.d_S.p, S.data(), nS * 4, hipMemcpyHostToDevice, c->stream));
}

// sm:163-225 on host state s with the scan on the device.
static int restricted_gibbs(Ctx* c, const std::vector<int>& S, HState& s, int i1, int i2, int t) {
  SmWork& W = smwork(c);
  const int c1 = s.c[i1], c2 = s.c[i2];
  const int nS = (int)S.size();
  sm_upload_S(c, W, S);
  std::vector<int> side(nS);
  std::vector<uint32_t> raw(nS);
  const double T = 54.0 * M_LN2 + std::log(2.0) + 0.5;
  for (int iter = 0; iter < t; ++iter) {
    int n1 = 0, n2 = 0;
    for (int i = 0; i < c->n; ++i) { n1 += (s.c[i] == c1); n2 += (s.c[i] == c2); }
    for (int q = 0; q < nS; ++q) side[q] = (s.c[S[q]] == c1) ? 0 : 1;
    c->rng.raw_block(raw.data(), nS);
    if (nS) {
      sm_upload_two(c, W, s, c1, c2);
      HIPCHK(hipMemcpyAsync(W.d_side.p, side.data(), (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipMemcpyAsync(W.d_raw.p, raw.data(), (size_t)nS * 4, hipMemcpyHostToDevice, c->stream));
      SmArgs a = sm_args(c, W, nS);
      a.n1 = n1; a.n2 = n2;
      HIPCHK(launch_sm_ll(a, c->stream));
      HIPCHK(launch_sm_scan(a, T, c->stream));
      HIPCHK(hipMemcpyAsync(side.data(), W.d_side.p, (size_t)nS * 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      for (int q = 0; q < nS; ++q) s.c[S[q]] = side[q] == 0 ? c1 : c2;
    }
    hrecount(c, s);
    int st = hupdate_phi(c, s, {c1, c2});   // sm:221 (mask -> ascending order)
    if (st) return st;
    st = hvalidate(s);
    if (st) return st;
  }
  return kOk;
}

// sm:96-161, gamma_star = gs, gamma = g (launch).  Device terms, compensated sum.
static double logprobgs_c_i(Ctx* c, const HState& gs, const HState& g, const std::vector<int>& S, int i1,
                            int i2) {
  SmWork& W = smwork(c);
  const int c1 = g.c[i1], c2 = g.c[i2];
  const int nS = (int)S.size();
  if (nS == 0) return 0.0;
  int n1 = 0, n2 = 0;
  for (int i = 0; i < c->n; ++i) { n1 += (g.c[i] == c1); n2 += (g.c[i] == c2); }
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
static double logdensity_hig(double sigmaj, double vv, double ww, double m, int* err, bool logspace) {
  double K = norm_const2(ww, vv, m, err, logspace);
  return K - (vv + ww) * std::log(1 + std::exp(-1 / sigmaj) * (m - 1)) - (ww + 1) / sigmaj - 2 * std::log(sigmaj);
}

// sm:20-94
static double logprobgs_phi(Ctx* c, const HState& gs, const HState& g, int idx, int* err) {
  const int k = gs.c[idx];
  std::vector<double> f;
  int nm;
  host_freq(c, gs, k, f, nm);
  const double* gsig = &g.sigma[(size_t)g.c[idx] * c->d];
  const uint8_t* cstar = &gs.center[(size_t)k * c->d];
  double log_center_prob = 0;
  std::vector<double> z(c->mmax);
  for (int j = 0; j < c->d; ++j) {
    const int mj = c->att[j];
    for (int l = 0; l < mj; ++l) z[l] = (-((double)nm - f[(size_t)j * c->mmax + l])) / gsig[j];
    double mx = z[0];
    for (int l = 1; l < mj; ++l) if (z[l] > mx) mx = z[l];
    for (int l = 0; l < mj; ++l) z[l] = std::exp(z[l] - mx);
    double sum = 0.0;
    for (int l = 0; l < mj; ++l) sum += z[l];
    for (int l = 0; l < mj; ++l) z[l] = z[l] / sum;
    log_center_prob += std::log(z[cstar[j] - 1]);
  }
  double log_sigma_prob = 0;
  const double* gss = &gs.sigma[(size_t)k * c->d];
  for (int j = 0; j < c->d; ++j) {
    const double sumdelta = f[(size_t)j * c->mmax + (cstar[j] - 1)];
    const double new_v = c->v[j] + sumdelta;
    const double new_w = c->w[j] + nm - sumdelta;
    log_sigma_prob += logdensity_hig(gss[j], new_v, new_w, c->att[j], err, c->hig_log);
  }
  return log_center_prob + log_sigma_prob;
}

// sm:393-417 (one running sum over members then attributes)
static double loglikelihood_hamming(Ctx* c, const HState& s, int k) {
  std::vector<double> tab;
  row_tables(c, &s.center[(size_t)k * c->d], &s.sigma[(size_t)k * c->d], tab);
  const uint8_t* cen = &s.center[(size_t)k * c->d];
  double ll = 0.0;
  for (int i = 0; i < c->n; ++i) {
    if (s.c[i] != k) continue;
    const uint8_t* x = &c->codes[(size_t)i * c->d];
    for (int j = 0; j < c->d; ++j) ll += tab[2 * j + (x[j] != cen[j] ? 1 : 0)];
  }
  return ll;
}

// sm:419-436
static double priors(Ctx* c, const HState& s, int k, int* err) {
  const double* sig = &s.sigma[(size_t)k * c->d];
  double priorg = 0;
  for (int j = 0; j < c->d; ++j) {
    priorg -= std::log((double)c->att[j]);
    priorg += logdensity_hig(sig[j], c->v[j], c->w[j], c->att[j], err, c->hig_log);
  }
  return priorg;
}

static int csize(const HState& s, int k) {
  int x = 0;
  for (int v : s.c) x += (v == k);
  return x;
}

static double min0(double x) { return (x < 0.0) ? x : 0.0; }

// cf:296-353 clean_var(updated, current (by value), unique(current.c_i))
static int clean_var(Ctx* c, HState& upd, const HState cur) {
  int maxl = 0;
  for (int x : cur.c) maxl = std::max(maxl, x);
  std::vector<char> seen(maxl + 1, 0);
  for (int x : cur.c) seen[x] = 1;
  std::vector<int> existing;
  for (int l = 0; l <= maxl; ++l) if (seen[l]) existing.push_back(l);
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
  for (int i = 0; i < num; ++i) {
    const int dst = map[existing[i]];
    std::memcpy(&nc[(size_t)dst * c->d], &cur.center[(size_t)existing[i] * c->d], c->d);
    std::memcpy(&ns[(size_t)dst * c->d], &cur.sigma[(size_t)existing[i] * c->d], (size_t)c->d * 8);
  }
  upd.center = nc;
  upd.sigma = ns;
  upd.K = num;
  upd.c.resize(cur.c.size());
  for (size_t i = 0; i < cur.c.size(); ++i) {
    const int l = cur.c[i];
    if (l >= 0 && l <= maxl && map[l] != -1) upd.c[i] = map[l];
  }
  hrecount(c, upd);
  return hvalidate(upd);
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
  std::vector<int> S;
  for (int i = 0; i < n; ++i) {
    if (i == i1 || i == i2) continue;
    if (st.c[i] == st.c[i1] || st.c[i] == st.c[i2]) S.push_back(i);
  }
  int e;
  // sm:303-352 split_launch_state
  HState sl = st;
  if (st.c[i1] == st.c[i2]) {
    sl.c[i1] = st.K;
    push_cluster(this, sl);
    sample_center_uniform(&sl.center[(size_t)sl.K * d]);
    e = sample_sigma(v.data(), w.data(), &sl.sigma[(size_t)sl.K * d]);
    if (e) { err = "rhig failed"; return e; }
    sl.K++;
  } else {
    sample_center_uniform(&sl.center[(size_t)st.c[i1] * d]);
    e = sample_sigma(v.data(), w.data(), &sl.sigma[(size_t)st.c[i1] * d]);
    if (e) { err = "rhig failed"; return e; }
  }
  sample_center_uniform(&sl.center[(size_t)st.c[i2] * d]);
  e = sample_sigma(v.data(), w.data(), &sl.sigma[(size_t)st.c[i2] * d]);
  if (e) { err = "rhig failed"; return e; }
  {
    const int ref[2] = {sl.c[i1], sl.c[i2]};
    for (int q : S) sl.c[q] = ref[(int)(2 * rng.unif())];
  }
  hrecount(this, sl);
  e = restricted_gibbs(this, S, sl, i1, i2, t);
  if (e) { err = "split launch state failed"; return e; }
  e = hvalidate(sl);
  if (e) { err = "State validation failed: split_launch_state"; return e; }
  // sm:354-391 merge_launch_state
  HState ml = st;
  if (ml.c[i1] != ml.c[i2]) {
    ml.c[i1] = ml.c[i2];
    for (int q : S) ml.c[q] = ml.c[i2];
  }
  sample_center_uniform(&ml.center[(size_t)ml.c[i2] * d]);
  e = sample_sigma(v.data(), w.data(), &ml.sigma[(size_t)ml.c[i2] * d]);
  if (e) { err = "rhig failed"; return e; }
  e = clean_var(this, ml, ml);
  if (e) { err = "State validation failed: clean_var"; return e; }
  for (int iter = 0; iter < r; ++iter) {
    e = hupdate_phi(this, ml, {ml.c[i2]});
    if (e) { err = "update_phi failed"; return e; }
  }
  e = hvalidate(ml);
  if (e) { err = "State validation failed: merge_launch_state"; return e; }
  // proposal
  HState ss;
  double acpt;
  int gerr = kOk;
  const double alpha = gamma;
  if (st.c[i1] == st.c[i2]) {
    ss = sl;
    e = restricted_gibbs(this, S, ss, i1, i2, 1);
    if (e) { err = "restricted gibbs failed"; return e; }
    // sm:438-487
    double log_prior = 0.0, log_likelihood = 0.0, log_proposal = 0.0;
    log_prior += std::log(alpha);
    log_prior += std::lgamma((double)csize(ss, ss.c[i1]));
    log_prior += std::lgamma((double)csize(ss, ss.c[i2]));
    log_prior += priors(this, ss, ss.c[i1], &gerr);
    log_prior += priors(this, ss, ss.c[i2], &gerr);
    log_prior -= std::lgamma((double)csize(st, st.c[i1]));
    log_prior -= priors(this, st, st.c[i1], &gerr);
    log_likelihood += loglikelihood_hamming(this, ss, ss.c[i1]);
    log_likelihood += loglikelihood_hamming(this, ss, ss.c[i2]);
    log_likelihood -= loglikelihood_hamming(this, st, st.c[i1]);
    log_proposal += logprobgs_phi(this, st, ml, i1, &gerr);
    log_proposal -= logprobgs_phi(this, ss, sl, i1, &gerr);
    log_proposal -= logprobgs_phi(this, ss, sl, i2, &gerr);
    log_proposal -= logprobgs_c_i(this, ss, sl, S, i1, i2);
    acpt = min0(log_prior + log_likelihood + log_proposal);
  } else {
    ss = ml;
    e = hupdate_phi(this, ss, {ss.c[i2]});
    if (e) { err = "update_phi failed"; return e; }
    // sm:489-540
    double log_prior = 0.0, log_likelihood = 0.0, log_proposal = 0.0;
    log_prior += std::lgamma((double)csize(ss, ss.c[i1]));
    log_prior += priors(this, ss, ss.c[i1], &gerr);
    log_prior -= std::log(alpha);
    log_prior -= std::lgamma((double)csize(st, st.c[i1]));
    log_prior -= std::lgamma((double)csize(st, st.c[i2]));
    log_prior -= priors(this, st, st.c[i1], &gerr);
    log_prior -= priors(this, st, st.c[i2], &gerr);
    log_likelihood += loglikelihood_hamming(this, ss, ss.c[i2]);
    log_likelihood -= loglikelihood_hamming(this, st, st.c[i1]);
    log_likelihood -= loglikelihood_hamming(this, st, st.c[i2]);
    log_proposal += logprobgs_phi(this, st, sl, i1, &gerr);
    log_proposal += logprobgs_phi(this, st, sl, i2, &gerr);
    log_proposal += logprobgs_c_i(this, st, sl, S, i1, i2);
    log_proposal -= logprobgs_phi(this, ss, ml, i2, &gerr);
    acpt = min0(log_prior + log_likelihood + log_proposal);
  }
  if (gerr) { err = "norm_const2 - hypergeometric diverging with infinity"; return gerr; }
  e = hvalidate(ss);
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
  std::vector<int> SS(S, S + nS);
  int st = restricted_gibbs(c, SS, s, i1, i2, t);
  if (st) { c->err = "restricted gibbs failed"; return st; }
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
  *out = logprobgs_c_i(c, gs, g, SS, i1, i2);
  return kOk;
}

}  // namespace hdpm
