// hdpm_chain.hpp -- the body of the reference's Rcpp export run_markov_chain
// (code/launcher.cpp:6-174) as a sequence of calls into the C ABI (include/hdpm.h), with no
// R types: launcher_hip.cpp wraps it in the Rcpp signature, tests/cpp/adapter_replay.cpp
// replays it against the CPU oracle.  Header-only, C++17.
//
// Call sequence (one call of the R function):
//   hdpm_ctx_create -> hdpm_set_data (NumericMatrix -> codes) -> hdpm_rng_set_state
//   (.Random.seed words 1..625, la: RNGScope entry) -> hdpm_init_chain (la:27-77) ->
//   hdpm_iterations_record over the (iterations + burnin) * thinning iterations in batches
//   (la:85-154; every saved iteration's K, labels, centers and sigmas recorded, la:140-153,
//   with the next sweep kept pipelined) + hdpm_record_take after each batch ->
//   hdpm_get_state (final_ass, la:170) -> hdpm_rng_get_state (the advanced stream back to R)
//   -> hdpm_ctx_destroy.
#pragma once

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "../include/hdpm.h"

namespace hdpm_adapter {

// la:57-63 results, one entry per saved iteration; centers / sigmas as K x d rows
struct ChainResult {
  std::vector<int32_t> total_cls;
  std::vector<std::vector<int32_t>> c_i;
  std::vector<std::vector<double>> centers, sigmas;
  std::vector<double> loglikelihood;
  std::vector<int32_t> accepted;
  std::vector<int32_t> final_ass;
  double time_s = 0.0;
};

// Owns one context for the duration of a call (destroyed on every exit path).
class Ctx {
 public:
  explicit Ctx(int device) { status_ = hdpm_ctx_create(device, &c_); }
  ~Ctx() {
    if (c_) hdpm_ctx_destroy(c_);
  }
  Ctx(const Ctx&) = delete;
  Ctx& operator=(const Ctx&) = delete;
  hdpm_ctx* get() const { return c_; }
  int status() const { return status_; }

 private:
  hdpm_ctx* c_ = nullptr;
  int status_ = HDPM_OK;
};

// run_markov_chain (la:6-174).  `data` is the N x D NumericMatrix (column-major doubles,
// values 1..m_j), `c_i_init` may be null (random init with L labels, la:28-31).
// `rng_state` holds the 625 words of .Random.seed after the kind word (mti, mt[624]): read
// on entry, overwritten with the advanced stream on success.  Returns HDPM_OK or the
// engine's status, with `err` set.
inline int run_markov_chain(const double* data, int n, int d, const int32_t* attrisize, double gamma, const double* v,
                            const double* w, const hdpm_chain_params& p, const int32_t* c_i_init,
                            int32_t* rng_state, ChainResult* out, std::string* err, int device = 0) {
  // NumericMatrix -> row-major codes.  The reference compares the doubles themselves
  // (n8:48 -> cf:355), so a value that is not one of the levels 1..m_j cannot be narrowed to
  // a byte: it is rejected here, before any cast (1.5 or 257.0 would otherwise become a valid
  // code silently).
  if (n <= 0 || d <= 0 || !data || !attrisize) {
    if (err) *err = "empty data matrix";
    return HDPM_E_ARG;
  }
  std::vector<uint8_t> codes((size_t)n * d);
  for (int j = 0; j < d; j++) {
    const double hi = (double)attrisize[j];
    for (int i = 0; i < n; i++) {
      const double x = data[(size_t)j * n + i];
      if (!(x >= 1.0 && x <= hi && x <= 255.0) || x != std::floor(x)) {
        if (err)
          *err = "data[" + std::to_string(i) + ", " + std::to_string(j) + "] = " + std::to_string(x) +
                 " is not an integer level in 1..attrisize[j]";
        return HDPM_E_ARG;
      }
      codes[(size_t)i * d + j] = (uint8_t)x;
    }
  }
  Ctx ctx(device);
  auto fail = [&](int st) {
    if (err) *err = ctx.get() ? hdpm_last_error(ctx.get()) : "no gfx950 device";
    return st;
  };
  if (ctx.status() != HDPM_OK) return fail(ctx.status());
  int st = hdpm_set_data(ctx.get(), codes.data(), n, d, attrisize, gamma, v, w);
  if (st) return fail(st);
  if ((st = hdpm_rng_set_state(ctx.get(), rng_state))) return fail(st);

  if ((st = hdpm_init_chain(ctx.get(), &p, c_i_init))) return fail(st);   // la:27-77
  // la:79: the clock starts after the initial state and the latent pool are built
  const auto t0 = std::chrono::steady_clock::now();
  const int saved = p.iterations;
  out->total_cls.assign(saved, 0);
  out->c_i.assign(saved, {});
  out->centers.assign(saved, {});
  out->sigmas.assign(saved, {});
  out->loglikelihood.assign(saved, 0.0);
  out->accepted.assign(saved, 0);
  std::vector<int32_t> lab(n);
  int32_t idx_1_sm = 0;
  const int total = (p.iterations + p.burnin) * p.thinning;
  // batches of iterations (la:85-154) with the saved ones recorded (la:140-153); 64 per call:
  // each call boundary restarts the pipeline, and a larger label block (256 x N, 1 GB at N = 1M)
  // measured 32% slower at C5 than 64 (profiles/r06/record6c/)
  const int kBatch = 64;
  std::vector<int32_t> acc(kBatch), kk(kBatch), labs;
  std::vector<double> lik(kBatch), cen, sig;
  for (int it0 = 0; it0 < total; it0 += kBatch) {
    const int cnt = std::min(kBatch, total - it0);
    labs.resize((size_t)cnt * n);
    int32_t ns = 0;
    if ((st = hdpm_iterations_record(ctx.get(), &p, it0, cnt, &idx_1_sm, acc.data(), lik.data(), kk.data(),
                                     labs.data(), &ns)))
      return fail(st);
    int64_t rows = 0;
    if ((st = hdpm_record_take(ctx.get(), nullptr, nullptr, &rows))) return fail(st);
    cen.resize((size_t)rows * d);
    sig.resize((size_t)rows * d);
    if ((st = hdpm_record_take(ctx.get(), cen.data(), sig.data(), &rows))) return fail(st);
    size_t row = 0;
    int q = 0;
    for (int k = 0; k < cnt; ++k) {
      const int iter = it0 + k;
      if (!(iter >= p.thinning * p.burnin && iter % p.thinning == 0)) continue;
      const int at = iter / p.thinning - p.burnin;
      const int K = kk[q];
      out->total_cls[at] = K;
      out->c_i[at].assign(labs.begin() + (size_t)q * n, labs.begin() + (size_t)(q + 1) * n);
      out->centers[at].assign(cen.begin() + row * d, cen.begin() + (row + K) * d);
      out->sigmas[at].assign(sig.begin() + row * d, sig.begin() + (row + K) * d);
      out->loglikelihood[at] = lik[k];
      out->accepted[at] = acc[k];
      row += (size_t)K;
      ++q;
    }
  }
  out->time_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int32_t K = 0;
  if ((st = hdpm_get_state(ctx.get(), lab.data(), &K, nullptr, nullptr, 0))) return fail(st);
  out->final_ass = lab;                                                      // la:170
  if ((st = hdpm_rng_get_state(ctx.get(), rng_state))) return fail(st);     // the stream back to R
  return HDPM_OK;
}

}  // namespace hdpm_adapter
