// launcher_hip.cpp -- Rcpp adapter: the reference's R entry point run_markov_chain
// (code/launcher.cpp:6-14, called by realdata_analysis/zoo_simulator.R:138-155 and
// digits_simulator.R:151-168) backed by the MI355X engine (libhdpm.so, include/hdpm.h).
//
// Use: build libhdpm.so (make -C split_and_merge_gibbs_sampling_amd/csrc), then in the R
// scripts replace Rcpp::sourceCpp("../code/launcher.cpp") with
//   Sys.setenv(PKG_CXXFLAGS = "-I/path/to/repo/include -I/path/to/repo/integration",
//              PKG_LIBS = "-L/path/to/repo/split_and_merge_gibbs_sampling_amd -lhdpm "
//                         "-Wl,-rpath,/path/to/repo/split_and_merge_gibbs_sampling_amd")
//   Rcpp::sourceCpp("/path/to/repo/integration/launcher_hip.cpp")
// The call run_markov_chain(data = zoo, attrisize = mm, ...) stays as it is.
//
// The body is hdpm_chain.hpp (R-free, replayed against the CPU oracle by
// tests/cpp/adapter_replay.cpp); this file only converts R objects and hands R's random
// stream in and out.  It compiles where R and Rcpp are installed (not in this image).
// [[Rcpp::plugins(cpp17)]]
#include <Rcpp.h>

#include "hdpm_chain.hpp"

using namespace Rcpp;

// rng = false: no RNGScope in the generated wrapper.  With one, its PutRNGstate() on exit
// would write R's internal generator table -- untouched by the engine -- over the advanced
// .Random.seed this function hands back, and the next chain (zoo_simulator.R:92-155 runs
// several without set.seed) would replay the same stream.  The hand-over is done here.
// [[Rcpp::export(rng = false)]]
List run_markov_chain(NumericMatrix data, IntegerVector attrisize, double gamma, NumericVector v, NumericVector w,
                      int verbose = 0, int m = 5, int iterations = 1000, int L = 1,
                      Rcpp::Nullable<Rcpp::IntegerVector> c_i = R_NilValue, int burnin = 5000, int t = 10,
                      int r = 10, bool neal8 = false, bool split_merge = true, int n8_step_size = 1,
                      int sam_step_size = 1, int thinning = 1) {
  const int n = data.nrow(), d = data.ncol();
  // R's stream -> the engine: GetRNGstate seeds R's generator if the session has none yet,
  // PutRNGstate makes .Random.seed = (kind, mti, mt[624]) current
  GetRNGstate();
  PutRNGstate();
  IntegerVector seed = clone(as<IntegerVector>(Environment::global_env()[".Random.seed"]));
  if (seed.size() != 626 || seed[0] % 100 != 3) Rcpp::stop("hdpm: RNGkind must be Mersenne-Twister");

  const hdpm_chain_params p = {verbose, m, iterations, L, burnin, t, r, neal8 ? 1 : 0, split_merge ? 1 : 0,
                               n8_step_size, sam_step_size, thinning};
  std::vector<int32_t> init;
  if (c_i.isNotNull()) init = as<std::vector<int32_t>>(c_i);
  hdpm_adapter::ChainResult res;
  std::string err;
  const int st = hdpm_adapter::run_markov_chain(data.begin(), n, d, attrisize.begin(), gamma, v.begin(), w.begin(), p,
                                                init.empty() ? nullptr : init.data(), seed.begin() + 1, &res, &err);
  if (st != HDPM_OK) Rcpp::stop("hdpm: " + err);   // Rcpp::stop / std::runtime_error in the reference

  // the advanced stream -> R: .Random.seed, then R's generator table from it (GetRNGstate),
  // so later R draws and the next chain continue where this one stopped
  Environment::global_env()[".Random.seed"] = seed;
  GetRNGstate();

  // la:57-63 / 139-153: lists per saved iteration; centers / sigmas as lists of K vectors
  // (clone(state.center), clone(state.sigma), la:144-147)
  List tot(iterations), cis(iterations), cen(iterations), sig(iterations);
  for (int at = 0; at < iterations; ++at) {
    const int K = res.total_cls[at];
    List ck(K), sk(K);
    for (int k = 0; k < K; k++) {
      ck[k] = NumericVector(res.centers[at].begin() + (size_t)k * d, res.centers[at].begin() + (size_t)(k + 1) * d);
      sk[k] = NumericVector(res.sigmas[at].begin() + (size_t)k * d, res.sigmas[at].begin() + (size_t)(k + 1) * d);
    }
    tot[at] = K;
    cis[at] = IntegerVector(res.c_i[at].begin(), res.c_i[at].end());
    cen[at] = ck;
    sig[at] = sk;
  }
  return List::create(Named("total_cls") = tot, Named("c_i") = cis, Named("centers") = cen, Named("sigmas") = sig,
                      Named("loglikelihood") = NumericVector(res.loglikelihood.begin(), res.loglikelihood.end()),
                      Named("final_ass") = IntegerVector(res.final_ass.begin(), res.final_ass.end()),
                      Named("time") = (int)res.time_s,
                      Named("accepted") = IntegerVector(res.accepted.begin(), res.accepted.end()));
}
