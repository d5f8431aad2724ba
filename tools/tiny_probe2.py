"""Probe 2: tiny-N chain, engine log-likelihood vs the log-likelihood of the engine's own
state (diagnostics)."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import split_and_merge_gibbs_sampling_amd as hd
from split_and_merge_gibbs_sampling_amd.data import hamming_mixture
import oracle_ffi as O
import pyref as P

hd.build()
for n, m in ((7, 1), (4, 3), (2, 1)):
    ds = hamming_mixture(n, 3, 2, 3, seed=40 + n + 3)
    for dbg in [int(x) for x in os.environ.get("DBGS", "0,4,1,2048").split(",")]:
        e = hd.Engine(0)
        e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
        e.set_seed(5)
        e.set_debug(dbg)
        p = e.chain_params(m=m, iterations=3, L=1, burnin=0, neal8=True, split_merge=False)
        e.init_chain(p, c_i=ds.truth)
        c, cen, sig = e.get_state()
        print("n", n, "m", m, "dbg", dbg, "init c", c.tolist(), "cen", cen.tolist(), "sig", np.round(sig, 4).tolist(), flush=True)
        for it in range(3):
            try:
                _, ll = e.iteration(it)
            except Exception as ex:
                print("  it", it, "error", ex, flush=True)
                break
            c, cen, sig = e.get_state()
            mine = sum(P.row_ll(ds.codes[i], cen[c[i]], sig[c[i]], ds.attrisize) for i in range(n))
            st = O.OracleState(c, cen.shape[0], cen.astype(np.float64) if cen.dtype != np.float64 else cen, sig)
            try:
                oll = O.compute_loglikelihood(ds.codes, ds.attrisize, st)
            except Exception as ex:
                oll = repr(ex)
            print("  it", it, "ll", ll, "ll(state)", mine, "oracle ll(state)", oll, "c", c.tolist(), "K", cen.shape[0],
                  "cen", cen.tolist(), flush=True)
        e.close()
