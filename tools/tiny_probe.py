"""Probe: tiny-shape chains, engine vs oracle, per mode and debug bits (diagnostics)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import split_and_merge_gibbs_sampling_amd as hd
from split_and_merge_gibbs_sampling_amd.data import hamming_mixture
import oracle_ffi as O

if len(sys.argv) == 1:
    import subprocess
    for n in [int(x) for x in os.environ.get("NS", "1,2,3,4,7,16,33,64,65,200").split(",")]:
        for mode in ("n8", "sm", "both"):
            if mode != "n8" and n < 2:
                continue
            r = subprocess.run([sys.executable, "-u", __file__, str(n), mode], timeout=60)
            if r.returncode:
                print("n", n, mode, "exit", r.returncode, flush=True)
    sys.exit(0)
hd.build()
n = int(sys.argv[1])
mode = sys.argv[2]
for shape in [(n, int(os.environ.get("D", "3")), min(n, 2), 3)]:
    n, d, k, lv = shape
    ds = hamming_mixture(n, d, k, lv, seed=40 + n + d)
    for m in (1, 3):
        for n8, sm in [{"n8": (True, False), "sm": (False, True), "both": (True, True)}[mode]]:
            kw = dict(m=m, iterations=5, L=1, c_i=ds.truth, burnin=0, neal8=n8, split_merge=sm)
            st, ref = O.run_markov_chain(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w, seed=5, fast=1, **kw)
            for dbg in [int(x) for x in os.environ.get("DBGS", "0,131072").split(",")]:
                e = hd.Engine(0)
                e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
                e.set_seed(5)
                e.set_debug(dbg)
                p = e.chain_params(m=m, iterations=5, L=1, burnin=0, neal8=n8, split_merge=sm)
                e.init_chain(p, c_i=ds.truth)
                out = []
                msg = "ok"
                for it in range(5):
                    try:
                        _, ll = e.iteration(it)
                    except Exception as ex:
                        msg = f"it{it} {ex}"
                        break
                    c, cen, sig = e.get_state()
                    same = np.array_equal(c, ref["c_i"][it]) and abs(ll - ref["loglikelihood"][it]) <= 1e-10 * abs(ref["loglikelihood"][it])
                    if not same:
                        msg = f"it{it} differs c={c.tolist()[:8]} ref={ref['c_i'][it].tolist()[:8]} ll={ll} ref={ref['loglikelihood'][it]}"
                        break
                e.close()
                print(shape, "m", m, "n8" if n8 else "", "sm" if sm else "", "dbg", dbg, "oracle", st, ref["total_cls"].tolist() if st == 0 else "", "->", msg, flush=True)
