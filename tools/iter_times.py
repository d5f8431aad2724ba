"""Per-iteration wall times of the bench workload right after a short warmup (what the
driver's `bench.py --steps 20 --warmup 5` window sees).  Prints one JSON line."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import split_and_merge_gibbs_sampling_amd as hd  # noqa: E402
from split_and_merge_gibbs_sampling_amd.data import config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
ds = config(cfg)
eng = hd.Engine(0)
eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
eng.set_seed(1)
params = eng.chain_params(m=3, iterations=warm + steps, L=0, burnin=0, neal8=True, split_merge=False, t=10, r=10)
eng.init_chain(params, c_i=ds.truth)
eng.iterations(0, warm)
eng.synchronize()
ts = []
for k in range(steps):
    t0 = time.perf_counter()
    eng.iterations(warm + k, 1)
    eng.synchronize()
    ts.append(1e6 * (time.perf_counter() - t0))
t0 = time.perf_counter()
eng.iterations(warm + steps, 20)
eng.synchronize()
batch = 1e6 * (time.perf_counter() - t0) / 20
st = eng.stats()
print(json.dumps({"config": cfg, "warmup": warm, "us_per_iteration": [round(x, 1) for x in ts],
                  "median_us": round(float(np.median(ts)), 1), "batch20_us": round(batch, 1),
                  "rng_windows": st["rng_windows"], "rng_windows_fresh": st["rng_windows_fresh"]}))
