"""Diagnostics: one device update_phi after a sweep on a synthetic shape, with the engine's
[phi] trace (debug bit 1)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import split_and_merge_gibbs_sampling_amd as hd
import oracle_ffi as O
from split_and_merge_gibbs_sampling_amd.data import hamming_mixture

ds = hamming_mixture(8000, 128, 12, 4, seed=5)
rng = np.random.default_rng(13)
K = 12
cen = np.stack([rng.integers(1, ds.attrisize + 1) for _ in range(K)]).astype(np.float64)
sig = rng.uniform(0.15, 2.5, size=(K, ds.d))
st = O.seed_state(43)
pc, ps, _ = O.pool_generate(ds.attrisize, ds.v, ds.w, ds.n * 3, st)
e = hd.Engine(0)
e.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
e.set_phi_device(True)
e.set_state(ds.truth, cen, sig)
e.set_pool(pc, ps)
e.rng_state = st
for it in range(3):
    e.neal8_sweep(3)
    e.set_debug(2)
    e.update_phi()
    e.set_debug(0)
    s = e.stats()
    print("it", it, {k: s[k] for k in ("phi_device_calls", "phi_device_fallbacks", "phi_device_last_status")}, flush=True)
e.close()
