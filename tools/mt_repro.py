"""Reproduces test_device_mt_stream_matches_r step by step with progress prints (host fault hunt)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import oracle_ffi as oracle
import split_and_merge_gibbs_sampling_amd as hd
from split_and_merge_gibbs_sampling_amd.data import load_zoo

zoo = load_zoo()
for pre in [int(x) for x in sys.argv[1:]] or [0, 1, 623]:
    e = hd.Engine(0)
    e.set_data(zoo.codes, zoo.attrisize, zoo.gamma, zoo.v, zoo.w)
    st = oracle.seed_state(77)
    oracle.runif(st, pre)
    print("pre", pre, "set", flush=True)
    e.rng_state = st
    for count in (1, 623, 624, 625, 20000):
        print(" fill", count, flush=True)
        got = e.rng_fill_device(count)
        print(" got", flush=True)
        ref = oracle.runif(st, count)
        u = got.astype(np.float64) * 2.3283064365386963e-10
        print(" eq", np.array_equal(u, ref), flush=True)
        s2 = e.rng_state
        print(" state eq", np.array_equal(s2, st), flush=True)
    e.close()
    print("closed", flush=True)
