"""Diagnostics: time the device R-stream generator (k_mt_gen_multi) for a window size.
Usage: HDPM_MT_WORKGROUPS=G python tools/mt_bench.py [--count N] [--reps R]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=4_200_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import split_and_merge_gibbs_sampling_amd as hd
    eng = hd.Engine(0)
    from split_and_merge_gibbs_sampling_amd.data import load_zoo
    z = load_zoo()
    eng.set_data(z.codes, z.attrisize, z.gamma, z.v, z.w)
    eng.set_seed(7)
    for r in range(args.reps):
        t0 = time.perf_counter()
        out = eng.rng_fill_device(args.count)
        dt = time.perf_counter() - t0
        print(f"rep {r}: {dt * 1e3:.2f} ms  (first {int(out[0])})", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
