"""Diagnostics: per-phase resolver timings and prepass precise-pass counts on a config.

Runs a few Neal-8 iterations with debug mode bit 1 (hdpm_set_debug(2)), which makes the
engine print '[prepass]' and '[resolve]' lines to stderr per resolver launch.
Usage: python tools/profile_sweep.py [--config c5] [--iters 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--m", type=int, default=3)
    args = ap.parse_args()
    import split_and_merge_gibbs_sampling_amd as hd
    from split_and_merge_gibbs_sampling_amd.data import config
    ds = config(args.config, n=args.n)
    eng = hd.Engine(0)
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(1)
    p = eng.chain_params(m=args.m, iterations=args.iters + 1, L=0, burnin=0, neal8=True, split_merge=False)
    eng.init_chain(p, c_i=ds.truth)
    for it in range(1, 3):
        eng.iteration(it)
    eng.set_debug(2)
    for it in range(3, 3 + args.iters):
        eng.iteration(it)
    eng.synchronize()
    print(eng.stats(), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
