"""How tight must the prepass's latent-entry bound be?  (design study, CPU only)

For a config's data at a reduced N, with the ground-truth partition and one update_phi,
draws m pool entries per point (oracle pool generator) and counts the point/entry pairs
whose upper bound on the entry's log-weight does NOT clear the certainty cut, under
  * the exact value (a floor for every bound),
  * the 4-plane precise bound of the full record (kernels.hpp),
  * the crude codes-only bound A - dmin H,
  * one penalty plane [d_j >= t] with dmin elsewhere, for several per-entry thresholds t
    ("best": t maximising (t - dmin) #{j: d_j >= t}, the expectation for a random mask).
Usage: python tools/latent_bound_study.py [--config c5] [--n 20000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_ffi as O  # noqa: E402  (design study: the oracle as the data source)
from split_and_merge_gibbs_sampling_amd.data import config  # noqa: E402


def tables(att, sig):
    e = np.exp(1.0 / sig)
    den = np.log(1.0 + (att - 1.0) / e)
    return -den, -1.0 / sig - den          # match, mismatch


def best_threshold(dd, dmin):
    s = -np.sort(-dd, axis=1)                       # descending
    k = np.arange(1, dd.shape[1] + 1)[None, :]
    score = (s - dmin[:, None]) * k
    return s[np.arange(dd.shape[0]), score.argmax(1)]


PAIRS = ((72, 88), (80, 92), (83, 93), (76, 90), (84, 94))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--m", type=int, default=3)
    args = ap.parse_args()
    ds = config(args.config, n=args.n)
    att = ds.attrisize.astype(np.float64)
    K = int(ds.truth.max()) + 1
    st = O.OracleState(ds.truth.copy(), K, np.ones((K, ds.d)), np.full((K, ds.d), 0.5))
    rng = O.seed_state(7)
    O.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, st, rng)
    P = 3 * args.n
    pc, ps, _ = O.pool_generate(ds.attrisize, ds.v, ds.w, P, rng)
    cen = st.centers[:K]
    cm, cx = tables(att[None, :], st.sigma[:K])
    cnt = np.bincount(ds.truth, minlength=K)
    own = ds.truth
    llo = np.where(ds.codes == cen[own], cm[own], cx[own]).sum(1)
    E = K + args.m
    thresh = 54 * np.log(2) + np.log(E) + 0.5 + 0.5
    cut = np.log(cnt[own] - 1.0) + llo - thresh - np.log(ds.gamma / args.m)
    gen = np.random.default_rng(1)
    picks = gen.integers(0, P, size=(ds.n, args.m))
    pm, px = tables(att[None, :], ps)
    dd = pm - px
    A = pm.sum(1)
    dmin = dd.min(1)
    delta = dd.max(1) / 15
    q = np.minimum(np.floor(dd / delta[:, None]), 15)
    ts = {"median": np.median(dd, 1), "q25": np.quantile(dd, 0.25, 1), "q75": np.quantile(dd, 0.75, 1),
          "msb(8delta)": 8 * delta, "best": best_threshold(dd, dmin)}
    res = {"exact": 0, "prec4": 0, "dmin": 0, **{"plane_" + k: 0 for k in ts}, "sortedH": 0, "sortedH_step8": 0,
           **{f"S{h0}+dmin": 0 for h0 in (64, 72, 80, 88)}, **{f"S{a},S{b}+dmin": 0 for a, b in PAIRS}}
    Ssort = np.concatenate([np.zeros((P, 1)), np.cumsum(np.sort(dd, 1), 1)], 1)     # sum of the h smallest d_j
    margins = []
    tot = 0
    for u in range(args.m):
        e = picks[:, u]
        M = ds.codes != pc[e]
        res["exact"] += int((A[e] - (M * dd[e]).sum(1) > cut).sum())
        res["prec4"] += int((A[e] - delta[e] * (M * q[e]).sum(1) > cut).sum())
        H = M.sum(1)
        res["dmin"] += int((A[e] - dmin[e] * H > cut).sum())
        res["sortedH"] += int((A[e] - Ssort[e, H] > cut).sum())
        Hs = (H // 8) * 8
        res["sortedH_step8"] += int((A[e] - Ssort[e, Hs] > cut).sum())
        for h0 in (64, 72, 80, 88):
            low = np.maximum(dmin[e] * H, np.where(H >= h0, Ssort[e, h0] + (H - h0) * dmin[e], 0))
            res[f"S{h0}+dmin"] += int((A[e] - low > cut).sum())
        for a, b in PAIRS:
            low = dmin[e] * H
            for h0 in (a, b):
                low = np.maximum(low, np.where(H >= h0, Ssort[e, h0] + (H - h0) * dmin[e], 0))
            res[f"S{a},S{b}+dmin"] += int((A[e] - low > cut).sum())
        for k, t in ts.items():
            S1 = (M & (dd[e] >= t[e][:, None])).sum(1)
            ub = A[e] - dmin[e] * (H - S1) - t[e] * S1
            res["plane_" + k] += int((ub > cut).sum())
            if k == "best":
                margins.append(cut - ub)
        tot += ds.n
    print(f"{args.config} n={ds.n} pairs={tot}: pairs whose bound does not clear the cut")
    for k, v in res.items():
        print(f"  {k:18s} {v:8d}  {v / tot:.2e}")
    mg = np.concatenate(margins)
    print("  best-plane slack below the cut: quantiles 0.1%/1%/50% =",
          np.round(np.quantile(mg, [0.001, 0.01, 0.5]), 2))


if __name__ == "__main__":
    main()
