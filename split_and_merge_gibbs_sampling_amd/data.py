"""Datasets and synthetic workloads for the Hamming-mixture sampler.

* ``load_zoo`` restates the Zoo preprocessing of realdata_analysis/zoo_simulator.R:18-38.
* ``hamming_mixture`` restates the generator model of code/old_code/data_generation.R:1-102
  (per-attribute level counts, uniform centers, P(x_j = c_j) = 1 / (1 + (m_j - 1) e^{-1/sigma}),
  otherwise uniform over the other levels).  It draws with numpy, not R's stream: the
  configs C2-C5 of BASELINE.json are synthetic surrogates, not R fixtures.
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# the UCI Zoo data the reference ships (data/zoo.data), kept as package data
ZOO_PATH = os.path.join(_HERE, "datasets", "zoo.data")


@dataclasses.dataclass
class Dataset:
    codes: np.ndarray          # N x D uint8, values 1..m_j
    attrisize: np.ndarray      # D int32 (m_j)
    v: np.ndarray              # D float64
    w: np.ndarray              # D float64
    gamma: float
    truth: np.ndarray          # N int32 ground-truth labels (0-based)
    name: str = ""

    @property
    def n(self) -> int:
        return int(self.codes.shape[0])

    @property
    def d(self) -> int:
        return int(self.codes.shape[1])


def load_zoo(path: str = ZOO_PATH) -> Dataset:
    """zoo_simulator.R:18-38: drop name/class, +1, recode legs (col 13), mm = #levels."""
    rows = [ln.strip().split(",") for ln in open(path) if ln.strip()]
    gt = np.array([int(r[17]) for r in rows], np.int32)
    x = np.array([[int(v) for v in r[1:17]] for r in rows], np.int64) + 1
    legs = x[:, 12]
    rec = np.ones_like(legs)
    for src, dst in ((3, 2), (5, 3), (6, 4), (7, 5), (9, 6)):
        rec[legs == src] = dst
    x[:, 12] = rec
    mm = np.array([len(np.unique(x[:, j])) for j in range(x.shape[1])], np.int32)
    v = np.array([6.0] * 12 + [3.0] + [6.0] * 3)
    w = np.array([0.25] * 12 + [0.5] + [0.25] * 3)
    return Dataset(x.astype(np.uint8), mm, v, w, 0.68, gt - gt.min(), "zoo")


def hamming_mixture(n: int, d: int, k: int, levels, sigma: float = 0.5, seed: int = 10091995,
                    v: float = 6.0, w: float = 0.25, gamma: float = 0.68, level1_skew: float | None = None,
                    name: str = "") -> Dataset:
    """data_generation.R model with equal cluster sizes.

    levels: int (same m_j for all attributes) or (lo, hi) to draw m_j ~ U{lo..hi}.
    level1_skew: if set, non-center levels put this mass on level 1 (MNIST-surrogate skew).
    """
    rng = np.random.Generator(np.random.MT19937(seed))
    if isinstance(levels, tuple):
        mm = rng.integers(levels[0], levels[1] + 1, size=d).astype(np.int32)
    else:
        mm = np.full(d, int(levels), np.int32)
    centers = (rng.random((k, d)) * mm[None, :]).astype(np.int64) + 1          # uniform levels
    sizes = np.full(k, n // k, np.int64)
    sizes[: n - sizes.sum()] += 1
    truth = np.repeat(np.arange(k, dtype=np.int32), sizes)
    p_c = 1.0 / (1.0 + (mm - 1.0) * np.exp(-1.0 / sigma))                         # P(x_j == c_j)
    cen = centers[truth]                                                       # n x d
    keep = rng.random((n, d)) < p_c[None, :]
    if level1_skew is None:
        # uniform over the m_j - 1 other levels
        off = (rng.random((n, d)) * (mm[None, :] - 1)).astype(np.int64) + 1
        other = (cen - 1 + off) % mm[None, :] + 1
    else:
        u = rng.random((n, d))
        off = (rng.random((n, d)) * (mm[None, :] - 1)).astype(np.int64) + 1
        other = (cen - 1 + off) % mm[None, :] + 1
        one = np.where(cen == 1, other, 1)
        other = np.where(u < level1_skew, one, other)
    codes = np.where(keep, cen, other).astype(np.uint8)
    return Dataset(codes, mm, np.full(d, v), np.full(d, w), gamma, truth, name)


# BASELINE.json configs (C1 is Zoo itself)
CONFIGS = {
    "c2": dict(n=10_000, d=32, k=20, levels=2, name="synthetic N=10k D=32 K=20"),
    "c3": dict(n=100_000, d=64, k=20, levels=(2, 6), name="synthetic N=100k D=64 K=20"),
    "c4": dict(n=70_000, d=784, k=10, levels=6, v=3.0, w=0.5, gamma=0.1514657, level1_skew=0.8,
               name="MNIST surrogate N=70k D=784 K=10"),
    "c5": dict(n=1_000_000, d=128, k=20, levels=4, name="synthetic N=1M D=128 K=20"),
}


def config(name: str, n: int | None = None, **over) -> Dataset:
    if name in ("c1", "zoo"):
        return load_zoo()
    kw = dict(CONFIGS[name])
    if n is not None:
        kw["n"] = n
    kw.update(over)
    return hamming_mixture(**kw)
