"""Posterior analysis of saved chains, as realdata_analysis/zoo_simulator.R:193-236, 339-344.

The reference script summarises every run with CRAN packages:
  * ``comp.psm(C)`` (mcclust) -- the posterior similarity matrix of the saved labels;
  * ``minVI(psm)`` (mcclust.ext) -- the partition minimising ``VI.lb``, the lower bound of
    the posterior expected variation of information (default method "avg": cuts of the
    average-linkage tree of 1 - psm into 1..ceiling(N / 8) clusters; "draws": the saved
    partitions themselves);
  * ``arandi(VI$cl, gt)`` (mcclust) -- the adjusted Rand index against the ground truth;
  * ``ESS`` and ``IAT`` (LaplacesDemon) of (total_cls, loglikelihood).

The N x N matrix is built and queried on the device (csrc/posterior.hip through
``hdpm_psm_*``): at C4 (N = 70k) it has 4.9e9 entries.  ``arandi``, ``ess`` and ``iat`` are
restated on the host.  None of these packages is installed here (no R), so their parity is
unpinned; ``arandi`` is checked against scikit-learn's adjusted Rand score.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import ptr


class PSM:
    """comp.psm(C) on the device: ``c_trace`` is the M x N matrix of saved labels
    (results$c_i, any integers).  The PSM depends only on which points share a label within
    an iteration, so each saved row is relabelled 0..K_m-1 first (the device packs one byte
    per label: at most 255 clusters in one iteration, else ValueError).  Rows come back as
    doubles (count / M)."""

    def __init__(self, c_trace, engine=None, device: int = 0):
        from .sampler import Engine
        tr = np.ascontiguousarray(c_trace, dtype=np.int32)
        if tr.ndim != 2:
            raise ValueError("c_trace must be M x N")
        self.M, self.N = tr.shape
        dense = np.empty_like(tr)
        for q in range(self.M):
            u, dense[q] = np.unique(tr[q], return_inverse=True)
            if u.size > 255:
                raise ValueError(f"iteration {q} has {u.size} clusters; the device PSM packs at most 255")
        tr = np.ascontiguousarray(dense, dtype=np.int32)
        self._own = engine is None
        self.eng = Engine(device) if engine is None else engine
        self.eng._check(self.eng._L.hdpm_psm_build(self.eng._h, ptr(tr), self.M, self.N))

    def close(self):
        if self._own and self.eng is not None:
            self.eng.close()
        self.eng = None

    def rows(self, row0: int, nrows: int) -> np.ndarray:
        out = np.zeros((nrows, self.N))
        self.eng._check(self.eng._L.hdpm_psm_rows(self.eng._h, int(row0), int(nrows), ptr(out)))
        return out

    def matrix(self) -> np.ndarray:
        return self.rows(0, self.N)

    def vi_lb(self, cls) -> np.ndarray:
        """mcclust.ext VI.lb(cls, psm) of each row of ``cls`` (candidate partitions)."""
        c = np.ascontiguousarray(np.atleast_2d(cls), dtype=np.int32)
        if c.shape[1] != self.N:
            raise ValueError("partitions must have N labels")
        c = np.stack([np.unique(r, return_inverse=True)[1] for r in c]).astype(np.int32)
        out = np.zeros(c.shape[0])
        self.eng._check(self.eng._L.hdpm_psm_vi_lb(self.eng._h, ptr(c), c.shape[0], ptr(out)))
        return out


def comp_psm(c_trace, device: int = 0) -> np.ndarray:
    """mcclust::comp.psm: the full N x N matrix (moderate N)."""
    p = PSM(c_trace, device=device)
    try:
        return p.matrix()
    finally:
        p.close()


def minvi(psm: PSM, cls_draw=None, method: str = "avg", max_k: int | None = None):
    """mcclust.ext::minVI for the methods "avg" (cuts of the average-linkage tree of
    1 - psm, k = 1..max_k, default ceiling(N / 8); the tree on the host, needs the full
    matrix) and "draws" (the saved partitions).  Returns (cl, value) with cl 1-based."""
    if method == "draws":
        if cls_draw is None:
            raise ValueError("method 'draws' needs cls_draw")
        cand = np.atleast_2d(np.asarray(cls_draw))
    elif method == "avg":
        from scipy.cluster.hierarchy import cut_tree, linkage
        from scipy.spatial.distance import squareform
        m = psm.matrix()
        dist = 1.0 - m
        np.fill_diagonal(dist, 0.0)
        Z = linkage(squareform(dist, checks=False), method="average")
        kmax = max_k if max_k is not None else math.ceil(psm.N / 8)
        cand = cut_tree(Z, n_clusters=list(range(1, kmax + 1))).T
    else:
        raise ValueError(f"unknown method {method!r}")
    vals = psm.vi_lb(cand)
    best = int(np.argmin(vals))
    cl = np.unique(cand[best], return_inverse=True)[1] + 1
    return cl, float(vals[best])


def arandi(cl1, cl2, adjust: bool = True) -> float:
    """mcclust::arandi (Hubert & Arabie's adjusted Rand index)."""
    a, b = np.asarray(cl1), np.asarray(cl2)
    if a.shape != b.shape:
        raise ValueError("cl1 and cl2 must have same length")
    _, ia = np.unique(a, return_inverse=True)
    _, ib = np.unique(b, return_inverse=True)
    tab = np.zeros((ia.max() + 1, ib.max() + 1), np.int64)
    np.add.at(tab, (ia, ib), 1)

    def ch2(x):
        x = np.asarray(x, np.float64)
        return x * (x - 1) / 2

    n = a.size
    t1, t2 = tab.sum(1), tab.sum(0)
    if adjust:
        correc = ch2(t1).sum() * ch2(t2).sum() / ch2(n)
        return float((ch2(tab).sum() - correc) / (0.5 * ch2(t1).sum() + 0.5 * ch2(t2).sum() - correc))
    return float(1 + ((tab.astype(np.float64) ** 2).sum() - 0.5 * (t1 ** 2).sum() - 0.5 * (t2 ** 2).sum()) / ch2(n))


def _ar_yw_spectrum0(x: np.ndarray) -> float:
    """R's ar(x, aic = TRUE) (Yule-Walker, ar.yw) and its spectral density at 0:
    var.pred / (1 - sum(ar))^2 (coda spectrum0.ar, used by LaplacesDemon::ESS)."""
    n = x.size
    xc = x - x.mean()
    order_max = min(n - 1, int(math.floor(10 * math.log10(n))))
    r = np.array([np.dot(xc[:n - k], xc[k:]) / n for k in range(order_max + 1)])
    # Levinson-Durbin (R's eureka): coefficients and prediction variances per order
    var = [r[0]]
    coefs = []
    a = np.zeros(0)
    v = r[0]
    for k in range(1, order_max + 1):
        if v <= 0:
            break
        kappa = (r[k] - np.dot(a, r[1:k][::-1])) / v
        a = np.concatenate([a - kappa * a[::-1], [kappa]])
        v = v * (1 - kappa * kappa)
        coefs.append(a.copy())
        var.append(v)
    var = np.array(var)
    aic = n * np.log(var) + 2 * np.arange(var.size) + 2
    order = int(np.argmin(aic))
    ar = coefs[order - 1] if order > 0 else np.zeros(0)
    vp = var[order] * n / (n - (order + 1))
    return float(vp / (1 - ar.sum()) ** 2)


def ess(x) -> np.ndarray:
    """LaplacesDemon::ESS (per column): n var(x) / spectrum0.ar(x), clamped to [1, n]
    (0 spectrum -> 0 -> 1)."""
    X = np.asarray(x, np.float64)
    if X.ndim == 1:
        X = X[:, None]
    n = X.shape[0]
    out = []
    for col in X.T:
        z = np.arange(1, n + 1, dtype=np.float64)
        resid = col - np.polyval(np.polyfit(z, col, 1), z)
        if np.isclose(resid.std(ddof=1), 0.0):
            out.append(1.0)
            continue
        spec = _ar_yw_spectrum0(col)
        e = n * col.var(ddof=1) / spec if spec != 0 else 0.0
        out.append(float(min(max(e, 1.0) if e > 0 else 1.0, n)))
    return np.array(out)


def iat(x) -> float:
    """LaplacesDemon::IAT: -1 + 2 sum of the autocorrelations up to the first non-positive
    one (Geyer's initial positive sequence on single lags), at most n / 2 lags."""
    dt = np.asarray(x, np.float64).ravel()
    n = dt.size
    mu, s2 = dt.mean(), dt.var(ddof=1)
    maxlag = max(3, n // 2)
    g1 = s2 * (n - 1) / n
    m = 1
    g2 = np.dot(dt[:n - m] - mu, dt[m:] - mu) / n
    t = g1 / s2
    while g2 > 0.0 and m < maxlag:
        m += 1
        g1 = g2
        g2 = np.dot(dt[:n - m] - mu, dt[m:] - mu) / n
        t += g1 / s2
    return float(-1 + 2 * t)
