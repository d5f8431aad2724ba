"""Independent pure-Python restatement of the reference sampler (TEST INFRASTRUCTURE ONLY).

Written separately from the C oracle (oracle/src) so that the two transcriptions of
code/neal8.cpp, code/common_functions.cpp, code/hyperg.cpp and code/split_merge.cpp can
be checked against each other bit for bit on small inputs (Zoo).  Differences from the C
oracle by construction:
  * R's MT19937 comes from numpy.random.MT19937 fed with R's scrambled seed words;
  * qbeta(0.1, a, b) is scipy.special.betaincinv (R nmath's qbeta is not available);
  * loops are plain Python.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import betaincinv

I2_32M1 = 2.328306437080797e-10


class RRng:
    """R's Mersenne-Twister unif_rand on top of numpy's MT19937 bit generator."""

    def __init__(self, seed: int | None = None, state625=None):
        self.bg = np.random.MT19937(0)
        if state625 is not None:
            st = np.asarray(state625, np.int64)
            key = (st[1:] & 0xFFFFFFFF).astype(np.uint32)
            self.bg.state = {"bit_generator": "MT19937", "state": {"key": key, "pos": int(st[0])}}
        else:
            s = seed & 0xFFFFFFFF
            for _ in range(50):
                s = (69069 * s + 1) & 0xFFFFFFFF
            words = []
            for _ in range(625):
                s = (69069 * s + 1) & 0xFFFFFFFF
                words.append(s)
            self.bg.state = {"bit_generator": "MT19937",
                             "state": {"key": np.array(words[1:], np.uint32), "pos": 624}}

    def unif(self) -> float:
        y = int(self.bg.random_raw())
        x = y * 2.3283064365386963e-10
        if x <= 0.0:
            return 0.5 * I2_32M1
        if 1.0 - x <= 0.0:
            return 1.0 - 0.5 * I2_32M1
        return x

    def export(self) -> np.ndarray:
        st = self.bg.state["state"]
        out = np.zeros(625, np.int32)
        out[0] = st["pos"]
        out[1:] = st["key"].astype(np.uint32).view(np.int32)
        return out


def revsort(a, ib):
    """R sort.c revsort on python lists (descending heapsort with index carry)."""
    n = len(a)
    if n <= 1:
        return
    a.insert(0, None)
    ib.insert(0, None)
    l = (n >> 1) + 1
    ir = n
    while True:
        if l > 1:
            l -= 1
            ra, ii = a[l], ib[l]
        else:
            ra, ii = a[ir], ib[ir]
            a[ir], ib[ir] = a[1], ib[1]
            ir -= 1
            if ir == 1:
                a[1], ib[1] = ra, ii
                break
        i, j = l, l << 1
        while j <= ir:
            if j < ir and a[j] > a[j + 1]:
                j += 1
            if ra > a[j]:
                a[i], ib[i] = a[j], ib[j]
                i = j
                j += j
            else:
                j = ir + 1
        a[i], ib[i] = ra, ii
    a.pop(0)
    ib.pop(0)


def sample_prob1(rng: RRng, probs) -> int:
    """Rcpp sample(x, 1, TRUE, probs) -> 0-based position."""
    p = [float(x) for x in probs]
    n = len(p)
    tot = 0.0
    for x in p:
        if not math.isfinite(x) or x < 0:
            raise ValueError("bad prob")
        if x > 0:
            tot += x
    p = [x / tot for x in p]
    if sum(1 for x in p if n * x > 0.1) > 200:
        return walker(p, rng.unif())
    perm = list(range(1, n + 1))
    revsort(p, perm)
    for i in range(1, n):
        p[i] = p[i] + p[i - 1]
    rU = rng.unif()
    j = 0
    while j < n - 1 and not (rU <= p[j]):
        j += 1
    return perm[j] - 1


def walker(p, u) -> int:
    """R random.c walker_ProbSampleReplace (Rcpp WalkerSample), one draw, 0-based."""
    n = len(p)
    q = [x * n for x in p]
    small = [i for i in range(n) if q[i] < 1.0]
    large = [i for i in range(n) if not q[i] < 1.0]
    HL = small + large[::-1]                 # smalls from the front, larges from the back
    a = list(range(n))
    lpos = len(small)                        # *L: first entry of the large region
    if small and large:
        for k in range(n - 1):
            i, j = HL[k], HL[lpos]
            a[i] = j
            q[j] += q[i] - 1
            if q[j] < 1.0:
                lpos += 1
            if lpos >= n:
                break
    q = [q[i] + i for i in range(n)]
    rU = u * n
    k = int(rU)
    return k if rU < q[k] else a[k]


def rbeta(rng: RRng, aa: float, bb: float) -> float:
    """R nmath rbeta, Cheng's BB (min > 1) and BC algorithms."""
    expmax = 1024 * math.log(2.0)
    a, b = min(aa, bb), max(aa, bb)
    alpha = a + b

    def vw(u1, beta, AA):
        v = beta * math.log(u1 / (1.0 - u1))
        if v <= expmax:
            w = AA * math.exp(v)
            if not math.isfinite(w):
                w = 1.7976931348623157e308
        else:
            w = 1.7976931348623157e308
        return v, w

    if a <= 1.0:
        beta = 1.0 / a
        delta = 1.0 + b - a
        k1 = delta * (0.0138889 + 0.0416667 * a) / (b * beta - 0.777778)
        k2 = 0.25 + (0.5 + 0.25 / delta) * a
        while True:
            u1, u2 = rng.unif(), rng.unif()
            if u1 < 0.5:
                y = u1 * u2
                z = u1 * y
                if 0.25 * u2 + z - y >= k1:
                    continue
            else:
                z = u1 * u1 * u2
                if z <= 0.25:
                    v, w = vw(u1, beta, b)
                    break
                if z >= k2:
                    continue
            v, w = vw(u1, beta, b)
            if alpha * (math.log(alpha / (a + w)) + v) - 1.3862944 >= math.log(z):
                break
        return a / (a + w) if aa == a else w / (a + w)
    beta = math.sqrt((alpha - 2.0) / (2.0 * a * b - alpha))
    gamma = a + 1.0 / beta
    while True:
        u1, u2 = rng.unif(), rng.unif()
        v, w = vw(u1, beta, a)
        z = u1 * u1 * u2
        r = gamma * v - 1.3862944
        s = a + r - w
        if s + 2.609438 >= 5.0 * z:
            break
        t = math.log(z)
        if s > t:
            break
        if not (r + alpha * math.log(alpha / (b + w)) < t):
            break
    return b / (b + w) if aa != a else w / (b + w)


def hyperg_series(a, b, c, x):
    """GSL hyperg_2F1_series (positive-term branch); returns (status, value)."""
    sum_pos, sum_neg, del_pos, del_neg, dl, k, i = 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 0
    while True:
        i += 1
        if i > 30000:
            return 11, sum_pos - sum_neg
        dl = dl * ((a + k) * (b + k) * x / ((c + k) * (k + 1.0)))
        if dl > 0.0:
            del_pos = dl
            sum_pos += dl
        elif dl == 0.0:
            del_pos = del_neg = 0.0
            break
        else:
            del_neg = -dl
            sum_neg -= dl
        k += 1.0
        with np.errstate(all="ignore"):
            crit = np.float64(del_pos + del_neg) / np.float64(sum_pos - sum_neg)
        if not (abs(crit) > 2.2204460492503131e-16):
            break
    return 0, sum_pos - sum_neg


def norm_const2(d, c, m):
    st, val = hyperg_series(d + c, 1.0, d + 2, (m - 1) / m)
    if st == 11:
        return -math.inf
    if not math.isfinite(val) or val == 0:
        raise RuntimeError("norm_const2")
    return math.log(d + 1) + (d + c) * math.log(m) - math.log(val)


def lF_conK2(u, d, c, m, lK):
    if u == 0:
        return -math.inf
    if u == 1:
        return 0.0
    x = u * (m - 1) / (1 + u * (m - 1))
    st, app = hyperg_series(1.0, d + c, d + 2, x)
    if st != 0:
        app = math.nan
    return lK - math.log(d + 1) + (d + 1) * math.log(u) - (d + c) * math.log(1 + u * (m - 1)) + math.log(app)


def bisec_hyper2(d, c, m, Omega):
    centro = 0.5
    lK = norm_const2(d, c, m)
    app = lF_conK2(centro, d, c, m, lK) - math.log(Omega)
    giu, su = (0.5, 1.0) if app < 0 else (0.0, 0.5)
    counter = 1
    while (su - giu) > 0.000000001 and counter < 150:
        centro = (su + giu) / 2
        app = lF_conK2(centro, d, c, m, lK) - math.log(Omega)
        if app < 0:
            giu = centro
        else:
            su = centro
        counter += 1
    return centro


def rhig1(rng, v, w, m):
    lim = (m - 1) / m
    if betaincinv(w + 1, v - 1, 0.1) < lim and lim > 0:
        x = rbeta(rng, w + 1, v - 1)
        while x > lim:
            x = rbeta(rng, w + 1, v - 1)
        out = x / ((m - 1) * (1 - x))
    else:
        out = bisec_hyper2(w, v, m, rng.unif())
    return -1 / math.log(out)


def dhamming(x, c, s, m):
    diff = 1 - (x == c)
    return (-diff) / s - math.log(1.0 + (m - 1.0) / math.exp(1.0 / s))


def row_ll(x, cen, sig, att):
    ll = 0.0
    for j in range(len(x)):
        ll += dhamming(int(x[j]), int(cen[j]), sig[j], int(att[j]))
    return ll


class Model:
    def __init__(self, codes, attrisize, gamma, v, w):
        self.X = [list(map(int, r)) for r in np.asarray(codes)]
        self.att = [int(a) for a in attrisize]
        self.gamma, self.v, self.w = float(gamma), [float(a) for a in v], [float(a) for a in w]
        self.n, self.d = len(self.X), len(self.att)

    def center1(self, rng, probs=None):
        out = []
        for j in range(self.d):
            if probs is None:
                out.append(float(int(self.att[j] * rng.unif() + 1)))
            else:
                out.append(float(sample_prob1(rng, probs[j]) + 1))
        return out

    def sigma1(self, rng, v, w):
        return [rhig1(rng, v[j], w[j], float(self.att[j])) for j in range(self.d)]

    def update_phi(self, rng, c, centers, sigmas, mask=None):
        for i in range(len(centers)):
            if mask is not None and i not in mask:
                continue
            mem = [q for q in range(self.n) if c[q] == i]
            nn = len(mem)
            if nn == 0:
                continue
            probs = []
            for j in range(self.d):
                mj = self.att[j]
                fr = [0.0] * mj
                for q in mem:
                    fr[self.X[q][j] - 1] += 1
                pt = [(-(nn - f)) / sigmas[i][j] for f in fr]
                mx = max(pt)
                pt = [math.exp(p - mx) for p in pt]
                tot = 0.0
                for p in pt:
                    tot += p
                probs.append([p / tot for p in pt])
            centers[i] = self.center1(rng, probs)
            nv, nw = [], []
            for j in range(self.d):
                sd = float(sum(1 for q in mem if self.X[q][j] == centers[i][j]))
                nw.append(self.w[j] + nn - sd)
                nv.append(self.v[j] + sd)
            sigmas[i] = self.sigma1(rng, nv, nw)

    def sample_allocation(self, idx, rng, c, centers, sigmas, m, pool_c, pool_s):
        k = len(set(c))
        k_minus = len(set(c[:idx] + c[idx + 1:]))
        x = self.X[idx]
        probs = []
        for i in range(k):
            ll = row_ll(x, centers[i], sigmas[i], self.att)
            nz = c.count(i) - (c[idx] == i)
            probs.append(math.log(nz) + ll if nz != 0 else -math.inf)
        P = len(pool_c)
        lat = []
        for _ in range(m):
            e = int(P * rng.unif() + 1) - 1
            lat.append((pool_c[e], pool_s[e]))
        if k_minus < k:
            lat[0] = (centers[c[idx]], sigmas[c[idx]])
        lf = math.log(self.gamma / m)
        for (lc, ls) in lat:
            probs.append(lf + row_ll(x, lc, ls, self.att))
        mx = max(probs)
        probs = [math.exp(p - mx) for p in probs]
        tot = 0.0
        for p in probs:
            tot += p
        probs = [p / tot for p in probs]
        new = sample_prob1(rng, probs)
        old = c[idx]
        single = c.count(old) == 1
        if not single and new < k:
            c[idx] = new
        elif new < k and single:
            c[idx] = new
            centers[old] = centers[k - 1]
            sigmas[old] = sigmas[k - 1]
            del centers[k - 1]
            del sigmas[k - 1]
            for i in range(self.n):
                if c[i] == k - 1:
                    c[i] = old
        elif new >= k and not single:
            c[idx] = k
            centers.append(lat[new - k][0])
            sigmas.append(lat[new - k][1])
        else:
            centers[old] = lat[new - k][0]
            sigmas[old] = lat[new - k][1]

    def loglik(self, c, centers, sigmas):
        ll = 0.0
        for i in range(self.n):
            for j in range(self.d):
                ll += dhamming(self.X[i][j], int(centers[c[i]][j]), sigmas[c[i]][j], self.att[j])
        return ll

    def run_neal8(self, rng, c_init, m, iterations):
        """run_markov_chain with neal8=TRUE, split_merge=FALSE, burnin=0, thinning=1."""
        mn = min(c_init)
        c = [int(x) - mn for x in c_init]
        K = len(set(c))
        centers = [self.center1(rng) for _ in range(K)]
        sigmas = [self.sigma1(rng, self.v, self.w) for _ in range(K)]
        self.update_phi(rng, c, centers, sigmas)
        P = self.n * m
        pool = [(self.center1(rng), self.sigma1(rng, self.v, self.w)) for _ in range(P)]
        pool_c = [p[0] for p in pool]
        pool_s = [p[1] for p in pool]
        trace, lls = [], []
        for it in range(iterations):
            for i in range(self.n):
                self.sample_allocation(i, rng, c, centers, sigmas, m, pool_c, pool_s)
            self.update_phi(rng, c, centers, sigmas)
            if it % 1000 == 0:
                for e in range(P):
                    pool_c[e] = self.center1(rng)
                    pool_s[e] = self.sigma1(rng, self.v, self.w)
            lls.append(self.loglik(c, centers, sigmas))
            trace.append(list(c))
        return trace, lls
