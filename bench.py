"""Benchmark: full Neal-8 Gibbs iterations per second on the MI355X engine.

One step = one pass of the reference loop body code/launcher.cpp:94-132 with neal8=TRUE,
split_merge=FALSE: N sequential reassignments (sample_allocation) + update_phi +
compute_loglikelihood, on synthetic data already resident in HBM.  The default workload
is BASELINE config C5 (N = 1,000,000, D = 128, m_j = 4, K_true = 20, m = 3 latent
clusters), initialised at the generator's ground truth (L = 0 path, la:32-39).

Multi-GPU: one process per GPU; every rank runs an independent chain with its own seed
(replicas, "scaling": "weak"); the only collectives are the timing barrier / max and a
gather of the per-rank setup.  Under torch.distributed.run (WORLD_SIZE set) this process is
one rank; `--gpus N > 1` without it starts the N ranks under torch.distributed.run as a
child process (before anything touches a GPU) and exits with its code.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c5] [--n N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PMC_ROUND = "r06"        # profiles/<round>/pmc_{fetch,write}_<config>.csv: this round's counter passes


def packed_layout(d: int, mmax: int):
    """(bits per attribute, bit-sliced words per row, bound words per entry) as in
    csrc/kernels.hpp (plane_words, bound_words)."""
    wb = 1 if mmax <= 2 else 2 if mmax <= 4 else 4 if mmax <= 16 else 8
    wd = -(-d // 64)
    Ws = 2 if wd <= 2 else 4 if wd <= 4 else wd
    return wb, wb * Ws, (wb + 4) * Ws + 4


# FETCH_SIZE calibration on gfx950 (tools/fetch_calib.hip, profiles/r01/fetch_calib.log;
# gather448g -- 16-lane groups gathering 448-B wide heads -- profiles/r02/fetch_calib_wide.log
# and profiles/r02/pmc_fetch_calib.csv): reported / true bytes and measured rates of the
# prepass's access shapes
FETCH_FACTOR = {"stream16": 0.5, "gather64": 1.0, "gather128": 0.584, "gather448g": 0.569}
RATE_GBPS = {"stream16": 5650.0, "gather64": 3080.0, "gather128": 3830.0, "gather448g": 5757.0}
# The prepass's whole access mix replayed without its arithmetic (tools/fetch_calib.hip k_mix64 /
# k_mix448g, best of 3, profiles/r05/fetch_calib.log): (points, us) for the layouts it models --
# C5 (rows of 4 words, three 64-B heads from a 192 MB pool: the pool sits in the Infinity Cache,
# which the 1 GiB gathers above do not model) and C4 (52-word rows, three 448-B heads, 16-lane groups)
MIX_US = {("gather64", 4, 3): (1048576, 72.4), ("gather448g", 52, 3): (70000, 29.9)}


def head_layout(d: int, mmax: int):
    """(has heads, head stride in words) as in csrc/kernels.hpp (templ_fits, wide_fits,
    head_stride): templated layouts pad wb Ws + 2 words to a power of two, wide ones
    (k_prepass_wide) to a multiple of 8 words."""
    wb, W, bw = packed_layout(d, mmax)
    Ws = W // wb
    templ = Ws == 2 or (Ws == 4 and wb <= 4)
    wide = not templ and Ws <= 32 and W <= 64
    if templ:
        hs = 4
        while hs < W + 2:
            hs *= 2
    else:
        hs = -(-(W + 2) // 8) * 8
    return templ or wide, hs, templ


def prepass_shape(d: int, mmax: int, m: int):
    """(streamed bytes, gathered bytes, gather shape) per point of k_prepass: streamed are
    the row, raw draws and label reads (margin / row index writes are WRITE_SIZE), gathered
    the m latent picks (heads, else full 8 bw-byte records)."""
    wb, W, bw = packed_layout(d, mmax)
    head, hs, templ = head_layout(d, mmax)
    g = m * 8 * (hs if head else bw)
    if head and templ:
        shape = "gather64" if hs == 8 else "gather128"
    elif head:
        shape = "gather448g"
    else:
        shape = "gather128"
    return 8 * W + 4 * (m + 1) + 4, g, shape


def prepass_kernel_name(d: int, mmax: int) -> str:
    """The prepass kernel the layout takes (csrc/kernels.hip launch_prepass)."""
    head, _, templ = head_layout(d, mmax)
    return "k_prepass" if templ else "k_prepass_wide" if head else "k_prepass_generic"


def prepass_bytes_per_point(d: int, mmax: int, m: int) -> int:
    """Compulsory bytes k_prepass moves per point: its bit-sliced row
    (8 W), its m+1 raw draws (4(m+1)), its label (4), the first gather of each of its m
    latent pool picks -- the pool-entry head (W + 2 words padded: 64 B at C5, 448 B at C4)
    when the layout has one, else the full bound record (8 bw) -- its margin (8) and row
    index (4).  The full records a head leaves uncertain (6e-5 of the picks at C5) are extra
    traffic, not counted here; cluster records are cache-resident (K of them per sweep)."""
    wb, W, bw = packed_layout(d, mmax)
    head, hs, _ = head_layout(d, mmax)
    return 8 * W + 4 * (m + 1) + 4 + m * 8 * (hs if head else bw) + 12


def survey_sweep_bytes(n: int, d: int, m: int) -> int:
    """B_sweep = N (D (2 + 9m) + 8)."""
    return n * (d * (2 + 9 * m) + 8)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv) -> int:
    """`--gpus N > 1` without a launcher: start N rank processes (one per GPU) under
    torch.distributed.run as a CHILD of this process -- nothing here has touched a GPU, and
    this process never re-executes itself -- and return its exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


def rank_setup(rank: int, local: int) -> dict:
    """Per-rank chain setup (replicas): GPU `local`, chain seed 1 + rank (the
    data seed is shared, so every rank samples the same posterior with its own stream); the
    engine homes its host pool on an L3 domain local to that GPU (engine.cpp gpu_home_domain)."""
    return {"rank": rank, "device": local, "seed": 1 + rank}


def aggregate(ws: int, steps: int, elapsed_max: float) -> float:
    """Whole-job throughput: the iterations all ranks ran over the slowest rank's time."""
    return ws * steps / elapsed_max


class Dist:
    """Barrier and max-over-ranks for the timing (RCCL when >1 rank, else no-op)."""

    def __init__(self, ws, rank, local, backend=None):
        self.ws, self.rank, self.local = ws, rank, local
        self.dist = None
        if ws > 1:
            import torch
            import torch.distributed as dist
            backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(local)
            dist.init_process_group(backend=backend)
            self.dist, self.torch, self.backend = dist, torch, backend

    def _dev(self):
        return f"cuda:{self.local}" if self.backend == "nccl" else "cpu"

    def barrier(self):
        if self.dist is not None:
            t = self.torch.zeros(1, device=self._dev())
            self.dist.all_reduce(t)
            if self.backend == "nccl":
                self.torch.cuda.synchronize()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self._dev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.ws
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def cuda_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def host_cpu():
    """CPU model and the cores this process may use (the GPU box shares a larger host)."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, len(os.sched_getaffinity(0)), os.cpu_count()


def cpu_baseline(ds, eng, m: int, budget_s: float, opt_threads: int, threads_source: str = ""):
    """The CPU baselines of SURVEY 8(d), timed on this host on the current chain state with
    the engine's latent pool (oracle/ is the checker; these legs only time it):
      1. reference-faithful restatement (O(N) bookkeeping per point as in code/neal8.cpp,
         one core, as the single-threaded reference): a full sweep when it fits the budget
         (C2), else consecutive sample_allocation calls from the middle of a sweep,
         extrapolated to one sweep;
      2. optimised oracle (oracle/src/fast.c: same trace; log-likelihoods in parallel on
         `opt_threads` threads, serial scan on one): one full sweep + update_phi +
         compute_loglikelihood, the step the GPU is timed on."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import oracle_ffi as O  # cpu_baseline leg only
    c, cen, sig = eng.get_state()
    P = ds.n * m
    pc, ps = eng.get_pool(P)
    st = O.seed_state(99)
    data_cm = O.colmajor(ds.codes)
    att = np.ascontiguousarray(ds.attrisize, np.int32)
    model, cores, ncpu = host_cpu()

    def run(first, count, fast=0):
        ost = O.OracleState(c, cen.shape[0], cen, sig, cap=max(4096, 2 * cen.shape[0]))
        K = C.c_int(ost.K)
        t0 = time.perf_counter()
        r = O.lib().orc_ffi_neal8_sweep(data_cm, ds.n, ds.d, att, ds.gamma, np.ascontiguousarray(ds.v),
                                        np.ascontiguousarray(ds.w), ost.c_i, C.byref(K), ost.centers.reshape(-1),
                                        ost.sigma.reshape(-1), ost.cap, m, pc.reshape(-1), ps.reshape(-1), P,
                                        st.copy(), fast, first, count)
        ost.K = K.value
        return time.perf_counter() - t0, r, ost

    t_probe, _, _ = run(ds.n // 2, 4)
    per = max(t_probe / 4, 1e-7)
    if per * ds.n <= budget_s:
        first, count = 0, ds.n
    else:
        first = ds.n // 2
        count = int(min(max(budget_s / per, 8), ds.n - first))
    t, r, _ = run(first, count)
    per_point = t / count
    full = count == ds.n
    faithful = {
        "value": 1.0 / (per_point * ds.n),
        "unit": "sweeps/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{'one full sweep' if full else f'{count} consecutive sample_allocation calls (points {first}..{first + count - 1}) of one sweep'}"
                   f", reference-faithful O(N) bookkeeping, {t:.1f} s"
                   f"{'' if full else f', extrapolated x{ds.n / count:.0f} to a full sweep'} (update_phi excluded); "
                   f"engine's latent pool ({P} entries); host {model}, {cores} of {ncpu} CPUs usable"),
    }
    O.set_threads(opt_threads)
    t, r, ost = run(0, -1, fast=2)
    t0 = time.perf_counter()
    O.update_phi(ds.codes, ds.attrisize, ds.v, ds.w, ost, st.copy())
    O.compute_loglikelihood(ds.codes, ds.attrisize, ost, fast=2)
    t_rest = time.perf_counter() - t0
    faithful["optimised"] = {
        "value": 1.0 / (t + t_rest), "unit": "sweeps/s", "cores": opt_threads, "kind": "port",
        "threads_source": threads_source,
        "sample": (f"one full step of the optimised oracle (oracle/src/fast.c, same trace): sweep {t:.2f} s "
                   f"(log-likelihoods on {opt_threads} threads, serial scan) + update_phi + compute_loglikelihood "
                   f"{t_rest:.2f} s; host {model}"),
    }
    return faithful


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 300 timed iterations (~0.05 s at C5): a 20-iteration window measured 10-20% below the
    # steady state (host pool and clocks still ramping); iteration 0's pool regeneration and
    # the next at iteration 1000 stay outside the timed window (reported under pool_generation)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c5")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--sm", action="store_true",
                    help="include the split-merge move in every step (t = r = 10, la:111-115)")
    ap.add_argument("--hig-logspace", choices=("auto", "on", "off"), default="auto",
                    help="HDPM_OPT_HIG_LOGSPACE (log-space 2F1, an extension): auto = on with --sm, where "
                         "clusters of thousands of members overflow the reference's series (it throws)")
    ap.add_argument("--init", choices=("truth", "one", "random20"), default="truth",
                    help="initial labels: the generator's ground truth (la:32-39, L = 0), one cluster (L = 1), or a "
                         "random assignment to 20 labels (la:31, the scripts' L = 20): the unconverged regime")
    ap.add_argument("--start-iter", type=int, default=0,
                    help="first iteration index (0: the warmup includes iteration 0's pool regeneration)")
    ap.add_argument("--phi", choices=("default", "auto", "host", "device"), default="default",
                    help="update_phi on the host job or the device (HDPM_OPT_PHI_DEVICE); auto = device for updates of "
                         ">= 4096 (cluster, attribute) items; default = the engine's (auto unless HDPM_PHI says otherwise)")
    ap.add_argument("--record", action="store_true",
                    help="the R driver's sampling phase: every iteration saved (thinning 1, la:139-153) -- K, labels, "
                         "centers and sigmas recorded through hdpm_iterations_record (the adapter's batches of 64, "
                         "buffers reused)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the optimised CPU baseline (0: every CPU this process may use, within the "
                         "share OMP_NUM_THREADS allots it -- 16 per GPU on the GPU box)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-csv", action="append", default=None,
                    help="rocprofv3 --pmc counter_collection CSV(s) with FETCH_SIZE / WRITE_SIZE of this workload "
                         "(separate passes); default: profiles/r01/pmc_{fetch,write}_<config>.csv when present")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank setup, barrier / max timing and the aggregate without the engine (CPU, gloo)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    ws, rank, local = dist_env()
    if ws != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    if args.dry_run:
        return dry_run(args, ws, rank, local)
    D = Dist(ws, rank, local)
    import split_and_merge_gibbs_sampling_amd as hd
    from split_and_merge_gibbs_sampling_amd.data import CONFIGS, config

    setup = rank_setup(rank, local)
    # torch's device context now, not between the warmup and the timed iterations (creating
    # it there idles the GPU and the host pool for a long stretch: a cold first timed window)
    cuda_sync()
    t_setup = time.perf_counter()
    ds = config(args.config, n=args.n)
    eng = hd.Engine(setup["device"])
    eng.set_data(ds.codes, ds.attrisize, ds.gamma, ds.v, ds.w)
    eng.set_seed(setup["seed"])
    hig_log = args.hig_logspace == "on" or (args.hig_logspace == "auto" and args.sm)
    if hig_log:
        eng.set_hig_logspace(True)
    if os.environ.get("HDPM_BENCH_HOST_POOL"):
        eng.set_debug(64)                        # sequential host pool generator (A/B runs)
    if args.phi != "default":
        eng.set_phi_device("auto" if args.phi == "auto" else args.phi == "device")
    phi_mode = eng.phi_mode
    L, ci = {"truth": (0, ds.truth), "one": (1, np.zeros(ds.n, np.int32)), "random20": (20, None)}[args.init]
    params = eng.chain_params(m=args.m, iterations=args.steps + args.warmup, L=L, burnin=0, neal8=True,
                              split_merge=args.sm, t=10, r=10)
    eng.init_chain(params, c_i=ci)               # la:27-77
    setup_s = time.perf_counter() - t_setup
    st_init = eng.stats()
    it = args.start_iter                         # iteration 0 regenerates the pool (la:123-129)
    eng.iterations(it, args.warmup)             # hdpm_iterations: the la:85-154 loop in one call
    it += args.warmup
    # the warmup's last iteration prepared the next sweep (its prepass on the device, its
    # speculative update_phi on the host pool): dropped here, so the timed window holds exactly
    # `steps` iterations of work, each started inside it (hdpm_drop_prepared)
    eng.drop_prepared()
    eng.synchronize()
    st0 = eng.stats()                            # + iteration 0's regeneration
    eng.reset_stats()
    if os.environ.get("HDPM_BENCH_DEBUG"):
        eng.set_debug(int(os.environ["HDPM_BENCH_DEBUG"]))    # A/B runs of engine variants (hdpm.h bits)
    if os.environ.get("HDPM_BENCH_TIMELINE"):
        eng.set_debug(32 | (64 if os.environ.get("HDPM_BENCH_HOST_POOL") else 0))                        # host timeline of the timed iterations (stderr)
    D.barrier()
    cuda_sync()
    # the adapter's batches (integration/hdpm_chain.hpp: 64 iterations per hdpm_iterations_record
    # call; a call boundary restarts the pipeline; HDPM_BENCH_RECORD_BATCH for A/B: 16 / 64 / 256
    # at C5 7,790 / 7,766 / 5,254 against 7,674 unrecorded, C4 5,904 / 6,063 / 5,818 against
    # 6,372, profiles/r06/record6c/)
    rec_batch = min(int(os.environ.get("HDPM_BENCH_RECORD_BATCH", "64")), args.steps)
    # (written through once here: the adapter's result buffers are reused, so their pages are
    # resident; a fresh calloc'd buffer would fault a page at a time inside the timed window)
    rec_buf = np.full((rec_batch, ds.n), -1, np.int32) if args.record else None
    t0 = time.perf_counter()
    if args.record:
        # every iteration saved (burnin 0, thinning 1): its K, labels, centers, sigmas, loglik
        for k0 in range(0, args.steps, rec_batch):
            eng.iterations_record(it + k0, min(rec_batch, args.steps - k0), out=rec_buf)
    else:
        eng.iterations(it, args.steps)
    it += args.steps
    eng.synchronize()
    cuda_sync()
    D.barrier()
    mine = time.perf_counter() - t0
    elapsed = D.max(mine)
    ranks = D.gather(dict(setup, ms_per_step=round(1e3 * mine / args.steps, 4)))
    st = eng.stats()
    c, cen, _ = eng.get_state()
    K = int(cen.shape[0])

    value = aggregate(ws, args.steps, elapsed)
    bpp = prepass_bytes_per_point(ds.d, int(ds.attrisize.max()), args.m)
    pre_ms = st["t_prepass_ms"]                  # HIP events around every 8th prepass launch
    achieved = (bpp * st["prepass_timed_points"] / 1e9) / (pre_ms / 1e3) if pre_ms > 0 else None
    launches = max(st["prepass_timed"], 1)
    traffic, traffic_src = None, None
    csvs = args.traffic_csv
    if csvs is None:
        csvs = [os.path.join(ROOT, "profiles", PMC_ROUND, f"pmc_{c}_{args.config}.csv") for c in ("fetch", "write")]
    csvs = [c for c in csvs if os.path.exists(c)]
    s_b, g_b, gshape = prepass_shape(ds.d, int(ds.attrisize.max()), args.m)
    if csvs and args.n is None:
        raw = traffic_from_csv(*csvs)
        if raw is not None:
            # calibrated: the streamed reads report half their bytes, the gathers FETCH_FACTOR
            fetch, write = raw
            stream = s_b * ds.n
            traffic = round(stream + (fetch - FETCH_FACTOR["stream16"] * stream) / FETCH_FACTOR[gshape] + write)
        traffic_src = [os.path.relpath(c, ROOT) for c in csvs] + ["profiles/r01/fetch_calib.log",
                                                                  "profiles/r02/pmc_fetch_calib.csv"]
    # the measured ceiling of this access mix: the replayed mix's time per point where
    # tools/fetch_calib.hip models the layout, else its streamed and gathered bytes at the
    # rates measured for those shapes on MI355X
    mix = MIX_US.get((gshape, packed_layout(ds.d, int(ds.attrisize.max()))[1], args.m))
    if mix:
        ceiling = bpp * mix[0] / (mix[1] * 1e3)
        ceiling_what = (f"the prepass's access mix ({s_b} B/point streamed, {g_b} B/point in {gshape[6:]}-B random "
                        f"gathers) replayed without its arithmetic: {mix[0]} points in {mix[1]} us "
                        f"(tools/fetch_calib.hip, profiles/r05/fetch_calib.log)")
    else:
        wb_ = bpp - s_b - g_b
        ceil_ns = s_b / RATE_GBPS["stream16"] + g_b / RATE_GBPS[gshape] + wb_ / RATE_GBPS["stream16"]
        ceiling = bpp / ceil_ns
        ceiling_what = (f"{s_b} B/point streamed + {g_b} B/point in {gshape[6:]}-B random gathers at the rates "
                        f"tools/fetch_calib.hip measured (profiles/r01/fetch_calib.log)")
    out = {
        "metric": "full Gibbs sweeps/sec (N-point reassign) at N=1M D=128; achieved HBM GB/s",
        "value": round(value, 4),
        "unit": "sweeps/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (data_generation.R model, numpy draws); R-compatible MT19937 chain stream",
        "config": {
            "workload": (f"{args.config}: {CONFIGS.get(args.config, {}).get('name', args.config)}, N={ds.n} D={ds.d} "
                         f"m={args.m}; one step = Neal-8 sweep + update_phi"
                         f"{' + split-merge (t=r=10)' if args.sm else ''} + compute_loglikelihood "
                         f"{'+ recording K / labels / centers / sigmas (thinning 1) ' if args.record else ''}"
                         f"(code/launcher.cpp:94-132), "
                         f"{ {'truth': 'ground-truth init', 'one': 'one-cluster init (L=1)', 'random20': 'random init, L=20'}[args.init]}"),
            "n": ds.n, "d": ds.d, "m": args.m, "K_final": K, "parallelism": f"replicas{ws}",
            "ranks": ranks,
            "sweep_effective_GBps": round(survey_sweep_bytes(ds.n, ds.d, args.m) * args.steps / elapsed / 1e9, 2),
            "setup_s": round(setup_s, 1),
            # device: prepass from its HIP-event-timed launches (x launches per step); exact rows
            # and resolver only when every kernel is timed (debug bit 9); host segments wall-clock
            "breakdown_ms_per_step": dict(
                {"t_prepass_ms": round(pre_ms / launches * st["rounds"] / args.steps, 4)},
                **{k: round(st[k] / args.steps, 4) for k in ("t_exact_ms", "t_resolve_ms") if st[k] > 0},
                **{k: round(st[k] / args.steps, 4) for k in ("t_stats_ms", "t_host_phi_ms", "t_rng_ms", "t_loglik_ms")},
                **{k: round(st[k] / args.steps, 4) for k in ("t_sm_ms", "t_sm_scan_ms", "t_sm_phi_ms", "t_sm_terms_ms")
                   if st["sm_moves"] > 0}),
            "exact_points_per_step": st["exact_points"] / args.steps,
            "listed_points_per_step": st["listed_points"] / args.steps,
            "moves_per_step": st["moves"] / args.steps,
            "split_merge": bool(args.sm),
            # restricted Gibbs samplers run as one device chain (split_merge.inl sm_chain), their
            # scans, and chains the host continued from their first unfinished step
            "sm_chain": ({k[9:]: int(st[k]) for k in ("sm_chain_runs", "sm_chain_scans", "sm_chain_resumes")}
                         if args.sm else None),
            "record": ({"labels_mirrored": int(st["labels_mirrored"]), "labels_downloaded": int(st["labels_downloaded"])}
                       if args.record else None),
            "hig_logspace": hig_log,
            "rounds_per_step": st["rounds"] / args.steps,
            # next sweeps enqueued while the update was drawn / run (engine pre_enqueue), and
            # update stream slices found in a copy made an iteration ahead
            "pipeline": {"enqueued": st["pipe_enqueued"], "ran": st["pipe_runs"],
                         "slice_lookahead_hits": st["phi_lookahead_hits"]},
            "rng_windows": {"launched": st["rng_windows"], "fresh": st["rng_windows_fresh"]},
            # recoveries inside the timed window (each keeps the chain; a non-zero count means a
            # slow path ran): device-wide resolver give-ups, restricted scans that gave up on many
            # CUs, sweeps enqueued ahead and re-run ungated, device update_phi handed to the host
            "fallbacks": {k: int(st[k]) for k in ("fpg_aborts", "sm_wide_fallbacks", "pipe_recovered",
                                                  "phi_device_fallbacks", "phi_fallback_status_mask",
                                                  "pipe_desync")},
            "update_phi": {"mode": phi_mode, "where": "device" if st["phi_device_calls"] > 0 else "host",
                           "device_calls": int(st["phi_device_calls"]), "spec_used": int(st["phi_dspec_used"]),
                           "fast_calls": int(st["phi_fast_calls"]), "fast_handbacks": int(st["phi_fast_handbacks"]),
                           "chained": int(st["phi_chain_used"]), "chain_dropped": int(st["phi_chain_dropped"]),
                           "state_direct": int(st["phi_state_direct"]), "device_go": int(st["pipe_auto"])},
            "pool_generation": {"init": pool_report(st_init, ds.n * args.m),
                                "regeneration": pool_report(stats_diff(st0, st_init), ds.n * args.m)},
        },
        "roofline": {
            "bound": "hbm",
            "kernel": prepass_kernel_name(ds.d, int(ds.attrisize.max())),
            "achieved": None if achieved is None else round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": None if achieved is None else round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "measured_ceiling": {"GBps": round(ceiling, 1),
                                 "frac": None if achieved is None else round(achieved / ceiling, 4),
                                 "what": ceiling_what},
            "bytes_per_point": bpp,
            "avg_launch_ms": round(pre_ms / launches, 4),
        },
        "cpu_baseline": None,
    }
    regen = out["config"]["pool_generation"]["regeneration"]
    if regen:
        # the la:85-154 loop rate: the timed step plus the pool regeneration of every 1000th
        # iteration (la:123-129, outside the timed window) amortised over its cadence
        out["config"]["full_loop"] = {
            "value": round(ws * 1e3 / (1e3 * elapsed / args.steps + regen["amortised_ms_per_iteration"]), 2),
            "unit": "sweeps/s", "what": "value with the latent pool regeneration (la:123-129) amortised per iteration"}
    # byte models: what the certified sweep moves vs SURVEY 8(d)'s direct design
    out["config"]["byte_model"] = {
        "certified_prepass_bytes_per_sweep": bpp * ds.n,
        "survey_8d_bytes_per_sweep": survey_sweep_bytes(ds.n, ds.d, args.m),
        "note": "the sweep proves 'stay' from bounds for most points (DESIGN.md 4.3-4.4) and moves the prepass bytes; "
                "SURVEY 8(d)'s N(D(2+9m)+8) is the direct design's traffic and is not the roofline of this path"}
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        # the optimised oracle's threads: --cpu-threads, else this process's CPU share
        # (OMP_NUM_THREADS: 16 per GPU on the GPU box, whose nproc counts the whole host),
        # else every usable CPU -- the source is recorded in the line
        usable = host_cpu()[1]
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        if args.cpu_threads:
            thr, src = args.cpu_threads, "--cpu-threads"
        elif share > 0:
            thr, src = min(usable, share), f"OMP_NUM_THREADS={share} (the GPU's CPU share), {usable} usable"
        else:
            thr, src = usable, "every usable CPU (OMP_NUM_THREADS unset)"
        out["cpu_baseline"] = cpu_baseline(ds, eng, args.m, args.cpu_baseline_seconds, thr, src)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    D.close()


def dry_run(args, ws, rank, local):
    """The multi-rank harness without the engine: per-rank setup, barrier, a stand-in step
    loop, max over ranks, gather and the aggregate line (tests/test_dist.py runs it on gloo)."""
    D = Dist(ws, rank, local, backend="gloo")
    setup = rank_setup(rank, local)
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))
    D.barrier()
    mine = time.perf_counter() - t0
    elapsed = D.max(mine)
    ranks = D.gather(dict(setup, ms_per_step=round(1e3 * mine / args.steps, 4)))
    if rank == 0:
        print(json.dumps({"metric": "dry run", "value": aggregate(ws, args.steps, elapsed), "unit": "steps/s",
                          "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(1e3 * elapsed / args.steps, 4), "scaling": "weak",
                          "config": {"parallelism": f"replicas{ws}", "ranks": ranks}}), flush=True)
    D.close()


def stats_diff(a, b):
    return {k: a[k] - b[k] for k in a}


def pool_report(st, P):
    """Latent pool generation (la:74-77 in init_chain; regenerated at iteration 0 and every
    1000 iterations, la:123-129) as timed by the engine: wall ms per call, its phases, and
    the cost per iteration amortised over the 1000-iteration cadence."""
    calls = int(st["pool_calls"])
    if calls == 0:
        return None
    ms = st["t_pool_ms"] / calls
    return {
        "entries": P, "device": st["pool_device_calls"] == calls, "ms_per_call": round(ms, 2),
        "phases_ms": {k[7:-3]: round(st[k] / calls, 2) for k in
                      ("t_pool_mt_ms", "t_pool_accept_ms", "t_pool_parse_ms", "t_pool_values_ms")},
        "amortised_ms_per_iteration": round(ms / 1000, 4),
    }


def traffic_from_csv(*paths):
    """Per-launch (FETCH_SIZE, WRITE_SIZE) bytes of k_prepass from rocprofv3 --pmc
    counter_collection CSVs (one pass per counter), as reported (KiB -> bytes); the caller
    applies the calibration (FETCH_FACTOR)."""
    import csv
    tot = {"FETCH_SIZE": [0.0, set()], "WRITE_SIZE": [0.0, set()]}
    for path in paths:
        for row in csv.DictReader(open(path)):
            if "k_prepass" not in row.get("Kernel_Name", ""):
                continue
            name = row.get("Counter_Name")
            if name in tot:
                tot[name][0] += float(row.get("Counter_Value", 0))
                tot[name][1].add((path, row.get("Dispatch_Id")))
    per = {k: (v / len(ids) if ids else None) for k, (v, ids) in tot.items()}
    if per["FETCH_SIZE"] is None:
        return None
    return per["FETCH_SIZE"] * 1024, (per["WRITE_SIZE"] or 0.0) * 1024


if __name__ == "__main__":
    main()
