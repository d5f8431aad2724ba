"""Multi-process timing harness of bench.py (replicas) on CPU/gloo.

bench.py runs one independent chain per rank; the only collectives are the timing barrier
and the max over ranks.  These tests run that harness with world_size 2 over gloo.
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    ws_, rank_, local_ = bench.dist_env()
    D = bench.Dist(ws_, rank_, local_, backend="gloo")
    setup = bench.rank_setup(rank_, local_)
    D.barrier()
    mx = D.max(float(10 * (rank + 1)))
    ranks = D.gather(setup)
    D.barrier()
    q.put((rank, mx, ws_, [(r["rank"], r["device"], r["seed"]) for r in ranks], bench.aggregate(ws_, 7, mx)))
    D.close()


def test_dist_env_defaults(monkeypatch):
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert bench.dist_env() == (1, 0, 0)
    D = bench.Dist(1, 0, 0)
    D.barrier()
    assert D.max(3.5) == 3.5
    D.close()


def test_gloo_world2_barrier_and_max():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0], codes
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert [r[0] for r in res] == [0, 1]
    assert all(r[1] == 20.0 for r in res)       # max over ranks reaches every rank
    assert all(r[2] == 2 for r in res)
    # every rank sees every rank's setup: GPU = local rank, chain seed 1 + rank
    assert all(r[3] == [(0, 0, 1), (1, 1, 2)] for r in res)
    assert all(r[4] == 2 * 7 / 20.0 for r in res)


def _clean_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE", "GROUP_RANK"):
        env.pop(k, None)
    return env


def test_bench_gpus2_starts_two_ranks():
    """`python bench.py --gpus 2` (no launcher) starts two rank processes and prints ONE
    aggregate line with n_gpus 2 (the dry run: the same harness without the engine)."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "0",
                        "--dry-run"], capture_output=True, text=True, timeout=300, env=_clean_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "replicas2"
    ranks = sorted(out["config"]["ranks"], key=lambda x: x["rank"])
    assert [(x["rank"], x["device"], x["seed"]) for x in ranks] == [(0, 0, 1), (1, 1, 2)]
    # aggregate = all ranks' steps over the slowest rank's time
    assert abs(out["value"] * out["ms_per_step"] / 1e3 - 2.0) < 1e-3
    assert out["ms_per_step"] >= max(x["ms_per_step"] for x in ranks) - 1e-3


def test_bench_rejects_gpus_world_size_mismatch():
    import subprocess
    env = _clean_env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_helpers():
    import bench
    wb, W, bw = bench.packed_layout(128, 4)
    assert (wb, W, bw) == (2, 4, 16)
    assert bench.prepass_bytes_per_point(128, 4, 3) == 8 * W + 16 + 4 + 3 * 64 + 12     # 64-B heads
    wb, W, bw = bench.packed_layout(784, 6)                                          # wide: 448-B heads
    assert (wb, W) == (4, 52)
    assert bench.head_layout(784, 6) == (True, 56, False)
    assert bench.prepass_bytes_per_point(784, 6, 3) == 8 * W + 16 + 4 + 3 * 448 + 12
    wb, W, bw = bench.packed_layout(2100, 2)                                         # Ws = 33: generic, full records
    assert bench.head_layout(2100, 2)[0] is False
    assert bench.prepass_bytes_per_point(2100, 2, 3) == 8 * W + 16 + 4 + 3 * 8 * bw + 12
    assert bench.survey_sweep_bytes(10, 4, 1) == 10 * (4 * 11 + 8)


@pytest.mark.parametrize("rows", [[("k_prepass<2,4>", 1, "FETCH_SIZE", 100.0), ("k_prepass<2,4>", 1, "WRITE_SIZE", 10.0),
                                   ("k_prepass<2,4>", 2, "FETCH_SIZE", 300.0), ("k_prepass<2,4>", 2, "WRITE_SIZE", 30.0),
                                   ("k_resolve", 3, "FETCH_SIZE", 5.0)]])
def test_traffic_from_csv(tmp_path, rows):
    import bench
    p = tmp_path / "c.csv"
    import csv
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for k, d, n, v in rows:
            w.writerow([d, k, n, v])
    # 400 KiB fetched and 40 KiB written over 2 dispatches (as reported)
    assert bench.traffic_from_csv(str(p)) == (200 * 1024, 20 * 1024)
    # one file per counter pass
    pf, pw = tmp_path / "f.csv", tmp_path / "w.csv"
    import csv
    for path, name, vals in ((pf, "FETCH_SIZE", (100.0, 300.0)), (pw, "WRITE_SIZE", (10.0, 30.0))):
        with open(path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            for d, v in enumerate(vals):
                w.writerow([d, "k_prepass<2,2>", name, v])
    assert bench.traffic_from_csv(str(pf), str(pw)) == (200 * 1024, 20 * 1024)
    # the C5 prepass shape: 52 B/point streamed, 3 x 64-B head gathers
    assert bench.prepass_shape(128, 4, 3) == (52, 192, "gather64")
    assert bench.prepass_shape(784, 6, 3) == (436, 3 * 448, "gather448g")
    assert bench.prepass_shape(2100, 2, 3)[2] == "gather128"
