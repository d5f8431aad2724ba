"""Per-kernel statistics from a rocprofv3 --kernel-trace database (rocpd sqlite):
count, total, mean, median, max duration (us) and grid, plus a timeline of the last N
dispatches.  Usage: python tools/kstats.py <run_results.db> [--last N] [--csv out.csv]"""
import argparse
import sqlite3
import statistics


def load(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end, grid_x, workgroup_x, stream_id, lds_size from kernels order by start").fetchall()
    return [(r[0].split("(")[0], r[1], r[2], r[3], r[4], r[5], r[6]) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N dispatches (setup)")
    a = ap.parse_args()
    rows = load(a.db)[a.skip:]
    by = {}
    for name, s, e, g, w, st, lds in rows:
        by.setdefault(name, []).append((e - s) / 1e3)
    out = []
    for name, v in by.items():
        out.append((sum(v), name, len(v), sum(v) / len(v), statistics.median(v), max(v)))
    out.sort(reverse=True)
    print(f"{'kernel':60s} {'n':>6s} {'total_us':>10s} {'mean':>8s} {'median':>8s} {'max':>8s}")
    for tot, name, n, mean, med, mx in out:
        print(f"{name[:60]:60s} {n:6d} {tot:10.1f} {mean:8.2f} {med:8.2f} {mx:8.2f}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("Name,Calls,TotalDurationUs,AverageUs,MedianUs,MaxUs\n")
            for tot, name, n, mean, med, mx in out:
                f.write(f'"{name}",{n},{tot:.3f},{mean:.3f},{med:.3f},{mx:.3f}\n')
    if a.last:
        t0 = rows[-a.last][1]
        for name, s, e, g, w, st, lds in rows[-a.last:]:
            print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} s{st} g{g}/{w} lds{lds} {name[:70]}")


if __name__ == "__main__":
    main()
