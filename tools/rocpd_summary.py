#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 rocpd database (rocprofv3 7.x writes
run_results.db by default): per-kernel stats, and the kernels between two
markers in launch order, e.g. one update batch.

    python tools/rocpd_summary.py <db> [--stats] [--timeline FIRST_KERNEL_SUBSTR --count N]
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*$", "", name)
    return name.replace("void ", "").replace("wharf::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--timeline", default=None, help="print dispatches from the k-th occurrence of this kernel")
    ap.add_argument("--occurrence", type=int, default=1)
    ap.add_argument("--count", type=int, default=60)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    kname = "name" if "name" in cols else "kernel_name"
    rows = con.execute(f"select {kname}, start, end from kernels order by start").fetchall()
    if a.stats:
        agg = {}
        for n, s, e in rows:
            d = agg.setdefault(short(n), [0, 0.0])
            d[0] += 1
            d[1] += (e - s) / 1e6
        tot = sum(v[1] for v in agg.values())
        print(f"{'kernel':70s} {'calls':>6s} {'total ms':>10s} {'avg ms':>9s} {'%':>6s}")
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{k[:70]:70s} {c:6d} {t:10.3f} {t / c:9.4f} {100 * t / tot:6.2f}")
    if a.timeline:
        occ = 0
        start = None
        for i, (n, s, e) in enumerate(rows):
            if a.timeline in n:
                occ += 1
                if occ == a.occurrence:
                    start = i
                    break
        if start is None:
            print("marker not found")
            return
        t0 = rows[start][1]
        for n, s, e in rows[start:start + a.count]:
            print(f"{(s - t0) / 1e6:9.3f} ms  {(e - s) / 1e6:8.4f} ms  {short(n)[:90]}")


if __name__ == "__main__":
    main()
