#!/usr/bin/env python3
"""Summarise rocprofv3 outputs for one kernel into profiles/.

    python tools/pmc_summary.py --tag gen_deepwalk_mh_s22 --kernel "k_walk<wharf::VRec32, 0, false, false>" \
        --fetch gpurun_out/pmc_fetch/run_counter_collection.csv \
        --write gpurun_out/pmc_write/run_counter_collection.csv \
        --stats gpurun_out/prof_gen/run_kernel_stats.csv --round r01

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB, collected in separate passes; on gfx950 FETCH_SIZE
counts 64 B per TCC_EA0_RDREQ while the requests are 128 B, so the read side
is doubled (the guide's correction for wide reads; our gathers miss whole
lines, so the same factor is applied and the raw value is kept beside it).
"""
import argparse
import csv
import json
import os
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel, counter, skip=0):
    vals = []
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals[skip:]


def trace_avg_ns(path, kernel, skip=0, take=0):
    """average duration from a --kernel-trace csv, dispatch order, first `skip` launches dropped
    (then the next `take`, if given: the bench's timed steps, not its later configs[2] launches)"""
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    rows = rows[skip:skip + take] if take else rows[skip:]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    return statistics.mean(d) if d else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--stats", default=None, help="rocprofv3 --stats kernel_stats.csv")
    ap.add_argument("--trace", default=None, help="rocprofv3 --kernel-trace kernel_trace.csv (with --skip)")
    ap.add_argument("--skip", type=int, default=0,
                    help="drop the first launches (node2vec: the first generation also initialises every anchor)")
    ap.add_argument("--trace-skip", type=int, default=None, help="launches to drop in the trace (default: --skip)")
    ap.add_argument("--trace-take", type=int, default=0, help="launches to keep in the trace after the skipped ones")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    a = ap.parse_args()
    f = per_launch(a.fetch, a.kernel, "FETCH_SIZE", a.skip)
    w = per_launch(a.write, a.kernel, "WRITE_SIZE", a.skip)
    avg_ns = None
    if a.trace:
        avg_ns = trace_avg_ns(a.trace, a.kernel, a.skip if a.trace_skip is None else a.trace_skip, a.trace_take)
    else:
        for r in csv.DictReader(open(a.stats)):
            if a.kernel in r["Name"]:
                avg_ns = float(r["AverageNs"])
                break
    fetch_raw = statistics.mean(f) * 1024
    write = statistics.mean(w) * 1024
    out = {
        "kernel": a.kernel,
        "launches": {"fetch_pass": len(f), "write_pass": len(w), "skipped_first": a.skip},
        "fetch_size_bytes_raw": fetch_raw,
        "fetch_bytes_corrected": 2 * fetch_raw,
        "write_bytes": write,
        "hbm_bytes_per_launch": 2 * fetch_raw + write,
        "avg_kernel_ns_kernel_trace": avg_ns,
        "effective_GBps": (2 * fetch_raw + write) / avg_ns if avg_ns else None,
        "algorithmic_bytes_per_launch": a.algorithmic_bytes,
        "sources": [os.path.relpath(p, REPO) for p in (a.fetch, a.write, a.trace or a.stats)],
    }
    dst = os.path.join(REPO, "profiles", f"pmc_{a.tag}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
