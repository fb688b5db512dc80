#!/usr/bin/env python3
"""Refresh the committed PMC summaries from one profiling session
(tools/gpu_round2.sh prof pmc): generation (DeepWalk MH, node2vec MH warm) and
the configs[2] streaming kernels.  HBM bytes per launch = 2 x FETCH_SIZE
(gfx950 counts 64 B per 128-B request, MI355X_MICROARCH.md §HBM) + WRITE_SIZE,
both KiB, from separate passes; durations from the kernel trace of the
default bench (timed launches only for generation).

    python tools/pmc_session.py <session dir under profiles/r02>
"""
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(path, kernel, name, skip=0):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    return v[skip:]


def durations(path, kernel):
    rows = sorted((r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]),
                  key=lambda r: int(r["Dispatch_Id"]))
    return [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]


def summary(kernel, fetch, write, trace, skip=0, dur_slice=slice(None), algorithmic=None):
    f = counter(fetch, kernel, "FETCH_SIZE", skip)
    w = counter(write, kernel, "WRITE_SIZE", skip)
    d = durations(trace, kernel)[dur_slice]
    fr, wb, ns = statistics.mean(f) * 1024, statistics.mean(w) * 1024, statistics.mean(d)
    return {"kernel": kernel, "launches": {"fetch_pass": len(f), "write_pass": len(w), "skipped_first": skip,
                                           "trace": len(d)},
            "fetch_size_bytes_raw": fr, "fetch_bytes_corrected": 2 * fr, "write_bytes": wb,
            "hbm_bytes_per_launch": 2 * fr + wb, "avg_kernel_ns_kernel_trace": ns,
            "effective_GBps": (2 * fr + wb) / ns, "algorithmic_bytes_per_launch": algorithmic,
            "sources": [os.path.relpath(p, REPO) for p in (fetch, write, trace)]}


def main():
    d = os.path.join(REPO, sys.argv[1])
    tr = os.path.join(d, "bench_kernel_trace_filtered.csv")
    gf, gw = os.path.join(d, "pmc_gen_fetch.csv"), os.path.join(d, "pmc_gen_write.csv")
    sf, sw = os.path.join(d, "pmc_str_fetch.csv"), os.path.join(d, "pmc_str_write.csv")
    out = {
        # the bench's 2 warmup + 5 timed DeepWalk launches come first; the configs[2] generations follow
        "r02_gen_deepwalk_mh_s22": summary("k_walk<0, false>", gf, gw, tr, dur_slice=slice(2, 7),
                                           algorithmic=3297052360 * 24),
        # node2vec: the first launch also fills the anchor cache; warm launches only
        "r02_gen_node2vec_mh_s22": summary("k_walk<1, false>", gf, gw, tr, skip=1, dur_slice=slice(1, 4)),
        "r02_streaming_s22": {
            "rewalk_point_scan": summary("k_rewalk_chunked<false", sf, sw, tr),
            "deterministic_rewalk_copy": summary("k_rewalk_chunked<true", sf, sw, tr),
            "in_edge_scan": summary("k_patch_in_edges", sf, sw, tr),
            "note": "configs[2] deterministic stream (bench.py --det-rewalk-batches 3 for the PMC passes; "
                    "the default bench under --kernel-trace for durations)"},
    }
    for tag, v in out.items():
        json.dump(v, open(os.path.join(REPO, "profiles", f"pmc_{tag}.json"), "w"), indent=1)
        print(tag, json.dumps(v)[:300])


if __name__ == "__main__":
    main()
