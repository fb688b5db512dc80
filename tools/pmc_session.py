#!/usr/bin/env python3
"""Refresh the committed rocprofv3 records from one profiling session
(`OUTDIR=gpurun_out/r4 tools/gpu_session.sh prof pmc`): copies the kernel statistics, a filtered
kernel trace and the PMC passes into profiles/<round>/rocprof/, and writes the
per-launch HBM summaries bench.py reads (profiles/pmc_<round>_*.json).

HBM bytes per launch = 2 x FETCH_SIZE (gfx950 counts 64 B per 128-B read
request, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both KiB, from separate passes.
Durations come from the kernel trace of the default bench run under the
profiler (timed launches only for generation: dispatch order 3-7).

    python tools/pmc_session.py gpurun_out/r4 r04
"""
import csv
import json
import os
import re
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = re.compile(r"k_walk|k_rewalk|k_patch_in_edges|k_patch_rev|k_anchor|k_det_suffix|k_park")


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
    if not f or not w or not d:
        return {"kernel": kernel, "missing": True}
    fr, wb, ns = statistics.mean(f) * 1024, statistics.mean(w) * 1024, statistics.mean(d)
    return {"kernel": kernel, "launches": {"fetch_pass": len(f), "write_pass": len(w), "skipped_first": skip,
                                           "trace": len(d)},
            "fetch_size_bytes_raw": fr, "fetch_bytes_corrected": 2 * fr, "write_bytes": wb,
            "hbm_bytes_per_launch": 2 * fr + wb, "avg_kernel_ns_kernel_trace": ns,
            "effective_GBps": (2 * fr + wb) / ns, "algorithmic_bytes_per_launch": algorithmic,
            "sources": [os.path.relpath(p, REPO) for p in (fetch, write, trace)]}


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main():
    sess, rnd = os.path.join(REPO, sys.argv[1]), sys.argv[2]
    out_dir = os.path.join(REPO, "profiles", rnd, "rocprof")
    os.makedirs(out_dir, exist_ok=True)
    prof = os.path.join(sess, "prof_bench")
    shutil.copy(os.path.join(prof, "run_kernel_stats.csv"), os.path.join(out_dir, "bench_kernel_stats.csv"))
    tr = os.path.join(out_dir, "bench_kernel_trace_filtered.csv")
    with open(os.path.join(prof, "run_kernel_trace.csv")) as fi, open(tr, "w", newline="") as fo:
        rd = csv.DictReader(fi)
        wr = csv.DictWriter(fo, fieldnames=rd.fieldnames)
        wr.writeheader()
        for r in rd:
            if KEEP.search(r["Kernel_Name"]):
                wr.writerow(r)
    pmc = {}
    for name in ("pmc_gen_fetch", "pmc_gen_write", "pmc_str_fetch", "pmc_str_write"):
        src = os.path.join(sess, name, "run_counter_collection.csv")
        if os.path.exists(src):
            pmc[name] = os.path.join(out_dir, f"{name}.csv")
            shutil.copy(src, pmc[name])
    line = bench_line(os.path.join(sess, "prof_bench.log"))
    shutil.copy(os.path.join(sess, "prof_bench.log"), os.path.join(out_dir, "prof_bench.log"))
    steps = line["config"]["transitions_per_step"]
    gen = summary("k_walk<0, false, false", pmc["pmc_gen_fetch"], pmc["pmc_gen_write"], tr, dur_slice=slice(2, 7),
                  algorithmic=steps * 24)
    gen["bench_line_avg_kernel_ms_same_run"] = line["roofline"]["avg_kernel_ms"]
    gen["bench_line_value_same_run"] = line["value"]
    out = {
        f"{rnd}_gen_deepwalk_mh_s22": gen,
        # node2vec: the first launch also fills the anchor cache; warm launches only
        f"{rnd}_gen_node2vec_mh_s22": summary("k_walk<1, false, false", pmc["pmc_gen_fetch"], pmc["pmc_gen_write"], tr,
                                              skip=1, dur_slice=slice(1, 4)),
    }
    str_trace = os.path.join(sess, "prof_str", "run_kernel_trace.csv")
    if "pmc_str_fetch" in pmc and os.path.exists(str_trace):
        trs = os.path.join(out_dir, "str_kernel_trace_filtered.csv")
        with open(str_trace) as fi, open(trs, "w", newline="") as fo:
            rd = csv.DictReader(fi)
            wr = csv.DictWriter(fo, fieldnames=rd.fieldnames)
            wr.writeheader()
            for r in rd:
                if KEEP.search(r["Kernel_Name"]):
                    wr.writerow(r)
        out[f"{rnd}_streaming_s22"] = {
            "rewalk_point_scan": summary("k_rewalk_scan_", pmc["pmc_str_fetch"], pmc["pmc_str_write"], trs),
            "deterministic_rewalk_copy": summary("k_rewalk_chunked<true", pmc["pmc_str_fetch"], pmc["pmc_str_write"], trs),
            "in_edge_scan": summary("k_patch_in_edges", pmc["pmc_str_fetch"], pmc["pmc_str_write"], trs),
            "in_edge_records": summary("k_patch_rev", pmc["pmc_str_fetch"], pmc["pmc_str_write"], trs),
            "note": "configs[2] deterministic stream (bench.py --det-rewalk-batches 3): PMC passes and the "
                    "durations of the same launches from a --kernel-trace run of the same command"}
    for tag, v in out.items():
        json.dump(v, open(os.path.join(REPO, "profiles", f"pmc_{tag}.json"), "w"), indent=1)
        print(tag, json.dumps(v)[:400])


if __name__ == "__main__":
    main()
