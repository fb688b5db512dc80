#!/usr/bin/env python3
"""Headline benchmark: MH walk-steps/s for initial walk generation on the
com-orkut-sized RMAT graph (BASELINE.json configs[1]: DeepWalk MH sampler,
10 walks/vertex, length 80), plus the re-walk latency of 10k-edge batches.

    python bench.py [--gpus N --steps K --warmup W]

N > 1 is launched by torch.distributed.run, one rank per GPU: every rank holds
the replicated CSR and owns a contiguous start-vertex range of the walks
(balanced by non-isolated start vertices); the timed step has no collective.

A "step" = one generate_initial_random_walks() over the whole graph (all
ranks' shards).  value = transitions appended by all ranks per second.

Scaling (--scaling, default weak): every rank keeps configs[1]'s per-GPU
workload ON configs[1]'s graph: the scale-22 RMAT graph is replicated, the
job generates 10 x N walks per vertex (rank g owns the start-vertex range g of
N, i.e. 4.19 M / N vertices x 10 N rounds = configs[1]'s 41.9 M walks), so the
per-GPU work and the graph stay configs[1]'s as N grows.  At N > 1 the line
also carries `strong_scaling`: configs[1] exactly (10 walks per vertex) split N
ways, value = its transitions / max-over-ranks time.  --scaling strong makes
that the headline.

Sub-records on rank 0 (same run): `mh_node2vec` (configs[4]'s model, p=.5
q=2 WEIGHT, on the configs[1] graph: first and warm generation, a configs[2]
re-walk stream), `rewalk_latency_10k_batch[_deterministic]` (configs[2]),
`streaming_rooflines` (rewalk-point scan, deterministic suffix copy, CSR move)
and `per_gpu_of_8`: the per-GPU work of configs[3] and configs[4] on 8 GPUs
(full graph, walk shard 0 of 8) run on this GPU, with configs[3]'s all-walks
1-GPU time beside it.  The box's random-gather rate is probed 3 times before the
timed region (`roofline.gather_ceiling`).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_STEP_DEEPWALK = 24     # offsets/deg record 16 B + 1 target 4 B + 1 output 4 B
# node2vec MH as built: 32-B edge record with the anchor entry + one 32-B has_edge bucket
# + 4-B output (SURVEY 8(d)'s 44 + 4*ceil(log2 deg) prices the reference's binary search instead)
BYTES_PER_STEP_NODE2VEC = 68
ORKUT_EDGES = 117_185_083        # com-orkut undirected edge count (configs[1])


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--samples", type=int, default=ORKUT_EDGES)
    p.add_argument("--seed", type=int, default=2)
    p.add_argument("--wpv", type=int, default=10)
    p.add_argument("--length", type=int, default=80)
    p.add_argument("--model", choices=["deepwalk", "node2vec"], default="deepwalk")
    p.add_argument("--paramP", type=float, default=0.5)
    p.add_argument("--paramQ", type=float, default=2.0)
    p.add_argument("--det", action="store_true", help="deterministic mode instead of MH")
    p.add_argument("--rewalk-batches", type=int, default=50, help="10k-edge insert batches (configs[2])")
    p.add_argument("--det-rewalk-batches", type=int, default=10,
                   help="the same stream in deterministic mode (DeepWalk MH runs only; 0 = off)")
    p.add_argument("--stream-samples", type=int, default=43_000_000, help="configs[2] base graph undirected samples")
    p.add_argument("--cpu-baseline", choices=["auto", "reference", "port", "off"], default="auto")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--cpu-timeout", type=int, default=300)
    p.add_argument("--cpu-length", type=int, default=24,
                   help="walk length of the bounded reference CPU sample (~15-25 s on 16 host threads)")
    p.add_argument("--cpu-scale", type=int, default=17,
                   help="RMAT scale of the same-shape CPU baseline (configs[1]'s density, wpv x L of the workload; "
                        "0 = off)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    p.add_argument("--n2v-steps", type=int, default=3, help="node2vec warm generations of the mh_node2vec record (0 = off)")
    p.add_argument("--n2v-rewalk-batches", type=int, default=5, help="configs[2] batches of the mh_node2vec record")
    p.add_argument("--gather-probes", type=int, default=3, help="tools/gather_roof runs before the timed region")
    p.add_argument("--per-gpu-of-8", type=int, default=1,
                   help="configs[3] / configs[4]: the per-GPU work of their 8-GPU runs on this GPU (0 = off)")
    p.add_argument("--per8-batches", type=int, default=5, help="update batches per per_gpu_of_8 case")
    p.add_argument("--per8-cases", default="", help="comma list of per_gpu_of_8 case names to run ('' = all; A/B runs)")
    p.add_argument("--jobs", default="configs3,configs4",
                   help="at N > 1: BASELINE's 8-GPU jobs run on the ranks of this run (comma list; '' = none)")
    p.add_argument("--job-batches", type=int, default=5, help="update batches per job (configs[4]: insert+delete pairs)")
    p.add_argument("--job-scale-delta", type=int, default=0,
                   help="rehearsals: RMAT scale of the jobs shifted by this (samples scaled alike), e.g. -4")
    p.add_argument("--job-gather", type=int, default=1, help="time the jobs' bounded corpus all-gatherv (0 = off)")
    p.add_argument("--job-one-gpu", type=int, default=1,
                   help="configs[3] job: rank 0 also runs every walk on its GPU (the 1-GPU time) (0 = off)")
    p.add_argument("--job-shards", choices=["blocks", "ranges"], default="blocks",
                   help="jobs' walk shards: vertex blocks dealt round-robin (balanced mix) or contiguous ranges")
    p.add_argument("--job-block-bits", type=int, default=16, help="block size (log2 vertices) of --job-shards blocks")
    p.add_argument("--gather-chunk-bytes", type=int, default=4 << 30,
                   help="device buffer of the bounded corpus gather (all ranks' rows of one chunk)")
    p.add_argument("--gather-check", type=int, default=1,
                   help="second gather pass checking the checksum of checksums (0 = off)")
    p.add_argument("--init-dist", action="store_true",
                   help="initialise torch.distributed even at N = 1 (one rank: runs the RCCL leg -- device "
                        "collectives, the chunked gather, the 8-GPU jobs -- on a one-GPU box)")
    return p.parse_args()


def balanced_shards(deg: np.ndarray, parts: int):
    from dynamicgraphrepresentationlearning_amd.distributed import balanced_shards as bs
    return bs(deg, parts)


def measure_gather_ceiling(runs: int = 3, gib: float = 3.48):
    """The chip's dependent random 16-B gather rate with the walk kernel's shape
    (41.9 M lanes x 79 dependent gathers from a 3.5 GiB table), measured on this
    box by tools/gather_roof `runs` times BEFORE the timed region, on an idle
    GPU (boxes differ by up to ~10 %; round 2 probed after ~55 s of load and got
    a rate the kernel then beat by 10 %).  None when the probe is not built."""
    exe = os.path.join(REPO, "tools", "gather_roof")
    if not os.access(exe, os.X_OK):
        return None
    rates = []
    for _ in range(runs):
        try:
            r = subprocess.run([exe, f"{gib:.2f}", "coarse", "dep"], capture_output=True, text=True, timeout=180)
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    rates.append(float(json.loads(line)["Ggathers_per_s"]))
        except (subprocess.SubprocessError, ValueError, KeyError, OSError):
            pass
    return rates or None


def gather_ceiling(steps_per_s: float, live, matched=None):
    """The generation kernel against the box's random-gather rate (one dependent
    16-B gather per step), probed before the timed region: min / max of the
    probes and the kernel's rate as a fraction of each.  A fraction above 1 is
    probe noise, not headroom: the probe is a yardstick for the box, the
    roofline is `roofline.frac`."""
    if not live:
        return None
    lo, hi = min(live), max(live)
    rec = {"Ggathers_per_s_min": round(lo, 2), "Ggathers_per_s_max": round(hi, 2), "probes": [round(x, 2) for x in live],
           "frac_of_min": round(steps_per_s / (lo * 1e9), 4), "frac_of_max": round(steps_per_s / (hi * 1e9), 4),
           "source": "tools/gather_roof 3.48 coarse dep (16-B records, the box's yardstick), this box, before the "
                     "timed region"}
    if matched and matched.get("probes"):
        mp = matched["probes"]
        rec["table_matched"] = {"table_GiB": matched["table_GiB"], "probes": [round(x, 2) for x in mp],
                                "frac_of_min": round(steps_per_s / (min(mp) * 1e9), 4),
                                "frac_of_max": round(steps_per_s / (max(mp) * 1e9), 4),
                                "source": "tools/gather_roof <the graph's edge-record table size> coarse dep, after "
                                          "the graph is built, before the timed region"}
    return rec


PMC_ROUNDS = ("r06_", "r05_", "r04_", "r03_", "r02_", "")   # newest round's rocprofv3 summary first


def load_traffic(tag: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (newest
    round first), and the file it came from."""
    for pre in PMC_ROUNDS:
        rel = os.path.join("profiles", f"pmc_{pre}{tag}.json")
        path = os.path.join(REPO, rel)
        if os.path.exists(path):
            try:
                return json.load(open(path)).get("hbm_bytes_per_launch"), f"{rel} (rocprofv3 PMC pass)"
            except Exception:
                pass
    return None, None


def load_requests(tag: str):
    """L2 (TCC) requests per step of the kernel from the committed rocprofv3 PMC summary, or None."""
    for pre in PMC_ROUNDS:
        path = os.path.join(REPO, "profiles", f"pmc_{pre}{tag}_requests.json")
        if os.path.exists(path):
            try:
                d = json.load(open(path))
                return {"per_step": d["tcc_req_per_step"], "ceiling": d["path_ceiling_G_requests_per_s"],
                        "source": f"profiles/pmc_{pre}{tag}_requests.json (rocprofv3 PMC pass)"}
            except Exception:
                pass
    return None


def request_rate(req, steps_per_launch: float, avg_kernel_ms: float):
    """The kernel's L2 request rate in this run: the committed requests per step x this run's steps
    per launch / its average launch time.  The path's random-access kernels all run at 40-47 G
    requests/s, a tighter yardstick for a gather kernel than bytes against HBM peak."""
    if not req or not avg_kernel_ms:
        return None
    rate = req["per_step"] * steps_per_launch / (avg_kernel_ms * 1e-3) / 1e9
    return {"per_step": req["per_step"], "G_per_s": round(rate, 2), "path_kernels_measured_G_per_s": req["ceiling"],
            "source": req["source"]}


def host_cpus():
    """What the host gives this job: nproc, the affinity set, the cgroup CPU
    quota (a GPU box shows the whole machine's CPUs but grants a share), the
    CPU model."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = info["nproc"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        info["model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        info["model"] = None
    info["usable"] = max(1, min(info["affinity"] or 1, quota or info["affinity"] or 1))
    return info


def cpu_cores(requested: int) -> int:
    """Every host core this job may use (affinity, capped by the cgroup quota), unless --cpu-threads."""
    return requested if requested > 0 else host_cpus()["usable"]


def cpu_baseline(args, n, active_vertices, off, adj, kind):
    """Reference CPU path (oracle/_ref/ref_harness, the reference's own headers)
    on a bounded sample: the same RMAT graph and model, MH mode, 1 walk per
    vertex (1/10 of the workload's walks) of length --cpu-length (24 instead
    of 80, so the sample is ~15-25 s of CPU work), timed generate only."""
    cores = cpu_cores(args.cpu_threads)
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if kind in ("auto", "reference") and os.path.exists(harness):
        cmd = [harness, "cfg", "1", str(args.cpu_length), args.model, str(args.paramP), str(args.paramQ), "weight",
               "1" if args.det else "0", "42",
               "graph-rmat", str(args.samples), str(2 * n), str(args.seed), str(n), "time-gen", "1"]
        env = dict(os.environ, NUM_THREADS=str(cores))
        log(f"cpu_baseline: reference harness, {cores} threads: {' '.join(cmd[1:])}")
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.cpu_timeout)
            m = re.search(r"time-gen seconds=([0-9.]+)", r.stdout)
            if r.returncode == 0 and m:
                secs = float(m.group(1))
                steps = active_vertices * (args.cpu_length - 1)
                full = active_vertices * args.wpv * (args.length - 1)
                return {"value": steps / secs, "unit": "walk-steps/s", "cores": cores, "kind": "reference",
                        "sample": f"reference WharfMH::generate_initial_random_walks on the same RMAT graph "
                                  f"(n={n}), walks_per_vertex=1 (1/{args.wpv} of the workload), L={args.cpu_length} "
                                  f"(workload: {args.length}), "
                                  f"{'deterministic' if args.det else 'MH'} {args.model}; {steps} steps in {secs:.2f} s",
                        "seconds": secs, "host": host_cpus(),
                        "full_workload_steps": full,
                        "full_workload_seconds_extrapolated": round(full / (steps / secs), 1)}
            log("cpu_baseline: harness failed", r.returncode, r.stderr[-500:])
        except subprocess.TimeoutExpired:
            log("cpu_baseline: harness timed out")
        if kind == "reference":
            return None
    # the C restatement (oracle/wharf_oracle.c), OpenMP over walks, same graph, bounded walk range
    from oracle import oracle as O
    eng = O.Engine(off, adj, wpv=args.wpv, L=args.length, model=O.NODE2VEC if args.model == "node2vec" else O.DEEPWALK,
                   p=args.paramP, q=args.paramQ, deterministic=args.det, seed=0x5EED)
    w1 = min(n * args.wpv, 2_000_000)
    secs = eng.time_generate_range(0, w1, cores)
    steps = eng.steps
    full = active_vertices * args.wpv * (args.length - 1)
    return {"value": steps / secs, "unit": "walk-steps/s", "cores": cores, "kind": "port",
            "sample": f"oracle/wharf_oracle.c restatement, same graph, walks [0, {w1}), L={args.length}; "
                      f"{steps} steps in {secs:.2f} s", "seconds": secs, "host": host_cpus(),
            "full_workload_steps": full, "full_workload_seconds_extrapolated": round(full / (steps / secs), 1)}


def cpu_baseline_same_shape(args, W, torch, dev, extrapolated):
    """The reference CPU path MEASURED at the workload's walk shape (VERDICT r04
    missing #2): walks_per_vertex and L of the headline (10 x 80), the
    headline's model and mode, on an RMAT graph of configs[1]'s density scaled
    down to --cpu-scale so that generation plus one 10k-edge insert batch fit
    the time budget; the GPU runs the same graph (same RMAT, bit-exact
    generator) in the same bench run.  `extrapolated` (the bounded configs[1]
    sample, linear in steps) is kept as a secondary field."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    cores = cpu_cores(args.cpu_threads)
    S = args.cpu_scale
    ns = 1 << S
    samples = args.samples >> max(0, args.scale - S)           # configs[1]'s samples per vertex
    mode = "deterministic" if args.det else "MH"
    # the GPU on the same graph: generation (first and warm), the index as the reference builds it
    # (per-vertex sorted (wid*L+pos, next), here exported to host), one insert batch
    cfg = W.WharfConfig(walks_per_vertex=args.wpv, walk_length=args.length,
                        model=W.NODE2VEC if args.model == "node2vec" else W.DEEPWALK, paramP=args.paramP,
                        paramQ=args.paramQ, deterministic=args.det, seed=0x5EED)
    g = W.WharfMH.from_rmat(ns, samples, 2 * ns, seed=args.seed, config=cfg, device=dev)
    m = g.number_of_edges()
    g.generate_initial_random_walks()
    g.generate_initial_random_walks()
    st = g.stats()
    gsteps, gms = st["steps"], st["last_walk_kernel_ms"]
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    g.generate_initial_random_walks()
    cnt, keys, nexts = g.inverted_index()
    gen_idx_ms = (time.perf_counter() - t1) * 1e3
    del cnt, keys, nexts
    batch = W.generate_batch_of_edges(5000, ns, 0, False, False, device=dev)
    out = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device=f"cuda:{dev}")
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    aff = g.insert_edges_batch(batch, remove_dups=True, out=out)
    torch.cuda.synchronize(dev)
    gpu_batch_ms = (time.perf_counter() - t1) * 1e3
    st2 = g.stats()
    gpu = {"generation_kernel_ms": round(gms, 3), "walk_steps": gsteps,
           "walk_steps_per_s": round(gsteps / (gms * 1e-3), 1),
           "generation_plus_index_export_ms": round(gen_idx_ms, 2),
           "insert_batch_ms": round(gpu_batch_ms, 3), "insert_batch_affected_walks": int(len(aff)),
           "insert_batch_graph_update_ms": round(st2["last_graph_update_ms"], 3),
           "insert_batch_walk_update_ms": round(st2["last_walk_update_ms"], 3)}
    g.destroy()
    cmd = [harness, "cfg", str(args.wpv), str(args.length), args.model, str(args.paramP), str(args.paramQ), "weight",
           "1" if args.det else "0", "42", "graph-rmat", str(samples), str(2 * ns), str(args.seed), str(ns),
           "time-gen", "1", "time-upd", "5000", "0", "0", "1"]
    log(f"cpu_baseline (same shape): reference harness, {cores} threads: {' '.join(cmd[1:])}")
    try:
        r = subprocess.run(cmd, env=dict(os.environ, NUM_THREADS=str(cores)), capture_output=True, text=True,
                           timeout=args.cpu_timeout)
    except subprocess.TimeoutExpired:
        log("cpu_baseline (same shape): harness timed out")
        return None
    gen = re.search(r"time-gen seconds=([0-9.]+)", r.stdout)
    upd = re.search(r"time-upd seconds=([0-9.]+) edges=(\d+) affected=(\d+)", r.stdout)
    if r.returncode != 0 or not gen:
        log("cpu_baseline (same shape): harness failed", r.returncode, r.stderr[-500:])
        return None
    secs = float(gen.group(1))
    steps = gsteps   # the same graph, start vertices and walk shape: the transitions both paths append
    rec = {"value": round(steps / secs, 1), "unit": "walk-steps/s", "cores": cores, "kind": "reference",
           "sample": f"reference WharfMH::generate_initial_random_walks MEASURED at the workload's walk shape "
                     f"(walks_per_vertex={args.wpv}, L={args.length}, {mode} {args.model}) on RMAT scale {S} "
                     f"(n={ns}, {samples} undirected samples = configs[1]'s per-vertex density, m={m}); "
                     f"{steps} transitions in {secs:.2f} s",
           "seconds": secs, "graph": {"scale": S, "n": ns, "m": m, "samples": samples, "seed": args.seed},
           "host": host_cpus(),
           "gpu_same_graph": gpu,
           "gpu_over_cpu_generation": round(gpu["walk_steps_per_s"] / (steps / secs), 1),
           "index_build_asymmetry": "the reference's timed generate also builds its per-vertex inverted index "
                                    "(wharfmh.h:329-354); the GPU's walk_steps_per_s is the walk kernel alone, its "
                                    "index is a derived export: gpu_same_graph.generation_plus_index_export_ms "
                                    "times generation + the full index sorted on the device and copied to host",
           "gpu_over_cpu_generation_with_index": round(secs * 1e3 / gen_idx_ms, 1)}
    if upd:
        rec["insert_batch"] = {"cpu_ms": round(float(upd.group(1)) * 1e3, 1), "edges": int(upd.group(2)),
                               "cpu_affected_walks": int(upd.group(3)), "gpu_ms": gpu["insert_batch_ms"],
                               "gpu_over_cpu": round(float(upd.group(1)) * 1e3 / gpu_batch_ms, 1),
                               "batch": "generate_batch_of_edges(5000, n, 0, false, undirected), remove_dups, "
                                        "walk update applied (memory-throughput-latency.cpp:126-134)"}
    if extrapolated:
        rec["configs1_extrapolation"] = extrapolated
    return rec


def cpu_baseline_deterministic_same_shape(args, W, torch, dev, extrapolated=None):
    """The reference's default mode (config::deterministic_mode = true,
    globals.h:29) MEASURED at the workload's walk shape:
    walks_per_vertex and L of the GPU line (10 x 80), DeepWalk, on the same
    scale --cpu-scale RMAT graph as cpu_baseline_same_shape (configs[1]'s
    per-vertex density); generation, then one 10k-edge insert batch
    generate_batch_of_edges(5000, n, 0, false, undirected) with the walk update
    applied (memory-throughput-latency.cpp:126-148).  The GPU runs the same
    graph and batch in the same mode beside it (bit-exact with the reference
    in this mode, tests/test_gpu_parity.py).  `extrapolated` (the configs[2]
    sample at 1 x 24, scaled linearly) is kept as a secondary field."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness) or args.cpu_scale <= 0:
        return extrapolated
    cores = cpu_cores(args.cpu_threads)
    S = args.cpu_scale
    ns = 1 << S
    samples = args.samples >> max(0, args.scale - S)
    cfg = W.WharfConfig(walks_per_vertex=args.wpv, walk_length=args.length, model=W.DEEPWALK, deterministic=True)
    g = W.WharfMH.from_rmat(ns, samples, 2 * ns, seed=args.seed, config=cfg, device=dev)
    m = g.number_of_edges()
    g.generate_initial_random_walks()
    g.generate_initial_random_walks()
    st = g.stats()
    batch = W.generate_batch_of_edges(5000, ns, 0, False, False, device=dev)
    out = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device=f"cuda:{dev}")
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    aff = g.insert_edges_batch(batch, remove_dups=True, out=out)
    torch.cuda.synchronize(dev)
    gpu_ms = (time.perf_counter() - t1) * 1e3
    st2 = g.stats()
    gpu = {"generation_kernel_ms": round(st["last_walk_kernel_ms"], 3), "walk_steps": st["steps"],
           "insert_batch_ms": round(gpu_ms, 3), "insert_batch_affected_walks": int(len(aff)),
           "insert_batch_graph_update_ms": round(st2["last_graph_update_ms"], 3),
           "insert_batch_walk_update_ms": round(st2["last_walk_update_ms"], 3),
           "insert_batch_rewalk_steps": st2["steps"]}
    g.destroy()
    cmd = [harness, "cfg", str(args.wpv), str(args.length), "deepwalk", str(args.paramP), str(args.paramQ), "weight",
           "1", "42", "graph-rmat", str(samples), str(2 * ns), str(args.seed), str(ns), "time-gen", "1",
           "time-upd", "5000", "0", "0", "1"]
    log(f"cpu_baseline_deterministic (same shape): reference harness, {cores} threads: {' '.join(cmd[1:])}")
    try:
        r = subprocess.run(cmd, env=dict(os.environ, NUM_THREADS=str(cores)), capture_output=True, text=True,
                           timeout=args.cpu_timeout)
    except subprocess.TimeoutExpired:
        log("cpu_baseline_deterministic (same shape): harness timed out")
        return extrapolated
    gen = re.search(r"time-gen seconds=([0-9.]+)", r.stdout)
    upd = re.search(r"time-upd seconds=([0-9.]+) edges=(\d+) affected=(\d+)", r.stdout)
    if r.returncode != 0 or not gen or not upd:
        log("cpu_baseline_deterministic (same shape): harness failed", r.returncode, r.stderr[-500:])
        return extrapolated
    cpu_batch_ms = float(upd.group(1)) * 1e3
    rec = {"kind": "reference", "cores": cores, "host": host_cpus(),
           "sample": f"reference WharfMH, deterministic mode, MEASURED at the workload's walk shape "
                     f"(walks_per_vertex={args.wpv}, L={args.length}, DeepWalk) on RMAT scale {S} (n={ns}, "
                     f"{samples} undirected samples = configs[1]'s per-vertex density, m={m}): generation, then "
                     f"one insert batch generate_batch_of_edges(5000, n, 0, false, undirected) with the walk "
                     f"update applied",
           "graph": {"scale": S, "n": ns, "m": m, "samples": samples, "seed": args.seed},
           "generation_seconds": float(gen.group(1)),
           "generation_walk_steps_per_s": round(gpu["walk_steps"] / float(gen.group(1)), 1),
           "insert_batch_ms": round(cpu_batch_ms, 1), "insert_batch_edges": int(upd.group(2)),
           "insert_batch_affected_walks": int(upd.group(3)),
           "gpu_same_graph": gpu,
           "gpu_over_cpu_insert_batch": round(cpu_batch_ms / gpu_ms, 1),
           "affected_walks_equal": int(upd.group(3)) == int(len(aff))}
    if extrapolated:
        rec["configs2_extrapolation"] = extrapolated
    return rec


def cpu_baseline_deterministic(args, batches=3):
    """The reference's default mode (config::deterministic_mode = true,
    globals.h:29) on the reference CPU path: configs[2]'s graph, generation and
    10k-edge insert batches with the walk update applied, on a bounded sample
    (1 walk per vertex of length --cpu-length; the GPU line runs 10 x 80), so
    it finishes in well under a minute.  Reported beside the GPU's
    deterministic re-walk latency, not compared with it as the same workload."""
    harness = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    cores = cpu_cores(args.cpu_threads)
    ns = 1 << args.scale
    cmd = [harness, "cfg", "1", str(args.cpu_length), "deepwalk", str(args.paramP), str(args.paramQ), "weight", "1",
           "42", "graph-rmat", str(args.stream_samples), str(2 * ns), str(args.seed + 1), str(ns), "time-gen", "1",
           "time-upd", "5000", "0", "0", str(batches)]
    log(f"cpu_baseline_deterministic: reference harness, {cores} threads: {' '.join(cmd[1:])}")
    try:
        r = subprocess.run(cmd, env=dict(os.environ, NUM_THREADS=str(cores)), capture_output=True, text=True,
                           timeout=args.cpu_timeout)
    except subprocess.TimeoutExpired:
        log("cpu_baseline_deterministic: harness timed out")
        return None
    gen = re.search(r"time-gen seconds=([0-9.]+)", r.stdout)
    upd = [(float(a), int(b)) for a, b in re.findall(r"time-upd seconds=([0-9.]+) edges=\d+ affected=(\d+)", r.stdout)]
    if r.returncode != 0 or not gen or not upd:
        log("cpu_baseline_deterministic: harness failed", r.returncode, r.stderr[-500:])
        return None
    return {"kind": "reference", "cores": cores, "host": host_cpus(),
            "sample": f"reference WharfMH, deterministic mode, configs[2]'s graph (RMAT scale {args.scale}, "
                      f"{args.stream_samples} undirected samples), walks_per_vertex=1, L={args.cpu_length} "
                      f"(the GPU line: {args.wpv} x {args.length}); {batches} insert batches of "
                      f"generate_batch_of_edges(5000, n, b, false, undirected), walk update applied",
            "generation_seconds": float(gen.group(1)),
            "insert_batch_median_ms": round(float(np.median([u[0] for u in upd])) * 1e3, 1),
            "mean_affected_walks": int(np.mean([u[1] for u in upd])),
            # the walk update re-walks ~(walks x remaining length): scaled linearly to the GPU line's wpv and L
            "insert_batch_ms_extrapolated_to_workload": round(float(np.median([u[0] for u in upd])) * 1e3 * args.wpv
                                                              * (args.length - 1) / (args.cpu_length - 1), 1)}


def record_bytes_per_slot(g, n, anchors):
    """Edge-record bytes per pool slot from the handle's footprint (vrec: 16 B per vertex)."""
    per = (g.memory_footprint(verbose=False)["records_bytes"] - 16 * n) / max(g.stats()["pool_capacity"], 1)
    per *= 2 if anchors else 1
    return min((8, 16, 32), key=lambda b: abs(b - per))


def stream_latency(args, W, torch, cfg, dev, world, rank, dist, comm_dev, barrier, batches, scan_batches=0):
    """configs[2]: per-batch latency of 10k-edge insert batches with the re-walk applied
    (memory-throughput-latency.cpp:126-134: generate_batch_of_edges(5000, n, seed=b, false, undirected))."""
    if batches <= 0:
        return None
    ns = 1 << args.scale   # configs[2] is a one-GPU graph: not grown with the ranks
    gs = W.WharfMH.from_rmat(ns, args.stream_samples, 2 * ns, seed=args.seed + 1, config=cfg, device=dev)
    gs.set_shard(*balanced_shards(np.diff(gs.offsets().astype(np.int64)), world)[rank])
    gs.generate_initial_random_walks()
    gs.generate_initial_random_walks()
    s1 = gs.stats()
    gen3 = {"ms": round(s1["last_walk_kernel_ms"], 3), "steps": s1["steps"]}
    # affected walk ids stay in HBM (WHARF_AFFECTED_DEVICE); the host-list
    # variant (PCIe-inclusive, the reference's return value) is timed after
    out = torch.empty(max(gs.number_of_walks, 1), dtype=torch.int32, device=f"cuda:{dev}")
    lat, aff, gu, wu, kern, rsteps, mv, mslots, imode = [], [], [], [], [], [], [], [], []
    for b in range(batches):
        batch = W.generate_batch_of_edges(5000, ns, b, False, False, device=dev)
        barrier()
        t1 = time.perf_counter()
        a = gs.insert_edges_batch(batch, remove_dups=True, out=out)
        barrier()
        lat.append((time.perf_counter() - t1) * 1e3)
        s2 = gs.stats()
        aff.append(len(a))
        gu.append(s2["last_graph_update_ms"])
        wu.append(s2["last_walk_update_ms"])
        kern.append(s2["last_walk_kernel_ms"])
        rsteps.append(s2["steps"])
        mv.append(s2["last_csr_move_ms"])
        mslots.append(s2["last_moved_slots"])
        imode.append(s2["last_in_edge_mode"])
    # rewalk points alone (apply_walk_updates = false): the scan over the whole walk matrix
    scan = []
    for b in range(scan_batches):
        batch = W.generate_batch_of_edges(5000, ns, 10_000 + b, False, False, device=dev)
        gs.insert_edges_batch(batch, remove_dups=True, apply_walk_updates=False, out=out)
        scan.append(gs.stats()["last_walk_kernel_ms"])
    hout = torch.empty(max(gs.number_of_walks, 1), dtype=torch.int32, pin_memory=True).numpy().view(np.uint32)
    lat_host = []
    for b in range(batches, batches + min(5, batches)):
        batch = W.generate_batch_of_edges(5000, ns, b, False, False, device=dev)
        barrier()
        t1 = time.perf_counter()
        gs.insert_edges_batch(batch, remove_dups=True, out=hout)
        barrier()
        lat_host.append((time.perf_counter() - t1) * 1e3)
    lat_all = lat
    if dist:
        tl = torch.tensor(lat, dtype=torch.float64, device=comm_dev)
        dist.all_reduce(tl, op=dist.ReduceOp.MAX)
        lat_all = tl.tolist()
    res = {"workload": f"configs[2] soc-LiveJournal-sized streaming: RMAT scale {args.scale}, "
                       f"{args.stream_samples} undirected samples (m={gs.number_of_edges()}), "
                       f"{batches} insert batches of generate_batch_of_edges(5000, n, b, false, "
                       f"undirected), re-walk applied",
           "batches": batches, "edges_per_batch": int(len(batch)),
           "median_ms": round(float(np.median(lat_all)), 3), "p90_ms": round(float(np.percentile(lat_all, 90)), 3),
           "median_ms_ids_to_host_pinned": round(float(np.median(lat_host)), 3),
           "mean_affected_walks_rank0": int(np.mean(aff)),
           "median_graph_update_ms": round(float(np.median(gu)), 3),
           "median_walk_update_ms": round(float(np.median(wu)), 3),
           "median_rewalk_kernel_ms": round(float(np.median(kern)), 3),
           "mean_rewalk_steps_rank0": int(np.mean(rsteps)),
           "rewalk_Gsteps_per_s": round(float(np.sum(rsteps) / np.sum(kern) / 1e6), 2),
           "generation_same_graph": gen3,
           "median_in_edge_scan_ms": round(float(np.median(mv)), 4), "pool_slots": int(np.median(mslots)),
           # in-edge records: 0 = streaming scan of the pool (pool_slots = slots read), 1 = reverse-slot
           # index (pool_slots = the sources' new row slots, at most)
           "in_edge_mode": "reverse_index" if np.median(imode) >= 1 else "scan",
           "stored_positions_rank0": int(gs.number_of_walks) * args.length,
           # bytes per pool slot of the edge-record table: 8 (compact), 16, or 32 (node2vec MH: the
           # footprint counts the anchor half of those records as samplers)
           "record_bytes": record_bytes_per_slot(gs, ns, cfg.model == W.NODE2VEC and not cfg.deterministic)}
    if scan:
        res["scan_only_median_ms"] = round(float(np.median(scan)), 4)
    gs.destroy()
    return res




def timed_generation(g, steps, warmup, barrier, log_rank=None):
    """W untimed + K timed generate_initial_random_walks(), barrier + sync on both
    sides.  Returns (elapsed s, per-launch kernel ms of the timed steps, warmup ms)."""
    warm_ms = []
    for i in range(warmup):
        g.generate_initial_random_walks()
        warm_ms.append(g.stats()["last_walk_kernel_ms"])
        if log_rank is not None:
            log(f"[rank {log_rank}] warmup {i}: {warm_ms[-1]:.1f} ms")
    barrier()
    t_start = time.perf_counter()
    kern_ms = []
    for _ in range(steps):
        g.generate_initial_random_walks()
        kern_ms.append(g.stats()["last_walk_kernel_ms"])
    barrier()
    return time.perf_counter() - t_start, kern_ms, warm_ms


def reduce_steps_time(torch, dist, comm_dev, steps_local, elapsed):
    """(sum of transitions over ranks, max elapsed over ranks)"""
    if not dist:
        return steps_local, elapsed
    tt = torch.tensor([float(steps_local), elapsed], dtype=torch.float64, device=comm_dev)
    s = tt.clone()
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    mx = tt.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    return int(s[0].item()), mx[1].item()


def node2vec_record(args, W, torch, dev, barrier, n):
    """configs[4]'s model (node2vec p, q, WEIGHT inits, MH) on the configs[1] graph:
    the first generation of a fresh handle (every anchor initialised), warm
    generations (anchors cached), then configs[2]'s re-walk stream."""
    cfg = W.WharfConfig(walks_per_vertex=args.wpv, walk_length=args.length, model=W.NODE2VEC, paramP=args.paramP,
                        paramQ=args.paramQ, deterministic=False, seed=0x5EED)
    g = W.WharfMH.from_rmat(n, args.samples, 2 * n, seed=args.seed, config=cfg, device=dev)
    elapsed, kern, warm = timed_generation(g, args.n2v_steps, 1, barrier)
    st = g.stats()
    steps = st["steps"]
    avg = float(np.mean(kern))
    achieved = steps * BYTES_PER_STEP_NODE2VEC / (avg * 1e-3) / 1e9
    n2v_traffic, n2v_traffic_src = load_traffic(f"gen_node2vec_mh_s{args.scale}")
    # SURVEY 8(d)'s node2vec unit prices the reference's has_edge binary search in
    # prev's row: 44 + 4 * ceil(log2 deg(prev)) B per step, with the mean probe
    # count measured over the transitions of 4096 walks of this corpus
    deg = np.diff(g.offsets().astype(np.int64))
    w0 = (g.number_of_walks // 2) & ~0xFFFF
    prevs = np.concatenate([g.walk_vertices(w0 + i)[:-1] for i in range(4096)]).astype(np.int64)
    probes = float(np.mean(np.ceil(np.log2(np.maximum(deg[prevs], 1)))))
    survey_bps = 44 + 4 * probes
    survey_achieved = steps * survey_bps / (avg * 1e-3) / 1e9
    rec = {"workload": f"configs[1] graph (RMAT scale {args.scale}, m={g.number_of_edges()}), node2vec "
                       f"p={args.paramP} q={args.paramQ} MH, WEIGHT sampler init, walks_per_vertex={args.wpv}, "
                       f"walk_length={args.length}",
           "value": round(steps * len(kern) / elapsed, 1), "unit": "walk-steps/s",
           "warm_generation_kernel_ms": round(avg, 3), "first_generation_kernel_ms": round(warm[0], 3),
           "first_generation_Gsteps_per_s": round(steps / (warm[0] * 1e-3) / 1e9, 2),
           "mh_accept_rate": round(st["accepts"] / steps, 5) if steps else None,
           "roofline": {"bound": "hbm", "kernel": "k_walk<node2vec, MH> (warm generation)",
                        "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 5), "bytes_per_step": BYTES_PER_STEP_NODE2VEC,
                        "bytes_per_step_basis": "as built: 32-B edge record with the anchor entry + one 32-B edge-hash "
                                                "bucket + 4-B output",
                        "survey_unit": {"bytes_per_step": round(survey_bps, 2),
                                        "mean_binary_search_probes": round(probes, 3),
                                        "formula": "44 + 4 * ceil(log2 deg(prev)) (SURVEY 8(d)), probes measured over "
                                                   "the transitions of 4096 walks",
                                        "achieved": round(survey_achieved, 2),
                                        "frac": round(survey_achieved / HBM_PEAK_GBS, 5)},
                        "traffic": n2v_traffic, "traffic_source": n2v_traffic_src}}
    g.destroy()
    rec["rewalk_latency_10k_batch"] = stream_latency(args, W, torch, cfg, dev, 1, 0, None, None, barrier,
                                                     args.n2v_rewalk_batches)
    return rec


def streaming_rooflines(rewalk, rewalk_det, scale):
    """The streaming kernels of the update path against the HBM peak, by
    algorithmic bytes: rewalk-point scan 4 B per stored position;
    deterministic re-walk (suffix table + chunked copy) 4 B per stored position
    (each position is read up to the walk's rewalk point and written after it);
    in-edge record scan of the slack-row CSR update 4 B per pool slot (the
    slots' targets are read; the few records of sources' in-edges written)."""
    out = {}
    pmc, pmc_rel = {}, None
    for pre in PMC_ROUNDS:   # the newest round's PMC pass of the same stream
        rel = os.path.join("profiles", f"pmc_{pre}streaming_s{scale}.json")
        if os.path.exists(os.path.join(REPO, rel)):
            pmc, pmc_rel = json.load(open(os.path.join(REPO, rel))), rel
            break

    def ent(name, kernel, bytes_, ms, per):
        if not ms:
            return None
        a = bytes_ / (ms * 1e-3) / 1e9
        e = {"kernel": kernel, "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(a / HBM_PEAK_GBS, 4), "ms": ms, "algorithmic_bytes": int(bytes_), "per_unit": per,
             "traffic": None}
        if name in pmc:   # HBM bytes per launch (PMC pass of the same stream) and the rate they move at
            e["traffic"] = pmc[name]["hbm_bytes_per_launch"]
            e["traffic_GBps"] = round(e["traffic"] / (ms * 1e-3) / 1e9, 1)
            e["traffic_source"] = f"{pmc_rel} (rocprofv3 PMC pass)"
        return e
    if rewalk_det:
        pos = rewalk_det["stored_positions_rank0"]
        out["rewalk_point_scan"] = ent("rewalk_point_scan", "k_rewalk_scan_lean (apply_walk_updates=false)",
                                       4 * pos, rewalk_det.get("scan_only_median_ms"), "4 B per stored position")
        out["deterministic_rewalk_copy"] = ent("deterministic_rewalk_copy", "k_det_suffix + k_rewalk_chunked<true, NTL, 1>",
                                               4 * pos, rewalk_det["median_rewalk_kernel_ms"],
                                               "4 B per stored position")
    src = rewalk or rewalk_det
    if src and src.get("in_edge_mode") == "reverse_index":
        # k_patch_rev: per slot of the sources' new rows, its target (4 B) and reverse entry (8 B) read, the
        # reverse slot's 16-B record and 8-B entry written
        out["in_edge_records"] = ent("in_edge_records", "k_patch_rev (in-edge records through the reverse-slot "
                                     "index)", 36 * src["pool_slots"], src["median_in_edge_scan_ms"],
                                     "36 B per slot of the sources' new rows")
    elif src:
        out["in_edge_scan"] = ent("in_edge_scan", "k_patch_in_edges (records of the batch sources' in-edges)",
                                  4 * src["pool_slots"], src["median_in_edge_scan_ms"], "4 B per pool slot")
    return out or None


def _update_stream(g, W, n, batches, mixed, out):
    """Insert batch b (and, mixed, delete it again: throughput-latency.cpp:126,135)
    for b < batches: generate_batch_of_edges(5000, n, b, false, undirected)
    (memory-throughput-latency.cpp:126-134).  Per-update device times."""
    rec = {k: [] for k in ("ms", "graph_ms", "walk_ms", "kernel_ms", "in_edge_ms", "steps", "affected", "inits",
                           "in_edge_mode")}
    for b in range(batches):
        batch = W.generate_batch_of_edges(5000, n, b, False, False)
        for ins in ((True, False) if mixed else (True,)):
            t1 = time.perf_counter()
            (g.insert_edges_batch if ins else g.delete_edges_batch)(batch, remove_dups=True, out=out)
            rec["ms"].append((time.perf_counter() - t1) * 1e3)
            st = g.stats()
            rec["graph_ms"].append(st["last_graph_update_ms"])
            rec["walk_ms"].append(st["last_walk_update_ms"])
            rec["kernel_ms"].append(st["last_walk_kernel_ms"])
            rec["in_edge_ms"].append(st["last_csr_move_ms"])
            rec["steps"].append(st["steps"])
            rec["affected"].append(st["affected"])
            rec["inits"].append(st["last_anchor_inits"])
            rec["in_edge_mode"].append(st["last_in_edge_mode"])
    med = lambda k: round(float(np.median(rec[k])), 3)
    return {"updates": len(rec["ms"]), "batch_median_ms": med("ms"), "batch_p90_ms": round(float(np.percentile(rec["ms"], 90)), 3),
            "graph_update_median_ms": med("graph_ms"), "walk_update_median_ms": med("walk_ms"),
            "rewalk_kernel_median_ms": med("kernel_ms"), "in_edge_scan_median_ms": round(float(np.median(rec["in_edge_ms"])), 4),
            "mean_affected_walks": int(np.mean(rec["affected"])), "mean_rewalk_steps": int(np.mean(rec["steps"])),
            "rewalk_Gsteps_per_s": round(float(np.sum(rec["steps"]) / np.sum(rec["walk_ms"]) / 1e6), 2),
            "mean_anchor_inits": int(np.mean(rec["inits"])),
            "in_edge_records": "reverse_index" if np.median(rec["in_edge_mode"]) >= 1 else "scan"}


def per_gpu_of_8(args, W, torch, dev, barrier):
    """The per-GPU work of BASELINE configs[3] and configs[4] on 8 GPUs, run on
    this one GPU: the full graph (replicated on every rank, wharfmh.h:275,761
    shard by walk) with the walks of start-vertex shard 0 of 8.  configs[3]:
    twitter-sized RMAT (scale 25, 1.2 G undirected samples), DeepWalk wpv 10,
    insert batches, MH and deterministic; beside it the same graph with every
    walk on this one GPU (the 1-GPU time an 8-GPU run divides).  configs[4]:
    friendster-sized RMAT (scale 26, 1.8 G samples), node2vec p=.5 q=2 MH WEIGHT,
    wpv 10 (the survey's 656 M walks / 8), mixed insert/delete batches.  The
    graphs use seed 4 (tools/bigscale.py).  Each case is skipped with its error
    when the device cannot hold it, so the headline line always prints."""
    from dynamicgraphrepresentationlearning_amd.distributed import block_shards
    out = {"note": "one GPU running the work one rank of an 8-GPU job does (the job's block shard 0 of 8: "
                   "2^16-vertex blocks dealt round-robin, as multi_gpu_job); graphs built on the device (seed 4)"}
    cases = [("configs3_deepwalk_mh_shard0of8", 25, 1_200_000_000, W.DEEPWALK, False, 8, False),
             ("configs3_deepwalk_det_shard0of8", 25, 1_200_000_000, W.DEEPWALK, True, 8, False),
             ("configs3_deepwalk_mh_all_walks_1gpu", 25, 1_200_000_000, W.DEEPWALK, False, 1, False),
             ("configs4_node2vec_mh_shard0of8", 26, 1_800_000_000, W.NODE2VEC, False, 8, True)]
    if args.per8_cases:
        keep = set(args.per8_cases.split(","))
        cases = [c for c in cases if c[0] in keep]
    for name, scale, samples, model, det, parts, mixed in cases:
        n = 1 << scale
        g = None
        try:
            t0 = time.time()
            cfg = W.WharfConfig(walks_per_vertex=10, walk_length=80, model=model, paramP=0.5, paramQ=2.0,
                                deterministic=det, seed=0x5EED)
            g = W.WharfMH.from_rmat(n, samples, 2 * n, seed=4, config=cfg, device=dev)
            sh = block_shards(n, parts, 16)[0]
            g.apply_shard(sh)
            build_s = time.time() - t0
            g.generate_initial_random_walks()
            first = g.stats()
            g.generate_initial_random_walks()
            warm = g.stats()
            ids = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device=f"cuda:{dev}")
            barrier()
            rec = {"graph": f"RMAT scale {scale}, {samples} undirected samples (seed 4), m={g.number_of_edges()}",
                   "model": f"{'node2vec p=0.5 q=2 WEIGHT' if model == W.NODE2VEC else 'DeepWalk'} "
                            f"{'deterministic' if det else 'MH'}, walks_per_vertex=10, L=80",
                   "walks": g.number_of_walks, "shard": str(sh), "of": parts, "build_s": round(build_s, 1),
                   "first_generation_ms": round(first["last_walk_kernel_ms"], 2),
                   "first_generation_anchor_inits": first["last_anchor_inits"],
                   "generation_ms": round(warm["last_walk_kernel_ms"], 2),
                   "generation_Gsteps_per_s": round(warm["steps"] / warm["last_walk_kernel_ms"] / 1e6, 2),
                   "batches": f"{args.per8_batches} x generate_batch_of_edges(5000, n, b, false, undirected)"
                              f"{', each inserted then deleted' if mixed else ', inserted'}",
                   "device_bytes": g.memory_footprint(verbose=False)["total_bytes"]}
            rec.update(_update_stream(g, W, n, args.per8_batches, mixed, ids))
            out[name] = rec
            log(f"per_gpu_of_8 {name}: {json.dumps(rec)}")
        except Exception as ex:   # noqa: BLE001 (a case that does not fit is reported, not fatal)
            out[name] = {"error": str(ex)[:500]}
            log(f"per_gpu_of_8 {name} failed: {ex}")
        finally:
            if g is not None:
                g.destroy()
            torch.cuda.empty_cache()
    a, b = out.get("configs3_deepwalk_mh_shard0of8", {}), out.get("configs3_deepwalk_mh_all_walks_1gpu", {})
    if "batch_median_ms" in a and "batch_median_ms" in b:
        out["configs3_batch_speedup_1gpu_to_shard"] = round(b["batch_median_ms"] / a["batch_median_ms"], 2)
        out["configs3_generation_speedup_1gpu_to_shard"] = round(b["generation_ms"] / a["generation_ms"], 2)
    return out


def _max_over_ranks(torch, dist, comm_dev, vals):
    t = torch.tensor(list(vals), dtype=torch.float64, device=comm_dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def _sum_over_ranks(torch, dist, comm_dev, vals):
    t = torch.tensor(list(vals), dtype=torch.float64, device=comm_dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def _per_rank(torch, dist, comm_dev, vals, world):
    """[world][len(vals)]: every rank's values (all-gathered)."""
    t = torch.tensor(list(vals), dtype=torch.float64, device=comm_dev)
    if not dist:
        return [t.tolist()]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def corpus_gather_record(args, torch, dist, g, shards, n, wpv, L, dev, comm_dev, world, rank, barrier, budget_bytes,
                         mem=None):
    """The corpus reassembled for the downstream consumer (yskip,
    vertex-classification.cpp:142-158) by the bounded full-mesh all-gatherv
    (distributed.gather_corpus_chunked): chunks of at most `budget_bytes` land
    in one reused buffer, local rows are read from the handle per chunk.  Timed
    pass (the chunk is dropped), then a checked pass: the checksum of everything
    every rank received equals the sum of the ranks' local checksums.

    `budget_bytes` is this rank's own (from its free memory); the rows per chunk
    are agreed (minimum over the ranks) before anything is allocated, and every
    fallible local step is agreed before the next collective (distributed.agree),
    so a rank that fails makes every rank raise RankFailure instead of hanging."""
    from dynamicgraphrepresentationlearning_amd.distributed import agree, agree_min, alloc_or_reclaim, \
        corpus_checksum, gather_corpus_chunked, injected_fault, local_corpus_checksum, shard_size
    on_dev = comm_dev != "cpu"
    K_local = max(1, int(budget_bytes // (world * L * 4)))
    K = max(1, agree_min(K_local, device=comm_dev) if dist else K_local)
    stage, err = None, None
    try:
        injected_fault("gather", rank)
        if not on_dev:
            stage = alloc_or_reclaim(lambda: torch.empty((K, L), dtype=torch.int32, device=f"cuda:{dev}"),
                                     g.release_caches, rank)
    except Exception as ex:   # noqa: BLE001 (agreed: every rank abandons the gather)
        err = ex
    agree(err, "corpus gather setup", device=comm_dev)

    def read_local(first, count, out):
        injected_fault("gather_read", rank)
        if mem is not None:   # the chunk buffer (and, after the first chunk, RCCL's buffers) are live here
            mem.probe("corpus gather")
        if on_dev:
            g.export_walk_rows(first, count, out)
        else:   # gloo rehearsal: rows staged through the device buffer to host memory
            g.export_walk_rows(first, count, stage[:count])
            out.copy_(stage[:count].cpu())

    barrier()
    t1 = time.perf_counter()
    st = gather_corpus_chunked(read_local, shards, n, wpv, L, K, None, device=comm_dev, on_oom=g.release_caches)
    barrier()
    ms = (time.perf_counter() - t1) * 1e3
    ms_all = _max_over_ranks(torch, dist, comm_dev, [ms])[0]
    rec = {"pattern": "gather_corpus_chunked: full-mesh batch_isend_irecv per chunk of local rows",
           "backend": "nccl (RCCL over xGMI)" if on_dev else "gloo (host staging)",
           "walks": sum(shard_size(sh) for sh in shards) * wpv,
           "corpus_bytes": sum(shard_size(sh) for sh in shards) * wpv * L * 4,
           "rows_per_rank_per_chunk": K, "rows_per_rank_this_rank_budget": K_local,
           "buffer_bytes": K * world * L * 4, "chunks": st["chunks"], "ms": round(ms_all, 2),
           "bytes_received_rank0": int(st["bytes_received"]),
           "GBps_received_per_rank": round(st["bytes_received"] / (ms_all * 1e-3) / 1e9, 1) if ms_all else None}
    if args.gather_check:
        acc = torch.zeros((), dtype=torch.int64, device=comm_dev)

        def sink(chunk, segs):
            for r0, c, g0 in segs:
                acc.add_(corpus_checksum(chunk[r0:r0 + c], g0, L))

        gather_corpus_chunked(read_local, shards, n, wpv, L, K, sink, device=comm_dev, on_oom=g.release_caches)
        mine, err = None, None
        try:
            mine = local_corpus_checksum(read_local, shards[rank], n, wpv, L, K, device=comm_dev)
        except Exception as ex:   # noqa: BLE001
            err = ex
        agree(err, "local corpus checksum", device=comm_dev)
        tot = mine.clone()
        if dist:
            dist.all_reduce(tot)
        ok = torch.tensor([1 if int(acc.item()) == int(tot.item()) else 0], dtype=torch.int64, device=comm_dev)
        if dist:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        rec["checksum_of_checksums_ok"] = bool(ok.item())
    if on_dev:
        torch.cuda.empty_cache()
    return rec


JOBS = {
    # BASELINE configs[3]: twitter-2010-sized, initial walks + streaming inserts, walks sharded over the
    # ranks (strong scaling of the one job), corpus all-gathered
    "configs3": dict(scale=25, samples=1_200_000_000, model="deepwalk", mixed=False, split="ranks",
                     desc="twitter-2010-sized RMAT, DeepWalk MH, walks_per_vertex=10, L=80, insert batches; "
                          "the 335 M walks split over the ranks"),
    # BASELINE configs[4]: friendster-sized, node2vec p=.5 q=2 MH, mixed insert/delete; 656 M walks need
    # 8 GPUs (253 GB per rank), so rank g runs shard g of 8 at every N (weak scaling: N/8 of the job)
    "configs4": dict(scale=26, samples=1_800_000_000, model="node2vec", mixed=True, split="eighths",
                     desc="friendster-sized RMAT, node2vec p=0.5 q=2 MH WEIGHT, walks_per_vertex=10, L=80, "
                          "insert/delete pairs; rank g runs start-vertex shard g of 8"),
}


class _MemLow:
    """Lowest free device memory (hipMemGetInfo) seen at the probes of a job:
    after the build, each generation, each gather chunk (buffer and RCCL
    buffers live) and each update -- the job's peak footprint on this rank."""

    def __init__(self, torch, dev, on):
        self.torch, self.dev, self.on = torch, dev, on
        self.low, self.total, self.where = None, None, None

    def probe(self, where):
        if not self.on:
            return
        free, total = self.torch.cuda.mem_get_info(self.dev)
        if self.low is None or free < self.low:
            self.low, self.where = free, where
        self.total = total

    def record(self):
        if self.low is None:
            return None
        return {"min_free_bytes": int(self.low), "total_bytes": int(self.total),
                "peak_used_bytes": int(self.total - self.low), "at": self.where,
                "source": "hipMemGetInfo (torch.cuda.mem_get_info) at the job's phase boundaries and gather chunks"}


class _Phase:
    """`with phase("name"):` runs one rank's local, fallible part of a job phase
    (no collective inside) and then agrees the outcome with every rank
    (distributed.agree): if any rank failed, every rank raises RankFailure at
    the end of the same phase, so no rank is left waiting in a later collective.
    WHARF_TEST_FAIL="<rank>:<phase>" (phase = the name's first word) makes that
    rank's phase fail at its end, as if its body had raised."""

    def __init__(self, dist, comm_dev, rank):
        self.dist, self.comm_dev, self.rank = dist, comm_dev, rank

    def __call__(self, name):
        self.name = name
        return self

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        from dynamicgraphrepresentationlearning_amd.distributed import agree, injected_fault
        if et is not None and not issubclass(et, Exception):
            return False   # KeyboardInterrupt / SystemExit: not a job failure
        if ev is None:
            try:
                injected_fault(self.name.split()[0], self.rank)
            except RuntimeError as ex:
                ev = ex
                if not self.dist:
                    raise
        if self.dist:
            agree(ev, self.name, device=self.comm_dev)   # raises RankFailure on every rank if any failed
            return False
        return False       # one process, no peers: the exception propagates as it is


def multi_gpu_job(args, name, W, torch, dev, world, rank, dist, comm_dev, barrier):
    """One of BASELINE's 8-GPU jobs on the ranks of this run: the graph built on
    every rank (replicated, wharfmh.h:275,761 shard by walk), the rank's walk
    shard, first and warm generation, the bounded corpus all-gatherv, then
    --job-batches update batches generate_batch_of_edges(5000, n, b, false,
    undirected) (configs[4]: each inserted, then deleted,
    throughput-latency.cpp:126,135).  Per update: barrier, the rank's wall time,
    max over ranks.  configs[3] also runs, on rank 0 alone, every walk on one
    GPU over the same graph: the 1-GPU time the job divides.

    Every fallible step (build, each generation, the gather, each update, the
    one-GPU leg) is a phase whose outcome all ranks agree on before the next
    collective: a rank that fails (e.g. out of device memory) makes every rank
    return {"error", "failed_rank", "phase"} together instead of leaving its
    peers inside a barrier."""
    from dynamicgraphrepresentationlearning_amd.distributed import RankFailure, balanced_shards, block_shards, \
        injected_fault, shard_size
    spec = JOBS[name]
    scale = spec["scale"] + args.job_scale_delta
    samples = spec["samples"] >> (-args.job_scale_delta) if args.job_scale_delta < 0 else spec["samples"]
    n = 1 << scale
    parts = world if spec["split"] == "ranks" else max(8, world)
    node2vec = spec["model"] == "node2vec"
    cfg = W.WharfConfig(walks_per_vertex=10, walk_length=80, model=W.NODE2VEC if node2vec else W.DEEPWALK,
                        paramP=0.5, paramQ=2.0, deterministic=False, seed=0x5EED)
    phase = _Phase(dist, comm_dev, rank)
    mem = _MemLow(torch, dev, comm_dev != "cpu" or dist is None)
    g = None
    try:
        t0 = time.time()
        with phase("build"):
            g = W.WharfMH.from_rmat(n, samples, 2 * n, seed=4, config=cfg, device=dev)
            if args.job_shards == "blocks":   # 64 Ki-vertex blocks round-robin: every rank the same mix
                shards = block_shards(n, parts, args.job_block_bits)
            else:                               # contiguous ranges with equal non-isolated vertex counts
                shards = balanced_shards(np.diff(g.offsets().astype(np.int64)), parts)
            g.apply_shard(shards[rank])
            mem.probe("build")
        build_s = time.time() - t0
        gen = []
        for i in range(2):   # first (node2vec: every anchor initialised) and warm generation
            barrier()
            with phase(f"generation {i}"):
                t1 = time.perf_counter()
                g.generate_initial_random_walks()
                torch.cuda.synchronize(dev)
                wall = (time.perf_counter() - t1) * 1e3
                st = g.stats()
                gen.append((wall, st["last_walk_kernel_ms"], st["steps"], st["last_anchor_inits"]))
                mem.probe(f"generation {i}")
        gmax = _max_over_ranks(torch, dist, comm_dev, [gen[0][0], gen[1][0], gen[0][1], gen[1][1]])
        gsum = _sum_over_ranks(torch, dist, comm_dev, [gen[1][2], gen[0][3]])
        rec = {"workload": f"BASELINE {name}: {spec['desc']}; RMAT scale {scale}, {samples} undirected samples "
                           f"(seed 4), m={g.number_of_edges()}",
               "ranks": world, "walk_shards": parts,
               "shard_kind": f"blocks of 2^{args.job_block_bits} vertices round-robin"
               if args.job_shards == "blocks" else "contiguous ranges, equal non-isolated counts",
               "walks_this_run": int(sum(shard_size(sh) for sh in shards[:world]) * 10),
               "walks_whole_job": n * 10, "scaling": "strong (the job's walks split over the ranks)"
               if spec["split"] == "ranks" else f"weak (rank g runs shard g of {parts}: {world}/{parts} of the job)",
               "build_s_rank0": round(build_s, 1),
               "first_generation_ms": round(gmax[0], 2), "generation_ms": round(gmax[1], 2),
               "generation_kernel_ms_max": round(gmax[3], 2),
               "generation_steps": int(gsum[0]),
               "generation_walk_steps_per_s": round(gsum[0] / (gmax[1] * 1e-3), 1),
               "first_generation_anchor_inits": int(gsum[1]),
               "device_bytes_rank0": g.memory_footprint(verbose=False)["total_bytes"]}
        if args.job_gather and dist:
            free = torch.cuda.mem_get_info(dev)[0] if comm_dev != "cpu" else (8 << 30)
            # this rank's budget; corpus_gather_record agrees the chunk (minimum over the ranks)
            budget = max(64 << 20, min(args.gather_chunk_bytes, free // 4))
            rec["corpus_allgatherv"] = corpus_gather_record(args, torch, dist, g, shards[:world], n, 10, 80, dev,
                                                            comm_dev, world, rank, barrier, budget, mem)
        with phase("ids"):
            ids = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device=f"cuda:{dev}")
        per = {k: [] for k in ("wall", "graph", "walk", "in_edge", "steps", "affected", "inits")}
        for b in range(args.job_batches):
            for ins in ((True, False) if spec["mixed"] else (True,)):
                barrier()
                with phase(f"batch {b} {'insert' if ins else 'delete'}"):
                    batch = W.generate_batch_of_edges(5000, n, b, False, False, device=dev)
                    t1 = time.perf_counter()
                    (g.insert_edges_batch if ins else g.delete_edges_batch)(batch, remove_dups=True, out=ids)
                    torch.cuda.synchronize(dev)
                    per["wall"].append((time.perf_counter() - t1) * 1e3)
                    st = g.stats()
                    per["graph"].append(st["last_graph_update_ms"])
                    per["walk"].append(st["last_walk_update_ms"])
                    per["in_edge"].append(st["last_csr_move_ms"])
                    per["steps"].append(st["steps"])
                    per["affected"].append(st["affected"])
                    per["inits"].append(st["last_anchor_inits"])
                    mem.probe(f"batch {b} {'insert' if ins else 'delete'}")
        if per["wall"]:
            job_ms = _max_over_ranks(torch, dist, comm_dev, per["wall"])
            steps = _sum_over_ranks(torch, dist, comm_dev, per["steps"])
            med = lambda k: float(np.median(per[k]))
            ranks = _per_rank(torch, dist, comm_dev, [med("wall"), med("graph"), med("walk"), med("in_edge"),
                                                     float(np.sum(per["steps"])), float(np.sum(per["walk"]))], world)
            rec.update({
                "updates": len(job_ms), "batch_median_ms": round(float(np.median(job_ms)), 3),
                "batch_p90_ms": round(float(np.percentile(job_ms, 90)), 3),
                "rewalk_walk_steps_per_update": int(np.mean(steps)),
                "rewalk_walk_steps_per_s": round(float(np.sum(steps) / (np.sum(job_ms) * 1e-3)), 1),
                "per_rank": {"batch_median_ms": [round(r[0], 3) for r in ranks],
                             "graph_update_median_ms": [round(r[1], 3) for r in ranks],
                             "walk_update_median_ms": [round(r[2], 3) for r in ranks],
                             "in_edge_scan_median_ms": [round(r[3], 3) for r in ranks],
                             "rewalk_Gsteps_per_s": [round(r[4] / r[5] / 1e6, 2) if r[5] else None for r in ranks]},
                "rank_balance_max_over_min": round(max(r[0] for r in ranks) / max(min(r[0] for r in ranks), 1e-9), 3),
                "mean_affected_walks_rank0": int(np.mean(per["affected"])),
                "mean_anchor_inits_rank0": int(np.mean(per["inits"]))})
        if spec["split"] == "ranks" and world > 1 and args.job_one_gpu:
            # the same graph (after this job's batches) with every walk on rank 0's GPU
            one = None
            barrier()
            with phase("one_gpu"):
                if rank == 0:
                    g.set_shard(0, n)
                    g.generate_initial_random_walks()
                    g.generate_initial_random_walks()
                    st = g.stats()
                    ids = torch.empty(max(g.number_of_walks, 1), dtype=torch.int32, device=f"cuda:{dev}")
                    o = _update_stream_from(g, W, n, args.job_batches, args.job_batches, spec["mixed"], ids, dev)
                    one = {"walks": g.number_of_walks, "generation_ms": round(st["last_walk_kernel_ms"], 2),
                           "batch_median_ms": o["batch_median_ms"], "graph_update_median_ms": o["graph_update_median_ms"],
                           "walk_update_median_ms": o["walk_update_median_ms"],
                           "batches": f"generate_batch_of_edges(5000, n, b, false, undirected), "
                                      f"b = {args.job_batches}..{2 * args.job_batches - 1}"}
            if one is not None:
                rec["one_gpu_same_graph"] = one
                if "batch_median_ms" in rec:
                    rec["batch_ratio_one_gpu_to_job"] = round(one["batch_median_ms"] / rec["batch_median_ms"], 2)
                rec["generation_ratio_one_gpu_to_job"] = round(one["generation_ms"] / rec["generation_kernel_ms_max"], 2)
        low = mem.record()
        if low:   # every rank's peak: the job fits where the largest does
            peaks = _per_rank(torch, dist, comm_dev, [float(low["peak_used_bytes"]), float(low["min_free_bytes"])],
                              world)
            low["peak_used_bytes_per_rank"] = [int(p[0]) for p in peaks]
            low["min_free_bytes_per_rank"] = [int(p[1]) for p in peaks]
            rec["device_memory"] = low
        return rec
    except RankFailure as ex:   # every rank is here together: the job is abandoned, the headline still prints
        log(f"[rank {rank}] job {name} abandoned: {ex}")
        return {"error": str(ex)[:500], "failed_rank": ex.rank, "phase": ex.phase}
    except Exception as ex:   # noqa: BLE001 (one process: a job that does not fit is reported)
        log(f"[rank {rank}] job {name} failed: {ex}")
        return {"error": str(ex)[:500]}
    finally:
        if g is not None:
            g.destroy()
        torch.cuda.empty_cache()


def _update_stream_from(g, W, n, first, batches, mixed, out, dev):
    """_update_stream over batch seeds first .. first + batches - 1."""
    lat, gu, wu = [], [], []
    for b in range(first, first + batches):
        batch = W.generate_batch_of_edges(5000, n, b, False, False, device=dev)
        for ins in ((True, False) if mixed else (True,)):
            t1 = time.perf_counter()
            (g.insert_edges_batch if ins else g.delete_edges_batch)(batch, remove_dups=True, out=out)
            lat.append((time.perf_counter() - t1) * 1e3)
            st = g.stats()
            gu.append(st["last_graph_update_ms"])
            wu.append(st["last_walk_update_ms"])
    return {"batch_median_ms": round(float(np.median(lat)), 3), "graph_update_median_ms": round(float(np.median(gu)), 3),
            "walk_update_median_ms": round(float(np.median(wu)), 3)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    # one process per GPU; more ranks than GPUs (a 1-GPU rehearsal) share devices round-robin
    dev = local % max(torch.cuda.device_count(), 1)
    backend = os.environ.get("WHARF_DIST_BACKEND", "nccl")   # gloo: rehearsal of the N>1 path on one GPU
    comm_dev = "cpu" if backend == "gloo" else f"cuda:{dev}"
    if world > 1 or args.init_dist:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    import dynamicgraphrepresentationlearning_amd as W

    # the box's random-gather rate, probed on the idle GPU before anything is timed
    live_ceiling = measure_gather_ceiling(args.gather_probes) if rank == 0 and args.gather_probes > 0 else None
    if live_ceiling:
        log(f"gather_roof probes (G gathers/s): {live_ceiling}")

    # weak scaling: configs[1]'s graph, 10 x N walks per vertex, so each rank's
    # start-vertex range carries configs[1]'s 41.9 M walks
    weak = args.scaling == "weak"
    wpv = args.wpv * world if weak else args.wpv
    if wpv > 255:
        raise SystemExit(f"walks_per_vertex {wpv} exceeds the reference's u8 config::walks_per_vertex")
    n = 1 << args.scale
    model = W.NODE2VEC if args.model == "node2vec" else W.DEEPWALK
    cfg = W.WharfConfig(walks_per_vertex=wpv, walk_length=args.length, model=model,
                        paramP=args.paramP, paramQ=args.paramQ, deterministic=args.det, seed=0x5EED)
    t0 = time.time()
    g = W.WharfMH.from_rmat(n, args.samples, 2 * n, seed=args.seed, config=cfg, device=dev)
    # the whole CSR on the host only where the CPU baseline may need it (N = 1)
    off, adj = g.flatten_graph() if world == 1 else (g.offsets(), None)
    deg = np.diff(off.astype(np.int64))
    shards = balanced_shards(deg, world)
    lo, hi = shards[rank]
    g.set_shard(lo, hi)
    m = g.number_of_edges()
    log(f"[rank {rank}] graph n={n} m={m} built in {time.time() - t0:.1f}s; shard [{lo},{hi}), wpv={wpv}")
    # the same probe over a table the size of this graph's edge records (8 B per slot when compact, 16 B
    # otherwise): the 3.48-GiB probe above is the box's yardstick, this one the kernel's own table size
    matched = None
    if live_ceiling:
        table_gib = (g.memory_footprint(verbose=False)["records_bytes"] - 16 * n) / 2 ** 30
        matched = {"table_GiB": round(table_gib, 3),
                   "probes": measure_gather_ceiling(args.gather_probes, table_gib)}
        log(f"gather_roof probes at the record table's size ({table_gib:.2f} GiB): {matched['probes']}")

    def barrier():
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)

    elapsed, kern_ms, warm_ms = timed_generation(g, args.steps, args.warmup, barrier, rank)
    st = g.stats()
    steps_local = st["steps"]
    steps_total, t_max = reduce_steps_time(torch, dist, comm_dev, steps_local, elapsed)
    value = steps_total * args.steps / t_max
    avg_kernel_ms = float(np.mean(kern_ms))
    bytes_per_step = BYTES_PER_STEP_DEEPWALK if args.model == "deepwalk" or args.det else BYTES_PER_STEP_NODE2VEC
    tag = f"gen_{args.model}_{'det' if args.det else 'mh'}_s{args.scale}"

    # corpus reassembly for the downstream consumer: bounded full-mesh all-gatherv over RCCL (not timed in `value`)
    corpus = None
    if dist:
        from dynamicgraphrepresentationlearning_amd.distributed import RankFailure
        free = torch.cuda.mem_get_info(dev)[0] if comm_dev != "cpu" else (8 << 30)
        try:   # the budget is this rank's; the chunk is agreed over the ranks inside
            corpus = corpus_gather_record(args, torch, dist, g, shards, n, wpv, args.length, dev, comm_dev, world,
                                          rank, barrier, max(64 << 20, min(args.gather_chunk_bytes, free // 4)))
        except RankFailure as ex:   # every rank abandons the gather together; the headline still prints
            corpus = {"error": str(ex)[:500], "failed_rank": ex.rank, "phase": ex.phase}
    g.destroy()

    # strong scaling beside the weak line: configs[1] exactly (10 walks per vertex) split N ways
    strong = None
    if world > 1 and weak:
        cfg1 = W.WharfConfig(walks_per_vertex=args.wpv, walk_length=args.length, model=model,
                             paramP=args.paramP, paramQ=args.paramQ, deterministic=args.det, seed=0x5EED)
        g1 = W.WharfMH.from_rmat(n, args.samples, 2 * n, seed=args.seed, config=cfg1, device=dev)
        g1.set_shard(lo, hi)
        e1, k1, _ = timed_generation(g1, args.steps, 1, barrier)
        st1, tm1 = reduce_steps_time(torch, dist, comm_dev, g1.stats()["steps"], e1)
        strong = {"workload": f"configs[1] exactly (walks_per_vertex={args.wpv}) split over {world} ranks",
                  "value": round(st1 * args.steps / tm1, 1), "unit": "walk-steps/s",
                  "ms_per_step": round(tm1 / args.steps * 1e3, 3), "transitions_per_step": st1,
                  "avg_kernel_ms_rank0": round(float(np.mean(k1)), 3)}
        g1.destroy()

    # configs[2]: soc-LiveJournal-sized streaming, 10k-edge insert batches, in the
    # benchmarked mode and (DeepWalk MH runs) in deterministic mode, the reference's default
    cfg2 = W.WharfConfig(walks_per_vertex=args.wpv, walk_length=args.length, model=model,
                         paramP=args.paramP, paramQ=args.paramQ, deterministic=args.det, seed=0x5EED)
    rewalk = stream_latency(args, W, torch, cfg2, dev, world, rank, dist, comm_dev, barrier, args.rewalk_batches)
    rewalk_det = None
    if args.det_rewalk_batches > 0 and not args.det and args.model == "deepwalk":
        cfg_det = W.WharfConfig(walks_per_vertex=args.wpv, walk_length=args.length, model=W.DEEPWALK,
                                deterministic=True)
        rewalk_det = stream_latency(args, W, torch, cfg_det, dev, world, rank, dist, comm_dev, barrier,
                                    args.det_rewalk_batches, scan_batches=3)
    n2v = None
    if world == 1 and args.model == "deepwalk" and not args.det and args.n2v_steps > 0:
        n2v = node2vec_record(args, W, torch, dev, barrier, n)

    per8 = None
    if world == 1 and args.per_gpu_of_8 and args.model == "deepwalk" and not args.det:
        torch.cuda.empty_cache()
        per8 = per_gpu_of_8(args, W, torch, dev, barrier)

    # BASELINE's two 8-GPU jobs on the ranks of this run (configs[3] strong, configs[4] g-of-8 weak)
    jobs = None
    if (world > 1 or dist) and args.jobs and args.model == "deepwalk" and not args.det:
        jobs = {}
        for name in [j for j in args.jobs.split(",") if j]:
            torch.cuda.empty_cache()
            jobs[name] = multi_gpu_job(args, name, W, torch, dev, world, rank, dist, comm_dev, barrier)
            log(f"[rank {rank}] job {name}: {json.dumps(jobs[name])}")

    if rank == 0:
        if rewalk and live_ceiling and bytes_per_step == BYTES_PER_STEP_DEEPWALK:
            # re-walk steps (one gather each) against the same yardstick, with the probes' spread: the
            # probe is a yardstick for the box, not a roof (a ratio above 1 is within its spread)
            rewalk["rewalk_vs_gather_probes"] = {
                "probe_Ggathers_per_s_min": round(min(live_ceiling), 2),
                "probe_Ggathers_per_s_max": round(max(live_ceiling), 2),
                "ratio_to_max_probe": round(rewalk["rewalk_Gsteps_per_s"] / max(live_ceiling), 4),
                "ratio_to_min_probe": round(rewalk["rewalk_Gsteps_per_s"] / min(live_ceiling), 4)}
        achieved = (steps_local * bytes_per_step / (avg_kernel_ms * 1e-3) / 1e9) if bytes_per_step else None
        traffic, traffic_src = load_traffic(tag)
        line = {
            "metric": "MH walk-steps/sec" if not args.det else "deterministic walk-steps/sec",
            "value": round(value, 1),
            "unit": "walk-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic RMAT (utility::generate_batch_of_edges semantics, a=.5 b=.2 c=.1), built on device",
            "config": {"workload": f"configs[1] com-orkut-sized initial walk generation: RMAT scale {args.scale} "
                                   f"(n={n}), {args.samples} undirected samples (seed {args.seed}) -> m={m} CSR "
                                   f"entries; {args.model} {'deterministic' if args.det else 'MH'}, "
                                   f"walks_per_vertex={wpv}"
                                   f"{f' ({args.wpv} per GPU x {world}: weak scaling)' if weak and world > 1 else ''}"
                                   f", walk_length={args.length}",
                       "n": n, "m": m, "walks": n * wpv, "transitions_per_step": steps_total,
                       "parallelism": f"walk shards by start-vertex range x{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_walk (generation)",
                         "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         # the PMC bytes per launch moved in this run's average launch time: how close the
                         # random line fetches run to the HBM peak (frac is by algorithmic bytes)
                         "traffic_GBps": round(traffic / (avg_kernel_ms * 1e-3) / 1e9, 1) if traffic else None,
                         "traffic_frac_of_peak": round(traffic / (avg_kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                         if traffic else None,
                         "bytes_per_step": bytes_per_step,
                         "avg_kernel_ms": round(avg_kernel_ms, 3),
                         # the first generation of a fresh handle (node2vec: every anchor initialised)
                         "first_generation_kernel_ms": round(warm_ms[0], 3) if warm_ms else None,
                         "gather_ceiling": gather_ceiling(steps_local / (avg_kernel_ms * 1e-3), live_ceiling, matched)
                         if bytes_per_step == BYTES_PER_STEP_DEEPWALK else None,
                         # L2 requests: one per step at the path's measured request-rate ceiling
                         "l2_requests": request_rate(load_requests(tag), steps_local, avg_kernel_ms)},
            "per_gpu_of_8": per8,
            "jobs_8gpu": jobs,
            "mh_accept_rate": round(st["accepts"] / st["steps"], 5) if st["steps"] else None,
            "strong_scaling": strong,
            "mh_node2vec": n2v,
            "rewalk_latency_10k_batch": rewalk,
            "rewalk_latency_10k_batch_deterministic": rewalk_det,
            "streaming_rooflines": streaming_rooflines(rewalk, rewalk_det, args.scale),
            "corpus_allgatherv": corpus,
            "dist_backend": (backend if backend == "gloo" else "nccl (RCCL)") if dist else None,
            "cpu_baseline": None,
        }
        if world == 1 and args.cpu_baseline != "off":
            active = int((deg > 0).sum())
            ext = cpu_baseline(args, n, active, off, adj, args.cpu_baseline)
            same = None
            if args.cpu_baseline in ("auto", "reference") and args.cpu_scale > 0:
                try:
                    same = cpu_baseline_same_shape(args, W, torch, dev, ext)
                except Exception as ex:   # noqa: BLE001 (the extrapolated sample stays the baseline)
                    log(f"cpu_baseline (same shape) failed: {ex}")
            line["cpu_baseline"] = same or ext
            if args.cpu_baseline in ("auto", "reference") and args.det_rewalk_batches > 0:
                ext_det = cpu_baseline_deterministic(args, batches=1)
                try:
                    line["cpu_baseline_deterministic"] = cpu_baseline_deterministic_same_shape(args, W, torch, dev,
                                                                                               ext_det)
                except Exception as ex:   # noqa: BLE001 (the extrapolated sample stays the baseline)
                    log(f"cpu_baseline_deterministic (same shape) failed: {ex}")
                    line["cpu_baseline_deterministic"] = ext_det
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
