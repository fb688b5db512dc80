"""The RCCL (`nccl`) leg of the multi-GPU path, executed on the one-GPU box.

RCCL refuses two ranks on one device, so a world of one is the only way to run
these lines before the driver's 8-GPU bench (missing #1):
  * tests/rccl_world1_worker.py: init_process_group("nccl", device_id=...),
    bench.py's device collectives and barrier, the chunked corpus gather
    (all-gatherv and gatherv) with device buffers, and a self-peer
    batch_isend_irecv (outcome recorded, not asserted);
  * bench.py --init-dist at N = 1 with both 8-GPU jobs shrunk by
    --job-scale-delta -6: multi_gpu_job end to end over RCCL (generation, the
    bounded gather with its checksum of checksums, update batches, the per-rank
    all-gathers of the records).
Set WHARF_TEST_ARTIFACTS=<dir> to keep the worker report and the bench line."""
import json
import os
import shutil
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, timeout):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", WHARF_DIST_BACKEND="nccl", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", *args]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=REPO)


def _keep(name, text):
    d = os.environ.get("WHARF_TEST_ARTIFACTS")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name), "w") as f:
            f.write(text)


def test_rccl_world1_collectives_and_chunked_gather(tmp_path):
    out = tmp_path / "rccl.json"
    r = _torchrun([os.path.join(HERE, "rccl_world1_worker.py"), str(out)], 240)
    _keep("rccl_world1_worker.log", r.stdout + "\n--- stderr ---\n" + r.stderr)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rep = json.load(open(out))
    _keep("rccl_world1_worker.json", json.dumps(rep, indent=1))
    assert rep["backend"] == "nccl" and rep["world"] == 1
    assert rep["collectives_ok"], rep
    assert rep["corpus_gather_record"]["checksum_of_checksums_ok"], rep
    assert rep["corpus_gather_record"]["backend"].startswith("nccl")
    assert rep["chunked_gather_eq_export"] and rep["gatherv_eq_export"], rep
    assert rep["chunked_gather_chunks"] >= 2
    assert "self_p2p" in rep   # accepted or refused: recorded, not required


def test_bench_jobs_over_rccl_at_world1(tmp_path):
    args = [os.path.join(REPO, "bench.py"), "--gpus", "1", "--init-dist", "--steps", "1", "--warmup", "1",
            "--scale", "16", "--samples", "400000", "--rewalk-batches", "2", "--det-rewalk-batches", "0",
            "--n2v-steps", "0", "--per-gpu-of-8", "0", "--gather-probes", "0", "--cpu-baseline", "off",
            "--job-scale-delta", "-6", "--job-batches", "2", "--gather-chunk-bytes", str(64 << 20)]
    r = _torchrun(args, 420)
    _keep("bench_init_dist_world1.log", r.stdout + "\n--- stderr ---\n" + r.stderr)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["dist_backend"].startswith("nccl") and line["n_gpus"] == 1
    assert line["corpus_allgatherv"]["checksum_of_checksums_ok"]
    for job in ("configs3", "configs4"):
        rec = line["jobs_8gpu"][job]
        assert "error" not in rec, rec
        assert rec["updates"] == (4 if job == "configs4" else 2)
        assert rec["corpus_allgatherv"]["checksum_of_checksums_ok"], rec
        assert rec["generation_steps"] > 0 and rec["rewalk_walk_steps_per_update"] > 0
