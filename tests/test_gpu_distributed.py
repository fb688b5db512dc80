"""Multi-process HIP path on the GPU box: N ranks (gloo, one process each), every
rank with its own libwharf_gpu.so handle over its start-vertex shard, corpus
reassembled by distributed.allgatherv_corpus from device exports and by the
bounded distributed.gather_corpus_chunked from per-chunk device row exports — bit-exact
against one unsharded handle and the CPU oracle after generation and after
every batch of a configs[4]-shaped node2vec MH stream (mixed insert/delete) and
a configs[3]-shaped deterministic DeepWalk stream.  (The RCCL backend runs the
same code at the driver's N = 2..8; here the ranks share the one GPU.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["node2vec", "det"])
def test_sharded_handles_reproduce_the_single_corpus(tmp_path, mode, world):
    out = tmp_path / "report.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "dist_shard_worker.py"), mode, str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rep = json.load(open(out))
    assert rep["world"] == world and len(rep["steps"]) >= 5
    for st in rep["steps"]:
        assert st["corpus_eq_single"] and st["corpus_eq_oracle"] and st["steps_eq"] and st["chunked_eq"], st
        assert st.get("affected_eq", True), st
