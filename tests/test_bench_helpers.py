"""bench.py's host-side helpers that shape the JSON line (CPU only, no GPU, no library calls):
the gather-ceiling record, the committed PMC traffic lookup, the record-bytes readout and
the host CPU accounting behind `cpu_baseline.cores`."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_gather_ceiling_fractions_and_table_matched_probe():
    assert bench.gather_ceiling(45e9, None) is None
    rec = bench.gather_ceiling(45e9, [40.0, 45.0], {"table_GiB": 1.981, "probes": [44.0, 50.0]})
    assert rec["Ggathers_per_s_min"] == 40.0 and rec["Ggathers_per_s_max"] == 45.0
    assert rec["frac_of_min"] == pytest.approx(45 / 40, abs=1e-4)
    assert rec["frac_of_max"] == pytest.approx(1.0, abs=1e-4)
    tm = rec["table_matched"]
    assert tm["table_GiB"] == 1.981 and tm["probes"] == [44.0, 50.0]
    assert tm["frac_of_min"] == pytest.approx(45 / 44, abs=1e-4) and tm["frac_of_max"] == pytest.approx(0.9, abs=1e-4)
    # a matched record without probes (the probe binary missing) adds nothing
    assert "table_matched" not in bench.gather_ceiling(45e9, [40.0], {"table_GiB": 2.0, "probes": None})


def test_traffic_comes_from_the_newest_committed_pmc_summary():
    traffic, src = bench.load_traffic("gen_deepwalk_mh_s22")
    assert src.startswith(f"profiles/pmc_{bench.PMC_ROUNDS[0]}gen_deepwalk_mh_s22.json")
    with open(os.path.join(REPO, src.split(" ")[0])) as f:
        assert traffic == json.load(f)["hbm_bytes_per_launch"] > 0
    assert bench.load_traffic("no_such_kernel_tag") == (None, None)


class _Handle:
    """What record_bytes_per_slot reads: records_bytes = 16 B per vertex (vrec) + the edge
    records of every pool slot (the footprint counts node2vec's anchor half as samplers)."""

    def __init__(self, n, pool, per_slot):
        self.n, self.pool, self.per_slot = n, pool, per_slot

    def memory_footprint(self, verbose=False):
        return {"records_bytes": 16 * self.n + self.per_slot * self.pool}

    def stats(self):
        return {"pool_capacity": self.pool}


@pytest.mark.parametrize("per_slot,anchors,want", [(8, False, 8), (16, False, 16), (16, True, 32)])
def test_record_bytes_per_slot(per_slot, anchors, want):
    assert bench.record_bytes_per_slot(_Handle(1 << 12, 5 << 12, per_slot), 1 << 12, anchors) == want


def test_cpu_cores_respects_an_explicit_request_and_the_host_share():
    info = bench.host_cpus()
    assert 1 <= info["usable"] <= info["nproc"]
    assert bench.cpu_cores(3) == 3
    assert bench.cpu_cores(0) == info["usable"]


def test_l2_request_rate_from_the_committed_summary():
    req = bench.load_requests("gen_deepwalk_mh_s22")
    assert req is not None and 1.0 <= req["per_step"] < 1.2 and req["source"].startswith("profiles/pmc_")
    rec = bench.request_rate(req, 3_297_052_360, 76.2)
    assert rec["G_per_s"] == pytest.approx(req["per_step"] * 3_297_052_360 / 0.0762 / 1e9, rel=1e-3)
    assert rec["path_kernels_measured_G_per_s"] == [40, 47]
    assert bench.load_requests("no_such_kernel_tag") is None and bench.request_rate(None, 1, 1.0) is None
