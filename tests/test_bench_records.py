"""The committed measurement records bench.py reads (CPU only): every bench
workload has a rocprofv3 PMC record (profiles/pmc_traffic.json, folded by
scripts/summarize_workloads.py) whose memory traffic is at or above its
algorithmic bytes, and whose kernel has an occupancy record
(profiles/kernel_resources.json, scripts/kernel_resources.py), so the aux
line's `vmem_issue` and `occupancy` describe the kernels that exist."""
import importlib
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAFFIC = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
bench = importlib.import_module("bench")


@pytest.mark.parametrize("wl", sorted(bench.WORKLOADS))
def test_workload_has_pmc_record(wl):
    t = TRAFFIC.get(wl)
    assert t, f"{wl}: no PMC record"
    assert os.path.exists(os.path.join(ROOT, t["profile"]))
    assert t["fetch_factor"] == 2  # reads = 2 x FETCH_SIZE (profiles/r04/pmc_calib.json)
    if "algorithmic_bytes_per_launch" in t:
        assert t["hbm_bytes_per_launch"] >= 0.995 * t["algorithmic_bytes_per_launch"]


@pytest.mark.parametrize("wl", sorted(bench.WORKLOADS))
def test_workload_has_occupancy_record(wl):
    oc = bench.occupancy(wl)
    assert oc, f"{wl}: its PMC kernel {TRAFFIC.get(wl, {}).get('kernel')} has no resource record"
    for rec in oc.values():
        assert 1 <= rec["waves_per_simd"] <= 8
