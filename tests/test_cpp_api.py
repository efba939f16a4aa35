"""C++ host API (include/etcd_quorum.hpp) — the reference's TestDataDriven
(raft/quorum/datadriven_test.go) and TestLeaderElectionInOneRoundRPC
(raft/raft_paper_test.go:192-232) restated in tests/cpp/quorum_golden_test.cpp
and run through the GPU kernels."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "quorum_golden_test")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])


def test_cpp_test_builds_and_links():
    if not os.path.exists(os.path.join(ROOT, "etcd_amd", "lib", "libetcd_quorum.so")):
        pytest.skip("library not built")
    _build()
    assert os.access(BIN, os.X_OK)
    out = subprocess.run(["nm", "-DC", os.path.join(ROOT, "etcd_amd", "lib", "libetcd_quorum.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ("etcd_amd::quorum::MajorityConfig::CommittedIndex",
                "etcd_amd::quorum::JointConfig::VoteResult",
                "etcd_amd::quorum::CommittedIndexBatch",
                "etcd_amd::tracker::ProgressTracker::TallyVotes",
                "etcd_amd::tracker::ProgressTracker::QuorumActive",
                "etcd_amd::confchange::Changer::EnterJoint",
                "etcd_amd::confchange::ChangeBatch"):
        assert sym in out, sym


@pytest.mark.gpu
def test_cpp_datadriven_on_gpu():
    _build()
    r = subprocess.run([BIN, ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS: 127 datadriven cases, 13 election rows" in r.stdout


@pytest.mark.gpu
def test_cpp_confchange_datadriven_on_gpu():
    """TestConfChangeDataDriven (raft/confchange/datadriven_test.go) through
    etcd_amd::confchange::Changer and the qe_confchange kernel."""
    _build()
    exe = os.path.join(ROOT, "tests", "cpp", "build", "confchange_golden_test")
    r = subprocess.run([exe, ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS: 58 confchange steps" in r.stdout


def test_cpp_describe_matches_testdata():
    """etcd_amd::quorum::{Majority,Joint}Config::Describe (host text
    rendering, majority.go:45-101) against the 66 texts the reference's
    datadriven harness printed (tests/golden/describe_testdata.txt)."""
    if not os.path.exists(os.path.join(ROOT, "etcd_amd", "lib", "libetcd_quorum.so")):
        pytest.skip("library not built")
    _build()
    exe = os.path.join(ROOT, "tests", "cpp", "build", "describe_test")
    r = subprocess.run([exe, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS: 66 Describe cases" in r.stdout
