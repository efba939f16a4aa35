"""The engine's multi-rank path, end to end through bench.py: `--gpus 2`
relaunches itself as two ranks (torch.distributed.run, spawned before any
GPU call), each rank evaluates its shard [r*G, (r+1)*G) through
group_offset, and the statistics are all-reduced.  On a 1-GPU box both ranks
share cuda:0 and reduce with gloo (QE_DEVICE_MOD=1, QE_DIST_BACKEND=gloo);
the driver's 8-GPU run uses RCCL through qe_allreduce_stats.  The aggregated
checksum must equal one process over the union of the shards."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("workload", ["config2_n5", "config4_repl", "config5_prevote_cq",
                                      "progress_step"])
def test_two_ranks_equal_one_process_over_the_union(workload):
    G = 1 << 18
    common = ["--workload", workload, "--no-aux", "--no-cpu-baseline", "--steps", "3",
              "--warmup", "1"]
    two = _bench(["--gpus", "2", "--groups", str(G)] + common,
                 {"QE_DEVICE_MOD": "1", "QE_DIST_BACKEND": "gloo"})
    one = _bench(["--gpus", "1", "--groups", str(2 * G)] + common, {})
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["global_groups"] == one["config"]["global_groups"] == 2 * G
    # inputs (the Progress workload's state and messages too: bench.py
    # counter_rows) and the election RNG are keyed by the global group id, so
    # the sharded run and the union agree launch for launch
    assert two["checks"]["stats_checksum"] == one["checks"]["stats_checksum"]
    assert two["checks"]["invariant_violations"] == 0


def test_gpus_mismatch_fails():
    """WORLD_SIZE set by a launcher that disagrees with --gpus: exit 2."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--no-aux", "--no-cpu-baseline", "--groups", "4096", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=120, env=env,
                       cwd=ROOT)
    assert r.returncode == 2, r.stdout + r.stderr
