"""bench.py's multi-GPU plumbing on the CPU: the rank launcher (`--gpus N` without
WORLD_SIZE starts N processes with the torch.distributed.run environment), the all-gather
of per-problem summaries that bench.py runs over RCCL after the timed region (here gloo,
world size 2 and 3, ragged shards), failure propagation, and the WORLD_SIZE / --gpus
consistency check."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "_rank_probe.py")


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as B
    return B


@pytest.mark.parametrize("world,gb", [(2, 6), (3, 10)])
def test_launcher_gathers_every_rank(bench, tmp_path, world, gb):
    out = str(tmp_path / "g.npy")
    assert bench.launch_ranks(world, script=PROBE, argv=[out, str(world), str(gb)]) == 0
    g = np.load(out)
    np.testing.assert_array_equal(g["index"], np.arange(gb))
    np.testing.assert_array_equal(g["J"], np.sqrt(np.arange(gb) + 1.0))
    np.testing.assert_array_equal(g["status"], np.arange(gb) % 3)
    np.testing.assert_array_equal(g["trace"][:, 5], np.arange(gb) * 7 + 5)


def test_launcher_propagates_a_failing_rank(bench, tmp_path):
    # rank 1 exits before joining the group: rank 0 would wait forever in init, so the
    # launcher must stop it and report rank 1's exit code
    rc = bench.launch_ranks(2, script=PROBE, argv=[str(tmp_path / "x.npy"), "2", "4", "1"])
    assert rc == 3


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_usable_cpus_is_positive(bench):
    n = bench.usable_cpus()
    assert 1 <= n <= (os.cpu_count() or n)


def test_knot_steps_per_rollout(bench):
    """SURVEY.md 8(d)'s knot-steps diagnostic: C3 rolls 4 x 79 knots per rollout, C5 (N = 80,
    100 alternating over 10 phases) 5 x 79 + 5 x 99; the mixed workload reports none."""
    from mhpc_minimal_env_amd import configs
    assert bench.knot_steps_per_rollout("c3", configs.c3_desc()) == 316
    d5 = configs.c5_desc()
    assert bench.knot_steps_per_rollout("c5", d5) == sum(d5.N[p] - 1 for p in range(10))
    assert bench.knot_steps_per_rollout("c5", d5) == 5 * 79 + 5 * 99
    assert bench.knot_steps_per_rollout("mixed", configs.c3_desc()) == 0
