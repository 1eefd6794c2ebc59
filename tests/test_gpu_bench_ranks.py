"""bench.py's N-rank path with the product library on one GPU: `--gpus 2` starts two ranks
itself (no WORLD_SIZE), each solves its contiguous shard through libmhpc_amd, the summaries
are all-gathered and rank 0 checks them bitwise against a 1-GPU solve of the global batch
(SURVEY.md 8e).  On a 1-GPU box both ranks share GPU 0 and the group is gloo; on a node the
same code runs one rank per GPU over RCCL."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_shard_and_gather(need_gpu):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--share-gpu", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "61",
           "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 122
    assert d["sharding"]["ranks"] == 2 and d["sharding"]["gathered_problems"] == 122
    assert d["sharding"]["check"]["bitwise_identical_to_1gpu"] is True


def test_rccl_group_world_one(need_gpu):
    """The RCCL (nccl) branch on one GPU: `--dist` under torch.distributed.run at world size 1
    (init with device_id, device-tensor timing reductions, summary all-gather, shard check).
    stdout must be exactly the JSON line: RCCL's version banner goes to stderr."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29533",
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist", "--steps", "2",
           "--warmup", "1", "--batch-per-gpu", "37", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    d = json.loads(lines[0])
    assert d["sharding"]["backend"] == "nccl" and d["sharding"]["gathered_problems"] == 37
    assert d["sharding"]["check"]["bitwise_identical_to_1gpu"] is True
