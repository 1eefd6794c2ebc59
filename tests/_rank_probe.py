"""Helper rank of tests/test_bench_launcher.py (not a test): joins a gloo group from the
environment bench.launch_ranks sets, all-gathers per-problem summaries through
mhpc_minimal_env_amd.sharding exactly as bench.py does with RCCL, rank 0 saves them.
usage: _rank_probe.py <out.npy> <expected world> <global batch> [fail-rank]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, want, gb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    fail = int(sys.argv[4]) if len(sys.argv) > 4 else -1
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert world == want and int(os.environ["LOCAL_RANK"]) == rank
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    if rank == fail:
        sys.exit(3)
    import torch.distributed as dist
    from mhpc_minimal_env_amd import sharding
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = sharding.shard_offsets(gb, world, rank)
    idx = np.arange(off, off + cnt)
    J = np.sqrt(idx + 1.0)
    V = np.stack([J, -J], axis=1)
    trace = (idx[:, None] * 7 + np.arange(64)[None, :]).astype(np.int32)
    local = sharding.make_summary(off, J, J / 3, (idx % 3).astype(np.int32), V, trace)
    allp = sharding.gather_summaries(local)
    if rank == 0:
        np.save(out, allp)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
