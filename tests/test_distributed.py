"""N > 1 path on CPU: world_size-2 gloo process group, contiguous batch shards solved
independently (CPU oracle standing in for the per-GPU solver) and the per-problem
summaries all-gathered -- identical, problem for problem, to the 1-process solve."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, global_batch, out_path):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from mhpc_minimal_env_amd import configs, locomotion as L, sharding
    desc = configs.c3_desc()
    off, cnt = sharding.shard_offsets(global_batch, world, rank)
    x0 = configs.x0_for(desc, cnt, offset=off)
    r = O.solve(desc, L.HSDDP_OPTION().to_c(), x0, nthreads=2)
    local = sharding.make_summary(off, r["J"], r["viol"], r["status"], r["V"], r["trace"])
    allp = sharding.gather_summaries(local)
    if rank == 0:
        np.save(out_path, allp)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_offsets_cover_batch():
    from mhpc_minimal_env_amd import sharding
    for gb in (1, 7, 8, 1024, 8193):
        for world in (1, 2, 3, 8):
            spans = [sharding.shard_offsets(gb, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == gb
            pos = 0
            for off, c in spans:
                assert off == pos
                pos += c


@pytest.mark.skipif(not __import__("oracle").available(), reason="oracle not built")
def test_two_rank_gloo_matches_single_process(tmp_path):
    import oracle as O
    from mhpc_minimal_env_amd import configs, locomotion as L
    gb = 6
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(2, _free_port(), gb, out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    desc = configs.c3_desc()
    ref = O.solve(desc, L.HSDDP_OPTION().to_c(), configs.x0_for(desc, gb), nthreads=2)
    np.testing.assert_array_equal(got["index"], np.arange(gb))
    np.testing.assert_array_equal(got["trace"], ref["trace"])
    np.testing.assert_array_equal(got["J"], ref["J"])
    np.testing.assert_array_equal(got["V"], ref["V"])
