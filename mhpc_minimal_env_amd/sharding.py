"""Batch sharding over GPUs.

Problems are independent, so a global batch is split into contiguous blocks, one per rank
(one process per GPU); the solve itself has no exchange.  The only collective is the
optional gather of per-problem summaries (J, status, trace) at the end, done with
torch.distributed (RCCL over xGMI with backend "nccl" on MI355X; gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_offsets(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous block; the remainder goes to the first ranks."""
    base, rem = divmod(global_batch, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def summary_dtype(n_phases: int, trace_len: int):
    return np.dtype([("index", np.int64), ("J", np.float64), ("viol", np.float64),
                     ("status", np.int32), ("V", np.float64, (n_phases,)),
                     ("trace", np.int32, (trace_len,))])


def make_summary(offset: int, J, viol, status, V, trace) -> np.ndarray:
    n = len(J)
    s = np.zeros(n, dtype=summary_dtype(V.shape[1], trace.shape[1]))
    s["index"] = np.arange(offset, offset + n)
    s["J"], s["viol"], s["status"], s["V"], s["trace"] = J, viol, status, V, trace
    return s


def gather_summaries(local: np.ndarray, device=None) -> np.ndarray:
    """All-gather the per-problem summaries of every rank (ordered by global index).
    Uses a byte tensor all_gather: ranks may hold different counts, so sizes go first."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    raw = np.frombuffer(local.tobytes(), dtype=np.uint8)
    n = torch.tensor([raw.size], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    cap = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(cap, dtype=torch.uint8, device=device)
    buf[:raw.size] = torch.from_numpy(raw.copy()).to(buf.device)
    outs = [torch.zeros(cap, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(outs, buf)
    parts = [np.frombuffer(o[:int(s.item())].cpu().numpy().tobytes(), dtype=local.dtype)
             for o, s in zip(outs, sizes)]
    allp = np.concatenate(parts)
    return allp[np.argsort(allp["index"], kind="stable")]
