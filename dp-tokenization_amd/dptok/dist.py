"""Multi-GPU plumbing: one process per GPU, corpus sharded by global
string index, ONE all-reduce per pass of the token-count histogram.

The tokenization itself has no exchange step (every string -- every word -- is an
independent DP, reference packages/tokenizer_utils.py:70), so shards never talk on
the data path.  The only collective sums the per-rank histogram + totals
(``dpt_token_histogram`` layout: n_bins count bins, then total ids, total strings,
and one bin per status) -- a few KB, latency-bound over xGMI (RCCL = the "nccl"
backend of torch.distributed on ROCm); the same code runs over gloo on CPU tests.
"""
from __future__ import annotations

import os
from typing import Tuple

N_EXTRA = 8  # total ids, total strings, status 0..4, spare


def rank_world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous global-index range [lo, hi) of ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def histogram_layout(n_bins: int) -> dict:
    return {"bins": slice(0, n_bins), "total_ids": n_bins, "total_strings": n_bins + 1,
            "status": slice(n_bins + 2, n_bins + 7)}


def allreduce_histogram(hist, group=None, async_op: bool = False):
    """Sum a histogram tensor (int64, n_bins + N_EXTRA) over all ranks in place.  async_op: return
    the collective's work handle (``wait()`` orders it before the caller's stream continues) -- the
    RCCL all-reduce then overlaps whatever the stream does next; None when there is nothing to do."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        work = dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        return work if async_op else hist
    return None if async_op else hist


def init_from_env(backend: str = "nccl", device=None):
    """Initialise the default process group from torch.distributed.run's environment
    (MASTER_ADDR defaults to 127.0.0.1: container host names may not resolve)."""
    import torch
    import torch.distributed as dist
    rank, world, local = rank_world()
    if world <= 1 or dist.is_initialized():
        return rank, world, local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dev = local if device is None else device
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    return rank, world, local
