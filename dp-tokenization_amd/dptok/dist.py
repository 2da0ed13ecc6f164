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


class RcclComm:
    """Direct RCCL through the C-ABI (ABI 6: dpt_rccl_get_unique_id / dpt_rccl_comm_create /
    dpt_hist_allreduce), SURVEY.md §8(e)'s "direct RCCL with a file-store unique id": rank 0 writes the
    communicator id to ``id_path`` (atomically: a temporary file renamed into place), the other ranks
    wait for it.  For a caller that binds only libdpt.so; bench.py uses torch.distributed instead."""

    def __init__(self, rank: int, world: int, device: int, id_path: str, timeout_s: float = 120.0):
        import ctypes
        from . import _lib
        self._L = _lib.lib()
        self.rank, self.world, self.device = rank, world, device
        idb = (ctypes.c_uint8 * _lib.DPT_RCCL_ID_BYTES)()
        if rank == 0:
            _lib.check(self._L.dpt_rccl_get_unique_id(idb), "dpt_rccl_get_unique_id")
            publish_id(id_path, bytes(idb))
        else:
            ctypes.memmove(idb, wait_for_id(id_path, _lib.DPT_RCCL_ID_BYTES, timeout_s), _lib.DPT_RCCL_ID_BYTES)
        self._comm = ctypes.c_void_p()
        _lib.check(self._L.dpt_rccl_comm_create(idb, world, rank, device, ctypes.byref(self._comm)),
                   "dpt_rccl_comm_create")

    def allreduce_histogram(self, hist, stream=None):
        """Sum the int64 device tensor ``hist`` over the ranks in place, ordered on ``stream`` (a
        torch.cuda.Stream; default: the current one).  Returns ``hist``."""
        import torch
        from . import _lib
        if hist.dtype != torch.int64 or not hist.is_cuda or not hist.is_contiguous():
            raise ValueError("hist must be a contiguous int64 device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(hist.device)
        _lib.check(self._L.dpt_hist_allreduce(hist.data_ptr(), hist.numel(), self._comm, s.cuda_stream),
                   "dpt_hist_allreduce")
        return hist

    def close(self):
        from . import _lib
        if self._comm:
            _lib.check(self._L.dpt_rccl_comm_destroy(self._comm), "dpt_rccl_comm_destroy")
            self._comm = None


def publish_id(path: str, blob: bytes) -> None:
    """Write the communicator id where the other ranks look (temporary file + rename: never half-read)."""
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(blob)
    os.replace(tmp, path)


def wait_for_id(path: str, n: int, timeout_s: float) -> bytes:
    """Poll for rank 0's id file; TimeoutError after ``timeout_s``."""
    import time
    t_end = time.monotonic() + timeout_s
    while True:
        try:
            with open(path, "rb") as f:
                blob = f.read()
            if len(blob) == n:
                return blob
        except FileNotFoundError:
            pass
        if time.monotonic() > t_end:
            raise TimeoutError(f"no communicator id at {path} after {timeout_s} s")
        time.sleep(0.01)
