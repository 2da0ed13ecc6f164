"""Llama-mode host pre-tokenization over worker processes.

In llama mode the reference runs ``tokenizer.encode`` (SentencePiece, third-party) per string and
merges the pieces into words on the host (packages/tokenizer_utils.py:24-31, :7-22) before every
word's DP; the GPU does the DP of a whole batch in one launch, so the host side is what bounds
``dp_tokenize.batch``.  ``PretokenizePool`` spreads it over processes: each worker holds an
unpickled copy of the caller's tokenizer, runs ``tokenizer.encode`` per text (or the library's
batched equivalent, ``packages.tokenizer_utils.batch_encoder``) over its chunk and packs the pieces
with ``PieceTable.pack``; the parent concatenates the chunks' pre-split buffers and launches once.

Workers are plain child processes (``python -m dptok._pretok_worker`` through subprocess: a fresh
interpreter that never touches the GPU and never re-imports the caller's main module, unlike
multiprocessing's spawn / forkserver), fed length-prefixed pickles over their stdin/stdout by one
parent thread each.  They start on the first large batch and are reused.  Batches below
``min_batch`` strings, and tokenizers that cannot be pickled, run in-process.
"""
from __future__ import annotations

import atexit
import os
import pickle
import select
import struct
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

_HDR = struct.Struct("<Q")


def send_msg(f, obj) -> None:
    b = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    f.write(_HDR.pack(len(b)))
    f.write(b)
    f.flush()


def _read_exact(fd: int, n: int, deadline: Optional[float]) -> bytes:
    """n bytes from a pipe's file descriptor; TimeoutError past the deadline (time.monotonic())."""
    parts, got = [], 0
    while got < n:
        if deadline is not None:
            left = deadline - time.monotonic()
            if left <= 0 or not select.select([fd], [], [], left)[0]:
                raise TimeoutError("pre-tokenization worker did not answer in time")
        b = os.read(fd, min(n - got, 1 << 20))
        if not b:
            raise EOFError("worker pipe closed")
        parts.append(b)
        got += len(b)
    return b"".join(parts)


def recv_msg(f, timeout: Optional[float] = None):
    """One length-prefixed pickle from a worker's (unbuffered) stdout; timeout: seconds or None."""
    fd = f.fileno()
    deadline = None if timeout is None else time.monotonic() + timeout
    n = _HDR.unpack(_read_exact(fd, _HDR.size, deadline))[0]
    return pickle.loads(_read_exact(fd, n, deadline))


def cpu_share() -> int:
    """Worker processes: the process's CPU share (OMP_NUM_THREADS on the GPU boxes, else its
    affinity), at most 16."""
    vis = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    return max(1, min(16, min(vis, omp) if omp > 0 else vis))


def concat_packed(parts):
    """Chunks of ``PieceTable.pack`` output, in order -> one batch's buffers."""
    if len(parts) == 1:
        return parts[0]
    texts, offs, cuts, cnts = [], [np.zeros(1, np.uint64)], [], []
    base = 0
    for text, off, cut, cnt in parts:
        nb = int(off[-1])
        texts.append(text[:nb])
        cuts.append(cut[:nb])
        offs.append(off[1:] + np.uint64(base))
        cnts.append(cnt)
        base += nb
    z = np.zeros(1, np.uint8)
    return (np.concatenate(texts + [z]), np.concatenate(offs), np.concatenate(cuts + [z]), np.concatenate(cnts))


# seconds a worker may take per chunk: a base plus a rate far below SentencePiece's (~1 MB/s per core)
TIMEOUT_BASE_S, TIMEOUT_PER_BYTE_S = 60.0, 1e-5


class PretokenizePool:
    def __init__(self, tokenizer, table, encode_ids, procs: Optional[int] = None, min_batch: int = 2048):
        self.tokenizer = tokenizer
        self.table = table              # the parent's PieceTable (same vocabulary as the workers')
        self.encode_ids = encode_ids    # the parent's batch encoder (small batches)
        self.procs = cpu_share() if procs is None else procs
        self.min_batch = min_batch
        self._workers: List[subprocess.Popen] = []
        self._broken = self.procs <= 1
        self._lock = threading.Lock()

    def _start(self) -> bool:
        if self._workers:
            return True
        if self._broken:
            return False
        try:
            tok_bytes = pickle.dumps(self.tokenizer, protocol=pickle.HIGHEST_PROTOCOL)
        except Exception:   # an unpicklable tokenizer object: in-process only
            self._broken = True
            return False
        here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = dict(os.environ)
        env["PYTHONPATH"] = here + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env["OMP_NUM_THREADS"] = "1"
        env.setdefault("TOKENIZERS_PARALLELISM", "false")   # one process per core already
        for _ in range(self.procs):
            p = subprocess.Popen([sys.executable, "-m", "dptok._pretok_worker"], stdin=subprocess.PIPE,
                                 stdout=subprocess.PIPE, env=env, cwd=here, bufsize=0)
            self._workers.append(p)
        try:
            for p in self._workers:
                send_msg(p.stdin, (list(sys.path), tok_bytes))
            for p in self._workers:
                if recv_msg(p.stdout, TIMEOUT_BASE_S) != "ready":
                    raise RuntimeError("pre-tokenization worker failed to start")
        except (EOFError, OSError, RuntimeError, TimeoutError):
            self.close()
            self._broken = True
            return False
        return True

    def pack(self, texts: Sequence[str]):
        n = len(texts)
        with self._lock:
            if n < self.min_batch or not self._start():
                return self.table.pack(self.encode_ids(texts))
            k = min(4 * len(self._workers), max(1, n // 256))
            bounds = [n * i // k for i in range(k + 1)]
            results: list = [None] * k
            errors: list = []
            nxt = [0]
            qlock = threading.Lock()

            def feed(p):
                try:
                    while True:
                        with qlock:
                            i = nxt[0]
                            nxt[0] += 1
                        if i >= k or errors:
                            return
                        chunk = list(texts[bounds[i]:bounds[i + 1]])
                        send_msg(p.stdin, chunk)
                        # bounded: a hung worker (e.g. inside the tokenizer's own threads) counts as a dead one
                        budget = TIMEOUT_BASE_S + TIMEOUT_PER_BYTE_S * sum(len(t) for t in chunk)
                        kind, val = recv_msg(p.stdout, budget)
                        if kind == "err":
                            errors.append(val)
                            return
                        results[i] = val
                except (EOFError, OSError, TimeoutError) as e:
                    errors.append(e)

            th = [threading.Thread(target=feed, args=(p,), daemon=True) for p in self._workers]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errors:
                e = errors[0]
                if isinstance(e, (EOFError, OSError, TimeoutError)):   # a worker died or hung: drop the pool, run in-process
                    self.close()
                    self._broken = True
                    return self.table.pack(self.encode_ids(texts))
                raise e   # the tokenizer's / PieceTable's own exception (e.g. KeyError for an unknown id)
            return concat_packed(results)

    def close(self) -> None:
        for p in self._workers:
            try:
                p.stdin.close()
            except OSError:
                pass
        for p in self._workers:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:   # (a hung worker: its own process only, by its handle)
                p.kill()
                p.wait()
            try:
                p.stdout.close()
            except OSError:
                pass
        self._workers = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# One pool per tokenizer object: every dp_tokenize_llama(tok, "llama") adapter over the same tokenizer
# shares its workers (each holds an unpickled tokenizer), and every pool is closed at exit.
_POOLS: Dict[int, "PretokenizePool"] = {}
_POOLS_LOCK = threading.Lock()


def shared_pool(tokenizer, table, encode_ids, **kw) -> "PretokenizePool":
    with _POOLS_LOCK:
        pool = _POOLS.get(id(tokenizer))
        if pool is None or pool.tokenizer is not tokenizer:   # (an id reused after its tokenizer died)
            if pool is not None:
                pool.close()
            pool = PretokenizePool(tokenizer, table, encode_ids, **kw)
            _POOLS[id(tokenizer)] = pool   # (keeps the tokenizer alive, so its id stays unique)
        return pool


@atexit.register
def _close_pools() -> None:
    with _POOLS_LOCK:
        for pool in _POOLS.values():
            try:
                pool.close()
            except Exception:
                pass
        _POOLS.clear()
