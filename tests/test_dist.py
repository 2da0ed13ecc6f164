"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path: corpus sharding by
global index and the single histogram all-reduce.  Per-rank token counts come from the
C oracle here (no GPU in this container); on the GPU box the same reduction runs over
RCCL in bench.py."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

WORKER = r'''
import os, sys, json
sys.path[:0] = [{root!r}, {pkg!r}]
import numpy as np, torch, torch.distributed as dist
from dptok import dist as ddist, synth
from oracle import oracle
rank, world, _ = ddist.init_from_env("gloo")
N, NB = 3000, 258
lo, hi = ddist.shard_range(N, rank, world)
text, offs = synth.random_ascii_corpus(hi - lo, 256, seed=9, start=lo)
ids, id_off, st, _ = oracle.OracleVocab(synth.llama_shaped_vocab()).encode_csr(text, offs)
cnt = np.diff(id_off.astype(np.int64))
h = np.zeros(NB + ddist.N_EXTRA, dtype=np.int64)
np.add.at(h, np.minimum(cnt, NB - 1), 1)
h[NB] = cnt.sum(); h[NB + 1] = hi - lo
np.add.at(h, NB + 2 + st, 1)
t = torch.from_numpy(h.copy())
ddist.allreduce_histogram(t)
# bench.py's overlapped form: two buffers in flight as async collectives, waited out of order
a, b = torch.from_numpy(h.copy()), torch.from_numpy(2 * h)
wa = ddist.allreduce_histogram(a, async_op=True)
wb = ddist.allreduce_histogram(b, async_op=True)
wb.wait(); wa.wait()
if rank == 0:
    print("HIST", json.dumps(t.tolist()))
    print("ASYNC", int(torch.equal(a, t) and torch.equal(b, 2 * t)))
dist.destroy_process_group()
'''


def _single_process_hist():
    from dptok import synth
    from oracle import oracle
    N, NB = 3000, 258
    text, offs = synth.random_ascii_corpus(N, 256, seed=9, start=0)
    ids, id_off, st, _ = oracle.OracleVocab(synth.llama_shaped_vocab()).encode_csr(text, offs)
    cnt = np.diff(id_off.astype(np.int64))
    h = np.zeros(NB + 8, dtype=np.int64)
    np.add.at(h, np.minimum(cnt, NB - 1), 1)
    h[NB] = cnt.sum(); h[NB + 1] = N
    np.add.at(h, NB + 2 + st, 1)
    return h


def test_shard_range_partitions():
    from dptok.dist import shard_range
    for n in (0, 1, 7, 1000, 1_000_003):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, k, w) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1


def test_synthetic_shards_are_rank_count_invariant():
    from dptok import synth
    full, offs = synth.random_ascii_corpus(1000, 256, seed=5)
    a, _ = synth.random_ascii_corpus(400, 256, seed=5, start=0)
    b, _ = synth.random_ascii_corpus(600, 256, seed=5, start=400)
    assert np.array_equal(full, np.concatenate([a, b]))


def test_histogram_allreduce_world2(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, pkg=PKG))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", str(script)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("HIST")][0]
    import json
    got = np.array(json.loads(line[5:]), dtype=np.int64)
    assert np.array_equal(got, _single_process_hist())
    assert "ASYNC 1" in out.stdout


def test_rccl_id_file_exchange(tmp_path):
    """dptok.dist.RcclComm's id hand-over (SURVEY.md §8e "file-store unique id"): rank 0 publishes the
    DPT_RCCL_ID_BYTES id with a rename, a waiting rank in another process reads exactly those bytes."""
    from dptok.dist import publish_id, wait_for_id
    path = str(tmp_path / "rccl.id")
    blob = bytes(range(128))
    code = ("import sys; sys.path[:0] = [%r]; from dptok.dist import wait_for_id; "
            "sys.stdout.buffer.write(wait_for_id(%r, 128, 60.0))") % (PKG, path)
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE)
    publish_id(path, blob)
    out, _ = child.communicate(timeout=60)
    assert child.returncode == 0 and out == blob
    with pytest.raises(TimeoutError):
        wait_for_id(str(tmp_path / "absent.id"), 128, 0.05)
