"""BASELINE configs[2] (cfg3) as the GPU suite runs it: bench.py's sharded path -- one corpus split
across ranks by dptok.dist.shard_range, each rank tokenizing its shard on the GPU and checking it
against the C oracle, ONE all-reduce of the token-count histogram per step.

The box has one GPU, so the two-rank run shares it over gloo (the all-reduce then runs on the host;
rank r uses device r mod 1); the RCCL all-reduce itself runs in a second child at world size 1 with
DPT_BENCH_COLL=1 (bench.py's async nccl path: two histogram buffers, work.wait() on the encode
stream).  Both are fresh child processes started with subprocess (never exec from a process that
touched the GPU).  The reduced histograms must equal each other: the shards tile the corpus and the
collective sums them.  Reference: words are independent DP problems,
/root/reference/packages/tokenizer_utils.py:70.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N = 20000


def _bench_line(cmd, env, timeout=240):
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, (out.returncode, out.stderr[-4000:])
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]   # rank 0 prints ONE JSON line
    return json.loads(lines[0])


def _env(**kw):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    env.pop("DPT_BENCH_COLL", None)
    env.update(kw)
    return env


ARGS = ["--strings", str(N), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


@pytest.fixture(scope="module")
def one_rccl_rank():
    return _bench_line([sys.executable, "bench.py", "--gpus", "1"] + ARGS, _env(DPT_BENCH_COLL="1", MASTER_PORT="29563"))


def _check(line, world):
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    assert line["config"]["strings_total"] == N
    assert line["exact_match"]["rate"] == 1.0 and line["exact_match"]["sample"] == N
    h = line["histogram"]
    assert h["total_strings"] == N and h["status"][0] == N   # cfg2 strings all tokenize (status 0)


@pytest.mark.timeout(600)
def test_cfg3_two_gloo_ranks_match_one_rccl_rank(one_rccl_rank):
    two = _bench_line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                       "--master-addr=127.0.0.1", "--master-port=29561", "bench.py", "--gpus", "2",
                       "--dist-backend", "gloo"] + ARGS, _env())
    _check(two, 2)
    _check(one_rccl_rank, 1)
    assert two["config"]["strings_per_gpu"] == N // 2
    # the two-rank reduced histogram is the one-rank histogram of the whole corpus
    assert two["histogram"] == one_rccl_rank["histogram"]


@pytest.mark.timeout(600)
def test_bench_gpus_flag_launches_the_ranks(one_rccl_rank):
    """`python bench.py --gpus 2` WITHOUT torchrun (the driver's scaling-run form): bench.py starts the two
    ranks itself as a torch.distributed.run child and relays rank 0's line -- n_gpus 2, both shards
    exact, the same reduced histogram as one rank over the whole corpus."""
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    two = _bench_line([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo"] + ARGS, env)
    _check(two, 2)
    assert two["config"]["strings_per_gpu"] == N // 2
    assert two["histogram"] == one_rccl_rank["histogram"]


_RCCL_DIRECT = r"""
import os, sys, json
import numpy as np, torch
from dptok import dist as ddist, synth, Vocab, Encoder, pack_strings
rank, world, id_path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
torch.cuda.set_device(0)
texts = synth.unpack(*synth.random_ascii_corpus(4000, 256, seed=41))
text, offs = pack_strings(texts)
m = len(offs) - 1
enc = Encoder(Vocab(synth.llama_shaped_vocab(32000, seed=0), 0))
dt = torch.from_numpy(np.array(text)).cuda(); do = torch.from_numpy(offs.view(np.int64)).cuda()
ids = torch.empty(len(text), dtype=torch.int32, device="cuda")
id_off = torch.empty(m + 1, dtype=torch.int64, device="cuda"); st = torch.empty(m, dtype=torch.int32, device="cuda")
hist = torch.zeros(258 + 8, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
enc.set_histogram(hist.data_ptr(), 258)
enc.encode_device(dt.data_ptr(), int(offs[-1]), do.data_ptr(), m, ids.data_ptr(), len(text), id_off.data_ptr(),
                  st.data_ptr(), stream=s)
before = hist.clone()
comm = ddist.RcclComm(rank, world, 0, id_path)
comm.allreduce_histogram(hist)
torch.cuda.synchronize()
comm.close()
print(json.dumps({"before": before.cpu().tolist(), "after": hist.cpu().tolist(), "m": m}))
"""


def test_direct_rccl_hist_allreduce_world1(tmp_path):
    """ABI 6: dpt_rccl_get_unique_id -> the id through a file (dptok.dist.RcclComm) ->
    dpt_rccl_comm_create -> dpt_hist_allreduce on the encode stream, in a fresh child process at world
    size 1 (one GPU on the box; RCCL refuses two ranks on one device).  The sum over one rank is the
    rank's own histogram; it counts every string."""
    script = tmp_path / "rccl_direct.py"
    script.write_text(_RCCL_DIRECT)
    env = _env(PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "dp-tokenization_amd"), ROOT]))
    out = subprocess.run([sys.executable, str(script), "0", "1", str(tmp_path / "rccl.id")], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, (out.returncode, out.stderr[-4000:])
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert r["before"] == r["after"]
    assert r["after"][258 + 1] == r["m"] == 4000
