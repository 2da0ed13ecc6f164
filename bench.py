#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X.

metric: input bytes/sec (whole job, all GPUs) + exact-match rate vs the CPU DP,
256-byte random printable-ASCII strings, synthetic Llama-shaped 32k vocab (no
Llama-2 tokenizer file is available offline: SURVEY.md §0 finding 6).

A step = one pass of the hot path (dpt_encode: the tokenize passes + the finish kernel's
offsets and CSR ids, then the token-count histogram and, for N>1, ONE RCCL all-reduce
of it) over the rank's resident shard (BASELINE.json configs[1] at N=1, configs[2] at N=8).
Strong scaling (the default for N > 1): ONE global corpus of --strings
(1M) strings keyed by (seed, global index) is split by dptok.dist.shard_range -- rank r
takes [r*N/W, (r+1)*N/W) -- and `value` = the corpus bytes / max-over-ranks time.
--scaling weak gives every rank its own --strings strings instead (labelled "weak").

Launch: python bench.py --gpus N --steps K --warmup W
  N = 1 runs in this process.  N > 1 without WORLD_SIZE in the environment: this process starts
  `python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ...
  bench.py <the same arguments>` as a CHILD (before anything here touches the GPU; never an exec)
  and exits with its return code -- rank 0's JSON line goes to the same stdout.  Under torchrun
  (WORLD_SIZE set) --gpus must equal WORLD_SIZE (else exit 2).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dp-tokenization_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)
N_BINS = 258                # tokens-per-string histogram (<= 256 ids for 256-byte strings, + overflow)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the job; default: WORLD_SIZE under torchrun, else 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["cfg1", "cfg2", "cfg4", "cfg5", "bloom", "cfg2p", "cfg4p"], default="cfg2",
                    help="cfg2 (the metric's config): 256-byte random ASCII; cfg1: BASELINE configs[0], 1k x 64-byte "
                         "random ASCII with the toy 1k vocabulary (the reference's CPU plumbing case); "
                         "cfg4: S2ORC-shaped; cfg5: Arabic-shaped; cfg2p / cfg4p: the same corpora in llama mode "
                         "(pretokenize_option='llama', the factory's default: BOS word + SentencePiece-shaped words, "
                         "pre-split on the host (dptok.synth.llama_words), DPT_MODE_PRESPLIT on the GPU); "
                         "bloom: row f3 at BLOOM scale (250,680-entry byte-level BPE, atoms mode, <= 256-byte strings)")
    ap.add_argument("--strings", type=int, default=None,
                    help="strings of the global corpus (strong) or per GPU (weak); default 1M (cfg4: 200k)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default=None,
                    help="strong (default for N > 1; identical at N = 1): the global corpus is sharded over the "
                         "ranks by dptok.dist.shard_range; weak: every rank owns --strings strings")
    ap.add_argument("--length", type=int, default=None, help="bytes per string (default 256; cfg1: 64)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--exact-sample", type=int, default=None,
                    help="strings checked against the C oracle (rank 0; default: every string of the rank's shard)")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="strings for the reference-port CPU baseline (default 2048; bloom 65536 -- bounded by --cpu-budget)")
    ap.add_argument("--gen-procs", type=int, default=None,
                    help="processes for the synthetic corpus (default: the CPU share, at most 16; 1 under a profiler "
                         "that follows forks)")
    ap.add_argument("--cpu-budget", type=float, default=25.0, help="seconds of CPU-baseline wall time")
    ap.add_argument("--inflight", type=int, choices=range(0, 9), default=0,
                    help="batches in flight per GPU: step k on context + stream k mod N (N = 2..8) or one stream (1); "
                         "0 = 4 for shards of >= 65,536 strings and <= 64 MiB, 3 up to 524,288 strings (not bloom), else 1")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-path", action="store_true",
                    help="instead of the headline line: the drop-in surface the reference's callers use "
                         "(dp_tokenize(str) per call and dp_tokenize.batch, raw and llama mode, cfg2 and cfg4)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, the real path) or gloo -- gloo lets a rehearsal put several ranks "
                         "on one GPU (device = local_rank mod visible GPUs)")
    return ap.parse_args()


def log(msg: str) -> None:
    """Progress on stderr (the JSON line stays the only stdout line)."""
    print("bench: " + msg, file=sys.stderr, flush=True)


def exact_matches(ids_h, off_h, st_h, rids, roff, rst, S: int) -> int:
    """Strings among the first S whose ids and status equal the oracle's (CSR on both sides)."""
    off_h = np.asarray(off_h, dtype=np.uint64)
    roff = np.asarray(roff, dtype=np.uint64)
    if np.array_equal(off_h[: S + 1] - off_h[0], roff[: S + 1] - roff[0]):
        # every count agrees: one vectorised compare, mismatching ids mapped back to strings
        n_id = int(roff[S] - roff[0])
        a0, b0 = int(off_h[0]), int(roff[0])
        diff = np.nonzero(ids_h[a0:a0 + n_id] != rids[b0:b0 + n_id])[0]
        bad = np.zeros(S, dtype=bool)
        bad[np.searchsorted(roff[: S + 1] - roff[0], diff.astype(np.uint64), side="right") - 1] = True
        bad |= st_h[:S] != rst[:S]
        return int(S - bad.sum())
    same = 0
    for i in range(S):
        a = ids_h[int(off_h[i]):int(off_h[i + 1])]
        b = rids[int(roff[i]):int(roff[i + 1])]
        same += int(st_h[i] == rst[i] and np.array_equal(a, b))
    return same


# ------------------------------------------------------------------ CPU baseline (port of the reference)
_PORT = {}


def _port_init(kind: str = "llama"):
    from dptok import synth
    from oracle import ref_port
    if kind == "bloom":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from bloom_fixture import big_vocab
        _PORT["t2i"] = big_vocab()
        _PORT["f"] = ref_port.dp_tokenize_word_atoms
    elif kind == "presplit":   # words of code points (llama mode: merge_tokens' strings, tokenizer_utils.py:70-71)
        _PORT["t2i"] = synth.llama_shaped_vocab()
        _PORT["f"] = ref_port.dp_tokenize_word_atoms
    else:
        _PORT["t2i"] = synth.toy_vocab() if kind == "toy" else synth.llama_shaped_vocab()
        _PORT["f"] = ref_port.dp_tokenize_raw

    def _alarm(signum, frame):
        raise TimeoutError()
    signal.signal(signal.SIGALRM, _alarm)


def _port_one(item):
    signal.alarm(10)
    try:
        x = item[0]
        if isinstance(x, tuple) and x[0] == "presplit":   # (tag, bytes, cut bytes) -> words of code points
            b, c = x[1], x[2]
            starts = [k for k in range(len(b)) if c[k] and (b[k] & 0xC0) != 0x80] + [len(b)]
            x = [list(b[starts[j]:starts[j + 1]].decode("utf-8")) for j in range(len(starts) - 1)]
        elif isinstance(x, tuple):   # bloom: (bytes, cut bytes) -> words of atoms, in the worker
            b, c = x
            x = words_of_atoms(np.frombuffer(b, np.uint8), np.array([0, len(b)], np.uint64), np.frombuffer(c, np.uint8))[0]
        _PORT["f"](x, _PORT["t2i"])
        ok = True
    except TimeoutError:
        ok = False
    finally:
        signal.alarm(0)
    return item[1], ok


def words_of_atoms(text: np.ndarray, offs: np.ndarray, cut: np.ndarray) -> list:
    """Atoms-mode buffers -> per string, words of atoms (cut bit 1: atom start, bit 0: word start)."""
    out = []
    raw = text.tobytes()
    for i in range(len(offs) - 1):
        a, b = int(offs[i]), int(offs[i + 1])
        words, atoms, p0 = [], [], a
        for p in range(a + 1, b + 1):
            if p == b or cut[p] & 2:
                atoms.append(raw[p0:p].decode("utf-8"))
                p0 = p
                if p == b or cut[p] & 1:
                    words.append(atoms)
                    atoms = []
        out.append(words)
    return out


def cpu_baseline(items, budget, cores, kind="llama"):
    """The reference's enumerate-then-select DP (oracle/ref_port.py) on `cores` processes; items =
    (input, bytes) pairs."""
    done_bytes, n_done, n_to = 0, 0, 0
    ctx = mp.get_context("fork")
    with ctx.Pool(cores, initializer=_port_init, initargs=(kind,)) as pool:
        t0 = time.perf_counter()
        it = pool.imap_unordered(_port_one, items, chunksize=4)
        for nb, ok in it:
            if ok:
                done_bytes += nb
                n_done += 1
            else:
                n_to += 1
            if time.perf_counter() - t0 > budget:
                break
        dt = time.perf_counter() - t0
        pool.terminate()
    return done_bytes / dt, n_done, n_to, dt


def traffic_for(n_str: int, lb: int):
    """HBM bytes per tokenize launch measured by tools/pmc_traffic.py (PMC FETCH_SIZE x2 +
    WRITE_SIZE) -- only when it was measured on these kernel sources and this workload."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from pmc_traffic import source_hash
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            rec = json.load(fh)
        if rec.get("source_sha256") == source_hash() and rec.get("n_str") == n_str and lb == 256:
            return rec["traffic_bytes_per_launch"]
    except (OSError, ValueError, KeyError, ImportError):
        pass
    return None


def cpu_share() -> tuple:
    """(threads the CPU legs use, host CPUs visible to this process).  The GPU box's CPU share is
    exported as OMP_NUM_THREADS (16 per GPU); os.sched_getaffinity shows what the process may run
    on, which on a shared box is the whole machine -- the share is what gets used and reported."""
    vis = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    return (max(1, min(vis, omp)) if omp > 0 else vis), vis


def rank_strings(n_global: int, rank: int, world: int, scaling: str):
    """Global string-index range [lo, hi) of this rank: its shard_range part of the one corpus
    (strong) or its own n_global strings (weak)."""
    from dptok.dist import shard_range
    if scaling == "strong":
        return shard_range(n_global, rank, world)
    return rank * n_global, (rank + 1) * n_global


INFLIGHT_MAX_STRINGS = 524288   # auto: batches in flight for shards up to this many strings ...
INFLIGHT4_MIN_STRINGS = 65536   # ... four of them for shards of at least this many strings
INFLIGHT4_MAX_BYTES = 1 << 26   # ... and at most 64 MiB of text, else three


def batches_in_flight(arg: int, n_str: int, rows64: bool = False, n_bytes: int = 0) -> int:
    """--inflight: 1..8 as given; 0 (auto) = 4 for shards of INFLIGHT4_MIN_STRINGS.. strings and <= 64 MiB of text
    (8 / 4 ranks of the strong-scaling run: 125k, 250k strings), 3 for others of <= INFLIGHT_MAX_STRINGS strings
    (2 ranks: 500k; cfg4; cfg1), else 1.  The small shards' last slot-round and finish pass the next steps' first
    passes then fill: 125k strings 91.8 -> 93.1 GB/s from two to three (r06ap); three -> four with the per-step RCCL
    all-reduce the N > 1 runs do: 94.9 -> 98.1 at 125k, 104.7 -> 106.7 at 250k (r06ih).  Four measured SLOWER where a
    batch holds more text (500k x 256 B: 84 against 104; cfg4's 200k x ~1.2 KB: 76 against 83.5) or is tiny (cfg1),
    and six or eight were slower everywhere (125k: 91; r06ig, r06ii).  1 for the 64-lane (BLOOM-scale) kernel, one
    string per wave, where two in flight measured 1.4 % slower (r06ev6)."""
    if arg:
        return arg
    if rows64 or n_str > INFLIGHT_MAX_STRINGS:
        return 1
    return 4 if n_str >= INFLIGHT4_MIN_STRINGS and n_bytes <= INFLIGHT4_MAX_BYTES else 3


def n_tok_rank_of(d_idoff) -> int:
    return int(d_idoff[-1].item())


def algorithmic_bytes(n_bytes: int, n_str: int, n_tok: int, id_bytes: int = 4) -> int:
    """B = N_in + 4*N_tok + 8(N+1) [in offsets] + 8(N+1) [out offsets] + 4N [status]."""
    return n_bytes + id_bytes * n_tok + 8 * (n_str + 1) + 8 * (n_str + 1) + 4 * n_str


def host_path(args):
    """Secondary line: the unchanged callers' shape (main_analyze_s2orc.py:74-78 one dp_tokenize call
    per row, :269-271 a serial loop) and the batched form, from Python str to List[List[int]], host
    buffers through dpt_encode_host (pinned staging, PCIe both ways).  llama mode runs the real
    SentencePiece model of tests/golden (sp_llama32k.model) through transformers.LlamaTokenizer: its
    encode is third-party host work and is timed with the rest."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dptok import synth
    from packages.tokenizer_utils import dp_tokenize_llama
    from sp_llama import hf_llama
    from fake_llama import FakeLlamaTokenizer
    t2i = synth.llama_shaped_vocab()
    cfg2 = synth.unpack(*synth.random_ascii_corpus(4096, 256, seed=args.seed))
    cfg4 = synth.unpack(*synth.s2orc_like_corpus(512, seed=4))
    out = {"metric": "drop-in host path: us per dp_tokenize(str) call, strings/s and bytes/s per dp_tokenize.batch",
           "unit": "mixed", "n_gpus": 1, "data": "synthetic", "rows": []}
    tokz = {"raw": FakeLlamaTokenizer(t2i), "llama": hf_llama()}
    for mode in ("raw", "llama"):
        dp_tokenize, _ = dp_tokenize_llama(tokz[mode], mode)
        for wl, texts in (("cfg2", cfg2), ("cfg4", cfg4)):
            nbytes = sum(len(t.encode()) for t in texts)
            for t in texts[:8]:
                dp_tokenize(t)                       # warm-up (workspace growth, code paths)
            dp_tokenize.batch(texts)
            k = 200 if wl == "cfg2" else 100
            t0 = time.perf_counter()
            for t in texts[:k]:
                dp_tokenize(t)
            per_call = (time.perf_counter() - t0) / k
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                dp_tokenize.batch(texts)
            bt = (time.perf_counter() - t0) / reps
            out["rows"].append({"mode": mode, "workload": wl, "us_per_call": per_call * 1e6,
                                "batch_strings": len(texts), "batch_strings_per_s": len(texts) / bt,
                                "batch_bytes_per_s": nbytes / bt,
                                "vocab": "synthetic llama-shaped 32000" if mode == "raw" else "SentencePiece BPE 32000 (tests/golden)"})
    print(json.dumps(out), flush=True)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def resolve_world(args, env=os.environ) -> int:
    """The job's rank count: --gpus, checked against WORLD_SIZE when torchrun started this process.
    Returns 0 when this process must launch the ranks itself (--gpus > 1, no WORLD_SIZE); raises
    SystemExit(2) on a mismatch (a silently smaller job would mis-measure the scaling run)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        g = 1 if args.gpus is None else args.gpus
        if g < 1:
            raise SystemExit("bench: --gpus must be >= 1")
        return 0 if g > 1 else 1
    if args.gpus is not None and args.gpus != int(ws):
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={ws}: refusing to run a job of another size",
              file=sys.stderr, flush=True)
        raise SystemExit(2)
    return int(ws)


def spawn_ranks(args, argv) -> int:
    """--gpus N > 1 from a plain `python bench.py`: one rank per GPU through torch.distributed.run, as a
    child process (this process has not touched the GPU); its exit code is ours.  A SIGTERM / SIGINT to
    this process is passed on to torchrun as SIGTERM (which stops its ranks), and we wait for it to exit,
    so no rank is left holding a GPU.  (The port is picked just before the launch; torchrun binds it
    first thing, so the window for another process to take it is the launch itself.)"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    child = subprocess.Popen(cmd, env=env)
    stop = []

    def forward(signum, frame):
        stop.append(signum)
        if child.poll() is None:
            child.send_signal(signal.SIGTERM)
    old = {sg: signal.signal(sg, forward) for sg in (signal.SIGTERM, signal.SIGINT)}
    try:
        rc = child.wait()
    finally:
        for sg, h in old.items():
            signal.signal(sg, h)
    if stop:
        log("stopped by signal %d; torchrun exited with %d" % (stop[0], rc))
        return 128 + stop[0]
    return rc


def main():
    args = parse()
    if args.host_path:
        return host_path(args)
    if resolve_world(args) == 0:
        raise SystemExit(spawn_ranks(args, sys.argv[1:]))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    scaling = args.scaling or "strong"   # N = 1: strong and weak are the same run
    from dptok import Encoder, Vocab, synth
    from dptok import dist as ddist
    bloom = args.workload == "bloom"
    presplit = args.workload in ("cfg2p", "cfg4p")
    base_wl = args.workload[:-1] if presplit else args.workload
    if bloom:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from bloom_fixture import big_vocab
        t2i = big_vocab()
    elif args.workload == "cfg1":
        t2i = synth.toy_vocab()
    else:
        t2i = synth.llama_shaped_vocab()
    Lb = args.length or (64 if args.workload == "cfg1" else 256)
    cores, cpus_visible = cpu_share()
    gen_procs = args.gen_procs or max(1, min(16, cores))
    if args.cpu_sample is None:
        args.cpu_sample = 262144 if bloom else 2048
    default_n = {"cfg1": 1000, "cfg4": 200_000, "bloom": 500_000}.get(base_wl, 1_000_000)
    N = args.strings or default_n
    lo, hi = rank_strings(N, rank, world, scaling)
    M = hi - lo
    per = "corpus, sharded over the GPUs" if scaling == "strong" else "per GPU"
    cut = None
    if bloom:
        text, offs, cut = synth.bloom_like_parallel(M, t2i, start=lo, procs=gen_procs, length=Lb)
        wl = (f"bloom: {N // 1000}k x <= {Lb}-byte pre-tokenized byte-level strings {per}, atoms mode, "
              "BLOOM-scale vocabulary")
        data = ("synthetic byte-level words (dptok.synth.bloom_like_corpus: 15% tokens > 16 code points); synthetic "
                "250,680-entry byte-level BPE (tests/golden/bloom_big_tokenizer.json.xz)")
    elif args.workload == "cfg1":
        text, offs = synth.random_ascii_corpus(M, Lb, seed=args.seed, start=lo)
        wl = f"cfg1: {N} x {Lb}-byte random ASCII strings {per}, raw pre-tokenization, toy 1k vocabulary"
        data = ("synthetic random printable ASCII (Philox keyed by seed+global index; tests/golden/cfg1_toy1k holds the "
                "reference's outputs for seed 1); synthetic toy 1000-entry vocab")
    elif base_wl == "cfg2":
        text, offs = synth.random_ascii_corpus(M, Lb, seed=args.seed, start=lo)
        wl = f"cfg2: {N // 1000}k x {Lb}-byte random ASCII strings {per}, raw pre-tokenization"
        data = "synthetic random printable ASCII (Philox keyed by seed+global index); synthetic Llama-shaped 32k vocab"
    elif base_wl == "cfg4":
        text, offs = synth.generate_parallel("s2orc", M, start=lo, procs=gen_procs, seed=4)
        wl = f"cfg4: {N // 1000}k S2ORC-shaped abstracts {per} (~1200 B, N(1200,400) clipped to [64,4096]), raw"
        data = "synthetic S2ORC-shaped pseudo-English (dptok.synth.s2orc_like_corpus); synthetic Llama-shaped 32k vocab"
    else:
        text, offs = synth.generate_parallel("arabic", M, start=lo, procs=gen_procs, length=Lb, seed=5)
        wl = f"cfg5: {N // 1000}k x ~{Lb}-byte Arabic-shaped strings {per} (2-byte code points), raw"
        data = "synthetic Arabic-shaped UTF-8 (dptok.synth.arabic_corpus); synthetic Llama-shaped 32k vocab + Arabic letters"
    raw_text_bytes = int(offs[-1])
    if presplit:
        # llama mode (reference tokenizer_utils.py:24-31, :64-65): the host's SentencePiece + merge_tokens words,
        # here the shape a Llama-2 model gives this text (BOS word, '▁' for spaces and the dummy prefix, the
        # byte-fallback piece for '\n'), as UTF-8 + a word-start mask; the timed step is the GPU part
        text, offs, cut = synth.llama_words(text, offs)
        wl = args.workload + wl[len(base_wl):]
        wl = wl.replace("raw pre-tokenization", "llama mode").replace("), raw", "), llama mode") + \
            " (pre-split words: <s>, then SentencePiece-shaped words; DPT_MODE_PRESPLIT)"
        data += "; words pre-split on the host by dptok.synth.llama_words (SentencePiece's shape for this text)"
    Lb = int(offs[-1]) // max(M, 1)
    log(f"corpus ready: {M} strings, {int(offs[-1])} bytes")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before any GPU call: the pool forks plain CPU workers
        args.cpu_sample = min(args.cpu_sample, M)
        sub = offs[: args.cpu_sample + 1]
        if bloom:
            tb, cb = text.tobytes(), cut.tobytes()
            inputs = [(tb[int(sub[i]):int(sub[i + 1])], cb[int(sub[i]):int(sub[i + 1])]) for i in range(args.cpu_sample)]
        elif presplit:
            tb, cb = text.tobytes(), cut.tobytes()
            inputs = [("presplit", tb[int(sub[i]):int(sub[i + 1])], cb[int(sub[i]):int(sub[i + 1])]) for i in range(args.cpu_sample)]
        else:
            inputs = synth.unpack(text[: int(offs[args.cpu_sample])], sub)
        items = list(zip(inputs, np.diff(sub).astype(int).tolist()))
        v, nd, nto, cdt = cpu_baseline(items, args.cpu_budget, cores,
                                       "bloom" if bloom else "presplit" if presplit else ("toy" if args.workload == "cfg1" else "llama"))
        cpu = {"value": v, "unit": "bytes/s", "cores": cores, "host_cpus_visible": cpus_visible, "kind": "port",
               "sample": f"{nd} of the first {args.cpu_sample} {args.workload} strings in {cdt:.1f}s "
                         f"(enumerate-then-select, oracle/ref_port.py, {cores} processes = the box's CPU share "
                         f"OMP_NUM_THREADS of {cpus_visible} visible CPUs; {nto} hit the 10s per-string limit)"}
        if args.workload == "cfg1":
            # BASELINE.md quotes the reference on cfg1 on ONE core (79.2 KB/s): the port on one core too
            _port_init("toy")
            t0c = time.perf_counter()
            for x, _ in items:
                _PORT["f"](x, _PORT["t2i"])
            cpu["port_1core_bytes_per_s"] = sum(nb for _, nb in items) / (time.perf_counter() - t0c)

    gpu = local % max(1, torch.cuda.device_count())
    if gpu != local and args.dist_backend == "nccl":
        raise SystemExit(f"local rank {local} has no GPU of its own; use --dist-backend gloo to share one")
    ddist.init_from_env(args.dist_backend, device=gpu)
    # DPT_BENCH_COLL=1: run the per-step all-reduce even at world size 1 (a rehearsal of the async RCCL
    # path on a one-GPU box; the real runs have world > 1)
    coll = world > 1 or os.environ.get("DPT_BENCH_COLL") == "1"
    if coll and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29655")
        torch.cuda.set_device(gpu)
        dist.init_process_group(args.dist_backend, rank=0, world_size=1,
                                **({"device_id": torch.device("cuda", gpu)} if args.dist_backend == "nccl" else {}))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    vocab = Vocab(t2i, device=gpu)
    # Batches in flight: with N > 1, step k runs on context + stream k % N, so a step's last slot-round (the
    # persistent grid's tail) and its finish pass overlap the next steps' first passes -- batches in flight,
    # as a serving loop keeps them; the outputs of every context are checked.  The small shards
    # of strong scaling gain (125k strings: +6 %, 250k: +7 % with three, r06ab / r06ap; four with the all-reduce:
    # +3.3 / +1.9 % more, r06ih), 1M does not (r06ai); batches_in_flight has the rule.
    inflight = batches_in_flight(args.inflight, M, rows64=bloom, n_bytes=int(offs[-1] - offs[0]))
    encs = [Encoder(vocab) for _ in range(inflight)]
    enc = encs[0]
    n_bytes = int(offs[-1] - offs[0])
    d_text = torch.from_numpy(text).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_cut = torch.from_numpy(cut).to(dev) if cut is not None else None
    outs = [(torch.empty(max(n_bytes, 1), dtype=torch.int32, device=dev), torch.empty(M + 1, dtype=torch.int64, device=dev),
             torch.empty(max(M, 1), dtype=torch.int32, device=dev)) for _ in range(inflight)]
    d_ids, d_idoff, d_status = outs[0]
    # histogram buffers, one per batch in flight and at least two: step k's all-reduce (RCCL, on its own
    # stream, async) overlaps step k+1's tokenize, which fills another buffer; buffer k mod len is written on
    # step k's stream only and reused only after its all-reduce completed
    d_hists = [torch.zeros(N_BINS + 8, dtype=torch.int64, device=dev) for _ in range(max(2, inflight))]
    pending = [None] * len(d_hists)
    n_step = [0]
    ran = [False] * inflight   # contexts that ran a step (a short run may not reach all of them)
    for e in encs:
        e.reserve(n_bytes, M)
    kmode = "atoms" if bloom else "presplit" if presplit else "raw"
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(inflight - 1)]
    stream = streams[0].cuda_stream

    def step(one_stream: bool = False):
        b = n_step[0] % len(d_hists)
        i = 0 if one_stream else n_step[0] % inflight
        n_step[0] += 1
        ran[i] = True
        h = d_hists[b]
        ids_i, idoff_i, st_i = outs[i]
        with torch.cuda.stream(streams[i]):   # (the collective below orders itself after this stream's work)
            if pending[b] is not None:   # the stream waits for this buffer's previous all-reduce
                pending[b].wait()
                pending[b] = None
            # the histogram is folded into the encode's finish pass, which replaces h's contents
            # (dpt_ctx_set_histogram_ex, DPT_HIST_OVERWRITE: no memset launch per step)
            encs[i].set_histogram(h.data_ptr(), N_BINS, overwrite=True)
            encs[i].encode_device(d_text.data_ptr(), n_bytes, d_off.data_ptr(), M, ids_i.data_ptr(), max(n_bytes, 1),
                                  idoff_i.data_ptr(), st_i.data_ptr(), stream=streams[i].cuda_stream,
                                  cut_ptr=d_cut.data_ptr() if d_cut is not None else 0, mode=kmode)
            if coll:   # the single collective: RCCL over xGMI with nccl, gloo in rehearsals
                if red_dev.type == "cpu":
                    hc = h.cpu()
                    ddist.allreduce_histogram(hc)
                    h.copy_(hc)
                else:
                    pending[b] = ddist.allreduce_histogram(h, async_op=True)

    def drain():   # every outstanding all-reduce is ordered before what the stream does next
        for b in range(len(d_hists)):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None

    def all_sum(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    log("GPU ready, warmup")
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if inflight == 1:   # the pass timings ride the timed steps' dispatches (dpt_ctx_profile)
        enc.profile(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # With batches in flight the passes of consecutive steps overlap, so a call's own pass times mean
    # little and their events cost the timed steps ~1 %: the roofline's pass timing then comes from a
    # separate one-stream run of prof_steps steps after the timed region (the same calls, one context).
    prof_steps = 0
    if inflight > 1:
        prof_steps = max(3, min(args.steps, 10))
        enc.profile(True)
        for _ in range(prof_steps):
            step(one_stream=True)
        drain()
        torch.cuda.synchronize()
    ms_stage, launches = enc.profile_read()
    enc.profile(False)
    # secondary: the encode alone through dpt_encode_padded (ids left at each string's byte offset,
    # per-string counts; no finish pass, no histogram) -- reported beside `value`, never as it
    d_pids = torch.empty(max(n_bytes, 1), dtype=torch.int32, device=dev)
    d_cnt = torch.empty(max(M, 1), dtype=torch.int64, device=dev)
    d_pst = torch.empty(max(M, 1), dtype=torch.int32, device=dev)

    def step_padded():
        enc.encode_device_padded(d_text.data_ptr(), n_bytes, d_off.data_ptr(), M, d_pids.data_ptr(), max(n_bytes, 1),
                                 d_cnt.data_ptr(), d_pst.data_ptr(), stream=stream,
                                 cut_ptr=d_cut.data_ptr() if d_cut is not None else 0, mode=kmode)

    for _ in range(args.warmup):
        step_padded()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0p = time.perf_counter()
    for _ in range(args.steps):
        step_padded()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dtp = time.perf_counter() - t0p
    if world > 1:
        t = torch.tensor([dtp], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dtp = float(t.item())
    padded_same = bool(torch.equal(d_cnt[:M], (d_idoff[1:] - d_idoff[:-1])[:M]) and torch.equal(d_pst[:M], d_status[:M]))
    # the other contexts' last steps (those that ran one): the same outputs, or the run is void
    for (ids_i, idoff_i, st_i), ran_i in list(zip(outs, ran))[1:]:
        if ran_i and not (torch.equal(idoff_i, d_idoff) and torch.equal(st_i[:M], d_status[:M]) and
                          torch.equal(ids_i[: n_tok_rank_of(d_idoff)], d_ids[: n_tok_rank_of(d_idoff)])):
            raise SystemExit("bench: the contexts' outputs differ")

    # every unbounded-pass string fitted the arena (else it has status 3 and the device path refused it)
    need, cap = enc.long_need()
    if need > cap:
        raise SystemExit(f"bench: the unbounded pass needed {need} arena bytes of {cap}: reserve more")
    hist = d_hists[(n_step[0] - 1) % len(d_hists)].cpu().numpy()   # the last step's reduced histogram
    n_tok_rank = int(d_idoff[-1].item())
    n_tok_all = int(hist[N_BINS])          # after the all-reduce: all ranks' ids
    ok_strings = int(hist[N_BINS + 2])
    bytes_all = all_sum(float(n_bytes))
    raw_all = all_sum(float(raw_text_bytes))
    strings_all = int(all_sum(float(M)))

    # roofline of the dominant kernel (tokenize), SURVEY.md §8d bytes per launch (ids at 4 bytes)
    k_ms = ms_stage[0] / max(launches, 1)
    # staged ids are int16 when every vocabulary id is in 0..32767 (dpt_api.cpp ids16), else int32
    id_bytes = 2 if 0 <= min(t2i.values()) and max(t2i.values()) <= 32767 else 4
    alg_bytes = algorithmic_bytes(n_bytes, M, n_tok_rank)
    alg_staged = algorithmic_bytes(n_bytes, M, n_tok_rank, id_bytes)
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9

    log(f"timed {args.steps} steps in {dt:.4f} s; exact-match check")
    # exact match vs the CPU DP (C oracle): every rank checks its own shard, counts are summed
    from oracle import oracle
    per_rank_threads = max(1, cores // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))
    S = M if args.exact_sample is None else min(args.exact_sample, M)
    ids_h = d_ids.cpu().numpy()
    off_h = d_idoff.cpu().numpy().view(np.uint64)
    st_h = d_status.cpu().numpy()
    ov = oracle.OracleVocab(t2i)
    omode = oracle.ATOMS if bloom else oracle.PRESPLIT if presplit else oracle.RAW
    rids, roff, rst, _ = ov.encode_csr(text, offs[: S + 1], mode=omode, cut_mask=cut, nthreads=per_rank_threads)
    same = exact_matches(ids_h, off_h, st_h, rids, roff, rst, S)
    same_all, checked_all = all_sum(float(same)), all_sum(float(S))
    exact = {"rate": same_all / max(checked_all, 1.0), "sample": int(checked_all), "checker": "oracle/dp_oracle.c",
             "per_rank": "each rank checks %s of its own shard" % ("all" if args.exact_sample is None else "a prefix")}
    if rank == 0 and cpu is not None:
        t0c = time.perf_counter()
        S2 = min(65536, M)
        ov.encode_csr(text, offs[: S2 + 1], mode=omode, cut_mask=cut, nthreads=cores)
        cpu["c_restatement_bytes_per_s"] = int(offs[S2]) / (time.perf_counter() - t0c)
        cpu["c_restatement_threads"] = cores

    if rank == 0:
        value = bytes_all * args.steps / dt
        line = {
            "metric": "input bytes/sec/GPU + exact-match rate vs CPU DP, 256-byte strings"
                      if args.workload == "cfg2" else "input bytes/sec/GPU + exact-match rate vs CPU DP (%s)" % args.workload,
            "value": value,
            "unit": "bytes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": data,
            "config": {"workload": wl, "strings_total": strings_all,
                       "strings_per_gpu": M, "bytes_per_string": Lb,
                       "vocab": ("synthetic byte-level BPE 250680" if bloom else
                                 "synthetic toy 1000" if args.workload == "cfg1" else "synthetic llama-shaped 32000"),
                       "parallelism": f"dp{world} ({scaling} scaling: corpus shards, 1 all-reduce of the histogram per step)"},
            "per_gpu_bytes_per_s": value / world,
            "tokens_per_byte": n_tok_all / max(bytes_all, 1.0),
            **({"raw_text_bytes_per_s": raw_all * args.steps / dt, "raw_text_bytes": int(raw_all)} if presplit else {}),
            "ok_strings": ok_strings,
            # the reduced histogram itself (tests/test_gpu_sharded.py compares ranks x shards runs)
            "histogram": {"n_bins": N_BINS, "sha256": hashlib.sha256(hist.astype("<i8").tobytes()).hexdigest(),
                          "total_ids": n_tok_all, "total_strings": int(hist[N_BINS + 1]),
                          "status": [int(x) for x in hist[N_BINS + 2:N_BINS + 7]]},
            "exact_match": exact,
            "batches_in_flight": inflight,   # N > 1: step k on context + stream k % N (small shards; see --inflight)
            "stage_ms_per_step": {"tokenize": ms_stage[0] / max(launches, 1)},   # finish (offsets + CSR ids): rocprof
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic_for(M, Lb) if (args.workload == "cfg2" and world == 1) else None,
                         # (template arguments: CH, G, BIG, WIDE, staged id width, RAW, SOLO, mode constant)
                         "kernel": ("tokenize_kernel<256,64,false,true,0,false,false,2>" if bloom else
                                    "tokenize_kernel<256,16,false,false,%d,%s,false,%d>" % (1 if id_bytes == 2 else 2,
                                                                                          "false" if presplit else "true",
                                                                                          1 if presplit else -1)),
                         "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes_formula": "N_in + 4*N_tok + 8(N+1) + 8(N+1) + 4N (SURVEY.md 8d)",
                         "alg_bytes_staged_width": alg_staged, "staged_id_bytes": id_bytes,
                         "frac_staged_width": alg_staged / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         **({"note": "%d batches in flight overlap consecutive steps' passes: the pass timing here "
                                     "is from a separate one-stream run of %d steps after the timed region (HIP events "
                                     "on its dispatches), not from the timed steps" % (inflight, prof_steps)} if inflight > 1 else {})},
            "cpu_baseline": cpu,
            "padded_layout": {"api": "dpt_encode_padded (ids at each string's byte offset + per-string counts, no CSR pass); encode only, no histogram",
                              "ms_per_step": dtp / args.steps * 1e3, "bytes_per_s": bytes_all * args.steps / dtp,
                              "counts_and_status_equal_csr": padded_same},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
