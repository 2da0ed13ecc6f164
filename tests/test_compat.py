"""The reference-compatible surface (dp-tokenization_amd/packages, inspect_tokenizer.py) against
fixtures produced by the reference itself (tests/golden/make_golden.py).

CPU tests cover the host-side string utilities; ``gpu`` tests cover every DP-backed name."""
import math
import os

import numpy as np
import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def compat():
    return load_golden("compat_cases.json.gz")


# ------------------------------------------------------------------ host utilities (CPU)

def test_merge_tokens_matches_reference(compat):
    from packages.tokenizer_utils import merge_tokens
    for c in compat["merge_tokens"]:
        assert merge_tokens(c["tokens"], sep=c["sep"]) == c["out"], c


def test_pretokenize_raw_matches_reference(compat):
    from packages.tokenizer_utils import _InverseDict, pretokenize_raw
    pre = pretokenize_raw(_InverseDict({"<0x0A>": "\n"}))
    for c in compat["pretokenize_raw"]:
        assert pre(c["text"]) == c["out"], c["text"]


def test_pretokenize_with_llama_matches_reference(compat):
    from dptok import synth
    from fake_llama import FakeLlamaTokenizer
    from packages.tokenizer_utils import _InverseDict, pretokenize_with_llama
    t2i = synth.llama_shaped_vocab()
    pre = pretokenize_with_llama(FakeLlamaTokenizer(t2i), _InverseDict(t2i))
    for c in compat["llama_mode"]:
        assert pre(c["text"]) == c["words"], c["text"]


def test_obtain_longest_token_semantics():
    from packages.dp_tokenize import obtain_longest_token
    assert obtain_longest_token([["ab", "c"], ["a", "bc"], ["abc"]]) == ["abc"]
    assert obtain_longest_token([["ab", "c"], ["a", "bc"]]) == ["ab", "c"]   # first argmax
    with pytest.raises(ValueError):
        obtain_longest_token([])


def test_inspect_obtain_token_compositions():
    import inspect_tokenizer as it
    vocab = {"a": 0, "b": 1, "c": 2, "ab": 3, "bc": 4, "abc": 5}
    merges = ["a b", "b c", "ab c"]
    assert it.obtain_token_compositions("abc", vocab, merges) == [["ab", "c"], ["a", "b", "c"]]
    assert it.obtain_token_compositions("a", vocab, merges) == [["a"]]


def test_obtain_token_compositions_matches_reference():
    """tests/golden/compositions.json.gz: the reference's own obtain_token_compositions
    (inspect_tokenizer.py:17-42) over the synthetic BPEs' merges (make_compositions.py) -- every
    token of the 1,800-entry BPE with its merges as a list, and tokens of 2..41 code points (and
    non-tokens) of the 250,680-entry BPE with its merges as a set."""
    import gzip
    import json
    import lzma
    import inspect_tokenizer as it
    from conftest import GOLDEN
    g = load_golden("compositions.json.gz")
    small = json.load(gzip.open(os.path.join(GOLDEN, "bloom_synth_tokenizer.json.gz"), "rt", encoding="utf-8"))
    with lzma.open(os.path.join(GOLDEN, "bloom_big_tokenizer.json.xz"), "rt", encoding="utf-8") as fh:
        big = json.load(fh)
    merges = lambda m: [x if isinstance(x, str) else " ".join(x) for x in m]   # noqa: E731
    src = {"small": (small["model"]["vocab"], merges(small["model"]["merges"])),
           "big": (big["model"]["vocab"], set(merges(big["model"]["merges"])))}
    assert len(g["cases"]) > 2000 and any(len(c["token"]) > 30 for c in g["cases"])
    for c in g["cases"]:
        v, m = src[c["source"]]
        assert it.obtain_token_compositions(c["token"], v, m) == c["compositions"], c["token"]


# ------------------------------------------------------------------ DP-backed names (GPU)

@pytest.mark.gpu
def test_dp_tokenize_llama_raw_mode(vocabs):
    from fake_llama import FakeLlamaTokenizer
    from packages.tokenizer_utils import dp_tokenize_llama
    g = load_golden("cfg2_llama32k.json.gz")
    dp_tokenize, decode = dp_tokenize_llama(FakeLlamaTokenizer(vocabs["llama32k"]), "raw")
    for c in g["cases"][:100]:
        assert dp_tokenize(c["text"]) == c["ids"]
    assert dp_tokenize.batch([c["text"] for c in g["cases"]]) == [c["ids"] for c in g["cases"]]
    e = load_golden("edge_llama32k.json.gz")
    for c in e["cases"]:
        if c["status"] == 0:
            assert dp_tokenize(c["text"]) == c["ids"]
        else:
            with pytest.raises(ValueError if c["status"] == 1 else IndexError):
                dp_tokenize(c["text"])


@pytest.mark.gpu
def test_dp_tokenize_llama_llama_mode(vocabs, compat):
    from fake_llama import FakeLlamaTokenizer
    from packages.tokenizer_utils import dp_tokenize_llama
    dp_tokenize, decode = dp_tokenize_llama(FakeLlamaTokenizer(vocabs["llama32k"]))   # default 'llama'
    for c in compat["llama_mode"]:
        if c["status"] == 0:
            ids = dp_tokenize(c["text"])
            assert ids == c["ids"], c["text"]
            assert isinstance(decode(ids), str)   # tokenizer.decode(ids)[4:] (fake decode, not Llama's)
        else:
            with pytest.raises((ValueError, IndexError)):
                dp_tokenize(c["text"])


@pytest.mark.gpu
def test_unknown_pretokenize_option_fails_at_call_time(vocabs):
    from fake_llama import FakeLlamaTokenizer
    from packages.tokenizer_utils import dp_tokenize_llama
    dp_tokenize, _ = dp_tokenize_llama(FakeLlamaTokenizer(vocabs["llama32k"]), "bogus")
    with pytest.raises(NameError):
        dp_tokenize("abc")


@pytest.mark.gpu
def test_compute_shortest_tokenizations_enumeration_order():
    """Every optimal tokenization, in the reference's DFS order, for 2000 tie-heavy words."""
    from packages.dp_tokenize import compute_shortest_tokenizations, obtain_longest_token
    g = load_golden("small_random.json.gz")
    n = 0
    for c in g["cases"]:
        for w in c["words"]:
            toks, length = compute_shortest_tokenizations(w["atoms"], set(c["vocab"]), False, None)
            assert toks == w["tokenizations"], (w["atoms"], c["vocab"])
            assert length == w["len"]
            if toks:
                obtain_longest_token(toks)
            n += 1
    assert n > 1000
    with pytest.raises(IndexError):
        compute_shortest_tokenizations([], {"a"}, False, None)


@pytest.mark.gpu
def test_reference_kats_through_drop_in():
    import inspect_tokenizer as it
    from packages.dp_tokenize import compute_shortest_tokenizations, obtain_longest_token
    k = load_golden("reference_kats.json")
    for t in k["lengths"]:
        assert it.min_tokens_for_string(t["text"], set(t["vocab"])) == t["expected"]
        toks, n = compute_shortest_tokenizations(list(t["text"]), set(t["vocab"]), False, None)
        assert toks == t["ref_tokenizations"] and n == t["ref_capped_len"]
    for t in k["membership"]:
        toks, n = compute_shortest_tokenizations(t["text"], t["vocab"], False, "")
        assert toks == t["ref_tokenizations"] and n == t["ref_len"]
        for m in t["must_contain"]:
            assert m in toks
        assert obtain_longest_token(toks) == t["ref_selected"]


@pytest.mark.gpu
def test_inspect_min_tokens_uncapped(compat):
    import inspect_tokenizer as it
    for c in compat["inspect_min_tokens"]:
        got = it.min_tokens_for_string(c["text"], set(c["vocab"]))
        want = math.inf if c["min"] == "inf" else c["min"]
        assert got == want, c
        assert it.compute_length_of_most_efficient_tokenization(list(c["text"]), set(c["vocab"])) == want


@pytest.mark.gpu
def test_disregard_word_initial_marker():
    from packages.dp_tokenize import compute_shortest_tokenizations
    V = {"##ab", "##c", "a", "b"}
    toks, n = compute_shortest_tokenizations(list("abc"), V, True, "##")
    assert n == 2 and toks == [["ab", "c"]]


# ------------------------------------------------------------------ BLOOM adapter (row f3)

def test_bloom_fixture_shape():
    """The synthetic BLOOM-shaped tokenizer loads where the reference reads it and pre-tokenizes
    into byte-level words; the reference-generated fixture covers the texts."""
    import tempfile
    from bloom_fixture import bloom_texts, bloom_tokenizer, make_hf_cache
    g = load_golden("bloom_cases.json.gz")
    assert [c["text"] for c in g["cases"]] == bloom_texts()
    with tempfile.TemporaryDirectory() as d:
        tokz = bloom_tokenizer(make_hf_cache(d))
        words = [w for w, _ in tokz._tokenizer.pre_tokenizer.pre_tokenize_str("hello  world, café 😀")]
        assert words[0] == "hello" and "Ġworld" in words and all(w for w in words)


@pytest.mark.gpu
def test_dp_tokenize_bloom_matches_reference():
    import tempfile
    from bloom_fixture import bloom_tokenizer, make_hf_cache
    from packages.tokenizer_utils import dp_tokenize_bloom
    g = load_golden("bloom_cases.json.gz")
    with tempfile.TemporaryDirectory() as d:
        hf = make_hf_cache(d)
        tokz = bloom_tokenizer(hf)
        dp_tokenize, decode = dp_tokenize_bloom(tokz, hf)
        for c in g["cases"][:60]:
            assert dp_tokenize(c["text"]) == c["ids"], c["text"]
        assert dp_tokenize.batch([c["text"] for c in g["cases"]]) == [c["ids"] for c in g["cases"]]
        assert isinstance(decode(g["cases"][3]["ids"]), str)


@pytest.mark.gpu
def test_dp_tokenize_bloom_key_error_outside_vocab():
    """A character outside tokenizer.json's vocab raises KeyError (reference :155)."""
    import json
    import os
    import tempfile
    from bloom_fixture import SNAPSHOT, bloom_tokenizer, make_hf_cache
    from packages.tokenizer_utils import dp_tokenize_bloom
    with tempfile.TemporaryDirectory() as d:
        hf = make_hf_cache(d)
        tokz = bloom_tokenizer(hf)
        p = os.path.join(hf, SNAPSHOT, "tokenizer.json")
        with open(p) as fh:
            tj = json.load(fh)
        tj["model"]["vocab"] = {t: i for t, i in tj["model"]["vocab"].items() if "z" not in t}
        with open(p, "w") as fh:
            json.dump(tj, fh)
        dp_tokenize, _ = dp_tokenize_bloom(tokz, hf)
        assert dp_tokenize("abc def") == dp_tokenize.batch(["abc def"])[0]
        with pytest.raises(KeyError):
            dp_tokenize("lazy")
        assert dp_tokenize("") == []


# ------------------------------------------------------------------ inspect_tokenizer.compute_shortest_tokenizations

@pytest.fixture(scope="module")
def inspect_cst():
    return load_golden("inspect_cst_cases.json.gz")["cases"]


def test_inspect_cst_exceptions_match_reference(inspect_cst):
    """Every input the reference's inspect_tokenizer.compute_shortest_tokenizations (:88-146) rejects --
    the empty one: IndexError at :132 -- the drop-in rejects with the same exception type, before any
    device work (no GPU needed)."""
    import inspect_tokenizer as it
    bad = [c for c in inspect_cst if c["error"]]
    assert len(bad) >= 3 and any(not c["atoms"] for c in bad)
    for c in bad:
        with pytest.raises(Exception) as e:
            it.compute_shortest_tokenizations(list(c["atoms"]), set(c["vocab"]), c["disregard"], c["marker"])
        assert type(e.value).__name__ == c["error"], c


def test_inspect_cst_lengths_pinned_by_the_oracle(inspect_cst):
    """The reference's lengths (its inf-initialised DP, :109-129) equal the CPU restatement's
    (oracle/ref_port.min_tokens_for_string, test infrastructure) after the marker rule (:106-107) --
    the checker the GPU test below relies on agrees with the reference on every case."""
    from oracle import ref_port
    good = [c for c in inspect_cst if not c["error"]]
    assert len(good) >= 200 and sum(c["length"] == "inf" for c in good) < len(good) // 2
    for c in good:
        vocab = set(c["vocab"])
        if c["disregard"]:
            vocab = {t.lstrip(c["marker"]) for t in vocab}
        want = math.inf if c["length"] == "inf" else c["length"]
        assert ref_port.min_tokens_for_string(list(c["atoms"]), vocab) == want, c


def test_inspect_cst_lists_pinned_by_the_oracle(inspect_cst):
    """The reference's LISTS (its one-stack backtrace, :131-146, mixed branches included) equal the CPU
    restatement's (oracle/ref_port.inspect_shortest_tokenizations) on every case: the checker of the GPU
    test below is pinned."""
    from oracle import ref_port
    good = [c for c in inspect_cst if not c["error"]]
    mixed = 0
    for c in good:
        vocab = set(c["vocab"])
        if c["disregard"]:
            vocab = {t.lstrip(c["marker"]) for t in vocab}
        toks, n = ref_port.inspect_shortest_tokenizations(list(c["atoms"]), vocab)
        assert toks == c["tokenizations"], c
        mixed += any(t not in vocab for tk in toks for t in tk)
    assert mixed >= 5   # the fixture exercises the backtrace's mixed branches


def test_inspect_cst_backtrace_replay_matches_oracle():
    """The drop-in's host replay of the backtrace (inspect_tokenizer._single_stack_backtrace), fed the
    optimal-predecessor lists of reachable ends, equals the restatement on random cases (no GPU: the lists
    come from a CPU DP here; on the GPU they come from the uncapped DP's edge masks)."""
    import random
    import inspect_tokenizer as it
    from oracle import ref_port
    rng = random.Random(7)
    for _ in range(400):
        alpha = "abc"[: rng.randint(2, 3)]
        vocab = set(alpha) | {"".join(rng.choice(alpha) for _ in range(rng.randint(2, 4))) for _ in range(rng.randint(0, 9))}
        atoms = [rng.choice(alpha) for _ in range(rng.randint(1, 11))]
        want, n = ref_port.inspect_shortest_tokenizations(atoms, vocab)
        cost, preds = ref_port.forward_dp(atoms, vocab)   # every atom is a token: capped == uncapped here
        assert cost[-1] == n
        assert it._single_stack_backtrace(atoms, lambda e: list(preds[e])) == want


@pytest.mark.gpu
def test_inspect_cst_lists_match_reference(inspect_cst):
    """Round 6: the drop-in's list AND length equal the reference's on every case (GPU uncapped DP with edges
    + the host replay of the one-stack backtrace)."""
    import inspect_tokenizer as it
    for c in inspect_cst:
        if c["error"]:
            continue
        toks, n = it.compute_shortest_tokenizations(list(c["atoms"]), set(c["vocab"]), c["disregard"], c["marker"])
        want = math.inf if c["length"] == "inf" else c["length"]
        assert n == want and toks == c["tokenizations"], c


@pytest.mark.gpu
def test_inspect_cst_random_vs_oracle():
    """Beyond the fixture: random cases with out-of-vocabulary atoms (unreachable ends, capped != uncapped)
    and tokens of up to 70 atoms (far predecessors), the drop-in against the restatement."""
    import random
    import inspect_tokenizer as it
    from oracle import ref_port
    rng = random.Random(17)
    for k in range(300):
        alpha = "abcd"[: rng.randint(2, 4)]
        vocab = {ch for ch in alpha if rng.random() < 0.85}
        vocab |= {"".join(rng.choice(alpha) for _ in range(rng.randint(2, 5))) for _ in range(rng.randint(0, 14))}
        atoms = [rng.choice(alpha) for _ in range(rng.randint(1, 14))]
        if k % 50 == 0:   # a token of 66..70 atoms: its predecessor comes back as a far pair
            long = [rng.choice(alpha) for _ in range(rng.randint(66, 70))]
            vocab.add("".join(long))
            atoms = atoms + long
        want = ref_port.inspect_shortest_tokenizations(atoms, vocab)
        assert it.compute_shortest_tokenizations(atoms, set(vocab), False, None) == want, (atoms, sorted(vocab))
