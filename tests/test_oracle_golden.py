"""Pin the oracle: the C restatement (oracle/dp_oracle.c) and the Python port
(oracle/ref_port.py) against the golden vectors produced by the reference itself
(tests/golden/make_golden.py) and against the reference's own KATs
(reference tests/test_tokenization_algorithms.py:14-48)."""
import pytest

from conftest import CORPUS_FIXTURES, load_golden
from oracle import oracle, ref_port
from conftest import vocab_sha


@pytest.mark.parametrize("name", CORPUS_FIXTURES)
def test_c_oracle_matches_reference_vectors(name, vocabs):
    g = load_golden(name)
    t2i = vocabs[g["vocab"]]
    assert vocab_sha(t2i) == g["vocab_sha256"], "synthetic vocab drifted from the golden fixtures"
    cases = [c for c in g["cases"] if not c.get("skipped")]
    ov = oracle.OracleVocab(t2i)
    got = ov.encode_strs([c["text"] for c in cases])
    bad = [(c["text"][:40], c["status"], st) for c, (ids, st) in zip(cases, got)
           if ids != c["ids"] or st != c["status"]]
    assert not bad, bad[:5]


def test_c_oracle_capped_lengths(vocabs):
    import numpy as np
    g = load_golden("cfg2_llama32k.json.gz")
    ov = oracle.OracleVocab(vocabs["llama32k"])
    enc = [c["text"].encode() for c in g["cases"]]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(e) for e in enc])
    _, _, st, capped = ov.encode_csr(np.frombuffer(b"".join(enc), dtype=np.uint8), offs)
    for c, cl in zip(g["cases"], capped):
        if c.get("capped") is not None:
            assert cl == c["capped"]


def test_small_random_cases():
    g = load_golden("small_random.json.gz")
    for c in g["cases"]:
        t2i = {t: i for i, t in enumerate(c["vocab"])}
        ov = oracle.OracleVocab(t2i)
        (ids, st), = ov.encode_strs([c["text"]])
        assert (ids, st) == (c["ids"], c["status"]), c["text"]
        pids, pst = ref_port.dp_tokenize_raw(c["text"], t2i)
        assert (pids, pst) == (c["ids"], c["status"]), c["text"]
        for w in c["words"]:
            toks, n = ref_port.enumerate_shortest(w["atoms"], set(c["vocab"]))
            assert toks == w["tokenizations"] and n == w["len"]


@pytest.mark.parametrize("name", ["edge_llama32k.json.gz", "cfg1_toy1k.json.gz"])
def test_python_port_matches_reference_vectors(name, vocabs):
    g = load_golden(name)
    t2i = vocabs[g["vocab"]]
    for c in g["cases"][:300]:
        assert ref_port.dp_tokenize_raw(c["text"], t2i) == (c["ids"], c["status"])


def test_reference_kats():
    k = load_golden("reference_kats.json")
    for t in k["lengths"]:
        assert t["ref_min_tokens"] == t["expected"]
        assert ref_port.min_tokens_for_string(t["text"], set(t["vocab"])) == t["expected"]
        toks, n = ref_port.enumerate_shortest(list(t["text"]), set(t["vocab"]))
        assert toks == t["ref_tokenizations"] and n == t["ref_capped_len"]
    for t in k["membership"]:
        toks, n = ref_port.enumerate_shortest(t["text"], t["vocab"])
        assert toks == t["ref_tokenizations"] and n == t["ref_len"]
        for m in t["must_contain"]:
            assert m in toks
        assert ref_port.longest_token_choice(toks) == t["ref_selected"]
        # the C oracle's selection == obtain_longest_token: pre-split mode with no cuts is the
        # bare DP over code-point atoms (no '▁' prefix), i.e. the KAT's own call
        import numpy as np
        t2i = {tok: i for i, tok in enumerate(dict.fromkeys(t["vocab"]))}
        inv = {i: tok for tok, i in t2i.items()}
        b = t["text"].encode()
        ids, id_off, st, _ = oracle.OracleVocab(t2i).encode_csr(
            np.frombuffer(b, dtype=np.uint8), np.array([0, len(b)], dtype=np.uint64),
            mode=oracle.PRESPLIT, cut_mask=np.zeros(len(b), dtype=np.uint8))
        assert st[0] == 0
        assert [inv[int(i)] for i in ids] == t["ref_selected"]
