"""Row f3 at BLOOM scale: the BLOOM adapter (reference
packages/tokenizer_utils.py:98-181) over a 250,680-entry synthetic byte-level BPE
(tests/golden/make_bloom_tokenizer.py --big) -- tokens of up to 41 code points (the one-string-
per-wave ``tokenize_kernel<256,64,..>``), ids up to 250,679 (int32 staging), a deep trie -- against
400 strings the reference's own dp_tokenize_bloom produced (tests/golden/make_golden.py bloom_big).

The real ``bigscience/bloom-3b`` tokenizer.json is not available offline: parity with the real
BLOOM vocabulary stays unpinned; this pins the same code path at the same scale."""
import tempfile

import numpy as np
import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def big():
    import bloom_fixture as bf
    g = load_golden("bloom_big_cases.json.gz")
    v = bf.big_vocab()
    d = tempfile.TemporaryDirectory()
    hf = bf.make_hf_cache(d.name, big=True)
    yield {"g": g, "vocab": v, "hf": hf, "tokz": bf.bloom_tokenizer(hf), "texts": bf.bloom_big_texts(v)}
    d.cleanup()


def _words_of_atoms(tokz, v, text):
    # the adapter's atomisation (reference tokenizer_utils.py:152-157, :160-162)
    words = [w for w, _ in tokz._tokenizer.pre_tokenizer.pre_tokenize_str(text)]
    return [tokz.convert_ids_to_tokens([v[c] for c in w]) for w in words]


def test_fixture_covers_the_scale(big):
    """The fixture exercises what the toy BLOOM fixture cannot: > 16-code-point tokens, ids past
    32767, and the generator reproduces its texts."""
    g, v = big["g"], big["vocab"]
    assert len(v) == 250680 and g["skipped_over_time_limit"] == 0
    assert [c["text"] for c in g["cases"]] == big["texts"]
    inv = {i: t for t, i in v.items()}
    ids = [i for c in g["cases"] if c["ids"] for i in c["ids"]]
    assert max(ids) > 32767 and sum(i > 32767 for i in ids) > 1000
    assert sum(len(inv[i]) > 16 for i in ids) > 1000
    assert max(len(w) for c in g["cases"] for w in c["text"].split()) > 64   # words past the 64-atom rows


def test_oracle_atoms_mode_matches_reference(big):
    """The C oracle in atoms mode (the adapter's DPT_MODE_ATOMS input) equals the reference on every
    fixture string -- pins the checker used by the GPU test and bench.py --workload bloom."""
    from dptok.engine import pack_word_atoms
    from oracle import oracle
    g, v, tokz = big["g"], big["vocab"], big["tokz"]
    strings = [_words_of_atoms(tokz, v, c["text"]) for c in g["cases"]]
    keep = [i for i, s in enumerate(strings) if s]
    text, offs, cut = pack_word_atoms([strings[i] for i in keep])
    ids, id_off, st, _ = oracle.OracleVocab(v).encode_csr(text, offs, mode=oracle.ATOMS, cut_mask=cut)
    assert not np.any(st)
    got = {i: ids[int(id_off[k]):int(id_off[k + 1])].tolist() for k, i in enumerate(keep)}
    for i, c in enumerate(g["cases"]):
        assert got.get(i, []) == c["ids"], c["text"]


@pytest.mark.gpu
def test_token_hash_table_builds_at_bloom_scale(big):
    """C2's token hash table (one bucket load per selected token) exists for the 250,680-entry
    vocabulary.  Round 2's fingerprint was a function of the bucket hash (32 bits per key): the
    vocabulary's ~7 expected full collisions made every seed fail, and C2 re-walked every token."""
    import dptok
    st = dptok.Vocab(big["vocab"]).stats
    assert st["n_tokens"] == 250680
    assert st["hash_max_probe"] == 2 and st["hash_buckets"] >= 250680 // 2   # two-choice buckets (round 5)


@pytest.mark.gpu
def test_dp_tokenize_bloom_scale_matches_reference(big):
    from packages.tokenizer_utils import dp_tokenize_bloom
    g = big["g"]
    dp_tokenize, decode = dp_tokenize_bloom(big["tokz"], big["hf"])
    st = dp_tokenize.engine.vocab.stats
    assert st["max_cp"] > 16 and st["max_cp"] <= 64      # the 64-lane rows kernel
    for c in g["cases"][:40]:
        assert dp_tokenize(c["text"]) == c["ids"], c["text"]
    assert dp_tokenize.batch([c["text"] for c in g["cases"]]) == [c["ids"] for c in g["cases"]]
    assert isinstance(decode(g["cases"][3]["ids"]), str)


@pytest.mark.gpu
def test_bloom_scale_synthetic_corpus_vs_oracle(big):
    """bench.py --workload bloom's corpus (dptok.synth.bloom_like_corpus, atoms mode) on the GPU
    against the C oracle, bit-exact ids and status."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    v = big["vocab"]
    text, offs, cut = synth.bloom_like_corpus(3000, v, seed=7)
    enc = Encoder(Vocab(v, 0))
    ids, id_off, st, _ = enc.encode_csr(text, offs, mode="atoms", cut_mask=cut)
    rids, roff, rst, _ = oracle.OracleVocab(v).encode_csr(text, offs, mode=oracle.ATOMS, cut_mask=cut)
    assert np.array_equal(st, rst)
    assert np.array_equal(np.asarray(id_off, dtype=np.uint64), np.asarray(roff, dtype=np.uint64))
    assert np.array_equal(ids[: int(roff[-1])], rids)


@pytest.mark.gpu
def test_bloom_scale_padded_layout_vs_oracle(big):
    """dpt_encode_padded with the 250k-entry vocabulary (64-lane rows kernel, int32 ids, atoms mode):
    each string's ids at its byte offset equal the C oracle's."""
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    v = big["vocab"]
    text, offs, cut = synth.bloom_like_corpus(2000, v, seed=11)
    enc = Encoder(Vocab(v, 0))
    n, nb = len(offs) - 1, int(offs[-1])
    dt = torch.from_numpy(np.array(text)).cuda()
    do = torch.from_numpy(np.asarray(offs, dtype=np.uint64).view(np.int64)).cuda()
    dc = torch.from_numpy(np.array(cut)).cuda()
    pids = torch.full((nb,), -9, dtype=torch.int32, device="cuda")
    cnt = torch.empty(n, dtype=torch.int64, device="cuda")
    pst = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    enc.encode_device_padded(dt.data_ptr(), nb, do.data_ptr(), n, pids.data_ptr(), nb, cnt.data_ptr(), pst.data_ptr(),
                             cut_ptr=dc.data_ptr(), stream=s, mode="atoms")
    torch.cuda.synchronize()
    rids, roff, rst, _ = oracle.OracleVocab(v).encode_csr(text, offs, mode=oracle.ATOMS, cut_mask=cut)
    p, c = pids.cpu().numpy(), cnt.cpu().numpy()
    assert np.array_equal(pst.cpu().numpy(), rst)
    assert np.array_equal(c.astype(np.uint64), np.diff(np.asarray(roff, dtype=np.uint64)))
    for i in range(n):
        a, b = int(offs[i]), int(roff[i])
        assert np.array_equal(p[a:a + int(c[i])], rids[b:b + int(c[i])]), i
