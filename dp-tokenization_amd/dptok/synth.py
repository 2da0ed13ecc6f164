"""Synthetic vocabularies and corpora for the five BASELINE.json configurations.

No Llama-2 ``tokenizer.model`` exists offline (SURVEY.md §0 finding 6), so every
report that uses ``llama_shaped_vocab`` says "synthetic Llama-shaped 32k vocab".

Vocabulary recipe, shaped like ``LlamaTokenizer.get_vocab()``
(the dict that ``dp_tokenize_llama`` turns into ``t2i``/``vocab`` at
reference ``packages/tokenizer_utils.py:53-57``):

* ids 0..2 ``<unk>``, ``<s>``, ``</s>``; ids 3..258 the byte tokens ``<0x00>``..``<0xFF>``;
* ``'▁'``, the 94 printable ASCII characters 0x21..0x7E, and ``'▁'+c`` for each;
* (our extension, for the Arabic-shaped config 5) the code points U+0621..U+064A,
  ``'▁'+c`` for each, and random 2..5-letter Arabic entries;
* seeded random fill up to ``size``: length drawn from {2,2,2,3,3,4,5,6,7,8}; each
  character from ``etaoinshrdlucmfwypvbgkjqxz`` with p=0.8, otherwise printable
  ASCII; a ``'▁'`` prefix with p=0.4; duplicates dropped.

This guarantees every raw-mode ASCII atom is in the vocab,
so random printable strings never fail except for a leading space (atom ``'▁ '``).

Corpora are generated from a counter-based PRNG (numpy Philox) keyed by
``(seed, global string index)``, so a shard is identical at any GPU count.
"""
from __future__ import annotations

import random
from typing import Dict, List, Tuple

import numpy as np

SPACE_MARK = "▁"  # '▁'
PRINTABLE = [chr(c) for c in range(0x21, 0x7F)]
LETTERS = "etaoinshrdlucmfwypvbgkjqxz"
ARABIC = [chr(c) for c in range(0x0621, 0x064B)]


def _fill(vocab: Dict[str, int], size: int, rng: random.Random, lengths, p_letter, p_mark):
    while len(vocab) < size:
        n = rng.choice(lengths)
        chars = []
        for _ in range(n):
            if rng.random() < p_letter:
                chars.append(rng.choice(LETTERS))
            else:
                chars.append(rng.choice(PRINTABLE))
        tok = "".join(chars)
        if rng.random() < p_mark:
            tok = SPACE_MARK + tok
        if tok not in vocab:
            vocab[tok] = len(vocab)


def llama_shaped_vocab(size: int = 32000, seed: int = 0, arabic: bool = True) -> Dict[str, int]:
    """Synthetic Llama-shaped vocabulary: token string -> id (ids contiguous)."""
    rng = random.Random(seed)
    vocab: Dict[str, int] = {}
    for t in ("<unk>", "<s>", "</s>"):
        vocab[t] = len(vocab)
    for b in range(256):
        vocab["<0x%02X>" % b] = len(vocab)
    vocab.setdefault(SPACE_MARK, len(vocab))
    for c in PRINTABLE:
        vocab.setdefault(c, len(vocab))
    for c in PRINTABLE:
        vocab.setdefault(SPACE_MARK + c, len(vocab))
    if arabic:
        for c in ARABIC:
            vocab.setdefault(c, len(vocab))
            vocab.setdefault(SPACE_MARK + c, len(vocab))
        n_ar = 0
        while n_ar < 1500:
            tok = "".join(rng.choice(ARABIC) for _ in range(rng.choice((2, 2, 3, 3, 4, 5))))
            if rng.random() < 0.4:
                tok = SPACE_MARK + tok
            if tok not in vocab:
                vocab[tok] = len(vocab)
                n_ar += 1
    _fill(vocab, size, rng, (2, 2, 2, 3, 3, 4, 5, 6, 7, 8), 0.8, 0.4)
    return vocab


def toy_vocab(size: int = 1000, seed: int = 0) -> Dict[str, int]:
    """1000-entry toy vocabulary for config 1 (CPU plumbing case)."""
    rng = random.Random(seed + 1000003)
    vocab: Dict[str, int] = {}
    for t in ("<unk>", "<s>", "</s>", "<0x0A>"):
        vocab[t] = len(vocab)
    vocab[SPACE_MARK] = len(vocab)
    for c in PRINTABLE:
        vocab.setdefault(c, len(vocab))
    for c in PRINTABLE:
        vocab.setdefault(SPACE_MARK + c, len(vocab))
    _fill(vocab, size, rng, (2, 2, 2, 3, 3, 4), 0.85, 0.4)
    return vocab


# --------------------------------------------------------------------------- corpora

def _philox_bytes(seed: int, first_block: int, n_u64: int) -> np.ndarray:
    bg = np.random.Philox(key=np.uint64(seed), counter=np.array([first_block, 0, 0, 0], dtype=np.uint64))
    return bg.random_raw(n_u64).view(np.uint8)


def random_ascii_corpus(n: int, length: int = 256, seed: int = 1, start: int = 0,
                        chunk: int = 1 << 16) -> Tuple[np.ndarray, np.ndarray]:
    """Config 1/2/3: ``n`` random printable-ASCII strings of ``length`` bytes.

    Byte 0 is drawn over 0x21..0x7E, bytes 1.. over 0x20..0x7E (space ~1/85).
    String ``g`` (global index ``start + i``) uses Philox blocks ``[g*B, (g+1)*B)``
    with ``B = ceil(length/32)`` (a block is 4 x u64 = 32 bytes).
    Returns ``(text u8[n*length], offsets u64[n+1])``.
    """
    blocks = (length + 31) // 32
    out = np.empty(n * length, dtype=np.uint8)
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        raw = _philox_bytes(seed, (start + c0) * blocks, m * blocks * 4).reshape(m, blocks * 32)[:, :length]
        raw = raw.astype(np.uint16)
        s = (0x20 + ((raw * 95) >> 8)).astype(np.uint8)
        s[:, 0] = (0x21 + ((raw[:, 0] * 94) >> 8)).astype(np.uint8)
        out[c0 * length:(c0 + m) * length] = s.reshape(-1)
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(length)
    return out, offs


_EN_FREQ = np.array([8.2, 1.5, 2.8, 4.3, 12.7, 2.2, 2.0, 6.1, 7.0, 0.15, 0.77, 4.0, 2.4, 6.7,
                     7.5, 1.9, 0.095, 6.0, 6.3, 9.1, 2.8, 0.98, 2.4, 0.15, 2.0, 0.074])
_EN_FREQ = _EN_FREQ / _EN_FREQ.sum()


def s2orc_like_corpus(n: int, seed: int = 4, start: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Config 4: abstract-shaped strings, lengths ~ N(1200, 400) clipped to [64, 4096].

    Pseudo-words (geometric lengths, mean ~6 letters, English letter frequencies,
    ~8% capitalised), separated by spaces; ~2% punctuation/digits; occasional
    '\\n'. Each string starts at a word. Keyed by (seed, global index).
    """
    parts: List[bytes] = []
    for g in range(start, start + n):
        rng = np.random.Generator(np.random.Philox(key=np.uint64(seed), counter=np.array([g, 0, 0, 0], dtype=np.uint64)))
        L = int(np.clip(rng.normal(1200, 400), 64, 4096))
        buf = bytearray()
        nw = L // 4 + 8
        wl = rng.geometric(1 / 6, size=nw)
        letters = rng.choice(26, size=int(wl.sum()), p=_EN_FREQ)
        extras = rng.random(size=(nw, 3))
        k = 0
        for w in range(nw):
            word = bytes((97 + letters[k:k + wl[w]]).astype(np.uint8))
            k += wl[w]
            if extras[w, 0] < 0.08:
                word = word[:1].upper() + word[1:]
            if extras[w, 1] < 0.02:
                word += b"0123456789.,;:()%-"[int(extras[w, 1] * 900) % 18:][:1]
            if buf:
                buf += b"\n" if extras[w, 2] < 0.01 else b" "
            buf += word
            if len(buf) >= L:
                break
        parts.append(bytes(buf[:L]))
    return _pack(parts)


def arabic_corpus(n: int, length: int = 256, seed: int = 5, start: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Config 5: Arabic-shaped UTF-8 (U+0621..U+064A, 2 bytes each), a space ~every 5 letters."""
    parts: List[bytes] = []
    for g in range(start, start + n):
        rng = np.random.Generator(np.random.Philox(key=np.uint64(seed), counter=np.array([g, 0, 0, 0], dtype=np.uint64)))
        cps = rng.integers(0x0621, 0x064B, size=length)
        sp = rng.random(size=length) < 0.2
        chars: List[str] = []
        nb = 0
        for i in range(length):
            c = " " if (sp[i] and i > 0 and chars and chars[-1] != " ") else chr(int(cps[i]))
            b = 1 if c == " " else 2
            if nb + b > length:
                break
            chars.append(c)
            nb += b
        parts.append("".join(chars).encode("utf-8"))
    return _pack(parts)


def _pack(parts: List[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    text = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return text, offs


def unpack(text: np.ndarray, offs: np.ndarray) -> List[str]:
    """CSR bytes -> list of Python strings (UTF-8)."""
    raw = text.tobytes()
    o = [int(x) for x in offs]
    return [raw[o[i]:o[i + 1]].decode("utf-8", "surrogatepass") for i in range(len(o) - 1)]


LLAMA_PREFIX = "<s>▁".encode("utf-8")   # the BOS piece, then SentencePiece's dummy-prefix '▁'
_SPACE_PIECE = "▁".encode("utf-8")
_NL_PIECE = b"<0x0A>"


def llama_words(text: np.ndarray, offs: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Raw strings -> the pre-split form llama mode hands the DP (reference tokenizer_utils.py:24-31, :7-22):
    per string the BOS word ``"<s>"``, then the text with every ``' '`` as ``'▁'`` opening a word (SentencePiece's
    normaliser, plus its dummy prefix before the first character) and ``'\\n'`` as its byte-fallback piece
    ``"<0x0A>"`` -- the words ``merge_tokens`` builds from the pieces of a Llama-2 SentencePiece model whose
    pieces never cross a '▁', written out as UTF-8 with a word-start mask (DPT_MODE_PRESPLIT).  Vectorised:
    -> (text, offs, cut) with cut[k] = 1 where a word starts."""
    offs = np.asarray(offs, dtype=np.uint64)
    text = np.asarray(text, dtype=np.uint8)[int(offs[0]):int(offs[-1])]
    offs = offs - offs[0]
    n = len(offs) - 1
    sp = text == 0x20
    nl = text == 0x0A
    width = 1 + 2 * sp.astype(np.int64) + 5 * nl.astype(np.int64)
    P = len(LLAMA_PREFIX)
    sid = np.repeat(np.arange(n, dtype=np.int64), np.diff(offs).astype(np.int64))   # string of each byte
    pos = np.cumsum(width) - width + P * (sid + 1)                                   # output position of each byte
    tot = np.zeros(n + 1, dtype=np.int64)
    tot[1:] = np.cumsum(np.bincount(sid, weights=width, minlength=n).astype(np.int64) + P)
    out = np.empty(int(tot[-1]), dtype=np.uint8)
    cut = np.zeros(int(tot[-1]), dtype=np.uint8)
    plain = ~(sp | nl)
    out[pos[plain]] = text[plain]
    for k in range(3):
        out[pos[sp] + k] = _SPACE_PIECE[k]
    for k in range(6):
        out[pos[nl] + k] = _NL_PIECE[k]
    base = tot[:-1]
    for k in range(P):
        out[base + k] = LLAMA_PREFIX[k]
    cut[base] = 1                    # "<s>"
    cut[base + 3] = 1                # the dummy prefix '▁' opens the first word
    cut[pos[sp]] = 1                 # every other '▁'
    return out, tot.astype(np.uint64), cut


def _gen_chunk(args):
    kind, n, start, kw = args
    return {"s2orc": s2orc_like_corpus, "arabic": arabic_corpus}[kind](n, start=start, **kw)


def generate_parallel(kind: str, n: int, start: int = 0, procs: int = 8, **kw) -> Tuple[np.ndarray, np.ndarray]:
    """``s2orc_like_corpus`` / ``arabic_corpus`` over [start, start+n) split across ``procs``
    forked processes (identical output: every string is keyed by its global index).  Call
    before any GPU work (fork)."""
    import multiprocessing as mp
    if procs <= 1 or n < 4096:
        return _gen_chunk((kind, n, start, kw))
    step = (n + procs - 1) // procs
    jobs = [(kind, min(step, n - s), start + s, kw) for s in range(0, n, step)]
    with mp.get_context("fork").Pool(len(jobs)) as pool:
        res = pool.map(_gen_chunk, jobs)
        pool.close()   # workers exit on their own (leaving the block would terminate them)
        pool.join()
    texts = [t for t, _ in res]
    lens = np.concatenate([np.diff(o) for _, o in res])
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens, dtype=np.uint64)
    return np.concatenate(texts), offs


# --------------------------------------------------------------------------- BLOOM-scale (row f3)

BYTE_SPACE = "Ġ"   # 'Ġ': the byte-level alphabet's space (GPT-2 bytes_to_unicode)


def bloom_word_pool(vocab: Dict[str, int]) -> Tuple[List[str], List[str]]:
    """(long, short): the vocabulary's all-ASCII-letter tokens (a leading 'Ġ' dropped), longer
    than 16 code points and 2..16 -- the words of ``bloom_like_corpus``."""
    words = sorted({t[1:] if t.startswith(BYTE_SPACE) else t for t in vocab})
    words = [w for w in words if w.isascii() and w.isalpha()]
    return [w for w in words if len(w) > 16], [w for w in words if 2 <= len(w) <= 16]


def bloom_like_corpus(n: int, vocab_or_pool, length: int = 256, seed: int = 8,
                      start: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The BLOOM-scale workload (``bench.py --workload bloom``): ``n`` pre-tokenized byte-level
    strings of at most ``length`` bytes, as the BLOOM adapter hands them to the GPU (atoms mode:
    every character an atom, words = the pre-tokenizer's blocks, 'Ġ'+word after the first).
    Words: 15 % the vocabulary's long tokens (> 16 code points), 60 % its shorter letter tokens,
    25 % random letter strings of 1..10.  Keyed by (seed, global index).
    Returns (text u8, offsets u64[n+1], cut mask u8: bit 1 atom start, bit 0 word start)."""
    longs, shorts = bloom_word_pool(vocab_or_pool) if isinstance(vocab_or_pool, dict) else vocab_or_pool
    parts: List[bytes] = []
    cuts: List[bytes] = []
    sp = BYTE_SPACE.encode("utf-8")
    for g in range(start, start + n):
        # counter word 1 = the string: streams never overlap (word 0 advances within a string)
        rng = np.random.Generator(np.random.Philox(key=np.uint64(seed), counter=np.array([0, g, 0, 0], dtype=np.uint64)))
        r = rng.random(size=64)
        pick = rng.integers(0, 1 << 62, size=64)
        rl = rng.integers(1, 11, size=64)
        lt = rng.integers(0, 26, size=(64, 10))
        buf, cut = bytearray(), bytearray()
        for k in range(64):
            if r[k] < 0.15:
                w = longs[int(pick[k]) % len(longs)]
            elif r[k] < 0.75:
                w = shorts[int(pick[k]) % len(shorts)]
            else:
                w = "".join(LETTERS[c] for c in lt[k, :rl[k]])
            wb = w.encode("ascii")
            pre = sp if buf else b""
            room = length - len(buf) - len(pre)
            if room <= 0:
                break
            wb = wb[:room]
            cut += b"\x03" + b"\x00" * (len(pre) - 1) + b"\x02" * len(wb) if pre else b"\x03" + b"\x02" * (len(wb) - 1)
            buf += pre + wb
        parts.append(bytes(buf))
        cuts.append(bytes(cut))
    text, offs = _pack(parts)
    return text, offs, np.frombuffer(b"".join(cuts), dtype=np.uint8).copy()


def _bloom_chunk(args):
    n, start, pool, kw = args
    return bloom_like_corpus(n, pool, start=start, **kw)


def bloom_like_parallel(n: int, vocab: Dict[str, int], start: int = 0, procs: int = 8,
                        **kw) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """``bloom_like_corpus`` over [start, start+n) in ``procs`` forked processes (identical
    output).  Call before any GPU work (fork)."""
    import multiprocessing as mp
    pool = bloom_word_pool(vocab)
    if procs <= 1 or n < 4096:
        return bloom_like_corpus(n, pool, start=start, **kw)
    step = (n + procs - 1) // procs
    jobs = [(min(step, n - s), start + s, pool, kw) for s in range(0, n, step)]
    with mp.get_context("fork").Pool(len(jobs)) as p:
        res = p.map(_bloom_chunk, jobs)
        p.close()
        p.join()
    lens = np.concatenate([np.diff(o) for _, o, _ in res])
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens, dtype=np.uint64)
    return np.concatenate([t for t, _, _ in res]), offs, np.concatenate([c for _, _, c in res])
