"""Host side of the engine: vocabulary upload, batch encode, status -> exception.

This mirrors the reference's L2 adapter (packages/tokenizer_utils.py:52-96) one
level down: a ``Vocab`` is the captured ``t2i``/``vocab`` of ``dp_tokenize_llama``
(:53-57), an ``Encoder`` runs the per-word DP loop of the ``dp_tokenize`` closure
(:66-80) for a whole batch on the GPU.
"""
from __future__ import annotations

import ctypes
import gc
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

try:   # built with libdpt.so (csrc/Makefile); the pure-Python conversion below gives the same lists
    from . import _pylists
except ImportError:   # pragma: no cover
    _pylists = None


def csr_lists(ids: np.ndarray, id_off: np.ndarray, status: np.ndarray, none: Optional[np.ndarray] = None,
              keep_failed: bool = True) -> List[Tuple[List[int], int]]:
    """CSR ids -> per string (List[int], status): ([], OK) where ``none``; the string's ids where its
    status is OK or ``keep_failed``; else ([], status).  One C pass (``_pylists``: cached int objects,
    no intermediate flat list) -- the host path's conversion was ~20x its GPU call."""
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    id_off = np.ascontiguousarray(id_off, dtype=np.uint64)
    status = np.ascontiguousarray(status, dtype=np.int32)
    if none is not None:
        none = np.ascontiguousarray(none, dtype=np.uint8)
    if _pylists is not None:
        # (the cyclic GC off while thousands of new lists appear: each gen-0 pass would re-scan them;
        # lists of ints hold no cycles, and the next collection sees them once)
        was = gc.isenabled()
        gc.disable()
        try:
            return _pylists.csr_lists(ids, id_off, status, none, _lib.STATUS_OK, 1 if keep_failed else 0)
        finally:
            if was:
                gc.enable()
    flat, o, sl = ids.tolist(), [int(x) - int(id_off[0]) for x in id_off.tolist()], status.tolist()
    nn = none.tolist() if none is not None else [0] * len(sl)
    return [([], _lib.STATUS_OK) if nn[i] else
            ((flat[o[i]:o[i + 1]] if (keep_failed or sl[i] == _lib.STATUS_OK) else []), sl[i])
            for i in range(len(sl))]
from ._lib import (DPT_FLAG_LEN_ONLY, DPT_FLAG_UNCAPPED, DPT_MODE_ATOMS, DPT_MODE_PRESPLIT, DPT_MODE_RAW, DptError,
                   check)

MODES = {"raw": DPT_MODE_RAW, "presplit": DPT_MODE_PRESPLIT, "atoms": DPT_MODE_ATOMS, DPT_MODE_RAW: DPT_MODE_RAW,
         DPT_MODE_PRESPLIT: DPT_MODE_PRESPLIT, DPT_MODE_ATOMS: DPT_MODE_ATOMS}


def atoms_to_csr(atom_lists: Sequence[Sequence[str]]):
    """Lists of atom strings -> (text, offsets, cut mask) for DPT_MODE_ATOMS (one word per list:
    bit 1 marks every atom start, bit 0 the first).  Empty atoms are not representable."""
    parts, cuts = [], []
    for atoms in atom_lists:
        for k, a in enumerate(atoms):
            e = encode_utf8(a)
            if not e:
                raise ValueError("empty atom")
            parts.append(e)
            c = bytearray(len(e))
            c[0] = 3 if k == 0 else 2
            cuts.append(bytes(c))
    lens = [sum(len(encode_utf8(a)) for a in atoms) for atoms in atom_lists]
    offs = np.zeros(len(atom_lists) + 1, dtype=np.uint64)
    if lens:
        offs[1:] = np.cumsum(lens, dtype=np.uint64)
    text = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8)
    cut = np.frombuffer(b"".join(cuts) + b"\0", dtype=np.uint8)
    return text, offs, cut


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def encode_utf8(s: str) -> bytes:
    return s.encode("utf-8", "surrogatepass")


def pack_strings(texts: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    enc = [encode_utf8(t) for t in texts]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    if enc:
        offs[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
    text = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
    return text, offs


def raise_for_status(status: int, text: str = "") -> None:
    """Re-raise the reference's exception for a per-string status."""
    if status == _lib.STATUS_OK:
        return
    if status == _lib.STATUS_NO_TOKENIZATION:
        # reference: ipdb.set_trace() then obtain_longest_token([]) -> max([]) (dp_tokenize.py:84)
        raise ValueError("max() arg is an empty sequence (no tokenization of a word of %r)" % text[:60])
    if status == _lib.STATUS_EMPTY_WORD:
        # reference: segment_index_dp[-1] on an empty word (dp_tokenize.py:49)
        raise IndexError("list index out of range (empty word)")
    if status == _lib.STATUS_TOO_LONG:
        raise DptError("input outside the engine's limits (status 3)")
    raise DptError("engine internal error (status %d)" % status)


class Vocab:
    """Device-resident vocabulary (double-array byte trie) built from ``t2i``."""

    def __init__(self, t2i: Dict[str, int], device: int = 0):
        L = _lib.lib()
        toks = list(t2i.keys())
        enc = [encode_utf8(t) for t in toks]
        off = np.zeros(len(enc) + 1, dtype=np.uint64)
        if enc:
            off[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
        blob = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
        ids = np.array([t2i[t] for t in toks], dtype=np.int32)
        h = ctypes.c_void_p()
        check(L.dpt_vocab_create(_ptr(blob), _ptr(off), _ptr(ids), len(toks), device, ctypes.byref(h)), "dpt_vocab_create")
        self.handle = h
        self.device = device
        self.t2i = t2i
        st = _lib.VocabStats()
        check(L.dpt_vocab_stats_get(self.handle, ctypes.byref(st)), "dpt_vocab_stats_get")
        self.stats = {f: getattr(st, f) for f, _ in st._fields_}

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib._lib is not None:
            _lib._lib.dpt_vocab_destroy(h)
            self.handle = None


def pack_word_atoms(strings: Sequence[Sequence[Sequence[str]]]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Strings given as words of atoms -> DPT_MODE_ATOMS buffers (text u8, offsets u64[n+1], cut
    mask u8: bit 1 at every atom's first byte, bit 0 at every word's).  Raises ValueError for an
    empty atom or an empty word."""
    parts, cuts, offs = [], [], [0]
    for words in strings:
        n = 0
        for atoms in words:
            for k, a in enumerate(atoms):
                e = encode_utf8(a)
                if not e:
                    raise ValueError("empty atom")
                c = bytearray(len(e))
                c[0] = 3 if k == 0 else 2          # bit 1: atom start, bit 0: word start
                parts.append(e)
                cuts.append(bytes(c))
                n += len(e)
            if not atoms:
                raise ValueError("empty word")
        offs.append(offs[-1] + n)
    text = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8)
    cut = np.frombuffer(b"".join(cuts) + b"\0", dtype=np.uint8)
    return text, np.array(offs, dtype=np.uint64), cut


def pack_presplit_words(strings: Sequence[Sequence[str]]):
    """Strings given as lists of words -> DPT_MODE_PRESPLIT buffers (text u8, offsets u64[n+1], cut
    mask u8 = 1 at every word's first byte) + per string its word count and the index of its first
    empty word (-1: none; the string is cut there, see ``Encoder.encode_presplit``)."""
    enc_words, n_words, cut_at = [], [], []
    for words in strings:
        k = next((i for i, w in enumerate(words) if not w), -1)
        ws = words if k < 0 else words[:k]
        enc_words.extend(encode_utf8(w) for w in ws)
        n_words.append(len(ws))
        cut_at.append(k)
    wl = np.fromiter((len(e) for e in enc_words), dtype=np.uint64, count=len(enc_words))
    wend = np.concatenate([np.zeros(1, np.uint64), np.cumsum(wl, dtype=np.uint64)])   # bytes of the first k words
    offs = np.concatenate([np.zeros(1, np.uint64), wend[np.cumsum(np.asarray(n_words, dtype=np.int64))]]) \
        if len(strings) else np.zeros(1, np.uint64)
    raw = b"".join(enc_words)
    cut = np.zeros(len(raw) + 1, dtype=np.uint8)
    if len(wl):
        cut[wend[:-1].astype(np.int64)] = 1   # every word's first byte
    text = np.frombuffer(raw + b"\0", dtype=np.uint8)
    return text, offs, cut, n_words, cut_at


_WS_BYTES = "\u2581".encode("utf-8")


class PieceTable:
    """Per vocabulary id: the piece's UTF-8 bytes and whether it starts with '\u2581' -- llama mode's
    host pre-tokenization (reference packages/tokenizer_utils.py:24-31: ids -> pieces through the
    inverted vocabulary, then ``merge_tokens(sep='\u2581')`` :7-22) as array gathers over a whole
    batch.  merge_tokens starts a word at the first piece and at every piece that starts with the
    separator and appends every other piece to the current word, so a string's pre-split text is
    the concatenation of its pieces' bytes, with a word start at the first piece and at each '\u2581'
    piece -- the bytes and cut mask ``Encoder.encode_presplit`` builds from the merged words."""

    def __init__(self, t2i: Dict[str, int]):
        ids = np.fromiter(t2i.values(), dtype=np.int64, count=len(t2i))
        n = int(ids.max()) + 1 if len(ids) else 0
        # a dense table only (ids of get_vocab() are 0..|V|-1); negative or very sparse ids: unusable
        self.ok = len(ids) > 0 and int(ids.min()) >= 0 and n <= 4 * len(ids) + 1024
        if not self.ok:
            return
        inv = {}
        for tok, i in t2i.items():   # the last token of a duplicated id wins, like {v: k for k, v in items}
            inv[i] = tok
        enc = [encode_utf8(inv[i]) if i in inv else b"" for i in range(n)]
        self.present = np.zeros(n, dtype=bool)
        self.present[list(inv.keys())] = True
        self.plen = np.fromiter((len(e) for e in enc), dtype=np.int64, count=n)
        self.poff = np.zeros(n, dtype=np.int64)
        if n > 1:
            self.poff[1:] = np.cumsum(self.plen[:-1])
        self.blob = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
        self.ws = np.fromiter((e.startswith(_WS_BYTES) for e in enc), dtype=bool, count=n)
        # merge_tokens of a list with an empty piece can yield an empty word (IndexError in the
        # reference's DP): such a vocabulary takes the word-list path
        self.empty_piece = bool((self.plen[self.present] == 0).any())

    def pack(self, id_lists: Sequence[Sequence[int]]):
        """Token ids per string -> (text u8, offsets u64[n+1], cut mask u8, pieces per string) for
        DPT_MODE_PRESPLIT.  KeyError for an id outside the vocabulary (the reference's
        ``vocab_bidict.inverse[token]``)."""
        import itertools
        n_str = len(id_lists)
        cnt = np.fromiter((len(x) for x in id_lists), dtype=np.int64, count=n_str)
        total = int(cnt.sum())
        flat = np.fromiter(itertools.chain.from_iterable(id_lists), dtype=np.int64, count=total)
        if total:
            bad = (flat < 0) | (flat >= len(self.present))
            bad[~bad] = ~self.present[flat[~bad]]
            if bad.any():
                raise KeyError(int(flat[np.argmax(bad)]))
        plen = self.plen[flat]
        pend = np.cumsum(plen)
        pstart = pend - plen
        nb = int(pend[-1]) if total else 0
        # byte k of the batch comes from blob[poff[id] + (k - pstart)]
        src = np.repeat(self.poff[flat] - pstart, plen) + np.arange(nb, dtype=np.int64)
        text = np.empty(nb + 1, dtype=np.uint8)
        text[:nb] = self.blob[src]
        text[nb] = 0
        first = np.zeros(total, dtype=bool)
        send = np.cumsum(cnt)
        first[(send - cnt)[cnt > 0]] = True   # every string's first piece opens its first word
        cut = np.zeros(nb + 1, dtype=np.uint8)
        cut[pstart[first | self.ws[flat]]] = 1
        offs = np.zeros(n_str + 1, dtype=np.uint64)
        if n_str:
            offs[1:] = np.concatenate([[0], pend])[send]
        return text, offs, cut, cnt


class Encoder:
    """Batch shortest-tokenization on one GPU (one workspace; use from one stream at a time)."""

    def __init__(self, vocab: Vocab):
        L = _lib.lib()
        self.vocab = vocab
        h = ctypes.c_void_p()
        check(L.dpt_ctx_create(vocab.device, ctypes.byref(h)), "dpt_ctx_create")
        self.handle = h

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib._lib is not None:
            _lib._lib.dpt_ctx_destroy(h)
            self.handle = None

    # ---------------------------------------------------------------- host buffers
    def encode_csr(self, text: np.ndarray, offs: np.ndarray, mode="raw", cut_mask: Optional[np.ndarray] = None):
        """CSR host arrays in -> (ids int32[], id_off u64[n+1], status int32[n], capped int32[n])."""
        text = np.ascontiguousarray(text, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        n = len(offs) - 1
        n_bytes = int(offs[-1] - offs[0]) if n >= 0 else 0
        ids = np.empty(max(n_bytes, 1), dtype=np.int32)
        id_off = np.empty(n + 1, dtype=np.uint64)
        status = np.empty(max(n, 1), dtype=np.int32)
        capped = np.empty(max(n, 1), dtype=np.int32)
        m = MODES[mode]
        if m != DPT_MODE_RAW:
            if cut_mask is None:
                raise ValueError("presplit/atoms mode needs cut_mask")
            cut_mask = np.ascontiguousarray(cut_mask, dtype=np.uint8)
        base = int(offs[0])
        tv = text[base:] if base else text
        check(_lib.lib().dpt_encode_host(self.handle, self.vocab.handle, m, _ptr(tv), n_bytes, _ptr(offs),
                                         _ptr(cut_mask[base:] if cut_mask is not None else None), n, _ptr(ids),
                                         max(n_bytes, 1), _ptr(id_off), _ptr(status), _ptr(capped)), "dpt_encode_host")
        return ids[: int(id_off[-1])], id_off, status[:n], capped[:n]

    def encode_one(self, s: str) -> Tuple[List[int], int]:
        """One raw-mode string -> (ids, status): the drop-in's per-string call (reference main_analyze_s2orc.py:74-78)
        with as little host work as a ctypes call allows -- the UTF-8 bytes passed as they are, the offsets,
        outputs and their pointers kept from the previous call (dpt_encode_host runs it as one zero-copy launch)."""
        b = s.encode("utf-8", "surrogatepass")
        n = len(b)
        one = self.__dict__.get("_one")
        if one is None or one[0] < n + 1:
            cap = max(4096, 2 * n + 2)
            ids = np.empty(cap, dtype=np.int32)
            off = np.zeros(4, dtype=np.uint64)   # [0:2] the string's offsets (in), [2:4] id_off (out)
            st = np.empty(2, dtype=np.int32)
            L = _lib.lib()
            fn = ctypes.cast(L.dpt_encode_host, ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                                 ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p,
                                                                 ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                                 ctypes.c_void_p))
            one = self._one = (cap, ids, off, st, fn, off.ctypes.data, ids.ctypes.data, st.ctypes.data,
                               st.ctypes.data + 4, off.ctypes.data + 16)
        cap, ids, off, st, fn, p_off, p_ids, p_st, p_cap, p_idoff = one
        off[1] = n
        rc = fn(self.handle, self.vocab.handle, DPT_MODE_RAW, b, n, p_off, None, 1, p_ids, max(n, 1), p_idoff, p_st, p_cap)
        if rc != _lib.DPT_OK:
            check(rc, "dpt_encode_host")
        return ids[:int(off[3])].tolist(), int(st[0])

    def encode_strs(self, texts: Sequence[str]) -> List[Tuple[List[int], int]]:
        text, offs = pack_strings(texts)
        ids, id_off, st, _ = self.encode_csr(text, offs)
        return csr_lists(ids, id_off, st)

    def encode_presplit(self, strings: Sequence[Sequence[str]]) -> List[Tuple[List[int], int]]:
        """Many strings, each pre-split into words (llama mode, DPT_MODE_PRESPLIT), in ONE launch:
        per string (ids, status).  Words are processed in order like the reference's loop
        (tokenizer_utils.py:70-75): an empty word raises IndexError there (dp_tokenize.py:49)
        unless an earlier word already failed (no tokenization -> ValueError), so a string is cut
        at its first empty word and that word's status is decided by the prefix before it."""
        text, offs, cut, n_words, cut_at = pack_presplit_words(strings)
        n_str = len(strings)
        ids, id_off, st, _ = self.encode_csr(text, offs, mode="presplit", cut_mask=cut)
        flat = ids.tolist()
        o = id_off.tolist()
        out = []
        for i in range(n_str):
            s = int(st[i])
            if cut_at[i] < 0 and n_words[i] == 0:
                out.append(([], _lib.STATUS_OK))           # no words: the reference's loop emits nothing
            elif cut_at[i] >= 0 and s in (_lib.STATUS_OK, _lib.STATUS_EMPTY_WORD):
                out.append(([], _lib.STATUS_EMPTY_WORD))   # the prefix tokenized (or was empty): IndexError
            else:
                out.append((flat[o[i]:o[i + 1]] if s == _lib.STATUS_OK else [], s))
        return out

    def encode_packed_presplit(self, text: np.ndarray, offs: np.ndarray, cut: np.ndarray,
                               n_pieces: np.ndarray) -> List[Tuple[List[int], int]]:
        """``PieceTable.pack`` output in ONE launch: per string (ids, status); a string of no pieces
        has no words (the reference's loop emits nothing, status 0).  Pieces are never empty here,
        so no word is."""
        ids, id_off, st, _ = self.encode_csr(text, offs, mode="presplit", cut_mask=cut)
        return csr_lists(ids, id_off, st, none=(np.asarray(n_pieces) == 0), keep_failed=False)

    def encode_words(self, words: Sequence[str]) -> Tuple[List[int], int]:
        """One string pre-split into words (llama mode, DPT_MODE_PRESPLIT): ids and status."""
        return self.encode_presplit([words])[0]

    def encode_word_atoms(self, strings: Sequence[Sequence[Sequence[str]]]) -> List[Tuple[List[int], int]]:
        """Strings given as words of atoms (DPT_MODE_ATOMS), one launch for the batch: per string
        (ids, status).  A string with no words gives ([], ok) -- the BLOOM adapter's empty input
        (reference tokenizer_utils.py:166-178 loops over zero words)."""
        text, o, cut = pack_word_atoms(strings)
        ids, id_off, st, _ = self.encode_csr(text, o, mode="atoms", cut_mask=cut)
        out = []
        for i, words in enumerate(strings):
            if not words:
                out.append(([], _lib.STATUS_OK))
            else:
                out.append((ids[int(id_off[i]):int(id_off[i + 1])].tolist(), int(st[i])))
        return out

    def dp(self, text: np.ndarray, offs: np.ndarray, mode="atoms", cut_mask: Optional[np.ndarray] = None,
           uncapped: bool = False, edges: bool = False, far: bool = False):
        """DP by-products without ids (dpt_dp_host): (status, lengths, edges or None), and with ``far``
        (edges only) a 4th value: the (edges index, back distance) pairs of optimal predecessors more
        than 64 atoms back (dpt_dp_host_far), an int array of shape (k, 2).  lengths are the capped
        len_dp[-1] sums (reference dp_tokenize.py:70) or, with ``uncapped``, the minimum token counts
        (65535 per impossible word, inspect_tokenizer.py:77-86)."""
        text = np.ascontiguousarray(text, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        if len(offs) and int(offs[0]) != 0:
            raise ValueError("dp(): offsets must start at 0")
        n = len(offs) - 1
        n_bytes = int(offs[-1] - offs[0])
        status = np.empty(max(n, 1), dtype=np.int32)
        lengths = np.empty(max(n, 1), dtype=np.int32)
        ed = np.zeros(max(n_bytes, 1), dtype=np.uint64) if (edges or far) else None
        m = MODES[mode] | (DPT_FLAG_UNCAPPED if uncapped else DPT_FLAG_LEN_ONLY)
        if cut_mask is not None:
            cut_mask = np.ascontiguousarray(cut_mask, dtype=np.uint8)
        L = _lib.lib()
        if not far:
            check(L.dpt_dp_host(self.handle, self.vocab.handle, m, _ptr(text), n_bytes, _ptr(offs), _ptr(cut_mask),
                                n, _ptr(status), _ptr(lengths), _ptr(ed)), "dpt_dp_host")
            return status[:n], lengths[:n], ed
        cap = 1024
        while True:
            fp = np.zeros((cap, 2), dtype=np.uint64)
            nf = ctypes.c_uint64(0)
            rc = L.dpt_dp_host_far(self.handle, self.vocab.handle, m, _ptr(text), n_bytes, _ptr(offs), _ptr(cut_mask),
                                   n, _ptr(status), _ptr(lengths), _ptr(ed), _ptr(fp), cap, ctypes.byref(nf))
            if rc == _lib.DPT_E_CAP and nf.value > cap:
                cap = int(nf.value)   # the DP runs again with room for every pair
                continue
            check(rc, "dpt_dp_host_far")
            return status[:n], lengths[:n], ed, fp[: nf.value].astype(np.int64)

    # ---------------------------------------------------------------- device buffers
    def encode_device(self, text_ptr: int, n_bytes: int, off_ptr: int, n_str: int, ids_ptr: int, ids_cap: int,
                      idoff_ptr: int, status_ptr: int, capped_ptr: int = 0, cut_ptr: int = 0, stream: int = 0,
                      mode="raw") -> None:
        """All pointers are device addresses (e.g. ``torch.Tensor.data_ptr()``); stream-ordered, no sync."""
        check(_lib.lib().dpt_encode(self.handle, self.vocab.handle, MODES[mode], ctypes.c_void_p(text_ptr), n_bytes,
                                    ctypes.c_void_p(off_ptr), ctypes.c_void_p(cut_ptr or None), n_str,
                                    ctypes.c_void_p(ids_ptr), ids_cap, ctypes.c_void_p(idoff_ptr),
                                    ctypes.c_void_p(status_ptr), ctypes.c_void_p(capped_ptr or None),
                                    ctypes.c_void_p(stream or None)), "dpt_encode")

    def encode_device_padded(self, text_ptr: int, n_bytes: int, off_ptr: int, n_str: int, ids_ptr: int, ids_cap: int,
                             counts_ptr: int, status_ptr: int, capped_ptr: int = 0, cut_ptr: int = 0, stream: int = 0,
                             mode="raw") -> None:
        """dpt_encode_padded: string s's ids stay at its byte offset, ids[str_off[s]-str_off[0] + k] for
        k < counts[s] (uint64); no CSR packing pass.  Device addresses, stream-ordered, no sync."""
        check(_lib.lib().dpt_encode_padded(self.handle, self.vocab.handle, MODES[mode], ctypes.c_void_p(text_ptr), n_bytes,
                                           ctypes.c_void_p(off_ptr), ctypes.c_void_p(cut_ptr or None), n_str,
                                           ctypes.c_void_p(ids_ptr), ids_cap, ctypes.c_void_p(counts_ptr),
                                           ctypes.c_void_p(status_ptr), ctypes.c_void_p(capped_ptr or None),
                                           ctypes.c_void_p(stream or None)), "dpt_encode_padded")

    def reserve(self, n_bytes: int, n_str: int, long_bytes: int = 0) -> None:
        """Pre-size the workspace for this vocabulary's staging width (a later call of that size is
        capture-safe); ``long_bytes``: input bytes the unbounded pass holds per call (0: default)."""
        check(_lib.lib().dpt_ctx_reserve_vocab(self.handle, self.vocab.handle, n_bytes, n_str, long_bytes),
              "dpt_ctx_reserve_vocab")

    def workspace_bytes(self) -> Tuple[int, int]:
        """(device-path workspace, host-path staging) bytes held on the device."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().dpt_ctx_workspace_bytes(self.handle, ctypes.byref(a), ctypes.byref(b)), "dpt_ctx_workspace_bytes")
        return a.value, b.value

    def long_need(self) -> Tuple[int, int]:
        """(input bytes the last call's unbounded pass took, its arena capacity); call after the
        encode's stream has completed."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().dpt_ctx_long_need(self.handle, ctypes.byref(a), ctypes.byref(b)), "dpt_ctx_long_need")
        return a.value, b.value

    def set_histogram(self, hist_ptr: int, n_bins: int, overwrite: bool = False) -> None:
        """Fold the token-count histogram into the next encode on this engine (dpt_ctx_set_histogram_ex:
        its finish pass adds to hist, device int64[n_bins + 8], or with ``overwrite`` replaces it -- the
        device zeroes it first, in stream order); 0 cancels."""
        check(_lib.lib().dpt_ctx_set_histogram_ex(self.handle, ctypes.c_void_p(hist_ptr) if hist_ptr else None, n_bins,
                                                  1 if overwrite else 0), "dpt_ctx_set_histogram_ex")

    def histogram_device(self, idoff_ptr: int, status_ptr: int, n_str: int, hist_ptr: int, n_bins: int,
                         stream: int = 0) -> None:
        check(_lib.lib().dpt_token_histogram(ctypes.c_void_p(idoff_ptr), ctypes.c_void_p(status_ptr), n_str,
                                             ctypes.c_void_p(hist_ptr), n_bins, ctypes.c_void_p(stream or None)),
              "dpt_token_histogram")

    def debug_counter_bias(self, bias: int) -> None:
        """TEST-ONLY (dpt_ctx_debug_counter_bias): later calls start the unbounded pass's arena and far-pair
        counters at ``bias`` (results unchanged; its kernels' offsets become >= bias)."""
        check(_lib.lib().dpt_ctx_debug_counter_bias(self.handle, bias), "dpt_ctx_debug_counter_bias")

    def profile(self, on: bool = True) -> None:
        check(_lib.lib().dpt_ctx_profile(self.handle, 1 if on else 0), "dpt_ctx_profile")

    def profile_read(self) -> Tuple[List[float], int]:
        ms = (ctypes.c_double * 3)()
        n = ctypes.c_uint64()
        check(_lib.lib().dpt_ctx_profile_read(self.handle, ms, ctypes.byref(n)), "dpt_ctx_profile_read")
        return [ms[0], ms[1], ms[2]], n.value
