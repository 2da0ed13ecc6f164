"""dptok -- MI355X-native shortest-tokenization engine (HIP kernels behind a ctypes C-ABI).

Public surface:
    Vocab, Encoder          batch engine (engine.py)
    dp_tokenize_batch       List[str] -> List[List[int]] for a t2i vocabulary
    synth                   synthetic vocabularies/corpora of the BASELINE configs
The reference-compatible names (dp_tokenize_llama, compute_shortest_tokenizations, ...)
live in the sibling ``packages`` / ``inspect_tokenizer`` modules of this directory.
"""
from ._lib import DptError, STATUS_EMPTY_WORD, STATUS_INTERNAL, STATUS_NO_TOKENIZATION, STATUS_OK, STATUS_TOO_LONG
from .engine import Encoder, Vocab, pack_strings, raise_for_status

__all__ = ["Vocab", "Encoder", "DptError", "pack_strings", "raise_for_status", "dp_tokenize_batch",
           "STATUS_OK", "STATUS_NO_TOKENIZATION", "STATUS_EMPTY_WORD", "STATUS_TOO_LONG", "STATUS_INTERNAL"]


_BATCH_CACHE = {}


def _encoder_for(t2i, device: int) -> Encoder:
    """One Encoder per (vocabulary object, size, device): the trie is built and uploaded once,
    not per call.  The cache holds the dict itself, so its id() cannot be reused while cached."""
    key = (id(t2i), len(t2i), device)
    hit = _BATCH_CACHE.get(key)
    if hit is None or hit[0] is not t2i:
        if len(_BATCH_CACHE) >= 4:
            _BATCH_CACHE.pop(next(iter(_BATCH_CACHE)))
        hit = (t2i, Encoder(Vocab(t2i, device)))
        _BATCH_CACHE[key] = hit
    return hit[1]


def dp_tokenize_batch(texts, t2i, device: int = 0, raise_errors: bool = True):
    """Tokenize many strings at once (raw pre-tokenization); the batched form of
    the reference's ``dp_tokenize`` closure (packages/tokenizer_utils.py:66-80).
    The vocabulary is uploaded once per ``t2i`` object (keyed by identity and size: a dict that
    is mutated in place without changing its size is not re-read)."""
    enc = _encoder_for(t2i, device)
    out = []
    for t, (ids, st) in zip(texts, enc.encode_strs(texts)):
        if raise_errors:
            raise_for_status(st, t)
        out.append(ids)
    return out
