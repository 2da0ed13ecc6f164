"""Drop-in for the reference's ``packages/tokenizer_utils.py`` (L2 adapters) backed by the
MI355X engine.  Same names, argument meaning and error behaviour:

* ``dp_tokenize_llama(llama_tokenizer, pretokenize_option='llama')`` -> ``(dp_tokenize,
  decode_dp_tokenization)`` (reference :52-96).  ``dp_tokenize(str) -> List[int]`` runs the
  per-word shortest-tokenization DP + longest-token selection on the GPU:
  - ``'raw'``: the pre-tokenizer runs inside the kernel (pretokenize_raw semantics, :33-50);
  - ``'llama'``: SentencePiece pieces from ``llama_tokenizer.encode`` are merged into words on
    the host (pretokenize_with_llama + merge_tokens, :7-31) and the GPU runs in pre-split mode.
  The DP call is the evident-intent 4-argument call; the shipped 5-argument call at :71 raises
  TypeError (SURVEY.md §0 finding 3), which this drop-in does not reproduce.
  Failures re-raise the reference's exceptions: a word with no tokenization -> ValueError
  (reference: ipdb.set_trace then max([]) at dp_tokenize.py:84), an empty word -> IndexError
  (dp_tokenize.py:49).  An unknown ``pretokenize_option`` fails at call time with NameError,
  like the reference's unbound ``pretokenize_func``.
* ``dp_tokenize.batch(List[str]) -> List[List[int]]``: the batched form (one GPU launch, in both
  modes).
* ``merge_tokens``, ``pretokenize_with_llama``, ``pretokenize_raw``: the reference's host-side
  string utilities with identical behaviour (pre-tokenization, not the DP).
"""
from __future__ import annotations

import os
import sys
from typing import Dict, List, Sequence

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from dptok import Encoder, Vocab, raise_for_status  # noqa: E402
from dptok.engine import PieceTable  # noqa: E402
from dptok.hostpool import shared_pool  # noqa: E402

SPACE_TOKEN = "▁"


class _InverseDict(dict):
    """Minimal stand-in for ``bidict`` (reference uses ``.inverse``)."""

    @property
    def inverse(self):
        return {v: k for k, v in self.items()}


def merge_tokens(tokens, sep="Ġ"):
    """Join runs of pieces that do not start with ``sep`` (reference tokenizer_utils.py:7-22)."""
    merged_tokens = []
    i = 0
    n = len(tokens)
    while i < n:
        cur = tokens[i]
        while i + 1 < n and not tokens[i + 1].startswith(sep):
            cur = cur + tokens[i + 1]
            i += 1
        merged_tokens.append(cur)
        i += 1
    return merged_tokens


def pretokenize_with_llama(tokenizer, vocab_bidict):
    """SentencePiece pieces merged into words (reference tokenizer_utils.py:24-31)."""
    inverse = vocab_bidict.inverse

    def pretokenize(input_str):
        pieces = [inverse[t] for t in tokenizer.encode(input_str)]
        return merge_tokens(pieces, sep=SPACE_TOKEN)

    return pretokenize


def pretokenize_raw(manual_mapping) -> callable:
    """Raw character pre-tokenizer (reference tokenizer_utils.py:33-50): first char gets the
    '▁' prefix, ' ' opens a word as '▁', characters in ``manual_mapping.inverse`` are replaced
    (``'\\n' -> '<0x0A>'``).  The GPU engine applies the same rules in-kernel."""
    inverse = manual_mapping.inverse

    def pretokenize(input_str):
        atoms = list(input_str)
        words = []
        start = 0
        for i, ch in enumerate(atoms):
            if i == 0:
                atoms[i] = SPACE_TOKEN + ch
            elif ch == " ":
                atoms[i] = SPACE_TOKEN
                words.append(atoms[start:i])
                start = i
            elif ch in inverse:
                atoms[i] = inverse[ch]
        words.append(atoms[start:])
        return words

    return pretokenize


def _device() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def batch_encoder(tokenizer):
    """``texts -> [tokenizer.encode(t) for t in texts]``, in one call of the Rust backend when the
    tokenizer is a ``transformers`` tokenizers-backed class whose ``encode`` is the library's own:
    that ``encode`` is ``_encode_plus`` over a one-text batch -- ``set_truncation_and_padding`` with
    the default strategies, ``encode_special_tokens = split_special_tokens``, then
    ``_tokenizer.encode_batch([text], add_special_tokens=True)`` -- so one ``encode_batch_fast``
    over every text returns the same ids per text (tests/test_llama_sp.py checks it on every
    fixture), with the backend's threads.  Any other tokenizer object: its ``encode``, per text."""
    try:
        from transformers.tokenization_utils_base import PreTrainedTokenizerBase
        from transformers.tokenization_utils_tokenizers import TokenizersBackend
        from transformers.utils import PaddingStrategy
        from transformers.tokenization_utils_base import TruncationStrategy
    except ImportError:
        TokenizersBackend = None
    if (TokenizersBackend is not None and isinstance(tokenizer, TokenizersBackend)
            and type(tokenizer).encode is PreTrainedTokenizerBase.encode
            and type(tokenizer)._encode_plus is TokenizersBackend._encode_plus
            and hasattr(tokenizer._tokenizer, "encode_batch_fast")):
        fast = [True]   # (the private calls below are pinned on transformers 5.x; any other signature: per text)

        def encode_batch(texts):
            if fast[0]:
                try:
                    pad, trunc, max_len, _ = tokenizer._get_padding_truncation_strategies(padding=False, truncation=None,
                                                                                          max_length=None)
                    if pad == PaddingStrategy.DO_NOT_PAD and trunc == TruncationStrategy.DO_NOT_TRUNCATE:
                        tokenizer.set_truncation_and_padding(padding_strategy=pad, truncation_strategy=trunc,
                                                             max_length=max_len, stride=0, pad_to_multiple_of=None,
                                                             padding_side=None)
                        if tokenizer._tokenizer.encode_special_tokens != tokenizer.split_special_tokens:
                            tokenizer._tokenizer.encode_special_tokens = tokenizer.split_special_tokens
                        return [e.ids for e in tokenizer._tokenizer.encode_batch_fast(list(texts), add_special_tokens=True)]
                except (TypeError, AttributeError):
                    fast[0] = False   # from now on the library's public encode, per text
            return [tokenizer.encode(t) for t in texts]
        return encode_batch
    return lambda texts: [tokenizer.encode(t) for t in texts]


def dp_tokenize_llama(llama_tokenizer, pretokenize_option="llama"):
    t2i: Dict[str, int] = dict(llama_tokenizer.get_vocab())
    vocab_bidict = _InverseDict(t2i)
    engine = Encoder(Vocab(t2i, _device()))
    manual_mapping = _InverseDict({"<0x0A>": "\n"})
    if manual_mapping.inverse != {"\n": "<0x0A>"}:  # the raw kernel hard-codes this mapping
        raise AssertionError("unexpected manual mapping")

    if pretokenize_option == "raw":
        def encode_many(texts: Sequence[str]) -> List[List[int]]:
            out = []
            for t, (ids, st) in zip(texts, engine.encode_strs(list(texts))):
                raise_for_status(st, t)
                out.append(ids)
            return out
    elif pretokenize_option == "llama":
        pretokenize = pretokenize_with_llama(llama_tokenizer, vocab_bidict)
        pieces = PieceTable(t2i)
        encode_ids = batch_encoder(llama_tokenizer)
        host = shared_pool(llama_tokenizer, pieces, encode_ids)   # worker processes for large batches (one per tokenizer)

        def encode_many(texts: Sequence[str]) -> List[List[int]]:
            # SentencePiece runs on the host (third-party); the pieces -> words merge is array
            # gathers over the whole batch (PieceTable), and the DP of every word of every text is
            # ONE pre-split launch
            texts = list(texts)
            if pieces.ok and not pieces.empty_piece:
                res = engine.encode_packed_presplit(*host.pack(texts))
            else:
                res = engine.encode_presplit([pretokenize(t) for t in texts])
            out = []
            for t, (ids, st) in zip(texts, res):
                raise_for_status(st, t)
                out.append(ids)
            return out
    else:
        def encode_many(texts):
            raise NameError("name 'pretokenize_func' is not defined")

    if pretokenize_option == "raw":
        def dp_tokenize(input_str) -> List[int]:
            ids, st = engine.encode_one(input_str)   # (the per-string call: one zero-copy launch)
            raise_for_status(st, input_str)
            return ids
    else:
        def dp_tokenize(input_str) -> List[int]:
            return encode_many([input_str])[0]

    def decode_dp_tokenization(encoding: List[int]):
        # reference tokenizer_utils.py:82-84: drop the 4-character "<s> " prefix
        return llama_tokenizer.decode(encoding)[4:]

    dp_tokenize.batch = encode_many
    dp_tokenize.engine = engine
    if pretokenize_option == "llama":
        dp_tokenize.host_pool = host
    return dp_tokenize, decode_dp_tokenization


BLOOM_TOKENIZER_JSON = ("{}/models--bigscience--bloom-3b/snapshots/"
                        "52bc5b43010b4844513826b8be3f78c7344c37d7/tokenizer.json")


def dp_tokenize_bloom(bloom_tokenizer, HF_CACHE_DIR):
    """BLOOM byte-level adapter (reference tokenizer_utils.py:98-181).

    * the vocabulary is ``tokenizer.json``'s ``model.vocab`` with ids = its **enumeration
      order** (reference :104-108, ``{token: index for index, token in enumerate(vocab)}``);
    * words come from the tokenizer's own pre-tokenizer (``pre_tokenize_str``, :160-162);
    * a word's atoms are ``convert_ids_to_tokens([vocab_to_index[c] for c in word])`` (:155-157;
      a character outside the vocabulary raises KeyError there, as in the reference);
    * the DP + longest-token selection + ids run on the GPU in atoms mode (one launch per
      call; ``dp_tokenize.batch`` for many strings), ids = enumeration-order indices (:174-177).
    The reference's ``merges`` -> ``token_to_source_merge`` map (:113-116) feeds only the unused
    ``unwind_to_base_tokenization``; merges are parsed here in either tokenizer.json form
    ("a b" strings or [a, b] pairs) and otherwise unused.
    """
    import json

    with open(BLOOM_TOKENIZER_JSON.format(HF_CACHE_DIR), "r") as f:
        tokenizer_json = json.load(f)
    merges = tokenizer_json["model"]["merges"]
    vocab_to_index = _InverseDict({token: index for index, token in enumerate(tokenizer_json["model"]["vocab"])})
    token_to_source_merge = {}
    for merge in merges:
        a, b = merge.split() if isinstance(merge, str) else merge
        token_to_source_merge[a + b] = (a, b)
    engine = Encoder(Vocab(dict(vocab_to_index), _device()))

    def pretokenize(input_str):
        pretokenized = bloom_tokenizer._tokenizer.pre_tokenizer.pre_tokenize_str(input_str)
        return [block[0] for block in pretokenized]

    def atoms_of(word):
        token_inds = [vocab_to_index[c] for c in word]   # KeyError for characters outside the vocab
        return bloom_tokenizer.convert_ids_to_tokens(token_inds)

    def encode_many(texts: Sequence[str]) -> List[List[int]]:
        batch = [[atoms_of(w) for w in pretokenize(t)] for t in texts]
        out = []
        for t, (ids, st) in zip(texts, engine.encode_word_atoms(batch)):
            raise_for_status(st, t)
            out.append(ids)
        return out

    def dp_tokenize(input_str) -> List[int]:
        return encode_many([input_str])[0]

    def decode_dp_tokenization(encoding: List[int]):
        return bloom_tokenizer.decode(encoding)   # reference :179-181

    dp_tokenize.batch = encode_many
    dp_tokenize.engine = engine
    dp_tokenize.vocab_to_index = vocab_to_index
    return dp_tokenize, decode_dp_tokenization
