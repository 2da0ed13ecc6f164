"""Drop-in for the reference's ``packages/dp_tokenize.py`` (L1 DP core), GPU-backed.

* ``compute_shortest_tokenizations(base_representation_s, vocabulary,
  disregard_word_initial_marker, word_initial_marker) -> (List[List[str]], int)``
  (reference dp_tokenize.py:6-70): the forward DP runs on the GPU over the caller's
  atoms (DPT_MODE_ATOMS) and returns, per atom end i, the reachable part of the
  optimal-predecessor set ``segment_index_dp[i-1]``; the host then lists every shortest
  tokenization in the reference's DFS order (largest predecessor popped first, a subtree
  finished before its siblings, dp_tokenize.py:49-69).  Dead ends (unreachable
  predecessors, which the reference explores and drops) are never entered, so the list
  and its order are the reference's.  The second value is ``len_dp[-1]`` (capped DP).
  Raises IndexError on an empty input like the reference (dp_tokenize.py:49).
* ``obtain_longest_token(tokenizations)`` (dp_tokenize.py:72-84): the first tokenization
  whose longest token (code points) is longest; ValueError on an empty list.

The enumeration is exponential in the worst case (SURVEY.md §0 finding 4) -- for the
tokenizer use case call ``dp_tokenize`` (packages.tokenizer_utils), which selects the
same tokenization on the GPU without enumerating.
"""
from __future__ import annotations

import os
import sys
from collections import OrderedDict
from typing import List, Sequence

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from dptok import DptError, Encoder, Vocab  # noqa: E402
from dptok.engine import atoms_to_csr  # noqa: E402

_CACHE: "OrderedDict[frozenset, Encoder]" = OrderedDict()   # by content: token set -> engine
_BY_ID: "OrderedDict[tuple, tuple]" = OrderedDict()          # by identity: (id, len) -> (object, engine)


def _engine_for(vocabulary) -> Encoder:
    """The engine of a vocabulary (set, dict or list of token strings; non-strings and '' are not
    tokens).  Looked up by object identity + size first (O(1) for the callers that pass the same
    vocabulary every call), then by content (O(|V|), e.g. a set rebuilt per call), and built and
    uploaded only for a vocabulary not seen before.  Restriction: a vocabulary object changed IN PLACE
    without a change of size (one token swapped for another) hits the identity entry and is not
    re-read -- pass a new object (or a frozenset) after such a change; the reference re-reads its
    ``vocabulary`` on every call (dp_tokenize.py:39)."""
    key_id = (id(vocabulary), len(vocabulary))
    hit = _BY_ID.get(key_id)
    if hit is not None and hit[0] is vocabulary:
        _BY_ID.move_to_end(key_id)
        return hit[1]
    key = frozenset(t for t in vocabulary if isinstance(t, str) and t)
    enc = _CACHE.get(key)
    if enc is None:
        t2i = {tok: i for i, tok in enumerate(sorted(key))}
        enc = Encoder(Vocab(t2i, int(os.environ.get("LOCAL_RANK", "0"))))
        _CACHE[key] = enc
        if len(_CACHE) > 4:
            _CACHE.popitem(last=False)
    else:
        _CACHE.move_to_end(key)
    _BY_ID[key_id] = (vocabulary, enc)
    if len(_BY_ID) > 8:
        _BY_ID.popitem(last=False)
    return enc


def _dp_edges(atoms: Sequence[str], vocabulary):
    """GPU DP over one atom list: (status, length, per-end reachable-predecessor masks, far pairs)."""
    enc = _engine_for(vocabulary)
    text, offs, cut = atoms_to_csr([atoms])
    # edges are indexed by the byte offset of the string + atom end - 1; one string at offset 0
    return enc.dp(text, offs, mode="atoms", cut_mask=cut, edges=True, far=True)


def _dp_length(atoms: Sequence[str], vocabulary, uncapped: bool = False):
    """GPU DP over one atom list, lengths only: (status, capped len_dp[-1] or uncapped minimum)."""
    enc = _engine_for(vocabulary)
    text, offs, cut = atoms_to_csr([atoms])
    status, lengths, _ = enc.dp(text, offs, mode="atoms", cut_mask=cut, uncapped=uncapped)
    return int(status[0]), int(lengths[0])


def compute_shortest_tokenizations(base_representation_s, vocabulary, disregard_word_initial_marker,
                                   word_initial_marker):
    if disregard_word_initial_marker:
        # dp_tokenize.py:24-25 (str.lstrip strips any leading characters of the marker string)
        vocabulary = {token.lstrip(word_initial_marker) for token in vocabulary}
    atoms = list(base_representation_s)
    n = len(atoms)
    if n == 0:
        raise IndexError("list index out of range")
    status, lengths, edges, far = _dp_edges(atoms, vocabulary)
    status, length = int(status[0]), int(lengths[0])
    if status not in (0, 1):
        raise DptError("engine status %d" % status)
    if status == 1:
        return [], length
    # optimal reachable predecessors more than 64 atoms back (tokens of more than 64 atoms), which
    # the 64-bit masks cannot hold: per end index, their back distances
    far_by_end = {}
    for e, d in far.tolist():
        far_by_end.setdefault(e, []).append(d)

    # preds(i): reachable optimal predecessors of end i, ascending (= segment_index_dp[i-1] order)
    def preds(i: int) -> List[int]:
        m = int(edges[i - 1])
        out = [i - 1 - d for d in far_by_end.get(i - 1, ())]
        while m:
            d = (m & -m).bit_length() - 1
            out.append(i - 1 - d)
            m &= m - 1
        return sorted(out)

    stack = [(j, n, []) for j in preds(n)]
    done: List[List[str]] = []
    while stack:
        j, i, partial = stack.pop()
        toks = ["".join(atoms[j:i])] + partial
        if j == 0:
            done.append(toks)
        else:
            for jj in preds(j):
                stack.append((jj, j, list(toks)))
    return done, length


def obtain_longest_token(tokenizations: List[List[str]]) -> List[str]:
    tokenization_lengths = [max([len(t) for t in tokenization]) for tokenization in tokenizations]
    return tokenizations[tokenization_lengths.index(max(tokenization_lengths))]
