"""Drop-in for the reference's ``inspect_tokenizer.py`` research helpers.

* ``min_tokens_for_string(s, vocabulary)`` (reference :77-86, the definition in effect):
  the minimum number of vocabulary tokens that spell ``s`` (characters are the atoms),
  ``float('inf')`` when impossible -- the inf-initialised (uncapped) DP, run on the GPU
  with DPT_FLAG_UNCAPPED.
* ``compute_length_of_most_efficient_tokenization(sequence, vocabulary)`` (reference
  :44-60, a ``pass`` stub whose docstring and the README TODO, README.md:3, specify it):
  the same minimum over a list of atoms.
* ``compute_shortest_tokenizations(base_representation_s, vocabulary, ...)`` (reference
  :88-146): returns ``(tokenizations, length)``; ``length`` is the uncapped minimum (inf when
  impossible), bit-exact with the reference.  The reference's list comes from a single-stack
  backtrace that mixes branches (440/3000 random cases differ from the
  packaged DP, e.g. ``babaaa`` -> ``['ba','baaa']`` with ``baaa`` not in V); this drop-in
  returns the well-formed shortest tokenizations of the packaged DP when its capped length
  equals the minimum, else ``[]``.  Callers use only the length (dialect_arabic.py:79-81).
  An empty input raises ``IndexError`` like the reference (``segment_index_dp[-1]`` of ``[]``,
  :132); lengths and exceptions are pinned by ``tests/golden/inspect_cst_cases.json.gz``.
* ``obtain_token_compositions(token_str, vocab, merges)`` (reference :17-42): merge-tree
  decompositions, host-side recursion over the merge list (no DP).
"""
from __future__ import annotations

import os
import sys
from typing import Dict, List, Set

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

from packages.dp_tokenize import _dp_length, compute_shortest_tokenizations as _packaged_cst  # noqa: E402

_INF_WORD = 0xFFFF


def obtain_token_compositions(token_str: str, vocab: Dict[str, int], merges: List[str]) -> List[List[str]]:
    if len(token_str) == 1:
        return [[token_str]]
    decompositions = []
    for i in range(len(token_str)):
        left = token_str[:i]
        right = token_str[i:]
        if f"{left} {right}" in merges:
            assert (left in vocab) and (right in vocab)
            decompositions.append([left, right])
            if len(left) > 1:
                decompositions.extend([d + [right] for d in obtain_token_compositions(left, vocab, merges)])
            if len(right) > 1:
                decompositions.extend([[left] + d for d in obtain_token_compositions(right, vocab, merges)])
    return decompositions


def _uncapped_min(atoms, vocabulary) -> float:
    atoms = list(atoms)
    if not atoms:
        return 0
    if not any(isinstance(t, str) and t for t in vocabulary):
        return float("inf")
    status, length = _dp_length(atoms, vocabulary, uncapped=True)
    if status not in (0, 1) or length >= _INF_WORD:
        return float("inf")
    return length


def compute_length_of_most_efficient_tokenization(sequence: List[str], vocabulary: Set[str]):
    return _uncapped_min(sequence, vocabulary)


def min_tokens_for_string(s: str, vocabulary: Set[str]):
    return _uncapped_min(list(s), vocabulary)


def compute_shortest_tokenizations(base_representation_s, vocabulary, disregard_word_initial_marker,
                                   word_initial_marker):
    if disregard_word_initial_marker:
        vocabulary = {token.lstrip(word_initial_marker) for token in vocabulary}
    atoms = list(base_representation_s)
    if not atoms:   # the reference indexes segment_index_dp[-1] of an empty list (:112, :132)
        raise IndexError("list index out of range")
    length = _uncapped_min(atoms, vocabulary)
    if length == float("inf"):
        return [], length
    toks, capped = _packaged_cst(atoms, vocabulary, False, None)
    return (toks if capped == length else []), length
