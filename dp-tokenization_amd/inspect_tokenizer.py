"""Drop-in for the reference's ``inspect_tokenizer.py`` research helpers.

* ``min_tokens_for_string(s, vocabulary)`` (reference :77-86, the definition in effect):
  the minimum number of vocabulary tokens that spell ``s`` (characters are the atoms),
  ``float('inf')`` when impossible -- the inf-initialised (uncapped) DP, run on the GPU
  with DPT_FLAG_UNCAPPED.
* ``compute_length_of_most_efficient_tokenization(sequence, vocabulary)`` (reference
  :44-60, a ``pass`` stub whose docstring and the README TODO, README.md:3, specify it):
  the same minimum over a list of atoms.
* ``compute_shortest_tokenizations(base_representation_s, vocabulary, ...)`` (reference
  :88-146): returns ``(tokenizations, length)``, both the reference's.  ``length`` is the uncapped
  minimum (inf when impossible).  The list is what the reference's single-stack backtrace (:131-146)
  produces -- including its mixed branches (e.g. ``babaaa`` -> ``['ba','baaa']`` with
  ``baaa`` not in V): the GPU runs the uncapped DP with edges (DPT_FLAG_UNCAPPED, DPT_MODE_ATOMS) and
  returns each end's optimal predecessors -- ``segment_index_dp[i-1]`` of :109-129, ascending -- and the
  host replays the backtrace over them (round 6; rounds 1-5 returned the packaged DP's well-formed list).
  Only reachable ends are ever visited by that backtrace, so the GPU's reachable-only masks are the whole
  of what it reads; an unreachable string end yields ``[]`` as in the reference.  An empty input raises
  ``IndexError`` like the reference (``segment_index_dp[-1]`` of ``[]``, :132); lengths, lists and
  exceptions are pinned by ``tests/golden/inspect_cst_cases.json.gz``.
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

from dptok import DptError  # noqa: E402
from dptok.engine import atoms_to_csr  # noqa: E402
from packages.dp_tokenize import _dp_length, _engine_for  # noqa: E402

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
    if not any(isinstance(t, str) and t for t in vocabulary):
        return [], float("inf")
    status, lengths, edges, far = _dp_uncapped_edges(atoms, vocabulary)
    if status not in (0, 1):
        raise DptError("engine status %d" % status)
    length = int(lengths[0])
    if status == 1 or length >= _INF_WORD:
        return [], float("inf")
    far_by_end: Dict[int, List[int]] = {}
    for e, d in far.tolist():
        far_by_end.setdefault(int(e), []).append(int(d))

    def preds(end: int) -> List[int]:   # segment_index_dp[end - 1] of a reachable end, ascending
        m = int(edges[end - 1])
        out = [end - 1 - d for d in far_by_end.get(end - 1, ())]
        while m:
            low = m & -m
            out.append(end - 1 - (low.bit_length() - 1))
            m ^= low
        out.sort()
        return out

    return _single_stack_backtrace(atoms, preds), length


def _dp_uncapped_edges(atoms, vocabulary):
    """GPU DP over one atom list, inf-initialised (:109-129): (status, minimum, per-end optimal-predecessor
    masks of reachable ends, far pairs for predecessors more than 64 atoms back)."""
    enc = _engine_for(vocabulary)
    text, offs, cut = atoms_to_csr([atoms])
    status, lengths, edges, far = enc.dp(text, offs, mode="atoms", cut_mask=cut, uncapped=True, edges=True,
                                         far=True)
    return int(status[0]), lengths, edges, far


def _single_stack_backtrace(atoms: List[str], preds) -> List[List[str]]:
    """The reference's backtrace (:131-146) as it behaves: ONE stack of start indices for all branches.  A
    popped start b closes the token atoms[b .. end] onto the tokenization being built, where `end` is the
    atom before the previous pop's start -- or the last atom once a tokenization has just been completed
    (the reference then restarts from the string end, whatever depth the next stacked start came from) --
    and pushes the optimal predecessors of b unless b == 0, which completes the tokenization."""
    n = len(atoms)
    pending = list(preds(n))
    last = n           # exclusive end of the next token
    building: List[str] = []
    done: List[List[str]] = []
    while pending:
        b = pending.pop()
        building = ["".join(atoms[b:last])] + building
        if b == 0:
            done.append(building)
            building = []
            last = n
        else:
            last = b
            pending.extend(preds(b))
    return done
