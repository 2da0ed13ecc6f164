"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

A fresh, reference-faithful Python restatement of the reference's
enumerate-then-select shortest tokenization, used (a) as the ``cpu_baseline``
"port" leg of ``bench.py`` (the algorithm the reference actually runs on the CPU,
timed on the GPU box's host cores -- the reference itself cannot travel) and
(b) to cross-check the C oracle on small cases in ``tests/``.

It follows, step by step:

* ``packages/dp_tokenize.py:27-47``  forward DP with the ``range(n+1)`` cap and
  the ascending optimal-predecessor lists (reset on strict decrease, append on
  equality);
* ``packages/dp_tokenize.py:49-70``  explicit-stack DFS that pops the largest
  predecessor first and completes a subtree before its siblings; dead ends
  (empty predecessor lists caused by the cap) are dropped;
* ``packages/dp_tokenize.py:72-84``  ``obtain_longest_token``: score = longest
  token in code points, FIRST argmax in enumeration order;
* ``packages/tokenizer_utils.py:33-50``  ``pretokenize_raw`` (first char gets
  the '▁' prefix, ' ' opens a word as atom '▁', '\\n' becomes atom '<0x0A>');
* ``packages/tokenizer_utils.py:66-80``  the ``dp_tokenize`` composition with the
  evident-intent 4-argument call (the shipped 5-argument call raises TypeError,
  SURVEY.md §0 finding 3).

Status codes mirror the C-ABI: 0 ok, 1 no complete tokenization (reference:
``ipdb.set_trace`` then ``ValueError`` from ``max([])``), 2 empty word
(reference: ``IndexError`` at ``dp_tokenize.py:49``).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

SPACE_MARK = "▁"
NEWLINE_ATOM = "<0x0A>"


def raw_words(text: str) -> List[List[str]]:
    """Atomise ``text`` like ``pretokenize_raw`` (tokenizer_utils.py:33-50)."""
    words: List[List[str]] = []
    cur: List[str] = []
    for i, ch in enumerate(text):
        if i == 0:
            cur.append(SPACE_MARK + ch)
        elif ch == " ":
            words.append(cur)
            cur = [SPACE_MARK]
        elif ch == "\n":
            cur.append(NEWLINE_ATOM)
        else:
            cur.append(ch)
    words.append(cur)
    return words


def forward_dp(atoms: Sequence[str], vocab) -> Tuple[List[int], List[List[int]]]:
    """cost[i] and the ascending optimal-predecessor list of each end i (dp_tokenize.py:27-47)."""
    n = len(atoms)
    cost = list(range(n + 1))
    preds: List[List[int]] = [[] for _ in range(n + 1)]
    for i in range(1, n + 1):
        best: List[int] = []
        for j in range(i):
            if "".join(atoms[j:i]) in vocab:
                c = cost[j] + 1
                if c < cost[i]:
                    cost[i] = c
                    best = [j]
                elif c == cost[i]:
                    best.append(j)
        preds[i] = best
    return cost, preds


def enumerate_shortest(atoms: Sequence[str], vocab, limit: int | None = None) -> Tuple[List[List[str]], int]:
    """All minimum-length tokenizations in the reference's DFS order (dp_tokenize.py:49-70).

    Raises IndexError on an empty word, like the reference. ``limit`` (optional)
    stops after that many complete tokenizations (the bench uses it as a guard).
    """
    n = len(atoms)
    if n == 0:
        raise IndexError("list index out of range")
    cost, preds = forward_dp(atoms, vocab)
    stack: List[Tuple[int, int, List[str]]] = [(j, n, []) for j in preds[n]]
    done: List[List[str]] = []
    while stack:
        j, i, partial = stack.pop()
        toks = ["".join(atoms[j:i])] + partial
        if j == 0:
            done.append(toks)
            if limit is not None and len(done) >= limit:
                break
        else:
            for jj in preds[j]:
                stack.append((jj, j, list(toks)))
    return done, cost[n]


def longest_token_choice(tokenizations: List[List[str]]) -> List[str]:
    """First tokenization whose longest token (code points) is longest (dp_tokenize.py:72-84)."""
    scores = [max(len(t) for t in tk) for tk in tokenizations]
    return tokenizations[scores.index(max(scores))]


def dp_tokenize_raw(text: str, t2i: Dict[str, int]) -> Tuple[List[int], int]:
    """Reference composition (tokenizer_utils.py:66-80, raw mode). Returns (ids, status)."""
    ids: List[int] = []
    for word in raw_words(text):
        try:
            toks, _ = enumerate_shortest(word, t2i)
        except IndexError:
            return [], 2
        if not toks:
            return [], 1
        ids.extend(t2i[t] for t in longest_token_choice(toks))
    return ids, 0


def dp_tokenize_word_atoms(words: Sequence[Sequence[str]], t2i: Dict[str, int]) -> Tuple[List[int], int]:
    """The BLOOM adapter's composition (tokenizer_utils.py:164-178): words of given atoms."""
    ids: List[int] = []
    for atoms in words:
        toks, _ = enumerate_shortest(atoms, t2i)
        if not toks:
            return [], 1
        ids.extend(t2i[t] for t in longest_token_choice(toks))
    return ids, 0


def min_tokens_for_string(s: Iterable[str], vocabulary) -> float:
    """Uncapped minimum token count, inf when impossible (inspect_tokenizer.py:77-86)."""
    s = list(s)
    n = len(s)
    best = [float("inf")] * (n + 1)
    best[0] = 0
    for i in range(1, n + 1):
        for j in range(i):
            if "".join(s[j:i]) in vocabulary:
                best[i] = min(best[i], best[j] + 1)
    return best[n]


def inspect_shortest_tokenizations(atoms: Sequence[str], vocabulary) -> Tuple[List[List[str]], float]:
    """``inspect_tokenizer.compute_shortest_tokenizations`` after its marker rule (inspect_tokenizer.py:109-146):
    the inf-initialised DP whose per-end lists keep every j with len[j] + 1 == len[i] -- for an unreachable
    end that is inf == inf, so they hold its unreachable in-vocabulary starts (:117-129) -- then the
    one-stack backtrace: pop a start, prepend atoms[start .. cursor], move the cursor before the start, and
    on reaching index -1 record the tokenization and put the cursor back at the last atom (:131-146)."""
    n = len(atoms)
    if n == 0:
        raise IndexError("list index out of range")
    inf = float("inf")
    length = [inf] * (n + 1)
    length[0] = 0
    lists: List[List[int]] = []
    for i in range(1, n + 1):
        cur: List[int] = []
        for j in range(i):
            if "".join(atoms[j:i]) not in vocabulary:
                continue
            if length[j] + 1 < length[i]:
                length[i] = length[j] + 1
                cur = [j]
            elif length[j] + 1 == length[i] and j not in cur:
                cur.append(j)
        lists.append(cur)
    stack = list(lists[n - 1])
    cursor = n - 1
    out: List[List[str]] = []
    part: List[str] = []
    while stack:
        s = stack.pop()
        part.insert(0, "".join(atoms[s:cursor + 1]))
        cursor = s - 1
        if cursor < 0:
            out.append(part)
            part = []
            cursor = n - 1
        else:
            stack.extend(lists[cursor])
    return out, length[n]
