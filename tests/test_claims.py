"""CPU model of the tokenize kernel's work distribution (dpt_kernels.hip tokenize_kernel, the
`claim` lambda and the refill loop): npart = min(NPART, max(1, n / 4096)) partition counters,
partition p holding the 256-string chunks p, p + npart, ... (part_size / part_string), claims of
as many strings as the wave has free slots (1..4), a used-up mask; each wave starts on partition
blockIdx mod npart and moves to the next unmarked partition after a claim reaches its partition's
end.  Under random interleavings of the waves' atomics every string is handed out exactly once and
every wave stops."""
import random

import pytest

NPART = 16
CHUNK = 256   # FIN_BATCH


def part_size(n, npart, p):
    nch = (n + CHUNK - 1) // CHUNK
    if nch <= p:
        return 0
    cnt = (nch - 1 - p) // npart + 1
    last = p + (cnt - 1) * npart
    return cnt * CHUNK - (nch * CHUNK - n if last == nch - 1 else 0)


def part_string(npart, p, v):
    return ((v // CHUNK) * npart + p) * CHUNK + v % CHUNK


def run(n_work, n_waves, seed):
    rnd = random.Random(seed)
    npart = min(NPART, max(1, n_work // 4096))
    ctr = [0] * npart
    mask = 0
    allm = (1 << npart) - 1
    got = [0] * n_work
    waves = [{"part": w % npart, "q": [], "done": False} for w in range(n_waves)]

    def claim(wv, req):
        nonlocal mask
        while True:
            p = wv["part"]
            hi = part_size(n_work, npart, p)
            b = ctr[p]; ctr[p] += req                 # atomicAdd
            nb = b
            ne = min(nb + req, hi) if nb < hi else nb
            claimed_all = False
            if nb + req >= hi:
                old = mask; mask |= 1 << p            # atomicOr
                m = old | (1 << p)
                if m & allm == allm:
                    claimed_all = True
                else:
                    free = ~m & allm
                    hi_free = free & ~((2 << p) - 1)
                    pick = hi_free if hi_free else free
                    wv["part"] = (pick & -pick).bit_length() - 1
            if ne > nb or claimed_all:
                return [part_string(npart, p, v) for v in range(nb, ne)], claimed_all

    live = list(range(n_waves))
    while live:
        w = rnd.choice(live)                           # any wave may take the next atomic
        wv = waves[w]
        idx, claimed_all = claim(wv, rnd.randint(1, 4))   # the wave's free slots
        for i in idx:
            got[i] += 1
        if claimed_all:
            live.remove(w)
    return got


@pytest.mark.parametrize("n_work,n_waves", [(1, 1), (3, 64), (4095, 50), (4096 * 16 + 3, 300), (100003, 700), (70000, 5632),
                                             (256 * 16 * 5 + 256, 400), (256 * 16 * 5 - 1, 400)])
def test_every_string_exactly_once(n_work, n_waves):
    for seed in range(3):
        assert run(n_work, n_waves, seed) == [1] * n_work


def test_partitions_tile_the_batch():
    # part_string maps each partition's local indices onto disjoint string sets covering [0, n)
    for n in [1, 255, 256, 257, 4096, 65535, 65536, 65537, 256 * 16 * 7 + 100, 1000000]:
        npart = min(NPART, max(1, n // 4096))
        seen = []
        for p in range(npart):
            seen += [part_string(npart, p, v) for v in range(part_size(n, npart, p))]
        assert sorted(seen) == list(range(n)), n
