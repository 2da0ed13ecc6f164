"""Diagnostic: a CPU model of the lane-mode B + C1 of tokenize_kernel (G = 16, capless windows),
phase by phase over the 16 lanes of a row, for checking the chunk algorithm against the oracle's
selection on single windows (raw mode, strings <= 256 bytes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd"), os.path.join(ROOT, "tests")]
from oracle import ref_port

FRESH = 31
NEAR_CUT = True   # mirrors dpt_kernels.hip DPT_NEAR_CUT
NEAR_CUT64 = False   # ... and NEAR_CUT64 (the 64-lane push recurrence)

def relax(sj, span):
    a1 = sj + 64
    a2 = (a1 | 31) - span
    return min(a1, a2)

def window(text):
    """atoms (expanded strings), word-start flags per atom, cpos (code-point prefix) per boundary"""
    words = ref_port.raw_words(text)
    atoms, ws = [], []
    for w in words:
        for k, a in enumerate(w):
            atoms.append(a); ws.append(k == 0)
    cpos = [0]
    for a in atoms:
        cpos.append(cpos[-1] + len(a))
    return atoms, ws + [True], cpos

def model(text, vocab, verbose=False):
    atoms, wsf, cpos = window(text)
    na = len(atoms)
    # end masks: bit d of em[i] = atoms i-1-d .. i-1 form a token (within a word)
    em = [0] * (na + 1)
    for j in range(na):
        s = ""
        for L in range(1, 17):
            if j + L > na or (L > 1 and wsf[j + L - 1]):
                break
            s += atoms[j + L - 1]
            if s in vocab:
                em[j + L] |= 1 << (L - 1)
    assert all(em[i] & 1 for i in range(1, na + 1)), "not capless"
    key = [0] * (na + 2); fin = [0] * (na + 2); lstar = [0] * (na + 2)
    C = ((na + 15) >> 4) | 1
    lanes = []
    for d in range(16):
        c0 = min(d * C, na); c1 = min(c0 + C, na)
        mloc, lcut = 0xFFFF, 0
        for k in range(16, -1, -1):
            i = c0 + 1 + k
            if i <= c1:
                hb = em[i].bit_length() - 1
                mloc = min(mloc, i - 1 - hb)
                if mloc >= i - 1:
                    lcut |= 1 << k
        lanes.append(dict(c0=c0, c1=c1, mloc=mloc, lcut=lcut))
    for d in range(16):
        S = min([l["mloc"] for l in lanes[d + 1:]] + [0xFFFF])
        c0 = lanes[d]["c0"]; lcut = lanes[d]["lcut"]
        cut = 0 if S < c0 else (lcut if S - c0 >= 16 else lcut & ((2 << (S - c0)) - 1))
        lanes[d]["fc"] = c0 + ((cut & -cut).bit_length() - 1) if cut else na
        lanes[d]["lc"] = c0 + cut.bit_length() - 1 if cut else 0   # the lane's last cut
    for d in range(16):
        lanes[d]["rs"] = min([l["fc"] for l in lanes[d:]])
    if NEAR_CUT:   # the kernel's DPT_NEAR_CUT: the nearest cut to c0 (ties: the later one)
        for d in range(16):
            c0 = lanes[d]["c0"]
            prev = max([l["lc"] for l in lanes[:d]] + [0])
            if c0 - prev < lanes[d]["rs"] - c0:
                lanes[d]["rs"] = prev
    for d in range(16):
        lanes[d]["re"] = lanes[d + 1]["rs"] if d < 15 else na
    # B loop
    for d, l in enumerate(lanes):
        rs, re = l["rs"], l["re"]
        i = rs; ws = rs; sprev = FRESH; pe = 0; T = 0
        while i < re:
            i += 1
            best = relax(sprev, cpos[i] - cpos[i - 1]); dg = de = 0
            for dd in range(1, 16):
                if em[i] >> dd & 1:
                    j = i - 1 - dd
                    assert j >= ws
                    sj = FRESH if j == ws else key[j]
                    kk = relax(sj, cpos[i] - cpos[j])
                    if (kk >> 5) < (best >> 5): de = dd
                    if kk < best: dg = dd
                    best = min(best, kk)
            key[i] = best; fin[i] = dg | de << 4
            if wsf[i]:
                lstar[i] = 31 - (best & 31)
                T += best >> 6
                if not pe: pe = i
                ws = i; sprev = FRESH
            else:
                sprev = best
        re_ws = i > rs and sprev == FRESH
        p1in = pe == 0 or pe == re
        if not re_ws: T += sprev >> 6
        gl1 = 31 - ((key[re] if re_ws else sprev) & 31)
        l.update(pe=pe, T=T, sprev=sprev, re_ws=re_ws, p1in=p1in, gl1=gl1)
    # transfer scan (left to right)
    inn = FRESH
    for d, l in enumerate(lanes):
        l["in"] = inn
        x = l["sprev"]
        if l["pe"]:
            inn = x
        else:
            inn = (inn & 0xFFC0) + (x & 0xFFC0) + min(inn & 31, x & 31)
    for d, l in enumerate(lanes):
        rs, re, pe, inn = l["rs"], l["re"], l["pe"], l["in"]
        gin = 31 - (inn & 31)
        l["gin"] = gin
        if gin:
            lim = pe if pe else re
            for q in range(rs + 1, lim + 1):
                if gin >= 31 - (key[q] & 31):
                    fin[q] = (fin[q] & 0xF0) | (fin[q] >> 4)
            if pe:
                kl = key[pe]
                key[pe] = (inn & 0xFFC0) + (kl & 0xFFC0) + min(inn & 31, kl & 31)
                if gin > 31 - (kl & 31):
                    lstar[pe] = gin
        l["gre"] = max(gin, l["gl1"]) if l["p1in"] else l["gl1"]
    # token bases
    tb = 0
    for l in lanes:
        l["tb"] = tb; tb += l["T"]
    # P1 L*: from the right
    for d, l in enumerate(lanes):
        if l["re_ws"]:
            l["ls1"] = l["gre"]
        else:
            nxt = [m for m in lanes[d + 1:] if m["pe"]]
            l["ls1"] = lstar[nxt[0]["pe"]] if nxt else 1
    starts = [None] * tb
    for d, l in enumerate(lanes):
        rs, re, T, tbd, ls1 = l["rs"], l["re"], l["T"], l["tb"], l["ls1"]
        left = l["gre"] < ls1
        l["left"] = left
        ii = re; k = tbd + T; A = ls1 if left else 0; Ls = ls1; pend = cpos[re]; inp1 = True; n1 = 0
        while k > tbd:
            if ii < re and wsf[ii]:
                Ls = lstar[ii]; A = 0; pend = cpos[ii]; inp1 = False
            n1 += inp1
            f = fin[ii]
            sp = pend - cpos[ii]; A = max(A, sp)
            dd = (f & 15) if A < Ls else (f >> 4)
            j = ii - 1 - dd
            k -= 1; starts[k] = j
            pend = cpos[ii]; ii = j
        assert ii == rs, (d, ii, rs)
        afin = max(A, pend - cpos[rs])
        l.update(n1=n1, sel=T > 0 and afin >= Ls, stop=(not l["p1in"]) or l["re_ws"])
    for d, l in enumerate(lanes):
        f = False
        if not l["re_ws"]:
            for m in lanes[d + 1:]:
                f = f or m["sel"]
                if m["stop"]:
                    break
        l["fin_in"] = f
        if f and not l["left"] and (not l["p1in"] or l["gin"] < l["ls1"]):
            ii = l["re"]; k = l["tb"] + l["T"]
            for c in range(l["n1"]):
                j = ii - 1 - (fin[ii] >> 4)
                k -= 1; starts[k] = j; ii = j
    toks = []
    for k in range(tb):
        e = starts[k + 1] if k + 1 < tb else na
        toks.append("".join(atoms[starts[k]:e]))
    if verbose:
        for d, l in enumerate(lanes):
            print(d, {k: l[k] for k in ("rs", "re", "pe", "T", "tb", "gin", "gre", "ls1", "left", "sel", "stop", "fin_in", "n1", "p1in", "re_ws")})
    return toks

FRESH64 = 0x7FFF

def model64(text, vocab, verbose=False):
    """forward_lanes64 (tokenize_kernel, G = 64, capless windows) over the 64 lanes of a wave, then
    the row-mode C1 walk (one word per lane: dg while the longest token so far is below the
    word's G, de after).  Keys: cost << 16 | 0x7FFF - G; entries {dg | de << 8 | cp(i) << 16, key}."""
    atoms, wsf, cpos = window(text)
    na = len(atoms)
    # start masks: bit d of sm[j] = atoms j .. j+d form a token (within a word, <= 64 atoms)
    sm = [0] * (na + 1)
    for j in range(na):
        s = ""
        for L in range(1, 65):
            if j + L > na or (L > 1 and wsf[j + L - 1]):
                break
            s += atoms[j + L - 1]
            if s in vocab:
                sm[j] |= 1 << (L - 1)
    assert all(sm[j] & 1 for j in range(na)), "not capless"
    # cut points: p is one iff max_{j < p} (j + 1 + hb(sm[j])) <= p
    cut = [False] * (na + 1)
    run = 0
    for p in range(na + 1):
        cut[p] = run <= p
        if p < na:
            run = max(run, p + sm[p].bit_length())
    nextcut = lambda c: next(p for p in range(c, na + 1) if cut[p])
    prevcut = lambda c: max(p for p in range(0, min(c, na) + 1) if cut[p])

    def snap(c):   # the kernel's nearest-cut rule (DPT_NEAR_CUT), else the next cut
        nx = nextcut(c)
        if not NEAR_CUT64:
            return nx
        pv = prevcut(c)
        return pv if c - pv < nx - c else nx
    C = (na + 63) >> 6
    fx = [0] * (na + 2); fy = [0] * (na + 2)
    lanes = []
    for d in range(64):
        c0 = min(d * C, na); c1 = min(c0 + C, na)
        rs, re = snap(c0), snap(c1)
        pe = 0
        for i in range(rs + 1, re + 1):
            fx[i] = cpos[i] << 16; fy[i] = 0xFFFFFFFF
            if not pe and wsf[i]:
                pe = i
        for j in range(rs, re):
            kj = FRESH64 if (j == rs or wsf[j]) else fy[j]
            a1 = kj + 0x10000
            m = sm[j]
            while m:
                dd = (m & -m).bit_length() - 1
                m &= m - 1
                i = j + 1 + dd
                assert i <= re
                a2 = (a1 | 0x7FFF) + cpos[j] - (fx[i] >> 16)
                kk = min(a1, a2)
                if (kk >> 15) <= (fy[i] >> 15):
                    fx[i] = (fx[i] & ~0x7F00) | dd << 8
                if kk <= fy[i]:
                    fx[i] = (fx[i] & ~0x7F) | dd
                fy[i] = min(kk, fy[i])
        x = FRESH64 if rs == re else ((0x80000000 if pe else 0) | (FRESH64 if wsf[re] else fy[re]))
        lanes.append(dict(rs=rs, re=re, pe=pe, x=x))
    inn = FRESH64
    for l in lanes:
        l["in"] = inn
        x = l["x"]
        if x & 0x80000000:
            inn = x & 0x7FFFFFFF
        else:
            inn = ((inn & 0x7FFF0000) + (x & 0x7FFF0000)) | min(inn & 0x7FFF, x & 0x7FFF)
    for l in lanes:
        rs, re, pe, inn = l["rs"], l["re"], l["pe"], l["in"]
        gin = 0x7FFF - (inn & 0x7FFF)
        if gin:
            lim = pe if pe else re
            for q in range(rs + 1, lim + 1):
                if gin >= 0x7FFF - (fy[q] & 0x7FFF):
                    fx[q] = (fx[q] & ~0x7F) | ((fx[q] >> 8) & 0x7F)
            if pe:
                kl = fy[pe]
                fy[pe] = ((inn & 0x7FFF0000) + (kl & 0x7FFF0000)) | min(inn & 0x7FFF, kl & 0x7FFF)
    if verbose:
        print([(l["rs"], l["re"], l["pe"]) for l in lanes if l["rs"] < l["re"]])
    # row-mode C1 per word
    toks = []
    wstarts = [i for i in range(na) if wsf[i]] + [na]
    for w in range(len(wstarts) - 1):
        e = wstarts[w + 1]
        F = fy[e]
        cost, Ls = F >> 16, 0x7FFF - (F & 0x7FFF)
        i, A, pend, out = e, 0, cpos[e], []
        for _ in range(cost):
            A = max(A, pend - cpos[i])
            dd = (fx[i] & 127) if A < Ls else ((fx[i] >> 8) & 127)
            j = i - 1 - dd
            out.append("".join(atoms[j:i]))
            pend = cpos[i]; i = j
        assert i == wstarts[w], (w, i)
        toks += out[::-1]
    return toks

def ref_tokens(text, vocab):
    out = []
    for w in ref_port.raw_words(text):
        toks, _ = ref_port.enumerate_shortest(w, vocab)
        out += ref_port.longest_token_choice(toks)
    return out

if __name__ == "__main__":
    from dptok import synth
    from conftest import load_golden
    vocab = set(synth.llama_shaped_vocab())
    g = load_golden("cfg2_llama32k.json.gz")
    bad = 0
    for n, c in enumerate(g["cases"][:int(sys.argv[1]) if len(sys.argv) > 1 else 40]):
        inv = {v: k for k, v in synth.llama_shaped_vocab().items()}
        want = [inv[i] for i in c["ids"]]
        got = model(c["text"], vocab)
        if got != want:
            bad += 1
            k = next(k for k in range(min(len(got), len(want))) if got[k] != want[k])
            print("case", n, "diff at", k, got[k-3:k+4], want[k-3:k+4])
            if bad == 1:
                model(c["text"], vocab, verbose=True)
    print("bad", bad)
