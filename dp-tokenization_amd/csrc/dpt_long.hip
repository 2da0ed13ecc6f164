// dpt_long.hip -- the unbounded pass: strings the windowed kernels cannot take.
//
// tokenize_kernel (dpt_kernels.hip) holds a window of <= 256 / 2048 bytes in LDS and walks
// tokens of <= 16 / 64 atoms.  A string that contains a word longer than 2048 bytes, an atom
// longer than 8 bytes, or -- when the vocabulary has tokens longer than 64 code points -- a
// word of more than 64 atoms is handed here through the long list.  The reference has no such
// limits (packages/dp_tokenize.py:24-84 runs on any word), so neither does this pass: every
// per-atom quantity lives in global scratch indexed by the string's own byte range, which
// bounds the atom count.
//
// One wavefront per string, the whole string at once:
//   atomise  chunks of 256 bytes, one DPP scan each: per atom a, rec[a] = {byte offset,
//            code-point prefix mod 2^30 | word start << 31}  (pretokenize_raw,
//            tokenizer_utils.py:33-50; DPT_MODE_PRESPLIT / ATOMS from the cut mask)
//   A        lanes walk the byte trie from 64 start atoms at a time; token spans of <= 64
//            atoms set bit L-1 of the start's 64-bit mask (rec[a].z/w), longer ones flag
//            their last atom (LONG_END) -- "join(atoms[j:i]) in vocabulary", dp_tokenize.py:39
//   B        sequential over end positions: lane d holds candidate j = i-1-d in 64-bit key form
//            (cost[j]+1) << 32 | invalid[j] << 31 | (0x7FFFFFFF - G[j]); a wave min gives
//            cost[i] (capped at the atom index within the word, dp_tokenize.py:28, or
//            uncapped for inspect_tokenizer.py:77-86), reachability and G[i] (SURVEY.md
//            Appendix A 1-3).  At a flagged end the wave also scans the starts more than 64
//            atoms back, re-walking each span through the trie.  Per end i: the largest j
//            attaining the key (dg) and the largest reachable j in E(i) (de), 16 bits each.
//   C0       word costs / validity, C1 selection (one lane per word: dg while the longest
//            token so far is below G of the word, de after -- the reference's first argmax
//            in DFS order, dp_tokenize.py:58, :84), C2 ids by re-walking every selected span
//            (t2i[token], tokenizer_utils.py:76-79), 64 tokens at a time.
//
// Scratch per string s (atoms n <= slen): a range [ao, ao+slen) of the ctx's arena, claimed in list
// order (ao = an atomic add of slen to the arena counter); a string whose range does not fit gets
// status 3 and the host path reruns the call with an arena as large as the counter says
// (dpt_api.cpp), so the arena need not hold 20 bytes per input byte of the whole batch:
//   rec[ao+a]      uint4 {off, cpb | WS | LONG_END, mask lo -> dg | de << 16 of end a+1,
//                         mask hi -> state of a (long candidates) / final key of the word ending at a+1}
//   stg[ao+a]      state of a (cost part) / word-final cost -> token starts (C1)
// The ids (C2) go to the staging row of the string, staging16 / staging at its byte offset sb + k.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dpt_internal.h"

namespace dpt {
namespace lng {

__device__ __forceinline__ unsigned lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ unsigned uni(unsigned x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ unsigned incl_scan_add(unsigned v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false); // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false); // row_bcast:31
    return v;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, unsigned m) {
    const int src = (int)((lane_id() ^ m) << 2);
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)(unsigned)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (unsigned m = 1; m < 64; m <<= 1) {
        const uint64_t o = shfl_xor64(v, m);
        v = o < v ? o : v;
    }
    return ((uint64_t)uni((unsigned)(v >> 32)) << 32) | uni((unsigned)v);
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) { return __builtin_amdgcn_readlane(incl_scan_add(v), 63); }

// lane l receives x[l-1]; lane 0 receives `in` (wave_shr:1)
__device__ __forceinline__ unsigned shift_in(unsigned x, unsigned in) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)in, (int)x, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t shift_in64(uint64_t x, uint64_t in) {
    return ((uint64_t)shift_in((unsigned)(x >> 32), (unsigned)(in >> 32)) << 32) | shift_in((unsigned)x, (unsigned)in);
}

// global-memory ordering between the phases of one wave (the scratch is written and read back
// by other lanes of the same wave)
__device__ __forceinline__ void phase_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
}

constexpr unsigned WS = 0x80000000u;         // rec.y: atom starts a word
constexpr unsigned LONG_END = 0x40000000u;   // rec.y: a token of more than 64 atoms ends with this atom
constexpr unsigned CPM = 0x3FFFFFFFu;        // rec.y: code-point prefix mod 2^30

constexpr int32_t TERM_BIT = (int32_t)0x80000000;
constexpr int32_t LEAF_BIT = 0x40000000;
constexpr int32_t BASE_MASK = 0x3FFFFFFF;

constexpr uint64_t NONE = ~0ull;
constexpr uint64_t SK0 = (1ull << 32) | 0x7FFFFFFFull;   // a word start: cost 0 (+1), reachable, G 0

struct Args {
    const uint8_t *text;
    const uint64_t *str_off;
    const uint8_t *cut_mask;
    int32_t *staging;     // the final ids at sb + k (int32 vocabularies)
    int16_t *staging16;   // non-null: the final ids go here as int16 instead
    uint4 *rec;           // arena: rec[arena_cap], then stg[arena_cap]
    int32_t *stg;
    uint64_t arena_cap;
    unsigned long long *arena_used;
    uint64_t *counts;
    unsigned long long *bsum;   // nullable: per FIN_BATCH strings, the sum of their counts
    int32_t *status;
    int32_t *capped;
    uint64_t *edges;
    uint64_t *far;
    uint64_t far_cap;
    unsigned long long *far_count;
    const uint32_t *list;
    const uint32_t *list_count;
    uint32_t *work_next;
    const int2 *__restrict__ slots;
    const int4 *__restrict__ slots4;
    uint32_t n_slots;
    int32_t root_base;
    uint32_t max_tok_bytes;
    int long_span;
    int mode;
};

__device__ __forceinline__ int2 trie_slot(const Args &a, int32_t t) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)a.slots, (short)0, (int)(a.n_slots * 8u), 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (unsigned)t * 8u, 0, 0);
    return make_int2((int32_t)v[0], (int32_t)v[1]);
}
__device__ __forceinline__ int4 trie_slot4(const Args &a, int32_t t) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)a.slots4, (short)0, (int)(a.n_slots * 16u), 0x00020000);
    return __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)t * 16u, 0, 0));
}

// One string's view of the scratch and its atoms.
struct Str {
    const uint8_t *t;   // bytes
    uint4 *rec;
    int32_t *stg;
    unsigned slen, na, cp_tot;
    bool raw;
    __device__ __forceinline__ unsigned off(unsigned a) const { return a < na ? rec[a].x : slen; }
    __device__ __forceinline__ unsigned cpb(unsigned a) const { return a < na ? (rec[a].y & CPM) : cp_tot; }
    __device__ __forceinline__ bool wstart(unsigned a) const { return a >= na || (rec[a].y & WS) != 0; }
};

// Expanded bytes of one atom, one at a time: a prefix of <= 8 substituted bytes ('▁' before the
// string's first code point, '▁' for ' ', "<0x0A>" for '\n' -- raw mode only), then the atom's
// own input bytes (none after a substitution).
struct Cursor {
    uint64_t pre;
    unsigned pcnt, p, rem;
    __device__ __forceinline__ void load(const Str &S, unsigned a) {
        const unsigned o = S.off(a), e = S.off(a + 1);
        const unsigned b0 = S.t[o];
        p = o; rem = e - o; pre = 0; pcnt = 0;
        if (S.raw) {
            if (a == 0) { pre = 0x8196E2ull; pcnt = 3; }
            else if (b0 == ' ') { pre = 0x8196E2ull; pcnt = 3; rem = 0; }
            else if (b0 == '\n') { pre = 0x3E413078303Cull; pcnt = 6; rem = 0; }
        }
    }
    __device__ __forceinline__ unsigned next(const Str &S) {
        if (pcnt) { const unsigned b = (unsigned)(pre & 0xFFu); pre >>= 8; pcnt--; return b; }
        rem--;
        return S.t[p++];
    }
    __device__ __forceinline__ bool at_end() const { return pcnt == 0 && rem == 0; }
};

// Is atoms [j, i) one vocabulary token?  Walks the expanded bytes through the trie.
__device__ bool span_is_token(const Args &a, const Str &S, unsigned j, unsigned i) {
    int32_t node = 0, nb = a.root_base;
    Cursor c;
    for (unsigned at = j; at < i; at++) {
        c.load(S, at);
        while (!c.at_end()) {
            const int32_t t = nb + (int32_t)c.next(S);
            const int2 ent = trie_slot(a, t);
            if (ent.y != node) return false;
            node = t;
            nb = ent.x & BASE_MASK;
            if ((ent.x & LEAF_BIT) && !(c.at_end() && at + 1 == i)) return false;
            if (c.at_end() && at + 1 == i) return (ent.x & TERM_BIT) != 0;
        }
    }
    return false;
}

// (the body of dpt_kernels.hip fallback_kernel's unbounded-pass blocks)
__device__ __forceinline__ void long_body(const Args &a) {
    const unsigned lane = lane_id();
    const int mode = a.mode & DPT_MODE_MASK;
    const bool raw = mode == DPT_MODE_RAW;
    const bool uncapped = (a.mode & DPT_FLAG_UNCAPPED) != 0;
    const bool len_only = (a.mode & (DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY)) != 0;
    const uint64_t base_off = a.str_off[0];
    const unsigned n_work = *a.list_count;
    if (n_work == 0) return;   // the usual case: no counter traffic

    for (;;) {
        unsigned idx = 0;
        if (lane == 0) idx = atomicAdd(a.work_next, 1u);
        idx = __builtin_amdgcn_readlane(idx, 0);
        if (idx >= n_work) break;
        const uint64_t s = a.list[idx];
        const uint64_t o0 = a.str_off[s], o1 = a.str_off[s + 1];
        const uint64_t sb = o0 - base_off;
        // the string's scratch range in the arena
        unsigned long long ao = 0;
        if (lane == 0) ao = atomicAdd(a.arena_used, (unsigned long long)(o1 - o0));
        // (each half through uint32_t: readlane returns int, and a low half >= 2^31 would sign-extend)
        ao = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((unsigned)(ao >> 32), 0) << 32) |
             (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((unsigned)ao, 0);
        if (ao + (o1 - o0) > a.arena_cap) {
            // does not fit: status 3 (dpt_encode_host / dpt_dp_host grow the arena and rerun)
            if (lane == 0) {
                a.status[s] = DPT_STATUS_TOO_LONG;
                a.counts[s] = 0;
                if (a.capped) a.capped[s] = -1;
            }
            continue;
        }
        Str S;
        S.t = a.text + sb;
        S.rec = a.rec + ao;
        S.stg = a.stg + ao;
        S.slen = (unsigned)(o1 - o0);
        S.raw = raw;
        const uint8_t *cut = raw ? nullptr : a.cut_mask + sb;

        // ------------------------------------------------------------ atomise
        unsigned na = 0, cp = 0;
        for (unsigned c0 = 0; c0 < S.slen; c0 += 256) {
            bool as[4], wsf[4];
            unsigned cl[4], an = 0, cs = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const unsigned k = c0 + lane * 4 + u;
                const bool in = k < S.slen;
                const unsigned b = in ? S.t[k] : 0u;
                const unsigned cm = (in && !raw) ? cut[k] : 0u;
                const bool first = in && k == 0;
                const bool cont = in && !first && (mode == DPT_MODE_ATOMS ? (cm & 3u) == 0 : (b & 0xC0u) == 0x80u);
                as[u] = in && !cont;
                if (raw) {
                    wsf[u] = as[u] && (k == 0 || b == ' ');
                    cl[u] = !in ? 0u : first ? 2u : (b == '\n' ? 6u : ((b & 0xC0u) == 0x80u ? 0u : 1u));
                } else {
                    wsf[u] = as[u] && (k == 0 || (mode == DPT_MODE_PRESPLIT ? cm != 0 : (cm & 1u) != 0));
                    cl[u] = (in && (b & 0xC0u) != 0x80u) ? 1u : 0u;
                }
                an += as[u];
                cs += cl[u];
            }
            const unsigned v = an | (cs << 9);   // atoms <= 256 per chunk, code points <= 1536
            const unsigned incl = incl_scan_add(v);
            const unsigned tot = __builtin_amdgcn_readlane(incl, 63);
            unsigned ai = na + ((incl - v) & 0x1FFu);
            unsigned cpi = cp + ((incl - v) >> 9);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (as[u]) {
                    S.rec[ai] = make_uint4(c0 + lane * 4 + u, (cpi & CPM) | (wsf[u] ? WS : 0u), 0u, 0u);
                    ai++;
                }
                cpi += cl[u];
            }
            na += tot & 0x1FFu;
            cp += tot >> 9;
        }
        S.na = na;
        S.cp_tot = cp & CPM;
        phase_sync();

        // ------------------------------------------------------------ A: match discovery
        for (unsigned j0 = 0; j0 < na; j0 += 64) {
            const unsigned j = j0 + lane;
            bool active = j < na;
            uint64_t mask = 0;
            unsigned at = j, len = 0;
            int32_t node = 0, nb = a.root_base;
            Cursor c;
            if (active) c.load(S, at);
            while (ballot(active)) {
                if (active) {
                    const int32_t t = nb + (int32_t)c.next(S);
                    const int2 ent = trie_slot(a, t);
                    if (ent.y != node) {
                        active = false;
                    } else {
                        node = t;
                        nb = ent.x & BASE_MASK;
                        const bool leaf = (ent.x & LEAF_BIT) != 0;
                        if (c.at_end()) {
                            len++;
                            if (ent.x & TERM_BIT) {
                                if (len <= 64) mask |= 1ull << (len - 1);
                                else atomicOr(&S.rec[at].y, LONG_END);
                            }
                            at++;
                            if (leaf || S.wstart(at) || (!a.long_span && len == 64)) active = false;
                            else c.load(S, at);
                        } else if (leaf) {
                            active = false;
                        }
                    }
                }
            }
            if (j < na) {
                S.rec[j].z = (unsigned)mask;
                S.rec[j].w = (unsigned)(mask >> 32);
            }
        }
        phase_sync();

        // ------------------------------------------------------------ B: forward recurrence
        unsigned status = 0;
        uint64_t last_key = 0;
        {
            uint64_t sk = lane == 0 ? SK0 : NONE;   // lane d: state of candidate j = i-1-d
            unsigned cpj = 0, mlo = 0, mhi = 0;
            if (lane == 0) { mlo = S.rec[0].z; mhi = S.rec[0].w; }
            unsigned ws = 0;
            uint4 prev = S.rec[0];
            for (unsigned i = 1; i <= na; i++) {
                const uint4 cur = i < na ? S.rec[i] : make_uint4(S.slen, S.cp_tot | WS, 0u, 0u);
                const unsigned cpi = cur.y & CPM;
                const unsigned bit = (lane < 32 ? (mlo >> lane) : (mhi >> (lane - 32))) & 1u;
                uint64_t kv = NONE;
                if (bit && sk != NONE) {
                    const unsigned span = (cpi - cpj) & CPM;
                    const uint64_t k2 = (sk | 0x7FFFFFFFull) - span;
                    kv = sk < k2 ? sk : k2;
                }
                uint64_t r = wave_min64(kv);
                // tokens of more than 64 atoms ending at i (rare): scan the far starts
                uint64_t rl = NONE;
                unsigned jgl = 0, jel = 0;
                if (prev.y & LONG_END) {
                    phase_sync();   // the states of the far starts were stored by earlier steps
                    // a token of B bytes spans at most B atoms
                    const unsigned lo = (i > a.max_tok_bytes && i - a.max_tok_bytes > ws) ? i - a.max_tok_bytes : ws;
                    // chunks of 64 starts, nearest first: jb, jb-1, ..., down to lo
                    for (unsigned jb = i - 65; i >= 65 + lo; jb -= 64) {
                        const unsigned jj = jb - lane;
                        uint64_t key = NONE;
                        if (lane <= jb - lo && span_is_token(a, S, jj, i)) {
                            const uint64_t st = (S.rec[jj].y & WS) ? SK0
                                : (((uint64_t)(uint32_t)S.stg[jj] << 32) | S.rec[jj].w);
                            if (st != NONE) {
                                const unsigned span = (cpi - (S.rec[jj].y & CPM)) & CPM;
                                const uint64_t k2 = (st | 0x7FFFFFFFull) - span;
                                key = st < k2 ? st : k2;
                            }
                        }
                        const uint64_t rc = wave_min64(key);
                        if (rc != NONE) {
                            const uint64_t gm = ballot(key == rc), em = ballot(key != NONE && (key >> 31) == (rc >> 31));
                            const unsigned jg_c = jb - (unsigned)__builtin_ctzll(gm), je_c = jb - (unsigned)__builtin_ctzll(em);
                            if (rl == NONE || rc < rl) {
                                if (rl == NONE || (rc >> 31) < (rl >> 31)) jel = je_c;
                                jgl = jg_c;
                                rl = rc;
                            }
                        }
                        if (jb < lo + 64) break;
                    }
                    r = rl < r ? rl : r;
                }
                if (!uncapped) {
                    const uint64_t capkey = ((uint64_t)(i - ws) << 32) | 0xFFFFFFFFull;   // len_dp = range(n+1)
                    r = capkey < r ? capkey : r;
                }
                const uint64_t gmb = ballot(kv == r);
                const uint64_t emb = ballot(kv != NONE && ((kv ^ r) >> 31) == 0);
                unsigned dg = 0xFFFFu, de = 0xFFFFu;
                if (gmb) dg = (unsigned)__builtin_ctzll(gmb);
                else if (rl != NONE && rl == r) dg = i - 1 - jgl;
                if (emb) de = (unsigned)__builtin_ctzll(emb);
                else if (rl != NONE && (rl >> 31) == (r >> 31)) de = i - 1 - jel;
                const bool wend = (cur.y & WS) != 0;
                if (lane == 0) {
                    S.rec[i - 1].z = (dg & 0xFFFFu) | (de << 16);
                    if (a.edges) a.edges[sb + i - 1] = emb;
                }
                if (a.edges && rl != NONE && (rl >> 31) == (r >> 31)) {
                    // E(i) has starts more than 64 atoms back, which the 64-bit edge mask cannot
                    // hold: list every one of them as an (end, back distance) pair (the far scan
                    // again, against the final key), or report status 3 without a far list
                    if (!a.far) {
                        status = 3;
                    } else {
                        const unsigned lo = (i > a.max_tok_bytes && i - a.max_tok_bytes > ws) ? i - a.max_tok_bytes : ws;
                        for (unsigned jb = i - 65; i >= 65 + lo; jb -= 64) {
                            const unsigned jj = jb - lane;
                            bool hit = false;
                            if (lane <= jb - lo && span_is_token(a, S, jj, i)) {
                                const uint64_t st = (S.rec[jj].y & WS) ? SK0
                                    : (((uint64_t)(uint32_t)S.stg[jj] << 32) | S.rec[jj].w);
                                if (st != NONE) {
                                    const unsigned span = (cpi - (S.rec[jj].y & CPM)) & CPM;
                                    const uint64_t k2 = (st | 0x7FFFFFFFull) - span;
                                    hit = (((st < k2 ? st : k2) ^ r) >> 31) == 0;
                                }
                            }
                            const uint64_t hm = ballot(hit);
                            if (hm) {
                                unsigned long long base = 0;
                                if (lane == 0) base = atomicAdd(a.far_count, (unsigned long long)__builtin_popcountll(hm));
                                // (each half through uint32_t: readfirstlane returns int, whose sign would extend)
                                base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(base >> 32)) << 32) |
                                       (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)base);
                                const uint64_t k = base + __builtin_amdgcn_mbcnt_hi((unsigned)(hm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)hm, 0u));
                                if (hit && k < a.far_cap) {
                                    a.far[2 * k] = sb + i - 1;
                                    a.far[2 * k + 1] = i - 1 - jj;
                                }
                            }
                            if (jb < lo + 64) break;
                        }
                    }
                }
                // state of position i in key form; "inf" (no candidate, uncapped) stays inf
                uint64_t st_i = (r >> 32) >= 0xFFFFFFFEull ? NONE : r + (1ull << 32);
                if (wend) {
                    if (i < na) {
                        if (lane == 0) { S.stg[i - 1] = (int32_t)(uint32_t)(r >> 32); S.rec[i - 1].w = (unsigned)r; }
                    } else {
                        last_key = r;
                    }
                    st_i = SK0;
                    ws = i;
                } else if (a.long_span && lane == 0) {
                    S.stg[i] = (int32_t)(uint32_t)(st_i >> 32);
                    S.rec[i].w = (unsigned)st_i;   // rec[i].w (mask hi of start i) is in `cur` already
                }
                sk = shift_in64(sk, st_i);
                cpj = shift_in(cpj, cpi);
                mlo = shift_in(mlo, cur.z);
                mhi = shift_in(mhi, cur.w);
                prev = cur;
            }
        }
        status = uni(status);
        phase_sync();

        // ------------------------------------------------------------ C0: word costs and validity
        // the word ending at e (a word start, or na) has its final key at e-1 (or in last_key)
        auto word_key = [&](unsigned e) -> uint64_t {
            return e < na ? (((uint64_t)(uint32_t)S.stg[e - 1] << 32) | S.rec[e - 1].w) : last_key;
        };
        auto key_cost = [](uint64_t k) -> unsigned {   // 65535: the uncapped "inf" (inspect_tokenizer.py:80)
            const unsigned c = (unsigned)(k >> 32);
            return c >= 0xFFFFFFFEu ? 0xFFFFu : c;
        };
        unsigned total = 0, capsum = 0;
        bool inval = false;
        for (unsigned e0 = 1; e0 <= na; e0 += 64) {
            const unsigned e = e0 + lane;
            unsigned c = 0;
            bool iv = false;
            if (e <= na && S.wstart(e)) {
                const uint64_t k = word_key(e);
                c = key_cost(k);
                iv = ((k >> 31) & 1u) != 0;
            }
            capsum += wave_sum(c);
            inval |= ballot(iv) != 0;
        }
        if (status == 0 && inval) status = 1;
        total = capsum;

        // ------------------------------------------------------------ C1: selection, one lane per word
        if (status == 0 && !len_only) {
            unsigned carry = 0;
            for (unsigned e0 = 1; e0 <= na; e0 += 64) {
                const unsigned e = e0 + lane;
                const bool mine = e <= na && S.wstart(e);
                const uint64_t k = mine ? word_key(e) : 0ull;
                const unsigned cost = mine ? (unsigned)(k >> 32) : 0u;
                const unsigned incl = incl_scan_add(cost);
                const unsigned kbase = carry + incl - cost;   // tokens of the words before this one
                carry += __builtin_amdgcn_readlane(incl, 63);
                if (mine) {
                    const unsigned Ls = 0x7FFFFFFFu - (unsigned)(k & 0x7FFFFFFFu);
                    unsigned i = e, c = cost, A = 0;
                    unsigned pend = S.cpb(e);
                    while (c > 0) {
                        const unsigned f = S.rec[i - 1].z;
                        const unsigned cpi = S.cpb(i);
                        const unsigned sp = (pend - cpi) & CPM;
                        A = A > sp ? A : sp;
                        const unsigned dd = A < Ls ? (f & 0xFFFFu) : (f >> 16);
                        const unsigned j = i - 1 - dd;
                        c--;
                        S.stg[kbase + c] = (int32_t)j;   // below e: only this word's and earlier words' keys live there
                        pend = cpi;
                        i = j;
                    }
                }
            }
            phase_sync();

            // -------------------------------------------------------- C2: ids, 64 tokens at a time
            for (unsigned k0 = 0; k0 < total; k0 += 64) {
                const unsigned k = k0 + lane;
                const bool in = k < total;
                unsigned at = 0, j1 = 0;
                if (in) {
                    at = (unsigned)S.stg[k];
                    j1 = k + 1 < total ? (unsigned)S.stg[k + 1] : na;
                }
                __builtin_amdgcn_wave_barrier();   // every start of this batch is read before any id lands
                int32_t node = 0, nb = a.root_base, id = -1;
                bool ok = true, active = in && at < j1;
                Cursor c;
                if (active) c.load(S, at);
                while (ballot(active)) {
                    if (active) {
                        const int32_t t = nb + (int32_t)c.next(S);
                        const int4 ent = trie_slot4(a, t);
                        ok &= ent.y == node;
                        node = t;
                        nb = ent.x & BASE_MASK;
                        id = ent.z;
                        if (!ok) active = false;
                        else if (c.at_end()) {
                            if (++at == j1) active = false;
                            else c.load(S, at);
                        }
                    }
                }
                phase_sync();
                if (in) {
                    if (a.staging16) a.staging16[sb + k] = (int16_t)(ok ? id : -1);
                    else a.staging[sb + k] = ok ? id : -1;
                }
            }
        }
        if (lane == 0) {
            a.status[s] = (int32_t)status;
            a.counts[s] = (status == 0 && !len_only) ? (uint64_t)total : 0ull;
            if (a.bsum && status == 0 && !len_only && total) atomicAdd(&a.bsum[(s / FIN_BATCH) * BS_LINE], (unsigned long long)total);
            if (a.capped) a.capped[s] = status == 3 ? -1 : (int32_t)capsum;
        }
        phase_sync();
    }
}

// the unbounded pass's arguments from a LongLaunch (fallback_kernel's unbounded-pass blocks)
inline Args long_args(const LongLaunch &p) {
    Args a;
    a.text = p.text; a.str_off = p.str_off; a.cut_mask = p.cut_mask;
    a.staging = p.staging; a.staging16 = p.staging16; a.counts = p.counts; a.bsum = p.bsum; a.status = p.status; a.capped = p.capped;
    // (a test-only arena_bias B: the counter starts at B, so offset ao addresses element ao - B; the
    // pointers are shifted by B elements, the capacity raised by B -- dpt_ctx_debug_counter_bias)
    a.rec = reinterpret_cast<uint4 *>(reinterpret_cast<uintptr_t>(p.arena) - 16 * p.arena_bias);
    a.stg = reinterpret_cast<int32_t *>(reinterpret_cast<uintptr_t>(p.arena + 16 * p.arena_cap) - 4 * p.arena_bias);
    a.arena_cap = p.arena_cap + p.arena_bias;
    a.arena_used = p.arena_used;
    a.edges = p.edges; a.far = p.far; a.far_cap = p.far_cap; a.far_count = p.far_count; a.list = p.list; a.list_count = p.list_count; a.work_next = p.work_next;
    a.slots = p.slots; a.slots4 = p.slots4; a.n_slots = p.n_slots; a.root_base = p.root_base;
    a.max_tok_bytes = p.max_tok_bytes; a.long_span = p.long_span; a.mode = p.mode;
    return a;
}

}  // namespace lng

}  // namespace dpt
