// dpt_lane.hip -- lane-per-string shortest-tokenization kernel for vocabularies whose
// tokens have at most 16 code points (Llama-2 and the synthetic Llama-shaped vocab).
//
// Each of the 64 lanes of a wave owns one string and runs the whole DP for it, in
// lockstep with the other lanes (one atom per step).  Nothing is staged in LDS, so
// occupancy is set by registers (16 waves/CU x 64 strings in flight per CU).
//
// Forward pass, one atom per step:
//   * the atom is read from the input and expanded on the fly like pretokenize_raw
//     (reference packages/tokenizer_utils.py:33-50): '▁'+c first, ' ' -> '▁' opening a
//     word, '\n' -> '<0x0A>', any other code point as itself (DPT_MODE_PRESPLIT: code
//     points, words from the cut mask);
//   * a ring of 16 trie walks (one started at each of the last 16 atoms, registers,
//     static ring slots thanks to a 16x unrolled step) is advanced through the double-
//     array trie by the atom's bytes; a walk that sits on a terminal after the atom is a
//     token span(j, i) ("join(atoms[j:i]) in vocabulary", dp_tokenize.py:39);
//   * each candidate forms the key (cost[j]+1)<<16 | invalid[j]<<15 | (0x7FFF - max(G[j],
//     cp(span))); the min with the cap key (i - word start)<<16 | 0xFFFF
//     (len_dp = range(n+1), dp_tokenize.py:28) gives cost[i], reachability and G[i];
//   * the smallest back-distance attaining the min (gm) and the smallest one in E(i)
//     that is reachable (em) go to an 8-byte per-atom record in global scratch together
//     with the atom's byte offset and code-point prefix.
// Backtrace, one token per step, right to left: take gm while the longest token so far
// is below the word's G, em once it is reached -- the first argmax of
// obtain_longest_token in the reference's DFS order (dp_tokenize.py:58, :84).  The id of
// each selected span is found by re-walking its bytes (tokenizer_utils.py:76-79).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dpt_internal.h"

namespace dpt {

namespace lane {

#ifdef DPT_STAMPS
__device__ unsigned long long g_lane_stamps[4];
#endif

constexpr int RING = 16;
#ifndef LANE_WAVES_PER_EU
#define LANE_WAVES_PER_EU 4
#endif

struct Args {
    const uint8_t *text;
    const uint64_t *str_off;
    const uint8_t *cut_mask;
    uint64_t n_str;
    int32_t *staging;       // ids at (str_off[s]-str_off[0]) + k
    uint4 *rec;             // per-atom backtrace records at (str_off[s]-str_off[0]) + i - 1
    uint64_t *counts;
    int32_t *status;
    int32_t *capped;
    uint32_t *retry_list;
    uint32_t *retry_count;
    const int2 *__restrict__ slots;    // {base | TERM<<31, check}
    const int32_t *__restrict__ ids;   // token id of a terminal slot
    uint32_t n_slots;
    int32_t root_base;
    int mode;
};

// trie slot t as {base word, check} through a buffer descriptor (32-bit offsets: fewer VGPRs
// than 64-bit flat addresses with 16 walks in flight)
__device__ __forceinline__ int2 load_slot(__amdgpu_buffer_rsrc_t r, int32_t t) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (unsigned)t * 8u, 0, 0);
    return make_int2((int32_t)v[0], (int32_t)v[1]);
}

// One atom at byte p of a string of length n: its expanded UTF-8 bytes (little-endian in
// `eb`, `ne` of them), its input byte length and its code-point length.
struct Atom {
    uint64_t eb;
    unsigned ne, la, cp;
};

__device__ __forceinline__ unsigned utf8_len(unsigned b) {
    return b < 0xC0u ? 1u : (b < 0xE0u ? 2u : (b < 0xF0u ? 3u : 4u));
}

__device__ __forceinline__ Atom load_atom(const uint8_t *str, uint64_t p, uint64_t n, unsigned b, bool raw) {
    Atom a;
    unsigned la = utf8_len(b);
    uint64_t chars = b;
    // continuation bytes (a truncated / invalid sequence ends at the first non-continuation byte)
    unsigned k = 1;
    for (; k < la; k++) {
        if (p + k >= n) break;
        const unsigned c = str[p + k];
        if ((c & 0xC0u) != 0x80u) break;
        chars |= (uint64_t)c << (8 * k);
    }
    la = k;
    if (raw && p == 0) {
        a.eb = 0x8196E2ull | (chars << 24);  // '▁' + first character
        a.ne = 3 + la;
        a.cp = 2;
    } else if (raw && b == ' ') {
        a.eb = 0x8196E2ull;                  // '▁'
        a.ne = 3;
        a.cp = 1;
    } else if (raw && b == '\n') {
        a.eb = 0x3E413078303Cull;            // "<0x0A>"
        a.ne = 6;
        a.cp = 6;
    } else {
        a.eb = chars;
        a.ne = la;
        a.cp = 1;
    }
    a.la = la;
    return a;
}

// record of end position i (16 B): {trie slot of the gm token, slot of the em token, byte
// offset of the atom end, cpos (16) | gm distance (4) | em distance (4) | word end (1) | word G (5)}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LANE_WAVES_PER_EU, 8)))
lane_kernel(Args a) {
    const unsigned lane = threadIdx.x;
    const uint64_t base_off = a.str_off[0];
    const bool raw = a.mode == 0;
    const int32_t root_base = a.root_base;
    const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc((void *)a.slots, (short)0, (int)(a.n_slots * 8u), 0x00020000);

    for (uint64_t s0 = (uint64_t)blockIdx.x * 64; s0 < a.n_str; s0 += (uint64_t)gridDim.x * 64) {
        const uint64_t s = s0 + lane;
        const bool have = s < a.n_str;
        const uint64_t sb = have ? a.str_off[s] - base_off : 0;
        const uint64_t n = have ? a.str_off[s + 1] - a.str_off[s] : 0;
        const uint8_t *str = a.text + sb;
        const uint8_t *cut = raw ? nullptr : a.cut_mask + sb;
        uint4 *rec = a.rec + sb;
        bool too_long = n > 0xFFFF0000ull;   // record offsets are 32-bit

#ifdef DPT_STAMPS
        const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
        // ------------------------------------------------------------------ forward pass
        // ring slot k: the walk started at the atom whose index is = k (mod 16)
        //   node[k] current trie slot (-1 = dead); nb[k] its raw base word (bit 31: a token ends
        //   here); st[k] = (cost[j]+1)<<16 | invalid[j]<<15 | cp(span so far)<<5 | G[j] for the
        //   walk's start j
        int32_t node[RING], nb[RING];
        unsigned st[RING];
#pragma unroll
        for (int k = 0; k < RING; k++) { node[k] = -1; nb[k] = 0; st[k] = 0; }
        uint64_t p = 0;
        unsigned i = 0, ws = 0, cpos = 0;
        unsigned stp = 0x10000u;            // state at the current position: word start
        unsigned tokens = 0, capsum = 0, invalid = 0;
        unsigned b = (have && n > 0) ? str[0] : 0;
        bool active = have && n > 0 && !too_long;

        for (;;) {
#pragma unroll
            for (int kc = 0; kc < RING; kc++) {
                if (!__builtin_amdgcn_ballot_w64(active)) break;
                const Atom at = load_atom(str, p, n, b, raw);
                const uint64_t pe = p + at.la;
                // start the walk for this atom
                if (active) { node[kc] = 0; nb[kc] = root_base; st[kc] = stp; }
                // advance every live walk over the atom's expanded bytes: first issue the loads of
                // all live walks (exec-masked: only live lanes touch memory), then consume them
                for (unsigned e = 0; __builtin_amdgcn_ballot_w64(active && e < at.ne); e++) {
                    const bool le = active && e < at.ne;
                    const int32_t byte = (int32_t)((at.eb >> (8 * (e & 7))) & 0xFFu);
                    int32_t t[RING];
                    int2 ent[RING];
#pragma unroll
                    for (int k = 0; k < RING; k++) {
                        t[k] = (nb[k] & 0x3FFFFFFF) + byte;   // bits 31/30: terminal / leaf
                        if (le && node[k] >= 0) ent[k] = load_slot(srd, t[k]);
                    }
#pragma unroll
                    for (int k = 0; k < RING; k++) {
                        if (le && node[k] >= 0) {
                            node[k] = ent[k].y == node[k] ? t[k] : -1;
                            nb[k] = ent[k].x;
                        }
                    }
                }
                if (active) {
                    const unsigned cpe = cpos + at.cp;
                    // candidates in order of increasing back-distance d (ring slot (kc - d) & 15):
                    // r = min key (cap included); gm = smallest d attaining r; em = smallest d in
                    // r's (cost, validity) class -- the class only ever improves as d grows.
                    unsigned r = ((i + 1 - ws) << 16) | 0xFFFFu;   // cap: len_dp[i] = i
                    unsigned gm = 0, em = 0;
                    int32_t id_gm = -1, id_em = -1;
#pragma unroll
                    for (int dd = 0; dd < RING; dd++) {
                        const int k = (kc - dd) & (RING - 1);
                        st[k] += at.cp << 5;                      // cp of the span grows by this atom
                        const unsigned gj = st[k] & 31u;
                        const unsigned span = (st[k] >> 5) & 0x3FFu;
                        const unsigned kv = (st[k] | 0x7FFFu) - (gj > span ? gj : span);
                        const unsigned key = (node[k] >= 0 && nb[k] < 0) ? kv : 0xFFFFFFFFu;
                        const bool better = key < r;
                        const bool cls = better && (key ^ r) >= 0x8000u;
                        em = cls ? (unsigned)dd : em;
                        id_em = cls ? node[k] : id_em;
                        gm = better ? (unsigned)dd : gm;
                        id_gm = better ? node[k] : id_gm;
                        r = better ? key : r;
                    }
                    // does a new word start after this atom?
                    unsigned bn = 0;
                    bool wend = pe >= n;
                    if (!wend) {
                        bn = str[pe];
                        wend = raw ? (bn == ' ') : (cut[pe] != 0 && (bn & 0xC0u) != 0x80u);
                    }
                    unsigned L = 0;
                    if (wend) {
                        capsum += r >> 16;
                        tokens += r >> 16;
                        invalid |= r & 0x8000u;
                        L = 0x7FFFu - (r & 0x7FFFu);
                    }
                    rec[i] = make_uint4((unsigned)id_gm, (unsigned)id_em, (unsigned)pe,
                                        (cpe & 0xFFFFu) | (gm << 16) | (em << 20) | ((wend ? 1u : 0u) << 24) | ((L & 31u) << 25));
                    stp = (r ^ 0x7FFFu) + 0x10000u;
                    if (wend) {
#pragma unroll
                        for (int k = 0; k < RING; k++) node[k] = -1;
                        stp = 0x10000u;
                        ws = i + 1;
                    }
                    p = pe;
                    i++;
                    cpos = cpe;
                    b = bn;
                    active = pe < n;
                }
            }
            if (!__builtin_amdgcn_ballot_w64(active)) break;
        }

#ifdef DPT_STAMPS
        const unsigned long long t_fw = __builtin_amdgcn_s_memtime();
#endif
        // ------------------------------------------------------------------ backtrace
        unsigned status = !have ? 0u : (n == 0 ? 2u : (too_long ? 3u : (invalid ? 1u : 0u)));
        bool bt = have && status == 0;
        unsigned k_out = tokens;
        unsigned ic = i;                     // current end (atom index)
        uint4 R = bt ? rec[ic - 1] : make_uint4(0, 0, 0, 0);
        unsigned A = 0, Lw = 0;
        int32_t *out = a.staging + sb;
        while (__builtin_amdgcn_ballot_w64(bt)) {
            if (bt) {
                if ((R.w >> 24) & 1u) { A = 0; Lw = (R.w >> 25) & 31u; }
                const bool use_gm = A < Lw;
                const unsigned dsel = use_gm ? (R.w >> 16) & 15u : (R.w >> 20) & 15u;
                const int32_t slot = (int32_t)(use_gm ? R.x : R.y);
                const int32_t id = slot >= 0 ? a.ids[slot] : -1;
                const unsigned j = ic - 1 - dsel;
                const uint4 Rj = j > 0 ? rec[j - 1] : make_uint4(0, 0, 0, 0);
                const unsigned cp = ((R.w & 0xFFFFu) - (Rj.w & 0xFFFFu)) & 0xFFFFu;
                A = A > cp ? A : cp;
                k_out--;
                out[k_out] = id;
                if (id < 0) status = 4;
                ic = j;
                R = Rj;
                bt = j > 0 && k_out > 0;
            }
        }
        if (have) {
            if (status == 0 && (k_out != 0 || ic != 0)) status = 4;
            if (status == 3) {
                const unsigned slot = atomicAdd(a.retry_count, 1u);
                a.retry_list[slot] = (uint32_t)s;
            }
            a.status[s] = (int32_t)status;
            a.counts[s] = status == 0 ? (uint64_t)tokens : 0ull;
            if (a.capped) a.capped[s] = status == 2 ? 0 : (status == 3 ? -1 : (int32_t)capsum);
        }
#ifdef DPT_STAMPS
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            atomicAdd(&g_lane_stamps[0], t_fw - t_start);
            atomicAdd(&g_lane_stamps[1], t_end - t_fw);
            atomicAdd(&g_lane_stamps[2], 1ull);
        }
#endif
    }
}

}  // namespace lane

#ifdef DPT_STAMPS
extern "C" int dpt_debug_lane_stamps(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lane::g_lane_stamps), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[4] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(lane::g_lane_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

void launch_lane(const EncodeLaunch &p, unsigned blocks, hipStream_t stream) {
    lane::Args a;
    a.text = p.text; a.str_off = p.str_off; a.cut_mask = p.cut_mask; a.n_str = p.n_str;
    a.staging = p.staging; a.rec = p.rec; a.counts = p.counts; a.status = p.status; a.capped = p.capped;
    a.retry_list = p.retry_list; a.retry_count = p.retry_count;
    a.slots = p.slots; a.ids = p.slot_ids; a.n_slots = p.n_slots; a.root_base = p.root_base; a.mode = p.mode;
    hipLaunchKernelGGL(lane::lane_kernel, dim3(blocks), dim3(64), 0, stream, a);
}

}  // namespace dpt
