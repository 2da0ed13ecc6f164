// dpt_kernels.hip -- CDNA4 (gfx950) kernels of the shortest-tokenization engine.
//
// One input string per wavefront (64 lanes).  Per window of <= CH input bytes
// (windows end at word boundaries; words are independent DP problems,
// reference packages/tokenizer_utils.py:70):
//
//   prep   atomise the window like pretokenize_raw (tokenizer_utils.py:33-50) into
//          an atom-expanded UTF-8 byte string in LDS ('▁'+c first, ' '->'▁',
//          '\n'->'<0x0A>'), with atom/word-end tags, atom offsets, code-point
//          prefix sums (cp(span) = cpos[i]-cpos[j], the len(t) of dp_tokenize.py:82)
//          and the word-start list -- two packed DPP wave scans.
//   A      match discovery: lanes walk the byte double-array trie (L2-resident)
//          from every atom start; a bit (L-1) of smask[j] records that the L-atom
//          span from atom j is a vocabulary token ("join(atoms[j:i]) in vocabulary",
//          dp_tokenize.py:39).  Lanes that finish pick up the next start (ballot +
//          mbcnt), so the wave stays busy.
//   B      forward recurrence, sequential over end positions i with lanes = back
//          distances d (j = i-1-d): per lane one 32-bit key
//              (cost[j]+1) << 16 | invalid[j] << 15 | (0x7FFF - max(G[j], cp(span)))
//          and ONE DPP wave-min gives cost[i] (capped at the atom index within the
//          word, dp_tokenize.py:28), reachability and the max-of-max token length
//          G[i].  The per-lane state (state, cpos,
//          smask of j) is shifted one lane per step with DPP wave_shr:1 -- no LDS
//          traffic on the critical path.
//   C1     selection: per word, right to left, lanes = back distances, ballot of
//          "j in E(i), valid, max(A, cp, G[j]) == G[n]", the LOWEST set lane is
//          the LARGEST j -- the reference's first argmax in DFS order
//          (dp_tokenize.py:58 pops the largest j first, :84 takes the first max).
//   C2     id resolution: lanes re-walk each selected span through the trie and
//          write t2i[token] (tokenizer_utils.py:76-79) to a staging row.
//
// A separate scan + compaction turns the staging rows into CSR ids.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "dpt_internal.h"

namespace dpt {

// ------------------------------------------------------------------ wave primitives

__device__ __forceinline__ unsigned lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// inclusive add-scan over 64 lanes (GFX9 DPP: row_shr 1/2/4/8, row_bcast 15/31)
__device__ __forceinline__ unsigned wave_incl_scan_add(unsigned v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false); // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false); // row_bcast:31
    return v;
}

// min over 64 lanes, result uniform (SGPR)
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false)); // row_half_mirror
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false)); // row_mirror
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false)); // row_bcast:15
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false)); // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// lane l receives x[l-1]; lane 0 receives `in` (DPP wave_shr:1, bound_ctrl off)
__device__ __forceinline__ unsigned shift_in(unsigned x, unsigned in) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)in, (int)x, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ unsigned uni(unsigned x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// ------------------------------------------------------------------ LDS layout

// tags on the LAST expanded byte of an atom
constexpr uint8_t TAG_ATOM_END = 1;
constexpr uint8_t TAG_WORD_END = 2;

constexpr unsigned ST_VALID = 0x8000u;
constexpr unsigned ST_RESET = ST_VALID;   // cost 0, reachable, G 0
constexpr unsigned MAXD = 64;             // longest span in atoms (vocab max_cp <= 64 enforced on the host)

template <int CH>
struct WaveLDS {
    static constexpr int NA = CH + 2;            // atoms + sentinel
    static constexpr int NE = 6 * CH + 8;        // expanded bytes ('\n' -> 6 bytes; first atom +3)
    uint64_t smask[NA];
    uint32_t state[NA];
    uint32_t tok[NA];
    uint32_t wfin[NA];
    uint16_t aoff[NA];
    uint16_t cpos[NA];
    uint16_t wsl[NA];
    uint8_t ebyte[NE];
    uint8_t etag[NE];
};

template <int CH>
constexpr int wave_lds_bytes() { return (int)((sizeof(WaveLDS<CH>) + 15) & ~size_t(15)); }

// ------------------------------------------------------------------ trie access

struct TrieView {
    const int2 *__restrict__ slots;   // .x = base | TERM<<31, .y = check (parent slot, -1 free)
    const int32_t *__restrict__ ids;  // token id of a terminal slot
    int32_t root_base;
};

constexpr int32_t TERM_BIT = (int32_t)0x80000000;

// ------------------------------------------------------------------ the tokenize kernel

struct EncodeArgs {
    const uint8_t *text;
    const uint64_t *str_off;
    const uint8_t *cut_mask;    // PRESPLIT only
    uint64_t n_str;
    uint64_t base_off;          // str_off[0] (read on device)
    int32_t *staging;           // ids staged at (str_off[s]-str_off[0]) + k
    uint64_t *counts;           // per string
    int32_t *status;
    int32_t *capped;            // nullable
    uint32_t *retry_list;       // strings that overflowed the window (status TOO_LONG) for the big pass
    uint32_t *retry_count;
    const uint32_t *work_list;  // big pass: list of string indices (nullable => all strings)
    const uint32_t *work_count;
    int mode;
};

template <int CH, int WPB, bool BIG>
__global__ void __launch_bounds__(WPB * 64)
tokenize_kernel(EncodeArgs a, TrieView tv) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const unsigned wid = threadIdx.x >> 6;
    const unsigned lane = lane_id();
    WaveLDS<CH> &L = *reinterpret_cast<WaveLDS<CH> *>(smem + wid * wave_lds_bytes<CH>());

    const uint64_t n_work = BIG ? (uint64_t)(*a.work_count) : a.n_str;
    const uint64_t wave_global = (uint64_t)blockIdx.x * WPB + wid;
    const uint64_t wave_stride = (uint64_t)gridDim.x * WPB;
    const uint64_t base_off = a.str_off[0];
    const bool raw = a.mode == 0;

    for (uint64_t w = wave_global; w < n_work; w += wave_stride) {
        const uint64_t s = BIG ? (uint64_t)a.work_list[w] : w;
        const uint64_t sb = a.str_off[s] - base_off;
        const uint64_t slen = a.str_off[s + 1] - a.str_off[s];
        const uint8_t *str = a.text + sb;
        const uint8_t *cut = raw ? nullptr : a.cut_mask + sb;
        int32_t *out = a.staging + sb;

        unsigned status = 0;
        unsigned ntok = 0;        // ids emitted so far
        unsigned capsum = 0;      // sum of capped word lengths
        bool capped_known = true;
        if (slen == 0) status = 2;  // pretokenize_raw('') == [[]] -> IndexError

        uint64_t pos = 0;
        while (status != 2 && status != 3 && pos < slen) {
            // ---------------------------------------------------------- window bounds
            const uint64_t rem = slen - pos;
            unsigned wlen;
            if (rem <= (uint64_t)CH) {
                wlen = (unsigned)rem;
            } else {
                // last word start q in [1, CH]: the window is [pos, pos+q)
                int best = -1;
                for (int k = lane; k <= CH; k += 64) {
                    if (k == 0) continue;
                    const uint64_t p = pos + k;
                    const uint8_t b = str[p];
                    bool ws = raw ? (b == ' ') : (cut[p] != 0 && (b & 0xC0) != 0x80);
                    if (ws) best = k;
                }
                const unsigned q = wave_max_u32((unsigned)(best + 1));
                if (q == 0) { status = 3; break; }  // one word longer than the window
                wlen = q - 1;
            }

            // ---------------------------------------------------------- prep: atomise
            // lane l owns bytes 4l..4l+3 of each 256-byte chunk of the window
            unsigned n_atoms = 0, n_ex = 0, cp_tot = 0, n_words = 0;
            for (unsigned c0 = 0; c0 < wlen; c0 += 256) {
                uint8_t bt[4];
                unsigned exl[4], cpl[4];
                bool ast[4], wst[4];
                unsigned ex_sum = 0, cp_sum = 0, a_sum = 0, w_sum = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const unsigned k = c0 + lane * 4 + u;
                    const bool in = k < wlen;
                    const uint64_t p = pos + k;
                    const uint8_t b = in ? str[p] : 0;
                    const bool first = in && p == 0;
                    const bool cont = in && !first && (b & 0xC0) == 0x80;
                    const bool as = in && !cont;
                    bool wsf;
                    unsigned el, cl;
                    if (raw) {
                        wsf = as && (k == 0 || b == ' ');
                        el = !in ? 0 : first ? 4 : (b == ' ' ? 3 : (b == '\n' ? 6 : 1));
                        cl = !in ? 0 : first ? 2 : (b == '\n' ? 6 : (cont ? 0 : 1));
                    } else {
                        wsf = as && (k == 0 || cut[p] != 0);
                        el = in ? 1 : 0;
                        cl = as ? 1 : 0;
                    }
                    bt[u] = b; exl[u] = el; cpl[u] = cl; ast[u] = as; wst[u] = wsf;
                    ex_sum += el; cp_sum += cl; a_sum += as; w_sum += wsf;
                }
                // packed scans: (ex | cp<<16), (atoms | words<<16); all fields < 65536
                const unsigned v1 = ex_sum | (cp_sum << 16);
                const unsigned v2 = a_sum | (w_sum << 16);
                const unsigned i1 = wave_incl_scan_add(v1);
                const unsigned i2 = wave_incl_scan_add(v2);
                const unsigned t1 = __builtin_amdgcn_readlane(i1, 63);
                const unsigned t2 = __builtin_amdgcn_readlane(i2, 63);
                unsigned ex = n_ex + ((i1 - v1) & 0xFFFF);
                unsigned cp = cp_tot + ((i1 - v1) >> 16);
                unsigned ai = n_atoms + ((i2 - v2) & 0xFFFF);
                unsigned wi = n_words + ((i2 - v2) >> 16);
                // does the byte after each of mine start an atom / word?
                const unsigned my_first_flags = (ast[0] ? 1u : 0u) | (wst[0] ? 2u : 0u);
                unsigned next_flags = (unsigned)__shfl_down((int)my_first_flags, 1);
                if (lane == 63) next_flags = 0;
                // the next chunk's first byte (crossing a 256-byte chunk inside the window)
                const unsigned kn = c0 + 256;
                unsigned chunk_next = 3;  // end of window: atom end + word end
                if (kn < wlen) {
                    const uint64_t p = pos + kn;
                    const uint8_t b = str[p];
                    const bool as = (b & 0xC0) != 0x80;
                    const bool wsf = as && (raw ? b == ' ' : cut[p] != 0);
                    chunk_next = (as ? 1u : 0u) | (wsf ? 2u : 0u);
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const unsigned k = c0 + lane * 4 + u;
                    if (k >= wlen) break;
                    const uint64_t p = pos + k;
                    unsigned nf;
                    if (k + 1 >= wlen) nf = 3;
                    else if (u < 3) nf = (ast[u + 1] ? 1u : 0u) | (wst[u + 1] ? 2u : 0u);
                    else nf = (lane == 63) ? chunk_next : next_flags;
                    if (ast[u]) {
                        L.aoff[ai] = (uint16_t)ex;
                        L.cpos[ai] = (uint16_t)cp;
                        if (wst[u]) { L.wsl[wi] = (uint16_t)ai; wi++; }
                        ai++;
                    }
                    const uint8_t b = bt[u];
                    if (raw && p == 0) {
                        L.ebyte[ex] = 0xE2; L.ebyte[ex + 1] = 0x96; L.ebyte[ex + 2] = 0x81; L.ebyte[ex + 3] = b;
                        L.etag[ex] = 0; L.etag[ex + 1] = 0; L.etag[ex + 2] = 0;
                        ex += 3;
                    } else if (raw && b == ' ') {
                        L.ebyte[ex] = 0xE2; L.ebyte[ex + 1] = 0x96; L.ebyte[ex + 2] = 0x81;
                        L.etag[ex] = 0; L.etag[ex + 1] = 0;
                        ex += 2;
                    } else if (raw && b == '\n') {
                        L.ebyte[ex] = '<'; L.ebyte[ex + 1] = '0'; L.ebyte[ex + 2] = 'x';
                        L.ebyte[ex + 3] = '0'; L.ebyte[ex + 4] = 'A'; L.ebyte[ex + 5] = '>';
                        L.etag[ex] = 0; L.etag[ex + 1] = 0; L.etag[ex + 2] = 0; L.etag[ex + 3] = 0; L.etag[ex + 4] = 0;
                        ex += 5;
                    } else {
                        L.ebyte[ex] = b;
                    }
                    // tag of the last expanded byte of byte k
                    L.etag[ex] = (uint8_t)(((nf & 1) ? TAG_ATOM_END : 0) | ((nf & 2) ? TAG_WORD_END : 0));
                    ex++;
                    cp += cpl[u];
                }
                n_ex += t1 & 0xFFFF; cp_tot += t1 >> 16;
                n_atoms += t2 & 0xFFFF; n_words += t2 >> 16;
            }
            if (lane == 0) {
                L.aoff[n_atoms] = (uint16_t)n_ex;
                L.cpos[n_atoms] = (uint16_t)cp_tot;
                L.wsl[n_words] = (uint16_t)n_atoms;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // ---------------------------------------------------------- A: match discovery
            {
                unsigned j = lane;
                unsigned e = j < n_atoms ? L.aoff[j] : 0;
                int32_t nb = tv.root_base;     // base of the current node
                int32_t node = 0;              // current slot (root = 0)
                unsigned len = 0;
                uint64_t mask = 0;
                unsigned next = 64;
                bool active = j < n_atoms;
                while (ballot(active)) {
                    bool done = false;
                    if (active) {
                        const uint8_t b = L.ebyte[e];
                        const uint8_t tg = L.etag[e];
                        const int32_t t = nb + (int32_t)b;
                        const int2 ent = tv.slots[t];
                        if (ent.y != node) {
                            done = true;
                        } else {
                            node = t;
                            nb = ent.x & 0x7FFFFFFF;
                            e++;
                            if (tg & TAG_ATOM_END) {
                                len++;
                                if (ent.x & TERM_BIT) mask |= 1ull << (len - 1);
                                if ((tg & TAG_WORD_END) || len == MAXD) done = true;
                            }
                        }
                    }
                    const uint64_t dm = ballot(done);
                    if (done) {
                        L.smask[j] = mask;
                        const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(dm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)dm, 0u));
                        j = next + rank;
                        active = j < n_atoms;
                        if (active) { e = L.aoff[j]; nb = tv.root_base; node = 0; len = 0; mask = 0; }
                    }
                    next += (unsigned)__builtin_popcountll(dm);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // ---------------------------------------------------------- B: forward recurrence
            {
                unsigned st = 0, cpj = 0, mlo = 0, mhi = 0;
                // position 0 (the first word start) enters lane 0
                {
                    const uint64_t m0 = L.smask[0];
                    st = shift_in(st, ST_RESET);
                    cpj = shift_in(cpj, 0u);
                    mlo = shift_in(mlo, uni((unsigned)m0));
                    mhi = shift_in(mhi, uni((unsigned)(m0 >> 32)));
                }
                if (lane == 0) L.state[0] = ST_RESET;
                unsigned wcur = 0, ws = 0;
                unsigned next_ws = n_words > 1 ? uni(L.wsl[1]) : n_atoms;
                const unsigned d = lane;
                for (unsigned i0 = 1; i0 <= n_atoms; i0 += 64) {
                    // preload the uniform per-position inputs of 64 steps
                    const unsigned pi = i0 + lane;
                    const unsigned pcp = pi <= n_atoms ? L.cpos[pi] : 0u;
                    const uint64_t pm = pi < n_atoms ? L.smask[pi] : 0ull;
                    const unsigned pml = (unsigned)pm, pmh = (unsigned)(pm >> 32);
                    const unsigned iend = min(n_atoms, i0 + 63);
                    for (unsigned i = i0; i <= iend; i++) {
                        const unsigned k = i - i0;
                        const unsigned cpi = __builtin_amdgcn_readlane(pcp, k);
                        const unsigned bit = (d < 32 ? (mlo >> d) : (mhi >> (d - 32))) & 1u;
                        const unsigned span = cpi - cpj;
                        const unsigned gj = st & 0x7FFFu;
                        const unsigned g = gj > span ? gj : span;
                        const unsigned key = bit ? ((((st >> 16) + 1u) << 16) | ((st & ST_VALID) ^ ST_VALID) | (0x7FFFu - g))
                                                 : 0xFFFFFFFFu;
                        unsigned r = wave_min_u32(key);
                        const unsigned capkey = ((i - ws) << 16) | 0xFFFFu;
                        r = r < capkey ? r : capkey;
                        const bool v = (r & ST_VALID) == 0;
                        const unsigned si = (r & 0xFFFF0000u) | (v ? (ST_VALID | (0x7FFFu - (r & 0x7FFFu))) : 0u);
                        unsigned sin = si;
                        if (i == next_ws && i < n_atoms) {
                            if (lane == 0) L.wfin[wcur] = si;
                            wcur++;
                            ws = i;
                            next_ws = (wcur + 1 < n_words) ? uni(L.wsl[wcur + 1]) : n_atoms;
                            sin = ST_RESET;
                        }
                        if (i == n_atoms && lane == 0) L.wfin[wcur] = si;
                        if (lane == 0) L.state[i] = sin;
                        st = shift_in(st, sin);
                        cpj = shift_in(cpj, cpi);
                        mlo = shift_in(mlo, __builtin_amdgcn_readlane(pml, k));
                        mhi = shift_in(mhi, __builtin_amdgcn_readlane(pmh, k));
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // ---------------------------------------------------------- C1: selection
            unsigned wtok = 0;   // tokens of this window
            for (unsigned w = 0; w < n_words; w++) {
                const unsigned F = uni(L.wfin[w]);
                capsum += F >> 16;
                if (status) continue;                 // keep summing capped lengths only
                if (!(F & ST_VALID)) { status = 1; continue; }
                const unsigned ws = uni(L.wsl[w]);
                unsigned i = uni(L.wsl[w + 1]);
                unsigned c = F >> 16;
                const unsigned Ls = F & 0x7FFFu;
                unsigned A = 0;
                unsigned cpi = uni(L.cpos[i]);
                const unsigned base = wtok;
                while (i > ws) {
                    const unsigned d = lane;
                    const int j = (int)i - 1 - (int)d;
                    bool cond = false;
                    unsigned cj = 0;
                    if (j >= (int)ws && d < MAXD) {
                        const uint64_t m = L.smask[j];
                        const unsigned sj = L.state[j];
                        cj = L.cpos[j];
                        const unsigned span = cpi - cj;
                        unsigned mx = A > span ? A : span;
                        const unsigned gj = sj & 0x7FFFu;
                        mx = mx > gj ? mx : gj;
                        cond = ((m >> d) & 1ull) && (sj >> 16) + 1u == c && (sj & ST_VALID) && mx == Ls;
                    }
                    const uint64_t bal = ballot(cond);
                    if (bal == 0) { status = 4; break; }
                    const unsigned dd = (unsigned)__builtin_ctzll(bal);
                    const unsigned jj = i - 1 - dd;
                    const unsigned cjj = __builtin_amdgcn_readlane(cj, dd);
                    c--;
                    if (lane == 0) L.tok[base + c] = jj | (i << 16);
                    const unsigned span = cpi - cjj;
                    A = A > span ? A : span;
                    i = jj;
                    cpi = cjj;
                }
                if (!status) wtok += F >> 16;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // ---------------------------------------------------------- C2: ids
            if (!status) {
                for (unsigned t = lane; t < wtok; t += 64) {
                    const unsigned ji = L.tok[t];
                    const unsigned e0 = L.aoff[ji & 0xFFFF], e1 = L.aoff[ji >> 16];
                    int32_t node = 0, nb = tv.root_base;
                    bool ok = true;
                    for (unsigned e = e0; e < e1; e++) {
                        const int32_t sl = nb + (int32_t)L.ebyte[e];
                        const int2 ent = tv.slots[sl];
                        ok &= ent.y == node;
                        node = sl;
                        nb = ent.x & 0x7FFFFFFF;
                    }
                    out[ntok + t] = ok ? tv.ids[node] : -1;
                }
                ntok += wtok;
            }
            pos += wlen;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (status == 3) capped_known = false;
        if (lane == 0) {
            if (status == 3 && !BIG) {
                const unsigned slot = atomicAdd(a.retry_count, 1u);
                a.retry_list[slot] = (uint32_t)s;
            }
            a.status[s] = (int32_t)status;
            a.counts[s] = status == 0 ? (uint64_t)ntok : 0ull;
            if (a.capped) a.capped[s] = capped_known ? (int32_t)capsum : -1;
        }
    }
}

// ------------------------------------------------------------------ compaction

__global__ void __launch_bounds__(256) compact_kernel(const int32_t *__restrict__ staging, const uint64_t *__restrict__ str_off,
                                                      const uint64_t *__restrict__ id_off, uint64_t n_str,
                                                      int32_t *__restrict__ ids) {
    const uint64_t base_off = str_off[0];
    const unsigned lane = threadIdx.x & 63;
    const uint64_t wstride = (uint64_t)gridDim.x * 4;
    for (uint64_t s = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); s < n_str; s += wstride) {
        const uint64_t src = str_off[s] - base_off, dst = id_off[s];
        const uint64_t n = id_off[s + 1] - dst;
        for (uint64_t k = lane; k < n; k += 64) ids[dst + k] = staging[src + k];
    }
}

__global__ void zero_first(uint64_t *p, uint32_t *rc) {
    if (threadIdx.x == 0) { p[0] = 0; *rc = 0; }
}

// ------------------------------------------------------------------ histogram

__global__ void __launch_bounds__(256) hist_kernel(const uint64_t *__restrict__ id_off, const int32_t *__restrict__ status,
                                                   uint64_t n_str, unsigned long long *hist, uint32_t n_bins) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lh[];
    const uint32_t nb = n_bins + 8;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) lh[b] = 0;
    __syncthreads();
    unsigned long long tok = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_str; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t n = id_off[s + 1] - id_off[s];
        tok += n;
        const uint32_t bin = n < n_bins - 1 ? (uint32_t)n : n_bins - 1;
        atomicAdd(&lh[bin], 1ull);
        const int32_t st = status[s];
        atomicAdd(&lh[n_bins + 2 + (st >= 0 && st <= 4 ? st : 4)], 1ull);
    }
    atomicAdd(&lh[n_bins], tok);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&lh[n_bins + 1], (unsigned long long)n_str);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
        if (lh[b]) atomicAdd(&hist[b], lh[b]);
}

// ------------------------------------------------------------------ launchers

constexpr int SMALL_CH = 256, SMALL_WPB = 4;
constexpr int BIG_CH = 2048, BIG_WPB = 1;

static_assert(wave_lds_bytes<SMALL_CH>() * SMALL_WPB <= 64 * 1024, "small LDS");
static_assert(wave_lds_bytes<BIG_CH>() * BIG_WPB <= 160 * 1024, "big LDS");

hipError_t launch_encode(const EncodeLaunch &p, hipStream_t stream, hipEvent_t ev[6]) {
    EncodeArgs a;
    a.text = p.text; a.str_off = p.str_off; a.cut_mask = p.cut_mask; a.n_str = p.n_str; a.base_off = 0;
    a.staging = p.staging; a.counts = p.counts; a.status = p.status; a.capped = p.capped;
    a.retry_list = p.retry_list; a.retry_count = p.retry_count; a.work_list = nullptr; a.work_count = nullptr;
    a.mode = p.mode;
    TrieView tv{p.slots, p.slot_ids, p.root_base};

    hipLaunchKernelGGL(zero_first, dim3(1), dim3(64), 0, stream, p.id_off, p.retry_count);
    if (ev) hipEventRecord(ev[0], stream);
    if (p.n_str > 0) {
        const uint64_t waves = p.n_str;
        uint64_t blocks = (waves + SMALL_WPB - 1) / SMALL_WPB;
        if (blocks > (uint64_t)p.max_blocks) blocks = p.max_blocks;
        hipLaunchKernelGGL((tokenize_kernel<SMALL_CH, SMALL_WPB, false>), dim3((unsigned)blocks), dim3(SMALL_WPB * 64),
                           wave_lds_bytes<SMALL_CH>() * SMALL_WPB, stream, a, tv);
        // second pass over the strings whose single word did not fit a 256-byte window
        EncodeArgs b = a;
        b.work_list = p.retry_list; b.work_count = p.retry_count;
        hipLaunchKernelGGL((tokenize_kernel<BIG_CH, BIG_WPB, true>), dim3(256), dim3(BIG_WPB * 64),
                           wave_lds_bytes<BIG_CH>() * BIG_WPB, stream, b, tv);
    }
    if (ev) hipEventRecord(ev[1], stream);
    if (p.n_str > 0) {
        size_t tb = p.scan_temp_bytes;
        hipError_t e = hipcub::DeviceScan::InclusiveSum(p.scan_temp, tb, p.counts, p.id_off + 1, (int)p.n_str, stream);
        if (e != hipSuccess) return e;
    }
    if (ev) hipEventRecord(ev[2], stream);
    if (p.n_str > 0) {
        uint64_t blocks = (p.n_str + 3) / 4;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL(compact_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p.staging, p.str_off, p.id_off, p.n_str, p.ids);
    }
    if (ev) hipEventRecord(ev[3], stream);
    return hipGetLastError();
}

size_t scan_temp_bytes(uint64_t n_str) {
    size_t tb = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, tb, (uint64_t *)nullptr, (uint64_t *)nullptr, (int)(n_str ? n_str : 1), (hipStream_t)0);
    return tb;
}

hipError_t launch_histogram(const uint64_t *id_off, const int32_t *status, uint64_t n_str, int64_t *hist,
                            uint32_t n_bins, hipStream_t stream) {
    if (n_str == 0) return hipSuccess;
    uint64_t blocks = (n_str + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(hist_kernel, dim3((unsigned)blocks), dim3(256), (n_bins + 8) * sizeof(unsigned long long), stream,
                       id_off, status, n_str, (unsigned long long *)hist, n_bins);
    return hipGetLastError();
}

hipError_t kernel_init() {
    static bool done = false;
    if (done) return hipSuccess;
    hipError_t e = hipFuncSetAttribute((const void *)tokenize_kernel<BIG_CH, BIG_WPB, true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, wave_lds_bytes<BIG_CH>() * BIG_WPB);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void *)tokenize_kernel<SMALL_CH, SMALL_WPB, false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, wave_lds_bytes<SMALL_CH>() * SMALL_WPB);
    if (e == hipSuccess) done = true;
    return e;
}

int small_window_bytes() { return SMALL_CH; }
int big_window_bytes() { return BIG_CH; }

}  // namespace dpt
