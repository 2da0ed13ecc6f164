// dpt_kernels.hip -- CDNA4 (gfx950) kernels of the shortest-tokenization engine.
//
// A wavefront holds NG = 64/G independent strings ("slots"), each in a G-lane
// group (G = 16 when every vocabulary token has <= 16 code points -- Llama-2 --
// else G = 64, one string per wave).  Per window of <= CH input bytes (windows
// end at word boundaries; words are independent DP problems, reference
// packages/tokenizer_utils.py:70):
//
//   prep   load the window bytes of every slot (aligned dword buffer loads, all slots in
//          flight) and atomise them like pretokenize_raw (tokenizer_utils.py:33-50): atom
//          offsets, code-point prefix sums (cp(span) = cpos[i]-cpos[j], the len(t) of
//          dp_tokenize.py:82) with word-start bits, and the word list -- one packed DPP scan.
//          Atoms are expanded ('▁'+c first, ' '->'▁', '\n'->'<0x0A>') on the fly later.
//   A      match discovery: one walk per lane over the byte double-array trie (L2-resident)
//          from every atom start of every slot (pure-ASCII raw windows: every walk's first
//          lookup byte-parallel first, A0); a token of L atoms ending at e clears bit L-1 of e's
//          inverted END mask ("join(atoms[j:i]) in vocabulary", dp_tokenize.py:39).  Walks that
//          finish take the next start (ballot + mbcnt), so the wave stays busy.
//   B      forward recurrence (cost capped at the atom index within
//          the word, dp_tokenize.py:28; reachability; the max-of-max token length G[i]).  Lane
//          mode (every atom a token by itself, the common case): each lane runs the recurrence
//          sequentially over a chunk cut at cut points (boundaries no token crosses), a row scan
//          of the chunk transfers supplies each chunk's incoming state.  Row mode (otherwise):
//          lane d of a group holds candidate j = i-1-d and forms one key
//              (cost[j]+1) << 16 | invalid[j] << 15 | (0x7FFF - max(G[j], cp(span)))
//          whose DPP group-min is the state of i; two ballots give the largest j in E(i)
//          (dp_tokenize.py:40-46) that is reachable (de) and the largest that attains G[i] (dg).
//   C0/C1  token counts, validity and the selection: walking right to left, take dg while the
//          longest token so far is below G[n], de once it is reached -- the reference's first
//          argmax in DFS order (dp_tokenize.py:58 pops the largest j first; :84 takes the first
//          max).  Lane mode walks its chunks, row mode one word per lane.
//   C2     id resolution, t2i[token] (tokenizer_utils.py:76-79) into the slot's staging row.  16-lane
//          first pass: a bulk pass takes every selected token of one or two expanded bytes with ONE
//          lookup (root child / two-byte root table) and lists the rest; a short list (< 64) waits
//          in the wave's pending row and is walked 64 at a time from its stored bytes, a long one
//          by the refill walker.  Other passes: the refill walker re-walks every selected span.
//
// Strings are claimed from 16 partition counters (see tokenize_kernel).  Strings whose single word
// exceeds CH bytes are re-run by the 2048-byte, one-string-per-wave instantiation, longer ones by
// the unbounded pass (dpt_long.hip).  The finish kernel turns the staging rows into CSR ids.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "dpt_internal.h"
// the unbounded pass (namespace dpt::lng): one translation unit with fallback_kernel, which runs it
// in the same launch as the 2048-byte pass
#include "dpt_long.hip"

namespace dpt {

// Compile-time options are diagnostics only (DPT_STOP, DPT_C2STOP, DPT_STAMPS: wrong results or extra
// counters by design, never in the product build).  The alternatives measured slower or neutral are
// gone from the source (the round-4 self-copy and pipelined CSR pass: git tag r04-experiments);
// DESIGN.md §9 lists them with their numbers.

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

// inclusive max-scan over 64 lanes (values >= 0; the same DPP steps as the add scan)
__device__ __forceinline__ unsigned wave_incl_scan_max(unsigned v) {
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true));  // row_shr:1
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true));  // row_shr:2
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true));  // row_shr:4
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true));  // row_shr:8
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false)); // row_bcast:15
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false)); // row_bcast:31
    return v;
}

// min within each row of 16 lanes, result in every lane of the row
// (mov_dpp with bound_ctrl lets hipcc fold each step into one v_min_u32_dpp)
__device__ __forceinline__ unsigned row_min_u32(unsigned v) {
    v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
    v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
    v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));  // row_half_mirror
    v = min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));  // row_mirror
    return v;
}

// min over 64 lanes, result uniform (SGPR)
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    v = row_min_u32(v);
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

// lane l receives x[l-1]; the first lane of each row (row_shr:1) / of the wave (wave_shr:1) receives `in`
__device__ __forceinline__ unsigned row_shift_in(unsigned x, unsigned in) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)in, (int)x, 0x111, 0xF, 0xF, false);
}
__device__ __forceinline__ unsigned wave_shift_in(unsigned x, unsigned in) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)in, (int)x, 0x138, 0xF, 0xF, false);
}

// Lane-group shifts for lane-mode B: lane l of a group of LW lanes receives x of lane l + K (gshl) / l - K (gshr),
// `fill` past the group's edge.  LW = 16: one DPP row op (row_shl / row_shr:K); LW = 64 (one string across the
// wave, the one-string kernel): ds_bpermute.
template <int LW, unsigned K>
__device__ __forceinline__ unsigned gshl(unsigned x, unsigned fill) {
    if constexpr (LW == 16) {
        return (unsigned)__builtin_amdgcn_update_dpp((int)fill, (int)x, 0x100 | K, 0xF, 0xF, false);
    } else {
        const unsigned l = lane_id();
        const unsigned v = (unsigned)__builtin_amdgcn_ds_bpermute((int)(((l + K) & 63u) << 2), (int)x);
        return l + K < 64u ? v : fill;
    }
}
template <int LW, unsigned K>
__device__ __forceinline__ unsigned gshr(unsigned x, unsigned fill) {
    if constexpr (LW == 16) {
        return (unsigned)__builtin_amdgcn_update_dpp((int)fill, (int)x, 0x110 | K, 0xF, 0xF, false);
    } else {
        const unsigned l = lane_id();
        const unsigned v = (unsigned)__builtin_amdgcn_ds_bpermute((int)(((l - K) & 63u) << 2), (int)x);
        return l >= K ? v : fill;
    }
}

// 64-bit inclusive add-scan over the wave (ds_bpermute shifts)
__device__ __forceinline__ uint64_t wave_incl_scan_add64(uint64_t v, unsigned lane) {
#pragma unroll
    for (unsigned k = 1; k < 64; k <<= 1) {
        const int src = (int)((lane >= k ? lane - k : lane) << 2);
        const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)(unsigned)v);
        const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)(unsigned)(v >> 32));
        v += lane >= k ? (((uint64_t)hi << 32) | lo) : 0ull;
    }
    return v;
}

__device__ __forceinline__ unsigned uni(unsigned x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((unsigned)(x >> 32)) << 32) | uni((unsigned)x);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// lowest set bit (v_ffbl_b32: 0xFFFFFFFF for 0, no select needed where 0 cannot matter)
__device__ __forceinline__ unsigned ffbl(unsigned x) {
    unsigned r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ------------------------------------------------------------------ group geometry

template <int G> struct Group;

// G = 16: four strings per wave, one per DPP row.  Per atom: {cpos, ~span mask} in one
// dword (after phase B the mask half of a word-end atom holds the word's final key, Wfin<16>,
// and in C1 the mask halves take the selected tokens); per end position i, one u16 `fin`:
// the back distances (minus one) of the largest reachable j in E(i) attaining G[i] (dg) and
// of the largest reachable j in E(i) (de), 4 bits each.  Both exist at every position of a
// valid word's selected path (Appendix A: a reachable i has a reachable j attaining its key),
// and C1 walks valid words only, so no "none" code is stored.
template <> struct Group<16> {
    using M = uint16_t;
    // smask: until phase B, the inverted END mask of end position i: bit d clear = atoms
    // i-1-d .. i-1 are a token (phase A clears the bits with LDS atomics)
    struct Rec { uint16_t cpos; uint16_t smask; };
    struct Fin { uint8_t v; };   // dg | de << 4
    static __device__ __forceinline__ unsigned dg(const Fin &x) { return x.v & 15u; }
    static __device__ __forceinline__ unsigned de(const Fin &x) { return (x.v >> 4) & 15u; }
};

// G = 64: one string per wave (vocabularies with tokens of 17..64 code points).
template <> struct Group<64> {
    using M = uint64_t;
    struct Rec { uint64_t smask; uint16_t cpos; uint16_t pad[3]; };
    struct Fin { uint32_t d; uint32_t w; };   // w: the final key (Wfin<64>)
    static __device__ __forceinline__ unsigned dg(const Fin &x) { return x.d & 127u; }
    static __device__ __forceinline__ unsigned de(const Fin &x) { return (x.d >> 8) & 127u; }
};

// ------------------------------------------------------------------ LDS layout

constexpr uint16_t CP_WS = 0x8000;        // cpos bit: atom starts a word
constexpr unsigned MAX_ATOM_BYTES = 8;    // expanded atom = one u64 (raw: '▁'+4-byte code point = 7)

// final state at a word end.  G = 16: 16 bits in the word-end atom's mask half:
// cost << 6 | invalid << 5 | 31-G, straight from the key (its bits 10..14 are constant 1s);
// cost 1023 = the uncapped DP's "inf" (0xFFFF, inspect_tokenizer.py:80), capped costs <= CH
template <int G> struct Wfin;
template <> struct Wfin<16> {
    using T = uint16_t;
    // one v_bfi: bits 5..15 from r >> 10, the rest from r (bits 16+ fall off in the u16)
    static __device__ __forceinline__ T pack(unsigned r) {
        unsigned o;
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(o) : "s"(0xFFE0u), "v"(r >> 10), "v"(r));
        return (T)o;
    }
    static __device__ __forceinline__ unsigned cost(T x) { return (x >> 6) == 1023u ? 0xFFFFu : (x >> 6); }
    static __device__ __forceinline__ bool invalid(T x) { return (x >> 5) & 1u; }
    static __device__ __forceinline__ unsigned gmax(T x) { return 31u - (x & 31u); }
};
template <> struct Wfin<64> {
    using T = uint32_t;   // the group-min key itself: cost<<16 | invalid<<15 | 0x7FFF-G
    static __device__ __forceinline__ T pack(unsigned r) { return r; }
    static __device__ __forceinline__ unsigned cost(T x) { return x >> 16; }
    static __device__ __forceinline__ bool invalid(T x) { return (x >> 15) & 1u; }
    static __device__ __forceinline__ unsigned gmax(T x) { return 0x7FFFu - (x & 0x7FFFu); }
};

// G = 64: rec[] as two arrays (span masks, code-point prefixes) -- 10 bytes per atom instead of the
// 16 of an aligned struct, so LDS per wave (5.2 KB) holds more resident waves than the 24 that 80
// VGPRs allow; rec[j] yields references to both fields, so the shared code reads L.rec[j].cpos alike
template <int NA> struct RecSoA {
    uint64_t sm[NA];
    uint16_t cp[NA];
    struct Ref { uint64_t &smask; uint16_t &cpos; };
    struct CRef { const uint64_t &smask; const uint16_t &cpos; };
    __device__ __forceinline__ Ref operator[](unsigned i) { return {sm[i], cp[i]}; }
    __device__ __forceinline__ CRef operator[](unsigned i) const { return {sm[i], cp[i]}; }
};

template <int CH, int G>
struct GroupLDS {
    using M = typename Group<G>::M;
    static constexpr int NA = CH + 2;            // atoms + sentinel
    // rec[j]: code-point prefix of atom j (| CP_WS at word starts and at the window end) and the
    //         span mask of tokens of 1..G atoms starting at j; after phase B the mask field holds
    //         the first atom of selected token j (tokens tile the window)
    std::conditional_t<(G == 64), RecSoA<NA>, typename Group<G>::Rec[NA]> rec;
    typename Group<G>::Fin fin[NA];   // per end position, see Group<G>
    // the final key of the word ending at atom e
    __device__ __forceinline__ typename Wfin<G>::T wkey(unsigned e) const {
        if constexpr (G == 16) return rec[e].smask;
        else return fin[e].w;
    }
    // CH = 256: u8, stored mod 256 -- offsets and word starts are < 256; the sentinels (wlen,
    // n_atoms <= 256) are recovered with modular differences (atom_len, word_end)
    using Idx = std::conditional_t<(CH <= 256), uint8_t, uint16_t>;
    // word -> first atom: in global scratch for 256-byte windows (WSLG; LDS is what limits the
    // resident waves there), in LDS for the 2048-byte pass
    static constexpr bool WSLG = CH <= 256;
    static constexpr int WSL_STRIDE = (NA + 15) & ~15;
    Idx aoff[NA];                   // atom -> byte offset in the window
    Idx wsl[WSLG ? 1 : NA];
    __device__ __forceinline__ unsigned atom_len(unsigned j) const { return (Idx)(aoff[j + 1] - aoff[j]); }
    // word w's first atom / its end (= the next word's first atom, or n_atoms)
    __device__ __forceinline__ unsigned word_start(const uint8_t *gw, unsigned w) const {
        if constexpr (WSLG) return gw[w];
        else return wsl[w];
    }
    __device__ __forceinline__ unsigned word_end(const uint8_t *gw, unsigned w) const {
        if constexpr (WSLG) return (((unsigned)gw[w + 1] + 255u) & 0xFFu) + 1u;
        else return wsl[w + 1];
    }
    __device__ __forceinline__ void set_word_start(uint8_t *gw, unsigned w, unsigned v) {
        if constexpr (WSLG) gw[w] = (uint8_t)v;
        else wsl[w] = (Idx)v;
    }
    // the window's input bytes (expanded on the fly); the dword reads of the last atoms run up to
    // 12 bytes past the end, into the next group or the slot states -- masked off, never used
    alignas(16) uint8_t bytes[CH];
    // G = 64, 256-byte windows, non-raw modes (no expansions: a token's bytes are the window's): per byte
    // position p <= wlen, byte[p] | BF_ATOM (an atom starts at p, or p == wlen) | BF_STOP (a word starts
    // at p, or p == wlen) -- phase A's byte-stream walker reads ONE u16 per trie step
    // (zero-length when unused: one spare byte here rounded the 16-lane group up 16 bytes -- 21 resident
    // waves per CU instead of 22, and the slots' bank interleaving off; the static_assert below holds it)
    static constexpr bool BSTREAM = G == 64 && CH == 256;
    uint16_t bf[BSTREAM ? CH + 2 : 0];
    // ... and per atom: 1 = it starts a word that is one vocabulary token (the whole-word shortcut)
    uint8_t scf[BSTREAM ? CH + 2 : 0];
};
constexpr unsigned BF_ATOM = 0x100u, BF_STOP = 0x200u;

// strings are < 4 GiB (dpt.h); abase: atoms of the string's earlier windows
// (48 bytes: LDS per slot is what bounds the resident waves)
struct SlotState {
    uint64_t sb;
    uint32_t s, slen, pos, ntok, capsum, wtok;
    uint32_t abase;
    uint16_t wlen, n_atoms, n_words;
    uint8_t active, status, inval, capb;   // capb: some atom of the window is not a token by itself (the cap can bind)
    uint8_t cpw;   // a '\u2581'-compressed PRESPLIT window (prep_window): raw mode's ASCII paths, no first-atom rule
    uint8_t pad;
};
static_assert(sizeof(SlotState) == 48, "slot state layout");

template <int CH, int G>
constexpr int group_lds_bytes() { return (int)((sizeof(GroupLDS<CH, G>) + 15) & ~size_t(15)); }

// A wave's LDS: per slot g its group's arrays, then its SlotState -- slot g at g * group_stride.  The
// 16-lane kernel's stride (1856 B = 464 dwords, 16 mod 32) puts the two DPP rows of a 32-lane LDS lane group
// (slots 0 / 1, 2 / 3) half a bank row apart: lane-mode B and C1 step through chunks 17 atoms apart, and
// two slots 452 dwords apart (the arrays back to back, then the slot states) made most of those reads
// 2-way bank conflicts; interleaved, the same bytes are conflict-free.
template <int CH, int G>
constexpr int group_stride() { return group_lds_bytes<CH, G>() + (int)sizeof(SlotState); }
static_assert(group_stride<256, 16>() == 1856, "16-lane group stride: 21 resident waves per CU (512-B LDS granule), slots 16 dwords mod 32 apart");
template <int CH, int G>
constexpr int block_lds_bytes() { return (64 / G) * group_stride<CH, G>(); }

// ------------------------------------------------------------------ trie access

struct TrieView {
    // .x = base | TERM<<31 | LEAF<<30, .y = check (parent slot, -1 free); followed by the 65536-entry
    // two-byte root table (entry b0 << 8 | b1 at slots[n_slots + ...], see dpt_api.cpp)
    const int2 *__restrict__ slots;
    const int32_t *__restrict__ ids;  // token id of a terminal slot
    const int4 *__restrict__ slots4;  // {base, check, id, 0}: C2's walks get the id with the last node
    int32_t root_base;
    uint32_t n_slots;
    // [b0 << 8 | b1]: id of the two-byte token, [65536 + b0]: of the one-byte one (-1: none); then, from
    // element PAIR16_N, A0's uint2 table [b0 << 8 | b1]: flags (root child b0, b0 a token, node b0 b1, its
    // TERM, LEAF) + that node's child filter
    const int16_t *__restrict__ pair16;
};

// Trie reads through buffer resources: 32-bit slot offsets (no 64-bit address arithmetic) and a
// range check that makes any index safe (out of range reads {0, 0}: a failed transition).
__device__ __forceinline__ int2 trie_slot(const TrieView &tv, int32_t t) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)tv.slots, (short)0, (int)((tv.n_slots + 65536u) * 8u), 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (unsigned)t * 8u, 0, 0);
    return make_int2((int32_t)v[0], (int32_t)v[1]);
}
// phase A: {base, check, id, child filter} per slot, then the root table as {.x, .y, 0, child
// filter} (dpt_api.cpp), so one 16-byte load serves both
__device__ __forceinline__ int4 trie_slotA(const TrieView &tv, int32_t t) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)tv.slots4, (short)0, (int)((tv.n_slots + 65536u) * 16u), 0x00020000);
    return __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)t * 16u, 0, 0));
}
__device__ __forceinline__ int4 trie_slot4(const TrieView &tv, int32_t t) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)tv.slots4, (short)0, (int)(tv.n_slots * 16u), 0x00020000);
    return __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)t * 16u, 0, 0));
}

[[maybe_unused]] constexpr int32_t TERM_BIT = (int32_t)0x80000000;
[[maybe_unused]] constexpr int32_t LEAF_BIT = 0x40000000;  // no children (dpt_long.hip ends walks on it; this kernel uses the child filters)
constexpr int32_t BASE_MASK = 0x3FFFFFFF;

// ------------------------------------------------------------------ arguments

struct EncodeArgs {
    const uint8_t *text;
    const uint64_t *str_off;
    const uint8_t *cut_mask;    // PRESPLIT / ATOMS only
    uint64_t n_str;
    int32_t *staging;           // ids staged at (str_off[s]-str_off[0]) + k
    int16_t *staging16;         // non-null: the ids are staged here as int16 instead (half the bytes)
    uint64_t *counts;           // per string
    unsigned long long *bsum;   // nullable: the batch lines (dpt_internal.h BS_LINE): per FIN_BATCH strings, the sum of
                                //   their counts (atomics as strings finish)
    int32_t *status;
    int32_t *capped;            // nullable
    uint32_t *retry_list;       // strings for the 2048-byte pass
    uint32_t *retry_count;
    uint32_t *long_list;        // strings for the unbounded pass (dpt_long.hip)
    uint32_t *long_count;
    const uint32_t *work_list;  // 2048-byte pass: the retry list
    const uint32_t *work_count;
    uint32_t *work_next;        // 2048-byte pass: its work counter (zeroed per launch)
    uint32_t *part_ctr;         // first pass: NPART partition counters (PART_STRIDE apart), then the used-up mask
    uint8_t *wsl_scratch;       // word lists of the 256-byte pass: grid x NG x WSL_STRIDE bytes
    uint4 *pend;                // 16-lane first pass: per wave, 64 pending residual tokens (walk_pending)
    int32_t ws_node, ws_base, ws_id;   // the trie node after U+2581, its base word and id (-1: none)
    int long_span;              // the vocabulary has tokens longer than 64 code points
    uint64_t *edges;            // nullable: per atom end, the E(i) & reachable back-distance mask
    int mode;                   // DPT_MODE_* | DPT_FLAG_*
    unsigned long long *hist_zero;   // 2048-byte pass, fin_fold calls with DPT_HIST_OVERWRITE: the histogram to
    uint32_t n_hist;                 //   zero before the finish pass adds to it (the scan kernel's duty otherwise)
    uint64_t *id_off;
    int32_t *ids;
    // one-string host-path calls (EncodeLaunch::solo): the string's ids go straight to ids (staging =
    // ids, counts = id_off + 1) and the lone wave writes id_off[0] and resets the counter block (its
    // first 64 bytes to ctr_snap) -- no fallback, scan or finish launch follows
    int solo;
    uint64_t *ctr_snap;
};

#ifdef DPT_STAMPS
// diagnostic build only: cycles per phase summed over waves (never in the product build)
__device__ unsigned long long g_stamps[10];
#define STAMP_DECL unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#define STAMP(k) do { const unsigned long long _t = __builtin_amdgcn_s_memtime(); st_acc[k] += _t - st_prev; st_prev = _t; } while (0)
#define STAMP_FLUSH do { if (lane == 0) for (int _k = 0; _k < 10; _k++) atomicAdd(&g_stamps[_k], st_acc[_k]); } while (0)
#else
#define STAMP_DECL
#define STAMP(k)
#define STAMP_FLUSH
#endif
#ifdef DPT_WSTAMPS
// diagnostic build only (its own library, no phase stamps): the first pass's per-wave timeline (tools/wave_timeline.py): per wave (blockIdx), [0] its first
// instruction, [1 + k] the end of its k-th slot round (| the round's busy slots << 56), [WST_N - 1] its exit
// (| its rounds << 48); s_memrealtime (100 MHz, one clock for the whole chip)
constexpr unsigned WST_MAXW = 8192, WST_N = 128;
__device__ unsigned long long g_wst[WST_MAXW * WST_N];
#define WST_REC(k, v) do { if (!BIG && lane == 0 && bid < WST_MAXW && (unsigned)(k) < WST_N) g_wst[(size_t)bid * WST_N + (k)] = (v); } while (0)
#define WST_NOW() ((unsigned long long)__builtin_amdgcn_s_memrealtime())
#else
#define WST_REC(k, v)
#define WST_NOW() 0ull
#endif

// Phase A's per-atom descriptor: byte offset | byte length << PB | "a word or the window ends
// after it" << PB+4 | "first atom of the string" << PB+5 (16 bits for 256-byte windows).  It is
// parked in the (not yet written) fin[] entry of the atom.
template <int CH> struct AInfo {
    static constexpr unsigned PB = CH <= 256 ? 8u : 12u;
    static constexpr unsigned STOP = 1u << (PB + 4), FIRST = 1u << (PB + 5);
    static __device__ __forceinline__ unsigned pack(unsigned p0, unsigned la, unsigned stop, unsigned first) {
        return p0 | (la << PB) | (stop ? STOP : 0u) | (first ? FIRST : 0u);
    }
    static __device__ __forceinline__ unsigned off(unsigned x) { return x & ((1u << PB) - 1u); }
    static __device__ __forceinline__ unsigned len(unsigned x) { return (x >> PB) & 15u; }
};

// G = 16 derives it from the atom offsets and the next atom's word-start bit (its u8 fin[]
// has no room; LDS per slot bounds the resident waves); G = 64 parks it in fin[].d
template <int CH, int G>
__device__ __forceinline__ unsigned ainfo_get(const GroupLDS<CH, G> &L, unsigned j, bool first) {
    if constexpr (G == 16) return AInfo<CH>::pack(L.aoff[j], L.atom_len(j), L.rec[j + 1].cpos >> 15, first && j == 0);
    else return L.fin[j].d;
}
template <int CH, int G>
__device__ __forceinline__ void ainfo_set(GroupLDS<CH, G> &L, unsigned j, unsigned v) {
    if constexpr (G != 16) L.fin[j].d = v;
}

// la (<= 8) window bytes from offset p: three aligned dword reads and a funnel shift
__device__ __forceinline__ uint64_t load_bytes(const uint8_t *bytes, unsigned p, unsigned la) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(bytes) + (p >> 2);
    const unsigned sh = p & 3u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    return v & (~0ull >> (64u - 8u * la));   // 1 <= la <= 8
}

// expanded bytes of the atom described by `info` (AInfo).  WIDE (ATOMS mode): atoms of up to 8
// bytes; otherwise (RAW / PRESPLIT) atoms are UTF-8 code points of at most 4 bytes, read with
// two dword loads.
template <int CH, bool WIDE>
__device__ __forceinline__ uint64_t atom_from_info(const uint8_t *bytes, uint32_t info, bool raw, unsigned &cnt) {
    const unsigned la = AInfo<CH>::len(info);
    const unsigned off = AInfo<CH>::off(info);
    uint64_t v;
    if constexpr (WIDE) {
        v = load_bytes(bytes, off, la);
    } else {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(bytes) + (off >> 2);
        const unsigned sh = 32u - 8u * la;   // 1 <= la <= 4
        v = (__builtin_amdgcn_alignbyte(w[1], w[0], off & 3u) << sh) >> sh;
    }
    const unsigned b0 = (unsigned)(v & 0xFFu);
    // expansions (raw mode only); the selects run only when some lane of the wave needs one
    const bool fi = raw && (info & AInfo<CH>::FIRST) != 0;
    const bool sp = raw && !fi && b0 == ' ';
    const bool nl = raw && !fi && b0 == '\n';
    uint64_t seq = v;
    cnt = la;
    if (ballot(fi || sp || nl)) {
        seq = fi ? (0x8196E2ull | (v << 24)) : seq;
        seq = sp ? 0x8196E2ull : seq;
        seq = nl ? 0x3E413078303Cull : seq;
        cnt = fi ? 3 + la : (sp ? 3u : (nl ? 6u : la));
    }
    return seq;
}

// C2's hash key of the token of `nbytes` window bytes from p0 (dpt_internal.h tokhash): its expanded
// bytes -- raw mode: the string's first atom is '\u2581' + its bytes, a leading ' ' is '\u2581' -- as
// four little-endian dwords, zero past the expanded length E.  False (the walkers take the token) when
// E > TOKHASH_MAX_BYTES or, in raw mode, a newline atom (expanded to "<0x0A>") is in the token.
template <int CH>
__device__ __forceinline__ bool token_key(const uint8_t *bytes, unsigned p0, unsigned nbytes, bool raw, unsigned first,
                                          uint32_t (&w)[4], unsigned &E) {
    const uint32_t *wp = reinterpret_cast<const uint32_t *>(bytes) + (p0 >> 2);
    const unsigned sh = p0 & 3u;
    // (reads up to 20 bytes past p0's dword: within the group's bytes, the next group or the slot states)
    const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2], d3 = wp[3], d4 = wp[4];
    uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, sh), r1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, sh), r3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
    const unsigned b0 = r0 & 0xFFu;
    const unsigned fi = raw ? first : 0u;
    const unsigned sp = (raw ? 1u : 0u) & (fi ^ 1u) & (unsigned)(b0 == ' ');
    E = nbytes + 3u * fi + 2u * sp;
    if (E > TOKHASH_MAX_BYTES || nbytes == 0) return false;
    // bytes [fi, nbytes) of the raw token must hold no '\n' (a non-first '\n' atom expands to 6 bytes)
    auto keep = [](unsigned n, unsigned k) -> uint32_t {   // bytes of dword k below n
        return n >= 4u * k + 4u ? 0xFFFFFFFFu : (n <= 4u * k ? 0u : (1u << (8u * (n - 4u * k))) - 1u);
    };
    if (raw) {
        uint32_t nl = 0;
        const uint32_t x[4] = {r0, r1, r2, r3};
#pragma unroll
        for (unsigned k = 0; k < 4; k++) {
            // bytes outside [fi, nbytes) read as 0xFF (never '\n'); haszero over x ^ '\n'
            uint32_t v = x[k] | ~keep(nbytes, k);
            if (k == 0) v |= fi ? 0xFFu : 0u;
            v ^= 0x0A0A0A0Au;
            nl |= (v - 0x01010101u) & ~v & 0x80808080u;
        }
        if (nl) return false;
        if (fi | sp) {
            // '\u2581' (E2 96 81) in front: a first atom keeps its bytes (shift 3), a leading space
            // becomes the 81 of the prefix (shift 2)
            const uint32_t s0 = sp ? ((r0 & 0xFFFFFF00u) | 0x81u) : r0;
            const uint32_t pm = fi ? 0x8196E200u : 0x96E20000u;
            const unsigned as = fi ? 1u : 2u;
            r3 = __builtin_amdgcn_alignbyte(r3, r2, as);
            r2 = __builtin_amdgcn_alignbyte(r2, r1, as);
            r1 = __builtin_amdgcn_alignbyte(r1, s0, as);
            r0 = __builtin_amdgcn_alignbyte(s0, pm, as);
        }
    }
    w[0] = r0 & keep(E, 0); w[1] = r1 & keep(E, 1); w[2] = r2 & keep(E, 2); w[3] = r3 & keep(E, 3);
    return true;
}

// The 64-lane kernels' hash of a token of up to TOKHASH_MAX_BYTES_LONG expanded bytes (BLOOM-scale
// vocabularies: tokens of up to 41 code points): the dwords streamed from the window bytes with the same
// expansion and newline rule as token_key, mixed as they come (dpt_internal.h).  False: the walkers.
template <int CH>
__device__ __forceinline__ bool token_hash_long(const uint8_t *bytes, unsigned p0, unsigned nbytes, bool raw, unsigned first,
                                                uint32_t seed, uint32_t &h, uint32_t &fp) {
    const uint32_t *wp = reinterpret_cast<const uint32_t *>(bytes) + (p0 >> 2);
    const unsigned sh = p0 & 3u;
    uint32_t d0 = wp[0], d1 = wp[1];
    const unsigned b0 = __builtin_amdgcn_alignbyte(d1, d0, sh) & 0xFFu;
    const unsigned fi = raw ? first : 0u;
    const unsigned sp = (raw ? 1u : 0u) & (fi ^ 1u) & (unsigned)(b0 == ' ');
    const unsigned E = nbytes + 3u * fi + 2u * sp;
    if (E > TOKHASH_MAX_BYTES_LONG || nbytes == 0) return false;
    const unsigned nd = E <= 16u ? 4u : (E + 3u) >> 2;
    const bool shift = (fi | sp) != 0;
    const unsigned as = fi ? 1u : 2u;
    uint32_t prev = fi ? 0x8196E200u : 0x96E20000u;   // the '\u2581' prefix ahead of raw dword 0
    TokHashState a = tokhash_start(E, seed);
    uint32_t nl = 0;
    for (unsigned k = 0; k < nd; k++) {
        uint32_t r = __builtin_amdgcn_alignbyte(d1, d0, sh);   // raw bytes 4k .. 4k+3
        d0 = d1;
        // (bytes past the token are masked off; the read stays within 16 bytes past the window's bytes:
        // the slot states follow them)
        const unsigned nxt = (p0 >> 2) + k + 2u;
        d1 = reinterpret_cast<const uint32_t *>(bytes)[nxt < (unsigned)CH / 4u + 4u ? nxt : (unsigned)CH / 4u + 3u];
        if (raw) {
            // bytes [fi, nbytes) hold no '\n' (a non-first newline atom expands to six bytes)
            const unsigned lo = 4u * k;
            uint32_t v = r | (nbytes >= lo + 4u ? 0u : (nbytes <= lo ? 0xFFFFFFFFu : ~((1u << (8u * (nbytes - lo))) - 1u)));
            if (k == 0 && fi) v |= 0xFFu;
            v ^= 0x0A0A0A0Au;
            nl |= (v - 0x01010101u) & ~v & 0x80808080u;
            if (k == 0 && sp) r = (r & 0xFFFFFF00u) | 0x81u;
        }
        uint32_t w = r;
        if (shift) {
            w = __builtin_amdgcn_alignbyte(r, prev, as);
            prev = r;
        }
        const unsigned lo = 4u * k;
        w &= E >= lo + 4u ? 0xFFFFFFFFu : (E <= lo ? 0u : (1u << (8u * (E - lo))) - 1u);
        a = tokhash_step(a, w, k);
    }
    if (nl) return false;
    tokhash_end(a, h, fp);
    return true;
}

// ------------------------------------------------------------------ prep: one slot's window


// The bytes (and cut-mask bytes) of a window, in registers: lane l holds bytes
// [256c + 4l, 256c + 4l + 4) of chunk c, little-endian; *_end is the byte at CH (the probe
// for the last word start when the string continues past the window).
template <int CH> struct WinRegs {
    static constexpr int NC = CH / 256;
    uint32_t t[NC], c[NC];
    uint32_t t_end, c_end;
};

__device__ __forceinline__ uint32_t load_u32_at(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned sh) {
    const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u, 0, 0);
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Aligned dword buffer loads over [base + pos, base + slen): bytes past the string's last
// aligned dword read as 0 (buffer range check), and no load leaves that dword, so no load
// can touch a page the string does not.
template <int CH>
__device__ __forceinline__ void load_window_bytes(const uint8_t *base, uint64_t pos, uint64_t slen, unsigned lane,
                                                  uint32_t (&out)[CH / 256], uint32_t &end) {
    const uint8_t *p = base + pos;
    const unsigned sh = (unsigned)((uintptr_t)p & 3u);
    uint64_t n = (slen - pos + sh + 3u) & ~(uint64_t)3;
    if (n > (uint64_t)(CH + 16)) n = CH + 16;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(p - sh), (short)0, (int)n, 0x00020000);
#pragma unroll
    for (int c = 0; c < CH / 256; c++) out[c] = load_u32_at(r, c * 256u + lane * 4u, sh);
    end = load_u32_at(r, (unsigned)CH, sh) & 0xFFu;
}

template <int CH>
__device__ __forceinline__ void load_window(WinRegs<CH> &W, const uint8_t *str, const uint8_t *cut, uint64_t pos,
                                            uint64_t slen, bool raw, unsigned lane) {
    load_window_bytes<CH>(str, pos, slen, lane, W.t, W.t_end);
    if (!raw) load_window_bytes<CH>(cut, pos, slen, lane, W.c, W.c_end);
}

__device__ __forceinline__ bool is_word_start(unsigned b, unsigned cm, int mode) {
    return mode == 0 ? (b == ' ') : (mode == 1 ? (cm != 0 && (b & 0xC0u) != 0x80u) : (cm & 1u) != 0);
}

// 0x80 in every byte of x equal to the matching byte of c4, 0 elsewhere (exact per byte)
__device__ __forceinline__ uint32_t eq_bytes(uint32_t x, uint32_t c4) {
    const uint32_t y = x ^ c4;
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}

// Finds the window [pos, pos+wlen) (ends at a word start or at the string end).
// Returns false when a single word does not fit in CH bytes.
template <int CH>
__device__ bool window_bounds(const WinRegs<CH> &W, uint64_t slen, uint64_t pos, int mode, unsigned lane, unsigned &wlen) {
    const uint64_t rem = slen - pos;
    if (rem <= (uint64_t)CH) {
        wlen = (unsigned)rem;
        return true;
    }
    int best = is_word_start(W.t_end, W.c_end, mode) ? CH : -1;
    if (CH == 256 && mode == 0) {
        // raw mode: the last space in bytes 1..255, from a per-byte equality mask of the lane's dword
        uint32_t sp = eq_bytes(W.t[0], 0x20202020u);
        if (lane == 0) sp &= ~0x80u;   // byte 0 starts the window anyway
        if (sp) best = max(best, (int)(4u * lane + ((31u - (unsigned)__builtin_clz(sp)) >> 3)));
        const unsigned q = wave_max_u32((unsigned)(best + 1));
        if (q == 0) return false;
        wlen = q - 1;
        return true;
    }
#pragma unroll
    for (int c = 0; c < CH / 256; c++)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = c * 256 + (int)lane * 4 + u;
            if (k > 0 && is_word_start((W.t[c] >> (8 * u)) & 0xFFu, (W.c[c] >> (8 * u)) & 0xFFu, mode)) best = max(best, k);
        }
    const unsigned q = wave_max_u32((unsigned)(best + 1));
    if (q == 0) return false;
    wlen = q - 1;
    return true;
}

// Atomise window bytes [pos, pos+wlen) into L: the bytes themselves, atom byte offsets,
// code-point prefixes (+ word-start bits) and the word list.  One packed DPP scan per 256
// bytes.  Returns false if an atom is longer than MAX_ATOM_BYTES (4 bytes in RAW mode).
// cpw_o: 1 when the window was stored '\u2581'-compressed (PRESPLIT, 16-lane first pass; below).
template <int CH, int G, bool WIDE>
__device__ bool prep_window(GroupLDS<CH, G> &L, uint8_t *gw, const WinRegs<CH> &W, uint64_t pos,
                            unsigned wlen, int mode, unsigned lane, unsigned &n_atoms_o, unsigned &n_words_o,
                            unsigned &cpw_o) {
    const bool raw = mode == 0;
    unsigned n_atoms = 0, cp_tot = 0, n_words = 0;
    bool hi_byte = false;   // some byte >= 0x80: atoms may be longer than one byte
    bool ast0[4] = {false, false, false, false};   // (256-byte windows: the lane's atom starts and atom indices)
    unsigned aiu0[4] = {0, 0, 0, 0};
    cpw_o = 0;
#pragma unroll
    for (int c = 0; c < CH / 256; c++) {
        const unsigned c0 = c * 256u;
        if (c0 >= wlen) break;
        bool ast[4], wst[4];
        unsigned cpl[4];
        unsigned a_sum = 0, w_sum = 0, cp_sum = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned k = c0 + lane * 4 + u;
            const bool in = k < wlen;
            const unsigned b = (W.t[c] >> (8 * u)) & 0xFFu;
            const unsigned cm = raw ? 0u : (W.c[c] >> (8 * u)) & 0xFFu;
            const bool first = in && pos + k == 0;
            // mode 2 (ATOMS): atom starts come from the mask (bit 1), word starts from bit 0
            const bool cont = in && !first && (mode == 2 ? (cm & 3) == 0 : (b & 0xC0) == 0x80);
            const bool as = in && !cont;
            bool wsf;
            unsigned cl;
            if (raw) {
                wsf = as && (k == 0 || b == ' ');
                cl = !in ? 0 : first ? 2 : (b == '\n' ? 6 : ((b & 0xC0) == 0x80 ? 0 : 1));
            } else {
                wsf = as && (k == 0 || (mode == 1 ? cm != 0 : (cm & 1) != 0));
                cl = (in && (b & 0xC0) != 0x80) ? 1 : 0;   // code points, whatever the atoms
            }
            ast[u] = as; wst[u] = wsf; cpl[u] = cl;
            hi_byte |= in && (b & 0x80u) != 0;
            a_sum += as; w_sum += wsf; cp_sum += cl;
            if constexpr (GroupLDS<CH, G>::BSTREAM)
                if (!raw && in) L.bf[k] = (uint16_t)(b | (as ? BF_ATOM : 0u) | (wsf ? BF_STOP : 0u));
        }
        // one packed scan: atoms (9 bits) | words (9 bits) << 9 | code points (14 bits) << 18
        const unsigned v = a_sum | (w_sum << 9) | (cp_sum << 18);
        const unsigned incl = wave_incl_scan_add(v);
        const unsigned tot = __builtin_amdgcn_readlane(incl, 63);
        const unsigned ex = incl - v;
        const unsigned ai0 = n_atoms + (ex & 0x1FFu);
        unsigned wi = n_words + ((ex >> 9) & 0x1FFu);
        const unsigned cp0 = cp_tot + (ex >> 18);
        if (c0 + lane * 4 < wlen) *reinterpret_cast<uint32_t *>(&L.bytes[c0 + lane * 4]) = W.t[c];
        // the lane's atoms and their code-point prefixes
        unsigned aiu[4];
        {
            unsigned ai = ai0, cp = cp0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                aiu[u] = ai;
                const unsigned k = c0 + lane * 4 + u;
                if (ast[u]) {
                    L.aoff[ai] = (typename GroupLDS<CH, G>::Idx)k;
                    if constexpr (G == 16)   // end masks start all-dead (inverted); phase A clears token bits
                        reinterpret_cast<uint32_t *>(L.rec)[ai] = 0xFFFF0000u | cp | (wst[u] ? CP_WS : 0u);
                    else
                        L.rec[ai].cpos = (uint16_t)(cp | (wst[u] ? CP_WS : 0));
                }
                ai += ast[u] ? 1u : 0u;
                cp += cpl[u];
            }
        }
        if (c == 0)
#pragma unroll
            for (int u = 0; u < 4; u++) { ast0[u] = ast[u]; aiu0[u] = aiu[u]; }
        // (the 256-byte pass's word list lives in global scratch and is needed only by row-mode
        // windows: C0 rebuilds it there -- a store here would hold phase A's first loads back)
        if constexpr (!GroupLDS<CH, G>::WSLG) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (ast[u] && wst[u]) { L.set_word_start(gw, wi, aiu[u]); wi++; }
        }
        n_atoms += tot & 0x1FFu;
        n_words += (tot >> 9) & 0x1FFu;
        cp_tot += tot >> 18;
    }
    if (lane == 0) {
        if constexpr (GroupLDS<CH, G>::BSTREAM)
            if (!raw) L.bf[wlen] = (uint16_t)(BF_ATOM | BF_STOP);
        L.aoff[n_atoms] = (typename GroupLDS<CH, G>::Idx)wlen;
        if constexpr (G == 16) reinterpret_cast<uint32_t *>(L.rec)[n_atoms] = 0xFFFF0000u | cp_tot | CP_WS;
        else L.rec[n_atoms].cpos = (uint16_t)(cp_tot | CP_WS);
        if constexpr (!GroupLDS<CH, G>::WSLG) L.set_word_start(gw, n_words, n_atoms);
    }
    n_atoms_o = n_atoms;
    n_words_o = n_words;
    wave_sync();
    // PRESPLIT windows of llama mode's words (reference tokenizer_utils.py:24-31: SentencePiece pieces merged
    // by merge_tokens, every word after the BOS one starting with '\u2581' = E2 96 81): when the window's only
    // non-ASCII bytes are such '\u2581's, each exactly at a word start, every word start after byte 0 is one,
    // and no literal ' ' or '\n' is in it, the window is a raw-mode window in disguise -- '\u2581' then a
    // word, as raw mode's ' ' is.  It is stored compressed: atom j's byte at bytes[j] ('\u2581' as ' '),
    // aoff[j] = j; the rest of the first pass runs raw mode's ASCII paths on it (A0, the ASCII walker,
    // C2's bulk and hash passes with the ' ' -> '\u2581' expansion) without raw mode's first-atom rule
    // (SlotState::cpw).  Other PRESPLIT windows keep the generic path.
    if constexpr (G == 16 && CH == 256 && !WIDE) {
        if (mode == 1 && n_atoms > 0) {
            const uint32_t *b32 = reinterpret_cast<const uint32_t *>(L.bytes);
            const uint32_t w0 = b32[lane], w1 = b32[lane + 1u];   // (past the window: masked by wlen below)
            const uint32_t n1w = __builtin_amdgcn_alignbyte(w1, w0, 1u), n2w = __builtin_amdgcn_alignbyte(w1, w0, 2u);
            const uint32_t cmw = W.c[0];
            unsigned bad = 0, cnt = 0;   // cnt: bytes >= 0x80 | '\u2581's << 16
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const unsigned k = 4u * lane + (unsigned)u;
                const unsigned in = (unsigned)(k < wlen);
                const unsigned b = (w0 >> (8 * u)) & 0xFFu, n1 = (n1w >> (8 * u)) & 0xFFu, n2 = (n2w >> (8 * u)) & 0xFFu;
                const unsigned c = (cmw >> (8 * u)) & 0xFFu;
                const unsigned bar = in & (unsigned)(k + 2u < wlen) & (unsigned)(b == 0xE2u) & (unsigned)(n1 == 0x96u) &
                                     (unsigned)(n2 == 0x81u);
                const unsigned ws = in & (unsigned)(k > 0u) & (unsigned)(c != 0u) & (unsigned)((b & 0xC0u) != 0x80u);
                bad |= in & ((unsigned)(b == 0x20u) | (unsigned)(b == 0x0Au));
                bad |= ws & (bar ^ 1u);
                bad |= bar & (unsigned)(k > 0u) & (unsigned)(c == 0u);
                cnt += (in & (b >> 7)) | (bar << 16);
            }
            const unsigned tot = __builtin_amdgcn_readlane(wave_incl_scan_add(cnt), 63);
            if (!ballot(bad != 0u) && (tot & 0xFFFFu) == 3u * (tot >> 16)) {
                wave_sync();   // (every lane has read the bytes it tested)
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (ast0[u]) {
                        const unsigned b = (W.t[0] >> (8 * u)) & 0xFFu;
                        L.bytes[aiu0[u]] = (uint8_t)(b == 0xE2u ? 0x20u : b);
                        L.aoff[aiu0[u]] = (typename GroupLDS<CH, G>::Idx)aiu0[u];
                    }
                }
                if (lane == 0) L.aoff[n_atoms] = (typename GroupLDS<CH, G>::Idx)n_atoms;
                wave_sync();
                cpw_o = 1;
                return true;   // (atoms of one byte each)
            }
        }
    }
    // per-atom walk descriptor for phase A (parked in fin[], which phase B overwrites):
    //   byte offset | byte length << 12 | "a word or the window ends after it" << 16 | "first atom of the string" << 17
    const unsigned lim = WIDE ? MAX_ATOM_BYTES : 4u;   // RAW / PRESPLIT: code points (and '▁' + one fits 8 bytes)
    // RAW / PRESPLIT windows of ASCII bytes have one-byte atoms only: nothing to check, and
    // 16-lane rows park no descriptors
    if (G == 16 && !WIDE && !ballot(hi_byte)) return true;
    bool bad = false;
    for (unsigned j = lane; j < n_atoms; j += 64) {
        const unsigned p0 = L.aoff[j], la = L.atom_len(j);
        const unsigned stop = L.rec[j + 1].cpos >> 15;
        const unsigned first = (raw && pos == 0 && j == 0) ? 1u : 0u;
        bad |= la == 0 || la > lim;   // 0: a 256-byte atom, wrapped
        ainfo_set(L, j, AInfo<CH>::pack(p0, la, stop, first));
    }
    return ballot(bad) == 0;
}

// ------------------------------------------------------------------ the tokenize kernel

constexpr unsigned NPART = 16;   // first-pass work partitions (<= NPART_MAX)
static_assert(NPART >= 1 && NPART <= NPART_MAX, "NPART");
// First-pass partition p of npart over n strings: the FIN_BATCH-string chunks c with c % npart == p,
// in order.  part_size: its strings; part_string: the string at partition-local index v (< part_size).
// (32-bit arithmetic: a call has fewer than 2^31 strings)
__device__ __forceinline__ unsigned part_size(unsigned n, unsigned npart, unsigned p) {
    const unsigned nch = (n + FIN_BATCH - 1) / FIN_BATCH;
    if (nch <= p) return 0;
    // (uniform: readfirstlane keeps the VALU-lowered division out of an SGPR copy ROCm 7.2 rejects)
    const unsigned cnt = __builtin_amdgcn_readfirstlane((nch - 1 - p) / npart) + 1;   // chunks of p
    const unsigned last = p + (cnt - 1) * npart;               // its last chunk
    return cnt * FIN_BATCH - (last == nch - 1 ? nch * FIN_BATCH - n : 0);   // (only the batch's last chunk is short)
}
__device__ __forceinline__ unsigned part_string(unsigned npart, unsigned p, unsigned v) {
    return ((v / FIN_BATCH) * npart + p) * FIN_BATCH + v % FIN_BATCH;
}
#ifndef DPT_NEAR_CUT   // A/B knob: lane-mode B snaps chunk starts to the nearest cut point (else the next one)
#define DPT_NEAR_CUT 1
#endif
constexpr bool NEAR_CUT = DPT_NEAR_CUT != 0;
// (the 64-lane push recurrence keeps the next cut: nearest measured 0.9 % slower on BLOOM, r05e)
constexpr bool NEAR_CUT64 = false;
#ifndef DPT_A0_SWAR     // A/B knob: phase A0's per-byte flags four bytes per VALU op (bit 7 of each byte)
#define DPT_A0_SWAR 1
#endif
constexpr bool A0_SWAR = DPT_A0_SWAR != 0;
#ifndef DPT_BULK_U      // A/B knob: C2's bulk pass, tokens per lane per round (their lookups before their stores)
#define DPT_BULK_U 4
#endif
#ifndef DPT_HASH_BOTH   // A/B knob: C2's hash lookups load both buckets at once (0: the partner only on a miss)
#define DPT_HASH_BOTH 0
#endif
constexpr bool HASH_BOTH = DPT_HASH_BOTH != 0;
#ifndef DPT_HP_U        // A/B knob: C2 hash-pass token rounds of 64 per iteration (loads before stores)
#define DPT_HP_U 2
#endif
#ifndef DPT_A0_R2       // A/B knob: A0's third-byte round for walks that go on past two bytes
#define DPT_A0_R2 1
#endif
constexpr bool A0_R2 = DPT_A0_R2 != 0;
#ifndef DPT_A0_R2_MIN   // ... taken when at least this many lanes of the slot have such a walk
#define DPT_A0_R2_MIN 24
#endif
constexpr int A0_R2_MIN = DPT_A0_R2_MIN;
constexpr unsigned A_REFILL = 32;     // phase A: idle lanes needed before a batched refill (1/8/16/32 within 2 %)
constexpr unsigned A_REFILL64 = 32;   // the same for the 64-lane kernels (8 / 1: neutral / -0.5 %, r03aa)
#ifndef DPT_STOP     // diagnostic builds only (wrong results): 1 = prep only, 21 = + A0, 2 = + A, 25 / 26 / 27 =
                     // + lane-mode B's cut points / recurrence / transfer scan + fix-up, 3 = + B/C0/C1
#define DPT_STOP 9
#endif
#ifndef DPT_DIAG_PREP   // diagnostic builds only (cfg2-shaped input): 1 = static claims (no counter atomics),
#define DPT_DIAG_PREP 0  // 2 = offsets computed as 256 s (no str_off loads), 3 = both, 4 = a second dependent claim
#endif                   // atomic, 8 = no batch-sum atomics (wrong CSR offsets) -- the refill chain's and the atomics' cost
#ifndef DPT_C2STOP   // diagnostic builds only (wrong results): C2 stops after its bulk pass (1) / hash pass (2)
#define DPT_C2STOP 0
#endif
#define DPT_RUN_B (DPT_STOP >= 3 && DPT_STOP != 21)
#define DPT_RUN_C2 (DPT_STOP == 9)

// Waves per SIMD by VGPRs (<= 80 VGPRs each).  The 256-byte 16-lane rows: LDS (22 waves per CU) then
// binds (96 VGPRs / 5 waves: no scratch spills, cfg2 -1.9 %, r03e).  The 256-byte 64-lane kernel: BLOOM
// 17.4 -> 19.8 GB/s against no cap (95 VGPRs, 20 waves; 7 or 8 waves spill more: r03aa, r03ac).
#ifndef DPT_WPC_LO      // small calls: the persistent grid's fewest resident waves per CU (launch_tok)
#define DPT_WPC_LO 20
#endif
#ifndef DPT_WPC_GRAN    // LDS allocation granule (bytes) that caps the resident waves per CU (resident_per_cu)
#define DPT_WPC_GRAN 512
#endif
#ifndef DPT_PLAIN_RAW   // A/B knob: the RAW kernels without the edges / uncapped / len_only loop versions too
#define DPT_PLAIN_RAW 0
#endif
#ifndef DPT_WPE16
#define DPT_WPE16 6
#endif
constexpr int WPE16 = DPT_WPE16;
#ifndef DPT_WPE64
#define DPT_WPE64 6
#endif
constexpr int WPE64 = DPT_WPE64;
// The kernel's arguments, as one struct at the start of the kernarg segment
struct KernArgs {
    EncodeArgs ea;
    TrieView tv;
};
typedef __attribute__((address_space(4))) const KernArgs ConstKernArgs;
// Arguments are read through the kernarg segment pointer, which KREFRESH makes opaque at every phase
// boundary: each phase then loads (s_load, scalar-cache hits) the few arguments it uses instead of
// the compiler keeping all ~30 of them in SGPRs across the whole loop -- the hot kernel sits at the
// SGPR limit and spills.
// (a field-wise copy: only the fields a use reads are loaded)
__device__ __forceinline__ TrieView tv_of(ConstKernArgs *kp) {
    TrieView t;
    t.slots = kp->tv.slots; t.ids = kp->tv.ids; t.slots4 = kp->tv.slots4;
    t.root_base = kp->tv.root_base; t.n_slots = kp->tv.n_slots; t.pair16 = kp->tv.pair16;
    return t;
}
// (the 16-lane instantiations: the 64-lane ones do not spill, and measured 1.7 % slower with it)
#define KREFRESH() do { if constexpr (G == 16) asm volatile("" : "+s"(kp)); } while (0)

// Counter block (EncodeLaunch::retry_count, CTR_ALLOC_BYTES; zeroed once at allocation, then reset for
// the next call by the batch scan or the finish pass -- or, in a one-string host-path call, by the lone
// wave of the first pass): uint32 [0] retry count, [1] 2048-byte blocks done (fallback_kernel), [2]
// 2048-byte pass work, [3] long count, [4] long work, [5] the 512-byte pass's work (mid_kernel), [6]
// fallback_kernel's block ticket, [7] the 2048-byte pass's list count when the 512-byte pass ran; uint64 [4] (byte
// 32) the unbounded pass's claimed bytes, [5] (byte 40) the last call's claimed bytes
// (dpt_ctx_long_need), [6] (byte 48) far edge pairs found, [7] (byte 56) the last call's far edge pairs
// (dpt_dp_host_far); from byte PART_CTR_OFFSET the first pass's partition counters and their used-up
// mask (dpt_internal.h).
constexpr unsigned CTR_ARENA64 = 4, CTR_LASTNEED64 = 5, CTR_FAR64 = 6, CTR_LASTFAR64 = 7;

// Reset the counter block for the next call (the claimed arena bytes and far pairs stay readable as
// the call's "last need" / "last far").
// snap (nullable): the block's first 64 bytes as the host reads them after the call (the host path's
// one device-to-host copy carries them, instead of a copy of the counter block of its own)
__device__ __forceinline__ void reset_counters(uint32_t *ctr, uint64_t *snap = nullptr) {
    uint64_t *c64 = reinterpret_cast<uint64_t *>(ctr);
    c64[CTR_LASTNEED64] = c64[CTR_ARENA64];
    c64[CTR_ARENA64] = 0;
    c64[CTR_LASTFAR64] = c64[CTR_FAR64];
    c64[CTR_FAR64] = 0;
    if (snap)
        for (unsigned q = 0; q < 8; q++) snap[q] = c64[q];
    ctr[0] = 0; ctr[1] = 0; ctr[2] = 0; ctr[3] = 0; ctr[4] = 0; ctr[5] = 0; ctr[6] = 0; ctr[7] = 0;
    uint32_t *pc = ctr + PART_CTR_OFFSET / 4;
    for (unsigned q = 0; q <= NPART; q++) pc[q * PART_STRIDE] = 0;   // the partition counters and the mask
}

// SW: staged id width 0 = by a.staging16, 1 = int16, 2 = int32; RAW: DPT_MODE_RAW as a compile-time
// constant (its expansions and word starts fold away in the other modes' code and vice versa -- the
// 16-lane kernel sits at its register limit)
// The body of tokenize_kernel (and of fallback_kernel's 2048-byte blocks); bid: the block's index
// among the blocks running it.  The kernel arguments start with a KernArgs (read through the kernarg
// segment pointer, KREFRESH).
template <int CH, int G, bool BIG, bool WIDE, int SW = 0, bool RAW = false, bool SOLO = false, int MC = -1>
__device__ __forceinline__ void tokenize_body(const unsigned bid) {
    ConstKernArgs *kp = (ConstKernArgs *)__builtin_amdgcn_kernarg_segment_ptr();
#define a (kp->ea)
#define tv (tv_of(kp))
    constexpr int NG = 64 / G;
    using GL = GroupLDS<CH, G>;
    using GR = Group<G>;
    using M = typename GR::M;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr unsigned GSTR = (unsigned)group_stride<CH, G>();
    auto SSr = [&](unsigned g) -> SlotState & { return *reinterpret_cast<SlotState *>(smem + g * GSTR + group_lds_bytes<CH, G>()); };
    auto grp = [&](unsigned g) -> GL & { return *reinterpret_cast<GL *>(smem + g * GSTR); };
    auto wsl_of = [&](unsigned g) -> uint8_t * {
        return GL::WSLG ? a.wsl_scratch + ((size_t)bid * NG + g) * GL::WSL_STRIDE : nullptr;
    };

    const unsigned lane = lane_id();
    const unsigned mg = lane / G;        // my group
    const unsigned d = lane % G;         // my back distance - 1
    const uint64_t n_work = BIG ? (uint64_t)(*a.work_count) : a.n_str;
    if constexpr (BIG)
        if (a.hist_zero && bid == 0)
            for (uint32_t b = lane; b < a.n_hist; b += 64u) a.hist_zero[b] = 0;
    if (BIG && n_work == 0) return;   // no retries: no counter traffic
    const uint64_t base_off = a.str_off[0];
    // (the other instantiations keep the mode a run-time value: folding raw = false into the atoms-mode
    // 16-lane kernel crashes ROCm 7.2's greedy register allocator)
    // RAW / MC >= 0: the mode as a compile-time constant (PRESPLIT, ATOMS; the other instantiations read it)
    const int mode = RAW ? 0 : (MC >= 0 ? MC : (a.mode & DPT_MODE_MASK));
    const bool raw = mode == 0;
    // PLAIN: the mode-constant instantiations serve only calls without edges, the uncapped DP or len_only
    // (launch_encode sends those to the runtime-mode kernels): their loop versions are compiled out
    constexpr bool PLAIN = ((RAW && DPT_PLAIN_RAW) || MC >= 0) && !SOLO;
    const bool uncapped = !PLAIN && (a.mode & DPT_FLAG_UNCAPPED) != 0;   // f2: inspect_tokenizer's inf-initialised DP
    const bool len_only = !PLAIN && (a.mode & (DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY)) != 0;
    // Strings are handed out by npart device counters (each in its own 256-byte line).  Partition p
    // holds the FIN_BATCH-string chunks p, p + npart, p + 2 npart, ... of the batch, in that order
    // (part_size / part_string): the partitions advance through the batch side by side, so strings
    // finish roughly in batch order.  A wave claims as many strings as it has free slots from its current partition (starting on
    // blockIdx mod npart) and, when a claim reaches the partition's end, marks the partition in a
    // shared mask and moves to the next unmarked one.  Round 1's single counter (one same-address
    // atomic per refill) bound the whole kernel: a prep-only build ran 2.91 of the full build's 2.99
    // ms, every wave queued behind ~5.6k others' atomics (profiles/r02_phase_diag.txt).  No string is
    // claimed ahead of a free slot: strings held in reserve by one wave left others idle at the end
    // of multi-window batches (cfg4 4.35 -> 4.56 ms with 4-string claims).
    const unsigned npart = (BIG || (DPT_DIAG_PREP & 1)) ? 1u : (unsigned)min((uint64_t)NPART, max((uint64_t)1, n_work / 4096u));
    [[maybe_unused]] uint64_t diag_k = 0;   // DPT_DIAG_PREP & 1: the wave's claims so far
    unsigned part = BIG ? 0u : bid % npart;
    bool exhausted = false, claimed_all = false;
    unsigned n_pend = 0;   // 16-lane first pass: residual tokens waiting in the wave's pending row
    // one claim of up to req strings (uniform): partition-local [nb, ne) of partition cp, possibly
    // empty once every partition is used up
#ifdef DPT_WSTAMPS
    unsigned wst_claims = 0;
#define WST_CLAIM() (wst_claims++)
#else
#define WST_CLAIM()
#endif
    auto claim = [&](unsigned req, uint64_t &nb, uint64_t &ne, unsigned &cp) {
        for (;;) {
            WST_CLAIM();
            uint32_t *ctr = BIG ? a.work_next : a.part_ctr + part * PART_STRIDE;
            const uint64_t hi = BIG ? n_work : part_size((unsigned)n_work, npart, part);
            unsigned b = 0;
            if constexpr (!BIG && (DPT_DIAG_PREP & 1)) {   // diagnostic: wave bid's k-th claim, blocks of 4
                b = (unsigned)((diag_k * gridDim.x + bid) * 4u);
                diag_k++;
            } else {
                if (lane == 0) b = atomicAdd(ctr, req);
                if constexpr (!BIG && (DPT_DIAG_PREP & 4)) {   // diagnostic: one more dependent atomic round trip
                    unsigned x = 0;
                    asm volatile("" : "+v"(b));
                    if (lane == 0) x = atomicAdd(ctr + (b >> 31), 0u);
                    asm volatile("" : "+v"(x));
                    b |= (x >> 31) << 31;
                }
            }
            cp = __builtin_amdgcn_readfirstlane(part);
            nb = (uint32_t)__builtin_amdgcn_readlane(b, 0);
            ne = nb < hi ? (nb + req < hi ? nb + req : hi) : nb;
            if (nb + req >= hi) {   // the partition is used up (by this claim or earlier ones)
                if (BIG) {
                    claimed_all = true;
                } else {
                    unsigned m = 0;
                    if (lane == 0) m = atomicOr(a.part_ctr + (unsigned)NPART * PART_STRIDE, 1u << part);
                    m = __builtin_amdgcn_readlane(m, 0) | (1u << part);
                    const unsigned all = (npart >= 32u ? 0u : (1u << npart)) - 1u;
                    if ((m & all) == all) {
                        claimed_all = true;
                    } else {   // the next unmarked partition after this one
                        const unsigned free = ~m & all;
                        const unsigned hi_free = free & ~((2u << part) - 1u);
                        part = (unsigned)__builtin_ctz(hi_free ? hi_free : free);
                    }
                }
            }
            if (ne > nb || claimed_all) return;
        }
    };
    // The wave's pending residual tokens (16-lane first pass, C2): one walk per lane from the entry's
    // bytes -- the C2 walker's byte rule (atom_from_info: raw mode expands the string's first atom to
    // '\u2581' + its bytes, ' ' to '\u2581', '\n' to "<0x0A>") as a byte generator, so one trie step
    // per expanded byte from one call site -- starting at the node after '\u2581' when the token
    // starts with it; the id of the node reached when every step's check held, else -1.  Entry:
    // staging element (.x, .y bits 0..15), byte length (.y bits 16..23, <= 8), first atom of the
    // string (.y bit 24), raw mode's expansions (.y bit 25: raw mode, or a '\u2581'-compressed PRESPLIT
    // window), the bytes (.z, .w).
    auto walk_pending = [&](unsigned P) {
        wave_sync();   // the entries other lanes stored
        if (lane < P) {
            const uint4 e = a.pend[(uint64_t)bid * 64u + lane];
            const uint64_t out = (uint64_t)e.x | ((uint64_t)(e.y & 0xFFFFu) << 32);
            const unsigned len = (e.y >> 16) & 0xFFu;
            const bool raw = RAW || ((e.y >> 25) & 1u);   // (shadows the mode's: this token's bytes)
            const bool fi = raw && ((e.y >> 24) & 1u);
            const uint64_t by = (uint64_t)e.z | ((uint64_t)e.w << 32);
            const unsigned b0 = (unsigned)(by & 0xFFu);
            const bool ws = (fi || (raw && b0 == ' ')) && a.ws_node >= 0;
            int32_t node = ws ? a.ws_node : 0, nb = ws ? a.ws_base : tv.root_base, id = ws ? a.ws_id : -1;
            bool ok = true;
            unsigned k = (ws && !fi) ? 1u : 0u;   // ws: '\u2581' is consumed (a first atom still emits its bytes)
            uint64_t pnd = 0;
            unsigned pc = 0;
            while (k < len || pc) {
                if (!pc) {
                    const unsigned b = (unsigned)(by >> (8u * k)) & 0xFFu;
                    const bool first = k == 0 && fi;
                    pnd = b; pc = 1;
                    if (first && !ws) { pnd = 0x8196E2ull | ((uint64_t)b << 24); pc = 4; }
                    else if (!first && raw && b == ' ') { pnd = 0x8196E2ull; pc = 3; }
                    else if (!first && raw && b == '\n') { pnd = 0x3E413078303Cull; pc = 6; }
                    k++;
                }
                const int32_t sl = nb + (int32_t)(pnd & 0xFFu);
                pnd >>= 8;
                pc--;
                const int4 en = trie_slot4(tv, sl);
                ok = ok && en.y == node;
                node = sl;
                nb = en.x & BASE_MASK;
                id = en.z;
            }
            id = ok ? id : -1;
            if (SW == 1 || (SW == 0 && a.staging16 != nullptr)) a.staging16[out] = (int16_t)id;
            else a.staging[out] = id;
        }
    };

    STAMP_DECL
    WST_REC(0, WST_NOW());
    [[maybe_unused]] unsigned wst_it = 0;

    if (lane < (unsigned)NG) SSr(lane).active = 0;
    wave_sync();

    for (;;) {
        KREFRESH();
        // ---------------------------------------------------------- slots: fetch strings, find windows, prep
        // Inactive slots are refilled together (one counter atomic, offsets loaded by one lane
        // per slot), and every slot's window bytes are loaded before any is atomised, so the
        // HBM round trips of the NG slots overlap.
        unsigned busy = 0, prepared = 0;
        for (;;) {
            unsigned need = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) need |= uni(SSr(g).active) ? 0u : (1u << g);
            if (need && !exhausted) {
                // claims until every free slot has a string or every partition is used up (a claim
                // that reaches a partition's end may return fewer strings than asked)
                unsigned rem = need;
                // partition-local strings [nb, ne) of partition cp into the free slots of rem, in order
                auto assign = [&](uint64_t nb, uint64_t ne, unsigned cp) {
                    const unsigned got = (unsigned)(ne - nb);
                    if (lane < (unsigned)NG && ((rem >> lane) & 1u)) {
                        const unsigned k = (unsigned)__builtin_popcount(rem & ((1u << lane) - 1u));
                        if (k < got) {
                            const uint64_t idx = nb + k;
                            const uint64_t s = BIG ? (uint64_t)a.work_list[idx] : part_string(npart, cp, (unsigned)idx);
                            uint64_t o0, o1;
                            if constexpr (!BIG && (DPT_DIAG_PREP & 2)) { o0 = s * 256u; o1 = o0 + 256u; }   // diagnostic (cfg2)
                            else { o0 = a.str_off[s]; o1 = a.str_off[s + 1]; }
                            SlotState &S = SSr(lane);
                            S.s = (uint32_t)s; S.sb = o0 - base_off; S.slen = (uint32_t)(o1 - o0); S.pos = 0; S.active = 1;
                            S.status = o1 == o0 ? 2u : 0u;  // pretokenize_raw('') == [[]] -> IndexError
                            S.ntok = 0; S.capsum = 0; S.abase = 0;
                        }
                    }
                    for (unsigned q = 0; q < got; q++) rem &= rem - 1u;   // those slots are filled
                };
                while (rem && !claimed_all) {
                    const unsigned n_need = (unsigned)__builtin_popcount(rem);
                    uint64_t nb = 0, ne = 0;
                    unsigned cp = 0;
                    claim(n_need, nb, ne, cp);
                    assign(nb, ne, cp);
                }
                if (claimed_all) exhausted = true;
                wave_sync();
            }
            unsigned todo = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) todo |= (uni(SSr(g).active) && !((prepared >> g) & 1u)) ? (1u << g) : 0u;
            if (!todo) break;
            WinRegs<CH> W[NG];
#pragma unroll
            for (int g = 0; g < NG; g++) {
                if (!((todo >> g) & 1u)) continue;
                const uint64_t sb = uni64(SSr(g).sb);
                load_window<CH>(W[g], a.text + sb, raw ? nullptr : a.cut_mask + sb, uni64(SSr(g).pos), uni64(SSr(g).slen), raw, lane);
            }
            bool refill = false;
#pragma unroll
            for (int g = 0; g < NG; g++) {
                if (!((todo >> g) & 1u)) continue;
                GL &L = grp(g);
                SlotState &S = SSr(g);
                const uint64_t slen = uni64(S.slen), pos = uni64(S.pos);
                unsigned status = uni(S.status);
                unsigned wlen = 0, na = 0, nw = 0, cpw = 0;
                bool ok = status != 2;
                if (ok) ok = window_bounds<CH>(W[g], slen, pos, mode, lane, wlen);
                if (ok) ok = prep_window<CH, G, WIDE>(L, wsl_of(g), W[g], pos, wlen, mode, lane, na, nw, cpw);
                if (ok) {
                    if (lane == 0) { S.wlen = wlen; S.n_atoms = na; S.n_words = nw; S.wtok = 0; S.inval = 0; S.capb = 0; S.cpw = (uint8_t)cpw; }
                    prepared |= 1u << g;
                    busy++;
                    continue;
                }
                // the string ends here: empty, or a word (or atom) too long for this pass -- the
                // 2048-byte pass retries it, then the unbounded pass (status 3 is overwritten there)
                if (status != 2) status = 3;
                if (lane == 0) {
                    const uint64_t s = S.s;
                    if (status == 3) {
                        // (the 512-byte pass, mid_kernel: its retry_* fields are the 2048-byte pass's list)
                        uint32_t *cnt = (BIG && CH > 512) ? a.long_count : a.retry_count;
                        uint32_t *lst = (BIG && CH > 512) ? a.long_list : a.retry_list;
                        lst[atomicAdd(cnt, 1u)] = (uint32_t)s;
                    }
                    a.status[s] = (int32_t)status;
                    if (a.capped) a.capped[s] = status == 2 ? 0 : -1;
                    S.active = 0;
                    a.counts[s] = 0;
                }
                refill = true;
            }
            wave_sync();
            if (!refill || exhausted) break;
        }
        if (lane < (unsigned)NG && !((prepared >> lane) & 1u)) { SSr(lane).n_atoms = 0; SSr(lane).n_words = 0; SSr(lane).capb = 0; }
        wave_sync();
        if (busy == 0) break;
        STAMP(0);

        // ---------------------------------------------------------- A: match discovery (all slots)
        KREFRESH();
        if (DPT_STOP > 1) {
            // A0 (16-lane rows, raw mode): slots whose window is pure ASCII -- atoms are its bytes --
            // get every walk's first lookup here, byte-parallel with four loads in flight per lane;
            // the walks it cannot finish (word starts, the string's first atom, '\n', and walks that
            // go on past the two-byte root entry: ~6 % in cfg2 with the child filters) are marked
            // (bit 4g + u of `mark`: atom 4 * lane + u of slot g) and redone by the walker below,
            // which also takes every atom of the other slots.
            unsigned a0mask = 0;
            uint32_t mark = 0;
            if constexpr (G == 16 && !BIG) {
                if (!raw) {   // PRESPLIT: the '\u2581'-compressed windows (prep_window)
#pragma unroll
                    for (int g = 0; g < NG; g++)
                        if (uni(SSr(g).n_atoms) > 0 && uni(SSr(g).cpw)) a0mask |= 1u << g;
                } else {
#pragma unroll
                    for (int g = 0; g < NG; g++) {
                        const unsigned wl = uni(SSr(g).n_atoms) > 0 ? uni(SSr(g).wlen) : 0u;
                        const uint32_t *b32 = reinterpret_cast<const uint32_t *>(grp(g).bytes);
                        const uint32_t w0 = 4u * lane < wl ? b32[lane] : 0u;
                        const unsigned nv = wl > 4u * lane ? min(wl - 4u * lane, 4u) : 0u;   // valid bytes in w0
                        const uint32_t hi = w0 & (nv >= 4u ? 0x80808080u : ((1u << (8u * nv)) - 1u) & 0x80808080u);
                        if (wl && !ballot(hi != 0)) a0mask |= 1u << g;
                    }
                }
            }
            unsigned nstart[NG];   // walker starts per slot: all atoms, or A0's marked ones
#pragma unroll
            for (int g = 0; g < NG; g++) nstart[g] = uni(SSr(g).n_atoms);
            unsigned fwmask = 0;   // slots whose window starts the string (raw: '▁' + first atom)
#pragma unroll
            for (int g = 0; g < NG; g++) fwmask |= (raw && uni(SSr(g).pos) == 0 ? 1u : 0u) << g;
            // One walk per lane.  Walk state: start atom j, the LDS byte offset of its slot's group,
            // atoms matched so far (len), the trie node, the expanded bytes left of the current atom
            // (seq, cnt) and its descriptor (info).  Finished walks take the next start (ballot +
            // mbcnt), so the wave stays busy.
            unsigned j = 0, lbase = 0, len = 0, cnt = 0, info = 0, t2 = 0, gsel = 0;
            unsigned capm = 0;   // bit g: slot g's capb (set after the walks)
            bool split = false;
            int32_t nb = tv.root_base, node = 0;
            uint64_t seq = 0;
            M mask = 0;   // G = 16: bit 0 only (the single-atom span is a token)
            // G = 16: the span of len atoms ending at end position e is a token: clear bit len-1
            // of e's inverted end mask (the high half of rec[e]; one LDS atomic, no return)
            auto end_token = [&](unsigned e, unsigned ln) {
                uint32_t *r32 = reinterpret_cast<uint32_t *>(smem + lbase);
                __hip_atomic_fetch_and(&r32[e], ~(1u << (15u + ln)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            auto end_token_at = [&](unsigned lb, unsigned e, unsigned ln) {   // (the group at LDS byte lb)
                uint32_t *r32 = reinterpret_cast<uint32_t *>(smem + lb);
                __hip_atomic_fetch_and(&r32[e], ~(1u << (15u + ln)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            auto grp_bytes_at = [&](unsigned lb, unsigned p) -> unsigned {   // window byte p (p < CH + 16) of that group
                return reinterpret_cast<const GL *>(smem + lb)->bytes[p];
            };
            auto start_gj = [&](unsigned gs, unsigned jj) {
                j = jj;
                gsel = gs;
                lbase = gs * GSTR;
                const GL &L = *reinterpret_cast<const GL *>(smem + lbase);
                info = ainfo_get(L, j, raw && ((fwmask >> gs) & 1u));
                seq = atom_from_info<CH, WIDE>(L.bytes, info, raw, cnt);
                nb = tv.root_base; node = 0; len = 0; mask = 0;
                // The first two expanded bytes go through one lookup of the two-byte root table
                // (TrieView): within atom j, or across its end when the word continues (then
                // atom j+1 is loaded now instead of at the first atom end).
                const unsigned b0 = (unsigned)(seq & 0xFFu);
                if (cnt >= 2) {
                    t2 = tv.n_slots + (b0 << 8) + (unsigned)((seq >> 8) & 0xFFu);
                    split = false;
                    seq >>= 16;
                    cnt -= 2;
                } else if (!(info & AInfo<CH>::STOP)) {
                    info = ainfo_get(L, j + 1, false);
                    seq = atom_from_info<CH, WIDE>(L.bytes, info, raw, cnt);
                    t2 = tv.n_slots + (b0 << 8) + (unsigned)(seq & 0xFFu);
                    split = true;
                    seq >>= 8;
                    cnt -= 1;
                } else {
                    t2 = 0;
                }
            };
            if constexpr (G == 16 && !BIG) {
                if (a0mask) {
                    constexpr unsigned END = 0x100u;
#pragma unroll
                    for (int g = 0; g < NG; g++) {
                        if (!((a0mask >> g) & 1u)) continue;
                        // (window bytes in LDS = atoms: raw ASCII windows and '\u2581'-compressed ones alike)
                        const unsigned wl = uni(SSr(g).n_atoms);
                        const bool first = raw && uni(SSr(g).pos) == 0;
                        const unsigned gbase = (unsigned)g * GSTR;
                        const uint32_t *b32 = reinterpret_cast<const uint32_t *>(grp(g).bytes);
                        const unsigned k0 = 4u * lane;
                        if constexpr (A0_SWAR) {
                            // The lane's four bytes as one 32-bit word (SWAR): every per-byte flag is bit 7 of
                            // its byte, so one VALU op tests four bytes.  Views: w0 = bytes k0..k0+3 (b), n1w =
                            // k0+1.. (the next byte), n2w = k0+2.. (the one after).
                            constexpr uint32_t H = 0x80808080u;
                            const uint32_t w0 = b32[lane], w1 = b32[lane + 1u];
                            const uint32_t n1w = __builtin_amdgcn_alignbyte(w1, w0, 1u);
                            const uint32_t n2w = __builtin_amdgcn_alignbyte(w1, w0, 2u);
                            // lookups at (b, n1) as read: the table holds (b, '<')'s entry at (b, '\n') too,
                            // and (b, END)'s flags of b are (b, anything)'s (dpt_api.cpp)
                            uint2 ent[4];
#pragma unroll
                            for (int u = 0; u < 4; u++)
                                ent[u] = reinterpret_cast<const uint2 *>(tv.pair16 + PAIR16_N)[
                                    __builtin_amdgcn_perm(w0, n1w, 0x0C0C0000u | ((4u + (unsigned)u) << 8) | (unsigned)u)];
                            // bytes past the window (END): byte q of the 8 is valid while q < nv
                            const unsigned nv = wl > k0 ? min(wl - k0, 8u) : 0u;
                            const uint64_t vm = nv >= 8u ? ~0ull : ((1ull << (8u * nv)) - 1ull);
                            const uint32_t vlo = (uint32_t)vm, vhi = (uint32_t)(vm >> 32);
                            const uint32_t v0 = vlo & H, v1 = __builtin_amdgcn_alignbyte(vhi, vlo, 1u) & H,
                                           v2 = __builtin_amdgcn_alignbyte(vhi, vlo, 2u) & H;
                            auto eq80 = [](uint32_t x, uint32_t c) -> uint32_t {   // bit 7 of each byte of x equal to c's
                                const uint32_t t = x ^ c;
                                return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
                            };
                            const uint32_t sp0 = eq80(w0, 0x20202020u), sp1w = eq80(w1, 0x20202020u);
                            const uint32_t nl0 = eq80(w0, 0x0A0A0A0Au), nl1w = eq80(w1, 0x0A0A0A0Au);
                            const uint32_t sp1 = __builtin_amdgcn_alignbyte(sp1w, sp0, 1u), sp2 = __builtin_amdgcn_alignbyte(sp1w, sp0, 2u);
                            const uint32_t nl1 = __builtin_amdgcn_alignbyte(nl1w, nl0, 1u), nl2 = __builtin_amdgcn_alignbyte(nl1w, nl0, 2u);
                            const uint32_t special = sp0 | nl0 | ((first && lane == 0) ? 0x80u : 0u);   // the walker's
                            const uint32_t norm = v0 & ~special;
                            const uint32_t cont = v1 & ~sp1;   // n1 is in the word
                            // the entries' flag bytes side by side (bit 0 root child, 1 b a token, 2 node b n1,
                            // 3 it ends a token, 4 it is a leaf) and their child-filter bits for n2
                            const uint32_t xs = __builtin_amdgcn_perm(ent[1].x, ent[0].x, 0x0C0C0400u) |
                                                (__builtin_amdgcn_perm(ent[3].x, ent[2].x, 0x0C0C0400u) << 16);
                            const uint32_t cb = n2w ^ ((n2w >> 5) & 0x07070707u);   // child_bit(byte) in each byte's low 5 bits
                            const uint32_t f0 = ent[0].y >> (cb & 31u), f1 = ent[1].y >> ((cb >> 8) & 31u),
                                           f2 = ent[2].y >> ((cb >> 16) & 31u), f3 = ent[3].y >> ((cb >> 24) & 31u);
                            const uint32_t fb = (__builtin_amdgcn_perm(f1, f0, 0x0C0C0400u) |
                                                 (__builtin_amdgcn_perm(f3, f2, 0x0C0C0400u) << 16)) << 7;
                            const uint32_t tok1 = (xs << 7) & (xs << 6);
                            const uint32_t has2 = norm & cont & (xs << 5);
                            // go on past two bytes: n2 in the word with a child for it; '\n' at n1 or n2 ("<0x0A>")
                            // always (the walker redoes such starts whole)
                            const uint32_t more = has2 & ~(xs << 3) & (nl1 | (v2 & (nl2 | (~sp2 & fb))));
                            const uint32_t tk1 = norm & tok1;                  // a one-atom token ends at k0+1+u
                            const uint32_t tk2 = has2 & ~nl1 & (xs << 4);      // a two-atom token ends at k0+2+u
                            uint32_t mk = ((v0 & special) | more) & H;   // walker starts
                            if constexpr (A0_R2) {
                                // Third-byte round: a walk that goes on past two plain bytes of the word takes
                                // its root-table step (the node after the pair) and its third step here,
                                // byte-parallel, and stays for the walker only if it goes on past three
                                // (cfg4: ~97 % of these walks end there).  The three-atom token, if any, is
                                // recorded here.  Slots with few such walks leave them to the walker.
                                const uint32_t r2 = more & ~nl1 & ~nl2 & H;
                                if (__builtin_popcountll(ballot(r2 != 0)) >= A0_R2_MIN) {
                                    const uint32_t v3 = __builtin_amdgcn_alignbyte(vhi, vlo, 3u) & H;
                                    const uint32_t sp3 = __builtin_amdgcn_alignbyte(sp1w, sp0, 3u);
                                    const uint32_t nl3 = __builtin_amdgcn_alignbyte(nl1w, nl0, 3u);
                                    const uint32_t n3w = __builtin_amdgcn_alignbyte(w1, w0, 3u);
                                    constexpr int32_t OOB = 0x7FFFFFF;   // past the table: the buffer load returns zeros
                                    int4 e2r[4], e3[4];
#pragma unroll
                                    for (int u = 0; u < 4; u++)   // the root table's entry of (b, n1)
                                        e2r[u] = trie_slotA(tv, ((r2 >> (8 * u + 7)) & 1u) ? (int32_t)(tv.n_slots +
                                                 __builtin_amdgcn_perm(w0, n1w, 0x0C0C0000u | ((4u + (unsigned)u) << 8) | (unsigned)u)) : OOB);
#pragma unroll
                                    for (int u = 0; u < 4; u++)   // the node after n2
                                        e3[u] = trie_slotA(tv, ((r2 >> (8 * u + 7)) & 1u) ?
                                                (int32_t)((e2r[u].x & BASE_MASK) + ((n2w >> (8 * u)) & 0xFFu)) : OOB);
                                    uint32_t c3 = 0, t3 = 0;
#pragma unroll
                                    for (int u = 0; u < 4; u++) {
                                        const unsigned n3 = (n3w >> (8 * u)) & 0xFFu;
                                        const unsigned ok3 = ((r2 >> (8 * u + 7)) & 1u) & (unsigned)(e3[u].y == (e2r[u].y & 0x3FFFFFFF));
                                        const unsigned leaf3 = ((unsigned)e3[u].x >> 30) & 1u;
                                        const unsigned in3 = ((v3 & ~sp3) >> (8 * u + 7)) & 1u;
                                        const unsigned ch3 = (((unsigned)e3[u].w >> child_bit(n3)) & 1u) | ((nl3 >> (8 * u + 7)) & 1u);
                                        t3 |= (ok3 & ((unsigned)e3[u].x >> 31)) << (8 * u + 7);
                                        c3 |= (ok3 & (leaf3 ^ 1u) & in3 & ch3) << (8 * u + 7);
                                    }
                                    mk = ((v0 & special) | (more & ~r2) | c3) & H;
                                    if (ballot(t3 != 0)) {   // a three-atom token ends at k0+3+u
                                        uint32_t *q32 = reinterpret_cast<uint32_t *>(smem + gbase);
#pragma unroll
                                        for (int u = 0; u < 4; u++)
                                            __hip_atomic_fetch_and(&q32[k0 + 3u + u],
                                                                   ~(((t3 >> (8 * u + 7)) & 1u) << 18),
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    }
                                }
                            }
                            const uint32_t t2e = (tk2 << 8) | wave_shift_in(tk2 >> 24, 0u);
                            // end k0+1+u: bit 0 of byte u of d a one-atom token, bit 1 a two-atom one
                            const uint32_t d = ((tk1 & H) >> 7) | ((t2e & H) >> 6);
                            uint32_t *r32 = reinterpret_cast<uint32_t *>(smem + gbase);
                            if (ballot(d != 0)) {
#pragma unroll
                                for (int u = 0; u < 4; u++)
                                    __hip_atomic_fetch_and(&r32[k0 + 1u + u], ~(((d >> (8 * u)) & 3u) << 16),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                            if (ballot((norm & ~tok1) != 0) && lane == 0) SSr(g).capb = 1;
                            // the slot's marked atoms, in order, into its fin[] (free until phase B)
                            const unsigned c = (unsigned)__builtin_popcount(mk);
                            const unsigned incl = wave_incl_scan_add(c);
                            unsigned o = incl - c;
                            GL &Lg = grp(g);
#pragma unroll
                            for (int u = 0; u < 4; u++)
                                if ((mk >> (8 * u + 7)) & 1u) Lg.fin[o++].v = (uint8_t)(k0 + (unsigned)u);
                            nstart[g] = __builtin_amdgcn_readlane(incl, 63);
                            continue;
                        }
                        // bytes k0 .. k0+7 (past the window: masked by wl below)
                        const uint64_t w = (uint64_t)b32[lane] | ((uint64_t)b32[lane + 1u] << 32);
                        auto byte_at = [&](unsigned q) -> unsigned {   // byte k0+q, END past the window
                            return k0 + q < wl ? (unsigned)((w >> (8u * q)) & 0xFFu) : END;
                        };
                        uint32_t *r32 = reinterpret_cast<uint32_t *>(smem + gbase);
                        bool nocap = false;
                        unsigned tk1 = 0, tk2 = 0;
                        // the packed byte-pair table over (byte, next byte): the flags of the first byte do
                        // not depend on the second; four lookups in flight per lane
                        uint2 ent[4];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const unsigned b = byte_at(u), n1 = byte_at(u + 1);
                            const unsigned e1 = n1 == '\n' ? (unsigned)'<' : n1;
                            ent[u] = reinterpret_cast<const uint2 *>(tv.pair16 + PAIR16_N)[((b & 0xFFu) << 8) | (e1 & 0xFFu)];
                        }
                        // Per byte: tk1 bit u = a one-atom token ends at k0+1+u, tk2 bit u = a two-atom
                        // token ends at k0+2+u (the end masks are written once below)
                        // (flags as 0/1 integers combined with & and |: short-circuit forms become
                        // exec-mask branches here)
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const unsigned k = k0 + (unsigned)u;
                            const unsigned b = byte_at(u), n1 = byte_at(u + 1), n2 = byte_at(u + 2);
                            const auto e = ent[u];
                            const unsigned valid = (unsigned)(b != END);
                            const unsigned special = (unsigned)(b == ' ') | (unsigned)(b == '\n') | ((unsigned)first & (unsigned)(k == 0));   // the walker's
                            const unsigned norm = valid & (special ^ 1u);
                            // n1 ends the word: the lookup was the atom's own root slot
                            const unsigned wend = (unsigned)(n1 == END) | (unsigned)(n1 == ' ');
                            const unsigned xterm = ((unsigned)e.x >> 3) & 1u, xleaf = ((unsigned)e.x >> 4) & 1u;
                            const unsigned tok1 = (unsigned)e.x & ((unsigned)e.x >> 1) & 1u;
                            const unsigned node2 = ((unsigned)e.x >> 2) & 1u;
                            const unsigned filt = (unsigned)e.y;
                            nocap |= (norm & (tok1 ^ 1u)) != 0;
                            // a node after two bytes: n1 = '\n' leaves the walk inside "<0x0A>" after
                            // its '<'; otherwise atom k+1 is consumed (the span k .. k+2)
                            const unsigned has2 = norm & (wend ^ 1u) & node2;
                            const unsigned nl1 = (unsigned)(n1 == '\n');
                            const unsigned e2 = nl1 ? (unsigned)'0' : (n2 == '\n' ? (unsigned)'<' : n2);
                            const unsigned more = has2 & (xleaf ^ 1u) & (nl1 | ((unsigned)(n2 != END) & (unsigned)(n2 != ' '))) &
                                                  ((filt >> child_bit(e2)) & 1u);
                            tk1 |= (norm & tok1) << u;
                            tk2 |= (has2 & (nl1 ^ 1u) & xterm) << u;
                            mark |= ((valid & special) | more) << (4 * g + u);
                        }
                        // end k0+1+u: tk1 bit u, and tk2 bit u-1 (u = 0: the previous lane's bit 3)
                        const unsigned t2e = ((tk2 << 1) & 0xEu) | wave_shift_in((tk2 >> 3) & 1u, 0u);
                        if (ballot((tk1 | t2e) != 0)) {
                            // (lane l's dwords are 4l+1 .. 4l+4: lanes l, l+8, l+16, l+24 of a 32-lane group hit
                            // one bank; a rotated order (r03) and a transposed one -- round q's lane l taking
                            // end 64q+l+1, its bits gathered by ds_bpermute (r04) -- cost VGPR spills instead)
#pragma unroll
                            for (int u = 0; u < 4; u++)
                                __hip_atomic_fetch_and(&r32[k0 + 1u + u], ~((((tk1 >> u) & 1u) << 16) | (((t2e >> u) & 1u) << 17)),
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        if (ballot(nocap) && lane == 0) SSr(g).capb = 1;
                        // the slot's marked atoms, in order, into its fin[] (free until phase B)
                        const unsigned mg = (mark >> (4 * g)) & 15u;
                        const unsigned c = (unsigned)__builtin_popcount(mg);
                        const unsigned incl = wave_incl_scan_add(c);
                        unsigned o = incl - c;
                        GL &Lg = grp(g);
#pragma unroll
                        for (int u = 0; u < 4; u++)
                            if ((mg >> u) & 1u) Lg.fin[o++].v = (uint8_t)(k0 + (unsigned)u);
                        nstart[g] = __builtin_amdgcn_readlane(incl, 63);
                    }
                }
            }
            // ASCII walker: the marked starts of A0 slots (pure-ASCII raw windows: an atom is one byte, a
            // word start ' ' is '\u2581' = the trie node ws_node, '\n' is "<0x0A>", the string's first
            // atom '\u2581' + its byte) walked byte by byte without the generic walker's atom
            // descriptors.  A "more" start (a plain byte whose walk goes past A0's two-byte lookup, its one-
            // and two-atom tokens already recorded by A0) repeats that lookup in the root table and goes on
            // from the node after two bytes.  The generic walker below takes the other slots.
            if constexpr (G == 16 && !BIG) {
                if (a0mask) {
                    unsigned fpre[NG + 1];
                    fpre[0] = 0;
#pragma unroll
                    for (int g = 0; g < NG; g++) {
                        fpre[g + 1] = fpre[g] + (((a0mask >> g) & 1u) ? nstart[g] : 0u);
                        if ((a0mask >> g) & 1u) nstart[g] = 0;
                    }
                    const unsigned ftotal = fpre[NG];
                    const int32_t wsn = a.ws_node, wsb = a.ws_base;
                    const unsigned wst = a.ws_id >= 0 ? 1u : 0u;   // '\u2581' alone is a token
                    const int32_t rb = tv.root_base;
                    const unsigned nsl = tv.n_slots;
                    // "<0x0A>" after its '<': with pc bytes left the next is byte 5 - pc of "0x0A>" (a 32-bit
                    // constant and '>' instead of a 64-bit register pair of the bytes still to come)
                    auto nl_byte = [](unsigned pc) -> unsigned { return pc >= 2u ? (0x41307830u >> (8u * (5u - pc))) & 0xFFu : 0x3Eu; };
                    unsigned fj = 0, flen = 0, fp = 0, fwl = 0, cur = 0, pc = 0, fgs = 0, fl = 0, isr = 0, one = 0;
                    // (the walker's "capb" flags, per lane and slot, written once after the walk)
                    int32_t fnode = 0, fnb = 0, ft2 = 0;
                    bool act = false;
                    // a start: (walk state, or over at once -- the '\u2581' node missing / the word ends)
                    auto fstart = [&](unsigned uu) -> bool {
                        unsigned gs = 0;
#pragma unroll
                        for (int g = 1; g < NG; g++) gs += uu >= fpre[g] ? 1u : 0u;
                        unsigned base = 0;
#pragma unroll
                        for (int g = 0; g < NG; g++) base = (gs == (unsigned)g) ? fpre[g] : base;
                        fgs = gs;
                        fl = gs * GSTR;
                        const GL &L = *reinterpret_cast<const GL *>(smem + fl);
                        const unsigned jj = L.fin[uu - base].v;
                        fj = jj;
                        fwl = SSr(gs).n_atoms;   // (= the LDS bytes: one per atom)
                        const unsigned b0 = L.bytes[jj];
                        isr = 0; one = 0; pc = 0;
                        if (((fwmask >> gs) & 1u) && jj == 0) {   // '\u2581' + b0: one atom
                            fnode = wsn; fnb = wsb; cur = b0; fp = 1; flen = 0;
                            return wsn >= 0;
                        }
                        if (b0 == '\n') {
                            fnode = 0; fnb = rb; cur = '<'; pc = 5; fp = jj + 1; flen = 0;
                            return true;
                        }
                        if (b0 != ' ') {   // a "more" start: the root table over (b0, next byte)
                            const unsigned n1 = L.bytes[jj + 1];
                            isr = 1; one = 1;
                            if (n1 == '\n') {   // inside atom jj+1's "<0x0A>" after its '<'
                                ft2 = (int32_t)(nsl + (b0 << 8) + (unsigned)'<');
                                flen = 1; cur = '0'; pc = 4; fp = jj + 2;
                            } else {             // two atoms; A0 saw a third that is no word start
                                ft2 = (int32_t)(nsl + (b0 << 8) + n1);
                                const unsigned n2 = L.bytes[jj + 2];
                                flen = 2; fp = jj + 3;
                                if (n2 == '\n') { cur = '<'; pc = 5; }
                                else cur = n2;
                            }
                            return true;
                        }
                        // a word start: the atom '\u2581' is the node ws_node
                        if (wsn < 0) return false;
                        fnode = wsn; fnb = wsb; flen = 1; one = wst;
                        if (wst) end_token_at(fl, jj + 1, 1);
                        if (jj + 1 >= fwl) return false;
                        const unsigned n1 = L.bytes[jj + 1];
                        if (n1 == ' ') return false;
                        fp = jj + 2;
                        if (n1 == '\n') { cur = '<'; pc = 5; }
                        else cur = n1;
                        return true;
                    };
                    unsigned nxt = DPT_STOP == 21 ? ftotal : 0u;   // diagnostic: A0 only
                    for (;;) {
                        {
                            const uint64_t im = ballot(!act);
                            const unsigned nidle = (unsigned)__builtin_popcountll(im);
                            if (nxt < ftotal && (nidle >= A_REFILL || ftotal - nxt <= nidle)) {
                                if (!act) {
                                    const unsigned uu = nxt + __builtin_amdgcn_mbcnt_hi((unsigned)(im >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)im, 0u));
                                    if (uu < ftotal) {
                                        act = fstart(uu);
                                        capm |= (unsigned)(!act && !one) << fgs;   // the start atom is no token
                                    }
                                }
                                nxt += nidle;
                            }
                        }
                        // (a start can be over at once, so a refill may leave every lane idle with starts left:
                        // the step then runs with no lane active and changes nothing -- one back edge, so
                        // the walk state stays in its registers across it)
                        if (!ballot(act) && nxt >= ftotal) break;
                        // the next raw byte, read before the trie load returns (masked off past the window)
                        // (kept ahead of the load by a scheduling barrier: else its address register may
                        // reuse the load's dead .z and wait for it)
                        const unsigned nbv = grp_bytes_at(fl, fp);
                        __builtin_amdgcn_sched_barrier(0);
                        const int32_t t = isr ? ft2 : fnb + (int32_t)cur;
                        const int4 ent = trie_slotA(tv, t);
                        const unsigned y = (unsigned)ent.y;
                        const unsigned av = act ? 1u : 0u;
                        // (both lookups' tests as 0/1 integers: a ?: over them became an exec-mask diamond)
                        const unsigned okr = ((y >> 30) & 1u) & (unsigned)((y & 0x3FFFFFFFu) != 0);
                        const unsigned okp = (unsigned)(ent.y == fnode);
                        const unsigned ok = av & ((isr & okr) | ((isr ^ 1u) & okp));
                        fnode = isr ? (int32_t)(y & 0x3FFFFFFFu) : t;
                        fnb = ent.x & BASE_MASK;
                        const unsigned leaf = ((unsigned)ent.x >> 30) & 1u;
                        // plain step: cur consumed; the atom ends unless its expansion has bytes left
                        const unsigned aend = ok & (isr ^ 1u) & (unsigned)(pc == 0);
                        const unsigned inexp = (isr ^ 1u) & (unsigned)(pc != 0);
                        cur = inexp ? nl_byte(pc) : cur;
                        pc = inexp ? pc - 1u : pc;
                        isr = 0;
                        flen += aend;
                        const unsigned term = aend & ((unsigned)ent.x >> 31);
                        one |= term & (unsigned)(flen == 1);
                        if (term) end_token_at(fl, fj + flen, flen);
                        // the next atom (after an atom end): a byte of the word, "<0x0A>", or the end
                        const unsigned past = (unsigned)(fp >= fwl) | (unsigned)(flen == 16u) | (unsigned)(nbv == ' ');
                        const unsigned stop = aend & past;
                        const unsigned nxa = aend & (past ^ 1u);
                        const unsigned isnl = (unsigned)(nbv == '\n');
                        cur = nxa ? (isnl ? (unsigned)'<' : nbv) : cur;
                        pc = (nxa & isnl) ? 5u : pc;
                        fp += nxa;
                        const unsigned nochild = (((unsigned)ent.w >> child_bit(cur)) & 1u) ^ 1u;
                        const unsigned done = av & ((ok ^ 1u) | leaf | stop | nochild);
                        capm |= (done & (one ^ 1u)) << fgs;
                        act = act && !done;
                    }
                }
            }
            // Byte-stream walker (the 64-lane 256-byte kernel, non-raw modes -- BLOOM-scale byte-level
            // vocabularies): no expansions, so a walk from atom j consumes the window's bytes from
            // aoff[j] on, and one u16 of bf[] per step says which byte comes next and whether an atom
            // ends (or the word) before it.  The first two bytes go through the root table; each later
            // step is one 8-byte trie load plus that one LDS read under it (the generic walker below reads
            // the next atom's descriptor and bytes -- four LDS reads and the expansion logic -- per step).
            // Whole-word shortcut (not when edges are an output): a word that is ONE vocabulary token has
            // cost 1 and that token as its only shortest tokenization (every other split costs >= 2:
            // dp_tokenize.py:24-47 then selects it); the walk from its first atom reaching the word's end
            // on a token marks it (scf[]) and B pushes only that edge (forward_lanes64).  (Walking the word
            // starts first, to skip the other atoms of such words, left the 64 lanes idle behind the
            // longest walks: BLOOM 4.90 -> 5.45 ms, r05f; and so did one pass over a word-starts-first list that
            // skips the starts inside words already known to be one token: +2 %, r05k.)
            if constexpr (GL::BSTREAM && !BIG) {
                if (!raw && nstart[0] > 0) {
                    const unsigned na_ = nstart[0];
                    nstart[0] = 0;   // (the generic walker gets nothing)
                    GL &L = grp(0);
                    const bool wsc = PLAIN || a.edges == nullptr;
                    const int32_t rb = tv.root_base;
                    const unsigned nsl = tv.n_slots;
                    for (unsigned jj = lane; jj < na_; jj += 64u) L.scf[jj] = 0;
                    {
                        const unsigned tot = na_;
                        unsigned bj = 0, bp = 0, blen = 0, bcur = 0;
                        int32_t bnode = 0, bnb = 0;
                        bool bisr = false, bact = false, bws = false;
                        uint64_t bmask = 0;
                        // a start: p = aoff[j]; two bytes of the word: the root table, else one root step
                        auto bstart = [&](unsigned jj) {
                            bj = jj;
                            const unsigned p = L.aoff[jj];
                            const unsigned f1 = L.bf[p + 1u];   // p + 1 <= wlen
                            const unsigned f0 = L.bf[p];
                            const unsigned b0 = f0 & 0xFFu;
                            bws = wsc && (f0 & BF_STOP) != 0;   // a word's first atom
                            bisr = (f1 & BF_STOP) == 0;         // the word has a second byte
                            bcur = bisr ? (nsl + (b0 << 8) + (f1 & 0xFFu)) : (unsigned)rb + b0;
                            bp = p;
                            bnode = 0; bnb = rb; blen = 0; bmask = 0;
                        };
                        unsigned nxt2 = DPT_STOP == 21 ? tot : 0u;
                        for (;;) {
                            {
                                const uint64_t im = ballot(!bact);
                                const unsigned nidle = (unsigned)__builtin_popcountll(im);
                                if (nxt2 < tot && (nidle >= A_REFILL64 || tot - nxt2 <= nidle)) {
                                    if (!bact) {
                                        const unsigned uu = nxt2 + __builtin_amdgcn_mbcnt_hi((unsigned)(im >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)im, 0u));
                                        if (uu < tot) { bact = true; bstart(uu); }
                                    }
                                    nxt2 += nidle;
                                }
                            }
                            if (!ballot(bact)) break;
                            const int2 e2 = trie_slot(tv, (int32_t)bcur);
                            // under the load: the flags (and byte) after this step's last byte
                            const unsigned q = bp + (bisr ? 2u : 1u);   // <= wlen
                            const unsigned fq = L.bf[q];
                            const unsigned fq1 = bisr ? (unsigned)L.bf[bp + 1u] : 0u;
                            const unsigned av = bact ? 1u : 0u;
                            const unsigned y = (unsigned)e2.y;
                            unsigned ok;
                            if (bisr) {
                                // root table: .y = node after two bytes | first byte exists << 30 | it ends a token << 31
                                const unsigned tok1 = av & (unsigned)((fq1 & BF_ATOM) != 0) & (y >> 30) & (y >> 31);
                                bmask |= (uint64_t)tok1;
                                blen = (fq1 & BF_ATOM) ? 1u : 0u;
                                ok = av & (y >> 30) & (unsigned)((y & 0x3FFFFFFFu) != 0);
                                bnode = (int32_t)(y & 0x3FFFFFFFu);
                            } else {
                                ok = av & (unsigned)(e2.y == bnode);
                                bnode = (int32_t)bcur;
                            }
                            bnb = e2.x & BASE_MASK;
                            const unsigned leaf = ((unsigned)e2.x >> 30) & 1u;
                            const unsigned aend = ok & (unsigned)((fq & BF_ATOM) != 0);
                            blen += aend;
                            const unsigned term = aend & ((unsigned)e2.x >> 31);
                            bmask |= term ? 1ull << (blen - 1u) : 0ull;
                            const unsigned stop = aend & (unsigned)((fq & BF_STOP) != 0);
                            const unsigned done = av & ((ok ^ 1u) | leaf | stop | (unsigned)(blen == (unsigned)G));
                            bcur = (unsigned)bnb + (fq & 0xFFu);
                            bp = q;
                            bisr = false;
                            if (done) {
                                L.rec[bj].smask = bmask;
                                if (bws && (stop & term)) L.scf[bj] = 1;   // the word is one token
                            }
                            capm |= done & (((unsigned)bmask & 1u) ^ 1u);
                            bact = bact && !done;
                        }
                    }
                }
            }
            unsigned pre[NG + 1];
            pre[0] = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) pre[g + 1] = pre[g] + nstart[g];
            const unsigned total = pre[NG];
            auto start = [&](unsigned uu) {
                unsigned gs = 0;
#pragma unroll
                for (int g = 1; g < NG; g++) gs += uu >= pre[g] ? 1u : 0u;
                unsigned base = 0;
#pragma unroll
                for (int g = 0; g < NG; g++) base = (gs == (unsigned)g) ? pre[g] : base;
                unsigned jj = uu - base;
                if constexpr (G == 16 && !BIG)
                    if ((a0mask >> gs) & 1u) jj = grp(gs).fin[jj].v;   // A0 slot: its marked list
                start_gj(gs, jj);
            };
            // Refills are batched: idle lanes take new starts only once A_REFILL of them are idle
            // (or the remaining starts fit), so the refill code runs on a fraction of the steps.
            bool active = false;
            unsigned nxt = DPT_STOP == 21 ? total : 0u;   // diagnostic: A0 only
            for (;;) {
                {
                    const uint64_t im = ballot(!active);
                    const unsigned nidle = (unsigned)__builtin_popcountll(im);
                    if (nxt < total && (nidle >= (G == 64 ? A_REFILL64 : A_REFILL) || total - nxt <= nidle)) {
                        if (!active) {
                            const unsigned uu = nxt + __builtin_amdgcn_mbcnt_hi((unsigned)(im >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)im, 0u));
                            if (uu < total) { active = true; start(uu); }
                        }
                        nxt += nidle;
                    }
                }
                if (!ballot(active)) break;
                const int32_t t = t2 ? (int32_t)t2 : nb + (int32_t)(seq & 0xFFu);
                // (the 64-lane kernels' walks read the 8-byte slots -- no child filter: half the footprint
                // of a BLOOM-scale trie, one more failing lookup per walk)
                int4 ent;
                if constexpr (G == 64) {
                    const int2 e2 = trie_slot(tv, t);
                    ent = make_int4(e2.x, e2.y, 0, -1);
                } else {
                    ent = trie_slotA(tv, t);   // buffer load: inactive lanes read harmlessly
                }
                // The step as selects (few exec-mask branches: their scalar bookkeeping costs issue
                // slots like the vector work does).  Root-table entry (t2): .y = node after two
                // bytes (0: none) | first byte exists << 30 | first byte ends a token << 31; .x =
                // that node's base word.  Plain step: the slot is the child iff its check is node.
                // (flags as 0/1 integers: && / || chains become exec-mask branches here)
                const unsigned act = active ? 1u : 0u;
                const unsigned isr = (unsigned)(t2 != 0);
                const unsigned y30 = ((unsigned)ent.y >> 30) & 1u, y31 = (unsigned)ent.y >> 31;
                const unsigned rsplit = act & isr & (split ? 1u : 0u);   // atom j ended after the first byte
                const unsigned rtok1 = rsplit & y30 & y31;
                const unsigned ok = act & (isr ? (y30 & (unsigned)((ent.y & 0x3FFFFFFF) != 0)) : (unsigned)(ent.y == node));
                len = rsplit ? 1u : len;
                mask = rtok1 ? (M)1 : mask;
                if constexpr (G == 16)
                    if (rtok1) end_token(j + 1, 1);
                seq = isr ? seq : seq >> 8;
                cnt = isr ? cnt : cnt - 1u;
                t2 = 0;
                node = isr ? (ent.y & 0x3FFFFFFF) : t;   // read only while ok
                nb = ent.x & BASE_MASK;
                const unsigned leaf = ((unsigned)ent.x >> 30) & 1u;
                const unsigned aend = ok & (unsigned)(cnt == 0);   // atom j+len-1 ends: span j..j+len is a candidate
                len += aend;
                const unsigned term = aend & ((unsigned)ent.x >> 31);
                if constexpr (G == 16) {
                    mask = (term & (unsigned)(len == 1)) ? (M)1 : mask;
                    if (term) end_token(j + len, len);
                } else {
                    mask |= term ? (M)1 << (len - 1) : (M)0;
                }
                const unsigned cont = aend & ((leaf | (unsigned)((info & AInfo<CH>::STOP) != 0) | (unsigned)(len == (unsigned)G)) ^ 1u);
                {
                    // the next atom, read by every lane (j + len <= n_atoms: in the window's arrays)
                    // (reading it a step ahead, before the trie load returns, measured slower: r03z)
                    const GL &L = *reinterpret_cast<const GL *>(smem + lbase);
                    unsigned cn = 0;
                    const unsigned inf = ainfo_get(L, j + len, false);
                    const uint64_t sq = atom_from_info<CH, WIDE>(L.bytes, inf, raw, cn);
                    info = cont ? inf : info;
                    seq = cont ? sq : seq;
                    cnt = cont ? cn : cnt;
                }
                // the walk ends at a failed lookup, at a leaf or a walk-ending atom, or when the
                // node has no child for the next byte (over without that lookup)
                const unsigned nochild = (((unsigned)ent.w >> child_bit((unsigned)(seq & 0xFFu))) & 1u) ^ 1u;
                const unsigned done = act & ((ok ^ 1u) | (aend ? ((cont ^ 1u) | nochild) : (leaf | nochild)));
                if constexpr (G != 16) {
                    if (done) {
                        GL &L = *reinterpret_cast<GL *>(smem + lbase);
                        L.rec[j].smask = mask;   // G = 16: end masks, set by end_token
                    }
                }
                capm |= (done & (((unsigned)mask & 1u) ^ 1u)) << gsel;
                active = active && !done;
            }
            // the slots whose walk found an atom that is no token by itself
#pragma unroll
            for (int g = 0; g < NG; g++)
                if (ballot((capm >> g) & 1u) && lane == 0) SSr(g).capb = 1;
        }
        wave_sync();
        STAMP(1);

        // ---------------------------------------------------------- B: forward recurrence
        KREFRESH();
        bool lane_mode = false;   // B ran per chunk and did C0 and C1 itself (G = 16, capless, no edges)
        if (DPT_RUN_B) {
            GL &L = grp(mg);
            const unsigned na = SSr(mg).n_atoms;
            unsigned imax = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) imax = max(imax, uni(SSr(g).n_atoms));
            // Steps past a slot's own n_atoms (up to the wave's imax <= CH) compute garbage that
            // lands in fin[] entries nobody reads, so the loop body has no per-slot guard.
            // Recording the edges (f1) and the uncapped DP (f2) are hoisted out as loop versions.
            // CAPM 0: the reference's capped DP (cost[i] <= i, dp_tokenize.py:28); 1: uncapped with
            // "inf" (inspect_tokenizer.py:77-86); 2: neither -- exact for both when every atom of
            // the wave's windows is a token by itself (then cost[i] <= i - ws on a valid path, so
            // the cap never wins and nothing is unreachable)
            auto forward = [&](auto EDGES, auto CAPM) {
                constexpr bool edges = decltype(EDGES)::value;
                constexpr int capm = decltype(CAPM)::value;
                // st (lane d, candidate j = i-1-d) = (cost[j]+1) << 16 | invalid[j] << 15 | G[j]
                constexpr unsigned ST0 = 0x10000u;   // word start: cost 0, reachable, G 0
                unsigned ws = 0;
                unsigned st = d == 0 ? ST0 : 0u;
                unsigned cpj = 0;
                if constexpr (G == 16) {
                    // Lane d carries x = rec[j] (its cpos) and its state in key form:
                    // (cost[j]+1) << 16 | invalid[j] << 15 | (0x7FFF - G[j]), so the candidate key is
                    // min(st, (st | 0x7FFF) - span); a dead span is one sign-extended bit of the
                    // inverted end mask of i (read by every lane of the row).
                    constexpr unsigned SK0 = 0x17FFFu;   // word start in key form
                    const uint32_t *rec32 = reinterpret_cast<const uint32_t *>(L.rec);
                    const unsigned sbit = 16u + d;
                    unsigned sk = d == 0 ? SK0 : 0u;
                    unsigned x = d == 0 ? rec32[0] : 0xFFFF0000u;
                    unsigned wsh = 0;                    // word start << 16
                    uint32_t nx = rec32[1];
                    // one step; (sk, x) in, (sk', x') out -- called alternately on two register sets
                    // so the DPP shifts need no copies
                    auto step = [&](unsigned i, unsigned skI, unsigned xI, unsigned &skO, unsigned &xO) {
                        const uint32_t cur = nx;
                        nx = rec32[i + 1];                         // i+1 <= CH+1 < NA: always in bounds
                        const unsigned span = (cur - xI) & 0x7FFFu;  // cp(j..i); borrows only move up
                        unsigned kv = (skI | 0x7FFFu) - span;
                        kv = skI < kv ? skI : kv;
                        const unsigned key = kv | (unsigned)__builtin_amdgcn_sbfe((int)cur, sbit, 1);
                        unsigned r = row_min_u32(key);
                        if constexpr (capm == 0) {
                            const unsigned capkey = ((i << 16) | 0xFFFFu) - wsh;
                            r = r < capkey ? r : capkey;
                        }
                        const uint64_t gmb = ballot(key == r);
                        const uint64_t emb = ballot((key ^ r) < 0x8000u);
                        if (d == 0) {
                            const unsigned sh = 16u * mg;
                            const unsigned gs = (unsigned)(gmb >> sh), es = (unsigned)(emb >> sh);
                            // lowest set bit of the row; bits of other rows only land in fields
                            // of positions C1 never reads (see Group<16>)
                            const unsigned dg = ffbl(gs), de = ffbl(es);
                            L.fin[i].v = (uint8_t)(dg | (de << 4));
                            L.rec[i].smask = Wfin<G>::pack(r);   // rec[i] was consumed at step i-1
                            if constexpr (edges)
                                if (i <= na) a.edges[SSr(mg).sb + SSr(mg).abase + i - 1] = es & 0xFFFFu;
                        }
                        const bool wend = (int16_t)cur < 0;     // CP_WS: word starts and the window end
                        wsh = wend ? (i << 16) : wsh;
                        unsigned nxt = r + 0x10000u;
                        if constexpr (capm == 1) nxt = r >= 0xFFFE0000u ? 0xFFFF8000u : nxt;   // unreachable: cost stays inf
                        skO = row_shift_in(skI, wend ? SK0 : nxt);
                        xO = row_shift_in(xI, cur);
                    };
                    unsigned sk2, x2;
                    unsigned i = 1;
                    for (; i + 1 <= imax; i += 2) {
                        step(i, sk, x, sk2, x2);
                        step(i + 1, sk2, x2, sk, x);
                    }
                    if (i <= imax) step(i, sk, x, sk2, x2);
                } else {
                    const uint64_t m0 = na > 0 ? L.rec[0].smask : 0ull;
                    unsigned mlo = d == 0 ? (unsigned)m0 : 0u, mhi = d == 0 ? (unsigned)(m0 >> 32) : 0u;
                    for (unsigned i = 1; i <= imax; i++) {
                        const unsigned cur = L.rec[i].cpos;
                        const uint64_t mi = L.rec[i].smask;
                        const unsigned cpi = cur & 0x7FFFu;
                        const unsigned span = cpi - cpj;
                        const unsigned gj = st & 0x7FFFu;
                        const unsigned kv = (st | 0x7FFFu) - (gj > span ? gj : span);
                        const unsigned bit = (d < 32 ? (mlo >> d) : (mhi >> (d - 32))) & 1u;
                        const unsigned key = bit ? kv : 0xFFFFFFFFu;
                        unsigned r = wave_min_u32(key);
                        if constexpr (capm == 0) {
                            const unsigned capkey = ((i - ws) << 16) | 0xFFFFu;
                            r = r < capkey ? r : capkey;
                        }
                        const uint64_t gmb = ballot(key == r);
                        const uint64_t emb = ballot((key ^ r) < 0x8000u);
                        if (lane == 0) {
                            const unsigned dg = gmb ? (unsigned)__builtin_ctzll(gmb) : 64u;
                            const unsigned de = emb ? (unsigned)__builtin_ctzll(emb) : 64u;
                            L.fin[i].d = dg | (de << 8);
                            L.fin[i].w = Wfin<G>::pack(r);
                            if constexpr (edges)
                                if (i <= na) a.edges[SSr(0).sb + SSr(0).abase + i - 1] = emb;
                        }
                        const bool wend = (cur & CP_WS) != 0;
                        ws = wend ? i : ws;
                        unsigned nxt = (r ^ 0x7FFFu) + 0x10000u;
                        if constexpr (capm == 1) nxt = r >= 0xFFFE0000u ? 0xFFFF8000u : nxt;
                        const unsigned sin = wend ? ST0 : nxt;
                        st = wave_shift_in(st, sin);
                        cpj = wave_shift_in(cpj, cpi);
                        mlo = wave_shift_in(mlo, (unsigned)mi);
                        mhi = wave_shift_in(mhi, (unsigned)(mi >> 32));
                    }
                }
            };
            // Capless windows without edge recording (the common case, G = 16): lanes take
            // chunks of end positions cut at "cut points" -- boundaries no token span crosses,
            // through which every tokenization of the word passes -- and run the recurrence
            // sequentially over their own chunk, one position per iteration for 64 lanes.
            // A chunk that starts inside a word starts from a local state (cost 0, G 0); a row
            // scan of the chunks' transfers gives each chunk its incoming state, and a fix-up
            // corrects the two things that depend on it: the final key of the word that ends
            // first in the chunk (cost offset, max with the incoming G) and dg at the positions
            // before that word end (dg = de wherever the incoming G already attains G[i]:
            // every j in E(i) then ties on max(G[j], cp(span))).  de and E(i) are local.
            auto forward_lanes = [&]() {
              if constexpr (G == 16) {
                // LW lanes share a window: a 16-lane row per slot, or (the one-string kernel, SOLO) the whole
                // wave on slot 0 -- chunks of <= 5 boundaries instead of 17, so the dependent LDS steps of the
                // recurrence and of the C1 walks are a quarter as many (the per-call floor)
                constexpr int LW = SOLO ? 64 : 16;
                constexpr unsigned CMAX = ((unsigned)(CH + LW - 1) / (unsigned)LW) | 1u;   // boundaries per lane, at most
                const unsigned mg = SOLO ? 0u : lane / 16u;
                const unsigned d = SOLO ? lane : lane % 16u;
                GL &L = grp(mg);
                const unsigned na = SSr(mg).n_atoms;
                uint32_t *rec32 = reinterpret_cast<uint32_t *>(L.rec);
                constexpr unsigned FRESH = 31u;   // key16 of a fresh start: cost 0, reachable, G 0
                // key16 = cost << 6 | invalid << 5 | 31 - G (the Wfin<16> form)
                auto relax = [](unsigned sj, unsigned span) {   // cost + 1, G = max(G, cp(span)); span <= 16
                    const unsigned a1 = sj + 64u;
                    const unsigned a2 = (a1 | 31u) - span;
                    return a1 < a2 ? a1 : a2;
                };
                // ---- cut points: boundary p is one iff min_{i > p} lo_i >= p, lo_i = the first atom
                //      of the longest token ending at i (i-1 - highest bit of its end mask)
                // boundaries per lane (na <= 256), odd: lanes stepping through their chunks together
                // then hit distinct LDS banks (ds_read_b32: 32 banks per 32-lane group; a stride of
                // 16 dwords put 8 lanes on a bank)
                const unsigned C = ((na + (unsigned)LW - 1u) / (unsigned)LW) | 1u;   // <= CMAX
                const unsigned c0 = min(d * C, na), c1 = min(c0 + C, na);
                // one backward pass over the chunk's ends (c0, c1]: the local suffix min of lo
                // decides the cuts as far as this chunk's ends go; the later chunks' ends (min S)
                // then only cap them: p is a cut iff both mins are >= p, i.e. p <= S
                // (the 512-byte pass's chunks have up to 33 boundaries: a 64-bit cut mask there)
                using CutM = std::conditional_t<(CMAX > 32u), uint64_t, uint32_t>;
                unsigned mloc = 0xFFFFu;
                CutM lcut = 0;
#pragma unroll 4
                for (int k = (int)CMAX - 1; k >= 0; k--) {
                    const unsigned i = c0 + 1u + (unsigned)k;
                    if (i <= c1) {
                        const unsigned hb = 31u - (unsigned)__builtin_clz((~rec32[i] >> 16) | 1u);   // bit 0 is set in a capless window
                        mloc = min(mloc, i - 1u - hb);
                        if (mloc >= i - 1u) lcut |= (CutM)1 << k;   // boundary p = i-1 = c0+k < c1
                    }
                }
                // min lo over the later lanes of the group (shift left: lane l reads lane l+k)
                unsigned sm = mloc;
                sm = min(sm, gshl<LW, 1>(sm, 0xFFFFu));
                sm = min(sm, gshl<LW, 2>(sm, 0xFFFFu));
                sm = min(sm, gshl<LW, 4>(sm, 0xFFFFu));
                sm = min(sm, gshl<LW, 8>(sm, 0xFFFFu));
                if constexpr (LW == 64) {
                    sm = min(sm, gshl<LW, 16>(sm, 0xFFFFu));
                    sm = min(sm, gshl<LW, 32>(sm, 0xFFFFu));
                }
                const unsigned S = gshl<LW, 1>(sm, 0xFFFFu);
                // boundaries c0 + k <= S
                const CutM cut = S < c0 ? (CutM)0 : (S - c0 >= CMAX - 1u ? lcut : lcut & (((CutM)2 << (S - c0)) - 1u));
                // rs = the first cut at or after c0 (in this lane's chunk or a later one; na is a cut)
                unsigned rs = na;
                if constexpr (CMAX > 32u) rs = cut ? c0 + (unsigned)__builtin_ctzll(cut) : na;
                else rs = cut ? c0 + ffbl(cut) : na;
                rs = min(rs, gshl<LW, 1>(rs, na));
                rs = min(rs, gshl<LW, 2>(rs, na));
                rs = min(rs, gshl<LW, 4>(rs, na));
                rs = min(rs, gshl<LW, 8>(rs, na));
                if constexpr (LW == 64) {
                    rs = min(rs, gshl<LW, 16>(rs, na));
                    rs = min(rs, gshl<LW, 32>(rs, na));
                }
                if constexpr (NEAR_CUT) {
                    // the NEAREST cut to c0 instead of the first one after it: snapping up made the longest
                    // chunk of a wave ~2x the mean on cfg4's long words (a 256-atom window: 36.7 ends
                    // against C = 17), and the wave steps as long as its longest chunk; nearest-cut
                    // rounding is monotone in c0, so the chunks still tile (0, na]
                    unsigned lastc = 0;   // (0 is a cut)
                    if constexpr (CMAX > 32u) lastc = cut ? c0 + (63u - (unsigned)__builtin_clzll(cut)) : 0u;
                    else lastc = cut ? c0 + (31u - (unsigned)__builtin_clz((unsigned)cut)) : 0u;
                    unsigned pm = lastc;   // max over the lanes <= d of the group, then shifted: lanes < d
                    pm = max(pm, gshr<LW, 1>(pm, 0u));
                    pm = max(pm, gshr<LW, 2>(pm, 0u));
                    pm = max(pm, gshr<LW, 4>(pm, 0u));
                    pm = max(pm, gshr<LW, 8>(pm, 0u));
                    if constexpr (LW == 64) {
                        pm = max(pm, gshr<LW, 16>(pm, 0u));
                        pm = max(pm, gshr<LW, 32>(pm, 0u));
                    }
                    const unsigned prevc = gshr<LW, 1>(pm, 0u);
                    rs = (c0 - prevc < rs - c0) ? prevc : rs;
                }
                const unsigned re = gshl<LW, 1>(rs, na);
                if (DPT_STOP == 25) return;   // diagnostic: cut points only

                // ---- the recurrence over ends (rs, re], one position per iteration
                unsigned i = rs, ws = rs, sprev = FRESH, pe = 0;
                unsigned cprev = rec32[rs] & 0x7FFu;
                unsigned nxt = rec32[rs + 1u];   // rs + 1 <= na + 1 < NA
                unsigned T = 0;                  // tokens of the chunk: the pieces' costs
                // (reading the next position's first candidates a step ahead, or two candidates per inner
                // iteration, measured slower: r03y, r03)
                while (ballot(i < re)) {
                    if (i < re) {
                        i++;
                        const unsigned r = nxt;
                        nxt = rec32[i + 1u];
                        const unsigned cpi = r & 0x7FFu;             // bits 11..14: see below
                        unsigned best = relax(sprev, cpi - cprev);   // j = i-1: the single atom
                        unsigned dg = 0, de = 0;
                        unsigned m = (~r >> 17) & 0x7FFFu;          // longer tokens ending at i: bit d-1
                        while (m) {
                            const unsigned dd = ffbl(m) + 1u;
                            m &= m - 1u;
                            const unsigned j = i - 1u - dd;          // j >= ws: spans cross no cut
                            const unsigned rj = rec32[j];
                            const unsigned sj = j == ws ? FRESH : (rj >> 16);
                            const unsigned kk = relax(sj, cpi - (rj & 0x7FFu));
                            // ascending d = descending j: the first strict improvement is the largest j
                            if ((kk >> 5) < (best >> 5)) de = dd;
                            if (kk < best) dg = dd;
                            best = kk < best ? kk : best;
                        }
                        L.rec[i].smask = (uint16_t)best;   // this end's mask was read above
                        L.fin[i].v = (uint8_t)(dg | (de << 4));
                        const bool wend = (r & CP_WS) != 0;
                        if (wend) {
                            // the word ending at i: its G (the longest token to select, L*) - 1 goes
                            // into bits 11..14 of rec[i].cpos (code-point prefixes are < 2048 in a
                            // 256-byte window), where C1 finds it (the mask halves take its tokens)
                            L.rec[i].cpos = (uint16_t)((r & 0x87FFu) | ((30u - (best & 31u)) << 11));
                            T += best >> 6;
                            if (!pe) pe = i;
                        }
                        ws = wend ? i : ws;
                        sprev = wend ? FRESH : best;
                        cprev = cpi;
                    }
                }
                if (DPT_STOP == 26) return;   // diagnostic: + the recurrence
                // P1 = the piece walked first in C1 (the one ending at re); p1in: no word start in
                // (rs, re), so P1 is the chunk's first piece too and starts from the incoming state
                const bool re_ws = i > rs && sprev == FRESH;   // re is a word start (its word ended)
                const bool p1in = pe == 0 || pe == re;
                if (!re_ws) T += sprev >> 6;
                unsigned gl1 = 31u - ((re_ws ? L.rec[re].smask : sprev) & 31u);   // local G of P1 at re
                // ---- row scan of the chunk transfers: (reset, value) -- a chunk with a word start
                //      ignores its input; otherwise out = in (+) local, (+) = costs add, G max
                unsigned x = (pe ? 0x10000u : 0u) | sprev;
                auto compose = [&](unsigned y) {   // y (the earlier lanes) then x
                    const unsigned comb = (y & 0xFFC0u) + (x & 0xFFC0u) + min(y & 31u, x & 31u);
                    x = (x >> 16) ? x : ((y & 0x10000u) | comb);
                };
                compose(gshr<LW, 1>(x, FRESH));
                compose(gshr<LW, 2>(x, FRESH));
                compose(gshr<LW, 4>(x, FRESH));
                compose(gshr<LW, 8>(x, FRESH));
                if constexpr (LW == 64) {
                    compose(gshr<LW, 16>(x, FRESH));
                    compose(gshr<LW, 32>(x, FRESH));
                }
                const unsigned in = gshr<LW, 1>(x, FRESH) & 0xFFFFu;
                const unsigned gin = 31u - (in & 31u);   // G at rs
                if (gin) {
                    const unsigned lim = pe ? pe : re;
                    for (unsigned q = rs + 1u; q <= lim; q++) {
                        const unsigned kl = L.rec[q].smask;
                        if (gin >= 31u - (kl & 31u)) {
                            const unsigned f = L.fin[q].v;
                            L.fin[q].v = (uint8_t)((f & 0xF0u) | (f >> 4));
                        }
                    }
                    if (pe) {
                        const unsigned kl = L.rec[pe].smask;
                        L.rec[pe].smask = (uint16_t)((in & 0xFFC0u) + (kl & 0xFFC0u) + min(in & 31u, kl & 31u));
                        if (gin > 31u - (kl & 31u)) L.rec[pe].cpos = (uint16_t)((L.rec[pe].cpos & 0x87FFu) | ((gin - 1u) << 11));
                    }
                }
                const unsigned gre = p1in ? max(gin, gl1) : gl1;   // G at re of P1's word (its L* if re_ws)
                if (DPT_STOP == 27) return;   // diagnostic: + the transfer scan and fix-up

                // ---- C1 (replaces C0 + C1 for the wave): the selection walks, one chunk per lane.
                // Every tokenization passes through the cuts, so a chunk's tokens are the ones its
                // own walk from re down to rs emits; their count T is fixed (the pieces' costs).
                // The walk rule is C1's (dg while the longest token so far A is below the word's
                // L*, de after).  What a chunk needs from the right: P1's L* (a copy scan from
                // the chunk holding its word end) and whether A has reached L* on entry.  Left of
                // q (the first cut where G reaches L*: gre < L*) it has -- the L* token lies in the
                // segment ending at q; right of q, dg == de everywhere (every j in E(i) is at or
                // after q, so G[j] == L*), so it does not matter; in q's chunk it has iff a chunk
                // to the right selected an L* token by chance -- the flag scan after the walks,
                // and that chunk re-walks P1 in de mode.
                // token base: exclusive prefix sum of T over the row; the window's count to wtok
                unsigned tb = T;
                tb += gshr<LW, 1>(tb, 0u);
                tb += gshr<LW, 2>(tb, 0u);
                tb += gshr<LW, 4>(tb, 0u);
                tb += gshr<LW, 8>(tb, 0u);
                if constexpr (LW == 64) {
                    tb += gshr<LW, 16>(tb, 0u);
                    tb += gshr<LW, 32>(tb, 0u);
                }
                if (d == (unsigned)LW - 1u) SSr(mg).wtok = tb;
                tb -= T;
                // P1's L*: from rec[re] when its word ends at re, else from the right (the first
                // word end of the next chunk that has one)
                unsigned lsr = pe ? (0x10000u | (((unsigned)L.rec[pe].cpos >> 11) & 15u)) : 0u;
                auto copy_r = [&](unsigned y) { lsr = (lsr >> 16) ? lsr : y; };
                copy_r(gshl<LW, 1>(lsr, 0u));
                copy_r(gshl<LW, 2>(lsr, 0u));
                copy_r(gshl<LW, 4>(lsr, 0u));
                copy_r(gshl<LW, 8>(lsr, 0u));
                if constexpr (LW == 64) {
                    copy_r(gshl<LW, 16>(lsr, 0u));
                    copy_r(gshl<LW, 32>(lsr, 0u));
                }
                // (DPP reads outside any branch: a lane masked off in EXEC reads as 0)
                const unsigned lsn = gshl<LW, 1>(lsr, 0u);
                const unsigned ls1 = re_ws ? gre : (lsn & 15u) + 1u;
                const bool walk = !len_only && SSr(mg).status == 0;   // per row (not uniform)
                const bool left_of_q = gre < ls1;
                unsigned n1 = 0;   // tokens of P1
                unsigned afin = 0, lsm = ls1;   // after the walk: A and L* of the last piece
                {
                    unsigned ii = re, k = walk ? tb + T : tb, A = left_of_q ? ls1 : 0u, Ls = ls1;
                    unsigned pend = rec32[re] & 0x7FFu;
                    bool inp1 = true;
                    while (ballot(k > tb)) {
                        if (k > tb) {
                            const unsigned rr = rec32[ii];
                            const unsigned cpi = rr & 0x7FFu;
                            if (ii < re && (rr & CP_WS)) {   // into the word ending at ii
                                Ls = ((rr >> 11) & 15u) + 1u;
                                A = 0;
                                pend = cpi;
                                inp1 = false;
                            }
                            n1 += inp1 ? 1u : 0u;
                            const unsigned f = L.fin[ii].v;
                            const unsigned sp = pend - cpi;
                            A = A > sp ? A : sp;
                            const unsigned dd = A < Ls ? (f & 15u) : (f >> 4);
                            const unsigned j = ii - 1u - dd;
                            k--;
                            L.rec[k].smask = (uint16_t)j;   // k < rs or a position this walk has left
                            pend = cpi;
                            ii = j;
                        }
                    }
                    const unsigned sp = pend - (rec32[rs] & 0x7FFu);
                    afin = A > sp ? A : sp;
                    lsm = Ls;
                }
                // flag scan, right to left: the chunk's last piece reached its L* (sel); a chunk
                // whose last piece is P1 also passes on what came in; none crosses a word start
                unsigned fl = ((T > 0 && afin >= lsm) ? 1u : 0u) | ((!p1in || re_ws) ? 2u : 0u);
                auto flag_r = [&](unsigned y) { fl = (fl & 2u) ? fl : (fl | (y & 3u)); };
                flag_r(gshl<LW, 1>(fl, 0u));
                flag_r(gshl<LW, 2>(fl, 0u));
                flag_r(gshl<LW, 4>(fl, 0u));
                flag_r(gshl<LW, 8>(fl, 0u));
                if constexpr (LW == 64) {
                    flag_r(gshl<LW, 16>(fl, 0u));
                    flag_r(gshl<LW, 32>(fl, 0u));
                }
                const unsigned fln = gshl<LW, 1>(fl, 0u);
                const bool fin_in = !re_ws && (fln & 1u) != 0;
                // q's chunk with a chance L* token to the right: P1 again in de mode (A = L*);
                // P1 starts below L* only from rs with gin < L* or from a word start inside
                if (walk && fin_in && !left_of_q && (!p1in || gin < ls1)) {
                    unsigned ii = re, k = tb + T;
                    for (unsigned c = 0; c < n1; c++) {
                        const unsigned j = ii - 1u - (unsigned)(L.fin[ii].v >> 4);
                        k--;
                        L.rec[k].smask = (uint16_t)j;
                        ii = j;
                    }
                }
              }
            };
            // Capless windows of the 256-byte 64-lane kernel without edge recording (one string per
            // wave: BLOOM-scale byte-level vocabularies).  The row recurrence is one wave-min per atom,
            // a dependent chain over the whole window (55 % of that kernel, profiles/r03_phase_diag.txt).
            // Here each lane takes a chunk of end positions cut at cut points, as forward_lanes does,
            // and relaxes forward ("push") from every start j of its chunk over j's span mask (phase
            // A's start masks, rec[j].smask): the token j..i updates i's entry {dg | de << 8 | cp(i)
            // << 16, key} in fin[].  Starts are taken in ascending order, so "<=" keeps the largest j
            // of a tie -- the row recurrence's lowest lane (dp_tokenize.py:40-46).  A wave scan of the
            // chunk transfers and forward_lanes' fix-up follow; C0/C1 then run as in row mode (they
            // read fin[] only).
            auto forward_lanes64 = [&]() {
              if constexpr (G == 64 && !BIG) {
                if (na == 0) return;
                constexpr unsigned FRESH = 0x7FFFu;       // key of a fresh start: cost 0, reachable, G 0
                constexpr unsigned RESET = 0x80000000u;   // transfer flag: a word ends in the chunk
                uint2 *fin2 = reinterpret_cast<uint2 *>(L.fin);
                // ---- cut points (bit p of cm[p / 64]): p is one iff max_{j < p} (j + 1 + hb(smask_j))
                //      <= p -- no token crosses it; 0 and na always are
                uint64_t cm[(CH + 64) / 64];
                unsigned carry = 0;
#pragma unroll
                for (int r = 0; r < (CH + 64) / 64; r++) {
                    const unsigned p = 64u * (unsigned)r + lane;
                    // the end of the longest token from p: p + 1 + (63 - clz)
                    const unsigned v = p < na ? p + 64u - (unsigned)__builtin_clzll(L.rec[p].smask | 1ull) : 0u;
                    const unsigned inc = wave_incl_scan_max(v);
                    const unsigned ex = max(carry, wave_shift_in(inc, 0u));
                    carry = max(carry, __builtin_amdgcn_readlane(inc, 63));
                    cm[r] = ballot(p <= na && ex <= p);
                }
                // the first cut at or after c (<= na)
                auto nextcut = [&](unsigned c) -> unsigned {
                    unsigned res = na;
#pragma unroll
                    for (int r = (CH + 64) / 64 - 1; r >= 0; r--) {
                        const unsigned lo = 64u * (unsigned)r;
                        const uint64_t keep = c <= lo ? ~0ull : (c >= lo + 64u ? 0ull : (~0ull << (c - lo)));
                        const uint64_t m = cm[r] & keep;
                        res = m ? lo + (unsigned)__builtin_ctzll(m) : res;
                    }
                    return res;
                };
                // the last cut at or before c (0 is a cut)
                auto prevcut = [&](unsigned c) -> unsigned {
                    unsigned res = 0;
#pragma unroll
                    for (int r = 0; r < (CH + 64) / 64; r++) {
                        const unsigned lo = 64u * (unsigned)r;
                        const uint64_t keep = c < lo ? 0ull : (c >= lo + 63u ? ~0ull : (~0ull >> (63u - (c - lo))));
                        const uint64_t m = cm[r] & keep;
                        res = m ? lo + 63u - (unsigned)__builtin_clzll(m) : res;
                    }
                    return res;
                };
                // chunk bounds snapped to the NEAREST cut (as forward_lanes, DPT_NEAR_CUT): monotone in c, so
                // lane l's end is lane l+1's start
                auto snap = [&](unsigned c) -> unsigned {
                    const unsigned nx = nextcut(c);
                    if constexpr (!NEAR_CUT64) return nx;
                    const unsigned pv = prevcut(c);
                    return (c - pv < nx - c) ? pv : nx;
                };
                const unsigned C = (na + 63u) >> 6;   // (odd chunk lengths: -0.5 %, r03ad)
                const unsigned c0 = min(lane * C, na), c1 = min(c0 + C, na);
                const unsigned rs = snap(c0);
                // (c1 = the next lane's c0: its start, by wave_shl:1; lane 63 ends at na)
                const unsigned re = (unsigned)__builtin_amdgcn_update_dpp((int)na, (int)rs, 0x130, 0xF, 0xF, false);
                (void)c1;
                if (DPT_STOP == 25) return;   // diagnostic: cut points only
                // ---- the chunk's entries: no candidate yet, cp(i) in the high half; pe = its first word end
                unsigned pe = 0;
                for (unsigned i = rs + 1u; i <= re; i++) {
                    const unsigned cp = L.rec[i].cpos;
                    fin2[i] = make_uint2((cp & 0x7FFFu) << 16, 0xFFFFFFFFu);
                    pe = (!pe && (cp & CP_WS)) ? i : pe;
                }
                // ---- push: j ascending; j's key is final once every earlier start of the chunk ran --
                //      it is the j-1 -> j edge's result (bit 0: capless windows have it at every start),
                //      carried in a register.  One edge at a time: batches of 2 / 4 edges with their reads
                //      in flight (r03x) and giving long chunks to the whole wave as a row recurrence (r03ae)
                //      measured slower -- the push is throughput-bound across the resident waves.
                unsigned kcarry = FRESH;
                for (unsigned j = rs; j < re; j++) {
                    const uint64_t sm = L.rec[j].smask;
                    const unsigned cj = L.rec[j].cpos;
                    const unsigned kj = (j == rs || (cj & CP_WS)) ? FRESH : kcarry;
                    const unsigned a1 = kj + 0x10000u;             // cost + 1
                    const unsigned a1g = (a1 | 0x7FFFu) + (cj & 0x7FFFu);
                    auto upd = [&](uint2 &f, unsigned dd) {
                        const unsigned a2 = a1g - (f.x >> 16);       // G = max(G[j], cp(j..i))
                        const unsigned kk = a1 < a2 ? a1 : a2;
                        f.x = ((kk >> 15) <= (f.y >> 15)) ? ((f.x & ~0x7F00u) | (dd << 8)) : f.x;   // de
                        f.x = (kk <= f.y) ? ((f.x & ~0x7Fu) | dd) : f.x;                            // dg
                        f.y = kk < f.y ? kk : f.y;
                    };
                    if (!raw && L.scf[j]) {
                        // a word that is one token (phase A's whole-word shortcut): only that edge, whose key
                        // (cost 1) is final at the word end; its inner positions are never read (C0/C1 read
                        // word ends, C1 walks from them; no cut lies inside the word).  Sound only because
                        // (1) every window ends at a word start or the string's end (window_bounds), so the
                        // BF_STOP the byte-stream walker stopped on is the word's real end, not a window cut
                        // through it, and (2) that walker never steps past a BF_STOP; a change to either
                        // must revisit this (tests/test_gpu_parity.py::test_bloom_words_across_windows)
                        const unsigned dd = 63u - (unsigned)__builtin_clzll(sm);   // the longest token from j
                        uint2 f = fin2[j + 1u + dd];
                        upd(f, dd);
                        fin2[j + 1u + dd] = f;
                        kcarry = f.y;
                        j += dd;
                        continue;
                    }
                    {   // the j -> j+1 edge (bit 0): j+1's final key
                        uint2 f = fin2[j + 1u];
                        upd(f, 0u);
                        fin2[j + 1u] = f;
                        kcarry = f.y;
                    }
                    // the span mask as two 32-bit halves: one v_ffbl and 32-bit arithmetic per edge
                    // (BLOOM 21.5 -> 22.1 GB/s against the 64-bit walk, r04l)
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        uint32_t m32 = hh == 0 ? ((uint32_t)sm & ~1u) : (uint32_t)(sm >> 32);
                        while (m32) {
                            const unsigned dd = ffbl(m32) + 32u * (unsigned)hh;
                            m32 &= m32 - 1u;
                            uint2 f = fin2[j + 1u + dd];   // <= re: no token crosses a cut
                            upd(f, dd);
                            fin2[j + 1u + dd] = f;
                        }
                    }
                }
                if (DPT_STOP == 26) return;   // diagnostic: + the recurrence
                // ---- wave scan of the chunk transfers (forward_lanes' compose, 64 lanes, keys)
                const bool re_wb = (L.rec[re].cpos & CP_WS) != 0;
                unsigned x = rs == re ? FRESH : ((pe ? RESET : 0u) | (re_wb ? FRESH : fin2[re].y));
                auto compose = [&](unsigned y) {   // y (the earlier lanes) then x
                    const unsigned comb = ((y & 0x7FFF0000u) + (x & 0x7FFF0000u)) | min(y & 0x7FFFu, x & 0x7FFFu);
                    x = (x & RESET) ? x : ((y & RESET) | comb);
                };
                compose((unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x111, 0xF, 0xF, false));   // row_shr:1
                compose((unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x112, 0xF, 0xF, false));   // row_shr:2
                compose((unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x114, 0xF, 0xF, false));   // row_shr:4
                compose((unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x118, 0xF, 0xF, false));   // row_shr:8
                compose((unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x142, 0xA, 0xF, false));   // row_bcast:15
                compose((unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x143, 0xC, 0xF, false));   // row_bcast:31
                const unsigned in = (unsigned)__builtin_amdgcn_update_dpp((int)FRESH, (int)x, 0x138, 0xF, 0xF, false) & ~RESET;   // wave_shr:1
                const unsigned gin = 0x7FFFu - (in & 0x7FFFu);   // G at rs (0: a word starts there, cost 0)
                if (gin) {
                    // before the first word end: dg = de wherever the incoming G attains G[q];
                    // the first word end's key = in (+) local
                    const unsigned lim = pe ? pe : re;
                    for (unsigned q = rs + 1u; q <= lim; q++) {
                        const uint2 f = fin2[q];
                        if (gin >= 0x7FFFu - (f.y & 0x7FFFu)) fin2[q].x = (f.x & ~0x7Fu) | ((f.x >> 8) & 0x7Fu);
                    }
                    if (pe) {
                        const unsigned kl = fin2[pe].y;
                        fin2[pe].y = ((in & 0x7FFF0000u) + (kl & 0x7FFF0000u)) | min(in & 0x7FFFu, kl & 0x7FFFu);
                    }
                }
              }
            };
            using T_ = std::true_type;
            using F_ = std::false_type;
            using C0_ = std::integral_constant<int, 0>;
            using C1_ = std::integral_constant<int, 1>;
            using C2_ = std::integral_constant<int, 2>;
            unsigned capb = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) capb |= uni(SSr(g).capb);
            if (!PLAIN && a.edges) {
                if (!capb) forward(T_{}, C2_{}); else if (uncapped) forward(T_{}, C1_{}); else forward(T_{}, C0_{});
            } else {
                if (!capb) {
                    if constexpr (G == 16) {
                        forward_lanes();
                        lane_mode = true;
                    } else if constexpr (!BIG) {
                        forward_lanes64();
                        lane_mode = DPT_STOP >= 25 && DPT_STOP <= 27;   // stop builds: no C0/C1 over unfinished fin[]
                    } else {
                        forward(F_{}, C2_{});
                    }
                } else if (uncapped) forward(F_{}, C1_{}); else forward(F_{}, C0_{});
            }
        }
        wave_sync();
        STAMP(2);

        // ---------------------------------------------------------- C0: per-window token counts and validity
        KREFRESH();
        // (word w ends at atom word_end(w); its final state is in fin[word_end(w)])
        if (DPT_RUN_B && !lane_mode) {
            if constexpr (GL::WSLG) {
                // the word list (word -> first atom, then the window end) from the word-start bits
#pragma unroll
                for (int g = 0; g < NG; g++) {
                    const unsigned na = uni(SSr(g).n_atoms);
                    if (na == 0) continue;
                    const GL &L = grp(g);
                    uint8_t *gw = wsl_of(g);
                    unsigned wi = 0;
                    for (unsigned j0 = 0; j0 <= na; j0 += 64u) {
                        const unsigned j = j0 + lane;
                        const bool ws = j <= na && (L.rec[j].cpos & CP_WS) != 0;   // atom na: the window end
                        const uint64_t m = ballot(ws);
                        if (ws) gw[wi + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] = (uint8_t)j;
                        wi += (unsigned)__builtin_popcountll(m);
                    }
                }
            }
            unsigned pre[NG + 1];
            pre[0] = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) pre[g + 1] = pre[g] + (uni(SSr(g).n_atoms) > 0 ? uni(SSr(g).n_words) : 0u);
            const unsigned total = pre[NG];
            for (unsigned u0 = 0; u0 < total; u0 += 64) {
                const unsigned u = u0 + lane;
                unsigned g = 0;
#pragma unroll
                for (int k = 1; k < NG; k++) g += u >= pre[k] ? 1u : 0u;
                unsigned wbase = 0;
#pragma unroll
                for (int k = 0; k < NG; k++) wbase = g == (unsigned)k ? pre[k] : wbase;
                unsigned cost = 0, inv = 0, lng = 0;
                if (u < total) {
                    const GL &L = grp(g);
                    const unsigned we = L.word_end(wsl_of(g), u - wbase);
                    const typename Wfin<G>::T F = L.wkey(we);
                    cost = Wfin<G>::cost(F);
                    inv = Wfin<G>::invalid(F) ? 1u : 0u;
                    // a vocabulary token longer than G code points could span more than G atoms,
                    // beyond the walks: such a word is outside the engine's limits (status 3)
                    if (a.long_span) lng = we - L.word_start(wsl_of(g), u - wbase) > (unsigned)G ? 1u : 0u;
                }
                // per-group sums over this chunk: groups own contiguous lane ranges
#pragma unroll
                for (int k = 0; k < NG; k++) {
                    const unsigned lo = pre[k] > u0 ? pre[k] - u0 : 0u, hi = pre[k + 1] > u0 ? pre[k + 1] - u0 : 0u;
                    if (hi <= lo) continue;
                    const bool mine = lane >= lo && lane < (hi < 64u ? hi : 64u);
                    const unsigned cs = wave_incl_scan_add(mine ? cost : 0u);
                    const unsigned csum = __builtin_amdgcn_readlane(cs, 63);
                    const unsigned anyinv = (ballot(mine && inv) != 0 ? 1u : 0u) | (ballot(mine && lng) != 0 ? 2u : 0u);
                    if (lane == 0) { SSr(k).wtok += csum; SSr(k).inval |= anyinv; }
                }
            }
        }
        wave_sync();

        // ---------------------------------------------------------- C1: selection, one lane per word
        KREFRESH();
        if (DPT_RUN_B && !lane_mode) {
            unsigned pre[NG + 1], tokpre[NG + 1], inv_g[NG];
            pre[0] = 0; tokpre[0] = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) {
                const unsigned nwg = uni(SSr(g).n_atoms) > 0 ? uni(SSr(g).n_words) : 0u;
                inv_g[g] = uni(SSr(g).inval) | (uni(SSr(g).status) != 0 ? 1u : 0u);
                pre[g + 1] = pre[g] + nwg;
                tokpre[g + 1] = tokpre[g] + (nwg ? uni(SSr(g).wtok) : 0u);
            }
            const unsigned total = pre[NG];
            unsigned carry = 0;
            for (unsigned u0 = 0; u0 < total; u0 += 64) {
                const unsigned u = u0 + lane;
                const bool in = u < total;
                unsigned g = 0;
#pragma unroll
                for (int k = 1; k < NG; k++) g += u >= pre[k] ? 1u : 0u;
                unsigned wbase = 0, tbase = 0, ginv = 0;
#pragma unroll
                for (int k = 0; k < NG; k++)
                    if (g == (unsigned)k) { wbase = pre[k]; tbase = tokpre[k]; ginv = inv_g[k]; }
                GL &L = grp(g);
                const unsigned w = u - wbase;
                const typename Wfin<G>::T F = in ? L.wkey(L.word_end(wsl_of(g), w)) : (typename Wfin<G>::T)0;
                const unsigned cost = in ? Wfin<G>::cost(F) : 0u;
                const unsigned incl = wave_incl_scan_add(cost);
                const unsigned tok_base = carry + incl - cost - tbase;
                carry += __builtin_amdgcn_readlane(incl, 63);
                if (in && !ginv && !len_only) {
                    // a valid word's walk emits exactly `cost` tokens and ends at its first atom
                    // (Appendix A), so the token count bounds the loop
                    unsigned i = L.word_end(wsl_of(g), w);
                    const unsigned Ls = Wfin<G>::gmax(F);   // G of the word = the longest token to reach
                    unsigned c = cost, A = 0;
                    unsigned pend = L.rec[i].cpos & 0x7FFFu;
                    while (c > 0) {
                        const typename GR::Fin f = L.fin[i];
                        const unsigned cpi = L.rec[i].cpos & 0x7FFFu;
                        const unsigned sp = pend - cpi;
                        A = A > sp ? A : sp;                 // the token emitted last step ended at pend
                        const unsigned dd = A < Ls ? GR::dg(f) : GR::de(f);
                        const unsigned j = i - 1 - dd;
                        c--;
                        L.rec[tok_base + c].smask = (M)j;   // span masks are dead after B
                        pend = cpi;
                        i = j;
                    }
                }
            }
        }
        wave_sync();
        STAMP(3);
        // ---------------------------------------------------------- C2: ids (lanes over all slots' tokens)
        KREFRESH();
        if (DPT_RUN_C2) {
            unsigned pre[NG + 1], na_g[NG];
            uint64_t obase[NG];       // staging element of the window's first token, per slot
            const bool n16 = SW == 1 || (SW == 0 && a.staging16 != nullptr);   // int16 staging (uniform)
            // per slot, bit 0: the window starts the string (raw '▁' + first atom); bit 1: a '\u2581'-compressed
            // PRESPLIT window (its ' ' bytes expand to '\u2581' as raw mode's do)
            unsigned firstmask = 0;
            pre[0] = 0;
#pragma unroll
            for (int g = 0; g < NG; g++) {
                const bool gv = !len_only && uni(SSr(g).inval) == 0 && uni(SSr(g).status) == 0 && uni(SSr(g).n_atoms) > 0;
                pre[g + 1] = pre[g] + (gv ? uni(SSr(g).wtok) : 0u);
                na_g[g] = uni(SSr(g).n_atoms);
                firstmask |= ((raw && uni64(SSr(g).pos) == 0 ? 1u : 0u) | (uni(SSr(g).cpw) ? 2u : 0u)) << (2 * g);
                const uint64_t e0 = uni64(SSr(g).sb) + uni(SSr(g).ntok);
                obase[g] = e0;
            }
            const unsigned total = pre[NG];
            // per-slot token range, atom count, first-window flag and staging row, in the slot's
            // fin[] (dead after C1): a token start reads its slot's record with one LDS load
            // instead of selecting among NG sets of registers
            struct C2Slot {
                uint32_t base, ntk, na, fw;
                uint64_t ob;   // staging element (an offset, not a pointer: stores through a.staging* stay
                               // global_store -- a pointer read back from LDS becomes a flat store, whose
                               // lgkmcnt makes the next LDS wait on the store's completion)
            };
            static_assert(sizeof(typename GR::Fin) * GL::NA >= sizeof(C2Slot), "C2Slot fits fin[]");
            if (lane == 0) {
#pragma unroll
                for (int g = 0; g < NG; g++) {
                    C2Slot &q = *reinterpret_cast<C2Slot *>(&grp(g).fin[0]);
                    q.base = pre[g]; q.ntk = pre[g + 1] - pre[g]; q.na = na_g[g]; q.fw = (firstmask >> (2 * g)) & 3u; q.ob = obase[g];
                }
            }
            wave_sync();
            // 16-lane first pass: a bulk pass resolves every token of one or two expanded bytes with
            // ONE lookup (a one-byte token's root child, a two-byte token's root-table entry: .z = the
            // id of the node reached) and lists the rest -- word starts ('\u2581'), newlines, tokens of
            // three or more bytes -- by their token number in the rec[].cpos halves (dead in C2:
            // entry i in group i / 256's rec[i % 256]).  A short list (< 64 tokens of <= 8 bytes: the
            // walker would run with idle lanes) joins the wave's pending row, which is walked from
            // the stored bytes once a round would overflow it (walk_pending); a longer one is walked
            // below by the refill walker.
            constexpr bool BULK = G == 16 && !BIG;
            constexpr unsigned PEND_CAP = 64;   // residual tokens a wave's pending row holds (its scratch row)
            unsigned wbeg = 0, wend = total;
            // the list of tokens left for the walkers: in the rec[].cpos halves (dead in C2) -- G = 16:
            // entry i in group i / 256's rec[i % 256]; G = 64 (one slot): rec[i]
            auto list_ref = [&](unsigned i) -> uint16_t & {
                if constexpr (G == 16)
                    return *reinterpret_cast<uint16_t *>(smem + (i >> 8) * GSTR + (i & 255u) * 4u);
                else
                    return grp(0).rec[i].cpos;
            };
            // hash pass over n tokens (token number of entry i: src(i)): a token of at most
            // TOKHASH_MAX_BYTES expanded bytes without a newline atom gets its id from ONE bucket load
            // of the token hash table (dpt_internal.h); the others are listed, in order, at the front of
            // the list for the walkers.  Returns their number (n without a table).
            auto hash_pass = [&](unsigned n, auto src) -> unsigned {
                const uint8_t *hbase = reinterpret_cast<const uint8_t *>(tv.pair16) + TOKHASH_OFFSET;
                const TokHashHeader hh = *reinterpret_cast<const TokHashHeader *>(hbase);
                if (!hh.max_probe) {
                    for (unsigned i = lane; i < n; i += 64u) list_ref(i) = (uint16_t)src(i);
                    return n;
                }
                const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(hbase + sizeof(TokHashHeader)), (short)0, (int)((hh.mask + 1u) * 16u), 0x00020000);
                // token rounds of 64 per iteration, their loads before any store (a load waits for every
                // older store of the wave; 1 or 4 rounds measured slower, r03)
                constexpr int HP_U = DPT_HP_U;
                unsigned r2 = 0;
                for (unsigned i0 = 0; i0 < n; i0 += 64u * HP_U) {
                    unsigned tt[HP_U], hh2[HP_U], fpv[HP_U];
                    uint64_t oqv[HP_U];
                    bool hs[HP_U], inr[HP_U];
#pragma unroll
                    for (int u = 0; u < HP_U; u++) {
                        const unsigned i = i0 + 64u * (unsigned)u + lane;
                        const bool in = i < n;
                        const unsigned t = in ? src(i) : 0u;
                        unsigned g = 0;
#pragma unroll
                        for (int k = 1; k < NG; k++) g += t >= pre[k] ? 1u : 0u;
                        const GL &L = *reinterpret_cast<const GL *>(smem + g * GSTR);
                        const C2Slot q = *reinterpret_cast<const C2Slot *>(&L.fin[0]);
                        const unsigned k = in ? t - q.base : 0u;
                        const unsigned jj = (unsigned)L.rec[k].smask;
                        const unsigned nx = (unsigned)L.rec[k + 1].smask;   // k + 1 <= ntk < NA
                        const unsigned j1 = k + 1 < q.ntk ? nx : q.na;
                        const unsigned p0 = L.aoff[jj];
                        const unsigned nbytes = (typename GL::Idx)(L.aoff[j1] - p0);
                        const unsigned fa = q.fw & 1u & (unsigned)(jj == 0);   // (bit 0: raw mode only)
                        uint32_t h = 0, fp = 0;
                        bool hashed;
                        if constexpr (G == 16) {
                            uint32_t w[4];
                            unsigned E = 0;
                            hashed = in && token_key<CH>(L.bytes, p0, nbytes, raw || (q.fw >> 1) != 0u, fa, w, E);
                            if (hashed) tokhash(w[0], w[1], w[2], w[3], E, hh.seed, h, fp);
                        } else {   // 64-lane rows (BLOOM-scale vocabularies): keys of up to 64 bytes
                            hashed = in && token_hash_long<CH>(L.bytes, p0, nbytes, raw, fa, hh.seed, h, fp);
                        }
                        tt[u] = t; hh2[u] = h & hh.mask; fpv[u] = fp; oqv[u] = q.ob + k; hs[u] = hashed; inr[u] = in;
                    }
                    int32_t idv[HP_U];
                    if constexpr (HASH_BOTH) {
                        // every round's two buckets (the key's two choices) at once, then the stores
#pragma unroll
                        for (int u = 0; u < HP_U; u++) {
                            const auto e = __builtin_amdgcn_raw_buffer_load_b128(hr, hh2[u] * 16u, 0, 0);
                            const auto f = __builtin_amdgcn_raw_buffer_load_b128(hr, tokhash_alt(hh2[u], fpv[u], hh.mask) * 16u, 0, 0);
                            idv[u] = e[0] == fpv[u] ? (int32_t)e[1] : e[2] == fpv[u] ? (int32_t)e[3] :
                                     f[0] == fpv[u] ? (int32_t)f[1] : f[2] == fpv[u] ? (int32_t)f[3] : -1;
                        }
                    } else {
                        // every round's home bucket, then the partner buckets of the keys not found there
                        // (one more load round for the wave, never a chain), then the stores
#pragma unroll
                        for (int u = 0; u < HP_U; u++) {
                            const auto e = __builtin_amdgcn_raw_buffer_load_b128(hr, hh2[u] * 16u, 0, 0);
                            idv[u] = e[0] == fpv[u] ? (int32_t)e[1] : (e[2] == fpv[u] ? (int32_t)e[3] : INT32_MIN);
                        }
                        bool miss = false;
#pragma unroll
                        for (int u = 0; u < HP_U; u++) miss |= hs[u] && idv[u] == INT32_MIN;
                        if (ballot(miss)) {
#pragma unroll
                            for (int u = 0; u < HP_U; u++) {
                                if (hs[u] && idv[u] == INT32_MIN) {
                                    const auto f = __builtin_amdgcn_raw_buffer_load_b128(hr, tokhash_alt(hh2[u], fpv[u], hh.mask) * 16u, 0, 0);
                                    idv[u] = f[0] == fpv[u] ? (int32_t)f[1] : (f[2] == fpv[u] ? (int32_t)f[3] : -1);
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int u = 0; u < HP_U; u++) {
                        if (hs[u]) {
                            if (n16) a.staging16[oqv[u]] = (int16_t)idv[u];
                            else a.staging[oqv[u]] = idv[u];
                        }
                    }
                    // every lane read its entries above (list sources): the compacted rest lands below i0 + 64 * HP_U
#pragma unroll
                    for (int u = 0; u < HP_U; u++) {
                        const bool rest = inr[u] && !hs[u];
                        const uint64_t m = ballot(rest);
                        if (rest) list_ref(r2 + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))) = (uint16_t)tt[u];
                        r2 += (unsigned)__builtin_popcountll(m);
                    }
                }
                return r2;
            };
            if constexpr (BULK) {
                const bool i16 = n16;
                unsigned r = 0;
                // The bulk pass over every selected token, 4 per lane per round of 256.  int16 ids from the
                // pair table: all the window-set's lookups first, then all its stores -- a load waits for
                // every OLDER vector-memory op of the wave, stores included (MI355X_MICROARCH.md: vmcnt
                // counts loads and stores together, in issue order), so a store between two rounds of
                // lookups put a store's full latency on every round.  (Every round's lookups before any
                // store held the ids in registers and spilled: cfg2 -4.1 %, r03.)
                constexpr int BU = DPT_BULK_U;   // tokens per lane per round
                auto bulk_round = [&](unsigned t0, int32_t (&ix)[BU], unsigned (&kind)[BU], uint64_t (&oq)[BU]) {
#pragma unroll
                    for (int u = 0; u < BU; u++) {
                        const unsigned t = t0 + 64u * (unsigned)u + lane;
                        const bool in = t < total;
                        unsigned g = 0;
#pragma unroll
                        for (int k = 1; k < NG; k++) g += t >= pre[k] ? 1u : 0u;
                        const GL &L = *reinterpret_cast<const GL *>(smem + g * GSTR);
                        const C2Slot q = *reinterpret_cast<const C2Slot *>(&L.fin[0]);
                        const unsigned k = in ? t - q.base : 0u;
                        const unsigned jj = (unsigned)L.rec[k].smask;
                        const unsigned nx = (unsigned)L.rec[k + 1].smask;   // k + 1 <= ntk < NA
                        const unsigned j1 = k + 1 < q.ntk ? nx : q.na;
                        const unsigned p0 = L.aoff[jj];
                        const unsigned nbytes = (uint8_t)(L.aoff[j1] - p0);
                        const uint32_t *w = reinterpret_cast<const uint32_t *>(L.bytes) + (p0 >> 2);
                        const unsigned two = __builtin_amdgcn_alignbyte(w[1], w[0], p0 & 3u);
                        const unsigned b0 = two & 0xFFu, b1 = (two >> 8) & 0xFFu;
                        // raw mode (and '\u2581'-compressed PRESPLIT windows, q.fw bit 1) expands ' ' (a word start),
                        // '\n' and the string's first atom
                        const unsigned expd = ((raw ? 1u : 0u) | (q.fw >> 1)) &
                                              ((unsigned)(b0 == ' ') | (unsigned)(b0 == '\n') | (q.fw & 1u & (unsigned)(jj == 0)) |
                                               ((unsigned)(nbytes == 2u) & ((unsigned)(b1 == ' ') | (unsigned)(b1 == '\n'))));
                        const unsigned bulk = (unsigned)in & (unsigned)(nbytes - 1u <= 1u) & (expd ^ 1u);
                        if constexpr (SW == 1)   // int16 ids: the 128-KB pair table (L1-resident for ASCII)
                            ix[u] = bulk ? (int32_t)(nbytes == 1u ? 65536u + b0 : (b0 << 8) + b1) : 0;
                        else
                            ix[u] = bulk ? (nbytes == 1u ? tv.root_base + (int32_t)b0 : (int32_t)(tv.n_slots + (b0 << 8) + b1)) : 0;
                        kind[u] = bulk ? nbytes : 0u;
                        oq[u] = q.ob + k;
                        const bool res = in && !bulk;
                        const uint64_t m = ballot(res);
                        if (res) list_ref(r + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))) = (uint16_t)t;
                        r += (unsigned)__builtin_popcountll(m);
                    }
                };
                for (unsigned t0 = 0; t0 < total; t0 += 64u * (unsigned)BU) {
                    int32_t ix[BU];
                    unsigned kind[BU];   // 0: not here, 1 / 2: a token of that many bytes
                    uint64_t oq[BU];
                    bulk_round(t0, ix, kind, oq);
                    if constexpr (SW == 1) {
                        int16_t pv[BU];
#pragma unroll
                        for (int u = 0; u < BU; u++) pv[u] = tv.pair16[ix[u]];
#pragma unroll
                        for (int u = 0; u < BU; u++)
                            if (kind[u]) a.staging16[oq[u]] = pv[u];
                        continue;
                    }
                    int4 ent[BU];
#pragma unroll
                    for (int u = 0; u < BU; u++) ent[u] = trie_slotA(tv, ix[u]);
#pragma unroll
                    for (int u = 0; u < BU; u++) {
                        if (kind[u]) {
                            // the walker's rule: the id of the node reached when every step's check held
                            const bool ok = kind[u] == 1u ? ent[u].y == 0 : (ent[u].y & 0x3FFFFFFF) != 0;
                            const int32_t idv = ok ? ent[u].z : -1;
                            if (i16) a.staging16[oq[u]] = (int16_t)idv;
                            else a.staging[oq[u]] = idv;
                        }
                    }
                }
                wave_sync();
                STAMP(5);
                if (DPT_C2STOP == 1) r = 0;   // diagnostic: the bulk pass only
                if (r > 0) {
                    r = hash_pass(r, [&](unsigned i) -> unsigned { return list_ref(i); });
                    wave_sync();
                }
                STAMP(6);
                if (DPT_C2STOP == 2) r = 0;   // diagnostic: + the hash pass
                wend = r;
                if (r > 0 && r < (unsigned)PEND_CAP) {
                    uint4 ent = make_uint4(0u, 0u, 0u, 0u);
                    bool lng = false;
                    if (lane < r) {
                        const unsigned t = list_ref(lane);
                        unsigned g = 0;
#pragma unroll
                        for (int k = 1; k < NG; k++) g += t >= pre[k] ? 1u : 0u;
                        const GL &L = *reinterpret_cast<const GL *>(smem + g * GSTR);
                        const C2Slot q = *reinterpret_cast<const C2Slot *>(&L.fin[0]);
                        const unsigned k = t - q.base;
                        const unsigned jj = (unsigned)L.rec[k].smask;
                        const unsigned nx = (unsigned)L.rec[k + 1].smask;
                        const unsigned j1 = k + 1 < q.ntk ? nx : q.na;
                        const unsigned p0 = L.aoff[jj];
                        const unsigned len = (uint8_t)(L.aoff[j1] - p0);
                        const unsigned fi = q.fw & 1u & (unsigned)(jj == 0);
                        const unsigned rl = (raw ? 1u : 0u) | (q.fw >> 1);   // raw mode's expansions
                        lng = len > 8u;
                        const uint64_t by = load_bytes(L.bytes, p0, lng ? 8u : len);
                        const uint64_t out = q.ob + k;
                        ent = make_uint4((uint32_t)out, ((uint32_t)(out >> 32) & 0xFFFFu) | (len << 16) | (fi << 24) | (rl << 25),
                                         (uint32_t)by, (uint32_t)(by >> 32));
                    }
                    if (!ballot(lng)) {
                        if (n_pend + r > (unsigned)PEND_CAP) {
                            walk_pending(n_pend);
                            n_pend = 0;
                        }
                        if (lane < r) a.pend[(uint64_t)bid * 64u + n_pend + lane] = ent;
                        n_pend += r;
                        wend = 0;
                    }
                }
            }
            if constexpr (!BULK) {   // the walkers take what the hash pass leaves
                if (total > 0) {
                    wend = hash_pass(total, [](unsigned i) -> unsigned { return i; });
                    wave_sync();
                }
            }
            auto tok_at = [&](unsigned i) -> unsigned { return list_ref(i); };
            // One token walk per lane; a lane whose token is resolved writes the id and takes the
            // next token (ballot + mbcnt), so each iteration is one trie step for 64 tokens.  A
            // token's bytes do not depend on the trie, so each iteration issues the trie load
            // first and does the LDS work of the next byte / atom / token (known before the
            // load returns: the token ends when its last atom's bytes run out) under it.
            struct Tok {
                unsigned jj, j1, cnt, lbase;
                uint64_t seq;
                uint64_t out;
                bool rl;   // raw mode's expansions (raw mode, or a '\u2581'-compressed PRESPLIT window)
            };
            auto tstart = [&](unsigned t) -> Tok {
                Tok T;
                unsigned g = 0;
#pragma unroll
                for (int k = 1; k < NG; k++) g += t >= pre[k] ? 1u : 0u;
                T.lbase = g * GSTR;
                const GL &L = *reinterpret_cast<const GL *>(smem + T.lbase);
                const C2Slot q = *reinterpret_cast<const C2Slot *>(&L.fin[0]);
                const unsigned k = t - q.base;
                T.jj = (unsigned)L.rec[k].smask;
                const unsigned nx = (unsigned)L.rec[k + 1].smask;   // k + 1 <= ntk < NA
                T.j1 = k + 1 < q.ntk ? nx : q.na;
                T.rl = raw || (q.fw >> 1) != 0u;
                T.seq = atom_from_info<CH, WIDE>(L.bytes, AInfo<CH>::pack(L.aoff[T.jj], L.atom_len(T.jj), 0, q.fw & 1u & (unsigned)(T.jj == 0)), T.rl, T.cnt);
                T.out = q.ob + k;
                return T;
            };
            // NW token walks per lane (tokens lane, lane + 64, ... first), so that many trie loads are
            // in flight per lane in every iteration
            constexpr int NW = 1;
            bool active[NW];
            Tok C[NW];
            int32_t node[NW], nb[NW];
            bool ok[NW];
#pragma unroll
            for (int w = 0; w < NW; w++) {
                active[w] = wbeg + lane + 64u * w < wend;
                C[w].jj = C[w].j1 = C[w].cnt = C[w].lbase = 0; C[w].seq = 0; C[w].out = 0; C[w].rl = raw;
                if (active[w]) C[w] = tstart(tok_at(wbeg + lane + 64u * w));
                node[w] = 0; nb[w] = tv.root_base; ok[w] = true;
            }
            unsigned nxt = wbeg + 64u * NW;
            for (;;) {
                bool any = false;
#pragma unroll
                for (int w = 0; w < NW; w++) any |= active[w];
                if (!ballot(any)) break;
                int32_t sl[NW];
                int4 ent[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    sl[w] = nb[w] + (int32_t)(C[w].seq & 0xFFu);
                    ent[w] = trie_slot4(tv, sl[w]);   // buffer load: inactive walks read harmlessly
                }
                // ---- under the loads: the next byte or atom
                bool done[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    C[w].seq >>= 8;
                    C[w].cnt -= 1u;
                    const unsigned aend = (active[w] ? 1u : 0u) & (unsigned)(C[w].cnt == 0);
                    const unsigned dn = aend & (unsigned)(C[w].jj + 1 == C[w].j1);
                    done[w] = dn != 0;
                    if (aend & (dn ^ 1u)) {
                        C[w].jj++;
                        const GL &L = *reinterpret_cast<const GL *>(smem + C[w].lbase);
                        C[w].seq = atom_from_info<CH, WIDE>(L.bytes, AInfo<CH>::pack(L.aoff[C[w].jj], L.atom_len(C[w].jj), 0, 0), C[w].rl, C[w].cnt);
                    }
                }
                // ---- the trie steps; finished walks write their id and take the next token
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    ok[w] &= ent[w].y == node[w];
                    node[w] = sl[w];
                    nb[w] = ent[w].x & BASE_MASK;
                    const uint64_t dm = ballot(done[w]);
                    if (done[w]) {
                        const int32_t idv = ok[w] ? ent[w].z : -1;   // the id arrives with the token's last node
                        if (n16) a.staging16[C[w].out] = (int16_t)idv;
                        else a.staging[C[w].out] = idv;
                        const unsigned uu = nxt + __builtin_amdgcn_mbcnt_hi((unsigned)(dm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)dm, 0u));
                        active[w] = uu < wend;
                        if (active[w]) C[w] = tstart(tok_at(uu));
                        node[w] = 0; nb[w] = tv.root_base; ok[w] = true;
                    }
                    nxt += (unsigned)__builtin_popcountll(dm);
                }
            }
        }
        wave_sync();
        STAMP(7);

        // ---------------------------------------------------------- advance slots, finish strings
        KREFRESH();
        if (lane < (unsigned)NG) {
            SlotState &S = SSr(lane);
            if (S.active && S.n_atoms > 0 && S.status == 0 && (S.inval & 2)) {
                // a word of more than G atoms while the vocabulary has longer tokens: the
                // unbounded pass redoes the whole string (and writes its status and count)
                a.long_list[atomicAdd(a.long_count, 1u)] = S.s;
                S.active = 0;
            } else if (S.active && S.n_atoms > 0) {
                S.capsum += S.wtok;
                if (S.status == 0 && S.inval) S.status = 1;
                if (S.status == 0 && !len_only) S.ntok += S.wtok;
                S.pos += S.wlen;
                S.abase += S.n_atoms;
                if (S.pos >= S.slen) {
                    const uint64_t s = S.s;
                    const uint64_t cnt = S.status == 0 ? (uint64_t)S.ntok : 0ull;
                    a.status[s] = (int32_t)S.status;
                    if (a.capped) a.capped[s] = S.status == 3 ? -1 : (int32_t)S.capsum;
                    S.active = 0;
                    if (!(DPT_DIAG_PREP & 8))
                        if (a.bsum && cnt) atomicAdd(a.bsum + (s / FIN_BATCH) * BS_LINE, cnt);
                    a.counts[s] = cnt;
                }
            }
        }
        wave_sync();
        STAMP(4);
        STAMP(8);
        WST_REC(1 + min(wst_it, WST_N - 4), WST_NOW() | ((unsigned long long)busy << 56));
        wst_it++;
    }
    if constexpr (G == 16 && !BIG)
        if (n_pend) {
            walk_pending(n_pend);
            n_pend = 0;
        }
    if (!BIG && a.solo && lane == 0) {   // the call's only string, the grid's only wave
        a.id_off[0] = 0;
        reset_counters(a.retry_count, a.ctr_snap);
    }
    STAMP(9);
    STAMP_FLUSH;
    WST_REC(WST_N - 1, WST_NOW() | ((unsigned long long)wst_it << 48));
#ifdef DPT_WSTAMPS
    WST_REC(WST_N - 2, wst_claims);
#endif
#undef a
#undef tv
}

template <int CH, int G, bool BIG, bool WIDE, int SW = 0, bool RAW = false, bool SOLO = false, int MC = -1>
// (the one-string kernel, SOLO, is one wave: no occupancy to keep, so no VGPR cap and no spills)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SOLO ? 1 : ((CH == 256 && G == 16) ? WPE16 : ((CH == 256 && G == 64) ? WPE64 : 1)))))
tokenize_kernel(KernArgs ka) {
    tokenize_body<CH, G, BIG, WIDE, SW, RAW, SOLO, MC>(blockIdx.x);
}

// ------------------------------------------------------------------ compaction

// ------------------------------------------------------------------ finish: offsets + CSR ids in one pass

constexpr unsigned FIN_U = 8;                 // loads in flight per thread of the copy (8 / 12 beat 4, 16 and 32: r04n)
constexpr unsigned FIN_THREADS = 512;         // threads per finish block (>= FIN_BATCH): all of them copy
constexpr unsigned FIN_MAP_ROWS = 8192;       // s_map entries (u8 string index): rows of 64 ids, coarser past 512k ids
#ifndef DPT_FIN_PIPE    // A/B knob: the finish copy issues round r+1's loads before round r's stores
#define DPT_FIN_PIPE 1
#endif
constexpr bool FIN_PIPE = DPT_FIN_PIPE != 0;
constexpr unsigned SCAN_THREADS = 1024;       // threads of the batch-scan block
constexpr uint64_t FIN_TARGET_BLOCKS = 2048;  // small batches: each batch's copy is split over slices until the grid has this many blocks
constexpr uint64_t FIN_MAX_SLICES = 8;

// inclusive add-scan over a block of NT threads; *total = the block's sum.  Uses s_w[NT / 64] and
// ends with the block synchronised (s_w reusable after it).
template <unsigned NT>
__device__ __forceinline__ uint64_t block_incl_scan_add64(uint64_t v, uint64_t *s_w, uint64_t *total) {
    const unsigned tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    uint64_t incl = wave_incl_scan_add64(v, lane);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint64_t agg = 0;
#pragma unroll
    for (unsigned k = 0; k < NT / 64; k++) {
        const uint64_t ws = s_w[k];
        if (k < w) incl += ws;
        agg += ws;
    }
    *total = agg;
    __syncthreads();
    return incl;
}


// Batch prefixes: the tokenize passes add every string's count to its FIN_BATCH-string batch's sum
// as the string finishes (one no-return atomic per string, dpt_kernels.hip / dpt_long.hip); this ONE
// block turns the batch sums (one per BS_LINE) into exclusive prefixes bpre[0..nb) (thread i over a contiguous chunk:
// chunk sums, one block scan, the chunk again), zeroes bsum for the next call and resets the counter
// block -- every tokenize pass has finished when it runs.  It replaces round 2's decoupled look-back
// inside a persistent finish kernel, which chained the batches: a finish block could not start its
// copy before its look-back, so each block took its batches one after another.
__global__ void __launch_bounds__(SCAN_THREADS) batch_scan_kernel(uint64_t n_str, unsigned long long *bsum,
                                                                  unsigned long long *bpre, uint32_t *ctr,
                                                                  unsigned long long *hist_zero, uint32_t n_hist,
                                                                  uint64_t *ctr_snap) {
    // DPT_HIST_OVERWRITE: the histogram the finish pass adds to starts from zero (stream order)
    if (hist_zero)
        for (uint32_t b = threadIdx.x; b < n_hist; b += SCAN_THREADS) hist_zero[b] = 0;
    __shared__ uint64_t s_w[SCAN_THREADS / 64];
    const unsigned tid = threadIdx.x;
    const uint64_t nb = (n_str + FIN_BATCH - 1) / FIN_BATCH;
    const uint64_t per = (nb + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint64_t c0 = (uint64_t)tid * per < nb ? (uint64_t)tid * per : nb, c1 = c0 + per < nb ? c0 + per : nb;
    uint64_t sum = 0, total;
    constexpr unsigned PER_REG = 8;   // up to 8 x 1024 batches (2M strings): the sums stay in registers, read once
    if (per <= PER_REG) {   // (all loads issued before the first is used: one round trip, not per batches)
        uint64_t v[PER_REG];
#pragma unroll
        for (unsigned u = 0; u < PER_REG; u++) {
            v[u] = c0 + u < c1 ? bsum[(c0 + u) * BS_LINE] : 0ull;
            sum += v[u];
        }
        uint64_t run = block_incl_scan_add64<SCAN_THREADS>(sum, s_w, &total) - sum;
#pragma unroll
        for (unsigned u = 0; u < PER_REG; u++) {
            if (c0 + u < c1) {
                bpre[c0 + u] = run;
                bsum[(c0 + u) * BS_LINE] = 0;
            }
            run += v[u];
        }
    } else {
        for (uint64_t k = c0; k < c1; k++) sum += bsum[k * BS_LINE];
        uint64_t run = block_incl_scan_add64<SCAN_THREADS>(sum, s_w, &total) - sum;
        for (uint64_t k = c0; k < c1; k++) {
            const uint64_t b = bsum[k * BS_LINE];
            bpre[k] = run;
            bsum[k * BS_LINE] = 0;
            run += b;
        }
    }
    if (tid == 0) reset_counters(ctr, ctr_snap);
}

struct FinishArgs {
    const void *staging;          // int16_t or int32_t (ST)
    const uint64_t *str_off;
    const uint64_t *counts;
    uint64_t n_str;
    uint64_t *id_off;
    int32_t *ids;
    const unsigned long long *bpre;   // per batch: its first id (batch_scan_kernel)
    unsigned slices;                  // blocks per batch
    unsigned long long *bsum;         // one-batch calls (no scan kernel): zeroed here ...
    uint32_t *ctr;                    // ... and the counter block reset here (null when the scan kernel ran)
    const unsigned long long *fold;   // fin_fold calls: the batch sums (BS_LINE apart), summed here per block (else null) ...
    unsigned long long *fold_zero;    // ... while the other parity's batch lines are zeroed for the next call
    uint64_t fold_n;                  // (its batches)
    unsigned long long *hist;         // nullable: the token-count histogram (dpt_ctx_set_histogram) ...
    int hist_store;                   // ... stored, not added (DPT_HIST_OVERWRITE in a one-batch call) ...
    const int32_t *status;            // ... with the statuses it counts
    uint32_t n_bins;
    uint64_t *ctr_snap;               // nullable: the counter block's first 64 bytes before the reset (reset_counters)
};

// CSR offsets and ids: block b takes slice b % slices of batch b / slices.  One count per thread of
// the first FIN_BATCH, a block scan (the batch's relative offsets), the batch's first id from bpre;
// slice 0 writes every string's end offset; then ALL the block's threads copy the slice's staged ids --
// threads over the OUTPUT ids, so every store is a coalesced row -- FIN_U independent loads in flight
// per thread.  At 1M strings a batch is one block (3 907 blocks); small calls split each batch's copy
// so the grid still has ~FIN_TARGET_BLOCKS blocks (a block's copy is a chain of dependent load rounds:
// 125k strings were 489 blocks of 7 rounds each).
template <typename ST>
__global__ void __launch_bounds__(FIN_THREADS) finish_kernel(FinishArgs f) {
    __shared__ uint64_t s_rel[FIN_BATCH + 1];   // ids of the batch's strings before string k, + the batch total
    __shared__ uint64_t s_src[FIN_BATCH];       // staging element of each string's first id
    __shared__ uint64_t s_w[FIN_THREADS / 64];
    // the string holding id r << gs of the batch, per row r: a copy element finds its string from
    // its row's in one or two LDS reads, all of a thread's elements independently
    __shared__ uint8_t s_map[FIN_MAP_ROWS];
    const unsigned tid = threadIdx.x;
    const uint64_t t = blockIdx.x / f.slices;
    const unsigned sl = blockIdx.x % f.slices;
    const uint64_t base_off = f.str_off[0];
    const ST *__restrict__ staging = reinterpret_cast<const ST *>(f.staging);
    const uint64_t s0 = t * FIN_BATCH;
    // the first FIN_BATCH threads hold one string each; every thread copies
    const bool has = tid < FIN_BATCH && tid < f.n_str - s0;
    const uint64_t c = has ? f.counts[s0 + tid] : 0ull;
    const uint64_t src = has ? f.str_off[s0 + tid] - base_off : 0ull;
    uint64_t total;
    uint64_t o0 = 0;   // one batch: its first id is 0
    if (f.fold) {   // the batch's first id: the sums of the batches before it (t <= FIN_FOLD_MAX)
        uint64_t ps = 0;
        for (uint64_t k = tid; k < t; k += FIN_THREADS) ps += f.fold[k * BS_LINE];
        (void)block_incl_scan_add64<FIN_THREADS>(ps, s_w, &o0);
        for (uint64_t k = (uint64_t)blockIdx.x * FIN_THREADS + tid; k < f.fold_n; k += (uint64_t)gridDim.x * FIN_THREADS)
            f.fold_zero[k * BS_LINE] = 0;
    } else if (!f.bsum) {
        o0 = f.bpre[t];
    }
    const uint64_t incl = block_incl_scan_add64<FIN_THREADS>(c, s_w, &total);
    if (tid < FIN_BATCH) {
        s_rel[tid] = incl - c;
        s_src[tid] = src;
    }
    // rows of 64 ids -- finer when the batch's strings average fewer ids, so that an element's string is at
    // most a step or two past its row's (short strings: a 64-id row spans tens of them); coarser when the
    // batch has more than FIN_MAP_ROWS rows
    unsigned gs = 6;
    {
        const uint64_t nb_s = f.n_str - s0 < FIN_BATCH ? f.n_str - s0 : FIN_BATCH;
        const uint64_t avg = total / nb_s;
        while (gs > 0 && (1ull << gs) > avg) gs--;
    }
    while ((total >> gs) >= FIN_MAP_ROWS) gs++;
    if (has && c) {   // the rows starting inside this string's ids [incl - c, incl)
        const uint64_t rb = (incl - c + (1ull << gs) - 1u) >> gs, re = (incl - 1u) >> gs;
        for (uint64_t r = rb; r <= re; r++) s_map[r] = (uint8_t)tid;
    }
    if (tid == FIN_BATCH - 1) s_rel[FIN_BATCH] = incl;
    __syncthreads();
    if (f.hist && sl == 0) {
        // the batch's histogram (dpt_token_histogram's layout) in LDS, added to the global one once:
        // one LDS atomic per string for its count bin, the statuses and totals by ballots
        __shared__ unsigned long long lh[FIN_MAX_BINS + 8];
        const uint32_t nbh = f.n_bins + 8;
        for (uint32_t b = tid; b < nbh; b += FIN_THREADS) lh[b] = 0;
        __syncthreads();
        int32_t st = -1;
        if (has) {
            atomicAdd(&lh[c < f.n_bins - 1 ? (uint32_t)c : f.n_bins - 1], 1ull);
            st = f.status[s0 + tid];
            st = st >= 0 && st <= 4 ? st : 4;
        }
        const unsigned lanei = tid & 63u;
#pragma unroll
        for (int v = 0; v < 5; v++) {
            const uint64_t m = __ballot(st == v);
            if (lanei == 0 && m) atomicAdd(&lh[f.n_bins + 2 + v], (unsigned long long)__builtin_popcountll(m));
        }
        if (tid == 0) {
            lh[f.n_bins] += total;   // (the block scan's sum: the batch's ids)
            lh[f.n_bins + 1] += (unsigned long long)(f.n_str - s0 < FIN_BATCH ? f.n_str - s0 : FIN_BATCH);
        }
        __syncthreads();
        for (uint32_t b = tid; b < nbh; b += FIN_THREADS) {
            if (f.hist_store) f.hist[b] = lh[b];   // the call's only batch
            else if (lh[b]) atomicAdd(&f.hist[b], lh[b]);
        }
    }
    if (sl == 0) {
        if (has) f.id_off[s0 + tid + 1] = o0 + incl;
        if (t == 0 && tid == 0) {
            f.id_off[0] = 0;
            // without the scan kernel: its other duties (every tokenize pass is done)
            if (f.bsum) f.bsum[0] = 0;   // one-batch call (fold calls zero the other array instead)
            if (f.ctr) reset_counters(f.ctr, f.ctr_snap);
        }
    }
    const uint64_t k_beg = total * sl / f.slices, k_end = total * (sl + 1) / f.slices;
    constexpr unsigned U = FIN_U;
    // a round: U ids per thread, FIN_THREADS apart (every store a coalesced row); each id's string
    // from its row's (s_map), then past the string starts inside the row -- rounds of U independent
    // LDS reads, not one chain through the batch's offsets
    auto gather = [&](uint64_t k0, int32_t (&v)[U]) {
        unsigned jj[U];
#pragma unroll
        for (unsigned u = 0; u < U; u++) {
            const uint64_t k = k0 + (uint64_t)u * FIN_THREADS + tid;
            jj[u] = k < k_end ? s_map[k >> gs] : 0u;
        }
#pragma unroll
        for (unsigned u = 0; u < U; u++) {
            const uint64_t k = k0 + (uint64_t)u * FIN_THREADS + tid;
            jj[u] += (k < k_end && s_rel[jj[u] + 1] <= k) ? 1u : 0u;
        }
#pragma unroll
        for (unsigned u = 0; u < U; u++) {
            const uint64_t k = k0 + (uint64_t)u * FIN_THREADS + tid;
            while (k < k_end && s_rel[jj[u] + 1] <= k) jj[u]++;   // (strings shorter than a row)
        }
#pragma unroll
        for (unsigned u = 0; u < U; u++) {
            const uint64_t k = k0 + (uint64_t)u * FIN_THREADS + tid;
            v[u] = k < k_end ? (int32_t)staging[s_src[jj[u]] + (k - s_rel[jj[u]])] : 0;
        }
    };
    auto put = [&](uint64_t k0, const int32_t (&v)[U]) {
#pragma unroll
        for (unsigned u = 0; u < U; u++) {
            const uint64_t k = k0 + (uint64_t)u * FIN_THREADS + tid;
            if (k < k_end) f.ids[o0 + k] = v[u];
        }
    };
    constexpr uint64_t STEP = (uint64_t)FIN_THREADS * U;
    if (FIN_PIPE && f.slices > 1 && total < (1ull << 30)) {
        // Calls split into slices (under ~512k strings, the strong-scaling shards): the next round's
        // loads go out before this round's stores -- a load waits for every older vector-memory op of
        // the wave, stores included, so loads behind the stores put a store's latency on every round.
        // Branch-free rounds (ids past the slice re-read its last one; buffer stores past the slice's
        // ids are dropped by the range check) let the waits count: the stores wait only for the older
        // round's loads.  32-bit batch-relative ids (total < 2^30).  125k strings -2.4 %; at 1M (one
        // slice, 13 rounds per block, the copy at HBM's pace) it measured +2.2 % (r05w), so one-slice
        // calls keep the plain rounds.
        // (the slice's bounds are block-uniform: readfirstlane keeps the store resource in SGPRs)
        const unsigned kb = uni((unsigned)k_beg);
        const unsigned n = uni((unsigned)(k_end - k_beg)), kl = kb + n - 1u;
        const uint64_t ob = (uint64_t)(uintptr_t)(f.ids + o0 + k_beg);
        const uint64_t obu = uni64(ob);   // (uni: unsigned halves -- a raw readfirstlane is int and sign-extends)
        const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(uintptr_t)obu, (short)0, (int)(n * 4u), 0x00020000);
        auto gather32 = [&](unsigned r0, int32_t (&v)[U]) {   // ids kb + r0 + u * FIN_THREADS + tid
            unsigned kk[U], jj[U];
#pragma unroll
            for (unsigned u = 0; u < U; u++) {
                kk[u] = min(kb + r0 + u * FIN_THREADS + tid, kl);
                jj[u] = s_map[kk[u] >> gs];
            }
#pragma unroll
            for (unsigned u = 0; u < U; u++) jj[u] += (unsigned)s_rel[jj[u] + 1] <= kk[u] ? 1u : 0u;
#pragma unroll
            for (unsigned u = 0; u < U; u++)
                while ((unsigned)s_rel[jj[u] + 1] <= kk[u]) jj[u]++;   // (strings shorter than a row)
#pragma unroll
            for (unsigned u = 0; u < U; u++) v[u] = (int32_t)staging[s_src[jj[u]] + (kk[u] - (unsigned)s_rel[jj[u]])];
        };
        auto put32 = [&](unsigned r0, const int32_t (&v)[U]) {
#pragma unroll
            for (unsigned u = 0; u < U; u++)
                __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v[u], out, (r0 + u * FIN_THREADS + tid) * 4u, 0, 0);
        };
        if (n) {
            // two register sets in turn (a copy between them would wait for the loads)
            int32_t va[U], vb[U];
            gather32(0, va);
            for (unsigned r0 = 0;;) {
                if (r0 + STEP >= n) { put32(r0, va); break; }
                gather32(r0 + (unsigned)STEP, vb);
                put32(r0, va);
                r0 += (unsigned)STEP;
                if (r0 + STEP >= n) { put32(r0, vb); break; }
                gather32(r0 + (unsigned)STEP, va);
                put32(r0, vb);
                r0 += (unsigned)STEP;
            }
        }
    } else {
        for (uint64_t k0 = k_beg; k0 < k_end; k0 += STEP) {
            int32_t v[U];
            gather(k0, v);
            put(k0, v);
        }
    }
}

// dpt_encode_padded runs no finish pass: one lane resets the counter block after the tokenize passes
__global__ void __launch_bounds__(64) reset_kernel(uint32_t *ctr) {
    if (threadIdx.x == 0) reset_counters(ctr);
}

// ------------------------------------------------------------------ histogram

// Token-count histogram: LDS-privatised int64 bins, one LDS atomic per string for its count bin
// (peeling distinct bins per wave with ballots measured slower: 36 vs 30 us on cfg2); statuses --
// nearly all 0, so per-lane atomics would serialise 64-way on one bin -- by one ballot per value.
constexpr unsigned HIST_THREADS = 1024;
__global__ void __launch_bounds__(HIST_THREADS) hist_kernel(const uint64_t *__restrict__ id_off, const int32_t *__restrict__ status,
                                                   uint64_t n_str, unsigned long long *hist, uint32_t n_bins) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lh[];
    const uint32_t nb = n_bins + 8;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) lh[b] = 0;
    __syncthreads();
    const unsigned lane = threadIdx.x & 63u;
    unsigned long long tok = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // every lane of a wave runs the same number of rounds (ballots over the whole wave)
    const uint64_t s_first = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    for (uint64_t s0 = s_first; s0 < n_str; s0 += stride) {
        const uint64_t s = s0 + lane;
        const bool in = s < n_str;
        uint32_t bin = 0xFFFFFFFFu;
        int32_t st = -1;
        if (in) {
            const uint64_t n = id_off[s + 1] - id_off[s];
            tok += n;
            bin = n < n_bins - 1 ? (uint32_t)n : n_bins - 1;
            st = status[s];
            st = st >= 0 && st <= 4 ? st : 4;
        }
        if (in) atomicAdd(&lh[bin], 1ull);
#pragma unroll
        for (int v = 0; v < 5; v++) {
            const uint64_t m = __ballot(st == v);
            if (lane == 0 && m) atomicAdd(&lh[n_bins + 2 + v], (unsigned long long)__builtin_popcountll(m));
        }
    }
    atomicAdd(&lh[n_bins], tok);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&lh[n_bins + 1], (unsigned long long)n_str);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
        if (lh[b]) atomicAdd(&hist[b], lh[b]);
}

// ------------------------------------------------------------------ the fallback passes in one launch

constexpr int SMALL_CH = 256;   // the first pass's window
constexpr int MID_CH = 512;     // the 512-byte pass's (PRESPLIT / ATOMS calls of 16-lane vocabularies)
constexpr int BIG_CH = 2048;    // the 2048-byte pass's

// The 2048-byte pass and the unbounded pass as ONE launch (they used to be two, ~5 us each on every call
// although their lists are usually empty).  Each block takes a ticket: the first n_big tickets run the
// 2048-byte pass (tokenize_body), the others the unbounded pass (lng::long_body) once every 2048-byte
// block has finished -- that pass appends to the unbounded pass's list.  A waiting block waits only for
// blocks that hold earlier tickets, so are running (no dispatch-order assumption).  The
// list's entries are published like any inter-workgroup hand-off on MI355X (per-XCD L2s): an agent-scope
// release by each 2048-byte block that stored any, a relaxed done counter, one acquire on the other side.
struct FallbackArgs {
    KernArgs k;              // first: tokenize_body reads it through the kernarg segment pointer
    lng::Args l;
    uint32_t *ticket, *big_done;   // counter block uint32 [6] / [1] (reset_counters zeroes them)
    unsigned n_big;
};

template <bool WIDE, bool RAW>
__global__ void __launch_bounds__(64) fallback_kernel(FallbackArgs fa) {
    const unsigned lane = lane_id();
    // Both lists are final here (the first pass ran before this launch): when both are empty -- nearly
    // every call -- no block takes a ticket or waits for the 2048-byte blocks (the same-address ticket and
    // done-counter atomics and the waits were most of the empty launch's ~10 us)
    if (*fa.k.ea.work_count == 0 && *fa.l.list_count == 0) {
        const auto &e = fa.k.ea;
        if (e.hist_zero && blockIdx.x == 0)
            for (uint32_t b = lane; b < e.n_hist; b += 64u) e.hist_zero[b] = 0;
        return;
    }
    unsigned t = 0;
    if (lane == 0) t = atomicAdd(fa.ticket, 1u);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t < fa.n_big) {
        const bool work = *fa.k.ea.work_count != 0;
        tokenize_body<BIG_CH, 64, true, WIDE, 0, RAW>(t);
        if (work) {   // (long-list entries may have been stored)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) atomicAdd(fa.big_done, 1u);
        return;
    }
    // the unbounded pass, after every 2048-byte block (bounded: they are running; 2 s at 100 MHz)
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(fa.big_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fa.n_big) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;   // (never expected; results then stale)
        __builtin_amdgcn_s_sleep(4);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    lng::long_body(fa.l);
}

// ------------------------------------------------------------------ launchers

static_assert(block_lds_bytes<SMALL_CH, 16>() <= 64 * 1024, "small LDS");
static_assert(block_lds_bytes<SMALL_CH, 64>() <= 64 * 1024, "small LDS");
static_assert(block_lds_bytes<BIG_CH, 64>() <= 160 * 1024, "big LDS");
static_assert(block_lds_bytes<MID_CH, 16>() <= 64 * 1024, "mid LDS");

// The 512-byte pass (PRESPLIT / ATOMS calls, 16-lane vocabularies): the first pass's retry list -- strings
// with a word of 257..512 bytes, which marker bytes make common there (cfg2p: a 256-character word plus
// its '\u2581' is 257 code points) -- four strings per wave in 16-lane rows like the first
// pass (the generic walker, C2's hash pass and walkers: no A0 / bulk pass), ~7 waves per CU (LDS); its own
// failures go on to the 2048-byte pass.  A persistent grid over the list: with no retries every wave reads
// a zero count and exits.
template <int SW, bool WIDE, int MC = -1>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) mid_kernel(KernArgs ka) {
    tokenize_body<MID_CH, 16, true, WIDE, SW, false, false, MC>(blockIdx.x);
}

constexpr int MAX_DEVICES = 64;
// Resident waves per CU for an instantiation (LDS / VGPR limited); DPT_WAVES_PER_CU overrides.
template <int CH, int G, bool BIG, bool WIDE, int SW = 0, bool RAW = false, bool SOLO = false, int MC = -1>
static unsigned resident_per_cu() {
    static unsigned cached[MAX_DEVICES] = {};   // per device: a process may drive several
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES) dev = 0;
    if (cached[dev]) return cached[dev];
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, tokenize_kernel<CH, G, BIG, WIDE, SW, RAW, SOLO, MC>, 64, block_lds_bytes<CH, G>()) != hipSuccess || nb <= 0)
        nb = 8;
    {   // the residency by LDS at its 512-byte allocation granule: the occupancy API counts 22 blocks of
        // 7 424 B per CU, the timeline shows 21 resident and the 22nd starting only when another exits
        // (profiles/r06_ab.log r06b; 21 against 22 at 175k / 250k: +0.9 %, r06o)
        constexpr int g = DPT_WPC_GRAN;
        const int fit = (160 * 1024) / ((block_lds_bytes<CH, G>() + g - 1) / g * g);
        if (fit < nb) nb = fit;
    }
    if (const char *e = getenv("DPT_WAVES_PER_CU")) {
        const int v = atoi(e);
        if (v > 0) nb = v;
    }
    cached[dev] = (unsigned)nb;
    return cached[dev];
}

// Persistent grid: every resident wave pulls strings from the work counter until it runs dry.
template <int CH, int G, bool BIG, bool WIDE, int SW = 0, bool RAW = false, bool SOLO = false, int MC = -1>
static void launch_tok(const EncodeArgs &a, const TrieView &tv, uint64_t n_units, unsigned n_cu, hipStream_t stream,
                       hipEvent_t ev_start = nullptr) {
    constexpr int lds = block_lds_bytes<CH, G>();
    uint64_t wpc = resident_per_cu<CH, G, BIG, WIDE, SW, RAW, SOLO, MC>();
    static const bool small_rule = getenv("DPT_NO_SMALL_WPC") == nullptr;   // (A/B: the rule below off)
    if (G == 16 && !BIG && small_rule) {
        // small calls: no more resident waves than give every slot ~7 strings (rounds of 4 strings per
        // wave; a wave's last round is the tail): 125k strings run 3 % faster at 18 waves per CU than
        // at the occupancy limit of 22, 250k and more are fastest at 22 (profiles/r02_ab_issue_model.log)
        const uint64_t want = (n_units + 7ull * n_cu - 1) / (7ull * n_cu);   // n_units = strings / 4
        const uint64_t lo = wpc < DPT_WPC_LO ? wpc : DPT_WPC_LO;
        if (want < wpc) {
            // of the wave counts from lo up, the one with the fewest slot-rounds w * ceil(rounds) -- the
            // work plus the idle part of the last round -- the smallest on ties (100k strings: 20 waves
            // per CU, 4.9 rounds).  lo = 20: a CU's string throughput grows up to 20-21 waves (r06c:
            // 0.411 / 0.424 / 0.431 / 0.434 string-rounds per us at 18..21), which a shorter last
            // round at 16-18 waves does not pay back (125k: 18 -> 21 waves, +1.9 %, r06o)
            uint64_t best = lo, bc = ~0ull;
            for (uint64_t w = lo; w <= wpc; w++) {
                const uint64_t c = w * ((n_units + w * n_cu - 1) / (w * n_cu));
                if (c < bc) { bc = c; best = w; }
            }
            wpc = best;
        }
    }
    uint64_t blocks = (uint64_t)n_cu * wpc;
    if (blocks > (uint64_t)n_cu * 64u) blocks = (uint64_t)n_cu * 64u;   // the scratch is sized for 64 per CU
    if (blocks > n_units) blocks = n_units ? n_units : 1;
    if (ev_start)   // the start timestamp rides on the dispatch (a separate hipEventRecord left a ~6 us bubble)
        hipExtLaunchKernelGGL((tokenize_kernel<CH, G, BIG, WIDE, SW, RAW, SOLO, MC>), dim3((unsigned)blocks), dim3(64), lds, stream,
                              ev_start, nullptr, 0, KernArgs{a, tv});
    else
        hipLaunchKernelGGL((tokenize_kernel<CH, G, BIG, WIDE, SW, RAW, SOLO, MC>), dim3((unsigned)blocks), dim3(64), lds, stream, KernArgs{a, tv});
}

hipError_t launch_encode(const EncodeLaunch &p, hipStream_t stream, hipEvent_t ev[2]) {
    EncodeArgs a;
    a.text = p.text; a.str_off = p.str_off; a.cut_mask = p.cut_mask; a.n_str = p.n_str;
    a.staging = p.staging; a.staging16 = p.staging16; a.counts = p.counts; a.bsum = p.padded ? nullptr : p.flags; a.status = p.status; a.capped = p.capped;
    a.retry_list = p.retry_list; a.retry_count = p.retry_count; a.work_list = nullptr; a.work_count = nullptr;
    a.long_list = p.retry_list + p.n_str; a.long_count = p.retry_count + 3;
    a.mode = p.mode;
    a.edges = p.edges;
    a.work_next = p.retry_count + 1;
    a.part_ctr = p.retry_count + PART_CTR_OFFSET / 4;
    a.wsl_scratch = p.wsl_scratch;
    a.pend = p.pend; a.ws_node = p.ws_node; a.ws_base = p.ws_base; a.ws_id = p.ws_id;
    a.long_span = p.long_span;
    a.hist_zero = nullptr; a.n_hist = 0;
    a.id_off = p.id_off; a.ids = p.ids;
    a.solo = p.solo ? 1 : 0; a.ctr_snap = p.ctr_snap;
    const bool solo = p.solo && p.n_str == 1 && !p.padded;
    int16_t *const st16 = solo ? nullptr : p.staging16;   // (the 16-lane launch below picks the width by it)
    if (solo) {
        a.staging = p.ids; a.staging16 = nullptr; a.counts = p.id_off + 1; a.bsum = nullptr;
    } else {
        a.solo = 0;
    }
    TrieView tv{p.slots, p.slot_ids, p.slots4, p.root_base, p.n_slots, p.pair16};
    const bool wide = (p.mode & DPT_MODE_MASK) == DPT_MODE_ATOMS;   // atoms of up to 8 bytes
    const bool raw = (p.mode & DPT_MODE_MASK) == DPT_MODE_RAW;

    if (p.n_str == 0) {
        // no finish kernel runs: id_off[0] = 0, and the call's claimed arena bytes ("last need") and
        // far edge pairs are 0 (bytes 40..63 of the counter block; the running counters are 0 already)
        if (p.id_off) {   // (dpt_encode_padded has no offsets)
            const hipError_t e0 = hipMemsetAsync(p.id_off, 0, sizeof(uint64_t), stream);
            if (e0 != hipSuccess) return e0;
        }
        if (p.hist && p.hist_overwrite) {   // the histogram of no strings
            const hipError_t e1 = hipMemsetAsync(p.hist, 0, ((size_t)p.hist_bins + 8u) * sizeof(int64_t), stream);
            if (e1 != hipSuccess) return e1;
        }
        return hipMemsetAsync(reinterpret_cast<uint64_t *>(p.retry_count) + CTR_LASTNEED64, 0, 3 * sizeof(uint64_t), stream);
    }
    // profiling (dpt_ctx_profile): the first pass's dispatch records ev[0], the unbounded pass's ev[1]
    hipEvent_t e0 = ev ? ev[0] : nullptr;
    // PRESPLIT (llama mode) and ATOMS run instantiations with the mode a compile-time constant (MC)
    static const bool generic_ps = getenv("DPT_GENERIC_PS") != nullptr;   // (A/B: the runtime-mode kernels)
    const bool presplit = (p.mode & DPT_MODE_MASK) == DPT_MODE_PRESPLIT;
    // ... and, like the RAW ones, only for calls without edges, the uncapped DP or len_only (PLAIN)
    const bool plain = p.edges == nullptr && (p.mode & (DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY)) == 0;
    const bool spec = plain && !generic_ps;
    if (p.n_str > 0) {
        {
            const unsigned n_cu = p.max_blocks / 64;
            // A/B knob (diagnostic): raw mode through the generic 16-lane kernel (r06i: cfg2 +9 %, cfg4 +7 %)
            static const bool generic_raw = getenv("DPT_GENERIC_RAW") != nullptr;
            if (p.variant == KERNEL_ROWS16) {
                // the hot kernel gets the staged id width as a template constant
                const uint64_t nu = (p.n_str + 3) / 4;
                static const bool solo_wave = getenv("DPT_NO_SOLO_WAVE") == nullptr;   // (A/B: solo calls on 16-lane rows)
                if (solo && !wide && solo_wave) {
                    // the one-string kernel: lane-mode B and its C1 walks over the whole wave (forward_lanes, SOLO)
                    if (raw) launch_tok<SMALL_CH, 16, false, false, 2, true, true>(a, tv, 1, n_cu, stream, e0);
                    else launch_tok<SMALL_CH, 16, false, false, 2, false, true>(a, tv, 1, n_cu, stream, e0);
                } else if (wide) {
                    if (!spec) {
                        if (st16) launch_tok<SMALL_CH, 16, false, true, 1>(a, tv, nu, n_cu, stream, e0);
                        else launch_tok<SMALL_CH, 16, false, true, 2>(a, tv, nu, n_cu, stream, e0);
                    } else {
                        if (st16) launch_tok<SMALL_CH, 16, false, true, 1, false, false, DPT_MODE_ATOMS>(a, tv, nu, n_cu, stream, e0);
                        else launch_tok<SMALL_CH, 16, false, true, 2, false, false, DPT_MODE_ATOMS>(a, tv, nu, n_cu, stream, e0);
                    }
                } else if (raw && plain && !generic_raw) {
                    if (st16) launch_tok<SMALL_CH, 16, false, false, 1, true>(a, tv, nu, n_cu, stream, e0);
                    else launch_tok<SMALL_CH, 16, false, false, 2, true>(a, tv, nu, n_cu, stream, e0);
                } else if (presplit && spec) {
                    if (st16) launch_tok<SMALL_CH, 16, false, false, 1, false, false, DPT_MODE_PRESPLIT>(a, tv, nu, n_cu, stream, e0);
                    else launch_tok<SMALL_CH, 16, false, false, 2, false, false, DPT_MODE_PRESPLIT>(a, tv, nu, n_cu, stream, e0);
                } else {
                    if (st16) launch_tok<SMALL_CH, 16, false, false, 1>(a, tv, nu, n_cu, stream, e0);
                    else launch_tok<SMALL_CH, 16, false, false, 2>(a, tv, nu, n_cu, stream, e0);
                }
            } else {
#if DPT_STOP == 3   // (this diagnostic build crashes ROCm 7.2's register allocator on the 64-lane first pass)
                return hipErrorNotSupported;
#else
                if (wide && spec) launch_tok<SMALL_CH, 64, false, true, 0, false, false, DPT_MODE_ATOMS>(a, tv, p.n_str, n_cu, stream, e0);
                else if (wide) launch_tok<SMALL_CH, 64, false, true>(a, tv, p.n_str, n_cu, stream, e0);
                else if (raw && plain) launch_tok<SMALL_CH, 64, false, false, 0, true>(a, tv, p.n_str, n_cu, stream, e0);
                else launch_tok<SMALL_CH, 64, false, false>(a, tv, p.n_str, n_cu, stream, e0);
#endif
            }
        }
        if (solo) return hipGetLastError();   // the lone wave did the rest
        // second pass over the strings whose single word (or expansion) did not fit the small window
        EncodeArgs b = a;
        b.work_list = p.retry_list; b.work_count = p.retry_count;
        b.work_next = p.retry_count + 2;
        static const bool mid_on = getenv("DPT_NO_MID") == nullptr;   // (A/B: the 512-byte pass off)
        if (!raw && p.variant == KERNEL_ROWS16 && mid_on) {
            // the 512-byte pass over the retry list; the strings it cannot hold go on to the 2048-byte pass
            EncodeArgs m = a;
            m.work_list = p.retry_list; m.work_count = p.retry_count; m.work_next = p.retry_count + 5;
            m.retry_list = p.retry_list + 2 * p.n_str; m.retry_count = p.retry_count + 7;
            m.hist_zero = nullptr; m.n_hist = 0;
            static unsigned mid_per_cu[MAX_DEVICES] = {};
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES) dev = 0;
            if (!mid_per_cu[dev]) {
                int nb = 0;
                if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, st16 ? (wide ? mid_kernel<1, true> : mid_kernel<1, false>)
                                                                            : (wide ? mid_kernel<2, true> : mid_kernel<2, false>),
                                                                 64, block_lds_bytes<MID_CH, 16>()) != hipSuccess || nb <= 0)
                    nb = 4;
                mid_per_cu[dev] = (unsigned)nb;
            }
            uint64_t mb = (uint64_t)(p.max_blocks / 64) * mid_per_cu[dev];
            mb = mb < p.n_str ? mb : p.n_str;
            constexpr int mlds = block_lds_bytes<MID_CH, 16>();
            // (wide <=> ATOMS mode; the mode-constant instantiations for PLAIN calls unless DPT_GENERIC_PS)
            auto mk = !spec ? (st16 ? (wide ? mid_kernel<1, true> : mid_kernel<1, false>) : (wide ? mid_kernel<2, true> : mid_kernel<2, false>))
                    : st16 ? (wide ? mid_kernel<1, true, DPT_MODE_ATOMS> : presplit ? mid_kernel<1, false, DPT_MODE_PRESPLIT> : mid_kernel<1, false>)
                           : (wide ? mid_kernel<2, true, DPT_MODE_ATOMS> : presplit ? mid_kernel<2, false, DPT_MODE_PRESPLIT> : mid_kernel<2, false>);
            hipLaunchKernelGGL(mk, dim3((unsigned)(mb ? mb : 1)), dim3(64), mlds, stream, KernArgs{m, tv});
            b.work_list = m.retry_list; b.work_count = m.retry_count;
        }
        if (!p.padded && fin_fold(p.n_str) && p.hist && p.hist_overwrite && p.hist_bins >= 2 &&
            p.hist_bins <= FIN_MAX_BINS) {
            b.hist_zero = reinterpret_cast<unsigned long long *>(p.hist);   // (the finish pass adds to it)
            b.n_hist = p.hist_bins + 8u;
        }
        // the fallback passes' grids: 1/FALLBACK_DIV of a full one (usually they find no work; 16 / 64
        // within noise, r03ah)
        constexpr unsigned FALLBACK_DIV = 4;
        // (n_units caps the grid: one block per FALLBACK_DIV CUs; the retry list is rare and short)
        uint64_t fb_units = (uint64_t)(p.max_blocks / 64) / FALLBACK_DIV;
        // PRESPLIT / ATOMS text carries its word markers as bytes ('\u2581' is 3 of them), so a word the
        // 256-byte window cannot hold is not rare there (cfg2p: the 6.8 % of 256-character strings without a
        // space are one 257-code-point word after the dummy prefix): a full grid of 2048-byte blocks (three
        // per CU: LDS) takes them, instead of one block per four CUs (DPT_FB_BIG_PER_CU overrides)
        {
            static const int per_cu = getenv("DPT_FB_BIG_PER_CU") ? atoi(getenv("DPT_FB_BIG_PER_CU")) : 3;
            if (!raw && per_cu > 0) fb_units = (uint64_t)(p.max_blocks / 64) * (uint64_t)per_cu;
        }
        fb_units = fb_units < p.n_str ? fb_units : p.n_str;
        // (skipped when the host showed no string needs them -- small host-path calls: two dispatches
        // of a per-string dp_tokenize call -- unless they time the call or zero its histogram)
        const bool fallback = !p.no_fallback || ev || b.hist_zero;
        // the unbounded pass over whatever the windowed passes could not hold (usually nothing:
        // its waves read a zero count and exit)
        LongLaunch l;
        l.mode = p.mode; l.text = p.text; l.str_off = p.str_off; l.cut_mask = p.cut_mask;
        l.staging = p.staging; l.staging16 = p.staging16; l.counts = p.counts; l.bsum = p.padded ? nullptr : p.flags; l.status = p.status; l.capped = p.capped;
        l.arena = p.arena; l.arena_cap = p.arena_cap; l.arena_bias = p.counter_bias;
        l.arena_used = reinterpret_cast<unsigned long long *>(p.retry_count + 8);
        l.edges = p.edges; l.far = p.far; l.far_cap = p.far_cap;
        l.far_count = reinterpret_cast<unsigned long long *>(p.retry_count) + CTR_FAR64;
        l.list = a.long_list; l.list_count = a.long_count; l.work_next = p.retry_count + 4;
        l.slots = p.slots; l.slots4 = p.slots4; l.n_slots = p.n_slots; l.root_base = p.root_base;
        l.max_tok_bytes = p.max_tok_bytes; l.long_span = p.long_span;
        const uint64_t lcap = (uint64_t)(p.max_blocks / 16) / FALLBACK_DIV;
        const uint64_t lb = p.n_str < lcap ? p.n_str : lcap;
        l.blocks = (unsigned)(lb ? lb : 1);
        if (fallback) {   // both passes, one launch (fallback_kernel); the end timestamp rides on it
            FallbackArgs fa;
            fa.k = KernArgs{b, tv};
            fa.l = lng::long_args(l);
            fa.ticket = p.retry_count + 6;
            fa.big_done = p.retry_count + 1;
            fa.n_big = (unsigned)(fb_units ? fb_units : 1);
            const dim3 grid(fa.n_big + l.blocks);
            constexpr int lds = block_lds_bytes<BIG_CH, 64>();
            auto go = [&](auto kern) {
                if (ev) hipExtLaunchKernelGGL(kern, grid, dim3(64), lds, stream, nullptr, ev[1], 0, fa);
                else hipLaunchKernelGGL(kern, grid, dim3(64), lds, stream, fa);
            };
            if (wide) go(fallback_kernel<true, false>);
            else if (raw) go(fallback_kernel<false, true>);
            else go(fallback_kernel<false, false>);
        }
    }
    if (p.padded) {   // dpt_encode_padded: the ids are in place; only the counters need their reset
        hipLaunchKernelGGL(reset_kernel, dim3(1), dim3(64), 0, stream, p.retry_count);
        return hipGetLastError();
    }
    // batch prefixes (and the counter block's reset), then the CSR pass; a one-batch call (<= 256
    // strings: the drop-in's per-string calls) needs no prefix, and its finish block does the rest.
    hipStream_t fs = stream;
    const uint64_t nb = (p.n_str + FIN_BATCH - 1) / FIN_BATCH;
    FinishArgs f;
    f.bsum = nullptr; f.ctr = nullptr; f.fold = nullptr; f.fold_zero = nullptr; f.fold_n = 0;
    f.ctr_snap = p.ctr_snap;
    const bool fold = fin_fold(p.n_str);
    const bool fold_hist = p.hist && p.hist_bins >= 2 && p.hist_bins <= FIN_MAX_BINS;
    f.hist = fold_hist ? reinterpret_cast<unsigned long long *>(p.hist) : nullptr;
    f.status = p.status;
    f.n_bins = p.hist_bins;
    f.hist_store = (fold_hist && p.hist_overwrite && nb <= 1) ? 1 : 0;
    unsigned long long *hz = (fold_hist && p.hist_overwrite && nb > 1 && !fold) ? f.hist : nullptr;
    if (fold) { f.fold = p.flags; f.fold_zero = p.zero_other; f.fold_n = p.zero_n; f.ctr = p.retry_count; }
    else if (nb > 1) hipLaunchKernelGGL(batch_scan_kernel, dim3(1), dim3(SCAN_THREADS), 0, fs, p.n_str, p.flags, p.bpre, p.retry_count,
                                        hz, p.hist_bins + 8u, p.ctr_snap);
    else { f.bsum = p.flags; f.ctr = p.retry_count; }
    f.staging = p.staging16 ? (const void *)p.staging16 : (const void *)p.staging;
    f.str_off = p.str_off; f.counts = p.counts; f.n_str = p.n_str; f.id_off = p.id_off; f.ids = p.ids;
    f.bpre = p.bpre;
    uint64_t sls = (FIN_TARGET_BLOCKS + nb - 1) / nb;
    f.slices = (unsigned)(sls < 1 ? 1 : (sls > FIN_MAX_SLICES ? FIN_MAX_SLICES : sls));
    const uint64_t fb = nb * f.slices;
    if (p.staging16) {
        hipLaunchKernelGGL(finish_kernel<int16_t>, dim3((unsigned)fb), dim3(FIN_THREADS), 0, fs, f);
    } else {
        hipLaunchKernelGGL(finish_kernel<int32_t>, dim3((unsigned)fb), dim3(FIN_THREADS), 0, fs, f);
    }
    hipError_t eh = hipGetLastError();
    if (eh == hipSuccess && p.hist && !fold_hist) {   // too many bins for the finish pass's LDS: the separate pass
        if (p.hist_overwrite && (eh = hipMemsetAsync(p.hist, 0, ((size_t)p.hist_bins + 8u) * sizeof(int64_t), fs)) != hipSuccess)
            return eh;
        eh = launch_histogram(p.id_off, p.status, p.n_str, p.hist, p.hist_bins, fs);
    }
    return eh;
}

size_t pend_scratch_bytes(unsigned max_blocks) { return (size_t)max_blocks * 64 * sizeof(uint4); }

size_t wsl_scratch_bytes(unsigned max_blocks) {
    return (size_t)max_blocks * 4 * GroupLDS<SMALL_CH, 16>::WSL_STRIDE;   // NG x stride covers both G at CH = 256
}

hipError_t launch_histogram(const uint64_t *id_off, const int32_t *status, uint64_t n_str, int64_t *hist,
                            uint32_t n_bins, hipStream_t stream) {
    if (n_str == 0) return hipSuccess;
    constexpr uint64_t HIST_BLOCKS = 256;
    uint64_t blocks = (n_str + HIST_THREADS - 1) / HIST_THREADS;
    if (blocks > HIST_BLOCKS) blocks = HIST_BLOCKS;   // each block adds its bins to the global ones once
    hipLaunchKernelGGL(hist_kernel, dim3((unsigned)blocks), dim3(HIST_THREADS), (n_bins + 8) * sizeof(unsigned long long), stream,
                       id_off, status, n_str, (unsigned long long *)hist, n_bins);
    return hipGetLastError();
}

hipError_t kernel_init() {
    // function attributes are per device: set them once on each device a call runs on
    static bool done[MAX_DEVICES] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES) dev = 0;
    if (done[dev]) return hipSuccess;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&tokenize_kernel<BIG_CH, 64, true, false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, block_lds_bytes<BIG_CH, 64>());
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(&tokenize_kernel<BIG_CH, 64, true, false, 0, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, block_lds_bytes<BIG_CH, 64>());
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(&tokenize_kernel<BIG_CH, 64, true, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, block_lds_bytes<BIG_CH, 64>());
    for (const void *k : {reinterpret_cast<const void *>(&fallback_kernel<true, false>), reinterpret_cast<const void *>(&fallback_kernel<false, true>),
                          reinterpret_cast<const void *>(&fallback_kernel<false, false>)})
        if (e == hipSuccess) e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, block_lds_bytes<BIG_CH, 64>());
    if (e == hipSuccess) done[dev] = true;
    return e;
}

int small_window_bytes() { return SMALL_CH; }
int big_window_bytes() { return BIG_CH; }

#ifdef DPT_STAMPS
extern "C" int dpt_debug_stamps(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 10) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[10] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
#ifdef DPT_WSTAMPS
// the first pass's per-wave timeline (WST_REC): WST_MAXW x WST_N u64 into out; reset zeroes it
extern "C" int dpt_debug_wstamps(unsigned long long *out, int reset) {
    const size_t nbytes = sizeof(unsigned long long) * WST_MAXW * WST_N;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wst), nbytes) != hipSuccess) return -1;
    if (reset) {
        void *p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_wst)) != hipSuccess || hipMemset(p, 0, nbytes) != hipSuccess) return -1;
    }
    return 0;
}
extern "C" int dpt_debug_wstamps_dims(unsigned *maxw, unsigned *n) { *maxw = WST_MAXW; *n = WST_N; return 0; }
#endif

}  // namespace dpt
