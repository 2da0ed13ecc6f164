// Internal interface between the C-ABI (dpt_api.cpp) and the kernels (dpt_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/dpt.h"

namespace dpt {

struct EncodeLaunch {
    int mode;                // DPT_MODE_* | DPT_FLAG_*
    uint64_t *edges;         // nullable: per atom end E(i)&reachable masks (n_bytes entries)
    uint64_t *far;           // nullable (with edges): optimal predecessors more than 64 atoms back, as
    uint64_t far_cap;        //   (end index, back distance) pairs -- far_cap pairs; the count is in the counter block
    const uint8_t *text;
    const uint64_t *str_off;
    const uint8_t *cut_mask;
    uint64_t n_str;
    int32_t *ids;
    uint64_t *id_off;
    int32_t *status;
    int32_t *capped;
    // workspace
    int32_t *staging;
    int16_t *staging16;      // non-null: ids staged as int16 here instead (every vocabulary id in 0..32767)
    uint64_t *counts;
    uint32_t *retry_list;    // 2 x n_str: the 2048-byte pass's list, then (at + n_str) the unbounded pass's list
    uint32_t *retry_count;   // the 64-byte counter block (dpt_kernels.hip, finish_kernel)
    uint8_t *wsl_scratch;    // max_blocks x wsl_scratch_bytes(1) bytes
    int long_span;           // vocabulary tokens longer than 64 code points: words over 64 atoms -> unbounded pass
    uint32_t max_tok_bytes;  // longest vocabulary token, bytes
    unsigned long long *flags;   // the batch lines (BS_LINE below): per FIN_BATCH-string batch, the sum of its counts,
                                 //   added by the tokenize passes as strings finish; zeroed for the next call
    unsigned long long *bpre;    // per batch (dense): its exclusive id prefix (batch_scan_kernel)
    unsigned long long *zero_other;   // fold calls: the other parity's batch lines, zeroed for the next call ...
    uint64_t zero_n;             // ... (batches)
    uint64_t *ctr_snap;          // nullable (host path): the counter block's first 64 bytes, copied here by its reset
    bool no_fallback;            // the host checked that no string needs the 2048-byte or unbounded pass: skip them
    uint64_t n_bytes = 0;        // the call's input bytes
    bool solo;                   // one-string host-path call without fallbacks, histogram, edges or profiling: the first
                                 //   pass writes the CSR arrays itself (ids at 0.., id_off = {0, count}) and resets
                                 //   the counter block (its snapshot to ctr_snap); nothing else is launched
    unsigned max_blocks;
    int variant;             // KERNEL_* below
    bool padded;             // dpt_encode_padded: staging = the caller's ids, counts = the caller's; no finish pass
    uint4 *pend;             // 16-lane first pass: each wave's pending residual tokens (pend_scratch_bytes)
    int64_t *hist;           // nullable: the token-count histogram to add to in the finish pass (dpt_ctx_set_histogram)
    uint32_t hist_bins;
    bool hist_overwrite;     // DPT_HIST_OVERWRITE: the call's histogram replaces hist (zeroed on the device first)
    uint8_t *arena;          // the unbounded pass's scratch: 20 bytes per input byte of the strings it takes
    uint64_t arena_cap;      // input bytes the arena holds
    uint64_t counter_bias;   // test-only (dpt_ctx_debug_counter_bias): the arena and far-pair counters start at it
    // vocabulary
    const int2 *slots;
    const int32_t *slot_ids;
    const int16_t *pair16;   // ids of the one- and two-byte tokens (PAIR16_N int16), then phase A0's byte-pair flags
                             //   + child filters (65536 uint2) -- dpt_api.cpp dpt_vocab_create
    const int4 *slots4;      // {base | TERM<<31 | LEAF<<30, check, id, child filter}
    uint32_t n_slots;
    int32_t root_base;
    int32_t ws_node, ws_base, ws_id;   // the trie node after U+2581, its base word and id (-1: none)
};

// first-pass work partitions (dpt_kernels.hip tokenize_kernel): up to NPART_MAX counters, one per
// PART_STRIDE uint32 (a 256-byte line each), from byte PART_CTR_OFFSET of the counter block, then the
// used-up mask; the counter block is CTR_ALLOC_BYTES long (the host path copies its first 64 bytes)
constexpr unsigned NPART_MAX = 32;
// entries of the pair-id table (65536 byte pairs + 256 single bytes, int16; a multiple of 4 so the
// A0 table after it is 8-byte aligned)
constexpr unsigned PAIR16_N = 65536 + 256;
// strings per finish batch (the batch arrays are sized one per 64 strings, two arrays)
constexpr unsigned FIN_BATCH = 256;
constexpr unsigned PART_STRIDE = 64;   // (counters 4 KB apart measured the same, r05i)
// Calls of 2..FIN_FOLD_MAX batches run no batch_scan_kernel: each finish block sums the batch sums
// before its own batch (<= FIN_FOLD_MAX / FIN_THREADS loads per thread), zeroes the OTHER array for
// the next call (the two arrays swap roles: dpt_ctx's flag parity) and block 0 resets the counter
// block.  Saves a launch (~5 us) on the strong-scaling shard sizes (125k..500k strings).
#ifndef FIN_FOLD_MAX_DEF
#define FIN_FOLD_MAX_DEF 2048   // A/B knob (both the API and the kernels must see the same value)
#endif
constexpr unsigned FIN_FOLD_MAX = FIN_FOLD_MAX_DEF;
__host__ __device__ inline bool fin_fold(uint64_t n_str) {
    const uint64_t nb = (n_str + FIN_BATCH - 1) / FIN_BATCH;
    return nb > 1 && nb <= FIN_FOLD_MAX;
}
constexpr unsigned FIN_MAX_BINS = 1024;   // histogram bins the finish pass folds in (more: the separate pass)

// Batch lines (EncodeLaunch::flags): one 128-byte line per batch, so the strings finishing in
// neighbouring batches -- the first pass's partitions run through the batches side by side -- add to
// different lines (16 batches' sums in one line serialised the adds: +0.05 ms at cfg2, +11 % at 125k
// strings, profiles/r04d_ab.log).  u64 [0]: the count sum -- one atomic add per finished string.
constexpr unsigned BS_LINE = 16;
constexpr size_t PART_CTR_OFFSET = 256;
constexpr size_t CTR_ALLOC_BYTES = PART_CTR_OFFSET + (NPART_MAX + 1) * PART_STRIDE * 4;

// child filter bit of next byte b (slots4[].w, host and device): XOR with b >> 5 permutes the
// low five bits inside each 32-byte block, so the 26 lowercase letters get distinct bits
__host__ __device__ inline unsigned child_bit(unsigned b) { return (b ^ (b >> 5)) & 31u; }

// Token hash table (C2's one-lookup ids for tokens of 3..16 expanded bytes; dpt_vocab_create builds
// it after the A0 table in the pair16 allocation).  Key: the token's bytes as four little-endian
// dwords, zero past its length, plus the length.  Buckets of two {fp, id} entries (fp != 0; 0 marks a
// free entry), two choices per key (cuckoo placement, round 5): bucket h & mask or its partner
// tokhash_alt(h & mask, fp).  The kernels load a key's home bucket first and its partner only when the
// key is not in its home bucket (one more load round for the wave, never a chain; DPT_HASH_BOTH=1 in
// dpt_kernels.hip loads both at once -- measured slower on cfg2 / cfg5, round 5 r05aj) -- a lookup never
// walks a probe chain (with linear probing 5.7 % of cfg4's hashed tokens were not in their home bucket,
// and almost every 64-token round ran the serial probe loop for some lane).  The builder checks that the first entry carrying a key's
// fp among its two buckets (in the kernel's order) is its own (else it re-seeds): a span the DP
// selected is a vocabulary token by construction (phase A matched it), so the lookup needs no key
// compare.
constexpr unsigned TOKHASH_MAX_BYTES = 16;        // the 16-lane kernels' keys (four dwords)
constexpr unsigned TOKHASH_MAX_BYTES_LONG = 64;   // the table's tokens; the 64-lane kernels hash keys this long
constexpr size_t TOKHASH_OFFSET = PAIR16_N * sizeof(int16_t) + 65536 * 8;   // bytes into the pair16 allocation
struct TokHashHeader {
    uint32_t mask;        // buckets - 1 (a power of two)
    uint32_t max_probe;   // buckets a lookup visits: 2 (its two choices); 0: no table -- the walkers resolve every token
    uint32_t seed;
    uint32_t nl_id1;      // 1 + the id of "<0x0A>" (0: none): raw mode's one-atom '\n' tokens take it without a lookup
};
// The key is max(4, ceil(len / 4)) little-endian dwords w_k of the token's bytes, zero past its
// length, mixed into one 64-bit state (lo, hi) by one 32 x 32 -> 64 multiply-add per dword (round 5;
// the two murmur/xxHash-style 32-bit chains before cost ~48 VALU per key, ~3 % of cfg4's first pass):
//   start  lo = seed ^ len, hi = seed * G;   per dword  (hi:lo) = (w_k ^ lo) * K[k] + hi;
//   end    (hi:lo) = (lo ^ C) * K[16] + hi,  h = lo ^ hi (the bucket is h & mask), fp = hi | 1.
// The product's high half mixes every bit of (w ^ lo) and is added into the next step's low half, so
// byte-level vocabularies' keys whose differences sit in the top bytes of two dwords do not cancel (a
// linear sum of w_k * K[k] mod 2^32 failed every seed on the 250,680-token BLOOM vocabulary).  (h, fp)
// carry the whole 64-bit state: a fingerprint derived from h alone (round 2) left 32 bits per key and
// ~7 full collisions among the BLOOM keys.
constexpr uint32_t TOKHASH_K[17] = {
    0xFB13EED5u, 0xE031651Bu, 0xD57B9AE9u, 0xF49344BFu, 0xB7A058D5u, 0xB4BC663Du, 0xE3606AA1u, 0x829E9285u, 0x9D183F11u,
    0xF3C85069u, 0xAEAD8A81u, 0xC9C1030Bu, 0xC71547B7u, 0xF78B48A3u, 0xB5FE207Fu, 0xEA0A7265u, 0xC71BEEC7u};
struct TokHashState {
    uint32_t lo, hi;
};
__host__ __device__ inline TokHashState tokhash_start(uint32_t len, uint32_t seed) {
    return {seed ^ len, seed * 0x9E3779B9u};
}
__host__ __device__ inline TokHashState tokhash_step(TokHashState s, uint32_t w, unsigned k) {
    const uint64_t t = (uint64_t)(w ^ s.lo) * TOKHASH_K[k] + s.hi;
    return {(uint32_t)t, (uint32_t)(t >> 32)};
}
__host__ __device__ inline void tokhash_end(TokHashState s, uint32_t &h, uint32_t &fp) {
    const uint64_t t = (uint64_t)(s.lo ^ 0x5BD1E995u) * TOKHASH_K[16] + s.hi;
    h = (uint32_t)t ^ (uint32_t)(t >> 32);
    fp = (uint32_t)(t >> 32) | 1u;
}
// the partner of bucket b for a key of fingerprint fp (an involution: from either bucket, the other)
__host__ __device__ inline uint32_t tokhash_alt(uint32_t b, uint32_t fp, uint32_t mask) { return (b ^ (fp >> 8)) & mask; }
// four-dword keys (tokens of at most 16 bytes)
__host__ __device__ inline void tokhash(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t len, uint32_t seed,
                                        uint32_t &h, uint32_t &fp) {
    TokHashState s = tokhash_start(len, seed);
    s = tokhash_step(s, w0, 0);
    s = tokhash_step(s, w1, 1);
    s = tokhash_step(s, w2, 2);
    s = tokhash_step(s, w3, 3);
    tokhash_end(s, h, fp);
}

// kernel variants for the first pass (the 2048-byte window pass always follows for retries)
constexpr int KERNEL_ROWS16 = 1;  // 4 strings per wave in 16-lane DPP rows, LDS windows (max_cp <= 16)
constexpr int KERNEL_ROWS64 = 2;  // 1 string per wave, 64-lane DPP (max_cp <= 64)

// the unbounded pass (dpt_long.hip): strings the windowed kernels routed to the long list
struct LongLaunch {
    int mode;
    const uint8_t *text;
    const uint64_t *str_off;
    const uint8_t *cut_mask;
    int32_t *staging;        // the final ids (int32 vocabularies) at the string's byte offset + k
    int16_t *staging16;      // as EncodeLaunch: the final ids go here instead when non-null
    uint8_t *arena;          // scratch: uint4 rec[arena_cap] then int32 stg[arena_cap], per string at its
    uint64_t arena_cap;      //   claimed offset (input bytes; 20 bytes of scratch per input byte)
    uint64_t arena_bias;     // test-only: the arena counter starts at it (the kernel's offsets >= bias)
    unsigned long long *arena_used;   // claimed input bytes (all long strings; > arena_cap: overflow)
    uint64_t *counts;
    int32_t *status;
    int32_t *capped;
    uint64_t *edges;
    uint64_t *far;                    // as EncodeLaunch
    uint64_t far_cap;
    unsigned long long *far_count;    // pairs found (all of them; > far_cap: the host grows and reruns)
    unsigned long long *bsum;         // nullable: per FIN_BATCH strings, the sum of their counts (EncodeLaunch::flags)
    const uint32_t *list;
    const uint32_t *list_count;
    uint32_t *work_next;
    const int2 *slots;
    const int4 *slots4;
    uint32_t n_slots;
    int32_t root_base;
    uint32_t max_tok_bytes;
    int long_span;
    unsigned blocks;
};

hipError_t launch_encode(const EncodeLaunch &p, hipStream_t stream, hipEvent_t ev[2]);
size_t wsl_scratch_bytes(unsigned max_blocks);
size_t pend_scratch_bytes(unsigned max_blocks);
hipError_t launch_histogram(const uint64_t *id_off, const int32_t *status, uint64_t n_str, int64_t *hist,
                            uint32_t n_bins, hipStream_t stream);
hipError_t kernel_init();
int small_window_bytes();
int big_window_bytes();

// host double-array trie over token bytes (dpt_vocab.cpp)
struct DoubleArray {
    // slot t: base[t] (| TERM bit 31 when a token ends here, | LEAF bit 30 when no child), check[t] = parent slot (-1 free)
    int32_t *base = nullptr;
    int32_t *check = nullptr;
    int32_t *id = nullptr;
    uint32_t n_slots = 0;
    uint32_t n_nodes = 0;
    uint32_t n_tokens = 0;
    uint32_t max_bytes = 0;
    uint32_t max_cp = 0;
    int32_t root_base = 0;
};

// returns 0 or an error message
const char *build_double_array(const uint8_t *blob, const uint64_t *off, const int32_t *ids, uint32_t n,
                               DoubleArray *out);
void free_double_array(DoubleArray *da);

}  // namespace dpt
