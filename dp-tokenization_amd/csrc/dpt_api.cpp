// dpt_api.cpp -- the C-ABI declared in include/dpt.h.
//
// Owns: the device copy of the vocabulary (dpt_vocab), per-stream workspaces
// (dpt_ctx), argument checking, the host-buffer convenience path and the
// event-based kernel timing used by bench.py.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <string>
#include <utility>
#include <unordered_map>
#include <vector>

#include "../../include/dpt.h"
#include "dpt_internal.h"

struct dpt_vocab {
    int device = 0;
    int2 *d_slots = nullptr;
    int32_t *d_ids = nullptr;
    int16_t *d_pair16 = nullptr;      // C2's pair-id table (dpt::PAIR16_N int16), then phase A0's byte-pair table (65536 uint2)
    int4 *d_slots4 = nullptr;         // {base | TERM, check, id, 0} for the lane kernel
    int32_t root_base = 0;
    int32_t ws_node = -1, ws_base = 0, ws_id = -1;   // the trie node after U+2581 (-1: no such path)
    bool ids16 = false;               // every id in 0..32767: ids are staged as int16 (half the staging traffic)
    uint32_t hash_buckets = 0, hash_probe = 0;   // C2's token hash table (0: none)
    dpt_vocab_stats stats{};
};

static uint64_t flag_words(uint64_t cap_batches) { return cap_batches * (2 * dpt::BS_LINE + 1); }

struct dpt_ctx {
    int device = 0;
    // workspace of the device path (ensure_workspace)
    int32_t *staging32 = nullptr;     // ids staged as int32 (vocabularies with an id outside 0..32767)
    uint64_t cap32 = 0;
    int16_t *staging16 = nullptr;     // ids staged as int16 (vocabularies with ids16)
    uint64_t cap16 = 0;
    uint8_t *arena = nullptr;         // the unbounded pass's scratch, 20 bytes per input byte it holds
    uint64_t arena_cap = 0;           // input bytes
    bool arena_reserved = false;      // dpt_ctx_reserve_vocab set it: the encode path does not resize it
    uint64_t *counts = nullptr;
    uint32_t *retry_list = nullptr;
    uint64_t cap_str = 0;
    uint32_t *retry_count = nullptr;  // counter block (dpt::CTR_ALLOC_BYTES): 8 uint32 counters, the uint64 arena
                                      // counter at byte 32, ..., the first pass's partition counters at byte 256
    uint8_t *wsl_scratch = nullptr;   // word lists of the 256-byte pass (dpt::wsl_scratch_bytes)
    uint4 *pend = nullptr;            // pending residual tokens of the 256-byte pass (dpt::pend_scratch_bytes)
    // two parity regions R0, R1 of batch lines (dpt::BS_LINE u64 per 256-string batch: its sum in the
    // first), then the batch prefixes of the scan path (cap_batches u64): the call of parity P uses R_P
    // and -- fold calls -- zeroes R_(1-P) for the next one (the parity flips); between calls R_parity
    // is all zero.  See dpt_internal.h fin_fold and BS_LINE.
    unsigned long long *flags = nullptr;
    uint64_t cap_batches = 0;
    int flag_parity = 0;
    unsigned max_blocks = 0;
    // host path: one device buffer in (text | offsets | cut) and one out (id_off | status | capped |
    // counters | ids | edges), each mirrored by a pinned host buffer so every copy is one async DMA
    uint8_t *d_in = nullptr, *p_in = nullptr, *d_out = nullptr, *p_out = nullptr;
    uint8_t *pd_in = nullptr, *pd_out = nullptr;   // p_in / p_out as the device addresses them (zero-copy calls)
    uint64_t cap_in = 0, cap_pin_in = 0, cap_out = 0, cap_pin_out = 0;
    // dpt_ctx_set_histogram: folded into the next encode's finish pass
    int64_t *hist = nullptr;
    uint32_t hist_bins = 0;
    bool hist_overwrite = false;
    // profiling
    bool profile = false;
    std::vector<hipEvent_t> events;   // groups of 4 per call
    uint64_t launches = 0;
    // test-only (dpt_ctx_debug_counter_bias): every call starts the unbounded pass's arena counter and the
    // far-pair counter at this value, the arena and far pointers passed down shifted by it
    uint64_t counter_bias = 0;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(DPT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Device buffer of at least `need` elements: exact on first allocation, +25 % when it grows.
template <typename T>
hipError_t grow(T **p, uint64_t *cap, uint64_t need) {
    if (need <= *cap && *p) return hipSuccess;
    uint64_t n = need < 64 ? 64 : need;
    if (*cap) n += n / 4;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e == hipSuccess) *cap = n;
    return e;
}

hipError_t grow_pinned(uint8_t **p, uint64_t *cap, uint64_t need) {
    if (need <= *cap && *p) return hipSuccess;
    uint64_t n = need < 4096 ? 4096 : need + (*cap ? need / 4 : 0);
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipHostMalloc((void **)p, n, hipHostMallocDefault);
    if (e == hipSuccess) *cap = n;
    return e;
}

// Input bytes the unbounded pass can hold per call when the caller does not say: every string for
// small batches, 1/32 of the batch for large ones (20 bytes of arena per held byte: 5/8 of the
// batch's size); the host path grows it on overflow, dpt_ctx_reserve_vocab sets it.
uint64_t default_long_bytes(uint64_t n_bytes) {
    const uint64_t floor = 4ull << 20;
    uint64_t lb = n_bytes / 32;
    if (lb < floor) lb = floor;
    return lb < n_bytes ? lb : n_bytes;
}

constexpr uint64_t ARENA_PER_BYTE = 20;   // uint4 rec + int32 stg (dpt_long.hip)
constexpr size_t COUNTER_BYTES = 64;

// v == nullptr: both staging widths (the vocabulary is not known yet); staging = false: no staging
// (dpt_encode_padded writes the ids into the caller's buffer)
int ensure_workspace(dpt_ctx *c, const dpt_vocab *v, uint64_t n_bytes, uint64_t n_str, uint64_t long_bytes,
                     bool staging = true) {
    hipError_t e;
    bool fresh = false;   // zeroed buffers were (re)allocated
    const bool need16 = staging && (!v || v->ids16), need32 = staging && (!v || !v->ids16);
    // (+8 elements: the finish pass reads staged ids as whole dwords, up to 2 elements past the last)
    if (need16 && (e = grow(&c->staging16, &c->cap16, n_bytes + 8)) != hipSuccess) return hip_fail(e, "hipMalloc(staging16)");
    if (need32 && (e = grow(&c->staging32, &c->cap32, n_bytes + 8)) != hipSuccess) return hip_fail(e, "hipMalloc(staging32)");
    // long_bytes = 0 (the encode path): the default size, unless the caller reserved the arena -- a
    // reserved arena is left alone, so a reserved call never reallocates (capture-safe, dpt.h)
    const uint64_t lb = long_bytes ? long_bytes : default_long_bytes(n_bytes);
    if (!c->arena || (lb > c->arena_cap && (long_bytes || !c->arena_reserved))) {
        uint64_t cap = c->arena_cap ? c->arena_cap * ARENA_PER_BYTE : 0;
        if ((e = grow(&c->arena, &cap, lb * ARENA_PER_BYTE)) != hipSuccess) return hip_fail(e, "hipMalloc(arena)");
        c->arena_cap = cap / ARENA_PER_BYTE;
    }
    if (n_str > c->cap_str || !c->counts) {
        uint64_t cap = c->cap_str, cap2 = 3 * c->cap_str;
        e = grow(&c->counts, &cap, n_str);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(counts)");
        // the first pass's retry list, the unbounded pass's list, the 2048-byte pass's list after the 512-byte pass
        e = grow(&c->retry_list, &cap2, 3 * n_str);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(retry_list)");
        cap2 /= 3;
        c->cap_str = cap < cap2 ? cap : cap2;
    }
    const uint64_t nbat = (n_str + dpt::FIN_BATCH - 1) / dpt::FIN_BATCH;
    if (nbat > c->cap_batches || !c->flags) {
        // (+25 % on growth; the regions start at zero and every call leaves the next one's zeroed)
        uint64_t capb = nbat > 1 ? nbat : 1;
        if (c->cap_batches) capb += capb / 4;
        if (c->flags) (void)hipFree(c->flags);
        c->flags = nullptr;
        c->cap_batches = 0;
        c->flag_parity = 0;
        if ((e = hipMalloc((void **)&c->flags, flag_words(capb) * sizeof(unsigned long long))) != hipSuccess) return hip_fail(e, "hipMalloc(flags)");
        if ((e = hipMemset(c->flags, 0, flag_words(capb) * sizeof(unsigned long long))) != hipSuccess) return hip_fail(e, "hipMemset(flags)");
        c->cap_batches = capb;
        fresh = true;
    }
    if (!c->wsl_scratch) {
        e = hipMalloc((void **)&c->wsl_scratch, dpt::wsl_scratch_bytes(c->max_blocks));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(wsl_scratch)");
    }
    if (!c->pend) {
        e = hipMalloc((void **)&c->pend, dpt::pend_scratch_bytes(c->max_blocks));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(pend)");
    }
    if (!c->retry_count) {
        // zeroed once here; every call's finish kernel resets it for the next call
        e = hipMalloc((void **)&c->retry_count, dpt::CTR_ALLOC_BYTES);
        if (e == hipSuccess) e = hipMemset(c->retry_count, 0, dpt::CTR_ALLOC_BYTES);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(retry_count)");
        fresh = true;
    }
    // the zero state every later call relies on must be in place before a call on any stream (a
    // non-blocking stream is not ordered after the null stream's memsets); allocations only
    if (fresh && (e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "hipDeviceSynchronize(zeroed workspace)");
    return DPT_OK;
}

// First-pass kernel: 16-lane rows (4 strings per wave) when every token has <= 16 code points,
// else 64-lane rows.  DPT_KERNEL=rows64 forces the 64-lane kernel (tests run it on the 32k vocab).
// C2's token hash table (dpt_internal.h TokHashHeader + buckets of two {fp, id}) over the tokens of at
// most TOKHASH_MAX_BYTES bytes, as uint32 words; {0, 0, 0, 0} (max_probe 0: no table) if no seed gives
// every token an unambiguous lookup.  For a token of the last vocabulary entry of equal bytes wins,
// like the trie (dpt_vocab.cpp).
std::vector<uint32_t> build_token_hash(const uint8_t *blob, const uint64_t *off, const int32_t *ids, uint32_t n) {
    struct Key { uint32_t w[dpt::TOKHASH_MAX_BYTES_LONG / 4]; uint32_t len; int32_t id; };
    std::vector<Key> keys;
    keys.reserve(n);
    // entries of equal bytes: one key, the last entry's id (dict semantics, as the trie: dpt_vocab.cpp) --
    // two keys of one byte string would share a fingerprint and no seed could build the table
    std::unordered_map<std::string, size_t> seen;
    seen.reserve(n);
    for (uint32_t t = 0; t < n; t++) {
        const uint64_t len = off[t + 1] - off[t];
        if (len == 0 || len > dpt::TOKHASH_MAX_BYTES_LONG) continue;
        const int32_t id = ids ? ids[t] : (int32_t)t;
        const auto ins = seen.emplace(std::string(reinterpret_cast<const char *>(blob + (off[t] - off[0])), (size_t)len), keys.size());
        if (!ins.second) {
            keys[ins.first->second].id = id;
            continue;
        }
        Key k;
        memset(k.w, 0, sizeof(k.w));
        k.len = (uint32_t)len;
        k.id = id;
        memcpy(k.w, blob + (off[t] - off[0]), len);   // little-endian dwords, zero past the token
        keys.push_back(k);
    }
    auto khash = [](const Key &k, uint32_t seed, uint32_t &h, uint32_t &fp) {
        const unsigned nd = k.len <= 16 ? 4u : (k.len + 3u) / 4u;
        dpt::TokHashState a = dpt::tokhash_start(k.len, seed);
        for (unsigned q = 0; q < nd; q++) a = dpt::tokhash_step(a, k.w[q], q);
        dpt::tokhash_end(a, h, fp);
    };
    std::vector<uint32_t> none(4, 0u);
    if (keys.empty()) return none;
    uint32_t nb = 1;
    while (nb < keys.size()) nb <<= 1;   // buckets of two entries: load <= 1/2
    const uint32_t mask = nb - 1;
    std::vector<uint32_t> H(keys.size()), F(keys.size());
    for (uint32_t seed = 0x2545F491u, tries = 0; tries < 8; tries++, seed = seed * 0x9E3779B9u + 0x7F4A7C15u) {
        for (size_t q = 0; q < keys.size(); q++) {
            khash(keys[q], seed, H[q], F[q]);
            H[q] &= mask;
        }
        std::vector<uint32_t> tab(4 + (size_t)nb * 4, 0u);
        uint32_t *bk = tab.data() + 4;
        std::vector<int32_t> who((size_t)nb * 2, -1);   // key per entry
        auto put = [&](uint32_t b, unsigned e, int32_t q) {
            bk[4 * (size_t)b + 2 * e] = F[q];
            bk[4 * (size_t)b + 2 * e + 1] = (uint32_t)keys[q].id;
            who[2 * (size_t)b + e] = q;
        };
        // cuckoo placement: a key takes a free entry of its two buckets, else evicts one (a pseudo-random
        // walk) and the evicted key moves to its other bucket
        bool bad = false;
        uint32_t rng = seed | 1u;
        for (size_t q0 = 0; q0 < keys.size() && !bad; q0++) {
            int32_t cur = (int32_t)q0;
            uint32_t b = H[q0];
            bool placed = false;
            for (int kick = 0; kick < 2000 && !placed; kick++) {
                const uint32_t b2 = dpt::tokhash_alt(b, F[cur], mask);
                const uint32_t cand[4][2] = {{b, 0}, {b, 1}, {b2, 0}, {b2, 1}};
                for (const auto &c : cand)
                    if (!placed && who[2 * (size_t)c[0] + c[1]] < 0) { put(c[0], c[1], cur); placed = true; }
                if (placed) break;
                rng = rng * 1664525u + 1013904223u;
                const uint32_t vb = (rng >> 16) & 1u ? b2 : b;
                const unsigned ve = (rng >> 17) & 1u;
                const int32_t victim = who[2 * (size_t)vb + ve];
                put(vb, ve, cur);
                cur = victim;
                b = dpt::tokhash_alt(vb, F[cur], mask);   // the victim's other bucket
            }
            bad = !placed;
        }
        if (bad) continue;
        // every key's lookup (the first entry of its fingerprint in bucket h, then in its partner) is its own
        for (size_t q = 0; q < keys.size() && !bad; q++) {
            const uint32_t b1 = H[q], b2 = dpt::tokhash_alt(b1, F[q], mask);
            const uint32_t cand[4][2] = {{b1, 0}, {b1, 1}, {b2, 0}, {b2, 1}};
            bool found = false;
            for (const auto &c : cand) {
                if (found || bk[4 * (size_t)c[0] + 2 * c[1]] != F[q]) continue;
                found = true;
                bad = who[2 * (size_t)c[0] + c[1]] != (int32_t)q;
            }
            bad = bad || !found;
        }
        if (bad) continue;
        tab[0] = mask;
        tab[1] = 2;   // a lookup visits two buckets
        tab[2] = seed;
        return tab;
    }
    return none;
}

int kernel_variant(uint32_t max_cp) {
    int v = max_cp <= 16 ? dpt::KERNEL_ROWS16 : dpt::KERNEL_ROWS64;
    if (const char *e = getenv("DPT_KERNEL"))
        if (!strcmp(e, "rows64")) v = dpt::KERNEL_ROWS64;
    return v;
}

}  // namespace

namespace dpt {
void set_last_error(const std::string &msg) { g_err = msg; }   // (dpt_rccl.cpp)
}

extern "C" {

const char *dpt_last_error(void) { return g_err.c_str(); }

int dpt_abi_version(void) { return DPT_ABI_VERSION; }

int dpt_vocab_create(const uint8_t *utf8_blob, const uint64_t *tok_off, const int32_t *ids, uint32_t n_tok,
                     int device, dpt_vocab **out) {
    if (!out || !tok_off || (!utf8_blob && n_tok && tok_off[n_tok] != tok_off[0])) return fail(DPT_E_ARG, "null argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(DPT_E_NODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(DPT_E_ARG, "bad device index");
    for (uint32_t t = 0; t < n_tok; t++)
        if (tok_off[t + 1] < tok_off[t]) return fail(DPT_E_ARG, "tok_off not monotone");
    dpt::DoubleArray da;
    const char *err = dpt::build_double_array(utf8_blob, tok_off, ids, n_tok, &da);
    if (err) return fail(DPT_E_VOCAB, err);
    DeviceGuard g(device);
    hipError_t e = dpt::kernel_init();
    if (e != hipSuccess) {
        dpt::free_double_array(&da);
        return hip_fail(e, "kernel_init");
    }
    dpt_vocab *v = new (std::nothrow) dpt_vocab();
    if (!v) {
        dpt::free_double_array(&da);
        return fail(DPT_E_ARG, "out of host memory");
    }
    v->device = device;
    // slots, then the two-byte root table: entry b0 << 8 | b1 describes the walk from the root over
    // bytes b0 b1 -- .x = base word of the node reached (0 if none), .y = that node's slot (0 if
    // none) | 1 << 30 if b0 is a root child | 1 << 31 if b0 alone is a token.  Phase A's first
    // lookup of every walk consumes two bytes through it.
    // slots4: {base, check, id, child filter} per slot, then the root table again as
    // {.x, .y, id of the node reached (-1 if none), child filter of the node reached} -- phase A of tokenize_kernel reads only these
    // (a filter bit per possible next byte, dpt::child_bit: a walk whose next byte has no bit ends
    // without the failing lookup), and its id serves C2's one-lookup tokens of two bytes
    std::vector<int2> slots((size_t)da.n_slots + 65536);
    std::vector<int4> slots4((size_t)da.n_slots + 65536);
    std::vector<uint32_t> filt(da.n_slots, 0u);
    // C2's one-lookup tokens (int16 vocabularies): pair16[b0 << 8 | b1] = id of the two-byte token
    // b0 b1, pair16[65536 + b0] = id of the one-byte token b0, -1 where none -- the ids the root table
    // and the root children give (slots4), in a 128-KB int16 table whose printable-ASCII part (24 KB
    // of lines) stays in a CU's L1 where the 16-B root-table entries (144 KB) do not
    std::vector<int16_t> pair16(65536 + 256, (int16_t)-1);
    // phase A0 (byte-parallel first lookups of pure-ASCII windows) needs only flags and the child
    // filter of the root-table entry: a0[b0 << 8 | b1] = {b0 is a root child | b0 is a token << 1 |
    // node b0 b1 exists << 2 | it ends a token << 3 | it is a leaf << 4, its child filter} -- 8 B
    // instead of the 16-B slots4 entry, so twice the entries per L1/L2 line
    std::vector<uint2> a0((size_t)65536, make_uint2(0u, 0u));
    for (uint32_t t = 0; t < da.n_slots; t++) {
        const int32_t p = da.check[t];
        if (p >= 0 && (uint32_t)p < da.n_slots) {
            const uint32_t b = t - (uint32_t)(da.base[p] & 0x3FFFFFFF);
            if (b < 256) filt[p] |= 1u << dpt::child_bit(b);
        }
    }
    for (uint32_t t = 0; t < da.n_slots; t++) {
        slots[t] = make_int2(da.base[t], da.check[t]);
        slots4[t] = make_int4(da.base[t], da.check[t], da.id[t], (int32_t)filt[t]);
    }
    for (uint32_t b0 = 0; b0 < 256; b0++) {
        const uint32_t s1 = (uint32_t)da.root_base + b0;
        const bool e1 = s1 < da.n_slots && da.check[s1] == 0;
        const bool term1 = e1 && (da.base[s1] & (int32_t)0x80000000);
        const bool leaf1 = e1 && (da.base[s1] & 0x40000000);
        const uint32_t base1 = e1 ? (uint32_t)(da.base[s1] & 0x3FFFFFFF) : 0u;
        for (uint32_t b1 = 0; b1 < 256; b1++) {
            const uint32_t s2 = base1 + b1;
            const bool e2 = e1 && !leaf1 && s2 < da.n_slots && da.check[s2] == (int32_t)s1;
            const uint32_t y = (e2 ? s2 : 0u) | (e1 ? 0x40000000u : 0u) | (term1 ? 0x80000000u : 0u);
            slots[(size_t)da.n_slots + (b0 << 8) + b1] = make_int2(e2 ? da.base[s2] : 0, (int32_t)y);
            slots4[(size_t)da.n_slots + (b0 << 8) + b1] = make_int4(e2 ? da.base[s2] : 0, (int32_t)y, e2 ? da.id[s2] : -1,
                                                                    e2 ? (int32_t)filt[s2] : 0);
            pair16[(b0 << 8) + b1] = (int16_t)(e2 ? da.id[s2] : -1);
            a0[(b0 << 8) + b1] = make_uint2((e1 ? 1u : 0u) | (term1 ? 2u : 0u) | (e2 ? 4u : 0u) |
                                                (e2 && (da.base[s2] & (int32_t)0x80000000) ? 8u : 0u) |
                                                (e2 && (da.base[s2] & 0x40000000) ? 16u : 0u),
                                            e2 ? filt[s2] : 0u);
        }
        pair16[65536 + b0] = (int16_t)(e1 ? da.id[s1] : -1);
        // a raw '\n' after b0 is "<0x0A>": A0 looks (b0, '\n') up as it reads and finds (b0, '<')'s entry
        a0[(b0 << 8) + '\n'] = a0[(b0 << 8) + '<'];
    }
    e = hipMalloc((void **)&v->d_slots, sizeof(int2) * slots.size());
    if (e == hipSuccess) e = hipMalloc((void **)&v->d_slots4, sizeof(int4) * slots4.size());
    if (e == hipSuccess) e = hipMemcpy(v->d_slots4, slots4.data(), sizeof(int4) * slots4.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void **)&v->d_ids, sizeof(int32_t) * da.n_slots);
    if (e == hipSuccess) e = hipMemcpy(v->d_slots, slots.data(), sizeof(int2) * slots.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->d_ids, da.id, sizeof(int32_t) * da.n_slots, hipMemcpyHostToDevice);
    // C2's token hash table (dpt_internal.h): header + buckets, after a0
    std::vector<uint32_t> th = build_token_hash(utf8_blob, tok_off, ids, n_tok);
    if (th[1]) {   // the header's last word: 1 + the id of "<0x0A>" (a '\n' atom's expansion; last duplicate wins), 0 = none
        for (uint32_t t = 0; t < n_tok; t++) {
            const uint64_t o = tok_off[t] - tok_off[0], len = tok_off[t + 1] - tok_off[t];
            const int32_t id = ids ? ids[t] : (int32_t)t;
            if (len == 6 && !memcmp(utf8_blob + o, "<0x0A>", 6)) th[3] = id >= 0 ? (uint32_t)id + 1u : 0u;
        }
    }
    // one allocation, one kernel pointer (SGPRs are what the hot kernel spills): pair16, then a0, then the hash
    if (e == hipSuccess) e = hipMalloc((void **)&v->d_pair16, dpt::TOKHASH_OFFSET + sizeof(uint32_t) * th.size());
    if (e == hipSuccess) e = hipMemcpy(v->d_pair16, pair16.data(), sizeof(int16_t) * pair16.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->d_pair16 + dpt::PAIR16_N, a0.data(), sizeof(uint2) * a0.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(reinterpret_cast<uint8_t *>(v->d_pair16) + dpt::TOKHASH_OFFSET, th.data(), sizeof(uint32_t) * th.size(), hipMemcpyHostToDevice);
    v->hash_buckets = th[1] ? th[0] + 1 : 0;
    v->hash_probe = th[1];
    if (e != hipSuccess) {
        dpt::free_double_array(&da);
        if (v->d_slots) (void)hipFree(v->d_slots);
        if (v->d_ids) (void)hipFree(v->d_ids);
        if (v->d_slots4) (void)hipFree(v->d_slots4);
        if (v->d_pair16) (void)hipFree(v->d_pair16);
        delete v;
        return hip_fail(e, "vocab upload");
    }
    v->root_base = da.root_base;
    {   // the node after '\u2581' (E2 96 81): the pending-token walks start word-start tokens there
        int32_t node = 0;
        for (uint32_t c : {0xE2u, 0x96u, 0x81u}) {
            const uint32_t t = (uint32_t)(da.base[node] & 0x3FFFFFFF) + c;
            if (node < 0 || t >= da.n_slots || da.check[t] != node) { node = -1; break; }
            node = (int32_t)t;
        }
        v->ws_node = node;
        v->ws_base = node >= 0 ? (da.base[node] & 0x3FFFFFFF) : 0;
        v->ws_id = node >= 0 ? da.id[node] : -1;
    }
    v->ids16 = true;
    for (uint32_t t = 0; t < da.n_slots; t++)
        if (da.check[t] >= 0 && (da.base[t] & (int32_t)0x80000000) && (da.id[t] < 0 || da.id[t] > 32767)) { v->ids16 = false; break; }
    v->stats.n_tokens = da.n_tokens;
    v->stats.n_nodes = da.n_nodes;
    v->stats.n_slots = da.n_slots;
    v->stats.max_bytes = da.max_bytes;
    v->stats.max_cp = da.max_cp;
    v->stats.hash_max_probe = v->hash_probe;
    v->stats.hash_buckets = v->hash_buckets;
    v->stats.device_bytes = (uint64_t)da.n_slots * (sizeof(int2) + sizeof(int32_t) + sizeof(int4)) + 65536 * (sizeof(int2) + sizeof(int4)) + (65536 + 256) * sizeof(int16_t) + 65536 * sizeof(uint2);
    dpt::free_double_array(&da);
    *out = v;
    return DPT_OK;
}

int dpt_vocab_destroy(dpt_vocab *v) {
    if (!v) return DPT_OK;
    DeviceGuard g(v->device);
    (void)hipFree(v->d_slots);
    (void)hipFree(v->d_ids);
    (void)hipFree(v->d_slots4);
    (void)hipFree(v->d_pair16);
    delete v;
    return DPT_OK;
}

int dpt_vocab_stats_get(const dpt_vocab *v, dpt_vocab_stats *out) {
    if (!v || !out) return fail(DPT_E_ARG, "null argument");
    *out = v->stats;
    return DPT_OK;
}

int dpt_ctx_create(int device, dpt_ctx **out) {
    if (!out) return fail(DPT_E_ARG, "null argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(DPT_E_NODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(DPT_E_ARG, "bad device index");
    dpt_ctx *c = new (std::nothrow) dpt_ctx();
    if (!c) return fail(DPT_E_ARG, "out of host memory");
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->max_blocks = (unsigned)prop.multiProcessorCount * 64u;
    if (c->max_blocks == 0) c->max_blocks = 256u * 64u;
    *out = c;
    return DPT_OK;
}

int dpt_ctx_destroy(dpt_ctx *c) {
    if (!c) return DPT_OK;
    DeviceGuard g(c->device);
    void *ps[] = {c->staging32, c->staging16, c->arena, c->counts, c->retry_list, c->retry_count, c->wsl_scratch,
                  c->pend, c->flags, c->d_in, c->d_out};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    if (c->p_in) (void)hipHostFree(c->p_in);
    if (c->p_out) (void)hipHostFree(c->p_out);
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    delete c;
    return DPT_OK;
}

int dpt_ctx_reserve(dpt_ctx *c, uint64_t n_bytes, uint64_t n_str) {
    return dpt_ctx_reserve_vocab(c, nullptr, n_bytes, n_str, 0);
}

int dpt_ctx_reserve_vocab(dpt_ctx *c, const dpt_vocab *v, uint64_t n_bytes, uint64_t n_str, uint64_t long_bytes) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    if (v && v->device != c->device) return fail(DPT_E_ARG, "ctx and vocab on different devices");
    DeviceGuard g(c->device);
    const int rc = ensure_workspace(c, v, n_bytes, n_str, long_bytes);
    if (rc == DPT_OK && long_bytes) c->arena_reserved = true;
    return rc;
}

int dpt_ctx_workspace_bytes(const dpt_ctx *c, uint64_t *device_path, uint64_t *host_path) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    if (device_path)
        *device_path = c->cap16 * 2 + c->cap32 * 4 + c->arena_cap * ARENA_PER_BYTE + c->cap_str * (8 + 3 * 4) +
                       flag_words(c->cap_batches) * 8 + (c->wsl_scratch ? dpt::wsl_scratch_bytes(c->max_blocks) : 0) +
                       (c->pend ? dpt::pend_scratch_bytes(c->max_blocks) : 0) +
                       (c->retry_count ? dpt::CTR_ALLOC_BYTES : 0);
    if (host_path) *host_path = c->cap_in + c->cap_out;
    return DPT_OK;
}

int dpt_ctx_long_need(dpt_ctx *c, uint64_t *need, uint64_t *cap) {
    if (!c || !need) return fail(DPT_E_ARG, "null argument");
    *need = 0;
    if (cap) *cap = c->arena_cap;
    if (!c->retry_count) return DPT_OK;
    DeviceGuard g(c->device);
    hipError_t e = hipMemcpy(need, reinterpret_cast<uint8_t *>(c->retry_count) + 40, sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "D2H arena counter");
    *need = *need >= c->counter_bias ? *need - c->counter_bias : 0;   // (0 after an empty call)
    return DPT_OK;
}

int dpt_ctx_debug_counter_bias(dpt_ctx *c, uint64_t bias) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    if (bias >= (1ull << 62)) return fail(DPT_E_ARG, "counter bias too large");
    c->counter_bias = bias;
    return DPT_OK;
}

// dev_call: dpt_encode itself (the call an armed histogram belongs to, dpt_ctx_set_histogram_ex); the
// host path and dpt_encode_padded leave it armed
static int encode_impl(dpt_ctx *c, const dpt_vocab *v, int mode_flags, const uint8_t *text, uint64_t n_bytes,
                       const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap,
                       uint64_t *id_off, int32_t *status, int32_t *capped_len, uint64_t *edges, void *hip_stream,
                       uint64_t *far = nullptr, uint64_t far_cap = 0, uint64_t *padded_counts = nullptr,
                       bool dev_call = false, uint64_t *ctr_snap = nullptr, bool no_fallback = false) {
    const int mode = mode_flags & DPT_MODE_MASK;
    if (!c || !v) return fail(DPT_E_ARG, "null ctx or vocab");
    // the armed histogram is this call's whatever happens below (one call only, failed ones included)
    int64_t *hist = dev_call ? c->hist : nullptr;
    const uint32_t hist_bins = c->hist_bins;
    const bool hist_overwrite = c->hist_overwrite;
    if (dev_call) {
        c->hist = nullptr;
        c->hist_overwrite = false;
    }
    if (mode != DPT_MODE_RAW && mode != DPT_MODE_PRESPLIT && mode != DPT_MODE_ATOMS) return fail(DPT_E_ARG, "bad mode");
    if (mode_flags & ~(DPT_MODE_MASK | DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY)) return fail(DPT_E_ARG, "bad flags");
    const bool padded = padded_counts != nullptr;
    if (!str_off || (!id_off && !padded) || (n_str && !status)) return fail(DPT_E_ARG, "null output/offsets");
    if (n_bytes && (!text || !ids)) return fail(DPT_E_ARG, "null text/ids");
    if (mode != DPT_MODE_RAW && n_bytes && !cut_mask) return fail(DPT_E_ARG, "PRESPLIT/ATOMS need cut_mask");
    if (ids_cap < n_bytes) return fail(DPT_E_CAP, "ids_cap must be >= n_bytes");
    if (n_str > 0x7FFFFFFFull) return fail(DPT_E_ARG, "too many strings for one call (max 2^31-1)");
    if (c->device != v->device) return fail(DPT_E_ARG, "ctx and vocab on different devices");
    DeviceGuard g(c->device);
    const int rc = ensure_workspace(c, v, n_bytes, n_str, 0, !padded);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)hip_stream;
    dpt::EncodeLaunch p;
    p.mode = mode_flags;
    p.edges = edges;
    p.far = edges ? far : nullptr;
    p.far_cap = far_cap;
    p.text = text;
    p.str_off = str_off;
    p.cut_mask = cut_mask;
    p.n_str = n_str;
    p.ids = ids;
    p.id_off = id_off;
    p.status = status;
    p.capped = capped_len;
    p.staging = c->staging32;
    p.counts = c->counts;
    p.retry_list = c->retry_list;
    p.retry_count = c->retry_count;
    p.wsl_scratch = c->wsl_scratch;
    p.long_span = v->stats.max_cp > 64 ? 1 : 0;
    p.max_tok_bytes = v->stats.max_bytes;
    {
        const uint64_t cb = c->cap_batches, rl = cb * dpt::BS_LINE;
        unsigned long long *r = c->flags + (c->flag_parity ? rl : 0);
        p.flags = r;
        p.zero_other = c->flags + (c->flag_parity ? 0 : rl);
        p.zero_n = cb;
        p.bpre = c->flags + 2 * rl;
    }
    p.max_blocks = c->max_blocks;
    p.arena = c->arena;
    p.arena_cap = c->arena_cap;
    p.counter_bias = c->counter_bias;
    if (c->counter_bias && n_str) {
        // test-only: the arena and far-pair counters start this call at the bias (the previous call's reset
        // left them 0), so the kernels' offsets have a low word >= 2^31 without a 40-GiB arena; the far
        // list is passed down shifted by as many pairs
        const uint64_t b = c->counter_bias;
        uint32_t *ctr = c->retry_count;
        for (unsigned w : {8u, 12u}) {   // (uint64 counters 4 and 6: the arena's claimed bytes, the far pairs)
            hipError_t e0 = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ctr + w), (int)(uint32_t)b, 1, st);
            if (e0 == hipSuccess) e0 = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ctr + w + 1), (int)(uint32_t)(b >> 32), 1, st);
            if (e0 != hipSuccess) return hip_fail(e0, "counter bias");
        }
        if (p.far) {
            p.far = reinterpret_cast<uint64_t *>(reinterpret_cast<uintptr_t>(p.far) - 16 * b);
            p.far_cap = far_cap + b;
        }
    }
    p.variant = kernel_variant(v->stats.max_cp);
    // int16 staging when every id fits in 0..32767 (half the staging traffic)
    p.staging16 = v->ids16 ? c->staging16 : nullptr;
    p.padded = padded;
    p.pend = c->pend;
    p.hist = hist;
    p.hist_bins = hist_bins;
    p.hist_overwrite = hist_overwrite;
    p.ctr_snap = ctr_snap;
    p.no_fallback = no_fallback;
    p.n_bytes = n_bytes;
    // (a per-string dp_tokenize call: one launch instead of two -- the finish kernel was 5 us of its 43)
    p.solo = !getenv("DPT_NO_SOLO") && no_fallback && n_str == 1 && !padded && !edges && !hist && !c->profile && ctr_snap;
    if (padded) {   // the ids go straight to their final place (int32), the counts to the caller's array
        p.staging = ids;
        p.staging16 = nullptr;
        p.counts = padded_counts;
    }
    p.slots = v->d_slots;
    p.slot_ids = v->d_ids;
    p.pair16 = v->d_pair16;
    p.n_slots = v->stats.n_slots;
    p.slots4 = v->d_slots4;
    p.root_base = v->root_base;
    p.ws_node = v->ws_node; p.ws_base = v->ws_base; p.ws_id = v->ws_id;
    hipEvent_t ev[2];
    hipEvent_t *evp = nullptr;
    if (c->profile) {
        for (int k = 0; k < 2; k++) {
            hipError_t e = hipEventCreate(&ev[k]);
            if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
            c->events.push_back(ev[k]);
        }
        evp = ev;
        c->launches++;
    }
    hipError_t e = dpt::launch_encode(p, st, evp);
    if (e != hipSuccess) {
        (void)hipMemsetAsync(c->retry_count, 0, dpt::CTR_ALLOC_BYTES, st);   // the scan kernel did not reset them
        (void)hipMemsetAsync(c->flags, 0, flag_words(c->cap_batches) * sizeof(unsigned long long), st);   // nor zero the batch lines
        c->flag_parity = 0;
        return hip_fail(e, "encode launch");
    }
    if (!padded && dpt::fin_fold(n_str)) c->flag_parity ^= 1;   // the finish pass zeroed the other region
    return DPT_OK;
}

int dpt_encode(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
               const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap,
               uint64_t *id_off, int32_t *status, int32_t *capped_len, void *hip_stream) {
    if (mode & ~DPT_MODE_MASK) return fail(DPT_E_ARG, "flags are for dpt_dp_host");
    return encode_impl(c, v, mode, text, n_bytes, str_off, cut_mask, n_str, ids, ids_cap, id_off, status, capped_len,
                       nullptr, hip_stream, nullptr, 0, nullptr, true);
}

int dpt_encode_padded(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
                      const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap,
                      uint64_t *counts, int32_t *status, int32_t *capped_len, void *hip_stream) {
    if (mode & ~DPT_MODE_MASK) return fail(DPT_E_ARG, "flags are for dpt_dp_host");
    if (!counts) return fail(DPT_E_ARG, "null counts");
    return encode_impl(c, v, mode, text, n_bytes, str_off, cut_mask, n_str, ids, ids_cap, nullptr, status, capped_len,
                       nullptr, hip_stream, nullptr, 0, counts);
}

static int rerun_too_long(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, const uint64_t *str_off,
                          const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap, uint64_t *id_off,
                          int32_t *status, int32_t *capped_len);

// Host path calls up to this many input bytes check whether any string needs the fallback passes.
constexpr uint64_t NO_FALLBACK_CHECK_BYTES = 16384;

// True when no string of a RAW / PRESPLIT call can leave the first pass (dpt_kernels.hip tokenize_kernel):
// every word fits one 256-byte window (consecutive word starts -- byte 0, then ' ' in RAW mode or a cut
// byte on a non-continuation byte in PRESPLIT mode -- at most 256 bytes apart, the last one at most 256
// bytes before the string's end) and every atom (a code point: a byte and its continuation bytes) has at
// most 4 bytes.  (Vocabularies with tokens of more than 64 code points are not checked: the caller.)
static bool no_fallback_needed(int mode, const uint8_t *text, const uint64_t *str_off, const uint8_t *cut,
                               uint64_t n_str) {
    if (mode != DPT_MODE_RAW && mode != DPT_MODE_PRESPLIT) return false;
    const uint64_t base = str_off[0];
    for (uint64_t i = 0; i < n_str; i++) {
        const uint64_t a = str_off[i] - base, b = str_off[i + 1] - base;
        uint64_t ws = a;        // the current word's start
        unsigned cont = 0;      // continuation bytes after the current atom's first byte
        for (uint64_t k = a; k < b; k++) {
            const uint8_t x = text[k];
            const bool is_cont = k > a && (x & 0xC0) == 0x80;   // (the string's first byte starts an atom)
            cont = is_cont ? cont + 1 : 0;
            if (cont > 3) return false;   // an atom of over 4 bytes
            const bool wstart = k > a && (mode == DPT_MODE_RAW ? x == ' ' : (cut[k] != 0 && !is_cont));
            if (wstart) {
                if (k - ws > 256) return false;
                ws = k;
            }
        }
        if (b - ws > 256) return false;
    }
    return true;
}

static int encode_host_impl(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
                            const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids,
                            uint64_t ids_cap, uint64_t *id_off, int32_t *status, int32_t *capped_len,
                            uint64_t *edges, uint64_t *far = nullptr, uint64_t far_cap = 0, uint64_t *n_far = nullptr,
                            int depth = 0) {
    // host arguments first (checkable without a device)
    if (!str_off || !id_off || (n_str && !status)) return fail(DPT_E_ARG, "null output/offsets");
    if (n_bytes && (!text || !ids)) return fail(DPT_E_ARG, "null text/ids");
    if (ids_cap < n_bytes) return fail(DPT_E_CAP, "ids_cap must be >= n_bytes");
    if (str_off[n_str] - str_off[0] != n_bytes) return fail(DPT_E_ARG, "n_bytes != str_off[n_str]-str_off[0]");
    // the kernels take string lengths as 32-bit values (dpt.h): offsets must be monotone and every
    // string shorter than 4 GiB, or a wrapped length would read past the text
    for (uint64_t i = 0; i < n_str; i++) {
        if (str_off[i + 1] < str_off[i]) return fail(DPT_E_ARG, "str_off not monotone");
        if (str_off[i + 1] - str_off[i] >= (1ull << 32)) return fail(DPT_E_ARG, "a string of 4 GiB or more");
    }
    if (!c || !v) return fail(DPT_E_ARG, "null ctx or vocab");
    DeviceGuard g(c->device);
    hipError_t e;
    const bool cut = (mode & DPT_MODE_MASK) != DPT_MODE_RAW && n_bytes;
    if (cut && !cut_mask) return fail(DPT_E_ARG, "PRESPLIT/ATOMS need cut_mask");
    auto al8 = [](uint64_t x) { return (x + 7) & ~7ull; };
    // in:  text | offsets rebased to 0 (the device view is self-contained) | cut mask
    const uint64_t o_off = al8(n_bytes + 1), o_cut = o_off + 8 * (n_str + 1), in_bytes = o_cut + al8(n_bytes + 1);
    // out: id_off | status | capped | counters | ids | edges | far edge pairs
    const uint64_t o_st = 8 * (n_str + 1), o_cap = o_st + al8(4 * n_str + 4), o_ctr = o_cap + al8(4 * n_str + 4);
    const uint64_t o_ids = o_ctr + COUNTER_BYTES, o_edges = o_ids + al8(4 * (n_bytes + 1));
    const uint64_t o_far = o_edges + (edges ? 8 * (n_bytes + 1) : 0);
    const bool want_far = edges && far;
    const uint64_t out_bytes = o_far + (want_far ? 16 * far_cap : 0);
    if ((e = grow(&c->d_in, &c->cap_in, in_bytes)) != hipSuccess) return hip_fail(e, "hipMalloc(host-path in)");
    if ((e = grow(&c->d_out, &c->cap_out, out_bytes)) != hipSuccess) return hip_fail(e, "hipMalloc(host-path out)");
    {
        uint8_t *pi = c->p_in, *po = c->p_out;
        if ((e = grow_pinned(&c->p_in, &c->cap_pin_in, in_bytes)) != hipSuccess) return hip_fail(e, "hipHostMalloc(in)");
        if ((e = grow_pinned(&c->p_out, &c->cap_pin_out, out_bytes)) != hipSuccess) return hip_fail(e, "hipHostMalloc(out)");
        if (pi != c->p_in || !c->pd_in) {
            if ((e = hipHostGetDevicePointer((void **)&c->pd_in, c->p_in, 0)) != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
        }
        if (po != c->p_out || !c->pd_out) {
            if ((e = hipHostGetDevicePointer((void **)&c->pd_out, c->p_out, 0)) != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
        }
    }
    if (n_bytes) memcpy(c->p_in, text, n_bytes);
    uint64_t *off = reinterpret_cast<uint64_t *>(c->p_in + o_off);
    for (uint64_t i = 0; i <= n_str; i++) off[i] = str_off[i] - str_off[0];
    if (cut) memcpy(c->p_in + o_cut, cut_mask, n_bytes);
    hipStream_t st = 0;
    uint64_t *d_idoff = reinterpret_cast<uint64_t *>(c->d_out);
    int32_t *d_status = reinterpret_cast<int32_t *>(c->d_out + o_st);
    int32_t *d_capped = reinterpret_cast<int32_t *>(c->d_out + o_cap);
    int32_t *d_ids = reinterpret_cast<int32_t *>(c->d_out + o_ids);
    uint64_t *d_edges = edges ? reinterpret_cast<uint64_t *>(c->d_out + o_edges) : nullptr;
    uint64_t *d_far = want_far ? reinterpret_cast<uint64_t *>(c->d_out + o_far) : nullptr;
    const uint64_t *p_idoff = reinterpret_cast<const uint64_t *>(c->p_out);
    // small batches: everything in one copy (ids up to the n_bytes bound); large: the head, then the ids.
    // The counter block's first 64 bytes ride in d_out's counter slot (the finish pass's reset copies
    // them there), so one copy brings them back.
    const bool one_copy = 4 * n_bytes <= (4ull << 20);
    // Small calls skip the 2048-byte and unbounded passes' dispatches when no string can need them
    // (no_fallback_needed): a per-string dp_tokenize call's launch chain loses two of its four kernels.
    const bool no_fb = n_bytes <= NO_FALLBACK_CHECK_BYTES && !edges && v->stats.max_cp <= 64 &&
                       no_fallback_needed(mode & DPT_MODE_MASK, text, str_off, cut ? cut_mask : nullptr, n_str);
    bool overflow = false;   // some strings got status 3 (arena full): they alone run again below
    // One string with no fallback pass (a per-string dp_tokenize call): zero-copy -- its lone wave
    // (EncodeLaunch::solo) reads the text from and writes the outputs to the pinned host buffers, so the
    // call is one launch and a sync (two copies and their gaps less)
    if (no_fb && n_str == 1 && !edges && !c->profile && !getenv("DPT_NO_SOLO")) {
        int rc = encode_impl(c, v, mode, c->pd_in, n_bytes, reinterpret_cast<const uint64_t *>(c->pd_in + o_off),
                             cut ? c->pd_in + o_cut : nullptr, n_str, reinterpret_cast<int32_t *>(c->pd_out + o_ids),
                             n_bytes ? n_bytes : 1, reinterpret_cast<uint64_t *>(c->pd_out),
                             reinterpret_cast<int32_t *>(c->pd_out + o_st), reinterpret_cast<int32_t *>(c->pd_out + o_cap),
                             nullptr, st, nullptr, 0, nullptr, false, reinterpret_cast<uint64_t *>(c->pd_out + o_ctr), true);
        if (rc) return rc;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "sync");
        const uint64_t total = p_idoff[1];
        if (total > ids_cap || total > n_bytes) return fail(DPT_E_CAP, "ids overflow");
        id_off[0] = 0;
        id_off[1] = total;
        status[0] = *reinterpret_cast<const int32_t *>(c->p_out + o_st);
        if (capped_len) capped_len[0] = *reinterpret_cast<const int32_t *>(c->p_out + o_cap);
        if (total) memcpy(ids, c->p_out + o_ids, 4 * total);
        return DPT_OK;
    }
    if ((e = hipMemcpyAsync(c->d_in, c->p_in, in_bytes, hipMemcpyHostToDevice, st)) != hipSuccess) return hip_fail(e, "H2D");
    for (int attempt = 0;; attempt++) {
        int rc = encode_impl(c, v, mode, c->d_in, n_bytes, reinterpret_cast<const uint64_t *>(c->d_in + o_off),
                             cut ? c->d_in + o_cut : nullptr, n_str, d_ids, n_bytes ? n_bytes : 1, d_idoff, d_status,
                             d_capped, d_edges, st, d_far, far_cap, nullptr, false,
                             reinterpret_cast<uint64_t *>(c->d_out + o_ctr), no_fb);
        if (rc) return rc;
        if ((e = hipMemcpyAsync(c->p_out, c->d_out, one_copy ? out_bytes : o_ctr + COUNTER_BYTES, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(e, "D2H");
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "sync");
        uint64_t used = 0;
        if (n_str) memcpy(&used, c->p_out + o_ctr + 40, sizeof(used));   // the call's claimed bytes (finish_kernel)
        if (n_str) used -= c->counter_bias;   // (test-only dpt_ctx_debug_counter_bias)
        if (used > n_bytes) return fail(DPT_E_HIP, "unbounded pass counter out of range");   // never expected
        if (used <= c->arena_cap) break;
        // the unbounded pass's arena was too small for the strings routed to it (those strings got
        // status 3): grow it to what the pass claimed and run the call again
        if (attempt > 0 || depth > 0) return fail(DPT_E_ARG, "unbounded pass arena overflow after growth");
        if ((rc = ensure_workspace(c, v, n_bytes, n_str, used))) return rc;
        // without edge outputs only the strings the arena could not hold run again (a sub-batch,
        // spliced in below); edge-recording calls (one string each from the drop-ins) rerun whole
        if (!edges) {
            overflow = true;
            break;
        }
    }
    const uint64_t total = p_idoff[n_str];
    if (total > ids_cap) return fail(DPT_E_CAP, "ids overflow");
    uint64_t nf = 0;
    if (want_far) {
        if (n_str) memcpy(&nf, c->p_out + o_ctr + 56, sizeof(nf));   // the call's far edge pairs (finish_kernel)
        if (n_str) nf -= c->counter_bias;
        if (n_far) *n_far = nf;
        if (nf > far_cap) return fail(DPT_E_CAP, "far edge list overflow (*n_far holds the pairs needed)");
    }
    if (!one_copy) {
        if (total && (e = hipMemcpyAsync(c->p_out + o_ids, d_ids, 4 * total, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(e, "D2H ids");
        if (edges && n_bytes &&
            (e = hipMemcpyAsync(c->p_out + o_edges, d_edges, 8 * n_bytes, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(e, "D2H edges");
        if (nf && (e = hipMemcpyAsync(c->p_out + o_far, d_far, 16 * nf, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(e, "D2H far edges");
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "sync");
    }
    memcpy(id_off, c->p_out, 8 * (n_str + 1));
    if (n_str) memcpy(status, c->p_out + o_st, 4 * n_str);
    if (capped_len && n_str) memcpy(capped_len, c->p_out + o_cap, 4 * n_str);
    if (total) memcpy(ids, c->p_out + o_ids, 4 * total);
    if (edges && n_bytes) memcpy(edges, c->p_out + o_edges, 8 * n_bytes);
    if (nf) memcpy(far, c->p_out + o_far, 16 * nf);
    if (overflow) return rerun_too_long(c, v, mode, text, str_off, cut_mask, n_str, ids, ids_cap, id_off, status, capped_len);
    return DPT_OK;
}

// After an arena overflow (the arena has since grown to what the pass claimed): the strings with
// status DPT_STATUS_TOO_LONG -- exactly those the unbounded pass could not hold -- as one sub-batch,
// their results spliced into the caller's CSR arrays.
static int rerun_too_long(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, const uint64_t *str_off,
                          const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap, uint64_t *id_off,
                          int32_t *status, int32_t *capped_len) {
    std::vector<uint64_t> sel;
    for (uint64_t i = 0; i < n_str; i++)
        if (status[i] == DPT_STATUS_TOO_LONG) sel.push_back(i);
    if (sel.empty()) return DPT_OK;
    const uint64_t k = sel.size();
    std::vector<uint64_t> soff(k + 1, 0);
    for (uint64_t q = 0; q < k; q++) soff[q + 1] = soff[q] + (str_off[sel[q] + 1] - str_off[sel[q]]);
    const uint64_t sb = soff[k];
    const bool cut = (mode & DPT_MODE_MASK) != DPT_MODE_RAW;
    std::vector<uint8_t> stext(sb ? sb : 1), scut(cut && sb ? sb : 1);
    for (uint64_t q = 0; q < k; q++) {
        const uint64_t a = str_off[sel[q]] - str_off[0], n = soff[q + 1] - soff[q];
        if (n) memcpy(stext.data() + soff[q], text + a, n);
        if (cut && n) memcpy(scut.data() + soff[q], cut_mask + a, n);
    }
    std::vector<int32_t> sids(sb ? sb : 1), sst(k), scap(k);
    std::vector<uint64_t> sidoff(k + 1);
    int rc = encode_host_impl(c, v, mode, stext.data(), sb, soff.data(), cut ? scut.data() : nullptr, k, sids.data(),
                              sb ? sb : 1, sidoff.data(), sst.data(), capped_len ? scap.data() : nullptr, nullptr,
                              nullptr, 0, nullptr, 1);
    if (rc) return rc;
    // splice: the overflowed strings had no ids; rebuild the CSR arrays around their new ones
    const uint64_t total = id_off[n_str] + sidoff[k];
    if (total > ids_cap) return fail(DPT_E_CAP, "ids overflow");
    std::vector<int32_t> old(ids, ids + id_off[n_str]);
    std::vector<uint64_t> old_off(id_off, id_off + n_str + 1);
    uint64_t o = 0, q = 0;
    for (uint64_t i = 0; i < n_str; i++) {
        id_off[i] = o;
        if (q < k && sel[q] == i) {
            const uint64_t n = sidoff[q + 1] - sidoff[q];
            if (n) memcpy(ids + o, sids.data() + sidoff[q], 4 * n);
            o += n;
            status[i] = sst[q];
            if (capped_len) capped_len[i] = scap[q];
            q++;
        } else {
            const uint64_t n = old_off[i + 1] - old_off[i];
            if (n) memcpy(ids + o, old.data() + old_off[i], 4 * n);
            o += n;
        }
    }
    id_off[n_str] = o;
    return DPT_OK;
}

int dpt_encode_host(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
                    const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap,
                    uint64_t *id_off, int32_t *status, int32_t *capped_len) {
    if (mode & ~DPT_MODE_MASK) return fail(DPT_E_ARG, "flags are for dpt_dp_host");
    return encode_host_impl(c, v, mode, text, n_bytes, str_off, cut_mask, n_str, ids, ids_cap, id_off, status,
                            capped_len, nullptr);
}

int dpt_dp_host(dpt_ctx *c, const dpt_vocab *v, int mode_flags, const uint8_t *text, uint64_t n_bytes,
                const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *status, int32_t *lengths,
                uint64_t *edges) {
    if (!lengths && !edges) return fail(DPT_E_ARG, "nothing to compute");
    if (!(mode_flags & (DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY))) mode_flags |= DPT_FLAG_LEN_ONLY;
    std::vector<uint64_t> id_off(n_str + 1);
    std::vector<int32_t> len_tmp(lengths ? 0 : n_str + 1);
    int32_t dummy_ids[1];
    return encode_host_impl(c, v, mode_flags, text, n_bytes, str_off, cut_mask, n_str, dummy_ids, n_bytes ? n_bytes : 1,
                            id_off.data(), status, lengths ? lengths : len_tmp.data(), edges);
}

int dpt_dp_host_far(dpt_ctx *c, const dpt_vocab *v, int mode_flags, const uint8_t *text, uint64_t n_bytes,
                    const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *status, int32_t *lengths,
                    uint64_t *edges, uint64_t *far, uint64_t far_cap, uint64_t *n_far) {
    if (!edges || !n_far || (far_cap && !far)) return fail(DPT_E_ARG, "dpt_dp_host_far needs edges, far and n_far");
    *n_far = 0;
    if (!(mode_flags & (DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY))) mode_flags |= DPT_FLAG_LEN_ONLY;
    std::vector<uint64_t> id_off(n_str + 1);
    std::vector<int32_t> len_tmp(lengths ? 0 : n_str + 1);
    int32_t dummy_ids[1];
    uint64_t dummy_far[2];
    return encode_host_impl(c, v, mode_flags, text, n_bytes, str_off, cut_mask, n_str, dummy_ids, n_bytes ? n_bytes : 1,
                            id_off.data(), status, lengths ? lengths : len_tmp.data(), edges, far ? far : dummy_far,
                            far_cap, n_far);
}

int dpt_token_histogram(const uint64_t *id_off, const int32_t *status, uint64_t n_str, int64_t *hist, uint32_t n_bins,
                        void *hip_stream) {
    if (!id_off || !hist || (n_str && !status) || n_bins < 2 || n_bins > DPT_HIST_MAX_BINS)
        return fail(DPT_E_ARG, "bad histogram arguments (2 <= n_bins <= DPT_HIST_MAX_BINS)");
    hipError_t e = dpt::launch_histogram(id_off, status, n_str, hist, n_bins, (hipStream_t)hip_stream);
    if (e != hipSuccess) return hip_fail(e, "histogram launch");
    return DPT_OK;
}

int dpt_ctx_set_histogram_ex(dpt_ctx *c, int64_t *hist, uint32_t n_bins, int flags) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    if (hist && (n_bins < 2 || n_bins > DPT_HIST_MAX_BINS)) return fail(DPT_E_ARG, "n_bins outside 2..DPT_HIST_MAX_BINS");
    if (flags & ~DPT_HIST_OVERWRITE) return fail(DPT_E_ARG, "unknown histogram flags");
    c->hist = hist;
    c->hist_bins = hist ? n_bins : 0;
    c->hist_overwrite = hist && (flags & DPT_HIST_OVERWRITE);
    return DPT_OK;
}

int dpt_ctx_set_histogram(dpt_ctx *c, int64_t *hist, uint32_t n_bins) { return dpt_ctx_set_histogram_ex(c, hist, n_bins, 0); }

int dpt_ctx_profile(dpt_ctx *c, int enable) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    c->profile = enable != 0;
    return DPT_OK;
}

int dpt_ctx_profile_read(dpt_ctx *c, double *ms, uint64_t *launches) {
    if (!c || !ms) return fail(DPT_E_ARG, "null argument");
    DeviceGuard g(c->device);
    ms[0] = 0.0;
    ms[1] = ms[2] = -1.0;   // not timed: one event pair per call (every event record costs the stream ~6 us)
    for (size_t k = 0; k + 1 < c->events.size(); k += 2) {
        hipError_t e = hipEventSynchronize(c->events[k + 1]);
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        float t = 0.f;
        e = hipEventElapsedTime(&t, c->events[k], c->events[k + 1]);
        if (e != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
        ms[0] += t;
    }
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    c->events.clear();
    if (launches) *launches = c->launches;
    c->launches = 0;
    return DPT_OK;
}

}  // extern "C"
