// dpt_api.cpp -- the C-ABI declared in include/dpt.h.
//
// Owns: the device copy of the vocabulary (dpt_vocab), per-stream workspaces
// (dpt_ctx), argument checking, the host-buffer convenience path and the
// event-based kernel timing used by bench.py.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/dpt.h"
#include "dpt_internal.h"

struct dpt_vocab {
    int device = 0;
    int2 *d_slots = nullptr;
    int32_t *d_ids = nullptr;
    int4 *d_slots4 = nullptr;         // {base | TERM, check, id, 0} for the lane kernel
    int32_t root_base = 0;
    bool ids16 = false;               // every id in 0..32767: ids are staged as int16 (half the staging traffic)
    dpt_vocab_stats stats{};
};

struct dpt_ctx {
    int device = 0;
    // workspace
    int32_t *staging = nullptr;
    int16_t *staging16 = nullptr;     // int16 staging for vocabularies with ids16
    uint4 *rec = nullptr;             // lane kernel backtrace records (cap_bytes entries)
    uint64_t cap_bytes = 0;
    uint64_t *counts = nullptr;
    uint32_t *retry_list = nullptr;
    uint64_t cap_str = 0;
    uint32_t *retry_count = nullptr;
    uint8_t *wsl_scratch = nullptr;   // word lists of the 256-byte pass (dpt::wsl_scratch_bytes)
    void *scan_temp = nullptr;
    size_t scan_bytes = 0;
    unsigned max_blocks = 0;
    // host-path device buffers
    uint8_t *h_text = nullptr;
    uint64_t h_cap_bytes = 0;
    uint8_t *h_cut = nullptr;
    int32_t *h_ids = nullptr;
    uint64_t *h_off = nullptr, *h_idoff = nullptr;
    int32_t *h_status = nullptr, *h_capped = nullptr;
    uint64_t h_cap_str = 0;
    uint64_t *h_edges = nullptr;
    uint64_t h_cap_edges = 0;
    // profiling
    bool profile = false;
    std::vector<hipEvent_t> events;   // groups of 4 per call
    uint64_t launches = 0;
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

template <typename T>
hipError_t grow(T **p, uint64_t *cap, uint64_t need) {
    if (need <= *cap && *p) return hipSuccess;
    uint64_t n = need < 1024 ? 1024 : need + need / 4;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e == hipSuccess) *cap = n;
    return e;
}

int ensure_workspace(dpt_ctx *c, uint64_t n_bytes, uint64_t n_str) {
    hipError_t e;
    if (n_bytes > c->cap_bytes || !c->staging) {
        uint64_t cap1 = c->cap_bytes, cap2 = c->cap_bytes;
        e = grow(&c->staging, &cap1, n_bytes);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(staging)");
        e = grow(&c->rec, &cap2, n_bytes);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(rec)");
        uint64_t cap3 = c->cap_bytes;
        e = grow(&c->staging16, &cap3, n_bytes);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(staging16)");
        c->cap_bytes = cap1 < cap2 ? cap1 : cap2;
        c->cap_bytes = c->cap_bytes < cap3 ? c->cap_bytes : cap3;
    }
    if (n_str > c->cap_str || !c->counts) {
        uint64_t cap = c->cap_str, cap2 = c->cap_str;
        e = grow(&c->counts, &cap, n_str);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(counts)");
        e = grow(&c->retry_list, &cap2, 2 * n_str);   // the 2048-byte pass's list, then the unbounded pass's
        cap2 /= 2;
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(retry_list)");
        c->cap_str = cap < cap2 ? cap : cap2;
        size_t tb = dpt::scan_temp_bytes(c->cap_str);
        if (tb > c->scan_bytes) {
            if (c->scan_temp) (void)hipFree(c->scan_temp);
            c->scan_temp = nullptr;
            e = hipMalloc(&c->scan_temp, tb);
            if (e != hipSuccess) return hip_fail(e, "hipMalloc(scan)");
            c->scan_bytes = tb;
        }
    }
    if (!c->wsl_scratch) {
        e = hipMalloc((void **)&c->wsl_scratch, dpt::wsl_scratch_bytes(c->max_blocks));
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(wsl_scratch)");
    }
    if (!c->retry_count) {
        e = hipMalloc((void **)&c->retry_count, 32);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(retry_count)");
    }
    return DPT_OK;
}

// First-pass kernel: 16-lane rows (4 strings per wave) when every token has <= 16 code
// points, else 64-lane rows.  DPT_KERNEL=lane|rows16|rows64 overrides (A/B measurements; the
// lane kernel measured slower on cfg2: 2x the VALU count and ~30 GB of scratch traffic per
// 1M strings, profiles/r01_pmc_*).
int kernel_variant(uint32_t max_cp) {
    int v = max_cp <= 16 ? dpt::KERNEL_ROWS16 : dpt::KERNEL_ROWS64;
    if (const char *e = getenv("DPT_KERNEL")) {
        if (!strcmp(e, "rows16")) v = dpt::KERNEL_ROWS16;
        else if (!strcmp(e, "rows64")) v = dpt::KERNEL_ROWS64;
        else if (!strcmp(e, "lane")) v = dpt::KERNEL_LANE;
    }
    if (max_cp > 16) v = dpt::KERNEL_ROWS64;
    return v;
}

}  // namespace

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
    // {.x, .y, 0, child filter of the node reached} -- phase A of tokenize_kernel reads only these
    // (a filter bit per possible next byte, dpt::child_bit: a walk whose next byte has no bit ends
    // without the failing lookup)
    std::vector<int2> slots((size_t)da.n_slots + 65536);
    std::vector<int4> slots4((size_t)da.n_slots + 65536);
    std::vector<uint32_t> filt(da.n_slots, 0u);
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
            slots4[(size_t)da.n_slots + (b0 << 8) + b1] = make_int4(e2 ? da.base[s2] : 0, (int32_t)y, 0, e2 ? (int32_t)filt[s2] : 0);
        }
    }
    e = hipMalloc((void **)&v->d_slots, sizeof(int2) * slots.size());
    if (e == hipSuccess) e = hipMalloc((void **)&v->d_slots4, sizeof(int4) * slots4.size());
    if (e == hipSuccess) e = hipMemcpy(v->d_slots4, slots4.data(), sizeof(int4) * slots4.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void **)&v->d_ids, sizeof(int32_t) * da.n_slots);
    if (e == hipSuccess) e = hipMemcpy(v->d_slots, slots.data(), sizeof(int2) * slots.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->d_ids, da.id, sizeof(int32_t) * da.n_slots, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        dpt::free_double_array(&da);
        if (v->d_slots) (void)hipFree(v->d_slots);
        if (v->d_ids) (void)hipFree(v->d_ids);
        if (v->d_slots4) (void)hipFree(v->d_slots4);
        delete v;
        return hip_fail(e, "vocab upload");
    }
    v->root_base = da.root_base;
    v->ids16 = true;
    for (uint32_t t = 0; t < da.n_slots; t++)
        if (da.check[t] >= 0 && (da.base[t] & (int32_t)0x80000000) && (da.id[t] < 0 || da.id[t] > 32767)) { v->ids16 = false; break; }
    v->stats.n_tokens = da.n_tokens;
    v->stats.n_nodes = da.n_nodes;
    v->stats.n_slots = da.n_slots;
    v->stats.max_bytes = da.max_bytes;
    v->stats.max_cp = da.max_cp;
    v->stats.device_bytes = (uint64_t)da.n_slots * (sizeof(int2) + sizeof(int32_t) + sizeof(int4)) + 65536 * (sizeof(int2) + sizeof(int4));
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
    void *ps[] = {c->staging, c->staging16, c->rec, c->counts, c->retry_list, c->retry_count, c->wsl_scratch, c->scan_temp, c->h_text, c->h_cut,
                  c->h_ids, c->h_off, c->h_idoff, c->h_status, c->h_capped, c->h_edges};
    for (void *p : ps)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    delete c;
    return DPT_OK;
}

int dpt_ctx_reserve(dpt_ctx *c, uint64_t n_bytes, uint64_t n_str) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    DeviceGuard g(c->device);
    return ensure_workspace(c, n_bytes, n_str);
}

static int encode_impl(dpt_ctx *c, const dpt_vocab *v, int mode_flags, const uint8_t *text, uint64_t n_bytes,
                       const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap,
                       uint64_t *id_off, int32_t *status, int32_t *capped_len, uint64_t *edges, void *hip_stream) {
    const int mode = mode_flags & DPT_MODE_MASK;
    if (!c || !v) return fail(DPT_E_ARG, "null ctx or vocab");
    if (mode != DPT_MODE_RAW && mode != DPT_MODE_PRESPLIT && mode != DPT_MODE_ATOMS) return fail(DPT_E_ARG, "bad mode");
    if (mode_flags & ~(DPT_MODE_MASK | DPT_FLAG_UNCAPPED | DPT_FLAG_LEN_ONLY)) return fail(DPT_E_ARG, "bad flags");
    if (!str_off || !id_off || (n_str && !status)) return fail(DPT_E_ARG, "null output/offsets");
    if (n_bytes && (!text || !ids)) return fail(DPT_E_ARG, "null text/ids");
    if (mode != DPT_MODE_RAW && n_bytes && !cut_mask) return fail(DPT_E_ARG, "PRESPLIT/ATOMS need cut_mask");
    if (ids_cap < n_bytes) return fail(DPT_E_CAP, "ids_cap must be >= n_bytes");
    if (n_str > 0x7FFFFFFFull) return fail(DPT_E_ARG, "too many strings for one call (max 2^31-1)");
    if (c->device != v->device) return fail(DPT_E_ARG, "ctx and vocab on different devices");
    DeviceGuard g(c->device);
    int rc = ensure_workspace(c, n_bytes, n_str);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)hip_stream;
    dpt::EncodeLaunch p;
    p.mode = mode_flags;
    if (const char *e = getenv("DPT_B"))   // A/B diagnostic only
        if (e[0] == 'r') p.mode |= dpt::DPT_FLAG_OLD_B;
    p.edges = edges;
    p.text = text;
    p.str_off = str_off;
    p.cut_mask = cut_mask;
    p.n_str = n_str;
    p.ids = ids;
    p.id_off = id_off;
    p.status = status;
    p.capped = capped_len;
    p.staging = c->staging;
    p.counts = c->counts;
    p.retry_list = c->retry_list;
    p.retry_count = c->retry_count;
    p.wsl_scratch = c->wsl_scratch;
    p.long_span = v->stats.max_cp > 64 ? 1 : 0;
    p.max_tok_bytes = v->stats.max_bytes;
    p.scan_temp = c->scan_temp;
    p.scan_temp_bytes = c->scan_bytes;
    p.max_blocks = c->max_blocks;
    p.rec = c->rec;
    p.variant = kernel_variant(v->stats.max_cp);
    // the lane kernel implements the plain raw / pre-split encode only
    if (p.variant == dpt::KERNEL_LANE && ((mode_flags != DPT_MODE_RAW && mode_flags != DPT_MODE_PRESPLIT) || edges))
        p.variant = v->stats.max_cp <= 16 ? dpt::KERNEL_ROWS16 : dpt::KERNEL_ROWS64;
    // int16 staging when every id fits (the lane kernel stages int32 only); DPT_WIDE_STAGING=1: A/B only
    p.staging16 = (v->ids16 && p.variant != dpt::KERNEL_LANE && !getenv("DPT_WIDE_STAGING")) ? c->staging16 : nullptr;
    p.slots = v->d_slots;
    p.slot_ids = v->d_ids;
    p.n_slots = v->stats.n_slots;
    p.slots4 = v->d_slots4;
    p.root_base = v->root_base;
    hipEvent_t ev[6];
    hipEvent_t *evp = nullptr;
    if (c->profile) {
        for (int k = 0; k < 4; k++) {
            hipError_t e = hipEventCreate(&ev[k]);
            if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
            c->events.push_back(ev[k]);
        }
        evp = ev;
        c->launches++;
    }
    hipError_t e = dpt::launch_encode(p, st, evp);
    if (e != hipSuccess) return hip_fail(e, "encode launch");
    return DPT_OK;
}

int dpt_encode(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
               const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids, uint64_t ids_cap,
               uint64_t *id_off, int32_t *status, int32_t *capped_len, void *hip_stream) {
    if (mode & ~DPT_MODE_MASK) return fail(DPT_E_ARG, "flags are for dpt_dp_host");
    return encode_impl(c, v, mode, text, n_bytes, str_off, cut_mask, n_str, ids, ids_cap, id_off, status, capped_len,
                       nullptr, hip_stream);
}

static int encode_host_impl(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
                            const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids,
                            uint64_t ids_cap, uint64_t *id_off, int32_t *status, int32_t *capped_len,
                            uint64_t *edges) {
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
    uint64_t cb = c->h_cap_bytes, cs = c->h_cap_str;
    if (n_bytes + 1 > c->h_cap_bytes || !c->h_text) {
        uint64_t c1 = cb, c2 = cb, c3 = cb;
        if ((e = grow(&c->h_text, &c1, n_bytes + 1)) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = grow(&c->h_cut, &c2, n_bytes + 1)) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = grow(&c->h_ids, &c3, n_bytes + 1)) != hipSuccess) return hip_fail(e, "hipMalloc");
        c->h_cap_bytes = c1 < c2 ? (c1 < c3 ? c1 : c3) : (c2 < c3 ? c2 : c3);
    }
    if (n_str + 2 > c->h_cap_str || !c->h_off) {
        uint64_t c1 = cs, c2 = cs, c3 = cs, c4 = cs;
        if ((e = grow(&c->h_off, &c1, n_str + 2)) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = grow(&c->h_idoff, &c2, n_str + 2)) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = grow(&c->h_status, &c3, n_str + 2)) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = grow(&c->h_capped, &c4, n_str + 2)) != hipSuccess) return hip_fail(e, "hipMalloc");
        uint64_t m = c1 < c2 ? c1 : c2;
        m = m < c3 ? m : c3;
        c->h_cap_str = m < c4 ? m : c4;
    }
    hipStream_t st = 0;
    if (n_bytes && (e = hipMemcpyAsync(c->h_text, text, n_bytes, hipMemcpyHostToDevice, st)) != hipSuccess)
        return hip_fail(e, "H2D text");
    if ((mode & DPT_MODE_MASK) != DPT_MODE_RAW && n_bytes &&
        (e = hipMemcpyAsync(c->h_cut, cut_mask, n_bytes, hipMemcpyHostToDevice, st)) != hipSuccess)
        return hip_fail(e, "H2D cut");
    // offsets rebased to 0 so that the device view is self-contained
    std::vector<uint64_t> off(n_str + 1);
    for (uint64_t i = 0; i <= n_str; i++) off[i] = str_off[i] - str_off[0];
    if ((e = hipMemcpyAsync(c->h_off, off.data(), (n_str + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st)) != hipSuccess)
        return hip_fail(e, "H2D offsets");
    uint64_t *d_edges = nullptr;
    if (edges) {
        uint64_t cap = c->h_cap_edges;
        if ((e = grow(&c->h_edges, &cap, n_bytes + 1)) != hipSuccess) return hip_fail(e, "hipMalloc(edges)");
        c->h_cap_edges = cap;
        d_edges = c->h_edges;
    }
    int rc = encode_impl(c, v, mode, c->h_text, n_bytes, c->h_off, c->h_cut, n_str, c->h_ids, c->h_cap_bytes, c->h_idoff,
                         c->h_status, c->h_capped, d_edges, st);
    if (rc) return rc;
    if (edges && n_bytes &&
        (e = hipMemcpyAsync(edges, d_edges, n_bytes * sizeof(uint64_t), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_fail(e, "D2H edges");
    if ((e = hipMemcpyAsync(id_off, c->h_idoff, (n_str + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_fail(e, "D2H id_off");
    if (n_str && (e = hipMemcpyAsync(status, c->h_status, n_str * sizeof(int32_t), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_fail(e, "D2H status");
    if (capped_len && n_str &&
        (e = hipMemcpyAsync(capped_len, c->h_capped, n_str * sizeof(int32_t), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_fail(e, "D2H capped");
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "sync");
    const uint64_t total = id_off[n_str];
    if (total > ids_cap) return fail(DPT_E_CAP, "ids overflow");
    if (total && (e = hipMemcpy(ids, c->h_ids, total * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "D2H ids");
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

int dpt_token_histogram(const uint64_t *id_off, const int32_t *status, uint64_t n_str, int64_t *hist, uint32_t n_bins,
                        void *hip_stream) {
    if (!id_off || !hist || (n_str && !status) || n_bins < 2) return fail(DPT_E_ARG, "bad histogram arguments");
    hipError_t e = dpt::launch_histogram(id_off, status, n_str, hist, n_bins, (hipStream_t)hip_stream);
    if (e != hipSuccess) return hip_fail(e, "histogram launch");
    return DPT_OK;
}

int dpt_ctx_profile(dpt_ctx *c, int enable) {
    if (!c) return fail(DPT_E_ARG, "null ctx");
    c->profile = enable != 0;
    return DPT_OK;
}

int dpt_ctx_profile_read(dpt_ctx *c, double *ms, uint64_t *launches) {
    if (!c || !ms) return fail(DPT_E_ARG, "null argument");
    DeviceGuard g(c->device);
    ms[0] = ms[1] = ms[2] = 0.0;
    for (size_t k = 0; k + 3 < c->events.size(); k += 4) {
        hipError_t e = hipEventSynchronize(c->events[k + 3]);
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        for (int s = 0; s < 3; s++) {
            float t = 0.f;
            e = hipEventElapsedTime(&t, c->events[k + s], c->events[k + s + 1]);
            if (e != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
            ms[s] += t;
        }
    }
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    c->events.clear();
    if (launches) *launches = c->launches;
    c->launches = 0;
    return DPT_OK;
}

}  // extern "C"
