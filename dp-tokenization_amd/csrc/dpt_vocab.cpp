// dpt_vocab.cpp -- host packer: the vocabulary key set (reference
// packages/tokenizer_utils.py:53-57, `vocab = set(llama_tokenizer.get_vocab())`)
// becomes a byte-level double-array trie that the kernels walk from L2.
//
//   slot t of a node reached by byte b from parent p:  t = base[p] + b, check[t] == p
//   base[t] carries bit 31 when a token ends at t (id[t] is that token's id) and bit 30 when
//   the node has no children (a walk that reaches it is over without another lookup).
//
// Placement is first-fit over free slots (a find-next-free forest with path
// compression), breadth-first from the root, so hot short prefixes sit in the
// first few KB of the table.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "dpt_internal.h"

namespace dpt {

namespace {

struct Node {
    uint32_t first_child = 0;   // 0 = none (node 0 is the root, never a child)
    uint32_t next_sibling = 0;
    int32_t id = -1;
    uint8_t label = 0;
};

struct FreeFinder {
    std::vector<uint32_t> parent;  // parent[x] = x if free, else a larger candidate
    explicit FreeFinder(size_t n) : parent(n) {
        for (size_t i = 0; i < n; i++) parent[i] = (uint32_t)i;
    }
    void grow(size_t n) {
        size_t o = parent.size();
        if (n <= o) return;
        parent.resize(n);
        for (size_t i = o; i < n; i++) parent[i] = (uint32_t)i;
    }
    uint32_t find(uint32_t x) {
        grow((size_t)x + 1024);
        uint32_t r = x;
        while (parent[r] != r) {
            r = parent[r];
            grow((size_t)r + 1024);
        }
        while (parent[x] != r) {
            uint32_t nx = parent[x];
            parent[x] = r;
            x = nx;
        }
        return r;
    }
    void take(uint32_t x) {
        grow((size_t)x + 1025);
        parent[x] = x + 1;
    }
};

}  // namespace

const char *build_double_array(const uint8_t *blob, const uint64_t *off, const int32_t *ids, uint32_t n,
                               DoubleArray *out) {
    std::vector<Node> nodes(1);
    uint32_t max_bytes = 0, max_cp = 0, n_tok = 0;
    for (uint32_t t = 0; t < n; t++) {
        const uint8_t *p = blob + (off[t] - off[0]);
        const uint64_t len = off[t + 1] - off[t];
        if (len == 0) continue;
        if (len > 0xFFFF) return "token longer than 65535 bytes";
        uint32_t cur = 0;
        uint32_t cp = 0;
        for (uint64_t k = 0; k < len; k++) {
            const uint8_t b = p[k];
            cp += (b & 0xC0) != 0x80;
            uint32_t c = nodes[cur].first_child, prev = 0;
            while (c && nodes[c].label < b) { prev = c; c = nodes[c].next_sibling; }
            if (!c || nodes[c].label != b) {
                Node nn;
                nn.label = b;
                nn.next_sibling = c;
                nodes.push_back(nn);
                const uint32_t ni = (uint32_t)nodes.size() - 1;
                if (prev) nodes[prev].next_sibling = ni;
                else nodes[cur].first_child = ni;
                c = ni;
            }
            cur = c;
        }
        if (nodes[cur].id < 0) n_tok++;
        nodes[cur].id = ids ? ids[t] : (int32_t)t;   // later duplicates win (dict semantics)
        if (len > max_bytes) max_bytes = (uint32_t)len;
        if (cp > max_cp) max_cp = cp;
    }

    // breadth-first placement
    std::vector<int32_t> base(1024, 0), check(1024, -1), tid(1024, -1);
    auto ensure = [&](size_t n) {
        if (n > base.size()) {
            size_t m = std::max(n, base.size() * 2);
            base.resize(m, 0);
            check.resize(m, -1);
            tid.resize(m, -1);
        }
    };
    FreeFinder ff(1 << 16);
    ff.take(0);                       // root occupies slot 0
    check[0] = -2;
    std::vector<std::pair<uint32_t, uint32_t>> queue;  // (trie node, slot)
    queue.reserve(nodes.size());
    queue.push_back({0u, 0u});
    uint32_t max_slot = 0;
    std::vector<uint8_t> labels;
    std::vector<uint32_t> kids;
    for (size_t qi = 0; qi < queue.size(); qi++) {
        const uint32_t nd = queue[qi].first, slot = queue[qi].second;
        if (nodes[nd].id >= 0) tid[slot] = nodes[nd].id;
        labels.clear();
        kids.clear();
        for (uint32_t c = nodes[nd].first_child; c; c = nodes[c].next_sibling) {
            labels.push_back(nodes[c].label);
            kids.push_back(c);
        }
        if (labels.empty()) { base[slot] = 0x40000000; continue; }   // leaf
        // smallest b >= 0 with every b+label free
        uint32_t x = labels[0];
        uint32_t b;
        for (;;) {
            const uint32_t f = ff.find(x);
            b = f - labels[0];
            bool ok = true;
            for (size_t k = 1; k < labels.size(); k++) {
                const uint32_t t = b + labels[k];
                if (ff.find(t) != t) { ok = false; break; }
            }
            if (ok) break;
            x = f + 1;
        }
        base[slot] = (int32_t)b;
        for (size_t k = 0; k < labels.size(); k++) {
            const uint32_t t = b + labels[k];
            ff.take(t);
            ensure((size_t)t + 1);
            check[t] = (int32_t)slot;
            if (t > max_slot) max_slot = t;
            queue.push_back({kids[k], t});
        }
        if (b > 0x3FFFFF00u) return "double array too large";
    }
    // mark terminals
    const uint32_t n_slots = max_slot + 1 + 256;
    ensure(n_slots);
    for (uint32_t t = 0; t < n_slots; t++)
        if (tid[t] >= 0) base[t] |= (int32_t)0x80000000;
    check[0] = -2;

    out->n_slots = n_slots;
    out->n_nodes = (uint32_t)nodes.size();
    out->n_tokens = n_tok;
    out->max_bytes = max_bytes;
    out->max_cp = max_cp;
    out->root_base = base[0] & 0x3FFFFFFF;
    out->base = (int32_t *)malloc(sizeof(int32_t) * n_slots);
    out->check = (int32_t *)malloc(sizeof(int32_t) * n_slots);
    out->id = (int32_t *)malloc(sizeof(int32_t) * n_slots);
    memcpy(out->base, base.data(), sizeof(int32_t) * n_slots);
    memcpy(out->check, check.data(), sizeof(int32_t) * n_slots);
    memcpy(out->id, tid.data(), sizeof(int32_t) * n_slots);
    return nullptr;
}

void free_double_array(DoubleArray *da) {
    free(da->base);
    free(da->check);
    free(da->id);
    da->base = da->check = da->id = nullptr;
}

}  // namespace dpt
