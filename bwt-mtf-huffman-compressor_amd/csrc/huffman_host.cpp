// huffman_host.cpp — Huffman tree, code table and tree serialisation for one block.
//
// Replaces the tree half of huffman() (reference main.cpp:229-257), traverse/build_hashmap
// (main.cpp:132-156) and dfs/tree_to_bytes (main.cpp:174-196). O(L log L) for L <= 256
// leaves, so it stays on the host between the MTF and pack kernels.
//
// Tie-break. The reference's std::priority_queue<pair<long, BTree*>> pops the smallest
// frequency and, among equal frequencies, the node with the HIGHER heap address. Node
// addresses come from glibc malloc in a standalone COMPRESS run; SURVEY.md Appendix B.3
// gives their ascending order as a function of the leaf count L (node ids: leaves 0..L-1
// in first-occurrence order of the MTF stream, internal nodes L, L+1, ... in creation
// order). addr_index() below maps a node id to its position in that order; below kBandCeil
// bytes the order comes from the reference's heap history instead (heap_order.cpp).
#include "bmh_internal.h"

#include <algorithm>
#include <queue>

namespace bmh {

namespace {

uint32_t addr_index(uint32_t L, uint32_t s)
{
    if (L <= 128) {
        // [1, 3..127, 0, 2, 128, 129, ...]
        if (s == 1) return 0;
        if (s >= 3 && s <= 127) return s - 2;
        if (s == 0) return 126;
        if (s == 2) return 127;
        return s;
    }
    // [1, 3..64, 129..192, 65..127, 0, 2, 128, 193, 194, ...]
    if (s == 1) return 0;
    if (s >= 3 && s <= 64) return s - 2;
    if (s >= 129 && s <= 192) return s - 66;
    if (s >= 65 && s <= 127) return s + 62;
    if (s == 0) return 190;
    if (s == 2) return 191;
    if (s == 128) return 192;
    return s;
}

struct Node {
    uint64_t freq;
    int16_t left, right;  // -1 for leaves
    uint8_t sym;
};

}  // namespace

void huffman_build(const uint64_t freq[256], const uint64_t first[256], bmh_code_table *out, uint64_t n)
{
    memset(out, 0, sizeof *out);
    // leaves in first-occurrence order (main.cpp:238-244)
    uint8_t order[256];
    uint32_t L = 0;
    for (int s = 0; s < 256; ++s)
        if (freq[s] > 0) order[L++] = (uint8_t)s;
    if (L == 0) fail(BMH_EINVAL, "huffman: empty histogram (the reference segfaults on empty input)");
    std::sort(order, order + L, [&](uint8_t a, uint8_t b) { return first[a] < first[b]; });

    Node nd[511];
    uint32_t nn = 0;
    // address ranks: the reference's heap history below kBandCeil (heap_order.cpp), else the
    // closed form
    uint16_t rank[511];
    const bool hist = n != 0 && n < kBandCeil;
    if (hist) node_ranks(n, L, rank);
    auto pops_first = [&](uint32_t a, uint32_t b) {  // true if node a leaves the queue before b
        if (nd[a].freq != nd[b].freq) return nd[a].freq < nd[b].freq;
        return hist ? rank[a] > rank[b] : addr_index(L, a) > addr_index(L, b);
    };
    auto cmp = [&](uint32_t a, uint32_t b) { return pops_first(b, a); };  // max-heap on pops_first
    std::priority_queue<uint32_t, std::vector<uint32_t>, decltype(cmp)> pq(cmp);
    for (uint32_t i = 0; i < L; ++i) {
        nd[nn] = Node{freq[order[i]], -1, -1, order[i]};
        pq.push(nn++);
    }
    // main.cpp:245-254: first pop -> left, second -> right
    while (pq.size() > 1) {
        const uint32_t a = pq.top();
        pq.pop();
        const uint32_t b = pq.top();
        pq.pop();
        nd[nn] = Node{nd[a].freq + nd[b].freq, (int16_t)a, (int16_t)b, 0};
        pq.push(nn++);
    }
    const uint32_t root = pq.top();

    // codes: left = 0, right = 1 (main.cpp:143-144); a root leaf gets the empty code.
    struct Item {
        uint32_t v;
        uint64_t code;
        uint32_t depth;
    };
    std::vector<Item> st;
    st.push_back({root, 0, 0});
    // preorder tree bits (main.cpp:174-187): internal 1, leaf 0 + 8 value bits MSB-first
    uint32_t bit = 0;
    auto put = [&](uint32_t b) {
        if (b) out->tree[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
        ++bit;
    };
    while (!st.empty()) {
        Item it = st.back();
        st.pop_back();
        const Node &x = nd[it.v];
        if (x.left < 0) {
            if (it.depth > 64) fail(BMH_ERANGE, "huffman: code longer than 64 bits");
            out->len[x.sym] = (uint8_t)it.depth;
            out->code[x.sym] = it.code;
            put(0);
            for (int k = 7; k >= 0; --k) put((x.sym >> k) & 1u);
        } else {
            put(1);
            st.push_back({(uint32_t)x.right, (it.code << 1) | 1u, it.depth + 1});
            st.push_back({(uint32_t)x.left, it.code << 1, it.depth + 1});
        }
    }
    out->tree_len = (bit + 7) >> 3;
    out->leaves = L;
}

uint64_t payload_bytes(const bmh_code_table *t, const uint64_t freq[256])
{
    uint64_t bits = 0;
    for (int s = 0; s < 256; ++s) bits += freq[s] * t->len[s];
    const uint64_t bytes = (bits + 7) / 8;
    return bytes ? bytes : 1;  // encode_with_huffman starts from one zero byte (main.cpp:162)
}

}  // namespace bmh
