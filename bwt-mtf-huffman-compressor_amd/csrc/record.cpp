// record.cpp — the reference record format, the multi-block container, and the host decoder.
//
// Record (write_bytes / read_bytes, reference io_utilities.h:7-55, little-endian):
//   [u64 primary][u64 n][u64 tree_len][tree_len bytes preorder tree][payload to end]
// Container (ours, for block_size < file size): "\xffBMHBLK1" | u64 block_size |
//   u64 nblocks | u64 total_n | u64 record_len[nblocks] | verbatim records.
//   A record's first u64 is its primary index (< n), so the 0xff-led magic cannot be one.
//
// Decoder replaces decompress() (main.cpp:327-345): tree parse (bytes_to_tree_dfs,
// main.cpp:198-219), Huffman decode (huffman_reverse, main.cpp:259-281 — here table-driven
// instead of a bit-serial hash lookup), inverse MTF (main.cpp:114-130), inverse BWT
// (bwt_reverse, main.cpp:61-75 — counting sort of L, then the chase from the primary row).
#include "bmh_internal.h"

#include <algorithm>
#include <thread>

namespace bmh {

const uint8_t kContainerMagic[8] = {0xff, 'B', 'M', 'H', 'B', 'L', 'K', '1'};

void put_u64(uint8_t *p, uint64_t v)
{
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
uint64_t get_u64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

namespace {

struct BitReader {
    const uint8_t *p;
    uint64_t nbytes, pos = 0;  // bit position
    int bit()
    {
        if ((pos >> 3) >= nbytes) fail(BMH_ECORRUPT, "record: bitstream truncated");
        int b = (p[pos >> 3] >> (7 - (pos & 7))) & 1;
        ++pos;
        return b;
    }
    // next 32 bits MSB-first (zero padded past the end)
    uint32_t peek32() const
    {
        uint64_t byte = pos >> 3;
        uint64_t v = 0;
        for (int i = 0; i < 5; ++i) v = (v << 8) | (byte + i < nbytes ? p[byte + i] : 0u);
        return (uint32_t)(v >> (8 - (pos & 7)));
    }
};

struct DTree {
    int16_t left[511], right[511];
    uint8_t sym[511];
    int n = 0;
    int parse(BitReader &r, int depth)
    {
        if (n >= 511 || depth > 256) fail(BMH_ECORRUPT, "record: malformed tree");
        const int v = n++;
        if (!r.bit()) {
            int s = 0;
            for (int i = 0; i < 8; ++i) s = (s << 1) | r.bit();
            left[v] = right[v] = -1;
            sym[v] = (uint8_t)s;
            return v;
        }
        const int l = parse(r, depth + 1);
        const int rr = parse(r, depth + 1);
        left[v] = (int16_t)l;
        right[v] = (int16_t)rr;
        sym[v] = 0;
        return v;
    }
};

constexpr int kLutBits = 12;

void decode_mtf(const uint8_t *rec, uint64_t len, uint8_t *mtf, uint64_t n, uint64_t tlen)
{
    BitReader tr{rec + kRecordHeader, tlen};
    DTree t;
    const int root = t.parse(tr, 0);
    const uint8_t *pay = rec + kRecordHeader + tlen;
    const uint64_t plen = len - kRecordHeader - tlen;
    if (t.left[root] < 0) {  // single leaf: empty code words
        memset(mtf, t.sym[root], n);
        return;
    }
    // LUT over the next kLutBits bits: leaf reached within them -> (sym, bits used); else the
    // internal node reached after kLutBits bits (flagged) to continue bit by bit.
    std::vector<uint32_t> lut(1u << kLutBits);
    for (uint32_t idx = 0; idx < (1u << kLutBits); ++idx) {
        int v = root, used = 0;
        while (t.left[v] >= 0 && used < kLutBits) {
            v = ((idx >> (kLutBits - 1 - used)) & 1u) ? t.right[v] : t.left[v];
            ++used;
        }
        lut[idx] = t.left[v] < 0 ? (uint32_t)t.sym[v] | ((uint32_t)used << 8) : (0x80000000u | (uint32_t)v);
    }
    BitReader r{pay, plen};
    const uint64_t total_bits = plen * 8;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t e = lut[r.peek32() >> (32 - kLutBits)];
        if (!(e & 0x80000000u)) {
            r.pos += e >> 8;
            if (r.pos > total_bits) fail(BMH_ECORRUPT, "record: bitstream truncated");
            mtf[i] = (uint8_t)e;
        } else {
            r.pos += kLutBits;
            int v = (int)(e & 0xffffu);
            while (t.left[v] >= 0) v = r.bit() ? t.right[v] : t.left[v];
            mtf[i] = t.sym[v];
        }
    }
}

void mtf_inverse(const uint8_t *in, uint64_t n, uint8_t *out)
{
    uint8_t a[256];
    for (int i = 0; i < 256; ++i) a[i] = (uint8_t)i;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t j = in[i], c = a[j];
        out[i] = c;
        memmove(a + 1, a, j);
        a[0] = c;
    }
}

void bwt_inverse(const uint8_t *L, uint64_t n, uint64_t primary, uint8_t *out)
{
    if (primary >= n) fail(BMH_ECORRUPT, "record: primary index out of range");
    std::vector<uint32_t> ls(n);
    uint64_t cnt[257] = {0};
    for (uint64_t i = 0; i < n; ++i) cnt[L[i] + 1]++;
    for (int c = 0; c < 256; ++c) cnt[c + 1] += cnt[c];
    for (uint64_t i = 0; i < n; ++i) ls[cnt[L[i]]++] = (uint32_t)i;
    uint64_t row = primary;
    for (uint64_t i = 0; i < n; ++i) {
        row = ls[row];
        out[i] = L[row];
    }
}

}  // namespace

void build_dec_table(const uint8_t *tree, uint64_t tree_len, DecTable *out)
{
    BitReader tr{tree, tree_len};
    DTree t;
    const int root = t.parse(tr, 0);
    memset(out, 0, sizeof *out);
    for (int v = 0; v < t.n; ++v) {
        out->child[v][0] = t.left[v] < 0 ? 0xffff : (uint16_t)t.left[v];
        out->child[v][1] = t.right[v] < 0 ? 0xffff : (uint16_t)t.right[v];
        out->sym[v] = t.sym[v];
    }
    if (t.left[root] < 0) {
        out->single = 1;
        out->sym[0] = t.sym[root];
        return;
    }
    // fill the LUT by walking the tree: a leaf at depth d <= 12 covers 2^(12-d) entries
    struct Item {
        int v;
        uint32_t code, depth;
    };
    std::vector<Item> st{{root, 0, 0}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        if (t.left[it.v] < 0) out->maxlen = std::max(out->maxlen, it.depth);
        if (t.left[it.v] < 0 || it.depth == kDecLutBits) {
            const uint32_t span = 1u << (kDecLutBits - it.depth), first = it.code << (kDecLutBits - it.depth);
            const uint32_t e = t.left[it.v] < 0 ? ((uint32_t)t.sym[it.v] << 8) | it.depth : (uint32_t)it.v << 16;
            for (uint32_t k = 0; k < span; ++k) out->lut[first + k] = e;
            if (t.left[it.v] < 0) continue;
            // a subtree below the LUT depth: its deepest leaf bounds the code length
            std::vector<std::pair<int, uint32_t>> sub{{it.v, it.depth}};
            while (!sub.empty()) {
                const auto [v, d] = sub.back();
                sub.pop_back();
                if (t.left[v] < 0) {
                    out->maxlen = std::max(out->maxlen, d);
                } else {
                    sub.push_back({t.left[v], d + 1});
                    sub.push_back({t.right[v], d + 1});
                }
            }
            continue;
        }
        st.push_back({t.right[it.v], (it.code << 1) | 1u, it.depth + 1});
        st.push_back({t.left[it.v], it.code << 1, it.depth + 1});
    }
}

uint64_t record_n(const uint8_t *rec, uint64_t len)
{
    // header sanity before anyone sizes a buffer from n
    if (len < kRecordHeader) fail(BMH_ECORRUPT, "record: shorter than its 24-byte header");
    const uint64_t n = get_u64(rec + 8), tlen = get_u64(rec + 16);
    if (n == 0) fail(BMH_ECORRUPT, "record: n == 0");
    if (tlen == 0 || tlen > len - kRecordHeader) fail(BMH_ECORRUPT, "record: tree length exceeds record");
    if (get_u64(rec) >= n) fail(BMH_ECORRUPT, "record: primary index out of range");
    // a root with two children gives every symbol a code of >= 1 bit
    const uint64_t pay = len - kRecordHeader - tlen;
    if ((rec[kRecordHeader] & 0x80u) && n / 8 > pay) fail(BMH_ECORRUPT, "record: n exceeds what the payload holds");
    return n;
}

void record_to_mtf(const uint8_t *rec, uint64_t len, uint8_t *mtf, uint64_t cap, uint64_t *n_out)
{
    const uint64_t n = record_n(rec, len);
    const uint64_t tlen = get_u64(rec + 16);
    if (tlen > len - kRecordHeader) fail(BMH_ECORRUPT, "record: tree length exceeds record");
    if (n == 0) fail(BMH_ECORRUPT, "record: n == 0");
    *n_out = n;
    if (!mtf) return;
    if (n > cap) fail(BMH_ERANGE, "record: output capacity too small");
    decode_mtf(rec, len, mtf, n, tlen);
}

void decode_record(const uint8_t *rec, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out)
{
    const uint64_t n = record_n(rec, len);
    *n_out = n;
    if (!out) return;
    if (n > cap) fail(BMH_ERANGE, "record: output capacity too small");
    std::vector<uint8_t> m(n), Lb(n);
    uint64_t got = 0;
    record_to_mtf(rec, len, m.data(), n, &got);
    mtf_inverse(m.data(), n, Lb.data());
    bwt_inverse(Lb.data(), n, get_u64(rec), out);
}

bool is_container(const uint8_t *in, uint64_t len) { return len >= 8 && memcmp(in, kContainerMagic, 8) == 0; }

ContainerView parse_container(const uint8_t *in, uint64_t len)
{
    if (!is_container(in, len) || len < 32) fail(BMH_ECORRUPT, "container: bad magic");
    ContainerView v;
    v.block_size = get_u64(in + 8);
    v.nblocks = get_u64(in + 16);
    v.total = get_u64(in + 24);
    if (v.nblocks == 0 || v.nblocks > (len - 32) / 8) fail(BMH_ECORRUPT, "container: bad block count");
    uint64_t o = 32 + 8 * v.nblocks;
    for (uint64_t b = 0; b < v.nblocks; ++b) {
        const uint64_t l = get_u64(in + 32 + 8 * b);
        if (l > len || o > len - l) fail(BMH_ECORRUPT, "container: record overruns input");
        v.rec_off.push_back(o);
        v.rec_len.push_back(l);
        o += l;
    }
    return v;
}

void decompress(const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out)
{
    if (!is_container(in, len)) {
        decode_record(in, len, out, cap, n_out);
        return;
    }
    ContainerView v = parse_container(in, len);
    *n_out = v.total;
    if (!out) return;
    if (v.total > cap) fail(BMH_ERANGE, "container: output capacity too small");
    std::vector<uint64_t> dst(v.nblocks + 1, 0);
    for (uint64_t b = 0; b < v.nblocks; ++b) dst[b + 1] = dst[b] + record_n(in + v.rec_off[b], v.rec_len[b]);
    if (dst[v.nblocks] != v.total) fail(BMH_ECORRUPT, "container: block sizes do not add up");
    // each thread holds ~6 bytes per symbol of its current block: cap the threads so the
    // concurrent working set stays under ~6 GiB
    uint64_t max_n = 1;
    for (uint64_t b = 0; b < v.nblocks; ++b) max_n = std::max(max_n, dst[b + 1] - dst[b]);
    const uint64_t mem_threads = std::max<uint64_t>(1, (6ull << 30) / (6 * max_n));
    const unsigned nt = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>({std::thread::hardware_concurrency(), 16u, mem_threads, v.nblocks}));
    std::vector<std::thread> th;
    std::vector<std::string> errs(nt);
    std::vector<bmh_status> sts(nt, BMH_OK);
    for (unsigned t = 0; t < nt; ++t) {
        th.emplace_back([&, t]() {
            try {
                for (uint64_t b = t; b < v.nblocks; b += nt) {
                    uint64_t got;
                    decode_record(in + v.rec_off[b], v.rec_len[b], out + dst[b], dst[b + 1] - dst[b], &got);
                }
            } catch (const Error &e) {
                sts[t] = e.status;
                errs[t] = e.what();
            } catch (const std::bad_alloc &) {
                sts[t] = BMH_ENOMEM;
                errs[t] = "container: host allocation failed while decoding";
            } catch (const std::exception &e) {
                sts[t] = BMH_EINVAL;
                errs[t] = e.what();
            } catch (...) {
                sts[t] = BMH_EINVAL;
                errs[t] = "container: unknown exception while decoding";
            }
        });
    }
    for (auto &x : th) x.join();
    for (unsigned t = 0; t < nt; ++t)
        if (sts[t] != BMH_OK) fail(sts[t], errs[t]);
}

}  // namespace bmh
