// pack.hip — Huffman bit-pack of a batch of MTF streams into reference records.
//
// Replaces encode_with_huffman() + append_bit (reference main.cpp:158-172,
// io_utilities.h:87-94): code words concatenated MSB-first, the first bit at bit 7 of the
// payload's first byte. Three steps per block, chunked 4096 symbols per workgroup:
//   bits   : per chunk, sum of code lengths (code-length table in LDS)
//   scan   : per block, exclusive scan of chunk bit counts (u64)
//   write  : per chunk, thread bit offsets by a workgroup scan; code words OR'd into an LDS
//            image of the chunk's 32-bit big-endian words; interior words stored, the two
//            edge words (shared with neighbouring chunks / record headers) updated under a
//            mask of this chunk's bits (atomicAnd + atomicOr), so the output needs no
//            zeroing pass. The block's last chunk owns the zero pad bits of its last byte.
// Record headers are written before the pack (huffman.hip); the payload of block b starts
// at byte pay_offs[b].
#include "bmh_internal.h"
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

constexpr uint32_t kPackChunk = kPackChunkSyms;  // symbols per workgroup (256 threads x 16)
constexpr uint32_t kPackIPT = kPackChunk / 256;

struct PChunk {
    uint32_t block, start, len, pad;
};

__global__ __launch_bounds__(256) void k_pack_bits(const uint8_t *__restrict__ mtf, const PChunk *__restrict__ chunks,
                                                   const DevTable *__restrict__ tabs, uint64_t *__restrict__ cbits)
{
    __shared__ uint8_t s_len[256];
    __shared__ uint64_t s_tmp[8];
    const PChunk ch = chunks[blockIdx.x];
    s_len[threadIdx.x] = tabs[ch.block].len[threadIdx.x];
    __syncthreads();
    uint64_t s = 0;
    for (uint32_t i = threadIdx.x; i < ch.len; i += 256) s += s_len[mtf[ch.start + i]];
    uint64_t total;
    block_excl_sum64<256>(s, s_tmp, &total);
    if (threadIdx.x == 0) cbits[blockIdx.x] = total;
}

// Chunk bit counts from the per-chunk MTF histograms, sum cnt[v] * len[v]: one wave per
// kBitsCPW consecutive chunks, every histogram and chunk entry loaded before the first code-length
// read (which depends on the chunk's block), so a wave waits for two loads, not two per chunk.
constexpr uint32_t kBitsCPW = 4;
__global__ __launch_bounds__(256) void k_pack_bits_hist(const uint16_t *__restrict__ chist,
                                                        const PChunk *__restrict__ chunks, uint32_t nch,
                                                        const DevTable *__restrict__ tabs, uint64_t *__restrict__ cbits)
{
    const uint32_t c0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kBitsCPW, l = threadIdx.x & 63u;
    if (c0 >= nch) return;
    uint2 h[kBitsCPW];
    uint32_t blk[kBitsCPW];
#pragma unroll
    for (uint32_t i = 0; i < kBitsCPW; ++i) {
        const uint32_t c = min(c0 + i, nch - 1);
        h[i] = *(const uint2 *)(chist + (size_t)c * 256 + 4 * l);
        blk[i] = chunks[c].block;
    }
#pragma unroll
    for (uint32_t i = 0; i < kBitsCPW; ++i) {
        const uint32_t lw = *(const uint32_t *)(tabs[blk[i]].len + 4 * l);
        uint64_t s = (uint64_t)(h[i].x & 0xffffu) * (lw & 255u) + (uint64_t)(h[i].x >> 16) * ((lw >> 8) & 255u) +
                     (uint64_t)(h[i].y & 0xffffu) * ((lw >> 16) & 255u) + (uint64_t)(h[i].y >> 16) * (lw >> 24);
        s = wave_sum64(s);
        if (l == 0 && c0 + i < nch) cbits[c0 + i] = s;
    }
}

// grid = nblocks; exclusive scan of the block's chunk bit counts (in place); btot (may be null)
// receives each block's payload bits
__global__ __launch_bounds__(256) void k_pack_scan(const uint32_t *__restrict__ cfirst, uint64_t *__restrict__ cbits,
                                                   uint64_t *__restrict__ btot)
{
    __shared__ uint64_t s_tmp[8];
    const uint32_t c0 = cfirst[blockIdx.x], c1 = cfirst[blockIdx.x + 1];
    uint64_t carry = 0;
    for (uint32_t base = c0; base < c1; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t v = i < c1 ? cbits[i] : 0ull;
        uint64_t total;
        const uint64_t ex = block_excl_sum64<256>(v, s_tmp, &total);
        if (i < c1) cbits[i] = carry + ex;
        carry += total;
    }
    if (btot && threadIdx.x == 0) btot[blockIdx.x] = carry;
}

// The chunk's image is built in LDS windows of kPackImgWords words: one window whenever the
// chunk averages <= 15.9 bits per symbol (8 on random data); longer codes take more windows,
// each thread re-walking its 16 symbols and keeping only the words inside the window.
constexpr uint32_t kPackImgWords = 2048;
// Consecutive chunks per workgroup: the code table is loaded once per block run, the next
// chunk's symbols are in flight while this one is packed, and the image is zeroed by the
// store pass that drains it (no zeroing pass and barrier per chunk).
#ifndef BMH_PACK_CPW
#define BMH_PACK_CPW 16
#endif
constexpr uint32_t kPackCPW = BMH_PACK_CPW;  // 4 -> 8 -> 16: 0.81 -> 0.75 -> 0.71 ms per GiB (round 6)
// chunks per workgroup for a batch: up to kPackCPW while that still leaves 4 workgroups a CU (a
// small batch — Calgary's pipelines — keeps one chunk a workgroup: 16 would walk them serially)
static uint32_t pack_cpw(const Ctx *c, uint32_t nch)
{
    const uint32_t slots = 4u * (uint32_t)std::max(c->cus, 1);
    return std::max(1u, std::min(kPackCPW, nch / slots));
}

__device__ __forceinline__ uint4 pack_load_syms(const uint8_t *__restrict__ mtf, const PChunk &ch, uint32_t t)
{
    const uint32_t i0 = t * kPackIPT;
    uint4 v4 = make_uint4(0, 0, 0, 0);
    if (i0 + kPackIPT <= ch.len && ((ch.start + i0) & 15u) == 0) {
        v4 = *(const uint4 *)(mtf + ch.start + i0);
    } else {
        uint32_t *vw = &v4.x;
        for (uint32_t k = 0; k < kPackIPT; ++k)
            if (i0 + k < ch.len) vw[k >> 2] |= (uint32_t)mtf[ch.start + i0 + k] << (8 * (k & 3));
    }
    return v4;
}

// LDS slot of image word w: one pad word per 64, so lanes whose words are 4 apart (8-bit codes,
// 16 symbols a thread) or 2 apart fall in distinct banks
__device__ __forceinline__ uint32_t img_at(uint32_t w)
{
#ifdef BMH_PACK_SWZ
    return w + (w >> 6);
#else
    return w;
#endif
}

// Bits [0, l) of a code word, left-aligned in a 32-bit word, appended MSB-first to the 64-bit
// accumulator (hi, lo) holding nacc < 32 bits; a completed word is OR'd into the image
// (kWin: only words inside the window [wb, wb + nw)).
template <bool kWin>
__device__ __forceinline__ void pack_push(uint32_t v, uint32_t l, uint32_t &hi, uint32_t &lo, uint32_t &nacc, uint32_t &w,
                                          uint32_t *s_img, uint32_t wb, uint32_t nw)
{
    hi |= v >> nacc;                                // (v : 0) >> nacc, high word
    lo |= __builtin_amdgcn_alignbit(v, 0u, nacc);  // and low word
    nacc += l;
    if (nacc >= 32) {
        if (!kWin || w - wb < nw) atomicOr(&s_img[img_at(w - wb)], hi);
        hi = lo;
        lo = 0;
        ++w;
        nacc -= 32;
    }
}

__global__ __launch_bounds__(256) void k_pack_write(const uint8_t *__restrict__ mtf, const PChunk *__restrict__ chunks,
                                                    uint32_t nch, const DevTable *__restrict__ tabs,
                                                    const uint64_t *__restrict__ cboff,
                                                    const uint64_t *__restrict__ pay_offs,
                                                    const uint32_t *__restrict__ cfirst, uint32_t *__restrict__ out,
                                                    const uint32_t *status, uint32_t cpw)
{
    // code word left-aligned in 64 bits, its length in the low 8 bits (lengths <= 56, so the
    // code's last bit is above bit 8): the high half is the whole code whenever it fits 32 bits
    __shared__ uint64_t s_tab[256];
    __shared__ uint32_t s_tmp[8];
    __shared__ uint32_t s_img[kPackImgWords + kPackImgWords / 64];
    // per chunk of the workgroup, fetched up front (no dependent global loads per chunk): its first
    // bit, its block's first payload bit and bit offset within the block; whether it is the block's last
    __shared__ uint64_t s_G[kPackCPW], s_P[kPackCPW], s_cb[kPackCPW];
    __shared__ uint32_t s_last[kPackCPW];
    // the loads of the start are issued together (the status word, the chunk's symbols, its code
    // book and the per-chunk offsets), then waited for once
    const uint32_t st = status ? *status : 0u;
    const uint32_t t = threadIdx.x;
    const uint32_t c0 = blockIdx.x * cpw, c1 = min(c0 + cpw, nch);  // cpw <= kPackCPW
    PChunk ch = chunks[c0];
    uint4 v4 = pack_load_syms(mtf, ch, t);  // this chunk's 16 symbols of the thread
    uint32_t tl = tabs[ch.block].len[t];
    uint64_t tc = tabs[ch.block].code[t];
    if (t < c1 - c0) {
        const uint32_t c = c0 + t, b = chunks[c].block;
        const uint64_t P = pay_offs[b] * 8, cb = cboff[c];
        s_P[t] = P;
        s_cb[t] = cb;
        s_G[t] = P + cb;
        s_last[t] = c + 1 == cfirst[b + 1];
    }
    if (st & kStatusCapacity) return;  // workgroup-uniform
    for (uint32_t w = t; w < kPackImgWords + kPackImgWords / 64; w += 256) s_img[w] = 0;
    uint32_t tblock = ~0u;
    bool long32 = false;  // the block's code book has words longer than 32 bits (workgroup-uniform)
    bool short16 = false;  // all its words are <= 16 bits: two per push
    for (uint32_t c = c0; c < c1; ++c) {
        // the next chunk's symbols are loaded while this one is packed
        PChunk nx = ch;
        uint4 nv4 = make_uint4(0, 0, 0, 0);
        if (c + 1 < c1) {
            nx = chunks[c + 1];
            nv4 = pack_load_syms(mtf, nx, t);
        }
        if (ch.block != tblock) {  // workgroup-uniform; the previous chunk's readers are past a barrier
            if (tblock != ~0u) {  // a later block of the workgroup's chunks
                tl = tabs[ch.block].len[t];
                tc = tabs[ch.block].code[t];
            }
            const uint32_t l = tl;
            s_tab[t] = l ? (tc << (64 - l)) | l : 0ull;
            tblock = ch.block;
            const int lx = __syncthreads_or(l > 16) | (__syncthreads_or(l > 32) << 1);
            short16 = lx == 0;
            long32 = lx > 1;
        }
        const uint32_t i0 = t * kPackIPT;
        const uint32_t nsym = i0 < ch.len ? min(kPackIPT, ch.len - i0) : 0u;
        // (s_G .. s_last were written before the first chunk's code book barrier)
        const uint64_t P = s_P[c - c0];  // the block's first payload bit
        const uint64_t G = s_G[c - c0];  // this chunk's first bit
        const uint64_t W0 = G >> 5;
        const uint32_t sh0 = (uint32_t)(G & 31u);
        const uint32_t *vw = &v4.x;
        // the thread's code word k (0 past the chunk's end)
        auto code = [&](uint32_t k) -> uint64_t { return k < nsym ? s_tab[(vw[k >> 2] >> (8 * (k & 3))) & 255u] : 0ull; };
        uint32_t mybits = 0;  // a chunk holds at most 4096 * 56 bits
        uint32_t hw[kPackIPT], ll[kPackIPT];  // code words' high halves; lengths
#pragma unroll
        for (uint32_t k = 0; k < kPackIPT; ++k) {
            const uint64_t ek = code(k);
            hw[k] = (uint32_t)(ek >> 32);
            ll[k] = (uint32_t)ek & 255u;
            mybits += ll[k];
        }
        uint32_t total32;
        const uint32_t tb = block_excl_sum1<256>(mybits, s_tmp, &total32) + sh0;  // bit offset from W0 * 32
        // the block's last chunk also owns the zero pad bits up to the payload's last byte
        // (at least one byte: encode_with_huffman starts from one zero byte, main.cpp:162)
        const bool last = s_last[c - c0] != 0;
        uint64_t own_end = G + total32;
        if (last) {
            const uint64_t bbits = s_cb[c - c0] + total32;
            const uint64_t pb = (bbits + 7) / 8;
            own_end = P + 8 * (pb ? pb : 1);
        }
        const uint32_t nwords = own_end == G ? 0u : (uint32_t)((own_end - W0 * 32 + 31) >> 5);
        for (uint32_t wb = 0; wb < nwords; wb += kPackImgWords) {
            const uint32_t nw = min(kPackImgWords, nwords - wb);
            // this thread's bits [tb, tb + mybits) accumulated MSB-first in 64 bits and OR'd into
            // the image a word at a time (the first and last words may be shared with the
            // neighbouring threads); words outside the window are dropped
            if (mybits && (tb >> 5) < wb + nw && ((tb + mybits + 31) >> 5) > wb) {
                uint32_t w = tb >> 5, nacc = tb & 31u, hi = 0, lo = 0;
                if (short16 && nwords <= kPackImgWords) {
                    // one window (wb = 0); two words of <= 16 bits joined per push (padding words
                    // are empty: no bits)
#pragma unroll
                    for (uint32_t k = 0; k < kPackIPT; k += 2)
                        pack_push<false>(hw[k] | (hw[k + 1] >> ll[k]), ll[k] + ll[k + 1], hi, lo, nacc, w, s_img, 0u, nw);
                } else if (!long32 && nwords <= kPackImgWords) {
                    // one window, one push per symbol
#pragma unroll
                    for (uint32_t k = 0; k < kPackIPT; ++k) pack_push<false>(hw[k], ll[k], hi, lo, nacc, w, s_img, 0u, nw);
                } else {
#pragma unroll
                    for (uint32_t k = 0; k < kPackIPT; ++k) {
                        const uint64_t ek = code(k);
                        const uint32_t l = (uint32_t)ek & 255u;
                        pack_push<true>((uint32_t)(ek >> 32), min(l, 32u), hi, lo, nacc, w, s_img, wb, nw);
                        if (l > 32) pack_push<true>((uint32_t)ek & ~255u, l - 32, hi, lo, nacc, w, s_img, wb, nw);
                    }
                }
                if (nacc && w - wb < nw) atomicOr(&s_img[img_at(w - wb)], hi);
            }
            __syncthreads();
            // words wholly inside [G, own_end) are stored; the edge words are shared with the
            // neighbouring chunks / record headers: only this chunk's bits are replaced,
            // atomically. Each word is zeroed as it is drained (the next window starts clean).
            uint32_t *ob = out + (W0 + wb);
            for (uint32_t w = t; w < nw; w += 256) {
                const uint32_t slot = img_at(w), v = __builtin_bswap32(s_img[slot]);
                s_img[slot] = 0;
                if (wb + w != 0 && wb + w + 1 != nwords) {  // interior words: whole
                    ob[w] = v;
                    continue;
                }
                const uint64_t ws = (W0 + wb + w) * 32;
                const uint32_t a = G > ws ? (uint32_t)(G - ws) : 0u;
                const uint32_t e2 = own_end < ws + 32 ? (uint32_t)(own_end - ws) : 32u;
                if (a == 0 && e2 == 32) {
                    ob[w] = v;
                } else {
                    const uint32_t m = __builtin_bswap32((0xffffffffu >> a) & (0xffffffffu << (32 - e2)));
                    atomicAnd(&ob[w], ~m);
                    atomicOr(&ob[w], v & m);
                }
            }
            __syncthreads();
        }
        if (nwords == 0) __syncthreads();  // s_tmp / s_tab reuse by the next chunk
        ch = nx;
        v4 = nv4;
    }
}

// Standalone histogram + first occurrence (huffman() main.cpp:231-244) for any byte stream.
__global__ __launch_bounds__(256) void k_histogram(const uint8_t *__restrict__ in, const PChunk *__restrict__ chunks,
                                                   const uint64_t *__restrict__ boffs, uint32_t *__restrict__ freq,
                                                   uint32_t *__restrict__ first)
{
    __shared__ uint32_t h[256], f[256];
    const PChunk ch = chunks[blockIdx.x];
    h[threadIdx.x] = 0;
    f[threadIdx.x] = 0xffffffffu;
    __syncthreads();
    const uint32_t rel0 = (uint32_t)(ch.start - boffs[ch.block]);
    for (uint32_t i = threadIdx.x; i < ch.len; i += 256) {
        const uint32_t v = in[ch.start + i];
        atomicAdd(&h[v], 1u);
        atomicMin(&f[v], rel0 + i);
    }
    __syncthreads();
    if (h[threadIdx.x]) {
        atomicAdd(&freq[(size_t)ch.block * 256 + threadIdx.x], h[threadIdx.x]);
        atomicMin(&first[(size_t)ch.block * 256 + threadIdx.x], f[threadIdx.x]);
    }
}

__global__ void k_fill(uint32_t *p, uint32_t v, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace

void histogram_batch(Ctx *c, const uint8_t *d_in, const Batch &bt, uint32_t *h_freq32, uint32_t *h_first32)
{
    const uint32_t nb = bt.nblocks;
    std::vector<PChunk> hc;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint64_t o = bt.offs[b], n = bt.offs[b + 1] - o;
        for (uint64_t s = 0; s < n; s += 65536) {
            PChunk p;
            p.block = b;
            p.start = (uint32_t)(o + s);
            p.len = (uint32_t)std::min<uint64_t>(65536, n - s);
            p.pad = 0;
            hc.push_back(p);
        }
    }
    const uint32_t nch = (uint32_t)hc.size();
    uint8_t *d_meta = (uint8_t *)c->get(WS_PACK_CHUNKS, nch * sizeof(PChunk) + (nb + 1) * 8 + 64);
    c->ws_tag[WS_PACK_CHUNKS] = 0;  // the pack's cached table is overwritten
    PChunk *d_chunks = (PChunk *)d_meta;
    uint64_t *d_offs = (uint64_t *)(d_meta + ((nch * sizeof(PChunk) + 15) & ~(size_t)15));
    uint32_t *d_freq = (uint32_t *)c->get(WS_FREQ, (size_t)nb * 256 * 4);
    uint32_t *d_first = (uint32_t *)c->get(WS_FIRST, (size_t)nb * 256 * 4);
    c->h2d(d_chunks, hc.data(), nch * sizeof(PChunk));
    c->h2d(d_offs, bt.offs.data(), (nb + 1) * 8);
    BMH_HIP(hipMemsetAsync(d_freq, 0, (size_t)nb * 256 * 4, c->stream));
    BMH_LAUNCH(c, "hist_fill", k_fill, (uint32_t)(((size_t)nb * 256 + 255) / 256), 256, 0, d_first, 0xffffffffu,
               (size_t)nb * 256);
    BMH_LAUNCH(c, "histogram", k_histogram, nch, 256, 0, d_in, d_chunks, d_offs, d_freq, d_first);
    c->d2h(h_freq32, d_freq, (size_t)nb * 256 * 4);
    c->d2h(h_first32, d_first, (size_t)nb * 256 * 4);
    c->sync();
}

namespace {
struct PackLayout {
    const PChunk *chunks;
    const uint32_t *cfirst;
    uint32_t nch;
};

// chunk table: rebuilt and uploaded only when the batch layout changed
PackLayout pack_layout(Ctx *c, const Batch &bt)
{
    const uint32_t nb = bt.nblocks;
    const uint64_t sig = layout_sig(3, bt.offs, 0);
    uint32_t nch;
    if (c->ws_tag[WS_PACK_CHUNKS] == sig) {
        nch = c->ws_aux[WS_PACK_CHUNKS][0];
    } else {
        std::vector<PChunk> hc;
        std::vector<uint32_t> cfirst(nb + 1);
        for (uint32_t b = 0; b < nb; ++b) {
            cfirst[b] = (uint32_t)hc.size();
            const uint64_t o = bt.offs[b], n = bt.offs[b + 1] - o;
            for (uint64_t s = 0; s < n; s += kPackChunk) {
                PChunk p;
                p.block = b;
                p.start = (uint32_t)(o + s);
                p.len = (uint32_t)std::min<uint64_t>(kPackChunk, n - s);
                p.pad = 0;
                hc.push_back(p);
            }
        }
        cfirst[nb] = (uint32_t)hc.size();
        nch = (uint32_t)hc.size();
        uint8_t *d_meta = (uint8_t *)c->get(WS_PACK_CHUNKS, nch * sizeof(PChunk) + (nb + 1) * 4 + 64);
        c->h2d(d_meta, hc.data(), nch * sizeof(PChunk));
        c->h2d(d_meta + nch * sizeof(PChunk), cfirst.data(), (nb + 1) * 4);
        c->ws_tag[WS_PACK_CHUNKS] = sig;
        c->ws_aux[WS_PACK_CHUNKS][0] = nch;
    }
    const uint8_t *d_meta = (const uint8_t *)c->ws[WS_PACK_CHUNKS];
    return PackLayout{(const PChunk *)d_meta, (const uint32_t *)(d_meta + nch * sizeof(PChunk)), nch};
}

// chunk bit counts, then their per-block exclusive scan (block totals into d_btot if non-null)
uint64_t *pack_bits_scan(Ctx *c, const uint8_t *d_mtf, const Batch &bt, const PackLayout &pl, const DevTable *d_tabs,
                         const uint16_t *d_chist, uint64_t *d_btot)
{
    uint64_t *d_cbits = (uint64_t *)c->get(WS_PACK_BITS, (size_t)pl.nch * 8);
    if (d_chist)
        BMH_LAUNCH(c, "pack_bits", k_pack_bits_hist, cdiv(pl.nch, 4 * kBitsCPW), 256, 0, d_chist, pl.chunks, pl.nch, d_tabs,
                   d_cbits);
    else
        BMH_LAUNCH(c, "pack_bits", k_pack_bits, pl.nch, 256, 0, d_mtf, pl.chunks, d_tabs, d_cbits);
    BMH_LAUNCH(c, "pack_scan", k_pack_scan, bt.nblocks, 256, 0, pl.cfirst, d_cbits, d_btot);
    return d_cbits;
}
}  // namespace

void pack_batch_dev(Ctx *c, const uint8_t *d_mtf, const Batch &bt, const DevTable *d_tabs, const uint64_t *d_pay_offs,
                    uint8_t *d_out, const uint32_t *d_status, const uint16_t *d_chist)
{
    if (((uintptr_t)d_out & 3u) != 0) fail(BMH_EINVAL, "pack: output buffer must be 4-byte aligned");
    const PackLayout pl = pack_layout(c, bt);
    const uint64_t *d_cbits = pack_bits_scan(c, d_mtf, bt, pl, d_tabs, d_chist, nullptr);
    const uint32_t cpw = pack_cpw(c, pl.nch);
    BMH_LAUNCH(c, "pack_write", k_pack_write, cdiv(pl.nch, cpw), 256, 0, d_mtf, pl.chunks, pl.nch, d_tabs, d_cbits,
               d_pay_offs, pl.cfirst, (uint32_t *)d_out, d_status, cpw);
}

// The standalone stage (bmh_pack_dev): payload sizes first (one wait), checked against the
// caller's buffer, then the write. The write touches whole 4-byte words (edge words under a mask),
// so every payload's word-rounded extent must lie inside [d_out, d_out + out_cap).
void pack_batch(Ctx *c, const uint8_t *d_mtf, const Batch &bt, const bmh_code_table *tables, uint8_t *d_out,
                uint64_t out_cap, const uint64_t *pay_offs, uint64_t *out_bytes)
{
    if (((uintptr_t)d_out & 3u) != 0) fail(BMH_EINVAL, "pack: output buffer must be 4-byte aligned");
    const uint32_t nb = bt.nblocks;
    std::vector<DevTable> ht(nb);
    for (uint32_t b = 0; b < nb; ++b) {
        memcpy(ht[b].code, tables[b].code, sizeof ht[b].code);
        memcpy(ht[b].len, tables[b].len, sizeof ht[b].len);
        for (int s = 0; s < 256; ++s)
            if (tables[b].len[s] > 64) fail(BMH_ERANGE, "pack: code longer than 64 bits");
    }
    DevTable *d_tab = (DevTable *)c->get(WS_TABLES, nb * sizeof(DevTable));
    uint64_t *d_pay = (uint64_t *)c->get(WS_ROFFS, (size_t)(2 * nb + 1) * 8 + 64);
    uint64_t *d_btot = d_pay + nb;
    c->h2d(d_tab, ht.data(), nb * sizeof(DevTable));
    const PackLayout pl = pack_layout(c, bt);
    const uint64_t *d_cbits = pack_bits_scan(c, d_mtf, bt, pl, d_tab, nullptr, d_btot);
    std::vector<uint64_t> bits(nb), bytes(nb), po(nb);
    c->d2h(bits.data(), d_btot, nb * 8);
    c->sync();
    uint64_t next = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        bytes[b] = std::max<uint64_t>(1, (bits[b] + 7) / 8);  // encode_with_huffman's one zero byte, main.cpp:162
        po[b] = pay_offs ? pay_offs[b] : next;
        next = po[b] + bytes[b];
        if (po[b] > out_cap || bytes[b] > out_cap - po[b] || ((po[b] + bytes[b] + 3) & ~(uint64_t)3) > out_cap)
            fail(BMH_ERANGE, "pack: payload of block " + std::to_string(b) + " (" + std::to_string(bytes[b]) +
                                 " B at " + std::to_string(po[b]) + ") does not fit out_cap " + std::to_string(out_cap) +
                                 " (whole 4-byte words)");
    }
    if (pay_offs) {  // payloads must not overlap (edge words are shared under a mask, bytes are not)
        std::vector<uint32_t> ord(nb);
        for (uint32_t b = 0; b < nb; ++b) ord[b] = b;
        std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return po[x] < po[y]; });
        for (uint32_t i = 1; i < nb; ++i)
            if (po[ord[i - 1]] + bytes[ord[i - 1]] > po[ord[i]])
                fail(BMH_EINVAL, "pack: payloads of blocks " + std::to_string(ord[i - 1]) + " and " +
                                     std::to_string(ord[i]) + " overlap");
    }
    c->h2d(d_pay, po.data(), nb * 8);
    const uint32_t cpw = pack_cpw(c, pl.nch);
    BMH_LAUNCH(c, "pack_write", k_pack_write, cdiv(pl.nch, cpw), 256, 0, d_mtf, pl.chunks, pl.nch, d_tab, d_cbits,
               d_pay, pl.cfirst, (uint32_t *)d_out, nullptr, cpw);
    c->sync();
    if (out_bytes) memcpy(out_bytes, bytes.data(), nb * 8);
}

}  // namespace bmh
