// bwt.hip — cyclic-rotation BWT of a batch of blocks on gfx950.
//
// Replaces bwt() + bwt_cmp_straight + cyclic_index (reference main.cpp:38-59, 77-91), which
// std::stable_sort's rotation indices with an O(LCP) byte comparator. Here the same order is
// built by prefix doubling on cyclic ranks:
//
//   rank_D[p] = number of rotations whose first D bytes are strictly smaller than those of
//   rotation p ("group start"). Sorting a depth-D group by rank_D[(p + D) mod n] yields
//   depth 2D. Identical rotations never split; they stop once D >= n (their L bytes are
//   equal, and the primary index is rank[0] = count of strictly smaller rotations, exactly
//   the row std::stable_sort gives rotation 0).
//
// Rounds over the whole batch (all blocks progress together, one segment list):
//   bucket  : LDS-histogram counting sort of every position by its first 2 bytes   -> D = 2
//   round 1 : every bucket of >= 2 positions sorted by the next 4 data bytes       -> D = 6
//   round r : every unresolved group sorted by rank_D[(p+D) mod n]                  -> D = 2D
// Segments are sorted by size class: tiny (<= 128: packed into ~1K-element tiles, rank by
// counting in LDS), medium (<= 4096: one workgroup, LDS LSD radix), large (global MSD radix
// passes, 8 bits each, splitting into sub-segments that re-enter the classes).
//
// Rank arrays are double buffered (rk_cur read, rk_nxt written) so that keys gathered inside
// the sort kernels never see this round's updates; elements that resolve in round >= 2 are
// committed to both arrays after the round (resolved list).
#include "bmh_internal.h"
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

constexpr uint32_t kHistChunk = 4u << 20;   // positions per bucket-histogram chunk
constexpr uint32_t kHalfBins = 32768;       // 16-bit digit space split in two LDS halves
constexpr uint32_t kTinyMax = 128;
constexpr uint32_t kTileT = 1024;
constexpr uint32_t kTileCap = kTileT + kTinyMax;  // 1152
constexpr uint32_t kTileSegMax = kTileCap / 2;
constexpr uint32_t kMedMax = 4096;
constexpr uint32_t kLargeTile = 4096;

struct Counters {
    uint32_t tiny, med, large, large_next, groups, next, tiles, resolved;
};

struct LSeg {
    uint32_t gstart, len, shift, gathered;
};
struct LTile {
    uint32_t seg, start, len, pad;
};

struct RoundArgs {
    const uint8_t *data;
    const uint32_t *boffs;
    uint32_t nb;
    uint32_t *sa;
    const uint32_t *rk_cur;
    uint32_t *rk_nxt;
    uint32_t *rkA, *rkB;
    uint32_t D;          // current depth (key = rank_D at p + D) — unused in round 1
    uint64_t newD;       // depth reached by this round
    int round1;          // key = 4 data bytes at p+2 (D = 2 -> 6)
    uint2 *next;
    uint32_t *resolved;  // round >= 2: positions resolved this round (global slot of p)
    Counters *cnt;
};

__device__ __forceinline__ uint32_t key_data4(const uint8_t *__restrict__ blk, uint32_t n, uint32_t p)
{
    if ((uint64_t)p + 5 < n) {
        return ((uint32_t)blk[p + 2] << 24) | ((uint32_t)blk[p + 3] << 16) | ((uint32_t)blk[p + 4] << 8) |
               (uint32_t)blk[p + 5];
    }
    uint32_t k = 0;
    for (int i = 0; i < 4; ++i) k = (k << 8) | blk[(uint32_t)(((uint64_t)p + 2 + i) % n)];
    return k;
}

__device__ __forceinline__ uint32_t round_key(const RoundArgs &a, uint32_t boff, uint32_t n, uint32_t p)
{
    if (a.round1) return key_data4(a.data + boff, n, p);
    uint64_t q = (uint64_t)p + (a.D % n);
    if (q >= n) q -= n;
    return a.rk_cur[boff + (uint32_t)q];
}

// Rank bookkeeping for element p (block-local) of a depth-newD group starting at block-local
// slot gs with gsz members; `first` marks one member per group (emits it for the next round).
__device__ __forceinline__ void finish(const RoundArgs &a, uint32_t boff, uint32_t n, uint32_t p, uint32_t gs,
                                       uint32_t gsz, bool first)
{
    const bool final_ = gsz == 1 || a.newD >= n;
    if (final_) {
        if (a.round1) {
            a.rkA[boff + p] = gs;
            a.rkB[boff + p] = gs;
        } else {
            a.rk_nxt[boff + p] = gs;
            uint32_t i = atomicAdd(&a.cnt->resolved, 1u);
            a.resolved[i] = boff + p;
        }
    } else {
        a.rk_nxt[boff + p] = gs;
        if (first) {
            uint32_t i = atomicAdd(&a.cnt->next, 1u);
            a.next[i] = make_uint2(boff + gs, gsz);
        }
    }
}

// ------------------------------------------------------------------ bucket round (D = 2)
__device__ __forceinline__ uint32_t digit16(const uint8_t *__restrict__ blk, uint32_t n, uint32_t p)
{
    uint32_t q = p + 1 == n ? 0 : p + 1;
    return ((uint32_t)blk[p] << 8) | blk[q];
}

// grid = chunks*2 (chunk, half); 1024 threads; dynamic LDS = 32768 u32 counters.
__global__ __launch_bounds__(1024) void k_bucket_hist(const uint8_t *__restrict__ data,
                                                      const BlockInfo *__restrict__ blocks,
                                                      const uint32_t *__restrict__ chunk_block,
                                                      const uint32_t *__restrict__ chunk_first,
                                                      uint32_t *__restrict__ chist)
{
    extern __shared__ uint32_t cnt[];
    const uint32_t chunk = blockIdx.x >> 1, half = blockIdx.x & 1;
    const uint32_t b = chunk_block[chunk];
    const BlockInfo bi = blocks[b];
    const uint32_t c = chunk - chunk_first[b];
    const uint32_t p0 = c * kHistChunk;
    const uint32_t p1 = min(p0 + kHistChunk, bi.n);
    for (uint32_t i = threadIdx.x; i < kHalfBins; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint8_t *blk = data + bi.off;
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        uint32_t d = digit16(blk, bi.n, p);
        if ((d >> 15) == half) atomicAdd(&cnt[d & (kHalfBins - 1)], 1u);
    }
    __syncthreads();
    uint32_t *out = chist + (size_t)blockIdx.x * kHalfBins;
    for (uint32_t i = threadIdx.x; i < kHalfBins; i += blockDim.x) out[i] = cnt[i];
}

// grid = nblocks; 1024 threads. Bucket totals -> starts (bstart[b][0..65536]); per-chunk
// histograms become per-chunk write offsets; buckets of >= 2 positions become segments.
__global__ __launch_bounds__(1024) void k_bucket_scan(const BlockInfo *__restrict__ blocks,
                                                      const uint32_t *__restrict__ chunk_first,
                                                      uint32_t *__restrict__ chist, uint32_t *__restrict__ bstart,
                                                      uint2 *__restrict__ segs, Counters *cnt)
{
    __shared__ uint32_t s_tmp[17];
    const uint32_t b = blockIdx.x;
    const BlockInfo bi = blocks[b];
    const uint32_t c0 = chunk_first[b], nc = chunk_first[b + 1] - c0;
    uint32_t carry = 0;
    uint32_t *bs = bstart + (size_t)b * 65537;
    for (uint32_t r = 0; r < 64; ++r) {
        const uint32_t d = r * 1024 + threadIdx.x;
        const uint32_t half = d >> 15, idx = d & (kHalfBins - 1);
        uint32_t tot = 0;
        for (uint32_t c = 0; c < nc; ++c) tot += chist[((size_t)(c0 + c) * 2 + half) * kHalfBins + idx];
        uint32_t total;
        uint32_t ex = block_excl_sum<1024>(tot, s_tmp, &total);
        const uint32_t start = carry + ex;
        bs[d] = start;
        uint32_t acc = start;
        for (uint32_t c = 0; c < nc; ++c) {
            uint32_t *h = &chist[((size_t)(c0 + c) * 2 + half) * kHalfBins + idx];
            uint32_t v = *h;
            *h = acc;
            acc += v;
        }
        if (tot >= 2 && bi.n > 2) {
            uint32_t i = atomicAdd(&cnt->next, 1u);
            segs[i] = make_uint2(bi.off + start, tot);
        }
        carry += total;
    }
    if (threadIdx.x == 0) bs[65536] = bi.n;
}

__global__ __launch_bounds__(1024) void k_bucket_scatter(const uint8_t *__restrict__ data,
                                                         const BlockInfo *__restrict__ blocks,
                                                         const uint32_t *__restrict__ chunk_block,
                                                         const uint32_t *__restrict__ chunk_first,
                                                         const uint32_t *__restrict__ chist,
                                                         const uint32_t *__restrict__ bstart, uint32_t *__restrict__ sa,
                                                         uint32_t *__restrict__ rkA, uint32_t *__restrict__ rkB)
{
    extern __shared__ uint32_t cur[];
    const uint32_t chunk = blockIdx.x >> 1, half = blockIdx.x & 1;
    const uint32_t b = chunk_block[chunk];
    const BlockInfo bi = blocks[b];
    const uint32_t c = chunk - chunk_first[b];
    const uint32_t p0 = c * kHistChunk;
    const uint32_t p1 = min(p0 + kHistChunk, bi.n);
    const uint32_t *in = chist + (size_t)blockIdx.x * kHalfBins;
    for (uint32_t i = threadIdx.x; i < kHalfBins; i += blockDim.x) cur[i] = in[i];
    __syncthreads();
    const uint8_t *blk = data + bi.off;
    const uint32_t *bs = bstart + (size_t)b * 65537;
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
        uint32_t d = digit16(blk, bi.n, p);
        if ((d >> 15) != half) continue;
        uint32_t slot = atomicAdd(&cur[d & (kHalfBins - 1)], 1u);
        sa[bi.off + slot] = p;
        uint32_t st = bs[d];
        if (bs[d + 1] - st == 1 || bi.n <= 2) {  // resolved (or final: D = 2 >= n)
            rkA[bi.off + p] = st;
            rkB[bi.off + p] = st;
        }
    }
}

// ------------------------------------------------------------------------- classification
__global__ void k_classify(const uint2 *__restrict__ segs, uint32_t nseg, uint2 *__restrict__ tiny,
                           uint2 *__restrict__ med, LSeg *__restrict__ large, Counters *cnt)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    const uint2 s = segs[i];
    if (s.y <= kTinyMax) {
        tiny[atomicAdd(&cnt->tiny, 1u)] = s;
    } else if (s.y <= kMedMax) {
        med[atomicAdd(&cnt->med, 1u)] = s;
    } else {
        LSeg l;
        l.gstart = s.x;
        l.len = s.y;
        l.shift = 24;
        l.gathered = 0;
        large[atomicAdd(&cnt->large, 1u)] = l;
    }
}

// ---------------------------------------------------------------- device-wide exclusive scan
constexpr uint32_t kScanItems = 4096;  // per workgroup (1024 threads x 4)

__global__ __launch_bounds__(1024) void k_scan_reduce(const uint32_t *__restrict__ in, uint32_t stride, uint32_t count,
                                                      uint32_t *__restrict__ partials)
{
    __shared__ uint32_t s_tmp[17];
    const uint32_t base = blockIdx.x * kScanItems + threadIdx.x * 4;
    uint32_t s = 0;
    for (int i = 0; i < 4; ++i)
        if (base + i < count) s += in[(size_t)(base + i) * stride];
    uint32_t total;
    block_excl_sum<1024>(s, s_tmp, &total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_partials(uint32_t *__restrict__ partials, uint32_t n)
{
    __shared__ uint32_t s_tmp[17];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < n; base += 1024) {
        uint32_t i = base + threadIdx.x;
        uint32_t v = i < n ? partials[i] : 0u;
        uint32_t total;
        uint32_t ex = block_excl_sum<1024>(v, s_tmp, &total);
        if (i < n) partials[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(1024) void k_scan_down(const uint32_t *__restrict__ in, uint32_t stride, uint32_t count,
                                                    const uint32_t *__restrict__ partials, uint32_t *__restrict__ out)
{
    __shared__ uint32_t s_tmp[17];
    const uint32_t base = blockIdx.x * kScanItems + threadIdx.x * 4;
    uint32_t v[4], s = 0;
    for (int i = 0; i < 4; ++i) {
        v[i] = base + i < count ? in[(size_t)(base + i) * stride] : 0u;
        s += v[i];
    }
    uint32_t ex = block_excl_sum<1024>(s, s_tmp, nullptr) + partials[blockIdx.x];
    for (int i = 0; i < 4; ++i) {
        if (base + i < count) out[base + i] = ex;
        ex += v[i];
    }
}

__global__ void k_tile_heads(const uint32_t *__restrict__ prefix, uint32_t n, uint32_t *__restrict__ tiles,
                             Counters *cnt)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = prefix[i] / kTileT;
    if (i == 0 || prefix[i - 1] / kTileT != t) tiles[atomicAdd(&cnt->tiles, 1u)] = i;
}

// ------------------------------------------------------------------------------ tiny tiles
// One workgroup per tile of consecutive tiny segments (<= 1152 elements). Each element's new
// slot = segment start + #(keys < mine) + #(equal keys before me); group = equal keys.
__global__ __launch_bounds__(256) void k_tiny(RoundArgs a, const uint2 *__restrict__ tiny, uint32_t ntiny,
                                              const uint32_t *__restrict__ prefix, const uint32_t *__restrict__ tiles)
{
    __shared__ uint32_t s_key[kTileCap], s_pos[kTileCap];
    __shared__ uint16_t s_seg[kTileCap];
    __shared__ uint32_t s_gstart[kTileSegMax], s_lstart[kTileSegMax], s_len[kTileSegMax], s_boff[kTileSegMax],
        s_n[kTileSegMax];
    const uint32_t head = tiles[blockIdx.x];
    const uint32_t base = prefix[head];
    const uint32_t t = base / kTileT;
    uint32_t nseg = 0;
    for (uint32_t w = 0;; w += 256) {
        const uint32_t i = head + w + threadIdx.x;
        const bool in = i < ntiny && prefix[i] / kTileT == t;
        const uint32_t c = __syncthreads_count(in);
        nseg += c;
        if (c < 256) break;
    }
    for (uint32_t k = threadIdx.x; k < nseg; k += 256) {
        const uint2 s = tiny[head + k];
        const uint32_t b = find_block(a.boffs, a.nb, s.x);
        s_gstart[k] = s.x;
        s_len[k] = s.y;
        s_lstart[k] = prefix[head + k] - base;
        s_boff[k] = a.boffs[b];
        s_n[k] = a.boffs[b + 1] - a.boffs[b];
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nseg; k += 256)
        for (uint32_t e = s_lstart[k], e1 = e + s_len[k]; e < e1; ++e) s_seg[e] = (uint16_t)k;
    const uint32_t total = s_lstart[nseg - 1] + s_len[nseg - 1];
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < total; e += 256) {
        const uint32_t k = s_seg[e];
        const uint32_t p = a.sa[s_gstart[k] + (e - s_lstart[k])];
        s_pos[e] = p;
        s_key[e] = round_key(a, s_boff[k], s_n[k], p);
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < total; e += 256) {
        const uint32_t k = s_seg[e];
        const uint32_t l0 = s_lstart[k], m = s_len[k];
        const uint32_t ke = s_key[e];
        uint32_t lt = 0, eqb = 0, eqt = 0;
        for (uint32_t f = l0; f < l0 + m; ++f) {
            const uint32_t kf = s_key[f];
            lt += kf < ke;
            const bool eq = kf == ke;
            eqt += eq;
            eqb += eq && f < e;
        }
        const uint32_t p = s_pos[e];
        a.sa[s_gstart[k] + lt + eqb] = p;
        const uint32_t boff = s_boff[k];
        finish(a, boff, s_n[k], p, s_gstart[k] - boff + lt, eqt, eqb == 0);
    }
}

// ----------------------------------------------------------------------- medium segments
// One workgroup per segment of 129..4096 elements: LSD radix sort (4-bit digits, constant
// digits skipped) in LDS, then equal-key groups via block max / suffix-min scans.
constexpr int kMedNT = 256, kMedIPT = kMedMax / kMedNT;

__global__ __launch_bounds__(256) void k_medium(RoundArgs a, const uint2 *__restrict__ med)
{
    __shared__ uint32_t s_k[2][kMedMax], s_v[2][kMedMax];
    __shared__ uint16_t s_cnt[16 * kMedNT];
    __shared__ uint32_t s_tmp[8];
    __shared__ uint32_t s_or, s_and;
    const uint2 sg = med[blockIdx.x];
    const uint32_t b = find_block(a.boffs, a.nb, sg.x);
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint32_t m = sg.y;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        s_or = 0;
        s_and = 0xffffffffu;
    }
    __syncthreads();
    uint32_t vor = 0, vand = 0xffffffffu;
    for (uint32_t e = tid; e < m; e += kMedNT) {
        const uint32_t p = a.sa[sg.x + e];
        const uint32_t k = round_key(a, boff, n, p);
        s_k[0][e] = k;
        s_v[0][e] = p;
        vor |= k;
        vand &= k;
    }
    atomicOr(&s_or, vor);
    atomicAnd(&s_and, vand);
    __syncthreads();
    const uint32_t vary = s_or ^ s_and;
    int cur = 0;
    for (int sh = 0; sh < 32; sh += 4) {
        if (((vary >> sh) & 15u) == 0) continue;
        for (int d = 0; d < 16; ++d) s_cnt[d * kMedNT + tid] = 0;
        __syncthreads();
        for (int i = 0; i < kMedIPT; ++i) {
            const uint32_t idx = tid * kMedIPT + i;
            if (idx < m) {
                const uint32_t d = (s_k[cur][idx] >> sh) & 15u;
                s_cnt[d * kMedNT + tid]++;
            }
        }
        __syncthreads();
        uint32_t loc[16], s = 0;
        for (int i = 0; i < 16; ++i) {
            loc[i] = s_cnt[tid * 16 + i];
            s += loc[i];
        }
        uint32_t ex = block_excl_sum<kMedNT>(s, s_tmp, nullptr);
        for (int i = 0; i < 16; ++i) {
            s_cnt[tid * 16 + i] = (uint16_t)ex;
            ex += loc[i];
        }
        __syncthreads();
        for (int i = 0; i < kMedIPT; ++i) {
            const uint32_t idx = tid * kMedIPT + i;
            if (idx < m) {
                const uint32_t k = s_k[cur][idx];
                const uint32_t d = (k >> sh) & 15u;
                const uint32_t pos = s_cnt[d * kMedNT + tid]++;
                s_k[cur ^ 1][pos] = k;
                s_v[cur ^ 1][pos] = s_v[cur][idx];
            }
        }
        __syncthreads();
        cur ^= 1;
    }
    // groups: start = last head at or before e, end = first head after e
    uint32_t hmax = 0, hmin = m;
    for (int i = 0; i < kMedIPT; ++i) {
        const uint32_t e = tid * kMedIPT + i;
        if (e < m && (e == 0 || s_k[cur][e] != s_k[cur][e - 1])) {
            hmax = e;
            if (hmin == m) hmin = e;
        }
    }
    const uint32_t carry_s = block_excl_max<kMedNT>(hmax, s_tmp);
    const uint32_t carry_e = block_excl_min_rev<kMedNT>(hmin, m, s_tmp);
    uint32_t gsa[kMedIPT];
    uint32_t run = carry_s;
    for (int i = 0; i < kMedIPT; ++i) {
        const uint32_t e = tid * kMedIPT + i;
        if (e < m && (e == 0 || s_k[cur][e] != s_k[cur][e - 1])) run = e;
        gsa[i] = run;
    }
    uint32_t nxt = carry_e;
    for (int i = kMedIPT - 1; i >= 0; --i) {
        const uint32_t e = tid * kMedIPT + i;
        if (e >= m) continue;
        const uint32_t gs = gsa[i], gz = nxt - gs;
        const uint32_t p = s_v[cur][e];
        a.sa[sg.x + e] = p;
        finish(a, boff, n, p, sg.x - boff + gs, gz, e == gs);
        if (e == gs) nxt = e;
    }
}

// ------------------------------------------------------------------------ large segments
__global__ __launch_bounds__(256) void k_lhist(RoundArgs a, const LSeg *__restrict__ lsegs,
                                               const LTile *__restrict__ tiles, uint32_t *__restrict__ key,
                                               uint32_t *__restrict__ thist)
{
    __shared__ uint32_t h[256];
    const LTile t = tiles[blockIdx.x];
    const LSeg s = lsegs[t.seg];
    const uint32_t b = find_block(a.boffs, a.nb, s.gstart);
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < t.len; e += 256) {
        const uint32_t j = t.start + e;
        uint32_t k;
        if (s.gathered) {
            k = key[j];
        } else {
            k = round_key(a, boff, n, a.sa[j]);
            key[j] = k;
        }
        atomicAdd(&h[(k >> s.shift) & 255u], 1u);
    }
    __syncthreads();
    thist[(size_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

__device__ __forceinline__ void push_sub(uint32_t gstart, uint32_t len, uint32_t shift, uint2 *tiny, uint2 *med,
                                         LSeg *large_next, uint2 *groups, Counters *cnt)
{
    if (len == 1) {
        groups[atomicAdd(&cnt->groups, 1u)] = make_uint2(gstart, len);
    } else if (len <= kTinyMax) {
        tiny[atomicAdd(&cnt->tiny, 1u)] = make_uint2(gstart, len);
    } else if (len <= kMedMax) {
        med[atomicAdd(&cnt->med, 1u)] = make_uint2(gstart, len);
    } else if (shift > 0) {
        LSeg l;
        l.gstart = gstart;
        l.len = len;
        l.shift = shift - 8;
        l.gathered = 1;
        large_next[atomicAdd(&cnt->large_next, 1u)] = l;
    } else {
        groups[atomicAdd(&cnt->groups, 1u)] = make_uint2(gstart, len);  // keys exhausted: equal
    }
}

// grid = nlseg; 256 threads (= digits)
__global__ __launch_bounds__(256) void k_lscan(const LSeg *__restrict__ lsegs, const uint2 *__restrict__ segtiles,
                                               uint32_t *__restrict__ thist, uint32_t *__restrict__ nomove,
                                               uint2 *tiny, uint2 *med, LSeg *large_next, uint2 *groups, Counters *cnt)
{
    __shared__ uint32_t s_tmp[8];
    const LSeg s = lsegs[blockIdx.x];
    const uint2 tr = segtiles[blockIdx.x];
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
    for (uint32_t t = tr.x; t < tr.x + tr.y; ++t) {
        uint32_t v = thist[(size_t)t * 256 + d];
        thist[(size_t)t * 256 + d] = run;
        run += v;
    }
    const uint32_t tot = run;
    const int nz = __syncthreads_count(tot > 0);
    const uint32_t base = block_excl_sum<256>(tot, s_tmp, nullptr);
    for (uint32_t t = tr.x; t < tr.x + tr.y; ++t) thist[(size_t)t * 256 + d] += s.gstart + base;
    if (nz == 1) {
        if (d == 0) {
            nomove[blockIdx.x] = 1;
            push_sub(s.gstart, s.len, s.shift, tiny, med, large_next, groups, cnt);
        }
    } else {
        if (d == 0) nomove[blockIdx.x] = 0;
        if (tot > 0) push_sub(s.gstart + base, tot, s.shift, tiny, med, large_next, groups, cnt);
    }
}

__global__ __launch_bounds__(256) void k_lscatter(const LSeg *__restrict__ lsegs, const LTile *__restrict__ tiles,
                                                  const uint32_t *__restrict__ nomove, const uint32_t *__restrict__ thist,
                                                  const uint32_t *__restrict__ sa, const uint32_t *__restrict__ key,
                                                  uint32_t *__restrict__ sa2, uint32_t *__restrict__ key2)
{
    __shared__ uint32_t cur[256];
    const LTile t = tiles[blockIdx.x];
    if (nomove[t.seg]) return;
    const uint32_t shift = lsegs[t.seg].shift;
    cur[threadIdx.x] = thist[(size_t)blockIdx.x * 256 + threadIdx.x];
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < t.len; e += 256) {
        const uint32_t j = t.start + e;
        const uint32_t k = key[j];
        const uint32_t slot = atomicAdd(&cur[(k >> shift) & 255u], 1u);
        sa2[slot] = sa[j];
        key2[slot] = k;
    }
}

__global__ __launch_bounds__(256) void k_lcopy(const LTile *__restrict__ tiles, const uint32_t *__restrict__ nomove,
                                               uint32_t *__restrict__ sa, uint32_t *__restrict__ key,
                                               const uint32_t *__restrict__ sa2, const uint32_t *__restrict__ key2)
{
    const LTile t = tiles[blockIdx.x];
    if (nomove[t.seg]) return;
    for (uint32_t e = threadIdx.x; e < t.len; e += 256) {
        const uint32_t j = t.start + e;
        sa[j] = sa2[j];
        key[j] = key2[j];
    }
}

// Groups produced by the large path (singletons, or key-exhausted equal-key groups).
__global__ __launch_bounds__(256) void k_groups(RoundArgs a, const uint2 *__restrict__ groups, uint32_t ng)
{
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t l = threadIdx.x & 63u;
    for (uint32_t g = wave; g < ng; g += nwaves) {
        const uint2 s = groups[g];
        const uint32_t b = find_block(a.boffs, a.nb, s.x);
        const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
        for (uint32_t e = l; e < s.y; e += 64) finish(a, boff, n, a.sa[s.x + e], s.x - boff, s.y, e == 0);
    }
}

__global__ void k_commit(const uint32_t *__restrict__ list, uint32_t cnt, const uint32_t *__restrict__ src,
                         uint32_t *__restrict__ dst)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cnt) dst[list[i]] = src[list[i]];
}

// ------------------------------------------------------------------------------ outputs
// L[r] = data[(SA[r] + n - 1) mod n] (main.cpp:87); grid = (ceil(max_n / 4096), nblocks).
__global__ __launch_bounds__(256) void k_lastcol(const uint8_t *__restrict__ data, const BlockInfo *__restrict__ blocks,
                                                 const uint32_t *__restrict__ sa, uint8_t *__restrict__ L)
{
    const BlockInfo bi = blocks[blockIdx.y];
    const uint32_t j0 = blockIdx.x * 4096u;
    if (j0 >= bi.n) return;
    const uint32_t j1 = min(j0 + 4096u, bi.n);
    for (uint32_t j = j0 + threadIdx.x; j < j1; j += 256) {
        const uint32_t p = sa[bi.off + j];
        L[bi.off + j] = data[bi.off + (p == 0 ? bi.n - 1 : p - 1)];
    }
}

__global__ void k_primary(const BlockInfo *__restrict__ blocks, uint32_t nb, const uint32_t *__restrict__ rk,
                          uint32_t *__restrict__ prim)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) prim[b] = rk[blocks[b].off];  // rank of rotation 0 = #strictly smaller rotations
}

inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace

void bwt_batch(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_L, uint64_t *h_primary)
{
    const uint32_t nb = bt.nblocks;
    const uint64_t N = bt.total;
    if (N >= 0xffffffffull) fail(BMH_ERANGE, "bwt: batch must be < 4 GiB");

    // ---- batch tables
    std::vector<BlockInfo> hb(nb);
    std::vector<uint32_t> hoffs(nb + 1), chunk_first(nb + 1), chunk_block;
    for (uint32_t b = 0; b < nb; ++b) {
        hb[b].off = (uint32_t)bt.offs[b];
        hb[b].n = (uint32_t)(bt.offs[b + 1] - bt.offs[b]);
        hoffs[b] = hb[b].off;
        chunk_first[b] = (uint32_t)chunk_block.size();
        for (uint32_t k = 0; k < cdiv(hb[b].n, kHistChunk); ++k) chunk_block.push_back(b);
    }
    hoffs[nb] = (uint32_t)N;
    chunk_first[nb] = (uint32_t)chunk_block.size();
    const uint32_t nchunks = (uint32_t)chunk_block.size();

    // blocks | boffs | chunk_first | chunk_block packed in one upload
    const size_t tb_bytes = nb * sizeof(BlockInfo) + (nb + 1) * 4 * 2 + nchunks * 4;
    uint8_t *d_tab = (uint8_t *)c->get(WS_BLOCKS, tb_bytes + 64);
    {
        std::vector<uint8_t> h(tb_bytes);
        size_t o = 0;
        memcpy(&h[o], hb.data(), nb * sizeof(BlockInfo));
        o += nb * sizeof(BlockInfo);
        memcpy(&h[o], hoffs.data(), (nb + 1) * 4);
        o += (nb + 1) * 4;
        memcpy(&h[o], chunk_first.data(), (nb + 1) * 4);
        o += (nb + 1) * 4;
        memcpy(&h[o], chunk_block.data(), nchunks * 4);
        BMH_HIP(hipMemcpyAsync(d_tab, h.data(), tb_bytes, hipMemcpyHostToDevice, c->stream));
        c->sync();  // h goes out of scope
    }
    const BlockInfo *d_blocks = (const BlockInfo *)d_tab;
    const uint32_t *d_boffs = (const uint32_t *)(d_tab + nb * sizeof(BlockInfo));
    const uint32_t *d_cfirst = d_boffs + (nb + 1);
    const uint32_t *d_cblock = d_cfirst + (nb + 1);

    uint32_t *sa = (uint32_t *)c->get(WS_SA, N * 4);
    uint32_t *rkA = (uint32_t *)c->get(WS_RKA, N * 4);
    uint32_t *rkB = (uint32_t *)c->get(WS_RKB, N * 4);
    uint32_t *key = (uint32_t *)c->get(WS_KEY, N * 4);
    uint32_t *sa2 = (uint32_t *)c->get(WS_SA2, N * 4);
    uint32_t *key2 = (uint32_t *)c->get(WS_KEY2, N * 4);
    const size_t seg_cap = N / 2 + 2;
    uint2 *seg_cur = (uint2 *)c->get(WS_SEG_CUR, seg_cap * 8);
    uint2 *seg_nxt = (uint2 *)c->get(WS_SEG_NXT, seg_cap * 8);
    uint2 *tiny = (uint2 *)c->get(WS_TINY, seg_cap * 8);
    uint2 *med = (uint2 *)c->get(WS_MED, (N / (kTinyMax + 1) + 2) * 8);
    const size_t lcap = N / (kMedMax + 1) + 2;
    LSeg *large = (LSeg *)c->get(WS_LARGE, lcap * sizeof(LSeg));
    LSeg *large2 = (LSeg *)c->get(WS_LARGE2, lcap * sizeof(LSeg));
    uint2 *groups = (uint2 *)c->get(WS_GROUPS, (N + 2) * 8);
    uint32_t *prefix = (uint32_t *)c->get(WS_PREFIX, seg_cap * 4);
    uint32_t *partials = (uint32_t *)c->get(WS_SCAN_PART, (seg_cap / kScanItems + 2) * 4);
    uint32_t *tiles = (uint32_t *)c->get(WS_TILES, seg_cap * 4);
    uint32_t *resolved = (uint32_t *)c->get(WS_RESOLVED, N * 4);
    Counters *d_cnt = (Counters *)c->get(WS_COUNTERS, sizeof(Counters) + 64);
    uint32_t *chist = (uint32_t *)c->get(WS_CHIST, (size_t)nchunks * 2 * kHalfBins * 4);
    uint32_t *bstart = (uint32_t *)c->get(WS_BSTART, (size_t)nb * 65537 * 4);
    Counters *h_cnt = (Counters *)c->host_pinned(sizeof(Counters) + 4096);

    auto read_counters = [&]() {
        BMH_HIP(hipMemcpyAsync(h_cnt, d_cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
        c->sync();
    };

    // ---- bucket round: D = 2
    BMH_HIP(hipMemsetAsync(d_cnt, 0, sizeof(Counters), c->stream));
    BMH_LAUNCH(c, "bwt_bucket_hist", k_bucket_hist, nchunks * 2, 1024, kHalfBins * 4, d_in, d_blocks, d_cblock,
               d_cfirst, chist);
    BMH_LAUNCH(c, "bwt_bucket_scan", k_bucket_scan, nb, 1024, 0, d_blocks, d_cfirst, chist, bstart, seg_cur, d_cnt);
    BMH_LAUNCH(c, "bwt_bucket_scatter", k_bucket_scatter, nchunks * 2, 1024, kHalfBins * 4, d_in, d_blocks,
               d_cblock, d_cfirst, chist, bstart, sa, rkA, rkB);
    read_counters();
    uint32_t ncur = h_cnt->next;

    uint64_t D = 2;
    int round = 1;
    std::vector<LSeg> hl;
    std::vector<LTile> ht;
    std::vector<uint2> hst;
    while (ncur > 0) {
        RoundArgs a;
        a.data = d_in;
        a.boffs = d_boffs;
        a.nb = nb;
        a.sa = sa;
        const bool odd = (round & 1) != 0;
        a.rk_cur = odd ? rkB : rkA;  // round 1 reads nothing
        a.rk_nxt = odd ? rkA : rkB;
        a.rkA = rkA;
        a.rkB = rkB;
        a.D = (uint32_t)std::min<uint64_t>(D, 0xffffffffull);
        a.newD = round == 1 ? 6 : 2 * D;
        a.round1 = round == 1;
        a.next = seg_nxt;
        a.resolved = resolved;
        a.cnt = d_cnt;

        BMH_HIP(hipMemsetAsync(d_cnt, 0, sizeof(Counters), c->stream));
        BMH_LAUNCH(c, "bwt_classify", k_classify, cdiv(ncur, 256), 256, 0, seg_cur, ncur, tiny, med, large, d_cnt);
        read_counters();

        // ---- large segments: MSD radix passes until every piece is tiny/medium/group
        uint32_t nl = h_cnt->large;
        LSeg *lcur = large, *lnxt = large2;
        while (nl > 0) {
            hl.resize(nl);
            BMH_HIP(hipMemcpyAsync(hl.data(), lcur, nl * sizeof(LSeg), hipMemcpyDeviceToHost, c->stream));
            c->sync();
            ht.clear();
            hst.resize(nl);
            for (uint32_t s = 0; s < nl; ++s) {
                hst[s].x = (uint32_t)ht.size();
                for (uint32_t o = 0; o < hl[s].len; o += kLargeTile) {
                    LTile t;
                    t.seg = s;
                    t.start = hl[s].gstart + o;
                    t.len = std::min<uint32_t>(kLargeTile, hl[s].len - o);
                    t.pad = 0;
                    ht.push_back(t);
                }
                hst[s].y = (uint32_t)ht.size() - hst[s].x;
            }
            const uint32_t ntl = (uint32_t)ht.size();
            uint8_t *d_lt = (uint8_t *)c->get(WS_LTILES, ntl * sizeof(LTile) + nl * 8 + nl * 4 + 64);
            LTile *d_tiles = (LTile *)d_lt;
            uint2 *d_segtiles = (uint2 *)(d_lt + ntl * sizeof(LTile));
            uint32_t *d_nomove = (uint32_t *)(d_lt + ntl * sizeof(LTile) + nl * 8);
            BMH_HIP(hipMemcpyAsync(d_tiles, ht.data(), ntl * sizeof(LTile), hipMemcpyHostToDevice, c->stream));
            BMH_HIP(hipMemcpyAsync(d_segtiles, hst.data(), nl * 8, hipMemcpyHostToDevice, c->stream));
            uint32_t *thist = (uint32_t *)c->get(WS_LTHIST, (size_t)ntl * 256 * 4);
            BMH_HIP(hipMemsetAsync(&d_cnt->large_next, 0, 4, c->stream));
            BMH_LAUNCH(c, "bwt_lhist", k_lhist, ntl, 256, 0, a, lcur, d_tiles, key, thist);
            BMH_LAUNCH(c, "bwt_lscan", k_lscan, nl, 256, 0, lcur, d_segtiles, thist, d_nomove, tiny, med, lnxt,
                       groups, d_cnt);
            BMH_LAUNCH(c, "bwt_lscatter", k_lscatter, ntl, 256, 0, lcur, d_tiles, d_nomove, thist, sa, key, sa2,
                       key2);
            BMH_LAUNCH(c, "bwt_lcopy", k_lcopy, ntl, 256, 0, d_tiles, d_nomove, sa, key, sa2, key2);
            read_counters();
            nl = h_cnt->large_next;
            std::swap(lcur, lnxt);
        }

        // ---- tiny segments: pack into tiles, rank by counting
        const uint32_t ntiny = h_cnt->tiny;
        if (ntiny > 0) {
            const uint32_t nparts = cdiv(ntiny, kScanItems);
            BMH_LAUNCH(c, "bwt_scan_reduce", k_scan_reduce, nparts, 1024, 0, &tiny[0].y, 2u, ntiny, partials);
            BMH_LAUNCH(c, "bwt_scan_partials", k_scan_partials, 1, 1024, 0, partials, nparts);
            BMH_LAUNCH(c, "bwt_scan_down", k_scan_down, nparts, 1024, 0, &tiny[0].y, 2u, ntiny, partials, prefix);
            BMH_LAUNCH(c, "bwt_tile_heads", k_tile_heads, cdiv(ntiny, 256), 256, 0, prefix, ntiny, tiles, d_cnt);
            read_counters();
            BMH_LAUNCH(c, "bwt_tiny", k_tiny, h_cnt->tiles, 256, 0, a, tiny, ntiny, prefix, tiles);
        }
        if (h_cnt->med > 0) BMH_LAUNCH(c, "bwt_medium", k_medium, h_cnt->med, kMedNT, 0, a, med);
        if (h_cnt->groups > 0)
            BMH_LAUNCH(c, "bwt_groups", k_groups, std::min<uint32_t>(cdiv(h_cnt->groups, 4), 65536), 256, 0, a,
                       groups, h_cnt->groups);
        read_counters();
        if (round > 1 && h_cnt->resolved > 0)
            BMH_LAUNCH(c, "bwt_commit", k_commit, cdiv(h_cnt->resolved, 256), 256, 0, resolved, h_cnt->resolved,
                       a.rk_nxt, (uint32_t *)a.rk_cur);
        ncur = h_cnt->next;
        std::swap(seg_cur, seg_nxt);
        D = a.newD;
        ++round;
    }

    // ---- outputs
    BMH_LAUNCH(c, "bwt_lastcol", k_lastcol, dim3(cdiv(bt.max_n, 4096), nb), 256, 0, d_in, d_blocks, sa, d_L);
    uint32_t *d_prim = (uint32_t *)c->get(WS_PRIMARY, nb * 4 + 64);
    BMH_LAUNCH(c, "bwt_primary", k_primary, cdiv(nb, 256), 256, 0, d_blocks, nb, rkA, d_prim);
    uint32_t *h_prim = (uint32_t *)c->host_pinned(nb * 4 + 4096);
    BMH_HIP(hipMemcpyAsync(h_prim, d_prim, nb * 4, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    for (uint32_t b = 0; b < nb; ++b) h_primary[b] = h_prim[b];
}

}  // namespace bmh
