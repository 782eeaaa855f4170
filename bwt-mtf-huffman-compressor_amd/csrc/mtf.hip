// mtf.hip — move-to-front of a batch of BWT last columns, plus the Huffman histogram and
// first-occurrence scan of its output.
//
// Replaces move_to_front() (reference main.cpp:93-112: find_if + std::rotate over a 256-byte
// alphabet initialised 0..255) and the two O(n) scans at the top of huffman()
// (main.cpp:231-244). MTF is sequential per block, so each block is cut into 4 KiB chunks:
//   1. recency : per chunk, its distinct symbols ordered by last occurrence (most recent
//                first): LDS atomicMax of positions, a bitset of last-occurrence positions,
//                then a suffix popcount gives each symbol's rank.
//   2. compose : per block, one wave walks its chunks in order: state_{c+1} =
//                recency_c ++ (state_c minus recency_c); this is each chunk's start state.
//   3. encode  : ONE LANE PER CHUNK. The alphabet is kept as time stamps, not as a list:
//                tm[s] = slot of the last access of symbol s in a 512-slot window, and a slot
//                bit is set iff it is some symbol's last access (always 256 marks). The MTF
//                index of c is the number of marks above tm[c] (symbols used more recently),
//                counted in two levels: whole superwords above (4 byte counters in a VGPR),
//                words above inside c's superword (byte counters in LDS), bits above inside
//                c's word (one popcount). An access clears one mark and sets the next slot —
//                O(1) work instead of moving up to 255 list entries; the window is renumbered
//                every 256 symbols. Stamps are stored as a byte + an "accessed this epoch" bit
//                (288 B per lane), one-wave workgroups. (tools/microbench/mtf_variants.hip:
//                4.6 ms per GiB vs 28-40 ms for whole-wave list updates on MI355X.)
//   4. hist    : freq + first occurrence of each MTF value per block (LDS atomics).
#include "bmh_internal.h"
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

constexpr uint32_t kMtfChunk = 4096;  // symbols per lane (one chunk)
constexpr int kLanes = 64;            // lanes (chunks) per encode workgroup (one wave)
constexpr int kMtfGroup = 2;          // symbols per batched MTF step

struct MChunk {
    uint32_t block, start, len, rel;  // rel = start - block offset
};

// grid = chunks; 256 threads x 16 symbols. R[c][0..d) = distinct symbols, most recent last
// occurrence first.
__global__ __launch_bounds__(256) void k_mtf_recency(const uint8_t *__restrict__ L, const MChunk *__restrict__ chunks,
                                                     uint8_t *__restrict__ R, uint32_t *__restrict__ dcount)
{
    __shared__ int lastpos[256];
    __shared__ uint32_t bset[kMtfChunk / 32];
    __shared__ uint32_t s_tmp[8];
    const MChunk ch = chunks[blockIdx.x];
    const uint32_t t = threadIdx.x;
    lastpos[t] = -1;
    if (t < kMtfChunk / 32) bset[t] = 0;
    // this thread's 16 symbols (zero past the chunk), one vector load when aligned
    uint32_t sw[4] = {0, 0, 0, 0};
    const uint32_t e0 = 16 * t;
    const uint32_t nv = e0 < ch.len ? min(16u, ch.len - e0) : 0u;
    if (nv == 16 && ((ch.start + e0) & 15u) == 0) {
        const uint4 v = *(const uint4 *)(L + ch.start + e0);
        sw[0] = v.x;
        sw[1] = v.y;
        sw[2] = v.z;
        sw[3] = v.w;
    } else {
        for (uint32_t k = 0; k < nv; ++k) sw[k >> 2] |= (uint32_t)L[ch.start + e0 + k] << (8 * (k & 3));
    }
    __syncthreads();
    for (uint32_t k = 0; k < nv; ++k) atomicMax(&lastpos[(sw[k >> 2] >> (8 * (k & 3))) & 255u], (int)(e0 + k));
    __syncthreads();
    const int lp = lastpos[t];
    if (lp >= 0) atomicOr(&bset[lp >> 5], 1u << (lp & 31));
    const int d = __syncthreads_count(lp >= 0);
    // thread t owns positions [16t, 16t+16); ranks count set bits at higher positions
    const uint32_t v = (bset[t >> 1] >> (16 * (t & 1))) & 0xffffu;
    const uint32_t cnt = __builtin_popcount(v);
    uint32_t total;
    const uint32_t ex = block_excl_sum<256>(cnt, s_tmp, &total);  // set bits in threads < t
    uint32_t off = total - ex - cnt;                               // set bits in threads > t
    uint8_t *Rc = R + (size_t)blockIdx.x * 256;
    for (int b = 15; b >= 0; --b)
        if (v & (1u << b)) Rc[off++] = (uint8_t)(sw[b >> 2] >> (8 * (b & 3)));
    if (t == 0) dcount[blockIdx.x] = (uint32_t)d;
}

// grid = nblocks, one wave each: sequential composition of the chunk recency lists. The
// recency lists (256 B per chunk) are fetched 32 chunks ahead into registers and parked in
// LDS, so the sequential chain never waits on global memory.
constexpr uint32_t kComposeBatch = 32;

__global__ __launch_bounds__(64) void k_mtf_compose(const uint32_t *__restrict__ chunk_first,
                                                    const uint8_t *__restrict__ R, const uint32_t *__restrict__ dcount,
                                                    uint32_t *__restrict__ S)
{
    __shared__ uint32_t s_R[kComposeBatch][64];
    __shared__ uint32_t s_d[kComposeBatch];
    __shared__ uint8_t s_S[256], s_flag[256];
    const uint32_t b = blockIdx.x, l = threadIdx.x;
    const uint32_t c0 = chunk_first[b], c1 = chunk_first[b + 1];
    const uint32_t *R32 = (const uint32_t *)R;
    uint32_t st[4];
    for (int k = 0; k < 4; ++k) st[k] = 4 * l + k;
    uint32_t pre[kComposeBatch], pred = 0;
    auto fetch = [&](uint32_t cb) {
#pragma unroll
        for (uint32_t j = 0; j < kComposeBatch; ++j)
            pre[j] = cb + j < c1 ? R32[(size_t)(cb + j) * 64 + l] : 0u;
        pred = (l < kComposeBatch && cb + l < c1) ? dcount[cb + l] : 0u;
    };
    fetch(c0);
    for (uint32_t cb = c0; cb < c1; cb += kComposeBatch) {
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kComposeBatch; ++j) s_R[j][l] = pre[j];
        if (l < kComposeBatch) s_d[l] = pred;
        __syncthreads();
        if (cb + kComposeBatch < c1) fetch(cb + kComposeBatch);
        const uint32_t ce = min(c1, cb + kComposeBatch);
        for (uint32_t c = cb; c < ce; ++c) {
            S[(size_t)c * 64 + l] = st[0] | (st[1] << 8) | (st[2] << 16) | (st[3] << 24);
            const uint32_t d = s_d[c - cb], rw = s_R[c - cb][l];
            *(uint32_t *)&s_flag[4 * l] = 0;
            __syncthreads();
            for (uint32_t k = 0; k < 4; ++k)
                if (4 * l + k < d) s_flag[(rw >> (8 * k)) & 255u] = 1;
            __syncthreads();
            uint32_t keep[4], cnt = 0;
            for (int k = 0; k < 4; ++k) {
                keep[k] = s_flag[st[k]] == 0;
                cnt += keep[k];
            }
            uint32_t pos = d + wave_incl_sum(cnt) - cnt;
            for (int k = 0; k < 4; ++k)
                if (keep[k]) s_S[pos++] = (uint8_t)st[k];
            for (uint32_t k = 0; k < 4; ++k)
                if (4 * l + k < d) s_S[4 * l + k] = (uint8_t)(rw >> (8 * k));
            __syncthreads();
            for (int k = 0; k < 4; ++k) st[k] = s_S[4 * l + k];
            __syncthreads();
        }
    }
}

// Time stamps are 9-bit slots kept as a byte (tm8, the low 8 bits) plus an epoch bit (ep: the
// symbol was accessed since the last renumbering, i.e. its slot is >= 256): 288 B of LDS per
// lane instead of 512, so six one-wave workgroups fit a CU instead of four waves. A lane's
// bytes for symbols 4k..4k+3 share one dword, and dword k of lane l sits at k * kLanes + l
// (every lane in its own bank).
__device__ __forceinline__ uint32_t tm8_index(uint32_t c, uint32_t l) { return ((c >> 2) * kLanes + l) * 4 + (c & 3u); }

__device__ __forceinline__ uint32_t stamp_read(const uint8_t *tm8, const uint32_t *ep, uint32_t c, uint32_t l)
{
    const uint32_t lo = tm8[tm8_index(c, l)];
    const uint32_t e = ep[(c >> 5) * kLanes + l];
    return lo | (((e >> (c & 31u)) & 1u) << 8);
}

// a new slot (>= 256) for symbol c
__device__ __forceinline__ void stamp_write_new(uint8_t *tm8, uint32_t *ep, uint32_t c, uint32_t l, uint32_t slot)
{
    tm8[tm8_index(c, l)] = (uint8_t)slot;
    atomicOr(&ep[(c >> 5) * kLanes + l], 1u << (c & 31u));
}

// Marks above slot t: bits above in t's word + words above in t's superword + superwords above.
__device__ __forceinline__ uint32_t marks_above(uint32_t t, uint32_t S, const uint32_t *bits, const uint32_t *cnt,
                                                uint32_t l)
{
    const uint32_t ws = t >> 5, sb = t & 31u, wq = ws >> 2, wr = ws & 3u;
    const uint32_t bw = bits[ws * kLanes + l];
    const uint32_t cw = cnt[wq * kLanes + l];
    uint32_t r = __builtin_popcount((bw >> sb) >> 1);
    r = __builtin_amdgcn_sad_u8(cw & (0xFFFFFF00u << (8 * wr)), 0u, r);
    r = __builtin_amdgcn_sad_u8(S & (0xFFFFFF00u << (8 * wq)), 0u, r);
    return r;
}

__device__ __forceinline__ void window_reset(uint32_t *bits, uint32_t *cnt, uint32_t l, uint32_t &S, uint32_t &now)
{
    for (uint32_t w = 0; w < 16; ++w) bits[w * kLanes + l] = w < 8 ? 0xffffffffu : 0u;
    for (uint32_t q = 0; q < 4; ++q) cnt[q * kLanes + l] = q < 2 ? 0x20202020u : 0u;
    S = 0x00008080u;
    now = 256;
}


// MTF of G consecutive symbols of one lane with ONE round of state reads (batched step).
// All reads see the state before the group; in registers, for symbol j:
//   first occurrence in the group: idx = marks above its stamp + #{i < j first in the group
//                                  whose stamp is below it} (those moved above it);
//   repeat of position p:          idx = #distinct symbols in (p, j) = popcount of the
//                                  "latest occurrence" set above p.
// Then the state update: each first occurrence clears its old mark, each last occurrence
// takes slot now0 + j (one OR per group: the G slots share a word).
template <int G>
__device__ __forceinline__ uint32_t mtf_group(const uint32_t (&c)[G], uint32_t vmask, uint8_t *tm8, uint32_t *ep,
                                              uint32_t *bits, uint32_t *cnt, uint32_t l, uint32_t &S, uint32_t now0,
                                              uint32_t (&idx)[G])
{
    uint32_t t[G], base[G], prev[G];
#pragma unroll
    for (int j = 0; j < G; ++j) t[j] = stamp_read(tm8, ep, c[j], l);
#pragma unroll
    for (int j = 0; j < G; ++j) base[j] = marks_above(t[j], S, bits, cnt, l);
    uint32_t first = 0, lastm = vmask;
#pragma unroll
    for (int j = 0; j < G; ++j) {
        prev[j] = G;
#pragma unroll
        for (int i = 0; i < j; ++i)
            if (((vmask >> i) & 1u) && c[i] == c[j]) prev[j] = i;
        if (((vmask >> j) & 1u) && prev[j] == G) first |= 1u << j;
        if (((vmask >> j) & 1u) && prev[j] < G) lastm &= ~(1u << prev[j]);
    }
    uint32_t M = 0;  // latest-occurrence positions among the group's symbols so far
#pragma unroll
    for (int j = 0; j < G; ++j) {
        uint32_t r;
        if ((first >> j) & 1u) {
            r = base[j];
#pragma unroll
            for (int i = 0; i < j; ++i) r += ((first >> i) & 1u) && t[i] < t[j];
        } else {
            r = __builtin_popcount(M >> (prev[j] + 1));
        }
        idx[j] = r;
        if ((vmask >> j) & 1u) M = (M & ~(prev[j] < G ? 1u << prev[j] : 0u)) | (1u << j);
    }
    // state update: clear the old marks of first occurrences, set the last occurrences' slots
#pragma unroll
    for (int j = 0; j < G; ++j) {
        if ((first >> j) & 1u) {
            const uint32_t ws = t[j] >> 5, wq = ws >> 2;
            atomicXor(&bits[ws * kLanes + l], 1u << (t[j] & 31u));
            atomicSub(&cnt[wq * kLanes + l], 1u << (8 * (ws & 3u)));
            S -= 1u << (8 * wq);
        }
    }
    const uint32_t wn = now0 >> 5, np = __builtin_popcount(lastm);
    atomicOr(&bits[wn * kLanes + l], lastm << (now0 & 31u));
    atomicAdd(&cnt[(wn >> 2) * kLanes + l], np << (8 * (wn & 3u)));
    S += np << (8 * (wn >> 2));
#pragma unroll
    for (int j = 0; j < G; ++j)
        if ((lastm >> j) & 1u) stamp_write_new(tm8, ep, c[j], l, now0 + j);
    return 0;
}

// grid = ceil(chunks / 256); one lane per chunk. Chunks start 16-byte aligned except a block's
// (<= 15-byte) first chunk; all lanes step through 16-symbol groups in lockstep so that the
// slot counter `now` (and the renumbering every 256 slots) stays wave-uniform; a lane whose
// group holds fewer than 16 of its symbols predicates the missing steps off (their slots stay
// unmarked, which is harmless: slots only order accesses).
__global__ __launch_bounds__(kLanes) void k_mtf_encode(const uint8_t *__restrict__ L, const MChunk *__restrict__ chunks,
                                                       uint32_t nch, const uint32_t *__restrict__ Sst,
                                                       uint8_t *__restrict__ out)
{
    __shared__ uint32_t tm32[64 * kLanes];  // the stamp bytes (tm8_index)
    __shared__ uint32_t ep[8 * kLanes];
    __shared__ uint32_t bits[16 * kLanes];
    uint8_t *tm8 = (uint8_t *)tm32;
    __shared__ uint32_t cnt[4 * kLanes];
    const uint32_t l = threadIdx.x;
    const uint32_t g = blockIdx.x * kLanes + l;
    const bool live = g < nch;
    const MChunk ch = live ? chunks[g] : MChunk{0, 0, 0, 0};
    if (live) {
        const uint32_t *st = Sst + (size_t)g * 64;
        for (uint32_t k4 = 0; k4 < 64; ++k4) {
            const uint32_t w = st[k4];
            for (uint32_t j = 0; j < 4; ++j) tm8[tm8_index((w >> (8 * j)) & 255u, l)] = (uint8_t)(255 - (4 * k4 + j));
        }
    }
    for (uint32_t w = 0; w < 8; ++w) ep[w * kLanes + l] = 0;
    uint32_t S, now;
    window_reset(bits, cnt, l, S, now);
    const uint32_t base = ch.start & ~15u, end = ch.start + ch.len;
    const uint32_t ngroups = live ? (((end + 15u) & ~15u) - base) >> 4 : 0u;
    // the input of group g (16 symbols, zero outside the chunk); fetched two groups ahead
    auto load_group = [&](uint32_t gi) {
        uint4 v = make_uint4(0, 0, 0, 0);
        const uint32_t a = base + 16 * gi;
        if (gi < ngroups) {
            if (a >= ch.start && a + 16 <= end) {
                v = *(const uint4 *)(L + a);
            } else {
                uint32_t *vw = &v.x;
                for (uint32_t k = 0; k < 16; ++k)
                    if (a + k >= ch.start && a + k < end) vw[k >> 2] |= (uint32_t)L[a + k] << (8 * (k & 3));
            }
        }
        return v;
    };
    uint4 pf0 = load_group(0), pf1 = load_group(1);
    for (uint32_t grp = 0; __builtin_amdgcn_ballot_w64(grp < ngroups) != 0; ++grp) {
        const uint32_t a = base + 16 * grp;
        const bool full = grp < ngroups && a >= ch.start && a + 16 <= end;
        const uint4 in4 = pf0;
        pf0 = pf1;
        pf1 = load_group(grp + 2);
        uint4 o4 = make_uint4(0, 0, 0, 0);
        uint32_t *o = &o4.x;
        const uint32_t *iw = &in4.x;
        uint32_t vm = 0;  // symbols of this group that belong to the lane's chunk
        if (grp < ngroups)
            for (uint32_t k = 0; k < 16; ++k) vm |= (uint32_t)(a + k >= ch.start && a + k < end) << k;
#pragma unroll
        for (int h = 0; h < 16 / kMtfGroup; ++h) {
            uint32_t cs[kMtfGroup], ix[kMtfGroup];
#pragma unroll
            for (int j = 0; j < kMtfGroup; ++j) {
                const int k = h * kMtfGroup + j;
                cs[j] = (iw[k >> 2] >> (8 * (k & 3))) & 255u;
            }
            mtf_group<kMtfGroup>(cs, (vm >> (h * kMtfGroup)) & ((1u << kMtfGroup) - 1), tm8, ep, bits, cnt, l, S, now,
                                 ix);
#pragma unroll
            for (int j = 0; j < kMtfGroup; ++j) {
                const int k = h * kMtfGroup + j;
                o[k >> 2] |= (ix[j] & 255u) << (8 * (k & 3));
            }
            now += kMtfGroup;
        }
        // a group of 16 symbols advances `now` by 16 from 256, so the window fills up
        // exactly at a group boundary
        if (now == 512) {  // wave-uniform: renumber slot of each symbol -> 255 - marks above
            uint32_t e8[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) e8[w] = ep[w * kLanes + l];
            for (uint32_t s0 = 0; s0 < 256; s0 += 16) {  // 16 independent reads in flight
                uint32_t tw[4], nw[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) tw[k] = tm32[((s0 >> 2) + k) * kLanes + l];
#pragma unroll
                for (int k = 0; k < 4; ++k) nw[k] = 0;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const uint32_t c = s0 + k;
                    uint32_t e = 0;
#pragma unroll
                    for (int w = 0; w < 8; ++w)  // c >> 5 is uniform per unrolled step
                        if ((uint32_t)w == (c >> 5)) e = e8[w];
                    const uint32_t ts = ((tw[k >> 2] >> (8 * (k & 3))) & 255u) | (((e >> (c & 31u)) & 1u) << 8);
                    nw[k >> 2] |= (255u - marks_above(ts, S, bits, cnt, l)) << (8 * (k & 3));
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) tm32[((s0 >> 2) + k) * kLanes + l] = nw[k];
            }
#pragma unroll
            for (int w = 0; w < 8; ++w) ep[w * kLanes + l] = 0;
            window_reset(bits, cnt, l, S, now);
        }
        if (full) {
            *(uint4 *)(out + a) = o4;
        } else if (grp < ngroups) {
            for (uint32_t k = 0; k < 16; ++k)
                if (a + k >= ch.start && a + k < end) out[a + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
        }
    }
}

struct HChunk {
    uint32_t block, start, len, rel;
};

// freq + first occurrence of each MTF value, per block (huffman() main.cpp:231-244), and the
// histogram of every 4 K-symbol pack chunk (u16; the pack sizes its chunks from these
// instead of re-reading the MTF stream). One workgroup per 64 K symbols of a block.
__global__ __launch_bounds__(256) void k_mtf_hist(const uint8_t *__restrict__ in, const HChunk *__restrict__ chunks,
                                                  const uint32_t *__restrict__ pfirst, uint32_t *__restrict__ freq,
                                                  uint32_t *__restrict__ first, uint16_t *__restrict__ chist)
{
    __shared__ uint32_t h[4][256], f[256];
    const HChunk ch = chunks[blockIdx.x];
    const uint32_t t = threadIdx.x, w = t >> 6;
    f[t] = 0xffffffffu;
    uint32_t tot = 0;
    for (uint32_t s0 = 0; s0 < ch.len; s0 += kPackChunkSyms) {
        for (int k = 0; k < 4; ++k) h[k][t] = 0;
        __syncthreads();
        const uint32_t len = min(kPackChunkSyms, ch.len - s0), a = ch.start + s0;
        if (len == kPackChunkSyms && (a & 15u) == 0) {
            const uint4 v4 = *(const uint4 *)(in + a + 16 * t);
            const uint32_t *vw = &v4.x;
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                const uint32_t v = (vw[k >> 2] >> (8 * (k & 3))) & 255u, pos = ch.rel + s0 + 16 * t + k;
                atomicAdd(&h[w][v], 1u);
                if (pos < f[v]) atomicMin(&f[v], pos);  // racy read only skips non-minima
            }
        } else {
            for (uint32_t i = t; i < len; i += 256) {
                const uint32_t v = in[a + i], pos = ch.rel + s0 + i;
                atomicAdd(&h[w][v], 1u);
                if (pos < f[v]) atomicMin(&f[v], pos);
            }
        }
        __syncthreads();
        const uint32_t c = h[0][t] + h[1][t] + h[2][t] + h[3][t];
        tot += c;
        chist[(size_t)(pfirst[ch.block] + ((ch.rel + s0) / kPackChunkSyms)) * 256 + t] = (uint16_t)c;
        __syncthreads();
    }
    if (tot) {
        atomicAdd(&freq[(size_t)ch.block * 256 + t], tot);
        atomicMin(&first[(size_t)ch.block * 256 + t], f[t]);
    }
}

__global__ void k_fill_u32(uint32_t *p, uint32_t v, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace

void mtf_batch(Ctx *c, const uint8_t *d_L, const Batch &bt, uint8_t *d_mtf, uint32_t *h_freq32, uint32_t *h_first32)
{
    const uint32_t nb = bt.nblocks;
    std::vector<MChunk> hc;
    std::vector<HChunk> hh;
    std::vector<uint32_t> cfirst(nb + 1), pfirst(nb + 1);
    pack_chunk_first(bt, pfirst.data());
    for (uint32_t b = 0; b < nb; ++b) {
        cfirst[b] = (uint32_t)hc.size();
        const uint64_t o = bt.offs[b], n = bt.offs[b + 1] - o;
        // chunk boundaries on 16-byte multiples of the batch (a block's first chunk takes the
        // unaligned prefix) so the encode kernel moves 16 symbols per vector load / store
        for (uint64_t s = 0; s < n;) {
            const uint64_t gpos = o + s;
            const uint64_t lim = (gpos & 15u) ? ((gpos + 15) & ~15ull) : gpos + kMtfChunk;
            const uint64_t e = std::min<uint64_t>(o + n, lim);
            MChunk m;
            m.block = b;
            m.start = (uint32_t)gpos;
            m.len = (uint32_t)(e - gpos);
            m.rel = (uint32_t)s;
            hc.push_back(m);
            s = e - o;
        }
        for (uint64_t s = 0; s < n; s += 65536)
            hh.push_back(HChunk{b, (uint32_t)(o + s), (uint32_t)std::min<uint64_t>(65536, n - s), (uint32_t)s});
    }
    cfirst[nb] = (uint32_t)hc.size();
    const uint32_t nch = (uint32_t)hc.size(), nhh = (uint32_t)hh.size();
    const size_t tb = nch * sizeof(MChunk) + nhh * sizeof(HChunk) + 2 * (nb + 1) * 4;
    uint8_t *d_tab = (uint8_t *)c->get(WS_MTF_CHUNKS, tb + 64);
    MChunk *d_chunks = (MChunk *)d_tab;
    HChunk *d_hh = (HChunk *)(d_tab + nch * sizeof(MChunk));
    uint32_t *d_cfirst = (uint32_t *)(d_tab + nch * sizeof(MChunk) + nhh * sizeof(HChunk));
    uint32_t *d_pfirst = d_cfirst + (nb + 1);
    c->h2d(d_chunks, hc.data(), nch * sizeof(MChunk));
    c->h2d(d_hh, hh.data(), nhh * sizeof(HChunk));
    c->h2d(d_cfirst, cfirst.data(), (nb + 1) * 4);
    c->h2d(d_pfirst, pfirst.data(), (nb + 1) * 4);
    uint16_t *d_chist = (uint16_t *)c->get(WS_PACK_HIST, (size_t)pfirst[nb] * 256 * 2 + 64);
    uint8_t *d_R = (uint8_t *)c->get(WS_MTF_R, (size_t)nch * 256 + (size_t)nch * 4 + 64);
    uint32_t *d_dcount = (uint32_t *)(d_R + (size_t)nch * 256);
    uint32_t *d_S = (uint32_t *)c->get(WS_MTF_S, (size_t)nch * 256);
    uint32_t *d_freq = (uint32_t *)c->get(WS_FREQ, (size_t)nb * 256 * 4);
    uint32_t *d_first = (uint32_t *)c->get(WS_FIRST, (size_t)nb * 256 * 4);
    BMH_HIP(hipMemsetAsync(d_freq, 0, (size_t)nb * 256 * 4, c->stream));
    BMH_LAUNCH(c, "mtf_fill", k_fill_u32, (uint32_t)(((size_t)nb * 256 + 255) / 256), 256, 0, d_first, 0xffffffffu,
               (size_t)nb * 256);
    BMH_LAUNCH(c, "mtf_recency", k_mtf_recency, nch, 256, 0, d_L, d_chunks, d_R, d_dcount);
    BMH_LAUNCH(c, "mtf_compose", k_mtf_compose, nb, 64, 0, d_cfirst, d_R, d_dcount, d_S);
    BMH_LAUNCH(c, "mtf_encode", k_mtf_encode, (nch + kLanes - 1) / kLanes, kLanes, 0, d_L, d_chunks, nch, d_S, d_mtf);
    BMH_LAUNCH(c, "mtf_hist", k_mtf_hist, nhh, 256, 0, d_mtf, d_hh, d_pfirst, d_freq, d_first, d_chist);
    if (h_freq32) c->d2h(h_freq32, d_freq, (size_t)nb * 256 * 4);
    if (h_first32) c->d2h(h_first32, d_first, (size_t)nb * 256 * 4);
    if (h_freq32 || h_first32) c->sync();
}

}  // namespace bmh
