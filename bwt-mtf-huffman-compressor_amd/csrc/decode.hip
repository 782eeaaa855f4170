// decode.hip — record decode on the GPU: Huffman -> inverse MTF -> inverse BWT, batched over
// blocks (replaces decompress(), reference main.cpp:327-345).
//
//   Huffman^-1 (huffman_reverse, main.cpp:259-281): each block's payload is cut into 8 Kbit
//     segments, one thread each. Pass 1 decodes every segment from its first bit and records
//     where it ends and its first codeword boundaries. A fix-up pass re-decodes each segment
//     from the previous segment's end until it meets one of its own recorded boundaries
//     (Huffman codes resynchronise within a few code words), iterated until no segment end
//     moves. A final pass decodes every segment from its true start into the MTF stream.
//   MTF^-1 (main.cpp:114-130): chunks of 4 K symbols, one lane each. The effect of a chunk on
//     the alphabet is a permutation of list positions that does not depend on the symbols, so
//     (1) every chunk computes its permutation from the identity list, (2) one wave per block
//     chains them into each chunk's start list, (3) every chunk decodes from its start list.
//     Lanes keep the alphabet as slots: sym_at[slot], a 512-slot mark bitset and two levels of
//     counts; the symbol at list position j is the mark with j marks above it (select).
//   BWT^-1 (bwt_reverse, main.cpp:61-75): LF(r) = C[L[r]] + occ(L[r], r) by a stable
//     counting sort (per-chunk histograms, block scan, ballot-matched ranks inside a chunk).
//     The text comes out of the LF cycle backwards from the primary row: rows r = 0 mod 256
//     and the primary row split the cycle into ~256-row segments; one thread walks each
//     segment (its length and the next splitter), pointer jumping ranks the splitter list,
//     and a second walk writes every segment at its place.
#include "bmh_internal.h"
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

constexpr uint32_t kSegBits = 8192;     // Huffman decode segment
constexpr uint32_t kSyncBnd = 32;       // codeword boundaries recorded per segment
constexpr int kFixRounds = 4;           // fix-up rounds before the offset-map fallback
constexpr uint32_t kImtfChunk = 4096;   // inverse-MTF chunk
constexpr int kImtfLanes = 256;
constexpr uint32_t kLfChunk = 4096;     // stable-rank chunk (4 waves x 16 x 64 rows)
constexpr uint32_t kSplit = 256;        // row spacing of the LF-cycle splitters
constexpr uint32_t kNil = 0xffffffffu;

struct DBlock {
    const uint8_t *pay;    // payload (device)
    uint64_t pay_bits;     // 8 * payload bytes
    uint64_t out_off;      // first output byte of the block
    uint32_t n, primary;   // symbols, primary row
    uint32_t seg0, nseg;   // Huffman segments
    uint32_t sp0, nsp;     // LF splitters
    uint32_t ch0, nch;     // inverse-MTF / LF chunks
};

// ------------------------------------------------------------------- Huffman decode
// 64 payload bits from bit position pos (MSB first), zero past the payload end.
__device__ __forceinline__ uint64_t bits64(const uint8_t *pay, uint64_t pay_bits, uint64_t pos)
{
    const uint64_t pay_bytes = pay_bits >> 3;
    const uint64_t by = pos >> 3;
    if (by + 12 <= pay_bytes) {
        // three aligned dwords hold the bytes [q, q + 9) (big-endian bit order)
        const uint8_t *q = pay + by;
        const uint32_t *aq = (const uint32_t *)((uintptr_t)q & ~(uintptr_t)3);
        const uint32_t al = (uint32_t)((uintptr_t)q & 3u) * 8u + (uint32_t)(pos & 7u);  // 0 .. 31
        const uint64_t hi = ((uint64_t)__builtin_bswap32(aq[0]) << 32) | __builtin_bswap32(aq[1]);
        const uint32_t lo = __builtin_bswap32(aq[2]);
        return al ? (hi << al) | (lo >> (32 - al)) : hi;
    }
    uint64_t hi = 0;
    for (int i = 0; i < 8; ++i) hi = (hi << 8) | (by + i < pay_bytes ? pay[by + i] : 0u);
    const uint32_t nx = by + 8 < pay_bytes ? pay[by + 8] : 0u;
    const uint32_t sh = (uint32_t)(pos & 7u);
    return sh ? (hi << sh) | (nx >> (8 - sh)) : hi;
}

// Decodes one symbol at pos; returns its code length (bits) and the symbol.
__device__ __forceinline__ uint32_t dec_sym(const DecTable *__restrict__ t, uint64_t w, uint32_t &sym)
{
    const uint32_t e = t->lut[w >> (64 - kDecLutBits)];
    if (e & 255u) {
        sym = (e >> 8) & 255u;
        return e & 255u;
    }
    uint32_t v = e >> 16, k = kDecLutBits;
    while (true) {
        v = t->child[v][(w >> (63 - k)) & 1u];
        ++k;
        if (t->child[v][0] == 0xffff || k >= 64) break;
    }
    sym = t->sym[v];
    return k;
}

// Decode tables of a workgroup's block staged in LDS (every workgroup of the Huffman passes
// holds segments of one block: each block's segment list starts on a multiple of 256).
struct DecLds {
    uint32_t lut[1u << kDecLutBits];
    uint32_t child[512];  // lo 16: left, hi 16: right (0xffff: leaf)
    uint8_t sym[512];
};

__device__ __forceinline__ void load_dec_lds(DecLds &d, const DecTable *__restrict__ t)
{
    for (uint32_t i = threadIdx.x; i < (1u << kDecLutBits); i += 256) d.lut[i] = t->lut[i];
    for (uint32_t i = threadIdx.x; i < 512; i += 256) {
        d.child[i] = (uint32_t)t->child[i][0] | ((uint32_t)t->child[i][1] << 16);
        d.sym[i] = t->sym[i];
    }
}

// MSB-first bit window over a payload: win holds the next `valid` (>= 32 after refill) bits.
struct BitWin {
    const uint32_t *p;  // next aligned dword to load
    const uint32_t *pend;  // first dword past the payload
    uint64_t win;
    uint32_t valid;
    __device__ __forceinline__ uint32_t ld(const uint32_t *q) const { return q < pend ? __builtin_bswap32(*q) : 0u; }
    __device__ __forceinline__ void init(const uint8_t *pay, uint64_t pay_bits, uint64_t pos)
    {
        const uint64_t abit = (uint64_t)(uintptr_t)pay * 8 + pos;  // absolute bit address
        const uint32_t *q = (const uint32_t *)(uintptr_t)((abit >> 5) << 2);
        pend = (const uint32_t *)(((uintptr_t)pay + (pay_bits >> 3) + 3) & ~(uintptr_t)3);
        const uint32_t o = (uint32_t)(abit & 31u);
        win = (((uint64_t)ld(q) << 32) | ld(q + 1)) << o;
        valid = 64 - o;
        p = q + 2;
    }
    __device__ __forceinline__ void refill()
    {
        if (valid < 32) {
            win |= (uint64_t)ld(p) << (32 - valid);
            valid += 32;
            ++p;
        }
    }
    __device__ __forceinline__ void consume(uint32_t n)
    {
        win = n < 64 ? win << n : 0ull;
        valid -= n;
    }
};

// one symbol from the window (codes up to 32 + 12 bits wide are decoded from the window;
// the window always holds >= 32 bits here)
__device__ __forceinline__ uint32_t dec_sym_lds(const DecLds &d, uint64_t w, uint32_t &sym)
{
    const uint32_t e = d.lut[w >> (64 - kDecLutBits)];
    if (e & 255u) {
        sym = (e >> 8) & 255u;
        return e & 255u;
    }
    uint32_t v = e >> 16, k = kDecLutBits;
    while (true) {
        const uint32_t ch = d.child[v];
        v = ((w >> (63 - k)) & 1u) ? ch >> 16 : ch & 0xffffu;
        ++k;
        if ((d.child[v] & 0xffffu) == 0xffffu || k >= 64) break;
    }
    sym = d.sym[v];
    return k;
}

__global__ __launch_bounds__(256) void k_hd_pass1(const DBlock *__restrict__ blks, const DecTable *__restrict__ tabs,
                                                  const uint32_t *__restrict__ seg_block, uint32_t nseg_total,
                                                  uint64_t *__restrict__ seg_end, uint32_t *__restrict__ seg_cnt,
                                                  uint16_t *__restrict__ bnd)
{
    __shared__ DecLds d;
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const uint32_t bw = seg_block[blockIdx.x * 256];  // the workgroup's block
    load_dec_lds(d, &tabs[bw]);
    __syncthreads();
    if (g >= nseg_total || seg_block[g] == kNil) return;
    const DBlock B = blks[bw];
    const uint64_t s0 = (uint64_t)(g - B.seg0) * kSegBits;
    const uint64_t stop = min(s0 + kSegBits, B.pay_bits);
    uint64_t pos = s0;
    uint32_t cnt = 0;
    uint16_t *bb = bnd + (size_t)g * kSyncBnd;
    BitWin r;
    r.init(B.pay, B.pay_bits, pos);
    while (pos < stop) {
        if (cnt < kSyncBnd) bb[cnt] = (uint16_t)(pos - s0);
        r.refill();
        uint32_t sym;
        const uint32_t len = dec_sym_lds(d, r.win, sym);
        r.consume(len);
        pos += len;
        ++cnt;
    }
    for (uint32_t k = cnt; k < kSyncBnd; ++k) bb[k] = 0xffff;
    seg_end[g] = pos;
    seg_cnt[g] = cnt;
}

// One fix-up round: segment g restarts from the previous segment's end (prev_end) and walks
// until it lands on one of its recorded boundaries; beyond that its pass-1 decode is valid.
__global__ __launch_bounds__(256) void k_hd_fix(const DBlock *__restrict__ blks, const DecTable *__restrict__ tabs,
                                                const uint32_t *__restrict__ seg_block, uint32_t nseg_total,
                                                const uint64_t *__restrict__ end_in, uint64_t *__restrict__ end_out,
                                                uint64_t *__restrict__ seg_start, uint32_t *__restrict__ seg_cnt,
                                                const uint16_t *__restrict__ bnd, uint32_t *changed)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nseg_total || seg_block[g] == kNil) return;
    const uint32_t b = seg_block[g];
    const DBlock B = blks[b];
    const uint64_t s0 = (uint64_t)(g - B.seg0) * kSegBits;
    const uint64_t T = g == B.seg0 ? 0ull : end_in[g - 1];
    const uint64_t e_old = end_in[g];
    if (T == seg_start[g]) {  // already consistent with its predecessor
        end_out[g] = e_old;
        return;
    }
    const DecTable *t = &tabs[b];
    const uint64_t stop = min(s0 + kSegBits, B.pay_bits);
    const uint16_t *bb = bnd + (size_t)g * kSyncBnd;
    uint64_t pos = T;
    uint32_t cnt = 0, k = 0;
    // the old decode started at the old start; its boundaries are s0 + bb[k] (pass 1 start)
    // or, after an earlier fix-up, unknown: then decode the whole segment
    const bool have_bnd = seg_start[g] == s0;
    while (pos < stop) {
        if (have_bnd) {
            while (k < kSyncBnd && bb[k] != 0xffff && s0 + bb[k] < pos) ++k;
            if (k < kSyncBnd && bb[k] != 0xffff && s0 + bb[k] == pos) {
                // synchronised with the pass-1 path: its remaining count and end hold
                seg_cnt[g] = cnt + (seg_cnt[g] - k);
                seg_start[g] = T;
                end_out[g] = e_old;
                return;
            }
        }
        uint32_t sym;
        pos += dec_sym(t, bits64(B.pay, B.pay_bits, pos), sym);
        ++cnt;
    }
    seg_cnt[g] = cnt;
    seg_start[g] = T;
    end_out[g] = pos;
    if (pos != e_old) atomicOr(changed, 1u);
}

// Fallback when the fix-up rounds do not settle (codes that never resynchronise, e.g. every
// code word the same length L with kSegBits not a multiple of L): a segment can only be
// entered at one of maxlen bit offsets past its nominal start (the previous segment's last
// code word starts before it), so P lanes per segment decode it from every offset o < maxlen
// and record where each decode leaves the segment and how many symbols it produced:
// map[g * P + o] = count << 8 | (end - stop). A lane that lands on a boundary of the offset-0
// decode (pass 1, first kSyncBnd boundaries) takes that decode's remainder.
__global__ __launch_bounds__(256) void k_hd_map(const DBlock *__restrict__ blks, const DecTable *__restrict__ tabs,
                                                const uint32_t *__restrict__ seg_block, uint32_t nseg_total, uint32_t P,
                                                const uint64_t *__restrict__ end0, const uint32_t *__restrict__ cnt0,
                                                const uint16_t *__restrict__ bnd, uint32_t *__restrict__ map)
{
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t g = (uint32_t)(t / P), o = (uint32_t)(t % P);
    if (g >= nseg_total || seg_block[g] == kNil) return;
    const uint32_t b = seg_block[g];
    const DBlock B = blks[b];
    const DecTable *tb = &tabs[b];
    if (o >= tb->maxlen && o != 0) return;
    const uint64_t s0 = (uint64_t)(g - B.seg0) * kSegBits;
    const uint64_t stop = min(s0 + kSegBits, B.pay_bits);
    if (o == 0) {
        map[t] = (cnt0[g] << 8) | (uint32_t)(end0[g] - stop);
        return;
    }
    const uint16_t *bb = bnd + (size_t)g * kSyncBnd;
    uint64_t pos = s0 + o;
    uint32_t cnt = 0, k = 0;
    while (pos < stop) {
        while (k < kSyncBnd && bb[k] != 0xffff && s0 + bb[k] < pos) ++k;
        if (k < kSyncBnd && bb[k] != 0xffff && s0 + bb[k] == pos) {
            map[t] = ((cnt + cnt0[g] - k) << 8) | (uint32_t)(end0[g] - stop);
            return;
        }
        uint32_t sym;
        pos += dec_sym(tb, bits64(B.pay, B.pay_bits, pos), sym);
        ++cnt;
    }
    map[t] = (cnt << 8) | (uint32_t)(pos - stop);
}

// One wave per block chains the offset maps from the block's first bit: segment g starts at
// T, produces map[g][T - s0] >> 8 symbols and hands T' = stop + (map & 255) to g + 1. The
// map rows do not depend on T, so they are loaded kChainAhead segments ahead.
constexpr uint32_t kChainAhead = 16;
__global__ __launch_bounds__(64) void k_hd_chain(const DBlock *__restrict__ blks, uint32_t P,
                                                 const uint32_t *__restrict__ map, uint64_t *__restrict__ seg_start,
                                                 uint32_t *__restrict__ seg_cnt, uint32_t *status)
{
    const DBlock B = blks[blockIdx.x];
    const uint32_t lane = threadIdx.x;
    uint64_t T = 0;
    for (uint32_t k0 = 0; k0 < B.nseg; k0 += kChainAhead) {
        uint32_t e[kChainAhead];
#pragma unroll
        for (uint32_t j = 0; j < kChainAhead; ++j)
            e[j] = (lane < P && k0 + j < B.nseg) ? map[(size_t)(B.seg0 + k0 + j) * P + lane] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < kChainAhead; ++j) {
            const uint32_t k = k0 + j;
            if (k < B.nseg) {  // (a guard, not a break: the loop stays unrolled, e[] in registers)
                const uint64_t s0 = (uint64_t)k * kSegBits;
                const uint64_t stop = min(s0 + kSegBits, B.pay_bits);
                uint32_t o = (uint32_t)(T - s0);
                if (o >= P) {  // cannot happen for a well-formed table; keep the walk in range
                    if (lane == 0) atomicOr(status, 1u);
                    o = 0;
                }
                const uint32_t v = __shfl(e[j], (int)o, 64);
                if (lane == 0) {
                    seg_start[B.seg0 + k] = T;
                    seg_cnt[B.seg0 + k] = v >> 8;
                }
                T = stop + (v & 255u);
            }
        }
    }
}

// grid = nblocks: exclusive scan of segment counts -> first output symbol of each segment
__global__ __launch_bounds__(256) void k_hd_scan(const DBlock *__restrict__ blks, uint32_t *__restrict__ seg_cnt)
{
    __shared__ uint32_t s_tmp[8];
    const DBlock B = blks[blockIdx.x];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < B.nseg; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < B.nseg ? seg_cnt[B.seg0 + i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_sum<256>(v, s_tmp, &total);
        if (i < B.nseg) seg_cnt[B.seg0 + i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(256) void k_hd_pass3(const DBlock *__restrict__ blks, const DecTable *__restrict__ tabs,
                                                  const uint32_t *__restrict__ seg_block, uint32_t nseg_total,
                                                  const uint64_t *__restrict__ seg_start,
                                                  const uint32_t *__restrict__ seg_first, uint8_t *__restrict__ mtf,
                                                  uint32_t *status)
{
    __shared__ DecLds d;
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const uint32_t bw = seg_block[blockIdx.x * 256];
    load_dec_lds(d, &tabs[bw]);
    __syncthreads();
    if (g >= nseg_total || seg_block[g] == kNil) return;
    const DBlock B = blks[bw];
    const uint64_t s0 = (uint64_t)(g - B.seg0) * kSegBits;
    const uint64_t stop = min(s0 + kSegBits, B.pay_bits);
    uint64_t pos = seg_start[g];
    uint32_t i = seg_first[g];
    uint8_t *o = mtf + B.out_off;
    BitWin r;
    r.init(B.pay, B.pay_bits, pos);
    // symbols are written four at a time once the output address is word-aligned
    uint32_t acc = 0, na = 0;
    while (pos < stop && i < B.n) {
        r.refill();
        uint32_t sym;
        const uint32_t len = dec_sym_lds(d, r.win, sym);
        r.consume(len);
        pos += len;
        const uint64_t a = B.out_off + i;
        if (na == 0 && (a & 3u)) {
            o[i] = (uint8_t)sym;
        } else {
            acc |= sym << (8 * na);
            if (++na == 4) {
                *(uint32_t *)(o + i - 3) = acc;
                acc = 0;
                na = 0;
            }
        }
        ++i;
    }
    for (uint32_t k = 0; k < na; ++k) o[i - na + k] = (uint8_t)(acc >> (8 * k));
    // the block's last segment must have produced exactly n symbols in total
    if (g + 1 == B.seg0 + B.nseg && i < B.n) atomicOr(status, 1u);
}

// Single-leaf trees: every symbol is the leaf, 0-bit codes (encode_with_huffman writes one
// zero byte).
__global__ void k_hd_single(const DBlock *__restrict__ blks, const DecTable *__restrict__ tabs, uint32_t b,
                            uint8_t *__restrict__ mtf)
{
    const DBlock B = blks[b];
    const uint8_t s = tabs[b].sym[0];
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < B.n; i += (uint64_t)gridDim.x * 256)
        mtf[B.out_off + i] = s;
}

// ------------------------------------------------------------------- inverse MTF
struct IChunk {
    uint32_t block, start, len, pad;  // start: batch offset
};

// select: the marked slot with exactly j marks above it (0 <= j < 256)
__device__ __forceinline__ uint32_t select_top(uint32_t j, uint32_t S, const uint32_t *bits, const uint32_t *cnt,
                                               uint32_t l)
{
    uint32_t q = 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t c = (S >> (8 * q)) & 255u;
        if (j >= c) {
            j -= c;
            --q;
        } else {
            break;
        }
    }
    const uint32_t cw = cnt[q * kImtfLanes + l];
    uint32_t r = 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t c = (cw >> (8 * r)) & 255u;
        if (j >= c) {
            j -= c;
            --r;
        } else {
            break;
        }
    }
    const uint32_t w = 4 * q + r;
    const uint32_t x = bits[w * kImtfLanes + l];
    // the (j+1)-th set bit of x from the most significant end: the largest b with
    // popcount(x >> b) > j
    uint32_t b = 0;
#pragma unroll
    for (uint32_t width = 16; width >= 1; width >>= 1)
        if ((uint32_t)__builtin_popcount(x >> (b + width)) > j) b += width;
    return w * 32 + b;
}

__device__ __forceinline__ void imtf_reset(uint32_t *bits, uint32_t *cnt, uint32_t l, uint32_t &S, uint32_t &now)
{
    for (uint32_t w = 0; w < 16; ++w) bits[w * kImtfLanes + l] = w < 8 ? 0xffffffffu : 0u;
    for (uint32_t q = 0; q < 4; ++q) cnt[q * kImtfLanes + l] = q < 2 ? 0x20202020u : 0u;
    S = 0x00008080u;
    now = 256;
}

// mode 0: start list = identity, output the final list (permutation of positions) per chunk.
// mode 1: start list = Sst[chunk], output the decoded symbols.
template <int MODE>
__global__ __launch_bounds__(kImtfLanes) void k_imtf(const uint8_t *__restrict__ in, const IChunk *__restrict__ chunks,
                                                     uint32_t nch, const uint8_t *__restrict__ Sst,
                                                     uint8_t *__restrict__ out)
{
    __shared__ uint8_t sym_at[512 * kImtfLanes];
    __shared__ uint32_t bits[16 * kImtfLanes];
    __shared__ uint32_t cnt[4 * kImtfLanes];
    const uint32_t l = threadIdx.x;
    const uint32_t g = blockIdx.x * kImtfLanes + l;
    const bool live = g < nch;
    const IChunk ch = live ? chunks[g] : IChunk{0, 0, 0, 0};
    // list position p <-> slot 255 - p
    for (uint32_t p = 0; p < 256; ++p)
        sym_at[(255 - p) * kImtfLanes + l] = MODE == 0 ? (uint8_t)p : (live ? Sst[(size_t)g * 256 + p] : (uint8_t)0);
    uint32_t S, now;
    imtf_reset(bits, cnt, l, S, now);
    const uint32_t base = ch.start & ~15u, end = ch.start + ch.len;
    const uint32_t ngroups = live ? (((end + 15u) & ~15u) - base) >> 4 : 0u;
    for (uint32_t grp = 0; __builtin_amdgcn_ballot_w64(grp < ngroups) != 0; ++grp) {
        const uint32_t a = base + 16 * grp;
        const bool full = grp < ngroups && a >= ch.start && a + 16 <= end;
        uint4 in4 = make_uint4(0, 0, 0, 0);
        if (full) {
            in4 = *(const uint4 *)(in + a);
        } else if (grp < ngroups) {
            uint32_t *iw = &in4.x;
            for (uint32_t k = 0; k < 16; ++k)
                if (a + k >= ch.start && a + k < end) iw[k >> 2] |= (uint32_t)in[a + k] << (8 * (k & 3));
        }
        uint4 o4 = make_uint4(0, 0, 0, 0);
        uint32_t *o = &o4.x;
        const uint32_t *iw = &in4.x;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t pos = a + k;
            if (grp < ngroups && pos >= ch.start && pos < end) {
                const uint32_t j = (iw[k >> 2] >> (8 * (k & 3))) & 255u;
                const uint32_t t = select_top(j, S, bits, cnt, l);
                const uint32_t c = sym_at[t * kImtfLanes + l];
                const uint32_t ws = t >> 5, wq = ws >> 2;
                atomicXor(&bits[ws * kImtfLanes + l], 1u << (t & 31u));
                atomicSub(&cnt[wq * kImtfLanes + l], 1u << (8 * (ws & 3u)));
                S -= 1u << (8 * wq);
                const uint32_t wn = now >> 5;
                atomicOr(&bits[wn * kImtfLanes + l], 1u << (now & 31u));
                atomicAdd(&cnt[(wn >> 2) * kImtfLanes + l], 1u << (8 * (wn & 3u)));
                S += 1u << (8 * (wn >> 2));
                sym_at[now * kImtfLanes + l] = (uint8_t)c;
                o[k >> 2] |= c << (8 * (k & 3));
            }
            if (++now == 512) {  // wave-uniform: compact the 256 marks into slots 0..255
                uint32_t kk = 0;
                for (uint32_t w = 0; w < 16; ++w) {
                    uint32_t x = bits[w * kImtfLanes + l];
                    while (x) {
                        const uint32_t b = __builtin_ctz(x);
                        x &= x - 1;
                        sym_at[kk * kImtfLanes + l] = sym_at[(w * 32 + b) * kImtfLanes + l];
                        ++kk;
                    }
                }
                imtf_reset(bits, cnt, l, S, now);
            }
        }
        if (MODE == 1) {
            if (full) {
                *(uint4 *)(out + a) = o4;
            } else if (grp < ngroups) {
                for (uint32_t k = 0; k < 16; ++k)
                    if (a + k >= ch.start && a + k < end) out[a + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
            }
        }
    }
    if (MODE == 0 && live) {
        // final list: position p = the mark with p marks above it
        for (uint32_t p = 0; p < 256; ++p)
            out[(size_t)g * 256 + p] = sym_at[select_top(p, S, bits, cnt, l) * kImtfLanes + l];
    }
}

// grid = nblocks, one wave: start list of every chunk = previous start list permuted.
__global__ __launch_bounds__(64) void k_imtf_compose(const DBlock *__restrict__ blks,
                                                     const uint8_t *__restrict__ perm, uint8_t *__restrict__ Sst)
{
    __shared__ uint8_t s_state[256], s_next[256];
    __shared__ uint32_t s_perm[32][64];
    const DBlock B = blks[blockIdx.x];
    const uint32_t l = threadIdx.x;
    for (uint32_t k = 0; k < 4; ++k) s_state[4 * l + k] = (uint8_t)(4 * l + k);
    const uint32_t *P32 = (const uint32_t *)perm;
    for (uint32_t cb = 0; cb < B.nch; cb += 32) {
        __syncthreads();
        const uint32_t ce = min(B.nch, cb + 32);
        for (uint32_t c = cb; c < ce; ++c) s_perm[c - cb][l] = P32[(size_t)(B.ch0 + c) * 64 + l];
        __syncthreads();
        for (uint32_t c = cb; c < ce; ++c) {
            const uint32_t sw = s_state[4 * l] | (s_state[4 * l + 1] << 8) | (s_state[4 * l + 2] << 16) |
                                ((uint32_t)s_state[4 * l + 3] << 24);
            ((uint32_t *)(Sst + (size_t)(B.ch0 + c) * 256))[l] = sw;
            const uint32_t pw = s_perm[c - cb][l];
            for (uint32_t k = 0; k < 4; ++k) s_next[4 * l + k] = s_state[(pw >> (8 * k)) & 255u];
            __syncthreads();
            for (uint32_t k = 0; k < 4; ++k) s_state[4 * l + k] = s_next[4 * l + k];
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------- inverse BWT
__global__ __launch_bounds__(256) void k_lf_hist(const uint8_t *__restrict__ L, const DBlock *__restrict__ blks,
                                                 const uint32_t *__restrict__ ch_block, uint32_t *__restrict__ chist)
{
    __shared__ uint32_t h[256];
    const uint32_t c = blockIdx.x, b = ch_block[c];
    const DBlock B = blks[b];
    const uint32_t r0 = (c - B.ch0) * kLfChunk, len = min(kLfChunk, B.n - r0);
    const uint8_t *Lb = L + B.out_off + r0;
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += 256) atomicAdd(&h[Lb[i]], 1u);
    __syncthreads();
    chist[(size_t)c * 256 + threadIdx.x] = h[threadIdx.x];
}

// grid = nblocks, thread per symbol: chist[chunk][s] <- C[s] + #s in earlier chunks
__global__ __launch_bounds__(256) void k_lf_scan(const DBlock *__restrict__ blks, uint32_t *__restrict__ chist)
{
    __shared__ uint32_t s_tmp[8];
    const DBlock B = blks[blockIdx.x];
    const uint32_t s = threadIdx.x;
    uint32_t run = 0;
    for (uint32_t c = 0; c < B.nch; ++c) {
        uint32_t *h = &chist[(size_t)(B.ch0 + c) * 256 + s];
        const uint32_t v = *h;
        *h = run;
        run += v;
    }
    const uint32_t Cs = block_excl_sum<256>(run, s_tmp, nullptr);
    for (uint32_t c = 0; c < B.nch; ++c) chist[(size_t)(B.ch0 + c) * 256 + s] += Cs;
}

// Stable ranks inside a chunk: wave w owns rows [1024w, 1024w + 1024) in 16 steps of 64; a
// row's rank among equal bytes of its step comes from 8 ballots, the counts of earlier steps
// and waves from LDS. Output E[r] = LF(r) | L[r] << 32.
// E[r] = LF(r) and L[r] in one word: u32 (LF < 2^24) when every block is <= 16 MiB, else u64
template <typename ET> __device__ __forceinline__ ET make_e(uint32_t lf, uint32_t l);
template <> __device__ __forceinline__ uint32_t make_e<uint32_t>(uint32_t lf, uint32_t l) { return lf | (l << 24); }
template <> __device__ __forceinline__ uint64_t make_e<uint64_t>(uint32_t lf, uint32_t l)
{
    return lf | ((uint64_t)l << 32);
}
__device__ __forceinline__ uint32_t e_lf(uint32_t e) { return e & 0xffffffu; }
__device__ __forceinline__ uint32_t e_lf(uint64_t e) { return (uint32_t)e; }
__device__ __forceinline__ uint32_t e_l(uint32_t e) { return e >> 24; }
__device__ __forceinline__ uint32_t e_l(uint64_t e) { return (uint32_t)(e >> 32); }

template <typename ET>
__global__ __launch_bounds__(256) void k_lf_rank(const uint8_t *__restrict__ L, const DBlock *__restrict__ blks,
                                                 const uint32_t *__restrict__ ch_block,
                                                 const uint32_t *__restrict__ chist, ET *__restrict__ E, uint32_t c0)
{
    __shared__ uint32_t s_wcnt[4][256];
    const uint32_t c = c0 + blockIdx.x, b = ch_block[c];
    const DBlock B = blks[b];
    const uint32_t r0 = (c - B.ch0) * kLfChunk, len = min(kLfChunk, B.n - r0);
    const uint8_t *Lb = L + B.out_off + r0;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    for (uint32_t k = 0; k < 4; ++k) s_wcnt[k][t] = 0;
    __syncthreads();
    const uint64_t lt_mask = (1ull << lane) - 1;
    uint32_t sym[16], rk[16];
    for (uint32_t it = 0; it < 16; ++it) {
        const uint32_t r = 1024 * w + 64 * it + lane;
        const bool v = r < len;
        const uint32_t x = v ? Lb[r] : 0u;
        uint64_t m = __ballot(v);
#pragma unroll
        for (int bt = 0; bt < 8; ++bt) {
            const uint64_t bl = __ballot(v && ((x >> bt) & 1u));
            m &= ((x >> bt) & 1u) ? bl : ~bl;
        }
        const uint32_t before = s_wcnt[w][x];
        sym[it] = x;
        rk[it] = before + (uint32_t)__popcll(m & lt_mask);
        // the highest lane of each byte group advances the wave's count of that byte
        if (v && (m >> lane) == 1ull) s_wcnt[w][x] = before + (uint32_t)__popcll(m);
    }
    __syncthreads();
    // exclusive prefix of the 4 waves' counts per byte
    {
        const uint32_t a0 = s_wcnt[0][t], a1 = s_wcnt[1][t], a2 = s_wcnt[2][t];
        s_wcnt[0][t] = 0;
        s_wcnt[1][t] = a0;
        s_wcnt[2][t] = a0 + a1;
        s_wcnt[3][t] = a0 + a1 + a2;
    }
    __syncthreads();
    const uint32_t *cb = chist + (size_t)c * 256;
    ET *Eb = E + B.out_off + r0;
    for (uint32_t it = 0; it < 16; ++it) {
        const uint32_t r = 1024 * w + 64 * it + lane;
        if (r < len) {
            const uint32_t x = sym[it];
            Eb[r] = make_e<ET>(cb[x] + s_wcnt[w][x] + rk[it], x);
        }
    }
}

__device__ __forceinline__ uint32_t split_id(uint32_t r, const DBlock &B)
{
    if ((r & (kSplit - 1)) == 0) return r / kSplit;
    return r == B.primary ? (B.n + kSplit - 1) / kSplit : kNil;
}

__device__ __forceinline__ uint32_t split_row(uint32_t id, const DBlock &B)
{
    return id * kSplit < B.n ? id * kSplit : B.primary;
}

// walk 1: each splitter follows LF to the next splitter (the list is cut before the primary),
// writing the first kSlot characters of its segment into its slot of `tmp` and remembering
// the row reached after kSlot steps, so only segments longer than kSlot are walked again.
constexpr uint32_t kSlot = 1024;

template <typename ET>
__global__ __launch_bounds__(256) void k_lf_walk1(const DBlock *__restrict__ blks, const uint32_t *__restrict__ sp_block,
                                                  uint32_t g0, uint32_t g1, const ET *__restrict__ E,
                                                  uint32_t *__restrict__ nxt, uint64_t *__restrict__ dist,
                                                  uint32_t *__restrict__ resume, uint8_t *__restrict__ tmp,
                                                  uint32_t *status)
{
    const uint32_t g = g0 + blockIdx.x * 256 + threadIdx.x;
    if (g >= g1) return;
    const uint32_t b = sp_block[g];
    const DBlock B = blks[b];
    const uint32_t id = g - B.sp0;
    const uint32_t r0 = split_row(id, B);
    if (id * kSplit >= B.n && B.primary % kSplit == 0) {  // no extra splitter for this block
        nxt[g] = kNil;
        dist[g] = 0;
        return;
    }
    const ET *Eb = E + B.out_off;
    uint8_t *slot = tmp + (size_t)g * kSlot;
    // the segment's first kSlot characters go to the slot 16 bytes at a time (4-byte stores
    // from every thread to its own slot cost a partial-line write each)
    uint32_t r = r0, len = 0, sid, acc = 0;
    uint32_t q[4] = {0, 0, 0, 0};
    do {
        const ET e = Eb[r];
        if (len < kSlot) {
            acc |= e_l(e) << (8 * (len & 3u));
            if ((len & 3u) == 3u) {
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (((len >> 2) & 3u) == j) q[j] = acc;
                acc = 0;
                if ((len & 15u) == 15u) *(uint4 *)(slot + len - 15) = make_uint4(q[0], q[1], q[2], q[3]);
            }
        } else if (len == kSlot) {
            resume[g] = r;
        }
        r = e_lf(e);
        ++len;
        sid = split_id(r, B);
    } while (sid == kNil && len <= B.n);
    if (len < kSlot && (len & 15u)) {  // the partial last piece (its unused bytes are never read)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (((len >> 2) & 3u) == j) q[j] = acc;
        *(uint4 *)(slot + (len & ~15u)) = make_uint4(q[0], q[1], q[2], q[3]);
    }
    if (len > B.n || r >= B.n) {
        atomicOr(status, 2u);
        sid = kNil;
    }
    nxt[g] = (sid == kNil || r == B.primary) ? kNil : B.sp0 + sid;
    dist[g] = len;
}

// pointer jumping: dist[g] <- rows from g to the end of the list
__global__ __launch_bounds__(256) void k_lf_jump(uint32_t nsp_total, const uint32_t *__restrict__ nxt_in,
                                                 const uint64_t *__restrict__ dist_in, uint32_t *__restrict__ nxt_out,
                                                 uint64_t *__restrict__ dist_out, uint32_t *more)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nsp_total) return;
    const uint32_t nx = nxt_in[g];
    if (nx == kNil) {
        nxt_out[g] = kNil;
        dist_out[g] = dist_in[g];
        return;
    }
    nxt_out[g] = nxt_in[nx];
    dist_out[g] = dist_in[g] + dist_in[nx];
    if (nxt_in[nx] != kNil) atomicOr(more, 1u);
}

// pointer jumping of one block's splitter list in LDS (blocks with <= kJumpLds splitters)
constexpr uint32_t kJumpLds = 16385, kJumpNT = 1024, kJumpIPT = (kJumpLds + kJumpNT - 1) / kJumpNT;

__global__ __launch_bounds__(kJumpNT) void k_lf_jump_lds(const DBlock *__restrict__ blks, uint32_t *__restrict__ nxt,
                                                         uint64_t *__restrict__ dist)
{
    __shared__ uint16_t s_nx[kJumpLds];
    __shared__ uint32_t s_d[kJumpLds];
    __shared__ int s_more;
    const DBlock B = blks[blockIdx.x];
    const uint32_t t = threadIdx.x, m = B.nsp;
    for (uint32_t i = t; i < m; i += kJumpNT) {
        const uint32_t x = nxt[B.sp0 + i];
        s_nx[i] = x == kNil ? 0xffffu : (uint16_t)(x - B.sp0);
        s_d[i] = (uint32_t)dist[B.sp0 + i];
    }
    for (int round = 0; round < 40; ++round) {
        if (t == 0) s_more = 0;
        __syncthreads();
        uint32_t nn[kJumpIPT], dd[kJumpIPT];
        bool any = false;
#pragma unroll
        for (uint32_t k = 0; k < kJumpIPT; ++k) {
            const uint32_t i = t + k * kJumpNT;
            nn[k] = 0xffffu;
            if (i < m) {
                const uint32_t x = s_nx[i];
                dd[k] = s_d[i];
                if (x != 0xffffu) {
                    nn[k] = s_nx[x];
                    dd[k] += s_d[x];
                    any |= nn[k] != 0xffffu;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < kJumpIPT; ++k) {
            const uint32_t i = t + k * kJumpNT;
            if (i < m) {
                s_nx[i] = (uint16_t)nn[k];
                s_d[i] = dd[k];
            }
        }
        if (any) s_more = 1;
        __syncthreads();
        if (!s_more) break;
    }
    for (uint32_t i = t; i < m; i += kJumpNT) {
        nxt[B.sp0 + i] = s_nx[i] == 0xffffu ? kNil : B.sp0 + s_nx[i];
        dist[B.sp0 + i] = s_d[i];
    }
}

// place: splitter g copies its segment from its slot to text positions dist[g] - 1 down to
// dist[g] - len (the text comes out of LF backwards); past kSlot it walks on from `resume`.
template <typename ET>
__global__ __launch_bounds__(256) void k_lf_place(const DBlock *__restrict__ blks, const uint32_t *__restrict__ sp_block,
                                                  uint32_t nsp_total, const ET *__restrict__ E,
                                                  const uint64_t *__restrict__ dist, const uint32_t *__restrict__ nxt,
                                                  const uint32_t *__restrict__ resume, const uint8_t *__restrict__ tmp,
                                                  const uint64_t *__restrict__ len_of, uint8_t *__restrict__ out,
                                                  uint32_t *status)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nsp_total) return;
    const uint32_t b = sp_block[g];
    const DBlock B = blks[b];
    const uint32_t id = g - B.sp0;
    if (id * kSplit >= B.n && B.primary % kSplit == 0) return;
    // a periodic text (u^k) has k LF cycles; only the primary's one is written (see k_lf_period)
    if (nxt[g] != kNil) return;
    uint8_t *ob = out + B.out_off;
    const uint64_t pos = dist[g], len = len_of[g];
    if (pos > B.n || len > pos) {
        atomicOr(status, 2u);
        return;
    }
    const uint8_t *slot = tmp + (size_t)g * kSlot;
    const uint64_t inslot = len < kSlot ? len : kSlot;
    // (byte stores: aligned word stores with the slot read by aligned words measured slower,
    // 6.7 against 4.8 ms per GiB)
    for (uint64_t t = 0; t < inslot; ++t) ob[pos - 1 - t] = slot[t];
    if (len > kSlot) {
        const ET *Eb = E + B.out_off;
        uint32_t r = resume[g];
        for (uint64_t t = kSlot; t < len; ++t) {
            const ET e = Eb[r];
            ob[pos - 1 - t] = (uint8_t)e_l(e);
            r = e_lf(e);
        }
    }
}

// grid = nblocks: if the primary's LF cycle is shorter than n, the text is u^k with |u| = p;
// walk 2 ranked that cycle alone and wrote u at [0, p): repeat it over the rest.
__global__ __launch_bounds__(256) void k_lf_period(const DBlock *__restrict__ blks, const uint64_t *__restrict__ dist,
                                                   uint8_t *__restrict__ out, uint32_t *status)
{
    const DBlock B = blks[blockIdx.x];
    const uint32_t pid = split_id(B.primary, B);
    const uint64_t p = dist[B.sp0 + pid];
    if (p >= B.n) return;
    if (p == 0 || B.n % p != 0) {
        if (threadIdx.x == 0) atomicOr(status, 2u);
        return;
    }
    uint8_t *ob = out + B.out_off;
    for (uint64_t i = p + threadIdx.x; i < B.n; i += 256) ob[i] = ob[i % p];
}

// header bytes of each record gathered for the host (u64 primary, n, tree_len + tree)
__global__ __launch_bounds__(64) void k_gather_headers(const uint8_t *__restrict__ rec, const uint64_t *__restrict__ offs,
                                                       uint8_t *__restrict__ hdr)
{
    const uint32_t b = blockIdx.x;
    const uint64_t o = offs[b], len = offs[b + 1] - o;
    for (uint32_t i = threadIdx.x; i < 352; i += 64) hdr[(size_t)b * 352 + i] = i < len ? rec[o + i] : 0;
}

}  // namespace

namespace {

// LF by stable counting sort, one LF-cycle walk that stages each segment in a slot, a
// pointer-jumping ranking of the splitters, and a placement pass.
template <typename ET>
void lf_inverse(Ctx *c, const std::vector<DBlock> &hb, uint32_t nb, uint64_t total, uint32_t nsp, uint32_t nch,
                uint32_t max_nsp, const uint8_t *d_L, const DBlock *d_blk, const uint32_t *d_ch_block,
                const uint32_t *d_sp_block, uint8_t *d_out, uint32_t *d_status)
{
    uint32_t *d_chist = (uint32_t *)c->get(WS_BSTART, (size_t)nch * 256 * 4 + 64);
    ET *d_E = (ET *)c->get(WS_KEY8, total * sizeof(ET) + 64);
    BMH_LAUNCH(c, "dec_lf_hist", k_lf_hist, nch, 256, 0, d_L, d_blk, d_ch_block, d_chist);
    BMH_LAUNCH(c, "dec_lf_scan", k_lf_scan, nb, 256, 0, d_blk, d_chist);
    uint8_t *d_sp = (uint8_t *)c->get(WS_RKA, (size_t)nsp * 36 + 64);
    uint32_t *d_nxt = (uint32_t *)d_sp, *d_nxt2 = d_nxt + nsp, *d_resume = d_nxt2 + nsp;
    uint64_t *d_dist = (uint64_t *)(((uintptr_t)(d_resume + nsp) + 7) & ~(uintptr_t)7), *d_dist2 = d_dist + nsp;
    uint64_t *d_len = (uint64_t *)c->get(WS_RKB, (size_t)nsp * 8 + 64);
    uint8_t *d_tmp = (uint8_t *)c->get(WS_KEY, (size_t)nsp * kSlot + 64);
    // (Ranking and walking groups of blocks whose E fits the 256 MiB Infinity Cache, one group
    // after the other, measured slower at every group size, 64-224 MiB: 34-65 ms against 21 ms
    // per GiB. The walk is bound by its random-request rate through the L2s, not by where the
    // line is served from, and a group has too few walks in flight.)
    BMH_LAUNCH(c, "dec_lf_rank", k_lf_rank<ET>, nch, 256, 0, d_L, d_blk, d_ch_block, d_chist, d_E, 0u);
    BMH_LAUNCH(c, "dec_lf_walk", k_lf_walk1<ET>, cdiv(nsp, 256), 256, 0, d_blk, d_sp_block, 0u, nsp, d_E, d_nxt, d_dist,
               d_resume, d_tmp, d_status);
    BMH_HIP(hipMemcpyAsync(d_len, d_dist, (size_t)nsp * 8, hipMemcpyDeviceToDevice, c->stream));
    // pointer jumping until the primary's chain is ranked; splitters on other LF cycles
    // (periodic text) never reach the cut, so the rounds are bounded by log2(splitters)
    if (max_nsp <= kJumpLds) {
        BMH_LAUNCH(c, "dec_lf_jump", k_lf_jump_lds, nb, kJumpNT, 0, d_blk, d_nxt, d_dist);
    } else {
        uint32_t *d_more = d_status + 2;
        int rounds = 1;
        while ((1u << rounds) < max_nsp) ++rounds;
        for (int round = 0; round <= rounds; ++round) {
            BMH_HIP(hipMemsetAsync(d_more, 0, 4, c->stream));
            BMH_LAUNCH(c, "dec_lf_jump", k_lf_jump, cdiv(nsp, 256), 256, 0, nsp, d_nxt, d_dist, d_nxt2, d_dist2,
                       d_more);
            std::swap(d_nxt, d_nxt2);
            std::swap(d_dist, d_dist2);
            uint32_t more = 0;
            c->d2h(&more, d_more, 4);
            c->sync();
            if (!more) break;
        }
    }
    BMH_LAUNCH(c, "dec_lf_place", k_lf_place<ET>, cdiv(nsp, 256), 256, 0, d_blk, d_sp_block, nsp, d_E, d_dist, d_nxt,
               d_resume, d_tmp, d_len, d_out, d_status);
    BMH_LAUNCH(c, "dec_lf_period", k_lf_period, nb, 256, 0, d_blk, d_dist, d_out, d_status);
}

}  // namespace

void decode_blocks(Ctx *c, const uint8_t *d_rec, const uint64_t *rec_offs, uint32_t nb, uint8_t *d_out,
                   uint64_t out_cap, uint64_t *out_offs)
{
    if (nb == 0) fail(BMH_EINVAL, "decode: no records");
    // ---- headers -> host: n, primary, tree; decode tables
    uint64_t *d_roffs = (uint64_t *)c->get(WS_ROFFS, (size_t)(2 * nb + 1) * 8 + 64);
    uint8_t *d_hdr = (uint8_t *)c->get(WS_HDR, (size_t)nb * 352 + 64);
    c->h2d(d_roffs, rec_offs, (nb + 1) * 8);
    BMH_LAUNCH(c, "dec_headers", k_gather_headers, nb, 64, 0, d_rec, d_roffs, d_hdr);
    std::vector<uint8_t> hdr((size_t)nb * 352);
    c->d2h(hdr.data(), d_hdr, hdr.size());
    c->sync();
    std::vector<DBlock> hb(nb);
    std::vector<DecTable> tabs(nb);
    std::vector<uint32_t> seg_block, sp_block, ch_block;
    std::vector<IChunk> ich;
    out_offs[0] = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint8_t *h = &hdr[(size_t)b * 352];
        const uint64_t len = rec_offs[b + 1] - rec_offs[b];
        if (len < kRecordHeader) fail(BMH_ECORRUPT, "record " + std::to_string(b) + ": shorter than its header");
        const uint64_t prim = get_u64(h), n = get_u64(h + 8), tlen = get_u64(h + 16);
        if (n == 0 || n >= 0xffffffffull) fail(BMH_ECORRUPT, "record " + std::to_string(b) + ": bad n");
        if (tlen == 0 || tlen > 320 || tlen > len - kRecordHeader)
            fail(BMH_ECORRUPT, "record " + std::to_string(b) + ": bad tree length");
        if (prim >= n) fail(BMH_ECORRUPT, "record " + std::to_string(b) + ": primary index out of range");
        build_dec_table(h + kRecordHeader, tlen, &tabs[b]);
        // n < 2^32 bounds a Huffman tree's depth far below 64 (Fibonacci growth of the weights)
        if (tabs[b].maxlen > 64) fail(BMH_ECORRUPT, "record " + std::to_string(b) + ": code longer than 64 bits");
        DBlock &B = hb[b];
        B.pay = d_rec + rec_offs[b] + kRecordHeader + tlen;
        B.pay_bits = (len - kRecordHeader - tlen) * 8;
        if (!tabs[b].single && n > B.pay_bits) fail(BMH_ECORRUPT, "record " + std::to_string(b) + ": n exceeds payload");
        B.n = (uint32_t)n;
        B.primary = (uint32_t)prim;
        B.out_off = out_offs[b];
        out_offs[b + 1] = out_offs[b] + n;
        B.seg0 = (uint32_t)seg_block.size();
        B.nseg = tabs[b].single ? 0u : (uint32_t)((B.pay_bits + kSegBits - 1) / kSegBits);
        seg_block.insert(seg_block.end(), B.nseg, b);
        seg_block.resize((seg_block.size() + 255) & ~(size_t)255, kNil);  // workgroups stay in one block
        B.sp0 = (uint32_t)sp_block.size();
        B.nsp = (uint32_t)((n + kSplit - 1) / kSplit) + 1;
        sp_block.insert(sp_block.end(), B.nsp, b);
        B.ch0 = (uint32_t)ch_block.size();
        B.nch = (uint32_t)((n + kLfChunk - 1) / kLfChunk);
        ch_block.insert(ch_block.end(), B.nch, b);
        for (uint32_t k = 0; k < B.nch; ++k) {
            const uint64_t s = (uint64_t)k * kImtfChunk;
            ich.push_back(IChunk{b, (uint32_t)(B.out_off + s), (uint32_t)std::min<uint64_t>(kImtfChunk, n - s), 0});
        }
    }
    const uint64_t total = out_offs[nb];
    if (total > out_cap) fail(BMH_ERANGE, "decode: output capacity too small");
    if (total >= 0xffffffffull) fail(BMH_ERANGE, "decode: batch output must be < 4 GiB");
    const uint32_t nseg = (uint32_t)seg_block.size(), nsp = (uint32_t)sp_block.size(), nch = (uint32_t)ch_block.size();

    // ---- device tables
    DBlock *d_blk = (DBlock *)c->get(WS_BLOCKS, nb * sizeof(DBlock) + 64);
    c->ws_tag[WS_BLOCKS] = c->ws_tag[WS_MTF_CHUNKS] = 0;  // the encode's cached tables are overwritten
    DecTable *d_tab = (DecTable *)c->get(WS_TABLES, nb * sizeof(DecTable) + 64);
    uint8_t *d_meta = (uint8_t *)c->get(WS_MTF_CHUNKS, (size_t)(nseg + nsp + nch) * 4 + nch * sizeof(IChunk) + 256);
    uint32_t *d_seg_block = (uint32_t *)d_meta;
    uint32_t *d_sp_block = d_seg_block + nseg;
    uint32_t *d_ch_block = d_sp_block + nsp;
    IChunk *d_ich = (IChunk *)(((uintptr_t)(d_ch_block + nch) + 15) & ~(uintptr_t)15);
    c->h2d(d_blk, hb.data(), nb * sizeof(DBlock));
    c->h2d(d_tab, tabs.data(), nb * sizeof(DecTable));
    if (nseg) c->h2d(d_seg_block, seg_block.data(), nseg * 4);
    c->h2d(d_sp_block, sp_block.data(), nsp * 4);
    c->h2d(d_ch_block, ch_block.data(), nch * 4);
    c->h2d(d_ich, ich.data(), nch * sizeof(IChunk));
    uint32_t *d_status = (uint32_t *)c->get(WS_STATUS, 256);
    c->ws_tag[WS_STATUS] = 0;  // the encode's status word / block offsets (capi.cpp) are rewritten
    BMH_HIP(hipMemsetAsync(d_status, 0, 16, c->stream));

    // ---- Huffman^-1 -> d_mtf (batch layout = output layout)
    uint8_t *d_mtf = (uint8_t *)c->get(WS_MTF, total + 64);
    for (uint32_t b = 0; b < nb; ++b)
        if (tabs[b].single)
            BMH_LAUNCH(c, "dec_single", k_hd_single, std::min<uint32_t>(1024, cdiv(hb[b].n, 256)), 256, 0, d_blk, d_tab,
                       b, d_mtf);
    if (nseg) {
        uint64_t *d_end = (uint64_t *)c->get(WS_SA, (size_t)nseg * 16 + 64);
        uint64_t *d_end2 = d_end + nseg;
        uint64_t *d_start = (uint64_t *)c->get(WS_SA2, (size_t)nseg * 8 + 64);
        uint32_t *d_cnt = (uint32_t *)c->get(WS_OFFS, (size_t)nseg * 4 + 64);
        uint16_t *d_bnd = (uint16_t *)c->get(WS_CHIST, (size_t)nseg * kSyncBnd * 2 + 64);
        BMH_LAUNCH(c, "dec_huff_pass1", k_hd_pass1, cdiv(nseg, 256), 256, 0, d_blk, d_tab, d_seg_block, nseg, d_end,
                   d_cnt, d_bnd);
        // pass-1 starts are the nominal segment starts
        std::vector<uint64_t> st0(nseg, 0);
        for (uint32_t b = 0; b < nb; ++b)
            for (uint32_t k = 0; k < hb[b].nseg; ++k) st0[hb[b].seg0 + k] = (uint64_t)k * kSegBits;
        c->h2d(d_start, st0.data(), nseg * 8);
        // the offset-0 decode of every segment, kept for the fallback below
        uint64_t *d_end0 = (uint64_t *)c->get(WS_KEY8, (size_t)nseg * 12 + 64);
        uint32_t *d_cnt0 = (uint32_t *)(d_end0 + nseg);
        BMH_HIP(hipMemcpyAsync(d_end0, d_end, (size_t)nseg * 8, hipMemcpyDeviceToDevice, c->stream));
        BMH_HIP(hipMemcpyAsync(d_cnt0, d_cnt, (size_t)nseg * 4, hipMemcpyDeviceToDevice, c->stream));
        uint32_t *d_changed = d_status + 1;
        uint32_t h_changed = 1;
        for (int round = 0; h_changed && round < kFixRounds; ++round) {
            BMH_HIP(hipMemsetAsync(d_changed, 0, 4, c->stream));
            BMH_LAUNCH(c, "dec_huff_fix", k_hd_fix, cdiv(nseg, 256), 256, 0, d_blk, d_tab, d_seg_block, nseg, d_end,
                       d_end2, d_start, d_cnt, d_bnd, d_changed);
            std::swap(d_end, d_end2);
            c->d2h(&h_changed, d_changed, 4);
            c->sync();
        }
        if (h_changed) {
            // not settled: every entry offset of every segment, then one chained walk per block
            uint32_t P = 2;
            for (uint32_t b = 0; b < nb; ++b)
                while (hb[b].nseg && P < tabs[b].maxlen) P <<= 1;
            uint32_t *d_map = (uint32_t *)c->get(WS_RKA, (size_t)nseg * P * 4 + 64);
            BMH_LAUNCH(c, "dec_huff_map", k_hd_map, (uint32_t)cdiv((uint64_t)nseg * P, 256), 256, 0, d_blk, d_tab,
                       d_seg_block, nseg, P, d_end0, d_cnt0, d_bnd, d_map);
            BMH_LAUNCH(c, "dec_huff_chain", k_hd_chain, nb, 64, 0, d_blk, P, d_map, d_start, d_cnt, d_status);
        }
        BMH_LAUNCH(c, "dec_huff_scan", k_hd_scan, nb, 256, 0, d_blk, d_cnt);
        BMH_LAUNCH(c, "dec_huff_pass3", k_hd_pass3, cdiv(nseg, 256), 256, 0, d_blk, d_tab, d_seg_block, nseg, d_start,
                   d_cnt, d_mtf, d_status);
    }

    // ---- MTF^-1 -> d_L
    uint8_t *d_L = (uint8_t *)c->get(WS_L, total + 64);
    uint8_t *d_perm = (uint8_t *)c->get(WS_MTF_R, (size_t)nch * 256 + 64);
    uint8_t *d_S = (uint8_t *)c->get(WS_MTF_S, (size_t)nch * 256 + 64);
    BMH_LAUNCH(c, "dec_imtf_perm", k_imtf<0>, cdiv(nch, kImtfLanes), kImtfLanes, 0, d_mtf, d_ich, nch, nullptr, d_perm);
    BMH_LAUNCH(c, "dec_imtf_compose", k_imtf_compose, nb, 64, 0, d_blk, d_perm, d_S);
    BMH_LAUNCH(c, "dec_imtf", k_imtf<1>, cdiv(nch, kImtfLanes), kImtfLanes, 0, d_mtf, d_ich, nch, d_S, d_L);

    // ---- BWT^-1 -> d_out
    bool small = true;
    uint32_t max_nsp = 1;
    for (uint32_t b = 0; b < nb; ++b) {
        small &= hb[b].n <= (1u << 24);
        max_nsp = std::max(max_nsp, hb[b].nsp);
    }
    if (small)
        lf_inverse<uint32_t>(c, hb, nb, total, nsp, nch, max_nsp, d_L, d_blk, d_ch_block, d_sp_block, d_out, d_status);
    else
        lf_inverse<uint64_t>(c, hb, nb, total, nsp, nch, max_nsp, d_L, d_blk, d_ch_block, d_sp_block, d_out, d_status);
    uint32_t st = 0;
    c->d2h(&st, d_status, 4);
    c->sync();
    if (st & 1u) fail(BMH_ECORRUPT, "decode: payload ends before n symbols");
    if (st & 2u) fail(BMH_ECORRUPT, "decode: corrupt BWT (LF cycle)");
}

}  // namespace bmh
