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
//                counted in two levels: the marks of the 64-slot words above (8 byte counters
//                in a VGPR pair, one masked byte sum), the marks above in c's word (one 64-bit
//                shift, two popcounts). An access clears one mark and sets the next slot —
//                O(1) work instead of moving up to 255 list entries; the window is renumbered
//                every 256 symbols (new slot = marks below the old one). Stamps are stored as a
//                byte + an "accessed this epoch" bit (352 B of state per lane: seven one-wave
//                workgroups a CU), branch-free steps (~30 VALU + 7 LDS ops per symbol, ~10 VALU
//                a symbol per renumbering; 1.89 ms per GiB on MI355X, round 5: 2.5 ms with 10
//                LDS ops and 6 workgroups a CU; whole-wave list updates: 28-40 ms).
//   4. hist    : freq + first occurrence of each MTF value per block (LDS atomics).
#include "bmh_internal.h"

#include <atomic>
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

constexpr uint32_t kMtfChunk = 4096;  // symbols per lane (one chunk)

// Chunk length used by the host tables (<= kMtfChunk, a multiple of 64; the kernels take any
// such length). One lane walks a chunk and every lane takes the same time per symbol, so the
// encode runs in rounds of resident lanes (kMtfWgPerCu one-wave workgroups per CU, LDS-bound)
// and costs rounds x chunk length steps. The length is chosen so the batch's chunks fill whole
// rounds: R = the rounds kMtfChunk-symbol chunks need, then the shortest length (>=
// kMtfChunkMin) whose chunks fit in R rounds. 4096-symbol chunks put 1 GiB of 4 MiB blocks in
// 2.67 rounds, i.e. 3 rounds of 4096 steps; 3648-symbol chunks fill 3 rounds of 3648. A 256 MiB
// batch in four pipelines: each 256 MiB sub-batch gets a quarter of the slots (3 rounds of 3648).
// 128 MiB (the strong-scaling N = 8 share) fits one round of 1408 instead of a third of a round
// of 4096.
// BMH_OPT_MTF_CHUNK (bmh_ctx_set_option) overrides it for experiments.
constexpr uint32_t kMtfChunkMin = 256;
constexpr uint32_t kMtfWgPerCu = 7;  // k_mtf_encode: 22 KB of LDS per one-wave workgroup
static uint64_t mtf_chunk_count(const Batch &bt, uint64_t x)
{
    uint64_t k = 0;
    for (uint32_t b = 0; b < bt.nblocks; ++b) {
        const uint64_t o = bt.offs[b], n = bt.offs[b + 1] - o;
        const uint64_t pre = std::min<uint64_t>(n, (64 - (o & 63u)) & 63u);  // unaligned first chunk
        k += (pre != 0) + (n - pre + x - 1) / x;
    }
    return k;
}
static uint32_t mtf_chunk_len(Ctx *c, const Batch &bt)
{
    if (c->opt.mtf_chunk) return (uint32_t)c->opt.mtf_chunk;
    const uint64_t sig = layout_sig(4, bt.offs, 0) ^ (c->screen_total * 0x9e3779b97f4a7c15ull);
    if (c->mtf_clen_sig == sig) return c->mtf_clen;
    // a pipeline's sub-batch (capi.cpp encode_blocks) gets its byte share of the lane slots: the
    // pipelines' encodes share the device (each filling it alone made a 128 MiB batch's four
    // pipelines walk 384-symbol chunks, 11 K chunks a block through the composition)
    const uint64_t whole = c->screen_total > bt.total ? c->screen_total : bt.total;
    const uint64_t slots = std::max<uint64_t>(64, (uint64_t)std::max(c->cus, 1) * kMtfWgPerCu * 64 * bt.total / whole);
    const uint64_t R = std::max<uint64_t>(1, (mtf_chunk_count(bt, kMtfChunk) + slots - 1) / slots);
    uint64_t x = std::max<uint64_t>(kMtfChunkMin, ((bt.total + R * slots - 1) / (R * slots) + 63) & ~63ull);
    while (x < kMtfChunk && mtf_chunk_count(bt, x) > R * slots) x += 64;
    x = std::min<uint64_t>(x, kMtfChunk);
    c->mtf_clen_sig = sig;
    c->mtf_clen = (uint32_t)x;
    return (uint32_t)x;
}
constexpr int kLanes = 64;            // lanes (chunks) per encode workgroup (one wave)

// Bytes [src, src + nv) (nv <= 64) into sw[16], zero past nv, from the 17 aligned dwords that
// cover them: every load in flight at once (a byte loop waits for each load in turn), the bytes
// funnel-shifted out; a dword past the last byte is read byte by byte (no read past the end).
__device__ __forceinline__ void load64_any(const uint8_t *src, uint32_t nv, uint32_t (&sw)[16])
{
    const uintptr_t p0 = (uintptr_t)src, pa = p0 & ~(uintptr_t)3, end = p0 + nv;
    const uint32_t sh = 8u * (uint32_t)(p0 & 3u);
    uint32_t dw[17];
#pragma unroll
    for (uint32_t q = 0; q < 17; ++q) {
        const uintptr_t qa = pa + 4 * q;
        uint32_t x = 0;
        if (qa + 4 <= end) {
            x = *(const uint32_t *)qa;
        } else if (qa < end) {
#pragma unroll
            for (uint32_t k = 0; k < 3; ++k)
                if (qa + k < end) x |= (uint32_t)((const uint8_t *)qa)[k] << (8 * k);
        }
        dw[q] = x;
    }
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) sw[q] = (uint32_t)(((uint64_t)dw[q + 1] << 32 | dw[q]) >> sh);
}

struct MChunk {
    uint32_t block, start, len, rel;  // rel = start - block offset
};

// One wave per chunk (four per workgroup, no workgroup barriers). R[c][0..d) = distinct
// symbols, most recent last occurrence first: LDS atomicMax of positions, a bitset of
// last-occurrence positions (lane l owns the 64 positions from 64l), then each symbol's rank =
// set bits above its last position (wave scan + one popcount), and the symbol is stored at its
// rank. The chunk is walked from its END in groups of 64 dwords (lane l: dword nd - 64 (g + 1)
// + l; every group's coalesced 256-byte load issued up front). Going backwards, a symbol's last
// occurrence lies in the first group that holds it, so once all 256 symbols have been seen no
// earlier byte can change a last position and the walk stops: a uniform-like chunk (random
// data) has met every byte value ~1.6 K symbols before its end (coupon collector), about half
// of a 3 K-symbol chunk. The values met are counted every 1 K symbols (four LDS reads a lane
// and ballots; atomics that return the old position cost their waits on every chunk, text's
// too). Round 6: 0.38 -> 0.33 ms per GiB (a persistent variant that loaded the next chunk
// during the current one: 0.41 ms, 88 VGPRs, 5 waves a SIMD instead of 8).
// (also resets what k_mtf_hist accumulates: the block histograms and first pack chunks; no
// memset launches). kRuns: one atomicMax per run of equal symbols (text); batches found dense
// (uniform-like bytes: no runs to save, and the check costs a third more VALU) take the plain loop.
template <bool kRuns>
__global__ __launch_bounds__(256) void k_mtf_recency(const uint8_t *__restrict__ L, const MChunk *__restrict__ chunks,
                                                     uint32_t nch, uint8_t *__restrict__ R, uint32_t *__restrict__ dcount,
                                                     uint32_t *__restrict__ freq, uint32_t *__restrict__ firstc,
                                                     uint32_t nfreq)
{
    __shared__ int lastpos[4][256 + (kRuns ? 64 : 0)];  // kRuns: + a sink slot per lane
    __shared__ uint32_t bset[4][kMtfChunk / 32];
    __shared__ uint32_t above[4][64];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nfreq; i += gridDim.x * 256) {
        freq[i] = 0;
        firstc[i] = 0xffffffffu;
    }
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u, c = blockIdx.x * 4 + w;
    if (c >= nch) return;  // the whole wave
    static_assert(kMtfChunk == 16 * 256, "k_mtf_recency: 16 groups of 64 dwords cover a chunk");
    // a chunk's dwords, group g in x[g]; aligned chunks read whole dwords (the index clamped at
    // the chunk start; a last dword past the chunk end stays inside the 256-byte-rounded
    // allocation), a block's first chunk that starts mid-dword (< 64 bytes) byte by byte
    auto load_chunk = [&](const MChunk &m, uint32_t (&x)[16]) {
        const uint32_t nd = (m.len + 3) >> 2;
        if ((m.start & 3u) == 0) {
            const uint32_t *s32 = (const uint32_t *)(L + m.start);
#pragma unroll
            for (uint32_t g = 0; g < 16; ++g) x[g] = s32[max((int)nd - 64 * (int)(g + 1) + (int)l, 0)];
        } else {
            const int i = (int)nd - 64 + (int)l;
            uint32_t v = 0;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
                if (i >= 0 && 4u * (uint32_t)i + k < m.len) v |= (uint32_t)L[m.start + 4u * (uint32_t)i + k] << (8 * k);
            x[0] = v;
#pragma unroll
            for (uint32_t g = 1; g < 16; ++g) x[g] = 0;
        }
    };
    const MChunk ch = chunks[c];
    uint32_t x[16];
    load_chunk(ch, x);
    {
#pragma unroll
        for (int k = 0; k < 4; ++k) lastpos[w][4 * l + k] = -1;
        bset[w][2 * l] = 0;
        bset[w][2 * l + 1] = 0;
        wave_sync();
        const uint32_t len = ch.len, nd = (len + 3) >> 2, ng = (nd + 63) >> 6;
        bool done = false;  // every byte value met (uniform)
#pragma unroll
        for (uint32_t g = 0; g < 16; ++g) {
            if (g < ng && !done) {  // uniform
                const int i = (int)nd - 64 * (int)(g + 1) + (int)l;
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    // a symbol followed by itself in the dword is not its last occurrence there:
                    // one atomic per run of equal symbols (a text block's last column is mostly runs)
                    const int pos = 4 * i + (int)k;
                    const uint32_t s = (x[g] >> (8 * k)) & 255u;
                    const bool again = kRuns && k < 3 && (uint32_t)pos + 1 < len && ((x[g] >> (8 * (k + 1))) & 255u) == s;
                    if (pos >= 0 && (uint32_t)pos < len)
                        atomicMax(&lastpos[w][again ? 256 + l : s], pos);  // (repeats: the lane's sink)
                }
                if ((g & 3u) == 3u && g + 1 < ng) {  // every 1 K symbols: all 256 values met yet?
                    wave_sync();
                    uint32_t met = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) met += (uint32_t)__builtin_popcountll(__ballot(lastpos[w][4 * l + k] >= 0));
                    done = met == 256;
                }
            }
        }
        wave_sync();
        uint32_t d = 0;
        int lp[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            lp[k] = lastpos[w][4 * l + k];
            if (lp[k] >= 0) atomicOr(&bset[w][lp[k] >> 5], 1u << (lp[k] & 31));
            d += lp[k] >= 0;
        }
        wave_sync();
        d = wave_sum_dpp(d);
        const uint64_t v = ((uint64_t)bset[w][2 * l + 1] << 32) | bset[w][2 * l];
        const uint32_t cnt = (uint32_t)__builtin_popcountll(v);
        above[w][l] = d - wave_incl_sum_dpp(cnt);  // set bits in lanes above this one
        wave_sync();
        uint8_t *Rc = R + (size_t)c * 256;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (lp[k] >= 0) {
                const uint32_t ol = (uint32_t)lp[k] >> 6, b = (uint32_t)lp[k] & 63u;
                const uint64_t ov = ((uint64_t)bset[w][2 * ol + 1] << 32) | bset[w][2 * ol];
                Rc[above[w][ol] + (uint32_t)__builtin_popcountll((ov >> b) >> 1)] = (uint8_t)(4 * l + k);
            }
        if (l == 0) dcount[c] = d;
    }
}

// Composition of recency lists. A list R (the distinct symbols of a span, most recent first,
// d entries) acts on an MTF state as S -> R ++ (S minus R), and two spans compose into a list
// of the same kind (later ++ (earlier minus later)), so chunk start states come from three
// short sequential levels instead of one walk over all of a block's chunks:
//   1. per superchunk (kSuper chunks): compose its chunk lists from the empty state -> the
//      superchunk's list (its "touched" prefix, d' entries);
//   2. per block: walk its superchunk lists from the identity alphabet -> each superchunk's
//      start state;
//   3. per superchunk: walk its chunk lists from that start -> each chunk's start state.
// One wave per run; a lane holds state positions 4l .. 4l + 3. The lists are fetched 32 steps
// ahead into registers and parked in LDS, so the sequential chain never waits on memory.
constexpr uint32_t kComposeBatch = 32;
constexpr uint32_t kSuper = 32;  // chunks per superchunk
constexpr uint32_t kFiveLevel = 1024;  // chunks per block past which the composition takes five levels

struct CRun {
    uint32_t c0, c1;  // list indices [c0, c1)
    uint32_t start;   // start state index (Sin), or kIdentity
    uint32_t out;     // final list index (Rout / dout)
};
constexpr uint32_t kIdentity = 0xffffffffu;

// kSteps: write the state BEFORE each step to Sout[list index]; kFinal: write the final state's
// touched prefix to Rout[run.out] and its length to dout[run.out].
template <bool kSteps, bool kFinal>
__global__ __launch_bounds__(64) void k_mtf_compose(const CRun *__restrict__ runs, const uint8_t *__restrict__ R,
                                                    const uint32_t *__restrict__ dcount,
                                                    const uint32_t *__restrict__ Sin, uint32_t *__restrict__ Sout,
                                                    uint8_t *__restrict__ Rout, uint32_t *__restrict__ dout)
{
    __shared__ uint32_t s_R[kComposeBatch][64];
    __shared__ uint32_t s_d[kComposeBatch];
    // slots 256 + l: each lane's sink for masked-off stores (the step runs unbranched). One wave
    // per workgroup: the steps' LDS hand-offs need only wave_sync (LDS executes a wave's
    // operations in order; no wait for the stores before the loads that read them)
    __shared__ uint8_t s_S[256 + 64], s_flag[256 + 64];
    const CRun run = runs[blockIdx.x];
    const uint32_t l = threadIdx.x, c0 = run.c0, c1 = run.c1;
    const uint32_t *R32 = (const uint32_t *)R;
    uint32_t st[4];
    if (run.start == kIdentity) {
        for (int k = 0; k < 4; ++k) st[k] = 4 * l + k;
    } else {
        const uint32_t w = Sin[(size_t)run.start * 64 + l];
        for (int k = 0; k < 4; ++k) st[k] = (w >> (8 * k)) & 255u;
    }
    uint32_t dt = 0;  // touched prefix of the state (kFinal: the run started empty)
    uint32_t pre[kComposeBatch], pred = 0;
    auto fetch = [&](uint32_t cb) {
#pragma unroll
        for (uint32_t j = 0; j < kComposeBatch; ++j)
            pre[j] = cb + j < c1 ? R32[(size_t)(cb + j) * 64 + l] : 0u;
        pred = (l < kComposeBatch && cb + l < c1) ? dcount[cb + l] : 0u;
    };
    fetch(c0);
    const uint32_t sink = 256 + l;
    for (uint32_t cb = c0; cb < c1; cb += kComposeBatch) {
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kComposeBatch; ++j) s_R[j][l] = pre[j];
        if (l < kComposeBatch) s_d[l] = pred;
        __syncthreads();
        if (cb + kComposeBatch < c1) fetch(cb + kComposeBatch);
        const uint32_t ce = min(c1, cb + kComposeBatch);
        uint32_t d = s_d[0], rw = s_R[0][l];  // this step's list; the next one is read with the state
        for (uint32_t c = cb; c < ce; ++c) {
            if (kSteps) Sout[(size_t)c * 64 + l] = st[0] | (st[1] << 8) | (st[2] << 16) | (st[3] << 24);
            *(uint32_t *)&s_flag[4 * l] = 0;
            wave_sync();
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) s_flag[4 * l + k < d ? (rw >> (8 * k)) & 255u : sink] = 1;
            wave_sync();
            uint32_t keep[4], cnt = 0, kt = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                keep[k] = s_flag[st[k]] == 0;
                cnt += keep[k];
                kt += keep[k] && 4 * l + k < dt;
            }
            if (kFinal) dt = d + wave_sum_dpp(kt);
            uint32_t pos = d + wave_incl_sum_dpp(cnt) - cnt;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                s_S[keep[k] ? pos : sink] = (uint8_t)st[k];
                pos += keep[k];
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) s_S[4 * l + k < d ? 4 * l + k : sink] = (uint8_t)(rw >> (8 * k));
            wave_sync();
            const uint32_t cn = c + 1 < ce ? c + 1 - cb : 0u;
            d = s_d[cn];
            rw = s_R[cn][l];
#pragma unroll
            for (int k = 0; k < 4; ++k) st[k] = s_S[4 * l + k];
            wave_sync();
        }
    }
    if (kFinal) {
        uint8_t *ro = Rout + (size_t)run.out * 256;
        for (int k = 0; k < 4; ++k)
            if (4 * l + k < dt) ro[4 * l + k] = (uint8_t)st[k];
        if (l == 0) dout[run.out] = dt;
    }
}

// Per-lane encode state in LDS, every lane in its own banks (row k of lane l = the dword at byte
// k * 256 + 4l; the marks are 64-bit rows: word w of lane l = the 8 bytes at kOffMarks + 512w + 8l):
//   rows 0..63  stamp bytes: the low 8 bits of symbol c's slot, byte c & 3 of row c >> 2
//   rows 64..71 epoch bits : bit 8 of the slot ("accessed since the last renumbering"),
//                            bit c & 31 of row 64 + (c >> 5)
//   marks       512 slot marks as eight 64-bit words: slot t is some symbol's last access
// and, in a VGPR pair, the number of marks in each 64-slot word (byte w of C). The MTF index of
// slot t = marks above t in its word (one 64-bit shift, two popcounts) + the counts of the words
// above (two masked byte sums). 352 B per lane, so seven one-wave workgroups fit a CU; a symbol
// costs 7 LDS operations (stamp, epoch and marks-word reads; mark clear, new mark, stamp, epoch).
// (Round 5's layout kept the 32-slot word counts in LDS: 368 B per lane, six workgroups a CU, 10
// LDS operations a symbol; LDS atomics cost what plain stores cost, tools/microbench/lds_ops.hip.)
constexpr uint32_t kRowEp = 64, kOffMarks = 72 * 256, kEncLds = kOffMarks + 8 * 512;  // 22528 B per wave
static_assert(kMtfWgPerCu * kEncLds <= 160 * 1024, "k_mtf_encode: LDS for kMtfWgPerCu workgroups a CU");

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *s, uint32_t a) { return *(const uint32_t *)(s + a); }
__device__ __forceinline__ uint64_t lds_u64(const uint8_t *s, uint32_t a) { return *(const uint64_t *)(s + a); }
__device__ __forceinline__ uint32_t a8_of(uint32_t c, uint32_t l4) { return ((c << 6) & 0x3F00u) | l4 | (c & 3u); }
__device__ __forceinline__ uint32_t ae_of(uint32_t c, uint32_t l4) { return (kRowEp << 8) + (((c >> 5) << 8) | l4); }
// marks above slot t given t's marks word W and the word counts C; the own mark is counted by the
// shift and taken off by the accumulator's start value (-1)
__device__ __forceinline__ uint32_t rank_words(uint64_t C, uint32_t t)
{
    const uint64_t M = 0xFFFFFFFFFFFFFF00ull << ((t >> 3) & 0x38u);
    const uint32_t r = __builtin_amdgcn_sad_u8((uint32_t)C & (uint32_t)M, 0u, 0xFFFFFFFFu);
    return __builtin_amdgcn_sad_u8((uint32_t)(C >> 32) & (uint32_t)(M >> 32), 0u, r);
}
// v_bcnt_u32_b32 with its accumulator (the compiler emits bcnt(x, 0) twice and an add3)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
__device__ __forceinline__ uint32_t rank_bits(uint64_t W, uint32_t t, uint32_t acc)
{
    const uint64_t ws = W >> (t & 63u);
    return bcnt_acc((uint32_t)(ws >> 32), bcnt_acc((uint32_t)ws, acc));
}
// (a & 4) | b in one v_and_or_b32 (the compiler splits it into an and and an add)
__device__ __forceinline__ uint32_t and4_or(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_and_or_b32 %0, %1, 4, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// MTF of symbol c at the wave-uniform slot `slot` (256..511). Returns the index; the state update
// (old mark cleared, new mark set, stamp rewritten) happens only for valid symbols.
template <bool kPred>
__device__ __forceinline__ uint32_t mtf_step(uint32_t c, bool valid, uint32_t slot, uint8_t *s, uint32_t l4, uint32_t l8,
                                             uint64_t &C)
{
    const uint32_t a8 = a8_of(c, l4), ae = ae_of(c, l4);
    const uint32_t lo = s[a8];
    const uint32_t e = lds_u32(s, ae);
    const uint32_t t = lo | (((e >> (c & 31u)) & 1u) << 8);
    const uint32_t am = kOffMarks + ((t >> 6) << 9) + l8;
    const uint64_t W = lds_u64(s, am);
    const uint32_t r = rank_bits(W, t, rank_words(C, t));
    if (!kPred || valid) {
        atomicXor((uint32_t *)(s + am + ((t >> 3) & 4u)), 1u << (t & 31u));
        C += ~0ull << ((t >> 3) & 0x38u);
        atomicOr((uint32_t *)(s + kOffMarks + ((slot >> 6) << 9) + l8 + ((slot >> 3) & 4u)), 1u << (slot & 31u));
        C += 1ull << (8 * (slot >> 6));
        s[a8] = (uint8_t)slot;
        atomicOr((uint32_t *)(s + ae), 1u << (c & 31u));
    }
    return r;
}

// A whole super-group (symbols j = 0..63 at slots now + j; now is a multiple of 64, so the group's
// new marks fill one 64-bit word), software-pipelined: symbol j + 1's stamp and epoch reads are
// issued before symbol j's state update, and symbol j's marks word is consumed only one symbol
// later, so each symbol waits on one LDS round trip that overlaps its neighbours' work. A read-ahead
// stamp predates the previous symbol's update, so a symbol equal to its predecessor takes the
// predecessor's slot (the only stamp that update can change). Same results as mtf_step.
__device__ __forceinline__ void mtf_whole(const uint4 (&in)[4], uint32_t now, uint8_t *s, uint32_t l4, uint32_t l8,
                                          uint64_t &C, uint4 (&o4)[4])
{
    const uint32_t iw[16] = {in[0].x, in[0].y, in[0].z, in[0].w, in[1].x, in[1].y, in[1].z, in[1].w,
                             in[2].x, in[2].y, in[2].z, in[2].w, in[3].x, in[3].y, in[3].z, in[3].w};
    auto sym = [&](int j) { return (iw[j >> 2] >> (8 * (j & 3))) & 255u; };
    const uint32_t amn = kOffMarks + ((now >> 6) << 9) + l8;  // the group's marks word
    const uint64_t cinc = 1ull << (8 * (now >> 6));
    uint32_t ow[16];
    uint32_t plo[64], pe[64];  // read-ahead stamp bytes / epoch words (registers once unrolled)
    plo[0] = s[a8_of(sym(0), l4)];
    pe[0] = lds_u32(s, ae_of(sym(0), l4));
    uint64_t pW = 0;
    uint32_t pt = 0, pr = 0;  // the previous symbol's marks word, slot and word-count term
    uint32_t slot = now, pslot = now;  // this / the previous symbol's slot, in a VGPR (stamp data and forward)
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        const uint32_t c = sym(j);
        if (j + 1 < 64) {
            const uint32_t cn = sym(j + 1);
            plo[j + 1] = s[a8_of(cn, l4)];
            pe[j + 1] = lds_u32(s, ae_of(cn, l4));
        }
        uint32_t t = plo[j] | (__builtin_amdgcn_ubfe(pe[j], c & 31u, 1u) << 8);
        if (j >= 1) t = c == sym(j - 1) ? pslot : t;
        // marks word w = t >> 6 at byte (w << 9) | 8l, its 32-bit half (t >> 5) & 1 at + 4, the
        // word counts' byte at bit 8w
        const uint32_t t3 = t >> 3;
        const uint32_t am = ((t << 3) & 0xE00u) | l8;
        const uint64_t W = lds_u64(s, kOffMarks + am);
        const uint32_t rw = rank_words(C, t);
        atomicXor((uint32_t *)(s + kOffMarks + and4_or(t3, am)), 1u << (t & 31u));
        C += ~0ull << (t3 & 0x38u);
        atomicOr((uint32_t *)(s + amn + 4 * (j >> 5)), 1u << (j & 31));
        C += cinc;
        s[a8_of(c, l4)] = (uint8_t)slot;
        atomicOr((uint32_t *)(s + ae_of(c, l4)), 1u << (c & 31u));
        __builtin_amdgcn_sched_barrier(0);
        if (j > 0) {
            uint32_t r = rank_bits(pW, pt, pr);
            asm volatile("" : "+v"(r));  // computed here, not sunk to the stores (64 symbols' terms live)
            const int q = j - 1;
            ow[q >> 2] = (q & 3) ? ow[q >> 2] | (r << (8 * (q & 3))) : r;
        }
        pW = W;
        pt = t;
        pr = rw;
        pslot = slot;
        slot += 1;
        asm volatile("" : "+v"(slot));
    }
    ow[15] |= rank_bits(pW, pt, pr) << 24;
#pragma unroll
    for (int q = 0; q < 4; ++q) o4[q] = make_uint4(ow[4 * q], ow[4 * q + 1], ow[4 * q + 2], ow[4 * q + 3]);
}

// Slots 0..255 marked (the start alphabet or the renumbered window), epochs cleared.
__device__ __forceinline__ void window_reset(uint8_t *s, uint32_t l4, uint32_t l8, uint64_t &C)
{
#pragma unroll
    for (uint32_t w = 0; w < 8; ++w) *(uint64_t *)(s + kOffMarks + (w << 9) + l8) = w < 4 ? ~0ull : 0ull;
#pragma unroll
    for (uint32_t w = 0; w < 8; ++w) *(uint32_t *)(s + ((kRowEp + w) << 8) + l4) = 0u;
    C = 0x0000000040404040ull;
}

// The window is full (slot 512 reached): every symbol's new slot is the number of marks below its
// slot t (0..255, order kept) = the marks in words 0..w (w = t >> 6) minus the marks of word w at
// or above t's bit: Q[w] - popcount(W_w >> (t & 63)), with Q the byte prefix sums of C shifted one
// word down (Q[7] = 256 = 0 mod 256; a byte only overflows past the last marked word, which no
// symbol reads), picked by a v_perm byte select. The four symbols of a stamp dword get their word
// indices in one SIMD-within-a-register step (their epoch bits spread by one multiply), and their
// new bytes are packed by three v_perm. About 10 VALU and one 8-byte LDS read a symbol, every 256
// symbols (round 5's form: 16 VALU).
__device__ __forceinline__ void window_renumber(uint8_t *s, uint32_t l4, uint32_t l8, uint64_t &C)
{
    uint64_t P = C << 8;
    P += P << 8;
    P += P << 16;
    P += P << 32;
    const uint64_t Q = P >> 8;  // byte w = marks in words 0..w
    const uint32_t Qlo = (uint32_t)Q, Qhi = (uint32_t)(Q >> 32);
#ifndef BMH_PROBE_NORENUM  // timing probe: renumbering skipped (wrong output)
#pragma nounroll
    for (uint32_t w = 0; w < 8; ++w) {  // symbols 32w .. 32w + 31
        const uint32_t e = lds_u32(s, ((kRowEp + w) << 8) + l4);
        uint32_t tw[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) tw[j] = lds_u32(s, ((8 * w + j) << 8) + l4);
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            // byte b of wd4 = word index of symbol 4j + b: stamp bits 6..7, epoch bit as bit 2
            const uint32_t spread = (((e >> (4 * j)) & 15u) * 0x00810204u) & 0x04040404u;
            const uint32_t wd4 = ((tw[j] >> 6) & 0x03030303u) | spread;
            uint32_t nb[4];
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t sel = wd4 >> (8 * b);  // byte 0 = w (higher bytes: unused result bytes)
                const uint32_t sh = tw[j] >> (8 * b);  // low 6 bits = t & 63
                const uint64_t W = lds_u64(s, kOffMarks + (((sel & 7u) << 9) | l8));
                const uint64_t at = W >> (sh & 63u);
                nb[b] = __builtin_amdgcn_perm(Qhi, Qlo, sel) - (uint32_t)__builtin_popcount((uint32_t)(at >> 32)) -
                        (uint32_t)__builtin_popcount((uint32_t)at);
            }
            const uint32_t p01 = __builtin_amdgcn_perm(nb[1], nb[0], 0x0C0C0400u);
            const uint32_t p23 = __builtin_amdgcn_perm(nb[3], nb[2], 0x0C0C0400u);
            *(uint32_t *)(s + ((8 * w + j) << 8) + l4) = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
        }
    }
#endif
    window_reset(s, l4, l8, C);
}

// grid = ceil(chunks / 64); one lane per chunk. Chunks start 64-byte aligned except a block's
// (<= 63-byte) first chunk; all lanes step through 64-symbol super-groups in lockstep so that
// the slot counter (and the renumbering every 256 slots = every 4 super-groups) stays
// wave-uniform. A super-group wholly inside the chunk is loaded and stored as one 64-byte
// sector per lane (four 16-byte accesses back to back) and runs the branch-free step; edge
// super-groups predicate the symbols outside the chunk off (their slots stay unmarked, which is
// harmless: slots only order accesses).
__global__ __launch_bounds__(kLanes) void k_mtf_encode(const uint8_t *__restrict__ L, const MChunk *__restrict__ chunks,
                                                       uint32_t nch, const uint32_t *__restrict__ Sst,
                                                       uint8_t *__restrict__ out)
{
    __shared__ uint64_t st64[kEncLds / 8];
    uint8_t *s = (uint8_t *)st64;
    const uint32_t l = threadIdx.x, l4 = 4 * l, l8 = 8 * l;
    const uint32_t g = blockIdx.x * kLanes + l;
    const bool live = g < nch;
    const MChunk ch = live ? chunks[g] : MChunk{0, 0, 0, 0};
    if (live) {  // start alphabet: front symbol -> slot 255
        const uint32_t *stv = Sst + (size_t)g * 64;
        for (uint32_t k4 = 0; k4 < 64; ++k4) {
            const uint32_t w = stv[k4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t c = (w >> (8 * j)) & 255u;
                s[a8_of(c, l4)] = (uint8_t)(255 - (4 * k4 + j));
            }
        }
    }
    uint64_t C;
    uint32_t now = 256;
    window_reset(s, l4, l8, C);
    const uint32_t base = ch.start & ~63u, end = ch.start + ch.len;
    const uint32_t nsg = live ? (((end + 63u) & ~63u) - base) >> 6 : 0u;
    auto whole = [&](uint32_t gi) {
        const uint32_t a = base + 64 * gi;
        return gi < nsg && a >= ch.start && a + 64 <= end;
    };
    auto load_sg = [&](uint32_t gi, uint4 (&v)[4]) {
        if (whole(gi)) {
            const uint4 *p = (const uint4 *)(L + base + 64 * gi);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = p[q];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = make_uint4(0, 0, 0, 0);
        }
    };
    uint4 pf[4];
    load_sg(0, pf);
    for (uint32_t sg = 0; __builtin_amdgcn_ballot_w64(sg < nsg) != 0; ++sg) {
        const uint32_t a0 = base + 64 * sg;
        uint4 in[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) in[q] = pf[q];
        load_sg(sg + 1, pf);
        if (whole(sg)) {
            uint4 o4[4];
            mtf_whole(in, now, s, l4, l8, C, o4);
            uint4 *po = (uint4 *)(out + a0);
#pragma unroll
            for (int q = 0; q < 4; ++q) po[q] = o4[q];
        } else if (sg < nsg) {  // an edge super-group: symbols outside the chunk predicated off
#pragma nounroll
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t a = a0 + 16 * q;
                uint32_t iw[4] = {0, 0, 0, 0};
                for (uint32_t k = 0; k < 16; ++k)
                    if (a + k >= ch.start && a + k < end) iw[k >> 2] |= (uint32_t)L[a + k] << (8 * (k & 3));
                uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k) {
                    const uint32_t c = (iw[k >> 2] >> (8 * (k & 3))) & 255u;
                    const bool v = a + k >= ch.start && a + k < end;
                    o[k >> 2] |= (mtf_step<true>(c, v, now + 16 * q + k, s, l4, l8, C) & 255u) << (8 * (k & 3));
                }
                for (uint32_t k = 0; k < 16; ++k)
                    if (a + k >= ch.start && a + k < end) out[a + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
            }
        }
        now += 64;  // 256 + 64 per super-group: the window fills up exactly at a boundary
        // (not after the last super-group: a chunk of a multiple of 256 symbols — Calgary's
        // pipelines walk 256 — would renumber for nothing)
        if (now == 512 && __builtin_amdgcn_ballot_w64(sg + 1 < nsg) != 0) {
            window_renumber(s, l4, l8, C);
            now = 256;
        }
    }
}

struct HChunk {
    uint32_t block, start, len, rel;
};

// freq of each MTF value per block (huffman() main.cpp:231-237) and the histogram of every
// 4 K-symbol pack chunk (u16; the pack sizes its chunks from these instead of re-reading the
// MTF stream). One workgroup per 64 K symbols of a block; wave w takes pack chunk w (lane l:
// symbols [64l, 64l + 64), one 64-byte sector) with its own LDS histogram, no workgroup
// barrier until the block totals. firstc[b][v] = the first pack chunk holding v (atomicMin over
// the workgroups, skipped when the value held is already smaller); the first occurrences inside
// those chunks come from k_mtf_first. kRuns: MTF values 0 and 1 counted in registers (text).
template <bool kRuns>
__global__ __launch_bounds__(1024) void k_mtf_hist(const uint8_t *__restrict__ in, const HChunk *__restrict__ chunks,
                                                   const uint32_t *__restrict__ pfirst, uint32_t *__restrict__ freq,
                                                   uint16_t *__restrict__ chist, uint32_t *__restrict__ firstc)
{
    constexpr uint32_t NW = 65536 / kPackChunkSyms;
    __shared__ uint32_t h[NW][256];
    __shared__ uint32_t s_sink[kRuns ? NW : 1][64];
    const HChunk ch = chunks[blockIdx.x];
    const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63u;
    const uint32_t s0 = w * kPackChunkSyms;
#pragma unroll
    for (int k = 0; k < 4; ++k) h[w][4 * l + k] = 0;
    if (s0 < ch.len) {
        wave_sync();
        const uint32_t len = min(kPackChunkSyms, ch.len - s0), a = ch.start + s0, e0 = 64 * l;
        if (len == kPackChunkSyms && ((a + e0) & 15u) == 0) {
            uint32_t sw[16];
            const uint4 *p = (const uint4 *)(in + a + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = p[q];
                sw[4 * q] = v.x;
                sw[4 * q + 1] = v.y;
                sw[4 * q + 2] = v.z;
                sw[4 * q + 3] = v.w;
            }
            // values 0 and 1 (most of a text block's MTF output) counted in a register: LDS
            // atomics on one address from many lanes serialise
            if (kRuns) {
                // (branch-free: a 0 / 1 goes to the lane's own sink counter instead)
                uint32_t z01 = 0;
#pragma unroll
                for (uint32_t k = 0; k < 64; ++k) {
                    const uint32_t v = (sw[k >> 2] >> (8 * (k & 3))) & 255u;
                    z01 += v < 2 ? 1u << (16 * v) : 0u;
                    atomicAdd(v < 2 ? &s_sink[w][l] : &h[w][v], 1u);
                }
                z01 = wave_sum_dpp(z01);  // <= 4096 per value: two 16-bit fields
                wave_sync();
                if (l == 0) {
                    h[w][0] += z01 & 0xffffu;
                    h[w][1] += z01 >> 16;
                }
            } else {
#pragma unroll
                for (uint32_t k = 0; k < 64; ++k) atomicAdd(&h[w][(sw[k >> 2] >> (8 * (k & 3))) & 255u], 1u);
            }
        } else {
            // unaligned (a block that starts mid-dword: whole files, Calgary) or the block's last
            // chunk; kRuns: values 0 and 1 in registers here too (every chunk of a whole-file text
            // block comes this way: 64 lanes adding to one counter took Calgary's hist 45 us)
            uint32_t sw[16];
            const uint32_t nv = e0 < len ? min(64u, len - e0) : 0u;
            load64_any(in + a + e0, nv, sw);
            if (kRuns) {
                uint32_t z01 = 0;
#pragma unroll
                for (uint32_t k = 0; k < 64; ++k) {
                    const uint32_t v = (sw[k >> 2] >> (8 * (k & 3))) & 255u;
                    if (k < nv) {
                        z01 += v < 2 ? 1u << (16 * v) : 0u;
                        atomicAdd(v < 2 ? &s_sink[w][l] : &h[w][v], 1u);
                    }
                }
                z01 = wave_sum_dpp(z01);
                wave_sync();
                if (l == 0) {
                    h[w][0] += z01 & 0xffffu;
                    h[w][1] += z01 >> 16;
                }
            } else {
#pragma unroll
                for (uint32_t k = 0; k < 64; ++k)
                    if (k < nv) atomicAdd(&h[w][(sw[k >> 2] >> (8 * (k & 3))) & 255u], 1u);
            }
        }
        wave_sync();
        uint16_t *co = chist + (size_t)(pfirst[ch.block] + (ch.rel + s0) / kPackChunkSyms) * 256;
#pragma unroll
        for (int k = 0; k < 4; ++k) co[4 * l + k] = (uint16_t)h[w][4 * l + k];
    }
    __syncthreads();
    if (t < 256) {
        uint32_t tot = 0, fx = NW;
#pragma unroll
        for (uint32_t x = 0; x < NW; ++x) {
            tot += h[x][t];
            fx = fx == NW && h[x][t] ? x : fx;
        }
        if (tot) {
            atomicAdd(&freq[(size_t)ch.block * 256 + t], tot);
            uint32_t *fp = &firstc[(size_t)ch.block * 256 + t];
            const uint32_t cand = ch.rel / kPackChunkSyms + fx;
            if (cand < __atomic_load_n(fp, __ATOMIC_RELAXED)) atomicMin(fp, cand);  // values only fall
        }
    }
}

// First occurrence of each MTF value per block (huffman() main.cpp:238-244 orders the leaves
// by it). k_mtf_hist found the chunk each value first appears in (firstc); only those chunks are
// scanned (on random data: the block's first chunk alone), one wave per distinct chunk. A value
// has one first chunk, so the chunks are independent and need no order. Grid (blocks,
// kFirstWG): every workgroup of a block derives the same sorted list of distinct first chunks
// (a bitmap over the block's chunks) and scans entries k = 16 g + wave (mod 16 kFirstWG), so a
// block whose values first appear in many chunks (Calgary's text files, pic: 100-256) scans
// them kFirstWG times wider; the one workgroup that scans a value's chunk writes its position.
constexpr uint32_t kFirstNT = 1024, kFirstWG = 8, kFirstBmWords = 256;  // bitmap: blocks of <= 8192 chunks
__global__ __launch_bounds__(kFirstNT) void k_mtf_first(const uint8_t *__restrict__ in, const uint32_t *__restrict__ boffs,
                                                        const uint32_t *__restrict__ pfirst,
                                                        const uint32_t *__restrict__ freq,
                                                        const uint32_t *__restrict__ firstc, uint32_t *__restrict__ first)
{
    __shared__ uint32_t f[256], s_cv[256], s_list[256], s_nlist, s_bm[kFirstBmWords], s_tmp[kFirstNT / 64 + 1];
    const uint32_t b = blockIdx.x, g = blockIdx.y, t = threadIdx.x, w = t >> 6, l = t & 63u;
    const uint32_t c0 = pfirst[b], nc = pfirst[b + 1] - c0;
    const uint32_t o = boffs[b], n = boffs[b + 1] - o;
    const bool bitmap = nc <= 32 * kFirstBmWords;  // else workgroup 0 alone, leads by value order
    if (!bitmap && g != 0) return;                 // workgroup-uniform
    if (t == 0) s_nlist = 0;
    if (t < kFirstBmWords) s_bm[t] = 0;
    if (t < 256) {
        f[t] = 0xffffffffu;
        // first chunk holding t (block-relative); none for absent values
        s_cv[t] = freq[(size_t)b * 256 + t] ? firstc[(size_t)b * 256 + t] : 0xffffffffu;
    }
    __syncthreads();
    if (bitmap) {
        if (t < 256 && s_cv[t] != 0xffffffffu) atomicOr(&s_bm[s_cv[t] >> 5], 1u << (s_cv[t] & 31u));
        __syncthreads();
        // the distinct first chunks in increasing order (the same list in every workgroup)
        uint32_t bits = t < kFirstBmWords ? s_bm[t] : 0u;
        uint32_t pos = block_excl_sum1<kFirstNT>((uint32_t)__builtin_popcount(bits), s_tmp, &s_nlist);
        while (bits) {
            s_list[pos++] = 32 * t + (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1;
        }
    } else if (t < 256) {  // the smallest value of each distinct first chunk lists it
        const uint32_t cv = s_cv[t];
        bool lead = cv != 0xffffffffu;
        for (uint32_t u = 0; u < t && lead; ++u) lead = s_cv[u] != cv;
        if (lead) s_list[atomicAdd(&s_nlist, 1u)] = cv;
    }
    __syncthreads();
    const uint32_t nl = s_nlist;
    const uint32_t k0 = bitmap ? 16 * g + w : w, kstep = bitmap ? 16 * kFirstWG : kFirstNT / 64;
    static_assert(kPackChunkSyms == 64 * 64, "k_mtf_first: a wave's 64 lanes x 64 symbols cover one pack chunk");
    for (uint32_t k = k0; k < nl; k += kstep) {  // lane l: symbols [64l, 64l + 64) of the chunk
        const uint32_t cm = s_list[k], p0 = cm * kPackChunkSyms, len = min(kPackChunkSyms, n - p0);
        const uint32_t e0 = 64 * l;
        uint32_t sw[16];
        if (e0 + 64 <= len && ((o + p0 + e0) & 15u) == 0) {
            const uint4 *p = (const uint4 *)(in + o + p0 + e0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 v = p[q];
                sw[4 * q] = v.x;
                sw[4 * q + 1] = v.y;
                sw[4 * q + 2] = v.z;
                sw[4 * q + 3] = v.w;
            }
        } else {
            load64_any(in + o + p0 + e0, e0 < len ? min(64u, len - e0) : 0u, sw);
        }
        const uint32_t m = e0 < len ? min(64u, len - e0) : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 64; ++j) {  // (a value repeating the one before is not a first one)
            const uint32_t x = (sw[j >> 2] >> (8 * (j & 3))) & 255u;
            const bool again = j > 0 && ((sw[(j - 1) >> 2] >> (8 * ((j - 1) & 3))) & 255u) == x;
            if (j < m && !again && s_cv[x] == cm) atomicMin(&f[x], p0 + e0 + j);
        }
    }
    __syncthreads();
    // each present value's first chunk was scanned by exactly one workgroup; absent values by 0
    if (t < 256 && (f[t] != 0xffffffffu || (g == 0 && s_cv[t] == 0xffffffffu))) first[(size_t)b * 256 + t] = f[t];
}

}  // namespace

void mtf_batch(Ctx *c, const uint8_t *d_L, const Batch &bt, uint8_t *d_mtf, uint32_t *h_freq32, uint32_t *h_first32)
{
    const uint32_t nb = bt.nblocks;
    // chunk / composition tables: rebuilt and uploaded only when the batch layout changed
    const uint32_t clen = mtf_chunk_len(c, bt);
    const uint64_t sig = layout_sig(2, bt.offs, clen);
    uint32_t nch, nhh, ng, npk, ng2;
    if (c->ws_tag[WS_MTF_CHUNKS] == sig) {
        nch = c->ws_aux[WS_MTF_CHUNKS][0];
        nhh = c->ws_aux[WS_MTF_CHUNKS][1];
        ng = c->ws_aux[WS_MTF_CHUNKS][2];
        npk = c->ws_aux[WS_MTF_CHUNKS][3];
        ng2 = c->ws_aux[WS_MTF_CHUNKS][4];
    } else {
        std::vector<MChunk> hc;
        std::vector<HChunk> hh;
        std::vector<uint32_t> cfirst(nb + 1), pfirst(nb + 1);
        pack_chunk_first(bt, pfirst.data());
        for (uint32_t b = 0; b < nb; ++b) {
            cfirst[b] = (uint32_t)hc.size();
            const uint64_t o = bt.offs[b], n = bt.offs[b + 1] - o;
            // chunk boundaries on 64-byte multiples of the batch (a block's first chunk takes the
            // unaligned prefix) so the encode kernel moves whole 64-byte sectors per lane
            for (uint64_t s = 0; s < n;) {
                const uint64_t gpos = o + s;
                const uint64_t lim = (gpos & 63u) ? ((gpos + 63) & ~63ull) : gpos + clen;
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
        // composition runs. Three levels (kSuper-chunk superchunks composed, the block walks its
        // superchunk lists, each superchunk walks its chunk lists) cost sup + chunks / sup + sup
        // sequential steps; blocks of more than kFiveLevel chunks (short chunks of small
        // batches) add a middle level: groups of s superchunks composed, the block walks the
        // group lists, each group walks its superchunk lists — five walks of ~cbrt(chunks per
        // block) steps each (a 128 MiB batch's 2980-chunk blocks: 74 steps instead of 166).
        uint32_t cpb = 1;
        for (uint32_t b = 0; b < nb; ++b) cpb = std::max(cpb, cfirst[b + 1] - cfirst[b]);
        uint32_t sup = kSuper, s2 = 0;
        if (cpb > kFiveLevel) {
            sup = 8;
            while (sup * sup * sup < cpb) ++sup;
            s2 = sup;
        } else {
            while (sup * sup < cpb) sup += 8;
        }
        std::vector<CRun> r1, r2, r3, r1b, r2b;
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t g0 = (uint32_t)r1.size();
            for (uint32_t x = cfirst[b]; x < cfirst[b + 1]; x += sup) {
                const uint32_t g = (uint32_t)r1.size(), e = std::min(cfirst[b + 1], x + sup);
                r1.push_back(CRun{x, e, kIdentity, g});
                r3.push_back(CRun{x, e, g, g});
            }
            const uint32_t g1 = (uint32_t)r1.size();
            if (!s2) {
                r2.push_back(CRun{g0, g1, kIdentity, 0});
                continue;
            }
            const uint32_t h0 = (uint32_t)r1b.size();
            for (uint32_t x = g0; x < g1; x += s2) {
                const uint32_t h = (uint32_t)r1b.size(), e = std::min(g1, x + s2);
                r1b.push_back(CRun{x, e, kIdentity, h});
                r2b.push_back(CRun{x, e, h, 0});
            }
            r2.push_back(CRun{h0, (uint32_t)r1b.size(), kIdentity, 0});
        }
        nch = (uint32_t)hc.size();
        nhh = (uint32_t)hh.size();
        ng = (uint32_t)r1.size();
        ng2 = (uint32_t)r1b.size();
        npk = pfirst[nb];
        // one staged upload: chunks | 64 K pieces | block offsets | pack-chunk firsts | runs
        const size_t tb = nch * sizeof(MChunk) + nhh * sizeof(HChunk) + 2 * (nb + 1) * 4;
        const size_t tbo = (tb + 15) & ~(size_t)15;
        const size_t tall = tbo + (2 * (size_t)ng + nb + 2 * (size_t)ng2) * sizeof(CRun);
        std::vector<uint8_t> h(tall, 0);
        size_t o = 0;
        memcpy(&h[o], hc.data(), nch * sizeof(MChunk));
        o += nch * sizeof(MChunk);
        memcpy(&h[o], hh.data(), nhh * sizeof(HChunk));
        o += nhh * sizeof(HChunk);
        for (uint32_t b = 0; b <= nb; ++b, o += 4) {
            const uint32_t v = (uint32_t)bt.offs[b];
            memcpy(&h[o], &v, 4);
        }
        memcpy(&h[o], pfirst.data(), (nb + 1) * 4);
        o = tbo;
        memcpy(&h[o], r1.data(), ng * sizeof(CRun));
        o += ng * sizeof(CRun);
        memcpy(&h[o], r3.data(), ng * sizeof(CRun));
        o += ng * sizeof(CRun);
        memcpy(&h[o], r2.data(), nb * sizeof(CRun));
        o += nb * sizeof(CRun);
        if (ng2) {
            memcpy(&h[o], r1b.data(), ng2 * sizeof(CRun));
            o += ng2 * sizeof(CRun);
            memcpy(&h[o], r2b.data(), ng2 * sizeof(CRun));
        }
        uint8_t *d_tab = (uint8_t *)c->get(WS_MTF_CHUNKS, tall + 64);
        c->h2d(d_tab, h.data(), tall);
        c->ws_tag[WS_MTF_CHUNKS] = sig;
        c->ws_aux[WS_MTF_CHUNKS][0] = nch;
        c->ws_aux[WS_MTF_CHUNKS][1] = nhh;
        c->ws_aux[WS_MTF_CHUNKS][2] = ng;
        c->ws_aux[WS_MTF_CHUNKS][3] = npk;
        c->ws_aux[WS_MTF_CHUNKS][4] = ng2;
    }
    const size_t tb = nch * sizeof(MChunk) + nhh * sizeof(HChunk) + 2 * (nb + 1) * 4;
    uint8_t *d_tab = (uint8_t *)c->ws[WS_MTF_CHUNKS];
    MChunk *d_chunks = (MChunk *)d_tab;
    HChunk *d_hh = (HChunk *)(d_tab + nch * sizeof(MChunk));
    uint32_t *d_boffs = (uint32_t *)(d_tab + nch * sizeof(MChunk) + nhh * sizeof(HChunk));  // block offsets
    uint32_t *d_pfirst = d_boffs + (nb + 1);
    CRun *d_r1 = (CRun *)(d_tab + ((tb + 15) & ~(size_t)15)), *d_r3 = d_r1 + ng, *d_r2 = d_r3 + ng;
    CRun *d_r1b = d_r2 + nb, *d_r2b = d_r1b + ng2;
    uint16_t *d_chist = (uint16_t *)c->get(WS_PACK_HIST, (size_t)npk * 256 * 2 + 64);
    uint8_t *d_R = (uint8_t *)c->get(WS_MTF_R, (size_t)nch * 256 + (size_t)nch * 4 + 64);
    uint32_t *d_dcount = (uint32_t *)(d_R + (size_t)nch * 256);
    uint32_t *d_S = (uint32_t *)c->get(WS_MTF_S, (size_t)nch * 256);
    // superchunk (then group) lists | start states | list lengths
    uint8_t *d_sup = (uint8_t *)c->get(WS_MTF_SUPER, (size_t)(ng + ng2) * (256 + 256 + 4) + 64);
    uint8_t *d_Rg = d_sup;                                       // superchunk lists
    uint32_t *d_Sg = (uint32_t *)(d_sup + (size_t)ng * 256);     // superchunk start states
    uint32_t *d_dg = (uint32_t *)(d_sup + (size_t)ng * 512);     // superchunk list lengths
    uint8_t *d_Rh = d_sup + (size_t)ng * 516;                    // group lists (five levels)
    uint32_t *d_Sh = (uint32_t *)(d_Rh + (size_t)ng2 * 256);     // group start states
    uint32_t *d_dh = (uint32_t *)(d_Rh + (size_t)ng2 * 512);     // group list lengths
    uint32_t *d_freq = (uint32_t *)c->get(WS_FREQ, (size_t)nb * 256 * 4);
    uint32_t *d_first = (uint32_t *)c->get(WS_FIRST, (size_t)nb * 256 * 8);
    uint32_t *d_firstc = d_first + (size_t)nb * 256;  // first pack chunk of each value (k_mtf_hist)
    const bool runs = !c->mtf_dense;  // (Ctx::mtf_dense: the batch's digram census found it dense)
    const uint32_t rgrid = (nch + 3) / 4;
    if (runs)
        BMH_LAUNCH(c, "mtf_recency", k_mtf_recency<true>, rgrid, 256, 0, d_L, d_chunks, nch, d_R, d_dcount,
                   d_freq, d_firstc, nb * 256);
    else
        BMH_LAUNCH(c, "mtf_recency", k_mtf_recency<false>, rgrid, 256, 0, d_L, d_chunks, nch, d_R, d_dcount, d_freq,
               d_firstc, nb * 256);
    BMH_LAUNCH(c, "mtf_compose", (k_mtf_compose<false, true>), ng, 64, 0, d_r1, d_R, d_dcount, nullptr, nullptr, d_Rg,
               d_dg);
    if (ng2) {
        BMH_LAUNCH(c, "mtf_compose", (k_mtf_compose<false, true>), ng2, 64, 0, d_r1b, d_Rg, d_dg, nullptr, nullptr,
                   d_Rh, d_dh);
        BMH_LAUNCH(c, "mtf_compose", (k_mtf_compose<true, false>), nb, 64, 0, d_r2, d_Rh, d_dh, nullptr, d_Sh,
                   nullptr, nullptr);
        BMH_LAUNCH(c, "mtf_compose", (k_mtf_compose<true, false>), ng2, 64, 0, d_r2b, d_Rg, d_dg, d_Sh, d_Sg,
                   nullptr, nullptr);
    } else {
        BMH_LAUNCH(c, "mtf_compose", (k_mtf_compose<true, false>), nb, 64, 0, d_r2, d_Rg, d_dg, nullptr, d_Sg,
                   nullptr, nullptr);
    }
    BMH_LAUNCH(c, "mtf_compose", (k_mtf_compose<true, false>), ng, 64, 0, d_r3, d_R, d_dcount, d_Sg, d_S, nullptr,
               nullptr);
    BMH_LAUNCH(c, "mtf_encode", k_mtf_encode, (nch + kLanes - 1) / kLanes, kLanes, 0, d_L, d_chunks, nch, d_S, d_mtf);
    if (runs)
        BMH_LAUNCH(c, "mtf_hist", k_mtf_hist<true>, nhh, 1024, 0, d_mtf, d_hh, d_pfirst, d_freq, d_chist, d_firstc);
    else
        BMH_LAUNCH(c, "mtf_hist", k_mtf_hist<false>, nhh, 1024, 0, d_mtf, d_hh, d_pfirst, d_freq, d_chist, d_firstc);
    BMH_LAUNCH(c, "mtf_first", k_mtf_first, dim3(nb, kFirstWG), kFirstNT, 0, d_mtf, d_boffs, d_pfirst, d_freq, d_firstc,
               d_first);
    if (h_freq32) c->d2h(h_freq32, d_freq, (size_t)nb * 256 * 4);
    if (h_first32) c->d2h(h_first32, d_first, (size_t)nb * 256 * 4);
    if (h_freq32 || h_first32) c->sync();
}

}  // namespace bmh
