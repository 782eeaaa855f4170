// bwt.hip — cyclic-rotation BWT of a batch of blocks on gfx950.
//
// Replaces bwt() + bwt_cmp_straight + cyclic_index (reference main.cpp:38-59, 77-91), which
// std::stable_sort's rotation indices with an O(LCP) byte comparator. The same order is built
// here by radix-sorting rotation prefixes, then prefix doubling on cyclic ranks for whatever
// is still tied:
//
// Data phase (no rank arrays touched):
//   global pass : counting sort of every position by the first kG1Bits = 10 rotation bits
//                 (1024 buckets per block; LDS histograms per 16 K chunk; chunks of one block
//                 mapped to one XCD so the block's bytes and record write frontier stay in that
//                 XCD's L2). Every rotation of a dense bucket leaves an 8-byte record: its next
//                 12 + R rotation bits, its position and its last-column byte (rec_rbits).
//   dense finish: one workgroup per bucket of <= 4608 rotations: LDS counting sort by the next
//                 12 bits, then every sub-bucket of <= 64 is ordered by the next R bits by rank
//                 counting (R = 22 for 4 MiB blocks: bit depth 44). Resolved slots get their L
//                 byte (and SA where a later pass reads it). Longer sub-buckets, and rotations
//                 still tied, are deferred to list passes.
//   list passes : deferred segments by size: tiny (<= 64, wave shuffles), bitonic (<= 4096, 64
//                 more rotation bits per round), counting-sort finish (12-bit digit + 32-bit
//                 ranks) and MSD passes (8 bits past the shared prefix) for longer ones.
// Doubling phase (only blocks that still hold tied groups, e.g. text or periodic input):
//   lazy rank fill: rank[p] = slot of p, or its group's start slot (ranks = #strictly smaller
//   rotations at the current depth); then rounds sorting each tied group by
//   rank_D[(p + D) mod n] -> depth 2D (tiny / medium / large-MSD segment classes). Identical
//   rotations stop once D >= n: their L bytes are equal, and the primary index is the group
//   start, i.e. the count of strictly smaller rotations — exactly the row std::stable_sort
//   gives rotation 0.
#include "bmh_internal.h"
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

// ---------------------------------------------------------------------------- constants
constexpr uint32_t kG1Chunk = 16384;            // positions per global-pass workgroup (LDS-staged)
constexpr uint32_t kG1Bits = 10;                // global-pass digit: first byte + 2 bits
constexpr uint32_t kG1Bins = 1u << kG1Bits;
constexpr uint32_t kSegDigit = 12;              // LDS digit of the finish passes
constexpr uint32_t kSegDigits1 = 1u << kSegDigit;
// finish workgroup shapes: dense (global-pass buckets of <= kDenseCap rotations, 12-bit digit,
// R-bit rests), list big (counting-sort finish). List segments over kFinCap take the
// counting-sort finish up to kSegCap (large batches) or the batch's big cap, MSD passes beyond.
// (Round 3's 9-bit pass with a wide finish and its persistent LDS-DMA scatter measured slower,
// DESIGN.md §11; they live in git history, commit dd60b97.)
constexpr uint32_t kDenseNT = 512, kDenseCap = 4608;
constexpr uint32_t kSegNT = 512, kSegCap = 4608;
constexpr uint32_t kFinCap = 4096;  // list segments <= this take the register bitonic sort
// List segments longer than the batch's big cap take MSD passes (8 bits past their shared prefix
// per pass); shorter ones over kFinCap a counting-sort finish (12-bit digit + 32-bit ranks).
// Large batches (throughput-bound) use kBigCapLarge: MSD down to bitonic-sized pieces measured
// faster than the counting-sort finish on 4097-19072 (Zipf 100 MB at 1 MiB blocks 13.5 -> 11.7
// ms). Small batches (latency-bound: Calgary) keep the counting-sort finish up to kBigCapSmall,
// which resolves 44 bits per round where an MSD pass takes 8 (half the rounds).
constexpr uint32_t kBigCapLarge = 4096, kBigCapSmall = 19072, kBigNT = 1024;
constexpr uint64_t kBigCapLargeBatch = 8ull << 20;  // batches of more bytes use kBigCapLarge
constexpr uint64_t kFullSaBatch = 16ull << 20;      // batches up to this size store the full SA
constexpr uint64_t kMergeSortBatch = 16ull << 20;   // ... and launch two bitonic list classes a round
static_assert(kFinCap <= kBigCapLarge && kBigCapLarge <= kSegCap && kSegCap <= kDenseCap, "list classes");
constexpr uint32_t kSmallM = 64;                // sub-bucket size sorted by rank counting
constexpr uint32_t kTinyFin = 64;               // list segments this small: one wave each
// Ties deeper than this go to rank doubling (DataArgs::dbl_bits): 512 bits in large batches,
// 256 in the latency-bound ones that store the full suffix array from the start (no data-phase
// re-run): Calgary 3.0 -> 2.8-2.9 ms whole files, 2.8 -> 2.6 ms at 256 KiB; Zipf text at 256
// would re-run large batches' data phase (100 MB: 10.0 -> 12.9 ms).
constexpr uint32_t kDblBitsLarge = 512, kDblBitsSmall = 256;
constexpr uint32_t kDTile = 4096;               // MSD / large-path tile
constexpr uint32_t kDeferQ = 256;               // LDS deferral queue entries per workgroup
constexpr uint32_t kTinyQ = 256;               // the packed tiny finish (256 segments per workgroup)
// doubling phase
constexpr uint32_t kTinyMax = 64;     // doubling-phase segments ranked by wave shuffles (k_dtiny)
constexpr uint32_t kTinyEpwShort = 16;           // tiny-list entries per wave for short lists
constexpr uint32_t kTinyWideList = 1u << 17;      // lists this long keep 64 entries per wave
constexpr uint32_t kDblGrid = 1024;   // fixed grid of the doubling-phase kernels (counts read on the device)
constexpr uint32_t kMedMax = 4096;
constexpr uint32_t kFinalFlag = 0x80000000u;
// Big-list segments flagged kRunMode (Seg4.w bit 30) were left holding >= 3/4 of their parent by
// the previous MSD pass (run-dominated data: a long run of one byte, e.g. the zero runs of a fax
// image). Their pass digit is the position of the first bit where a rotation's window differs
// from the segment's smallest window (order-preserving: sharing more bits with the minimum
// means smaller), so a pass advances up to 64 bits instead of 8.
constexpr uint32_t kRunMode = 1u << 30;
// Big-list segments whose windows are already in the window buffer carry the number K of
// known window bits in Seg4.w bits 16..22 (0: gather them): the global pass's buckets (it
// stores rotation bits [10, 64): K = 54), and MSD children, whose parent's scatter stored the
// window shifted past the bits that pass consumed (K = parent K - consumed). The pass digit
// starts at most K - kMsdBits bits in, inside the known bits; a segment sharing all of them then
// has one digit, stays in place and goes on in run mode with gathered windows.
// (10-bit digits measured slower on Zipf text: DESIGN.md §9)
constexpr uint32_t kMsdBits = 8, kMsdBins = 1u << kMsdBits;  // MSD pass digit; one thread per bin
static_assert(kMsdBins >= 65 && kMsdBins <= 1024, "MSD digit (run-mode digits 0..64)");
constexpr uint32_t kWinShift = 16;
__device__ __forceinline__ uint32_t seg_known(uint32_t w) { return (w >> kWinShift) & 127u; }

struct Counters {
    uint32_t tiny, med, large, large_next, groups, next, tiles, resolved;  // doubling phase
    // data phase, per parity: entries of the tiny / fin / finb / big lists per XCD lane; row 4
    // [0]: the bitonic size classes present in the fin list (fin_class_bit)
    uint32_t lc[2][5][8];
    uint32_t lgroups;   // data phase: entries of the groups list (grows over the whole phase)
    uint32_t dtiles;    // tiles of the current MSD pass (k_tiles)
    uint32_t dmin_bits, flagged;
    uint32_t coop_fill, coop_groups;  // groups too long for one wave (k_group_fill / k_groups)
    uint32_t ltiles;                  // tiles of the current large-path MSD pass (k_tiles)
    uint32_t tstart[9];               // data-phase MSD tiles of each XCD lane (k_dtiles)
    uint32_t g1next[8];               // persistent global pass: chunks handed out per XCD lane
    uint32_t next2;                   // doubling rounds: next / next2 hold the segments of
                                      // alternate rounds (the one a round appends to is zero)
};
// Workgroup lanes -> list sub-lists of one launch: workgroup i runs on XCD i mod 8 (v = i & 7);
// the 8 values of v are dealt over the non-empty sub-lists (a batch of few blocks fills few
// lanes), v -> lane[v], the r[v]-th of rep[v] workgroup lanes serving that sub-list.
struct LaneMap {
    uint8_t lane[8], r[8], rep[8];
};
__device__ __forceinline__ void lane_of(const LaneMap &m, uint32_t i, uint32_t &x, uint32_t &j0, uint32_t &step,
                                        uint32_t nrows)
{
    const uint32_t v = i & 7u;
    x = m.lane[v];
    j0 = (i >> 3) * m.rep[v] + m.r[v];  // this workgroup's first row of sub-list x
    step = nrows * m.rep[v];            // rows between its iterations (striding kernels)
}
constexpr uint32_t kCoopGroup = 8192;  // a group this long is walked by the whole grid
constexpr uint32_t kCoopGrid = 1024;   // workgroups of the cooperative group kernels

// Data-phase segment / group: {gstart (batch slot), len, bit depth, block (| kFinalFlag)}
using Seg4 = uint4;

struct GChunk {
    uint32_t block, start, len, boff, n, pad0, pad1, pad2;  // start: block-relative position; boff, n: the block's
};

struct LSeg {
    uint32_t gstart, len, shift, gathered;
};
struct LTile {
    uint32_t seg, start, len, pad;
};

struct DataArgs {
    const uint8_t *data;
    const uint32_t *boffs;
    uint32_t nb;
    uint32_t *sa;
    uint8_t *L;
    uint32_t *prim;
    uint32_t *bflag;   // block keeps tied groups -> needs the rank phase
    Seg4 *lists[5];      // the list each deferral class appends to (kList*)
    uint32_t *lcnt;      // their counters (cnt->lc[parity], [class][lane]; groups: cnt->lgroups)
    const uint32_t *loff;  // [class][lane] first entry of each lane's sub-list (9 per class)
    Counters *cnt;
    const uint32_t *ainfo;  // per block: 0 = raw 10-bit global digit, else s | k << 8 (g1_alpha)
    const uint8_t *arank;   // per block: 256-entry byte -> rank map of a compacted alphabet
    uint32_t full_sa;  // 0: SA only for slots a later pass reads (deferred / tied / MSD)
    uint32_t big_cap;  // list segments longer than this take MSD passes (kBigCapLarge / kBigCapSmall)
    uint32_t dbl_bits; // tied segments this deep go to rank doubling (kDblBitsLarge / kDblBitsSmall)
};

__device__ __forceinline__ uint8_t lastcol_byte(const uint8_t *blk, uint32_t n, uint32_t p)
{
    return blk[p == 0 ? n - 1 : p - 1];
}

// Resolved slot: SA, L and (for rotation 0) the primary index. gslot is a batch slot.
__device__ __forceinline__ void put_final(const DataArgs &a, uint32_t b, uint32_t boff, uint32_t n,
                                          const uint8_t *blk, uint32_t gslot, uint32_t p, uint32_t rank_local)
{
    a.L[gslot] = lastcol_byte(blk, n, p);
    if (p == 0) a.prim[b] = rank_local;
}

// Bits [db, db + 64) of rotation p (MSB first), cyclic.
__device__ __forceinline__ uint64_t rot_window(const uint8_t *__restrict__ blk, uint32_t n, uint32_t p, uint32_t db)
{
    const uint32_t B = db >> 3, sh = db & 7u;
    uint64_t w = 0;
    uint32_t x;
    if ((uint64_t)p + B + 12 <= n) {
        // three aligned dwords cover the 9 bytes [q, q + 9); none lies past q + 12
        const uint8_t *q = blk + p + B;
        const uint32_t *aq = (const uint32_t *)((uintptr_t)q & ~(uintptr_t)3);
        const uint32_t al = (uint32_t)((uintptr_t)q & 3u) * 8u;
        const uint32_t d0 = aq[0], d1 = aq[1], d2 = aq[2];
        const uint64_t lo = ((uint64_t)d1 << 32) | d0;
        const uint64_t v = al ? ((lo >> al) | ((uint64_t)d2 << (64 - al))) : lo;
        x = (d2 >> al) & 255u;
        w = __builtin_bswap64(v);
    } else {
        uint64_t s = ((uint64_t)p + B) % n;
        for (int i = 0; i < 8; ++i) {
            w = (w << 8) | blk[s];
            if (++s == n) s = 0;
        }
        x = blk[s];
    }
    if (sh) w = (w << sh) | (x >> (8 - sh));
    return w;
}

// The lists a deferred segment can go to.
// The first four are refilled every round; the groups list grows over the whole data phase.
enum : uint32_t { kListTiny = 0, kListFin = 1, kListFinb = 2, kListBig = 3, kListGroups = 4, kNumLists = 5 };

// The tiny / fin / finb / big lists are cut into 8 sub-lists by XCD lane (block b -> lane b & 7,
// the dense finish's mapping): every list kernel runs workgroup i on lane i & 7, so the text
// windows a lane's rotations gather stay in one XCD's L2. A lane's sub-list is sized from the
// bytes of its blocks (entries are disjoint runs of >= the class's minimum length), so it never
// overflows. Queue slots: class * 8 + lane (classes 0..3), kSlotGroups for the groups list.
constexpr uint32_t kSlotGroups = 32, kSlots = 33;
__device__ __forceinline__ uint32_t list_slot(uint32_t l, uint32_t w) { return l == kListGroups ? kSlotGroups : l * 8 + (w & 7u); }
__device__ __forceinline__ uint32_t *slot_counter(const DataArgs &a, uint32_t slot)
{
    return slot == kSlotGroups ? &a.cnt->lgroups : &a.lcnt[slot];
}
__device__ __forceinline__ Seg4 *slot_base(const DataArgs &a, uint32_t slot)
{
    return slot == kSlotGroups ? a.lists[kListGroups] : a.lists[slot >> 3] + a.loff[(slot >> 3) * 9 + (slot & 7u)];
}

// A tied run of m rotations, grouped up to bit depth nd (sg = {gs, m, nd, b}): another finish
// pass by size class, or rank doubling once it is deep (long repeats), or final when nd
// covers the whole rotation (block flag in sg.w).
__device__ __forceinline__ uint32_t defer_list(const DataArgs &a, Seg4 &sg, uint32_t n)
{
    if (sg.z >= 8ull * n) {
        sg.w |= kFinalFlag;
        return kListGroups;
    }
    if (sg.z >= a.dbl_bits) {
        a.bflag[sg.w] = 1;
        a.cnt->flagged = 1;
        return kListGroups;
    }
    if (sg.y > kFinCap) return sg.y > a.big_cap && sg.y > kSegCap ? kListBig : kListFinb;
    return sg.y <= kTinyFin ? kListTiny : kListFin;
}

// Deferred segments queued per workgroup in LDS; one global atomic per list reserves the
// workgroup's entries at the flush. (Single-entry pushes from every workgroup onto the same
// few counters serialise at the L2: on text, millions of them cost tens of ms per round.)
template <uint32_t Q>
struct DeferQueue {
    uint32_t n;                  // entries pushed (beyond Q they went to the lists directly)
    uint32_t fmask;              // fin-list size classes pushed (fin_class_bit)
    uint32_t cnt[kSlots], base[kSlots];
    Seg4 e[Q];
    uint32_t tag[Q];             // slot << 24 | index inside the slot's reservation
};

// before the first push; a barrier must separate it from the pushes
template <uint32_t Q>
__device__ __forceinline__ void dq_init(DeferQueue<Q> &q)
{
    if (threadIdx.x < kSlots) q.cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        q.n = 0;
        q.fmask = 0;
    }
}

// the register-bitonic launch a fin-list segment of len (65..kFinCap) takes: <= 128, 512, 1024,
// 2048, 4096; the host launches only the classes some segment of the round needs
__device__ __forceinline__ uint32_t fin_class_bit(uint32_t len)
{
    return len <= 128 ? 1u : len <= 512 ? 2u : len <= 1024 ? 4u : len <= 2048 ? 8u : 16u;
}

template <uint32_t Q>
__device__ __forceinline__ void dq_push_list(const DataArgs &a, DeferQueue<Q> &q, Seg4 sg, uint32_t l)
{
    const uint32_t slot = list_slot(l, sg.w);
    if (l == kListFin) atomicOr(&q.fmask, fin_class_bit(sg.y));
    const uint32_t i = atomicAdd(&q.n, 1u);
    if (i < Q) {
        q.e[i] = sg;
        q.tag[i] = (slot << 24) | atomicAdd(&q.cnt[slot], 1u);
    } else {
        // lanes of one wave may overflow into different sub-lists: one aggregated append per
        // slot, each under its own branch so that the wave's active lanes share the counter
        // (kept rolled: the overflow is rare and every push site inlines it)
#pragma unroll 1
        for (uint32_t k = 0; k < kSlots; ++k)
            if (slot == k) slot_base(a, k)[wave_append(slot_counter(a, k))] = sg;
    }
}

template <uint32_t Q>
__device__ __forceinline__ void dq_push(const DataArgs &a, DeferQueue<Q> &q, uint32_t gs, uint32_t m, uint32_t nd,
                                        uint32_t b, uint32_t n)
{
    Seg4 sg = make_uint4(gs, m, nd, b);
    const uint32_t l = defer_list(a, sg, n);
    dq_push_list(a, q, sg, l);
}

// all threads, once per queue; starts with a barrier, and ends with one when anything was
// queued (the common empty case costs the one barrier)
template <uint32_t NT, uint32_t Q>
__device__ __forceinline__ void dq_flush(const DataArgs &a, DeferQueue<Q> &q)
{
    __syncthreads();
    const uint32_t qn = min(q.n, Q);
    if (qn == 0) return;  // workgroup-uniform
    const uint32_t t = threadIdx.x;
    if (t < kSlots && q.cnt[t]) q.base[t] = atomicAdd(slot_counter(a, t), q.cnt[t]);
    if (t == kSlots && q.fmask) atomicOr(&a.lcnt[4 * 8], q.fmask);
    __syncthreads();
    for (uint32_t i = t; i < qn; i += NT) {
        const uint32_t tg = q.tag[i], sl = tg >> 24;
        slot_base(a, sl)[q.base[sl] + (tg & 0xffffffu)] = q.e[i];
    }
    __syncthreads();
}

// Compact rotation record the global pass writes for dense buckets (u64): rotation bits
// [kG1Bits, kG1Bits + 12 + R) | p (P bits) | last-column byte, with P = bits of the block's
// largest position and R = min(32, 44 - P) (4 MiB blocks: P = 22, R = 22, so one dense
// finish resolves rotation bits up to 44; rarer deeper ties go to list passes).
__device__ __forceinline__ uint32_t rec_pbits(uint32_t n) { return n <= 2 ? 1u : 32u - (uint32_t)__builtin_clz(n - 1); }
// R also keeps db + 12 + R within the 64 rotation bits the global pass reads (db <= 24); a
// packed record (below) reads no raw window, so only the record's 64 bits bound it
__device__ __forceinline__ uint32_t rec_rbits(uint32_t P, uint32_t db, bool packed)
{
    return packed ? min(32u, 44u - P) : min(min(32u, 44u - P), 52u - db);
}

// Per-block global-pass alphabet: a block of k <= 32 distinct bytes keys its
// global pass on s = 2 (k <= 32) or 3 (k <= 10) whole symbols, each replaced by its rank among the
// block's distinct bytes (order-preserving), mixed radix k: digit = ((r0 k + r1) k + r2) < k^s <=
// 1024. Every rotation of a bucket then shares its first s bytes, i.e. db = 8 s raw rotation bits
// (text: 2 characters, against 1 character + 2 bits of the raw 10-bit digit, where every
// lowercase letter has the same top bits); later passes stay in raw bits. info = s | k << 8,
// 0 for the raw digit (db = kG1Bits).
__device__ __forceinline__ uint32_t g1_db(uint32_t info) { return info ? 8u * (info & 255u) : kG1Bits; }
// Packed records: a compacted block's dense-bucket record carries, in place
// of raw rotation bits [db, db + 12 + R), the w-bit ranks of its next nsym symbols (w = bits of
// k - 1, left-aligned: order-preserving, since the rank map is monotone), so the dense finish
// resolves nsym whole symbols (27 letters at 1 MiB blocks: 7 instead of 4.5 characters) and its
// tied groups go on in raw bits at the whole-symbol depth they reached. kPackSymMax bounds the
// bytes the global pass reads past each position (its LDS halo).
constexpr uint32_t kPackSymMax = 12;
__device__ __forceinline__ uint32_t g1_w(uint32_t info)
{
    const uint32_t k = info >> 8;
    return k <= 1 ? 0u : 32u - (uint32_t)__builtin_clz(k - 1);
}
__device__ __forceinline__ uint32_t rec_nsym(uint32_t info, uint32_t R)
{
    const uint32_t w = g1_w(info);
    return w ? min(kPackSymMax, (12u + R) / w) : 0u;
}
// Raw bit depths a dense bucket's rotations are known equal to after the finish: dep_dig for a
// sub-bucket grouped by the 12-bit digit, dep_full after the rest too.
__device__ __forceinline__ void dense_depths(uint32_t info, uint32_t R, uint32_t &dep_dig, uint32_t &dep_full)
{
    const uint32_t db = g1_db(info), ns = info ? rec_nsym(info, R) : 0u;
    if (ns) {
        const uint32_t s = info & 255u;
        dep_dig = 8u * (s + min(ns, kSegDigit / g1_w(info)));
        dep_full = 8u * (s + ns);
    } else {
        dep_dig = db + kSegDigit;
        dep_full = db + kSegDigit + R;
    }
}
__device__ __forceinline__ uint32_t g1_digit3(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t info, const uint8_t *rk)
{
    if (!info) return (b0 << (kG1Bits - 8)) | (b1 >> (16 - kG1Bits));
    const uint32_t k = info >> 8;
    uint32_t d = rk[b0] * k + rk[b1];
    if ((info & 255u) == 3) d = d * k + rk[b2];
    return d;
}

// ------------------------------------------------------------------------- global pass
// Counting sort of every block by its first kG1Bits rotation bits. Chunks of <= 16 K
// positions whose batch boundaries are 16-byte multiples (a block's first chunk takes the
// unaligned prefix), dealt into 8 XCD lanes so one block's chunks share an L2.
__device__ __forceinline__ void g1_load16(const uint8_t *__restrict__ blk, uint32_t start, uint32_t len, uint32_t e,
                                          uint32_t (&dg)[4])
{
    // bytes [start + e, start + e + 16) of the block, zero past len
    if (e + 16 <= len && (((uintptr_t)(blk + start + e)) & 15u) == 0) {
        const uint4 v = *(const uint4 *)(blk + start + e);
        dg[0] = v.x;
        dg[1] = v.y;
        dg[2] = v.z;
        dg[3] = v.w;
    } else {
        dg[0] = dg[1] = dg[2] = dg[3] = 0;
        for (uint32_t k = 0; k < 16; ++k)
            if (e + k < len) dg[k >> 2] |= (uint32_t)blk[start + e + k] << (8 * (k & 3));
    }
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&dg)[4], uint32_t k)
{
    return (dg[k >> 2] >> (8 * (k & 3))) & 255u;
}

// digit of chunk element k (< nv) from its byte and the next two (nx, nx2 = the bytes after the run)
__device__ __forceinline__ uint32_t g1_digit(const uint32_t (&dg)[4], uint32_t k, uint32_t nv, uint32_t nx, uint32_t nx2,
                                             uint32_t info, const uint8_t *rk)
{
    const uint32_t b1 = k + 1 < nv ? byte_of(dg, k + 1) : nx;
    const uint32_t b2 = k + 2 < nv ? byte_of(dg, k + 2) : k + 2 == nv ? nx : nx2;
    return g1_digit3(byte_of(dg, k), b1, b2, info, rk);
}

// Census of each block's distinct bytes, from the global pass's raw histograms (every position's
// byte is the first byte of its rotation's digit): k_g1_hist stores each chunk's 256-bit set
// (plain stores, 8 words a chunk: no atomics on a block's few words from its hundreds of
// chunks), k_g1_census_fin ORs a block's chunk sets and decides its alphabet, and a second
// k_g1_hist launch recounts the chunks of the blocks that take compacted digits (the others'
// workgroups exit at once).
constexpr uint32_t kAlphaMax = 32;
// grid = nblocks: the block's alphabet info and rank map from its chunks' sets (list indices
// c0 + 8k); a compacted block appends its chunks to the recount list
__global__ __launch_bounds__(256) void k_g1_census_fin(const uint32_t *__restrict__ cbits,
                                                       const uint32_t *__restrict__ bchunks,
                                                       const uint32_t *__restrict__ bchunk0,
                                                       uint32_t *__restrict__ ainfo, uint8_t *__restrict__ arank,
                                                       uint32_t *__restrict__ rlist)
{
    __shared__ uint32_t s_w[8];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t c0 = bchunk0[b], nc = bchunks[b];
    if (t < 8) s_w[t] = 0;
    __syncthreads();
    uint32_t acc = 0;
    for (uint32_t k = t >> 3; k < nc; k += 32) acc |= cbits[(size_t)(c0 + 8 * k) * 8 + (t & 7u)];
    if (acc) atomicOr(&s_w[t & 7u], acc);
    __syncthreads();
    uint32_t k = 0, below = 0;
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t c = __builtin_popcount(s_w[j]);
        k += c;
        if (j < (t >> 5)) below += c;
    }
    below += __builtin_popcount(s_w[t >> 5] & ((1u << (t & 31u)) - 1u));
    const bool compact = k <= kAlphaMax && k >= 1;
    arank[(size_t)b * 256 + t] = (uint8_t)below;
    if (t == 0) ainfo[b] = compact ? ((k <= 10 ? 3u : 2u) | (k << 8)) : 0u;
    if (compact) {  // the block's chunks go on the recount list (rlist[-1] = its length)
        __shared__ uint32_t s_base;
        if (t == 0) s_base = atomicAdd(rlist - 1, nc);
        __syncthreads();
        for (uint32_t j = t; j < nc; j += 256) rlist[s_base + j] = c0 + 8 * j;
    }
}

// Phase timing (experiment builds only): -DBMH_PROF_SCATTER times k_g1_scatter's phases,
// -DBMH_PROF_DENSE k_finish_dense's; thread 0 of each workgroup stores its s_memtime ticks per
// phase, and the host prints the means after the dense finish.
#if defined(BMH_PROF_SCATTER) || defined(BMH_PROF_DENSE)
__device__ uint32_t g_dprof[(1u << 18) * 8];
#define PROF_MARK(i)                                                                            \
    do {                                                                                        \
        if (threadIdx.x == 0) {                                                                 \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                                   \
            if (blockIdx.x < (1u << 18)) g_dprof[blockIdx.x * 8 + (i)] = (uint32_t)(_t - _t0); \
            _t0 = _t;                                                                           \
        }                                                                                       \
    } while (0)
#define PROF_START uint64_t _t0 = __builtin_amdgcn_s_memtime()
#endif
#ifdef BMH_PROF_SCATTER
#define GPROF(i) PROF_MARK(i)
#define GPROF_START PROF_START
#else
#define GPROF(i) \
    do {         \
    } while (0)
#define GPROF_START
#endif
#ifdef BMH_PROF_DENSE
#define DPROF(i) PROF_MARK(i)
#define DPROF_START PROF_START
#else
#define DPROF(i) \
    do {         \
    } while (0)
#define DPROF_START
#endif

// 512 threads x 32 positions a chunk (two 16-byte loads a thread: twice the bytes in flight of
// one, at the same four workgroups' worth of waves a CU). recount = 0 (grid = the chunk list): raw 10-bit digits
// for every block, plus the census (bits); recount = 1 (a grid of <= 2048 striding over rlist,
// the chunks of compacted blocks k_g1_census_fin listed): those chunks' digits by the block's
// alphabet (ainfo / arank) — on a batch with none, a few thousand workgroups read a zero count.
constexpr uint32_t kG1HistNT = 512;
__global__ __launch_bounds__(kG1HistNT) void k_g1_hist(const uint8_t *__restrict__ data, const uint32_t *__restrict__ boffs,
                                                  const GChunk *__restrict__ chunks, uint32_t *__restrict__ rlist,
                                                  uint16_t *__restrict__ ccnt, const uint32_t *__restrict__ ainfo,
                                                  const uint8_t *__restrict__ arank, uint32_t *__restrict__ bits,
                                                  uint32_t recount)  // bits: 8 words a chunk
{
    __shared__ __align__(16) uint32_t h[4][kG1Bins];
    __shared__ uint8_t s_rk[256];
    const uint32_t t = threadIdx.x, w = (t >> 6) & 3u;
    uint32_t *const rcount = rlist - 1;  // rlist[-1] = its length, zeroed by the raw pass
    if (!recount && blockIdx.x == 0 && t == 0) *rcount = 0;
    const uint32_t nsel = recount ? *rcount : 1u;
    for (uint32_t q = recount ? blockIdx.x : 0u; q < nsel; q += recount ? gridDim.x : 1u) {
        const uint32_t ci = recount ? rlist[q] : blockIdx.x;
        const GChunk ch = chunks[ci];
        if (ch.len == 0) {
            if (t < 8) bits[(size_t)ci * 8 + t] = 0;  // an empty chunk's set (never listed)
            continue;
        }
        const uint32_t info = recount ? ainfo[ch.block] : 0u;
        __syncthreads();                 // the previous chunk's reads of h / s_rk
        for (uint32_t i = t; i < 4 * kG1Bins; i += kG1HistNT) (&h[0][0])[i] = 0;
        if (info && t < 256) s_rk[t] = arank[(size_t)ch.block * 256 + t];
        __syncthreads();
        // the block's offset and length ride in the chunk entry (no dependent load of boffs)
        const uint32_t n = ch.n;
        const uint8_t *blk = data + ch.boff;
        const uint32_t e = 32 * t;
        if (e < ch.len) {
            uint32_t dg[4], dgb[4];  // the thread's run [e, e + nv): pieces A and B
            g1_load16(blk, ch.start, ch.len, e, dg);
            g1_load16(blk, ch.start, ch.len, e + 16, dgb);
            const uint32_t nv = min(32u, ch.len - e);
            // the two bytes after the run (cyclic; n may be 1 or 2): start + e + nv <= n
            const uint32_t x = ch.start + e + nv, ni = x >= n ? x - n : x, ni2 = ni + 1 >= n ? ni + 1 - n : ni + 1;
            const uint32_t nx = blk[ni], nx2 = blk[ni2];
            if (nv == 32) {
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k)
                    atomicAdd(&h[w][g1_digit(dg, k, 16, byte_of(dgb, 0), byte_of(dgb, 1), info, s_rk)], 1u);
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k) atomicAdd(&h[w][g1_digit(dgb, k, 16, nx, nx2, info, s_rk)], 1u);
            } else {
                // piece A's following bytes: B's first two while inside the run, then the run's
                const uint32_t nva = min(16u, nv);
                const uint32_t a1 = nv > 16 ? byte_of(dgb, 0) : nx;
                const uint32_t a2 = nv > 17 ? byte_of(dgb, 1) : nv == 17 ? nx : nx2;
                for (uint32_t k = 0; k < nva; ++k) atomicAdd(&h[w][g1_digit(dg, k, nva, a1, a2, info, s_rk)], 1u);
                for (uint32_t k = 0; k + 16 < nv; ++k) atomicAdd(&h[w][g1_digit(dgb, k, nv - 16, nx, nx2, info, s_rk)], 1u);
            }
        }
        __syncthreads();
        // u16 counts (a chunk holds <= 16 K rotations), two adjacent digits a thread
        static_assert(kG1Chunk <= 65535 && kG1Bins == 2 * kG1HistNT, "u16 digit counts, two a thread");
        {
            const uint32_t d = 2 * t;
            const uint32_t lo = h[0][d] + h[1][d] + h[2][d] + h[3][d];
            const uint32_t hi = h[0][d + 1] + h[1][d + 1] + h[2][d + 1] + h[3][d + 1];
            ((uint32_t *)ccnt)[(size_t)ci * (kG1Bins / 2) + t] = lo | (hi << 16);
        }
        if (!recount) {
            // the chunk's bytes: byte v is present iff one of the digits 4v .. 4v + 3 is counted
            // (read from the four waves' partial counts: no further barrier)
            static_assert(kG1Bits == 10, "census: 4 raw digits per first byte");
            if (t < 256) {
                uint32_t any = 0;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint4 v = *(const uint4 *)&h[q][4 * t];
                    any |= v.x | v.y | v.z | v.w;
                }
                const bool present = any != 0;
                const uint64_t bal = __ballot(present);
                const uint32_t l = t & 63u;
                if (l < 2) bits[(size_t)ci * 8 + 2 * (t >> 6) + l] = (uint32_t)(bal >> (32 * l));
            }
        }
    }
}

// The bucket scan in three launches so a block's chunk counts are walked by kG1ScanParts
// workgroups instead of one (a small batch's few blocks left the single walk latency-bound:
// 128 MiB 0.043 ms; at 1 GiB it is HBM-bound either way). Grid (nblocks, kG1ScanParts), one
// thread per digit: part q of block b walks its chunks [q nq, q nq + nq) (list indices c0 + 8k,
// the XCD lane stride), 32 loads in flight. k_g1_scan_sum: the part's digit counts.
constexpr uint32_t kG1ScanParts = 4;
__global__ __launch_bounds__(kG1Bins) void k_g1_scan_sum(const uint32_t *__restrict__ bchunks,
                                                         const uint32_t *__restrict__ bchunk0,
                                                         const uint16_t *__restrict__ ccnt, uint32_t *__restrict__ part)
{
    const uint32_t b = blockIdx.x, q = blockIdx.y, d = threadIdx.x;
    const uint32_t c0 = bchunk0[b], nc = bchunks[b], nq = (nc + kG1ScanParts - 1) / kG1ScanParts;
    const uint32_t k0 = q * nq, k1 = min(nc, k0 + nq);
    constexpr uint32_t U = 32;
    uint32_t run = 0;
    for (uint32_t k = k0; k < k1; k += U) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) v[j] = k + j < k1 ? ccnt[(size_t)(c0 + 8 * (k + j)) * kG1Bins + d] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) run += v[j];
    }
    part[((size_t)b * kG1ScanParts + q) * kG1Bins + d] = run;
}

// grid = nblocks; one thread per digit: the digit's total from the parts, the bucket table
// bk[b][d] = {start, len}, each part's first write offset (in place over its count), and the
// routing of buckets too big for a dense workgroup.
__global__ __launch_bounds__(kG1Bins) void k_g1_scan(const uint32_t *__restrict__ boffs, uint32_t *__restrict__ part,
                                                     uint2 *__restrict__ bk, Seg4 *finb, Seg4 *big, Counters *cnt,
                                                     const uint32_t *__restrict__ loff, uint32_t big_cap,
                                                     const uint32_t *__restrict__ ainfo)
{
    __shared__ uint32_t s_tmp[kG1Bins / 64 + 1];
    const uint32_t b = blockIdx.x, d = threadIdx.x;
    uint32_t *pp = part + (size_t)b * kG1ScanParts * kG1Bins + d;
    uint32_t pv[kG1ScanParts], run = 0;
#pragma unroll
    for (uint32_t q = 0; q < kG1ScanParts; ++q) {
        pv[q] = pp[q * kG1Bins];
        run += pv[q];
    }
    const uint32_t start = block_excl_sum<kG1Bins>(run, s_tmp, nullptr);
    uint32_t acc = start;
#pragma unroll
    for (uint32_t q = 0; q < kG1ScanParts; ++q) {
        pp[q * kG1Bins] = acc;
        acc += pv[q];
    }
    bk[(size_t)b * kG1Bins + d] = make_uint2(start, run);
    const uint32_t x = b & 7u;  // the block's XCD lane sub-lists (parity 0)
    // buckets <= kDenseCap are the dense finish's; longer ones take MSD passes, or the
    // counting-sort list finish up to big_cap
    const uint32_t db = g1_db(ainfo[b]);  // the bucket's shared prefix (raw bits), 64 - db window bits known
    if (run > kDenseCap && run > big_cap)
        big[loff[kListBig * 9 + x] + wave_append(&cnt->lc[0][kListBig][x])] =
            make_uint4(boffs[b] + start, run, db, b | ((64u - db) << kWinShift));
    else if (run > kDenseCap)
        finb[loff[kListFinb * 9 + x] + wave_append(&cnt->lc[0][kListFinb][x])] =
            make_uint4(boffs[b] + start, run, db, b);
}

// grid (nblocks, kG1ScanParts): per-chunk write offsets (block-relative, in place over the
// chunk counts), part q from its first offset
__global__ __launch_bounds__(kG1Bins) void k_g1_scan_offs(const uint32_t *__restrict__ bchunks,
                                                          const uint32_t *__restrict__ bchunk0,
                                                          const uint16_t *__restrict__ ccnt, uint32_t *__restrict__ chist,
                                                          const uint32_t *__restrict__ part)
{
    const uint32_t b = blockIdx.x, q = blockIdx.y, d = threadIdx.x;
    const uint32_t c0 = bchunk0[b], nc = bchunks[b], nq = (nc + kG1ScanParts - 1) / kG1ScanParts;
    const uint32_t k0 = q * nq, k1 = min(nc, k0 + nq);
    constexpr uint32_t U = 32;
    // counts (u16) in, write offsets (u32) out
    auto idx = [&](uint32_t k) -> size_t { return (size_t)(c0 + 8 * k) * kG1Bins + d; };
    uint32_t acc = part[((size_t)b * kG1ScanParts + q) * kG1Bins + d];
    for (uint32_t k = k0; k < k1; k += U) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) v[j] = k + j < k1 ? ccnt[idx(k + j)] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < U; ++j)
            if (k + j < k1) {
                chist[idx(k + j)] = acc;
                acc += v[j];
            }
    }
}

// Local counting sort of the chunk in LDS, then SA written in contiguous per-digit runs
// together with each rotation's 8-byte key: bits 63..8 = rotation bytes 1..7 (big-endian),
// bits 7..0 = the last-column byte. The chunk's text (with a cyclic halo) is staged in LDS,
// so the keys cost no global gathers; the dense finish pass reads them coalesced.
__global__ __launch_bounds__(1024) void k_g1_scatter(DataArgs a, const GChunk *__restrict__ chunks,
                                                     const uint32_t *__restrict__ chist, const uint2 *__restrict__ bk,
                                                     uint64_t *__restrict__ rec)
{
    __shared__ uint16_t s_ent[kG1Chunk + 1];  // chunk-relative position (+ a dummy slot)
    // byte j <-> block position start - 16 + j (cyclic), j < len + 48 (16-byte pieces; a packed
    // record reads up to 3 + kPackSymMax bytes past a position, as whole dwords)
    __shared__ __align__(16) uint32_t s_txt[(kG1Chunk + 48) / 4];
    __shared__ uint32_t s_cnt[kG1Bins + 1], s_off[kG1Bins], s_blen[kG1Bins];  // s_off: global - local start
    // (s_cnt[kG1Bins]: sink digit of the slots past the chunk, so the LDS phases run unbranched)
    __shared__ uint32_t s_tmp[17];
    __shared__ uint8_t s_rk[256];
    const GChunk ch = chunks[blockIdx.x];
    if (ch.len == 0) return;
    GPROF_START;
    const uint32_t t = threadIdx.x;
    const uint32_t b = ch.block, boff = ch.boff, n = ch.n;  // (carried by the chunk entry: no dependent load)
    const uint32_t info = a.ainfo[b], db = g1_db(info);
    // packed records for a compacted block's dense buckets (nsym symbols of wsym bits; 0: raw)
    const uint32_t nsym = info ? rec_nsym(info, min(32u, 44u - rec_pbits(n))) : 0u, wsym = g1_w(info);
    if (info && t < 256) s_rk[t] = a.arank[(size_t)b * 256 + t];
    const uint8_t *blk = a.data + boff;
    static_assert(kG1Bins <= 1024 && kG1Bits >= 8, "at most one digit per thread");
    const bool tdig = kG1Bins == 1024 || t < kG1Bins;  // this thread owns digit t
    // the chunk's digit offsets and bucket sizes: loads issued together with the text's
    uint32_t cv = 0, bl = 0;
    if (tdig) {
        cv = chist[(size_t)blockIdx.x * kG1Bins + t];
        bl = bk[(size_t)b * kG1Bins + t].y;
    }
    {
        // 16-byte pieces, all loads in flight before the first LDS store (a load under a
        // per-piece branch waits inside it: one HBM round trip per piece); pieces that wrap
        // around the block or are unaligned take the byte path
        const uint32_t np = (ch.len + 42 + 15) / 16;  // bytes up to len + 41 are read
        constexpr uint32_t PPT = (kG1Chunk + 42 + 15) / 16 / 1024 + 1;  // pieces per thread
        static_assert(16 + 3 + kPackSymMax + 3 <= 42 && (kG1Chunk + 42 + 15) / 16 * 16 <= kG1Chunk + 48, "halo");
        uint4 v[PPT];
        bool fast[PPT];
#pragma unroll
        for (uint32_t j = 0; j < PPT; ++j) {
            const uint32_t pc = t + 1024 * j;
            const int64_t q = (int64_t)ch.start - 16 + 16 * (int64_t)pc;
            fast[j] = pc < np && q >= 0 && q + 16 <= (int64_t)n && (((uintptr_t)(blk + q)) & 15u) == 0;
            v[j] = fast[j] ? *(const uint4 *)(blk + q) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t j = 0; j < PPT; ++j) {
            const uint32_t pc = t + 1024 * j;
            if (pc >= np) continue;
            if (!fast[j]) {
                uint32_t u[4] = {0, 0, 0, 0};
                const int64_t q = (int64_t)ch.start - 16 + 16 * (int64_t)pc;
                for (int k = 0; k < 16; ++k) {
                    int64_t r = (q + k) % (int64_t)n;
                    if (r < 0) r += n;
                    u[k >> 2] |= (uint32_t)blk[r] << (8 * (k & 3));
                }
                v[j] = make_uint4(u[0], u[1], u[2], u[3]);
            }
            *(uint4 *)&s_txt[4 * pc] = v[j];
        }
    }
    if (tdig) {
        s_cnt[t] = 0;
        s_off[t] = cv;
        s_blen[t] = bl;
    }
    GPROF(5);
    __syncthreads();
    GPROF(0);
    const uint32_t e0 = 16 * t;
    uint32_t dg[4] = {0, 0, 0, 0}, nx = 0, nx2 = 0;
    const uint32_t nv = e0 < ch.len ? min(16u, ch.len - e0) : 0u;
    if (nv) {
        // bytes e0 .. e0 + 16 of the chunk = s_txt bytes e0 + 16 .. e0 + 32 (dword aligned)
        for (int k = 0; k < 4; ++k) dg[k] = s_txt[(e0 >> 2) + 4 + k];
        const uint32_t j = e0 + 16 + nv;
        nx = (s_txt[j >> 2] >> (8 * (j & 3u))) & 255u;
        nx2 = (s_txt[(j + 1) >> 2] >> (8 * ((j + 1) & 3u))) & 255u;
        for (uint32_t k = nv; k < 16; ++k) dg[k >> 2] &= ~(255u << (8 * (k & 3)));
    }
    uint32_t dgt[16];
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) dgt[k] = k < nv ? g1_digit(dg, k, nv, nx, nx2, info, s_rk) : kG1Bins;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) atomicAdd(&s_cnt[dgt[k]], 1u);
    __syncthreads();
    GPROF(1);
    {
        const uint32_t ex = block_excl_sum1<1024>(tdig ? s_cnt[t] : 0u, s_tmp);
        if (tdig) {
            s_off[t] -= ex;  // slot of local element i with digit d = s_off[d] + i
            s_cnt[t] = ex;
        }
    }
    __syncthreads();
    GPROF(2);
    {
        uint32_t dst[16];  // all 16 slot reservations in flight before the first wait
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) dst[k] = atomicAdd(&s_cnt[dgt[k]], 1u);
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) s_ent[dgt[k] < kG1Bins ? dst[k] : kG1Chunk] = (uint16_t)(e0 + k);
    }
    __syncthreads();
    GPROF(3);
#pragma unroll 4
    for (uint32_t i = t; i < ch.len; i += 1024) {
        const uint32_t rel = s_ent[i];
        const uint32_t p = ch.start + rel;
        // s_txt bytes rel + 15 .. rel + 23: L byte, byte p, bytes p + 1 .. p + 7
        const uint32_t j0 = rel + 15, w0 = j0 >> 2, al = (j0 & 3u) * 8u;
        const uint32_t d0 = s_txt[w0], d1 = s_txt[w0 + 1], d2 = s_txt[w0 + 2];
        const uint64_t lo = ((uint64_t)d1 << 32) | d0;
        const uint64_t v64 = al ? ((lo >> al) | ((uint64_t)d2 << (64 - al))) : lo;  // bytes j0 .. j0 + 7
        const uint64_t b8 = (d2 >> al) & 255u;                                       // byte j0 + 8
        const uint64_t key = __builtin_bswap64((v64 >> 16) | (b8 << 48)) | (v64 & 255u);
        const uint32_t d = g1_digit3((uint32_t)(v64 >> 8) & 255u, (uint32_t)(v64 >> 16) & 255u,
                                     (uint32_t)(v64 >> 24) & 255u, info, s_rk);
        const uint32_t slot = s_off[d] + i;
        const uint32_t blen = s_blen[d];
        if (blen >= 2 && blen <= kDenseCap) {  // the dense finish reads the record, writes SA
            const uint32_t P = rec_pbits(n), R = rec_rbits(P, db, nsym != 0);
            uint64_t sub;
            if (nsym) {
                // the ranks of symbols s .. s + nsym - 1 (s_txt bytes rel + 16 + s ..), w bits each
                const uint32_t j1 = rel + 16 + (info & 255u), w1 = j1 >> 2, a1 = j1 & 3u;
                static_assert(kPackSymMax <= 12, "three aligned dwords");
                uint32_t dw[4], al[3];
#pragma unroll
                for (int q = 0; q < 4; ++q) dw[q] = s_txt[w1 + q];
#pragma unroll
                for (int q = 0; q < 3; ++q) al[q] = __builtin_amdgcn_alignbyte(dw[q + 1], dw[q], a1);  // bytes 4q ..
                uint64_t acc = 0;
#pragma unroll
                for (uint32_t q = 0; q < kPackSymMax; ++q)
                    if (q < nsym) acc = (acc << wsym) | s_rk[(al[q >> 2] >> (8 * (q & 3))) & 255u];
                sub = acc << (12 + R - nsym * wsym);
            } else {
                // rotation bits [db, db + 12 + R) (key >> 8 holds bits [8, 64))
                sub = ((key >> 8) >> (52 - db - R)) & ((1ull << (12 + R)) - 1);
            }
            rec[boff + slot] = (sub << (P + 8)) | ((uint64_t)p << 8) | (key & 255u);
        } else if (blen > 1 || a.full_sa) {
            a.sa[boff + slot] = p;
            // a bucket for the MSD passes: its first pass reads rotation bits [10, 64) from here
            // (MSB-aligned, low kG1Bits bits zero) instead of gathering them (kG1WinBits known)
            if (blen > kDenseCap && blen > a.big_cap) rec[boff + slot] = (key << (db - 8)) & ~((1ull << db) - 1);
        }
        if (blen == 1) {
            a.L[boff + slot] = (uint8_t)key;
            if (p == 0) a.prim[b] = slot;
        }
    }
    GPROF(7);
}

// ------------------------------------------------------------------------- finish pass
// One workgroup of NT threads sorts one segment of <= CAP rotations that are equal in bits
// [0, db). dense = 1: the buckets of the global pass (db = kG1Bits), XCD-aware: workgroup
// i -> lane i % 8 -> blocks b = lane mod 8, compact records read coalesced. dense = 0: the
// list entries with lo < len <= CAP, rotation windows gathered from the text.
// Each thread keeps its elements (position, last-column byte, next 12-bit digit, next R-bit
// rest) in registers; LDS holds only the rests and the 12-bit counters (packed two per
// word, 16-bit halves). Counting sort by the digit, then every element ranks itself inside
// its sub-bucket (bounds = neighbouring counters) by the rest: bit depth db + 12 + R.
// Sub-buckets > kSmallM, and rotations still tied, are deferred to list passes.

template <uint32_t NT, uint32_t CAP>
struct FinishShape {
    static constexpr uint32_t IPT = (CAP + NT - 1) / NT;
    static constexpr uint32_t NDIG = 1u << kSegDigit, WPT = NDIG / 2 / NT;  // counter words per thread
    static_assert(CAP < 65536 && WPT >= 1 && NDIG / 2 == WPT * NT, "finish shape");
};

// The finish of one segment once every element is in registers: pl = position (<< 8 | last-
// column byte when packL), dd = 12-bit digit, rv = R-bit rest. s_cnt must be zero on entry
// and is zero again on return (ends with a barrier); s_tmp holds NT / 64 + 2 words, the last
// one zero on entry (set when some slot is deferred: then the segment's SA is stored).
template <uint32_t NT, uint32_t CAP>
__device__ __forceinline__ void finish_core(const DataArgs &a, uint32_t gstart, uint32_t len, uint32_t dep_dig,
                                            uint32_t dep_full, uint32_t b, bool packL,
                                            uint32_t (&pl)[FinishShape<NT, CAP>::IPT],
                                            uint32_t (&dd)[FinishShape<NT, CAP>::IPT],
                                            uint32_t (&rv)[FinishShape<NT, CAP>::IPT], uint32_t *s_rest,
                                            uint32_t *s_cnt, uint32_t *s_tmp, DeferQueue<kDeferQ> &dq)
{
    constexpr uint32_t IPT = FinishShape<NT, CAP>::IPT, WPT = FinishShape<NT, CAP>::WPT;
    const uint32_t t = threadIdx.x;
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint8_t *blk = a.data + boff;
    DPROF_START;
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k)
        if (t + k * NT < len) atomicAdd(&s_cnt[dd[k] >> 1], 1u << (16 * (dd[k] & 1u)));
    __syncthreads();
    DPROF(1);
    {
        // thread t owns counter words WPT*t .. WPT*t + WPT - 1: counts -> starts
        uint32_t c[2 * WPT], sum = 0;
        for (uint32_t j = 0; j < WPT; ++j) {
            const uint32_t w = s_cnt[WPT * t + j];
            c[2 * j] = w & 0xffffu;
            c[2 * j + 1] = w >> 16;
            sum += c[2 * j] + c[2 * j + 1];
        }
        uint32_t ex = block_excl_sum1<NT>(sum, s_tmp);
        for (uint32_t j = 0; j < WPT; ++j) {
            const uint32_t e0 = ex, e1 = ex + c[2 * j];
            s_cnt[WPT * t + j] = e0 | (e1 << 16);
            ex = e1 + c[2 * j + 1];
        }
    }
    __syncthreads();
    DPROF(2);
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k) {
        if (t + k * NT < len) {
            const uint32_t d = dd[k], sh = 16 * (d & 1u);
            const uint32_t me = (atomicAdd(&s_cnt[d >> 1], 1u << sh) >> sh) & 0xffffu;
            s_rest[me] = rv[k];
            dd[k] = d | (me << kSegDigit);
        }
    }
    __syncthreads();
    DPROF(3);
    // s_cnt now holds every sub-bucket's end; its start is the previous digit's end. Rank in
    // registers; outputs are parked in LDS at their segment slot and stored in slot order.
    const uint64_t newbits = dep_full;
    const bool final_depth = newbits >= 8ull * n;
    // the next element's counter words are read before this element's ranking (one LDS round
    // trip of latency hidden per element)
    auto bound_words = [&](uint32_t k, uint32_t &w0, uint32_t &w1) {
        const uint32_t d = t + k * NT < len ? dd[k] & (kSegDigits1 - 1) : 0u;
        w1 = s_cnt[d >> 1];
        w0 = s_cnt[((d - 1) >> 1) & (FinishShape<NT, CAP>::NDIG / 2 - 1)];
    };
    uint32_t nw0, nw1;
    bound_words(0, nw0, nw1);
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k) {
        const uint32_t w0 = nw0, w1 = nw1;
        if (k + 1 < IPT) bound_words(k + 1, nw0, nw1);
        if (t + k * NT >= len) continue;
        const uint32_t d = dd[k] & (kSegDigits1 - 1), me = dd[k] >> kSegDigit;
        const uint32_t p = packL ? pl[k] >> 8 : pl[k];
        const uint32_t s1 = (w1 >> (16 * (d & 1u))) & 0xffffu;
        const uint32_t s0 = d ? (w0 >> (16 * ((d - 1) & 1u))) & 0xffffu : 0u;
        const uint32_t m = s1 - s0;
        if (m > kSmallM) {
            dd[k] = me;  // deferred, grouped by the 12-bit digit
            if (me == s0) {
                dq_push(a, dq, gstart + s0, m, dep_dig, b, n);
                s_tmp[NT / 64 + 1] = 1;
            }
            continue;
        }
        // rank = #(rest, slot) pairs below this element's (one 64-bit compare per member;
        // sub-buckets hold ~1-4 rotations on random data); ties in the rest are rare and get
        // a second pass for their group's start
        uint32_t c = 0, eqt = 1;
        const uint32_t r = rv[k];
        if (m > 1) {
            const uint64_t key = ((uint64_t)r << 32) | me;
            eqt = 0;
            // the first four members read together (one LDS round trip; m <= 4 for ~99 % of
            // the sub-buckets on random data), the rest one by one
            uint32_t rf4[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                // members 2 and 3 exist for ~40 % / ~13 % of the ranked elements: the reads of
                // lanes without them are masked off (no bank cycles)
                rf4[j] = 0;
                if (j < 2 || s0 + j < s1) rf4[j] = s_rest[s0 + j];
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const bool in = s0 + j < s1;
                c += in && ((((uint64_t)rf4[j]) << 32) | (s0 + j)) < key;
                eqt += in && rf4[j] == r;
            }
#pragma nounroll
            for (uint32_t f = s0 + 4; f < s1; ++f) {
                const uint32_t rf = s_rest[f];
                c += ((((uint64_t)rf) << 32) | f) < key;
                eqt += rf == r;
            }
        }
        const uint32_t local = s0 + c;
        uint32_t gs = gstart + local;
        if (eqt > 1) {  // tied so far: the group starts after the strictly smaller rests
            uint32_t lt = 0;
            for (uint32_t f = s0; f < s1; ++f) lt += s_rest[f] < r;
            gs = gstart + s0 + lt;
            if (c == lt) {  // the group's first slot pushes it
                dq_push(a, dq, gs, eqt, (uint32_t)newbits, b, n);
                s_tmp[NT / 64 + 1] = 1;
            }
        }
        dd[k] = local;  // dd now holds the element's slot in the segment
        if (p == 0 && (eqt == 1 || final_depth)) a.prim[b] = gs - boff;
    }
    DPROF(4);
    dq_flush<NT>(a, dq);
    DPROF(5);
    // slot -> position (<< 8 | L); a slot whose rotation is not final yet gets its L
    // rewritten when a later pass resolves it
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k)
        if (t + k * NT < len) s_rest[dd[k]] = pl[k];
    for (uint32_t i = t; i < FinishShape<NT, CAP>::NDIG / 2; i += NT) s_cnt[i] = 0;
    __syncthreads();
    DPROF(6);
    // the SA of a segment nothing defers is never read again (unless rank doubling needs it)
    const bool wsa = a.full_sa || s_tmp[NT / 64 + 1] != 0;
    if (packL) {
        for (uint32_t i = t; i < len; i += NT) {
            const uint32_t v = s_rest[i];
            if (wsa) a.sa[gstart + i] = v >> 8;
            a.L[gstart + i] = (uint8_t)v;
        }
    } else {
        for (uint32_t i = t; i < len; i += NT) {
            const uint32_t p = s_rest[i];
            if (wsa) a.sa[gstart + i] = p;
            a.L[gstart + i] = lastcol_byte(blk, n, p);
        }
    }
    __syncthreads();
    DPROF(7);
}

// Tiny list segments (len <= kTinyFin), packed: each wave takes 64 consecutive list entries
// and lays their rotations side by side over its lanes in rounds of <= 64 (a segment never
// splits across rounds); each rotation is ranked inside its segment by the next 64 rotation
// bits with wave shuffles. Tie groups of 2-5 rotations are the common case on text, so a wave
// per segment would leave most lanes idle.
// epw = list entries per wave (64, or 16 / 32 when a round's tiny list is short: a wave walks
// its entries' rotations in rounds of 64, so short lists finish sooner spread over more waves)
constexpr uint32_t kTinyPairExt = 4;
__global__ __launch_bounds__(256) void k_finish_tiny(DataArgs a, const Seg4 *__restrict__ lists,
                                                     const uint32_t *__restrict__ loff, const uint32_t *__restrict__ cnt,
                                                     LaneMap lm, uint32_t epw)
{
    __shared__ DeferQueue<kTinyQ> dq;
    // workgroup i: sub-list x of its XCD lane, entries [4 epw j, + 4 epw)
    uint32_t x, j, step;
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    const uint32_t nlist = cnt[x];
    const Seg4 *__restrict__ list = lists + loff[x];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    {
        const uint32_t g0 = j * 4 * epw;
        dq_init(dq);
        __syncthreads();
        const uint32_t i0 = g0 + w * epw;
        if (i0 < nlist) {  // wave-uniform
            const Seg4 sgl = l < epw && i0 + l < nlist ? list[i0 + l] : make_uint4(0, 0, 0, 0);
            const uint32_t incl = wave_incl_sum(sgl.y), st = incl - sgl.y;
            const uint32_t total = __shfl(incl, 63, 64);
            for (uint32_t base = 0; base < total;) {  // wave-uniform rounds
                // the round: the run of segments from `base` that fits in 64 lanes
                const bool in = sgl.y > 0 && st >= base && incl <= base + 64;
                const uint64_t inm = __ballot(in), afterm = __ballot(sgl.y > 0 && st >= base && incl > base + 64);
                const uint32_t s0 = (uint32_t)__ffsll((unsigned long long)inm) - 1;
                const uint32_t nbase = afterm ? (uint32_t)__shfl((int)st, __ffsll((unsigned long long)afterm) - 1, 64) : total;
                uint64_t B = in ? 1ull << (st - base) : 0ull;  // segment starts inside the round
    #pragma unroll
                for (int off = 32; off >= 1; off >>= 1) B |= __shfl_xor(B, off, 64);
                const bool live = l < nbase - base;
                const uint64_t below = l == 63 ? B : B & ((2ull << l) - 1);
                const uint32_t pos = live ? 63u - (uint32_t)__builtin_clzll(below) : 0u;  // my segment's first lane
                const uint32_t sl = s0 + (uint32_t)__builtin_popcountll(B & ((1ull << pos) - 1));
                // (shuffles with the whole wave active: a source lane may be past this round)
                const uint32_t gstart = __shfl((int)sgl.x, (int)sl, 64), slen = __shfl((int)sgl.y, (int)sl, 64);
                const uint32_t db = __shfl((int)sgl.z, (int)sl, 64), b = __shfl((int)sgl.w, (int)sl, 64);
                const uint32_t len = slen * (uint32_t)live;
                const uint32_t idx = l - pos;
                uint32_t p = 0, boff = 0, n = 1;
                uint64_t key = ~0ull;
                const uint8_t *blk = a.data;
                if (live) {
                    boff = a.boffs[b];
                    n = a.boffs[b + 1] - boff;
                    blk = a.data + boff;
                    p = a.sa[gstart + idx];
                    key = rot_window(blk, n, p, db);
                }
                uint32_t mx = len;
    #pragma unroll
                for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
                uint32_t lt = 0, eqb = 0, eqt = 0;
                for (uint32_t j = 0; j < mx; ++j) {  // every lane takes part in the shuffles
                    const int src = (int)min(pos + j, 63u);
                    const uint32_t klo = __shfl((uint32_t)key, src, 64), khi = __shfl((uint32_t)(key >> 32), src, 64);
                    const uint64_t kj = ((uint64_t)khi << 32) | klo;
                    const bool m = j < len;
                    lt += m && kj < key;
                    eqt += m && kj == key;
                    eqb += m && kj == key && j < idx;
                }
                uint64_t newbits = (uint64_t)db + 64;
                // a tied pair (the common text case) looks further right here, up to kTinyPairExt
                // windows, instead of going round the deferred list again
                bool pt = live && len == 2 && eqt == 2 && newbits < 8ull * n;
                for (uint32_t it = 0; it < kTinyPairExt && __ballot(pt); ++it) {  // wave-uniform
                    const uint64_t k2 = pt ? rot_window(blk, n, p, newbits) : 0ull;
                    const int src = (int)(pos + (idx ^ 1u));
                    const uint32_t plo = __shfl((uint32_t)k2, src, 64), phi = __shfl((uint32_t)(k2 >> 32), src, 64);
                    const uint64_t kp = ((uint64_t)phi << 32) | plo;
                    if (pt) {
                        if (kp != k2) {
                            lt = kp < k2;
                            eqb = 0;
                            eqt = 1;
                            pt = false;
                        } else {
                            newbits += 64;
                            pt = newbits < 8ull * n;
                        }
                    }
                }
                if (live) {
                    const bool final_depth = newbits >= 8ull * n;
                    const uint32_t slot = gstart + lt + eqb, gs = gstart + lt;
                    if (eqt > 1 && eqb == 0)
                        dq_push(a, dq, gs, eqt, (uint32_t)min<uint64_t>(newbits, 0xffffffffull), b, n);
                    a.sa[slot] = p;
                    if (eqt == 1 || final_depth) {
                        a.L[slot] = lastcol_byte(blk, n, p);
                        if (p == 0) a.prim[b] = (eqt == 1 ? slot : gs) - boff;
                    }
                }
                base = nbase;
            }
        }
        dq_flush<256>(a, dq);
    }
}

// List segments (lo < len <= CAP) at any depth: rotation windows gathered from the text.
template <uint32_t NT, uint32_t CAP>
__device__ __forceinline__ void finish_seg_one(const DataArgs &a, const Seg4 sg, uint32_t lo)
{
    constexpr uint32_t IPT = FinishShape<NT, CAP>::IPT;
    __shared__ uint32_t s_rest[CAP];
    __shared__ uint32_t s_cnt[FinishShape<NT, CAP>::NDIG / 2];
    __shared__ uint32_t s_tmp[NT / 64 + 2];
    __shared__ DeferQueue<kDeferQ> dq;
    const uint32_t gstart = sg.x, len = sg.y, db = sg.z, b = sg.w;
    if (len <= lo || len > CAP) return;
    dq_init(dq);
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint8_t *blk = a.data + boff;
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < FinishShape<NT, CAP>::NDIG / 2; i += NT) s_cnt[i] = 0;
    if (t == 0) s_tmp[NT / 64 + 1] = 0;
    __shared__ uint32_t s_or[2];
    if (t < 2) s_or[t] = 0;
    // skip the bits every rotation of the segment shares (on text, runs inside words): the
    // counting sort starts at the first bit where two of them differ
    const uint64_t w0 = rot_window(blk, n, a.sa[gstart], db);
    uint32_t pl[IPT], dd[IPT], rv[IPT];
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k) {
        if (t + k * NT < len) {
            pl[k] = a.sa[gstart + t + k * NT];
            const uint64_t w = rot_window(blk, n, pl[k], db);
            acc |= w ^ w0;
            dd[k] = (uint32_t)(w >> (64 - kSegDigit));
            rv[k] = (uint32_t)(w >> (32 - kSegDigit));
        }
    }
    __syncthreads();
    if (acc) {
        atomicOr(&s_or[0], (uint32_t)acc);
        atomicOr(&s_or[1], (uint32_t)(acc >> 32));
    }
    __syncthreads();
    const uint64_t orv = ((uint64_t)s_or[1] << 32) | s_or[0];
    if (orv == 0) {  // equal in all 64 bits: the whole segment goes on, 64 bits deeper
        if (t == 0) dq_push(a, dq, gstart, len, (uint32_t)min<uint64_t>((uint64_t)db + 64, 0xffffffffull), b, n);
        dq_flush<NT>(a, dq);
        return;
    }
    const uint32_t cp = (uint32_t)__builtin_clzll(orv);
    if (cp) {  // the 44 bits after the shared prefix, gathered again
#pragma unroll
        for (uint32_t k = 0; k < IPT; ++k) {
            if (t + k * NT < len) {
                const uint64_t w = rot_window(blk, n, pl[k], db + cp);
                dd[k] = (uint32_t)(w >> (64 - kSegDigit));
                rv[k] = (uint32_t)(w >> (32 - kSegDigit));
            }
        }
    }
    finish_core<NT, CAP>(a, gstart, len, db + cp + kSegDigit, db + cp + kSegDigit + 32u, b, false, pl, dd, rv, s_rest,
                         s_cnt, s_tmp, dq);
}

// one segment per workgroup (grid 8 x the largest lane count from the last wait)
template <uint32_t NT, uint32_t CAP>
__global__ __launch_bounds__(NT) void k_finish_seg(DataArgs a, const Seg4 *__restrict__ list,
                                                   const uint32_t *__restrict__ loff, const uint32_t *__restrict__ cnt,
                                                   uint32_t lo, LaneMap lm)
{
    uint32_t x, j, step;  // sub-list of this workgroup's XCD lane, and its entry
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    if (j < cnt[x]) finish_seg_one<NT, CAP>(a, list[loff[x] + j], lo);
}


// List segments (lo < len <= NT * E) sorted by their whole next 64 rotation bits: bitonic sort of
// (window, position) pairs, then runs of equal windows become the next round's tie groups at
// depth db + 64. On text most rotations share several bytes with their neighbours (SURVEY
// App. D Zipf: median 10, max 44 bytes at 1 MiB blocks), so advancing 64 bits per round instead
// of 12 takes a block through in ~5 rounds instead of ~20.
//
// The network is register-blocked: thread t holds the E elements of indices t * E + e, so the
// stages of distance < E compare registers, distances < 64 E swap with the partner lane by
// shuffles, and only distances >= 64 E (segments > 64 E with NT > 64) go through LDS. Segments
// of <= 512 rotations take one-wave workgroups: no LDS stage and no barrier in the sort.

// compare-exchange of (window, position) pairs: afterwards a <= b when up, else a >= b
__device__ __forceinline__ void rs_cx(uint64_t &ka, uint32_t &pa, uint64_t &kb, uint32_t &pb, bool up)
{
    const bool gt = ka > kb || (ka == kb && pa > pb);
    const bool sw = gt == up;
    const uint64_t k0 = ka, k1 = kb;
    const uint32_t p0 = pa, p1 = pb;
    ka = sw ? k1 : k0;
    kb = sw ? k0 : k1;
    pa = sw ? p1 : p0;
    pb = sw ? p0 : p1;
}

// keep the smaller (keep_min) or the larger of (k, p) and the partner's (ko, po)
__device__ __forceinline__ void rs_keep(uint64_t &k, uint32_t &p, uint64_t ko, uint32_t po, bool keep_min)
{
    const bool mine_gt = k > ko || (k == ko && p > po);
    if (mine_gt == keep_min) {
        k = ko;
        p = po;
    }
}

// LDS slot of index i = u * E + e for the cross-wave stages (e rotated by u: no bank conflicts)
template <uint32_t E>
__device__ __forceinline__ uint32_t rs_phys(uint32_t u, uint32_t e)
{
    return u * E + (e ^ (u & (E - 1)));
}

// Sorts the first M (power of two) of the NT * E elements ascending (the rest are +inf); t is
// the thread's index in the NT sorting it.
template <uint32_t NT, uint32_t E>
__device__ __forceinline__ void reg_bitonic(uint64_t (&k)[E], uint32_t (&p)[E], uint32_t M, uint64_t *s_key,
                                            uint32_t *s_pos, uint32_t t)
{
    for (uint32_t kk = 2; kk <= M; kk <<= 1) {
        const bool tup = ((t * E) & kk) == 0;  // direction of this thread's elements once kk >= E
        for (uint32_t j = kk >> 1; j >= E; j >>= 1) {
            const uint32_t m = j / E;  // partner thread t ^ m
            const bool keep_min = ((t & m) == 0) == tup;
            if (m >= 64) {  // workgroup-uniform: across waves, through LDS
                __syncthreads();
#pragma unroll
                for (uint32_t e = 0; e < E; ++e) {
                    s_key[rs_phys<E>(t, e)] = k[e];
                    s_pos[rs_phys<E>(t, e)] = p[e];
                }
                __syncthreads();
#pragma unroll
                for (uint32_t e = 0; e < E; ++e)
                    rs_keep(k[e], p[e], s_key[rs_phys<E>(t ^ m, e)], s_pos[rs_phys<E>(t ^ m, e)], keep_min);
            } else {
#pragma unroll
                for (uint32_t e = 0; e < E; ++e) {
                    const uint32_t lo = __shfl_xor((uint32_t)k[e], (int)m, 64);
                    const uint32_t hi = __shfl_xor((uint32_t)(k[e] >> 32), (int)m, 64);
                    const uint32_t po = __shfl_xor(p[e], (int)m, 64);
                    rs_keep(k[e], p[e], ((uint64_t)hi << 32) | lo, po, keep_min);
                }
            }
        }
#pragma unroll
        for (uint32_t j = E / 2; j >= 1; j >>= 1) {
            if (j < kk) {
#pragma unroll
                for (uint32_t e = 0; e < E; ++e)
                    if (!(e & j)) rs_cx(k[e], p[e], k[e + j], p[e + j], ((t * E + e) & kk) == 0);
            }
        }
    }
}

// One segment (lo < len <= NT * E) sorted by NT threads (t = index among them; NT = 64: one wave,
// synchronised as a wave). Leaves the sorted windows and positions in s_key / s_pos, writes SA,
// L (resolved slots) and the primary, and returns in hm[e] the length of the tie run headed by
// slot t + e * NT (0: no run of >= 2 starts there) for the caller to defer.
template <uint32_t NT, uint32_t E>
__device__ __forceinline__ void sort_seg(const DataArgs &a, const Seg4 sg, uint32_t t, uint64_t *s_key, uint32_t *s_pos,
                                         uint32_t *s_tail, uint32_t (&hm)[E])
{
    constexpr uint32_t CAP = NT * E;
    static_assert((E & (E - 1)) == 0 && NT % 64 == 0, "register bitonic shape");
    auto sync = [] {
        if constexpr (NT == 64)
            wave_sync();
        else
            __syncthreads();
    };
    const uint32_t gstart = sg.x, len = sg.y, db = sg.z, b = sg.w;
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint8_t *blk = a.data + boff;
    const uint32_t M = len <= 2 ? 2u : 1u << (32 - __builtin_clz(len - 1));  // pow2 >= len
    // the network sorts slots [0, M): threads t < M / E hold them (slot t * E + e); the order
    // inside is free, so the loads are coalesced (element e * R + t of the segment)
    const uint32_t R = M >= E ? M / E : 1u;
    uint64_t k[E];
    uint32_t p[E];
#pragma unroll
    for (uint32_t e = 0; e < E; ++e) {
        const uint32_t i = e * R + t;
        k[e] = ~0ull;
        p[e] = 0xffffffffu;
        if (t < R && i < len) {
            p[e] = a.sa[gstart + i];
            k[e] = rot_window(blk, n, p[e], db);
        }
    }
    for (uint32_t i = t; i < CAP / 32; i += NT) s_tail[i] = 0;
    reg_bitonic<NT, E>(k, p, M, s_key, s_pos, t);
    if (M > 64 * E) sync();  // the last LDS stage's reads
#pragma unroll
    for (uint32_t e = 0; e < E; ++e) {
        s_key[t * E + e] = k[e];
        s_pos[t * E + e] = p[e];
    }
    sync();
    // runs of equal windows: tails marked in a bitset, each head finds its tail
    for (uint32_t i = t; i < len; i += NT)
        if (i + 1 == len || s_key[i + 1] != s_key[i]) atomicOr(&s_tail[i >> 5], 1u << (i & 31u));
    sync();
    const bool final_depth = (uint64_t)db + 64 >= 8ull * n;
#pragma unroll
    for (uint32_t e = 0; e < E; ++e) {
        const uint32_t i = t + e * NT;
        hm[e] = 0;
        if (i >= len) continue;
        const uint32_t pp = s_pos[i];
        const bool head = i == 0 || s_key[i - 1] != s_key[i];
        bool single = true;
        if (!(head && ((s_tail[i >> 5] >> (i & 31u)) & 1u))) {  // part of a tie run
            single = false;
            if (head) {
                uint32_t w = i >> 5, bits = s_tail[w] & (0xffffffffu << (i & 31u));
                while (bits == 0) bits = s_tail[++w];
                hm[e] = 32 * w + __builtin_ctz(bits) + 1 - i;
            }
        }
        a.sa[gstart + i] = pp;
        if (single || final_depth) {
            a.L[gstart + i] = lastcol_byte(blk, n, pp);
            if (pp == 0) {
                uint32_t gs = i;
                if (!single)
                    while (gs > 0 && s_key[gs - 1] == s_key[i]) --gs;
                a.prim[b] = gstart + gs - boff;
            }
        }
    }
}

// the tie runs sort_seg found, deferred 64 bits deeper
template <uint32_t NT, uint32_t E, uint32_t Q>
__device__ __forceinline__ void sort_seg_defer(const DataArgs &a, const Seg4 sg, uint32_t t, const uint32_t (&hm)[E],
                                               DeferQueue<Q> &dq)
{
    const uint32_t n = a.boffs[sg.w + 1] - a.boffs[sg.w];
    const uint32_t nd = (uint32_t)min<uint64_t>((uint64_t)sg.z + 64, 0xffffffffull);
#pragma unroll
    for (uint32_t e = 0; e < E; ++e)
        if (hm[e]) dq_push(a, dq, sg.x + t + e * NT, hm[e], nd, sg.w, n);
}

// Segments of 2 .. NT * E rotations (NT >= 128), one per workgroup (grid 8 x the rows of the
// fullest sub-list from the last wait); the deferral queue overlays the windows once sorted.
template <uint32_t NT, uint32_t E>
__global__ __launch_bounds__(NT) void k_finish_sort(DataArgs a, const Seg4 *__restrict__ list,
                                                    const uint32_t *__restrict__ loff, const uint32_t *__restrict__ cnt,
                                                    uint32_t lo, LaneMap lm)
{
    constexpr uint32_t CAP = NT * E;
    constexpr uint32_t Q = CAP / 4;
    static_assert(sizeof(DeferQueue<Q>) <= CAP * 8, "deferral queue overlays the windows");
    __shared__ __align__(16) uint64_t s_key[CAP];
    __shared__ uint32_t s_pos[CAP];
    __shared__ uint32_t s_tail[CAP / 32];
    uint32_t x, j, step;  // sub-list of this workgroup's XCD lane, and its entry
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    if (j >= cnt[x]) return;
    const Seg4 sg = list[loff[x] + j];
    if (sg.y <= lo || sg.y > CAP) return;
    uint32_t hm[E];
    sort_seg<NT, E>(a, sg, threadIdx.x, s_key, s_pos, s_tail, hm);
    __syncthreads();
    DeferQueue<Q> &dq = *reinterpret_cast<DeferQueue<Q> *>(s_key);
    dq_init(dq);
    __syncthreads();
    sort_seg_defer<NT, E>(a, sg, threadIdx.x, hm, dq);
    dq_flush<NT>(a, dq);
}

// Segments of 2 .. 64 E rotations, W per workgroup: one per wave (entries W j .. W j + W - 1 of
// the sub-list), one shared deferral queue (a workgroup per segment would flush a queue, i.e.
// take global atomics on the same few list counters, per segment).
constexpr uint32_t kSortWQ = 256;
template <uint32_t E, uint32_t W>
__global__ __launch_bounds__(64 * W) void k_finish_sortw(DataArgs a, const Seg4 *__restrict__ list,
                                                         const uint32_t *__restrict__ loff,
                                                         const uint32_t *__restrict__ cnt, uint32_t lo, LaneMap lm)
{
    constexpr uint32_t CAP = 64 * E;
    __shared__ __align__(16) uint64_t s_key[W][CAP];
    __shared__ uint32_t s_pos[W][CAP];
    __shared__ uint32_t s_tail[W][CAP / 32];
    __shared__ DeferQueue<kSortWQ> dq;
    uint32_t x, j, step;
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    dq_init(dq);
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6, l = threadIdx.x & 63u, jj = j * W + wv;
    if (jj < cnt[x]) {  // wave-uniform
        const Seg4 sg = list[loff[x] + jj];
        if (sg.y > lo && sg.y <= CAP) {
            uint32_t hm[E];
            sort_seg<64, E>(a, sg, l, s_key[wv], s_pos[wv], s_tail[wv], hm);
            sort_seg_defer<64, E>(a, sg, l, hm, dq);
        }
    }
    dq_flush<64 * W>(a, dq);
}

// Dense finish of the global pass's buckets (db = kG1Bits), one workgroup per bucket,
// XCD-aware: workgroup i -> lane i % 8 -> blocks b = lane mod 8. Compact records read
// coalesced. (A persistent variant that prefetched the next bucket into registers measured
// slower: the extra registers cost a workgroup per CU.)
template <uint32_t NT, uint32_t CAP>
__global__ __launch_bounds__(NT) void k_finish_dense(DataArgs a, const uint2 *__restrict__ bk,
                                                     const uint64_t *__restrict__ rec)
{
    constexpr uint32_t IPT = FinishShape<NT, CAP>::IPT;
    __shared__ uint32_t s_rest[CAP];
    __shared__ uint32_t s_cnt[FinishShape<NT, CAP>::NDIG / 2];
    __shared__ uint32_t s_tmp[NT / 64 + 2];
    __shared__ DeferQueue<kDeferQ> dq;
    const uint32_t x = blockIdx.x & 7u, kb = blockIdx.x >> 3;
    const uint32_t b = x + 8u * (kb >> kG1Bits);
    if (b >= a.nb) return;
    const uint2 e = bk[(size_t)b * kG1Bins + (kb & (kG1Bins - 1))];
    if (e.y < 2 || e.y > CAP) return;
    const uint32_t t = threadIdx.x;
    DPROF_START;
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint32_t info = __builtin_amdgcn_readfirstlane(a.ainfo[b]);  // uniform (keeps it out of VGPRs)
    const uint32_t P = rec_pbits(n), R = __builtin_amdgcn_readfirstlane(rec_rbits(P, g1_db(info), rec_nsym(info, 32u) != 0));
    uint32_t dep_dig, dep_full;
    dense_depths(info, R, dep_dig, dep_full);
    dep_dig = __builtin_amdgcn_readfirstlane(dep_dig);  // uniform: SGPRs (65 VGPRs cost a workgroup per CU)
    dep_full = __builtin_amdgcn_readfirstlane(dep_full);
    const bool packL = P <= 24;
    for (uint32_t i = t; i < FinishShape<NT, CAP>::NDIG / 2; i += NT) s_cnt[i] = 0;
    if (t == 0) s_tmp[NT / 64 + 1] = 0;
    dq_init(dq);
    const uint64_t *r0 = rec + boff + e.x;
    uint32_t pl[IPT], dd[IPT], rv[IPT];
    // every record load in flight before the first is decoded (a load under a per-element
    // branch waits for its data inside the branch: IPT HBM round trips in a row)
    uint64_t raw[IPT];
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k) raw[k] = r0[min(t + k * NT, e.y - 1)];
#pragma unroll
    for (uint32_t k = 0; k < IPT; ++k) {
        if (t + k * NT < e.y) {
            const uint64_t r = raw[k];
            const uint64_t sub = r >> (P + 8);
            const uint32_t p = (uint32_t)(r >> 8) & (uint32_t)((1ull << P) - 1);
            pl[k] = packL ? (p << 8) | ((uint32_t)r & 255u) : p;
            dd[k] = (uint32_t)(sub >> R);
            rv[k] = (uint32_t)(sub & ((1ull << R) - 1));
        }
    }
    __syncthreads();
    DPROF(0);
    finish_core<NT, CAP>(a, boff + e.x, e.y, dep_dig, dep_full, b, packL, pl, dd, rv, s_rest, s_cnt, s_tmp, dq);
}

// ------------------------------------------------------------- MSD passes on data bits
struct DTile {
    uint32_t seg, start, len, pad;
};

__device__ __forceinline__ uint32_t seg_blk(uint32_t w) { return w & 0xffffu; }

// Bits every rotation of an MSD segment shares below its depth (OR of window XORs against
// the segment's first rotation), and its smallest window; the digit of the pass is taken right
// after the shared bits (or, kRunMode, from the first difference to the smallest window). Each
// rotation's 64-bit window is kept in kbuf (by slot) so the histogram and scatter passes read it
// coalesced instead of gathering it from the text again.
__device__ __forceinline__ void dcp_one(const DataArgs &a, const Seg4 *__restrict__ segs, const DTile t,
                                        unsigned long long *__restrict__ segor, unsigned long long *__restrict__ segmin,
                                        uint64_t *__restrict__ kbuf)
{
    __shared__ uint32_t s_or[2];
    __shared__ unsigned long long s_min;
    const Seg4 s = segs[t.seg];
    const uint32_t b = seg_blk(s.w), boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint8_t *blk = a.data + boff;
    if (threadIdx.x < 2) s_or[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_min = ~0ull;
    __syncthreads();
    const bool recw = seg_known(s.w) != 0;  // windows already in kbuf
    const uint64_t w0 = recw ? kbuf[s.x] : rot_window(blk, n, a.sa[s.x], s.z);
    uint64_t acc = 0, mn = ~0ull;
    for (uint32_t e = threadIdx.x; e < t.len; e += 256) {
        uint64_t w;
        if (recw) {
            w = kbuf[t.start + e];
        } else {
            w = rot_window(blk, n, a.sa[t.start + e], s.z);
            kbuf[t.start + e] = w;
        }
        acc |= w ^ w0;
        mn = w < mn ? w : mn;
    }
    if (acc) {
        atomicOr(&s_or[0], (uint32_t)acc);
        atomicOr(&s_or[1], (uint32_t)(acc >> 32));
    }
    if (s.w & kRunMode) atomicMin(&s_min, (unsigned long long)mn);
    __syncthreads();
    if (threadIdx.x == 0 && (s_or[0] | s_or[1])) atomicOr(&segor[t.seg], ((unsigned long long)s_or[1] << 32) | s_or[0]);
    if (threadIdx.x == 0 && (s.w & kRunMode)) atomicMin(&segmin[t.seg], s_min);
}

// grid-stride over the pass's tiles (count on the device, k_tiles)
__global__ __launch_bounds__(256) void k_dcp(DataArgs a, const Seg4 *__restrict__ segs, const DTile *__restrict__ tiles,
                                             const uint32_t *__restrict__ tstart, unsigned long long *__restrict__ segor,
                                             unsigned long long *__restrict__ segmin, uint64_t *__restrict__ kbuf, LaneMap lm)
{
    // workgroup i strides over the tiles of its XCD lane's sub-list
    uint32_t x, j, step;
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    for (uint32_t tb = tstart[x] + j; tb < tstart[x + 1]; tb += step) {
        dcp_one(a, segs, tiles[tb], segor, segmin, kbuf);
        __syncthreads();
    }
}

// depth of the pass digit: the segment depth plus its shared bits (64: no digit in the window)
__device__ __forceinline__ uint32_t seg_cp(const unsigned long long *segor, uint32_t seg, uint32_t w)
{
    const unsigned long long o = segor[seg];
    const uint32_t cp = o ? (uint32_t)__builtin_clzll(o) : 64u;
    const uint32_t K = seg_known(w);
    return K ? min(cp, K - kMsdBits) : cp;
}

// the pass digit of slot j: from the stored window, or (digit past the window) from the text
__device__ __forceinline__ uint32_t msd_digit(const uint64_t *kbuf, uint32_t j, uint32_t cp, const uint8_t *blk, uint32_t n,
                                              uint32_t p, uint32_t depth)
{
    return cp <= 64 - kMsdBits ? (uint32_t)((kbuf[j] << cp) >> (64 - kMsdBits))
                               : (uint32_t)(rot_window(blk, n, p, depth + cp) >> (64 - kMsdBits));
}

// Known window bits of a (non-run-mode) segment's children after a pass whose digit starts cp
// bits in: the parent's (64 for gathered windows) minus the cp + kMsdBits consumed; 0 (gather)
// when fewer than a digit's worth would remain.
__device__ __forceinline__ uint32_t child_known(uint32_t w, uint32_t cp)
{
    if ((w & kRunMode) || cp == 64) return 0;
    const uint32_t K = seg_known(w) ? seg_known(w) : 64u, used = cp + kMsdBits;
    return K >= used + kMsdBits ? K - used : 0u;
}

// kRunMode digit: 0 for the smallest window, else 64 - (bits shared with it), in 1..64
__device__ __forceinline__ uint32_t run_digit(uint64_t w, uint64_t wmin)
{
    const uint64_t x = w ^ wmin;
    return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u;
}

__device__ __forceinline__ void dhist_one(const DataArgs &a, const Seg4 *__restrict__ segs, const DTile t, uint32_t tb,
                                          const unsigned long long *__restrict__ segor,
                                          const unsigned long long *__restrict__ segmin,
                                          const uint64_t *__restrict__ kbuf, uint32_t *__restrict__ thist)
{
    __shared__ uint32_t h[kMsdBins];
    const Seg4 s = segs[t.seg];
    const uint32_t b = seg_blk(s.w), boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint8_t *blk = a.data + boff;
    const uint32_t cp = seg_cp(segor, t.seg, s.w);
    h[threadIdx.x] = 0;
    __syncthreads();
    if (s.w & kRunMode) {
        const uint64_t wmin = segmin[t.seg];
        for (uint32_t e = threadIdx.x; e < t.len; e += kMsdBins) atomicAdd(&h[run_digit(kbuf[t.start + e], wmin)], 1u);
    } else if (cp == 64) {
        if (threadIdx.x == 0) h[0] = t.len;
    } else {
        for (uint32_t e = threadIdx.x; e < t.len; e += kMsdBins) {
            const uint32_t j = t.start + e;
            atomicAdd(&h[msd_digit(kbuf, j, cp, blk, n, cp <= 64 - kMsdBits ? 0u : a.sa[j], s.z)], 1u);
        }
    }
    __syncthreads();
    thist[(size_t)tb * kMsdBins + threadIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(kMsdBins) void k_dhist(DataArgs a, const Seg4 *__restrict__ segs, const DTile *__restrict__ tiles,
                                               const uint32_t *__restrict__ tstart,
                                               const unsigned long long *__restrict__ segor,
                                               const unsigned long long *__restrict__ segmin,
                                               const uint64_t *__restrict__ kbuf, uint32_t *__restrict__ thist, LaneMap lm)
{
    // workgroup i strides over the tiles of its XCD lane's sub-list
    uint32_t x, j, step;
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    for (uint32_t tb = tstart[x] + j; tb < tstart[x + 1]; tb += step) {
        dhist_one(a, segs, tiles[tb], tb, segor, segmin, kbuf, thist);
        __syncthreads();
    }
}

// grid = nsegs; 256 threads (digits). Offsets in place; sub-segment routing. A child left
// with >= 3/4 of its parent and still too big for a finish pass goes on in kRunMode.
__device__ __forceinline__ void dscan_one(const DataArgs &a, const Seg4 *__restrict__ segs, uint32_t sgi,
                                          const uint2 *__restrict__ segtiles, const unsigned long long *__restrict__ segor,
                                          uint32_t *__restrict__ thist, uint32_t *__restrict__ stot,
                                          uint32_t *__restrict__ nomove)
{
    __shared__ uint32_t s_tmp[kMsdBins / 64 + 1];
    const Seg4 s = segs[sgi];
    const uint2 tr = segtiles[sgi];
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
    for (uint32_t t = tr.x; t < tr.x + tr.y; ++t) {
        const uint32_t v = thist[(size_t)t * kMsdBins + d];
        thist[(size_t)t * kMsdBins + d] = run;
        run += v;
    }
    const uint32_t tot = run;
    const int nz = __syncthreads_count(tot > 0);
    const uint32_t base = block_excl_sum<kMsdBins>(tot, s_tmp, nullptr);
    for (uint32_t t = tr.x; t < tr.x + tr.y; ++t) thist[(size_t)t * kMsdBins + d] += s.x + base;
    stot[(size_t)sgi * kMsdBins + d] = tot;
    const uint32_t b = seg_blk(s.w), n = a.boffs[b + 1] - a.boffs[b];
    const uint32_t cp = seg_cp(segor, sgi, s.w);
    // depth of this thread's child: kRunMode digit d shares 64 - d bits with the minimum and
    // differs in the next one (d = 0: all 64 window bits equal the minimum's)
    const uint32_t add = (s.w & kRunMode) ? (d == 0 ? 64u : 64u - d + 1u) : (cp == 64 ? 64u : cp + kMsdBits);
    const uint32_t nd = (uint32_t)min<uint64_t>((uint64_t)s.z + add, 0xffffffffull);
    const bool final_depth = (uint64_t)nd >= 8ull * n;
    __shared__ DeferQueue<kMsdBins> dq;
    dq_init(dq);
    __syncthreads();
    auto route = [&](uint32_t gs, uint32_t len) {
        if (len == 1) return;  // resolved by the scatter
        if (final_depth || nd >= a.dbl_bits) {
            if (!final_depth) {
                a.bflag[b] = 1;
                a.cnt->flagged = 1;
            }
            dq_push_list(a, dq, make_uint4(gs, len, nd, b | (final_depth ? kFinalFlag : 0u)), kListGroups);
        } else if (len <= a.big_cap) {
            dq_push(a, dq, gs, len, nd, b, n);
        } else {
            const bool stuck = (uint64_t)len * 4 >= (uint64_t)s.y * 3;
            // a child keeps its window in the next window buffer (written by the scatter)
            dq_push_list(a, dq, make_uint4(gs, len, nd, b | (stuck ? kRunMode : child_known(s.w, cp) << kWinShift)),
                         kListBig);
        }
    };
    if (nz == 1) {
        if (d == 0) nomove[sgi] = 1;
        if (tot > 0) route(s.x, s.y);
    } else {
        if (d == 0) nomove[sgi] = 0;
        if (tot > 0) route(s.x + base, tot);
    }
    dq_flush<kMsdBins>(a, dq);
}

__global__ __launch_bounds__(kMsdBins) void k_dscan(DataArgs a, const Seg4 *__restrict__ segs, const uint32_t *__restrict__ loff,
                                               const uint32_t *__restrict__ cnt, const uint2 *__restrict__ segtiles,
                                               const unsigned long long *__restrict__ segor, uint32_t *__restrict__ thist,
                                               uint32_t *__restrict__ stot, uint32_t *__restrict__ nomove, LaneMap lm)
{
    // segment ids are big-list indices; workgroup i strides over its XCD lane's sub-list
    uint32_t x, j0, step;
    lane_of(lm, blockIdx.x, x, j0, step, gridDim.x >> 3);
    for (uint32_t j = j0; j < cnt[x]; j += step) {
        dscan_one(a, segs, loff[x] + j, segtiles, segor, thist, stot, nomove);
        __syncthreads();
    }
}

__device__ __forceinline__ void dscatter_one(const DataArgs &a, const Seg4 *__restrict__ segs, const DTile t, uint32_t tb,
                                             const unsigned long long *__restrict__ segor,
                                             const unsigned long long *__restrict__ segmin,
                                             const uint64_t *__restrict__ kbuf, const uint32_t *__restrict__ nomove,
                                             const uint32_t *__restrict__ thist, const uint32_t *__restrict__ stot,
                                             uint32_t *__restrict__ sa2, uint64_t *__restrict__ kbuf_next)
{
    __shared__ uint32_t cur[kMsdBins];
    const Seg4 s = segs[t.seg];
    const uint32_t b = seg_blk(s.w), boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint8_t *blk = a.data + boff;
    if (nomove[t.seg]) return;  // one digit only: nothing moves (the segment goes on in run mode)
    const uint32_t cp = seg_cp(segor, t.seg, s.w);
    const bool runm = (s.w & kRunMode) != 0;
    const uint64_t wmin = runm ? segmin[t.seg] : 0ull;
    const uint32_t kc = child_known(s.w, cp), used = cp + kMsdBits;
    cur[threadIdx.x] = thist[(size_t)tb * kMsdBins + threadIdx.x];
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < t.len; e += kMsdBins) {
        const uint32_t j = t.start + e;
        const uint32_t p = a.sa[j];
        const uint32_t d = runm ? run_digit(kbuf[j], wmin) : msd_digit(kbuf, j, cp, blk, n, p, s.z);
        const uint32_t slot = atomicAdd(&cur[d], 1u);
        sa2[slot] = p;
        const uint32_t cn = stot[(size_t)t.seg * kMsdBins + d];  // the child's length
        // a child that returns to the big list (not in run mode) keeps its window, past this
        // pass's bits (dscan_one routes by the same rule)
        if (kc && cn > a.big_cap && (uint64_t)cn * 4 < (uint64_t)s.y * 3) kbuf_next[slot] = kbuf[j] << used;
        if (cn == 1) put_final(a, b, boff, n, blk, slot, p, slot - boff);
    }
}

__global__ __launch_bounds__(kMsdBins) void k_dscatter(DataArgs a, const Seg4 *__restrict__ segs, const DTile *__restrict__ tiles,
                                                  const uint32_t *__restrict__ tstart,
                                                  const unsigned long long *__restrict__ segor,
                                                  const unsigned long long *__restrict__ segmin,
                                                  const uint64_t *__restrict__ kbuf, const uint32_t *__restrict__ nomove,
                                                  const uint32_t *__restrict__ thist, const uint32_t *__restrict__ stot,
                                                  uint32_t *__restrict__ sa2, uint64_t *__restrict__ kbuf_next, LaneMap lm)
{
    // workgroup i strides over the tiles of its XCD lane's sub-list
    uint32_t x, j, step;
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    for (uint32_t tb = tstart[x] + j; tb < tstart[x + 1]; tb += step) {
        dscatter_one(a, segs, tiles[tb], tb, segor, segmin, kbuf, nomove, thist, stot, sa2, kbuf_next);
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_dcopy(const DTile *__restrict__ tiles, const uint32_t *__restrict__ tstart,
                                               const uint32_t *__restrict__ nomove, uint32_t *__restrict__ sa,
                                               const uint32_t *__restrict__ sa2, LaneMap lm)
{
    uint32_t x, j, step;
    lane_of(lm, blockIdx.x, x, j, step, gridDim.x >> 3);
    for (uint32_t tb = tstart[x] + j; tb < tstart[x + 1]; tb += step) {
        const DTile t = tiles[tb];
        if (nomove[t.seg]) continue;
        for (uint32_t e = threadIdx.x; e < t.len; e += 256) sa[t.start + e] = sa2[t.start + e];
    }
}

// -------------------------------------------------------------------- lazy rank fill
// rank[p] = slot of p for every slot of a flagged block (both rank buffers).
__global__ __launch_bounds__(256) void k_rank_fill(const uint32_t *__restrict__ boffs, const uint32_t *__restrict__ bflag,
                                                   const uint32_t *__restrict__ sa, uint32_t *__restrict__ rkA,
                                                   uint32_t *__restrict__ rkB)
{
    const uint32_t b = blockIdx.y;
    if (!bflag[b]) return;
    const uint32_t boff = boffs[b], n = boffs[b + 1] - boff;
    const uint32_t j0 = blockIdx.x * 4096u;
    if (j0 >= n) return;
    const uint32_t j1 = min(j0 + 4096u, n);
    for (uint32_t j = j0 + threadIdx.x; j < j1; j += 256) {
        const uint32_t p = sa[boff + j];
        rkA[boff + p] = j;
        rkB[boff + p] = j;
    }
}

// Tied groups of the data phase: members get the group start as rank (flagged blocks);
// identical-rotation (final) groups also get their L bytes / primary. Unresolved ones are
// appended to the first doubling round's segment list. One wave per group; groups longer than
// kCoopGroup (long runs: a wave would walk 100 K+ rotations alone) are listed in `coop` for
// k_group_fill_coop, which spreads each over the whole grid.
__device__ __forceinline__ void group_fill_elem(const DataArgs &a, const Seg4 &s, uint32_t e, uint32_t *__restrict__ rkA,
                                                uint32_t *__restrict__ rkB)
{
    const uint32_t b = s.w & ~kFinalFlag;
    const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
    const uint32_t p = a.sa[s.x + e];
    if (a.bflag[b]) {
        rkA[boff + p] = s.x - boff;
        rkB[boff + p] = s.x - boff;
    }
    if (s.w & kFinalFlag) put_final(a, b, boff, n, a.data + boff, s.x + e, p, s.x - boff);
}

// Groups of up to kLaneGroup members are filled one per lane (a text's data phase leaves
// ~100 K groups of 2-3 rotations; a wave per group idled 62 lanes and appended with one atomic
// per group); longer ones take the whole wave, one at a time. One atomicMin per wave.
constexpr uint32_t kLaneGroup = 16;
__global__ __launch_bounds__(256) void k_group_fill(DataArgs a, const Seg4 *__restrict__ groups, uint32_t ng,
                                                    uint32_t *__restrict__ rkA, uint32_t *__restrict__ rkB,
                                                    uint2 *__restrict__ segs, uint32_t *__restrict__ coop, Counters *cnt)
{
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t l = threadIdx.x & 63u;
    uint32_t dmin = 0xffffffffu;
    for (uint32_t base = wave * 64u; base < ng; base += nwaves * 64u) {
        const uint32_t g = base + l;
        const Seg4 s = g < ng ? groups[g] : Seg4{0, 0, 0, 0};
        if (g < ng && s.y <= kLaneGroup) {
            for (uint32_t e = 0; e < s.y; ++e) group_fill_elem(a, s, e, rkA, rkB);
            if (!(s.w & kFinalFlag)) {
                segs[wave_append(&cnt->next)] = make_uint2(s.x, s.y);
                dmin = min(dmin, s.z);
            }
        }
        uint64_t big = __ballot(g < ng && s.y > kLaneGroup);
        while (big) {
            const uint32_t j = (uint32_t)__builtin_ctzll(big);
            big &= big - 1;
            const Seg4 t = groups[base + j];
            if (t.y > kCoopGroup) {
                if (l == 0) coop[atomicAdd(&cnt->coop_fill, 1u)] = base + j;
                continue;
            }
            for (uint32_t e = l; e < t.y; e += 64) group_fill_elem(a, t, e, rkA, rkB);
            if (!(t.w & kFinalFlag) && l == 0) {
                segs[atomicAdd(&cnt->next, 1u)] = make_uint2(t.x, t.y);
                dmin = min(dmin, t.z);
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) dmin = min(dmin, (uint32_t)__shfl_xor((int)dmin, off, 64));
    if (l == 0 && dmin != 0xffffffffu) atomicMin(&cnt->dmin_bits, dmin);
}

__global__ __launch_bounds__(256) void k_group_fill_coop(DataArgs a, const Seg4 *__restrict__ groups,
                                                         const uint32_t *__restrict__ coop, uint32_t *__restrict__ rkA,
                                                         uint32_t *__restrict__ rkB, uint2 *__restrict__ segs, Counters *cnt)
{
    const uint32_t nc = cnt->coop_fill;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    for (uint32_t i = 0; i < nc; ++i) {
        const Seg4 s = groups[coop[i]];
        for (uint32_t e = tid; e < s.y; e += nt) group_fill_elem(a, s, e, rkA, rkB);
        if (!(s.w & kFinalFlag) && tid == 0) {
            segs[atomicAdd(&cnt->next, 1u)] = make_uint2(s.x, s.y);
            atomicMin(&cnt->dmin_bits, s.z);
        }
    }
}

// ======================================================================= doubling phase
struct RoundArgs {
    const uint8_t *data;
    const uint32_t *boffs;
    uint32_t nb;
    uint32_t *sa;
    uint8_t *L;
    uint32_t *prim;
    const uint32_t *rk_cur;
    uint32_t *rk_nxt;
    uint32_t D;          // current depth in bytes (key = rank_D at p + D)
    uint64_t newD;       // depth reached by this round
    uint2 *next;
    uint32_t *resolved;  // positions resolved this round (batch index of p) -> committed after
    Counters *cnt;
    uint32_t *next_cnt;  // entries of `next` (cnt->next or cnt->next2, alternating by round)
};

__device__ __forceinline__ uint32_t round_key(const RoundArgs &a, uint32_t boff, uint32_t n, uint32_t p)
{
    uint64_t q = (uint64_t)p + (a.D % n);
    if (q >= n) q -= n;
    return a.rk_cur[boff + (uint32_t)q];
}

// Element p (block-local) now at batch slot gslot, in a depth-newD group starting at
// block-local slot gs with gsz members; `first` marks one member per group.
__device__ __forceinline__ void finish(const RoundArgs &a, uint32_t boff, uint32_t n, uint32_t p, uint32_t gslot,
                                       uint32_t gs, uint32_t gsz, bool first)
{
    const bool final_ = gsz == 1 || a.newD >= n;
    a.rk_nxt[boff + p] = gs;
    if (final_) {
        const uint32_t i = wave_append(&a.cnt->resolved);
        a.resolved[i] = boff + p;
        a.L[gslot] = a.data[boff + (p == 0 ? n - 1 : p - 1)];
        if (p == 0) {
            const uint32_t b = find_block(a.boffs, a.nb, boff);
            a.prim[b] = gs;
        }
    } else if (first) {
        const uint32_t i = wave_append(a.next_cnt);
        a.next[i] = make_uint2(boff + gs, gsz);
    }
}

__device__ __forceinline__ void classify_one(const uint2 s, uint2 *__restrict__ tiny, uint2 *__restrict__ med,
                                             LSeg *__restrict__ large, Counters *cnt, const uint32_t *__restrict__ boffs,
                                             uint32_t nb)
{
    if (s.y <= kTinyMax) {
        tiny[wave_append(&cnt->tiny)] = s;
    } else if (s.y <= kMedMax) {
        med[wave_append(&cnt->med)] = s;
    } else {
        LSeg l;
        // keys are block-local ranks (< n): the first MSD pass takes their highest nonzero byte
        const uint32_t b = find_block(boffs, nb, s.x), n = boffs[b + 1] - boffs[b];
        l.gstart = s.x;
        l.len = s.y;
        l.shift = n > (1u << 24) ? 24u : n > (1u << 16) ? 16u : n > 256u ? 8u : 0u;
        l.gathered = 0;
        large[wave_append(&cnt->large)] = l;
    }
}

// Grid-stride over the nseg_p[0] segments the previous round left (read on the device: the
// host learns the class counts from the same wait that gives it the segment count).
__global__ void k_classify(const uint2 *__restrict__ segs, const uint32_t *__restrict__ nseg_p, uint2 *__restrict__ tiny,
                           uint2 *__restrict__ med, LSeg *__restrict__ large, Counters *cnt,
                           const uint32_t *__restrict__ boffs, uint32_t nb)
{
    const uint32_t nseg = *nseg_p;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nseg; i += gridDim.x * blockDim.x)
        classify_one(segs[i], tiny, med, large, cnt, boffs, nb);
}

// Tiles of <= kDTile slots over a segment list whose length is on the device: one workgroup
// scans the tile counts (1024 segments per step) and writes tiles[] (seg, start, len),
// segtiles[s] = {first tile, tile count} and *ntiles. S: {gstart, len, ...} in its first two
// words (Seg4, LSeg). With `orv`/`mnv`, the per-segment OR / minimum accumulators of the data
// phase's MSD pass are reset too.
template <class S, class T>
__global__ __launch_bounds__(1024) void k_tiles(const S *__restrict__ segs, const uint32_t *__restrict__ nseg_p,
                                                T *__restrict__ tiles, uint2 *__restrict__ segtiles,
                                                uint32_t *__restrict__ ntiles, unsigned long long *__restrict__ orv,
                                                unsigned long long *__restrict__ mnv)
{
    __shared__ uint32_t s_tmp[17];
    const uint32_t nseg = *nseg_p;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nseg; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        uint32_t st = 0, ln = 0, nt = 0;
        if (i < nseg) {
            const uint32_t *w = (const uint32_t *)&segs[i];
            st = w[0];
            ln = w[1];
            nt = (ln + kDTile - 1) / kDTile;
        }
        uint32_t total;
        const uint32_t ex = carry + block_excl_sum<1024>(nt, s_tmp, &total);
        if (i < nseg) {
            segtiles[i] = make_uint2(ex, nt);
            for (uint32_t j = 0; j < nt; ++j) {
                T t;
                t.seg = i;
                t.start = st + j * kDTile;
                t.len = min(kDTile, ln - j * kDTile);
                t.pad = 0;
                tiles[ex + j] = t;
            }
            if (orv) orv[i] = 0;
            if (mnv) mnv[i] = ~0ull;
        }
        carry += total;
    }
    if (threadIdx.x == 0) *ntiles = carry;
}

// Data-phase MSD tiles: the big list's lane sub-lists in lane order (tiles of lane x from
// cnt->tstart[x]); segment ids are big-list indices (loff[x] + j). Resets the per-segment OR /
// minimum accumulators. One workgroup.
__global__ __launch_bounds__(1024) void k_dtiles(const Seg4 *__restrict__ segs, const uint32_t *__restrict__ loff,
                                                 const uint32_t *__restrict__ cnt, DTile *__restrict__ tiles,
                                                 uint2 *__restrict__ segtiles, uint32_t *__restrict__ tstart,
                                                 unsigned long long *__restrict__ orv, unsigned long long *__restrict__ mnv)
{
    __shared__ uint32_t s_tmp[17];
    uint32_t carry = 0;
    for (uint32_t x = 0; x < 8; ++x) {
        if (threadIdx.x == 0) tstart[x] = carry;
        const uint32_t nseg = cnt[x], s0 = loff[x];
        for (uint32_t base = 0; base < nseg; base += 1024) {
            const uint32_t j = base + threadIdx.x, i = s0 + j;
            uint32_t st = 0, ln = 0, nt = 0;
            if (j < nseg) {
                st = segs[i].x;
                ln = segs[i].y;
                nt = (ln + kDTile - 1) / kDTile;
            }
            uint32_t total;
            const uint32_t ex = carry + block_excl_sum<1024>(nt, s_tmp, &total);
            if (j < nseg) {
                segtiles[i] = make_uint2(ex, nt);
                for (uint32_t k = 0; k < nt; ++k) {
                    DTile t;
                    t.seg = i;
                    t.start = st + k * kDTile;
                    t.len = min(kDTile, ln - k * kDTile);
                    t.pad = 0;
                    tiles[ex + k] = t;
                }
                orv[i] = 0;
                mnv[i] = ~0ull;
            }
            carry += total;
        }
    }
    if (threadIdx.x == 0) tstart[8] = carry;
}

// Doubling-phase segments of <= kTinyMax (64) rotations, packed like k_finish_tiny: each wave
// takes 64 consecutive list entries and lays their rotations side by side over its lanes in
// rounds of <= 64; each rotation's new slot = segment start + #(keys < mine) + #(equal keys
// before me), by wave shuffles; group = equal keys. Grid-stride over the list (count on the
// device).
__global__ __launch_bounds__(256) void k_dtiny(RoundArgs a, const uint2 *__restrict__ tiny)
{
    const uint32_t ntiny = a.cnt->tiny;
    const uint32_t l = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t i0 = wave * 64; i0 < ntiny; i0 += nwaves * 64) {  // wave-uniform
        const uint2 sgl = i0 + l < ntiny ? tiny[i0 + l] : make_uint2(0, 0);
        const uint32_t incl = wave_incl_sum(sgl.y), st = incl - sgl.y;
        const uint32_t total = __shfl(incl, 63, 64);
        for (uint32_t base = 0; base < total;) {  // wave-uniform rounds
            const bool in = sgl.y > 0 && st >= base && incl <= base + 64;
            const uint64_t inm = __ballot(in), afterm = __ballot(sgl.y > 0 && st >= base && incl > base + 64);
            const uint32_t s0 = (uint32_t)__ffsll((unsigned long long)inm) - 1;
            const uint32_t nbase = afterm ? (uint32_t)__shfl((int)st, __ffsll((unsigned long long)afterm) - 1, 64) : total;
            uint64_t B = in ? 1ull << (st - base) : 0ull;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) B |= __shfl_xor(B, off, 64);
            const bool live = l < nbase - base;
            const uint64_t below = l == 63 ? B : B & ((2ull << l) - 1);
            const uint32_t pos = live ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
            const uint32_t sl = s0 + (uint32_t)__builtin_popcountll(B & ((1ull << pos) - 1));
            const uint32_t gstart = __shfl((int)sgl.x, (int)sl, 64), slen = __shfl((int)sgl.y, (int)sl, 64);
            const uint32_t len = slen * (uint32_t)live;
            const uint32_t idx = l - pos;
            uint32_t p = 0, boff = 0, n = 1, key = 0xffffffffu;
            if (live) {
                const uint32_t b = find_block(a.boffs, a.nb, gstart);
                boff = a.boffs[b];
                n = a.boffs[b + 1] - boff;
                p = a.sa[gstart + idx];
                key = round_key(a, boff, n, p);
            }
            uint32_t mx = len;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
            uint32_t lt = 0, eqb = 0, eqt = 0;
            for (uint32_t j = 0; j < mx; ++j) {  // every lane takes part in the shuffles
                const uint32_t kj = __shfl(key, (int)min(pos + j, 63u), 64);
                const bool m = j < len;
                lt += m && kj < key;
                eqt += m && kj == key;
                eqb += m && kj == key && j < idx;
            }
            if (live) {
                const uint32_t slot = gstart + lt + eqb;
                a.sa[slot] = p;
                finish(a, boff, n, p, slot, gstart - boff + lt, eqt, eqb == 0);
            }
            base = nbase;
        }
    }
}

// One workgroup per segment of 129..4096 elements: LSD radix sort (4-bit digits, constant
// digits skipped) in LDS, then equal-key groups via block max / suffix-min scans.
constexpr int kMedNT = 512, kMedIPT = kMedMax / kMedNT;

__device__ __forceinline__ void medium_one(const RoundArgs &a, const uint2 sg, uint32_t (&s_k)[2][kMedMax],
                                           uint32_t (&s_v)[2][kMedMax], uint16_t (&s_cnt)[16 * kMedNT],
                                           uint32_t (&s_tmp)[kMedNT / 64 + 1], uint32_t &s_or, uint32_t &s_and);
__global__ __launch_bounds__(kMedNT) void k_medium(RoundArgs a, const uint2 *__restrict__ med)
{
    __shared__ uint32_t s_k[2][kMedMax], s_v[2][kMedMax];
    __shared__ uint16_t s_cnt[16 * kMedNT];
    __shared__ uint32_t s_tmp[kMedNT / 64 + 1];
    __shared__ uint32_t s_or, s_and;
    const uint32_t nmed = a.cnt->med;
    for (uint32_t it = blockIdx.x; it < nmed; it += gridDim.x) {
        medium_one(a, med[it], s_k, s_v, s_cnt, s_tmp, s_or, s_and);
        __syncthreads();
    }
}

__device__ __forceinline__ void medium_one(const RoundArgs &a, const uint2 sg, uint32_t (&s_k)[2][kMedMax],
                                           uint32_t (&s_v)[2][kMedMax], uint16_t (&s_cnt)[16 * kMedNT],
                                           uint32_t (&s_tmp)[kMedNT / 64 + 1], uint32_t &s_or, uint32_t &s_and)
{
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
            if (idx < m) s_cnt[((s_k[cur][idx] >> sh) & 15u) * kMedNT + tid]++;
        }
        __syncthreads();
        uint32_t loc[16], s = 0;
        for (int i = 0; i < 16; ++i) {
            loc[i] = s_cnt[tid * 16 + i];
            s += loc[i];
        }
        uint32_t ex = block_excl_sum1<kMedNT>(s, s_tmp);
        for (int i = 0; i < 16; ++i) {
            s_cnt[tid * 16 + i] = (uint16_t)ex;
            ex += loc[i];
        }
        __syncthreads();
        for (int i = 0; i < kMedIPT; ++i) {
            const uint32_t idx = tid * kMedIPT + i;
            if (idx < m) {
                const uint32_t k = s_k[cur][idx];
                const uint32_t pos = s_cnt[((k >> sh) & 15u) * kMedNT + tid]++;
                s_k[cur ^ 1][pos] = k;
                s_v[cur ^ 1][pos] = s_v[cur][idx];
            }
        }
        __syncthreads();
        cur ^= 1;
    }
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
        finish(a, boff, n, p, sg.x + e, sg.x - boff + gs, gz, e == gs);
        if (e == gs) nxt = e;
    }
}

// Large segments of the doubling phase: global MSD passes on the 32-bit rank key, 8 bits per
// pass, grid-stride over tiles / segments whose counts k_tiles left on the device.
__global__ __launch_bounds__(256) void k_lhist(RoundArgs a, const LSeg *__restrict__ lsegs,
                                               const LTile *__restrict__ tiles, uint32_t *__restrict__ key,
                                               uint32_t *__restrict__ thist)
{
    __shared__ uint32_t h[256];
    const uint32_t ntl = a.cnt->ltiles;
    for (uint32_t tb = blockIdx.x; tb < ntl; tb += gridDim.x) {
        const LTile t = tiles[tb];
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
        thist[(size_t)tb * 256 + threadIdx.x] = h[threadIdx.x];
        __syncthreads();
    }
}

__device__ __forceinline__ void push_sub(uint32_t gstart, uint32_t len, uint32_t shift, uint2 *tiny, uint2 *med,
                                         LSeg *large_next, uint32_t *large_next_cnt, uint2 *groups, Counters *cnt)
{
    if (len == 1) {
        groups[wave_append(&cnt->groups)] = make_uint2(gstart, len);
    } else if (len <= kTinyMax) {
        tiny[wave_append(&cnt->tiny)] = make_uint2(gstart, len);
    } else if (len <= kMedMax) {
        med[wave_append(&cnt->med)] = make_uint2(gstart, len);
    } else if (shift > 0) {
        LSeg l;
        l.gstart = gstart;
        l.len = len;
        l.shift = shift - 8;
        l.gathered = 1;
        large_next[wave_append(large_next_cnt)] = l;
    } else {
        groups[wave_append(&cnt->groups)] = make_uint2(gstart, len);  // keys exhausted: equal
    }
}

__global__ __launch_bounds__(256) void k_lscan(const LSeg *__restrict__ lsegs, const uint32_t *__restrict__ nseg_p,
                                               const uint2 *__restrict__ segtiles, uint32_t *__restrict__ thist,
                                               uint32_t *__restrict__ nomove, uint2 *tiny, uint2 *med, LSeg *large_next,
                                               uint32_t *large_next_cnt, uint2 *groups, Counters *cnt)
{
    __shared__ uint32_t s_tmp[8];
    const uint32_t nseg = *nseg_p;
    const uint32_t d = threadIdx.x;
    for (uint32_t sgi = blockIdx.x; sgi < nseg; sgi += gridDim.x) {
        const LSeg s = lsegs[sgi];
        const uint2 tr = segtiles[sgi];
        uint32_t run = 0;
        for (uint32_t t = tr.x; t < tr.x + tr.y; ++t) {
            const uint32_t v = thist[(size_t)t * 256 + d];
            thist[(size_t)t * 256 + d] = run;
            run += v;
        }
        const uint32_t tot = run;
        const int nz = __syncthreads_count(tot > 0);
        const uint32_t base = block_excl_sum<256>(tot, s_tmp, nullptr);
        for (uint32_t t = tr.x; t < tr.x + tr.y; ++t) thist[(size_t)t * 256 + d] += s.gstart + base;
        if (nz == 1) {
            if (d == 0) {
                nomove[sgi] = 1;
                push_sub(s.gstart, s.len, s.shift, tiny, med, large_next, large_next_cnt, groups, cnt);
            }
        } else {
            if (d == 0) nomove[sgi] = 0;
            if (tot > 0) push_sub(s.gstart + base, tot, s.shift, tiny, med, large_next, large_next_cnt, groups, cnt);
        }
    }
}

__global__ __launch_bounds__(256) void k_lscatter(const LSeg *__restrict__ lsegs, const LTile *__restrict__ tiles,
                                                  const uint32_t *__restrict__ ntl_p, const uint32_t *__restrict__ nomove,
                                                  const uint32_t *__restrict__ thist, const uint32_t *__restrict__ sa,
                                                  const uint32_t *__restrict__ key, uint32_t *__restrict__ sa2,
                                                  uint32_t *__restrict__ key2)
{
    __shared__ uint32_t cur[256];
    const uint32_t ntl = *ntl_p;
    for (uint32_t tb = blockIdx.x; tb < ntl; tb += gridDim.x) {
        const LTile t = tiles[tb];
        if (nomove[t.seg]) continue;  // workgroup-uniform
        const uint32_t shift = lsegs[t.seg].shift;
        cur[threadIdx.x] = thist[(size_t)tb * 256 + threadIdx.x];
        __syncthreads();
        for (uint32_t e = threadIdx.x; e < t.len; e += 256) {
            const uint32_t j = t.start + e;
            const uint32_t k = key[j];
            const uint32_t slot = atomicAdd(&cur[(k >> shift) & 255u], 1u);
            sa2[slot] = sa[j];
            key2[slot] = k;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_lcopy(const LTile *__restrict__ tiles, const uint32_t *__restrict__ ntl_p,
                                               const uint32_t *__restrict__ nomove, uint32_t *__restrict__ sa,
                                               uint32_t *__restrict__ key, const uint32_t *__restrict__ sa2,
                                               const uint32_t *__restrict__ key2)
{
    const uint32_t ntl = *ntl_p;
    for (uint32_t tb = blockIdx.x; tb < ntl; tb += gridDim.x) {
        const LTile t = tiles[tb];
        if (nomove[t.seg]) continue;
        for (uint32_t e = threadIdx.x; e < t.len; e += 256) {
            const uint32_t j = t.start + e;
            sa[j] = sa2[j];
            key[j] = key2[j];
        }
    }
}

// Groups produced by the large path (singletons, or key-exhausted equal-key groups). One wave
// per group; groups longer than kCoopGroup go to `coop` for k_groups_coop (the whole grid).
__global__ __launch_bounds__(256) void k_groups(RoundArgs a, const uint2 *__restrict__ groups, uint32_t *__restrict__ coop)
{
    const uint32_t ng = a.cnt->groups;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const uint32_t l = threadIdx.x & 63u;
    for (uint32_t g = wave; g < ng; g += nwaves) {
        const uint2 s = groups[g];
        if (s.y > kCoopGroup) {
            if (l == 0) coop[atomicAdd(&a.cnt->coop_groups, 1u)] = g;
            continue;
        }
        const uint32_t b = find_block(a.boffs, a.nb, s.x);
        const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
        for (uint32_t e = l; e < s.y; e += 64)
            finish(a, boff, n, a.sa[s.x + e], s.x + e, s.x - boff, s.y, e == 0);
    }
}

__global__ __launch_bounds__(256) void k_groups_coop(RoundArgs a, const uint2 *__restrict__ groups,
                                                     const uint32_t *__restrict__ coop)
{
    const uint32_t nc = a.cnt->coop_groups;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    for (uint32_t i = 0; i < nc; ++i) {
        const uint2 s = groups[coop[i]];
        const uint32_t b = find_block(a.boffs, a.nb, s.x);
        const uint32_t boff = a.boffs[b], n = a.boffs[b + 1] - boff;
        for (uint32_t e = tid; e < s.y; e += nt) finish(a, boff, n, a.sa[s.x + e], s.x + e, s.x - boff, s.y, e == 0);
    }
}

__global__ void k_commit(const uint32_t *__restrict__ list, const uint32_t *__restrict__ cnt_p,
                         const uint32_t *__restrict__ src, uint32_t *__restrict__ dst)
{
    const uint32_t cnt = *cnt_p;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x)
        dst[list[i]] = src[list[i]];
}

// End of a doubling round (or of the group fill): the per-round counters zeroed for the next
// one in one launch (class counts before k_classify rebuilds them; `zero_next` = the segment
// count the next round appends to, i.e. the one this round read).
__global__ void k_dbl_reset(Counters *cnt, uint32_t *zero_next)
{
    if (threadIdx.x == 0) {
        cnt->tiny = cnt->med = cnt->large = 0;
        cnt->large_next = cnt->groups = cnt->tiles = cnt->resolved = 0;
        cnt->coop_groups = 0;
        *zero_next = 0;
    }
}

// Start of the data phase in one launch: primaries unset, block flags and counters zero.
__global__ void k_phase_init(uint32_t *prim, uint32_t *bflag, uint32_t nb, uint32_t *cnt, uint32_t ncnt)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) {
        prim[i] = 0xffffffffu;
        bflag[i] = 0;
    }
    if (i < ncnt) cnt[i] = 0;
}



// Host-side tiling of a segment list into <= kDTile pieces.
template <class S, class T>
void build_tiles(const std::vector<S> &segs, uint32_t tile, std::vector<T> &tiles, std::vector<uint2> &segtiles,
                 uint32_t (*gstart)(const S &), uint32_t (*len)(const S &))
{
    tiles.clear();
    segtiles.resize(segs.size());
    for (uint32_t s = 0; s < segs.size(); ++s) {
        segtiles[s].x = (uint32_t)tiles.size();
        for (uint32_t o = 0; o < len(segs[s]); o += tile) {
            T t;
            t.seg = s;
            t.start = gstart(segs[s]) + o;
            t.len = std::min<uint32_t>(tile, len(segs[s]) - o);
            t.pad = 0;
            tiles.push_back(t);
        }
        segtiles[s].y = (uint32_t)tiles.size() - segtiles[s].x;
    }
}

}  // namespace

constexpr uint32_t kSpecRows = 4;  // speculative tiny round: 4 * 4 * kTinyEpwShort = 256 entries per XCD lane

bool bwt_spec_ok(const Ctx *c)
{
    const Counters *h = (const Counters *)c->spec_cnt;
    if (h->lgroups || h->flagged) return false;
    for (uint32_t x = 0; x < 8; ++x) {
        if (h->lc[0][kListTiny][x] > kSpecRows * 4 * kTinyEpwShort) return false;
        if (h->lc[0][kListFin][x] | h->lc[0][kListFinb][x] | h->lc[0][kListBig][x]) return false;
        for (uint32_t cl = 0; cl < 4; ++cl)
            if (h->lc[1][cl][x]) return false;
    }
    return true;
}

void bwt_batch_core(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_L, uint64_t *h_primary,
                    bool prologue_only)
{
    const uint32_t nb = bt.nblocks;
    const uint64_t N = bt.total;
    const uint32_t big_cap = N > kBigCapLargeBatch ? kBigCapLarge : kBigCapSmall;
    if (N >= 0xffffffffull) fail(BMH_ERANGE, "bwt: batch must be < 4 GiB");
    WallPhase wall_data(c, "bwt_data");
    // the prologue (k_phase_init .. k_g1_scan) may have been queued already (dense_batch)
    const uint64_t psig = layout_sig(6, bt.offs, (uintptr_t)d_in);
    bool pre_done = !prologue_only && c->pre_sig == psig;
    c->pre_sig = 0;

    // ---- global-pass chunks, dealt into 8 XCD lanes (blocks b = lane mod 8); the table is
    // rebuilt and uploaded only when the batch layout changed since this context's last batch
    // (the table depends on the input only through its 16-byte misalignment)
    const uint64_t sig = layout_sig(1, bt.offs, (uintptr_t)d_in & 15u);
    // deferral lists cut by XCD lane (block b -> lane b & 7): each lane's sub-list holds at most
    // (its bytes / the class's shortest entry) + 2 entries; hloff[c * 9 + x] = its first entry
    uint32_t hloff[4 * 9];
    size_t ccap[4];
    {
        uint64_t lane_bytes[8] = {};
        for (uint32_t b = 0; b < nb; ++b) lane_bytes[b & 7] += bt.offs[b + 1] - bt.offs[b];
        const uint64_t cmin[4] = {2, kTinyFin + 1, kFinCap + 1, (uint64_t)big_cap + 1};
        for (uint32_t cl = 0; cl < 4; ++cl) {
            uint64_t off = 0;
            for (uint32_t x = 0; x < 8; ++x) {
                hloff[cl * 9 + x] = (uint32_t)off;
                off += lane_bytes[x] / cmin[cl] + 2;
            }
            hloff[cl * 9 + 8] = (uint32_t)off;
            ccap[cl] = off;
        }
    }
    uint32_t nchunks;
    uint8_t *d_tab;
    if (c->ws_tag[WS_BLOCKS] == sig) {
        nchunks = c->ws_aux[WS_BLOCKS][0];
        d_tab = (uint8_t *)c->ws[WS_BLOCKS];
    } else {
        std::vector<uint32_t> hoffs(nb + 1);
        for (uint32_t b = 0; b <= nb; ++b) hoffs[b] = (uint32_t)bt.offs[b];
        std::vector<std::vector<GChunk>> lane(8);
        for (uint32_t b = 0; b < nb; ++b) {
            // the first chunk takes the unaligned prefix so the others start on 16-byte addresses
            const uint32_t n = hoffs[b + 1] - hoffs[b];
            const uint32_t mis = (uint32_t)(((uintptr_t)d_in + hoffs[b]) & 15u);
            uint32_t s = 0, l = std::min(n, kG1Chunk - mis);
            while (s < n) {
                lane[b & 7].push_back(GChunk{b, s, l, hoffs[b], n, 0, 0, 0});
                s += l;
                l = std::min(n - s, kG1Chunk);
            }
        }
        size_t lmax = 0;
        for (auto &l : lane) lmax = std::max(lmax, l.size());
        std::vector<GChunk> chunks(lmax * 8, GChunk{0, 0, 0, 0, 0, 0, 0, 0});
        std::vector<uint32_t> bchunks(nb, 0), bchunk0(nb, 0);
        for (uint32_t x = 0; x < 8; ++x)
            for (size_t k = 0; k < lane[x].size(); ++k) {
                const GChunk &g = lane[x][k];
                chunks[k * 8 + x] = g;
                if (bchunks[g.block]++ == 0) bchunk0[g.block] = (uint32_t)(k * 8 + x);
            }
        nchunks = (uint32_t)chunks.size();
        const size_t tab_bytes = (nb + 1) * 4 + nb * 8 + nchunks * sizeof(GChunk) + sizeof(hloff);
        d_tab = (uint8_t *)c->get(WS_BLOCKS, tab_bytes + 64);
        std::vector<uint8_t> h(tab_bytes);
        size_t o = 0;
        memcpy(&h[o], hoffs.data(), (nb + 1) * 4);
        o += (nb + 1) * 4;
        memcpy(&h[o], bchunks.data(), nb * 4);
        o += nb * 4;
        memcpy(&h[o], bchunk0.data(), nb * 4);
        o += nb * 4;
        memcpy(&h[o], chunks.data(), nchunks * sizeof(GChunk));
        o += nchunks * sizeof(GChunk);
        memcpy(&h[o], hloff, sizeof(hloff));
        c->h2d(d_tab, h.data(), tab_bytes);
        c->ws_tag[WS_BLOCKS] = sig;
        c->ws_aux[WS_BLOCKS][0] = nchunks;
    }
    const uint32_t *d_boffs = (const uint32_t *)d_tab;
    const uint32_t *d_bchunks = d_boffs + (nb + 1);
    const uint32_t *d_bchunk0 = d_bchunks + nb;
    const GChunk *d_chunks = (const GChunk *)(d_bchunk0 + nb);
    const uint32_t *d_loff = (const uint32_t *)(d_chunks + nchunks);

    uint32_t *sa = (uint32_t *)c->get(WS_SA, N * 4);
    uint32_t *sa2 = (uint32_t *)c->get(WS_SA2, N * 4);
    uint64_t *rec = (uint64_t *)c->get(WS_KEY8, N * 8);
    // chunk write offsets (u32, the scatter's) | chunk digit counts (u16)
    uint32_t *chist = (uint32_t *)c->get(WS_CHIST, (size_t)nchunks * kG1Bins * 6);
    uint16_t *ccnt = (uint16_t *)(chist + (size_t)nchunks * kG1Bins);
    // per-chunk byte sets (8 words a chunk) | per-block alphabet info | rank maps
    // | recount list length + chunk list
    uint8_t *d_alpha = (uint8_t *)c->get(WS_ALPHA, (size_t)nchunks * 36 + (size_t)nb * (4 + 256) + 64);
    uint32_t *abits = (uint32_t *)d_alpha, *ainfo = abits + 8 * (size_t)nchunks;
    uint8_t *arank = (uint8_t *)(ainfo + nb);
    uint32_t *rlist = (uint32_t *)(arank + (size_t)nb * 256) + 1;
    uint2 *bk = (uint2 *)c->get(WS_BSTART, (size_t)nb * kG1Bins * 8);
    uint32_t *g1part = (uint32_t *)c->get(WS_SCAN_PART, (size_t)nb * kG1ScanParts * kG1Bins * 4);
    const size_t seg_cap = N / 2 + 2;
    // every list entry covers >= 2 positions, so N / 2 entries bound every list; the finish
    // lists by size class and XCD lane (ccap, hloff above)
    Seg4 *const fint_a = (Seg4 *)c->get(WS_FINT_CUR, ccap[kListTiny] * 16);
    Seg4 *const fint_b = (Seg4 *)c->get(WS_FINT_NXT, ccap[kListTiny] * 16);
    Seg4 *const fin_a = (Seg4 *)c->get(WS_FIN_CUR, ccap[kListFin] * 16);
    Seg4 *const fin_b = (Seg4 *)c->get(WS_FIN_NXT, ccap[kListFin] * 16);
    Seg4 *const finb_a = (Seg4 *)c->get(WS_FINB_CUR, ccap[kListFinb] * 16);
    Seg4 *const finb_b = (Seg4 *)c->get(WS_FINB_NXT, ccap[kListFinb] * 16);
    Seg4 *dgroups = (Seg4 *)c->get(WS_GROUPS, seg_cap * 16);
    Seg4 *const big = (Seg4 *)c->get(WS_LARGE, ccap[kListBig] * 16);
    Seg4 *const big2 = (Seg4 *)c->get(WS_LARGE2, ccap[kListBig] * 16);
    uint32_t *bflag = (uint32_t *)c->get(WS_OFFS, nb * 4 + 64);
    uint32_t *d_prim = (uint32_t *)c->get(WS_PRIMARY, nb * 4 + 64);
    Counters *d_cnt = (Counters *)c->get(WS_COUNTERS, sizeof(Counters) + 64);
    Counters *h_cnt = (Counters *)c->host_pinned(sizeof(Counters) + 4096);
    auto read_counters = [&]() {
        c->d2h(h_cnt, d_cnt, sizeof(Counters));
        c->sync();
    };

    DataArgs da;
    da.data = d_in;
    da.boffs = d_boffs;
    da.nb = nb;
    da.sa = sa;
    da.L = d_L;
    da.prim = d_prim;
    da.bflag = bflag;
    da.cnt = d_cnt;
    da.ainfo = ainfo;
    da.arank = arank;
    // list buffers of the two parities: parity 0 holds what the global pass and the dense finish
    // defer (round 1's input); round r reads parity (r - 1) & 1 and appends to parity r & 1
    Seg4 *const lt[2] = {fint_a, fint_b}, *const lf[2] = {fin_a, fin_b}, *const lb[2] = {finb_a, finb_b};
    Seg4 *const lg[2] = {big, big2};
    auto set_out = [&](uint32_t par) {
        da.lists[kListTiny] = lt[par];
        da.lists[kListFin] = lf[par];
        da.lists[kListFinb] = lb[par];
        da.lists[kListBig] = lg[par];
        da.lists[kListGroups] = dgroups;
        da.lcnt = &d_cnt->lc[par][0][0];
        da.loff = d_loff;
    };
    // data-phase MSD tiles (built on the device, k_tiles): the big list's slots over kDTile plus
    // one partial tile per segment
    const size_t bcap = ccap[kListBig], dtcap = N / kDTile + bcap + 2;
    const bool dbg_lists = c->opt.check_lists != 0;  // BMH_OPT_CHECK_LISTS
    // bitonic list classes merged into two launches per round for latency-bound batches
    const bool merge_sort_classes = N <= kMergeSortBatch;

    // SA-lite (default): the finish passes store SA only where a later pass reads it. If some
    // block then needs rank doubling (which reads every slot's SA), the data phase is re-run
    // with every SA entry stored, and the context keeps that mode while its batches need it.
    // Small (latency-bound) batches store every SA entry from the start: the stores cost a few
    // microseconds, a re-run of the data phase (when a block turns out to need rank doubling,
    // e.g. Calgary's pic on a fresh context) costs milliseconds.
    bool full_sa = c->bwt_full_sa || N <= kFullSaBatch;
    uint64_t *kb_cur = rec, *kb_nxt = nullptr;  // MSD window buffers (see the big-list passes)
    for (;;) {
        da.full_sa = full_sa ? 1u : 0u;
        da.big_cap = big_cap;
        da.dbl_bits = N <= kFullSaBatch ? kDblBitsSmall : kDblBitsLarge;
        if (kb_cur != rec) std::swap(kb_cur, kb_nxt);  // the global pass writes its windows into rec
        static_assert(sizeof(Counters) % 4 == 0, "counter words");
        constexpr uint32_t kCntWords = sizeof(Counters) / 4;
        if (!pre_done) {
            BMH_LAUNCH(c, "bwt_fill", k_phase_init, cdiv(std::max(nb, kCntWords), 256), 256, 0, d_prim, bflag, nb,
                       (uint32_t *)d_cnt, kCntWords);

            // ---- data phase
            // raw digits + each block's byte census, the blocks' alphabets, then the chunks of
            // compacted blocks recounted
            BMH_LAUNCH(c, "bwt_g1_hist", k_g1_hist, nchunks, kG1HistNT, 0, d_in, d_boffs, d_chunks, rlist, ccnt, ainfo,
                       arank, abits, 0u);
            BMH_LAUNCH(c, "bwt_g1_census", k_g1_census_fin, nb, 256, 0, abits, d_bchunks, d_bchunk0, ainfo, arank,
                       rlist);
            BMH_LAUNCH(c, "bwt_g1_hist2", k_g1_hist, std::min<uint32_t>(nchunks, 2048), kG1HistNT, 0, d_in, d_boffs,
                       d_chunks, rlist, ccnt, ainfo, arank, abits, 1u);
            BMH_LAUNCH(c, "bwt_g1_scan", k_g1_scan_sum, dim3(nb, kG1ScanParts), kG1Bins, 0, d_bchunks, d_bchunk0, ccnt,
                       g1part);
            BMH_LAUNCH(c, "bwt_g1_scan", k_g1_scan, nb, kG1Bins, 0, d_boffs, g1part, bk, lb[0], lg[0], d_cnt, d_loff,
                       big_cap, ainfo);
            BMH_LAUNCH(c, "bwt_g1_scan", k_g1_scan_offs, dim3(nb, kG1ScanParts), kG1Bins, 0, d_bchunks, d_bchunk0, ccnt,
                       chist, g1part);
        }
        pre_done = false;
        if (prologue_only) {
            c->pre_sig = psig;
            return;
        }
        set_out(0);
        BMH_LAUNCH(c, "bwt_g1_scatter", k_g1_scatter, nchunks, 1024, 0, da, d_chunks, chist, bk, rec);
        // the dense finish appends deferred segments after the global pass's list entries
        BMH_LAUNCH(c, "bwt_finish_dense", (k_finish_dense<kDenseNT, kDenseCap>), 8u * cdiv(nb, 8) * kG1Bins, kDenseNT, 0,
                   da, bk, rec);
#if defined(BMH_PROF_SCATTER) || defined(BMH_PROF_DENSE)
        {
            std::vector<uint32_t> h((1u << 18) * 8);
            BMH_HIP(hipStreamSynchronize(c->stream));
            BMH_HIP(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_dprof), h.size() * 4));
            unsigned long long sum[8] = {}, cnt = 0;
            for (size_t w = 0; w < (1u << 18); ++w) {
                if (!h[w * 8 + 7]) continue;
                ++cnt;
                for (int i = 0; i < 8; ++i) sum[i] += h[w * 8 + i];
            }
            fprintf(stderr, "phases (mean s_memtime ticks per workgroup, %llu workgroups):", cnt);
            for (int i = 0; i < 8; ++i) fprintf(stderr, " %.0f", cnt ? (double)sum[i] / cnt : 0.0);
            fprintf(stderr, "\n");
        }
#endif
        if (c->spec_lists && !full_sa && !dbg_lists && !h_primary) {
            // speculative round (Ctx::spec_lists): on random-like data the global pass and the
            // dense finish leave only a few tied pairs, all in the tiny list, which one round
            // resolves. That round runs on a fixed grid (kSpecRows rows of 4 * kTinyEpwShort
            // entries per XCD lane, identity lane map) without the host wait for the counters;
            // the counters are read back at the encode's final sync and bwt_spec_ok checks that
            // nothing was past the grid, in another list class, deferred again or sent to rank
            // doubling. Saves two host round trips (≈ 70 µs of idle GPU on a 128 MiB batch).
            set_out(1);  // (lc[1] zeroed by k_phase_init: the data phase appends to parity 0 only)
            LaneMap lm;
            for (uint32_t v = 0; v < 8; ++v) {
                lm.lane[v] = (uint8_t)v;
                lm.r[v] = 0;
                lm.rep[v] = 1;
            }
            BMH_LAUNCH(c, "bwt_finish_tiny", k_finish_tiny, 8u * kSpecRows, 256, 0, da, lt[0], d_loff + kListTiny * 9,
                       &d_cnt->lc[0][kListTiny][0], lm, kTinyEpwShort);
            static_assert(sizeof(Counters) <= sizeof(c->spec_cnt), "spec counters");
            c->d2h(c->spec_cnt, d_cnt, sizeof(Counters));
            c->spec_pending = true;
            return;
        }
        // List rounds: every kernel of a round reads its list lengths from the device counters
        // and strides over them with a fixed grid, and the MSD tiles are built on the device, so
        // the host waits once per round (for the loop condition).
        read_counters();
        int round = 0;
        for (uint32_t in = 0;; in ^= 1u) {
            // per class: entries over all lanes
            uint32_t tot[4] = {};
            for (uint32_t cl = 0; cl < 4; ++cl)
                for (uint32_t x = 0; x < 8; ++x) tot[cl] += h_cnt->lc[in][cl][x];
            if (!(tot[kListTiny] | tot[kListFin] | tot[kListFinb] | tot[kListBig])) break;
            if (dbg_lists) {  // per-round list census (diagnostics only)
                auto census = [&](const char *name, const Seg4 *d, uint32_t cl) {
                    uint64_t segs = 0, tsum = 0, mxl = 0, dmin = ~0ull, dmax = 0, lg2[33] = {};
                    for (uint32_t x = 0; x < 8; ++x) {
                        const uint32_t cnt = h_cnt->lc[in][cl][x];
                        std::vector<Seg4> h(cnt);
                        c->d2h(h.data(), d + hloff[cl * 9 + x], cnt * sizeof(Seg4));
                        c->sync();
                        for (auto &e : h) {
                            tsum += e.y;
                            lg2[e.y > 1 ? 32 - __builtin_clz(e.y - 1) : 0] += e.y;
                            mxl = std::max<uint64_t>(mxl, e.y);
                            dmin = std::min<uint64_t>(dmin, e.z);
                            dmax = std::max<uint64_t>(dmax, e.z);
                        }
                        segs += cnt;
                    }
                    fprintf(stderr, "round %d %-5s segs %llu elems %llu max %llu depth %llu..%llu\n", round, name,
                            (unsigned long long)segs, (unsigned long long)tsum, (unsigned long long)mxl,
                            (unsigned long long)(segs ? dmin : 0), (unsigned long long)dmax);
                    if (tsum) {  // elements by segment length <= 2^k
                        fprintf(stderr, "   ");
                        for (int k = 0; k < 33; ++k)
                            if (lg2[k]) fprintf(stderr, " 2^%d:%llu", k, (unsigned long long)lg2[k]);
                        fprintf(stderr, "\n");
                    }
                };
                census("tiny", lt[in], kListTiny);
                census("fin", lf[in], kListFin);
                census("finb", lb[in], kListFinb);
                census("big", lg[in], kListBig);
            }
            // workgroup lanes dealt over the non-empty sub-lists of each class; rows[cl] = the
            // grid's rows (grid = 8 x rows) so every entry of the fullest sub-list has a workgroup
            LaneMap lm[4];
            uint32_t rows[4] = {};
            for (uint32_t cl = 0; cl < 4; ++cl) {
                uint32_t used[8], nu = 0;
                for (uint32_t x = 0; x < 8; ++x)
                    if (h_cnt->lc[in][cl][x]) used[nu++] = x;
                if (!nu) used[nu++] = 0;
                for (uint32_t v = 0; v < 8; ++v) {
                    const uint32_t k = v % nu;
                    lm[cl].lane[v] = (uint8_t)used[k];
                    lm[cl].r[v] = (uint8_t)(v / nu);
                    lm[cl].rep[v] = (uint8_t)((8 - k + nu - 1) / nu);
                }
                for (uint32_t v = 0; v < 8; ++v)
                    rows[cl] = std::max(rows[cl], cdiv(h_cnt->lc[in][cl][lm[cl].lane[v]], lm[cl].rep[v]));
            }
            ++round;
            const uint32_t out = in ^ 1u;
            // the parity this round appends to (round 1's is still zero from k_phase_init)
            if (round > 1) BMH_HIP(hipMemsetAsync(&d_cnt->lc[out][0][0], 0, sizeof(d_cnt->lc[out]), c->stream));
            set_out(out);
            const uint32_t *dc = &d_cnt->lc[in][0][0];
            if (tot[kListTiny]) {
#ifndef BMH_TINY_EPW_LONG
#define BMH_TINY_EPW_LONG 32u  // (64: 2.23 -> 1.78 ms of tiny rounds on 100 MB at 1 MiB with 32; 16: 2.17)
#endif
                const uint32_t epw = tot[kListTiny] >= kTinyWideList ? BMH_TINY_EPW_LONG : kTinyEpwShort;
                BMH_LAUNCH(c, "bwt_finish_tiny", k_finish_tiny, 8u * cdiv(rows[kListTiny], 4 * epw), 256, 0, da, lt[in],
                           d_loff + kListTiny * 9, dc + kListTiny * 8, lm[kListTiny], epw);
            }
            if (tot[kListFin]) {
                // size classes: <= 128 and <= 512 one wave each (4 segments per workgroup), then 2, 4
                // and 8 waves of 8 elements a thread (every wave of a class holds slots of its
                // segments' sorting network); only the classes some segment of the round needs
                const uint32_t fm = h_cnt->lc[in][4][0];
                const uint32_t gf = 8u * rows[kListFin], gw = 8u * cdiv(rows[kListFin], 4);
                const uint32_t *lof = d_loff + kListFin * 9, *cf = dc + kListFin * 8;
                if (merge_sort_classes) {
                    // latency-bound batches: two launches per round instead of up to five (each
                    // network is sized to its segment, so the wider shapes sort the shorter
                    // segments of their range with the same stages; the launches of one stream
                    // run one after another, so fewer of them shorten the round)
                    if (fm & 3u)
                        BMH_LAUNCH(c, "bwt_finish", (k_finish_sortw<8, 4>), gw, 256, 0, da, lf[in], lof, cf, 1u,
                                   lm[kListFin]);
                    if (fm & 28u)
                        BMH_LAUNCH(c, "bwt_finish", (k_finish_sort<512, 8>), gf, 512, 0, da, lf[in], lof, cf, 512u,
                                   lm[kListFin]);
                } else {
                if (fm & 1u)
                    BMH_LAUNCH(c, "bwt_finish", (k_finish_sortw<2, 4>), gw, 256, 0, da, lf[in], lof, cf, 1u, lm[kListFin]);
                if (fm & 2u)
                    BMH_LAUNCH(c, "bwt_finish", (k_finish_sortw<8, 4>), gw, 256, 0, da, lf[in], lof, cf, 128u, lm[kListFin]);
                if (fm & 4u)
                    BMH_LAUNCH(c, "bwt_finish", (k_finish_sort<128, 8>), gf, 128, 0, da, lf[in], lof, cf, 512u,
                               lm[kListFin]);
                if (fm & 8u)
                    BMH_LAUNCH(c, "bwt_finish", (k_finish_sort<256, 8>), gf, 256, 0, da, lf[in], lof, cf, 1024u,
                               lm[kListFin]);
                if (fm & 16u)
                    BMH_LAUNCH(c, "bwt_finish", (k_finish_sort<512, 8>), gf, 512, 0, da, lf[in], lof, cf, 2048u,
                               lm[kListFin]);
                }
            }
            if (tot[kListFinb]) {  // counting-sort finish: dense shape, or 1024 threads up to kBigCapSmall
                if (big_cap > kSegCap)
                    BMH_LAUNCH(c, "bwt_finish_big", (k_finish_seg<kBigNT, kBigCapSmall>), 8u * rows[kListFinb], kBigNT, 0,
                               da, lb[in], d_loff + kListFinb * 9, dc + kListFinb * 8, kFinCap, lm[kListFinb]);
                else
                    BMH_LAUNCH(c, "bwt_finish_big", (k_finish_seg<kSegNT, kSegCap>), 8u * rows[kListFinb], kSegNT, 0,
                               da, lb[in], d_loff + kListFinb * 9, dc + kListFinb * 8, kFinCap, lm[kListFinb]);
            }
            if (tot[kListBig]) {
                uint8_t *d_dt = (uint8_t *)c->get(WS_LTILES, dtcap * sizeof(DTile) + bcap * 12 + 64);
                DTile *d_tiles = (DTile *)d_dt;
                uint2 *d_segtiles = (uint2 *)(d_dt + dtcap * sizeof(DTile));
                uint32_t *d_nomove = (uint32_t *)(d_dt + dtcap * sizeof(DTile) + bcap * 8);
                uint32_t *thist = (uint32_t *)c->get(WS_LTHIST, dtcap * kMsdBins * 4);
                uint32_t *stot = (uint32_t *)c->get(WS_LSEGS, bcap * kMsdBins * 4);
                unsigned long long *segor = (unsigned long long *)c->get(WS_SEGOR, bcap * 16 + 64);
                unsigned long long *segmin = segor + bcap;
                const uint32_t *loffb = d_loff + kListBig * 9, *cntb = dc + kListBig * 8;
                const uint32_t gt = 2048;  // tile kernels: 256 workgroups per lane, striding over its tiles
                BMH_LAUNCH(c, "bwt_dtiles", k_dtiles, 1, 1024, 0, lg[in], loffb, cntb, d_tiles, d_segtiles,
                           d_cnt->tstart, segor, segmin);
                // the global-pass records are no longer read: their buffer holds the windows
                const LaneMap &lb_ = lm[kListBig];
                // window buffers: the current pass reads kb_cur (the global pass's windows, or the
                // previous pass's scatter output) and its scatter writes the children's to kb_nxt
                if (!kb_nxt) kb_nxt = (uint64_t *)c->get(WS_KEY8B, N * 8);
                BMH_LAUNCH(c, "bwt_dcp", k_dcp, gt, 256, 0, da, lg[in], d_tiles, d_cnt->tstart, segor, segmin, kb_cur,
                           lb_);
                BMH_LAUNCH(c, "bwt_dhist", k_dhist, gt, kMsdBins, 0, da, lg[in], d_tiles, d_cnt->tstart, segor, segmin, kb_cur,
                           thist, lb_);
                BMH_LAUNCH(c, "bwt_dscan", k_dscan, 8u * std::min<uint32_t>(rows[kListBig], 512u), kMsdBins, 0, da, lg[in],
                           loffb, cntb, d_segtiles, segor, thist, stot, d_nomove, lb_);
                BMH_LAUNCH(c, "bwt_dscatter", k_dscatter, gt, kMsdBins, 0, da, lg[in], d_tiles, d_cnt->tstart, segor, segmin,
                           kb_cur, d_nomove, thist, stot, sa2, kb_nxt, lb_);
                BMH_LAUNCH(c, "bwt_dcopy", k_dcopy, gt, 256, 0, d_tiles, d_cnt->tstart, d_nomove, sa, sa2, lb_);
                std::swap(kb_cur, kb_nxt);
            }
            read_counters();
        }
        if (full_sa || h_cnt->flagged == 0) break;
        full_sa = true;
    }
    c->bwt_full_sa = h_cnt->flagged != 0;

    // ---- doubling phase, only if some block still holds tied groups
    wall_data.stop();
    WallPhase wall_dbl(c, "bwt_doubling");
    const uint32_t ngroups = h_cnt->lgroups;
    if (ngroups > 0) {
        uint32_t *rkA = (uint32_t *)c->get(WS_RKA, N * 4);
        uint32_t *rkB = (uint32_t *)c->get(WS_RKB, N * 4);
        uint32_t *key = (uint32_t *)c->get(WS_KEY, N * 4);
        uint32_t *key2 = (uint32_t *)c->get(WS_KEY2, N * 4);
        uint2 *seg_cur = (uint2 *)c->get(WS_DSEG_CUR, seg_cap * 8);
        uint2 *seg_nxt = (uint2 *)c->get(WS_DSEG_NXT, seg_cap * 8);
        uint2 *tiny = (uint2 *)c->get(WS_TINY, seg_cap * 8);
        uint2 *med = (uint2 *)c->get(WS_MED, (N / (kTinyMax + 1) + 2) * 8);
        const size_t lcap = N / (kMedMax + 1) + 2;
        LSeg *large = (LSeg *)c->get(WS_DLARGE, lcap * sizeof(LSeg));
        LSeg *large2 = (LSeg *)c->get(WS_DLARGE2, lcap * sizeof(LSeg));
        uint2 *groups = (uint2 *)c->get(WS_DGROUPS, (N + 2) * 8);
        uint32_t *resolved = (uint32_t *)c->get(WS_RESOLVED, N * 4);
        // large-path tiles, bounded by the slots over kDTile plus one partial tile per segment
        const size_t tcap = N / kDTile + lcap + 2;
        uint8_t *d_lt = (uint8_t *)c->get(WS_LTILES, tcap * sizeof(LTile) + lcap * 12 + 64);
        LTile *d_ltiles = (LTile *)d_lt;
        uint2 *d_lsegtiles = (uint2 *)(d_lt + tcap * sizeof(LTile));
        uint32_t *d_lnomove = (uint32_t *)(d_lt + tcap * sizeof(LTile) + lcap * 8);
        uint32_t *thist = (uint32_t *)c->get(WS_LTHIST, tcap * 256 * 4);
        uint32_t *gcoop = (uint32_t *)c->get(WS_COOP, (size_t)ngroups * 4 + (N / kCoopGroup + 2) * 4 + 64) + ngroups;
        // MSD passes per round: ranks are block-local (< n), the first pass takes their highest
        // nonzero byte (k_classify), 8 bits per pass
        const uint32_t npass = bt.max_n > (1u << 24) ? 4u : bt.max_n > (1u << 16) ? 3u : bt.max_n > 256u ? 2u : 1u;

        BMH_LAUNCH(c, "bwt_rank_fill", k_rank_fill, dim3(cdiv(bt.max_n, 4096), nb), 256, 0, d_boffs, bflag, sa, rkA,
                   rkB);
        BMH_HIP(hipMemsetAsync(&d_cnt->next, 0, 4, c->stream));
        BMH_HIP(hipMemsetAsync(&d_cnt->dmin_bits, 0xff, 4, c->stream));
        uint32_t *coop = (uint32_t *)c->get(WS_COOP, (size_t)ngroups * 4 + (N / kCoopGroup + 2) * 4 + 64);
        BMH_HIP(hipMemsetAsync(&d_cnt->coop_fill, 0, 4, c->stream));
        BMH_LAUNCH(c, "bwt_group_fill", k_group_fill, std::min<uint32_t>(cdiv(ngroups, 256), 65536), 256, 0, da, dgroups,
                   ngroups, rkA, rkB, seg_cur, coop, d_cnt);
        BMH_LAUNCH(c, "bwt_group_fill", k_group_fill_coop, kCoopGrid, 256, 0, da, dgroups, coop, rkA, rkB, seg_cur, d_cnt);
        // each round's segments are classified at the end of the round before (here: of the
        // fill), so the one host wait per round also says which segment classes the next one
        // holds and the launches of empty classes are skipped (each costs a few microseconds of
        // a latency-bound round: up to 5 per MSD pass)
        // round r reads the segment count of counter in(r) and appends to out(r): next / next2
        // alternate (the fill wrote next), so the reset at the end of a round zeroes the count
        // it read and nothing is zeroed at the start of the next
        const uint32_t cgrid = std::min<uint32_t>(cdiv(seg_cap, 256), 256);
        auto cnt_of = [&](int r) { return (r & 1) ? &d_cnt->next2 : &d_cnt->next; };  // in(r); out(r) = in(r + 1)
        auto classify = [&](const uint2 *segs, int r, uint32_t *zero_next) {  // segs: round r's input
            BMH_LAUNCH(c, "bwt_classify", k_dbl_reset, 1, 64, 0, d_cnt, zero_next);
            BMH_LAUNCH(c, "bwt_classify", k_classify, cgrid, 256, 0, segs, cnt_of(r), tiny, med, large, d_cnt, d_boffs,
                       nb);
        };
        classify(seg_cur, 0, cnt_of(1));
        read_counters();
        const uint32_t ncur0 = h_cnt->next;
        const uint64_t D0 = h_cnt->dmin_bits / 8;  // every tied group shares at least D bytes
        if (ncur0 > 0 && D0 == 0) fail(BMH_EHIP, "bwt: internal error (zero doubling depth)");
        // Every kernel of a round reads its list lengths from the device counters and strides
        // over them with a fixed grid; the large path's tiles are built on the device (k_tiles).
        // The host reads each round's counters one round late: round r + 1 is queued before the
        // wait for round r's, so the GPU never idles on the wait; the one round queued past the
        // last finds no segments and leaves everything as it was. A round launched before its
        // counters are known runs the tiny and medium kernels (empty lists exit at once) and the
        // large passes if the round before it had large segments (groups only split, so a
        // large segment's parent was large).
        if (!c->dbl_cnt_host) BMH_HIP(hipHostMalloc(&c->dbl_cnt_host, 2 * sizeof(Counters), hipHostMallocDefault));
        for (auto &e : c->dbl_ev)
            if (!e) BMH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        Counters *hc = (Counters *)c->dbl_cnt_host;
        uint2 *seg_in[2] = {seg_cur, seg_nxt};
        auto launch_round = [&](int round, uint64_t D, bool has_large, bool run_tiny, bool run_med) {
            uint2 *seg_out = seg_in[(round + 1) & 1];
            RoundArgs a;
            a.data = d_in;
            a.boffs = d_boffs;
            a.nb = nb;
            a.sa = sa;
            a.L = d_L;
            a.prim = d_prim;
            const bool odd = (round & 1) != 0;
            a.rk_cur = odd ? rkB : rkA;
            a.rk_nxt = odd ? rkA : rkB;
            a.D = (uint32_t)std::min<uint64_t>(D, 0xffffffffull);
            a.newD = 2 * D;
            a.next = seg_out;
            a.resolved = resolved;
            a.cnt = d_cnt;
            a.next_cnt = cnt_of(round + 1);

            // (the large path also appends tiny / medium segments)
            for (uint32_t pass = 0; has_large && pass < npass; ++pass) {  // passes with no segments exit at once
                uint32_t *cnt_in = pass & 1 ? &d_cnt->large_next : &d_cnt->large;
                uint32_t *cnt_out = pass & 1 ? &d_cnt->large : &d_cnt->large_next;
                LSeg *lin = pass & 1 ? large2 : large, *lout = pass & 1 ? large : large2;
                BMH_HIP(hipMemsetAsync(cnt_out, 0, 4, c->stream));
                BMH_LAUNCH(c, "bwt_ltiles", (k_tiles<LSeg, LTile>), 1, 1024, 0, lin, cnt_in, d_ltiles, d_lsegtiles,
                           &d_cnt->ltiles, nullptr, nullptr);
                BMH_LAUNCH(c, "bwt_lhist", k_lhist, kDblGrid, 256, 0, a, lin, d_ltiles, key, thist);
                BMH_LAUNCH(c, "bwt_lscan", k_lscan, kDblGrid, 256, 0, lin, cnt_in, d_lsegtiles, thist, d_lnomove, tiny, med,
                           lout, cnt_out, groups, d_cnt);
                BMH_LAUNCH(c, "bwt_lscatter", k_lscatter, kDblGrid, 256, 0, lin, d_ltiles, &d_cnt->ltiles, d_lnomove, thist,
                           sa, key, sa2, key2);
                BMH_LAUNCH(c, "bwt_lcopy", k_lcopy, kDblGrid, 256, 0, d_ltiles, &d_cnt->ltiles, d_lnomove, sa, key, sa2,
                           key2);
            }
            if (has_large || run_tiny) BMH_LAUNCH(c, "bwt_tiny", k_dtiny, kDblGrid, 256, 0, a, tiny);
            if (has_large || run_med) BMH_LAUNCH(c, "bwt_medium", k_medium, kDblGrid, kMedNT, 0, a, med);
            BMH_LAUNCH(c, "bwt_groups", k_groups, kDblGrid, 256, 0, a, groups, gcoop);
            BMH_LAUNCH(c, "bwt_groups", k_groups_coop, kCoopGrid, 256, 0, a, groups, gcoop);
            BMH_LAUNCH(c, "bwt_commit", k_commit, kDblGrid, 256, 0, resolved, &d_cnt->resolved, a.rk_nxt,
                       (uint32_t *)a.rk_cur);
            classify(seg_out, round + 1, cnt_of(round));
            BMH_HIP(hipMemcpyAsync(hc + (round & 1), d_cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
            BMH_HIP(hipEventRecord(c->dbl_ev[round & 1], c->stream));
        };
        if (ncur0 > 0) {
            uint64_t D = D0;
            launch_round(0, D, h_cnt->large != 0, h_cnt->tiny != 0, h_cnt->med != 0);
            bool large_ub = h_cnt->large != 0;  // round r - 1's counters: a bound for round r + 1
            for (int round = 0;; ++round) {
                launch_round(round + 1, 2 * D, large_ub, true, true);
                for (;;) {  // spin: a blocking wait can sleep the host thread for milliseconds
                    const hipError_t e = hipEventQuery(c->dbl_ev[round & 1]);
                    if (e == hipSuccess) break;
                    if (e != hipErrorNotReady) BMH_HIP(e);
                    spin_pause();
                }
                const Counters &cr = hc[round & 1];
                const uint32_t ncur = (round & 1) ? cr.next : cr.next2;  // in(round + 1)
                large_ub = cr.large != 0;
                if (ncur == 0) break;  // round + 1 (queued) had nothing to do
                D *= 2;
            }
        }
    }

    // ---- primary indices
    if (!h_primary) return;  // the primaries stay on the device (WS_PRIMARY), checked there
    uint32_t *h_prim = (uint32_t *)c->host_pinned(nb * 4 + 4096);
    c->d2h(h_prim, d_prim, nb * 4);
    c->sync();
    for (uint32_t b = 0; b < nb; ++b) {
        if (h_prim[b] == 0xffffffffu) fail(BMH_EHIP, "bwt: internal error (primary index not produced)");
        h_primary[b] = h_prim[b];
    }
}

}  // namespace bmh
