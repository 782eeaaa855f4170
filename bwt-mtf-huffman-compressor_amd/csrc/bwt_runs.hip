// bwt_runs.hip — the BWT of run-heavy blocks (long runs of one byte value: bitmaps with blank
// areas such as Calgary pic, zero-padded binaries) through their run-length encoding, and the
// batch entry point that routes such blocks here and the rest to the rotation sorter (bwt.hip).
//
// Same output as the reference bwt() (main.cpp:77-91: std::stable_sort of the n cyclic rotations
// with bwt_cmp_straight, main.cpp:46-59), derived without comparing long runs byte by byte:
//
// Cut the cyclic block into maximal runs; run i starts at H[i], holds L_i copies of byte c_i and
// is followed by run i + 1, whose byte d_i != c_i. The rotation at a position p of run i with r
// run bytes left (1 <= r <= L_i) reads c_i^r, then the rotation at H[i + 1]. Two rotations with
// the same first byte c and r_p < r_q differ first at offset r_p, where p reads d_p and q reads
// c, so p < q iff d_p < c. Hence the rotation order is the order of the keys
//     ( c_i, [d_i > c_i], d_i > c_i ? -r : r, rank of the rotation at H[i + 1] )
// and the rotations at run starts (r = L_i) compare exactly like the cyclic rotations of the
// run sequence over the alphabet K_i = (c_i, [d_i > c_i], +-L_i): equal K means an equal run, so
// the comparison moves on to the next run. So:
//   1. heads   : H = positions p with T[p] != T[p - 1] (cyclic), m of them (the screen counted m);
//   2. runs    : K_i per run, sorted -> initial ranks (rank = first sorted slot of its key);
//   3. doubling: ranks of the m cyclic run-sequence rotations by prefix doubling over run
//                indices, (rank_i, rank_{i+h}) per round, until all distinct or h >= m
//                (equal ranks then mean identical rotations);
//   4. place   : each position's 57-bit key above, sorted stably by position -> the sorted
//                rotations; L[j] = T[sp[j] - 1], primary = slot of position 0. Stable order
//                keeps identical rotations in position order, as std::stable_sort does.
// A block of one byte value (m = 0) has n identical rotations: L = T, primary 0.
// Pic (513 KB, 76 K runs) takes 7 doubling rounds over 76 K runs instead of ~20 data / rank
// rounds over 440 K positions sitting in long zero runs.
//
// The screen (k_run_count) runs only on batches up to kRunScreenMax bytes: it costs a pass over
// the input and one host wait, which the large random-data batches of the headline never repay.
#include "bmh_internal.h"

#include <algorithm>
#include <exception>
#include <thread>

#include "device_util.h"

namespace bmh {

namespace {

constexpr uint64_t kRunScreenMax = 64ull << 20;  // batches screened for run-heavy blocks
constexpr uint32_t kRunMinBlock = 1u << 16;      // shorter blocks stay on the rotation sorter
constexpr uint32_t kRunMaxBlock = 1u << 24;      // run lengths fit 24 bits of the key
// The position key's low 24 bits hold a run's rank among ALL runs of a run batch (blocks are
// sorted together, run_blocks_batch), so a batch's runs M must stay below 2^24: run_blocks groups
// close before that. One screened batch can never reach it (runs <= n / kRunShare per block).
constexpr uint32_t kRunRankLimit = 1u << 24;
constexpr uint32_t kRunShare = 4;                // run-heavy: runs <= n / kRunShare
constexpr uint32_t kMask24 = (1u << 24) - 1;
static_assert(kRunScreenMax / kRunShare <= kRunRankLimit, "a screened batch's runs fit the 24-bit rank field");

// Digram census (dense_batch): distinct byte pairs among the first kProbeSample positions of each
// block, one workgroup a block, a 65 536-bit LDS bitmap. Uniform-random bytes give ~3 970
// distinct pairs in 4 K positions, text a few hundred (16 K samples: the same split at twice
// the kernel time, 10.6 vs 5.2 us for 32 blocks).
constexpr uint32_t kProbeSample = 4096, kProbeNT = 1024;
// boffs null: block b is [b * bs, b * bs + bs). out: pinned host memory (vector stores).
__global__ __launch_bounds__(kProbeNT) void k_probe_digrams(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ boffs, uint64_t bs,
                                                            uint32_t *__restrict__ out)
{
    __shared__ uint32_t bm[2048];
    __shared__ uint32_t s_tot;
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint64_t o = boffs ? boffs[b] : b * bs;
    const uint32_t m = (uint32_t)min<uint64_t>((boffs ? boffs[b + 1] : o + bs) - o, kProbeSample);
    for (uint32_t i = t; i < 2048; i += kProbeNT) bm[i] = 0;
    if (t == 0) s_tot = 0;
    __syncthreads();
    const uint8_t *x = in + o;
    for (uint32_t i = t; i + 1 < m; i += kProbeNT) {
        const uint32_t d = ((uint32_t)x[i] << 8) | x[i + 1];
        atomicOr(&bm[d >> 5], 1u << (d & 31u));
    }
    __syncthreads();
    uint32_t k = 0;
    for (uint32_t i = t; i < 2048; i += kProbeNT) k += __builtin_popcount(bm[i]);
    k = wave_sum_dpp(k);
    if ((t & 63u) == 0) atomicAdd(&s_tot, k);
    __syncthreads();
    if (t == 0) out[b] = s_tot;
}

// Run heads per block: grid (tiles of 4096 positions, blocks); thread t takes 16 positions.
__global__ __launch_bounds__(256) void k_run_count(const uint8_t *__restrict__ in, const uint64_t *__restrict__ boffs,
                                                   uint32_t *__restrict__ count)
{
    const uint32_t b = blockIdx.y;
    const uint64_t o = boffs[b];
    const uint32_t n = (uint32_t)(boffs[b + 1] - o);
    const uint32_t p0 = blockIdx.x * 4096u + threadIdx.x * 16u;
    uint32_t k = 0;
    if (p0 < n) {
        const uint8_t *t = in + o;
        uint32_t prev = t[p0 ? p0 - 1 : n - 1];
        const uint32_t e = min(n, p0 + 16u);
        for (uint32_t p = p0; p < e; ++p) {
            const uint32_t x = t[p];
            k += x != prev;
            prev = x;
        }
    }
    k = wave_sum_dpp(k);
    if ((threadIdx.x & 63u) == 0 && k) atomicAdd(&count[b], k);
}

// Gather / scatter whole blocks between two layouts: grid (tiles of kMoveTile bytes, blocks),
// 16 bytes a thread (byte loads; the offsets carry no alignment).
constexpr uint32_t kMoveTile = 4096;
__global__ __launch_bounds__(256) void k_move_blocks(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                     const uint64_t *__restrict__ so, const uint64_t *__restrict__ dofs,
                                                     const uint64_t *__restrict__ len)
{
    const uint32_t b = blockIdx.y;
    const uint64_t n = len[b], s0 = so[b], d0 = dofs[b];
    const uint64_t i0 = (uint64_t)blockIdx.x * kMoveTile + threadIdx.x;
    uint8_t v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = i0 + 256u * k;
        v[k] = i < n ? src[s0 + i] : 0;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = i0 + 256u * k;
        if (i < n) dst[d0 + i] = v[k];
    }
}

__global__ __launch_bounds__(256) void k_prim_scatter(const uint32_t *__restrict__ tmp, const uint32_t *__restrict__ map,
                                                      uint32_t nb, uint32_t *__restrict__ prim)
{
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j < nb) prim[map[j]] = tmp[j];
}

// ---- in-house primitives (no library sort on the hot path): tiles of kPrimTile elements,
// 256 threads x 16 each.
constexpr uint32_t kPrimTile = 4096;

// Run heads in position order (stream compaction of T[p] != T[p - 1], cyclic): per-tile head
// counts, their exclusive scan (k_tiles_excl), then each thread writes the heads of its 16
// consecutive positions at its tile's offset + its workgroup prefix (k_bheads_*).
__device__ __forceinline__ uint32_t head_bits16(const uint8_t *__restrict__ t, uint32_t n, uint32_t p0)
{
    uint32_t f = 0;
    if (p0 < n) {
        uint32_t prev = t[p0 ? p0 - 1 : n - 1];
        const uint32_t e = min(n, p0 + 16u);
        for (uint32_t p = p0; p < e; ++p) {
            const uint32_t x = t[p];
            f |= (uint32_t)(x != prev) << (p - p0);
            prev = x;
        }
    }
    return f;
}
// One workgroup: exclusive prefix (op = sum, or max with identity 0) of cnt[0..m) into out.
// gate: non-null and set -> no work (unused since round 6's active-run doubling; kept for the sorts)
#define RUN_GATED(gate) \
    if ((gate) && *(gate)) return
template <bool MAX>
__global__ __launch_bounds__(1024) void k_tiles_excl(const uint32_t *__restrict__ cnt, uint32_t m, uint32_t *__restrict__ out,
                                                     const uint32_t *gate)
{
    RUN_GATED(gate);
    __shared__ uint32_t s_tmp[17];
    const uint32_t per = (m + 1023) / 1024, t = threadIdx.x, a = min(m, t * per), e = min(m, a + per);
    uint32_t acc = 0;
    for (uint32_t i = a; i < e; ++i) acc = MAX ? max(acc, cnt[i]) : acc + cnt[i];
    uint32_t run = MAX ? block_excl_max<1024>(acc, s_tmp) : block_excl_sum<1024>(acc, s_tmp, nullptr);
    for (uint32_t i = a; i < e; ++i) {
        const uint32_t v = cnt[i];
        out[i] = run;
        run = MAX ? max(run, v) : run + v;
    }
}

// LSD radix sort of (u64 key, u32 value) pairs by kRsBits-bit digits, stable. Tiles of kRsTile
// elements, 256 threads; wave w holds the tile's elements [1024 w, 1024 w + 1024) in 16 rounds of
// 64. Per pass: a tile histogram (digit-major [kRsBins][tiles]), then a scatter: each wave ranks
// its elements by digit with no barrier (a ballot match gives the rank among the round's equal
// digits, running per-wave digit counters in LDS carry it across rounds), one barrier, then the
// waves' counts are scanned per digit and every element goes to tile offset + waves below + its
// rank. The scatter takes its digit offsets from the counts of the tiles before it (up to
// kRsInlineTiles tiles: two launches a pass), or from a per-digit scan (k_rsort_rows) beyond.
constexpr uint32_t kRsBits = 11, kRsBins = 1u << kRsBits, kRsDPT = kRsBins / 256;  // digits per thread
constexpr uint32_t kRsTile = 4096, kRsInlineTiles = 4;  // inline: each tile reads kRsBins x tiles counts
__global__ __launch_bounds__(256) void k_rsort_hist(const uint64_t *__restrict__ key, uint32_t n, uint32_t shift,
                                                    uint32_t ntiles, uint32_t *__restrict__ cnt, const uint32_t *gate)
{
    RUN_GATED(gate);
    __shared__ uint32_t h[kRsBins];
    const uint32_t t = threadIdx.x;
    for (uint32_t d = t; d < kRsBins; d += 256) h[d] = 0;
    __syncthreads();
#pragma unroll 4
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t i = blockIdx.x * kRsTile + j * 256u + t;
        if (i < n) atomicAdd(&h[(uint32_t)(key[i] >> shift) & (kRsBins - 1)], 1u);
    }
    __syncthreads();
    for (uint32_t d = t; d < kRsBins; d += 256) cnt[(size_t)d * ntiles + blockIdx.x] = h[d];
}
// grid = kRsBins digits: row d of cnt -> exclusive prefix over the tiles (in place), total in dtot[d]
__global__ __launch_bounds__(256) void k_rsort_rows(uint32_t *__restrict__ cnt, uint32_t ntiles, uint32_t *__restrict__ dtot,
                                                    const uint32_t *gate)
{
    RUN_GATED(gate);
    __shared__ uint32_t s_tmp[8];
    uint32_t *row = cnt + (size_t)blockIdx.x * ntiles;
    uint32_t carry = 0;
    for (uint32_t b = 0; b < ntiles; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < ntiles ? row[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_sum1<256>(v, s_tmp, &tot);
        if (i < ntiles) row[i] = carry + ex;
        carry += tot;
        __syncthreads();  // s_tmp reuse
    }
    if (threadIdx.x == 0) dtot[blockIdx.x] = carry;
}
// INLINE: cnt holds raw tile counts (<= kRsInlineTiles tiles); else rowpre / dtot from k_rsort_rows
template <bool INLINE>
__global__ __launch_bounds__(256) void k_rsort_scatter(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                       uint64_t *__restrict__ kout, uint32_t *__restrict__ vout, uint32_t n,
                                                       uint32_t shift, uint32_t ntiles, const uint32_t *__restrict__ cnt,
                                                       const uint32_t *__restrict__ dtot, const uint32_t *gate)
{
    RUN_GATED(gate);
    __shared__ uint32_t s_wc[4][kRsBins + 1], s_tmp[8];
    const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63u;
    // thread t owns digits kRsDPT t .. kRsDPT t + kRsDPT - 1: their totals and this tile's prefix
    uint32_t tot[kRsDPT], pre[kRsDPT];
#pragma unroll
    for (uint32_t q = 0; q < kRsDPT; ++q) {
        const uint32_t d = kRsDPT * t + q;
        const uint32_t *row = cnt + (size_t)d * ntiles;
        tot[q] = pre[q] = 0;
        if (INLINE) {
            for (uint32_t u = 0; u < ntiles; ++u) {
                const uint32_t c = row[u];
                pre[q] += u < blockIdx.x ? c : 0u;
                tot[q] += c;
            }
        } else {
            pre[q] = row[blockIdx.x];
            tot[q] = dtot[d];
        }
    }
    for (uint32_t i = t; i < 4 * (kRsBins + 1); i += 256) (&s_wc[0][0])[i] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << l) - 1;
    const uint32_t i0 = blockIdx.x * kRsTile + w * 1024u + l;
    uint64_t k[16];
    uint32_t v[16], r[16];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t i = i0 + 64u * j;
        k[j] = i < n ? kin[i] : 0ull;
        v[j] = i < n ? vin[i] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        // digit of element j, kRsBins for padding (its own value, apart from every digit)
        const uint32_t d = i0 + 64u * j < n ? (uint32_t)(k[j] >> shift) & (kRsBins - 1) : kRsBins;
        uint64_t m = ~0ull;
#pragma unroll
        for (uint32_t bit = 0; bit <= kRsBits; ++bit) {
            const uint64_t bal = __ballot((d >> bit) & 1u);
            m &= ((d >> bit) & 1u) ? bal : ~bal;
        }
        const uint32_t below = (uint32_t)__builtin_popcountll(m & lt);
        const uint32_t base = s_wc[w][d];
        wave_sync();  // every lane's read before the leader's update (a wave's LDS ops run in order)
        if (below == 0) s_wc[w][d] = base + (uint32_t)__builtin_popcountll(m);
        wave_sync();
        r[j] = (base + below) | (d << 16);
    }
    __syncthreads();
    // digits of thread t: offset of the tile's run + the counts of the waves below each wave
    {
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < kRsDPT; ++q) sum += tot[q];
        uint32_t base = block_excl_sum1<256>(sum, s_tmp);
        uint32_t c[kRsDPT][3];
#pragma unroll
        for (uint32_t q = 0; q < kRsDPT; ++q)
#pragma unroll
            for (uint32_t u = 0; u < 3; ++u) c[q][u] = s_wc[u][kRsDPT * t + q];
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < kRsDPT; ++q) {
            const uint32_t d = kRsDPT * t + q, b0 = base + pre[q];
            s_wc[0][d] = b0;
            s_wc[1][d] = b0 + c[q][0];
            s_wc[2][d] = b0 + c[q][0] + c[q][1];
            s_wc[3][d] = b0 + c[q][0] + c[q][1] + c[q][2];
            base += tot[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        if (i0 + 64u * j >= n) continue;
        const uint32_t pos = s_wc[w][r[j] >> 16] + (r[j] & 0xffffu);
        kout[pos] = k[j];
        vout[pos] = v[j];
    }
}
__global__ __launch_bounds__(256) void k_rsort_copy(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                    uint64_t *__restrict__ kout, uint32_t *__restrict__ vout, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        kout[i] = kin[i];
        vout[i] = vin[i];
    }
}

// first sorted slot of each key's group (0 elsewhere) per thread run of 16 slots, the tile's
// largest (its last head) in tmax, and the group count
__global__ __launch_bounds__(256) void k_group_heads(const uint64_t *__restrict__ sk, uint32_t m, uint32_t *__restrict__ tmax,
                                                     uint32_t *__restrict__ ngroups, const uint32_t *gate)
{
    RUN_GATED(gate);
    __shared__ uint32_t s_tmp[8];
    const uint32_t j0 = blockIdx.x * kPrimTile + 16u * threadIdx.x;
    uint32_t last = 0, heads = 0;
    for (uint32_t j = j0; j < min(m, j0 + 16u); ++j)
        if (j == 0 || sk[j] != sk[j - 1]) {
            last = j;
            ++heads;
        }
    const uint32_t mx = wave_incl_max(last);
    const uint32_t k = wave_sum_dpp(heads);
    if ((threadIdx.x & 63u) == 63u) s_tmp[threadIdx.x >> 6] = mx;
    if ((threadIdx.x & 63u) == 0 && k) atomicAdd(ngroups, k);
    __syncthreads();
    if (threadIdx.x == 0) tmax[blockIdx.x] = max(max(s_tmp[0], s_tmp[1]), max(s_tmp[2], s_tmp[3]));
}

// rank[sidx[j]] = the slot of the last group head <= j: the tiles' exclusive max prefix (tpre),
// then within the tile a workgroup max-scan over the 16-slot runs
__global__ __launch_bounds__(256) void k_rank_scatter(const uint64_t *__restrict__ sk, const uint32_t *__restrict__ sidx,
                                                      uint32_t m, const uint32_t *__restrict__ tpre,
                                                      uint32_t *__restrict__ rank, const uint32_t *gate)
{
    RUN_GATED(gate);
    __shared__ uint32_t s_tmp[8];
    const uint32_t j0 = blockIdx.x * kPrimTile + 16u * threadIdx.x, e = min(m, j0 + 16u);
    uint32_t last = 0;
    for (uint32_t j = j0; j < e; ++j)
        if (j == 0 || sk[j] != sk[j - 1]) last = j;
    uint32_t g = max(tpre[blockIdx.x], block_excl_max<256>(last, s_tmp));
    for (uint32_t j = j0; j < e; ++j) {
        if (j == 0 || sk[j] != sk[j - 1]) g = j;
        rank[sidx[j]] = g;
    }
}

// ---- a batch of run-heavy blocks, sorted together: run j of block b is global run R_b + j,
// position p of block b is global position P_b + p; the block index sits above every sort key,
// so one sort (and one host wait a doubling round) serves all of them.
struct RBlk {
    uint64_t toff;      // byte offset of the block in the batch (input and L)
    uint32_t n, m;      // positions, cyclic runs
    uint32_t R, P, T;   // first global run, position, 4 K tile
    uint32_t slot;      // index of the block's primary in the output array
};

// run heads: grid (tiles of kPrimTile positions, blocks)
__global__ __launch_bounds__(256) void k_bheads_count(const uint8_t *__restrict__ in, const RBlk *__restrict__ tab,
                                                      uint32_t *__restrict__ tcnt)
{
    __shared__ uint32_t s_tmp[8];
    const RBlk B = tab[blockIdx.y];
    if (blockIdx.x * kPrimTile >= B.n) return;  // workgroup-uniform
    const uint32_t c = (uint32_t)__builtin_popcount(head_bits16(in + B.toff, B.n, blockIdx.x * kPrimTile + 16u * threadIdx.x));
    uint32_t tot;
    block_excl_sum1<256>(c, s_tmp, &tot);
    if (threadIdx.x == 0) tcnt[B.T + blockIdx.x] = tot;
}
// H[global run] = block-relative head position, rblk[global run] = block (toff: the tiles' exclusive
// prefix, so block b's heads start at R_b)
__global__ __launch_bounds__(256) void k_bheads_write(const uint8_t *__restrict__ in, const RBlk *__restrict__ tab,
                                                      const uint32_t *__restrict__ toff, uint32_t *__restrict__ H,
                                                      uint32_t *__restrict__ rblk)
{
    __shared__ uint32_t s_tmp[8];
    const RBlk B = tab[blockIdx.y];
    if (blockIdx.x * kPrimTile >= B.n) return;
    const uint32_t p0 = blockIdx.x * kPrimTile + 16u * threadIdx.x;
    uint32_t f = head_bits16(in + B.toff, B.n, p0);
    uint32_t o = toff[B.T + blockIdx.x] + block_excl_sum1<256>((uint32_t)__builtin_popcount(f), s_tmp);
    while (f) {
        const uint32_t k = (uint32_t)__builtin_ctz(f);
        H[o] = p0 + k;
        rblk[o++] = blockIdx.y;
        f &= f - 1;
    }
}

// K_i = b << 33 | c_i << 25 | [d_i > c_i] << 24 | (d_i > c_i ? ~L_i : L_i) & 0xffffff, value i
__global__ __launch_bounds__(256) void k_brun_keys(const uint8_t *__restrict__ in, const RBlk *__restrict__ tab,
                                                   const uint32_t *__restrict__ H, const uint32_t *__restrict__ rblk,
                                                   uint32_t M, uint64_t *__restrict__ key, uint32_t *__restrict__ idx)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= M) return;
    const uint32_t b = rblk[i];
    const RBlk B = tab[b];
    const uint8_t *t = in + B.toff;
    const uint32_t li = i - B.R;
    const uint32_t h = H[i], hn = H[B.R + (li + 1 < B.m ? li + 1 : 0)];
    const uint32_t len = hn > h ? hn - h : hn + B.n - h;
    const uint32_t cc = t[h], d = t[hn], up = d > cc;
    key[i] = (uint64_t)b << 33 | (uint64_t)cc << 25 | (uint64_t)up << 24 | (up ? kMask24 - len : len);
    idx[i] = i;
}

// ---- prefix doubling over the still-tied runs only (round 6). After a round,
// a run whose rank group is a singleton is finished (its rank is its final slot); the next round
// sorts only the members of groups of two or more (the "active" runs, listed in `act`) by
// (rank_i, rank_{i+h}). The members of one old group stay contiguous in the sorted list, so a
// member's new rank = its old group's first slot + (its new group's first index - its old group's
// first index) in the list, the first-slot ranks a full re-sort would give. pic (76 K runs) keeps
// 76 K, 72 K, 28 K, 6 K, 1.4 K, 342 and 72 runs active in its seven rounds: the rounds over more
// than kTailMax runs are multi-launch (keys, radix sort, rank + compaction: one host wait each),
// and every round after that runs inside ONE single-workgroup launch (k_act_tail).

// key = rank_i << bits | rank_{i + h} (cyclic in the run's block), value i, for the active runs
// (act null: runs 0 .. m - 1)
__global__ __launch_bounds__(256) void k_act_keys(const RBlk *__restrict__ tab, const uint32_t *__restrict__ rblk,
                                                  const uint32_t *__restrict__ rank, const uint32_t *__restrict__ act,
                                                  uint32_t m, uint32_t h, uint32_t bits, uint64_t *__restrict__ key,
                                                  uint32_t *__restrict__ idx)
{
    const uint32_t e = blockIdx.x * 256u + threadIdx.x;
    if (e >= m) return;
    const uint32_t i = act ? act[e] : e;
    const RBlk B = tab[rblk[i]];
    const uint32_t j = B.R + (uint32_t)(((uint64_t)(i - B.R) + h) % B.m);
    key[e] = (uint64_t)rank[i] << bits | rank[j];
    idx[e] = i;
}

// Slots [j0, j1) of sorted keys sk[0, m): the last new-group head and the last old-group start
// (0 when none: slot 0 is both) and the survivors (slots whose new group has two or more members).
__device__ __forceinline__ void act_slots(const uint64_t *sk, uint32_t m, uint32_t bits, uint32_t j0, uint32_t j1,
                                          uint32_t &lh, uint32_t &lg, uint32_t &sv)
{
    lh = lg = sv = 0;
    for (uint32_t j = j0; j < j1; ++j) {
        const uint64_t k = sk[j];
        const bool nh = j == 0 || k != sk[j - 1];
        const bool ng = j == 0 || (k >> bits) != (sk[j - 1] >> bits);
        const bool nn = j + 1 == m || sk[j + 1] != k;
        lh = nh ? j : lh;
        lg = ng ? j : lg;
        sv += !(nh && nn);
    }
}
// per tile of kPrimTile sorted slots: its last head, last old-group start and survivor count
__global__ __launch_bounds__(256) void k_act_tiles(const uint64_t *__restrict__ sk, uint32_t m, uint32_t bits,
                                                   uint32_t *__restrict__ tH, uint32_t *__restrict__ tG,
                                                   uint32_t *__restrict__ tC)
{
    __shared__ uint32_t s_h[4], s_g[4], s_c[4];
    const uint32_t j0 = min(m, blockIdx.x * kPrimTile + 16u * threadIdx.x);
    uint32_t lh, lg, sv;
    act_slots(sk, m, bits, j0, min(m, j0 + 16u), lh, lg, sv);
    lh = wave_incl_max(lh);
    lg = wave_incl_max(lg);
    sv = wave_sum_dpp(sv);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 63u) {
        s_h[w] = lh;
        s_g[w] = lg;
        s_c[w] = sv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        tH[blockIdx.x] = max(max(s_h[0], s_h[1]), max(s_h[2], s_h[3]));
        tG[blockIdx.x] = max(max(s_g[0], s_g[1]), max(s_g[2], s_g[3]));
        tC[blockIdx.x] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    }
}
// one workgroup: the tiles' exclusive max prefixes (tH, tG) and exclusive sum (tC), in place;
// cnt[0] = survivors of the round
__global__ __launch_bounds__(1024) void k_act_scan(uint32_t *__restrict__ tH, uint32_t *__restrict__ tG,
                                                   uint32_t *__restrict__ tC, uint32_t nt, uint32_t *__restrict__ cnt)
{
    __shared__ uint32_t s_tmp[17];
    const uint32_t per = (nt + 1023) / 1024, t = threadIdx.x, a = min(nt, t * per), e = min(nt, a + per);
    uint32_t mh = 0, mg = 0, sc = 0;
    for (uint32_t i = a; i < e; ++i) {
        mh = max(mh, tH[i]);
        mg = max(mg, tG[i]);
        sc += tC[i];
    }
    uint32_t rh = block_excl_max<1024>(mh, s_tmp);
    uint32_t rg = block_excl_max<1024>(mg, s_tmp);
    uint32_t tot;
    uint32_t rc = block_excl_sum<1024>(sc, s_tmp, &tot);
    for (uint32_t i = a; i < e; ++i) {
        const uint32_t h = tH[i], g = tG[i], c = tC[i];
        tH[i] = rh;
        tG[i] = rg;
        tC[i] = rc;
        rh = max(rh, h);
        rg = max(rg, g);
        rc += c;
    }
    if (t == 0) cnt[0] = tot;
}
// new ranks of the sorted active runs (rank[sv[j]]) and the survivors, in sorted order, to act_out
__global__ __launch_bounds__(256) void k_act_rank(const uint64_t *__restrict__ sk, const uint32_t *__restrict__ sv,
                                                  uint32_t m, uint32_t bits, const uint32_t *__restrict__ oH,
                                                  const uint32_t *__restrict__ oG, const uint32_t *__restrict__ oC,
                                                  uint32_t *__restrict__ rank, uint32_t *__restrict__ act_out)
{
    __shared__ uint32_t s_tmp[8];
    const uint32_t j0 = min(m, blockIdx.x * kPrimTile + 16u * threadIdx.x), j1 = min(m, j0 + 16u);
    uint32_t lh, lg, nsv;
    act_slots(sk, m, bits, j0, j1, lh, lg, nsv);
    uint32_t gh = max(oH[blockIdx.x], block_excl_max<256>(lh, s_tmp));
    uint32_t gg = max(oG[blockIdx.x], block_excl_max<256>(lg, s_tmp));
    uint32_t pos = oC[blockIdx.x] + block_excl_sum1<256>(nsv, s_tmp);
    for (uint32_t j = j0; j < j1; ++j) {
        const uint64_t k = sk[j];
        const bool nh = j == 0 || k != sk[j - 1];
        const bool ng = j == 0 || (k >> bits) != (sk[j - 1] >> bits);
        const bool nn = j + 1 == m || sk[j + 1] != k;
        gh = nh ? j : gh;
        gg = ng ? j : gg;
        const uint32_t i = sv[j];
        rank[i] = (uint32_t)(k >> bits) + gh - gg;
        if (!(nh && nn)) act_out[pos++] = i;
    }
}

// Every remaining round in one launch, once at most kTailMax runs are active: one workgroup keeps
// the active list in LDS; a round builds the keys (ranks read at agent scope, past this CU's L1:
// the previous round's rank stores are this workgroup's own), sorts them with a bitonic network in
// LDS (equal keys are one group, so the order among them does not matter), writes the new ranks
// and compacts the survivors, until none is left or h reaches the longest run sequence.
constexpr uint32_t kTailMax = 8192, kTailNT = 1024;
__global__ __launch_bounds__(kTailNT) void k_act_tail(const RBlk *__restrict__ tab, const uint32_t *__restrict__ rblk,
                                                      uint32_t *rank, const uint32_t *__restrict__ act, uint32_t m,
                                                      uint32_t h, uint32_t maxm, uint32_t bits)
{
    __shared__ uint64_t s_key[kTailMax];
    __shared__ uint32_t s_val[kTailMax], s_act[kTailMax];
    __shared__ uint32_t s_tmp[kTailNT / 64 + 1];
    const uint32_t t = threadIdx.x;
    for (uint32_t e = t; e < m; e += kTailNT) s_act[e] = act ? act[e] : e;
    __syncthreads();
    while (m > 0 && h < maxm) {  // m, h: workgroup-uniform
        uint32_t n2 = 1;
        while (n2 < m) n2 <<= 1;
        for (uint32_t e = t; e < n2; e += kTailNT) {
            uint64_t k = ~0ull;
            uint32_t i = 0;
            if (e < m) {
                i = s_act[e];
                const RBlk B = tab[rblk[i]];
                const uint32_t j = B.R + (uint32_t)(((uint64_t)(i - B.R) + h) % B.m);
                const uint32_t ri = __hip_atomic_load(rank + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t rj = __hip_atomic_load(rank + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                k = (uint64_t)ri << bits | rj;
            }
            s_key[e] = k;
            s_val[e] = i;
        }
        __syncthreads();
        for (uint32_t kk = 2; kk <= n2; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                for (uint32_t i = t; i < n2; i += kTailNT) {
                    const uint32_t ixj = i ^ jj;
                    if (ixj > i) {
                        const uint64_t a = s_key[i], b = s_key[ixj];
                        if ((a > b) == ((i & kk) == 0)) {
                            s_key[i] = b;
                            s_key[ixj] = a;
                            const uint32_t v = s_val[i];
                            s_val[i] = s_val[ixj];
                            s_val[ixj] = v;
                        }
                    }
                }
                __syncthreads();
            }
        const uint32_t per = (m + kTailNT - 1) / kTailNT, j0 = min(m, t * per), j1 = min(m, j0 + per);
        uint32_t lh, lg, nsv;
        act_slots(s_key, m, bits, j0, j1, lh, lg, nsv);
        uint32_t gh = block_excl_max<kTailNT>(lh, s_tmp);
        uint32_t gg = block_excl_max<kTailNT>(lg, s_tmp);
        uint32_t tot;
        uint32_t pos = block_excl_sum<kTailNT>(nsv, s_tmp, &tot);
        for (uint32_t j = j0; j < j1; ++j) {
            const uint64_t k = s_key[j];
            const bool nh = j == 0 || k != s_key[j - 1];
            const bool ng = j == 0 || (k >> bits) != (s_key[j - 1] >> bits);
            const bool nn = j + 1 == m || s_key[j + 1] != k;
            gh = nh ? j : gh;
            gg = ng ? j : gg;
            const uint32_t i = s_val[j];
            rank[i] = (uint32_t)(k >> bits) + gh - gg;
            if (!(nh && nn)) s_act[pos++] = i;
        }
        __threadfence();  // the new ranks reach the L2 before the next round's agent-scope reads
        __syncthreads();
        m = tot;
        h *= 2;
    }
}

// position keys (header comment) below the block index, value p: grid (tiles of 256, blocks)
__global__ __launch_bounds__(256) void k_bpos_keys(const uint8_t *__restrict__ in, const RBlk *__restrict__ tab,
                                                   const uint32_t *__restrict__ H, const uint32_t *__restrict__ rank,
                                                   uint64_t *__restrict__ key, uint32_t *__restrict__ val)
{
    const RBlk B = tab[blockIdx.y];
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= B.n) return;
    if (B.m == 0) {  // one byte value: identical rotations, kept in position order
        key[B.P + p] = (uint64_t)blockIdx.y << 57 | p;
        val[B.P + p] = p;
        return;
    }
    const uint8_t *t = in + B.toff;
    const uint32_t *Hb = H + B.R, m = B.m;
    // run of p: the last head <= p, or the wrapping last run when p precedes H[0]
    uint32_t lo = 0, hi = m;  // Hb[lo] <= p < Hb[hi] (Hb[m] = infinity)
    if (p < Hb[0]) {
        lo = m - 1;
    } else {
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (Hb[mid] <= p) lo = mid;
            else hi = mid;
        }
    }
    const uint32_t nx = lo + 1 < m ? lo + 1 : 0, hn = Hb[nx];
    const uint32_t r = hn > p ? hn - p : hn + B.n - p;
    const uint32_t cc = t[p], up = t[hn] > cc;
    key[B.P + p] = (uint64_t)blockIdx.y << 57 | (uint64_t)cc << 49 | (uint64_t)up << 48 |
                   (uint64_t)(up ? kMask24 - r : r) << 24 | rank[B.R + nx];
    val[B.P + p] = p;
}

// L and primaries from the sorted positions: grid (tiles of 256, blocks)
__global__ __launch_bounds__(256) void k_brun_out(const uint8_t *__restrict__ in, const RBlk *__restrict__ tab,
                                                  const uint32_t *__restrict__ sp, uint8_t *__restrict__ L,
                                                  uint32_t *__restrict__ prim)
{
    const RBlk B = tab[blockIdx.y];
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= B.n) return;
    const uint8_t *t = in + B.toff;
    const uint32_t p = B.m ? sp[B.P + j] : j;  // one byte value: n identical rotations in order
    L[B.toff + j] = t[p ? p - 1 : B.n - 1];
    if (p == 0) prim[B.slot] = j;
}

inline uint32_t bits_for(uint32_t v)  // bits holding 0 .. v
{
    uint32_t b = 1;
    while (b < 32 && (v >> b)) ++b;
    return b;
}

struct RunWs {
    uint32_t *H, *rblk, *idx, *idx2, *rank, *act, *act2, *cnt, *tcnt, *toff, *tC, *rowpre, *dtot;
    uint64_t *key, *key2;
    uint64_t *pkey, *pkey2;
    uint32_t *pval, *pval2;
    RBlk *tab;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace of a run batch (N positions, M runs, NT position tiles, B blocks), carved from one slot.
RunWs run_ws(Ctx *c, uint64_t N, uint32_t M, uint32_t NT, uint32_t B)
{
    const size_t mm = std::max(M, 1u), nt = std::max<size_t>(NT, cdiv(std::max<uint64_t>(N, 1), kRsTile));
    const size_t sizes[] = {align256(mm * 4) * 7 + 256, align256(nt * 4) * 3, align256(kRsBins * nt * 4) + kRsBins * 4,
                            align256(mm * 8) * 2, align256((size_t)N * 8) * 2, align256((size_t)N * 4) * 2,
                            align256((size_t)B * sizeof(RBlk))};
    size_t total = 0;
    for (size_t z : sizes) total += z;
    uint8_t *p = (uint8_t *)c->get(WS_RUNS, total);
    RunWs w;
    uint32_t **u32s[] = {&w.H, &w.rblk, &w.idx, &w.idx2, &w.rank, &w.act, &w.act2};
    for (auto q : u32s) {
        *q = (uint32_t *)p;
        p += align256(mm * 4);
    }
    w.cnt = (uint32_t *)p;
    p += 256;
    w.tcnt = (uint32_t *)p;
    p += align256(nt * 4);
    w.toff = (uint32_t *)p;
    p += align256(nt * 4);
    w.tC = (uint32_t *)p;
    p += align256(nt * 4);
    w.rowpre = (uint32_t *)p;
    p += align256(kRsBins * nt * 4);
    w.dtot = (uint32_t *)p;
    p += kRsBins * 4;
    w.key = (uint64_t *)p;
    p += align256(mm * 8);
    w.key2 = (uint64_t *)p;
    p += align256(mm * 8);
    w.pkey = (uint64_t *)p;
    p += align256((size_t)N * 8);
    w.pkey2 = (uint64_t *)p;
    p += align256((size_t)N * 8);
    w.pval = (uint32_t *)p;
    p += align256((size_t)N * 4);
    w.pval2 = (uint32_t *)p;
    p += align256((size_t)N * 4);
    w.tab = (RBlk *)p;
    return w;
}

// Ranks of sorted keys sk (m of them, values sidx): rank[sidx[j]] = first slot of sk[j]'s
// group; the group count lands in w.cnt[0] (zeroed before by a memset).
void rank_groups_async(Ctx *c, RunWs &w, const uint64_t *sk, const uint32_t *sidx, uint32_t m, const uint32_t *gate)
{
    const uint32_t nt = cdiv(m, kPrimTile);
    BMH_LAUNCH(c, "bwt_run_groups", k_group_heads, nt, 256, 0, sk, m, w.tcnt, w.cnt, gate);
    BMH_LAUNCH(c, "bwt_run_scan", k_tiles_excl<true>, 1, 1024, 0, w.tcnt, nt, w.toff, gate);
    BMH_LAUNCH(c, "bwt_run_groups", k_rank_scatter, nt, 256, 0, sk, sidx, m, w.toff, w.rank, gate);
}
// The same, returning the group count (one host wait).
uint32_t rank_groups(Ctx *c, RunWs &w, const uint64_t *sk, const uint32_t *sidx, uint32_t m, uint32_t *h_cnt)
{
    BMH_HIP(hipMemsetAsync(w.cnt, 0, 4, c->stream));
    rank_groups_async(c, w, sk, sidx, m, nullptr);
    c->d2h(h_cnt, w.cnt, 4);
    c->sync();
    return *h_cnt;
}

// Stable sort of cnt (key, value) pairs by key bits [0, end_bit): result in (kout, vout), or
// (any_out) in whichever of the two buffers the last pass wrote (returned: true = kin / vin);
// the other pair is scratch.
bool sort_pairs(Ctx *c, RunWs &w, uint64_t *kin, uint64_t *kout, uint32_t *vin, uint32_t *vout, uint32_t cnt,
                uint32_t end_bit, const uint32_t *gate = nullptr, bool any_out = false)
{
    const uint32_t nt = cdiv(cnt, kRsTile), passes = (end_bit + kRsBits - 1) / kRsBits;
    uint64_t *ks = kin, *kd = kout;
    uint32_t *vs = vin, *vd = vout;
    for (uint32_t ps = 0; ps < passes; ++ps) {
        const uint32_t sh = kRsBits * ps;
        BMH_LAUNCH(c, "bwt_run_sort", k_rsort_hist, nt, 256, 0, ks, cnt, sh, nt, w.rowpre, gate);
        if (nt <= kRsInlineTiles) {
            BMH_LAUNCH(c, "bwt_run_sort", k_rsort_scatter<true>, nt, 256, 0, ks, vs, kd, vd, cnt, sh, nt, w.rowpre,
                       w.dtot, gate);
        } else {
            BMH_LAUNCH(c, "bwt_run_sort", k_rsort_rows, kRsBins, 256, 0, w.rowpre, nt, w.dtot, gate);
            BMH_LAUNCH(c, "bwt_run_sort", k_rsort_scatter<false>, nt, 256, 0, ks, vs, kd, vd, cnt, sh, nt, w.rowpre,
                       w.dtot, gate);
        }
        std::swap(ks, kd);
        std::swap(vs, vd);
    }
    if (any_out) return ks == kin;
    if (ks != kout) BMH_LAUNCH(c, "bwt_run_sort", k_rsort_copy, cdiv(cnt, 256), 256, 0, ks, vs, kout, vout, cnt);
    return false;
}

// The BWT of run-heavy blocks, all at once: block i = bytes [offs[i], offs[i] + ns[i]) of the
// batch `in` with ms[i] >= 0 cyclic runs; L at the same offsets of `L`, primary i in prim[i]
// (device). At most kRunBatchBlocks blocks (the block index takes the top bits of the keys).
constexpr uint32_t kRunBatchBlocks = 128;
void run_blocks_batch(Ctx *c, const uint8_t *in, const std::vector<uint64_t> &offs, const std::vector<uint32_t> &ns,
                      const std::vector<uint32_t> &ms, uint8_t *L, uint32_t *prim, uint32_t *h_cnt)
{
    const uint32_t B = (uint32_t)offs.size();
    if (B == 0) return;
    if (B > kRunBatchBlocks) fail(BMH_EINVAL, "bwt: too many run blocks in one batch");
    uint64_t Mtot = 0;
    for (uint32_t m : ms) Mtot += m;
    if (Mtot >= kRunRankLimit) fail(BMH_EINVAL, "bwt: too many runs in one run batch (24-bit ranks)");
    std::vector<RBlk> tab(B);
    uint64_t N = 0;
    uint32_t M = 0, NT = 0, maxn = 0, maxm = 0;
    for (uint32_t i = 0; i < B; ++i) {
        tab[i] = RBlk{offs[i], ns[i], ms[i], M, (uint32_t)N, NT, i};
        N += ns[i];
        M += ms[i];
        NT += cdiv(ns[i], kPrimTile);
        maxn = std::max(maxn, ns[i]);
        maxm = std::max(maxm, ms[i]);
    }
    RunWs w = run_ws(c, N, M, NT, B);
    c->h2d(w.tab, tab.data(), (size_t)B * sizeof(RBlk));
    const uint32_t bb = bits_for(B - 1);
    if (M > 0) {
        const dim3 tgrid(cdiv(maxn, kPrimTile), B);
        BMH_HIP(hipMemsetAsync(w.tcnt, 0, (size_t)NT * 4, c->stream));
        BMH_LAUNCH(c, "bwt_run_heads", k_bheads_count, tgrid, 256, 0, in, w.tab, w.tcnt);
        BMH_LAUNCH(c, "bwt_run_heads", k_tiles_excl<false>, 1, 1024, 0, w.tcnt, NT, w.toff, nullptr);
        BMH_LAUNCH(c, "bwt_run_heads", k_bheads_write, tgrid, 256, 0, in, w.tab, w.toff, w.H, w.rblk);
        BMH_LAUNCH(c, "bwt_run_keys", k_brun_keys, cdiv(M, 256), 256, 0, in, w.tab, w.H, w.rblk, M, w.key, w.idx);
        sort_pairs(c, w, w.key, w.key2, w.idx, w.idx2, M, 33 + bb);
        const uint32_t groups = rank_groups(c, w, w.key2, w.idx2, M, h_cnt);
        const uint32_t bits = bits_for(M - 1);
        // prefix doubling over the run sequence: round h sorts (rank_i, rank_{i+h}) of the runs
        // still tied and re-ranks them, until none is tied (or h >= the longest run sequence);
        // rounds over more than kTailMax runs take one host wait each, the rest one launch
        if (groups < M && maxm > 1) {
            uint64_t h = 1;
            uint32_t ma = M;
            const uint32_t *act = nullptr;  // all runs
            uint32_t *abuf[2] = {w.act, w.act2};
            for (int ab = 0; ma > kTailMax; ab ^= 1) {
                BMH_LAUNCH(c, "bwt_run_keys", k_act_keys, cdiv(ma, 256), 256, 0, w.tab, w.rblk, w.rank, act, ma,
                           (uint32_t)h, bits, w.key, w.idx);
                const bool in_key = sort_pairs(c, w, w.key, w.key2, w.idx, w.idx2, ma, 2 * bits, nullptr, true);
                const uint64_t *sk = in_key ? w.key : w.key2;
                const uint32_t *sv = in_key ? w.idx : w.idx2;
                const uint32_t nt = cdiv(ma, kPrimTile);
                BMH_LAUNCH(c, "bwt_run_groups", k_act_tiles, nt, 256, 0, sk, ma, bits, w.tcnt, w.toff, w.tC);
                BMH_LAUNCH(c, "bwt_run_scan", k_act_scan, 1, 1024, 0, w.tcnt, w.toff, w.tC, nt, w.cnt);
                BMH_LAUNCH(c, "bwt_run_groups", k_act_rank, nt, 256, 0, sk, sv, ma, bits, w.tcnt, w.toff, w.tC, w.rank,
                           abuf[ab]);
                c->d2h(h_cnt, w.cnt, 4);
                c->sync();
                ma = *h_cnt;
                act = abuf[ab];
                h *= 2;
                if (h >= maxm) ma = 0;  // the runs still tied are identical rotations
            }
            if (ma > 0)
                BMH_LAUNCH(c, "bwt_run_tail", k_act_tail, 1, kTailNT, 0, w.tab, w.rblk, w.rank, act, ma, (uint32_t)h,
                           maxm, bits);
        }
        const dim3 pgrid(cdiv(maxn, 256), B);
        BMH_LAUNCH(c, "bwt_run_place", k_bpos_keys, pgrid, 256, 0, in, w.tab, w.H, w.rank, w.pkey, w.pval);
        sort_pairs(c, w, w.pkey, w.pkey2, w.pval, w.pval2, (uint32_t)N, 57 + bb);
    }
    BMH_LAUNCH(c, "bwt_run_out", k_brun_out, dim3(cdiv(maxn, 256), B), 256, 0, in, w.tab, w.pval2, L, prim);
}
}  // namespace

// Whether a batch is dense (uniform-like bytes: the BWT's two data passes resolve it with one
// short list round, no host-synchronised rounds), by the digram census of each block's first
// 4 K positions: at least half of the sampled pairs distinct, for blocks holding >= 90 % of the
// bytes. encode_blocks runs such batches on one pipeline: on random data the pipelines only
// contend (128 MiB: 1.77 ms on one, 1.99 on four). One launch (1024 threads a block; block
// offsets from the block size when the blocks are equal) whose counts land in pinned memory,
// and one wait (≈ 60 -> ≈ 25 us of a 128 MiB batch's 1.7 ms: no staging copies).
bool dense_batch(Ctx *c, const uint8_t *d_in, const Batch &bt)
{
    const uint32_t nb = bt.nblocks;
    const uint64_t bs = bt.offs[1];
    bool uniform = true;
    for (uint32_t b = 1; b < nb && uniform; ++b) uniform = bt.offs[b + 1] - bt.offs[b] == bs;
    uint8_t *d_misc = (uint8_t *)c->get(WS_RUN_MISC, (size_t)(nb + 1) * 8 + (size_t)nb * 8 + 1024);
    uint64_t *d_boffs = (uint64_t *)d_misc;
    if (c->probe_cap < nb) {
        if (c->probe_host) {
            BMH_HIP(hipStreamSynchronize(c->stream));
            BMH_HIP(hipHostFree(c->probe_host));
            c->probe_host = nullptr;
        }
        BMH_HIP(hipHostMalloc((void **)&c->probe_host, (size_t)nb * 4, hipHostMallocDefault));
        c->probe_cap = nb;
    }
    if (!uniform) c->h2d(d_boffs, bt.offs.data(), (size_t)(nb + 1) * 8);
    if (!c->probe_ev) BMH_HIP(hipEventCreateWithFlags(&c->probe_ev, hipEventDisableTiming));
    BMH_LAUNCH(c, "probe_digrams", k_probe_digrams, nb, kProbeNT, 0, d_in, uniform ? nullptr : d_boffs, bs,
               c->probe_host);
    BMH_HIP(hipEventRecord(c->probe_ev, c->stream));
    // a batch past the run screen that turns out dense runs bwt_batch_core on this context and
    // stream: its global-pass prologue is queued behind the census now, so the GPU works through
    // the host's wait and the launches that follow it. Only when the last batch of this layout was
    // dense: the prologue sizes every BWT workspace of this context (~40 B per input byte), which a
    // text batch, encoded on the sub-pipelines' own contexts, would leave allocated here unused
    // (ADVICE r5). A prologue that cannot allocate is skipped (pre_sig stays unset; the batch then
    // runs its own prologue).
    const uint64_t lsig = layout_sig(11, bt.offs, 0);
    if (bt.total > kRunScreenMax && !c->opt.pipelines && c->dense_sig == lsig) {
        try {
            bwt_batch_core(c, d_in, bt, nullptr, nullptr, true);
        } catch (const Error &e) {
            if (e.status != BMH_ENOMEM) throw;
            c->pre_sig = 0;
        }
    }
    for (;;) {  // spin: a blocking wait can sleep the host thread for milliseconds
        const hipError_t e = hipEventQuery(c->probe_ev);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) BMH_HIP(e);
        spin_pause();
    }
    uint64_t dense = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint64_t n = bt.offs[b + 1] - bt.offs[b];
        const uint64_t m = std::min<uint64_t>(n, kProbeSample);
        if (m >= 4096 && 2ull * c->probe_host[b] >= m) dense += n;
    }
    const bool is_dense = dense * 10 >= bt.total * 9;
    c->dense_sig = is_dense ? lsig : 0;
    return is_dense;
}

// Batch BWT: small batches are screened for run-heavy blocks, which take the run path above;
// every other block goes through the rotation sorter (bwt_batch_core), gathered into one
// contiguous sub-batch when run blocks sit between them.
void bwt_batch(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_L, uint64_t *h_primary)
{
    const uint32_t nb = bt.nblocks;
    bool screen = (c->screen_total ? c->screen_total : bt.total) <= kRunScreenMax;
    if (screen) {
        screen = false;
        for (uint32_t b = 0; b < nb && !screen; ++b) {
            const uint64_t n = bt.offs[b + 1] - bt.offs[b];
            screen = n >= kRunMinBlock && n <= kRunMaxBlock;
        }
    }
    if (!screen) {
        bwt_batch_core(c, d_in, bt, d_L, h_primary);
        return;
    }
    // ---- screen: cyclic run count of every block
    uint8_t *d_misc = (uint8_t *)c->get(WS_RUN_MISC, (size_t)(nb + 1) * 8 + (size_t)nb * 8 + 1024);
    uint64_t *d_boffs = (uint64_t *)d_misc;
    uint32_t *d_count = (uint32_t *)(d_misc + (size_t)(nb + 1) * 8);
    uint32_t *d_rmap = d_count + nb;  // run-path block indices
    std::vector<uint32_t> runs(nb);
    c->h2d(d_boffs, bt.offs.data(), (size_t)(nb + 1) * 8);
    BMH_HIP(hipMemsetAsync(d_count, 0, (size_t)nb * 4, c->stream));
    BMH_LAUNCH(c, "bwt_run_count", k_run_count, dim3(cdiv(bt.max_n, 4096), nb), 256, 0, d_in, d_boffs, d_count);
    c->d2h(runs.data(), d_count, (size_t)nb * 4);
    c->sync();
    std::vector<uint32_t> rb, keep;  // run-path blocks, sorter blocks
    for (uint32_t b = 0; b < nb; ++b) {
        const uint64_t n = bt.offs[b + 1] - bt.offs[b];
        const bool heavy = n >= kRunMinBlock && n <= kRunMaxBlock && (uint64_t)runs[b] * kRunShare <= n;
        (heavy ? rb : keep).push_back(b);
    }
    if (rb.empty()) {
        bwt_batch_core(c, d_in, bt, d_L, h_primary);
        return;
    }
    uint32_t *d_prim = (uint32_t *)c->get(WS_PRIMARY, nb * 4 + 64);  // full-batch capacity first
    // the run blocks' primaries go to a side array of the context that runs them, then to d_prim
    uint32_t *rp = nullptr;
    auto run_blocks = [&](Ctx *x) {
        WallPhase wall(x, "bwt_runs");
        uint32_t *p = (uint32_t *)x->get(WS_RUN_PRIM, rb.size() * 4 + 64);
        uint32_t h_cnt = 0;
        // all run blocks sorted together (one host wait a doubling round for all of them), in
        // groups of at most kRunBatchBlocks blocks and fewer than kRunRankLimit runs
        for (size_t g = 0; g < rb.size();) {
            std::vector<uint64_t> offs;
            std::vector<uint32_t> ns, ms;
            uint64_t m = 0;
            size_t i = g;
            for (; i < rb.size() && i - g < kRunBatchBlocks && (i == g || m + runs[rb[i]] < kRunRankLimit); ++i) {
                offs.push_back(bt.offs[rb[i]]);
                ns.push_back((uint32_t)(bt.offs[rb[i] + 1] - bt.offs[rb[i]]));
                ms.push_back(runs[rb[i]]);
                m += runs[rb[i]];
            }
            run_blocks_batch(x, d_in, offs, ns, ms, d_L, p + g, &h_cnt);
            g = i;
        }
        rp = p;
    };
    auto sorter_blocks = [&]() {
        // the sorter blocks as one contiguous batch (in place when they already are one); its
        // primaries land in WS_PRIMARY[0 .. keep) and are moved to their blocks' slots
        const uint32_t nk = (uint32_t)keep.size();
        Batch sb;
        sb.nblocks = nk;
        sb.offs.assign(1, 0);
        for (uint32_t b : keep) {
            const uint64_t n = bt.offs[b + 1] - bt.offs[b];
            sb.offs.push_back(sb.offs.back() + n);
            sb.max_n = std::max<uint32_t>(sb.max_n, (uint32_t)n);
        }
        sb.total = sb.offs.back();
        const bool contiguous = keep.back() - keep.front() + 1 == nk;
        // per kept block: source offset, compact offset, length (u64), block index, primary (u32)
        uint8_t *d_mv = (uint8_t *)c->get(WS_RUN_MOVE, (size_t)nk * 32 + 1024);
        uint64_t *d_so = (uint64_t *)d_mv, *d_co = d_so + nk, *d_len = d_co + nk;
        uint32_t *d_map = (uint32_t *)(d_len + nk), *d_tprim = d_map + nk;
        std::vector<uint64_t> hv(3 * (size_t)nk);
        std::vector<uint32_t> hmap(nk);
        for (uint32_t j = 0; j < nk; ++j) {
            hv[j] = bt.offs[keep[j]];
            hv[nk + j] = sb.offs[j];
            hv[2 * nk + j] = sb.offs[j + 1] - sb.offs[j];
            hmap[j] = keep[j];
        }
        c->h2d(d_so, hv.data(), hv.size() * 8);
        c->h2d(d_map, hmap.data(), (size_t)nk * 4);
        if (contiguous) {
            const uint64_t base = bt.offs[keep.front()];
            bwt_batch_core(c, d_in + base, sb, d_L + base, nullptr);
        } else {
            uint8_t *tin = (uint8_t *)c->get(WS_RUN_IN, sb.total);
            uint8_t *tL = (uint8_t *)c->get(WS_RUN_L, sb.total);
            const dim3 grid(cdiv(sb.max_n, kMoveTile), nk);
            BMH_LAUNCH(c, "bwt_run_move", k_move_blocks, grid, 256, 0, d_in, tin, d_so, d_co, d_len);
            bwt_batch_core(c, tin, sb, tL, nullptr);
            BMH_LAUNCH(c, "bwt_run_move", k_move_blocks, grid, 256, 0, tL, d_L, d_co, d_so, d_len);
        }
        if (keep.front() != 0 || !contiguous) {
            BMH_HIP(hipMemcpyAsync(d_tprim, d_prim, (size_t)nk * 4, hipMemcpyDeviceToDevice, c->stream));
            BMH_LAUNCH(c, "bwt_run_move", k_prim_scatter, cdiv(nk, 256), 256, 0, d_tprim, d_map, nk, d_prim);
        }
    };
    if (keep.empty()) {
        run_blocks(c);
    } else {
        // the run path on the side context (its own stream and workspaces, one host thread)
        // beside the rotation sorter: they write disjoint L ranges and primary arrays
        Ctx *x = aux_ctx(c);
        std::exception_ptr err;
        std::thread th([&] {
            try {
                BMH_HIP(hipSetDevice(c->device));
                run_blocks(x);
                x->sync();
            } catch (...) {
                err = std::current_exception();
            }
        });
        try {
            sorter_blocks();
        } catch (...) {
            th.join();
            throw;
        }
        th.join();
        if (err) std::rethrow_exception(err);
        if (c->timing) {
            for (auto &kv : x->stats) {
                c->stats[kv.first].launches += kv.second.launches;
                c->stats[kv.first].ms += kv.second.ms;
            }
            x->stats.clear();
        }
    }
    c->h2d(d_rmap, rb.data(), rb.size() * 4);
    BMH_LAUNCH(c, "bwt_run_move", k_prim_scatter, cdiv(rb.size(), 256), 256, 0, rp, d_rmap, (uint32_t)rb.size(), d_prim);
    if (h_primary) {
        std::vector<uint32_t> hp(nb);
        c->d2h(hp.data(), d_prim, (size_t)nb * 4);
        c->sync();
        for (uint32_t b = 0; b < nb; ++b) h_primary[b] = hp[b];
    }
}

}  // namespace bmh
