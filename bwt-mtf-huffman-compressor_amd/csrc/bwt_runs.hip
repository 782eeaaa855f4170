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
#include <rocprim/rocprim.hpp>

#include "device_util.h"

namespace bmh {

void bwt_batch_core(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_L, uint64_t *h_primary);

namespace {

constexpr uint64_t kRunScreenMax = 64ull << 20;  // batches screened for run-heavy blocks
constexpr uint32_t kRunMinBlock = 1u << 16;      // shorter blocks stay on the rotation sorter
constexpr uint32_t kRunMaxBlock = 1u << 24;      // run lengths and ranks fit 24 bits of the key
constexpr uint32_t kRunShare = 4;                // run-heavy: runs <= n / kRunShare
constexpr uint32_t kMask24 = (1u << 24) - 1;

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

__global__ __launch_bounds__(256) void k_head_flags(const uint8_t *__restrict__ t, uint32_t n, uint8_t *__restrict__ f)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p < n) f[p] = t[p] != t[p ? p - 1 : n - 1];
}

// K_i = c_i << 25 | [d_i > c_i] << 24 | (d_i > c_i ? ~L_i : L_i) & 0xffffff, value i
__global__ __launch_bounds__(256) void k_run_keys(const uint8_t *__restrict__ t, uint32_t n, const uint32_t *__restrict__ H,
                                                  uint32_t m, uint64_t *__restrict__ key, uint32_t *__restrict__ idx)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= m) return;
    const uint32_t h = H[i], hn = H[i + 1 < m ? i + 1 : 0];
    const uint32_t len = hn > h ? hn - h : hn + n - h;
    const uint32_t cc = t[h], d = t[hn], up = d > cc;
    key[i] = (uint64_t)cc << 25 | (uint64_t)up << 24 | (up ? kMask24 - len : len);
    idx[i] = i;
}

// (rank_i, rank_{i+h}) packed in 2 * bits, value i
__global__ __launch_bounds__(256) void k_pair_keys(const uint32_t *__restrict__ rank, uint32_t m, uint32_t h,
                                                   uint32_t bits, uint64_t *__restrict__ key, uint32_t *__restrict__ idx)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= m) return;
    const uint32_t j = i + h < m ? i + h : i + h - m;
    key[i] = (uint64_t)rank[i] << bits | rank[j];
    idx[i] = i;
}

// first sorted slot of each key's group (0 elsewhere; a max-scan spreads it) + group count
__global__ __launch_bounds__(256) void k_group_heads(const uint64_t *__restrict__ sk, uint32_t m, uint32_t *__restrict__ g,
                                                     uint32_t *__restrict__ ngroups)
{
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    const bool head = j < m && (j == 0 || sk[j] != sk[j - 1]);
    if (j < m) g[j] = head ? j : 0u;
    const uint32_t k = wave_sum_dpp((uint32_t)head);
    if ((threadIdx.x & 63u) == 0 && k) atomicAdd(ngroups, k);
}

__global__ __launch_bounds__(256) void k_rank_scatter(const uint32_t *__restrict__ gs, const uint32_t *__restrict__ sidx,
                                                      uint32_t m, uint32_t *__restrict__ rank)
{
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j < m) rank[sidx[j]] = gs[j];
}

// position keys (header comment), value p
__global__ __launch_bounds__(256) void k_pos_keys(const uint8_t *__restrict__ t, uint32_t n, const uint32_t *__restrict__ H,
                                                  uint32_t m, const uint32_t *__restrict__ rank, uint64_t *__restrict__ key,
                                                  uint32_t *__restrict__ val)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n) return;
    // run of p: the last head <= p, or the wrapping last run when p precedes H[0]
    uint32_t lo = 0, hi = m;  // H[lo] <= p < H[hi] (H[m] = infinity)
    if (p < H[0]) {
        lo = m - 1;
    } else {
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (H[mid] <= p) lo = mid;
            else hi = mid;
        }
    }
    const uint32_t nx = lo + 1 < m ? lo + 1 : 0, hn = H[nx];
    const uint32_t r = hn > p ? hn - p : hn + n - p;
    const uint32_t cc = t[p], up = t[hn] > cc;
    key[p] = (uint64_t)cc << 49 | (uint64_t)up << 48 | (uint64_t)(up ? kMask24 - r : r) << 24 | rank[nx];
    val[p] = p;
}

__global__ __launch_bounds__(256) void k_run_out(const uint8_t *__restrict__ t, uint32_t n, const uint32_t *__restrict__ sp,
                                                 uint8_t *__restrict__ L, uint32_t *__restrict__ prim)
{
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= n) return;
    const uint32_t p = sp ? sp[j] : j;
    L[j] = t[p ? p - 1 : n - 1];
    if (p == 0) *prim = j;
}

inline uint32_t bits_for(uint32_t v)  // bits holding 0 .. v
{
    uint32_t b = 1;
    while (b < 32 && (v >> b)) ++b;
    return b;
}

struct RunWs {
    uint8_t *flags;
    uint32_t *H, *idx, *idx2, *g, *gs, *rank, *cnt;
    uint64_t *key, *key2;
    uint64_t *pkey, *pkey2;
    uint32_t *pval, *pval2;
    void *tmp;
    size_t tmp_bytes;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace of one block's run BWT (n positions, m runs), carved from one slot.
RunWs run_ws(Ctx *c, uint32_t n, uint32_t m)
{
    size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    BMH_HIP(rocprim::select(nullptr, t1, rocprim::counting_iterator<uint32_t>(0), (const uint8_t *)nullptr,
                            (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, c->stream));
    BMH_HIP(rocprim::radix_sort_pairs(nullptr, t2, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                      (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)std::max(m, 1u), 0, 64,
                                      c->stream));
    BMH_HIP(rocprim::radix_sort_pairs(nullptr, t3, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                      (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0, 64, c->stream));
    BMH_HIP(rocprim::inclusive_scan(nullptr, t4, (const uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)std::max(m, 1u),
                                    rocprim::maximum<uint32_t>(), c->stream));
    const size_t tb = align256(std::max(std::max(t1, t2), std::max(t3, t4)));
    const size_t mm = std::max(m, 1u);
    const size_t sizes[] = {align256(n), align256(mm * 4) * 6 + 256, align256(mm * 8) * 2, align256((size_t)n * 8) * 2,
                            align256((size_t)n * 4) * 2, tb};
    size_t total = 0;
    for (size_t s : sizes) total += s;
    uint8_t *p = (uint8_t *)c->get(WS_RUNS, total);
    RunWs w;
    w.flags = p;
    p += sizes[0];
    uint32_t **u32s[] = {&w.H, &w.idx, &w.idx2, &w.g, &w.gs, &w.rank};
    for (auto q : u32s) {
        *q = (uint32_t *)p;
        p += align256(mm * 4);
    }
    w.cnt = (uint32_t *)p;
    p += 256;
    w.key = (uint64_t *)p;
    p += align256(mm * 8);
    w.key2 = (uint64_t *)p;
    p += align256(mm * 8);
    w.pkey = (uint64_t *)p;
    p += align256((size_t)n * 8);
    w.pkey2 = (uint64_t *)p;
    p += align256((size_t)n * 8);
    w.pval = (uint32_t *)p;
    p += align256((size_t)n * 4);
    w.pval2 = (uint32_t *)p;
    p += align256((size_t)n * 4);
    w.tmp = p;
    w.tmp_bytes = tb;
    return w;
}

// Ranks of sorted keys sk (m of them, values sidx): rank[sidx[j]] = first slot of sk[j]'s
// group. Returns the group count (one host wait).
uint32_t rank_groups(Ctx *c, RunWs &w, const uint64_t *sk, const uint32_t *sidx, uint32_t m, uint32_t *h_cnt)
{
    BMH_HIP(hipMemsetAsync(w.cnt, 0, 4, c->stream));
    BMH_LAUNCH(c, "bwt_run_groups", k_group_heads, cdiv(m, 256), 256, 0, sk, m, w.g, w.cnt);
    size_t tb = w.tmp_bytes;
    const int p = c->tbegin("bwt_run_scan");
    BMH_HIP(rocprim::inclusive_scan(w.tmp, tb, w.g, w.gs, (size_t)m, rocprim::maximum<uint32_t>(), c->stream));
    c->tend(p);
    BMH_LAUNCH(c, "bwt_run_groups", k_rank_scatter, cdiv(m, 256), 256, 0, w.gs, sidx, m, w.rank);
    c->d2h(h_cnt, w.cnt, 4);
    c->sync();
    return *h_cnt;
}

void sort_pairs(Ctx *c, RunWs &w, const uint64_t *kin, uint64_t *kout, const uint32_t *vin, uint32_t *vout, size_t cnt,
                uint32_t end_bit)
{
    size_t tb = w.tmp_bytes;
    const int p = c->tbegin("bwt_run_sort");
    BMH_HIP(rocprim::radix_sort_pairs(w.tmp, tb, kin, kout, vin, vout, cnt, 0, end_bit, c->stream));
    c->tend(p);
}

// The BWT of one run-heavy block t[0..n) with m >= 0 cyclic runs: L[0..n) and *prim (device).
void run_block(Ctx *c, const uint8_t *t, uint32_t n, uint32_t m, uint8_t *L, uint32_t *prim, uint32_t *h_cnt)
{
    if (m == 0) {  // one byte value: n identical rotations
        BMH_LAUNCH(c, "bwt_run_out", k_run_out, cdiv(n, 256), 256, 0, t, n, (const uint32_t *)nullptr, L, prim);
        return;
    }
    RunWs w = run_ws(c, n, m);
    BMH_LAUNCH(c, "bwt_run_heads", k_head_flags, cdiv(n, 256), 256, 0, t, n, w.flags);
    {
        size_t tb = w.tmp_bytes;
        const int p = c->tbegin("bwt_run_heads");
        BMH_HIP(rocprim::select(w.tmp, tb, rocprim::counting_iterator<uint32_t>(0), w.flags, w.H, w.cnt, (size_t)n,
                                c->stream));
        c->tend(p);
    }
    BMH_LAUNCH(c, "bwt_run_keys", k_run_keys, cdiv(m, 256), 256, 0, t, n, w.H, m, w.key, w.idx);
    sort_pairs(c, w, w.key, w.key2, w.idx, w.idx2, m, 33);
    uint32_t groups = rank_groups(c, w, w.key2, w.idx2, m, h_cnt);
    const uint32_t bits = bits_for(m - 1);
    for (uint64_t h = 1; groups < m && h < m; h *= 2) {
        BMH_LAUNCH(c, "bwt_run_keys", k_pair_keys, cdiv(m, 256), 256, 0, w.rank, m, (uint32_t)h, bits, w.key, w.idx);
        sort_pairs(c, w, w.key, w.key2, w.idx, w.idx2, m, 2 * bits);
        groups = rank_groups(c, w, w.key2, w.idx2, m, h_cnt);
    }
    BMH_LAUNCH(c, "bwt_run_place", k_pos_keys, cdiv(n, 256), 256, 0, t, n, w.H, m, w.rank, w.pkey, w.pval);
    sort_pairs(c, w, w.pkey, w.pkey2, w.pval, w.pval2, n, 57);
    BMH_LAUNCH(c, "bwt_run_out", k_run_out, cdiv(n, 256), 256, 0, t, n, w.pval2, L, prim);
}

}  // namespace

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
        for (size_t i = 0; i < rb.size(); ++i) {
            const uint64_t o = bt.offs[rb[i]];
            run_block(x, d_in + o, (uint32_t)(bt.offs[rb[i] + 1] - o), runs[rb[i]], d_L + o, p + i, &h_cnt);
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
