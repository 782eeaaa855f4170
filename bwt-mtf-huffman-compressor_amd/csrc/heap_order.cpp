// heap_order.cpp — the reference's Huffman tie-break for small blocks.
//
// The reference's std::priority_queue<pair<long, BTree*>> (main.cpp:232) pops equal
// frequencies in descending BTree* order, and the nodes come from `new BTree` (:240, :252), so
// its tree bytes depend on where glibc places 24-byte blocks. SURVEY App. B.3's closed-form
// order (addr_rank in huffman.hip / huffman_host.cpp) holds from 64.6 KB up; below that the
// blocks freed earlier in the run (the input vector's growth, the BWT / MTF temporaries, the
// queue's own vector) are reused and the order changes with the block size n.
//
// A standalone COMPRESS run makes a fixed sequence of heap calls that depends only on n and on
// the leaf count L (read_bytes io_utilities.h:40-54, bwt main.cpp:77-91, move_to_front :93-112,
// huffman :229-257; listed in heap_calls below). This file restates glibc 2.35's main-arena
// allocator for those calls (malloc/malloc.c: tcache, fastbins, unsorted / small / large bins,
// top, sysmalloc, systrim, malloc_consolidate; x86-64 constants) and replays them, so the
// address order of the 2L - 1 nodes is exact for every n and L. band_ranks(n) returns, per L,
// the rank of every node id where it differs from the closed-form order (cached per n).
// Checked call by call and address by address against traces of the reference binary
// (oracle/alloc_trace) and byte for byte against its records in the bands (tests/test_bands.py).
#include "bmh_internal.h"

#include <algorithm>
#include <atomic>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <unordered_map>

namespace bmh {

namespace {

constexpr uint64_t kSizeSz = 8, kAlign = 16, kMinSize = 32, kPage = 4096;
constexpr uint32_t kTcBins = 64, kTcCount = 7;
constexpr uint64_t kMaxFast = 128, kMinLarge = 1024, kConsolidateAt = 65536, kTopPad = 128 * 1024;
constexpr uint64_t kMmapThresholdMax = 32ull << 20, kMmapBase = 1ull << 44;

uint64_t request2size(uint64_t req)
{
    const uint64_t s = (req + kSizeSz + kAlign - 1) & ~(kAlign - 1);
    return s < kMinSize ? kMinSize : s;
}

uint32_t largebin_index(uint64_t sz)
{
    if ((sz >> 6) <= 48) return 48 + (uint32_t)(sz >> 6);
    if ((sz >> 9) <= 20) return 91 + (uint32_t)(sz >> 9);
    if ((sz >> 12) <= 10) return 110 + (uint32_t)(sz >> 12);
    if ((sz >> 15) <= 4) return 119 + (uint32_t)(sz >> 15);
    if ((sz >> 18) <= 2) return 124 + (uint32_t)(sz >> 18);
    return 126;
}

uint32_t bin_index(uint64_t sz) { return sz < kMinLarge ? (uint32_t)(sz >> 4) : largebin_index(sz); }

// glibc 2.35 main arena, one thread; addresses are offsets from the heap start (brk start).
struct HeapSim {
    struct Chunk {
        uint64_t size;
        int32_t bin;  // -1: allocated, in a tcache bin or a fastbin (inuse bit set); else its bin
    };
    // every chunk carved from the heap (top excluded), by address: a sorted vector (a few
    // hundred entries; copied once per leaf count by compute_band_ranks)
    struct Map {
        std::vector<std::pair<uint64_t, Chunk>> v;
        using It = std::vector<std::pair<uint64_t, Chunk>>::iterator;
        It lb(uint64_t a)
        {
            return std::lower_bound(v.begin(), v.end(), a,
                                    [](const std::pair<uint64_t, Chunk> &e, uint64_t x) { return e.first < x; });
        }
        It find(uint64_t a)
        {
            It it = lb(a);
            return it != v.end() && it->first == a ? it : v.end();
        }
        It begin() { return v.begin(); }
        It end() { return v.end(); }
        Chunk &at(uint64_t a)
        {
            It it = find(a);
            if (it == v.end()) throw std::logic_error("heap_order: no chunk");
            return it->second;
        }
        Chunk &operator[](uint64_t a)
        {
            It it = lb(a);
            if (it == v.end() || it->first != a) it = v.insert(it, {a, Chunk{0, -1}});
            return it->second;
        }
        It erase(It it) { return v.erase(it); }
    } ch;
    std::vector<uint64_t> bins[128];    // unsorted (1), small, large; head (fd side) first
    std::vector<uint64_t> tc[kTcBins];  // back = head
    std::vector<uint64_t> fb[10];       // back = head
    std::vector<std::pair<uint64_t, uint64_t>> mm;  // mmapped blocks: (mem, chunk size)
    bool have_fast = false, tc_ready = false;
    uint64_t top = 0, top_size = 0, last_rem = ~0ull, mm_next = kMmapBase;
    uint64_t mmap_thr = 128 * 1024, trim_thr = 128 * 1024;

    void unlink(uint64_t p)
    {
        Chunk &c = ch.at(p);
        auto &b = bins[c.bin];
        b.erase(std::find(b.begin(), b.end(), p));
        c.bin = -1;
    }
    void to_unsorted(uint64_t p)
    {
        bins[1].insert(bins[1].begin(), p);
        ch.at(p).bin = 1;
    }
    void place(uint64_t p)  // unsorted -> small bin (head) or large bin (glibc's sorted insert)
    {
        Chunk &c = ch.at(p);
        const uint64_t sz = c.size;
        uint32_t i;
        if (sz < kMinLarge) {
            i = (uint32_t)(sz >> 4);
            bins[i].insert(bins[i].begin(), p);
        } else {
            i = largebin_index(sz);
            auto &b = bins[i];
            auto S = [&](size_t k) { return ch.at(b[k]).size; };
            if (b.empty() || sz < S(b.size() - 1)) {
                b.push_back(p);
            } else {
                size_t k = 0;
                while (sz < S(k)) {  // walk the size groups from the largest down
                    const uint64_t s = S(k);
                    while (k < b.size() && S(k) == s) ++k;
                }
                b.insert(b.begin() + (ptrdiff_t)(sz == S(k) ? k + 1 : k), p);  // equal size: second
            }
        }
        c.bin = (int32_t)i;
    }
    uint64_t take_tail(uint32_t i)
    {
        const uint64_t v = bins[i].back();
        bins[i].pop_back();
        ch.at(v).bin = -1;
        return v;
    }
    uint64_t from_top(uint64_t nb)
    {
        const uint64_t p = top;
        ch[p] = Chunk{nb, -1};
        top += nb;
        top_size -= nb;
        return p + 16;
    }
    uint64_t sysmalloc(uint64_t nb)
    {
        if (nb >= mmap_thr) {
            const uint64_t sz = (nb + kSizeSz + kPage - 1) & ~(kPage - 1);
            const uint64_t mem = mm_next + 16;
            mm_next += sz + kPage;
            mm.push_back({mem, sz});
            return mem;
        }
        const uint64_t size = (nb + kTopPad + kMinSize - top_size + kPage - 1) & ~(kPage - 1);
        top_size += size;
        return from_top(nb);
    }
    uint64_t split(uint64_t p, uint64_t nb, bool small_req)
    {
        Chunk &c = ch.at(p);
        const uint64_t sz = c.size;
        if (sz - nb >= kMinSize) {
            c.size = nb;
            const uint64_t r = p + nb;
            ch[r] = Chunk{sz - nb, -1};
            to_unsorted(r);
            if (small_req) last_rem = r;
        }
        return p + 16;
    }
    // free-side merging of chunk p (in no bin); returns the merged size (top's if merged into it)
    uint64_t coalesce(uint64_t p)
    {
        auto it = ch.find(p);
        uint64_t sz = it->second.size;
        if (it != ch.begin()) {
            auto pv = std::prev(it);
            if (pv->second.bin >= 0 && pv->first + pv->second.size == p) {
                unlink(pv->first);
                sz += pv->second.size;
                ch.erase(it);
                p = pv->first;
                pv->second.size = sz;
                it = pv;
            }
        }
        const uint64_t nx = p + sz;
        if (nx == top) {
            ch.erase(it);
            top = p;
            top_size += sz;
            return top_size;
        }
        auto nt = ch.find(nx);
        if (nt != ch.end() && nt->second.bin >= 0) {
            unlink(nx);
            sz += nt->second.size;
            ch.erase(nt);
            ch.at(p).size = sz;
        }
        to_unsorted(p);
        return sz;
    }
    void consolidate()
    {
        have_fast = false;
        for (auto &f : fb) {
            std::vector<uint64_t> chain(f.rbegin(), f.rend());  // from the head, following fd
            f.clear();
            for (uint64_t p : chain) coalesce(p);
        }
    }
    void systrim()
    {
        const uint64_t area = top_size - kMinSize - 1;
        if (area <= kTopPad) return;
        const uint64_t extra = (area - kTopPad) & ~(kPage - 1);
        top_size -= extra;
    }
    bool tc_put(uint64_t p)
    {
        const uint64_t ti = (ch.at(p).size - kMinSize) / kAlign;
        if (ti < kTcBins && tc[ti].size() < kTcCount) {
            tc[ti].push_back(p);
            return true;
        }
        return false;
    }

    uint64_t malloc(uint64_t req)
    {
        if (!tc_ready) {  // tcache_init: the per-thread struct (0x280 bytes) is the first chunk
            tc_ready = true;
            int_malloc(request2size(0x280));
        }
        const uint64_t nb = request2size(req), ti = (nb - kMinSize) / kAlign;
        if (ti < kTcBins && !tc[ti].empty()) {
            const uint64_t p = tc[ti].back();
            tc[ti].pop_back();
            return p + 16;
        }
        return int_malloc(nb);
    }

    uint64_t int_malloc(uint64_t nb)
    {
        const uint64_t ti = (nb - kMinSize) / kAlign;
        const bool tc_ok = ti < kTcBins, small = nb < kMinLarge;
        if (nb <= kMaxFast) {
            auto &f = fb[(nb >> 4) - 2];
            if (!f.empty()) {
                const uint64_t v = f.back();
                f.pop_back();
                while (tc_ok && tc[ti].size() < kTcCount && !f.empty()) {
                    tc[ti].push_back(f.back());
                    f.pop_back();
                }
                return v + 16;
            }
        }
        if (small) {
            const uint32_t i = (uint32_t)(nb >> 4);
            if (!bins[i].empty()) {
                const uint64_t v = take_tail(i);
                while (tc_ok && tc[ti].size() < kTcCount && !bins[i].empty()) tc[ti].push_back(take_tail(i));
                return v + 16;
            }
        } else if (have_fast) {
            consolidate();
        }
        for (;;) {
            bool cached = false;
            uint32_t iters = 0;
            auto &ub = bins[1];
            while (!ub.empty()) {
                const uint64_t v = ub.back();
                const uint64_t sz = ch.at(v).size;
                if (small && ub.size() == 1 && v == last_rem && sz > nb + kMinSize) {
                    take_tail(1);
                    return split(v, nb, true);
                }
                take_tail(1);
                if (sz == nb) {
                    if (tc_ok && tc[ti].size() < kTcCount) {
                        tc[ti].push_back(v);
                        cached = true;
                        continue;
                    }
                    return v + 16;
                }
                place(v);
                if (++iters >= 10000) break;
            }
            if (cached) {
                const uint64_t p = tc[ti].back();
                tc[ti].pop_back();
                return p + 16;
            }
            if (!small) {
                auto &b = bins[largebin_index(nb)];
                auto S = [&](size_t k) { return ch.at(b[k]).size; };
                if (!b.empty() && S(0) >= nb) {
                    // the smallest size group >= nb; its second member when it has one
                    size_t k = b.size() - 1;
                    while (S(k) < nb) --k;
                    const uint64_t s = S(k);
                    while (k > 0 && S(k - 1) == s) --k;
                    if (k + 1 < b.size() && S(k + 1) == s) ++k;
                    const uint64_t v = b[k];
                    b.erase(b.begin() + (ptrdiff_t)k);
                    ch.at(v).bin = -1;
                    return split(v, nb, false);
                }
            }
            for (uint32_t i = bin_index(nb) + 1; i < 128; ++i)
                if (!bins[i].empty()) return split(take_tail(i), nb, small);
            if (top_size >= nb + kMinSize) return from_top(nb);
            if (have_fast) {
                consolidate();
                continue;
            }
            return sysmalloc(nb);
        }
    }

    void free(uint64_t mem)
    {
        auto m = std::find_if(mm.begin(), mm.end(), [&](const std::pair<uint64_t, uint64_t> &e) { return e.first == mem; });
        if (m != mm.end()) {
            const uint64_t sz = m->second;
            mm.erase(m);
            if (sz > mmap_thr && sz <= kMmapThresholdMax) {
                mmap_thr = sz;
                trim_thr = 2 * sz;
            }
            return;
        }
        const uint64_t p = mem - 16;
        if (tc_put(p)) return;
        const uint64_t sz0 = ch.at(p).size;
        if (sz0 <= kMaxFast) {
            fb[(sz0 >> 4) - 2].push_back(p);
            have_fast = true;
            return;
        }
        if (coalesce(p) >= kConsolidateAt) {
            if (have_fast) consolidate();
            if (top_size >= trim_thr) systrim();
        }
    }
};

// The heap calls of a standalone COMPRESS run up to huffman()'s queue (main.cpp:232-237):
// libstdc++'s emergency pool, read_bytes (io_utilities.h:40-54), bwt (main.cpp:77-91),
// compress's copy of the BWT output (:308), move_to_front (:93-112), frequencies and
// already_in_queue (:231,:234).
void replay_to_huffman(HeapSim &h, uint64_t n)
{
    h.malloc(72704);
    const uint64_t file = h.malloc(472), fbuf = h.malloc(8192);
    uint64_t c = 1, bytes = h.malloc(1);  // istreambuf_iterator growth of `bytes`
    while (c < n) {
        const uint64_t nb = h.malloc(2 * c);
        h.free(bytes);
        bytes = nb;
        c *= 2;
    }
    h.free(fbuf);
    h.free(file);
    const uint64_t data = h.malloc(n);
    h.malloc(n);  // the returned tuple's vector (lives to the end of compress)
    h.free(bytes);
    h.free(data);
    const uint64_t arg = h.malloc(n), order = h.malloc(8 * n);
    h.free(h.malloc(8 * ((n + 1) / 2)));  // stable_sort's buffer
    const uint64_t enc = h.malloc(n);
    h.malloc(n);  // make_pair copy (bwt_result)
    h.free(enc);
    h.free(order);
    h.free(arg);
    h.malloc(n);  // bwt_data
    const uint64_t marg = h.malloc(n), alpha = h.malloc(256);
    h.malloc(n);  // mtf_data
    h.free(alpha);
    h.free(marg);
    h.malloc(2048);  // frequencies
    h.malloc(32);    // already_in_queue
}

// SURVEY App. B.3's closed-form ascending-address list (the same order as addr_rank).
uint32_t model_index(uint32_t L, uint32_t s)
{
    if (L <= 128) {
        if (s == 1) return 0;
        if (s >= 3 && s <= 127) return s - 2;
        if (s == 0) return 126;
        if (s == 2) return 127;
        return s;
    }
    if (s == 1) return 0;
    if (s >= 3 && s <= 64) return s - 2;
    if (s >= 129 && s <= 192) return s - 66;
    if (s >= 65 && s <= 127) return s + 62;
    if (s == 0) return 190;
    if (s == 2) return 191;
    if (s == 128) return 192;
    return s;
}

// No free block can serve a 24-byte request: the top serves the next ones in address order
// (a top too small for one is extended in place: the brk heap is contiguous).
bool top_only(const HeapSim &h)
{
    if (!h.tc[0].empty() || !h.fb[0].empty()) return false;
    for (uint32_t i = 1; i < 128; ++i)
        if (!h.bins[i].empty()) return false;
    return true;
}

// k 24-byte allocations from state s (the internal nodes, main.cpp:252; no frees in between),
// addresses to out. Two runs are carved in address order without the full allocator path: the
// top, and a last remainder that is the unsorted bin's only chunk (each request splits 32 bytes
// off it while it is larger than 64: malloc.c's last-remainder rule for small requests). The
// allocated chunks are not recorded: nothing is freed afterwards.
void m24_run(HeapSim &s, uint32_t k, uint64_t *out)
{
    for (uint32_t j = 0; j < k;) {
        if (top_only(s)) {
            for (uint64_t a = s.top + 16; j < k; ++j, a += 32) out[j] = a;
            return;
        }
        if (s.tc[0].empty() && s.fb[0].empty() && s.bins[2].empty() && s.bins[1].size() == 1 &&
            s.bins[1][0] == s.last_rem) {
            const uint64_t p0 = s.last_rem;
            uint64_t p = p0, sz = s.ch.at(p0).size;
            if (sz > 64) {
                while (j < k && sz > 64) {
                    out[j++] = p + 16;
                    p += 32;
                    sz -= 32;
                }
                s.ch.erase(s.ch.find(p0));
                s.ch[p] = HeapSim::Chunk{sz, 1};
                s.bins[1][0] = p;
                s.last_rem = p;
                continue;
            }
        }
        out[j++] = s.malloc(24);
    }
}

std::unique_ptr<BandRanks> compute_band_ranks(uint64_t n)
{
    auto out = std::make_unique<BandRanks>();
    out->off.assign(257, kModelOrder);
    HeapSim h;
    replay_to_huffman(h, n);
    const uint32_t lmax = (uint32_t)std::min<uint64_t>(256, n);
    uint64_t addr[511];
    uint64_t cap = 0, pq = 0;
    bool any = false;
    for (uint32_t i = 0; i < lmax; ++i) {
        addr[i] = h.malloc(24);  // leaf i (main.cpp:240), then its push grows a full vector
        if (i == cap) {
            const uint64_t nc = cap ? 2 * cap : 1;
            const uint64_t nbuf = h.malloc(16 * nc);
            if (cap) h.free(pq);
            pq = nbuf;
            cap = nc;
        }
        const uint32_t L = i + 1, nn = 2 * L - 1;
        if (top_only(h)) {  // every internal node is carved from the top, one after another
            for (uint32_t j = L; j < nn; ++j) addr[j] = h.top + 16 + 32 * (uint64_t)(j - L);
        } else {
            HeapSim s = h;
            m24_run(s, nn - L, addr + L);  // internal nodes (main.cpp:252)
        }
        uint16_t idx[511];
        for (uint32_t j = 0; j < nn; ++j) idx[j] = (uint16_t)j;
        std::sort(idx, idx + nn, [&](uint16_t a, uint16_t b) { return addr[a] < addr[b]; });
        uint16_t rank[511];
        bool same = true;
        for (uint32_t k = 0; k < nn; ++k) rank[idx[k]] = (uint16_t)k;
        // the closed form indexes the full 511-entry list: compare the two as orders
        for (uint32_t a = 0; a + 1 < nn && same; ++a)
            same = model_index(L, idx[a]) < model_index(L, idx[a + 1]);
        if (!same) {
            any = true;
            out->off[L] = (uint32_t)out->rank.size();
            out->rank.insert(out->rank.end(), rank, rank + nn);
        }
    }
    if (!any) return nullptr;
    return out;
}

// Process-wide cache of band_ranks per block size, bounded: least recently used
// sizes are dropped past kBandCacheBytes of rank tables or kBandCacheEntries sizes. Entries are
// shared_ptr, so a table a caller still holds survives its eviction.
constexpr size_t kBandCacheBytes = 64u << 20;
constexpr size_t kBandCacheEntries = 1u << 16;
struct BandEntry {
    std::shared_ptr<const BandRanks> r;  // null: the closed form holds for every L
    uint64_t used;
    size_t bytes;
};
std::mutex g_band_mu;
std::unordered_map<uint64_t, BandEntry> g_band;
size_t g_band_bytes = 0;
uint64_t g_band_clock = 0;

void band_evict_locked()
{
    while (g_band.size() > 1 && (g_band_bytes > kBandCacheBytes || g_band.size() > kBandCacheEntries)) {
        auto lru = g_band.begin();
        for (auto it = g_band.begin(); it != g_band.end(); ++it)
            if (it->second.used < lru->second.used) lru = it;
        g_band_bytes -= lru->second.bytes;
        g_band.erase(lru);
    }
}

}  // namespace

size_t band_cache_entries()
{
    std::lock_guard<std::mutex> lk(g_band_mu);
    return g_band.size();
}

std::shared_ptr<const BandRanks> band_ranks(uint64_t n)
{
    if (n == 0 || n >= kBandCeil) return nullptr;
    {
        std::lock_guard<std::mutex> lk(g_band_mu);
        auto it = g_band.find(n);
        if (it != g_band.end()) {
            it->second.used = ++g_band_clock;
            return it->second.r;
        }
    }
    std::shared_ptr<const BandRanks> r(compute_band_ranks(n).release());  // outside the lock
    std::lock_guard<std::mutex> lk(g_band_mu);
    auto it = g_band.find(n);
    if (it == g_band.end()) {
        const size_t bytes = 64 + (r ? r->off.size() * 4 + r->rank.size() * 2 : 0);
        it = g_band.emplace(n, BandEntry{std::move(r), ++g_band_clock, bytes}).first;
        g_band_bytes += bytes;
        std::shared_ptr<const BandRanks> keep = it->second.r;
        band_evict_locked();
        return keep;
    }
    it->second.used = ++g_band_clock;
    return it->second.r;
}

std::map<uint64_t, std::shared_ptr<const BandRanks>> band_ranks_batch(const std::vector<uint64_t> &sizes)
{
    // every distinct size's table, the missing ones computed in parallel; the returned
    // shared_ptrs keep the batch's tables alive even if the LRU cache evicts them meanwhile
    std::vector<uint64_t> todo;
    for (uint64_t n : sizes)
        if (n && n < kBandCeil) todo.push_back(n);
    std::sort(todo.begin(), todo.end());
    todo.erase(std::unique(todo.begin(), todo.end()), todo.end());
    std::vector<std::shared_ptr<const BandRanks>> got(todo.size());
    const unsigned nt = std::min<unsigned>((unsigned)todo.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    if (nt <= 1) {
        for (size_t i = 0; i < todo.size(); ++i) got[i] = band_ranks(todo[i]);
    } else {
        std::atomic<size_t> next{0};
        std::mutex emu;
        std::exception_ptr err;  // the first failure of a worker, rethrown on this thread
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&] {
                try {
                    for (size_t i; (i = next.fetch_add(1)) < todo.size();) got[i] = band_ranks(todo[i]);
                } catch (...) {
                    std::lock_guard<std::mutex> lk(emu);
                    if (!err) err = std::current_exception();
                    next.store(todo.size());
                }
            });
        for (auto &x : th) x.join();
        if (err) std::rethrow_exception(err);
    }
    std::map<uint64_t, std::shared_ptr<const BandRanks>> out;
    for (size_t i = 0; i < todo.size(); ++i) out.emplace(todo[i], std::move(got[i]));
    return out;
}

void node_ranks(uint64_t n, uint32_t L, uint16_t *rank)
{
    const auto br = band_ranks(n);
    if (br && L <= 256 && br->off[L] != kModelOrder) {
        memcpy(rank, br->rank.data() + br->off[L], (2 * L - 1) * sizeof(uint16_t));
        return;
    }
    // the closed form, as ranks among the 2L - 1 nodes
    uint16_t idx[511];
    const uint32_t nn = 2 * L - 1;
    for (uint32_t j = 0; j < nn; ++j) idx[j] = (uint16_t)j;
    std::sort(idx, idx + nn, [&](uint16_t a, uint16_t b) { return model_index(L, a) < model_index(L, b); });
    for (uint32_t k = 0; k < nn; ++k) rank[idx[k]] = (uint16_t)k;
}

}  // namespace bmh
