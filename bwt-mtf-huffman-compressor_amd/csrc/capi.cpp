// capi.cpp — the C ABI (include/bmh.h): contexts, workspace, timing, and the batch encode
// that chains the three device stages with the host Huffman build in between.
//
// Orchestration of one batch (compress(), reference main.cpp:300-325, minus file I/O):
//   bwt kernels -> L, primary        (bwt(), main.cpp:77-91)
//   mtf kernels -> MTF, freq, first  (move_to_front() main.cpp:93-112, huffman() :231-244)
//   host        -> code tables, tree bytes, record sizes/offsets (huffman() :245-254, :132-196)
//   pack kernels-> payloads in place behind the headers (encode_with_huffman() :158-172,
//                  write_bytes() io_utilities.h:7-27)
#include "bmh_internal.h"

#include <algorithm>
#include <cstdlib>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <sched.h>
#include <cstring>

namespace bmh {

static thread_local std::string g_last_error;

void set_last_error(const std::string &msg) { g_last_error = msg; }
[[noreturn]] void fail(bmh_status s, const std::string &msg) { throw Error(s, msg); }

void *Ctx::get(Slot s, size_t bytes)
{
    if (bytes == 0) bytes = 1;
    if (ws_size[s] >= bytes) return ws[s];
    ws_tag[s] = 0;
    if (ws[s]) {
        BMH_HIP(hipStreamSynchronize(stream));
        BMH_HIP(hipFree(ws[s]));
        ws[s] = nullptr;
        ws_size[s] = 0;
    }
    size_t sz = ((bytes + bytes / 8) + 255) & ~(size_t)255;
    void *p = nullptr;
    if (hipMalloc(&p, sz) != hipSuccess) {
        (void)hipGetLastError();
        fail(BMH_ENOMEM, "device allocation of " + std::to_string(sz) + " bytes failed");
    }
    ws[s] = p;
    ws_size[s] = sz;
    return p;
}

void *Ctx::host_pinned(size_t bytes)
{
    if (pinned_size >= bytes) return pinned;
    if (pinned) {
        BMH_HIP(hipStreamSynchronize(stream));
        BMH_HIP(hipHostFree(pinned));
        pinned = nullptr;
    }
    size_t sz = std::max<size_t>(bytes, 1 << 16);
    BMH_HIP(hipHostMalloc(&pinned, sz, hipHostMallocDefault));
    pinned_size = sz;
    return pinned;
}

hipEvent_t Ctx::ev()
{
    if (!event_pool.empty()) {
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    BMH_HIP(hipEventCreate(&e));
    return e;
}

int Ctx::tbegin(const char *name)
{
    if (!timing) return -1;
    Pending p{name, ev(), ev()};
    BMH_HIP(hipEventRecord(p.a, stream));
    pending.push_back(p);
    return (int)pending.size() - 1;
}

void Ctx::tend(int idx)
{
    if (idx < 0) return;
    BMH_HIP(hipEventRecord(pending[idx].b, stream));
}

static size_t arena_take(Ctx *c, size_t bytes)
{
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (c->arena_used + need > c->arena_size) {
        c->sync();
        if (need > c->arena_size) {
            if (c->arena) BMH_HIP(hipHostFree(c->arena));
            c->arena = nullptr;
            const size_t sz = std::max<size_t>(need, 16u << 20);
            BMH_HIP(hipHostMalloc((void **)&c->arena, sz, hipHostMallocDefault));
            c->arena_size = sz;
        }
    }
    const size_t off = c->arena_used;
    c->arena_used += need;
    return off;
}

void Ctx::h2d(void *d_dst, const void *h_src, size_t bytes)
{
    if (!bytes) return;
    const size_t off = arena_take(this, bytes);
    memcpy(arena + off, h_src, bytes);
    BMH_HIP(hipMemcpyAsync(d_dst, arena + off, bytes, hipMemcpyHostToDevice, stream));
}

void Ctx::d2h(void *h_dst, const void *d_src, size_t bytes)
{
    if (!bytes) return;
    const size_t off = arena_take(this, bytes);
    BMH_HIP(hipMemcpyAsync(arena + off, d_src, bytes, hipMemcpyDeviceToHost, stream));
    deferred.push_back(Deferred{h_dst, off, bytes});
}

void Ctx::sync()
{
    // spin on the stream: a blocking wait can sleep the host thread for milliseconds, and
    // the encode path synchronises a handful of times per batch
    for (;;) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) BMH_HIP(e);
        spin_pause();
    }
    for (auto &d : deferred) memcpy(d.dst, arena + d.off, d.bytes);
    deferred.clear();
    arena_used = 0;
    for (auto &p : pending) {
        float ms = 0.f;
        BMH_HIP(hipEventElapsedTime(&ms, p.a, p.b));
        KStat &k = stats[p.name];
        k.launches++;
        k.ms += ms;
        event_pool.push_back(p.a);
        event_pool.push_back(p.b);
    }
    pending.clear();
}

Batch make_batch(const uint64_t *offs, uint32_t nblocks)
{
    if (!offs || nblocks == 0) fail(BMH_EINVAL, "batch: no blocks");
    Batch b;
    b.nblocks = nblocks;
    b.offs.assign(offs, offs + nblocks + 1);
    for (uint32_t i = 0; i < nblocks; ++i) {
        if (offs[i + 1] <= offs[i])
            fail(BMH_EINVAL, "batch: empty or negative block " + std::to_string(i) +
                                 " (the reference segfaults on empty input)");
        const uint64_t n = offs[i + 1] - offs[i];
        if (n >= 0xffffffffull) fail(BMH_ERANGE, "batch: block larger than 4 GiB - 2");
        b.max_n = std::max<uint32_t>(b.max_n, (uint32_t)n);
    }
    b.total = offs[nblocks] - offs[0];
    if (offs[0] != 0) fail(BMH_EINVAL, "batch: offs[0] must be 0");
    if (b.total >= 0xffffffffull) fail(BMH_ERANGE, "batch: total must be < 4 GiB");
    if (nblocks > 65535) fail(BMH_ERANGE, "batch: at most 65535 blocks per call");
    return b;
}

uint64_t record_bound(uint64_t n) { return kRecordHeader + 320 + n + 16; }

static void encode_blocks_one_(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_out, uint64_t out_cap,
                               uint64_t *rec_offs, OffsetChain *chain, int sub, bool spec);

// Device batch encode -> records at d_out; fills rec_offs (nblocks + 1). An exception can leave a
// status bit set on the device (k_huff_build sets it before the read-back): the status tag is
// cleared then, so the next batch of the same layout zeroes the word again.
static void encode_blocks_one(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_out, uint64_t out_cap,
                              uint64_t *rec_offs, OffsetChain *chain, int sub, bool spec = false)
{
    try {
        encode_blocks_one_(c, d_in, bt, d_out, out_cap, rec_offs, chain, sub, spec);
    } catch (...) {
        c->ws_tag[WS_STATUS] = 0;
        throw;
    }
}

static void encode_blocks_one_(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_out, uint64_t out_cap,
                               uint64_t *rec_offs, OffsetChain *chain, int sub, bool spec)
{
    // BWT -> MTF (+ histograms) -> code books, record offsets and headers -> bit pack, all
    // on the context stream; the host waits on the BWT's list counters, and once at the end
    // (spec: not even on the list counters, Ctx::spec_lists)
    const uint32_t nb = bt.nblocks;
    uint8_t *d_L = (uint8_t *)c->get(WS_L, bt.total);
    uint8_t *d_mtf = (uint8_t *)c->get(WS_MTF, bt.total);
    {
        WallPhase w(c, "bwt");
        c->spec_lists = spec && !chain;
        c->spec_pending = false;
        try {
            bwt_batch(c, d_in, bt, d_L, nullptr);
        } catch (...) {
            c->spec_lists = false;
            throw;
        }
        c->spec_lists = false;
    }
    {
        WallPhase w(c, "mtf");
        c->mtf_dense = spec;
        mtf_batch(c, d_L, bt, d_mtf, nullptr, nullptr);
        c->mtf_dense = false;
    }
    WallPhase wt(c, "huffman+pack");
    const uint32_t *d_prim = (const uint32_t *)c->get(WS_PRIMARY, nb * 4 + 64);
    const uint32_t *d_freq = (const uint32_t *)c->get(WS_FREQ, (size_t)nb * 256 * 4);
    const uint32_t *d_first = (const uint32_t *)c->get(WS_FIRST, (size_t)nb * 256 * 4);
    DevTable *d_tabs = (DevTable *)c->get(WS_TABLES, nb * sizeof(DevTable));
    // record offsets [0, nb] | the batch's status word (k_rec_offs) | payload offsets
    uint64_t *d_roffs = (uint64_t *)c->get(WS_ROFFS, (size_t)(2 * nb + 2) * 8 + 64);
    uint64_t *d_pay_offs = d_roffs + nb + 2;
    uint8_t *d_misc = (uint8_t *)c->get(WS_STATUS, (size_t)(nb + 1) * 8 + 64);
    uint32_t *d_status = (uint32_t *)d_misc;
    uint64_t *d_boffs = (uint64_t *)(d_misc + 64);
    // status word zero and block offsets: set when the layout changes (get() clears the tag on
    // reallocation), and the status word cleared again after an error is read below
    const uint64_t sig = layout_sig(7, bt.offs, 0);
    if (c->ws_tag[WS_STATUS] != sig) {
        BMH_HIP(hipMemsetAsync(d_status, 0, 4, c->stream));
        c->h2d(d_boffs, bt.offs.data(), (nb + 1) * 8);
        c->ws_tag[WS_STATUS] = sig;
    }
    codebook_batch(c, bt, d_boffs, d_freq, d_first, d_prim, d_tabs, d_roffs, d_pay_offs, d_out, out_cap, d_status, chain,
                   sub);
    const uint16_t *d_chist = (const uint16_t *)c->get(WS_PACK_HIST, 64);  // written by mtf_batch
    pack_batch_dev(c, d_mtf, bt, d_tabs, d_pay_offs, d_out, d_status, d_chist);
    std::vector<uint64_t> &ro = c->roffs_host;  // offsets and status in one copy
    ro.resize(nb + 2);
    c->d2h(ro.data(), d_roffs, (nb + 2) * 8);
    c->sync();
    memcpy(rec_offs, ro.data(), (nb + 1) * 8);
    const uint32_t st = (uint32_t)ro[nb + 1];
    if (st) {  // keep the status word zero for the next batch
        BMH_HIP(hipMemsetAsync(d_status, 0, 4, c->stream));
        c->sync();
    }
    if (c->spec_pending) {
        c->spec_pending = false;
        if (!bwt_spec_ok(c)) {  // list work was left: the batch again, waiting on the counters
            ++c->spec_fallbacks;
            encode_blocks_one(c, d_in, bt, d_out, out_cap, rec_offs, chain, sub, false);
            return;
        }
    }
    if (st & kStatusCapacity) fail(BMH_ERANGE, "encode: output capacity too small");
    if (st & kStatusEmpty) fail(BMH_EINVAL, "huffman: empty histogram (the reference segfaults on empty input)");
    if (st & kStatusCodeLen) fail(BMH_ERANGE, "huffman: code longer than 64 bits");
    if (st & kStatusPrimary) fail(BMH_EHIP, "bwt: internal error (primary index not produced)");
}

// Streams and hardware queues: the device exposes 4 hardware queues per process
// (GPU_MAX_HW_QUEUES); HIP gives each of the first 4 streams its own and makes later ones share
// the least-used queue, and a stream that shares a queue serialises with the other's work. So a
// context creates exactly 4 streams, once, and gives them roles that are never busy together:
//   A = the context stream = pipeline 0        C = pipeline 2 = the H2D copy stream
//   B = pipeline 1                             D = the D2H copy stream
// Device-resident batches run up to 3 pipelines (A, B, C); the host-buffer path runs 2 (A, B)
// next to its copies (C, D). Streams made on demand instead put a third pipeline on pipeline
// 0's queue when the copy streams came first (Calgary 4.4 -> 7.3 ms), or the D2H copies behind a
// pipeline when it came first (PCIe-inclusive 30 -> 47-59 ms per GiB); per-call streams paid a
// queue set-up each call (Calgary 8.5 ms). Pipelines past 3 (BMH_OPT_PIPELINES) get streams of their
// own and share queues.
static Ctx *new_sub(Ctx *c, hipStream_t borrowed)
{
    Ctx *x = new bmh_ctx();
    x->device = c->device;
    x->cus = c->cus;
    if (borrowed) {
        x->stream = borrowed;
        x->own_stream = false;
    } else if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) {
        delete x;
        fail(BMH_EHIP, "stream creation failed");
    }
    c->subs.push_back(x);
    return x;
}

static void create_streams(Ctx *c)
{
    new_sub(c, c->stream);  // pipeline 0 on A
    new_sub(c, nullptr);    // pipeline 1: B
    BMH_HIP(hipStreamCreateWithFlags(&c->s_h2d, hipStreamNonBlocking));  // C
    new_sub(c, c->s_h2d);   // pipeline 2 on C
    BMH_HIP(hipStreamCreateWithFlags(&c->s_d2h, hipStreamNonBlocking));  // D
    c->aux_stream = c->s_d2h;
    for (Ctx *x : c->subs) x->aux_stream = c->s_d2h;
}

Ctx *aux_ctx(Ctx *c)
{
    if (!c->aux) {
        Ctx *x = new bmh_ctx();
        x->device = c->device;
        x->cus = c->cus;
        x->stream = c->aux_stream ? c->aux_stream : c->stream;
        x->own_stream = false;
        c->aux = x;
    }
    c->aux->timing = c->timing;
    c->aux->opt = c->opt;
    return c->aux;
}

// A persistent host thread running one task at a time (encode_blocks' sub-pipelines).
struct Ctx::Worker {
    std::mutex m;
    std::condition_variable cv;
    std::function<void()> task;
    bool busy = false, quit = false;
    std::thread th;
    Worker()
        : th([this] {
              std::unique_lock<std::mutex> lk(m);
              for (;;) {
                  cv.wait(lk, [&] { return busy || quit; });
                  if (!busy) return;  // quit with nothing queued
                  auto fn = std::move(task);
                  lk.unlock();
                  fn();  // (catches its own errors)
                  lk.lock();
                  busy = false;
                  cv.notify_all();
              }
          })
    {
    }
    void run(std::function<void()> fn)
    {
        std::lock_guard<std::mutex> lk(m);
        task = std::move(fn);
        busy = true;
        cv.notify_all();
    }
    void wait()
    {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return !busy; });
    }
    ~Worker()
    {
        {
            std::lock_guard<std::mutex> lk(m);
            quit = true;
            cv.notify_all();
        }
        th.join();
    }
};

static Ctx *sub_ctx(Ctx *c, size_t i)
{
    // a fourth pipeline runs on stream D, the D2H / run-path side stream, which
    // device-resident batches past the run screen leave idle; later ones get streams of their own
    while (c->subs.size() <= i) new_sub(c, c->subs.size() == 3 ? c->s_d2h : nullptr)->aux_stream = c->s_d2h;
    Ctx *x = c->subs[i];
    x->timing = c->timing;
    x->opt = c->opt;
    return x;
}

// Default sub-pipelines: 3 for batches under 128 MiB of at least 12 blocks (their list rounds leave the GPU idle
// between host waits, so a third pipeline fills it: Calgary 5.9 -> 5.1 ms, Zipf 100 MB at 1 MiB
// blocks 11.8 -> 11.1-11.4 ms), 2 above (the 128 MiB text batch, the 256 MiB streamed batches
// and the 1 GiB headline measured equal or slower with 3; 4+ exceed the device's 4 hardware
// queues and serialise: Calgary 7.9 ms).
static int stream_count(Ctx *c, uint64_t total, uint32_t nblocks)
{
    const int v = (int)std::min<uint64_t>(c->opt.pipelines, 16);  // BMH_OPT_PIPELINES
    // Batches past the run screen (> 64 MiB) leave stream D idle: four pipelines, one per
    // hardware queue (1 GiB random 11.08-11.20 -> 10.96-10.98 ms; Zipf 100 MB at 1 MiB blocks
    // 10.94 -> 10.65 ms), from 8 blocks on (round 6: 128 MB of Zipf in 8 x 16 MiB blocks
    // 16.32-16.40 ms on two, 15.61-15.77 on four; three split them 3 / 3 / 2: 17.2-17.4 ms).
    if (v > 0) return v;
    if (nblocks >= 8 && total > (64ull << 20)) return 4;
    return total < (128ull << 20) && nblocks >= 12 ? 3 : 2;
}

static uint32_t pipelines_for(Ctx *c, uint64_t total, uint32_t nb, int max_pipes);
constexpr uint64_t kDenseProbeMin = 32ull << 20, kDenseProbeMax = 256ull << 20;

// The batch is cut into S runs of whole blocks (balanced by bytes), each encoded on its own
// stream by its own host thread, so that one run's bandwidth-bound kernels overlap another's
// LDS-bound ones. Records land back to back in block order: each run's offset scan starts
// from the previous run's end (OffsetChain).
void encode_blocks(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_out, uint64_t out_cap,
                   uint64_t *rec_offs, int max_pipes)
{
    const uint32_t nb = bt.nblocks;
    int S = (int)pipelines_for(c, bt.total, nb, max_pipes);
    // dense batches of 32-256 MiB run on one pipeline (dense_batch): on random data four
    // pipelines only contend (128 / 256 MiB of 4 MiB blocks: 1.99 / 3.49 ms against 1.77 / 3.14
    // on one; 1 GiB: equal), while text keeps them for its host-synchronised list rounds
    // (Zipf 128 MB at 4 MiB blocks: 14.1 ms on four, 16.8 on one)
    // (and, on one pipeline, run their one expected list round speculatively: Ctx::spec_lists)
    bool spec = false;
    if (S > 1 && !c->opt.pipelines && bt.total >= kDenseProbeMin && bt.total <= kDenseProbeMax &&
        dense_batch(c, d_in, bt)) {
        S = 1;
        spec = true;
    }
    c->pre_sig = spec ? c->pre_sig : 0;  // a prologue dense_batch launched for one pipeline, unused
    if (c->opt.one_pipeline) S = 1;       // (a timing pass: the decisions above stand)
    c->last_pipelines = (uint32_t)std::max(S, 1);
    if (S <= 1) {
        encode_blocks_one(c, d_in, bt, d_out, out_cap, rec_offs, nullptr, 0, spec);
        return;
    }
    std::vector<uint32_t> cut(S + 1, nb);
    cut[0] = 0;
    for (int s = 1; s < S; ++s) {
        const uint64_t target = bt.total * s / S;
        uint32_t b = cut[s - 1] + 1;
        while (b < nb - (uint32_t)(S - s) && bt.offs[b] < target) ++b;
        cut[s] = b;
    }
    OffsetChain chain;
    chain.ev.resize(S);
    chain.d_end.resize(S, nullptr);
    std::vector<Ctx *> cs(S);
    for (int s = 0; s < S; ++s) {
        cs[s] = sub_ctx(c, s);
        cs[s]->screen_total = bt.total;  // the run screen follows the whole batch (bwt_runs.hip)
        BMH_HIP(hipEventCreateWithFlags(&chain.ev[s], hipEventDisableTiming));
    }
    std::vector<std::vector<uint64_t>> ro(S);
    std::vector<bmh_status> st(S, BMH_OK);
    std::vector<std::string> err(S);
    auto run = [&](int s) {
        try {
            BMH_HIP(hipSetDevice(c->device));
            Batch sb;
            sb.nblocks = cut[s + 1] - cut[s];
            sb.offs.resize(sb.nblocks + 1);
            for (uint32_t i = 0; i <= sb.nblocks; ++i) sb.offs[i] = bt.offs[cut[s] + i] - bt.offs[cut[s]];
            sb.total = sb.offs[sb.nblocks];
            for (uint32_t i = 0; i < sb.nblocks; ++i)
                sb.max_n = std::max<uint32_t>(sb.max_n, (uint32_t)(sb.offs[i + 1] - sb.offs[i]));
            ro[s].resize(sb.nblocks + 1);
            encode_blocks_one(cs[s], d_in + bt.offs[cut[s]], sb, d_out, out_cap, ro[s].data(), &chain, s);
        } catch (const Error &e) {
            st[s] = e.status;
            err[s] = e.what();
        } catch (const std::bad_alloc &) {
            st[s] = BMH_ENOMEM;
            err[s] = "host allocation failed";
        } catch (const std::exception &e) {
            st[s] = BMH_EHIP;
            err[s] = e.what();
        }
        if (st[s] != BMH_OK) {
            std::lock_guard<std::mutex> lk(chain.m);
            chain.failed = true;
            chain.cv.notify_all();
        }
    };
    while (c->workers.size() < (size_t)S - 1) c->workers.emplace_back(new Ctx::Worker());
    for (int s = 1; s < S; ++s) c->workers[s - 1]->run([&run, s] { run(s); });
    run(0);
    for (int s = 1; s < S; ++s) c->workers[s - 1]->wait();
    for (int s = 0; s < S; ++s) (void)hipEventDestroy(chain.ev[s]);
    if (c->timing)  // fold the sub-pipelines' kernel times into the parent's statistics
        for (int s = 0; s < S; ++s) {
            for (auto &kv : cs[s]->stats) {
                c->stats[kv.first].launches += kv.second.launches;
                c->stats[kv.first].ms += kv.second.ms;
            }
            cs[s]->stats.clear();
        }
    for (int s = 0; s < S; ++s)
        if (st[s] != BMH_OK) fail(st[s], err[s]);
    for (int s = 0; s < S; ++s)
        for (uint32_t i = 0; i < cut[s + 1] - cut[s]; ++i) rec_offs[cut[s] + i] = ro[s][i];
    rec_offs[nb] = ro[S - 1][cut[S] - cut[S - 1]];
}

// Pipelines (streams) encode_blocks runs a device-resident batch of this shape on.
static uint32_t pipelines_for(Ctx *c, uint64_t total, uint32_t nb, int max_pipes)
{
    const uint32_t S = std::min<uint32_t>(std::min<uint32_t>((uint32_t)stream_count(c, total, nb), (uint32_t)max_pipes),
                                          nb / 2);
    return S <= 1 ? 1u : S;
}

static uint64_t max_batch_bytes(const Ctx *c)
{
    const uint64_t v = c->opt.max_batch;  // BMH_OPT_MAX_BATCH
    return v ? v : (1ull << 30);
}

static uint64_t stream_batch_bytes(const Ctx *c)
{
    const uint64_t v = c->opt.stream_batch;  // BMH_OPT_STREAM_BATCH
    return std::min<uint64_t>(v ? v : (256ull << 20), max_batch_bytes(c));
}

// memcpy on up to `nt` threads (pageable <-> pinned staging copies are CPU-bound)
static void par_memcpy(uint8_t *dst, const uint8_t *src, uint64_t bytes, unsigned nt)
{
    const uint64_t kMin = 8ull << 20;
    nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nt, bytes / kMin));
    if (nt <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> th;
    const uint64_t part = (bytes / nt + 4095) & ~4095ull;
    for (unsigned t = 0; t < nt; ++t) {
        const uint64_t o = std::min<uint64_t>(bytes, part * t), e = std::min<uint64_t>(bytes, o + part);
        if (e > o) th.emplace_back([=] { memcpy(dst + o, src + o, e - o); });
    }
    for (auto &x : th) x.join();
}

// CPUs this process may run on: its affinity set, capped by the cgroup CPU quota (cgroup v2
// cpu.max, else v1 cfs_quota_us / cfs_period_us, rounded up). hardware_concurrency() reports the
// whole machine: 256 on the driver's boxes, whose cgroup grants 16 (bench.py's cpu_baseline
// learned the same: 256 processes under that quota ran at 59 MB/s against 96 with 16).
static unsigned read_quota_cpus()
{
    long long q = -1, per = -1;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char a[32] = {0};
        if (fscanf(f, "%31s %lld", a, &per) == 2 && strcmp(a, "max") != 0) q = atoll(a);
        fclose(f);
    } else if (FILE *g = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
        if (fscanf(g, "%lld", &q) != 1) q = -1;
        fclose(g);
        if (FILE *h = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (fscanf(h, "%lld", &per) != 1) per = -1;
            fclose(h);
        }
    }
    if (q <= 0 || per <= 0) return 0;  // no quota
    return (unsigned)std::max<long long>(1, (q + per - 1) / per);
}

static unsigned host_cpus()
{
    static const unsigned v = [] {
        unsigned n = 0;
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (unsigned)CPU_COUNT(&set);
        if (n == 0) n = std::max(1u, std::thread::hardware_concurrency());
        const unsigned q = read_quota_cpus();
        return q ? std::min(n, q) : n;
    }();
    return v;
}

// Copy threads per copy site (the loader's pageable -> pinned staging copies and the writer's
// record copies run side by side): the process's CPUs divided among the contexts that stream at
// once (bmh_compress_host_multi sets Ctx::copy_share), at most 16 and at least 1. Before round 6
// every context sized its copies from hardware_concurrency(): 8 contexts started up to 128 copy
// threads a site on a box granting 16 CPUs.
static unsigned copy_threads_for(unsigned cpus, unsigned share)
{
    return std::max(1u, std::min(16u, cpus / std::max(1u, share)));
}
static unsigned copy_threads(const Ctx *c = nullptr)
{
    if (c && c->opt.copy_threads) return (unsigned)c->opt.copy_threads;  // BMH_OPT_COPY_THREADS
    return copy_threads_for(host_cpus(), c ? c->copy_share : 1u);
}

// Page-locked (hipHostMalloc'd or hipHostRegister'ed) host range that device `dev`'s DMA engines
// may read and write directly, so the streaming encoder skips its staging copies. The range is
// probed at both ends and every 64 MiB in between (a range over two pinned allocations with an
// unpinned gap fails the probe in the gap unless the gap is < 64 MiB; callers pass one
// allocation). Memory registered for another device counts only when it is portable.
static bool is_pinned(const void *p, uint64_t bytes, int dev)
{
    if (!p || bytes == 0) return false;
    const uint8_t *b = (const uint8_t *)p;
    constexpr uint64_t kStride = 64ull << 20;
    for (uint64_t off = 0;; off = std::min(off + kStride, bytes - 1)) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, b + off) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
        if (off == 0 && a.device != dev) {
            unsigned int fl = 0;
            if (hipHostGetFlags(&fl, (void *)b) != hipSuccess) {
                (void)hipGetLastError();
                return false;
            }
            if (!(fl & hipHostMallocPortable)) return false;
        }
        if (off == bytes - 1) return true;
    }
}

// Page-locked staging for the first `ns` slots, each direction only when it is used (a pinned
// caller buffer needs none) and sized to the call's largest batch: a slot grows, never shrinks,
// and is released with the context.
static void ensure_staging(Ctx *c, size_t in_bytes, size_t out_bytes, int ns)
{
    auto grow = [](uint8_t *&p, size_t &have, size_t need) {
        if (need == 0 || have >= need) return;
        if (p) BMH_HIP(hipHostFree(p));
        p = nullptr;
        have = 0;
        BMH_HIP(hipHostMalloc((void **)&p, need, hipHostMallocDefault));
        have = need;
    };
    for (int s = 0; s < ns; ++s) {
        grow(c->stage_in[s], c->stage_in_size[s], in_bytes);
        grow(c->stage_out[s], c->stage_out_size[s], out_bytes);
    }
}

// Host-buffer encode of blocks `blist` of `in` (block size bs) on one context, pipelined over
// batches through Ctx::kStageSlots staging slots (BASELINE config 5):
//   loader thread : batch k+1 pageable -> pinned (parallel memcpy), H2D on the h2d stream
//   this thread   : encode batch k (context streams), then its records D2H on the d2h stream
//   writer thread : records of batch k-1 pinned -> recs[] (parallel memcpy)
// so PCIe traffic both ways and the host copies overlap the device encode.
struct RecRef {
    const uint8_t *p = nullptr;
    uint64_t len = 0;
};

// Receives the records of consecutive entries [i0, i0 + cnt) of the block list: record j at
// src + ro[j] .. src + ro[j + 1] (pinned staging, valid only during the call; or, with a
// pinned destination, their final place).
using RecordSink = std::function<void(size_t i0, size_t cnt, const uint8_t *src, const uint64_t *ro)>;

// Pinned fast path (the caller's buffers are page-locked): `in_pinned` issues the H2D copies
// straight from the caller's input; a PinnedOut lets the D2H copies land the records at their
// final place, back to back from `at` (capacity `cap`), with no host copy at all.
struct PinnedOut {
    uint8_t *base = nullptr;
    uint64_t cap = 0, at = 0;
};

static void encode_host_blocks(Ctx *c, const uint8_t *in, uint64_t n, uint64_t bs, const std::vector<uint64_t> &blist,
                               const RecordSink &sink, bool in_pinned = false, PinnedOut *pout = nullptr)
{
    struct B {
        std::vector<uint64_t> blocks, offs;
        uint64_t cap = 0;
    };
    const uint64_t cap_batch = stream_batch_bytes(c);
    // (a halving tail of batch sizes, to shorten the ramp-down after the last H2D, measured no
    // better: every new batch layout rebuilds the encode's tables on the host)
    std::vector<B> batches;
    std::vector<size_t> first;  // block-list index of each batch's first block
    for (size_t i = 0; i < blist.size();) {
        first.push_back(i);
        B bt;
        bt.offs.push_back(0);
        size_t j = i;
        while (j < blist.size()) {
            const uint64_t len = std::min(bs, n - blist[j] * bs);
            if (j > i && bt.offs.back() + len > cap_batch) break;
            bt.blocks.push_back(blist[j]);
            bt.offs.push_back(bt.offs.back() + len);
            bt.cap += record_bound(len);
            ++j;
        }
        batches.push_back(std::move(bt));
        i = j;
    }
    const size_t K = batches.size();
    if (K == 0) return;
    uint64_t max_in = 0, max_cap = 0;
    for (auto &bt : batches) {
        max_in = std::max(max_in, bt.offs.back());
        max_cap = std::max(max_cap, bt.cap);
    }
    std::vector<uint8_t *> dst(K, nullptr);  // pinned destination of each batch's records
    // kStageSlots batches in flight: the H2D of batch k waits only for the encode of k - NS
    constexpr int NS = Ctx::kStageSlots;
    const int ns = (int)std::min<size_t>(NS, K);  // slots k % NS for k < K
    ensure_staging(c, in_pinned ? 0 : max_in, pout ? 0 : max_cap, ns);
    const Slot ws_in[NS] = {WS_IN, WS_IN2, WS_IN3}, ws_out[NS] = {WS_OUT, WS_OUT2, WS_OUT3};
    uint8_t *d_in[NS] = {}, *d_out[NS] = {};
    for (int s = 0; s < ns; ++s) {
        d_in[s] = (uint8_t *)c->get(ws_in[s], max_in);
        d_out[s] = (uint8_t *)c->get(ws_out[s], max_cap);
    }
    hipEvent_t ev_h2d[NS], ev_d2h[NS];
    for (int s = 0; s < NS; ++s) {
        BMH_HIP(hipEventCreateWithFlags(&ev_h2d[s], hipEventDisableTiming));
        BMH_HIP(hipEventCreateWithFlags(&ev_d2h[s], hipEventDisableTiming));
    }
    const unsigned nt = copy_threads(c);
    std::mutex m;
    std::condition_variable cv;
    size_t loaded = 0;    // batches whose H2D is issued
    size_t encoded = 0;   // batches whose encode finished (their input slot is free)
    size_t written = 0;   // batches whose records left their output slot
    size_t d2h_issued = 0;
    bool abort_ = false;
    std::vector<std::vector<uint64_t>> ro(K);
    std::string err;
    bmh_status st = BMH_OK;
    auto wait_for = [&](auto pred) {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return abort_ || pred(); });
        return !abort_;
    };
    auto bump = [&](size_t &ctr) {
        std::lock_guard<std::mutex> lk(m);
        ++ctr;
        cv.notify_all();
    };
    auto fail_all = [&](bmh_status s, const std::string &e) {
        std::lock_guard<std::mutex> lk(m);
        if (st == BMH_OK) {
            st = s;
            err = e;
        }
        abort_ = true;
        cv.notify_all();
    };
    auto guarded = [&](auto fn) {
        return [&, fn] {
            try {
                BMH_HIP(hipSetDevice(c->device));
                fn();
            } catch (const Error &e) {
                fail_all(e.status, e.what());
            } catch (const std::bad_alloc &) {
                fail_all(BMH_ENOMEM, "host allocation failed");
            } catch (const std::exception &e) {
                fail_all(BMH_EHIP, e.what());
            }
        };
    };
    std::thread loader(guarded([&] {
        for (size_t k = 0; k < K; ++k) {
            const int s = (int)(k % NS);
            if (!wait_for([&] { return encoded + NS > k; })) return;  // encode k-NS has read d_in[s]
            if (k >= (size_t)NS) BMH_HIP(hipEventSynchronize(ev_h2d[s]));  // H2D k-NS has read stage_in[s]
            const B &bt = batches[k];
            // consecutive blocks of the input are copied as one run
            for (size_t i = 0; i < bt.blocks.size();) {
                size_t j = i + 1;
                while (j < bt.blocks.size() && bt.blocks[j] == bt.blocks[j - 1] + 1) ++j;
                if (in_pinned)
                    BMH_HIP(hipMemcpyAsync(d_in[s] + bt.offs[i], in + bt.blocks[i] * bs, bt.offs[j] - bt.offs[i],
                                           hipMemcpyHostToDevice, c->s_h2d));
                else
                    par_memcpy(c->stage_in[s] + bt.offs[i], in + bt.blocks[i] * bs, bt.offs[j] - bt.offs[i], nt);
                i = j;
            }
            if (!in_pinned)
                BMH_HIP(hipMemcpyAsync(d_in[s], c->stage_in[s], bt.offs.back(), hipMemcpyHostToDevice, c->s_h2d));
            BMH_HIP(hipEventRecord(ev_h2d[s], c->s_h2d));
            bump(loaded);
        }
    }));
    std::thread writer(guarded([&] {
        for (size_t k = 0; k < K; ++k) {
            const int s = (int)(k % NS);
            if (!wait_for([&] { return d2h_issued > k; })) return;
            BMH_HIP(hipEventSynchronize(ev_d2h[s]));
            sink(first[k], batches[k].blocks.size(), pout ? dst[k] : c->stage_out[s], ro[k].data());
            bump(written);
        }
    }));
    guarded([&] {
        for (size_t k = 0; k < K; ++k) {
            const int s = (int)(k % NS);
            if (!wait_for([&] { return loaded > k; })) return;
            BMH_HIP(hipEventSynchronize(ev_h2d[s]));
            if (k >= (size_t)NS) BMH_HIP(hipEventSynchronize(ev_d2h[s]));  // D2H k-NS has read d_out[s]
            const B &bt = batches[k];
            Batch b = make_batch(bt.offs.data(), (uint32_t)bt.blocks.size());
            ro[k].resize(bt.blocks.size() + 1);
            encode_blocks(c, d_in[s], b, d_out[s], bt.cap, ro[k].data(), 2);  // pipelines A, B (create_streams)
            bump(encoded);
            if (!wait_for([&] { return written + NS > k; })) return;  // the writer is done with stage_out[s]
            const uint64_t bytes = ro[k][bt.blocks.size()];
            uint8_t *to = c->stage_out[s];
            if (pout) {
                if (pout->at + bytes > pout->cap) fail(BMH_ERANGE, "compress: output capacity too small");
                to = dst[k] = pout->base + pout->at;
                pout->at += bytes;
            }
            BMH_HIP(hipMemcpyAsync(to, d_out[s], bytes, hipMemcpyDeviceToHost, c->s_d2h));
            BMH_HIP(hipEventRecord(ev_d2h[s], c->s_d2h));
            bump(d2h_issued);
        }
    })();
    loader.join();
    writer.join();
    for (int s = 0; s < NS; ++s) {
        (void)hipEventDestroy(ev_h2d[s]);
        (void)hipEventDestroy(ev_d2h[s]);
    }
    if (st != BMH_OK) fail(st, err);
}

static void assemble(uint64_t n, uint64_t bs, uint64_t nblocks, const std::vector<RecRef> &recs, uint8_t *out,
                     uint64_t out_cap, uint64_t *out_len)
{
    uint64_t total = 0;
    if (nblocks == 1) {
        total = recs[0].len;
        if (total > out_cap) fail(BMH_ERANGE, "compress: output capacity too small");
        par_memcpy(out, recs[0].p, total, copy_threads());
    } else {
        total = 32 + 8 * nblocks;
        for (auto &r : recs) total += r.len;
        if (total > out_cap) fail(BMH_ERANGE, "compress: output capacity too small");
        memcpy(out, kContainerMagic, 8);
        put_u64(out + 8, bs);
        put_u64(out + 16, nblocks);
        put_u64(out + 24, n);
        std::vector<uint64_t> at(nblocks);
        uint64_t o = 32 + 8 * nblocks;
        for (uint64_t b = 0; b < nblocks; ++b) {
            put_u64(out + 32 + 8 * b, recs[b].len);
            at[b] = o;
            o += recs[b].len;
        }
        // the records in parallel: contiguous runs of blocks per thread
        const unsigned nt = copy_threads();
        std::vector<std::thread> th;
        const uint64_t per = (nblocks + nt - 1) / nt;
        for (uint64_t b0 = 0; b0 < nblocks; b0 += per)
            th.emplace_back([&, b0] {
                for (uint64_t b = b0; b < std::min(nblocks, b0 + per); ++b) memcpy(out + at[b], recs[b].p, recs[b].len);
            });
        for (auto &x : th) x.join();
    }
    *out_len = total;
}

// Checked builds: every kernel translation unit registers the reader of its violation table.
static std::vector<uint32_t (*)(uint32_t)> &check_readers()
{
    static std::vector<uint32_t (*)(uint32_t)> v;
    return v;
}
void check_register(uint32_t (*reader)(uint32_t kind)) { check_readers().push_back(reader); }

}  // namespace bmh

using namespace bmh;

#define API_BEGIN try {
#define API_END                                      \
    }                                                \
    catch (const Error &e)                           \
    {                                                \
        set_last_error(e.what());                    \
        return e.status;                             \
    }                                                \
    catch (const std::bad_alloc &)                   \
    {                                                \
        set_last_error("host allocation failed");    \
        return BMH_ENOMEM;                           \
    }                                                \
    catch (const std::exception &e)                  \
    {                                                \
        set_last_error(e.what());                    \
        return BMH_EINVAL;                           \
    }                                                \
    set_last_error("");                              \
    return BMH_OK;

static void use_device(bmh_ctx *c)
{
    if (!c) fail(BMH_EINVAL, "null context");
    BMH_HIP(hipSetDevice(c->device));
}

extern "C" {

const char *bmh_version(void) { return "bmh 0.1.0 (gfx950)"; }

int64_t bmh_check_violations(bmh_ctx *c, uint32_t kind)
{
#ifdef BMH_CHECK
    if (!c || kind >= kCheckKinds || hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return -2;
    if (check_readers().empty()) return -2;
    int64_t tot = 0;
    for (auto *r : check_readers()) {
        const uint32_t v = r(kind);
        if (v == 0xffffffffu) return -2;
        tot += v;
    }
    return tot;
#else
    (void)c;
    (void)kind;
    return -1;
#endif
}

const char *bmh_status_str(int s)
{
    switch (s) {
    case BMH_OK: return "ok";
    case BMH_EINVAL: return "invalid argument";
    case BMH_ENOMEM: return "out of memory";
    case BMH_EHIP: return "HIP runtime error";
    case BMH_ERANGE: return "size limit exceeded";
    case BMH_ECORRUPT: return "corrupt input";
    case BMH_ENODEV: return "no gfx950 device";
    default: return "unknown status";
    }
}

const char *bmh_last_error(void) { return g_last_error.c_str(); }

int bmh_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

bmh_status bmh_ctx_create(int device, bmh_ctx **out)
{
    API_BEGIN
    if (!out) fail(BMH_EINVAL, "null out pointer");
    *out = nullptr;
    const int n = bmh_device_count();
    if (device < 0 || device >= n) fail(BMH_ENODEV, "no HIP device " + std::to_string(device));
    hipDeviceProp_t prop;
    BMH_HIP(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        fail(BMH_ENODEV, std::string("device is ") + prop.gcnArchName + ", libbmh is built for gfx950");
    BMH_HIP(hipSetDevice(device));
    bmh_ctx *c = new bmh_ctx();
    c->device = device;
    c->cus = std::max(1, prop.multiProcessorCount);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        fail(BMH_EHIP, "stream creation failed");
    }
    try {
        create_streams(c);
    } catch (...) {
        bmh_ctx_destroy(c);
        throw;
    }
    *out = c;
    API_END
}

void bmh_ctx_destroy(bmh_ctx *c)
{
    if (!c) return;
    c->workers.clear();  // (idle between calls: each joins its thread)
    for (auto *x : c->subs) bmh_ctx_destroy(static_cast<bmh_ctx *>(x));
    c->subs.clear();
    if (c->aux) bmh_ctx_destroy(static_cast<bmh_ctx *>(c->aux));
    c->aux = nullptr;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->arena) (void)hipHostFree(c->arena);
    if (c->probe_host) (void)hipHostFree(c->probe_host);
    if (c->probe_ev) (void)hipEventDestroy(c->probe_ev);
    if (c->dbl_cnt_host) (void)hipHostFree(c->dbl_cnt_host);
    for (auto e : c->dbl_ev)
        if (e) (void)hipEventDestroy(e);
    for (int s = 0; s < WS_COUNT_; ++s)
        if (c->ws[s]) (void)hipFree(c->ws[s]);
    if (c->pinned) (void)hipHostFree(c->pinned);
    for (int s = 0; s < Ctx::kStageSlots; ++s) {
        if (c->stage_in[s]) (void)hipHostFree(c->stage_in[s]);
        if (c->stage_out[s]) (void)hipHostFree(c->stage_out[s]);
    }
    if (c->s_h2d) (void)hipStreamDestroy(c->s_h2d);
    if (c->s_d2h) (void)hipStreamDestroy(c->s_d2h);
    for (auto &p : c->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void *bmh_ctx_stream(bmh_ctx *c) { return c ? (void *)c->stream : nullptr; }

bmh_status bmh_dev_alloc(bmh_ctx *c, uint64_t bytes, void **d_ptr)
{
    API_BEGIN
    use_device(c);
    if (!d_ptr) fail(BMH_EINVAL, "null out pointer");
    if (hipMalloc(d_ptr, bytes ? bytes : 1) != hipSuccess) {
        (void)hipGetLastError();
        fail(BMH_ENOMEM, "hipMalloc failed");
    }
    API_END
}

bmh_status bmh_dev_free(bmh_ctx *c, void *d_ptr)
{
    API_BEGIN
    use_device(c);
    BMH_HIP(hipStreamSynchronize(c->stream));
    BMH_HIP(hipFree(d_ptr));
    API_END
}

bmh_status bmh_host_alloc(bmh_ctx *c, uint64_t bytes, void **h_ptr)
{
    API_BEGIN
    use_device(c);
    if (!h_ptr) fail(BMH_EINVAL, "null argument");
    *h_ptr = nullptr;
    if (hipHostMalloc(h_ptr, std::max<uint64_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        *h_ptr = nullptr;
        fail(BMH_ENOMEM, "pinned host allocation of " + std::to_string(bytes) + " bytes failed");
    }
    API_END
}

bmh_status bmh_host_free(bmh_ctx *c, void *h_ptr)
{
    API_BEGIN
    if (c) use_device(c);
    if (h_ptr) BMH_HIP(hipHostFree(h_ptr));
    API_END
}

bmh_status bmh_memcpy_h2d(bmh_ctx *c, void *d_dst, const void *h_src, uint64_t bytes)
{
    API_BEGIN
    use_device(c);
    BMH_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, c->stream));
    c->sync();
    API_END
}

bmh_status bmh_memcpy_d2h(bmh_ctx *c, void *h_dst, const void *d_src, uint64_t bytes)
{
    API_BEGIN
    use_device(c);
    BMH_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    API_END
}

bmh_status bmh_bwt_dev(bmh_ctx *c, const uint8_t *d_in, const uint64_t *offs, uint32_t nblocks, uint8_t *d_L,
                       uint64_t *h_primary)
{
    API_BEGIN
    use_device(c);
    if (!d_in || !d_L || !h_primary) fail(BMH_EINVAL, "null buffer");
    Batch bt = make_batch(offs, nblocks);
    bwt_batch(c, d_in, bt, d_L, h_primary);
    API_END
}

bmh_status bmh_mtf_dev(bmh_ctx *c, const uint8_t *d_L, const uint64_t *offs, uint32_t nblocks, uint8_t *d_mtf,
                       uint64_t *h_freq, uint64_t *h_first)
{
    API_BEGIN
    use_device(c);
    if (!d_L || !d_mtf) fail(BMH_EINVAL, "null buffer");
    Batch bt = make_batch(offs, nblocks);
    std::vector<uint32_t> f((size_t)nblocks * 256), fi((size_t)nblocks * 256);
    mtf_batch(c, d_L, bt, d_mtf, f.data(), fi.data());
    for (size_t i = 0; i < f.size(); ++i) {
        if (h_freq) h_freq[i] = f[i];
        if (h_first) h_first[i] = fi[i] == 0xffffffffu ? UINT64_MAX : fi[i];
    }
    API_END
}

bmh_status bmh_histogram_dev(bmh_ctx *c, const uint8_t *d_in, const uint64_t *offs, uint32_t nblocks, uint64_t *h_freq,
                             uint64_t *h_first)
{
    API_BEGIN
    use_device(c);
    if (!d_in || !h_freq) fail(BMH_EINVAL, "null argument");
    Batch bt = make_batch(offs, nblocks);
    std::vector<uint32_t> f((size_t)nblocks * 256), fi((size_t)nblocks * 256);
    histogram_batch(c, d_in, bt, f.data(), fi.data());
    for (size_t i = 0; i < f.size(); ++i) {
        h_freq[i] = f[i];
        if (h_first) h_first[i] = fi[i] == 0xffffffffu ? UINT64_MAX : fi[i];
    }
    API_END
}

bmh_status bmh_huffman_build(const uint64_t freq[256], const uint64_t first[256], bmh_code_table *out)
{
    API_BEGIN
    if (!freq || !first || !out) fail(BMH_EINVAL, "null argument");
    huffman_build(freq, first, out);
    API_END
}

bmh_status bmh_huffman_build_sized(const uint64_t freq[256], const uint64_t first[256], uint64_t n,
                                   bmh_code_table *out)
{
    API_BEGIN
    if (!freq || !first || !out) fail(BMH_EINVAL, "null argument");
    huffman_build(freq, first, out, n);
    API_END
}

int bmh_node_ranks(uint64_t n, uint32_t L, uint16_t *rank)
{
    if (!rank || L == 0 || L > 256) return -1;
    try {
        node_ranks(n, L, rank);
        const auto br = band_ranks(n);
        return br && br->off[L] != kModelOrder ? 1 : 0;
    } catch (...) {
        return -1;
    }
}

uint32_t bmh_encode_pipelines(bmh_ctx *c, uint64_t total, uint32_t nblocks)
{
    if (!c || nblocks == 0) return 0;
    return pipelines_for(c, total, nblocks, 16);  // as bmh_encode_blocks_dev, before its data probe
}

uint32_t bmh_ctx_last_pipelines(bmh_ctx *c) { return c ? c->last_pipelines : 0u; }
uint32_t bmh_host_cpus(void) { return host_cpus(); }
uint32_t bmh_copy_threads(uint32_t nctx, uint32_t cpus) { return copy_threads_for(cpus ? cpus : host_cpus(), nctx); }
uint32_t bmh_ctx_spec_fallbacks(bmh_ctx *c) { return c ? c->spec_fallbacks : 0u; }

uint64_t bmh_payload_bytes(const bmh_code_table *t, const uint64_t freq[256])
{
    return (t && freq) ? payload_bytes(t, freq) : 0;
}

bmh_status bmh_pack_dev(bmh_ctx *c, const uint8_t *d_mtf, const uint64_t *offs, uint32_t nblocks,
                        const bmh_code_table *tables, uint8_t *d_out, uint64_t out_cap, const uint64_t *pay_offs,
                        uint64_t *out_bytes)
{
    API_BEGIN
    use_device(c);
    if (!d_mtf || !tables || !d_out) fail(BMH_EINVAL, "null argument");
    Batch bt = make_batch(offs, nblocks);
    pack_batch(c, d_mtf, bt, tables, d_out, out_cap, pay_offs, out_bytes);
    API_END
}

bmh_status bmh_encode_blocks_dev(bmh_ctx *c, const uint8_t *d_in, const uint64_t *offs, uint32_t nblocks,
                                 uint8_t *d_out, uint64_t out_cap, uint64_t *h_rec_offs)
{
    API_BEGIN
    use_device(c);
    if (!d_in || !d_out || !h_rec_offs) fail(BMH_EINVAL, "null argument");
    Batch bt = make_batch(offs, nblocks);
    encode_blocks(c, d_in, bt, d_out, out_cap, h_rec_offs, 16);
    API_END
}

uint64_t bmh_record_bound(uint64_t n) { return record_bound(n); }

uint64_t bmh_compress_bound(uint64_t n, uint64_t bs)
{
    if (bs == 0 || bs >= n) return record_bound(n);
    const uint64_t nb = (n + bs - 1) / bs;
    return 32 + 8 * nb + nb * (kRecordHeader + 320 + 16) + n;
}

bmh_status bmh_compress_host(bmh_ctx *c, const uint8_t *in, uint64_t n, uint64_t block_size, uint8_t *out,
                             uint64_t out_cap, uint64_t *out_len)
{
    bmh_ctx *cs[1] = {c};
    return bmh_compress_host_multi(cs, 1, in, n, block_size, out, out_cap, out_len);
}

bmh_status bmh_compress_host_multi(bmh_ctx **ctxs, uint32_t nctx, const uint8_t *in, uint64_t n, uint64_t block_size,
                                   uint8_t *out, uint64_t out_cap, uint64_t *out_len)
{
    API_BEGIN
    if (!ctxs || nctx == 0 || !in || !out || !out_len) fail(BMH_EINVAL, "null argument");
    // each context is driven by its own host thread: a context listed twice would be used by
    // two threads at once (several contexts may share one device: they time-share it)
    for (uint32_t g = 0; g < nctx; ++g) {
        if (!ctxs[g]) fail(BMH_EINVAL, "null context in the list");
        for (uint32_t h = 0; h < g; ++h)
            if (ctxs[h] == ctxs[g]) fail(BMH_EINVAL, "context listed twice");
    }
    if (n == 0) fail(BMH_EINVAL, "empty input (the reference segfaults on empty input)");
    const uint64_t bs = (block_size == 0 || block_size >= n) ? n : block_size;
    if (bs >= 0xffffffffull) fail(BMH_ERANGE, "block size must be < 4 GiB - 1");
    const uint64_t nblocks = (n + bs - 1) / bs;
    std::vector<RecRef> recs(nblocks);
    std::vector<std::vector<std::unique_ptr<uint8_t[]>>> store(nctx);
    std::vector<std::string> err(nctx);
    // one context: records go straight from the staging slots to their place in `out`
    const bool direct = nctx == 1;
    const uint64_t table = nblocks == 1 ? 0 : 32 + 8 * nblocks;
    use_device(ctxs[0]);
    // the DMA-only paths, decided per context device (several contexts may sit on other GPUs)
    std::vector<char> in_pinned(nctx);
    for (uint32_t g = 0; g < nctx; ++g) in_pinned[g] = is_pinned(in, n, ctxs[g]->device);
    const bool out_pinned = direct && is_pinned(out, out_cap, ctxs[0]->device);
    uint64_t at = table;
    if (direct && table > out_cap) fail(BMH_ERANGE, "compress: output capacity too small");
    std::vector<bmh_status> st(nctx, BMH_OK);
    struct Share {  // the contexts streaming at once split the host's copy threads
        Ctx *c;
        Share(Ctx *x, uint32_t n) : c(x) { c->copy_share = n; }
        ~Share() { c->copy_share = 1; }
    };
    auto work = [&](uint32_t g) {
        try {
            Share share(ctxs[g], nctx);
            use_device(ctxs[g]);
            std::vector<uint64_t> bl;
            for (uint64_t b = g; b < nblocks; b += nctx) bl.push_back(b);
            if (direct) {
                PinnedOut po{out, out_cap, table};
                encode_host_blocks(
                    ctxs[g], in, n, bs, bl,
                    [&](size_t i0, size_t cnt, const uint8_t *src, const uint64_t *ro) {
                        const uint64_t bytes = ro[cnt];
                        if (at + bytes > out_cap) fail(BMH_ERANGE, "compress: output capacity too small");
                        if (src != out + at) par_memcpy(out + at, src, bytes, copy_threads(ctxs[g]));
                        for (size_t i = 0; i < cnt; ++i) {
                            if (table) put_u64(out + 32 + 8 * (i0 + i), ro[i + 1] - ro[i]);
                        }
                        at += bytes;
                    },
                    in_pinned[g] != 0, out_pinned ? &po : nullptr);
            } else {
                encode_host_blocks(ctxs[g], in, n, bs, bl,
                                   [&](size_t i0, size_t cnt, const uint8_t *src, const uint64_t *ro) {
                                       const uint64_t bytes = ro[cnt];
                                       std::unique_ptr<uint8_t[]> buf(new uint8_t[std::max<uint64_t>(bytes, 1)]);
                                       par_memcpy(buf.get(), src, bytes, copy_threads(ctxs[g]));
                                       for (size_t i = 0; i < cnt; ++i)
                                           recs[bl[i0 + i]] = RecRef{buf.get() + ro[i], ro[i + 1] - ro[i]};
                                       store[g].push_back(std::move(buf));
                                   },
                                   in_pinned[g] != 0);
            }
        } catch (const Error &e) {
            st[g] = e.status;
            err[g] = e.what();
        } catch (const std::bad_alloc &) {
            st[g] = BMH_ENOMEM;
            err[g] = "host allocation failed";
        } catch (const std::exception &e) {
            st[g] = BMH_EINVAL;
            err[g] = e.what();
        }
    };
    if (nctx == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < nctx; ++g) th.emplace_back(work, g);
        for (auto &t : th) t.join();
    }
    for (uint32_t g = 0; g < nctx; ++g)
        if (st[g] != BMH_OK) fail(st[g], err[g]);
    if (direct) {
        if (table) {
            memcpy(out, kContainerMagic, 8);
            put_u64(out + 8, bs);
            put_u64(out + 16, nblocks);
            put_u64(out + 24, n);
        }
        *out_len = at;
    } else {
        assemble(n, bs, nblocks, recs, out, out_cap, out_len);
    }
    API_END
}

bmh_status bmh_decompress_host(const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out)
{
    API_BEGIN
    if (!in || !n_out) fail(BMH_EINVAL, "null argument");
    decompress(in, len, out, cap, n_out);
    API_END
}

bmh_status bmh_decode_blocks_dev(bmh_ctx *c, const uint8_t *d_rec, const uint64_t *rec_offs, uint32_t nblocks,
                                 uint8_t *d_out, uint64_t out_cap, uint64_t *h_out_offs)
{
    API_BEGIN
    use_device(c);
    if (!d_rec || !rec_offs || !d_out || !h_out_offs || nblocks == 0) fail(BMH_EINVAL, "null argument");
    decode_blocks(c, d_rec, rec_offs, nblocks, d_out, out_cap, h_out_offs);
    API_END
}

bmh_status bmh_decompress_dev(bmh_ctx *c, const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out)
{
    API_BEGIN
    use_device(c);
    if (!in || !n_out) fail(BMH_EINVAL, "null argument");
    // record list (a single record, or the records of a container)
    std::vector<uint64_t> ro, rl;
    if (is_container(in, len)) {
        ContainerView v = parse_container(in, len);
        ro = v.rec_off;
        rl = v.rec_len;
    } else {
        ro.push_back(0);
        rl.push_back(len);
    }
    uint64_t total = 0;
    std::vector<uint64_t> ns(ro.size());
    for (size_t b = 0; b < ro.size(); ++b) {
        ns[b] = record_n(in + ro[b], rl[b]);
        total += ns[b];
    }
    *n_out = total;
    if (!out) return BMH_OK;
    if (total > cap) fail(BMH_ERANGE, "decompress: output capacity too small");
    // batches of consecutive records: output < 1 GiB (BMH_OPT_MAX_BATCH), <= 65535 records
    const uint64_t cap_batch = max_batch_bytes(c);
    uint64_t done = 0;
    for (size_t i = 0; i < ro.size();) {
        size_t j = i;
        uint64_t nout = 0, nin = 0;
        while (j < ro.size() && j - i < 65535 && (j == i || nout + ns[j] <= cap_batch)) {
            nout += ns[j];
            nin += rl[j];
            ++j;
        }
        uint8_t *d_in = (uint8_t *)c->get(WS_IN, nin + 64);
        uint8_t *d_o = (uint8_t *)c->get(WS_OUT, nout + 64);
        std::vector<uint64_t> offs(j - i + 1, 0), oo(j - i + 1, 0);
        for (size_t k = i; k < j; ++k) {
            BMH_HIP(hipMemcpyAsync(d_in + offs[k - i], in + ro[k], rl[k], hipMemcpyHostToDevice, c->stream));
            offs[k - i + 1] = offs[k - i] + rl[k];
        }
        decode_blocks(c, d_in, offs.data(), (uint32_t)(j - i), d_o, nout, oo.data());
        BMH_HIP(hipMemcpyAsync(out + done, d_o, nout, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        done += nout;
        i = j;
    }
    API_END
}

bmh_status bmh_record_to_mtf(const uint8_t *rec, uint64_t len, uint8_t *mtf, uint64_t cap, uint64_t *n_out)
{
    API_BEGIN
    if (!rec || !n_out) fail(BMH_EINVAL, "null argument");
    record_to_mtf(rec, len, mtf, cap, n_out);
    API_END
}

int bmh_is_container(const uint8_t *in, uint64_t len) { return in && is_container(in, len) ? 1 : 0; }

bmh_status bmh_container_info(const uint8_t *in, uint64_t len, uint64_t *nblocks, uint64_t *total_n)
{
    API_BEGIN
    if (!in || !is_container(in, len) || len < 32) fail(BMH_ECORRUPT, "not a BMH container");
    if (nblocks) *nblocks = get_u64(in + 16);
    if (total_n) *total_n = get_u64(in + 24);
    API_END
}

bmh_status bmh_container_record(const uint8_t *in, uint64_t len, uint64_t b, const uint8_t **rec, uint64_t *rec_len)
{
    API_BEGIN
    if (!in || !is_container(in, len) || len < 32) fail(BMH_ECORRUPT, "not a BMH container");
    const uint64_t nb = get_u64(in + 16);
    if (b >= nb || nb > (len - 32) / 8) fail(BMH_EINVAL, "block index out of range");
    uint64_t o = 32 + 8 * nb;
    for (uint64_t k = 0; k < b; ++k) o += get_u64(in + 32 + 8 * k);
    const uint64_t l = get_u64(in + 32 + 8 * b);
    if (o > len || l > len - o) fail(BMH_ECORRUPT, "container: record overruns input");
    if (rec) *rec = in + o;
    if (rec_len) *rec_len = l;
    API_END
}

bmh_status bmh_ctx_set_option(bmh_ctx *c, uint32_t option, uint64_t value)
{
    API_BEGIN
    use_device(c);
    c->sync();
    switch (option) {
    case BMH_OPT_PIPELINES:
        if (value > 16) fail(BMH_ERANGE, "set_option: at most 16 pipelines");
        c->opt.pipelines = value;
        break;
    case BMH_OPT_STREAM_BATCH: c->opt.stream_batch = value; break;
    case BMH_OPT_MAX_BATCH: c->opt.max_batch = value; break;
    case BMH_OPT_MTF_CHUNK:
        if (value > 4096 || (value && value < 64)) fail(BMH_ERANGE, "set_option: MTF chunk of 64..4096 symbols (0: adaptive)");
        c->opt.mtf_chunk = value;
        break;
    case BMH_OPT_CHECK_LISTS: c->opt.check_lists = value != 0; break;
    case BMH_OPT_ONE_PIPELINE: c->opt.one_pipeline = value != 0; break;
    case BMH_OPT_COPY_THREADS:
        if (value > 64) fail(BMH_ERANGE, "set_option: at most 64 copy threads");
        c->opt.copy_threads = value;
        break;
    default: fail(BMH_EINVAL, "set_option: unknown option " + std::to_string(option));
    }
    API_END
}

bmh_status bmh_ctx_set_timing(bmh_ctx *c, int enable)
{
    API_BEGIN
    use_device(c);
    c->sync();
    c->timing = enable != 0;
    API_END
}

bmh_status bmh_ctx_reset_stats(bmh_ctx *c)
{
    API_BEGIN
    use_device(c);
    c->sync();
    c->stats.clear();
    API_END
}

int bmh_ctx_kernel_stats(bmh_ctx *c, char (*names)[64], uint64_t *launches, double *total_ms, int cap)
{
    if (!c) return 0;
    try {
        c->sync();
    } catch (...) {
        return 0;
    }
    int i = 0;
    for (auto &kv : c->stats) {
        if (i < cap) {
            if (names) {
                strncpy(names[i], kv.first.c_str(), 63);
                names[i][63] = 0;
            }
            if (launches) launches[i] = kv.second.launches;
            if (total_ms) total_ms[i] = kv.second.ms;
        }
        ++i;
    }
    return i;
}

bmh_status bmh_synth_splitmix64_dev(bmh_ctx *c, uint8_t *d_out, uint64_t nbytes, uint64_t seed, uint64_t offset)
{
    API_BEGIN
    use_device(c);
    if (!d_out) fail(BMH_EINVAL, "null buffer");
    if (nbytes) synth_splitmix64(c, d_out, nbytes, seed, offset);
    API_END
}

bmh_status bmh_synth_zipf_dev(bmh_ctx *c, uint8_t *d_out, uint64_t nbytes, uint64_t offset)
{
    API_BEGIN
    use_device(c);
    if (!d_out) fail(BMH_EINVAL, "null buffer");
    if (nbytes) synth_zipf(c, d_out, nbytes, offset);
    API_END
}

}  // extern "C"
