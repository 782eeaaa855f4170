// bmh_internal.h — shared internals of libbmh: the per-GPU context (stream, workspace arena,
// per-kernel HIP-event timing) and error plumbing. Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/bmh.h"

namespace bmh {

// Checked builds (-DBMH_CHECK): kinds of device-side precondition violations (device_util.h)
// and the registry of per-translation-unit readers (capi.cpp, bmh_check_violations).
enum : uint32_t { kCheckExec = 0, kCheckKinds = 4 };
void check_register(uint32_t (*reader)(uint32_t kind));

struct Error : std::runtime_error {
    bmh_status status;
    Error(bmh_status s, const std::string &m) : std::runtime_error(m), status(s) {}
};

[[noreturn]] void fail(bmh_status s, const std::string &msg);
void set_last_error(const std::string &msg);

#define BMH_HIP(call)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            ::bmh::fail(BMH_EHIP, std::string(#call) + ": " + hipGetErrorString(e_) + " @" + \
                                      __FILE__ + ":" + std::to_string(__LINE__));              \
    } while (0)

struct KStat {
    uint64_t launches = 0;
    double ms = 0.0;
};

// Grow-only device buffers keyed by slot; reused across calls so the hot path does no
// hipMalloc (arrays are sized for the largest batch seen).
enum Slot : int {
    WS_SA, WS_SA2, WS_RKA, WS_RKB, WS_KEY, WS_KEY2, WS_SEG_CUR, WS_SEG_NXT, WS_TINY, WS_MED,
    WS_LARGE, WS_LARGE2, WS_GROUPS, WS_PREFIX, WS_SCAN_PART, WS_TILES, WS_BLOCKS, WS_OFFS,
    WS_CHIST, WS_BSTART, WS_COUNTERS, WS_LTILES, WS_LTHIST, WS_LSEGS, WS_SEGOR, WS_COOP, WS_LISTS, WS_L, WS_MTF,
    WS_MTF_R, WS_MTF_S, WS_MTF_SUPER, WS_MTF_CHUNKS, WS_FREQ, WS_FIRST, WS_PRIMARY, WS_PACK_BITS,
    WS_PACK_CHUNKS, WS_TABLES, WS_HDR, WS_HDR_OFFS, WS_IN, WS_OUT, WS_IN2, WS_OUT2, WS_IN3, WS_OUT3, WS_RESOLVED, WS_FIN_CUR, WS_FIN_NXT,
    WS_DSEG_CUR, WS_DSEG_NXT, WS_DLARGE, WS_DLARGE2, WS_DGROUPS, WS_KEY8, WS_ROFFS, WS_STATUS, WS_PACK_HIST, WS_FINT_CUR, WS_FINT_NXT, WS_FINB_CUR, WS_FINB_NXT, WS_KEY8B, WS_RUN_MISC, WS_RUN_MOVE, WS_RUN_IN, WS_RUN_L, WS_RUNS, WS_RUN_PRIM, WS_BAND, WS_SYNTH, WS_ALPHA, WS_COUNT_
};

struct Ctx {
    int device = 0;
    int cus = 256;  // compute units of the device (persistent-grid sizing)
    hipStream_t stream = nullptr;
    bool own_stream = true;  // sub-pipelines 0 and 2 borrow the context / H2D stream (capi.cpp)
    bool timing = false;
    std::map<std::string, KStat> stats;
    struct Pending {
        const char *name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    void *ws[WS_COUNT_] = {};
    size_t ws_size[WS_COUNT_] = {};
    // host-built tables kept in a workspace slot: signature of what was uploaded (0 = none or
    // overwritten; get() clears it on reallocation) and a few counts derived with it, so a
    // batch with the same layout as the previous one skips the rebuild and the upload
    uint64_t ws_tag[WS_COUNT_] = {};
    uint32_t ws_aux[WS_COUNT_][6] = {};
    // pinned host staging
    void *pinned = nullptr;
    size_t pinned_size = 0;
    // pinned upload/download arena: every small host<->device copy goes through it so the
    // copies stay asynchronous; reset at each sync()
    uint8_t *arena = nullptr;
    size_t arena_size = 0, arena_used = 0;
    struct Deferred {
        void *dst;
        size_t off, bytes;
    };
    std::vector<Deferred> deferred;

    // sub-pipelines (own stream + workspaces) a batch is split across (capi.cpp)
    std::vector<Ctx *> subs;
    // side context on the context's D2H stream (idle outside host-buffer calls): the run-length
    // BWT of a batch's run-heavy blocks runs there beside the rotation sorter (bwt_runs.hip)
    hipStream_t aux_stream = nullptr;
    Ctx *aux = nullptr;
    // tuning options (bmh_ctx_set_option; 0 = the library's rule); sub-pipelines and the side
    // context copy their parent's at every call
    struct Options {
        uint64_t pipelines = 0, stream_batch = 0, max_batch = 0, mtf_chunk = 0, check_lists = 0, one_pipeline = 0, copy_threads = 0;
    } opt;
    uint32_t last_pipelines = 0;  // pipelines of the last device batch encode (encode_blocks)
    uint64_t zipf_resume_tok0 = 0, zipf_resume_base = 0;  // synth_zipf: start of its last round
    uint64_t mtf_clen_sig = 0;  // MTF chunk length of the last batch layout (mtf.hip)
    uint32_t mtf_clen = 0;
    // size of the batch a sub-pipeline's sub-batch was cut from (0: its own batch): the run
    // screen is decided on it, so a batch past the screen never sends its sub-batches' run-heavy
    // blocks to the side stream D, which a fourth pipeline holds (bwt_runs.hip)
    uint64_t screen_total = 0;
    // BWT: write the suffix array of every slot (needed by rank doubling) instead of only the
    // slots later passes read; set after a batch needed doubling, cleared when one did not
    bool bwt_full_sa = false;
    // speculative list round (bwt.hip): a dense batch on one pipeline runs its one expected
    // (tiny) list round on a fixed grid without waiting for the list counters, and the MTF /
    // Huffman / pack stages follow at once; encode_blocks_one reads the counters at its final
    // sync (bwt_spec_ok) and encodes the batch again the waiting way if any list work was left
    uint32_t *probe_host = nullptr, probe_cap = 0;  // dense_batch's census (pinned, written by the kernel)
    hipEvent_t probe_ev = nullptr;
    void *dbl_cnt_host = nullptr;  // rank doubling: two rounds' counters (pinned), read one round late
    hipEvent_t dbl_ev[2] = {};
    uint64_t pre_sig = 0;  // bwt_batch_core's prologue already launched for this input + layout
    uint32_t copy_share = 1;  // contexts streaming host buffers at once (bmh_compress_host_multi)
    uint64_t dense_sig = 0;  // layout of the last batch dense_batch found dense (prologue queued early)
    bool spec_lists = false, spec_pending = false;
    bool mtf_dense = false;  // the batch was found dense: MTF stages skip their run-aware paths
    std::vector<uint64_t> roffs_host;  // encode_blocks_one: record offsets + status, one copy
    // host threads of sub-pipelines 1.. (capi.cpp encode_blocks): kept across calls, so a small
    // batch's later pipelines do not wait for a thread to be created on every call
    struct Worker;
    std::vector<std::unique_ptr<Worker>> workers;
    uint32_t spec_fallbacks = 0;
    uint32_t spec_cnt[128] = {};  // the list counters after the speculative round
    // host-buffer streaming (capi.cpp): copy streams and two pinned staging slots each way
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    static constexpr int kStageSlots = 3;  // host-buffer streaming: batches in flight (H2D / encode / D2H)
    uint8_t *stage_in[kStageSlots] = {}, *stage_out[kStageSlots] = {};
    size_t stage_in_size[kStageSlots] = {}, stage_out_size[kStageSlots] = {};  // per slot, allocated on first use

    void *get(Slot s, size_t bytes);
    void *host_pinned(size_t bytes);
    void h2d(void *d_dst, const void *h_src, size_t bytes);  // staged, asynchronous
    void d2h(void *h_dst, const void *d_src, size_t bytes);  // staged; h_dst valid after sync()
    void sync();  // stream sync (spin-wait) + staged downloads + timing events
    hipEvent_t ev();
    int tbegin(const char *name);  // -1 when timing is off
    void tend(int idx);
};

// Back-off between two polls of a HIP stream or event in the host spin-waits (~0.5 us of x86
// pause): several host threads polling back to back (pipelines, the run path) contend in the
// runtime with each other's launches.
inline void spin_pause()
{
    for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
}

// Signature of a batch layout for the table cache (Ctx::ws_tag): kind, block offsets and the
// input's 16-byte misalignment (chunk boundaries depend on it).
inline uint64_t layout_sig(uint64_t kind, const std::vector<uint64_t> &offs, uintptr_t base)
{
    uint64_t h = 1469598103934665603ull ^ kind;
    auto mix = [&](uint64_t v) {
        h ^= v;
        h *= 1099511628211ull;
        h ^= h >> 29;
    };
    mix(offs.size());
    mix(base & 63u);
    for (uint64_t o : offs) mix(o);
    return h | 1u;  // never 0
}

// Host wall-clock of a phase (device work included when the phase synchronises), recorded
// under "wall:<name>" when timing is enabled.
struct WallPhase {
    Ctx *c;
    const char *name;
    std::chrono::steady_clock::time_point t0;
    WallPhase(Ctx *c_, const char *n) : c(c_), name(n), t0(std::chrono::steady_clock::now()) {}
    ~WallPhase() { stop(); }
    void stop()
    {
        if (!name || !c->timing) return;
        KStat &k = c->stats[std::string("wall:") + name];
        k.launches++;
        k.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        name = nullptr;
    }
};

// Kernel launch on the context stream, bracketed by timing events when enabled.
#define BMH_LAUNCH(ctx, kname, kern, grid, block, shmem, ...)                             \
    do {                                                                                  \
        const int p_ = (ctx)->tbegin(kname);                                              \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(block), shmem, (ctx)->stream, __VA_ARGS__); \
        BMH_HIP(hipGetLastError());                                                       \
        (ctx)->tend(p_);                                                                  \
    } while (0)

// Batch description shared by the stages.
struct BlockInfo {
    uint32_t off;     // global byte offset of the block in the batch buffer
    uint32_t n;       // block length
};

struct Batch {
    std::vector<uint64_t> offs;  // nblocks + 1
    uint32_t nblocks = 0;
    uint64_t total = 0;
    uint32_t max_n = 0;
};
Batch make_batch(const uint64_t *offs, uint32_t nblocks);

// Per-block code book on the device (huffman.hip, pack.hip).
struct DevTable {
    uint64_t code[256];
    uint8_t len[256];
};
inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Pack chunks: 4 K symbols, aligned to each block's start; mtf_batch writes one u16
// histogram per pack chunk (WS_PACK_HIST), pack_batch_dev sizes the chunks from them.
constexpr uint32_t kPackChunkSyms = 4096;
inline void pack_chunk_first(const Batch &bt, uint32_t *first)
{
    first[0] = 0;
    for (uint32_t b = 0; b < bt.nblocks; ++b)
        first[b + 1] = first[b] + (uint32_t)((bt.offs[b + 1] - bt.offs[b] + kPackChunkSyms - 1) / kPackChunkSyms);
}

// device status word bits (encode pipeline; checked by the host after the final sync)
constexpr uint32_t kStatusEmpty = 1, kStatusCodeLen = 2, kStatusPrimary = 4, kStatusCapacity = 8;

// Stage implementations (device buffers). bwt_batch / mtf_batch synchronise only when they
// return host outputs (h_primary / h_freq32 non-null).
void bwt_batch(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_L, uint64_t *h_primary);  // bwt_runs.hip
Ctx *aux_ctx(Ctx *c);  // capi.cpp
bool dense_batch(Ctx *c, const uint8_t *d_in, const Batch &bt);  // digram census (bwt_runs.hip)
// the rotation sorter alone (bwt.hip); bwt_batch routes run-heavy blocks of small batches around it
// prologue_only: launch the global pass's first kernels (up to the bucket scan) and return; the
// next call for the same input and layout on this context skips them (Ctx::pre_sig)
void bwt_batch_core(Ctx *c, const uint8_t *d_in, const Batch &bt, uint8_t *d_L, uint64_t *h_primary,
                    bool prologue_only = false);
bool bwt_spec_ok(const Ctx *c);  // after the sync that follows a speculative list round
void mtf_batch(Ctx *c, const uint8_t *d_L, const Batch &bt, uint8_t *d_mtf, uint32_t *h_freq32,
               uint32_t *h_first32);
void pack_batch(Ctx *c, const uint8_t *d_mtf, const Batch &bt, const bmh_code_table *tables, uint8_t *d_out,
                uint64_t out_cap, const uint64_t *pay_offs, uint64_t *out_bytes);
// Record offsets of consecutive sub-batches encoded concurrently on several streams: sub-batch
// s starts where s - 1 ends (a device value), so s waits for s - 1's offset scan.
struct OffsetChain {
    std::mutex m;
    std::condition_variable cv;
    int recorded = -1;  // highest sub-batch whose offset scan has been enqueued
    bool failed = false;
    std::vector<hipEvent_t> ev;
    std::vector<const uint64_t *> d_end;  // device: end offset of each sub-batch's records
};
void codebook_batch(Ctx *c, const Batch &bt, const uint64_t *d_boffs, const uint32_t *d_freq, const uint32_t *d_first,
                    const uint32_t *d_prim, DevTable *d_tabs, uint64_t *d_roffs, uint64_t *d_pay_offs,
                    uint8_t *d_out, uint64_t out_cap, uint32_t *d_status, OffsetChain *chain, int sub);
void pack_batch_dev(Ctx *c, const uint8_t *d_mtf, const Batch &bt, const DevTable *d_tabs, const uint64_t *d_pay_offs,
                    uint8_t *d_out, const uint32_t *d_status, const uint16_t *d_chist);
void histogram_batch(Ctx *c, const uint8_t *d_in, const Batch &bt, uint32_t *h_freq32, uint32_t *h_first32);
void synth_splitmix64(Ctx *c, uint8_t *d_out, uint64_t nbytes, uint64_t seed, uint64_t offset);  // synth.hip
void synth_zipf(Ctx *c, uint8_t *d_out, uint64_t nbytes, uint64_t offset);

// Host Huffman (huffman_host.cpp). n = the block's size: below kBandCeil the tie-break follows
// the reference's heap history (heap_order.cpp); n = 0 takes the closed-form order.
void huffman_build(const uint64_t freq[256], const uint64_t first[256], bmh_code_table *out, uint64_t n = 0);

// The reference's BTree address order for small blocks (heap_order.cpp): per leaf count L,
// off[L] = first entry of L's 2L - 1 node ranks in `rank`, or kModelOrder where the
// closed-form order holds. band_ranks(n) is nullptr when it holds for every
// L (always for n >= kBandCeil); results are cached per n, process-wide.
constexpr uint64_t kBandCeil = 1u << 17;
constexpr uint32_t kModelOrder = 0xffffffffu;
struct BandRanks {
    std::vector<uint32_t> off;   // 257 entries
    std::vector<uint16_t> rank;  // node id -> ascending-address rank among the 2L - 1 nodes
};
std::shared_ptr<const BandRanks> band_ranks(uint64_t n);  // LRU-bounded cache (heap_order.cpp)
// the tables of a batch's sizes (< kBandCeil), the missing ones computed in parallel; the
// returned pointers outlive any eviction from the cache
std::map<uint64_t, std::shared_ptr<const BandRanks>> band_ranks_batch(const std::vector<uint64_t> &sizes);
size_t band_cache_entries();  // sizes currently cached
void node_ranks(uint64_t n, uint32_t L, uint16_t *rank);  // exact ranks (model or heap history)
uint64_t payload_bytes(const bmh_code_table *t, const uint64_t freq[256]);

// Device Huffman decode table of one record (built on the host by build_dec_table).
constexpr uint32_t kDecLutBits = 12;
struct DecTable {
    uint32_t lut[1u << kDecLutBits];  // next 12 bits -> sym << 8 | code length, or node << 16 (longer code)
    uint16_t child[512][2];           // internal nodes: children (node ids); leaves: 0xffff
    uint8_t sym[512];                 // leaf symbols
    uint32_t single;                  // the root is a leaf: every symbol is sym[0], 0-bit codes
    uint32_t maxlen;                  // longest code (tree depth), bits
    uint32_t pad[2];
};
// Parses the preorder tree bytes of a record (bytes_to_tree_dfs, main.cpp:198-219).
void build_dec_table(const uint8_t *tree, uint64_t tree_len, DecTable *out);
void decode_blocks(Ctx *c, const uint8_t *d_rec, const uint64_t *rec_offs, uint32_t nblocks, uint8_t *d_out,
                   uint64_t out_cap, uint64_t *out_offs);

// Records / container / decode (record.cpp)
constexpr uint64_t kRecordHeader = 24;
void put_u64(uint8_t *p, uint64_t v);
uint64_t get_u64(const uint8_t *p);
extern const uint8_t kContainerMagic[8];
uint64_t record_n(const uint8_t *rec, uint64_t len);
void record_to_mtf(const uint8_t *rec, uint64_t len, uint8_t *mtf, uint64_t cap, uint64_t *n_out);
void decode_record(const uint8_t *rec, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out);
struct ContainerView {
    uint64_t block_size, nblocks, total;
    std::vector<uint64_t> rec_off, rec_len;
};
ContainerView parse_container(const uint8_t *in, uint64_t len);
bool is_container(const uint8_t *in, uint64_t len);
void decompress(const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out);

}  // namespace bmh

struct bmh_ctx : bmh::Ctx {};
