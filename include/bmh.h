/*
 * bmh.h — C ABI of the MI355X-native BWT -> MTF -> Huffman block encoder (libbmh.so).
 *
 * The reference (komour/bwt-mtf-huffman-compressor) has no plugin/FFI API: its seam is the
 * set of free C++ stage functions that compress() calls in sequence (main.cpp:305-316).
 * Each entry point below replaces one of them (cited), batched over independent blocks and
 * running on one GPU per context. All functions return a bmh_status; nothing throws.
 *
 * Memory: functions named *_dev take device (HBM) pointers allocated with bmh_dev_alloc (or
 * any hipMalloc'd / torch CUDA tensor memory of the context's device); host arrays are
 * plain host memory. A "batch" of nblocks blocks is described by `offs`, a HOST array of
 * nblocks+1 uint64 prefix offsets: block b is bytes [offs[b], offs[b+1]) of the buffer.
 * Limits: every block 1 <= n < 2^32 - 1; a batch totals < 2^32 bytes (split bigger jobs).
 *
 * Threading: a context is used by one host thread at a time (one context per GPU).
 * All calls are synchronous: they return when their results are complete.
 */
#ifndef BMH_H
#define BMH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    BMH_OK = 0,
    BMH_EINVAL = 1,   /* bad argument (e.g. empty block: the reference segfaults there) */
    BMH_ENOMEM = 2,   /* host or device allocation failed */
    BMH_EHIP = 3,     /* a HIP runtime call failed */
    BMH_ERANGE = 4,   /* output capacity too small / size limit exceeded */
    BMH_ECORRUPT = 5, /* malformed record or container */
    BMH_ENODEV = 6    /* no usable gfx950 device */
} bmh_status;

typedef struct bmh_ctx bmh_ctx;

/* Per-block Huffman code table: the data the reference keeps in its BTree + the
 * unordered_map<u8, vector<bool>> of build_hashmap (main.cpp:149-156). */
typedef struct {
    uint64_t code[256];  /* code word of symbol s, MSB-first, right-aligned */
    uint8_t len[256];    /* code length in bits (0 for absent symbols / single-leaf tree) */
    uint8_t tree[320];   /* preorder tree bytes, tree_to_bytes (main.cpp:174-196) */
    uint32_t tree_len;   /* ceil((10*leaves - 1) / 8) */
    uint32_t leaves;     /* number of distinct MTF symbols */
} bmh_code_table;

/* ---- library / context ------------------------------------------------------------ */
const char *bmh_version(void);
const char *bmh_status_str(int status);
/* Last error message of the calling thread (empty string if none). */
const char *bmh_last_error(void);
int bmh_device_count(void);
bmh_status bmh_ctx_create(int device, bmh_ctx **out);
void bmh_ctx_destroy(bmh_ctx *ctx);
/* The context's HIP stream (hipStream_t), for callers that order their own work after it. */
void *bmh_ctx_stream(bmh_ctx *ctx);

/* Device memory helpers (so FFI callers need no HIP headers). */
bmh_status bmh_dev_alloc(bmh_ctx *ctx, uint64_t bytes, void **d_ptr);
bmh_status bmh_dev_free(bmh_ctx *ctx, void *d_ptr);
/* Page-locked host memory (hipHostMalloc). bmh_compress_host detects page-locked input and
 * output buffers and then moves the data by DMA only: no staging copies on the host.
 * The block is not tied to the context: bmh_host_free accepts ctx == NULL (e.g. after the
 * context that allocated it was destroyed). */
bmh_status bmh_host_alloc(bmh_ctx *ctx, uint64_t bytes, void **h_ptr);
bmh_status bmh_host_free(bmh_ctx *ctx, void *h_ptr);
bmh_status bmh_memcpy_h2d(bmh_ctx *ctx, void *d_dst, const void *h_src, uint64_t bytes);
bmh_status bmh_memcpy_d2h(bmh_ctx *ctx, void *h_dst, const void *d_src, uint64_t bytes);

/* ---- stage entry points (device buffers, batched over blocks) --------------------- */
/* Replaces bwt() (main.cpp:77-91): cyclic-rotation BWT of every block. d_L receives the
 * last column (same layout as d_in); h_primary[b] = the row of rotation 0
 * (= number of rotations strictly smaller than rotation 0). */
bmh_status bmh_bwt_dev(bmh_ctx *ctx, const uint8_t *d_in, const uint64_t *offs, uint32_t nblocks,
                       uint8_t *d_L, uint64_t *h_primary);

/* Replaces move_to_front() (main.cpp:93-112) plus the histogram and first-occurrence scan
 * of huffman() (main.cpp:231-244). h_freq and h_first are nblocks*256 arrays (may be NULL):
 * freq of each MTF symbol, and the block-relative index of its first occurrence
 * (UINT64_MAX if absent). */
bmh_status bmh_mtf_dev(bmh_ctx *ctx, const uint8_t *d_L, const uint64_t *offs, uint32_t nblocks,
                       uint8_t *d_mtf, uint64_t *h_freq, uint64_t *h_first);

/* The histogram + first-occurrence scan of huffman() (main.cpp:231-244) on its own, for an
 * arbitrary device byte stream (bmh_mtf_dev already returns both for its output). */
bmh_status bmh_histogram_dev(bmh_ctx *ctx, const uint8_t *d_in, const uint64_t *offs, uint32_t nblocks,
                             uint64_t *h_freq, uint64_t *h_first);

/* Replaces the tree part of huffman() (main.cpp:245-254), traverse/build_hashmap
 * (main.cpp:132-156) and tree_to_bytes (main.cpp:174-196). Host-only. Leaves are ordered by
 * first occurrence; equal frequencies break ties by the reference's heap-address order
 * under glibc. */
bmh_status bmh_huffman_build(const uint64_t freq[256], const uint64_t first[256], bmh_code_table *out);
/* The same for a block of n bytes: below 128 KiB the tie-break follows the heap history of a
 * standalone reference COMPRESS run of n bytes (glibc 2.35; the `new BTree` addresses of
 * main.cpp:240,252 depend on the blocks read_bytes / bwt / move_to_front freed before,
 * io_utilities.h:40-54, main.cpp:77-112), which decides the records of the small-input bands
 * (SURVEY §8(f) row 4). bmh_encode_blocks_dev applies the same order per block. */
bmh_status bmh_huffman_build_sized(const uint64_t freq[256], const uint64_t first[256], uint64_t n,
                                   bmh_code_table *out);
/* Node address ranks the above uses for n bytes and L leaves: rank[s] for node ids s < 2L - 1
 * (leaves by first occurrence, then internal nodes in creation order). Returns 1 when they
 * come from the heap history, 0 when the closed-form order of SURVEY App. B.3 holds. */
int bmh_node_ranks(uint64_t n, uint32_t L, uint16_t *rank);
/* Payload bytes encode_with_huffman (main.cpp:158-172) emits: max(1, ceil(sum freq*len / 8)). */
uint64_t bmh_payload_bytes(const bmh_code_table *table, const uint64_t freq[256]);

/* Replaces encode_with_huffman() (main.cpp:158-172): MSB-first concatenation of code words,
 * max(1, ceil(bits / 8)) bytes per block. tables[b] is block b's table; block b's payload is
 * written at d_out + pay_offs[b] (pay_offs: host array of nblocks entries, or NULL for payloads
 * back to back from d_out). d_out must be 4-byte aligned: the pack writes whole 4-byte words
 * (bytes of an edge word outside the payload are preserved), so each payload's extent rounded up
 * to a 4-byte boundary must fit in out_cap, else BMH_ERANGE and nothing is written; overlapping
 * payloads are BMH_EINVAL. out_bytes (host, nblocks entries, may be NULL) receives each
 * payload's byte count (= bmh_payload_bytes). */
bmh_status bmh_pack_dev(bmh_ctx *ctx, const uint8_t *d_mtf, const uint64_t *offs, uint32_t nblocks,
                        const bmh_code_table *tables, uint8_t *d_out, uint64_t out_cap, const uint64_t *pay_offs,
                        uint64_t *out_bytes);

/* Whole encode (compress(), main.cpp:300-325, minus file I/O): one reference record per
 * block, [u64 primary][u64 n][u64 tree_len][tree][payload] (io_utilities.h:7-27), written
 * back to back at d_out. h_rec_offs (nblocks+1 entries) receives the record offsets. */
bmh_status bmh_encode_blocks_dev(bmh_ctx *ctx, const uint8_t *d_in, const uint64_t *offs, uint32_t nblocks,
                                 uint8_t *d_out, uint64_t out_cap, uint64_t *h_rec_offs);
/* Pipelines (HIP streams, each driven by its own host thread) bmh_encode_blocks_dev runs a batch
 * of nblocks blocks totalling `total` bytes on (the library's rule; BMH_OPT_PIPELINES overrides). */
uint32_t bmh_encode_pipelines(bmh_ctx *ctx, uint64_t total, uint32_t nblocks);
/* Pipelines the context's last bmh_encode_blocks_dev call ran on: the rule above, or 1 when a
 * 32-256 MiB batch's digram census found it dense (uniform-like bytes). */
uint32_t bmh_ctx_last_pipelines(bmh_ctx *ctx);
/* Dense one-pipeline batches run their one expected BWT list round without waiting for its
 * counts and check them at the end; this counts the context's batches whose check found list
 * work left, so they were encoded again the waiting way (records are the same either way). */
uint32_t bmh_ctx_spec_fallbacks(bmh_ctx *ctx);
/* Capacity sufficient for one record of an n-byte block. */
uint64_t bmh_record_bound(uint64_t n);

/* ---- host-buffer convenience (H2D + encode + D2H) ---------------------------------- */
/* Encodes `in` (n bytes) cut into block_size blocks (block_size 0 or >= n: one block).
 * One block => exactly the reference record; several => the BMH container (bmh_container_*).
 * Returns the output size in *out_len. Batches stream through H2D / encode / D2H on separate
 * streams; with page-locked `in` / `out` (bmh_host_alloc) the copies are DMA-only. */
bmh_status bmh_compress_host(bmh_ctx *ctx, const uint8_t *in, uint64_t n, uint64_t block_size,
                             uint8_t *out, uint64_t out_cap, uint64_t *out_len);
/* Same, spreading blocks round-robin (block b -> ctxs[b % nctx]) over several contexts
 * (one per GPU), each driven by its own host thread. */
bmh_status bmh_compress_host_multi(bmh_ctx **ctxs, uint32_t nctx, const uint8_t *in, uint64_t n,
                                   uint64_t block_size, uint8_t *out, uint64_t out_cap, uint64_t *out_len);
uint64_t bmh_compress_bound(uint64_t n, uint64_t block_size);
/* CPUs this process may use: its affinity set capped by the cgroup CPU quota. */
uint32_t bmh_host_cpus(void);
/* Copy threads per copy site each of nctx contexts streaming at once uses for its pageable <->
 * page-locked staging copies (cpus 0: bmh_host_cpus()): cpus / nctx, clamped to [1, 16]. */
uint32_t bmh_copy_threads(uint32_t nctx, uint32_t cpus);

/* ---- decode (host C++; replaces decompress(), main.cpp:327-345) -------------------- */
/* Decodes one reference record or one BMH container. *n_out receives the decoded size;
 * if out is NULL only the size is reported. */
bmh_status bmh_decompress_host(const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *n_out);
/* GPU decode (replaces decompress(), main.cpp:327-345 — tree parse :198-219, huffman_reverse
 * :259-281, inverse MTF :114-130, bwt_reverse :61-75) of a batch of records in device
 * memory: record b = d_rec[rec_offs[b], rec_offs[b+1]) (rec_offs: host, nblocks+1 entries).
 * Block b's bytes land at d_out + h_out_offs[b]; h_out_offs (host, nblocks+1) is filled
 * from the record headers. The batch output must be < 4 GiB. */
bmh_status bmh_decode_blocks_dev(bmh_ctx *ctx, const uint8_t *d_rec, const uint64_t *rec_offs, uint32_t nblocks,
                                 uint8_t *d_out, uint64_t out_cap, uint64_t *h_out_offs);
/* decompress() of a record or BMH container held in host memory, decoded on the GPU (same
 * contract as bmh_decompress_host). */
bmh_status bmh_decompress_dev(bmh_ctx *ctx, const uint8_t *in, uint64_t len, uint8_t *out, uint64_t cap,
                              uint64_t *n_out);
/* Huffman stage inverse only (huffman_reverse, main.cpp:259-281): record -> MTF stream. */
bmh_status bmh_record_to_mtf(const uint8_t *rec, uint64_t len, uint8_t *mtf, uint64_t cap, uint64_t *n_out);

/* ---- container helpers ------------------------------------------------------------ */
/* A BMH container is: magic "\xffBMHBLK1" | u64 block_size | u64 nblocks | u64 total_n |
 * u64 record_len[nblocks] | records (each a verbatim reference record). */
int bmh_is_container(const uint8_t *in, uint64_t len);
bmh_status bmh_container_info(const uint8_t *in, uint64_t len, uint64_t *nblocks, uint64_t *total_n);
/* Pointer/length of record b inside a container. */
bmh_status bmh_container_record(const uint8_t *in, uint64_t len, uint64_t b, const uint8_t **rec, uint64_t *rec_len);

/* ---- tuning options ---------------------------------------------------------------- */
/* Per-context overrides of the library's own rules (not part of the reference interface; the
 * library reads no environment variables). Value 0 restores the default. Results never depend
 * on them: every setting produces the same records. */
enum {
    BMH_OPT_PIPELINES = 1,    /* pipelines (streams) per device batch, 1..16 (default: the size rule) */
    BMH_OPT_STREAM_BATCH = 2, /* bmh_compress_host batch bytes (default 256 MiB) */
    BMH_OPT_MAX_BATCH = 3,    /* largest device batch bytes of the host-buffer paths (default 1 GiB) */
    BMH_OPT_MTF_CHUNK = 4,    /* MTF chunk symbols, 64..4096 (default: adaptive) */
    BMH_OPT_CHECK_LISTS = 5,  /* 1: check every BWT list round and print its census (diagnostic, slow) */
    BMH_OPT_ONE_PIPELINE = 6, /* 1: run each device batch on one pipeline AFTER the library's own
                               * decisions (the dense-batch census and its speculative list round
                               * still apply), so a one-stream timing pass runs the default path */
    BMH_OPT_COPY_THREADS = 7  /* host-buffer paths: copy threads per copy site, 1..64 (default:
                               * bmh_copy_threads(contexts streaming at once, 0)) */
};
bmh_status bmh_ctx_set_option(bmh_ctx *ctx, uint32_t option, uint64_t value);

/* ---- measurement ------------------------------------------------------------------- */
/* When enabled, every kernel launch of the context is bracketed by HIP events on the
 * context's stream; stats accumulate per kernel name. */
bmh_status bmh_ctx_set_timing(bmh_ctx *ctx, int enable);
bmh_status bmh_ctx_reset_stats(bmh_ctx *ctx);
/* Kernel stats: returns how many distinct kernels were recorded; fills up to cap entries. */
int bmh_ctx_kernel_stats(bmh_ctx *ctx, char (*names)[64], uint64_t *launches, double *total_ms, int cap);

/* Checked builds (`make check` -> lib_check/libbmh.so, -DBMH_CHECK): number of device-side
 * precondition violations of `kind` so far (0: a full-wave primitive ran with a partial EXEC
 * mask). -1 in a regular build, -2 on error. Not part of the reference interface (test aid). */
int64_t bmh_check_violations(bmh_ctx *ctx, uint32_t kind);

/* Synthetic input: bytes [offset, offset+nbytes) of the little-endian
 * splitmix64(seed) stream, generated on the device. */
bmh_status bmh_synth_splitmix64_dev(bmh_ctx *ctx, uint8_t *d_out, uint64_t nbytes, uint64_t seed, uint64_t offset);
/* Synthetic input: bytes [offset, offset+nbytes) of the integer-Zipf text
 * stream (configs 3 and 5), generated on the device. */
bmh_status bmh_synth_zipf_dev(bmh_ctx *ctx, uint8_t *d_out, uint64_t nbytes, uint64_t offset);

#ifdef __cplusplus
}
#endif
#endif
