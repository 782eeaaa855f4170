/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. A from-scratch C restatement of the reference
 * komour/bwt-mtf-huffman-compressor encode/decode path, used as the parity checker.
 * The product (libbmh) never links or calls this; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may.
 *
 * Parity pinning: checked against the golden records produced by the real reference
 * (oracle/_ref/ref_COMPRESS, built from /root/reference/main.cpp by oracle/Makefile) and
 * committed under tests/golden/ (see tests/golden/make_golden.py).
 */
#ifndef BMH_ORACLE_H
#define BMH_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Cyclic-rotation BWT, algorithm-faithful: stable merge sort of rotation indices with a
 * byte-wise cyclic comparator (main.cpp:38-59, 77-91). O(n log n * LCP). */
int orc_bwt_ref(const uint8_t *data, size_t n, uint8_t *L, uint64_t *primary);
/* Same result by prefix doubling on cyclic ranks; O(n log^2 n) worst case. */
int orc_bwt_fast(const uint8_t *data, size_t n, uint8_t *L, uint64_t *primary);
/* Move-to-front over the 256-symbol alphabet initialised 0..255 (main.cpp:93-112). */
void orc_mtf(const uint8_t *in, size_t n, uint8_t *out);
/* Inverse MTF (main.cpp:114-130). */
void orc_mtf_inverse(const uint8_t *in, size_t n, uint8_t *out);
/* Inverse BWT: stable sort of L by byte, then the chase from the primary row (main.cpp:61-75). */
int orc_bwt_inverse(const uint8_t *L, size_t n, uint64_t primary, uint8_t *out);
/* Huffman histogram + first-occurrence ranks of the MTF stream (main.cpp:231-244).
 * freq[256]; first[256] = first index of each symbol (UINT64_MAX if absent). */
void orc_histogram(const uint8_t *mtf, size_t n, uint64_t freq[256], uint64_t first[256]);
/* Build the reference's Huffman tree with the glibc-2.35 address-rank tie-break
 * (main.cpp:245-254). Outputs per-symbol code length and code
 * (MSB-first, right-aligned in code[s]; lengths <= 64), and the preorder tree bytes
 * (main.cpp:174-196). Returns the tree byte count, or -1 on error. */
int orc_huffman_build(const uint64_t freq[256], const uint64_t first[256], uint8_t len[256],
                      uint64_t code[256], uint8_t *tree_out, size_t tree_cap);
/* Whole-block encode to the reference record (main.cpp:300-325, io_utilities.h:7-27).
 * use_ref_bwt selects orc_bwt_ref vs orc_bwt_fast. Returns record length or -1. */
int64_t orc_encode_record(const uint8_t *data, size_t n, uint8_t *out, size_t cap, int use_ref_bwt);
/* Upper bound on a record's size for n input bytes. */
size_t orc_record_bound(size_t n);
/* Decode one reference record (main.cpp:327-345). Returns n or -1. */
int64_t orc_decode_record(const uint8_t *rec, size_t len, uint8_t *out, size_t cap);
/* Huffman-decode only (main.cpp:259-281): record -> MTF stream. Returns n or -1. */
int64_t orc_decode_to_mtf(const uint8_t *rec, size_t len, uint8_t *mtf_out, size_t cap);

/* SURVEY App. D integer-Zipf text stream (config 5's input), generated sequentially:
 * state of orc_zipf_state_size() bytes, orc_zipf_init, then orc_zipf_fill for the next n bytes. */
struct orc_zipf;
size_t orc_zipf_state_size(void);
void orc_zipf_init(struct orc_zipf *z);
void orc_zipf_fill(struct orc_zipf *z, uint8_t *out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
