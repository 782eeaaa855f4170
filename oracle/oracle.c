/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h). A from-scratch C restatement of the
 * reference encode/decode path, written from the behaviour of /root/reference/main.cpp and
 * io_utilities.h (cited per function). No reference source is copied here.
 *
 * Parity pinned against records of the real reference (tests/golden/, produced by
 * oracle/_ref/ref_COMPRESS); tests/test_oracle.py checks this file against them.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ BWT (faithful) */
/* Reference: cyclic_index main.cpp:38-44, bwt_cmp_straight main.cpp:46-59.
 * Compare rotation l vs r byte by byte for up to n bytes; equal => "not less". */
static int rot_less(const uint8_t *d, size_t n, size_t l, size_t r)
{
    size_t i = 0;
    size_t a = l, b = r;
    while (i < n && d[a] == d[b]) {
        ++i;
        if (++a == n) a = 0;
        if (++b == n) b = 0;
    }
    return d[a] < d[b];
}

/* std::stable_sort equivalent: top-down merge sort keeping index order on ties. */
static void merge_sort(const uint8_t *d, size_t n, uint64_t *v, uint64_t *tmp, size_t lo, size_t hi)
{
    if (hi - lo < 2) return;
    size_t mid = lo + (hi - lo) / 2;
    merge_sort(d, n, v, tmp, lo, mid);
    merge_sort(d, n, v, tmp, mid, hi);
    size_t i = lo, j = mid, k = lo;
    while (i < mid && j < hi) {
        if (rot_less(d, n, v[j], v[i])) tmp[k++] = v[j++];
        else tmp[k++] = v[i++];
    }
    while (i < mid) tmp[k++] = v[i++];
    while (j < hi) tmp[k++] = v[j++];
    memcpy(v + lo, tmp + lo, (hi - lo) * sizeof(uint64_t));
}

/* Reference: bwt main.cpp:77-91 — L[r] = data[(SA[r]+n-1) mod n]; primary = r with SA[r]==0. */
int orc_bwt_ref(const uint8_t *data, size_t n, uint8_t *L, uint64_t *primary)
{
    if (n == 0) return -1; /* the reference segfaults on empty input */
    uint64_t *sa = malloc(n * sizeof(uint64_t));
    uint64_t *tmp = malloc(n * sizeof(uint64_t));
    if (!sa || !tmp) { free(sa); free(tmp); return -1; }
    for (size_t i = 0; i < n; ++i) sa[i] = i;
    merge_sort(data, n, sa, tmp, 0, n);
    for (size_t r = 0; r < n; ++r) {
        L[r] = data[(sa[r] + n - 1) % n];
        if (sa[r] == 0) *primary = r;
    }
    free(sa);
    free(tmp);
    return 0;
}

/* ------------------------------------------------------------ BWT (prefix doubling) */
/* Same output as orc_bwt_ref: sort rotations by (rank_k[i], rank_k[(i+k)%n]);
 * rank = number of rotations with a strictly smaller k-prefix; stop when all ranks are
 * distinct or k >= n (remaining ties are identical rotations, whose L bytes are equal and
 * whose primary index is the count of strictly smaller rotations). */
static const uint64_t *g_r1, *g_r2;
static int cmp_pair(const void *pa, const void *pb)
{
    uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
    if (g_r1[a] != g_r1[b]) return g_r1[a] < g_r1[b] ? -1 : 1;
    if (g_r2[a] != g_r2[b]) return g_r2[a] < g_r2[b] ? -1 : 1;
    return a < b ? -1 : (a > b);
}

int orc_bwt_fast(const uint8_t *data, size_t n, uint8_t *L, uint64_t *primary)
{
    if (n == 0) return -1;
    uint64_t *sa = malloc(n * 8), *rk = malloc(n * 8), *r2 = malloc(n * 8), *nr = malloc(n * 8);
    if (!sa || !rk || !r2 || !nr) { free(sa); free(rk); free(r2); free(nr); return -1; }
    /* depth 1: rank = count of strictly smaller bytes */
    uint64_t cnt[257] = {0};
    for (size_t i = 0; i < n; ++i) cnt[data[i] + 1]++;
    for (int c = 0; c < 256; ++c) cnt[c + 1] += cnt[c];
    for (size_t i = 0; i < n; ++i) rk[i] = cnt[data[i]];
    for (size_t i = 0; i < n; ++i) sa[i] = i;
    size_t k = 1;
    for (;;) {
        for (size_t i = 0; i < n; ++i) r2[i] = rk[(i + k) % n];
        g_r1 = rk; g_r2 = r2;
        qsort(sa, n, 8, cmp_pair);
        size_t distinct = 1;
        nr[sa[0]] = 0;
        size_t head = 0;
        for (size_t j = 1; j < n; ++j) {
            if (rk[sa[j]] != rk[sa[j - 1]] || r2[sa[j]] != r2[sa[j - 1]]) { head = j; ++distinct; }
            nr[sa[j]] = head;
        }
        uint64_t *t = rk; rk = nr; nr = t;
        k *= 2;
        if (distinct == n || k >= n) break;
    }
    for (size_t r = 0; r < n; ++r) L[r] = data[(sa[r] + n - 1) % n];
    *primary = rk[0];
    free(sa); free(rk); free(r2); free(nr);
    return 0;
}

/* --------------------------------------------------------------------------- MTF */
/* Reference: move_to_front main.cpp:93-112 (find_if over the alphabet, rotate to front). */
void orc_mtf(const uint8_t *in, size_t n, uint8_t *out)
{
    uint8_t a[256];
    for (int i = 0; i < 256; ++i) a[i] = (uint8_t)i;
    for (size_t i = 0; i < n; ++i) {
        uint8_t c = in[i];
        int j = 0;
        while (a[j] != c) ++j;
        out[i] = (uint8_t)j;
        memmove(a + 1, a, (size_t)j);
        a[0] = c;
    }
}

/* Reference: move_to_front_reverse main.cpp:114-130. */
void orc_mtf_inverse(const uint8_t *in, size_t n, uint8_t *out)
{
    uint8_t a[256];
    for (int i = 0; i < 256; ++i) a[i] = (uint8_t)i;
    for (size_t i = 0; i < n; ++i) {
        int j = in[i];
        uint8_t c = a[j];
        out[i] = c;
        memmove(a + 1, a, (size_t)j);
        a[0] = c;
    }
}

/* ------------------------------------------------------------------- inverse BWT */
/* Reference: bwt_reverse main.cpp:61-75 — l_shift = stable sort of row indices by L byte
 * (bwt_cmp_reverse main.cpp:28-36); out[i] = L[l_shift[row]]; row = l_shift[row]. */
int orc_bwt_inverse(const uint8_t *L, size_t n, uint64_t primary, uint8_t *out)
{
    if (n == 0 || primary >= n) return -1;
    uint64_t *ls = malloc(n * 8);
    if (!ls) return -1;
    uint64_t cnt[257] = {0};
    for (size_t i = 0; i < n; ++i) cnt[L[i] + 1]++;
    for (int c = 0; c < 256; ++c) cnt[c + 1] += cnt[c];
    for (size_t i = 0; i < n; ++i) ls[cnt[L[i]]++] = i; /* counting sort == stable sort */
    uint64_t row = primary;
    for (size_t i = 0; i < n; ++i) {
        out[i] = L[ls[row]];
        row = ls[row];
    }
    free(ls);
    return 0;
}

/* ------------------------------------------------------------------------ Huffman */
/* Reference: huffman main.cpp:231-244 — histogram, then leaves pushed in first-occurrence
 * order of the MTF stream. */
void orc_histogram(const uint8_t *mtf, size_t n, uint64_t freq[256], uint64_t first[256])
{
    for (int s = 0; s < 256; ++s) { freq[s] = 0; first[s] = UINT64_MAX; }
    for (size_t i = 0; i < n; ++i) {
        if (first[mtf[i]] == UINT64_MAX) first[mtf[i]] = i;
        freq[mtf[i]]++;
    }
}

/* ascending heap-address order of the BTree nodes of a standalone
 * COMPRESS run under glibc 2.35, as a function of the leaf count L. Node ids: leaves 0..L-1
 * in first-occurrence order, internal nodes L, L+1, ... in creation order. The priority
 * queue element is (-freq, BTree*) (main.cpp:232,241,253): among equal frequencies the node
 * with the higher address pops first. */
static void addr_ranks(int L, int *rank)
{
    int total = 2 * L - 1, k = 0;
    int order[512];
    int m = 0;
    if (L <= 128) {
        order[m++] = 1;
        for (int s = 3; s <= 127; ++s) order[m++] = s;
        order[m++] = 0;
        order[m++] = 2;
        for (int s = 128; s < 512; ++s) order[m++] = s;
    } else {
        order[m++] = 1;
        for (int s = 3; s <= 64; ++s) order[m++] = s;
        for (int s = 129; s <= 192; ++s) order[m++] = s;
        for (int s = 65; s <= 127; ++s) order[m++] = s;
        order[m++] = 0;
        order[m++] = 2;
        order[m++] = 128;
        for (int s = 193; s < 512; ++s) order[m++] = s;
    }
    for (int i = 0; i < m; ++i)
        if (order[i] < total) rank[order[i]] = k++;
}

typedef struct { uint64_t f; int sym; int left, right; } onode;

static void assign_codes(const onode *nd, int v, uint64_t code, int depth, uint8_t *len, uint64_t *codes,
                         int *err)
{
    /* Reference: traverse main.cpp:132-147 — left = 0, right = 1; root leaf = empty code. */
    if (nd[v].left < 0) {
        if (depth > 64) { *err = 1; return; }
        len[nd[v].sym] = (uint8_t)depth;
        codes[nd[v].sym] = code;
        return;
    }
    assign_codes(nd, nd[v].left, code << 1, depth + 1, len, codes, err);
    assign_codes(nd, nd[v].right, (code << 1) | 1u, depth + 1, len, codes, err);
}

typedef struct { uint8_t *buf; size_t cap, bits; int err; } bitw;
static void bw_put(bitw *w, int bit)
{
    /* Reference: append_bit io_utilities.h:87-94 — MSB-first within each byte. */
    size_t byte = w->bits >> 3;
    if (byte >= w->cap) { w->err = 1; return; }
    if ((w->bits & 7) == 0) w->buf[byte] = 0;
    if (bit) w->buf[byte] |= (uint8_t)(0x80u >> (w->bits & 7));
    w->bits++;
}

static void tree_dfs(const onode *nd, int v, bitw *w)
{
    /* Reference: dfs main.cpp:174-187 — internal = 1; leaf = 0 + 8 value bits MSB-first. */
    if (nd[v].left < 0) {
        bw_put(w, 0);
        for (int b = 7; b >= 0; --b) bw_put(w, (nd[v].sym >> b) & 1);
        return;
    }
    bw_put(w, 1);
    tree_dfs(nd, nd[v].left, w);
    tree_dfs(nd, nd[v].right, w);
}

int orc_huffman_build(const uint64_t freq[256], const uint64_t first[256], uint8_t len[256],
                      uint64_t code[256], uint8_t *tree_out, size_t tree_cap)
{
    onode nd[511];
    int leaves[256], L = 0;
    /* leaves in first-occurrence order (main.cpp:238-244) */
    int syms[256];
    for (int s = 0; s < 256; ++s) syms[s] = s;
    for (int i = 0; i < 256; ++i)
        for (int j = i + 1; j < 256; ++j)
            if (first[syms[j]] < first[syms[i]]) { int t = syms[i]; syms[i] = syms[j]; syms[j] = t; }
    for (int i = 0; i < 256; ++i)
        if (freq[syms[i]] > 0) leaves[L++] = syms[i];
    if (L == 0) return -1;
    int rank[512];
    addr_ranks(L, rank);
    int alive[511], nalive = 0, nn = 0;
    for (int i = 0; i < L; ++i) {
        nd[nn] = (onode){freq[leaves[i]], leaves[i], -1, -1};
        alive[nalive++] = nn++;
    }
    /* main.cpp:245-254: pop a (left), pop b (right), push (a+b). */
    while (nalive > 1) {
        int pick[2];
        for (int t = 0; t < 2; ++t) {
            int best = 0;
            for (int i = 1; i < nalive; ++i) {
                const onode *x = &nd[alive[i]], *y = &nd[alive[best]];
                if (x->f < y->f || (x->f == y->f && rank[alive[i]] > rank[alive[best]])) best = i;
            }
            pick[t] = alive[best];
            alive[best] = alive[--nalive];
        }
        nd[nn] = (onode){nd[pick[0]].f + nd[pick[1]].f, 0, pick[0], pick[1]};
        alive[nalive++] = nn++;
    }
    int root = alive[0], err = 0;
    memset(len, 0, 256);
    memset(code, 0, 256 * sizeof(uint64_t));
    assign_codes(nd, root, 0, 0, len, code, &err);
    if (err) return -1;
    bitw w = {tree_out, tree_cap, 0, 0};
    tree_dfs(nd, root, &w);
    if (w.err) return -1;
    return (int)((w.bits + 7) / 8);
}

/* ------------------------------------------------------------------ record encode */
static void put_u64(uint8_t *p, uint64_t v)
{
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
static uint64_t get_u64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

size_t orc_record_bound(size_t n) { return 24 + 320 + 8 * n + 16; }

/* Reference: compress main.cpp:300-325 + write_bytes io_utilities.h:7-27:
 * [u64 primary][u64 n][u64 tree_len][tree][payload], payload = max(1, ceil(B/8)) bytes
 * (encode_with_huffman main.cpp:158-172 starts from one zero byte). */
int64_t orc_encode_record(const uint8_t *data, size_t n, uint8_t *out, size_t cap, int use_ref_bwt)
{
    if (n == 0 || cap < orc_record_bound(n)) return -1;
    uint8_t *Lb = malloc(n), *m = malloc(n);
    if (!Lb || !m) { free(Lb); free(m); return -1; }
    uint64_t primary = 0;
    int rc = use_ref_bwt ? orc_bwt_ref(data, n, Lb, &primary) : orc_bwt_fast(data, n, Lb, &primary);
    if (rc) { free(Lb); free(m); return -1; }
    orc_mtf(Lb, n, m);
    uint64_t freq[256], first[256], code[256];
    uint8_t len[256], tree[512];
    orc_histogram(m, n, freq, first);
    int tlen = orc_huffman_build(freq, first, len, code, tree, sizeof tree);
    if (tlen < 0) { free(Lb); free(m); return -1; }
    put_u64(out, primary);
    put_u64(out + 8, n);
    put_u64(out + 16, (uint64_t)tlen);
    memcpy(out + 24, tree, (size_t)tlen);
    bitw w = {out + 24 + tlen, cap - 24 - (size_t)tlen, 0, 0};
    for (size_t i = 0; i < n; ++i) {
        int l = len[m[i]];
        for (int b = l - 1; b >= 0; --b) bw_put(&w, (int)((code[m[i]] >> b) & 1));
    }
    size_t pbytes = (w.bits + 7) / 8;
    if (pbytes == 0) { out[24 + tlen] = 0; pbytes = 1; }
    free(Lb);
    free(m);
    if (w.err) return -1;
    return (int64_t)(24 + (size_t)tlen + pbytes);
}

/* ------------------------------------------------------------------ record decode */
typedef struct { const uint8_t *p; size_t len, bit; int err; } bitr;
static int br_get(bitr *r)
{
    /* Reference: read_bit io_utilities.h:61-72 — MSB-first. */
    size_t byte = r->bit >> 3;
    if (byte >= r->len) { r->err = 1; return 0; }
    int b = (r->p[byte] >> (7 - (r->bit & 7))) & 1;
    r->bit++;
    return b;
}

typedef struct { int left, right, sym; } dnode;
static int parse_tree(bitr *r, dnode *nd, int *nn, int depth)
{
    /* Reference: bytes_to_tree_dfs main.cpp:198-219. */
    if (*nn >= 511 || depth > 300 || r->err) { r->err = 1; return -1; }
    int v = (*nn)++;
    if (!br_get(r)) {
        int s = 0;
        for (int i = 0; i < 8; ++i) s = (s << 1) | br_get(r);
        nd[v] = (dnode){-1, -1, s};
        return v;
    }
    nd[v].sym = 0;
    int l = parse_tree(r, nd, nn, depth + 1);
    int rr = parse_tree(r, nd, nn, depth + 1);
    nd[v].left = l;
    nd[v].right = rr;
    return v;
}

int64_t orc_decode_to_mtf(const uint8_t *rec, size_t len, uint8_t *mtf_out, size_t cap)
{
    if (len < 24) return -1;
    uint64_t n = get_u64(rec + 8), tlen = get_u64(rec + 16);
    if (24 + tlen > len || n > cap) return -1;
    dnode nd[511];
    int nn = 0;
    bitr tr = {rec + 24, (size_t)tlen, 0, 0};
    int root = parse_tree(&tr, nd, &nn, 0);
    if (tr.err || root < 0) return -1;
    bitr pr = {rec + 24 + tlen, len - 24 - (size_t)tlen, 0, 0};
    /* Reference: huffman_reverse main.cpp:259-281 — walk from the root bit by bit. */
    for (uint64_t i = 0; i < n; ++i) {
        int v = root;
        while (nd[v].left >= 0) {
            v = br_get(&pr) ? nd[v].right : nd[v].left;
            if (pr.err) return -1;
        }
        mtf_out[i] = (uint8_t)nd[v].sym;
    }
    return (int64_t)n;
}

int64_t orc_decode_record(const uint8_t *rec, size_t len, uint8_t *out, size_t cap)
{
    if (len < 24) return -1;
    uint64_t primary = get_u64(rec), n = get_u64(rec + 8);
    if (n == 0 || n > cap) return -1;
    uint8_t *m = malloc(n), *Lb = malloc(n);
    if (!m || !Lb) { free(m); free(Lb); return -1; }
    int64_t got = orc_decode_to_mtf(rec, len, m, n);
    int64_t ret = -1;
    if (got == (int64_t)n) {
        orc_mtf_inverse(m, n, Lb);
        if (orc_bwt_inverse(Lb, n, primary, out) == 0) ret = (int64_t)n;
    }
    free(m);
    free(Lb);
    return ret;
}

/* ---- synthetic Zipf text (not reference code: the config-5 input) ----
 * A sequential restatement of the App. D generator, used as the checker of the device generator
 * (bmh_synth_zipf_dev) and to stream the 8 GiB config-5 input through the reference when the
 * golden manifest is made (tests/golden/make_golden.py). */
#define ORC_ZIPF_VOCAB 8192
struct orc_zipf {
    uint64_t cdf[ORC_ZIPF_VOCAB];
    uint8_t word[ORC_ZIPF_VOCAB][12]; /* letters + ' ' */
    uint8_t wlen[ORC_ZIPF_VOCAB];     /* including the space */
    uint64_t tok;                     /* tokens drawn so far from splitmix64(seed 2) */
    uint8_t pend[12];                 /* tail of a token cut at the previous call's end */
    int npend, ipend;
};

static uint64_t sm64_at(uint64_t seed, uint64_t k) /* k-th output, k >= 1 */
{
    uint64_t z = seed + k * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

size_t orc_zipf_state_size(void) { return sizeof(struct orc_zipf); }

void orc_zipf_init(struct orc_zipf *z)
{
    uint64_t k = 0, acc = 0;
    for (int w = 0; w < ORC_ZIPF_VOCAB; ++w) {
        uint64_t r = sm64_at(1, ++k);
        int ln = 2 + (int)(r % 9);
        for (int i = 0; i < ln; ++i) z->word[w][i] = (uint8_t)('a' + sm64_at(1, ++k) % 26);
        z->word[w][ln] = ' ';
        z->wlen[w] = (uint8_t)(ln + 1);
        acc += (1ull << 32) / (uint64_t)(w + 1);
        z->cdf[w] = acc;
    }
    z->tok = 0;
    z->npend = z->ipend = 0;
}

/* Next n bytes of the stream. */
void orc_zipf_fill(struct orc_zipf *z, uint8_t *out, size_t n)
{
    size_t o = 0;
    const uint64_t T = z->cdf[ORC_ZIPF_VOCAB - 1];
    while (o < n && z->ipend < z->npend) out[o++] = z->pend[z->ipend++];
    while (o < n) {
        uint64_t x = sm64_at(2, ++z->tok) % T;
        int lo = 0, hi = ORC_ZIPF_VOCAB - 1; /* first k with cdf[k] > x */
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (z->cdf[mid] > x) hi = mid; else lo = mid + 1;
        }
        int ln = z->wlen[lo];
        if (o + (size_t)ln <= n) {
            memcpy(out + o, z->word[lo], (size_t)ln);
            o += (size_t)ln;
        } else {
            int take = (int)(n - o);
            memcpy(out + o, z->word[lo], (size_t)take);
            o = n;
            memcpy(z->pend, z->word[lo] + take, (size_t)(ln - take));
            z->npend = ln - take;
            z->ipend = 0;
        }
    }
}
