/* lcp_sim.c — model of the BWT's list work on one block (diagnostic).
 * Reads a block from a file, builds its cyclic suffix array (prefix doubling, radix sorted) and
 * the LCP of neighbouring rotations, then for every rotation its resolution depth
 * d = max(LCP with either neighbour) + 1 characters. The pipeline's global pass buckets by the
 * first s symbols (compacted alphabet, s = 2 for <= 32 distinct bytes, 3 for <= 10); buckets of
 * <= 4608 rotations take the dense finish, which resolves D1 characters:
 *   raw record    : D1 = (db + 12 + R) / 8, db = 8 s, R = min(32, 44 - P, 52 - db)  (bits -> chars)
 *   packed record : D1 = s + floor((12 + R) / w), w = bits of (k - 1)
 * and list rounds then add 8 characters each. Reported: the rotations in dense / big buckets, and
 * the list element-rounds (sum over dense-bucket rotations of ceil((d - D1) / 8)) both ways.
 * usage: lcp_sim FILE [block_bytes]   (first block of the file) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void radix_pairs(uint32_t n, const uint32_t *k1, const uint32_t *k2, uint32_t *idx, uint32_t *tmp, uint32_t K)
{
    /* stable LSD by k2 then k1 (keys < K) */
    uint32_t *cnt = calloc((size_t)K + 1, 4);
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t *k = pass == 0 ? k2 : k1;
        memset(cnt, 0, ((size_t)K + 1) * 4);
        for (uint32_t i = 0; i < n; ++i) cnt[k[idx[i]] + 1]++;
        for (uint32_t i = 0; i < K; ++i) cnt[i + 1] += cnt[i];
        for (uint32_t i = 0; i < n; ++i) tmp[cnt[k[idx[i]]]++] = idx[i];
        memcpy(idx, tmp, (size_t)n * 4);
    }
    free(cnt);
}

int main(int argc, char **argv)
{
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint32_t n = argc > 2 ? (uint32_t)strtoul(argv[2], 0, 10) : (1u << 20);
    uint8_t *t = malloc(n);
    n = (uint32_t)fread(t, 1, n, f);
    fclose(f);
    uint32_t *sa = malloc((size_t)n * 4), *rk = malloc((size_t)n * 4), *k2 = malloc((size_t)n * 4),
             *tmp = malloc((size_t)n * 4), *nr = malloc((size_t)n * 4);
    for (uint32_t i = 0; i < n; ++i) { sa[i] = i; rk[i] = t[i]; }
    uint32_t K = 256;
    for (uint32_t h = 1;; h <<= 1) {
        for (uint32_t i = 0; i < n; ++i) k2[i] = rk[(i + h) % n];
        radix_pairs(n, rk, k2, sa, tmp, K);
        uint32_t r = 0;
        nr[sa[0]] = 0;
        for (uint32_t i = 1; i < n; ++i) {
            if (rk[sa[i]] != rk[sa[i - 1]] || k2[sa[i]] != k2[sa[i - 1]]) ++r;
            nr[sa[i]] = r;
        }
        memcpy(rk, nr, (size_t)n * 4);
        K = r + 1;
        if (r == n - 1 || h >= n) break;
    }
    /* cyclic LCP of neighbours in SA order (Kasai over the doubled text, capped at n) */
    uint32_t *lcp = calloc(n, 4); /* lcp[i] = LCP(sa[i-1], sa[i]) */
    uint32_t hh = 0;
    for (uint32_t p = 0; p < n; ++p) {
        const uint32_t r = rk[p];
        if (r == 0) { hh = 0; continue; }
        const uint32_t q = sa[r - 1];
        while (hh < n && t[(p + hh) % n] == t[(q + hh) % n]) ++hh;
        lcp[r] = hh;
        if (hh) --hh;
    }
    /* alphabet */
    int seen[256] = {0}, rank8[256], k = 0;
    for (uint32_t i = 0; i < n; ++i) seen[t[i]] = 1;
    for (int c = 0; c < 256; ++c) { rank8[c] = k; k += seen[c]; }
    const uint32_t s = k <= 10 ? 3 : k <= 32 ? 2 : 0;
    const uint32_t P = n <= 2 ? 1 : 32 - __builtin_clz(n - 1);
    const uint32_t db = s ? 8 * s : 10;
    uint32_t R = 44 - P < 32 ? 44 - P : 32;
    if (52 - db < R) R = 52 - db;
    uint32_t w = 0;
    while ((1u << w) < (uint32_t)k) ++w;
    const double D1raw = (db + 12.0 + R) / 8.0;
    const uint32_t D1pk = s ? s + (12 + R) / (w ? w : 1) : 0;
    /* buckets by the first s symbols (or 10 raw bits) */
    uint64_t dense = 0, big = 0, er_raw = 0, er_pk = 0, rounds_raw = 0, rounds_pk = 0;
    uint32_t b0 = 0;
    for (uint32_t i = 1; i <= n; ++i) {
        int same = 0;
        if (i < n) same = lcp[i] >= (s ? s : 2) ; /* raw 10 bits ~ 1.25 chars: approximate by 2 chars */
        if (same) continue;
        const uint32_t m = i - b0;
        for (uint32_t j = b0; j < i; ++j) {
            uint32_t d = lcp[j];
            if (j + 1 < n && lcp[j + 1] > d) d = lcp[j + 1];
            d += 1; /* chars needed to separate the rotation from both neighbours */
            if (m > 4608) { ++big; continue; }
            ++dense;
            const double xr = d - D1raw;
            const uint64_t rr = xr > 0 ? (uint64_t)((xr + 7.999) / 8) : 0;
            const uint64_t rp = d > D1pk ? (d - D1pk + 7) / 8 : 0;
            er_raw += rr;
            er_pk += rp;
            if (rr > rounds_raw) rounds_raw = rr;
            if (rp > rounds_pk) rounds_pk = rp;
        }
        b0 = i;
    }
    printf("{\"n\": %u, \"k\": %d, \"s\": %u, \"w\": %u, \"P\": %u, \"R\": %u, \"D1_raw_chars\": %.2f, \"D1_packed_chars\": %u, "
           "\"dense_rotations\": %llu, \"big_bucket_rotations\": %llu, \"list_element_rounds_raw\": %llu, "
           "\"list_element_rounds_packed\": %llu, \"per_dense_rotation_raw\": %.3f, \"per_dense_rotation_packed\": %.3f, "
           "\"max_rounds_raw\": %llu, \"max_rounds_packed\": %llu}\n",
           n, k, s, w, P, R, D1raw, D1pk, (unsigned long long)dense, (unsigned long long)big, (unsigned long long)er_raw,
           (unsigned long long)er_pk, dense ? (double)er_raw / dense : 0, dense ? (double)er_pk / dense : 0,
           (unsigned long long)rounds_raw, (unsigned long long)rounds_pk);
    return 0;
}
