// synth.hip — the benchmark configs' synthetic inputs, generated in HBM.
//
//   splitmix64(seed) bytes (config 4): counter-based, one 8-byte word per thread.
//   integer-Zipf text (configs 3 and 5): vocabulary of 8192 words from splitmix64(seed 1)
//   (length 2 + r % 9, letters 'a' + next() % 26), token k from splitmix64(seed 2): x = next() % T,
//   word = first w with cdf[w] > x (cdf = inclusive sum of floor(2^32 / (w + 1))), emitted as
//   word + ' '. The text is a sequential concatenation, so the device form draws tokens in rounds
//   of 2^26: count (per-workgroup byte sums), scan (token-run start positions, carried across
//   rounds on the device), write (each thread re-draws its 16 tokens and stores the bytes that fall
//   in the requested window). Any window [offset, offset + nbytes) of the stream can be produced;
//   rounds before the window only count. Checked against the App. D sha256 and the oracle's
//   sequential generator (tests/test_gpu_parity.py::test_device_zipf_matches_oracle).
#include "device_util.h"

namespace bmh {
namespace {

constexpr uint32_t kZipfVocab = 8192;
constexpr uint32_t kZipfNT = 256;          // threads per workgroup
constexpr uint32_t kZipfE = 16;            // consecutive tokens per thread
constexpr uint32_t kZipfWG = kZipfNT * kZipfE;
constexpr uint32_t kZipfRoundWG = 16384;   // workgroups per round
constexpr uint64_t kZipfRound = (uint64_t)kZipfWG * kZipfRoundWG;  // 2^26 tokens

__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_splitmix(uint8_t *__restrict__ out, uint64_t nbytes, uint64_t seed, uint64_t offset)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * 8;
    if (i0 >= nbytes) return;
    const uint64_t g = offset + i0;
    const uint64_t w = g >> 3;
    const uint32_t s = (uint32_t)(g & 7u);
    const uint64_t z0 = splitmix_word(seed, w);
    uint64_t v = z0 >> (8 * s);
    if (s) v |= splitmix_word(seed, w + 1) << (64 - 8 * s);
    if (i0 + 8 <= nbytes && (((uintptr_t)(out + i0)) & 7u) == 0) {
        *(uint64_t *)(out + i0) = v;
    } else {
        for (uint32_t j = 0; j < 8 && i0 + j < nbytes; ++j) out[i0 + j] = (uint8_t)(v >> (8 * j));
    }
}

// Word id of token k (0-based) of the stream: first w with cdf[w] > x, cdf staged in LDS.
__device__ __forceinline__ uint32_t zipf_word(const uint64_t *s_cdf, uint64_t T, uint64_t k)
{
    const uint64_t x = splitmix_word(2, k) % T;
    uint32_t lo = 0, hi = kZipfVocab - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_cdf[mid] > x) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

__device__ __forceinline__ void stage_cdf(const uint64_t *__restrict__ cdf, uint64_t *s_cdf)
{
    for (uint32_t i = threadIdx.x; i < kZipfVocab; i += kZipfNT) s_cdf[i] = cdf[i];
    __syncthreads();
}

// Per-workgroup byte count of tokens [tok0 + wg * kZipfWG, +kZipfWG).
__global__ __launch_bounds__(kZipfNT) void k_zipf_count(const uint64_t *__restrict__ cdf,
                                                         const uint8_t *__restrict__ wlen, uint64_t tok0,
                                                         uint32_t *__restrict__ part)
{
    __shared__ uint64_t s_cdf[kZipfVocab];
    __shared__ uint32_t s_tmp[kZipfNT / 64 + 1];
    stage_cdf(cdf, s_cdf);
    const uint64_t T = s_cdf[kZipfVocab - 1];
    const uint64_t k0 = tok0 + ((uint64_t)blockIdx.x * kZipfNT + threadIdx.x) * kZipfE;
    uint32_t sum = 0;
#pragma unroll 4
    for (uint32_t e = 0; e < kZipfE; ++e) sum += wlen[zipf_word(s_cdf, T, k0 + e)];
    uint32_t tot;
    block_excl_sum1<kZipfNT>(sum, s_tmp, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// Exclusive scan of the round's workgroup counts into stream positions (u64), base carried in
// base[0] across rounds. One workgroup of 1024 threads, kZipfRoundWG / 1024 counts per thread.
__global__ __launch_bounds__(1024) void k_zipf_scan(const uint32_t *__restrict__ part, uint64_t *__restrict__ start,
                                                     uint64_t *__restrict__ base)
{
    __shared__ uint64_t s_tmp[1024 / 64 + 1];
    constexpr uint32_t PER = kZipfRoundWG / 1024;
    const uint32_t t = threadIdx.x;
    uint64_t v[PER], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        v[j] = part[t * PER + j];
        sum += v[j];
    }
    uint64_t tot;
    uint64_t pre = block_excl_sum64<1024>(sum, s_tmp, &tot) + base[0];
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        start[t * PER + j] = pre;
        pre += v[j];
    }
    __syncthreads();
    if (t == 0) base[0] += tot;
}

// Bytes of the round's tokens that fall inside [offset, offset + nbytes), stored at out[p - offset].
__global__ __launch_bounds__(kZipfNT) void k_zipf_write(const uint64_t *__restrict__ cdf,
                                                         const uint4 *__restrict__ words, uint64_t tok0,
                                                         const uint64_t *__restrict__ start, uint8_t *__restrict__ out,
                                                         uint64_t offset, uint64_t nbytes)
{
    __shared__ uint64_t s_cdf[kZipfVocab];
    __shared__ uint32_t s_tmp[kZipfNT / 64 + 1];
    const uint64_t wg0 = start[blockIdx.x];
    if (wg0 >= offset + nbytes) return;  // uniform: the whole workgroup starts past the window
    stage_cdf(cdf, s_cdf);
    const uint64_t T = s_cdf[kZipfVocab - 1];
    const uint64_t k0 = tok0 + ((uint64_t)blockIdx.x * kZipfNT + threadIdx.x) * kZipfE;
    uint16_t id[kZipfE];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t e = 0; e < kZipfE; ++e) {
        id[e] = (uint16_t)zipf_word(s_cdf, T, k0 + e);
        sum += (uint32_t)(words[id[e]].w >> 24);  // length (incl. the space) in byte 15
    }
    uint64_t p = wg0 + block_excl_sum1<kZipfNT>(sum, s_tmp);
    if (p + sum <= offset || p >= offset + nbytes) return;
    const uint64_t end = offset + nbytes;
#pragma unroll 1
    for (uint32_t e = 0; e < kZipfE; ++e) {
        const uint4 w = words[id[e]];
        const uint32_t ln = w.w >> 24;
        const uint32_t q[4] = {w.x, w.y, w.z, w.w};
        for (uint32_t j = 0; j < ln; ++j, ++p)
            if (p >= offset && p < end) out[p - offset] = (uint8_t)(q[j >> 2] >> (8 * (j & 3)));
    }
}

struct ZipfTables {
    uint64_t cdf[kZipfVocab];
    uint8_t wlen[kZipfVocab];
    uint8_t words[kZipfVocab][16];  // letters, ' ', zero pad; byte 15 = length incl. the space
};

const ZipfTables &zipf_tables()
{
    static const ZipfTables t = [] {
        ZipfTables z{};
        uint64_t k = 0, acc = 0;
        auto next = [&] {
            uint64_t x = 1 + (++k) * 0x9E3779B97F4A7C15ull;
            x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
            x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
            return x ^ (x >> 31);
        };
        for (uint32_t w = 0; w < kZipfVocab; ++w) {
            const uint32_t ln = 2 + (uint32_t)(next() % 9);
            for (uint32_t i = 0; i < ln; ++i) z.words[w][i] = (uint8_t)('a' + next() % 26);
            z.words[w][ln] = ' ';
            z.words[w][15] = (uint8_t)(ln + 1);
            z.wlen[w] = (uint8_t)(ln + 1);
            acc += (1ull << 32) / (w + 1);
            z.cdf[w] = acc;
        }
        return z;
    }();
    return t;
}

}  // namespace

void synth_splitmix64(Ctx *c, uint8_t *d_out, uint64_t nbytes, uint64_t seed, uint64_t offset)
{
    const uint64_t threads = (nbytes + 7) / 8;
    BMH_LAUNCH(c, "synth_splitmix64", k_splitmix, (uint32_t)((threads + 255) / 256), 256, 0, d_out, nbytes, seed, offset);
    c->sync();
}

void synth_zipf(Ctx *c, uint8_t *d_out, uint64_t nbytes, uint64_t offset)
{
    const ZipfTables &zt = zipf_tables();
    // device tables: cdf | words | wlen | base (u64) | part (u32 per workgroup) | start (u64)
    const size_t o_words = sizeof zt.cdf, o_wlen = o_words + sizeof zt.words, o_base = o_wlen + sizeof zt.wlen,
                 o_part = o_base + 64, o_start = o_part + kZipfRoundWG * 4, bytes = o_start + kZipfRoundWG * 8;
    uint8_t *d = (uint8_t *)c->get(WS_SYNTH, bytes);
    if (c->ws_tag[WS_SYNTH] != 1) {
        c->h2d(d, zt.cdf, sizeof zt.cdf);
        c->h2d(d + o_words, zt.words, sizeof zt.words);
        c->h2d(d + o_wlen, zt.wlen, sizeof zt.wlen);
        c->ws_tag[WS_SYNTH] = 1;
    }
    const uint64_t *d_cdf = (const uint64_t *)d;
    uint64_t *d_base = (uint64_t *)(d + o_base);
    uint32_t *d_part = (uint32_t *)(d + o_part);
    uint64_t *d_start = (uint64_t *)(d + o_start);
    // resume from the round the previous call ended in when this window starts at or after it
    // (a stream generated piece by piece), else from token 0: d_base = bytes before
    // the first round run
    uint64_t tok0 = 0, h_base = 0;
    if (c->zipf_resume_tok0 && offset >= c->zipf_resume_base) {
        tok0 = c->zipf_resume_tok0;
        h_base = c->zipf_resume_base;
    }
    c->h2d(d_base, &h_base, 8);
    for (;; tok0 += kZipfRound) {
        c->zipf_resume_tok0 = tok0;
        c->zipf_resume_base = h_base;
        BMH_LAUNCH(c, "synth_zipf_count", k_zipf_count, kZipfRoundWG, kZipfNT, 0, d_cdf, d + o_wlen, tok0, d_part);
        BMH_LAUNCH(c, "synth_zipf_scan", k_zipf_scan, 1, 1024, 0, d_part, d_start, d_base);
        BMH_LAUNCH(c, "synth_zipf_write", k_zipf_write, kZipfRoundWG, kZipfNT, 0, d_cdf, (const uint4 *)(d + o_words),
                   tok0, d_start, d_out, offset, nbytes);
        c->d2h(&h_base, d_base, 8);
        c->sync();
        if (h_base >= offset + nbytes) break;
    }
}

}  // namespace bmh
