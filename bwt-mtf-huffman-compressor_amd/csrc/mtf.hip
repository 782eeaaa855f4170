// mtf.hip — move-to-front of a batch of BWT last columns, plus the Huffman histogram and
// first-occurrence scan of its output.
//
// Replaces move_to_front() (reference main.cpp:93-112: find_if + std::rotate over a 256-byte
// alphabet initialised 0..255) and the two O(n) scans at the top of huffman()
// (main.cpp:231-244). MTF is sequential per block, so each block is cut into chunks:
//   1. recency  : per chunk, its distinct symbols ordered by last occurrence (most recent
//                 first) — LDS atomicMax of positions, then a rank count.
//   2. compose  : per block, one wave walks its chunks in order: state_{c+1} =
//                 recency_c ++ (state_c minus recency_c); writes each chunk's start state.
//   3. encode   : one wave per chunk runs MTF from its start state. The alphabet is held as
//                 pos[s] (current index of symbol s), 4 symbols per lane in 4 VGPRs; a step
//                 is readlane(pos[c]) + "pos += pos < pc" on all 256 entries + writelane 0.
//                 Output bytes also feed per-wave LDS histograms / first-occurrence minima.
#include "bmh_internal.h"
#include "device_util.h"

#include <algorithm>

namespace bmh {

namespace {

struct MChunk {
    uint32_t block, start, len, rel;  // rel = start - block offset
};

__global__ __launch_bounds__(256) void k_mtf_recency(const uint8_t *__restrict__ L, const MChunk *__restrict__ chunks,
                                                     uint8_t *__restrict__ R, uint32_t *__restrict__ dcount)
{
    __shared__ int lastpos[256];
    const MChunk ch = chunks[blockIdx.x];
    lastpos[threadIdx.x] = -1;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < ch.len; i += 256) atomicMax(&lastpos[L[ch.start + i]], (int)i);
    __syncthreads();
    const int lp = lastpos[threadIdx.x];
    uint32_t rank = 0;
    for (int s = 0; s < 256; ++s) rank += lastpos[s] > lp;
    const int d = __syncthreads_count(lp >= 0);
    if (lp >= 0) R[(size_t)blockIdx.x * 256 + rank] = (uint8_t)threadIdx.x;
    if (threadIdx.x == 0) dcount[blockIdx.x] = (uint32_t)d;
}

// grid = nblocks, one wave each.
__global__ __launch_bounds__(64) void k_mtf_compose(const uint32_t *__restrict__ chunk_first,
                                                    const uint8_t *__restrict__ R, const uint32_t *__restrict__ dcount,
                                                    uint32_t *__restrict__ S)
{
    __shared__ uint8_t s_S[256], s_flag[256];
    const uint32_t b = blockIdx.x, l = threadIdx.x;
    uint32_t st[4];
    for (int k = 0; k < 4; ++k) st[k] = 4 * l + k;
    for (uint32_t c = chunk_first[b]; c < chunk_first[b + 1]; ++c) {
        S[(size_t)c * 64 + l] = st[0] | (st[1] << 8) | (st[2] << 16) | (st[3] << 24);
        const uint32_t d = dcount[c];
        const uint8_t *Rc = R + (size_t)c * 256;
        for (int k = 0; k < 4; ++k) s_flag[4 * l + k] = 0;
        __syncthreads();
        for (uint32_t j = l; j < d; j += 64) s_flag[Rc[j]] = 1;
        __syncthreads();
        uint32_t keep[4], cnt = 0;
        for (int k = 0; k < 4; ++k) {
            keep[k] = s_flag[st[k]] == 0;
            cnt += keep[k];
        }
        uint32_t pos = d + wave_incl_sum(cnt) - cnt;
        __syncthreads();
        for (int k = 0; k < 4; ++k)
            if (keep[k]) s_S[pos++] = (uint8_t)st[k];
        for (uint32_t j = l; j < d; j += 64) s_S[j] = Rc[j];
        __syncthreads();
        for (int k = 0; k < 4; ++k) st[k] = s_S[4 * l + k];
        __syncthreads();
    }
}

#define MTF_STEP(SYM, OUTV)                                                                 \
    do {                                                                                    \
        const uint32_t c_ = (SYM);                                                          \
        const uint32_t ln_ = c_ >> 2;                                                       \
        uint32_t pc_;                                                                       \
        switch (c_ & 3u) {                                                                  \
        case 0: pc_ = __builtin_amdgcn_readlane(p0, ln_); break;                            \
        case 1: pc_ = __builtin_amdgcn_readlane(p1, ln_); break;                            \
        case 2: pc_ = __builtin_amdgcn_readlane(p2, ln_); break;                            \
        default: pc_ = __builtin_amdgcn_readlane(p3, ln_); break;                           \
        }                                                                                   \
        p0 += p0 < pc_ ? 1u : 0u;                                                           \
        p1 += p1 < pc_ ? 1u : 0u;                                                           \
        p2 += p2 < pc_ ? 1u : 0u;                                                           \
        p3 += p3 < pc_ ? 1u : 0u;                                                           \
        switch (c_ & 3u) {                                                                  \
        case 0: p0 = writelane(0, ln_, p0); break;                         \
        case 1: p1 = writelane(0, ln_, p1); break;                         \
        case 2: p2 = writelane(0, ln_, p2); break;                         \
        default: p3 = writelane(0, ln_, p3); break;                        \
        }                                                                                   \
        OUTV = pc_;                                                                         \
    } while (0)

// grid = chunks, one wave each.
__global__ __launch_bounds__(64) void k_mtf_encode(const uint8_t *__restrict__ L, const MChunk *__restrict__ chunks,
                                                   const uint32_t *__restrict__ S, uint8_t *__restrict__ out,
                                                   uint32_t *__restrict__ freq, uint32_t *__restrict__ first)
{
    __shared__ uint8_t s_pos[256];
    __shared__ uint32_t s_hist[256], s_first[256];
    const MChunk ch = chunks[blockIdx.x];
    const uint32_t l = threadIdx.x;
    {
        const uint32_t w = S[(size_t)blockIdx.x * 64 + l];
        for (int k = 0; k < 4; ++k) s_pos[(w >> (8 * k)) & 255u] = (uint8_t)(4 * l + k);
        for (int k = 0; k < 4; ++k) {
            s_hist[4 * l + k] = 0;
            s_first[4 * l + k] = 0xffffffffu;
        }
    }
    __syncthreads();
    uint32_t p0 = s_pos[4 * l + 0], p1 = s_pos[4 * l + 1], p2 = s_pos[4 * l + 2], p3 = s_pos[4 * l + 3];
    for (uint32_t base = 0; base < ch.len; base += 256) {
        const uint32_t nb = min(256u, ch.len - base);
        const uint32_t i0 = base + 4 * l;
        uint32_t w = 0;
        for (int k = 0; k < 4; ++k)
            if (i0 + k < ch.len) w |= (uint32_t)L[ch.start + i0 + k] << (8 * k);
        uint32_t outw = 0;
        const uint32_t nq = (nb + 3) >> 2;
        for (uint32_t q = 0; q < nq; ++q) {
            const uint32_t wq = __builtin_amdgcn_readlane(w, q);
            uint32_t o0, o1 = 0, o2 = 0, o3 = 0;
            MTF_STEP(wq & 255u, o0);
            if (4 * q + 3 < nb) {
                MTF_STEP((wq >> 8) & 255u, o1);
                MTF_STEP((wq >> 16) & 255u, o2);
                MTF_STEP(wq >> 24, o3);
            } else {
                if (4 * q + 1 < nb) MTF_STEP((wq >> 8) & 255u, o1);
                if (4 * q + 2 < nb) MTF_STEP((wq >> 16) & 255u, o2);
            }
            outw = writelane(o0 | (o1 << 8) | (o2 << 16) | (o3 << 24), q, outw);
        }
        for (int k = 0; k < 4; ++k) {
            if (i0 + k < ch.len) {
                const uint32_t v = (outw >> (8 * k)) & 255u;
                out[ch.start + i0 + k] = (uint8_t)v;
                atomicAdd(&s_hist[v], 1u);
                atomicMin(&s_first[v], ch.rel + i0 + k);
            }
        }
    }
    __syncthreads();
    for (int k = 0; k < 4; ++k) {
        const uint32_t s = 4 * l + k;
        if (s_hist[s]) {
            atomicAdd(&freq[(size_t)ch.block * 256 + s], s_hist[s]);
            atomicMin(&first[(size_t)ch.block * 256 + s], s_first[s]);
        }
    }
}

__global__ void k_fill_u32(uint32_t *p, uint32_t v, size_t n)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace

void mtf_batch(Ctx *c, const uint8_t *d_L, const Batch &bt, uint8_t *d_mtf, uint32_t *h_freq32, uint32_t *h_first32)
{
    const uint32_t nb = bt.nblocks;
    // chunk length: aim for >= ~8K waves on a big batch, 4K..64K symbols per chunk
    uint64_t target = bt.total / 8192;
    uint32_t ch = 4096;
    while (ch < target && ch < 65536) ch <<= 1;
    std::vector<MChunk> hc;
    std::vector<uint32_t> cfirst(nb + 1);
    for (uint32_t b = 0; b < nb; ++b) {
        cfirst[b] = (uint32_t)hc.size();
        const uint64_t o = bt.offs[b], n = bt.offs[b + 1] - o;
        for (uint64_t s = 0; s < n; s += ch) {
            MChunk m;
            m.block = b;
            m.start = (uint32_t)(o + s);
            m.len = (uint32_t)std::min<uint64_t>(ch, n - s);
            m.rel = (uint32_t)s;
            hc.push_back(m);
        }
    }
    cfirst[nb] = (uint32_t)hc.size();
    const uint32_t nch = (uint32_t)hc.size();
    uint8_t *d_tab = (uint8_t *)c->get(WS_MTF_CHUNKS, nch * sizeof(MChunk) + (nb + 1) * 4 + 64);
    MChunk *d_chunks = (MChunk *)d_tab;
    uint32_t *d_cfirst = (uint32_t *)(d_tab + nch * sizeof(MChunk));
    BMH_HIP(hipMemcpyAsync(d_chunks, hc.data(), nch * sizeof(MChunk), hipMemcpyHostToDevice, c->stream));
    BMH_HIP(hipMemcpyAsync(d_cfirst, cfirst.data(), (nb + 1) * 4, hipMemcpyHostToDevice, c->stream));
    uint8_t *d_R = (uint8_t *)c->get(WS_MTF_R, (size_t)nch * 256 + (size_t)nch * 4 + 64);
    uint32_t *d_dcount = (uint32_t *)(d_R + (size_t)nch * 256);
    uint32_t *d_S = (uint32_t *)c->get(WS_MTF_S, (size_t)nch * 256);
    uint32_t *d_freq = (uint32_t *)c->get(WS_FREQ, (size_t)nb * 256 * 4);
    uint32_t *d_first = (uint32_t *)c->get(WS_FIRST, (size_t)nb * 256 * 4);
    BMH_HIP(hipMemsetAsync(d_freq, 0, (size_t)nb * 256 * 4, c->stream));
    BMH_LAUNCH(c, "mtf_fill", k_fill_u32, (uint32_t)(((size_t)nb * 256 + 255) / 256), 256, 0, d_first, 0xffffffffu,
               (size_t)nb * 256);
    BMH_LAUNCH(c, "mtf_recency", k_mtf_recency, nch, 256, 0, d_L, d_chunks, d_R, d_dcount);
    BMH_LAUNCH(c, "mtf_compose", k_mtf_compose, nb, 64, 0, d_cfirst, d_R, d_dcount, d_S);
    BMH_LAUNCH(c, "mtf_encode", k_mtf_encode, nch, 64, 0, d_L, d_chunks, d_S, d_mtf, d_freq, d_first);
    if (h_freq32) BMH_HIP(hipMemcpyAsync(h_freq32, d_freq, (size_t)nb * 256 * 4, hipMemcpyDeviceToHost, c->stream));
    if (h_first32) BMH_HIP(hipMemcpyAsync(h_first32, d_first, (size_t)nb * 256 * 4, hipMemcpyDeviceToHost, c->stream));
    c->sync();
}

}  // namespace bmh
