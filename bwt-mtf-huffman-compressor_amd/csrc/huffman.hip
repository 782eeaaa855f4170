// huffman.hip — per-block Huffman code books and record layout on the device.
//
// Replaces the tree half of huffman() (reference main.cpp:229-257), traverse/build_hashmap
// (main.cpp:132-156), dfs/tree_to_bytes (main.cpp:174-196) and the record header of
// write_to_file (io_utilities.h:7-27) for a whole batch, so the encode pipeline never
// round-trips histograms through the host. One wave per block:
//   leaves   : symbols with freq > 0 ranked by first occurrence in the MTF stream
//   tree     : the reference's std::priority_queue simulated exactly. Node ids: leaves
//              0..L-1, internal nodes L, L+1, ... in creation order; a pop takes the
//              smallest (freq, -addr_rank(id)) — equal frequencies leave the heap in
//              descending glibc heap-address order (same model as
//              huffman_host.cpp) — run as two queues (sorted leaves, internal-node groups);
//              blocks below 128 KiB whose order follows the reference's heap history instead
//              (heap_order.cpp) pop by wave-wide minimum over per-node keys.
//   codes    : pointer jumping on parent links (left = 0); preorder tree bits (internal 1,
//              leaf 0 + 8 value bits MSB-first) placed per leaf in parallel.
//   header   : [u64 primary][u64 n][u64 tree_len][tree bytes] staged per block.
// k_rec_offs then scans header + payload sizes into record offsets (capacity checked on the
// device), and k_rec_headers copies each header to its record.
#include "bmh_internal.h"
#include "device_util.h"

namespace bmh {

namespace {

constexpr uint32_t kHdrStride = 352;  // 24 header bytes + <= 320 tree bytes, 16-aligned

// Phase timing (experiment builds only, -DBMH_PROF_HUFF): lane 0 of each block's wave stores its
// s_memtime ticks per phase of k_huff_build; codebook_batch prints the means after the launch.
#ifdef BMH_PROF_HUFF
__device__ uint32_t g_hprof[4096 * 8];
#define HPROF_START uint64_t _t0 = __builtin_amdgcn_s_memtime()
#define HPROF(i)                                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0) {                                                           \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                             \
            if (blockIdx.x < 4096) g_hprof[blockIdx.x * 8 + (i)] = (uint32_t)(_t - _t0); \
            _t0 = _t;                                                                     \
        }                                                                                 \
    } while (0)
#else
#define HPROF_START
#define HPROF(i) \
    do {         \
    } while (0)
#endif

__device__ __forceinline__ uint32_t addr_rank(uint32_t L, uint32_t s)
{
    if (L <= 128) {
        // [1, 3..127, 0, 2, 128, 129, ...]
        if (s == 1) return 0;
        if (s >= 3 && s <= 127) return s - 2;
        if (s == 0) return 126;
        if (s == 2) return 127;
        return s;
    }
    // [1, 3..64, 129..192, 65..127, 0, 2, 128, 193, 194, ...]
    if (s == 1) return 0;
    if (s >= 3 && s <= 64) return s - 2;
    if (s >= 129 && s <= 192) return s - 66;
    if (s >= 65 && s <= 127) return s + 62;
    if (s == 0) return 190;
    if (s == 2) return 191;
    if (s == 128) return 192;
    return s;
}

// Priority-queue key of node id (pop order = ascending key): frequency, then descending
// heap-address rank, then the id itself in the low bits (never decides: ranks are distinct).
__device__ __forceinline__ uint64_t heap_key(uint64_t freq, uint32_t L, uint32_t id)
{
    return (freq << 32) | ((0xffffu - addr_rank(L, id)) << 16) | id;
}
// A 64-bit value made wave-uniform (two 32-bit reads of lane 0; the builtin returns a signed int,
// so each half is widened as unsigned — a sign-extended low half would overwrite the high one).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// The closed-form address rank of internal node v >= L (ascending with v).
__device__ __forceinline__ uint32_t internal_rank(uint32_t L, uint32_t v)
{
    return L <= 128u ? (v == 2u ? 127u : v - 2u * (uint32_t)(v <= 127u)) : v - 66u * (uint32_t)(v <= 192u);
}

// Rank of key x among the 256 keys of s_keys (padding entries ~0): the number of smaller keys.
// Every thread of the workgroup reads the same two keys at a time (LDS broadcast), 8 in flight.
__device__ __forceinline__ uint32_t rank_u64(const uint64_t *s_keys, uint64_t x)
{
    uint32_t pos = 0;
#pragma unroll 8
    for (uint32_t u = 0; u < 256; u += 2) {
        const uint4 v = *(const uint4 *)&s_keys[u];
        const uint64_t a = ((uint64_t)v.y << 32) | v.x, c = ((uint64_t)v.w << 32) | v.z;
        pos += (uint32_t)(a < x) + (uint32_t)(c < x);
    }
    return pos;
}

// The queue phases run on wave 0 alone: LDS traffic between its lanes needs only the wave's own
// ordering (a fence the compiler cannot move accesses across, then a wave barrier).
#define WAVE_SYNC()                                          \
    do {                                                     \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); \
        __builtin_amdgcn_wave_barrier();                     \
    } while (0)

// grid = nblocks, 256 threads (four waves per block): the per-symbol and per-leaf phases take a
// thread each; the queue (a chain of dependent pops) runs on wave 0.
constexpr uint32_t kHuffThreads = 256;
__global__ __launch_bounds__(kHuffThreads) void k_huff_build(const uint32_t *__restrict__ freq32,
                                                   const uint32_t *__restrict__ first32,
                                                   const uint32_t *__restrict__ prim, const uint64_t *__restrict__ boffs,
                                                   DevTable *__restrict__ tabs, uint8_t *__restrict__ hdr,
                                                   uint32_t *__restrict__ hdr_len, uint64_t *__restrict__ pay_bytes,
                                                   uint32_t *status, const uint32_t *__restrict__ rbase,
                                                   const uint32_t *__restrict__ ridx, const uint16_t *__restrict__ rrank)
{
    __shared__ uint32_t s_freq[256];
    __shared__ uint8_t s_order[256];
    __shared__ int16_t s_left[512], s_right[512];
    __shared__ uint64_t s_code[256];
    __shared__ uint8_t s_len[256];
    __shared__ uint32_t s_tree32[80];                  // tree bytes (320), stream byte i = byte i
    __shared__ uint16_t s_par[512];                    // parent, then jump target (root: itself)
    __shared__ uint16_t s_dep[512];                    // path length to the jump target
    __shared__ uint64_t s_pcode[512];                  // path bits to the jump target (left 0, right 1)
    __shared__ uint64_t s_lkey[256];                   // leaf keys, then left-aligned leaf codes
    __shared__ uint64_t s_k1[256], s_q2[512];          // leaves in pop order; the pop sequence P
    __shared__ uint32_t s_err;
    __shared__ uint64_t s_bits;
    uint8_t *s_tree = (uint8_t *)s_tree32;
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    HPROF_START;
    const uint32_t fq = freq32[(size_t)b * 256 + tid], fs = first32[(size_t)b * 256 + tid];
    s_freq[tid] = fq;
    s_len[tid] = 0;
    s_code[tid] = 0;
    // leaves in first-occurrence order (main.cpp:238-244); first positions are distinct
    s_lkey[tid] = fq ? fs : ~0ull;
    if (tid == 0) {
        s_err = 0;
        s_bits = 0;
    }
    const uint32_t L = (uint32_t)__syncthreads_count(fq > 0);
    if (fq) s_order[rank_u64(s_lkey, fs)] = (uint8_t)tid;
    __syncthreads();
    if (L == 0) {
        if (tid == 0) atomicOr(status, kStatusEmpty);
        return;
    }
    HPROF(0);  // loads, leaf count, leaf order
    // small blocks whose node addresses follow the reference's heap history (heap_order.cpp):
    // ro = the first of this L's 2L - 1 ranks, or kModelOrder (the closed form holds)
    uint32_t ro = kModelOrder;
    if (rbase) {
        const uint32_t rb = rbase[b];
        if (rb != kModelOrder) ro = ridx[rb + L];
    }
    if (ro != kModelOrder) {
      if (wave == 0) {
        // the internal nodes' ranks need not ascend, so the queue is simulated as it is: every
        // live node's key in a register slot (node v: lane v & 63, slot v >> 6), each pop a
        // wave-wide minimum (smallest frequency, then the larger address rank). The blocks here
        // are below kBandCeil = 2^17 bytes, so a key fits 32 bits: frequency (< 2^17) << 9 |
        // 511 - rank (ranks < 2L - 1 <= 511 are distinct, so keys are too, and the popped node is
        // the one lane slot holding the minimum)
        static_assert(kBandCeil <= (1u << 17), "32-bit heap-history keys");
        const uint16_t *rk = rrank + ro;
        uint32_t key[8];
        uint32_t rkr[8];  // the ranks of this lane's nodes (id = lane + 64 k), all loads at once
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) rkr[k] = lane + 64 * k < 2 * L - 1 ? rk[lane + 64 * k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            const uint32_t id = lane + 64 * k;
            key[k] = id < L ? (s_freq[s_order[id]] << 9) | (511u - rkr[k]) : ~0u;
        }
        for (uint32_t m = 0; m + 1 < L; ++m) {
            uint32_t r[2], f = 0;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                uint32_t mn = key[0];
#pragma unroll
                for (int k = 1; k < 8; ++k) mn = min(mn, key[k]);
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
                uint32_t mine = ~0u;
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k)
                    if (key[k] == mn) {
                        key[k] = ~0u;
                        mine = lane + 64 * k;
                    }
                const uint64_t bal = __ballot(mine != ~0u);
                r[t] = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)__builtin_ctzll(bal));
                f += mn >> 9;
            }
            const uint32_t v = L + m;
            if (lane == 0) {
                s_left[v] = (int16_t)r[0];
                s_right[v] = (int16_t)r[1];
            }
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k)  // the owning lane builds the new node's key
                if (lane + 64 * k == v) key[k] = (f << 9) | (511u - rkr[k]);
        }
      }
    } else {
        // The reference's priority queue (main.cpp:245-254: first pop -> left child, second ->
        // right) in parallel rounds. A new node's frequency is the sum of the two it was made from,
        // so it exceeds the frequency of everything popped so far, and its key is larger than
        // every popped key: the pops come out in ascending key order, i.e. the pop sequence P is
        // the sorted sequence of all non-root node keys, and internal node j (id L + j) is made
        // of P[2j] and P[2j + 1]. Internal frequencies F[j] never decrease with j and their
        // address ranks ascend with j, so the internal keys sort by F, newest first among equals.
        // A round takes the known nodes 0 .. m-1: every node made later has a key >= B = (F[m-1],
        // the largest internal rank), so all known items below B are the smallest |D| items of P;
        // they are merged into P (two sorted runs, the leaves and the internals of complete
        // frequency groups), and every node j with 2j + 1 < |D| is made at once. When that is no
        // progress (a chain where each new node is popped next), the round pops the two smallest
        // remaining items as the heap would. Random data takes ~10 rounds, text and Calgary
        // 15-27, instead of L - 1 sequential merges (tests/test_huffman_queue.py restates it).
        // leaf keys (frequency, descending address rank, id), sorted into s_k1
        const uint64_t lk = tid < L ? heap_key(s_freq[s_order[tid]], L, tid) : ~0ull;
        s_lkey[tid] = lk;
        __syncthreads();
        if (tid < L) s_k1[rank_u64(s_lkey, lk)] = lk;
        __syncthreads();
        HPROF(5);  // (model path) leaf keys ranked
      if (wave == 0) {
        uint64_t *s_P = s_q2;          // P (keys), 2 L - 2 entries
        uint64_t *s_IK = s_pcode;      // sorted internal keys (s_pcode is free until the codes)
        __shared__ uint32_t s_F[256];  // F[j]
        const uint32_t rmax = internal_rank(L, 2 * L - 2);
        uint64_t lkr[4];  // sorted leaf keys, slot lane + 64 k
#pragma unroll
        for (int k = 0; k < 4; ++k) lkr[k] = lane + 64 * k < L ? s_k1[lane + 64 * k] : ~0ull;
        uint32_t fr[4] = {~0u, ~0u, ~0u, ~0u};  // F of node lane + 64 k (nodes < m)
        uint64_t gm[4] = {0, 0, 0, 0};          // group starts among nodes 0 .. m-1 (uniform)
        uint32_t m = 0, lc = 0, ic = 0;         // known nodes; leaves / internals placed in P
        // sorted internal index x -> node: x's frequency group [gs, ge) reversed
        auto node_of = [&](uint32_t x) -> uint32_t {
            uint32_t q = x >> 6;
            uint64_t w = gm[q] & (((2ull << (x & 63u)) - 1) | ((x & 63u) == 63u ? ~0ull : 0ull));
            for (uint32_t t = 0; t < 3 && !w && q > 0; ++t) w = gm[--q];
            const uint32_t gs = 64 * q + 63 - (uint32_t)__builtin_clzll(w);
            q = x >> 6;
            w = (x & 63u) == 63u ? 0ull : gm[q] & ~((2ull << (x & 63u)) - 1);
            for (uint32_t t = 0; t < 3 && !w && q < 3; ++t) w = gm[++q];
            const uint32_t ge = w ? 64 * q + (uint32_t)__builtin_ctzll(w) : m;
            return gs + ge - 1 - x;
        };
        auto ikey = [&](uint32_t j) -> uint64_t {
            return ((uint64_t)s_F[j] << 32) | ((uint64_t)(0xffffu - internal_rank(L, L + j)) << 16) | (L + j);
        };
        // first index in [lo, hi) of the sorted array a whose key is >= x
        auto lower = [&](const uint64_t *a, uint32_t lo, uint32_t hi, uint64_t x) -> uint32_t {
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (a[mid] < x) lo = mid + 1;
                else hi = mid;
            }
            return lo;
        };
        for (uint32_t guard = 0; m + 1 < L && guard < L; ++guard) {  // m grows every round
            uint32_t la = 0, ia = 0;
            bool bound = false;
            if (m > 0) {
                const uint32_t fm1 = __builtin_amdgcn_readfirstlane(s_F[m - 1]);
                const uint64_t B = ((uint64_t)fm1 << 32) | ((uint64_t)(0xffffu - rmax) << 16);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    la += (uint32_t)__builtin_popcountll(__ballot(lkr[k] < B));
                    ia += (uint32_t)__builtin_popcountll(__ballot(lane + 64u * k < m && fr[k] < fm1));
                }
                bound = la + ia >= 2 * m + 2;
            }
            if (bound) {
                for (uint32_t x = ic + lane; x < ia; x += 64) s_IK[x] = ikey(node_of(x));
                WAVE_SYNC();
                const uint32_t base = lc + ic;
                for (uint32_t i = lc + lane; i < la; i += 64) {
                    const uint64_t key = s_k1[i];
                    s_P[base + (i - lc) + (lower(s_IK, ic, ia, key) - ic)] = key;
                }
                for (uint32_t x = ic + lane; x < ia; x += 64) {
                    const uint64_t key = s_IK[x];
                    s_P[base + (x - ic) + (lower(s_k1, lc, la, key) - lc)] = key;
                }
                lc = la;
                ic = ia;
            } else {
                // the smallest remaining items (the heads of the two sorted runs), uniformly, up to
                // P[2m + 1] (P[2m] may be placed already)
                while (lc + ic < 2 * m + 2) {
                    const uint64_t a = lc < L ? s_k1[lc] : ~0ull;
                    uint64_t c = ~0ull;
                    if (ic < m) c = ikey(node_of(ic));
                    const uint64_t au = uniform_u64(a), cu = uniform_u64(c);
                    s_P[lc + ic] = au < cu ? au : cu;  // every lane stores the same value
                    if (au < cu) ++lc;
                    else ++ic;
                }
            }
            WAVE_SYNC();
            const uint32_t m2 = min((lc + ic) / 2, L - 1);
            for (uint32_t j = m + lane; j < m2; j += 64) {
                const uint64_t a = s_P[2 * j], c = s_P[2 * j + 1];
                s_left[L + j] = (int16_t)(a & 0xffffu);
                s_right[L + j] = (int16_t)(c & 0xffffu);
                s_F[j] = (uint32_t)(a >> 32) + (uint32_t)(c >> 32);
            }
            WAVE_SYNC();
            m = m2;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = lane + 64u * k;
                fr[k] = j < m ? s_F[j] : ~0u;
                const bool st = j < m && (j == 0 || s_F[j - 1] != fr[k]);
                gm[k] = __ballot(st);
            }
        }
      }
    }
    __syncthreads();
    HPROF(1);  // the queue (merges; key ranking too on the heap-history path)
    // codes (left 0, right 1; a root leaf gets the empty code) by pointer jumping on parent
    // links: node x keeps (target a, path bits c, path length d) with code(x) = code(a) << d | c
    const uint32_t nn = 2 * L - 1;  // nodes; the root (nn - 1) is its own target
    for (uint32_t v = tid; v < nn; v += kHuffThreads) {
        s_par[v] = (uint16_t)v;
        s_dep[v] = 0;
        s_pcode[v] = 0;
    }
    __syncthreads();
    for (uint32_t v = L + tid; v < nn; v += kHuffThreads) {
        const uint32_t a = (uint32_t)s_left[v], c = (uint32_t)s_right[v];
        s_par[a] = (uint16_t)v;
        s_dep[a] = 1;
        s_par[c] = (uint16_t)v;
        s_dep[c] = 1;
        s_pcode[c] = 1;
    }
    __syncthreads();
    // depth <= 255 < 2^9: at most 9 rounds; done as soon as every target is the root (a code
    // tree of depth D takes ceil(log2 D) rounds: ~5 for a 256-leaf tree)
    for (uint32_t round = 0; round < 9; ++round) {
        uint32_t na[2], nd[2];
        uint64_t nc[2];
        bool more = false;
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {  // all reads of the round before any write
            const uint32_t v = tid + kHuffThreads * k;
            na[k] = v;
            nd[k] = 0;
            nc[k] = 0;
            if (v < nn) {
                const uint32_t a = s_par[v], d = s_dep[v];
                const uint64_t c = s_pcode[v];
                const uint32_t a2 = s_par[a], d2 = s_dep[a];
                const uint64_t c2 = s_pcode[a];
                na[k] = a2;
                nd[k] = d + d2;
                nc[k] = d >= 64 ? c : (c2 << d) | c;  // (longer paths are flagged below)
                more |= a2 != nn - 1;
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
            const uint32_t v = tid + kHuffThreads * k;
            if (v < nn) {
                s_par[v] = (uint16_t)na[k];
                s_dep[v] = (uint16_t)min(nd[k], 0xffffu);
                s_pcode[v] = nc[k];
            }
        }
        if (!__syncthreads_or(more)) break;  // the barrier of the writes; a uniform exit
    }
    HPROF(2);  // pointer jumping
    // leaves: code book, and the left-aligned codes, whose order is the preorder of the leaves
    uint32_t dv = 0, symv = 0;
    uint64_t lcode = ~0ull;  // this thread's leaf (v = tid < L): depth, symbol, left-aligned code
    if (tid < L) {
        dv = s_dep[tid];
        symv = s_order[tid];
        if (dv > 64) atomicOr(&s_err, kStatusCodeLen);
        const uint64_t code = dv > 64 ? 0ull : s_pcode[tid];
        s_len[symv] = (uint8_t)min(dv, 255u);
        s_code[symv] = code;
        lcode = dv == 0 ? 0ull : dv > 64 ? ~0ull : code << (64 - dv);
    }
    s_lkey[tid] = lcode;
    // preorder tree bits (tree_to_bytes main.cpp:174-196): all 10L - 1 bits start as internal
    // '1's; leaf j in preorder (j leaves and depth + j - popcount(code) internal nodes before
    // it) owns bits [10j + depth - popcount, +9): a '0' then its 8 value bits MSB-first
    const uint32_t tbits = 10 * L - 1;
    if (tid < 80) {
        const uint32_t w = tid;
        uint32_t x = 0;
        for (uint32_t k = 0; k < 32; ++k) {
            const uint32_t bit = 32 * w + 8 * (k >> 3) + (7 - (k & 7));  // stream bit of u32 bit k
            if (bit < tbits) x |= 1u << k;
        }
        s_tree32[w] = x;
    }
    __syncthreads();
    if (tid < L) {
        const uint32_t j = rank_u64(s_lkey, lcode);
        const uint32_t off = 10 * j + min(dv, 64u) - (uint32_t)__builtin_popcountll(s_pcode[tid]);
        for (uint32_t i = 0; i < 9; ++i) {
            const uint32_t one = i == 0 ? 0u : (symv >> (8 - i)) & 1u;
            if (!one) {
                const uint32_t pbit = off + i, byte = pbit >> 3;
                atomicAnd(&s_tree32[byte >> 2], ~(1u << (8 * (byte & 3) + 7 - (pbit & 7))));
            }
        }
    }
    __syncthreads();
    DevTable *t = &tabs[b];
    HPROF(3);  // codes, preorder ranks, tree bits
    const uint32_t ln = s_len[tid];
    t->code[tid] = s_code[tid];
    t->len[tid] = (uint8_t)ln;
    uint64_t bits = (uint64_t)s_freq[tid] * ln;
    for (int off = 32; off >= 1; off >>= 1) bits += __shfl_xor(bits, off, 64);
    if (lane == 0) atomicAdd((unsigned long long *)&s_bits, (unsigned long long)bits);
    const uint32_t tree_len = (tbits + 7) >> 3;
    const uint64_t n = boffs[b + 1] - boffs[b];
    const uint32_t p = prim[b];
    uint8_t *h = hdr + (size_t)b * kHdrStride;
    for (uint32_t i = tid; i < 24 + tree_len; i += kHuffThreads) {
        uint8_t v;
        if (i < 8) v = (uint8_t)((uint64_t)p >> (8 * i));
        else if (i < 16) v = (uint8_t)(n >> (8 * (i - 8)));
        else if (i < 24) v = (uint8_t)((uint64_t)tree_len >> (8 * (i - 16)));
        else v = s_tree[i - 24];
        h[i] = v;
    }
    __syncthreads();
    if (tid == 0) {
        hdr_len[b] = 24 + tree_len;
        const uint64_t pb = (s_bits + 7) / 8;
        pay_bytes[b] = pb ? pb : 1;  // encode_with_huffman starts from one zero byte (main.cpp:162)
        uint32_t e = s_err;
        if (p == 0xffffffffu) e |= kStatusPrimary;
        if (e) atomicOr(status, e);
    }
    HPROF(4);  // outputs
}

// One workgroup: record offsets = exclusive scan of (header + payload) sizes.
// hdr non-null (batches of <= kRecHdrFused blocks): the same workgroup then copies the headers
// (wave w: blocks w, w + 16, ...), so a latency-bound batch saves the k_rec_headers launch
constexpr uint32_t kRecHdrFused = 256;
__global__ __launch_bounds__(1024) void k_rec_offs(uint32_t nb, const uint32_t *__restrict__ hdr_len,
                                                   const uint64_t *__restrict__ pay_bytes, uint64_t *__restrict__ roffs,
                                                   uint64_t *__restrict__ pay_offs, uint64_t out_cap, uint32_t *status,
                                                   const uint64_t *base, const uint8_t *__restrict__ hdr,
                                                   uint8_t *__restrict__ out)
{
    __shared__ uint64_t s_tmp[17];
    uint64_t carry = base ? *base : 0ull;  // sub-batches chain on the previous one's end
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t b = base + threadIdx.x;
        const uint64_t v = b < nb ? hdr_len[b] + pay_bytes[b] : 0ull;
        uint64_t total;
        const uint64_t ex = carry + block_excl_sum64<1024>(v, s_tmp, &total);
        if (b < nb) {
            roffs[b] = ex;
            pay_offs[b] = ex + hdr_len[b];
        }
        carry += total;
    }
    if (threadIdx.x == 0) {
        roffs[nb] = carry;
        if (carry > out_cap) atomicOr(status, kStatusCapacity);
        // the batch's final status (k_huff_build's bits + capacity) beside the offsets: the host
        // reads both with one copy (nothing later in the encode sets status bits)
        roffs[nb + 1] = *(volatile uint32_t *)status | (carry > out_cap ? kStatusCapacity : 0u);
    }
    if (!hdr || carry > out_cap) return;  // (workgroup-uniform: every thread holds the total)
    __syncthreads();                      // roffs of every block written
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    for (uint32_t b = w; b < nb; b += 16) {
        const uint8_t *h = hdr + (size_t)b * kHdrStride;
        uint8_t *o = out + roffs[b];
        for (uint32_t i = l; i < hdr_len[b]; i += 64) o[i] = h[i];
    }
}

__global__ __launch_bounds__(64) void k_rec_headers(const uint8_t *__restrict__ hdr, const uint32_t *__restrict__ hdr_len,
                                                    const uint64_t *__restrict__ roffs, uint8_t *__restrict__ out,
                                                    const uint32_t *status)
{
    if (*status & kStatusCapacity) return;
    const uint32_t b = blockIdx.x;
    const uint8_t *h = hdr + (size_t)b * kHdrStride;
    uint8_t *o = out + roffs[b];
    for (uint32_t i = threadIdx.x; i < hdr_len[b]; i += 64) o[i] = h[i];
}

}  // namespace

void codebook_batch(Ctx *c, const Batch &bt, const uint64_t *d_boffs, const uint32_t *d_freq, const uint32_t *d_first,
                    const uint32_t *d_prim, DevTable *d_tabs, uint64_t *d_roffs, uint64_t *d_pay_offs,
                    uint8_t *d_out, uint64_t out_cap, uint32_t *d_status, OffsetChain *chain, int sub)
{
    const uint32_t nb = bt.nblocks;
    uint8_t *d_hdr = (uint8_t *)c->get(WS_HDR, (size_t)nb * kHdrStride + (size_t)nb * 12 + 64);
    uint64_t *d_payb = (uint64_t *)(d_hdr + (size_t)nb * kHdrStride);
    uint32_t *d_hlen = (uint32_t *)(d_payb + nb);
    // heap-history node ranks of the blocks below kBandCeil whose order differs from the closed
    // form for some leaf count (heap_order.cpp), uploaded once per batch layout: rbase[nb] | per
    // distinct size a 257-entry index (first u16 rank of each L, or kModelOrder) | u16 ranks
    const uint32_t *d_rbase = nullptr, *d_ridx = nullptr;
    const uint16_t *d_rrank = nullptr;
    const uint64_t bsig = layout_sig(3, bt.offs, 0);
    if (c->ws_tag[WS_BAND] != bsig) {
        std::vector<uint32_t> rbase(nb, kModelOrder), idx;
        std::vector<uint16_t> ranks;
        std::map<uint64_t, uint32_t> seen;
        std::vector<uint64_t> sizes;
        for (uint32_t b = 0; b < nb; ++b)
            if (bt.offs[b + 1] - bt.offs[b] < kBandCeil) sizes.push_back(bt.offs[b + 1] - bt.offs[b]);
        const auto tabs = band_ranks_batch(sizes);  // held until the upload below
        for (uint32_t b = 0; b < nb; ++b) {
            const uint64_t n = bt.offs[b + 1] - bt.offs[b];
            const auto it_t = tabs.find(n);
            if (it_t == tabs.end() || !it_t->second) continue;
            const auto &br = it_t->second;
            auto it = seen.find(n);
            if (it == seen.end()) {
                const uint32_t at = (uint32_t)idx.size();
                for (uint32_t L = 0; L <= 256; ++L)
                    idx.push_back(br->off[L] == kModelOrder ? kModelOrder : (uint32_t)ranks.size() + br->off[L]);
                ranks.insert(ranks.end(), br->rank.begin(), br->rank.end());
                it = seen.emplace(n, at).first;
            }
            rbase[b] = it->second;
        }
        c->ws_aux[WS_BAND][0] = idx.empty() ? 0u : 1u;
        c->ws_aux[WS_BAND][1] = (uint32_t)idx.size();
        if (!idx.empty()) {
            const size_t bytes = (rbase.size() + idx.size()) * 4 + ranks.size() * 2;
            std::vector<uint8_t> h(bytes);
            memcpy(h.data(), rbase.data(), rbase.size() * 4);
            memcpy(h.data() + rbase.size() * 4, idx.data(), idx.size() * 4);
            memcpy(h.data() + (rbase.size() + idx.size()) * 4, ranks.data(), ranks.size() * 2);
            c->h2d(c->get(WS_BAND, bytes + 64), h.data(), bytes);
        }
        c->ws_tag[WS_BAND] = bsig;
    }
    if (c->ws_aux[WS_BAND][0]) {
        d_rbase = (const uint32_t *)c->ws[WS_BAND];
        d_ridx = d_rbase + nb;
        d_rrank = (const uint16_t *)(d_ridx + c->ws_aux[WS_BAND][1]);
    }
    BMH_LAUNCH(c, "huff_build", k_huff_build, nb, kHuffThreads, 0, d_freq, d_first, d_prim, d_boffs, d_tabs, d_hdr, d_hlen, d_payb,
               d_status, d_rbase, d_ridx, d_rrank);
#ifdef BMH_PROF_HUFF
    {
        std::vector<uint32_t> h(4096 * 8);
        BMH_HIP(hipStreamSynchronize(c->stream));
        BMH_HIP(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_hprof), h.size() * 4));
        double sum[8] = {};
        const uint32_t m = std::min<uint32_t>(nb, 4096);
        for (uint32_t w = 0; w < m; ++w)
            for (int i = 0; i < 8; ++i) sum[i] += h[w * 8 + i];
        fprintf(stderr, "huff_build phases (mean s_memtime ticks over %u blocks):", m);
        for (int i = 0; i < 6; ++i) fprintf(stderr, " %.0f", m ? sum[i] / m : 0.0);
        fprintf(stderr, "\n");
    }
#endif
    const uint64_t *d_base = nullptr;
    if (chain && sub > 0) {
        std::unique_lock<std::mutex> lk(chain->m);
        chain->cv.wait(lk, [&] { return chain->recorded >= sub - 1 || chain->failed; });
        if (chain->failed) fail(BMH_EHIP, "encode: a concurrent sub-batch failed");
        BMH_HIP(hipStreamWaitEvent(c->stream, chain->ev[sub - 1], 0));
        d_base = chain->d_end[sub - 1];
    }
    const bool fused = nb <= kRecHdrFused;
    BMH_LAUNCH(c, "rec_offs", k_rec_offs, 1, 1024, 0, nb, d_hlen, d_payb, d_roffs, d_pay_offs, out_cap, d_status, d_base,
               fused ? d_hdr : nullptr, d_out);
    if (chain) {
        BMH_HIP(hipEventRecord(chain->ev[sub], c->stream));
        {
            std::lock_guard<std::mutex> lk(chain->m);
            chain->d_end[sub] = d_roffs + nb;
            chain->recorded = sub;
        }
        chain->cv.notify_all();
    }
    if (!fused) BMH_LAUNCH(c, "rec_headers", k_rec_headers, nb, 64, 0, d_hdr, d_hlen, d_roffs, d_out, d_status);
}

}  // namespace bmh
