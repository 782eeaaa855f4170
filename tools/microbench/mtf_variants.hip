// mtf_variants.hip — microbenchmark of MTF inner-loop formulations on gfx950.
//
// Each variant runs exact move-to-front (reference main.cpp:93-112) over independent chunks
// (identity start state per chunk) of 1 GiB of random bytes, one or more chunks ("streams")
// per wave interleaved for ILP. Output is checked against a CPU MTF on a few chunks; timing
// uses HIP events. Build: hipcc -O3 --offload-arch=gfx950 mtf_variants.hip -o mtf_variants
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);               \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

extern "C" __device__ int llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// ---------------------------------------------------------------- A: switch (current)
#define STEP_A(SYM, OUTV)                                                                   \
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
        case 0: p0 = llvm_writelane(0, ln_, p0); break;                                     \
        case 1: p1 = llvm_writelane(0, ln_, p1); break;                                     \
        case 2: p2 = llvm_writelane(0, ln_, p2); break;                                     \
        default: p3 = llvm_writelane(0, ln_, p3); break;                                    \
        }                                                                                   \
        OUTV = pc_;                                                                         \
    } while (0)

__global__ __launch_bounds__(64) void k_A(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, uint32_t ch)
{
    const uint32_t l = threadIdx.x;
    const size_t base0 = (size_t)blockIdx.x * ch;
    uint32_t p0 = 4 * l, p1 = 4 * l + 1, p2 = 4 * l + 2, p3 = 4 * l + 3;
    for (uint32_t base = 0; base < ch; base += 256) {
        const uint32_t w = *(const uint32_t *)(in + base0 + base + 4 * l);
        uint32_t outw = 0;
        for (uint32_t q = 0; q < 64; ++q) {
            const uint32_t wq = __builtin_amdgcn_readlane(w, q);
            uint32_t o0, o1, o2, o3;
            STEP_A(wq & 255u, o0);
            STEP_A((wq >> 8) & 255u, o1);
            STEP_A((wq >> 16) & 255u, o2);
            STEP_A(wq >> 24, o3);
            outw = llvm_writelane(o0 | (o1 << 8) | (o2 << 16) | (o3 << 24), q, outw);
        }
        *(uint32_t *)(out + base0 + base + 4 * l) = outw;
    }
}

// ------------------------------------------- B: packed u16, branch-free, S streams/wave
// symbol s -> lane s>>2, VGPR (s>>1)&1, half s&1. Update per 2-entry VGPR:
//   x' = min(x + 1, max(x, pc), (x ^ pc) << 8)   (x < pc: x+1; x > pc: x; x == pc: 0)
template <int S>
__global__ __launch_bounds__(256) void k_B(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, uint32_t ch)
{
    typedef uint16_t h2 __attribute__((ext_vector_type(2)));
    const uint32_t l = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const size_t stream0 = ((size_t)blockIdx.x * 4 + wv) * S;
    h2 P[S][2];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        P[s][0] = h2{(uint16_t)(4 * l), (uint16_t)(4 * l + 1)};
        P[s][1] = h2{(uint16_t)(4 * l + 2), (uint16_t)(4 * l + 3)};
    }
    for (uint32_t base = 0; base < ch; base += 256) {
        uint32_t w[S], outw[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            w[s] = *(const uint32_t *)(in + (stream0 + s) * ch + base + 4 * l);
            outw[s] = 0;
        }
        for (uint32_t q = 0; q < 64; ++q) {
            uint32_t wq[S], o[S];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                wq[s] = __builtin_amdgcn_readlane(w[s], q);
                o[s] = 0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const uint32_t c = (wq[s] >> (8 * k)) & 255u;
                    const uint32_t ln = c >> 2;
                    const h2 sel = ((c >> 1) & 1u) ? P[s][1] : P[s][0];
                    const uint32_t wsel = __builtin_bit_cast(uint32_t, sel);
                    const uint32_t wrd = __builtin_amdgcn_readlane(wsel, ln);
                    const uint32_t pc = (c & 1u) ? (wrd >> 16) : (wrd & 0xffffu);
                    const h2 pcv = h2{(uint16_t)pc, (uint16_t)pc};
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const h2 x = P[s][j];
                        const h2 a = x + h2{1, 1};
                        const h2 bmax = __builtin_elementwise_max(x, pcv);
                        const h2 xx = (x ^ pcv) << h2{8, 8};
                        P[s][j] = __builtin_elementwise_min(__builtin_elementwise_min(a, bmax), xx);
                    }
                    o[s] |= pc << (8 * k);
                }
            }
#pragma unroll
            for (int s = 0; s < S; ++s) outw[s] = llvm_writelane(o[s], q, outw[s]);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) *(uint32_t *)(out + (stream0 + s) * ch + base + 4 * l) = outw[s];
    }
}

// ------------------------------------------------ C: u32, branch-free select, S streams
template <int S>
__global__ __launch_bounds__(256) void k_C(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, uint32_t ch)
{
    const uint32_t l = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const size_t stream0 = ((size_t)blockIdx.x * 4 + wv) * S;
    uint32_t P[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) P[s][j] = 4 * l + j;
    for (uint32_t base = 0; base < ch; base += 256) {
        uint32_t w[S], outw[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            w[s] = *(const uint32_t *)(in + (stream0 + s) * ch + base + 4 * l);
            outw[s] = 0;
        }
        for (uint32_t q = 0; q < 64; ++q) {
            uint32_t wq[S], o[S];
#pragma unroll
            for (int s = 0; s < S; ++s) {
                wq[s] = __builtin_amdgcn_readlane(w[s], q);
                o[s] = 0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll
                for (int s = 0; s < S; ++s) {
                    const uint32_t c = (wq[s] >> (8 * k)) & 255u;
                    const uint32_t ln = c >> 2, r = c & 3u;
                    uint32_t v = P[s][0];
                    v = r == 1 ? P[s][1] : v;
                    v = r == 2 ? P[s][2] : v;
                    v = r == 3 ? P[s][3] : v;
                    const uint32_t pc = __builtin_amdgcn_readlane(v, ln);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t x = P[s][j];
                        const uint32_t a = x + 1;
                        const uint32_t bm = x > pc ? x : pc;
                        const uint32_t xx = (x ^ pc) << 8;
                        const uint32_t m = a < bm ? a : bm;
                        P[s][j] = m < xx ? m : xx;
                    }
                    o[s] |= pc << (8 * k);
                }
            }
#pragma unroll
            for (int s = 0; s < S; ++s) outw[s] = llvm_writelane(o[s], q, outw[s]);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) *(uint32_t *)(out + (stream0 + s) * ch + base + 4 * l) = outw[s];
    }
}


// ------------------------------- D/E: packed u16 with named registers (no array demotion)
// D: select the VGPR with v_cndmask, one readlane.  E: readlane both VGPRs, select in SALU.
#define PK_UPD(X, PCV)                                                                     \
    do {                                                                                   \
        const h2 a_ = (X) + h2{1, 1};                                                      \
        const h2 m_ = __builtin_elementwise_max((X), (PCV));                               \
        const h2 z_ = ((X) ^ (PCV)) << h2{8, 8};                                           \
        (X) = __builtin_elementwise_min(__builtin_elementwise_min(a_, m_), z_);           \
    } while (0)
typedef uint16_t h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t u32of(h2 v) { return __builtin_bit_cast(uint32_t, v); }

template <int MODE>
__device__ __forceinline__ uint32_t pk_step(h2 &A, h2 &B, uint32_t c)
{
    const uint32_t ln = c >> 2;
    uint32_t wrd;
    if (MODE == 0) {
        const uint32_t sel = ((c >> 1) & 1u) ? u32of(B) : u32of(A);
        wrd = __builtin_amdgcn_readlane(sel, ln);
    } else {
        const uint32_t wa = __builtin_amdgcn_readlane(u32of(A), ln);
        const uint32_t wb = __builtin_amdgcn_readlane(u32of(B), ln);
        wrd = ((c >> 1) & 1u) ? wb : wa;
    }
    const uint32_t pc = (wrd >> ((c & 1u) * 16)) & 0xffffu;
    const h2 pcv = h2{(uint16_t)pc, (uint16_t)pc};
    PK_UPD(A, pcv);
    PK_UPD(B, pcv);
    return pc;
}

template <int MODE, int S>
__global__ __launch_bounds__(256) void k_D(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, uint32_t ch)
{
    const uint32_t l = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const size_t st0 = ((size_t)blockIdx.x * 4 + wv) * S;
    h2 A0 = h2{(uint16_t)(4 * l), (uint16_t)(4 * l + 1)}, B0 = h2{(uint16_t)(4 * l + 2), (uint16_t)(4 * l + 3)};
    h2 A1 = A0, B1 = B0;
    for (uint32_t base = 0; base < ch; base += 256) {
        const uint32_t w0 = *(const uint32_t *)(in + st0 * ch + base + 4 * l);
        const uint32_t w1 = S > 1 ? *(const uint32_t *)(in + (st0 + 1) * ch + base + 4 * l) : 0u;
        uint32_t ow0 = 0, ow1 = 0;
        for (uint32_t q = 0; q < 64; ++q) {
            const uint32_t q0 = __builtin_amdgcn_readlane(w0, q);
            const uint32_t q1 = S > 1 ? __builtin_amdgcn_readlane(w1, q) : 0u;
            uint32_t o0 = 0, o1 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o0 |= pk_step<MODE>(A0, B0, (q0 >> (8 * k)) & 255u) << (8 * k);
                if (S > 1) o1 |= pk_step<MODE>(A1, B1, (q1 >> (8 * k)) & 255u) << (8 * k);
            }
            ow0 = llvm_writelane(o0, q, ow0);
            if (S > 1) ow1 = llvm_writelane(o1, q, ow1);
        }
        *(uint32_t *)(out + st0 * ch + base + 4 * l) = ow0;
        if (S > 1) *(uint32_t *)(out + (st0 + 1) * ch + base + 4 * l) = ow1;
    }
}

// --------------------------------------------- F: per-lane chunk, time-stamp + 2-level bitset
// Lane l owns one chunk. tm[s] = slot of the last access of symbol s (512-slot window); a slot
// bit is set iff it is some symbol's last access (always exactly 256 marks). MTF index of c =
// marks above tm[c] = A (whole superwords above) + B (words of c's superword above c's word)
// + C (bits above in c's word); superword counts S (4 bytes, register), word counts cnt
// (4 bytes per superword, LDS), bits (LDS). When the window fills, slots are renumbered.
constexpr int FNL = 256;
__device__ __forceinline__ uint32_t f_above(uint32_t t, uint32_t S, const uint32_t *bits, const uint32_t *cnt, uint32_t l)
{
    const uint32_t ws = t >> 5, sb = t & 31u, wq = ws >> 2, wr = ws & 3u;
    const uint32_t bw = bits[ws * FNL + l];
    const uint32_t cw = cnt[wq * FNL + l];
    uint32_t r = __builtin_popcount((bw >> sb) >> 1);
    r = __builtin_amdgcn_sad_u8(cw & (0xFFFFFF00u << (8 * wr)), 0u, r);
    r = __builtin_amdgcn_sad_u8(S & (0xFFFFFF00u << (8 * wq)), 0u, r);
    return r;
}
__global__ __launch_bounds__(256) void k_F(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, uint32_t ch)
{
    __shared__ uint16_t tm[256 * FNL];
    __shared__ uint32_t bits[16 * FNL];
    __shared__ uint32_t cnt[4 * FNL];
    const uint32_t l = threadIdx.x;
    const uint8_t *src = in + ((size_t)blockIdx.x * FNL + l) * ch;
    uint8_t *dst = out + ((size_t)blockIdx.x * FNL + l) * ch;
    for (uint32_t s = 0; s < 256; ++s) tm[s * FNL + l] = (uint16_t)(255 - s);  // identity start
    for (uint32_t w = 0; w < 16; ++w) bits[w * FNL + l] = w < 8 ? 0xffffffffu : 0u;
    for (uint32_t q = 0; q < 4; ++q) cnt[q * FNL + l] = q < 2 ? 0x20202020u : 0u;
    uint32_t S = 0x00008080u;
    uint32_t now = 256;
    for (uint32_t i = 0; i < ch; i += 4) {
        const uint32_t w4 = *(const uint32_t *)(src + i);
        uint32_t o = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = (w4 >> (8 * k)) & 255u;
            const uint32_t t = tm[c * FNL + l];
            const uint32_t idx = f_above(t, S, bits, cnt, l);
            o |= idx << (8 * k);
            const uint32_t ws = t >> 5, wq = ws >> 2;
            tm[c * FNL + l] = (uint16_t)now;
            atomicXor(&bits[ws * FNL + l], 1u << (t & 31u));
            atomicSub(&cnt[wq * FNL + l], 1u << (8 * (ws & 3u)));
            S -= 1u << (8 * wq);
            const uint32_t wn = now >> 5;
            atomicOr(&bits[wn * FNL + l], 1u << (now & 31u));
            atomicAdd(&cnt[(wn >> 2) * FNL + l], 1u << (8 * (wn & 3u)));
            S += 1u << (8 * (wn >> 2));
            if (++now == 512) {  // renumber: slot of each symbol -> 255 - marks above it
                for (uint32_t s = 0; s < 256; ++s) {
                    const uint32_t ts = tm[s * FNL + l];
                    tm[s * FNL + l] = (uint16_t)(255 - f_above(ts, S, bits, cnt, l));
                }
                for (uint32_t w = 0; w < 16; ++w) bits[w * FNL + l] = w < 8 ? 0xffffffffu : 0u;
                for (uint32_t q = 0; q < 4; ++q) cnt[q * FNL + l] = q < 2 ? 0x20202020u : 0u;
                S = 0x00008080u;
                now = 256;
            }
        }
        *(uint32_t *)(dst + i) = o;
    }
}

static void cpu_mtf(const uint8_t *in, uint8_t *out, size_t n)
{
    uint8_t a[256];
    for (int i = 0; i < 256; ++i) a[i] = (uint8_t)i;
    for (size_t i = 0; i < n; ++i) {
        uint8_t c = in[i];
        int j = 0;
        while (a[j] != c) ++j;
        out[i] = (uint8_t)j;
        memmove(a + 1, a, j);
        a[0] = c;
    }
}

int main(int argc, char **argv)
{
    const size_t N = (size_t)1 << 30;
    const uint32_t ch = argc > 1 ? (uint32_t)atoi(argv[1]) : 32768;
    const int text = argc > 2 ? atoi(argv[2]) : 0;
    std::vector<uint8_t> h(N);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < N; i += 8) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        uint64_t v = x;
        if (text) {  // skewed alphabet: mostly small symbols
            for (int k = 0; k < 8; ++k) ((uint8_t *)&v)[k] = (uint8_t)(((v >> (8 * k)) & 255) % 5);
        }
        memcpy(&h[i], &v, 8);
    }
    uint8_t *d_in, *d_out;
    CK(hipMalloc(&d_in, N));
    CK(hipMalloc(&d_out, N));
    CK(hipMemcpy(d_in, h.data(), N, hipMemcpyHostToDevice));
    const uint32_t nch = (uint32_t)(N / ch);
    std::vector<uint8_t> ref(ch), got(ch);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        CK(hipMemset(d_out, 0, N));
        launch();
        CK(hipDeviceSynchronize());
        // check 3 chunks
        bool ok = true;
        for (uint32_t c : {0u, nch / 2 + 1, nch - 1}) {
            cpu_mtf(h.data() + (size_t)c * ch, ref.data(), ch);
            CK(hipMemcpy(got.data(), d_out + (size_t)c * ch, ch, hipMemcpyDeviceToHost));
            ok &= memcmp(ref.data(), got.data(), ch) == 0;
        }
        float best = 1e9f;
        for (int it = 0; it < 3; ++it) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%-14s chunk=%6u ok=%d  %8.3f ms  %7.2f Gsym/s\n", name, ch, (int)ok, best, N / best / 1e6);
        fflush(stdout);
    };
    run("F_lane_ts", [&]() { hipLaunchKernelGGL(k_F, dim3(nch / FNL), dim3(FNL), 0, 0, d_in, d_out, ch); });
    run("A_switch", [&]() { hipLaunchKernelGGL(k_A, dim3(nch), dim3(64), 0, 0, d_in, d_out, ch); });
    run("B_pk16_s1", [&]() { hipLaunchKernelGGL(k_B<1>, dim3(nch / 4), dim3(256), 0, 0, d_in, d_out, ch); });
    run("B_pk16_s2", [&]() { hipLaunchKernelGGL(k_B<2>, dim3(nch / 8), dim3(256), 0, 0, d_in, d_out, ch); });
    run("B_pk16_s4", [&]() { hipLaunchKernelGGL(k_B<4>, dim3(nch / 16), dim3(256), 0, 0, d_in, d_out, ch); });
    run("D_pk_cnd_s1", [&]() { hipLaunchKernelGGL((k_D<0, 1>), dim3(nch / 4), dim3(256), 0, 0, d_in, d_out, ch); });
    run("D_pk_cnd_s2", [&]() { hipLaunchKernelGGL((k_D<0, 2>), dim3(nch / 8), dim3(256), 0, 0, d_in, d_out, ch); });
    run("E_pk_2rl_s1", [&]() { hipLaunchKernelGGL((k_D<1, 1>), dim3(nch / 4), dim3(256), 0, 0, d_in, d_out, ch); });
    run("E_pk_2rl_s2", [&]() { hipLaunchKernelGGL((k_D<1, 2>), dim3(nch / 8), dim3(256), 0, 0, d_in, d_out, ch); });
    run("C_u32_s1", [&]() { hipLaunchKernelGGL(k_C<1>, dim3(nch / 4), dim3(256), 0, 0, d_in, d_out, ch); });
    run("C_u32_s2", [&]() { hipLaunchKernelGGL(k_C<2>, dim3(nch / 8), dim3(256), 0, 0, d_in, d_out, ch); });
    return 0;
}
