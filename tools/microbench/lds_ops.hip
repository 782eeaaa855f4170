// LDS instruction cost on gfx950: cycles per wave-instruction (per CU) for the LDS operations the
// MTF encode step issues, each lane in its own bank (row k of lane l = dword k * 64 + l, the
// encode's layout), 1..8 waves per CU. Also the encode step's current op mix and candidates.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench/lds_ops.hip -o tools/microbench/lds_ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kIters = 2048;

// op: 0 rd_b32, 1 rd_u8, 2 rd_b64, 3 wr_b32, 4 wr_b8, 5 or_b32, 6 add_u32, 7 xor_b32, 8 or_b64,
//     9 wr_b64, 10 rd2_b32 (two rows), 11 mix_old (10 ops), 12 mix_new (7 ops), 13 mix_new_plain
//     (7 ops, the two epoch / mark ORs as plain stores), 14 rd_b128
template <int OP>
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, uint64_t *cyc, uint32_t seed)
{
    extern __shared__ uint32_t lds[];  // waves x 92 rows x 64 lanes
    const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63u;
    const uint32_t wr = w % 6; uint32_t *base = lds + wr * (96 * 64);
    for (int k = 0; k < 96; ++k) base[k * 64 + l] = k + l;
    __syncthreads();
    const uint32_t l4 = 4 * l + wr * 96 * 256;
    uint32_t x = seed * 2654435761u + t * 40503u, acc = 0;
    const uint64_t t0 = clock64();
    for (int i = 0; i < kIters; ++i) {
        x = x * 1664525u + 1013904223u;
        const uint32_t r0 = (x >> 8) & 63u, r1 = (x >> 14) & 63u, r2 = (x >> 20) & 63u, r3 = (x >> 26) & 31u;
        const uint32_t a0 = (r0 << 8) + l4, a1 = (r1 << 8) + l4, a2 = (r2 << 8) + l4, a3 = (r3 << 8) + l4;
        const uint32_t a64 = ((r3 & 15u) << 9) + 8 * l + wr * 96 * 256;  // 64-bit rows (b64 ops)
        uint32_t v0, v1, v2, v3;
        if constexpr (OP == 0) {
            asm volatile("ds_read_b32 %0, %4\n ds_read_b32 %1, %5\n ds_read_b32 %2, %6\n ds_read_b32 %3, %7\n s_waitcnt lgkmcnt(0)"
                         : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
            acc += v0 ^ v1 ^ v2 ^ v3;
        } else if constexpr (OP == 1) {
            asm volatile("ds_read_u8 %0, %4\n ds_read_u8 %1, %5\n ds_read_u8 %2, %6\n ds_read_u8 %3, %7\n s_waitcnt lgkmcnt(0)"
                         : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3) : "v"(a0 + 1), "v"(a1 + 2), "v"(a2 + 3), "v"(a3));
            acc += v0 ^ v1 ^ v2 ^ v3;
        } else if constexpr (OP == 2) {
            uint64_t q0, q1, q2, q3;
            const uint32_t b0 = ((r0 & 15u) << 9) + 8 * l + wr * 96 * 256, b1 = ((r1 & 15u) << 9) + 8 * l + wr * 96 * 256;
            const uint32_t b2 = ((r2 & 15u) << 9) + 8 * l + wr * 96 * 256;
            asm volatile("ds_read_b64 %0, %4\n ds_read_b64 %1, %5\n ds_read_b64 %2, %6\n ds_read_b64 %3, %7\n s_waitcnt lgkmcnt(0)"
                         : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3) : "v"(b0), "v"(b1), "v"(b2), "v"(a64));
            acc += (uint32_t)(q0 ^ q1 ^ q2 ^ q3) ^ (uint32_t)((q0 ^ q3) >> 32);
        } else if constexpr (OP == 3) {
            asm volatile("ds_write_b32 %0, %4\n ds_write_b32 %1, %4\n ds_write_b32 %2, %4\n ds_write_b32 %3, %4"
                         :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(x));
        } else if constexpr (OP == 4) {
            asm volatile("ds_write_b8 %0, %4\n ds_write_b8 %1, %4\n ds_write_b8 %2, %4\n ds_write_b8 %3, %4"
                         :: "v"(a0 + 1), "v"(a1 + 2), "v"(a2 + 3), "v"(a3), "v"(x));
        } else if constexpr (OP == 5) {
            asm volatile("ds_or_b32 %0, %4\n ds_or_b32 %1, %4\n ds_or_b32 %2, %4\n ds_or_b32 %3, %4"
                         :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(x));
        } else if constexpr (OP == 6) {
            asm volatile("ds_add_u32 %0, %4\n ds_add_u32 %1, %4\n ds_add_u32 %2, %4\n ds_add_u32 %3, %4"
                         :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(x));
        } else if constexpr (OP == 7) {
            asm volatile("ds_xor_b32 %0, %4\n ds_xor_b32 %1, %4\n ds_xor_b32 %2, %4\n ds_xor_b32 %3, %4"
                         :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(x));
        } else if constexpr (OP == 8) {
            const uint64_t d = ((uint64_t)x << 32) | x;
            asm volatile("ds_or_b64 %0, %4\n ds_or_b64 %1, %4\n ds_or_b64 %2, %4\n ds_or_b64 %3, %4"
                         :: "v"(a64), "v"(a64 + 512), "v"(a64 + 1024), "v"(a64 + 1536), "v"(d));
        } else if constexpr (OP == 9) {
            const uint64_t d = ((uint64_t)x << 32) | x;
            asm volatile("ds_write_b64 %0, %4\n ds_write_b64 %1, %4\n ds_write_b64 %2, %4\n ds_write_b64 %3, %4"
                         :: "v"(a64), "v"(a64 + 512), "v"(a64 + 1024), "v"(a64 + 1536), "v"(d));
        } else if constexpr (OP == 10) {
            uint64_t q0, q1, q2, q3;
            asm volatile("ds_read2st64_b32 %0, %4 offset1:1\n ds_read2st64_b32 %1, %5 offset1:1\n ds_read2st64_b32 %2, %6 offset1:1\n ds_read2st64_b32 %3, %7 offset1:1\n s_waitcnt lgkmcnt(0)"
                         : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3) : "v"(a0 & 0x7fffu), "v"(a1 & 0x7fffu), "v"(a2 & 0x7fffu), "v"(a3 & 0x7fffu));
            acc += (uint32_t)(q0 ^ q1 ^ q2 ^ q3) ^ (uint32_t)((q0 ^ q3) >> 32);
        }
        if constexpr (OP == 11) {  // the current step: 4 reads, 6 writes / atomics
            asm volatile(
                "ds_read_u8 %0, %4\n ds_read_b32 %1, %5 offset:16384\n ds_read_b32 %2, %6 offset:18432\n ds_read_b32 %3, %7 offset:22528\n"
                "ds_xor_b32 %6, %8 offset:18432\n ds_add_u32 %7, %8 offset:22528\n ds_or_b32 %5, %8 offset:18432\n ds_add_u32 %5, %8 offset:22528\n"
                "ds_write_b8 %4, %8\n ds_or_b32 %5, %8 offset:16384\n s_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
                : "v"(a0 + 1), "v"(((r1 & 7u) << 8) + l4), "v"(((r2 & 15u) << 8) + l4), "v"(((r3 & 3u) << 8) + l4), "v"(x));
            acc += v0 ^ v1 ^ v2 ^ v3;
        } else if constexpr (OP == 12) {  // candidate: u8 + b32 + b64 reads, xor + or + or atomics, b8 store
            uint64_t q;
            asm volatile(
                "ds_read_u8 %0, %3\n ds_read_b32 %1, %4 offset:16384\n ds_read_b64 %2, %5 offset:18432\n"
                "ds_xor_b32 %5, %6 offset:18432\n ds_or_b32 %4, %6 offset:18436\n"
                "ds_write_b8 %3, %6\n ds_or_b32 %4, %6 offset:16384\n s_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(q)
                : "v"(a0 + 1), "v"(((r1 & 7u) << 8) + l4), "v"(((r2 & 7u) << 9) + 8 * l + wr * 96 * 256), "v"(x));
            acc += v0 ^ v1 ^ (uint32_t)q ^ (uint32_t)(q >> 32);
        } else if constexpr (OP == 13) {  // candidate with the ORs as plain stores
            uint64_t q;
            asm volatile(
                "ds_read_u8 %0, %3\n ds_read_b32 %1, %4 offset:16384\n ds_read_b64 %2, %5 offset:18432\n"
                "ds_xor_b32 %5, %6 offset:18432\n ds_write_b32 %4, %6 offset:18436\n"
                "ds_write_b8 %3, %6\n ds_write_b32 %4, %6 offset:16384\n s_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(q)
                : "v"(a0 + 1), "v"(((r1 & 7u) << 8) + l4), "v"(((r2 & 7u) << 9) + 8 * l + wr * 96 * 256), "v"(x));
            acc += v0 ^ v1 ^ (uint32_t)q ^ (uint32_t)(q >> 32);
        } else if constexpr (OP == 14) {
            uint4 q0, q1;
            const uint32_t b0 = ((r0 & 7u) << 10) + 16 * l + wr * 96 * 256, b1 = ((r1 & 7u) << 10) + 16 * l + wr * 96 * 256;
            asm volatile("ds_read_b128 %0, %2\n ds_read_b128 %1, %3\n s_waitcnt lgkmcnt(0)" : "=&v"(q0), "=&v"(q1) : "v"(b0), "v"(b1));
            acc += q0.x ^ q1.y ^ q0.z ^ q1.w;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t1 = clock64();
    if (l == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
    out[blockIdx.x * blockDim.x + t] = acc;
}

template <int OP>
static double run(int waves, uint32_t *d_out, uint64_t *d_cyc, int cus)
{
    const size_t lds = (size_t)(waves < 6 ? waves : 6) * 96 * 256;
    hipFuncSetAttribute((const void *)k_lds<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_lds<OP>, dim3(cus), dim3(64 * waves), lds, 0, d_out, d_cyc, 1u);
    hipLaunchKernelGGL(k_lds<OP>, dim3(cus), dim3(64 * waves), lds, 0, d_out, d_cyc, 2u);
    hipDeviceSynchronize();
    std::vector<uint64_t> h((size_t)cus * 16);
    hipMemcpy(h.data(), d_cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < cus; ++b)
        for (int w = 0; w < waves; ++w) s += (double)h[(size_t)b * 16 + w];
    const double mean = s / (cus * waves);                         // cycles per wave for the loop
    const int ops = OP == 11 ? 10 : OP == 12 || OP == 13 ? 7 : OP == 14 ? 2 : 4;
    return mean / ((double)kIters * ops) / waves;                  // CU cycles per wave-instruction
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *d_out;
    uint64_t *d_cyc;
    CK(hipMalloc(&d_out, (size_t)cus * 1024 * 4));
    CK(hipMalloc(&d_cyc, (size_t)cus * 16 * 8));
    const char *names[] = {"rd_b32", "rd_u8", "rd_b64", "wr_b32", "wr_b8", "or_b32", "add_u32", "xor_b32", "or_b64",
                           "wr_b64", "rd2st64", "mix_old10", "mix_new7", "mix_new7pl", "rd_b128"};
    printf("CU cycles per wave-instruction (own-bank rows), by waves per CU (one workgroup per CU)\n%-12s", "op");
    const int wv[] = {1, 2, 4, 6, 7, 8, 12, 16};
    for (int w : wv) printf(" %7d", w);
    printf("\n");
    for (int op = 11; op < 15; ++op) {
        printf("%-12s", names[op]);
        for (int w : wv) {
            double c = 0;
            switch (op) {
            case 0: c = run<0>(w, d_out, d_cyc, cus); break;
            case 1: c = run<1>(w, d_out, d_cyc, cus); break;
            case 2: c = run<2>(w, d_out, d_cyc, cus); break;
            case 3: c = run<3>(w, d_out, d_cyc, cus); break;
            case 4: c = run<4>(w, d_out, d_cyc, cus); break;
            case 5: c = run<5>(w, d_out, d_cyc, cus); break;
            case 6: c = run<6>(w, d_out, d_cyc, cus); break;
            case 7: c = run<7>(w, d_out, d_cyc, cus); break;
            case 8: c = run<8>(w, d_out, d_cyc, cus); break;
            case 9: c = run<9>(w, d_out, d_cyc, cus); break;
            case 10: c = run<10>(w, d_out, d_cyc, cus); break;
            case 11: c = run<11>(w, d_out, d_cyc, cus); break;
            case 12: c = run<12>(w, d_out, d_cyc, cus); break;
            case 13: c = run<13>(w, d_out, d_cyc, cus); break;
            case 14: c = run<14>(w, d_out, d_cyc, cus); break;
            }
            printf(" %7.2f", c);
        }
        printf("\n");
    }
    CK(hipGetLastError());
    return 0;
}
