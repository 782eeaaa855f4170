// Standalone check of the wave lane-exchange primitives used by the BWT bitonic network
// (bwt.hip lane_xor<X>): every lane must read lane l ^ X. Prints "lane_xor ok" or the mismatches.
#include <hip/hip_runtime.h>

#include <cstdio>

template <unsigned X>
__device__ __forceinline__ unsigned lane_xor(unsigned v)
{
    if constexpr (X == 1) {
        return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    } else if constexpr (X == 2) {
        return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    } else if constexpr (X == 4 || X == 8) {
        return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (X << 10));
    } else if constexpr (X == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (__lane_id() & 16u) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (__lane_id() & 32u) ? r[0] : r[1];
    }
}

__global__ void k(unsigned *out)
{
    const unsigned l = threadIdx.x, v = 1000u + l;
    out[0 * 64 + l] = lane_xor<1>(v);
    out[1 * 64 + l] = lane_xor<2>(v);
    out[2 * 64 + l] = lane_xor<4>(v);
    out[3 * 64 + l] = lane_xor<8>(v);
    out[4 * 64 + l] = lane_xor<16>(v);
    out[5 * 64 + l] = lane_xor<32>(v);
}

int main()
{
    unsigned *d, h[6 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    (void)hipFree(d);
    int bad = 0;
    for (int s = 0; s < 6; ++s)
        for (unsigned l = 0; l < 64; ++l)
            if (h[s * 64 + l] != 1000u + (l ^ (1u << s))) {
                if (bad++ < 10) printf("X=%u lane %u got %u want %u\n", 1u << s, l, h[s * 64 + l] - 1000u, l ^ (1u << s));
            }
    printf(bad ? "lane_xor FAILED\n" : "lane_xor ok\n");
    return bad ? 1 : 0;
}
