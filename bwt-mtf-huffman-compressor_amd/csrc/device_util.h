// device_util.h — wave64 / workgroup primitives shared by the kernels (gfx950: wave = 64).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "bmh_internal.h"

namespace bmh {

constexpr int kWave = 64;

// v_writelane_b32: the LLVM intrinsic bound directly (no clang builtin for it in ROCm 7.2).
extern "C" __device__ int __bmh_llvm_writelane(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t writelane(uint32_t val, uint32_t lane, uint32_t old)
{
    return (uint32_t)__bmh_llvm_writelane((int)val, (int)lane, (int)old);
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Checked builds (-DBMH_CHECK, `make check`): device-side preconditions are counted, never
// trapped, in a per-translation-unit table the host reads through bmh_check_violations().
//   kCheckExec: a full-wave primitive (DPP scans, the one-barrier workgroup scan) ran with
//   a partial EXEC mask — inactive lanes feed stale values into the DPP row shifts and
//   broadcasts, so the sums (and every slot derived from them) are wrong.
#ifdef BMH_CHECK
namespace {
__device__ uint32_t g_check_bad[kCheckKinds];
uint32_t check_read_tu(uint32_t kind)
{
    uint32_t v[kCheckKinds] = {};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_check_bad), sizeof(v)) != hipSuccess) return 0xffffffffu;
    return v[kind];
}
const bool check_registered = (check_register(&check_read_tu), true);
}  // namespace
__device__ __forceinline__ void check_full_exec()
{
    if (__builtin_amdgcn_read_exec() != ~0ull) atomicAdd(&g_check_bad[kCheckExec], 1u);
}
#else
__device__ __forceinline__ void check_full_exec() {}
#endif

// Ordering point for LDS data that only the calling wave reads and writes: a wave's LDS
// operations execute in order, so no barrier is needed, only that the compiler keeps the
// accesses on their side of this point.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One slot of a global list for every active lane, with ONE atomic per wave: callers in
// divergent code get consecutive indices (single-lane atomics on a shared counter serialise
// at the L2 when thousands of waves append). `ctr` must be the same for every active lane.
__device__ __forceinline__ uint32_t wave_append(uint32_t *ctr)
{
    const uint64_t act = __ballot(1);
    const uint32_t leader = (uint32_t)__builtin_ctzll(act);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(ctr, (uint32_t)__builtin_popcountll(act));
    base = (uint32_t)__shfl((int)base, (int)leader, 64);
    return base + rank;
}

// Raw buffer loads: a buffer resource over [p, p + bytes), and loads by 32-bit byte offset
// whose out-of-range lanes read 0 (the hardware bounds check: no branch, no clamp, and no
// 64-bit address registers per load). The whole offset is in the VGPR operand (the SGPR
// offset is not part of the range check).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint64_t buf_load_u64(__amdgpu_buffer_rsrc_t r, uint32_t byte_off)
{
    return __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)byte_off, 0, 0));
}

// Inclusive wave64 scans.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t x)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    return x;
}
// Wave-wide totals (every lane gets the sum).
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x = x > y ? x : y;
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_min_rev(uint32_t x)  // suffix min (from the right)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_down(x, o, 64);
        if (l + o < 64u) x = x < y ? x : y;
    }
    return x;
}

// Workgroup exclusive sum of one value per thread. s_tmp needs NT/64 + 1 words.
// Inclusive wave64 sum by DPP (row shifts inside each 16-lane row, then the row broadcasts
// of lanes 15 and 31): six VALU steps instead of six dependent ds_bpermute round trips. Every
// lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t x)
{
    check_full_exec();
    // update_dpp(old, src, ctrl, row_mask, bank_mask, bound_ctrl): lanes whose source is out of
    // the row, and rows outside row_mask, get `old` = 0
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Wave64 total by the DPP scan and a read of lane 63 (every lane active).
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_dpp(x), 63);
}

// Workgroup exclusive sum with ONE barrier: each wave publishes its total, then every wave adds
// the totals of the waves below it (broadcast LDS reads). The caller must pass a barrier before
// s_tmp[0, NT / 64) is written again. All threads of the workgroup must call it.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_sum1(uint32_t v, uint32_t *s_tmp, uint32_t *total = nullptr)
{
    constexpr int NW = NT / 64;
    check_full_exec();
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t inc = wave_incl_sum_dpp(v);
    if (lane_id() == 63) s_tmp[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        const uint32_t x = s_tmp[j];
        pre += (uint32_t)j < w ? x : 0u;
        tot += x;
    }
    if (total) *total = tot;
    return pre + inc - v;
}

template <int NT>
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t *s_tmp, uint32_t *total)
{
    constexpr int NW = NT / 64;
    const uint32_t w = threadIdx.x >> 6, l = lane_id();
    uint32_t inc = wave_incl_sum(v);
    if (l == 63) s_tmp[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint32_t t = l < (uint32_t)NW ? s_tmp[l] : 0u;
        uint32_t ti = wave_incl_sum(t);
        if (l < (uint32_t)NW) s_tmp[l] = ti - t;
        if (l == (uint32_t)NW - 1) s_tmp[NW] = ti;
    }
    __syncthreads();
    uint32_t r = s_tmp[w] + inc - v;
    if (total) *total = s_tmp[NW];
    __syncthreads();
    return r;
}

template <int NT>
__device__ __forceinline__ uint64_t block_excl_sum64(uint64_t v, uint64_t *s_tmp, uint64_t *total)
{
    constexpr int NW = NT / 64;
    const uint32_t w = threadIdx.x >> 6, l = lane_id();
    uint64_t inc = wave_incl_sum64(v);
    if (l == 63) s_tmp[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint64_t t = l < (uint32_t)NW ? s_tmp[l] : 0ull;
        uint64_t ti = wave_incl_sum64(t);
        if (l < (uint32_t)NW) s_tmp[l] = ti - t;
        if (l == (uint32_t)NW - 1) s_tmp[NW] = ti;
    }
    __syncthreads();
    uint64_t r = s_tmp[w] + inc - v;
    if (total) *total = s_tmp[NW];
    __syncthreads();
    return r;
}

// Workgroup exclusive max (identity 0) and exclusive suffix min (identity `ident`).
template <int NT>
__device__ __forceinline__ uint32_t block_excl_max(uint32_t v, uint32_t *s_tmp)
{
    constexpr int NW = NT / 64;
    const uint32_t w = threadIdx.x >> 6, l = lane_id();
    uint32_t inc = wave_incl_max(v);
    uint32_t prev = __shfl_up(inc, 1, 64);
    if (l == 0) prev = 0;
    if (l == 63) s_tmp[w] = inc;
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t i = 0; i < w; ++i) carry = carry > s_tmp[i] ? carry : s_tmp[i];
    __syncthreads();
    (void)NW;
    return carry > prev ? carry : prev;
}
template <int NT>
__device__ __forceinline__ uint32_t block_excl_min_rev(uint32_t v, uint32_t ident, uint32_t *s_tmp)
{
    constexpr int NW = NT / 64;
    const uint32_t w = threadIdx.x >> 6, l = lane_id();
    uint32_t inc = wave_incl_min_rev(v);
    uint32_t nxt = __shfl_down(inc, 1, 64);
    if (l == 63) nxt = ident;
    if (l == 0) s_tmp[w] = inc;
    __syncthreads();
    uint32_t carry = ident;
    for (uint32_t i = w + 1; i < (uint32_t)NW; ++i) carry = carry < s_tmp[i] ? carry : s_tmp[i];
    __syncthreads();
    return carry < nxt ? carry : nxt;
}

// Block containing global slot g: boffs has nb+1 ascending entries.
__device__ __forceinline__ uint32_t find_block(const uint32_t *__restrict__ boffs, uint32_t nb, uint32_t g)
{
    uint32_t lo = 0, hi = nb;  // boffs[lo] <= g < boffs[hi]
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (boffs[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

}  // namespace bmh
