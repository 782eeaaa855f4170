// Write ceiling of the global pass's record scatter: k_g1_scatter stores one
// 8-byte record per rotation, sorted per 16 K-rotation chunk into contiguous runs of ~16 records
// (~128 B) per 10-bit digit, each run landing at its digit's cursor in the block's bucket (1,024
// buckets of ~4,096 records per 4 MiB block, so consecutive chunks' runs of one digit are
// adjacent). This kernel writes the same pattern with no text, no histogram and no sort: chunk c
// of block b, sorted slot s = k * 1024 + thread: digit d = s / 16, record at
// rec[b][d][c mod 256][s mod 16] (+ an optional per-digit byte shift so runs straddle 128-B lines
// as the real, count-dependent runs do). One 1024-thread workgroup per chunk, 65,536 chunks = 1 GiB
// of rotations = 8 GiB of records, the real grid. Reported: TB/s of record bytes.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench/scatter_ceiling.hip -o tools/microbench/scatter_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr uint32_t kChunk = 16384, kChunksPerBlock = 256, kDigits = 1024;

// mode 0: runs 128-B aligned; mode 1: each digit's region shifted by 8 * (hash(d) % 16) bytes;
// mode 2: as 1, plus the chunk's 16 KiB of text read (one byte per rotation, as the staging does)
// kXcd: workgroup g runs on XCD g mod 8; its chunk is taken from the blocks b = x mod 8 of that
// XCD (k_g1_scatter's lane map), so the two chunks writing the halves of a straddled line share
// an L2 and the line leaves it whole
template <int kMode, bool kXcd>
__global__ __launch_bounds__(1024) void k_scatter(uint64_t *__restrict__ rec, const uint8_t *__restrict__ text, uint32_t nchunks)
{
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    uint32_t c = g;
    if (kXcd) {
        const uint32_t x = g & 7u, k = g >> 3;
        c = ((k / kChunksPerBlock) * 8 + x) * kChunksPerBlock + k % kChunksPerBlock;
    }
    if (c >= nchunks) return;
    const uint32_t b = c / kChunksPerBlock, cb = c % kChunksPerBlock;
    uint32_t salt = 0;
    if (kMode == 2) {  // stage the chunk's text (16 B a thread) and fold it into the records
        const uint4 v = ((const uint4 *)(text + (size_t)c * kChunk))[t];
        salt = v.x ^ v.y ^ v.z ^ v.w;
    }
    // block b's records: 1024 digits x (256 chunks x 16 records) + per-digit slack of 16 records
    uint64_t *rb = rec + (size_t)b * kDigits * (kChunksPerBlock * 16 + 16);
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t s = k * 1024 + t, d = s >> 4, r = s & 15u;
        const uint32_t shift = kMode ? ((d * 2654435761u) >> 28) : 0u;  // 0..15 records
        uint64_t *p = rb + (size_t)d * (kChunksPerBlock * 16 + 16) + shift + cb * 16 + r;
        *p = ((uint64_t)s << 32) | (c ^ salt);
    }
}

int main()
{
    const uint32_t nchunks = 65536;
    const size_t nrec = (size_t)(nchunks / kChunksPerBlock) * kDigits * (kChunksPerBlock * 16 + 16);
    uint64_t *rec;
    uint8_t *text;
    CK(hipMalloc(&rec, nrec * 8));
    CK(hipMalloc(&text, (size_t)nchunks * kChunk));
    CK(hipMemset(text, 7, (size_t)nchunks * kChunk));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)nchunks * kChunk * 8;
    const char *names[] = {"aligned 128-B runs", "runs straddling lines", "straddling + 1 B/rotation text read",
                           "aligned, XCD-mapped chunks", "straddling, XCD-mapped chunks",
                           "straddling + text read, XCD-mapped chunks (k_g1_scatter's pattern)"};
    for (int mode = 0; mode < 6; ++mode) {
        float best = 1e30f, sum = 0;
        const int reps = 10;
        for (int i = 0; i < reps + 2; ++i) {
            CK(hipEventRecord(e0));
            if (mode == 0) hipLaunchKernelGGL((k_scatter<0, false>), dim3(nchunks), dim3(1024), 0, 0, rec, text, nchunks);
            if (mode == 1) hipLaunchKernelGGL((k_scatter<1, false>), dim3(nchunks), dim3(1024), 0, 0, rec, text, nchunks);
            if (mode == 2) hipLaunchKernelGGL((k_scatter<2, false>), dim3(nchunks), dim3(1024), 0, 0, rec, text, nchunks);
            if (mode == 3) hipLaunchKernelGGL((k_scatter<0, true>), dim3(nchunks), dim3(1024), 0, 0, rec, text, nchunks);
            if (mode == 4) hipLaunchKernelGGL((k_scatter<1, true>), dim3(nchunks), dim3(1024), 0, 0, rec, text, nchunks);
            if (mode == 5) hipLaunchKernelGGL((k_scatter<2, true>), dim3(nchunks), dim3(1024), 0, 0, rec, text, nchunks);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (i >= 2) {
                best = ms < best ? ms : best;
                sum += ms;
            }
        }
        printf("{\"pattern\": \"%s\", \"ms_best\": %.4f, \"ms_mean\": %.4f, \"record_TBps_best\": %.3f}\n", names[mode], best,
               sum / reps, bytes / best / 1e9);
    }
    CK(hipGetLastError());
    return 0;
}
