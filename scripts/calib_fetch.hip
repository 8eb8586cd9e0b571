// calib_fetch.hip -- what TCC_EA0_RDREQ counts per byte read, for the access patterns of this repo's kernels
// (PMC calibration, not part of the library). Each kernel reads every byte of a 1 GiB buffer exactly once:
//   k_coal      16 B per lane, consecutive lanes on consecutive 16 B (k_dense's streaming reads)
//   k_pix       16 B per lane, lane l on pixel l (128-byte pixels), the 8 pieces of a pixel by 8 successive
//               instructions (the row conv's operand gathers, as plain loads)
//   k_pix_dma   the same pattern by LDS-DMA (global_load_lds_dwordx4, the conv kernels' staging)
// Run under rocprofv3 --pmc TCC_EA0_RDREQ_sum ...: RDREQ x 128 B == 1 GiB means 128-byte requests.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr size_t BYTES = size_t(1) << 30;
constexpr int BLOCK = 256;

__global__ __launch_bounds__(BLOCK) void k_coal(const u32x4 *src, uint32_t *sink, size_t n16) {
    uint32_t x = 0;
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n16; i += (size_t)gridDim.x * BLOCK) {
        const u32x4 v = src[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) sink[0] = x;
}

// a wave per 64 pixels: instruction p reads piece p of the wave's 64 pixels
__global__ __launch_bounds__(BLOCK) void k_pix(const u32x4 *src, uint32_t *sink, size_t n_px) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * BLOCK + threadIdx.x) >> 6, waves = ((size_t)gridDim.x * BLOCK) >> 6;
    uint32_t x = 0;
    for (size_t px0 = wave * 64; px0 < n_px; px0 += waves * 64) {
        const size_t px = px0 + lane;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const u32x4 v = src[px * 8 + p];
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (x == 0x12345678u) sink[0] = x;
}

__global__ __launch_bounds__(BLOCK) void k_pix_dma(const u32x4 *src, uint32_t *sink, size_t n_px) {
    __shared__ __attribute__((aligned(1024))) uint8_t lds[4][8][1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t wave = ((size_t)blockIdx.x * BLOCK + threadIdx.x) >> 6, waves = ((size_t)gridDim.x * BLOCK) >> 6;
    for (size_t px0 = wave * 64; px0 < n_px; px0 += waves * 64) {
        const size_t px = px0 + lane;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const uint32_t m0 = (uint32_t)(uintptr_t)&lds[w][p][0];
            asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src + px * 8 + p), "{m0}"(m0) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (lane == 0 && lds[w][0][0] == 0x5a && sink[1] == 0x12345678u) sink[0] = 1;
}

int main() {
    u32x4 *src;
    uint32_t *sink;
    if (hipMalloc(&src, BYTES) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(src, 1, BYTES);
    hipMemset(sink, 0, 64);
    const int grid = 256 * 8;
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_coal, dim3(grid), dim3(BLOCK), 0, 0, src, sink, BYTES / 16);
        hipLaunchKernelGGL(k_pix, dim3(grid), dim3(BLOCK), 0, 0, src, sink, BYTES / 128);
        hipLaunchKernelGGL(k_pix_dma, dim3(grid), dim3(BLOCK), 0, 0, src, sink, BYTES / 128);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("calib_fetch: 3 x (k_coal, k_pix, k_pix_dma) over %zu bytes each\n", BYTES);
    hipFree(src);
    hipFree(sink);
    return 0;
}
