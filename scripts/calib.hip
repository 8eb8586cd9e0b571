// Calibration kernels for the pull sweep (not part of libshpl): the best a
// plain streaming kernel does on this box for the same traffic shapes.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t n) {
    uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x);
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (; i0 < n; i0 += U * step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * step;
            if (i < n) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u * step;
            if (i < n) {
                if (NT) __builtin_nontemporal_store(v[u], d + i); else d[i] = v[u];
            }
        }
    }
}

// out row r (cpr chunks): first cpass chunks copied from src row r, rest zero
template <bool NT>
__global__ __launch_bounds__(256) void k_concat_zero(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint32_t rows,
                                                     uint32_t cpr, uint32_t cpass) {
    const uint32_t total = rows * cpr;
    for (uint32_t g = blockIdx.x * 256 + threadIdx.x; g < total; g += gridDim.x * 256) {
        const uint32_t r = g / cpr, c = g - r * cpr;
        u32x4 v = {0, 0, 0, 0};
        if (c < cpass) v = NT ? __builtin_nontemporal_load(s + (uint64_t)r * cpass + c) : s[(uint64_t)r * cpass + c];
        if (NT) __builtin_nontemporal_store(v, d + g); else d[g] = v;
    }
}

// zero fill only
__global__ __launch_bounds__(256) void k_zero(u32x4 *__restrict__ d, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        u32x4 z = {0, 0, 0, 0};
        __builtin_nontemporal_store(z, d + i);
    }
}

extern "C" int calib_copy(const void *s, void *d, uint64_t n16, int unroll, int nt, int grid, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (grid <= 0) grid = (int)((n16 + 256ull * unroll - 1) / (256ull * unroll));
#define L(U, N) hipLaunchKernelGGL((k_copy<U, N>), dim3(grid), dim3(256), 0, st, (const u32x4 *)s, (u32x4 *)d, n16)
    if (unroll == 1) { if (nt) L(1, true); else L(1, false); }
    else if (unroll == 2) { if (nt) L(2, true); else L(2, false); }
    else { if (nt) L(4, true); else L(4, false); }
#undef L
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

extern "C" int calib_concat_zero(const void *s, void *d, uint32_t rows, uint32_t cpr, uint32_t cpass, int nt, int grid,
                                 void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (grid <= 0) grid = (int)(((uint64_t)rows * cpr + 255) / 256);
    if (nt) hipLaunchKernelGGL(k_concat_zero<true>, dim3(grid), dim3(256), 0, st, (const u32x4 *)s, (u32x4 *)d, rows, cpr, cpass);
    else hipLaunchKernelGGL(k_concat_zero<false>, dim3(grid), dim3(256), 0, st, (const u32x4 *)s, (u32x4 *)d, rows, cpr, cpass);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

extern "C" int calib_zero(void *d, uint64_t n16, int grid, void *stream) {
    if (grid <= 0) grid = (int)((n16 + 255) / 256);
    hipLaunchKernelGGL(k_zero, dim3(grid), dim3(256), 0, (hipStream_t)stream, (u32x4 *)d, n16);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
