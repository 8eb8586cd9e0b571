// shpl_common.h -- device helpers shared by the SHPL HIP kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shpl.h"

#define SHPL_WAVE 64
#define SHPL_BLOCK 256

#define SHPL_HIP_CHECK(expr)                         \
    do {                                             \
        if ((expr) != hipSuccess) return SHPL_ERR_HIP; \
    } while (0)

#define SHPL_LAUNCH_CHECK()                                   \
    do {                                                      \
        if (hipGetLastError() != hipSuccess) return SHPL_ERR_HIP; \
    } while (0)

namespace shpl {

// Number of set bits of `mask` in lanes below this lane (wave64).
// Wave-wide integer sum and inclusive scan (the device library's DPP / swizzle forms: a chain of ds_bpermute
// shuffles per value was most of the aggregate reads' time in k_index1). Integer sums: any order, same result.
extern "C" __device__ int __ockl_wfred_add_i32(int);
extern "C" __device__ int __ockl_wfscan_add_i32(int, bool);
__device__ __forceinline__ int32_t wave_sum(int32_t v) { return __ockl_wfred_add_i32(v); }
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) { return __ockl_wfscan_add_i32(v, true); }

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Exclusive scan of one int per thread across a 256-thread block.
// `lds` needs SHPL_BLOCK/64 + 1 ints. Returns the exclusive prefix; *total gets the block sum.
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t *lds, int64_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t s = 0;
        for (int w = 0; w < SHPL_BLOCK / 64; ++w) {
            const int64_t t = lds[w];
            lds[w] = s;
            s += t;
        }
        lds[SHPL_BLOCK / 64] = s;
    }
    __syncthreads();
    const int64_t r = x - v + lds[wid];
    *total = lds[SHPL_BLOCK / 64];
    __syncthreads();
    return r;
}

// f32 -> bf16 round-to-nearest-even; NaN stays NaN (quiet): gfx950's
// v_cvt_pk_bf16_f32 (one instruction instead of five integer ones -- the bf16
// conv epilogue converts 64 values per wave and output row).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    const __bf16 b = (__bf16)f;
    uint16_t u;
    __builtin_memcpy(&u, &b, 2);
    return u;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Make this workgroup's global stores visible to its other waves: every wave
// drains its vector-memory stores before the barrier (a workgroup-scope
// __syncthreads does not wait for them on gfx950), then invalidates the
// CU's L1 and waits for the invalidate before its next load
// (MI355X_MICROARCH.md, inter-workgroup visibility: producer / consumer forms).
__device__ __forceinline__ void block_publish() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One row of a 3x4 (or 4x4) matrix times [a0; a1; a2; 1] the way numpy's
// np.dot evaluates it for N >= 2 columns (OpenBLAS dgemm): the first product
// rounded, then a fused multiply-add per k in k order (checked bit-exact
// against numpy; tests/golden/index_*, kitti_frames).
__device__ __forceinline__ double dot4_chain(const double *row, double a0, double a1, double a2) {
    double s = __dmul_rn(row[0], a0);
    s = __fma_rn(row[1], a1, s);
    s = __fma_rn(row[2], a2, s);
    return __fma_rn(row[3], 1.0, s);
}

// The same row product when np.dot has ONE column (a frame of one point, one
// clip survivor): numpy calls OpenBLAS dgemv, which sums the rounded products
// as (p0*a0 + p2*a2) + (p1*a1 + p3*a3) (probed against np.dot; pinned by
// tests/golden/index_single_*, index_one_survivor, kitti_single).
__device__ __forceinline__ double dot4_gemv(const double *row, double a0, double a1, double a2) {
    return __dadd_rn(__dadd_rn(__dmul_rn(row[0], a0), __dmul_rn(row[2], a2)),
                     __dadd_rn(__dmul_rn(row[1], a1), row[3]));
}

__device__ __forceinline__ double dot4(const double *row, double a0, double a1, double a2, bool gemv) {
    return gemv ? dot4_gemv(row, a0, a1, a2) : dot4_chain(row, a0, a1, a2);
}

// projectToImage (avod/avod/utils/transform.py:3-26; calib_utils.project_to_image
// :281-298): [u;v;w] = P [x;y;z;1]; u/=w; v/=w (IEEE division). gemv: the
// product had one column (see dot4_gemv).
// P's 12 values are loaded into registers first, all in flight at once: read inside the two summation
// orders' branches they were 4-8 dependent round trips per point (the index build's longest latency chain).
__device__ __forceinline__ void project(const double *P, double x, double y, double z, double &u, double &v,
                                        bool gemv = false) {
    double p[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) p[k] = P[k];
    const double r0 = dot4(p, x, y, z, gemv), r1 = dot4(p + 4, x, y, z, gemv), r2 = dot4(p + 8, x, y, z, gemv);
    u = __ddiv_rn(r0, r2);
    v = __ddiv_rn(r1, r2);
}

// Workgroup bid of n -> logical block, so that each XCD (blocks dealt round
// robin: bid, bid + 8, ... share one; MI355X_MICROARCH.md §Workgroup dispatch)
// gets one contiguous run of logical blocks and its L2 sees one stretch of the
// data. A bijection on [0, n) for any n (the first n % 8 XCDs get one more).
// Speed only: nothing depends on the placement.
__device__ __forceinline__ int64_t xcd_block(int64_t bid, int64_t n) {
    const int64_t q = n >> 3, r = n & 7, xcd = bid & 7, i = bid >> 3;
    return xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------- buckets
// Destination buckets of the index builder's entries (shpl_build_index_buckets
// -> shpl_build_csr_buckets): per key (0 = BEV cells, 1 = image pixels) a frame's
// destinations are cut into ranges of BK_KEYS; bucket (key, frame, range)
// lists the frame's entries of that range in entry order -- TF's order inside
// every destination -- as 32-bit words (local destination << 24 | entry slot
// - frame start). Workspace, in this order (host-computed, both calls agree):
//   bar   [2][F]                  i32  the one-launch index build's frame barrier words (zero between calls:
//                                        the workspace is zeroed once before its first use)
//   hist  [2][F][n_chunks][nrmax] i32  entries per (index chunk, range)
//   ext   [2][F][nrmax][2]        i32  bucket (start from the frame's first slot, entries)
//   words [2][nnz_cap]            u32  the buckets, frame f's at [off[f], off[f] + nnz_f)
constexpr int BK_KEYS = 128;        // destinations per range
constexpr int BK_MAX_RANGES = 512;  // ranges per frame (65536 destinations)
constexpr int BK_RBITS = 9;         // range bits matched by the placement's multisplit

struct BkLayout {
    int n_frames, n_chunks, nr[2], nrmax;
    int64_t nnz_cap, kpf[2];
    size_t bar, hist, ext, words, bytes;  // byte offsets into the workspace, total
};

inline BkLayout bk_layout(int n_frames, int n_chunks, int64_t nnz_cap, int64_t cells_per_frame,
                          int64_t pix_per_frame) {
    BkLayout l = {};
    l.n_frames = n_frames;
    l.n_chunks = n_chunks;
    l.nnz_cap = nnz_cap;
    l.kpf[0] = cells_per_frame;
    l.kpf[1] = pix_per_frame;
    for (int k = 0; k < 2; ++k) l.nr[k] = (int)((l.kpf[k] + BK_KEYS - 1) / BK_KEYS);
    l.nrmax = l.nr[0] > l.nr[1] ? l.nr[0] : l.nr[1];
    if (l.nrmax < 1) l.nrmax = 1;
    const size_t F = (size_t)n_frames, cap = (size_t)(nnz_cap > 0 ? nnz_cap : 1);
    size_t o = 0;
    l.bar = o;
    o = align_up(o + 4 * 2 * F, 256);
    l.hist = o;
    o = align_up(o + 4 * 2 * F * (size_t)n_chunks * (size_t)l.nrmax, 256);
    l.ext = o;
    o = align_up(o + 4 * 2 * F * (size_t)l.nrmax * 2, 256);
    l.words = o;
    o = align_up(o + 4 * 2 * cap, 256);
    l.bytes = o;
    return l;
}

inline int grid_for(int64_t work, int64_t per_block, int cap) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

namespace {
// Zeros at the streaming rate: one nontemporal 16-byte store per thread over
// a full grid (hipMemsetAsync's fill kernel ran at ~2.2 TB/s on MI355X; this
// shape measured 6.7 TB/s, scripts/calib.hip). Sizes in 8-byte words.
__global__ __launch_bounds__(SHPL_BLOCK) void k_zero_fill(uint64_t *p, uint64_t n8) {
    const uint64_t i = (uint64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x;
    typedef uint32_t u32x4z __attribute__((ext_vector_type(4)));
    if (2 * i + 1 < n8) {
        __builtin_nontemporal_store(u32x4z{0u, 0u, 0u, 0u}, reinterpret_cast<u32x4z *>(p) + i);
    } else if (2 * i < n8) {
        p[2 * i] = 0;  // an odd word count's last word
    }
}

// Zero `bytes` (a multiple of 8) at `ptr` on `s`; hipMemsetAsync when the
// pointer is not 16-byte aligned or the size not a whole number of words.
inline hipError_t zero_fill(void *ptr, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (((uintptr_t)ptr & 15u) || (bytes & 7u)) return hipMemsetAsync(ptr, 0, bytes, s);
    const uint64_t n8 = bytes / 8, threads = (n8 + 1) / 2;
    const uint64_t blocks = (threads + SHPL_BLOCK - 1) / SHPL_BLOCK;
    if (blocks >= (1ull << 31)) return hipMemsetAsync(ptr, 0, bytes, s);
    hipLaunchKernelGGL(k_zero_fill, dim3((unsigned)blocks), dim3(SHPL_BLOCK), 0, s, reinterpret_cast<uint64_t *>(ptr),
                       n8);
    return hipGetLastError();
}
}  // namespace

}  // namespace shpl
