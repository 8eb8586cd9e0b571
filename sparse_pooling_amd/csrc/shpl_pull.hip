// shpl_pull.hip -- the SHPL gather / scatter-add as destination-keyed pulls.
//
// Reference ops (TF 1.8 stock kernels, avod/avod/utils/sparse_pool_utils.py):
//   img->BEV  :96-103  gather_nd + sparse_tensor_dense_matmul (+ concat :72)
//   BEV->img  :105-117 sparse_transpose + matmul + scatter_nd  (+ concat :87)
//   and their autodiff gradients.
// TF's GPU kernels scatter with atomics; here every output element is owned by
// exactly one thread, which walks its destination's CSR entries in TF-CPU
// order and writes the element once -- zeros included, the concat fused in.
// No atomics, bitwise reproducible, and the fp32 result equals TF-CPU's
// sequential `out += a*b` (separate multiply and add, no FMA contraction).
//
// Work unit: one 16-byte chunk of one output row (4 f32 / 8 bf16). A
// 64-lane wave stores 1 KiB contiguous; each thread handles U chunks per
// grid-stride step and issues their independent loads (the pass-through row
// read or the two row-pointer words) before any dependent work, so enough
// bytes are in flight to stream HBM.
#include "shpl_common.h"

namespace shpl {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int BYTES>
struct Raw;
template <>
struct Raw<16> {
    typedef u32x4 type;
};
template <>
struct Raw<8> {
    typedef u32x2 type;
};
template <>
struct Raw<4> {
    typedef uint32_t type;
};
template <>
struct Raw<2> {
    typedef uint16_t type;
};

template <typename T, int VEC>
struct Chunk {
    typedef typename Raw<sizeof(T) * VEC>::type raw_t;

    static __device__ __forceinline__ raw_t load(const T *p) { return *reinterpret_cast<const raw_t *>(p); }
    static __device__ __forceinline__ raw_t load_nt(const T *p) {
        return __builtin_nontemporal_load(reinterpret_cast<const raw_t *>(p));
    }
    static __device__ __forceinline__ void store_nt(T *p, raw_t v) {
        __builtin_nontemporal_store(v, reinterpret_cast<raw_t *>(p));
    }
    static __device__ __forceinline__ void to_f32(raw_t r, float (&x)[VEC]) {
        T e[VEC];
        __builtin_memcpy(e, &r, sizeof(r));
#pragma unroll
        for (int j = 0; j < VEC; ++j) x[j] = cvt(e[j]);
    }
    static __device__ __forceinline__ raw_t from_f32(const float (&x)[VEC]) {
        T e[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) e[j] = back(x[j]);
        raw_t r;
        __builtin_memcpy(&r, e, sizeof(r));
        return r;
    }
    static __device__ __forceinline__ float cvt(float v) { return v; }
    static __device__ __forceinline__ float cvt(uint16_t v) { return bf16_to_f32(v); }
    static __device__ __forceinline__ T back(float v) {
        if constexpr (sizeof(T) == 4)
            return v;
        else
            return f32_to_bf16(v);
    }
};

struct PullParams {
    // CSR (sparse role)
    const int32_t *nnz_live;  // &rowptr[n_keys]
    const int32_t *ent_dst, *ent_src, *ent_col;
    const float *ent_val;
    const uint32_t *occ;
    // features
    const void *src;
    int64_t src_stride, src_off;
    const void *pass;
    int64_t pass_stride, pass_off;
    void *out;
    int64_t out_stride;
    // geometry (chunks of VEC elements)
    uint32_t row0, n_rows;  // dense rows of this launch
    uint32_t cpr;           // chunks per output row
    uint32_t cpass;         // chunks of the pass-through half (CONCAT)
    uint32_t cpool;         // chunks of the pooled part
    uint32_t sparse_blocks; // blocks [0, sparse_blocks) run the sparse role
    int mode;
};

template <int VEC>
__device__ __forceinline__ void fma_free_accumulate(float (&acc)[VEC], float w, const float (&x)[VEC]) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], __fmul_rn(w, x[j]));
}

__device__ __forceinline__ bool occupied(const uint32_t *occ, uint32_t row) {
    return (occ[row >> 5] >> (row & 31u)) & 1u;
}

// Sparse role: one thread per (sorted entry s, pooled chunk c); the thread at
// the first entry of a destination walks that destination's entries in CSR
// (= TF) order and writes its pooled chunk once.
template <typename T, int VEC, bool GROUP>
__device__ __forceinline__ void sparse_role(const PullParams &p) {
    typedef Chunk<T, VEC> C;
    const int64_t nnz = *p.nnz_live;
    const int64_t total = nnz * (int64_t)p.cpool;
    const T *src = reinterpret_cast<const T *>(p.src) + p.src_off;
    const T *pass = reinterpret_cast<const T *>(p.pass) + p.pass_off;
    T *out = reinterpret_cast<T *>(p.out);
    const bool concat = p.mode == SHPL_OUT_CONCAT;
    for (int64_t t = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; t < total;
         t += (int64_t)p.sparse_blocks * SHPL_BLOCK) {
        const int64_t s = t / p.cpool;
        const uint32_t c = (uint32_t)(t - s * p.cpool);
        const int32_t key = p.ent_dst[s];
        if (s > 0 && p.ent_dst[s - 1] == key) continue;
        const T *sc = src + (int64_t)c * VEC;
        float acc[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = 0.0f;
        if (GROUP) {
            // TF: Q[k] = sum of k's entries; out = 0 + Q[k1] + Q[k2] ... (ScatterNd order)
            float q[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) q[j] = 0.0f;
            int32_t kprev = p.ent_col[s];
            for (int64_t e = s; e < nnz && p.ent_dst[e] == key; ++e) {
                const int32_t k = p.ent_col[e];
                if (k != kprev) {
#pragma unroll
                    for (int j = 0; j < VEC; ++j) {
                        acc[j] = __fadd_rn(acc[j], q[j]);
                        q[j] = 0.0f;
                    }
                    kprev = k;
                }
                float x[VEC];
                C::to_f32(C::load(sc + (int64_t)p.ent_src[e] * p.src_stride), x);
                fma_free_accumulate<VEC>(q, p.ent_val[e], x);
            }
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], q[j]);
        } else {
            for (int64_t e = s; e < nnz && p.ent_dst[e] == key; ++e) {
                float x[VEC];
                C::to_f32(C::load(sc + (int64_t)p.ent_src[e] * p.src_stride), x);
                fma_free_accumulate<VEC>(acc, p.ent_val[e], x);
            }
        }
        if (p.mode == SHPL_OUT_ADD) {
            float a[VEC];
            C::to_f32(C::load(pass + (int64_t)key * p.pass_stride + (int64_t)c * VEC), a);
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(a[j], acc[j]);
        }
        const uint32_t oc = (concat ? p.cpass : 0u) + c;
        C::store_nt(out + (int64_t)key * p.out_stride + (int64_t)oc * VEC, C::from_f32(acc));
    }
}

// Dense role: every chunk of every row that the sparse role does not own --
// the pass-through half of CONCAT, zeros of empty rows (POOL / CONCAT),
// pass + 0 of empty rows (ADD). U chunks per thread, loads issued first.
template <typename T, int VEC, int U>
__device__ __forceinline__ void dense_role(const PullParams &p, uint32_t vblock, uint32_t vgrid) {
    typedef Chunk<T, VEC> C;
    typedef typename C::raw_t raw_t;
    const uint32_t total = p.n_rows * p.cpr;
    const uint32_t step = vgrid * SHPL_BLOCK;
    const T *pass = reinterpret_cast<const T *>(p.pass) + p.pass_off;
    T *out = reinterpret_cast<T *>(p.out);
    const bool concat = p.mode == SHPL_OUT_CONCAT;
    const bool add = p.mode == SHPL_OUT_ADD;
    for (uint32_t g0 = vblock * SHPL_BLOCK + threadIdx.x; g0 < total; g0 += U * step) {
        uint32_t row[U], ch[U];
        bool store[U], load[U];
        raw_t r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t g = g0 + u * step;
            const bool live = g < total && g >= g0;
            row[u] = live ? p.row0 + g / p.cpr : 0u;
            ch[u] = live ? g - (row[u] - p.row0) * p.cpr : 0u;
            const bool copy = concat && ch[u] < p.cpass;
            store[u] = live && (copy || !occupied(p.occ, row[u]));
            load[u] = store[u] && (copy || add);
            if (load[u]) r[u] = C::load_nt(pass + (int64_t)row[u] * p.pass_stride + (int64_t)ch[u] * VEC);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!store[u]) continue;
            if (add) {  // pass + 0.0f (TF's add_n with an all-zero scatter turns -0 into +0)
                float a[VEC];
                C::to_f32(r[u], a);
#pragma unroll
                for (int j = 0; j < VEC; ++j) a[j] = __fadd_rn(a[j], 0.0f);
                r[u] = C::from_f32(a);
            } else if (!load[u]) {
                float z[VEC];
#pragma unroll
                for (int j = 0; j < VEC; ++j) z[j] = 0.0f;
                r[u] = C::from_f32(z);
            }
            C::store_nt(out + (int64_t)row[u] * p.out_stride + (int64_t)ch[u] * VEC, r[u]);
        }
    }
}

template <typename T, int VEC, bool GROUP, int U>
__global__ __launch_bounds__(SHPL_BLOCK) void k_pull(const PullParams p) {
    if (blockIdx.x < p.sparse_blocks)
        sparse_role<T, VEC, GROUP>(p);
    else
        dense_role<T, VEC, U>(p, blockIdx.x - p.sparse_blocks, gridDim.x - p.sparse_blocks);
}

constexpr int PULL_U = 4;
constexpr int DENSE_BLOCKS_MAX = 256 * 8;
constexpr int SPARSE_BLOCKS_MAX = 512;

template <typename T, int VEC>
int launch_pull(PullParams p, bool group, int64_t nnz_cap, hipStream_t s) {
    const uint64_t total = (uint64_t)p.n_rows * p.cpr;
    const int dense = grid_for((int64_t)((total + PULL_U - 1) / PULL_U), SHPL_BLOCK, DENSE_BLOCKS_MAX);
    const int grid = dense + (int)p.sparse_blocks;
    if (group)
        hipLaunchKernelGGL((k_pull<T, VEC, true, PULL_U>), dim3(grid), dim3(SHPL_BLOCK), 0, s, p);
    else
        hipLaunchKernelGGL((k_pull<T, VEC, false, PULL_U>), dim3(grid), dim3(SHPL_BLOCK), 0, s, p);
    SHPL_LAUNCH_CHECK();
    (void)nnz_cap;
    return SHPL_OK;
}

bool aligned(const void *ptr, int64_t a) { return ((uintptr_t)ptr) % (uintptr_t)a == 0; }

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_pull(int direction, int dtype, const shpl_csr *csr, const void *d_src, int64_t src_stride,
                         int64_t src_off, int64_t c_pool, const void *d_pass, int64_t pass_stride, int64_t pass_off,
                         int64_t c_pass, int mode, void *d_out, int64_t out_stride, void *stream) {
    if (!csr) return SHPL_ERR_ARG;
    if (direction != SHPL_BY_CELL && direction != SHPL_BY_PIXEL) return SHPL_ERR_ARG;
    if (direction == SHPL_BY_PIXEL && csr->nnz_cap > 0 && !csr->ent_col) return SHPL_ERR_ARG;
    if (dtype != SHPL_F32 && dtype != SHPL_BF16) return SHPL_ERR_ARG;
    if (mode < SHPL_OUT_POOL || mode > SHPL_OUT_ADD) return SHPL_ERR_ARG;
    const int64_t n_dst = csr->n_keys;
    if (n_dst < 0 || n_dst >= 2147483647LL || c_pool < 0 || c_pass < 0) return SHPL_ERR_BAD_SHAPE;
    if (n_dst == 0) return SHPL_OK;
    if (!csr->rowptr || !csr->occ || !d_out || (c_pool > 0 && !d_src)) return SHPL_ERR_ARG;
    if (csr->nnz_cap > 0 && (!csr->ent_dst || !csr->ent_src || !csr->ent_val)) return SHPL_ERR_ARG;
    if (mode != SHPL_OUT_POOL && !d_pass) return SHPL_ERR_ARG;
    if (mode == SHPL_OUT_ADD && c_pass != c_pool) return SHPL_ERR_BAD_SHAPE;
    const int64_t width = mode == SHPL_OUT_CONCAT ? c_pass + c_pool : c_pool;
    if (out_stride < width || (c_pool > 0 && src_stride < src_off + c_pool) ||
        (mode != SHPL_OUT_POOL && pass_stride < pass_off + c_pass))
        return SHPL_ERR_BAD_SHAPE;
    if (width == 0) return SHPL_OK;
    const int64_t esz = dtype == SHPL_F32 ? 4 : 2;
    const int64_t vec = 16 / esz;
    // 16-byte chunks need every row start and every channel split on a 16-byte boundary
    bool v16 = c_pool % vec == 0 && out_stride % vec == 0 && aligned(d_out, 16);
    if (c_pool > 0)
        v16 = v16 && src_stride % vec == 0 && src_off % vec == 0 && aligned(d_src, 16);
    if (mode != SHPL_OUT_POOL)
        v16 = v16 && c_pass % vec == 0 && pass_stride % vec == 0 && pass_off % vec == 0 && aligned(d_pass, 16);
    const int64_t v = v16 ? vec : 1;
    PullParams p;
    p.nnz_live = csr->rowptr + n_dst;
    p.ent_dst = csr->ent_dst;
    p.ent_src = csr->ent_src;
    p.ent_col = csr->ent_col;
    p.ent_val = csr->ent_val;
    p.occ = csr->occ;
    p.src = d_src;
    p.src_stride = src_stride;
    p.src_off = src_off;
    p.pass = d_pass;
    p.pass_stride = pass_stride;
    p.pass_off = pass_off;
    p.out = d_out;
    p.out_stride = out_stride;
    p.mode = mode;
    p.cpr = (uint32_t)(width / v);
    p.cpass = mode == SHPL_OUT_CONCAT ? (uint32_t)(c_pass / v) : 0u;
    p.cpool = (uint32_t)(c_pool / v);
    hipStream_t s = (hipStream_t)stream;
    const bool group = direction == SHPL_BY_PIXEL;
    // a launch covers at most 2^31 dense chunks (u32 index math); the sparse
    // role rides on the first launch only
    const int64_t rows_per_launch = ((int64_t)1 << 31) / (int64_t)p.cpr;
    for (int64_t r0 = 0; r0 < n_dst; r0 += rows_per_launch) {
        const int64_t nr = (n_dst - r0) < rows_per_launch ? (n_dst - r0) : rows_per_launch;
        p.row0 = (uint32_t)r0;
        p.n_rows = (uint32_t)nr;
        p.sparse_blocks = (r0 == 0 && c_pool > 0 && csr->nnz_cap > 0)
                              ? (uint32_t)grid_for(csr->nnz_cap * (int64_t)p.cpool, SHPL_BLOCK, SPARSE_BLOCKS_MAX)
                              : 0u;
        int rc;
        if (dtype == SHPL_F32)
            rc = v16 ? launch_pull<float, 4>(p, group, csr->nnz_cap, s) : launch_pull<float, 1>(p, group, csr->nnz_cap, s);
        else
            rc = v16 ? launch_pull<uint16_t, 8>(p, group, csr->nnz_cap, s)
                     : launch_pull<uint16_t, 1>(p, group, csr->nnz_cap, s);
        if (rc) return rc;
    }
    return SHPL_OK;
}
