// shpl_csr.hip -- the correspondence matrix M on the device: validation /
// packing of the reference's SparseTensor and the destination-keyed CSR
// that turns TF's atomic scatter into a deterministic pull.
//
// Reference: M = tf.SparseTensor(Mij, M_val, M_size) built from the
// placeholders (avod/avod/core/models/rpn_model.py:328-336,
// retinanet_model.py:330-340, MV3D_TF_release/lib/networks/MV3D_voxel_train.py:41-46)
// and consumed by gather_nd / sparse_tensor_dense_matmul / sparse_transpose /
// scatter_nd (avod/avod/utils/sparse_pool_utils.py:96-117).
//
// CSR build (all launches stream-ordered, no host sync):
//   memset counts -> histogram (atomicAdd per entry) -> 3-phase exclusive scan
//   -> placement (atomicSub slot, arbitrary order inside a destination)
//   -> rank fix-up: each entry counts the entries of its destination that
//      precede it in TF order and moves to that rank (deterministic, stable).
// Destinations hold few entries (one to a few dozen), so the quadratic rank
// is cheaper than a second sort pass.
#include "shpl_common.h"

namespace shpl {
namespace {

// ------------------------------------------------------------------ pack
template <typename IT>
__global__ __launch_bounds__(SHPL_BLOCK) void k_pack(int64_t nnz, const int64_t *mij, const float *values,
                                                     int64_t n_values, int64_t n_rows, int64_t n_cols,
                                                     const IT *idx, int64_t img_b, int64_t img_h,
                                                     int64_t img_w, int64_t row_base, int64_t col_base,
                                                     int64_t pix_base, int32_t *cell, int32_t *col,
                                                     float *val, int32_t *pix, uint32_t *err) {
    const int64_t n = nnz > n_cols ? nnz : n_cols;
    uint32_t bits = 0;
    for (int64_t t = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * SHPL_BLOCK) {
        if (t < nnz) {
            const int64_t r = mij[2 * t], k = mij[2 * t + 1];
            const bool rok = r >= 0 && r < n_rows;
            const bool kok = k >= 0 && k < n_cols;
            bits |= (rok ? 0u : SHPL_EBIT_ROW) | (kok ? 0u : SHPL_EBIT_COL);
            cell[t] = (rok && kok) ? (int32_t)(row_base + r) : -1;
            col[t] = kok ? (int32_t)(col_base + k) : -1;
            val[t] = t < n_values ? values[t] : 0.0f;
        }
        if (t < n_cols) {  // GatherNd / ScatterNd index check of every row of idx
            const int64_t b = (int64_t)idx[3 * t], y = (int64_t)idx[3 * t + 1], x = (int64_t)idx[3 * t + 2];
            const bool ok = b >= 0 && b < img_b && y >= 0 && y < img_h && x >= 0 && x < img_w;
            bits |= ok ? 0u : SHPL_EBIT_PIXEL;
            pix[col_base + t] = ok ? (int32_t)(pix_base + (b * img_h + y) * img_w + x) : -1;
        }
    }
    if (n_values != nnz && blockIdx.x == 0 && threadIdx.x == 0) bits |= SHPL_EBIT_VALUES;
    if (bits && err) atomicOr(err, bits);
}

// ------------------------------------------------------------------ CSR
struct CsrIn {
    int direction, order;
    int64_t nnz_cap;
    const int64_t *d_nnz;
    const int32_t *cell, *col, *pix;
    const float *val;
};

__device__ __forceinline__ int64_t live_nnz(const CsrIn &c) {
    if (!c.d_nnz) return c.nnz_cap;
    const int64_t n = *c.d_nnz;
    return n < c.nnz_cap ? n : c.nnz_cap;
}

__device__ __forceinline__ int32_t col_of(const CsrIn &c, int64_t e) { return c.col ? c.col[e] : (int32_t)e; }

// Destination key of entry e, or -1 if the entry is invalid (already flagged).
__device__ __forceinline__ int32_t key_of(const CsrIn &c, int64_t e) {
    const int32_t r = c.cell[e];
    const int32_t k = col_of(c, e);
    if (r < 0 || k < 0) return -1;
    const int32_t p = c.pix[k];
    if (p < 0) return -1;
    return c.direction == SHPL_BY_CELL ? r : p;
}

__global__ __launch_bounds__(SHPL_BLOCK) void k_hist(CsrIn c, int32_t *cnt) {
    const int64_t n = live_nnz(c);
    for (int64_t e = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; e < n; e += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int32_t key = key_of(c, e);
        if (key >= 0) atomicAdd(&cnt[key], 1);
    }
}

// ---- exclusive scan of cnt[0..n) into rowptr[0..n], rowptr[n] = total
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SHPL_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ void load_items(const int32_t *a, int64_t n, int64_t first, int32_t (&v)[SCAN_ITEMS]) {
    if (first + SCAN_ITEMS <= n) {
        const int4 *p = reinterpret_cast<const int4 *>(a + first);
#pragma unroll
        for (int q = 0; q < SCAN_ITEMS / 4; ++q) {
            const int4 t = p[q];
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j) v[j] = (first + j < n) ? a[first + j] : 0;
    }
}

__global__ __launch_bounds__(SHPL_BLOCK) void k_scan_tiles(const int32_t *cnt, int64_t n, int64_t *tile_sum) {
    int32_t v[SCAN_ITEMS];
    load_items(cnt, n, (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS, v);
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) s += v[j];
    __shared__ int64_t lds[SHPL_BLOCK / 64 + 1];
    int64_t tot;
    block_excl_scan(s, lds, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SHPL_BLOCK) void k_scan_tile_sums(int64_t *tile_sum, int64_t n_tiles, int32_t *rowptr,
                                                               int64_t n) {
    __shared__ int64_t lds[SHPL_BLOCK / 64 + 1];
    int64_t carry = 0;
    for (int64_t base = 0; base < n_tiles; base += SHPL_BLOCK) {
        const int64_t j = base + threadIdx.x;
        const int64_t v = j < n_tiles ? tile_sum[j] : 0;
        int64_t tot;
        const int64_t ex = block_excl_scan(v, lds, &tot);
        if (j < n_tiles) tile_sum[j] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) rowptr[n] = (int32_t)carry;
}

// Also writes the occupancy bitmap: thread pairs own one 32-bit word.
__global__ __launch_bounds__(SHPL_BLOCK) void k_scan_apply(const int32_t *cnt, int64_t n, const int64_t *tile_off,
                                                           int32_t *rowptr, uint32_t *occ) {
    static_assert(SCAN_ITEMS == 16, "two threads per bitmap word");
    int32_t v[SCAN_ITEMS];
    const int64_t first = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    load_items(cnt, n, first, v);
    int64_t s = 0;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        s += v[j];
        bits |= (v[j] > 0 ? 1u : 0u) << j;
    }
    const uint32_t hi = __shfl_down(bits, 1, 64);
    if ((threadIdx.x & 1) == 0 && first < n) occ[first >> 5] = bits | (hi << 16);
    __shared__ int64_t lds[SHPL_BLOCK / 64 + 1];
    int64_t tot;
    int64_t run = block_excl_scan(s, lds, &tot) + tile_off[blockIdx.x];
    if (first + SCAN_ITEMS <= n) {
        int32_t o[SCAN_ITEMS];
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j) {
            o[j] = (int32_t)run;
            run += v[j];
        }
        int4 *p = reinterpret_cast<int4 *>(rowptr + first);
#pragma unroll
        for (int q = 0; q < SCAN_ITEMS / 4; ++q) p[q] = make_int4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    } else {
        for (int j = 0; j < SCAN_ITEMS; ++j) {
            if (first + j < n) rowptr[first + j] = (int32_t)run;
            run += v[j];
        }
    }
}

// Placement: slots of a destination are handed out downwards from its end;
// cnt returns to zero.
__global__ __launch_bounds__(SHPL_BLOCK) void k_place(CsrIn c, const int32_t *rowptr, int32_t *cnt, int32_t *tmp) {
    const int64_t n = live_nnz(c);
    for (int64_t e = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; e < n; e += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int32_t key = key_of(c, e);
        if (key < 0) continue;
        const int32_t slot = rowptr[key] + atomicSub(&cnt[key], 1) - 1;
        tmp[slot] = (int32_t)e;
    }
}

// Sort key of entry e inside its destination, TF-CPU order (see shpl_order).
__device__ __forceinline__ uint64_t order_key(const CsrIn &c, int32_t e) {
    switch (c.order) {
        case SHPL_ORDER_COL_ROW:
            return ((uint64_t)(uint32_t)col_of(c, e) << 32) | (uint32_t)c.cell[e];
        case SHPL_ORDER_COL_ENTRY:
            return (uint64_t)(uint32_t)col_of(c, e);
        default:
            return 0;
    }
}

__global__ __launch_bounds__(SHPL_BLOCK) void k_fix(CsrIn c, const int32_t *rowptr, int64_t n_keys, const int32_t *tmp,
                                                    int32_t *ent_dst, int32_t *ent_src, float *ent_val,
                                                    int32_t *ent_col) {
    const int64_t n = rowptr[n_keys];
    for (int64_t s = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; s < n; s += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int32_t e = tmp[s];
        const int32_t key = key_of(c, e);
        const int32_t a = rowptr[key], b = rowptr[key + 1];
        int32_t rank = 0;
        if (b - a > 1) {
            const uint64_t ke = order_key(c, e);
            for (int32_t t = a; t < b; ++t) {
                const int32_t o = tmp[t];
                const uint64_t ko = order_key(c, o);
                rank += (ko < ke || (ko == ke && o < e)) ? 1 : 0;
            }
        }
        const int32_t d = a + rank;
        const int32_t k = col_of(c, e);
        ent_dst[d] = key;
        ent_src[d] = c.direction == SHPL_BY_CELL ? c.pix[k] : c.cell[e];
        ent_val[d] = c.val[e];
        if (ent_col) ent_col[d] = k;
    }
}

struct CsrWs {
    int32_t *cnt;
    int64_t *tile;
    int32_t *tmp;
    size_t bytes;
};

CsrWs carve_csr(int64_t n_keys, int64_t nnz_cap, void *base) {
    CsrWs w;
    char *b = (char *)base;
    size_t o = 0;
    w.cnt = (int32_t *)(b + o);
    o = align_up(o + sizeof(int32_t) * (size_t)(n_keys + 1), 256);
    const int64_t n_tiles = (n_keys + SCAN_TILE - 1) / SCAN_TILE + 1;
    w.tile = (int64_t *)(b + o);
    o = align_up(o + sizeof(int64_t) * (size_t)n_tiles, 256);
    w.tmp = (int32_t *)(b + o);
    o = align_up(o + sizeof(int32_t) * (size_t)(nnz_cap > 0 ? nnz_cap : 1), 256);
    w.bytes = o;
    return w;
}

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_pack_map(int64_t nnz, const int64_t *d_mij, const float *d_values, int64_t n_values,
                             int64_t n_rows, int64_t n_cols, const void *d_idx, int idx_itype, int64_t img_b,
                             int64_t img_h, int64_t img_w, int64_t row_base, int64_t col_base, int64_t pix_base,
                             int32_t *d_cell, int32_t *d_col, float *d_val, int32_t *d_pix, uint32_t *d_err,
                             void *stream) {
    if (nnz < 0 || n_cols < 0 || n_values < 0) return SHPL_ERR_ARG;
    if ((nnz > 0 && (!d_mij || !d_cell || !d_col || !d_val)) || (n_values > 0 && !d_values) ||
        (n_cols > 0 && (!d_idx || !d_pix)))
        return SHPL_ERR_ARG;
    if (row_base + n_rows >= 2147483647LL || col_base + n_cols >= 2147483647LL ||
        pix_base + img_b * img_h * img_w >= 2147483647LL)
        return SHPL_ERR_BAD_SHAPE;
    const int64_t n = nnz > n_cols ? nnz : n_cols;
    const int grid = grid_for(n > 0 ? n : 1, SHPL_BLOCK, 4096);
    hipStream_t s = (hipStream_t)stream;
    if (idx_itype == SHPL_I32)
        hipLaunchKernelGGL(k_pack<int32_t>, dim3(grid), dim3(SHPL_BLOCK), 0, s, nnz, d_mij, d_values, n_values,
                           n_rows, n_cols, (const int32_t *)d_idx, img_b, img_h, img_w, row_base, col_base,
                           pix_base, d_cell, d_col, d_val, d_pix, d_err);
    else if (idx_itype == SHPL_I64)
        hipLaunchKernelGGL(k_pack<int64_t>, dim3(grid), dim3(SHPL_BLOCK), 0, s, nnz, d_mij, d_values, n_values,
                           n_rows, n_cols, (const int64_t *)d_idx, img_b, img_h, img_w, row_base, col_base,
                           pix_base, d_cell, d_col, d_val, d_pix, d_err);
    else
        return SHPL_ERR_ARG;
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

extern "C" int shpl_csr_workspace_bytes(int64_t n_keys, int64_t nnz_cap, size_t *bytes) {
    if (!bytes || n_keys < 0 || nnz_cap < 0) return SHPL_ERR_ARG;
    *bytes = carve_csr(n_keys, nnz_cap, nullptr).bytes;
    return SHPL_OK;
}

extern "C" int shpl_build_csr(int direction, int order, const int64_t *d_nnz, const int32_t *d_cell,
                              const int32_t *d_col, const float *d_val, const int32_t *d_pix, const shpl_csr *csr,
                              void *d_ws, size_t ws_bytes, void *stream) {
    if (!csr) return SHPL_ERR_ARG;
    if (direction != SHPL_BY_CELL && direction != SHPL_BY_PIXEL) return SHPL_ERR_ARG;
    if (order < SHPL_ORDER_ENTRY || order > SHPL_ORDER_COL_ENTRY) return SHPL_ERR_ARG;
    const int64_t n_keys = csr->n_keys, nnz_cap = csr->nnz_cap;
    if (n_keys < 0 || nnz_cap < 0 || n_keys >= 2147483647LL || nnz_cap >= 2147483647LL) return SHPL_ERR_BAD_SHAPE;
    if (!csr->rowptr || !csr->occ || !d_ws) return SHPL_ERR_ARG;
    if (nnz_cap > 0 && (!d_cell || !d_val || !d_pix || !csr->ent_dst || !csr->ent_src || !csr->ent_val))
        return SHPL_ERR_ARG;
    if (direction == SHPL_BY_PIXEL && nnz_cap > 0 && !csr->ent_col) return SHPL_ERR_ARG;
    if (((uintptr_t)csr->rowptr & 15u) != 0) return SHPL_ERR_BAD_SHAPE;  // int4 stores in the scan
    CsrWs w = carve_csr(n_keys, nnz_cap, d_ws);
    if (w.bytes > ws_bytes) return SHPL_ERR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    CsrIn c{direction, order, nnz_cap, d_nnz, d_cell, d_col, d_pix, d_val};
    SHPL_HIP_CHECK(hipMemsetAsync(w.cnt, 0, sizeof(int32_t) * (size_t)(n_keys + 1), s));
    const int ge = grid_for(nnz_cap > 0 ? nnz_cap : 1, SHPL_BLOCK, 8192);
    if (nnz_cap > 0) {
        hipLaunchKernelGGL(k_hist, dim3(ge), dim3(SHPL_BLOCK), 0, s, c, w.cnt);
        SHPL_LAUNCH_CHECK();
    }
    const int64_t n_tiles = (n_keys + SCAN_TILE - 1) / SCAN_TILE;
    if (n_tiles > 0) {
        hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)n_tiles), dim3(SHPL_BLOCK), 0, s, w.cnt, n_keys, w.tile);
        SHPL_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_scan_tile_sums, dim3(1), dim3(SHPL_BLOCK), 0, s, w.tile, n_tiles, csr->rowptr, n_keys);
    SHPL_LAUNCH_CHECK();
    if (n_tiles > 0) {
        hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)n_tiles), dim3(SHPL_BLOCK), 0, s, w.cnt, n_keys, w.tile,
                           csr->rowptr, csr->occ);
        SHPL_LAUNCH_CHECK();
    }
    if (nnz_cap > 0) {
        hipLaunchKernelGGL(k_place, dim3(ge), dim3(SHPL_BLOCK), 0, s, c, csr->rowptr, w.cnt, w.tmp);
        SHPL_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_fix, dim3(ge), dim3(SHPL_BLOCK), 0, s, c, csr->rowptr, n_keys, w.tmp, csr->ent_dst,
                           csr->ent_src, csr->ent_val, csr->ent_col);
        SHPL_LAUNCH_CHECK();
    }
    return SHPL_OK;
}
