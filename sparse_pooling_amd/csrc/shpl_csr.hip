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
// CSR build: one workgroup per frame, one launch (k_csr_frame): an LDS
// histogram over destination tiles, a scan, an LDS-atomic placement and a
// rank fix-up that restores TF's order inside each tile. Nothing is sized by
// the number of destinations (no per-cell counters in HBM), and tiles hold
// a few entries each, so the quadratic rank costs less than a sort pass.
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
constexpr int CSR_BLOCK = 1024;           // one workgroup per frame
constexpr int CSR_TILES = 16384;          // LDS tile counters (64 KiB)
#ifndef SHPL_CSR_PROBE
#define SHPL_CSR_PROBE 0  // timing probes of k_csr_frame (wrong results): 1 return after the scan, 2 after placement
#endif

struct CsrIn {
    int direction, order, n_frames;
    const int64_t *frame_off, *frame_nnz;
    int64_t keys_per_frame;
    int log_tile;  // destinations per tile = 1 << log_tile
    const int32_t *cell, *col, *pix;
    const float *val;
};

__device__ __forceinline__ int32_t col_of(const CsrIn &c, int64_t e) { return c.col ? c.col[e] : (int32_t)e; }

// Destination of entry e, or -1 if the entry is invalid (flagged upstream).
__device__ __forceinline__ int32_t key_of(const CsrIn &c, int64_t e) {
    const int32_t r = c.cell[e];
    const int32_t k = col_of(c, e);
    if (r < 0 || k < 0) return -1;
    const int32_t p = c.pix[k];
    if (p < 0) return -1;
    return c.direction == SHPL_BY_CELL ? r : p;
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

constexpr int CSR_BATCH = 8;     // entries per thread whose loads are in flight together
constexpr int CSR_WIN = 10240;   // packed words staged in LDS for the rank fix-up (80 KiB)

// Destinations of entries first + u*CSR_BLOCK (u < U), -1 for invalid or past e1.
// All loads of the batch are issued before any is used.
template <bool HAS_COL, int U>
__device__ __forceinline__ void keys_batch(const CsrIn &c, int64_t first, int64_t e1, int32_t (&key)[U]) {
    int32_t r[U], k[U], p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t e = first + (int64_t)u * CSR_BLOCK;
        const bool ok = e < e1;
        r[u] = ok ? c.cell[e] : -1;
        k[u] = ok ? (HAS_COL ? c.col[e] : (int32_t)e) : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) p[u] = k[u] >= 0 ? c.pix[k[u]] : -1;
#pragma unroll
    for (int u = 0; u < U; ++u)
        key[u] = (r[u] < 0 || k[u] < 0 || p[u] < 0) ? -1 : (c.direction == SHPL_BY_CELL ? r[u] : p[u]);
}

// One frame per workgroup:
//  1. LDS histogram of the frame's entries over destination tiles
//  2. exclusive scan of the tile counts (in place)
//  3. placement into tile segments (LDS atomics: arbitrary order inside a tile)
//  4. rank fix-up: each entry counts the tile entries that precede it in
//     (destination, TF order, entry) and moves to that rank -> stable, sorted.
//     With identity columns (or ORDER_ENTRY) the packed word alone orders a
//     tile; the words are then staged in LDS windows so that the quadratic
//     count reads LDS, not HBM.
// Unused capacity of every frame, [off[f] + nnz[f], off[f+1]), and the slots
// past the last frame: empty (dst = -1), skipped by the pulls. Done by extra
// workgroups of the CSR launch (blockIdx.x >= n_frames), each clearing a span
// of HOLE_SPAN slots beside the sorting workgroups; they need only the index
// builder's frame counts, not the sort.
constexpr int HOLE_SPAN = 16384;

__device__ void clear_unused(const CsrIn &c, int64_t nnz_cap, int32_t *ent_dst, int span) {
    __shared__ int f0s;
    const int64_t b0 = (int64_t)span * HOLE_SPAN;
    if (threadIdx.x == 0) {
        int lo = 0, hi = c.n_frames;  // last f with frame_off[f] <= b0 (n_frames: past the last frame)
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (c.frame_off[mid] <= b0)
                lo = mid;
            else
                hi = mid - 1;
        }
        f0s = lo;
    }
    __syncthreads();
    const int64_t b1 = b0 + HOLE_SPAN < nnz_cap ? b0 + HOLE_SPAN : nnz_cap;
    int f = f0s;
    int64_t fend = 0, live = 0;
    auto bounds = [&]() {
        if (f < c.n_frames) {
            fend = c.frame_off[f + 1];
            const int64_t l = c.frame_off[f] + c.frame_nnz[f];
            live = l < fend ? l : fend;
        }
    };
    bounds();
    for (int64_t d = b0 + threadIdx.x; d < b1; d += CSR_BLOCK) {
        while (f < c.n_frames && d >= fend) {
            ++f;
            bounds();
        }
        if (f >= c.n_frames || d >= live) ent_dst[d] = -1;
    }
}

// Exclusive scan of the TILES LDS tile counters in place (1024 threads):
// cnt[t] = start of tile t.
template <int TILES>
__device__ __forceinline__ void tile_scan(int32_t *cnt, int32_t *wsum) {
    constexpr int CSR_PER_THREAD = TILES / CSR_BLOCK;
    int32_t v[CSR_PER_THREAD];
    int32_t sum = 0;
#pragma unroll
    for (int q = 0; q < CSR_PER_THREAD; ++q) {
        v[q] = cnt[threadIdx.x * CSR_PER_THREAD + q];
        sum += v[q];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int32_t run = x - sum;
    for (int w = 0; w < wid; ++w) run += wsum[w];
#pragma unroll
    for (int q = 0; q < CSR_PER_THREAD; ++q) {
        cnt[threadIdx.x * CSR_PER_THREAD + q] = run;
        run += v[q];
    }
}

// Rank fix-up + emission. words[0, n_valid) hold packed (destination << 32 |
// entry) words grouped by destination tile (cnt[t] = end of tile t, tiles of
// 2^log_tile destinations from kbase); each entry counts the tile entries
// that precede it in (destination, TF order, entry), which makes the order
// stable and sorted, and is written to out_base + its rank with its source
// row, value and column. With identity columns (or ORDER_ENTRY) the packed
// word alone orders a tile and the words are staged in LDS windows, so the
// quadratic count reads LDS, not HBM.
template <bool HAS_COL, int CSR_WIN>
__device__ void emit_sorted(const CsrIn &c, const uint64_t *words, int32_t n_valid, int64_t out_base, int64_t kbase,
                            int log_tile, const int32_t *cnt, uint64_t *win, int32_t *ent_dst, int32_t *ent_src,
                            float *ent_val, int32_t *ent_col) {
    // With identity columns every TF order collapses to entry order.
    const bool entry_order = c.order == SHPL_ORDER_ENTRY || !HAS_COL;
    if (entry_order) {
        for (int32_t w0 = 0; w0 < n_valid; w0 += CSR_WIN) {
            const int32_t w1 = w0 + CSR_WIN < n_valid ? w0 + CSR_WIN : n_valid;
            for (int32_t s = w0 + threadIdx.x; s < w1; s += CSR_BLOCK) win[s - w0] = words[s];
            __syncthreads();
            for (int32_t s0 = w0 + threadIdx.x; s0 < w1; s0 += CSR_BLOCK * CSR_BATCH) {
                int32_t d[CSR_BATCH], ee[CSR_BATCH], kk[CSR_BATCH], key[CSR_BATCH];
#pragma unroll
                for (int u = 0; u < CSR_BATCH; ++u) {
                    const int32_t s = s0 + u * CSR_BLOCK;
                    d[u] = -1;
                    if (s >= w1) continue;
                    const uint64_t me = win[s - w0];
                    key[u] = (int32_t)(me >> 32);
                    ee[u] = (int32_t)(uint32_t)me;
                    const int t = (int)((key[u] - kbase) >> log_tile);
                    const int32_t a = t ? cnt[t - 1] : 0, b = cnt[t];
                    int32_t rank = 0;
                    if (b - a > 1) {
                        if (a >= w0 && b <= w1) {
                            for (int32_t x = a; x < b; ++x) rank += win[x - w0] < me ? 1 : 0;
                        } else {  // tile straddles the window edge
                            for (int32_t x = a; x < b; ++x) rank += words[x] < me ? 1 : 0;
                        }
                    }
                    d[u] = a + rank;
                }
#pragma unroll
                for (int u = 0; u < CSR_BATCH; ++u) kk[u] = d[u] >= 0 ? (HAS_COL ? c.col[ee[u]] : ee[u]) : 0;
                int32_t src[CSR_BATCH];
                float val[CSR_BATCH];
#pragma unroll
                for (int u = 0; u < CSR_BATCH; ++u) {
                    if (d[u] < 0) continue;
                    src[u] = c.direction == SHPL_BY_CELL ? c.pix[kk[u]] : c.cell[ee[u]];
                    val[u] = c.val[ee[u]];
                }
#pragma unroll
                for (int u = 0; u < CSR_BATCH; ++u) {
                    if (d[u] < 0) continue;
                    const int64_t o = out_base + d[u];
                    ent_dst[o] = key[u];
                    ent_src[o] = src[u];
                    ent_val[o] = val[u];
                    if (ent_col) ent_col[o] = kk[u];
                }
            }
            __syncthreads();  // the next window overwrites win
        }
    } else {
        for (int32_t s = threadIdx.x; s < n_valid; s += CSR_BLOCK) {
            const uint64_t me = words[s];
            const int32_t key = (int32_t)(me >> 32);
            const int32_t e = (int32_t)(uint32_t)me;
            const int t = (int)((key - kbase) >> log_tile);
            const int32_t a = t ? cnt[t - 1] : 0, b = cnt[t];
            int32_t rank = 0;
            const uint64_t ke = order_key(c, e);
            for (int32_t u = a; u < b; ++u) {
                const uint64_t ot = words[u];
                const int32_t ko = (int32_t)(ot >> 32), o = (int32_t)(uint32_t)ot;
                bool before = ko < key;
                if (ko == key && o != e) {
                    const uint64_t oo = order_key(c, o);
                    before = oo < ke || (oo == ke && o < e);
                }
                rank += before ? 1 : 0;
            }
            const int64_t d = out_base + a + rank;
            const int32_t k = col_of(c, e);
            ent_dst[d] = key;
            ent_src[d] = c.direction == SHPL_BY_CELL ? c.pix[k] : c.cell[e];
            ent_val[d] = c.val[e];
            if (ent_col) ent_col[d] = k;
        }
    }
}

// Live entry range [e0, e1) and capacity end of frame f.
__device__ __forceinline__ void frame_range(const CsrIn &c, int f, int64_t &e0, int64_t &e1, int64_t &cap_end) {
    e0 = c.frame_off[f];
    cap_end = c.frame_off[f + 1];
    e1 = cap_end;
    if (c.frame_nnz) {
        const int64_t n = c.frame_nnz[f];
        e1 = e0 + n < cap_end ? e0 + n : cap_end;
    }
}

// Slots of invalid entries (flagged upstream) become empty; the unused
// capacity past the frame's live entries is cleared by the launch's extra
// workgroups (frame_nnz given), or here (no frame_nnz: the frame's capacity
// is all live, so only invalid entries leave slots).
__device__ __forceinline__ void clear_holes(const CsrIn &c, int f, int64_t from, int64_t e1, int64_t cap_end,
                                            int64_t nnz_cap, int32_t *ent_dst) {
    const int64_t hole_end = c.frame_nnz ? e1 : (f == c.n_frames - 1 ? nnz_cap : cap_end);
    for (int64_t d = from + threadIdx.x; d < hole_end; d += CSR_BLOCK) ent_dst[d] = -1;
}

template <bool HAS_COL>
__global__ __launch_bounds__(CSR_BLOCK) void k_csr_frame(CsrIn c, uint64_t *tmp, int64_t nnz_cap, int32_t *ent_dst,
                                                         int32_t *ent_src, float *ent_val, int32_t *ent_col) {
    __shared__ int32_t cnt[CSR_TILES];
    __shared__ int32_t wsum[CSR_BLOCK / 64];
    __shared__ uint64_t win[CSR_WIN];
    if ((int)blockIdx.x >= c.n_frames) {
        clear_unused(c, nnz_cap, ent_dst, (int)blockIdx.x - c.n_frames);
        return;
    }
    const int f = blockIdx.x;
    int64_t e0, e1, cap_end;
    frame_range(c, f, e0, e1, cap_end);
    const int64_t kbase = (int64_t)f * c.keys_per_frame;
    const int n_tiles = (int)(((c.keys_per_frame - 1) >> c.log_tile) + 1);
    for (int t = threadIdx.x; t < CSR_TILES; t += CSR_BLOCK) cnt[t] = 0;
    __syncthreads();
    // 1. histogram
    for (int64_t b = e0 + threadIdx.x; b < e1; b += (int64_t)CSR_BLOCK * CSR_BATCH) {
        int32_t key[CSR_BATCH];
        keys_batch<HAS_COL>(c, b, e1, key);
#pragma unroll
        for (int u = 0; u < CSR_BATCH; ++u) {
            const int64_t k = (int64_t)key[u] - kbase;
            if (key[u] >= 0 && k >= 0 && k < c.keys_per_frame) atomicAdd(&cnt[k >> c.log_tile], 1);
        }
    }
    __syncthreads();
    // 2. exclusive scan
    tile_scan<CSR_TILES>(cnt, wsum);
    __syncthreads();
    if (SHPL_CSR_PROBE == 1) return;
    // 3. placement of (destination << 32 | entry): cnt[t] advances from start(t) to end(t) = start(t+1)
    for (int64_t b = e0 + threadIdx.x; b < e1; b += (int64_t)CSR_BLOCK * CSR_BATCH) {
        int32_t key[CSR_BATCH];
        keys_batch<HAS_COL>(c, b, e1, key);
#pragma unroll
        for (int u = 0; u < CSR_BATCH; ++u) {
            const int64_t k = (int64_t)key[u] - kbase;
            const int64_t e = b + (int64_t)u * CSR_BLOCK;
            if (key[u] >= 0 && k >= 0 && k < c.keys_per_frame)
                tmp[e0 + atomicAdd(&cnt[k >> c.log_tile], 1)] = ((uint64_t)(uint32_t)key[u] << 32) | (uint32_t)e;
        }
    }
    block_publish();  // tmp was written by other waves of this workgroup through memory
    if (SHPL_CSR_PROBE == 2) return;
    const int32_t n_valid = cnt[n_tiles - 1];
    // 4. rank fix-up
    emit_sorted<HAS_COL, CSR_WIN>(c, tmp + e0, n_valid, e0, kbase, c.log_tile, cnt, win, ent_dst, ent_src, ent_val, ent_col);
    clear_holes(c, f, e0 + n_valid, e1, cap_end, nnz_cap, ent_dst);
}

// ---------------------------------------------------------------- segmented CSR
// For batches too small to fill the chip with one workgroup per frame (config
// 3: 4 frames), each frame's destinations are cut into S segments holding
// about the same number of entries, sorted by S workgroups:
//   k_csr_count   every entry's destination -> kbuf; a histogram of the
//                 frame's destinations over n_bins bins of 2^log_bin
//   k_csr_bucket  bins -> balanced segments (bin b goes to segment
//                 excl(b) * S / total); entries scattered to their segment's
//                 bucket (any order)
//   k_csr_segment one workgroup per (frame, segment): the frame kernel's tile
//                 histogram / placement / rank fix-up over its bucket
// Segments are contiguous destination ranges, so the result is identical to
// k_csr_frame's. Balancing matters: image points crowd a few rows around the
// horizon, and equal destination ranges left one segment with most of a
// frame (measured: pixel CSR 50 us with equal ranges at config 3).
constexpr int SEG_BLOCK = 256;
constexpr int SEG_MAX = 1024;   // bins per frame (LDS histogram of count / bucket / segment)
constexpr int SEG_BATCH = 4;    // entries per thread in flight
constexpr int SEG_TILES = 4096; // tile counters of a segment workgroup (16 KiB)
constexpr int SEG_WIN = 4096;   // rank fix-up window of a segment workgroup (32 KiB): two per CU

struct SegIn {
    int S;              // segments per frame
    int n_bins;         // destination bins per frame (<= SEG_MAX)
    int log_bin;        // destinations per bin = 1 << log_bin
    int32_t *hist;      // [n_frames * n_bins] entries per bin
    int32_t *cur;       // [n_frames * S] bucket fill cursors
    int32_t *kbuf;      // [nnz_cap] destination of each entry slot (-1: invalid)
    uint64_t *bucket;   // [nnz_cap] words grouped by segment
    uint64_t *sorted;   // [nnz_cap] words grouped by tile inside a segment
};

// Zeroes the bin and cursor counters (a kernel node: cheaper than a memset
// node inside the bench's captured graph).
__global__ __launch_bounds__(SEG_BLOCK) void k_zero32(int32_t *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * SEG_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * SEG_BLOCK) p[i] = 0;
}

// key_range of a sorted entry list that is not the range builder's (shpl_build_csr_path(SHPL_CSR_FRAME) with
// key_range): after k_zero32 over key_range (every destination's run empty), each slot that starts a run
// writes its destination's first entry and each slot that ends one its end.
__global__ __launch_bounds__(SEG_BLOCK) void k_key_range(const int32_t *ent_dst, int64_t nnz_cap, int32_t *key_range) {
    for (int64_t s = (int64_t)blockIdx.x * SEG_BLOCK + threadIdx.x; s < nnz_cap; s += (int64_t)gridDim.x * SEG_BLOCK) {
        const int32_t d = ent_dst[s];
        if (d < 0) continue;
        if (s == 0 || ent_dst[s - 1] != d) key_range[2 * (int64_t)d] = (int32_t)s;
        if (s + 1 == nnz_cap || ent_dst[s + 1] != d) key_range[2 * (int64_t)d + 1] = (int32_t)(s + 1);
    }
}

template <bool HAS_COL>
__global__ __launch_bounds__(SEG_BLOCK) void k_csr_count(CsrIn c, SegIn g) {
    __shared__ int32_t h[SEG_MAX];
    const int f = blockIdx.y;
    int64_t e0, e1, cap_end;
    frame_range(c, f, e0, e1, cap_end);
    const int64_t kbase = (int64_t)f * c.keys_per_frame;
    for (int b = threadIdx.x; b < g.n_bins; b += SEG_BLOCK) h[b] = 0;
    __syncthreads();
    const int64_t step = (int64_t)gridDim.x * SEG_BLOCK;
    for (int64_t b = e0 + (int64_t)blockIdx.x * SEG_BLOCK + threadIdx.x; b < e1; b += step * SEG_BATCH) {
        int32_t r[SEG_BATCH], k[SEG_BATCH], p[SEG_BATCH];
#pragma unroll
        for (int u = 0; u < SEG_BATCH; ++u) {
            const int64_t e = b + u * step;
            const bool ok = e < e1;
            r[u] = ok ? c.cell[e] : -1;
            k[u] = ok ? (HAS_COL ? c.col[e] : (int32_t)e) : -1;
        }
#pragma unroll
        for (int u = 0; u < SEG_BATCH; ++u) p[u] = k[u] >= 0 ? c.pix[k[u]] : -1;
#pragma unroll
        for (int u = 0; u < SEG_BATCH; ++u) {
            const int64_t e = b + u * step;
            if (e >= e1) continue;
            int32_t key = (r[u] < 0 || k[u] < 0 || p[u] < 0) ? -1 : (c.direction == SHPL_BY_CELL ? r[u] : p[u]);
            const int64_t kk = (int64_t)key - kbase;
            if (key >= 0 && (kk < 0 || kk >= c.keys_per_frame)) key = -1;  // outside the frame: left out
            g.kbuf[e] = key;
            if (key >= 0) atomicAdd(&h[(int)(kk >> g.log_bin)], 1);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < g.n_bins; b += SEG_BLOCK)
        if (h[b]) atomicAdd(&g.hist[(int64_t)f * g.n_bins + b], h[b]);
}

// Balanced segments of frame f from its bin histogram (BLOCK threads, every
// thread calls): seg_of[b] for each bin; per segment its first entry offset
// in the frame (seg_start), entry count (seg_n), first bin (seg_lo) and bin
// count (seg_nb). Returns the frame's entry total.
template <int BLOCK>
__device__ int32_t seg_map(const SegIn &g, int f, int32_t *seg_of, int32_t *seg_start, int32_t *seg_n,
                           int32_t *seg_lo, int32_t *seg_nb, int32_t *wsum) {
    constexpr int PER = SEG_MAX / BLOCK;
    const int32_t *hist = g.hist + (int64_t)f * g.n_bins;
    int32_t v[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int b = threadIdx.x * PER + q;
        v[q] = b < g.n_bins ? hist[b] : 0;
        sum += v[q];
    }
    for (int s = threadIdx.x; s < g.S; s += BLOCK) {
        seg_n[s] = 0;
        seg_nb[s] = 0;
        seg_start[s] = 0;
        seg_lo[s] = 0;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int32_t run = x - sum, total = 0;
    for (int w = 0; w < BLOCK / 64; ++w) {
        if (w < wid) run += wsum[w];
        total += wsum[w];
    }
    const int64_t S = g.S;
    auto seg_at = [&](int32_t excl) { return total ? (int)min(S - 1, (int64_t)excl * S / total) : 0; };
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int b = threadIdx.x * PER + q;
        if (b < g.n_bins) {
            const int sg = seg_at(run);
            seg_of[b] = sg;
            const bool first = b == 0 || seg_at(run - (q ? v[q - 1] : hist[b - 1])) != sg;
            if (first) {
                seg_start[sg] = run;
                seg_lo[sg] = b;
            }
            atomicAdd(&seg_n[sg], v[q]);
            atomicAdd(&seg_nb[sg], 1);
        }
        run += v[q];
    }
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(SEG_BLOCK) void k_csr_bucket(CsrIn c, SegIn g) {
    __shared__ int32_t seg_of[SEG_MAX], seg_start[SEG_MAX], seg_n[SEG_MAX], seg_lo[SEG_MAX], seg_nb[SEG_MAX];
    __shared__ int32_t h[SEG_MAX], base[SEG_MAX];
    __shared__ int32_t wsum[SEG_BLOCK / 64];
    const int f = blockIdx.y;
    int64_t e0, e1, cap_end;
    frame_range(c, f, e0, e1, cap_end);
    const int64_t kbase = (int64_t)f * c.keys_per_frame;
    seg_map<SEG_BLOCK>(g, f, seg_of, seg_start, seg_n, seg_lo, seg_nb, wsum);
    const int64_t step = (int64_t)gridDim.x * SEG_BLOCK;
    // uniform trip count: every thread takes part in every round's barriers
    for (int64_t b0 = e0 + (int64_t)blockIdx.x * SEG_BLOCK; b0 < e1; b0 += step) {
        for (int s = threadIdx.x; s < g.S; s += SEG_BLOCK) h[s] = 0;
        __syncthreads();
        const int64_t e = b0 + threadIdx.x;
        const int32_t key = e < e1 ? g.kbuf[e] : -1;
        int seg = 0, loc = 0;
        if (key >= 0) {
            seg = seg_of[(int)((key - kbase) >> g.log_bin)];
            loc = atomicAdd(&h[seg], 1);
        }
        __syncthreads();
        for (int s = threadIdx.x; s < g.S; s += SEG_BLOCK)
            if (h[s]) base[s] = atomicAdd(&g.cur[(int64_t)f * g.S + s], h[s]);
        __syncthreads();
        if (key >= 0)
            g.bucket[e0 + seg_start[seg] + base[seg] + loc] = ((uint64_t)(uint32_t)key << 32) | (uint32_t)e;
        __syncthreads();
    }
}

template <bool HAS_COL>
__global__ __launch_bounds__(CSR_BLOCK) void k_csr_segment(CsrIn c, SegIn g, int64_t nnz_cap, int32_t *ent_dst,
                                                           int32_t *ent_src, float *ent_val, int32_t *ent_col) {
    __shared__ int32_t cnt[SEG_TILES];
    __shared__ int32_t wsum[CSR_BLOCK / 64];
    __shared__ uint64_t win[SEG_WIN];
    __shared__ int32_t seg_of[SEG_MAX], seg_start[SEG_MAX], seg_n[SEG_MAX], seg_lo[SEG_MAX], seg_nb[SEG_MAX];
    if ((int)blockIdx.y >= c.n_frames) {
        clear_unused(c, nnz_cap, ent_dst, (int)blockIdx.x + (int)(blockIdx.y - c.n_frames) * (int)gridDim.x);
        return;
    }
    const int f = blockIdx.y, s = blockIdx.x;
    int64_t e0, e1, cap_end;
    frame_range(c, f, e0, e1, cap_end);
    const int32_t total = seg_map<CSR_BLOCK>(g, f, seg_of, seg_start, seg_n, seg_lo, seg_nb, wsum);
    if (s == g.S - 1) clear_holes(c, f, e0 + total, e1, cap_end, nnz_cap, ent_dst);
    const int32_t n = seg_n[s];
    if (n == 0) return;  // uniform
    const int64_t b0 = e0 + seg_start[s];
    const int64_t kbase = (int64_t)f * c.keys_per_frame + ((int64_t)seg_lo[s] << g.log_bin);
    const int64_t nkeys = (int64_t)seg_nb[s] << g.log_bin;
    int log_tile = 0;
    while (((nkeys - 1) >> log_tile) + 1 > SEG_TILES) ++log_tile;
    for (int t = threadIdx.x; t < SEG_TILES; t += CSR_BLOCK) cnt[t] = 0;
    __syncthreads();
    const uint64_t *in = g.bucket + b0;
    for (int32_t i = threadIdx.x; i < n; i += CSR_BLOCK)
        atomicAdd(&cnt[(int)((((int64_t)(in[i] >> 32)) - kbase) >> log_tile)], 1);
    __syncthreads();
    tile_scan<SEG_TILES>(cnt, wsum);
    __syncthreads();
    for (int32_t i = threadIdx.x; i < n; i += CSR_BLOCK) {
        const uint64_t w = in[i];
        g.sorted[b0 + atomicAdd(&cnt[(int)((((int64_t)(w >> 32)) - kbase) >> log_tile)], 1)] = w;
    }
    block_publish();  // sorted was written by other waves of this workgroup through memory
    emit_sorted<HAS_COL, SEG_WIN>(c, g.sorted + b0, n, b0, kbase, log_tile, cnt, win, ent_dst, ent_src, ent_val,
                                  ent_col);
}

// ---------------------------------------------------------------- range CSR
// One launch, no workgroup waiting for another: one workgroup per (frame,
// range of RANGE_KEYS destinations). Small batches of frames with few
// destinations (config 3: 4 frames of 8,800 cells / 6,750 pixels) sort in
// one launch instead of four, and the per-destination (first, end) ranges the
// row-keyed pull reads (csr->key_range) come out of the same pass:
//   1. every workgroup reads all of its frame's entries once (L2-resident,
//      8-12 B each, RANGE_BATCH in flight per thread): the entries of its
//      range go to an LDS list as 32-bit words (local destination << 24 |
//      entry offset in the frame; wave-aggregated slots), with LDS counts per
//      destination; the valid entries below its range are counted (its
//      output offset inside the frame);
//   2. exclusive scan of the counts: each destination's start;
//   3. the list placed by destination (LDS atomics: any order inside one);
//   4. each word's rank among its destination's words in (TF order, entry)
//      order -> its sorted slot; emitted with source row, value and column;
//   5. key_range of its destinations; the frame's last range clears the
//      frame's unused capacity (and, for the last frame, the slots after it).
// A range holding more than RANGE_LIST entries (a pathological frame) reads
// its frame a second time and places 64-bit words in its own stretch of the
// workspace instead.
#ifndef SHPL_RANGE_KEYS
#define SHPL_RANGE_KEYS 128
#endif
constexpr int RANGE_KEYS = SHPL_RANGE_KEYS;
constexpr int RANGE_LIST = 10240;  // words of one range in LDS (2 arrays, 80 KiB)
constexpr int RANGE_BATCH = 16;    // entries per thread whose loads are in flight together

// Rank of entry `me` (order key `ke` if !entry_order) among words[a, z) of one
// destination and the emission of entry e at slot o. W(i) -> (entry, word
// compare value); entry_order: the words' numeric order is TF's.
template <bool HAS_COL, typename W>
__device__ __forceinline__ void range_emit(const CsrIn &c, int32_t total, const int32_t *beg, const int32_t *endk,
                                           int64_t k0, int64_t out0, W words, int32_t *ent_dst, int32_t *ent_src,
                                           float *ent_val, int32_t *ent_col) {
    const bool entry_order = c.order == SHPL_ORDER_ENTRY || !HAS_COL;
    for (int32_t s0 = threadIdx.x; s0 < total; s0 += CSR_BLOCK * CSR_BATCH) {
        int32_t d[CSR_BATCH], ee[CSR_BATCH], key[CSR_BATCH], kk[CSR_BATCH], src[CSR_BATCH];
        float val[CSR_BATCH];
#pragma unroll
        for (int u = 0; u < CSR_BATCH; ++u) {
            const int32_t sl = s0 + u * CSR_BLOCK;
            d[u] = -1;
            if (sl >= total) continue;
            int32_t t;
            const uint64_t me = words.get(sl, t, ee[u]);
            key[u] = (int32_t)(k0 + t);
            const int32_t a = beg[t], z = endk[t];
            int32_t rank = 0;
            if (z - a > 1) {
                if (entry_order) {
                    for (int32_t y = a; y < z; ++y) rank += words.cmp(y) < me ? 1 : 0;
                } else {
                    const uint64_t ke = order_key(c, ee[u]);
                    for (int32_t y = a; y < z; ++y) {
                        int32_t ty, o;
                        words.get(y, ty, o);
                        if (o == ee[u]) continue;
                        const uint64_t oo = order_key(c, o);
                        rank += (oo < ke || (oo == ke && o < ee[u])) ? 1 : 0;
                    }
                }
            }
            d[u] = a + rank;
        }
#pragma unroll
        for (int u = 0; u < CSR_BATCH; ++u) kk[u] = d[u] >= 0 ? (HAS_COL ? c.col[ee[u]] : ee[u]) : 0;
#pragma unroll
        for (int u = 0; u < CSR_BATCH; ++u) {
            if (d[u] < 0) continue;
            src[u] = c.direction == SHPL_BY_CELL ? c.pix[kk[u]] : c.cell[ee[u]];
            val[u] = c.val[ee[u]];
        }
#pragma unroll
        for (int u = 0; u < CSR_BATCH; ++u) {
            if (d[u] < 0) continue;
            const int64_t o = out0 + d[u];
            ent_dst[o] = key[u];
            ent_src[o] = src[u];
            ent_val[o] = val[u];
            if (ent_col) ent_col[o] = kk[u];
        }
    }
}

struct LdsWords {  // (local destination << 24 | entry - e0) words in LDS
    const uint32_t *w;
    int64_t e0;
    __device__ __forceinline__ uint64_t get(int32_t i, int32_t &t, int32_t &e) const {
        const uint32_t x = w[i];
        t = (int32_t)(x >> 24);
        e = (int32_t)(e0 + (x & 0xffffffu));
        return x;
    }
    __device__ __forceinline__ uint64_t cmp(int32_t i) const { return w[i]; }
};

struct GlobalWords {  // (destination << 32 | entry) words in the workspace
    const uint64_t *w;
    int64_t k0;
    __device__ __forceinline__ uint64_t get(int32_t i, int32_t &t, int32_t &e) const {
        const uint64_t x = w[i];
        t = (int32_t)((int64_t)(x >> 32) - k0);
        e = (int32_t)(uint32_t)x;
        return x;
    }
    __device__ __forceinline__ uint64_t cmp(int32_t i) const { return w[i]; }
};

template <bool HAS_COL>
__global__ __launch_bounds__(CSR_BLOCK) void k_csr_range(CsrIn c, uint64_t *tmp, int64_t nnz_cap, int64_t n_keys,
                                                         int n_ranges, int32_t *ent_dst, int32_t *ent_src,
                                                         float *ent_val, int32_t *ent_col, int32_t *key_range) {
    __shared__ int32_t cnt[RANGE_KEYS], beg[RANGE_KEYS];
    __shared__ int32_t wsum[CSR_BLOCK / 64];
    __shared__ int32_t n_list;
    __shared__ uint32_t list[RANGE_LIST], srt[RANGE_LIST];
    const int f = blockIdx.y, r = blockIdx.x;
    int64_t e0, e1, cap_end;
    frame_range(c, f, e0, e1, cap_end);
    const int64_t kf = (int64_t)f * c.keys_per_frame, kend = kf + c.keys_per_frame;
    const int64_t k0 = kf + (int64_t)r * RANGE_KEYS;
    const int nk = (int)(k0 + RANGE_KEYS < kend ? RANGE_KEYS : kend - k0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int t = threadIdx.x; t < RANGE_KEYS; t += CSR_BLOCK) cnt[t] = 0;
    if (threadIdx.x == 0) n_list = 0;
    __syncthreads();
    // 1. this range's entries -> LDS list + counts; valid entries below the range
    int32_t below = 0;
    for (int64_t b = e0 + threadIdx.x; b < e1; b += (int64_t)CSR_BLOCK * RANGE_BATCH) {
        int32_t key[RANGE_BATCH];
        keys_batch<HAS_COL>(c, b, e1, key);
#pragma unroll
        for (int u = 0; u < RANGE_BATCH; ++u) {
            const int64_t k = key[u];
            below += (k >= kf && k < k0) ? 1 : 0;  // invalid (-1) or outside the frame: left out
            const bool in = k >= k0 && k < k0 + nk;
            const uint64_t m = __ballot(in);
            if (m == 0) continue;  // wave-uniform
            int32_t base = 0;
            if (lane == 0) base = atomicAdd(&n_list, (int32_t)__popcll(m));
            base = __shfl(base, 0, 64);
            if (!in) continue;
            const int32_t slot = base + (int32_t)lane_rank(m);
            const int32_t t = (int32_t)(k - k0);
            if (slot < RANGE_LIST) list[slot] = ((uint32_t)t << 24) | (uint32_t)(b + (int64_t)u * CSR_BLOCK - e0);
            atomicAdd(&cnt[t], 1);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
    if (lane == 0) wsum[wid] = below;
    __syncthreads();
    below = 0;
    for (int w = 0; w < CSR_BLOCK / 64; ++w) below += wsum[w];
    const int32_t total = n_list;
    __syncthreads();  // wsum is reused by the scan
    // 2. exclusive scan: beg[t] = start of destination k0 + t; cnt becomes the fill cursor
    const int32_t v = threadIdx.x < RANGE_KEYS ? cnt[threadIdx.x] : 0;
    int32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int32_t run = x - v;
    for (int w = 0; w < wid; ++w) run += wsum[w];
    if (threadIdx.x < RANGE_KEYS) {
        beg[threadIdx.x] = run;
        cnt[threadIdx.x] = run;
    }
    __syncthreads();
    const int64_t out0 = e0 + below;
    // 3. placement by destination; 4. rank + emission (cnt[t] ends up at the end of destination k0 + t)
    if (total <= RANGE_LIST) {
        for (int32_t s = threadIdx.x; s < total; s += CSR_BLOCK) {
            const uint32_t w = list[s];
            srt[atomicAdd(&cnt[w >> 24], 1)] = w;
        }
        __syncthreads();
        range_emit<HAS_COL>(c, total, beg, cnt, k0, out0, LdsWords{srt, e0}, ent_dst, ent_src, ent_val, ent_col);
    } else {
        uint64_t *words = tmp + out0;  // this range's stretch of the frame's slots
        for (int64_t b = e0 + threadIdx.x; b < e1; b += (int64_t)CSR_BLOCK * RANGE_BATCH) {
            int32_t key[RANGE_BATCH];
            keys_batch<HAS_COL>(c, b, e1, key);
#pragma unroll
            for (int u = 0; u < RANGE_BATCH; ++u) {
                const int64_t k = key[u];
                if (k < k0 || k >= k0 + nk) continue;
                words[atomicAdd(&cnt[k - k0], 1)] =
                    ((uint64_t)(uint32_t)k << 32) | (uint32_t)(b + (int64_t)u * CSR_BLOCK);
            }
        }
        block_publish();  // the words went through memory to the other waves
        range_emit<HAS_COL>(c, total, beg, cnt, k0, out0, GlobalWords{words, k0}, ent_dst, ent_src, ent_val,
                            ent_col);
    }
    // 5. key ranges; holes after the frame's valid entries (the frame's last range)
    if (key_range) {
        for (int t = threadIdx.x; t < nk; t += CSR_BLOCK) {
            key_range[2 * (k0 + t)] = (int32_t)(out0 + beg[t]);
            key_range[2 * (k0 + t) + 1] = (int32_t)(out0 + cnt[t]);
        }
    }
    if (r != n_ranges - 1) return;
    for (int64_t h = out0 + total + threadIdx.x; h < cap_end; h += CSR_BLOCK) ent_dst[h] = -1;
    if (f != c.n_frames - 1) return;
    for (int64_t h = cap_end + threadIdx.x; h < nnz_cap; h += CSR_BLOCK) ent_dst[h] = -1;
    if (key_range)
        for (int64_t k = kend + threadIdx.x; k < n_keys; k += CSR_BLOCK) {
            key_range[2 * k] = 0;
            key_range[2 * k + 1] = 0;
        }
}

static_assert(RANGE_KEYS == 128, "the sort multisplit matches 7 destination bits");
static_assert(BK_KEYS == RANGE_KEYS, "the index builder's buckets are the sort's ranges");

// A bucket's counting sort (k_bsort2): words[0, n) = the bucket of destinations
// [k0, k0 + nk) (global ids, word = local destination << 24 | entry - e0) in entry order, placed stably
// by destination at out0.. with source row, value and column; key_range of its destinations. BY_CELL:
// source = pix[e]; BY_PIXEL: source = cell[e] and column e (the builder's identity columns). All threads
// call it. The bucket is cut into one contiguous slice per wave: the slices' per-destination counts
// (LDS atomics), one exclusive scan over (destination, slice) gives every (slice, destination) its first
// slot, and each wave then places its own slice in order, 64 words at a time (ballots over the 7
// destination bits rank a word among its batch's equals, one lane per destination moves the slice's
// cursor) -- three block barriers whatever the bucket's size. Buckets of at most LCAP words are read
// into LDS first together with their entries' source rows and values (every load in flight at once).
template <int BLOCK, int LCAP>
__device__ __forceinline__ void bucket_sort_emit(const uint32_t *words, int32_t n, int64_t e0, int64_t out0,
                                                 int64_t k0, int nk, int direction, const int32_t *col,
                                                 const int32_t *cell, const int32_t *pix, const float *vals,
                                                 int32_t *ent_dst, int32_t *ent_src, float *ent_val,
                                                 int32_t *ent_col, int32_t *key_range, int2 *heads = nullptr,
                                                 int head_k = 0) {
    constexpr int NW = BLOCK / 64;
    __shared__ int32_t cnt[NW][RANGE_KEYS], s_tot[RANGE_KEYS], s_beg[RANGE_KEYS];
    __shared__ uint64_t s_peer[NW][RANGE_KEYS];  // per wave and destination: its batch's lanes (zero between uses)
    __shared__ uint32_t l_w[LCAP > 0 ? LCAP : 1];
    __shared__ int32_t l_s[LCAP > 0 ? LCAP : 1];
    __shared__ float l_v[LCAP > 0 ? LCAP : 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const bool staged = n <= LCAP;
    const int32_t L = (n + NW - 1) / NW;  // words per wave slice
    for (int i = threadIdx.x; i < NW * RANGE_KEYS; i += BLOCK) {
        cnt[i / RANGE_KEYS][i % RANGE_KEYS] = 0;
        s_peer[i / RANGE_KEYS][i % RANGE_KEYS] = 0;
    }
    __syncthreads();
    // 1. per-slice counts (and, staged, the words with their sources and values into LDS)
    for (int32_t i0 = threadIdx.x; i0 < n; i0 += 4 * BLOCK) {  // 4 words per thread in flight
        uint32_t w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = i0 + u * BLOCK < n ? words[i0 + u * BLOCK] : 0u;
        if (staged) {
            int32_t sr[4];
            float vl[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i0 + u * BLOCK >= n) continue;
                const int64_t e = e0 + (w[u] & 0xffffffu);
                const int32_t kk = col ? col[e] : (int32_t)e;
                vl[u] = vals[e];
                sr[u] = direction == SHPL_BY_CELL ? pix[kk] : cell[e];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int32_t i = i0 + u * BLOCK;
                if (i >= n) continue;
                l_w[i] = w[u];
                l_s[i] = sr[u];
                l_v[i] = vl[u];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int32_t i = i0 + u * BLOCK;
            if (i < n) atomicAdd(&cnt[i / L][w[u] >> 24], 1);
        }
    }
    __syncthreads();
    // 2. (destination, slice) starts: totals per destination, scanned (first two waves), then the slices
    if ((int)threadIdx.x < RANGE_KEYS) {
        int32_t v = 0;
#pragma unroll
        for (int s = 0; s < NW; ++s) v += cnt[s][threadIdx.x];
        s_tot[threadIdx.x] = wave_incl_scan(v);  // inclusive prefix inside the wave
    }
    __syncthreads();
    if ((int)threadIdx.x < RANGE_KEYS) {
        const int32_t incl = s_tot[threadIdx.x] + (threadIdx.x >= 64 ? s_tot[63] : 0);
        int32_t run = incl;
        for (int s = NW - 1; s >= 0; --s) {  // slice cursors, last slice first (run ends at the start)
            run -= cnt[s][threadIdx.x];
            cnt[s][threadIdx.x] = run;
        }
        s_beg[threadIdx.x] = run;
        if (key_range && (int)threadIdx.x < nk) {
            key_range[2 * (k0 + threadIdx.x)] = (int32_t)(out0 + run);
            key_range[2 * (k0 + threadIdx.x) + 1] = (int32_t)(out0 + incl);
        }
    }
    __syncthreads();
    // 3. each wave places its slice in order, 64 words at a time (no block barrier)
    const int32_t s0 = wid * L, s1 = min(n, s0 + L);
    for (int32_t b0 = s0; b0 < s1; b0 += 64) {
        const int32_t i = b0 + lane;
        const bool ok = i < s1;
        uint32_t w = 0u;
        int32_t kk = 0, src = 0;
        float val = 0.0f;
        if (ok) {
            if (staged) {
                w = l_w[i];
                src = l_s[i];
                val = l_v[i];
                if (ent_col) kk = col ? col[e0 + (w & 0xffffffu)] : (int32_t)(e0 + (w & 0xffffffu));
            } else {
                w = words[i];
                const int64_t e = e0 + (w & 0xffffffu);
                kk = col ? col[e] : (int32_t)e;
                val = vals[e];
                src = direction == SHPL_BY_CELL ? pix[kk] : cell[e];
            }
        }
        const int t = (int)(w >> 24);
        // the batch's lanes of destination t: each ORs its bit into the wave's word of t, reads it back, and the
        // lanes zero it again (one wave's LDS operations run in order; 7 ballots over the destination bits cost
        // more VALU)
        uint64_t peers = 0;
        if (ok) atomicOr(reinterpret_cast<unsigned long long *>(&s_peer[wid][t]), 1ull << lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ok) peers = s_peer[wid][t];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ok) s_peer[wid][t] = 0;
        const int32_t rank = (int32_t)lane_rank(peers);
        const int32_t base = ok ? cnt[wid][t] : 0;
        // the batch's last lane of each destination moves the slice's cursor (after every lane's read: one
        // wave's LDS operations complete in order)
        if (ok && (peers >> lane) == 1ull) cnt[wid][t] = base + (int32_t)__popcll(peers);
        if (ok) {
            const int64_t o = out0 + base + rank;
            ent_dst[o] = (int32_t)(k0 + t);
            ent_src[o] = src;
            ent_val[o] = val;
            if (ent_col) ent_col[o] = kk;
            const int32_t hp = base + rank - s_beg[t];  // the entry's place in its destination's run
            if (heads && hp < head_k) heads[(k0 + t) * head_k + hp] = int2{src, __float_as_int(val)};
        }
    }
}

// ------------------------------------------------ both CSRs from the index build's buckets
// (shpl_build_csr_buckets). One launch: a BS_BLOCK-thread workgroup per (key, frame, range) sorts its
// bucket with bucket_sort_emit -- the buckets are the index builder's (shpl_common.h BkLayout), so no
// counting or bucketing pass precedes it. A frame of at most one entry has no bucket: that entry is
// read from the index arrays.
struct BsSide {
    int nr;            // ranges per frame (0: side absent)
    int64_t kpf, n_keys, nnz_cap;
    int32_t *ent_dst, *ent_src;
    float *ent_val;
    int32_t *ent_col, *key_range;
    int64_t blocks;    // n_frames * nr
    int2 *heads;       // optional run heads (shpl_csr.heads)
    int head_k;
};

struct BsIn {
    const int64_t *frame_off, *frame_nnz;
    const int32_t *cell, *pix;
    const float *val;
    const int32_t *ext;
    const uint32_t *words;
    const uint32_t *err;  // the index build's error word (shpl_buckets.err; NULL: no one-launch build, none failed)
    int n_frames, nrmax;
    int64_t nnz_cap;
};

constexpr int BS_BLOCK = 1024;  // threads of a k_bsort2 workgroup (the horizon's 2 k-entry pixel buckets: 3 rounds)
constexpr int BS_LCAP = 4096;   // bucket words staged in LDS with their source rows and values (48 KiB)

__global__ __launch_bounds__(BS_BLOCK) void k_bsort2(BsIn in, BsSide s0, BsSide s1) {
    __shared__ uint32_t one[1];
    // the pixel-keyed buckets first (the horizon's heavy ones start early instead of forming the tail)
    const bool second = (int64_t)blockIdx.x < s1.blocks;
    const int64_t b = second ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - s1.blocks;
    const BsSide &sd = second ? s1 : s0;
    const int key = second ? 1 : 0;
    const int f = (int)(b / sd.nr), q = (int)(b - (int64_t)f * sd.nr);
    const int64_t p0 = in.frame_off[f], cap_end = in.frame_off[f + 1];
    int64_t nnz = in.frame_nnz[f];
    nnz = nnz < 0 ? 0 : (nnz > cap_end - p0 ? cap_end - p0 : nnz);
    const int64_t kf = (int64_t)f * sd.kpf, kend = kf + sd.kpf;
    const int64_t k0 = kf + (int64_t)q * RANGE_KEYS;
    const int nk = (int)(k0 + RANGE_KEYS < kend ? RANGE_KEYS : kend - k0);
    const int direction = key ? SHPL_BY_PIXEL : SHPL_BY_CELL;
    int32_t start = 0, n = 0, valid = 0;
    const uint32_t *W = one;
    if (nnz >= 2) {
        const int32_t *x = in.ext + (((int64_t)key * in.n_frames + f) * in.nrmax + q) * 2;
        start = x[0];
        n = x[1];
        // after an index build whose frame barrier failed (it reported SHPL_EBIT_BARRIER; its buckets may be
        // half-written) every bucket reads as empty, and so does one outside the frame's entries: a wrong map
        // (the call is reported invalid), never a stray access; one scalar test, nothing per word
        if ((in.err && (*in.err & SHPL_EBIT_BARRIER)) || start < 0 || n < 0 || (int64_t)start + n > nnz)
            start = n = 0;
        W = in.words + (int64_t)key * in.nnz_cap + p0 + start;
        if (q == sd.nr - 1) valid = start + n;  // the frame's entries with valid destinations
    } else if (nnz == 1) {
        // no bucket: the frame's one entry, in this range or not
        const int32_t c = in.cell[p0], p = in.pix[p0];
        if (c >= 0 && p >= 0) {
            valid = 1;
            const int64_t k = key ? p : c;
            if (k >= k0 && k < k0 + nk) {
                if (threadIdx.x == 0) one[0] = (uint32_t)(k - k0) << 24;
                n = 1;
            }
        }
        __syncthreads();
    }
    const int64_t out0 = p0 + start;
    bucket_sort_emit<BS_BLOCK, BS_LCAP>(W, n, p0, out0, k0, nk, direction, nullptr, in.cell, in.pix, in.val, sd.ent_dst,
                                        sd.ent_src, sd.ent_val, sd.ent_col, sd.key_range, sd.heads, sd.head_k);
    // the frame's unused capacity (its last range), the slots and key ranges after the last frame
    if (q != sd.nr - 1) return;
    for (int64_t h = p0 + valid + threadIdx.x; h < cap_end; h += BS_BLOCK) sd.ent_dst[h] = -1;
    if (f != in.n_frames - 1) return;
    for (int64_t h = cap_end + threadIdx.x; h < sd.nnz_cap; h += BS_BLOCK) sd.ent_dst[h] = -1;
    if (sd.key_range)
        for (int64_t kk = kend + threadIdx.x; kk < sd.n_keys; kk += BS_BLOCK) {
            sd.key_range[2 * kk] = 0;
            sd.key_range[2 * kk + 1] = 0;
        }
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

// Workspace: [tmp words | segmented path: kbuf | sorted words | counters].
// The segmented path is taken when its counters fit (n_frames * S <=
// seg_cap, i.e. up to ~4096 frames) -- see csr_plan.
namespace {
constexpr int64_t SEG_TARGET = 2048;  // entries per segment the host aims for
constexpr int SEG_FRAMES = 32;        // batches from this many frames sort one frame per workgroup
constexpr int64_t RANGE_MAX_KEYS = 65536;  // destinations per frame up to which small batches take the range CSR

int64_t seg_cap_of(int64_t nnz_cap) { return nnz_cap / 16 + 65536; }  // bin + cursor counters

struct CsrLayout {
    size_t tmp, kbuf, sorted, counters, total;
};

CsrLayout csr_layout(int64_t n_keys, int64_t nnz_cap) {
    CsrLayout l = {};
    const size_t cap = (size_t)(nnz_cap > 0 ? nnz_cap : 1);
    l.tmp = 0;
    l.kbuf = align_up(sizeof(uint64_t) * cap, 256);
    l.sorted = l.kbuf + align_up(sizeof(int32_t) * cap, 256);
    l.counters = l.sorted + align_up(sizeof(uint64_t) * cap, 256);
    l.total = l.counters + align_up(2 * sizeof(int32_t) * (size_t)seg_cap_of(nnz_cap), 256);
    return l;
}
}  // namespace

extern "C" int shpl_csr_workspace_bytes(int64_t n_keys, int64_t nnz_cap, size_t *bytes) {
    if (!bytes || n_keys < 0 || nnz_cap < 0) return SHPL_ERR_ARG;
    *bytes = csr_layout(n_keys, nnz_cap).total;
    return SHPL_OK;
}

extern "C" int shpl_build_csr_path(int path, int direction, int order, int n_frames, const int64_t *d_frame_off,
                                   const int64_t *d_frame_nnz, int64_t keys_per_frame, const int32_t *d_cell,
                                   const int32_t *d_col, const float *d_val, const int32_t *d_pix,
                                   const shpl_csr *csr, void *d_ws, size_t ws_bytes, void *stream) {
    if (path < SHPL_CSR_AUTO || path > SHPL_CSR_RANGE) return SHPL_ERR_ARG;
    if (!csr || !d_frame_off || n_frames < 1) return SHPL_ERR_ARG;
    if (csr->heads) return SHPL_ERR_ARG;  // run heads: shpl_build_csr_buckets only
    if (direction != SHPL_BY_CELL && direction != SHPL_BY_PIXEL) return SHPL_ERR_ARG;
    if (order < SHPL_ORDER_ENTRY || order > SHPL_ORDER_COL_ENTRY) return SHPL_ERR_ARG;
    const int64_t nnz_cap = csr->nnz_cap;
    if (keys_per_frame < 1 || nnz_cap < 0 || csr->n_keys < (int64_t)n_frames * keys_per_frame ||
        csr->n_keys >= 2147483647LL || nnz_cap >= 2147483647LL)
        return SHPL_ERR_BAD_SHAPE;
    if (nnz_cap == 0) {
        // an empty map: every destination's run is empty (first == end == 0)
        if (csr->key_range && csr->n_keys > 0 &&
            hipMemsetAsync(csr->key_range, 0, sizeof(int32_t) * 2 * (size_t)csr->n_keys, (hipStream_t)stream) !=
                hipSuccess)
            return SHPL_ERR_HIP;
        return SHPL_OK;
    }
    if (!d_cell || !d_val || !d_pix || !csr->ent_dst || !csr->ent_src || !csr->ent_val || !d_ws) return SHPL_ERR_ARG;
    if (direction == SHPL_BY_PIXEL && !csr->ent_col) return SHPL_ERR_ARG;
    const CsrLayout lay = csr_layout(csr->n_keys, nnz_cap);
    hipStream_t st = (hipStream_t)stream;
    uint8_t *ws = (uint8_t *)d_ws;
    // The range CSR: always when key ranges are asked for; by default for batches under
    // SEG_FRAMES frames of at most RANGE_MAX_KEYS destinations (each workgroup reads its
    // whole frame, so many ranges per frame would multiply those reads).
    // (entry offsets inside a frame travel in 24 bits: capacities under 2^24 entries)
    const bool small_cap = nnz_cap < ((int64_t)1 << 24);
    if (csr->key_range && !small_cap) return SHPL_ERR_BAD_SHAPE;
    // key ranges from the frame builder instead (asked for by name): its sort, then k_key_range
    const bool frame_ranges = csr->key_range != nullptr && path == SHPL_CSR_FRAME;
    const bool ranged = (csr->key_range != nullptr && !frame_ranges) ||
                        (small_cap && !frame_ranges && (path != SHPL_CSR_AUTO
                                           ? path == SHPL_CSR_RANGE
                                           : (n_frames < SEG_FRAMES && keys_per_frame <= RANGE_MAX_KEYS)));
    if (ranged) {
        if (ws_bytes < align_up(sizeof(uint64_t) * (size_t)nnz_cap, 256)) return SHPL_ERR_WORKSPACE;
        const int64_t n_ranges = (keys_per_frame + RANGE_KEYS - 1) / RANGE_KEYS;
        if (n_ranges > 65535) return SHPL_ERR_BAD_SHAPE;
        CsrIn c{direction, order, n_frames, d_frame_off, d_frame_nnz, keys_per_frame, 0,
                d_cell, d_col, d_pix, d_val};
        const dim3 grid((unsigned)n_ranges, (unsigned)n_frames);
        if (d_col)
            hipLaunchKernelGGL(k_csr_range<true>, grid, dim3(CSR_BLOCK), 0, st, c, (uint64_t *)ws, nnz_cap,
                               csr->n_keys, (int)n_ranges, csr->ent_dst, csr->ent_src, csr->ent_val, csr->ent_col,
                               csr->key_range);
        else
            hipLaunchKernelGGL(k_csr_range<false>, grid, dim3(CSR_BLOCK), 0, st, c, (uint64_t *)ws, nnz_cap,
                               csr->n_keys, (int)n_ranges, csr->ent_dst, csr->ent_src, csr->ent_val, csr->ent_col,
                               csr->key_range);
        SHPL_LAUNCH_CHECK();
        return SHPL_OK;
    }
    // segments: about SEG_TARGET entries each (estimated from the capacity per frame)
    const int64_t est = (nnz_cap + n_frames - 1) / n_frames;
    int log_bin = 0;
    while (((keys_per_frame - 1) >> log_bin) + 1 > SEG_MAX) ++log_bin;
    const int64_t n_bins = ((keys_per_frame - 1) >> log_bin) + 1;
    int64_t S = (est + SEG_TARGET - 1) / SEG_TARGET;
    if (S < 1) S = 1;
    if (S > n_bins) S = n_bins;
    // Small batches take the segmented path (config 3, 4 frames: 0.305 -> 0.259 ms per step); from
    // SEG_FRAMES frames on, one workgroup per frame fills enough of the chip and, overlapped with the
    // dense stream, measured faster (config 2, 64 frames: 2.34 vs 2.42 ms per step).
    // shpl_build_csr_path(SHPL_CSR_FRAME | _SEGMENT | _RANGE, ...) forces a path (tests, measurements).
    const bool want = path != SHPL_CSR_AUTO ? path == SHPL_CSR_SEGMENT : n_frames < SEG_FRAMES;
    const bool segmented = want && ws_bytes >= lay.total && (int64_t)n_frames * (n_bins + S) <= seg_cap_of(nnz_cap);
    if (frame_ranges) {
        hipLaunchKernelGGL(k_zero32, dim3(grid_for(2 * csr->n_keys, SEG_BLOCK, 4096)), dim3(SEG_BLOCK), 0, st,
                           csr->key_range, 2 * csr->n_keys);
        SHPL_LAUNCH_CHECK();
    }
    if (!segmented) {
        // one workgroup per frame; needs only the tmp words
        if (ws_bytes < align_up(sizeof(uint64_t) * (size_t)nnz_cap, 256)) return SHPL_ERR_WORKSPACE;
        int log_tile = 0;
        while (((keys_per_frame - 1) >> log_tile) + 1 > CSR_TILES) ++log_tile;
        CsrIn c{direction, order, n_frames, d_frame_off, d_frame_nnz, keys_per_frame, log_tile,
                d_cell, d_col, d_pix, d_val};
        // n_frames sorting workgroups + the workgroups clearing the unused capacity
        const int64_t spans = d_frame_nnz ? (nnz_cap + HOLE_SPAN - 1) / HOLE_SPAN : 0;
        const dim3 grid((unsigned)(n_frames + spans));
        if (d_col)
            hipLaunchKernelGGL(k_csr_frame<true>, grid, dim3(CSR_BLOCK), 0, st, c, (uint64_t *)ws, nnz_cap,
                               csr->ent_dst, csr->ent_src, csr->ent_val, csr->ent_col);
        else
            hipLaunchKernelGGL(k_csr_frame<false>, grid, dim3(CSR_BLOCK), 0, st, c, (uint64_t *)ws, nnz_cap,
                               csr->ent_dst, csr->ent_src, csr->ent_val, csr->ent_col);
        SHPL_LAUNCH_CHECK();
        if (frame_ranges) {
            hipLaunchKernelGGL(k_key_range, dim3(grid_for(nnz_cap, SEG_BLOCK, 4096)), dim3(SEG_BLOCK), 0, st,
                               csr->ent_dst, nnz_cap, csr->key_range);
            SHPL_LAUNCH_CHECK();
        }
        return SHPL_OK;
    }
    CsrIn c{direction, order, n_frames, d_frame_off, d_frame_nnz, keys_per_frame, 0,
            d_cell, d_col, d_pix, d_val};
    SegIn g = {};
    g.S = (int)S;
    g.n_bins = (int)n_bins;
    g.log_bin = log_bin;
    g.hist = (int32_t *)(ws + lay.counters);
    g.cur = g.hist + (int64_t)n_frames * n_bins;
    g.kbuf = (int32_t *)(ws + lay.kbuf);
    g.bucket = (uint64_t *)(ws + lay.tmp);
    g.sorted = (uint64_t *)(ws + lay.sorted);
    const int64_t n_ctr = (int64_t)n_frames * (n_bins + S);
    hipLaunchKernelGGL(k_zero32, dim3(grid_for(n_ctr, SEG_BLOCK, 1024)), dim3(SEG_BLOCK), 0, st, g.hist, n_ctr);
    SHPL_LAUNCH_CHECK();
    const int gx = (int)(est / 1024 < 1 ? 1 : (est / 1024 > 1024 ? 1024 : est / 1024));
    const dim3 grid_fr((unsigned)gx, (unsigned)n_frames);
    if (d_col)
        hipLaunchKernelGGL(k_csr_count<true>, grid_fr, dim3(SEG_BLOCK), 0, st, c, g);
    else
        hipLaunchKernelGGL(k_csr_count<false>, grid_fr, dim3(SEG_BLOCK), 0, st, c, g);
    SHPL_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_csr_bucket, grid_fr, dim3(SEG_BLOCK), 0, st, c, g);
    SHPL_LAUNCH_CHECK();
    const int64_t spans = d_frame_nnz ? (nnz_cap + HOLE_SPAN - 1) / HOLE_SPAN : 0;
    const dim3 grid_seg((unsigned)S, (unsigned)(n_frames + (spans + S - 1) / S));
    if (d_col)
        hipLaunchKernelGGL(k_csr_segment<true>, grid_seg, dim3(CSR_BLOCK), 0, st, c, g, nnz_cap, csr->ent_dst,
                           csr->ent_src, csr->ent_val, csr->ent_col);
    else
        hipLaunchKernelGGL(k_csr_segment<false>, grid_seg, dim3(CSR_BLOCK), 0, st, c, g, nnz_cap, csr->ent_dst,
                           csr->ent_src, csr->ent_val, csr->ent_col);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

extern "C" int shpl_build_csr(int direction, int order, int n_frames, const int64_t *d_frame_off,
                              const int64_t *d_frame_nnz, int64_t keys_per_frame, const int32_t *d_cell,
                              const int32_t *d_col, const float *d_val, const int32_t *d_pix, const shpl_csr *csr,
                              void *d_ws, size_t ws_bytes, void *stream) {
    return shpl_build_csr_path(SHPL_CSR_AUTO, direction, order, n_frames, d_frame_off, d_frame_nnz, keys_per_frame,
                               d_cell, d_col, d_val, d_pix, csr, d_ws, ws_bytes, stream);
}

extern "C" int shpl_build_csr_buckets(const shpl_buckets *bk, const shpl_csr *by_cell, const shpl_csr *by_pixel,
                                      void *stream) {
    if (!bk || bk->n_frames < 1 || !bk->frame_off || !bk->frame_nnz || !bk->ws) return SHPL_ERR_ARG;
    size_t need = 0;
    int rc = shpl_bucket_workspace_bytes(bk->n_frames, bk->max_points_per_frame, bk->nnz_cap, bk->cells_per_frame,
                                         bk->pix_per_frame, &need);
    if (rc) return rc;
    if (bk->ws_bytes < need) return SHPL_ERR_WORKSPACE;
    if (bk->nnz_cap > 0 && (!bk->cell || !bk->pix || !bk->val)) return SHPL_ERR_ARG;
    const int64_t chunks = (bk->max_points_per_frame + 1023) / 1024;
    const BkLayout l = bk_layout(bk->n_frames, (int)(chunks < 1 ? 1 : chunks), bk->nnz_cap, bk->cells_per_frame,
                                 bk->pix_per_frame);
    const shpl_csr *cs[2] = {by_cell, by_pixel};
    BsSide s[2] = {};
    for (int k = 0; k < 2; ++k) {
        const shpl_csr *c = cs[k];
        if (!c) continue;
        if (c->n_keys < (int64_t)bk->n_frames * l.kpf[k] || c->n_keys >= 2147483647LL || c->nnz_cap < bk->nnz_cap)
            return SHPL_ERR_BAD_SHAPE;
        if (bk->nnz_cap > 0 && (!c->ent_dst || !c->ent_src || !c->ent_val)) return SHPL_ERR_ARG;
        if (k == 1 && !c->ent_col && !(c->flags & SHPL_CSR_IDENTITY_COLS)) return SHPL_ERR_ARG;
        if (c->heads && (c->head_k < 1 || c->head_k > SHPL_CSR_MAX_HEAD || !c->key_range)) return SHPL_ERR_ARG;
        s[k] = BsSide{l.nr[k], l.kpf[k], c->n_keys, c->nnz_cap, c->ent_dst, c->ent_src, c->ent_val, c->ent_col,
                      c->key_range, (int64_t)bk->n_frames * l.nr[k], (int2 *)c->heads, (int)c->head_k};
        if (l.nr[k] == 0) s[k].blocks = 0;
    }
    hipStream_t st = (hipStream_t)stream;
    if (bk->nnz_cap == 0) {  // an empty map: empty runs everywhere
        for (int k = 0; k < 2; ++k) {
            if (cs[k] && cs[k]->key_range && cs[k]->n_keys > 0 &&
                hipMemsetAsync(cs[k]->key_range, 0, sizeof(int32_t) * 2 * (size_t)cs[k]->n_keys, st) != hipSuccess)
                return SHPL_ERR_HIP;
        }
        return SHPL_OK;
    }
    const int64_t blocks = s[0].blocks + s[1].blocks;
    if (blocks == 0) return SHPL_OK;
    if (blocks > 0x7fffffffLL) return SHPL_ERR_BAD_SHAPE;
    char *w = (char *)bk->ws;
    const BsIn in{bk->frame_off, bk->frame_nnz, bk->cell, bk->pix, bk->val, (const int32_t *)(w + l.ext),
                  (const uint32_t *)(w + l.words), bk->err, bk->n_frames, l.nrmax, bk->nnz_cap};
    hipLaunchKernelGGL(k_bsort2, dim3((unsigned)blocks), dim3(BS_BLOCK), 0, st, in, s[0], s[1]);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}
