// shpl_pull.hip -- the SHPL gather / scatter-add as destination-keyed pulls.
//
// Reference ops (TF 1.8 stock kernels, avod/avod/utils/sparse_pool_utils.py):
//   img->BEV  :96-103  gather_nd + sparse_tensor_dense_matmul (+ concat :72)
//   BEV->img  :105-117 sparse_transpose + matmul + scatter_nd  (+ concat :87)
//   and their autodiff gradients.
// TF's GPU kernels scatter with atomics. Here the output is produced by two
// launches on one stream, both free of atomics and bitwise reproducible:
//
//   k_dense  -- streams every output row: the pass-through half of a concat
//               is copied, the pooled part is written as 0 (POOL / CONCAT) or
//               pass + 0 (ADD). It reads no index at all, so it runs at the
//               chip's streaming rate and may start before M is even built.
//   k_sparse -- one thread per (sorted CSR entry, 16-byte chunk); the thread
//               sitting on the first entry of a destination walks that
//               destination's entries in TF-CPU order (separate multiply and
//               add, no FMA contraction: bit-identical to TF's sequential
//               `out += a*b`) and overwrites the pooled chunk of that row.
// The zeros k_dense writes into occupied rows are rewritten by k_sparse:
// nnz*16 B per chunk column (about 1 % of the stream at config 2), against a
// read-before-write occupancy test that cost ~17 % of the stream (measured,
// scripts/pull_sweep.py).
//
// Work unit: one 16-byte chunk (4 f32 / 8 bf16); a 64-lane wave stores 1 KiB
// contiguous. k_dense is a full grid, one chunk per thread (no grid-stride
// loop): the fastest streaming shape measured on MI355X for this traffic
// (read 1 : write 2) -- see DESIGN.md.
#include "shpl_common.h"

#ifndef SHPL_NT_LOAD
#define SHPL_NT_LOAD 1
#endif
#ifndef SHPL_NT_STORE
#define SHPL_NT_STORE 1
#endif

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
#if SHPL_NT_LOAD
        return __builtin_nontemporal_load(reinterpret_cast<const raw_t *>(p));
#else
        return *reinterpret_cast<const raw_t *>(p);
#endif
    }
    static __device__ __forceinline__ void store_nt(T *p, raw_t v) {
#if SHPL_NT_STORE
        __builtin_nontemporal_store(v, reinterpret_cast<raw_t *>(p));
#else
        *reinterpret_cast<raw_t *>(p) = v;
#endif
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
    static __device__ __forceinline__ raw_t zero() {
        raw_t r;
        __builtin_memset(&r, 0, sizeof(r));
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

struct Feat {  // strided feature rows: row r, element c at base + r*stride + off + c
    const void *src;
    int64_t src_stride, src_off;
    const void *pass;
    int64_t pass_stride, pass_off;
    void *out;
    int64_t out_stride;
    uint32_t cpr;    // chunks per output row
    uint32_t cpass;  // chunks of the pass-through half (CONCAT)
    uint32_t cpool;  // chunks of the pooled part
    int mode;
    int cpr_shift;   // log2(cpr) when cpr is a power of two, else -1
};

// ---------------------------------------------------------------- k_dense
template <typename T, int VEC, bool POW2>
__global__ __launch_bounds__(SHPL_BLOCK) void k_dense(const Feat f, uint32_t row0, uint32_t n_rows) {
    typedef Chunk<T, VEC> C;
    const uint32_t g = blockIdx.x * SHPL_BLOCK + threadIdx.x;
    if (g >= n_rows * f.cpr) return;
    const uint32_t r = POW2 ? g >> f.cpr_shift : g / f.cpr;  // a shift instead of a division when it can
    const uint32_t ch = g - r * f.cpr;
    // row < 2^32 and row widths < 2^31 (plan() checks): 32 x 32 -> 64-bit offsets
    const uint32_t row = row0 + r;
    const T *pass = reinterpret_cast<const T *>(f.pass) + f.pass_off;
    const uint64_t pass_at = (uint64_t)row * (uint32_t)f.pass_stride + ch * VEC;
    typename C::raw_t v;
    if (f.mode == SHPL_OUT_ADD) {
        // pass + 0.0f: TF's add_n with an all-zero scatter turns -0 into +0
        float a[VEC];
        C::to_f32(C::load_nt(pass + pass_at), a);
#pragma unroll
        for (int j = 0; j < VEC; ++j) a[j] = __fadd_rn(a[j], 0.0f);
        v = C::from_f32(a);
    } else if (f.mode == SHPL_OUT_CONCAT && ch < f.cpass) {
        v = C::load_nt(pass + pass_at);
    } else {
        v = C::zero();
    }
    C::store_nt(reinterpret_cast<T *>(f.out) + ((uint64_t)row * (uint32_t)f.out_stride + ch * VEC), v);
}

// ---------------------------------------------------------------- k_sparse
struct Ents {
    int64_t n;  // capacity; empty slots carry dst = -1
    const int32_t *dst, *src, *col;
    const float *val;
    // optional frame layout (n_frames > 0): frame f's live entries are the first frame_nnz[f] slots of
    // [frame_off[f], frame_off[f+1]), the rest of the capacity is empty
    const int64_t *frame_off, *frame_nnz;
    int n_frames;
    // optional run heads (shpl_csr.heads, row-keyed pulls): (source, value bits) of each destination's first
    // head_k entries, loaded in the round trip of its key_range
    const int2 *heads;
    int head_k;
};

// The live-entry table of a frame layout in LDS (one per workgroup): s_off[f] = frame f's first slot
// (s_off[F] = the end of the last frame), s_pre[f] = live entries of the frames before f (s_pre[F] =
// all). Returns the live total.
constexpr int LIVE_MAX_FRAMES = SHPL_LIVE_MAX_FRAMES;
__device__ __forceinline__ int32_t live_table(const Ents &e, int32_t *s_off, int32_t *s_pre, int64_t *s_scan) {
    const int F = e.n_frames;
    int32_t cnt[LIVE_MAX_FRAMES / SHPL_BLOCK];
    int64_t sum = 0;
#pragma unroll
    for (int k = 0; k < LIVE_MAX_FRAMES / SHPL_BLOCK; ++k) {
        const int fi = (LIVE_MAX_FRAMES / SHPL_BLOCK) * threadIdx.x + k;
        cnt[k] = 0;
        if (fi < F) {
            const int64_t o0 = e.frame_off[fi], o1 = e.frame_off[fi + 1], n = e.frame_nnz[fi];
            cnt[k] = (int32_t)(n < 0 ? 0 : (n < o1 - o0 ? n : o1 - o0));
            s_off[fi] = (int32_t)o0;
            if (fi == F - 1) s_off[F] = (int32_t)o1;
        }
        sum += cnt[k];
    }
    int64_t total;
    int64_t run = block_excl_scan(sum, s_scan, &total);
#pragma unroll
    for (int k = 0; k < LIVE_MAX_FRAMES / SHPL_BLOCK; ++k) {
        const int fi = (LIVE_MAX_FRAMES / SHPL_BLOCK) * threadIdx.x + k;
        if (fi < F) s_pre[fi] = (int32_t)run;
        run += cnt[k];
    }
    if (threadIdx.x == 0) s_pre[F] = (int32_t)total;
    __syncthreads();
    return (int32_t)total;
}

// The frame holding live entry L (0 <= L < s_pre[F]): the last f with s_pre[f] <= L (never an empty one).
__device__ __forceinline__ int live_frame(const int32_t *s_pre, int F, int64_t L) {
    int lo = 0, hi = F;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (s_pre[mid] <= L) lo = mid; else hi = mid;
    }
    return lo;
}

template <int VEC>
__device__ __forceinline__ void fma_free_accumulate(float (&acc)[VEC], float w, const float (&x)[VEC]) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], __fmul_rn(w, x[j]));
}

#ifndef SHPL_WALK
#define SHPL_WALK 2
#endif
constexpr int WALK = SHPL_WALK;
// Runs longer than LONG_RUN entries (config 3: up to 54 image points on one
// pixel) are left to k_sparse_long, which batches LONG_WALK entries per
// feature round trip with the index words staged in LDS; k_sparse then never walks more than LONG_RUN / WALK
// steps, and the common short runs keep its low register count.
constexpr int LONG_RUN = 8;
constexpr int LONG_WALK = 16;

// Sum of one destination's run starting at sorted entry s, chunk c (VEC
// elements of the pooled part), in TF-CPU order: entries in CSR order with
// separate multiply and add; GROUP (BY_PIXEL): per column partial Q[k] first
// (ScatterNd's order). W entries per step: their index loads, then their
// feature loads, are each in flight together.
// Index words of W consecutive entries from i (past nnz: dst -1).
template <bool GROUP, int W>
struct IdxBatch {
    int32_t d[W], sr[W], kc[W];
    float w[W];
    __device__ __forceinline__ void load(const Ents &e, int64_t i) {
#pragma unroll
        for (int u = 0; u < W; ++u) {
            const bool ok = i + u < e.n;
            d[u] = ok ? e.dst[i + u] : -1;
            sr[u] = ok ? e.src[i + u] : 0;
            w[u] = ok ? e.val[i + u] : 0.0f;
            kc[u] = (GROUP && ok) ? e.col[i + u] : 0;
        }
    }
};

template <typename T, int VEC, bool GROUP, int W>
__device__ __forceinline__ void walk_run(const Feat &f, const Ents &e, int64_t s, int32_t key, uint32_t c,
                                         float (&acc)[VEC], const IdxBatch<GROUP, W> *first = nullptr) {
    typedef Chunk<T, VEC> C;
    const T *sc = reinterpret_cast<const T *>(f.src) + f.src_off + (int64_t)c * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.0f;
    float q[VEC];  // GROUP: the current column's partial, TF's Q[k]
#pragma unroll
    for (int j = 0; j < VEC; ++j) q[j] = 0.0f;
    int32_t kprev = -1;  // no column yet: the first flush adds a zero partial (0 + 0 = +0)
    for (int64_t i = s;; i += W) {
        bool in[W];
        int32_t d[W], sr[W], kc[W];
        float w[W];
        // index loads of the batch do not wait for each other (dst need not match yet);
        // the first batch may come preloaded (issued with the caller's head test)
        IdxBatch<GROUP, W> b;
        if (first && i == s)
            b = *first;
        else
            b.load(e, i);
#pragma unroll
        for (int u = 0; u < W; ++u) {
            d[u] = b.d[u];
            sr[u] = b.sr[u];
            w[u] = b.w[u];
            kc[u] = b.kc[u];
        }
#pragma unroll
        for (int u = 0; u < W; ++u) in[u] = d[u] == key && (u == 0 || in[u - 1]);
        typename C::raw_t raw[W];
#pragma unroll
        for (int u = 0; u < W; ++u)
            if (in[u]) raw[u] = C::load(sc + (int64_t)sr[u] * f.src_stride);
#pragma unroll
        for (int u = 0; u < W; ++u) {
            if (!in[u]) break;
            float x[VEC];
            C::to_f32(raw[u], x);
            if (GROUP) {
                // TF: Q[k] = sum of column k's entries; out = 0 + Q[k1] + Q[k2] ... (ScatterNd order)
                if (kc[u] != kprev) {
#pragma unroll
                    for (int j = 0; j < VEC; ++j) {
                        acc[j] = __fadd_rn(acc[j], q[j]);
                        q[j] = 0.0f;
                    }
                    kprev = kc[u];
                }
                fma_free_accumulate<VEC>(q, w[u], x);
            } else {
                fma_free_accumulate<VEC>(acc, w[u], x);
            }
        }
        if (!in[W - 1]) break;
    }
    if (GROUP) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], q[j]);
    }
}

template <typename T, int VEC>
__device__ __forceinline__ void store_pooled(const Feat &f, int32_t key, uint32_t c, float (&acc)[VEC]) {
    typedef Chunk<T, VEC> C;
    if (f.mode == SHPL_OUT_ADD) {
        const T *pass = reinterpret_cast<const T *>(f.pass) + f.pass_off;
        float a[VEC];
        C::to_f32(C::load(pass + (int64_t)key * f.pass_stride + (int64_t)c * VEC), a);
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(a[j], acc[j]);
    }
    const uint32_t oc = (f.mode == SHPL_OUT_CONCAT ? f.cpass : 0u) + c;
    C::store_nt(reinterpret_cast<T *>(f.out) + (int64_t)key * f.out_stride + (int64_t)oc * VEC, C::from_f32(acc));
}

// One thread per (sorted entry, chunk); the thread on the first entry of a
// destination's run sums it and writes the pooled chunk -- for runs of at
// most LONG_RUN entries (SPLIT) or all runs (!SPLIT).
// LIVE: with a frame layout, threads walk (live entry, chunk) pairs of a grid sized for the GPU, not
// the capacity's (entry, chunk) pairs (the empty slots' waves cost more than the work at raw-scan
// occupancy), and take every run (no k_sparse_long pass over the capacity); the sums and stores are
// the same.
template <typename T, int VEC, bool GROUP, bool SPLIT, bool POW2, bool LIVE>
__device__ __forceinline__ void sparse_body(const Feat &f, const Ents &e, int cpool_shift, int64_t bid, int64_t nblk) {
    __shared__ int32_t s_off[LIVE ? LIVE_MAX_FRAMES + 1 : 1], s_pre[LIVE ? LIVE_MAX_FRAMES + 1 : 1];
    __shared__ int64_t s_scan[SHPL_BLOCK / 64 + 1];
    const int64_t nnz = e.n;
    const int64_t total = (LIVE ? (int64_t)live_table(e, s_off, s_pre, s_scan) : nnz) * (int64_t)f.cpool;
    for (int64_t t = bid * SHPL_BLOCK + threadIdx.x; t < total; t += nblk * SHPL_BLOCK) {
        // a shift, not a 64-bit division, when the chunk count is a power of two
        const int64_t l = POW2 ? t >> cpool_shift : t / f.cpool;
        const uint32_t c = (uint32_t)(t - l * f.cpool);
        int64_t s = l;
        if (LIVE) {
            const int fr = live_frame(s_pre, e.n_frames, l);
            s = (int64_t)s_off[fr] + (l - s_pre[fr]);
        }
        // the head test's loads and the walk's first index batch are
        // independent: one round trip
        IdxBatch<GROUP, WALK> b0;
        b0.load(e, s);
        const int32_t key = b0.d[0];
        const int32_t prev = s > 0 ? e.dst[s - 1] : -1;
        const int32_t ahead = (SPLIT && s + LONG_RUN < nnz) ? e.dst[s + LONG_RUN] : -1;
        if (key < 0 || prev == key) continue;  // empty, or not the first entry of key
        if (SPLIT && ahead == key) continue;   // a run longer than LONG_RUN: k_sparse_long's
        float acc[VEC];
        walk_run<T, VEC, GROUP, WALK>(f, e, s, key, c, acc, &b0);
        store_pooled<T, VEC>(f, key, c, acc);
    }
}

template <typename T, int VEC, bool GROUP, bool SPLIT, bool POW2, bool LIVE>
__global__ __launch_bounds__(SHPL_BLOCK) void k_sparse(const Feat f, const Ents e, int cpool_shift) {
    sparse_body<T, VEC, GROUP, SPLIT, POW2, LIVE>(f, e, cpool_shift, blockIdx.x, gridDim.x);
}

// shpl_pull_once: the pooled part of every destination row written exactly once, in ONE launch and with no
// streaming pass before it. The sblocks run-walking blocks write the occupied rows: seg_window's wave per 64
// sorted entries for wide cell-keyed rows (once_seg), else k_sparse's (entry, chunk) walk over every run; the
// rest zero the rows whose key_range is empty: a wave per ONCE_ROWS rows, one key_range load for all of them,
// then their zero chunks stored with nothing to wait for. Rows and stores are disjoint between the two parts.
#ifndef SHPL_ONCE_ROWS
#define SHPL_ONCE_ROWS 16
#endif
#ifndef SHPL_ONCE_XCD
#define SHPL_ONCE_XCD 1
#endif
#ifndef SHPL_ONCE_ZERO_FIRST
#define SHPL_ONCE_ZERO_FIRST 1  // the zeroing blocks first: 1.401-1.404 vs 1.408-1.410 ms at config 6 (profiles/r05_once_ab.log)
#endif
constexpr int ONCE_ROWS = SHPL_ONCE_ROWS;
#ifndef SHPL_ONCE_SEG
#define SHPL_ONCE_SEG 1
#endif
#ifndef SHPL_SEG_BATCH
#define SHPL_SEG_BATCH 8
#endif
constexpr int SEG_BATCH = SHPL_SEG_BATCH;
#ifndef SHPL_SEG_CONT
#define SHPL_SEG_CONT 2
#endif
// entries per step past the window (a run crossing it: rare, short); 2 keeps k_once at 84 VGPRs without spills
// under its 5-waves bound (8: 136 VGPRs, 3 waves per SIMD, 0.578 vs 0.513-0.520 ms at config 6;
// profiles/r05_c6c2_ab.log)
constexpr int SEG_CONT = SHPL_SEG_CONT;
// the window walk for cell-keyed rows of at least half a wave of chunks (RetinaNet's 256 channels: 64 f32 /
// 32 bf16 chunks); narrower rows would leave most lanes idle through the window's serial walk (measured as
// shpl_pull_sparse's form at config 2's 32 channels: 205 vs 80 us)
__host__ __device__ constexpr bool once_seg(bool group, uint32_t cpool) {
    return SHPL_ONCE_SEG && !group && cpool >= 32;
}

template <typename T, int VEC>
__device__ __forceinline__ void seg_load(const T *sc, int64_t stride, int32_t sr, bool ok,
                                         typename Chunk<T, VEC>::raw_t &raw) {
    if (ok) raw = Chunk<T, VEC>::load(sc + (int64_t)sr * stride);
}

// The occupied rows of shpl_pull_once by windows of 64 sorted entries, one wave per window (cell-keyed, no
// column partials): the window's index words in one coalesced round trip (lane l holds entry s0 + l), the run
// heads and boundaries as ballots, then the window's entries walked in order, wave-uniform, SEG_BATCH
// gathered rows in flight at a time (lane = 16-byte chunk of the pooled part); each run's sum is stored where
// the run ends. A run that starts in the window and runs past it is finished from the entries after it;
// entries before the window's first head belong to the previous window's last run. Same sums as walk_run
// (entries in CSR order, separate multiply and add), one wave per 64 entries instead of one per entry.
template <typename T, int VEC>
__device__ __forceinline__ void seg_window(const Feat &f, const Ents &e, int64_t s0) {
    typedef Chunk<T, VEC> C;
    const int lane = threadIdx.x & 63;
    const int64_t i = s0 + lane;
    const bool ok = i < e.n;
    const int32_t d = ok ? e.dst[i] : -1;
    const int32_t sr = ok ? e.src[i] : 0;
    const int32_t wb = ok ? __float_as_int(e.val[i]) : 0;
    const int32_t before = s0 > 0 ? e.dst[s0 - 1] : -1;
    int32_t prev = __shfl_up(d, 1);
    if (lane == 0) prev = before;
    const uint64_t heads = __ballot(d >= 0 && d != prev);
    if (!heads) return;
    const uint64_t bnd = __ballot(d != prev);  // a run, or an empty stretch, starts here
    const int first = __builtin_ctzll(heads);
    for (uint32_t c = lane; c - lane < f.cpool; c += SHPL_WAVE) {
        const bool act = c < f.cpool;
        const T *sc = reinterpret_cast<const T *>(f.src) + f.src_off + (int64_t)c * VEC;
        float acc[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = 0.0f;
        int32_t key = -1;
        for (int j = first; j < SHPL_WAVE; j += SEG_BATCH) {
            typename C::raw_t raw[SEG_BATCH];
#pragma unroll
            for (int u = 0; u < SEG_BATCH; ++u) {
                const int jj = j + u < SHPL_WAVE ? j + u : SHPL_WAVE - 1;
                const int32_t dd = __builtin_amdgcn_readlane(d, jj);
                seg_load<T, VEC>(sc, f.src_stride, __builtin_amdgcn_readlane(sr, jj), act && j + u < SHPL_WAVE && dd >= 0,
                                 raw[u]);
            }
#pragma unroll
            for (int u = 0; u < SEG_BATCH; ++u) {
                const int jj = j + u;
                if (jj < SHPL_WAVE) {
                    const int32_t dd = __builtin_amdgcn_readlane(d, jj);
                    if ((bnd >> jj) & 1) {
                        if (key >= 0 && act) store_pooled<T, VEC>(f, key, c, acc);
#pragma unroll
                        for (int q = 0; q < VEC; ++q) acc[q] = 0.0f;
                        key = dd;
                    }
                    if (dd >= 0) {
                        float x[VEC];
                        C::to_f32(raw[u], x);
                        fma_free_accumulate<VEC>(acc, __int_as_float(__builtin_amdgcn_readlane(wb, jj)), x);
                    }
                }
            }
        }
        if (key < 0) continue;
        // the window's last run: on past the window while the destination stays
        for (int64_t t = s0 + SHPL_WAVE;; t += SEG_CONT) {
            int32_t dd[SEG_CONT], ss[SEG_CONT];
            float ww[SEG_CONT];
            bool in[SEG_CONT];
#pragma unroll
            for (int u = 0; u < SEG_CONT; ++u) {
                const bool okk = t + u < e.n;
                dd[u] = okk ? e.dst[t + u] : -1;
                ss[u] = okk ? e.src[t + u] : 0;
                ww[u] = okk ? e.val[t + u] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < SEG_CONT; ++u) in[u] = dd[u] == key && (u == 0 || in[u - 1]);
            typename C::raw_t raw[SEG_CONT];
#pragma unroll
            for (int u = 0; u < SEG_CONT; ++u) seg_load<T, VEC>(sc, f.src_stride, ss[u], act && in[u], raw[u]);
#pragma unroll
            for (int u = 0; u < SEG_CONT; ++u) {
                if (in[u]) {
                    float x[VEC];
                    C::to_f32(raw[u], x);
                    fma_free_accumulate<VEC>(acc, ww[u], x);
                }
            }
            if (!in[SEG_CONT - 1]) break;
        }
        if (act) store_pooled<T, VEC>(f, key, c, acc);
    }
}

#ifndef SHPL_ONCE_WPE
#define SHPL_ONCE_WPE 5  // k_once at 5 waves per SIMD: the zero rows' write-only stream and the window walks
#endif
template <typename T, int VEC, bool GROUP, bool POW2>
__global__ __launch_bounds__(SHPL_BLOCK)
#if SHPL_ONCE_WPE
__attribute__((amdgpu_waves_per_eu(SHPL_ONCE_WPE, SHPL_ONCE_WPE)))
#endif
void k_once(const Feat f, const Ents e, int cpool_shift,
                                                     const int32_t *key_range, int64_t n_rows, int64_t sblocks) {
    const int64_t zblocks = (int64_t)gridDim.x - sblocks;
    const int64_t zb = SHPL_ONCE_ZERO_FIRST ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - sblocks;
    if (zb < 0 || zb >= zblocks) {
        int64_t sb = SHPL_ONCE_ZERO_FIRST ? zb - zblocks : (int64_t)blockIdx.x;
#if SHPL_ONCE_XCD
        // workgroups go to the 8 XCDs round-robin by id: sb % 8 picks the XCD, so each XCD walks a contiguous
        // eighth of the entries in order and the image rows its neighbouring destinations share stay in its
        // own L2 (the launcher makes sblocks a multiple of 8)
        sb = (sb & 7) * (sblocks >> 3) + (sb >> 3);
#endif
        if (once_seg(GROUP, f.cpool)) {
            const int64_t wpb = SHPL_BLOCK / SHPL_WAVE;
            for (int64_t win = sb * wpb + (threadIdx.x >> 6); win * SHPL_WAVE < e.n; win += sblocks * wpb)
                seg_window<T, VEC>(f, e, win * SHPL_WAVE);
        } else {
            sparse_body<T, VEC, GROUP, false, POW2, false>(f, e, cpool_shift, sb, sblocks);
        }
        return;
    }
    typedef Chunk<T, VEC> C;
    const int lane = threadIdx.x & 63;
    const int64_t row0 = (zb * (SHPL_BLOCK / SHPL_WAVE) + (threadIdx.x >> 6)) * ONCE_ROWS;
    bool empty = false;
    if (lane < ONCE_ROWS && row0 + lane < n_rows) {
        const int2 kr = *reinterpret_cast<const int2 *>(key_range + 2 * (row0 + lane));
        empty = kr.x == kr.y;
    }
    const uint64_t mask = __ballot(empty);
    if (!mask) return;
    T *out = reinterpret_cast<T *>(f.out);
    const uint32_t cp = f.cpool, n = ONCE_ROWS * cp;
    for (uint32_t q = lane; q < n; q += SHPL_WAVE) {
        const uint32_t r = POW2 ? q >> cpool_shift : q / cp;
        const uint32_t c = q - r * cp;
        if ((mask >> r) & 1) C::store_nt(out + ((row0 + r) * f.out_stride + (int64_t)c * VEC), C::zero());
    }
}

// The runs longer than LONG_RUN. Each workgroup lists the long runs that
// start among its LONG_SLOTS entry slots and stages, in one round trip, the
// index words (dst, src, val, col) of the LONG_IDX entries from its first
// long run on; its threads then take (run, chunk) pairs in parallel and walk
// them LONG_WALK entries per step with the index read from LDS (global past
// the staged range), so a step costs one feature round trip. (Measured and
// dropped: staging the feature rows of one run at a time in LDS -- the runs
// of a workgroup then go in series; at config 3 a quarter of the pixel runs
// are long.)
constexpr int LONG_IDX = 512;
constexpr int LONG_SLOTS = 64;  // entry slots per workgroup when the grid is not capped: few runs each
constexpr int LONG_GRID = 2048; // workgroups of k_sparse_long at most (config 2: ~625 slots each)
template <typename T, int VEC, bool GROUP>
__global__ __launch_bounds__(SHPL_BLOCK) void k_sparse_long(const Feat f, const Ents e, int64_t per_block) {
    typedef Chunk<T, VEC> C;
    __shared__ int32_t s_run[SHPL_BLOCK];
    __shared__ int32_t s_dst[LONG_IDX], s_src[LONG_IDX], s_col[GROUP ? LONG_IDX : 1];
    __shared__ float s_val[LONG_IDX];
    __shared__ int s_n, s_first;
    const int64_t nnz = e.n;
    const int64_t r_end = (int64_t)(blockIdx.x + 1) * per_block < nnz ? (int64_t)(blockIdx.x + 1) * per_block : nnz;
    const T *sc0 = reinterpret_cast<const T *>(f.src) + f.src_off;
    // the block's slots, up to SHPL_BLOCK per round (uniform trip count)
    const int64_t span = per_block < SHPL_BLOCK ? per_block : SHPL_BLOCK;
    for (int64_t blk = (int64_t)blockIdx.x * per_block; blk < r_end; blk += span) {
        if (threadIdx.x == 0) {
            s_n = 0;
            s_first = SHPL_BLOCK;
        }
        __syncthreads();
        if ((int64_t)threadIdx.x < span) {
            const int64_t s = blk + threadIdx.x;
            if (s < r_end) {
                const int32_t key = e.dst[s];
                const int32_t prev = s > 0 ? e.dst[s - 1] : -1;
                const int32_t ahead = s + LONG_RUN < nnz ? e.dst[s + LONG_RUN] : -1;
                if (key >= 0 && prev != key && ahead == key) {
                    s_run[atomicAdd(&s_n, 1)] = (int32_t)threadIdx.x;
                    atomicMin(&s_first, (int)threadIdx.x);
                }
            }
        }
        __syncthreads();
        const int n_run = s_n;
        if (n_run == 0) continue;  // uniform
        const int64_t base = blk + s_first;
        for (int j = threadIdx.x; j < LONG_IDX; j += SHPL_BLOCK) {
            const int64_t i = base + j;
            const bool ok = i < nnz;
            s_dst[j] = ok ? e.dst[i] : -1;
            s_src[j] = ok ? e.src[i] : 0;
            s_val[j] = ok ? e.val[i] : 0.0f;
            if (GROUP) s_col[j] = ok ? e.col[i] : 0;
        }
        __syncthreads();
        for (int p = threadIdx.x; p < n_run * (int)f.cpool; p += SHPL_BLOCK) {
            const int r = p / (int)f.cpool;
            const uint32_t c = (uint32_t)(p - r * (int)f.cpool);
            const int64_t s0 = blk + s_run[r];
            const T *sc = sc0 + (int64_t)c * VEC;
            const int32_t key = s_dst[s0 - base];
            float acc[VEC], q[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] = q[j] = 0.0f;
            int32_t kprev = -1;
            for (int64_t i = s0;; i += LONG_WALK) {
                bool in[LONG_WALK];
                int32_t sr[LONG_WALK], kc[LONG_WALK];
                float w[LONG_WALK];
#pragma unroll
                for (int u = 0; u < LONG_WALK; ++u) {
                    const int64_t x = i + u, j = x - base;
                    int32_t d;
                    if (j < LONG_IDX) {
                        d = s_dst[j];
                        sr[u] = s_src[j];
                        w[u] = s_val[j];
                        kc[u] = GROUP ? s_col[j] : 0;
                    } else {
                        const bool ok = x < nnz;
                        d = ok ? e.dst[x] : -1;
                        sr[u] = ok ? e.src[x] : 0;
                        w[u] = ok ? e.val[x] : 0.0f;
                        kc[u] = (GROUP && ok) ? e.col[x] : 0;
                    }
                    in[u] = d == key && (u == 0 || in[u - 1]);
                }
                typename C::raw_t raw[LONG_WALK];
#pragma unroll
                for (int u = 0; u < LONG_WALK; ++u)
                    if (in[u]) raw[u] = C::load(sc + (int64_t)sr[u] * f.src_stride);
#pragma unroll
                for (int u = 0; u < LONG_WALK; ++u) {
                    if (!in[u]) break;
                    float x[VEC];
                    C::to_f32(raw[u], x);
                    if (GROUP) {
                        // TF: Q[k] = sum of column k's entries; out = 0 + Q[k1] + Q[k2] ... (ScatterNd order)
                        if (kc[u] != kprev) {
#pragma unroll
                            for (int j = 0; j < VEC; ++j) {
                                acc[j] = __fadd_rn(acc[j], q[j]);
                                q[j] = 0.0f;
                            }
                            kprev = kc[u];
                        }
                        fma_free_accumulate<VEC>(q, w[u], x);
                    } else {
                        fma_free_accumulate<VEC>(acc, w[u], x);
                    }
                }
                if (!in[LONG_WALK - 1]) break;
            }
            if (GROUP) {
#pragma unroll
                for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], q[j]);
            }
            store_pooled<T, VEC>(f, key, c, acc);
        }
        __syncthreads();  // s_run / s_dst are refilled for the next slots
    }
}

// ---------------------------------------------------------------- k_rows
// The whole pull in ONE launch keyed by output row, for CSRs that carry
// key_range (small, latency-bound layers: config 3). A group of G lanes owns a
// row (64 / G rows per wave): lane g copies pass-through chunks g, g+G, ...
// and sums pooled chunks g, g+G, ... over the row's run [first, end) in TF
// order. The run's index words are loaded G at a time, one entry per lane,
// and handed to the group's lanes by shuffles; ROWS_WALK feature rows are in
// flight per step (8: ~90 VGPRs, 5 waves per SIMD -- rows in flight matter
// more than entries in flight when the average run is ~3 entries). The first
// pass-through chunk and the ADD operand are loaded with the row's range, so
// their latency overlaps the index loads. Trip counts are wave-uniform (the
// longest run of the wave's rows), so the shuffles always see every lane.
// Arithmetic is k_sparse's: bitwise the same output as k_dense + k_sparse.
#ifndef SHPL_ROWS_WALK
#define SHPL_ROWS_WALK 8
#endif
constexpr int ROWS_WALK = SHPL_ROWS_WALK;
#ifndef SHPL_RPROBE
// timing probes of the row walk: 1 every gather from the first 64 rows, 2 no stores (wrong results); 3 each
// k_rows2 wave's start / end s_memrealtime stamps into g_probe (read by shpl_probe_stamps)
#define SHPL_RPROBE 0
#endif
#if SHPL_RPROBE == 3
constexpr int64_t PROBE_WAVES = 1 << 16;
__device__ uint64_t g_probe[2 * PROBE_WAVES];
#endif

// The walk of one row's run [first, end) (all lanes of the wave, wave-uniform trip counts); pv / av: the
// lane's first pass-through chunk (CONCAT, when p0) and first ADD operand, loaded by the caller.
// MODE: the output mode at compile time (SHPL_OUT_*), or -1: f.mode at run time.
template <typename T, int VEC, bool GROUP, int G, int MODE = -1>
__device__ __forceinline__ void row_walk(const Feat &f, const Ents &e, int64_t row, bool live, int32_t first,
                                         int32_t end, bool p0, typename Chunk<T, VEC>::raw_t pv,
                                         typename Chunk<T, VEC>::raw_t av, int2 head = int2{0, 0},
                                         bool has_head = false) {
    typedef Chunk<T, VEC> C;
    const int lane = threadIdx.x & 63, lg = lane & (G - 1), gbase = lane & ~(G - 1);
    T *out = reinterpret_cast<T *>(f.out);
    const T *pass = reinterpret_cast<const T *>(f.pass) + f.pass_off;
    const T *src = reinterpret_cast<const T *>(f.src) + f.src_off;
    const int mode = MODE >= 0 ? MODE : f.mode;
    const bool concat = mode == SHPL_OUT_CONCAT, add = mode == SHPL_OUT_ADD;
    const uint32_t oc0 = concat ? f.cpass : 0u;
    const int32_t len = end - first;
    int32_t wlen = len;  // longest run among the wave's rows: the walk's trip count
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wlen = max(wlen, __shfl_xor(wlen, o, 64));
    if (p0) C::store_nt(out + (row * f.out_stride + (int64_t)lg * VEC), pv);
    if (live && concat)
        for (uint32_t c = lg + G; c < f.cpass; c += G)
            C::store_nt(out + (row * f.out_stride + (int64_t)c * VEC),
                        C::load_nt(pass + (row * f.pass_stride + (int64_t)c * VEC)));
    for (uint32_t pc0 = 0; pc0 < f.cpool; pc0 += G) {
        const uint32_t pc = pc0 + lg;
        const bool mine = live && pc < f.cpool;
        float acc[VEC], q[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = q[j] = 0.0f;
        int32_t kprev = -1;
        for (int32_t j0 = 0; j0 < wlen; j0 += G) {
            // index words of entries first + j0 + lg of this lane's row (the first ones from the run heads,
            // already in registers, when the CSR carries them)
            const bool has = j0 + lg < len;
            const bool from_head = has_head && j0 == 0;
            const int32_t my_src = !has ? 0 : from_head ? head.x : e.src[first + j0 + lg];
            const float my_val = !has ? 0.0f : from_head ? __int_as_float(head.y) : e.val[first + j0 + lg];
            const int32_t my_col = (GROUP && has) ? e.col[first + j0 + lg] : 0;
            const int32_t n = min(G, wlen - j0);
            for (int32_t u0 = 0; u0 < n; u0 += ROWS_WALK) {
                typename C::raw_t raw[ROWS_WALK];
#pragma unroll
                for (int u = 0; u < ROWS_WALK; ++u) {
                    const int32_t sr = __shfl(my_src, gbase + ((u0 + u) & (G - 1)), 64);
                    if (mine && j0 + u0 + u < len && u0 + u < G)
                        raw[u] = C::load(src + ((int64_t)(SHPL_RPROBE == 1 ? (sr & 63) : sr) * f.src_stride + (int64_t)pc * VEC));
                }
#pragma unroll
                for (int u = 0; u < ROWS_WALK; ++u) {
                    const int srcl = gbase + ((u0 + u) & (G - 1));
                    const float w = __shfl(my_val, srcl, 64);
                    const int32_t kc = GROUP ? __shfl(my_col, srcl, 64) : 0;
                    if (!(mine && j0 + u0 + u < len && u0 + u < G)) continue;
                    float x[VEC];
                    C::to_f32(raw[u], x);
                    if (GROUP) {
                        // TF: Q[k] = sum of column k's entries; out = 0 + Q[k1] + Q[k2] ... (ScatterNd order)
                        if (kc != kprev) {
#pragma unroll
                            for (int j = 0; j < VEC; ++j) {
                                acc[j] = __fadd_rn(acc[j], q[j]);
                                q[j] = 0.0f;
                            }
                            kprev = kc;
                        }
                        fma_free_accumulate<VEC>(q, w, x);
                    } else {
                        fma_free_accumulate<VEC>(acc, w, x);
                    }
                }
            }
        }
        if (!mine) continue;
        if (GROUP) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(acc[j], q[j]);
        }
        if (add) {
            // pass + pooled (pass + 0.0f for an empty row: k_dense's -0 -> +0)
            float a[VEC];
            C::to_f32(pc0 == 0 ? av : C::load(pass + (row * f.pass_stride + (int64_t)pc * VEC)), a);
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] = __fadd_rn(a[j], acc[j]);
        } else if (len == 0) {
            C::store_nt(out + (row * f.out_stride + (int64_t)(oc0 + pc) * VEC), C::zero());
            continue;
        }
        if (SHPL_RPROBE == 2) {  // timing probe: no pooled stores (wrong results)
            if (acc[0] == 1234.5f) C::store_nt(out, C::from_f32(acc));
            continue;
        }
        C::store_nt(out + (row * f.out_stride + (int64_t)(oc0 + pc) * VEC), C::from_f32(acc));
    }
}

// Rows [row0 + blk * rows per block, ...) of a pull, those below row_end live.
template <typename T, int VEC, bool GROUP, int G, int MODE = -1>
__device__ __forceinline__ void rows_body(const Feat &f, const Ents &e, const int32_t *key_range, int64_t row0,
                                          int64_t row_end, int64_t blk) {
    typedef Chunk<T, VEC> C;
    constexpr int RPW = SHPL_WAVE / G;
    const int lane = threadIdx.x & 63, lg = lane & (G - 1);
    const int64_t row = row0 + (blk * (SHPL_BLOCK / SHPL_WAVE) + (threadIdx.x >> 6)) * RPW + lane / G;
    const bool live = row < row_end;
    const T *pass = reinterpret_cast<const T *>(f.pass) + f.pass_off;
    // the row's range, its first pass-through chunk and its first ADD operand: one round trip
    int32_t first = 0, end = 0;
    typename C::raw_t pv = C::zero(), av = C::zero();
    const int mode = MODE >= 0 ? MODE : f.mode;
    const bool p0 = live && mode == SHPL_OUT_CONCAT && (uint32_t)lg < f.cpass;
    const bool a0 = live && mode == SHPL_OUT_ADD && (uint32_t)lg < f.cpool;
    if (live) {
        first = key_range[2 * row];
        end = key_range[2 * row + 1];
    }
    // the run's first head_k entries from the run heads, in the same round trip (lanes past head_k, and
    // entries past it, read the CSR arrays in row_walk)
    const bool has_head = !GROUP && e.heads != nullptr && lg < e.head_k;
    int2 head = int2{0, 0};
    if (live && has_head) head = e.heads[row * e.head_k + lg];
    if (p0) pv = C::load_nt(pass + (row * f.pass_stride + (int64_t)lg * VEC));
    if (a0) av = C::load(pass + (row * f.pass_stride + (int64_t)lg * VEC));
    row_walk<T, VEC, GROUP, G, MODE>(f, e, row, live, first, end, p0, pv, av, head, has_head);
}

template <typename T, int VEC, bool GROUP, int G>
__global__ __launch_bounds__(SHPL_BLOCK) void k_rows(const Feat f, const Ents e, const int32_t *key_range,
                                                     int64_t n_rows) {
    rows_body<T, VEC, GROUP, G>(f, e, key_range, 0, n_rows, blockIdx.x);
}

// Two row-keyed pulls in ONE launch (shpl_pull_pair): s0 the first pull (no per-column partials: the
// cell-keyed one), s1 the second (with them: the pixel-keyed one) -- k_rows each.
struct RowsSide {
    Feat f;
    Ents e;
    const int32_t *key_range;
    int64_t n_rows, blocks;
};

// The pixel-keyed pull's blocks come first: its longer runs (6.7 entries on average at config 3, up to 54 at
// the horizon) then start early instead of forming the launch's tail (k_rows2 31.1 -> 24.0 us per pair,
// profiles/r03_pixel_first_ab.log; reversing the order inside either side measured within noise).
#ifndef SHPL_ROWS2_WPE
#define SHPL_ROWS2_WPE 0
#endif
template <typename T, int VEC, int G, bool GR1, int MODE>
__global__ __launch_bounds__(SHPL_BLOCK)
#if SHPL_ROWS2_WPE
__attribute__((amdgpu_waves_per_eu(SHPL_ROWS2_WPE, SHPL_ROWS2_WPE)))
#endif
void k_rows2(const RowsSide s0, const RowsSide s1) {
#if SHPL_RPROBE == 3
    uint64_t t0;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
#endif
    if ((int64_t)blockIdx.x < s1.blocks)
        rows_body<T, VEC, GR1, G, MODE>(s1.f, s1.e, s1.key_range, 0, s1.n_rows, (int64_t)blockIdx.x);
    else
        rows_body<T, VEC, false, G, MODE>(s0.f, s0.e, s0.key_range, 0, s0.n_rows, (int64_t)blockIdx.x - s1.blocks);
#if SHPL_RPROBE == 3
    uint64_t t1;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    const int64_t w = (int64_t)blockIdx.x * (SHPL_BLOCK / SHPL_WAVE) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && w < PROBE_WAVES) {
        g_probe[2 * w] = t0;
        g_probe[2 * w + 1] = t1;
    }
#endif
}

bool aligned(const void *ptr, int64_t a) { return ((uintptr_t)ptr) % (uintptr_t)a == 0; }

struct Plan {
    Feat f = {};
    int64_t n_dst;
    bool v16;
    int dtype;
};

int plan(int direction, int dtype, const shpl_csr *csr, const void *d_src, int64_t src_stride, int64_t src_off,
         int64_t c_pool, const void *d_pass, int64_t pass_stride, int64_t pass_off, int64_t c_pass, int mode,
         void *d_out, int64_t out_stride, Plan *pl) {
    if (!csr) return SHPL_ERR_ARG;
    if (direction != SHPL_BY_CELL && direction != SHPL_BY_PIXEL) return SHPL_ERR_ARG;
    if (dtype != SHPL_F32 && dtype != SHPL_BF16) return SHPL_ERR_ARG;
    if (mode < SHPL_OUT_POOL || mode > SHPL_OUT_ADD) return SHPL_ERR_ARG;
    const int64_t n_dst = csr->n_keys;
    if (n_dst < 0 || n_dst >= 2147483647LL || c_pool < 0 || c_pass < 0) return SHPL_ERR_BAD_SHAPE;
    if (n_dst > 0 && (!d_out || (c_pool > 0 && !d_src))) return SHPL_ERR_ARG;
    if (csr->nnz_cap > 0 && (!csr->ent_dst || !csr->ent_src || !csr->ent_val)) return SHPL_ERR_ARG;
    // a pixel-keyed CSR sums per-column partials (TF's Q[k]) unless it is marked as one column per entry
    if (direction == SHPL_BY_PIXEL && csr->nnz_cap > 0 && !csr->ent_col && !(csr->flags & SHPL_CSR_IDENTITY_COLS))
        return SHPL_ERR_ARG;
    if (mode != SHPL_OUT_POOL && !d_pass) return SHPL_ERR_ARG;
    if (mode == SHPL_OUT_ADD && c_pass != c_pool) return SHPL_ERR_BAD_SHAPE;
    if (csr->heads && (csr->head_k < 1 || csr->head_k > SHPL_CSR_MAX_HEAD || !csr->key_range)) return SHPL_ERR_ARG;
    const int64_t width = mode == SHPL_OUT_CONCAT ? c_pass + c_pool : c_pool;
    if (out_stride < width || (c_pool > 0 && src_stride < src_off + c_pool) ||
        (mode != SHPL_OUT_POOL && pass_stride < pass_off + c_pass))
        return SHPL_ERR_BAD_SHAPE;
    const int64_t row_max = (int64_t)1 << 31;  // row widths index in 32 bits (k_dense)
    if (out_stride >= row_max || src_stride >= row_max || pass_stride >= row_max) return SHPL_ERR_BAD_SHAPE;
    const int64_t esz = dtype == SHPL_F32 ? 4 : 2;
    const int64_t vec = 16 / esz;
    // 16-byte chunks need every row start and every channel split on a 16-byte boundary
    bool v16 = c_pool % vec == 0 && out_stride % vec == 0 && aligned(d_out, 16);
    if (c_pool > 0) v16 = v16 && src_stride % vec == 0 && src_off % vec == 0 && aligned(d_src, 16);
    if (mode != SHPL_OUT_POOL)
        v16 = v16 && c_pass % vec == 0 && pass_stride % vec == 0 && pass_off % vec == 0 && aligned(d_pass, 16);
    const int64_t v = v16 ? vec : 1;
    Feat &f = pl->f;
    f.src = d_src;
    f.src_stride = src_stride;
    f.src_off = src_off;
    f.pass = d_pass;
    f.pass_stride = pass_stride;
    f.pass_off = pass_off;
    f.out = d_out;
    f.out_stride = out_stride;
    f.mode = mode;
    f.cpr = (uint32_t)(width / v);
    f.cpass = mode == SHPL_OUT_CONCAT ? (uint32_t)(c_pass / v) : 0u;
    f.cpool = (uint32_t)(c_pool / v);
    f.cpr_shift = -1;
    for (int k = 0; k < 31; ++k)
        if (f.cpr == (1u << k)) f.cpr_shift = k;
    pl->n_dst = n_dst;
    pl->v16 = v16;
    pl->dtype = dtype;
    return SHPL_OK;
}

template <typename T, int VEC>
int dense_t(const Plan &pl, hipStream_t s) {
    if (pl.f.cpr == 0) return SHPL_OK;
    // u32 chunk index per launch: at most 2^31 chunks each
    const int64_t rows_per_launch = ((int64_t)1 << 31) / (int64_t)pl.f.cpr;
    for (int64_t r0 = 0; r0 < pl.n_dst; r0 += rows_per_launch) {
        const int64_t nr = (pl.n_dst - r0) < rows_per_launch ? (pl.n_dst - r0) : rows_per_launch;
        const int64_t blocks = (nr * pl.f.cpr + SHPL_BLOCK - 1) / SHPL_BLOCK;
        if (pl.f.cpr_shift >= 0)
            hipLaunchKernelGGL((k_dense<T, VEC, true>), dim3((unsigned)blocks), dim3(SHPL_BLOCK), 0, s, pl.f,
                               (uint32_t)r0, (uint32_t)nr);
        else
            hipLaunchKernelGGL((k_dense<T, VEC, false>), dim3((unsigned)blocks), dim3(SHPL_BLOCK), 0, s, pl.f,
                               (uint32_t)r0, (uint32_t)nr);
        SHPL_LAUNCH_CHECK();
    }
    return SHPL_OK;
}

int dense(const Plan &pl, hipStream_t s) {
    if (pl.n_dst == 0) return SHPL_OK;
    if (pl.dtype == SHPL_F32) return pl.v16 ? dense_t<float, 4>(pl, s) : dense_t<float, 1>(pl, s);
    return pl.v16 ? dense_t<uint16_t, 8>(pl, s) : dense_t<uint16_t, 1>(pl, s);
}

#ifndef SHPL_LIVE_GRID
#define SHPL_LIVE_GRID 4096  // workgroups of the live-entry k_sparse at most (a grid-stride loop)
#endif

template <typename T, int VEC, bool GROUP, bool LIVE>
void sparse_launch(const Plan &pl, const Ents &e, int grid, int shift, bool split, hipStream_t s) {
#define SHPL_SPARSE(SPLIT, POW2)                                                                                   \
    hipLaunchKernelGGL((k_sparse<T, VEC, GROUP, SPLIT, POW2, LIVE>), dim3(grid), dim3(SHPL_BLOCK), 0, s, pl.f, e, \
                       shift)
    if (split) {
        if (shift >= 0) SHPL_SPARSE(true, true); else SHPL_SPARSE(true, false);
    } else {
        if (shift >= 0) SHPL_SPARSE(false, true); else SHPL_SPARSE(false, false);
    }
#undef SHPL_SPARSE
}

template <typename T, int VEC, bool GROUP>
int sparse_tg(const Plan &pl, const Ents &e, int64_t nnz_cap, hipStream_t s) {
    // one thread per (entry, chunk) of the capacity (the live count is read on the device), or, with a
    // frame layout, a bounded grid walking the live entries' (entry, chunk) pairs
    const bool live = e.n_frames > 0;
    int grid = grid_for(nnz_cap * (int64_t)pl.f.cpool, SHPL_BLOCK, 1 << 20);
    if (live && grid > SHPL_LIVE_GRID) grid = SHPL_LIVE_GRID;
    int shift = -1;
    for (int k = 0; k < 31; ++k)
        if (pl.f.cpool == (1u << k)) shift = k;
    // without a run longer than LONG_RUN possible, k_sparse takes every run (the short part); so it does
    // over live entries (raw scans: runs of at most a few voxel points per cell -- k_sparse_long would only
    // scan the capacity)
    const bool split = !live && nnz_cap > LONG_RUN;
    if (live)
        sparse_launch<T, VEC, GROUP, true>(pl, e, grid, shift, split, s);
    else
        sparse_launch<T, VEC, GROUP, false>(pl, e, grid, shift, split, s);
    SHPL_LAUNCH_CHECK();
    if (!split) return SHPL_OK;
    // a bounded grid: each workgroup scans per_block slots, LONG_SLOTS at a time
    int64_t lgrid = (nnz_cap + LONG_SLOTS - 1) / LONG_SLOTS;
    if (lgrid > LONG_GRID) lgrid = LONG_GRID;
    const int64_t per_block = (nnz_cap + lgrid - 1) / lgrid;
    hipLaunchKernelGGL((k_sparse_long<T, VEC, GROUP>), dim3((unsigned)lgrid), dim3(SHPL_BLOCK), 0, s, pl.f, e,
                       per_block);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

template <typename T, int VEC, bool GROUP>
int once_tg(const Plan &pl, const shpl_csr *csr, hipStream_t s) {
    Ents e{csr->nnz_cap, csr->ent_dst, csr->ent_src, csr->ent_col, csr->ent_val};
    // the run-walking blocks: a thread per (entry, chunk), or (cell-keyed) a wave per 64 entries
    const int64_t swork = once_seg(GROUP, pl.f.cpool) ? csr->nnz_cap : csr->nnz_cap * (int64_t)pl.f.cpool;
    int64_t sblocks = csr->nnz_cap > 0 ? grid_for(swork, SHPL_BLOCK, 1 << 20) : 0;
    if (SHPL_ONCE_XCD) sblocks = (sblocks + 7) & ~(int64_t)7;  // k_once's XCD-contiguous block order
    const int64_t zblocks = (pl.n_dst + ONCE_ROWS * (SHPL_BLOCK / SHPL_WAVE) - 1) / (ONCE_ROWS * (SHPL_BLOCK / SHPL_WAVE));
    if (sblocks + zblocks > 0x7fffffffLL) return SHPL_ERR_BAD_SHAPE;
    int shift = -1;
    for (int k = 0; k < 31; ++k)
        if (pl.f.cpool == (1u << k)) shift = k;
    if (shift >= 0)
        hipLaunchKernelGGL((k_once<T, VEC, GROUP, true>), dim3((unsigned)(sblocks + zblocks)), dim3(SHPL_BLOCK), 0, s,
                           pl.f, e, shift, (const int32_t *)csr->key_range, pl.n_dst, sblocks);
    else
        hipLaunchKernelGGL((k_once<T, VEC, GROUP, false>), dim3((unsigned)(sblocks + zblocks)), dim3(SHPL_BLOCK), 0,
                           s, pl.f, e, shift, (const int32_t *)csr->key_range, pl.n_dst, sblocks);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

template <typename T, int VEC>
int once_t(const Plan &pl, const shpl_csr *csr, bool group, hipStream_t s) {
    return group ? once_tg<T, VEC, true>(pl, csr, s) : once_tg<T, VEC, false>(pl, csr, s);
}

template <typename T, int VEC>
int sparse_t(const Plan &pl, const shpl_csr *csr, bool group, hipStream_t s) {
    const bool live = csr->n_frames > 0 && csr->frame_off && csr->frame_nnz;
    Ents e{csr->nnz_cap, csr->ent_dst, csr->ent_src, csr->ent_col, csr->ent_val,
           live ? csr->frame_off : nullptr, live ? csr->frame_nnz : nullptr, live ? (int)csr->n_frames : 0};
    return group ? sparse_tg<T, VEC, true>(pl, e, csr->nnz_cap, s)
                 : sparse_tg<T, VEC, false>(pl, e, csr->nnz_cap, s);
}

// Per-column partials (TF's Q[k]) only where columns can repeat: a pixel-keyed CSR without ent_col has every
// entry in a column of its own (the index builder's maps), where Q[k] is one product and the plain sum is
// bitwise the same (0 + p differs from p only for p = -0, and an accumulator that starts at +0 never becomes
// -0, so adding +0 or -0 to it gives the same bits).
bool grouped(const shpl_csr *csr, int direction) { return direction == SHPL_BY_PIXEL && csr->ent_col != nullptr; }

int sparse(const Plan &pl, const shpl_csr *csr, int direction, hipStream_t s) {
    if (pl.n_dst == 0 || pl.f.cpool == 0 || csr->nnz_cap == 0) return SHPL_OK;
    if (csr->n_frames < 0 || csr->n_frames > LIVE_MAX_FRAMES) return SHPL_ERR_ARG;
    const bool group = grouped(csr, direction);
    if (pl.dtype == SHPL_F32)
        return pl.v16 ? sparse_t<float, 4>(pl, csr, group, s) : sparse_t<float, 1>(pl, csr, group, s);
    return pl.v16 ? sparse_t<uint16_t, 8>(pl, csr, group, s) : sparse_t<uint16_t, 1>(pl, csr, group, s);
}

template <typename T, int VEC, bool GROUP>
int rows_t(const Plan &pl, const shpl_csr *csr, hipStream_t s) {
    Ents e{csr->nnz_cap, csr->ent_dst, csr->ent_src, csr->ent_col, csr->ent_val};
    e.heads = (const int2 *)csr->heads;
    e.head_k = (int)csr->head_k;
    // lanes per row: the pooled chunks of a row, at least 8 (index words come G at a time), at most a wave
    int G = 8;
    while (G < 64 && (uint32_t)G < pl.f.cpool) G <<= 1;
    const int64_t rows_per_block = (int64_t)(SHPL_BLOCK / G);
    const int64_t blocks = (pl.n_dst + rows_per_block - 1) / rows_per_block;
    if (blocks > 0x7fffffffLL) return SHPL_ERR_BAD_SHAPE;
#define SHPL_ROWS(GG) \
    hipLaunchKernelGGL((k_rows<T, VEC, GROUP, GG>), dim3((unsigned)blocks), dim3(SHPL_BLOCK), 0, s, pl.f, e, \
                       (const int32_t *)csr->key_range, pl.n_dst)
    switch (G) {
        case 8: SHPL_ROWS(8); break;
        case 16: SHPL_ROWS(16); break;
        case 32: SHPL_ROWS(32); break;
        default: SHPL_ROWS(64); break;
    }
#undef SHPL_ROWS
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

template <typename T, int VEC>
int rows_tv(const Plan &pl, const shpl_csr *csr, bool group, hipStream_t s) {
    return group ? rows_t<T, VEC, true>(pl, csr, s) : rows_t<T, VEC, false>(pl, csr, s);
}

int rows(const Plan &pl, const shpl_csr *csr, int direction, hipStream_t s) {
    if (pl.n_dst == 0) return SHPL_OK;
    const bool group = grouped(csr, direction);
    if (pl.dtype == SHPL_F32)
        return pl.v16 ? rows_tv<float, 4>(pl, csr, group, s) : rows_tv<float, 1>(pl, csr, group, s);
    return pl.v16 ? rows_tv<uint16_t, 8>(pl, csr, group, s) : rows_tv<uint16_t, 1>(pl, csr, group, s);
}

}  // namespace
}  // namespace shpl

using namespace shpl;

#define SHPL_PULL_ARGS                                                                                           \
    int direction, int dtype, const shpl_csr *csr, const void *d_src, int64_t src_stride, int64_t src_off,       \
        int64_t c_pool, const void *d_pass, int64_t pass_stride, int64_t pass_off, int64_t c_pass, int mode,     \
        void *d_out, int64_t out_stride, void *stream
#define SHPL_PLAN()                                                                                              \
    Plan pl;                                                                                                     \
    int rc = plan(direction, dtype, csr, d_src, src_stride, src_off, c_pool, d_pass, pass_stride, pass_off,      \
                  c_pass, mode, d_out, out_stride, &pl);                                                         \
    if (rc) return rc;

extern "C" int shpl_pull(SHPL_PULL_ARGS) {
    SHPL_PLAN();
    // row-keyed form only over a built CSR: an empty map (nnz_cap == 0) has no sorted entries and
    // shpl_build_csr leaves nothing for k_rows to walk -- the streaming pass alone is the whole pull
    if (csr->key_range && csr->nnz_cap > 0) return rows(pl, csr, direction, (hipStream_t)stream);
    rc = dense(pl, (hipStream_t)stream);
    if (rc) return rc;
    return sparse(pl, csr, direction, (hipStream_t)stream);
}

extern "C" int shpl_pull_dense(SHPL_PULL_ARGS) {
    SHPL_PLAN();
    return dense(pl, (hipStream_t)stream);
}

extern "C" int shpl_pull_sparse(SHPL_PULL_ARGS) {
    SHPL_PLAN();
    return sparse(pl, csr, direction, (hipStream_t)stream);
}

extern "C" int shpl_pull_once(SHPL_PULL_ARGS) {
    SHPL_PLAN();
    if (mode != SHPL_OUT_POOL || !csr->key_range) return SHPL_ERR_ARG;
    if (pl.n_dst == 0 || pl.f.cpool == 0) return SHPL_OK;
    const bool group = grouped(csr, direction);
    hipStream_t s = (hipStream_t)stream;
    if (pl.dtype == SHPL_F32)
        return pl.v16 ? once_t<float, 4>(pl, csr, group, s) : once_t<float, 1>(pl, csr, group, s);
    return pl.v16 ? once_t<uint16_t, 8>(pl, csr, group, s) : once_t<uint16_t, 1>(pl, csr, group, s);
}

// ---------------------------------------------------------------- paired pulls
namespace shpl {
namespace {

template <typename T, int VEC>
int pair_t(RowsSide s[2], int G, hipStream_t st) {
    const int rpb = SHPL_BLOCK / G;
    for (int k = 0; k < 2; ++k)
        if (s[k].n_rows > 0) s[k].blocks = (s[k].n_rows + rpb - 1) / rpb;
    const int64_t blocks = s[0].blocks + s[1].blocks;
    if (blocks == 0) return SHPL_OK;
    if (blocks > 0x7fffffffLL) return SHPL_ERR_BAD_SHAPE;
    const bool gr1 = s[1].e.col != nullptr;  // the pixel-keyed side's per-column partials (grouped())
    // the output mode at compile time when both pulls share it (the forward pair's pooled halves, the gradient
    // pair's add): the other modes' preloaded operands leave the registers (config 3: 78 -> VGPRs below)
    int mode = -1;
    if (s[0].n_rows == 0 || s[1].n_rows == 0 || s[0].f.mode == s[1].f.mode)
        mode = s[0].n_rows ? s[0].f.mode : s[1].f.mode;
#define SHPL_ROWS2_M(GG, GR, M) \
    hipLaunchKernelGGL((k_rows2<T, VEC, GG, GR, M>), dim3((unsigned)blocks), dim3(SHPL_BLOCK), 0, st, s[0], s[1])
#define SHPL_ROWS2_G(GG, GR)                                                  \
    if (mode == SHPL_OUT_POOL) SHPL_ROWS2_M(GG, GR, SHPL_OUT_POOL);          \
    else if (mode == SHPL_OUT_ADD) SHPL_ROWS2_M(GG, GR, SHPL_OUT_ADD);       \
    else if (mode == SHPL_OUT_CONCAT) SHPL_ROWS2_M(GG, GR, SHPL_OUT_CONCAT); \
    else SHPL_ROWS2_M(GG, GR, -1);
#define SHPL_ROWS2(GG)              \
    if (gr1) {                      \
        SHPL_ROWS2_G(GG, true)      \
    } else {                        \
        SHPL_ROWS2_G(GG, false)     \
    }
    switch (G) {
        case 8: SHPL_ROWS2(8); break;
        case 16: SHPL_ROWS2(16); break;
        case 32: SHPL_ROWS2(32); break;
        default: SHPL_ROWS2(64); break;
    }
#undef SHPL_ROWS2
#undef SHPL_ROWS2_G
#undef SHPL_ROWS2_M
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

}  // namespace
}  // namespace shpl

extern "C" int shpl_pull_pair(const shpl_csr *by_cell, const shpl_pull_desc *d_cell, const shpl_csr *by_pixel,
                              const shpl_pull_desc *d_pixel, void *stream) {
    const shpl_csr *cs[2] = {by_cell, by_pixel};
    const shpl_pull_desc *ds[2] = {d_cell, d_pixel};
    hipStream_t st = (hipStream_t)stream;
    Plan pl[2];
    bool on[2] = {false, false};
    for (int k = 0; k < 2; ++k) {
        if (!ds[k]) continue;
        const shpl_csr *c = cs[k];
        if (!c) return SHPL_ERR_ARG;
        if (!c->key_range && c->nnz_cap > 0) return SHPL_ERR_ARG;  // row-keyed: the CSR must carry key_range
        const shpl_pull_desc *d = ds[k];
        const int rc = plan(k ? SHPL_BY_PIXEL : SHPL_BY_CELL, d->dtype, c, d->src, d->src_stride, d->src_off,
                            d->c_pool, d->pass, d->pass_stride, d->pass_off, d->c_pass, d->mode, d->out, d->out_stride,
                            &pl[k]);
        if (rc) return rc;
        on[k] = pl[k].n_dst > 0;
        if (on[k] && c->nnz_cap == 0) {  // an empty map: the streaming pass is the whole pull
            const int r2 = dense(pl[k], st);
            if (r2) return r2;
            on[k] = false;
        }
    }
    if (on[0] && on[1] && (pl[0].dtype != pl[1].dtype || pl[0].v16 != pl[1].v16)) {
        // one template per launch: two launches (shpl_pull's row-keyed form each)
        for (int k = 0; k < 2; ++k) {
            const int rc = rows(pl[k], cs[k], k ? SHPL_BY_PIXEL : SHPL_BY_CELL, st);
            if (rc) return rc;
        }
        return SHPL_OK;
    }
    RowsSide s[2] = {};
    int dtype = -1, v16 = 0, G = 8;
    for (int k = 0; k < 2; ++k) {
        if (!on[k]) continue;
        const shpl_csr *c = cs[k];
        dtype = pl[k].dtype;
        v16 = pl[k].v16;
        while (G < 64 && (uint32_t)G < pl[k].f.cpool) G <<= 1;  // lanes per row: the widest pooled row
        s[k] = RowsSide{pl[k].f, Ents{c->nnz_cap, c->ent_dst, c->ent_src, c->ent_col, c->ent_val}, c->key_range,
                        pl[k].n_dst, 0};
        s[k].e.heads = (const int2 *)c->heads;
        s[k].e.head_k = (int)c->head_k;
    }
    if (dtype < 0) return SHPL_OK;
    if (dtype == SHPL_F32) return v16 ? pair_t<float, 4>(s, G, st) : pair_t<float, 1>(s, G, st);
    return v16 ? pair_t<uint16_t, 8>(s, G, st) : pair_t<uint16_t, 1>(s, G, st);
}

#if SHPL_RPROBE == 3
// probe builds only: the last k_rows2 launch's per-wave (start, end) stamps, 100 MHz ticks
extern "C" int shpl_probe_stamps(uint64_t *host, size_t n_waves) {
    if (n_waves > (size_t)PROBE_WAVES) n_waves = PROBE_WAVES;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_probe), 16 * n_waves, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? SHPL_OK
               : SHPL_ERR_HIP;
}
#endif
