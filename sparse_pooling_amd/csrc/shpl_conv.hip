// shpl_conv.hip -- the post-fusion 3x3 convolution, with
// the SHPL concat (and, optionally, the img->BEV pooling itself) fused into
// its input staging.
//
// Reference (avod/avod/core/models/rpn_model.py:338-355, config switch
// rpn_sparse_pooling_conv_after_fusion, model.proto:88):
//     bv_fused = sparse_pool_layer([bev, img], ...)          # [1,Hb,Wb,Cb+Ci]
//     bev_out  = slim.conv2d(bv_fused, Ci, [3,3], normalizer_fn=slim.batch_norm,
//                            normalizer_params={'is_training': ...})
// i.e. SAME padding, stride 1, no bias, BatchNorm (center, no scale,
// eps 1e-3, decay 0.999), ReLU; and retinanet_model.py:343-348 (conv2d with
// bias + ReLU, no BN). Both epilogues are  y = act((acc - center) * scale + shift).
//
// Implicit GEMM on MFMA: M = output pixels, N = output channels (32 per
// workgroup), K = 9 taps x input channels. One workgroup owns an 8 x 32
// output tile of one frame; wave w owns tile rows 2w and 2w+1 (two 32-pixel
// M subtiles against all 32 channels: v_mfma_f32_32x32x2_f32 for f32,
// v_mfma_f32_32x32x16_bf16 for bf16 storage, f32 accumulation in both).
// The input channels are walked in chunks (8 f32 / 16 bf16 channels): a
// chunk of the 10 x 34 halo tile and the chunk's 9 x 32 weights are staged
// in LDS as 32-byte rows, unpadded and swizzled (conflict-free ds_read_b128)
// by LDS-DMA, then 9 taps of MFMAs consume them. Staging is synchronous;
// 5 workgroups per CU keep the MFMAs busy across each other's staging.
//
// Input channels [0, c_a) come from tensor A (the BEV map), [c_a, c_a+c_b)
// from tensor B. B is either a dense tensor (the materialised pooled map, or
// nothing) or -- POOLED -- the image feature map read through the img->BEV
// CSR of shpl_build_csr: the tile's runs of entries (one per occupied halo
// cell) are listed once in LDS; each pooled chunk is zero where no entry
// lands and the run's pooled vector elsewhere, computed on the spot with the
// arithmetic of k_sparse (shpl_pull.hip: TF order, separate multiply and
// add), so the conv of the fused form is bitwise the conv of
// [bev || shpl_pull(...)] and bv_fused never reaches HBM.
#include <type_traits>

#include "shpl_common.h"
#include "shpl_conv_rows.h"
#include "shpl_conv_wide.h"

namespace shpl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int TH = 8, TW = 32;              // output tile (rows x columns)
constexpr int HH = TH + 2, HWD = TW + 2;    // halo tile
constexpr int NCO = 32;                     // output channels per workgroup
constexpr int CONV_BLOCK = 256;             // 4 waves, wave w: tile rows 2w, 2w+1
constexpr int W_ROWS = 9 * NCO;             // weight rows of a chunk (tap, out channel)

// One chunk = the input channels staged per LDS round, 32 B per pixel: 8
// f32 channels (4 f32 MFMAs of K=2 per tap) or 16 bf16 channels (one bf16
// MFMA of K=16 per tap). 64 B bf16 chunks measured slower (fewer workgroups
// per CU).
template <typename T>
struct Elem {
    static constexpr int CB = 32;                        // chunk bytes per pixel
    static constexpr int CK = CB / sizeof(T);            // channels per chunk
    static constexpr int HE = 16 / sizeof(T);            // channels per 16-byte piece
    static constexpr int NP = CB / 16;                   // pieces per pixel
    static __device__ __forceinline__ float f(T v) {
        if constexpr (sizeof(T) == 4)
            return v;
        else
            return bf16_to_f32(v);
    }
    static __device__ __forceinline__ T back(float v) {
        if constexpr (sizeof(T) == 4)
            return v;
        else
            return f32_to_bf16(v);
    }
};

// ReLU of a stored value as max(bits, 0) on its bit pattern as a signed integer of its width: negatives,
// -0 and -NaN become +0, +NaN stays -- k_conv_rows' packed 16-bit max, so both kernels give the same bits.
__device__ __forceinline__ float relu_bits(float v, bool on) {
    const int32_t b = __float_as_int(v);
    return on ? __int_as_float(b > 0 ? b : 0) : v;
}
__device__ __forceinline__ uint16_t relu_bits(uint16_t v, bool on) {
    return on ? ((int16_t)v > 0 ? v : (uint16_t)0) : v;
}

struct ConvArgs {
    int n_frames, h, w;
    int tiles_x, tiles_per_frame, n_tiles;
    const void *a;
    int64_t a_stride, a_off;
    int c_a, qa;  // channels of A, chunks of A
    const void *b;
    int64_t b_stride, b_off;
    int c_b, qb;
    bool vec_a, vec_b;  // 16-byte aligned rows and offsets
    // POOLED: B rows are image pixels read through the cell-keyed CSR
    const int32_t *ent_dst, *ent_src, *row_ptr;
    const float *ent_val;
    const void *wp;  // packed weights [co_block][chunk][tap][32][CK]
    const float *center, *scale, *shift;
    int act;
    void *out;
    int64_t out_stride;
    int c_out;
    // channels >= c_split go to out2 (channel co - c_split), when out2 is set
    void *out2;
    int64_t out2_stride;
    int c_split;
    const uint32_t *occ2;  // rows form: out2 written only at the cells set in these occupancy words (NULL: all)
    bool vec_out;  // out (and out2) rows and c_split 16-byte aligned: 16-byte stores
    double *part;  // STATS: [(co_block*32 + co)*2 + stat][n_tiles]
};

// 16 bytes of channels [c, c + HE) of one row, channels >= c_src read as 0.
template <typename T>
__device__ __forceinline__ u32x4 load_piece(const T *row, int c, int c_src, bool vec) {
    constexpr int HE = Elem<T>::HE;
    if (vec && c + HE <= c_src) return *reinterpret_cast<const u32x4 *>(row + c);
    T e[HE];
#pragma unroll
    for (int j = 0; j < HE; ++j) e[j] = c + j < c_src ? row[c + j] : T(0);
    u32x4 r;
    __builtin_memcpy(&r, e, 16);
    return r;
}

// A 16-byte word of zeros in global memory: the LDS-DMA source of pieces
// outside the map (an LDS-DMA writes what it reads; it cannot write zeros).
__device__ u32x4 g_zero_piece;

// One LDS-DMA of 16 bytes per lane: lane l's piece lands at wave_dst + 16 l.
__device__ __forceinline__ void dma16(const void *src, uint8_t *wave_dst) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const u32x4 *>(src), wave_dst, 16, 0, 0);
}

// Piece g (0/1) of LDS row `row` (32-byte rows: two 16-byte pieces). SWZ: the
// unpadded, swizzled image the forward conv reads with ds_read_b128 -- slot
// 2 row + (g ^ bit 3 of row): any 16 consecutive rows of one half fall on 16
// distinct bank quads -- which an LDS-DMA can fill (its destination is
// lane-linear; the swizzle goes on the source side). Otherwise rows of PSTR bytes.
template <bool SWZ, int PSTR>
__device__ __forceinline__ int piece_off(int row, int g) {
    if constexpr (SWZ)
        return (2 * row + (g ^ ((row >> 3) & 1))) * 16;
    else
        return row * PSTR + g * 16;
}

// The piece of channels [c, c + HE) of `row` (NULL: outside the map) into the
// lane's LDS slot: an LDS-DMA when the piece is whole or all padding, a
// masked load + ds_write when it straddles the channel count (or the rows are
// not 16-byte aligned).
template <typename T>
__device__ __forceinline__ void piece_to_lds(const T *row, int c, int c_src, bool vec, uint8_t *wave_dst, int lane) {
    constexpr int HE = Elem<T>::HE;
    if (!row || c >= c_src || (vec && c + HE <= c_src))
        dma16(row && c < c_src ? static_cast<const void *>(row + c) : &g_zero_piece, wave_dst);
    else
        *reinterpret_cast<u32x4 *>(wave_dst + lane * 16) = load_piece<T>(row, c, c_src, vec);
}

// blockIdx -> tile, so that each XCD gets one contiguous run of tiles:
// neighbouring tiles share halo rows through that XCD's L2.
__device__ __forceinline__ int xcd_tile(int bid, int n) { return (int)xcd_block(bid, n); }

// Pooled vector of one occupied cell for the channels [c0, c0 + CK) of the
// chunk: sum over the cell's run of CSR entries [e0, e1) of val * img[src],
// in entry order with separate multiply and add from 0 -- the arithmetic of
// k_sparse (shpl_pull.hip) -- written to the cell's LDS row.
template <typename T, bool SWZ, int PSTR>
__device__ __forceinline__ void pool_run(const ConvArgs &p, const T *img, int c0, int32_t e0, int32_t e1,
                                         int32_t src0, float val0, uint8_t *s_base, int pix) {
    typedef Elem<T> E;
    constexpr int HE = E::HE;
    for (int g = 0; g < E::NP; ++g) {  // one 16-byte piece (4 f32 / 8 bf16 channels) at a time
        float sum[HE];
#pragma unroll
        for (int c = 0; c < HE; ++c) sum[c] = 0.0f;
        for (int32_t i = e0; i < e1; ++i) {
            const T *row = img + (int64_t)(i == e0 ? src0 : p.ent_src[i]) * p.b_stride;
            const float wv = i == e0 ? val0 : p.ent_val[i];
            const u32x4 raw = load_piece<T>(row, c0 + g * HE, p.c_b, p.vec_b);
            T x[HE];
            __builtin_memcpy(x, &raw, sizeof(raw));
#pragma unroll
            for (int c = 0; c < HE; ++c) sum[c] = __fadd_rn(sum[c], __fmul_rn(wv, E::f(x[c])));
        }
        T o[HE];
#pragma unroll
        for (int c = 0; c < HE; ++c) o[c] = E::back(sum[c]);
        __builtin_memcpy(s_base + piece_off<SWZ, PSTR>(pix, g), o, 16);
    }
}

// One 16-byte piece (channels [c, c + HE)) of an occupied cell's pooled
// vector: pool_run's sum for one piece, its entries' loads issued
// POOL_BATCH at a time (one round trip for runs of up to POOL_BATCH entries)
// and summed in entry order.
#ifndef SHPL_POOL_PIECES
#define SHPL_POOL_PIECES 1
#endif
constexpr int POOL_BATCH = 4;
template <typename T, bool SWZ, int PSTR>
__device__ __forceinline__ void pool_piece(const ConvArgs &p, const T *img, int c, int32_t e0, int32_t e1,
                                           int32_t src0, float val0, uint8_t *s_base, int pix, int g) {
    typedef Elem<T> E;
    constexpr int HE = E::HE;
    float sum[HE];
#pragma unroll
    for (int j = 0; j < HE; ++j) sum[j] = 0.0f;
    for (int32_t i0 = e0; i0 < e1; i0 += POOL_BATCH) {
        u32x4 raw[POOL_BATCH];
        float wv[POOL_BATCH];
#pragma unroll
        for (int u = 0; u < POOL_BATCH; ++u) {
            const int32_t i = i0 + u;
            if (i < e1) {
                const int32_t sr = i == e0 ? src0 : p.ent_src[i];
                wv[u] = i == e0 ? val0 : p.ent_val[i];
                raw[u] = load_piece<T>(img + (int64_t)sr * p.b_stride, c, p.c_b, p.vec_b);
            }
        }
#pragma unroll
        for (int u = 0; u < POOL_BATCH; ++u) {
            if (i0 + u >= e1) break;
            T x[HE];
            __builtin_memcpy(x, &raw[u], sizeof(raw[u]));
#pragma unroll
            for (int j = 0; j < HE; ++j) sum[j] = __fadd_rn(sum[j], __fmul_rn(wv[u], E::f(x[j])));
        }
    }
    T o[HE];
#pragma unroll
    for (int j = 0; j < HE; ++j) o[j] = E::back(sum[j]);
    __builtin_memcpy(s_base + piece_off<SWZ, PSTR>(pix, g), o, 16);
}

// The halo tile's runs of CSR entries in LDS (POOLED): one run per occupied
// halo cell, with its first entry's source row and weight.
struct HaloRuns {
    int32_t *lo, *pre;                    // [HH], [HH+1]: entry range of each halo row
    int32_t *pix, *e, *end, *src;         // [HH*HWD]
    float *val;                           // [HH*HWD]
    uint8_t *occ;                         // [HH*HWD]: cell holds a run
    int64_t *scan;                        // [SHPL_BLOCK/64+1]
};

// Lists the runs of the HHT-row halo of output tile (f, y0, x0): per halo
// row the entry range of cells [x0-1, x0+TW+1) (row pointers + counting the
// row's sorted entries below each bound), then one block scan in entry
// order. Every thread of the 256 calls it.
template <int HHT = HH>
__device__ int find_runs(const ConvArgs &p, int f, int y0, int x0, const HaloRuns &r) {
    constexpr int NPIX = HHT * HWD;
    const int tid = threadIdx.x;
    const int H = p.h, W = p.w;
    const int64_t frame_row0 = (int64_t)f * H * W;
    for (int j = tid; j < NPIX; j += CONV_BLOCK) r.occ[j] = 0;
    // wave w takes halo rows w, w+4, w+8; a row's sorted entries are counted
    // 64 at a time against the two cell bounds (ballots), the rows' loads in
    // flight together: two round trips for rows of up to 64 entries.
    const int lane = tid & 63, wave = tid >> 6;
    constexpr int RPW = (HHT + 3) / 4;  // rows per wave
    int32_t ra[RPW], rb[RPW], kl[RPW], kh[RPW];
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        const int k = wave + 4 * u, y = y0 - 1 + k;
        ra[u] = rb[u] = 0;
        kl[u] = kh[u] = 0;
        if (k < HHT && y >= 0 && y < H) {
            ra[u] = p.row_ptr[(int64_t)f * (H + 1) + y];
            rb[u] = p.row_ptr[(int64_t)f * (H + 1) + y + 1];
            kl[u] = (int32_t)(frame_row0 + (int64_t)y * W + (x0 > 0 ? x0 - 1 : 0));
            kh[u] = (int32_t)(frame_row0 + (int64_t)y * W + (x0 + TW + 1 < W ? x0 + TW + 1 : W));
        }
    }
    int32_t d[RPW];
#pragma unroll
    for (int u = 0; u < RPW; ++u) d[u] = ra[u] + lane < rb[u] ? p.ent_dst[ra[u] + lane] : 0x7fffffff;
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        const int k = wave + 4 * u;
        int32_t n_lo = __popcll(__ballot(d[u] < kl[u])), n_hi = __popcll(__ballot(d[u] < kh[u]));
        for (int32_t base = ra[u] + 64; base < rb[u] && n_hi == base - ra[u]; base += 64) {  // rows over 64 entries
            const int32_t dd = base + lane < rb[u] ? p.ent_dst[base + lane] : 0x7fffffff;
            n_lo += __popcll(__ballot(dd < kl[u]));
            n_hi += __popcll(__ballot(dd < kh[u]));
        }
        if (lane == 0 && k < HHT) {
            r.lo[k] = ra[u] + n_lo;
            r.pre[k + 1] = n_hi - n_lo;
        }
    }
    __syncthreads();
    if (tid == 0) {
        r.pre[0] = 0;
        for (int k = 0; k < HHT; ++k) r.pre[k + 1] += r.pre[k];
    }
    __syncthreads();
    const int n_ent = r.pre[HHT];
    int n_run = 0, n_tail = 0;
    for (int base = 0; base < n_ent; base += CONV_BLOCK) {
        const int j = base + tid;
        int64_t flags = 0;
        int32_t e = 0, pix = 0;
        if (j < n_ent) {
            int k = 0;
            while (j >= r.pre[k + 1]) ++k;
            e = r.lo[k] + (j - r.pre[k]);
            const int32_t last = r.lo[k] + (r.pre[k + 1] - r.pre[k]) - 1;
            const int32_t d = p.ent_dst[e];
            const bool head = j == r.pre[k] || p.ent_dst[e - 1] != d;
            const bool tail = e == last || p.ent_dst[e + 1] != d;
            flags = (head ? 1 : 0) | (tail ? (int64_t)1 << 32 : 0);
            const int y = y0 - 1 + k;
            pix = k * HWD + (int)((int64_t)d - frame_row0 - (int64_t)y * W) - (x0 - 1);
        }
        int64_t tot;
        const int64_t ex = block_excl_scan(flags, r.scan, &tot);
        if (flags & 1) {
            const int k = n_run + (int)(ex & 0xffffffff);
            r.e[k] = e;
            r.pix[k] = pix;
            r.occ[pix] = 1;
            r.src[k] = p.ent_src[e];
            r.val[k] = p.ent_val[e];
        }
        if (flags >> 32) r.end[n_tail + (int)(ex >> 32)] = e + 1;
        n_run += (int)(tot & 0xffffffff);
        n_tail += (int)(tot >> 32);  // a run may open in one round and close in the next
    }
    __syncthreads();
    return n_run;
}

// Stages input chunk q (channels of A, then of B) of the 10 x 34 halo of
// output tile (f, y0, x0) into s_in ([pixel][chunk] rows, piece_off); zero
// outside the map. Pooled chunks: zeros where no entry lands, each run's sum
// elsewhere (disjoint cells: no barrier between the two). The caller
// synchronises after.
template <typename T, bool POOLED, int PSTR, bool SWZ = false, int HHT = HH>
__device__ __forceinline__ void stage_halo(const ConvArgs &p, int q, int f, int y0, int x0, uint8_t *s_in,
                                           const HaloRuns &r, int n_run) {
    typedef Elem<T> E;
    constexpr int CK = E::CK, HE = E::HE, NP = E::NP;
    constexpr int IN_PIECES = HHT * HWD * NP;
    constexpr int IN_IT = (IN_PIECES + CONV_BLOCK - 1) / CONV_BLOCK;
    const int tid = threadIdx.x;
    const int H = p.h, W = p.w;
    const int64_t frame_row0 = (int64_t)f * H * W;
    const bool from_a = q < p.qa;
    if (from_a || !POOLED) {
        const T *src = reinterpret_cast<const T *>(from_a ? p.a : p.b) + (from_a ? p.a_off : p.b_off);
        const int64_t stride = from_a ? p.a_stride : p.b_stride;
        const int c_src = from_a ? p.c_a : p.c_b;
        const int c0 = (from_a ? q : q - p.qa) * CK;
        const bool vec = from_a ? p.vec_a : p.vec_b;
        u32x4 v[IN_IT];
#pragma unroll
        for (int u = 0; u < IN_IT; ++u) {
            const int j = tid + u * CONV_BLOCK;
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (j < IN_PIECES) {
                const int pix = j / NP, hr = pix / HWD, hc = pix - hr * HWD;
                const int y = y0 - 1 + hr, x = x0 - 1 + hc;
                if (y >= 0 && y < H && x >= 0 && x < W)
                    v[u] = load_piece<T>(src + (frame_row0 + (int64_t)y * W + x) * stride, c0 + (j % NP) * HE, c_src,
                                         vec);
            }
        }
#pragma unroll
        for (int u = 0; u < IN_IT; ++u) {
            const int j = tid + u * CONV_BLOCK;
            if (j < IN_PIECES) *reinterpret_cast<u32x4 *>(s_in + piece_off<SWZ, PSTR>(j / NP, j % NP)) = v[u];
        }
    } else {
#pragma unroll
        for (int u = 0; u < IN_IT; ++u) {
            const int j = tid + u * CONV_BLOCK;
            if (j < IN_PIECES && !r.occ[j / NP])
                *reinterpret_cast<u32x4 *>(s_in + piece_off<SWZ, PSTR>(j / NP, j % NP)) = u32x4{0u, 0u, 0u, 0u};
        }
        const T *img = reinterpret_cast<const T *>(p.b) + p.b_off;
#if SHPL_POOL_PIECES
        // one (run, 16-byte piece) pair per thread, POOL_BATCH entries' loads in flight per round trip
        for (int t = tid; t < n_run * NP; t += CONV_BLOCK)
            pool_piece<T, SWZ, PSTR>(p, img, (q - p.qa) * CK + (t % NP) * HE, r.e[t / NP], r.end[t / NP],
                                     r.src[t / NP], r.val[t / NP], s_in, r.pix[t / NP], t % NP);
#else
        for (int k = tid; k < n_run; k += CONV_BLOCK)
            pool_run<T, SWZ, PSTR>(p, img, (q - p.qa) * CK, r.e[k], r.end[k], r.src[k], r.val[k], s_in, r.pix[k]);
#endif
    }
}

#define SHPL_HALO_RUNS_LDS(POOLED, HHT)                                                                       \
    __shared__ int32_t s_lo[HHT], s_pre[HHT + 1];                                                            \
    __shared__ int32_t s_run_pix[POOLED ? HHT * HWD : 1], s_run_e[POOLED ? HHT * HWD : 1],                   \
        s_run_end[POOLED ? HHT * HWD : 1], s_run_src[POOLED ? HHT * HWD : 1];                               \
    __shared__ float s_run_val[POOLED ? HHT * HWD : 1];                                                      \
    __shared__ uint8_t s_occ[POOLED ? HHT * HWD : 1];                                                        \
    __shared__ int64_t s_scan[SHPL_BLOCK / 64 + 1];                                                          \
    const HaloRuns runs{s_lo, s_pre, s_run_pix, s_run_e, s_run_end, s_run_src, s_run_val, s_occ, s_scan};

// Forward tile shape: output rows per wave, 2 at f32 (8 x 32 tiles) and 4 at
// bf16 (16 x 32 tiles). A bf16 chunk's MFMAs are 16x faster than an f32
// chunk's: the taller tile halves the staging round trips, halo rows and
// weight rows per output pixel, and each wave reuses every A operand it reads
// for up to three kernel rows (0.75 KB of LDS reads per MFMA instead of 1.5).
#ifndef SHPL_BF16_RPW
#define SHPL_BF16_RPW 2
#endif
template <typename T>
struct ConvTile {
    static constexpr int RPW = sizeof(T) == 2 ? SHPL_BF16_RPW : 2;
    static constexpr int TH = 4 * RPW, HH = TH + 2;
};

// Stages input chunk q of output tile (f, y0, x0) -- its 9x32 weight rows
// and its HH x 34 halo -- into one LDS buffer pair (swizzled 32-byte rows).
// Weights and dense halo chunks are LDS-DMAs (lane k of the wave fills slot
// k: it loads the piece the swizzle puts there); pooled chunks are computed
// (stage_halo). The caller waits and synchronises.
template <typename T, bool POOLED, int NCB = 1>
__device__ __forceinline__ void conv_stage(const ConvArgs &p, int q, int f, int y0, int x0, const T *wq,
                                           int64_t wq_cb, uint8_t *s_in, uint8_t *s_w, const HaloRuns &runs,
                                           int n_run) {
    typedef Elem<T> E;
    constexpr int CK = E::CK, HE = E::HE, NP = E::NP, HHT = ConvTile<T>::HH;
    constexpr int IN_PIECES = HHT * HWD * NP, W_PIECES = W_ROWS * NP;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {  // the weight rows of each output block, W_PIECES slots apart
#pragma unroll
        for (int u = 0; u < (W_PIECES + CONV_BLOCK - 1) / CONV_BLOCK; ++u) {
            const int base = u * CONV_BLOCK + wave * 64;  // the wave's first slot
            if (base >= W_PIECES) break;
            const int k = base + lane, row = k >> 1, g = (k & 1) ^ ((row >> 3) & 1);
            if (k < W_PIECES)
                dma16(wq + cb * wq_cb + ((int64_t)q * W_ROWS + row) * CK + g * HE, s_w + (cb * W_PIECES + base) * 16);
        }
    }
    if (!POOLED || q < p.qa) {
        const int H = p.h, W = p.w;
        const int64_t frame_row0 = (int64_t)f * H * W;
        const bool from_a = q < p.qa;
        const T *src = reinterpret_cast<const T *>(from_a ? p.a : p.b) + (from_a ? p.a_off : p.b_off);
        const int64_t stride = from_a ? p.a_stride : p.b_stride;
        const int c_src = from_a ? p.c_a : p.c_b;
        const int c0 = (from_a ? q : q - p.qa) * CK;
        const bool vec = from_a ? p.vec_a : p.vec_b;
#pragma unroll
        for (int u = 0; u < (IN_PIECES + CONV_BLOCK - 1) / CONV_BLOCK; ++u) {
            const int base = u * CONV_BLOCK + wave * 64;
            if (base >= IN_PIECES) break;
            const int k = base + lane, pix = k >> 1, g = (k & 1) ^ ((pix >> 3) & 1);
            const int hr = pix / HWD, hc = pix - hr * HWD;
            const int y = y0 - 1 + hr, x = x0 - 1 + hc;
            const bool ok = y >= 0 && y < H && x >= 0 && x < W;
            if (k < IN_PIECES)
                piece_to_lds<T>(ok ? src + (frame_row0 + (int64_t)y * W + x) * stride : nullptr, c0 + g * HE, c_src, vec,
                                s_in + base * 16, lane);
        }
    } else {
        stage_halo<T, true, E::CB, true, HHT>(p, q, f, y0, x0, s_in, runs, n_run);
    }
}

// NCB: output-channel blocks per workgroup (blockIdx.y covers NCB of them):
// 2 for the input gradient's 64 output channels, so each staged input chunk
// feeds twice the MFMAs (one halo staging per tile instead of two).
template <typename T, bool POOLED, bool STATS, int NCB = 1>
__global__ __launch_bounds__(CONV_BLOCK, NCB == 2 ? 3 : 4) void k_conv3x3(const ConvArgs p) {
    typedef Elem<T> E;
    constexpr int CK = E::CK, NP = E::NP, RPW = ConvTile<T>::RPW, HHT = ConvTile<T>::HH;
    static_assert(NCB == 1 || !STATS, "statistics: one output block per workgroup");
    static_assert(NP == 2, "two 16-byte pieces per LDS row (the swizzle)");
    constexpr int IN_BYTES = HHT * HWD * NP * 16, W_BYTES = W_ROWS * NP * 16 * NCB;
    // the output rows' transpose (epilogue) reuses the chunk buffers: 4 waves x 32 pixels x OPITCH
    constexpr int OPITCH = NCO * (int)sizeof(T) + 16;
    static_assert(4 * 32 * OPITCH <= IN_BYTES + W_BYTES, "epilogue rows fit the chunk buffers");
    __shared__ __attribute__((aligned(16))) uint8_t s_buf[IN_BYTES + W_BYTES];
    uint8_t *const s_in = s_buf, *const s_w = s_buf + IN_BYTES;
    __shared__ float s_red[4][2][NCO];
    __shared__ __attribute__((aligned(16))) float s_par[NCB][2][NCO];  // scale, shift - center * scale of the block's channels
    SHPL_HALO_RUNS_LDS(POOLED, HHT)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pl = lane & 31, hf = lane >> 5;
    const int tile = xcd_tile(blockIdx.x, p.n_tiles);
    const int cob0 = blockIdx.y * NCB;
    const int f = tile / p.tiles_per_frame;
    const int t_in = tile - f * p.tiles_per_frame;
    const int ty = t_in / p.tiles_x, tx = t_in - ty * p.tiles_x;
    const int y0 = ty * ConvTile<T>::TH, x0 = tx * TW;
    const int H = p.h, W = p.w;
    const int64_t frame_row0 = (int64_t)f * H * W;
    const int Q = p.qa + p.qb;

    // epilogue coefficients, as k_conv_rows: scale (1 when absent) and shift - center * scale, applied
    // as one fma -- the two kernels give the same bits for the same call
    if (tid < NCO * NCB) {
        const int cb = tid / NCO, c = (cob0 + cb) * NCO + (tid & 31);
        const bool in = c < p.c_out;
        const float sc = p.scale && in ? p.scale[c] : 1.0f;
        const float ce = p.center && in ? p.center[c] : 0.0f;
        const float sh = p.shift && in ? p.shift[c] : 0.0f;
        s_par[cb][0][tid & 31] = sc;
        s_par[cb][1][tid & 31] = __fsub_rn(sh, __fmul_rn(ce, sc));
    }
    const int n_run = POOLED ? find_runs<HHT>(p, f, y0, x0, runs) : 0;  // (s_par: published by the next barrier)

    f32x16 acc[NCB][RPW];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int m = 0; m < RPW; ++m)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[cb][m][i] = 0.0f;

    const int64_t wq_cb = (int64_t)Q * W_ROWS * CK;  // one output block further in the packed weights
    const T *wq = reinterpret_cast<const T *>(p.wp) + cob0 * wq_cb;
    for (int q = 0; q < Q; ++q) {
        // ---- stage chunk q, synchronously: the other workgroups on the CU (5
        // at f32) keep the MFMAs busy meanwhile. Measured and dropped: two LDS
        // buffers with chunk q+1's LDS-DMAs in flight under chunk q's MFMAs
        // (3 workgroups per CU: f32 fused 11.3 -> 12.1 ms), and a register-staged
        // prefetch (VGPRs 62 -> 86-168: 11.8 -> 12.5 ms)
        conv_stage<T, POOLED, NCB>(p, q, f, y0, x0, wq, wq_cb, s_in, s_w, runs, n_run);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMAs have landed
        __syncthreads();
        const uint8_t *si = s_in, *sw = s_w;
        // ---- 9 taps of MFMA over chunk q
        if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    f32x4 b4[NCB];
#pragma unroll
                    for (int cb = 0; cb < NCB; ++cb)
                        b4[cb] = *reinterpret_cast<const f32x4 *>(
                            sw + cb * (W_BYTES / NCB) + piece_off<true, 0>((ky * 3 + kx) * NCO + pl, hf));
#pragma unroll
                    for (int m = 0; m < RPW; ++m) {
                        const uint8_t *arow = si + piece_off<true, 0>((RPW * wave + m + ky) * HWD + pl + kx, hf);
                        // lane half h supplies channels 4h+s of the chunk to MFMA s (both operands)
                        const f32x4 a4 = *reinterpret_cast<const f32x4 *>(arow);
#pragma unroll
                        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                            for (int s = 0; s < 4; ++s)
                                acc[cb][m] =
                                    __builtin_amdgcn_mfma_f32_32x32x2f32(b4[cb][s], a4[s], acc[cb][m], 0, 0, 0);
                    }
                }
            }
        } else {
            // channels 0..15 of the chunk; lane half h holds 8h .. 8h+7. Per kernel
            // column kx: the three kernel rows' weights, then each of the wave's
            // RPW + 2 halo rows read once and fed to every output row it reaches.
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                bf16x8 b8[NCB][3];
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
                        b8[cb][ky] = *reinterpret_cast<const bf16x8 *>(
                            sw + cb * (W_BYTES / NCB) + piece_off<true, 0>((ky * 3 + kx) * NCO + pl, hf));
#pragma unroll
                for (int r = 0; r < RPW + 2; ++r) {
                    const bf16x8 a8 = *reinterpret_cast<const bf16x8 *>(
                        si + piece_off<true, 0>((RPW * wave + r) * HWD + pl + kx, hf));
#pragma unroll
                    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                        for (int ky = 0; ky < 3; ++ky)
                            if (r - ky >= 0 && r - ky < RPW)
                                acc[cb][r - ky] =
                                    __builtin_amdgcn_mfma_f32_32x32x16_bf16(b8[cb][ky], a8, acc[cb][r - ky], 0, 0, 0);
                }
            }
        }
        __syncthreads();  // the chunk's buffers are restaged next
    }

    // ---- epilogue. The MFMAs take the weights as A and the pixels as B (D =
    // W^T X^T), so acc element i of subtile m is channel cob*32 + 8(i>>2) +
    // 4h + (i&3) of pixel (y0 + RPW w + m, x0 + pl): four runs of 4 channels
    // per lane. A row of 32 pixels goes through LDS (wave-private, rows of
    // OPITCH bytes) and out as 16-byte pieces, consecutive lanes on
    // consecutive pieces: 2 (bf16) / 4 (f32) store instructions per row, each
    // one contiguous 1 KB, instead of 16 two- or four-byte stores (the texture
    // addresser was the bf16 conv's busiest unit). Blocks whose channels are not
    // whole or whose rows are not 16-byte aligned store channel by channel.
    constexpr int HE = E::HE, PPP = NCO / HE;  // channels per piece, pieces per pixel
    const int x = x0 + pl;
    uint8_t *const s_o = s_buf + wave * 32 * OPITCH;
    float s1[16], s2[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s1[i] = s2[i] = 0.0f;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
        const int cob = cob0 + cb;
        const bool fast = p.vec_out && cob * NCO + NCO <= p.c_out;
#pragma unroll
        for (int m = 0; m < RPW; ++m) {
            const int y = y0 + RPW * wave + m;
            const bool ok = y < H && x < W;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int cl = 8 * g + 4 * hf, c = cob * NCO + cl;  // first channel of the run
                const f32x4 scl = *reinterpret_cast<const f32x4 *>(&s_par[cb][0][cl]);
                const f32x4 sft = *reinterpret_cast<const f32x4 *>(&s_par[cb][1][cl]);
                T o[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v = acc[cb][m][4 * g + j];
                    if (STATS && ok) {
                        s1[4 * g + j] = __fadd_rn(s1[4 * g + j], v);
                        s2[4 * g + j] = __fadd_rn(s2[4 * g + j], __fmul_rn(v, v));
                    }
                    o[j] = relu_bits(E::back(__builtin_fmaf(v, scl[j], sft[j])), p.act == 1);
                }
                if (fast) {
                    __builtin_memcpy(s_o + pl * OPITCH + cl * sizeof(T), o, sizeof(o));
                } else if (ok) {
                    const int64_t row = frame_row0 + (int64_t)y * W + x;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (c + j >= p.c_out) break;
                        T *d = p.out2 && c + j >= p.c_split
                                   ? reinterpret_cast<T *>(p.out2) + row * p.out2_stride + (c + j - p.c_split)
                                   : reinterpret_cast<T *>(p.out) + row * p.out_stride + c + j;
                        *d = o[j];
                    }
                }
            }
            if (fast) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's row is in LDS (one wave: in order)
#pragma unroll
                for (int k = 0; k < 32 * PPP / 64; ++k) {
                    const int pc = lane + 64 * k, px = pc / PPP, pi = pc % PPP;
                    const u32x4 v = *reinterpret_cast<const u32x4 *>(s_o + px * OPITCH + pi * 16);
                    if (y < H && x0 + px < W) {
                        const int64_t row = frame_row0 + (int64_t)y * W + x0 + px;
                        const int c = cob * NCO + pi * HE;
                        T *d = p.out2 && c >= p.c_split
                                   ? reinterpret_cast<T *>(p.out2) + row * p.out2_stride + (c - p.c_split)
                                   : reinterpret_cast<T *>(p.out) + row * p.out_stride + c;
                        *reinterpret_cast<u32x4 *>(d) = v;
                    }
                }
            }
        }
    }
    if (STATS) {
        // per channel: sum over the 32 pixels of the lane half by a halving
        // butterfly (each exchange hands the partner the half of the values it
        // keeps: 8 + 4 + 2 + 1 + 1 shuffles per statistic instead of 16 x 5),
        // after which lanes 2j and 2j+1 both hold value j; then over the 4
        // waves in double
#pragma unroll
        for (int n = 8, off = 16; n >= 1; n >>= 1, off >>= 1) {
            const bool up = (pl & off) != 0;
#pragma unroll
            for (int i = 0; i < n; ++i) {
                const float g1 = up ? s1[i] : s1[i + n], k1 = up ? s1[i + n] : s1[i];
                const float g2 = up ? s2[i] : s2[i + n], k2 = up ? s2[i + n] : s2[i];
                s1[i] = __fadd_rn(k1, __shfl_xor(g1, off, 64));
                s2[i] = __fadd_rn(k2, __shfl_xor(g2, off, 64));
            }
        }
        s1[0] = __fadd_rn(s1[0], __shfl_xor(s1[0], 1, 64));
        s2[0] = __fadd_rn(s2[0], __shfl_xor(s2[0], 1, 64));
        if ((pl & 1) == 0) {
            const int i = pl >> 1, cl = 8 * (i >> 2) + 4 * hf + (i & 3);
            s_red[wave][0][cl] = s1[0];
            s_red[wave][1][cl] = s2[0];
        }
        __syncthreads();
        if (tid < 2 * NCO) {
            const int st = tid >> 5, c = tid & 31;
            double sum = 0.0;
            for (int w = 0; w < 4; ++w) sum += (double)s_red[w][st][c];
            p.part[((int64_t)(cob0 * NCO + c) * 2 + st) * p.n_tiles + tile] = sum;
        }
    }
}

// Packed weights: HWIO [3][3][c_a+c_b][c_out] -> [co_block][chunk][tap][32][CK],
// chunks of A's channels first, then B's, zero padded. transpose (the input
// gradient): w is the forward's HWIO [3][3][c_out][c_a+c_b] and the packed
// tap t takes W[8-t] transposed (W'[ky][kx][co][ci] = W[2-ky][2-kx][ci][co]).
template <typename T>
__global__ __launch_bounds__(SHPL_BLOCK) void k_pack_w(const T *w, int c_a, int qa, int c_b, int qb, int c_out,
                                                       int n_cob, int transpose, T *wp) {
    constexpr int CK = Elem<T>::CK;
    const int Q = qa + qb;
    const int64_t total = (int64_t)n_cob * Q * W_ROWS * CK;
    const int cin = c_a + c_b;
    for (int64_t t = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int k = (int)(t % CK);
        int64_t r = t / CK;
        const int co_l = (int)(r % NCO);
        r /= NCO;
        const int tap = (int)(r % 9);
        r /= 9;
        const int q = (int)(r % Q);
        const int cob = (int)(r / Q);
        const int co = cob * NCO + co_l;
        int ci;
        bool ok;
        if (q < qa) {
            ci = q * CK + k;
            ok = ci < c_a;
        } else {
            const int cb = (q - qa) * CK + k;
            ci = c_a + cb;
            ok = cb < c_b;
        }
        const int64_t src = transpose ? ((int64_t)(8 - tap) * c_out + co) * cin + ci
                                      : ((int64_t)tap * cin + ci) * c_out + co;
        wp[t] = (ok && co < c_out) ? w[src] : T(0);
    }
}

// Entry pointer of every BEV row of every frame over the destination-sorted
// CSR: row_ptr[f*(H+1) + y] = first entry of frame f whose cell lies in row
// >= y (empty slots, dst -1, count as row H).
__global__ __launch_bounds__(SHPL_BLOCK) void k_row_ptr(const int32_t *dst, const int64_t *frame_off, int H, int W,
                                                        int32_t *row_ptr) {
    const int f = blockIdx.y;
    const int64_t s = frame_off[f], e_end = frame_off[f + 1];
    const int64_t base = (int64_t)f * H * W;
    int32_t *rp = row_ptr + (int64_t)f * (H + 1);
    for (int64_t e = s + (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; e <= e_end;
         e += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int32_t dc = e < e_end ? dst[e] : -1;
        const int yc = dc < 0 ? H : (int)((dc - base) / W);
        int yp = -1;
        if (e > s) {
            const int32_t dp = dst[e - 1];
            yp = dp < 0 ? H : (int)((dp - base) / W);
        }
        for (int y = yp + 1; y <= yc; ++y) rp[y] = (int32_t)e;
    }
}

// Per-channel sum / sum of squares of the pre-activation output, summed over
// the per-tile partials in a fixed order (deterministic): one block per
// (channel, statistic).
// Deterministic sums of long strided lists (the per-tile / per-block /
// per-group partials): thread t adds elements t, t + n_thr, ... into 8
// independent accumulators (8 loads in flight, then a fixed pairwise
// combine), the wave and the block then reduce in a fixed order. A thread per
// list walking it serially (550-4096 dependent loads) cost 0.2-0.3 ms per
// reduction.
template <int NT>
__device__ __forceinline__ double strided_sum(const double *v, int64_t n, int64_t step, int t) {
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int64_t i = t;
    for (; i + 7 * NT < n; i += 8 * NT) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += v[(i + u * NT) * step];
    }
    for (int u = 0; i < n; i += NT, ++u) acc[u & 7] += v[i * step];
    return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// Block sum of one double per thread (fixed order); valid in thread 0.
template <int NT>
__device__ __forceinline__ double block_sum(double s, double *red) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0)
        for (int w = 1; w < NT / 64; ++w) s += red[w];
    __syncthreads();
    return s;
}

constexpr int RED_BLOCK = 1024;
__global__ __launch_bounds__(RED_BLOCK) void k_stats_reduce(const double *part, int n_tiles, int c_out,
                                                            double *stats) {
    __shared__ double red[RED_BLOCK / 64];
    const int ch = blockIdx.x >> 1, st = blockIdx.x & 1;
    const double s = block_sum<RED_BLOCK>(
        strided_sum<RED_BLOCK>(part + ((int64_t)ch * 2 + st) * n_tiles, n_tiles, 1, threadIdx.x), red);
    if (threadIdx.x == 0 && ch < c_out) stats[st * c_out + ch] = s;
}

// BatchNorm (training) from the batch statistics: mean, biased variance for
// the normalisation, Bessel-corrected variance for the moving average (TF
// FusedBatchNorm), then y = act((x - mean) * gamma / sqrt(var + eps) + beta)
// in place.
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_finalize(const double *stats, double count, int c, float eps,
                                                            const float *gamma, float *mean_out, float *scale_out,
                                                            float *moving_mean, float *moving_var, float decay,
                                                            float *batch_mean, float *batch_var) {
    for (int ch = threadIdx.x; ch < c; ch += SHPL_BLOCK) {
        const double mean = stats[ch] / count;
        double var = stats[c + ch] / count - mean * mean;
        if (var < 0.0) var = 0.0;
        const float mf = (float)mean, vf = (float)var;
        const float g = gamma ? gamma[ch] : 1.0f;
        mean_out[ch] = mf;
        scale_out[ch] = __fmul_rn(g, __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(vf, eps))));
        const float vu = count > 1.0 ? (float)(var * count / (count - 1.0)) : vf;
        if (moving_mean) moving_mean[ch] = __fsub_rn(moving_mean[ch], __fmul_rn(__fsub_rn(moving_mean[ch], mf), 1.0f - decay));
        if (moving_var) moving_var[ch] = __fsub_rn(moving_var[ch], __fmul_rn(__fsub_rn(moving_var[ch], vu), 1.0f - decay));
        if (batch_mean) batch_mean[ch] = mf;
        if (batch_var) batch_var[ch] = vu;
    }
}

template <typename T>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_apply(const T *x, T *y, int64_t rows, int64_t stride, int c,
                                                         const float *mean, const float *scale, const float *beta,
                                                         int act) {
    const int64_t total = rows * c;
    for (int64_t t = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int64_t r = t / c;
        const int ch = (int)(t - r * c);
        float v = __fmul_rn(__fsub_rn(Elem<T>::f(x[r * stride + ch]), mean[ch]), scale[ch]);
        if (beta) v = __fadd_rn(v, beta[ch]);
        if (act == 1) v = v > 0.0f ? v : 0.0f;
        y[r * stride + ch] = Elem<T>::back(v);
    }
}

// 16-byte pieces of a row (VEC channels): the vector forms of the BatchNorm
// streams, used when rows and channel counts are multiples of VEC and aligned.
// Rows per thread of the BatchNorm apply kernels' grid-stride loops: enough
// to amortise the per-thread channel parameters (six loads and a division
// per channel in the backward), few enough to keep loads in flight. Measured
// at 64 frames: f32 17 -> 4 rows took apply 1.78 -> 1.61 ms and backward
// apply 2.68 -> 2.35 ms; bf16 at 2 rows per thread was 1.7x slower than at 8.
constexpr int64_t bn_rows_per_thread(int esz) { return esz == 4 ? 4 : 8; }

// f(std::bool_constant<b0>{}, std::bool_constant<b1>{}, ...) for run-time switches b0, b1, ...: the
// instance of a vector BatchNorm kernel for one combination of its compile-time forms.
template <bool... Bs, typename F>
void bn_forms(F &&f) {
    f(std::bool_constant<Bs>{}...);
}
template <bool... Bs, typename F, typename... R>
void bn_forms(F &&f, bool b, R... rest) {
    if (b)
        bn_forms<Bs..., true>(f, rest...);
    else
        bn_forms<Bs..., false>(f, rest...);
}

// 16-byte pieces of the BatchNorm streams, nontemporal (each byte is touched
// once per pass; the maps are far larger than the caches).
template <typename T, int VEC>
struct Piece {
    static __device__ __forceinline__ void load(const T *p, float (&x)[VEC]) {
        const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        T e[VEC];
        __builtin_memcpy(e, &r, 16);
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[k] = Elem<T>::f(e[k]);
    }
    static __device__ __forceinline__ void store(T *p, const float (&x)[VEC]) {
        T e[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) e[k] = Elem<T>::back(x[k]);
        u32x4 r;
        __builtin_memcpy(&r, e, 16);
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(p));
    }
};

constexpr int BN_U = 4;  // rows per iteration of the vector apply kernels: their loads in flight together

// Thread layout of the vector forms: c / VEC piece lanes (a power of two
// dividing the block) times SHPL_BLOCK / (c / VEC) row lanes, so each thread
// keeps one channel group and its per-channel coefficients in registers.
// The vector apply kernels take their switches (ReLU, beta, y, training) as
// template arguments: as run-time flags they put a branch around every element
// of the unrolled loops (bn_forms picks the instance; bf16 at 64 frames: the
// backward apply 1,199 -> 1,147 us, the forward apply 777 -> 750 us,
// profiles/r04_bn_ab.log).
template <typename T, bool BETA, bool ACT>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_apply_vec(const T *x, T *y, int64_t rows, int64_t stride, int c,
                                                             const float *mean, const float *scale,
                                                             const float *beta) {
    constexpr int VEC = 16 / sizeof(T);
    const int pr = c / VEC, rpb = SHPL_BLOCK / pr;
    const int ch0 = (threadIdx.x % pr) * VEC;
    float m[VEC], sc[VEC], b[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        m[k] = mean[ch0 + k];
        sc[k] = scale[ch0 + k];
        b[k] = BETA ? beta[ch0 + k] : 0.0f;
    }
    const int64_t step = (int64_t)gridDim.x * rpb;
    for (int64_t r0 = (int64_t)blockIdx.x * rpb + threadIdx.x / pr; r0 < rows; r0 += BN_U * step) {
        float v[BN_U][VEC];
#pragma unroll
        for (int u = 0; u < BN_U; ++u)
            if (r0 + u * step < rows) Piece<T, VEC>::load(x + (r0 + u * step) * stride + ch0, v[u]);
#pragma unroll
        for (int u = 0; u < BN_U; ++u) {
            if (r0 + u * step >= rows) break;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                float t = __fmul_rn(__fsub_rn(v[u][k], m[k]), sc[k]);
                if constexpr (BETA) t = __fadd_rn(t, b[k]);
                v[u][k] = (ACT && !(t > 0.0f)) ? 0.0f : t;
            }
            Piece<T, VEC>::store(y + (r0 + u * step) * stride + ch0, v[u]);
        }
    }
}

// ---------------------------------------------------------------- backward
// BatchNorm (+ ReLU) backward. g_bn = g * [y > 0] (act), xhat = (raw - mean)
// * scale / gamma; per-channel sums dbeta = sum g_bn, dgamma = sum g_bn xhat
// over rows in a fixed order (f64 partials per block, then per channel), and
//   training:  g_raw = scale * (g_bn - dbeta / N - xhat * dgamma / N)
//   inference: g_raw = scale * g_bn     (moving statistics are constants)
// mean / scale NULL: 0 / 1 (a conv bias instead of BN: g_raw = g_bn).
// The ReLU mask [y > 0] is read from y, or (y NULL) recomputed from the BN
// input with the forward's rounded operations, u = (raw - mean) * scale
// (+ beta), so that it is bitwise the forward's: [u > 0] == [y > 0].
__device__ __forceinline__ float bn_pre_act(float x, float m, float sc, const float *beta, int ch) {
    const float u = __fmul_rn(__fsub_rn(x, m), sc);
    return beta ? __fadd_rn(u, beta[ch]) : u;
}

template <typename T>
__device__ __forceinline__ float bn_gbn(const T *y, const T *raw, const T *gy, int64_t o, int ch, int act,
                                        const float *mean, const float *scale, const float *beta) {
    const float gv = Elem<T>::f(gy[o]);
    if (act != 1) return gv;
    const float yv = y ? Elem<T>::f(y[o])
                       : bn_pre_act(Elem<T>::f(raw[o]), mean ? mean[ch] : 0.0f, scale ? scale[ch] : 1.0f, beta, ch);
    return yv > 0.0f ? gv : 0.0f;
}

template <typename T>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_bwd_partial(const T *y, const T *raw, const T *gy, int64_t rows,
                                                               int64_t stride, int c, const float *mean,
                                                               const float *scale, const float *gamma,
                                                               const float *beta, int act, int64_t rows_per_block,
                                                               double *part) {
    __shared__ double red[2][SHPL_BLOCK];
    int cc_n = 1;
    while (cc_n * 2 <= c && cc_n * 2 <= SHPL_BLOCK) cc_n *= 2;  // channels per pass (a power of two)
    const int rl_n = SHPL_BLOCK / cc_n, rl = threadIdx.x / cc_n, cc = threadIdx.x % cc_n;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    for (int c0 = 0; c0 < c; c0 += cc_n) {
        const int ch = c0 + cc;
        double s1 = 0.0, s2 = 0.0;
        if (ch < c) {
            const float m = mean ? mean[ch] : 0.0f;
            const float inv = scale ? __fdiv_rn(scale[ch], gamma ? gamma[ch] : 1.0f) : 1.0f;
            for (int64_t r = r0 + rl; r < r1; r += rl_n) {
                const int64_t o = r * stride + ch;
                const float gb = bn_gbn(y, raw, gy, o, ch, act, mean, scale, beta);
                const float xh = __fmul_rn(__fsub_rn(Elem<T>::f(raw[o]), m), inv);
                s1 += (double)gb;
                s2 += (double)gb * (double)xh;
            }
        }
        red[0][threadIdx.x] = s1;
        red[1][threadIdx.x] = s2;
        __syncthreads();
        if ((int)threadIdx.x < cc_n && c0 + (int)threadIdx.x < c) {
            double a = 0.0, b = 0.0;
            for (int k = 0; k < rl_n; ++k) {
                a += red[0][k * cc_n + threadIdx.x];
                b += red[1][k * cc_n + threadIdx.x];
            }
            part[((int64_t)blockIdx.x * 2 + 0) * c + c0 + threadIdx.x] = a;
            part[((int64_t)blockIdx.x * 2 + 1) * c + c0 + threadIdx.x] = b;
        }
        __syncthreads();
    }
}

// Vector form of k_bn_bwd_partial: thread (row lane rl, channel group cg)
// reads VEC channels of every rl_n-th row; c / VEC a power of two <= 256.
template <typename T>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_bwd_partial_vec(const T *y, const T *raw, const T *gy,
                                                                   int64_t rows, int64_t stride, int c,
                                                                   const float *mean, const float *scale,
                                                                   const float *gamma, const float *beta, int act,
                                                                   int64_t rows_per_block, double *part) {
    constexpr int VEC = 16 / sizeof(T);
    __shared__ double red[2][SHPL_BLOCK * VEC];
    const int cg_n = c / VEC, rl_n = SHPL_BLOCK / cg_n;
    const int rl = threadIdx.x / cg_n, cg = threadIdx.x % cg_n, ch0 = cg * VEC;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    float m[VEC], inv[VEC], sc[VEC], b[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        m[k] = mean ? mean[ch0 + k] : 0.0f;
        sc[k] = scale ? scale[ch0 + k] : 1.0f;
        inv[k] = scale ? __fdiv_rn(scale[ch0 + k], gamma ? gamma[ch0 + k] : 1.0f) : 1.0f;
        b[k] = beta ? beta[ch0 + k] : 0.0f;
    }
    double s1[VEC], s2[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) s1[k] = s2[k] = 0.0;
    // rows in flight per iteration (the sums stay in row order): bf16 4 (0.81 -> 0.73 ms per 64-frame
    // step; the apply kernels are slower with more, profiles/r02_bn_sweep.log)
    constexpr int U = sizeof(T) == 2 ? 4 : BN_U / 2;
    for (int64_t rb = r0 + rl; rb < r1; rb += U * rl_n) {
        float gv[U][VEC], xv[U][VEC], yv[U][VEC];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (rb + u * rl_n >= r1) break;
            const int64_t o = (rb + u * rl_n) * stride + ch0;
            Piece<T, VEC>::load(gy + o, gv[u]);
            Piece<T, VEC>::load(raw + o, xv[u]);
            if (act == 1 && y) Piece<T, VEC>::load(y + o, yv[u]);
        }
        // the sums in row order, as before
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (rb + u * rl_n >= r1) break;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                if (act == 1 && !y) {
                    const float t = __fmul_rn(__fsub_rn(xv[u][k], m[k]), sc[k]);
                    yv[u][k] = beta ? __fadd_rn(t, b[k]) : t;
                }
                const float gb = (act == 1 && !(yv[u][k] > 0.0f)) ? 0.0f : gv[u][k];
                const float xh = __fmul_rn(__fsub_rn(xv[u][k], m[k]), inv[k]);
                s1[k] += (double)gb;
                s2[k] += (double)gb * (double)xh;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        red[0][threadIdx.x * VEC + k] = s1[k];
        red[1][threadIdx.x * VEC + k] = s2[k];
    }
    __syncthreads();
    for (int ch = threadIdx.x; ch < c; ch += SHPL_BLOCK) {
        const int g2 = ch / VEC, k = ch % VEC;
        double a = 0.0, b = 0.0;
        for (int q = 0; q < rl_n; ++q) {
            a += red[0][(q * cg_n + g2) * VEC + k];
            b += red[1][(q * cg_n + g2) * VEC + k];
        }
        part[((int64_t)blockIdx.x * 2 + 0) * c + ch] = a;
        part[((int64_t)blockIdx.x * 2 + 1) * c + ch] = b;
    }
}

template <typename T, bool ACT, bool HASY, bool BETA, bool TRAIN>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_bwd_apply_vec(const T *y, const T *raw, const T *gy,
                                                                 int64_t rows, int64_t stride, int c,
                                                                 const float *mean, const float *scale,
                                                                 const float *gamma, const float *beta,
                                                                 const float *mean_terms, T *graw) {
    constexpr int VEC = 16 / sizeof(T);
    const int pr = c / VEC, rpb = SHPL_BLOCK / pr;
    const int ch0 = (threadIdx.x % pr) * VEC;
    float sc[VEC], m[VEC], inv[VEC], t0[VEC], t1[VEC], b[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const int ch = ch0 + k;
        b[k] = BETA ? beta[ch] : 0.0f;
        sc[k] = scale ? scale[ch] : 1.0f;
        m[k] = mean ? mean[ch] : 0.0f;
        inv[k] = __fdiv_rn(sc[k], gamma ? gamma[ch] : 1.0f);
        t0[k] = TRAIN ? mean_terms[ch] : 0.0f;
        t1[k] = TRAIN ? mean_terms[c + ch] : 0.0f;
    }
    const int64_t step = (int64_t)gridDim.x * rpb;
    constexpr int U = BN_U / 2;  // two or three streams in per row
    for (int64_t r0 = (int64_t)blockIdx.x * rpb + threadIdx.x / pr; r0 < rows; r0 += U * step) {
        float gv[U][VEC], yv[U][VEC], xv[U][VEC];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r0 + u * step >= rows) break;
            const int64_t o = (r0 + u * step) * stride + ch0;
            Piece<T, VEC>::load(gy + o, gv[u]);
            if constexpr (ACT && HASY) Piece<T, VEC>::load(y + o, yv[u]);
            if constexpr (TRAIN || (ACT && !HASY)) Piece<T, VEC>::load(raw + o, xv[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r0 + u * step >= rows) break;
            float out[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                if constexpr (ACT && !HASY) {
                    const float t = __fmul_rn(__fsub_rn(xv[u][k], m[k]), sc[k]);
                    yv[u][k] = BETA ? __fadd_rn(t, b[k]) : t;
                }
                const float gb = (ACT && !(yv[u][k] > 0.0f)) ? 0.0f : gv[u][k];
                if constexpr (TRAIN) {
                    const float xh = __fmul_rn(__fsub_rn(xv[u][k], m[k]), inv[k]);
                    out[k] = __fmul_rn(sc[k], __fsub_rn(__fsub_rn(gb, t0[k]), __fmul_rn(xh, t1[k])));
                } else {
                    out[k] = __fmul_rn(sc[k], gb);
                }
            }
            Piece<T, VEC>::store(graw + (r0 + u * step) * stride + ch0, out);
        }
    }
}

// one block per channel (strided_sum / block_sum above)
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_bwd_finalize(const double *part, int n_blocks, int c,
                                                                double count, float *dbeta, float *dgamma,
                                                                float *mean_terms) {
    __shared__ double red[SHPL_BLOCK / 64];
    const int ch = blockIdx.x;
    const double a = block_sum<SHPL_BLOCK>(strided_sum<SHPL_BLOCK>(part + ch, n_blocks, 2 * c, threadIdx.x), red);
    const double b =
        block_sum<SHPL_BLOCK>(strided_sum<SHPL_BLOCK>(part + c + ch, n_blocks, 2 * c, threadIdx.x), red);
    if (threadIdx.x == 0) {
        if (dbeta) dbeta[ch] = (float)a;
        if (dgamma) dgamma[ch] = (float)b;
        mean_terms[ch] = (float)(a / count);
        mean_terms[c + ch] = (float)(b / count);
    }
}

template <typename T>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bn_bwd_apply(const T *y, const T *raw, const T *gy, int64_t rows,
                                                             int64_t stride, int c, const float *mean,
                                                             const float *scale, const float *gamma, const float *beta,
                                                             int act, int training, const float *mean_terms, T *graw) {
    const int64_t total = rows * c;
    for (int64_t t = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * SHPL_BLOCK) {
        const int64_t r = t / c;
        const int ch = (int)(t - r * c);
        const int64_t o = r * stride + ch;
        const float gb = bn_gbn(y, raw, gy, o, ch, act, mean, scale, beta);
        const float sc = scale ? scale[ch] : 1.0f;
        float v;
        if (training) {
            const float inv = __fdiv_rn(sc, gamma ? gamma[ch] : 1.0f);
            const float xh = __fmul_rn(__fsub_rn(Elem<T>::f(raw[o]), mean ? mean[ch] : 0.0f), inv);
            v = __fmul_rn(sc, __fsub_rn(__fsub_rn(gb, mean_terms[ch]), __fmul_rn(xh, mean_terms[c + ch])));
        } else {
            v = __fmul_rn(sc, gb);
        }
        graw[o] = Elem<T>::back(v);
    }
}

// Weight gradient: dW[tap][ci][co] = sum over pixels p of x[p + tap offset][ci] * g[p][co].
// One workgroup per (group of output tiles, 32 input channels, 32 output
// channels). Per tile it stages the input halo of its 32 channels ([chunk]
// [pixel][32 B], unpadded) and the 8x32-pixel gradient tile ([pixel][32
// channels], raw) in LDS -- dense sources by LDS-DMA, the whole tile in one
// round trip; pooled channels recomputed from the CSR by stage_halo, so
// bv_fused need not exist -- and wave w accumulates the 9 taps over tile
// rows 2w, 2w+1 with v_mfma_f32_16x16x4_f32 (M = 16 input channels, N = 16
// output channels, K = 4 pixels; 2 x 2 blocks per tap). Lane group kq walks
// 16 consecutive pixels of one row, so the three kx taps of a (ky, channel)
// are a sliding window: one new LDS read per (ky, channel half) per step.
// ~76 KB of LDS (f32): two workgroups per CU, so one stages while the
// other multiplies. The four waves' sums and then the groups' partials are
// added in a fixed order (k_wgrad_reduce): deterministic. Measured and
// dropped: 32 channels per workgroup with padded rows at one workgroup per
// CU (3.3x the forward's time), 16 channels per workgroup (2x: the gradient
// tile and the run list staged once per 16 channels), a register-staged
// prefetch of the next tile's halo (2 %: 256 registers).
constexpr int WG_CI = 32;  // input channels per workgroup

typedef float f32x4v __attribute__((ext_vector_type(4)));

struct WgArgs {
    const void *gy;
    int64_t gy_stride;
    int n_cib, n_cob, tiles_per_group;
    bool vec_g;
    bool whole;   // every 16-byte piece of A, B and gy lies inside its row: unmasked vector loads
    float *part;  // [((group * n_cib + cib) * n_cob + cob)][9][32][32]
};

// Stages one tile's inputs of the weight gradient in LDS, as 16-byte pieces:
// HALO: the 10x34 halo of the workgroup's WG_CI input channels (dense
// sources), s_x [chunk][pixel][CB bytes]; always: the 8x32 gradient tile of
// output channels [cob*32, cob*32+32), s_g [pixel][32 channels] raw. With
// g.whole (every piece inside its row) each piece is one LDS-DMA
// (global_load_lds_dwordx4: no registers, the whole tile in one round trip,
// the destination lane-linear per wave); otherwise masked loads + ds_write.
// The caller waits (vmcnt(0)) and synchronises.
template <typename T, bool HALO>
__device__ __forceinline__ void wg_stage(const ConvArgs &p, const WgArgs &g, int f, int y0, int x0, int cib, int cob,
                                         uint8_t *s_x, uint8_t *s_g) {
    typedef Elem<T> E;
    constexpr int CK = E::CK, HE = E::HE, NP = E::NP, CB = E::CB, NQ = WG_CI / CK;
    constexpr int NPIX = HH * HWD, IN_PIECES = NPIX * NP;
    constexpr int GPP = NCO / HE, G_PIECES = TH * TW * GPP;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = p.h, W = p.w;
    const int64_t frame_row0 = (int64_t)f * H * W;
    const u32x4 *zero = &g_zero_piece;
    const u32x4 z = u32x4{0u, 0u, 0u, 0u};
    if constexpr (HALO) {
        const int Q = p.qa + p.qb;
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
            const int q = cib * NQ + j;
            // chunks past the last (q >= Q) are zeros, addressed in a source that exists
            const bool from_a = p.c_a > 0 && (q < p.qa || q >= Q);
            const T *src = reinterpret_cast<const T *>(from_a ? p.a : p.b) + (from_a ? p.a_off : p.b_off);
            const int64_t stride = from_a ? p.a_stride : p.b_stride;
            const int c_src = from_a ? p.c_a : p.c_b;
            const int c0 = (from_a ? q : q - p.qa) * CK;
            const bool vec = from_a ? p.vec_a : p.vec_b;
#pragma unroll
            for (int u = 0; u < (IN_PIECES + CONV_BLOCK - 1) / CONV_BLOCK; ++u) {
                const int base = u * CONV_BLOCK + wave * 64;  // the wave's first piece
                if (base >= IN_PIECES) break;
                const int jj = base + lane;
                const int pix = jj / NP, hr = pix / HWD, hc = pix - hr * HWD;
                const int y = y0 - 1 + hr, xx = x0 - 1 + hc;
                const bool ok = q < Q && jj < IN_PIECES && y >= 0 && y < H && xx >= 0 && xx < W;
                const int64_t row = frame_row0 + (int64_t)y * W + xx;
                const int c = c0 + (jj % NP) * HE;
                uint8_t *dst = s_x + j * NPIX * CB + base * 16;
                if (jj < IN_PIECES) {
                    if (g.whole)
                        __builtin_amdgcn_global_load_lds(ok ? reinterpret_cast<const u32x4 *>(src + row * stride + c) : zero,
                                                         dst, 16, 0, 0);
                    else
                        *reinterpret_cast<u32x4 *>(dst + lane * 16) = ok ? load_piece<T>(src + row * stride, c, c_src, vec) : z;
                }
            }
        }
    }
    const T *gy = reinterpret_cast<const T *>(g.gy);
#pragma unroll
    for (int u = 0; u < G_PIECES / CONV_BLOCK; ++u) {
        const int base = u * CONV_BLOCK + wave * 64;
        const int i = base + lane;
        const int pix = i / GPP, pc = i - pix * GPP;
        const int y = y0 + pix / TW, xx = x0 + pix % TW;
        const bool ok = y < H && xx < W;
        const int64_t row = frame_row0 + (int64_t)y * W + xx;
        const int c = cob * NCO + pc * HE;
        uint8_t *dst = s_g + base * 16;
        if (g.whole)
            __builtin_amdgcn_global_load_lds(ok ? reinterpret_cast<const u32x4 *>(gy + row * g.gy_stride + c) : zero, dst,
                                             16, 0, 0);
        else
            *reinterpret_cast<u32x4 *>(dst + lane * 16) = ok ? load_piece<T>(gy + row * g.gy_stride, c, p.c_out, g.vec_g) : z;
    }
    static_assert(G_PIECES % CONV_BLOCK == 0, "gradient pieces");
}

template <typename T, bool POOLED>
__global__ __launch_bounds__(CONV_BLOCK, POOLED ? 1 : 2) void k_conv3x3_wgrad(const ConvArgs p, const WgArgs g) {
    typedef Elem<T> E;
    constexpr int CK = E::CK, CB = E::CB, NQ = WG_CI / CK;
    constexpr int NPIX = HH * HWD;
    __shared__ __attribute__((aligned(16))) uint8_t s_x[NQ * NPIX * CB];
    __shared__ __attribute__((aligned(16))) uint8_t s_g[TH * TW * NCO * sizeof(T)];
    SHPL_HALO_RUNS_LDS(POOLED, HH)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, kq = lane >> 4;
    const int grp = blockIdx.x, cib = blockIdx.y, cob = blockIdx.z;
    const int Q = p.qa + p.qb;
    f32x4v acc[9][2][2];  // [tap][input-channel half][output-channel half]
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int o = 0; o < 2; ++o) acc[t][h][o] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    const int t0 = grp * g.tiles_per_group;
    const int t1 = t0 + g.tiles_per_group < p.n_tiles ? t0 + g.tiles_per_group : p.n_tiles;
    // this lane's input channels (rows of A): h*16 + l16 -> chunk (h*16 + l16) / CK, element % CK
    int a_off[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) a_off[h] = ((h * 16 + l16) / CK) * NPIX * CB + ((h * 16 + l16) % CK) * (int)sizeof(T);
    for (int tile = t0; tile < t1; ++tile) {
        const int f = tile / p.tiles_per_frame;
        const int t_in = tile - f * p.tiles_per_frame;
        const int ty = t_in / p.tiles_x, tx = t_in - ty * p.tiles_x;
        const int y0 = ty * TH, x0 = tx * TW;
        if constexpr (POOLED) {
            const int n_run = find_runs(p, f, y0, x0, runs);
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const int q = cib * NQ + j;
                if (q < Q) stage_halo<T, POOLED, CB>(p, q, f, y0, x0, s_x + j * NPIX * CB, runs, n_run);
            }
        }
        wg_stage<T, !POOLED>(p, g, f, y0, x0, cib, cob, s_x, s_g);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMAs have landed
        __syncthreads();
        // lane group kq walks tile row 2w + (kq >> 1), columns (kq & 1) * 16 + sp, sp = 0..15: the
        // three kx taps of a (ky, channel) are a sliding window over the halo row, so each
        // step reads one new input value per (ky, channel half) instead of three
        const int r = 2 * wave + (kq >> 1), cb = (kq & 1) * 16;
        float win[3][2][3];  // [ky][h][kx]: x at halo (r + ky, cb + sp + kx), channel h*16 + l16
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int kx = 0; kx < 2; ++kx)
                    win[ky][h][kx] = E::f(*reinterpret_cast<const T *>(s_x + a_off[h] + ((r + ky) * HWD + cb + kx) * CB));
#pragma unroll 2
        for (int sp = 0; sp < 16; ++sp) {
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    win[ky][h][2] =
                        E::f(*reinterpret_cast<const T *>(s_x + a_off[h] + ((r + ky) * HWD + cb + sp + 2) * CB));
            float b[2];
#pragma unroll
            for (int o = 0; o < 2; ++o)
                b[o] = E::f(reinterpret_cast<const T *>(s_g)[(r * TW + cb + sp) * NCO + o * 16 + l16]);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int o = 0; o < 2; ++o)
                            acc[ky * 3 + kx][h][o] =
                                __builtin_amdgcn_mfma_f32_16x16x4f32(win[ky][h][kx], b[o], acc[ky * 3 + kx][h][o], 0, 0, 0);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    win[ky][h][0] = win[ky][h][1];
                    win[ky][h][1] = win[ky][h][2];
                }
        }
        __syncthreads();
    }
    // the four waves' sums, in wave order, into this workgroup's partial
    // (D of 16x16x4: column = lane & 15 (output channel), row = 4 (lane >> 4) + reg (input channel))
    float *red = reinterpret_cast<float *>(s_x);  // 4 x 1024 floats
    float *out = g.part + (((int64_t)grp * g.n_cib + cib) * g.n_cob + cob) * (9 * WG_CI * NCO);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int o = 0; o < 2; ++o)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    red[wave * 1024 + (h * 16 + 4 * kq + i) * NCO + o * 16 + l16] = acc[t][h][o][i];
        __syncthreads();
        for (int e = tid; e < WG_CI * NCO; e += CONV_BLOCK)
            out[t * 1024 + e] = __fadd_rn(__fadd_rn(__fadd_rn(red[e], red[1024 + e]), red[2048 + e]), red[3072 + e]);
        __syncthreads();
    }
}

// bf16 weight gradient on bf16 MFMA (v_mfma_f32_16x16x32_bf16: M = 16 input
// channels, N = 16 output channels, K = 32 pixels of one tile row). K runs
// along each lane's registers, so the staging transposes: the halo goes to
// LDS as [kx][channel][halo row][32 columns] -- three copies shifted by the
// tap's kx, so that every A fragment (8 pixels of one channel) is one
// aligned ds_read_b128 -- and the gradient tile as [co][row][32 columns]; the
// channel pitches are padded by 16 bytes (16 lanes' reads on distinct bank
// quads). Dense sources only (the pooled form stays on k_conv3x3_wgrad).
// Products of bf16 values are exact in f32; sums in f32 per workgroup, the
// same partials and k_wgrad_reduce as k_conv3x3_wgrad. Staging goes through
// registers, synchronously (one round trip per tile; two workgroups per CU).
// Measured and dropped: loading the next tile's pieces under this tile's
// MFMAs (4.50 -> 4.57 ms, 167 -> 197 VGPRs).
constexpr int WB_CIP = HH * TW * 2 + 16;  // bytes per input channel of one kx copy (10 rows x 32 bf16 + pad)
constexpr int WB_KXS = WG_CI * WB_CIP;    // bytes per kx copy
constexpr int WB_COP = TH * TW * 2 + 16;  // bytes per output channel of the gradient tile

__global__ __launch_bounds__(CONV_BLOCK, 2) void k_wgrad_bf16(const ConvArgs p, const WgArgs g) {
    typedef Elem<uint16_t> E;
    constexpr int CK = E::CK, HE = E::HE, NQ = WG_CI / CK;  // 16 channels per chunk, 2 chunks
    constexpr int IN_PIECES = NQ * HH * HWD * 2;              // (chunk, halo pixel, 8-channel piece)
    constexpr int IN_IT = (IN_PIECES + CONV_BLOCK - 1) / CONV_BLOCK;
    constexpr int G_PIECES = TH * TW * (NCO / HE);            // (pixel, 8-channel piece)
    constexpr int G_IT = G_PIECES / CONV_BLOCK;
    __shared__ __attribute__((aligned(16))) uint8_t s_x[3 * WB_KXS];
    __shared__ __attribute__((aligned(16))) uint8_t s_g[NCO * WB_COP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, kq = lane >> 4;
    const int grp = blockIdx.x, cib = blockIdx.y, cob = blockIdx.z;
    const int Q = p.qa + p.qb;
    const int H = p.h, W = p.w;
    const uint16_t *gy = reinterpret_cast<const uint16_t *>(g.gy);
    // wave w owns input-channel half h = w >> 1 and output-channel half o = w & 1, all 8 rows and 9 taps
    const int h = wave >> 1, o = wave & 1;
    f32x4v acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    const int t0 = grp * g.tiles_per_group;
    const int t1 = t0 + g.tiles_per_group < p.n_tiles ? t0 + g.tiles_per_group : p.n_tiles;
    const u32x4 z = u32x4{0u, 0u, 0u, 0u};
    u32x4 xv[IN_IT], gv[G_IT];
    // the tile's pieces into registers, issued together
    auto load = [&](int tile) {
        const int f = tile / p.tiles_per_frame;
        const int t_in = tile - f * p.tiles_per_frame;
        const int ty = t_in / p.tiles_x, tx = t_in - ty * p.tiles_x;
        const int y0 = ty * TH, x0 = tx * TW;
        const int64_t frame_row0 = (int64_t)f * H * W;
#pragma unroll
        for (int u = 0; u < IN_IT; ++u) {
            const int j = tid + u * CONV_BLOCK;
            const int q = cib * NQ + j / (HH * HWD * 2);
            const int rem = j % (HH * HWD * 2), pix = rem >> 1, pc = rem & 1;
            const int hr = pix / HWD, hc = pix - hr * HWD;
            const int y = y0 - 1 + hr, x = x0 - 1 + hc;
            const bool ok = j < IN_PIECES && q < Q && y >= 0 && y < H && x >= 0 && x < W;
            const bool from_a = p.c_a > 0 && (q < p.qa || q >= Q);
            const uint16_t *src = reinterpret_cast<const uint16_t *>(from_a ? p.a : p.b) + (from_a ? p.a_off : p.b_off);
            const int64_t row = ok ? frame_row0 + (int64_t)y * W + x : frame_row0;
            const int c = ok ? (from_a ? q : q - p.qa) * CK + pc * HE : 0;
            if (g.whole) {  // unmasked, branch-free: out-of-map pieces read row 0 and are zeroed
                const u32x4 v = *reinterpret_cast<const u32x4 *>(src + row * (from_a ? p.a_stride : p.b_stride) + c);
                xv[u] = ok ? v : z;
            } else {
                xv[u] = ok ? load_piece<uint16_t>(src + row * (from_a ? p.a_stride : p.b_stride), c,
                                                  from_a ? p.c_a : p.c_b, from_a ? p.vec_a : p.vec_b)
                           : z;
            }
        }
#pragma unroll
        for (int u = 0; u < G_IT; ++u) {
            const int i = tid + u * CONV_BLOCK;
            const int pix = i / (NCO / HE), pc = i % (NCO / HE);
            const int y = y0 + pix / TW, x = x0 + pix % TW;
            const bool ok = y < H && x < W;
            const int64_t row = ok ? frame_row0 + (int64_t)y * W + x : frame_row0;
            if (g.whole) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(gy + row * g.gy_stride + cob * NCO + pc * HE);
                gv[u] = ok ? v : z;
            } else {
                gv[u] = ok ? load_piece<uint16_t>(gy + row * g.gy_stride, cob * NCO + pc * HE, p.c_out, g.vec_g) : z;
            }
        }
    };
    for (int tile = t0; tile < t1; ++tile) {
        load(tile);
        // ---- transposed writes: halo pixel (hr, hc) feeds column hc - kx of copy kx
#pragma unroll
        for (int u = 0; u < IN_IT; ++u) {
            const int j = tid + u * CONV_BLOCK;
            if (j >= IN_PIECES) continue;
            const int jq = j / (HH * HWD * 2);
            const int rem = j % (HH * HWD * 2), pix = rem >> 1, pc = rem & 1;
            const int hr = pix / HWD, hc = pix - hr * HWD;
            uint16_t e[HE];
            __builtin_memcpy(e, &xv[u], 16);
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int c = hc - kx;
                if (c < 0 || c >= TW) continue;
                uint8_t *base = s_x + kx * WB_KXS + (jq * CK + pc * HE) * WB_CIP + (hr * TW + c) * 2;
#pragma unroll
                for (int k = 0; k < HE; ++k) *reinterpret_cast<uint16_t *>(base + k * WB_CIP) = e[k];
            }
        }
#pragma unroll
        for (int u = 0; u < G_IT; ++u) {
            const int i = tid + u * CONV_BLOCK;
            const int pix = i / (NCO / HE), pc = i % (NCO / HE);
            uint16_t e[HE];
            __builtin_memcpy(e, &gv[u], 16);
            uint8_t *base = s_g + (pc * HE) * WB_COP + pix * 2;
#pragma unroll
            for (int k = 0; k < HE; ++k) *reinterpret_cast<uint16_t *>(base + k * WB_COP) = e[k];
        }
        __syncthreads();
        // ---- one K step (the 32 pixels of a tile row) per row and tap
#pragma unroll 2
        for (int r = 0; r < TH; ++r) {
            const bf16x8 b = *reinterpret_cast<const bf16x8 *>(s_g + (o * 16 + l16) * WB_COP + (r * TW + kq * 8) * 2);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const bf16x8 a = *reinterpret_cast<const bf16x8 *>(
                        s_x + kx * WB_KXS + (h * 16 + l16) * WB_CIP + ((r + ky) * TW + kq * 8) * 2);
                    acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[ky * 3 + kx], 0, 0, 0);
                }
        }
        __syncthreads();
    }
    // this wave's block of the workgroup's partial
    // (D of 16x16x32: column = lane & 15 (output channel), row = 4 (lane >> 4) + reg (input channel))
    float *out = g.part + (((int64_t)grp * g.n_cib + cib) * g.n_cob + cob) * (9 * WG_CI * NCO);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) out[t * 1024 + (h * 16 + 4 * kq + i) * NCO + o * 16 + l16] = acc[t][i];
}

// dW (f32, HWIO [3][3][c_a+c_b][c_out]) = the groups' partials summed in
// group order (f64), channels mapped back from the chunk layout.
// dW[tap][ci][co] = sum over the n_groups partials, in group order. A block
// takes 32 consecutive outputs; its 8 lane groups walk every 8th group (4
// independent accumulators each, 4 loads in flight) and their sums are
// added in lane-group order: deterministic.
constexpr int WR_OUT = 32, WR_K = SHPL_BLOCK / WR_OUT;
__global__ __launch_bounds__(SHPL_BLOCK) void k_wgrad_reduce(const float *part, int n_groups, int n_cib, int n_cob,
                                                             int c_a, int c_b, int qa, int ck, int c_out, float *dw) {
    __shared__ double red[WR_K][WR_OUT];
    const int cin = c_a + c_b;
    const int64_t total = (int64_t)9 * cin * c_out;
    const int j = threadIdx.x % WR_OUT, kk = threadIdx.x / WR_OUT;
    for (int64_t t0 = (int64_t)blockIdx.x * WR_OUT; t0 < total; t0 += (int64_t)gridDim.x * WR_OUT) {
        const int64_t t = t0 + j;
        double sum = 0.0;
        if (t < total) {
            const int co = (int)(t % c_out);
            const int ci = (int)((t / c_out) % cin);
            const int tap = (int)(t / ((int64_t)c_out * cin));
            const int cs = ci < c_a ? ci : qa * ck + (ci - c_a);  // channel in the chunk layout
            const int cib = cs / WG_CI, cil = cs % WG_CI, cob = co / NCO, col = co % NCO;
            const int64_t gstride = (int64_t)n_cib * n_cob * (9 * WG_CI * NCO);  // one group further
            const float *v = part + ((int64_t)cib * n_cob + cob) * (9 * WG_CI * NCO) + tap * (WG_CI * NCO) +
                             cil * NCO + col;
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
            int k = kk;
            for (; k + 3 * WR_K < n_groups; k += 4 * WR_K) {
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] += (double)v[(int64_t)(k + u * WR_K) * gstride];
            }
            for (int u = 0; k < n_groups; k += WR_K, ++u) acc[u & 3] += (double)v[(int64_t)k * gstride];
            sum = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        }
        red[kk][j] = sum;
        __syncthreads();
        if (kk == 0 && t < total) {
            double s2 = red[0][j];
            for (int q = 1; q < WR_K; ++q) s2 += red[q][j];
            dw[t] = (float)s2;
        }
        __syncthreads();
    }
}

struct ConvPlan {
    int ck, qa, qb, n_cob, tiles_x, tiles_y, tiles_per_frame;
    int64_t n_tiles;
    size_t wp_bytes, rp_bytes, part_bytes, total;
    // k_conv_rows (bf16, at most 4 input chunks): band rows, bands per frame,
    // occupancy words per BEV row; the pooled runs' buffers (pooled only)
    bool rows;
    int band, n_bands, wpr;
    size_t occ_bytes, cmp_bytes, junk_bytes;
    // k_conv_wide (bf16, input chunks of 64 channels, whole 256-channel output blocks, no statistics); pooled:
    // the pooled map materialised in the workspace (map_bytes) by shpl_pull first
    bool wide, wide_cmp;
    size_t map_bytes;
    int64_t pool_cap;
};

#ifndef SHPL_CONV_ROWS
#define SHPL_CONV_ROWS 1  // 0: the tiled kernel for every forward (A/B builds)
#endif
#ifndef SHPL_CONV_WIDE
#define SHPL_CONV_WIDE 1  // 0: wide bf16 convs on the tiled kernel (A/B builds)
#endif
#ifndef SHPL_ROWS_BAND
#define SHPL_ROWS_BAND 0  // 0: about 60 rows, equal bands (k_conv_rows stages band + 2 rows, at most 64)
#endif

// th: output tile rows -- the forward's ConvTile (8 f32, 16 bf16) unless the
// weight gradient asks for its own 8. pool_cap: the pooling CSR's entry
// capacity (pooled forward: sizes the compact buffer of pooled runs).
int conv_plan(int dtype, int n_frames, int64_t h, int64_t w, int64_t c_a, int64_t c_b, int64_t c_out, bool pooled,
              bool stats, ConvPlan *pl, int th = 0, int64_t pool_cap = 0) {
    if (dtype != SHPL_F32 && dtype != SHPL_BF16) return SHPL_ERR_ARG;
    if (n_frames < 0 || h < 0 || w < 0 || c_a < 0 || c_b < 0 || c_out < 1 || c_a + c_b < 1) return SHPL_ERR_BAD_SHAPE;
    if (h > (1 << 20) || w > (1 << 20) || c_a + c_b > (1 << 16) || c_out > (1 << 16)) return SHPL_ERR_BAD_SHAPE;
    if (pool_cap < 0 || pool_cap >= (1LL << 31)) return SHPL_ERR_BAD_SHAPE;
    const int esz = dtype == SHPL_F32 ? 4 : 2;
    const int chunk_b = 32;  // Elem<T>::CB
    pl->ck = chunk_b / esz;
    pl->qa = (int)((c_a + pl->ck - 1) / pl->ck);
    pl->qb = (int)((c_b + pl->ck - 1) / pl->ck);
    pl->n_cob = (int)((c_out + NCO - 1) / NCO);
    pl->tiles_x = (int)((w + TW - 1) / TW);
    if (th == 0) th = dtype == SHPL_F32 ? ConvTile<float>::TH : ConvTile<uint16_t>::TH;
    pl->tiles_y = (int)((h + th - 1) / th);
    pl->tiles_per_frame = pl->tiles_x * pl->tiles_y;
    pl->n_tiles = (int64_t)n_frames * pl->tiles_per_frame;
    if (pl->n_tiles >= (1LL << 31) || (int64_t)n_frames * h * w >= (1LL << 31)) return SHPL_ERR_BAD_SHAPE;
    pl->wp_bytes = align_up((size_t)pl->n_cob * (pl->qa + pl->qb) * W_ROWS * chunk_b, 256);
    pl->rp_bytes = pooled ? align_up((size_t)n_frames * (h + 1) * 4, 256) : 0;
    pl->part_bytes = stats ? align_up((size_t)pl->n_cob * NCO * 2 * pl->n_tiles * 8, 256) : 0;
    pl->wpr = (int)((w + 31) / 32);
    pl->rows = SHPL_CONV_ROWS && dtype == SHPL_BF16 && pl->qa + pl->qb <= 4 && c_a % 8 == 0 && c_b % 8 == 0 && h > 0 &&
               w > 0 && rows::supported(pl->qa + pl->qb, pl->qa) &&
               (!pooled || (h * pl->wpr <= rows::OCC_MAX_WORDS && pool_cap * c_b * esz < (1LL << 31)));
    pl->n_bands = (int)((h + 59) / 60);
    pl->band = (int)((h + pl->n_bands - 1) / pl->n_bands);
    if (SHPL_ROWS_BAND > 0 && SHPL_ROWS_BAND <= 62) {
        pl->band = SHPL_ROWS_BAND;
        pl->n_bands = (int)((h + pl->band - 1) / pl->band);
    }
    if ((int64_t)n_frames * pl->n_bands * pl->tiles_x >= (1LL << 31)) pl->rows = false;
    // statistics partials: one per tile (tiled kernel) or per item (k_conv_rows, SHPL_ROWS_BAND may cut more
    // bands than there are tile rows)
    if (stats && pl->rows) {
        const int64_t n_items = (int64_t)n_frames * pl->n_bands * pl->tiles_x;
        if (n_items > pl->n_tiles) pl->part_bytes = align_up((size_t)pl->n_cob * NCO * 2 * n_items * 8, 256);
    }
    pl->occ_bytes = pl->rows && pooled ? 2 * align_up((size_t)n_frames * h * pl->wpr * 4, 256) : 0;
    pl->pool_cap = pool_cap;
    pl->cmp_bytes = pl->rows && pooled ? align_up((size_t)pool_cap * c_b * esz, 256) : 0;
    pl->junk_bytes = pl->rows ? 32 * NCO * 2 : 0;
    pl->wide = SHPL_CONV_WIDE && dtype == SHPL_BF16 && !stats && !pl->rows && h > 0 && w > 0 &&
               wide::supported(c_a, c_b, c_out) && (int64_t)n_frames * h * w * (c_b > 0 ? c_b : 1) < (1LL << 40);
    pl->map_bytes = 0;
    pl->wide_cmp = false;
    if (pl->wide) {
        const size_t wb = align_up(wide::packed_bytes(c_a, c_b, c_out), 256);
        if (wb > pl->wp_bytes) pl->wp_bytes = wb;
        // pooled: the occupancy words + prefixes and the compact pooled runs (wide::prep), read by the halo
        // staging -- or, past the occupancy table's limits, the pooled map materialised by shpl_pull
        pl->wide_cmp = pooled && h * pl->wpr <= rows::OCC_MAX_WORDS && pool_cap * c_b * 2 < (1LL << 31);
        if (pooled && pl->wide_cmp)
            pl->map_bytes = 2 * align_up((size_t)n_frames * h * pl->wpr * 4, 256) + align_up((size_t)pool_cap * c_b * 2, 256);
        else if (pooled)
            pl->map_bytes = align_up((size_t)n_frames * h * w * c_b * 2, 256);
    }
    pl->total = pl->wp_bytes + pl->rp_bytes + pl->part_bytes + pl->occ_bytes + pl->cmp_bytes + pl->junk_bytes +
                pl->map_bytes;
    return SHPL_OK;
}

bool aligned16(const void *ptr) { return ((uintptr_t)ptr & 15u) == 0; }

// k_conv_rows (shpl_conv_rows.hip) and, pooled, its two preparatory launches
// (occupancy words + prefix counts per frame; the pooled vector of every run
// into the compact buffer). The packed weights are already in a.wp.
int conv_rows_launch(const ConvPlan &pl, const ConvArgs &a, bool pooled, bool stats, const int64_t *frame_off,
                     double *d_stats, hipStream_t s) {
    rows::RowArgs r = {};
    r.a = reinterpret_cast<const uint16_t *>(a.a) + a.a_off;
    r.b = reinterpret_cast<const uint16_t *>(a.b) + a.b_off;
    r.a_stride = a.a_stride;
    r.b_stride = a.b_stride;
    r.c_a = a.c_a;
    r.c_b = a.c_b;
    r.h = a.h;
    r.w = a.w;
    r.strips = pl.tiles_x;
    r.band = pl.band;
    r.n_bands = pl.n_bands;
    r.n_items = a.n_frames * pl.n_bands * pl.tiles_x;
    r.wp = reinterpret_cast<const uint16_t *>(a.wp);
    r.center = a.center;
    r.scale = a.scale;
    r.shift = a.shift;
    r.out = reinterpret_cast<uint16_t *>(a.out);
    r.out_stride = a.out_stride;
    r.wpr = pl.wpr;
    r.frame_off = frame_off;
    r.out2 = reinterpret_cast<uint16_t *>(a.out2);
    r.out2_stride = a.out2_stride;
    r.c_split = a.c_split;
    r.occ2 = a.occ2;
    r.n_cob = pl.n_cob;
    r.part = stats ? a.part : nullptr;  // n_items <= n_tiles: the tiled plan's partials hold the rows kernel's
    uint8_t *ws = reinterpret_cast<uint8_t *>(const_cast<void *>(a.wp)) + pl.wp_bytes + pl.rp_bytes + pl.part_bytes;
    r.junk = reinterpret_cast<uint16_t *>(ws + pl.occ_bytes + pl.cmp_bytes);
    if (pooled) {
        uint32_t *occ = reinterpret_cast<uint32_t *>(ws);
        int32_t *occ_base = reinterpret_cast<int32_t *>(ws + pl.occ_bytes / 2);
        uint16_t *cmp = reinterpret_cast<uint16_t *>(ws + pl.occ_bytes);
        const int rc = rows::prep_pooled(a.n_frames, a.h, a.w, pl.wpr, a.ent_dst, a.ent_src, a.ent_val, pl.pool_cap,
                                         frame_off, reinterpret_cast<const uint16_t *>(a.b), a.b_stride, a.b_off,
                                         a.c_b, occ, occ_base, cmp, s);
        if (rc) return rc;
        r.occ = occ;
        r.occ_base = occ_base;
        r.cmp = cmp;
    }
    int rc = rows::launch(r, pl.qa + pl.qb, pl.qa, pooled, a.act == 1, stats, s);
    if (rc || !stats) return rc;
    hipLaunchKernelGGL(k_stats_reduce, dim3(pl.n_cob * NCO * 2), dim3(RED_BLOCK), 0, s, a.part, r.n_items, a.c_out,
                       d_stats);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

// Whether a bf16 call with this plan and these arguments runs the row-streaming form (k_conv_rows, and pooled
// its prep: the occupancy maps and per-run pooled rows in the workspace). The one predicate conv_launch and
// shpl_conv3x3_rows_form (which the weight gradient's reuse of the forward's workspace hangs on) share.
bool rows_forward(const ConvPlan &pl, const ConvArgs &a, bool pooled, bool stats) {
    return pl.rows && a.vec_a && (a.c_b == 0 || a.vec_b) && (!a.out2 || a.c_split % NCO == 0) && a.vec_out &&
           a.c_out % NCO == 0 && a.n_frames > 0 &&
           (!stats || (a.act == 0 && rows::supported_st(pl.qa + pl.qb, pl.qa, pooled)));
}

// The wide bf16 form (k_conv_wide): pooled, the pooled map first into the workspace's last region by
// shpl_pull (the same arithmetic as the tiled staging: the conv of [a || map] is the fused conv's).
int conv_wide_launch(const ConvPlan &pl, const ConvArgs &a, const shpl_csr *pool, const int64_t *frame_off,
                     const void *w, hipStream_t s) {
    wide::WideArgs r = {};
    r.a = reinterpret_cast<const uint16_t *>(a.a) + a.a_off;
    r.a_stride = a.a_stride;
    r.c_a = a.c_a;
    r.c_b = a.c_b;
    if (pool && pl.wide_cmp) {
        uint8_t *ws = reinterpret_cast<uint8_t *>(const_cast<void *>(a.wp)) + pl.total - pl.map_bytes;
        const size_t ob = align_up((size_t)a.n_frames * a.h * pl.wpr * 4, 256);
        uint32_t *occ = reinterpret_cast<uint32_t *>(ws);
        int32_t *occ_base = reinterpret_cast<int32_t *>(ws + ob);
        uint16_t *cmp = reinterpret_cast<uint16_t *>(ws + 2 * ob);
        const int rc = wide::prep(a.n_frames, a.h, a.w, pl.wpr, pool->ent_dst, pool->ent_src, pool->ent_val,
                                  pool->nnz_cap, frame_off, reinterpret_cast<const uint16_t *>(a.b), a.b_stride, a.b_off,
                                  a.c_b, occ, occ_base, cmp, s);
        if (rc) return rc;
        r.occ = occ;
        r.occ_base = occ_base;
        r.frame_off = frame_off;
        r.cmp = cmp;
        r.wpr = pl.wpr;
    } else if (pool) {
        uint16_t *map = reinterpret_cast<uint16_t *>(reinterpret_cast<uint8_t *>(const_cast<void *>(a.wp)) + pl.total -
                                                     pl.map_bytes);
        const int rc = shpl_pull(SHPL_BY_CELL, SHPL_BF16, pool, a.b, a.b_stride, a.b_off, a.c_b, nullptr, 0, 0, 0,
                                 SHPL_OUT_POOL, map, a.c_b, s);
        if (rc) return rc;
        r.b = map;
        r.b_stride = a.c_b;
    } else {
        r.b = a.c_b > 0 ? reinterpret_cast<const uint16_t *>(a.b) + a.b_off : nullptr;
        r.b_stride = a.b_stride;
    }
    r.n_frames = a.n_frames;
    r.h = a.h;
    r.w = a.w;
    r.center = a.center;
    r.scale = a.scale;
    r.shift = a.shift;
    r.act = a.act;
    r.out = reinterpret_cast<uint16_t *>(a.out);
    r.out_stride = a.out_stride;
    r.c_out = a.c_out;
    return wide::launch(r, reinterpret_cast<const uint16_t *>(w),
                        reinterpret_cast<uint16_t *>(const_cast<void *>(a.wp)), s);
}

template <typename T>
int conv_launch(const ConvPlan &pl, ConvArgs &a, bool pooled, bool stats, const void *w, const int64_t *frame_off,
                double *d_stats, hipStream_t s, int transpose = 0, const shpl_csr *pool = nullptr) {
    if constexpr (sizeof(T) == 2) {
        if (pl.wide && !stats && !transpose && !a.out2 && a.vec_a && (a.c_b == 0 || a.vec_b) && a.vec_out &&
            a.n_frames > 0 && (!pooled || pool))
            return conv_wide_launch(pl, a, pooled ? pool : nullptr, frame_off, w, s);
    }
    T *wp = reinterpret_cast<T *>(const_cast<void *>(a.wp));
    const int64_t wtot = (int64_t)pl.n_cob * (pl.qa + pl.qb) * W_ROWS * Elem<T>::CK;
    hipLaunchKernelGGL(k_pack_w<T>, dim3(grid_for(wtot, SHPL_BLOCK, 4096)), dim3(SHPL_BLOCK), 0, s,
                       reinterpret_cast<const T *>(w), a.c_a, pl.qa, a.c_b, pl.qb, a.c_out, pl.n_cob, transpose, wp);
    SHPL_LAUNCH_CHECK();
    if constexpr (sizeof(T) == 2) {
        // bf16 with at most 64 input channels: the row-streaming kernel (k_conv_rows), also for the input
        // gradient's two maps (split at a whole output block) and the training forward's statistics
        if (rows_forward(pl, a, pooled, stats)) return conv_rows_launch(pl, a, pooled, stats, frame_off, d_stats, s);
    }
    if (pooled) {
        hipLaunchKernelGGL(k_row_ptr, dim3(16, a.n_frames), dim3(SHPL_BLOCK), 0, s, a.ent_dst, frame_off, a.h, a.w,
                           const_cast<int32_t *>(a.row_ptr));
        SHPL_LAUNCH_CHECK();
    }
    const dim3 grid((unsigned)pl.n_tiles, (unsigned)pl.n_cob);
    // f32, an even number of dense output blocks (the input gradient's 64
    // channels): two per workgroup, 12.11 -> 11.47 ms at 64 frames. bf16 gains
    // nothing (2.73 / 2.77 ms: 3 waves per SIMD instead of 6 for a
    // memory-pipeline-bound kernel) and keeps one.
    const bool pair = sizeof(T) == 4 && !pooled && !stats && pl.n_cob % 2 == 0;
    if (pooled) {
        if (stats)
            hipLaunchKernelGGL((k_conv3x3<T, true, true>), grid, dim3(CONV_BLOCK), 0, s, a);
        else
            hipLaunchKernelGGL((k_conv3x3<T, true, false>), grid, dim3(CONV_BLOCK), 0, s, a);
    } else {
        if (stats)
            hipLaunchKernelGGL((k_conv3x3<T, false, true>), grid, dim3(CONV_BLOCK), 0, s, a);
        else if (pair)
            hipLaunchKernelGGL((k_conv3x3<T, false, false, 2>), dim3(grid.x, grid.y / 2), dim3(CONV_BLOCK), 0, s, a);
        else
            hipLaunchKernelGGL((k_conv3x3<T, false, false>), grid, dim3(CONV_BLOCK), 0, s, a);
    }
    SHPL_LAUNCH_CHECK();
    if (stats) {
        hipLaunchKernelGGL(k_stats_reduce, dim3(pl.n_cob * NCO * 2), dim3(RED_BLOCK), 0, s, a.part, (int)pl.n_tiles,
                           a.c_out, d_stats);
        SHPL_LAUNCH_CHECK();
    }
    return SHPL_OK;
}

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_conv3x3_workspace_bytes(int dtype, int n_frames, int64_t h, int64_t w, int64_t c_a, int64_t c_b,
                                            int64_t c_out, int64_t pool_nnz_cap, int stats, size_t *bytes) {
    if (!bytes) return SHPL_ERR_ARG;
    ConvPlan pl;
    const bool pooled = pool_nnz_cap >= 0;
    const int rc = conv_plan(dtype, n_frames, h, w, c_a, c_b, c_out, pooled, stats != 0, &pl, 0,
                             pooled ? pool_nnz_cap : 0);
    if (rc) return rc;
    *bytes = pl.total;
    return SHPL_OK;
}

namespace shpl {
namespace {
// shpl_conv3x3's argument checks and kernel arguments (shared with shpl_conv3x3_rows_form). *empty: no pixel.
int forward_setup(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride, int64_t a_off,
                  int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off, int64_t c_b, const shpl_csr *pool,
                  const int64_t *d_frame_off, const void *d_weights, int64_t c_out, const float *d_center,
                  const float *d_scale, const float *d_shift, int act, void *d_out, int64_t out_stride,
                  bool stats, void *d_ws, size_t ws_bytes, bool check_ws, ConvPlan &pl, ConvArgs &a, bool *empty) {
    const bool pooled = pool != nullptr;
    *empty = false;
    int rc = conv_plan(dtype, n_frames, h, w, c_a, c_b, c_out, pooled, stats, &pl, 0, pooled ? pool->nnz_cap : 0);
    if (rc) return rc;
    if (act != 0 && act != 1) return SHPL_ERR_ARG;
    if (!d_weights || (check_ws && ws_bytes > 0 && !d_ws)) return SHPL_ERR_ARG;
    if (check_ws && ws_bytes < pl.total) return SHPL_ERR_WORKSPACE;
    if (a_stride < a_off + c_a || out_stride < c_out || a_off < 0 || b_off < 0) return SHPL_ERR_BAD_SHAPE;
    if (c_b > 0 && b_stride < b_off + c_b) return SHPL_ERR_BAD_SHAPE;
    if (pooled) {
        if (!d_frame_off || c_b < 1 || !d_b) return SHPL_ERR_ARG;
        if (pool->n_keys != (int64_t)n_frames * h * w) return SHPL_ERR_BAD_SHAPE;
        if (pool->nnz_cap > 0 && (!pool->ent_dst || !pool->ent_src || !pool->ent_val)) return SHPL_ERR_ARG;
    } else if (c_b > 0 && !d_b) {
        return SHPL_ERR_ARG;
    }
    if (pl.n_tiles == 0) {
        *empty = true;
        return SHPL_OK;
    }
    if (!d_out || (c_a > 0 && !d_a)) return SHPL_ERR_ARG;
    const int esz = dtype == SHPL_F32 ? 4 : 2, he = 16 / esz;
    a = ConvArgs{};  // every field the forward does not set (out2: the dgrad split) is zero
    a.n_frames = n_frames;
    a.h = (int)h;
    a.w = (int)w;
    a.tiles_x = pl.tiles_x;
    a.tiles_per_frame = pl.tiles_per_frame;
    a.n_tiles = (int)pl.n_tiles;
    a.a = d_a;
    a.a_stride = a_stride;
    a.a_off = a_off;
    a.c_a = (int)c_a;
    a.qa = pl.qa;
    a.b = d_b;
    a.b_stride = b_stride;
    a.b_off = b_off;
    a.c_b = (int)c_b;
    a.qb = pl.qb;
    a.vec_a = aligned16(d_a) && a_stride % he == 0 && a_off % he == 0;
    a.vec_b = aligned16(d_b) && b_stride % he == 0 && b_off % he == 0;
    a.ent_dst = pooled ? pool->ent_dst : nullptr;
    a.ent_src = pooled ? pool->ent_src : nullptr;
    a.ent_val = pooled ? pool->ent_val : nullptr;
    uint8_t *ws = reinterpret_cast<uint8_t *>(d_ws);
    a.wp = ws;
    a.row_ptr = pooled && ws ? reinterpret_cast<const int32_t *>(ws + pl.wp_bytes) : nullptr;
    a.part = stats && ws ? reinterpret_cast<double *>(ws + pl.wp_bytes + pl.rp_bytes) : nullptr;
    a.center = d_center;
    a.scale = d_scale;
    a.shift = d_shift;
    a.act = act;
    a.out = d_out;
    a.out_stride = out_stride;
    a.c_out = (int)c_out;
    a.vec_out = aligned16(d_out) && out_stride % he == 0;
    return SHPL_OK;
}
}  // namespace
}  // namespace shpl

extern "C" int shpl_conv3x3(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride,
                            int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off,
                            int64_t c_b, const shpl_csr *pool, const int64_t *d_frame_off, const void *d_weights,
                            int64_t c_out, const float *d_center, const float *d_scale, const float *d_shift,
                            int act, void *d_out, int64_t out_stride, double *d_stats, void *d_ws, size_t ws_bytes,
                            void *stream) {
    const bool pooled = pool != nullptr, stats = d_stats != nullptr;
    ConvPlan pl;
    ConvArgs a;
    bool empty;
    const int rc = forward_setup(dtype, n_frames, h, w, d_a, a_stride, a_off, c_a, d_b, b_stride, b_off, c_b, pool,
                                 d_frame_off, d_weights, c_out, d_center, d_scale, d_shift, act, d_out, out_stride,
                                 stats, d_ws, ws_bytes, true, pl, a, &empty);
    if (rc || empty) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == SHPL_F32) return conv_launch<float>(pl, a, pooled, stats, d_weights, d_frame_off, d_stats, s);
    return conv_launch<uint16_t>(pl, a, pooled, stats, d_weights, d_frame_off, d_stats, s, 0, pool);
}

extern "C" int shpl_conv3x3_rows_form(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a,
                                      int64_t a_stride, int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride,
                                      int64_t b_off, int64_t c_b, const shpl_csr *pool, const int64_t *d_frame_off,
                                      const void *d_weights, int64_t c_out, int act, const void *d_out,
                                      int64_t out_stride, int stats, int *rows_form) {
    if (!rows_form) return SHPL_ERR_ARG;
    *rows_form = 0;
    ConvPlan pl;
    ConvArgs a;
    bool empty;
    const int rc = forward_setup(dtype, n_frames, h, w, d_a, a_stride, a_off, c_a, d_b, b_stride, b_off, c_b, pool,
                                 d_frame_off, d_weights, c_out, nullptr, nullptr, nullptr, act,
                                 const_cast<void *>(d_out), out_stride, stats != 0, nullptr, 0, false, pl, a, &empty);
    if (rc) return rc;
    *rows_form = !empty && dtype == SHPL_BF16 && rows_forward(pl, a, pool != nullptr, stats != 0);
    return SHPL_OK;
}

extern "C" int shpl_batch_norm(int dtype, int64_t rows, void *d_x, void *d_y, int64_t stride, int64_t c,
                               const double *d_stats, double count, float eps, const float *d_gamma,
                               const float *d_beta, int act, float *d_moving_mean, float *d_moving_var, float decay,
                               float *d_batch_mean, float *d_batch_var, float *d_ws, void *stream) {
    if (dtype != SHPL_F32 && dtype != SHPL_BF16) return SHPL_ERR_ARG;
    if (rows < 0 || c < 1 || stride < c || c > (1 << 16)) return SHPL_ERR_BAD_SHAPE;
    if (act != 0 && act != 1) return SHPL_ERR_ARG;
    if (!d_stats || !d_ws || (rows > 0 && !d_x) || !(count > 0.0)) return SHPL_ERR_ARG;
    if (!d_y) d_y = d_x;
    hipStream_t s = (hipStream_t)stream;
    float *mean = d_ws, *scale = d_ws + c;
    hipLaunchKernelGGL(k_bn_finalize, dim3(1), dim3(SHPL_BLOCK), 0, s, d_stats, count, (int)c, eps, d_gamma, mean,
                       scale, d_moving_mean, d_moving_var, decay, d_batch_mean, d_batch_var);
    SHPL_LAUNCH_CHECK();
    if (rows == 0) return SHPL_OK;
    const int vec = dtype == SHPL_F32 ? 4 : 8;
    const int pr = (int)(c / vec);
    const bool vform = c % vec == 0 && stride % vec == 0 && pr <= SHPL_BLOCK && (pr & (pr - 1)) == 0 &&
                       aligned16(d_x) && aligned16(d_y);
    const int grid = grid_for(rows * c / (vform ? vec : 1), SHPL_BLOCK * bn_rows_per_thread(16 / vec), 1 << 22);
    if (dtype == SHPL_F32) {
        if (vform)
            bn_forms([&](auto B, auto A) {
                hipLaunchKernelGGL((k_bn_apply_vec<float, B.value, A.value>), dim3(grid), dim3(SHPL_BLOCK), 0, s,
                                   reinterpret_cast<const float *>(d_x), reinterpret_cast<float *>(d_y), rows, stride,
                                   (int)c, mean, scale, d_beta);
            }, d_beta != nullptr, act == 1);
        else
            hipLaunchKernelGGL(k_bn_apply<float>, dim3(grid), dim3(SHPL_BLOCK), 0, s,
                               reinterpret_cast<const float *>(d_x), reinterpret_cast<float *>(d_y), rows, stride,
                               (int)c, mean, scale, d_beta, act);
    } else {
        if (vform)
            bn_forms([&](auto B, auto A) {
                hipLaunchKernelGGL((k_bn_apply_vec<uint16_t, B.value, A.value>), dim3(grid), dim3(SHPL_BLOCK), 0, s,
                                   reinterpret_cast<const uint16_t *>(d_x), reinterpret_cast<uint16_t *>(d_y), rows,
                                   stride, (int)c, mean, scale, d_beta);
            }, d_beta != nullptr, act == 1);
        else
            hipLaunchKernelGGL(k_bn_apply<uint16_t>, dim3(grid), dim3(SHPL_BLOCK), 0, s,
                               reinterpret_cast<const uint16_t *>(d_x), reinterpret_cast<uint16_t *>(d_y), rows,
                               stride, (int)c, mean, scale, d_beta, act);
    }
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

namespace {
int bn_bwd_blocks(int64_t rows) {
    int64_t nb = (rows + 4095) / 4096;
    if (nb < 1) nb = 1;
    if (nb > 1024) nb = 1024;
    return (int)nb;
}
}  // namespace

extern "C" int shpl_batch_norm_backward_workspace_bytes(int64_t rows, int64_t c, size_t *bytes) {
    if (!bytes || rows < 0 || c < 1) return SHPL_ERR_ARG;
    *bytes = align_up((size_t)bn_bwd_blocks(rows) * 2 * c * sizeof(double), 256) + align_up(2 * c * sizeof(float), 256);
    return SHPL_OK;
}

extern "C" int shpl_batch_norm_backward(int dtype, int64_t rows, const void *d_y, const void *d_raw,
                                        const void *d_gy, int64_t stride, int64_t c, const float *d_mean,
                                        const float *d_scale, const float *d_gamma, const float *d_beta, int act,
                                        int training, void *d_graw, float *d_dbeta, float *d_dgamma, void *d_ws,
                                        size_t ws_bytes, void *stream) {
    if (dtype != SHPL_F32 && dtype != SHPL_BF16) return SHPL_ERR_ARG;
    if (rows < 0 || c < 1 || stride < c || c > (1 << 16)) return SHPL_ERR_BAD_SHAPE;
    if (act != 0 && act != 1) return SHPL_ERR_ARG;
    size_t need;
    shpl_batch_norm_backward_workspace_bytes(rows, c, &need);
    if (!d_ws || ws_bytes < need) return SHPL_ERR_WORKSPACE;
    if (rows > 0 && (!d_gy || !d_graw || (act == 1 && !d_y && !d_raw) || (training && !d_raw))) return SHPL_ERR_ARG;
    if (rows == 0) return SHPL_OK;
    hipStream_t s = (hipStream_t)stream;
    const int nb = bn_bwd_blocks(rows);
    const int64_t rpb = (rows + nb - 1) / nb;
    double *part = reinterpret_cast<double *>(d_ws);
    float *mt = reinterpret_cast<float *>((uint8_t *)d_ws + align_up((size_t)nb * 2 * c * sizeof(double), 256));
    // x-hat needs raw only in training (dgamma); otherwise any row-shaped input stands in
    const void *rw = d_raw ? d_raw : d_gy;
    const int vec = dtype == SHPL_F32 ? 4 : 8;
    const int cg = (int)(c / vec);
    const bool vform = c % vec == 0 && stride % vec == 0 && cg <= SHPL_BLOCK && (cg & (cg - 1)) == 0 &&
                       aligned16(d_gy) && aligned16(rw) && aligned16(d_graw) && (!d_y || aligned16(d_y));
    // y NULL: the ReLU mask from raw (bn_pre_act), so only the y argument of the kernels changes
    const float *beta = act == 1 && !d_y ? d_beta : nullptr;
    const int grid = grid_for(rows * c / (vform ? vec : 1), SHPL_BLOCK * bn_rows_per_thread(16 / vec), 1 << 22);
    auto launch = [&](auto tag) {
        typedef decltype(tag) T;
        const T *y = (const T *)d_y, *r = (const T *)rw, *g = (const T *)d_gy;
        if (vform)
            // (its switches as template arguments measured slower: 785 vs 747 us, profiles/r04_bn_ab.log)
            hipLaunchKernelGGL(k_bn_bwd_partial_vec<T>, dim3(nb), dim3(SHPL_BLOCK), 0, s, y, r, g, rows, stride,
                               (int)c, d_mean, d_scale, d_gamma, beta, act, rpb, part);
        else
            hipLaunchKernelGGL(k_bn_bwd_partial<T>, dim3(nb), dim3(SHPL_BLOCK), 0, s, y, r, g, rows, stride, (int)c,
                               d_mean, d_scale, d_gamma, beta, act, rpb, part);
        hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((unsigned)c), dim3(SHPL_BLOCK), 0, s, part, nb,
                           (int)c, (double)rows, d_dbeta, d_raw ? d_dgamma : nullptr, mt);
        if (vform)
            bn_forms([&](auto A, auto Y, auto B, auto TR) {
                hipLaunchKernelGGL((k_bn_bwd_apply_vec<T, A.value, Y.value, B.value, TR.value>), dim3(grid),
                                   dim3(SHPL_BLOCK), 0, s, y, r, g, rows, stride, (int)c, d_mean, d_scale, d_gamma,
                                   beta, mt, (T *)d_graw);
            }, act == 1, d_y != nullptr, beta != nullptr, training != 0);
        else
            hipLaunchKernelGGL(k_bn_bwd_apply<T>, dim3(grid), dim3(SHPL_BLOCK), 0, s, y, r, g, rows, stride, (int)c,
                               d_mean, d_scale, d_gamma, beta, act, training, mt, (T *)d_graw);
    };
    if (dtype == SHPL_F32)
        launch(float());
    else
        launch(uint16_t());
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

namespace {
// shpl_conv3x3_dgrad; occ2: the occupancy words (wpr per row) limiting d_dx_b's stores (shpl_conv3x3_dgrad_reuse)
int dgrad_impl(int dtype, int n_frames, int64_t h, int64_t w, const void *d_gy, int64_t gy_stride, int64_t c_gy,
               const void *d_weights, int64_t c_dx, void *d_dx, int64_t dx_stride, int64_t c_split, void *d_dx_b,
               int64_t dx_b_stride, void *d_ws, size_t ws_bytes, const uint32_t *occ2, void *stream) {
    ConvPlan pl;
    int rc = conv_plan(dtype, n_frames, h, w, c_gy, 0, c_dx, false, false, &pl);
    if (rc) return rc;
    if (!d_weights || (ws_bytes > 0 && !d_ws)) return SHPL_ERR_ARG;
    if (ws_bytes < pl.total) return SHPL_ERR_WORKSPACE;
    if (!d_dx_b) c_split = c_dx;
    if (c_split < 0 || c_split > c_dx) return SHPL_ERR_BAD_SHAPE;
    if (gy_stride < c_gy || dx_stride < c_split || (d_dx_b && dx_b_stride < c_dx - c_split))
        return SHPL_ERR_BAD_SHAPE;
    if (pl.n_tiles == 0) return SHPL_OK;
    if (!d_gy || (c_split > 0 && !d_dx)) return SHPL_ERR_ARG;
    const int esz = dtype == SHPL_F32 ? 4 : 2, he = 16 / esz;
    ConvArgs a = {};
    a.n_frames = n_frames;
    a.h = (int)h;
    a.w = (int)w;
    a.tiles_x = pl.tiles_x;
    a.tiles_per_frame = pl.tiles_per_frame;
    a.n_tiles = (int)pl.n_tiles;
    a.a = d_gy;
    a.a_stride = gy_stride;
    a.a_off = 0;
    a.c_a = (int)c_gy;
    a.qa = pl.qa;
    a.vec_a = aligned16(d_gy) && gy_stride % he == 0;
    a.wp = d_ws;
    a.act = 0;
    a.out = d_dx;
    a.out_stride = dx_stride;
    a.c_out = (int)c_dx;
    a.out2 = d_dx_b;
    a.out2_stride = dx_b_stride;
    a.c_split = (int)c_split;
    a.vec_out = (!d_dx || (aligned16(d_dx) && dx_stride % he == 0)) &&
                (!d_dx_b || (aligned16(d_dx_b) && dx_b_stride % he == 0 && c_split % he == 0));
    a.occ2 = d_dx_b ? occ2 : nullptr;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == SHPL_F32) return conv_launch<float>(pl, a, false, false, d_weights, nullptr, nullptr, s, 1);
    return conv_launch<uint16_t>(pl, a, false, false, d_weights, nullptr, nullptr, s, 1);
}
}  // namespace

extern "C" int shpl_conv3x3_dgrad(int dtype, int n_frames, int64_t h, int64_t w, const void *d_gy, int64_t gy_stride,
                                  int64_t c_gy, const void *d_weights, int64_t c_dx, void *d_dx, int64_t dx_stride,
                                  int64_t c_split, void *d_dx_b, int64_t dx_b_stride, void *d_ws, size_t ws_bytes,
                                  void *stream) {
    return dgrad_impl(dtype, n_frames, h, w, d_gy, gy_stride, c_gy, d_weights, c_dx, d_dx, dx_stride, c_split, d_dx_b,
                      dx_b_stride, d_ws, ws_bytes, nullptr, stream);
}

extern "C" int shpl_conv3x3_dgrad_reuse(int dtype, int n_frames, int64_t h, int64_t w, const void *d_gy,
                                        int64_t gy_stride, int64_t c_gy, const void *d_weights, int64_t c_dx,
                                        void *d_dx, int64_t dx_stride, int64_t c_split, void *d_dx_b,
                                        int64_t dx_b_stride, void *d_ws, size_t ws_bytes, const shpl_csr *pool,
                                        const void *d_fwd_ws, size_t fwd_ws_bytes, int fwd_stats, void *stream) {
    // the forward's occupancy words, where its plan put them: the forward is the conv of [A (c_split) || B pooled
    // (c_dx - c_split)] to c_gy channels, the plan wgrad_impl's reuse checks too
    if (!pool || !d_fwd_ws || !d_dx_b) return SHPL_ERR_ARG;
    if (pool->n_keys != (int64_t)n_frames * h * w || c_split < 1 || c_split >= c_dx) return SHPL_ERR_BAD_SHAPE;
    ConvPlan fp;
    int rc = conv_plan(dtype, n_frames, h, w, c_split, c_dx - c_split, c_gy, true, fwd_stats != 0, &fp, 0,
                       pool->nnz_cap);
    if (rc) return rc;
    if (!fp.rows || fwd_ws_bytes < fp.total || c_gy % NCO != 0 ||
        (fwd_stats != 0 && !rows::supported_st(fp.qa + fp.qb, fp.qa, true)))
        return SHPL_ERR_ARG;
    const uint32_t *occ = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(d_fwd_ws) + fp.wp_bytes +
                                                             fp.rp_bytes + fp.part_bytes);
    return dgrad_impl(dtype, n_frames, h, w, d_gy, gy_stride, c_gy, d_weights, c_dx, d_dx, dx_stride, c_split, d_dx_b,
                      dx_b_stride, d_ws, ws_bytes, occ, stream);
}

namespace {
struct WgPlan {
    ConvPlan cp;
    int n_cib, n_groups, tiles_per_group;
    size_t rp_bytes, part_bytes, total;
    bool rows;  // bf16: k_wgrad_rows when the pointers are 16-byte aligned
    int r_groups;
    size_t r_part_bytes, r_part2_bytes, r_occ_bytes, r_cmp_bytes;
};

int wgrad_plan(int dtype, int n_frames, int64_t h, int64_t w, int64_t c_a, int64_t c_b, int64_t c_out, bool pooled,
               WgPlan *wp, int64_t pool_cap = 0) {
    int rc = conv_plan(dtype, n_frames, h, w, c_a, c_b, c_out, pooled, false, &wp->cp, TH);
    if (rc) return rc;
    const int Q = wp->cp.qa + wp->cp.qb;
    wp->n_cib = (Q * wp->cp.ck + WG_CI - 1) / WG_CI;
    const int64_t blocks_per_group = (int64_t)wp->n_cib * wp->cp.n_cob;
    int64_t ng = 1024 / blocks_per_group;
    if (ng < 1) ng = 1;
    if (ng > wp->cp.n_tiles) ng = wp->cp.n_tiles > 0 ? wp->cp.n_tiles : 1;
    wp->tiles_per_group = (int)((wp->cp.n_tiles + ng - 1) / ng);
    if (wp->tiles_per_group < 1) wp->tiles_per_group = 1;
    wp->n_groups = (int)((wp->cp.n_tiles + wp->tiles_per_group - 1) / wp->tiles_per_group);
    if (wp->n_groups < 1) wp->n_groups = 1;
    wp->rp_bytes = wp->cp.rp_bytes;
    wp->part_bytes = align_up((size_t)wp->n_groups * blocks_per_group * 9 * WG_CI * NCO * sizeof(float), 256);
    wp->total = wp->rp_bytes + wp->part_bytes;
    // the row-streaming bf16 weight gradient: bands and strips of the forward's row kernel
    const int n_bands = (int)((h + 59) / 60);
    const int64_t n_items = (int64_t)n_frames * n_bands * ((w + TW - 1) / TW);
    // pooled: B gathered from the compact pooled rows of prep_pooled (the forward's k_occ_frame + k_pool_runs)
    const int64_t wpr = (w + 31) / 32;
    wp->rows = SHPL_CONV_ROWS && dtype == SHPL_BF16 && h > 0 && w > 0 && n_items > 0 && n_items < (1LL << 31) &&
               rows::wgrad_supported((int)c_a, (int)c_b, (int)c_out) &&
               (!pooled || (c_a > 0 && c_b <= 64 && h * wpr <= rows::OCC_MAX_WORDS && pool_cap >= 0 &&
                            pool_cap * c_b * 2 < (1LL << 31)));
    if (wp->rows) {
        rows::wgrad_sizes((int)n_items, (int)c_a, (int)c_b, (int)c_out, &wp->r_groups, &wp->r_part_bytes,
                          &wp->r_part2_bytes);
        wp->r_part_bytes = align_up(wp->r_part_bytes, 256);
        wp->r_part2_bytes = align_up(wp->r_part2_bytes, 256);
        wp->r_occ_bytes = pooled ? 2 * align_up((size_t)n_frames * h * wpr * 4, 256) : 0;
        wp->r_cmp_bytes = pooled ? align_up((size_t)pool_cap * c_b * 2, 256) : 0;
        const size_t rt = wp->r_part_bytes + wp->r_part2_bytes + wp->r_occ_bytes + wp->r_cmp_bytes;
        if (rt > wp->total) wp->total = rt;
    }
    return SHPL_OK;
}
}  // namespace

extern "C" int shpl_conv3x3_wgrad_workspace_bytes(int dtype, int n_frames, int64_t h, int64_t w, int64_t c_a,
                                                  int64_t c_b, int64_t c_out, int64_t pool_nnz_cap, size_t *bytes) {
    if (!bytes) return SHPL_ERR_ARG;
    WgPlan wp;
    const bool pooled = pool_nnz_cap >= 0;
    const int rc = wgrad_plan(dtype, n_frames, h, w, c_a, c_b, c_out, pooled, &wp, pooled ? pool_nnz_cap : 0);
    if (rc) return rc;
    *bytes = wp.total;
    return SHPL_OK;
}

namespace {
// shpl_conv3x3_wgrad; d_fwd_ws: the workspace of a pooled bf16 forward shpl_conv3x3 call over the same map
// (shpl_conv3x3_wgrad_reuse) whose pooled operand the row-streaming form reads instead of preparing its own
int wgrad_impl(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride, int64_t a_off,
               int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off, int64_t c_b, const shpl_csr *pool,
               const int64_t *d_frame_off, const void *d_gy, int64_t gy_stride, int64_t c_out, float *d_dw,
               void *d_ws, size_t ws_bytes, const void *d_fwd_ws, size_t fwd_ws_bytes, int fwd_stats,
               void *stream) {
    const bool pooled = pool != nullptr;
    WgPlan wp;
    int rc = wgrad_plan(dtype, n_frames, h, w, c_a, c_b, c_out, pooled, &wp, pooled ? pool->nnz_cap : 0);
    if (rc) return rc;
    if (!d_dw || (ws_bytes > 0 && !d_ws)) return SHPL_ERR_ARG;
    if (ws_bytes < wp.total) return SHPL_ERR_WORKSPACE;
    if (a_stride < a_off + c_a || a_off < 0 || b_off < 0 || gy_stride < c_out) return SHPL_ERR_BAD_SHAPE;
    if (c_b > 0 && b_stride < b_off + c_b) return SHPL_ERR_BAD_SHAPE;
    if (pooled) {
        if (!d_frame_off || c_b < 1 || !d_b) return SHPL_ERR_ARG;
        if (pool->n_keys != (int64_t)n_frames * h * w) return SHPL_ERR_BAD_SHAPE;
        if (pool->nnz_cap > 0 && (!pool->ent_dst || !pool->ent_src || !pool->ent_val)) return SHPL_ERR_ARG;
    } else if (c_b > 0 && !d_b) {
        return SHPL_ERR_ARG;
    }
    if ((c_a > 0 && !d_a) || !d_gy) return SHPL_ERR_ARG;
    const ConvPlan &pl = wp.cp;
    const int esz = dtype == SHPL_F32 ? 4 : 2, he = 16 / esz;
    hipStream_t s = (hipStream_t)stream;
    if (pl.n_tiles == 0) {  // no pixels: dW = 0
        SHPL_HIP_CHECK(hipMemsetAsync(d_dw, 0, sizeof(float) * 9 * (size_t)(c_a + c_b) * c_out, s));
        return SHPL_OK;
    }
    if (wp.rows && (c_a == 0 || (aligned16(d_a) && a_stride % he == 0 && a_off % he == 0)) &&
        (c_b == 0 || (aligned16(d_b) && b_stride % he == 0 && b_off % he == 0)) && aligned16(d_gy) &&
        gy_stride % he == 0 && (!pooled || c_a % 32 == 0)) {
        rows::WgRowArgs r = {};
        r.a = reinterpret_cast<const uint16_t *>(d_a) + a_off;
        r.b = c_b > 0 ? reinterpret_cast<const uint16_t *>(d_b) + b_off : nullptr;
        r.a_stride = a_stride;
        r.b_stride = b_stride;
        r.c_a = (int)c_a;
        r.c_b = (int)c_b;
        r.gy = reinterpret_cast<const uint16_t *>(d_gy);
        r.gy_stride = gy_stride;
        r.c_out = (int)c_out;
        r.h = (int)h;
        r.w = (int)w;
        r.strips = (int)((w + TW - 1) / TW);
        r.n_bands = (int)((h + 59) / 60);
        r.band = (int)((h + r.n_bands - 1) / r.n_bands);
        r.n_items = n_frames * r.n_bands * r.strips;
        r.n_cit = (int)((c_a + 31) / 32 + (c_b + 31) / 32);
        r.n_cot = (int)((c_out + 31) / 32);
        r.n_groups = wp.r_groups;
        uint8_t *ws = reinterpret_cast<uint8_t *>(d_ws);
        r.part = reinterpret_cast<float *>(ws);
        if (pooled) {  // the pooled vector of every run once into the compact buffer (the forward's prep)
            uint8_t *po = ws + wp.r_part_bytes + wp.r_part2_bytes;
            uint32_t *occ = reinterpret_cast<uint32_t *>(po);
            int32_t *occ_base = reinterpret_cast<int32_t *>(po + wp.r_occ_bytes / 2);
            uint16_t *cmp = reinterpret_cast<uint16_t *>(po + wp.r_occ_bytes);
            const int wpr = (int)((w + 31) / 32);
            // the forward call's occupancy maps and pooled runs, where its plan put them (when it has them)
            ConvPlan fp;
            const bool reuse = d_fwd_ws &&
                               conv_plan(dtype, n_frames, h, w, c_a, c_b, c_out, true, fwd_stats != 0, &fp, 0,
                                         pool->nnz_cap) == SHPL_OK &&
                               fp.rows && fwd_ws_bytes >= fp.total && fp.wpr == wpr && c_out % NCO == 0 &&
                               (fwd_stats == 0 || rows::supported_st(fp.qa + fp.qb, fp.qa, true));
            // the rest of rows_forward (the forward's act and output alignment) is the caller's to establish
            // with shpl_conv3x3_rows_form (shpl.h); what is checkable here and fails is an error, not a fallback
            if (d_fwd_ws && !reuse) return SHPL_ERR_ARG;
            if (reuse) {
                uint8_t *fo = reinterpret_cast<uint8_t *>(const_cast<void *>(d_fwd_ws)) + fp.wp_bytes + fp.rp_bytes +
                              fp.part_bytes;
                occ = reinterpret_cast<uint32_t *>(fo);
                occ_base = reinterpret_cast<int32_t *>(fo + fp.occ_bytes / 2);
                cmp = reinterpret_cast<uint16_t *>(fo + fp.occ_bytes);
            } else {
                rc = rows::prep_pooled(n_frames, (int)h, (int)w, wpr, pool->ent_dst, pool->ent_src, pool->ent_val,
                                       pool->nnz_cap, d_frame_off, reinterpret_cast<const uint16_t *>(d_b), b_stride,
                                       b_off, (int)c_b, occ, occ_base, cmp, s);
                if (rc) return rc;
            }
            r.b = nullptr;
            r.cmp = cmp;
            r.cmp_stride = (int)c_b;
            r.occ = occ;
            r.occ_base = occ_base;
            r.wpr = wpr;
            r.frame_off = d_frame_off;
        }
        return rows::wgrad_launch(r, d_dw, reinterpret_cast<double *>(ws + wp.r_part_bytes), s);
    }
    ConvArgs a = {};
    a.n_frames = n_frames;
    a.h = (int)h;
    a.w = (int)w;
    a.tiles_x = pl.tiles_x;
    a.tiles_per_frame = pl.tiles_per_frame;
    a.n_tiles = (int)pl.n_tiles;
    a.a = d_a;
    a.a_stride = a_stride;
    a.a_off = a_off;
    a.c_a = (int)c_a;
    a.qa = pl.qa;
    a.b = d_b;
    a.b_stride = b_stride;
    a.b_off = b_off;
    a.c_b = (int)c_b;
    a.qb = pl.qb;
    a.vec_a = aligned16(d_a) && a_stride % he == 0 && a_off % he == 0;
    a.vec_b = aligned16(d_b) && b_stride % he == 0 && b_off % he == 0;
    a.ent_dst = pooled ? pool->ent_dst : nullptr;
    a.ent_src = pooled ? pool->ent_src : nullptr;
    a.ent_val = pooled ? pool->ent_val : nullptr;
    uint8_t *ws = reinterpret_cast<uint8_t *>(d_ws);
    a.row_ptr = pooled ? reinterpret_cast<const int32_t *>(ws) : nullptr;
    a.c_out = (int)c_out;
    WgArgs g = {};
    g.gy = d_gy;
    g.gy_stride = gy_stride;
    g.n_cib = wp.n_cib;
    g.n_cob = pl.n_cob;
    g.tiles_per_group = wp.tiles_per_group;
    g.vec_g = aligned16(d_gy) && gy_stride % he == 0;
    g.whole = (c_a == 0 || (a.vec_a && c_a % pl.ck == 0)) && (c_b == 0 || (a.vec_b && c_b % pl.ck == 0)) &&
              g.vec_g && c_out % NCO == 0;
    g.part = reinterpret_cast<float *>(ws + wp.rp_bytes);
    if (pooled) {
        hipLaunchKernelGGL(k_row_ptr, dim3(16, n_frames), dim3(SHPL_BLOCK), 0, s, a.ent_dst, d_frame_off, a.h, a.w,
                           const_cast<int32_t *>(a.row_ptr));
        SHPL_LAUNCH_CHECK();
    }
    const dim3 grid((unsigned)wp.n_groups, (unsigned)wp.n_cib, (unsigned)pl.n_cob);
    if (dtype == SHPL_F32) {
        if (pooled)
            hipLaunchKernelGGL((k_conv3x3_wgrad<float, true>), grid, dim3(CONV_BLOCK), 0, s, a, g);
        else
            hipLaunchKernelGGL((k_conv3x3_wgrad<float, false>), grid, dim3(CONV_BLOCK), 0, s, a, g);
    } else {
        if (pooled)
            hipLaunchKernelGGL((k_conv3x3_wgrad<uint16_t, true>), grid, dim3(CONV_BLOCK), 0, s, a, g);
        else
            hipLaunchKernelGGL(k_wgrad_bf16, grid, dim3(CONV_BLOCK), 0, s, a, g);
    }
    SHPL_LAUNCH_CHECK();
    const int64_t n_out = 9 * (c_a + c_b) * c_out;
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(grid_for(n_out, WR_OUT, 4096)), dim3(SHPL_BLOCK), 0, s, g.part,
                       wp.n_groups, wp.n_cib, pl.n_cob, (int)c_a, (int)c_b, pl.qa, pl.ck, (int)c_out, d_dw);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}
}  // namespace

extern "C" int shpl_conv3x3_wgrad(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride,
                                  int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off,
                                  int64_t c_b, const shpl_csr *pool, const int64_t *d_frame_off, const void *d_gy,
                                  int64_t gy_stride, int64_t c_out, float *d_dw, void *d_ws, size_t ws_bytes,
                                  void *stream) {
    return wgrad_impl(dtype, n_frames, h, w, d_a, a_stride, a_off, c_a, d_b, b_stride, b_off, c_b, pool, d_frame_off,
                      d_gy, gy_stride, c_out, d_dw, d_ws, ws_bytes, nullptr, 0, 0, stream);
}

extern "C" int shpl_conv3x3_wgrad_reuse(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a,
                                        int64_t a_stride, int64_t a_off, int64_t c_a, const void *d_b,
                                        int64_t b_stride, int64_t b_off, int64_t c_b, const shpl_csr *pool,
                                        const int64_t *d_frame_off, const void *d_gy, int64_t gy_stride,
                                        int64_t c_out, float *d_dw, void *d_ws, size_t ws_bytes,
                                        const void *d_fwd_ws, size_t fwd_ws_bytes, int fwd_stats, void *stream) {
    if (!pool || !d_fwd_ws || dtype != SHPL_BF16) return SHPL_ERR_ARG;
    return wgrad_impl(dtype, n_frames, h, w, d_a, a_stride, a_off, c_a, d_b, b_stride, b_off, c_b, pool, d_frame_off,
                      d_gy, gy_stride, c_out, d_dw, d_ws, ws_bytes, d_fwd_ws, fwd_ws_bytes, fwd_stats, stream);
}
