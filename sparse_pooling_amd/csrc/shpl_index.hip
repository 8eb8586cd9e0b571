// shpl_index.hip -- device index builder of SHPL.
//
// Reference (host numpy, once per frame inside the data loader):
//   projectToImage / clip3DwithinImage      avod/avod/utils/transform.py:3-40
//   gen_sparse_pooling_input_avod           avod/avod/utils/sparse_pool_utils.py:6-20
//   produce_sparse_pooling_input            avod/avod/utils/sparse_pool_utils.py:22-58
//
// Two launches over 4096-point chunks of every frame (shpl_compact.h): a
// per-chunk count of the kept points, then the placement, where each thread
// evaluates one point per row and the kept points are ranked by wave ballots
// + an LDS prefix and written in point order (a stable compaction). A frame's
// entries start at its first input point ("capacity layout"); the tail up to
// the next frame is filled with -1 sentinels that every consumer skips, so no
// cross-frame scan is needed.
// Projection runs in f64 with the exact operation order numpy uses (an FMA
// chain over k for np.dot, dgemv's order when the product has one column,
// IEEE division, rint = round-half-even), so the integer outputs are
// bit-identical to the reference (tests/golden/index_*). The reference
// projects twice: the clip over the frame's N points (transform.py:34 via
// sparse_pool_utils.py:13), then projectToImage over the clip's survivors
// (:16) -- one column each when N == 1, resp. when one point survives.
#include "shpl_compact.h"

namespace shpl {
namespace {

template <typename PT>
__device__ __forceinline__ void load_point(const void *pts, int64_t i, double &x, double &y, double &z) {
    const PT *p = reinterpret_cast<const PT *>(pts) + 3 * i;
    x = (double)p[0];
    y = (double)p[1];
    z = (double)p[2];
}

template <typename IT>
__device__ __forceinline__ int64_t load_idx(const void *a, int64_t i) {
    return (int64_t)reinterpret_cast<const IT *>(a)[i];
}

// clip3DwithinImage (transform.py:28-40): 0 <= u < W-1, 0 <= v < H-1.
__device__ __forceinline__ bool in_image(double u, double v, double w, double h) {
    return (u < w - 1.0) && (u >= 0.0) && (v >= 0.0) && (v < h - 1.0);
}

struct Geometry {
    double im_w, im_h, s_img, s_bv;
    double wq, hq, bhq, bwq;  // floor(size / stride)
    int64_t n_cells;          // int(bhq*bwq)
    int64_t n_pix;            // hq*wq
    double inv_img, inv_bv;   // 1 / stride when the stride is a power of two (x / 2^k == x * 2^-k exactly), else 0
};

// 1 / s when s is a power of two (its reciprocal exact, so x * (1 / s) is bitwise x / s for every finite x that
// stays normal -- the image and voxel indices here), else 0: the division then stays a division.
#ifndef SHPL_POW2_DIV
#define SHPL_POW2_DIV 1
#endif
inline double pow2_reciprocal(double s) {
    if (!SHPL_POW2_DIV) return 0.0;
    int e = 0;
    return (s > 0.0 && frexp(s, &e) == 0.5 && e > -1000 && e < 1000) ? ldexp(1.0, 1 - e) : 0.0;
}

// x / s (IEEE), as a multiply when the reciprocal is exact (inv != 0)
__device__ __forceinline__ double div_stride(double x, double s, double inv) {
    return inv != 0.0 ? __dmul_rn(x, inv) : __ddiv_rn(x, s);
}

Geometry make_geometry(double im_w, double im_h, double bv_h, double bv_w, double s_img, double s_bv) {
    Geometry g = {};
    g.im_w = im_w;
    g.im_h = im_h;
    g.s_img = s_img;
    g.s_bv = s_bv;
    g.wq = floor(im_w / s_img);
    g.hq = floor(im_h / s_img);
    g.bhq = floor(bv_h / s_bv);
    g.bwq = floor(bv_w / s_bv);
    g.n_cells = (int64_t)(g.bhq * g.bwq);
    g.n_pix = (int64_t)g.hq * (int64_t)g.wq;
    g.inv_img = pow2_reciprocal(s_img);
    g.inv_bv = pow2_reciprocal(s_bv);
    return g;
}

// produce_sparse_pooling_input (sparse_pool_utils.py:22-58) on one rounded
// image index (ur, vr) and one voxel index (vx, vz).
struct Produced {
    double u, v;   // strided + clamped image index (what the reference writes back)
    int64_t r;     // flattened BEV row
    bool inside;   // r < n_cells
};

__device__ __forceinline__ Produced produce(const Geometry &g, double ur, double vr, int64_t vx,
                                            int64_t vz) {
    Produced o = {};
    double u = floor(div_stride(ur, g.s_img, g.inv_img));
    double v = floor(div_stride(vr, g.s_img, g.inv_img));
    if (u >= g.wq) u = g.wq - 1.0;
    if (v >= g.hq) v = g.hq - 1.0;
    o.u = u;
    o.v = v;
    const double bx = floor(div_stride((double)vx, g.s_bv, g.inv_bv));
    const double bz = floor(div_stride((double)vz, g.s_bv, g.inv_bv));
    o.r = (int64_t)__dadd_rn(__dmul_rn(bz, g.bwq), bx);
    o.inside = o.r < g.n_cells;
    return o;
}

// ------------------------------------------------------------------ stages
// Each stage: eval() decides whether point i (of frame f) is kept; emit()
// writes kept point i at global position pos (frame starts at fstart);
// touch() runs for every point in the write pass (in-place side effects).

template <typename PT, typename VT>
struct FusedStage {
    static constexpr bool HAS_BUCKETS = true;
    const void *pts;
    const void *vox;
    int64_t vstride;
    const double *P;
    Geometry g = {};
    const float *mval;
    int32_t *cell, *pix;
    float *val;
    int64_t *mij, *flip;
    uint32_t *err;
    const double *P_frame = nullptr;  // k_index1: this frame's P, staged in LDS at the launch's start

    struct Payload {
        Produced pr;
    };
    struct In {
        double x, y, z;
        int64_t vx, vz;
    };

    __device__ void load(int64_t i, In &in) const {
        load_point<PT>(pts, i, in.x, in.y, in.z);
        in.vx = load_idx<VT>(vox, i * vstride);
        in.vz = load_idx<VT>(vox, i * vstride + 1);
    }
    // AUX = inside the clip (the columns of the second projection)
    __device__ uint32_t eval(const Ctx &c, int f, int64_t, const In &in, Payload &pl) const {
        double u, v, Pf[12];
        if (P_frame) {  // (LDS: flat loads only on this path; the global one keeps global loads)
#pragma unroll
            for (int k = 0; k < 12; ++k) Pf[k] = P_frame[k];
        } else {
#pragma unroll
            for (int k = 0; k < 12; ++k) Pf[k] = P[12 * f + k];
        }
        project(Pf, in.x, in.y, in.z, u, v, c.n_live == 1);
        if (!in_image(u, v, g.im_w, g.im_h)) return 0u;
        if (c.n_aux == 1 && c.n_live != 1) project(Pf, in.x, in.y, in.z, u, v, true);
        const double ur = (double)(int64_t)rint(u);
        const double vr = (double)(int64_t)rint(v);
        pl.pr = produce(g, ur, vr, in.vx, in.vz);
        return AUX | (pl.pr.inside ? KEEP_MULTI | KEEP_ONE : 0u);
    }
    __device__ void touch(int, int64_t, const Payload &, bool) const {}
    __device__ void emit(int f, int64_t i, int64_t pos, int64_t fstart, const Payload &pl) const {
        const int64_t r = pl.pr.r;
        const int64_t vi = (int64_t)pl.pr.v, ui = (int64_t)pl.pr.u;
        const bool rok = r >= 0;
        const bool pok = vi >= 0 && ui >= 0;
        if ((!rok || !pok) && err) atomicOr(err, (rok ? 0u : SHPL_EBIT_ROW) | (pok ? 0u : SHPL_EBIT_PIXEL));
        cell[pos] = rok ? (int32_t)(f * g.n_cells + r) : -1;
        pix[pos] = pok ? (int32_t)(f * g.n_pix + vi * (int64_t)g.wq + ui) : -1;
        val[pos] = mval ? mval[i] : 1.0f;
        if (mij) {
            mij[2 * pos] = r;
            mij[2 * pos + 1] = pos - fstart;
        }
        if (flip) {
            flip[3 * pos] = 0;
            flip[3 * pos + 1] = vi;
            flip[3 * pos + 2] = ui;
        }
    }
    __device__ void hole(int64_t pos) const {  // capacity slot past the frame's last entry
        cell[pos] = -1;
        pix[pos] = -1;
        val[pos] = 0.0f;
    }
    // frame-local destinations of a kept entry (buckets): the cell and pixel emit() writes, unless -1
    __device__ bool bucket_keys(const Payload &pl, int32_t &kc, int32_t &kp) const {
        const int64_t r = pl.pr.r, vi = (int64_t)pl.pr.v, ui = (int64_t)pl.pr.u;
        if (r < 0 || vi < 0 || ui < 0) return false;
        kc = (int32_t)r;
        kp = (int32_t)(vi * (int64_t)g.wq + ui);
        return true;
    }
};

template <typename PT, typename VT>
struct GenStage {  // gen_sparse_pooling_input_avod
    static constexpr bool HAS_BUCKETS = false;
    const void *pts;
    const void *vox;
    int64_t vstride;
    const double *P;
    double im_w, im_h;
    int64_t *bv_index;
    double *img_index;
    int64_t ld;

    struct Payload {
        double u, v;
    };
    struct In {
        double x, y, z;
    };

    __device__ void load(int64_t i, In &in) const { load_point<PT>(pts, i, in.x, in.y, in.z); }
    __device__ uint32_t eval(const Ctx &c, int f, int64_t, const In &in, Payload &pl) const {
        project(P + 12 * f, in.x, in.y, in.z, pl.u, pl.v, c.n_live == 1);
        if (!in_image(pl.u, pl.v, im_w, im_h)) return 0u;
        if (c.n_aux == 1 && c.n_live != 1) project(P + 12 * f, in.x, in.y, in.z, pl.u, pl.v, true);
        return AUX | KEEP_MULTI | KEEP_ONE;
    }
    __device__ void touch(int, int64_t, const Payload &, bool) const {}
    __device__ void emit(int, int64_t i, int64_t pos, int64_t, const Payload &pl) const {
        bv_index[2 * pos] = load_idx<VT>(vox, i * vstride);
        bv_index[2 * pos + 1] = load_idx<VT>(vox, i * vstride + 1);
        img_index[pos] = (double)(int64_t)rint(pl.u);
        img_index[ld + pos] = (double)(int64_t)rint(pl.v);
        img_index[2 * ld + pos] = 0.0;
    }
    __device__ void hole(int64_t) const {}
};

template <typename VT>
struct ProduceStage {  // produce_sparse_pooling_input (in-place img_index update)
    static constexpr bool HAS_BUCKETS = false;
    const void *bv;
    int64_t bstride;
    double *img;  // 3 rows, stride ld
    int64_t ld;
    Geometry g = {};
    int64_t *mij, *flip;
    int32_t *cell, *pix;
    uint32_t *err;

    struct Payload {
        Produced pr;
        double w;  // third row
    };
    struct In {
        double u, v, w;
        int64_t vx, vz;
    };

    __device__ void load(int64_t i, In &in) const {
        in.u = img[i];
        in.v = img[ld + i];
        in.w = img[2 * ld + i];
        in.vx = load_idx<VT>(bv, i * bstride);
        in.vz = load_idx<VT>(bv, i * bstride + 1);
    }
    __device__ uint32_t eval(const Ctx &, int, int64_t, const In &in, Payload &pl) const {
        pl.pr = produce(g, in.u, in.v, in.vx, in.vz);
        pl.w = in.w;
        return pl.pr.inside ? KEEP_MULTI | KEEP_ONE : 0u;
    }
    // img_index[0:2] = floor(img_index/stride), clamped -- for EVERY point
    // (sparse_pool_utils.py:30-34), after this thread has read its own value.
    __device__ void touch(int, int64_t i, const Payload &pl, bool) const {
        img[i] = pl.pr.u;
        img[ld + i] = pl.pr.v;
    }
    __device__ void emit(int, int64_t, int64_t pos, int64_t, const Payload &pl) const {
        const int64_t r = pl.pr.r;
        const int64_t vi = (int64_t)pl.pr.v, ui = (int64_t)pl.pr.u;
        const bool rok = r >= 0, pok = vi >= 0 && ui >= 0;
        if ((!rok || !pok) && err) atomicOr(err, (rok ? 0u : SHPL_EBIT_ROW) | (pok ? 0u : SHPL_EBIT_PIXEL));
        mij[2 * pos] = r;
        mij[2 * pos + 1] = pos;
        flip[3 * pos] = (int64_t)floor(pl.w);
        flip[3 * pos + 1] = vi;
        flip[3 * pos + 2] = ui;
        if (cell) cell[pos] = rok ? (int32_t)r : -1;
        if (pix) pix[pos] = pok ? (int32_t)(vi * (int64_t)g.wq + ui) : -1;
    }
    __device__ void hole(int64_t pos) const {
        if (cell) cell[pos] = -1;
        if (pix) pix[pos] = -1;
    }
};

// ------------------------------------------------- per-frame stable compaction

__global__ void k_set_pair(int64_t *o, int64_t a, int64_t b) {
    o[0] = a;
    o[1] = b;
}

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_build_index_workspace_bytes(int n_frames, int64_t max_points_per_frame, size_t *bytes) {
    if (!bytes || n_frames < 1 || max_points_per_frame < 0) return SHPL_ERR_ARG;
    *bytes = index_ws_bytes(n_frames, max_points_per_frame);  // [0, n] pair of the single-frame calls + chunk counts
    return SHPL_OK;
}

// shpl_build_index, optionally with the destination buckets (bk != NULL)
static int build_index(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                       int64_t max_points_per_frame, const void *d_points, int points_dtype, const void *d_voxels,
                       int voxels_itype, int64_t vox_stride, const double *d_P, const Geometry &g,
                       const float *d_mval, int32_t *d_cell, int32_t *d_pix, float *d_val, int64_t *d_mij,
                       int64_t *d_flip, int64_t *d_frame_nnz, int64_t *d_frame_out_off, uint32_t *d_err, void *d_ws,
                       size_t ws_bytes, hipStream_t s, const Bkt *bk) {
#define SHPL_FUSED(PT, VT)                                                                       \
    {                                                                                            \
        FusedStage<PT, VT> st{d_points, d_voxels, vox_stride, d_P, g, d_mval, d_cell, d_pix,     \
                              d_val, d_mij, d_flip, d_err};                                      \
        return run_compaction(st, n_frames, max_points_per_frame, d_point_offsets, d_point_counts, d_frame_nnz, \
                              d_frame_out_off, d_err, d_ws, ws_bytes, s, bk);                    \
    }
    if (points_dtype == SHPL_F64 && voxels_itype == SHPL_I64) SHPL_FUSED(double, int64_t)
    if (points_dtype == SHPL_F64 && voxels_itype == SHPL_I32) SHPL_FUSED(double, int32_t)
    if (points_dtype == SHPL_F32 && voxels_itype == SHPL_I64) SHPL_FUSED(float, int64_t)
    if (points_dtype == SHPL_F32 && voxels_itype == SHPL_I32) SHPL_FUSED(float, int32_t)
#undef SHPL_FUSED
    return SHPL_ERR_ARG;
}

static int index_args(int n_frames, const int64_t *d_point_offsets, int64_t max_points_per_frame,
                      const void *d_points, const void *d_voxels, int64_t vox_stride, const double *d_P,
                      double s_img, double s_bv, const int32_t *d_cell, const int32_t *d_pix, const float *d_val,
                      const void *d_ws, const Geometry &g) {
    if (n_frames < 1 || !d_point_offsets || !d_P || !d_ws) return SHPL_ERR_ARG;
    if (max_points_per_frame > 0 && (!d_points || !d_voxels || !d_cell || !d_pix || !d_val)) return SHPL_ERR_ARG;
    if (vox_stride < 2 || !(s_img > 0) || !(s_bv > 0)) return SHPL_ERR_BAD_SHAPE;
    if ((double)n_frames * (double)(g.n_cells > 0 ? g.n_cells : 0) >= 2147483647.0 ||
        (double)n_frames * (double)(g.n_pix > 0 ? g.n_pix : 0) >= 2147483647.0)
        return SHPL_ERR_BAD_SHAPE;
    return SHPL_OK;
}

extern "C" int shpl_build_index(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                                int64_t max_points_per_frame,
                                const void *d_points, int points_dtype, const void *d_voxels,
                                int voxels_itype, int64_t vox_stride, const double *d_P, double im_w,
                                double im_h, double bv_h, double bv_w, double s_img, double s_bv,
                                const float *d_mval, int32_t *d_cell, int32_t *d_pix, float *d_val,
                                int64_t *d_mij, int64_t *d_flip, int64_t *d_frame_nnz,
                                int64_t *d_frame_out_off, uint32_t *d_err, void *d_ws, size_t ws_bytes,
                                void *stream) {
    const Geometry g = make_geometry(im_w, im_h, bv_h, bv_w, s_img, s_bv);
    const int rc = index_args(n_frames, d_point_offsets, max_points_per_frame, d_points, d_voxels, vox_stride, d_P,
                              s_img, s_bv, d_cell, d_pix, d_val, d_ws, g);
    if (rc) return rc;
    return build_index(n_frames, d_point_offsets, d_point_counts, max_points_per_frame, d_points, points_dtype,
                       d_voxels, voxels_itype, vox_stride, d_P, g, d_mval, d_cell, d_pix, d_val, d_mij, d_flip,
                       d_frame_nnz, d_frame_out_off, d_err, d_ws, ws_bytes, (hipStream_t)stream, nullptr);
}

// bucket limits: 24-bit entry offsets, 512 ranges of BK_KEYS destinations per frame and key
static bool bucket_shape_ok(int64_t max_points_per_frame, int64_t nnz_cap, int64_t cells, int64_t pix) {
    return (int64_t)n_chunks_for(max_points_per_frame) * IDX_CHUNK <= ((int64_t)1 << 24) && nnz_cap >= 0 &&
           nnz_cap < ((int64_t)1 << 31) && cells <= (int64_t)BK_KEYS * BK_MAX_RANGES &&
           pix <= (int64_t)BK_KEYS * BK_MAX_RANGES;
}

extern "C" int shpl_bucket_workspace_bytes(int n_frames, int64_t max_points_per_frame, int64_t nnz_cap,
                                           int64_t cells_per_frame, int64_t pix_per_frame, size_t *bytes) {
    if (!bytes || n_frames < 1 || max_points_per_frame < 0 || cells_per_frame < 0 || pix_per_frame < 0)
        return SHPL_ERR_ARG;
    if (!bucket_shape_ok(max_points_per_frame, nnz_cap, cells_per_frame, pix_per_frame)) return SHPL_ERR_BAD_SHAPE;
    *bytes = bk_layout(n_frames, n_chunks_for(max_points_per_frame), nnz_cap, cells_per_frame, pix_per_frame).bytes;
    return SHPL_OK;
}

extern "C" int shpl_bucket_workspace_reset(int n_frames, void *d_bkt, size_t bkt_bytes, void *stream) {
    if (n_frames < 1 || !d_bkt) return SHPL_ERR_ARG;
    const BkLayout l = bk_layout(n_frames, 1, 0, 0, 0);  // the barrier words' place depends on n_frames alone
    const size_t bytes = 4 * 2 * (size_t)n_frames;
    if (bkt_bytes < l.bar + bytes) return SHPL_ERR_WORKSPACE;
    return hipMemsetAsync((char *)d_bkt + l.bar, 0, bytes, (hipStream_t)stream) == hipSuccess ? SHPL_OK
                                                                                             : SHPL_ERR_HIP;
}

extern "C" int shpl_build_index_buckets(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                                        int64_t max_points_per_frame, const void *d_points, int points_dtype,
                                        const void *d_voxels, int voxels_itype, int64_t vox_stride, const double *d_P,
                                        double im_w, double im_h, double bv_h, double bv_w, double s_img,
                                        double s_bv, const float *d_mval, int32_t *d_cell, int32_t *d_pix,
                                        float *d_val, int64_t *d_frame_nnz, int64_t *d_frame_out_off,
                                        uint32_t *d_err, void *d_ws, size_t ws_bytes, int64_t nnz_cap, void *d_bkt,
                                        size_t bkt_bytes, const shpl_pass_copy *cell_copy,
                                        const shpl_pass_copy *pixel_copy, void *stream) {
    const Geometry g = make_geometry(im_w, im_h, bv_h, bv_w, s_img, s_bv);
    int rc = index_args(n_frames, d_point_offsets, max_points_per_frame, d_points, d_voxels, vox_stride, d_P, s_img,
                        s_bv, d_cell, d_pix, d_val, d_ws, g);
    if (rc) return rc;
    if (!d_bkt || !d_frame_nnz) return SHPL_ERR_ARG;
    if (!bucket_shape_ok(max_points_per_frame, nnz_cap, g.n_cells, g.n_pix)) return SHPL_ERR_BAD_SHAPE;
    const BkLayout l = bk_layout(n_frames, n_chunks_for(max_points_per_frame), nnz_cap, g.n_cells, g.n_pix);
    if (bkt_bytes < l.bytes) return SHPL_ERR_WORKSPACE;
    char *b = (char *)d_bkt;
    // which index launch each rider copy rides (SHPL_RIDERS: 0 = cell copy with the count, pixel copy with the
    // placement; 1 = both with the count; 2 = both with the placement)
#ifndef SHPL_RIDERS
#define SHPL_RIDERS 0
#endif
    Bkt bk{{l.nr[0], l.nr[1]}, l.nrmax, nnz_cap, (int32_t *)(b + l.hist), (int32_t *)(b + l.ext),
           (uint32_t *)(b + l.words), {}, {SHPL_RIDERS == 2 ? 1 : 0, SHPL_RIDERS == 1 ? 0 : 1}, 0,
           (int32_t *)(b + l.bar)};
    const shpl_pass_copy *cps[2] = {cell_copy, pixel_copy};
    int64_t copy_bytes = 0;
    for (int k = 0; k < 2; ++k) {
        rc = make_pass_copy(cps[k], k ? g.n_pix : g.n_cells, &bk.cp[k], &copy_bytes);
        if (rc) return rc;
    }
    bk.cp_blocks = rider_blocks(n_frames, copy_bytes);
    return build_index(n_frames, d_point_offsets, d_point_counts, max_points_per_frame, d_points, points_dtype,
                       d_voxels, voxels_itype, vox_stride, d_P, g, d_mval, d_cell, d_pix, d_val, nullptr, nullptr,
                       d_frame_nnz, d_frame_out_off, d_err, d_ws, ws_bytes, (hipStream_t)stream, &bk);
}

// Writes the device [0, n] offsets of a single frame into the workspace tail.
static int single_frame_offsets(int64_t n, void *ws, size_t ws_bytes, hipStream_t s, int64_t **off) {
    if (ws_bytes < 2 * sizeof(int64_t)) return SHPL_ERR_WORKSPACE;
    // A single frame needs device-side [0, n] offsets; they live in the workspace.
    int64_t *o = (int64_t *)ws;
    hipLaunchKernelGGL(k_set_pair, dim3(1), dim3(1), 0, s, o, (int64_t)0, n);
    SHPL_LAUNCH_CHECK();
    *off = o;
    return SHPL_OK;
}

extern "C" int shpl_gen_index(int64_t n, const void *d_points, int points_dtype, const void *d_voxels,
                              int voxels_itype, int64_t vox_stride, const double *d_P, double im_w,
                              double im_h, int64_t *d_bv_index, double *d_img_index, int64_t ld,
                              int64_t *d_nv, void *d_ws, size_t ws_bytes, void *stream) {
    if (n < 0 || !d_P || !d_bv_index || !d_img_index || !d_nv || !d_ws) return SHPL_ERR_ARG;
    if (n > 0 && (!d_points || !d_voxels)) return SHPL_ERR_ARG;
    if (vox_stride < 2 || ld < n) return SHPL_ERR_BAD_SHAPE;
    hipStream_t s = (hipStream_t)stream;
    int64_t *off;
    int rc = single_frame_offsets(n, d_ws, ws_bytes, s, &off);
    if (rc) return rc;
#define SHPL_GEN(PT, VT)                                                                          \
    {                                                                                             \
        GenStage<PT, VT> st{d_points, d_voxels, vox_stride, d_P, im_w, im_h, d_bv_index,          \
                            d_img_index, ld};                                                     \
        return run_compaction(st, 1, n, off, nullptr, d_nv, nullptr, nullptr, d_ws, ws_bytes, s);   \
    }
    if (points_dtype == SHPL_F64 && voxels_itype == SHPL_I64) SHPL_GEN(double, int64_t)
    if (points_dtype == SHPL_F64 && voxels_itype == SHPL_I32) SHPL_GEN(double, int32_t)
    if (points_dtype == SHPL_F32 && voxels_itype == SHPL_I64) SHPL_GEN(float, int64_t)
    if (points_dtype == SHPL_F32 && voxels_itype == SHPL_I32) SHPL_GEN(float, int32_t)
#undef SHPL_GEN
    return SHPL_ERR_ARG;
}

extern "C" int shpl_produce_index(int64_t nv, const void *d_bv_index, int bv_itype, int64_t bv_stride,
                                  double *d_img_index, int64_t ld, double im_w, double im_h, double bv_h,
                                  double bv_w, double s_img, double s_bv, int64_t *d_mij, int64_t *d_flip,
                                  int32_t *d_cell, int32_t *d_pix, int64_t *d_nk, uint32_t *d_err,
                                  void *d_ws, size_t ws_bytes, void *stream) {
    if (nv < 0 || !d_mij || !d_flip || !d_nk || !d_ws) return SHPL_ERR_ARG;
    if (nv > 0 && (!d_bv_index || !d_img_index)) return SHPL_ERR_ARG;
    if (bv_stride < 2 || ld < nv || !(s_img > 0) || !(s_bv > 0)) return SHPL_ERR_BAD_SHAPE;
    const Geometry g = make_geometry(im_w, im_h, bv_h, bv_w, s_img, s_bv);
    hipStream_t s = (hipStream_t)stream;
    int64_t *off;
    int rc = single_frame_offsets(nv, d_ws, ws_bytes, s, &off);
    if (rc) return rc;
    if (bv_itype == SHPL_I64) {
        ProduceStage<int64_t> st{d_bv_index, bv_stride, d_img_index, ld, g, d_mij, d_flip, d_cell, d_pix, d_err};
        return run_compaction(st, 1, nv, off, nullptr, d_nk, nullptr, d_err, d_ws, ws_bytes, s);
    }
    if (bv_itype == SHPL_I32) {
        ProduceStage<int32_t> st{d_bv_index, bv_stride, d_img_index, ld, g, d_mij, d_flip, d_cell, d_pix, d_err};
        return run_compaction(st, 1, nv, off, nullptr, d_nk, nullptr, d_err, d_ws, ws_bytes, s);
    }
    return SHPL_ERR_ARG;
}

#if SHPL_IDX1_PROBE
// probe builds only: the last k_index1 launch's per-chunk stamps (start, phase 1 done, past the frame barrier,
// aggregates read, points placed, buckets placed, holes written, end), 100 MHz ticks, chunks in launch order
extern "C" int shpl_probe_idx1(uint64_t *host, size_t n_blocks) {
    if (n_blocks > (size_t)shpl::IDX1_PROBE_BLOCKS) n_blocks = shpl::IDX1_PROBE_BLOCKS;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(shpl::g_idx1_probe), 64 * n_blocks, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? SHPL_OK
               : SHPL_ERR_HIP;
}
#endif
