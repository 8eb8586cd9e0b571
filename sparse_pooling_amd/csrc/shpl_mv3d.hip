// shpl_mv3d.hip -- MV3D_TF's SHPL producer on the device.
//
// Reference: point_cloud_2_top_sparse   MV3D_TF_release/lib/utils/construct_voxel.py:37-162
// (called per minibatch from roi_data_layer/minibatch_mv3d_img.py:88-93 with
// img_index2 = np.round(projectToImage(points, P2)).astype(int)).
// Per frame, with camera-frame points reordered to (forward, side, height):
//   keep points strictly inside the forward / side / height ranges;
//   voxel (side, fwd, height) = int((coord - range_min) / res)   [astype(int32)]
//   np.unique(axis=0) orders voxels lexicographically by (side, fwd, height);
//   walking the points in order, a voxel accepts its first VOXEL_POINT_COUNT
//   points; the accepted points, in point order, give
//     img_index = [img_index2; 0], bv_index = (fwd, side),
//     M_val = 1 / (points accepted by the point's voxel)   (MV3D's mean pooling).
// Optionally the front-view augmentation's index transform follows
// (augment_fv, MV3D_TF_release/lib/roi_data_layer/minibatch_mv3d_img.py:191-209).
// Here one workgroup per frame sorts the packed (voxel, point) words
// (shpl_tilesort.h); the thread at the start of each voxel run marks the run's
// first VOXEL_POINT_COUNT points accepted with weight 1/min(run, cap); a
// ballot compaction then emits the accepted points in point order.
#include "shpl_tilesort.h"

namespace shpl {
namespace {

struct Mv3dGeom {
    double fwd_lo, fwd_hi, side_lo, side_hi, h_lo, h_hi;  // strict ranges
    double res, zres;
    int n_side, n_fwd, n_h;  // voxel_full_size = (n_h, n_side, n_fwd)
    int cap;                 // VOXEL_POINT_COUNT
    int log_tile;
    int has_proj;            // 1: img_index2 from P2 on the device
};

// projectToImage + np.round (minibatch_mv3d_img.py:88-91)
// (gemv: the frame has one point, so np.dot has one column -- dgemv's order)
__device__ __forceinline__ void project_round(const double *P, double x, double y, double z, int64_t &u, int64_t &v,
                                              bool gemv) {
    double uf, vf;
    project(P, x, y, z, uf, vf, gemv);
    u = (int64_t)rint(uf);
    v = (int64_t)rint(vf);
}

// voxel key of camera-frame point (x, y, z) or -1 when outside the ranges
__device__ __forceinline__ int64_t voxel_key(const Mv3dGeom &g, double x, double y, double z, int &si, int &fi) {
    const double fwd = z, side = x, h = y;  // points[:, [2, 0, 1, 3]]
    if (!(fwd > g.fwd_lo && fwd < g.fwd_hi && side > g.side_lo && side < g.side_hi && h > g.h_lo && h < g.h_hi))
        return -1;
    si = (int)__ddiv_rn(__dsub_rn(side, g.side_lo), g.res);
    fi = (int)__ddiv_rn(__dsub_rn(fwd, g.fwd_lo), g.res);
    const int hi = (int)__ddiv_rn(__dsub_rn(h, g.h_lo), g.zres);
    return ((int64_t)si * g.n_fwd + fi) * g.n_h + hi;
}

__global__ __launch_bounds__(TS_BLOCK) void k_mv3d_frame(Mv3dGeom g, const int64_t *pt_off, const double *pts,
                                                         int64_t pt_stride, const int64_t *img2, int64_t img2_ld,
                                                         const double *P, const double *fv_aug, uint64_t *tmp,
                                                         uint64_t *srt, int32_t *acc,
                                                         double *img_index, int64_t ld, int64_t *bv_index,
                                                         double *mval, int64_t *frame_n, int32_t *vox_count,
                                                         int64_t *frame_nvox) {
    __shared__ TileSortLds lds;
    const int f = blockIdx.x;
    const int64_t p0 = pt_off[f], p1 = pt_off[f + 1];
    const int64_t n_keys = (int64_t)g.n_side * g.n_fwd * g.n_h;
    const int n_tiles = (int)(((n_keys - 1) >> g.log_tile) + 1);
    // per point: points accepted by its voxel, 0 = rejected (outside the ranges or over the cap)
    for (int64_t i = p0 + threadIdx.x; i < p1; i += TS_BLOCK) acc[i] = 0;
    const int32_t n = tile_sort(
        lds, n_tiles, tmp + p0, srt + p0,
        [&](auto &&emit) {
            for (int64_t i = p0 + threadIdx.x; i < p1; i += TS_BLOCK) {
                const double *q = pts + i * pt_stride;
                int si, fi;
                const int64_t key = voxel_key(g, q[0], q[1], q[2], si, fi);
                if (key >= 0) emit(((uint64_t)key << 32) | (uint32_t)(i - p0));
            }
        },
        [&](uint64_t w) { return (int)((w >> 32) >> g.log_tile); });
    // run starts: accept the first `cap` points of every voxel (point order = word order)
    for (int32_t s = threadIdx.x; s < n; s += TS_BLOCK) {
        const uint64_t key = srt[p0 + s] >> 32;
        if (s > 0 && (srt[p0 + s - 1] >> 32) == key) continue;
        int32_t run = 1;
        while (s + run < n && (srt[p0 + s + run] >> 32) == key) ++run;
        const int32_t a = run < g.cap ? run : g.cap;
        for (int32_t u = 0; u < a; ++u) acc[p0 + (uint32_t)srt[p0 + s + u]] = a;
    }
    block_publish();
    // optional VFE buffers: number_buffer per voxel in voxel order
    if (vox_count) {
        int64_t base = 0;
        for (int32_t b0 = 0; b0 < n; b0 += TS_BLOCK) {
            const int32_t s = b0 + threadIdx.x;
            bool first = false;
            int32_t run = 0;
            if (s < n) {
                const uint64_t key = srt[p0 + s] >> 32;
                first = s == 0 || (srt[p0 + s - 1] >> 32) != key;
                if (first) {
                    run = 1;
                    while (s + run < n && (srt[p0 + s + run] >> 32) == key) ++run;
                }
            }
            const uint64_t m = __ballot(first);
            if ((threadIdx.x & 63) == 0) lds.wsum[threadIdx.x >> 6] = (int32_t)__popcll(m);
            __syncthreads();
            int32_t before = 0, tot = 0;
            for (int w = 0; w < TS_BLOCK / 64; ++w) {
                before += w < (int)(threadIdx.x >> 6) ? lds.wsum[w] : 0;
                tot += lds.wsum[w];
            }
            if (first) vox_count[p0 + base + before + lane_rank(m)] = run < g.cap ? run : g.cap;
            base += tot;
            __syncthreads();
        }
        if (threadIdx.x == 0) frame_nvox[f] = base;
    }
    // emit accepted points in point order
    int64_t kept = 0;
    for (int64_t b0 = p0; b0 < p1; b0 += TS_BLOCK) {
        const int64_t i = b0 + threadIdx.x;
        const int32_t a = i < p1 ? acc[i] : 0;
        const bool keep = a > 0;
        const uint64_t m = __ballot(keep);
        if ((threadIdx.x & 63) == 0) lds.wsum[threadIdx.x >> 6] = (int32_t)__popcll(m);
        __syncthreads();
        int32_t before = 0, tot = 0;
        for (int w = 0; w < TS_BLOCK / 64; ++w) {
            before += w < (int)(threadIdx.x >> 6) ? lds.wsum[w] : 0;
            tot += lds.wsum[w];
        }
        if (keep) {
            const int64_t pos = p0 + kept + before + lane_rank(m);
            const double *q = pts + i * pt_stride;
            int si = 0, fi = 0;
            voxel_key(g, q[0], q[1], q[2], si, fi);
            int64_t u, v;
            if (g.has_proj) {
                project_round(P + 12 * f, q[0], q[1], q[2], u, v, p1 - p0 == 1);
            } else {
                u = img2[i];
                v = img2[img2_ld + i];
            }
            if (fv_aug) {
                // augment_fv (minibatch_mv3d_img.py:205-206): (img_index * ratio + shift).astype(int)
                const double *a = fv_aug + 3 * f;
                u = (int64_t)__dadd_rn(__dmul_rn((double)u, a[0]), a[1]);
                v = (int64_t)__dadd_rn(__dmul_rn((double)v, a[0]), a[2]);
            }
            img_index[pos] = (double)u;
            img_index[ld + pos] = (double)v;
            img_index[2 * ld + pos] = 0.0;
            bv_index[2 * pos] = fi;
            bv_index[2 * pos + 1] = si;
            mval[pos] = __ddiv_rn(1.0, (double)a);  // 1.0 / accepted count (construct_voxel.py:160)
        }
        kept += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) frame_n[f] = kept;
}

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_mv3d_workspace_bytes(int64_t total_points, size_t *bytes) {
    if (!bytes || total_points < 0) return SHPL_ERR_ARG;
    const size_t n = (size_t)(total_points > 0 ? total_points : 1);
    *bytes = 2 * align_up(n * sizeof(uint64_t), 256) + align_up(n * sizeof(int32_t), 256);
    return SHPL_OK;
}

extern "C" int shpl_mv3d_voxels(int n_frames, const int64_t *d_point_offsets, int64_t total_points,
                                const double *d_points, int64_t point_stride, const int64_t *d_img_index2,
                                const double *d_P, const double *d_fv_aug, const double *ranges, double res,
                                double zres, int voxel_point_count, double *d_img_index, int64_t ld, int64_t *d_bv_index,
                                double *d_mval, int64_t *d_frame_n, int32_t *d_number_buffer,
                                int64_t *d_frame_nvox, void *d_ws, size_t ws_bytes, void *stream) {
    if (n_frames < 1 || !d_point_offsets || !ranges || !d_frame_n || !d_ws) return SHPL_ERR_ARG;
    if (total_points > 0 && (!d_points || !d_img_index || !d_bv_index || !d_mval)) return SHPL_ERR_ARG;
    if (!d_img_index2 && !d_P) return SHPL_ERR_ARG;
    if (d_number_buffer && !d_frame_nvox) return SHPL_ERR_ARG;
    if (point_stride < 3 || ld < total_points || !(res > 0) || !(zres > 0) || voxel_point_count < 1 ||
        total_points >= ((int64_t)1 << 31))
        return SHPL_ERR_BAD_SHAPE;
    size_t need;
    shpl_mv3d_workspace_bytes(total_points, &need);
    if (need > ws_bytes) return SHPL_ERR_WORKSPACE;
    Mv3dGeom g{};
    g.fwd_lo = ranges[0];
    g.fwd_hi = ranges[1];
    g.side_lo = ranges[2];
    g.side_hi = ranges[3];
    g.h_lo = ranges[4];
    g.h_hi = ranges[5];
    g.res = res;
    g.zres = zres;
    // construct_voxel.py:77-80: x_max = int((side_hi - side_lo) / res) etc.; sizes are max + 1
    g.n_side = (int)((g.side_hi - g.side_lo) / res) + 1;
    g.n_fwd = (int)((g.fwd_hi - g.fwd_lo) / res) + 1;
    g.n_h = (int)((g.h_hi - g.h_lo) / zres) + 1;
    g.cap = voxel_point_count;
    g.has_proj = d_img_index2 ? 0 : 1;
    const int64_t n_keys = (int64_t)g.n_side * g.n_fwd * g.n_h;
    if (n_keys >= ((int64_t)1 << 31)) return SHPL_ERR_BAD_SHAPE;
    g.log_tile = 0;
    while (((n_keys - 1) >> g.log_tile) + 1 > TS_TILES) ++g.log_tile;
    const size_t n = (size_t)(total_points > 0 ? total_points : 1);
    uint64_t *tmp = (uint64_t *)d_ws;
    uint64_t *srt = (uint64_t *)((char *)d_ws + align_up(n * sizeof(uint64_t), 256));
    int32_t *acc = (int32_t *)((char *)d_ws + 2 * align_up(n * sizeof(uint64_t), 256));
    hipLaunchKernelGGL(k_mv3d_frame, dim3(n_frames), dim3(TS_BLOCK), 0, (hipStream_t)stream, g, d_point_offsets,
                       d_points, point_stride, d_img_index2, total_points, d_P, d_fv_aug, tmp, srt, acc, d_img_index, ld,
                       d_bv_index, d_mval,
                       d_frame_n, d_number_buffer, d_frame_nvox);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}
