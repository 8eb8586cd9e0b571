// shpl_kitti.hip -- KITTI velodyne scans -> camera-frame point clouds on the
// device: the loader side of the SHPL path.
//
// Reference (host numpy, per frame in the data loader):
//   obj_utils.get_lidar_point_cloud   avod/wavedata/wavedata/tools/obj_detection/obj_utils.py:220-268
//   calib_utils.lidar_to_cam_frame    avod/wavedata/wavedata/tools/core/calib_utils.py:371-410
//   calib_utils.project_to_image      calib_utils.py:281-298
//   kitti_aug.flip_point_cloud        avod/avod/datasets/kitti/kitti_aug.py:24-29
//     (applied to the camera-frame cloud, kitti_dataset.py:305-306)
// Per point: p_cam = rect . [x; y; z; 1] where rect = rows 0-2 of
// R0_rect4 . Tr_velo_to_cam4 (numpy's 4x4 product, done on the host), as the
// dgemm FMA chain numpy uses (dgemv's order for a one-point scan); with an
// image size: keep z > 0, project with P2 (dgemv's order when exactly one
// point has z > 0: the projection's only column) and keep 0 < u < W,
// 0 < v < H (strict). The kept points are compacted in
// scan order by the chunked stable compaction of shpl_compact.h.
// File parsing (read_calibration, read_lidar, get_road_plane) is host code
// (sparse_pooling_amd/kitti.py); the scans arrive here as one [N,4] f32 batch.
#include "shpl_compact.h"

namespace shpl {
namespace {

struct VeloStage {
    static constexpr bool HAS_BUCKETS = false;
    const float *xyzi;  // [N,4]
    const double *rect;  // [F,3,4]
    const double *P;     // [F,3,4] or null (no image filter)
    const double *im;    // [F,2] (w, h)
    double min_int;      // NaN = none
    const int32_t *flip;
    double *out;  // [N,3]

    struct In {
        float x, y, z, i;
    };
    struct Payload {
        double c[3];
    };

    __device__ void load(int64_t i, In &in) const {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        const f32x4 v = reinterpret_cast<const f32x4 *>(xyzi)[i];
        in.x = v[0];
        in.y = v[1];
        in.z = v[2];
        in.i = v[3];
    }
    // AUX = z > 0 (the columns of project_to_image); KEEP_MULTI / KEEP_ONE: the
    // image filter with the projection in dgemm / dgemv order
    __device__ uint32_t eval(const Ctx &c, int f, int64_t, const In &in, Payload &pl) const {
        const double *r = rect + 12 * f;
        const double x = (double)in.x, y = (double)in.y, z = (double)in.z;
        const bool one = c.n_live == 1;
        pl.c[0] = dot4(r, x, y, z, one);
        pl.c[1] = dot4(r + 4, x, y, z, one);
        pl.c[2] = dot4(r + 8, x, y, z, one);
        if (!P) return KEEP_MULTI | KEEP_ONE;  // im_size=None: every point (obj_utils.py:244-246)
        if (!(pl.c[2] > 0.0)) return 0u;
        if (!(isnan(min_int) || (double)in.i > min_int)) return AUX;
        const double w = im[2 * f], h = im[2 * f + 1];
        uint32_t m = AUX;
        double u, v;
        project(P + 12 * f, pl.c[0], pl.c[1], pl.c[2], u, v, false);
        if (u > 0.0 && u < w && v > 0.0 && v < h) m |= KEEP_MULTI;
        project(P + 12 * f, pl.c[0], pl.c[1], pl.c[2], u, v, true);
        if (u > 0.0 && u < w && v > 0.0 && v < h) m |= KEEP_ONE;
        return m;
    }
    __device__ void touch(int, int64_t, const Payload &, bool) const {}
    __device__ void emit(int f, int64_t, int64_t pos, int64_t, const Payload &pl) const {
        const bool fl = flip && flip[f];
        out[3 * pos] = fl ? -pl.c[0] : pl.c[0];
        out[3 * pos + 1] = pl.c[1];
        out[3 * pos + 2] = pl.c[2];
    }
    __device__ void hole(int64_t pos) const {  // NaN rows fail every later range test
        const double nan = __builtin_nan("");
        out[3 * pos] = nan;
        out[3 * pos + 1] = nan;
        out[3 * pos + 2] = nan;
    }
};

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_velo_workspace_bytes(int n_frames, int64_t max_points_per_frame, size_t *bytes) {
    if (!bytes || n_frames < 1 || max_points_per_frame < 0) return SHPL_ERR_ARG;
    *bytes = index_ws_bytes(n_frames, max_points_per_frame);
    return SHPL_OK;
}

extern "C" int shpl_velo_to_cam(int n_frames, const int64_t *d_point_offsets, int64_t max_points_per_frame,
                                const float *d_xyzi, const double *d_rect, const double *d_P,
                                const double *d_im_size, double min_intensity, const int32_t *d_flip,
                                double *d_points, int64_t *d_counts, uint32_t *d_err, void *d_ws, size_t ws_bytes,
                                void *stream) {
    if (n_frames < 1 || !d_point_offsets || !d_rect || !d_counts || !d_ws) return SHPL_ERR_ARG;
    if (max_points_per_frame > 0 && (!d_xyzi || !d_points)) return SHPL_ERR_ARG;
    if ((d_P == nullptr) != (d_im_size == nullptr)) return SHPL_ERR_ARG;
    if (max_points_per_frame < 0) return SHPL_ERR_BAD_SHAPE;
    if (d_xyzi && ((uintptr_t)d_xyzi % 16) != 0) return SHPL_ERR_BAD_SHAPE;  // [N,4] f32 rows, 16-byte loads
    VeloStage st{d_xyzi, d_rect, d_P, d_im_size, min_intensity, d_flip, d_points};
    return run_compaction(st, n_frames, max_points_per_frame, d_point_offsets, nullptr, d_counts, nullptr, d_err,
                          d_ws, ws_bytes, (hipStream_t)stream);
}
