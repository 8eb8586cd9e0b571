/*
 * shpl.h -- C ABI of libshpl.so, the MI355X (gfx950) Sparse Non-homogeneous
 * Pooling Layer (SHPL).
 *
 * The reference (YeungLy/Sparse_Pooling) has no native SHPL code: its path is
 * numpy on the host plus four stock TensorFlow 1.8 ops. Each entry point
 * below replaces one piece of that path; the reference interface it stands in
 * for is cited as file:line relative to the reference checkout.
 *
 * Conventions
 *   - Every pointer named d_* is DEVICE memory (HBM), owned by the caller.
 *     The library never allocates: work buffers come from a caller-provided
 *     workspace whose size is returned by the *_workspace_bytes queries.
 *   - Feature maps are NHWC, contiguous per pixel row. A "row" is one BEV
 *     cell (b*Hb*Wb + y*Wb + x) or one image pixel (b*Hi*Wi + v*Wi + u);
 *     several frames of one batch are addressed by these global row ids.
 *   - All calls are stream-ordered on `stream` (a hipStream_t), reentrant,
 *     keep no global mutable state, and never synchronise the host.
 *   - Index errors are reported through a caller-provided device word
 *     (d_err, bit mask SHPL_EBIT_*), mirroring TF-CPU's InvalidArgumentError
 *     without a device->host sync on the hot path; kernels skip offending
 *     entries and never touch memory out of bounds.
 *   - Return value: shpl_status (launch/argument errors only).
 */
#ifndef SHPL_H
#define SHPL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SHPL_OK = 0,
    SHPL_ERR_BAD_SHAPE = 1,  /* inconsistent sizes / strides / alignment */
    SHPL_ERR_INDEX_OOB = 2,  /* host-detectable out-of-range index */
    SHPL_ERR_HIP = 3,        /* a HIP runtime call failed */
    SHPL_ERR_WORKSPACE = 4,  /* workspace too small */
    SHPL_ERR_ARG = 5         /* null pointer / bad enum */
} shpl_status;

/* bits of the device error word */
#define SHPL_EBIT_ROW 1u     /* M row (BEV cell) outside [0, M_size[0]) */
#define SHPL_EBIT_COL 2u     /* M column outside [0, M_size[1]) */
#define SHPL_EBIT_PIXEL 4u   /* source index (b,v,u) outside the image */
#define SHPL_EBIT_VALUES 8u  /* len(M_val) != nnz */
#define SHPL_EBIT_CAPACITY 16u /* a frame holds more points than max_points_per_frame */
#define SHPL_EBIT_BARRIER 32u  /* shpl_build_index_buckets' one-launch form gave up waiting at a frame barrier
                                  (its chunks were not all resident: results of that call are invalid) */

typedef enum { SHPL_F32 = 0, SHPL_BF16 = 1, SHPL_F64 = 2 } shpl_dtype;
typedef enum { SHPL_I32 = 0, SHPL_I64 = 1 } shpl_itype;

/* CSR direction: which side of M the destination rows live on. */
typedef enum {
    SHPL_BY_CELL = 0,   /* destination = BEV cell (M row): img->BEV pooling, d_bev of trans */
    SHPL_BY_PIXEL = 1   /* destination = image pixel of column k: BEV->img, d_img of pooling */
} shpl_direction;

/* Order of the entries that share one destination (TF-CPU accumulation order). */
typedef enum {
    SHPL_ORDER_ENTRY = 0,    /* nnz order: SparseTensorDenseMatMul(M, .)            */
    SHPL_ORDER_COL_ROW = 1,  /* (col,row) order: matmul(sparse_transpose(M), .)     */
    SHPL_ORDER_COL_ENTRY = 2 /* (col, nnz) order: matmul(M, ., adjoint_a=True) and   */
                             /* the gradient of the transposed product              */
} shpl_order;

/* Output composition of a pull. */
typedef enum {
    SHPL_OUT_POOL = 0,    /* out = pooled                                  */
    SHPL_OUT_CONCAT = 1,  /* out = [pass || pooled]   (tf.concat axis=3)    */
    SHPL_OUT_ADD = 2      /* out = pass + pooled      (gradient add_n)      */
} shpl_out_mode;

const char *shpl_version(void);
const char *shpl_status_string(int status);

/* ---------------------------------------------------------------------------
 * Index builder
 * ------------------------------------------------------------------------- */

/* Fused, batched: points -> projection (f64, FMA chain as numpy/OpenBLAS) ->
 * image clip (strict bounds) -> round half-even -> strides -> BEV flatten ->
 * in-grid filter -> stable compaction, for n_frames frames in two launches
 * (a per-chunk count, then the placement), each with one 1024-thread
 * workgroup per 4096 points of every frame. max_points_per_frame bounds the
 * capacity off[f+1]-off[f] of every frame (SHPL_EBIT_CAPACITY otherwise).
 * Replaces gen_sparse_pooling_input_avod + produce_sparse_pooling_input
 * (avod/avod/utils/sparse_pool_utils.py:6-58; projection/clip
 * avod/avod/utils/transform.py:3-40) as called per frame by
 * KittiDataset.load_samples (avod/avod/datasets/kitti/kitti_dataset.py:374-379).
 *
 *   d_point_offsets [n_frames+1] i64 : frame f owns point slots [off[f], off[f+1])
 *   d_point_counts  optional [n_frames] i64: only the first count[f] slots are live
 *                   (the capacity layout shpl_bev_slices emits)
 *   d_points        [N,3] f64 or f32 (camera frame)
 *   d_voxels        [N, vox_stride] i32/i64, columns 0,1 = (x, z) BEV voxel index
 *   d_P             [n_frames, 3, 4] f64 camera matrices (stereo_calib.p2)
 *   im_w, im_h      image size the projection is clipped to ([W,H])
 *   bv_h, bv_w      full-resolution BEV size ((H,W))
 *   s_img, s_bv     strides (stride[0], stride[1] of the reference)
 *   d_mval          optional [N] f32 weight per INPUT point (MV3D 1/count); NULL = 1.0
 * Outputs (capacity layout: frame f's entries at [off[f], off[f] + nnz_f) in
 * point order, -1 sentinels up to off[f+1]; global ids):
 *   d_cell [N] i32  = f*Hb'*Wb' + r           (M row)
 *   d_pix  [N] i32  = f*Hi'*Wi' + v'*Wi' + u' (image pixel of column k)
 *   d_val  [N] f32
 *   d_mij  optional [N,2] i64 = reference Mij_pool rows [r, k_local]
 *   d_flip optional [N,3] i64 = reference img_index_flip_pool rows [0, v', u']
 *   d_frame_nnz     [n_frames] i64 (reference M_size[1] per frame)
 *   d_frame_out_off [n_frames+1] i64 (= d_point_offsets: entry slots of each frame)
 * The column of entry e is e itself (M's columns are arange per frame).
 * A kept entry whose flattened row is negative (the reference keeps it and TF
 * then rejects it) or whose pixel is negative gets cell/pix = -1 and sets
 * SHPL_EBIT_ROW / SHPL_EBIT_PIXEL in *d_err (nullable).
 */
int shpl_build_index_workspace_bytes(int n_frames, int64_t max_points_per_frame, size_t *bytes);
int shpl_build_index(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                     int64_t max_points_per_frame,
                     const void *d_points, int points_dtype, const void *d_voxels, int voxels_itype,
                     int64_t vox_stride, const double *d_P, double im_w, double im_h, double bv_h,
                     double bv_w, double s_img, double s_bv, const float *d_mval,
                     int32_t *d_cell, int32_t *d_pix, float *d_val, int64_t *d_mij,
                     int64_t *d_flip, int64_t *d_frame_nnz, int64_t *d_frame_out_off,
                     uint32_t *d_err, void *d_ws, size_t ws_bytes, void *stream);

/* gen_sparse_pooling_input_avod alone (sparse_pool_utils.py:6-20), one frame:
 * outputs bv_index [nv,2] i64 and img_index 3 rows of stride ld f64 ([u;v;0]),
 * *d_nv = nv. Capacity n. */
int shpl_gen_index(int64_t n, const void *d_points, int points_dtype, const void *d_voxels,
                   int voxels_itype, int64_t vox_stride, const double *d_P, double im_w,
                   double im_h, int64_t *d_bv_index, double *d_img_index, int64_t ld,
                   int64_t *d_nv, void *d_ws, size_t ws_bytes, void *stream);

/* produce_sparse_pooling_input alone (sparse_pool_utils.py:22-58), one frame.
 * d_img_index (3 rows, stride ld, f64) is UPDATED IN PLACE like the
 * reference mutates its input dict. Outputs mij/flip (reference layout) and the
 * device map (cell, pix; val = 1). *d_nk = nk. Capacity nv. */
int shpl_produce_index(int64_t nv, const void *d_bv_index, int bv_itype, int64_t bv_stride,
                       double *d_img_index, int64_t ld, double im_w, double im_h, double bv_h,
                       double bv_w, double s_img, double s_bv, int64_t *d_mij, int64_t *d_flip,
                       int32_t *d_cell, int32_t *d_pix, int64_t *d_nk, uint32_t *d_err,
                       void *d_ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * BEV slice voxelizer: the index builder's input
 * ------------------------------------------------------------------------- */

/* BevSlices.generate_bev(output_indices=True) (avod/avod/core/bev_generators/
 * bev_slices.py:33-156) with VoxelGrid2D.voxelize_2d (avod/wavedata/wavedata/
 * tools/core/voxel_grid_2d.py:43-162), for n_frames frames in one launch.
 *   d_points       [N,3] f64 camera-frame points; frame f owns [off[f], off[f+1])
 *   d_point_counts optional [n_frames] i64: only the first count[f] points are live
 *   d_planes       [n_frames,4] f64 ground planes (a, b, c, d)
 *   area_extents   host [3][2] f64 ([[xmin,xmax],[ymin,ymax],[zmin,zmax]])
 *   slice_lo/hi    host [num_slices] plane offsets of each height slice, computed
 *                  as the reference does (height_lo + s*hpd, + hpd)
 *   density_lo/hi  offsets of the density map's slice (height_lo, height_hi)
 *   density_table  host [16]: min(1, log(n+1)/norm_value), n >= 15 saturates
 * Outputs (capacity N, frame f at [off[f], off[f] + d_frame_nvox[f]); the rest
 * of the frame's slots is left untouched):
 *   d_voxel_indices [N,2] i32 = reference voxel_indices_rot rows (x, nz - z)
 *   d_pts_in_voxel  [N,3] f64 = the first point of each cell (unique_pts)
 *   d_height_maps   optional [n_frames, num_slices, nz, nx] f64 (rotated like the reference)
 *   d_density_map   optional [n_frames, nz, nx] f64
 * Slices are emitted in order and cells in (x, z) order, matching
 * np.vstack(voxel_indices_stack). Workspace: shpl_bev_workspace_bytes. */
int shpl_bev_workspace_bytes(int64_t total_points, int num_slices, size_t *bytes);
int shpl_bev_slices(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                    int64_t total_points,
                    const void *d_points, int points_dtype, const double *d_planes,
                    const double *area_extents, double voxel_size, int num_slices,
                    const double *slice_lo, const double *slice_hi, double density_lo,
                    double density_hi, double height_per_division, const double *density_table,
                    int32_t *d_voxel_indices, double *d_pts_in_voxel, int64_t *d_frame_nvox,
                    double *d_height_maps, double *d_density_map, uint32_t *d_err, void *d_ws,
                    size_t ws_bytes, void *stream);
/* The height and density maps of the last shpl_bev_slices call that used the
 * same workspace d_ws (and the same frames, points and geometry), from the
 * sorted words it left there: a caller can run the voxelizer without maps
 * (d_height_maps = d_density_map = NULL) where its outputs are on a critical
 * path, and write the maps -- ~27 MB of f64 per frame, almost all zeros --
 * later, on another stream (FramePipeline.velo_step: after the layer's
 * streaming pass). zero != 0 first zero-fills both maps (shpl_bev_slices'
 * maps arrive zero-filled; here the caller may have zeroed them itself).
 * Same values as shpl_bev_slices' maps, bit for bit. At most 4096 frames (a
 * shpl_bev_slices call over more frames keeps no per-frame word counts in the
 * workspace: SHPL_ERR_BAD_SHAPE here; its own maps are unaffected). */
int shpl_bev_maps(int n_frames, const int64_t *d_point_offsets, int64_t total_points, const void *d_points,
                  int points_dtype, const double *d_planes, const double *area_extents, double voxel_size,
                  int num_slices, const double *slice_lo, const double *slice_hi, double density_lo,
                  double density_hi, double height_per_division, const double *density_table,
                  double *d_height_maps, double *d_density_map, int zero, const void *d_ws,
                  size_t ws_bytes, void *stream);

/* The network's BEV input from the same sorted words as shpl_bev_maps: the
 * tensor KittiDataset.load_samples stacks, bev_input = np.dstack((*height_maps,
 * density_map)) (avod/avod/datasets/kitti/kitti_dataset.py:368), as the
 * tf.float32 placeholder receives it (rpn_model.py:185-186, filled at :823):
 * d_bev_input [n_frames, nz, nx, num_slices + 1] f32, element (f, y, x, v) =
 * (float) height map v (v < num_slices) or the density map (v = num_slices) of
 * shpl_bev_maps at (f, y, x), rounded to nearest once -- the feed's cast. Half
 * the bytes of the f64 maps, already in the layout the BEV feature extractor
 * reads. Zero-filled first. Same arguments as shpl_bev_maps otherwise. */
int shpl_bev_input(int n_frames, const int64_t *d_point_offsets, int64_t total_points, const void *d_points,
                   int points_dtype, const double *d_planes, const double *area_extents, double voxel_size,
                   int num_slices, const double *slice_lo, const double *slice_hi, double density_lo,
                   double density_hi, double height_per_division, const double *density_table,
                   float *d_bev_input, const void *d_ws, size_t ws_bytes, void *stream);

/* MV3D_TF's producer point_cloud_2_top_sparse
 * (MV3D_TF_release/lib/utils/construct_voxel.py:37-162), n_frames at once:
 *   d_points     [N, point_stride] f64 camera-frame points (x, y, z, ...)
 *   d_img_index2 optional [2, N] i64 rounded projections (minibatch_mv3d_img.py:88-91);
 *                NULL: computed on the device from d_P [n_frames,3,4] like the reference
 *   d_fv_aug     optional [n_frames,3] f64 (expansion_ratio, sx, sy) of augment_fv
 *                (minibatch_mv3d_img.py:191-209): u = int(u*ratio + sx), v = int(v*ratio + sy)
 *   ranges       host [6] f64: fwd (lo, hi), side (lo, hi), height (lo, hi), strict bounds
 *   res, zres, voxel_point_count  cfg.VOXEL_X_SIZE, VOXEL_Z_SIZE, VOXEL_POINT_COUNT
 * Outputs, capacity layout (frame f at [off[f], off[f] + d_frame_n[f])):
 *   d_img_index [3, ld] f64 ([u; v; 0]), d_bv_index [N,2] i64 (fwd, side),
 *   d_mval [N] f64 = 1 / points accepted by the point's voxel;
 *   d_number_buffer optional [N] i32: accepted points per voxel in voxel order,
 *   d_frame_nvox voxels per frame. */
int shpl_mv3d_workspace_bytes(int64_t total_points, size_t *bytes);
int shpl_mv3d_voxels(int n_frames, const int64_t *d_point_offsets, int64_t total_points,
                     const double *d_points, int64_t point_stride, const int64_t *d_img_index2,
                     const double *d_P, const double *d_fv_aug, const double *ranges, double res,
                     double zres, int voxel_point_count, double *d_img_index, int64_t ld, int64_t *d_bv_index,
                     double *d_mval, int64_t *d_frame_n, int32_t *d_number_buffer,
                     int64_t *d_frame_nvox, void *d_ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * KITTI velodyne loader: the BEV voxelizer's input
 * ------------------------------------------------------------------------- */

/* obj_utils.get_lidar_point_cloud (avod/wavedata/wavedata/tools/obj_detection/
 * obj_utils.py:220-268) after read_lidar, for n_frames scans at once:
 * calib_utils.lidar_to_cam_frame (calib_utils.py:371-410), then with an image
 * size: z > 0, project with P2 (calib_utils.py:281-298), 0 < u < W, 0 < v < H;
 * then optionally kitti_aug.flip_point_cloud (kitti_aug.py:24-29).
 *   d_point_offsets [n_frames+1] i64: scan f is rows [off[f], off[f+1]) of d_xyzi
 *   d_xyzi      [N,4] f32 velodyne points (x, y, z, intensity), 16-byte aligned
 *   d_rect      [n_frames,3,4] f64 rows 0-2 of R0_rect4 . Tr_velo_to_cam4 (numpy's
 *               4x4 product on the host, as calib_utils.py:404 forms it)
 *   d_P, d_im_size  [n_frames,3,4] P2 and [n_frames,2] (w, h); both NULL = no filter
 *   min_intensity   NaN = none (see DESIGN.md for the reference's mask bug)
 *   d_flip      optional [n_frames] i32, nonzero = negate x of the kept points
 * Outputs, capacity layout: d_points [N,3] f64 (frame f's kept points at
 * [off[f], off[f] + d_counts[f]) in scan order, NaN rows after). The result
 * feeds shpl_bev_slices (d_point_counts = d_counts) directly. */
int shpl_velo_workspace_bytes(int n_frames, int64_t max_points_per_frame, size_t *bytes);
int shpl_velo_to_cam(int n_frames, const int64_t *d_point_offsets, int64_t max_points_per_frame,
                     const float *d_xyzi, const double *d_rect, const double *d_P, const double *d_im_size,
                     double min_intensity, const int32_t *d_flip, double *d_points, int64_t *d_counts,
                     uint32_t *d_err, void *d_ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Correspondence matrix M: validation + device map (SURVEY a8-a10 inputs)
 * ------------------------------------------------------------------------- */

/* Pack a reference-format M = tf.SparseTensor(indices=Mij [nnz,2] i64,
 * values [n_values] f32, dense_shape=[R, ncols]) and the gather/scatter index
 * img_index_flip [ncols,3] (b,v,u) into the device map used by the pulls,
 * checking every index like TF-CPU's GatherNd / SparseTensorDenseMatMul /
 * ScatterNd kernels (rpn_model.py:328-336, retinanet_model.py:330-340,
 * network.py:243-246 build that SparseTensor from the placeholders).
 * Global ids: cell = row_base + r, col = col_base + k, pix = pix_base +
 * (b*img_h + v)*img_w + u. Invalid entries get -1 and set bits in *d_err. */
int shpl_pack_map(int64_t nnz, const int64_t *d_mij, const float *d_values, int64_t n_values,
                  int64_t n_rows, int64_t n_cols, const void *d_idx, int idx_itype,
                  int64_t img_b, int64_t img_h, int64_t img_w, int64_t row_base, int64_t col_base,
                  int64_t pix_base, int32_t *d_cell, int32_t *d_col, float *d_val,
                  int32_t *d_pix, uint32_t *d_err, void *stream);

/* ---------------------------------------------------------------------------
 * CSR keyed by destination (stable, TF accumulation order)
 * ------------------------------------------------------------------------- */

/* M's entries sorted by destination (all device arrays, caller-owned): a CSR
 * whose row segments are the runs of equal ent_dst. Layout follows the frames
 * of the map: frame f's entries occupy [frame_off[f], frame_off[f] + nnz_f)
 * sorted by (destination, TF order); its remaining capacity slots, and every
 * slot past frame_off[n_frames], hold ent_dst = -1 and are skipped. */
typedef struct {
    int32_t *ent_dst;  /* [nnz_cap] destination row of each sorted entry (-1 = empty slot) */
    int32_t *ent_src;  /* [nnz_cap] source row of each sorted entry                        */
    float *ent_val;    /* [nnz_cap] M value of each sorted entry                           */
    int32_t *ent_col;  /* [nnz_cap] column k of each sorted entry (SHPL_BY_PIXEL; else NULL). A pixel-keyed
                          CSR of shpl_build_csr_buckets may leave it NULL, marked SHPL_CSR_IDENTITY_COLS in
                          flags: every entry of the index builder's maps is a column of its own, and the pulls
                          then sum without per-column partials (bitwise the same: each partial is one product).
                          Any other pixel-keyed CSR without ent_col is SHPL_ERR_ARG for the pulls */
    int64_t n_keys;    /* destination rows (all frames)                                      */
    int64_t nnz_cap;   /* capacity of the entry arrays                                       */
    int32_t *key_range; /* optional [n_keys][2]: (first, end) sorted entry of each destination's
                           run (first == end: no entry). NULL: not built. When set,
                           shpl_build_csr fills it and shpl_pull runs one row-keyed launch. */
    /* optional, read by the sparse pass only (n_frames 0: it walks the whole capacity): the frame
       layout shpl_build_csr was given, so that it walks only the live entries -- frame f's
       [frame_off[f], frame_off[f] + min(frame_nnz[f], frame_off[f+1] - frame_off[f])) -- when
       most of the capacity is empty (raw scans: ~9 k voxel points in 120 k slots per frame).
       At most SHPL_LIVE_MAX_FRAMES frames. */
    const int64_t *frame_off; /* [n_frames + 1] */
    const int64_t *frame_nnz; /* [n_frames]     */
    int64_t n_frames;
    int64_t flags;     /* SHPL_CSR_IDENTITY_COLS: a pixel-keyed CSR whose every entry is a column of its own
                          (built by shpl_build_csr_buckets), so ent_col may be NULL; 0 otherwise */
    int32_t *heads;    /* optional [n_keys][head_k][2] run heads: (ent_src, ent_val bits) of each destination's
                          first min(run, head_k) sorted entries, filled by shpl_build_csr_buckets beside
                          key_range (the other builders take a CSR without them: SHPL_ERR_ARG otherwise). The
                          row-keyed pulls read them in the round trip of key_range instead of reading the
                          entries after it (bitwise the same). NULL: not built. */
    int64_t head_k;    /* 1 .. SHPL_CSR_MAX_HEAD when heads is set */
} shpl_csr;
#define SHPL_CSR_MAX_HEAD 32
#define SHPL_LIVE_MAX_FRAMES 1024
#define SHPL_CSR_IDENTITY_COLS 1

/* Sort the entries of every frame by destination (cell for SHPL_BY_CELL,
 * pix[col] for SHPL_BY_PIXEL) keeping `order` among equal destinations, and
 * gather the per-entry source ids so the pulls read one contiguous list:
 *   BY_CELL : ent_src = pix[col[e]] (image pixel), ent_col unused
 *   BY_PIXEL: ent_src = cell[e] (BEV row),         ent_col = col[e]
 * Frame f owns entries [d_frame_off[f], d_frame_off[f] + d_frame_nnz[f])
 * (d_frame_nnz NULL: the whole range) and destinations
 * [f*keys_per_frame, (f+1)*keys_per_frame); one workgroup sorts one frame
 * (LDS tile histogram + stable rank inside each tile). d_col NULL means
 * col[e] = e. Entries whose row, column or pixel is -1 or whose destination
 * lies outside the frame are left out.
 * With csr->key_range set (or for small batches of frames with at most 65536
 * destinations each) the sort is ONE launch of one workgroup per (frame, range
 * of 1024 destinations): each reads its frame's entries, counts its
 * destinations and the entries below them, places and ranks its own -- no
 * workgroup waits for another -- and writes key_range for its destinations. */
int shpl_csr_workspace_bytes(int64_t n_keys, int64_t nnz_cap, size_t *bytes);
int shpl_build_csr(int direction, int order, int n_frames, const int64_t *d_frame_off,
                   const int64_t *d_frame_nnz, int64_t keys_per_frame, const int32_t *d_cell,
                   const int32_t *d_col, const float *d_val, const int32_t *d_pix,
                   const shpl_csr *csr, void *d_ws, size_t ws_bytes, void *stream);
/* The same sort with the builder chosen explicitly instead of by batch shape
 * (tests and measurements; every builder yields the same entry lists):
 * SHPL_CSR_AUTO = shpl_build_csr's choice, SHPL_CSR_FRAME one workgroup per
 * frame, SHPL_CSR_SEGMENT balanced destination segments, SHPL_CSR_RANGE one
 * workgroup per (frame, destination range) reading the whole frame. Each is
 * the default of some batch shape (shpl_build_csr picks FRAME from 32 frames
 * on, SEGMENT below, RANGE for small batches of at most 65536 destinations
 * per frame); a key_range CSR always takes the range builder. Same arguments
 * and errors as shpl_build_csr otherwise. */
#define SHPL_CSR_AUTO 0
#define SHPL_CSR_FRAME 1
#define SHPL_CSR_SEGMENT 2
#define SHPL_CSR_RANGE 3
int shpl_build_csr_path(int path, int direction, int order, int n_frames, const int64_t *d_frame_off,
                        const int64_t *d_frame_nnz, int64_t keys_per_frame, const int32_t *d_cell,
                        const int32_t *d_col, const float *d_val, const int32_t *d_pix,
                        const shpl_csr *csr, void *d_ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Pull kernels: the sparse gather / scatter-add of SHPL
 * ------------------------------------------------------------------------- */

/* For every destination row d in [0, csr->n_keys):
 *   pooled[d] = sum over its CSR entries e (in CSR order) of
 *               ent_val[e] * src[ent_src[e]*src_stride + src_off + c],  c < c_pool
 *   with csr->ent_col set (SHPL_BY_PIXEL) the entries of one column k are
 *   first summed into a partial (TF's Q[k]) which is then added to pooled
 *   (ScatterNd order); every output element is written exactly once.
 *   mode SHPL_OUT_POOL  : out[d, 0:c_pool] = pooled          (0 where d is empty)
 *   mode SHPL_OUT_CONCAT: out[d, 0:c_pass] = pass[d]; out[d, c_pass:] = pooled
 *   mode SHPL_OUT_ADD   : out[d, 0:c_pool] = pass[d] + pooled
 * f32 arithmetic without FMA contraction (matches TF-CPU bit for bit);
 * SHPL_BF16 stores bf16 and accumulates in f32.
 * Two stream-ordered launches: k_dense writes every row (pass-through half
 * copied, pooled part 0 -- or pass + 0 for ADD) reading no index at all,
 * then k_sparse walks the sorted entries and overwrites the occupied rows'
 * pooled part. shpl_pull = shpl_pull_dense + shpl_pull_sparse on one stream;
 * the split entry points let a caller start the dense pass before M is built
 * (the sparse pass must follow the dense pass of the same output).
 * With csr->key_range set, shpl_pull is instead ONE launch keyed by output row
 * (k_rows: a group of lanes per row writes its pass-through chunks and walks
 * the row's run from key_range for the pooled ones) -- for small, latency-bound
 * layers (config 3), where two dependent launches and a thread per
 * (entry, chunk) cost more than the extra key_range read per row. Results are
 * bitwise the same. shpl_pull_dense / shpl_pull_sparse ignore key_range.
 * Replaces: _sparse_pool_op + concat  (sparse_pool_utils.py:96-103, :72)  -> BY_CELL, CONCAT
 *           _sparse_pool_trans_op + concat (sparse_pool_utils.py:105-117, :87) -> BY_PIXEL, CONCAT
 *           their TF autodiff gradients                       -> the other direction */
int shpl_pull(int direction, int dtype, const shpl_csr *csr, const void *d_src, int64_t src_stride,
              int64_t src_off, int64_t c_pool, const void *d_pass, int64_t pass_stride,
              int64_t pass_off, int64_t c_pass, int mode, void *d_out, int64_t out_stride,
              void *stream);
int shpl_pull_dense(int direction, int dtype, const shpl_csr *csr, const void *d_src,
                    int64_t src_stride, int64_t src_off, int64_t c_pool, const void *d_pass,
                    int64_t pass_stride, int64_t pass_off, int64_t c_pass, int mode, void *d_out,
                    int64_t out_stride, void *stream);
int shpl_pull_sparse(int direction, int dtype, const shpl_csr *csr, const void *d_src,
                     int64_t src_stride, int64_t src_off, int64_t c_pool, const void *d_pass,
                     int64_t pass_stride, int64_t pass_off, int64_t c_pass, int mode, void *d_out,
                     int64_t out_stride, void *stream);
/* The pooled part of every destination row written exactly once, with no streaming pass before it: mode
 * SHPL_OUT_POOL only (out rows' pooled columns; a concat's pass-through half is the caller's, e.g. a
 * shpl_pull_dense with c_pool = 0 beside the index build), csr->key_range required (shpl_build_csr_path(
 * SHPL_CSR_FRAME) fills it from the frame sort). Destinations whose run is empty get zeros; the others the
 * sums of shpl_pull (same order, bitwise). ONE launch: the occupied rows by a wave per 64 sorted entries
 * (cell-keyed rows of >= 32 chunks of 16 bytes; else a thread per (entry, chunk)) beside a wave per 16 rows
 * storing the empty rows' zeros. Replaces: the pooled half of sparse_pool_utils.py:96-103
 * + :72 where k_dense's zeros would be rewritten (wide channels: RetinaNet's 256). */
int shpl_pull_once(int direction, int dtype, const shpl_csr *csr, const void *d_src, int64_t src_stride,
                   int64_t src_off, int64_t c_pool, const void *d_pass, int64_t pass_stride, int64_t pass_off,
                   int64_t c_pass, int mode, void *d_out, int64_t out_stride, void *stream);

/* ---------------------------------------------------------------------------
 * Bucketed pulls: the index build hands the pulls M already cut by
 * destination (small batches, one stream, no CSR launch)
 * ------------------------------------------------------------------------- */

/* shpl_build_index, and in the same two launches the destination buckets of
 * both keys in d_bkt: per key (BEV cell, image pixel) every frame's
 * destinations are cut into ranges of 128, and each (frame, range) bucket
 * lists the frame's entries of that range in entry order -- TF's accumulation
 * order inside every destination, for both directions (the builder's columns
 * are the identity: SHPL_ORDER_ENTRY == SHPL_ORDER_COL_ROW). The count launch
 * adds per-chunk range histograms, the placement launch a stable multisplit.
 * No d_mij / d_flip outputs; nnz_cap = the point capacity (d_cell's length).
 * Limits (SHPL_ERR_BAD_SHAPE otherwise): at most 65536 cells and 65536 pixels
 * per frame, max_points_per_frame below 2^24.
 * Frames of at most 32 chunks of 1024 points run both passes in ONE launch
 * (k_index1: a frame barrier between them inside the launch) when every chunk
 * workgroup of the batch fits on the GPU at once and d_err is given (else the
 * two-launch form);
 * its barrier words live at the start of d_bkt, which must be ZEROED before
 * its first use (shpl_bucket_workspace_reset, or a memset of the whole
 * workspace) -- every call leaves them zero. SHPL_EBIT_BARRIER in *d_err: a
 * barrier gave up, or found its words not zeroed; the call's results are
 * invalid, and after a dirty start the words need shpl_bucket_workspace_reset.
 * Replaces what shpl_build_index + two shpl_build_csr calls feed the pulls
 * (kitti_dataset.py:374-379, then rpn_model.py:330-331's SparseTensor). */
/* Optional riders of shpl_build_index_buckets: the concat's pass-through half
 * of a forward pull, which needs no index -- out row r, channels [0,
 * channels) = src row r (rows: the BEV cells for cell_copy, the pixels for
 * pixel_copy, all frames). Extra workgroups of the two index launches do the
 * copies beside the latency-bound index work (one stream, no fork). Rows and
 * strides 16-byte aligned, channels * element size a multiple of 16
 * (SHPL_ERR_BAD_SHAPE otherwise). Strides in elements. */
typedef struct {
    int dtype;
    const void *src;
    int64_t src_stride;
    void *out;
    int64_t out_stride;
    int64_t channels;
} shpl_pass_copy;

int shpl_bucket_workspace_bytes(int n_frames, int64_t max_points_per_frame, int64_t nnz_cap,
                                int64_t cells_per_frame, int64_t pix_per_frame, size_t *bytes);
/* Zero the frame barrier words of a bucket workspace sized for n_frames (stream-ordered): before its first
 * shpl_build_index_buckets, and after a call that reported SHPL_EBIT_BARRIER. */
int shpl_bucket_workspace_reset(int n_frames, void *d_bkt, size_t bkt_bytes, void *stream);
int shpl_build_index_buckets(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                             int64_t max_points_per_frame, const void *d_points, int points_dtype,
                             const void *d_voxels, int voxels_itype, int64_t vox_stride, const double *d_P,
                             double im_w, double im_h, double bv_h, double bv_w, double s_img, double s_bv,
                             const float *d_mval, int32_t *d_cell, int32_t *d_pix, float *d_val,
                             int64_t *d_frame_nnz, int64_t *d_frame_out_off, uint32_t *d_err, void *d_ws,
                             size_t ws_bytes, int64_t nnz_cap, void *d_bkt, size_t bkt_bytes,
                             const shpl_pass_copy *cell_copy, const shpl_pass_copy *pixel_copy, void *stream);

/* The map shpl_build_index_buckets left: its frame layout, index arrays and
 * bucket workspace (the same sizes as that call). */
typedef struct {
    int n_frames;
    int64_t max_points_per_frame, nnz_cap;
    int64_t cells_per_frame, pix_per_frame;
    const int64_t *frame_off, *frame_nnz; /* [n_frames + 1], [n_frames] */
    const int32_t *cell, *pix;            /* [nnz_cap] global rows, as shpl_build_index writes them */
    const float *val;                     /* [nnz_cap] */
    void *ws;                             /* the bucket workspace */
    size_t ws_bytes;
    const uint32_t *err;                  /* the index call's d_err (NULL if it had none): after a
                                           * SHPL_EBIT_BARRIER the bucket sort reads every bucket as empty, so a
                                           * failed barrier's half-written buckets never address anything; the bit
                                           * stays until the caller clears the word (its maps stay empty until
                                           * then: FusedPipeline.check() clears it and resets the barrier words) */
} shpl_buckets;

/* One pull of shpl_pull_pair: the arguments of shpl_pull after its csr. */
typedef struct {
    int dtype;
    const void *src;
    int64_t src_stride, src_off, c_pool;
    const void *pass;
    int64_t pass_stride, pass_off, c_pass;
    int mode;
    void *out;
    int64_t out_stride;
} shpl_pull_desc;

/* Both CSRs of the map (by_cell: SHPL_BY_CELL, SHPL_ORDER_ENTRY; by_pixel:
 * SHPL_BY_PIXEL, SHPL_ORDER_COL_ROW, ent_col optional; either may be NULL) from
 * the buckets, in ONE launch: a workgroup per (key, frame, range) sorts its
 * bucket by destination, stably (the bucket is in entry order), emits the
 * sorted entries and key_range (when set) and clears the unused capacity --
 * the same lists shpl_build_csr makes of the same index arrays. No counting or
 * bucketing pass: the index build did both. */
int shpl_build_csr_buckets(const shpl_buckets *bk, const shpl_csr *by_cell, const shpl_csr *by_pixel,
                           void *stream);

/* Two row-keyed pulls in ONE launch (shpl_pull over CSRs with key_range):
 * d_cell over by_cell (SHPL_BY_CELL), d_pixel over by_pixel (SHPL_BY_PIXEL);
 * either pair may be NULL (two launches if their dtypes or vector widths
 * differ). Same results, bit for bit,
 * as the two shpl_pull calls. Replaces the forward pair
 * (sparse_pool_utils.py:96-117, with the concats of :72, :87) or, with
 * SHPL_OUT_ADD, its gradient pair. */
int shpl_pull_pair(const shpl_csr *by_cell, const shpl_pull_desc *d_cell, const shpl_csr *by_pixel,
                   const shpl_pull_desc *d_pixel, void *stream);

/* ---------------------------------------------------------------------------
 * Post-fusion 3x3 convolution
 * ------------------------------------------------------------------------- */

typedef enum { SHPL_ACT_NONE = 0, SHPL_ACT_RELU = 1 } shpl_act;

/* out[f,y,x,co] = act(round(fma(acc, scale[co], shift[co] - center[co]*scale[co])))
 *   acc = sum_{ky,kx,ci} in[f, y+ky-1, x+kx-1, ci] * W[ky,kx,ci,co]
 * i.e. (acc - center) * scale + shift with one fused rounding (the per-channel
 * shift - center*scale rounded once in f32); round = to the storage dtype;
 * act RELU = max(bits, 0) on the stored value's bit pattern as a signed
 * integer (negatives, -0 and -NaN -> +0, +NaN stays NaN). Every kernel behind
 * this call (row-streaming or tiled) applies exactly this epilogue, so the
 * same call gives the same bits whichever runs, up to the accumulation order
 * of acc (the kernels sum the MFMA products in different orders). SAME padding (zeros outside the map), stride 1, n_frames frames of h x w
 * pixels, NHWC rows of global id (f*h + y)*w + x. Input channels
 * [0, c_a) are row r of d_a (element r*a_stride + a_off + c), channels
 * [c_a, c_a + c_b) come from d_b:
 *   pool == NULL: row r of d_b (r*b_stride + b_off + c), a second dense map;
 *   pool != NULL: the img->BEV pooled map, computed in the staging from the
 *                 cell-keyed CSR (shpl_build_csr SHPL_BY_CELL, SHPL_ORDER_ENTRY,
 *                 n_keys = n_frames*h*w, entry slots of frame f from
 *                 d_frame_off[f] on) over the image map d_b, with the
 *                 arithmetic of shpl_pull: the result is the conv of
 *                 [a || shpl_pull(SHPL_BY_CELL, ...)] without writing it --
 *                 bitwise, when c_a is a multiple of the staging chunk (8 f32
 *                 / 16 bf16 channels; otherwise the K order differs).
 * d_weights: HWIO [3][3][c_a+c_b][c_out] in the feature dtype (slim.conv2d's
 * variable). d_center / d_scale / d_shift: optional [c_out] f32 (NULL = 0 / 1
 * / 0) -- BatchNorm inference: center = moving_mean, scale = gamma /
 * sqrt(moving_var + eps), shift = beta; conv bias: shift = bias.
 * d_stats (optional, [2][c_out] f64): per-channel sum and sum of squares of
 * the pre-epilogue output, for BatchNorm in training mode (shpl_batch_norm).
 * f32: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation);
 * SHPL_BF16: bf16 storage, v_mfma_f32_32x32x16_bf16, f32 accumulation, one
 * rounding at the store. Workspace: shpl_conv3x3_workspace_bytes, with
 * pool_nnz_cap = pool->nnz_cap for a pooled call and -1 without a pool.
 * bf16 inputs of at most 64 channels (c_a, c_b multiples of 8, 16-byte rows)
 * without d_stats run the row-streaming kernel; pooled, the pooled vector of
 * each occupied cell is computed once into the workspace (shpl_pull's
 * arithmetic) and gathered by the conv's staging.
 * Replaces: bv_fused = sparse_pool_layer(...) (sparse_pool_utils.py:61-92)
 *   followed by slim.conv2d(bv_fused, Ci, [3,3], normalizer_fn=slim.batch_norm)
 *   (avod/avod/core/models/rpn_model.py:338-346, scope pyramid_fusion_pooled_bev;
 *   the img side :347-354) and slim.conv2d(bev_fused, 256, [3,3])
 *   (avod/avod/core/models/retinanet_model.py:343-348). */
int shpl_conv3x3_workspace_bytes(int dtype, int n_frames, int64_t h, int64_t w, int64_t c_a, int64_t c_b,
                                 int64_t c_out, int64_t pool_nnz_cap, int stats, size_t *bytes);
int shpl_conv3x3(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride,
                 int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off,
                 int64_t c_b, const shpl_csr *pool, const int64_t *d_frame_off, const void *d_weights,
                 int64_t c_out, const float *d_center, const float *d_scale, const float *d_shift,
                 int act, void *d_out, int64_t out_stride, double *d_stats, void *d_ws,
                 size_t ws_bytes, void *stream);

/* Whether shpl_conv3x3 with these arguments (d_ws / ws_bytes / d_center / d_scale / d_shift / stream aside;
 * stats = d_stats != NULL) runs the row-streaming form (*rows_form = 1), whose pooled call leaves the
 * occupancy maps and per-run pooled rows in its workspace that shpl_conv3x3_wgrad_reuse reads; 0 for the
 * tiled form, f32, or no pixel. The same predicate shpl_conv3x3 decides by. */
int shpl_conv3x3_rows_form(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride,
                           int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off, int64_t c_b,
                           const shpl_csr *pool, const int64_t *d_frame_off, const void *d_weights, int64_t c_out,
                           int act, const void *d_out, int64_t out_stride, int stats, int *rows_form);

/* BatchNorm in training mode over rows x c, from d_stats of shpl_conv3x3 and
 * count = rows: mean = sum/count, var = sumsq/count - mean^2,
 * y = act((x - mean) * gamma / sqrt(var + eps) + beta), written to d_y
 * (NULL: in place over d_x); moving averages m -= (m - v) * (1 - decay) with
 * the Bessel-corrected variance (TF FusedBatchNorm, slim.batch_norm defaults
 * eps 1e-3, decay 0.999, gamma NULL = 1). d_batch_mean / d_batch_var
 * (optional) receive the batch moments (variance Bessel-corrected, as
 * FusedBatchNorm's outputs). d_ws: 2*c floats; on return it holds the mean
 * and scale = gamma / sqrt(var + eps) that shpl_batch_norm_backward takes. */
int shpl_batch_norm(int dtype, int64_t rows, void *d_x, void *d_y, int64_t stride, int64_t c,
                    const double *d_stats, double count, float eps, const float *d_gamma, const float *d_beta,
                    int act, float *d_moving_mean, float *d_moving_var, float decay, float *d_batch_mean,
                    float *d_batch_var, float *d_ws, void *stream);

/* ---------------------------------------------------------------------------
 * Post-fusion conv backward (the TF autodiff of rpn_model.py:338-354)
 * ------------------------------------------------------------------------- */

/* BatchNorm (+ ReLU) backward over rows x c. g_bn = g * [y > 0] when act is
 * SHPL_ACT_RELU (d_y = the layer output; d_y NULL: y recomputed from d_raw
 * as (raw - mean) * scale + beta with the forward's rounding -- the same mask,
 * one map less to read), xhat = (raw - mean) * scale / gamma
 * (d_raw = the conv output). Per channel (f64, fixed order):
 * dbeta = sum g_bn, dgamma = sum g_bn * xhat; then
 *   training:  g_raw = scale * (g_bn - dbeta / rows - xhat * dgamma / rows)
 *   inference: g_raw = scale * g_bn   (mean / scale from the moving statistics)
 * d_mean / d_scale NULL: 0 / 1 -- a conv bias instead of BatchNorm (dbeta is
 * then the bias gradient). Workspace: shpl_batch_norm_backward_workspace_bytes. */
int shpl_batch_norm_backward_workspace_bytes(int64_t rows, int64_t c, size_t *bytes);
int shpl_batch_norm_backward(int dtype, int64_t rows, const void *d_y, const void *d_raw, const void *d_gy,
                             int64_t stride, int64_t c, const float *d_mean, const float *d_scale,
                             const float *d_gamma, const float *d_beta, int act, int training, void *d_graw,
                             float *d_dbeta, float *d_dgamma, void *d_ws, size_t ws_bytes, void *stream);

/* Input gradient: dx = conv3x3_SAME(gy, W') with W'[ky][kx][co][ci] =
 * W[2-ky][2-kx][ci][co], the forward conv kernel on transposed packed
 * weights. d_weights: the forward's HWIO [3][3][c_dx][c_gy]. With d_dx_b
 * set, channels [0, c_split) go to d_dx and [c_split, c_dx) to d_dx_b (the
 * gradients of the conv's two sources, e.g. BEV and pooled image channels,
 * as separate dense maps); with d_dx_b NULL, c_split is ignored. Workspace:
 * shpl_conv3x3_workspace_bytes(dtype, n_frames, h, w, c_gy, 0, c_dx, -1, 0). */
int shpl_conv3x3_dgrad(int dtype, int n_frames, int64_t h, int64_t w, const void *d_gy, int64_t gy_stride,
                       int64_t c_gy, const void *d_weights, int64_t c_dx, void *d_dx, int64_t dx_stride,
                       int64_t c_split, void *d_dx_b, int64_t dx_b_stride, void *d_ws, size_t ws_bytes,
                       void *stream);

/* shpl_conv3x3_dgrad of the pooled bf16 fusion conv's two maps, d_dx_b (the pooled channels' gradient) written
 * only at the cells the pool's CSR has entries for -- the rows a pixel-keyed pull of it back to the image reads
 * (shpl_pull SHPL_BY_PIXEL); its other cells are left as they were. The occupancy comes from the forward
 * shpl_conv3x3 call over the same map, frames and shape (A = c_split channels, B = c_dx - c_split pooled
 * channels, c_gy outputs) that left it in d_fwd_ws (fwd_stats: whether that call took statistics), as
 * shpl_conv3x3_wgrad_reuse reads it: valid only for a forward for which shpl_conv3x3_rows_form reported 1;
 * what this call can check of that is SHPL_ERR_ARG when false. d_dx and the written cells of d_dx_b are
 * shpl_conv3x3_dgrad's, bit for bit. When the input gradient itself does not run the row-streaming form (f32,
 * misaligned maps) or has more than 32 gradient channels (c_gy), d_dx_b is written whole.
 * Replaces: the image half of TF's conv2d backprop input in the rpn_model.py:338-354 fusion, which the
 * gradient of tf.gather_nd / tf.segment_sum (sparse_pool_utils.py:96-117) reads only at occupied cells. */
int shpl_conv3x3_dgrad_reuse(int dtype, int n_frames, int64_t h, int64_t w, const void *d_gy, int64_t gy_stride,
                             int64_t c_gy, const void *d_weights, int64_t c_dx, void *d_dx, int64_t dx_stride,
                             int64_t c_split, void *d_dx_b, int64_t dx_b_stride, void *d_ws, size_t ws_bytes,
                             const shpl_csr *pool, const void *d_fwd_ws, size_t fwd_ws_bytes, int fwd_stats,
                             void *stream);

/* Weight gradient: dw[ky][kx][ci][co] = sum over pixels of x[p + (ky-1, kx-1)][ci]
 * * gy[p][co], x given exactly as shpl_conv3x3's input (A channels, then B
 * channels, dense or pooled from the CSR -- recomputed, never stored). f32
 * MFMA (bf16: bf16 MFMA, exact products, f32 accumulation), per-workgroup
 * partials summed in a fixed order (f64): deterministic. d_dw: f32 HWIO
 * [3][3][c_a+c_b][c_out]. Workspace: pool_nnz_cap as shpl_conv3x3's (-1: B
 * dense or absent; with a pool, its CSR's nnz_cap, which sizes the compact
 * buffer of pooled runs of the bf16 form). */
int shpl_conv3x3_wgrad_workspace_bytes(int dtype, int n_frames, int64_t h, int64_t w, int64_t c_a, int64_t c_b,
                                       int64_t c_out, int64_t pool_nnz_cap, size_t *bytes);
int shpl_conv3x3_wgrad(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride,
                       int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off, int64_t c_b,
                       const shpl_csr *pool, const int64_t *d_frame_off, const void *d_gy, int64_t gy_stride,
                       int64_t c_out, float *d_dw, void *d_ws, size_t ws_bytes, void *stream);

/* shpl_conv3x3_wgrad of the pooled bf16 form reading the pooled operand (the cell-keyed CSR's occupancy maps
 * and per-run pooled rows) that a forward shpl_conv3x3 call over the same map, image, frames, shape and
 * channels left in its workspace, instead of preparing it again (k_occ_frame + k_pool_runs): the training
 * step's weight gradient after its forward. d_fwd_ws / fwd_ws_bytes: that call's workspace, not written since;
 * fwd_stats: whether that call took statistics (its workspace layout). Valid only for a forward call for which
 * shpl_conv3x3_rows_form reported 1 (the caller's to establish: the forward's act and output pointer are not
 * arguments here); what this call can check of that predicate and finds false is SHPL_ERR_ARG. When the
 * weight gradient itself does not run the row-streaming form the workspace is not read. Same results as
 * shpl_conv3x3_wgrad, bit for bit. */
int shpl_conv3x3_wgrad_reuse(int dtype, int n_frames, int64_t h, int64_t w, const void *d_a, int64_t a_stride,
                             int64_t a_off, int64_t c_a, const void *d_b, int64_t b_stride, int64_t b_off,
                             int64_t c_b, const shpl_csr *pool, const int64_t *d_frame_off, const void *d_gy,
                             int64_t gy_stride, int64_t c_out, float *d_dw, void *d_ws, size_t ws_bytes,
                             const void *d_fwd_ws, size_t fwd_ws_bytes, int fwd_stats, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SHPL_H */
