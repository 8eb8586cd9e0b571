// shpl_bev.hip -- device BEV slice voxelizer: the input side of the SHPL
// index builder.
//
// Reference (host numpy, once per frame in the data loader, ~32 ms/frame):
//   BevSlices.generate_bev(output_indices=True)  avod/avod/core/bev_generators/bev_slices.py:33-156
//   VoxelGrid2D.voxelize_2d                      avod/wavedata/wavedata/tools/core/voxel_grid_2d.py:43-162
//   create_slice_filter / get_point_filter       avod/avod/datasets/kitti/kitti_utils.py:79-107,
//                                                avod/wavedata/wavedata/tools/obj_detection/obj_utils.py:444-491
//   dist_to_plane                                avod/wavedata/wavedata/tools/core/geometry_utils.py:26-40
//   _create_density_map                          avod/avod/core/bev_generators/bev_generator.py:23-41
//
// What the reference computes, per height slice s (and once more over the
// whole height range for the density map): keep the points inside the area
// extents whose plane offset lies in [lo_s, hi_s); discretise by
// floor(p / voxel_size); lexsort by (x, z, y) (stable); keep the first point
// of every (x, z) cell -- the smallest discrete y, ties by point order; emit
// the cells in (x, z) order with that point, its height above the ground
// plane and the cell's point count.
//
// Here one 1024-thread workgroup voxelizes one frame, all slices at once:
// every (point, slice) membership is an entry keyed
//   v * n_cells + x_idx * nz + z_idx   (v = slice, or num_slices = density)
// and packed with (discrete y, point index) into one 64-bit word whose
// numeric order IS the reference's lexsort order. An LDS tile histogram +
// scan + LDS-atomic placement + in-tile rank (the k_csr_frame scheme) sorts
// the words; the first word of each key run is the cell's point and the run
// length its count. Outputs keep the reference's order: slice-major, then
// (x, z) ascending, exactly np.vstack(voxel_indices_stack).
#include "shpl_tilesort.h"

namespace shpl {
namespace {

constexpr int BEV_BLOCK = TS_BLOCK;
constexpr int BEV_TILES = TS_TILES;
constexpr int BEV_MAX_SLICES = 8;
constexpr int KEY_SHIFT = 42;  // [63:42] key, [41:32] discrete y - y0, [31:0] point index in frame

struct BevGeom {
    double ext[3][2];     // area extents (strict bounds)
    double vs;            // voxel size
    double lo[BEV_MAX_SLICES + 1], hi[BEV_MAX_SLICES + 1];  // plane offsets; [num_slices] = density range
    double hpd;           // height per division
    double dens[16];      // min(1, log(n + 1) / norm_value) for n = 0..15 (n >= 15 -> 1.0)
    int num_slices;
    int min_x, min_y, min_z;  // floor(ext_min / vs)
    int nx, nz;           // divisions
    int log_tile;
};

__device__ __forceinline__ bool below(const double *pl, double off, double x, double y, double z) {
    // obj_utils.get_point_filter: np.dot(plane + [0,0,0,-off], [x;y;z;1]) < 0
    double s = __dmul_rn(pl[0], x);
    s = __fma_rn(pl[1], y, s);
    s = __fma_rn(pl[2], z, s);
    s = __fma_rn(__dsub_rn(pl[3], off), 1.0, s);
    return s < 0.0;
}

template <typename PT>
struct Pt {
    static __device__ __forceinline__ void load(const void *p, int64_t i, double &x, double &y, double &z) {
        const PT *q = reinterpret_cast<const PT *>(p) + 3 * i;
        x = (double)q[0];
        y = (double)q[1];
        z = (double)q[2];
    }
};

// Entries of one point: calls emit(word) for each slice it is in and for the density range.
template <typename PT, typename F>
__device__ __forceinline__ void point_entries(const BevGeom &g, const double *plane, const void *pts, int64_t i,
                                              uint32_t li, int64_t n_cells, F &&emit) {
    double x, y, z;
    Pt<PT>::load(pts, i, x, y, z);
    const bool inside = x > g.ext[0][0] && x < g.ext[0][1] && y > g.ext[1][0] && y < g.ext[1][1] &&
                        z > g.ext[2][0] && z < g.ext[2][1];
    if (!inside) return;
    // voxelize_2d: floor(pts / voxel_size).astype(int32)
    const int xd = (int)floor(__ddiv_rn(x, g.vs));
    const int yd = (int)floor(__ddiv_rn(y, g.vs));
    const int zd = (int)floor(__ddiv_rn(z, g.vs));
    const int64_t cell = (int64_t)(xd - g.min_x) * g.nz + (zd - g.min_z);
    const uint64_t low = ((uint64_t)(uint32_t)(yd - g.min_y) << 32) | li;
    for (int s = 0; s <= g.num_slices; ++s) {
        // create_slice_filter: xor(filter(hi), filter(lo)), both inside the extents
        if (below(plane, g.hi[s], x, y, z) != below(plane, g.lo[s], x, y, z))
            emit(((uint64_t)(s * n_cells + cell) << KEY_SHIFT) | low);
    }
}

template <typename PT>
__global__ __launch_bounds__(BEV_BLOCK) void k_bev_frame(BevGeom g, const int64_t *pt_off, const int64_t *pt_count,
                                                         const void *pts,
                                                         const double *planes, uint64_t *tmp, uint64_t *srt,
                                                         int64_t ent_per_point, int32_t *vox_out, double *pts_out,
                                                         int64_t *frame_nvox, double *hmaps, double *dmap,
                                                         int32_t *frame_nent, uint32_t *err) {
    __shared__ TileSortLds lds;
    const int f = blockIdx.x;
    const int64_t p0 = pt_off[f], cap_end = pt_off[f + 1];
    // live points: [p0, p0 + count) when counts are given (capacity layout input, e.g. shpl_velo_to_cam)
    const int64_t p1 = pt_count ? (p0 + pt_count[f] < cap_end ? p0 + pt_count[f] : cap_end) : cap_end;
    const int64_t t0 = p0 * ent_per_point;  // this frame's entry slots
    const double *plane = planes + 4 * f;
    const int64_t n_cells = (int64_t)g.nx * g.nz;
    const int64_t n_keys = n_cells * (g.num_slices + 1);
    const int n_tiles = (int)(((n_keys - 1) >> g.log_tile) + 1);
    // 1-4. sort all (point, slice) words: numeric order = (key, discrete y, point index)
    const int32_t n_ent = tile_sort(
        lds, n_tiles, tmp + t0, srt + t0,
        [&](auto &&emit) {
            for (int64_t i = p0 + threadIdx.x; i < p1; i += BEV_BLOCK)
                point_entries<PT>(g, plane, pts, i, (uint32_t)(i - p0), n_cells, emit);
        },
        [&](uint64_t w) { return (int)((w >> KEY_SHIFT) >> g.log_tile); });
    int32_t *wsum = lds.wsum;
    // 5. one output per key run, slice cells compacted in sorted order
    const double a = plane[0], b = plane[1], c = plane[2], d = plane[3];
    const double norm = sqrt(__dadd_rn(__dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b)), __dmul_rn(c, c)));
    const int64_t cap = cap_end - p0;
    int64_t kept = 0;
    const int wid = threadIdx.x >> 6;
    for (int32_t base = 0; base < n_ent; base += BEV_BLOCK) {
        const int32_t s = base + threadIdx.x;
        bool first = false, slice_cell = false;
        uint64_t me = 0, key = 0;
        if (s < n_ent) {
            me = srt[t0 + s];
            key = me >> KEY_SHIFT;
            first = s == 0 || (srt[t0 + s - 1] >> KEY_SHIFT) != key;
            slice_cell = first && (int64_t)key < (int64_t)g.num_slices * n_cells;
        }
        const uint64_t m = __ballot(slice_cell);
        if ((threadIdx.x & 63) == 0) wsum[wid] = (int32_t)__popcll(m);
        __syncthreads();
        int32_t before = 0, tot = 0;
        for (int w = 0; w < BEV_BLOCK / 64; ++w) {
            before += w < wid ? wsum[w] : 0;
            tot += wsum[w];
        }
        if (first) {
            const int v = (int)((int64_t)key / n_cells);
            const int64_t cell = (int64_t)key - (int64_t)v * n_cells;
            const int xi = (int)(cell / g.nz), zi = (int)(cell - (int64_t)xi * g.nz);
            const int64_t pix = (int64_t)(g.nz - 1 - zi) * g.nx + xi;  // np.flip(map.T, axis=0)
            if (v < g.num_slices) {
                const int64_t pos = kept + before + lane_rank(m);
                const int64_t li = (int64_t)(uint32_t)me;
                double x, y, z;
                Pt<PT>::load(pts, p0 + li, x, y, z);
                if (pos < cap) {
                    vox_out[2 * (p0 + pos)] = xi;
                    vox_out[2 * (p0 + pos) + 1] = g.nz - zi;  // bev_slices.py:108 (num_div_z - z)
                    pts_out[3 * (p0 + pos)] = x;
                    pts_out[3 * (p0 + pos) + 1] = y;
                    pts_out[3 * (p0 + pos) + 2] = z;
                } else if (err) {
                    atomicOr(err, SHPL_EBIT_ROW);
                }
                if (hmaps) {
                    // dist_to_plane: (a*x + b*y + c*z + d) / sqrt(a^2 + b^2 + c^2)
                    const double dist =
                        __ddiv_rn(__dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(a, x), __dmul_rn(b, y)), __dmul_rn(c, z)), d),
                                  norm);
                    hmaps[((int64_t)f * g.num_slices + v) * n_cells + pix] = __ddiv_rn(__dsub_rn(dist, g.lo[v]), g.hpd);
                }
            } else if (dmap) {
                int32_t n = 1;
                while (s + n < n_ent && (srt[t0 + s + n] >> KEY_SHIFT) == key) ++n;
                dmap[(int64_t)f * n_cells + pix] = n < 16 ? g.dens[n] : 1.0;
            }
        }
        kept += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        frame_nvox[f] = kept < cap ? kept : cap;
        if (frame_nent) frame_nent[f] = n_ent;  // the sorted words stay in the workspace for shpl_bev_maps
    }
}

// The height and density maps from the sorted words a k_bev_frame launch left in the workspace
// (shpl_bev_maps): the same values step 5 above writes, by a grid of BEV_MAP_SPLIT workgroups per
// frame over its words -- a cell's first word writes its height (slices) or count-derived density.
constexpr int BEV_MAP_SPLIT = 16;
// bev_in (shpl_bev_input): the same values, rounded to f32, interleaved [F, nz, nx, S + 1] instead of the
// planar f64 maps (channel v < S: height slice v, channel S: density).
template <typename PT>
__global__ __launch_bounds__(SHPL_BLOCK) void k_bev_maps(BevGeom g, const int64_t *pt_off, const void *pts,
                                                        const double *planes, const uint64_t *srt,
                                                        int64_t ent_per_point, const int32_t *frame_nent,
                                                        double *hmaps, double *dmap, float *bev_in) {
    const int f = blockIdx.y;
    const int64_t p0 = pt_off[f], t0 = p0 * ent_per_point;
    const int32_t n_ent = frame_nent[f];
    const int64_t n_cells = (int64_t)g.nx * g.nz;
    const double *plane = planes + 4 * f;
    const double a = plane[0], b = plane[1], c = plane[2], d = plane[3];
    const double norm = sqrt(__dadd_rn(__dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b)), __dmul_rn(c, c)));
    for (int32_t s = blockIdx.x * SHPL_BLOCK + threadIdx.x; s < n_ent; s += BEV_MAP_SPLIT * SHPL_BLOCK) {
        const uint64_t me = srt[t0 + s];
        const uint64_t key = me >> KEY_SHIFT;
        if (s > 0 && (srt[t0 + s - 1] >> KEY_SHIFT) == key) continue;  // not the cell's first word
        const int v = (int)((int64_t)key / n_cells);
        const int64_t cell = (int64_t)key - (int64_t)v * n_cells;
        const int xi = (int)(cell / g.nz), zi = (int)(cell - (int64_t)xi * g.nz);
        const int64_t pix = (int64_t)(g.nz - 1 - zi) * g.nx + xi;  // np.flip(map.T, axis=0)
        const int64_t in_at = ((int64_t)f * n_cells + pix) * (g.num_slices + 1) + v;  // bev_in element
        if (v < g.num_slices) {
            if (!hmaps && !bev_in) continue;
            double x, y, z;
            Pt<PT>::load(pts, p0 + (int64_t)(uint32_t)me, x, y, z);
            const double dist =
                __ddiv_rn(__dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(a, x), __dmul_rn(b, y)), __dmul_rn(c, z)), d), norm);
            const double h = __ddiv_rn(__dsub_rn(dist, g.lo[v]), g.hpd);
            if (hmaps) hmaps[((int64_t)f * g.num_slices + v) * n_cells + pix] = h;
            if (bev_in) bev_in[in_at] = __double2float_rn(h);
        } else if (dmap || bev_in) {
            int32_t n = 1;
            while (s + n < n_ent && (srt[t0 + s + n] >> KEY_SHIFT) == key) ++n;
            const double dn = n < 16 ? g.dens[n] : 1.0;
            if (dmap) dmap[(int64_t)f * n_cells + pix] = dn;
            if (bev_in) bev_in[in_at] = __double2float_rn(dn);
        }
    }
}

// frames of one call whose sorted words shpl_bev_maps / shpl_bev_input can read back (the per-frame word
// counts in the workspace); a larger shpl_bev_slices call works as before but leaves no counts
constexpr int BEV_MAX_FRAMES = 4096;

size_t bev_half_bytes(int64_t total_points, int num_slices) {
    const size_t n = (size_t)(total_points > 0 ? total_points : 1) * (size_t)(num_slices + 1);
    return align_up(n * sizeof(uint64_t), 256);
}

// BevGeom of the call's host arguments (SHPL_OK or a status).
int bev_geom(const double *area_extents, double voxel_size, int num_slices, const double *slice_lo,
             const double *slice_hi, double density_lo, double density_hi, double height_per_division,
             const double *density_table, BevGeom &g) {
    if (!area_extents || !slice_lo || !slice_hi || !density_table) return SHPL_ERR_ARG;
    if (num_slices < 1 || num_slices > BEV_MAX_SLICES || !(voxel_size > 0)) return SHPL_ERR_BAD_SHAPE;
    g = BevGeom{};
    for (int i = 0; i < 3; ++i) {
        g.ext[i][0] = area_extents[2 * i];
        g.ext[i][1] = area_extents[2 * i + 1];
    }
    g.vs = voxel_size;
    g.num_slices = num_slices;
    for (int s = 0; s < num_slices; ++s) {
        g.lo[s] = slice_lo[s];
        g.hi[s] = slice_hi[s];
    }
    g.lo[num_slices] = density_lo;
    g.hi[num_slices] = density_hi;
    g.hpd = height_per_division;
    for (int n = 0; n < 16; ++n) g.dens[n] = density_table[n];
    // voxel_grid_2d.py:127-149: min = floor(ext_min / vs), max = ceil(ext_max / vs - 1), y collapsed
    g.min_x = (int)floor(g.ext[0][0] / voxel_size);
    g.min_y = (int)floor(g.ext[1][0] / voxel_size);
    g.min_z = (int)floor(g.ext[2][0] / voxel_size);
    g.nx = (int)(ceil(g.ext[0][1] / voxel_size - 1) - g.min_x + 1);
    g.nz = (int)(ceil(g.ext[2][1] / voxel_size - 1) - g.min_z + 1);
    const int ny = (int)(floor(g.ext[1][1] / voxel_size) - g.min_y + 1);
    if (g.nx < 1 || g.nz < 1 || ny < 1 || ny >= 1024) return SHPL_ERR_BAD_SHAPE;
    const int64_t n_keys = (int64_t)g.nx * g.nz * (num_slices + 1);
    if (n_keys >= ((int64_t)1 << 22)) return SHPL_ERR_BAD_SHAPE;  // key field of the packed word
    g.log_tile = 0;
    while (((n_keys - 1) >> g.log_tile) + 1 > BEV_TILES) ++g.log_tile;
    return SHPL_OK;
}

}  // namespace
}  // namespace shpl

using namespace shpl;

extern "C" int shpl_bev_workspace_bytes(int64_t total_points, int num_slices, size_t *bytes) {
    if (!bytes || total_points < 0 || num_slices < 1 || num_slices > BEV_MAX_SLICES) return SHPL_ERR_ARG;
    *bytes = 2 * bev_half_bytes(total_points, num_slices) + align_up(sizeof(int32_t) * BEV_MAX_FRAMES, 256);
    return SHPL_OK;
}

extern "C" int shpl_bev_slices(int n_frames, const int64_t *d_point_offsets, const int64_t *d_point_counts,
                               int64_t total_points,
                               const void *d_points, int points_dtype, const double *d_planes,
                               const double *area_extents, double voxel_size, int num_slices,
                               const double *slice_lo, const double *slice_hi, double density_lo,
                               double density_hi, double height_per_division, const double *density_table,
                               int32_t *d_voxel_indices, double *d_pts_in_voxel, int64_t *d_frame_nvox,
                               double *d_height_maps, double *d_density_map, uint32_t *d_err, void *d_ws,
                               size_t ws_bytes, void *stream) {
    if (n_frames < 1 || !d_point_offsets || !d_planes || !area_extents || !slice_lo || !slice_hi ||
        !density_table || !d_frame_nvox || !d_ws)
        return SHPL_ERR_ARG;
    if (num_slices < 1 || num_slices > BEV_MAX_SLICES || !(voxel_size > 0)) return SHPL_ERR_BAD_SHAPE;
    if (total_points > 0 && (!d_points || !d_voxel_indices || !d_pts_in_voxel)) return SHPL_ERR_ARG;
    if (total_points >= ((int64_t)1 << 31)) return SHPL_ERR_BAD_SHAPE;
    size_t need;
    shpl_bev_workspace_bytes(total_points, num_slices, &need);
    if (need > ws_bytes) return SHPL_ERR_WORKSPACE;
    BevGeom g;
    const int rc = bev_geom(area_extents, voxel_size, num_slices, slice_lo, slice_hi, density_lo, density_hi,
                            height_per_division, density_table, g);
    if (rc) return rc;
    const size_t half = bev_half_bytes(total_points, num_slices);
    uint64_t *tmp = (uint64_t *)d_ws;
    uint64_t *srt = (uint64_t *)((char *)d_ws + half);
    int32_t *nent = n_frames <= BEV_MAX_FRAMES ? (int32_t *)((char *)d_ws + 2 * half) : nullptr;
    hipStream_t s = (hipStream_t)stream;
    const int64_t per_map = (int64_t)g.nx * g.nz;
    // the maps' zeros: a streaming kernel (hipMemsetAsync's fill ran at ~2.2 TB/s, beside k_dense)
    if (d_height_maps)
        SHPL_HIP_CHECK(zero_fill(d_height_maps, sizeof(double) * (size_t)(per_map * num_slices * n_frames), s));
    if (d_density_map) SHPL_HIP_CHECK(zero_fill(d_density_map, sizeof(double) * (size_t)(per_map * n_frames), s));
    if (points_dtype == SHPL_F64)
        hipLaunchKernelGGL(k_bev_frame<double>, dim3(n_frames), dim3(BEV_BLOCK), 0, s, g, d_point_offsets,
                           d_point_counts, d_points,
                           d_planes, tmp, srt, (int64_t)(num_slices + 1), d_voxel_indices, d_pts_in_voxel,
                           d_frame_nvox, d_height_maps, d_density_map, nent, d_err);
    else
        return SHPL_ERR_ARG;
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

extern "C" int shpl_bev_maps(int n_frames, const int64_t *d_point_offsets, int64_t total_points, const void *d_points,
                             int points_dtype, const double *d_planes, const double *area_extents, double voxel_size,
                             int num_slices, const double *slice_lo, const double *slice_hi, double density_lo,
                             double density_hi, double height_per_division, const double *density_table,
                             double *d_height_maps, double *d_density_map, int zero, const void *d_ws,
                             size_t ws_bytes, void *stream) {
    if (n_frames < 1 || !d_point_offsets || !d_planes || !d_ws) return SHPL_ERR_ARG;
    if (points_dtype != SHPL_F64 || (total_points > 0 && !d_points)) return SHPL_ERR_ARG;
    if (total_points < 0 || total_points >= ((int64_t)1 << 31) || n_frames > BEV_MAX_FRAMES) return SHPL_ERR_BAD_SHAPE;
    BevGeom g;
    const int rc = bev_geom(area_extents, voxel_size, num_slices, slice_lo, slice_hi, density_lo, density_hi,
                            height_per_division, density_table, g);
    if (rc) return rc;
    size_t need;
    shpl_bev_workspace_bytes(total_points, num_slices, &need);
    if (need > ws_bytes) return SHPL_ERR_WORKSPACE;
    const size_t half = bev_half_bytes(total_points, num_slices);
    const uint64_t *srt = (const uint64_t *)((const char *)d_ws + half);
    const int32_t *nent = (const int32_t *)((const char *)d_ws + 2 * half);
    hipStream_t s = (hipStream_t)stream;
    const int64_t per_map = (int64_t)g.nx * g.nz;
    if (zero) {
        if (d_height_maps)
            SHPL_HIP_CHECK(zero_fill(d_height_maps, sizeof(double) * (size_t)(per_map * num_slices * n_frames), s));
        if (d_density_map) SHPL_HIP_CHECK(zero_fill(d_density_map, sizeof(double) * (size_t)(per_map * n_frames), s));
    }
    if (!d_height_maps && !d_density_map) return SHPL_OK;
    hipLaunchKernelGGL(k_bev_maps<double>, dim3(BEV_MAP_SPLIT, n_frames), dim3(SHPL_BLOCK), 0, s, g, d_point_offsets,
                       d_points, d_planes, srt, (int64_t)(num_slices + 1), nent, d_height_maps, d_density_map,
                       (float *)nullptr);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

extern "C" int shpl_bev_input(int n_frames, const int64_t *d_point_offsets, int64_t total_points, const void *d_points,
                              int points_dtype, const double *d_planes, const double *area_extents, double voxel_size,
                              int num_slices, const double *slice_lo, const double *slice_hi, double density_lo,
                              double density_hi, double height_per_division, const double *density_table,
                              float *d_bev_input, const void *d_ws, size_t ws_bytes, void *stream) {
    if (n_frames < 1 || !d_point_offsets || !d_planes || !d_ws || !d_bev_input) return SHPL_ERR_ARG;
    if (points_dtype != SHPL_F64 || (total_points > 0 && !d_points)) return SHPL_ERR_ARG;
    if (total_points < 0 || total_points >= ((int64_t)1 << 31) || n_frames > BEV_MAX_FRAMES) return SHPL_ERR_BAD_SHAPE;
    BevGeom g;
    const int rc = bev_geom(area_extents, voxel_size, num_slices, slice_lo, slice_hi, density_lo, density_hi,
                            height_per_division, density_table, g);
    if (rc) return rc;
    size_t need;
    shpl_bev_workspace_bytes(total_points, num_slices, &need);
    if (need > ws_bytes) return SHPL_ERR_WORKSPACE;
    const size_t half = bev_half_bytes(total_points, num_slices);
    const uint64_t *srt = (const uint64_t *)((const char *)d_ws + half);
    const int32_t *nent = (const int32_t *)((const char *)d_ws + 2 * half);
    hipStream_t s = (hipStream_t)stream;
    const int64_t per_map = (int64_t)g.nx * g.nz;
    SHPL_HIP_CHECK(zero_fill(d_bev_input, sizeof(float) * (size_t)(per_map * (num_slices + 1) * n_frames), s));
    hipLaunchKernelGGL(k_bev_maps<double>, dim3(BEV_MAP_SPLIT, n_frames), dim3(SHPL_BLOCK), 0, s, g, d_point_offsets,
                       d_points, d_planes, srt, (int64_t)(num_slices + 1), nent, (double *)nullptr, (double *)nullptr,
                       d_bev_input);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}
