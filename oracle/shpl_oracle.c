/*
 * shpl_oracle.c -- CPU restatement of the reference SHPL path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker and the
 * bench's `cpu_baseline` ("port"); it is never linked into, loaded by or
 * called from the product library (sparse_pooling_amd/libshpl.so).
 *
 * What it restates (file:line relative to the reference checkout):
 *   index builder  avod/avod/utils/transform.py:3-40          (projectToImage, clip3DwithinImage)
 *                  avod/avod/utils/sparse_pool_utils.py:6-20   (gen_sparse_pooling_input_avod)
 *                  avod/avod/utils/sparse_pool_utils.py:22-58  (produce_sparse_pooling_input)
 *   pooling ops    avod/avod/utils/sparse_pool_utils.py:96-117 (_sparse_pool_op, _sparse_pool_trans_op)
 *                  whose arithmetic lives in TensorFlow 1.8.0 (avod/README.md:31,
 *                  MV3D_TF_release/README.md:11), a dependency absent from the
 *                  reference tree. Restated from TF 1.8's CPU kernels:
 *                    GatherNd                  copy params[idx[k]] -> P[k]; OOB is InvalidArgument
 *                    SparseTensorDenseMatMul   out = 0; for i in nnz order: out[m] += a_i * B[k]
 *                                              (adjoint_a swaps m/k; separate mul and add, the
 *                                              pip TF 1.8 binaries are built without FMA).
 *                                              TF 1.8's sparse_tensor_dense_matmul_op.cc has two
 *                                              CPU branches: below kNumVectorize = 32 right-hand
 *                                              columns a scalar loop `out(m, n) += a * b(k, n)`;
 *                                              from 32 on (config 2: Ci = 32; config 3: 256) the
 *                                              Eigen form `out.chip<0>(m) += b.chip(k) * a`, a
 *                                              coefficient-wise padd(out, pmul(b, a)) -- Eigen
 *                                              emits pmadd only inside its GEMM kernels, and the
 *                                              AVX-only build cannot contract. Both branches walk
 *                                              nnz in order and round the product before the add,
 *                                              so one restatement covers both.
 *                    SparseTranspose           permute index columns, then SparseReorder:
 *                                              lexicographic (col,row) order; equal keys keep
 *                                              input order here (TF's std::sort leaves them unspecified)
 *                    ScatterNd                 out = 0; for k in update order: out[idx[k]] += U[k]
 *                  and TF 1.8's registered gradients: GatherNd' = ScatterNd,
 *                  SparseTensorDenseMatMul'(B) = matmul(A, dY, adjoint_a=True),
 *                  ScatterNd'(updates) = GatherNd.
 *   post-fusion    avod/avod/core/models/rpn_model.py:338-355 (slim.conv2d 3x3 SAME, no bias,
 *   conv + BN      slim.batch_norm: center, no scale, eps 1e-3, decay 0.999, ReLU) and
 *                  avod/avod/core/models/retinanet_model.py:343-348 (conv2d + bias + ReLU).
 *                  TF's Conv2D / FusedBatchNorm CPU kernels (Eigen contractions) fix no
 *                  summation order, so the oracle sums in double: the tests compare
 *                  within a stated tolerance, cross-checked against torch's CPU conv2d.
 *
 * Parity status: the index builder is PINNED by tests/golden/index_*.npz,
 * produced by running the reference's own numpy builders in the survey
 * container (tests/golden/make_golden.py). The pooling ops are pinned to the
 * reference's call sites only: TensorFlow cannot be run here and the
 * reference holds no SHPL fixtures -- their numerics
 * are "parity unpinned" beyond TF's documented kernel order.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SHPLO_OK 0
#define SHPLO_ERR_INDEX 2
#define SHPLO_ERR_SHAPE 1

/* ---- a1: projectToImage (avod/avod/utils/transform.py:3-26) -----------------
 * numpy evaluates np.dot(P, [x;y;z;1]) through OpenBLAS. With two or more
 * columns that is dgemm, which accumulates the K=4 products as one
 * fused-multiply-add chain in k order (checked bit-exact against np.dot on 2M
 * random points, column counts 2 .. 120000). With ONE column (a frame of one
 * point, or one survivor of the clip) numpy calls dgemv, which sums
 * (a0*x0 + a2*x2) + (a1*x1 + a3*x3) with every product rounded (probed
 * against np.dot for 3x4 and 4x4 matrices; pinned by tests/golden/
 * index_single_*.npz, index_one_survivor.npz, kitti_single.npz). */
static double dot4(const double *p, const double *a, int gemv)
{
    if (gemv)
        return (p[0] * a[0] + p[2] * a[2]) + (p[1] * a[1] + p[3] * a[3]);
    double s = p[0] * a[0];
    for (int k = 1; k < 4; ++k)
        s = fma(p[k], a[k], s);
    return s;
}

static void project(const double *P, double x, double y, double z, int gemv, double *u, double *v)
{
    const double a[4] = {x, y, z, 1.0};
    double r[3];
    for (int i = 0; i < 3; ++i)
        r[i] = dot4(P + 4 * i, a, gemv);
    *u = r[0] / r[2];
    *v = r[1] / r[2];
}

/* a2: clip3DwithinImage (transform.py:28-40) -- strict upper bounds, image_size=[W,H]. */
static int inside_image(double u, double v, double w_img, double h_img)
{
    return (u < w_img - 1.0) && (u >= 0.0) && (v >= 0.0) && (v < h_img - 1.0);
}

/* a3: gen_sparse_pooling_input_avod (sparse_pool_utils.py:6-20).
 * pts: n x 3 (camera frame), vox: n x 2, P: 3 x 4 (row-major).
 * Outputs (capacity n): bv_index nv x 2, img_index 3 rows of stride `ld`
 * ([u; v; 0], rounded half-to-even like np.round). Returns nv.
 * Two projections as in the reference: the clip over all n columns (:13),
 * then projectToImage over the nv survivors (:16) -- dgemv when either
 * count is one. */
int64_t shplo_gen_index(int64_t n, const double *pts, const int64_t *vox, const double *P,
                        double im_w, double im_h, int64_t *bv_index, double *img_index, int64_t ld)
{
    int64_t nv = 0;
    for (int64_t i = 0; i < n; ++i) {
        double u, v;
        project(P, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], n == 1, &u, &v);
        if (!inside_image(u, v, im_w, im_h))
            continue;
        bv_index[2 * nv] = vox[2 * i];
        bv_index[2 * nv + 1] = vox[2 * i + 1];
        img_index[nv] = (double)(int64_t)nearbyint(u);
        img_index[ld + nv] = (double)(int64_t)nearbyint(v);
        img_index[2 * ld + nv] = (double)i;  /* the survivor's point, re-projected below */
        ++nv;
    }
    for (int64_t j = 0; j < nv; ++j) {
        const int64_t i = (int64_t)img_index[2 * ld + j];
        img_index[2 * ld + j] = 0.0;
        if (nv != 1 || n == 1)
            continue;  /* same order as the clip's projection */
        double u, v;
        project(P, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], 1, &u, &v);
        img_index[j] = (double)(int64_t)nearbyint(u);
        img_index[ld + j] = (double)(int64_t)nearbyint(v);
    }
    return nv;
}

/* a4: produce_sparse_pooling_input (sparse_pool_utils.py:22-58).
 * stride[0] (s_img) applies to the image, stride[1] (s_bv) to BEV.
 * img_index (3 rows, stride ld) is MUTATED in place exactly as the reference
 * mutates the caller's dict. bv_size is (H, W), im_size is (W, H).
 * Outputs: mij nk x 2 = [r, k], flip nk x 3 = [0, v, u], msize = [Hb'*Wb', nk].
 * Returns nk. */
int64_t shplo_produce(int64_t nv, const int64_t *bv_index, double *img_index, int64_t ld,
                      double im_w, double im_h, double bv_h, double bv_w,
                      double s_img, double s_bv, int64_t *mij, int64_t *flip, int64_t *msize)
{
    const double wq = floor(im_w / s_img), hq = floor(im_h / s_img);
    const double bhq = floor(bv_h / s_bv), bwq = floor(bv_w / s_bv);
    const int64_t n_cells = (int64_t)(bhq * bwq);
    int64_t nk = 0;
    for (int64_t j = 0; j < nv; ++j) {
        double u = floor(img_index[j] / s_img);
        double v = floor(img_index[ld + j] / s_img);
        if (u >= wq) u = wq - 1.0;
        if (v >= hq) v = hq - 1.0;
        img_index[j] = u;
        img_index[ld + j] = v;
        const double bx = floor((double)bv_index[2 * j] / s_bv);
        const double bz = floor((double)bv_index[2 * j + 1] / s_bv);
        const int64_t r = (int64_t)(bz * bwq + bx);
        if (!(r < n_cells))
            continue;
        mij[2 * nk] = r;
        mij[2 * nk + 1] = nk;
        flip[3 * nk] = (int64_t)floor(img_index[2 * ld + j]);
        flip[3 * nk + 1] = (int64_t)v;
        flip[3 * nk + 2] = (int64_t)u;
        ++nk;
    }
    msize[0] = (int64_t)(bhq * bwq);
    msize[1] = nk;
    return nk;
}

/* ---- TF op restatements ---------------------------------------------------- */

/* GatherNd index check for a [B,H,W,C] params tensor; returns flat pixel or -1. */
static int64_t pixel_of(const int64_t *idx, int64_t k, int64_t B, int64_t H, int64_t W)
{
    const int64_t b = idx[3 * k], y = idx[3 * k + 1], x = idx[3 * k + 2];
    if (b < 0 || b >= B || y < 0 || y >= H || x < 0 || x >= W)
        return -1;
    return (b * H + y) * W + x;
}

static int check_m(const int64_t *mij, int64_t nnz, int64_t R, int64_t ncols)
{
    for (int64_t i = 0; i < nnz; ++i)
        if (mij[2 * i] < 0 || mij[2 * i] >= R || mij[2 * i + 1] < 0 || mij[2 * i + 1] >= ncols)
            return SHPLO_ERR_INDEX;
    return SHPLO_OK;
}

/* a8: _sparse_pool_op = reshape(sparse_tensor_dense_matmul(M, gather_nd(img, idx))).
 * img [B,H,W,C] f32; idx n_idx x 3; M (mij nnz x 2, mval nnz, shape R x ncols).
 * out R x C. */
int shplo_pool(const float *img, int64_t B, int64_t H, int64_t W, int64_t C,
               const int64_t *idx, int64_t n_idx, const int64_t *mij, const float *mval,
               int64_t nnz, int64_t R, int64_t ncols, float *out)
{
    if (ncols != n_idx)
        return SHPLO_ERR_SHAPE;
    for (int64_t k = 0; k < n_idx; ++k)
        if (pixel_of(idx, k, B, H, W) < 0)
            return SHPLO_ERR_INDEX;
    if (check_m(mij, nnz, R, ncols))
        return SHPLO_ERR_INDEX;
    memset(out, 0, sizeof(float) * (size_t)(R * C));
    for (int64_t i = 0; i < nnz; ++i) {
        const int64_t m = mij[2 * i], k = mij[2 * i + 1];
        const float a = mval[i];
        const float *b = img + pixel_of(idx, k, B, H, W) * C;
        float *o = out + m * C;
        for (int64_t c = 0; c < C; ++c) {
            const float prod = a * b[c];
            o[c] = o[c] + prod;
        }
    }
    return SHPLO_OK;
}

/* SparseReorder order of M^T: entries sorted by (col, row), ties by input order. */
static const int64_t *g_mij;
static int cmp_col_row(const void *pa, const void *pb)
{
    const int64_t a = *(const int64_t *)pa, b = *(const int64_t *)pb;
    const int64_t ca = g_mij[2 * a + 1], cb = g_mij[2 * b + 1];
    if (ca != cb) return ca < cb ? -1 : 1;
    const int64_t ra = g_mij[2 * a], rb = g_mij[2 * b];
    if (ra != rb) return ra < rb ? -1 : 1;
    return a < b ? -1 : (a > b);
}

static int64_t *transpose_order(const int64_t *mij, int64_t nnz)
{
    int64_t *ord = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nnz > 0 ? nnz : 1));
    for (int64_t i = 0; i < nnz; ++i)
        ord[i] = i;
    g_mij = mij;
    qsort(ord, (size_t)nnz, sizeof(int64_t), cmp_col_row);
    return ord;
}

/* a9: _sparse_pool_trans_op = scatter_nd(idx, sparse_tensor_dense_matmul(
 *     sparse_transpose(M), reshape(bev, [-1, C])), [B,H,W,C]).
 * bev R x C; out B*H*W x C. */
int shplo_pool_trans(const float *bev, int64_t R, int64_t C, const int64_t *mij,
                     const float *mval, int64_t nnz, int64_t ncols, const int64_t *idx,
                     int64_t n_idx, int64_t B, int64_t H, int64_t W, float *out)
{
    if (ncols != n_idx)
        return SHPLO_ERR_SHAPE;
    if (check_m(mij, nnz, R, ncols))
        return SHPLO_ERR_INDEX;
    for (int64_t k = 0; k < n_idx; ++k)
        if (pixel_of(idx, k, B, H, W) < 0)
            return SHPLO_ERR_INDEX;
    float *q = (float *)calloc((size_t)(ncols * C > 0 ? ncols * C : 1), sizeof(float));
    int64_t *ord = transpose_order(mij, nnz);
    for (int64_t t = 0; t < nnz; ++t) {
        const int64_t i = ord[t];
        const int64_t m = mij[2 * i + 1], k = mij[2 * i]; /* transposed: row=col(M), col=row(M) */
        const float a = mval[i];
        for (int64_t c = 0; c < C; ++c) {
            const float prod = a * bev[k * C + c];
            q[m * C + c] = q[m * C + c] + prod;
        }
    }
    memset(out, 0, sizeof(float) * (size_t)(B * H * W * C));
    for (int64_t k = 0; k < n_idx; ++k) {
        float *o = out + pixel_of(idx, k, B, H, W) * C;
        for (int64_t c = 0; c < C; ++c)
            o[c] = o[c] + q[k * C + c];
    }
    free(ord);
    free(q);
    return SHPLO_OK;
}

/* a11 (part): gradient of a8 w.r.t. img.
 * grad_P = sparse_tensor_dense_matmul(M, dY, adjoint_a=True) (nnz order);
 * d_img = scatter_nd(idx, grad_P, img.shape).  dY is R x C. */
int shplo_pool_grad_img(const float *dY, int64_t R, int64_t C, const int64_t *mij,
                        const float *mval, int64_t nnz, int64_t ncols, const int64_t *idx,
                        int64_t n_idx, int64_t B, int64_t H, int64_t W, float *d_img)
{
    if (ncols != n_idx)
        return SHPLO_ERR_SHAPE;
    if (check_m(mij, nnz, R, ncols))
        return SHPLO_ERR_INDEX;
    for (int64_t k = 0; k < n_idx; ++k)
        if (pixel_of(idx, k, B, H, W) < 0)
            return SHPLO_ERR_INDEX;
    float *g = (float *)calloc((size_t)(ncols * C > 0 ? ncols * C : 1), sizeof(float));
    for (int64_t i = 0; i < nnz; ++i) {
        const int64_t m = mij[2 * i + 1], k = mij[2 * i];
        const float a = mval[i];
        for (int64_t c = 0; c < C; ++c) {
            const float prod = a * dY[k * C + c];
            g[m * C + c] = g[m * C + c] + prod;
        }
    }
    memset(d_img, 0, sizeof(float) * (size_t)(B * H * W * C));
    for (int64_t k = 0; k < n_idx; ++k) {
        float *o = d_img + pixel_of(idx, k, B, H, W) * C;
        for (int64_t c = 0; c < C; ++c)
            o[c] = o[c] + g[k * C + c];
    }
    free(g);
    return SHPLO_OK;
}

/* a11 (part): gradient of a9 w.r.t. bev.
 * dQ = gather_nd(dZ, idx); d_bev = sparse_tensor_dense_matmul(M^T, dQ, adjoint_a=True)
 * iterating M^T's reordered (col,row) entries. dZ is [B,H,W,C]; d_bev R x C. */
int shplo_pool_trans_grad_bev(const float *dZ, int64_t B, int64_t H, int64_t W, int64_t C,
                              const int64_t *idx, int64_t n_idx, const int64_t *mij,
                              const float *mval, int64_t nnz, int64_t R, int64_t ncols,
                              float *d_bev)
{
    if (ncols != n_idx)
        return SHPLO_ERR_SHAPE;
    for (int64_t k = 0; k < n_idx; ++k)
        if (pixel_of(idx, k, B, H, W) < 0)
            return SHPLO_ERR_INDEX;
    if (check_m(mij, nnz, R, ncols))
        return SHPLO_ERR_INDEX;
    int64_t *ord = transpose_order(mij, nnz);
    memset(d_bev, 0, sizeof(float) * (size_t)(R * C));
    for (int64_t t = 0; t < nnz; ++t) {
        const int64_t i = ord[t];
        const int64_t r = mij[2 * i], k = mij[2 * i + 1];
        const float a = mval[i];
        const float *b = dZ + pixel_of(idx, k, B, H, W) * C;
        for (int64_t c = 0; c < C; ++c) {
            const float prod = a * b[c];
            d_bev[r * C + c] = d_bev[r * C + c] + prod;
        }
    }
    free(ord);
    return SHPLO_OK;
}

/* ---- a5/a6: BevSlices.generate_bev(output_indices=True) ------------------
 * avod/avod/core/bev_generators/bev_slices.py:58-154 and
 * avod/wavedata/wavedata/tools/core/voxel_grid_2d.py:64-152, restated per
 * slice: slice filter (kitti_utils.py:79-107 -> obj_utils.py:444-491),
 * floor(p / vs), stable lexsort by (x, z, y), first point of every (x, z)
 * cell, cells in (x, z) order. The plane test np.dot(plane', [p;1]) goes
 * through OpenBLAS dgemv whose accumulation order is not reproduced here
 * (an FMA chain is used): results can differ only for points within one ulp
 * of a slice plane. Slices with <= 1 point are voxelized too (the reference
 * reuses the previous slice's grid there, bev_slices.py:79-93, a bug). */
typedef struct { int32_t x, y, z; int64_t i; } shplo_vox;

static int cmp_vox(const void *pa, const void *pb)
{
    const shplo_vox *a = (const shplo_vox *)pa, *b = (const shplo_vox *)pb;
    if (a->x != b->x) return a->x < b->x ? -1 : 1;
    if (a->z != b->z) return a->z < b->z ? -1 : 1;
    if (a->y != b->y) return a->y < b->y ? -1 : 1;
    return a->i < b->i ? -1 : (a->i > b->i);
}

static int plane_below(const double *pl, double off, double x, double y, double z)
{
    double s = pl[0] * x;
    s = fma(pl[1], y, s);
    s = fma(pl[2], z, s);
    s = fma(pl[3] - off, 1.0, s);
    return s < 0.0;
}

/* pts n x 3; ext [3][2]; outputs: vox (cap x 2: x, nz - z), upts (cap x 3),
 * hmaps [num_slices][nz][nx] (zero-filled here), dmap [nz][nx]; returns the
 * number of voxel rows (all slices) or -1 if cap is too small. */
int64_t shplo_bev_slices(int64_t n, const double *pts, const double *plane, const double *ext, double vs,
                         int num_slices, const double *lo, const double *hi, double dlo, double dhi,
                         double hpd, const double *dens_table, int64_t cap, int64_t *vox, double *upts,
                         double *hmaps, double *dmap)
{
    const int min_x = (int)floor(ext[0] / vs), min_z = (int)floor(ext[4] / vs);
    const int nx = (int)(ceil(ext[1] / vs - 1) - min_x + 1), nz = (int)(ceil(ext[5] / vs - 1) - min_z + 1);
    const double norm = sqrt(plane[0] * plane[0] + plane[1] * plane[1] + plane[2] * plane[2]);
    memset(hmaps, 0, sizeof(double) * (size_t)num_slices * nx * nz);
    memset(dmap, 0, sizeof(double) * (size_t)nx * nz);
    shplo_vox *buf = (shplo_vox *)malloc(sizeof(shplo_vox) * (size_t)(n > 0 ? n : 1));
    int64_t out = 0;
    for (int s = 0; s <= num_slices; ++s) {
        const double l = s < num_slices ? lo[s] : dlo, h = s < num_slices ? hi[s] : dhi;
        int64_t m = 0;
        for (int64_t i = 0; i < n; ++i) {
            const double x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
            if (!(x > ext[0] && x < ext[1] && y > ext[2] && y < ext[3] && z > ext[4] && z < ext[5])) continue;
            if (plane_below(plane, h, x, y, z) == plane_below(plane, l, x, y, z)) continue;
            buf[m].x = (int32_t)floor(x / vs);
            buf[m].y = (int32_t)floor(y / vs);
            buf[m].z = (int32_t)floor(z / vs);
            buf[m].i = i;
            ++m;
        }
        qsort(buf, (size_t)m, sizeof(shplo_vox), cmp_vox);
        for (int64_t j = 0; j < m;) {
            int64_t k = j + 1;
            while (k < m && buf[k].x == buf[j].x && buf[k].z == buf[j].z) ++k;
            const int xi = buf[j].x - min_x, zi = buf[j].z - min_z;
            const int64_t pix = (int64_t)(nz - 1 - zi) * nx + xi;
            const double *p = pts + 3 * buf[j].i;
            if (s < num_slices) {
                if (out >= cap) { free(buf); return -1; }
                vox[2 * out] = xi;
                vox[2 * out + 1] = nz - zi;
                upts[3 * out] = p[0];
                upts[3 * out + 1] = p[1];
                upts[3 * out + 2] = p[2];
                ++out;
                const double dist = (plane[0] * p[0] + plane[1] * p[1] + plane[2] * p[2] + plane[3]) / norm;
                hmaps[(int64_t)s * nx * nz + pix] = (dist - l) / hpd;
            } else {
                const int64_t c = k - j;
                dmap[pix] = c < 16 ? dens_table[c] : 1.0;
            }
            j = k;
        }
    }
    free(buf);
    return out;
}

/* ---- a7: MV3D point_cloud_2_top_sparse (construct_voxel.py:37-162) --------
 * pts n x stride camera frame (x, y, z, ...), img2 [2][n] rounded projections
 * of every point (minibatch_mv3d_img.py:88-91); ranges fwd/side/height (lo, hi).
 * The per-point loop of the reference (:134-140) is kept as is: a voxel
 * accepts points in point order until it holds `cap`. Outputs img_index
 * [3][ld] f64, bv_index n' x 2 (fwd, side), mval n' (1 / accepted count).
 * Returns n'. */
static int64_t *g_vkey;
static int cmp_key_idx(const void *pa, const void *pb)
{
    const int64_t a = *(const int64_t *)pa, b = *(const int64_t *)pb;
    if (g_vkey[a] != g_vkey[b]) return g_vkey[a] < g_vkey[b] ? -1 : 1;
    return a < b ? -1 : (a > b);
}

int64_t shplo_mv3d_voxels(int64_t n, const double *pts, int64_t stride, const int64_t *img2, const double *ranges,
                          double res, double zres, int cap, double *img_index, int64_t ld, int64_t *bv_index,
                          double *mval, int32_t *number_buffer, int64_t *n_vox)
{
    const int n_fwd = (int)((ranges[1] - ranges[0]) / res) + 1;
    const int n_h = (int)((ranges[5] - ranges[4]) / zres) + 1;
    int64_t *key = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t *ord = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int32_t *vid = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *fi = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *si = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double *q = pts + i * stride;
        const double fwd = q[2], side = q[0], h = q[1];
        key[i] = -1;
        if (!(fwd > ranges[0] && fwd < ranges[1] && side > ranges[2] && side < ranges[3] && h > ranges[4] &&
              h < ranges[5]))
            continue;
        si[i] = (int32_t)((side - ranges[2]) / res);
        fi[i] = (int32_t)((fwd - ranges[0]) / res);
        const int32_t hi = (int32_t)((h - ranges[4]) / zres);
        key[i] = ((int64_t)si[i] * n_fwd + fi[i]) * n_h + hi;
        ord[m++] = i;
    }
    /* np.unique(xyz_img, axis=0, return_inverse=True): voxel ids in lexicographic order */
    g_vkey = key;
    qsort(ord, (size_t)m, sizeof(int64_t), cmp_key_idx);
    int32_t nv = 0;
    for (int64_t j = 0; j < m; ++j) {
        if (j > 0 && key[ord[j]] != key[ord[j - 1]]) ++nv;
        vid[ord[j]] = nv;
    }
    const int32_t n_voxels = m > 0 ? nv + 1 : 0;
    int32_t *count = (int32_t *)calloc((size_t)(n_voxels > 0 ? n_voxels : 1), sizeof(int32_t));
    unsigned char *keep = (unsigned char *)calloc((size_t)(n > 0 ? n : 1), 1);
    for (int64_t i = 0; i < n; ++i) { /* the reference's per-point loop, in point order */
        if (key[i] < 0) continue;
        if (count[vid[i]] < cap) {
            ++count[vid[i]];
            keep[i] = 1;
        }
    }
    int64_t out = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (!keep[i]) continue;
        img_index[out] = (double)img2[i];
        img_index[ld + out] = (double)img2[n + i];
        img_index[2 * ld + out] = 0.0;
        bv_index[2 * out] = fi[i];
        bv_index[2 * out + 1] = si[i];
        mval[out] = 1.0 / (double)count[vid[i]];
        ++out;
    }
    if (number_buffer)
        for (int32_t v = 0; v < n_voxels; ++v) number_buffer[v] = count[v];
    if (n_vox) *n_vox = n_voxels;
    free(key); free(ord); free(vid); free(fi); free(si); free(count); free(keep);
    return out;
}

/* ---- §8f item 3: KITTI velodyne -> camera-frame point cloud ------------------
 * obj_utils.get_lidar_point_cloud (avod/wavedata/wavedata/tools/obj_detection/obj_utils.py:220-268):
 *   lidar_to_cam_frame (calib_utils.py:371-410): p_cam = (R0_rect4 . Tr_velo_to_cam4) . [x;y;z;1]
 *     -- `rect` is that 4x4 product's rows 0-2, computed by numpy on the host; the
 *     per-point np.dot is OpenBLAS dgemm, i.e. the same FMA chain as project()
 *     (checked bit-exact against numpy for N = 2 .. 120000), dgemv's order for a
 *     one-point scan (dot4);
 *   keep z > 0 (:250), project with P2 (calib_utils.project_to_image :281-298;
 *   dgemv's order when exactly one point has z > 0),
 *   keep 0 < u < W and 0 < v < H (strict, :256-259), im_size = [W, H].
 * has_filter = 0 mirrors im_size=None (every point, :244-246).
 * min_intensity (NaN = none): the reference compares the intensities of ALL
 * points against a mask of the z-filtered ones (:265-267), which raises as
 * soon as one point has z <= 0; restated here with the evident intent
 * (intensity of the same point), documented in DESIGN.md.
 * flip != 0 applies kitti_aug.flip_point_cloud (x -> -x, kitti_aug.py:24-29)
 * after the filter, as kitti_dataset.py:305-306 does.
 * xyzi: n x 4 f32 (read_lidar, calib_utils.py:328-368). out: n x 3. Returns kept. */
int64_t shplo_velo_to_cam(int64_t n, const float *xyzi, const double *rect, const double *P, int has_filter,
                          double im_w, double im_h, double min_intensity, int flip, double *out)
{
    int64_t k = 0, front = 0;
    for (int64_t pass = has_filter ? 0 : 1; pass < 2; ++pass)
    for (int64_t i = 0; i < n; ++i) {
        const double a[4] = {(double)xyzi[4 * i], (double)xyzi[4 * i + 1], (double)xyzi[4 * i + 2], 1.0};
        double c[3];
        for (int r = 0; r < 3; ++r)
            c[r] = dot4(rect + 4 * r, a, n == 1);
        if (pass == 0) {  /* the columns of project_to_image: points with z > 0 */
            front += c[2] > 0.0;
            continue;
        }
        if (has_filter) {
            if (!(c[2] > 0.0))
                continue;
            double u, v;
            project(P, c[0], c[1], c[2], front == 1, &u, &v);
            if (!(u > 0.0 && u < im_w && v > 0.0 && v < im_h))
                continue;
            if (!isnan(min_intensity) && !((double)xyzi[4 * i + 3] > min_intensity))
                continue;
        }
        out[3 * k] = flip ? -c[0] : c[0];
        out[3 * k + 1] = c[1];
        out[3 * k + 2] = c[2];
        ++k;
    }
    return k;
}

/* ---- f4: post-fusion 3x3 convolution + epilogue ----------------------------
 * out[f,y,x,co] = act((sum in[f,y+ky-1,x+kx-1,ci] * w[ky][kx][ci][co]
 *                      - center[co]) * scale[co] + shift[co]),
 * SAME zero padding, stride 1, sums in double, one rounding to f32 at the
 * end (NULL center / scale / shift = 0 / 1 / 0). `raw` (optional) receives
 * the pre-epilogue sums in double (for the training BatchNorm statistics). */
void shplo_conv3x3(const float *in, int64_t B, int64_t H, int64_t W, int64_t Cin, const float *w,
                   int64_t Cout, const float *center, const float *scale, const float *shift, int relu,
                   float *out, double *raw)
{
    double *acc = (double *)malloc(sizeof(double) * (size_t)(Cout > 0 ? Cout : 1));
    for (int64_t f = 0; f < B; ++f)
        for (int64_t y = 0; y < H; ++y)
            for (int64_t x = 0; x < W; ++x) {
                for (int64_t co = 0; co < Cout; ++co) acc[co] = 0.0;
                for (int64_t ky = 0; ky < 3; ++ky) {
                    const int64_t yy = y + ky - 1;
                    if (yy < 0 || yy >= H) continue;
                    for (int64_t kx = 0; kx < 3; ++kx) {
                        const int64_t xx = x + kx - 1;
                        if (xx < 0 || xx >= W) continue;
                        const float *a = in + ((f * H + yy) * W + xx) * Cin;
                        const float *wt = w + (ky * 3 + kx) * Cin * Cout;
                        for (int64_t ci = 0; ci < Cin; ++ci) {
                            const double av = a[ci];
                            const float *wr = wt + ci * Cout;
                            for (int64_t co = 0; co < Cout; ++co) acc[co] += av * (double)wr[co];
                        }
                    }
                }
                const int64_t row = (f * H + y) * W + x;
                for (int64_t co = 0; co < Cout; ++co) {
                    double v = acc[co];
                    if (raw) raw[row * Cout + co] = v;
                    if (center) v -= center[co];
                    if (scale) v *= scale[co];
                    if (shift) v += shift[co];
                    if (relu && v < 0.0) v = 0.0;
                    out[row * Cout + co] = (float)v;
                }
            }
    free(acc);
}

/* BatchNorm in training mode (TF FusedBatchNorm, is_training=True) over the
 * double pre-activation `raw` [rows][C]: batch mean and biased variance
 * normalise, y = act((x - mean) * gamma / sqrt(var + eps) + beta); the
 * moving averages take the Bessel-corrected variance:
 * m -= (m - batch) * (1 - decay). */
void shplo_bn_train(const double *raw, int64_t rows, int64_t C, double eps, const float *gamma,
                    const float *beta, int relu, float *out, float *moving_mean, float *moving_var,
                    double decay, double *batch_mean, double *batch_var)
{
    for (int64_t c = 0; c < C; ++c) {
        double s = 0.0, s2 = 0.0;
        for (int64_t r = 0; r < rows; ++r) s += raw[r * C + c];
        const double mean = s / (double)rows;
        for (int64_t r = 0; r < rows; ++r) {
            const double d = raw[r * C + c] - mean;
            s2 += d * d;
        }
        const double var = s2 / (double)rows;
        const double g = gamma ? gamma[c] : 1.0;
        const double k = g / sqrt(var + eps);
        for (int64_t r = 0; r < rows; ++r) {
            double v = (raw[r * C + c] - mean) * k;
            if (beta) v += beta[c];
            if (relu && v < 0.0) v = 0.0;
            out[r * C + c] = (float)v;
        }
        const double vu = rows > 1 ? var * (double)rows / (double)(rows - 1) : var;
        if (moving_mean) moving_mean[c] = (float)(moving_mean[c] - (moving_mean[c] - mean) * (1.0 - decay));
        if (moving_var) moving_var[c] = (float)(moving_var[c] - (moving_var[c] - vu) * (1.0 - decay));
        if (batch_mean) batch_mean[c] = mean;
        if (batch_var) batch_var[c] = vu;
    }
}

/* Weight gradient of the 3x3 SAME conv: dw[ky][kx][ci][co] =
 * sum over (f, y, x) of in[f, y+ky-1, x+kx-1, ci] * g[f, y, x, co]
 * (zero outside the map), summed in double. */
void shplo_conv3x3_wgrad(const float *in, int64_t B, int64_t H, int64_t W, int64_t Cin, const float *g,
                         int64_t Cout, double *dw)
{
    memset(dw, 0, sizeof(double) * (size_t)(9 * Cin * Cout));
    for (int64_t f = 0; f < B; ++f)
        for (int64_t y = 0; y < H; ++y)
            for (int64_t x = 0; x < W; ++x) {
                const float *gr = g + ((f * H + y) * W + x) * Cout;
                for (int64_t ky = 0; ky < 3; ++ky) {
                    const int64_t yy = y + ky - 1;
                    if (yy < 0 || yy >= H) continue;
                    for (int64_t kx = 0; kx < 3; ++kx) {
                        const int64_t xx = x + kx - 1;
                        if (xx < 0 || xx >= W) continue;
                        const float *a = in + ((f * H + yy) * W + xx) * Cin;
                        double *d = dw + (ky * 3 + kx) * Cin * Cout;
                        for (int64_t ci = 0; ci < Cin; ++ci) {
                            const double av = a[ci];
                            for (int64_t co = 0; co < Cout; ++co) d[ci * Cout + co] += av * (double)gr[co];
                        }
                    }
                }
            }
}

/* BatchNorm + ReLU backward in double. raw: the conv output (pre-BN), g: the
 * gradient of the layer output. training: batch moments (biased variance)
 * normalise, as in the forward; otherwise mean / var are the moving
 * statistics (constants). Writes d_raw, dbeta = sum g_bn, dgamma =
 * sum g_bn * xhat, with g_bn = g * [y > 0] (ReLU) and
 *   training:  d_raw = gamma r / N (N g_bn - dbeta - xhat dgamma)
 *   inference: d_raw = gamma r g_bn,     r = 1 / sqrt(var + eps). */
void shplo_bn_bwd(const double *raw, const float *g, int64_t rows, int64_t C, int training, const double *mean_in,
                  const double *var_in, double eps, const float *gamma, const float *beta, int relu, double *d_raw,
                  double *dbeta, double *dgamma)
{
    for (int64_t c = 0; c < C; ++c) {
        double mean, var;
        if (training) {
            double s = 0.0, s2 = 0.0;
            for (int64_t r = 0; r < rows; ++r) s += raw[r * C + c];
            mean = s / (double)rows;
            for (int64_t r = 0; r < rows; ++r) {
                const double d = raw[r * C + c] - mean;
                s2 += d * d;
            }
            var = s2 / (double)rows;
        } else {
            mean = mean_in[c];
            var = var_in[c];
        }
        const double rr = 1.0 / sqrt(var + eps);
        const double gm = gamma ? gamma[c] : 1.0, bt = beta ? beta[c] : 0.0;
        double db = 0.0, dg = 0.0;
        for (int64_t r = 0; r < rows; ++r) {
            const double xh = (raw[r * C + c] - mean) * rr;
            const double y = gm * xh + bt;
            const double gb = (relu && !(y > 0.0)) ? 0.0 : g[r * C + c];
            db += gb;
            dg += gb * xh;
        }
        dbeta[c] = db;
        dgamma[c] = dg;
        for (int64_t r = 0; r < rows; ++r) {
            const double xh = (raw[r * C + c] - mean) * rr;
            const double y = gm * xh + bt;
            const double gb = (relu && !(y > 0.0)) ? 0.0 : g[r * C + c];
            d_raw[r * C + c] = training ? gm * rr / (double)rows * ((double)rows * gb - db - xh * dg) : gm * rr * gb;
        }
    }
}
