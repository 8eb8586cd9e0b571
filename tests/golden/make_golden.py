"""Generate the committed golden fixtures by RUNNING the reference's own numpy
index builders in this container.

This script is the only place the reference is executed. It needs
``/root/reference`` (absent on the GPU box) and trivial stubs for
``tensorflow`` / ``cv2`` / ``easydict`` (TensorFlow 1.8 is not installable
here; the builders below use only numpy -- the stubs merely satisfy
module-level imports). Fixtures are data only: inputs and the reference's
outputs, written as ``.npz`` next to this file.

Reference functions executed (file:line, relative to /root/reference):

* ``gen_sparse_pooling_input_avod``   avod/avod/utils/sparse_pool_utils.py:6-20
* ``produce_sparse_pooling_input``    avod/avod/utils/sparse_pool_utils.py:22-58
* MV3D ``produce_sparse_pooling_input`` MV3D_TF_release/lib/utils/sparse_pool_utils.py:22-55
* ``BevSlices.generate_bev(output_indices=True)``
                                      avod/avod/core/bev_generators/bev_slices.py:33-156
* MV3D ``point_cloud_2_top_sparse``   MV3D_TF_release/lib/utils/construct_voxel.py:37-162
* ``obj_utils.get_lidar_point_cloud``  avod/wavedata/wavedata/tools/obj_detection/obj_utils.py:220-268
  (``calib_utils.read_calibration`` / ``read_lidar`` / ``lidar_to_cam_frame``,
  calib_utils.py:55-112, 328-410), ``obj_utils.get_road_plane`` :271-303 and
  ``kitti_aug.flip_point_cloud`` / ``flip_stereo_calib_p2`` / ``flip_ground_plane``
  (avod/avod/datasets/kitti/kitti_aug.py:24-29, 88-121) on synthetic KITTI files

Run:  python tests/golden/make_golden.py [case ...]   (e.g. ``kitti``; no argument: all)
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from sparse_pooling_amd import synth  # noqa: E402


def _install_stubs():
    tf = types.ModuleType("tensorflow")
    tf.contrib = types.SimpleNamespace(slim=types.SimpleNamespace())
    sys.modules.setdefault("tensorflow", tf)
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    ed = types.ModuleType("easydict")

    class EasyDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    ed.EasyDict = EasyDict
    sys.modules.setdefault("easydict", ed)
    for p in (os.path.join(REF, "avod"), os.path.join(REF, "avod", "wavedata"),
              os.path.join(REF, "MV3D_TF_release", "lib")):
        if p not in sys.path:
            sys.path.append(p)


def _ref_avod():
    import importlib
    return importlib.import_module("avod.utils.sparse_pool_utils")


def _index_case(name, frame, im_size, bv_size, stride, M_val=None, mv3d=False):
    spu = _ref_avod()
    calib = synth.StereoCalib(frame.P)
    g = spu.gen_sparse_pooling_input_avod(frame.points.copy(), frame.voxel_indices.copy(),
                                          calib, list(im_size), tuple(bv_size))
    gen = {k: np.array(v, copy=True) for k, v in g.items()}
    if mv3d:
        import importlib
        mv = importlib.import_module("utils.sparse_pool_utils")
        out = mv.produce_sparse_pooling_input(g, M_val=M_val, stride=list(stride))
    else:
        out = spu.produce_sparse_pooling_input(g, M_val=M_val, stride=list(stride))
    rec = dict(points=frame.points, voxel_indices=frame.voxel_indices, P=frame.P,
               im_size=np.array(im_size), bv_size=np.array(bv_size),
               stride=np.array(stride, dtype=np.float64),
               gen_bv_index=gen["bv_index"], gen_img_index=gen["img_index"],
               gen_bv_size=gen["bv_size"], gen_img_size=gen["img_size"],
               mutated_img_index=np.asarray(g["img_index"]),
               Mij_pool=np.asarray(out["Mij_pool"]), M_val=np.asarray(out["M_val"]),
               M_size=np.asarray(out["M_size"]),
               img_index_flip_pool=np.asarray(out["img_index_flip_pool"]),
               bev_index_flip_pool=np.asarray(out["bev_index_flip_pool"]))
    if M_val is not None:
        rec["M_val_in"] = np.asarray(M_val)
    np.savez_compressed(os.path.join(HERE, f"index_{name}.npz"), **rec)
    print(f"index_{name}: N={frame.points.shape[0]} nnz={rec['Mij_pool'].shape[0]} M_size={rec['M_size']}")


def _kat_frame():
    """Known-answer points: with P = [[1,0,0,0],[0,1,0,0],[0,0,0,1]] the
    projection is u=x, v=y exactly, so round-half-even ties, the strict
    ``< W-1`` / ``>= 0`` clip bounds and the ``>= W'`` clamp are hit exactly."""
    P = np.array([[1.0, 0, 0, 0], [0, 1.0, 0, 0], [0, 0, 0, 1.0]])
    W, H = 1201, 363
    xs = [0.0, -0.0, -1e-300, 0.5, 1.5, 2.5, 3.49999999, W - 1.0, W - 1.0 - 1e-9,
          W - 1.5, W - 1.49, 1196.0, 1199.5, 598.5, 7.5, -0.5, 10.0, 11.0]
    ys = [0.0, 0.5, 1.5, H - 1.0, H - 1 - 1e-9, H - 1.5, -1e-12, 2.5, 100.5, 361.6]
    pts = []
    for i, x in enumerate(xs):
        for j, y in enumerate(ys):
            pts.append((x, y, 1.0 + 0.25 * ((i + j) % 5)))
    pts = np.array(pts, dtype=np.float64)
    n = pts.shape[0]
    hb, wb = 707, 803
    rng = np.random.default_rng(7)
    vox = np.stack([rng.integers(0, wb, n), rng.integers(0, hb + 2, n)], axis=1).astype(np.int64)
    vox[:6] = [[0, 0], [wb - 1, hb - 1], [wb - 1, hb], [0, hb], [wb, hb - 1], [wb + 3, hb - 1]]
    fr = synth.Frame(pts, vox, P, synth.FrameSpec(n, (W, H), (hb, wb)))
    return fr, (W, H), (hb, wb)


def _bev_slices_case():
    """BevSlices.generate_bev(output_indices=True): voxel indices + one point per
    BEV cell per slice (the input of the index builder)."""
    from avod.core.bev_generators.bev_slices import BevSlices
    from wavedata.tools.obj_detection import obj_utils

    class _Utils:
        # KittiUtils.create_slice_filter (avod/avod/datasets/kitti/kitti_utils.py:79-107)
        # = xor of two obj_utils.get_point_filter masks.
        @staticmethod
        def create_slice_filter(pc, ext, gp, lo, hi):
            a = obj_utils.get_point_filter(pc, ext, gp, hi)
            b = obj_utils.get_point_filter(pc, ext, gp, lo)
            return np.logical_xor(a, b)

    cfg = types.SimpleNamespace(height_lo=-0.2, height_hi=2.3, num_slices=5)
    bev = BevSlices(cfg, _Utils())
    rng = np.random.default_rng(11)
    n = 20000
    pts = np.stack([rng.uniform(-39.9, 39.9, n), rng.uniform(-0.5, 2.2, n),
                    rng.uniform(0.05, 69.9, n)], axis=0)
    area = np.array([[-40, 40], [-5, 3], [0, 70]], dtype=np.float64)
    gp = np.array([0.0, -1.0, 0.0, 1.65])
    maps, vox, upts = bev.generate_bev("lidar", pts, gp, area, 0.1, output_indices=True)
    np.savez_compressed(os.path.join(HERE, "bev_slices.npz"), point_cloud=pts, ground_plane=gp,
                        area_extents=area, voxel_size=np.array(0.1), height_lo=np.array(-0.2),
                        height_hi=np.array(2.3), num_slices=np.array(5),
                        voxel_indices=vox, pts_in_voxel=upts,
                        height_maps=np.stack(maps["height_maps"]), density_map=maps["density_map"])
    print(f"bev_slices: N={n} voxel_indices={vox.shape} maps={np.stack(maps['height_maps']).shape}")


def _mv3d_voxel_case(dense=False):
    """MV3D point_cloud_2_top_sparse: img_index, bv_index and M_val = 1/count.
    dense: clustered points so that many voxels exceed VOXEL_POINT_COUNT (45)."""
    import importlib
    cv = importlib.import_module("utils.construct_voxel")
    rng = np.random.default_rng(13 + dense)
    n = 6000
    # camera frame: x side, y height (down), z forward; some points outside the ranges
    pts = np.stack([rng.uniform(-21, 21, n), rng.uniform(-1.2, 3.2, n), rng.uniform(-0.5, 49, n),
                    rng.uniform(0, 1, n)], axis=1)
    if dense:
        centers = np.stack([rng.uniform(-15, 15, 40), rng.uniform(0, 2, 40), rng.uniform(5, 40, 40)], 1)
        pick = rng.integers(0, 40, n)
        pts[:, :3] = centers[pick] + rng.normal(0, 0.08, (n, 3))
    P = synth.KITTI_P2
    uvw = P @ np.vstack((pts[:, :3].T, np.ones(n)))
    img_index2 = np.round(uvw[:2] / uvw[2]).astype(int)
    calib = np.zeros((4, 12))
    calib[0] = P.reshape(-1)
    vd, full, img_index, bv_index, M_val = cv.point_cloud_2_top_sparse(
        pts.copy(), points_in_cam=True, calib=calib, img_index2=img_index2.copy())
    np.savez_compressed(os.path.join(HERE, "mv3d_voxel_dense.npz" if dense else "mv3d_voxel.npz"),
                        points=pts, img_index2=img_index2,
                        voxel_full_size=np.asarray(full), img_index=img_index, bv_index=bv_index,
                        M_val=M_val, coordinate_buffer=vd["coordinate_buffer"],
                        number_buffer=vd["number_buffer"])
    print(f"mv3d_voxel(dense={dense}): N={n} kept={bv_index.shape[0]} voxels={vd['number_buffer'].shape[0]} "
          f"capped={(vd['number_buffer'] >= 45).sum()}")


KITTI_CALIB = synth.KITTI_CALIB
synthetic_scan = synth.synthetic_scan


# ---- single-column products: np.dot(A, x) with x of one column goes through
# OpenBLAS dgemv, whose sum order ((a0*x0 + a2*x2) + (a1*x1 + a3*x3)) differs
# from dgemm's FMA chain. The searches below look for points where the two
# orders give different integer outputs (rounded pixel, clip decision), so the
# goldens discriminate; the reference then runs on them as on any frame.
def _fma(a, b, c):
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _dot_chain(p, a):
    return _fma(p[3], a[3], _fma(p[2], a[2], _fma(p[1], a[1], p[0] * a[0])))


def _dot_gemv(p, a):
    return (p[0] * a[0] + p[2] * a[2]) + (p[1] * a[1] + p[3] * a[3])


def _uv(P, pt, dot):
    a = (pt[0], pt[1], pt[2], 1.0)
    r = [dot(P[i], a) for i in range(3)]
    return r[0] / r[2], r[1] / r[2]


def _search_x(P, y, z, target, pred, rng, span=600):
    """x near the point whose u equals `target` (y, z given; z nudged until one is
    found) with pred(u_chain, u_gemv) true: a linear walk over x's neighbours."""
    for _ in range(200):
        base = (target * (P[2, 2] * z + P[2, 3]) - P[0, 2] * z - P[0, 3]) / P[0, 0]
        lo = base
        for _ in range(span):
            lo = np.nextafter(lo, -np.inf)
        x = lo
        for _ in range(2 * span):
            uc, _ = _uv(P, (x, y, z), _dot_chain)
            ug, _ = _uv(P, (x, y, z), _dot_gemv)
            if pred(uc, ug):
                return x
            x = np.nextafter(x, np.inf)
        z = z + rng.uniform(0.01, 0.5)
    raise RuntimeError("no discriminating point found")


def _single_case():
    """Frames whose projections go through dgemv (transform.py:17-19 with one column):
    single_tie  -- one point, round(u) differs between the two orders;
    single_clip -- one point, u < W-1 under one order and not the other;
    one_survivor -- 40 points, exactly one inside the clip, at a rounding tie (the clip
                    runs as dgemm over all columns, the projection of the survivor as dgemv)."""
    rng = np.random.default_rng(31)
    P = synth.KITTI_P2
    im, bv = (1200, 360), (704, 800)
    spec = synth.FrameSpec(1, im, bv)

    def frame(pts, vox):
        return synth.Frame(np.asarray(pts, dtype=np.float64).reshape(-1, 3), np.asarray(vox, dtype=np.int64),
                           P, spec)
    y, z = 0.7, 23.0
    tie = lambda uc, ug: np.round(uc) != np.round(ug) and 0 <= min(uc, ug) and max(uc, ug) < im[0] - 1  # noqa
    x = _search_x(P, y, z, 500.5, tie, rng)
    _index_case("single_tie", frame([x, y, z], [[300, 400]]), im, bv, (1, 1))
    clip = lambda uc, ug: (uc < im[0] - 1) != (ug < im[0] - 1)  # noqa
    x = _search_x(P, -1.1, 31.0, im[0] - 1.0, clip, rng)
    _index_case("single_clip", frame([x, -1.1, 31.0], [[10, 20]]), im, bv, (1, 1))
    x = _search_x(P, 0.3, 12.0, 731.5, tie, rng)
    out = np.stack([rng.uniform(60, 90, 39), rng.uniform(-2, 2, 39), rng.uniform(5, 10, 39)], 1)
    pts = np.insert(out, 17, [x, 0.3, 12.0], axis=0)
    vox = np.stack([rng.integers(0, bv[1], 40), rng.integers(0, bv[0], 40)], 1)
    _index_case("one_survivor", frame(pts, vox), im, bv, (2, 2))


def _mv3d_calib_case():
    """MV3D transform.calib_to_P / calib_to_L2C (MV3D_TF_release/lib/utils/transform.py:13-30)
    on a random imdb-layout calib (4 x 12 rows)."""
    import importlib
    tr = importlib.import_module("utils.transform")
    rng = np.random.default_rng(51)
    calib = rng.normal(0, 1, (4, 12)) * np.array([700, 1, 600, 40, 1, 700, 170, 0.2, 1, 1, 1, 0.003])
    np.savez_compressed(os.path.join(HERE, "mv3d_calib.npz"), calib=calib, P=tr.calib_to_P(calib.copy()),
                        P_cam=tr.calib_to_P(calib.copy(), from_camera=True), L2C=tr.calib_to_L2C(calib.copy()))
    print("mv3d_calib: P", tr.calib_to_P(calib.copy()).shape)


def _kitti_single_case():
    """get_lidar_point_cloud on scans whose products are single-column (dgemv):
    a one-point scan (lidar_to_cam_frame with one column, then the FOV projection),
    and a scan whose only point in front of the camera is its one FOV candidate."""
    import tempfile
    from wavedata.tools.core import calib_utils
    from wavedata.tools.obj_detection import obj_utils
    rng = np.random.default_rng(41)
    rec = {}
    text = "".join(f"{k}: " + " ".join(f"{v:.12e}" for v in vals) + "\n" for k, vals in KITTI_CALIB.items())
    shape = (375, 1242)
    with tempfile.TemporaryDirectory() as d:
        for sub in ("calib", "velodyne"):
            os.makedirs(os.path.join(d, sub))
        scans = {0: np.array([[11.3, 1.7, -0.4, 0.5]], np.float32)}
        behind = np.stack([rng.uniform(-30, -5, 30), rng.uniform(-5, 5, 30), rng.uniform(-1, 1, 30),
                           rng.uniform(0, 1, 30)], 1).astype(np.float32)
        scans[1] = np.insert(behind, 11, [9.6, -2.2, 0.3, 0.9], axis=0)
        for idx, scan in scans.items():
            with open(os.path.join(d, "calib", "%06d.txt" % idx), "w") as fh:
                fh.write(text)
            scan.tofile(os.path.join(d, "velodyne", "%06d.bin" % idx))
            pc = obj_utils.get_lidar_point_cloud(idx, os.path.join(d, "calib"), os.path.join(d, "velodyne"),
                                                 im_size=[shape[1], shape[0]])
            pc_all = obj_utils.get_lidar_point_cloud(idx, os.path.join(d, "calib"), os.path.join(d, "velodyne"))
            fc = calib_utils.read_calibration(os.path.join(d, "calib"), idx)
            rec.update({f"{idx}_velo": scan, f"{idx}_point_cloud": pc, f"{idx}_point_cloud_all": pc_all,
                        f"{idx}_p2": fc.p2, f"{idx}_r0_rect": fc.r0_rect, f"{idx}_tr": fc.tr_velodyne_to_cam})
            print(f"kitti_single {idx}: scan {scan.shape[0]} -> FOV {pc.shape[1]}")
    rec["image_shape"] = np.array(shape)
    np.savez_compressed(os.path.join(HERE, "kitti_single.npz"), **rec)


def _kitti_case():
    """obj_utils.get_lidar_point_cloud / calib_utils.read_calibration /
    get_road_plane + the kitti_aug flips on synthetic KITTI files."""
    import tempfile
    from wavedata.tools.core import calib_utils
    from wavedata.tools.obj_detection import obj_utils
    from avod.datasets.kitti import kitti_aug
    rng = np.random.default_rng(21)
    rec = {}
    with tempfile.TemporaryDirectory() as d:
        for sub in ("calib", "velodyne", "planes"):
            os.makedirs(os.path.join(d, sub))
        for idx, (n, plane_b_sign, shape) in {7: (5000, -1, (375, 1242)), 8: (4000, 1, (376, 1241))}.items():
            calib = dict(KITTI_CALIB)
            if idx == 8:  # a second camera geometry
                calib["P2"] = list(np.array(calib["P2"]) * np.array([1, 1, 1.0003, 1, 1, 1, 0.999, 1, 1, 1, 1, 1]))
            text = "".join(f"{k}: " + " ".join(f"{v:.12e}" for v in vals) + "\n" for k, vals in calib.items())
            with open(os.path.join(d, "calib", "%06d.txt" % idx), "w") as fh:
                fh.write(text)
            scan = synthetic_scan(rng, n)
            scan.tofile(os.path.join(d, "velodyne", "%06d.bin" % idx))
            plane = np.array([-1.851372e-02, plane_b_sign * 9.998285e-01, -5.362401e-04, 1.678541e+00])
            ptext = "# Plane\nWidth 4\nHeight 1\n" + " ".join(f"{v:e}" for v in plane) + "\n"
            with open(os.path.join(d, "planes", "%06d.txt" % idx), "w") as fh:
                fh.write(ptext)
            fc = calib_utils.read_calibration(os.path.join(d, "calib"), idx)
            im_size = [shape[1], shape[0]]  # kitti_utils.get_point_cloud: (w, h)
            pc = obj_utils.get_lidar_point_cloud(idx, os.path.join(d, "calib"), os.path.join(d, "velodyne"),
                                                 im_size=im_size)
            pc_all = obj_utils.get_lidar_point_cloud(idx, os.path.join(d, "calib"), os.path.join(d, "velodyne"))
            gp = obj_utils.get_road_plane(idx, os.path.join(d, "planes"))
            rec.update({f"{idx}_calib_text": np.array(text), f"{idx}_plane_text": np.array(ptext),
                        f"{idx}_velo": scan, f"{idx}_image_shape": np.array(shape),
                        f"{idx}_p2": fc.p2, f"{idx}_r0_rect": fc.r0_rect, f"{idx}_tr": fc.tr_velodyne_to_cam,
                        f"{idx}_point_cloud": pc, f"{idx}_point_cloud_all": pc_all, f"{idx}_ground_plane": gp,
                        f"{idx}_flip_point_cloud": kitti_aug.flip_point_cloud(pc),
                        f"{idx}_flip_p2": kitti_aug.flip_stereo_calib_p2(fc.p2, shape),
                        f"{idx}_flip_ground_plane": kitti_aug.flip_ground_plane(gp)})
            print(f"kitti {idx}: scan {n} -> FOV {pc.shape[1]} points; plane {gp}")
    np.savez_compressed(os.path.join(HERE, "kitti_frames.npz"), **rec)


def main():
    _install_stubs()
    c1 = synth.CONFIG1
    f1 = synth.make_frame(c1, seed=0, n_outside=64)
    _index_case("config1", f1, c1.im_size, c1.bv_size, c1.stride)
    s2 = synth.FrameSpec(4000, (1200, 360), (704, 800), (1, 1))
    _index_case("stride1", synth.make_frame(s2, seed=1, n_outside=32), s2.im_size, s2.bv_size, (1, 1))
    s3 = synth.FrameSpec(3000, (1242, 375), (700, 800), (8, 2))
    f3 = synth.make_frame(s3, seed=2)
    # MV3D convention: stride[0] applies to the image, stride[1] to BEV; M_val given.
    # All voxel rows kept in range so that len(M_val) == nnz (MV3D never drops).
    f3.voxel_indices[:, 1] = np.minimum(f3.voxel_indices[:, 1], s3.bv_size[0] - 1)
    mval = 1.0 / np.random.default_rng(3).integers(1, 9, f3.points.shape[0])
    _index_case("mv3d", f3, s3.im_size, s3.bv_size, s3.stride, M_val=mval, mv3d=True)
    s4 = synth.FrameSpec(2500, (1200, 360), (704, 800), (3, 5))
    _index_case("oddstride", synth.make_frame(s4, seed=4, n_outside=16), s4.im_size, s4.bv_size, s4.stride)
    fk, imk, bvk = _kat_frame()
    _index_case("kat", fk, imk, bvk, (4, 4))
    _index_case("kat_s1", _kat_frame()[0], imk, bvk, (1, 1))
    s0 = synth.FrameSpec(0, (1200, 360), (704, 800), (4, 4))
    e = synth.Frame(np.zeros((0, 3)), np.zeros((0, 2), dtype=np.int64), synth.KITTI_P2, s0)
    try:
        _index_case("empty", e, s0.im_size, s0.bv_size, s0.stride)
    except Exception as ex:  # record what the reference does with no points
        print("empty frame: reference raised", type(ex).__name__, ex)
    _single_case()
    _bev_slices_case()
    _mv3d_voxel_case()
    _mv3d_voxel_case(dense=True)
    _kitti_case()
    _kitti_single_case()
    _mv3d_calib_case()


if __name__ == "__main__":
    if len(sys.argv) > 1:  # regenerate only the named cases, e.g. `kitti`
        _install_stubs()
        for name in sys.argv[1:]:
            globals()[f"_{name}_case"]()
    else:
        main()
