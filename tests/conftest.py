import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


KITTI_IDX = (7, 8)


@pytest.fixture(scope="session")
def kitti_dir(tmp_path_factory):
    """The reference-generated KITTI fixture (tests/golden/kitti_frames.npz) written
    back to disk in KITTI's layout: calib/, velodyne/, planes/ (%06d names)."""
    import numpy as np
    g = np.load(os.path.join(GOLDEN, "kitti_frames.npz"))
    d = tmp_path_factory.mktemp("kitti")
    for sub in ("calib", "velodyne", "planes"):
        (d / sub).mkdir()
    for idx in KITTI_IDX:
        (d / "calib" / ("%06d.txt" % idx)).write_text(str(g[f"{idx}_calib_text"]))
        (d / "planes" / ("%06d.txt" % idx)).write_text(str(g[f"{idx}_plane_text"]))
        g[f"{idx}_velo"].astype(np.float32).tofile(str(d / "velodyne" / ("%06d.bin" % idx)))
    return str(d), g
