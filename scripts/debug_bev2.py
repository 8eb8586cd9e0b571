import sys, os, types
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from sparse_pooling_amd import bev, synth
g = np.load("tests/golden/bev_slices.npz")
cfg = types.SimpleNamespace(height_lo=-0.2, height_hi=2.3, num_slices=5)
maps, vox, upts = bev.BevSlices(cfg).generate_bev("lidar", g["point_cloud"], g["ground_plane"], g["area_extents"], 0.1, output_indices=True)
print("generate_bev golden", vox.shape)
pts = torch.from_numpy(np.ascontiguousarray(g["point_cloud"].T)).cuda()
for name, off in [("tensor list", torch.tensor([0, pts.shape[0]], dtype=torch.int64, device="cuda")),
                  ("np concat", torch.tensor(np.concatenate([[0], np.cumsum([pts.shape[0]])])).cuda())]:
    for pname, pl in [("gp", torch.as_tensor(g["ground_plane"].reshape(1, 4)).cuda()),
                      ("synth", torch.from_numpy(np.stack([synth.GROUND_PLANE])).cuda())]:
        for ename, ext in [("g", g["area_extents"]), ("synth", synth.AREA_EXTENTS)]:
            b = bev.bev_slices_batch(pts, off, pl, ext, 0.1, -0.2, 2.3, 5)
            torch.cuda.synchronize()
            print(name, off.dtype, pname, ename, int(b.frame_nvox[0]), g["area_extents"].dtype, synth.AREA_EXTENTS.dtype)
