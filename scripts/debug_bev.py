import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from sparse_pooling_amd import bev, synth
from oracle import shpl_oracle as orc
g = np.load("tests/golden/bev_slices.npz")
def run(clouds, planes):
    pts = torch.from_numpy(np.concatenate([c.T for c in clouds])).cuda()
    off = torch.tensor(np.concatenate([[0], np.cumsum([c.shape[1] for c in clouds])])).cuda()
    b = bev.bev_slices_batch(pts, off, torch.from_numpy(np.stack(planes)).cuda(), synth.AREA_EXTENTS, 0.1, -0.2, 2.3, 5)
    torch.cuda.synchronize()
    res = []
    for f, c in enumerate(clouds):
        hm, dm, vox, upts = orc.bev_slices(c, planes[f], synth.AREA_EXTENTS, 0.1, -0.2, 2.3, 5)
        res.append((int(b.frame_nvox[f]), len(vox)))
    return res
gc = g["point_cloud"]
print("golden x1", run([gc], [synth.GROUND_PLANE]))
print("golden x2", run([gc, gc], [synth.GROUND_PLANE] * 2))
c0 = synth.make_cloud(15000, 200)
print("cloud x1", run([c0], [synth.GROUND_PLANE]))
inside = c0[:, (c0[0] > -40) & (c0[0] < 40) & (c0[2] > 0) & (c0[2] < 70)]
print("cloud inside x1", run([inside], [synth.GROUND_PLANE]))
print("golden first 15000", run([gc[:, :15000]], [synth.GROUND_PLANE]))
