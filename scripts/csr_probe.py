"""k_csr_frame phase timing (scripts/r04_csrp.sh): the config-2 index build + cell CSR of 64 frames in a loop
(no consumer of the CSR: the probe variants leave it incomplete)."""
import sys

import torch

sys.path.insert(0, ".")
from sparse_pooling_amd import dist as sd, pipeline, synth  # noqa: E402

dev = torch.device("cuda", 0)
spec = synth.CONFIG2
frames = [synth.make_frame(spec, seed=s, n_outside=200) for s in range(64)]
pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
pl = pipeline.FusedPipeline(64, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                            dtype=torch.bfloat16, device=dev)
pl.build_index(pts, vox, off, P)
torch.cuda.synchronize()
for _ in range(20):
    pl.build_csr(("cell",))
torch.cuda.synchronize()
print("done")
