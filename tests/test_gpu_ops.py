"""torch.ops.shpl.* (sparse_pooling_amd/ops.py) on MI355X: torch.library's
own consistency checks (schema, fake tensor, autograd registration, AOT
dispatch), the registered gradient == the opposite-direction pull == the
oracle's TF gradient (bitwise, TF order), and the gradient of the gradient
== the forward pull."""
import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc
from sparse_pooling_amd import _lib as L, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module")
def case():
    from sparse_pooling_amd import shpl_map as sm
    L.lib()
    spec = synth.CONFIGS[1]
    fr = synth.make_frame(spec, seed=31, n_outside=10)
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                            tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    img = synth.make_features((1, Hi, Wi, spec.c_img), 32)
    bev = synth.make_features((1, Hb, Wb, spec.c_bev), 33)
    smap = sm.pack_map(_t(ref["Mij_pool"]), _t(ref["M_val"].astype(np.float32)), ref["M_size"],
                       _t(ref["img_index_flip_pool"]), img.shape)
    return spec, ref, smap, img, bev


def test_opcheck(case):
    from sparse_pooling_amd import ops  # noqa: F401
    spec, ref, smap, img, bev = case
    f = smap.csr_tensors(L.BY_CELL, L.ORDER_ENTRY)
    b = smap.csr_tensors(L.BY_PIXEL, L.ORDER_COL_ENTRY)
    ti = _t(img).requires_grad_(True)
    torch.library.opcheck(torch.ops.shpl.spmm, (ti, *f, *b, L.BY_CELL, list(bev.shape[:3]) + [img.shape[-1]]))
    torch.library.opcheck(torch.ops.shpl.pull, (_t(img), *f, L.BY_CELL, list(bev.shape[:3]) + [bev.shape[-1] + img.shape[-1]],
                                                0, img.shape[-1], _t(bev), 0, bev.shape[-1], L.OUT_CONCAT))


def test_gradients_map_fwd_to_trans(case):
    from sparse_pooling_amd import ops
    spec, ref, smap, img, bev = case
    idx = ref["img_index_flip_pool"]
    ti = _t(img).requires_grad_(True)
    y = ops.sparse_pool(ti, smap, bev.shape)
    ey = orc.sparse_pool_op(ref["Mij_pool"], ref["M_val"], ref["M_size"], img, idx)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), ey.reshape(y.shape))
    g = _t(synth.make_features(tuple(y.shape), 34)).requires_grad_(True)
    (d_img,) = torch.autograd.grad(y, ti, g, create_graph=True)
    e_img = orc.sparse_pool_grad_img(ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                     g.detach().cpu().numpy().reshape(-1, spec.c_img), idx, img.shape)
    np.testing.assert_array_equal(d_img.detach().cpu().numpy(), e_img)
    # the registered gradient is the transposed op, so the trans op on g's layout gives the same map
    np.testing.assert_array_equal(d_img.detach().cpu().numpy(),
                                  ops.sparse_pool_trans(g.detach(), smap, img.shape).cpu().numpy())
    # gradient of the gradient (d/dg of <d_img, h>) == the forward pull of h
    h = _t(synth.make_features(img.shape, 35))
    (gg,) = torch.autograd.grad(d_img, g, h)
    np.testing.assert_array_equal(gg.cpu().numpy(), ops.sparse_pool(h, smap, bev.shape).detach().cpu().numpy())
    tb = _t(bev).requires_grad_(True)
    z = ops.sparse_pool_trans(tb, smap, img.shape)
    gz = _t(synth.make_features(tuple(z.shape), 36))
    z.backward(gz)
    e_bev = orc.sparse_pool_trans_grad_bev(ref["Mij_pool"], ref["M_val"], ref["M_size"], gz.cpu().numpy(), idx)
    np.testing.assert_array_equal(tb.grad.cpu().numpy(), e_bev.reshape(bev.shape))
