"""torch.library registration of the SHPL pulls (the Python layer
wraps the C ABI as torch.library ops, autograd mapping fwd <-> trans), checked
on CPU: schemas, fake-tensor shape functions, and that CPU tensors are
refused (the ops have no CPU implementation -- no fallback). Their GPU
behaviour: tests/test_gpu_ops.py."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from sparse_pooling_amd import _lib as L
from sparse_pooling_amd import ops  # noqa: F401 -- registers torch.ops.shpl


def _csr(n, fake_col):
    i32 = dict(dtype=torch.int32)
    return (torch.empty(n, **i32), torch.empty(n, **i32), torch.empty(n, dtype=torch.float32),
            torch.empty(n, **i32) if fake_col else None)


def test_ops_registered_with_schemas():
    spmm = str(torch.ops.shpl.spmm.default._schema)
    pull = str(torch.ops.shpl.pull.default._schema)
    assert spmm.startswith("shpl::spmm(Tensor src, Tensor f_dst, Tensor f_src, Tensor f_val, Tensor? f_col")
    assert "SymInt direction, SymInt[] out_shape) -> Tensor" in spmm
    assert pull.startswith("shpl::pull(Tensor src, Tensor ent_dst, Tensor ent_src, Tensor ent_val, Tensor? ent_col")
    assert "Tensor? pass_, SymInt pass_off, SymInt c_pass, SymInt mode) -> Tensor" in pull


def test_fake_tensor_shapes():
    with FakeTensorMode():
        img = torch.empty(2, 9, 30, 16)
        bev = torch.empty(2, 17, 20, 12)
        cell, pix = _csr(300, False), _csr(300, True)
        y = torch.ops.shpl.spmm(img, *cell, *pix, L.BY_CELL, [2, 17, 20, 16])
        assert tuple(y.shape) == (2, 17, 20, 16) and y.dtype == img.dtype
        z = torch.ops.shpl.spmm(bev, *pix, *cell, L.BY_PIXEL, [2, 9, 30, 12])
        assert tuple(z.shape) == (2, 9, 30, 12)
        cat = torch.ops.shpl.pull(img, *cell, L.BY_CELL, [2, 17, 20, 28], 0, 16, bev, 0, 12, L.OUT_CONCAT)
        assert tuple(cat.shape) == (2, 17, 20, 28)


def test_cpu_tensors_are_refused():
    img = torch.zeros(1, 3, 4, 8)
    cell, pix = _csr(5, False), _csr(5, True)
    with pytest.raises(NotImplementedError):
        torch.ops.shpl.spmm(img, *cell, *pix, L.BY_CELL, [1, 2, 2, 8])
