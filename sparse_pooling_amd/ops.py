"""The SHPL pulls as PyTorch operators, ``torch.ops.shpl.*``, registered with
``torch.library`` over the libshpl C ABI (the Python layer wraps
the ABI as torch.library ops, and autograd maps fwd <-> trans).

* ``torch.ops.shpl.pull``: one destination-keyed pull (``shpl_pull``) with
  every output mode -- pooled, ``[pass || pooled]`` (the concat of
  sparse_pool_utils.py:72 / :87 fused in), ``pass + pooled`` (the add_n of
  the gradients). No autograd: the primitive.
* ``torch.ops.shpl.spmm``: ``out = M-pull(src)`` through a forward CSR, with
  its gradient registered as the pull through the backward CSR (the other
  direction). With ``direction = SHPL_BY_CELL`` and the cell-keyed CSR in
  entry order it is ``_sparse_pool_op`` (sparse_pool_utils.py:96-103), whose
  TF gradient is the pixel-keyed pull in (column, entry) order; with
  ``SHPL_BY_PIXEL`` and the (column, row) pixel-keyed CSR it is
  ``_sparse_pool_trans_op`` (:105-117), whose gradient is the cell-keyed pull
  in (column, entry) order. The gradient's gradient is the forward pull again.

A CSR crosses the op boundary as its tensors (``ent_dst``, ``ent_src``,
``ent_val`` and, pixel-keyed, ``ent_col``); ``ShplMap.csr_tensors`` hands
them out. The ops run on the GPU only: calling them on CPU tensors raises
(there is no CPU fallback); fake tensors get shapes from the registered
fake functions, so the ops trace under ``torch.compile`` / ``torch.export``.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
from torch import Tensor

from . import _lib as L

__all__ = ["pull", "spmm", "sparse_pool", "sparse_pool_trans"]


def _csr(ent_dst, ent_src, ent_val, ent_col, n_keys):
    return L.ShplCsr(ent_dst.data_ptr(), ent_src.data_ptr(), ent_val.data_ptr(),
                     None if ent_col is None else ent_col.data_ptr(), int(n_keys), int(ent_dst.numel()))


def _rows(t: Tensor) -> int:
    return t.numel() // t.shape[-1] if t.dim() > 0 and t.shape[-1] > 0 else 0


def _check_csr(ent_dst, ent_src, ent_val, ent_col, direction):
    for t in (ent_dst, ent_src, ent_col):
        if t is not None and t.dtype != torch.int32:
            raise TypeError("CSR index arrays must be int32")
    if ent_val.dtype != torch.float32:
        raise TypeError("CSR values must be float32")
    n = ent_dst.numel()
    if ent_src.numel() != n or ent_val.numel() != n or (ent_col is not None and ent_col.numel() != n):
        raise ValueError("CSR arrays differ in length")
    if direction == L.BY_PIXEL and ent_col is None:
        raise ValueError("a pixel-keyed CSR carries ent_col")


@torch.library.custom_op("shpl::pull", mutates_args=(), device_types="cuda")
def pull(src: Tensor, ent_dst: Tensor, ent_src: Tensor, ent_val: Tensor, ent_col: Optional[Tensor],
         direction: int, out_shape: List[int], src_off: int, c_pool: int, pass_: Optional[Tensor], pass_off: int,
         c_pass: int, mode: int) -> Tensor:
    """shpl_pull: channels [src_off, src_off + c_pool) of the rows of ``src``
    ([.., C_src], row-contiguous) pooled into the destination rows of
    ``out_shape``; with ``pass_``, its channels [pass_off, pass_off + c_pass)
    are concatenated in front (CONCAT: c_pass + c_pool output channels) or
    added (ADD: c_pass == c_pool)."""
    _check_csr(ent_dst, ent_src, ent_val, ent_col, direction)
    src = src.contiguous()
    pass_ = None if pass_ is None else pass_.contiguous()
    out = torch.empty(out_shape, dtype=src.dtype, device=src.device)
    if pass_ is None:
        c_pass = 0
    if src_off < 0 or src_off + c_pool > src.shape[-1] or (
            pass_ is not None and (pass_off < 0 or pass_off + c_pass > pass_.shape[-1])):
        raise ValueError("channel range outside the row")
    n_keys = _rows(out)
    if mode == L.OUT_CONCAT and out.shape[-1] != c_pass + c_pool:
        raise ValueError(f"concat output has {out.shape[-1]} channels, expected {c_pass} + {c_pool}")
    if mode != L.OUT_CONCAT and out.shape[-1] != c_pool:
        raise ValueError(f"output has {out.shape[-1]} channels, expected {c_pool}")
    if pass_ is not None and _rows(pass_) != n_keys:
        raise ValueError("pass-through rows differ from the output rows")
    csr = _csr(ent_dst, ent_src, ent_val, ent_col, n_keys)
    L.check(L.lib().shpl_pull(int(direction), L.dtype_code(out), ctypes.byref(csr), L.ptr(src), int(src.shape[-1]),
                              int(src_off), int(c_pool), L.ptr(pass_), 0 if pass_ is None else int(pass_.shape[-1]),
                              int(pass_off), int(c_pass), int(mode), L.ptr(out), int(out.shape[-1]),
                              L.stream_of(src.device)), "shpl_pull")
    return out


@pull.register_fake
def _pull_fake(src, ent_dst, ent_src, ent_val, ent_col, direction, out_shape, src_off, c_pool, pass_, pass_off,
               c_pass, mode):
    return src.new_empty(out_shape)


@torch.library.custom_op("shpl::spmm", mutates_args=(), device_types="cuda")
def spmm(src: Tensor, f_dst: Tensor, f_src: Tensor, f_val: Tensor, f_col: Optional[Tensor], b_dst: Tensor,
         b_src: Tensor, b_val: Tensor, b_col: Optional[Tensor], direction: int, out_shape: List[int]) -> Tensor:
    """out[.., C] = the pull of src's rows through the forward CSR (f_*) in
    ``direction``; the backward CSR (b_*, the other direction) is carried for
    the gradient."""
    c = int(src.shape[-1])
    return pull(src, f_dst, f_src, f_val, f_col, direction, list(out_shape[:-1]) + [c], 0, c, None, 0, 0, L.OUT_POOL)


@spmm.register_fake
def _spmm_fake(src, f_dst, f_src, f_val, f_col, b_dst, b_src, b_val, b_col, direction, out_shape):
    return src.new_empty(list(out_shape[:-1]) + [src.shape[-1]])


def _spmm_setup(ctx, inputs, output):
    src, f_dst, f_src, f_val, f_col, b_dst, b_src, b_val, b_col, direction, out_shape = inputs
    ctx.src_shape = list(src.shape)
    ctx.direction = direction
    ctx.save_for_backward(f_dst, f_src, f_val, f_col, b_dst, b_src, b_val, b_col)


def _spmm_backward(ctx, grad):
    f_dst, f_src, f_val, f_col, b_dst, b_src, b_val, b_col = ctx.saved_tensors
    other = L.BY_PIXEL if ctx.direction == L.BY_CELL else L.BY_CELL
    # the TF gradient: the pull in the other direction through the backward CSR, itself differentiable
    d = torch.ops.shpl.spmm(grad, b_dst, b_src, b_val, b_col, f_dst, f_src, f_val, f_col, other, ctx.src_shape)
    return d, None, None, None, None, None, None, None, None, None, None


spmm.register_autograd(_spmm_backward, setup_context=_spmm_setup)


def sparse_pool(img: Tensor, smap, bev_shape) -> Tensor:
    """_sparse_pool_op(M, img, img_index_flip, pooled_size) as torch.ops.shpl.spmm."""
    f = smap.csr_tensors(L.BY_CELL, L.ORDER_ENTRY)
    b = smap.csr_tensors(L.BY_PIXEL, L.ORDER_COL_ENTRY)
    return torch.ops.shpl.spmm(img, *f, *b, L.BY_CELL, list(bev_shape[:3]) + [int(img.shape[-1])])


def sparse_pool_trans(bev: Tensor, smap, img_shape) -> Tensor:
    """_sparse_pool_trans_op(M, bev, img_index_flip, img_size) as torch.ops.shpl.spmm."""
    f = smap.csr_tensors(L.BY_PIXEL, L.ORDER_COL_ROW)
    b = smap.csr_tensors(L.BY_CELL, L.ORDER_COL_ENTRY)
    return torch.ops.shpl.spmm(bev, *f, *b, L.BY_PIXEL, list(img_shape[:3]) + [int(bev.shape[-1])])
