"""Link-prediction head: Philox negative sampler (A10) + dot-product decoder (A11) on libhgin.so.

NOT IN REFERENCE: the reference trains a path-delay regressor; BASELINE.json's north
star asks for a negative-edge sampler and a dot-product link decoder as HIP kernels.  This module is an
*additional* head over HetroGIN's node embeddings; it does not replace the readout train.py calls.

Specs (include/hgin.h): sampler out[i] = hi32(philox4x32_10(block (offset+i)>>2)[(offset+i)&3] * n_dst);
decoder score[e] = <z_src[src[e]], z_dst[dst[e]]>, backward = weighted segmented sums over the pairs'
CSR / CSC (bit-exact against oracle/hgin_oracle.c).
"""
from __future__ import annotations

import torch
from torch import Tensor

from . import _lib, ops


def sample_negative_dst(n: int, n_dst: int, seed: int, offset: int = 0, device="cuda") -> Tensor:
    out = torch.empty(n, dtype=torch.int32, device=device)
    if n:
        _lib.call("hgin_neg_sample", int(seed) & (2**64 - 1), int(offset), n, int(n_dst), ops._p(out),
                  ops._stream(out))
    return out


def negative_edges(edge_index: Tensor, n_dst: int, k: int, seed: int, offset: int = 0) -> Tensor:
    """k corrupted copies of every positive edge: src kept, dst drawn uniformly."""
    ops.require_device(edge_index, what="negative_edges")
    E = int(edge_index.size(1))
    dst = sample_negative_dst(E * k, n_dst, seed, offset, edge_index.device).long()
    src = edge_index[0].repeat_interleave(k)
    return torch.stack([src, dst])


class _DotDecodeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z_src, z_dst, pairs: Tensor, graph: ops.RelationGraph):
        n = int(pairs.size(1))
        F = int(z_src.size(1))
        src32 = pairs[0].to(torch.int32).contiguous()
        dst32 = pairs[1].to(torch.int32).contiguous()
        score = torch.empty(n, dtype=torch.float32, device=z_src.device)
        _lib.call("hgin_dot_decode_fwd_f32", ops._p(src32), ops._p(dst32), n, ops._p(z_src), z_src.stride(0),
                  ops._p(z_dst), z_dst.stride(0), F, ops._p(score), ops._stream(score))
        ctx.graph = graph
        ctx.save_for_backward(z_src, z_dst)
        return score

    @staticmethod
    def backward(ctx, g):
        z_src, z_dst = ctx.saved_tensors
        g = g.contiguous()
        graph = ctx.graph
        F = int(z_src.size(1))
        g_src = g_dst = None
        if ctx.needs_input_grad[0]:
            csc = graph.csc           # rows = src, col = dst
            g_src = torch.empty_like(z_src)
            _lib.call("hgin_dot_decode_bwd_f32", ops._p(csc.rowptr), ops._p(csc.col), ops._p(csc.perm), csc.n_rows,
                      ops._p(g), ops._p(z_dst), z_dst.stride(0), F, ops._p(g_src), g_src.stride(0),
                      ops._stream(g))
        if ctx.needs_input_grad[1]:
            csr = graph.csr           # rows = dst, col = src
            g_dst = torch.empty_like(z_dst)
            _lib.call("hgin_dot_decode_bwd_f32", ops._p(csr.rowptr), ops._p(csr.col), ops._p(csr.perm), csr.n_rows,
                      ops._p(g), ops._p(z_src), z_src.stride(0), F, ops._p(g_dst), g_dst.stride(0),
                      ops._stream(g))
        return g_src, g_dst, None, None


def dot_decode(z_src: Tensor, z_dst: Tensor, pairs: Tensor) -> Tensor:
    """score[e] = <z_src[pairs[0, e]], z_dst[pairs[1, e]]> with a HIP backward."""
    ops.require_device(z_src, z_dst, pairs, what="dot_decode")
    z_src = ops._rowmajor(ops._f32(z_src, "z_src"))
    z_dst = ops._rowmajor(ops._f32(z_dst, "z_dst"))
    if z_src.size(1) != z_dst.size(1):
        raise RuntimeError("dot_decode: embedding widths differ")
    graph = ops.relation_graph(pairs, z_src.size(0), z_dst.size(0))
    return _DotDecodeFn.apply(z_src, z_dst, pairs, graph)


def link_loss(z_src: Tensor, z_dst: Tensor, pos: Tensor, k: int, seed: int, offset: int = 0) -> Tensor:
    """BCE-with-logits over positives and k uniform negatives per positive."""
    neg = negative_edges(pos, z_dst.size(0), k, seed, offset)
    s_pos = dot_decode(z_src, z_dst, pos)
    s_neg = dot_decode(z_src, z_dst, neg)
    bce = torch.nn.functional.binary_cross_entropy_with_logits
    return bce(s_pos, torch.ones_like(s_pos)) * 0.5 + bce(s_neg, torch.zeros_like(s_neg)) * 0.5
