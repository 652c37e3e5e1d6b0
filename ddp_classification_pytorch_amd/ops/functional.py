"""Autograd functions over the gfx950 primitives.

Every function is written once against the primitive API (``torch.ops.dcp``
on GPU tensors, :mod:`._ref` on CPU tensors) via :func:`K`.  On a GPU tensor
the HIP library is mandatory: :func:`K` raises if it cannot be loaded.

Layouts: activations NHWC (bf16 on GPU), conv weights [Co,KH,KW,Ci] fp32
masters, linear weights [out,in] fp32 masters.  bf16 GEMM copies of the
weights are produced by one ``weight_prep`` launch per layer per weight
version and cached on the parameter.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import weakref

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.autograd import Function

from .. import _ext
from ..parallel import peer as _peer
from . import _ref

ACT = {"none": 0, "relu": 1, "leaky": 2, "leaky_relu": 2, None: 0}


def K(t: torch.Tensor):
    """Primitive namespace for tensor ``t``: HIP kernels on GPU, reference math on CPU."""
    return _ext.hip_ops() if t.is_cuda else _ref


def act_dtype(device: torch.device) -> torch.dtype:
    return torch.bfloat16 if device.type == "cuda" else torch.float32


def round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


# ----------------------------------------------------------------------------- host tables
_DEV_ANCHOR = {}


def table_to_device(rows, dtype, device) -> torch.Tensor:
    """Small host table (kernel argument lists: pointers, shapes) -> device tensor.  On the GPU
    the values travel in the arguments of a fill kernel (``dcp::table_fill``), not a host->device
    copy, so a table built while a step is being captured into a HIP graph replays correctly
    (a captured memcpy would re-read a host buffer that is gone, and pinning memory is not
    allowed during capture)."""
    host = rows.to(dtype).contiguous() if torch.is_tensor(rows) else torch.tensor(rows, dtype=dtype)
    device = torch.device(device)
    if device.type != "cuda":
        return host.to(device)
    flat = host.reshape(-1)
    if dtype == torch.int32:
        if flat.numel() % 2:
            flat = torch.cat([flat, flat.new_zeros(1)])
        words = flat.view(torch.int64)
    else:
        words = flat.to(torch.int64) if dtype != torch.int64 else flat
    anchor = _DEV_ANCHOR.get(device)
    if anchor is None:
        anchor = _DEV_ANCHOR[device] = torch.empty(1, device=device)
    out = _ext.hip_ops().table_fill(words.contiguous(), anchor)
    if dtype == torch.int32:
        out = out.view(torch.int32)[:host.numel()]
    return out.view(host.shape)


# ----------------------------------------------------------------------------- weight cache
_GEN = [0]


def bump_weight_generation():
    """Invalidate cached bf16 weight copies (called by optimizers / state loads)."""
    _GEN[0] += 1


def prepared_weight(w: torch.Tensor, co_pad: int = 0, transposed: bool = True, ci: int = 0):
    """(bf16 copy padded to co_pad rows, transposed copy) of a fp32 master, cached per version.

    On the GPU every registered weight lives in a persistent bf16 buffer and all stale
    ones are refreshed together by ONE multi-tensor launch (the first prepared_weight
    call after an optimizer step re-converts the whole model).  ``ci`` zero-pads the
    input-channel (last) dim (the stem's 3 -> 8)."""
    if w.is_cuda and w.dtype == torch.float32 and w.is_contiguous():
        return _MT.get(w, co_pad, transposed, ci)
    key = (w._version, _GEN[0], w.data_ptr(), co_pad, transposed, ci)
    cached = getattr(w, "_dcp_prep", None)
    if cached is not None and cached[0] == key:
        return cached[1], cached[2]
    wd = w.detach()
    if ci and ci != wd.shape[-1]:
        wd = F.pad(wd, (0, ci - wd.shape[-1]))
    if not wd.is_contiguous():
        wd = wd.contiguous()
    wb, wt = K(wd).weight_prep(wd, co_pad, transposed)
    if not wd.is_cuda:
        wb, wt = wb.to(act_dtype(wd.device)), wt.to(act_dtype(wd.device))
    try:
        w._dcp_prep = (key, wb, wt)
    except Exception:  # non-leaf / functional tensors cannot carry attributes
        pass
    return wb, wt


class _MTWeightCache:
    """Persistent bf16 (and transposed) copies of the fp32 master weights, refreshed in
    one `mt_weight_prep` launch per step from a packed device table of
    {fp32 src, bf16 dst, bf16 dst^T, shape} entries plus a (entry, tile) block list,
    both built once per set of stale weights and reused every step."""

    def __init__(self):
        self.entries = {}   # (id(w), co_pad, transposed, ci) -> entry dict
        self.tables = {}    # tuple of entry ids -> (entries tensor, blocks tensor)

    @staticmethod
    def _stamp(w):
        return (w._version, _GEN[0], w.data_ptr())

    def get(self, w, co_pad, transposed, ci):
        ek = (id(w), co_pad, bool(transposed), ci)
        e = self.entries.get(ek)
        if e is None or e["ref"]() is not w:
            e = self._register(w, co_pad, transposed, ci)
            self.entries[ek] = e
        if e["stamp"] != self._stamp(w):
            self.refresh()
        return e["wb"], e["wt"]

    def _register(self, w, co_pad, transposed, ci):
        Co, Ci_src = w.shape[0], w.shape[-1]
        mid = tuple(w.shape[1:-1])
        T = 1
        for d in mid:
            T *= d
        Ci = ci or Ci_src
        Cp = co_pad or Co
        wb = torch.empty((Cp,) + mid + (Ci,), dtype=torch.bfloat16, device=w.device)
        wt = (torch.empty((Ci,) + mid + (Cp,), dtype=torch.bfloat16, device=w.device) if transposed
              else torch.empty(0, dtype=torch.bfloat16, device=w.device))
        return {"ref": weakref.ref(w), "wb": wb, "wt": wt, "stamp": None,
                "shape": (Co, T, Ci_src, Ci, Cp), "transposed": bool(transposed)}

    def refresh(self):
        stale = []
        for k in list(self.entries):
            e = self.entries[k]
            w = e["ref"]()
            if w is None:
                del self.entries[k]
                continue
            if e["stamp"] != self._stamp(w):
                stale.append((k, e, w))
        if not stale:
            return
        # keyed by every pointer the table holds: a model rebuilt in the same process can reuse
        # the ids and master-weight addresses of a freed one while its bf16 copies moved
        tkey = tuple((k, w.data_ptr(), e["wb"].data_ptr(), e["wt"].data_ptr() if e["transposed"] else 0)
                     for k, e, w in stale)
        tab = self.tables.get(tkey)
        if tab is None:
            rows, blocks = [], []
            for i, (_, e, w) in enumerate(stale):
                Co, T, Ci_src, Ci, Cp = e["shape"]
                tci, tco = (Ci + 63) // 64, (Cp + 63) // 64
                wt_ptr = e["wt"].data_ptr() if e["transposed"] else 0
                rows.append([w.data_ptr(), e["wb"].data_ptr(), wt_ptr, Co | (T << 32), Ci_src | (Ci << 32),
                             Cp | (tci << 32), tco])
                blocks.extend((i, t) for t in range(T * tci * tco))
            dev = stale[0][2].device
            ent = table_to_device(rows, torch.int64, dev)
            blk = table_to_device(blocks, torch.int32, dev)
            if len(self.tables) > 16:
                self.tables.clear()
            tab = self.tables[tkey] = (ent, blk)
        _ext.hip_ops().mt_weight_prep(*tab)
        for _, e, w in stale:
            e["stamp"] = self._stamp(w)


_MT = _MTWeightCache()


# ----------------------------------------------------------------------------- convolution
class GradJoin:
    """Gradient hand-off for a block input consumed by several ops.

    The ``secondaries`` other consumers (an identity block's last BN+add+ReLU backward,
    a projection block's downsample-conv dgrad) *deposit* their gradient here instead
    of returning it to autograd; the block's first conv (the primary consumer) *claims*
    the sum and adds it in its dgrad epilogue -- no separate bf16 add kernel over the
    block-input gradient.  A deposit that arrives after the claim is handed back to
    autograd unchanged, so every backward order stays correct; the primary fuses the
    producer BN's backward (see :class:`BNSource`) only when all secondaries arrived.
    """

    __slots__ = ("grad", "expected", "arrived", "closed")

    def __init__(self, secondaries: int = 1):
        self.grad, self.expected, self.arrived, self.closed = None, secondaries, 0, False

    def deposit(self, g):
        if g is None:
            return g
        if self.closed:
            return g.full() if isinstance(g, StridedGrad) else g
        if self.grad is None:
            self.grad = g
        else:
            a = self.grad.full() if isinstance(self.grad, StridedGrad) else self.grad
            self.grad = a + (g.full() if isinstance(g, StridedGrad) else g)
        self.arrived += 1
        return None

    def claim(self, strided_ok: bool = False):
        """(summed deposits, all secondaries arrived).  A compact :class:`StridedGrad` is returned
        as such only to a caller that adds it itself (``strided_ok``), expanded otherwise."""
        self.closed = True
        g, self.grad = self.grad, None
        if isinstance(g, StridedGrad) and not strided_ok:
            g = g.full()
        return g, self.arrived >= self.expected


class StridedGrad:
    """The input gradient of a 1x1 / stride-2 / pad-0 conv (a projection block's downsample), kept
    compact: ``compact`` [N, ceil(H/2), ceil(W/2), C] holds the gradient of the even (y, x) pixels
    of the [N, H, W, C] input; every other pixel's is zero.  Computing it is a stride-1 1x1 GEMM
    over the output grid (no parity classes, no zero tiles), and the block's first conv adds it in
    its dgrad epilogue reading a quarter of the bytes (``conv_dgrad_bn``'s stride-2 add source)
    instead of a full-size, 3/4-zero tensor written and read back through HBM."""

    __slots__ = ("compact", "H", "W")

    def __init__(self, compact, H, W):
        self.compact, self.H, self.W = compact, H, W

    def full(self):
        N, _, _, C = self.compact.shape
        out = self.compact.new_zeros((N, self.H, self.W, C))
        out[:, ::2, ::2, :] = self.compact
        return out


ResidualLink = GradJoin  # identity-block residual hand-off (one secondary: the last BN's residual)

# DCP_STRIDED_DEPOSIT=0: the downsample conv's input gradient as a full-size tensor (A/B)
_STRIDED_DEPOSIT = [os.environ.get("DCP_STRIDED_DEPOSIT", "1") != "0"]


def set_strided_deposit(enabled: bool):
    _STRIDED_DEPOSIT[0] = bool(enabled)


class BNSource:
    """Attached (as ``_dcp_bnsrc``) to the output z of a training-mode BN(+ReLU)(+residual)
    layer so that the stride-1 conv consuming z can run that layer's backward reduction in
    its dgrad epilogue (``conv_dgrad_bn``): the epilogue emits the activation-masked
    gradient and the per-channel (sum g', sum g' xhat), and the BN backward is left with
    one elementwise pass -- no separate reduction pass re-reading the gradient and the BN
    input.  ``fused`` keeps a reference to the masked gradient, which also stops autograd
    from accumulating another consumer's gradient into that buffer in place; the BN
    backward uses the fused result only if it receives exactly that buffer."""

    __slots__ = ("tensors", "act", "slope", "fused")

    def __init__(self, act: int, slope: float = 0.0):
        # leaky ReLU (act 2): the conv returns the RAW gradient and only its sums are masked, so
        # the BN backward re-applies act' and another consumer's gradient can still be added
        self.tensors, self.act, self.slope, self.fused = None, act, float(slope), None

    def release(self):
        self.tensors = self.fused = None


_FUSE_BN_BWD = [os.environ.get("DCP_BN_FUSE", "masked") != "none"]


# Leaky-ReLU BNs through the fused dgrad epilogue: measured a net loss on TResNet-M at b1024
# (the EPI-3 dgrads grew by 2.1 ms/step, the reduction passes they replace took 1.5 ms), so off
# by default; kept selectable for A/B runs and tested.
_FUSE_LEAKY = [False]
# The dgrad-epilogue BN fusion is used for BN + residual + ReLU layers (activation mask bits,
# EPI 4).  For the plain BN + ReLU layers (mask recomputed from the BN input, EPI 3) it depends on
# the layer size: on large activations the separate reduction pass measured as fast or faster
# (ResNet-50 b1024: 14,240 vs 14,170 img/s in round 2, 14,099 vs 14,079 in round 3), on small ones
# the fusion saves a launch-bound reduction + partial-sum pair per layer (b32 graph 4,392 -> 4,592,
# b128 9,742 -> 9,933 img/s; profiles/r3/bn_fuse_ab_batch.txt).  Default ("auto"): fuse plain
# layers whose activation has at most _PLAIN_FUSE_MAX elements (every layer at batch <= 128, stage 4
# at 1024); DCP_BN_FUSE=all fuses every plain layer, =masked none of them.
_BN_FUSE_MODE = os.environ.get("DCP_BN_FUSE", "auto")
_FUSE_PLAIN = [_BN_FUSE_MODE == "all"]
_PLAIN_FUSE_MAX = [0 if _BN_FUSE_MODE == "masked" else int(os.environ.get("DCP_BN_FUSE_PLAIN_MAX", str(1 << 25)))]


def set_plain_bn_backward_fusion(enabled: bool, max_elems: "int | None" = None):
    """Fuse every plain BN + ReLU backward reduction (True) or apply the size rule (False) with
    threshold ``max_elems`` (unchanged when None; 0 = never)."""
    _FUSE_PLAIN[0] = bool(enabled)
    if max_elems is not None:
        _PLAIN_FUSE_MAX[0] = int(max_elems)


def set_leaky_bn_backward_fusion(enabled: bool):
    _FUSE_LEAKY[0] = bool(enabled)


_FUSE_SHORTCUT_BN = [True]


def set_shortcut_bn_fusion(enabled: bool):
    """Toggle normalising projection shortcuts inside the block's last BN pass (A/B, tests)."""
    _FUSE_SHORTCUT_BN[0] = bool(enabled)


def shortcut_bn_fusion() -> bool:
    return _FUSE_SHORTCUT_BN[0]


def set_bn_backward_fusion(enabled: bool):
    """Toggle the dgrad-epilogue BN backward (A/B tests; default on)."""
    _FUSE_BN_BWD[0] = bool(enabled)


def bn_source(x):
    return getattr(x, "_dcp_bnsrc", None)


# ----------------------------------------------------------------------------- wgrad stream
# A conv's weight gradient does not feed the rest of the backward pass, only the optimizer (and
# the DDP buckets): with DCP_WGRAD_STREAM=1 it runs on a second HIP stream beside the data
# gradient, so the two kernels fill each other's tail waves (a 128-row conv grid is 3-7 rounds
# of 256 CUs; the last round runs part-empty).  The main stream joins the side stream before the
# backward function returns (the gradient is complete when autograd / the DDP hook sees it).
_WGRAD_STREAM = [os.environ.get("DCP_WGRAD_STREAM", "0") == "1"]
_SIDE = {}


def set_wgrad_stream(enabled: bool):
    _WGRAD_STREAM[0] = bool(enabled)


def _side_stream(device) -> "torch.cuda.Stream":
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device=device)
    return s


class _WgradOnSide:
    """``with _WgradOnSide(t) as side: dw = ...`` runs the body on the side stream (forked from
    the current stream); ``side.join()`` makes the current stream wait for it.  A no-op on the
    CPU or when the option is off."""

    def __init__(self, t: torch.Tensor):
        self.on = _WGRAD_STREAM[0] and t.is_cuda
        self.main = torch.cuda.current_stream(t.device) if self.on else None
        self.side = _side_stream(t.device) if self.on else None
        self._ctx = None

    def __enter__(self):
        if self.on:
            self.side.wait_stream(self.main)
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self._ctx is not None:
            self._ctx.__exit__(*exc)
            self._ctx = None
        return False

    def join(self):
        if self.on:
            self.main.wait_stream(self.side)


class _Conv2d(Function):
    @staticmethod
    def forward(ctx, x, weight, wb, wt, stride, pad, stats, link, bnsrc, deposit):
        y, slabs = K(x).conv_fwd(x, wb, stride, pad, stats)
        ctx.save_for_backward(x, wt)
        ctx.geo = (weight.shape[1], weight.shape[2], stride, pad)
        ctx.link, ctx.bnsrc, ctx.deposit = link, bnsrc, deposit
        ctx.mark_non_differentiable(slabs)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics slabs
        return y, slabs

    @staticmethod
    def backward(ctx, dy, _dslabs):
        if dy is None:
            return (None,) * 10
        x, wt = ctx.saved_tensors
        KH, KW, stride, pad = ctx.geo
        dy = dy.contiguous()
        k = K(dy)
        add, complete = None, True
        src = ctx.bnsrc
        fuse = (ctx.needs_input_grad[0] and src is not None and stride == 1 and src.tensors is not None)
        if ctx.link is not None:
            # a compact stride-2 deposit is added by the fused BN-backward epilogue itself
            add, complete = ctx.link.claim(strided_ok=fuse)
            if isinstance(add, StridedGrad) and not complete:
                add = add.full()
            if add is not None and not isinstance(add, StridedGrad):
                add = add.contiguous()
        dx = dw = None
        side = _WgradOnSide(dy)
        if ctx.needs_input_grad[1] and side.on:
            with side:
                dw = k.conv_wgrad(dy, x, KH, KW, stride, pad)
        if ctx.needs_input_grad[0]:
            if fuse and complete:
                y, res, scale, shift, mean, invstd, mask = src.tensors
                if mask is not None:
                    res = None  # the activation mask bits replace the residual read
                a = add.compact.contiguous() if isinstance(add, StridedGrad) else add
                dx, sums = k.conv_dgrad_bn(dy, wt, pad, a, y, res, scale, shift, mean, invstd, src.act, mask,
                                           src.slope)
                src.fused = (dx, sums)
            else:
                if isinstance(add, StridedGrad):
                    add = add.full()
                if (ctx.deposit is not None and stride == 2 and KH == 1 and KW == 1 and pad == 0
                        and _STRIDED_DEPOSIT[0]):
                    # projection downsample: the compact subgrid gradient (a stride-1 1x1 GEMM over
                    # dY's grid), added on the subgrid by the block's first conv (StridedGrad)
                    dx = StridedGrad(k.conv_dgrad(dy, wt, dy.shape[1], dy.shape[2], 1, 0), x.shape[1], x.shape[2])
                elif add is not None:
                    dx = k.conv_dgrad(dy, wt, x.shape[1], x.shape[2], stride, pad, add)
                else:
                    dx = k.conv_dgrad(dy, wt, x.shape[1], x.shape[2], stride, pad)
            if ctx.deposit is not None:
                dx = ctx.deposit.deposit(dx)
            if isinstance(dx, StridedGrad):  # handed back to autograd: materialise
                dx = dx.full()
        if ctx.needs_input_grad[1] and not side.on:
            dw = k.conv_wgrad(dy, x, KH, KW, stride, pad)
        side.join()
        ctx.link = ctx.bnsrc = ctx.deposit = None
        return dx, dw, None, None, None, None, None, None, None, None


def conv2d(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, pad: int = 0, stats: bool = False,
           link: "GradJoin | None" = None, deposit: "GradJoin | None" = None):
    """NHWC conv; returns (y, bn_stat_slabs).  weight: fp32 [Co,KH,KW,Ci].

    `link`: the block's GradJoin when this conv is the primary consumer of the block input
    (its dgrad epilogue adds the other consumers' gradient); `deposit`: the GradJoin this
    conv's input gradient is handed to (secondary consumer, e.g. a downsample conv).
    A stride-1 conv whose input carries a BNSource fuses that BN's backward reduction."""
    bnsrc = bn_source(x) if (stride == 1 and deposit is None and _FUSE_BN_BWD[0]) else None
    if weight.shape[3] != x.shape[3]:  # stem: input channels zero-padded to a multiple of 8
        wb, wt = prepared_weight(weight, 0, True, ci=x.shape[3])
        weight = F.pad(weight, (0, x.shape[3] - weight.shape[3]))  # autograd view for the padded dW
        return _Conv2d.apply(x, weight, wb, wt, stride, pad, stats, link, None, deposit)
    wb, wt = prepared_weight(weight, 0, True)
    return _Conv2d.apply(x, weight, wb, wt, stride, pad, stats, link, bnsrc, deposit)


class _GroupedConv2d(Function):
    @staticmethod
    def forward(ctx, x, weight, wb, groups, stride, pad, stats, bnsrc):
        if stats:  # BN partials of the output from the MFMA epilogue (empty: BN computes them)
            y, part = K(x).grouped_conv_fwd_stats(x, wb, groups, stride, pad)
        else:
            y, part = K(x).grouped_conv_fwd(x, wb, groups, stride, pad), x.new_empty(0, dtype=torch.float32)
        ctx.save_for_backward(x, wb)
        ctx.geo = (weight.shape[1], weight.shape[2], groups, stride, pad)
        ctx.bnsrc = bnsrc
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:
            return (None,) * 8
        x, wb = ctx.saved_tensors
        KH, KW, groups, stride, pad = ctx.geo
        dy = dy.contiguous()
        k = K(dy)
        dx = dw = None
        side = _WgradOnSide(dy)
        if ctx.needs_input_grad[1] and side.on:
            with side:
                dw = k.grouped_conv_wgrad(dy, x, KH, KW, groups, stride, pad)
        if ctx.needs_input_grad[0]:
            src = ctx.bnsrc
            if src is not None and src.act == 1 and src.tensors is not None and src.tensors[1] is None:
                # the input came from a ReLU BN without residual: fuse its backward reduction
                z, _, scale, shift, mean, invstd, _ = src.tensors
                dx, sums = k.grouped_conv_dgrad_bn(dy, wb, x.shape[1], x.shape[2], groups, stride, pad, z, scale,
                                                   shift, mean, invstd)
                if sums.numel() > 0:
                    src.fused = (dx, sums)
            else:
                dx = k.grouped_conv_dgrad(dy, wb, x.shape[1], x.shape[2], groups, stride, pad)
        if ctx.needs_input_grad[1] and not side.on:
            dw = k.grouped_conv_wgrad(dy, x, KH, KW, groups, stride, pad)
        side.join()
        ctx.bnsrc = None
        return dx, dw, None, None, None, None, None, None


def grouped_conv2d(x, weight, groups, stride=1, pad=0, stats=False):
    """Grouped NHWC conv -> y, or (y, BN partials or None) with ``stats=True`` (GPU: the partials
    come from the MFMA kernel's epilogue, so the following BN reads no extra pass over y)."""
    if groups == 1:
        y, slabs = conv2d(x, weight, stride, pad, stats and x.is_cuda)
        return (y, slabs if stats and x.is_cuda else None) if stats else y
    wb, _ = prepared_weight(weight, 0, False)
    bnsrc = bn_source(x) if (stride == 1 and _FUSE_BN_BWD[0]) else None
    y, part = _GroupedConv2d.apply(x, weight, wb, groups, stride, pad, bool(stats and x.is_cuda), bnsrc)
    if not stats:
        return y
    return y, (part if part.numel() > 0 else None)


# ----------------------------------------------------------------------------- linear
class _Linear(Function):
    @staticmethod
    def forward(ctx, x, weight, bias_p, wb, wt, act):
        y = K(x).linear_fwd(x, wb, bias_p, act)
        ctx.save_for_backward(x, wt, y if act else None)
        ctx.act = act
        ctx.out = weight.shape[0]
        ctx.has_bias = bias_p is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt, y = ctx.saved_tensors
        dy = dy.contiguous()
        k = K(dy)
        if ctx.act:
            dy = k.act_bwd(dy, y, ctx.act)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = k.linear_fwd(dy, wt, None, 0)
        if ctx.needs_input_grad[1]:
            dw = k.linear_wgrad(dy, x)[: ctx.out]
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = k.colsum(dy)[: ctx.out]  # the padded GEMM's column sums, the real outputs only
        return dx, dw, db, None, None, None


def linear(x, weight, bias=None, relu=False, keep_padded=False, act=None):
    """y = act(x W^T + b), act in {None/'none', 'relu', 'sigmoid'} (``relu=True`` = 'relu').
    Output features are padded to a multiple of 64 for the GEMM; the returned
    tensor is the [B, out] view unless ``keep_padded``."""
    act_code = {None: 0, "none": 0, "relu": 1, "sigmoid": 2}[act] if act is not None else (1 if relu else 0)
    out, inf = weight.shape
    x = x.contiguous()
    if x.shape[1] != inf:
        raise ValueError(f"linear: input width {x.shape[1]} != {inf}")
    npad = round_up(out, 64) if x.is_cuda else out
    wb, wt = prepared_weight(weight, npad, True)
    # the bias goes in unpadded: the GEMM epilogue adds 0 past its length (no per-step pad copy)
    y = _Linear.apply(x, weight, bias, wb, wt, act_code)
    return y if keep_padded or npad == out else y[:, :out]


# ----------------------------------------------------------------------------- batch norm (+act, +residual)
class BNConfig:
    __slots__ = ("training_stats", "momentum", "eps", "act", "slope", "group", "world", "iabn", "rgamma", "iabn_eps")

    def __init__(self, training_stats, momentum, eps, act, slope, group, world, iabn=False, rgamma=None,
                 iabn_eps=None):
        self.training_stats = training_stats
        self.momentum = momentum
        self.eps = eps
        self.act = act
        self.slope = slope
        self.group = group
        self.world = world
        self.iabn = iabn  # InplaceABN: backward from the output (see _BNAct)
        self.rgamma = rgamma  # InplaceABN: 1 / gamma, when the caller has it (iabn_gamma)
        # InplaceABN with the RAW weight (iabn_eps set): the BN finalize applies |g| + iabn_eps and writes
        # 1 / it into rgamma, the backward's elementwise pass returns the raw weight's gradient -- no
        # iabn_gamma / sign_mul launches per layer
        self.iabn_eps = iabn_eps


def _bn_train_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg: BNConfig):
    """Training-mode BN coefficients -> (mean, invstd, scale, shift, count).  Local BN runs the
    statistics and the finalize as one launch pair; SyncBN all-gathers the per-rank
    (n, mean, M2) between them."""
    count = x.numel() // x.shape[-1]
    ieps = -1.0 if cfg.iabn_eps is None else float(cfg.iabn_eps)
    rg = cfg.rgamma if cfg.iabn_eps is not None else None
    if cfg.group is None:
        return (*k.bn_stats_finalize(x, slabs, gamma, beta, run_mean, run_var, cfg.momentum, cfg.eps, ieps, rg), count)
    st = k.bn_stats(x, slabs)  # [1,3,C] (n, mean, M2)
    gathered = st.new_empty((cfg.world,) + tuple(st.shape[1:]))
    _peer.all_gather_into_tensor(gathered, st, cfg.group)
    _check_equal_counts(gathered, count)
    # the forward merge is exact for any counts; the backward normaliser assumes equal per-rank
    # batches (the sharded sampler pads every rank to the same length; parallel/ddp.py)
    count = count * cfg.world
    return (*k.bn_finalize(gathered, gamma, beta, run_mean, run_var, cfg.momentum, cfg.eps, ieps, rg), count)


# torch's SyncBatchNorm synchronises only when the group has more than one rank
# (torch/nn/modules/batchnorm.py: need_sync = world_size > 1) -- the reference's SyncBN
# (BASELINE/main.py:148) at world 1 is plain batch norm.  DCP_SYNCBN_WORLD1=1 keeps the collectives
# at world 1 anyway (tests and probes that exercise the SyncBN transport on one GPU).
_SYNCBN_WORLD1 = [os.environ.get("DCP_SYNCBN_WORLD1", "0") == "1"]


def set_syncbn_world1(enabled: bool):
    _SYNCBN_WORLD1[0] = bool(enabled)


# local training BN: statistics finalize + apply in one launch (bn_fin_act, DCP_BN_FIN_ACT=1), bit-identical
# to the two launches.  Opt-in: its in-kernel wait for the finalize workgroups measured slower than the
# kernel boundary it replaces (R50 b32 graph 5,167 vs 5,273 img/s, profiles/r6/bn_fin_act_ab_s19_s20.txt)
_FIN_ACT = [os.environ.get("DCP_BN_FIN_ACT", "0") == "1"]


def set_bn_fin_act(enabled: bool):
    _FIN_ACT[0] = bool(enabled)


def _sync_group(group):
    """(group, world) for a BN's statistics: (None, 1) when there is nothing to synchronise."""
    if group is None:
        return None, 1
    world = dist.get_world_size(group)
    if world == 1 and not _SYNCBN_WORLD1[0]:
        return None, 1
    return group, world


_SYNCBN_CHECK = [os.environ.get("DCP_SYNCBN_CHECK", "0") == "1"]


def _check_equal_counts(gathered, count):
    """DCP_SYNCBN_CHECK=1: every rank's gathered count must equal this rank's (a host sync)."""
    if _SYNCBN_CHECK[0]:
        n = gathered[:, 0, 0].float().cpu()
        if not bool((n == float(count)).all()):
            raise RuntimeError(f"SyncBN: unequal per-rank batch counts {n.tolist()} (the backward assumes equal "
                               "counts; pad the shards to equal length)")


class _BNAct(Function):
    @staticmethod
    def forward(ctx, x, slabs, gamma, beta, res, run_mean, run_var, cfg: BNConfig, link, src):
        k = K(x)
        C = x.shape[-1]
        count = x.numel() // C
        # BN + residual + ReLU feeding a fused-backward conv: keep the ReLU mask as bits so that
        # backward reads 1/16 of the residual's bytes for it
        want_mask = src is not None and res is not None and cfg.act == 1
        mask = None
        if cfg.training_stats and cfg.group is None and _FIN_ACT[0]:
            # local BN from the producing conv's statistics: finalize + apply as ONE launch (without
            # slabs the op falls back to the statistics pass + apply)
            ieps = -1.0 if cfg.iabn_eps is None else float(cfg.iabn_eps)
            rg = cfg.rgamma if cfg.iabn_eps is not None else None
            st = slabs if slabs is not None else x.new_empty(0, dtype=torch.float32)
            y, mask, mean, invstd, scale, shift = k.bn_fin_act(x, st, res, gamma, beta, run_mean, run_var,
                                                               cfg.momentum, cfg.eps, cfg.act, cfg.slope, want_mask,
                                                               ieps, rg)
            if not want_mask:
                mask = None
        else:
            if cfg.training_stats:
                mean, invstd, scale, shift, count = _bn_train_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg)
            else:
                mean, invstd, scale, shift = k.bn_eval_coeff(gamma, beta, run_mean, run_var, cfg.eps)
            if want_mask:
                y, mask = k.bn_act_mask(x, res, scale, shift, cfg.act, cfg.slope)
            else:
                y = k.bn_act(x, res, scale, shift, cfg.act, cfg.slope)
        if cfg.iabn:
            # InplaceABN (mapillary inplace_abn, X3/K21): keep only the output.  The BN input x is
            # not saved (the consumer conv saves y anyway), so one activation per layer is freed;
            # backward recovers z = act^-1(y) and xhat = (z - beta) / gamma in registers.
            ctx.save_for_backward(y, None, gamma, scale, shift, beta, invstd)
        else:
            ctx.save_for_backward(x, res, gamma, scale, shift, mean, invstd)
        ctx.cfg = cfg
        ctx.count = count
        ctx.has_res = res is not None
        ctx.link = link
        ctx.src = src
        if src is not None:
            src.tensors = (x, res, scale, shift, mean, invstd, mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, res, gamma, scale, shift, mean, invstd = ctx.saved_tensors
        cfg = ctx.cfg
        dy = dy.contiguous()
        k = K(dy)
        src, ctx.src = ctx.src, None
        fused = src.fused if src is not None else None
        if src is not None:
            src.release()
        want_dres = ctx.has_res and ctx.needs_input_grad[4]
        if cfg.iabn:
            y, beta = x, mean  # saved (y, beta) in place of (x, mean)
            rgamma = cfg.rgamma if cfg.rgamma is not None else torch.reciprocal(gamma.detach().float())
            need_affine = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
            local = sums = None
            if cfg.training_stats or need_affine:
                local = k.bn_bwd_reduce(dy, y, None, scale, shift, beta.detach().float(), rgamma, cfg.act, cfg.slope,
                                        True)
                sums = local
                if cfg.training_stats and cfg.group is not None:
                    sums = local.clone()
                    _peer.all_reduce(sums, cfg.group)
            raw = cfg.iabn_eps is not None  # gamma is the RAW weight: its gradient carries sign(g)
            fold = raw and cfg.training_stats and sums is local and ctx.needs_input_grad[2]
            dx, dg = k.bn_bwd_elemt(dy, y, None, scale, shift, beta.detach().float(), rgamma,
                                    sums if cfg.training_stats else None, float(ctx.count), cfg.act, cfg.slope, False,
                                    True, gamma.detach().float() if fold else None)
            dgamma = None
            if local is not None and ctx.needs_input_grad[2]:
                if fold:
                    dgamma = dg
                elif raw:
                    dgamma = k.sign_mul(local[1].contiguous(), gamma.detach().float())
                else:
                    dgamma = local[1]
            dbeta = local[0] if (local is not None and ctx.needs_input_grad[3]) else None
            return dx, None, dgamma, dbeta, None, None, None, None, None, None
        if fused is not None and fused[0].data_ptr() == dy.data_ptr() and fused[0].shape == dy.shape:
            # the consuming conv's dgrad epilogue already masked the gradient and reduced it
            g, local = fused
            sums = local
            if cfg.group is not None:
                sums = local.clone()
                _peer.all_reduce(sums, cfg.group)
            # ReLU / identity: g is already masked; leaky: g is raw and the elementwise pass applies act'
            post_act = cfg.act if cfg.act == 2 else 0
            dx, _ = k.bn_bwd_elemt(g, x, None, scale, shift, mean, invstd, sums, float(ctx.count), post_act,
                                   cfg.slope, False)
            dres = g if want_dres else None
        else:
            need_affine = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
            sums = None
            local = None
            if cfg.training_stats or need_affine:
                local = k.bn_bwd_reduce(dy, x, res, scale, shift, mean, invstd, cfg.act, cfg.slope)
                sums = local
                if cfg.training_stats and cfg.group is not None:
                    sums = local.clone()
                    _peer.all_reduce(sums, cfg.group)
            dx, dres = k.bn_bwd_elemt(dy, x, res, scale, shift, mean, invstd, sums if cfg.training_stats else None,
                                      float(ctx.count), cfg.act, cfg.slope, want_dres)
            if not want_dres:
                dres = None
        dgamma = local[1] if (local is not None and ctx.needs_input_grad[2]) else None
        dbeta = local[0] if (local is not None and ctx.needs_input_grad[3]) else None
        if dres is not None and ctx.link is not None:
            dres = ctx.link.deposit(dres)  # summed into the block input gradient by the first conv's dgrad
        ctx.link = None
        return dx, None, dgamma, dbeta, dres, None, None, None, None, None


# ----------------------------------------------------------------------------- BN + ReLU as a conv prologue
# A training-mode BN + ReLU whose only consumer is a 1x1 stride-1 conv (a bottleneck's bn2 ->
# conv3) can be applied inside that conv: the forward tap GEMM normalises its A fragments in
# registers, the weight-gradient GEMM its B fragments.  The activation
# relu(bn(x)) is then never written nor kept for backward (ResNet-50 b1024: 2.8 GB less
# activation memory).  Off by default because it measured slower on MI355X: every column tile of
# the GEMM (Co / 128 of them, up to 16) and every wave sharing a fragment re-applies the
# transform, which costs more VALU time than the 0.9 ms/step BN-apply pass it removes
# (profiles/r3/bn_prologue_ab_b1024.txt: conv3 fwd + wgrad 7.61 -> 9.34 ms/step against
# 0.92 ms of BN-apply saved; headline 14,222 -> 14,090 img/s).  DCP_BN_PROLOGUE=1 /
# set_bn_prologue(True) turns it on (memory-bound runs, A/B).
_BN_PROLOGUE = [os.environ.get("DCP_BN_PROLOGUE", "0") == "1"]


def set_bn_prologue(enabled: bool):
    _BN_PROLOGUE[0] = bool(enabled)


def bn_prologue_enabled() -> bool:
    return _BN_PROLOGUE[0]


def bn_prologue_fits(C: int, Co: int) -> bool:
    """Channel layouts the prologue kernels take: C % 64 == 0 (one tap per 64-deep k-tile),
    C <= 2048 (the LDS table), and not the narrow Co <= 64 / C >= 128 weight-gradient tile."""
    return C % 64 == 0 and Co % 8 == 0 and C <= 2048 and not (Co <= 64 and C >= 128)


class _BNReluConv(Function):
    """y = conv(relu(BN(x))) with the BN + ReLU applied to the conv's operands on the fly: a 1x1
    stride-1 conv (in registers between the LDS fragment read and the MFMA, K5) or the 64 -> 64
    channel 3x3 stride-1 conv of the direct kernels (once per staged window element -- each feeds
    nine taps -- in conv3x3_c64 and wgrad3x3).

    Forward: the BN coefficients from x's producer statistics (SyncBN: the all-gather), then
    ``conv_fwd_pro`` / ``conv3x3_fwd_pro`` (and the statistics of y for the next BN).  Backward: the
    conv's dgrad gives the gradient of relu(BN(x)); the weight gradient recomputes relu(BN(x))
    from x; the BN + ReLU backward runs from x as in :class:`_BNAct`.  The normalised activation
    is never written."""

    @staticmethod
    def forward(ctx, x, slabs, gamma, beta, run_mean, run_var, cfg: BNConfig, weight, wb, wt, stats, k3):
        k = K(x)
        if cfg.training_stats:
            mean, invstd, scale, shift, count = _bn_train_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg)
        else:
            mean, invstd, scale, shift = k.bn_eval_coeff(gamma, beta, run_mean, run_var, cfg.eps)
            count = x.numel() // x.shape[-1]
        if k3:
            y, yslabs = k.conv3x3_fwd_pro(x, wb, scale, shift, stats)
        else:
            y, yslabs = k.conv_fwd_pro(x, wb, scale, shift, stats)
        ctx.save_for_backward(x, scale, shift, mean, invstd, wt)
        ctx.cfg, ctx.count, ctx.k3 = cfg, count, k3
        ctx.mark_non_differentiable(yslabs)
        ctx.set_materialize_grads(False)
        return y, yslabs

    @staticmethod
    def backward(ctx, dy, _dslabs):
        if dy is None:
            return (None,) * 12
        x, scale, shift, mean, invstd, wt = ctx.saved_tensors
        cfg = ctx.cfg
        dy = dy.contiguous()
        k = K(dy)
        dx = dgamma = dbeta = dw = None
        need_x = ctx.needs_input_grad[0] or ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        pad = 1 if ctx.k3 else 0
        g = k.conv_dgrad(dy, wt, x.shape[1], x.shape[2], 1, pad) if need_x else None
        if ctx.needs_input_grad[7]:
            dw = k.conv3x3_wgrad_pro(dy, x, scale, shift) if ctx.k3 else k.conv_wgrad_pro(dy, x, scale, shift)
        if g is not None:
            need_affine = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
            local = sums = None
            if cfg.training_stats or need_affine:
                local = k.bn_bwd_reduce(g, x, None, scale, shift, mean, invstd, 1, 0.0)
                sums = local
                if cfg.training_stats and cfg.group is not None:
                    sums = local.clone()
                    _peer.all_reduce(sums, cfg.group)
            dx, _ = k.bn_bwd_elemt(g, x, None, scale, shift, mean, invstd, sums if cfg.training_stats else None,
                                   float(ctx.count), 1, 0.0, False)
            dgamma = local[1] if (local is not None and ctx.needs_input_grad[2]) else None
            dbeta = local[0] if (local is not None and ctx.needs_input_grad[3]) else None
        return dx, None, dgamma, dbeta, None, None, None, dw, None, None, None, None


_BNReluConv1x1 = _BNReluConv


def _bn_relu_conv(x, slabs, gamma, beta, run_mean, run_var, training_stats, momentum, eps, weight, stats, group, k3):
    group, world = _sync_group(group)
    cfg = BNConfig(training_stats, momentum, eps, 1, 0.0, group, world)
    if slabs is not None and slabs.numel() == 0:
        slabs = None
    wb, wt = prepared_weight(weight, 0, True)
    want = bool(stats and x.is_cuda)
    y, yslabs = _BNReluConv.apply(x, slabs, gamma, beta, run_mean, run_var, cfg, weight, wb, wt, want, k3)
    return y, (yslabs if want else None)


def bn_relu_conv1x1(x, slabs, gamma, beta, run_mean, run_var, training_stats, momentum, eps, weight, stats=False,
                    group=None):
    """conv1x1(relu(BN(x))) through :class:`_BNReluConv` -> (y, statistics slabs of y or None).
    weight: fp32 [Co, 1, 1, C]."""
    return _bn_relu_conv(x, slabs, gamma, beta, run_mean, run_var, training_stats, momentum, eps, weight, stats,
                         group, False)


def bn_relu_conv3x3(x, slabs, gamma, beta, run_mean, run_var, training_stats, momentum, eps, weight, stats=False,
                    group=None):
    """conv3x3 / stride 1 / pad 1 (relu(BN(x))) for 64 -> 64 channels through the direct kernels'
    window prologue -> (y, statistics partials of y or None).  weight: fp32 [Co, 3, 3, C]."""
    return _bn_relu_conv(x, slabs, gamma, beta, run_mean, run_var, training_stats, momentum, eps, weight, stats,
                         group, True)


# BN + ReLU inside a 64 -> 64 channel 3x3 consumer's staged window (bn_relu_conv3x3): on by default
# (DCP_BN_PROLOGUE3=0 / set_bn_prologue3x3(False) off, A/B)
_BN_PROLOGUE3 = [os.environ.get("DCP_BN_PROLOGUE3", "1") != "0"]


def set_bn_prologue3x3(enabled: bool):
    _BN_PROLOGUE3[0] = bool(enabled)


def bn_prologue3x3_enabled() -> bool:
    return _BN_PROLOGUE3[0]


def bn_prologue3x3_fits(x, C: int, Co: int) -> bool:
    return bool(K(x).conv3x3_pro_fits(x.shape[0], x.shape[1], x.shape[2], C, Co))


def _bn_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg: BNConfig):
    if cfg.training_stats:
        return _bn_train_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg)
    return (*k.bn_eval_coeff(gamma, beta, run_mean, run_var, cfg.eps), x.numel() // x.shape[-1])


def _bn_backward(k, g, x, scale, shift, mean, invstd, count, cfg: BNConfig, need_affine):
    """Input gradient (and local [dbeta, dgamma] sums) of a BN layer whose output gradient after
    the activation is ``g``."""
    local = sums = None
    if cfg.training_stats or need_affine:
        local = k.bn_bwd_reduce(g, x, None, scale, shift, mean, invstd, 0, cfg.slope)
        sums = local
        if cfg.training_stats and cfg.group is not None:
            sums = local.clone()
            _peer.all_reduce(sums, cfg.group)
    dx, _ = k.bn_bwd_elemt(g, x, None, scale, shift, mean, invstd, sums if cfg.training_stats else None,
                           float(count), 0, cfg.slope, False)
    return dx, local


class _BNAddBNAct(Function):
    """act(BN(x) + BN_r(r)): a bottleneck's last BN fused with its projection shortcut's BN
    (the ``downsample`` conv output ``r`` is normalised while it is read as the residual, so the
    shortcut BN never writes an activation).  Backward: the masked gradient
    ``g`` feeds both BN backwards (the main one through the consuming conv's fused dgrad epilogue
    when available)."""

    @staticmethod
    def forward(ctx, x, slabs, gamma, beta, run_mean, run_var, r, rslabs, rgamma, rbeta, rrun_mean, rrun_var,
                cfg: BNConfig, rcfg: BNConfig, src):
        k = K(x)
        if cfg.training_stats and rcfg.training_stats and cfg.group is not None and rcfg.group is cfg.group:
            # SyncBN: both layers' (n, mean, M2) in ONE all-gather (one small-message latency, not two)
            C = x.shape[-1]
            st = torch.cat([k.bn_stats(x, slabs), k.bn_stats(r, rslabs)], dim=2)
            gathered = st.new_empty((cfg.world,) + tuple(st.shape[1:]))
            _peer.all_gather_into_tensor(gathered, st, cfg.group)
            _check_equal_counts(gathered, x.numel() // C)
            count = rcount = (x.numel() // C) * cfg.world
            mean, invstd, scale, shift = k.bn_finalize(gathered[..., :C].contiguous(), gamma, beta, run_mean, run_var,
                                                       cfg.momentum, cfg.eps)
            rmean, rinvstd, rscale, rshift = k.bn_finalize(gathered[..., C:].contiguous(), rgamma, rbeta, rrun_mean,
                                                           rrun_var, rcfg.momentum, rcfg.eps)
        else:
            mean, invstd, scale, shift, count = _bn_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg)
            rmean, rinvstd, rscale, rshift, rcount = _bn_coeff(k, r, rslabs, rgamma, rbeta, rrun_mean, rrun_var,
                                                               rcfg)
        y, mask = k.bn2_act_mask(x, r, scale, shift, rscale, rshift, cfg.act, cfg.slope)
        ctx.save_for_backward(x, r, scale, shift, mean, invstd, rscale, rshift, rmean, rinvstd, mask)
        ctx.cfg, ctx.rcfg, ctx.count, ctx.rcount = cfg, rcfg, count, rcount
        ctx.src = src
        if src is not None:
            # the consuming conv masks the gradient with the bits; the residual is never read there
            src.tensors = (x, None, scale, shift, mean, invstd, mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, r, scale, shift, mean, invstd, rscale, rshift, rmean, rinvstd, mask = ctx.saved_tensors
        cfg, rcfg = ctx.cfg, ctx.rcfg
        dy = dy.contiguous()
        k = K(dy)
        src, ctx.src = ctx.src, None
        fused = src.fused if src is not None else None
        if src is not None:
            src.release()
        nig = ctx.needs_input_grad
        if fused is not None and fused[0].data_ptr() == dy.data_ptr() and fused[0].shape == dy.shape:
            g, local = fused
            if rcfg.training_stats and ctx.rcount == ctx.count and rcfg.group is cfg.group:
                # both input gradients in one pass over g (the shortcut BN's sums first); SyncBN
                # reduces both layers' sums in one all-reduce
                rlocal = k.bn_bwd_reduce(g, r, None, rscale, rshift, rmean, rinvstd, 0, rcfg.slope)
                sums, rsums = local, rlocal
                if cfg.group is not None:
                    both = torch.cat([local, rlocal], dim=1)
                    _peer.all_reduce(both, cfg.group)
                    C = local.shape[1]
                    sums, rsums = both[:, :C].contiguous(), both[:, C:].contiguous()
                dx, dr = k.bn2_bwd_elemt(g, x, r, scale, mean, invstd, sums, rscale, rmean, rinvstd, rsums,
                                         float(ctx.count))
                dgamma = local[1] if nig[2] else None
                dbeta = local[0] if nig[3] else None
                rdgamma = rlocal[1] if nig[8] else None
                rdbeta = rlocal[0] if nig[9] else None
                return (dx, None, dgamma, dbeta, None, None, dr if nig[6] else None, None, rdgamma, rdbeta, None,
                        None, None, None, None)
            sums = local
            if cfg.group is not None:
                sums = local.clone()
                _peer.all_reduce(sums, cfg.group)
            dx, _ = k.bn_bwd_elemt(g, x, None, scale, shift, mean, invstd, sums, float(ctx.count), 0, cfg.slope,
                                   False)
        else:
            rv = k.bn_act(r, None, rscale, rshift, 0, 0.0)  # the shortcut activation, recomputed
            need_affine = nig[2] or nig[3]
            local = sums = None
            if cfg.training_stats or need_affine:
                local = k.bn_bwd_reduce(dy, x, rv, scale, shift, mean, invstd, cfg.act, cfg.slope)
                sums = local
                if cfg.training_stats and cfg.group is not None:
                    sums = local.clone()
                    _peer.all_reduce(sums, cfg.group)
            dx, g = k.bn_bwd_elemt(dy, x, rv, scale, shift, mean, invstd, sums if cfg.training_stats else None,
                                   float(ctx.count), cfg.act, cfg.slope, True)
        dr, rlocal = None, None
        if nig[6] or nig[8] or nig[9]:
            dr, rlocal = _bn_backward(k, g, r, rscale, rshift, rmean, rinvstd, ctx.rcount, rcfg, nig[8] or nig[9])
        dgamma = local[1] if (local is not None and nig[2]) else None
        dbeta = local[0] if (local is not None and nig[3]) else None
        rdgamma = rlocal[1] if (rlocal is not None and nig[8]) else None
        rdbeta = rlocal[0] if (rlocal is not None and nig[9]) else None
        return (dx, None, dgamma, dbeta, None, None, dr if nig[6] else None, None, rdgamma, rdbeta, None, None,
                None, None, None)


def batch_norm_add_bn_act(x, slabs, gamma, beta, run_mean, run_var, r, rslabs, rgamma, rbeta, rrun_mean, rrun_var,
                          training_stats, momentum, eps, rmomentum, reps, act="relu", slope=0.01, group=None):
    """act(BN(x) + BN_r(r)) with both BNs in training or eval mode (see :class:`_BNAddBNAct`)."""
    group, world = _sync_group(group)
    cfg = BNConfig(training_stats, momentum, eps, ACT[act], float(slope), group, world)
    rcfg = BNConfig(training_stats, rmomentum, reps, 0, float(slope), group, world)
    slabs = None if slabs is None or slabs.numel() == 0 else slabs
    rslabs = None if rslabs is None or rslabs.numel() == 0 else rslabs
    src = None
    if training_stats and cfg.act in (0, 1) and _FUSE_BN_BWD[0] and torch.is_grad_enabled():
        src = BNSource(cfg.act)
    out = _BNAddBNAct.apply(x, slabs, gamma, beta, run_mean, run_var, r, rslabs, rgamma, rbeta, rrun_mean, rrun_var,
                            cfg, rcfg, src)
    if src is not None:
        out._dcp_bnsrc = src
    return out


class _IABNGamma(Function):
    """InplaceABN's effective weight |gamma| + eps (and its reciprocal for the backward from the
    output) in one launch; gradient d * sign(gamma) in one launch."""

    @staticmethod
    def forward(ctx, g, eps):
        geff, rg = K(g).iabn_gamma(g, eps)
        ctx.save_for_backward(g)
        ctx.mark_non_differentiable(rg)
        return geff, rg

    @staticmethod
    def backward(ctx, dgeff, _drg):
        (g,) = ctx.saved_tensors
        return (K(g).sign_mul(dgeff.contiguous(), g) if dgeff is not None else None), None


def iabn_gamma(g, eps):
    """(|g| + eps, 1 / (|g| + eps)) -- differentiable in g through the first output."""
    return _IABNGamma.apply(g, float(eps))


# Training-mode InplaceABN layers hand the RAW weight to batch_norm_act (iabn_eps): the BN finalize
# and the backward's elementwise pass apply |g| + eps and sign(g) (TResNet-M: 36 + 36 launches per
# step fewer).  DCP_IABN_FOLD=0: the separate iabn_gamma / sign_mul launches (A/B).
_IABN_FOLD = [os.environ.get("DCP_IABN_FOLD", "1") != "0"]


def set_iabn_fold(enabled: bool):
    _IABN_FOLD[0] = bool(enabled)


def iabn_fold_enabled() -> bool:
    return _IABN_FOLD[0]


def batch_norm_act(x, slabs, gamma, beta, run_mean, run_var, training_stats, momentum, eps, act="relu",
                   slope=0.01, residual=None, group=None, link=None, iabn=False, fuse_bwd=False, rgamma=None,
                   iabn_eps=None):
    """``iabn``: InplaceABN storage (invertible act: identity / leaky, no residual, a gamma bounded
    away from 0 -- BatchNorm2d passes |gamma| + eps, the inplace_abn convention; with ``iabn_eps``
    (training statistics only) it passes the RAW weight and the kernels apply |gamma| + iabn_eps and
    sign(gamma) themselves).  ``fuse_bwd``: offer this plain BN + ReLU's backward reduction to its
    consumer even under the masked-only default (the consumer is a grouped conv, whose dgrad fusion
    measured a win: ResNeXt)."""
    group, world = _sync_group(group)
    iabn = bool(iabn) and residual is None and ACT[act] in (0, 2) and gamma is not None and beta is not None
    if iabn_eps is not None and not (iabn and training_stats):
        raise ValueError("batch_norm_act: iabn_eps needs an InplaceABN layer with training statistics")
    cfg = BNConfig(training_stats, momentum, eps, ACT[act], float(slope), group, world, iabn, rgamma if iabn else None)
    if iabn_eps is not None:
        cfg.iabn_eps = float(iabn_eps)
        cfg.rgamma = torch.empty(gamma.shape, dtype=torch.float32, device=gamma.device)  # written by the finalize
    if slabs is None or (slabs.numel() == 0):
        slabs = None
    # ReLU / identity only: their masks are idempotent, so a consumer that masked the
    # gradient early composes with any unfused fallback
    src = None
    plain = _FUSE_PLAIN[0] or fuse_bwd or x.numel() <= _PLAIN_FUSE_MAX[0]
    fusable = not iabn and ((cfg.act in (0, 1) and (residual is not None or plain)) or
                            (cfg.act == 2 and residual is None and _FUSE_LEAKY[0]))
    if training_stats and fusable and _FUSE_BN_BWD[0] and torch.is_grad_enabled():
        src = BNSource(cfg.act, cfg.slope)
    out = _BNAct.apply(x, slabs, gamma, beta, residual, run_mean, run_var, cfg, link, src)
    if src is not None:
        out._dcp_bnsrc = src
    return out


# ----------------------------------------------------------------------------- eval-mode BN folded into the conv
_EVAL_COEFF = weakref.WeakKeyDictionary()


def bn_eval_coefficients(bn):
    """(mean, invstd, scale, shift) of a BatchNorm2d's running statistics, cached until any of the
    four source tensors changes (frozen BN recomputes nothing per step; a HIP-graph replay reads the
    same cached tensors).

    On the GPU two writers change those tensors without bumping ``_version``: the BN statistics
    kernels update running_mean / running_var in place, and the fused optimizers update gamma /
    beta through pointer tables.  So the key also carries the weight generation (bumped by every
    optimizer step and state load) and the BN's training-forward count (``_nbt_pending`` grows by
    one per statistics forward and is flushed into ``num_batches_tracked``, whose ``_version`` the
    flush bumps: the pair never repeats)."""
    g, b, rm, rv = bn.weight, bn.bias, bn.running_mean, bn.running_var
    key = tuple((t._version, t.data_ptr()) if t is not None else None for t in (g, b, rm, rv)) + (bn.eps,)
    nbt = getattr(bn, "num_batches_tracked", None)
    trainable = any(t is not None and t.requires_grad for t in (g, b))  # frozen BN: no per-step refresh
    key += (_GEN[0] if trainable else None, getattr(bn, "_nbt_pending", 0), nbt._version if nbt is not None else None)
    hit = _EVAL_COEFF.get(bn)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        gd = g.detach() if g is not None else None
        if gd is not None and getattr(bn, "inplace_abn", False):
            gd = gd.abs() + bn.iabn_eps  # InplaceABN's effective weight
        coeff = K(rm).bn_eval_coeff(gd, b.detach() if b is not None else None, rm, rv, bn.eps)
    _EVAL_COEFF[bn] = (key, coeff)
    return coeff


def bn_foldable(bn) -> bool:
    """A BN that normalises with its running statistics (model.eval(), NESTED's frozen BN) and whose
    affine parameters need no gradient can be folded into the producing conv's epilogue."""
    if bn.training and not bn.frozen:
        return False
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (bn.weight, bn.bias)):
        return False
    return True


class _ConvAffine(Function):
    """y = act(conv(x) * scale + shift [+ res]) with the affine (an eval-mode BN) applied in the
    conv's store epilogue (``conv_fwd_affine``).  Backward from the stored output: one pass
    g = dy * act'(y), dc = g * scale (``act_scale_bwd``), then the conv's dgrad / wgrad of dc."""

    @staticmethod
    def forward(ctx, x, weight, wb, wt, stride, pad, scale, shift, act, slope, res):
        y = K(x).conv_fwd_affine(x, wb, stride, pad, scale, shift, act, slope, res)
        ctx.save_for_backward(x, wt, y, scale)
        ctx.geo = (weight.shape[1], weight.shape[2], stride, pad, act, slope, res is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt, y, scale = ctx.saved_tensors
        KH, KW, stride, pad, act, slope, has_res = ctx.geo
        k = K(dy)
        want_g = has_res and ctx.needs_input_grad[10]
        dc, g = k.act_scale_bwd(dy.contiguous(), y, scale, act, slope, want_g)
        dx = k.conv_dgrad(dc, wt, x.shape[1], x.shape[2], stride, pad) if ctx.needs_input_grad[0] else None
        dw = k.conv_wgrad(dc, x, KH, KW, stride, pad) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None, None, None, None, None, None, None, (g if want_g else None)


def conv_bn_folded(x, weight, stride, pad, bn, act="relu", slope=0.01, residual=None):
    """conv -> eval-mode BN -> (+ residual) -> act as ONE conv launch (see :class:`_ConvAffine`)."""
    _, _, scale, shift = bn_eval_coefficients(bn)
    wb, wt = prepared_weight(weight, 0, True)
    res = residual.contiguous() if residual is not None else None
    return _ConvAffine.apply(x, weight, wb, wt, stride, pad, scale, shift, ACT[act], float(slope), res)


class _BNActPoolEval(Function):
    """Eval-mode BN + ReLU/identity + max pool (the stem tail of a frozen-BN / eval network) in one
    pass (``bn_act_maxpool`` with running-statistics coefficients); backward: the pooled gradient
    scattered, masked and scaled in one pass (``maxpool_bn_bwd_elemt`` with zero batch sums)."""

    @staticmethod
    def forward(ctx, x, scale, shift, mean, invstd, act, pool):
        y, idx = K(x).bn_act_maxpool(x, scale, shift, act, *pool)
        ctx.save_for_backward(x, idx, scale, shift, mean, invstd)
        ctx.act, ctx.pool = act, pool
        ctx.mark_non_differentiable(idx)
        ctx.set_materialize_grads(False)
        return y, idx

    @staticmethod
    def backward(ctx, dy, _didx):
        if dy is None or not ctx.needs_input_grad[0]:
            return (None,) * 7
        x, idx, scale, shift, mean, invstd = ctx.saved_tensors
        zeros = torch.zeros(2, x.shape[-1], dtype=torch.float32, device=x.device)
        dx = K(dy).maxpool_bn_bwd_elemt(dy.contiguous(), idx, x, scale, shift, mean, invstd, ctx.act, zeros, 1.0,
                                        *ctx.pool)
        return dx, None, None, None, None, None, None


def bn_eval_act_maxpool(x, bn, act="relu", k=3, s=2, p=1):
    mean, invstd, scale, shift = bn_eval_coefficients(bn)
    y, _ = _BNActPoolEval.apply(x, scale, shift, mean, invstd, ACT[act], (k, s, p))
    return y


class _BNActPool(Function):
    """Training-mode BN + ReLU/identity + k x k max pool (the ResNet stem tail) without the
    full-resolution activation: forward pools act(bn(x)) on the fly; backward gathers the
    pooled gradient per input pixel and runs the BN reduction and elementwise passes on it."""

    @staticmethod
    def forward(ctx, x, slabs, gamma, beta, run_mean, run_var, cfg: BNConfig, pool):
        k = K(x)
        mean, invstd, scale, shift, count = _bn_train_coeff(k, x, slabs, gamma, beta, run_mean, run_var, cfg)
        y, idx = k.bn_act_maxpool(x, scale, shift, cfg.act, *pool)
        ctx.save_for_backward(x, idx, scale, shift, mean, invstd)
        ctx.cfg, ctx.count, ctx.pool = cfg, count, pool
        ctx.mark_non_differentiable(idx)
        ctx.set_materialize_grads(False)
        return y, idx

    @staticmethod
    def backward(ctx, dy, _didx):
        if dy is None:
            return (None,) * 8
        x, idx, scale, shift, mean, invstd = ctx.saved_tensors
        cfg = ctx.cfg
        dy = dy.contiguous()
        k = K(dy)
        local = k.maxpool_bn_bwd_reduce(dy, idx, x, scale, shift, mean, invstd, cfg.act, *ctx.pool)
        sums = local
        if cfg.group is not None:
            sums = local.clone()
            _peer.all_reduce(sums, cfg.group)
        dx = k.maxpool_bn_bwd_elemt(dy, idx, x, scale, shift, mean, invstd, cfg.act, sums, float(ctx.count),
                                    *ctx.pool)
        dgamma = local[1] if ctx.needs_input_grad[2] else None
        dbeta = local[0] if ctx.needs_input_grad[3] else None
        return dx, None, dgamma, dbeta, None, None, None, None


def batch_norm_act_maxpool(x, slabs, gamma, beta, run_mean, run_var, momentum, eps, act="relu", k=3, s=2, p=1,
                           group=None):
    """Training-mode BN(+act) followed by a max pool, fused (returns the pooled activations)."""
    group, world = _sync_group(group)
    cfg = BNConfig(True, momentum, eps, ACT[act], 0.0, group, world)
    if slabs is None or slabs.numel() == 0:
        slabs = None
    y, _ = _BNActPool.apply(x, slabs, gamma, beta, run_mean, run_var, cfg, (k, s, p))
    return y


# ----------------------------------------------------------------------------- dropout
_DROPOUT_STATE = {}


def _dropout_state(device):
    """(seed, device call counter) per device: the counter is advanced by every dropout launch
    on the device itself, so a replayed HIP graph draws a new mask each replay."""
    key = str(device)
    st = _DROPOUT_STATE.get(key)
    if st is None:
        if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("dropout: first use inside a HIP-graph capture (run an eager step first)")
        st = _DROPOUT_STATE[key] = (int(torch.initial_seed()) & ((1 << 63) - 1),
                                    torch.zeros(1, dtype=torch.int64, device=device))
    return st


class _Dropout(Function):
    @staticmethod
    def forward(ctx, x, p):
        seed, offset = _dropout_state(x.device)
        y, used = K(x).dropout_fwd(x.contiguous(), float(p), seed, offset)
        ctx.save_for_backward(used)
        ctx.p, ctx.seed = float(p), seed
        return y

    @staticmethod
    def backward(ctx, dy):
        (used,) = ctx.saved_tensors
        return K(dy).dropout_bwd(dy, ctx.p, ctx.seed, used), None


def dropout(x, p=0.5, training=True):
    """Inverted dropout on the Philox HIP kernel (the mask is regenerated in backward, not stored);
    SURVEY.md §2.5 K24 (NESTED --dropout, NESTED/train.py:252; VGG classifier)."""
    if not training or p <= 0:
        return x
    return _Dropout.apply(x, p)


# ----------------------------------------------------------------------------- adaptive average pool
class _AdaptiveAvg(Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        ctx.hw = (x.shape[1], x.shape[2])
        return K(x).adaptive_avg_pool(x.contiguous(), oh, ow)

    @staticmethod
    def backward(ctx, dy):
        return K(dy).adaptive_avg_pool_bwd(dy.contiguous(), *ctx.hw), None, None


def adaptive_avg_pool2d(x, oh, ow):
    """NHWC adaptive average pool (torchvision VGG's AdaptiveAvgPool2d((7, 7))); identity when the
    map already has the target size."""
    if x.shape[1] == oh and x.shape[2] == ow:
        return x
    return _AdaptiveAvg.apply(x, oh, ow)


# ----------------------------------------------------------------------------- pooling
class _MaxPool(Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = K(x).maxpool_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geo = (x.shape[1], x.shape[2], k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.geo
        return K(dy).maxpool_bwd(dy.contiguous(), idx, H, W, k, s, p), None, None, None


def max_pool2d(x, k=3, s=2, p=1):
    return _MaxPool.apply(x, k, s, p)


class _GAP(Function):
    @staticmethod
    def forward(ctx, x, link):
        ctx.hw = (x.shape[1], x.shape[2])
        ctx.link = link
        return K(x).gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        add = None
        if ctx.link is not None:
            add, _ = ctx.link.claim()  # the other consumers' gradient, summed in the same pass
            ctx.link = None
            if add is not None:
                add = add.contiguous()
        return K(dy).gap_bwd(dy.contiguous(), *ctx.hw, add), None


def global_avg_pool(x, link: "GradJoin | None" = None):
    """[N,H,W,C] -> [N,C] (torchvision AdaptiveAvgPool2d(1) + flatten).  ``link``: a GradJoin
    whose deposited gradient of ``x`` (e.g. a squeeze-excitation channel scale's) the backward
    adds while broadcasting."""
    return _GAP.apply(x, link)


class _S2D(Function):
    @staticmethod
    def forward(ctx, x, b):
        ctx.b = b
        return K(x).space_to_depth(x, b, False)

    @staticmethod
    def backward(ctx, dy):
        return K(dy).space_to_depth(dy.contiguous(), ctx.b, True), None


def space_to_depth(x, b=4):
    return _S2D.apply(x, b)


class _DWConv(Function):
    @staticmethod
    def forward(ctx, x, filt, k, s, p, reflect, deposit):
        ctx.save_for_backward(filt)
        ctx.geo = (x.shape[1], x.shape[2], k, s, p, reflect)
        ctx.deposit = deposit
        return K(x).dwconv_fwd(x, filt, k, s, p, reflect)

    @staticmethod
    def backward(ctx, dy):
        (filt,) = ctx.saved_tensors
        H, W, k, s, p, reflect = ctx.geo
        dx = K(dy).dwconv_bwd(dy.contiguous(), filt, H, W, k, s, p, reflect)
        if ctx.deposit is not None:
            dx = ctx.deposit.deposit(dx)  # summed by the block's first conv (GradJoin)
        ctx.deposit = None
        return dx, None, None, None, None, None, None


def blur_pool(x, filt, k=3, s=2, p=1, reflect=True, deposit: "GradJoin | None" = None):
    """Fixed depthwise low-pass filter + stride (anti-aliased downsampling).  ``deposit``: hand the
    input gradient to a GradJoin (a TResNet shortcut pool is the block input's second consumer)."""
    return _DWConv.apply(x, filt, k, s, p, reflect, deposit)


class _ChanScale(Function):
    @staticmethod
    def forward(ctx, x, g, res, relu, link, deposit):
        ctx.save_for_backward(x, g, res)
        ctx.relu, ctx.link, ctx.deposit = relu, link, deposit
        return K(x).chan_scale_fwd(x, g, res, relu)

    @staticmethod
    def backward(ctx, dy):
        x, g, res = ctx.saved_tensors
        want_dres = res is not None and ctx.needs_input_grad[2]
        dx, dg, dres = K(dy).chan_scale_bwd(dy.contiguous(), x, g, res, ctx.relu, want_dres)
        dres = dres if want_dres else None
        if dres is not None and ctx.link is not None:
            dres = ctx.link.deposit(dres)  # summed into the block input gradient by the first conv
        if ctx.deposit is not None:
            dx = ctx.deposit.deposit(dx)  # summed by the SE pooling's backward
        ctx.link = ctx.deposit = None
        return dx, dg.to(g.dtype), dres, None, None, None


# squeeze-excitation gate of a small batch as one kernel per direction (se_gate_fwd / se_gate_bwd);
# DCP_SE_FUSED=0 keeps the GEMM chain (two GEMMs forward, ~10 small launches backward)
_SE_FUSED = [os.environ.get("DCP_SE_FUSED", "1") != "0"]
_SE_MAX_N, _SE_MAX_C, _SE_MAX_R = 32, 256, 128  # csrc/extra.hip kSeN / kSeMaxC / kSeMaxR


def set_se_fused(enabled: bool):
    _SE_FUSED[0] = bool(enabled)


class _SEGate(Function):
    @staticmethod
    def forward(ctx, p, w1, b1, w2, b2, w1b, w1t, w2b, w2t):
        h, g = K(p).se_gate_fwd(p, w1b, b1, w2b, b2, w1.shape[0])
        ctx.save_for_backward(p, h, g, w1t, w2t)
        ctx.has_b = (b1 is not None, b2 is not None)
        return g

    @staticmethod
    def backward(ctx, dg):
        p, h, g, w1t, w2t = ctx.saved_tensors
        dp, dw1, db1, dw2, db2 = K(dg).se_gate_bwd(dg.contiguous(), g, h, p, w1t, w2t)
        return (dp, dw1, db1 if ctx.has_b[0] else None, dw2, db2 if ctx.has_b[1] else None, None, None, None, None)


def se_gate_fusable(p, w1, w2) -> bool:
    if not _SE_FUSED[0] or p.dim() != 2:
        return False
    N, C = p.shape
    R = w1.shape[0]
    return (tuple(w1.shape) == (R, C) and tuple(w2.shape) == (C, R) and C % 32 == 0 and R % 32 == 0
            and N <= _SE_MAX_N and C <= _SE_MAX_C and R <= _SE_MAX_R)


def se_gate(p, w1, b1, w2, b2):
    """sigmoid(relu(p W1^T + b1) W2^T + b2) for pooled features p [N, C] (a squeeze-excitation gate,
    TResNet-M's SE blocks, timm ``SEModule``): one kernel forward, one backward, the GEMM chain's bf16
    roundings.  Callers check :func:`se_gate_fusable` (small N: one workgroup)."""
    R, C = w1.shape
    w1b, w1t = prepared_weight(w1, round_up(R, 64) if p.is_cuda else 0, True)
    w2b, w2t = prepared_weight(w2, round_up(C, 64) if p.is_cuda else 0, True)
    return _SEGate.apply(p.contiguous(), w1, b1, w2, b2, w1b, w1t, w2b, w2t)


def channel_scale(x, g, residual=None, relu=False, link: "GradJoin | None" = None,
                  deposit: "GradJoin | None" = None):
    """act(x[n,h,w,c] * g[n,c] (+ residual)) — squeeze-and-excitation apply fused
    with the block's residual add and ReLU.  ``link``: the identity residual's gradient goes to
    the block's GradJoin instead of an autograd add; ``deposit``: likewise for the gradient of
    ``x`` (the SE block's pooling adds it)."""
    return _ChanScale.apply(x, g.contiguous(), residual, bool(relu), link, deposit)


# ----------------------------------------------------------------------------- losses
class _XEnt(Function):
    @staticmethod
    def forward(ctx, logits, labels, C, smoothing, reduction):
        loss_rows, rank = K(logits).xent_fwd(logits, labels, C, smoothing)
        ctx.save_for_backward(logits, labels)
        ctx.C, ctx.smoothing, ctx.reduction = C, smoothing, reduction
        ctx.mark_non_differentiable(rank)
        ctx.set_materialize_grads(False)
        loss = loss_rows.mean() if reduction == "mean" else loss_rows.sum()
        return loss, rank

    @staticmethod
    def backward(ctx, g, _grank):
        if g is None:
            return None, None, None, None, None
        logits, labels = ctx.saved_tensors
        B = logits.shape[0]
        scale = 1.0 / B if ctx.reduction == "mean" else 1.0
        d = K(logits).xent_bwd(logits, labels, ctx.C, g.reshape(1), scale, ctx.smoothing,
                               logits.dtype == torch.bfloat16)
        return d, None, None, None, None


def cross_entropy(logits, labels, num_classes=None, smoothing=0.0, reduction="mean", return_rank=False):
    """Softmax cross-entropy (one fused pass) -> loss [, rank of the true label]."""
    C = num_classes or logits.shape[1]
    loss, rank = _XEnt.apply(logits, labels, C, float(smoothing), reduction)
    return (loss, rank) if return_rank else loss


@torch.no_grad()
def metric_accum(acc: torch.Tensor, loss: torch.Tensor, loss_scale: float, rank: torch.Tensor, nrows: int):
    """acc (fp64 [4], on the device) += [loss_scale * sum(loss), #(rank < 1), #(rank < 3), nrows] over
    ``rank[:nrows]``: the loops' per-step top-1 / top-3 / loss bookkeeping as ONE launch, with the
    row count a kernel argument (no host->device copy, so no stream sync)."""
    loss = loss.detach().reshape(-1)
    rank = rank.detach().reshape(-1)
    if rank.dtype != torch.int32:
        rank = rank.int()
    K(acc).metric_accum(acc, loss.contiguous(), float(loss_scale), rank.contiguous(), int(nrows))
    return acc


def cross_entropy_rows(logits, labels, num_classes=None):
    """Per-sample CE loss and label rank (evaluation; no autograd)."""
    return K(logits).xent_fwd(logits, labels, num_classes or logits.shape[1], 0.0)


@torch.no_grad()
def arcface_rows(x, weight, labels, s=30.0, m=0.5, easy_margin=True, with_margin=True):
    """Per-sample (loss, rank) of the ArcFace head.  ``with_margin=False`` ranks the
    plain scaled cosines (a label-free prediction)."""
    k = K(x)
    C, D = weight.shape
    Dp = round_up(D, 8) if x.is_cuda else D
    Cp = round_up(C, 64) if x.is_cuda else C
    xn, _ = k.l2norm_rows(x.contiguous(), Dp, 1e-12)
    wn, _ = k.l2norm_rows(weight.detach().contiguous(), Dp, 1e-12, Cp)  # zero rows C..Cp
    if not x.is_cuda:
        xn, wn = xn.float(), wn.float()
    cos = k.linear_fwd(xn, wn, None, 0)
    if with_margin:
        loss, rank, _, _ = k.arcface_fwd(cos, labels, C, s, m, easy_margin, False)
        return loss, rank
    return k.xent_fwd(cos[:, :C] * s if not x.is_cuda else cos[:, :C], labels, C, 0.0)


class _LogSoftmax(Function):
    @staticmethod
    def forward(ctx, x, C):
        y = K(x).log_softmax_fwd(x, C)
        ctx.save_for_backward(y)
        ctx.ldo = x.shape[1]
        ctx.bf = x.dtype == torch.bfloat16
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return K(y).log_softmax_bwd(y, dy.contiguous(), ctx.ldo, ctx.bf), None


def log_softmax(x, num_classes=None):
    """Row log-softmax -> fp32 [B, C]."""
    return _LogSoftmax.apply(x, num_classes or x.shape[1])


class _ArcFace(Function):
    """Fused ArcMarginProduct + cross-entropy (ARCFACE/arc_main.py:130-176, 245).

    cos = normalize(x) . normalize(W)^T on the MFMA GEMM, margin + softmax-CE +
    label rank in one row kernel; backward through the margin, the cosine
    GEMM (dgrad + wgrad) and both L2 normalisations.
    """

    @staticmethod
    def forward(ctx, x, weight, labels, s, m, easy, want_logits):
        k = K(x)
        C, D = weight.shape
        Dp = round_up(D, 8) if x.is_cuda else D
        Cp = round_up(C, 64) if x.is_cuda else C
        xn, inv_x = k.l2norm_rows(x.contiguous(), Dp, 1e-12)
        wn, inv_w = k.l2norm_rows(weight.detach().contiguous(), Dp, 1e-12, Cp)  # zero rows C..Cp
        if not x.is_cuda:
            xn, wn = xn.float(), wn.float()
        cos = k.linear_fwd(xn, wn, None, 0)  # [B, Cp]
        loss_rows, rank, dphi, logits = k.arcface_fwd(cos, labels, C, s, m, easy, want_logits)
        ctx.save_for_backward(xn, inv_x, wn, inv_w, cos, labels, dphi)
        ctx.cfg = (C, D, s, m, easy)
        ctx.mark_non_differentiable(rank, logits)
        ctx.set_materialize_grads(False)
        return loss_rows.mean(), rank, logits

    @staticmethod
    def backward(ctx, g, _grank, _glogits):
        if g is None:
            return (None,) * 7
        xn, inv_x, wn, inv_w, cos, labels, dphi = ctx.saved_tensors
        C, D, s, m, easy = ctx.cfg
        k = K(cos)
        B = cos.shape[0]
        dcos = k.arcface_bwd(cos, labels, C, s, m, easy, dphi, g.reshape(1), 1.0 / B)  # [B, Cp]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wnt = k.transpose2d(wn)  # [Dp, Cp]
            dxn = k.linear_fwd(dcos, wnt, None, 0)  # [B, Dp]
            dx = k.l2norm_bwd(dxn, xn, inv_x, D, False)
        if ctx.needs_input_grad[1]:
            dwn = k.linear_wgrad(dcos, xn)  # [Cp, Dp] fp32
            dw = k.l2norm_bwd(dwn[:C].contiguous(), wn, inv_w, D, False)  # the C real rows only
        return dx, dw, None, None, None, None, None


class _ArcFaceFused(Function):
    """The ArcFace head without a [B, C] tensor (csrc/arcface.hip): the cosine tiles
    live in MFMA registers only -- forward streams the normalised class weights through an online
    log-sum-exp (loss, label rank, lse), backward recomputes each tile and feeds dcos straight into
    the dX / dW MFMAs (the normalisation backward fused into their epilogues).  The per-step
    memory is O((B + C) * D), so 100k+ classes fit where the unfused path needs 4 B*C bytes."""

    @staticmethod
    def forward(ctx, x, weight, labels, s, m, easy):
        k = K(x)
        B, D = x.shape
        C = weight.shape[0]
        Dp = 128 if D <= 128 else 256
        Bp, Cp = round_up(B, 64), round_up(C, 64)
        # normalised operands and their transposes (the backward's MFMA A operands), one pass each
        xn, xnT, inv_x = k.arcface_l2norm_t(x.contiguous(), Bp, Dp, 1e-12)  # zero rows B..Bp
        wn, wnT, inv_w = k.arcface_l2norm_t(weight.detach().contiguous(), Cp, Dp, 1e-12)  # zero rows C..Cp
        lab64 = labels.to(torch.int64).contiguous()
        loss_rows, rank, lse, lab = k.arcface_fused_fwd(xn, wn, lab64, B, C, s, m, easy)
        ctx.save_for_backward(xn, xnT, inv_x, wn, wnT, inv_w, lab64, lse, lab)
        ctx.cfg = (B, C, D, s, x.dtype == torch.bfloat16)
        ctx.mark_non_differentiable(rank)
        ctx.set_materialize_grads(False)
        return loss_rows.mean(), rank

    @staticmethod
    def backward(ctx, g, _grank):
        if g is None:
            return (None,) * 6
        xn, xnT, inv_x, wn, wnT, inv_w, lab64, lse, lab = ctx.saved_tensors
        B, C, D, s, x_bf16 = ctx.cfg
        k = K(xn)
        g = g.reshape(1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = k.arcface_fused_dx(xn, wn, wnT, lab64, lse, lab, g, 1.0 / B, inv_x, B, C, D, s, x_bf16)
        if ctx.needs_input_grad[1]:
            dw = k.arcface_fused_dw(xn, xnT, wn, lab64, lse, lab, g, 1.0 / B, inv_w, B, C, D, s)
        return dx, dw, None, None, None, None


def arcface_fused_enabled() -> bool:
    """The fused head is the GPU default; DCP_ARCFACE_FUSED=0 selects the unfused path (A/B)."""
    return os.environ.get("DCP_ARCFACE_FUSED", "1") != "0"


def arcface_fused_supported(B: int, D: int) -> bool:
    """Shapes the fused kernels cover: D <= 256 (padded to 128 / 256), and the dW kernel's LDS
    (two staged row tiles of 2 x 16 KB x Dp / 128 plus 16 B per padded row) within 160 KB."""
    if D > 256:
        return False
    Dp = 128 if D <= 128 else 256
    return 4 * 64 * Dp * 2 + round_up(B, 64) * 16 <= 160 * 1024


def arcface_loss(x, weight, labels, s=30.0, m=0.5, easy_margin=True, return_logits=False):
    """Returns (mean loss, rank of label, margin logits or empty).  On the GPU without
    ``return_logits`` (training, the reference's loss) the fused head runs: no [B, C] tensor."""
    if (x.is_cuda and not return_logits and x.dim() == 2 and arcface_fused_supported(x.shape[0], x.shape[1])
            and arcface_fused_enabled() and x.dtype in (torch.float32, torch.bfloat16)):
        loss, rank = _ArcFaceFused.apply(x, weight, labels, float(s), float(m), bool(easy_margin))
        return loss, rank, torch.empty(0, device=x.device)
    return _ArcFace.apply(x, weight, labels, float(s), float(m), bool(easy_margin), bool(return_logits))


# ----------------------------------------------------------------------------- misc
def s2d_block(s2d) -> int:
    """The space-to-depth block of an input-layout ``s2d`` value: False / 0 none, True / 2 the
    ResNet s2d stem's 2x2 (16 channels), 4 TResNet's SpaceToDepth(4) (48 channels)."""
    if s2d is True:
        return 2
    return int(s2d or 0)


def s2d_for(s2d, h: int, w: int) -> int:
    """``s2d``'s block if an h x w image divides into it, else 0 (plain NHWC input)."""
    b = s2d_block(s2d)
    return b if b and h % b == 0 and w % b == 0 else 0


def to_device_nhwc(images: torch.Tensor, mean=None, std=None, cpad: int = 8, nchw: bool = True, in_scale: float = 1.0,
                   s2d=False):
    """Image batch (uint8 or fp32, NCHW/NHWC, already on the target device) -> normalised
    NHWC activations with channels zero-padded to ``cpad``; ``s2d=True`` (or 2) emits the 2x2
    space-to-depth layout [N, H/2, W/2, 16] of the s2d stem (:func:`stem_conv_s2d`), ``s2d=4``
    TResNet's 4x4 space-to-depth input [N, H/4, W/4, 48] (one pass from the images)."""
    if mean is not None and not torch.is_tensor(mean):
        mean = torch.tensor(mean, dtype=torch.float32, device=images.device)
    if std is not None and not torch.is_tensor(std):
        std = torch.tensor(std, dtype=torch.float32, device=images.device)
    blk = s2d_block(s2d)
    if blk:
        out = K(images).to_nhwc_s2d(images.contiguous(), nchw, in_scale, mean, std, blk)
    else:
        out = K(images).to_nhwc(images.contiguous(), nchw, cpad, in_scale, mean, std)
    return out.to(act_dtype(images.device)) if not images.is_cuda else out


def crop_resize(src: torch.Tensor, meta: torch.Tensor, Ho: int, Wo: int) -> torch.Tensor:
    """Gathered raw uint8 records ``src`` (1-D, on the target device) + host int64 ``meta``
    [B, 8] = {byte offset, H, W, y0, x0, h, w, flip} -> uint8 [B, Ho, Wo, 3]: the resample half of
    RandomResizedCrop / Resize+CenterCrop + horizontal flip (see data/shards.py)."""
    return K(src).crop_resize(src, meta, int(Ho), int(Wo))


# ----------------------------------------------------------------------------- space-to-depth stem
def nhwc_to_s2d(x: torch.Tensor) -> torch.Tensor:
    """[N, H, W, C>=4] NHWC image activations (channels >= 3 zero) -> [N, H/2, W/2, 16]."""
    N, H, W, _ = x.shape
    return (x[..., :4].reshape(N, H // 2, 2, W // 2, 2, 4).permute(0, 1, 3, 2, 4, 5)
            .reshape(N, H // 2, W // 2, 16).contiguous())


def stem_s2d_weight(w: torch.Tensor) -> torch.Tensor:
    """[Co, 7, 7, C<=4] weight of a 7x7 / stride-2 / pad-3 conv -> [Co, 4, 4, 16] weight of the
    equivalent 4x4 / stride-1 conv over the 2x2 space-to-depth input (top/left pad 2):
    w'[co][ta][tb][(py*2+px)*4 + c] = w[co][2ta+py-1][2tb+px-1][c] (zero outside 0..6).
    Differentiable, so autograd maps the 4x4 weight gradient back onto the 7x7 master."""
    co, _, _, c = w.shape
    w8 = F.pad(w, (0, 4 - c, 1, 0, 1, 0))  # [co, 8, 8, 4], kernel index u = k + 1
    return w8.reshape(co, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(co, 4, 4, 16)


def _s2d_weight_refresh(weight, buf):
    """buf <- the s2d form of the 7x7 master, one launch (no pad / permute / copy chain per step)."""
    with torch.no_grad():
        K(weight).s2d_weight(weight.detach().contiguous(), buf)
    # the kernel writes buf behind autograd's back: bump its version so the bf16 weight cache
    # (stamped with buf._version) refreshes even without a weight-generation bump
    torch.autograd.graph.increment_version(buf)


class _StemS2D(Function):
    """The s2d stem conv; autograd input is the 7x7 master itself (the 4x4 weight gradient goes
    back onto it through s2d_weight_bwd)."""

    @staticmethod
    def forward(ctx, x, w7, wb, stats):
        y, slabs = K(x).stem_fwd(x, wb, stats)  # slabs: BN partials [P,3,64] or conv slabs
        ctx.save_for_backward(x)
        ctx.c7 = w7.shape[3]
        ctx.mark_non_differentiable(slabs)
        ctx.set_materialize_grads(False)
        return y, slabs

    @staticmethod
    def backward(ctx, dy, _dslabs):
        if dy is None:
            return None, None, None, None
        (x,) = ctx.saved_tensors
        dw = None
        if ctx.needs_input_grad[1]:
            k = K(dy)
            dw = k.s2d_weight_bwd(k.conv_wgrad_geo(dy.contiguous(), x, 4, 4, 1, 2).float().contiguous(), ctx.c7)
        return None, dw, None, None


def stem_conv_s2d(x16: torch.Tensor, weight: torch.Tensor, buf: torch.Tensor, stats: bool = False):
    """The ResNet 7x7/2 stem as a 4x4/1 implicit GEMM over the space-to-depth input:
    K = 16 taps x 16 channels = 256 (4 MFMA k-tiles) instead of 49 taps x 8 padded
    channels = 392 (7 k-tiles).  ``buf``: persistent fp32 [Co,4,4,16] holding the
    transformed master weight (its bf16 copy rides the multi-tensor weight cache)."""
    _s2d_weight_refresh(weight, buf)
    wb, _ = prepared_weight(buf, 0, False)
    return _StemS2D.apply(x16, weight, wb, bool(stats and x16.is_cuda))


class _StemBNPool(Function):
    """The ResNet stem as one op: s2d 4x4 conv (statistics from its kernel) + training-mode
    BN + ReLU + 3x3/2 max pool.  Backward runs the fused stem kernel (stem.hip stem_bwd): the
    BN / max-pool backward and the stem weight gradient in one pass, the weight gradient
    formed from G1 = sum g' X, G2 = sum (z - mu) X, G3 = sum X once the BN sums are known, so
    neither the full-resolution activation gradient nor a second BN-backward pass exists."""

    @staticmethod
    def forward(ctx, x16, w7, wb, gamma, beta, run_mean, run_var, cfg: BNConfig):
        k = K(x16)
        ctx.c7 = w7.shape[3]
        z, part = k.stem_fwd(x16, wb, True)
        mean, invstd, scale, shift, count = _bn_train_coeff(k, z, part, gamma, beta, run_mean, run_var, cfg)
        y, idx = k.bn_act_maxpool(z, scale, shift, cfg.act, 3, 2, 1)
        ctx.save_for_backward(x16, z, idx, scale, shift, mean, invstd)
        ctx.cfg, ctx.count = cfg, count
        ctx.mark_non_differentiable(idx)
        ctx.set_materialize_grads(False)
        return y, idx

    @staticmethod
    def backward(ctx, dy, _didx):
        if dy is None:
            return (None,) * 8
        x16, z, idx, scale, shift, mean, invstd = ctx.saved_tensors
        cfg = ctx.cfg
        k = K(dy)
        tot, local = k.stem_bn_pool_bwd(dy.contiguous(), idx, z, x16, scale, shift, mean, invstd, cfg.act)
        sums = local
        if cfg.group is not None:
            sums = local.clone()
            _peer.all_reduce(sums, cfg.group)
        dw = None
        if ctx.needs_input_grad[1]:  # the 4x4 s2d weight gradient, onto the 7x7 master
            dw = k.s2d_weight_bwd(k.stem_bwd_dw(tot, sums, scale, invstd, float(ctx.count)), ctx.c7)
        dgamma = local[1] if ctx.needs_input_grad[3] else None
        dbeta = local[0] if ctx.needs_input_grad[4] else None
        return None, dw, None, dgamma, dbeta, None, None, None


def stem_bn_pool_fusable(x16: torch.Tensor, act: str = "relu") -> bool:
    """Whether stem_bn_pool's fused kernels cover this input (GPU, training, ReLU/identity,
    even H, W a multiple of 16 up to 112, or 56: the 112 px input)."""
    if not (x16.is_cuda and x16.dim() == 4 and x16.shape[-1] == 16 and act in ("relu", "none")
            and torch.is_grad_enabled()):
        return False
    z_like = x16.new_empty((1, x16.shape[1], x16.shape[2], 64))
    return bool(K(x16).stem_bwd_fusable(z_like))


def stem_bn_pool(x16, weight, buf, gamma, beta, run_mean, run_var, momentum, eps, act="relu", group=None):
    """s2d stem conv + training-mode BN + act + 3x3/2 max pool as one autograd op (see
    _StemBNPool); ``weight`` is the 7x7 master, ``buf`` the persistent [64,4,4,16] fp32 buffer
    of its s2d form (as stem_conv_s2d)."""
    group, world = _sync_group(group)
    cfg = BNConfig(True, momentum, eps, ACT[act], 0.0, group, world)
    _s2d_weight_refresh(weight, buf)
    wb, _ = prepared_weight(buf, 0, False)
    y, _ = _StemBNPool.apply(x16, weight, wb, gamma, beta, run_mean, run_var, cfg)
    return y


class _PrefixMask(Function):
    @staticmethod
    def forward(ctx, x, keep):
        ctx.save_for_backward(keep)
        return K(x).prefix_mask(x.contiguous(), keep)

    @staticmethod
    def backward(ctx, dy):
        (keep,) = ctx.saved_tensors
        return K(dy).prefix_mask(dy.contiguous(), keep), None


def nested_mask(feature, k_index):
    """feature * 1[:k+1] (nested dropout, NESTED/train.py:247-250); k_index int."""
    # a fill kernel with K as its argument: torch.tensor(..., device=) would be a pageable
    # host->device copy, which synchronises the stream every step
    keep = torch.full((1,), int(k_index) + 1, dtype=torch.int32, device=feature.device)
    return _PrefixMask.apply(feature, keep)


def nested_eval_counts(feature: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Per-K (top-1, top-3) correct counts for every prefix length K (int32 [D,2])."""
    return K(feature).nested_eval(feature.float().contiguous(), weight.float().contiguous(), labels)


def gaussian_dist(mu: float, std: float, n: int):
    """NESTED/train.py:93-97: p(i) ∝ exp(-((i-mu)/std)^2), i = 1..n."""
    import numpy as np

    d = np.array([math.exp(-(((i - mu) / std) ** 2)) for i in range(1, n + 1)])
    return d / d.sum()
