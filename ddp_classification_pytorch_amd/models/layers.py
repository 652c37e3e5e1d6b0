"""NHWC building blocks over the gfx950 primitives.

* :class:`Conv2d` stores its master weight as fp32 ``[Co, KH, KW, Ci]``
  (K-contiguous per output channel, the implicit-GEMM B operand layout).
  ``load_state_dict`` accepts torchvision-layout ``[Co, Ci, KH, KW]`` weights
  and permutes them, so pretrained torchvision/timm checkpoints load.
* :class:`BatchNorm2d` is called with the conv's statistics slabs, an
  activation and an optional residual: BN-apply + ReLU/leaky-ReLU + residual
  add are one kernel.  SyncBN (``process_group``, reference BASELINE/main.py:148)
  all-gathers each rank's per-channel (n, mean, M2) in forward -- Chan-merged by the
  finalize kernel (torch gathers (mean, invstd, count)) -- and all-reduces (sum g, sum g*xhat) in backward; a projection
  block's two BNs share one collective each way (ops/functional.py).
* :class:`Linear` is an nn.Linear-compatible module over the MFMA GEMM.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as Fn


class Conv2d(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, groups=1, bias=False):
        super().__init__()
        assert not bias, "convolutions feeding BN carry no bias"
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding, self.groups = kernel_size, stride, padding, groups
        self.weight = nn.Parameter(torch.empty(out_channels, kernel_size, kernel_size, in_channels // groups))
        self.reset_parameters()

    def reset_parameters(self):
        # Kaiming normal, fan_out, ReLU gain (NESTED/model/imagenet_resnet.py init; torchvision ResNet)
        fan_out = self.out_channels * self.kernel_size * self.kernel_size // self.groups
        nn.init.normal_(self.weight, 0.0, math.sqrt(2.0 / fan_out))

    def forward(self, x, stats=False, link=None, deposit=None):
        """Returns (y, bn_stat_slabs_or_None).  `link` / `deposit`: block-input gradient
        hand-off as primary / secondary consumer (ops.functional.GradJoin)."""
        if self.groups > 1:
            if stats:
                return Fn.grouped_conv2d(x, self.weight, self.groups, self.stride, self.padding, stats=True)
            return Fn.grouped_conv2d(x, self.weight, self.groups, self.stride, self.padding), None
        y, slabs = Fn.conv2d(x, self.weight, self.stride, self.padding, stats and x.is_cuda, link, deposit)
        return y, (slabs if stats and x.is_cuda else None)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        key = prefix + "weight"
        w = state_dict.get(key)
        if w is not None and w.dim() == 4 and tuple(w.shape) != tuple(self.weight.shape):
            # torchvision layout [Co, Ci, KH, KW] -> [Co, KH, KW, Ci]
            if tuple(w.permute(0, 2, 3, 1).shape) == tuple(self.weight.shape):
                state_dict[key] = w.permute(0, 2, 3, 1).contiguous()
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        Fn.bump_weight_generation()

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, k={self.kernel_size}, s={self.stride}, "
                f"p={self.padding}, groups={self.groups}, layout=NHWC")


class BatchNorm2d(nn.Module):
    """BatchNorm over the channel (last) dim of NHWC activations, fused with act/residual.

    ``frozen`` (NESTED ``freeze_bn``, NESTED/model/model.py:44-55) uses running
    statistics even in training mode and keeps gamma/beta fixed.
    """

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))
        self.process_group = None  # set by parallel.convert_sync_batchnorm
        self.frozen = False
        self._nbt_pending = 0
        # InplaceABN semantics (mapillary inplace_abn, used by timm's TResNet): the
        # effective weight is |gamma| + eps and only the activation output is kept for backward
        self.inplace_abn = False
        self.iabn_eps = 1e-5

    def forward(self, x, slabs=None, act="relu", residual=None, slope=0.01, link=None, residual_bn=None,
                fuse_bwd=False):
        """``residual_bn=(bn, rslabs)``: ``residual`` is the raw input of BatchNorm2d ``bn`` (a
        projection shortcut), normalised inside this layer's apply pass (Fn.batch_norm_add_bn_act)."""
        stats = self.training and not self.frozen
        if residual_bn is not None:
            rbn, rslabs = residual_bn
            rstats = rbn.training and not rbn.frozen
            if (rstats != stats or rbn.process_group is not self.process_group or link is not None
                    or not Fn.shortcut_bn_fusion()):
                residual = rbn(residual, rslabs, act="none")  # unfusable combination: BN the shortcut first
            else:
                if stats:
                    self._nbt_pending += 1
                    rbn._nbt_pending += 1
                return Fn.batch_norm_add_bn_act(x, slabs, self.weight, self.bias, self.running_mean,
                                                self.running_var, residual, rslabs, rbn.weight, rbn.bias,
                                                rbn.running_mean, rbn.running_var, stats, self.momentum, self.eps,
                                                rbn.momentum, rbn.eps, act=act, slope=slope,
                                                group=self.process_group if stats else None)
        if stats:
            self._nbt_pending += 1  # folded into num_batches_tracked lazily (no per-step device add)
        iabn = self.inplace_abn and residual is None and act in ("none", "leaky", "leaky_relu")
        gamma, rgamma, iabn_eps = self.weight, None, None
        if iabn and self.weight is not None:
            if stats and self.bias is not None and Fn.iabn_fold_enabled():
                iabn_eps = self.iabn_eps  # |gamma| + eps and sign(gamma) inside the BN kernels
            else:
                gamma, rgamma = Fn.iabn_gamma(self.weight, self.iabn_eps)
        return Fn.batch_norm_act(x, slabs, gamma, self.bias, self.running_mean, self.running_var, stats, self.momentum,
                                 self.eps, act=act, slope=slope, residual=residual,
                                 group=self.process_group if stats else None, link=link, iabn=iabn,
                                 fuse_bwd=fuse_bwd, rgamma=rgamma, iabn_eps=iabn_eps)

    def forward_pool(self, x, slabs=None, act="relu", k=3, s=2, p=1):
        """BN + act + k x k / s max pool.  Training-mode statistics with a ReLU/identity
        activation and a channel count the fused kernel covers run as ONE fused op
        (the full-resolution activation is never stored); otherwise BN then pool."""
        C = x.shape[-1]
        if (self.training and not self.frozen and act in ("relu", "none") and C % 8 == 0 and 256 % (C // 8) == 0
                and torch.is_grad_enabled()):
            self._nbt_pending += 1
            return Fn.batch_norm_act_maxpool(x, slabs, self.weight, self.bias, self.running_mean, self.running_var,
                                             self.momentum, self.eps, act=act, k=k, s=s, p=p,
                                             group=self.process_group)
        return Fn.max_pool2d(self(x, slabs, act=act), k, s, p)

    def flush_batches_tracked(self):
        if self._nbt_pending:
            self.num_batches_tracked.add_(self._nbt_pending)
            self._nbt_pending = 0

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self.flush_batches_tracked()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}, sync={self.process_group is not None}"


class Linear(nn.Module):
    """nn.Linear-compatible ([out, in] fp32 weight) on the MFMA GEMM, optional fused ReLU."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):  # identical to nn.Linear
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, relu=False):
        return Fn.linear(x, self.weight, self.bias, relu=relu)

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        Fn.bump_weight_generation()

    def extra_repr(self):
        return f"in={self.in_features}, out={self.out_features}, bias={self.bias is not None}"


def bn_relu_conv(bn: BatchNorm2d, conv: Conv2d, x, slabs=None, stats=False, fuse_bwd=False):
    """conv(relu(bn(x))) where ``conv`` is the BN output's only consumer.  A training-mode BN is
    then applied inside the conv: the normalised activation is never written.
      * a 1x1 stride-1 conv (a bottleneck's bn2 -> conv3): in the GEMMs' operand registers
        (``Fn.bn_relu_conv1x1``; opt-in, ``DCP_BN_PROLOGUE=1``: VALU-bound at K = 64);
      * a 64 -> 64 channel 3x3 stride-1 conv (ResNet-50 layer1's bn1 -> conv2): once per staged
        window element of the direct kernels, each element feeding nine taps
        (``Fn.bn_relu_conv3x3``; default on, ``DCP_BN_PROLOGUE3=0`` off).
    Any other case runs bn then conv.  Returns (y, statistics slabs of y or None)."""
    C, Co = x.shape[-1], conv.out_channels
    train_bn = (bn.training and not bn.frozen and not bn.inplace_abn and conv.groups == 1 and bn.weight is not None
                and conv.weight.shape[3] == C)
    if (train_bn and Fn.bn_prologue_enabled() and conv.kernel_size == 1 and conv.stride == 1 and conv.padding == 0
            and Fn.bn_prologue_fits(C, Co)):
        bn._nbt_pending += 1
        return Fn.bn_relu_conv1x1(x, slabs, bn.weight, bn.bias, bn.running_mean, bn.running_var, True, bn.momentum,
                                  bn.eps, conv.weight, stats, group=bn.process_group)
    if (train_bn and Fn.bn_prologue3x3_enabled() and x.is_cuda and conv.kernel_size == 3 and conv.stride == 1
            and conv.padding == 1 and Fn.bn_prologue3x3_fits(x, C, Co)):
        bn._nbt_pending += 1
        return Fn.bn_relu_conv3x3(x, slabs, bn.weight, bn.bias, bn.running_mean, bn.running_var, True, bn.momentum,
                                  bn.eps, conv.weight, stats, group=bn.process_group)
    return conv(bn(x, slabs, act="relu", fuse_bwd=fuse_bwd), stats=stats)


def conv_bn(conv: Conv2d, bn: BatchNorm2d, x, act="relu", residual=None, slope=0.01):
    """act(BN(conv(x)) [+ residual]) for a BN that normalises with its running statistics
    (``Fn.bn_foldable``: model.eval(), NESTED's frozen BN): the BN is folded
    into the conv's store epilogue, so no un-normalised output is written and no BN pass runs.
    Grouped convs (no folded kernel) run conv -> BN."""
    if conv.groups == 1 and conv.weight.shape[3] == x.shape[3]:
        return Fn.conv_bn_folded(x, conv.weight, conv.stride, conv.padding, bn, act=act, slope=slope,
                                 residual=residual)
    y, _ = conv(x)
    return bn(y, None, act=act, residual=residual, slope=slope)


class ConvBN(nn.Module):
    """conv -> BN (stats from the conv epilogue) -> act, optional residual."""

    def __init__(self, cin, cout, k, stride=1, padding=None, groups=1, act="relu", slope=0.01, inplace_abn=False):
        super().__init__()
        padding = k // 2 if padding is None else padding
        self.conv = Conv2d(cin, cout, k, stride, padding, groups)
        self.bn = BatchNorm2d(cout)
        self.bn.inplace_abn = bool(inplace_abn)
        self.act, self.slope = act, slope

    def forward(self, x, residual=None):
        if Fn.bn_foldable(self.bn):
            return conv_bn(self.conv, self.bn, x, act=self.act, residual=residual, slope=self.slope)
        y, slabs = self.conv(x, stats=self.bn.training and not self.bn.frozen)
        return self.bn(y, slabs, act=self.act, residual=residual, slope=self.slope)
