"""Reference (plain PyTorch, fp32-accumulating) implementations of every
primitive registered by the HIP library under ``torch.ops.dcp``.

Same names, same signatures, same layouts (NHWC activations, [Co,KH,KW,Ci]
weights).  They serve two purposes only:

* the CPU path (unit tests, gloo multi-process plumbing, BASELINE.json
  config 1) -- never a GPU fallback;
* the numerics oracle the GPU kernel tests compare against.

Activation outputs keep the input dtype (fp32 on CPU in practice).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2


def _f(t):
    return t.float()


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _w_oihw(w):  # [Co,KH,KW,Ci] -> [Co,Ci,KH,KW]
    return w.permute(0, 3, 1, 2)


# ----------------------------------------------------------------------------- conv
def conv_fwd(x, w, stride, pad, stats):
    y = F.conv2d(_nchw(_f(x)), _w_oihw(_f(w)), stride=stride, padding=pad)
    y = _nhwc(y).to(x.dtype)
    return y, torch.empty(0, device=x.device)


def conv_dgrad(dy, wt, H, W, stride, pad, add=None):
    # wt: [C,KH,KW,Co] (transposed); recover w [Co,KH,KW,C]
    w = wt.permute(3, 1, 2, 0)
    N = dy.shape[0]
    C = wt.shape[0]
    KH, KW = wt.shape[1], wt.shape[2]
    Ho, Wo = dy.shape[1], dy.shape[2]
    op_h = H - ((Ho - 1) * stride - 2 * pad + KH)
    op_w = W - ((Wo - 1) * stride - 2 * pad + KW)
    dx = F.conv_transpose2d(_nchw(_f(dy)), _w_oihw(_f(w)), stride=stride, padding=pad, output_padding=(op_h, op_w))
    assert dx.shape == (N, C, H, W)
    dx = _nhwc(dx)
    if add is not None:
        dx = dx + _f(add)
    return dx.to(dy.dtype)


def unpack_mask(mask):
    """[..., C/8] uint8 activation-mask bits (bit e of byte c = channel 8c+e) -> [..., C] float."""
    bits = (mask.to(torch.int32).unsqueeze(-1) >> torch.arange(8, dtype=torch.int32)) & 1
    return bits.reshape(*mask.shape[:-1], mask.shape[-1] * 8).float()


def conv_dgrad_bn(dy, wt, pad, add, y, res, scale, shift, mean, invstd, act, mask=None, slope=0.0):
    """Stride-1 dgrad + the backward reduction of the BN(+act)(+res) layer producing its input:
    -> (gradient, [2, C] = (sum g', sum g' * xhat)) with g' = act'(z) * dgrad.  ReLU / identity
    return g' itself (masking is idempotent); leaky ReLU returns the RAW dgrad (its BN backward
    re-applies act', so any other consumer's gradient can still be added).  ``mask``: the
    activation mask bits from :func:`bn_act_mask` (then ``res`` is not read)."""
    if add is not None and add.shape != y.shape:  # compact stride-2 add source (StridedGrad)
        full = add.new_zeros(y.shape)
        full[:, ::2, ::2] = add
        add = full
    g = conv_dgrad(dy, wt, y.shape[1], y.shape[2], 1, pad, add)
    if mask is not None:
        d = unpack_mask(mask) if act == ACT_RELU else torch.ones_like(_f(y))
    else:
        z = _f(y) * scale + shift
        if res is not None:
            z = z + _f(res)
        d = _act_d(z, act, slope)
    if act == ACT_LEAKY:
        gm = _f(g.to(dy.dtype)) * d
        out = g.to(dy.dtype)
    else:
        out = (_f(g) * d).to(dy.dtype)
        gm = _f(out)
    xh = (_rows(y) - mean) * invstd
    gr = _rows(gm)
    return out, torch.stack([gr.sum(0), (gr * xh).sum(0)])


def _pad_geo(xc, KH, KW, stride, pad, Ho, Wo):
    """NCHW input padded by `pad` at the top/left and padded/cropped at the bottom/right to
    exactly (Ho-1)*stride + K rows/columns (the explicit output grid of conv_fwd_geo)."""
    H, W = xc.shape[2], xc.shape[3]
    Hp, Wp = (Ho - 1) * stride + KH, (Wo - 1) * stride + KW
    xc = F.pad(xc, (pad, max(0, Wp - pad - W), pad, max(0, Hp - pad - H)))
    return xc[:, :, :Hp, :Wp]


def conv_fwd_geo(x, w, stride, pad, Ho, Wo, stats):
    xc = _pad_geo(_nchw(_f(x)), w.shape[1], w.shape[2], stride, pad, Ho, Wo)
    y = F.conv2d(xc, _w_oihw(_f(w)), stride=stride)
    return _nhwc(y).to(x.dtype), torch.empty(0, device=x.device)


def stem_fwd(x, w, stats):
    """the space-to-depth stem: 4x4 / stride 1, pad 2 top/left, output grid = input grid"""
    return conv_fwd_geo(x, w, 1, 2, x.shape[1], x.shape[2], stats)


def conv_wgrad_geo(dy, x, KH, KW, stride, pad):
    Co, C, Ho, Wo = dy.shape[3], x.shape[3], dy.shape[1], dy.shape[2]
    xc = _pad_geo(_nchw(_f(x)), KH, KW, stride, pad, Ho, Wo)
    dw = torch.nn.grad.conv2d_weight(xc, (Co, C, KH, KW), _nchw(_f(dy)), stride=stride)
    return dw.permute(0, 2, 3, 1).contiguous()


def conv_wgrad(dy, x, KH, KW, stride, pad):
    Co, C = dy.shape[3], x.shape[3]
    dw = torch.nn.grad.conv2d_weight(_nchw(_f(x)), (Co, C, KH, KW), _nchw(_f(dy)), stride=stride, padding=pad)
    return dw.permute(0, 2, 3, 1).contiguous()


def linear_fwd(x, w, bias, act):
    y = _f(x) @ _f(w).t()
    if bias is not None:
        b = _f(bias)[: y.shape[1]]
        if b.numel() < y.shape[1]:  # an unpadded bias of a padded GEMM
            b = F.pad(b, (0, y.shape[1] - b.numel()))
        y = y + b
    if int(act) == 1:
        y = torch.relu(y)
    elif int(act) == 2:
        y = torch.sigmoid(y)
    return y.to(x.dtype)


def linear_wgrad(dy, x):
    return _f(dy).t() @ _f(x)


def weight_prep(w, co_pad, transposed):
    Co = w.shape[0]
    cp = max(co_pad, Co)
    wb = w
    if cp > Co:
        pad_shape = (cp - Co,) + tuple(w.shape[1:])
        wb = torch.cat([w, w.new_zeros(pad_shape)], 0)
    if transposed:
        wt = wb.transpose(0, -1).contiguous() if w.dim() == 2 else wb.permute(3, 1, 2, 0).contiguous()
    else:
        wt = w.new_empty(0)
    return wb.contiguous(), wt


def grouped_conv_fwd(x, w, groups, stride, pad):
    y = F.conv2d(_nchw(_f(x)), _w_oihw(_f(w)), stride=stride, padding=pad, groups=groups)
    return _nhwc(y).to(x.dtype)


def grouped_conv_fwd_stats(x, w, groups, stride, pad):
    return grouped_conv_fwd(x, w, groups, stride, pad), x.new_empty(0, dtype=torch.float32)


def grouped_conv_dgrad_bn(dy, w, H, W, groups, stride, pad, z, scale, shift, mean, invstd):
    dx = _f(grouped_conv_dgrad(dy, w, H, W, groups, stride, pad))
    zf = _f(z)
    g = torch.where(zf * scale + shift > 0, dx, torch.zeros_like(dx)).to(dy.dtype)
    gf = _rows(_f(g))
    xh = (_rows(zf) - mean) * invstd
    return g, torch.stack([gf.sum(0), (gf * xh).sum(0)])


def grouped_conv_dgrad(dy, w, H, W, groups, stride, pad):
    N, Co = dy.shape[0], dy.shape[3]
    C = w.shape[3] * groups
    KH, KW = w.shape[1], w.shape[2]
    dx = torch.nn.grad.conv2d_input((N, C, H, W), _w_oihw(_f(w)), _nchw(_f(dy)), stride=stride, padding=pad,
                                    groups=groups)
    return _nhwc(dx).to(dy.dtype)


def grouped_conv_wgrad(dy, x, KH, KW, groups, stride, pad):
    Co, C = dy.shape[3], x.shape[3]
    dw = torch.nn.grad.conv2d_weight(_nchw(_f(x)), (Co, C // groups, KH, KW), _nchw(_f(dy)), stride=stride,
                                     padding=pad, groups=groups)
    return dw.permute(0, 2, 3, 1).contiguous()


# ----------------------------------------------------------------------------- batch norm
def _rows(x):
    return _f(x).reshape(-1, x.shape[-1])


def bn_stats(x, slabs):
    """-> [1, 3, C] = (n, mean, M2) per channel."""
    r = x.double().reshape(-1, x.shape[-1])
    n = r.shape[0]
    mean = r.mean(0)
    m2 = ((r - mean) ** 2).sum(0)
    return torch.stack([torch.full_like(mean, float(n)), mean, m2]).float().unsqueeze(0)


def colsum(x):
    return _rows(x).sum(0)


def bn_finalize(stats, gamma, beta, run_mean, run_var, momentum, eps, iabn_eps=-1.0, rgamma_out=None):
    """stats [W,3,C] (n, mean, M2 per rank) merged with Chan's formula.  iabn_eps >= 0: InplaceABN's
    effective weight |gamma| + iabn_eps, its reciprocal written to rgamma_out."""
    if iabn_eps >= 0 and gamma is not None:
        gamma = gamma.abs() + iabn_eps
        if rgamma_out is not None:
            rgamma_out.copy_(1.0 / gamma)
    st = stats.double()
    n_t = st[:, 0].sum(0)
    mu = (st[:, 0] * st[:, 1]).sum(0) / n_t
    m2 = st[:, 2].sum(0) + (st[:, 0] * (st[:, 1] - mu) ** 2).sum(0)
    var = m2 / n_t
    invstd = 1.0 / torch.sqrt(var + eps)
    g = gamma.double() if gamma is not None else torch.ones_like(mu)
    b = beta.double() if beta is not None else torch.zeros_like(mu)
    scale = g * invstd
    shift = b - mu * scale
    if run_mean is not None:
        unb = torch.where(n_t > 1, m2 / (n_t - 1).clamp_min(1), var)
        run_mean.mul_(1 - momentum).add_(momentum * mu.float())
        run_var.mul_(1 - momentum).add_(momentum * unb.float())
    return mu.float(), invstd.float(), scale.float(), shift.float()


def bn_stats_finalize(x, slabs, gamma, beta, run_mean, run_var, momentum, eps, iabn_eps=-1.0, rgamma_out=None):
    return bn_finalize(bn_stats(x, slabs), gamma, beta, run_mean, run_var, momentum, eps, iabn_eps, rgamma_out)


def bn_eval_coeff(gamma, beta, run_mean, run_var, eps):
    invstd = torch.rsqrt(run_var.float() + eps)
    g = gamma.float() if gamma is not None else torch.ones_like(invstd)
    b = beta.float() if beta is not None else torch.zeros_like(invstd)
    scale = g * invstd
    return run_mean.float().clone(), invstd, scale, b - run_mean.float() * scale


def _act(z, act, slope):
    if act == ACT_RELU:
        return torch.relu(z)
    if act == ACT_LEAKY:
        return torch.where(z >= 0, z, z * slope)
    return z


def _act_d(z, act, slope):
    if act == ACT_RELU:
        return (z > 0).float()
    if act == ACT_LEAKY:
        return torch.where(z >= 0, torch.ones_like(z), torch.full_like(z, slope))
    return torch.ones_like(z)


def bn_act(x, res, scale, shift, act, slope):
    z = _f(x) * scale + shift
    if res is not None:
        z = z + _f(res)
    return _act(z, act, slope).to(x.dtype)


def conv_fwd_affine(x, w, stride, pad, scale, shift, act, slope, res):
    """conv -> eval-mode BN (per-channel scale / shift) [+ res] -> act, through the bf16-rounded
    conv output like the unfused chain."""
    c, _ = conv_fwd(x, w, stride, pad, False)
    return bn_act(c, res, scale, shift, act, slope)


def conv_fwd_pro(x, w, scale, shift, stats):
    """1x1 conv of the bf16 activation bf16(relu(x * scale + shift)) (the BN + ReLU the kernel
    applies to its A operand, K5)."""
    return conv_fwd(bn_act(x, None, scale, shift, 1, 0.0), w, 1, 0, stats)


def conv_wgrad_pro(dy, x, scale, shift):
    return conv_wgrad(dy, bn_act(x, None, scale, shift, 1, 0.0), 1, 1, 1, 0)


def conv3x3_fwd_pro(x, w, scale, shift, stats):
    """3x3 / stride-1 / pad-1 conv of bf16(relu(x * scale + shift)); the padding is of the BN output."""
    return conv_fwd(bn_act(x, None, scale, shift, 1, 0.0), w, 1, 1, stats)


def conv3x3_wgrad_pro(dy, x, scale, shift):
    return conv_wgrad(dy, bn_act(x, None, scale, shift, 1, 0.0), 3, 3, 1, 1)


def conv3x3_pro_fits(N, H, W, C, Co):
    return C == 64 and Co == 64


def act_scale_bwd(dy, y, scale, act, slope, want_g):
    g = _f(dy) * _act_d(_f(y), act, slope)
    gd = g.to(dy.dtype)
    dc = (_f(gd) * scale.float()).to(dy.dtype)
    return dc, (gd if want_g else torch.empty(0, dtype=dy.dtype))


def bn_act_mask(x, res, scale, shift, act, slope):
    z = _f(x) * scale + shift
    if res is not None:
        z = z + _f(res)
    pos = (z > 0).to(torch.int32).reshape(*z.shape[:-1], z.shape[-1] // 8, 8)
    mask = (pos << torch.arange(8, dtype=torch.int32)).sum(-1).to(torch.uint8)
    return _act(z, act, slope).to(x.dtype), mask


def bn_fin_act(x, slabs, res, gamma, beta, run_mean, run_var, momentum, eps, act, slope, want_mask, iabn_eps=-1.0,
               rgamma_out=None):
    """bn_stats_finalize + bn_act / bn_act_mask (the GPU op runs them as one launch)."""
    mean, invstd, scale, shift = bn_stats_finalize(x, slabs if slabs.numel() else None, gamma, beta, run_mean, run_var,
                                                   momentum, eps, iabn_eps, rgamma_out)
    if want_mask:
        y, mask = bn_act_mask(x, res, scale, shift, act, slope)
    else:
        y, mask = bn_act(x, res, scale, shift, act, slope), torch.empty(0, dtype=torch.uint8)
    return y, mask, mean, invstd, scale, shift


def bn2_act_mask(x, res, scale, shift, rscale, rshift, act, slope):
    return bn_act_mask(x, _f(res) * rscale + rshift, scale, shift, act, slope)


def _act_inv(y, act, slope):
    y = _f(y)
    return torch.where(y < 0, y / slope, y) if act == ACT_LEAKY else y


def bn_bwd_reduce(dy, x, res, scale, shift, mean, invstd, act, slope, inv=False):
    if inv:  # InplaceABN: x is the output y; mean / invstd carry beta / 1/gamma
        x = _act_inv(x, act, slope)
        z = x
    else:
        z = _f(x) * scale + shift
    if res is not None:
        z = z + _f(res)
    dz = _rows(dy * 1.0) * _act_d(z, act, slope).reshape(-1, x.shape[-1])
    xh = (_rows(x) - mean) * invstd
    return torch.stack([dz.sum(0), (dz * xh).sum(0)])


def bn_bwd_elemt(dy, x, res, scale, shift, mean, invstd, sums, count, act, slope, want_dres, inv=False, graw=None):
    if inv:  # InplaceABN: x is the output y; mean / invstd carry beta / 1/gamma
        x = _act_inv(x, act, slope)
        z = x
        dz = _f(dy) * _act_d(z, act, slope)
        xh = (x - mean) * invstd
        dx = scale * (dz - sums[0] / count - xh * sums[1] / count) if sums is not None else scale * dz
        if graw is not None:  # the raw InplaceABN weight's gradient sign(g) * sums[1]
            return dx.to(dy.dtype), (sums[1] * torch.sign(graw)).float()
        return dx.to(dy.dtype), (dz.to(dy.dtype) if want_dres else dy.new_empty(0))
    z = _f(x) * scale + shift
    if res is not None:
        z = z + _f(res)
    dz = _f(dy) * _act_d(z, act, slope)
    if sums is not None:
        xh = (_f(x) - mean) * invstd
        dx = scale * (dz - sums[0] / count - xh * sums[1] / count)
    else:
        dx = scale * dz
    dres = dz.to(dy.dtype) if want_dres else dy.new_empty(0)
    return dx.to(dy.dtype), dres


def bn2_bwd_elemt(g, x, r, scale, mean, invstd, sums, rscale, rmean, rinvstd, rsums, count):
    dx, _ = bn_bwd_elemt(g, x, None, scale, torch.zeros_like(scale), mean, invstd, sums, count, 0, 0.0, False)
    dr, _ = bn_bwd_elemt(g, r, None, rscale, torch.zeros_like(rscale), rmean, rinvstd, rsums, count, 0, 0.0, False)
    return dx, dr


# ----------------------------------------------------------------------------- pooling / layout
def maxpool_fwd(x, k, s, p):
    y, idx = F.max_pool2d(_nchw(_f(x)), k, s, p, return_indices=True)
    # window-local index (kh*k+kw) like the kernel
    N, C, Ho, Wo = y.shape
    W = x.shape[2]
    hi = torch.div(idx, W, rounding_mode="floor")
    wi = idx - hi * W
    ho = torch.arange(Ho).view(1, 1, Ho, 1)
    wo = torch.arange(Wo).view(1, 1, 1, Wo)
    kh = hi - (ho * s - p)
    kw = wi - (wo * s - p)
    loc = (kh * k + kw).to(torch.uint8)
    return _nhwc(y).to(x.dtype), _nhwc(loc)


def maxpool_bwd(dy, idx, H, W, k, s, p):
    N, Ho, Wo, C = dy.shape
    loc = _nchw(idx).long()
    kh = torch.div(loc, k, rounding_mode="floor")
    kw = loc - kh * k
    ho = torch.arange(Ho).view(1, 1, Ho, 1)
    wo = torch.arange(Wo).view(1, 1, 1, Wo)
    flat = (ho * s - p + kh) * W + (wo * s - p + kw)
    dx = torch.zeros(N, C, H * W, dtype=torch.float32)
    dx.scatter_add_(2, flat.reshape(N, C, -1), _nchw(_f(dy)).reshape(N, C, -1))
    return _nhwc(dx.view(N, C, H, W)).to(dy.dtype)


def bn_act_maxpool(x, scale, shift, act, k, s, p):
    return maxpool_fwd(bn_act(x, None, scale, shift, act, 0.0), k, s, p)


def maxpool_bn_bwd_reduce(dy, idx, x, scale, shift, mean, invstd, act, k, s, p):
    g = maxpool_bwd(dy, idx, x.shape[1], x.shape[2], k, s, p)
    return bn_bwd_reduce(g, x, None, scale, shift, mean, invstd, act, 0.0)


def maxpool_bn_bwd_elemt(dy, idx, x, scale, shift, mean, invstd, act, sums, count, k, s, p):
    g = maxpool_bwd(dy, idx, x.shape[1], x.shape[2], k, s, p)
    return bn_bwd_elemt(g, x, None, scale, shift, mean, invstd, sums, count, act, 0.0, False)[0]


def gap_fwd(x):
    N, C = x.shape[0], x.shape[-1]
    return _f(x).reshape(N, -1, C).mean(1).to(x.dtype)


def gap_bwd(dy, H, W, add=None):
    N, C = dy.shape
    g = (_f(dy) / (H * W)).view(N, 1, 1, C).expand(N, H, W, C)
    if add is not None:
        g = g + _f(add)
    return g.contiguous().to(dy.dtype)


def space_to_depth(x, b, inverse):
    if not inverse:
        N, H, W, C = x.shape
        return x.reshape(N, H // b, b, W // b, b, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H // b, W // b, b * b * C)
    N, Hb, Wb, Cb = x.shape
    C = Cb // (b * b)
    return x.reshape(N, Hb, Wb, b, b, C).permute(0, 1, 3, 2, 4, 5).reshape(N, Hb * b, Wb * b, C)


def to_nhwc(src, nchw, cpad, in_scale, mean, std):
    x = src.float() * in_scale
    if nchw:
        x = x.permute(0, 2, 3, 1)
    C = x.shape[-1]
    if mean is not None:
        x = x - mean.float()
    if std is not None:
        x = x / std.float()
    if cpad > C:
        x = F.pad(x, (0, cpad - C))
    return x.contiguous()


def crop_resize(src, meta, Ho, Wo):
    """Bilinear crop+resize(+hflip) of gathered uint8 records (see csrc/augment.hip): the same
    fp32 half-pixel formula as the kernel, rounded half-up."""
    B = meta.shape[0]
    out = torch.empty((B, Ho, Wo, 3), dtype=torch.uint8, device=src.device)
    oy = torch.arange(Ho, dtype=torch.float32)
    ox = torch.arange(Wo, dtype=torch.float32)
    for b in range(B):
        off, H, W, y0, x0, h, w, flip = (int(v) for v in meta[b].tolist())
        img = src[off:off + H * W * 3].view(H, W, 3)[y0:y0 + h, x0:x0 + w].float()
        sy = ((oy + 0.5) * (float(h) / Ho) - 0.5).clamp_min(0)
        sx = ((ox + 0.5) * (float(w) / Wo) - 0.5).clamp_min(0)
        if flip:
            sx = sx.flip(0)
        ya = sy.long().clamp_max(h - 1)
        xa = sx.long().clamp_max(w - 1)
        ly = (sy - ya.float()).view(-1, 1, 1)
        lx = (sx - xa.float()).view(1, -1, 1)
        yb = (ya + 1).clamp_max(h - 1)
        xb = (xa + 1).clamp_max(w - 1)
        a, bb = img[ya][:, xa], img[ya][:, xb]
        c, d = img[yb][:, xa], img[yb][:, xb]
        top = a + (bb - a) * lx
        bot = c + (d - c) * lx
        v = top + (bot - top) * ly
        out[b] = torch.floor(v + 0.5).clamp(0, 255).to(torch.uint8)
    return out


def to_nhwc_s2d(src, nchw, in_scale, mean, std, block=2):
    cq = 4 if block == 2 else 3
    x = to_nhwc(src, nchw, cq, in_scale, mean, std)
    return space_to_depth(x, block, False).contiguous()


def act_bwd(dy, y, act):
    if int(act) == 2:
        return (_f(dy) * _f(y) * (1 - _f(y))).to(dy.dtype)
    return torch.where(y > 0, dy, torch.zeros_like(dy))


def prefix_mask(x, keep):
    D = x.shape[1]
    m = (torch.arange(D, device=x.device) < int(keep.item())).to(x.dtype)
    return x * m


def nested_eval(feat, W, labels):
    # scores for every prefix length: [D,B,C] via cumulative sum (reference-sized; CPU only)
    contrib = feat.float().unsqueeze(2) * W.float().unsqueeze(0)  # [B,D,C]
    scores = contrib.cumsum(1)  # [B,D,C]
    lab = labels.view(-1, 1, 1).expand(-1, scores.shape[1], 1)
    sl = scores.gather(2, lab)
    gt = (scores > sl).sum(2)  # [B,D] (label itself never counted)
    top1 = (gt == 0).sum(0)
    top3 = (gt < 3).sum(0)
    return torch.stack([top1, top3], 1).int()


def dwconv_fwd(x, filt, k, s, p, reflect):
    C = x.shape[-1]
    xin = _nchw(_f(x))
    if reflect and p > 0:
        xin = F.pad(xin, (p, p, p, p), mode="reflect")
        pad = 0
    else:
        pad = p
    w = filt.float().view(1, 1, k, k).expand(C, 1, k, k)
    y = F.conv2d(xin, w, stride=s, padding=pad, groups=C)
    return _nhwc(y).to(x.dtype)


def dwconv_bwd(dy, filt, H, W, k, s, p, reflect):
    x = torch.zeros(dy.shape[0], H, W, dy.shape[-1], requires_grad=True)
    with torch.enable_grad():
        y = dwconv_fwd(x, filt, k, s, p, reflect)
        (g,) = torch.autograd.grad(y, x, _f(dy))
    return g.to(dy.dtype)


def chan_scale_fwd(x, g, res, relu):
    N, C = x.shape[0], x.shape[-1]
    z = _f(x) * _f(g).view(N, *([1] * (x.dim() - 2)), C)
    if res is not None:
        z = z + _f(res)
    if relu:
        z = torch.relu(z)
    return z.to(x.dtype)


def chan_scale_bwd(dy, x, g, res, relu, want_dres):
    N, C = x.shape[0], x.shape[-1]
    gg = _f(g).view(N, *([1] * (x.dim() - 2)), C)
    dz = _f(dy)
    if relu:
        z = _f(x) * gg + (_f(res) if res is not None else 0)
        dz = torch.where(z > 0, dz, torch.zeros_like(dz))
    dx = (dz * gg).to(dy.dtype)
    dg = (dz * _f(x)).reshape(N, -1, C).sum(1).to(g.dtype)  # the gate's dtype, like the GPU op
    return dx, dg, (dz.to(dy.dtype) if want_dres else dy.new_empty(0))


# ----------------------------------------------------------------------------- losses
def xent_fwd(logits, labels, C, smoothing):
    x = _f(logits)[:, :C]
    lse = torch.logsumexp(x, 1)
    xl = x.gather(1, labels.view(-1, 1)).squeeze(1)
    loss = lse - xl
    if smoothing > 0:
        loss = (1 - smoothing) * loss + smoothing * (lse - x.mean(1))
    rank = (x > xl.unsqueeze(1)).sum(1).int()
    return loss, rank


def metric_accum(acc, loss, loss_scale, rank, nrows):
    r = rank[:nrows]
    acc += torch.stack([loss.double().sum() * loss_scale, (r < 1).sum().double(), (r < 3).sum().double(),
                        torch.full((), float(nrows), dtype=torch.float64, device=acc.device)])


def xent_bwd(logits, labels, C, grad_out, scale, smoothing, out_bf16):
    B, ld = logits.shape
    x = _f(logits)[:, :C]
    p = torch.softmax(x, 1)
    tgt = torch.full_like(p, smoothing / C)
    tgt.scatter_add_(1, labels.view(-1, 1), torch.full((B, 1), 1 - smoothing))
    d = torch.zeros(B, ld)
    d[:, :C] = (p - tgt) * (float(grad_out.float().reshape(-1)[0]) * scale)
    return d.to(torch.bfloat16 if out_bf16 else torch.float32)


def log_softmax_fwd(x, C):
    return torch.log_softmax(_f(x)[:, :C], 1)


def log_softmax_bwd(y, dy, ldo, out_bf16):
    d = _f(dy) - torch.exp(y) * _f(dy).sum(1, keepdim=True)
    out = torch.zeros(y.shape[0], ldo)
    out[:, : y.shape[1]] = d
    return out.to(torch.bfloat16 if out_bf16 else torch.float32)


def l2norm_rows(x, ldo, eps, rows_out=-1):
    xf = _f(x)
    n = xf.norm(dim=1).clamp_min(eps)
    y = xf / n.unsqueeze(1)
    inv = 1.0 / n
    pad_r = max(0, rows_out - y.shape[0])
    if ldo > y.shape[1] or pad_r:
        y = F.pad(y, (0, ldo - y.shape[1], 0, pad_r))
        inv = F.pad(inv, (0, pad_r))
    return y, inv


def l2norm_bwd(dy, y, inv, D, out_bf16):
    yf = _f(y)[:, :D]
    dyf = _f(dy)[:, :D]
    dot = (dyf * yf).sum(1, keepdim=True)
    dx = inv.unsqueeze(1) * (dyf - yf * dot)
    return dx.to(torch.bfloat16 if out_bf16 else torch.float32)


def _arc_consts(m):
    return math.cos(m), math.sin(m), math.cos(math.pi - m), math.sin(math.pi - m) * m


def arcface_fwd(cosv, labels, C, s, m, easy, want_logits):
    cm, sm, th, mm = _arc_consts(m)
    cos = _f(cosv)[:, :C]
    c = cos.gather(1, labels.view(-1, 1)).squeeze(1).clamp(-1, 1)
    sn = torch.sqrt((1 - c * c).clamp(0, 1))
    p = c * cm - sn * sm
    dp = cm + torch.where(sn > 1e-6, sm * c / sn.clamp_min(1e-6), torch.zeros_like(c))
    if easy:
        phi = torch.where(c > 0, p, c)
        dphi = torch.where(c > 0, dp, torch.ones_like(c))
    else:
        phi = torch.where(c > th, p, c - mm)
        dphi = torch.where(c > th, dp, torch.ones_like(c))
    logits = s * cos.clone()
    logits.scatter_(1, labels.view(-1, 1), (s * phi).view(-1, 1))
    loss = torch.logsumexp(logits, 1) - s * phi
    rank = (logits > (s * phi).unsqueeze(1)).sum(1).int()
    return loss, rank, dphi, (logits if want_logits else torch.empty(0))


def arcface_bwd(cosv, labels, C, s, m, easy, dphi, grad_out, scale):
    B, ld = cosv.shape
    cm, sm, th, mm = _arc_consts(m)
    cos = _f(cosv)[:, :C]
    c = cos.gather(1, labels.view(-1, 1)).squeeze(1).clamp(-1, 1)
    sn = torch.sqrt((1 - c * c).clamp(0, 1))
    p = c * cm - sn * sm
    phi = torch.where(c > 0, p, c) if easy else torch.where(c > th, p, c - mm)
    logits = s * cos.clone()
    logits.scatter_(1, labels.view(-1, 1), (s * phi).view(-1, 1))
    pr = torch.softmax(logits, 1)
    oh = torch.zeros_like(pr).scatter_(1, labels.view(-1, 1), 1.0)
    mult = torch.ones_like(pr).scatter_(1, labels.view(-1, 1), dphi.view(-1, 1))
    g = float(grad_out.float().reshape(-1)[0]) * scale
    d = torch.zeros(B, ld)
    d[:, :C] = g * s * (pr - oh) * mult
    return d.to(cosv.dtype)


def transpose2d(x):
    return x.t().contiguous()


# ----------------------------------------------------------------------------- dropout / adaptive pool
def _drop_mask(shape, p, seed, offset, device):
    g = torch.Generator().manual_seed((int(seed) * 1000003 + int(offset)) & ((1 << 63) - 1))
    return (torch.rand(shape, generator=g) >= p).to(device)


def dropout_fwd(x, p, seed, offset):
    used = offset.clone()
    y = (_f(x) * _drop_mask(x.shape, p, seed, int(used.item()), x.device) / (1.0 - p)).to(x.dtype)
    offset.add_(1)
    return y, used


def dropout_bwd(dy, p, seed, used):
    return (_f(dy) * _drop_mask(dy.shape, p, seed, int(used.item()), dy.device) / (1.0 - p)).to(dy.dtype)


def adaptive_avg_pool(x, oh, ow):
    return _nhwc(F.adaptive_avg_pool2d(_nchw(_f(x)), (oh, ow))).to(x.dtype)


def adaptive_avg_pool_bwd(dy, H, W):
    N, OH, OW, C = dy.shape
    xin = torch.zeros(N, C, H, W, dtype=torch.float64, requires_grad=True)
    with torch.enable_grad():  # called from an autograd backward, where grad mode is off
        y = F.adaptive_avg_pool2d(xin, (OH, OW))
        y.backward(_nchw(dy.double()))
    return _nhwc(xin.grad).to(dy.dtype)


def iabn_gamma(g, eps):
    e = g.abs() + eps
    return e, 1.0 / e


def sign_mul(d, g):
    return d * torch.sign(g)


def s2d_weight(w7, w16):
    """In place: w16 = the space-to-depth 4x4 form of the 7x7 stem weight (functional.stem_s2d_weight)."""
    from .functional import stem_s2d_weight

    w16.copy_(stem_s2d_weight(w7.float()))


def s2d_weight_bwd(g16, C):
    Co = g16.shape[0]
    g8 = g16.float().reshape(Co, 4, 4, 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(Co, 8, 8, 4)
    return g8[:, 1:, 1:, :C].contiguous()



def se_gate_fwd(p, w1, b1, w2, b2, R):
    """Squeeze-excitation gate h = relu(p W1^T + b1), g = sigmoid(h W2^T + b2) with the unfused chain's
    bf16 roundings (h and g)."""
    C = p.shape[1]
    a = _f(p) @ _f(w1[:R]).t()
    if b1 is not None:
        a = a + _f(b1)[:R]
    h = torch.relu(a).to(p.dtype)
    z = _f(h) @ _f(w2[:C]).t()
    if b2 is not None:
        z = z + _f(b2)[:C]
    return h, torch.sigmoid(z).to(p.dtype)


def se_gate_bwd(dg, g, h, p, w1t, w2t):
    """w1t = W1^T [C, >=R], w2t = W2^T [R, >=C] (the transposed prepared weights)."""
    C, R = p.shape[1], h.shape[1]
    d2 = (_f(dg) * _f(g) * (1 - _f(g))).to(p.dtype)
    dw2 = _f(d2).t() @ _f(h)
    db2 = _f(d2).sum(0)
    dh = (_f(d2) @ _f(w2t[:, :C]).t()).to(p.dtype)
    d1 = torch.where(h > 0, dh, torch.zeros_like(dh))
    dw1 = _f(d1).t() @ _f(p)
    db1 = _f(d1).sum(0)
    dp = (_f(d1) @ _f(w1t[:, :R]).t()).to(p.dtype)
    return dp, dw1, db1, dw2, db2
