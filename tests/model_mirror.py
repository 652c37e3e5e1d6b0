"""Plain-PyTorch (NCHW, fp32, autograd) rendering of our NHWC ResNet using the
SAME parameter tensors — the oracle for end-to-end model parity tests."""
import torch
import torch.nn.functional as F

from ddp_classification_pytorch_amd.models.resnet import BasicBlock, Bottleneck


def _conv(x, conv):
    w = conv.weight.permute(0, 3, 1, 2)
    return F.conv2d(x, w, stride=conv.stride, padding=conv.padding, groups=conv.groups)


def _bn(x, bn, training):
    rm = bn.running_mean.clone()
    rv = bn.running_var.clone()
    return F.batch_norm(x, rm, rv, bn.weight, bn.bias, training=training, momentum=bn.momentum, eps=bn.eps)


def mirror_forward(model, x_nchw, training=True):
    y = F.relu(_bn(_conv(x_nchw, model.conv1), model.bn1, training))
    if model.variant == "imagenet":
        y = F.max_pool2d(y, 3, 2, 1)
    for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
        for blk in layer:
            r = y
            if blk.downsample is not None:
                r = _bn(_conv(y, blk.downsample[0]), blk.downsample[1], training)
            if isinstance(blk, Bottleneck):
                z = F.relu(_bn(_conv(y, blk.conv1), blk.bn1, training))
                z = F.relu(_bn(_conv(z, blk.conv2), blk.bn2, training))
                z = _bn(_conv(z, blk.conv3), blk.bn3, training)
            else:
                z = F.relu(_bn(_conv(y, blk.conv1), blk.bn1, training))
                z = _bn(_conv(z, blk.conv2), blk.bn2, training)
            y = F.relu(z + r)
    f = y.mean((2, 3))
    return F.linear(f, model.fc.weight, model.fc.bias) if model.fc is not None else f
