"""Model zoo (NHWC, gfx950 kernels).  ``build_model(name, num_classes)``."""
from .layers import BatchNorm2d, Conv2d, ConvBN, Linear
from .resnet import (ResNet, build_resnet, cifar_resnet18, cifar_resnet34, cifar_resnet50, cifar_resnet101,
                     cifar_resnet152, resnet18, resnet34, resnet50, resnet101, resnet152, resnext50_32x4d)

MODEL_NAMES = ["resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "resnext50_32x4d", "resnext101_32x8d",
               "cifar_resnet18", "cifar_resnet34", "cifar_resnet50", "cifar_resnet101", "cifar_resnet152",
               "tresnet_m", "vgg19_bn"]


def build_model(name: str, num_classes: int = 1000, **kw):
    name = name.lower()
    if name in ("tresnet", "tresnet_m", "tresnet_m_miil_in21k"):
        from .tresnet import tresnet_m

        return tresnet_m(num_classes=num_classes, **kw)
    if name in ("vgg19_bn", "vgg19"):
        from .vgg import vgg19_bn

        return vgg19_bn(num_classes=num_classes, **kw)
    return build_resnet(name, num_classes=num_classes, **kw)


def input_layout(model) -> dict:
    """How the device input pipeline should lay out images for ``model``:
    ``{"cpad": channels per pixel, "s2d": space-to-depth stem input}``
    (kwargs of :func:`ops.functional.to_device_nhwc` / the loaders)."""
    mods = list(model.modules())
    if any(getattr(m, "stem_s2d", False) for m in mods):
        return {"cpad": 8, "s2d": True}
    if any(type(m).__name__ == "TResNet" for m in mods):
        return {"cpad": 3, "s2d": 4}  # SpaceToDepth(4) stem input written by the input kernel
    return {"cpad": 8, "s2d": False}


__all__ = ["BatchNorm2d", "Conv2d", "ConvBN", "Linear", "ResNet", "build_model", "input_layout", "build_resnet", "MODEL_NAMES",
           "resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "resnext50_32x4d", "cifar_resnet18",
           "cifar_resnet34", "cifar_resnet50", "cifar_resnet101", "cifar_resnet152"]
