from .fused import FusedAdam, FusedSGD
from .schedulers import LinearWarmup, MultiStepLR, StepLR


def build_optimizer(name: str, params, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                    nesterov: bool = False, betas=(0.9, 0.999)):
    name = name.lower()
    if name == "sgd":
        return FusedSGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov)
    if name in ("adam", "adamw"):
        return FusedAdam(params, lr=lr, betas=betas, weight_decay=weight_decay, decoupled=name == "adamw")
    raise ValueError(f"unknown optimizer {name}")


__all__ = ["FusedSGD", "FusedAdam", "LinearWarmup", "MultiStepLR", "StepLR", "build_optimizer"]
