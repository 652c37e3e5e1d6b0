"""Loader for the in-tree gfx950 kernel library (`_dcp_kernels.so`).

GPU tensors are ALWAYS served by the HIP kernels: if the library is missing
or fails to load while a GPU op is requested, this raises instead of
silently falling back to PyTorch/MIOpen.  CPU tensors use the reference
math in :mod:`ddp_classification_pytorch_amd.ops._ref` (tests and gloo
plumbing only).

Set ``DCP_AUTOBUILD=1`` to compile the library on first use when it is
missing (needs hipcc), ``DCP_AUTOTUNE=1`` to time the conv GEMM configurations per problem
shape on first use and keep the fastest (like ``cudnn.benchmark``), ``DCP_TUNE="name=v,..."``
to override kernel configuration slots (A/B experiments).
"""
from __future__ import annotations

import os
import threading

import torch

# DCP_LIB: load another build of the library (same-box A/B of two kernel versions)
LIB_PATH = os.environ.get("DCP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dcp_kernels.so")
_lock = threading.Lock()
_state = {"loaded": False, "error": None}


def library_path() -> str:
    return LIB_PATH


def try_load() -> bool:
    """Load the kernel library if present; returns True when torch.ops.dcp is usable."""
    if _state["loaded"]:
        return True
    with _lock:
        if _state["loaded"]:
            return True
        if not os.path.exists(LIB_PATH) and os.environ.get("DCP_AUTOBUILD", "0") == "1":
            from . import build_ext

            build_ext.build(verbose=False)
        if not os.path.exists(LIB_PATH):
            _state["error"] = f"kernel library not built: {LIB_PATH} (run python -m ddp_classification_pytorch_amd.build_ext)"
            return False
        try:
            torch.ops.load_library(LIB_PATH)
        except Exception as e:  # pragma: no cover - exercised only on broken builds
            _state["error"] = f"failed to load {LIB_PATH}: {e}"
            return False
        _state["loaded"] = True
        from . import tuning

        if os.environ.get("DCP_LIB"):
            # another build (same-box A/B): its slot table may predate this tree's; only the slots
            # both share are meaningful, so a mismatch is reported, not fatal
            try:
                tuning.verify(torch.ops.dcp)
            except RuntimeError as e:
                import warnings

                warnings.warn(f"DCP_LIB={LIB_PATH}: {e}")
        else:
            tuning.verify(torch.ops.dcp)
        if os.environ.get("DCP_AUTOTUNE", "0") == "1":
            # per-shape timing of the conv GEMM configurations on first use (conv_igemm.hip)
            torch.ops.dcp.set_tuning(tuning.slot("autotune"), 1)
        # A/B experiments: DCP_TUNE="name=value,..." (csrc/tune.h names) sets kernel-config
        # overrides in any process that loads the library (bench.py, main.py, tests)
        tuning.apply(torch.ops.dcp, os.environ.get("DCP_TUNE", ""))
        return True


def hip_ops():
    """torch.ops.dcp, loading the library; raises loudly if it is unavailable."""
    if not try_load():
        raise RuntimeError("gfx950 kernels unavailable for a GPU op: " + str(_state["error"]))
    return torch.ops.dcp


def is_loaded() -> bool:
    return _state["loaded"]
