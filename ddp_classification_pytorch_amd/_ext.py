"""Loader for the in-tree gfx950 kernel library (`_dcp_kernels.so`).

GPU tensors are ALWAYS served by the HIP kernels: if the library is missing
or fails to load while a GPU op is requested, this raises instead of
silently falling back to PyTorch/MIOpen.  CPU tensors use the reference
math in :mod:`ddp_classification_pytorch_amd.ops._ref` (tests and gloo
plumbing only).

Set ``DCP_AUTOBUILD=1`` to compile the library on first use when it is
missing (needs hipcc), ``DCP_AUTOTUNE=1`` to time the conv GEMM configurations per problem
shape on first use and keep the fastest (like ``cudnn.benchmark``), ``DCP_TUNE="name=v,..."``
to override kernel configuration slots (A/B experiments), ``DCP_TUNE_CACHE=<file>`` to replay the
autotuner's per-shape decisions recorded by an earlier process (and record this process's new ones
there at exit): the same kernels run to run, and no tuning dispatches in a profile.
"""
from __future__ import annotations

import os
import threading

import torch

# DCP_LIB: load another build of the library (same-box A/B of two kernel versions)
LIB_PATH = os.environ.get("DCP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dcp_kernels.so")
_lock = threading.Lock()
_state = {"loaded": False, "error": None, "failed": False}


def library_path() -> str:
    return LIB_PATH


def try_load() -> bool:
    """Load the kernel library if present; returns True when torch.ops.dcp is usable."""
    if _state["loaded"]:
        return True
    with _lock:
        if _state["loaded"]:
            return True
        if _state["failed"]:  # loaded once and found unusable (stale slot table): stays refused
            return False
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
        from . import tuning

        # the slot table is checked BEFORE the library counts as loaded: a stale build is refused on
        # this and every later call (the error is kept), never used half-verified
        if os.environ.get("DCP_LIB"):
            # another build (same-box A/B): its slot table may predate this tree's; only the slots
            # both share (same name AND index) are meaningful -- tuning.apply skips the others
            try:
                tuning.verify(torch.ops.dcp)
            except RuntimeError as e:
                import warnings

                warnings.warn(f"DCP_LIB={LIB_PATH}: {e}; DCP_TUNE entries not in its table are skipped")
        else:
            try:
                tuning.verify(torch.ops.dcp)
            except RuntimeError as e:
                _state["error"], _state["failed"] = f"{LIB_PATH}: {e}", True
                raise
        _state["loaded"] = True
        if os.environ.get("DCP_AUTOTUNE", "0") == "1":
            # per-shape timing of the conv GEMM configurations on first use (conv_igemm.hip)
            torch.ops.dcp.set_tuning(tuning.slot("autotune"), 1)
        # A/B experiments: DCP_TUNE="name=value,..." (csrc/tune.h names) sets kernel-config
        # overrides in any process that loads the library (bench.py, main.py, tests)
        tuning.apply(torch.ops.dcp, os.environ.get("DCP_TUNE", ""))
        cache = os.environ.get("DCP_TUNE_CACHE")
        if cache:
            tuning.load_cache(torch.ops.dcp, cache)
            if os.environ.get("RANK", "0") == "0":  # one writer (every rank tunes the same shapes)
                import atexit

                atexit.register(_save_cache, cache)
        return True


def _save_cache(path):
    from . import tuning

    try:
        tuning.save_cache(torch.ops.dcp, path)
    except Exception as e:  # noqa: BLE001 - never fail a finished run over the cache
        import sys

        print(f"[dcp] tuning cache {path} not written: {e}", file=sys.stderr)


def hip_ops():
    """torch.ops.dcp, loading the library; raises loudly if it is unavailable."""
    if not try_load():
        raise RuntimeError("gfx950 kernels unavailable for a GPU op: " + str(_state["error"]))
    return torch.ops.dcp


def is_loaded() -> bool:
    return _state["loaded"]
