"""Named kernel-configuration slots (mirror of ``csrc/tune.h``).

The HIP library selects kernel variants from a small table of integer switches (0 = the shipped
heuristic): in-process A/B experiments (``tools/conv_bench.py --cfgs``), the per-shape conv
autotuner, and ``DCP_TUNE="name=value,..."`` from the environment.  Python code addresses a slot
only by name through this module; ``SLOTS`` must equal the library's own table (checked against
``csrc/tune.h`` by tests/test_tuning_cpu.py and against the loaded library by :func:`verify`).
"""
from __future__ import annotations

SLOTS = {
    "tg_tile_n": 0, "tg_stages": 1, "ablate": 2, "tg_pingpong": 3, "tg_big_cvar": 4, "wg_splits_per_cu": 5,
    "wg_flush_ablate": 6, "wg_tile_mode": 7, "tg_kdepth": 8, "ew_grid_cap": 9, "ew_rows": 10,
    "bn_act_variant": 11, "wg_rows": 12, "narrow_kdepth": 13, "wg_cols": 14, "wg3x3": 15, "gconv_sg": 16,
    "stem_ablate": 17, "c3_off": 18, "c3_variant": 19, "dgrad_parity_streams": 20, "tg_big_stages": 21, "tg_big_persist": 22, "tg_big_sk": 23, "tg_big": 24, "autotune": 25, "gconv_spw": 26, "wg_split_cap": 27,
    "bn_bwd_cap": 28, "row_reduce": 29, "c3_epilogue": 30, "c3_window_kb": 31, "tg_ws": 32, "tg_ps": 33,
    "bn_fin_act": 34, "tg_split_k": 35,
}
NUM_SLOTS = 40
# the loaded library's own table (set by verify); apply() skips names it does not have at the same
# index -- a DCP_LIB build from another tree may number its slots differently
LIB_SLOTS = None


def slot(name) -> int:
    """Slot index of ``name`` (a registered name, or a plain integer for old-style specs)."""
    if isinstance(name, int):
        return name
    name = str(name).strip()
    if name.lstrip("-").isdigit():
        return int(name)
    try:
        return SLOTS[name]
    except KeyError:
        raise KeyError(f"unknown tuning slot {name!r}; known: {', '.join(sorted(SLOTS))}") from None


def parse_spec(spec: str, sep: str = ","):
    """``"tg_tile_n=64,tg_stages=3"`` (or ``;``-separated) -> [(slot, value), ...]."""
    out = []
    for kv in filter(None, (t.strip() for t in (spec or "").replace(";", sep).split(sep))):
        k, v = kv.split("=")
        out.append((slot(k), int(v)))
    return out


def apply(K, spec, reset: bool = False):
    """Set the slots of ``spec`` on the kernel library ``K`` (optionally zeroing every slot first)."""
    if reset:
        for i in range(NUM_SLOTS):
            K.set_tuning(i, 0)
    items = []
    if isinstance(spec, str):
        for kv in filter(None, (t.strip() for t in (spec or "").replace(";", ",").split(","))):
            k, v = kv.split("=")
            items.append((k.strip(), int(v)))
    else:
        items = list(spec)
    for name, v in items:
        i = slot(name)
        if LIB_SLOTS is not None and not isinstance(name, int) and not str(name).strip().lstrip("-").isdigit():
            if LIB_SLOTS.get(str(name).strip()) != i:
                import warnings

                warnings.warn(f"tuning slot {name!r} (index {i}) is not in the loaded library's table; skipped")
                continue
        K.set_tuning(i, int(v))


def verify(K) -> None:
    """Fail loudly if the loaded library's slot table differs from this mirror."""
    global LIB_SLOTS
    lib = {}
    for kv in filter(None, K.tuning_slots().split(";")):
        k, v = kv.split("=")
        lib[k] = int(v)
    LIB_SLOTS = lib
    if lib != SLOTS:
        raise RuntimeError(f"tuning slot table mismatch: library {lib} vs tuning.py {SLOTS} (stale build?)")


def parse_header(path: str):
    """The name -> slot table of csrc/tune.h (tests)."""
    import re

    text = open(path).read()
    enum = {k: int(v) for k, v in re.findall(r"\b(k\w+)\s*=\s*(\d+)", text)}
    return {name: enum[ident] for name, ident in re.findall(r'\{"(\w+)",\s*(k\w+)\}', text)}


def load_cache(K, path: str) -> int:
    """Replay an autotuning cache written by :func:`save_cache`: every listed problem runs the
    recorded kernel configuration without being timed again (returns the entries accepted)."""
    import os

    if not path or not os.path.exists(path):
        return 0
    with open(path) as f:
        return int(K.autotune_import(f.read()))


def save_cache(K, path: str) -> int:
    """Write the autotuner's decisions of this process (merged with what ``path`` already holds)
    atomically: the per-shape choices of ``cudnn.benchmark``-style tuning, kept across processes so
    a later run uses exactly the same kernels (reproducible numerics, profiles without tuning)."""
    import os
    import tempfile

    if not path:
        return 0
    if os.path.exists(path):
        load_cache(K, path)  # merge: entries of this process win (imported first, then re-exported)
    text = K.autotune_export()
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tune_cache.")
    with os.fdopen(fd, "w") as f:
        f.write(text)
    os.replace(tmp, path)
    return text.count("\n")
