"""Build driver for the gfx950 HIP extension (`_dcp_kernels.so`, in-tree).

Compiles every `csrc/*.hip` kernel file with `hipcc --offload-arch=gfx950`
(no hipify, no multi-arch fat binary) and `csrc/bindings.cpp` (the
TORCH_LIBRARY operator registrations) against the installed PyTorch-ROCm
headers, then links one shared object next to this file.  Objects are
rebuilt only when a source or header is newer; independent objects compile
in parallel.

    python -m ddp_classification_pytorch_amd.build_ext [-j N] [--force]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB_NAME = "_dcp_kernels.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
# host-only native runtime pieces (no torch, no device code), loaded with ctypes
HOST_SRC = os.path.join(CSRC, "host")
LOADER_PATH = os.path.join(HERE, "_dcp_loader.so")
ARCH = os.environ.get("DCP_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the extension)")


def _torch_paths():
    import torch  # noqa: F401  (only for paths)

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(root, "lib")


COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"]
# per-file extras: the stem kernel's statistics run beside MFMAs, where packed fp32 (which the
# SLP vectorizer forms from adjacent scalar adds / FMAs) issues slower than scalar fp32
FILE_FLAGS = {"stem.hip": ["-fno-slp-vectorize"]}


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".cuh"))]


def _stale(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, obj: str, torch_inc, force: bool) -> str:
    deps = [src] + _headers() + [os.path.abspath(__file__)]
    if not force and not _stale(obj, deps):
        return f"up-to-date {os.path.basename(obj)}"
    cmd = [_hipcc()] + COMMON_FLAGS
    if src.endswith(".hip"):
        cmd += [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-x", "hip"]
        cmd += FILE_FLAGS.get(os.path.basename(src), [])
    else:
        # host-only translation unit (bindings): torch headers, no device code
        cmd += ["-D_GLIBCXX_USE_CXX11_ABI=1"] + [f"-I{p}" for p in torch_inc]
        cmd += ["-Wno-unused-result", "-Wno-deprecated-declarations"]
    cmd += ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return f"built {os.path.basename(obj)}"


def build_host(force: bool = False, verbose: bool = True) -> str:
    """The shard loader (`csrc/host/loader.cpp`): plain C++17 + pthreads, C ABI for ctypes."""
    srcs = sorted(os.path.join(HOST_SRC, f) for f in os.listdir(HOST_SRC) if f.endswith(".cpp"))
    if force or _stale(LOADER_PATH, srcs + [os.path.abspath(__file__)]):
        cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
        if not cxx:
            raise RuntimeError("no host C++ compiler (g++) found for the shard loader")
        tmp = LOADER_PATH + f".tmp{os.getpid()}"
        cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-o", tmp] + srcs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"host build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LOADER_PATH)
        if verbose:
            print("[dcp-build] linked", LOADER_PATH, flush=True)
    return LOADER_PATH


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    build_host(force=force, verbose=verbose)
    torch_inc, torch_lib = _torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    objs = [os.path.join(BUILD, os.path.basename(s) + ".o") for s in srcs]
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for msg in ex.map(lambda so: _compile(so[0], so[1], torch_inc, force), zip(srcs, objs)):
            if verbose:
                print("[dcp-build]", msg, flush=True)
    # the object list of the last link: a source added or REMOVED since then relinks too (a removed
    # file leaves every remaining object older than the library)
    manifest = os.path.join(BUILD, "link_manifest.txt")
    listing = "\n".join(os.path.basename(o) for o in objs)
    old_listing = open(manifest).read() if os.path.exists(manifest) else None
    if force or _stale(LIB_PATH, objs) or old_listing != listing:
        tmp = LIB_PATH + f".tmp{os.getpid()}"
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
        cmd += [f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                "-ltorch_hip", "-lamdhip64"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB_PATH)
        with open(manifest, "w") as f:
            f.write(listing)
        if verbose:
            print("[dcp-build] linked", LIB_PATH, flush=True)
    return LIB_PATH


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
