"""Race detection and memory checking of the native host code: the shard
loader's thread pool (csrc/host/loader.cpp) built with AddressSanitizer + UBSan and with
ThreadSanitizer, driven by tests/native/loader_sanitize.cpp with every batch in flight at
once.  Host code only -- GPU sanitizers are not available on this pool."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from ddp_classification_pytorch_amd.data.shards import write_shard

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "native", "loader_sanitize.cpp")
CXX = shutil.which("g++") or shutil.which("clang++")


@pytest.fixture(scope="module")
def shard(tmp_path_factory):
    rng = np.random.default_rng(3)
    imgs = [(rng.integers(0, 256, (int(rng.integers(8, 60)), int(rng.integers(8, 60)), 3), dtype=np.uint8), i)
            for i in range(53)]
    p = str(tmp_path_factory.mktemp("san") / "s.dcps")
    write_shard(p, imgs)
    return p


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_loader_under_sanitizer(tmp_path, shard, san):
    exe = str(tmp_path / f"loader_{san.split(',')[0]}")
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-pthread", f"-fsanitize={san}", "-fno-omit-frame-pointer", DRIVER,
           "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitizer" in (r.stderr or "").lower():
        pytest.skip(f"{san} sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    run = subprocess.run([exe, shard], capture_output=True, text=True, env=env, timeout=300)
    out = run.stdout + run.stderr
    assert run.returncode == 0, out[-3000:]
    assert "loader_sanitize ok=1" in out
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "runtime error" not in out
