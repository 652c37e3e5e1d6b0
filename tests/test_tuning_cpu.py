"""The named kernel-configuration slots: the Python mirror equals csrc/tune.h, names and specs
parse, unknown names fail loudly."""
import os

import pytest

from ddp_classification_pytorch_amd import tuning

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_python_mirror_matches_header():
    hdr = tuning.parse_header(os.path.join(ROOT, "ddp_classification_pytorch_amd", "csrc", "tune.h"))
    assert hdr == tuning.SLOTS
    assert len(set(hdr.values())) == len(hdr) and max(hdr.values()) < tuning.NUM_SLOTS


def test_parse_spec_names_and_indices():
    assert tuning.parse_spec("tg_tile_n=64,tg_stages=3") == [(0, 64), (1, 3)]
    assert tuning.parse_spec("tg_big=2;autotune=1") == [(24, 2), (25, 1)]
    assert tuning.parse_spec("8=32") == [(8, 32)]
    assert tuning.parse_spec("") == []


def test_unknown_slot_raises():
    with pytest.raises(KeyError, match="unknown tuning slot"):
        tuning.slot("no_such_slot")


def test_apply_sets_slots():
    class Fake:
        def __init__(self):
            self.t = [0] * tuning.NUM_SLOTS

        def set_tuning(self, i, v):
            self.t[i] = v

    k = Fake()
    k.t[5] = 9
    tuning.apply(k, "tg_pingpong=1,wg_rows=32", reset=True)
    assert k.t[3] == 1 and k.t[12] == 32 and k.t[5] == 0


def test_autotune_cache_round_trip(tmp_path):
    """DCP_TUNE_CACHE: the autotuner's per-shape decisions survive a save / load (merged, atomic
    file), malformed or out-of-range lines are skipped (the library refuses choices its candidate
    table does not have)."""
    import pytest

    from ddp_classification_pytorch_amd import _ext, tuning

    if not _ext.try_load():
        pytest.skip("kernel library not built")
    K = _ext.hip_ops()
    n = K.autotune_import("tg\tcachetest 1 2 3|000000|\t5\nwg\tcachetest 7 7 64\t3\ntg\tcachetest bad\t9999\n"
                          "zz\tq\t1\nnot a line\n")
    assert n == 2
    path = tmp_path / "sub" / "tune.txt"
    assert tuning.save_cache(K, str(path)) >= 2
    text = path.read_text()
    assert "tg\tcachetest 1 2 3|000000|\t5\n" in text and "wg\tcachetest 7 7 64\t3\n" in text
    assert "cachetest bad" not in text
    assert tuning.load_cache(K, str(path)) == text.count("\n")
    assert tuning.load_cache(K, str(tmp_path / "missing.txt")) == 0
