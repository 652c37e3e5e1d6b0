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
