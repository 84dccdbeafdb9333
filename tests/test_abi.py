"""The C-ABI library loads and exports every symbol include/chordx.h declares
(CPU-only; no compute call is made without a GPU except to show it fails)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    txt = open(os.path.join(ROOT, "include", "chordx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cx_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    import chordx._lib as L
    lib = L.lib()
    declared = _declared()
    assert len(declared) >= 20
    assert set(declared) == set(L.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name


def test_version_and_device_count():
    import chordx
    assert chordx.lib().cx_version() == 1
    n = chordx.device_count()
    assert n >= 0


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES", None) is None and
                    os.path.exists("/dev/kfd"), reason="a GPU may be present")
def test_no_host_fallback_without_gpu():
    """Without a HIP device every compute entry fails with CX_E_HIP."""
    import numpy as np
    import chordx
    from chordx._lib import CX_E_HIP
    if chordx.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(chordx.ChordError) as e:
        chordx.Ring(np.zeros((4, 2), np.uint64))
    assert e.value.code == CX_E_HIP and "no host compute path" in str(e.value)
    with pytest.raises(chordx.ChordError):
        chordx.in_between(np.zeros((1, 4)), np.zeros((1, 4)), np.zeros((1, 4)))


def test_chordkey_host_values():
    """ChordKey mirror: construction/formatting/arithmetic (key.h:41-47,70-93,236-270)."""
    from chordx import ChordKey
    k = ChordKey("091186395ae2562aaa1ff7f3513747e9")
    assert str(k) == "91186395ae2562aaa1ff7f3513747e9"  # no leading zero
    assert (ChordKey(1) - 1).value == 1 << 128
    assert (ChordKey(0) - 1).value == (1 << 256) - 1
    assert ((ChordKey(0) - 1) + 1).value == 0
    assert (ChordKey((1 << 128) - 1) + 1).value == 0
    assert (ChordKey(5) - ChordKey(5)).value == 1 << 128
