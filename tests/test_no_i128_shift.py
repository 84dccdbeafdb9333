"""No device code of libchordx shifts a 128-bit value by a variable amount
(round 6): every such shift goes through cx_common.hpp's
64-bit-half helpers (pow2_128 / shr128 / shl128 / bits64).  The round-5
level-plane route-table build wrote nondeterministic words in lanes 48-63
around a compiled `u128 >> gs` (tests/test_gpu_u128.py, profiles/r06/u128/).

CPU test: compiles each HIP source's device side to LLVM IR (hipcc, gfx950)
and counts `shl` / `lshr` / `ashr` of i128 whose amount is not a constant."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "p2p-dhts_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
VAR_SHIFT = re.compile(r"= (shl|lshr|ashr) i128 %[\w.]+, %[\w.]+")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src", ["cx_kernels.hip", "cx_walk.hip", "cx_api.hip"])
def test_no_variable_i128_shift_in_device_code(src, tmp_path):
    out = tmp_path / (src + ".ll")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "--cuda-device-only", "-S", "-emit-llvm", os.path.join(CSRC, src),
                        "-o", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    ir = out.read_text()
    if src != "cx_api.hip":  # the API file launches kernels, it defines none
        assert "define" in ir
    hits = VAR_SHIFT.findall(ir)
    assert not hits, f"{src}: {len(hits)} variable i128 shifts in device code"
    shutil.rmtree(tmp_path, ignore_errors=True)
