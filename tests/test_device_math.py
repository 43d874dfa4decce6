"""Device math helpers (csrc/mpcg_device.h) checked on the host against the C library.

fsincos, fatan and fatan2 replace the ROCm device library's functions in the bicycle
instance (no large-argument / special-value branches whose registers the linearisation
otherwise holds): sin / cos within 1 ulp of the C library over the argument ranges the
path sees (sin(-0) = -0), atan / atan2 within 2 ulp with the IEEE quotient (the device
uses frcp, itself within 1 ulp), and the atan2 quadrants and limits exact.
"""
import math
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd", "csrc")


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_fsincos_within_one_ulp(tmp_path):
    exe = str(tmp_path / "device_math")
    subprocess.run(["hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", f"-I{ROOT}/include", f"-I{CSRC}",
                    "-x", "hip", os.path.join(ROOT, "tests", "cpp", "test_device_math.cpp"), "-o", exe],
                   check=True, capture_output=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    rows = [ln.split() for ln in out if ln.startswith("range")]
    assert len(rows) == 6
    for r in rows:
        assert int(r[3]) <= 1 and int(r[5]) <= 1, r
    arows = [ln.split() for ln in out if ln.startswith("arange")]
    assert len(arows) == 6
    for r in arows:
        assert int(r[3]) <= 2 and int(r[5]) <= 2, r
    sp = [float(v) for v in next(ln for ln in out if ln.startswith("aspecial")).split()[1:]]
    assert sp[0] == math.pi and sp[1] == math.pi / 2 and sp[2] == -math.pi / 2
    assert sp[3] == math.pi / 2 and sp[4] == math.pi / 2 and sp[5] == 1.0
    neg = next(ln for ln in out if ln.startswith("negzero")).split()
    assert neg[1] == "1" and float(neg[2]) == 1.0
