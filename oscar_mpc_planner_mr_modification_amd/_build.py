"""In-tree build of the HIP backend (libmpcg.so, gfx950) and of the C++
drop-in `MPCPlanner::Solver` shim.  Outputs stay inside the package directory
(git-ignored, but they travel to the GPU box with the snapshot)."""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libmpcg.so")
ARCH = os.environ.get("MPCG_OFFLOAD_ARCH", "gfx950")

SOURCES = ["mpcg_kernels.hip"]
HEADERS = ["mpcg_device.h", "mpcg_sqp.h"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(INCLUDE, "mpcg.h"), __file__]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           f"-I{INCLUDE}", f"-I{CSRC}", "-o", LIB + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build_lib(force=True, verbose=True))
