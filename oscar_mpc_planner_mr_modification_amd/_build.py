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

# source -> extra flags.  The producers are compiled without floating-point
# contraction so that they agree bit for bit with the host restatement.
SOURCES = {"mpcg_kernels.hip": [], "mpcg_prepare.hip": ["-ffp-contract=off"]}
HEADERS = ["mpcg_device.h", "mpcg_sqp.h", "mpcg_prepare.h", "mpcg_bicycle.h"]
HOST_SOURCES = ["host/mpcg_yaml.cpp", "host/mpcg_solver.cpp"]
HOST_HEADERS = ["mpc_planner_solver/mpcg_yaml.h", "mpc_planner_solver/mpcg_config.h", "mpc_planner_solver/state.h",
                "mpc_planner_solver/mpcg_solver_interface.h", "mpc_planner_solver/solver_interface.h"]
BUILD = os.path.join(PKG, "build")


def source_hash() -> str:
    """sha256 over the HIP kernel sources, the C ABI header and the build flags: the identity of
    the kernels a PMC profile was taken on (bench.py drops counters of other sources)."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(list(SOURCES) + HEADERS):
        h.update(f.encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(INCLUDE, "mpcg.h"), "rb") as fh:
        h.update(fh.read())
    h.update(repr((ARCH, sorted(SOURCES.items()))).encode())
    return h.hexdigest()


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = False, extra_flags=(), out: str = LIB) -> str:
    deps = [os.path.join(CSRC, s) for s in list(SOURCES) + HEADERS] + [os.path.join(INCLUDE, "mpcg.h"), __file__]
    if not force and not _stale(out, deps):
        return out
    objdir = os.path.join(BUILD, "obj" + ("_" + "_".join(f.strip("-").replace("=", "") for f in extra_flags)
                                          if extra_flags else ""))
    os.makedirs(objdir, exist_ok=True)
    common = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{INCLUDE}", f"-I{CSRC}"]
    objs, procs = [], []
    for src, flags in SOURCES.items():
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        cmd = common + list(flags) + list(extra_flags) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, "hipcc")
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_cpp(config: str = "C2", force: bool = False, verbose: bool = False) -> dict:
    """The drop-in C++ MPCPlanner::Solver for one generated solver
    (dimensions are compile-time, as in the reference): codegen into
    build/<config>/, then libmpc_planner_solver.so and the test program
    tests/cpp/test_solver.cpp linked against libmpcg.so."""
    from . import codegen
    from .layouts import config_layout

    lib_mpcg = build_lib()
    out = os.path.join(BUILD, config)
    codegen.generate(config_layout(config), out)
    so = os.path.join(out, "libmpc_planner_solver.so")
    exe = os.path.join(out, "test_solver")
    srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES] + [os.path.join(out, "mpc_planner_parameters.cpp")]
    deps = srcs + [os.path.join(INCLUDE, h) for h in HOST_HEADERS] + [os.path.join(INCLUDE, "mpcg.h"), lib_mpcg,
                                                                     __file__]
    inc = [f"-I{os.path.join(out, 'include')}", f"-I{INCLUDE}"]
    if force or _stale(so, deps):
        cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-Wextra"] + inc + srcs + \
              ["-o", so + ".tmp", f"-L{PKG}", "-lmpcg", f"-Wl,-rpath,{PKG}"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(so + ".tmp", so)
    test_src = os.path.join(ROOT, "tests", "cpp", "test_solver.cpp")
    if os.path.exists(test_src) and (force or _stale(exe, [test_src, so])):
        cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra"] + inc + [test_src, "-o", exe, f"-L{out}",
                                                                      "-lmpc_planner_solver", f"-L{PKG}", "-lmpcg",
                                                                      f"-Wl,-rpath,{out}:{PKG}"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return {"dir": out, "lib": so, "test": exe}


if __name__ == "__main__":
    print(build_lib(force=True, verbose=True))
    print(build_cpp("C2", force=True, verbose=True))
