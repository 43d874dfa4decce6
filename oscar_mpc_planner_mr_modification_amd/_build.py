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
SOURCES = {"mpcg_kernels.hip": [], "mpcg_prepare.hip": ["-ffp-contract=off"],
           # built-in kernel instances, one translation unit per family (compiled in parallel)
           "mpcg_inst_tmpc20.hip": [], "mpcg_inst_tmpc30.hip": [], "mpcg_inst_shmpc.hip": [],
           "mpcg_inst_bicycle.hip": []}
HEADERS = ["mpcg_device.h", "mpcg_sqp.h", "mpcg_sqp_body.inc", "mpcg_prepare.h", "mpcg_bicycle.h", "mpcg_instance.h"]
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


def build_lib(force: bool = False, verbose: bool = False, extra_flags=(), out: str = LIB, sources=None) -> str:
    """libmpcg.so (or a diagnostic / variant build of it with extra_flags at `out`; `sources`
    restricts the built-in instance files of such a build)"""
    srcs = SOURCES if sources is None else {k: v for k, v in SOURCES.items() if k in sources}
    deps = [os.path.join(CSRC, s) for s in list(SOURCES) + HEADERS] + [os.path.join(INCLUDE, "mpcg.h"), __file__]
    if not force and not _stale(out, deps):
        return out
    objdir = os.path.join(BUILD, "obj" + ("_" + "_".join(f.strip("-").replace("=", "") for f in extra_flags)
                                          if extra_flags else ""))
    os.makedirs(objdir, exist_ok=True)
    common = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{INCLUDE}", f"-I{CSRC}"]
    objs, procs = [], []
    for src, flags in srcs.items():
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        cmd = common + list(flags) + list(extra_flags) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, "hipcc")
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-soname,libmpcg.so", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def _hipcc_obj(src, obj, extra=()):
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{INCLUDE}", f"-I{CSRC}",
           *extra, "-c", src, "-o", obj]
    subprocess.run(cmd, check=True)
    return obj


def build_instance(layout, out_dir: str, force: bool = False) -> str:
    """libmpcg_inst_<name>.so: the kernel instance of `layout`'s dimensions (codegen
    mpcg_instance.hip) as a library that registers itself with libmpcg.so on load
    (native.load_instances)."""
    from . import codegen

    lib_mpcg = build_lib()
    os.makedirs(out_dir, exist_ok=True)
    src = os.path.join(out_dir, "mpcg_instance.hip")
    text = codegen.instance_source(layout)
    if not os.path.exists(src) or open(src).read() != text:
        with open(src, "w") as fh:
            fh.write(text)
    so = os.path.join(out_dir, f"libmpcg_inst_{layout.name}.so")
    deps = [src, lib_mpcg, os.path.join(INCLUDE, "mpcg.h")] + [os.path.join(CSRC, h) for h in HEADERS]
    if force or _stale(so, deps):
        obj = _hipcc_obj(src, os.path.join(out_dir, "mpcg_instance.o"))
        subprocess.run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so + ".tmp", obj, f"-L{PKG}",
                        "-lmpcg", f"-Wl,-rpath,{PKG}"], check=True)
        os.replace(so + ".tmp", so)
    return so


def build_cpp(config="C2", force: bool = False, verbose: bool = False) -> dict:
    """The drop-in C++ MPCPlanner::Solver for one generated solver
    (dimensions are compile-time, as in the reference): codegen into
    build/<name>/, then libmpc_planner_solver.so -- the host sources plus the
    generated kernel instance of these dimensions -- and the test program
    tests/cpp/test_solver.cpp, linked against libmpcg.so.  `config` is a
    config name or a Layout."""
    from . import codegen
    from .layouts import config_layout

    lay = config_layout(config) if isinstance(config, str) else config
    lib_mpcg = build_lib()
    out = os.path.join(BUILD, lay.name)
    codegen.generate(lay, out)
    so = os.path.join(out, "libmpc_planner_solver.so")
    exe = os.path.join(out, "test_solver")
    srcs = [os.path.join(CSRC, s) for s in HOST_SOURCES] + [os.path.join(out, "mpc_planner_parameters.cpp")]
    inst = os.path.join(out, "mpcg_instance.hip")
    deps = srcs + [inst] + [os.path.join(INCLUDE, h) for h in HOST_HEADERS] + \
        [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "mpcg.h"), lib_mpcg, __file__]
    inc = [f"-I{os.path.join(out, 'include')}", f"-I{INCLUDE}"]
    if force or _stale(so, deps):
        objs = []
        for src in srcs:
            obj = os.path.join(out, os.path.basename(src).replace(".cpp", ".o"))
            cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-Wall", "-Wextra"] + inc + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
            objs.append(obj)
        objs.append(_hipcc_obj(inst, os.path.join(out, "mpcg_instance.o")))
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + \
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
