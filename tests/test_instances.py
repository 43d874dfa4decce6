"""Kernel instances for any generated solver (mpcg_instance.h): the built-in table
covers C1-C5 and the reference's shipped robot solvers, and a generated solver of
other dimensions brings its own instance (codegen mpcg_instance.hip) that
registers with libmpcg.so when its library loads.  CPU: registration and the
generated source; GPU: parity of a generated instance and of the shipped
jackalsimulator shape against the oracle."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "oscar_mpc_planner_mr_modification_amd")
G25 = os.path.join(PKG, "build", "G25", "libmpcg_inst_G25.so")


def _g25():
    from oscar_mpc_planner_mr_modification_amd.layouts import tmpc_layout
    return tmpc_layout(N=25, max_obstacles=3, name="G25")


def test_codegen_writes_the_instance_of_the_generated_dimensions(tmp_path):
    from oscar_mpc_planner_mr_modification_amd import codegen
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    codegen.generate(config_layout("JS"), str(tmp_path))
    src = open(tmp_path / "mpcg_instance.hip").read()
    assert "MPCG_DEFINE_INSTANCE(30, 4, 4, 0, 5, 0)" in src
    codegen.generate(config_layout("C3"), str(tmp_path))
    assert "MPCG_DEFINE_INSTANCE(30, 0, 0, 12, 6, 1)" in open(tmp_path / "mpcg_instance.hip").read()


def test_shipped_robot_solvers_have_builtin_instances():
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout, tmpc_layout
    from oscar_mpc_planner_mr_modification_amd.native_spec import problem_from_layout
    lib = C.CDLL(os.path.join(PKG, "libmpcg.so"))
    # jackalsimulator (N 30, 4 obstacles), jackal / dingo (N 30, 5 obstacles)
    for lay in (config_layout("JS"), tmpc_layout(N=30, max_obstacles=5)):
        assert lib.mpcg_supported(C.byref(problem_from_layout(lay))) == 0, lay.name


def test_instance_of_another_abi_is_refused():
    """An instance library compiled against other sources (another MPCG_ABI_VERSION) must not
    register: its kernels would read another mpcg_problem / workspace layout.  libmpcg.so refuses
    it and counts it; native.load_instances turns the count into an ImportError."""
    code = f"""
import ctypes as C
lib = C.CDLL({os.path.join(PKG, "libmpcg.so")!r})
lib.mpcg_register_instance.argtypes = [C.c_int] * 7 + [C.c_void_p, C.c_int, C.c_longlong, C.c_char_p]
abi = lib.mpcg_abi_version()
rc = lib.mpcg_register_instance(abi - 1, 0, 25, 3, 0, 0, 4, C.c_void_p(1), 1, 8, b"")
print(rc, lib.mpcg_rejected_instances())
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["-3", "1"]
    assert "rebuild" in r.stderr


def test_generated_instance_registers_on_load():
    """In a fresh process: the G25 shape is unknown to libmpcg.so until the generated
    instance library is loaded (no GPU call: registration is host code)."""
    code = f"""
import ctypes as C, sys
sys.path.insert(0, {ROOT!r})
from oscar_mpc_planner_mr_modification_amd.layouts import tmpc_layout
from oscar_mpc_planner_mr_modification_amd.native_spec import problem_from_layout
lib = C.CDLL({os.path.join(PKG, "libmpcg.so")!r}, mode=C.RTLD_GLOBAL)
pr = problem_from_layout(tmpc_layout(N=25, max_obstacles=3))
before = lib.mpcg_supported(C.byref(pr))
C.CDLL({G25!r}, mode=C.RTLD_GLOBAL)
after = lib.mpcg_supported(C.byref(pr))
lib.mpcg_qp_mem_size.restype = C.c_int
print(before, after, lib.mpcg_qp_mem_size(C.byref(pr)))
"""
    if not os.path.exists(G25):
        from oscar_mpc_planner_mr_modification_amd import _build
        _build.build_instance(_g25(), os.path.dirname(G25))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    before, after, qpm = (int(v) for v in r.stdout.split())
    assert (before, after) == (-1, 0)
    assert qpm > 0


def _parity(native, oracle_mod, lay, S, G, seed):
    import torch
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch
    b = make_batch(lay, S, G, seed=seed)
    ref = oracle_mod.Oracle(lay).solve_batch(b.params, b.warm, b.xinit)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = native.solve_batch_device(native.problem_from_layout(lay), t(b.params), t(b.warm), t(b.xinit))
    got = {k: v.cpu().numpy() for k, v in out.items()}
    same = got["exit"] == ref["status"]
    ok = same & (got["exit"] == 1)
    dx = np.abs(got["xtraj"] - ref["xtraj"]).reshape(len(same), -1).max(1)
    print(f"{lay.name}: {len(same)} solves, success {ok.mean():.2f}, max|dx| {dx[ok].max():.2e}")
    assert same.all()
    assert ok.mean() >= 0.8
    assert dx[ok].max() <= 1e-4


@pytest.mark.gpu
def test_generated_instance_parity_on_gpu(oracle_mod):
    from oscar_mpc_planner_mr_modification_amd import native
    lay = _g25()
    native.load_instances(G25)
    assert native.supported(native.problem_from_layout(lay))
    _parity(native, oracle_mod, lay, 8, 8, 2525)


@pytest.mark.gpu
def test_jackalsimulator_shipped_solver_parity_on_gpu(oracle_mod):
    """mpc_planner_jackalsimulator as shipped: N 30, 4 obstacles, 4 guided + 1 non-guided planners."""
    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    _parity(native, oracle_mod, config_layout("JS"), 16, 5, 3030)


@pytest.mark.gpu
def test_jackal_dingo_shipped_solver_parity_on_gpu(oracle_mod):
    """mpc_planner_jackal / mpc_planner_dingo as shipped: N 30, 5 obstacles
    (mpc_planner_jackal/config/settings.yaml:3,38), 4 guided + 1 non-guided planners; the
    built-in Cfg<30,5,5,0,5,0> (constant [B A] rows, paired chains)."""
    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    _parity(native, oracle_mod, config_layout("JD"), 16, 5, 3131)


def test_builtin_instances_storage_choices():
    """Which storage each built-in instance compiles to (mpcg_sqp.h: LEAN / GFH / FCONST /
    PAIR_CHAINS / STORE_IT / PARTS), reported by the host-side query the library exports;
    the shipped N 30 robot solvers stay on the four-solves-per-CU line without GFH."""
    import ctypes as C
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.native_spec import problem_from_layout
    lib = C.CDLL(os.path.join(PKG, "libmpcg.so"))
    lib.mpcg_instance_traits.restype = C.c_int
    got = {}
    for cfg in ("C1", "C2", "C3", "C4", "C5", "JS", "JD"):
        buf = C.create_string_buffer(256)
        assert lib.mpcg_instance_traits(C.byref(problem_from_layout(config_layout(cfg))), buf, 256) == 0, cfg
        got[cfg] = dict(kv.split("=") for kv in buf.value.decode().split())
    print(got)
    for cfg in ("JS", "JD"):
        t = got[cfg]
        assert (t["parts"], t["fconst"], t["pair"], t["gfh"], t["lean"]) == ("2", "1", "1", "0", "1"), (cfg, t)
        assert int(t["lds"]) <= 40 * 1024, (cfg, t)
    assert got["C4"]["gfh"] == "1" and got["C3"]["gfh"] == "1"
    assert got["C2"]["parts"] == "3" and got["C2"]["store_it"] == "1"
    # stored 1/t up to 13 row slots per lane on three-part instances (C1, C2); the two-part ones (JS, JD)
    # keep the round-2 gate (mpcg_sqp.h Cfg::STORE_IT: the cause of that build's fault was never named);
    # C5 (14, round 5: profiles/r05c_ab_st14_C5.jsonl), C3 (16) and C4 (20) recompute it
    for cfg, want in (("C1", "1"), ("C5", "0"), ("JS", "0"), ("JD", "0"), ("C3", "0"), ("C4", "0")):
        assert got[cfg]["store_it"] == want, (cfg, got[cfg])
    # conflict-minimal LDS stage strides (h-row gradients, h-row gaps, cost-to-go rows; doubles),
    # every instance still under the four-solves-per-CU line
    for cfg, want in (("C2", "49,17,18"), ("C1", "25,9,18"), ("C4", "26,14,18"), ("JS", "10,6,15")):
        assert got[cfg]["strides"] == want, (cfg, got[cfg])
    for cfg, t in got.items():
        assert int(t["lds"]) <= 40 * 1024, (cfg, t)


def test_lds_stride_model():
    """The compile-time bank model (mpcg_sqp.h lds_b64_cycles) restated: C2's unpadded
    h-row gradient rows (48 doubles per stage, part offset 3) cost 12 LDS cycles per
    ds_read_b64, the padded 49 cost 4; conflict-free is 2."""
    def cycles(s, off, parts):
        total = 0
        for half in range(2):
            dw = {2 * (s * (lane // parts) + off * (lane % parts)) + h
                  for lane in range(32 * half, 32 * half + 32) for h in range(2)}
            per_bank = {}
            for d in dw:
                per_bank[d % 64] = per_bank.get(d % 64, 0) + 1
            total += max(per_bank.values())
        return total
    assert cycles(48, 3, 3) == 12 and cycles(49, 3, 3) == 4      # C2 gradients
    assert cycles(16, 1, 3) == 12 and cycles(17, 1, 3) == 4      # C2 gaps
    assert cycles(16, 0, 3) == 12 and cycles(18, 0, 3) == 2      # C2 cost-to-go (even strides)
    assert cycles(24, 2, 2) == 8 and cycles(26, 2, 2) == 4       # C4 gradients (even strides)
    assert cycles(15, 0, 2) == 2                                  # N 30 cost-to-go, unpadded
