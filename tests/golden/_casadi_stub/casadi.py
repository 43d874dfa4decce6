"""Scratch sympy-backed stand-in for the `casadi` module.

TEST INFRASTRUCTURE ONLY.  casadi 3.5.5 (pinned by the reference's
requirements.txt:2 / pyproject.toml:10) is not installed in this image and no
package can be fetched.  `tests/golden/gen_golden.py` puts this directory at
the front of sys.path so that the reference's own problem-definition Python
(solver_generator/*, mpc_planner_modules/scripts/*) can build its symbolic
stage cost / constraints / dynamics, which are then differentiated with sympy
to produce the committed golden vectors.  Nothing under oscar_mpc_planner_mr_modification_amd/,
bench.py or __graft_entry__.py imports this file.
"""
import numpy as _np
import sympy as _sp

pi = _sp.pi

# numpy's ufuncs (np.exp in spline.py:37) call the method of the same name on
# object-array elements.
_sp.Expr.exp = lambda self: _sp.exp(self)
_sp.Expr.sqrt = lambda self: _sp.sqrt(self)


def _flatten(args):
    out = []
    for a in args:
        if isinstance(a, _sp.MatrixBase):
            out.extend(list(a))
        elif isinstance(a, (list, tuple)):
            out.extend(_flatten(a))
        elif isinstance(a, _np.ndarray):
            out.extend(_flatten(list(a.ravel())))
        else:
            out.append(a)
    return out


class SX:
    """Only the constructors the reference uses: SX(), SX(r, c), SX(array)."""

    def __new__(cls, *args):
        if len(args) == 0:
            return _sp.Matrix(0, 1, [])
        if len(args) == 2 and all(isinstance(a, int) for a in args):
            return _sp.zeros(args[0], args[1])
        a = args[0]
        if isinstance(a, _np.ndarray):
            if a.ndim == 1:
                return _sp.Matrix([[e] for e in a])
            return _sp.Matrix(a.tolist())
        return _sp.Matrix(a)

    @staticmethod
    def sym(name, n=1):
        if n == 1:
            return _sp.Symbol(name, real=True)
        return _sp.Matrix([_sp.Symbol(f"{name}_{i}", real=True) for i in range(n)])


def vertcat(*args):
    return _sp.Matrix(_flatten(args))


cos = _sp.cos
sin = _sp.sin
tan = _sp.tan
exp = _sp.exp
log = _sp.log
sqrt = _sp.sqrt
fabs = _sp.Abs
erf = _sp.erf
atan = _sp.atan
arctan = _sp.atan
atan2 = _sp.atan2


def fmax(a, b):
    return _sp.Max(a, b)


class fmod(_sp.Function):
    """C fmod (casadi's fmod), left unevaluated: sympy's Mod would try to
    simplify the symbolic dividend (slow) and takes the floor convention.
    d/da = 1; lambdify it with {"fmod": numpy.fmod}."""

    def fdiff(self, argindex=1):
        a, b = self.args
        if argindex == 1:
            return _sp.S.One
        q = a / b
        return -_sp.sign(q) * _sp.floor(_sp.Abs(q))
