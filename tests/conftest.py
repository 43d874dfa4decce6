import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle_py
    oracle_py.build()
    return oracle_py


def picks_equivalent(best_gpu, best_ref, pobj_ref, rel=1e-9):
    """ScenarioConstraints' pick on both sides (scenario_constraints.cpp:86-103): the same
    copy, or copies whose oracle costs tie to `rel` (copies with no active scenario row
    reach the same plan, and rounding decides between exact ties)."""
    import numpy as np
    best_gpu, best_ref = np.asarray(best_gpu), np.asarray(best_ref)
    P = len(pobj_ref) // len(best_ref)
    po = np.asarray(pobj_ref).reshape(-1, P)
    if not np.array_equal(best_gpu < 0, best_ref < 0):
        return False
    s = np.flatnonzero(best_ref >= 0)
    a, b = po[s, best_gpu[s]], po[s, best_ref[s]]
    return bool(np.all(np.abs(a - b) <= rel * np.maximum(1.0, np.abs(b))))
