"""The deterministic float32 math both the oracle and the kernels implement (oracle/detmath.h,
csrc/rmr_math.h): accuracy against float64 numpy."""
import numpy as np
import pytest

from oracle import oracle


def _ulp(x):
    return np.spacing(np.abs(np.float32(x))).astype(np.float64)


@pytest.mark.parametrize("fn,ref,lo,hi,tol", [
    ("sin", np.sin, -10.0, 10.0, 2e-7), ("cos", np.cos, -10.0, 10.0, 2e-7),
    ("sin", np.sin, 0.0, 3.15, 1.5e-7), ("acos", np.arccos, -1.0, 1.0, 4e-7),
    ("log", np.log, 1e-6, 1e6, 4e-7), ("exp", np.exp, -20.0, 20.0, 1e-6),
])
def test_det_functions_accuracy(fn, ref, lo, hi, tol):
    xs = np.linspace(lo, hi, 4001).astype(np.float32)
    got = np.array([oracle.det(fn, float(x)) for x in xs], np.float64)
    want = ref(xs.astype(np.float64))
    err = np.abs(got - want) / np.maximum(1.0, np.abs(want))
    assert err.max() < tol


def test_det_atan2_quadrants():
    for y, x in [(1, 1), (1, -1), (-1, -1), (-1, 1), (0, -1), (2, 0.1), (-0.1, -3)]:
        assert abs(oracle.det("atan2", y, x) - np.arctan2(y, x)) < 2e-5


def test_det_acos_edges():
    assert oracle.det("acos", 1.0) == 0.0
    assert oracle.det("acos", -1.0) == np.float32(np.pi)
    assert np.isnan(oracle.det("acos", 1.5))
