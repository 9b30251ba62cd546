"""Accuracy of the frm builtins (DESIGN.md §frm math) against float64, measured on the
ranges the hot path uses. WGSL only bounds its builtins (e.g. sin/cos absolute error
<= 2^-11); frm is within a few f32 ulp."""
import numpy as np
import pytest


def ulp_err(got, ref):
    got = got.astype(np.float64)
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return np.abs(got - ref) / ulp


RNG = np.random.default_rng(11)
CASES = {
    "sin": (RNG.uniform(-30, 30, 100000), None, np.sin, "abs", 2e-7),
    "cos": (RNG.uniform(-30, 30, 100000), None, np.cos, "abs", 2e-7),
    "acos": (RNG.uniform(-1, 1, 100000), None, np.arccos, "ulp", 4),
    "atan2": (RNG.uniform(-3, 3, 100000), RNG.uniform(-3, 3, 100000), np.arctan2, "ulp", 4),
    "log": (np.exp(RNG.uniform(-20, 20, 100000)), None, np.log, "abs_rel", 3),
    "log2": (np.exp(RNG.uniform(-20, 20, 100000)), None, np.log2, "abs_rel", 3),
    "exp2": (RNG.uniform(-60, 60, 100000), None, np.exp2, "ulp", 3),
    "pow": (RNG.uniform(0.01, 100, 100000), RNG.uniform(0, 9, 100000), np.power, "rel", 3e-6),
}


@pytest.mark.parametrize("name", list(CASES))
def test_frm_builtin_accuracy(oracle, name):
    a, b, fn, kind, bound = CASES[name]
    a32 = a.astype(np.float32)
    b32 = None if b is None else b.astype(np.float32)
    got = oracle.math_fn(name, a32, b32)
    ref = fn(a32.astype(np.float64)) if b is None else fn(a32.astype(np.float64), b32.astype(np.float64))
    if kind == "abs":
        assert np.max(np.abs(got - ref)) < bound
    elif kind == "ulp":
        assert np.max(ulp_err(got, ref)) <= bound
    elif kind == "rel":
        assert np.max(np.abs(got - ref) / np.abs(ref)) < bound
    else:  # ulp away from zero, absolute 2^-22 near the zero of log
        err = np.abs(got - ref)
        assert np.all((err <= bound * np.spacing(np.abs(ref).astype(np.float32))) | (err < 2.5e-7))


def test_special_values(oracle):
    inf, nan = np.inf, np.nan
    assert oracle.math_fn("log", [0.0])[0] == -inf
    assert np.isnan(oracle.math_fn("log", [-1.0])[0])
    assert oracle.math_fn("log2", [inf])[0] == inf
    assert oracle.math_fn("log2", [1.0])[0] == 0.0
    assert oracle.math_fn("exp2", [-inf])[0] == 0.0 and oracle.math_fn("exp2", [inf])[0] == inf
    assert np.isnan(oracle.math_fn("exp2", [nan])[0])
    assert oracle.math_fn("pow", [0.0], [16.0])[0] == 0.0  # specular of a back-facing normal
    assert oracle.math_fn("pow", [1.0], [100.0])[0] == 1.0  # AO at zero steps
    assert oracle.math_fn("atan2", [0.0], [0.0])[0] == 0.0
    assert oracle.math_fn("acos", [1.0])[0] == 0.0
    assert oracle.math_fn("exp2", [3.0])[0] == 8.0 and oracle.math_fn("exp2", [-3.0])[0] == 0.125


def test_libm_mode_is_double_rounded_once(oracle):
    x = np.random.default_rng(2).uniform(-10, 10, 10000).astype(np.float32)
    got = oracle.math_fn("sin", x, mode=oracle.MODE_LIBM)
    assert np.array_equal(got, np.sin(x.astype(np.float64)).astype(np.float32))
