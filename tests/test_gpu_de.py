"""GPU parity of the building blocks: every frm builtin and every scene's distance
estimator + colour evaluated on the device equal the CPU oracle bit for bit."""
import numpy as np
import pytest

import frm
from helpers import params_for, same_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(gpu_renderer_factory):
    r = gpu_renderer_factory()
    yield r
    r.close()


def _inputs(name, rng):
    n = 200000
    if name in ("sin", "cos"):
        a = np.concatenate([rng.uniform(-30, 30, n), rng.uniform(-1, 1, 1000), [0.0, -0.0, np.pi, 1e6, np.inf, np.nan]])
        return a, None
    if name == "acos":
        return np.concatenate([rng.uniform(-1, 1, n), [1, -1, 0.5, -0.5, 0, 1.0000001, np.nan]]), None
    if name == "atan2":
        a = np.concatenate([rng.uniform(-2, 2, n), [0.0, -0.0, 0.0, 1.0, -1.0, 1e-30]])
        b = np.concatenate([rng.uniform(-2, 2, n), [0.0, 0.0, -0.0, 0.0, -0.0, 1e30]])
        return a, b
    if name in ("log", "log2"):
        a = np.concatenate([np.exp(rng.uniform(-80, 80, n)), [0.0, -1.0, np.inf, np.nan, 1.0, 1e-40, 2e-45]])
        return a, None
    if name == "exp2":
        return np.concatenate([rng.uniform(-160, 140, n), rng.uniform(-1, 1, 1000), [np.inf, -np.inf, np.nan]]), None
    if name == "pow":
        a = np.concatenate([rng.uniform(0, 100, n), [0.0, 1.0, 2.0]])
        b = np.concatenate([rng.uniform(-1, 16, n), [16.0, 100.0, 0.0]])
        return a, b
    if name == "sqrt":
        return np.concatenate([np.exp(rng.uniform(-100, 80, n)), [0.0, 1e-45, 4.0]]), None
    a = rng.uniform(-10, 10, n)
    b = np.concatenate([rng.uniform(-10, 10, n - 3), [0.0, 1e-40, -0.0]])
    return a, b


@pytest.mark.parametrize("name", ["sin", "cos", "acos", "atan2", "log", "log2", "exp2", "pow", "sqrt", "div"])
def test_builtin_bit_exact(gpu, oracle, name):
    rng = np.random.default_rng(7)
    a, b = _inputs(name, rng)
    a = a.astype(np.float32)
    b = None if b is None else b.astype(np.float32)
    got = gpu.eval_math(name, a, b)
    ref = oracle.math_fn(name, a, b)
    bad = ~((got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref)))
    assert not bad.any(), f"{name}: {bad.sum()} mismatches, e.g. a={a[bad][:3]} gpu={got[bad][:3]} cpu={ref[bad][:3]}"


@pytest.mark.parametrize("scene", list(range(19)) + ["sphere"])
def test_scene_de_bit_exact(gpu_renderer_factory, oracle, scene):
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1.5, 1.5, size=(20000, 3)).astype(np.float32)
    flags = frm.FRM_FLAG_SCENE_SPHERE if scene == "sphere" else 0
    s = 0 if scene == "sphere" else scene
    for iters, time in ((0, 0.0), (3, 3.2175055), (8, 1.0), (12, 3.2175055)):
        p = params_for(s, iters, time, 64, 64)
        with gpu_renderer_factory(flags=flags) as r:
            r.update_parameters_buffer(p)
            d, col = r.eval_scene(pts)
        rd, rcol, _ = oracle.scene_de(p, pts, flags=flags)
        assert same_bits(d, rd), f"scene {scene} N={iters}: {np.sum(d.view(np.uint32) != rd.view(np.uint32))} DE mismatches"
        assert same_bits(col, rcol), f"scene {scene} N={iters}: colour mismatch"


def test_mandelbulb_tame_and_exact_paths(gpu_renderer_factory, oracle):
    """Waves whose lanes all have tame operands take the fast body (frm_fast.h); a wave
    with one non-tame lane (component below 2^-60, |z| below 2^-40, |z|^2 below 2^-96)
    takes the exact body. Both must equal the oracle."""
    rng = np.random.default_rng(42)
    tame = rng.uniform(-1.3, 1.3, size=(64 * 200, 3)).astype(np.float32)
    odd = tame.copy()
    odd[::64, 0] = 1e-30          # one tiny component per wave
    odd[1::64] = [1e-25, 2e-26, -3e-25]  # |z|^2 < 2^-96
    odd[2::64] = [0.0, 0.0, 1e-13]
    odd[3::64] = [0.0, 0.0, 0.0]
    odd[4::64] = [1e-5, -2e-5, 3e-5]  # |z| in [2^-40, 2^-13): exact body since exp2_tame's domain
    for iters in (3, 12):
        p = params_for(18, iters, frm.POWER8_TIME, 64, 64)
        with gpu_renderer_factory() as r:
            r.update_parameters_buffer(p)
            for pts in (tame, odd):
                d, col = r.eval_scene(pts)
                rd, rcol, _ = oracle.scene_de(p, pts)
                assert same_bits(d, rd), f"N={iters}: {np.sum(~((d.view(np.uint32) == rd.view(np.uint32)) | (np.isnan(d) & np.isnan(rd))))} mismatches"


def _tame(rng, n, lo=-60, hi=40, zeros=True):
    """Values 0 (if zeros) or +-2^e * mantissa with e in [lo, hi): the tame operand range."""
    mag = np.clip(np.exp2(rng.uniform(lo, hi, n)), 2.0 ** lo, 2.0 ** hi)
    v = (mag * rng.choice([-1.0, 1.0], n)).astype(np.float32)
    if zeros:
        v[rng.random(n) < 0.02] = 0.0
    return v


def _fast_inputs(name, rng):
    n = 200000
    if name == "sqrt_nosmall":
        # the rsq-based fast sqrt (frm_fast.h): +-0, [2^-96, 2^126], negatives and NaN; both ends of
        # the range and every mantissa boundary around 1 and 4
        edge = np.array([1.0, 4.0, 2.0 ** -96, 2.0 ** 126], np.float32).view(np.uint32)
        edge = (edge[:, None] + np.arange(-3, 4)).ravel().astype(np.uint32).view(np.float32).astype(np.float64)
        edge = edge[(edge >= 2.0 ** -96) & (edge <= 2.0 ** 126)]
        a = np.concatenate([np.exp2(rng.uniform(-96, 126, n)), edge, [0.0, -0.0, -1.0, -(2.0 ** -100), np.nan,
                                                                      2.0 ** -96, 2.0 ** 126, 1.0]])
        return "sqrt", a, None
    if name in ("div_tame", "div_tame_nz"):
        a, b = _tame(rng, n), _tame(rng, n, zeros=False)
        if name == "div_tame":
            a = np.concatenate([a, [0.0, -0.0, -0.0, 2.0 ** -60, 2.0 ** 40]])
            b = np.concatenate([b, [-3.0, 5.0, -5.0, 2.0 ** 40, 2.0 ** -60]])
        else:  # the numerator is never -0 there (frm_fast.h)
            a[a == 0] = 0.0
        return "div", a, b
    if name in ("sin_small", "cos_small"):
        lim = 2.0 ** 20  # sincos_small is sincos_'s |x| <= 2^20 branch (frm_math.h)
        a = np.concatenate([rng.uniform(-30, 30, n), rng.uniform(-lim, lim, n // 4),
                            [0.0, -0.0, np.pi, -np.pi, 9 * np.pi, lim, -lim, np.pi / 2, 0.5, -1.5]])
        return name.split("_")[0], a, None
    if name == "acos_dev":
        return "acos", np.concatenate([rng.uniform(-1, 1, n), [1, -1, 0.5, -0.5, 0.0, -0.0, 1.0000001, np.nan]]), None
    if name == "atan2_tame":
        # + signed-zero pairs (x = y = 0: the 2^-100 floor of mx) and the range edges
        edge = np.array([0.0, -0.0, 2.0 ** -60, -(2.0 ** -60), 2.0 ** 40, -(2.0 ** 40), 1.0])
        ey, ex = (g.ravel() for g in np.meshgrid(edge, edge))
        return "atan2", np.concatenate([_tame(rng, n), ey]), np.concatenate([_tame(rng, n), ex])
    if name in ("log2_tame", "log_posnormal"):
        # positive normal finite x, incl. both sides of every sqrt(1/2) mantissa boundary
        edge = np.float32(0.70710677).view(np.uint32) + np.arange(-2, 3, dtype=np.int64)
        edge = np.concatenate([np.ldexp(edge.astype(np.uint32).view(np.float32).astype(np.float64), e)
                               for e in range(-125, 128, 7)])
        a = np.concatenate([np.exp2(rng.uniform(-126, 128, n)), edge,
                            [1.0, 2.0 ** -126, 0.7071067, np.finfo(np.float32).max, 2.0, 0.5]])
        return ("log2" if name == "log2_tame" else "log"), a, None
    # exp2_tame: finite y with rint(y) in [-125, 127]: [-125.5, 127.5), the half-way points
    # rounding to even at both ends included
    a = np.concatenate([rng.uniform(-125.5, 127.49, n), rng.uniform(-1, 1, 1000), np.arange(-125, 128),
                        np.arange(-125, 127) + 0.5, [-125.5, 127.499]])
    return "exp2", a, None


FAST = ["sqrt_nosmall", "div_tame", "div_tame_nz", "sin_small", "cos_small", "acos_dev", "atan2_tame",
        "log2_tame", "exp2_tame", "log_posnormal"]


@pytest.mark.parametrize("name", FAST)
def test_fast_path_bit_exact_on_its_domain(gpu, oracle, name):
    """Each device fast path (frm_fast.h) equals the exact builtin bit for bit on the operand
    domain the tame Mandelbulb body guarantees for it."""
    rng = np.random.default_rng(11)
    ref_name, a, b = _fast_inputs(name, rng)
    a = a.astype(np.float32)
    b = None if b is None else b.astype(np.float32)
    got = gpu.eval_math(name, a, b)
    ref = oracle.math_fn(ref_name, a, b)
    bad = ~((got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref)))
    assert not bad.any(), f"{name}: {bad.sum()} mismatches, e.g. a={a[bad][:3]} gpu={got[bad][:3]} cpu={ref[bad][:3]}"


def test_div_tame_nz_zero_numerator_sign(gpu):
    """The documented difference: -0 / b gives +0 (acos_dev(+-0) agree, so it cannot matter)."""
    got = gpu.eval_math("div_tame_nz", np.array([-0.0, 0.0], np.float32), np.array([2.0, -2.0], np.float32))
    assert got.view(np.uint32).tolist() == [0, 0x80000000]  # -0/2 -> +0 (exact: -0); +0/-2 -> -0
    assert gpu.eval_math("acos_dev", np.array([-0.0], np.float32)).view(np.uint32)[0] == \
        gpu.eval_math("acos_dev", np.array([0.0], np.float32)).view(np.uint32)[0]
