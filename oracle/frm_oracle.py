"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/frm_oracle.c).

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only; the
product never uses it. See frm_oracle.c for what is restated and how parity is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libfrm_oracle.so")

MODE_FRM = 0   # bit-exact spec of the kernel's builtins (gate P0)
MODE_LIBM = 1  # double-precision libm builtins rounded to f32 (gate P1)

INFO_HIT = 1
INFO_SUN_HIT = 2
INFO_NAN = 4
INFO_SHADOW_FIRST_NONPOS = 8
INFO_ZERO_NORMAL = 16

# per-pixel trace (render(trace=True)): the geometric inputs of the shading
TRACE_FIELDS = ("hit", "steps", "nx", "ny", "nz", "sun_hit", "sun_closeness", "cr", "cg", "cb")

MATH_FN = {"sin": 0, "cos": 1, "acos": 2, "atan2": 3, "log": 4, "log2": 5, "exp2": 6,
           "pow": 7, "sqrt": 8, "div": 9}

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = ctypes.CDLL(LIB_PATH)
        u8p, f32p, u32p, u64p = (ctypes.c_void_p,) * 4
        lib.om_render.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_int, u32p, ctypes.c_uint32, ctypes.c_int,
                                  u8p, u64p, f32p, u32p]
        lib.om_render.restype = ctypes.c_int
        lib.om_render_trace.argtypes = lib.om_render.argtypes + [f32p]
        lib.om_render_trace.restype = ctypes.c_int
        lib.om_shade_trace.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_int, u32p, ctypes.c_uint32, f32p, u8p]
        lib.om_shade_trace.restype = ctypes.c_int
        lib.om_scene_de.argtypes = [u8p, ctypes.c_uint32, ctypes.c_int, f32p, ctypes.c_uint32, f32p,
                                    f32p, u64p]
        lib.om_scene_de.restype = ctypes.c_int
        lib.om_math.argtypes = [ctypes.c_int, ctypes.c_int, f32p, f32p, ctypes.c_uint32, f32p]
        lib.om_math.restype = ctypes.c_int
        lib.om_srgb_thresholds.argtypes = [f32p]
        lib.om_srgb_thresholds.restype = None
        lib.om_encode_srgb.argtypes = [f32p, ctypes.c_uint32, u8p]
        lib.om_encode_srgb.restype = ctypes.c_int
        lib.om_srgb_decode.argtypes = [f32p]
        lib.om_srgb_decode.restype = None
        lib.om_blit.argtypes = [u8p, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_uint32]
        lib.om_blit.restype = ctypes.c_int
        lib.om_frame_info.argtypes = [u8p, ctypes.c_uint32, ctypes.c_int, f32p]
        lib.om_frame_info.restype = ctypes.c_int
        _lib = lib
    return _lib


def _params_buf(params):
    b = params.to_bytes() if hasattr(params, "to_bytes") else bytes(params)
    assert len(b) == 96
    return np.frombuffer(b, dtype=np.uint8).copy()


def render(params, width, height, max_steps, flags=0, mode=MODE_FRM, rows=None, threads=None,
           linear=False, info=False, trace=False):
    """Render rows (default all) -> dict(rgba=[n,W,4] u8, counters=[8] u64, ...); info: the
    per-pixel INFO_* bits | primary steps << 8; trace: [n,W,len(TRACE_FIELDS)] f32."""
    lib = load()
    pb = _params_buf(params)
    if rows is None:
        nrows, rows_arr, rows_ptr = height, None, None
    else:
        rows_arr = np.ascontiguousarray(rows, dtype=np.uint32)
        nrows, rows_ptr = len(rows_arr), rows_arr.ctypes.data
    threads = threads or os.cpu_count() or 1
    rgba = np.zeros((nrows, width, 4), dtype=np.uint8)
    counters = np.zeros(8, dtype=np.uint64)
    lin = np.zeros((nrows, width, 3), dtype=np.float32) if linear else None
    inf = np.zeros((nrows, width), dtype=np.uint32) if info else None
    tr = np.zeros((nrows, width, len(TRACE_FIELDS)), dtype=np.float32) if trace else None
    rc = lib.om_render_trace(pb.ctypes.data, width, height, max_steps, flags, mode, rows_ptr, nrows, threads,
                             rgba.ctypes.data, counters.ctypes.data,
                             lin.ctypes.data if linear else None, inf.ctypes.data if info else None,
                             tr.ctypes.data if trace else None)
    if rc != 0:
        raise RuntimeError(f"om_render failed ({rc})")
    out = {"rgba": rgba, "counters": counters}
    if linear:
        out["linear"] = lin
    if info:
        out["info"] = inf
    if trace:
        out["trace"] = tr
    return out


def shade_trace(params, width, height, max_steps, xs, ys, trace, flags=0, mode=MODE_FRM):
    """RGBA8 of pixels (xs[i], ys[i]) shaded (fragment.wgsl:336-346, builtins of `mode`) from
    the given traces ([n, len(TRACE_FIELDS)]) instead of their own march results."""
    lib = load()
    xy = np.ascontiguousarray(np.stack([xs, ys], axis=-1), dtype=np.uint32)
    tr = np.ascontiguousarray(trace, dtype=np.float32).reshape(-1, len(TRACE_FIELDS))
    out = np.zeros((len(tr), 4), dtype=np.uint8)
    rc = lib.om_shade_trace(_params_buf(params).ctypes.data, width, height, max_steps, flags, mode,
                            xy.ctypes.data, len(tr), tr.ctypes.data, out.ctypes.data)
    if rc != 0:
        raise ValueError("om_shade_trace")
    return out


def scene_de(params, points, flags=0, mode=MODE_FRM):
    lib = load()
    pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    n = pts.shape[0]
    d = np.zeros(n, dtype=np.float32)
    col = np.zeros((n, 3), dtype=np.float32)
    cnt = np.zeros(2, dtype=np.uint64)
    lib.om_scene_de(_params_buf(params).ctypes.data, flags, mode, pts.ctypes.data, n, d.ctypes.data,
                    col.ctypes.data, cnt.ctypes.data)
    return d, col, cnt


def math_fn(name, a, b=None, mode=MODE_FRM):
    lib = load()
    a = np.ascontiguousarray(a, dtype=np.float32)
    bb = None if b is None else np.ascontiguousarray(np.broadcast_to(b, a.shape), dtype=np.float32)
    out = np.zeros_like(a)
    rc = lib.om_math(MATH_FN[name], mode, a.ctypes.data, None if bb is None else bb.ctypes.data,
                     a.size, out.ctypes.data)
    if rc != 0:
        raise ValueError(name)
    return out


def srgb_thresholds():
    out = np.zeros(256, dtype=np.float32)
    load().om_srgb_thresholds(out.ctypes.data)
    return out


def encode_srgb(c):
    c = np.ascontiguousarray(c, dtype=np.float32)
    out = np.zeros(c.shape, dtype=np.uint8)
    load().om_encode_srgb(c.ctypes.data, c.size, out.ctypes.data)
    return out


def frame_info(params, flags=0, mode=MODE_FRM):
    out = np.zeros(8, dtype=np.float32)
    load().om_frame_info(_params_buf(params).ctypes.data, flags, mode, out.ctypes.data)
    return {"family": int(out[0]), "mb_power": float(out[1]), "menger_cross": float(out[2]),
            "menger_scale": float(out[3]), "koch_normal_z": float(out[4]),
            "origin": tuple(float(v) for v in out[5:8])}


def srgb_decode():
    out = np.zeros(256, dtype=np.float32)
    load().om_srgb_decode(out.ctypes.data)
    return out


def blit(rgba, out_width, out_height, flags=1):
    """Presentation resample of an RGBA8 sRGB frame [H, W, 4] (om_blit): flags 1 = sRGB output,
    2 = BGRA byte order."""
    src = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w = src.shape[:2]
    out = np.zeros((out_height, out_width, 4), dtype=np.uint8)
    rc = load().om_blit(src.ctypes.data, w, h, out.ctypes.data, out_width, out_height, flags)
    if rc != 0:
        raise ValueError("om_blit")
    return out
