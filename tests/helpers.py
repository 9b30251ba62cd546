"""Shared helpers for the test suite (parameter construction, host replay calls)."""
import ctypes

import numpy as np

import frm


def params_for(scene, iters, time, width, height, pose="P1"):
    w = frm.WORKLOADS["HEADLINE"]
    p = frm.make_parameters(w, pose=pose, time=time, width=width, height=height)
    p.scene_index = scene
    p.num_iterations = iters
    return p


def pbytes(p):
    return np.frombuffer(p.to_bytes(), dtype=np.uint8).copy()


def hr_render(hr, p, width, height, max_steps, flags=0, rows=None):
    pb = pbytes(p)
    if rows is None:
        nrows, rptr = height, None
    else:
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        nrows, rptr = len(rows), ctypes.c_void_p(rows.ctypes.data)
    out = np.zeros((nrows, width, 4), np.uint8)
    c = np.zeros(8, np.uint64)
    hr.hr_render(ctypes.c_void_p(pb.ctypes.data), width, height, max_steps, flags, rptr, nrows,
                 ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(c.ctypes.data))
    return out, c


def hr_scene_de(hr, p, pts, flags=0):
    pts = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 3)
    out = np.zeros(len(pts), np.float32)
    col = np.zeros((len(pts), 3), np.float32)
    pb = pbytes(p)
    hr.hr_scene_de(ctypes.c_void_p(pb.ctypes.data), flags, ctypes.c_void_p(pts.ctypes.data), len(pts),
                   ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(col.ctypes.data))
    return out, col


def same_bits(a, b):
    """Bitwise float equality with all NaNs equal."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all((a.view(np.uint32) == b.view(np.uint32)) | nan))
