"""Renderer: the Python host's view of libfrm, mirroring the reference's `Graphics`
API (src/graphics.rs): init -> resize -> update_parameters_buffer -> render ->
(read_frame replaces the blit+present). Errors raise FrmError; nothing falls back to
the CPU."""
import ctypes
import os

import numpy as np

from . import _lib


class Renderer:
    def __init__(self, device=0, max_steps=0, flags=0, frames_in_flight=1, devices=None):
        """devices: a list of HIP device ordinals for a GROUP context (frm_config.device_count):
        every frame is row-tiled over them and gathered on devices[0] (RCCL, or device copies
        when a device repeats); the rest of the API is the same."""
        lib = _lib.load()
        self._lib = lib
        self.ctx = ctypes.c_void_p()
        cfg = _lib.FrmConfig(device, max_steps, flags, frames_in_flight)
        if devices is not None:
            devices = list(devices)
            if not 1 <= len(devices) <= 16:
                raise ValueError("a group holds 1..16 devices")
            cfg.device_count = len(devices)
            for i, d in enumerate(devices):
                cfg.devices[i] = d
            device = devices[0]
        _lib.check(lib.frm_create(ctypes.byref(self.ctx), ctypes.byref(cfg)))
        self.devices = devices
        self.device = device
        self.frames_in_flight = max(1, frames_in_flight)
        self.width = self.height = 0

    def close(self):
        if self.ctx:
            self._lib.frm_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        return _lib.check(rc, self.ctx)

    # graphics.rs:54-57 (render texture size) — arbitrary W x H here
    def resize(self, width, height):
        self._check(self._lib.frm_resize(self.ctx, width, height))
        self.width, self.height = width, height

    # graphics.rs:59-61
    def update_parameters_buffer(self, parameters):
        raw = parameters.raw if hasattr(parameters, "raw") else parameters
        self._check(self._lib.frm_set_parameters(self.ctx, ctypes.byref(raw)))

    # graphics.rs:91-110 (one frame); returns frm_stats as a dict when stats=True
    def render(self, stats=True):
        if not stats:
            self._check(self._lib.frm_render(self.ctx, None))
            return None
        st = _lib.FrmStats()
        self._check(self._lib.frm_render(self.ctx, ctypes.byref(st)))
        return st.as_dict()

    def read_frame(self):
        buf = np.empty((self.height, self.width, 4), dtype=np.uint8)
        self._check(self._lib.frm_read_frame(self.ctx, buf.ctypes.data, buf.nbytes))
        return buf

    # blit.wgsl + present (graphics.rs:91-110): the frame resampled to a window size
    def present(self, width, height, srgb=True, bgra=False):
        buf = np.empty((height, width, 4), dtype=np.uint8)
        flags = (_lib.FRM_BLIT_SRGB if srgb else 0) | (_lib.FRM_BLIT_BGRA if bgra else 0)
        self._check(self._lib.frm_present(self.ctx, width, height, flags, buf.ctypes.data, buf.nbytes))
        return buf

    # asynchronous readback (frm_read_frame_async / frm_present_async + frm_frame_pixels): the
    # reference's surface presents with a frame of latency (wgpu's desired_maximum_frame_latency
    # 2), so a loop renders frame k, starts its readback and then waits for frame k-1's pixels
    def read_frame_async(self):
        t = ctypes.c_uint64()
        self._check(self._lib.frm_read_frame_async(self.ctx, ctypes.byref(t)))
        return self._remember(t.value, (self.height, self.width, 4))

    def present_async(self, width, height, srgb=True, bgra=False):
        t = ctypes.c_uint64()
        flags = (_lib.FRM_BLIT_SRGB if srgb else 0) | (_lib.FRM_BLIT_BGRA if bgra else 0)
        self._check(self._lib.frm_present_async(self.ctx, width, height, flags, ctypes.byref(t)))
        return self._remember(t.value, (height, width, 4))

    def _remember(self, ticket, shape):
        # a ticket keeps the shape of its frame across a later resize (frm_resize does not drain)
        shapes = self.__dict__.setdefault("_ticket_shapes", {})
        shapes[ticket] = shape
        if len(shapes) > 64:
            del shapes[min(shapes)]
        return ticket

    def frame_pixels(self, ticket, shape=None, copy=True):
        """Waits for the readback `ticket` and returns its pixels as a uint8 array of `shape`
        (default: the frame's (height, width, 4)); copy=False returns a view of the library's
        pinned image, valid until frames_in_flight further renders."""
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        self._check(self._lib.frm_frame_pixels(self.ctx, int(ticket), ctypes.byref(ptr), ctypes.byref(n)))
        view = np.ctypeslib.as_array(ptr, shape=(n.value,))
        shape = shape or self.__dict__.get("_ticket_shapes", {}).get(int(ticket), (self.height, self.width, 4))
        view = view.reshape(shape)
        return view.copy() if copy else view

    def synchronize(self):
        self._check(self._lib.frm_synchronize(self.ctx))

    def kernel_for(self, pixels):
        """'persistent' or 'simple': the kernel a launch of `pixels` pixels runs here."""
        k = ctypes.c_uint32()
        self._check(self._lib.frm_kernel_for_pixels(self.ctx, int(pixels), ctypes.byref(k)))
        return "simple" if k.value == _lib.FRM_KERNEL_SIMPLE else "persistent"

    # graphics.rs:44-48 (reload): recompile the render kernels from an edited copy of csrc/
    # (hiprtc); raises FrmError (FRM_ERR_COMPILE + compiler log) and keeps the previous
    # kernels on failure. source_dir=None returns to the built-in kernels.
    def reload(self, source_dir):
        arg = None if source_dir is None else os.fsencode(source_dir)
        self._check(self._lib.frm_reload(self.ctx, arg))

    # graphics.rs:39-43 (try_reload): print the error instead of raising
    def try_reload(self, source_dir):
        try:
            self.reload(source_dir)
            return True
        except _lib.FrmError as e:
            print(e)
            return False

    # multi-GPU row tiling (device pointers, e.g. torch tensors' data_ptr())
    def render_bands(self, dev_ptr, nbytes, band_rows, first_band, band_stride, stream=0,
                     dev_counters=0):
        self._check(self._lib.frm_render_bands(self.ctx, dev_ptr, nbytes, band_rows, first_band,
                                               band_stride, stream or None, dev_counters or None))

    def render_bands_batch(self, params_list, dev_ptr, *, dst_bytes, frame_stride, band_rows, first_band,
                           band_stride, stream=0, dev_counters=0):
        """frm_render_bands_batch: len(params_list) frames (same scene; the camera, and for the
        Mandelbulb the time, may differ) in
        one launch, frame k at dev_ptr + k * frame_stride; dst_bytes = the size of the buffer at
        dev_ptr (the library checks every frame against it: pass the real allocation, e.g.
        tensor.numel(), never a size derived from the stride)."""
        from ._lib import FrmParameters
        arr = (FrmParameters * len(params_list))()
        for k, p in enumerate(params_list):
            ctypes.memmove(ctypes.addressof(arr[k]), p.to_bytes(), ctypes.sizeof(FrmParameters))
        self._check(self._lib.frm_render_bands_batch(self.ctx, len(params_list), ctypes.addressof(arr), dev_ptr,
                                                     dst_bytes, frame_stride, band_rows, first_band, band_stride,
                                                     stream or None, dev_counters or None))

    def unshuffle_bands(self, src_ptr, rank_stride, dst_ptr, dst_bytes, band_rows, ranks, stream=0):
        self._check(self._lib.frm_unshuffle_bands(self.ctx, src_ptr, rank_stride, dst_ptr, dst_bytes,
                                                  band_rows, ranks, stream or None))

    # diagnostics: scene() and builtins evaluated on the GPU
    MATH_FN = {"sin": 0, "cos": 1, "acos": 2, "atan2": 3, "log": 4, "log2": 5, "exp2": 6,
               "pow": 7, "sqrt": 8, "div": 9,
               # device fast paths (frm_fast.h), each bit-identical to a builtin on its domain
               "sqrt_nosmall": 10, "div_tame": 11, "div_tame_nz": 12, "sin_small": 13,
               "cos_small": 14, "acos_dev": 15, "atan2_tame": 16, "log2_tame": 17,
               "exp2_tame": 18, "log_posnormal": 19,
               # the sRGB store's code (frm_scene.h encode_srgb), as a float
               "srgb_encode": 20}

    def eval_scene(self, points):
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        d = np.zeros(len(pts), np.float32)
        col = np.zeros((len(pts), 3), np.float32)
        self._check(self._lib.frm_eval_scene(self.ctx, pts.ctypes.data, len(pts), d.ctypes.data,
                                             col.ctypes.data))
        return d, col

    def eval_math(self, name, a, b=None):
        a = np.ascontiguousarray(a, dtype=np.float32)
        bb = None if b is None else np.ascontiguousarray(np.broadcast_to(b, a.shape), dtype=np.float32)
        out = np.zeros_like(a)
        self._check(self._lib.frm_eval_math(self.ctx, self.MATH_FN[name], a.ctypes.data,
                                            None if bb is None else bb.ctypes.data, a.size,
                                            out.ctypes.data))
        return out

    def pixel_keys(self):
        """The 8-bit cost keys (16 log2(bodies + 1)) the last persistent launch recorded per
        local pixel, row-major (scheduling diagnostics)."""
        n = self.width * self.height
        out = np.zeros(n, np.uint8)
        got = self._lib.frm_debug_pixel_keys(self.ctx, out.ctypes.data, n)
        if got < 0:
            self._check(got)
        return out[:got]

    def set_pixel_keys(self, keys):
        """Replace the cost keys the next persistent launch sorts its pixels by."""
        k = np.ascontiguousarray(keys, dtype=np.uint8)
        self._check(self._lib.frm_debug_set_pixel_keys(self.ctx, k.ctypes.data, k.size))

    def trace(self):
        """frm_debug_trace: the shading inputs of every pixel of the last render, (H, W, 10) float32
        in the oracle's trace layout (hit, steps, normal xyz, sun hit, sun closeness, colour xyz)."""
        out = np.zeros((self.height, self.width, 10), np.float32)
        self._check(self._lib.frm_debug_trace(self.ctx, out.ctypes.data, out.size))
        return out

    def stats_from_counters(self, counters):
        arr = (ctypes.c_uint64 * _lib.FRM_NUM_COUNTERS)(*[int(c) for c in counters])
        st = _lib.FrmStats()
        self._check(self._lib.frm_stats_from_counters(self.ctx, arr, ctypes.byref(st)))
        return st.as_dict()


def device_count():
    n = ctypes.c_int32(0)
    rc = _lib.load().frm_device_count(ctypes.byref(n))
    return n.value if rc == _lib.FRM_OK else 0
