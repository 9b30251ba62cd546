"""C ABI boundary (include/frm.h): the library loads, exports every declared entry point,
struct layouts match the reference's Parameters byte for byte, and errors are reported
as status codes + messages (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

import frm
from frm import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "frm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(frm_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported(frm_lib):
    names = declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(frm_lib, name), f"libfrm.so does not export {name}"
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(names) == bound, f"ctypes bindings out of sync: {set(names) ^ bound}"


def test_abi_version(frm_lib):
    assert frm_lib.frm_abi_version() == 5


def test_struct_layout_matches_c(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "frm.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(frm_parameters), offsetof(frm_parameters, aspect_scale),
         offsetof(frm_parameters, time), offsetof(frm_parameters, num_iterations),
         offsetof(frm_parameters, scene_index), offsetof(frm_parameters, padding));
  printf("%zu %zu\n", sizeof(frm_config), sizeof(frm_stats));
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)])
    lines = subprocess.check_output([str(exe)]).decode().split("\n")
    got = [int(v) for v in lines[0].split()]
    P = _lib.FrmParameters
    assert got == [96, 64, 72, 76, 80, 84]  # src/parameters.rs:6-15 (verified offsets)
    assert got == [ctypes.sizeof(P), P.aspect_scale.offset, P.time.offset, P.num_iterations.offset,
                   P.scene_index.offset, P.padding.offset]
    cfg, stats = (int(v) for v in lines[1].split())
    assert cfg == ctypes.sizeof(_lib.FrmConfig) and stats == ctypes.sizeof(_lib.FrmStats)


def test_errors_are_codes_not_crashes(frm_lib):
    L = frm_lib
    assert L.frm_resize(None, 10, 10) == _lib.FRM_ERR_INVALID_ARGUMENT
    assert b"NULL" in L.frm_last_error(None)
    assert L.frm_render(None, None) == _lib.FRM_ERR_INVALID_ARGUMENT
    assert L.frm_create(None, None) == _lib.FRM_ERR_INVALID_ARGUMENT
    out = ctypes.c_uint32()
    assert L.frm_band_rows_for(0, 4, 0, 1, ctypes.byref(out)) == _lib.FRM_ERR_INVALID_ARGUMENT
    assert L.frm_destroy(None) == _lib.FRM_OK
    ctx = ctypes.c_void_p()
    bad = _lib.FrmConfig(0, 0, 0, _lib.FRM_MAX_FRAMES_IN_FLIGHT + 1)  # frames_in_flight above the cap
    assert L.frm_create(ctypes.byref(ctx), ctypes.byref(bad)) == _lib.FRM_ERR_INVALID_ARGUMENT
    bad = _lib.FrmConfig(0, _lib.FRM_MAX_STEPS_LIMIT + 1, 0, 1)  # max_steps above the record's 22 bits
    assert L.frm_create(ctypes.byref(ctx), ctypes.byref(bad)) == _lib.FRM_ERR_INVALID_ARGUMENT
    assert b"max_steps" in L.frm_last_error(None)


def test_create_without_gpu_reports_no_device(frm_lib):
    if frm.device_count() > 0:
        pytest.skip("a GPU is visible (covered by the gpu tests)")
    with pytest.raises(frm.FrmError) as e:
        frm.Renderer(device=0)
    assert e.value.code == _lib.FRM_ERR_NO_DEVICE


@pytest.mark.parametrize("height,band_rows,ranks", [(2160, 270, 8), (2160, 15, 8), (1080, 16, 3), (7, 4, 2), (4320, 45, 4)])
def test_band_rows_for_matches_tiling(frm_lib, height, band_rows, ranks):
    from frm import tiling
    for rank in range(ranks):
        out = ctypes.c_uint32()
        assert frm_lib.frm_band_rows_for(height, band_rows, rank, ranks, ctypes.byref(out)) == 0
        assert out.value == tiling.rank_rows(height, band_rows, rank, ranks)


@pytest.mark.parametrize("height,devices", [(2160, 8), (2160, 4), (2160, 2), (4320, 8), (16384, 8), (1080, 3),
                                            (7, 2), (100, 16), (2160, 1), (17, 5)])
def test_group_band_rows_matches_tiling(frm_lib, height, devices):
    """A group context's row split (frm_config.device_count) uses the band height of frm/tiling.py,
    the one the multi-process row split uses, and its rank shares cover the frame exactly."""
    from frm import tiling
    out = ctypes.c_uint32()
    assert frm_lib.frm_group_band_rows(height, devices, ctypes.byref(out)) == _lib.FRM_OK
    assert out.value == tiling.choose_band_rows(height, devices)
    rows = []
    for r in range(devices):
        got = ctypes.c_uint32()
        assert frm_lib.frm_band_rows_for(height, out.value, r, devices, ctypes.byref(got)) == 0
        rows.append(got.value)
    nb = -(-height // out.value)
    assert sum(rows) == nb * out.value  # every band once (the last one padded to band_rows)
    assert rows[0] == max(rows)  # rank 0's share sizes the gather buffer's rank stride


def test_group_config_errors(frm_lib):
    L = frm_lib
    out = ctypes.c_uint32()
    for h, n in ((0, 2), (2160, 0), (2160, 17)):
        assert L.frm_group_band_rows(h, n, ctypes.byref(out)) == _lib.FRM_ERR_INVALID_ARGUMENT
    assert L.frm_group_band_rows(2160, 2, None) == _lib.FRM_ERR_INVALID_ARGUMENT
    ctx = ctypes.c_void_p()
    bad = _lib.FrmConfig(0, 0, 0, 1)
    bad.device_count = _lib.FRM_MAX_DEVICES + 1  # above the device list
    assert L.frm_create(ctypes.byref(ctx), ctypes.byref(bad)) == _lib.FRM_ERR_INVALID_ARGUMENT
    assert b"device_count" in L.frm_last_error(None)
    assert not ctx.value
    if frm.device_count() == 0:  # no GPU here: a valid group config reports the missing device
        ok = _lib.FrmConfig(0, 0, 0, 2)
        ok.device_count = 2
        assert L.frm_create(ctypes.byref(ctx), ctypes.byref(ok)) == _lib.FRM_ERR_NO_DEVICE
    with pytest.raises(ValueError):
        frm.Renderer(devices=[])
