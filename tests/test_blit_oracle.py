"""§8(f) row 4 — the presentation resample, CPU side: the oracle's restatement (om_blit)
pinned by known answers: the sRGB decode table against mpmath at 50 digits, exact
decode/encode round trips, nearest texel selection when minifying, constant images,
byte order."""
import mpmath as mp
import numpy as np

from oracle import frm_oracle as o


def test_decode_table_is_the_correctly_rounded_inverse_transfer():
    mp.mp.dps = 50
    want = []
    for k in range(256):
        s = mp.mpf(k) / 255
        lin = s / mp.mpf("12.92") if s <= mp.mpf("0.04045") else ((s + mp.mpf("0.055")) / mp.mpf("1.055")) ** mp.mpf("2.4")
        want.append(np.float32(float(lin)))
    assert np.array_equal(o.srgb_decode(), np.array(want, np.float32))


def test_decode_then_encode_is_identity():
    assert np.array_equal(o.encode_srgb(o.srgb_decode()), np.arange(256, dtype=np.uint8))


def frame(h, w, seed=0):
    rgba = np.random.default_rng(seed).integers(0, 256, (h, w, 4), dtype=np.uint8)
    rgba[..., 3] = 255
    return rgba


def test_same_size_is_identity_and_bgra_swaps():
    f = frame(9, 16)
    assert np.array_equal(o.blit(f, 16, 9, 1), f)
    assert np.array_equal(o.blit(f, 16, 9, 3), f[..., [2, 1, 0, 3]])


def test_minify_takes_the_nearest_texel():
    f = frame(20, 40, 1)
    got = o.blit(f, 20, 10, 1)  # 2 texels per pixel: u*W = 2x + 1 up to f32 rounding
    f32 = np.float32
    x, y = np.arange(20, dtype=np.uint32), np.arange(10, dtype=np.uint32)
    u = (f32(2 * x + 1) / f32(20) - f32(1) + f32(1)) * f32(0.5)
    v = f32(1) - (f32(1) - f32(2 * y + 1) / f32(10) + f32(1)) * f32(0.5)
    ix = np.clip(np.floor(u * f32(40)).astype(int), 0, 39)
    iy = np.clip(np.floor(v * f32(20)).astype(int), 0, 19)
    assert set(ix - 2 * x.astype(int)) <= {0, 1}  # the texel under the pixel centre, or its left neighbour
    assert np.array_equal(got, f[iy][:, ix])


def test_magnify_keeps_constant_images_and_linear_output():
    f = np.zeros((6, 8, 4), np.uint8)
    f[..., :3] = 188
    f[..., 3] = 255
    assert np.array_equal(o.blit(f, 21, 13, 1), np.broadcast_to(f[0, 0], (13, 21, 4)))
    lin = o.blit(f, 21, 13, 0)  # linear unorm surface: round(255 * decode(188))
    assert (lin[..., :3] == int(np.rint(o.srgb_decode()[188] * 255))).all()
