"""Gate P1, classified (SURVEY.md §8c "flagged classes"): where the frm builtins (MODE_FRM,
bit-exact with the GPU) and float64-libm builtins rounded once (MODE_LIBM, "precise WGSL")
give frames that differ by more than one code in some channel, say why, pixel by pixel.

Both modes render the frame with a per-pixel trace of the shading's geometric inputs (hit,
primary steps, normal, sun hit, sun closeness, object colour; oracle om_render_trace). Two
checks:

1. Shading and encode are mode-independent to within one code: every pixel re-shaded with
   the frm shading (MODE_FRM's pows) from the LIBM march's trace equals the LIBM frame
   within one code. A pixel that fails this is UNEXPLAINED: its difference would come from
   the shading/encode path (fragment.wgsl:336-346 + the Rgba8UnormSrgb store), not from the
   march. Its count must be 0.
2. Every pixel that differs by more than one code is assigned to the first geometric class
   it belongs to:
     hit_miss_flip            the primary march hits in one mode only (fragment.wgsl:334)
     shadow_first_nonpositive the shadow march's first DE is <= 0: closeness = d / 0 is NaN
                              or -inf (fragment.wgsl:292, 344), in either mode
     zero_normal              the four normal taps sum to the zero vector (NaN normal)
     sun_hit_flip             the shadow march hits in one mode only (fragment.wgsl:344)
     ao_step_count            the primary step count differs (ambient occlusion, :341)
   and, for pixels with the same hit, steps and sun hit in both modes, by which single
   geometric input, moved from its FRM value to its LIBM value, brings the frm-shaded pixel
   within one code of the LIBM frame:
     normal                   the hit normal (specular; fragment.wgsl:338-339, 345)
     shadow_closeness         the soft-shadow closeness (:343-345)
     hit_colour               the object colour at the hit point (colorize(position))
     several                  none alone does; all of them together do (check 1)
The chaotic power-8 Mandelbulb moves hit points under a one-ulp builtin change; these
classes are how that shows in the bytes.
"""
import numpy as np

FIELDS = {"hit": 0, "steps": 1, "n": slice(2, 5), "sun_hit": 5, "sun_closeness": 6, "colour": slice(7, 10)}
TOPOLOGY = ("hit_miss_flip", "shadow_first_nonpositive", "zero_normal", "sun_hit_flip", "ao_step_count")
SUBST = (("normal", FIELDS["n"]), ("shadow_closeness", FIELDS["sun_closeness"]), ("hit_colour", FIELDS["colour"]))
CLASSES = TOPOLOGY + tuple(k for k, _ in SUBST) + ("several",)


def _within1(a, b):
    return np.abs(a[..., :3].astype(np.int16) - b[..., :3].astype(np.int16)).max(-1) <= 1


def classify(oracle, params, width, height, max_steps, flags=0, threads=None):
    a = oracle.render(params, width, height, max_steps, flags=flags, threads=threads, info=True, trace=True)
    b = oracle.render(params, width, height, max_steps, flags=flags, mode=oracle.MODE_LIBM, threads=threads,
                      info=True, trace=True)
    ys, xs = np.mgrid[0:height, 0:width]
    xs, ys = xs.ravel(), ys.ravel()
    ra, rb = a["rgba"].reshape(-1, 4), b["rgba"].reshape(-1, 4)
    ia, ib = a["info"].ravel(), b["info"].ravel()
    ta, tb = a["trace"].reshape(-1, 10), b["trace"].reshape(-1, 10)

    # check 1, on every pixel: frm shading of the LIBM geometry vs the LIBM frame
    frm_on_libm = oracle.shade_trace(params, width, height, max_steps, xs, ys, tb, flags=flags)
    shading_ok = _within1(frm_on_libm, rb)
    # ... and the trace reproduces each mode's own frame exactly (the trace is complete)
    own_a = oracle.shade_trace(params, width, height, max_steps, xs, ys, ta, flags=flags)
    assert np.array_equal(own_a, ra), "trace does not reproduce the FRM frame"

    diff = ~_within1(ra, rb)
    idx = np.nonzero(diff)[0]
    cls = np.full(idx.size, "", dtype=object)
    fa, fb = ia[idx], ib[idx]
    rules = [
        ("hit_miss_flip", ((fa ^ fb) & oracle.INFO_HIT) != 0),
        ("shadow_first_nonpositive", ((fa | fb) & oracle.INFO_SHADOW_FIRST_NONPOS) != 0),
        ("zero_normal", ((fa | fb) & oracle.INFO_ZERO_NORMAL) != 0),
        ("sun_hit_flip", ((fa ^ fb) & oracle.INFO_SUN_HIT) != 0),
        ("ao_step_count", (fa >> 8) != (fb >> 8)),
    ]
    for name, m in rules:
        cls[(cls == "") & m] = name
    rest = np.nonzero(cls == "")[0]
    stats = {}
    if rest.size:
        p = idx[rest]
        for name, sl in SUBST:
            t = ta[p].copy()
            t[:, sl] = tb[p][:, sl]
            ok = _within1(oracle.shade_trace(params, width, height, max_steps, xs[p], ys[p], t, flags=flags), rb[p])
            sel = ok & (cls[rest] == "")
            cls[rest[sel]] = name
        cls[cls == ""] = "several"
        # size of the geometric moves behind the continuous classes
        na, nb = ta[p][:, 2:5].astype(np.float64), tb[p][:, 2:5].astype(np.float64)
        cosang = np.clip(np.sum(na * nb, -1) / np.maximum(1e-30, np.linalg.norm(na, axis=-1) * np.linalg.norm(nb, axis=-1)),
                         -1, 1)
        ang = np.degrees(np.arccos(cosang))
        stats["normal_angle_deg_median"] = float(np.median(ang))
        stats["normal_angle_deg_p99"] = float(np.percentile(ang, 99))
    counts = {k: int(np.sum(cls == k)) for k in CLASSES}
    unexplained = int(np.sum(~shading_ok[idx]))
    hits = int(np.sum((ia & oracle.INFO_HIT) != 0))
    return {
        "width": width, "height": height, "pixels": width * height, "hit_pixels": hits,
        "differ_gt1": int(idx.size), "differ_gt1_frac": idx.size / (width * height),
        "differ_any": int(np.sum(np.any(ra[:, :3] != rb[:, :3], -1))),
        "classes": counts,
        "unexplained": unexplained,
        "shading_mode_gt1_anywhere": int(np.sum(~shading_ok)),
        "march_steps_frm": int(a["counters"][2] + a["counters"][3]),
        "march_steps_libm": int(b["counters"][2] + b["counters"][3]),
        **stats,
    }


def trace_info(oracle, trace):
    """The oracle's per-pixel info word (flags + primary steps << 8) rebuilt from a trace, for a
    frame that has a trace but no oracle render (a GPU frame, frm_debug_trace)."""
    t = trace.reshape(-1, 10)
    hit = t[:, 0] != 0
    cl = t[:, 6]
    info = np.where(hit, oracle.INFO_HIT, 0)
    info |= np.where(hit & (t[:, 5] != 0), oracle.INFO_SUN_HIT, 0)
    info |= np.where(hit & (np.isnan(cl) | (cl == -np.inf)), oracle.INFO_SHADOW_FIRST_NONPOS, 0)
    info |= np.where(hit & np.isnan(t[:, 2]), oracle.INFO_ZERO_NORMAL, 0)
    return (info | (t[:, 1].astype(np.int64) << 8)).astype(np.int64)


def classify_frame(oracle, params, width, height, max_steps, rgba, trace, flags=0, threads=None):
    """classify() for a frame that is not the oracle's own (e.g. the GPU's FRM_FLAG_HW_MATH frame,
    with its trace from frm_debug_trace) against the MODE_LIBM oracle: first, the frame's trace
    re-shaded with the frm shading reproduces the frame's bytes exactly (`trace_reproduces`:
    every difference is then geometric, none comes from the shading or the encode); then the same
    classes and the same `unexplained` count as classify()."""
    b = oracle.render(params, width, height, max_steps, flags=flags, mode=oracle.MODE_LIBM, threads=threads,
                      info=True, trace=True)
    ys, xs = np.mgrid[0:height, 0:width]
    xs, ys = xs.ravel(), ys.ravel()
    ra, rb = rgba.reshape(-1, 4), b["rgba"].reshape(-1, 4)
    ta, tb = trace.reshape(-1, 10).astype(np.float32), b["trace"].reshape(-1, 10)
    ia, ib = trace_info(oracle, trace), b["info"].ravel().astype(np.int64)
    own_a = oracle.shade_trace(params, width, height, max_steps, xs, ys, ta, flags=flags)
    reproduces = int(np.sum(np.any(own_a != ra, -1)))
    frm_on_libm = oracle.shade_trace(params, width, height, max_steps, xs, ys, tb, flags=flags)
    shading_ok = _within1(frm_on_libm, rb)
    diff = ~_within1(ra, rb)
    idx = np.nonzero(diff)[0]
    cls = np.full(idx.size, "", dtype=object)
    fa, fb = ia[idx], ib[idx]
    rules = [
        ("hit_miss_flip", ((fa ^ fb) & oracle.INFO_HIT) != 0),
        ("shadow_first_nonpositive", ((fa | fb) & oracle.INFO_SHADOW_FIRST_NONPOS) != 0),
        ("zero_normal", ((fa | fb) & oracle.INFO_ZERO_NORMAL) != 0),
        ("sun_hit_flip", ((fa ^ fb) & oracle.INFO_SUN_HIT) != 0),
        ("ao_step_count", (fa >> 8) != (fb >> 8)),
    ]
    for name, m in rules:
        cls[(cls == "") & m] = name
    rest = np.nonzero(cls == "")[0]
    if rest.size:
        p = idx[rest]
        for name, sl in SUBST:
            t = ta[p].copy()
            t[:, sl] = tb[p][:, sl]
            ok = _within1(oracle.shade_trace(params, width, height, max_steps, xs[p], ys[p], t, flags=flags), rb[p])
            sel = ok & (cls[rest] == "")
            cls[rest[sel]] = name
        cls[cls == ""] = "several"
    return {
        "width": width, "height": height, "pixels": width * height,
        "trace_mismatch_pixels": reproduces,
        "differ_gt1": int(idx.size), "differ_gt1_frac": idx.size / (width * height),
        "differ_any": int(np.sum(np.any(ra[:, :3] != rb[:, :3], -1))),
        "classes": {k: int(np.sum(cls == k)) for k in CLASSES},
        "unexplained": int(np.sum(~shading_ok[idx])),
        "march_steps_libm": int(b["counters"][2] + b["counters"][3]),
    }
