"""First-frame cost after a resize: headline frames (3840x2160, pose P1) timed one
at a time (frm_render with stats: the launch's own HIP-event time), on a fresh context (no
scheduling history: row-major fetch order), in the steady state, and right after a resize
(history resampled from the previous size's keys). The previous sizes: 1920x1080, and the
reference's own resize step, RenderTextureConfig's factor +-1 (render_texture_config.rs:7-13:
160*f x 90*f; 4K is f = 24, so f = 23 and f = 25). Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fractal-ray-marching_amd")]
import frm  # noqa: E402


def frame_ms(r):
    return r.render(stats=True)["kernel_ms"]


w = frm.WORKLOADS["HEADLINE"]
p4k = frm.make_parameters(w, pose="P1")
out = {}
with frm.Renderer(device=0, max_steps=w.max_steps) as r:
    r.resize(w.width, w.height)
    r.update_parameters_buffer(p4k)
    out["first_frame_no_history_ms"] = frame_ms(r)
    out["steady_ms"] = min(frame_ms(r) for _ in range(5))
    for name, (pw, ph) in (("1080p", (1920, 1080)), ("factor23", (160 * 23, 90 * 23)),
                           ("factor25", (160 * 25, 90 * 25))):
        pp = frm.make_parameters(w, pose="P1", width=pw, height=ph)
        for rnd in range(3):
            r.resize(pw, ph)
            r.update_parameters_buffer(pp)
            for _ in range(3):
                frame_ms(r)
            r.resize(w.width, w.height)
            r.update_parameters_buffer(p4k)
            out.setdefault(f"first_frame_after_resize_from_{name}_ms", []).append(frame_ms(r))
            out.setdefault(f"second_frame_after_resize_from_{name}_ms", []).append(frame_ms(r))
print(json.dumps(out))
