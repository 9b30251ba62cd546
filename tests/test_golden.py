"""The oracle (and the host-side Parameters construction) against the committed golden
fixtures of tests/golden/ (made by tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import frm
from helpers import params_for

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_frames():
    with open(os.path.join(GOLD, "frames.json")) as f:
        return json.load(f)


def test_parameters_blobs_are_reproduced():
    for case in load_frames():
        p = params_for(case["scene"], case["iters"], case["time"], case["width"], case["height"])
        assert p.to_bytes().hex() == case["params"]
    cams = json.load(open(os.path.join(GOLD, "camera.json")))
    for pose, blob in cams.items():
        assert frm.make_parameters(frm.WORKLOADS["HEADLINE"], pose=pose).to_bytes().hex() == blob


def test_oracle_frames_match_golden(oracle):
    for case in load_frames():
        p = frm.Parameters.from_bytes(bytes.fromhex(case["params"]))
        r = oracle.render(p, case["width"], case["height"], case["max_steps"])
        assert hashlib.sha256(r["rgba"].tobytes()).hexdigest() == case["sha256"], case
        assert [int(c) for c in r["counters"]] == case["counters"], case


def test_oracle_full_frames_match_golden(oracle):
    g = np.load(os.path.join(GOLD, "frames.npz"))
    for pose in ("P0", "P1", "P2"):
        p = frm.Parameters.from_bytes(g[f"mandelbulb_{pose}_params"].tobytes())
        assert np.array_equal(oracle.render(p, 96, 54, 256)["rgba"], g[f"mandelbulb_{pose}"])
    p = frm.Parameters.from_bytes(g["sphere_c1_params"].tobytes())
    assert np.array_equal(oracle.render(p, 256, 256, 64, flags=frm.FRM_FLAG_SCENE_SPHERE)["rgba"],
                          g["sphere_c1"])


def test_oracle_de_matches_golden(oracle):
    g = np.load(os.path.join(GOLD, "de.npz"))
    pts = g["points"]
    for scene in (0, 15, 16, 18):
        for n in (0, 3, 8, 12):
            p = params_for(scene, n, 3.2175055, 64, 36)
            d, col, _ = oracle.scene_de(p, pts)
            assert np.array_equal(d.view(np.uint32), g[f"s{scene}_n{n}_d"].view(np.uint32))
            assert np.array_equal(col, g[f"s{scene}_n{n}_c"])


def test_default_parameters_blob_and_oracle_at_5000_steps(oracle):
    """tests/golden/defaults.json (make_defaults_golden.py): the DEFAULT frame's Parameters are
    Parameters::default() + update_aspect(1920, 1080) + update_camera(Camera::default())
    (initialized_app.rs:24, camera.rs:176-187), every sweep blob is P1 with the recorded scene,
    iterations and time, and the oracle still renders the cheap frames' recorded hashes and
    counters at 5000 steps (the GPU side is tests/test_gpu_defaults.py)."""
    g = json.load(open(os.path.join(GOLD, "defaults.json")))
    p = frm.Parameters()
    p.update_aspect(1920, 1080)
    p.update_camera(frm.Camera())
    assert p.to_bytes().hex() == g["DEFAULT"]["params"]
    for key, e in g.items():
        if key.startswith("S"):
            q = frm.make_parameters(frm.WORKLOADS["C2"], pose="P1")
            q.scene_index, q.num_iterations, q.time = e["scene_index"], e["num_iterations"], e["time"]
            assert q.to_bytes().hex() == e["params"], key
    for key in ("DEFAULT", "S0_N3_t0", "S16_N3_t0"):
        e = g[key]
        r = oracle.render(frm.Parameters.from_bytes(bytes.fromhex(e["params"])), e["width"], e["height"],
                          e["max_steps"], threads=os.cpu_count())
        assert hashlib.sha256(r["rgba"].tobytes()).hexdigest() == e["sha256"], key
        assert [int(c) for c in r["counters"]] == e["counters"], key
