"""bench.py's multi-rank launch on a 1-GPU box: `python bench.py --gpus 2` with no launcher
environment starts its own two ranks (a child torch.distributed.run), renders the row split
(interleaved bands, gather to rank 0, reassembly) and checks the reassembled frame against
the oracle's whole-frame golden hash. The two ranks share device 0 over gloo (bench.py's test
hooks: RCCL refuses two ranks on one GPU); the driver's multi-GPU runs use RCCL."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("split", ["rows", "frames"])
def test_bench_launches_its_own_ranks(split):
    env = dict(os.environ, FRM_BENCH_SHARED_DEVICE="1", FRM_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "C2", "--split", split,
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["comm"] == {
        "backend": "gloo", "ranks": 2,
        "data_path": "dist.gather of row bands to rank 0" if split == "rows" else "none (timing only)"}
    assert out["frame_sha_ok"] is True, out.get("frame_sha256")
    assert out["launcher"].startswith("bench.py")
    # the row split renders one frame per step over both ranks; alternate frames two
    per_frame = out["march_steps_per_frame"]
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))["C2_P1"]["counters"]
    if split == "rows":
        assert per_frame == gold[2] + gold[3]
