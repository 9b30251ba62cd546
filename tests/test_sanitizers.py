"""Host code under sanitizers: libfrm's host mirrors (csrc/frm_host.cpp) and the
CPU oracle (oracle/frm_oracle.c, including its thread pool) built with gcc's
AddressSanitizer + UndefinedBehaviorSanitizer, and separately ThreadSanitizer, then driven
through every entry point by tests/native/sanitize_driver.cpp. Any report fails the run
(-fno-sanitize-recover, halt_on_error). GPU sanitizers are not available for gfx950 here."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
CSRC = os.path.join(ROOT, "fractal-ray-marching_amd", "csrc")

FLAGS = {
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


def build(kind, tmp_path):
    out = str(tmp_path / f"sanitize_{kind}")
    common = ["-g", "-O1", "-ffp-contract=off", "-fno-fast-math", "-I", os.path.join(ROOT, "include"), "-I", CSRC]
    obj = str(tmp_path / f"oracle_{kind}.o")
    subprocess.check_call(["gcc", "-std=gnu11", "-c", os.path.join(ROOT, "oracle", "frm_oracle.c"), "-o", obj]
                          + common + FLAGS[kind])
    subprocess.check_call(["g++", "-std=c++17", os.path.join(NATIVE, "sanitize_driver.cpp"),
                           os.path.join(CSRC, "frm_host.cpp"), obj, "-o", out, "-lm", "-lpthread"]
                          + common + FLAGS[kind])
    return out


@pytest.mark.parametrize("kind", ["asan_ubsan", "tsan"])
def test_host_code_under_sanitizers(tmp_path, kind):
    exe = build(kind, tmp_path)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:halt_on_error=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    r = subprocess.run([exe, "4"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, f"{kind}: rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert "sanitize_driver ok" in r.stdout
