"""Compiler canary for the ITERS workaround (csrc/frm_scene.h `iterations<>`).

ROCm 7.2's AMDGPU backend miscompiled the fold loops' uniform guard "num_iterations > 0" inside
the divergent march loop: the guard is materialised as a 0/1 VGPR before the loop and turned
back into a lane mask by a `v_cmp ... 1, vN` INSIDE the loop, under the loop's exec mask. Lanes
that left the march in an earlier iteration get a 0 bit, and after the loop (normal taps, under
the hit lanes' exec mask) that stale mask re-enters the fold loop with n = 0: about 2^32 folds.
The product never evaluates the guard (the fold loops are instantiated for n = 0 and for
n >= 1 with the trip count asserted).

This test compiles tests/canary/iters_guard.hip (the Sierpinski simple kernel; assembly only,
never run) twice with hipcc for gfx950:
* without the workaround: the signature must still be there. If a compiler update removes
  it, this test fails to say so: re-run the num_iterations == 0 sweeps without the split
  (tests/test_gpu_parity.py) before simplifying `iterations<>`;
* with the workaround (the product's form): the signature must be absent.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fractal-ray-marching_amd")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SRC = os.path.join(ROOT, "tests", "canary", "iters_guard.hip")
KERNEL = "_ZN3frm13render_simpleILj1ELb1EEEvNS_10KernelArgsE"  # render_simple<kSierpinski, true>


def compile_asm(tmp_path, workaround):
    out = tmp_path / ("with.s" if workaround else "without.s")
    # the product's device flags (fractal-ray-marching_amd/Makefile COMMON + HIPFLAGS)
    cmd = [HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-function",
           "-Wno-unknown-pragmas", "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"),
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "--cuda-device-only", "-S", SRC, "-o", str(out)]
    if workaround:
        cmd.insert(1, "-DFRM_CANARY_WITH_WORKAROUND")
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    return out.read_text()


def kernel_lines(asm, name):
    lines, inside = [], False
    for line in asm.splitlines():
        if line.startswith(name + ":"):
            inside = True
            continue
        if inside:
            if line.startswith(".Lfunc_end") or line.strip().startswith(".end_amdhsa_kernel"):
                break
            lines.append(line)
    assert lines, f"kernel {name} not found in the assembly"
    return lines


def block_loops(lines):
    """For every line, the loops (by header block) its basic block belongs to, from the loop
    annotations the compiler writes on block labels ("This Loop Header", "in Loop: Header=",
    "Parent Loop"; an inner header's depth-2 note sits on the line after its label)."""
    out, cur = [], frozenset()
    for i, line in enumerate(lines):
        m = re.match(r"^\.L(BB\d+_\d+):(.*)$", line)
        if m:
            note = m.group(2) + (lines[i + 1] if i + 1 < len(lines) and lines[i + 1].lstrip().startswith(";") else "")
            hdrs = set(re.findall(r"(?:Header=|Parent Loop )(BB\d+_\d+)", note))
            if "Loop Header" in note:
                hdrs.add(m.group(1))
            cur = frozenset(hdrs)
        out.append(cur)
    return out


def guard_remat_in_loop(lines):
    """Sites where a 0/1 VGPR defined outside a loop is compared against 1 inside it."""
    sites = []
    where = block_loops(lines)
    for c, line in enumerate(lines):
        m = re.match(r"^\s*v_cndmask_b32_e64 (v\d+), 0, 1, s\[\d+:\d+\]", line)
        if not m:
            continue
        v = m.group(1)
        redef = re.compile(r"^\s*v_\w+ " + v + r",")
        use = re.compile(r"^\s*v_cmp_(ne|eq)_u32_e(32|64) (s\[\d+:\d+\]|vcc), 1, " + v + r"\s*$")
        for k in range(c + 1, len(lines)):
            if redef.match(lines[k]):
                break
            if use.match(lines[k]) and where[k] - where[c]:
                sites.append((c, k, v, sorted(where[k] - where[c])))
    return sites


pytestmark = pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="no hipcc")


def test_miscompile_signature_without_workaround(tmp_path):
    sites = guard_remat_in_loop(kernel_lines(compile_asm(tmp_path, workaround=False), KERNEL))
    assert sites, ("this hipcc no longer rematerialises the fold-loop guard inside the march loop: "
                   "re-check whether the ITERS split of csrc/frm_scene.h is still needed (DESIGN.md §8)")


def test_no_signature_in_product_form(tmp_path):
    assert guard_remat_in_loop(kernel_lines(compile_asm(tmp_path, workaround=True), KERNEL)) == []
