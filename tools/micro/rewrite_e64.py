# Usage (container): hipcc --cuda-device-only -S ... -o a.s; python rewrite_e64.py a.s b.s;
#   clang -target amdgcn-amd-amdhsa -mcpu=gfx950 -c b.s -o b.o; ld.lld -shared b.o -o b.hsaco
"""Peephole over hipcc device asm: VOP2 v_cndmask_b32_e32 (implicit VCC mask) -> VOP3
v_cndmask_b32_e64 with VCC as an explicit operand, where src0 is a register or inline
constant (VOP3 on gfx9 takes no literal)."""
import re
import sys

pat = re.compile(r"^(\s*)v_cndmask_b32_e32 (v\d+), ([^,]+), (v\d+), vcc\s*$")
n = skipped = 0
out = []
for line in open(sys.argv[1]):
    m = pat.match(line.rstrip("\n"))
    if m:
        ind, d, s0, s1 = m.groups()
        if s0.startswith("0x") and s0 not in ("0x0",):
            skipped += 1
            out.append(line)
            continue
        out.append(f"{ind}v_cndmask_b32_e64 {d}, {s0}, {s1}, vcc\n")
        n += 1
    else:
        out.append(line)
open(sys.argv[2], "w").writelines(out)
print(f"rewrote {n}, kept {skipped} (literal src0)", file=sys.stderr)
