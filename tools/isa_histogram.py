"""Instruction histogram of march_persistent's hot blocks from the gfx950 ISA (`make asm` ->
build/frm_kernels.s), priced with the measured issue costs of tools/micro/isa_rate.hip
(profiles/round1/micro/isa_rate.txt: wall cycles per wave-instruction per SIMD at 8 waves/SIMD;
opcodes it did not measure are priced by the class they resemble and marked '~').

usage: python tools/isa_histogram.py build/frm_kernels.s [KERNEL_SUBSTRING]

Blocks of the Mandelbulb kernel (found from the structure the compiler emits):
  tame test    the inner loop's head up to the branch into the exact body
  tame body    the fast-path body (frm_fast.h) up to the join with the exact body
  loop tail    body count, magnitude (the common sqrt_nosmall path), bailout test, back edge
  service      from the inner loop's exit to the outer loop's back edge (all paths counted once)
"""
import re
import sys
from collections import Counter

PRICE = {  # measured (isa_rate.txt, w8 wall column)
    "v_fma_f32": 2.97, "v_fmac_f32": 2.97, "v_fmaak_f32": 2.86, "v_fmamk_f32": 2.86, "v_mul_f32": 3.23,
    "v_add_u32": 3.17, "v_sub_u32": 3.17, "v_cndmask_b32_e64": 4.45, "v_cmp": 4.80, "v_cmpx": 4.80,
    "v_rndne_f32": 4.36, "v_cvt": 4.30, "v_ldexp_f32": 4.41, "v_frexp_mant_f32": 4.41, "v_frexp_exp_i32_f32": 4.24,
    "v_rcp_f32": 8.55, "v_sqrt_f32": 8.26, "v_bfi_b32": 4.42, "v_max3_f32": 4.44, "v_mov_b32": 2.55,
    "v_sub_f32": 2.64, "v_add_f32": 2.64, "v_cmp_class_f32": 4.81, "v_subbrev_co_u32": 4.66,
    "v_cndmask_b32_e32": 3.6,  # a compare + VOP2 select pair measured 7.2 (isa_rate 'cmp vcc + cndmask e32')
}
GUESS = {  # not measured: priced like the closest measured class
    "v_and_b32": 3.17, "v_or_b32": 3.17, "v_xor_b32": 3.17, "v_lshlrev_b32": 3.17, "v_lshrrev_b32": 3.17,
    "v_ashrrev_i32": 3.17, "v_max_f32": 2.64, "v_min_f32": 2.64, "v_bfe_i32": 4.42, "v_bitop3_b32": 4.42,
    "v_lshl_add_u32": 4.42, "v_lshl_or_b32": 4.42, "v_min3_u32": 4.44, "v_med3_f32": 4.44, "v_or3_b32": 4.42,
    "v_pk_fma_f32": 5.94, "v_pk_mul_f32": 6.46, "v_pk_add_f32": 5.28, "v_mov_b64": 2.55, "v_div_scale_f32": 4.41,
    "v_div_fmas_f32": 4.41, "v_div_fixup_f32": 4.41, "v_mbcnt_lo_u32_b32": 3.17, "v_mbcnt_hi_u32_b32": 3.17,
    "v_readfirstlane_b32": 4.8, "v_mul_hi_u32": 8.55, "v_mul_lo_u32": 8.55, "v_mad_u64_u32": 8.55,
    "v_exp_f32": 8.55, "v_log_f32": 8.55, "v_sin_f32": 8.55, "v_cos_f32": 8.55,
}


def base(op):
    if op.startswith("v_cmp_class"):
        return "v_cmp_class_f32"
    if op.startswith("v_cmpx"):
        return "v_cmpx"
    if op.startswith("v_cmp"):
        return "v_cmp"
    if op.startswith("v_cvt"):
        return "v_cvt"
    if op in ("v_cndmask_b32_e64", "v_cndmask_b32_e32"):
        return op
    return re.sub(r"_e(32|64)$", "", op)


def price(op):
    b = base(op)
    if b in PRICE:
        return PRICE[b], ""
    if b in GUESS:
        return GUESS[b], "~"
    return 3.2, "?"


def kernel_lines(path, want):
    lines, on = [], False
    for line in open(path):
        if re.match(r"^_Z\S+:", line):
            on = want in line
            continue
        if on:
            if line.strip() == "s_endpgm":
                break
            lines.append(line.rstrip("\n"))
    return lines


def block(lines, start, end):
    return lines[start:end]


def hist(lines):
    c = Counter()
    for l in lines:
        s = l.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith(("v_", "s_", "ds_", "global_", "buffer_", "flat_")):
            c[op] += 1
    return c


def report(name, c):
    v = {op: n for op, n in c.items() if op.startswith("v_")}
    other = {op: n for op, n in c.items() if not op.startswith("v_")}
    cyc = sum(price(op)[0] * n for op, n in v.items())
    print(f"== {name}: {sum(v.values())} VALU ({cyc:.0f} priced cycles per wave-pass), "
          f"{sum(n for op, n in other.items() if op.startswith('s_'))} SALU/branch, "
          f"{sum(n for op, n in other.items() if not op.startswith('s_'))} memory")
    for op, n in sorted(v.items(), key=lambda kv: -price(kv[0])[0] * kv[1]):
        p, mark = price(op)
        print(f"   {op:28s} {n:4d} x {p:5.2f}{mark:1s} = {p * n:6.1f}")


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "march_persistentILj3ELb1ELb1E"
    L = kernel_lines(path, want)
    head = next(i for i, l in enumerate(L) if "Inner Loop Header: Depth=2" in l)
    while not L[head].startswith(".LBB"):
        head -= 1  # the header comment follows its label
    lab = lambda i: L[i].split(":")[0]  # noqa: E731
    # tame test: from the header to the vccz branch into the exact body (taken when all lanes are tame)
    br = next(i for i in range(head, len(L)) if L[i].strip().startswith("s_cbranch_vccz"))
    tame_target = L[br].split()[-1]
    t0 = next(i for i in range(br, len(L)) if L[i].startswith(tame_target + ":"))
    t_start = t0 + 1
    while not L[t_start].startswith(".LBB"):
        t_start += 1  # the fall-through label after the (empty) target is the tame body
    # tame body ends at the next label that other paths join (the body-count increment)
    t_end = next(i for i in range(t_start + 1, len(L)) if L[i].startswith(".LBB") and "v_add_u32" in L[i + 1])
    back = next(i for i in range(t_end, len(L)) if re.search(r"s_cbranch_vccz " + re.escape(lab(head)) + r"$", L[i]))
    tail = block(L, t_end, back + 1)
    # the exact (small-magnitude) sqrt path of the tail is the block with the 2^32 rescale
    tail_common = [l for l in tail]
    exact_sqrt = [i for i, l in enumerate(tail) if "0x4f800000" in l]
    if exact_sqrt:
        s0 = exact_sqrt[0]
        s1 = next(i for i in range(s0, len(tail)) if tail[i].strip().startswith("s_cbranch_execnz"))
        tail_common = tail[:s0] + tail[s1 + 1:]
    outer = next(i for i in range(back, len(L)) if re.search(r"s_cbranch_\w+ \.LBB\d+_[12]$", L[i]))
    print(f"kernel {want}: inner loop {lab(head)}, tame body {L[t_start].split(':')[0]} .. {L[t_end].split(':')[0]}, "
          f"service {back + 1} .. {outer} (lines in the kernel)")
    report("tame test", hist(block(L, head, br + 1)))
    report("tame body", hist(block(L, t_start, t_end)))
    report("loop tail (common sqrt path)", hist(tail_common))
    report("service pass (every path once)", hist(block(L, back + 1, outer + 1)))


if __name__ == "__main__":
    main()
