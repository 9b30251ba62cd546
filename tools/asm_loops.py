"""List the loops (backward branches) of a kernel in hipcc -S output with their
instruction mix: VALU / trans / SALU / memory counts per loop body (straight-line
count of the blocks between the loop label and the back edge)."""
import re
import sys

TRANS = re.compile(r"^v_(rcp|rsq|sqrt|log|exp|sin|cos|frexp|ldexp)_")


def functions(path):
    cur, name = None, None
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
                yield name, cur
                cur = None
                continue
            cur.append(line.rstrip("\n"))


def mix(lines):
    c = {"valu": 0, "trans": 0, "salu": 0, "vmem": 0, "lds": 0, "branch": 0, "total": 0}
    for l in lines:
        s = l.strip()
        if not s or s.startswith(("//", ".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c["total"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
            if TRANS.match(op):
                c["trans"] += 1
        elif op.startswith("s_cbranch") or op == "s_branch":
            c["branch"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    return c


def main(path, pat):
    for name, body in functions(path):
        if pat not in name:
            continue
        labels = {}
        for i, l in enumerate(body):
            m = re.match(r"^(\.LBB\S+):", l)
            if m:
                labels[m.group(1)] = i
        print(name, "lines", len(body), "mix", mix(body))
        for i, l in enumerate(body):
            m = re.match(r"^\s*s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
            if m and m.group(2) in labels and labels[m.group(2)] < i:
                j = labels[m.group(2)]
                print(f"  loop {m.group(2)} lines {j}-{i}: {mix(body[j:i + 1])}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "march_persistent")
