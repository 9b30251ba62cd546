"""Which kernel sources a measurement belongs to: a hash of csrc/ + include/frm.h + the
Makefile, recorded in every committed PMC summary (tools/pmc_summary.py) and checked by
bench.py before it cites one, so counters measured on an older kernel are never reported
as the current kernel's."""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)


def source_files():
    csrc = os.path.join(PKG, "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".h", ".hip", ".cpp")))
    return files + [os.path.join(ROOT, "include", "frm.h"), os.path.join(PKG, "Makefile")]


def source_sha256():
    h = hashlib.sha256()
    for path in source_files():
        h.update(os.path.relpath(path, ROOT).encode() + b"\0")
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()
