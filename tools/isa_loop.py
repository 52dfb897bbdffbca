#!/usr/bin/env python3
"""Compact listing of a kernel's K loop from the gfx950 assembly: the basic block
with the most MFMAs that also issues LDS-DMA, as a one-line sequence —
M<n> (n MFMAs), R / W (ds_read / ds_write), DMA (global_load_lds), LD (other
global loads), v (VALU), [waitcnt], BARRIER.  Shows where the compiler put its
waits and how the DMA pieces and LDS reads interleave with the MFMAs.

    python tools/isa_loop.py "conv_x3_a3_kernel<3>" [--src csrc/conv_x3.hip]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mangled(name):
    """conv_x3_a3_kernel<3> -> _ZN3hkp17conv_x3_a3_kernelILi3EEEvNS_6X3ArgsE (int args only)."""
    m = re.match(r"(\w+)<([\d,\s]*)>", name)
    base, args = m.group(1), [a.strip() for a in m.group(2).split(",") if a.strip()]
    return "_ZN3hkp%d%sI%sEEvNS_6X3ArgsE" % (len(base), base, "".join("Li%sE" % a for a in args))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--src", default=os.path.join(REPO, "hulk-keypoints_amd", "csrc", "conv_x3.hip"))
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-ffp-contract=off", "-Wno-unused-function", "-Wno-unused-variable",
                        "-I" + os.path.join(REPO, "include"), "-S", "--offload-device-only", "-c", args.src,
                        "-o", out], check=True)
        s = open(out).read()
    sym = mangled(args.kernel)
    i = s.find("\n" + sym + ":")
    if i < 0:
        sys.exit("no kernel %s (%s)" % (args.kernel, sym))
    body = s[i:s.index(".Lfunc_end", i)].split("\n")
    lab = [k for k, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)]
    blocks = [(a, b) for a, b in zip(lab, lab[1:] + [len(body)])]
    blocks.sort(key=lambda ab: (any("global_load_lds" in l for l in body[ab[0]:ab[1]]),
                                sum("mfma" in l for l in body[ab[0]:ab[1]])), reverse=True)
    a, b = blocks[0]
    out, run = [], 0
    for line in body[a + 1:b]:
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if "mfma" in op:
            run += 1
            continue
        if run:
            out.append("M%d" % run)
            run = 0
        if op.startswith("ds_read"):
            out.append("R")
        elif op.startswith("ds_write"):
            out.append("W")
        elif op.startswith("s_waitcnt"):
            out.append("[" + t[10:] + "]")
        elif op.startswith("s_barrier"):
            out.append("BARRIER")
        elif op.startswith("global_load_lds"):
            out.append("DMA")
        elif op.startswith("global_load"):
            out.append("LD")
        elif op.startswith("v_"):
            out.append("v")
    if run:
        out.append("M%d" % run)
    comp, prev, cnt = [], None, 0
    for o in out + [None]:
        if o == prev:
            cnt += 1
            continue
        if prev is not None:
            comp.append(prev + ("x%d" % cnt if cnt > 1 else ""))
        prev, cnt = o, 1
    print(" ".join(comp))


if __name__ == "__main__":
    main()
