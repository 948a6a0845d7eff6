#!/usr/bin/env python3
"""Static instruction mix per function of a gfx950 code object's disassembly (llvm-objdump -d):
VALU (v_*, split into dot / pk (VOP3P) / permlane-DPP), SALU (s_*), LDS (ds_*), vector memory
(global_ / buffer_ / flat_ / scratch_), MFMA, and branches.  Used for the search kernel's
per-class callees (tools/isa_count.sh builds the disassembly the way the Makefile builds the
kernel, occupancy pass included).

usage: isa_count.py DISASM.s [name-filter] [--ops]
  --ops: also the opcode histogram of each matching function's plain-VALU class ("valu": not a dot
  product, not VOP3P packed, not a cross-lane op)"""
import re
import sys

_DEMANGLE = re.compile(r"lane_unitILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E")


def short(name):
    m = _DEMANGLE.search(name)
    if m:
        return "lane_unit<%s,%s,%s,%s>" % m.groups()
    m = re.search(r"N_\d+(\w+?)E|3fme\d+(\w+?)E", name)
    return (m.group(1) or m.group(2)) if m else name[:60]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        if "dot" in op:
            return "v_dot"
        if op.startswith("v_pk_"):
            return "v_pk"
        if "permlane" in op or "_dpp" in op or op.startswith("v_readlane") or op.startswith("v_writelane"):
            return "v_xlane"
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


COLS = ["valu", "v_dot", "v_pk", "v_xlane", "mfma", "salu", "lds", "vmem", "scratch", "wait", "branch"]


def main():
    args = [a for a in sys.argv[1:] if a != "--ops"]
    ops_mode = "--ops" in sys.argv
    path = args[0]
    filt = args[1] if len(args) > 1 else ""
    funcs, cur = {}, None
    ops = {}
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            funcs[cur] = dict.fromkeys(COLS + ["other"], 0)
            ops[cur] = {}
            continue
        if cur is None:
            continue
        t = line.strip().split()
        if not t or t[0].endswith(":"):
            continue
        k = classify(t[0])
        funcs[cur][k] += 1
        if k == "valu":
            ops[cur][t[0]] = ops[cur].get(t[0], 0) + 1
    print("%-30s " % "function" + " ".join("%8s" % c for c in COLS) + " %8s" % "VALU all")
    for name, c in funcs.items():
        if filt and filt not in name:
            continue
        v = c["valu"] + c["v_dot"] + c["v_pk"] + c["v_xlane"]
        print("%-30s " % short(name) + " ".join("%8d" % c[k] for k in COLS) + " %8d" % v)
    if ops_mode:
        for name, h in ops.items():
            if filt and filt not in name:
                continue
            tot = sum(h.values())
            if not tot:
                continue
            print("\n%s: %d plain-VALU instructions by opcode" % (short(name), tot))
            for op, n in sorted(h.items(), key=lambda kv: -kv[1]):
                print("  %-28s %6d  %5.1f %%" % (op, n, 100.0 * n / tot))


if __name__ == "__main__":
    main()
