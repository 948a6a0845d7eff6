#!/usr/bin/env python3
"""Build step of fme_lane.o: give the search kernel's non-inlined callees the kernel's occupancy.

k_search_lane calls one noinline function per PU class (lane_unit<PW, PH, UW, UH>, fme_lane.hip).
clang accepts amdgpu_waves_per_eu only on kernels and this compiler does not propagate it to
callees, so each callee is register-allocated for one wave per SIMD (256 VGPRs + AGPR spill
space) and the kernel's descriptor then asks for ~290 registers: one wave per SIMD for the whole
launch.  This pass copies the largest "amdgpu-waves-per-eu" of the module's kernels onto the
attribute groups of every non-kernel function defined in the module (LLVM reads the attribute
on any function when it sizes the register budget), before llc generates the code object.

usage: callee_occupancy.py module.ll   (rewritten in place; prints what it changed)
"""
import re
import sys


def main(path):
    text = open(path).read()
    defs = re.findall(r"^define\s+([^@\n]*)@([\w.$]+)\(.*?\)\s*([^{\n]*)\{", text, re.M)
    group_of = {}
    kernels, callees = [], []
    for prefix, name, suffix in defs:
        m = re.search(r"#(\d+)", suffix)
        if not m:
            continue
        group_of[name] = m.group(1)
        (kernels if "amdgpu_kernel" in prefix else callees).append(name)
    groups = dict(re.findall(r"^attributes #(\d+) = \{(.*)\}$", text, re.M))
    waves = []
    for k in kernels:
        m = re.search(r'"amdgpu-waves-per-eu"="(\d+)', groups[group_of[k]])
        if m:
            waves.append(int(m.group(1)))
    if not waves:
        print("callee_occupancy: no kernel asks for an occupancy; module unchanged")
        return
    w = max(waves)
    kernel_groups = {group_of[k] for k in kernels}
    todo = sorted({group_of[c] for c in callees}, key=int)
    for g in todo:
        if g in kernel_groups:
            raise SystemExit(f"callee_occupancy: attribute group #{g} is shared by a kernel and a callee")
        if '"amdgpu-waves-per-eu"' in groups[g]:
            continue
        text = re.sub(rf"^attributes #{g} = \{{", f'attributes #{g} = {{ "amdgpu-waves-per-eu"="{w},{w}"',
                      text, count=1, flags=re.M)
    open(path, "w").write(text)
    print(f"callee_occupancy: {len(callees)} callees in groups {todo} -> waves-per-eu {w}")


if __name__ == "__main__":
    main(sys.argv[1])
