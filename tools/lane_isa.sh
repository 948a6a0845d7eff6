#!/bin/bash
# Disassembly of the search kernel's code object built the way the Makefile builds it (device
# bitcode -> callee occupancy pass -> llc), for tools/isa_count.py.  usage: tools/lane_isa.sh OUT.s [DEFS]
set -e
out=${1:-/tmp/lane.s}; defs=${2:-}
LLVM=/opt/rocm/lib/llvm/bin
d=$(mktemp -d)
cd "$(dirname "$0")/../hm16.9-nn_fme_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $defs --cuda-device-only -emit-llvm -c csrc/fme_lane.hip -o $d/l.bc
$LLVM/llvm-dis $d/l.bc -o $d/l.ll
python3 csrc/callee_occupancy.py $d/l.ll > /dev/null
$LLVM/llc -O3 -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -filetype=obj $d/l.ll -o $d/l.o
$LLVM/llvm-objdump -d --mcpu=gfx950 $d/l.o > "$out"
rm -rf $d
