"""Summarise the envab runs: PCIe-inclusive / resident rate and the host stalls of each log."""
import glob
import json
import sys

for f in sorted(glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out") + "/*.log")):
    line = None
    for ln in open(f, errors="replace"):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    if not line:
        continue
    p = line.get("pcie_inclusive") or {}
    slow = p.get("slow_host_calls", [])
    print(f"{f.split('/')[-1]:40s} value {line['value'] / 1e6:7.1f} M  {line['ms_per_step']:.3f} ms/step  "
          f"resident {line['resident']['value'] / 1e6:7.1f} M  stalls {len(slow)}: "
          + ", ".join(f"{c[0].split()[-1]}:{c[2]:.1f}" for c in slow[:8]))
