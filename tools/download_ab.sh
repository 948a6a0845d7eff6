#!/bin/bash
# A/B of the replay's results-download placement (bench.py --download) on the 1080p and 416x240 workloads.
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-pi --no-tz --no-mc"
summ() { python -c "
import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1], round(d['value']/1e6,1), round(d['ms_per_step'],4))" $1; }
for w in c1 c2 c3_qp22 c4; do for m in deferred immediate deferred immediate; do
  timeout -k 10 200 $B --workload $w --download $m > gpurun_out/dl_${w}_$m.log 2>&1 && summ gpurun_out/dl_${w}_$m.log || exit 1
done; done
