"""Producer probe: fme_pred_inter_p / fme_pred_inter_b over one 1080p frame, wall time per call
(run under rocprofv3 --kernel-trace --stats for the per-kernel split)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hm16.9-nn_fme_amd"), ROOT]
import numpy as np  # noqa: E402

from nnfme import synth, weights  # noqa: E402
from nnfme.runtime import FmeContext  # noqa: E402

W, H = int(os.environ.get("PI_W", 1920)), int(os.environ.get("PI_H", 1080))
mode = sys.argv[1] if len(sys.argv) > 1 else "p"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rng = np.random.default_rng(2)
pics = {i: synth.synth_luma(W, H, t) for i, t in zip(range(6), (7, 6, 5, 4, 0, 3))}
ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1)
for k, v in pics.items():
    ctx.set_picture(k, v)
for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
    ctx.set_lambda(lid, lam)
if mode == "p":
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=3)
    run = ctx.pred_inter_p
else:
    reqs = synth.make_pu_requests_b(rng, W, H, org_id=4, l0=[(0, 1), (1, 2)], l1=[(5, -1), (2, -2)], lambda_id=0,
                                    max_depth=3)
    run = ctx.pred_inter_b
run(reqs[:2000])
for r in range(reps):
    ctx.pred_inter_reset()
    t0 = time.perf_counter()
    out = run(reqs)
    print(f"{mode} {len(reqs)} requests: {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
if mode == "b":
    print("inter_dir", np.bincount(out["inter_dir"]).tolist())
