import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "hm16.9-nn_fme_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfme_amd.so)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def golden_cases():
    """Sub-pel refinement fixtures (fme_job -> fme_result)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN)
                  if f.endswith(".npz") and not f.startswith(("mc_", "mc10_", "mcwp", "tz_", "tz10_", "ring_", "main10_")))


def main10_golden_cases():
    """Sub-pel refinement fixtures at bit depth 10 (the main10 configurations)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("main10_"))


def ring_golden_cases():
    """The backups' NN input path (configs[4]): integer search with the final square + ring
    (fme_job + fme_tz_ext -> MV, ruiSAD, nine NN inputs), then FME_JOB_NN_IN refinements."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("ring_"))


def tz_golden_cases():
    """Integer motion-estimation fixtures (fme_job + fme_tz_ext -> integer MV, ruiSAD)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith(("tz_", "tz10_")))


def golden_bit_depth(g):
    """The fixture's luma bit depth (10 for the main10 fixtures, else 8)."""
    return int(g["bit_depth"][0]) if "bit_depth" in g else 8


def mc_golden_cases():
    """Motion-compensation fixtures (fme_mc_job + reference YUV -> predicted planes)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("mc_"))


def mc10_golden_cases():
    """Motion-compensation fixtures at bit depth 10 (uint16 planes, from oracle/_ref at bitDepth 10)."""
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f.startswith("mc10_"))


def mc_inputs(g):
    """(pictures {id: (Y, Cb, Cr)}, jobs, fresh output planes filled like the fixture's)."""
    import numpy as np
    pics = {k: (g["ref_y"][k], g["ref_cb"][k], g["ref_cr"][k]) for k in range(len(g["ref_y"]))}
    fill = int(g["fill"][0])
    h, w = g["pred_y"].shape
    dt = g["pred_y"].dtype   # uint8, or uint16 at bit depth 10 (mc10_*)
    planes = (np.full((h, w), fill, dt), np.full((h // 2, w // 2), fill, dt), np.full((h // 2, w // 2), fill, dt))
    return pics, g["jobs"], planes


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
