"""Per-QP NN_pred weight sets (converted from the reference CSVs by tools/convert_weights.py).

TEncSearch::init selects the set from the base QP: 27, 32, 37, anything else -> 22
(TEncSearch.cpp:472, 625, 775, 925).  The blob holds float64 values; the C++ initialisers
assign double literals to float Eigen arrays, so the float32 cast here is the same rounding.
"""
import os

import numpy as np

from .abi import NN_PARAMS

WEIGHTS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "weights")

# (name, shape) in blob order — include/fme.h fme_load_nn_weights().
LAYOUT = [
    ("embs0", (8, 4)), ("embs1", (8, 4)), ("in_h1", (22, 17)), ("h1_h2", (20, 22)),
    ("h2_out", (49, 20)), ("b1", (22,)), ("BN_gamma_1", (22,)), ("BN_beta_1", (22,)),
    ("b2", (20,)), ("BN_gamma_2", (20,)), ("BN_beta_2", (20,)), ("bout", (49,)),
    ("BN_gamma_in", (9,)), ("mean", (9,)), ("stdev", (9,)),
]


def weight_set_for_qp(qp):
    return qp if qp in (27, 32, 37) else 22


def load_weights(qp):
    """float32[2060] for the weight set TEncSearch::init would pick for base QP `qp`."""
    path = os.path.join(WEIGHTS_DIR, f"nn2_qp{weight_set_for_qp(qp)}.bin")
    blob = np.fromfile(path, dtype="<f8")
    if blob.size != NN_PARAMS:
        raise ValueError(f"{path}: {blob.size} parameters, expected {NN_PARAMS}")
    return blob.astype(np.float32)


def unpack(params):
    out, o = {}, 0
    for name, shape in LAYOUT:
        n = int(np.prod(shape))
        out[name] = np.asarray(params[o:o + n]).reshape(shape)
        o += n
    return out
