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


# ---- the reference's weight files ------------------------------------
# DL/<name>/<qp>/*.csv as NN_training.ipynb's export_parameters / export_mapper write them and
# DL/edit.sh renumbers and indents them for pasting into TEncSearch::init: one line per matrix
# row, "\t\t\t" indent, "," separated, ";" after the last value; mapper_<qp>.csv holds the mean
# and std rows of the nine distortions.
CSV_FILES = [
    ("embs0", "1.emb0-weight"), ("embs1", "2.emb1-weight"), ("in_h1", "3.lins0-weight"),
    ("h1_h2", "4.lins1-weight"), ("h2_out", "5.outp-weight"), ("b1", "6.lins0-bias"),
    ("b2", "7.lins1-bias"), ("bout", "8.outp-bias"), ("BN_gamma_in", "9.bn-weight"),
    ("BN_gamma_1", "10.bns0-weight"), ("BN_gamma_2", "11.bns1-weight"),
    ("BN_beta_1", "12.bns0-bias"), ("BN_beta_2", "13.bns1-bias"),
]
# fastai v0.7 MixedInputModel state_dict keys (DL/models/QP<qp>_*.h5 are torch.save'd dicts)
STATE_DICT_KEYS = {
    "embs0": "embs.0.weight", "embs1": "embs.1.weight", "in_h1": "lins.0.weight",
    "h1_h2": "lins.1.weight", "h2_out": "outp.weight", "b1": "lins.0.bias", "b2": "lins.1.bias",
    "bout": "outp.bias", "BN_gamma_1": "bns.0.weight", "BN_beta_1": "bns.0.bias",
    "BN_gamma_2": "bns.1.weight", "BN_beta_2": "bns.1.bias", "BN_gamma_in": "bn.weight",
}
_NUM = None


def _numbers(text):
    global _NUM
    if _NUM is None:
        import re
        _NUM = re.compile(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?")
    return [float(t) for t in _NUM.findall(text)]


def pack(tensors):
    """{name: array} in LAYOUT -> float32[2060] (the fme_load_nn_weights order)."""
    flat = []
    for name, shape in LAYOUT:
        a = np.asarray(tensors[name], dtype=np.float64)
        if a.size != int(np.prod(shape)):
            raise ValueError(f"{name}: {a.size} values, expected {int(np.prod(shape))}")
        flat.append(a.reshape(-1))
    return np.concatenate(flat).astype(np.float32)


def load_csv_dir(path, qp):
    """A DL/<name>/<qp>/ directory (edit.sh layout) -> float32[2060].  The values are parsed as
    double and cast to float, as TEncSearch::init's comma initialisers do."""
    t = {}
    for name, stem in CSV_FILES:
        with open(os.path.join(path, stem + ".csv")) as f:
            t[name] = _numbers(f.read())
    with open(os.path.join(path, f"14.mapper_{qp}.csv")) as f:
        rows = [l for l in f.read().splitlines() if l.strip()]
    if len(rows) != 2:
        raise ValueError(f"{path}: mapper_{qp}.csv has {len(rows)} rows, expected mean and std")
    t["mean"], t["stdev"] = _numbers(rows[0]), _numbers(rows[1])
    return pack(t)


def _fmt(v):
    return np.format_float_positional(np.float32(v), unique=True, trim="-")


def write_csv_dir(path, params, qp):
    """float32[2060] -> a DL/<name>/<qp>/ directory in edit.sh's layout (load_csv_dir reads it
    back bit-exactly: every value is the shortest decimal that round-trips its float32)."""
    os.makedirs(path, exist_ok=True)
    t = unpack(np.asarray(params, np.float32))
    for name, stem in CSV_FILES:
        a = np.atleast_2d(t[name])
        sep = ", " if a.shape[0] == 1 else ","
        rows = ["\t\t\t" + sep.join(_fmt(v) for v in row) for row in a]
        with open(os.path.join(path, stem + ".csv"), "w") as f:
            f.write((sep + "\n").join(rows) + ";\n")
    with open(os.path.join(path, f"14.mapper_{qp}.csv"), "w") as f:
        for row in (t["mean"], t["stdev"]):
            f.write(",".join(repr(float(v)) for v in np.asarray(row, np.float64)) + ";\n")


def from_state_dict(sd, mean, stdev):
    """fastai v0.7 MixedInputModel state_dict (+ the mapper's mean / std) -> float32[2060].
    NN_pred() uses the BatchNorm weights and biases only (TEncSearch.cpp:139-186): running
    statistics and the input BatchNorm's bias are not read."""
    t = {name: np.asarray(sd[key].detach().cpu().numpy() if hasattr(sd[key], "detach") else sd[key])
         for name, key in STATE_DICT_KEYS.items()}
    t["mean"], t["stdev"] = mean, stdev
    return pack(t)


def to_state_dict(params):
    """float32[2060] -> {state_dict key: torch tensor} (the inverse of from_state_dict)."""
    import torch
    t = unpack(np.asarray(params, np.float32))
    return {key: torch.from_numpy(np.ascontiguousarray(t[name])) for name, key in STATE_DICT_KEYS.items()}


def load_checkpoint(path, mean, stdev):
    """DL/models/QP<qp>_*.h5 (a torch.save'd state_dict despite the suffix) -> float32[2060].
    Loaded with torch.load(weights_only=True): nothing in the file is executed."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return from_state_dict(sd, mean, stdev)


# ---- generic (deeper) NN_pred nets: fme_load_nn_net, BASELINE.json configs[4] ---------------------
# Blobs written by tools/convert_deep_weights.py from the reference's in-tree backups:
#   nn3x40_scr.nnd   Backups/4 "SCR 3 layers" (9 -> 3 x 40 -> 49, double, sigmoid output)
#   nn4x40_qp22.nnd  Backups/15 "blowing 4 lyrs qp 22" (17 -> 4 x 40 -> 49, float, X3/X4 carried)
F32, F64 = 0, 1
EMB_NONE, EMB_MASTER, EMB_SWAP = 0, 1, 2
OUT_LINEAR, OUT_SIGMOID = 0, 1
SLOT_RESET = 1   # FME_NN_IN_SLOT_RESET
TZ_RING = 2      # FME_NN_IN_TZ_RING: the backups' own input path (FME_JOB_NN_IN rows)
NET_FILES = {"scr3x40": "nn3x40_scr.nnd", "blowing4x40": "nn4x40_qp22.nnd"}


class NnNet:
    """A generic net: the fme_nn_net descriptor fields plus float64 parameters in
    fme_load_nn_net order (include/fme.h)."""

    def __init__(self, precision, widths, embedding, out_act, carry_hidden, params, input_flags=0):
        self.precision = int(precision)
        self.widths = [int(w) for w in widths]
        self.embedding = int(embedding)
        self.out_act = int(out_act)
        self.carry_hidden = int(carry_hidden)
        self.input_flags = int(input_flags)
        self.params = np.ascontiguousarray(params, dtype=np.float64)
        if self.params.size != param_count(self):
            raise ValueError(f"{self.params.size} parameters, descriptor needs {param_count(self)}")

    @property
    def n_hidden(self):
        return len(self.widths)

    def desc_struct(self):
        from .abi import NnNetStruct
        w = (self.widths + [0] * 4)[:4]
        return NnNetStruct(self.precision, self.n_hidden, (C_INT4)(*w), self.embedding, self.out_act,
                           self.carry_hidden, self.input_flags)

    def with_carry(self, carry_hidden):
        return NnNet(self.precision, self.widths, self.embedding, self.out_act, carry_hidden, self.params,
                     self.input_flags)

    def with_input_flags(self, input_flags):
        """FME_NN_IN_SLOT_RESET (1): array_e slots a call did not push read 0, as after the
        backups' per-call memset (Backups/4:4421-4422, Backups/15:4961-4962)."""
        return NnNet(self.precision, self.widths, self.embedding, self.out_act, self.carry_hidden, self.params,
                     input_flags)

    def __repr__(self):
        return (f"NnNet({'f64' if self.precision else 'f32'}, {self.widths}, emb={self.embedding}, "
                f"out_act={self.out_act}, carry=0b{self.carry_hidden:b}, in=0x{self.input_flags:x})")


def _c_int4():
    import ctypes
    return ctypes.c_int32 * 4


C_INT4 = _c_int4()


def param_count(net):
    n = 64 if net.embedding else 0
    fan = 17 if net.embedding else 9
    for w in net.widths:
        n += w * fan + 3 * w
        fan = w
    return n + 49 * fan + 49 + 27


def load_net(name_or_path):
    """Read an .nnd blob (tools/convert_deep_weights.py)."""
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(WEIGHTS_DIR, NET_FILES.get(name_or_path, name_or_path))
    raw = open(path, "rb").read()
    if raw[:8] != b"FMENND01":
        raise ValueError(f"{path}: not an FMENND01 blob")
    hdr = np.frombuffer(raw, dtype="<i4", count=12, offset=8)
    prec, nh = int(hdr[0]), int(hdr[1])
    widths = [int(v) for v in hdr[2:2 + nh]]
    emb, out_act, carry, count = int(hdr[6]), int(hdr[7]), int(hdr[8]) & 0xFFFFFFFF, int(hdr[10])
    params = np.frombuffer(raw, dtype="<f8", count=count, offset=56)
    return NnNet(prec, widths, emb, out_act, carry, params)


def master_net(qp=22):
    """The shipped 2-layer master net (nn2_qp<QP>) in the generic layout: the generic path must
    reproduce nn_mode 1 bit for bit with it."""
    blob = np.fromfile(os.path.join(WEIGHTS_DIR, f"nn2_qp{weight_set_for_qp(qp)}.bin"), dtype="<f8")
    t = {}
    o = 0
    for name, shape in LAYOUT:
        n = int(np.prod(shape))
        t[name] = blob[o:o + n]
        o += n
    params = np.concatenate([
        t["embs0"], t["embs1"],
        t["in_h1"], t["b1"], t["BN_gamma_1"], t["BN_beta_1"],
        t["h1_h2"], t["b2"], t["BN_gamma_2"], t["BN_beta_2"],
        t["h2_out"], t["bout"], t["BN_gamma_in"], t["mean"], t["stdev"]])
    return NnNet(F32, [22, 20], EMB_MASTER, OUT_LINEAR, 0, params)


def case_net(name):
    """Nets named by fixtures and bench workloads: an .nnd blob (NET_FILES key), "<name>+rezero" =
    that net with carry_hidden cleared, "+slotreset" / "+tzring" = with FME_NN_IN_SLOT_RESET /
    FME_NN_IN_TZ_RING, "master" = the shipped QP22 2-layer net, generic layout."""
    if name == "master":
        return master_net(22)
    base, *mods = str(name).split("+")
    net = load_net(base)
    for mod in mods:
        if mod == "rezero":
            net = net.with_carry(0)
        elif mod == "slotreset":
            net = net.with_input_flags(SLOT_RESET)
        elif mod == "tzring":
            net = net.with_input_flags(TZ_RING)
        else:
            raise ValueError(f"unknown net modifier {mod!r} in {name!r}")
    return net
