#!/usr/bin/env python3
"""Convert the reference's per-QP NN weight CSVs into the blob the C-ABI loads.

Source data: /root/reference/DL/blowing/<qp>/{1..14}.*.csv (fixtures shipped with the
reference; SURVEY.md §2 "Per-QP weights").  Output: hm16.9-nn_fme_amd/weights/nn2_qp<qp>.bin,
FME_NN_PARAMS (2060) little-endian float64 values, parsed as double exactly like the C++
comma initialisers in TEncSearch::init (TEncSearch.cpp:470-1073) before their float cast.

Order (include/fme.h, fme_load_nn_weights): embs0[8][4], embs1[8][4], in_h1[22][17],
h1_h2[20][22], h2_out[49][20], b1, BN_gamma_1, BN_beta_1, b2, BN_gamma_2, BN_beta_2, bout,
BN_gamma_in, mean, stdev.

With --check, every tensor is also compared (value-parsed) with the `name << ...;`
initialiser of the matching QP branch in TEncSearch.cpp (27: 472-623, 32: 625-773,
37: 775-923, default/22: 925-1073).  Run in the build container only (needs the reference).
"""
import argparse
import os
import re
import struct
import sys

REF = "/root/reference"
QPS = (22, 27, 32, 37)

# (blob name, csv stem, shape)
TENSORS = [
    ("embs0", "1.emb0-weight", (8, 4)),
    ("embs1", "2.emb1-weight", (8, 4)),
    ("in_h1", "3.lins0-weight", (22, 17)),
    ("h1_h2", "4.lins1-weight", (20, 22)),
    ("h2_out", "5.outp-weight", (49, 20)),
    ("b1", "6.lins0-bias", (22,)),
    ("BN_gamma_1", "10.bns0-weight", (22,)),
    ("BN_beta_1", "12.bns0-bias", (22,)),
    ("b2", "7.lins1-bias", (20,)),
    ("BN_gamma_2", "11.bns1-weight", (20,)),
    ("BN_beta_2", "13.bns1-bias", (20,)),
    ("bout", "8.outp-bias", (49,)),
    ("BN_gamma_in", "9.bn-weight", (9,)),
    ("mean", None, (9,)),
    ("stdev", None, (9,)),
]
NUM = re.compile(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?")


def numbers(text):
    return [float(t) for t in NUM.findall(text)]


def csv_tensors(qp):
    d = os.path.join(REF, "DL", "blowing", str(qp))
    out = {}
    for name, stem, shape in TENSORS:
        if stem is None:
            continue
        vals = numbers(open(os.path.join(d, stem + ".csv")).read())
        n = 1
        for s in shape:
            n *= s
        if len(vals) != n:
            raise SystemExit(f"qp{qp} {stem}: {len(vals)} values, expected {n}")
        out[name] = vals
    mapper = [l for l in open(os.path.join(d, f"14.mapper_{qp}.csv")).read().splitlines() if l.strip()]
    out["mean"] = numbers(mapper[0])
    out["stdev"] = numbers(mapper[1])
    for k in ("mean", "stdev"):
        if len(out[k]) != 9:
            raise SystemExit(f"qp{qp} mapper {k}: {len(out[k])} values")
    return out


def source_tensors(qp):
    """Parse the `name << v, v, ...;` initialisers of one QP branch of TEncSearch::init."""
    src = open(os.path.join(REF, "source/Lib/TLibEncoder/TEncSearch.cpp"), encoding="latin-1").read().split("\n")
    ranges = {27: (472, 623), 32: (625, 773), 37: (775, 923), 22: (925, 1073)}
    a, b = ranges[qp]
    body = "\n".join(src[a - 1:b])
    out = {}
    for m in re.finditer(r"\b(\w+)\s*<<([^;]*);", body):
        out[m.group(1)] = numbers(m.group(2))
    return out


def write_blob(qp, tensors, outdir):
    flat = []
    for name, _, _ in TENSORS:
        flat.extend(tensors[name])
    assert len(flat) == 2060, len(flat)
    path = os.path.join(outdir, f"nn2_qp{qp}.bin")
    with open(path, "wb") as f:
        f.write(struct.pack("<2060d", *flat))
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "hm16.9-nn_fme_amd", "weights"))
    ap.add_argument("--check", action="store_true", help="compare with the TEncSearch.cpp initialisers")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    for qp in QPS:
        t = csv_tensors(qp)
        if args.check:
            s = source_tensors(qp)
            for name, _, _ in TENSORS:
                if s.get(name) != t[name]:
                    raise SystemExit(f"qp{qp} {name}: CSV differs from TEncSearch.cpp initialiser")
        print(write_blob(qp, t, args.out), "checked" if args.check else "")
    return 0


if __name__ == "__main__":
    sys.exit(main())
