import os

import numpy as np
import pytest

from nnfme import weights

REF = "/root/reference/DL/blowing"


@pytest.mark.parametrize("qp", [22, 27, 32, 37])
def test_weight_blob_shapes(qp):
    p = weights.load_weights(qp)
    assert p.dtype == np.float32 and p.size == 2060
    t = weights.unpack(p)
    assert t["in_h1"].shape == (22, 17) and t["h2_out"].shape == (49, 20)
    assert np.all(t["stdev"] > 0)


def test_weight_set_selection_follows_tencsearch_init():
    # TEncSearch.cpp:472/625/775/925: 27, 32, 37, anything else -> 22
    assert [weights.weight_set_for_qp(q) for q in (22, 27, 32, 37, 30, 0)] == [22, 27, 32, 37, 22, 22]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference CSVs not present")
@pytest.mark.parametrize("qp", [22, 27, 32, 37])
def test_weight_blob_equals_reference_csv(qp):
    import re
    num = re.compile(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?")
    t = weights.unpack(np.fromfile(os.path.join(weights.WEIGHTS_DIR, f"nn2_qp{qp}.bin"), "<f8"))
    csv = np.array([float(v) for v in num.findall(open(f"{REF}/{qp}/3.lins0-weight.csv").read())])
    np.testing.assert_array_equal(t["in_h1"].reshape(-1), csv)
