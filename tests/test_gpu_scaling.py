"""configs[4] on the GPU against the reference's finite-length scaling law (see
tests/test_scaling_law.py for the law, its constants and the band): the expurgated (3,6)
n = 64,800 ensemble at eps = 0.425, 200 iterations, X = 3, run to the reference's 200-frame-error
stop rule (parallel_simulator.py:198; expurgation parallel_simulator_expurgated.py:238) on fresh
device-sampled graphs."""
import json
import math
import os

import pytest

from iib_project_ldpc_codes_amd import de

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL_TOL = 0.30


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def test_cfg5_waterfall_point_on_scaling_law(torch):
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "de_golden.json")))
    eps = 0.425
    mc = MonteCarlo.ensemble(64800, 3, 6, "bec", eps, 200, seed=404, batch=4096, expurgation=3)
    r = mc.run(0, stop_frame_errors=200)
    assert r["frame_errors"] == 200
    fer = r["frame_errors"] / r["num_tests"]
    law = float(de.scaling_fer(64800, eps, gold["calc_threshold_3_6"], gold["alpha_3_6"], gold["beta_shift_3_6"]))
    sig = math.sqrt((1 - fer) / 200)
    print(f"eps={eps} trials={r['num_tests']} fer={fer:.4g} law={law:.4g} ratio={fer / law:.3f}")
    assert abs(math.log(fer / law)) <= math.log(1 + MODEL_TOL) + 3 * sig, (fer, law)
