"""GPU convergence parity (W = 1, native HIP codecs) on the reference's MNIST fixture: the same
pipelines and margins as tests/test_convergence.py (W = 2 gloo on CPU)."""
import os
import sys

import pytest

from grace_amd.ops import _native
from grace_amd.utils.mnist import find_fixture, train_eval

sys.path.insert(0, os.path.dirname(__file__))
from test_convergence import EPOCHS, MARGIN, PIPELINES  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(find_fixture() is None, reason="MNIST t10k fixture missing")
def test_gpu_compressed_training_converges_like_uncompressed():
    assert _native.available()
    res = {name: train_eval(p, epochs=EPOCHS, device="cuda") for name, p in PIPELINES.items()}
    print(res)
    base = res["none"]["accuracy"]
    assert base > 0.9, res["none"]
    for name, m in MARGIN.items():
        assert res[name]["accuracy"] >= base - m, (name, res[name], base)
    assert res["randomk"]["accuracy"] > 0.5
