import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: full-size config run (seconds to minutes)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def oracle():
    from pyoracle import Oracle
    return Oracle("port")


@pytest.fixture(scope="session")
def ref_oracle():
    from pyoracle import Oracle, ref_available
    if not ref_available():
        pytest.skip("oracle/_ref/libfpnn_ref.so not built (needs /root/reference)")
    return Oracle("reference")


@pytest.fixture(scope="session")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    import fpnn_amd
    eng = fpnn_amd.Engine(0)
    yield eng
    eng.sync()
    eng.close()


@pytest.fixture(scope="session")
def queue_engine():
    """An engine that always uses the K2q work-queue encrypt for ragged batches
    (by default it only does so when chains outnumber the chip's lane quads)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    import fpnn_amd
    old = os.environ.get("FPNN_AES_QUEUE")
    os.environ["FPNN_AES_QUEUE"] = "2"
    try:
        eng = fpnn_amd.Engine(0)
    finally:
        if old is None:
            del os.environ["FPNN_AES_QUEUE"]
        else:
            os.environ["FPNN_AES_QUEUE"] = old
    yield eng
    eng.sync()
    eng.close()


@pytest.fixture(params=["lane", "wave"])
def scan_mode(request):
    """Run a receive test through both device frame walks (framing.hip: one lane per
    segment, or one wavefront per segment with length-guessing header reads); by default
    the engine picks by segment count."""
    old = os.environ.get("FPNN_AES_SCAN")
    os.environ["FPNN_AES_SCAN"] = request.param
    yield request.param
    if old is None:
        del os.environ["FPNN_AES_SCAN"]
    else:
        os.environ["FPNN_AES_SCAN"] = old
