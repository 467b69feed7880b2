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


def missing_reference_build(what):
    """A reference checker under oracle/_ref/ is absent.  Where a GPU is present (the GPU
    box, which gets the tree with the checkers built here) that is an error: the parity
    evidence must not vanish as a skip.  On a CPU-only machine without /root/reference it
    is a skip."""
    import torch
    if torch.cuda.is_available():
        pytest.fail(f"{what} missing on a GPU machine: build it with __graft_entry__.build() "
                    "(make -C oracle ref framing echo percall ecdh dropin) before the GPU run")
    pytest.skip(f"{what} not built (needs /root/reference)")


@pytest.fixture(scope="session")
def ref_oracle():
    from pyoracle import Oracle, ref_available
    if not ref_available():
        missing_reference_build("oracle/_ref/libfpnn_ref.so")
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


def _env_engine(env):
    """An engine created under extra FPNN_AES_* settings (read once, at creation)."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    import fpnn_amd
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fpnn_amd.Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


# K2h (k_hybrid.hip) on every ragged batch, with the long-chain threshold and the number
# of waves that start on quads set so that small test batches exercise each session:
#   hybrid_engine       chains of >= 64 blocks on quads, 3 quad waves per workgroup
#   hybrid_lane_engine  every chain one lane (no quad queue)
#   hybrid_quad_engine  every chain on quads, no quad waves at start (lane waves join)
# (wire-prefix batches run on quads alone in every setting, as in the product)
HYBRID_ENGINES = {
    "hybrid_engine": {"FPNN_AES_HYB_LONG": "64", "FPNN_AES_HYB_QW": "3"},
    "hybrid_lane_engine": {"FPNN_AES_HYB_LONG": "1000000000", "FPNN_AES_HYB_QW": "2"},
    "hybrid_quad_engine": {"FPNN_AES_HYB_LONG": "1", "FPNN_AES_HYB_QW": "0"},
}


def _hybrid(name):
    env = {"FPNN_AES_HYB_FORCE": "1"}
    env.update(HYBRID_ENGINES[name])
    return _env_engine(env)


@pytest.fixture(scope="session")
def hybrid_engine():
    eng = _hybrid("hybrid_engine")
    yield eng
    eng.sync()
    eng.close()


@pytest.fixture(scope="session")
def hybrid_lane_engine():
    eng = _hybrid("hybrid_lane_engine")
    yield eng
    eng.sync()
    eng.close()


@pytest.fixture(scope="session")
def hybrid_quad_engine():
    eng = _hybrid("hybrid_quad_engine")
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
