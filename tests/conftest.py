import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "alphazero-gomoku_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _study_tuning():
    """AZG_TEST_TUNE="KEY=VALUE,..." runs the suite under non-default tuning keys (studies
    that test a variant, e.g. scripts/gpu_r6j.sh's split-fp16 dgrad, key 50 = 2); unset in
    every product run."""
    spec = os.environ.get("AZG_TEST_TUNE", "")
    if spec:
        import _native
        lib = _native.load_library()
        for kv in spec.split(","):
            k, v = (int(t) for t in kv.split("="))
            lib.azg_pv_set_tuning(k, v)
    yield


def load_golden(tag: str) -> dict:
    with np.load(os.path.join(GOLDEN, f"net_{tag}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_state(g: dict) -> dict:
    """fp16-stored fixture weights widened to the dtypes of a state_dict (exact)."""
    out = {}
    for k, v in g.items():
        if k.startswith("w/"):
            out[k[2:]] = v.astype(np.float32) if v.dtype == np.float16 else v
    return out


@pytest.fixture(scope="session")
def golden_3x64():
    return load_golden("3x64")


@pytest.fixture(scope="session")
def golden_6x128():
    return load_golden("6x128")


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
