import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
REFERENCE_PKL = Path(os.environ.get("COBALT_REFERENCE_PKL", "/root/reference/src/api/models/xgb_model_tree.pkl"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the native HIP library")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    # device_count() does not initialise HIP (is_available() does), so multi-process GPU tests can
    # still spawn their ranks from an uninitialised parent.
    if torch.cuda.device_count() > 0:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def reference_model_bytes():
    """The shipped reference checkpoint, or the in-repo copy made by tests/fixtures (read as bytes only)."""
    for p in (REFERENCE_PKL, ROOT / "tests" / "fixtures" / "xgb_model_tree.pkl"):
        if p.exists():
            return p.read_bytes()
    pytest.skip("reference checkpoint not available")


@pytest.fixture(scope="session")
def reference_booster(reference_model_bytes):
    from cobalt_smart_lender_ai_amd.models.booster import load_pickle_bytes

    return load_pickle_bytes(reference_model_bytes)[1]
