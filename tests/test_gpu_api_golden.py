"""The REST golden values (BASELINE.md / SURVEY.md §4: prob 0.0941799, SHAP, base value, bulk CSV with
nulls) through the MI355X serving path: ScoringEngine on ``cuda`` with hipGraph buckets behind the
micro-batcher (reference: src/api/cobalt_fast_api.py:96-126). ``tests/test_api.py`` runs the same
assertions wherever it runs; this file pins them on the GPU engine explicitly."""
import pytest
import torch
from fastapi.testclient import TestClient

import test_api
from cobalt_smart_lender_ai_amd.config import ServeConfig
from cobalt_smart_lender_ai_amd.serve.app import create_app

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu_client(reference_booster):
    app = create_app(ServeConfig(device="cuda", use_graphs=True), booster=reference_booster)
    with TestClient(app) as c:
        eng = app.state.cobalt["engine"]
        assert eng.device.type == "cuda" and eng.use_graphs
        yield c


def test_gpu_predict_golden(gpu_client):
    test_api.test_predict_golden(gpu_client)


def test_gpu_bulk_csv_and_nulls(gpu_client):
    test_api.test_bulk_csv_and_nulls(gpu_client)


def test_gpu_feature_importance(gpu_client):
    test_api.test_feature_importance(gpu_client)


def test_gpu_engine_loaded_native_library():
    from cobalt_smart_lender_ai_amd import _native

    assert torch.cuda.is_available()
    assert _native.loaded_path().endswith("libcobalt_hip.so")
