"""The reference's OWN Streamlit UI, unmodified, against this framework's API.

``/root/reference/src/streamlit_ui/cobalt_streamlit.py`` is executed as shipped (read from the
reference checkout, as tests/conftest.py reads the reference pkl; skipped when absent). Its
hard-coded ``API_URL = "http://cobalt-lender-api:8000"`` is served by routing ``requests.post`` for
that host to FastAPI's TestClient over ``serve.app.create_app`` (the reference model loaded by the
static decoder). ``streamlit`` and ``shap`` are not installed here, so recording stand-ins replace
them: the UI's widget calls return their defaults, and ``shap.Explanation`` /
``shap.plots.waterfall`` record what the UI hands them (reference:
src/streamlit_ui/cobalt_streamlit.py:10,85,102-110,140,159). Both tests run against the host engine and,
under ``-m gpu``, against the hipGraph GPU engine.""" 
import io
import math
import os
import runpy
import sys
import types
from contextlib import contextmanager
from pathlib import Path

import numpy as np
import pytest

REF_UI = Path(os.environ.get("COBALT_REFERENCE_UI", "/root/reference/src/streamlit_ui/cobalt_streamlit.py"))
HOST = "http://cobalt-lender-api:8000"

pytestmark = pytest.mark.skipif(not REF_UI.exists(), reason="reference UI script not available")


class _Upload(io.BytesIO):
    def __init__(self, name, data):
        super().__init__(data)
        self.name = name


def _streamlit(mode, upload=None):
    st = types.ModuleType("streamlit")
    st.events = []

    @contextmanager
    def _ctx():
        yield st

    st.set_page_config = lambda **k: None
    st.title = st.subheader = st.text = lambda *a, **k: st.events.append(("text", a))
    st.sidebar = types.SimpleNamespace(radio=lambda label, opts: mode)
    st.columns = lambda n: [_ctx() for _ in range(n)]
    st.number_input = lambda label, value=0.0, **k: value
    st.selectbox = lambda label, opts, index=0: opts[index]
    st.checkbox = lambda label: False
    st.button = lambda label: True
    st.success = lambda m: st.events.append(("success", m))
    st.error = lambda m: st.events.append(("error", m))
    st.pyplot = lambda fig: st.events.append(("pyplot", fig))
    st.write = lambda *a, **k: st.events.append(("write", a))
    st.dataframe = lambda df: st.events.append(("dataframe", df))
    st.download_button = lambda *a, **k: st.events.append(("download", a))
    st.file_uploader = lambda *a, **k: upload

    def _stop():
        raise RuntimeError("st.stop")

    st.stop = _stop
    return st


def _shap():
    shap = types.ModuleType("shap")
    shap.calls = []

    class Explanation:
        def __init__(self, values, base_values, data, feature_names):
            self.values, self.base_values, self.data, self.feature_names = values, base_values, data, feature_names

    def waterfall(exp, max_display=10, show=True):
        shap.calls.append(("waterfall", exp, max_display, show))

    shap.Explanation = Explanation
    shap.plots = types.SimpleNamespace(waterfall=waterfall)
    return shap


@pytest.fixture(params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def routed_api(request, reference_booster, monkeypatch):
    """The API behind the UI: the host engine, and (``-m gpu``) the MI355X engine the north star names
    -- hipGraph-captured predictor + TreeSHAP buckets behind the micro-batcher, device CSV parsing for
    the bulk upload (ServeConfig(device="cuda", use_graphs=True))."""
    import requests
    from fastapi.testclient import TestClient

    from cobalt_smart_lender_ai_amd.config import ServeConfig
    from cobalt_smart_lender_ai_amd.serve.app import create_app

    cfg = ServeConfig(device="cpu") if request.param == "cpu" else ServeConfig(device="cuda", use_graphs=True)
    with TestClient(create_app(cfg, booster=reference_booster)) as client:
        sent = []

        def post(url, **kw):
            assert url.startswith(HOST + "/"), url  # the UI's hard-coded API_URL, unchanged
            sent.append(url[len(HOST):])
            return client.post(url[len(HOST):], **kw)

        monkeypatch.setattr(requests, "post", post)
        yield sent


def _run(monkeypatch, st, shap):
    import matplotlib

    matplotlib.use("Agg")
    monkeypatch.setitem(sys.modules, "streamlit", st)
    monkeypatch.setitem(sys.modules, "shap", shap)
    runpy.run_path(str(REF_UI), run_name="__main__")


def test_reference_ui_single_prediction(routed_api, monkeypatch):
    st, shap = _streamlit("🔍 Single Prediction"), _shap()
    _run(monkeypatch, st, shap)
    kinds = [e[0] for e in st.events]
    assert "error" not in kinds, st.events
    assert routed_api == ["/predict"]
    (msg,) = [e[1] for e in st.events if e[0] == "success"]
    assert msg == "Estimated Default Probability: 9.42%"  # SURVEY §4 golden: p = 0.0941799
    (call,) = shap.calls
    _, exp, max_display, show = call
    assert max_display == 10 and show is False
    assert len(exp.values) == 20 and len(exp.feature_names) == 20 and len(exp.data) == 20
    assert exp.feature_names[15] == "application_type_Joint App"
    # local accuracy: base value + SHAP values = the model margin of the predicted probability
    p = 0.0941799
    assert math.isclose(float(exp.base_values) + float(np.sum(exp.values)), math.log(p / (1 - p)), abs_tol=2e-5)
    assert "pyplot" in kinds


def test_reference_ui_bulk_prediction(routed_api, monkeypatch):
    from cobalt_smart_lender_ai_amd.config import DEPLOYED_FEATURES

    rng = np.random.default_rng(1)
    rows = rng.random((6, 20)) * 100
    csv = ",".join(DEPLOYED_FEATURES) + "\n" + "\n".join(",".join(f"{v:.3f}" for v in r) for r in rows) + "\n"
    st, shap = _streamlit("📤 Bulk Prediction + SHAP", _Upload("batch.csv", csv.encode())), _shap()
    _run(monkeypatch, st, shap)
    kinds = [e[0] for e in st.events]
    assert "error" not in kinds, st.events
    assert routed_api == ["/predict_bulk_csv", "/feature_importance_bulk"]
    (df,) = [e[1] for e in st.events if e[0] == "dataframe"]
    assert len(df) == 6 and "prob_default" in df.columns
    assert ((df["prob_default"] > 0) & (df["prob_default"] < 1)).all()
    assert kinds.count("pyplot") == 1 and "download" in kinds
