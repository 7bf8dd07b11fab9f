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
import base64
import io
import json
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

FIXTURE = Path(__file__).parent / "fixtures" / "reference_ui_exchanges.json"
needs_ref = pytest.mark.skipif(not REF_UI.exists(), reason="reference UI script not available")


class _Sent(list):
    """Paths the UI posted to, plus the full exchanges (request payload + JSON response)."""

    def __init__(self):
        super().__init__()
        self.exchanges = []


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
        sent = _Sent()

        def post(url, **kw):
            assert url.startswith(HOST + "/"), url  # the UI's hard-coded API_URL, unchanged
            path = url[len(HOST):]
            sent.append(path)
            res = client.post(path, **kw)
            ex = {"path": path, "status": res.status_code, "response": res.json()}
            if "json" in kw:
                ex["json"] = kw["json"]
            if "files" in kw:
                ex["files"] = {k: [v[0], base64.b64encode(v[1]).decode(), v[2]] for k, v in kw["files"].items()}
            sent.exchanges.append(ex)
            return res

        monkeypatch.setattr(requests, "post", post)
        yield sent


def _run(monkeypatch, st, shap):
    import matplotlib

    matplotlib.use("Agg")
    monkeypatch.setitem(sys.modules, "streamlit", st)
    monkeypatch.setitem(sys.modules, "shap", shap)
    runpy.run_path(str(REF_UI), run_name="__main__")


@needs_ref
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


def _bulk_upload():
    from cobalt_smart_lender_ai_amd.config import DEPLOYED_FEATURES

    rng = np.random.default_rng(1)
    rows = rng.random((6, 20)) * 100
    csv = ",".join(DEPLOYED_FEATURES) + "\n" + "\n".join(",".join(f"{v:.3f}" for v in r) for r in rows) + "\n"
    return _Upload("batch.csv", csv.encode())


@needs_ref
def test_reference_ui_bulk_prediction(routed_api, monkeypatch):
    st, shap = _streamlit("📤 Bulk Prediction + SHAP", _bulk_upload()), _shap()
    _run(monkeypatch, st, shap)
    kinds = [e[0] for e in st.events]
    assert "error" not in kinds, st.events
    assert routed_api == ["/predict_bulk_csv", "/feature_importance_bulk"]
    (df,) = [e[1] for e in st.events if e[0] == "dataframe"]
    assert len(df) == 6 and "prob_default" in df.columns
    assert ((df["prob_default"] > 0) & (df["prob_default"] < 1)).all()
    assert kinds.count("pyplot") == 1 and "download" in kinds


def _close(a, b, path=""):
    """Recorded vs replayed JSON: equal structure, numbers within 2e-6 (float32 GPU vs host engine)."""
    if isinstance(a, dict):
        assert isinstance(b, dict) and set(a) == set(b), (path, a, b)
        for k in a:
            _close(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, list):
        assert isinstance(b, list) and len(a) == len(b), (path, len(a), len(b))
        for i, (x, y) in enumerate(zip(a, b)):
            _close(x, y, f"{path}[{i}]")
    elif isinstance(a, float) or isinstance(b, float):
        assert math.isclose(float(a), float(b), rel_tol=2e-6, abs_tol=2e-6), (path, a, b)
    else:
        assert a == b, (path, a, b)


@needs_ref
def test_reference_ui_exchanges_fixture_is_current(monkeypatch, reference_booster):
    """The reference UI's HTTP exchanges (both modes) against the host engine, recorded into
    tests/fixtures/reference_ui_exchanges.json: the requests the unmodified script sends and the
    responses it renders (p = 9.42%). Where the reference checkout exists this asserts the fixture is
    current; COBALT_RECORD_UI=1 rewrites it."""
    import requests
    from fastapi.testclient import TestClient

    from cobalt_smart_lender_ai_amd.config import ServeConfig
    from cobalt_smart_lender_ai_amd.serve.app import create_app

    got = {}
    for mode, upload in (("single", None), ("bulk", _bulk_upload())):
        with TestClient(create_app(ServeConfig(device="cpu"), booster=reference_booster)) as client:
            sent = _Sent()

            def post(url, **kw):
                path = url[len(HOST):]
                res = client.post(path, **kw)
                ex = {"path": path, "status": res.status_code, "response": res.json()}
                if "json" in kw:
                    ex["json"] = kw["json"]
                if "files" in kw:
                    ex["files"] = {k: [v[0], base64.b64encode(v[1]).decode(), v[2]] for k, v in kw["files"].items()}
                sent.exchanges.append(ex)
                return res

            monkeypatch.setattr(requests, "post", post)
            name = "🔍 Single Prediction" if mode == "single" else "📤 Bulk Prediction + SHAP"
            _run(monkeypatch, _streamlit(name, upload), _shap())
            got[mode] = sent.exchanges
    if os.environ.get("COBALT_RECORD_UI") == "1" or not FIXTURE.exists():
        FIXTURE.write_text(json.dumps(got, indent=1, ensure_ascii=False))
    want = json.loads(FIXTURE.read_text())
    for mode in ("single", "bulk"):
        assert [e["path"] for e in want[mode]] == [e["path"] for e in got[mode]]
        for w, g in zip(want[mode], got[mode]):
            _close(w, g, mode)


@pytest.mark.gpu
def test_reference_ui_exchanges_on_the_gpu_engine(reference_booster):
    """On a box without the reference checkout: the reference UI's recorded exchanges replayed against
    the hipGraph GPU engine (ServeConfig(device="cuda", use_graphs=True)) -- every response equals the
    host engine's that the unmodified script rendered (single: 9.42%; bulk: the 6-row table and the
    top-10 importance)."""
    from fastapi.testclient import TestClient

    from cobalt_smart_lender_ai_amd.config import ServeConfig
    from cobalt_smart_lender_ai_amd.serve.app import create_app

    rec = json.loads(FIXTURE.read_text())
    with TestClient(create_app(ServeConfig(device="cuda", use_graphs=True), booster=reference_booster)) as client:
        for mode in ("single", "bulk"):
            for ex in rec[mode]:
                kw = {}
                if "json" in ex:
                    kw["json"] = ex["json"]
                if "files" in ex:
                    kw["files"] = {k: (v[0], base64.b64decode(v[1]), v[2]) for k, v in ex["files"].items()}
                res = client.post(ex["path"], **kw)
                assert res.status_code == ex["status"] == 200
                _close(ex["response"], res.json(), f"{mode}{ex['path']}")
    p = rec["single"][0]["response"]["prob_default"]
    assert f"{p:.2%}" == "9.42%"
