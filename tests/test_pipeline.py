"""Model selection, metrics, training pipeline, CLI and UI helpers (CPU; SURVEY.md §4 strategy:
compare against scikit-learn's own implementations where the reference uses them)."""
import json

import numpy as np
import pandas as pd
import pytest

from cobalt_smart_lender_ai_amd.config import (BEST_MODEL_FILENAME, CLEAN_DATA_KEY_NN, CLEAN_DATA_KEY_TREE,
                                               DEPLOYED_FEATURES, FEATURES_FILENAME, METRICS_JSON, TrainConfig)
from cobalt_smart_lender_ai_amd.metrics import classification as cm
from cobalt_smart_lender_ai_amd.models import gbdt
from cobalt_smart_lender_ai_amd.models.booster import load_pickle_bytes
from cobalt_smart_lender_ai_amd.select.rfe import rfe
from cobalt_smart_lender_ai_amd.select.search import randomized_search, sample_candidates


def _toy(n=1500, f=8, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, f)).astype(np.float32)
    X[rng.random((n, f)) < 0.05] = np.nan
    logit = 1.5 * np.nan_to_num(X[:, 0]) - np.nan_to_num(X[:, 2]) + 0.5 * np.nan_to_num(X[:, 5]) - 1.0
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    return X, y


# ------------------------------------------------------------------------------ metrics
def test_classification_report_matches_sklearn():
    from sklearn import metrics as skm

    rng = np.random.default_rng(1)
    y = rng.integers(0, 2, 500)
    p = np.where(rng.random(500) < 0.8, y, 1 - y)
    assert np.array_equal(cm.confusion_matrix(y, p), skm.confusion_matrix(y, p))
    ours = cm.classification_report(y, p, output_dict=True)
    ref = skm.classification_report(y, p, output_dict=True)
    assert ours.keys() == ref.keys()
    for k, v in ref.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                assert ours[k][kk] == pytest.approx(vv, rel=1e-12)
        else:
            assert ours[k] == pytest.approx(v, rel=1e-12)
    assert cm.classification_report(y, p) == skm.classification_report(y, p)
    assert cm.accuracy_score(y, p) == pytest.approx(skm.accuracy_score(y, p))
    q = np.clip(rng.random(500), 1e-3, 1 - 1e-3)
    assert cm.log_loss(y, q) == pytest.approx(skm.log_loss(y, q), rel=1e-10)


# ------------------------------------------------------------------------------ RFE
def test_rfe_matches_sklearn_rfe_over_refits():
    """Single-binning masked RFE == sklearn RFE re-fitting the estimator on each column subset."""
    from sklearn.feature_selection import RFE

    X, y = _toy()
    params = dict(n_estimators=6, max_depth=3, learning_rate=0.3, random_state=42)
    ours = rfe(X, y, params, n_features_to_select=3, step=1, device="cpu")
    sk = RFE(gbdt.GBDTClassifier(device="cpu", **params), n_features_to_select=3, step=1).fit(X, y)
    assert np.array_equal(ours.support_, sk.support_)
    assert np.array_equal(ours.ranking_, sk.ranking_)
    assert ours.n_features_ == 3
    assert set(np.nonzero(ours.support_)[0]) >= {0, 2}


# ------------------------------------------------------------------------------ randomized search
def test_search_candidates_match_parameter_sampler():
    from sklearn.model_selection import ParameterSampler

    from cobalt_smart_lender_ai_amd.config import SEARCH_SPACE

    ours = sample_candidates(SEARCH_SPACE, 20, 22)
    ref = list(ParameterSampler(SEARCH_SPACE, n_iter=20, random_state=22))
    assert ours == ref


def test_search_matches_sklearn_randomized_search():
    from sklearn.model_selection import RandomizedSearchCV, StratifiedKFold

    X, y = _toy(n=1200, f=6, seed=3)
    space = {"n_estimators": [4, 8], "max_depth": [2, 3], "learning_rate": [0.1, 0.3], "gamma": [0, 1]}
    base = dict(gbdt.XGB_DEFAULTS, scale_pos_weight=2.0, random_state=78)
    ours = randomized_search(X, y, space, base, n_iter=4, cv=3, random_state=22, device="cpu")
    sk = RandomizedSearchCV(gbdt.GBDTClassifier(device="cpu", scale_pos_weight=2.0, random_state=78), space,
                            n_iter=4, scoring="roc_auc", cv=StratifiedKFold(3), random_state=22, n_jobs=1).fit(X, y)
    np.testing.assert_allclose(ours.cv_results_["mean_test_score"], sk.cv_results_["mean_test_score"], rtol=1e-12)
    assert np.array_equal(ours.cv_results_["rank_test_score"], sk.cv_results_["rank_test_score"])
    assert ours.best_params_ == sk.best_params_
    a = ours.best_estimator_.predict_margin(X, device="cpu")
    b = sk.best_estimator_.get_booster().predict_margin(X, device="cpu")
    np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


# ------------------------------------------------------------------------------ pipeline + CLI
@pytest.fixture(scope="module")
def lake(tmp_path_factory):
    from cobalt_smart_lender_ai_amd.cli import main

    root = tmp_path_factory.mktemp("lake")
    assert main(["--store", str(root), "--device", "cpu", "synth", "--rows", "3000", "--full", "--both"]) == 0
    assert main(["--store", str(root), "--device", "cpu", "clean", "--full"]) == 0
    assert main(["--store", str(root), "--device", "cpu", "features", "--reference-date", "2025-07-04"]) == 0
    return root


def test_cli_prep_stages_write_datasets(lake):
    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore

    st = LocalStore(lake)
    tree = st.read_csv(CLEAN_DATA_KEY_TREE)
    nn = st.read_csv(CLEAN_DATA_KEY_NN)
    assert "loan_default" in tree.columns and "loan_default" in nn.columns
    assert len(tree) == len(nn) > 1000
    assert "grade_E" in tree.columns


def test_training_pipeline_writes_reference_artifacts(lake, tmp_path):
    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore
    from cobalt_smart_lender_ai_amd.pipeline.train_tree import run_training

    st = LocalStore(lake)
    df = st.read_csv(CLEAN_DATA_KEY_TREE)
    cfg = TrainConfig(rfe_n_features=6, search_n_iter=2,
                      search_space={"n_estimators": [5, 10], "max_depth": [2, 3], "learning_rate": [0.3]})
    m = run_training(df, cfg, store=st, local_dir=tmp_path, device="cpu",
                     rfe_params=dict(n_estimators=5, max_depth=3))
    assert 0.5 < m["auc"] <= 1.0
    assert set(m["classification_report"]) == {"0", "1", "accuracy", "macro avg", "weighted avg"}
    assert len(m["selected_features"]) == 6
    for name in (BEST_MODEL_FILENAME, FEATURES_FILENAME, METRICS_JSON, "confusion_matrix.png",
                 "feature_importance.png"):
        assert (tmp_path / name).exists(), name
        assert st.exists(cfg.output_path + name), name
    feats = (tmp_path / FEATURES_FILENAME).read_text().splitlines()
    assert feats[:6] == m["selected_features"] and feats[-1].startswith("#")
    saved = json.loads((tmp_path / METRICS_JSON).read_text())
    assert set(saved) == {"auc", "classification_report", "best_params"}
    state, bst = load_pickle_bytes((tmp_path / BEST_MODEL_FILENAME).read_bytes())
    assert bst.feature_names == m["selected_features"]
    assert state["eval_metric"] == "logloss" and state["random_state"] == 78
    assert bst.num_trees == saved["best_params"]["n_estimators"]


def test_device_frame_hand_off_trains_the_same_models(lake, tmp_path):
    """run_training on a DeviceFrame (device-resident matrix, device gathers for split / RFE repack /
    folds / eval rows) selects the same features and best params, with the same AUC and the same
    pickled model, as the pandas hand-off of the same tree CSV."""
    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore
    from cobalt_smart_lender_ai_amd.pipeline.train_tree import run_training
    from cobalt_smart_lender_ai_amd.prep.device_frame import DeviceFrame

    st = LocalStore(lake)
    cfg = TrainConfig(rfe_n_features=6, search_n_iter=2,
                      search_space={"n_estimators": [5, 10], "max_depth": [2, 3], "learning_rate": [0.3]})
    kw = dict(device="cpu", rfe_params=dict(n_estimators=5, max_depth=3))
    ref = run_training(st.read_csv(CLEAN_DATA_KEY_TREE), cfg, local_dir=tmp_path / "pd", **kw)
    frame = DeviceFrame.read_csv(st.get_bytes(CLEAN_DATA_KEY_TREE), "cpu", engine="arrow")
    got = run_training(frame, cfg, local_dir=tmp_path / "dev", **kw)
    assert got["hand_off"] == "device" and ref["hand_off"] == "pandas"
    assert got["selected_features"] == ref["selected_features"]
    assert got["best_params"] == ref["best_params"] and got["auc"] == ref["auc"]
    assert (tmp_path / "dev" / BEST_MODEL_FILENAME).read_bytes() == (tmp_path / "pd" / BEST_MODEL_FILENAME).read_bytes()


# ------------------------------------------------------------------------------ UI + automation
def test_ui_payload_matches_api_schema():
    from cobalt_smart_lender_ai_amd.serve.app import SingleInput
    from cobalt_smart_lender_ai_amd.ui import client

    p = client.single_payload({"loan_amnt": 5000.0}, grade_e=True, hardship="No_Hardship")
    assert set(p) == set(DEPLOYED_FEATURES)
    assert p["grade_E"] == 1 and p["hardship_status_No Hardship"] == 1 and p["hardship_status_BROKEN"] == 0
    SingleInput.model_validate(p)
    fig = client.waterfall_figure(np.linspace(-1, 1, 20), -2.0, np.arange(20.0), list(DEPLOYED_FEATURES))
    assert len(fig.axes[0].patches) == 10
    client.importance_figure([{"feature": "a", "importance": 2.0}, {"feature": "b", "importance": 1.0}])


def test_automation_sample_and_score(tmp_path, reference_booster):
    from cobalt_smart_lender_ai_amd.serve.automation import make_sample, score_file

    rng = np.random.default_rng(0)
    df = pd.DataFrame(rng.random((50, len(DEPLOYED_FEATURES))), columns=DEPLOYED_FEATURES)
    df["loan_default"] = rng.integers(0, 2, 50)
    y = make_sample(df, tmp_path / "in" / "test_sample.csv")
    assert len(y) == 10
    out = score_file(reference_booster, tmp_path / "in" / "test_sample.csv", tmp_path / "out" / "latest.csv",
                     device="cpu")
    assert out["prob_default"].between(0, 1).all() and len(out) == 10


def test_rfecv_matches_sklearn():
    from sklearn.feature_selection import RFECV
    from sklearn.model_selection import StratifiedKFold

    from cobalt_smart_lender_ai_amd.select.rfecv import rfecv

    X, y = _toy(n=1500, f=9, seed=7)
    params = dict(n_estimators=5, max_depth=3, learning_rate=0.3, random_state=1)
    ours = rfecv(X, y, params, step=2, cv=3, min_features_to_select=3, device="cpu")
    sk = RFECV(gbdt.GBDTClassifier(device="cpu", **params), step=2, cv=StratifiedKFold(3), scoring="roc_auc",
               min_features_to_select=3).fit(X, y)
    np.testing.assert_array_equal(ours.cv_results_["n_features"], sk.cv_results_["n_features"])
    np.testing.assert_allclose(ours.cv_results_["mean_test_score"], sk.cv_results_["mean_test_score"], rtol=1e-12)
    assert ours.n_features_ == sk.n_features_
    np.testing.assert_array_equal(ours.support_, sk.support_)


def test_raw_data_manifest_verify(tmp_path):
    from cobalt_smart_lender_ai_amd.dataio import datasets
    from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore

    blob = b"loan_amnt,term\n1000, 36 months\n"
    f = datasets.RawFile("raw/sample.csv", __import__("hashlib").md5(blob).hexdigest(), len(blob), "dataset/1-raw/x")
    assert datasets.verify(tmp_path, (f,)) == {"raw/sample.csv": "missing"}
    (tmp_path / "raw").mkdir()
    (tmp_path / "raw" / "sample.csv").write_bytes(blob)
    assert datasets.verify(tmp_path, (f,)) == {"raw/sample.csv": "ok"}
    st = LocalStore(tmp_path / "lake")
    assert datasets.stage_into_store(st, tmp_path, (f,)) == ["dataset/1-raw/x"]
    assert st.get_bytes("dataset/1-raw/x") == blob
    (tmp_path / "raw" / "sample.csv").write_bytes(blob[:-1] + b"!")
    assert datasets.verify(tmp_path, (f,)) == {"raw/sample.csv": "md5 mismatch"}


def test_baseline_plumbing_config_runs_end_to_end():
    """BASELINE.json config 1 (10k-row sample, sklearn LogisticRegression on CPU): raw rows through the
    reference cleaning + feature engineering into a working classifier (scripts/bench_configs.py)."""
    import importlib.util
    from pathlib import Path

    spec = importlib.util.spec_from_file_location("bench_configs",
                                                  Path(__file__).resolve().parents[1] / "scripts/bench_configs.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    r = mod.plumbing_10k(rows=4_000, trees=20)
    assert r["rows_after_prep"] > 3_500 and r["features"] > 40
    assert r["logreg_auc"] > 0.85 and r["gbdt_cpu_auc"] > 0.85


def test_rfe_repacked_fits_equal_masked_fits():
    """RFE fits on the surviving columns only (repacked bins) grow exactly the trees of masked fits on
    the full-width matrix: same boosters at every step, same support and ranking."""
    from cobalt_smart_lender_ai_amd.select.rfe import rfe

    rng = np.random.default_rng(4)
    n, F = 6000, 12
    X = rng.normal(size=(n, F)).astype(np.float32)
    X[:, 3] = np.round(X[:, 3])
    X[rng.random((n, F)) < 0.05] = np.nan
    y = (np.nan_to_num(X[:, 0]) + 0.5 * np.nan_to_num(X[:, 5]) - np.nan_to_num(X[:, 7]) + rng.normal(size=n) > 0)
    y = y.astype(np.float32)
    params = dict(n_estimators=8, max_depth=4, learning_rate=0.3, colsample_bytree=0.7, random_state=3)
    names = [f"c{i}" for i in range(F)]
    got, ref = [], []
    a = rfe(X, y, params, n_features_to_select=5, step=2, device="cpu", feature_names=names,
            step_score=lambda b, s: got.append(b.save_raw("ubj")))
    b = rfe(X, y, params, n_features_to_select=5, step=2, device="cpu", feature_names=names, repack=False,
            step_score=lambda b, s: ref.append(b.save_raw("ubj")))
    assert got == ref and len(got) == 5
    assert np.array_equal(a.support_, b.support_) and np.array_equal(a.ranking_, b.ranking_)
    assert a.estimator_.save_raw("ubj") == b.estimator_.save_raw("ubj")
