"""AUC parity at the headline configuration (BASELINE.md "AUC parity: the GPU model's test AUC must be
within +-0.002 of a CPU oracle trained on the same synthetic data with the same config").

2M training rows of the LendingClub-shaped data, the deployed hyper-parameters (300 trees, depth 7,
eta 0.05, gamma 5, lambda 1, max_bin 256, scale_pos_weight = neg/pos; the reference's AUC printout:
/root/reference/src/model_train_test/model_tree_train_test.py:175-179), every row sketched (the exact
device sketch, XGBoost `hist`'s all-row semantics). The CPU oracle is an independent implementation --
scikit-learn's OpenMP HistGradientBoostingClassifier with the same trees / rate / L2 / class weight
(XGBoost itself is not installed) -- so the parity is not the GPU trainer agreeing with its own NumPy
twin (that is tests/test_gpu_gbdt.py, bit for bit, at small sizes)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS, TEST_ROWS = 2_000_000, 500_000


@pytest.mark.timeout(900)
def test_headline_config_auc_parity_with_cpu_oracle_at_2m_rows():
    from sklearn.ensemble import HistGradientBoostingClassifier

    from cobalt_smart_lender_ai_amd.dataio import synth
    from cobalt_smart_lender_ai_amd.metrics.auc import roc_auc
    from cobalt_smart_lender_ai_amd.models import gbdt

    dev = torch.device("cuda", 0)
    X, y = synth.make_lendingclub(ROWS, seed=11, device=dev)
    Xte, yte = synth.make_lendingclub(TEST_ROWS, seed=11, row_offset=ROWS, device=dev)
    spw = float((y == 0).sum() / (y == 1).sum())
    params = gbdt.GBDTParams(n_estimators=300, max_depth=7, learning_rate=0.05, gamma=5.0, reg_lambda=1.0,
                             min_child_weight=1.0, max_bin=256, scale_pos_weight=spw, random_state=78,
                             sketch_rows=None)
    b = gbdt.train(X, y, params, device=dev)
    auc_gpu = float(roc_auc(yte, b.predict_proba(Xte, device=dev)))

    Xh, yh, Xth, yth = X.cpu().numpy(), y.cpu().numpy(), Xte.cpu().numpy(), yte.cpu().numpy()
    clf = HistGradientBoostingClassifier(max_iter=300, max_depth=7, learning_rate=0.05, l2_regularization=1.0,
                                         max_bins=255, min_samples_leaf=1, max_leaf_nodes=None, early_stopping=False,
                                         class_weight={0: 1.0, 1: spw}, random_state=78)
    clf.fit(Xh, yh)
    auc_cpu = float(roc_auc(yth, clf.predict_proba(Xth)[:, 1]))
    print(f"AUC at {ROWS} rows: GPU {auc_gpu:.5f}  CPU oracle {auc_cpu:.5f}")
    assert np.isfinite(auc_gpu) and auc_gpu > 0.9
    assert abs(auc_gpu - auc_cpu) <= 0.002, (auc_gpu, auc_cpu)
