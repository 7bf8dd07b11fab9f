"""Evaluation figures of the training job (reference: model_tree_train_test.py:184-210)."""
import io

import numpy as np

from cobalt_smart_lender_ai_amd.utils import plots


def test_feature_importance_figure_top10_order():
    names = [f"f{i}" for i in range(15)]
    imp = np.array([3, 9, 1, 7, 7, 0, 2, 8, 4, 6, 5, 0.5, 11, 10, 0.1])
    fig = plots.feature_importance_figure(names, imp)
    ax = fig.axes[0]
    labels = [t.get_text() for t in ax.get_yticklabels()]
    # barh draws bottom-up: the most important feature is the last label; ties keep input order
    assert labels[::-1] == ["f12", "f13", "f1", "f7", "f3", "f4", "f9", "f10", "f8", "f0"]
    widths = [p.get_width() for p in ax.patches][::-1]
    assert widths == sorted(widths, reverse=True)
    assert ax.get_title() == "Top 10 Most Important Features"
    buf = io.BytesIO()
    fig.savefig(buf, format="png")
    assert buf.getvalue()[:8] == b"\x89PNG\r\n\x1a\n"
    plots.close(fig)


def test_confusion_matrix_figure_annotations():
    cm = np.array([[90, 10], [5, 45]])
    fig = plots.confusion_matrix_figure(cm)
    ax = fig.axes[0]
    texts = sorted(t.get_text() for t in ax.texts)
    assert texts == sorted(["90", "10", "5", "45"])
    assert ax.get_xlabel() == "Predicted" and ax.get_ylabel() == "Actual"
    plots.close(fig)
