"""Evaluation figures written by the training pipeline (reference:
src/model_train_test/model_tree_train_test.py:184-210 -- seaborn confusion-matrix heatmap and a
top-10 gain-importance bar chart). Rendered with matplotlib's Agg backend (seaborn is optional)."""
from __future__ import annotations

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402


def confusion_matrix_figure(cm: np.ndarray):
    fig, ax = plt.subplots(figsize=(6, 4))
    im = ax.imshow(cm, cmap="Blues")
    for (i, j), v in np.ndenumerate(cm):
        ax.text(j, i, f"{int(v)}", ha="center", va="center",
                color="white" if v > cm.max() / 2 else "black")
    ax.set_xticks(range(cm.shape[1]))
    ax.set_yticks(range(cm.shape[0]))
    ax.set_title("Confusion Matrix")
    ax.set_xlabel("Predicted")
    ax.set_ylabel("Actual")
    fig.colorbar(im, ax=ax)
    return fig


def feature_importance_figure(names: list[str], importances: np.ndarray, top: int = 10):
    order = np.argsort(-np.asarray(importances), kind="stable")[:top]
    fig, ax = plt.subplots(figsize=(8, 5))
    ax.barh([names[i] for i in order][::-1], np.asarray(importances)[order][::-1], color="skyblue")
    ax.set_xlabel("Feature Importance (Gain)")
    ax.set_title(f"Top {top} Most Important Features")
    fig.tight_layout()
    return fig


def close(fig) -> None:
    plt.close(fig)
