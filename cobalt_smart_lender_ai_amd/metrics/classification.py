"""Binary classification metrics (K25): confusion matrix, precision/recall/F1, report, logloss.

Replaces ``sklearn.metrics.classification_report`` / ``confusion_matrix`` as used at
src/model_train_test/model_tree_train_test.py:174-179; the report dict has sklearn's exact layout
(per-class dicts keyed by label string, ``accuracy``, ``macro avg``, ``weighted avg``) because the
reference writes it verbatim into ``metrics.json`` (:235-242). Counting is one device pass
(``torch.bincount`` of ``2*y + pred``).
"""
from __future__ import annotations

import numpy as np
import torch


def _t(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.reshape(-1)
    return torch.as_tensor(np.asarray(x)).reshape(-1)


def confusion_matrix(y_true, y_pred) -> np.ndarray:
    """2x2 [[TN, FP], [FN, TP]] for 0/1 labels."""
    yt, yp = _t(y_true), _t(y_pred).to(_t(y_true).device)
    idx = yt.to(torch.int64) * 2 + yp.to(torch.int64)
    return torch.bincount(idx, minlength=4)[:4].reshape(2, 2).cpu().numpy()


def accuracy_score(y_true, y_pred) -> float:
    cm = confusion_matrix(y_true, y_pred)
    return float(np.trace(cm) / max(cm.sum(), 1))


def classification_report(y_true, y_pred, output_dict: bool = False, digits: int = 2):
    cm = confusion_matrix(y_true, y_pred).astype(np.float64)
    labels = ["0", "1"]
    out: dict = {}
    prec, rec, f1, sup = [], [], [], []
    for k in range(2):
        tp = cm[k, k]
        p_den = cm[:, k].sum()
        r_den = cm[k, :].sum()
        p = tp / p_den if p_den > 0 else 0.0
        r = tp / r_den if r_den > 0 else 0.0
        f = 2 * p * r / (p + r) if (p + r) > 0 else 0.0
        prec.append(p), rec.append(r), f1.append(f), sup.append(r_den)
        out[labels[k]] = {"precision": float(p), "recall": float(r), "f1-score": float(f), "support": float(r_den)}
    total = float(sum(sup))
    out["accuracy"] = float(np.trace(cm) / total) if total else 0.0
    out["macro avg"] = {"precision": float(np.mean(prec)), "recall": float(np.mean(rec)),
                        "f1-score": float(np.mean(f1)), "support": total}
    w = np.asarray(sup) / total if total else np.zeros(2)
    out["weighted avg"] = {"precision": float(np.dot(w, prec)), "recall": float(np.dot(w, rec)),
                           "f1-score": float(np.dot(w, f1)), "support": total}
    if output_dict:
        return out
    width = max(len("weighted avg"), digits)
    row = "{:>{w}s} " + " {:>9.{d}f}" * 3 + " {:>9}\n"
    lines = ["{:>{w}s} ".format("", w=width) + "".join(f" {h:>9}" for h in ("precision", "recall", "f1-score",
                                                                            "support")) + "\n\n"]
    for lab in labels:
        d = out[lab]
        lines.append(row.format(lab, d["precision"], d["recall"], d["f1-score"], int(d["support"]), w=width,
                                d=digits))
    lines.append("\n")
    lines.append("{:>{w}s} ".format("accuracy", w=width) + f" {'':>9} {'':>9} {out['accuracy']:>9.{digits}f}"
                 f" {int(total):>9}\n")
    for k in ("macro avg", "weighted avg"):
        d = out[k]
        lines.append(row.format(k, d["precision"], d["recall"], d["f1-score"], int(total), w=width, d=digits))
    return "".join(lines)


def log_loss(y_true, p, eps: float = 1e-15) -> float:
    y = _t(y_true).to(torch.float64)
    q = _t(p).to(torch.float64).to(y.device).clamp(eps, 1 - eps)
    return float(-(y * torch.log(q) + (1 - y) * torch.log1p(-q)).mean())
