"""Classification metrics computed from confusion matrices.

The reference converts every prediction to a host ``int`` and calls sklearn per task
(utils.py:297-322).  The framework accumulates confusion matrices on the device (one atomic per
sample in the head kernel) and derives the same numbers from them, with sklearn's definitions:

  accuracy            trace / total
  per-class F1        over the labels present in y_true U y_pred (sklearn ``average=None``)
  weighted F1/P/R     support-weighted means (``average='weighted'``); ill-defined ratios are 0
                      (sklearn's zero_division default, without the warning)

``sklearn_confusion`` reproduces ``sklearn.metrics.confusion_matrix(y_true, y_pred)``'s label set
(sorted union of observed labels) for printing parity; the saved artefacts use the full fixed-size
matrix (16x16 / 2x2) so that downstream plotting never depends on which classes happened to occur.
"""
from __future__ import annotations

from typing import Dict

import numpy as np


def _safe_div(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    out = np.zeros_like(a)
    np.divide(a, b, out=out, where=b != 0)
    return out


def present_labels(cm: np.ndarray) -> np.ndarray:
    cm = np.asarray(cm)
    return np.nonzero((cm.sum(0) + cm.sum(1)) > 0)[0]


def sklearn_confusion(cm: np.ndarray) -> np.ndarray:
    lab = present_labels(cm)
    return np.asarray(cm)[np.ix_(lab, lab)]


def metrics_from_confusion(cm: np.ndarray) -> Dict[str, object]:
    """cm[true, pred] -> accuracy, per-class F1 (present labels), weighted F1 / precision / recall."""
    cm = np.asarray(cm, dtype=np.float64)
    total = cm.sum()
    tp = np.diag(cm)
    support = cm.sum(1)
    predicted = cm.sum(0)
    prec = _safe_div(tp, predicted)
    rec = _safe_div(tp, support)
    f1 = _safe_div(2 * tp, support + predicted)
    lab = present_labels(cm)
    w = _safe_div(support, total) if total else np.zeros_like(support)
    return {
        "accuracy": float(tp.sum() / total) if total else 0.0,
        "f1_per_class": f1[lab],
        "labels": lab,
        "f1_weighted": float((f1 * w).sum()),
        "precision_weighted": float((prec * w).sum()),
        "recall_weighted": float((rec * w).sum()),
        "total": int(total),
    }


def confusion_from_lists(y_true, y_pred, n: int) -> np.ndarray:
    cm = np.zeros((n, n), dtype=np.int64)
    np.add.at(cm, (np.asarray(y_true, dtype=np.int64), np.asarray(y_pred, dtype=np.int64)), 1)
    return cm


def mae_from_confusion(cm: np.ndarray) -> float:
    """Mean |pred - true| over the samples of a distance confusion matrix (1 class = 1 m): the radial
    distance localisation error in metres (an addition; the reference only reports accuracy)."""
    cm = np.asarray(cm, dtype=np.float64)
    n = cm.shape[0]
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    tot = cm.sum()
    return float((np.abs(i - j) * cm).sum() / tot) if tot else 0.0


def format_task_report(name: str, cm: np.ndarray) -> str:
    """The per-task block the reference prints after each validation (utils.py:314-322)."""
    m = metrics_from_confusion(cm)
    lines = [name, str(sklearn_confusion(cm)), "Accuracy：{}".format(m["accuracy"]), str(m["f1_per_class"]),
             "F1_Score：{}".format(m["f1_weighted"]), "Precision：{}".format(m["precision_weighted"]),
             "Recall：{}".format(m["recall_weighted"])]
    return "\n".join(lines)
