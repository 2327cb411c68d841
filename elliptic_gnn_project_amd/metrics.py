"""Evaluation metrics of the training loop (restates src/utils/metrics.py:1-75).

Host-side sklearn/numpy over the probabilities eval_split copies back; pinned against golden
vectors produced by the reference module itself (tests/golden/make_metrics_golden.py).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def pr_auc_illicit(y_true: np.ndarray, y_score: np.ndarray) -> float:
    """Average precision of the illicit class (metrics.py:10-12)."""
    from sklearn.metrics import average_precision_score
    return float(average_precision_score(y_true, y_score))


def roc_auc_illicit(y_true: np.ndarray, y_score: np.ndarray) -> float:
    """metrics.py:14-15."""
    from sklearn.metrics import roc_auc_score
    return float(roc_auc_score(y_true, y_score))


def f1_at_threshold(y_true: np.ndarray, y_score: np.ndarray, thr: float) -> float:
    """F1 of (score >= thr) (metrics.py:17-19)."""
    from sklearn.metrics import f1_score
    return float(f1_score(y_true, (y_score >= thr).astype(int)))


def _pr_curve(y_true, y_score):
    from sklearn.metrics import precision_recall_curve
    return precision_recall_curve(y_true, y_score)


def pick_threshold_max_f1(y_true: np.ndarray, y_score: np.ndarray) -> Tuple[float, float]:
    """Threshold maximising F1 along the PR curve; the curve's last point gets threshold 1.0
    (metrics.py:21-26)."""
    prec, rec, thr = _pr_curve(y_true, y_score)
    thr = np.concatenate([thr, [1.0]])
    f1 = 2.0 * prec * rec / (prec + rec + 1e-12)
    i = int(np.nanargmax(f1))
    return float(thr[i]), float(f1[i])


def pick_threshold_for_precision(y_true: np.ndarray, y_score: np.ndarray, target_p: float) -> float:
    """First PR-curve point with precision >= target, else the max-F1 threshold (metrics.py:28-35)."""
    prec, _, thr = _pr_curve(y_true, y_score)
    hit = prec >= target_p
    if not hit.any():
        return pick_threshold_max_f1(y_true, y_score)[0]
    return float(np.concatenate([thr, [1.0]])[int(np.argmax(hit))])


def precision_at_k(y_true: np.ndarray, y_score: np.ndarray, k: int) -> float:
    """Mean label of the k highest scores (metrics.py:37-39)."""
    top = np.argsort(-y_score)[:k]
    return float(np.mean(y_true[top]))


def recall_at_precision(y_true: np.ndarray, y_score: np.ndarray, target_p: float) -> float:
    """Best recall among PR-curve points with precision >= target, 0 if none (metrics.py:41-46)."""
    prec, rec, _ = _pr_curve(y_true, y_score)
    hit = prec >= target_p
    return float(rec[hit].max()) if hit.any() else 0.0


def expected_calibration_error(y_true: np.ndarray, y_prob: np.ndarray, bins: int = 15) -> float:
    """Equal-width-bin ECE of positive-class probabilities, last bin closed (metrics.py:48-66)."""
    y_true = y_true.astype(int)
    edges = np.linspace(0.0, 1.0, bins + 1)
    idx = np.clip(np.searchsorted(edges, y_prob, side="right") - 1, 0, bins - 1)  # [lo, hi); p == 1 -> last
    ece = 0.0
    for b in range(bins):
        m = idx == b
        if m.any():
            ece += m.mean() * abs(y_true[m].mean() - y_prob[m].mean())
    return float(ece)
