"""Training-loop metrics (elliptic_gnn_project_amd/metrics.py) against golden vectors produced by
the reference's own src/utils/metrics.py (tests/golden/make_metrics_golden.py), including the
reference unit test's input (tests/test_masks_and_metrics.py:21-28)."""
import json
import os

import numpy as np
import pytest

from elliptic_gnn_project_amd import metrics as M

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "metrics_golden.json")))


@pytest.mark.parametrize("i", range(len(GOLD["cases"])))
def test_metrics_match_reference_vectors(i):
    c = GOLD["cases"][i]
    y, s = np.array(c["y"]), np.array(c["s"])
    assert M.pr_auc_illicit(y, s) == pytest.approx(c["pr_auc"], abs=1e-12)
    assert M.roc_auc_illicit(y, s) == pytest.approx(c["roc_auc"], abs=1e-12)
    thr, f1 = M.pick_threshold_max_f1(y, s)
    assert thr == c["thr_max_f1"] and f1 == pytest.approx(c["f1_max"], abs=1e-12)
    assert M.f1_at_threshold(y, s, 0.5) == pytest.approx(c["f1_at_0.5"], abs=1e-12)
    assert M.pick_threshold_for_precision(y, s, 0.90) == c["thr_p90"]
    assert M.pick_threshold_for_precision(y, s, 0.999) == c["thr_p999"]
    assert M.precision_at_k(y, s, 10) == c["p_at_10"] and M.precision_at_k(y, s, 100) == c["p_at_100"]
    assert M.recall_at_precision(y, s, 0.80) == c["r_at_p80"]
    assert M.recall_at_precision(y, s, 0.999) == c["r_at_p999"]
    assert M.expected_calibration_error(y, s, 15) == pytest.approx(c["ece15"], abs=1e-12)
    assert M.expected_calibration_error(y, s, 10) == pytest.approx(c["ece10"], abs=1e-12)


def test_reference_unit_case():
    c = GOLD["reference_unit_case"]
    y, s = np.array(c["y"]), np.array(c["s"])
    assert M.pr_auc_illicit(y, s) == pytest.approx(c["pr_auc"], abs=1e-12)
    assert M.pick_threshold_max_f1(y, s)[0] == c["thr_max_f1"]
    assert M.precision_at_k(y, s, 3) == c["p_at_3"]
    assert M.expected_calibration_error(y, s) == pytest.approx(c["ece15"], abs=1e-12)
