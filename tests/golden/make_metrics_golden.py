"""Golden vectors for elliptic_gnn_project_amd/metrics.py, produced by the REFERENCE module
(/root/reference/src/utils/metrics.py, importable here: it needs only numpy and sklearn).

    python tests/golden/make_metrics_golden.py   # writes tests/golden/metrics_golden.json

Run in the build container only (the reference does not travel to the GPU box); the JSON it
writes is the committed fixture the CPU test suite checks against.
"""
import importlib.util
import json
import os

import numpy as np

REF = "/root/reference/src/utils/metrics.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "metrics_golden.json")


def main():
    spec = importlib.util.spec_from_file_location("ref_metrics", REF)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    cases = []
    for seed, n, pos in [(0, 200, 0.1), (1, 1000, 0.05), (2, 57, 0.4), (3, 3000, 0.02)]:
        rng = np.random.default_rng(seed)
        y = (rng.random(n) < pos).astype(np.int64)
        y[0], y[1] = 1, 0  # both classes present
        s = np.clip(0.35 * y + rng.random(n) * 0.8, 0.0, 1.0)
        s = np.round(s, 3)  # ties, as calibrated probabilities have
        s[2] = 1.0
        thr, f1 = m.pick_threshold_max_f1(y, s)
        cases.append({
            "y": y.tolist(), "s": s.tolist(),
            "pr_auc": m.pr_auc_illicit(y, s), "roc_auc": m.roc_auc_illicit(y, s),
            "thr_max_f1": thr, "f1_max": f1,
            "f1_at_0.5": m.f1_at_threshold(y, s, 0.5),
            "thr_p90": m.pick_threshold_for_precision(y, s, 0.90),
            "thr_p999": m.pick_threshold_for_precision(y, s, 0.999),
            "p_at_10": m.precision_at_k(y, s, 10), "p_at_100": m.precision_at_k(y, s, 100),
            "r_at_p80": m.recall_at_precision(y, s, 0.80), "r_at_p999": m.recall_at_precision(y, s, 0.999),
            "ece15": m.expected_calibration_error(y, s, 15), "ece10": m.expected_calibration_error(y, s, 10),
        })
    # the reference's own unit-test input (tests/test_masks_and_metrics.py:21-28)
    y = np.array([0, 1, 0, 1, 0, 0, 0, 1])
    s = np.linspace(0, 1, len(y))
    with open(OUT, "w") as fh:
        json.dump({"source": REF, "cases": cases,
                   "reference_unit_case": {"y": y.tolist(), "s": s.tolist(),
                                           "pr_auc": m.pr_auc_illicit(y, s),
                                           "thr_max_f1": m.pick_threshold_max_f1(y, s)[0],
                                           "p_at_3": m.precision_at_k(y, s, 3),
                                           "ece15": m.expected_calibration_error(y, s)}}, fh)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
