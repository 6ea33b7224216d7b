"""Fixture for row f4 (patient-stratified splits): runs the REFERENCE's own
spine_vision/training/datasets/stratification.py (imported with make_golden.py's shims; iterstrat is a
stub there, so only the functions that do not call it are exercised) on seeded synthetic patient
records and stores the outputs in stratification.json.

    python tests/golden/make_strat_golden.py      (needs /root/reference; not run by the tests)
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def synthetic_records(n_patients: int = 60, seed: int = 3) -> list[dict]:
    rng = np.random.RandomState(seed)
    recs = []
    for p in range(n_patients):
        for lvl in range(5):
            recs.append({
                "patient_key": f"src{p % 3}_{p:03d}",
                "level": lvl,
                "pfirrmann": int(rng.choice(5, p=[0.1, 0.3, 0.3, 0.2, 0.1]) + 1),
                "modic": int(rng.choice(4, p=[0.7, 0.15, 0.1, 0.05])),
                "herniation": int(rng.rand() < 0.25),
                "bulging": int(rng.rand() < 0.4),
                "upper_endplate": int(rng.rand() < 0.2),
                "lower_endplate": int(rng.rand() < 0.2),
                "spondylolisthesis": int(rng.rand() < 0.1),
                "narrowing": int(rng.rand() < 0.3),
            })
    return recs


def main():
    import make_golden

    make_golden.import_reference()
    from spine_vision.training.datasets import stratification as ref

    recs = synthetic_records()
    patients = sorted(set(r["patient_key"] for r in recs))
    out = {"n_patients": len(patients), "record_seed": 3, "single": [], "single_labels": {}, "multilabel_matrix": {}}
    for label in ("pfirrmann", "modic", "herniation", "spondy"):
        out["single_labels"][label] = ref.get_patient_single_label(patients, recs, label).tolist()
    for labels in (["pfirrmann", "modic", "herniation"], ["bulging", "narrowing"]):
        out["multilabel_matrix"][",".join(labels)] = ref.get_patient_multilabel_matrix(patients, recs, labels).tolist()
    for label, val, test, seed in (("pfirrmann", 0.1, 0.1, 42), ("modic", 0.15, 0.1, 7), ("herniation", 0.2, 0.0, 1),
                                   ("pfirrmann", 0.0, 0.2, 5)):
        tr, va, te = ref.split_patients(patients, recs, [label], val, test, seed)
        out["single"].append({"label": label, "val": val, "test": test, "seed": seed,
                              "train": sorted(tr), "val_set": sorted(va), "test_set": sorted(te)})
    with open(os.path.join(HERE, "stratification.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote stratification.json")


if __name__ == "__main__":
    main()
