"""CPU, row f4: patient-stratified splits (spine_vision/training/datasets/stratification.py).

Pinned: the per-patient labels, the multilabel matrix and the single-label splits against outputs of the
reference's own module (tests/golden/stratification.json, made by make_strat_golden.py).  The multilabel
split restates iterstrat's iterative stratification, which is absent here: parity UNPINNED, so its tests
check the algorithm's invariants instead."""

import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from make_strat_golden import synthetic_records  # noqa: E402
from spine_vision_amd.training.datasets import stratification as st  # noqa: E402

GOLD = json.load(open(os.path.join(HERE, "golden", "stratification.json")))


def _data():
    recs = synthetic_records(seed=GOLD["record_seed"])
    return sorted(set(r["patient_key"] for r in recs)), recs


def test_patient_labels_match_reference():
    patients, recs = _data()
    assert len(patients) == GOLD["n_patients"]
    for label, ref in GOLD["single_labels"].items():
        assert st.get_patient_single_label(patients, recs, label).tolist() == ref, label
    for key, ref in GOLD["multilabel_matrix"].items():
        assert st.get_patient_multilabel_matrix(patients, recs, key.split(",")).tolist() == ref, key


def test_single_label_splits_match_reference():
    patients, recs = _data()
    for case in GOLD["single"]:
        tr, va, te = st.split_patients(patients, recs, [case["label"]], case["val"], case["test"], case["seed"])
        assert sorted(tr) == case["train"] and sorted(va) == case["val_set"] and sorted(te) == case["test_set"], case


@pytest.mark.parametrize("seed", [0, 1, 42])
def test_multilabel_split_invariants(seed):
    patients, recs = _data()
    labels = ["pfirrmann", "modic", "herniation"]
    tr, va, te = st.split_patients(patients, recs, labels, 0.15, 0.15, seed)
    assert not (tr & va) and not (tr & te) and not (va & te)
    assert tr | va | te == set(patients)
    n = len(patients)
    # iterative stratification trades exact fold sizes for label balance (a patient positive for several
    # columns goes where its rarest label is most wanted), so sizes are only approximately 15 %
    assert abs(len(te) - 0.15 * n) <= 0.1 * n and abs(len(va) - 0.15 * n) <= 0.1 * n
    # every label column keeps (about) its share in each split: iterative stratification hands each
    # positive patient to the split that still wants the most of that label
    m = st.get_patient_multilabel_matrix(patients, recs, labels)
    idx = {p: i for i, p in enumerate(patients)}
    tot = m.sum(0)
    for part, share in ((te, 0.15), (va, 0.15)):
        got = m[[idx[p] for p in part]].sum(0)
        assert np.all(np.abs(got - share * tot) <= 2.0 + 0.1 * tot), (got, share * tot)
    # deterministic in the seed
    assert st.split_patients(patients, recs, labels, 0.15, 0.15, seed) == (tr, va, te)


def test_iterative_stratification_small_example():
    """Hand-checkable case: 2 labels, 8 samples, folds 3/4 : 1/4."""
    y = np.array([[1, 0], [1, 0], [1, 0], [1, 0], [0, 1], [0, 1], [0, 1], [0, 1]], dtype=bool)
    tr, te = st.multilabel_stratified_shuffle_split(y, 0.25, seed=3)
    assert len(te) == 2 and len(tr) == 6
    assert y[te].sum(0).tolist() == [1, 1]  # one positive of each label in the test fold
