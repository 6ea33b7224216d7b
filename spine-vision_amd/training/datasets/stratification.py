"""Patient-level stratified train/val/test splits for the classification datasets (row f4 of the scope
table) -- drop-in for spine_vision/training/datasets/stratification.py:15-307.

* Single target label (stratification.py:144-206): sklearn ``StratifiedShuffleSplit`` on each patient's
  largest label value, test split first, then val on the remainder with val/(1 - test) -- the same calls
  as the reference, so the same patients land in the same splits.
* Several target labels (stratification.py:209-270): the reference calls iterstrat's
  ``MultilabelStratifiedShuffleSplit`` (iterstrat is not installed here and not vendored by the
  reference).  ``multilabel_stratified_shuffle_split`` below restates that published algorithm --
  Sechidis et al. 2011 iterative stratification as iterstrat implements it: shuffle, then repeatedly take
  the label with the fewest remaining positive patients and hand each of them to the split that still
  wants the most of that label (ties: the split wanting the most patients, then random), all-negative
  patients last to whichever split is emptiest.  Parity with iterstrat itself is UNPINNED (no fixture in
  the reference holds its output); the tests check the algorithm's invariants.
"""

from __future__ import annotations

import numpy as np
from sklearn.model_selection import StratifiedShuffleSplit

from ...core.tasks import get_task

_RECORD_KEY = {
    "pfirrmann": "pfirrmann",
    "modic": "modic",
    "herniation": "herniation",
    "bulging": "bulging",
    "upper_endplate": "upper_endplate",
    "lower_endplate": "lower_endplate",
    "spondy": "spondylolisthesis",
    "narrowing": "narrowing",
}


def get_patient_single_label(patients: list[str], records: list[dict], label: str) -> np.ndarray:
    """Largest value of ``label`` over each patient's IVD levels (stratification.py:15-64)."""
    key = _RECORD_KEY.get(label, label)
    vals: dict[str, list[int]] = {p: [] for p in patients}
    for r in records:
        if r["patient_key"] in vals:
            vals[r["patient_key"]].append(r[key])
    return np.array([max(vals[p]) if vals[p] else 0 for p in patients])


def get_patient_multilabel_matrix(patients: list[str], records: list[dict], target_labels: list[str]) -> np.ndarray:
    """[n_patients, columns] 0/1 matrix: one column per class of a multiclass label (pfirrmann classes are
    1-indexed in the records), one per binary label, OR-ed over the IVD levels (stratification.py:67-141)."""
    columns: list[tuple[str, int | None]] = []
    for label in target_labels:
        t = get_task(label)
        columns += [(label, c) for c in range(t.num_classes)] if t.is_multiclass else [(label, None)]
    row = {p: i for i, p in enumerate(patients)}
    m = np.zeros((len(patients), len(columns)), dtype=np.float32)
    for r in records:
        i = row.get(r["patient_key"])
        if i is None:
            continue
        for j, (label, c) in enumerate(columns):
            v = r[_RECORD_KEY.get(label, label)]
            if c is None:
                hit = v > 0
            else:
                hit = v == c + 1 if label == "pfirrmann" else v == c
            if hit:
                m[i, j] = 1.0
    return m


def _iterative_stratification(labels: np.ndarray, r: np.ndarray, rng: np.random.RandomState) -> np.ndarray:
    """Fold index per sample for fold proportions ``r`` (iterative stratification)."""
    n = labels.shape[0]
    folds = np.zeros(n, dtype=int)
    want = r * n  # desired samples per fold
    want_lab = np.outer(r, labels.sum(axis=0))  # desired positives per (fold, label)
    todo = np.ones(n, dtype=bool)
    while todo.any():
        remaining = labels[todo].sum(axis=0)
        if remaining.sum() == 0:  # only all-negative samples left: fill the emptiest folds
            for i in np.where(todo)[0]:
                f = np.where(want == want.max())[0]
                f = f[rng.choice(f.shape[0])] if f.shape[0] > 1 else f[0]
                folds[i] = f
                want[f] -= 1
            break
        lab = np.where(remaining == remaining[np.nonzero(remaining)].min())[0]
        lab = lab[rng.choice(lab.shape[0])] if lab.shape[0] > 1 else lab[0]
        for i in np.where(np.logical_and(labels[:, lab] > 0, todo))[0]:
            lf = want_lab[:, lab]
            f = np.where(lf == lf.max())[0]
            if f.shape[0] > 1:
                t = np.where(want[f] == want[f].max())[0]
                f = f[t]
                f = f[rng.choice(t.shape[0])] if t.shape[0] > 1 else f[0]
            else:
                f = f[0]
            folds[i] = f
            todo[i] = False
            want_lab[f, labels[i] > 0] -= 1
            want[f] -= 1
    return folds


def multilabel_stratified_shuffle_split(labels: np.ndarray, test_size: float, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """(train_idx, test_idx) of one multilabel stratified shuffle split (test share ``test_size``)."""
    n = labels.shape[0]
    n_test = int(np.ceil(test_size * n))
    n_train = n - n_test
    rng = np.random.RandomState(seed)
    perm = np.arange(n)
    rng.shuffle(perm)
    folds = _iterative_stratification(labels[perm] > 0, np.array([n_train, n_test], dtype=float) / n, rng)
    is_test = folds[np.argsort(perm)] == 1
    return np.where(~is_test)[0], np.where(is_test)[0]


def _two_stage(patients: list[str], labels: np.ndarray, val_ratio: float, test_ratio: float, seed: int, split_fn):
    arr = np.array(patients)
    if test_ratio > 0:
        tv, te = split_fn(arr, labels, test_ratio, seed)
        test, arr, labels = set(arr[te]), arr[tv], labels[tv]
    else:
        test = set()
    if val_ratio > 0:
        tr, va = split_fn(arr, labels, val_ratio / (1 - test_ratio), seed)
        return set(arr[tr]), set(arr[va]), test
    return set(arr), set(), test


def _sklearn_split(arr, labels, size, seed):
    return next(StratifiedShuffleSplit(n_splits=1, test_size=size, random_state=seed).split(arr, labels))


def _ml_split(arr, labels, size, seed):
    return multilabel_stratified_shuffle_split(labels, size, seed)


def split_patients_single_label(patients, records, target_label, val_ratio, test_ratio, seed):
    return _two_stage(patients, get_patient_single_label(patients, records, target_label), val_ratio, test_ratio,
                      seed, _sklearn_split)


def split_patients_multilabel(patients, records, target_labels, val_ratio, test_ratio, seed):
    return _two_stage(patients, get_patient_multilabel_matrix(patients, records, target_labels), val_ratio,
                      test_ratio, seed, _ml_split)


def split_patients(patients: list[str], records: list[dict], target_labels: list[str], val_ratio: float,
                   test_ratio: float, seed: int) -> tuple[set[str], set[str], set[str]]:
    """Train/val/test patient sets (stratification.py:273-307): multilabel iterative stratification for
    two or more target labels, sklearn single-label stratification otherwise."""
    if len(target_labels) > 1:
        return split_patients_multilabel(patients, records, target_labels, val_ratio, test_ratio, seed)
    return split_patients_single_label(patients, records, target_labels[0], val_ratio, test_ratio, seed)
