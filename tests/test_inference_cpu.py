"""Row f2 host logic of the inference consumer (spine_vision_amd.inference): the min-max to uint8 of
the reference's ``normalize_to_uint8`` (spine_vision/io/__init__.py:15-30) against the fixture the
reference itself produced (tests/golden/make_golden_predict.py)."""

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
GOLD = json.load(open(os.path.join(HERE, "golden", "predict_ivd.json")))


def test_normalize_to_uint8_matches_reference():
    from make_golden_predict import test_images

    from spine_vision_amd.inference import normalize_to_uint8

    for im, g in zip(test_images(), GOLD["images"]):
        u8 = normalize_to_uint8(im)
        assert u8.dtype == np.uint8 and u8.shape == im.shape
        assert int(u8.astype(np.int64).sum()) == g["u8_sum"]
        assert int((u8.astype(np.int64) ** 2).sum()) == g["u8_sq"]
    # a constant slice is cast as is (no division by a zero range)
    c = np.full((4, 5), 7.9, dtype=np.float32)
    assert np.array_equal(normalize_to_uint8(c), np.full((4, 5), 7, dtype=np.uint8))
