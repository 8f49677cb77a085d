"""Pins the CPU metric restatement (oracle/vtd_map.py) to the reference's own known-answer
tests (testcases_vision_transformer_detector.py:11-734)."""
import numpy as np
import pytest

from oracle import vtd_map as M
from tests.map_cases import CASES, case_3, case_4, case_5_2


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_map_known_answers(name):
    y, p, expected = CASES[name]()
    m = M.MeanAveragePrecision()
    m.update_state(y, p)
    # the reference asserts float32 equality (assertEqual on a float32 tensor)
    assert m.result() == np.float32(expected), (name, m.result(), expected)


def test_oracle_reset_state():
    """tests.py:713-734: after reset every state is zero and result() is 0."""
    m = M.MeanAveragePrecision()
    y, p, _ = CASES["11_two_categories_two_images"]()
    m.update_state(y, p)
    assert m.result() > 0
    m.reset_state()
    assert not m.latest_positive_bboxes.any()
    assert not m.labels_quantity_per_image.any()
    assert not m.showed_up_classes.any()
    assert m.result() == 0


def test_oracle_iou_values_of_the_kats():
    """The IoUs the reference tests print: 0.64 (test 3), 0.49 (test 4), 0.9801 (test 5.2)."""
    y, p, _ = case_3()
    assert abs(M.iou_calculator(y, p).max() - 0.64) < 1e-6
    y, p, _ = case_4()
    assert abs(M.iou_calculator(y, p).max() - 0.49) < 1e-6
    y, p, _ = case_5_2()
    iou = M.iou_calculator(np.broadcast_to(y[0, 1], p[0].shape), p[0])
    assert abs(iou[2] - 0.9801) < 1e-6 and iou[1] == np.float32(1.0)


def test_oracle_thresholds_float32():
    t = M.MeanAveragePrecision.thresholds()
    assert len(t) == 10 and t[0] == np.float32(0.5) and t[-1] == np.float32(0.95)
    assert all(a < b for a, b in zip(t, t[1:]))


def test_oracle_latest_related_images_window():
    """Only the LATEST_RELATED_IMAGES (3) most recent related images of a category are
    kept (vtd.py:1538-1544, 1856-1862): four updates, newest first in slot 0."""
    m = M.MeanAveragePrecision()
    for k in range(4):
        y, p, _ = CASES["1_one_image_one_category"]()
        y[0, 1, 4:] = 10 + k          # distinct sizes per image
        m.update_state(y, y)
    assert m.labels_quantity_per_image[79].tolist() == [1, 1, 1]
    assert np.allclose(m.latest_positive_bboxes[79, :, -1], 1.0, atol=1e-6)
    assert not m.latest_positive_bboxes[79, :, :-1].any()


def test_oracle_scenario_c_pads_at_end_and_scenario_d_at_front():
    m = M.MeanAveragePrecision()
    y = np.full((1, 10, 6), -8.0, np.float32)
    y[..., 0] = 0
    p = np.zeros((1, 10, 6), np.float32)
    p[0, 3] = (0.9, 5.2, 100, 100, 10, 10)      # category 5 predicted, not labelled
    m.update_state(y, p)
    e = m.latest_positive_bboxes[5, 0]
    assert e[0, 0] == M._confidence(np.float32(5.2)) and not e[1:].any()
    assert m.showed_up_classes[5] and m.labels_quantity_per_image[5, 0] == 0
    y, p, _ = CASES["1_one_image_one_category"]()
    m.update_state(y, p)
    e = m.latest_positive_bboxes[79, 0]
    assert e[-1].tolist() == [1.0, 1.0] and not e[:-1].any()
