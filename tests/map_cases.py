"""Known-answer cases of the reference's metric tests, restated as data.

Each case follows one test of testcases_vision_transformer_detector.py (TestMeanAveragePrecision,
lines 11-734): the label / prediction arrays it builds (shape (B, 10, 6), rows
(objectness, class, x, y, height, width), empty label rows (0, -8, -8, -8, -8, -8)) and the
mAP it asserts.  The predictions are already decoded (the reference calls update_state with
use_transform_predictions=False).
"""
import numpy as np

BOX = (1.0, 79.0, 10.2, 10.2, 10.0, 10.0)   # the reference's standard object (tests.py:68-73)


def empty(batch):
    a = np.full((batch, 10, 6), -8.0, np.float32)
    a[..., 0] = 0.0
    return a


def case_1():          # tests.py:49-89: label == prediction, one object
    y = empty(1)
    y[0, 1] = BOX
    return y, y.copy(), 1.0


def case_2():          # tests.py:91-142: two categories, label == prediction
    y = empty(1)
    y[0, 1] = BOX
    y[0, 2] = (1.0, 78.0, 9.5, 9.5, 5.0, 5.0)
    return y, y.copy(), 1.0


def case_3():          # tests.py:144-195: IoU 0.64 -> AP 0.3
    y = empty(1)
    y[0, 1] = BOX
    p = y.copy()
    p[..., -4:] = (9.5, 9.5, 8.0, 8.0)
    return y, p, 0.3


def case_4():          # tests.py:197-248: IoU 0.49 -> AP 0
    y = empty(1)
    y[0, 1] = BOX
    p = y.copy()
    p[..., -4:] = (9.5, 9.5, 7.0, 7.0)
    return y, p, 0.0


def case_5_1():        # tests.py:250-303: objectness 0.49 -> AP 0
    y = empty(1)
    y[0, 1] = BOX
    p = y.copy()
    p[0, 1, 0] = 0.49
    return y, p, 0.0


def case_5_2():        # tests.py:305-370: extra wrong prediction (obj 0.51) -> AP 0.75
    y = empty(1)
    y[0, 1] = BOX
    p = y.copy()
    p[0, 2, 0] = 0.51
    p[0, 2, 1] = 79.0
    p[0, 2, -4:] = (10.2, 10.2, 9.9, 9.9)
    return y, p, 0.75


def case_6():          # tests.py:372-426: class confidence 0.49 -> AP 0
    y = empty(1)
    y[0, 1] = BOX
    p = y.copy()
    p[0, 1, 1] = 79.255
    return y, p, 0.0


def case_7():          # tests.py:428-471: two images, label == prediction
    y = empty(2)
    y[0, 1] = BOX
    y[1, 5] = BOX
    return y, y.copy(), 1.0


def case_8():          # tests.py:473-530: second image IoU 0.49 -> AP 0.375
    y = empty(2)
    y[0, 1] = BOX
    y[1, 0] = BOX
    p = y.copy()
    p[1, 0, 1] = 79.001
    p[1, 0, -4:] = (9.5, 9.5, 7.0, 7.0)
    return y, p, 0.375


def case_9():          # tests.py:532-585: second image objectness 0.49 -> AP 0.5
    y = empty(2)
    y[0, 1] = BOX
    y[1, 0] = BOX
    p = y.copy()
    p[1, 0, 0] = 0.49
    return y, p, 0.5


def case_10():         # tests.py:587-641: second image class 79.3 -> AP 0.5
    y = empty(2)
    y[0, 1] = BOX
    y[1, 0] = BOX
    p = y.copy()
    p[1, 0, 1] = 79.3
    return y, p, 0.5


def case_11():         # tests.py:643-710: two categories x two images -> AP 0.6875
    y = empty(2)
    y[0, 1] = BOX
    y[0, 2] = BOX
    y[0, 2, 1] = 78.0
    y[1] = y[0]
    p = y.copy()
    p[0, 1, 1] = 79.005
    p[0, 1, -4:] = (9.5, 9.5, 7.0, 7.0)
    return y, p, 0.6875


CASES = {
    "1_one_image_one_category": case_1,
    "2_one_image_two_categories": case_2,
    "3_one_image_low_iou": case_3,
    "4_one_image_zero_ap": case_4,
    "5_1_one_image_low_objectness": case_5_1,
    "5_2_two_predictions_one_wrong": case_5_2,
    "6_low_classification_confidence": case_6,
    "7_two_images_one_category": case_7,
    "8_two_images_one_zero_ap": case_8,
    "9_one_objectness_below_threshold": case_9,
    "10_classification_confidence_below_threshold": case_10,
    "11_two_categories_two_images": case_11,
}


def random_batch(rng, batch, boxes=17, classes=(0, 80), jitter=True):
    """Seeded label / decoded-prediction pairs for GPU-vs-oracle fuzzing: labels with a
    random number of objects, predictions that perturb them (box jitter, class offset,
    objectness around the threshold) plus false positives and duplicates."""
    y = np.full((batch, boxes, 6), -8.0, np.float32)
    y[..., 0] = 0.0
    p = np.zeros((batch, boxes, 6), np.float32)
    lo, hi = classes
    for b in range(batch):
        n = int(rng.integers(0, boxes + 1))
        for i in range(n):
            w, h = rng.uniform(4, 200, 2)
            y[b, i] = (1.0, float(rng.integers(lo, hi)), rng.uniform(0, 608),
                       rng.uniform(0, 608), h, w)
        for i in range(boxes):
            if i < n and rng.random() < 0.8:
                src = y[b, i].copy()
                if jitter:
                    src[2:4] += rng.normal(0, 3, 2)
                    src[4:6] *= rng.uniform(0.7, 1.3, 2)
                src[1] += rng.uniform(-0.45, 0.45)
                src[0] = rng.uniform(0.3, 1.0)
                p[b, i] = src
            else:
                p[b, i] = (rng.uniform(0, 1), rng.uniform(lo - 0.5, hi - 0.5),
                           rng.uniform(0, 608), rng.uniform(0, 608), rng.uniform(2, 300),
                           rng.uniform(2, 300))
        if n >= 2 and rng.random() < 0.3:        # exact duplicate prediction (isclose tie)
            p[b, boxes - 1] = p[b, 0]
    return y, p
