"""CPU restatement of the reference's detection metric (TEST INFRASTRUCTURE ONLY).

Restates `iou_calculator` (vision_transformer_detector.py:761-875) and
`MeanAveragePrecision` (vision_transformer_detector.py:1268-2060) in float32 scalar
arithmetic, in the reference's operation order, so the HIP metric kernels
(vision_transformer_detector_amd/csrc/vtd_metrics.hip) can be checked bit-for-bit.

Parity PINNED: the 12 known-answer tests of
testcases_vision_transformer_detector.py:11-734 (AP = 1, 1, 0.3, 0, 0, 0.75, 0, 1, 0.375,
0.5, 0.5, 0.6875, and the reset state) are restated in tests/test_map_kat.py and must hold
for this module and for the GPU path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.

Conventions of the reference kept here (file:line):
  * a box row is (objectness, class, x, y, height, width); labels mark empty rows with
    class -8 (vtd.py:1315-1325);
  * tf.round is round-half-to-even (np.rint);
  * tf.argsort / tf.sort are top_k based: ties keep the lower index first (the 0.75 KAT
    of test 5.2 depends on it);
  * tf.experimental.numpy.isclose: |a-b| <= 1e-8 + 1e-5 |b|;
  * tf.linspace(0.5, 0.95, 10) in float32: start + i * step, last element = stop.
"""
from __future__ import annotations

import numpy as np

F = np.float32
CLASSES = 80                    # vtd.py:20
EPSILON = F(1e-8)               # vtd.py:24
LATEST_RELATED_IMAGES = 3       # vtd.py:32
BBOXES_PER_IMAGE = 14           # vtd.py:37
OBJECTNESS_THRESHOLD = F(0.5)   # vtd.py:41
CLASSIFICATION_CONFIDENCE_THRESHOLD = F(0.5)  # vtd.py:43


def iou_calculator(label_bbox, prediction_bbox):
    """vtd.py:761-875, elementwise over the leading dims; boxes are (x, y, h, w) in the
    last 4 channels.  The sort-of-4-edges intersection equals min(right) - max(left) for
    intersecting boxes, and 0 otherwise (vtd.py:839-854)."""
    lb = np.asarray(label_bbox, F)
    pb = np.asarray(prediction_bbox, F)
    two = F(2)
    ll, lr = lb[..., -4] - lb[..., -1] / two, lb[..., -4] + lb[..., -1] / two
    pl, pr = pb[..., -4] - pb[..., -1] / two, pb[..., -4] + pb[..., -1] / two
    lt, lbo = lb[..., -3] - lb[..., -2] / two, lb[..., -3] + lb[..., -2] / two
    pt, pbo = pb[..., -3] - pb[..., -2] / two, pb[..., -3] + pb[..., -2] / two
    cond = (ll < pr) & (lr > pl) & (lt < pbo) & (lbo > pt)
    ih = np.where(cond, np.minimum(lbo, pbo) - np.maximum(lt, pt), F(0))
    iw = np.where(cond, np.minimum(lr, pr) - np.maximum(ll, pl), F(0))
    inter = (ih * iw).astype(F)
    union = (pb[..., -1] * pb[..., -2] + lb[..., -1] * lb[..., -2] - inter).astype(F)
    return (inter / (union + EPSILON)).astype(F)


def _isclose(a, b):
    return abs(F(a) - F(b)) <= F(1e-8) + F(1e-5) * abs(F(b))


def _confidence(cls):
    """(0.5 - |c - round(c)|) / 0.5 (vtd.py:1367-1376)."""
    c = F(cls)
    return F((F(0.5) - abs(c - F(np.rint(c)))) / F(0.5))


def _stable_desc(values):
    """Indices sorting `values` descending, ties lower index first (tf.argsort)."""
    return sorted(range(len(values)), key=lambda i: (-float(values[i]), i))


def _positives(pred):
    """vtd.py:1458-1475: positive mask and per-row category (-8 on negatives)."""
    pos, cat = [], []
    for row in pred:
        c = F(row[1])
        ok = bool(F(row[0]) > OBJECTNESS_THRESHOLD and
                  _confidence(c) > CLASSIFICATION_CONFIDENCE_THRESHOLD)
        pos.append(ok)
        cat.append(F(np.rint(c)) if ok else F(-8))
    return pos, cat


def image_category_record(label, pred, category):
    """One image x one category of update_state (vtd.py:1480-1852).

    Returns (related, labels_quantity, entries[BBOXES_PER_IMAGE][2]) where `related` is
    scenario b/c/d and entries are (class confidence, IoU) pairs."""
    P = BBOXES_PER_IMAGE
    label = np.asarray(label, F)
    pred = np.asarray(pred, F)
    pos, pcat = _positives(pred)
    lab_mask = [_isclose(row[1], category) for row in label]
    pred_mask = [_isclose(pcat[i], category) for i in range(len(pred))]
    any_l, any_p = any(lab_mask), any(pred_mask)
    if not (any_l or any_p):
        return False, 0, None
    count = int(sum(lab_mask))
    if not any_p:                                       # scenario b (vtd.py:1552-1556)
        return True, count, [(F(0), F(0))] * P
    if not any_l:                                       # scenario c (vtd.py:1560-1621)
        confs = [_confidence(pred[i][1]) for i in range(len(pred)) if pred_mask[i]]
        if len(confs) < P:
            confs = confs + [F(0)] * (P - len(confs))
        else:
            confs = sorted(confs, key=lambda v: -float(v))[:P]
        return True, count, [(c, F(0)) for c in confs]
    # scenario d (vtd.py:1625-1852)
    neg = np.full(4, F(-8))
    boxes = [pred[i][-4:].copy() if pred_mask[i] else neg.copy() for i in range(len(pred))]
    labs = [label[i][-4:] for i in range(len(label)) if lab_mask[i]]
    areas = [F(b[-1] * b[-2]) for b in labs]
    order = sorted(range(len(labs)), key=lambda i: (float(areas[i]), i))   # stable asc
    entries = [(F(0), F(0))] * P
    new = 0
    for li in order:
        ious = iou_calculator(np.broadcast_to(labs[li], (len(boxes), 4)), np.stack(boxes))
        mx = F(ious.max())
        if mx > F(0.5):
            new += 1
            hit = [j for j in range(len(boxes)) if _isclose(ious[j], mx)]
            conf = _confidence(pred[hit[0]][1])
            entries = (entries + [(conf, mx)])[-P:]
            for j in hit:
                boxes[j] = neg.copy()
        if new == P:
            break
    left = [i for i in range(len(boxes)) if pred_mask[i] and bool(np.all(boxes[i] >= 0))]
    # vtd.py:1767-1768 keeps a row when all 4 box values are >= 0 (removed rows are -8);
    # rows of other categories are -8 too, so `pred_mask` only restates that.
    if left and new < P:
        confs = [_confidence(pred[i][1]) for i in left]
        if new + len(confs) > P:
            confs = sorted(confs, key=lambda v: -float(v))[:P - new]
        entries = (entries + [(c, F(0)) for c in confs])[-P:]
    return True, count, entries


class MeanAveragePrecision:
    """vtd.py:1268-2060 restated; state layout identical to the reference's Variables."""

    def __init__(self):
        self.reset_state()

    def reset_state(self):                              # vtd.py:2052-2060
        self.latest_positive_bboxes = np.zeros(
            (CLASSES, LATEST_RELATED_IMAGES, BBOXES_PER_IMAGE, 2), F)
        self.labels_quantity_per_image = np.zeros((CLASSES, LATEST_RELATED_IMAGES), F)
        self.showed_up_classes = np.zeros(CLASSES, bool)

    def update_state(self, y_true, y_pred):
        """vtd.py:1310-1862 with use_transform_predictions=False (the caller decodes)."""
        y_true = np.asarray(y_true, F)
        y_pred = np.asarray(y_pred, F)
        for b in range(y_true.shape[0]):
            cl = y_true[b, :, 1]
            for c in cl[cl >= 0]:                       # vtd.py:1347-1352
                if 0 <= int(c) < CLASSES:
                    self.showed_up_classes[int(c)] = True
            pos, pcat = _positives(y_pred[b])
            for i, ok in enumerate(pos):                # vtd.py:1359-1392
                if ok and 0 <= int(pcat[i]) < CLASSES:
                    self.showed_up_classes[int(pcat[i])] = True
            for c in range(CLASSES):
                rel, cnt, ent = image_category_record(y_true[b], y_pred[b], c)
                if not rel:
                    continue
                self.labels_quantity_per_image[c, 1:] = self.labels_quantity_per_image[c, :-1]
                self.labels_quantity_per_image[c, 0] = cnt
                self.latest_positive_bboxes[c, 1:] = self.latest_positive_bboxes[c, :-1].copy()
                self.latest_positive_bboxes[c, 0] = np.array(ent, F)

    @staticmethod
    def thresholds():
        """tf.linspace(0.5, 0.95, num=10) in float32 (TF LinSpace kernel)."""
        start, stop = F(0.5), F(0.95)
        step = F((stop - start) / F(9))
        return [F(start + step * F(i)) for i in range(9)] + [stop]

    def category_ap(self, category, thr):
        """vtd.py:1886-2007 for one category and one IoU threshold."""
        ent = self.latest_positive_bboxes[category].reshape(-1, 2)
        rp = [F(1)]
        tp, fp = F(0), F(0)
        for i in _stable_desc(ent[:, 0]):
            conf, iou = F(ent[i, 0]), F(ent[i, 1])
            if conf > 0:
                if iou > thr:
                    tp = F(tp + F(1))
                    rp.append(F(tp / F(tp + fp)))
                else:
                    fp = F(fp + F(1))
                    rp[-1] = F(tp / F(tp + fp))
        lq = F(np.sum(self.labels_quantity_per_image[category], dtype=F))
        if lq > 0:
            h = F(F(1) / lq)
            if len(rp) - 1 == 0:
                return F(0)
            acc = F(0)
            for i in range(len(rp) - 1):
                acc = F(acc + F(rp[i] + rp[i + 1]))
            return F(F(acc * h) / F(2))
        return F(0)

    def per_iou(self):
        out = []
        for thr in self.thresholds():
            aps = [self.category_ap(c, thr) for c in range(CLASSES) if self.showed_up_classes[c]]
            if aps:
                s = F(0)
                for a in aps:
                    s = F(s + a)
                out.append(F(s / F(len(aps))))
            else:
                out.append(F(0))
        return out

    def result(self):                                   # vtd.py:1865-2049
        s = F(0)
        for a in self.per_iou():
            s = F(s + a)
        return F(s / F(10))
