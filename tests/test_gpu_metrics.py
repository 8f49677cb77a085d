"""Device metric (vtd_map_update / vtd_map_result / vtd_iou) against the reference's
known answers (testcases_vision_transformer_detector.py:11-734) and, bit for bit, against
the float32 CPU restatement (oracle/vtd_map.py) on seeded random batches."""
import numpy as np
import pytest
import torch

from oracle import vtd_map as M
from oracle import vtd_numpy as V
from tests.map_cases import CASES, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vtd(cuda):
    import vision_transformer_detector_amd as m
    return m


@pytest.mark.parametrize("name", sorted(CASES))
def test_map_known_answers(vtd, cuda, name):
    y, p, expected = CASES[name]()
    m = vtd.MeanAveragePrecision()
    m.update_state(torch.from_numpy(y), torch.from_numpy(p), use_transform_predictions=False)
    got = m.result().item()
    assert np.float32(got) == np.float32(expected), (name, got, expected)


def test_map_reset_state(vtd, cuda):
    """tests.py:713-734."""
    m = vtd.MeanAveragePrecision()
    y, p, _ = CASES["11_two_categories_two_images"]()
    m.update_state(y, p, use_transform_predictions=False)
    assert m.result().item() > 0
    m.reset_state()
    assert not m.latest_positive_bboxes.any()
    assert not m.labels_quantity_per_image.any()
    assert not m.showed_up_classes.any()
    assert m.result().item() == 0


def _compare_state(m, ref):
    np.testing.assert_array_equal(m.latest_positive_bboxes.cpu().numpy(), ref.latest_positive_bboxes)
    np.testing.assert_array_equal(m.labels_quantity_per_image.cpu().numpy(),
                                  ref.labels_quantity_per_image)
    np.testing.assert_array_equal(m.showed_up_classes.cpu().numpy(), ref.showed_up_classes)


@pytest.mark.parametrize("seed,classes", [(0, (0, 80)), (1, (0, 3)), (2, (77, 80)), (3, (0, 1))])
def test_map_random_batches_match_oracle(vtd, cuda, seed, classes):
    """Several batch updates (ragged object counts, duplicate predictions, classes near
    the rounding boundary, >14 boxes of one class so the sort/truncate branches run):
    the whole state and every per-threshold AP must equal the restatement exactly."""
    rng = np.random.default_rng(seed)
    m, ref = vtd.MeanAveragePrecision(), M.MeanAveragePrecision()
    for step, batch in enumerate((5, 1, 9)):
        y, p = random_batch(rng, batch, boxes=17, classes=classes)
        m.update_state(y, p, use_transform_predictions=False)
        ref.update_state(y, p)
        _compare_state(m, ref)
        got = m.average_precision_per_iou().cpu().numpy()
        np.testing.assert_array_equal(got, np.array(ref.per_iou(), np.float32))
        assert m.result().item() == ref.result()


def test_map_batch_larger_than_block(vtd, cuda):
    """More images than threads per block: the latest-3 search must still pick the
    newest related images of each class."""
    rng = np.random.default_rng(7)
    y, p = random_batch(rng, 600, boxes=8, classes=(0, 4))
    m, ref = vtd.MeanAveragePrecision(), M.MeanAveragePrecision()
    m.update_state(y, p, use_transform_predictions=False)
    ref.update_state(y, p)
    _compare_state(m, ref)
    assert m.result().item() == ref.result()


def test_map_update_from_logits(vtd, cuda):
    """Default use_transform_predictions=True: logits decode on the device first."""
    rng = np.random.default_rng(3)
    y, _ = random_batch(rng, 4, boxes=17)
    logits = rng.normal(0, 2, (4, 17, 6)).astype(np.float32)
    m = vtd.MeanAveragePrecision()
    m.update_state(y, logits)
    dec = vtd.transform_predictions(torch.from_numpy(logits).cuda()).cpu().numpy()
    ref = M.MeanAveragePrecision()
    ref.update_state(y, dec)
    _compare_state(m, ref)
    assert np.abs(dec - V.transform_predictions(logits)).max() < 1e-3


def test_map_rejects_bad_shapes(vtd, cuda):
    m = vtd.MeanAveragePrecision()
    with pytest.raises(ValueError):
        m.update_state(np.zeros((2, 10, 6)), np.zeros((2, 11, 6)))
    with pytest.raises(ValueError):
        m.update_state(np.zeros((1, 65, 6)), np.zeros((1, 65, 6)))
    m.update_state(np.zeros((0, 10, 6)), np.zeros((0, 10, 6)), use_transform_predictions=False)
    assert m.result().item() == 0


def test_iou_calculator_matches_oracle(vtd, cuda):
    rng = np.random.default_rng(11)
    lab = np.concatenate([rng.uniform(-10, 620, (4096, 2)), rng.uniform(-5, 300, (4096, 2))], 1)
    pred = lab + rng.normal(0, 20, lab.shape)
    lab, pred = lab.astype(np.float32), pred.astype(np.float32)
    got = vtd.iou_calculator(lab, pred).cpu().numpy()
    np.testing.assert_array_equal(got, M.iou_calculator(lab, pred))
    # 6-channel rows (boxes in the last 4) and the KAT values
    y = np.zeros((2, 6), np.float32)
    y[:, 2:] = (10.2, 10.2, 10, 10)
    p = y.copy()
    p[0, 2:] = (9.5, 9.5, 8, 8)
    p[1, 2:] = (9.5, 9.5, 7, 7)
    got = vtd.iou_calculator(torch.from_numpy(y).cuda(), torch.from_numpy(p).cuda()).cpu().numpy()
    assert abs(got[0] - 0.64) < 1e-6 and abs(got[1] - 0.49) < 1e-6
