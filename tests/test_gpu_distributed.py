"""Data parallelism on the device: DataParallelDetector on the real model
through an RCCL ("nccl") process group -- world size 1 on the one-GPU test box (the
world-2/3 sharding logic is covered on CPU by test_distributed_gloo.py; 8-GPU runs are the
driver's) -- and the collective itself, all_gather_into_tensor on device memory."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import vtd_numpy as V
from vision_transformer_detector_amd import distributed as D

pytestmark = pytest.mark.gpu

KW = dict(input_shape=(40, 36, 3), patch_size=8, embedding_dim=24, encoder_num_heads=3,
          encoder_key_dim=10, encoder_mlp_quantities=3, encoder_repeat_times=2,
          mlp_head_last_units=8, mlp_head_dense_layers_quantity=3)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_world1(cuda):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda)
    yield
    dist.destroy_process_group()


def test_data_parallel_detector_over_rccl(cuda, nccl_world1):
    import vision_transformer_detector_amd as vtd
    assert dist.get_backend() == "nccl"
    w = V.init_weights(seed=5, **KW)
    x = V.synthetic_images(5, KW["input_shape"], seed=6)
    expect = V.transform_predictions(V.forward(w, x, **KW))
    model = vtd.create_vision_transformer_detector(**KW, dtype="float32", device=cuda)
    model.set_weights(w)
    dets = D.DataParallelDetector(model)(torch.from_numpy(x).to(cuda))
    assert dets.is_cuda and tuple(dets.shape) == (5, 17, 6)
    np.testing.assert_allclose(dets.cpu().numpy(), expect, rtol=1e-3, atol=1e-3 * 608)
    # the path's collective on device memory (RCCL all_gather_into_tensor), padded shard
    padded = torch.zeros((8, 17, 6), device=cuda)
    padded[:5] = dets
    out = D.gather_padded(padded)
    torch.cuda.synchronize()
    assert torch.equal(out, padded)
    assert torch.equal(D.all_gather_detections(dets, 5), dets)
