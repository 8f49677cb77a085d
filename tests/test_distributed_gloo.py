"""world_size-2 (and 3) data-parallel tests on CPU with the gloo backend: sharding of
ragged global batches, the all-gather of detections in rank order, and weight broadcast.
The per-rank compute is the oracle's torch-CPU forward (the product kernels need a GPU),
so these test exactly the distributed logic the GPU path uses (distributed.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vision_transformer_detector_amd import distributed as D

KW = dict(input_shape=(24, 24, 3), patch_size=8, embedding_dim=16, encoder_num_heads=2,
          encoder_key_dim=8, encoder_mlp_quantities=2, encoder_repeat_times=1,
          mlp_head_last_units=4, mlp_head_dense_layers_quantity=2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_batch():
    for b in (0, 1, 5, 8, 256, 2049):
        for w in (1, 2, 3, 8):
            spans = [D.shard_bounds(b, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == b
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [s1 - s0 for s0, s1 in spans]
            assert max(sizes) - min(sizes) <= 1 and max(sizes) == D.max_shard(b, w) or b == 0
    with pytest.raises(ValueError):
        D.shard_bounds(4, 2, 2)


def _worker(rank, world, port, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import vtd_numpy as V
        from oracle.vtd_torch_cpu import TorchCpuDetector
        w = V.init_weights(seed=1, **KW)
        det = TorchCpuDetector(w, **KW)
        x = torch.from_numpy(V.synthetic_images(batch, KW["input_shape"], seed=2))
        dp = D.DataParallelDetector(forward_fn=lambda t: det(t))
        out = dp(x)
        # inputs already resident per rank
        s0, s1 = D.shard_bounds(batch, rank, world)
        out2 = dp.run_local(x[s0:s1], batch)

        class FakeModel:                       # broadcast_weights contract
            device = torch.device("cpu")

            def __init__(self, seed):
                self.w = {"a/kernel": np.full((3, 2), float(seed), np.float32),
                          "a/bias": np.arange(2, dtype=np.float32) + seed}

            def weight_names(self):
                return list(self.w)

            def get_weight_dict(self):
                return dict(self.w)

            def set_weights(self, d):
                self.w = {k: np.asarray(v) for k, v in d.items()}

        fm = FakeModel(seed=rank + 10)
        D.broadcast_weights(fm, src=0)
        q.put((rank, out.numpy(), out2.numpy(), fm.w["a/kernel"].copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 6), (2, 5), (3, 4)])
def test_data_parallel_gather_matches_single_process(world, batch):
    from oracle import vtd_numpy as V
    from oracle.vtd_torch_cpu import TorchCpuDetector
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = V.init_weights(seed=1, **KW)
    x = V.synthetic_images(batch, KW["input_shape"], seed=2)
    full = TorchCpuDetector(w, **KW)(x).numpy()
    for rank, out, out2, kern in res:
        assert out.shape == (batch, 17, 6)
        np.testing.assert_array_equal(out, out2)
        np.testing.assert_allclose(out, full, rtol=0, atol=1e-6)
        assert (kern == 10.0).all()            # everyone now holds rank 0's weights


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_launches_ranks_itself(world):
    """`python bench.py --gpus N` with no launcher starts N rank processes (the driver's
    command shape); --dry-run rehearses the rendezvous, max-over-ranks timing and the
    all-gather on gloo.  rank 0 prints one JSON line with n_gpus = N."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world),
                        "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "5"],
                       capture_output=True, text=True, timeout=180, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["global_batch"] == 5 * world
    assert out["gather_rank_order_ok"] is True
    # correctness evidence of the N > 1 line: each rank finds its own shard in the gather
    assert out["gather_ok"] is True
    assert 0 <= out["rank_ms_min"] <= out["rank_ms_max"]


@pytest.mark.parametrize("world", [2, 8])
def test_bench_under_the_drivers_launcher(world):
    """The driver's N > 1 command shape: `python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...`
    (WORLD_SIZE / RANK from the launcher), rehearsed with --dry-run on gloo."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", str(world), "--master-addr", "127.0.0.1",
                        "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", str(world), "--dry-run", "--steps", "3", "--warmup", "1",
                        "--batch", "5"], capture_output=True, text=True, timeout=240, env=env,
                       cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["global_batch"] == 5 * world
    assert out["gather_rank_order_ok"] is True and out["gather_ok"] is True


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4",
                        "--dry-run"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "disagrees" in r.stderr
