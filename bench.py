"""Headline benchmark: images/s of the ViT-B/16 detector forward at batch 256 per GPU
(BASELINE.json metric), bf16 operands / fp32 accumulate, synthetic COCO-shaped batches.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--dtype bf16|f32|fp8]
                  [--preset vit_b16_224|vit_b16_640|vit_l16_384|c1]
  N > 1 either under a launcher (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE from env):
      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
  or standalone: `python bench.py --gpus N` starts the N rank processes itself (before
  anything touches the GPU) with MASTER_ADDR=127.0.0.1 and waits for them.
  --dry-run: the launcher and the all-gather on CPU (gloo), no GPU and no forward.

One step = one forward of B images per rank (images already resident in HBM) + the
device-side decode (transform_predictions) + the RCCL all-gather of the (B, 17, 6)
detections over all ranks (the path's only exchange; skipped at N = 1).
Prints ONE JSON line on rank 0; after the timed region every rank checks that the gathered
detections hold its own shard bit for bit (`gather_ok`) and reports its own time
(`rank_ms_min` / `rank_ms_max` over ranks).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

# Kernel arguments in device memory instead of host memory: every workgroup's first scalar
# loads then stay on the device (+1.8 % on the C2 forward, 20.16k vs 19.80k img/s, two
# interleaved rounds on one box, profiles/r04_dev_kernarg_ab.log).  Read by the HIP runtime
# when it initialises, so set before torch touches the GPU; a caller's own setting wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = {"bf16": 2516.6, "f32": 157.3,    # MI355X dense: 256 CU x 2.4 GHz (MICROARCH)
               "fp8": 5033.2,                    # block-scaled MX-fp8 MFMA: 2x bf16 per clock
               "bf16x3": 2516.6}                 # split-bf16: bf16 MFMA (3 products per FLOP)
HBM_PEAK_GBS = 8000.0


def letterbox_images(b, shape, gen, device):
    """U(-1, 1) NHWC images with -1 letterbox bands: a 640x480 COCO image resized with
    pad to a square (utils.py:438-447) keeps 3/4 of the rows."""
    h, w, c = shape
    x = torch.rand((b, h, w, c), generator=gen, device=device) * 2 - 1
    band = h // 8
    x[:, :band] = -1.0
    x[:, h - band:] = -1.0
    return x


def algorithmic_flops_per_image(kw, dims):
    """2 x MAC over every Dense / attention product as written in the reference
    (no padding), SURVEY.md §8d.  Returns (total, attention+MLP)."""
    n, d = dims.tokens, kw["embedding_dim"]
    h, dk = kw["encoder_num_heads"], kw["encoder_key_dim"]
    inner = h * dk
    patch = 2.0 * n * dims.patch_dim * d
    qkv = 2.0 * n * d * 3 * inner
    attn = 4.0 * h * n * n * dk
    out = 2.0 * n * inner * d
    mlp, k = 0.0, d
    for j in range(kw["encoder_mlp_quantities"]):
        mlp += 2.0 * n * k * dims.mlp_units[j]
        k = dims.mlp_units[j]
    L = kw["encoder_repeat_times"]
    head = 2.0 * n * d * 17
    k = n
    for j in range(dims.n_head):
        head += 2.0 * 17 * k * dims.head_units[j]
        k = dims.head_units[j]
    head += 2.0 * 17 * k * 6
    total = patch + L * (qkv + attn + out + mlp) + head
    return total, L * (qkv + attn + out + mlp)


def traffic_per_launch():
    """HBM bytes per GEMM launch from the rocprofv3 PMC passes committed under
    profiles/ (tools/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE, separate passes of
    this same bench command), or None when no such measurement exists."""
    p = os.path.join(ROOT, "profiles", "gemm_traffic_latest.json")
    try:
        j = json.load(open(p))
        return round(j["traffic_bytes_per_launch"]), j.get("source", "see the file")
    except (OSError, KeyError, ValueError):
        return None, None


def gemm_alg_bytes(kw, dims, b, rb=2):
    """Algorithmic bytes of one forward's GEMMs (each operand read once, output written
    once, residual read once), averaged per GEMM launch: the `traffic` yardstick.
    rb = bytes per residual-stream element (2: the bf16 stream of the bf16 / fp8 modes)."""
    rows, d = b * dims.tokens, kw["embedding_dim"]
    inner = kw["encoder_num_heads"] * kw["encoder_key_dim"]
    g = [(rows, d, dims.patch_dim, rb, False)]
    for _ in range(kw["encoder_repeat_times"]):
        g.append((rows, 3 * inner, d, 2, False))
        g.append((rows, d, inner, rb, True))
        k = d
        for j in range(kw["encoder_mlp_quantities"]):
            n = dims.mlp_units[j]
            last = j == kw["encoder_mlp_quantities"] - 1
            g.append((rows, n, k, rb if last else 2, last))
            k = n
    g.append((rows, 17, d, 2, False))
    hr, k = b * 17, dims.tokens
    for j in range(dims.n_head):
        g.append((hr, dims.head_units[j], k, 2, False))
        k = dims.head_units[j]
    g.append((hr, 6, k, 4, False))
    tot = sum(2 * m * kk + 2 * n * kk + ob * m * n + (rb * m * n if r else 0)
              for m, n, kk, ob, r in g)
    return tot / len(g)


# ---- parity mode (north_star's tolerance on the driver's line): the committed batched golden
# case of the headline config (tests/golden/batched_forward.json "c2_vitb16_imgs8": 8 images,
# fp64 oracle logits, made by tests/golden/make_golden.py) placed among filler images exactly
# as tests/test_gpu_batch_parity.py places them.  The weights and images are regenerated from
# the fixture's seeds by the same numpy draws the golden script used (glorot / N(0, perturb)
# in Keras weight order; U(-1, 1) images) -- tests/test_host_cpu.py checks these two functions
# against the oracle's generators.
GOLDEN_CASE, GOLDEN_POS = "c2_vitb16_imgs8", [0, 1, 97, 127, 128, 200, 254, 255]


def golden_weights(weight_shapes, seed, perturb):
    """Keras-default-like init with N(0, perturb) on biases / gamma / beta, drawn in Keras
    weight-creation order (the golden fixture's generator)."""
    import math
    import numpy as np
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in weight_shapes.items():
        shape = tuple(shape)
        if name.endswith("/embeddings"):
            v = rng.uniform(-0.05, 0.05, size=shape)
        elif name.endswith("/kernel"):
            if len(shape) == 2:
                fi, fo = shape
            else:
                rf = int(np.prod(shape[:-2]))
                fi, fo = shape[-2] * rf, shape[-1] * rf
            lim = math.sqrt(6.0 / (fi + fo))
            v = rng.uniform(-lim, lim, size=shape)
        elif name.endswith("/gamma"):
            v = np.ones(shape) + (rng.normal(0, perturb, size=shape) if perturb else 0)
        else:
            v = rng.normal(0, perturb, size=shape) if perturb else np.zeros(shape)
        out[name] = v.astype(np.float32)
    return out


def golden_images(n, shape, seed, letterbox):
    import numpy as np
    rng = np.random.default_rng(seed)
    h, w, c = shape
    img = rng.uniform(-1.0, 1.0, size=(n, h, w, c)).astype(np.float32)
    if letterbox:
        band = h // 8
        img[:, :band] = -1.0
        img[:, h - band:] = -1.0
    return img


def parity_mode(args, dev, kw_run):
    """North_star's fp32 tolerance on the headline workload, timed like the headline: the fp32
    parity mode and the split-bf16 mode (bf16x3) at C2 B = 256, W warm-up + K timed steps
    (forward + fused decode, two streams), the GEMM class's fraction of the fp32 peak from a
    one-stream profiled pass, and the max relative error of the 8 golden rows against their
    fp64 oracle logits ("rel": max |y - ref| / max |ref| per image; "within_1e-3": the
    |y - ref| <= 1e-3 |ref| + 1e-3 max|ref| test of tests/test_gpu_batch_parity.py) -- checked
    outside the timed region."""
    import ctypes
    import hashlib
    import numpy as np
    import vision_transformer_detector_amd as vtd
    from vision_transformer_detector_amd import _lib as L
    spec = json.load(open(os.path.join(ROOT, "tests", "golden", "batched_forward.json")))[GOLDEN_CASE]
    kw = dict(spec["kwargs"])
    kw["input_shape"] = tuple(kw["input_shape"])
    probe = vtd.create_vision_transformer_detector(**kw, dtype="float32", device=dev, seed=0)
    shape = probe.input_shape
    imgs = golden_images(spec["n"], shape, spec["image_seed"], spec["letterbox"])
    if hashlib.sha256(np.ascontiguousarray(imgs).tobytes()).hexdigest() != spec["images_sha256"]:
        return {"error": "golden images do not regenerate from their seed"}
    w = golden_weights(probe.weight_shapes, spec["weight_seed"], spec["perturb"])
    del probe
    B = 256
    gen = torch.Generator(device=dev).manual_seed(77)
    x = torch.rand((B,) + tuple(shape), generator=gen, device=dev) * 2 - 1
    for i, p in enumerate(GOLDEN_POS):
        x[p] = torch.from_numpy(imgs[i]).to(dev)
    ref = [np.asarray(r, np.float64) for r in spec["logits"]]
    out = {"workload": f"{GOLDEN_CASE}: ViT-B/16 @224 (the headline preset), batch {B}, "
                       f"golden rows at {GOLDEN_POS}", "steps": args.steps, "warmup": args.warmup}
    for mode in ("float32", "bf16x3"):
        model = vtd.create_vision_transformer_detector(**kw, dtype=mode, device=dev, seed=0)
        model.set_weights(w)
        for _ in range(args.warmup):
            model.detect(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            model.detect(x)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        logits, _ = model.detect(x)
        y = logits.cpu().numpy().astype(np.float64)
        rel, ok = 0.0, True
        for i, p in enumerate(GOLDEN_POS):
            err = np.abs(y[p] - ref[i])
            rel = max(rel, float(err.max() / np.abs(ref[i]).max()))
            ok = ok and bool(np.all(err <= 1e-3 * np.abs(ref[i]) + 1e-3 * np.abs(ref[i]).max()))
        # the GEMM class alone (one stream, hipEvents around every launch)
        L.check(L.lib.vtd_profile_reset())
        L.check(L.lib.vtd_profile_enable(1))
        for _ in range(max(1, args.steps // 4)):
            model.detect(x)
        torch.cuda.synchronize()
        L.check(L.lib.vtd_profile_enable(0))
        ms = (ctypes.c_double * L.PROF_CLASSES)()
        nl = (ctypes.c_int64 * L.PROF_CLASSES)()
        fl = (ctypes.c_double * L.PROF_CLASSES)()
        L.check(L.lib.vtd_profile_read(ms, nl, fl, L.PROF_CLASSES))
        gemm_tf = fl[0] / (ms[0] * 1e-3) / 1e12 if ms[0] > 0 else None
        rec = {"value": round(B * args.steps / el, 2), "unit": "images/s",
               "ms_per_step": round(1e3 * el / args.steps, 3),
               "max_rel_err_golden_rows": float(f"{rel:.3e}"), "within_1e-3": ok,
               "gemm_tflops": round(gemm_tf, 1) if gemm_tf else None,
               "gemm_frac_of_fp32_peak": round(gemm_tf / PEAK_TFLOPS["f32"], 4) if gemm_tf else None}
        if mode == "bf16x3" and gemm_tf:
            # three bf16 MFMA products per algorithmic one: the matrix cores' own load
            rec["gemm_mfma_frac_of_bf16_peak"] = round(3 * gemm_tf / PEAK_TFLOPS["bf16"], 4)
        out[mode] = rec
        del model
        torch.cuda.empty_cache()
    if out.get("float32", {}).get("value"):
        out["bf16x3_over_float32"] = round(out["bf16x3"]["value"] / out["float32"]["value"], 3)
    return out


def cpu_baseline(model, kw, shape, preset):
    """The oracle's fp32 torch-CPU restatement (oracle/vtd_torch_cpu.py) of the same graph on
    the host cores: the reference's TF-CPU path cannot run in this pipeline (TF/Keras/tfa
    absent), so this is the "port" baseline.  SURVEY.md §8(d)'s plan: C1 (the
    reference default) and C2 (ViT-B/16 @224), batch 1 and 8, median of 5 forwards after 1
    warm-up, len(os.sched_getaffinity(0)) host threads (capped by OMP_NUM_THREADS).  `value` = the bench preset's batch-8 median when it is one of
    the two (else C2's)."""
    import statistics
    import numpy as np
    import vision_transformer_detector_amd as vtd
    from oracle import vtd_numpy as ref
    from oracle.vtd_torch_cpu import TorchCpuDetector
    # torch.set_num_threads(len(os.sched_getaffinity(0))), capped by
    # OMP_NUM_THREADS where the job's host-core share is set (16 per GPU on the GPU box,
    # whose affinity mask shows the whole machine)
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(affinity, omp) if omp > 0 else affinity
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    cases = {}
    t_all = time.perf_counter()
    for name in ("c1", "vit_b16_224"):
        pkw = dict(vtd.presets.PRESETS[name])
        if name == preset:
            det = TorchCpuDetector(model.get_weight_dict(), **kw)
            pshape = shape
        else:
            det = TorchCpuDetector(ref.init_weights(seed=0, **pkw), **pkw)
            pshape = tuple(ref.resolve_kwargs(**pkw)["input_shape"])
        for b in (1, 8):
            x = letterbox_images(b, pshape, torch.Generator().manual_seed(7), "cpu")
            det(x)                                           # warm-up
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                det(x)
                ts.append(time.perf_counter() - t0)
            med = statistics.median(ts)
            cases[f"{name}_b{b}"] = {"images_per_s": round(b / med, 3),
                                     "median_s": round(med, 4)}
    torch.set_num_threads(prev_threads)
    key = f"{preset if preset in ('c1', 'vit_b16_224') else 'vit_b16_224'}_b8"
    return {"value": cases[key]["images_per_s"], "unit": "images/s", "cores": threads,
            "kind": "port",
            "sample": f"median of 5 forwards after 1 warm-up, batch 1 and 8, C1 (608x608 "
                      f"default) and C2 (ViT-B/16 @224), fp32 torch-CPU restatement, "
                      f"{threads} threads (affinity {affinity}, OMP_NUM_THREADS "
                      f"{omp or 'unset'}), {time.perf_counter() - t_all:.1f} s in all; "
                      f"value = {key}",
            "cases": cases}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`--gpus N` with no launcher around us: start N rank processes of this same command
    line (rank r on GPU r, rendezvous on 127.0.0.1) and wait for them.  Runs before this
    process makes any GPU call.  If a rank fails, the others (which would wait in a
    collective forever) are terminated by their own handles.  Returns the exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] +
                                      sys.argv[1:], env=env))
    code = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and code == 0:
                code = rc if rc > 0 else 128 - rc
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return code


def rank_spread(elapsed, world, device):
    """Every rank's own timed-region length -> (min, max) over ranks (max = the job's)."""
    if world == 1:
        return {"min_s": elapsed, "max_s": elapsed}
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    ts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(ts, t)
    v = [float(x.item()) for x in ts]
    return {"min_s": min(v), "max_s": max(v)}


def check_gather(dets, world, rank, B, device):
    """Outside the timed region: one more all-gather of this rank's detections; every rank
    checks that the gathered (world*B, 17, 6) holds its own shard bit for bit at its offset
    and that every shard is finite.  Returns the AND over ranks."""
    from vision_transformer_detector_amd.distributed import all_gather_detections
    g = all_gather_detections(dets, world * B) if world > 1 else dets
    ok = (g.shape[0] == world * B and torch.equal(g[rank * B:(rank + 1) * B], dets)
          and bool(torch.isfinite(g).all()))
    if world > 1:
        f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item())
    return ok


def dry_run(args, world, rank):
    """CPU rehearsal of the multi-rank path (gloo): the launcher, the rendezvous, the
    barrier / max-over-ranks timing and the all-gather of (B, 17, 6) detections, without
    the GPU forward.  Prints the same JSON line shape with `value` = gathered images/s."""
    from vision_transformer_detector_amd.distributed import all_gather_detections
    if world > 1:
        dist.init_process_group("gloo")
    B = args.batch
    dets = torch.full((B, 17, 6), float(rank))
    for _ in range(args.warmup):
        out = all_gather_detections(dets, world * B) if world > 1 else dets
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = all_gather_detections(dets, world * B) if world > 1 else dets
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    spread = rank_spread(elapsed, world, "cpu")
    elapsed = spread["max_s"]
    ranks_ok = out.shape[0] == world * B and all(
        bool((out[r * B:(r + 1) * B] == r).all()) for r in range(world))
    gather_ok = check_gather(dets, world, rank, B, "cpu")
    if rank == 0:
        print(json.dumps({
            "metric": "dry-run: all-gather of detections only (no GPU forward)",
            "value": round(world * B * args.steps / max(elapsed, 1e-9), 2),
            "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / max(1, args.steps), 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic", "gather_rank_order_ok": ranks_ok,
            "gather_ok": gather_ok,
            "rank_ms_min": round(1e3 * spread["min_s"] / max(1, args.steps), 3),
            "rank_ms_max": round(1e3 * spread["max_s"] / max(1, args.steps), 3),
            "config": {"workload": "dry-run (gloo, CPU)", "per_gpu_batch": B,
                       "global_batch": world * B, "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not ranks_ok:
        raise SystemExit(f"rank {rank}: all-gather returned the wrong rank order")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE from the launcher, else 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal: launcher + gloo all-gather, no GPU forward")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32", "fp8", "bf16x3"],
                    help="bf16x3: the split-bf16 parity mode (the drop-in default dtype; "
                         "roofline against the bf16 peak, FLOPs counted once although each is "
                         "three bf16 MFMA products)")
    ap.add_argument("--preset", default="vit_b16_224")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--images", default="letterbox", choices=["letterbox", "uniform"],
                    help="synthetic inputs: COCO-shaped letterboxed U(-1, 1) images (SURVEY "
                         "8(d), the default) or plain U(-1, 1) (A/B of the data's effect)")
    ap.add_argument("--no-parity-mode", action="store_true",
                    help="skip the f32 / split-bf16 parity-mode sub-record (headline config only)")
    ap.add_argument("--streams", type=int, default=2,
                    help="vtd_forward micro-batch streams (VTD_STREAMS; 1 = one stream)")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: the forward of a step is one HIP-graph replay (captured once after "
                         "warm-up); 0: eager vtd_forward calls")
    args = ap.parse_args()
    os.environ["VTD_STREAMS"] = str(args.streams)      # read once by libvtd.so

    if "WORLD_SIZE" not in os.environ:
        if args.gpus is not None and args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))          # no GPU call has happened yet
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"--gpus {args.gpus} disagrees with WORLD_SIZE={world} "
                             "from the launcher")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import vision_transformer_detector_amd as vtd
    from vision_transformer_detector_amd import _lib as L
    kw = dict(vtd.presets.PRESETS[args.preset])
    # identical weights on every rank (same seed): replicated-weight data parallelism
    model = vtd.create_vision_transformer_detector(
        **kw, dtype={"bf16": "bfloat16", "f32": "float32", "fp8": "float8",
                     "bf16x3": "bf16x3"}[args.dtype],
        device=dev, seed=0)
    kw = {k: model.kwargs[k] for k in model.kwargs}
    shape = model.input_shape
    B = args.batch
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    images = (letterbox_images(B, shape, gen, dev) if args.images == "letterbox"
              else torch.rand((B,) + tuple(shape), generator=gen, device=dev) * 2 - 1)

    from vision_transformer_detector_amd.distributed import all_gather_detections

    def eager_step():
        logits, dets = model.detect(images)
        if world > 1:                        # the path's one exchange: RCCL all-gather
            all_gather_detections(dets, world * B)
        return logits

    step = eager_step
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.graph:
        # the whole forward (every kernel of vtd_forward, both micro-batch streams, the
        # decode) captured once as a HIP graph on a side stream and replayed per step: the
        # same launches without per-launch host work or inter-kernel gaps.  The RCCL
        # all-gather stays outside the graph.
        cs = torch.cuda.Stream(device=dev)
        cs.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cs):
            model.detect(images)             # workspace / internal stream exist before capture
            with torch.cuda.graph(graph, stream=cs):
                g_logits, g_dets = model.detect(images)
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()

        def step():
            graph.replay()
            if world > 1:
                all_gather_detections(g_dets, world * B)
            return g_logits

        step()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    spread = rank_spread(elapsed, world, dev)
    elapsed = spread["max_s"]
    # correctness evidence of the timed path (outside the timed region): this rank's
    # detections, gathered over all ranks, sit bit for bit at its shard offset, all finite
    _, dets_chk = model.detect(images)
    gather_ok = check_gather(dets_chk, world, rank, B, dev)

    # ---- per-kernel timing: hipEvents recorded around every launch of vtd_forward on
    # the stream it launches on, over K more steps of the same workload.  Profiling runs
    # vtd_forward on one stream (no micro-batch overlap), so each launch's event pair
    # times that kernel alone: the roofline below is the kernel's own, while `value`
    # (the timed region above) includes the two-stream overlap.
    L.check(L.lib.vtd_profile_reset())
    L.check(L.lib.vtd_profile_enable(1))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        eager_step()                         # profiling hooks run at launch time: eager
    torch.cuda.synchronize()
    prof_elapsed = time.perf_counter() - t1
    L.check(L.lib.vtd_profile_enable(0))
    import ctypes
    ms = (ctypes.c_double * L.PROF_CLASSES)()
    nl = (ctypes.c_int64 * L.PROF_CLASSES)()
    fl = (ctypes.c_double * L.PROF_CLASSES)()
    L.check(L.lib.vtd_profile_read(ms, nl, fl, L.PROF_CLASSES))
    classes = ["gemm", "attention", "layernorm", "patches", "other"]
    kernels = {c: {"ms_total": ms[i], "launches": int(nl[i]),
                   "avg_us": 1e3 * ms[i] / max(1, nl[i]),
                   "tflops": (fl[i] / (ms[i] * 1e-3) / 1e12) if ms[i] > 0 and fl[i] > 0 else None}
               for i, c in enumerate(classes)}

    total_fl, attn_mlp_fl = algorithmic_flops_per_image(kw, model.dims)
    ms_per_step = 1e3 * elapsed / args.steps
    img_s = world * B * args.steps / elapsed
    peak = PEAK_TFLOPS[args.dtype]
    g = kernels["gemm"]
    gemm_tf = g["tflops"]
    headline = args.preset == "vit_b16_224" and B == 256 and args.dtype == "bf16"
    # the committed PMC passes are of the headline command (C2, B = 256, bf16)
    headline_cfg = headline
    traffic, traffic_src = traffic_per_launch()
    metric = ("images/sec ViT-B/16 detector fwd, batch 256, 1/2/4/8 MI355X; MFMA util %"
              if headline else
              f"images/sec {args.preset} detector fwd, batch {B} per GPU, {args.dtype}, "
              f"{world} MI355X; MFMA util %")
    out = {
        "metric": metric,
        "value": round(img_s, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": ("synthetic (U(-1,1) NHWC letterboxed images generated on device; "
                 if args.images == "letterbox" else
                 "synthetic (U(-1,1) NHWC images, no letterbox, generated on device; ") +
                "random Keras-default-init weights)",
        "config": {"workload": f"{args.preset} detector forward + decode" +
                               (" + RCCL all-gather of detections" if world > 1 else ""),
                   "per_gpu_batch": B, "global_batch": world * B,
                   "input_shape": list(shape), "tokens": model.dims.tokens,
                   "parallelism": f"dp{world}", "streams_per_gpu": args.streams,
                   "hip_graph": bool(args.graph)},
        "mfma_util_attn_mlp": round(attn_mlp_fl * img_s / world / (peak * 1e12), 4),
        "model_tflops_per_gpu": round(total_fl * img_s / world / 1e12, 1),
        "roofline": {"bound": "mfma",
                     "kernel": "gemm_mx8 (encoder Dense) + gemm_tn_bf16 (head)" if args.dtype == "fp8"
                     else "gemm_tn_* (all Dense layers)",
                     "achieved": round(gemm_tf, 1) if gemm_tf else None, "peak": peak,
                     "unit": "TFLOP/s",
                     "frac": round(gemm_tf / peak, 4) if gemm_tf else None,
                     "traffic": traffic if headline_cfg else None,
                     "traffic_source": (f"profiles/gemm_traffic_latest.json ({traffic_src}): "
                                        "rocprofv3 PMC passes of this command on a builder box, "
                                        "not measured in this run") if headline_cfg and traffic
                     else None,
                     "algorithmic_bytes_per_launch": round(gemm_alg_bytes(
                         kw, model.dims, B, 4 if (args.dtype in ("f32", "float32") or
                                              os.environ.get("VTD_RESID_F32", "0") != "0") else 2)),
                     "avg_launch_us": round(g["avg_us"], 2),
                     "launches_per_step": g["launches"] // max(1, args.steps),
                     # the GEMM class in the TIMED step (two streams: tails filled, epilogues
                     # beside the other part's K loops): its algorithmic FLOPs per step over
                     # the whole step time (non-GEMM kernels included) -- a lower bound of the
                     # GEMMs' in-step rate; frac above is the isolated-launch figure
                     "step_frac": round(fl[0] / max(1, args.steps) / (ms_per_step * 1e-3) /
                                        (peak * 1e12), 4) if fl[0] > 0 else None},
        "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv)
                        for kk, vv in v.items()} for k, v in kernels.items()},
        "profiled_ms_per_step": round(1e3 * prof_elapsed / args.steps, 3),
        "gather_ok": gather_ok,
        "rank_ms_min": round(1e3 * spread["min_s"] / args.steps, 3),
        "rank_ms_max": round(1e3 * spread["max_s"] / args.steps, 3),
    }
    if args.dtype == "bf16x3":
        # the split-bf16 mode runs each algorithmic FLOP as three bf16 MFMA products: the
        # matrix cores' load is 3x the algorithmic utilisation above
        out["mfma_util_hw"] = round(3 * out["mfma_util_attn_mlp"], 4)
        out["roofline"]["frac_hw"] = (round(3 * out["roofline"]["frac"], 4)
                                      if out["roofline"]["frac"] else None)
    if world == 1 and headline and not args.no_parity_mode:
        out["parity_mode"] = parity_mode(args, dev, kw)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(model, kw, shape, args.preset)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
