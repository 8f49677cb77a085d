"""TEST INFRASTRUCTURE ONLY — independent float32 torch-CPU restatement of the forward.

A second implementation of the same Keras graph (`/root/reference/vision_transformer_detector.py:239-583`)
written with different primitives from `vtd_numpy` (tensor.unfold for the SAME patches,
torch.layer_norm, batched matmul attention).  Used (1) to cross-check the fp64 oracle (and, run with dtype=float64, as a fast fp64
reference for large configs) and (2) as `bench.py`'s CPU baseline ("port": the reference's TF-CPU path cannot run here).
Parity against executed reference output is UNPINNED (see `oracle/__init__.py`).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import vtd_numpy as _spec

MAX_DETECT = _spec.MAX_DETECT_OBJECTS_QUANTITY


def _patches(x, p):
    b, h, w, c = x.shape
    gh, gw = -(-h // p), -(-w // p)
    ph, pw = max(gh * p - h, 0), max(gw * p - w, 0)
    # F.pad pads trailing dims first: (C: 0,0), (W: left,right), (H: top,bottom)
    x = F.pad(x, (0, 0, pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
    x = x.unfold(1, p, p).unfold(2, p, p)          # (B, gh, gw, C, kh, kw)
    x = x.permute(0, 1, 2, 4, 5, 3)                 # (B, gh, gw, kh, kw, C)
    return x.reshape(b, gh * gw, p * p * c)


def _mish(x):
    return x * torch.tanh(F.softplus(x))


def _gelu(x):
    return F.gelu(x, approximate="tanh")


class TorchCpuDetector:
    """Holds fp32 torch weights (keyed by Keras names) and runs the forward on CPU."""

    def __init__(self, weights, dtype=torch.float32, **kw):
        self.kw = _spec.resolve_kwargs(**kw)
        self.dtype = dtype
        self.w = {n: torch.as_tensor(v).to(dtype) for n, v in weights.items()}
        k = self.kw
        self.act = _mish if k["use_mish"] else _gelu
        self.nh, self.dk = k["encoder_num_heads"], k["encoder_key_dim"]
        # fuse q/k/v kernels into one (D, 3*H*dk) matrix per layer
        self.layers = []
        for i in range(1, k["encoder_repeat_times"] + 1):
            ln1 = "layer_normalization" + ("" if i == 1 else f"_{2 * (i - 1)}")
            ln2 = f"layer_normalization_{2 * (i - 1) + 1}"
            mha = "multi_head_attention" + ("" if i == 1 else f"_{i - 1}")
            g = lambda n: self.w[f"{mha}/{n}"]
            d = g("query/kernel").shape[0]
            wqkv = torch.cat([g(f"{n}/kernel").reshape(d, -1) for n in ("query", "key", "value")], 1)
            bqkv = torch.cat([g(f"{n}/bias").reshape(-1) for n in ("query", "key", "value")])
            mlp = [(self.w[f"MLP_{i}_{j}/kernel"], self.w[f"MLP_{i}_{j}/bias"])
                   for j in range(1, k["encoder_mlp_quantities"] + 1)]
            self.layers.append(dict(
                g1=self.w[f"{ln1}/gamma"], b1=self.w[f"{ln1}/beta"],
                wqkv=wqkv, bqkv=bqkv,
                wo=g("attention_output/kernel").reshape(-1, d), bo=g("attention_output/bias"),
                g2=self.w[f"{ln2}/gamma"], b2=self.w[f"{ln2}/beta"], mlp=mlp))
        self.head = []
        idx = 1
        while f"dense_{idx}/kernel" in self.w:
            self.head.append((self.w[f"dense_{idx}/kernel"], self.w[f"dense_{idx}/bias"]))
            idx += 1

    @torch.no_grad()
    def __call__(self, images):
        w = self.w
        x = torch.as_tensor(images).to(self.dtype)
        b = x.shape[0]
        pt = _patches(x, self.kw["patch_size"])
        n = pt.shape[1]
        e = torch.addmm(w["linear_projection/bias"], pt.reshape(b * n, -1),
                        w["linear_projection/kernel"]).reshape(b, n, -1)
        e = e + w["position_encoding/position_embedding/embeddings"][:n].reshape(1, n, 1)
        d = e.shape[-1]
        nh, dk = self.nh, self.dk
        scale = 1.0 / math.sqrt(float(dk))
        for L in self.layers:
            h = F.layer_norm(e, (d,), L["g1"], L["b1"], eps=1e-3)
            qkv = torch.addmm(L["bqkv"], h.reshape(b * n, d), L["wqkv"])
            qkv = qkv.reshape(b, n, 3, nh, dk).permute(2, 0, 3, 1, 4)   # (3,B,H,N,dk)
            q, k_, v = qkv[0] * scale, qkv[1], qkv[2]
            s = torch.softmax(q @ k_.transpose(-1, -2), dim=-1)
            o = (s @ v).permute(0, 2, 1, 3).reshape(b * n, nh * dk)
            e = e + torch.addmm(L["bo"], o, L["wo"]).reshape(b, n, d)
            h = F.layer_norm(e, (d,), L["g2"], L["b2"], eps=1e-3).reshape(b * n, d)
            for wk, bk in L["mlp"]:
                h = self.act(torch.addmm(bk, h, wk))
            e = e + h.reshape(b, n, d)
        t = torch.addmm(w["dense/bias"], e.reshape(b * n, d), w["dense/kernel"])
        u = t.reshape(b * MAX_DETECT, n)            # Reshape((17, -1)): row-major view
        for wk, bk in self.head:
            u = self.act(torch.addmm(bk, u, wk))
        out = torch.addmm(w["MLP_Head_no_Sigmoid/bias"], u, w["MLP_Head_no_Sigmoid/kernel"])
        return out.reshape(b, MAX_DETECT, 6)
