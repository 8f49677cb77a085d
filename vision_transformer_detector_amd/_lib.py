"""ctypes binding of libvtd.so (the C-ABI declared in include/vtd.h).

Import order matters: torch is imported first so that the HIP runtime SONAME
`libamdhip64.so.7` needed by libvtd.so resolves to the copy torch already loaded
(one HIP runtime per process).  There is no fallback: if the shared library is
missing or incomplete, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede loading libvtd.so, see module doc)

# VTD_LIB_PATH: an alternative build of the same sources (A/B experiments of build-time knobs)
LIB_PATH = os.environ.get("VTD_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "libvtd.so")

ABI_VERSION = 16
KALIGN = 64
MAX_MLP = 16
MAX_HEAD = 64
MAX_DETECT = 17
PROF_CLASSES = 5
MAP_CLASSES, MAP_LATEST, MAP_PER_IMAGE, MAP_MAX_BOXES = 80, 3, 14, 64

F32, BF16, FP8, BF16X3 = 0, 1, 2, 3
# run-time A/B knobs (vtd_set_knob; -1 = the library default)
KNOB_ATTN_VARIANT, KNOB_ATTN_GRID, KNOB_GEMM_NGW, KNOB_SPLITK, KNOB_JPEG_CHUNK_BITS = 0, 1, 2, 3, 4
KNOB_SKINNY, KNOB_F32_PP2, KNOB_STAGGER, KNOB_GEMM_TR, KNOB_FIN_WGS = 5, 6, 7, 8, 9
KNOB_GEMM_TPW = 10
ACT_NONE, ACT_GELU_TANH, ACT_MISH = 0, 1, 2
STATUS = {0: "VTD_OK", -1: "VTD_ERR_INVALID_ARG", -2: "VTD_ERR_UNSUPPORTED",
          -3: "VTD_ERR_HIP", -4: "VTD_ERR_WORKSPACE"}

c_int, c_int64, c_size_t, c_float, c_void_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_size_t,
                                                ctypes.c_float, ctypes.c_void_p)


class VtdConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "batch", "image_h", "image_w", "channels", "patch_size", "embedding_dim",
        "num_heads", "key_dim", "mlp_quantities", "repeat_times", "head_last_units",
        "head_layers", "head_repeats", "use_mish", "dtype")]


class VtdDims(ctypes.Structure):
    _fields_ = [
        ("grid_h", c_int), ("grid_w", c_int), ("tokens", c_int), ("pad_top", c_int),
        ("pad_left", c_int), ("patch_dim", c_int), ("patch_dim_p", c_int), ("d", c_int),
        ("d_p", c_int), ("key_dim_p", c_int), ("inner_p", c_int), ("qkv_p", c_int),
        ("mlp_units", c_int * MAX_MLP), ("mlp_units_p", c_int * MAX_MLP),
        ("n_head", c_int), ("head_units", c_int * MAX_HEAD),
        ("head_units_p", c_int * MAX_HEAD), ("tokens_p", c_int), ("rows", c_int64),
        ("head_rows", c_int64)]


class VtdLayerWeights(ctypes.Structure):
    _fields_ = [
        ("ln1_gamma", c_void_p), ("ln1_beta", c_void_p), ("w_qkv", c_void_p),
        ("b_qkv", c_void_p), ("w_out", c_void_p), ("b_out", c_void_p),
        ("ln2_gamma", c_void_p), ("ln2_beta", c_void_p),
        ("w_mlp", c_void_p * MAX_MLP), ("b_mlp", c_void_p * MAX_MLP),
        ("s_qkv", c_void_p), ("s_out", c_void_p), ("s_mlp", c_void_p * MAX_MLP),
        ("ln1_colsum", c_void_p), ("ln2_colsum", c_void_p)]


class VtdWeights(ctypes.Structure):
    _fields_ = [
        ("w_patch", c_void_p), ("b_patch", c_void_p), ("pos_embedding", c_void_p),
        ("layers", ctypes.POINTER(VtdLayerWeights)), ("w_det", c_void_p),
        ("b_det", c_void_p), ("w_head", c_void_p * MAX_HEAD),
        ("b_head", c_void_p * MAX_HEAD), ("w_final", c_void_p), ("b_final", c_void_p)]


class VtdEpilogue(ctypes.Structure):
    _fields_ = [
        ("bias", c_void_p), ("rowadd", c_void_p), ("rowadd_period", c_int),
        ("rowadd_ncols", c_int), ("act", c_int), ("resid", c_void_p), ("ldr", c_int),
        ("out", c_void_p), ("ldo", c_int), ("out_dtype", c_int), ("out2", c_void_p),
        ("ldo2", c_int), ("scatter_tokens", c_int), ("lnstat", c_void_p), ("colsum", c_void_p),
        ("statout", c_void_p), ("stat_ld", c_int), ("scale_out", c_void_p),
        ("scale_rows", c_int64), ("detections", c_void_p)]


# name -> (restype, argtypes)
SIGNATURES = {
    "vtd_abi_version": (c_int, []),
    "vtd_last_error": (ctypes.c_char_p, []),
    "vtd_derive_dims": (c_int, [ctypes.POINTER(VtdConfig), ctypes.POINTER(VtdDims)]),
    "vtd_workspace_bytes": (c_int, [ctypes.POINTER(VtdConfig), ctypes.POINTER(c_size_t)]),
    "vtd_pack_dense": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                               c_int, c_int, c_int, c_void_p]),
    "vtd_pack_vector": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "vtd_extract_patches": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                    c_int, c_int, c_void_p]),
    "vtd_gemm": (c_int, [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                         ctypes.POINTER(VtdEpilogue), c_void_p]),
    "vtd_gemm_splitk": (c_int, [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                                ctypes.POINTER(VtdEpilogue), c_void_p, c_size_t, c_int, c_void_p]),
    "vtd_gemm_splitk_choice": (c_int, [c_int, c_int, c_int, c_int]),
    "vtd_quantize_mx8": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_int, c_void_p, c_int,
                                 c_void_p, c_int64, c_void_p]),
    "vtd_layernorm_mx8": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_void_p,
                                  c_float, c_void_p, c_int, c_int, c_void_p, c_int64, c_void_p]),
    "vtd_gemm_mx8": (c_int, [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int64, c_void_p,
                             c_int, c_void_p, c_int64, ctypes.POINTER(VtdEpilogue), c_void_p]),
    "vtd_layernorm": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_void_p, c_float,
                              c_void_p, c_int, c_int, c_void_p]),
    "vtd_layernorm_stats": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_float, c_void_p,
                                    c_void_p]),
    "vtd_layernorm_stats_finalize": (c_int, [c_void_p, c_int64, c_int, c_int, c_float, c_void_p,
                                             c_void_p]),
    "vtd_fold_layernorm": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "vtd_attention": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_float,
                              c_void_p, c_int, c_int, c_void_p]),
    "vtd_attention_mx8": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p,
                                  c_int, c_void_p, c_int64, c_void_p]),
    "vtd_split_bf16x3": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_int, c_int,
                                 c_void_p]),
    "vtd_decode": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "vtd_decode_detections": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                      c_float, c_float, c_void_p]),
    "vtd_resize_with_pad": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                    c_void_p]),
    "vtd_jpeg_info": (c_int, [c_void_p, c_size_t, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                              ctypes.POINTER(c_int)]),
    "vtd_jpeg_workspace_bytes": (c_int, [c_void_p, c_void_p, c_int, c_void_p,
                                         ctypes.POINTER(c_size_t)]),
    "vtd_jpeg_decode": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                c_size_t, c_void_p]),
    "vtd_png_info": (c_int, [c_void_p, c_size_t, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                             ctypes.POINTER(c_int)]),
    "vtd_png_workspace_bytes": (c_int, [c_void_p, c_void_p, c_int, c_void_p,
                                        ctypes.POINTER(c_size_t)]),
    "vtd_png_decode": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                               c_size_t, c_void_p]),
    "vtd_png_inflate": (c_int, [c_void_p, c_size_t, c_void_p, c_size_t, ctypes.POINTER(c_size_t)]),
    "vtd_bmp_info": (c_int, [c_void_p, c_size_t, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                             ctypes.POINTER(c_int)]),
    "vtd_bmp_workspace_bytes": (c_int, [c_void_p, c_void_p, c_int, c_void_p,
                                        ctypes.POINTER(c_size_t)]),
    "vtd_bmp_decode": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                               c_size_t, c_void_p]),
    "vtd_iou": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    "vtd_map_reset": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "vtd_map_update": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                               c_void_p]),
    "vtd_map_result": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vtd_forward": (c_int, [ctypes.POINTER(VtdConfig), ctypes.POINTER(VtdWeights), c_void_p,
                            c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "vtd_set_knob": (c_int, [c_int, c_int]),
    "vtd_get_knob": (c_int, [c_int]),
    "vtd_profile_enable": (c_int, [c_int]),
    "vtd_profile_reset": (c_int, []),
    "vtd_profile_read": (c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64),
                                 ctypes.POINTER(ctypes.c_double), c_int]),
}


class VtdError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libvtd.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)           # AttributeError if a symbol is missing
        fn.restype, fn.argtypes = res, args
    if lib.vtd_abi_version() != ABI_VERSION:
        raise ImportError(f"libvtd.so ABI {lib.vtd_abi_version()} != {ABI_VERSION}")
    return lib


lib = _load()


def check(rc: int, what: str = "") -> None:
    """Raise like the reference would: invalid shapes -> ValueError, else RuntimeError."""
    if rc == 0:
        return
    msg = lib.vtd_last_error().decode(errors="replace")
    text = f"{what}: {STATUS.get(rc, rc)}: {msg}" if what else f"{STATUS.get(rc, rc)}: {msg}"
    if rc == -1:
        raise ValueError(text)
    raise VtdError(text)


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t) -> int | None:
    return None if t is None else int(t.data_ptr())


class knob:
    """Context manager: `with knob(KNOB_ATTN_VARIANT, 2): ...` sets a run-time knob of the
    library (vtd_set_knob) and restores the previous value on exit."""

    def __init__(self, k: int, value: int):
        self.k, self.value, self.prev = k, int(value), None

    def __enter__(self):
        self.prev = lib.vtd_set_knob(self.k, self.value)
        return self

    def __exit__(self, *exc):
        lib.vtd_set_knob(self.k, self.prev)
        return False
