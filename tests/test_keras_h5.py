"""Keras HDF5 weight import (vtd.py:2146, 2179): the pure-Python
HDF5 reader (vision_transformer_detector_amd/keras_h5.py) against
- tests/golden/tiny_keras.h5 (tests/golden/make_keras_h5.py: the Keras 2.9 layout with the
  oracle's seeded weights) -- PARITY UNPINNED against a file Keras itself saved (none ships
  with the reference; h5py / TF are absent here);
- a file written by the HDF5 library itself (scipy's MATLAB v7.3 test file, when present);
- writer-generated edge cases: multi-level group B-trees, weights-only layout, a 512-B
  user block, attributes Keras split into name0 / name1."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)

from h5_writer import H5Writer, write_keras_model  # noqa: E402
from make_keras_h5 import SEED, TINY  # noqa: E402
from oracle import vtd_numpy as ref  # noqa: E402
from vision_transformer_detector_amd.keras_h5 import (H5Error, H5File,  # noqa: E402
                                                      read_keras_weights)

FIXTURE = os.path.join(GOLDEN, "tiny_keras.h5")


def test_fixture_weights_equal_the_seeded_oracle_weights():
    w, cfg = read_keras_weights(FIXTURE)
    exp = ref.init_weights(seed=SEED, **TINY)
    assert list(w) != [] and set(w) == set(exp)
    for k, v in exp.items():
        assert w[k].dtype == np.float32 and np.array_equal(w[k], v), k
    assert cfg["class_name"] == "Functional"


def test_fixture_keras_structure():
    with H5File(FIXTURE) as f:
        assert f.keys() == ["model_weights"]
        assert f.attrs["keras_version"] == b"2.9.0"
        mw = f["model_weights"]
        names = [n.decode() for n in mw.attrs["layer_names"]]
        assert names[:4] == ["images", "split_image_into_patches", "flatten_patches",
                             "linear_projection"]
        assert names[-1] == "MLP_Head_no_Sigmoid"
        assert len(mw["images"].attrs["weight_names"]) == 0          # weightless layer
        mha = mw["multi_head_attention"]
        wn = [n.decode() for n in mha.attrs["weight_names"]]
        assert "multi_head_attention/query/kernel:0" in wn
        ds = f["model_weights/multi_head_attention/multi_head_attention/query/kernel:0"]
        assert ds.shape == (24, 3, 10) and ds.dtype == np.float32


HDF5_MAT = "/usr/local/lib/python3.10/dist-packages/scipy/io/matlab/tests/data/testhdf5_7.4_GLNX86.mat"


@pytest.mark.skipif(not os.path.exists(HDF5_MAT), reason="scipy test data absent")
def test_reads_a_file_written_by_the_hdf5_library():
    # MATLAB -v7.3 file (512-B user block, superblock v0) from scipy's test data:
    # testdouble = 0:pi/4:2*pi stored as a 9 x 1 float64 dataset
    with H5File(HDF5_MAT) as f:
        assert f.base == 512
        d = f["testdouble"]
        assert d.attrs["MATLAB_class"] == b"double"
        np.testing.assert_array_equal(d.read()[:, 0], np.arange(9) * (np.pi / 4))


def _weights(n_layers, seed=0):
    rng = np.random.default_rng(seed)
    order = [f"layer_{i:03d}" for i in range(n_layers)]
    weights = {n: [(f"{n}/kernel:0", rng.standard_normal((3, 4)).astype(np.float32)),
                   (f"{n}/bias:0", rng.standard_normal((4,)).astype(np.float32))]
               for n in order[1:]}
    return order, weights


@pytest.mark.parametrize("opts", [dict(leaf_k=2, internal_k=2), dict(leaf_k=4, internal_k=16),
                                  dict(userblock=512), dict(weights_only=True)])
def test_writer_edge_cases_round_trip(tmp_path, opts):
    order, weights = _weights(70)
    p = str(tmp_path / "m.h5")
    write_keras_model(p, weights, order, model_config={"a": 1}, **opts)
    got, cfg = read_keras_weights(p)
    exp = {k.split(":")[0]: v for ws in weights.values() for k, v in ws}
    assert list(got) == list(exp)                    # the file's layer / weight order
    for k in exp:
        assert np.array_equal(got[k], exp[k])
    assert cfg == (None if opts.get("weights_only") else {"a": 1})


def test_split_attribute_and_scalar_dataset(tmp_path):
    w = H5Writer()
    g = w.group("")
    g.attrs["layer_names0"] = np.array([b"a", b"b"])
    g.attrs["layer_names1"] = np.array([b"c"])
    for n in "abc":
        w.group(n).attrs["weight_names"] = np.array([f"{n}/w:0".encode()])
        w.dataset(f"{n}/{n}/w:0", np.float32(ord(n)).reshape(()))
    p = str(tmp_path / "s.h5")
    w.save(p)
    got, _ = read_keras_weights(p)
    assert list(got) == ["a/w", "b/w", "c/w"] and got["c/w"].shape == () and float(got["c/w"]) == ord("c")


def test_errors(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file" * 64)
    with pytest.raises(H5Error):
        H5File(str(p))
    w = H5Writer()
    w.dataset("d", np.zeros(3, np.float32))
    w.save(str(p))
    with pytest.raises(H5Error, match="layer_names"):
        read_keras_weights(str(p))


def _self_continuing_file(path):
    """A minimal superblock-v0 file whose root object header (v1) holds only a continuation
    message pointing back at its own message block: a crafted header chain that loops."""
    import struct
    A = 96                                        # root object header address
    sb = (b"\x89HDF\r\n\x1a\n" + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0)
          + struct.pack("<QQQQ", 0, 0xFFFFFFFFFFFFFFFF, 4096, 0xFFFFFFFFFFFFFFFF)
          + struct.pack("<QQII16x", 0, A, 0, 0))
    msg = struct.pack("<HHB3x", 0x10, 16, 0) + struct.pack("<QQ", A + 16, 24)
    hdr = struct.pack("<BBHII4x", 1, 0, 1, 1, len(msg)) + msg
    buf = bytearray(4096)
    buf[:len(sb)] = sb
    buf[A:A + len(hdr)] = hdr
    path.write_bytes(bytes(buf))


def test_continuation_loop_is_refused(tmp_path):
    """A header continuation chain that loops back on itself raises H5Error instead of
    walking forever (load_weights of an untrusted file must return)."""
    p = tmp_path / "loop.h5"
    _self_continuing_file(p)
    with pytest.raises(H5Error, match="continuation"):
        H5File(str(p))
