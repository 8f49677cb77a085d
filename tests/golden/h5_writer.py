"""Minimal HDF5 writer (test infrastructure): produces the file structures that h5py at its
default settings (libver 'earliest') writes for a Keras 2.x weight file -- version 0
superblock, version 1 object headers, symbol-table groups (v1 B-tree + local heap +
symbol-table nodes), fixed-length string / numeric attributes, contiguous datasets --
so that `vision_transformer_detector_amd.keras_h5` can be tested without h5py.

`leaf_k` / `internal_k` are the superblock's group B-tree parameters: small values force
several symbol-table nodes and a two-level B-tree in a group with many links.
"""
import struct

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF


def _pad8(b):
    return b + b"\0" * (-len(b) % 8)


def _dtype_msg(arr):
    dt = arr.dtype
    if dt.kind == "S":
        return struct.pack("<B3sI", 0x13, b"\0\0\0", max(1, dt.itemsize))
    if dt.kind == "f":
        n = dt.itemsize
        e, m, bias = {2: (5, 10, 15), 4: (8, 23, 127), 8: (11, 52, 1023)}[n]
        bits = bytes([0x20, 8 * n - 1, 0])
        return (struct.pack("<B3sI", 0x11, bits, n) +
                struct.pack("<HHBBBBI", 0, 8 * n, m, e, 0, m, bias))
    if dt.kind in "iu":
        n = dt.itemsize
        bits = bytes([0x08 if dt.kind == "i" else 0, 0, 0])
        return struct.pack("<B3sI", 0x10, bits, n) + struct.pack("<HH", 0, 8 * n)
    raise ValueError(dt)


def _space_msg(shape):
    return struct.pack("<BBB5x", 1, len(shape), 0) + b"".join(struct.pack("<Q", d) for d in shape)


class _Group:
    def __init__(self):
        self.children = {}     # name -> _Group | np.ndarray
        self.attrs = {}


class H5Writer:
    def __init__(self, leaf_k=4, internal_k=16, userblock=0):
        self.root = _Group()
        self.leaf_k, self.internal_k, self.userblock = leaf_k, internal_k, userblock

    def group(self, path):
        g = self.root
        for p in [p for p in path.split("/") if p]:
            g = g.children.setdefault(p, _Group())
        return g

    def dataset(self, path, arr):
        *parent, name = [p for p in path.split("/") if p]
        self.group("/".join(parent)).children[name] = np.array(arr, order="C")

    # ------------------------------------------------------------------ layout
    def _alloc(self, data):
        addr = len(self.buf)
        self.buf += _pad8(data)
        return addr

    def _attr_msg(self, name, val):
        if isinstance(val, (bytes, str)):
            v = val.encode() if isinstance(val, str) else val
            arr = np.array(v, dtype=f"S{max(1, len(v))}")
        else:
            arr = np.asarray(val)
            if arr.dtype.kind == "U":
                arr = arr.astype("S")
        nm = name.encode() + b"\0"
        dt = _dtype_msg(arr)
        sp = _space_msg(arr.shape)
        body = (struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(sp)) + _pad8(nm) + _pad8(dt) +
                _pad8(sp) + arr.tobytes())
        return 0x0C, body

    def _header(self, msgs):
        body = b""
        for t, d in msgs:
            d = _pad8(d)
            body += struct.pack("<HHB3x", t, len(d), 0) + d
        hdr = struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body))
        return self._alloc(hdr + body)

    def _write_dataset(self, arr):
        addr = self._alloc(arr.tobytes()) if arr.nbytes else UNDEF
        layout = struct.pack("<BBQQ", 3, 1, addr, arr.nbytes)
        return self._header([(0x01, _space_msg(arr.shape)), (0x03, _dtype_msg(arr)),
                             (0x08, layout)])

    def _write_group(self, g):
        names = sorted(g.children)
        addrs = {n: (self._write_group(c) if isinstance(c, _Group) else self._write_dataset(c))
                 for n, c in ((n, g.children[n]) for n in names)}
        heap = b"\0" * 8
        offs = {}
        for n in names:
            offs[n] = len(heap)
            heap += _pad8(n.encode() + b"\0")
        heap_data = self._alloc(heap)
        heap_hdr = self._alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), UNDEF, heap_data))
        per = 2 * self.leaf_k
        snods = []
        for i in range(0, max(1, len(names)), per):
            chunk = names[i:i + per]
            ent = b"".join(struct.pack("<QQII16x", offs[n], addrs[n], 0, 0) for n in chunk)
            ent += b"\0" * (40 * (per - len(chunk)))
            snods.append((self._alloc(b"SNOD" + struct.pack("<BBH", 1, 0, len(chunk)) + ent),
                          offs[chunk[-1]] if chunk else 0))

        def node(level, kids):
            # kids: [(addr, key of its last name)]; key 0 = the heap's empty string
            body = struct.pack("<Q", 0)
            for a, k in kids:
                body += struct.pack("<QQ", a, k)
            return (self._alloc(b"TREE" + struct.pack("<BBHQQ", 0, level, len(kids), UNDEF, UNDEF)
                                + body), kids[-1][1])

        fan = 2 * self.internal_k
        level, nodes = 0, snods
        while True:
            nodes = [node(level, nodes[i:i + fan]) for i in range(0, len(nodes), fan)]
            if len(nodes) == 1:
                break
            level += 1
        msgs = [(0x11, struct.pack("<QQ", nodes[0][0], heap_hdr))]
        msgs += [self._attr_msg(k, v) for k, v in g.attrs.items()]
        return self._header(msgs)

    def save(self, path):
        self.buf = bytearray(96)                   # superblock v0 + root symbol-table entry
        root = self._write_group(self.root)
        sb = (b"\x89HDF\r\n\x1a\n" + bytes([0, 0, 0, 0, 0, 8, 8, 0]) +
              struct.pack("<HHI", self.leaf_k, self.internal_k, 0) +
              struct.pack("<QQQQ", 0, UNDEF, len(self.buf), UNDEF) +
              struct.pack("<QQII16x", 0, root, 0, 0))
        self.buf[:96] = sb
        with open(path, "wb") as f:
            f.write(b"\0" * self.userblock + bytes(self.buf))


def write_keras_model(path, weights, layer_order, model_config=None, weights_only=False,
                      **kw):
    """Keras 2.9 `model.save('*.h5' / '*.keras')` layout (keras/saving/hdf5_format.py):
    weights = {layer: [(weight name with ':0', array), ...]} for every layer in
    `layer_order` (layers without weights get an empty list)."""
    w = H5Writer(**kw)
    base = "" if weights_only else "model_weights"
    root = w.group(base)
    if not weights_only:
        w.root.attrs["keras_version"] = b"2.9.0"
        w.root.attrs["backend"] = b"tensorflow"
        if model_config is not None:
            import json
            w.root.attrs["model_config"] = json.dumps(model_config).encode()
    root.attrs["layer_names"] = np.array([n.encode() for n in layer_order])
    root.attrs["backend"] = b"tensorflow"
    root.attrs["keras_version"] = b"2.9.0"
    for layer in layer_order:
        g = w.group(f"{base}/{layer}")
        ws = weights.get(layer, [])
        g.attrs["weight_names"] = (np.array([n.encode() for n, _ in ws]) if ws
                                   else np.zeros((0,), np.float64))
        for n, a in ws:
            w.dataset(f"{base}/{layer}/{n}", np.asarray(a, np.float32))
    w.save(path)
