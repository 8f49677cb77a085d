"""Read-only HDF5 reader for Keras weight files (`model.save('*.keras')` / `'*.h5'` under
TF 2.9, vtd.py:2146, 2179; `model.save_weights('*.h5')`), with no dependency on h5py or
the HDF5 library and nothing executed from the file: it parses the on-disk structures of
the HDF5 file format specification (version 0-3 superblocks, version 1 and 2 object
headers, symbol-table and compact-link groups, contiguous and compact datasets,
attributes) and returns numpy arrays and strings.

Keras 2.9's HDF5 layout (keras/saving/hdf5_format.py, the save path the reference's
callback takes):
  /                          attrs: keras_version, backend, model_config (JSON bytes), ...
  /model_weights             attrs: layer_names (fixed-length byte strings, in model order)
  /model_weights/<layer>     attrs: weight_names ("<layer>/.../kernel:0", ...)
  /model_weights/<layer>/<weight name>   dataset (the '/' in a weight name nests groups)
A weights-only file (`save_weights('*.h5')`) has the same layout rooted at `/`.
Attributes larger than 64 KiB are split by Keras into `<name>0`, `<name>1`, ...

Unsupported structures (dense attribute / link storage in fractal heaps, chunked or
filtered datasets, non-numeric element types) raise `H5Error` naming what was found;
h5py writes none of them for a Keras weight file at its default settings.
"""
import json
import mmap
import struct

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


_MAX_HEADER_CHUNKS = 4096     # continuation chunks followed per object header

class H5Error(ValueError):
    pass


class _Reader:
    """Little-endian cursor over the file bytes."""

    def __init__(self, buf, pos, so, sl):
        self.b, self.p, self.so, self.sl = buf, pos, so, sl

    def u(self, n):
        v = int.from_bytes(self.b[self.p:self.p + n], "little")
        self.p += n
        return v

    def off(self):
        return self.u(self.so)

    def length(self):
        return self.u(self.sl)

    def raw(self, n):
        v = bytes(self.b[self.p:self.p + n])
        self.p += n
        return v

    def skip(self, n):
        self.p += n

    def align(self, base, a=8):
        self.p = base + ((self.p - base + a - 1) // a) * a


# ------------------------------------------------------------------ datatypes
class Datatype:
    def __init__(self, cls, size, order="<", signed=False, strpad=0, base=None, vlen_str=False):
        self.cls, self.size, self.order = cls, size, order
        self.signed, self.strpad, self.base, self.vlen_str = signed, strpad, base, vlen_str

    def numpy(self):
        if self.cls == 0:
            return np.dtype(f"{self.order}{'i' if self.signed else 'u'}{self.size}")
        if self.cls == 1:
            return np.dtype(f"{self.order}f{self.size}")
        if self.cls == 3:
            return np.dtype(f"S{self.size}")
        raise H5Error(f"datatype class {self.cls} has no numpy equivalent here")


def _parse_datatype(r):
    b0 = r.u(1)
    cls, ver = b0 & 0x0F, b0 >> 4
    bits = r.u(3)
    size = r.u(4)
    if cls == 0:                                  # fixed-point
        r.skip(4)                                 # bit offset, precision
        return Datatype(0, size, ">" if bits & 1 else "<", signed=bool(bits & 8))
    if cls == 1:                                  # floating-point (IEEE layouts only)
        r.skip(12)
        if size not in (2, 4, 8):
            raise H5Error(f"float of {size} bytes")
        return Datatype(1, size, ">" if bits & 1 else "<")
    if cls == 3:                                  # fixed-length string
        return Datatype(3, size, strpad=bits & 0x0F)
    if cls == 9:                                  # variable-length (sequence or string)
        base = _parse_datatype(r)
        return Datatype(9, size, base=base, vlen_str=(bits & 0x0F) == 1)
    raise H5Error(f"unsupported datatype class {cls} (version {ver})")


def _parse_dataspace(r):
    ver = r.u(1)
    ndim = r.u(1)
    flags = r.u(1)
    if ver == 1:
        r.skip(5)
        dims = [r.length() for _ in range(ndim)]
        if flags & 1:
            r.skip(ndim * r.sl)
        if flags & 2:
            r.skip(ndim * r.sl)
        return tuple(dims)
    if ver == 2:
        kind = r.u(1)
        dims = [r.length() for _ in range(ndim)]
        if flags & 1:
            r.skip(ndim * r.sl)
        if kind == 2:
            return None                           # null dataspace
        return tuple(dims)
    raise H5Error(f"dataspace version {ver}")


# ------------------------------------------------------------------ objects
class Node:
    def __init__(self, f, addr, name):
        self.file, self.addr, self.name = f, addr, name
        self.attrs = {}


class Group(Node):
    def __init__(self, f, addr, name, links):
        super().__init__(f, addr, name)
        self._links = links                       # ordered {name: object header address}

    def keys(self):
        return list(self._links)

    def __contains__(self, key):
        try:
            self[key]
            return True
        except KeyError:
            return False

    def __getitem__(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            if not isinstance(node, Group) or part not in node._links:
                raise KeyError(f"{path!r}: no {part!r} in {node.name!r}")
            node = node.file._object(node._links[part], f"{node.name.rstrip('/')}/{part}")
        return node

    def visit_datasets(self, prefix=""):
        """(relative path, Dataset) of every dataset below this group, in link order."""
        for k in self._links:
            obj = self[k]
            if isinstance(obj, Dataset):
                yield prefix + k, obj
            else:
                yield from obj.visit_datasets(prefix + k + "/")


class Dataset(Node):
    def __init__(self, f, addr, name, dtype, shape, layout):
        super().__init__(f, addr, name)
        self.dtype_h5, self.shape, self._layout = dtype, shape, layout

    @property
    def dtype(self):
        return self.dtype_h5.numpy()

    def read(self):
        kind, a, b = self._layout
        n = int(np.prod(self.shape)) if self.shape else 1
        dt = self.dtype
        if kind == "contiguous":
            if a == UNDEF:                        # never written: the fill value (0)
                return np.zeros(self.shape, dt)
            data = self.file._bytes(a, n * dt.itemsize)
        elif kind == "compact":
            data = b[:n * dt.itemsize]
        else:
            raise H5Error(f"{self.name}: {kind} storage is not supported")
        out = np.frombuffer(data, dtype=dt, count=n).reshape(self.shape)
        return out.astype(dt.newbyteorder("=")) if dt.byteorder == ">" else out.copy()


class H5File(Group):
    """`H5File(path)`: the root group of an HDF5 file (read-only, memory-mapped)."""

    def __init__(self, path):
        self._fh = open(path, "rb")
        self._mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        buf = self._mm
        base = None
        for cand in [0] + [512 << i for i in range(16)]:     # user block: 0, 512, 1024, ...
            if cand + 8 <= len(buf) and buf[cand:cand + 8] == SIGNATURE:
                base = cand
                break
        if base is None:
            raise H5Error(f"{path}: not an HDF5 file (no signature)")
        self.buf, self.base = buf, base
        ver = buf[base + 8]
        if ver in (0, 1):
            so, sl = buf[base + 13], buf[base + 14]
            self.so, self.sl = so, sl
            r = _Reader(buf, base + 24 + (4 if ver == 1 else 0), so, sl)
            r.off()                               # base address (user block size)
            r.off()                               # free-space info
            r.off()                               # end of file
            r.off()                               # driver info
            r.off()                               # root entry: link name offset
            root = r.off()                        # root entry: object header address
        elif ver in (2, 3):
            so, sl = buf[base + 9], buf[base + 10]
            self.so, self.sl = so, sl
            r = _Reader(buf, base + 12, so, sl)
            r.off()                               # base address
            r.off()                               # superblock extension
            r.off()                               # end of file
            root = r.off()
        else:
            raise H5Error(f"superblock version {ver}")
        self._cache = {}
        obj = self._object(root, "/")
        if not isinstance(obj, Group):
            raise H5Error("root object is not a group")
        Node.__init__(self, self, root, "/")
        self._links, self.attrs = obj._links, obj.attrs

    def close(self):
        self._mm.close()
        self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # addresses are relative to the superblock (the base address)
    def _bytes(self, addr, n):
        a = self.base + addr
        if addr == UNDEF or a + n > len(self.buf):
            raise H5Error(f"address {addr:#x} + {n} beyond the end of the file")
        return self.buf[a:a + n]

    def _r(self, addr):
        if addr == UNDEF or self.base + addr >= len(self.buf):
            raise H5Error(f"bad address {addr:#x}")
        return _Reader(self.buf, self.base + addr, self.so, self.sl)

    # -------------------------------------------------------------- object headers
    def _messages(self, addr):
        """[(type, data bytes)] of the object header at addr, continuations followed."""
        r = self._r(addr)
        out = []
        if bytes(self.buf[r.p:r.p + 4]) == b"OHDR":
            r.skip(4)
            ver, flags = r.u(1), r.u(1)
            if ver != 2:
                raise H5Error(f"object header v{ver}")
            if flags & 0x20:
                r.skip(16)
            if flags & 0x10:
                r.skip(4)
            size = r.u(1 << (flags & 3))
            todo = [(r.p, size)]
            seen = set()
            while todo:
                start, n = todo.pop(0)
                # a crafted file could chain continuations in a loop: every chunk once, and
                # a bounded number of chunks
                if start in seen or len(seen) >= _MAX_HEADER_CHUNKS:
                    raise H5Error("object header continuation loop / too many chunks")
                seen.add(start)
                p, end = start, start + n
                while p + 4 <= end:
                    t = self.buf[p]
                    sz = int.from_bytes(self.buf[p + 1:p + 3], "little")
                    p += 4 + (2 if flags & 0x04 else 0)
                    data = bytes(self.buf[p:p + sz])
                    p += sz
                    if t == 0x10:
                        cr = _Reader(data, 0, self.so, self.sl)
                        ca, cl = cr.off(), cr.length()
                        cp = self.base + ca
                        if bytes(self.buf[cp:cp + 4]) != b"OCHK":
                            raise H5Error("bad continuation block")
                        todo.append((cp + 4, cl - 8))
                    elif t != 0:
                        out.append((t, data))
            return out
        ver = r.u(1)
        if ver != 1:
            raise H5Error(f"object header version {ver} at {addr:#x}")
        r.skip(1)
        nmsg = r.u(2)
        r.skip(4)
        size = r.u(4)
        r.skip(4)                                 # pad to 8 (header is 16 bytes)
        todo = [(r.p, size)]
        seen = set()
        while todo and len(out) < nmsg + 64:
            start, n = todo.pop(0)
            if start in seen or len(seen) >= _MAX_HEADER_CHUNKS:
                raise H5Error("object header continuation loop / too many chunks")
            seen.add(start)
            p, end = start, start + n
            while p + 8 <= end:
                t = int.from_bytes(self.buf[p:p + 2], "little")
                sz = int.from_bytes(self.buf[p + 2:p + 4], "little")
                data = bytes(self.buf[p + 8:p + 8 + sz])
                p += 8 + sz
                if t == 0x10:
                    cr = _Reader(data, 0, self.so, self.sl)
                    ca, cl = cr.off(), cr.length()
                    todo.append((self.base + ca, cl))
                elif t != 0:
                    out.append((t, data))
        return out

    def _object(self, addr, name):
        if addr in self._cache:
            obj = self._cache[addr]
            return obj
        msgs = self._messages(addr)
        types = {t for t, _ in msgs}
        attrs = {}
        for t, d in msgs:
            if t == 0x0C:
                k, v = self._attribute(d)
                attrs[k] = v
            elif t == 0x15:
                raise H5Error(f"{name}: dense attribute storage (fractal heap) is not supported")
        if 0x11 in types or 0x06 in types or 0x02 in types:
            links = {}
            for t, d in msgs:
                if t == 0x11:
                    r = _Reader(d, 0, self.so, self.sl)
                    btree, heap = r.off(), r.off()
                    links.update(self._symbol_table(btree, heap))
                elif t == 0x06:
                    k, a = self._link(d)
                    if a is not None:
                        links[k] = a
                elif t == 0x02:
                    r = _Reader(d, 0, self.so, self.sl)
                    r.skip(1)
                    fl = r.u(1)
                    if fl & 1:
                        r.skip(8)
                    heap_addr = r.off()
                    if heap_addr != UNDEF:
                        raise H5Error(f"{name}: dense link storage (fractal heap) is not supported")
            obj = Group(self, addr, name, links)
        elif 0x01 in types and 0x03 in types and 0x08 in types:
            shape = dtype = layout = None
            for t, d in msgs:
                r = _Reader(d, 0, self.so, self.sl)
                if t == 0x01:
                    shape = _parse_dataspace(r)
                elif t == 0x03:
                    dtype = _parse_datatype(r)
                elif t == 0x08:
                    layout = self._layout(d, shape)
                elif t == 0x0B:
                    raise H5Error(f"{name}: filtered (compressed) datasets are not supported")
            obj = Dataset(self, addr, name, dtype, shape or (), layout)
        else:
            raise H5Error(f"{name}: object with messages {sorted(types)} is neither a group "
                          "nor a dataset")
        obj.attrs = attrs
        self._cache[addr] = obj
        return obj

    def _layout(self, d, shape):
        r = _Reader(d, 0, self.so, self.sl)
        ver = r.u(1)
        if ver in (1, 2):
            ndim = r.u(1)
            cls = r.u(1)
            r.skip(5)
            addr = r.off() if cls != 0 else None
            r.skip(4 * ndim)
            if cls == 0:
                n = r.u(4)
                return ("compact", None, r.raw(n))
            if cls == 1:
                return ("contiguous", addr, None)
            return ("chunked", addr, None)
        if ver in (3, 4):
            cls = r.u(1)
            if cls == 0:
                n = r.u(2)
                return ("compact", None, r.raw(n))
            if cls == 1:
                return ("contiguous", r.off(), r.length())
            return ("chunked" if cls == 2 else "virtual", None, None)
        raise H5Error(f"data layout version {ver}")

    def _attribute(self, d):
        r = _Reader(d, 0, self.so, self.sl)
        ver = r.u(1)
        r.skip(1)
        nlen, tlen, slen = r.u(2), r.u(2), r.u(2)
        if ver == 3:
            r.skip(1)                             # name character set
        pad = ver == 1
        name = r.raw(nlen).split(b"\0", 1)[0].decode("utf-8")
        if pad:
            r.p = (r.p + 7) & ~7
        t0 = r.p
        dtype = _parse_datatype(r)
        r.p = t0 + tlen
        if pad:
            r.p = (r.p + 7) & ~7
        s0 = r.p
        shape = _parse_dataspace(r)
        r.p = s0 + slen
        if pad:
            r.p = (r.p + 7) & ~7
        if shape is None:
            return name, None
        n = int(np.prod(shape)) if shape else 1
        raw = d[r.p:]
        if dtype.cls == 9:
            vals = []
            for i in range(n):
                q = _Reader(raw, i * (4 + self.so + 4), self.so, self.sl)
                ln = q.u(4)
                coll, idx = q.off(), q.u(4)
                vals.append(self._global_heap(coll, idx)[:ln * dtype.base.size])
            if dtype.vlen_str:
                vals = [v.decode("utf-8") for v in vals]
            return name, (vals[0] if not shape else np.array(vals, dtype=object).reshape(shape))
        arr = np.frombuffer(raw, dtype=dtype.numpy(), count=n)
        if dtype.cls == 3:
            vals = [v.split(b"\0", 1)[0] if dtype.strpad < 2 else v.rstrip(b" ") for v in arr]
            return name, (vals[0] if not shape else np.array(vals, dtype=object).reshape(shape))
        arr = arr.astype(arr.dtype.newbyteorder("="))
        return name, (arr[0] if not shape else arr.reshape(shape))

    def _global_heap(self, coll, idx):
        r = self._r(coll)
        if r.raw(4) != b"GCOL":
            raise H5Error("bad global heap collection")
        r.skip(4)
        size = r.length()
        end = r.p - 8 - self.sl + size
        while r.p + 8 + self.sl <= end:
            i = r.u(2)
            r.skip(6)
            n = r.length()
            if i == 0:
                break
            if i == idx:
                return r.raw(n)
            r.skip((n + 7) & ~7)
        raise H5Error(f"global heap object {idx} not found")

    def _link(self, d):
        r = _Reader(d, 0, self.so, self.sl)
        r.skip(1)
        fl = r.u(1)
        ltype = r.u(1) if fl & 0x08 else 0
        if fl & 0x04:
            r.skip(8)
        if fl & 0x10:
            r.skip(1)
        n = r.u(1 << (fl & 3))
        name = r.raw(n).decode("utf-8")
        if ltype != 0:
            return name, None                     # soft / external links are not followed
        return name, r.off()

    def _symbol_table(self, btree, heap):
        h = self._r(heap)
        if h.raw(4) != b"HEAP":
            raise H5Error("bad local heap")
        h.skip(4)
        h.length()
        h.length()
        data_addr = h.off()
        links = {}

        def name_at(off):
            a = self.base + data_addr + off
            e = self.buf.find(b"\0", a)
            return bytes(self.buf[a:e]).decode("utf-8")

        def walk(addr, depth=0):
            if depth > 64:
                raise H5Error("group B-tree too deep")
            r = self._r(addr)
            if r.raw(4) != b"TREE":
                raise H5Error("bad group B-tree node")
            ntype, level, used = r.u(1), r.u(1), r.u(2)
            if ntype != 0:
                raise H5Error("not a group B-tree")
            r.off()
            r.off()
            children = []
            for _ in range(used):
                r.length()                        # key (heap offset)
                children.append(r.off())
            for c in children:
                if level > 0:
                    walk(c, depth + 1)
                else:
                    s = self._r(c)
                    if s.raw(4) != b"SNOD":
                        raise H5Error("bad symbol table node")
                    s.skip(2)
                    cnt = s.u(2)
                    for _ in range(cnt):
                        noff, oaddr = s.off(), s.off()
                        s.skip(24)
                        links[name_at(noff)] = oaddr

        walk(btree)
        return links


# ------------------------------------------------------------------ Keras layout
def _str(v):
    return v.decode("utf-8") if isinstance(v, (bytes, np.bytes_)) else str(v)


def keras_attribute(group, name):
    """A Keras list attribute, re-joined when Keras split it into name0, name1, ..."""
    if name in group.attrs:
        return [_str(v) for v in np.atleast_1d(group.attrs[name])]
    out, i = [], 0
    while f"{name}{i}" in group.attrs:
        out += [_str(v) for v in np.atleast_1d(group.attrs[f"{name}{i}"])]
        i += 1
    return out


def read_keras_weights(path):
    """{weight name without ':0' -> float32 array} and the file's model_config (a dict, or
    None) from a Keras 2.x HDF5 model or weights file, in the file's layer / weight order."""
    with H5File(path) as f:
        root = f["model_weights"] if "model_weights" in f.keys() else f
        layers = keras_attribute(root, "layer_names")
        if not layers:
            raise H5Error(f"{path}: no 'layer_names' attribute (not a Keras weight file)")
        out = {}
        for layer in layers:
            g = root[layer]
            names = keras_attribute(g, "weight_names")
            for wn in names:
                ds = g[wn]
                if not isinstance(ds, Dataset):
                    raise H5Error(f"{path}: {layer}/{wn} is not a dataset")
                out[wn.split(":")[0]] = ds.read().astype(np.float32)
        cfg = f.attrs.get("model_config")
        if cfg is not None:
            cfg = json.loads(_str(cfg))
        return out, cfg
