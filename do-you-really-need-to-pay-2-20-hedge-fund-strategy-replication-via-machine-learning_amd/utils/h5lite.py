"""Minimal, read-only HDF5 parser for Keras 2.x ``.h5`` model files (no h5py dependency).

``h5py`` is not installed in this environment, yet the reference ships its trained generators
as Keras HDF5 files (GAN/trained_generator/*.h5).  This module implements exactly
the subset of the HDF5 format those files use — superblock v0, v1 object headers (with
continuation blocks), symbol-table groups (v1 B-trees, local heaps, SNOD nodes), contiguous /
compact datasets of little-endian floats/ints, fixed and variable-length (global-heap) string
attributes — and nothing else.  It only reads bytes and decodes numbers/strings: no code in the
file is executed.

:func:`read_keras_model` returns ``{"config", "weights", "weight_names", "keras_model_config"}``
in the same shape as :func:`hfrep.utils.checkpoint.read_generator_payload`.
"""
from __future__ import annotations

import json
import struct

import numpy as np


class H5Error(ValueError):
    pass


class _Object:
    def __init__(self, f: "H5File", addr: int):
        self.f, self.addr = f, addr
        self.msgs = f._messages(addr)

    def _find(self, mtype):
        return [d for t, d in self.msgs if t == mtype]

    @property
    def attrs(self) -> dict:
        out = {}
        for d in self._find(0x000C):
            name, val = self.f._attribute(d)
            out[name] = val
        return out

    def is_group(self) -> bool:
        return bool(self._find(0x0011))

    def children(self) -> dict:
        st = self._find(0x0011)
        if not st:
            raise H5Error("not a group")
        btree, heap = struct.unpack_from("<QQ", st[0], 0)
        return self.f._group_entries(btree, heap)

    def __getitem__(self, path: str):
        obj = self
        for part in [p for p in path.split("/") if p]:
            ch = obj.children()
            if part not in ch:
                raise KeyError(path)
            obj = _Object(self.f, ch[part])
        return obj

    def read(self) -> np.ndarray:
        dt = self.f._datatype(self._find(0x0003)[0])
        shape = self.f._dataspace(self._find(0x0001)[0])
        raw = self.f._layout_data(self._find(0x0008)[0], int(np.prod(shape)) * dt.itemsize if shape else dt.itemsize)
        arr = np.frombuffer(raw, dtype=dt, count=int(np.prod(shape)) if shape else 1)
        return arr.reshape(shape).copy()


class H5File:
    def __init__(self, path: str):
        self.buf = open(path, "rb").read()
        if self.buf[:8] != b"\x89HDF\r\n\x1a\n":
            raise H5Error("not an HDF5 file")
        if self.buf[8] != 0:
            raise H5Error(f"superblock version {self.buf[8]} unsupported (only v0)")
        if self.buf[13] != 8 or self.buf[14] != 8:
            raise H5Error("only 8-byte offsets/lengths supported")
        # root group symbol table entry at byte 56: (link name off, header addr, cache type, ...)
        _, hdr = struct.unpack_from("<QQ", self.buf, 56)
        self.root = _Object(self, hdr)

    # ---- object headers ------------------------------------------------------------------
    def _messages(self, addr: int):
        b = self.buf
        ver = b[addr]
        if ver != 1:
            raise H5Error(f"object header version {ver} unsupported")
        nmsg = struct.unpack_from("<H", b, addr + 2)[0]
        size = struct.unpack_from("<I", b, addr + 8)[0]
        blocks = [(addr + 16, size)]
        msgs = []
        while blocks and len(msgs) < nmsg:
            start, length = blocks.pop(0)
            p, end = start, start + length
            while p + 8 <= end and len(msgs) < nmsg:
                mtype, msize, _flags = struct.unpack_from("<HHB", b, p)
                data = b[p + 8:p + 8 + msize]
                p += 8 + msize
                if mtype == 0x0010:  # continuation
                    caddr, clen = struct.unpack_from("<QQ", data, 0)
                    blocks.append((caddr, clen))
                msgs.append((mtype, data))
        return msgs

    # ---- groups ----------------------------------------------------------------------------
    def _heap_name(self, heap_addr: int, off: int) -> str:
        b = self.buf
        if b[heap_addr:heap_addr + 4] != b"HEAP":
            raise H5Error("bad local heap")
        data_addr = struct.unpack_from("<Q", b, heap_addr + 24)[0]
        s = data_addr + off
        e = b.index(b"\x00", s)
        return b[s:e].decode()

    def _group_entries(self, btree: int, heap: int) -> dict:
        b = self.buf
        out = {}
        stack = [btree]
        while stack:
            node = stack.pop()
            if b[node:node + 4] != b"TREE":
                raise H5Error("bad B-tree node")
            ntype, level = b[node + 4], b[node + 5]
            used = struct.unpack_from("<H", b, node + 6)[0]
            if ntype != 0:
                raise H5Error("expected a group B-tree")
            p = node + 24 + 8  # skip header + key0
            children = []
            for _ in range(used):
                children.append(struct.unpack_from("<Q", b, p)[0])
                p += 16  # child + next key
            if level > 0:
                stack.extend(children)
                continue
            for snod in children:
                if b[snod:snod + 4] != b"SNOD":
                    raise H5Error("bad symbol node")
                nsym = struct.unpack_from("<H", b, snod + 6)[0]
                q = snod + 8
                for _ in range(nsym):
                    name_off, hdr = struct.unpack_from("<QQ", b, q)
                    out[self._heap_name(heap, name_off)] = hdr
                    q += 40
        return out

    # ---- datatypes / dataspaces / layouts -----------------------------------------------------
    def _datatype(self, d: bytes):
        cls = d[0] & 0x0F
        bits0 = d[1]
        size = struct.unpack_from("<I", d, 4)[0]
        if cls == 1:  # float
            if bits0 & 1:
                raise H5Error("big-endian floats unsupported")
            return np.dtype({4: "<f4", 8: "<f8", 2: "<f2"}[size])
        if cls == 0:  # fixed-point
            signed = bool(bits0 & 0x08)
            return np.dtype(("<i" if signed else "<u") + str(size))
        if cls == 3:  # fixed-length string
            return np.dtype(f"S{size}")
        if cls == 9:  # variable length
            return ("vlen", (bits0 & 0x0F) == 1, size)
        raise H5Error(f"datatype class {cls} unsupported")

    def _dataspace(self, d: bytes):
        ver, ndim, flags = d[0], d[1], d[2]
        if ver == 1:
            p = 8
        elif ver == 2:
            p = 4
        else:
            raise H5Error(f"dataspace version {ver}")
        if ver == 2 and d[3] == 0:  # scalar
            return ()
        return tuple(struct.unpack_from("<Q", d, p + 8 * i)[0] for i in range(ndim))

    def _layout_data(self, d: bytes, nbytes: int) -> bytes:
        ver = d[0]
        if ver == 3:
            cls = d[1]
            if cls == 0:
                sz = struct.unpack_from("<H", d, 2)[0]
                return d[4:4 + sz]
            if cls == 1:
                addr, sz = struct.unpack_from("<QQ", d, 2)
                if addr == 0xFFFFFFFFFFFFFFFF:
                    return b"\x00" * nbytes
                return self.buf[addr:addr + sz]
            raise H5Error("chunked datasets unsupported")
        if ver in (1, 2):
            ndim, cls = d[1], d[2]
            p = 8
            if cls != 0:
                addr = struct.unpack_from("<Q", d, p)[0]
                return self.buf[addr:addr + nbytes]
            p += 4 * ndim
            sz = struct.unpack_from("<I", d, p)[0]
            return d[p + 4:p + 4 + sz]
        raise H5Error(f"layout version {ver}")

    def _gheap_object(self, coll: int, idx: int) -> bytes:
        b = self.buf
        if b[coll:coll + 4] != b"GCOL":
            raise H5Error("bad global heap")
        size = struct.unpack_from("<Q", b, coll + 8)[0]
        p, end = coll + 16, coll + size
        while p + 16 <= end:
            oid, _rc = struct.unpack_from("<HH", b, p)
            osz = struct.unpack_from("<Q", b, p + 8)[0]
            if oid == idx:
                return b[p + 16:p + 16 + osz]
            if oid == 0:
                break
            p += 16 + ((osz + 7) // 8) * 8
        raise H5Error("global heap object not found")

    def _attribute(self, d: bytes):
        ver = d[0]
        name_sz, dt_sz, ds_sz = struct.unpack_from("<HHH", d, 2)
        if ver == 1:
            pad = lambda n: (n + 7) // 8 * 8  # noqa: E731
            p = 8
            name = d[p:p + name_sz].rstrip(b"\x00").decode()
            p += pad(name_sz)
            dtb = d[p:p + dt_sz]
            p += pad(dt_sz)
            dsb = d[p:p + ds_sz]
            p += pad(ds_sz)
        elif ver in (2, 3):
            p = 8 if ver == 2 else 9
            name = d[p:p + name_sz].rstrip(b"\x00").decode()
            p += name_sz
            dtb = d[p:p + dt_sz]
            p += dt_sz
            dsb = d[p:p + ds_sz]
            p += ds_sz
        else:
            raise H5Error(f"attribute version {ver}")
        dt = self._datatype(dtb)
        shape = self._dataspace(dsb)
        n = int(np.prod(shape)) if shape else 1
        if isinstance(dt, tuple):  # vlen
            _, is_str, _ = dt
            vals = []
            for i in range(n):
                ln, coll, idx = struct.unpack_from("<IQI", d, p + 16 * i)
                raw = self._gheap_object(coll, idx)[: ln if is_str else None]
                vals.append(raw.decode() if is_str else raw)
            return name, (vals[0] if not shape else vals)
        arr = np.frombuffer(d[p:p + n * dt.itemsize], dtype=dt, count=n)
        if dt.kind == "S":
            vals = [x.rstrip(b"\x00").decode() for x in arr]
            return name, (vals[0] if not shape else vals)
        return name, (arr[0] if not shape else arr.reshape(shape))


def read_keras_model(path: str) -> dict:
    """Read a Keras 2.x ``model.save(...h5)`` generator into an hfrep generator payload."""
    f = H5File(path)
    attrs = f.root.attrs
    mc = json.loads(attrs["model_config"])
    mw = f.root["model_weights"]
    names, weights = [], []
    for layer in mw.attrs.get("layer_names", []):
        g = mw[layer]
        for wn in g.attrs.get("weight_names", []):
            names.append(wn)
            weights.append(g[wn].read().astype(np.float32))
    # infer the generator architecture from the (nested) Keras config
    layers = mc["config"]["layers"]
    seq = next((l for l in layers if l["class_name"] == "Sequential"), None)
    inner = seq["config"]["layers"] if seq else layers
    kinds = [l["class_name"] for l in inner if l["class_name"] != "InputLayer"]
    inp = None
    for l in layers:
        if l["class_name"] == "InputLayer":
            inp = l["config"]["batch_input_shape"]
    T, F = int(inp[1]), int(inp[2])
    if "LSTM" in kinds:
        arch = "lstm"
        hidden = next(l["config"]["units"] for l in inner if l["class_name"] == "LSTM")
        lrelu_first = kinds[:2] == ["LSTM", "LeakyReLU"]
    else:
        arch = "mlp"
        hidden = next(l["config"]["units"] for l in inner if l["class_name"] == "Dense")
        lrelu_first = False
    out_units = next(l["config"]["units"] for l in reversed(inner) if l["class_name"] == "Dense")
    cfg = {"arch": arch, "window": T, "features": int(out_units), "hidden": int(hidden),
           "lrelu_after_first": bool(lrelu_first), "keras_layers": kinds,
           "keras_version": attrs.get("keras_version"), "source": "keras-h5"}
    return {"format": "keras-h5", "config": cfg, "weight_names": names, "weights": weights,
            "keras_model_config": mc}
