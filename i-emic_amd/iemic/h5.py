"""Minimal HDF5 reader/writer for the Model state files.

The reference writes its states with EpetraExt::HDF5 (Model::saveStateToFile,
src/utils/Model.H:254-330; Ocean's extra fields, Ocean.C:1904-2113): groups "State"
(an Epetra_MultiVector: datasets "Values", "GlobalLength", "NumVectors", attribute
"__type__"), "Parameters" (one scalar dataset per continuation parameter) and "Grid"
(n, m, l, nun, aux, bounds, hdim and the coordinate arrays).  libhdf5 / h5py are not
available to this build, so this module reads and writes the subset of the HDF5 file
format those files use:

* superblock version 0, 8-byte offsets and lengths;
* groups as symbol tables (version-1 B-tree "TREE", local heap "HEAP", symbol nodes "SNOD");
* version-1 object headers with dataspace, datatype (IEEE float / little-endian integer /
  fixed string), fill value, data layout (contiguous or compact) and attribute messages.

It reads the reference's own test/ocean/ocean_reference.h5 and writes files it reads back;
the written layout follows the same conventions (one B-tree leaf per group, contiguous
little-endian datasets).  Not a general HDF5 implementation: chunked/compressed data,
dense (fractal-heap) groups and superblock versions > 0 are rejected loudly.
"""
from __future__ import annotations

import struct
from typing import Dict, Optional, Tuple, Union

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF
LEAF_K = 64        # group leaf node K: a symbol node holds up to 2K entries
NODE_K = 16        # group internal node K: a B-tree node has room for 2K children


class H5Error(RuntimeError):
    pass


# ------------------------------------------------------------------------------------
# reading

class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        if data[:8] != SIG:
            raise H5Error("not an HDF5 file")
        if data[8] != 0:
            raise H5Error(f"superblock version {data[8]} not supported (only 0)")
        if data[13] != 8 or data[14] != 8:
            raise H5Error("only 8-byte offsets/lengths are supported")
        self.base = struct.unpack_from("<Q", data, 24)[0]
        # root group symbol table entry at 56
        self.root = self._entry(56)

    def u8(self, o):
        return self.d[o]

    def q(self, o):
        return struct.unpack_from("<Q", self.d, o)[0]

    def _entry(self, o):
        name_off, hdr, cache = struct.unpack_from("<QQI", self.d, o)
        scratch = self.d[o + 24:o + 40]
        return {"name_off": name_off, "header": hdr, "cache": cache, "scratch": scratch}

    def _heap_name(self, heap_addr, off):
        if self.d[heap_addr:heap_addr + 4] != b"HEAP":
            raise H5Error("bad local heap")
        data_addr = self.q(heap_addr + 24)
        end = self.d.index(b"\x00", data_addr + off)
        return self.d[data_addr + off:end].decode()

    def _messages(self, addr):
        d = self.d
        if d[addr] != 1:
            raise H5Error(f"object header version {d[addr]} not supported")
        nmsg = struct.unpack_from("<H", d, addr + 2)[0]
        size = struct.unpack_from("<I", d, addr + 8)[0]
        msgs = []
        blocks = [(addr + 16, size)]
        while blocks and len(msgs) < nmsg:
            o, sz = blocks.pop(0)
            end = o + sz
            while o + 8 <= end and len(msgs) < nmsg:
                mtype, msize, flags = struct.unpack_from("<HHB", d, o)
                body = d[o + 8:o + 8 + msize]
                if mtype == 0x10:                               # continuation
                    blocks.append((struct.unpack_from("<Q", body, 0)[0], struct.unpack_from("<Q", body, 8)[0]))
                msgs.append((mtype, body))
                o += 8 + msize
        return msgs

    def _children(self, btree, heap):
        """name -> symbol table entry of a symbol-table group"""
        out = {}
        d = self.d
        stack = [btree]
        while stack:
            node = stack.pop()
            if d[node:node + 4] != b"TREE":
                raise H5Error("bad B-tree node")
            ntype, level, used = d[node + 4], d[node + 5], struct.unpack_from("<H", d, node + 6)[0]
            if ntype != 0:
                raise H5Error("unexpected B-tree node type")
            o = node + 24
            for i in range(used):
                child = self.q(o + 8 + 16 * i)
                if level > 0:
                    stack.append(child)
                    continue
                if d[child:child + 4] != b"SNOD":
                    raise H5Error("bad symbol node")
                nsym = struct.unpack_from("<H", d, child + 6)[0]
                for k in range(nsym):
                    e = self._entry(child + 8 + 40 * k)
                    out[self._heap_name(heap, e["name_off"])] = e
        return out

    def group(self, header):
        for mtype, body in self._messages(header):
            if mtype == 0x11:
                btree, heap = struct.unpack_from("<QQ", body, 0)
                return self._children(btree, heap)
            if mtype in (0x02, 0x06, 0x0A):
                raise H5Error("new-style (link/dense) groups are not supported")
        return None

    def _dtype(self, body):
        cls = body[0] & 0x0F
        size = struct.unpack_from("<I", body, 4)[0]
        bits = body[1] | (body[2] << 8) | (body[3] << 16)
        if cls == 1:                                            # IEEE float
            if bits & 1:
                raise H5Error("big-endian floats are not supported")
            return np.dtype("<f8" if size == 8 else "<f4")
        if cls == 0:                                            # fixed point
            signed = bool(bits & 0x08)
            if bits & 1:
                raise H5Error("big-endian integers are not supported")
            return np.dtype(("<i" if signed else "<u") + str(size))
        if cls == 3:                                            # fixed-length string
            return np.dtype(f"S{size}")
        raise H5Error(f"datatype class {cls} not supported")

    def _dspace(self, body):
        ver, rank, flags = body[0], body[1], body[2]
        o = 8 if ver == 1 else 4
        return tuple(struct.unpack_from("<Q", body, o + 8 * i)[0] for i in range(rank))

    def dataset(self, header):
        shape = dt = None
        raw = None
        attrs = {}
        for mtype, body in self._messages(header):
            if mtype == 0x01:
                shape = self._dspace(body)
            elif mtype == 0x03:
                dt = self._dtype(body)
            elif mtype == 0x08:
                ver = body[0]
                if ver != 3:
                    raise H5Error(f"layout message version {ver} not supported")
                cls = body[1]
                if cls == 1:
                    addr, size = struct.unpack_from("<QQ", body, 2)
                    raw = (addr, size)
                elif cls == 0:
                    n = struct.unpack_from("<H", body, 2)[0]
                    raw = bytes(body[4:4 + n])
                else:
                    raise H5Error("chunked datasets are not supported")
            elif mtype == 0x0C:
                k, v = self._attribute(body)
                attrs[k] = v
        if shape is None or dt is None or raw is None:
            raise H5Error("incomplete dataset header")
        count = int(np.prod(shape)) if shape else 1
        if isinstance(raw, tuple):
            addr, size = raw
            if addr == UNDEF:
                arr = np.zeros(count, dtype=dt)
            else:
                arr = np.frombuffer(self.d, dtype=dt, count=count, offset=addr).copy()
        else:
            arr = np.frombuffer(raw, dtype=dt, count=count).copy()
        return arr.reshape(shape) if shape else arr.reshape(()), attrs

    def _attribute(self, body):
        ver = body[0]
        if ver != 1:
            raise H5Error(f"attribute message version {ver} not supported")
        nlen, tlen, slen = struct.unpack_from("<HHH", body, 2)
        o = 8
        name = body[o:o + nlen].split(b"\x00")[0].decode()
        o += (nlen + 7) // 8 * 8
        dt = self._dtype(body[o:o + tlen])
        o += (tlen + 7) // 8 * 8
        shape = self._dspace(body[o:o + slen])
        o += (slen + 7) // 8 * 8
        count = int(np.prod(shape)) if shape else 1
        val = np.frombuffer(body, dtype=dt, count=count, offset=o)
        if dt.kind == "S":
            return name, val[0].split(b"\x00")[0].decode()
        return name, val.reshape(shape) if shape else val[0]

    def walk(self, header=None, prefix=""):
        """{path: (array, attrs)} of every dataset"""
        out = {}
        ch = self.group(self.root["header"] if header is None else header)
        for name, e in (ch or {}).items():
            path = f"{prefix}/{name}"
            sub = self.group(e["header"])
            if sub is not None:
                out.update(self.walk(e["header"], path))
            else:
                out[path] = self.dataset(e["header"])
        return out


def read(path: str) -> Dict[str, Tuple[np.ndarray, dict]]:
    """{"/Group/Dataset": (array, attributes)} of an HDF5 file in the supported subset"""
    with open(path, "rb") as f:
        return _Reader(f.read()).walk()


# ------------------------------------------------------------------------------------
# writing

def _pad8(b: bytes) -> bytes:
    return b + b"\x00" * ((-len(b)) % 8)


def _dtype_msg(dt: np.dtype) -> bytes:
    if dt.kind == "f":
        size = dt.itemsize
        if size == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        else:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        # class 1 version 1; bit field: little endian, pad 0, mantissa norm implied (0x20),
        # sign at bit 63 / 31
        sign = 63 if size == 8 else 31
        return bytes([0x11, 0x20, sign, 0]) + struct.pack("<I", size) + props
    if dt.kind in "iu":
        bits = 0x08 if dt.kind == "i" else 0
        return bytes([0x10, bits, 0, 0]) + struct.pack("<I", dt.itemsize) + struct.pack("<HH", 0, 8 * dt.itemsize)
    if dt.kind == "S":
        return bytes([0x13, 0, 0, 0]) + struct.pack("<I", dt.itemsize)
    raise H5Error(f"cannot write dtype {dt}")


def _dspace_msg(shape) -> bytes:
    b = bytes([1, len(shape), 0, 0]) + b"\x00" * 4
    for n in shape:
        b += struct.pack("<Q", n)
    return b


class _Writer:
    def __init__(self):
        self.buf = bytearray(b"\x00" * 96)            # superblock (v0) + root entry

    def alloc(self, data: bytes, align: int = 8) -> int:
        while len(self.buf) % align:
            self.buf += b"\x00"
        a = len(self.buf)
        self.buf += data
        return a

    def header(self, msgs) -> int:
        body = b""
        for mtype, data in msgs:
            data = _pad8(data)
            body += struct.pack("<HHB3x", mtype, len(data), 0) + data
        hdr = struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body))
        return self.alloc(hdr + body)

    def dataset(self, arr: np.ndarray, attrs: Optional[dict] = None) -> int:
        arr = np.ascontiguousarray(arr)
        if arr.dtype.byteorder == ">":
            arr = arr.astype(arr.dtype.newbyteorder("<"))
        addr = self.alloc(arr.tobytes())
        msgs = [(0x01, _dspace_msg(arr.shape)), (0x03, _dtype_msg(arr.dtype)),
                (0x05, bytes([2, 2, 2, 0])),          # fill value v2: never written, undefined
                (0x08, bytes([3, 1]) + struct.pack("<QQ", addr, arr.nbytes))]
        for name, val in (attrs or {}).items():
            msgs.append((0x0C, self._attr(name, val)))
        return self.header(msgs)

    def _attr(self, name: str, val) -> bytes:
        if isinstance(val, str):
            raw = val.encode() + b"\x00"
            arr = np.frombuffer(raw, dtype=f"S{len(raw)}")
            shape = ()
        else:
            arr = np.atleast_1d(np.asarray(val))
            shape = np.shape(val)
        nm = name.encode() + b"\x00"
        dt = _dtype_msg(arr.dtype)
        ds = _dspace_msg(shape)
        return (struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds)) + _pad8(nm) + _pad8(dt) + _pad8(ds)
                + arr.tobytes())

    def group(self, children: Dict[str, int]) -> Tuple[int, int, int]:
        """children: name -> object header address; returns (header, btree, heap)"""
        names = sorted(children)
        heap_data = b"\x00" * 8                         # offset 0: the empty name
        offs = {}
        for nme in names:
            offs[nme] = len(heap_data)
            heap_data += _pad8(nme.encode() + b"\x00")
        heap_seg = self.alloc(heap_data)
        heap = self.alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap_data), UNDEF, heap_seg))
        if len(names) > 2 * LEAF_K:
            raise H5Error(f"more than {2 * LEAF_K} members in one group")
        ents = b""
        for nme in names:
            ents += struct.pack("<QQI4x16x", offs[nme], children[nme], 0)
        ents += b"\x00" * (40 * (2 * LEAF_K - len(names)))      # full-size symbol node
        snod = self.alloc(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names)) + ents)
        # one leaf: key0 (empty name), child, key1 (largest name); node sized for 2K children
        last = offs[names[-1]] if names else 0
        tree = (b"TREE" + bytes([0, 0]) + struct.pack("<H", 1) + struct.pack("<QQ", UNDEF, UNDEF) +
                struct.pack("<QQQ", 0, snod, last))
        tree += b"\x00" * (24 + 8 * (2 * NODE_K + 1) + 8 * 2 * NODE_K - len(tree))
        btree = self.alloc(tree)
        hdr = self.header([(0x11, struct.pack("<QQ", btree, heap))])
        return hdr, btree, heap

    def finish(self, root_children: Dict[str, int]) -> bytes:
        hdr, btree, heap = self.group(root_children)
        sb = SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HH", LEAF_K, NODE_K) + struct.pack("<I", 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, len(self.buf), UNDEF)
        sb += struct.pack("<QQI4x", 0, hdr, 1) + struct.pack("<QQ", btree, heap)
        assert len(sb) == 96
        self.buf[0:96] = sb
        return bytes(self.buf)


Tree = Dict[str, Union["Tree", np.ndarray, Tuple[np.ndarray, dict]]]


def write(path: str, tree: Tree) -> None:
    """tree: {group: {name: array | (array, attrs) | subgroup-dict}}, nested"""
    w = _Writer()

    def build(node: Tree) -> Dict[str, int]:
        out = {}
        for name, v in node.items():
            if isinstance(v, dict):
                out[name] = w.group(build(v))[0]
            elif isinstance(v, tuple):
                out[name] = w.dataset(np.asarray(v[0]), v[1])
            else:
                out[name] = w.dataset(np.asarray(v))
        return out
    data = w.finish(build(tree))
    with open(path, "wb") as f:
        f.write(data)
