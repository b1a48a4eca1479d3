"""Minimal HDF5 reader / writer for Keras weight files (h5py is not in the image).

Keras 3 writes `*.weights.h5` (ModelCheckpoint(save_weights_only=True),
audiomodel.py:878-938) and the `model.weights.h5` member of a `.keras` zip
(model.save, audiomodel.py:515-518) through h5py with the HDF5 library's
default ("earliest") format: a version-0 superblock, version-1 object
headers, groups as symbol tables (a version-1 B-tree of symbol-table nodes
plus a local heap of names) and datasets with contiguous (or, when tiny,
compact) storage, no filters.  This module reads exactly that subset -- plus
the compact link messages of newer writers -- into a {path: numpy array} dict,
and writes the same subset (used to export weights and for round-trip tests).
Anything else (version-2 object headers, dense link storage in fractal heaps,
chunked / filtered datasets) raises NotImplementedError naming the feature.

Format reference: the published "HDF5 File Format Specification Version 3.0"
(sections II.A superblock, III.A-C B-tree / symbol table / local heap, IV.A
object headers and the dataspace / datatype / layout / link / continuation
messages).
"""
from __future__ import annotations

import struct

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class H5Error(ValueError):
    pass


# ---------------------------------------------------------------- reader
class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        if data[:8] != SIG:
            raise H5Error("not an HDF5 file (signature)")
        ver = data[8]
        if ver not in (0, 1):
            raise NotImplementedError(f"HDF5 superblock version {ver} (only 0/1: the 'earliest' format)")
        self.so, self.sl = data[13], data[14]
        if self.so != 8 or self.sl != 8:
            raise NotImplementedError("HDF5 offsets/lengths other than 8 bytes")
        p = 24 if ver == 0 else 28  # v1 adds indexed-storage K (2) + reserved (2)
        self.base = self._u(p, 8)
        root = p + 32  # base, free-space, EOF, driver addresses
        self.root_oh = self._u(root + 8, 8)

    def _u(self, off, n):
        return int.from_bytes(self.d[off:off + n], "little")

    # -- object headers
    def messages(self, addr):
        d = self.d
        if d[addr:addr + 4] == b"OHDR":
            raise NotImplementedError("HDF5 version-2 object headers")
        if d[addr] != 1:
            raise H5Error(f"object header version {d[addr]} at {addr}")
        nmsg = self._u(addr + 2, 2)
        size = self._u(addr + 8, 4)
        blocks = [(addr + 16, size)]
        out = []
        while blocks and len(out) < nmsg:
            p, n = blocks.pop(0)
            end = p + n
            while p + 8 <= end and len(out) < nmsg:
                mtype, msize = self._u(p, 2), self._u(p + 2, 2)
                body = d[p + 8:p + 8 + msize]
                if mtype == 0x10:  # continuation
                    blocks.append((int.from_bytes(body[:8], "little"), int.from_bytes(body[8:16], "little")))
                out.append((mtype, body))
                p += 8 + msize
        return out

    # -- groups
    def heap_name(self, heap_addr, off):
        d = self.d
        if d[heap_addr:heap_addr + 4] != b"HEAP":
            raise H5Error("local heap signature")
        seg = self._u(heap_addr + 24, 8)
        p = seg + off
        e = d.index(b"\0", p)
        return d[p:e].decode()

    def btree_entries(self, btree, heap):
        d = self.d
        if d[btree:btree + 4] != b"TREE":
            raise H5Error("B-tree signature")
        ntype, level, used = d[btree + 4], d[btree + 5], self._u(btree + 6, 2)
        if ntype != 0:
            raise H5Error("expected a group B-tree node")
        p = btree + 24 + 8  # past the header and key 0
        out = []
        for _ in range(used):
            child = self._u(p, 8)
            p += 16  # child address + next key
            if level > 0:
                out += self.btree_entries(child, heap)
            else:
                out += self.snod_entries(child, heap)
        return out

    def snod_entries(self, addr, heap):
        d = self.d
        if d[addr:addr + 4] != b"SNOD":
            raise H5Error("symbol table node signature")
        n = self._u(addr + 6, 2)
        out = []
        for i in range(n):
            e = addr + 8 + 40 * i
            out.append((self.heap_name(heap, self._u(e, 8)), self._u(e + 8, 8)))
        return out

    def children(self, msgs):
        """(name, object header address) of a group's members, or None."""
        for mtype, body in msgs:
            if mtype == 0x11:  # symbol table
                return self.btree_entries(int.from_bytes(body[:8], "little"), int.from_bytes(body[8:16], "little"))
        links = [b for t, b in msgs if t == 0x06]
        if links:
            return [self.link(b) for b in links]
        if any(t == 0x02 for t, _ in msgs):
            raise NotImplementedError("HDF5 dense link storage (fractal heap)")
        return None

    def link(self, b):
        """Link message (0x0006), hard links only."""
        if b[0] != 1:
            raise H5Error("link message version")
        flags = b[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = b[p]
            p += 1
        if flags & 0x04:
            p += 8  # creation order
        if flags & 0x10:
            p += 1  # charset
        ln_size = 1 << (flags & 3)
        nlen = int.from_bytes(b[p:p + ln_size], "little")
        p += ln_size
        name = b[p:p + nlen].decode()
        p += nlen
        if ltype != 0:
            raise NotImplementedError("HDF5 soft / external links")
        return name, int.from_bytes(b[p:p + 8], "little")

    # -- datasets
    def dataset(self, msgs):
        shape = dtype = None
        layout = None
        for mtype, b in msgs:
            if mtype == 0x01:  # dataspace
                ver, nd, flags = b[0], b[1], b[2]
                p = 8 if ver == 1 else 4
                shape = tuple(int.from_bytes(b[p + 8 * i:p + 8 * i + 8], "little") for i in range(nd))
            elif mtype == 0x03:  # datatype
                cls, bits, size = b[0] & 0x0F, b[1] | (b[2] << 8) | (b[3] << 16), int.from_bytes(b[4:8], "little")
                order = ">" if bits & 1 else "<"
                if cls == 1:
                    dtype = np.dtype(f"{order}f{size}")
                elif cls == 0:
                    dtype = np.dtype(f"{order}{'i' if bits & 0x08 else 'u'}{size}")
                else:
                    raise NotImplementedError(f"HDF5 datatype class {cls}")
            elif mtype == 0x08:
                layout = b
            elif mtype == 0x0B:
                raise NotImplementedError("HDF5 filtered (compressed) datasets")
        if shape is None or dtype is None or layout is None:
            return None
        ver = layout[0]
        if ver != 3:
            raise NotImplementedError(f"HDF5 layout message version {ver}")
        cls = layout[1]
        n = int(np.prod(shape)) if shape else 1
        if cls == 1:  # contiguous
            addr = int.from_bytes(layout[2:10], "little")
            raw = self.d[addr:addr + n * dtype.itemsize] if addr != UNDEF else b"\0" * (n * dtype.itemsize)
        elif cls == 0:  # compact
            size = int.from_bytes(layout[2:4], "little")
            raw = layout[4:4 + size]
        else:
            raise NotImplementedError("HDF5 chunked datasets")
        return np.frombuffer(bytes(raw), dtype=dtype, count=n).reshape(shape).astype(dtype.newbyteorder("="))

    def walk(self, addr, path, out):
        msgs = self.messages(addr)
        kids = self.children(msgs)
        if kids is not None:
            for name, child in sorted(kids):
                self.walk(child, f"{path}/{name}" if path else name, out)
            return
        arr = self.dataset(msgs)
        if arr is not None:
            out[path] = arr


def read_h5(data: bytes | str) -> dict[str, np.ndarray]:
    """All datasets of an HDF5 file as {'group/.../name': array}."""
    if not isinstance(data, (bytes, bytearray)):
        with open(data, "rb") as f:
            data = f.read()
    r = _Reader(bytes(data))
    out: dict[str, np.ndarray] = {}
    r.walk(r.root_oh, "", out)
    return out


# ---------------------------------------------------------------- writer
class _Writer:
    LEAF_K, NODE_K = 4, 16

    def __init__(self):
        self.buf = bytearray(96)  # superblock, filled at the end

    def alloc(self, data: bytes, align=8) -> int:
        while len(self.buf) % align:
            self.buf.append(0)
        a = len(self.buf)
        self.buf += data
        return a

    @staticmethod
    def _msg(mtype, body):
        body = bytes(body)
        body += b"\0" * (-len(body) % 8)
        return struct.pack("<HHB3x", mtype, len(body), 0) + body

    def object_header(self, msgs) -> int:
        body = b"".join(self._msg(t, b) for t, b in msgs)
        return self.alloc(struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4 + body)

    def dataset(self, arr: np.ndarray) -> int:
        arr = np.ascontiguousarray(arr)
        if arr.dtype == np.float32:
            dt = struct.pack("<BBBBI", 0x11, 0x20, 31, 0, 4) + struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        elif arr.dtype == np.float64:
            dt = struct.pack("<BBBBI", 0x11, 0x20, 63, 0, 8) + struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        elif arr.dtype in (np.int64, np.int32):
            dt = struct.pack("<BBBBI", 0x10, 0x08, 0, 0, arr.dtype.itemsize) + struct.pack("<HH", 0,
                                                                                            8 * arr.dtype.itemsize)
        else:
            raise NotImplementedError(f"dtype {arr.dtype}")
        arr = arr.astype(arr.dtype.newbyteorder("<"), copy=False)
        data_addr = self.alloc(arr.tobytes(), align=8)
        space = struct.pack("<BBBB4x", 1, arr.ndim, 0, 0) + b"".join(struct.pack("<Q", s) for s in arr.shape)
        fill = struct.pack("<BBBB", 2, 2, 2, 0)  # fill value v2: late allocation, write if set, undefined
        layout = struct.pack("<BBQQ", 3, 1, data_addr, arr.nbytes)
        return self.object_header([(0x01, space), (0x03, dt), (0x05, fill), (0x08, layout)])

    def finish(self, root) -> bytes:
        oh, btree, heap = root
        sb = SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", self.LEAF_K, self.NODE_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, len(self.buf), UNDEF)
        sb += struct.pack("<QQII", 0, oh, 1, 0) + struct.pack("<QQ", btree, heap)
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def write_h5(tree: dict) -> bytes:
    """Serialise {name: array | {name: ...}} as an HDF5 file (the subset read_h5
    reads: superblock v0, v1 object headers, symbol-table groups of at most
    256 members, contiguous little-endian datasets)."""
    w = _Writer()

    def build(members):
        return _write_group(w, {k: (_Sub(build(v)) if isinstance(v, dict) else v) for k, v in members.items()})

    return w.finish(build(tree))


class _Sub:
    def __init__(self, res):
        self.res = res


def _write_group(w: _Writer, members):
    names = sorted(members)
    cap = 2 * w.LEAF_K
    if len(names) > cap * 2 * w.NODE_K:
        raise NotImplementedError("groups of more than 256 members")
    addrs = {}
    for n in names:
        v = members[n]
        addrs[n] = v.res[0] if isinstance(v, _Sub) else w.dataset(np.asarray(v))
    heap = bytearray(b"\0" * 8)
    off = {}
    for n in names:
        off[n] = len(heap)
        heap += n.encode() + b"\0"
        heap += b"\0" * (-len(heap) % 8)
    seg = w.alloc(bytes(heap))
    heap_addr = w.alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap), UNDEF, seg))
    snods, keys = [], [0]
    for i in range(0, len(names), cap):
        chunk = names[i:i + cap]
        ent = b"".join(struct.pack("<QQII16x", off[n], addrs[n], 0, 0) for n in chunk)
        ent += b"\0" * (40 * (cap - len(chunk)))
        snods.append(w.alloc(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(chunk)) + ent))
        keys.append(off[chunk[-1]])
    tree = b"TREE" + bytes([0, 0]) + struct.pack("<HQQ", len(snods), UNDEF, UNDEF) + struct.pack("<Q", keys[0])
    for c, k in zip(snods, keys[1:]):
        tree += struct.pack("<QQ", c, k)
    tree += b"\0" * (16 * (2 * w.NODE_K - len(snods)))
    btree = w.alloc(tree)
    oh = w.object_header([(0x11, struct.pack("<QQ", btree, heap_addr))])
    return oh, btree, heap_addr
