"""Minimal self-contained HDF5 writer/reader for the ``.diff.h5`` output layout.

h5py is not installed beside torch here (nor, likely, on the GPU box), yet downstream
consumers (``predict.py:173-194``) open the files with h5py.  This module writes what
``h5py.File(path,'w').create_dataset(name, data=arr)`` writes for contiguous fp32/fp64
arrays (``chromatin.py:282-286``): superblock v0, a v1 root object header with a
symbol-table message, a v1 group B-tree, a local heap, one symbol-table node, and per
dataset a v1 object header (dataspace with max dims, IEEE float datatype, fill value
v2, layout v3 contiguous) -- byte layout modelled on the reference's own
``example/*.diff.h5`` (see tests/golden/example.vcf.shift_0.diff.h5) -- followed by the
raw little-endian data.  ``read`` parses the same subset (contiguous datasets in the
root group), which also covers files written by h5py with default settings.
"""
from __future__ import annotations

import struct

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
_SIG = b"\x89HDF\r\n\x1a\n"
_LEAF_K = 4
_INTERNAL_K = 16
_DATA_ALIGN = 2048


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * ((-len(b)) % 8)


def _msg(mtype: int, data: bytes, flags: int = 0) -> bytes:
    data = _pad8(data)
    return struct.pack("<HHB3x", mtype, len(data), flags) + data


def _datatype(dt: np.dtype) -> bytes:
    if dt == np.float32:
        return struct.pack("<BBBBI", 0x11, 0x20, 31, 0, 4) + struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
    if dt == np.float64:
        return struct.pack("<BBBBI", 0x11, 0x20, 63, 0, 8) + struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
    if dt.kind == "S":   # fixed-length ASCII, null-padded (what h5py writes for numpy 'S' arrays)
        return struct.pack("<BBBBI", 0x13, 0x01, 0, 0, dt.itemsize)
    raise TypeError(f"unsupported dtype {dt} (float32/float64/fixed-length bytes only)")


def _dataset_header(shape, dt, data_addr, nbytes) -> bytes:
    rank = len(shape)
    space = struct.pack("<BBBB4x", 1, rank, 1, 0) + b"".join(struct.pack("<Q", d) for d in shape) * 2
    msgs = [
        _msg(0x0001, space),
        _msg(0x0003, _datatype(dt), flags=1),
        _msg(0x0005, struct.pack("<BBBBI", 2, 2, 2, 1, 0), flags=1),
        _msg(0x0008, struct.pack("<BBQQ", 3, 1, data_addr, nbytes)),
    ]
    body = b"".join(msgs)
    return struct.pack("<BBHII4x", 1, 0, len(msgs), 1, len(body)) + body


def _layout(names, shapes, dtypes):
    """(header bytes, data addresses, eof) of root datasets `names` (sorted) with the given shapes
    and dtypes: everything ahead of the first data byte, and where each dataset's data goes."""
    if len(names) > 2 * _LEAF_K:
        raise ValueError("at most 8 datasets per file in this minimal writer")
    nbytes = [int(np.prod(sh, dtype=np.int64)) * dt.itemsize for sh, dt in zip(shapes, dtypes)]
    # heap data segment: "" at 0 then each name, 8-byte padded
    heap = b"\0" * 8
    name_off = []
    for n in names:
        name_off.append(len(heap))
        heap += _pad8(n.encode() + b"\0")

    sb_size = 96
    root_oh = sb_size                              # 16-B prefix + symbol-table message
    root_oh_size = 16 + 24
    btree = root_oh + root_oh_size
    btree_size = 24 + (2 * _INTERNAL_K + 1) * 8 + 2 * _INTERNAL_K * 8
    lheap = btree + btree_size
    lheap_data = lheap + 32
    snod = lheap_data + len(heap)
    snod_size = 8 + 2 * _LEAF_K * 40
    ds_oh = []
    pos = snod + snod_size
    for sh, dt in zip(shapes, dtypes):
        ds_oh.append(pos)
        pos += len(_dataset_header(sh, dt, 0, 0))
    data_addr = []
    pos = (pos + _DATA_ALIGN - 1) // _DATA_ALIGN * _DATA_ALIGN
    for nb in nbytes:
        data_addr.append(pos)
        pos += nb
    eof = pos

    header_len = data_addr[0] if names else eof
    out = bytearray(header_len)
    sb = _SIG + struct.pack("<BBBBBBBB", 0, 0, 0, 0, 0, 8, 8, 0) + struct.pack("<HHI", _LEAF_K, _INTERNAL_K, 0)
    sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
    sb += struct.pack("<QQI4xQQ", 0, root_oh, 1, btree, lheap)
    out[0:sb_size] = sb
    root = struct.pack("<BBHII4x", 1, 0, 1, 1, 24) + _msg(0x0011, struct.pack("<QQ", btree, lheap))
    out[root_oh:root_oh + len(root)] = root
    last_key = name_off[-1] if names else 0
    bt = b"TREE" + struct.pack("<BBHQQ", 0, 0, 1 if names else 0, UNDEF, UNDEF)
    bt += struct.pack("<QQQ", 0, snod, last_key)
    out[btree:btree + len(bt)] = bt
    lh = b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, lheap_data)
    out[lheap:lheap + 32] = lh
    out[lheap_data:lheap_data + len(heap)] = heap
    sn = b"SNOD" + struct.pack("<BBH", 1, 0, len(names))
    for i in range(len(names)):
        sn += struct.pack("<QQI4x16x", name_off[i], ds_oh[i], 0)
    out[snod:snod + len(sn)] = sn
    for i in range(len(names)):
        hdr = _dataset_header(shapes[i], dtypes[i], data_addr[i], nbytes[i])
        out[ds_oh[i]:ds_oh[i] + len(hdr)] = hdr
    return bytes(out), data_addr, eof


def _check_dtype(dt):
    if dt not in (np.float32, np.float64) and dt.kind != "S":
        raise TypeError(f"{dt}: only float32/float64/'S' datasets are supported")


def write(path: str, datasets: dict) -> None:
    """Write ``{name: ndarray}`` (float32/float64, C-contiguous) as root datasets."""
    names = sorted(datasets)                      # symbol-table entries are name-ordered
    arrays = [np.array(datasets[n], order="C", copy=True) for n in names]   # 0-d arrays -> scalar dataspace
    for a in arrays:
        _check_dtype(a.dtype)
    head, data_addr, _ = _layout(names, [a.shape for a in arrays], [a.dtype for a in arrays])
    with open(path, "wb") as f:
        f.write(head)
        for i, a in enumerate(arrays):
            cur = f.tell()
            if cur < data_addr[i]:
                f.write(b"\0" * (data_addr[i] - cur))
            f.write(a.tobytes() if a.dtype.kind == "S" else a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())


class RowWriter:
    """A file of fixed-shape root datasets filled row block by row block (streamed outputs).

    ``RowWriter(path, {name: (shape, dtype)})`` writes the header and sizes the file (unwritten
    data reads as zeros); ``write_rows(name, row0, block)`` stores ``block`` (C-contiguous, same
    dtype, trailing dims of the dataset) at rows ``row0..`` in place.  Once every row is written
    the file is byte-identical to ``write`` of the full arrays."""

    def __init__(self, path: str, specs: dict, create: bool = True):
        """create=False attaches to a file another process created with the same specs (its
        header is checked, nothing is truncated): several ranks then write disjoint rows of one
        file, each with its own descriptor (pwrite at row offsets; no locking needed)."""
        import os
        self.names = sorted(specs)
        self.shapes = {n: tuple(int(x) for x in specs[n][0]) for n in self.names}
        self.dtypes = {n: np.dtype(specs[n][1]) for n in self.names}
        for n in self.names:
            _check_dtype(self.dtypes[n])
        head, addr, eof = _layout(self.names, [self.shapes[n] for n in self.names],
                                  [self.dtypes[n] for n in self.names])
        self.addr = dict(zip(self.names, addr))
        self.fd = None
        if create:
            self.fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
            os.pwrite(self.fd, head, 0)
            os.ftruncate(self.fd, eof)
        else:
            fd = os.open(path, os.O_RDWR)
            try:
                if os.fstat(fd).st_size != eof or os.pread(fd, len(head), 0) != head:
                    raise ValueError(f"{path}: not a row file of these datasets (header or size differ)")
            except BaseException:
                os.close(fd)
                raise
            self.fd = fd

    def write_rows(self, name: str, row0: int, block: np.ndarray) -> None:
        import os
        shape, dt = self.shapes[name], self.dtypes[name]
        block = np.ascontiguousarray(block, dtype=dt.newbyteorder("<"))
        if block.shape[1:] != shape[1:] or row0 < 0 or row0 + block.shape[0] > shape[0]:
            raise ValueError(f"{name}: rows {row0}..{row0 + block.shape[0]} of {shape} do not fit {block.shape}")
        row_bytes = int(np.prod(shape[1:], dtype=np.int64)) * dt.itemsize
        mv = memoryview(block).cast("B")
        off, done = self.addr[name] + row0 * row_bytes, 0
        while done < len(mv):
            done += os.pwrite(self.fd, mv[done:], off + done)

    def sync(self) -> None:
        """fsync: the header and size reach the file system before other processes attach."""
        import os
        os.fsync(self.fd)

    def close(self) -> None:
        import os
        if self.fd is not None:
            os.close(self.fd)
            self.fd = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---------------------------------------------------------------------------- reader
def _read_messages(buf: bytes, addr: int):
    ver, _, nmsg, _, size = struct.unpack_from("<BBHII", buf, addr)
    if ver != 1:
        raise ValueError(f"object header version {ver} not supported")
    p = addr + 16
    end = p + size
    msgs = []
    while p < end and len(msgs) < nmsg:
        mtype, msize, _ = struct.unpack_from("<HHB", buf, p)
        msgs.append((mtype, buf[p + 8:p + 8 + msize]))
        p += 8 + msize
    return msgs


def _parse_dataset(buf: bytes, addr: int):
    shape = dtype = data = None
    for mtype, m in _read_messages(buf, addr):
        if mtype == 0x0001:
            ver, rank = m[0], m[1]
            off = 8 if ver == 1 else 4
            shape = tuple(struct.unpack_from("<%dQ" % rank, m, off))
        elif mtype == 0x0003:
            cls = m[0] & 0x0F
            size = struct.unpack_from("<I", m, 4)[0]
            if cls == 3:
                dtype = np.dtype(f"S{size}")
            elif cls != 1 or size not in (4, 8):
                raise ValueError("only IEEE float and fixed-length string datasets are supported")
            else:
                be = m[1] & 1
                dtype = np.dtype(("<" if not be else ">") + ("f4" if size == 4 else "f8"))
        elif mtype == 0x0008:
            if m[0] != 3 or m[1] != 1:
                raise ValueError("only contiguous layout (v3) is supported")
            data = struct.unpack_from("<QQ", m, 2)
    if shape is None or dtype is None or data is None:
        raise ValueError("incomplete dataset header")
    addr_, nbytes = data
    if addr_ == UNDEF:
        return np.zeros(shape, dtype)
    arr = np.frombuffer(buf, dtype, count=int(np.prod(shape)), offset=addr_).reshape(shape)
    return arr.copy() if dtype.kind == "S" else arr.astype(dtype.newbyteorder("="))


def read(path: str) -> dict:
    """``{name: ndarray}`` for every contiguous float / fixed-length string dataset in the root group."""
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:8] != _SIG:
        raise ValueError("not an HDF5 file (superblock v0 expected at offset 0)")
    if buf[8] != 0:
        raise ValueError("superblock version %d not supported" % buf[8])
    root_oh = struct.unpack_from("<Q", buf, 64)[0]
    btree = lheap = None
    for mtype, m in _read_messages(buf, root_oh):
        if mtype == 0x0011:
            btree, lheap = struct.unpack_from("<QQ", m, 0)
    if btree is None:
        raise ValueError("root group has no symbol table")
    heap_data = struct.unpack_from("<Q", buf, lheap + 24)[0]
    out = {}

    def walk(node):
        sig, ntype, level, used = struct.unpack_from("<4sBBH", buf, node)
        assert sig == b"TREE" and ntype == 0
        children = [struct.unpack_from("<Q", buf, node + 24 + 8 + 16 * i)[0] for i in range(used)]
        for c in children:
            if level > 0:
                walk(c)
            else:
                s, _, _, nsym = struct.unpack_from("<4sBBH", buf, c)
                assert s == b"SNOD"
                for j in range(nsym):
                    noff, oh = struct.unpack_from("<QQ", buf, c + 8 + 40 * j)
                    end = buf.index(b"\0", heap_data + noff)
                    out[buf[heap_data + noff:end].decode()] = _parse_dataset(buf, oh)

    walk(btree)
    return out
