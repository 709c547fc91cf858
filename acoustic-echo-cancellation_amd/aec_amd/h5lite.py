"""Minimal HDF5 reader / writer for the reference's utterance container.

The reference stores each test set as an HDF5 file (`test.ex`):
- root groups are named "0" .. "n-1";
- each group holds four 1-D float32 datasets: nearend_speech, nearend_mic,
  farend_speech and echo, each with its own length;
- h5py writes them with its defaults (`chunks=True`, no compression);
- files come from Stage2_lhm/generate_h5files/test_wav2h5.py:44-48 and are
  read by scripts/test.py:19-36.

h5py (and libhdf5) are not available in this image, so this module restates
the published HDF5 File Format Specification for exactly the structures
those files use:
- superblock version 0 or 1;
- version-1 object headers, with continuation blocks;
- "old-style" groups: a symbol-table message pointing to a version-1 B-tree
  of symbol-table nodes plus a local heap of names;
- datasets with a dataspace (v1/v2), an IEEE float or integer datatype, and
  a layout message v1-v3. The layout may be compact, contiguous, or chunked
  with a version-1 B-tree index. The chunk filters deflate (gzip) and
  shuffle are supported.

Files written by libhdf5 with `libver='latest'` are rejected with a clear
error: version-2/3 superblocks, v2 object headers, dense link storage and
v4 chunk indexes. The writer emits the same structures, with chunked
datasets by default as h5py's `chunks=True` does.

libhdf5 itself is not in this image. The reader is checked against files
libhdf5 wrote (tests/golden/foreign/, tests/test_h5lite.py): a MATLAB 7.3
file with a 512-byte user block, checked value for value against scipy's
reader of the same variable in MATLAB v5 format, and the HDF5 example files
PyTables ships (chunked, big-endian, float16/32/64).  Files from its own
writer cover multi-level group B-trees (over 256 utterances) and
multi-chunk datasets.
"""
from __future__ import annotations

import mmap
import os
import struct
import zlib
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np

SIGNATURE = b'\x89HDF\r\n\x1a\n'
UNDEF = 0xFFFFFFFFFFFFFFFF

# message types (spec §IV.A.2)
MSG_NIL, MSG_DATASPACE, MSG_LINFO, MSG_DATATYPE, MSG_FILL_OLD, MSG_FILL = 0x0, 0x1, 0x2, 0x3, 0x4, 0x5
MSG_LINK, MSG_LAYOUT, MSG_GINFO, MSG_FILTER, MSG_CONT, MSG_STAB = 0x6, 0x8, 0xA, 0xB, 0x10, 0x11

SIGNALS = ('nearend_speech', 'nearend_mic', 'farend_speech', 'echo')


class H5Error(ValueError):
    pass


def _pad8(n: int) -> int:
    return (n + 7) & ~7


# ============================================================================
# reader
# ============================================================================
class Dataset:
    """A dataset handle: shape, dtype and lazy read (`np.array(ds)` / `ds[()]`)."""

    def __init__(self, f: 'File', name: str, shape, dtype, layout, filters):
        self._f = f
        self.name = name
        self.shape = tuple(shape)
        self.dtype = dtype
        self._layout = layout
        self._filters = filters

    def __len__(self):
        return self.shape[0] if self.shape else 1

    def __array__(self, dtype=None, copy=None):
        a = self.read()
        return a.astype(dtype) if dtype is not None else a

    def __getitem__(self, key):
        return self.read()[key]

    def read(self) -> np.ndarray:
        n = int(np.prod(self.shape)) if self.shape else 1
        es = self.dtype.itemsize
        kind = self._layout[0]
        if kind == 'compact':
            raw = self._layout[1]
        elif kind == 'contiguous':
            addr, size = self._layout[1], self._layout[2]
            if addr == UNDEF:
                raw = b'\0' * (n * es)
            else:
                raw = self._f._buf[addr:addr + n * es]
        else:
            raw = self._read_chunked(n, es)
        out = np.frombuffer(raw, dtype=self.dtype, count=n).reshape(self.shape)
        return out.astype(self.dtype.newbyteorder('='), copy=True)

    def _read_chunked(self, n: int, es: int) -> bytes:
        _, btree, cdims = self._layout
        rank = len(self.shape)
        cshape = cdims[:rank]
        out = np.zeros(self.shape if rank else (1,), dtype=np.uint8 if es == 1 else np.dtype(f'V{es}'))
        if btree == UNDEF:                                 # no chunk written yet: all fill value (0)
            return out.tobytes()
        for offs, size, mask, addr in self._f._chunk_records(btree, rank):
            raw = self._f._buf[addr:addr + size]
            raw = _unfilter(raw, self._filters, mask, es)
            chunk = np.frombuffer(raw, dtype=out.dtype, count=int(np.prod(cshape))).reshape(cshape)
            sl_out, sl_in = [], []
            for d in range(rank):
                lo = offs[d]
                hi = min(lo + cshape[d], self.shape[d])
                if hi <= lo:
                    break
                sl_out.append(slice(lo, hi))
                sl_in.append(slice(0, hi - lo))
            else:
                out[tuple(sl_out)] = chunk[tuple(sl_in)]
        return out.tobytes()


class Group:
    def __init__(self, f: 'File', name: str, links: Dict[str, int]):
        self._f = f
        self.name = name
        self._links = links

    def keys(self):
        return list(self._links.keys())

    def __len__(self):
        return len(self._links)

    def __contains__(self, k):
        return k in self._links

    def __iter__(self):
        return iter(self._links)

    def __getitem__(self, path: str):
        parts = [p for p in path.split('/') if p]
        node = self
        for p in parts:
            if not isinstance(node, Group):
                raise KeyError(path)
            if p not in node._links:
                raise KeyError(f'{p!r} not in group {node.name!r}')
            node = node._f._object(node._links[p], node.name.rstrip('/') + '/' + p)
        return node


class File(Group):
    """Read-only HDF5 file (h5py-like surface: `len(f)`, `f['0']['nearend_mic']`)."""

    def __init__(self, path: str, mode: str = 'r'):
        if mode != 'r':
            raise ValueError("h5lite.File is read-only; use h5lite.write_utterances to write")
        self._fh = open(path, 'rb')
        size = os.fstat(self._fh.fileno()).st_size
        if size == 0:
            raise H5Error(f'{path}: empty file')
        self._map = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        self._buf = memoryview(self._map)
        base = self._find_superblock()
        # Every address in the file is relative to the base address, the
        # superblock's own position (spec §II.A "Base Address"): a file with a
        # user block (superblock at 512, 1024, ...) is read through a view that
        # starts at the superblock
        self._buf = self._buf[base:]
        self._parse_superblock(0)
        root_links = self._group_links(self._root_addr)
        super().__init__(self, '/', root_links)

    # -- context manager / close
    def close(self):
        if getattr(self, '_buf', None) is not None:
            self._buf.release()
            self._buf = None
        if getattr(self, '_map', None) is not None:
            self._map.close()
            self._map = None
            self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- low level
    def _u(self, off: int, n: int) -> int:
        return int.from_bytes(self._buf[off:off + n], 'little')

    def _find_superblock(self) -> int:
        off = 0
        while off + 8 <= len(self._buf):
            if bytes(self._buf[off:off + 8]) == SIGNATURE:
                return off
            off = 512 if off == 0 else off * 2
        raise H5Error('not an HDF5 file (no superblock signature)')

    def _parse_superblock(self, base: int):
        ver = self._buf[base + 8]
        if ver > 1:
            raise H5Error(f'superblock version {ver} (libver="latest" files) is not supported; '
                          'write the file with h5py defaults (libver="earliest")')
        self._so = self._buf[base + 13]
        self._sl = self._buf[base + 14]
        if self._so != 8 or self._sl != 8:
            raise H5Error('only 8-byte offsets / lengths are supported')
        p = base + 24 + (4 if ver == 1 else 0)            # versions, sizes, K values, flags (+ v1 K)
        # the stored base address is 0 (or the superblock's absolute offset, which
        # the view already applies): either way addresses count from the superblock
        p += 8 * 4                                        # base, free-space, EOF, driver
        # root group symbol table entry: name offset, object header address, cache type, scratch
        self._root_addr = self._u(p + 8, 8)

    def _messages(self, addr: int) -> List[Tuple[int, int, int]]:
        """(type, data offset, size) of every message of a v1 object header,
        following continuation messages."""
        if self._buf[addr:addr + 4] == b'OHDR':
            raise H5Error('version-2 object headers (libver="latest") are not supported')
        if self._buf[addr] != 1:
            raise H5Error(f'bad object header version {self._buf[addr]} at {addr:#x}')
        nmsg = self._u(addr + 2, 2)
        hsize = self._u(addr + 8, 4)
        blocks = [(addr + 16, hsize)]
        out = []
        while blocks and len(out) < nmsg:
            start, size = blocks.pop(0)
            p = start
            while p + 8 <= start + size and len(out) < nmsg:
                mtype = self._u(p, 2)
                msize = self._u(p + 2, 2)
                data = p + 8
                if mtype == MSG_CONT:
                    blocks.append((self._u(data, 8), self._u(data + 8, 8)))
                out.append((mtype, data, msize))
                p = data + msize
        return out

    def _group_links(self, addr: int) -> Dict[str, int]:
        msgs = self._messages(addr)
        stab = [m for m in msgs if m[0] == MSG_STAB]
        if not stab:
            if any(m[0] in (MSG_LINK, MSG_LINFO) for m in msgs):
                raise H5Error('new-style (link message) groups are not supported')
            raise H5Error(f'object at {addr:#x} is not a group')
        d = stab[0][1]
        btree, heap = self._u(d, 8), self._u(d + 8, 8)
        heap_data = self._local_heap(heap)
        links: Dict[str, int] = {}
        for name_off, obj in self._group_entries(btree):
            end = heap_data.index(b'\0', name_off)
            links[heap_data[name_off:end].decode('utf-8')] = obj
        return links

    def _local_heap(self, addr: int) -> bytes:
        if self._buf[addr:addr + 4] != b'HEAP':
            raise H5Error(f'bad local heap signature at {addr:#x}')
        size = self._u(addr + 8, 8)
        data = self._u(addr + 24, 8)
        return bytes(self._buf[data:data + size])

    def _btree_node(self, addr: int):
        if self._buf[addr:addr + 4] != b'TREE':
            raise H5Error(f'bad v1 B-tree signature at {addr:#x}')
        return self._buf[addr + 4], self._buf[addr + 5], self._u(addr + 6, 2)

    def _group_entries(self, addr: int) -> Iterable[Tuple[int, int]]:
        ntype, level, used = self._btree_node(addr)
        if ntype != 0:
            raise H5Error('group B-tree has the wrong node type')
        p = addr + 24 + 8                                  # header, key 0
        for _ in range(used):
            child = self._u(p, 8)
            p += 16                                        # child, next key
            if level > 0:
                yield from self._group_entries(child)
            else:
                if self._buf[child:child + 4] != b'SNOD':
                    raise H5Error(f'bad symbol table node at {child:#x}')
                nsym = self._u(child + 6, 2)
                e = child + 8
                for _ in range(nsym):
                    yield self._u(e, 8), self._u(e + 8, 8)
                    e += 40

    def _chunk_records(self, addr: int, rank: int):
        """(offsets, size, filter mask, address) of every chunk of a v1 chunk B-tree."""
        ntype, level, used = self._btree_node(addr)
        if ntype != 1:
            raise H5Error('chunk B-tree has the wrong node type')
        ksz = 8 + 8 * (rank + 1)
        p = addr + 24
        for _ in range(used):
            size = self._u(p, 4)
            mask = self._u(p + 4, 4)
            offs = [self._u(p + 8 + 8 * d, 8) for d in range(rank)]
            child = self._u(p + ksz, 8)
            p += ksz + 8
            if level > 0:
                yield from self._chunk_records(child, rank)
            else:
                yield offs, size, mask, child

    def _object(self, addr: int, name: str):
        msgs = self._messages(addr)
        if any(m[0] == MSG_STAB for m in msgs):
            return Group(self, name, self._group_links(addr))
        shape = dtype = layout = None
        filters: List[Tuple[int, List[int]]] = []
        for mtype, d, size in msgs:
            if mtype == MSG_DATASPACE:
                shape = self._dataspace(d)
            elif mtype == MSG_DATATYPE:
                dtype = self._datatype(d)
            elif mtype == MSG_LAYOUT:
                layout = self._layout(d)
            elif mtype == MSG_FILTER:
                filters = self._filters(d)
        if shape is None or dtype is None or layout is None:
            raise H5Error(f'object {name!r} is neither a group nor a readable dataset')
        return Dataset(self, name, shape, dtype, layout, filters)

    def _dataspace(self, d: int):
        ver, rank, flags = self._buf[d], self._buf[d + 1], self._buf[d + 2]
        if ver == 1:
            p = d + 8
        elif ver == 2:
            if self._buf[d + 3] == 2:                      # null dataspace
                return (0,)
            p = d + 4
        else:
            raise H5Error(f'dataspace version {ver} unsupported')
        return tuple(self._u(p + 8 * i, 8) for i in range(rank))

    def _datatype(self, d: int) -> np.dtype:
        cv = self._buf[d]
        cls, ver = cv & 0x0F, cv >> 4
        bits0 = self._buf[d + 1]
        size = self._u(d + 4, 4)
        order = '>' if bits0 & 1 else '<'
        if cls == 1:                                       # floating point
            if size not in (2, 4, 8):
                raise H5Error(f'float size {size} unsupported')
            return np.dtype(f'{order}f{size}')
        if cls == 0:                                       # fixed point
            signed = bool(bits0 & 0x08)
            return np.dtype(f'{order}{"i" if signed else "u"}{size}')
        raise H5Error(f'datatype class {cls} unsupported')

    def _layout(self, d: int):
        ver = self._buf[d]
        if ver == 3:
            cls = self._buf[d + 1]
            if cls == 0:
                n = self._u(d + 2, 2)
                return ('compact', bytes(self._buf[d + 4:d + 4 + n]))
            if cls == 1:
                return ('contiguous', self._u(d + 2, 8), self._u(d + 10, 8))
            if cls == 2:
                nd = self._buf[d + 2]
                bt = self._u(d + 3, 8)
                dims = [self._u(d + 11 + 4 * i, 4) for i in range(nd)]
                return ('chunked', bt, dims)
            raise H5Error(f'layout class {cls} unsupported')
        if ver in (1, 2):
            nd, cls = self._buf[d + 1], self._buf[d + 2]
            p = d + 8
            addr = None
            if cls != 0:
                addr = self._u(p, 8)
                p += 8
            dims = [self._u(p + 4 * i, 4) for i in range(nd)]
            p += 4 * nd
            if cls == 0:
                n = self._u(p, 4)
                return ('compact', bytes(self._buf[p + 4:p + 4 + n]))
            if cls == 1:
                return ('contiguous', addr, int(np.prod(dims)))
            return ('chunked', addr, dims)
        raise H5Error(f'layout message version {ver} (libver="latest") unsupported')

    def _filters(self, d: int) -> List[Tuple[int, List[int]]]:
        ver, nf = self._buf[d], self._buf[d + 1]
        p = d + (8 if ver == 1 else 2)
        out = []
        for _ in range(nf):
            fid = self._u(p, 2)
            if ver == 1 or fid >= 256:
                nlen = self._u(p + 2, 2)
                p += 4
            else:
                nlen = 0
                p += 2
            nvals = self._u(p + 2, 2)
            p += 4
            p += _pad8(nlen) if ver == 1 else nlen
            vals = [self._u(p + 4 * i, 4) for i in range(nvals)]
            p += 4 * nvals
            if ver == 1 and nvals % 2:
                p += 4
            out.append((fid, vals))
        return out


def _unfilter(raw, filters, mask: int, es: int) -> bytes:
    data = bytes(raw)
    for i in range(len(filters) - 1, -1, -1):
        if mask & (1 << i):
            continue
        fid, vals = filters[i]
        if fid == 1:                                       # deflate
            data = zlib.decompress(data)
        elif fid == 2:                                     # shuffle
            a = np.frombuffer(data, np.uint8)
            n = len(a) // es
            body = a[:n * es].reshape(es, n).T.reshape(-1)
            data = body.tobytes() + a[n * es:].tobytes()
        elif fid == 3:                                     # fletcher32: drop the 4-byte checksum
            data = data[:-4]
        else:
            raise H5Error(f'filter {fid} unsupported')
    return data


# ============================================================================
# writer
# ============================================================================
class _Writer:
    """Appends objects to a byte buffer; addresses are file offsets."""

    def __init__(self):
        self.buf = bytearray()

    def alloc(self, n: int) -> int:
        addr = len(self.buf)
        self.buf += b'\0' * _pad8(n)
        return addr

    def put(self, addr: int, data: bytes):
        self.buf[addr:addr + len(data)] = data

    def append(self, data: bytes) -> int:
        addr = self.alloc(len(data))
        self.put(addr, data)
        return addr


def _msg(mtype: int, body: bytes, flags: int = 0) -> bytes:
    body = body + b'\0' * (_pad8(len(body)) - len(body))
    return struct.pack('<HHB3x', mtype, len(body), flags) + body


def _object_header(msgs: List[bytes]) -> bytes:
    body = b''.join(msgs)
    return struct.pack('<BBHII', 1, 0, len(msgs), 1, len(body)) + b'\0' * 4 + body


def _f32_datatype() -> bytes:
    # class 1 (float) version 1; little-endian, implied mantissa msb (bits 4-5 = 2), sign at bit 31
    return struct.pack('<B3BI', 0x11, 0x20, 31, 0, 4) + struct.pack('<HHBBBBI', 0, 32, 23, 8, 0, 23, 127)


def _dataspace(n: int) -> bytes:
    return struct.pack('<BBBB4xQ', 1, 1, 0, 0, n)


def _write_group(w: _Writer, children: List[Tuple[str, int]]) -> int:
    """Old-style group: local heap of names, symbol-table nodes (<= 8 entries,
    sorted by name as libhdf5 requires), v1 B-tree over them. Returns the
    object header address."""
    names = sorted(children, key=lambda c: c[0].encode('utf-8'))
    heap = bytearray(b'\0' * 8)                             # offset 0: empty string
    name_off = {}
    for name, _ in names:
        name_off[name] = len(heap)
        nb = name.encode('utf-8') + b'\0'
        heap += nb + b'\0' * (_pad8(len(nb)) - len(nb))
    heap_data = w.append(bytes(heap))
    heap_hdr = w.append(b'HEAP' + struct.pack('<B3xQQQ', 0, len(heap), UNDEF, heap_data))
    leafK = 4
    snods = []
    for i in range(0, max(1, len(names)), 2 * leafK):
        chunk = names[i:i + 2 * leafK]
        body = b'SNOD' + struct.pack('<BBH', 1, 0, len(chunk))
        for name, obj in chunk:
            body += struct.pack('<QQII16x', name_off[name], obj, 0, 0)
        body += b'\0' * (40 * (2 * leafK - len(chunk)))
        snods.append((chunk[0][0] if chunk else '', w.append(body), chunk[-1][0] if chunk else ''))
    # group B-tree (internal K = 16): keys are heap offsets of names; the key
    # before child i is the last name under child i-1 (key 0: the empty
    # string), the final key the last name under the last child
    groupK = 16
    cur, prev_last = [], None
    for first, addr, last in snods:
        cur.append((name_off[prev_last] if prev_last else 0, addr, last))
        prev_last = last
    level = 0
    while True:
        cap = 2 * groupK
        groups = [cur[i:i + cap] for i in range(0, len(cur), cap)]
        addrs = [w.alloc(24 + 8 + cap * 16) for _ in groups]
        nxt = []
        for gi, g in enumerate(groups):
            left = addrs[gi - 1] if gi > 0 else UNDEF
            right = addrs[gi + 1] if gi + 1 < len(groups) else UNDEF
            body = b'TREE' + struct.pack('<BBHQQ', 0, level, len(g), left, right)
            for key, child, _ in g:
                body += struct.pack('<QQ', key, child)
            body += struct.pack('<Q', name_off.get(g[-1][2], 0) if g[-1][2] else 0)
            w.put(addrs[gi], body)
            nxt.append((g[0][0], addrs[gi], g[-1][2]))
        if len(nxt) == 1:
            root_bt = nxt[0][1]
            break
        cur, level = nxt, level + 1
    return w.append(_object_header([_msg(MSG_STAB, struct.pack('<QQ', root_bt, heap_hdr))])), root_bt, heap_hdr


def _write_dataset(w: _Writer, data: np.ndarray, chunk: Optional[int]) -> int:
    data = np.ascontiguousarray(data, dtype='<f4').reshape(-1)
    n = data.size
    fill = struct.pack('<BBBB', 2, 2 if chunk is None else 3, 2, 0)
    if chunk is None or n == 0:
        addr = w.append(data.tobytes()) if n else UNDEF
        layout = struct.pack('<BBQQ', 3, 1, addr, n * 4)
    else:
        recs = []
        for lo in range(0, n, chunk):
            piece = np.zeros(chunk, '<f4')
            piece[:min(chunk, n - lo)] = data[lo:lo + chunk]
            recs.append((lo, w.append(piece.tobytes())))
        K = 32                                             # indexed-storage internal node K (default)
        ksz = 8 + 16                                       # size, mask, 2 offsets (rank 1 + element dim)
        cur = [(lo, addr, lo) for lo, addr in recs]
        level = 0
        while True:
            cap = 2 * K
            groups = [cur[i:i + cap] for i in range(0, len(cur), cap)]
            addrs = [w.alloc(24 + ksz + cap * (ksz + 8)) for _ in groups]
            nxt = []
            for gi, g in enumerate(groups):
                left = addrs[gi - 1] if gi > 0 else UNDEF
                right = addrs[gi + 1] if gi + 1 < len(groups) else UNDEF
                body = b'TREE' + struct.pack('<BBHQQ', 1, level, len(g), left, right)
                for lo, child, _ in g:
                    body += struct.pack('<IIQQ', chunk * 4, 0, lo, 0) + struct.pack('<Q', child)
                body += struct.pack('<IIQQ', 0, 0, g[-1][2] + chunk, 0)
                w.put(addrs[gi], body)
                nxt.append((g[0][0], addrs[gi], g[-1][2]))
            if len(nxt) == 1:
                bt = nxt[0][1]
                break
            cur, level = nxt, level + 1
        layout = struct.pack('<BBBQII', 3, 2, 2, bt, chunk, 4)
    msgs = [_msg(MSG_DATASPACE, _dataspace(n)), _msg(MSG_DATATYPE, _f32_datatype(), flags=1),
            _msg(MSG_FILL, fill, flags=1), _msg(MSG_LAYOUT, layout)]
    return w.append(_object_header(msgs))


def default_chunk(n: int, itemsize: int = 4) -> int:
    """h5py's guess_chunk for a 1-D dataset (h5py/_hl/filters.py): halve the
    extent until the chunk is near a size target that grows with the dataset."""
    CHUNK_BASE, CHUNK_MIN, CHUNK_MAX = 16 * 1024, 8 * 1024, 1024 * 1024
    n = n if n != 0 else 1024                              # h5py guesses 1024 for a zero extent
    dset = n * itemsize
    target = CHUNK_BASE * (2 ** np.log10(dset / (1024.0 * 1024)))
    target = min(max(target, CHUNK_MIN), CHUNK_MAX)
    c = n
    while True:
        cb = c * itemsize
        if (cb < target or abs(cb - target) / target < 0.5) and cb < CHUNK_MAX:
            break
        if c == 1:
            break
        c = (c + 1) // 2                                   # np.ceil(c / 2)
    return c


def _write_file(path: str, w: '_Writer', sb: int, root_items) -> None:
    root, root_bt, root_heap = _write_group(w, root_items)
    eof = len(w.buf)
    sbody = SIGNATURE + struct.pack('<8B', 0, 0, 0, 0, 0, 8, 8, 0) + struct.pack('<HHI', 4, 16, 0)
    sbody += struct.pack('<QQQQ', 0, UNDEF, eof, UNDEF)
    sbody += struct.pack('<QQII', 0, root, 1, 0) + struct.pack('<QQ', root_bt, root_heap)
    assert len(sbody) == 96
    w.put(sb, sbody)
    tmp = path + '.tmp'
    with open(tmp, 'wb') as fh:
        fh.write(w.buf)
    os.replace(tmp, path)


def write_utterances(path: str, utterances: List[Dict[str, np.ndarray]], chunks: bool = True) -> None:
    """Write the reference's test-set layout: groups "0".."n-1", each with the
    four float32 signals (generate_h5files/test_wav2h5.py:44-48)."""
    w = _Writer()
    sb = w.alloc(96)
    groups = []
    for i, utt in enumerate(utterances):
        kids = []
        for key in SIGNALS:
            a = np.asarray(utt[key], np.float32).reshape(-1)
            kids.append((key, _write_dataset(w, a, default_chunk(a.size) if chunks else None)))
        gaddr, _, _ = _write_group(w, kids)
        groups.append((str(i), gaddr))
    _write_file(path, w, sb, groups)


def write_signals(path: str, utt: Dict[str, np.ndarray], chunks: bool = True) -> None:
    """Write the reference's training-file layout: one utterance per file, the
    four float32 signals at the root (generate_h5files/train_wav2h5.py:38-42,
    read by scripts/train1.py:33-40)."""
    w = _Writer()
    sb = w.alloc(96)
    kids = []
    for key in SIGNALS:
        a = np.asarray(utt[key], np.float32).reshape(-1)
        kids.append((key, _write_dataset(w, a, default_chunk(a.size) if chunks else None)))
    _write_file(path, w, sb, kids)


def read_utterance(f: File, k: int) -> Dict[str, np.ndarray]:
    """Group str(k) as scripts/test.py:25-33 reads it."""
    g = f[str(k)]
    out = {key: np.array(g[key]) for key in SIGNALS}
    out['n_samples'] = len(out['nearend_speech'])
    return out
