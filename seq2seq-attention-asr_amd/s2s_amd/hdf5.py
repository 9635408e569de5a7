"""A minimal pure-Python HDF5 reader for the corpus files of the reference.

The reference's preprocessing writes its corpora with h5py's defaults (timit/preprocess_timit.py:341-363,
librispeech/preprocess.py:230-253): superblock version 0, groups as symbol tables (v1 B-tree + local
heap), datasets of little-endian integers / floats in contiguous (or compact) storage.  h5py is not part
of this image, so this module reads exactly that subset of the HDF5 file format -- enough for
`s2s_amd.data` to load the reference's files offline:
  * superblock v0 / v1 (8-byte offsets and lengths);
  * object headers v1 and v2 ("OHDR"), with continuation blocks;
  * groups: symbol-table message (0x11) -> v1 B-tree ("TREE") of symbol-table nodes ("SNOD"), names
    in the local heap ("HEAP"); compact link messages (0x06) of v2 groups;
  * datasets: dataspace (0x01), datatype (0x03: fixed-point and IEEE float, either byte order), data
    layout (0x08: compact or contiguous; unallocated storage reads as zeros).
Chunked / filtered storage and other datatype classes raise NotImplementedError for that dataset.

    tree = read_tree(path)          # {"group/sub/name": np.ndarray}
"""
import struct

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class _File:
    def __init__(self, path):
        with open(path, "rb") as f:
            self.b = f.read()
        if self.b[:8] != SIG:
            raise ValueError(f"{path}: not an HDF5 file")
        ver = self.b[8]
        if ver not in (0, 1):
            raise NotImplementedError(f"{path}: HDF5 superblock version {ver} (only 0 and 1 are read)")
        self.so, self.sl = self.b[13], self.b[14]
        if self.so != 8 or self.sl != 8:
            raise NotImplementedError("HDF5 offsets / lengths other than 8 bytes")
        p = 24 + (4 if ver == 1 else 0)
        self.base = self.u(p, 8)
        self.root_entry = p + 4 * 8  # base, free-space, EOF, driver info addresses

    def u(self, p, n):
        return int.from_bytes(self.b[p:p + n], "little")

    # ---------------------------------------------------------------- object headers
    def messages(self, addr):
        """[(type, data bytes)] of the object header at addr (v1 or v2), continuations followed."""
        b, out = self.b, []
        if b[addr:addr + 4] == b"OHDR":
            flags = b[addr + 5]
            p = addr + 6 + (16 if flags & 0x20 else 0) + (4 if flags & 0x10 else 0)
            csz = 1 << (flags & 3)
            size = self.u(p, csz)
            p += csz
            blocks = [(p, p + size)]
            track = bool(flags & 0x04)
            while blocks:
                s, e = blocks.pop(0)
                while s + 4 <= e - 4:  # leave the 4-byte checksum
                    mtype, msize = b[s], self.u(s + 1, 2)
                    s += 4 + (2 if track else 0)
                    data = b[s:s + msize]
                    s += msize
                    if mtype == 0x10:
                        caddr, clen = struct.unpack_from("<QQ", data)
                        blocks.append((caddr + 4, caddr + clen))  # skip "OCHK"
                    elif mtype:
                        out.append((mtype, data))
            return out
        if b[addr] != 1:
            raise NotImplementedError(f"HDF5 object header version {b[addr]}")
        nmsg = self.u(addr + 2, 2)
        size = self.u(addr + 8, 4)
        blocks = [(addr + 16, addr + 16 + size)]
        while blocks and len(out) < nmsg:
            s, e = blocks.pop(0)
            while s + 8 <= e and len(out) < nmsg:
                mtype, msize = self.u(s, 2), self.u(s + 2, 2)
                data = b[s + 8:s + 8 + msize]
                s += 8 + msize
                if mtype == 0x10:
                    caddr, clen = struct.unpack_from("<QQ", data)
                    blocks.append((caddr, caddr + clen))
                out.append((mtype, data))
        return out

    # ---------------------------------------------------------------- groups
    def heap_name(self, heap, off):
        if self.b[heap:heap + 4] != b"HEAP":
            raise ValueError("bad HDF5 local heap")
        data = self.u(heap + 24, 8)
        end = self.b.index(b"\0", data + off)
        return self.b[data + off:end].decode()

    def group_children(self, msgs):
        """{name: object header address} of a group's links."""
        kids = {}
        for mtype, data in msgs:
            if mtype == 0x11:  # symbol table: v1 B-tree + local heap
                btree, heap = struct.unpack_from("<QQ", data)
                self._btree(btree, heap, kids)
            elif mtype == 0x06:  # link message (compact v2 groups), hard links only
                flags = data[1]
                p = 2 + (1 if flags & 0x08 else 0)
                ltype = data[p - 1] if flags & 0x08 else 0
                p += 8 if flags & 0x04 else 0
                p += 1 if flags & 0x10 else 0
                nlen_sz = 1 << (flags & 3)
                nlen = int.from_bytes(data[p:p + nlen_sz], "little")
                p += nlen_sz
                name = data[p:p + nlen].decode()
                p += nlen
                if ltype == 0:
                    kids[name] = int.from_bytes(data[p:p + 8], "little")
        return kids

    def _btree(self, addr, heap, kids):
        b = self.b
        if b[addr:addr + 4] != b"TREE":
            raise ValueError("bad HDF5 B-tree node")
        level, used = b[addr + 5], self.u(addr + 6, 2)
        p = addr + 24 + 8  # header, then key 0
        for _ in range(used):
            child = self.u(p, 8)
            p += 16  # child, next key
            if level > 0:
                self._btree(child, heap, kids)
            else:
                self._snod(child, heap, kids)

    def _snod(self, addr, heap, kids):
        if self.b[addr:addr + 4] != b"SNOD":
            raise ValueError("bad HDF5 symbol table node")
        n = self.u(addr + 6, 2)
        p = addr + 8
        for _ in range(n):
            name_off, ohdr = struct.unpack_from("<QQ", self.b, p)
            kids[self.heap_name(heap, name_off)] = ohdr
            p += 40

    # ---------------------------------------------------------------- datasets
    def dataset(self, msgs):
        shape = dtype = layout = None
        for mtype, data in msgs:
            if mtype == 0x01:
                ver, ndim, flags = data[0], data[1], data[2]
                p = 8 if ver == 1 else 4
                shape = tuple(struct.unpack_from(f"<{ndim}Q", data, p)) if ndim else ()
                if ver == 2 and data[3] == 0:
                    shape = ()
            elif mtype == 0x03:
                cls, bits, size = data[0] & 0x0F, data[1], struct.unpack_from("<I", data, 4)[0]
                order = ">" if bits & 1 else "<"
                if cls == 0:
                    dtype = np.dtype(f"{order}{'i' if bits & 0x08 else 'u'}{size}")
                elif cls == 1 and size in (2, 4, 8):
                    dtype = np.dtype(f"{order}f{size}")
                else:
                    raise NotImplementedError(f"HDF5 datatype class {cls} (size {size})")
            elif mtype == 0x08:
                layout = data
            elif mtype == 0x0B:
                raise NotImplementedError("filtered (compressed) HDF5 datasets")
        if shape is None or dtype is None or layout is None:
            raise ValueError("HDF5 dataset without dataspace / datatype / layout")
        n = int(np.prod(shape)) if shape else 1
        ver = layout[0]
        if ver == 3:
            cls = layout[1]
            if cls == 0:
                size = struct.unpack_from("<H", layout, 2)[0]
                raw = layout[4:4 + size]
            elif cls == 1:
                addr, size = struct.unpack_from("<QQ", layout, 2)
                raw = None if addr == UNDEF else self.b[addr:addr + size]
            else:
                raise NotImplementedError("chunked HDF5 datasets")
        elif ver in (1, 2):
            ndim, cls = layout[1], layout[2]
            if cls == 1:
                addr = struct.unpack_from("<Q", layout, 8)[0]
                raw = None if addr == UNDEF else self.b[addr:addr + n * dtype.itemsize]
            elif cls == 0:
                p = 8 + 4 * ndim
                size = struct.unpack_from("<I", layout, p)[0]
                raw = layout[p + 4:p + 4 + size]
            else:
                raise NotImplementedError("chunked HDF5 datasets")
        else:
            raise NotImplementedError(f"HDF5 data layout message version {ver}")
        if raw is None:
            return np.zeros(shape, dtype.newbyteorder("="))
        return np.frombuffer(raw, dtype, count=n).reshape(shape).astype(dtype.newbyteorder("="))


def read_tree(path, skip_unsupported=True):
    """{hdf5 path: ndarray} of every dataset in the file (groups flattened with '/')."""
    f = _File(path)
    root = struct.unpack_from("<Q", f.b, f.root_entry + 8)[0]
    out = {}

    def walk(addr, prefix, seen):
        if addr in seen:
            return
        seen.add(addr)
        msgs = f.messages(addr)
        types = {t for t, _ in msgs}
        if 0x11 in types or (0x06 in types and 0x08 not in types):
            try:
                kids = f.group_children(msgs)
            except (ValueError, IndexError, NotImplementedError):  # e.g. soft / external links
                if not skip_unsupported:
                    raise
                return
            for name, child in kids.items():
                walk(child, prefix + name + "/", seen)
        elif 0x08 in types:
            try:
                out[prefix[:-1]] = f.dataset(msgs)
            except NotImplementedError:
                if not skip_unsupported:
                    raise

    walk(root, "", set())
    return out
