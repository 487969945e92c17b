"""Read Keras 2.13 ``.h5`` checkpoints in-process: the reference's model files
(``Model-96/test.py:31`` and ``BlazePoser/blazeFaceDetectorH5.py:90`` call keras.models.load_model on
them) load straight into hpe, without h5py (absent from the image's Python).

A minimal HDF5 reader for the subset Keras / h5py ('earliest' file format) writes: superblock v0/v1,
version-1 object headers (+ continuation blocks), symbol-table groups (v1 B-trees, symbol-table
nodes, local heaps), attributes (v1-v3 messages) of fixed-length / variable-length strings (global
heap) and numbers, contiguous / compact datasets of little-endian floats and ints.  Read as data
only: the ``model_config`` JSON attribute and the weight arrays; Lambda layers' marshalled bytecode
is dropped, never executed.
"""
import json
import struct

import numpy as np


class H5Error(ValueError):
    pass


class _File:
    def __init__(self, path):
        with open(path, 'rb') as fh:
            self.b = fh.read()
        b = self.b
        if b[:8] != b'\x89HDF\r\n\x1a\n':
            raise H5Error('%s: not an HDF5 file' % path)
        ver = b[8]
        if ver not in (0, 1):
            raise H5Error('HDF5 superblock version %d not supported (Keras/h5py "earliest" files use 0)' % ver)
        self.so, self.sl = b[13], b[14]
        if self.so != 8 or self.sl != 8:
            raise H5Error('HDF5 offsets/lengths of %d/%d bytes not supported' % (self.so, self.sl))
        p = 24 if ver == 0 else 28
        self.base = self.u(p, 8)
        p += 32  # base, free-space, EOF, driver-info addresses
        # root group symbol table entry
        self.root = self.u(p + 8, 8)
        self._gheap = {}

    def u(self, off, n):
        return int.from_bytes(self.b[off:off + n], 'little')

    # -- object headers --------------------------------------------------------------------------
    def messages(self, addr):
        b = self.b
        if b[addr:addr + 4] == b'OHDR':
            raise H5Error('version-2 object headers not supported')
        if b[addr] != 1:
            raise H5Error('object header version %d not supported' % b[addr])
        nmsg = self.u(addr + 2, 2)
        size = self.u(addr + 8, 4)
        blocks = [(addr + 16, size)]
        out = []
        while blocks and len(out) < nmsg:
            p, n = blocks.pop(0)
            end = p + n
            while p + 8 <= end and len(out) < nmsg:
                mtype, msize = self.u(p, 2), self.u(p + 2, 2)
                data = p + 8
                if mtype == 0x10:  # continuation
                    blocks.append((self.u(data, 8), self.u(data + 8, 8)))
                out.append((mtype, data, msize))
                p = data + msize
        return out

    # -- datatypes / dataspaces ------------------------------------------------------------------
    def dtype(self, p):
        b0 = self.b[p]
        cls, ver = b0 & 0x0F, b0 >> 4
        bits = self.u(p + 1, 3)
        size = self.u(p + 4, 4)
        props = p + 8
        if cls == 0:   # fixed point
            signed = bool(bits & 0x08)
            big = bool(bits & 0x01)
            dt = np.dtype(('>' if big else '<') + ('i' if signed else 'u') + str(size))
            return ('num', dt, size, props + 4)
        if cls == 1:   # floating point
            big = bool(bits & 0x01)
            dt = np.dtype(('>' if big else '<') + 'f' + str(size))
            return ('num', dt, size, props + 12)
        if cls == 3:   # fixed-length string
            return ('str', None, size, props)
        if cls == 9:   # variable length
            vtype = bits & 0x0F
            base = self.dtype(props)
            if vtype == 1:
                return ('vstr', None, size, props)
            return ('vseq', base, size, props)
        raise H5Error('HDF5 datatype class %d not supported' % cls)

    def dspace(self, p):
        ver, nd, flags = self.b[p], self.b[p + 1], self.b[p + 2]
        q = p + (8 if ver == 1 else 4)
        if ver == 2 and self.b[p + 3] == 0:
            return ()  # scalar
        return tuple(self.u(q + 8 * i, 8) for i in range(nd))

    def gheap_obj(self, coll, idx):
        if coll not in self._gheap:
            b = self.b
            if b[coll:coll + 4] != b'GCOL':
                raise H5Error('bad global heap collection')
            csize = self.u(coll + 8, 8)
            objs = {}
            p, end = coll + 16, coll + csize
            while p + 16 <= end:
                oi, osz = self.u(p, 2), self.u(p + 8, 8)
                if oi == 0:
                    break
                objs[oi] = b[p + 16:p + 16 + osz]
                p += 16 + ((osz + 7) & ~7)
            self._gheap[coll] = objs
        return self._gheap[coll][idx]

    def values(self, dt, shape, data):
        kind, ndt, size, _ = dt
        n = int(np.prod(shape)) if shape else 1
        if kind == 'num':
            a = np.frombuffer(self.b, dtype=ndt, count=n, offset=data)
            return a.reshape(shape) if shape else a[0]
        if kind == 'str':
            items = [self.b[data + i * size:data + (i + 1) * size].split(b'\0')[0] for i in range(n)]
            return np.array(items).reshape(shape) if shape else items[0]
        if kind == 'vstr':
            items = []
            for i in range(n):
                q = data + i * 16
                ln, coll, idx = self.u(q, 4), self.u(q + 4, 8), self.u(q + 12, 4)
                items.append(self.gheap_obj(coll, idx)[:ln].decode('utf-8') if ln else '')
            return items if shape else items[0]
        raise H5Error('HDF5 value kind %s not supported' % kind)

    # -- attributes ------------------------------------------------------------------------------
    def attrs(self, addr):
        out = {}
        for mtype, p, _ in self.messages(addr):
            if mtype != 0x0C:
                continue
            ver = self.b[p]
            nsz, tsz, ssz = self.u(p + 2, 2), self.u(p + 4, 2), self.u(p + 6, 2)
            q = p + 8 + (1 if ver == 3 else 0)
            pad = (lambda n: (n + 7) & ~7) if ver == 1 else (lambda n: n)
            name = self.b[q:q + nsz].split(b'\0')[0].decode()
            q += pad(nsz)
            dt = self.dtype(q)
            q += pad(tsz)
            shape = self.dspace(q)
            q += pad(ssz)
            out[name] = self.values(dt, shape, q)
        return out

    # -- groups / datasets -----------------------------------------------------------------------
    def children(self, addr):
        st = [(p) for t, p, _ in self.messages(addr) if t == 0x11]
        if not st:
            return None  # not a group
        btree, heap = self.u(st[0], 8), self.u(st[0] + 8, 8)
        if self.b[heap:heap + 4] != b'HEAP':
            raise H5Error('bad local heap')
        hdata = self.u(heap + 24, 8)
        out = {}

        def walk(node):
            b = self.b
            if b[node:node + 4] != b'TREE':
                raise H5Error('bad B-tree node')
            level, used = b[node + 5], self.u(node + 6, 2)
            p = node + 24 + 8  # header, then key 0
            for i in range(used):
                child = self.u(p, 8)
                p += 16  # child + next key
                if level > 0:
                    walk(child)
                    continue
                if b[child:child + 4] != b'SNOD':
                    raise H5Error('bad symbol table node')
                ns = self.u(child + 6, 2)
                for j in range(ns):
                    e = child + 8 + 40 * j
                    nm = b[hdata + self.u(e, 8):].split(b'\0', 1)[0].decode()
                    out[nm] = self.u(e + 8, 8)
        walk(btree)
        return out

    def dataset(self, addr):
        dt = shape = None
        data = None
        for mtype, p, msize in self.messages(addr):
            if mtype == 0x03:
                dt = self.dtype(p)
            elif mtype == 0x01:
                shape = self.dspace(p)
            elif mtype == 0x08:
                ver = self.b[p]
                if ver != 3:
                    raise H5Error('data layout message v%d not supported' % ver)
                cls = self.b[p + 1]
                if cls == 1:
                    data = self.u(p + 2, 8)
                elif cls == 0:
                    data = p + 4
                else:
                    raise H5Error('chunked datasets not supported (Keras writes contiguous ones)')
        if dt is None or shape is None or data is None:
            raise H5Error('incomplete dataset header')
        n = int(np.prod(shape)) if shape else 1
        if data == (1 << 64) - 1:  # never written: fill value zeros
            return np.zeros(shape, dt[1])
        return np.array(self.values(dt, shape, data), copy=True)

    def get(self, path):
        addr = self.root
        for part in [p for p in path.split('/') if p]:
            ch = self.children(addr)
            if ch is None or part not in ch:
                raise KeyError(path)
            addr = ch[part]
        return addr


def _txt(v):
    return v.decode() if isinstance(v, (bytes, np.bytes_)) else str(v)


def read_keras_h5(path, with_optimizer=False):
    """(model_config dict, weights {'<layer>/<var>': float32 array}) of a Keras .h5 checkpoint
    (optionally also the legacy optimizer state {'<name>': array})."""
    f = _File(path)
    ra = f.attrs(f.root)
    if 'model_config' not in ra:
        raise H5Error('%s: no model_config attribute (weights-only file?)' % path)
    mc = json.loads(_txt(ra['model_config']))
    for l in mc.get('config', {}).get('layers', []):
        if l.get('class_name') == 'Lambda':
            l['config']['function'] = '<bytecode stripped>'  # data only, never executed
    mw = f.get('model_weights')
    names = f.attrs(mw).get('layer_names', [])
    w = {}
    for ln in np.atleast_1d(names):
        ln = _txt(ln)
        g = f.get('model_weights/' + ln)
        for wn in np.atleast_1d(f.attrs(g).get('weight_names', [])):
            wn = _txt(wn)
            arr = f.dataset(f.get('model_weights/%s/%s' % (ln, wn)))
            # '<layer>/<var>'; a nested Functional layer's weights get its name in front
            # ('model/conv2d/kernel'), as the executors' flattened graphs name them
            key = wn.replace(':0', '')
            if not key.startswith(ln + '/'):
                key = ln + '/' + key
            w[key] = np.asarray(arr, dtype=np.float32) if arr.dtype.kind == 'f' else arr
    if not with_optimizer:
        return mc, w
    opt = {}
    try:
        og = f.get('optimizer_weights')
    except KeyError:
        return mc, w, opt
    for wn in np.atleast_1d(f.attrs(og).get('weight_names', [])):
        wn = _txt(wn)
        opt[wn.replace(':0', '')] = f.dataset(f.get('optimizer_weights/' + wn))
    return mc, w, opt
