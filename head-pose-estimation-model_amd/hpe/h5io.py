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


def read_training_config(path):
    """The root 'training_config' JSON attribute (None for weights-only / uncompiled saves)."""
    f = _File(path)
    tc = f.attrs(f.root).get('training_config')
    return json.loads(_txt(tc)) if tc is not None else None


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


# =============================================================================================
# Writer: Keras 2.13 legacy-HDF5 checkpoints, byte-compatible in structure with
# the files ModelCheckpoint wrote in the reference (Model-96/train_96.py:153-158): superblock v0
# (group leaf K 4, internal K 16), version-1 object headers, symbol-table groups (v1 B-tree + SNOD
# + local heap), variable-length string attributes in one global heap collection, contiguous
# little-endian datasets.  Layout of the content (keras/saving/legacy/hdf5_format.py in Keras 2.13,
# as found in the reference's files):
#   /            attrs keras_version, backend, model_config (JSON), training_config (JSON)
#   /model_weights                  attrs layer_names[], backend, keras_version
#   /model_weights/<layer>          attr weight_names[] ('<layer>/kernel:0', ...)
#   /model_weights/<layer>/<layer>/kernel:0           dataset
#   /model_weights/top_level_model_weights             attr weight_names = []
#   /optimizer_weights              attr weight_names[] ('Adam/iter:0', 'Adam/<layer>/kernel/m:0', ...)
# =============================================================================================
_UNDEF = (1 << 64) - 1
_LEAF_K, _INT_K = 4, 16
_SNOD_SIZE = 8 + 2 * _LEAF_K * 40
_TREE_SIZE = 24 + (2 * _INT_K + 1) * 8 + 2 * _INT_K * 8


def _pad8(b):
    return b + b'\0' * (-len(b) % 8)


def _dt_bytes(dt):
    dt = np.dtype(dt)
    if dt.kind == 'f' and dt.itemsize in (4, 8):
        if dt.itemsize == 4:
            return bytes([0x11, 0x20, 0x1F, 0x00]) + struct.pack('<IHHBBBBI', 4, 0, 32, 23, 8, 0, 23, 127)
        return bytes([0x11, 0x20, 0x3F, 0x00]) + struct.pack('<IHHBBBBI', 8, 0, 64, 52, 11, 0, 52, 1023)
    if dt.kind in 'iu':
        return bytes([0x10, 0x08 if dt.kind == 'i' else 0x00, 0, 0]) + struct.pack('<IHH', dt.itemsize, 0, 8 * dt.itemsize)
    raise H5Error('cannot write dtype %s' % dt)


def _vstr_dt(utf8):
    # variable-length string (class 9, type 1, null-terminated), base type uint8
    return bytes([0x19, 0x01, 0x01 if utf8 else 0x00, 0x00]) + struct.pack('<I', 16) + \
        bytes([0x10, 0, 0, 0]) + struct.pack('<IHH', 1, 0, 8)


def _space_bytes(shape):
    if shape == ():
        return bytes([1, 0, 0, 0]) + b'\0' * 4
    return bytes([1, len(shape), 1, 0]) + b'\0' * 4 + \
        b''.join(struct.pack('<Q', d) for d in shape) + b''.join(struct.pack('<Q', d) for d in shape)


class _Writer:
    def __init__(self):
        self.buf = bytearray(96)  # superblock, patched last
        self.strings = {}          # str -> global heap object index
        self.gcol = None

    def put(self, b):
        off = len(self.buf)
        self.buf += _pad8(bytes(b))
        return off

    # -- global heap ---------------------------------------------------------------------------
    def collect(self, s):
        if s not in self.strings:
            self.strings[s] = len(self.strings) + 1

    def write_gheap(self):
        objs = b''
        for s, i in sorted(self.strings.items(), key=lambda t: t[1]):
            data = s.encode('utf-8')
            objs += struct.pack('<HHIQ', i, 0, 0, len(data)) + _pad8(data)
        size = 16 + len(objs) + 16
        size = (size + 4095) // 4096 * 4096
        free = size - 16 - len(objs)
        body = b'GCOL' + bytes([1, 0, 0, 0]) + struct.pack('<Q', size) + objs + \
            struct.pack('<HHIQ', 0, 0, 0, free) + b'\0' * (free - 16)
        self.gcol = self.put(body)

    def vref(self, s):
        return struct.pack('<IQI', len(s.encode('utf-8')), self.gcol, self.strings[s])

    # -- messages -----------------------------------------------------------------------------
    def attr_msg(self, name, value):
        nm = name.encode() + b'\0'
        if not isinstance(value, str) and len(value) == 0:
            # an empty list is stored as Keras leaves it: a float64 array of shape (0,)
            dt, sp = _dt_bytes(np.float64), _space_bytes((0,))
            body = struct.pack('<BBHHH', 1, 0, len(nm), len(dt), len(sp)) + _pad8(nm) + _pad8(dt) + _pad8(sp)
            return (0x0C, 0, body)
        if isinstance(value, str):
            vals, shape = [value], ()
        else:
            vals, shape = [str(v) for v in value], (len(value),)
        utf8 = any(ord(c) > 127 for v in vals for c in v)
        dt = _vstr_dt(utf8)
        sp = _space_bytes(shape)
        data = b''.join(self.vref(v) for v in vals)
        body = struct.pack('<BBHHH', 1, 0, len(nm), len(dt), len(sp)) + _pad8(nm) + _pad8(dt) + _pad8(sp) + data
        return (0x0C, 0, body)

    def header(self, msgs):
        body = b''
        for t, flags, data in msgs:
            data = _pad8(data)
            body += struct.pack('<HHB3x', t, len(data), flags) + data
        return self.put(struct.pack('<BBHII4x', 1, 0, len(msgs), 1, len(body)) + body)

    # -- objects ------------------------------------------------------------------------------
    def dataset(self, arr):
        arr = np.asarray(arr)  # (not ascontiguousarray: it turns 0-d into shape (1,))
        dt = arr.dtype.newbyteorder('<') if arr.dtype.byteorder == '>' else arr.dtype
        raw = np.asarray(arr, dtype=dt).tobytes(order='C')
        addr = self.put(raw) if raw else _UNDEF
        msgs = [(0x01, 0, _space_bytes(tuple(arr.shape))),
                (0x03, 1, _dt_bytes(dt)),
                (0x05, 1, bytes([2, 2, 2, 1, 0, 0, 0, 0])),
                (0x08, 0, struct.pack('<BBQQ', 3, 1, addr, len(raw)))]
        return self.header(msgs)

    def group(self, node):
        """node: {'attrs': [(name, value)], 'children': {name: node | ndarray}} -> (ohdr, btree, heap)"""
        ents = []
        for name in sorted(node['children'], key=lambda s: s.encode()):
            ch = node['children'][name]
            if isinstance(ch, dict):
                oh, bt, hp = self.group(ch)
                ents.append((name, oh, 1, struct.pack('<QQ', bt, hp)))
            else:
                ents.append((name, self.dataset(ch), 0, b'\0' * 16))
        # local heap: "" at 0, then the names, then one free block (as libhdf5 leaves it)
        heap_data = b'\0' * 8
        name_off = {}
        for name, *_ in ents:
            name_off[name] = len(heap_data)
            heap_data += _pad8(name.encode() + b'\0')
        free_off = len(heap_data)
        heap_data += struct.pack('<QQ', 1, 16)
        heap = len(self.buf)
        self.put(b'HEAP' + bytes([0, 0, 0, 0]) + struct.pack('<QQQ', len(heap_data), free_off, heap + 32) + heap_data)
        # symbol-table nodes of <= 2K entries, then the B-tree over them
        leaves = []
        for i in range(0, len(ents), 2 * _LEAF_K):
            chunk = ents[i:i + 2 * _LEAF_K]
            b = b'SNOD' + bytes([1, 0]) + struct.pack('<H', len(chunk))
            for name, oh, ctype, scratch in chunk:
                b += struct.pack('<QQII', name_off[name], oh, ctype, 0) + scratch
            b += b'\0' * (_SNOD_SIZE - len(b))
            leaves.append((self.put(b), name_off[chunk[-1][0]]))
        level = 0
        nodes = leaves
        while True:
            parents = []
            for i in range(0, max(len(nodes), 1), 2 * _INT_K):
                chunk = nodes[i:i + 2 * _INT_K]
                b = b'TREE' + bytes([0, level]) + struct.pack('<HQQ', len(chunk), _UNDEF, _UNDEF)
                b += struct.pack('<Q', 0)
                for child, key in chunk:
                    b += struct.pack('<QQ', child, key)
                b += b'\0' * (_TREE_SIZE - len(b))
                parents.append((self.put(b), chunk[-1][1] if chunk else 0))
            if len(parents) == 1:
                btree = parents[0][0]
                break
            nodes, level = parents, level + 1
        msgs = [(0x11, 0, struct.pack('<QQ', btree, heap))]
        msgs += [self.attr_msg(n, v) for n, v in node.get('attrs', [])]
        return self.header(msgs), btree, heap

    def finish(self, root):
        oh, bt, hp = root
        sb = b'\x89HDF\r\n\x1a\n' + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack('<HHI', _LEAF_K, _INT_K, 0)
        sb += struct.pack('<QQQQ', 0, _UNDEF, len(self.buf), _UNDEF)
        sb += struct.pack('<QQII', 0, oh, 1, 0) + struct.pack('<QQ', bt, hp)
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def _walk_strings(node, w):
    for n, v in node.get('attrs', []):
        for s in ([v] if isinstance(v, str) else v):
            w.collect(str(s))
    for ch in node['children'].values():
        if isinstance(ch, dict):
            _walk_strings(ch, w)


def _insert(node, path, leaf):
    parts = path.split('/')
    for p in parts[:-1]:
        node = node['children'].setdefault(p, {'attrs': [], 'children': {}})
    node['children'][parts[-1]] = leaf


def write_keras_h5(path, model_config, layer_weights, training_config=None, optimizer_weights=None,
                   keras_version='2.13.1', backend='tensorflow'):
    """Write a Keras 2.13 legacy .h5 checkpoint.

    layer_weights: [(layer_name, [(weight_name, array), ...]), ...] in model.layers order, weight
    names as Keras gives them ('conv2d/kernel:0'); optimizer_weights: [(name, array), ...] with
    legacy names ('Adam/iter:0', 'Adam/conv2d/kernel/m:0', ...) or None."""
    root = {'attrs': [('keras_version', keras_version), ('backend', backend),
                      ('model_config', json.dumps(model_config))], 'children': {}}
    if training_config is not None:
        root['attrs'].append(('training_config', json.dumps(training_config)))
    mw = {'attrs': [('layer_names', [ln for ln, _ in layer_weights]), ('backend', backend),
                    ('keras_version', keras_version)], 'children': {}}
    root['children']['model_weights'] = mw
    for ln, ws in layer_weights:
        g = {'attrs': [('weight_names', [wn for wn, _ in ws])], 'children': {}}
        mw['children'][ln] = g
        for wn, arr in ws:
            _insert(g, wn, np.asarray(arr))
    mw['children'].setdefault('top_level_model_weights', {'attrs': [('weight_names', [])], 'children': {}})
    if optimizer_weights:
        og = {'attrs': [('weight_names', [n for n, _ in optimizer_weights])], 'children': {}}
        root['children']['optimizer_weights'] = og
        for n, arr in optimizer_weights:
            _insert(og, n, np.asarray(arr))
    w = _Writer()
    _walk_strings(root, w)
    w.write_gheap()
    data = w.finish(w.group(root))
    with open(path, 'wb') as fh:
        fh.write(data)
