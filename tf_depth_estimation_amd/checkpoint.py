"""TF-1 checkpoint (V2 tensor bundle) reader/writer for the TF-named variables of the variable store.

The reference saves and restores with `tf.train.Saver(tf.model_variables())` (batch_prediction.py:49-55,
refine_depth.py:222-236) or `tf.train.Saver(GLOBAL_VARIABLES of a scope)` (split_training.py:147-202),
i.e. TensorFlow's tensor-bundle format V2.  This module reads and writes that
format directly, so a checkpoint trained with the reference restores into `disp_net` / `depth_net` here
(and one saved here restores in TF), with the Appendix D names and TF layouts kept end to end.

Format (TensorFlow tensor_bundle, restated; TF itself is not installed here, so the layout is pinned by
its published specification, not by files TF wrote -- "parity unpinned" against TF):
  <prefix>.data-00000-of-00001   raw little-endian tensor bytes, concatenated in key order
  <prefix>.index                 a LevelDB-format sorted table (SSTable):
      key ""      -> BundleHeaderProto {num_shards=1 (1), endianness=LITTLE (2), version{producer=1} (3)}
      key <name>  -> BundleEntryProto {dtype (1), shape (2), shard_id (3), offset (4), size (5),
                                       crc32c (6, fixed32: masked crc32c of the tensor bytes, as
                                       BundleWriter stores it; the reader accepts masked or raw)}
    table: data blocks of prefix-compressed entries (shared, non_shared, value_len varints + key suffix +
    value) with restart offsets every 16 entries, each block followed by a 5-byte trailer (compression
    type byte + masked crc32c of block+type); an index block mapping each data block's last key to its
    BlockHandle (offset, size varints); an empty metaindex block; a 48-byte footer (metaindex handle,
    index handle, zero padding to 40 bytes, magic 0xdb4775248b80fb57 little-endian).
  checkpoint                     CheckpointState text: model_checkpoint_path: "<basename>".
Snappy-compressed blocks (table compression type 1) are decoded too.
"""
import os
import struct

import numpy as np

# ---------------------------------------------------------------- crc32c (Castagnoli), masked form
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data, crc=0):
    """CRC-32C of `data`, continuing from `crc` (check value: crc32c(b'123456789') == 0xE3069283).
    Payloads go through libtde.so's host slicing-by-8 routine (tde_crc32c; no GPU needed)."""
    data = bytes(data)
    if len(data) > 256:
        import ctypes
        from . import _lib
        buf = ctypes.create_string_buffer(data, len(data))
        return int(_lib.load().tde_crc32c(ctypes.cast(buf, ctypes.c_void_p), len(data), crc))
    crc ^= 0xFFFFFFFF
    tab = _CRC_TABLE
    for b in data:
        crc = tab[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def mask_crc(crc):
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask_crc(m):
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------- varints and minimal protobuf
def put_varint(n):
    out = bytearray()
    n &= 0xFFFFFFFFFFFFFFFF
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def get_varint(buf, pos):
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _pb_field(num, wire, payload):
    key = put_varint((num << 3) | wire)
    if wire == 0:
        return key + put_varint(payload)
    if wire == 2:
        return key + put_varint(len(payload)) + payload
    if wire == 5:
        return key + struct.pack("<I", payload)
    raise ValueError(wire)


def _pb_parse(buf):
    """-> {field number: [values]} (varint ints, bytes for length-delimited, ints for fixed32/64)."""
    out, pos = {}, 0
    while pos < len(buf):
        key, pos = get_varint(buf, pos)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, pos = get_varint(buf, pos)
        elif wire == 2:
            n, pos = get_varint(buf, pos)
            v, pos = bytes(buf[pos:pos + n]), pos + n
        elif wire == 5:
            v, pos = struct.unpack_from("<I", buf, pos)[0], pos + 4
        elif wire == 1:
            v, pos = struct.unpack_from("<Q", buf, pos)[0], pos + 8
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
        out.setdefault(num, []).append(v)
    return out


# TensorFlow DataType enum values (types.proto) <-> numpy
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 6: np.int8, 9: np.int64, 10: np.bool_,
       19: np.float16}
_DT_INV = {np.dtype(v): k for k, v in _DT.items()}


def _entry_proto(dtype, shape, offset, size, crc):
    shp = b"".join(_pb_field(2, 2, _pb_field(1, 0, int(d))) for d in shape)
    msg = _pb_field(1, 0, dtype) + _pb_field(2, 2, shp)
    if offset:
        msg += _pb_field(4, 0, offset)
    if size:
        msg += _pb_field(5, 0, size)
    return msg + _pb_field(6, 5, crc)


def _header_proto():
    return _pb_field(1, 0, 1) + _pb_field(3, 2, _pb_field(1, 0, 1))   # num_shards 1, LITTLE (0), producer 1


# ---------------------------------------------------------------- SSTable (LevelDB table format)
_MAGIC = 0xDB4775248B80FB57


class _BlockBuilder:
    def __init__(self, restart_interval=16):
        self.buf, self.restarts, self.count, self.last, self.ri = bytearray(), [0], 0, b"", restart_interval
        self.n = 0   # entries in the block

    def add(self, key, value):
        shared = 0
        if self.count < self.ri:
            n = min(len(key), len(self.last))
            while shared < n and key[shared] == self.last[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.count = 0
        self.buf += put_varint(shared) + put_varint(len(key) - shared) + put_varint(len(value))
        self.buf += key[shared:] + value
        self.last, self.count, self.n = key, self.count + 1, self.n + 1

    def finish(self):
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))

    def size(self):
        return len(self.buf) + 4 * len(self.restarts) + 4


def _write_block(f, contents):
    off = f.tell()
    f.write(contents)
    f.write(b"\x00" + struct.pack("<I", mask_crc(crc32c(contents + b"\x00"))))
    return put_varint(off) + put_varint(len(contents))


def write_table(path, items, block_size=4096):
    """items: iterable of (key bytes, value bytes) in strictly increasing key order."""
    with open(path, "wb") as f:
        index = _BlockBuilder(restart_interval=1)
        blk = _BlockBuilder()
        last = None
        for k, v in items:
            if last is not None and k <= last:
                raise ValueError("table keys must be strictly increasing")
            blk.add(k, v)
            last = k
            if blk.size() >= block_size:
                index.add(last, _write_block(f, blk.finish()))
                blk = _BlockBuilder()
        if blk.n or not index.n:
            index.add(last if last is not None else b"", _write_block(f, blk.finish()))
        meta = _write_block(f, _BlockBuilder().finish())
        idx = _write_block(f, index.finish())
        footer = meta + idx
        f.write(footer + b"\x00" * (40 - len(footer)) + struct.pack("<Q", _MAGIC))


def _snappy_decompress(src):
    n, pos = get_varint(src, 0)
    out = bytearray()
    while pos < len(src):
        tag = src[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:                                       # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += src[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | src[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 4], "little")
            pos += 4
        for _ in range(ln):                                 # copies may overlap their source
            out.append(out[-off])
    if len(out) != n:
        raise ValueError("corrupt snappy block")
    return bytes(out)


def _read_block(data, handle, verify=True):
    off, pos = get_varint(handle, 0)
    size, _ = get_varint(handle, pos)
    contents = data[off:off + size]
    ctype = data[off + size]
    if verify:
        (m,) = struct.unpack_from("<I", data, off + size + 1)
        if unmask_crc(m) != crc32c(bytes(contents) + bytes([ctype])):
            raise ValueError("table block checksum mismatch")
    if ctype == 1:
        contents = _snappy_decompress(bytes(contents))
    elif ctype != 0:
        raise ValueError(f"unsupported table compression type {ctype}")
    return bytes(contents)


def _block_entries(block):
    (nrest,) = struct.unpack_from("<I", block, len(block) - 4)
    end = len(block) - 4 - 4 * nrest
    pos, last = 0, b""
    while pos < end:
        shared, pos = get_varint(block, pos)
        nons, pos = get_varint(block, pos)
        vlen, pos = get_varint(block, pos)
        key = last[:shared] + block[pos:pos + nons]
        pos += nons
        yield key, block[pos:pos + vlen]
        pos += vlen
        last = key


def read_table(path, verify=True):
    """-> list of (key, value) of a LevelDB-format table, in key order."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != _MAGIC:
        raise ValueError(f"{path}: not a table file (bad footer magic)")
    footer = data[len(data) - 48:]
    _, pos = get_varint(footer, 0)
    _, pos = get_varint(footer, pos)                        # metaindex handle (unused)
    idx_off, p2 = get_varint(footer, pos)
    idx_size, _ = get_varint(footer, p2)
    index = _read_block(data, put_varint(idx_off) + put_varint(idx_size), verify)
    out = []
    for _, handle in _block_entries(index):
        out.extend(_block_entries(_read_block(data, handle, verify)))
    return out


# ---------------------------------------------------------------- tensor bundle
def write_bundle(prefix, tensors):
    """tensors: {name: array-like}; writes <prefix>.index and <prefix>.data-00000-of-00001."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    entries = []
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        for name in sorted(tensors):
            a = _to_numpy(tensors[name])
            dt = _DT_INV.get(a.dtype)
            if dt is None:
                raise TypeError(f"{name}: unsupported dtype {a.dtype}")
            raw = np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            off = f.tell()
            f.write(raw)
            entries.append((name.encode(), _entry_proto(dt, a.shape, off, len(raw), mask_crc(crc32c(raw)))))
    write_table(prefix + ".index", [(b"", _header_proto())] + entries)
    return prefix


def read_bundle(prefix, names=None, verify=True):
    """-> {name: numpy array} of the bundle at `prefix` (all tensors, or `names`)."""
    items = read_table(prefix + ".index", verify)
    if not items or items[0][0] != b"":
        raise ValueError(f"{prefix}.index: missing bundle header")
    hdr = _pb_parse(items[0][1])
    nshards = hdr.get(1, [1])[0]
    if hdr.get(2, [0])[0] != 0:
        raise ValueError("big-endian bundles are not supported")
    want = None if names is None else set(names)
    shards = {}
    out = {}
    for key, val in items[1:]:
        name = key.decode()
        if want is not None and name not in want:
            continue
        e = _pb_parse(val)
        if 7 in e:
            raise ValueError(f"{name}: partitioned (sliced) variables are not supported")
        dtype = np.dtype(_DT[e[1][0]]).newbyteorder("<")
        shape = [_pb_parse(dim).get(1, [0])[0] for dim in _pb_parse(e[2][0]).get(2, [])] if 2 in e else []
        sid, off, size = e.get(3, [0])[0], e.get(4, [0])[0], e.get(5, [0])[0]
        path = f"{prefix}.data-{sid:05d}-of-{nshards:05d}"
        if path not in shards:
            with open(path, "rb") as f:
                shards[path] = f.read()
        raw = shards[path][off:off + size]
        if verify and 6 in e and crc32c(raw) not in (e[6][0], unmask_crc(e[6][0])):
            raise ValueError(f"{name}: tensor checksum mismatch")
        out[name] = np.frombuffer(raw, dtype=dtype).astype(dtype.newbyteorder("="), copy=True).reshape(shape)
    if want is not None and want - set(out):
        raise KeyError(f"not in checkpoint {prefix}: {sorted(want - set(out))}")
    return out


def list_variables(prefix):
    """tf.train.list_variables: [(name, shape)] of a bundle."""
    out = []
    for key, val in read_table(prefix + ".index")[1:]:
        e = _pb_parse(val)
        shape = [_pb_parse(dim).get(1, [0])[0] for dim in _pb_parse(e[2][0]).get(2, [])] if 2 in e else []
        out.append((key.decode(), shape))
    return out


def latest_checkpoint(checkpoint_dir):
    """tf.train.latest_checkpoint: the prefix named by <dir>/checkpoint, or None."""
    path = os.path.join(checkpoint_dir, "checkpoint")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        for line in f:
            if line.startswith("model_checkpoint_path:"):
                p = line.split(":", 1)[1].strip().strip('"')
                return p if os.path.isabs(p) else os.path.join(checkpoint_dir, p)
    return None


def _to_numpy(t):
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    return np.asarray(t)


# ---------------------------------------------------------------- Saver over the variable store
class Saver:
    """tf.train.Saver analogue over the process variable store (variables.get_store()).

    var_list: None (every model variable: weights, biases, BatchNorm/beta, BatchNorm/moving_mean,
    BatchNorm/moving_variance -- `tf.model_variables()`), a scope prefix string (GLOBAL_VARIABLES under it),
    or an explicit list of TF names.  `optimizer=True` also saves/restores the Adam slots as TF names them
    (`<var>/Adam`, `<var>/Adam_1`) -- the GLOBAL_VARIABLES form of split_training.py:147."""

    def __init__(self, var_list=None, optimizer=False):
        self.var_list, self.optimizer = var_list, optimizer

    def _tensors(self):
        from . import variables
        out = {}
        for ch in variables.get_store().chunks.values():
            # a deferred-Adam trainer may still owe this chunk the last step's update (Trainer.flush): apply it
            # before the variables are read or overwritten
            fl = getattr(ch, "pending_flush", None)
            if fl is not None:
                fl()
            out.update(ch.state_dict())
            if self.optimizer:
                for n in ch.names():
                    o, shp = ch.offsets[n], ch.shapes[n]
                    k = int(np.prod(shp))
                    out[n + "/Adam"] = ch.adam_m[o:o + k].view(shp)
                    out[n + "/Adam_1"] = ch.adam_v[o:o + k].view(shp)
        if self.var_list is None:
            return out
        if isinstance(self.var_list, str):
            pre = self.var_list.rstrip("/") + "/"
            return {k: v for k, v in out.items() if k.startswith(pre)}
        missing = [n for n in self.var_list if n not in out]
        if missing:
            raise KeyError(f"unknown variables: {missing}")
        return {n: out[n] for n in self.var_list}

    def save(self, sess, save_path, global_step=None):
        """Writes <save_path>[-<global_step>].{index,data-00000-of-00001} and the directory's `checkpoint`
        state file; returns the prefix (tf.train.Saver.save)."""
        prefix = save_path if global_step is None else f"{save_path}-{int(global_step)}"
        write_bundle(prefix, self._tensors())
        d = os.path.dirname(prefix) or "."
        base = os.path.basename(prefix)
        with open(os.path.join(d, "checkpoint"), "w") as f:
            f.write(f'model_checkpoint_path: "{base}"\nall_model_checkpoint_paths: "{base}"\n')
        return prefix

    def restore(self, sess, save_path):
        """Loads every variable of var_list from the bundle (missing names raise, like TF's
        NotFoundError); values are copied into the flat HBM buffers in place."""
        import torch
        targets = self._tensors()
        vals = read_bundle(save_path, names=list(targets))
        with torch.no_grad():
            for name, dst in targets.items():
                v = vals[name]
                if tuple(v.shape) != tuple(dst.shape):
                    raise ValueError(f"{name}: checkpoint shape {tuple(v.shape)} != variable {tuple(dst.shape)}")
                dst.copy_(torch.from_numpy(np.ascontiguousarray(v)).to(dst.dtype))
