"""TensorFlow V2 checkpoint ("tensor bundle") writer / reader in pure Python.

The reference trains with TF and saves through ``tf.train.Saver`` /
MonitoredTrainingSession (run_tffm.py:213-221): ``<prefix>.index`` +
``<prefix>.data-00000-of-00001`` + a ``checkpoint`` text file, holding
``vocab_block_{i}`` [V//N+1, K+1] float32, their ``vocab_block_{i}/Adagrad``
slots and ``global_step``.  This module writes and reads that
format without TensorFlow, so a model trained here can be handed to TF tooling
(``tf.train.load_checkpoint``) and a reference checkpoint can be imported.

Format (TF core/util/tensor_bundle + core/lib/io/table, i.e. the LevelDB table):
* ``.data-00000-of-00001``: the tensors' raw little-endian bytes, back to back;
* ``.index``: an SSTable whose keys are tensor names (sorted) and whose values
  are serialized ``BundleEntryProto`` (dtype, shape, shard_id, offset, size,
  masked crc32c of the bytes); the empty key holds a ``BundleHeaderProto``
  (num_shards, endianness, version).  Blocks: prefix-compressed entries with a
  restart array, a 5-byte trailer (compression type 0 + masked crc32c); then an
  empty metaindex block, an index block of BlockHandles and the 48-byte footer
  with magic 0xdb4775248b80fb57.
Protobufs are encoded by hand (no generated classes are available).

Parity status: unpinned — no TF install and no TF checkpoint fixture exist in
this environment; tests check the byte-level structure and a write/read round
trip against this module's own independent parser.
"""

from __future__ import annotations

import os
import struct

import numpy as np

from .metrics import crc32c, masked_crc32c

MAGIC = 0xDB4775248B80FB57
_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.int64): 9,
       np.dtype(np.bool_): 10}
_NP = {v: k for k, v in _DT.items()}
_RESTART_INTERVAL = 16
_BLOCK_SIZE = 4096


# --------------------------------------------------------------------------- protobuf wire helpers
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, pos: int) -> tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _pb_varint(num: int, v: int) -> bytes:
    return _field(num, 0) + _varint(v)


def _pb_bytes(num: int, v: bytes) -> bytes:
    return _field(num, 2) + _varint(len(v)) + v


def _pb_fixed32(num: int, v: int) -> bytes:
    return _field(num, 5) + struct.pack("<I", v)


def _parse_pb(buf: bytes) -> dict[int, list]:
    out: dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, pos = _read_varint(buf, pos)
        elif wire == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wire == 2:
            n, pos = _read_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wire == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
        out.setdefault(num, []).append(v)
    return out


def _header_proto(num_shards: int = 1) -> bytes:
    version = _pb_varint(1, 1)  # VersionDef.producer = 1 (TF's kTensorBundleVersion)
    return _pb_varint(1, num_shards) + _pb_varint(2, 0) + _pb_bytes(3, version)


def _entry_proto(dtype: int, shape: tuple[int, ...], offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_pb_bytes(2, _pb_varint(1, d)) for d in shape)
    out = _pb_varint(1, dtype) + _pb_bytes(2, dims)
    out += _pb_varint(3, 0)  # shard_id (default 0, written explicitly)
    if offset:
        out += _pb_varint(4, offset)
    out += _pb_varint(5, size) + _pb_fixed32(6, crc)
    return out


# --------------------------------------------------------------------------- SSTable (LevelDB table)
class _BlockBuilder:
    def __init__(self):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""

    def add(self, key: bytes, value: bytes) -> None:
        shared = 0
        if self.counter < _RESTART_INTERVAL:
            n = min(len(self.last), len(key))
            while shared < n and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def finish(self) -> bytes:
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4


def _write_block(f, contents: bytes) -> bytes:
    """Write a block + trailer; returns its BlockHandle encoding."""
    off = f.tell()
    f.write(contents)
    trailer_type = b"\x00"  # no compression
    f.write(trailer_type + struct.pack("<I", masked_crc32c(contents + trailer_type)))
    return _varint(off) + _varint(len(contents))


def _write_table(path: str, items: list[tuple[bytes, bytes]]) -> None:
    items = sorted(items)
    with open(path, "wb") as f:
        index = _BlockBuilder()
        blk = _BlockBuilder()
        last_key = b""
        for k, v in items:
            blk.add(k, v)
            last_key = k
            if blk.size() >= _BLOCK_SIZE:
                index.add(last_key, _write_block(f, blk.finish()))
                blk = _BlockBuilder()
        if blk.counter or not items:
            index.add(last_key, _write_block(f, blk.finish()))
        meta = _write_block(f, _BlockBuilder().finish())
        idx = _write_block(f, index.finish())
        footer = meta + idx
        footer += b"\x00" * (40 - len(footer))
        f.write(footer + struct.pack("<Q", MAGIC))


def _read_block(data: bytes, handle: bytes, pos: int = 0) -> tuple[list[tuple[bytes, bytes]], int]:
    off, pos = _read_varint(handle, pos)
    size, pos = _read_varint(handle, pos)
    contents = data[off:off + size]
    trailer = data[off + size:off + size + 5]
    if trailer[0] != 0:
        raise ValueError("compressed SSTable blocks are not supported")
    if struct.unpack("<I", trailer[1:])[0] != masked_crc32c(contents + trailer[:1]):
        raise ValueError("SSTable block checksum mismatch")
    nrest = struct.unpack_from("<I", contents, len(contents) - 4)[0]
    end = len(contents) - 4 - 4 * nrest
    out, p, key = [], 0, b""
    while p < end:
        shared, p = _read_varint(contents, p)
        nonshared, p = _read_varint(contents, p)
        vlen, p = _read_varint(contents, p)
        key = key[:shared] + contents[p:p + nonshared]
        p += nonshared
        out.append((key, contents[p:p + vlen]))
        p += vlen
    return out, pos


def _read_table(path: str) -> list[tuple[bytes, bytes]]:
    data = open(path, "rb").read()
    if len(data) < 48 or struct.unpack("<Q", data[-8:])[0] != MAGIC:
        raise ValueError(f"{path}: not an SSTable (bad magic)")
    footer = data[-48:-8]
    _, p = _read_varint(footer, 0)          # metaindex handle (skipped)
    _, p = _read_varint(footer, p)
    index, _ = _read_block(data, footer, p)
    items = []
    for _, handle in index:
        blk, _ = _read_block(data, handle)
        items.extend(blk)
    return items


# --------------------------------------------------------------------------- bundle API
def write_bundle(prefix: str, tensors: dict[str, np.ndarray]) -> list[str]:
    """Write ``<prefix>.index`` and ``<prefix>.data-00000-of-00001``; returns the two paths."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    data_path = prefix + ".data-00000-of-00001"
    entries = [(b"", _header_proto(1))]
    off = 0
    with open(data_path, "wb") as f:
        for name in sorted(tensors):
            a = np.asarray(tensors[name])
            if not a.flags.c_contiguous:  # (ascontiguousarray would turn a scalar into shape (1,))
                a = a.copy(order="C")
            if a.dtype not in _DT:
                raise TypeError(f"{name}: unsupported dtype {a.dtype}")
            raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(raw)
            entries.append((name.encode(), _entry_proto(_DT[a.dtype], a.shape, off, len(raw), masked_crc32c(raw))))
            off += len(raw)
    _write_table(prefix + ".index", entries)
    return [prefix + ".index", data_path]


def read_bundle(prefix: str) -> dict[str, np.ndarray]:
    """Read every tensor of a (single-shard) bundle, verifying each tensor's checksum."""
    items = _read_table(prefix + ".index")
    header = _parse_pb(dict(items).get(b"", b""))
    shards = header.get(1, [1])[0]
    datas = {}
    out = {}
    for key, val in items:
        if key == b"":
            continue
        e = _parse_pb(val)
        dtype = _NP[e[1][0]]
        shape = tuple(_parse_pb(dim).get(1, [0])[0] for dim in _parse_pb(e.get(2, [b""])[0]).get(2, []))
        shard = e.get(3, [0])[0]
        offset, size = e.get(4, [0])[0], e.get(5, [0])[0]
        path = f"{prefix}.data-{shard:05d}-of-{shards:05d}"
        if path not in datas:
            datas[path] = open(path, "rb").read()
        raw = datas[path][offset:offset + size]
        if 6 in e and e[6][0] != masked_crc32c(raw):
            raise ValueError(f"{key.decode()}: tensor checksum mismatch")
        out[key.decode()] = np.frombuffer(raw, dtype=dtype.newbyteorder("<")).reshape(shape).astype(dtype)
    return out


def write_checkpoint_state(log_dir: str, prefix_name: str) -> None:
    """The ``checkpoint`` text file TF's get_checkpoint_state() reads."""
    with open(os.path.join(log_dir, "checkpoint"), "w") as f:
        f.write(f'model_checkpoint_path: "{prefix_name}"\nall_model_checkpoint_paths: "{prefix_name}"\n')


__all__ = ["write_bundle", "read_bundle", "write_checkpoint_state", "crc32c"]
