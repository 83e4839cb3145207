"""Metrics: stdout lines, JSONL, and TensorBoard event files.

Reference: ``tf.summary.scalar('loss')`` and ``tf.summary.scalar('exq_size')``
(tffm/fm_model.py:338-339) written by MonitoredTrainingSession every
``save_summaries_steps`` to ``log_dir`` (run_tffm.py:217-220), read with
TensorBoard (README.md:78-88); everything else is stdout ``print``.

TensorBoard is not installed in this image, so :class:`EventFileWriter`
writes the event-file format directly: TFRecord framing (length, masked
CRC32C, payload, masked CRC32C) around hand-encoded ``Event``/``Summary``
protobuf messages.  The files open in any TensorBoard.
"""

from __future__ import annotations

import json
import os
import socket
import struct
import time

# ---------------------------------------------------------------------------
# CRC32C (Castagnoli), table driven
# ---------------------------------------------------------------------------
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def _crc32c_py(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def crc32c(data) -> int:
    """CRC-32C of bytes / a contiguous buffer (native SSE4.2 path, Python fallback)."""
    try:
        from ..ops import native

        return int(native.cpu().crc32c(memoryview(data).cast("B")))
    except Exception:  # noqa: BLE001  (extension unavailable)
        return _crc32c_py(bytes(data))


def masked_crc32c(data) -> int:
    """TFRecord / LevelDB checksum masking: rotate right by 15, add 0xa282ead8."""
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


_masked_crc = masked_crc32c


# ---------------------------------------------------------------------------
# protobuf wire encoding (just what Event/Summary need)
# ---------------------------------------------------------------------------
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


def _key(field: int, wtype: int) -> bytes:
    return _varint((field << 3) | wtype)


def _len_delim(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _summary_value(tag: str, value: float) -> bytes:
    # Summary.Value { string tag = 1; float simple_value = 2; }
    return _len_delim(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))


def _event(wall_time: float, step: int, *, file_version: str | None = None,
           scalars: dict[str, float] | None = None) -> bytes:
    # Event { double wall_time = 1; int64 step = 2; string file_version = 3; Summary summary = 5; }
    msg = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        msg += _len_delim(3, file_version.encode())
    if scalars:
        summary = b"".join(_len_delim(1, _summary_value(k, v)) for k, v in scalars.items())
        msg += _len_delim(5, summary)
    return msg


class EventFileWriter:
    """Append-only TensorBoard event file (events.out.tfevents.<time>.<host>)."""

    def __init__(self, log_dir: str, suffix: str = ""):
        os.makedirs(log_dir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{suffix}"
        self.path = os.path.join(log_dir, name)
        self._f = open(self.path, "ab")
        self._write(_event(time.time(), 0, file_version="brain.Event:2"))

    def _write(self, rec: bytes) -> None:
        header = struct.pack("<Q", len(rec))
        self._f.write(header + struct.pack("<I", _masked_crc(header)) + rec + struct.pack("<I", _masked_crc(rec)))

    def scalars(self, step: int, values: dict[str, float]) -> None:
        self._write(_event(time.time(), step, scalars=values))
        self._f.flush()

    def close(self) -> None:
        self._f.close()


def read_event_scalars(path: str) -> list[tuple[int, dict[str, float]]]:
    """Minimal reader (tests): [(step, {tag: value})] for scalar events."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, pos)
        rec = data[pos + 12: pos + 12 + n]
        assert struct.unpack_from("<I", data, pos + 8)[0] == _masked_crc(data[pos:pos + 8])
        assert struct.unpack_from("<I", data, pos + 12 + n)[0] == _masked_crc(rec)
        pos += 12 + n + 4
        step, vals = _decode_event(rec)
        if vals:
            out.append((step, vals))
    return out


def _read_varint(b: bytes, i: int):
    shift = val = 0
    while True:
        c = b[i]
        i += 1
        val |= (c & 0x7F) << shift
        if not c & 0x80:
            return val, i
        shift += 7


def _decode_event(rec: bytes):
    i, step, vals = 0, 0, {}
    while i < len(rec):
        k, i = _read_varint(rec, i)
        field, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(rec, i)
            if field == 2:
                step = v
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        elif wt == 2:
            ln, i = _read_varint(rec, i)
            payload = rec[i:i + ln]
            i += ln
            if field == 5:
                j = 0
                while j < len(payload):
                    _, j = _read_varint(payload, j)
                    vl, j = _read_varint(payload, j)
                    val_msg = payload[j:j + vl]
                    j += vl
                    tag, x, q = None, None, 0
                    while q < len(val_msg):
                        kk, q = _read_varint(val_msg, q)
                        if kk >> 3 == 1:
                            ll, q = _read_varint(val_msg, q)
                            tag = val_msg[q:q + ll].decode()
                            q += ll
                        elif kk >> 3 == 2:
                            (x,) = struct.unpack_from("<f", val_msg, q)
                            q += 4
                        else:
                            break
                    if tag is not None:
                        vals[tag] = x
    return step, vals


class MetricsLogger:
    """Per-step metrics -> JSONL (``metrics.jsonl``) and TensorBoard events in ``log_dir``."""

    def __init__(self, log_dir: str | None, every: int = 100, enabled: bool = True):
        self.every = max(1, int(every))
        self.enabled = enabled and log_dir is not None
        self._jsonl = None
        self._tb = None
        if self.enabled:
            os.makedirs(log_dir, exist_ok=True)
            self._jsonl = open(os.path.join(log_dir, "metrics.jsonl"), "a")
            self._tb = EventFileWriter(log_dir)

    def log(self, step: int, force: bool = False, **values) -> None:
        if not self.enabled or (step % self.every and not force):
            return
        rec = {"step": int(step), "time": time.time()}
        rec.update({k: float(v) for k, v in values.items()})
        self._jsonl.write(json.dumps(rec) + "\n")
        self._jsonl.flush()
        self._tb.scalars(step, {k: float(v) for k, v in values.items()})

    def close(self) -> None:
        if self._jsonl:
            self._jsonl.close()
        if self._tb:
            self._tb.close()
