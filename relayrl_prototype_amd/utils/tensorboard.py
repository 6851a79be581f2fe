"""TensorBoard scalars without the tensorboard package (not installed on the image).

Reference: training_tensorboard.py tails the newest ``progress.txt`` and writes the
configured ``scalar_tags`` with ``SummaryWriter`` (training_tensorboard.py:118-253); the
Rust side spawned it without arguments, so it never worked (A8).  Here a thread tails the
same file and writes TF event files directly: TFRecord framing (length, masked CRC32C,
payload, masked CRC32C) around hand-encoded ``Event{wall_time, step, summary{value{tag,
simple_value}}}`` protobufs.
"""
from __future__ import annotations

import glob
import os
import socket
import struct
import threading
import time
from typing import List, Optional

_CRC_TABLE = []


def _crc_table():
    if not _CRC_TABLE:
        poly = 0x82F63B78
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            _CRC_TABLE.append(c)
    return _CRC_TABLE


def crc32c(data: bytes) -> int:
    t = _crc_table()
    c = 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wt: int) -> bytes:
    return _varint((num << 3) | wt)


def _ld(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    val = _ld(1, tag.encode()) + _field(2, 5) + struct.pack("<f", float(value))  # Summary.Value
    summary = _ld(1, val)
    ev = _field(1, 1) + struct.pack("<d", wall_time or time.time()) + _field(2, 0) + _varint(int(step))
    return ev + _ld(5, summary)


def encode_file_version_event() -> bytes:
    return _field(1, 1) + struct.pack("<d", time.time()) + _ld(3, b"brain.Event:2")


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}"
        self.path = os.path.join(logdir, name)
        self.f = open(self.path, "wb")
        self._write(encode_file_version_event())

    def _write(self, rec: bytes):
        hdr = struct.pack("<Q", len(rec))
        self.f.write(hdr + struct.pack("<I", _masked(crc32c(hdr))) + rec + struct.pack("<I", _masked(crc32c(rec))))

    def add_scalar(self, tag: str, value: float, step: int):
        self._write(encode_scalar_event(tag, value, step))

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()


def read_events(path: str):
    """Decode (tag, value, step) triples back (used by tests)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i + 12 <= len(data):
        (n,) = struct.unpack("<Q", data[i:i + 8])
        rec = data[i + 12:i + 12 + n]
        assert struct.unpack("<I", data[i + 12 + n:i + 16 + n])[0] == _masked(crc32c(rec))
        i += 16 + n
        if b"brain.Event" in rec:
            continue
        # minimal parse: step varint after field 2, tag/value inside field 5
        j = 9  # skip wall_time
        step = 0
        if rec[j] == 0x10:
            j += 1
            shift = 0
            while True:
                b = rec[j]
                step |= (b & 0x7F) << shift
                j += 1
                shift += 7
                if not b & 0x80:
                    break
        k = rec.find(b"\x0a", j + 2)
        tl = rec[k + 3]
        tag = rec[k + 4:k + 4 + tl].decode()
        (val,) = struct.unpack("<f", rec[k + 5 + tl:k + 9 + tl])
        out.append((tag, val, step))
    return out


class ProgressTensorboard:
    """Tail the newest logs/**/progress.txt and mirror ``scalar_tags`` into event files."""

    def __init__(self, logs_dir: str, scalar_tags: List[str], global_step_tag: str = "Epoch", poll_s: float = 1.0):
        self.logs_dir = logs_dir
        self.tags = [t for t in scalar_tags if t]
        self.step_tag = global_step_tag
        self.poll_s = poll_s
        self._stop = threading.Event()
        self._thread = None
        self._writer = None
        self._file = None
        self._pos = 0
        self._header = None

    def _newest(self):
        files = glob.glob(os.path.join(self.logs_dir, "**", "progress.txt"), recursive=True)
        return max(files, key=os.path.getmtime) if files else None

    def poll_once(self):
        path = self._newest()
        if path is None:
            return 0
        if path != self._file:
            self._file, self._pos, self._header = path, 0, None
            if self._writer:
                self._writer.close()
            self._writer = EventWriter(os.path.join(os.path.dirname(path), "tb"))
        n = 0
        with open(path) as f:
            f.seek(self._pos)
            for line in f:
                if not line.endswith("\n"):
                    break
                self._pos += len(line)
                cols = line.rstrip("\n").split("\t")
                if self._header is None:
                    self._header = cols
                    continue
                row = dict(zip(self._header, cols))
                try:
                    step = int(float(row.get(self.step_tag, "0")))
                except ValueError:
                    step = 0
                for t in self.tags:
                    if t in row:
                        try:
                            self._writer.add_scalar(t, float(row[t]), step)
                            n += 1
                        except ValueError:
                            pass
        if self._writer:
            self._writer.flush()
        return n

    def _run(self):
        while not self._stop.is_set():
            try:
                self.poll_once()
            except Exception as e:
                print(f"[ProgressTensorboard] {e!r}", flush=True)
            self._stop.wait(self.poll_s)

    def start(self):
        self._thread = threading.Thread(target=self._run, daemon=True, name="rrl-tensorboard")
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
        self.poll_once()
        if self._writer:
            self._writer.close()
