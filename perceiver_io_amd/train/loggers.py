"""Loggers: ``TensorBoardLogger``-compatible directory layout and API without TensorBoard.

Reference: ``TensorBoardLogger(save_dir=trainer.default_root_dir, name=experiment)``
(``scripts/cli.py:40-42``) → ``<save_dir>/<name>/version_<n>/``.  Each scalar goes to
``metrics.jsonl`` (always) and to a ``events.out.tfevents.*`` file written by a minimal
self-contained TFRecord/Event encoder (TensorBoard reads it; no tensorboard package needed).
Text summaries (MLM sample predictions, ``lightning.py:255-256``) go to ``text.jsonl`` and the
event file.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Any, Dict, Optional


# ---- minimal protobuf + TFRecord encoding ------------------------------------------------
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


def _field(num: int, wire: int, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _ld(num: int, data: bytes) -> bytes:
    return _field(num, 2, _varint(len(data)) + data)


def _crc32c_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_T = _crc32c_table()


def _crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked(_crc32c(hdr))) + data + struct.pack("<I", _masked(_crc32c(data)))


def _event(step: int, summary: Optional[bytes] = None, file_version: Optional[str] = None) -> bytes:
    ev = _field(1, 1, struct.pack("<d", time.time())) + _field(2, 0, _varint(max(0, int(step))))
    if file_version is not None:
        ev += _ld(3, file_version.encode())
    if summary is not None:
        ev += _ld(5, summary)
    return ev


def _scalar_summary(tag: str, value: float) -> bytes:
    v = _ld(1, tag.encode()) + _field(2, 5, struct.pack("<f", float(value)))
    return _ld(1, v)


def _text_summary(tag: str, text: str) -> bytes:
    plugin = _ld(1, b"text")  # PluginData.plugin_name
    meta = _ld(1, plugin)  # SummaryMetadata.plugin_data
    # TensorProto: dtype=DT_STRING(7), tensor_shape {dim {size:1}}, string_val
    shape = _ld(2, _ld(2, _field(1, 0, _varint(1))))
    tensor = _field(1, 0, _varint(7)) + shape + _ld(8, text.encode())
    v = _ld(1, tag.encode()) + _ld(9, meta) + _ld(8, tensor)
    return _ld(1, v)


class EventWriter:
    def __init__(self, log_dir: str):
        os.makedirs(log_dir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0"
        self.f = open(os.path.join(log_dir, name), "ab")
        self.f.write(_record(_event(0, file_version="brain.Event:2")))
        self.f.flush()

    def scalar(self, tag, value, step):
        self.f.write(_record(_event(step, _scalar_summary(tag, value))))

    def text(self, tag, text, step):
        self.f.write(_record(_event(step, _text_summary(tag, text))))

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()


class TensorBoardLogger:
    def __init__(self, save_dir: str = "logs", name: Optional[str] = "default", version: Optional[Any] = None,
                 log_graph: bool = False, default_hp_metric: bool = True, prefix: str = "", sub_dir: Optional[str] = None,
                 **_):
        self.save_dir = os.path.abspath(save_dir or ".")
        self.name = name or ""
        self._version = version
        self._writer = None
        self._jsonl = None
        self.enabled = True

    @property
    def root_dir(self) -> str:
        return os.path.join(self.save_dir, self.name) if self.name else self.save_dir

    @property
    def version(self):
        if self._version is None:
            self._version = self._next_version()
        return self._version

    def _next_version(self) -> int:
        root = self.root_dir
        if not os.path.isdir(root):
            return 0
        vs = [int(d.split("_")[1]) for d in os.listdir(root) if d.startswith("version_") and d.split("_")[1].isdigit()]
        return max(vs) + 1 if vs else 0

    @property
    def log_dir(self) -> str:
        v = self.version
        v = v if isinstance(v, str) else f"version_{v}"
        return os.path.join(self.root_dir, v)

    @property
    def experiment(self):
        return self

    def _open(self):
        if self._writer is None:
            os.makedirs(self.log_dir, exist_ok=True)
            self._writer = EventWriter(self.log_dir)
            self._jsonl = open(os.path.join(self.log_dir, "metrics.jsonl"), "a")

    def log_metrics(self, metrics: Dict[str, float], step: int):
        self._open()
        rec = {"step": int(step), "time": time.time()}
        for k, v in metrics.items():
            v = float(v)
            rec[k] = v
            self._writer.scalar(k, v, step)
        self._jsonl.write(json.dumps(rec) + "\n")
        self._jsonl.flush()
        self._writer.flush()

    def add_scalar(self, tag, value, step):
        self.log_metrics({tag: value}, step)

    def add_text(self, tag: str, text: str, step: int):
        self._open()
        self._writer.text(tag, text, step)
        with open(os.path.join(self.log_dir, "text.jsonl"), "a") as f:
            f.write(json.dumps({"step": int(step), "tag": tag, "text": text}) + "\n")
        self._writer.flush()

    def log_hyperparams(self, params: Dict[str, Any]):
        self._open()
        import yaml

        with open(os.path.join(self.log_dir, "hparams.yaml"), "w") as f:
            yaml.safe_dump(json.loads(json.dumps(params, default=str)), f)

    def finalize(self, status: str = "success"):
        if self._writer is not None:
            self._writer.flush()
            self._jsonl.flush()

    def close(self):
        if self._writer is not None:
            self._writer.close()
            self._jsonl.close()
            self._writer = None


class CSVLogger(TensorBoardLogger):
    """Same layout; scalars only to metrics.jsonl (no event file)."""

    def _open(self):
        if self._jsonl is None:
            os.makedirs(self.log_dir, exist_ok=True)
            self._jsonl = open(os.path.join(self.log_dir, "metrics.jsonl"), "a")

            class _Null:
                def scalar(self, *a): pass
                def text(self, *a): pass
                def flush(self): pass
                def close(self): pass

            self._writer = _Null()
