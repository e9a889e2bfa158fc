"""Python handle on the C++ host processors (odigos_amd/csrc/host.cpp).

``Processor(type, cfg)`` mirrors ``NewFactory().CreateTraces(...)`` of the
reference's ``odigossampling`` / ``odigosurltemplate`` /
``odigostrafficmetrics`` (plus ``pipeline``: all three in gateway order), and
``consume`` mirrors ``ProcessTracesFunc`` on OTLP/JSON traces.
"""
from __future__ import annotations

import ctypes as C
import json
from typing import Any

from . import native

PROCESSOR_TYPES = ("odigossampling", "odigosurltemplate", "odigostrafficmetrics", "pipeline")


def _enc_str(s) -> str:
    """JSON string literal; `bytes` values are emitted with the host parser's
    \\xHH extension so invalid UTF-8 reaches the processors unchanged."""
    if isinstance(s, bytes):
        out = ['"']
        for b in s:
            ch = chr(b)
            if b >= 0x80 or b < 0x20:
                out.append("\\x%02x" % b)
            elif ch in '"\\':
                out.append("\\" + ch)
            else:
                out.append(ch)
        out.append('"')
        return "".join(out)
    return json.dumps(s)


def dumps(obj: Any) -> str:
    if isinstance(obj, dict):
        return "{" + ",".join(_enc_str(k) + ":" + dumps(v) for k, v in obj.items()) + "}"
    if isinstance(obj, (list, tuple)):
        return "[" + ",".join(dumps(v) for v in obj) + "]"
    if isinstance(obj, (str, bytes)):
        return _enc_str(obj)
    return json.dumps(obj)


def _fix(obj):
    """Host-layer output strings carry raw bytes as U+0000..U+00FF: map them
    back to Python str (utf-8, invalid bytes as surrogate escapes)."""
    if isinstance(obj, dict):
        return {_fix(k): _fix(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_fix(v) for v in obj]
    if isinstance(obj, str):
        return obj.encode("latin-1").decode("utf-8", "surrogateescape")
    return obj


def loads(s: str):
    return _fix(json.loads(s))


def attr_value(v) -> dict:
    if isinstance(v, bool):
        return {"boolValue": v}
    if isinstance(v, int):
        return {"intValue": str(v)}
    if isinstance(v, float):
        if v != v or v in (float("inf"), float("-inf")):   # protobuf JSON mapping of non-finite doubles
            return {"doubleValue": "NaN" if v != v else ("Infinity" if v > 0 else "-Infinity")}
        return {"doubleValue": v}
    if isinstance(v, dict) and len(v) == 1 and next(iter(v)).endswith("Value"):
        return v
    return {"stringValue": v}


def attrs(d: dict) -> list:
    return [{"key": k, "value": attr_value(v)} for k, v in d.items()]


def span(name="span", kind=0, attributes=None, trace_id="", span_id="", start=0, end=0, status=0, **extra) -> dict:
    s = {"traceId": trace_id, "spanId": span_id, "name": name, "kind": kind,
         "startTimeUnixNano": str(start), "endTimeUnixNano": str(end),
         "attributes": attrs(attributes or {}), "status": {"code": status} if status else {}}
    s.update(extra)
    return s


def resource_spans(resource_attrs=None, spans=(), scopes=None) -> dict:
    if scopes is None:
        scopes = [{"scope": {}, "spans": list(spans)}]
    return {"resource": {"attributes": attrs(resource_attrs or {})}, "scopeSpans": scopes}


def traces(*rs) -> dict:
    return {"resourceSpans": list(rs)}


def find_attr(span_json: dict, key: str):
    for kv in span_json.get("attributes", []):
        if kv["key"] == key:
            return kv["value"]
    return None


def as_string(value_json: dict) -> str:
    """pcommon.Value.AsString (host implementation)."""
    L = native.lib()
    return native.take_bytes(L.osehost_as_string(dumps(value_json).encode())).decode("utf-8", "surrogateescape")


class Processor:
    def __init__(self, ptype: str, cfg: dict | None = None):
        if ptype not in PROCESSOR_TYPES:
            raise ValueError(f"unknown processor type {ptype}")
        self.L = native.lib()
        self.type = ptype
        self.cfg = cfg or {}
        self.h = self.L.osehost_processor_create(ptype.encode(), dumps(self.cfg).encode())
        if not self.h:
            raise ValueError((self.L.osehost_last_error() or b"").decode("utf-8", "replace"))

    def close(self):
        if self.h:
            self.L.osehost_processor_destroy(self.h)
            self.h = None

    __del__ = close

    def configure(self, seed: int = 0x0D16A5EE, group_mode: int = native.GROUP_BATCH):
        self.L.osehost_processor_set(self.h, seed, group_mode)

    def consume(self, td: dict) -> dict:
        """ConsumeTraces on the device (HIP) path."""
        out = C.c_void_p()
        rc = self.L.osehost_consume(self.h, dumps(td).encode(), C.byref(out))
        if rc != 0:
            raise native.OseError(rc, (self.L.osehost_last_error() or b"").decode("utf-8", "replace"))
        return loads(native.take_bytes(out.value).decode("ascii"))

    # --- host half of ConsumeTraces, for checking against the CPU oracle ---
    def columnarize(self, td: dict) -> "HostBatch":
        h = self.L.osehost_columnarize(self.h, dumps(td).encode())
        if not h:
            raise ValueError((self.L.osehost_last_error() or b"").decode())
        return HostBatch(self, h)

    def metrics(self) -> dict:
        return loads(native.take_bytes(self.L.osehost_metrics_json(self.h)).decode("ascii"))


class HostBatch:
    def __init__(self, proc: Processor, h):
        self.proc, self.h, self.L = proc, h, proc.L
        self.cols = self.L.osehost_batch_columns(h).contents
        self.outs = self.L.osehost_batch_outputs(h).contents

    def apply(self) -> dict:
        out = C.c_void_p()
        self.L.osehost_apply(self.proc.h, self.h, C.byref(out))
        return loads(native.take_bytes(out.value).decode("ascii"))

    def __del__(self):
        if self.h:
            self.L.osehost_batch_free(self.h)
            self.h = None
