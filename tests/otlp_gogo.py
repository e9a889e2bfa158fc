"""Test infrastructure for the output side, written
independently of the engine:

* marshal_traces: what pdata's generated marshalers (gogo-style, pdata
  v1.47 internal/data/protogen) write for an OTLP/JSON TracesData — fields
  in ascending number, proto3 defaults omitted, except that the non-nullable
  embedded messages (Resource, InstrumentationScope, Status, KeyValue.value)
  and the custom-typed ids (trace / span / parent ids, an all-zero id as
  empty) are always framed;
* apply: the processors' writes on pdata (odigossamplingprocessor
  processor.go:23-25 with the per-trace grouping, odigosurltemplateprocessor
  processor.go:230-232 and 259) given the per-span decisions;
* routing: odigosrouterconnector BuildSignalRoutingMap (routingmap.go:34-57),
  NormalizeKind (routingmap.go:62-70), GetSignalsForDataStream
  (routingmap.go:84-103) and determineRoutingPipelines (connector.go:147-172).
"""
from __future__ import annotations

import base64
import copy
import struct

from odigos_amd import host

M64 = (1 << 64) - 1


def _varint(x: int) -> bytes:
    x &= M64
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _tag(f: int, wt: int) -> bytes:
    return _varint((f << 3) | wt)


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else s.encode("utf-8", "surrogateescape")


def _len(f: int, b: bytes) -> bytes:
    return _tag(f, 2) + _varint(len(b)) + b


def _str(f: int, s) -> bytes:
    b = _b(s or "")
    return _len(f, b) if b else b""


def _uvar(f: int, v) -> bytes:
    v = int(v or 0)
    return _tag(f, 0) + _varint(v) if v else b""


def _fixed64(f: int, v) -> bytes:
    v = int(v or 0)
    return _tag(f, 1) + struct.pack("<Q", v) if v else b""


def _fixed32(f: int, v) -> bytes:
    v = int(v or 0)
    return _tag(f, 5) + struct.pack("<I", v) if v else b""


def _id(f: int, hexs) -> bytes:
    b = bytes.fromhex(hexs or "")
    if b == bytes(len(b)):
        b = b""
    return _len(f, b)


def _double(x) -> float:
    if isinstance(x, str):
        return {"NaN": float("nan"), "Infinity": float("inf"), "-Infinity": float("-inf")}.get(x, None) or float(x)
    return float(x)


def any_value(v: dict) -> bytes:
    if not v:
        return b""
    k, x = next(iter(v.items()))
    if k == "stringValue":
        return _len(1, _b(x))
    if k == "boolValue":
        return _tag(2, 0) + _varint(1 if x else 0)
    if k == "intValue":
        return _tag(3, 0) + _varint(int(x))
    if k == "doubleValue":
        return _tag(4, 1) + struct.pack("<d", _double(x))
    if k == "arrayValue":
        return _len(5, b"".join(_len(1, any_value(e)) for e in (x or {}).get("values", [])))
    if k == "kvlistValue":
        return _len(6, b"".join(_len(1, key_value(e)) for e in (x or {}).get("values", [])))
    if k == "bytesValue":
        return _len(7, base64.b64decode(x))
    raise ValueError(k)


def key_value(d: dict) -> bytes:
    return _str(1, d.get("key", "")) + _len(2, any_value(d.get("value") or {}))


def _attrs(f: int, lst) -> bytes:
    return b"".join(_len(f, key_value(d)) for d in lst or [])


def span(sp: dict) -> bytes:
    st = sp.get("status") or {}
    out = [_id(1, sp.get("traceId")), _id(2, sp.get("spanId")), _str(3, sp.get("traceState")),
           _id(4, sp.get("parentSpanId")), _str(5, sp.get("name")), _uvar(6, sp.get("kind")),
           _fixed64(7, sp.get("startTimeUnixNano")), _fixed64(8, sp.get("endTimeUnixNano")),
           _attrs(9, sp.get("attributes")), _uvar(10, sp.get("droppedAttributesCount"))]
    for ev in sp.get("events") or []:
        out.append(_len(11, _fixed64(1, ev.get("timeUnixNano")) + _str(2, ev.get("name")) +
                        _attrs(3, ev.get("attributes")) + _uvar(4, ev.get("droppedAttributesCount"))))
    out.append(_uvar(12, sp.get("droppedEventsCount")))
    for lk in sp.get("links") or []:
        out.append(_len(13, _id(1, lk.get("traceId")) + _id(2, lk.get("spanId")) + _str(3, lk.get("traceState")) +
                        _attrs(4, lk.get("attributes")) + _uvar(5, lk.get("droppedAttributesCount")) +
                        _fixed32(6, lk.get("flags"))))
    out.append(_uvar(14, sp.get("droppedLinksCount")))
    out.append(_len(15, _str(2, st.get("message")) + _uvar(3, st.get("code"))))
    out.append(_fixed32(16, sp.get("flags")))
    return b"".join(out)


def resource_spans(rs: dict) -> bytes:
    r = rs.get("resource") or {}
    out = [_len(1, _attrs(1, r.get("attributes")) + _uvar(2, r.get("droppedAttributesCount")))]
    for ss in rs.get("scopeSpans") or []:
        sc = ss.get("scope") or {}
        body = _len(1, _str(1, sc.get("name")) + _str(2, sc.get("version")) + _attrs(3, sc.get("attributes")) +
                    _uvar(4, sc.get("droppedAttributesCount")))
        body += b"".join(_len(2, span(sp)) for sp in ss.get("spans") or [])
        body += _str(3, ss.get("schemaUrl"))
        out.append(_len(2, body))
    out.append(_str(3, rs.get("schemaUrl")))
    return b"".join(out)


def marshal_traces(td: dict) -> bytes:
    return b"".join(_len(1, resource_spans(rs)) for rs in td.get("resourceSpans") or [])


# ---- the processors' writes ---------------------------------------------------

SET_ATTR, RENAME = 0x01, 0x02
KIND_CLIENT = 3


def _find(attrs, key):
    for kv in attrs or []:
        if kv["key"] == key:
            return kv
    return None


def _as_string(v: dict) -> str:
    if "stringValue" in v:
        return v["stringValue"]
    if "intValue" in v:
        return str(int(v["intValue"]))
    if "boolValue" in v:
        return "true" if v["boolValue"] else "false"
    return host.as_string(v)   # pdata AsString (host restatement, pinned in test_url_*)


def apply(td: dict, keep=None, url_out=None, tmpls=None, drop_all=False) -> dict:
    td = copy.deepcopy(td)
    i = 0
    for rs in td["resourceSpans"]:
        for ss in rs["scopeSpans"]:
            for sp in ss["spans"]:
                kept = keep is None or bool(keep[i])
                u = int(url_out[i]) if url_out is not None else 0
                if kept and u:
                    t = tmpls[i]
                    attrs = sp.setdefault("attributes", [])
                    if u & SET_ATTR:   # Map.PutStr
                        key = "url.template" if sp.get("kind", 0) == KIND_CLIENT else "http.route"
                        kv = _find(attrs, key)
                        if kv is None:
                            attrs.append({"key": key, "value": {"stringValue": t}})
                        else:
                            kv["value"] = {"stringValue": t}
                    if u & RENAME:
                        m = _find(attrs, "http.request.method")
                        if m is None:
                            m = _find(attrs, "http.method")
                        sp["name"] = (_as_string(m["value"]) if m is not None else "") + " " + t
                i += 1
    if drop_all:
        td["resourceSpans"] = []
    elif keep is not None:
        k = 0
        rout = []
        for rs in td["resourceSpans"]:
            had, sout = False, []
            for ss in rs["scopeSpans"]:
                shad = bool(ss["spans"])
                had |= shad
                kept = []
                for sp in ss["spans"]:
                    if keep[k]:
                        kept.append(sp)
                    k += 1
                ss["spans"] = kept
                if not shad or kept:
                    sout.append(ss)
            rs["scopeSpans"] = sout
            if not had or sout:
                rout.append(rs)
        td["resourceSpans"] = rout
    return td


# ---- odigosrouterconnector ----------------------------------------------------

def normalize_kind(kind: str) -> str:
    low = kind.lower()
    return low if low in ("deployment", "statefulset", "daemonset", "cronjob", "deploymentconfig") else kind


def signals_for(ds: dict) -> list:
    sigs = []
    for d in ds.get("destinations") or []:
        for s in d.get("configuredsignals") or []:
            if s not in sigs:
                sigs.append(s)
            if len(sigs) == 3:
                return sigs
    return sigs


def build_routing_map(datastreams: list) -> dict:
    m: dict = {}
    for ds in datastreams:
        sigs = signals_for(ds)
        for src in ds.get("sources") or []:
            key = "%s/%s/%s" % (src.get("namespace", ""), normalize_kind(src.get("kind", "")), src.get("name", ""))
            idx = m.setdefault(key, {})
            for s in sigs:
                lst = idx.setdefault(s, [])
                if ds.get("name", "") not in lst:
                    lst.append(ds.get("name", ""))
    return m


def _str_of(v: dict) -> str:   # pcommon.Value.Str
    return v["stringValue"] if "stringValue" in v else ""


def route(attrs: list, m: dict, signal: str):
    """(pipelines or None, key)"""
    ns = _find(attrs, "k8s.namespace.name")
    if ns is None:
        return None, ""
    name = kind = ""
    for key, k in (("k8s.deployment.name", "Deployment"), ("k8s.statefulset.name", "StatefulSet"),
                   ("k8s.daemonset.name", "DaemonSet")):
        v = _find(attrs, key)
        if v is not None:
            name, kind = _str_of(v["value"]), k
            break
    if not name or not kind:
        return None, ""
    key = "%s/%s/%s" % (_str_of(ns["value"]), normalize_kind(kind), name)
    p = m.get(key, {}).get(signal)
    if not p:
        return None, ""
    return p, key


def split_by_pipeline(td: dict, datastreams: list, pipelines: list, signal: str = "TRACES") -> list:
    """ConsumeTraces: [(pipeline, TracesData)] for `pipelines` then "default"."""
    m = build_routing_map(datastreams)
    by = {p: [] for p in pipelines}
    default = []
    for rs in td["resourceSpans"]:
        p, _ = route((rs.get("resource") or {}).get("attributes") or [], m, signal)
        if not p:
            default.append(rs)
            continue
        for name in p:
            by[name].append(rs)
    return [(p, {"resourceSpans": by[p]}) for p in pipelines] + [("default", {"resourceSpans": default})]
