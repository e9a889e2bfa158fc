"""ctypes binding of oracle/liboracle.so — the CPU restatement used as the
checker (test infrastructure; the product never loads it)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

from odigos_amd import native

ORACLE_PATH = Path(__file__).resolve().parent.parent / "oracle" / "liboracle.so"
_p = C.c_void_p
_L = None


def lib():
    global _L
    if _L is None:
        L = C.CDLL(str(ORACLE_PATH))
        sig = {
            "orc_re_compile": (_p, [C.c_char_p, C.c_char_p, C.c_size_t]),
            "orc_re_match": (C.c_int, [_p, C.c_char_p, C.c_size_t]),
            "orc_re_free": (None, [_p]),
            "orc_url_create": (_p, [C.POINTER(C.c_char_p), C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                    C.c_int, C.c_char_p, C.c_size_t]),
            "orc_url_free": (None, [_p]),
            "orc_url_segment_name": (C.c_int, [_p, C.c_char_p, C.c_size_t, C.c_char_p]),
            "orc_url_apply_path": (C.c_long, [_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
            "orc_url_process": (C.c_int, [_p, C.POINTER(native.Columns), C.POINTER(native.Outputs), C.c_int]),
        }
        for name, (res, args) in sig.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                continue
            fn.restype = res
            fn.argtypes = args
        _L = L
    return _L


def _arr(strs):
    a = (C.c_char_p * max(len(strs), 1))()
    for i, s in enumerate(strs):
        a[i] = s if isinstance(s, bytes) else s.encode()
    return a


class Regex:
    def __init__(self, pattern: str):
        err = C.create_string_buffer(256)
        self.h = lib().orc_re_compile(pattern.encode(), err, 256)
        if not self.h:
            raise ValueError(err.value.decode())

    def match(self, s) -> bool:
        b = s if isinstance(s, bytes) else s.encode("utf-8", "surrogateescape")
        return bool(lib().orc_re_match(self.h, b, len(b)))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_re_free(self.h)


class UrlOracle:
    """newUrlTemplateProcessor + processTraces restated (oracle/url.c)."""

    def __init__(self, cfg: dict | None = None):
        cfg = cfg or {}
        rules = cfg.get("templatization_rules", []) or []
        cids = cfg.get("custom_ids", []) or []
        err = C.create_string_buffer(512)
        self._keep = (_arr(rules), _arr([c.get("regexp", "") for c in cids]),
                      _arr([c.get("template_name", "") or "" for c in cids]))
        self.h = lib().orc_url_create(self._keep[0], len(rules), self._keep[1], self._keep[2], len(cids), err, 512)
        if not self.h:
            raise ValueError(err.value.decode())

    def segment_name(self, seg) -> str | None:
        b = seg if isinstance(seg, bytes) else seg.encode("utf-8", "surrogateescape")
        out = C.create_string_buffer(256)
        n = lib().orc_url_segment_name(self.h, b, len(b), out)
        return None if n < 0 else out.raw[:n].decode()

    def apply_path(self, path) -> bytes:
        b = path if isinstance(path, bytes) else path.encode("utf-8", "surrogateescape")
        cap = 64 + len(b) * 64
        out = C.create_string_buffer(cap)
        n = lib().orc_url_apply_path(self.h, b, len(b), out, cap)
        assert n >= 0
        return out.raw[:n]

    def process(self, cols, outs, nthreads: int = 1) -> int:
        return lib().orc_url_process(self.h, C.byref(cols), C.byref(outs), nthreads)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_url_free(self.h)
