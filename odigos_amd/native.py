"""ctypes view of the C ABI (include/odigos_amd.h) and the host-layer C API.

The product path is ``libodigos_amd.so`` only: if it is missing the import
fails loudly; nothing here falls back to a CPU implementation.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libodigos_amd.so"

# ---- constants (mirror include/odigos_amd.h) ----
OSE_OK = 0
OSE_EINVAL = -22
OSE_ENOMEM = -12
OSE_ENOTSUP = -95
OSE_EDEVICE = -5
OSE_ERANGE = -34
OSE_ETIMEDOUT = -110
OSE_NONE = 0xFFFFFFFF

KIND_UNSPECIFIED, KIND_INTERNAL, KIND_SERVER, KIND_CLIENT, KIND_PRODUCER, KIND_CONSUMER = range(6)
STATUS_UNSET, STATUS_OK, STATUS_ERROR = range(3)

URL_HAS_METHOD = 0x01
URL_TGT_MASK = 0x06
URL_TGT_ABSENT = 0x00
URL_TGT_STR_EMPTY = 0x02
URL_TGT_STR = 0x04
URL_TGT_NONSTR = 0x06
URL_NAME_EQ_METHOD = 0x08
URL_PATH_MASK = 0x30
URL_PATH_NONE = 0x00
URL_PATH_RAW = 0x10
URL_PATH_TARGET = 0x20

OUT_SET_ATTR = 0x01
OUT_RENAME = 0x02

STAGE_SAMPLE = 0x1
STAGE_TEMPLATE = 0x2
STAGE_SIZE = 0x4
STAGE_APPLY_KEEP = 0x8
STAGE_TEMPLATE_REFS = 0x10
STAGE_APPLY_TEMPLATE = 0x20
XREC_BYTES = 56

GROUP_TRACE_ID = 0
GROUP_BATCH = 1

# attr_type values (include/odigos_amd.h OSE_ATTR_*)
ATTR_ABSENT, ATTR_STR, ATTR_INT, ATTR_DOUBLE, ATTR_BOOL, ATTR_OTHER = range(6)

_p = C.c_void_p


class StrRef(C.Structure):
    _fields_ = [("off", C.c_uint32), ("len", C.c_uint32)]


class Rand(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("traffic_u", C.c_double)]


COLUMN_FIELDS = [
    "arena", "trace_id", "start_ns", "end_ns", "status", "kind", "resource", "scope", "url_flags",
    "path", "route", "span_size", "name_len", "route_match", "attr_match", "res_svc", "res_svc_str", "res_url_ok", "res_attrset",
    "res_size", "scope_size", "scope_resource",
]


class Columns(C.Structure):
    _fields_ = [
        ("n_spans", C.c_uint64), ("n_resources", C.c_uint32), ("n_scopes", C.c_uint32),
        ("n_attrsets", C.c_uint32), ("attr_match_words", C.c_uint32), ("arena_bytes", C.c_uint64),
    ] + [(f, _p) for f in COLUMN_FIELDS] + [("svc_match", _p), ("n_attr_keys", C.c_uint32), ("match_planes", C.c_uint32),
                                            ("attr_type", _p), ("attr_val", _p)]


class Outputs(C.Structure):
    _fields_ = [
        ("keep", _p), ("trace_count", _p), ("trace_first_span", _p), ("trace_keep", _p),
        ("trace_level", _p), ("trace_ratio", _p),
        ("url_out", _p), ("tmpl", _p), ("tmpl_arena", _p), ("tmpl_arena_cap", C.c_uint64),
        ("tmpl_arena_used", _p),
        ("attrset_bytes", _p), ("accepted_spans", _p), ("res_bytes", _p),
        ("device_status", _p),
    ]


class EngineInfo(C.Structure):
    _fields_ = [("stages", C.c_uint32), ("max_template_name", C.c_uint32),
                ("inverse_sampling", C.c_int64), ("traffic_sampling_ratio", C.c_double),
                ("n_attr_rules", C.c_uint32), ("n_attr_keys", C.c_uint32), ("attr_host_rules", C.c_uint64)]


_lib = None


def lib() -> C.CDLL:
    """Loads libodigos_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = LIB_PATH
    variant = os.environ.get("OSE_LIB_VARIANT", "")   # A/B diagnostics (odigos_amd/build.py --variant)
    if variant:
        path = LIB_PATH.with_name(f"libodigos_amd{variant}.so")
    if not path.exists():
        raise RuntimeError(f"{path} is missing: run `python -m odigos_amd.build` (hipcc, gfx950)")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, loaded by file name from torch/lib).  Loading torch
    # first makes this library bind to that same copy instead of a second
    # /opt/rocm runtime, which would leave torch without devices.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(path))
    sig = {
        "ose_last_error": (C.c_char_p, []),
        "ose_engine_create": (C.c_int, [C.c_char_p, C.POINTER(_p)]),
        "ose_engine_destroy": (None, [_p]),
        "ose_dropped_errors": (C.c_uint64, [C.c_char_p, C.c_size_t]),
        "ose_engine_service_id": (C.c_uint32, [_p, C.c_char_p, C.c_size_t]),
        "ose_engine_get_info": (C.c_int, [_p, C.POINTER(EngineInfo)]),
        "ose_set_device": (C.c_int, [C.c_int]),
        "ose_otlp_decode": (C.c_int, [_p, _p, C.c_size_t, _p, C.POINTER(_p)]),
        "ose_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(_p)]),
        "ose_host_free": (None, [_p]),
        "ose_otlp_columns": (C.POINTER(Columns), [_p]),
        "ose_otlp_host_spans": (C.c_uint32, [_p]),
        "ose_otlp_timings": (C.c_int, [_p, C.POINTER(C.c_double)]),
        "ose_otlp_attrset": (C.c_int, [_p, C.c_uint32, C.c_char_p, C.c_size_t]),
        "ose_otlp_download": (C.c_int, [_p, C.POINTER(Columns)]),
        "ose_otlp_release": (None, [_p]),
        "ose_router_create": (C.c_int, [C.c_char_p, C.POINTER(_p)]),
        "ose_router_destroy": (None, [_p]),
        "ose_router_pipelines": (C.c_uint32, [_p]),
        "ose_router_pipeline": (C.c_char_p, [_p, C.c_uint32]),
        "ose_otlp_encode": (C.c_int, [_p, _p, C.POINTER(Outputs), C.c_uint32, C.c_uint32, _p, _p, C.POINTER(_p)]),
        "ose_otlp_out_count": (C.c_uint32, [_p]),
        "ose_otlp_out_get": (C.c_int, [_p, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(_p),
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
        "ose_otlp_out_release": (None, [_p]),
        "ose_gbt_create": (C.c_int, [_p, C.c_char_p, C.c_uint64, C.c_uint64, C.POINTER(_p)]),
        "ose_gbt_destroy": (None, [_p]),
        "ose_gbt_add": (C.c_int, [_p, C.POINTER(Columns), _p, C.c_int64, _p]),
        "ose_gbt_release": (C.c_int, [_p, C.c_int64, _p, C.POINTER(C.POINTER(Columns)), C.POINTER(C.c_uint32)]),
        "ose_gbt_stats": (C.c_int, [_p, C.POINTER(C.c_uint64)]),
        "ose_gbt_download": (C.c_int, [_p, C.POINTER(Columns)]),
        "ose_engine_attr_key": (C.c_int, [_p, C.c_uint32, C.POINTER(C.c_char_p), C.POINTER(C.c_uint32)]),
        "ose_engine_attr_host_rules": (C.c_uint32, [_p, C.POINTER(C.c_uint64), C.c_uint32]),
        "ose_otlp_pipeline_create": (C.c_int, [_p, _p, C.c_uint32, C.c_uint64, C.POINTER(_p)]),
        "ose_otlp_pipeline_consume": (C.c_int, [_p, C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(_p)]),
        "ose_otlp_pipeline_counters": (C.c_int, [_p, C.c_char_p, C.c_size_t]),
        "ose_otlp_pipeline_destroy": (None, [_p]),
        "osehost_otlp_pipeline_hold": (C.c_int, [_p, C.c_uint32]),
        "osehost_otlp_pipeline_tune": (C.c_int, [_p, C.c_uint32, C.c_uint32, C.c_uint32]),
        "ose_engine_path_counts": (C.c_uint32, [_p, C.POINTER(C.c_uint64), C.c_uint32]),
        "ose_engine_set_option": (C.c_int, [_p, C.c_char_p, C.c_int64]),
        "ose_batch_acquire": (C.c_int, [_p, C.POINTER(Columns), C.POINTER(_p)]),
        "ose_batch_columns": (C.POINTER(Columns), [_p]),
        "ose_batch_outputs": (C.POINTER(Outputs), [_p]),
        "ose_batch_release": (None, [_p]),
        "ose_process": (C.c_int, [_p, _p, C.c_uint32, C.c_uint32, C.POINTER(Rand)]),
        "ose_process_device": (C.c_int, [_p, C.POINTER(Columns), C.POINTER(Outputs), C.c_uint32, C.c_uint32,
                                         C.POINTER(Rand), _p]),
        "ose_reserve": (C.c_int, [_p, C.c_uint64, C.c_uint64]),
        "ose_device_info": (C.c_int, [C.c_char_p, C.c_size_t]),
        "ose_shard_owner": (C.c_uint32, [C.c_uint64, C.c_uint64, C.c_uint32]),
        "ose_shard_pack": (C.c_int, [_p, C.POINTER(Columns), C.c_uint32, _p, _p, _p, _p]),
        "ose_shard_unpack": (C.c_int, [_p, C.c_uint64, C.c_uint32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
        "ose_shard_decide": (C.c_int, [_p, _p, C.c_uint64, C.c_uint32, _p, _p, _p, _p]),
        "ose_shard_record_bytes": (C.c_uint32, [_p]),
        "ose_shard_scatter_keep": (C.c_int, [_p, _p, C.c_uint64, _p, _p]),
        "ose_nccl_unique_id": (C.c_int, [_p, C.c_size_t]),
        "ose_nccl_comm_init": (C.c_int, [C.POINTER(_p), C.c_int, _p, C.c_int]),
        "ose_nccl_comm_destroy": (None, [_p]),
        "ose_exchange_sample": (C.c_int, [_p, C.POINTER(Columns), C.POINTER(Outputs), _p, C.c_int, C.c_int,
                                          C.POINTER(Rand), _p, _p]),
        "ose_allreduce_counters": (C.c_int, [_p, _p, C.c_uint64, _p, _p]),
        "ose_profile_enable": (C.c_int, [_p, C.c_int]),
        "ose_profile_read": (C.c_int, [_p, C.c_char_p, C.c_size_t]),
        # host layer (odigos_amd/csrc/host.cpp)
        "osehost_last_error": (C.c_char_p, []),
        "osehost_sampling_chunks": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32)]),
        "osehost_stream_copy": (C.c_int, [_p, _p, C.c_size_t, C.c_int, _p, C.POINTER(C.c_double)]),
        "osehost_xgroup_create": (C.c_int, [C.c_int, C.POINTER(_p)]),
        "osehost_owner_last_general": (C.c_uint32, [_p]),
        "osehost_xgroup_destroy": (None, [_p]),
        "osehost_exchange_sample_local": (C.c_int, [_p, C.POINTER(Columns), C.POINTER(Outputs), _p, C.c_int,
                                                    C.POINTER(Rand), _p, C.POINTER(C.c_uint64)]),
        "osehost_allreduce_counters_local": (C.c_int, [_p, _p, C.c_uint64, _p, C.c_int, _p]),
        "osehost_processor_create": (_p, [C.c_char_p, C.c_char_p]),
        "osehost_processor_destroy": (None, [_p]),
        "osehost_processor_set": (None, [_p, C.c_uint64, C.c_uint32]),
        "osehost_consume": (C.c_int, [_p, C.c_char_p, C.POINTER(_p)]),
        "osehost_columnarize": (_p, [_p, C.c_char_p]),
        "osehost_batch_columns": (C.POINTER(Columns), [_p]),
        "osehost_batch_outputs": (C.POINTER(Outputs), [_p]),
        "osehost_apply": (C.c_int, [_p, _p, C.POINTER(_p)]),
        "osehost_bench": (C.c_int, [_p, C.c_char_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]),
        "osehost_batch_free": (None, [_p]),
        "osehost_metrics_json": (_p, [_p]),
        "osehost_roundtrip": (_p, [C.c_char_p]),
        "osehost_pb_to_json": (_p, [C.c_char_p, C.c_size_t]),
        "osehost_otlp_walk": (_p, [C.c_char_p, C.c_char_p, C.c_size_t]),
        "osehost_otlp_encode": (C.c_int, [C.c_char_p, C.c_size_t, _p, C.c_int, _p, _p, _p, C.c_uint64, _p, C.c_int,
                                          C.POINTER(_p)]),
        "osehost_router_create_signal": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(_p)]),
        "osehost_router_route": (_p, [_p, C.c_char_p]),
        "osehost_otlp_out_timings": (C.c_int, [_p, C.POINTER(C.c_double)]),
        "osehost_otlp_out_path": (C.c_int, [_p, C.POINTER(C.c_uint32)]),
        "osehost_parse_duration": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
        "osehost_resource_sizes": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_uint64), C.c_size_t]),
        "osehost_as_string": (_p, [C.c_char_p]),
        "osehost_free": (None, [_p]),
        "osehost_regex_match": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t]),
        "osehost_regex_match_host": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint64,
                                               C.POINTER(C.c_int)]),
        "osehost_span_attr_eval": (C.c_int, [C.c_char_p, C.c_char_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def exported_symbols() -> list[str]:
    """Names of every entry point declared in include/odigos_amd.h."""
    import re
    hdr = (Path(__file__).resolve().parent.parent / "include" / "odigos_amd.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(ose_\w+)\s*\(", hdr, re.M)))


def last_error() -> str:
    return (lib().ose_last_error() or b"").decode("utf-8", "replace")


def take_bytes(ptr) -> bytes:
    """Copies (and frees) a malloc'ed C string returned by the host layer."""
    if not ptr:
        raise RuntimeError((lib().osehost_last_error() or b"").decode("utf-8", "replace"))
    b = C.string_at(ptr)
    lib().osehost_free(ptr)
    return b


class OseError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ose error {code}: {msg}")
        self.code = code


def check(rc: int) -> None:
    if rc != 0:
        raise OseError(rc, last_error())
