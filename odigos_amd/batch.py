"""Device-resident columnar batches for ``ose_process_device``.

PyTorch is used only as the HBM allocator / stream / copy engine: every
column is a flat ``torch.uint8`` tensor whose data pointer is handed to the
C ABI.  Also wraps the seeded synthetic generator (libosegen.so).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from . import native

# element size and the dimension each column is indexed by
COLUMN_LAYOUT = {
    "arena": ("arena", 1),
    "trace_id": ("span", 16), "start_ns": ("span", 8), "end_ns": ("span", 8), "status": ("span", 1),
    "kind": ("span", 1), "resource": ("span", 4), "scope": ("span", 4), "url_flags": ("span", 1),
    "path": ("span", 8), "route": ("span", 8), "span_size": ("span", 4), "name_len": ("span", 4),
    "route_match": ("span", 8), "attr_match": ("span_words", 8),
    "res_svc": ("res", 4), "res_svc_str": ("res", 4), "res_url_ok": ("res", 1), "res_attrset": ("res", 4),
    "res_size": ("res", 4), "scope_size": ("scope", 4), "scope_resource": ("scope", 4),
    "attr_type": ("span_key", 1), "attr_val": ("span_key", 8),
}
OUTPUT_LAYOUT = {
    "keep": ("span", 1), "trace_count": ("one", 4), "trace_first_span": ("span", 4), "trace_keep": ("span", 1),
    "trace_level": ("span", 1), "trace_ratio": ("span", 8), "url_out": ("span", 1), "tmpl": ("span", 8),
    "attrset_bytes": ("attrset", 8), "accepted_spans": ("one", 8), "res_bytes": ("res", 8),
    "device_status": ("one", 16),
}


def _count(cols, dim: str) -> int:
    return {"span": cols.n_spans, "res": cols.n_resources, "scope": cols.n_scopes, "arena": cols.arena_bytes,
            "attrset": cols.n_attrsets, "one": 1, "span_key": cols.n_spans * cols.n_attr_keys,
            "span_words": cols.n_spans * max(1, cols.attr_match_words)}[dim]


def default_tmpl_cap(cols) -> int:
    """Output arena capacity: every template fits in 2x the input bytes plus
    16 per span, capped at the 32-bit offset range of ose_strref."""
    return min(int(2 * cols.arena_bytes + 16 * cols.n_spans + 4096), 0xFFFFFFF0)


def host_array(ptr: int, nbytes: int) -> np.ndarray:
    if nbytes == 0 or not ptr:
        return np.zeros(0, dtype=np.uint8)
    return np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(ptr))


class Generator:
    """Seeded synthetic batch (odigos_amd/csrc/gen_batch.cpp)."""
    LIB = Path(__file__).resolve().parent / "_lib" / "libosegen.so"
    _L = None

    def __init__(self, workload: str, seed: int, n_spans: int, threads: int = 8, shuffle: bool = False,
                 rank: int | None = None, world: int | None = None):
        """world given: split mode, the batch node-collector source `rank` of
        `world` holds of a global batch of n_spans spans (gen_batch.cpp)."""
        if Generator._L is None:
            L = C.CDLL(str(self.LIB))
            L.osegen_create.restype = C.c_void_p
            L.osegen_create.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
            L.osegen_create_split.restype = C.c_void_p
            L.osegen_create_split.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint32, C.c_uint32]
            L.osegen_columns.restype = C.POINTER(native.Columns)
            L.osegen_columns.argtypes = [C.c_void_p]
            L.osegen_free.argtypes = [C.c_void_p]
            L.osegen_otlp.restype = C.c_void_p
            L.osegen_otlp.argtypes = [C.POINTER(native.Columns), C.c_int, C.POINTER(C.c_uint64)]
            L.osegen_otlp_free.argtypes = [C.c_void_p]
            Generator._L = L
        if world is None:
            self.h = Generator._L.osegen_create(workload.encode(), seed, n_spans, threads, int(shuffle))
        else:
            assert not shuffle and 0 <= (rank or 0) < world
            self.h = Generator._L.osegen_create_split(workload.encode(), seed, n_spans, threads, rank or 0, world)
        if not self.h:
            raise ValueError("osegen: bad arguments")
        self.cols = Generator._L.osegen_columns(self.h).contents
        self.workload = workload

    def array(self, field: str) -> np.ndarray:
        dim, size = COLUMN_LAYOUT[field]
        n = _count(self.cols, dim) * size
        if field == "arena":
            n = (n + 15) // 16 * 16 + 16
        return host_array(getattr(self.cols, field), n)

    def otlp(self, threads: int = 8) -> bytes:
        """The batch as a serialized OTLP TracesData (gen_otlp.cpp)."""
        n = C.c_uint64()
        p = Generator._L.osegen_otlp(C.byref(self.cols), threads, C.byref(n))
        try:   # (string_at takes an int size: messages above 2 GiB need the array view)
            return C.cast(p, C.POINTER(C.c_char * n.value)).contents.raw
        finally:
            Generator._L.osegen_otlp_free(p)

    def __del__(self):
        if getattr(self, "h", None):
            Generator._L.osegen_free(self.h)
            self.h = None


class HostOutputs:
    """Host output buffers (numpy) for the oracle."""

    def __init__(self, cols: native.Columns, tmpl_cap: int | None = None):
        self.bufs = {}
        self.outs = native.Outputs()
        for name, (dim, size) in OUTPUT_LAYOUT.items():
            a = np.zeros(max(_count(cols, dim) * size, 16), dtype=np.uint8)
            self.bufs[name] = a
            setattr(self.outs, name, a.ctypes.data)
        cap = tmpl_cap if tmpl_cap is not None else default_tmpl_cap(cols)
        self.bufs["tmpl_arena"] = np.zeros(cap + 16, dtype=np.uint8)
        self.outs.tmpl_arena = self.bufs["tmpl_arena"].ctypes.data
        self.outs.tmpl_arena_cap = cap
        self.used = np.zeros(1, dtype=np.uint64)
        self.outs.tmpl_arena_used = self.used.ctypes.data

    def view(self, name, dtype):
        return self.bufs[name].view(dtype)


def device_outputs(dims: native.Columns, device="cuda", tmpl_cap: int | None = None):
    """ose_outputs for a batch of these dimensions, in HBM (torch tensors)."""
    import torch
    outs = native.Outputs()
    o = {}
    for name, (dim, size) in OUTPUT_LAYOUT.items():
        n = max(_count(dims, dim) * size, 16)
        t = torch.zeros(n + 16, dtype=torch.uint8, device=device)
        o[name] = t
        setattr(outs, name, t.data_ptr())
    cap = tmpl_cap if tmpl_cap is not None else default_tmpl_cap(dims)
    o["tmpl_arena"] = torch.zeros(cap + 16, dtype=torch.uint8, device=device)
    outs.tmpl_arena = o["tmpl_arena"].data_ptr()
    outs.tmpl_arena_cap = cap
    o["used"] = torch.zeros(2, dtype=torch.int64, device=device)
    outs.tmpl_arena_used = o["used"].data_ptr()
    return outs, o


class DeviceBatch:
    """Columns + outputs resident in HBM (torch uint8 tensors)."""

    def __init__(self, host_cols: native.Columns, device="cuda", tmpl_cap: int | None = None, fields=None):
        import torch
        self.torch = torch
        self.cols = native.Columns()
        for f in ("n_spans", "n_resources", "n_scopes", "n_attrsets", "arena_bytes", "n_attr_keys", "attr_match_words"):
            setattr(self.cols, f, getattr(host_cols, f))
        self.t = {}
        for name, (dim, size) in COLUMN_LAYOUT.items():
            if (fields is not None and name not in fields) or not getattr(host_cols, name):
                continue
            n = _count(host_cols, dim) * size
            if name == "arena":
                n = (n + 15) // 16 * 16 + 16
            src = host_array(getattr(host_cols, name), n)
            t = torch.zeros(max(n, 16) + 16, dtype=torch.uint8, device=device)
            if n:
                t[:n].copy_(torch.from_numpy(src))
            self.t[name] = t
            setattr(self.cols, name, t.data_ptr())
        self.outs, self.o = device_outputs(host_cols, device, tmpl_cap)

    def out_numpy(self, name: str, dtype=np.uint8, n: int | None = None) -> np.ndarray:
        """Host copy of an output (the first n elements of dtype, or all)."""
        t = self.o[name]
        if n is not None:
            t = t[: n * np.dtype(dtype).itemsize]
        return t.cpu().numpy().view(dtype)

    def used(self) -> int:
        return int(self.o["used"][0].item())


_ENGINES = None


def _close_engines():
    """atexit: engines (and the batches / stores they own) are released while
    the HIP runtime is still up, not by finalizers during interpreter
    teardown."""
    for e in list(_ENGINES or ()):
        e.close()


class Engine:
    """ose_engine handle (product path: raises if the HIP library cannot run)."""

    def __init__(self, cfg: dict):
        from .host import dumps
        self.L = native.lib()
        h = C.c_void_p()
        native.check(self.L.ose_engine_create(dumps(cfg).encode(), C.byref(h)))
        self.h = h
        # objects that must be released before the engine (the ABI's rule):
        # a garbage cycle may finalize the engine first, so it closes them
        import weakref
        self._children = weakref.WeakSet()
        global _ENGINES
        if _ENGINES is None:
            import atexit
            _ENGINES = weakref.WeakSet()
            atexit.register(_close_engines)
        _ENGINES.add(self)

    def adopt(self, obj):
        self._children.add(obj)

    def info(self) -> native.EngineInfo:
        i = native.EngineInfo()
        native.check(self.L.ose_engine_get_info(self.h, C.byref(i)))
        return i

    def service_id(self, name: str) -> int:
        b = name.encode()
        return self.L.ose_engine_service_id(self.h, b, len(b))

    def reserve(self, n_spans: int, arena_bytes: int = 0):
        native.check(self.L.ose_reserve(self.h, n_spans, arena_bytes))

    def process_device(self, db: DeviceBatch, stages: int, group_mode: int = native.GROUP_TRACE_ID,
                       seed: int = 0, traffic_u: float = 0.0, stream=None):
        rnd = native.Rand(seed, traffic_u)
        s = None if stream is None else C.c_void_p(stream)
        native.check(self.L.ose_process_device(self.h, C.byref(db.cols), C.byref(db.outs), stages, group_mode,
                                               C.byref(rnd), s))

    def profile(self, on: bool = True):
        native.check(self.L.ose_profile_enable(self.h, int(on)))

    def set_option(self, name: str, value: int = 1):
        """ose_engine_set_option: the alternative OTLP legs (tests)."""
        native.check(self.L.ose_engine_set_option(self.h, name.encode(), int(value)))

    def path_counts(self) -> dict:
        """ose_engine_path_counts: how often SAMPLE left its fast path."""
        c = (C.c_uint64 * 3)()
        self.L.ose_engine_path_counts(self.h, c, 3)
        return {"run_list": int(c[0]), "sort": int(c[1]), "long_runs": int(c[2])}

    def profile_read(self) -> dict:
        import json
        buf = C.create_string_buffer(1 << 16)
        native.check(self.L.ose_profile_read(self.h, buf, len(buf)))
        return json.loads(buf.value.decode())

    def close(self):
        if getattr(self, "h", None):
            for c in list(getattr(self, "_children", ())):
                c.close()
            self.L.ose_engine_destroy(self.h)
            self.h = None

    __del__ = close


class PinnedBatch:
    """An engine-owned pinned host batch (ose_batch_acquire) for the
    synchronous drop-in call ose_process: H2D of the columns, the stages,
    D2H of the results — what the cgo shim calls per ConsumeTraces."""

    def __init__(self, engine: "Engine", dims: native.Columns):
        self.L = engine.L
        self.eng = engine
        h = C.c_void_p()
        native.check(self.L.ose_batch_acquire(engine.h, C.byref(dims), C.byref(h)))
        self.h = h
        engine.adopt(self)
        self.cols = self.L.ose_batch_columns(h).contents
        self.outs = self.L.ose_batch_outputs(h).contents

    def fill(self, src: native.Columns):
        """Copies a host batch of the acquired dimensions into the pinned
        columns (the shim's fillColumns step); columns the source lacks are
        NULLed, which tells ose_process they are absent."""
        for f, (dim, size) in COLUMN_LAYOUT.items():
            if dim in ("attrset", "one"):
                continue
            dst, srcp = getattr(self.cols, f, None), getattr(src, f, None)
            if dst and srcp:
                C.memmove(dst, srcp, _count(src, dim) * size)
            elif dst:
                setattr(self.cols, f, None)

    def process(self, stages: int, group_mode: int = native.GROUP_TRACE_ID, seed: int = 0, traffic_u: float = 0.0):
        rnd = native.Rand(seed, traffic_u)
        native.check(self.L.ose_process(self.eng.h, self.h, stages, group_mode, C.byref(rnd)))

    def close(self):
        if getattr(self, "h", None):
            self.L.ose_batch_release(self.h)
            self.h = None

    __del__ = close


def take_otlp_out(L, h, copy: bool = True, timings: list | None = None, path: dict | None = None) -> list:
    """The outputs of an ose_otlp_out (then released); copy=False gives the
    byte counts instead of the bytes; `timings` receives the encoder's phase
    times (ms: decisions D2H, sizing pass, buffers, writing pass); `path`
    whether the GPU encoder wrote them ("gpu") and why it handed the call to
    the host encoder ("fallback", kEncFb* bits)."""
    try:
        if timings is not None:
            t = (C.c_double * 4)()
            native.check(L.osehost_otlp_out_timings(h, t))
            timings[:] = list(t)
        if path is not None:
            fb = C.c_uint32()
            path["gpu"] = bool(L.osehost_otlp_out_path(h, C.byref(fb)))
            path["fallback"] = fb.value
        res = []
        for k in range(L.ose_otlp_out_count(h)):
            name, data, n, nres = C.c_char_p(), C.c_void_p(), C.c_uint64(), C.c_uint32()
            native.check(L.ose_otlp_out_get(h, k, C.byref(name), C.byref(data), C.byref(n), C.byref(nres)))
            if copy:
                raw = (C.c_char * n.value).from_address(data.value).raw if n.value else b""
            else:
                raw = n.value
            res.append((name.value.decode("utf-8", "surrogateescape"), raw, nres.value))
        return res
    finally:
        L.ose_otlp_out_release(h)


class Router:
    """odigosrouterconnector's routing table (ose_router_create); `signal`
    other than TRACES builds it through the test seam (routing KATs)."""

    def __init__(self, cfg, signal: str | None = None):
        import json
        self.L = native.lib()
        text = cfg if isinstance(cfg, str) else json.dumps(cfg)
        h = C.c_void_p()
        if signal is None:
            native.check(self.L.ose_router_create(text.encode(), C.byref(h)))
        else:
            native.check(self.L.osehost_router_create_signal(text.encode(), signal.encode(), C.byref(h)))
        self.h = h
        self.pipelines = [self.L.ose_router_pipeline(h, k).decode() for k in range(self.L.ose_router_pipelines(h))]

    def route(self, attrs: dict) -> tuple:
        """determineRoutingPipelines on {"key": value}: (pipelines, key)."""
        import json
        out = json.loads(native.take_bytes(self.L.osehost_router_route(self.h, json.dumps(attrs).encode())))
        return out["pipelines"], out["key"]

    def close(self):
        if getattr(self, "h", None):
            self.L.ose_router_destroy(self.h)
            self.h = None

    __del__ = close


class GroupByTrace:
    """The GPU-resident groupbytrace store (ose_gbt_*): add device batches
    with the caller's clock, release the traces whose wait is over as one
    device batch (DeviceView) for Engine.process_device."""

    STATS = ("waiting_traces", "held_spans", "created", "released", "evicted", "released_spans", "added_spans",
             "held_bytes")

    def __init__(self, engine: "Engine", cfg: dict, span_capacity: int, arena_capacity: int):
        import json
        self.L = engine.L
        self.eng = engine
        h = C.c_void_p()
        native.check(self.L.ose_gbt_create(engine.h, json.dumps(cfg).encode(), span_capacity, arena_capacity,
                                           C.byref(h)))
        self.h = h
        engine.adopt(self)

    def add(self, cols: native.Columns, now_ns: int, attrset_map=None, stream=None):
        m = None
        if attrset_map is not None:
            m = np.ascontiguousarray(attrset_map, dtype=np.uint32)
        s = None if stream is None else C.c_void_p(stream)
        native.check(self.L.ose_gbt_add(self.h, C.byref(cols), None if m is None else m.ctypes.data, now_ns, s))

    def release(self, now_ns: int, stream=None):
        """(columns of the released batch (device pointers), traces released)"""
        out = C.POINTER(native.Columns)()
        nt = C.c_uint32()
        s = None if stream is None else C.c_void_p(stream)
        native.check(self.L.ose_gbt_release(self.h, now_ns, s, C.byref(out), C.byref(nt)))
        return native.Columns.from_buffer_copy(out.contents), nt.value

    def stats(self) -> dict:
        v = (C.c_uint64 * 8)()
        native.check(self.L.ose_gbt_stats(self.h, v))
        return dict(zip(self.STATS, list(v)))

    def download(self, cols: native.Columns) -> dict:
        """Host copies (numpy) of the last release's columns."""
        dst = native.Columns()
        for f in ("n_spans", "n_resources", "n_scopes", "n_attrsets", "arena_bytes", "n_attr_keys", "attr_match_words"):
            setattr(dst, f, getattr(cols, f))
        out = {}
        for name, (dim, size) in COLUMN_LAYOUT.items():
            if not getattr(cols, name):
                continue
            nb = _count(cols, dim) * size
            a = np.zeros(max(nb, 1) + 16, dtype=np.uint8)
            out[name] = a
            setattr(dst, name, a.ctypes.data)
        native.check(self.L.ose_gbt_download(self.h, C.byref(dst)))
        return out

    def close(self):
        if getattr(self, "h", None):
            self.L.ose_gbt_destroy(self.h)
            self.h = None

    __del__ = close


class DeviceView:
    """Device columns owned elsewhere (an OTLP batch, a groupbytrace release)
    plus HBM outputs: what Engine.process_device takes."""

    def __init__(self, cols: native.Columns, tmpl_cap: int | None = None):
        self.cols = cols
        self.outs, self.o = device_outputs(cols, tmpl_cap=tmpl_cap)

    def out_numpy(self, name: str, dtype=np.uint8, n: int | None = None) -> np.ndarray:
        t = self.o[name]
        if n is not None:
            t = t[: n * np.dtype(dtype).itemsize]
        return t.cpu().numpy().view(dtype)


class OtlpBatch:
    """A serialized TracesData decoded on the GPU (ose_otlp_decode): device
    columns owned by the engine plus HBM outputs, usable wherever a
    DeviceBatch is (Engine.process_device)."""

    def __init__(self, engine: "Engine", pb, stream=None, tmpl_cap: int | None = None, length: int | None = None,
                 outputs=None):
        """pb: the message bytes, or the address of a buffer (e.g. PinnedBuffer) with `length`;
        outputs: an (outs, tensors) pair from device_outputs to reuse."""
        self.L = engine.L
        self.eng = engine   # the engine must outlive its batches (ose_otlp_release before ose_engine_destroy)
        h = C.c_void_p()
        s = None if stream is None else C.c_void_p(stream)
        if isinstance(pb, (bytes, bytearray)):
            self._msg = bytes(pb) if isinstance(pb, bytearray) else pb   # read again by encode()
            buf = C.c_char_p(self._msg)
            addr, n = C.cast(buf, C.c_void_p), len(pb)
        else:
            addr, n = C.c_void_p(int(pb)), int(length)
        native.check(self.L.ose_otlp_decode(engine.h, addr, n, s, C.byref(h)))
        self.h = h
        engine.adopt(self)
        self.cols = native.Columns.from_buffer_copy(self.L.ose_otlp_columns(h).contents)
        self.host_spans = int(self.L.ose_otlp_host_spans(h))
        t = (C.c_double * 5)()
        native.check(self.L.ose_otlp_timings(h, t))
        self.timings_ms = dict(zip(("bytes_in", "walk", "columns", "span_kernel", "host_pass"), list(t)))
        self.outs, self.o = outputs if outputs is not None else device_outputs(self.cols, tmpl_cap=tmpl_cap)

    def attrset(self, k: int) -> dict:
        import json
        buf = C.create_string_buffer(1 << 16)
        native.check(self.L.ose_otlp_attrset(self.h, k, buf, len(buf)))
        return json.loads(buf.value.decode("utf-8", "surrogateescape"))

    def download(self) -> dict:
        """Host copies of every column (numpy), dims and the arena."""
        c = self.cols
        dst = native.Columns()
        for f in ("n_spans", "n_resources", "n_scopes", "n_attrsets", "arena_bytes", "n_attr_keys", "attr_match_words"):
            setattr(dst, f, getattr(c, f))
        out = {}
        for name, (dim, size) in COLUMN_LAYOUT.items():
            if not getattr(c, name):
                continue
            nb = _count(c, dim) * size
            a = np.zeros(max(nb, 1) + 16, dtype=np.uint8)
            out[name] = a
            setattr(dst, name, a.ctypes.data)
        native.check(self.L.ose_otlp_download(self.h, C.byref(dst)))
        return out

    def out_numpy(self, name: str, dtype=np.uint8, n: int | None = None) -> np.ndarray:
        t = self.o[name]
        if n is not None:
            t = t[: n * np.dtype(dtype).itemsize]
        return t.cpu().numpy().view(dtype)

    def used(self) -> int:
        return int(self.o["used"][0].item())

    def encode(self, stages: int, group_mode: int = native.GROUP_TRACE_ID, router: "Router | None" = None,
               stream=None, copy: bool = True) -> list:
        """ose_otlp_encode after Engine.process_device(self, stages, group_mode):
        [(pipeline, TracesData bytes, n_resources)] — the router's pipelines
        then "default", or one ("", bytes, n) without a router."""
        h = C.c_void_p()
        s = None if stream is None else C.c_void_p(stream)
        native.check(self.L.ose_otlp_encode(self.eng.h, self.h, C.byref(self.outs), stages, group_mode,
                                            router.h if router is not None else None, s, C.byref(h)))
        self.encode_ms = []
        self.encode_path = {}
        return take_otlp_out(self.L, h, copy, self.encode_ms, self.encode_path)

    def close(self):
        if getattr(self, "h", None):
            self.L.ose_otlp_release(self.h)
            self.h = None

    __del__ = close


class OtlpPipeline:
    """ose_otlp_pipeline: an OTLP receiver's concurrent requests (serialized
    TracesData) coalesced into one device batch per wave of calls; consume()
    is called from any number of threads and returns the request's outputs
    as OtlpBatch.encode does."""

    def __init__(self, eng: "Engine", router: "Router | None" = None,
                 stages: int = native.STAGE_SAMPLE | native.STAGE_TEMPLATE | native.STAGE_SIZE,
                 max_batch_bytes: int = 0):
        self.L = native.lib()
        self.eng, self.router = eng, router   # both outlive the pipeline
        h = C.c_void_p()
        native.check(self.L.ose_otlp_pipeline_create(eng.h, router.h if router is not None else None, stages,
                                                     max_batch_bytes, C.byref(h)))
        self.h = h

    def consume(self, data, length: int | None = None, seed: int = 0x5EED, traffic_u: float = 0.0,
                copy: bool = True, path: dict | None = None) -> list:
        """data: bytes, or the address of `length` bytes (pinned or not)."""
        rnd = native.Rand(seed, traffic_u)
        if isinstance(data, (bytes, bytearray)):
            buf = C.create_string_buffer(bytes(data), len(data))
            ptr, n = C.cast(buf, C.c_void_p), len(data)
        else:
            ptr, n = C.c_void_p(data), int(length)
        h = C.c_void_p()
        native.check(self.L.ose_otlp_pipeline_consume(self.h, ptr, n, C.byref(rnd), C.byref(h)))
        return take_otlp_out(self.L, h, copy, None, path)

    def counters(self) -> dict:
        """the traffic counters and batching statistics since the last read"""
        import json
        buf = C.create_string_buffer(1 << 20)
        native.check(self.L.ose_otlp_pipeline_counters(self.h, buf, len(buf)))
        return json.loads(buf.value.decode())

    def hold(self, n: int):
        """test seam: batches run only once n requests joined them"""
        native.check(self.L.osehost_otlp_pipeline_hold(self.h, n))

    def tune(self, max_running: int, window_us: int = 200, target: int = 16):
        """diagnostics: batches on the GPU at once, the batching window"""
        native.check(self.L.osehost_otlp_pipeline_tune(self.h, max_running, window_us, target))

    def close(self):
        if getattr(self, "h", None):
            self.L.ose_otlp_pipeline_destroy(self.h)
            self.h = None

    __del__ = close


class PinnedBuffer:
    """Pinned host memory from the engine library (ose_host_alloc)."""

    def __init__(self, data: bytes):
        self.L = native.lib()
        p = C.c_void_p()
        native.check(self.L.ose_host_alloc(len(data), C.byref(p)))
        self.p, self.n = p.value, len(data)
        C.memmove(self.p, data, len(data))

    def close(self):
        if getattr(self, "p", None):
            self.L.ose_host_free(C.c_void_p(self.p))
            self.p = None

    __del__ = close
