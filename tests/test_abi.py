"""The C-ABI library loads without a GPU and exports every entry point that
include/odigos_amd.h declares (no compute calls here)."""
import ctypes as C
import subprocess

from odigos_amd import native


def test_header_symbols_exported():
    syms = native.exported_symbols()
    assert len(syms) >= 15, syms
    lib = C.CDLL(str(native.LIB_PATH))
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", str(native.LIB_PATH)], capture_output=True, text=True).stdout
    for s in syms:
        assert f" T {s}" in out, s


def test_engine_create_validates_before_device():
    # Validate() errors surface as OSE_EINVAL even without a GPU
    h = C.c_void_p()
    bad = b'{"odigossampling": {"global_rules": [{"name": "r", "type": "error", "rule_details": {"fallback_sampling_ratio": 150}}]}}'
    assert native.lib().ose_engine_create(bad, C.byref(h)) == native.OSE_EINVAL
    assert "between 0 and 100" in native.last_error()
    bad = b'{"odigostrafficmetrics": {"sampling_ratio": 2}}'
    assert native.lib().ose_engine_create(bad, C.byref(h)) == native.OSE_EINVAL
    bad = b'{"odigosurltemplate": {"templatization_rules": ["{foo:}"]}}'
    assert native.lib().ose_engine_create(bad, C.byref(h)) == native.OSE_EINVAL


def test_no_device_is_loud():
    import torch
    if torch.cuda.is_available():
        return
    h = C.c_void_p()
    assert native.lib().ose_engine_create(b'{"odigosurltemplate": {}}', C.byref(h)) == native.OSE_EDEVICE


def test_blob_offsets_guarded(tmp_path):
    # device-table sections past 4 GiB are refused (blob.hpp), never wrapped
    import subprocess
    from pathlib import Path
    src = Path(__file__).with_name("blob_check.cpp")
    exe = tmp_path / "blob_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(src)], check=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout
