"""In-tree build of the native libraries.

* ``odigos_amd/_lib/libodigos_amd.so`` — the product: HIP kernels for gfx950,
  the C ABI (include/odigos_amd.h) and the C++ host processors, built with
  hipcc.  It is the only thing the processors call.
* ``oracle/liboracle.so`` — the CPU restatement used by tests/, smoke() and
  bench.py's cpu_baseline leg (test infrastructure, never linked by the
  product).
* ``odigos_amd/_lib/libosegen.so`` — the seeded synthetic batch generator
  (bench/test infrastructure).

Objects go to ``build/`` (git-ignored); the .so files stay in-tree so gpurun
ships them to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "odigos_amd" / "csrc"
LIBDIR = ROOT / "odigos_amd" / "_lib"
OBJDIR = ROOT / "build"
ORACLE = ROOT / "oracle"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
HIP_FLAGS = ["-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]
# the CPU restatement must run on the GPU box's host CPU too: no -march=native
C_FLAGS = ["-O3", "-fPIC", "-march=x86-64-v2", "-Wall", "-Wextra", "-Wno-unused-parameter", "-pthread"]

PRODUCT_SOURCES = sorted(p for p in CSRC.iterdir() if p.suffix in (".cpp", ".hip") and not p.name.startswith("gen"))
GEN_SOURCES = sorted(p for p in CSRC.iterdir() if p.name.startswith("gen") and p.suffix in (".cpp", ".c"))
ORACLE_SOURCES = sorted(p for p in ORACLE.iterdir() if p.suffix == ".c")


def _deps_mtime(paths) -> float:
    return max(p.stat().st_mtime for p in paths)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def _compile_all(jobs, items):
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_run, cmd) for cmd in items]
        for f in futs:
            f.result()


def build_product(force: bool = False, jobs: int = 8, variant: str = "", defines=()) -> Path:
    """variant/defines: an A/B build of the same sources with extra -D flags
    (libodigos_amd<variant>.so, loaded when OSE_LIB_VARIANT=<variant>;
    diagnostics only — the product is the default build)."""
    LIBDIR.mkdir(parents=True, exist_ok=True)
    objdir = OBJDIR / ("variant" + variant) if variant else OBJDIR
    objdir.mkdir(parents=True, exist_ok=True)
    out = LIBDIR / f"libodigos_amd{variant}.so"
    flags = HIP_FLAGS + [d if d.startswith("-") else f"-D{d}" for d in defines]   # -flags pass through
    headers = list(CSRC.glob("*.hpp")) + [ROOT / "include" / "odigos_amd.h"]
    hdr_t = _deps_mtime(headers)
    cmds, objs = [], []
    for src in PRODUCT_SOURCES:
        obj = objdir / (src.name + ".o")
        objs.append(obj)
        if force or variant or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_t):
            cmds.append([HIPCC, *flags, "-c", str(src), "-o", str(obj)])
    _compile_all(jobs, cmds)
    if force or cmds or not out.exists() or out.stat().st_mtime < _deps_mtime(objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(out), *map(str, objs)])
    return out


def build_gen(force: bool = False) -> Path:
    out = LIBDIR / "libosegen.so"
    LIBDIR.mkdir(parents=True, exist_ok=True)
    if GEN_SOURCES and (force or not out.exists() or out.stat().st_mtime < _deps_mtime(GEN_SOURCES + [ROOT / "include" / "odigos_amd.h"])):
        _run(["g++", "-std=c++17", *C_FLAGS, "-shared", "-o", str(out), *map(str, GEN_SOURCES)])
    return out


def build_oracle(force: bool = False) -> Path:
    out = ORACLE / "liboracle.so"
    deps = ORACLE_SOURCES + [ORACLE / "oracle.h", ROOT / "include" / "odigos_amd.h"]
    if force or not out.exists() or out.stat().st_mtime < _deps_mtime(deps):
        _run(["gcc", "-std=c11", *C_FLAGS, "-shared", "-o", str(out), *map(str, ORACLE_SOURCES), "-lm"])
    return out


# ASan + UBSan build of the host code that parses untrusted input (OTLP
# protobuf and JSON, regexps, jsonpath, configs, URLs), driven by
# tests/fuzz/host_fuzz.cpp (tests/test_sanitize.py): test infrastructure,
# never loaded by the product.
SAN_SOURCES = ["pdata", "otlp_pb", "config", "regex_dfa", "unicode_tables", "span_attr", "urlparse"]
SAN_FLAGS = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
             "-fno-omit-frame-pointer", "-pthread", f"-I{ROOT / 'include'}"]


def build_sanitized(force: bool = False, jobs: int = 8) -> Path:
    objdir = OBJDIR / "asan"
    objdir.mkdir(parents=True, exist_ok=True)
    out = objdir / "host_fuzz"
    srcs = [CSRC / f"{n}.cpp" for n in SAN_SOURCES] + [ROOT / "tests" / "fuzz" / "host_fuzz.cpp"]
    hdr_t = _deps_mtime(list(CSRC.glob("*.hpp")) + [ROOT / "include" / "odigos_amd.h"])
    cmds, objs = [], []
    for src in srcs:
        obj = objdir / (src.name + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_t):
            cmds.append(["g++", *SAN_FLAGS, "-c", str(src), "-o", str(obj)])
    _compile_all(jobs, cmds)
    if force or cmds or not out.exists():
        _run(["g++", *SAN_FLAGS, "-o", str(out), *map(str, objs)])
    return out


def build_all(force: bool = False, jobs: int = 8) -> None:
    build_product(force, jobs)
    build_gen(force)
    build_oracle(force)


if __name__ == "__main__":
    if "--variant" in sys.argv:   # python -m odigos_amd.build --variant _b NAME=VALUE ...
        k = sys.argv.index("--variant")
        print("built:", build_product(variant=sys.argv[k + 1], defines=sys.argv[k + 2:]))
        sys.exit(0)
    build_all(force="--force" in sys.argv)
    print("built:", LIBDIR / "libodigos_amd.so", LIBDIR / "libosegen.so", ORACLE / "liboracle.so")
