import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: large CPU-side sizes")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Incremental in-tree build (no-op when up to date).  On the GPU box the
    prebuilt .so files travel with the snapshot; hipcc is present there too."""
    if os.environ.get("OSE_SKIP_BUILD") != "1":
        from odigos_amd import build
        try:
            build.build_all()
        except Exception as e:  # pragma: no cover - surfaced by the tests that need the libs
            if not (build.LIBDIR / "libodigos_amd.so").exists():
                raise
            print("warning: rebuild failed, using prebuilt libraries:", e, file=sys.stderr)
    yield


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
