import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from orc_bind import load_oracle
    return load_oracle()


@pytest.fixture(scope="session")
def tunings():
    import json
    return json.loads((Path(__file__).resolve().parent / "golden" / "tunings.json").read_text())


@pytest.fixture(scope="session")
def refchk():
    from orc_bind import load_ref
    lib = load_ref()
    if lib is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    return lib


@pytest.fixture(scope="session", autouse=True)
def _torch_device_first():
    """Tests that hand torch device buffers to the engine need torch's HIP runtime
    initialised before libtbf initialises HIP in the same process (bench.py does the
    same: torch.cuda.set_device before the engine)."""
    try:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    except Exception:
        pass
    yield
