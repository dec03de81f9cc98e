import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


def pytest_collection_modifyitems(config, items):
    # GPU runs: bring up torch's HIP runtime before any test opens a context
    # through the C-ABI library (a test that needs torch device memory after
    # the library initialised HIP in-process otherwise sees no device)
    if any(it.get_closest_marker("gpu") for it in items) and config.getoption("-m") != "not gpu":
        try:
            import torch
            torch.cuda.is_available()
        except Exception:
            pass
