"""Test configuration: registers the `gpu` marker and puts the repo root / oracle on sys.path.

`-m "not gpu"` tests run in the CPU build container (oracle vs reference KATs, host logic, ABI exports).
`-m gpu` tests run on an MI355X and compare liblachain_bls.so (the product) against oracle/ (the checker).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
# the tests drive the library's tuning hooks (kernel-family thresholds, stream layouts, line mode): opt in for this
# process; production processes leave it unset and the hooks refuse (include/lachain_bls.h)
os.environ.setdefault("LCB_ALLOW_TUNING", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


import pytest  # noqa: E402


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """GPU sessions: initialise torch's HIP runtime before liblachain_bls.so initialises its own.  torch's wheel
    bundles a HIP runtime; when the library's (system ROCm) runtime comes up first, torch's later lazy init can report
    no devices.  bench.py orders it the same way."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda:0")
    yield
