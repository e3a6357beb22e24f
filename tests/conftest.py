"""Test configuration: registers the `gpu` marker and puts the repo root / oracle on sys.path.

`-m "not gpu"` tests run in the CPU build container (oracle vs reference KATs, host logic, ABI exports).
`-m gpu` tests run on an MI355X and compare liblachain_bls.so (the product) against oracle/ (the checker).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
