"""Shared helpers for the tests: deterministic inputs and golden-fixture access."""
import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


class Drbg:
    """Counter-mode SHA-256 DRBG -> Fr by 64-byte wide reduction."""

    def __init__(self, seed: bytes):
        self.seed = seed
        self.ctr = 0

    def bytes(self, n):
        out = b""
        while len(out) < n:
            out += hashlib.sha256(self.seed + self.ctr.to_bytes(8, "little")).digest()
            self.ctr += 1
        return out[:n]

    def fr_int(self):
        return int.from_bytes(self.bytes(64), "little") % R

    def fr(self):
        return self.fr_int().to_bytes(32, "little")


def gpu_native():
    """The product library, initialised for GPU tests.  torch's HIP runtime is brought up first: the tests that
    hand torch-allocated device buffers to the *_dev entry points need torch and liblachain_bls to share the
    device, and torch's bundled runtime refuses to initialise after another runtime has opened it."""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    from lachain_amd import native
    native.lib()  # fails loudly without the library or a gfx950 device
    return native
