"""Row a13: the consensus decisions taken from the combined CommonCoin signature bytes.

CoinResult.Parity (src/Lachain.Consensus/CommonCoin/CoinResult.cs:16-20) and RootProtocol.GetNonceFromCoin
(src/Lachain.Consensus/RootProtocol/RootProtocol.cs:316-322).  CPU tests: the library's host forms
(lcb_coin_parity / lcb_coin_nonce — byte work, no device needed) against the oracle's restatement and a
line-by-line Python reading of the C# code, on random and edge-case byte strings.  The device batch form
(lcb_coin_fold_dev) is compared in tests/test_gpu_configs.py on GPU-assembled signatures.
"""
import ctypes
import os
import random

import pytest

import oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lachain_amd", "liblachain_bls.so")


def csharp_parity(raw: bytes) -> bool:
    # var p = RawBytes.Aggregate(0u, (i, b) => i ^ b, x => x); return BitsUtils.Popcount(p) % 2 == 1;
    p = 0
    for b in raw:
        p ^= b
    return bin(p).count("1") % 2 == 1


def csharp_nonce(raw: bytes) -> int:
    # res[i % 8] ^= RawBytes[i]; return res.AsReadOnlySpan().ToUInt64()   (little-endian)
    res = bytearray(8)
    for i, b in enumerate(raw):
        res[i % 8] ^= b
    return int.from_bytes(res, "little")


CASES = [b"", b"\x00" * 96, b"\xff" * 96, bytes(range(96)), b"\x01", b"\x80" + b"\x00" * 95]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    from lachain_amd import native
    return native


def test_oracle_matches_csharp_reading():
    rng = random.Random(11)
    for raw in CASES + [bytes(rng.getrandbits(8) for _ in range(rng.choice([48, 96, 97, 5]))) for _ in range(200)]:
        assert o.coin_parity(raw) == csharp_parity(raw)
        assert o.coin_nonce(raw) == csharp_nonce(raw)


def test_library_host_forms_match_oracle(lib):
    rng = random.Random(12)
    for raw in CASES + [bytes(rng.getrandbits(8) for _ in range(96)) for _ in range(300)]:
        assert lib.coin_parity(raw) == o.coin_parity(raw)
        assert lib.coin_nonce(raw) == o.coin_nonce(raw)


def test_parity_of_known_signature_bytes():
    # the G2 generator's serialization (SerializationTest.cs:51) as a coin: the fold is fixed by the bytes alone
    from helpers import kats
    g2 = bytes.fromhex(kats()["g2_generator"]["hex"])
    assert o.coin_parity(g2) == csharp_parity(g2)
    assert o.coin_nonce(g2) == csharp_nonce(g2)
