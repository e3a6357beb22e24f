"""GPU Reed-Solomon erasure coding of the reliable broadcast (k_rs.hip) against the oracle
(oracle/rs.c, pinned by the codec README's known answer and ErasureCodingTest.cs): ErasureCodingShards and
DecodeFromEchos (src/Lachain.Consensus/ReliableBroadcast/ReliableBroadcast.cs:393-446) at the validator counts of the
BASELINE configs, random erasure patterns, odd shard sizes, AugmentInput's length prefix + padding, and the
unsolvable 256-shard pattern.  Bit-exact: every shard byte."""
import random
import struct

import pytest

import oracle as o
from helpers import gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


def augment(payload: bytes, n, f):
    """ReliableBroadcast.AugmentInput (ReliableBroadcast.cs:311-319): int32 LE length prefix, zero padding"""
    data = struct.pack("<i", len(payload)) + payload
    k = n - 2 * f
    size = (len(data) + k - 1) // k
    return data + bytes(k * size - len(data))


def test_erasure_coding_test_vector(nat):
    data = bytes(range(100))
    shards = nat.rs_encode(data, 4, 2)
    assert shards == o.rs_encode_shards(data, 4, 2)
    S = len(shards) // 4
    assert nat.rs_decode([(1, shards[S:2 * S]), (2, shards[2 * S:3 * S])], S, 4, 2) == shards


@pytest.mark.parametrize("n", [4, 7, 22, 100, 256])
def test_encode_decode_vs_oracle(nat, n):
    f = (n - 1) // 3
    rng = random.Random(n)
    for plen in (1, 180, 4093, 65536):
        data = augment(bytes(rng.randrange(256) for _ in range(plen)), n, f)
        k = n - 2 * f
        shards = nat.rs_encode(data, n, 2 * f)
        assert shards == o.rs_encode_shards(data, n, 2 * f), (n, plen)
        S = len(data) // k
        for _ in range(2):
            keep = sorted(rng.sample(range(n), k))
            if n == 256 and 0 not in keep and 255 not in keep:
                keep = sorted(set(keep[1:]) | {0})   # keep the pattern solvable (see the collision test)
            echos = [(j, shards[j * S:(j + 1) * S]) for j in keep]
            rng.shuffle(echos)                        # echoes arrive in any order
            got = nat.rs_decode(echos, S, n, 2 * f)
            assert got == shards == o.rs_decode_shards(echos, S, n, 2 * f), (n, plen)
            # DecodeFromEchos then reads the int32 length prefix back (ReliableBroadcast.cs:270-271)
            assert struct.unpack_from("<i", got, 0)[0] == plen


def test_256_shards_unsolvable_pattern_fails(nat):
    n, f = 256, 85
    data = augment(bytes(range(200)), n, f)
    shards = nat.rs_encode(data, n, 2 * f)
    S = len(data) // (n - 2 * f)
    erased = {0, 255} | set(range(1, 2 * f - 1))
    echos = [(j, shards[j * S:(j + 1) * S]) for j in range(n) if j not in erased]
    assert o.rs_decode_shards(echos, S, n, 2 * f) is None
    with pytest.raises(RuntimeError):
        nat.rs_decode(echos, S, n, 2 * f)


def test_bad_arguments(nat):
    with pytest.raises(RuntimeError):
        nat.rs_encode(bytes(10), 5, 2)                # 10 bytes are not a multiple of the 3 data shards
    with pytest.raises(RuntimeError):
        nat.rs_decode([(0, b"ab")], 2, 4, 2)         # needs exactly N - 2F echoes
