"""CPU checks of the Reed-Solomon restatement (oracle/rs.c) used as the checker for the reliable-broadcast erasure
coding (ReliableBroadcast.ErasureCodingShards / DecodeFromEchos, src/Lachain.Consensus/ReliableBroadcast/
ReliableBroadcast.cs:393-446; ErasureCoding.cs:13 GenericGF(285, 256, 0)).  The codec library is a submodule the
reference tree does not check out; its README (ReliableBroadcast/ReedSolomon/README.md) holds the known answers used
here, and test/Lachain.ConsensusTest/ErasureCodingTest.cs the round-trip property.  A pure-Python restatement
(polynomial remainder + linear-algebra erasure solve, a different algorithm from rs.c's Forney decoder) cross-checks
random cases."""
import random

import oracle as o

# README.md: "Hello World" + 9 ecc symbols
HELLO = [0x48, 0x65, 0x6C, 0x6C, 0x6F, 0x20, 0x57, 0x6F, 0x72, 0x6C, 0x64]
HELLO_ECC = [0x40, 0x86, 0x08, 0xD5, 0x2C, 0xAE, 0xB5, 0x8F, 0x83]

EXP, LOG = [0] * 512, [0] * 256
_x = 1
for _i in range(255):
    EXP[_i], LOG[_x] = _x, _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def gmul(a, b):
    return EXP[LOG[a] + LOG[b]] if a and b else 0


def ginv(a):
    return EXP[255 - LOG[a]]


def py_encode(data, ecc):
    """ZXing-style: remainder of D(x) x^ecc mod prod (x - alpha^i), i < ecc"""
    g = [1]
    for i in range(ecc):
        r = EXP[i]
        g = [a ^ gmul(b, r) for a, b in zip(g + [0], [0] + g)]
    rem = list(data) + [0] * ecc
    for j in range(len(data)):
        c = rem[j]
        if c:
            for t in range(1, ecc + 1):
                rem[j + t] ^= gmul(g[t], c)
    return list(data) + rem[len(data):]


def py_erasure_solve(cw, erased, ecc):
    """solve H_E c_E = H_K c_K (H[i][j] = alpha^(i (n-1-j))) by Gaussian elimination"""
    n = len(cw)
    known = [j for j in range(n) if j not in erased]
    rows = []
    for i in range(ecc):
        lhs = [EXP[(i * (n - 1 - j)) % 255] for j in erased]
        rhs = 0
        for j in known:
            rhs ^= gmul(EXP[(i * (n - 1 - j)) % 255], cw[j])
        rows.append(lhs + [rhs])
    m = len(erased)
    for c in range(m):
        p = next(r for r in range(c, len(rows)) if rows[r][c])
        rows[c], rows[p] = rows[p], rows[c]
        iv = ginv(rows[c][c])
        rows[c] = [gmul(v, iv) for v in rows[c]]
        for r in range(len(rows)):
            if r != c and rows[r][c]:
                f = rows[r][c]
                rows[r] = [a ^ gmul(f, b) for a, b in zip(rows[r], rows[c])]
    out = list(cw)
    for idx, j in enumerate(erased):
        out[j] = rows[idx][m]
    return out


def test_readme_known_answer():
    assert o.rs_encode_codeword(HELLO, 9)[11:] == HELLO_ECC
    assert py_encode(HELLO, 9)[11:] == HELLO_ECC


def test_readme_decode_example_as_erasures():
    # README's decode example marks positions 0, 1, 2 (and corrupts 3..5); the reliable broadcast only ever has
    # erasures, so erase all six and recover the codeword
    import ctypes
    cw = HELLO + HELLO_ECC
    bad = [0x00, 0x02, 0x02, 0x02, 0x02, 0x02] + cw[6:]
    arr = (ctypes.c_int * 20)(*bad)
    pos = (ctypes.c_int * 6)(0, 1, 2, 3, 4, 5)
    assert o.lib().orc_rs_decode_erasures(arr, 20, 9, pos, 6) == 0
    assert list(arr) == cw


def test_erasure_coding_test_round_trip():
    # test/Lachain.ConsensusTest/ErasureCodingTest.cs: 100 bytes, 4 shards, 2 erasures, decode from shards 1 and 2
    data = bytes(range(100))
    shards = o.rs_encode_shards(data, 4, 2)
    S = len(shards) // 4
    assert shards[:100] == data
    assert o.rs_decode_shards([(1, shards[S:2 * S]), (2, shards[2 * S:3 * S])], S, 4, 2) == shards


def test_random_cases_match_python_restatement():
    rng = random.Random(7)
    for n, f in ((4, 1), (7, 2), (22, 7), (100, 33), (255, 84)):
        ecc, k = 2 * f, n - 2 * f
        for _ in range(3):
            data = [rng.randrange(256) for _ in range(k)]
            cw = o.rs_encode_codeword(data, ecc)
            assert cw == py_encode(data, ecc)
            erased = sorted(rng.sample(range(n), ecc))
            assert py_erasure_solve([0 if j in erased else v for j, v in enumerate(cw)], erased, ecc) == cw
            S = 3
            payload = bytes(rng.randrange(256) for _ in range(k * S))
            shards = o.rs_encode_shards(payload, n, ecc)
            keep = sorted(set(range(n)) - set(erased))
            assert o.rs_decode_shards([(j, shards[j * S:(j + 1) * S]) for j in keep], S, n, ecc) == shards


def test_256_shards_collision_is_unsolvable():
    # N = 256 validators exceeds GF(2^8)'s 255 distinct evaluation points: positions 0 and 255 share alpha^0, so an
    # erasure set holding both cannot be solved (the reference codec reports "too many errors-erasures")
    n, f = 256, 85
    data = bytes(range(256)) * 1
    payload = (data * 2)[:n - 2 * f]
    shards = o.rs_encode_shards(payload, n, 2 * f)
    erased = [0, 255] + list(range(1, 2 * f - 1))
    keep = [j for j in range(n) if j not in erased]
    assert o.rs_decode_shards([(j, shards[j:j + 1]) for j in keep], 1, n, 2 * f) is None
    erased = list(range(1, 2 * f + 1))               # 0 kept, 255 kept: solvable
    keep = [j for j in range(n) if j not in erased]
    assert o.rs_decode_shards([(j, shards[j:j + 1]) for j in keep], 1, n, 2 * f) == shards
