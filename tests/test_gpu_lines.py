"""The five-lane line-set kernel (k_lines.hip, the small preparations' latency path) against the one-lane kernel
(pairing.hpp lineset_compute via k_lineset_fill): word-for-word equal sets — normalised lines, the normalisation's
scratch, the point and the flags — and equal G2 flags, over G2 points, points with a cofactor-torsion component, a
point of order 13 (exceptional Miller steps: some A_k = 0, the set stays un-normalised), the point at infinity, an
undecodable encoding and the force-general flag, across several blocks of 12 sets (LCB_ALLOW_TEST_HOOKS=1)."""
import os

import numpy as np
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native
from test_gpu_batched import off_subgroup_g2, order13_g2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    n = gpu_native()
    os.environ["LCB_ALLOW_TEST_HOOKS"] = "1"
    yield n
    del os.environ["LCB_ALLOW_TEST_HOOKS"]


def _points(d, n):
    pts = [o.g2_mul(o.g2_gen(), d.fr()) for _ in range(n)]
    q = off_subgroup_g2(d)
    pts[1] = q                                            # odd index: its G2 flag is reported
    pts[3] = o.g2_add(pts[2], o.g2_add(o.g2_mul(q, o.fr(R - 1)), q))   # G2 point + cofactor torsion
    pts[4] = bytes(96)                                    # the point at infinity
    pts[5] = order13_g2(d)
    pts[7] = bytes([0xff] * 96)                           # undecodable: the hook stages infinity
    return pts


def test_coop_line_sets_equal_one_lane_sets(nat):
    d = Drbg(b"gpu-lines-coop")
    pts = _points(d, 30)
    force = bytearray(30)
    force[8] = force[9] = 1
    coop, g2c = nat.test_linesets(pts, True, force)
    ref, g2r = nat.test_linesets(pts, False, force)
    for k in range(30):
        assert np.array_equal(coop[k], ref[k]), k
    assert g2c.tolist() == g2r.tolist()
    want = [int(p == bytes(96) or p == bytes([0xff] * 96) or o.g2_in_subgroup(p)) for p in pts[1::2]]
    assert g2c.tolist() == want
    flag = 6576
    assert coop[8][flag] == 0 and coop[9][flag] == 0     # forced to the on-the-fly path
    assert coop[0][flag] == 1 and coop[4][flag] == 1      # normalised; infinity: every line 1
    assert coop[5][flag] == 0                              # order 13: an A_k == 0 leaves the set un-normalised
    assert not coop[4][:68 * 48].any()


def test_two_wave_coop_line_sets_equal_one_lane_sets(nat):
    """k_lineset_coop_2w (k_prep.hip, the fused census's instance at 256 registers) gives the same sets"""
    d = Drbg(b"gpu-lines-coop-2w")
    pts = _points(d, 26)
    force = bytearray(26)
    force[8] = 1
    two, g2t = nat.test_linesets(pts, 2, force)
    ref, g2r = nat.test_linesets(pts, False, force)
    for k in range(26):
        assert np.array_equal(two[k], ref[k]), k
    assert g2t.tolist() == g2r.tolist()


def test_coop_line_sets_single_and_partial_block(nat):
    d = Drbg(b"gpu-lines-coop-small")
    for n in (1, 2, 13):
        pts = [o.g2_mul(o.g2_gen(), d.fr()) for _ in range(n)]
        coop, g2c = nat.test_linesets(pts, True)
        ref, g2r = nat.test_linesets(pts, False)
        assert np.array_equal(coop, ref), n
        assert g2c.tolist() == g2r.tolist() == [1] * (n // 2)
