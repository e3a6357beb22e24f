"""lcb_tpke_verify_shares_cached (the prepared-ciphertext and key caches behind the aggregation queue): decisions equal
to the uncached exact path and to the transcripts when a ciphertext's shares arrive one call at a time, across more
distinct ciphertexts than the cache holds (evictions), after the prepare flags change (the cache is emptied), and
across more distinct verification keys than the key cache holds (it starts afresh)."""
import json
import os

import numpy as np
import pytest

from helpers import gpu_native

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
T = json.load(open(os.path.join(HERE, "golden", "transcripts.json")))
H = bytes.fromhex


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


@pytest.mark.parametrize("key", ["tpke_n4", "tpke_n22"])
def test_one_share_per_call_matches_transcripts(nat, key):
    t = T[key]
    ys = [H(y) for y in t["y_i"]]
    cts = [(H(c["u"]), H(c["v"]), H(c["w"])) for c in t["ciphertexts"]]
    want = [a for c in t["ciphertexts"] for a in c["accept"]]
    shares = [(ci, i, H(s)) for ci, c in enumerate(t["ciphertexts"]) for i, s in enumerate(c["shares"])]
    for general in (False, True, False):             # a flag change empties the cache
        nat.set_line_mode(general)
        try:
            got = []
            for ci, i, s in shares:                  # HoneyBadger.cs:211-212: one share per call
                got += nat.tpke_verify_shares(ys, [cts[ci]], [(0, i, s)], cached=True)
            assert got == want
            assert nat.tpke_verify_shares(ys, cts, shares, cached=True) == want
        finally:
            nat.set_line_mode(False)


def test_evictions_beyond_capacity(nat):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    n_cts = 2100                                     # > the 2048 slots
    inp = bench.make_inputs(nat, 0, 22 * n_cts, 22, 7, 32)
    ys = inp["keys_list"]
    cts = inp["cts_list"]
    exp = inp["expect"].astype(bool)
    ct_idx, dec_idx, ui = inp["ct_idx"], inp["dec_idx"], inp["ui"]

    def run(c0, c1):
        sel = np.nonzero((ct_idx >= c0) & (ct_idx < c1))[0]
        sh = [(int(ct_idx[i]) - c0, int(dec_idx[i]), ui[48 * i:48 * i + 48]) for i in sel]
        got = nat.tpke_verify_shares(ys, cts[c0:c1], sh, cached=True)
        assert got == exp[sel].tolist(), (c0, c1)
    for c0 in range(0, n_cts, 100):                  # every ciphertext once: fills and then evicts
        run(c0, min(n_cts, c0 + 100))
    run(0, 50)                                       # evicted early ones come back
    run(2050, 2100)                                  # recent ones hit
    run(0, 50)


def test_key_cache_reorder_and_overflow(nat):
    """keys are cached by their bytes: the same keys at other indices, undecodable keys beside them, and calls whose
    distinct keys overflow the 4096-slot key cache (it starts afresh inside the call) all keep the decisions"""
    t = T["tpke_n4"]
    ys = [H(y) for y in t["y_i"]]
    cts = [(H(c["u"]), H(c["v"]), H(c["w"])) for c in t["ciphertexts"]]
    want = [a for c in t["ciphertexts"] for a in c["accept"]]
    shares = [(ci, i, H(s)) for ci, c in enumerate(t["ciphertexts"]) for i, s in enumerate(c["shares"])]
    assert nat.tpke_verify_shares(ys, cts, shares, cached=True) == want
    rev = ys[::-1]                                   # the same keys, reversed indices
    sh_rev = [(ci, len(ys) - 1 - i, s) for ci, i, s in shares]
    assert nat.tpke_verify_shares(rev, cts, sh_rev, cached=True) == want
    rng = np.random.default_rng(7)
    for rep in range(3):                             # 3 x 3000 distinct junk keys: the second call overflows
        junk = [b"\x9f" + rng.bytes(47) for _ in range(3000)]
        keys = junk + ys
        sh = [(ci, 3000 + i, s) for ci, i, s in shares] + [(0, 5, shares[0][2])]   # + one share under a junk key
        assert nat.tpke_verify_shares(keys, cts, sh, cached=True) == want + [False], rep
    assert nat.tpke_verify_shares(ys, cts, shares, cached=True) == want


def test_more_keys_than_the_key_cache(nat):
    """a call with more distinct keys than the 4096-slot key cache runs uncached and keeps the decisions (ADVICE r5:
    it returned -1 before)"""
    t = T["tpke_n4"]
    ys = [H(y) for y in t["y_i"]]
    cts = [(H(c["u"]), H(c["v"]), H(c["w"])) for c in t["ciphertexts"]]
    want = [a for c in t["ciphertexts"] for a in c["accept"]]
    shares = [(ci, i, H(s)) for ci, c in enumerate(t["ciphertexts"]) for i, s in enumerate(c["shares"])]
    rng = np.random.default_rng(11)
    junk = [b"\x9f" + rng.bytes(47) for _ in range(4097)]
    keys = junk + ys
    sh = [(ci, 4097 + i, s) for ci, i, s in shares] + [(0, 4096, shares[0][2])]
    assert nat.tpke_verify_shares(keys, cts, sh, cached=True) == want + [False]
    assert nat.tpke_verify_shares(ys, cts, shares, cached=True) == want      # the caches still work afterwards
