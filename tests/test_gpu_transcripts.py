"""GPU replay of the committed TPKE / threshold-signature transcripts (tests/golden/transcripts.json):
TPKE N=4 F=1 and N=22 F=7 with reversed, random off-subgroup, other-player and infinity shares
(HoneyBadgerMalicious.cs:23, HoneyBadgerSmartMalicious.cs:28-48); threshold signatures N=7 F=2 and N=100 F=33 with the
same kinds in G2.  Every decision, plaintext and assembled signature must equal the fixture."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "transcripts.json")))
H = bytes.fromhex


def fr(v):
    return (v % 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001).to_bytes(32, "little")


@pytest.fixture(scope="module")
def nat():
    from lachain_amd import native
    native.load()
    return native


@pytest.fixture(params=["normalised", "on_the_fly"])
def line_mode(nat, request):
    """every transcript runs through the normalised line sets (default) and through the on-the-fly fallback that
    a set with a zero line coefficient takes (forced by lcb_set_line_mode): both must reproduce the fixture"""
    nat.set_line_mode(request.param == "on_the_fly")
    yield request.param
    nat.set_line_mode(False)


@pytest.mark.parametrize("key", ["tpke_n4", "tpke_n22"])
def test_tpke_transcript(nat, key, line_mode):
    t = T[key]
    cts = [(H(c["u"]), H(c["v"]), H(c["w"])) for c in t["ciphertexts"]]
    shares = [(ci, i, H(s)) for ci, c in enumerate(t["ciphertexts"]) for i, s in enumerate(c["shares"])]
    got = nat.tpke_verify_shares([H(y) for y in t["y_i"]], cts, shares)
    assert got == [a for c in t["ciphertexts"] for a in c["accept"]]
    probs = [([fr(i + 1) for i in c["combine_ids"]], [H(c["shares"][i]) for i in c["combine_ids"]])
             for c in t["ciphertexts"]]
    us = nat.lagrange_batch(1, probs)
    for c, u in zip(t["ciphertexts"], us):
        assert nat.xor_with_hash(u, H(c["v"])).hex() == c["plaintext"]


@pytest.mark.parametrize("key", ["ts_n7", "ts_n100"])
def test_ts_transcript(nat, key, line_mode):
    t = T[key]
    msgs = [H(r["msg"]) for r in t["rounds"]]
    items = [(ri, i, H(s)) for ri, r in enumerate(t["rounds"]) for i, s in enumerate(r["sigs"])]
    got = nat.ts_verify_shares([H(p) for p in t["pk_i"]], msgs, items)
    assert got == [a for r in t["rounds"] for a in r["accept"]]
    probs = [([fr(i + 1) for i in r["assemble_ids"]], [H(r["sigs"][i]) for i in r["assemble_ids"]])
             for r in t["rounds"]]
    assert [c.hex() for c in nat.lagrange_batch(2, probs)] == [r["combined"] for r in t["rounds"]]
    assert [h.hex() for h in nat.g2_hash_batch(msgs)] == [r["h"] for r in t["rounds"]]
