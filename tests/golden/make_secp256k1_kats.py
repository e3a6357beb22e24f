#!/usr/bin/env python3
"""tests/golden/make_secp256k1_kats.py — extracts the known-answer DATA the reference's own tests hold for the
secp256k1 ECDSA / Keccak path into tests/golden/secp256k1_kats.json.

Run in the build container (reads /root/reference); the JSON is data only (hex vectors and the file:line they come
from).  Source: test/Lachain.CryptoTest/CryptographyTest.cs
  :33-34   TestString, :68-73 its Keccak-256 (Test_KeccakTestVector)
  :115-128 Test_HeaderKeccak: header {zero hashes, Index 0, Nonce 1} -> Keccak
  :176-178 Test_SignRoundTrip private key -> address
  :236-271 Test_TxHash2: unsigned EIP-155 RLP (chain id 25), the two signed RLPs the reference's signer produced
           (old chain id 25, new chain id 225) and their full hashes
  :316-380 Test_External_Signature: RLPs (chain ids 25 / 225) and the externally produced 65 / 66-byte signatures
Every signature must verify under the key of :176 (DefaultCrypto.VerifySignatureHashed semantics).  The unsigned RLP
for chain id 225 in Test_TxHash2 is not spelled out in the test; it is the chain-id-25 RLP with the chain-id element
0x19 replaced by 0x81e1 and the list header re-derived (EIP-155), recorded as "derived".
"""
import json
import os
import re
import sys

REF = "/root/reference"
SRC = "test/Lachain.CryptoTest/CryptographyTest.cs"


def rlp_items(b):
    """top-level items of one RLP list (strings only, as in a legacy transaction)"""
    p = b[0]
    if p >= 0xf8:
        ll = p - 0xf7
        off = 1 + ll
    else:
        off = 1
    out = []
    while off < len(b):
        h = b[off]
        if h < 0x80:
            out.append(bytes([h])); off += 1
        elif h <= 0xb7:
            n = h - 0x80; out.append(b[off + 1:off + 1 + n]); off += 1 + n
        else:
            ll = h - 0xb7; n = int.from_bytes(b[off + 1:off + 1 + ll], "big")
            out.append(b[off + 1 + ll:off + 1 + ll + n]); off += 1 + ll + n
    return out


def rlp_list(items):
    def el(x):
        if len(x) == 1 and x[0] < 0x80:
            return x
        if len(x) < 56:
            return bytes([0x80 + len(x)]) + x
        n = len(x).to_bytes((len(x).bit_length() + 7) // 8, "big")
        return bytes([0xb7 + len(n)]) + n + x
    body = b"".join(el(x) for x in items)
    if len(body) < 56:
        return bytes([0xc0 + len(body)]) + body
    n = len(body).to_bytes((len(body).bit_length() + 7) // 8, "big")
    return bytes([0xf7 + len(n)]) + n + body


def main(out):
    lines = open(os.path.join(REF, SRC)).read().splitlines()

    def find(pat, start=0):
        for i in range(start, len(lines)):
            if re.search(pat, lines[i]):
                return i
        raise KeyError(pat)

    def hex_at(i):
        return re.search(r'"0x([0-9a-fA-F]+)"', lines[i]).group(1).lower()

    def src(i):
        return f"{SRC}:{i + 1}"

    k = {}
    i = find(r"TestString =")
    msg = re.search(r'GetBytes\("([^"]*)"\)', lines[i + 1]).group(1)
    j = find(r"0x45d3b367", i)
    k["keccak256"] = {"msg_ascii": msg, "hex": hex_at(j), "source": src(j)}
    j = find(r"Test_HeaderKeccak")
    h = find(r"Assert.AreEqual\(\"0x", j)
    assert "Nonce = 1" in "".join(lines[j:h]) and "Index = 0" in "".join(lines[j:h])
    k["header_keccak"] = {"prev": "00" * 32, "state": "00" * 32, "merkle": "00" * 32, "index": 0, "nonce": 1,
                          "hex": hex_at(h), "source": src(h)}
    j = find(r"Test_SignRoundTrip")
    pk = find(r"privateKey = \"0x", j)
    ad = find(r"address = \"0x", j)
    k["priv_address"] = {"priv": hex_at(pk), "address": hex_at(ad), "source": f"{src(pk)},{ad + 1}"}

    sigs = []
    j = find(r"Test_TxHash2")
    u = find(r"f84d0101", j)
    unsigned25 = bytes.fromhex(hex_at(u))
    s_old = find(r"f88d0101", j)
    fh_old = find(r"0x4f0da38b", j)
    s_new = find(r"f88f0101", j)
    fh_new = find(r"0x0d3515b2", j)
    for sl, fl, chain, new in ((s_old, fh_old, 25, False), (s_new, fh_new, 225, True)):
        signed = bytes.fromhex(hex_at(sl))
        it = rlp_items(signed)
        v, r, s = it[6], it[7], it[8]
        assert int.from_bytes(v, "big") in (chain * 2 + 35, chain * 2 + 36)
        unsigned = rlp_list(it[:6] + [chain.to_bytes((chain.bit_length() + 7) // 8, "big"), b"", b""])
        if chain == 25:
            assert unsigned == unsigned25
        sig = r.rjust(32, b"\0") + s.rjust(32, b"\0") + (v.rjust(2, b"\0") if new else v)
        sigs.append({"msg_rlp": unsigned.hex(), "msg_rlp_note": "from the test" if chain == 25 else "derived",
                     "signed_rlp": signed.hex(), "full_hash": hex_at(fl), "sig": sig.hex(), "chain_id": chain,
                     "use_new_chain_id": new, "source": f"{src(sl)} (signature), {src(u)} (unsigned RLP)"})
    j = find(r"public void Test_External_Signature")
    for chain, new in ((25, False), (225, True)):
        r = find(r'^\s*"0xf[0-9a-f]*8080"\s*$', j)
        s = find(r'^\s*"0x[0-9A-F]{130,132}"\s*$', r)
        sigs.append({"msg_rlp": hex_at(r), "sig": hex_at(s), "chain_id": chain, "use_new_chain_id": new,
                     "source": f"{src(s)} (signature), {src(r)} (RLP)"})
        j = s + 1
    k["signatures"] = sigs
    with open(out, "w") as fo:
        json.dump(k, fo, indent=1, sort_keys=True)
    print("wrote", out, "with", len(sigs), "signatures")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "secp256k1_kats.json"))
