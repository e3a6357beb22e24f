#!/usr/bin/env python3
"""tests/golden/make_reference_kats.py — extracts the known-answer DATA the reference's own tests and
sample configs hold for the BLS12-381 path into tests/golden/reference_kats.json.

Run in the build container (reads /root/reference); the JSON it writes is data only (hex vectors and the
file:line they come from), so nothing from the reference has to travel to the GPU box.
Sources:
  test/Lachain.CryptoTest/SerializationTest.cs:20-57   Fr / G1 / G2 serialization vectors
  test/Lachain.CryptoTest/CryptographyTest.cs:103-113  DigestRandomGenerator(Sha3Digest) keystream KAT
  */config*.json  "thresholdSignaturePublicKey" / "TPKEPublicKey"  real G1 encodings (decode acceptance)
"""
import json
import os
import re
import sys

REF = "/root/reference"


def main(out):
    ser = open(os.path.join(REF, "test/Lachain.CryptoTest/SerializationTest.cs")).read().splitlines()
    hexes = []
    for i, line in enumerate(ser, 1):
        m = re.search(r'"0x([0-9a-f]+)"', line)
        if m:
            hexes.append((i, m.group(1)))
    names = ["fr_0", "fr_1", "g1_zero", "g1_generator", "g1_generator_x2", "g2_zero", "g2_generator",
             "g2_generator_x2"]
    assert len(hexes) == len(names), hexes
    kats = {n: {"hex": h, "source": f"test/Lachain.CryptoTest/SerializationTest.cs:{ln}"} for n, (ln, h) in zip(names, hexes)}
    cry = open(os.path.join(REF, "test/Lachain.CryptoTest/CryptographyTest.cs")).read().splitlines()
    for i, line in enumerate(cry, 1):
        if "0x4439ed26" in line:
            kats["kdf_deadbeef_32"] = {"seed_hex": "deadbeef", "hex": re.search(r'"0x([0-9a-f]+)"', line).group(1),
                                       "source": f"test/Lachain.CryptoTest/CryptographyTest.cs:{i}"}
    keys = {}
    for root, _, files in os.walk(REF):
        for f in files:
            if not f.endswith(".json"):
                continue
            p = os.path.join(root, f)
            try:
                lines = open(p, errors="ignore").read().splitlines()
            except OSError:
                continue
            for i, line in enumerate(lines, 1):
                m = re.search(r'"(thresholdSignaturePublicKey|TPKEPublicKey)"\s*:\s*"0x([0-9a-fA-F]+)"', line, re.I)
                if m:
                    h = m.group(2).lower()
                    if m.group(1).lower() == "tpkepublickey":
                        h = h[8:]  # 4-byte LE threshold || 48-byte G1
                    keys.setdefault(h, f"{os.path.relpath(p, REF)}:{i}")
    kats["g1_config_keys"] = [{"hex": h, "source": s} for h, s in sorted(keys.items())]
    with open(out, "w") as fo:
        json.dump(kats, fo, indent=1, sort_keys=True)
    print("wrote", out, "with", len(keys), "config keys")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json"))
