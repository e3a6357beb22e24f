"""lachain_amd — MI355X (gfx950) batch engine for Lachain's BLS12-381 threshold-crypto hot path.

Product: lachain_amd/liblachain_bls.so (C ABI in include/lachain_bls.h: mcl-shaped single operations +
batch entry points).  Python mirrors of the reference's C# API: lachain_amd.mcl (Fr/G1/G2/GT/MclBls12381),
lachain_amd.tpke (Lachain.Crypto.TPKE), lachain_amd.threshold_signature (Lachain.Crypto.ThresholdSignature).
"""
__all__ = ["native", "mcl", "tpke", "threshold_signature"]
