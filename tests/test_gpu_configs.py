"""GPU parity at the BASELINE.json config sizes that the round-1 tests did not reach, against the oracle.

* configs[2] CommonCoin N=100 F=33: share verification, first-34-valid selection with invalid shares among the
  first 34, G2 Lagrange (k=34), combined-signature check — ThresholdSigner.AddShare
  (src/Lachain.Crypto/ThresholdSignature/ThresholdSigner.cs:44-87, PublicKeySet.cs:34-42).
* configs[4] epoch-replay slice N=256 F=85: TPKE share verification of two ciphertexts with malicious shares
  (reversed bytes as test/Lachain.ConsensusTest/HoneyBadgerMalicious.cs:23, a cofactor-torsion share that still
  passes the pairing check), FullDecrypt combination k=86 (TPKE/PublicKey.cs:55-86), and two coins of 256
  signature shares assembled at k=86 with their parity / nonce (CoinResult.cs:16-20, RootProtocol.cs:316-322).
* configs[3] MSM known answers at 2^20 (default window) and 2^24 points (c = 20).
* Lagrange interpolation with inputs outside the r-torsion (G1.FromBytes / G2.FromBytes accept them):
  the GPU lanes must equal the oracle's plain double-and-add (MclBls12381.LagrangeInterpolate, PublicKey.cs:83).
Bit-exact throughout: accept bitmaps, serialized points, plaintext bytes.
"""
import numpy as np
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


@pytest.fixture(scope="module")
def tdev():
    import torch
    return torch, torch.device("cuda", 0)


def coin_id(era, agreement, epoch):
    """CoinId.ToBytes() = Era || Agreement || Epoch, int64 LE two's complement (CoinId.cs:21-24)"""
    return b"".join((v & M64).to_bytes(8, "little") for v in (era, agreement, epoch))


def keyset(d, n, f):
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    return [poly(i + 1) for i in range(n)], poly(0)


def up(torch, dev, b):
    if isinstance(b, np.ndarray):
        b = b.tobytes()
    return torch.frombuffer(bytearray(b if len(b) else b"\0"), dtype=torch.uint8).to(dev)


def off_subgroup_g1(d):
    """an on-curve G1 encoding outside the r-torsion"""
    while True:
        x = int.from_bytes(d.bytes(48), "little") % o.P
        enc = bytearray(x.to_bytes(48, "little"))
        enc[47] |= 0x80 * (d.bytes(1)[0] & 1)
        enc = bytes(enc)
        if o.g1_valid(enc) and enc != bytes(48) and not o.g1_in_subgroup(enc):
            return enc


def off_subgroup_g2(d):
    while True:
        xa = int.from_bytes(d.bytes(48), "little") % o.P
        xb = int.from_bytes(d.bytes(48), "little") % o.P
        enc = bytearray(xa.to_bytes(48, "little") + xb.to_bytes(48, "little"))
        enc[95] |= 0x80 * (d.bytes(1)[0] & 1)
        enc = bytes(enc)
        if o.g2_valid(enc) and not o.g2_in_subgroup(enc):
            return enc


def torsion_g1(d):
    """a nonzero point of the cofactor torsion: T = [r]Q = [r-1]Q + Q for an off-subgroup Q"""
    q = off_subgroup_g1(d)
    t = o.g1_add(o.g1_mul(q, o.fr(R - 1)), q)
    assert t != bytes(48) and not o.g1_in_subgroup(t)
    return t


# ---------------------------------------------------------------- configs[2]: CommonCoin N=100, F=33
def test_commoncoin_n100_k34(nat, tdev):
    torch, dev = tdev
    n, f, rounds = 100, 33, 3
    d = Drbg(b"gpu-cc-n100")
    sks, shared = keyset(d, n, f)
    pks = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in sks] + [o.g1_mul(o.g1_gen(), o.fr(shared))]
    msgs = [coin_id(7, r, 3) for r in range(rounds)]
    sigs = [[o.ts_sign(o.fr(sks[i]), msgs[r]) for i in range(n)] for r in range(rounds)]
    # round 1: shares 3, 10, 33 invalid (another share's signature, a doubled one, the wrong message's);
    # round 2: 67 invalid shares, only 33 valid (< F+1): no signature
    sigs[1][3] = sigs[1][4]
    sigs[1][10] = o.g2_add(sigs[1][10], sigs[1][10])
    sigs[1][33] = sigs[0][33]
    for i in range(67):
        sigs[2][i] = sigs[2][i + 1]
    flat = [s for row in sigs for s in row]
    expect = [o.ts_validate(pks[i % n], flat[i], msgs[i // n]) == 1 for i in range(rounds * n)]
    assert sum(expect[n:2 * n]) == n - 3 and sum(expect[2 * n:]) == 33
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_pks, d_msg = up(torch, dev, b"".join(pks)), up(torch, dev, b"".join(msgs))
    d_moff = up(torch, dev, np.arange(0, 24 * (rounds + 1), 24, dtype=np.uint32))
    d_sigs = up(torch, dev, b"".join(flat))
    d_midx = up(torch, dev, np.repeat(np.arange(rounds, dtype=np.uint32), n))
    d_pidx = up(torch, dev, np.tile(np.arange(n, dtype=np.uint32), rounds))
    d_acc = torch.zeros(rounds * n, dtype=torch.uint8, device=dev)
    d_comb = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_cacc = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_par = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_non = torch.zeros(8 * rounds, dtype=torch.uint8, device=dev)
    assert lib.lcb_ts_prepare_dev(d_pks.data_ptr(), n + 1, d_msg.data_ptr(), d_moff.data_ptr(), rounds, sh) == 0
    assert lib.lcb_ts_verify_prepared_dev(d_acc.data_ptr(), rounds * n, n + 1, rounds, d_sigs.data_ptr(),
                                          d_midx.data_ptr(), d_pidx.data_ptr(), sh) == 0
    assert lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(), d_sigs.data_ptr(), n,
                                   f + 1, rounds, sh) == 0
    d_ridx = up(torch, dev, np.arange(rounds, dtype=np.uint32))
    d_shared = up(torch, dev, np.full(rounds, n, dtype=np.uint32))
    assert lib.lcb_ts_verify_prepared_dev(d_cacc.data_ptr(), rounds, n + 1, rounds, d_comb.data_ptr(),
                                          d_ridx.data_ptr(), d_shared.data_ptr(), sh) == 0
    assert lib.lcb_coin_fold_dev(d_par.data_ptr(), d_non.data_ptr(), d_comb.data_ptr(), rounds, sh) == 0
    torch.cuda.synchronize(dev)
    assert [bool(x) for x in d_acc.cpu().numpy()] == expect
    assert d_cst.cpu().numpy().tolist() == [1, 1, 0]
    assert d_cacc.cpu().numpy().tolist() == [1, 1, 0]
    comb = d_comb.cpu().numpy().tobytes()
    par = d_par.cpu().numpy().tolist()
    non = np.frombuffer(d_non.cpu().numpy().tobytes(), dtype="<u8").tolist()
    for r in (0, 1):
        valid = [i for i in range(n) if expect[r * n + i]][:f + 1]
        assert len(valid) == f + 1
        got = comb[96 * r:96 * r + 96]
        assert got == o.g2_lagrange([o.fr(i + 1) for i in valid], [sigs[r][i] for i in valid])
        assert got == o.ts_sign(o.fr(shared), msgs[r])
        assert bool(par[r]) == o.coin_parity(got) and non[r] == o.coin_nonce(got)


# ---------------------------------------------------------------- configs[4]: epoch-replay slice N=256, F=85
def test_epoch_slice_n256_k86(nat, tdev):
    torch, dev = tdev
    n, f = 256, 85
    k = f + 1
    d = Drbg(b"gpu-epoch-n256")
    xs, y_secret = keyset(d, n, f)
    y = o.g1_mul(o.g1_gen(), o.fr(y_secret))
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    plains = [d.bytes(32), d.bytes(32)]
    cts = [o.tpke_encrypt(y, p, o.fr(d.fr_int())) for p in plains]
    # U_i = x_i U (PrivateKey.Decrypt after its validity check, checked below on the GPU)
    shares = [[o.g1_mul(U, o.fr(x)) for x in xs] for (U, _, _) in cts]
    # ciphertext 0: the first ten shares belong to other decryptors (wrong), share 40 reversed (malformed or
    # wrong, HoneyBadgerMalicious.cs:23); ciphertext 1: share 7 carries a cofactor-torsion component (passes the
    # pairing check, so it enters the combination), share 9 is off the subgroup altogether
    for j in range(10):
        shares[0][j] = shares[0][j + 1]
    shares[0][40] = shares[0][40][::-1]
    shares[1][7] = o.g1_add(shares[1][7], torsion_g1(d))
    shares[1][9] = off_subgroup_g1(d)
    flat = [s for row in shares for s in row]

    def ok(i):
        c, j = divmod(i, n)
        if not o.g1_valid(flat[i]):
            return False
        return o.tpke_verify_share(yi[j], *cts[c], flat[i]) == 1
    expect = [ok(i) for i in range(2 * n)]
    assert expect[n + 7] and not expect[n + 9] and sum(expect[:n]) in (n - 10, n - 11)
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_y = up(torch, dev, b"".join(yi))
    d_u = up(torch, dev, b"".join(c[0] for c in cts))
    d_w = up(torch, dev, b"".join(c[2] for c in cts))
    d_v = up(torch, dev, b"".join(c[1] for c in cts))
    d_voff = up(torch, dev, np.array([0, 32, 64], dtype=np.uint32))
    d_ct = up(torch, dev, np.repeat(np.arange(2, dtype=np.uint32), n))
    d_dec = up(torch, dev, np.tile(np.arange(n, dtype=np.uint32), 2))
    d_sh = up(torch, dev, b"".join(flat))
    d_acc = torch.zeros(2 * n, dtype=torch.uint8, device=dev)
    d_uc = torch.zeros(96, dtype=torch.uint8, device=dev)
    d_ust = torch.zeros(2, dtype=torch.uint8, device=dev)
    d_x = up(torch, dev, b"".join(o.fr(xs[j]) for j in (5, 200)))
    d_own = torch.zeros(96, dtype=torch.uint8, device=dev)
    d_own_st = torch.zeros(2, dtype=torch.uint8, device=dev)
    assert lib.lcb_tpke_prepare_dev(d_y.data_ptr(), n, d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(),
                                    d_voff.data_ptr(), 2, sh) == 0
    assert lib.lcb_tpke_partial_decrypt_prepared_dev(d_own.data_ptr(), d_own_st.data_ptr(), d_x.data_ptr(), 1,
                                                     d_u.data_ptr(), 2, sh) == 0
    assert lib.lcb_tpke_verify_prepared_dev(d_acc.data_ptr(), 2 * n, n, 2, d_ct.data_ptr(), d_dec.data_ptr(),
                                            d_sh.data_ptr(), sh) == 0
    assert lib.lcb_tpke_combine_dev(d_uc.data_ptr(), d_ust.data_ptr(), d_acc.data_ptr(), d_sh.data_ptr(), n, k, 2,
                                    sh) == 0
    torch.cuda.synchronize(dev)
    assert [bool(a) for a in d_acc.cpu().numpy()] == expect
    own = d_own.cpu().numpy().tobytes()
    assert d_own_st.cpu().numpy().tolist() == [1, 1]
    assert own[:48] == o.tpke_decrypt(*cts[0], o.fr(xs[5])) and own[48:] == o.tpke_decrypt(*cts[1], o.fr(xs[200]))
    assert d_ust.cpu().numpy().tolist() == [1, 1]
    uc = d_uc.cpu().numpy().tobytes()
    for c in (0, 1):
        valid = [j for j in range(n) if expect[c * n + j]][:k]
        u_exp = o.g1_lagrange([o.fr(j + 1) for j in valid], [shares[c][j] for j in valid])
        assert uc[48 * c:48 * c + 48] == u_exp, c
        assert o.tpke_full_decrypt(cts[c][1], valid, [shares[c][j] for j in valid]) == \
            o.xor_with_hash(uc[48 * c:48 * c + 48], cts[c][1])
    # ciphertext 0 decrypts; ciphertext 1's combination includes the torsion share, so both sides get the same
    # (wrong) plaintext — bit-exact agreement is what matters for consensus
    assert o.xor_with_hash(uc[:48], cts[0][1]) == plains[0]
    assert o.xor_with_hash(uc[48:], cts[1][1]) != plains[1]
    # arrival order (HoneyBadger.cs:237-247 combines the first F+1 valid shares to ARRIVE): ciphertext 0 in reverse
    # order, ciphertext 1 in a shuffled order in which the torsion share 7 arrives last and 20 decryptors never send
    rng = np.random.default_rng(7)
    perm = [j for j in rng.permutation(n).tolist() if j != 7] + [7]
    order1 = perm[:n - 21] + [7] + [0xFFFFFFFF] * 20
    orders = [list(range(n - 1, -1, -1)), order1]
    d_ord = up(torch, dev, np.array(orders, dtype=np.uint32))
    assert lib.lcb_tpke_combine_ordered_dev(d_uc.data_ptr(), d_ust.data_ptr(), d_acc.data_ptr(), d_sh.data_ptr(),
                                            d_ord.data_ptr(), n, k, 2, sh) == 0
    torch.cuda.synchronize(dev)
    assert d_ust.cpu().numpy().tolist() == [1, 1]
    uc = d_uc.cpu().numpy().tobytes()
    for c in (0, 1):
        valid = [j for j in orders[c] if j < n and expect[c * n + j]][:k]
        assert 7 not in valid or c == 0
        u_exp = o.g1_lagrange([o.fr(j + 1) for j in valid], [shares[c][j] for j in valid])
        assert uc[48 * c:48 * c + 48] == u_exp, c
        assert o.xor_with_hash(uc[48 * c:48 * c + 48], cts[c][1]) == plains[c]     # no torsion share combined
    # a decryptor listed twice is a repeated abscissa: the group fails
    dup = [orders[0], [3, 3] + [j for j in range(n) if j != 3]][:2]
    d_ord = up(torch, dev, np.array([dup[0], dup[1][:n]], dtype=np.uint32))
    assert lib.lcb_tpke_combine_ordered_dev(d_uc.data_ptr(), d_ust.data_ptr(), d_acc.data_ptr(), d_sh.data_ptr(),
                                            d_ord.data_ptr(), n, k, 2, sh) == 0
    torch.cuda.synchronize(dev)
    assert d_ust.cpu().numpy().tolist() == [1, 0]

    # two coins of the era (root coin agreement -1, one BA coin), 256 signature shares each, k = 86
    sks, shared = keyset(d, n, f)
    pks = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in sks] + [o.g1_mul(o.g1_gen(), o.fr(shared))]
    msgs = [coin_id(0, -1, 0), coin_id(0, 0, 0)]
    sigs = [[o.ts_sign(o.fr(x), m) for x in sks] for m in msgs]
    sigs[0][0] = sigs[0][1]
    sigs[1][85] = sigs[1][85][::-1]
    sflat = [s for row in sigs for s in row]

    def sok(i):
        m, j = divmod(i, n)
        return o.g2_valid(sflat[i]) and o.ts_validate(pks[j], sflat[i], msgs[m]) == 1
    sexp = [sok(i) for i in range(2 * n)]
    d_pks, d_msg = up(torch, dev, b"".join(pks)), up(torch, dev, b"".join(msgs))
    d_moff = up(torch, dev, np.array([0, 24, 48], dtype=np.uint32))
    d_sigs = up(torch, dev, b"".join(sflat))
    d_sacc = torch.zeros(2 * n, dtype=torch.uint8, device=dev)
    d_comb = torch.zeros(192, dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(2, dtype=torch.uint8, device=dev)
    d_par = torch.zeros(2, dtype=torch.uint8, device=dev)
    d_non = torch.zeros(16, dtype=torch.uint8, device=dev)
    assert lib.lcb_ts_prepare_dev(d_pks.data_ptr(), n + 1, d_msg.data_ptr(), d_moff.data_ptr(), 2, sh) == 0
    assert lib.lcb_ts_verify_prepared_dev(d_sacc.data_ptr(), 2 * n, n + 1, 2, d_sigs.data_ptr(), d_ct.data_ptr(),
                                          d_dec.data_ptr(), sh) == 0
    assert lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_sacc.data_ptr(), d_sigs.data_ptr(), n, k,
                                   2, sh) == 0
    assert lib.lcb_coin_fold_dev(d_par.data_ptr(), d_non.data_ptr(), d_comb.data_ptr(), 2, sh) == 0
    torch.cuda.synchronize(dev)
    assert [bool(a) for a in d_sacc.cpu().numpy()] == sexp
    assert d_cst.cpu().numpy().tolist() == [1, 1]
    comb = d_comb.cpu().numpy().tobytes()
    par = d_par.cpu().numpy().tolist()
    non = np.frombuffer(d_non.cpu().numpy().tobytes(), dtype="<u8").tolist()
    for m in (0, 1):
        valid = [j for j in range(n) if sexp[m * n + j]][:k]
        got = comb[96 * m:96 * m + 96]
        assert got == o.g2_lagrange([o.fr(j + 1) for j in valid], [sigs[m][j] for j in valid])
        assert got == o.ts_sign(o.fr(shared), msgs[m])
        assert bool(par[m]) == o.coin_parity(got) and non[m] == o.coin_nonce(got)


# ---------------------------------------------------------------- off-subgroup Lagrange inputs
def test_lagrange_off_subgroup_inputs(nat):
    d = Drbg(b"gpu-lagrange-off-subgroup")
    G1, G2 = o.g1_gen(), o.g2_gen()
    for k in (1, 2, 5, 34):
        xs = [o.fr(3 * i + 2) for i in range(k)]
        ys1 = [o.g1_mul(G1, d.fr()) for _ in range(k)]
        ys2 = [o.g2_mul(G2, d.fr()) for _ in range(k)]
        for j in range(0, k, 2):          # every other input outside the r-torsion
            ys1[j] = off_subgroup_g1(d)
            ys2[j] = off_subgroup_g2(d)
        got1, got2 = nat.lagrange_batch(1, [(xs, ys1)])[0], nat.lagrange_batch(2, [(xs, ys2)])[0]
        assert got1 == o.g1_lagrange(xs, ys1), k
        assert got2 == o.g2_lagrange(xs, ys2), k
    # a verified share plus cofactor torsion, mixed with honest shares (the FullDecrypt case)
    xs = [o.fr(i + 1) for i in range(4)]
    ys = [o.g1_mul(G1, d.fr()) for _ in range(4)]
    ys[2] = o.g1_add(ys[2], torsion_g1(d))
    assert nat.lagrange_batch(1, [(xs, ys)])[0] == o.g1_lagrange(xs, ys)
    # a point of order 3 ((0, -2)): the G1 lanes' 4-bit window table meets infinity (3 P = O), so the lane takes the
    # binary ladder; alone and beside honest inputs, and plus a subgroup point
    k3 = bytearray(48)
    k3[47] |= 0x80
    k3 = bytes(k3)
    assert o.g1_valid(k3) and o.g1_mul(k3, o.fr(3)) == bytes(48)
    for ys in ([k3, ys[0], ys[1], ys[3]], [ys[0], o.g1_add(ys[1], k3), k3, ys[3]]):
        assert nat.lagrange_batch(1, [(xs, ys)])[0] == o.g1_lagrange(xs, ys)


# ---------------------------------------------------------------- configs[3]: MSM at 2^20 and 2^24 points
def _msm_known_answer(nat, torch, dev, n, window_bits, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(1, 1 << 63, size=n, dtype=np.uint64)
    s = rng.integers(0, np.iinfo(np.uint64).max, size=(n, 4), dtype=np.uint64, endpoint=True)
    s[:, 3] = rng.integers(0, R >> 192, size=n, dtype=np.uint64)
    ab = np.zeros((n, 4), dtype=np.uint64)
    ab[:, 0] = a
    pts = nat.mul_batch_raw(1, b"", ab.tobytes(), n, generator=True)
    a16 = a.view(np.uint16).reshape(n, 4).astype(np.int64)
    s16 = s.view(np.uint16).reshape(n, 16).astype(np.int64)
    total = 0
    for i in range(4):
        for j in range(16):
            total += int(np.dot(a16[:, i], s16[:, j])) << (16 * (i + j))
    lib = nat.lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    d_in = torch.frombuffer(bytearray(pts), dtype=torch.uint8).to(dev)
    del pts
    d_aff = torch.empty(96 * n, dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_sc = torch.from_numpy(s.view(np.uint8).reshape(-1).copy()).to(dev)
    d_jac = torch.zeros(144, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
    assert lib.lcb_g1_to_affine_dev(d_aff.data_ptr(), d_ok.data_ptr(), d_in.data_ptr(), n, st) == 0
    del d_in
    assert lib.lcb_g1_msm_dev(d_jac.data_ptr(), d_aff.data_ptr(), d_sc.data_ptr(), n, window_bits, st) == 0, \
        nat.last_error()
    assert lib.lcb_g1_jac_sum_dev(d_out.data_ptr(), None, d_jac.data_ptr(), 1, st) == 0
    torch.cuda.synchronize(dev)
    assert bool(d_ok.all().item())
    return bytes(d_out.cpu().numpy().tobytes()), total % R


def test_msm_known_answer_2p20(nat, tdev):
    torch, dev = tdev
    got, exp = _msm_known_answer(nat, torch, dev, 1 << 20, 0, 20)
    assert got == o.g1_mul(o.g1_gen(), o.fr(exp))


def test_msm_known_answer_2p24_c20(nat, tdev):
    torch, dev = tdev
    assert nat.lib().lcb_g1_msm_window(1 << 24) == 20
    got, exp = _msm_known_answer(nat, torch, dev, 1 << 24, 20, 24)
    assert got == o.g1_mul(o.g1_gen(), o.fr(exp))
    torch.cuda.empty_cache()


def test_tpke_verify_beyond_one_chunk(nat, tdev):
    """More shares than one Miller / final-exponentiation launch pair takes (LCB_VERIFY_CHUNK = 2^21): 2,097,280
    shares tiled from 32 known decisions (4 ciphertexts x 8 decryptors with wrong, reversed and off-subgroup
    shares), so chunk boundaries and the park-slot addressing beyond 2^21 items are checked bit-exactly."""
    torch, dev = tdev
    n, f, c = 8, 2, 4
    d = Drbg(b"gpu-verify-chunks")
    xs, y_secret = keyset(d, n, f)
    y = o.g1_mul(o.g1_gen(), o.fr(y_secret))
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    plains = [d.bytes(32) for _ in range(c)]
    cts = [o.tpke_encrypt(y, p, o.fr(d.fr_int())) for p in plains]
    shares = [[o.g1_mul(U, o.fr(x)) for x in xs] for (U, _, _) in cts]
    shares[0][1] = shares[0][2]
    shares[1][3] = shares[1][3][::-1]
    shares[2][5] = off_subgroup_g1(d)
    shares[3][0] = o.g1_add(shares[3][0], shares[3][0])
    base = [s for row in shares for s in row]
    ok = lambda i: o.g1_valid(base[i]) and o.tpke_verify_share(yi[i % n], *cts[i // n], base[i]) == 1
    expect = np.array([ok(i) for i in range(c * n)], dtype=np.uint8)
    assert expect.sum() in (c * n - 4, c * n - 3)
    reps = 65540
    total = reps * c * n
    assert total > (1 << 21)
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_y = up(torch, dev, b"".join(yi))
    d_u = up(torch, dev, b"".join(ct[0] for ct in cts))
    d_w = up(torch, dev, b"".join(ct[2] for ct in cts))
    d_v = up(torch, dev, b"".join(ct[1] for ct in cts))
    d_voff = up(torch, dev, np.arange(0, 32 * (c + 1), 32, dtype=np.uint32))
    d_ct = up(torch, dev, np.tile(np.repeat(np.arange(c, dtype=np.uint32), n), reps))
    d_dec = up(torch, dev, np.tile(np.arange(n, dtype=np.uint32), c * reps))
    d_sh = up(torch, dev, b"".join(base)).repeat(reps)
    d_acc = torch.full((total,), 7, dtype=torch.uint8, device=dev)
    assert lib.lcb_tpke_prepare_dev(d_y.data_ptr(), n, d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(),
                                    d_voff.data_ptr(), c, sh) == 0
    assert lib.lcb_tpke_verify_prepared_dev(d_acc.data_ptr(), total, n, c, d_ct.data_ptr(), d_dec.data_ptr(),
                                            d_sh.data_ptr(), sh) == 0
    torch.cuda.synchronize(dev)
    got = d_acc.cpu().numpy()
    assert np.array_equal(got, np.tile(expect, reps))
