"""GPU parity of the batched CommonCoin path (BASELINE configs[2]) against the oracle: ValidateSignature for
every share (ThresholdSignature/PublicKey.cs:16-21), ThresholdSigner.AddShare's assembly over the first F+1
valid shares in index order (ThresholdSigner.cs:62-75, PublicKeySet.cs:34-42) and the combined signature's
validation against the shared key.  Bit-exact: accept bitmaps and serialized G2 signatures.
"""
import numpy as np
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


def coin_id(era, agreement, epoch):
    return era.to_bytes(8, "little") + agreement.to_bytes(8, "little") + epoch.to_bytes(8, "little")


def test_ts_rounds_verify_assemble_combined(nat):
    import torch
    dev = torch.device("cuda", 0)
    n, f, rounds = 7, 2, 4
    d = Drbg(b"gpu-ts-rounds")
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    sks = [poly(i + 1) for i in range(n)]
    pks = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in sks] + [o.g1_mul(o.g1_gen(), o.fr(poly(0)))]
    msgs = [coin_id(3, r, 5) for r in range(rounds)]
    sigs = [[o.ts_sign(o.fr(sks[i]), msgs[r]) for i in range(n)] for r in range(rounds)]
    # round 1: shares 0 and 2 carry other shares' signatures; round 2: only 2 valid shares (< F+1);
    # round 3: share 5 is doubled (a valid G2 point, wrong signature)
    sigs[1][0], sigs[1][2] = sigs[1][1], sigs[1][3]
    for i in range(n):
        if i not in (4, 6):
            sigs[2][i] = sigs[2][(i + 1) % n]
    sigs[3][5] = o.g2_add(sigs[3][5], sigs[3][5])
    flat = [s for row in sigs for s in row]
    expect = [o.ts_validate(pks[i % n], flat[i], msgs[i // n]) == 1 for i in range(rounds * n)]
    assert sum(expect[2 * n:3 * n]) == 2 and not expect[n] and not expect[n + 2] and not expect[3 * n + 5]

    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_pks, d_msg = t(b"".join(pks)), t(b"".join(msgs))
    d_moff = t(np.arange(0, 24 * (rounds + 1), 24, dtype=np.uint32).tobytes())
    d_sigs = t(b"".join(flat))
    d_midx = t(np.repeat(np.arange(rounds, dtype=np.uint32), n).tobytes())
    d_pidx = t(np.tile(np.arange(n, dtype=np.uint32), rounds).tobytes())
    d_acc = torch.zeros(rounds * n, dtype=torch.uint8, device=dev)
    d_comb = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_cacc = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_ridx = t(np.arange(rounds, dtype=np.uint32).tobytes())
    d_shared = t(np.full(rounds, n, dtype=np.uint32).tobytes())
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    assert lib.lcb_ts_prepare_dev(d_pks.data_ptr(), n + 1, d_msg.data_ptr(), d_moff.data_ptr(), rounds, sh) == 0
    assert lib.lcb_ts_verify_prepared_dev(d_acc.data_ptr(), rounds * n, n + 1, rounds, d_sigs.data_ptr(),
                                          d_midx.data_ptr(), d_pidx.data_ptr(), sh) == 0
    assert lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(), d_sigs.data_ptr(), n,
                                   f + 1, rounds, sh) == 0
    assert lib.lcb_ts_verify_prepared_dev(d_cacc.data_ptr(), rounds, n + 1, rounds, d_comb.data_ptr(),
                                          d_ridx.data_ptr(), d_shared.data_ptr(), sh) == 0
    torch.cuda.synchronize(dev)
    assert [bool(x) for x in d_acc.cpu().numpy()] == expect
    st = d_cst.cpu().numpy().tolist()
    assert st == [1, 1, 0, 1]
    comb = d_comb.cpu().numpy().tobytes()
    for r in (0, 1, 3):
        # the oracle's own AssembleSignature over the first F+1 valid shares, and the shared-key signature
        valid = [i for i in range(n) if expect[r * n + i]][:f + 1]
        xs = [o.fr(i + 1) for i in valid]
        ys = [sigs[r][i] for i in valid]
        assert comb[96 * r:96 * r + 96] == o.g2_lagrange(xs, ys)
        assert comb[96 * r:96 * r + 96] == o.ts_sign(o.fr(poly(0)), msgs[r])
    assert d_cacc.cpu().numpy().tolist() == [1, 1, 0, 1]


def test_tpke_partial_decrypt_and_combine_dev(nat):
    """TPKE Decrypt with one secret per ciphertext (lcb_tpke_partial_decrypt_prepared_dev) and FullDecrypt's
    combination over the first F+1 valid shares (lcb_tpke_combine_dev), checked against the oracle's
    tpke_decrypt / tpke_full_decrypt (TPKE/PrivateKey.cs:21-31, TPKE/PublicKey.cs:55-86)."""
    import torch
    dev = torch.device("cuda", 0)
    n, f = 4, 1
    d = Drbg(b"gpu-tpke-combine")
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    xs = [poly(i + 1) for i in range(n)]
    y = o.g1_mul(o.g1_gen(), o.fr(poly(0)))
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    plains = [b"epoch replay payload %02d........" % c for c in range(3)]
    cts = [o.tpke_encrypt(y, p, o.fr(d.fr_int())) for p in plains]
    # shares[c][j] by DecryptorId; ciphertext 1 loses decryptor 0 (corrupted), ciphertext 2 keeps one valid share
    shares = [[o.tpke_decrypt(U, V, W, o.fr(xs[j])) for j in range(n)] for (U, V, W) in cts]
    shares[1][0] = o.g1_add(shares[1][0], o.g1_gen())
    for j in (0, 1, 2):
        shares[2][j] = o.g1_add(shares[2][j], o.g1_gen())
    flat = [s for row in shares for s in row]
    accept = [o.tpke_verify_share(yi[i % n], *cts[i // n], flat[i]) == 1 for i in range(len(flat))]
    t = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_y = t(b"".join(yi))
    d_u = t(b"".join(c[0] for c in cts))
    d_w = t(b"".join(c[2] for c in cts))
    d_v = t(b"".join(c[1] for c in cts))
    d_voff = t(np.cumsum([0] + [len(c[1]) for c in cts]).astype(np.uint32).tobytes())
    assert lib.lcb_tpke_prepare_dev(d_y.data_ptr(), n, d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(),
                                    d_voff.data_ptr(), len(cts), sh) == 0
    # decryptor 2 decrypts ciphertexts 0 and 2, decryptor 3 ciphertext 1
    who = [2, 3, 2]
    d_x = t(b"".join(o.fr(xs[j]) for j in who))
    d_ui = torch.zeros(48 * len(cts), dtype=torch.uint8, device=dev)
    d_st = torch.zeros(len(cts), dtype=torch.uint8, device=dev)
    assert lib.lcb_tpke_partial_decrypt_prepared_dev(d_ui.data_ptr(), d_st.data_ptr(), d_x.data_ptr(), 1,
                                                     d_u.data_ptr(), len(cts), sh) == 0
    d_acc = t(bytes(int(a) for a in accept))
    d_sh = t(b"".join(flat))
    d_out = torch.zeros(48 * len(cts), dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(len(cts), dtype=torch.uint8, device=dev)
    assert lib.lcb_tpke_combine_dev(d_out.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(), d_sh.data_ptr(), n,
                                    f + 1, len(cts), sh) == 0
    torch.cuda.synchronize(dev)
    ui = d_ui.cpu().numpy().tobytes()
    assert d_st.cpu().numpy().tolist() == [1, 1, 1]
    for c, j in enumerate(who):
        assert ui[48 * c:48 * c + 48] == o.tpke_decrypt(*cts[c], o.fr(xs[j]))
    assert d_cst.cpu().numpy().tolist() == [1, 1, 0]
    u = d_out.cpu().numpy().tobytes()
    for c in (0, 1):
        valid = [j for j in range(n) if accept[c * n + j]][:f + 1]
        assert o.xor_with_hash(u[48 * c:48 * c + 48], cts[c][1]) == plains[c]
        assert o.tpke_full_decrypt(cts[c][1], valid, [shares[c][j] for j in valid]) == plains[c]
