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
