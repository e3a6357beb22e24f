"""Register-spill and scratch gate for the built library (CPU test; no GPU needed).

Reads every kernel's code-object metadata (tools/kernel_resources.py: .vgpr_spill_count, .private_segment_fixed_size)
and fails when a kernel spills more VGPRs, or uses more per-lane scratch, than its budget below.  Kernels not listed
must not spill at all.  The budgets are the figures of the current build: a change that adds spills to a kernel has to
lower another figure or justify the new budget here.  The cooperative pairing kernels (k_coop.hip), the batch-check
bookkeeping kernels and the MSM / ECDSA hot loops are held at zero spills.
"""
import os
import shutil

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "lachain_amd", "liblachain_bls.so")

# kernel: (max VGPR spills, max scratch bytes per lane) — measured on this build
BUDGET = {
    "k_lineset_coop_2w": (270, 1080),         # k_prep.hip: the fused census's line sets at 256 registers
    "k_coop_debug": (204, 7620),              # test hook: the one-lane reference routines beside the coop ones
    "k_coop_final_exp_check": (36, 576),
    "k_coop_final_exp_check_2w": (36, 576),   # k_prep.hip: 248 registers (every batched level); census copies at 256
    "k_ts_rlc_sum2": (20, 2464),              # k_prep.hip: two lanes per group
    "k_ts_rlc_sum_census": (34, 2336),
    "k_ts_rlc_miller_census": (2, 4180),     # round 5: three quads saved around the one binary-GCD call per check
    "k_coop_tpke_miller": (0, 0),
    "k_dkg_exact_combine": (0, 312),
    "k_dkg_exact_terms": (0, 408),
    "k_dkg_horner": (0, 896),
    "k_dkg_rows": (0, 312),
    "k_final_exp_check": (2, 3880),          # round 5: the asm Fp12 products clobber a0..a215 (2 spills around the calls)
    "k_g1_decompress": (0, 800),
    "k_g1_jac_compress": (0, 704),
    "k_g1_jac_reduce_block": (0, 456),
    "k_g1_jac_reduce_groups": (0, 168),
    "k_g1_mul": (0, 1040),
    "k_g1_mul_lanes": (0, 896),
    "k_g1_subgroup_any": (24, 0),
    "k_g1_sum": (0, 752),
    "k_g1_to_affine": (0, 704),
    "k_g2_decompress": (0, 992),
    "k_g2_hash": (0, 3400),
    "k_g2_mul": (288, 1272),                  # 4-bit window, table in the lanetab workspace (was 10,624 B)
    "k_g2_mul2_lanes": (3506, 1768),          # paired GLS ladders, tables in the lanetab workspace (was 22,672 B of scratch)
    "k_g2_mul_lanes": (856, 952),           # GLS ladder, table in the lanetab workspace (was 10,288 B)
    "k_g2_sum": (192, 488),
    "k_lineset_coop": (86, 280),              # five-lane line sets (latency path): T, Q, acc and five products live
    "k_lineset_fill": (0, 984),
    "k_mcl_from_bytes": (0, 800),
    "k_mcl_g1_sum": (0, 168),
    "k_mcl_g1_terms": (0, 880),
    "k_mcl_g1_terms_wide": (12, 312),         # round 6: G1 EvaluatePolynomial's 384-bit terms (the 12-word scalar live)
    "k_mcl_g2_hash": (168, 3400),             # mclBnG2_hashAndMapTo's map (SHA-512, calcBN) on one lane
    "k_mcl_g2_clear": (564, 1108),            # round 6: its cofactor clearing on four-lane groups (Fp2 point rounds at 512 registers)
    "k_mcl_horner": (0, 1320),
    "k_mcl_to_bytes": (0, 1024),
    "k_msm_bucket_fix": (0, 168),
    "k_msm_bucket_reduce": (0, 744),          # + the prefetched next bucket
    "k_msm_horner": (0, 168),
    "k_op_debug": (96, 6956),
    "k_op_grp": (372, 4008),                  # round 6: the exponentiation routine's table in VGPRs (lcb_r_fp_pow)
    "k_op_gt": (1788, 8148),                  # single-lane mcl operations (one wave per dispatch), one kernel per family
    "k_op_pair": (842, 7620),
    "k_ptmul_g2_multi": (36, 68),             # round 6: G2 Lagrange / EvaluatePolynomial terms, 16 ladders per block
    "k_ptmul_g2": (36, 68),                   # mcl G2 multiplication latency kernel: four ladder lanes share each op (signed digits: 34)
    "k_rlc_key_tables": (12, 168),            # k_rlc_rand.hip: spills to scratch, not AGPRs (<= 256 registers)
    "k_rlc_miller_fallback": (0, 2376),
    "k_rlc_search": (106, 4056),              # round 5: baby-step giant-step (fingerprint table + the confirming power)
    "k_secp_scalars": (0, 528),
    "k_tpke_ct_prepare": (0, 3800),
    "k_tpke_ct_prepare_h": (5, 4800),
    "k_tpke_ct_prepare_w": (5, 1208),
    "k_tpke_ct_prepare_hw": (8, 4800),        # round 6: both lane kinds in one dispatch (fork mode 4)
    "k_tpke_encrypt1": (0, 1184),
    "k_tpke_encrypt2": (0, 3976),
    "k_tpke_exact_points": (0, 704),
    "k_tpke_miller": (0, 2376),          # round 5: the two-pair loop in assembly (lcb_r_miller2); scratch = the fallback path
    "k_tpke_pd_miller": (962, 2664),          # partial decryption split in three (was k_tpke_partial_decrypt, 7,652 B)
    "k_tpke_pd_mul": (0, 992),
    "k_tpke_rlc_miller": (0, 2376),          # round 5: the two-pair loop in assembly (lcb_r_miller2); scratch = the fallback path
    "k_tpke_rlc_points": (0, 664),            # k_rlc_rand.hip: 248 registers, two waves per SIMD (round 6: 60 -> 0 spills)
    "k_tpke_rlc_search2a": (97, 3448),        # level-2 searches: four Fp12 values per lane, four lanes per group
    "k_tpke_rlc_search2b": (0, 3656),
    "k_tpke_rlc_search2b_asm": (0, 0),        # round 6: the two-error search on the assembly Fp12 products (park slots)
    "k_tpke_rlc_sum": (0, 1168),
    "k_tpke_rlc_wsum": (48, 576),             # round 6: binary-GCD conversions; the live record saved around the calls
    "k_tpke_rlc_wsum2": (0, 648),
    "k_ts_miller": (1248, 3292),
    "k_ts_msg_prepare": (5, 4800),            # round 5: k_prep.hip at 256 registers (was 346, 0 spills, 3,688 B)
    "k_ts_rlc_miller": (0, 2524),
    "k_ts_rlc_points": (396, 1960),           # k_rlc_rand.hip: 256 registers, two waves per SIMD (round 6: 677 -> 396; G2 addends in the record)
    "k_ts_rlc_sum": (26, 2136),               # round 5: binary-GCD affine conversions (spills around the two calls)
    "k_ts_rlc_wsum": (96, 992),               # round 5: binary-GCD affine conversions
    "k_ts_sign": (0, 3976),
}
# Round 5: no kernel that runs on more than one wave may take more than 4 KB of scratch per lane — the
# HIP runtime reserves a dispatch's scratch for min(waves, device wave slots) waves per hardware queue, and the 22.7 KB
# paired G2 lanes aborted processes with HSA_STATUS_ERROR_OUT_OF_RESOURCES.  The single-lane kernels below run one wave.
SCRATCH_CAP = 4096
SINGLE_WAVE = {"k_op_grp", "k_op_pair", "k_op_gt", "k_op_debug", "k_coop_debug"}
# one lane per ciphertext (748 waves for configs[1]'s 1M shares: a 222 MB reservation at 4.6 KB per lane), at 256
# registers so a wave shares its SIMD with a randomisation wave (k_prep.hip)
PER_CIPHERTEXT = {"k_tpke_ct_prepare_h": 4900, "k_tpke_ct_prepare_hw": 4900, "k_ts_msg_prepare": 4900,   # (the same hash lane, one per message)
                  "k_ts_rlc_miller_census": 4200}   # the census's <= 1,024 lanes (16 waves: a 4.3 MB reservation)
ZERO_SPILL = ["k_coop_tpke_miller", "k_tpke_rlc_points", "k_msm_bucket_acc", "k_secp_verify",
              "k_rlc_census_stats", "k_rlc_suspect_split", "k_rlc_resolve", "k_tpke_rlc_sum", "k_ts_rlc_miller"]


@pytest.fixture(scope="module")
def resources():
    if not os.path.exists(SO):
        pytest.skip("liblachain_bls.so not built")
    if not shutil.which("llvm-objdump", path="/opt/rocm/lib/llvm/bin"):
        pytest.skip("llvm-objdump not available")
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import kernel_resources
    return kernel_resources(SO)


def test_every_kernel_within_its_spill_and_scratch_budget(resources):
    over = []
    for name, r in resources.items():
        if name.startswith("lcb_asm_") or name.startswith("_Z"):      # asm-library stubs, hipCUB sort kernels
            continue
        spill, scratch = BUDGET.get(name, (0, None))
        if r["vgpr_spill_count"] > spill:
            over.append((name, "vgpr_spill", r["vgpr_spill_count"], spill))
        if scratch is not None and r["private_segment_fixed_size"] > scratch:
            over.append((name, "scratch", r["private_segment_fixed_size"], scratch))
    assert not over, over


def test_hot_kernels_do_not_spill(resources):
    for name in ZERO_SPILL:
        assert name in resources, name
        assert resources[name]["vgpr_spill_count"] == 0, name


def test_multi_wave_kernels_within_4kb_scratch(resources):
    over = [(n, r["private_segment_fixed_size"]) for n, r in resources.items()
            if not n.startswith(("lcb_asm_", "_Z")) and n not in SINGLE_WAVE
            and r["private_segment_fixed_size"] > PER_CIPHERTEXT.get(n, SCRATCH_CAP)]
    assert not over, over


def test_every_kernel_fits_the_gate_reserve(resources):
    """the gate queue binds at most LCB_GATE_RESERVE (4.5 GiB, lcb_host.cpp): every kernel's full-device scratch
    (per lane rounded to 16 B x 64 lanes x 256 CUs x 32 wave slots, the runtime's request) must fit it"""
    reserve = 9 << 29
    over = []
    for k, r in resources.items():
        full = ((r.get("private_segment_fixed_size", 0) + 15) // 16 * 16) * 64 * 256 * 32
        if full > reserve:
            over.append((k, full))
    assert not over, over
