// lachain_amd/csrc/ops.h — operation codes of the single-operation kernel (k_ops.hip)
#pragma once
enum {
    OP_FR_FROM_RAW = 1, OP_FR_TO_RAW, OP_FR_ADD, OP_FR_SUB, OP_FR_MUL, OP_FR_INV, OP_FR_NEG,
    OP_G1_DESER = 20, OP_G1_SER, OP_G1_ADD, OP_G1_DBL, OP_G1_NEG, OP_G1_MUL, OP_G1_EQ, OP_G1_VALID, OP_G1_NORM,
    OP_G2_DESER = 40, OP_G2_SER, OP_G2_ADD, OP_G2_DBL, OP_G2_NEG, OP_G2_MUL, OP_G2_EQ, OP_G2_VALID, OP_G2_NORM,
    OP_G2_HASH,
    OP_PAIRING = 60, OP_MILLER, OP_FINAL_EXP, OP_GT_MUL, OP_GT_POW, OP_GT_EQ, OP_GT_SER, OP_GT_DESER,
    OP_DEBUG_FP12 = 90, /* io[548] selects a tower routine applied to io[252..396) (tools/debug) */
    OP_G1_GEN = 80, OP_G2_GEN
};
