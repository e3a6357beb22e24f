/* oracle/rs.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the Reed–Solomon erasure coding of Lachain's reliable
 * broadcast.
 *
 * Reference: ReliableBroadcast.ErasureCodingShards / DecodeFromEchos
 *   (/root/reference/src/Lachain.Consensus/ReliableBroadcast/ReliableBroadcast.cs:393-446) over
 *   ErasureCoding (ErasureCoding.cs:13: GenericGF(285, 256, 0)), i.e. the "Universal Reed-Solomon Codec"
 *   (ReliableBroadcast/ReedSolomon/README.md: ZXing.Net's encoder + the Wikiversity errata decoder), a git submodule
 *   that is NOT checked out in the reference tree.  Restated from that published algorithm:
 *   - field GF(2^8) with primitive polynomial x^8+x^4+x^3+x^2+1 (0x11D = 285), alpha = 2, generator base 0;
 *   - codeword symbols c_0..c_{n-1}, c_0 the highest-degree coefficient: C(x) = sum_j c_j x^(n-1-j);
 *   - systematic encoding (ZXing ReedSolomonEncoder.Encode): data first, then the remainder of
 *     D(x) x^ecc mod g(x), g(x) = prod_{i<ecc} (x - alpha^i), right-aligned into the ecc symbols;
 *   - erasure decoding (Wikiversity rs_correct_errata with known erasure positions, no unknown errors): syndromes
 *     S_i = R(alpha^i), erasure locator Lambda(x) = prod_e (1 - X_e x) with X_e = alpha^(n-1-pos_e),
 *     Omega = S Lambda mod x^ecc, Forney magnitude e = X Omega(X^-1) / Lambda'(X^-1) (fcr = 0, characteristic 2).
 * Pinned by the README's known answer ("Hello World" + 9 ecc symbols -> 40 86 08 D5 2C AE B5 8F 83) and by
 * test/Lachain.ConsensusTest/ErasureCodingTest.cs's round trip.  With exactly `ecc` erasures the decoded codeword is
 * the unique codeword through the remaining symbols, so any correct erasure decoder gives the same bytes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static uint8_t g_exp[512], g_log[256];
static int g_ready = 0;

static void gf_init(void) {
    if (g_ready) return;
    int x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) g_exp[i] = g_exp[i - 255];
    g_ready = 1;
}
static uint8_t gmul(uint8_t a, uint8_t b) { return (a && b) ? g_exp[g_log[a] + g_log[b]] : 0; }
static uint8_t gdiv(uint8_t a, uint8_t b) { return a ? g_exp[(g_log[a] + 255 - g_log[b]) % 255] : 0; } /* b != 0 */
static uint8_t gpow2(int e) { e %= 255; if (e < 0) e += 255; return g_exp[e]; }                      /* alpha^e */

/* ZXing ReedSolomonEncoder.Encode(cw, ecc) on ints: cw[0..n-ecc) data in, cw[n-ecc..n) ecc out */
int orc_rs_encode_codeword(int *cw, int n, int ecc) {
    gf_init();
    if (ecc <= 0 || ecc >= n) return -1;
    int k = n - ecc;
    uint8_t *g = calloc((size_t)ecc + 1, 1), *rem = calloc((size_t)n, 1);
    if (!g || !rem) { free(g); free(rem); return -1; }
    /* g(x) = prod (x - alpha^i), coefficients highest degree first: g[0] = 1 */
    g[0] = 1;
    for (int i = 0; i < ecc; i++) {
        uint8_t r = gpow2(i);
        for (int j = i + 1; j >= 1; j--) g[j] ^= gmul(g[j - 1], r);
    }
    for (int j = 0; j < k; j++) {
        if (cw[j] < 0 || cw[j] > 255) { free(g); free(rem); return -1; }
        rem[j] = (uint8_t)cw[j];
    }
    /* synthetic division of D(x) x^ecc by the monic g */
    for (int j = 0; j < k; j++) {
        uint8_t coef = rem[j];
        if (coef)
            for (int t = 1; t <= ecc; t++) rem[j + t] ^= gmul(g[t], coef);
    }
    for (int t = 0; t < ecc; t++) cw[k + t] = rem[k + t];
    free(g); free(rem);
    return 0;
}

/* erasure decoding in place: cw (n symbols, erased ones arbitrary), erasure positions pos[0..m), m <= ecc.
   Returns 0, or -1 when the erasure set cannot be solved (two erased positions with the same evaluation point:
   only possible for n > 255). */
int orc_rs_decode_erasures(int *cw, int n, int ecc, const int *pos, int m) {
    gf_init();
    if (m > ecc || m < 0) return -1;
    uint8_t *r = malloc((size_t)n), *S = calloc((size_t)ecc, 1), *L = calloc((size_t)m + 1, 1), *W = calloc((size_t)ecc, 1);
    uint8_t *X = malloc((size_t)m + 1);
    int rc = 0;
    if (!r || !S || !L || !W || !X) { rc = -1; goto out; }
    for (int j = 0; j < n; j++) r[j] = (uint8_t)cw[j];
    for (int e = 0; e < m; e++) r[pos[e]] = 0;
    for (int i = 0; i < ecc; i++) {              /* S_i = R(alpha^i), Horner over c_0 (highest degree) .. c_{n-1} */
        uint8_t a = gpow2(i), acc = 0;
        for (int j = 0; j < n; j++) acc = (uint8_t)(gmul(acc, a) ^ r[j]);
        S[i] = acc;
    }
    L[0] = 1;                                    /* Lambda(x) = prod (1 - X_e x), L[d] = coefficient of x^d */
    for (int e = 0; e < m; e++) {
        X[e] = gpow2(n - 1 - pos[e]);
        for (int d = e + 1; d >= 1; d--) L[d] ^= gmul(L[d - 1], X[e]);
    }
    for (int i = 0; i < ecc; i++) {              /* Omega = S Lambda mod x^ecc */
        uint8_t acc = 0;
        for (int d = 0; d <= m && d <= i; d++) acc ^= gmul(S[i - d], L[d]);
        W[i] = acc;
    }
    for (int e = 0; e < m; e++) {
        uint8_t xi = gdiv(1, X[e]);              /* X^-1 */
        uint8_t om = 0, dl = 0, p = 1;
        for (int i = 0; i < ecc; i++) { om ^= gmul(W[i], p); p = gmul(p, xi); }
        p = 1;                                   /* Lambda'(x) = sum of odd-degree terms L[d] x^(d-1) */
        for (int d = 1; d <= m; d++) { if (d & 1) dl ^= gmul(L[d], p); p = gmul(p, xi); }
        if (!dl) { rc = -1; goto out; }
        r[pos[e]] = gdiv(gmul(X[e], om), dl);
    }
    for (int j = 0; j < n; j++) cw[j] = r[j];
out:
    free(r); free(S); free(L); free(W); free(X);
    return rc;
}

/* ReliableBroadcast.ErasureCodingShards(input, shards, erasures) (ReliableBroadcast.cs:393-419): out = shards x S bytes */
int orc_rs_encode_shards(uint8_t *out, const uint8_t *input, size_t len, int shards, int erasures) {
    int k = shards - erasures;
    if (k <= 0 || len % (size_t)k) return -1;
    size_t S = len / (size_t)k;
    memcpy(out, input, len);
    if (erasures == 0) return 0;
    int *cw = malloc(sizeof(int) * (size_t)shards);
    if (!cw) return -1;
    for (size_t i = 0; i < S; i++) {
        for (int j = 0; j < k; j++) cw[j] = input[i + (size_t)j * S];
        if (orc_rs_encode_codeword(cw, shards, erasures)) { free(cw); return -1; }
        for (int j = k; j < shards; j++) out[(size_t)j * S + i] = (uint8_t)cw[j];
    }
    free(cw);
    return 0;
}
/* ReliableBroadcast.DecodeFromEchos (ReliableBroadcast.cs:421-446): echo e carries shard from[e]; out = shards x S */
int orc_rs_decode_shards(uint8_t *out, const uint8_t *echo_data, const int32_t *from, int n_echos, size_t S, int shards,
                         int erasures) {
    memset(out, 0, (size_t)shards * S);
    char *have = calloc((size_t)shards, 1);
    int *cw = malloc(sizeof(int) * (size_t)shards), *pos = malloc(sizeof(int) * (size_t)shards);
    int rc = 0, m = 0;
    if (!have || !cw || !pos) { rc = -1; goto out; }
    for (int e = 0; e < n_echos; e++) {
        if (from[e] < 0 || from[e] >= shards) { rc = -1; goto out; }
        memcpy(out + (size_t)from[e] * S, echo_data + (size_t)e * S, S);
        have[from[e]] = 1;
    }
    if (erasures == 0) goto out;
    for (int j = 0; j < shards; j++) if (!have[j]) pos[m++] = j;
    for (size_t i = 0; i < S && rc == 0; i++) {
        for (int j = 0; j < shards; j++) cw[j] = out[i + (size_t)j * S];
        rc = orc_rs_decode_erasures(cw, shards, erasures, pos, m);
        for (int j = 0; j < shards; j++) out[i + (size_t)j * S] = (uint8_t)cw[j];
    }
out:
    free(have); free(cw); free(pos);
    return rc;
}
