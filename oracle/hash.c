/*
 * oracle/hash.c — TEST INFRASTRUCTURE ONLY (see bls_oracle.h).
 * SHA-256 / SHA-512 (FIPS 180-4), SHA3-256 (FIPS 202) and the BouncyCastle 1.8.8
 * DigestRandomGenerator(Sha3Digest) keystream used by Lachain's TPKE KDF
 * (/root/reference/src/Lachain.Crypto/TPKE/Utils.cs:12-19; KAT CryptographyTest.cs:103-113).
 */
#include <stdint.h>
#include <string.h>
#include "bls_oracle.h"

typedef uint64_t u64;
typedef uint32_t u32;

/* ------------------------------------------------------------------ SHA-256 */
static const u32 K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(u32 h[8], const uint8_t *b) {
    u32 w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((u32)b[4 * i] << 24) | ((u32)b[4 * i + 1] << 16) | ((u32)b[4 * i + 2] << 8) | b[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        u32 s0 = ROR32(w[i - 15], 7) ^ ROR32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        u32 s1 = ROR32(w[i - 2], 17) ^ ROR32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    u32 a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        u32 S1 = ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25);
        u32 ch = (e & f) ^ (~e & g);
        u32 t1 = hh + S1 + ch + K256[i] + w[i];
        u32 S0 = ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22);
        u32 mj = (a & bb) ^ (a & c) ^ (bb & c);
        u32 t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
void orc_sha256(uint8_t out[32], const uint8_t *m, size_t n) {
    u32 h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t i = 0;
    for (; i + 64 <= n; i += 64) sha256_block(h, m + i);
    uint8_t buf[128];
    size_t rem = n - i;
    memset(buf, 0, sizeof buf);
    memcpy(buf, m + i, rem);
    buf[rem] = 0x80;
    size_t tot = (rem + 9 <= 64) ? 64 : 128;
    u64 bits = (u64)n * 8;
    for (int k = 0; k < 8; k++) buf[tot - 1 - k] = (uint8_t)(bits >> (8 * k));
    sha256_block(h, buf);
    if (tot == 128) sha256_block(h, buf + 64);
    for (int k = 0; k < 8; k++) {
        out[4 * k] = h[k] >> 24; out[4 * k + 1] = h[k] >> 16; out[4 * k + 2] = h[k] >> 8; out[4 * k + 3] = h[k];
    }
}

/* ------------------------------------------------------------------ SHA-512 */
static const u64 K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))
static void sha512_block(u64 h[8], const uint8_t *b) {
    u64 w[80];
    for (int i = 0; i < 16; i++) {
        u64 v = 0;
        for (int k = 0; k < 8; k++) v = (v << 8) | b[8 * i + k];
        w[i] = v;
    }
    for (int i = 16; i < 80; i++) {
        u64 s0 = ROR64(w[i - 15], 1) ^ ROR64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        u64 s1 = ROR64(w[i - 2], 19) ^ ROR64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    u64 a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 80; i++) {
        u64 S1 = ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41);
        u64 ch = (e & f) ^ (~e & g);
        u64 t1 = hh + S1 + ch + K512[i] + w[i];
        u64 S0 = ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39);
        u64 mj = (a & bb) ^ (a & c) ^ (bb & c);
        u64 t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
void orc_sha512(uint8_t out[64], const uint8_t *m, size_t n) {
    u64 h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    size_t i = 0;
    for (; i + 128 <= n; i += 128) sha512_block(h, m + i);
    uint8_t buf[256];
    size_t rem = n - i;
    memset(buf, 0, sizeof buf);
    memcpy(buf, m + i, rem);
    buf[rem] = 0x80;
    size_t tot = (rem + 17 <= 128) ? 128 : 256;
    u64 bits = (u64)n * 8;
    for (int k = 0; k < 8; k++) buf[tot - 1 - k] = (uint8_t)(bits >> (8 * k));
    sha512_block(h, buf);
    if (tot == 256) sha512_block(h, buf + 128);
    for (int k = 0; k < 8; k++)
        for (int j = 0; j < 8; j++) out[8 * k + j] = (uint8_t)(h[k] >> (56 - 8 * j));
}

/* ------------------------------------------------------------------ SHA3-256 (Keccak-f[1600]) */
static const u64 KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static void keccakf(u64 s[25]) {
    for (int round = 0; round < 24; round++) {
        u64 C[5], D[5], B[25];
        for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ ((C[(x + 1) % 5] << 1) | (C[(x + 1) % 5] >> 63));
        for (int i = 0; i < 25; i++) s[i] ^= D[i % 5];
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) {
                int r = KROT[x + 5 * y];
                u64 v = s[x + 5 * y];
                B[y + 5 * ((2 * x + 3 * y) % 5)] = r ? ((v << r) | (v >> (64 - r))) : v;
            }
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++)
                s[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
        s[0] ^= KRC[round];
    }
}
typedef struct { u64 s[25]; size_t pos; } sha3_ctx;
static void sha3_init(sha3_ctx *c) { memset(c, 0, sizeof *c); }
static void sha3_update(sha3_ctx *c, const uint8_t *m, size_t n) {
    const size_t rate = 136;
    for (size_t i = 0; i < n; i++) {
        c->s[c->pos / 8] ^= (u64)m[i] << (8 * (c->pos % 8));
        if (++c->pos == rate) { keccakf(c->s); c->pos = 0; }
    }
}
static void sha3_final(sha3_ctx *c, uint8_t out[32]) {
    const size_t rate = 136;
    c->s[c->pos / 8] ^= (u64)0x06 << (8 * (c->pos % 8));
    c->s[(rate - 1) / 8] ^= (u64)0x80 << (8 * ((rate - 1) % 8));
    keccakf(c->s);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(c->s[i / 8] >> (8 * (i % 8)));
    sha3_init(c);
}
void orc_sha3_256(uint8_t out[32], const uint8_t *m, size_t n) {
    sha3_ctx c;
    sha3_init(&c);
    sha3_update(&c, m, n);
    sha3_final(&c, out);
}

/* original Keccak-256 (domain byte 0x01, BouncyCastle KeccakDigest(256) behind HashUtils.KeccakBytes,
   src/Lachain.Crypto/HashUtils.cs:30-38) */
void orc_keccak256(uint8_t out[32], const uint8_t *m, size_t n) {
    const size_t rate = 136;
    sha3_ctx c;
    sha3_init(&c);
    sha3_update(&c, m, n);
    c.s[c.pos / 8] ^= (u64)0x01 << (8 * (c.pos % 8));
    c.s[(rate - 1) / 8] ^= (u64)0x80 << (8 * ((rate - 1) % 8));
    keccakf(c.s);
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(c.s[i / 8] >> (8 * (i % 8)));
}

/* HashUtils.Keccak(BlockHeader) (HashUtils.cs:40-53): Keccak-256 of the RLP list [PrevBlockHash, StateHash,
   MerkleRoot, Index, Nonce] with the hashes as their 32 raw bytes and Index / Nonce as 8 little-endian bytes
   (ulong.ToBytes, SerialiaztionUtils.cs:210-213); Nethereum RLP: 0xa0 || 32 B, 0x88 || 8 B, list 0xf8 0x75 || 117 B */
void orc_header_keccak(uint8_t out[32], const uint8_t prev[32], const uint8_t state[32], const uint8_t merkle[32],
                       uint64_t index, uint64_t nonce) {
    uint8_t b[119], *q = b;
    *q++ = 0xf8; *q++ = 0x75;
    const uint8_t *h[3] = {prev, state, merkle};
    for (int i = 0; i < 3; i++) { *q++ = 0xa0; memcpy(q, h[i], 32); q += 32; }
    uint64_t v[2] = {index, nonce};
    for (int i = 0; i < 2; i++) {
        *q++ = 0x88;
        for (int j = 0; j < 8; j++) *q++ = (uint8_t)(v[i] >> (8 * j));
    }
    orc_keccak256(out, b, sizeof b);
}

/* BouncyCastle DigestRandomGenerator (Org.BouncyCastle.Crypto.Prng), CYCLE_COUNT = 10 */
typedef struct { uint8_t seed[32], state[32]; int64_t seed_ctr, state_ctr; } drg_t;
static void drg_add_counter(sha3_ctx *c, int64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) { b[i] = (uint8_t)v; v >>= 8; }
    sha3_update(c, b, 8);
}
static void drg_cycle_seed(drg_t *g) {
    sha3_ctx c; sha3_init(&c);
    sha3_update(&c, g->seed, 32);
    drg_add_counter(&c, g->seed_ctr++);
    sha3_final(&c, g->seed);
}
static void drg_generate_state(drg_t *g) {
    sha3_ctx c; sha3_init(&c);
    drg_add_counter(&c, g->state_ctr++);
    sha3_update(&c, g->state, 32);
    sha3_update(&c, g->seed, 32);
    sha3_final(&c, g->state);
    if ((g->state_ctr % 10) == 0) drg_cycle_seed(g);
}
void orc_xor_with_hash(uint8_t *out, const uint8_t g1[48], const uint8_t *data, size_t len) {
    drg_t g;
    memset(&g, 0, sizeof g);
    g.seed_ctr = 1; g.state_ctr = 1;
    /* AddSeedMaterial(inSeed): seed = H(inSeed || seed) */
    sha3_ctx c; sha3_init(&c);
    sha3_update(&c, g1, 48);
    sha3_update(&c, g.seed, 32);
    sha3_final(&c, g.seed);
    /* NextBytes */
    size_t off = 0;
    drg_generate_state(&g);
    for (size_t i = 0; i < len; i++) {
        if (off == 32) { drg_generate_state(&g); off = 0; }
        out[i] = data[i] ^ g.state[off++];
    }
}

/* generic-seed variant used only by the KAT test (CryptographyTest.cs:103-113 seeds with 4 bytes) */
void orc_drg_bytes(uint8_t *out, size_t len, const uint8_t *seed, size_t seedlen) {
    drg_t g;
    memset(&g, 0, sizeof g);
    g.seed_ctr = 1; g.state_ctr = 1;
    sha3_ctx c; sha3_init(&c);
    sha3_update(&c, seed, seedlen);
    sha3_update(&c, g.seed, 32);
    sha3_final(&c, g.seed);
    size_t off = 0;
    drg_generate_state(&g);
    for (size_t i = 0; i < len; i++) {
        if (off == 32) { drg_generate_state(&g); off = 0; }
        out[i] = g.state[off++];
    }
}

/* ---- CommonCoin consumers of the combined signature bytes (row a13) ----
   CoinResult.Parity (src/Lachain.Consensus/CommonCoin/CoinResult.cs:16-20):
     p = RawBytes.Aggregate(0u, (i, b) => i ^ b); return Popcount(p) % 2 == 1   (BitsUtils.Popcount)
   RootProtocol.GetNonceFromCoin (src/Lachain.Consensus/RootProtocol/RootProtocol.cs:316-322):
     res[i % 8] ^= RawBytes[i]; return res.ToUInt64()  (little-endian, SerialiaztionUtils.cs:256-259) */
int orc_coin_parity(const uint8_t *bytes, size_t len) {
    uint32_t p = 0;
    for (size_t i = 0; i < len; i++) p ^= bytes[i];
    /* BitsUtils.Popcount, restated */
    p -= p >> 1 & 0x55555555u;
    p = (p & 0x33333333u) + (p >> 2 & 0x33333333u);
    p = (p + (p >> 4)) & 0x0f0f0f0fu;
    p += p >> 8;
    p += p >> 16;
    return (int)((p & 0x7f) % 2 == 1);
}
uint64_t orc_coin_nonce(const uint8_t *bytes, size_t len) {
    uint8_t res[8] = {0};
    for (size_t i = 0; i < len; i++) res[i % 8] ^= bytes[i];
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v |= (uint64_t)res[j] << (8 * j);
    return v;
}
