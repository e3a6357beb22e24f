// lachain_amd/csrc/host_sha3.hpp — host-side SHA3-256 and the BouncyCastle 1.8.8
// DigestRandomGenerator(Sha3Digest) keystream behind Lachain's TPKE Utils.XorWithHash
// (/root/reference/src/Lachain.Crypto/TPKE/Utils.cs:12-19; KAT test/Lachain.CryptoTest/CryptographyTest.cs:103-113).
// Pure byte work on the host (one 48-byte seed + |V| output bytes per ciphertext).
#pragma once
#include <stdint.h>
#include <string.h>

namespace lcb_host {

struct Sha3 {
    uint64_t s[25];
    size_t pos;
    Sha3() { reset(); }
    void reset() { memset(s, 0, sizeof s); pos = 0; }
    static void f1600(uint64_t st[25]) {
        static const uint64_t RC[24] = {
            0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
            0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
            0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
            0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
            0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
            0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
        static const int RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
        for (int r = 0; r < 24; r++) {
            uint64_t c[5], b[25];
            for (int x = 0; x < 5; x++) c[x] = st[x] ^ st[x + 5] ^ st[x + 10] ^ st[x + 15] ^ st[x + 20];
            for (int x = 0; x < 5; x++) {
                uint64_t d = c[(x + 4) % 5] ^ ((c[(x + 1) % 5] << 1) | (c[(x + 1) % 5] >> 63));
                for (int y = 0; y < 25; y += 5) st[x + y] ^= d;
            }
            for (int x = 0; x < 5; x++)
                for (int y = 0; y < 5; y++) {
                    uint64_t v = st[x + 5 * y];
                    int n = RHO[x + 5 * y];
                    b[y + 5 * ((2 * x + 3 * y) % 5)] = n ? (v << n) | (v >> (64 - n)) : v;
                }
            for (int x = 0; x < 5; x++)
                for (int y = 0; y < 5; y++)
                    st[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
            st[0] ^= RC[r];
        }
    }
    void update(const uint8_t *m, size_t n) {
        for (size_t i = 0; i < n; i++) {
            s[pos >> 3] ^= (uint64_t)m[i] << (8 * (pos & 7));
            if (++pos == 136) { f1600(s); pos = 0; }
        }
    }
    void final(uint8_t out[32]) {
        s[pos >> 3] ^= (uint64_t)0x06 << (8 * (pos & 7));
        s[135 >> 3] ^= (uint64_t)0x80 << (8 * (135 & 7));
        f1600(s);
        for (int i = 0; i < 32; i++) out[i] = (uint8_t)(s[i >> 3] >> (8 * (i & 7)));
        reset();
    }
};

// Org.BouncyCastle.Crypto.Prng.DigestRandomGenerator with Sha3Digest(256); CYCLE_COUNT = 10
struct DigestRandom {
    uint8_t seed[32], state[32];
    int64_t seed_ctr = 1, state_ctr = 1;
    DigestRandom() { memset(seed, 0, 32); memset(state, 0, 32); }
    static void add_counter(Sha3 &h, int64_t v) {
        uint8_t b[8];
        for (int i = 0; i < 8; i++) { b[i] = (uint8_t)v; v >>= 8; }
        h.update(b, 8);
    }
    void add_seed(const uint8_t *m, size_t n) {
        Sha3 h;
        h.update(m, n);
        h.update(seed, 32);
        h.final(seed);
    }
    void generate_state() {
        Sha3 h;
        add_counter(h, state_ctr++);
        h.update(state, 32);
        h.update(seed, 32);
        h.final(state);
        if (state_ctr % 10 == 0) {
            Sha3 c;
            c.update(seed, 32);
            add_counter(c, seed_ctr++);
            c.final(seed);
        }
    }
    void next_bytes(uint8_t *out, size_t n) {
        size_t off = 0;
        generate_state();
        for (size_t i = 0; i < n; i++) {
            if (off == 32) { generate_state(); off = 0; }
            out[i] = state[off++];
        }
    }
};

inline void xor_with_hash(uint8_t *out, const uint8_t g1[48], const uint8_t *data, size_t len) {
    DigestRandom g;
    g.add_seed(g1, 48);
    // the keystream is drawn by ONE NextBytes call (GenerateState runs once up front, then every 32 bytes)
    uint8_t *ks = new uint8_t[len ? len : 1];
    g.next_bytes(ks, len);
    for (size_t i = 0; i < len; i++) out[i] = data[i] ^ ks[i];
    delete[] ks;
}

} // namespace lcb_host
