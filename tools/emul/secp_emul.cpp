// tools/emul/secp_emul.cpp — TEST INFRASTRUCTURE: compiles lachain_amd/csrc/k_secp.hip for the CPU and runs its
// kernels one lane at a time (they use no LDS and no barriers, so sequential execution is exact).  Lets the CPU test
// suite and a debugger check the device code's logic against the oracle without a GPU; the product path never
// loads this library.
#define SECP_HOST_EMULATION
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
struct emu_dim3 { unsigned x = 0, y = 0, z = 0; };
static emu_dim3 blockIdx, threadIdx, blockDim, gridDim;
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__
#define __global__
#define __constant__
#define __launch_bounds__(...)
#include "../../lachain_amd/csrc/k_secp.hip"

template <class F> static void run(size_t lanes, F f) {
    blockDim.x = 256;
    gridDim.x = (unsigned)((lanes + 255) / 256);
    for (unsigned b = 0; b < gridDim.x; b++)
        for (unsigned t = 0; t < 256; t++) {
            blockIdx.x = b;
            threadIdx.x = t;
            f();
        }
}

extern "C" {
// field element helpers: 32-byte little-endian in/out
void emu_fe_mul(uint8_t *r, const uint8_t *a, const uint8_t *b) { fe x, y, z; memcpy(&x, a, 32); memcpy(&y, b, 32); fe_mul(z, x, y); memcpy(r, &z, 32); }
void emu_fe_sqr(uint8_t *r, const uint8_t *a) { fe x, z; memcpy(&x, a, 32); fe_sqr(z, x); memcpy(r, &z, 32); }
void emu_fe_add(uint8_t *r, const uint8_t *a, const uint8_t *b) { fe x, y, z; memcpy(&x, a, 32); memcpy(&y, b, 32); fe_add(z, x, y); memcpy(r, &z, 32); }
void emu_fe_sub(uint8_t *r, const uint8_t *a, const uint8_t *b) { fe x, y, z; memcpy(&x, a, 32); memcpy(&y, b, 32); fe_sub(z, x, y); memcpy(r, &z, 32); }
void emu_fe_inv(uint8_t *r, const uint8_t *a) { fe x, z; memcpy(&x, a, 32); fe_inv(z, x); memcpy(r, &z, 32); }
void emu_fe_canon(uint8_t *r, const uint8_t *a) { fe x; memcpy(&x, a, 32); x = fe_canon(x); memcpy(r, &x, 32); }
void emu_sc_mont_mul(uint8_t *r, const uint8_t *a, const uint8_t *b) { sc x, y, z; memcpy(&x, a, 32); memcpy(&y, b, 32); sc_mont_mul(z, x, y); memcpy(r, &z, 32); }
void emu_sc_mont_inv(uint8_t *r, const uint8_t *a) { sc x, z; memcpy(&x, a, 32); sc_mont_inv(z, x); memcpy(r, &z, 32); }

// the whole pipeline: keys (pk_len each) -> tables; hashes or headers -> jobs -> accept
int emu_verify(uint8_t *accept, const uint8_t *hashes, const uint8_t *headers, uint64_t era, const uint8_t *sigs,
               uint32_t sig_len, const uint8_t *pks, uint32_t pk_len, uint32_t n_keys, const int32_t *key_idx,
               uint32_t n, int use_new, int chain_id) {
    std::vector<secp_aff> gaff(1), kaff(n_keys);
    std::vector<u32> gok(1), kok(n_keys);
    std::vector<secp_aff> gtab(33 * 128), ktab((size_t)n_keys * 33 * 128);
    blockIdx.x = threadIdx.x = 0;
    k_secp_gen(gaff.data(), gok.data());
    {
        std::vector<fe> tmp(2 * 128 * 33);
        run(33, [&] { k_secp_comb_build(gaff.data(), gok.data(), 1, gtab.data(), tmp.data(), tmp.data() + 128 * 33); });
    }
    run(n_keys, [&] { k_secp_key_parse(pks, pk_len, n_keys, kaff.data(), kok.data()); });
    {
        std::vector<fe> tmp((size_t)2 * 128 * 33 * n_keys);
        size_t lanes = (size_t)33 * n_keys;
        run(lanes, [&] { k_secp_comb_build(kaff.data(), kok.data(), n_keys, ktab.data(), tmp.data(), tmp.data() + 128 * lanes); });
    }
    std::vector<uint8_t> h(32 * (size_t)n), pre(n);
    const uint8_t *hp = hashes, *pp = nullptr;
    if (!hashes) {
        run(n, [&] { k_secp_header_hash(headers, n, era, h.data(), pre.data()); });
        hp = h.data();
        pp = pre.data();
    }
    std::vector<secp_job> jobs(n);
    size_t threads = (n + SECP_BATCH - 1) / SECP_BATCH;
    run(threads, [&] { k_secp_scalars(hp, sigs, sig_len, use_new ? 66 : 65, chain_id, key_idx, n_keys, kok.data(), pp, n, jobs.data()); });
    run(n, [&] { k_secp_verify(jobs.data(), n, gtab.data(), ktab.data(), accept); });
    return 0;
}
}
extern "C" int emu_job(uint8_t *job_out, const uint8_t *hash, const uint8_t *sig, uint32_t sig_len, int use_new, int chain_id) {
    u32 kok = 1;
    int32_t idx = 0;
    secp_job j;
    run(1, [&] { k_secp_scalars(hash, sig, sig_len, use_new ? 66 : 65, chain_id, &idx, 1, &kok, nullptr, 1, &j); });
    memcpy(job_out, &j, sizeof j);
    return 0;
}
// same stages as tools/emul/secp_stage_dump.hip, same output layout
extern "C" int emu_stage_dump(uint8_t *out, const uint8_t *keys, uint32_t n_keys, uint32_t pk_len, const uint8_t *hashes,
                              const uint8_t *sigs, uint32_t sig_len, const int32_t *idx, uint32_t n, int use_new, int chain) {
    std::vector<secp_aff> gaff(1), kaff(n_keys), gtab(33 * 128), ktab((size_t)n_keys * 33 * 128);
    std::vector<u32> gok(1), kok(n_keys);
    blockIdx.x = threadIdx.x = 0;
    k_secp_gen(gaff.data(), gok.data());
    std::vector<fe> tmp((size_t)2 * 128 * 33 * (n_keys > 1 ? n_keys : 1));
    run(33, [&] { k_secp_comb_build(gaff.data(), gok.data(), 1, gtab.data(), tmp.data(), tmp.data() + 128 * 33); });
    run(n_keys, [&] { k_secp_key_parse(keys, pk_len, n_keys, kaff.data(), kok.data()); });
    size_t lanes = (size_t)33 * n_keys;
    run(lanes, [&] { k_secp_comb_build(kaff.data(), kok.data(), n_keys, ktab.data(), tmp.data(), tmp.data() + 128 * lanes); });
    std::vector<secp_job> jobs(n);
    std::vector<uint8_t> acc(n);
    run((n + SECP_BATCH - 1) / SECP_BATCH, [&] { k_secp_scalars(hashes, sigs, sig_len, use_new ? 66 : 65, chain, idx, n_keys, kok.data(), nullptr, n, jobs.data()); });
    run(n, [&] { k_secp_verify(jobs.data(), n, gtab.data(), ktab.data(), acc.data()); });
    uint8_t *p = out;
    auto cp = [&](const void *src, size_t b) { memcpy(p, src, b); p += b; };
    cp(gaff.data(), 64); cp(gok.data(), 4); cp(gtab.data(), gtab.size() * 64); cp(kaff.data(), 64 * n_keys);
    cp(kok.data(), 4 * n_keys); cp(ktab.data(), ktab.size() * 64); cp(jobs.data(), sizeof(secp_job) * n); cp(acc.data(), n);
    return (int)(p - out);
}
