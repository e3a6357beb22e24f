// tools/emul/secp_stage_dump.hip — TEST INFRASTRUCTURE: runs the k_secp.hip stages on the GPU for one input file and
// writes every intermediate buffer, so tools/emul/secp_emul.cpp (the same code on the CPU) can be diffed against it.
// input file: u32 n_keys, pk_len, n, sig_len, use_new, chain_id | keys | hashes (32 n) | sigs | idx (i32 n)
#include "../../lachain_amd/csrc/k_secp.hip"
#include <stdio.h>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
template <class T> static T *dev(const void *h, size_t bytes) {
    T *d = nullptr;
    if (hipMalloc(&d, bytes ? bytes : 16) != hipSuccess) return nullptr;
    if (h && bytes) (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    else (void)hipMemset(d, 0, bytes ? bytes : 16);
    return d;
}
static void put(FILE *f, const void *d, size_t bytes) {
    std::vector<uint8_t> h(bytes);
    (void)hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost);
    fwrite(h.data(), 1, bytes, f);
}
int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    u32 hdr[6];
    if (fread(hdr, 4, 6, f) != 6) return 2;
    u32 n_keys = hdr[0], pk_len = hdr[1], n = hdr[2], sig_len = hdr[3], use_new = hdr[4];
    int chain = (int)hdr[5];
    std::vector<uint8_t> keys(n_keys * pk_len), hashes(32 * n), sigs(sig_len * n);
    std::vector<int32_t> idx(n);
    if (fread(keys.data(), 1, keys.size(), f) != keys.size() || fread(hashes.data(), 1, hashes.size(), f) != hashes.size() ||
        fread(sigs.data(), 1, sigs.size(), f) != sigs.size() || fread(idx.data(), 4, n, f) != n) return 2;
    fclose(f);
    hipStream_t s = nullptr;
    secp_aff *gaff = dev<secp_aff>(nullptr, 64), *kaff = dev<secp_aff>(nullptr, 64 * n_keys);
    u32 *gok = dev<u32>(nullptr, 4), *kok = dev<u32>(nullptr, 4 * n_keys);
    size_t tb = lcbk_secp_table_bytes();
    void *gtab = dev<uint8_t>(nullptr, tb), *ktab = dev<uint8_t>(nullptr, tb * n_keys);
    void *tmp = dev<uint8_t>(nullptr, 2 * 128 * 33 * 32 * (size_t)(n_keys > 1 ? n_keys : 1));
    uint8_t *dk = dev<uint8_t>(keys.data(), keys.size()), *dh = dev<uint8_t>(hashes.data(), hashes.size());
    uint8_t *ds = dev<uint8_t>(sigs.data(), sigs.size());
    int32_t *di = dev<int32_t>(idx.data(), 4 * n);
    void *jobs = dev<uint8_t>(nullptr, lcbk_secp_job_bytes() * n);
    uint8_t *acc = dev<uint8_t>(nullptr, n);
    lcbk_secp_gen(s, gaff, gok);
    CK(hipDeviceSynchronize());
    lcbk_secp_comb_build(s, gaff, gok, 1, gtab, tmp);
    CK(hipDeviceSynchronize());
    lcbk_secp_key_parse(s, dk, pk_len, n_keys, kaff, kok);
    CK(hipDeviceSynchronize());
    lcbk_secp_comb_build(s, kaff, kok, n_keys, ktab, tmp);
    CK(hipDeviceSynchronize());
    lcbk_secp_scalars(s, dh, ds, sig_len, use_new ? 66 : 65, chain, di, n_keys, kok, nullptr, n, jobs);
    CK(hipDeviceSynchronize());
    lcbk_secp_verify(s, jobs, n, gtab, ktab, acc);
    CK(hipDeviceSynchronize());
    FILE *o = fopen(argv[2], "wb");
    put(o, gaff, 64); put(o, gok, 4); put(o, gtab, tb); put(o, kaff, 64 * n_keys); put(o, kok, 4 * n_keys);
    put(o, ktab, tb * n_keys); put(o, jobs, lcbk_secp_job_bytes() * n); put(o, acc, n);
    fclose(o);
    printf("ok\n");
    return 0;
}
