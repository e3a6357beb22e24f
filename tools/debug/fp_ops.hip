// Debug probe: inline-asm Fp add/sub/neg vs the C carry versions on random inputs < p (and edge cases).
#include "../../lachain_amd/csrc/field.hpp"
#include <stdio.h>
#include <stdlib.h>
__global__ void k(const fp *a, const fp *b, fp *out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp x = a[i], y = b[i], r;
    fp_add(r, x, y); out[6 * i + 0] = r;
    fp_add_c(r, x, y); out[6 * i + 1] = r;
    fp_sub(r, x, y); out[6 * i + 2] = r;
    fp_sub_c(r, x, y); out[6 * i + 3] = r;
    fp_neg(r, x); out[6 * i + 4] = r;
    fp_neg_c(r, x); out[6 * i + 5] = r;
}
static const uint32_t PH[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
int main() {
    const int n = 1 << 16;
    fp *ha = (fp *)malloc(n * sizeof(fp)), *hb = (fp *)malloc(n * sizeof(fp)), *ho = (fp *)malloc(6 * n * sizeof(fp));
    srand(1);
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < 12; j++) { ha[i].v[j] = rand() ^ (rand() << 16); hb[i].v[j] = rand() ^ (rand() << 16); }
        ha[i].v[11] &= 0x0fffffff; hb[i].v[11] &= 0x0fffffff;   // < p
        if (i % 7 == 0) hb[i] = ha[i];
        if (i % 11 == 0) for (int j = 0; j < 12; j++) ha[i].v[j] = 0;
        if (i % 13 == 0) { for (int j = 0; j < 12; j++) ha[i].v[j] = PH[j]; ha[i].v[0] -= 1; }
    }
    fp *da, *db, *dout;
    hipMalloc(&da, n * sizeof(fp)); hipMalloc(&db, n * sizeof(fp)); hipMalloc(&dout, 6 * n * sizeof(fp));
    hipMemcpy(da, ha, n * sizeof(fp), hipMemcpyHostToDevice); hipMemcpy(db, hb, n * sizeof(fp), hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(da, db, dout, n);
    hipMemcpy(ho, dout, 6 * n * sizeof(fp), hipMemcpyDeviceToHost);
    int bad[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int o = 0; o < 3; o++)
            for (int j = 0; j < 12; j++)
                if (ho[6 * i + 2 * o].v[j] != ho[6 * i + 2 * o + 1].v[j]) { if (bad[o] < 3) printf("op %d mismatch at %d limb %d\n", o, i, j); bad[o]++; break; }
    printf("add bad %d, sub bad %d, neg bad %d of %d\n", bad[0], bad[1], bad[2], n);
    return 0;
}
