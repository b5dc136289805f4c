// Row-walk chain microbenchmark (gfx950, development tool): clk per row of 64-row unrolled blocks
// with the instruction sequences of tools/microbench/gen_walkchain.py. One wave, windows of a fixed
// dense pattern (the search never runs out: the 64-bit shift wraps u at 64).
//   python3 tools/microbench/gen_walkchain.py && hipcc -O3 --offload-arch=gfx950 tools/microbench/walkchain.hip -o tools/microbench/walkchain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "walkchain.inc"

#define WC_KERNEL(V)                                                                                     \
    __global__ __launch_bounds__(64) void wc_##V(const unsigned *tab, int reps, unsigned *out, long long *cyc) \
    {                                                                                                    \
        const int lane = threadIdx.x;                                                                    \
        unsigned w0 = tab[lane] | 0x11111111u, rec = 0;                                                  \
        int u = 0;                                                                                       \
        asm volatile("v_readlane_b32 s88, %0, 0\n\tv_readlane_b32 s90, %0, 1" ::"v"(w0) : "s88", "s90"); \
        long long t0 = clock64();                                                                        \
        for (int r = 0; r < reps; ++r)                                                                   \
            asm volatile(WC_##V : [u] "+s"(u), [rec] "+v"(rec) : [w0] "v"(w0)                            \
                         : "scc", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");                \
        long long t1 = clock64();                                                                        \
        out[lane] = rec + u;                                                                             \
        if (lane == 0) *cyc = t1 - t0;                                                                   \
    }
WC_KERNEL(A) WC_KERNEL(B) WC_KERNEL(C) WC_KERNEL(D) WC_KERNEL(E) WC_KERNEL(F) WC_KERNEL(G) WC_KERNEL(H) WC_KERNEL(I)

int main()
{
    unsigned *tab, *out;
    long long *cyc;
    (void)hipMalloc(&tab, 256 * 4);
    (void)hipMalloc(&out, 256 * 4);
    (void)hipMalloc(&cyc, 8);
    unsigned h[256];
    for (int i = 0; i < 256; ++i) h[i] = 0x01020408u * (i % 7 + 1) ^ (0x9e3779b9u * i);
    (void)hipMemcpy(tab, h, sizeof h, hipMemcpyHostToDevice);
    const int reps = 256;
    const char *names = "ABCDEFGHI";
    void (*ks[])(const unsigned *, int, unsigned *, long long *) = {wc_A, wc_B, wc_C, wc_D, wc_E, wc_F, wc_G, wc_H, wc_I};
    for (int v = 0; v < 9; ++v)
    {
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, tab, reps, out, cyc);
        (void)hipDeviceSynchronize();
        long long c;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("{\"variant\": \"%c\", \"clk_per_row\": %.2f}\n", names[v], (double)c / (reps * 64.0));
    }
    return 0;
}
