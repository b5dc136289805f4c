// Lone-wave clocks per step of the score-chain recurrence with R rows per lane (development tool).
// Steps come from tools/microbench/gen_bandbench.py (bandbench.inc). One wave per SIMD, 256
// workgroups of 4 waves; then two waves per SIMD (8 waves per workgroup).
//   python3 tools/microbench/gen_bandbench.py && hipcc -O3 --offload-arch=gfx950 \
//       tools/microbench/bandbench.hip -o tools/microbench/bandbench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "bandbench.inc"

#define KERNEL(NAME)                                                                          \
    __global__ __launch_bounds__(512) void k_##NAME(int iters, long long *out, int *sink, int g) \
    {                                                                                         \
        const int lane = threadIdx.x & 63;                                                    \
        int r[NAME##_nregs];                                                                  \
        for (int i = 0; i < NAME##_nregs; ++i) r[i] = lane * (i + 1);                         \
        uint64_t t0, t1;                                                                      \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));                      \
        for (int it = 0; it < iters; ++it) NAME(r, lane * 0x01020304, g);                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));                      \
        int s = 0;                                                                            \
        for (int i = 0; i < NAME##_nregs; ++i) s += r[i];                                     \
        sink[blockIdx.x * blockDim.x + threadIdx.x] = s;                                      \
        if (lane == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = (long long)(t1 - t0);        \
    }                                                                                         \
    void run_##NAME(long long *out, int *sink, int wpg)                                       \
    {                                                                                         \
        const int iters = 2048, grid = 256;                                                   \
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(64 * wpg), 0, 0, iters, out, sink, 5); \
        (void)hipDeviceSynchronize();                                                         \
        static long long h[256 * 8];                                                          \
        (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);                            \
        double s = 0;                                                                         \
        for (int b = 0; b < grid; ++b)                                                        \
            for (int w = 0; w < wpg; ++w) s += (double)h[b * 8 + w] / ((double)iters * NAME##_steps); \
        printf("{\"stream\": \"%s\", \"waves_per_simd\": %d, \"steps_per_block\": %d, \"clk_per_step\": %.2f}\n", #NAME, wpg / 4, NAME##_steps, s / (grid * wpg)); \
    }

KERNEL(band_r1g)
KERNEL(band_r1l)
KERNEL(band_r2g)
KERNEL(band_r2l)
KERNEL(band_r3g)
KERNEL(band_r3l)
KERNEL(band_r4g)
KERNEL(band_r4l)

int main()
{
    long long *out;
    int *sink;
    (void)hipMalloc(&out, sizeof(long long) * 256 * 8);
    (void)hipMalloc(&sink, 256 * 512 * 4);
    for (int wpg = 4; wpg <= 8; wpg += 4)
    {
        run_band_r1g(out, sink, wpg);
        run_band_r1l(out, sink, wpg);
        run_band_r2g(out, sink, wpg);
        run_band_r2l(out, sink, wpg);
        run_band_r3g(out, sink, wpg);
        run_band_r4g(out, sink, wpg);
    }
    return 0;
}
