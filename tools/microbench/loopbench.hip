// Prototype steady loops of the fused R = 1 fill step (tools/microbench/gen_loopbench.py): clocks per
// step for one wave per SIMD, 4 compute waves + 1 partner wave per workgroup. Timing only.
//   python3 tools/microbench/gen_loopbench.py && hipcc -O3 --offload-arch=gfx950 tools/microbench/loopbench.hip -o tools/microbench/loopbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "loopbench.inc"

constexpr int kIters = 512;

template <int V>
__global__ __launch_bounds__(320) void loop_kernel(const int *sbuf, uint32_t *planes, long long *out)
{
    extern __shared__ int lds[];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int e = threadIdx.x; e < 64 * 1024 / 4 - 64; e += blockDim.x) lds[e] = 0;
    __syncthreads();
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    if (w < 4)
    {
        const uint32_t ldsbase = (uint32_t)(uintptr_t)lds;
        const uint32_t ring = ldsbase + w * 8192, rout = ldsbase + (w + 1) * 8192;
        const uint32_t sink = ldsbase + 5 * 8192;
        const uint32_t vpubbase = lane == 63 ? rout : sink + 16 * lane;
        const uint32_t vlmask = lane == 63 ? 0x1fffu : 0u;
        const uint32_t vpaddr = ldsbase + 5 * 8192 + 9216 + 4 * w;
        const uint32_t vsoff = (uint32_t)((lane & 3) * (1 << 20) + (64 - lane) * 4);
        const uint32_t vmoff = lane * 8;
        const uint64_t sb = (uint64_t)sbuf;
        const uint64_t mb = (uint64_t)(planes + (size_t)(blockIdx.x * 4 + w) * kIters * 3 * 128);
        const int sp0 = (64 * w * 4) & 0x1fff;
        const int sneed = -1000000;
        const int iters = kIters;
#define LB_CALL(X) asm volatile(X :: [iters] "s"(iters), [sb] "s"(sb), [mb] "s"(mb), [sp0] "s"(sp0), [sneed] "s"(sneed), \
                         [vsoff] "v"(vsoff), [vmoff] "v"(vmoff), [vlmask] "v"(vlmask), [vpubbase] "v"(vpubbase), \
                         [vrin] "v"(ring), [vpaddr] "v"(vpaddr) : LB_VCLOB, LB_SCLOB, "vcc", "scc", "memory")
        if constexpr (V == 0) LB_CALL(LB_LOOP0);
        else if constexpr (V == 1) LB_CALL(LB_LOOP1);
        else if constexpr (V == 2) LB_CALL(LB_LOOP2);
        else if constexpr (V == 100) LB_CALL(LB_NONE);
        else if constexpr (V == 101) LB_CALL(LB_LDS);
        else if constexpr (V == 102) LB_CALL(LB_LDSR);
        else if constexpr (V == 103) LB_CALL(LB_LDSW);
        else if constexpr (V == 104) LB_CALL(LB_LDSWX);
        else if constexpr (V == 105) LB_CALL(LB_LDSX);
        else if constexpr (V == 106) LB_CALL(LB_LDSEARLY);
        else if constexpr (V == 107) LB_CALL(LB_LDSEARLYX);
        else if constexpr (V == 108) LB_CALL(LB_LOADS);
        else if constexpr (V == 109) LB_CALL(LB_LOADSL2);
        else if constexpr (V == 110) LB_CALL(LB_ALL_L2);
        else if constexpr (V == 111) LB_CALL(LB_ALL_L2X);
    }
    else if (V == 1)
    {
        for (int i = 0; i < kIters * 12; ++i) asm volatile("s_barrier" ::: "memory");
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    if (lane == 0) out[blockIdx.x * 8 + w] = (long long)(t1 - t0);
}

template <int V>
void run(const char *name, int grid, const int *s, uint32_t *p, long long *out)
{
    const size_t lds = 64 * 1024;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&loop_kernel<V>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(loop_kernel<V>, dim3(grid), dim3(320), lds, 0, s, p, out);
    if (hipDeviceSynchronize() != hipSuccess) { printf("{\"test\": \"%s\", \"error\": true}\n", name); return; }
    static long long h[256 * 8];
    (void)hipMemcpy(h, out, sizeof(long long) * grid * 8, hipMemcpyDeviceToHost);
    double sum = 0, mx = 0;
    for (int b = 0; b < grid; ++b)
        for (int w = 0; w < 4; ++w)
        {
            const double c = (double)h[b * 8 + w] / (kIters * 96.0);
            sum += c;
            mx = c > mx ? c : mx;
        }
    printf("{\"test\": \"%s\", \"grid\": %d, \"clk_per_step_mean\": %.2f, \"clk_per_step_max\": %.2f}\n", name, grid, sum / (grid * 4), mx);
    fflush(stdout);
}

int main()
{
    int *s;
    uint32_t *p;
    long long *out;
    (void)hipMalloc(&s, 8 << 20);
    (void)hipMemset(s, 0, 8 << 20);
    (void)hipMalloc(&p, (size_t)132 * 4 * kIters * 3 * 512 + 4096);
    (void)hipMalloc(&out, sizeof(long long) * 256 * 8);
    for (int grid : {1, 132})
    {
        run<100>("NONE", grid, s, p, out);
        run<101>("LDS", grid, s, p, out);
        run<102>("LDSR", grid, s, p, out);
        run<103>("LDSW", grid, s, p, out);
        run<104>("LDSWX", grid, s, p, out);
        run<105>("LDSX", grid, s, p, out);
        run<106>("LDSEARLY", grid, s, p, out);
        run<107>("LDSEARLYX", grid, s, p, out);
        run<108>("LOADS", grid, s, p, out);
        run<109>("LOADSL2", grid, s, p, out);
        run<110>("ALL_L2", grid, s, p, out);
        run<111>("ALL_L2X", grid, s, p, out);
    }
    return 0;
}
