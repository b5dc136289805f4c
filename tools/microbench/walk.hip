// Dependent-lookup latency microbenchmark (gfx950, development tool): a single wave follows a chain
// of data-dependent lookups, the shape of a traceback walk step. Prints clk per dependent step for
// each access method.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/walk.hip -o tools/microbench/walk
#include <hip/hip_runtime.h>
#include <cstdio>

// V: 0 LDS (ds_read_b32 at an SGPR-derived address) + readfirstlane
//    1 LDS ds_read_b64 + 2 readfirstlane + ~8 dependent SALU (a walk step's decode)
//    2 scalar load (s_load_dword) from a global table (K$ / L2)
//    3 VGPR table + v_readlane with an SGPR lane index (no memory)
//    4 SALU only: 8 dependent SALU ops
template <int V>
__global__ __launch_bounds__(64) void walk_kernel(const unsigned *tab, int steps, unsigned *out, long long *cyc)
{
    __shared__ unsigned lds[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) lds[i] = tab[i];
    __syncthreads();
    unsigned vt = tab[lane * 7 & 4095];
    unsigned x = 1;
    long long t0 = clock64();
    for (int s = 0; s < steps; ++s)
    {
        if constexpr (V == 0)
        {
            x = __builtin_amdgcn_readfirstlane(lds[x & 4095]);
        }
        else if constexpr (V == 1)
        {
            const unsigned idx = (x * 2) & 4094;
            const unsigned long long w = *(const unsigned long long *)&lds[idx];
            const unsigned w0 = __builtin_amdgcn_readfirstlane((unsigned)w);
            const unsigned w1 = __builtin_amdgcn_readfirstlane((unsigned)(w >> 32));
            unsigned t = (w0 | w1) >> (x & 15);
            const unsigned r = t ? __builtin_ctz(t) : 7;
            x = x + r + ((w0 >> r) & 1) + 1;
        }
        else if constexpr (V == 2)
        {
            const unsigned off = (x & 4095) * 4;
            asm volatile("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(x) : "s"(tab), "s"(off) : "memory");
        }
        else if constexpr (V == 3)
        {
            x = __builtin_amdgcn_readlane(vt, x & 63) + x;
        }
        else
        {
            asm volatile("s_add_u32 %0, %0, 3\n\ts_lshr_b32 %0, %0, 1\n\ts_xor_b32 %0, %0, 5\n\ts_add_u32 %0, %0, 1\n\t"
                         "s_and_b32 %0, %0, 0xffff\n\ts_or_b32 %0, %0, 2\n\ts_add_u32 %0, %0, 7\n\ts_bfe_u32 %0, %0, 0x100001"
                         : "+s"(x));
        }
    }
    long long t1 = clock64();
    out[lane] = x;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
void run(const unsigned *tab, unsigned *out, long long *cyc)
{
    const int steps = 20000;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(walk_kernel<V>, dim3(1), dim3(64), 0, 0, tab, steps, out, cyc);
    (void)hipDeviceSynchronize();
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"variant\": %d, \"clk_per_step\": %.1f}\n", V, (double)c / steps);
    fflush(stdout);
}

int main()
{
    unsigned *tab, *out;
    long long *cyc;
    (void)hipMalloc(&tab, 4096 * 4);
    (void)hipMalloc(&out, 64 * 4);
    (void)hipMalloc(&cyc, 8);
    unsigned h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (unsigned)(i * 2654435761u) >> 7;
    (void)hipMemcpy(tab, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>(tab, out, cyc); run<1>(tab, out, cyc); run<2>(tab, out, cyc); run<3>(tab, out, cyc); run<4>(tab, out, cyc);
    return 0;
}
