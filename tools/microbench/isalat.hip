// Instruction latency / issue microbenchmark for the scalar traceback walk (gfx950, development
// tool): dependent SALU chains, v_readlane -> SALU, SALU -> v_writelane, taken branches.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/isalat.hip -o tools/microbench/isalat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

template <int V>
__global__ __launch_bounds__(64) void lat(const unsigned *tab, int iters, unsigned *out, long long *cyc)
{
    const int lane = threadIdx.x;
    unsigned v = tab[lane];
    unsigned s = __builtin_amdgcn_readfirstlane(tab[1]), s2 = s + 1, s3 = s + 2, s4 = s + 3;
    unsigned w = 0;
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    for (int it = 0; it < iters; ++it)
    {
        if constexpr (V == 0)  // 16 dependent s_add
            asm volatile(R16("s_add_u32 %0, %0, 3\n\t") : "+s"(s) : : "scc");
        else if constexpr (V == 1)  // 16 independent SALU (4 chains)
            asm volatile(R4("s_add_u32 %0, %0, 3\n\ts_add_u32 %1, %1, 3\n\ts_add_u32 %2, %2, 3\n\ts_add_u32 %3, %3, 3\n\t")
                         : "+s"(s), "+s"(s2), "+s"(s3), "+s"(s4) : : "scc");
        else if constexpr (V == 2)  // 16 x (readlane const lane -> dependent s_add into chain)
            asm volatile(R16("v_readlane_b32 %1, %2, 5\n\ts_add_u32 %0, %0, %1\n\t") : "+s"(s), "=&s"(s2) : "v"(v) : "scc");
        else if constexpr (V == 3)  // 16 x readlane alone (independent)
            asm volatile(R16("v_readlane_b32 %0, %1, 5\n\t") : "=s"(s2) : "v"(v) : "scc");
        else if constexpr (V == 4)  // 16 x dependent (lshr -> ff1 -> add)
            asm volatile(R16("s_lshr_b32 %1, %2, %0\n\ts_ff1_i32_b32 %1, %1\n\ts_add_u32 %0, %0, %1\n\ts_and_b32 %0, %0, 15\n\t")
                         : "+s"(s), "=&s"(s2) : "s"(s3 | 0x80008000u) : "scc");
        else if constexpr (V == 5)  // 16 x writelane const lane from a chained SGPR
            asm volatile(R16("s_add_u32 %0, %0, 3\n\tv_writelane_b32 %1, %0, 7\n\t") : "+s"(s), "+v"(w) : : "scc");
        else if constexpr (V == 6)  // 16 x taken forward branch
            asm volatile(R16("s_add_u32 %0, %0, 3\n\ts_branch 1f\n\ts_nop 0\n1:\n\t") : "+s"(s) : : "scc");
        else if constexpr (V == 7)  // 16 x not-taken conditional branch (scc from chain)
            asm volatile(R16("s_add_u32 %0, %0, 3\n\ts_cmp_eq_u32 %0, 1\n\ts_cbranch_scc1 2f\n\t") "2:\n\t" : "+s"(s) : : "scc");
        else if constexpr (V == 8)  // readlane with SGPR lane index from chain: k -> readlane -> add
            asm volatile(R16("s_and_b32 %1, %0, 63\n\tv_readlane_b32 %1, %2, %1\n\ts_add_u32 %0, %0, %1\n\t") : "+s"(s), "=&s"(s2) : "v"(v) : "scc");
        else if constexpr (V == 9)  // 16 x dependent s_bitcmp1 -> s_addc
            asm volatile(R16("s_bitcmp1_b32 %1, %0\n\ts_addc_u32 %0, %0, 0\n\t") : "+s"(s) : "s"(s3) : "scc");
        else if constexpr (V == 10)  // 16 x dependent 64-bit shift + ff1_b64 + add
            asm volatile(R16("s_lshr_b64 s[40:41], %1, %0\n\ts_ff1_i32_b64 s42, s[40:41]\n\ts_add_u32 %0, %0, s42\n\ts_and_b32 %0, %0, 31\n\t")
                         : "+s"(s) : "s"(((uint64_t)s3 << 32) | s3 | 0x8000000080000000ull) : "s40", "s41", "s42", "scc");
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    out[lane] = s + s2 + s3 + s4 + w;
    if (lane == 0) cyc[0] = (long long)(t1 - t0);
}

template <int V>
void run(const char *name, const unsigned *tab, unsigned *out, long long *cyc)
{
    const int iters = 4096;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(lat<V>, dim3(1), dim3(64), 0, 0, tab, iters, out, cyc);
    (void)hipDeviceSynchronize();
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"test\": \"%s\", \"clk_per_unit\": %.2f}\n", name, (double)c / (iters * 16.0));
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
    run<0>("salu_dep", tab, out, cyc);
    run<1>("salu_indep", tab, out, cyc);
    run<2>("readlane_to_salu", tab, out, cyc);
    run<3>("readlane_only", tab, out, cyc);
    run<4>("lshr_ff1_add_and", tab, out, cyc);
    run<5>("salu_to_writelane", tab, out, cyc);
    run<6>("taken_branch+add", tab, out, cyc);
    run<7>("add+cmp+notaken", tab, out, cyc);
    run<8>("and+readlane_sidx+add", tab, out, cyc);
    run<9>("bitcmp+addc", tab, out, cyc);
    run<10>("lshr64_ff1_add_and", tab, out, cyc);
    return 0;
}
