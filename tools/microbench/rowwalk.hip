// Row-walk traceback microbenchmark (gfx950, development tool). One wave walks rows of a strip: for
// each row it reads the row's non-LEFT / DIAG window words from VGPRs (v_readlane at lane k), finds the
// first non-LEFT cell at or left of the current column (shift + find-first-one), and moves up one row
// (left one more column on DIAG). Prints clk per row for each loop shape.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/rowwalk.hip -o tools/microbench/rowwalk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ int wl(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// V0: 8 dependent SALU ops per "row" (SALU issue/latency floor)
// V1: 32-bit windows, dynamic lane k, wrap t at 32 (C++)
// V2: 64-bit windows (two readlanes per word), dynamic k (C++)
// V3: 32-bit windows, 64 rows unrolled with constant lanes (C++)
template <int V>
__global__ __launch_bounds__(64) void rowwalk(const unsigned *tab, int rows, unsigned *out, long long *cyc)
{
    const int lane = threadIdx.x;
    const unsigned nl0 = tab[lane] | 0x80000000u, nl1 = tab[64 + lane] | 0x80000000u;
    const unsigned d0 = tab[128 + lane] & nl0, d1 = tab[192 + lane] & nl1;
    unsigned rec = 0;
    unsigned t = 0, acc = 0;
    long long t0 = clock64();
    if constexpr (V == 0)
    {
        unsigned x = __builtin_amdgcn_readfirstlane(tab[0]);
        for (int s = 0; s < rows; ++s)
            asm volatile("s_add_u32 %0, %0, 3\n\ts_lshr_b32 %0, %0, 1\n\ts_xor_b32 %0, %0, 5\n\ts_add_u32 %0, %0, 1\n\t"
                         "s_and_b32 %0, %0, 0xffff\n\ts_or_b32 %0, %0, 2\n\ts_add_u32 %0, %0, 7\n\ts_bfe_u32 %0, %0, 0x100001"
                         : "+s"(x));
        acc = x;
    }
    else if constexpr (V == 1)
    {
        int k = 63;
        for (int s = 0; s < rows; ++s)
        {
            const unsigned n = __builtin_amdgcn_readlane(nl0, k);
            const unsigned d = __builtin_amdgcn_readlane(d0, k);
            const unsigned x = n >> t;
            unsigned r = x ? __builtin_ctz(x) : 0;
            t += r;
            const unsigned dg = (d >> t) & 1u;
            rec = (unsigned)wl((int)(2 * t + dg), k, (int)rec);
            t += dg;
            t &= 31;
            k = (k - 1) & 63;
        }
    }
    else if constexpr (V == 2)
    {
        int k = 63;
        for (int s = 0; s < rows; ++s)
        {
            const uint64_t n = ((uint64_t)__builtin_amdgcn_readlane(nl1, k) << 32) | __builtin_amdgcn_readlane(nl0, k);
            const uint64_t d = ((uint64_t)__builtin_amdgcn_readlane(d1, k) << 32) | __builtin_amdgcn_readlane(d0, k);
            const uint64_t x = n >> t;
            unsigned r = x ? __builtin_ctzll(x) : 0;
            t += r;
            const unsigned dg = (unsigned)(d >> t) & 1u;
            rec = (unsigned)wl((int)(2 * t + dg), k, (int)rec);
            t += dg;
            if (t >= 32) t -= 32;
            k = (k - 1) & 63;
        }
    }
    else
    {
        for (int s = 0; s < rows; s += 64)
        {
#pragma unroll
            for (int k = 63; k >= 0; --k)
            {
                const unsigned n = __builtin_amdgcn_readlane(nl0, k);
                const unsigned d = __builtin_amdgcn_readlane(d0, k);
                const unsigned x = n >> t;
                unsigned r = x ? __builtin_ctz(x) : 0;
                t += r;
                const unsigned dg = (d >> t) & 1u;
                rec = (unsigned)wl((int)(2 * t + dg), k, (int)rec);
                t += dg;
                t &= 31;
            }
        }
    }
    long long t1 = clock64();
    out[lane] = rec + acc + t;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
void run(const unsigned *tab, unsigned *out, long long *cyc)
{
    const int rows = 64 * 1024;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(rowwalk<V>, dim3(1), dim3(64), 0, 0, tab, rows, out, cyc);
    (void)hipDeviceSynchronize();
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"variant\": %d, \"clk_per_row\": %.1f}\n", V, (double)c / rows);
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
    uint64_t s = 12345;
    for (int i = 0; i < 4096; ++i)
    {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        h[i] = (unsigned)(s >> 32) | (unsigned)(s >> 17);  // ~3/4 density
    }
    (void)hipMemcpy(tab, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>(tab, out, cyc);
    run<1>(tab, out, cyc);
    run<2>(tab, out, cyc);
    run<3>(tab, out, cyc);
    return 0;
}
