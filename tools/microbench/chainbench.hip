// Dependent-chain vs issue-rate microbenchmark for the fill step (gfx950, development tool).
// Each stream runs 16 unrolled "steps" per iteration; the kernel reports shader clocks per step for
// one wave per SIMD (4 waves, one workgroup per CU, 256 workgroups). Streams:
//   A score5     Qn = shl(Q); D = diag + S (sdwa); up = shr(F) in place; M = max(F, up); F' = max(D, M)
//                (the split fill's score step: dependent chain F -> up -> M -> F', 3 deep)
//   B chain3     up = shr(F); M = max(F, up); F' = max(D, M)     (the same chain, nothing else)
//   C fused6     Qn = shl(Q); m = max(F, Q); m = max_dpp(shr F, F) (lanes 1..63); d = S + Qp;
//                d = add_dpp(shr Fp, S) (lanes 1..63); F' = max(d, m)   (chain F -> m -> F', 2 deep)
//   D chain2     m = max_dpp(shr F, F); F' = max(d, m)            (2 deep, nothing else)
//   E indep6     6 independent VALU per step                      (issue rate)
//   F indep5     5 independent VALU per step
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/chainbench.hip -o tools/microbench/chainbench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define SHR "wave_shr:1 row_mask:0xf bank_mask:0xf"
#define SHL "wave_shl:1 row_mask:0xf bank_mask:0xf"

// A: regs rotate q, qn, dg, f as in tools/gen_split_asm.py (period 4)
#define SCORE5(QD, QR, DG, FP, T, B)                                                            \
    "v_mov_b32_dpp " QD ", " QR " " SHL "\n\t"                                                  \
    "v_add_u32_sdwa %[d], " DG ", sext(" T ") dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_" B "\n\t" \
    "v_mov_b32_dpp " QR ", " FP " " SHR "\n\t"                                                  \
    "v_max_i32_e32 %[m], " FP ", " QR "\n\t"                                                   \
    "v_max_i32_e32 " DG ", %[d], %[m]\n\t"
#define CHAIN3(U, F0, F1)                                                                        \
    "s_nop 1\n\t"                                                                                \
    "v_mov_b32_dpp " U ", " F0 " " SHR "\n\t"                                                   \
    "v_max_i32_e32 %[m], " F0 ", " U "\n\t"                                                    \
    "v_max_i32_e32 " F1 ", %[d], %[m]\n\t"
// C: F2 = F two steps back, F1 = previous, F0 = written
#define FUSED6(F2, F1, F0)                                                                       \
    "v_mov_b32_dpp %[qn], %[q] " SHL "\n\t"                                                     \
    "v_max_i32_e32 %[m], " F1 ", %[q]\n\t"                                                     \
    "v_add_u32_e32 %[d], %[s0], %[qn]\n\t"                                                     \
    "v_max_i32_dpp %[m], " F1 ", " F1 " " SHR "\n\t"                                            \
    "v_add_u32_dpp %[d], " F2 ", %[s0] " SHR "\n\t"                                             \
    "v_max_i32_e32 " F0 ", %[d], %[m]\n\t"
#define CHAIN2(F1, F0)                                                                           \
    "s_nop 1\n\t"                                                                                \
    "v_max_i32_dpp %[m], " F1 ", " F1 " " SHR "\n\t"                                            \
    "v_max_i32_e32 " F0 ", %[d], %[m]\n\t"
#define INDEP6                                                                                   \
    "v_add_u32 %[x0], %[x0], %[s0]\n\tv_add_u32 %[x1], %[x1], %[s0]\n\tv_add_u32 %[x2], %[x2], %[s0]\n\t" \
    "v_add_u32 %[x3], %[x3], %[s0]\n\tv_add_u32 %[x4], %[x4], %[s0]\n\tv_add_u32 %[x5], %[x5], %[s0]\n\t"
#define INDEP5                                                                                   \
    "v_add_u32 %[x0], %[x0], %[s0]\n\tv_add_u32 %[x1], %[x1], %[s0]\n\tv_add_u32 %[x2], %[x2], %[s0]\n\t" \
    "v_add_u32 %[x3], %[x3], %[s0]\n\tv_add_u32 %[x4], %[x4], %[s0]\n\t"

struct R {
    int q, qn, dg, f, d, m, f0, f1, f2, f3, s0, x0, x1, x2, x3, x4, x5;
};

template <int K>
__device__ __forceinline__ void stream(int iters, R &r)
{
    for (int it = 0; it < iters; ++it)
    {
        if constexpr (K == 0)
            asm volatile("s_nop 1\n\t"
                         SCORE5("%[qn]", "%[q]", "%[dg]", "%[f]", "%[s0]", "0") SCORE5("%[f]", "%[qn]", "%[q]", "%[dg]", "%[s0]", "1")
                         SCORE5("%[dg]", "%[f]", "%[qn]", "%[q]", "%[s0]", "2") SCORE5("%[q]", "%[dg]", "%[f]", "%[qn]", "%[s0]", "3")
                         SCORE5("%[qn]", "%[q]", "%[dg]", "%[f]", "%[s0]", "0") SCORE5("%[f]", "%[qn]", "%[q]", "%[dg]", "%[s0]", "1")
                         SCORE5("%[dg]", "%[f]", "%[qn]", "%[q]", "%[s0]", "2") SCORE5("%[q]", "%[dg]", "%[f]", "%[qn]", "%[s0]", "3")
                         SCORE5("%[qn]", "%[q]", "%[dg]", "%[f]", "%[s0]", "0") SCORE5("%[f]", "%[qn]", "%[q]", "%[dg]", "%[s0]", "1")
                         SCORE5("%[dg]", "%[f]", "%[qn]", "%[q]", "%[s0]", "2") SCORE5("%[q]", "%[dg]", "%[f]", "%[qn]", "%[s0]", "3")
                         SCORE5("%[qn]", "%[q]", "%[dg]", "%[f]", "%[s0]", "0") SCORE5("%[f]", "%[qn]", "%[q]", "%[dg]", "%[s0]", "1")
                         SCORE5("%[dg]", "%[f]", "%[qn]", "%[q]", "%[s0]", "2") SCORE5("%[q]", "%[dg]", "%[f]", "%[qn]", "%[s0]", "3")
                         : [q] "+v"(r.q), [qn] "+v"(r.qn), [dg] "+v"(r.dg), [f] "+v"(r.f), [d] "+v"(r.d), [m] "+v"(r.m)
                         : [s0] "v"(r.s0));
        else if constexpr (K == 1)
            asm volatile("s_nop 1\n\t"
                         CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]") CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]")
                         CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]") CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]")
                         CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]") CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]")
                         CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]") CHAIN3("%[q]", "%[f0]", "%[f1]") CHAIN3("%[q]", "%[f1]", "%[f0]")
                         : [q] "+v"(r.q), [f0] "+v"(r.f0), [f1] "+v"(r.f1), [d] "+v"(r.d), [m] "+v"(r.m)
                         :);
        else if constexpr (K == 2)
            asm volatile("s_nop 1\n\t"
                         FUSED6("%[f2]", "%[f3]", "%[f0]") FUSED6("%[f3]", "%[f0]", "%[f1]") FUSED6("%[f0]", "%[f1]", "%[f2]") FUSED6("%[f1]", "%[f2]", "%[f3]")
                         FUSED6("%[f2]", "%[f3]", "%[f0]") FUSED6("%[f3]", "%[f0]", "%[f1]") FUSED6("%[f0]", "%[f1]", "%[f2]") FUSED6("%[f1]", "%[f2]", "%[f3]")
                         FUSED6("%[f2]", "%[f3]", "%[f0]") FUSED6("%[f3]", "%[f0]", "%[f1]") FUSED6("%[f0]", "%[f1]", "%[f2]") FUSED6("%[f1]", "%[f2]", "%[f3]")
                         FUSED6("%[f2]", "%[f3]", "%[f0]") FUSED6("%[f3]", "%[f0]", "%[f1]") FUSED6("%[f0]", "%[f1]", "%[f2]") FUSED6("%[f1]", "%[f2]", "%[f3]")
                         : [q] "+v"(r.q), [qn] "+v"(r.qn), [f0] "+v"(r.f0), [f1] "+v"(r.f1), [f2] "+v"(r.f2), [f3] "+v"(r.f3),
                           [d] "+v"(r.d), [m] "+v"(r.m)
                         : [s0] "v"(r.s0));
        else if constexpr (K == 3)
            asm volatile("s_nop 1\n\t"
                         CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]") CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]")
                         CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]") CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]")
                         CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]") CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]")
                         CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]") CHAIN2("%[f0]", "%[f1]") CHAIN2("%[f1]", "%[f0]")
                         : [f0] "+v"(r.f0), [f1] "+v"(r.f1), [d] "+v"(r.d), [m] "+v"(r.m)
                         :);
        else if constexpr (K == 4)
            asm volatile(INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6 INDEP6
                         : [x0] "+v"(r.x0), [x1] "+v"(r.x1), [x2] "+v"(r.x2), [x3] "+v"(r.x3), [x4] "+v"(r.x4), [x5] "+v"(r.x5)
                         : [s0] "v"(r.s0));
        else
            asm volatile(INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5 INDEP5
                         : [x0] "+v"(r.x0), [x1] "+v"(r.x1), [x2] "+v"(r.x2), [x3] "+v"(r.x3), [x4] "+v"(r.x4)
                         : [s0] "v"(r.s0));
    }
}

template <int K>
__global__ __launch_bounds__(256) void bench(int iters, long long *out, int *sink)
{
    const int lane = threadIdx.x & 63;
    R r{lane, 0, 1, lane * 3, 2, 3, lane, lane + 1, 7, 9, 5, 1, 2, 3, 4, 5, 6};
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    stream<K>(iters, r);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    sink[blockIdx.x * blockDim.x + threadIdx.x] = r.q + r.qn + r.dg + r.f + r.d + r.m + r.f0 + r.f1 + r.f2 + r.f3 + r.x0 + r.x5;
    if (lane == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = (long long)(t1 - t0);
}

template <int K>
void run(const char *name, long long *out, int *sink)
{
    const int iters = 4096, grid = 256;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(bench<K>, dim3(grid), dim3(256), 0, 0, iters, out, sink);
    (void)hipDeviceSynchronize();
    static long long h[256 * 4];
    (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid * 4; ++i) s += (double)h[i] / (iters * 16.0);
    printf("{\"stream\": \"%s\", \"clk_per_step\": %.2f}\n", name, s / (grid * 4));
}

int main()
{
    long long *out;
    int *sink;
    (void)hipMalloc(&out, sizeof(long long) * 256 * 4);
    (void)hipMalloc(&sink, 256 * 256 * 4);
    run<0>("A score5 (chain 3)", out, sink);
    run<1>("B chain3 only (s_nop 1 + 3)", out, sink);
    run<2>("C fused6 (chain 2)", out, sink);
    run<3>("D chain2 only (s_nop 1 + 2)", out, sink);
    run<4>("E indep6", out, sink);
    run<5>("F indep5", out, sink);
    return 0;
}
