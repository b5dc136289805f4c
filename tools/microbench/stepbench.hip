// Step-cost microbenchmark for the R = 1 fill step (gfx950, development tool).
// Measures shader clocks per DP step of candidate instruction streams for one wave, and for two
// waves sharing a SIMD (an 8-wave workgroup: waves w and w+4 share a SIMD), plus a functional check
// of the lane-0 semantics the fused step relies on (VOP2 DPP wave_shr:1, bound_ctrl off: lane 0 is
// not written).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/stepbench.hip -o tools/microbench/stepbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

#define SHR "wave_shr:1 row_mask:0xf bank_mask:0xf"
#define SHL "wave_shl:1 row_mask:0xf bank_mask:0xf"

// ---- stream kinds ----
// 0: current 9-VALU step (queue shl, up shr, sdwa add, 2 max, 2 sub, 2 alignbit)
#define CUR(F0, F1, Q, QN, T, B)                                                           \
    "v_mov_b32_dpp " QN ", " Q " " SHL "\n\t"                                              \
    "v_mov_b32_dpp " Q ", " F0 " " SHR "\n\t"                                              \
    "v_add_u32_sdwa %[d], %[dg], sext(" T ") dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_" B "\n\t" \
    "v_max_i32 %[m], " F0 ", " Q "\n\t"                                                   \
    "v_sub_u32 %[y], " F0 ", " Q "\n\t"                                                   \
    "v_max_i32 " F1 ", %[d], %[m]\n\t"                                                    \
    "v_sub_u32 %[x], %[m], %[d]\n\t"                                                      \
    "v_alignbit_b32 %[a0], %[a0], %[x], 31\n\t"                                           \
    "v_alignbit_b32 %[a1], %[a1], %[y], 31\n\t"
// 1: fused 3-VALU score + 4 direction ops. F2 = F_{s-2}, F1 = F_{s-1}, F0 = F_s (written)
#define FUSED(F2, F1, F0, S)                                                               \
    "v_add_u32_dpp %[d], " F2 ", " S " " SHR "\n\t"                                        \
    "v_max_i32_dpp %[m], " F1 ", " F1 " " SHR "\n\t"                                       \
    "v_max_i32 " F0 ", %[d], %[m]\n\t"                                                    \
    "v_sub_u32 %[x], %[m], %[d]\n\t"                                                      \
    "v_sub_u32 %[y], " F1 ", %[m]\n\t"                                                    \
    "v_alignbit_b32 %[a0], %[a0], %[x], 31\n\t"                                           \
    "v_alignbit_b32 %[a1], %[a1], %[y], 31\n\t"
// 2: fused score only, one s_nop 0 (the DPP wait states)
#define SCORE(F2, F1, F0, S)                                                               \
    "v_add_u32_dpp %[d], " F2 ", " S " " SHR "\n\t"                                        \
    "v_max_i32_dpp %[m], " F1 ", " F1 " " SHR "\n\t"                                       \
    "v_max_i32 " F0 ", %[d], %[m]\n\t"                                                    \
    "s_nop 0\n\t"
// 4: fused score + byte-lane direction differences (SDWA dst byte q, preserve), inserted per 4 steps
#define BYTEDIR(F2, F1, F0, S, B)                                                          \
    "v_add_u32_dpp %[d], " F2 ", " S " " SHR "\n\t"                                        \
    "v_max_i32_dpp %[m], " F1 ", " F1 " " SHR "\n\t"                                       \
    "v_max_i32 " F0 ", %[d], %[m]\n\t"                                                    \
    "v_sub_u32_sdwa %[x], %[m], %[d] dst_sel:BYTE_" B " dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_sub_u32_sdwa %[y], " F1 ", %[m] dst_sel:BYTE_" B " dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
#define BYTEINS                                                                            \
    "v_lshrrev_b32 %[a0], 1, %[a0]\n\t"                                                   \
    "v_and_or_b32 %[a0], %[x], %[msk], %[a0]\n\t"                                         \
    "v_lshrrev_b32 %[a1], 1, %[a1]\n\t"                                                   \
    "v_and_or_b32 %[a1], %[y], %[msk], %[a1]\n\t"
// 6: direction-wave-like stream (independent of the score chain)
#define DIRW(L, U, S)                                                                      \
    "v_add_u32 %[d], " U ", " S "\n\t"                                                     \
    "v_max_i32 %[m], " L ", " U "\n\t"                                                     \
    "v_sub_u32 %[x], %[m], %[d]\n\t"                                                      \
    "v_sub_u32 %[y], " L ", %[m]\n\t"                                                     \
    "v_alignbit_b32 %[a0], %[a0], %[x], 31\n\t"                                           \
    "v_alignbit_b32 %[a1], %[a1], %[y], 31\n\t"

struct Regs
{
    int f0, f1, f2, f3, q, qn, dg, d, m, x, y, a0, a1, msk;
    int s0, s1, s2, s3;
};

template <int K>
__device__ __forceinline__ void run_stream(int iters, Regs &r, uint32_t *lds_addr_dummy, const int *gbase, int lane, int *ldsbuf)
{
    (void)lds_addr_dummy;
    const uint32_t la = (uint32_t)(uintptr_t)(ldsbuf + 4 * lane);
    const uint32_t lr = (uint32_t)(uintptr_t)(ldsbuf + 256);
    const int *gp = gbase + ((lane & 3) * 1024) + 64 - lane;
    for (int it = 0; it < iters; ++it)
    {
        if constexpr (K == 0)
        {
            asm volatile(
                CUR("%[f0]", "%[f1]", "%[q]", "%[qn]", "%[s0]", "0") CUR("%[f1]", "%[f2]", "%[qn]", "%[q]", "%[s0]", "1")
                CUR("%[f2]", "%[f3]", "%[q]", "%[qn]", "%[s0]", "2") CUR("%[f3]", "%[f0]", "%[qn]", "%[q]", "%[s0]", "3")
                CUR("%[f0]", "%[f1]", "%[q]", "%[qn]", "%[s1]", "0") CUR("%[f1]", "%[f2]", "%[qn]", "%[q]", "%[s1]", "1")
                CUR("%[f2]", "%[f3]", "%[q]", "%[qn]", "%[s1]", "2") CUR("%[f3]", "%[f0]", "%[qn]", "%[q]", "%[s1]", "3")
                CUR("%[f0]", "%[f1]", "%[q]", "%[qn]", "%[s2]", "0") CUR("%[f1]", "%[f2]", "%[qn]", "%[q]", "%[s2]", "1")
                CUR("%[f2]", "%[f3]", "%[q]", "%[qn]", "%[s2]", "2") CUR("%[f3]", "%[f0]", "%[qn]", "%[q]", "%[s2]", "3")
                CUR("%[f0]", "%[f1]", "%[q]", "%[qn]", "%[s3]", "0") CUR("%[f1]", "%[f2]", "%[qn]", "%[q]", "%[s3]", "1")
                CUR("%[f2]", "%[f3]", "%[q]", "%[qn]", "%[s3]", "2") CUR("%[f3]", "%[f0]", "%[qn]", "%[q]", "%[s3]", "3")
                : [f0] "+v"(r.f0), [f1] "+v"(r.f1), [f2] "+v"(r.f2), [f3] "+v"(r.f3), [q] "+v"(r.q), [qn] "+v"(r.qn),
                  [dg] "+v"(r.dg), [d] "+v"(r.d), [m] "+v"(r.m), [x] "+v"(r.x), [y] "+v"(r.y), [a0] "+v"(r.a0), [a1] "+v"(r.a1)
                : [s0] "v"(r.s0), [s1] "v"(r.s1), [s2] "v"(r.s2), [s3] "v"(r.s3));
        }
        else if constexpr (K == 1 || K == 5)
        {
            if constexpr (K == 5)
            {
                // per 16 steps: 4 x (global 16-B load, ds_read_b128, ds_write_b128), one wait at the end
                asm volatile("global_load_dwordx4 %[t], %[p], off\n\t"
                             "ds_read_b128 %[u], %[lr]\n\t"
                             : [t] "=&v"(*(int __attribute__((ext_vector_type(4))) *)&r.s0),
                               [u] "=&v"(*(int __attribute__((ext_vector_type(4))) *)&r.x)
                             : [p] "v"(gp + (it & 63) * 4), [lr] "v"(lr));
            }
            asm volatile(
                FUSED("%[f2]", "%[f3]", "%[f0]", "%[s0]") FUSED("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                FUSED("%[f0]", "%[f1]", "%[f2]", "%[s2]") FUSED("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                FUSED("%[f2]", "%[f3]", "%[f0]", "%[s0]") FUSED("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                FUSED("%[f0]", "%[f1]", "%[f2]", "%[s2]") FUSED("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                FUSED("%[f2]", "%[f3]", "%[f0]", "%[s0]") FUSED("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                FUSED("%[f0]", "%[f1]", "%[f2]", "%[s2]") FUSED("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                FUSED("%[f2]", "%[f3]", "%[f0]", "%[s0]") FUSED("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                FUSED("%[f0]", "%[f1]", "%[f2]", "%[s2]") FUSED("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                : [f0] "+v"(r.f0), [f1] "+v"(r.f1), [f2] "+v"(r.f2), [f3] "+v"(r.f3),
                  [d] "+v"(r.d), [m] "+v"(r.m), [x] "+v"(r.x), [y] "+v"(r.y), [a0] "+v"(r.a0), [a1] "+v"(r.a1)
                : [s0] "v"(r.s0), [s1] "v"(r.s1), [s2] "v"(r.s2), [s3] "v"(r.s3));
            if constexpr (K == 5)
            {
                asm volatile("ds_write_b128 %[la], %[v]\n\t"
                             "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
                             :: [la] "v"(la), [v] "v"(*(int __attribute__((ext_vector_type(4))) *)&r.f0) : "memory");
            }
        }
        else if constexpr (K == 2)
        {
            asm volatile(
                SCORE("%[f2]", "%[f3]", "%[f0]", "%[s0]") SCORE("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                SCORE("%[f0]", "%[f1]", "%[f2]", "%[s2]") SCORE("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                SCORE("%[f2]", "%[f3]", "%[f0]", "%[s0]") SCORE("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                SCORE("%[f0]", "%[f1]", "%[f2]", "%[s2]") SCORE("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                SCORE("%[f2]", "%[f3]", "%[f0]", "%[s0]") SCORE("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                SCORE("%[f0]", "%[f1]", "%[f2]", "%[s2]") SCORE("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                SCORE("%[f2]", "%[f3]", "%[f0]", "%[s0]") SCORE("%[f3]", "%[f0]", "%[f1]", "%[s1]")
                SCORE("%[f0]", "%[f1]", "%[f2]", "%[s2]") SCORE("%[f1]", "%[f2]", "%[f3]", "%[s3]")
                : [f0] "+v"(r.f0), [f1] "+v"(r.f1), [f2] "+v"(r.f2), [f3] "+v"(r.f3), [d] "+v"(r.d), [m] "+v"(r.m)
                : [s0] "v"(r.s0), [s1] "v"(r.s1), [s2] "v"(r.s2), [s3] "v"(r.s3));
        }
        else if constexpr (K == 4)
        {
            asm volatile(
                BYTEDIR("%[f2]", "%[f3]", "%[f0]", "%[s0]", "0") BYTEDIR("%[f3]", "%[f0]", "%[f1]", "%[s1]", "1")
                BYTEDIR("%[f0]", "%[f1]", "%[f2]", "%[s2]", "2") BYTEDIR("%[f1]", "%[f2]", "%[f3]", "%[s3]", "3") BYTEINS
                BYTEDIR("%[f2]", "%[f3]", "%[f0]", "%[s0]", "0") BYTEDIR("%[f3]", "%[f0]", "%[f1]", "%[s1]", "1")
                BYTEDIR("%[f0]", "%[f1]", "%[f2]", "%[s2]", "2") BYTEDIR("%[f1]", "%[f2]", "%[f3]", "%[s3]", "3") BYTEINS
                BYTEDIR("%[f2]", "%[f3]", "%[f0]", "%[s0]", "0") BYTEDIR("%[f3]", "%[f0]", "%[f1]", "%[s1]", "1")
                BYTEDIR("%[f0]", "%[f1]", "%[f2]", "%[s2]", "2") BYTEDIR("%[f1]", "%[f2]", "%[f3]", "%[s3]", "3") BYTEINS
                BYTEDIR("%[f2]", "%[f3]", "%[f0]", "%[s0]", "0") BYTEDIR("%[f3]", "%[f0]", "%[f1]", "%[s1]", "1")
                BYTEDIR("%[f0]", "%[f1]", "%[f2]", "%[s2]", "2") BYTEDIR("%[f1]", "%[f2]", "%[f3]", "%[s3]", "3") BYTEINS
                : [f0] "+v"(r.f0), [f1] "+v"(r.f1), [f2] "+v"(r.f2), [f3] "+v"(r.f3),
                  [d] "+v"(r.d), [m] "+v"(r.m), [x] "+v"(r.x), [y] "+v"(r.y), [a0] "+v"(r.a0), [a1] "+v"(r.a1)
                : [s0] "v"(r.s0), [s1] "v"(r.s1), [s2] "v"(r.s2), [s3] "v"(r.s3), [msk] "v"(r.msk));
        }
        else if constexpr (K == 6)
        {
            asm volatile(
                "ds_read_b128 %[u], %[lr]\n\t"
                DIRW("%[f0]", "%[f1]", "%[s0]") DIRW("%[f1]", "%[f2]", "%[s1]") DIRW("%[f2]", "%[f3]", "%[s2]") DIRW("%[f3]", "%[f0]", "%[s3]")
                DIRW("%[f0]", "%[f1]", "%[s0]") DIRW("%[f1]", "%[f2]", "%[s1]") DIRW("%[f2]", "%[f3]", "%[s2]") DIRW("%[f3]", "%[f0]", "%[s3]")
                "ds_read_b128 %[u], %[lr]\n\t"
                DIRW("%[f0]", "%[f1]", "%[s0]") DIRW("%[f1]", "%[f2]", "%[s1]") DIRW("%[f2]", "%[f3]", "%[s2]") DIRW("%[f3]", "%[f0]", "%[s3]")
                DIRW("%[f0]", "%[f1]", "%[s0]") DIRW("%[f1]", "%[f2]", "%[s1]") DIRW("%[f2]", "%[f3]", "%[s2]") DIRW("%[f3]", "%[f0]", "%[s3]")
                "s_waitcnt lgkmcnt(0)\n\t"
                : [f0] "+v"(r.f0), [f1] "+v"(r.f1), [f2] "+v"(r.f2), [f3] "+v"(r.f3),
                  [d] "+v"(r.d), [m] "+v"(r.m), [x] "+v"(r.x), [y] "+v"(r.y), [a0] "+v"(r.a0), [a1] "+v"(r.a1),
                  [u] "=&v"(*(int __attribute__((ext_vector_type(4))) *)&r.s0)
                : [s0] "v"(r.s0), [s1] "v"(r.s1), [s2] "v"(r.s2), [s3] "v"(r.s3), [lr] "v"(lr));
        }
    }
}

// Waves 0..3 run stream KA, waves 4..7 (when the block has 8 waves) stream KB. PA / PB: s_setprio.
template <int KA, int KB, int PA, int PB>
__global__ __launch_bounds__(512) void step_kernel(int iters, long long *out, const int *g, int *sink)
{
    __shared__ int ldsbuf[64 * 4 + 64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    ldsbuf[threadIdx.x & 255] = threadIdx.x;
    __syncthreads();
    Regs r;
    r.f0 = lane; r.f1 = lane + 1; r.f2 = lane * 3; r.f3 = 7; r.q = lane; r.qn = 0; r.dg = 1; r.d = 2; r.m = 3;
    r.x = 4; r.y = 5; r.a0 = 0; r.a1 = 0; r.msk = 0x80808080; r.s0 = g[lane]; r.s1 = g[lane + 1]; r.s2 = 3; r.s3 = 1;
    const bool first = w < 4;
    if (first ? PA : PB) __builtin_amdgcn_s_setprio(3);
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    if (first) run_stream<KA>(iters, r, nullptr, g, lane, ldsbuf);
    else run_stream<KB>(iters, r, nullptr, g, lane, ldsbuf);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    sink[blockIdx.x * blockDim.x + threadIdx.x] = r.f0 + r.f1 + r.f2 + r.f3 + r.a0 + r.a1 + r.q + r.x;
    if (lane == 0)
    {
        const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
        out[2 * (blockIdx.x * 8 + w)] = (long long)(t1 - t0);
        out[2 * (blockIdx.x * 8 + w) + 1] = hw;
    }
}

// Functional check: v_add_u32_dpp / v_max_i32_dpp with wave_shr:1 (bound_ctrl off) leave lane 0 of
// the destination untouched and take lane k-1's src0 elsewhere.
__global__ void sem_kernel(int *o)
{
    const int lane = threadIdx.x;
    int a = 100 + lane, b = 1000 * lane, d = -7, m = -9;
    asm volatile("v_add_u32_dpp %0, %2, %3 " SHR "\n\t"
                 "v_max_i32_dpp %1, %2, %3 " SHR "\n\t"
                 : "+v"(d), "+v"(m) : "v"(a), "v"(b));
    int d2 = -5, m2 = -6;
    asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %2, %3 " SHR " bound_ctrl:1\n\t"
                 "v_max_i32_dpp %1, %2, %3 " SHR " bound_ctrl:1\n\t"
                 : "+v"(d2), "+v"(m2) : "v"(a), "v"(b));
    o[lane] = d;
    o[64 + lane] = m;
    o[128 + lane] = d2;
    o[192 + lane] = m2;
}

template <int KA, int KB, int PA, int PB>
void run(const char *name, int grid, int waves, int *g, int *sink, long long *out)
{
    const int iters = 2048;
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((step_kernel<KA, KB, PA, PB>), dim3(grid), dim3(64 * waves), 0, 0, iters, out, g, sink);
    (void)hipDeviceSynchronize();
    static long long h[2 * 256 * 8];
    (void)hipMemcpy(h, out, sizeof(long long) * 2 * grid * 8, hipMemcpyDeviceToHost);
    double sa = 0, sb = 0;
    int na = 0, nb = 0;
    for (int b = 0; b < grid; ++b)
        for (int w = 0; w < waves; ++w)
        {
            const double c = (double)h[2 * (b * 8 + w)] / (iters * 16.0);
            if (w < 4) { sa += c; ++na; } else { sb += c; ++nb; }
        }
    printf("{\"test\": \"%s\", \"grid\": %d, \"waves\": %d, \"clk_per_step_A\": %.2f, \"clk_per_step_B\": %.2f, \"simd_ids\": \"",
           name, grid, waves, na ? sa / na : 0.0, nb ? sb / nb : 0.0);
    for (int w = 0; w < waves; ++w) printf("%d", (int)((h[2 * w + 1] >> 4) & 3));
    printf("\"}\n");
    fflush(stdout);
}

int main()
{
    int *g, *sink, *o;
    long long *out;
    (void)hipMalloc(&g, 1 << 20);
    (void)hipMemset(g, 1, 1 << 20);
    (void)hipMalloc(&sink, 256 * 512 * 4);
    (void)hipMalloc(&out, sizeof(long long) * 2 * 256 * 8);
    (void)hipMalloc(&o, 256 * 4);
    hipLaunchKernelGGL(sem_kernel, dim3(1), dim3(64), 0, 0, o);
    int h[256];
    (void)hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
    bool ok = h[0] == -7 && h[64] == -9;
    for (int l = 1; l < 64; ++l) ok = ok && h[l] == 100 + l - 1 + 1000 * l && h[64 + l] == 1000 * l;
    printf("{\"test\": \"dpp_lane0_keep\", \"ok\": %s, \"lane0\": [%d, %d], \"lane1\": [%d, %d], \"bc1_lane0\": [%d, %d], \"bc1_lane1\": [%d, %d]}\n",
           ok ? "true" : "false", h[0], h[64], h[1], h[65], h[128], h[192], h[129], h[193]);
    for (int grid : {1, 256})
    {
        run<0, 0, 0, 0>("cur9", grid, 4, g, sink, out);
        run<1, 0, 0, 0>("fused7", grid, 4, g, sink, out);
        run<2, 0, 0, 0>("score3+nop", grid, 4, g, sink, out);
        run<4, 0, 0, 0>("fused_bytedir6", grid, 4, g, sink, out);
        run<5, 0, 0, 0>("fused7+mem", grid, 4, g, sink, out);
        run<6, 0, 0, 0>("dirwave", grid, 4, g, sink, out);
        run<0, 0, 0, 0>("cur9 x2/simd", grid, 8, g, sink, out);
        run<1, 1, 0, 0>("fused7 x2/simd", grid, 8, g, sink, out);
        run<2, 6, 0, 0>("score3 + dirwave", grid, 8, g, sink, out);
        run<2, 6, 1, 0>("score3(prio) + dirwave", grid, 8, g, sink, out);
        run<1, 6, 1, 0>("fused7(prio) + dirwave", grid, 8, g, sink, out);
        run<4, 6, 1, 0>("bytedir(prio) + dirwave", grid, 8, g, sink, out);
    }
    return 0;
}
