// Lone-wave cost of one band body by text-code source (development tool; see gen_bodybench.py).
//   python3 tools/microbench/gen_bodybench.py && hipcc -O3 --offload-arch=gfx950 \
//       tools/microbench/bodybench.hip -o tools/microbench/bodybench
// One wave per SIMD (4 waves per workgroup, one workgroup per CU, 256 workgroups); LDS holds 16 rows
// of 2304 bytes (row stride 2368: 16 dwords mod 64 banks) like the staged band codes would.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "bodybench.inc"

constexpr int kStride = 2368;
#define CLOBBER                                                                                              \
    "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", \
        "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v40", "v41", "v42", "v43", "v44", "v45", "v46",   \
        "v47", "v48", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "scc", "memory"

#define RUN(BODYSEL) \
    asm volatile( \
        "v_mov_b32 v41, %[pfa]\n\tv_mov_b32 v42, %[paddr]\n\tv_mov_b32 v43, 0x80000000\n\tv_mov_b32 v45, %[va]\n\t" \
        "v_mov_b32 v46, %[vb]\n\tv_mov_b32 v47, %[la]\n\tv_mov_b32 v48, %[lb]\n\ts_mov_b32 s22, 0\n\ts_mov_b32 s23, 0\n\t" \
        "s_mov_b64 s[24:25], %[cp]\n\ts_mov_b32 s26, 0x100000\n\ts_mov_b32 s27, 0x20000\n\ts_mov_b32 s28, 0\n\ts_mov_b32 s29, %[it]\n\t" \
        "v_mov_b32 v10, 0\n\tv_mov_b32 v11, 0\n\tv_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\tv_mov_b32 v14, 0\n\t" \
        "v_mov_b32 v15, 0\n\tv_mov_b32 v16, 0\n\tv_mov_b32 v17, 0\n\t" \
        "1:\n\t" BODYSEL "\n\ts_and_b32 s28, s28, %[mask]\n\ts_sub_u32 s29, s29, 1\n\ts_cmp_lg_u32 s29, 0\n\ts_cbranch_scc1 1b\n\t" \
        "s_waitcnt vmcnt(0) lgkmcnt(0)" \
        : \
        : [pfa] "v"(pfa), [paddr] "v"(paddr), [va] "v"(va), [vb] "v"(vb), [la] "v"(la), [lb] "v"(lb), \
          [cp] "s"(codes), [it] "s"(iters), [mask] "s"(mask) \
        : CLOBBER);

template <int V>
__global__ __launch_bounds__(256) void k_body(const int *codes, const int *letters, int iters, int mask, long long *out)
{
    extern __shared__ int lds[];
    for (int i = threadIdx.x; i < 16 * kStride / 4 + 4096; i += blockDim.x) lds[i] = i;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = letters[(w * 64 + lane) * 2], c1 = letters[(w * 64 + lane) * 2 + 1];
    const int ring = 16 * kStride;  // feed ring and publish slots after the code rows
    const unsigned pfa = (unsigned)(ring + 4 * lane), paddr = (unsigned)(ring + 8192 + 4 * lane);
    unsigned la = (unsigned)((c0 * 4 + (lane & 3)) * kStride + 64 - (lane & ~3));
    unsigned lb = (unsigned)((c1 * 4 + (lane & 3)) * kStride + 64 - (lane & ~3));
    if (V == 3)
    {
        la &= ~15u;
        lb &= ~15u;
    }
    const unsigned va = (unsigned)((c0 * 4 + (lane & 3)) * 65536 + 64 - (lane & ~3));
    const unsigned vb = (unsigned)((c1 * 4 + (lane & 3)) * 65536 + 64 - (lane & ~3));
    uint64_t t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    if constexpr (V == 0) RUN(BODY_NONE)
    else if constexpr (V == 1) RUN(BODY_BUF)
    else if constexpr (V == 2) RUN(BODY_DS2)
    else if constexpr (V == 3) RUN(BODY_B128)
    else RUN(BODY_B128U)
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
    if (lane == 0) out[blockIdx.x * 4 + w] = (long long)(t1 - t0);
}

int main()
{
    const char *names[] = {"none", "buf", "ds2", "b128", "b128u", "buf_l2"};
    int *codes, *letters;
    long long *out;
    (void)hipMalloc(&codes, 16 * 65536);
    (void)hipMemset(codes, 1, 16 * 65536);
    (void)hipMalloc(&letters, 512 * 4);
    int h[512];
    unsigned x = 12345;
    for (int &v : h) v = (x = x * 1103515245u + 12345u) >> 16 & 3;
    (void)hipMemcpy(letters, h, sizeof(h), hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 256 * 4 * 8);
    const int iters = 4096, grid = 256;
    const size_t lds = (16 * kStride / 4 + 4096) * 4;
    for (int vv = 0; vv < 6; ++vv)
    {
        const int v = vv == 5 ? 1 : vv, mask = vv == 5 ? 0xffff : 0xfff;
        for (int rep = 0; rep < 2; ++rep)
        {
            switch (v)
            {
            case 0: hipLaunchKernelGGL(k_body<0>, dim3(grid), dim3(256), lds, 0, codes, letters, iters, mask, out); break;
            case 1: hipLaunchKernelGGL(k_body<1>, dim3(grid), dim3(256), lds, 0, codes, letters, iters, mask, out); break;
            case 2: hipLaunchKernelGGL(k_body<2>, dim3(grid), dim3(256), lds, 0, codes, letters, iters, mask, out); break;
            case 3: hipLaunchKernelGGL(k_body<3>, dim3(grid), dim3(256), lds, 0, codes, letters, iters, mask, out); break;
            default: hipLaunchKernelGGL(k_body<4>, dim3(grid), dim3(256), lds, 0, codes, letters, iters, mask, out); break;
            }
            (void)hipDeviceSynchronize();
        }
        static long long hh[256 * 4];
        (void)hipMemcpy(hh, out, sizeof(hh), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < grid * 4; ++i) s += (double)hh[i] / ((double)iters * 32);
        printf("{\"codes\": \"%s\", \"clk_per_step\": %.2f}\n", names[vv], s / (grid * 4));
    }
    return 0;
}
