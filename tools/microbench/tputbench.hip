// Issue cost of single instruction kinds for one wave64 on gfx950 (independent instructions,
// inline asm so the sequence is exact). Cycles per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
template <int K>
__global__ __launch_bounds__(64) void tput_kernel(int iters, int *out, long long *cyc, uint32_t *mem)
{
    int a = threadIdx.x, b = threadIdx.x * 3, c = 5, d = 9;
    long long t0 = clock64();
    __shared__ int lds[256];
    const uint64_t pv = (uint64_t)mem;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pv);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pv >> 32));
    uint32_t *base = (uint32_t *)(((uint64_t)hi << 32) | lo);
    int la = (int)(uint32_t)(uint64_t)(lds + threadIdx.x);  // LDS byte address of this lane's slot
    for (int i = 0; i < iters; ++i)
    {
        if constexpr (K == 0) asm volatile(R8("v_max_i32 %0, %1, %2\n\tv_max_i32 %2, %1, %3\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if constexpr (K == 1) asm volatile(R8("v_cmp_gt_i32 s[20:21], %0, %1\n\tv_cmp_gt_i32 s[22:23], %2, %3\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "s20","s21","s22","s23");
        if constexpr (K == 2) asm volatile(R8("v_cmp_gt_i32 vcc, %0, %1\n\tv_max_i32 %2, %1, %3\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "vcc");
        if constexpr (K == 3) asm volatile(R8("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if constexpr (K == 4) asm volatile(R8("v_cmp_gt_i32 s[20:21], %0, %1\n\tv_max_i32 %2, %1, %3\n\ts_and_b64 s[24:25], s[20:21], s[22:23]\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "s20","s21","s22","s23","s24","s25","scc");
        if constexpr (K == 6) asm volatile(R8("s_nop 0\n\tv_max_i32 %2, %1, %3\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if constexpr (K == 7) asm volatile(R8("ds_write_b32 %4, %1\n\tv_max_i32 %2, %1, %3\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(la) : "memory");
        if constexpr (K == 10) asm volatile(R8("v_max_i32 %0, %1, %2\n\tv_max_i32 %2, %1, %3\n\ts_and_b64 s[24:25], s[20:21], s[22:23]\n\ts_or_b64 s[26:27], s[20:21], s[22:23]\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "s20","s21","s22","s23","s24","s25","s26","s27","scc");
        if constexpr (K == 11) asm volatile(R8("v_max_i32 %0, %1, %2\n\tv_max_i32 %3, %1, %1\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        if constexpr (K == 9) asm volatile(R8("v_max_i32 %0, %1, %2\n\ts_and_b64 s[24:25], s[20:21], s[22:23]\n\t") : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "s20","s21","s22","s23","s24","s25","scc");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    out[threadIdx.x] = a + b + c + d + lds[threadIdx.x];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int K>
void run(int *out, long long *cyc, uint32_t *mem, int per)
{
    const int iters = 4096;
    hipLaunchKernelGGL(tput_kernel<K>, dim3(1), dim3(64), 0, 0, iters, out, cyc, mem);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(tput_kernel<K>, dim3(1), dim3(64), 0, 0, iters, out, cyc, mem);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"kind\": %d, \"clk_per_group\": %.2f}\n", K, (double)c / (iters * 8.0));
    fflush(stdout);
    (void)per;
}

int main()
{
    int *out; long long *cyc; uint32_t *mem;
    (void)hipMalloc(&out, 64 * 4);
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&mem, 1 << 20);
    run<0>(out, cyc, mem, 2); run<1>(out, cyc, mem, 2); run<2>(out, cyc, mem, 2); run<3>(out, cyc, mem, 2);
    run<4>(out, cyc, mem, 3); run<6>(out, cyc, mem, 2); run<7>(out, cyc, mem, 2);
    run<9>(out, cyc, mem, 2); run<10>(out, cyc, mem, 4); run<11>(out, cyc, mem, 2);
    return 0;
}
