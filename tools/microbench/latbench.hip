// Dependent-chain latency of single VALU / DPP / ballot instructions for one wave64 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ __launch_bounds__(64) void lat_kernel(int iters, int x, int *out, long long *cyc)
{
    int F = threadIdx.x, G = threadIdx.x * 3;
    uint64_t acc = 0;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
    {
#pragma unroll
        for (int k = 0; k < 16; ++k)
        {
            if constexpr (K == 0) F = max(F, G + k);                                   // v_max chain
            if constexpr (K == 1) F = __builtin_amdgcn_update_dpp(G, F, 0x138, 0xf, 0xf, false);  // wave_shr:1
            if constexpr (K == 2) F = __builtin_amdgcn_update_dpp(G, F, 0x111, 0xf, 0xf, false);  // row_shr:1
            if constexpr (K == 3) F = __builtin_amdgcn_update_dpp(G, F, 0x134, 0xf, 0xf, false);  // wave_rol:1
            if constexpr (K == 4) { F = max(__builtin_amdgcn_update_dpp(G, F, 0x138, 0xf, 0xf, false), x); }
            if constexpr (K == 5) { F = max(__builtin_amdgcn_update_dpp(G, F, 0x111, 0xf, 0xf, false), x); }
            if constexpr (K == 6) { acc += __builtin_amdgcn_ballot_w64(F > k); F += (int)acc; }  // cmp -> salu -> valu
            if constexpr (K == 7) F = F + G;                                             // v_add chain
            if constexpr (K == 8) F = __builtin_amdgcn_mov_dpp(F, 0x138, 0xf, 0xf, true);  // wave_shr bound_ctrl
        }
    }
    long long t1 = clock64();
    out[blockIdx.x * 64 + threadIdx.x] = F + (int)acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(int *out, long long *cyc)
{
    const int iters = 4096;
    hipLaunchKernelGGL(lat_kernel<K>, dim3(1), dim3(64), 0, 0, iters, 7, out, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(lat_kernel<K>, dim3(1), dim3(64), 0, 0, iters, 7, out, cyc);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"chain\": %d, \"clk_per_link\": %.2f}\n", K, (double)c / (iters * 16.0));
}

int main()
{
    int *out; long long *cyc;
    (void)hipMalloc(&out, 64 * 4);
    (void)hipMalloc(&cyc, 8);
    run<0>(out, cyc); run<1>(out, cyc); run<2>(out, cyc); run<3>(out, cyc); run<4>(out, cyc);
    run<5>(out, cyc); run<6>(out, cyc); run<7>(out, cyc); run<8>(out, cyc);
    return 0;
}
