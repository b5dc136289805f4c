// Development microbenchmark: ds_read_b128 at 4-byte (not 16-byte) aligned LDS addresses on gfx950 --
// (1) correctness of the returned dwords, (2) issue cost per wave-instruction for the band fill's code
// pattern (lane k reads row (letter_k, k & 3) of 16 profile rows at byte offset x - (k & ~3)), against
// 16-byte aligned reads of the same rows. One wave per SIMD, 4 waves per workgroup, one workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kRow = 2048 + 256;
typedef int i4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_check(int *bad)
{
    __shared__ unsigned char lds[16 * kRow];
    for (int i = threadIdx.x; i < 16 * kRow; i += blockDim.x) lds[i] = (unsigned char)(i * 7 + (i >> 8));
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int nbad = 0;
    for (int base = 0; base < 256; base += 4)
    {
        const unsigned addr = (unsigned)((lane & 15) * kRow + base + 4 * (lane >> 4) + 64);
        i4 v;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
        for (int d = 0; d < 4; ++d)
        {
            unsigned e = 0;
            for (int b = 0; b < 4; ++b) e |= (unsigned)lds[addr + 4 * d + b] << (8 * b);
            if ((unsigned)v[d] != e) ++nbad;
        }
    }
    atomicAdd(bad, nbad);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_time(const int *letters, long long *clk, int *sink)
{
    __shared__ unsigned char lds[16 * kRow];
    for (int i = threadIdx.x; i < 16 * kRow; i += blockDim.x) lds[i] = (unsigned char)i;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int c0 = letters[(w * 64 + lane) * 2], c1 = letters[(w * 64 + lane) * 2 + 1];
    // MODE 0: the band pattern (4-byte aligned); MODE 1: the same rows, 16-byte aligned offsets
    const int d = MODE == 0 ? 64 - (lane & ~3) : 64 - 4 * (lane & ~3) / 4 / 4 * 4;
    unsigned a0 = (unsigned)((c0 * 4 + (lane & 3)) * kRow + d + (MODE == 1 ? 0 : 0));
    unsigned a1 = (unsigned)((c1 * 4 + (lane & 3)) * kRow + d);
    if (MODE == 1)
    {
        a0 &= ~15u;
        a1 &= ~15u;
    }
    i4 acc = {0, 0, 0, 0};
    const long long t0 = clock64();
    for (int it = 0; it < 1024; ++it)
    {
        i4 x, y;
        const unsigned o = (unsigned)((it * 16) & 2047);
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x), "=&v"(y) : "v"(a0 + o), "v"(a1 + o));
        acc += x ^ y;
    }
    const long long t1 = clock64();
    if (lane == 0) clk[blockIdx.x * 4 + w] = t1 - t0;
    sink[threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main()
{
    int *bad;
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    k_check<<<1, 256>>>(bad);
    int hb = -1;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"test\": \"ds_read_b128 4-byte aligned\", \"mismatched_dwords\": %d}\n", hb);
    std::vector<int> L(256 * 2);
    srand(5);
    for (auto &x : L) x = rand() % 4;
    int *dL, *sink;
    long long *clk;
    hipMalloc(&dL, L.size() * 4);
    hipMalloc(&clk, 8 * 4);
    hipMalloc(&sink, 256 * 4);
    hipMemcpy(dL, L.data(), L.size() * 4, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 2; ++mode)
    {
        for (int rep = 0; rep < 2; ++rep)
        {
            if (mode == 0) k_time<0><<<1, 256>>>(dL, clk, sink);
            else k_time<1><<<1, 256>>>(dL, clk, sink);
            hipDeviceSynchronize();
        }
        long long h[4];
        hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        printf("{\"mode\": \"%s\", \"clk_per_pair_with_wait\": [%.1f, %.1f, %.1f, %.1f]}\n", mode == 0 ? "band 4B-aligned" : "16B-aligned",
               h[0] / 1024.0, h[1] / 1024.0, h[2] / 1024.0, h[3] / 1024.0);
    }
    return hb == 0 ? 0 : 1;
}
