// Fill-step microbenchmark (gfx950): cost per DP step of one wave64 for several formulations of
// the R=1 global step, to decide the fill kernel's per-step instruction mix. Not part of the
// product; results recorded in DESIGN.md / profiles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <utility>

template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, Is...>) { (f(std::integral_constant<int, Is>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

__device__ __forceinline__ int dpp_shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int dpp_shl1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false); }
__device__ __forceinline__ int dpp_rol1(int src) { return __builtin_amdgcn_update_dpp(src, src, 0x134, 0xf, 0xf, false); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) int lds_int;
typedef __attribute__((address_space(3))) i32x4 lds_i32x4;

template <int OFF>
__device__ __forceinline__ void sstore(uint32_t *base, uint64_t p0, uint64_t p1, bool nop)
{
    const u32x4 v = {(uint32_t)p0, (uint32_t)(p0 >> 32), (uint32_t)p1, (uint32_t)(p1 >> 32)};
    if (nop) asm volatile("s_store_dwordx4 %0, %1, %2\n\ts_nop 0" ::"s"(v), "s"(base), "i"(OFF) : "memory");
    else asm volatile("s_store_dwordx4 %0, %1, %2" ::"s"(v), "s"(base), "i"(OFF) : "memory");
}
template <typename T>
__device__ __forceinline__ T *uniform_ptr(T *p)
{
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (T *)(((uint64_t)hi << 32) | lo);
}

constexpr int U = 16;

// V: 0 current v1 step; 1 v1 without direction store; 2 v1, store without s_nop;
//    3 lean (LDS feed in place, ds_write bottom row, raw planes); 4 lean without store;
//    5 lean with dword codes (dwordx4 per 4 steps); 6 = 5 without store; 7 = 5 local-mode (H domain + 0 clamp)
template <int V>
__global__ __launch_bounds__(64) void step_kernel(const int8_t *codes8, const int *codes32, uint32_t *masks, int nsteps, int prof, int *out, long long *cyc)
{
    __shared__ int ring[2048 + 128];
    const int lane = threadIdx.x;
    for (int i = lane; i < 2048 + 128; i += 64) ring[i] = i * 3;
    __syncthreads();
    uint32_t *mk = masks + (size_t)blockIdx.x * nsteps * 4;
    const int8_t *c8 = codes8 + 64;
    const int *c32 = codes32 + 64;
    int F = 0, upPrev = 0, FB = lane, O = 0, G = -5;
    uint64_t sink = 0;
    long long t0 = clock64();
    int T[U], Tn[U], X[U];
    uint64_t P0[3], P1[3];
    int pfp = 0, pfv = 0;
    constexpr bool LEAN = V >= 3;
    constexpr bool DW = V >= 5;
    (void)P0; (void)P1;
    sfor<U>([&](auto Q) { constexpr int q = decltype(Q)::value; T[q] = DW ? c32[q - lane] : c8[q - lane]; });
    volatile lds_int *R = (volatile lds_int *)ring;
    for (int s0 = 0; s0 < nsteps; s0 += U)
    {
        const int s1 = s0 + U;
        if constexpr (DW)
        {
            sfor<U / 4>([&](auto Q) {
                constexpr int q = decltype(Q)::value * 4;
                typedef int i4u __attribute__((ext_vector_type(4), aligned(4)));
                const i4u v = *(const i4u *)(c32 + s1 + q - lane);
                Tn[q] = v.x; Tn[q + 1] = v.y; Tn[q + 2] = v.z; Tn[q + 3] = v.w;
            });
        }
        else
        {
            sfor<U>([&](auto Q) { constexpr int q = decltype(Q)::value; Tn[q] = c8[s1 + q - lane]; });
        }
        if constexpr (LEAN)
        {
            sfor<U / 4>([&](auto Q) {
                constexpr int q = decltype(Q)::value * 4;
                const i32x4 v = *(volatile lds_i32x4 *)(R + ((s0 + q) & 2047));
                X[q] = v.x; X[q + 1] = v.y; X[q + 2] = v.z; X[q + 3] = v.w;
            });
        }
        uint32_t *mbase = uniform_ptr(mk + (size_t)s0 * 4);
        volatile lds_int *wr = R + ((s0 & 2047) + (lane == 63 ? 0 : 2048 + 64 - lane));
        sfor<U>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            const int sc = __builtin_amdgcn_sbfe(prof, T[q], 8);
            int up;
            if constexpr (LEAN) up = dpp_shr1(X[q], F);
            else { up = dpp_shr1(FB, F); FB = dpp_rol1(FB); }
            const int diag = upPrev;
            upPrev = up;
            uint64_t p0, p1;
            if constexpr (V == 7)
            {
                const int gu = up - 5;
                const int D = diag + sc;
                const int M = max(G, gu);
                const int Hn = max(max(D, M), 0);
                p0 = ballot(D > M);
                p1 = ballot(gu > G);
                G = Hn - 5;
                F = Hn;
            }
            else
            {
                const int left = F;
                const int D = diag + sc;
                const int M = max(left, up);
                const int Fn = max(D, M);
                p0 = ballot(D > M);
                p1 = ballot(up > left);
                if constexpr (!LEAN) p1 &= ~p0;
                F = Fn;
            }
            if constexpr (V == 1 || V == 4 || V == 6) sink ^= p0 ^ (p1 << 1);
            else if constexpr (V == 8 || V == 9)
            {
                // software-pipelined: store the ballots of step q-DL (their SGPRs are long ready)
                constexpr int DL = V == 8 ? 1 : 2;
                if constexpr (q >= DL) sstore<(q - DL) * 16>(mbase, P0[(q - DL) % 3], P1[(q - DL) % 3], true);
                P0[q % 3] = p0;
                P1[q % 3] = p1;
            }
            else sstore<q * 16>(mbase, p0, p1, V != 2);
            if constexpr (LEAN) wr[q] = F;
            else O = dpp_shl1(F, O);
        });
        if constexpr (V == 8 || V == 9)
        {
            constexpr int DL = V == 8 ? 1 : 2;
            sfor<DL>([&](auto Q) {
                constexpr int q = U - DL + decltype(Q)::value;
                sstore<q * 16>(mbase, P0[q % 3], P1[q % 3], true);
            });
        }
        if constexpr (V == 10)
        {
            const int pv = __builtin_amdgcn_readfirstlane(R[2048 + 100]);
            if (pv == 12345) F += 1;
        }
        if constexpr (V == 13 || V == 15)
        {
            // producer: lanes 48..63 publish 16 columns, lane 63 the progress word
            typedef __attribute__((address_space(3))) int li;
            if (lane >= 48) __hip_atomic_store((li *)(ring + ((s0 + lane) & 2047)), O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lane == 63) __hip_atomic_store((li *)(ring + 2048 + 100), s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (V == 14 || V == 15)
        {
            typedef __attribute__((address_space(3))) int li;
            const int pv = __builtin_amdgcn_readfirstlane(pfp);
            if (pv == 12345) F += 1;
            FB = lane < 16 ? pfv : FB;
            pfp = __hip_atomic_load((li *)(ring + 2048 + 101), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            pfv = __hip_atomic_load((li *)(ring + ((s0 + lane) & 2047)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lane == 0) __hip_atomic_store((li *)(ring + 2048 + 102), s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (V == 11)
        {
            if (lane >= 48) __hip_atomic_store((uint64_t *)(masks + 64) + (s0 & 1023) + lane, (uint64_t)F, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (V == 12)
        {
            if (lane >= 48) ((uint64_t *)(masks + 64))[(s0 & 1023) + lane] = (uint64_t)F;
        }
        sfor<U>([&](auto Q) { constexpr int q = decltype(Q)::value; T[q] = Tn[q]; });
    }
    __builtin_amdgcn_s_dcache_wb();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    out[blockIdx.x * 64 + lane] = F + O + (int)sink + FB;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
void run(int blocks, int nsteps, int8_t *c8, int *c32, uint32_t *mk, int *out, long long *cyc)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(step_kernel<V>, dim3(blocks), dim3(64), 0, 0, c8, c32, mk, nsteps, 0x05fcfcfc, out, cyc);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r)
    {
        hipEventRecord(e0);
        hipLaunchKernelGGL(step_kernel<V>, dim3(blocks), dim3(64), 0, 0, c8, c32, mk, nsteps, 0x05fcfcfc, out, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"variant\": %d, \"blocks\": %d, \"ns_per_step\": %.2f, \"clk_per_step\": %.1f}\n", V, blocks, best * 1e6 / nsteps, (double)c / nsteps);
}

int main(int argc, char **argv)
{
    const int nsteps = 1 << 16;
    int8_t *c8; int *c32; uint32_t *mk; int *out; long long *cyc;
    const int maxb = 1024;
    hipMalloc(&c8, nsteps + 256);
    hipMalloc(&c32, (nsteps + 256) * 4);
    hipMemset(c8, 8, nsteps + 256);
    hipMemset(c32, 0, (nsteps + 256) * 4);
    hipMalloc(&mk, (size_t)maxb * nsteps * 16 + 64);
    hipMalloc(&out, maxb * 64 * 4);
    hipMalloc(&cyc, maxb * 8);
    for (int blocks : {1})
    {
        run<0>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<1>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<2>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<3>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<4>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<5>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<6>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<7>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<8>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<9>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<10>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<11>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<12>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<13>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<14>(blocks, nsteps, c8, c32, mk, out, cyc);
        run<15>(blocks, nsteps, c8, c32, mk, out, cyc);
    }
    return 0;
}
