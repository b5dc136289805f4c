// Hand-off cost microbenchmark (gfx950, development tool, not part of the product): one wave runs
// bodies of 16 DP steps shaped like the fill kernel's R=1 global step (2 DPP, add, 2 max, 2 x (sub +
// alignbit)) and, per body, one variant of the strip hand-off work. Prints cycles per body.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/handoff.hip -o tools/microbench/handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>

template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, Is...>) { (f(std::integral_constant<int, Is>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

typedef __attribute__((address_space(3))) int lds_int;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i32x4 lds_i32x4;
__device__ __forceinline__ int lds_ld(lds_int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(lds_int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

constexpr int U = 16;

// V: 0 steps only; 1 + lane-63 publish (4 x ds_write_b128); 2 + lane-63 progress word;
//    3 + consumer prefetch (2 ds_read_b32 + readfirstlane next body); 4 = 1+2+3 + cons word;
//    5 + one ds_write_b32 by 16 lanes; 6 + 8 x ds_write_b64 by lane 63; 7 + exec-mask toggling only;
//    8 + one taken uniform branch per body; 9 + 4 x global_load_dwordx4 (text codes) per body;
//    10 + 4 x ds_write_b128 by all lanes; 11 + 1 x ds_write_b128 by lane 63; 12 + 4 x ds_write_b32 by
//    all lanes; 13 + readlane/writelane gather into 16 lanes + one ds_write_b32
template <int V>
__global__ __launch_bounds__(64) void body_kernel(const int *codes, int bodies, int *out, long long *cyc)
{
    __shared__ int ring[4096 + 64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096 + 64; i += 64) ring[i] = i;
    __syncthreads();
    lds_int *R = (lds_int *)ring;
    int F = lane, upPrev = 0, Q = lane * 3;
    unsigned a0 = 0, a1 = 0;
    int T[U];
    sfor<U>([&](auto Qc) { T[decltype(Qc)::value] = (decltype(Qc)::value * 7 + lane) & 15; });
    int pfProg = 0, pfVal = 0, sink = 0;
    long long t0 = clock64();
    for (int b = 0; b < bodies; ++b)
    {
        int Fs[U];
        if constexpr (V == 9)
        {
            sfor<U / 4>([&](auto Qc) {
                constexpr int q = decltype(Qc)::value * 4;
                const i32x4 v = *(const i32x4 *)(codes + ((b * U + q) & 1023) - lane + 64);
                T[q] += v.x; T[q + 1] += v.y; T[q + 2] += v.z; T[q + 3] += v.w;
            });
        }
        sfor<U>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value;
            const int Qn = __builtin_amdgcn_mov_dpp(Q, 0x130, 0xf, 0xf, true);
            int up = __builtin_amdgcn_update_dpp(Q, F, 0x138, 0xf, 0xf, false);
            Q = Qn;
            const int diag = upPrev;
            upPrev = up;
            const int D = diag + T[q];
            const int M = max(F, up);
            const int Fn = max(D, M);
            a0 = __builtin_amdgcn_alignbit(a0, (unsigned)(M - D), 31);
            a1 = __builtin_amdgcn_alignbit(a1, (unsigned)(F - up), 31);
            F = Fn;
            Fs[q] = Fn;
        });
        if constexpr (V == 3 || V == 4)
        {
            const int pv = __builtin_amdgcn_readfirstlane(pfProg);
            Q = pv > b ? pfVal : 0;
        }
        else
        {
            asm volatile("v_mov_b32 %0, %1" : "=v"(Q) : "v"(lane));
        }
        if constexpr (V == 1 || V == 4)
        {
            if (lane == 63)
            {
                lds_i32x4 *dst = (lds_i32x4 *)(R + ((b * U) & 2047));
                sfor<U / 4>([&](auto Xc) {
                    constexpr int x = decltype(Xc)::value;
                    dst[x] = i32x4{Fs[4 * x], Fs[4 * x + 1], Fs[4 * x + 2], Fs[4 * x + 3]};
                });
            }
        }
        if constexpr (V == 2 || V == 4)
        {
            asm volatile("" ::: "memory");
            if (lane == 63) lds_st(R + 4096, b);
        }
        if constexpr (V == 4)
        {
            if (lane == 0) lds_st(R + 4097, b);
        }
        if constexpr (V == 3 || V == 4)
        {
            pfProg = lds_ld(R + 4096);
            pfVal = lds_ld(R + ((b * U + lane) & 2047));
        }
        if constexpr (V == 5)
        {
            if (lane >= 48) lds_st(R + ((b * U + lane) & 2047), Fs[lane & 15 ? 3 : 5]);
        }
        if constexpr (V == 6)
        {
            if (lane == 63)
            {
                typedef int i32x2 __attribute__((ext_vector_type(2)));
                typedef __attribute__((address_space(3))) i32x2 lds_i32x2;
                lds_i32x2 *dst = (lds_i32x2 *)(R + ((b * U) & 2047));
                sfor<U / 2>([&](auto Xc) {
                    constexpr int x = decltype(Xc)::value;
                    dst[x] = i32x2{Fs[2 * x], Fs[2 * x + 1]};
                });
            }
        }
        if constexpr (V == 7)
        {
            if (lane == 63) asm volatile("v_add_u32 %0, %0, 1" : "+v"(sink));
        }
        if constexpr (V == 8)
        {
            if (__builtin_amdgcn_readfirstlane(F) == 123456789) sink += 1;
        }
        if constexpr (V == 10)
        {
            // 4 x ds_write_b128 by every lane (no exec mask), lane-distinct addresses
            lds_i32x4 *dst = (lds_i32x4 *)(R + ((b * U * 4 + lane * 16) & 4095));
            sfor<U / 4>([&](auto Xc) {
                constexpr int x = decltype(Xc)::value;
                dst[x] = i32x4{Fs[4 * x], Fs[4 * x + 1], Fs[4 * x + 2], Fs[4 * x + 3]};
            });
        }
        if constexpr (V == 11)
        {
            // one ds_write_b128 by lane 63
            if (lane == 63) *(lds_i32x4 *)(R + ((b * U) & 2047)) = i32x4{Fs[0], Fs[5], Fs[10], Fs[15]};
        }
        if constexpr (V == 12)
        {
            // 4 x ds_write_b32 by every lane (no exec mask)
            sfor<4>([&](auto Xc) {
                constexpr int x = decltype(Xc)::value;
                lds_st(R + ((b * U * 4 + x * 64 + lane) & 4095), Fs[4 * x + 3]);
            });
        }
        if constexpr (V == 13)
        {
            // 16 x v_readlane + v_writelane gather of lane 63's values into lanes 0..15, one ds_write_b32
            int G = 0;
#define WL(q) { const int v = __builtin_amdgcn_readlane(Fs[q], 63); asm volatile("v_writelane_b32 %0, %1, " #q : "+v"(G) : "s"(v)); }
            WL(0) WL(1) WL(2) WL(3) WL(4) WL(5) WL(6) WL(7) WL(8) WL(9) WL(10) WL(11) WL(12) WL(13) WL(14) WL(15)
#undef WL
            lds_st(R + ((b * U + lane) & 2047), G);
        }
        sink += Fs[(b & 3)];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t1 = clock64();
    out[lane] = F + (int)a0 + (int)a1 + sink + Q;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
void run(const int *codes, int *out, long long *cyc)
{
    const int bodies = 4096;
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(body_kernel<V>, dim3(1), dim3(64), 0, 0, codes, bodies, out, cyc);
    (void)hipDeviceSynchronize();
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"variant\": %d, \"clk_per_body\": %.1f, \"clk_per_step\": %.2f}\n", V, (double)c / bodies, (double)c / bodies / U);
    fflush(stdout);
}

int main()
{
    int *out, *codes;
    long long *cyc;
    (void)hipMalloc(&out, 64 * 4);
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&codes, 4096 * 4);
    (void)hipMemset(codes, 0, 4096 * 4);
    run<0>(codes, out, cyc); run<1>(codes, out, cyc); run<2>(codes, out, cyc); run<3>(codes, out, cyc);
    run<4>(codes, out, cyc); run<5>(codes, out, cyc); run<6>(codes, out, cyc); run<7>(codes, out, cyc);
    run<8>(codes, out, cyc); run<9>(codes, out, cyc); run<10>(codes, out, cyc); run<11>(codes, out, cyc);
    run<12>(codes, out, cyc); run<13>(codes, out, cyc);
    return 0;
}
