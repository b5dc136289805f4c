// Wave-level helpers shared by the fill (sa_engine.hip) and traceback (sa_walk.hip) kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <utility>

#include "sa_layout.h"

namespace sa {

// ------------------------------------------------------------------------------------------------
// wave-level helpers
// ------------------------------------------------------------------------------------------------
template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, Is...>)
{
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f)
{
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// DPP lane moves (GFX9 wavefront shifts). wave_shr:1 — lane i reads lane i-1, lane 0 keeps `old`;
// wave_shl:1 — lane i reads lane i+1, lane 63 keeps `old`; wave_rol:1 — lane i reads lane i+1 mod 64.
__device__ __forceinline__ int dpp_shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int dpp_shl1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false); }
__device__ __forceinline__ int dpp_rol1(int src) { return __builtin_amdgcn_update_dpp(src, src, 0x134, 0xf, 0xf, false); }

// v_writelane_b32 through the LLVM intrinsic (clang exposes no builtin), so the compiler's hazard
// recognizer sees it: a v_cmp that writes the SGPR pair needs one wait state before a v_writelane
// reads it, which an inline-asm writelane silently violates (stale ballot bits).
__device__ int amdgcn_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
template <int L>
__device__ __forceinline__ void writelane(uint32_t &acc, uint32_t v)
{
    acc = (uint32_t)amdgcn_writelane((int)v, L, (int)acc);
}

// Direction bits are accumulated per lane, in VGPRs: push_sign shifts a word left by one and moves
// the sign bit of x in (v_alignbit_b32 {acc, x} >> 31), so "a > b" costs one subtraction and one
// alignbit, with no SGPR round trip. After 32 pushes a word holds 32 consecutive (step,row) slots of
// one plane, most recent in bit 0; a chunk of words goes to HBM as one coalesced vector store per
// lane (sa_layout.h). All values are bounded well inside int32, so the differences
// never overflow.
__device__ __forceinline__ uint32_t push_sign(uint32_t acc, int x)
{
    return __builtin_amdgcn_alignbit(acc, (uint32_t)x, 31);
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// Inclusive prefix sum over the wave's lanes (lane l: sum of lanes 0..l): row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast:15 / row_bcast:31 carry the row totals up
__device__ __forceinline__ int wave_prefix_sum(int x)
{
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
template <typename T>
__device__ __forceinline__ T *uniform_ptr(T *p)
{
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (T *)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ bool all_lanes(bool p) { return ballot(p) == ballot(true); }

// Maximum of a 64-bit value over the wave without divergent control flow (readlane into SGPRs).
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
    const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    uint64_t best = 0;
    for (int l = 0; l < kWave; ++l)
    {
        const uint64_t x = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(hi, l) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane(lo, l);
        best = x > best ? x : best;
    }
    return best;
}

__device__ __forceinline__ uint64_t load_granule(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_granule(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace sa
