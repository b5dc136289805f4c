// Fill-kernel interface shared by the fill translation units (sa_fill.hip, one per strip height R:
// fill_r<R>.hip) and the host side (sa_engine.hip): launch arguments, score kinds, launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "sa_hip.h"
#include "sa_layout.h"

namespace sa {

struct FillArgs {
    const int8_t *pattern;      // device pattern arena (alphabet indices)
    const int32_t *codes;       // padded text codes, one dword per letter (8*c packed profile, c otherwise)
    const StripDesc *strips;
    const PairDesc *pairs;
    const int32_t *prof_tab;    // packed profile: one word per pattern letter (A <= 4)
    const int32_t *score_tab;   // generic: A*A scores (+2g for global)
    uint32_t *masks;            // direction entries, viewed as dwords
    uint64_t *bnd;              // hand-off granules
    uint64_t *strip_best;       // local: best-cell key per strip
    int32_t *pair_score;        // global: H[m][n] per pair
    Control *ctrl;
    int32_t num_strips;
    int32_t num_groups;         // ceil(num_strips / W)
    int32_t gap;
    int32_t A;
    uint32_t epoch;
    int32_t key_bits;
    int32_t key_rowbits;        // local best-cell key: H | ~row (key_rowbits) | ~col (key_rowbits)
    uint64_t timeout_ticks;     // hand-off give-up time in s_memrealtime ticks (100 MHz)
    uint64_t *timeline;         // debug (SA_TIMELINE): per strip {start, fed, end, hw id}, or null
    int32_t io_sleep;           // I/O wave idle poll period, in units of s_sleep 1 (64 clocks)
    int32_t chain_lds;          // chain launches: dynamic LDS bytes (>= group_lds_bytes(W); more
                                // than half a CU's LDS keeps one workgroup per CU)
    // BAND fill (R = 1 int8-profile chains, sa_fill.hip process_band): 128-row score strips (bands)
    // run the recurrence alone on workgroups [0, band_wgs) and feed the 64-row strips, which the other
    // workgroups run in groups of W (the first strip of a group from the band above's granules)
    const StripDesc *bands;     // the bands (null / num_bands = 0: no band fill)
    int32_t num_bands;
    int32_t num_band_groups;    // ceil(num_bands / W)
    int32_t band_wgs;
    int32_t pair_text_len;      // pair-packed chains (fill_pair_chain_kernel): the pairs' common text length
};

constexpr int kTimelineWords = 48;  // SA_TIMELINE record per strip, then per band (words 6..37: experiment progress stamps)
constexpr int kMaxWaves = 4;       // compute waves per chain workgroup (+1 I/O wave: 320 threads; one
                                   // compute wave per SIMD: two per SIMD ran 2.2x slower per step)
constexpr int kPairWaves = 4;      // waves per workgroup of the pair-packed batch kernel
constexpr int kPairChainMax = 8;   // strips per pair (waves per workgroup) of a pair-packed chain
constexpr int kPairFeedOff = 64;   // LDS row entry of column c: c + kPairFeedOff (c >= -63)
// (entries: columns -63 .. n + 2U published, and every lane of a consumer's feed read up to column
// nSteps + 63 <= n + 2U + 126)
__host__ __device__ constexpr int pair_row_entries(int n) { return (n + kPairFeedOff + 4 * kWave + 63) / 64 * 64; }


// Where a strip's substitution scores come from (SK). Every table already holds S + 2g (global) or
// S + g (local), the offsets the recurrences below fold in:
//   kProf   DNA-sized alphabets, R > 1: a per-row packed profile (four int8 scores in one VGPR)
//           selected by v_bfe_i32 with the text code 8*c;
//   kTable  other alphabets, R > 1: the A x A table in LDS indexed by row letter * A + text letter;
//   kArr    R = 1: per-letter score arrays over the text ("text profiles": arr[a][x] = S[a][t[x]]),
//           zero padded on both sides, so the load delivers the score itself;
//   kArr8   R = 1 when the scores fit int8: the same profiles as bytes, four byte-shifted copies
//           per letter so that every lane's 16-byte load is dword aligned (lane k reads copy k%4);
//           one global_load_dwordx4 serves a whole 16-step body and the byte is picked by the
//           add itself (SDWA src1_sel:BYTE_q, sign-extended).
//   kPair   pair-packed strips (fill_pair_kernel; chains: fill_pair_chain_kernel): per column the
//           two pairs' column profiles.
//   kArr8A  (a launch selector, not a plan's kind) kArr8 chains of alphabets larger than 4: every
//           lane reads copy 0 of its letters only, dword aligned, and shifts the bytes into place
//           with v_alignbyte (fill_r1a.hip, launch_fill_align). A wave's 64 lanes then touch one
//           array per letter instead of one per letter and copy: the CU's L1 holds the working set.
// The zero padding of the profiles keeps the ramp cells left of column 1 at the boundary value.
enum ScoreKind { kProf = 0, kTable = 1, kArr = 2, kArr8 = 3, kPair = 4, kArr8A = 5 };
template <int SK>
constexpr bool kIsArr = SK == kArr || SK == kArr8;

// Fill launch for strip height R (instantiated in fill_r<R>.hip).
template <int R>
void launch_fill_r(const FillArgs &a, bool local, int sk, int grid, int W, bool chain, hipStream_t st);
// R = 1 kArr8 chains read through copy 0 (kArr8A; fill_r1a.hip, a code object of its own so that the
// DNA kernels' code and placement stay as they are)
void launch_fill_align(const FillArgs &a, bool local, int grid, int W, hipStream_t st);
#ifndef SA_FILL_R
extern template void launch_fill_r<1>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<2>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<4>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<8>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<16>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<32>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
#endif

}  // namespace sa
