// MI355X (gfx950 / CDNA4) alignment engine: Needleman-Wunsch / Smith-Waterman DP fill and traceback.
//
// Replaces the reference's GPU path (robertszafa/sequence-alignment-gpu alignSequenceGPU.cu:73-653)
// with a new design; see DESIGN.md and sa_layout.h for the data layout. Semantics follow the
// reference CPU path (alignSequenceCPU.cpp), bit-exact:
//   cell recurrence and tie rule      alignSequenceCPU.cpp:175-190 (local), :259-273 (global)
//   boundaries                        :145-149, :163-164 (local), :232-236, :247-248 (global)
//   local best cell (first max)       :191-192
//   tracebacks                        traceBackNW :64-114, traceBackSW :10-62
//
// Fill kernel (one wave64 per strip; workgroups of W strips + an I/O wave; dynamic group queue):
//   * lane k owns R rows and works on column s-k+1 at step s; the value from the row above
//     arrives by a DPP wave_shr:1 lane shift, lane 0 is fed from the strip above through an LDS
//     ring (inside a workgroup) or epoch-tagged global granules moved by the I/O wave;
//   * the substitution score comes from a per-row profile register (DNA: four int8 scores packed
//     in one VGPR, selected by v_bfe_i32 on the text code) or from an LDS table (protein);
//   * global alignment runs in the shifted domain F = H + g*(i+j), where the recurrence
//     becomes F = max(Fdiag + s + 2g, Fleft, Fup) and every boundary is 0;
//   * the direction of each cell is two bits pushed into per-lane VGPR words (one subtraction and
//     one v_alignbit per bit, no SGPR round trip); every 32 (step,row) slots a lane's words go to
//     HBM in one coalesced vector store per wave.
// Traceback kernel (one wave per pair): a scalar walk over the bit-planes through double-buffered
// LDS windows, then a parallel pass that converts the op string to letters.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "sa_hip.h"
#include "sa_layout.h"

#include "sa_walk.h"
#include "sa_wave.h"

namespace sa {


// ------------------------------------------------------------------------------------------------
// fill kernel
// ------------------------------------------------------------------------------------------------
template <int R>
struct Cfg {
    static constexpr int U = (16 / R) > 4 ? (16 / R) : 4;  // steps per unrolled body
    static constexpr int SB = U * R;                        // (step,row) slots per body
    static constexpr int CS = SB > 32 ? SB : 32;            // slots per stored chunk (sa_layout.h)
    static constexpr int NW = CS / 32;                      // words per plane per lane per chunk
    static constexpr int LW = 2 * NW;                       // dwords per lane per chunk (2 planes)
    static constexpr int BPC = CS / SB;                     // bodies per chunk (1 or 2)
    static_assert(SB % 16 == 0 && (CS % SB) == 0, "bodies must tile chunks");
};

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
};

// Work unit of the fill kernel: a GROUP of W consecutive strips. A workgroup has W compute waves
// (one strip each) and one I/O wave. Compute waves only ever exchange rows through LDS rings:
// ring[w] feeds compute wave w; wave w writes its bottom row into ring[w+1]. The I/O wave links the
// group to its neighbours in global memory: it copies the previous group's granules into ring[0]
// and drains ring[W] into granules for the next group. Keeping every global store and poll out of
// the compute waves matters: on gfx9 a store shares the vmcnt counter with the text-code loads, and
// a cross-XCD (sc1) store takes ~0.7 us to retire, which would stall the next load wait.
typedef __attribute__((address_space(3))) int lds_int;  // ds_read/ds_write, never flat
// Ring and progress-word accesses are relaxed workgroup-scope atomics: the compiler keeps them in
// program order and re-reads them every time, without the s_waitcnt lgkmcnt(0) it puts after every
// volatile access.
// LDS executes one wave's ds operations in order, which is the only ordering the rings rely on.
__device__ __forceinline__ int lds_ld(lds_int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(lds_int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
constexpr int kRing = 2048;        // ring entries (columns), power of two
constexpr int kRingMask = kRing - 1;
#ifndef SA_CODE_AHEAD
#define SA_CODE_AHEAD 2  // R = 1 text-code loads run this many bodies ahead (1 or 2)
#endif
#ifndef SA_PF_FIRST
#define SA_PF_FIRST 1  // body boundary order: feed check, prefetch, publish, consumption word
#endif
#ifndef SA_ABL
#define SA_ABL 0  // timing ablations of the hand-off (development builds only; results are wrong)
#endif
#ifndef SA_CODE_AHEAD_LOCAL
#define SA_CODE_AHEAD_LOCAL 2
#endif
constexpr int kTimelineWords = 6;  // SA_TIMELINE record per strip
constexpr int kMaxWaves = 4;       // compute waves per workgroup (+1 I/O wave: 320 threads, <= 256 VGPRs)

struct GroupHdr {
    int S[32 * 32];                // generic score table (A <= 32)
    int prog[kMaxWaves + 1];       // prog[w]: columns published into ring[w]
    int cons[kMaxWaves + 1];       // cons[w]: columns read from ring[w] (producer backpressure)
    int group;                     // group index taken from the queue
    int pad[1];
};
__host__ __device__ constexpr size_t group_lds_bytes(int W) { return sizeof(GroupHdr) + (size_t)(W + 1) * kRing * 4; }

// Bounded-spin helper, called every few polls: false (and the abort word raised) after the
// timeout, or as soon as another wave has given up.
__device__ __forceinline__ bool keep_waiting(const FillArgs &a, uint64_t t0, int lane)
{
    // 100 MHz constant clock
    const bool late = __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks;
    if (late && lane == 0) __hip_atomic_store(&a.ctrl->abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int aborted = uniform((int)__hip_atomic_load(&a.ctrl->abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return !(aborted || late);
}

// Waits until the producer wave has published columns 1..need into the ring (LDS progress word),
// or until the fill is aborted (timeout): the strip then runs on with whatever the ring holds and
// the launch reports the abort, so the hot loop carries no error-path control flow.
__device__ __forceinline__ void wait_ring(const FillArgs &a, lds_int *prog, int need, int &avail, int lane)
{
    avail = uniform(lds_ld(prog));
    if (avail >= need) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t spin = 1;; ++spin)
    {
        __builtin_amdgcn_s_sleep(1);
        avail = uniform(lds_ld(prog));
        if (avail >= need) return;
        if ((spin & 255) == 0 && !keep_waiting(a, t0, lane)) return;
    }
}

// Ring slot of column c (1-based) in every LDS ring. The +14 puts the first column of a producer
// body's bottom-row values (c = s0 - 62, s0 a multiple of U) on a slot that is a multiple of U, so
// lane 63 publishes a body with U/4 ds_write_b128 that never straddle the ring's end.
__device__ __forceinline__ int ring_slot(int c) { return (c + 14) & kRingMask; }
static_assert(kRing % 16 == 0, "ring must hold whole bodies");

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
//   kPair   pair-packed lone strips (fill_pair_kernel): per column the two pairs' column profiles.
// The zero padding of the profiles keeps the ramp cells left of column 1 at the boundary value.
enum ScoreKind { kProf = 0, kTable = 1, kArr = 2, kArr8 = 3, kPair = 4 };
template <int SK>
constexpr bool kIsArr = SK == kArr || SK == kArr8;

// a + sign_extend(byte B of w), one VALU op
template <int B>
__device__ __forceinline__ int add_sbyte(int a, int w)
{
    int r;
    if constexpr (B == 0) asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(a), "v"(w));
    else if constexpr (B == 1) asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(a), "v"(w));
    else if constexpr (B == 2) asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(a), "v"(w));
    else asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(a), "v"(w));
    return r;
}

// Text-code dwords per body: one per step, or one per four steps (kArr8).
template <int R, int SK>
struct Codes {
    static constexpr int NT = SK == kArr8 ? Cfg<R>::U / 4 : Cfg<R>::U;
};

// One unrolled body of U steps. Body kinds (KIND):
//   kSteady  every lane is on a column >= 1. Lanes past column n compute garbage, which is harmless:
//            it only ever flows to lanes that are past n as well, their direction planes are never
//            read, their bottom-row values are never read and their local best-cell keys are
//            filtered by column; only the global score and the local best-cell keys need the exact
//            final state (kGeneric).
//   kStart   the first bodies (s < 63, kProf / kTable only): lane k is still left of column 1 while
//            s < k. Forcing the substitution score of those virtual cells to 0 keeps their state at
//            the boundary value (see the recurrences), so lane k enters column 1 with exactly the
//            column-0 state. Text profiles need no kStart bodies: their padding scores are 0.
//   kGeneric lanes outside [1, n] keep their state (the strip holding the global score's row, and
//            local strips' last bodies).
enum BodyKind { kSteady = 0, kStart = 1, kGeneric = 2 };
// Recurrences (per lane-row; diag/up/left are the neighbours' values):
//   global, shifted domain F = H + g(i+j): F = max(Fdiag + S + 2g, Fleft, Fup), boundaries 0;
//     DIAG iff Fdiag + S + 2g > max(Fleft, Fup); plane 1 = raw "up > left".
//   local, H with the gap folded into the score: X = max(Hdiag + S + g, max(Hleft, Hup)),
//     H = max(X - g, 0) (one saturating subtraction: X >= 0); DIAG iff Hdiag + S + g > max(Hleft,
//     Hup) (the reference's D > max(L, U) with every candidate shifted by +g); raw TOP iff Hup >
//     Hleft; STOP iff H == 0 (alignSequenceCPU.cpp:175-190).
// Lane moves per step: `up` (the row above each lane's first row) is F[R-1] of lane k-1 by a DPP
// wave_shr:1 whose `old` operand is this step's feed register Q (lane 0 keeps Q's lane 0 = the
// strip above's bottom value for this column); Q is dead afterwards, so the DPP writes in place. The
// next step's feed register is Q shifted down one lane (wave_shl:1, bound_ctrl), computed first.
// The strip's bottom row (F[R-1] of lane 63 after each step) is not moved at all: every step's F[R-1]
// stays in its own register Fs[q] until the body ends, when lane 63 publishes all U of them.
template <int R, bool LOCAL, int SK, int KIND>
__device__ __forceinline__ void run_body(const int *__restrict__ ldsS, int s0, int lane, int n, int g,
                                         int kb, const int (&prof)[R], const int (&T)[Codes<R, SK>::NT],
                                         int (&F)[R], int (&best)[R], int &upPrev, int Q,
                                         int (&Fs)[Cfg<R>::U], uint32_t (&acc)[3][Cfg<R>::NW])
{
    constexpr int U = Cfg<R>::U;
    sfor<U>([&](auto Qc) {
        constexpr int q = decltype(Qc)::value;
        const int s = s0 + q;
        const int Qn = __builtin_amdgcn_mov_dpp(Q, 0x130, 0xf, 0xf, true);  // wave_shl:1
        int up = dpp_shr1(Q, F[R - 1]);
        Q = Qn;
        int diag = upPrev;
        upPrev = up;
        constexpr bool RAMP = KIND == kGeneric;
        bool act = true;
        if constexpr (RAMP)
        {
            const int c = s - lane;
            act = (c >= 0) && (c < n);
        }
        const bool real = KIND != kStart || lane <= s;  // kStart: column s-lane+1 >= 1
        const int kmask = (1 << kb) - 1;
        const int Ks = kmask - (s & kmask);  // local: later column in a block = smaller key
        sfor<R>([&](auto Rc) {
            constexpr int rho = decltype(Rc)::value;
            constexpr int w = ((q * R + rho) / 32) % Cfg<R>::NW;
            int D;
            if constexpr (SK == kArr8) D = add_sbyte<q & 3>(diag, T[q >> 2]);
            else
            {
                int sc;
                if constexpr (SK == kArr) sc = T[q];
                else if constexpr (SK == kProf) sc = __builtin_amdgcn_sbfe(prof[rho], T[q], 8);
                else sc = ldsS[prof[rho] + T[q]];
                if constexpr (KIND == kStart) sc = real ? sc : 0;
                D = diag + sc;
            }
            const int left = F[rho];
            const int M = max(left, up);
            acc[0][w] = push_sign(acc[0][w], M - D);      // DIAG
            acc[1][w] = push_sign(acc[1][w], left - up);  // raw "up > left" (global) / raw TOP (local)
            int Fn;
            if constexpr (!LOCAL)
            {
                Fn = max(D, M);
            }
            else
            {
                const unsigned X = (unsigned)max(D, M);
                Fn = (int)__builtin_elementwise_sub_sat(X, (unsigned)g);
                acc[2][w] = push_sign(acc[2][w], Fn - 1);  // STOP (H == 0)
                const int key = (Fn << kb) + Ks;
                if constexpr (RAMP) best[rho] = act ? max(best[rho], key) : best[rho];
                else best[rho] = max(best[rho], key);
            }
            if constexpr (RAMP) Fn = act ? Fn : left;
            diag = left;
            up = Fn;
            F[rho] = Fn;
        });
        Fs[q] = F[R - 1];
    });
}

// Stores one finished chunk: lane k's LW dwords at chunk*64*LW + k*LW (one coalesced wave store).
template <int R, bool LOCAL>
__device__ __forceinline__ void store_chunk(uint32_t *dst, const uint32_t (&acc)[3][Cfg<R>::NW])
{
    constexpr int NW = Cfg<R>::NW;
    uint32_t v[2 * NW];
    sfor<NW>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        if constexpr (LOCAL)
        {
            const uint32_t d = acc[0][w], t = acc[1][w], z = acc[2][w];
            v[w] = d | z;
            v[NW + w] = (t & ~d) | z;
        }
        else
        {
            v[w] = acc[0][w];
            v[NW + w] = acc[1][w];
        }
    });
    if constexpr (NW == 1)
    {
        *reinterpret_cast<u32x2 *>(dst) = u32x2{v[0], v[1]};
    }
    else
    {
        sfor<NW / 2>([&](auto Xc) {
            constexpr int x = decltype(Xc)::value;
            *reinterpret_cast<u32x4 *>(dst + 4 * x) = u32x4{v[4 * x], v[4 * x + 1], v[4 * x + 2], v[4 * x + 3]};
        });
    }
}

// One strip. HP / HN: the strip has a strip above (feeds from rin) / below (publishes into rout);
// compile-time, so a body boundary carries no per-body decisions. Bodies run in pairs (the text
// codes double-buffer across the two bodies of a pair) in three phases: ramp pairs (kStart, only
// kProf / kTable), steady pairs, and tail pairs (kGeneric, only where the final state is read).
template <int R, bool LOCAL, int SK, bool HP, bool HN>
__device__ __forceinline__ void process_strip(const FillArgs &a, GroupHdr &H, lds_int *rings, int idx, int w, int lane)
{
    constexpr int U = Cfg<R>::U;
    constexpr int NT = Codes<R, SK>::NT;
    // Descriptors come in through vector loads (the kernel stores to global memory, so the compiler
    // cannot use scalar loads); making every field uniform keeps the sizes and every address derived
    // from them in SGPRs
    idx = uniform(idx);
    StripDesc sd = a.strips[idx];
    sd.pair = uniform(sd.pair);
    sd.row0 = uniform(sd.row0);
    sd.nsteps = uniform(sd.nsteps);
    sd.mask_off = uniform64(sd.mask_off);
    PairDesc pd = a.pairs[sd.pair];
    pd.text_len = uniform64(pd.text_len);
    pd.pattern_len = uniform64(pd.pattern_len);
    pd.pattern_off = uniform64(pd.pattern_off);
    pd.code_off = uniform64(pd.code_off);
    pd.code_len = uniform64(pd.code_len);
    const int n = (int)pd.text_len, m = (int)pd.pattern_len;
    const int g = a.gap;
    const int kb = a.key_bits;
    const int rowTop = sd.row0 + lane * R;
    int prof[R];
    sfor<R>([&](auto Rc) {
        constexpr int rho = decltype(Rc)::value;
        const int i = rowTop + rho;
        int c = i <= m ? (int)a.pattern[pd.pattern_off + i - 1] : 0;
        c = min(max(c, 0), a.A - 1);
        prof[rho] = SK == kProf ? a.prof_tab[c] : SK == kTable ? c * a.A : c;
    });
    // lane k at step s needs the score / code of column s-k+1: text index s - k. Addresses are a
    // uniform base (SGPRs) plus a 32-bit lane byte offset, so every load is one global_load with an
    // SGPR base and one 32-bit add, without 64-bit VALU address arithmetic.
    const char *cbase = reinterpret_cast<const char *>(a.codes + pd.code_off);
    uint32_t coff;
    if constexpr (SK == kArr8)
        // byte copy r = k % 4 of letter a: byte kPad + x holds S[a][t[x - r]]; read from x = s0 - (k & ~3)
        coff = (uint32_t)(((uint64_t)prof[0] * 4 + (lane & 3)) * pd.code_len + kPad - (lane & ~3));
    else if constexpr (SK == kArr)
        coff = (uint32_t)(((uint64_t)prof[0] * pd.code_len + kPad - lane) * 4);
    else
        coff = (uint32_t)((kPad - lane) * 4);
    lds_int *rin = (lds_int *)(rings + w * kRing);
    lds_int *rout = (lds_int *)(rings + (w + 1) * kRing);
    lds_int *progIn = (lds_int *)&H.prog[w];
    lds_int *consIn = (lds_int *)&H.cons[w];
    lds_int *progOut = (lds_int *)&H.prog[w + 1];
    lds_int *consOut = (lds_int *)&H.cons[w + 1];
    // the strip's direction chunks (uniform base) and this lane's byte offset in a chunk
    uint32_t *mbase = a.masks + sd.mask_off * 4;
    const uint32_t moff = (uint32_t)(lane * Cfg<R>::LW * 4);
    uint32_t acc[3][Cfg<R>::NW];
    sfor<Cfg<R>::NW>([&](auto Wc) {
        acc[0][decltype(Wc)::value] = 0;
        acc[1][decltype(Wc)::value] = 0;
        acc[2][decltype(Wc)::value] = 0;
    });
    const int nSteps = sd.nsteps;  // a multiple of 2U
    // Lanes must stop at column n (kGeneric bodies at the end) where the final state is read: the
    // global score H(m, n) in the strip holding row m, and the local best-cell keys (a garbage key
    // past column n could shadow a real one of the same key block). Other strips run their tail
    // unmasked.
    const bool needFinal = LOCAL || (m - sd.row0 >= 0 && m - sd.row0 < kWave * R);

    // column-0 boundary: global F(i,0) = 0; local H(i,0) = 0
    int F[R], best[R];
    sfor<R>([&](auto Rc) {
        constexpr int rho = decltype(Rc)::value;
        F[rho] = 0;
        best[rho] = 0;
    });
    int upPrev = 0, Q = 0;
    int Fs[U];
    // text codes, double-buffered across the two bodies of a pair (no register copies)
    // text codes: SA_CODE_AHEAD = 1 double-buffers across the two bodies of a pair; 2 keeps four
    // buffers and loads every body's codes two bodies ahead (bodies run in quads)
    constexpr int kAhead = R != 1 ? 1 : LOCAL ? SA_CODE_AHEAD_LOCAL : SA_CODE_AHEAD;  // taller strips: long bodies
    int TA[NT], TB[NT], TC[NT], TD[NT];
    auto load_codes = [&](int s0, int (&dst)[NT]) __attribute__((always_inline)) {
        typedef int i32x4u __attribute__((ext_vector_type(4), aligned(4)));
        const uint32_t off = coff + (uint32_t)(SK == kArr8 ? s0 : s0 * 4);
        sfor<NT / 4>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value * 4;
            const i32x4u v = *(const i32x4u *)(cbase + off + q * 4);
            dst[q] = v.x;
            dst[q + 1] = v.y;
            dst[q + 2] = v.z;
            dst[q + 3] = v.w;
        });
    };
    const uint64_t tStart = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
    load_codes(0, TA);
    if constexpr (kAhead == 2) load_codes(U, TB);
    int avail = 0;       // columns known to be in rin
    int consKnown = 0;   // columns the consumer of rout is known to have read
    // The progress word and the feed values for body k+2 are read speculatively at the end of body
    // k and used at the end of body k+1 without an LDS round trip (LDS is in order per wave: values
    // read after a progress word that covers them are valid). At a body boundary the order is feed
    // check -> next prefetch -> publish -> consumption word: the only LDS wait (the feed check, one
    // body after its reads) never waits for a boundary's writes. Feeds and publications are not
    // masked at the ends of the text: values of columns <= 0 or > n only ever reach cells outside
    // [1, n].
    int pfProg = 0, pfVal = 0;
    auto prefetch = [&](int base) __attribute__((always_inline)) {
        if constexpr (HP && SA_ABL != 1)
        {
            pfProg = lds_ld(progIn);
            pfVal = lds_ld(rin + ring_slot(base + 1 + lane));
        }
    };
    // lanes 0..U-1 of Q take the bottom values of columns base+1 .. base+U of the strip above
    auto feed = [&](int base) __attribute__((always_inline)) {
        if constexpr (SA_ABL != 0)
        {
            Q = pfVal;  // timing ablation (development only): never waits, results are garbage
            return;
        }
        if constexpr (!HP)
        {
            // row 0 boundary. The zero is opaque on purpose: with a known-zero `old` the compiler
            // folds the up-DPP into its consumers with bound_ctrl:1, and on gfx950 wave_shr with
            // bound_ctrl does not hand lane 0 a zero (measured: wrong row 1 in strip 0)
            asm volatile("v_mov_b32 %0, 0" : "=v"(Q));
            return;
        }
        const int need = min(n, base + U);
        if (__builtin_expect(uniform(pfProg) < need, 0))
        {
            wait_ring(a, progIn, need, avail, lane);
            pfVal = lds_ld(rin + ring_slot(base + 1 + lane));
        }
        Q = pfVal;  // lanes >= U: don't care
    };
    auto consumed = [&](int upto) __attribute__((always_inline)) {
        if constexpr (HP && SA_ABL != 1)
            if (lane == 0) lds_st(consIn, upto);
    };
    prefetch(0);
    feed(0);
    consumed(U);
    prefetch(U);
    const uint64_t tFed = a.timeline ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t cFed = a.timeline ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t lbest = 0;
    auto body = [&](auto kind, auto second, int s0, int (&T)[NT], int (&Tn)[NT]) __attribute__((always_inline)) {
        constexpr int KIND = decltype(kind)::value;
        const int s1 = s0 + U;
        load_codes(s0 + kAhead * U, Tn);
        run_body<R, LOCAL, SK, KIND>(H.S, s0, lane, n, g, kb, prof, T, F, best, upPrev, Q, Fs, acc);
        if constexpr (Cfg<R>::BPC == 1 || decltype(second)::value)
        {
            const int chunk = (s1 * R) / Cfg<R>::CS - 1;
            store_chunk<R, LOCAL>(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(mbase + (size_t)chunk * (kWave * Cfg<R>::LW)) + moff), acc);
        }
        if constexpr (LOCAL)
        {
            const int kmask = (1 << kb) - 1;
            if (((s1 & kmask) == 0) || s1 >= nSteps)
            {
                const int blockBase = s0 & ~kmask;
                sfor<R>([&](auto Rc) {
                    constexpr int rho = decltype(Rc)::value;
                    const int key = best[rho];
                    const int Hv = key >> kb;
                    const int st = blockBase + (kmask - (key & kmask));
                    const int c = st - lane + 1;
                    const int row = rowTop + rho;
                    if (Hv > 0 && row <= m && c >= 1 && c <= n)
                    {
                        const int rb = a.key_rowbits;
                        const uint64_t km = (1ull << rb) - 1;
                        const uint64_t k64 = ((uint64_t)Hv << (2 * rb)) | ((km - (uint64_t)row) << rb) |
                                             (km - (uint64_t)c);
                        lbest = max(lbest, k64);
                    }
                    best[rho] = 0;
                });
            }
        }
        // (after the last body this waits for the strip above's final progress word, n)
        // The prefetched words must not be read before the body's steps: left alone, the compiler
        // hoists the feed check (and its LDS wait) above the body, stalling right after the prefetch
        // and asking for the strip above's values a body early.
        if constexpr (HP) asm volatile("" : "+v"(pfProg), "+v"(pfVal) : "v"(Fs[U - 1]));
        feed(s1);
#if SA_PF_FIRST
        prefetch(s1 + U);  // reads before this boundary's writes: waiting for them never waits for the writes
#endif
        if constexpr (HN && SA_ABL != 1)
        {
            // lane 63's Fs[q] is the bottom-row value of column c0 + q (lane 63 is on column s-62);
            // ring slots of columns c0..c0+U-1 must have been read: c - kRing <= consumed
            const int c0 = s0 - (kWave - 2);
            const int top = min(n, max(0, s1 - 1 - (kWave - 2)));
            if (__builtin_expect(c0 + U - 1 - kRing > consKnown, 0))
            {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (uint32_t spin = 1;; ++spin)
                {
                    consKnown = uniform(lds_ld(consOut));
                    if (c0 + U - 1 - kRing <= consKnown) break;
                    __builtin_amdgcn_s_sleep(1);
                    if ((spin & 255) == 0 && !keep_waiting(a, t0, lane)) break;
                }
            }
            if (lane == kWave - 1)
            {
                typedef int i32x4 __attribute__((ext_vector_type(4)));
                typedef __attribute__((address_space(3))) i32x4 lds_i32x4;
                lds_i32x4 *dst = (lds_i32x4 *)(rout + ring_slot(c0));
                sfor<U / 4>([&](auto Xc) {
                    constexpr int x = decltype(Xc)::value;
                    dst[x] = i32x4{Fs[4 * x], Fs[4 * x + 1], Fs[4 * x + 2], Fs[4 * x + 3]};
                });
                // the values go before the progress word: a compiler-only fence (LDS executes one
                // wave's operations in order)
                asm volatile("" ::: "memory");
                lds_st(progOut, top);
            }
        }
        consumed(s1 + U);
#if !SA_PF_FIRST
        prefetch(s1 + U);
#endif
    };
    using KSteady = std::integral_constant<int, kSteady>;
    using KStart = std::integral_constant<int, kStart>;
    using KGeneric = std::integral_constant<int, kGeneric>;
    using First = std::false_type;
    using Second = std::true_type;
    // tail pairs: from the first pair holding a body with s1 > n (only where the final state is read)
    const int sTail = needFinal ? max(0, (n - 2 * U + 1 + 2 * U - 1) / (2 * U) * (2 * U)) : nSteps;
    int s0 = 0;
    if constexpr (kAhead == 2)
    {
        // bodies in quads up to `end` (a multiple of 2U), then at most one pair, after which the codes
        // loaded into TC / TD move back to TA / TB (once per phase)
        auto phase = [&](auto kind, int end) __attribute__((always_inline)) {
            for (; s0 + 2 * U < end; s0 += 4 * U)
            {
                body(kind, First{}, s0, TA, TC);
                body(kind, Second{}, s0 + U, TB, TD);
                body(kind, First{}, s0 + 2 * U, TC, TA);
                body(kind, Second{}, s0 + 3 * U, TD, TB);
            }
            if (s0 < end)
            {
                body(kind, First{}, s0, TA, TC);
                body(kind, Second{}, s0 + U, TB, TD);
                s0 += 2 * U;
                sfor<NT>([&](auto Qc) {
                    constexpr int q = decltype(Qc)::value;
                    TA[q] = TC[q];
                    TB[q] = TD[q];
                });
            }
        };
        if constexpr (!kIsArr<SK>) phase(KStart{}, min(kWave, sTail));
        phase(KSteady{}, sTail);
        phase(KGeneric{}, nSteps);
    }
    else
    {
        if constexpr (!kIsArr<SK>)
            for (; s0 < min(kWave, sTail); s0 += 2 * U)
            {
                body(KStart{}, First{}, s0, TA, TB);
                body(KStart{}, Second{}, s0 + U, TB, TA);
            }
        for (; s0 < sTail; s0 += 2 * U)
        {
            body(KSteady{}, First{}, s0, TA, TB);
            body(KSteady{}, Second{}, s0 + U, TB, TA);
        }
        for (; s0 < nSteps; s0 += 2 * U)
        {
            body(KGeneric{}, First{}, s0, TA, TB);
            body(KGeneric{}, Second{}, s0 + U, TB, TA);
        }
    }
    if (HN && lane == kWave - 1) lds_st(progOut, n);  // never leave the consumer waiting (abort)
    if (a.timeline && lane == 0)
    {
        uint64_t *tl = a.timeline + kTimelineWords * (size_t)idx;
        tl[0] = tStart;
        tl[1] = tFed;
        tl[2] = __builtin_amdgcn_s_memrealtime();
        tl[4] = cFed;  // shader clock (s_memtime): effective frequency = clocks / real time
        tl[5] = __builtin_amdgcn_s_memtime();
        // XCC_ID (hwreg 20) and HW_ID (hwreg 4: wave, SIMD, CU, SE fields)
        tl[3] = ((uint64_t)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32) |
                (uint32_t)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    }
    if constexpr (LOCAL)
    {
        const uint64_t wbest = wave_max_u64(lbest);
        if (lane == 0) a.strip_best[idx] = wbest;  // (after an abort the launch reports the error)
    }
    else
    {
        const int rm = m - sd.row0;  // strip-relative row of the last DP row
        if (rm >= 0 && rm < kWave * R && lane == rm / R)
        {
            int v = F[0];
            sfor<R>([&](auto Rc) {
                constexpr int rho = decltype(Rc)::value;
                if (rho == rm % R) v = F[rho];
            });
            a.pair_score[sd.pair] = v - g * (m + n);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// pair-packed fill (global mode, lone strips, DNA-sized alphabets): two independent pairs of the same
// shape in the two 16-bit halves of every register
// ------------------------------------------------------------------------------------------------
// The shifted-domain global recurrence only needs unsigned add / max and sign bits of differences,
// so when every value fits u16 (0 <= S + 2g <= 255, (max S + 2g) * min(m, n) <= 65535: F is
// non-negative and bounded by that) and every difference compared fits i16 (|M - D|, |left - up| <=
// 2 (max S + 2g)), one v_pk_* instruction advances both pairs.
//   * Scores: per text column the code block holds two "column profiles" {colA, colB}, byte r of
//     colA = S[r][tA] + 2g (zero in the padding); each row keeps one fixed selector
//     rA | 0x0c00 | (4 + rB) << 16 | 0x0c000000, and one v_perm_b32(colB, colA, sel) gives the row's
//     two scores as u16 halves.
//   * Direction bits: slot σ of a 16-slot group sits at bit 15 - σ of each half. Slots s and s+8
//     (s < 8) are rows ρ and ρ+8 of the same step (R >= 16); one v_perm_b32 gathers the four sign
//     bits (both pairs, both slots) onto byte MSBs (bits 15, 7, 31, 23), one shift by s moves them to
//     15-s, 7-s, 31-s, 23-s, and one v_and_or_b32 inserts them: 3 VALU per 4 bits.
//   * At the body's end v_perm_b32 splits the packed words back into each pair's ordinary 32-slot
//     words, so the stored planes, the traceback and the decoders are exactly those of the unpacked
//     kernel.
// About 4.5 VALU per cell instead of 8.2.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as16(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

template <int R>
__device__ __forceinline__ void process_pair(const FillArgs &a, int sA, int lane)
{
    constexpr int U = Cfg<R>::U;
    constexpr int SB = Cfg<R>::SB;      // slots per body (per pair)
    constexpr int NP = SB / 16;         // packed words per plane per body
    constexpr int NW = Cfg<R>::NW, LW = Cfg<R>::LW;
    static_assert(R >= 16 && Cfg<R>::BPC == 1 && SB % 32 == 0, "pair kernel: R >= 16, a body is one chunk");
    const StripDesc dA = a.strips[sA], dB = a.strips[sA + 1];
    const PairDesc pA = a.pairs[dA.pair], pB = a.pairs[dB.pair];
    const int n = (int)pA.text_len, m = (int)pA.pattern_len;
    const int g = a.gap;
    const int rowTop = 1 + lane * R;
    uint32_t rsel[R];
    sfor<R>([&](auto Rc) {
        constexpr int rho = decltype(Rc)::value;
        const int i = rowTop + rho;
        const int cA = i <= m ? min(max((int)a.pattern[pA.pattern_off + i - 1], 0), a.A - 1) : 0;
        const int cB = i <= m ? min(max((int)a.pattern[pB.pattern_off + i - 1], 0), a.A - 1) : 0;
        rsel[rho] = (uint32_t)cA | 0x0c00u | ((uint32_t)(4 + cB) << 16) | 0x0c000000u;
    });
    // column profiles {colA, colB} per column, in pair A's code block (2 dwords per column)
    const int32_t *codes = a.codes + pA.code_off + 2 * (kPad - lane);
    uint32_t *mkA = a.masks + dA.mask_off * 4 + lane * LW;
    uint32_t *mkB = a.masks + dB.mask_off * 4 + lane * LW;
    const int nSteps = dA.nsteps;
    uint32_t F[R];
    sfor<R>([&](auto Rc) { F[decltype(Rc)::value] = 0; });
    uint32_t upPrev = 0;
    int Q;
    int TA[2 * U], TB[2 * U];
    auto load_codes = [&](int s0, int (&dst)[2 * U]) __attribute__((always_inline)) {
        typedef int i32x4u __attribute__((ext_vector_type(4), aligned(8)));
        sfor<U / 2>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value * 4;
            const i32x4u v = *(const i32x4u *)(codes + 2 * s0 + q);
            dst[q] = v.x;
            dst[q + 1] = v.y;
            dst[q + 2] = v.z;
            dst[q + 3] = v.w;
        });
    };
    load_codes(0, TA);
    auto body = [&](auto kind, int s0, int (&T)[2 * U], int (&Tn)[2 * U]) __attribute__((always_inline)) {
        constexpr bool RAMP = decltype(kind)::value;  // tail: lanes outside [1, n] keep their state
        const int s1 = s0 + U;
        load_codes(s1, Tn);
        uint32_t acc[2][NP];
        asm volatile("v_mov_b32 %0, 0" : "=v"(Q));  // row 0 boundary (opaque zero: see feed())
        sfor<U>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value;
            const int Qn = __builtin_amdgcn_mov_dpp(Q, 0x130, 0xf, 0xf, true);  // wave_shl:1
            uint32_t up = (uint32_t)dpp_shr1(Q, (int)F[R - 1]);
            Q = Qn;
            uint32_t diag = upPrev;
            upPrev = up;
            bool act = true;
            if constexpr (RAMP)
            {
                const int c = s0 + q - lane;
                act = (c >= 0) && (c < n);
            }
            const uint32_t colA = (uint32_t)T[2 * q], colB = (uint32_t)T[2 * q + 1];
            uint32_t x0[R], x1[R];
            sfor<R>([&](auto Rc) {
                constexpr int rho = decltype(Rc)::value;
                const uint32_t sc = __builtin_amdgcn_perm(colB, colA, rsel[rho]);
                const u16x2 D = as16(diag) + as16(sc);
                const uint32_t left = F[rho];
                const u16x2 M = __builtin_elementwise_max(as16(left), as16(up));
                uint32_t Fn = as32(__builtin_elementwise_max(D, M));
                x0[rho] = as32(M - D);                     // DIAG iff sign
                x1[rho] = as32(as16(left) - as16(up));     // up > left iff sign
                if constexpr (RAMP) Fn = act ? Fn : left;
                diag = left;
                up = Fn;
                F[rho] = Fn;
                // rows rho-8 and rho of a 16-row group are slots s and s+8 of packed word w: insert
                // as soon as both exist (keeps at most 8 rows of differences live)
                if constexpr (rho % 16 >= 8)
                {
                    constexpr int sl = rho % 16 - 8;
                    constexpr int w = (q * R + rho) / 16;
                    constexpr uint32_t mask = (0x80808080u >> sl);
                    const uint32_t y0 = __builtin_amdgcn_perm(x0[rho - 8], x0[rho], 0x07030501u) >> sl;
                    const uint32_t y1 = __builtin_amdgcn_perm(x1[rho - 8], x1[rho], 0x07030501u) >> sl;
                    if constexpr (sl == 0)
                    {
                        acc[0][w] = y0 & mask;
                        acc[1][w] = y1 & mask;
                    }
                    else
                    {
                        acc[0][w] |= y0 & mask;
                        acc[1][w] |= y1 & mask;
                    }
                }
            });
        });
        // split the packed words into each pair's 32-slot words: {plane 0 words, plane 1 words}
        const int chunk = (s1 * R) / Cfg<R>::CS - 1;
        uint32_t vA[LW], vB[LW];
        sfor<NW>([&](auto Wc) {
            constexpr int w = decltype(Wc)::value;
            sfor<2>([&](auto Pc) {
                constexpr int p = decltype(Pc)::value;
                vA[p * NW + w] = __builtin_amdgcn_perm(acc[p][2 * w], acc[p][2 * w + 1], 0x05040100u);
                vB[p * NW + w] = __builtin_amdgcn_perm(acc[p][2 * w], acc[p][2 * w + 1], 0x07060302u);
            });
        });
        uint32_t *dA_ = mkA + (size_t)chunk * (kWave * LW);
        uint32_t *dB_ = mkB + (size_t)chunk * (kWave * LW);
        sfor<LW / 4>([&](auto Xc) {
            constexpr int x = decltype(Xc)::value;
            *reinterpret_cast<u32x4 *>(dA_ + 4 * x) = u32x4{vA[4 * x], vA[4 * x + 1], vA[4 * x + 2], vA[4 * x + 3]};
            *reinterpret_cast<u32x4 *>(dB_ + 4 * x) = u32x4{vB[4 * x], vB[4 * x + 1], vB[4 * x + 2], vB[4 * x + 3]};
        });
    };
    // tail pairs of bodies from the first pair holding a body with s1 > n (the global score row is
    // in every lone strip)
    const int sTail = max(0, n / (2 * U) * (2 * U));
    int s0 = 0;
    for (; s0 < sTail; s0 += 2 * U)
    {
        body(std::false_type{}, s0, TA, TB);
        body(std::false_type{}, s0 + U, TB, TA);
    }
    for (; s0 < nSteps; s0 += 2 * U)
    {
        body(std::true_type{}, s0, TA, TB);
        body(std::true_type{}, s0 + U, TB, TA);
    }
    const int rm = m - 1;  // strip-relative row of the last DP row
    if (lane == rm / R)
    {
        uint32_t v = F[0];
        sfor<R>([&](auto Rc) {
            constexpr int rho = decltype(Rc)::value;
            if (rho == rm % R) v = F[rho];
        });
        a.pair_score[dA.pair] = (int)(v & 0xffffu) - g * (m + n);
        a.pair_score[dB.pair] = (int)(v >> 16) - g * (m + n);
    }
}

// One wave per two strips (pairs sA, sA+1); 4 waves per workgroup; dynamic queue over strip pairs.
template <int R>
__global__ __launch_bounds__(kWave * kMaxWaves, 2) void fill_pair_kernel(FillArgs a)
{
    __shared__ int unit;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = uniform((int)(threadIdx.x / kWave));
    const int W = (int)(blockDim.x / kWave);
    const int units = a.num_strips / 2;
    while (true)
    {
        __syncthreads();
        if (threadIdx.x == 0) unit = (int)atomicAdd(&a.ctrl->queue_head, 1u);
        __syncthreads();
        const int grp = uniform(unit);
        if (grp * W >= units) break;
        const int u = grp * W + w;
        if (u < units) process_pair<R>(a, 2 * u, lane);
    }
}

// The I/O wave of a group: global granules of the previous group's last strip -> ring[0], and
// ring[W'] (W' = compute waves with a strip) -> granules for the next group. Only lane 0 polls the
// granules while nothing is there (8 bytes per poll: up to a few hundred waiting groups must not
// load the fabric the running strips use); the bytes move 64 columns per instruction.
__device__ void io_wave(const FillArgs &a, GroupHdr &H, lds_int *rings, int grp, int W, int lane)
{
    const int first = grp * W;
    const int last = min(first + W, a.num_strips) - 1;
    const StripDesc sf = a.strips[first];
    const StripDesc sl = a.strips[last];
    const int nIn = (sf.flags & kHasPrev) ? (int)a.pairs[sf.pair].text_len : 0;
    const int nOut = (sl.flags & kHasNext) ? (int)a.pairs[sl.pair].text_len : 0;
    if (nIn == 0 && nOut == 0) return;
    const int wl = last - first + 1;  // ring fed by the last strip
    lds_int *r0 = (lds_int *)rings;
    lds_int *prog0 = (lds_int *)&H.prog[0];
    lds_int *cons0 = (lds_int *)&H.cons[0];
    lds_int *rl = (lds_int *)(rings + wl * kRing);
    lds_int *progL = (lds_int *)&H.prog[wl];
    lds_int *consL = (lds_int *)&H.cons[wl];
    const uint64_t *bin = a.bnd + sf.bnd_in;
    uint64_t *bout = a.bnd + sl.bnd_out;
    int copied = 0, drained = 0;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t spin = 1; copied < nIn || drained < nOut; ++spin)
    {
        bool moved = false;
        if (copied < nIn)
        {
            const int room = uniform(lds_ld(cons0)) + kRing - copied;  // free ring slots
            const int want = min(min(kWave, nIn - copied), room);
            if (want >= min(16, nIn - copied))
            {
                uint64_t probe = 0;
                if (lane == 0) probe = load_granule(bin + copied + min(want, 16) - 1);
                if ((uint32_t)uniform((int)(uint32_t)(probe >> 32)) == a.epoch)
                {
                    const uint64_t v = lane < want ? load_granule(bin + copied + lane) : 0;
                    const uint64_t rdy = ballot(lane < want && (uint32_t)(v >> 32) == a.epoch);
                    const int cnt = ~rdy == 0 ? kWave : (int)__builtin_ctzll(~rdy);  // ready prefix
                    if (lane < cnt) lds_st(r0 + ring_slot(copied + lane + 1), (int)(uint32_t)v);
                    copied += cnt;
                    if (lane == 0) lds_st(prog0, copied);
                    moved = cnt > 0;
                }
            }
        }
        if (drained < nOut)
        {
            const int avail = uniform(lds_ld(progL));
            const int upto = min(avail, drained + kWave);
            if (upto - drained >= 16 || (avail >= nOut && upto > drained))
            {
                const int c = drained + lane;
                if (c < upto) store_granule(bout + c, ((uint64_t)a.epoch << 32) | (uint32_t)lds_ld(rl + ring_slot(c + 1)));
                drained = upto;
                if (lane == 0) lds_st(consL, drained);
                moved = true;
            }
        }
        if (moved)
        {
            t0 = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        for (int z = 0; z < a.io_sleep; ++z) __builtin_amdgcn_s_sleep(1);
        if ((spin & 127) == 0 && !keep_waiting(a, t0, lane))
        {
            // release both sides so the group drains (the launch reports the abort)
            if (lane == 0)
            {
                lds_st(prog0, nIn);
                lds_st(consL, nOut + kRing);
            }
            return;
        }
    }
}

// One workgroup = W compute waves + 1 I/O wave; it takes groups of W consecutive strips from the
// dynamic queue until the queue is empty. The queue order is the strip order, so a strip's
// predecessor has always been handed out before it: progress is guaranteed whatever the residency.
template <int R, bool LOCAL, int SK, bool CHAIN>
__global__ __launch_bounds__(kWave * (kMaxWaves + 1)) void fill_kernel(FillArgs a)
{
    extern __shared__ int lds_dyn[];
    GroupHdr &H = *reinterpret_cast<GroupHdr *>(lds_dyn);
    lds_int *rings = (lds_int *)(lds_dyn + sizeof(GroupHdr) / 4);
    const int lane = threadIdx.x & (kWave - 1);
    const int w = uniform((int)(threadIdx.x / kWave));
    // compute waves; with CHAIN wave W is the I/O wave (plans without strip chains have none, and no
    // rings in LDS either: more workgroups fit a CU)
    const int W = (int)(blockDim.x / kWave) - (CHAIN ? 1 : 0);
    if constexpr (SK == kTable)
        for (int e = threadIdx.x; e < a.A * a.A; e += blockDim.x) H.S[e] = a.score_tab[e];
    while (true)
    {
        __syncthreads();  // every wave is done with the previous group's rings
        if (threadIdx.x == 0)
        {
            const bool aborted = __hip_atomic_load(&a.ctrl->abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
            H.group = aborted ? a.num_groups : (int)atomicAdd(&a.ctrl->queue_head, 1u);
        }
        if (threadIdx.x <= kMaxWaves)
        {
            H.prog[threadIdx.x] = 0;
            H.cons[threadIdx.x] = 0;
        }
        __syncthreads();
        const int grp = uniform(H.group);
        if (grp >= a.num_groups) break;
        if (CHAIN && w == W)
        {
            io_wave(a, H, rings, grp, W, lane);
        }
        else
        {
            const int idx = grp * W + w;
            if (idx < a.num_strips)
            {
                // the strip kind is compile-time inside process_strip (branch-free body boundaries)
                // (CHAIN: some pair has several strips; otherwise every strip is alone and only one
                // variant is instantiated, which keeps the register count of the batch kernel down)
                const int f = uniform(a.strips[idx].flags) & (kHasPrev | kHasNext);
                if constexpr (CHAIN)
                {
                    if (f == (kHasPrev | kHasNext)) process_strip<R, LOCAL, SK, true, true>(a, H, rings, idx, w, lane);
                    else if (f == kHasPrev) process_strip<R, LOCAL, SK, true, false>(a, H, rings, idx, w, lane);
                    else if (f == kHasNext) process_strip<R, LOCAL, SK, false, true>(a, H, rings, idx, w, lane);
                    else process_strip<R, LOCAL, SK, false, false>(a, H, rings, idx, w, lane);
                }
                else
                {
                    (void)f;
                    process_strip<R, LOCAL, SK, false, false>(a, H, rings, idx, w, lane);
                }
            }
        }
    }
}

// Fill launches, one translation unit per strip height R (fill_r<R>.hip instantiates
// launch_fill_r<R>; the main unit only declares them), so the 48 fill kernels compile in parallel.
template <int R, bool LOCAL, int SK>
void launch_fill_t(const FillArgs &a, int grid, int W, bool chain, hipStream_t st)
{
    if (chain)
    {
        const size_t lds = std::max(group_lds_bytes(W), (size_t)a.chain_lds);
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&fill_kernel<R, LOCAL, SK, true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((fill_kernel<R, LOCAL, SK, true>), dim3(grid), dim3(kWave * (W + 1)), lds, st, a);
    }
    else hipLaunchKernelGGL((fill_kernel<R, LOCAL, SK, false>), dim3(grid), dim3(kWave * W), sizeof(GroupHdr), st, a);
}

// R = 1 uses text profiles (kArr8 when the scores fit int8, kArr otherwise); taller strips use the
// packed profile when the scores fit (kProf) and the LDS table otherwise (kTable).
template <int R>
void launch_fill_r(const FillArgs &a, bool local, int sk, int grid, int W, bool chain, hipStream_t st)
{
    if constexpr (R == 1)
    {
        if (sk == kArr8)
        {
            if (local) launch_fill_t<1, true, kArr8>(a, grid, W, chain, st);
            else launch_fill_t<1, false, kArr8>(a, grid, W, chain, st);
        }
        else
        {
            if (local) launch_fill_t<1, true, kArr>(a, grid, W, chain, st);
            else launch_fill_t<1, false, kArr>(a, grid, W, chain, st);
        }
    }
    else if (sk == kPair)
    {
        if constexpr (R >= 16)
            hipLaunchKernelGGL(fill_pair_kernel<R>, dim3(grid), dim3(kWave * W), 0, st, a);
    }
    else if (local)
    {
        if (sk == kProf) launch_fill_t<R, true, kProf>(a, grid, W, chain, st);
        else launch_fill_t<R, true, kTable>(a, grid, W, chain, st);
    }
    else
    {
        if (sk == kProf) launch_fill_t<R, false, kProf>(a, grid, W, chain, st);
        else launch_fill_t<R, false, kTable>(a, grid, W, chain, st);
    }
}

#ifdef SA_FILL_R
template void launch_fill_r<SA_FILL_R>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
}  // namespace sa
#else
extern template void launch_fill_r<1>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<2>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<4>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<8>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<16>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
extern template void launch_fill_r<32>(const FillArgs &, bool, int, int, int, bool, hipStream_t);

// Text codes for the fill (layout per score kind, see ScoreKind):
//   kProf / kTable  one dword per letter, 8*c (packed-profile bit offset) or c (LDS table index);
//   kArr            A dword arrays of code_len: array a holds table[a][t[x]] at kPad + x;
//   kArr8           4A byte arrays of code_len bytes: copy (a, r) holds table[a][t[x]] at kPad + x + r.
__global__ void encode_text_kernel(const int8_t *text, const PairDesc *pairs, int32_t *codes, int A, int SK,
                                   const int32_t *table)
{
    const PairDesc pd = pairs[blockIdx.y];
    if (SK == kPair)
    {
        // selectors of pairs (2q, 2q+1) in pair 2q's block, padding included (0x0c0c0c0c = zeros)
        if ((blockIdx.y & 1) != 0) return;
        const PairDesc pb = pairs[blockIdx.y + 1];
        for (uint64_t xx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; xx < pd.code_len;
             xx += (uint64_t)gridDim.x * blockDim.x)
        {
            const int64_t x = (int64_t)xx - kPad;
            uint32_t colA = 0, colB = 0;  // padding: zero scores
            if (x >= 0 && x < (int64_t)pd.text_len)
            {
                const int tA = min(max((int)text[pd.text_off + x], 0), A - 1);
                const int tB = min(max((int)text[pb.text_off + x], 0), A - 1);
                for (int r = 0; r < A; ++r)
                {
                    colA |= ((uint32_t)table[r * A + tA] & 0xffu) << (8 * r);
                    colB |= ((uint32_t)table[r * A + tB] & 0xffu) << (8 * r);
                }
            }
            codes[pd.code_off + 2 * xx] = (int32_t)colA;
            codes[pd.code_off + 2 * xx + 1] = (int32_t)colB;
        }
        return;
    }
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < pd.text_len;
         x += (uint64_t)gridDim.x * blockDim.x)
    {
        int c = text[pd.text_off + x];
        c = min(max(c, 0), A - 1);
        if (SK == kArr8)
        {
            int8_t *b8 = reinterpret_cast<int8_t *>(codes + pd.code_off);
            for (int r = 0; r < A; ++r)
                for (int sh = 0; sh < 4; ++sh) b8[((uint64_t)r * 4 + sh) * pd.code_len + kPad + x + sh] = (int8_t)table[r * A + c];
        }
        else if (SK == kArr)
            for (int r = 0; r < A; ++r) codes[pd.code_off + (uint64_t)r * pd.code_len + kPad + x] = table[r * A + c];
        else
            codes[pd.code_off + kPad + x] = SK == kProf ? 8 * c : c;
    }
}

// ------------------------------------------------------------------------------------------------
// traceback kernel
// ------------------------------------------------------------------------------------------------
constexpr int kWinEntries = 512;   // entries (16 bytes each) per LDS window buffer: 2 x 8 KiB
constexpr int kWinPerLane = kWinEntries / 64;
#ifndef SA_TB_NEARTOP
#define SA_TB_NEARTOP 8
#endif
constexpr int kNearTop = SA_TB_NEARTOP;  // rows below a strip's top at which the next strip is prefetched

struct TbArgs {
    const int8_t *text, *pattern;
    const StripDesc *strips;
    const PairDesc *pairs;
    const uint4 *masks;
    const uint64_t *strip_best;
    const int32_t *pair_score;
    uint8_t *ops;
    char *out_text, *out_pattern;
    sa_result *results;
    uint64_t *timing;           // debug (SA_TB_TIMING): per pair {start, walk done, pass 1, pass 2}
    int32_t mode, gap, A, key_rowbits;
    char alphabet[33];
};

template <int R, int MODE>
__global__ __launch_bounds__(64) void traceback_kernel(TbArgs a)
{
    __shared__ uint4 win[2][kWinEntries];
    __shared__ char alpha[40];
    constexpr int RB = kWave * R;
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const PairDesc pd = a.pairs[p];
    const int n = (int)pd.text_len, m = (int)pd.pattern_len;
    if (lane < 33) alpha[lane] = a.alphabet[lane];
    const uint64_t tT0 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;

    int score, i, j;
    if constexpr (MODE == SA_GLOBAL)
    {
        score = pd.num_strips > 0 ? a.pair_score[p] : -a.gap * (n + m);
        i = m;
        j = n;
    }
    else
    {
        uint64_t k = 0;
        for (int s = lane; s < pd.num_strips; s += kWave) k = max(k, a.strip_best[pd.first_strip + s]);
        k = wave_max_u64(k);
        const int rb = a.key_rowbits;
        const uint64_t km = (1ull << rb) - 1;
        const int H = (int)(k >> (2 * rb));
        if (H > 0)
        {
            score = H;
            i = (int)(km - ((k >> rb) & km));
            j = (int)(km - (k & km));
        }
        else
        {
            score = 0;  // no positive cell: maxIJ stays 0 (alignSequenceCPU.cpp:152)
            i = 0;
            j = 0;
        }
    }

    // ---- the walk: a uniform state machine (scalar registers) --------------------------------
    // Row i lives in strip b at in-strip row il = (i-1) - b*RB, i.e. lane k = il/R, slot il%R; the
    // entry of cell (i, j) is e = (j-1+k)*R + il%R of strip b. A move changes e by a constant:
    //   TOP  -1 (also across a lane boundary),  LEFT -R,  DIAG -R-1,
    // and il by -1 for TOP/DIAG; only leaving the strip (il < 0) re-derives e. Within a strip e only
    // decreases, so the walk reads a strip's entries top-down through windows of kWinEntries entries
    // held in LDS (one of two buffers). The next window is loaded ahead into registers (16 x 16 bytes
    // per lane, in flight while the walk goes on): the one below in the same strip, or, once the walk
    // is within kNearTop rows of the strip's top, the top window of the strip above. Each step reads
    // just the two dwords that hold bit k of the two planes.
    constexpr int LOG2R = R == 1 ? 0 : R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5;
    constexpr int CS = Cfg<R>::CS, NW = Cfg<R>::NW, LW = Cfg<R>::LW;
    constexpr int LOG2CS = CS == 32 ? 5 : CS == 64 ? 6 : 7;
    static_assert((1 << LOG2CS) == CS && kWinEntries % CS == 0, "windows hold whole chunks");
    // all strips of a pair have the same step count and consecutive entry ranges, so no strip
    // descriptor is loaded inside the walk (such a load would drain the prefetch in flight: gfx9
    // retires vector loads in order)
    uint64_t maskOff0 = 0;
    int stripEntries = 0;
    if (pd.num_strips > 0)
    {
        const StripDesc s0d = a.strips[pd.first_strip];
        maskOff0 = s0d.mask_off;
        stripEntries = s0d.nsteps * R;
    }
    int b = 0, il = 0, e = 0;
    auto enter = [&](int ii, int jj) __attribute__((always_inline)) {  // (i, j) -> b, il, e
        b = (ii - 1) / RB;
        il = (ii - 1) - b * RB;
        e = (jj - 1 + (il >> LOG2R)) * R + (il & (R - 1));
    };
    u32x4 stage[kWinPerLane];  // native vectors: promoted to registers (HIP's uint4 struct is not)
    int cur = 0, curStrip = -1, curLo = 0;
    int pfStrip = -1, pfLo = 0;  // window held in `stage` (pfStrip -1: none)
    auto stage_load = [&](int strip, int lo) __attribute__((always_inline)) {
        const int last = stripEntries - 1;
        const u32x4 *src = reinterpret_cast<const u32x4 *>(a.masks + maskOff0 + (uint64_t)strip * stripEntries);
        sfor<kWinPerLane>([&](auto Tc) {
            constexpr int t = decltype(Tc)::value;
            stage[t] = src[min(lo + t * kWave + lane, last)];
        });
        pfStrip = strip;
        pfLo = lo;
    };
    auto stage_commit = [&]() __attribute__((always_inline)) {  // staged window -> the other buffer
        const int nb = cur ^ 1;
        sfor<kWinPerLane>([&](auto Tc) {
            constexpr int t = decltype(Tc)::value;
            *reinterpret_cast<u32x4 *>(&win[nb][t * kWave + lane]) = stage[t];
        });
        cur = nb;
        curStrip = pfStrip;
        curLo = pfLo;
        pfStrip = -1;
    };
    // make entry e of strip b readable; prefetch what comes next
    auto ensure = [&](int jj) __attribute__((always_inline)) {
        if (b != curStrip || e < curLo)
        {
            if (!(b == pfStrip && e >= pfLo && e < pfLo + kWinEntries)) stage_load(b, e & ~(kWinEntries - 1));
            stage_commit();
#ifndef SA_TB_NO_BELOW
            if (curLo > 0) stage_load(b, curLo - kWinEntries);
#endif
        }
        if (il < kNearTop && b > 0 && pfStrip != b - 1)
            stage_load(b - 1, ((jj - 1 + kWave - 1) * R + R - 1) & ~(kWinEntries - 1));
    };
    const uint32_t *winw = reinterpret_cast<const uint32_t *>(&win[0][0]);
    auto code_at = [&](int jj) __attribute__((always_inline)) -> int {
        ensure(jj);
        // slot rel of the window: chunk rel/CS, lane k's words, bit 31 - rel%32 (sa_layout.h)
        const int k = il >> LOG2R;
        const int rel = e - curLo;
        const int dw = cur * (kWinEntries * 4) + (rel >> LOG2CS) * (kWave * LW) + k * LW + ((rel & (CS - 1)) >> 5);
        const uint32_t w0 = (uint32_t)uniform((int)winw[dw]);
        const uint32_t w1 = (uint32_t)uniform((int)winw[dw + NW]);
        const int sh = 31 - (rel & 31);
        const int b0 = (int)((w0 >> sh) & 1u), b1 = (int)((w1 >> sh) & 1u);
        // global: plane1 is the raw "up > left" bit, DIAG wins; local: {DIAG|STOP, TOP&~DIAG|STOP}
        return MODE == SA_GLOBAL ? (b0 ? kDiag : (b1 ? kTop : kLeft)) : (b0 | (b1 << 1));
    };
    auto move = [&](int tt, int tp, int ni, int nj) __attribute__((always_inline)) {  // after i -= tp, j -= tt
        e -= (tt << LOG2R) + tp;
        il -= tp;
        if (il < 0 && ni > 0) enter(ni, nj);
    };

    // ops are collected 64 at a time in one VGPR (v_writelane at lane len%64), then stored by all
    // lanes as 64 consecutive bytes
    uint8_t *ops = a.ops + pd.out_off;
    int opsAcc = 0;
    int len = 0;
    auto emit = [&](int d) __attribute__((always_inline)) {
        opsAcc = amdgcn_writelane(d, len & (kWave - 1), opsAcc);
        ++len;
        if ((len & (kWave - 1)) == 0) ops[len - kWave + lane] = (uint8_t)opsAcc;
    };
    // text / pattern index of the first letter the walk emits (the start cell's)
    const int ti0 = MODE == SA_GLOBAL ? n - 1 : j - 1;
    const int pi0 = MODE == SA_GLOBAL ? m - 1 : i - 1;
    int ti, pi;
    if (i > 0 && j > 0) enter(i, j);
    if constexpr (MODE == SA_GLOBAL)
    {
        // traceBackNW (alignSequenceCPU.cpp:64-114): row 0 forces LEFT, column 0 forces TOP
        ti = n - 1;
        pi = m - 1;
        while (i > 0 && j > 0)
        {
            const int d = code_at(j);
            const int tt = d != kTop;   // DIAG or LEFT
            const int tp = d != kLeft;  // DIAG or TOP
            emit(d);
            ti = max(0, ti - tt);
            pi = max(0, pi - tp);
            i -= tp;
            j -= tt;
            move(tt, tp, i, j);
        }
        // the boundary: only TOP moves down column 0, only LEFT moves along row 0
        while (i > 0 || j > 0)
        {
            const int tp = j == 0;
            emit(tp ? kTop : kLeft);
            ti = max(0, ti - (1 - tp));
            pi = max(0, pi - tp);
            i -= tp;
            j -= 1 - tp;
        }
    }
    else
    {
        // traceBackSW (alignSequenceCPU.cpp:10-62): stop at STOP; a move into row 0 / column 0
        // ends the walk before the index update.
        ti = j - 1;
        pi = i - 1;
        while (i > 0 && j > 0)
        {
            const int d = code_at(j);
            if (d == kStop) break;
            const int tt = d != kTop;
            const int tp = d != kLeft;
            emit(d);
            i -= tp;
            j -= tt;
            if (i == 0 || j == 0) break;
            ti -= tt;
            pi -= tp;
            move(tt, tp, i, j);
        }
    }
    {
        const int rem = len & (kWave - 1);
        if (lane < rem) ops[len - rem + lane] = (uint8_t)opsAcc;
    }
    if (lane == 0)
    {
        sa_result r;
        r.score = score;
        r.status = SA_OK;
        r.num_alignment_bytes = (uint64_t)len;
        r.start_text = (uint64_t)(int64_t)ti;
        r.start_pattern = (uint64_t)(int64_t)pi;
        a.results[p] = r;
    }
    const uint64_t tT1 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
    __syncthreads();  // the op bytes are visible to every lane (one wave: LDS / global order)

    // ops (walk order, i.e. reversed) -> letters (forward order), 64 ops per block with one op per
    // lane: the text / pattern index of op t is the start index minus the number of text / pattern
    // letters the ops before it consumed, i.e. a running base minus an in-block exclusive count
    // (ballot + mbcnt). kUnroll blocks per trip keep their loads in flight together.
    const uint64_t tT2 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
    {
        constexpr int kUnroll = 8;
        const char GAPC = alpha[a.A];
        char *ot = a.out_text + pd.out_off;
        char *op = a.out_pattern + pd.out_off;
        const int8_t *tx = a.text + pd.text_off;
        const int8_t *px = a.pattern + pd.pattern_off;
        int bt = ti0, bp = pi0;  // text / pattern index consumed by the next op
        for (int t0 = 0; t0 < len; t0 += kWave * kUnroll)
        {
            int d[kUnroll];
            sfor<kUnroll>([&](auto Uc) {
                constexpr int u = decltype(Uc)::value;
                const int t = t0 + u * kWave + lane;
                d[u] = t < len ? ops[t] : kStop;
            });
            int xt[kUnroll], xp[kUnroll], ct[kUnroll], cp[kUnroll];
            sfor<kUnroll>([&](auto Uc) {
                constexpr int u = decltype(Uc)::value;
                const bool tt = d[u] == kDiag || d[u] == kLeft;
                const bool tp = d[u] == kDiag || d[u] == kTop;
                const uint64_t mt = ballot(tt), mp = ballot(tp);
                xt[u] = bt - (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mt >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mt, 0));
                xp[u] = bp - (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mp >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mp, 0));
                ct[u] = tt ? (int)tx[max(xt[u], 0)] : -1;
                cp[u] = tp ? (int)px[max(xp[u], 0)] : -1;
                bt -= __builtin_popcountll(mt);
                bp -= __builtin_popcountll(mp);
            });
            sfor<kUnroll>([&](auto Uc) {
                constexpr int u = decltype(Uc)::value;
                const int t = t0 + u * kWave + lane;
                if (t < len)
                {
                    ot[len - 1 - t] = ct[u] >= 0 ? alpha[ct[u]] : GAPC;
                    op[len - 1 - t] = cp[u] >= 0 ? alpha[cp[u]] : GAPC;
                }
            });
        }
    }
    if (a.timing)
    {
        __syncthreads();
        if (lane == 0)
        {
            uint64_t *tm = a.timing + 4 * (size_t)p;
            tm[0] = tT0;
            tm[1] = tT1;
            tm[2] = tT2;
            tm[3] = __builtin_amdgcn_s_memrealtime();

        }
    }
}

// ------------------------------------------------------------------------------------------------
// self test of the wave primitives the kernels rely on
// ------------------------------------------------------------------------------------------------
__global__ void selftest_kernel(int *out)
{
    const int lane = threadIdx.x;
    const int v = 100 + lane;
    out[0 * 64 + lane] = dpp_shr1(-1, v);   // expect lane-1 (lane 0: -1)
    out[1 * 64 + lane] = dpp_shl1(-2, v);   // expect lane+1 (lane 63: -2)
    out[2 * 64 + lane] = dpp_rol1(v);       // expect lane+1 mod 64
    const uint64_t b = ballot((lane % 3) == 0);
    uint32_t acc = 0;
    writelane<5>(acc, (uint32_t)b);
    writelane<6>(acc, (uint32_t)(b >> 32));
    out[3 * 64 + lane] = (int)acc;
    out[4 * 64 + lane] = __builtin_amdgcn_sbfe(0x18F70A05, 8 * (lane & 3), 8);  // 5, 10, -9, 24
    // constant 100 MHz clock used by the hand-off timeout must advance
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 2000; ++k) __builtin_amdgcn_s_sleep(10);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[5 * 64 + lane] = (int)(t1 - t0);
}

}  // namespace sa

// ==================================================================================================
// host side
// ==================================================================================================
using namespace sa;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(SA_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// Environment knobs, read once per process (the first time the engine needs one) and never again:
// every field is a tuning or debugging switch; the defaults are the measured best settings.
struct Knobs {
    bool debug_sync = false;        // SA_DEBUG_SYNC: synchronise and check after every launch
    int rows_per_lane = 0;          // SA_ROWS_PER_LANE: force R (1..32)
    int waves_per_group = 0;        // SA_WAVES_PER_GROUP: force W (1..4)
    bool no_pair16 = false;         // SA_NO_PAIR16: disable the pair-packed batch fill
    double handoff_timeout_s = 20;  // SA_HANDOFF_TIMEOUT_S: in-kernel hand-off give-up time
    int io_sleep = 4;               // SA_IO_SLEEP: I/O wave idle poll period (s_sleep units)
    int chain_lds_kb = 0;           // SA_CHAIN_LDS_KB: dynamic LDS per chain workgroup
    const char *timeline = nullptr; // SA_TIMELINE=<file>: per-strip fill timestamps
    const char *tb_timing = nullptr;// SA_TB_TIMING=<file>: per-pair traceback timestamps
    bool tb_legacy = false;         // SA_TB_LEGACY: the step-by-step traceback kernel (A/B reference)
    bool tb_generic = false;        // SA_TB_GENERIC: row walk without the unrolled strip code
};

const Knobs &knobs()
{
    static const Knobs k = [] {
        Knobs v;
        auto get = [](const char *name) -> const char * { return std::getenv(name); };
        v.debug_sync = get("SA_DEBUG_SYNC") != nullptr;
        if (const char *e = get("SA_ROWS_PER_LANE")) v.rows_per_lane = std::atoi(e);
        if (const char *e = get("SA_WAVES_PER_GROUP")) v.waves_per_group = std::atoi(e);
        v.no_pair16 = get("SA_NO_PAIR16") != nullptr;
        if (const char *e = get("SA_HANDOFF_TIMEOUT_S")) v.handoff_timeout_s = std::atof(e);
        if (const char *e = get("SA_IO_SLEEP")) v.io_sleep = std::max(0, std::atoi(e));
        if (const char *e = get("SA_CHAIN_LDS_KB")) v.chain_lds_kb = std::max(0, std::atoi(e));
        v.timeline = get("SA_TIMELINE");
        v.tb_timing = get("SA_TB_TIMING");
        v.tb_legacy = get("SA_TB_LEGACY") != nullptr;
        v.tb_generic = get("SA_TB_GENERIC") != nullptr;
        return v;
    }();
    return k;
}

// SA_DEBUG_SYNC=1: synchronise and check after every launch (names the failing kernel).
int debug_sync(hipStream_t st, const char *what)
{
    if (!knobs().debug_sync) return SA_OK;
    hipError_t e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    std::fprintf(stderr, "[sa debug] %s ok\n", what);
    return SA_OK;
}

template <typename T>
int dmalloc(T **p, size_t bytes)
{
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    if (hipMalloc((void **)p, bytes) != hipSuccess)
    {
        (void)hipGetLastError();
        *p = nullptr;
        return fail(SA_ERR_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes failed");
    }
    return SA_OK;
}

}  // namespace

struct sa_plan {
    int device = 0;
    int mode = 0, A = 0, gap = 0, R = 0, U = 0, W = 1, key_bits = 12, key_rowbits = 21;
    int sk = 0;          // ScoreKind of the fill
    bool chain = false;  // some pair has more than one strip
    int num_cu = 0;
    std::vector<PairDesc> pairs;
    std::vector<StripDesc> strips;
    char alphabet[33] = {0};
    uint32_t epoch = 0;
    hipStream_t own = nullptr;
    // device
    PairDesc *d_pairs = nullptr;
    StripDesc *d_strips = nullptr;
    int32_t *d_prof = nullptr, *d_table = nullptr;
    int32_t *d_codes = nullptr;
    uint32_t *d_masks = nullptr;
    uint64_t *d_bnd = nullptr, *d_best = nullptr;
    int32_t *d_score = nullptr;
    Control *d_ctrl = nullptr;
    uint8_t *d_ops = nullptr;
    int32_t *d_rec = nullptr;  // traceback records (sa_walk.h)
    TbHead *d_heads = nullptr;
    char *d_out_text = nullptr, *d_out_pattern = nullptr;
    sa_result *d_results = nullptr;
    const int8_t *d_text_in = nullptr, *d_pattern_in = nullptr;
    uint64_t bytes_total = 0, bytes_masks = 0, out_bytes = 0;
    bool filled = false;
};

namespace {

int choose_R(const sa_params *P, const sa_pair *pairs, int64_t np)
{
    int R = P->rows_per_lane;
    if (knobs().rows_per_lane) R = knobs().rows_per_lane;
    if (R == 1 || R == 2 || R == 4 || R == 8 || R == 16 || R == 32) return R;
    uint64_t mmax = 0;
    for (int64_t p = 0; p < np; ++p) mmax = std::max<uint64_t>(mmax, pairs[p].pattern_len);
    if (np >= 256)
    {
        // many independent pairs: one strip per pair where possible (no hand-offs at all); local
        // mode keeps 3 registers per row (H, G, best key) and stops at 16 rows per lane, where
        // its working set still fits the register file
        const int rmax = P->mode == SA_LOCAL ? 16 : 32;
        int r = 1;
        while (r < rmax && (uint64_t)kWave * r < mmax) r <<= 1;
        return r;
    }
    // few long pairs: the shortest strips keep the wavefront deepest (one row per lane)
    return 1;
}

// Waves per workgroup (strips per group). Chains of strips (pairs taller than one strip) hand
// their rows off through LDS inside a group; single-strip pairs gain nothing from grouping.
int choose_W(const std::vector<PairDesc> &pairs)
{
    const int w = knobs().waves_per_group;
    if (w >= 1 && w <= kMaxWaves) return w;
    (void)pairs;
    return 4;
}

void launch_fill(int R, const FillArgs &a, bool local, int sk, int grid, int W, bool chain, hipStream_t st)
{
    switch (R)
    {
    case 1: launch_fill_r<1>(a, local, sk, grid, W, chain, st); break;
    case 2: launch_fill_r<2>(a, local, sk, grid, W, chain, st); break;
    case 4: launch_fill_r<4>(a, local, sk, grid, W, chain, st); break;
    case 8: launch_fill_r<8>(a, local, sk, grid, W, chain, st); break;
    case 16: launch_fill_r<16>(a, local, sk, grid, W, chain, st); break;
    default: launch_fill_r<32>(a, local, sk, grid, W, chain, st); break;
    }
}

template <int MODE>
void launch_tb_m(int R, const TbArgs &a, int np, hipStream_t st)
{
    switch (R)
    {
    case 1: hipLaunchKernelGGL((traceback_kernel<1, MODE>), dim3(np), dim3(kWave), 0, st, a); break;
    case 2: hipLaunchKernelGGL((traceback_kernel<2, MODE>), dim3(np), dim3(kWave), 0, st, a); break;
    case 4: hipLaunchKernelGGL((traceback_kernel<4, MODE>), dim3(np), dim3(kWave), 0, st, a); break;
    case 8: hipLaunchKernelGGL((traceback_kernel<8, MODE>), dim3(np), dim3(kWave), 0, st, a); break;
    case 16: hipLaunchKernelGGL((traceback_kernel<16, MODE>), dim3(np), dim3(kWave), 0, st, a); break;
    default: hipLaunchKernelGGL((traceback_kernel<32, MODE>), dim3(np), dim3(kWave), 0, st, a); break;
    }
}

void launch_tb(int R, const TbArgs &a, int np, hipStream_t st)
{
    if (a.mode == SA_GLOBAL) launch_tb_m<SA_GLOBAL>(R, a, np, st);
    else launch_tb_m<SA_LOCAL>(R, a, np, st);
}

void free_plan(sa_plan *p)
{
    if (!p) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(p->device);
    void *bufs[] = {p->d_pairs, p->d_strips, p->d_prof, p->d_table, p->d_codes, p->d_masks, p->d_bnd,
                    p->d_best, p->d_score, p->d_ctrl, p->d_ops, p->d_rec, p->d_heads, p->d_out_text,
                    p->d_out_pattern, p->d_results};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (p->own) (void)hipStreamDestroy(p->own);
    (void)hipSetDevice(cur);
    delete p;
}

int bitlen(uint64_t v)
{
    int b = 0;
    while (v) { ++b; v >>= 1; }
    return b;
}

}  // namespace

extern "C" {

const char *sa_last_error(void) { return g_err.c_str(); }
int sa_abi_version(void) { return SA_ABI_VERSION; }

int sa_device_count(int *count)
{
    HIP_TRY(hipGetDeviceCount(count));
    return SA_OK;
}

int sa_plan_create(const sa_params *P, const sa_pair *pairs, int64_t np, int device, sa_plan **out)
{
    if (!P || !out || np < 0 || (np > 0 && !pairs) || !P->score_matrix)
        return fail(SA_ERR_INVALID, "sa_plan_create: null argument");
    *out = nullptr;
    const int A = P->alphabet_size;
    if (A < 1 || A > 32) return fail(SA_ERR_INVALID, "alphabet_size must be 1..32");
    if (P->mode != SA_GLOBAL && P->mode != SA_LOCAL) return fail(SA_ERR_INVALID, "mode must be SA_GLOBAL or SA_LOCAL");
    // the reference takes a positive gap penalty (utilities.cpp parseArguments); the local
    // recurrence's saturating subtraction relies on g >= 0
    if (P->gap_penalty < 0) return fail(SA_ERR_UNSUPPORTED, "gap_penalty must be >= 0");
    const int64_t g = P->gap_penalty;
    int64_t smax = INT32_MIN, smin = INT32_MAX, sabs = 0;
    for (int e = 0; e < A * A; ++e)
    {
        smax = std::max<int64_t>(smax, P->score_matrix[e]);
        smin = std::min<int64_t>(smin, P->score_matrix[e]);
        sabs = std::max<int64_t>(sabs, std::llabs((long long)P->score_matrix[e]));
    }
    // numeric limits of the engine: every intermediate fits in int32, local keys fit.
    uint64_t hmax_local = 0, lmax = 0;
    for (int64_t p = 0; p < np; ++p)
    {
        const uint64_t n = pairs[p].text_len, m = pairs[p].pattern_len;
        if (n >= (1u << 24) - 1 || m >= (1u << 24) - 1)
            return fail(SA_ERR_UNSUPPORTED, "sequence longer than 2^24-2 letters");
        lmax = std::max(lmax, std::max(n, m));
        const uint64_t span = n + m;
        const uint64_t bound = ((uint64_t)sabs + (uint64_t)std::llabs(g)) * span + (uint64_t)std::llabs(g) * span;
        if (bound >= (1ull << 30)) return fail(SA_ERR_UNSUPPORTED, "scores may exceed the int32 range");
        const uint64_t h = g >= 0 ? (uint64_t)std::max<int64_t>(smax, 0) * std::min(n, m)
                                  : ((uint64_t)sabs + (uint64_t)(-g)) * span;
        hmax_local = std::max(hmax_local, h);
    }
    // local best-cell keys: H | ~row | ~col in 64 bits, row / column fields sized for the longest
    // sequence; the in-kernel block key (H << key_bits) + step must stay inside int32
    const int key_rowbits = std::max(1, bitlen(lmax + 1));
    if (P->mode == SA_LOCAL && (bitlen(hmax_local) > 26 || bitlen(hmax_local) > 64 - 2 * key_rowbits))
        return fail(SA_ERR_UNSUPPORTED, "local scores may exceed the best-cell key range");

    sa_plan *pl = new sa_plan();
    pl->device = device;
    pl->mode = P->mode;
    pl->A = A;
    pl->gap = (int)g;
    pl->R = choose_R(P, pairs, np);
    pl->U = (16 / pl->R) > 4 ? 16 / pl->R : 4;
    pl->key_bits = std::min(12, std::max(4, 30 - bitlen(hmax_local)));
    pl->key_rowbits = key_rowbits;
    // the tables hold S + 2g (global, shifted domain) or S + g (local), see run_body
    const int64_t off2 = P->mode == SA_GLOBAL ? 2 * g : g;
    bool fits8 = true;
    for (int e = 0; e < A * A; ++e)
    {
        const int64_t v = P->score_matrix[e] + off2;
        if (v < -128 || v > 127) fits8 = false;
    }
    if (pl->R == 1) pl->sk = fits8 ? kArr8 : kArr;
    else pl->sk = (A <= 4 && fits8) ? kProf : kTable;
    if (P->alphabet) std::memcpy(pl->alphabet, P->alphabet, std::min<size_t>(A + 1, 33));
    else for (int c = 0; c <= A; ++c) pl->alphabet[c] = c == A ? '-' : (char)('A' + c);

    int cur = 0;
    (void)hipGetDevice(&cur);
    auto restore = [&]() { (void)hipSetDevice(cur); };
    if (hipSetDevice(device) != hipSuccess) { delete pl; restore(); return fail(SA_ERR_HIP, "hipSetDevice failed"); }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { delete pl; restore(); return fail(SA_ERR_HIP, "hipGetDeviceProperties failed"); }
    pl->num_cu = prop.multiProcessorCount;

    // ---- layout ----
    const int R = pl->R, U = pl->U, RB = kWave * R;
    uint64_t code_bytes = 0, mask_entries = 0, granules = 0, outb = 0, recw = 0;
    pl->pairs.resize(np);
    for (int64_t p = 0; p < np; ++p)
    {
        PairDesc &d = pl->pairs[p];
        d.text_off = pairs[p].text_offset;
        d.text_len = pairs[p].text_len;
        d.pattern_off = pairs[p].pattern_offset;
        d.pattern_len = pairs[p].pattern_len;
        d.code_off = code_bytes;
        // kArr8: code_len bytes per copy (4A copies); kArr: A arrays of code_len dwords; else one
        d.code_len = (kPad + d.text_len + 4 * kPad + 3) / 4 * 4;
        // (a possible pair-packed plan, decided below, needs two column profiles per column)
        const bool maybePair = P->mode == SA_GLOBAL && R >= 16 && A <= 4;
        code_bytes += pl->sk == kArr8 ? (uint64_t)A * d.code_len : pl->sk == kArr ? (uint64_t)A * d.code_len
                                                                                : (maybePair ? 2 : 1) * d.code_len;
        d.out_off = outb;
        outb += d.text_len + d.pattern_len + 16;
        d.rec_off = recw;
        recw += std::max(d.text_len, d.pattern_len) + 64;
        d.first_strip = (int32_t)pl->strips.size();
        const uint64_t n = d.text_len, m = d.pattern_len;
        const int ns = (n == 0 || m == 0) ? 0 : (int)((m + RB - 1) / RB);
        d.num_strips = ns;
        const int nsteps = (int)(((n + kWave - 1) + 2 * U - 1) / (2 * U) * (2 * U));  // two bodies per loop trip
        for (int b = 0; b < ns; ++b)
        {
            StripDesc s;
            s.pair = (int32_t)p;
            s.row0 = 1 + b * RB;
            s.flags = (b > 0 ? kHasPrev : 0) | (b + 1 < ns ? kHasNext : 0);
            s.nsteps = nsteps;
            s.mask_off = mask_entries;
            mask_entries += (uint64_t)nsteps * R;
            s.bnd_in = b > 0 ? pl->strips.back().bnd_out : 0;
            s.bnd_out = granules;
            if (b + 1 < ns) granules += n + 8;
            pl->strips.push_back(s);
        }
    }
    if (pl->strips.size() >= (1u << 31)) { delete pl; restore(); return fail(SA_ERR_UNSUPPORTED, "too many strips"); }
    pl->out_bytes = outb;
    pl->bytes_masks = mask_entries * 16;
    pl->W = choose_W(pl->pairs);
    for (const PairDesc &d : pl->pairs) pl->chain = pl->chain || d.num_strips > 1;
    {
        // pair-packed fill (fill_pair_kernel): global, lone strips of one shape, DNA-sized alphabet,
        // every S + 2g in [0, 255] and every value within u16 (see process_pair)
        bool pair = P->mode == SA_GLOBAL && !pl->chain && np >= 2 && np % 2 == 0 && A <= 4 && R >= 16 &&
                    !knobs().no_pair16;
        int64_t smaxp = 0;
        for (int e = 0; e < A * A; ++e)
        {
            const int64_t v = P->score_matrix[e] + off2;
            if (v < 0 || v > 255) pair = false;
            smaxp = std::max(smaxp, v);
        }
        for (int64_t p = 0; p < np && pair; ++p)
        {
            const PairDesc &d = pl->pairs[p];
            if (d.text_len != pl->pairs[0].text_len || d.pattern_len != pl->pairs[0].pattern_len || d.num_strips != 1)
                pair = false;
            else if ((uint64_t)smaxp * std::min(d.text_len, d.pattern_len) > 65535)
                pair = false;
        }
        if (pair) pl->sk = kPair;
    }

    // ---- tables ----
    std::vector<int32_t> prof(4, 0), table(A * A);
    for (int e = 0; e < A * A; ++e) table[e] = (int32_t)(P->score_matrix[e] + off2);
    if (pl->sk == kProf || pl->sk == kPair)
        for (int cp = 0; cp < A; ++cp)
        {
            uint32_t w = 0;
            for (int ct = 0; ct < A; ++ct) w |= (uint32_t)(table[cp * A + ct] & 0xff) << (8 * ct);
            prof[cp] = (int32_t)w;
        }

    // ---- device buffers ----
    int rc = SA_OK;
    auto alloc = [&](auto **ptr, size_t bytes) {
        if (rc == SA_OK) { rc = dmalloc(ptr, bytes); pl->bytes_total += bytes; }
    };
    alloc(&pl->d_pairs, sizeof(PairDesc) * std::max<size_t>(1, np));
    alloc(&pl->d_strips, sizeof(StripDesc) * std::max<size_t>(1, pl->strips.size()));
    alloc(&pl->d_prof, sizeof(int32_t) * 4);
    alloc(&pl->d_table, sizeof(int32_t) * A * A);
    alloc(&pl->d_codes, 4 * code_bytes + 16);
    // (+8 KiB: the traceback's plane prefetch may read a few chunks past a strip)
    alloc(&pl->d_masks, pl->bytes_masks + 8192);
    alloc(&pl->d_bnd, granules * 8 + 16);
    alloc(&pl->d_best, sizeof(uint64_t) * std::max<size_t>(1, pl->strips.size()));
    alloc(&pl->d_score, sizeof(int32_t) * std::max<size_t>(1, np));
    alloc(&pl->d_ctrl, sizeof(Control));
    alloc(&pl->d_ops, outb + 16);
    alloc(&pl->d_rec, 4 * recw + 16);
    alloc(&pl->d_heads, sizeof(TbHead) * std::max<size_t>(1, np));
    alloc(&pl->d_out_text, outb + 16);
    alloc(&pl->d_out_pattern, outb + 16);
    alloc(&pl->d_results, sizeof(sa_result) * std::max<size_t>(1, np));
    if (rc != SA_OK) { free_plan(pl); restore(); return rc; }
    if (hipStreamCreateWithFlags(&pl->own, hipStreamNonBlocking) != hipSuccess) { free_plan(pl); restore(); return fail(SA_ERR_HIP, "stream creation failed"); }
    bool okc = hipMemcpy(pl->d_pairs, pl->pairs.data(), sizeof(PairDesc) * np, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(pl->d_strips, pl->strips.data(), sizeof(StripDesc) * pl->strips.size(), hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(pl->d_prof, prof.data(), sizeof(int32_t) * 4, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(pl->d_table, table.data(), sizeof(int32_t) * A * A, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemset(pl->d_codes, 0, 4 * code_bytes + 16) == hipSuccess &&
               hipMemset(pl->d_bnd, 0, granules * 8 + 16) == hipSuccess &&
               hipMemset(pl->d_best, 0, sizeof(uint64_t) * std::max<size_t>(1, pl->strips.size())) == hipSuccess;
    if (!okc) { free_plan(pl); restore(); return fail(SA_ERR_HIP, "plan upload failed"); }
    restore();
    *out = pl;
    return SA_OK;
}

int sa_plan_destroy(sa_plan *plan)
{
    free_plan(plan);
    return SA_OK;
}

int sa_plan_fill(sa_plan *pl, const void *d_text, const void *d_pattern, void *stream)
{
    if (!pl || (!pl->pairs.empty() && (!d_text || !d_pattern))) return fail(SA_ERR_INVALID, "sa_plan_fill: null argument");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(pl->device));
    pl->d_text_in = (const int8_t *)d_text;
    pl->d_pattern_in = (const int8_t *)d_pattern;
    pl->epoch += 1;
    if (pl->epoch == 0) pl->epoch = 1;
    HIP_TRY(hipMemsetAsync(pl->d_ctrl, 0, sizeof(Control), st));
    const int np = (int)pl->pairs.size();
    if (np > 0)
    {
        uint64_t nmax = 1;
        for (auto &d : pl->pairs) nmax = std::max<uint64_t>(nmax, d.text_len);
        const int gx = (int)std::min<uint64_t>((nmax + 255) / 256, 64);
        for (int y0 = 0; y0 < np; y0 += 65534)
        {
            // pairs beyond 65535 are handled by re-basing the pair pointer
            const int cnt = std::min(65534, np - y0);  // even: kPair pairs (2q, 2q+1) stay in one launch
            hipLaunchKernelGGL(encode_text_kernel, dim3(gx, cnt), dim3(256), 0, st, (const int8_t *)d_text,
                               pl->d_pairs + y0, pl->d_codes, pl->A, pl->sk, pl->d_table);
        }
        HIP_TRY(hipGetLastError());
        if (int rc = debug_sync(st, "encode_text_kernel")) return rc;
    }
    const int ns = (int)pl->strips.size();
    if (ns > 0)
    {
        FillArgs a;
        a.pattern = (const int8_t *)d_pattern;
        a.codes = pl->d_codes;
        a.strips = pl->d_strips;
        a.pairs = pl->d_pairs;
        a.prof_tab = pl->d_prof;
        a.score_tab = pl->d_table;
        a.masks = pl->d_masks;
        a.bnd = pl->d_bnd;
        a.strip_best = pl->d_best;
        a.pair_score = pl->d_score;
        a.ctrl = pl->d_ctrl;
        a.num_strips = ns;
        a.gap = pl->gap;
        a.A = pl->A;
        a.epoch = pl->epoch;
        a.key_bits = pl->key_bits;
        a.key_rowbits = pl->key_rowbits;
        a.timeout_ticks = (uint64_t)(knobs().handoff_timeout_s * 1e8);
        a.io_sleep = knobs().io_sleep;
        a.chain_lds = knobs().chain_lds_kb * 1024;
        // SA_TIMELINE=<file>: debug dump of per-strip timestamps (s_memrealtime, 100 MHz)
        const char *tlPath = knobs().timeline;
        a.timeline = nullptr;
        if (tlPath) HIP_TRY(hipMalloc((void **)&a.timeline, sizeof(uint64_t) * kTimelineWords * ns));
        const int W = pl->W;
        a.num_groups = (ns + W - 1) / W;
        // chains: two workgroups of W compute waves + an I/O wave per CU; lone strips: W compute
        // waves per workgroup and up to 16 waves per CU (the batch kernel stays under 128 VGPRs)
        const int perCU = pl->chain ? std::max(1, 8 / W) : std::max(1, 16 / W);
        int grid = std::min(a.num_groups, std::max(1, pl->num_cu) * perCU);
        if (pl->sk == kPair)
        {
            // one wave per two strips
            const int units = ns / 2;
            a.num_groups = (units + W - 1) / W;
            grid = std::min(a.num_groups, std::max(1, pl->num_cu) * std::max(1, 8 / W));
        }
        launch_fill(pl->R, a, pl->mode == SA_LOCAL, pl->sk, grid, W, pl->chain, st);
        HIP_TRY(hipGetLastError());
        if (tlPath)
        {
            std::vector<uint64_t> tl(kTimelineWords * (size_t)ns);
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipMemcpy(tl.data(), a.timeline, tl.size() * 8, hipMemcpyDeviceToHost));
            HIP_TRY(hipFree(a.timeline));
            if (FILE *f = std::fopen(tlPath, "wb"))
            {
                std::fwrite(tl.data(), 8, tl.size(), f);
                std::fclose(f);
            }
        }
        if (int rc = debug_sync(st, "fill_kernel")) return rc;
    }
    pl->filled = true;
    HIP_TRY(hipSetDevice(cur));
    return SA_OK;
}

int sa_plan_traceback(sa_plan *pl, void *stream)
{
    if (!pl || !pl->filled) return fail(SA_ERR_INVALID, "sa_plan_traceback: plan not filled");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    const int np = (int)pl->pairs.size();
    if (np == 0) return SA_OK;
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(pl->device));
    const Knobs &kn = knobs();
    // SA_TB_TIMING=<file>: debug dump of per-pair phase timestamps (s_memrealtime, 100 MHz)
    const char *tmPath = kn.tb_timing;
    uint64_t *timing = nullptr;
    if (tmPath) HIP_TRY(hipMalloc((void **)&timing, sizeof(uint64_t) * 4 * np));
    if (!kn.tb_legacy)
    {
        // row / column walk (records) + expansion (sa_walk.hip)
        WalkArgs w;
        w.strips = pl->d_strips;
        w.pairs = pl->d_pairs;
        w.masks = pl->d_masks;
        w.strip_best = pl->d_best;
        w.pair_score = pl->d_score;
        w.rec = pl->d_rec;
        w.heads = pl->d_heads;
        w.timing = timing;
        w.gap = pl->gap;
        w.key_rowbits = pl->key_rowbits;
        w.fast = kn.tb_generic ? 0 : 1;
        launch_walk(pl->R, pl->mode == SA_LOCAL, w, np, st);
        HIP_TRY(hipGetLastError());
        if (int rc = debug_sync(st, "walk kernel")) return rc;
        ExpandArgs x;
        x.text = pl->d_text_in;
        x.pattern = pl->d_pattern_in;
        x.pairs = pl->d_pairs;
        x.rec = pl->d_rec;
        x.heads = pl->d_heads;
        x.out_text = pl->d_out_text;
        x.out_pattern = pl->d_out_pattern;
        x.results = pl->d_results;
        x.A = pl->A;
        std::memcpy(x.alphabet, pl->alphabet, 33);
        launch_expand(x, np, st);
        HIP_TRY(hipGetLastError());
        if (int rc = debug_sync(st, "expand_kernel")) return rc;
    }
    else
    {
        TbArgs a;
        a.text = pl->d_text_in;
        a.pattern = pl->d_pattern_in;
        a.strips = pl->d_strips;
        a.pairs = pl->d_pairs;
        a.masks = (const uint4 *)pl->d_masks;
        a.strip_best = pl->d_best;
        a.pair_score = pl->d_score;
        a.ops = pl->d_ops;
        a.out_text = pl->d_out_text;
        a.out_pattern = pl->d_out_pattern;
        a.results = pl->d_results;
        a.mode = pl->mode;
        a.gap = pl->gap;
        a.A = pl->A;
        a.key_rowbits = pl->key_rowbits;
        std::memcpy(a.alphabet, pl->alphabet, 33);
        a.timing = timing;
        launch_tb(pl->R, a, np, st);
        HIP_TRY(hipGetLastError());
        if (int rc = debug_sync(st, "traceback_kernel")) return rc;
    }
    if (tmPath)
    {
        std::vector<uint64_t> tm(4 * (size_t)np);
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipMemcpy(tm.data(), timing, tm.size() * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(timing));
        if (FILE *f = std::fopen(tmPath, "wb"))
        {
            std::fwrite(tm.data(), 8, tm.size(), f);
            std::fclose(f);
        }
    }
    HIP_TRY(hipSetDevice(cur));
    return SA_OK;
}

int sa_plan_fetch_results(sa_plan *pl, sa_result *out, void *stream)
{
    if (!pl || !out) return fail(SA_ERR_INVALID, "sa_plan_fetch_results: null argument");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(pl->device));
    Control ctrl;
    HIP_TRY(hipMemcpyAsync(&ctrl, pl->d_ctrl, sizeof(Control), hipMemcpyDeviceToHost, st));
    if (!pl->pairs.empty())
        HIP_TRY(hipMemcpyAsync(out, pl->d_results, sizeof(sa_result) * pl->pairs.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipSetDevice(cur));
    if (ctrl.abort_flag) return fail(SA_ERR_TIMEOUT, "fill aborted: a strip hand-off timed out");
    return SA_OK;
}

int sa_plan_fetch_alignment(sa_plan *pl, int64_t index, char *at, char *ap, uint64_t cap, void *stream)
{
    if (!pl || index < 0 || index >= (int64_t)pl->pairs.size()) return fail(SA_ERR_INVALID, "sa_plan_fetch_alignment: bad index");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(pl->device));
    sa_result r;
    HIP_TRY(hipMemcpyAsync(&r, pl->d_results + index, sizeof(r), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (r.num_alignment_bytes > cap) { (void)hipSetDevice(cur); return fail(SA_ERR_INVALID, "output capacity too small"); }
    const uint64_t off = pl->pairs[index].out_off;
    if (r.num_alignment_bytes)
    {
        if (at) HIP_TRY(hipMemcpyAsync(at, pl->d_out_text + off, r.num_alignment_bytes, hipMemcpyDeviceToHost, st));
        if (ap) HIP_TRY(hipMemcpyAsync(ap, pl->d_out_pattern + off, r.num_alignment_bytes, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    HIP_TRY(hipSetDevice(cur));
    return SA_OK;
}

int sa_plan_fetch_directions(sa_plan *pl, int64_t index, uint8_t *M, void *stream)
{
    if (!pl || !M || index < 0 || index >= (int64_t)pl->pairs.size()) return fail(SA_ERR_INVALID, "sa_plan_fetch_directions: bad argument");
    hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream
    const PairDesc &pd = pl->pairs[index];
    const uint64_t n = pd.text_len, m = pd.pattern_len, cols = n + 1;
    const bool local = pl->mode == SA_LOCAL;
    for (uint64_t j = 0; j < cols; ++j) M[j] = local ? 3 : 0;          // row 0: STOP / LEFT
    for (uint64_t i = 1; i <= m; ++i) M[i * cols] = local ? 3 : 2;     // column 0: STOP / TOP
    if (pd.num_strips == 0) return SA_OK;
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(pl->device));
    const StripDesc &first = pl->strips[pd.first_strip];
    const StripDesc &last = pl->strips[pd.first_strip + pd.num_strips - 1];
    const uint64_t e0 = first.mask_off, e1 = last.mask_off + (uint64_t)last.nsteps * pl->R;
    std::vector<uint32_t> h((e1 - e0) * 4);
    HIP_TRY(hipMemcpyAsync(h.data(), pl->d_masks + e0 * 4, h.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipSetDevice(cur));
    const int R = pl->R, RB = kWave * R;
    const uint64_t CS = std::max(32, pl->U * R), NW = CS / 32, LW = 2 * NW;  // Cfg<R>
    for (uint64_t i = 1; i <= m; ++i)
    {
        const uint64_t b = (i - 1) / RB, il = (i - 1) % RB, k = il / R, rho = il % R;
        const StripDesc &sd = pl->strips[pd.first_strip + b];
        for (uint64_t j = 1; j <= n; ++j)
        {
            // slot e of the strip: chunk e/CS, lane k's LW words, plane word (e%CS)/32, bit 31-e%32
            const uint64_t e = (j - 1 + k) * R + rho;
            const uint32_t *w = &h[(sd.mask_off - e0) * 4 + (e / CS) * kWave * LW + k * LW + (e % CS) / 32];
            const uint32_t b0 = (w[0] >> (31 - e % 32)) & 1u;
            const uint32_t b1 = (w[NW] >> (31 - e % 32)) & 1u;
            // global: plane1 is the raw "up > left" bit and DIAG wins (see run_body)
            M[i * cols + j] = (uint8_t)(pl->mode == SA_GLOBAL ? (b0 ? 1u : (b1 ? 2u : 0u)) : (b0 | (b1 << 1)));
        }
    }
    return SA_OK;
}

int sa_plan_info(const sa_plan *pl, int64_t *num_strips, int32_t *rows_per_lane, uint64_t *device_bytes,
                 uint64_t *mask_bytes)
{
    if (!pl) return fail(SA_ERR_INVALID, "sa_plan_info: null plan");
    if (num_strips) *num_strips = (int64_t)pl->strips.size();
    if (rows_per_lane) *rows_per_lane = pl->R;
    if (device_bytes) *device_bytes = pl->bytes_total;
    if (mask_bytes) *mask_bytes = pl->bytes_masks;
    return SA_OK;
}

const void *sa_plan_device_results(const sa_plan *pl) { return pl ? (const void *)pl->d_results : nullptr; }

int sa_align_pair(const sa_params *P, const char *text, uint64_t n, const char *pattern, uint64_t m, int device,
                  sa_result *out, char *at, char *ap, uint64_t cap, double *fill_us)
{
    if (!P || !out || (n && !text) || (m && !pattern)) return fail(SA_ERR_INVALID, "sa_align_pair: null argument");
    const bool fillOnly = !at && !ap;  // -DBENCHMARK contract: DP fill only
    if (!fillOnly && cap < n + m) return fail(SA_ERR_INVALID, "sa_align_pair: output capacity below text_len + pattern_len");
    for (uint64_t x = 0; x < n; ++x)
        if (text[x] < 0 || text[x] >= P->alphabet_size) return fail(SA_ERR_INVALID, "text byte outside the alphabet");
    for (uint64_t x = 0; x < m; ++x)
        if (pattern[x] < 0 || pattern[x] >= P->alphabet_size) return fail(SA_ERR_INVALID, "pattern byte outside the alphabet");
    sa_pair pr{0, n, 0, m};
    sa_plan *pl = nullptr;
    int rc = sa_plan_create(P, &pr, 1, device, &pl);
    if (rc) return rc;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    int8_t *dt = nullptr, *dp = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto cleanup = [&]() {
        if (dt) (void)hipFree(dt);
        if (dp) (void)hipFree(dp);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        sa_plan_destroy(pl);
        (void)hipSetDevice(cur);
    };
    if ((rc = dmalloc(&dt, n + 16)) || (rc = dmalloc(&dp, m + 16))) { cleanup(); return rc; }
    if (hipMemcpyAsync(dt, text, n, hipMemcpyHostToDevice, pl->own) != hipSuccess ||
        hipMemcpyAsync(dp, pattern, m, hipMemcpyHostToDevice, pl->own) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    {
        cleanup();
        return fail(SA_ERR_HIP, "sa_align_pair: upload failed");
    }
    (void)hipEventRecord(e0, pl->own);
    rc = sa_plan_fill(pl, dt, dp, pl->own);
    (void)hipEventRecord(e1, pl->own);
    if (!rc && !fillOnly) rc = sa_plan_traceback(pl, pl->own);
    if (!rc && !fillOnly) rc = sa_plan_fetch_results(pl, out, pl->own);
    if (!rc && !fillOnly) rc = sa_plan_fetch_alignment(pl, 0, at, ap, cap, pl->own);
    if (!rc && fillOnly && hipStreamSynchronize(pl->own) != hipSuccess) rc = fail(SA_ERR_HIP, "sa_align_pair: sync failed");
    if (!rc && fill_us)
    {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        *fill_us = 1000.0 * ms;
    }
    cleanup();
    return rc;
}

int sa_selftest(int device)
{
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(device));
    int *d = nullptr;
    HIP_TRY(hipMalloc(&d, 6 * 64 * sizeof(int)));
    hipLaunchKernelGGL(selftest_kernel, dim3(1), dim3(64), 0, 0, d);
    std::vector<int> h(6 * 64);
    HIP_TRY(hipMemcpy(h.data(), d, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(d));
    HIP_TRY(hipSetDevice(cur));
    uint64_t b = 0;
    for (int l = 0; l < 64; ++l)
        if (l % 3 == 0) b |= 1ull << l;
    const int sbfe[4] = {5, 10, -9, 24};
    for (int l = 0; l < 64; ++l)
    {
        if (h[l] != (l == 0 ? -1 : 100 + l - 1)) return fail(SA_ERR_UNSUPPORTED, "DPP wave_shr:1 mismatch at lane " + std::to_string(l));
        if (h[64 + l] != (l == 63 ? -2 : 100 + l + 1)) return fail(SA_ERR_UNSUPPORTED, "DPP wave_shl:1 mismatch at lane " + std::to_string(l));
        if (h[128 + l] != 100 + (l + 1) % 64) return fail(SA_ERR_UNSUPPORTED, "DPP wave_rol:1 mismatch at lane " + std::to_string(l));
        const int wl = l == 5 ? (int)(uint32_t)b : (l == 6 ? (int)(uint32_t)(b >> 32) : 0);
        if (h[192 + l] != wl) return fail(SA_ERR_UNSUPPORTED, "ballot/writelane mismatch at lane " + std::to_string(l));
        if (h[256 + l] != sbfe[l & 3]) return fail(SA_ERR_UNSUPPORTED, "v_bfe_i32 mismatch at lane " + std::to_string(l));
        if (h[320 + l] <= 0) return fail(SA_ERR_UNSUPPORTED, "s_memrealtime does not advance (" + std::to_string(h[320 + l]) + ")");
    }
    return SA_OK;
}

}  // extern "C"

#endif  // SA_FILL_R
