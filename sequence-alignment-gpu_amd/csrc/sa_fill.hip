// MI355X (gfx950 / CDNA4) DP fill kernels: Needleman-Wunsch / Smith-Waterman direction planes.
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
//
// Compiled once per strip height R: fill_r<R>.hip defines SA_FILL_R and includes this file.
#ifndef SA_FILL_R
#error "sa_fill.hip is compiled through fill_r<R>.hip (SA_FILL_R = strip rows per lane)"
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "sa_fill.h"
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
__device__ __forceinline__ uint32_t lds_off(const lds_int *p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ void ds_write_async(lds_int *p, int v) { asm volatile("ds_write_b32 %0, %1" ::"v"(lds_off(p)), "v"(v)); }
// LDS read and wait in one statement (slow paths: the register cannot be touched before the data
// is there, and the compiler's waitcnt pass sees no pending LDS load it would have to merge into the
// fast path's state; a compiler-visible read here put an s_waitcnt lgkmcnt(0) at every body's top)
__device__ __forceinline__ int ds_read_sync(const lds_int *p)
{
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_off(p)));
    return v;
}
constexpr int kRing = 2048;        // ring entries (columns), power of two
constexpr int kRingMask = kRing - 1;
// Tuning constants of the shipped build. Development builds (tools/build_exp.sh defines
// SA_EXPERIMENT) may override the ones below and enable timing ablations (SA_EXP_*: results wrong by
// design); the shipped build refuses any override, so a stray -D cannot change what it computes.
#ifdef SA_EXPERIMENT
#ifndef SA_PF_LEAD
#define SA_PF_LEAD 4
#endif
#ifndef SA_FILL_ASM
#define SA_FILL_ASM 1
#endif
#ifndef SA_DRAIN_WAVES
#define SA_DRAIN_WAVES 1
#endif
#else
#if defined(SA_PF_LEAD) || defined(SA_FILL_ASM) || defined(SA_EXP_CODES_CONST) || defined(SA_EXP_NO_STORE) || \
    defined(SA_EXP_NO_FEED_WAIT) || defined(SA_EXP_NODIR) || defined(SA_EXP_NO_MERGE) || defined(SA_EXP_FILL_INC) || \
    defined(SA_EXP_BROW_AUX) || defined(SA_EXP_NO_STRIPS) || defined(SA_EXP_NO_DRAIN) || defined(SA_DRAIN_WAVES) || \
    defined(SA_EXP_BAND_STAMPS) || defined(SA_EXP_BAND_WAIT_SLEEP)
#error "experiment switches need SA_EXPERIMENT (tools/build_exp.sh)"
#endif
#define SA_PF_LEAD 4   // R = 1: steps between a body's feed read and its use (sa_fill_steps.inc matches)
#define SA_FILL_ASM 1  // hand-scheduled steady steps (0: the compiler-scheduled run_body)
#define SA_DRAIN_WAVES 1  // band workgroups: drain waves (three, one per ring, measured no faster global and 5 % slower local)
#endif
constexpr int kDrainWaves = SA_DRAIN_WAVES;
constexpr int kBufRsrcWord3 = 0x00020000;  // gfx9 raw buffer resource, dword 3 (no format, no swizzle)
constexpr int kAuxSc1 = 16;                // buffer access cache policy: sc1 (agent-coherent, as the granules)
constexpr int kCodeAhead = 2;  // R = 1: text-code loads run two bodies ahead (bodies in quads)

struct GroupHdr {
    int S[32 * 32];                // generic score table (A <= 32)
    int cons[kMaxWaves + 1];       // cons[w]: columns read from ring[w] (producer backpressure)
    int drain[kMaxWaves + 1];      // band fill: drain[w]: columns of ring[w] copied to granules
    int group;                     // group index taken from the queue
    int nwaves;                    // compute waves of the workgroup (W)
};
// chain workgroup LDS: header, W + 1 rings, then one shared sink that the lanes carrying no
// bottom-row value write into when their wave publishes (a ring's size plus a wave, so that a
// lane's sink slot is its ring slot offset: the publish address is one add per body)
constexpr int kSink = kRing + kWave;
__host__ __device__ constexpr size_t group_lds_bytes(int W) { return sizeof(GroupHdr) + ((size_t)(W + 1) * kRing + kSink) * 4; }
// What a strip's waves see of their workgroup's LDS (GroupHdr)
struct StripLds {
    const int *S;   // generic score table (kTable)
    int *cons;      // cons[w]: columns read from ring[w] (producer backpressure)
    int nwaves;     // strips of the workgroup (W): the shared sink follows ring W
    int *drain;     // band fill: drain[w] = columns of ring[w] copied to granules (drain / I/O wave)
};

// Constant 100 MHz clock, read and waited for in one statement: a compiler-visible s_memrealtime
// in a slow path can leave its SMEM result "pending" at the join with the fast path, and the
// waitcnt pass then puts an s_waitcnt lgkmcnt(0) into every body that reads the reused SGPRs.
__device__ __forceinline__ uint64_t now_ticks()
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

// Bounded-spin helper, called every few polls: false (and the abort word raised) after the
// timeout, or as soon as another wave has given up.
__device__ __forceinline__ bool keep_waiting(const FillArgs &a, uint64_t t0, int lane)
{
    // 100 MHz constant clock
    const bool late = now_ticks() - t0 > a.timeout_ticks;
    if (late && lane == 0) __hip_atomic_store(&a.ctrl->abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int aborted = uniform((int)__hip_atomic_load(&a.ctrl->abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return !(aborted || late);
}

// Ring slot of column c (1-based) in every LDS ring, and the tag its entry carries in bit 31.
// Entries are self-validating: a value (always in [0, 2^30)) is stored with bit 31 =
// the complement of its lap's parity, lap = (c + 63) / kRing, so a reader needs no progress word: a
// slot holds column c exactly when its tag is c's (the zeroed ring of a new group matches no lap-0
// column; a slot still holding the previous lap's column has the other parity). The +63 makes a
// producer body's columns (s0 - 63 .. s0 - 64 + U, s0 a multiple of U) one aligned run of slots
// inside one lap, so its tag is uniform.
__device__ __forceinline__ int ring_slot(int c) { return (c + 63) & kRingMask; }
__device__ __forceinline__ int ring_tag(int c) { return (int)((((uint32_t)(c + 63) >> 11) & 1u) ^ 1u) << 31; }
// (c + 63) << 20: bit 31 is the complement of ring_tag(c); the asm bodies apply it with one v_bitop3
// (tag = ~raw & 0x80000000), which saves the SALU masking per body
__device__ __forceinline__ int ring_tag_raw(int c) { return (int)((uint32_t)(c + 63) << 20); }
static_assert(kRing == 2048, "ring_tag assumes 2048-entry rings");
constexpr int kConsEvery = 256;  // a consumer publishes its consumption word every this many columns
constexpr int kIoWin = 4;        // I/O wave: 64-column windows polled / drained per round


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
//            Local with g < 0 cannot use this (an all-zero neighbourhood gives H = -g, not 0): its
//            first bodies are kGeneric instead.
//   kGeneric lanes outside [1, n] keep their state (the strip holding the global score's row,
//            local strips' last bodies, and local strips' first bodies when g < 0).
enum BodyKind { kSteady = 0, kStart = 1, kGeneric = 2 };
// Recurrences (per lane-row; diag/up/left are the neighbours' values):
//   global, shifted domain F = H + g(i+j): F = max(Fdiag + S + 2g, Fleft, Fup), boundaries 0;
//     DIAG iff Fdiag + S + 2g > max(Fleft, Fup); plane 1 = raw "up > left".
//   local, H with the gap folded into the score: X = max(Hdiag + S + g, max(Hleft, Hup), g),
//     H = X - g (= max(X' - g, 0) for g > 0, X' - g for g <= 0: X' >= 0); DIAG iff Hdiag + S + g > max(Hleft,
//     Hup) (the reference's D > max(L, U) with every candidate shifted by +g); raw TOP iff Hup >
//     Hleft; STOP iff H == 0 (alignSequenceCPU.cpp:175-190), stored only for R > 1 (R = 1: the row
//     walk recomputes H along the path, sa_walk.hip).
// Lane moves per step: `up` (the row above each lane's first row) is F[R-1] of lane k-1 by a DPP
// wave_shr:1 whose `old` operand is this step's feed register Q (lane 0 keeps Q's lane 0 = the
// strip above's bottom value for this column); Q is dead afterwards, so the DPP writes in place. The
// next step's feed register is Q shifted down one lane (wave_shl:1), computed first. With a strip
// below (HN) that shift's `old` is F[R-1], so lane 63 takes in the previous step's bottom-row value:
// after U steps lanes 64-U..63 of Q hold the bottom row of steps s0-1 .. s0+U-2, and one full-wave
// ds_write publishes them (the other lanes write a dummy slot). Steps [QB, QE) of the body.
template <int R, bool LOCAL, int SK, int KIND, bool HN, int QB, int QE>
__device__ __forceinline__ void run_body(const int *__restrict__ ldsS, int s0, int lane, int n, int g,
                                         int kb, const int (&prof)[R], const int (&T)[Codes<R, SK>::NT],
                                         int (&F)[R], int (&best)[R], int &upPrev, int &Q,
                                         uint32_t (&acc)[3][Cfg<R>::NW])
{
    sfor<QE - QB>([&](auto Qc) {
        constexpr int q = QB + decltype(Qc)::value;
        const int s = s0 + q;
        int Qn;
        if constexpr (HN) Qn = dpp_shl1(F[R - 1], Q);                         // lane 63 <- bottom row
        else Qn = __builtin_amdgcn_mov_dpp(Q, 0x130, 0xf, 0xf, true);         // wave_shl:1
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
            if constexpr (R > 1)
            {
                acc[0][w] = push_sign(acc[0][w], M - D);      // DIAG
                acc[1][w] = push_sign(acc[1][w], left - up);  // raw "up > left" (global) / raw TOP (local)
            }
            else
            {
                // R = 1: interleaved word, DIAG then raw "up > left" (local: raw TOP) per slot (sa_layout.h);
                // local STOP (H == 0) is not stored: the row walk recomputes H along the path
                acc[0][0] = push_sign(push_sign(acc[0][0], M - D), left - up);
            }
            int Fn;
            if constexpr (!LOCAL)
            {
                Fn = max(D, M);
            }
            else
            {
                // H = max(X, g) - g: max(X - g, 0) for g > 0, and X - g for g <= 0 (X >= 0)
                const int X = max(max(D, M), g);
                Fn = X - g;
                if constexpr (R > 1) acc[2][w] = push_sign(acc[2][w], Fn - 1);  // STOP (H == 0)
                const int key = (Fn << kb) + Ks;
                if constexpr (RAMP) best[rho] = act ? max(best[rho], key) : best[rho];
                else best[rho] = max(best[rho], key);
            }
            if constexpr (RAMP) Fn = act ? Fn : left;
            diag = left;
            up = Fn;
            F[rho] = Fn;
        });
    });
}

// Stores one finished chunk: lane k's LW dwords at chunk*64*LW + k*LW (one coalesced wave store).
template <int R, bool LOCAL>
__device__ __forceinline__ void store_chunk(uint32_t *dst, const uint32_t (&acc)[3][Cfg<R>::NW])
{
    constexpr int NW = Cfg<R>::NW;
    if constexpr (R == 1)
    {
        // interleaved words: slots 0..15 (the chunk's first body), slots 16..31
        *reinterpret_cast<u32x2 *>(dst) = u32x2{acc[1][0], acc[0][0]};
        return;
    }
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

// Register state of the hand-scheduled steady steps (R = 1, kArr8; sa_fill_steps.inc, generated by
// tools/gen_fill_asm.py): Q, Qn, diag and F rotate through the roles with period 4, so after a body
// of U = 16 steps every value is back in its field (F2 is a spare).
struct StepRegs {
    int Q, Qn, diag, F;
    int X[8], Y[8];        // the plane word's direction differences, one byte per step (DIAG, TOP)
    int mk[8];             // mk[s] = 0x80808080 >> s (merge_asm)
    uint32_t acc0, acc1;   // the chunk's two interleaved words (merge_asm)
    int bm;      // local: running max of (H << kb) - q over the body
    int T[4];    // text-profile words of the body (4 steps each)
    int g, kb;
    int pfaddr, pf;  // HP: LDS address of this lane's next feed slot, and the value read there
    int pubaddr, pubtag;  // HN: this lane's publish address and the body's raw lap tag (ring_tag_raw)
    int ctag;             // HP: raw lap tag the feed entries must carry
    int msb;              // 0x80000000 in a VGPR (the bitop3 operand that applies raw tags)
    uint64_t bad;         // HP: lanes 0..U-1 whose feed entry did not carry it
};
template <bool LOCAL, bool HN, bool HP, int HALF>
__device__ __forceinline__ void steps_asm(StepRegs &r);
template <bool LOCAL>
__device__ __forceinline__ void merge_asm(StepRegs &r);
// Register state of the band fill's score steps (two rows per lane; sa_fill_steps.inc, generated by
// tools/gen_fill_asm.py band_block): eight registers rotate with period 8, four carry state across
// bodies
struct BandRegs {
    int Q, diag, F0, F1;  // feed queue, up of the previous step (row 0's diag), rows 0 / 1
    int TA[4], TB[4];     // text-profile words of the body for row 0 / row 1 (4 steps each)
    int g;                // local: the gap (H = X - g, saturated at 0)
    int pfaddr, pf;       // HP: as StepRegs
    int pubaddr, pubtag, ctag, msb;
    uint64_t bad;
};
template <bool LOCAL, bool HN, bool HP>
__device__ __forceinline__ void band_steps_asm(BandRegs &r);
#if defined(SA_EXPERIMENT) && defined(SA_EXP_FILL_INC)
#include SA_EXP_FILL_INC  // tools/gen_fill_asm.py variants (timing ablations)
#else
#include "sa_fill_steps.inc"
#endif

// One strip. HP / HN: the strip has a strip above (feeds from rin) / below (publishes into rout);
// compile-time, so a body boundary carries no per-body decisions. Bodies run in pairs (the text
// codes double-buffer across the two bodies of a pair) in three phases: ramp pairs (kStart, only
// kProf / kTable), steady pairs, and tail pairs (kGeneric, only where the final state is read).
template <int R, bool LOCAL, int SK, bool HP, bool HN, bool ALIGN = false>
__device__ __forceinline__ void process_strip(const FillArgs &a, const StripLds &L, lds_int *rings, int idx, int w, int lane)
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
    static_assert(!ALIGN || (R == 1 && SK == kArr8), "kArr8A is the R = 1 kArr8 layout read through copy 0");
    if constexpr (ALIGN)
        // kArr8A: copy 0 of letter a (byte kPad + x holds S[a][t[x]]); the body's 16 bytes start at
        // x = s0 - k, i.e. byte ash = (kPad - k) & 3 of the dword at x4 = s0 + ((kPad - k) & ~3). The
        // loads fetch the four dwords after x4 and the body takes x4's dword from the body before
        coff = (uint32_t)((uint64_t)prof[0] * 4 * pd.code_len + ((kPad - lane) & ~3) + 4);
    else if constexpr (SK == kArr8)
        // byte copy r = k % 4 of letter a: byte kPad + x holds S[a][t[x - r]]; read from x = s0 - (k & ~3)
        coff = (uint32_t)(((uint64_t)prof[0] * 4 + (lane & 3)) * pd.code_len + kPad - (lane & ~3));
    else if constexpr (SK == kArr)
        coff = (uint32_t)(((uint64_t)prof[0] * pd.code_len + kPad - lane) * 4);
    else
        coff = (uint32_t)((kPad - lane) * 4);
    lds_int *rin = (lds_int *)(rings + w * kRing);
    lds_int *rout = (lds_int *)(rings + (w + 1) * kRing);
    lds_int *consIn = (lds_int *)&L.cons[w];
    lds_int *consOut = (lds_int *)&L.cons[w + 1];
    // publish target of this lane at ring offset 0: lanes 64-U..63 their column's slot, the others
    // the sink (rings + (W+1) * kRing, shared by the waves: its contents are never read)
    lds_int *pubBase = lane >= kWave - U ? rout + (lane - (kWave - U)) : rings + (L.nwaves + 1) * kRing + lane;
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
    // global score H(m, n) in the strip holding row m, and the local best-cell keys when a garbage
    // key past column n could shadow a real one of the same key block. Other strips run their tail
    // unmasked. Local strips with text profiles and g > 0 need no masked tail: past column n the
    // profile holds zeros (S + g = 0), so a cell there has H <= max(its neighbours' H) - g, every
    // key past n is below the pair's best H, and the fold discards it by column. (The masked tail
    // mattered: strip k+1 ends only after strip k's tail, so slow tails set the chain's end cadence
    // and stretched every strip behind them, 3.34 -> DESIGN.md §3.1.)
    const bool needFinal = LOCAL ? !(kIsArr<SK> && g > 0) : (m - sd.row0 >= 0 && m - sd.row0 < kWave * R);

    // column-0 boundary: global F(i,0) = 0; local H(i,0) = 0
    int F[R], best[R];
    sfor<R>([&](auto Rc) {
        constexpr int rho = decltype(Rc)::value;
        F[rho] = 0;
        best[rho] = 0;
    });
    int upPrev = 0, Q = 0;
    // text codes, double-buffered across the two bodies of a pair (no register copies)
    // text codes: R = 1 keeps four buffers and loads every body's codes two bodies ahead (bodies run
    // in quads; with one body of look-ahead a lone strip took 54.6 clk/step instead of 42: the first
    // touch of a code line misses L2); taller strips double-buffer across the two bodies of a pair
    constexpr int kAhead = R != 1 ? 1 : kCodeAhead;
    int TA[NT], TB[NT], TC[NT], TD[NT];
    // R = 1: the text codes and the direction chunks go through buffer resources (SGPR base, the
    // lane's constant 32-bit offset in a VGPR, the step-dependent part in an SGPR soffset), so a body's
    // load and a chunk's store need no VALU address arithmetic and no 64-bit adds
    constexpr bool kBuf = R == 1;
    const __amdgpu_buffer_rsrc_t crsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(cbase), 0, 0x7fffffff, kBufRsrcWord3);
    // kArr8A: the byte shift of the lane's window and the dword before the next body's four
    const uint32_t ash = (uint32_t)((kPad - lane) & 3);
    int wprev = 0;
    if constexpr (ALIGN) wprev = __builtin_amdgcn_raw_buffer_load_b32(crsrc, coff - 4, 0, 0);
    const __amdgpu_buffer_rsrc_t mrsrc = __builtin_amdgcn_make_buffer_rsrc(mbase, 0, 0x7ffffff0, kBufRsrcWord3);
    auto load_codes = [&](int s0, int (&dst)[NT]) __attribute__((always_inline)) {
        typedef int i32x4u __attribute__((ext_vector_type(4), aligned(4)));
#if defined(SA_EXPERIMENT) && defined(SA_EXP_CODES_CONST)
        const uint32_t off = coff + (uint32_t)(s0 & 63);  // timing ablation: results are wrong
#else
        const uint32_t off = coff + (uint32_t)(SK == kArr8 ? s0 : s0 * 4);
#endif
        if constexpr (kBuf)
        {
            const int soff = SK == kArr8 ? s0 : s0 * 4;
            sfor<NT / 4>([&](auto Qc) {
                constexpr int q = decltype(Qc)::value * 4;
                const i32x4u v = __builtin_amdgcn_raw_buffer_load_b128(crsrc, coff, soff + q * 4, 0);
                dst[q] = v.x;
                dst[q + 1] = v.y;
                dst[q + 2] = v.z;
                dst[q + 3] = v.w;
            });
            (void)off;
            return;
        }
        sfor<NT / 4>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value * 4;
            const i32x4u v = *(const i32x4u *)(cbase + off + q * 4);
            dst[q] = v.x;
            dst[q + 1] = v.y;
            dst[q + 2] = v.z;
            dst[q + 3] = v.w;
        });
    };
    int consKnown = 0;   // columns the consumer of rout is known to have read
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
    uint32_t dbgFeedSlow = 0, dbgFeedSpins = 0, dbgPubSlow = 0, dbgPubSpins = 0;  // slow-path counts
    uint32_t dbgFeedSlowSteady = 0, dbgFeedSpinsSteady = 0;  // the same past column 4096
#endif
    // Feed values for the body starting at step base (columns base+1 .. base+U, lanes 0..U-1 of Q)
    // are read kPfLead steps before that body starts, in the middle of the previous body: early
    // enough to cover the LDS latency, late enough that the strip above has published them by then
    // without the chain growing a body of lag per strip (a read one body ahead costs U steps of lag).
    // The read is checked at the boundary by the entries' tags (ring_tag); a slot not yet written
    // sends the wave to the slow path, which re-reads until every needed lane is there.
    int pfVal = 0;
    bool pfTagged = false;  // pfVal already XORed with its tag by the asm body, bad lanes in pfBad
    uint64_t pfBad = 0;
    // address of this lane's feed slot for the body starting at step base (column base+1+lane): the
    // body's 16 slots are one aligned run (ring_slot), so the wrap is applied to the uniform part only
    // (lanes >= U read past it, into the next ring or the sink: their values are never used)
    lds_int *rinLane = rin + lane;
    const uint32_t rinLaneOff = lds_off(rinLane);
    auto feed_addr = [&](int base) __attribute__((always_inline)) { return rinLane + ring_slot(base + 1); };
    auto prefetch = [&](int base) __attribute__((always_inline)) {
        if constexpr (HP)
        {
            int c = base + 1 + lane;
            // the read may not move above the steps before this point (the compiler would hoist it)
            asm volatile("" : "+v"(c) : "v"(F[R - 1]));
            pfVal = lds_ld(rin + ring_slot(c));
        }
    };
    // full: every lane 0..U-1 of this feed is needed and delivered (base + U <= n), so the check
    // needs no per-body lane count
    auto feed = [&](int base, bool full) __attribute__((always_inline)) {
        if constexpr (!HP)
        {
            // row 0 boundary. The zero is opaque on purpose: with a known-zero `old` the compiler
            // folds the up-DPP into its consumers with bound_ctrl:1, and on gfx950 wave_shr with
            // bound_ctrl does not hand lane 0 a zero (measured: wrong row 1 in strip 0)
            asm volatile("v_mov_b32 %0, 0" : "=v"(Q));
            return;
        }
        else
        {
            // lanes 0..cnt-1 carry columns base+1 .. base+cnt <= n; one aligned run: one tag. The asm
            // bodies have applied the tag already (pfTagged) and left the bad-lane mask in pfBad.
            const int tag = ring_tag(base + 1);
            // need = (1 << clamp(n - base, 0, U)) - 1, as four SALU ops (left to itself the compiler
            // clamps in VALU and round-trips through v_readfirstlane)
            uint64_t need = (1ull << U) - 1;
            if (!full)  // (a constant at every call: the clamp is compiled out of the full bodies)
            {
                int cnt;
                asm("s_sub_i32 %1, %2, %3\n\ts_max_i32 %1, %1, 0\n\ts_min_i32 %1, %1, %4\n\ts_bfm_b64 %0, %1, 0"
                    : "=s"(need), "=&s"(cnt)
                    : "s"(n), "s"(base), "i"(U)
                    : "scc");
            }
            int x = pfTagged ? pfVal : pfVal ^ tag;
            // (the asm bodies' mask already holds only lanes 0..U-1)
            const uint64_t bad = pfTagged ? pfBad : (ballot(x < 0) & ((1ull << U) - 1));
            pfTagged = false;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_NO_FEED_WAIT)
            if (base > 0 && false)  // timing ablation: never waits after the first feed (results wrong)
#else
            if (__builtin_expect((full ? bad : (bad & need)) != 0, 0))
#endif
            {
                // a chained strip is paced by the strip above and often arrives a little early:
                // re-read at once for a while (this wave is alone on its SIMD), sleep only when the
                // wait is long (the strip's start); the give-up clock starts after 256 polls
                uint64_t t0 = 0;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
                ++dbgFeedSlow;
                if (base >= 4096) ++dbgFeedSlowSteady;
#endif
                for (uint32_t spin = 1;; ++spin)
                {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
                    ++dbgFeedSpins;
                    if (base >= 4096) ++dbgFeedSpinsSteady;
#endif
                    if (spin > 16) __builtin_amdgcn_s_sleep(1);
                    x = ds_read_sync(feed_addr(base)) ^ tag;
                    if ((ballot(x < 0) & need) == 0) break;
                    if ((spin & 255) == 0)
                    {
                        if (t0 == 0) t0 = now_ticks();
                        else if (!keep_waiting(a, t0, lane)) break;
                    }
                }
            }
            Q = x;  // lanes >= cnt: don't care
        }
    };
    // consumption word for the strip above (its backpressure), at most every kConsEvery columns
    // (once per loop trip: every lane writes, lane 0 the word and the others into the sink, so the
    // write is one instruction instead of an exec-masked branch; asm: no LDS operation of the
    // compiler's may stay in flight into the next body)
    const uint32_t consAddr = lane == 0 ? lds_off(consIn) : lds_off(rings + (L.nwaves + 1) * kRing + lane);
    auto consumed = [&](int upto) __attribute__((always_inline)) {
        if constexpr (HP) asm volatile("ds_write_b32 %0, %1" ::"v"(consAddr), "v"(upto));
    };
    // lanes 64-U..63 of Q hold the bottom row of columns s0-63 .. s0-64+U: one ds_write_b32 by every
    // lane (the others into the sink), tagged, after making sure the consumer has read the slots'
    // previous lap
    auto pub_wait = [&](int s0) __attribute__((always_inline)) {
        if constexpr (HN)
        {
            const int cLast = s0 - 64 + U;
            if (__builtin_expect(cLast - kRing > consKnown, 0))
            {
                const uint64_t t0 = now_ticks();
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
                ++dbgPubSlow;
#endif
                for (uint32_t spin = 1;; ++spin)
                {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
                    ++dbgPubSpins;
#endif
                    consKnown = uniform(lds_ld(consOut));
                    if (cLast - kRing <= consKnown) break;
                    __builtin_amdgcn_s_sleep(1);
                    if ((spin & 255) == 0 && !keep_waiting(a, t0, lane)) break;
                }
            }
        }
    };
    auto publish = [&](int s0) __attribute__((always_inline)) {
        if constexpr (HN)
        {
            pub_wait(s0);
            lds_st(pubBase + (s0 & kRingMask), Q | ring_tag(s0 - 63));
        }
    };
    int msbv;  // one VGPR for the strip (the compiler would rematerialize a literal per body)
    asm volatile("v_mov_b32 %0, 0x80000000" : "=v"(msbv));
    // the asm bodies' direction-difference bytes (kept across the two bodies of a plane word) and the
    // merge masks 0x80808080 >> g (opaque: built once per strip, not rematerialized per word)
    int dX[8], dY[8], mkv[8];
    sfor<8>([&](auto Gc) {
        constexpr int g = decltype(Gc)::value;
        dX[g] = dY[g] = 0;
        int m;
        asm volatile("v_mov_b32 %0, %1" : "=v"(m) : "i"((int)(0x80808080u >> g)));
        mkv[g] = m;
    });
    const uint64_t tStart = a.timeline ? now_ticks() : 0;
    // the compiler's vector-memory wait before each steady body is the most conservative over the
    // paths into the loop: the first trip must see the steady trips' order (TA's loads, TB's, then one
    // op standing in for the chunk store that precedes every later trip), or it waits one op further
    // back on every first body of a quad (a load or store issued a body ago); measured in the asm:
    // vmcnt(2) -> vmcnt(3) on all steady bodies
    load_codes(0, TA);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kAhead == 2) load_codes(U, TB);
    __builtin_amdgcn_sched_barrier(0);
    int vmPad = 0;
    if constexpr (kBuf && kAhead == 2) vmPad = __builtin_amdgcn_raw_buffer_load_b32(crsrc, coff, 0, 0);
    prefetch(0);
    feed(0, false);
    const uint64_t tFed = a.timeline ? now_ticks() : 0;
    const uint64_t cFed = a.timeline ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t lbest = 0;
    constexpr int kPfLead = U >= 8 ? SA_PF_LEAD * U / 16 : 1;  // steps between the feed read and its use
    // steady R = 1 bodies with int8 text profiles run hand-scheduled asm steps (sa_fill_steps.inc)
    constexpr bool kAsm = R == 1 && SK == kArr8 && SA_FILL_ASM;
    // pos: the body's place in its loop trip (0..3 in quads, 0..1 in pairs): odd bodies store the
    // direction chunk (two bodies per chunk for R = 1), the trip's last one writes the consumption word.
    // full: the next body's feed is known to be fully published (feed()) and s1 < nSteps.
    // the loop trip's feed-slot byte offset 4 (s0q + U + 64) (the trip's bodies add 4 U POS and wrap),
    // opaque so the compiler computes it once per trip instead of per body from the step
    uint32_t quadPf = 0;
    auto set_quad = [&](int s0q) __attribute__((always_inline)) {
        quadPf = 4u * (uint32_t)s0q + 4u * (U + 64);
        asm volatile("" : "+s"(quadPf));
    };
    auto body = [&](auto kind, auto pos, auto full, int s0, int (&T)[NT], int (&Tn)[NT]) __attribute__((always_inline)) {
        constexpr int KIND = decltype(kind)::value;
        constexpr int POS = decltype(pos)::value;
        constexpr bool FULL = decltype(full)::value;
        using second = std::integral_constant<bool, (POS & 1) == 1>;
        const int s1 = s0 + U;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
        // progress stamps every 4096 columns (timeline words 6..15)
        if (a.timeline && (s0 & 4095) == 0 && (s0 >> 12) < 10 && lane == 0)
        {
            a.timeline[kTimelineWords * (size_t)idx + 6 + (s0 >> 12)] = now_ticks();
            a.timeline[kTimelineWords * (size_t)idx + 26 + (s0 >> 12)] = __builtin_amdgcn_s_memtime();
        }
#endif
        load_codes(s0 + kAhead * U, Tn);
        if constexpr (ALIGN)
        {
            // the body's 16 score bytes into place (in the buffer itself: its raw words are not read
            // again), the last raw dword kept for the next body
            const int w4 = T[3];
            T[3] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[3], (uint32_t)T[2], ash);
            T[2] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[2], (uint32_t)T[1], ash);
            T[1] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[1], (uint32_t)T[0], ash);
            T[0] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[0], (uint32_t)wprev, ash);
            wprev = w4;
        }
        if constexpr (kAsm && KIND == kSteady)
        {
            static_assert(U == 16 && NT == 4, "sa_fill_steps.inc is generated for these");
            StepRegs r;
            r.Q = Q;
            r.diag = upPrev;
            r.F = F[0];
            sfor<8>([&](auto Gc) {
                constexpr int g = decltype(Gc)::value;
                r.X[g] = dX[g];
                r.Y[g] = dY[g];
            });
            r.bm = -16;  // below every (H << kb) - q
            sfor<4>([&](auto Wc) { r.T[decltype(Wc)::value] = T[decltype(Wc)::value]; });
            r.g = g;
            r.kb = kb;
            // 4 * ring_slot(s1 + 1) = (4 s0 + 4 (U + 64)) mod 8 KiB, from the loop trip's base (quadPf)
            r.pfaddr = HP ? (int)(rinLaneOff + ((quadPf + 4u * U * POS) & (4u * kRingMask))) : 0;
            r.ctag = ring_tag_raw(s1 + 1);
            r.msb = msbv;
            // the block ends with the publish write (HN); one backpressure check covers the bodies up
            // to the trip's last (a quad from pos 0, a pair from pos 2)
            if constexpr (POS == 0) pub_wait(s0 + 3 * U);
            else if constexpr (POS == 2) pub_wait(s0 + U);
            r.pubaddr = (int)lds_off(pubBase + (s0 & kRingMask));
            r.pubtag = ring_tag_raw(s0 - 63);
            steps_asm<LOCAL, HN, HP, POS & 1>(r);  // with HP: reads the next body's feed after step 12
            if constexpr (HP)
            {
                pfVal = r.pf;
                pfBad = r.bad;
                pfTagged = true;
            }
            Q = r.Q;
            upPrev = r.diag;
            F[0] = r.F;
            sfor<8>([&](auto Gc) {
                constexpr int g = decltype(Gc)::value;
                dX[g] = r.X[g];
                dY[g] = r.Y[g];
            });
            if constexpr ((POS & 1) == 1)
            {
                // the chunk's second body: its bits into the two interleaved words for the store below
                sfor<8>([&](auto Gc) { r.mk[decltype(Gc)::value] = mkv[decltype(Gc)::value]; });
#if defined(SA_EXPERIMENT) && defined(SA_EXP_NO_MERGE)
                // timing ablation: the chunk's words are two raw difference registers (results wrong)
                acc[1][0] = (uint32_t)r.X[0] ^ (uint32_t)r.X[5];
                acc[0][0] = (uint32_t)r.Y[0] ^ (uint32_t)r.Y[5];
#else
                merge_asm<LOCAL>(r);
                acc[1][0] = r.acc0;
                acc[0][0] = r.acc1;
#endif
            }
            if constexpr (LOCAL)
            {
                const int kmask = (1 << kb) - 1;
                best[0] = max(best[0], r.bm + (kmask - (s0 & kmask)));
            }
        }
        else
        {
            run_body<R, LOCAL, SK, KIND, HN, 0, U - kPfLead>(L.S, s0, lane, n, g, kb, prof, T, F, best, upPrev, Q, acc);
            prefetch(s1);
            run_body<R, LOCAL, SK, KIND, HN, U - kPfLead, U>(L.S, s0, lane, n, g, kb, prof, T, F, best, upPrev, Q, acc);
            // R = 1: a body fills one interleaved word; the chunk's first word waits in acc[1][0]
            if constexpr (R == 1 && !second::value) acc[1][0] = acc[0][0];
        }
#if defined(SA_EXPERIMENT) && defined(SA_EXP_NO_STORE)
        if constexpr (false)  // timing ablation: no direction planes are written
#else
        if constexpr (Cfg<R>::BPC == 1 || second::value)
#endif
        {
            const int chunk = (int)((uint32_t)(s1 * R) / Cfg<R>::CS) - 1;
            if constexpr (kBuf)
                // R = 1: the chunk's two interleaved words (store_chunk), soffset = the chunk's byte offset
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{acc[1][0], acc[0][0]}, mrsrc, moff, chunk * (kWave * Cfg<R>::LW * 4), 0);
            else
                store_chunk<R, LOCAL>(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(mbase + (size_t)chunk * (kWave * Cfg<R>::LW)) + moff), acc);
        }
        if constexpr (LOCAL)
        {
            const int kmask = (1 << kb) - 1;
            if (((s1 & kmask) == 0) || (!FULL && s1 >= nSteps))
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
        if constexpr (!(kAsm && KIND == kSteady)) publish(s0);
        feed(s1, FULL);
        if constexpr (POS == (kAhead == 2 ? 3 : 1)) consumed(s1 + U);
    };
    using KSteady = std::integral_constant<int, kSteady>;
    using KStart = std::integral_constant<int, kStart>;
    using KGeneric = std::integral_constant<int, kGeneric>;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    // tail pairs: from the first pair holding a body with s1 > n (only where the final state is read)
    const int sTail = needFinal ? max(0, (n - 2 * U + 1 + 2 * U - 1) / (2 * U) * (2 * U)) : nSteps;
    int s0 = 0;
    if constexpr (kAhead == 2)
    {
        // bodies in quads up to `end` (a multiple of 2U), then at most one pair, after which the codes
        // loaded into TC / TD move back to TA / TB (once per phase)
        auto phase = [&](auto kind, auto full, int end) __attribute__((always_inline)) {
            for (; s0 + 2 * U < end; s0 += 4 * U)
            {
                set_quad(s0);
                body(kind, P0{}, full, s0, TA, TC);
                body(kind, P1{}, full, s0 + U, TB, TD);
                body(kind, P2{}, full, s0 + 2 * U, TC, TA);
                body(kind, P3{}, full, s0 + 3 * U, TD, TB);
            }
            if (s0 < end)
            {
                set_quad(s0 - 2 * U);
                body(kind, P2{}, full, s0, TA, TC);
                body(kind, P3{}, full, s0 + U, TB, TD);
                s0 += 2 * U;
                sfor<NT>([&](auto Qc) {
                    constexpr int q = decltype(Qc)::value;
                    TA[q] = TC[q];
                    TB[q] = TD[q];
                });
            }
        };
        // steady bodies whose next feed lies in columns 1..n (base + U <= n: every lane is needed and
        // delivered, by a neighbour wave or by the I/O wave, which copies columns 1..n), then the rest
        // of the steady bodies with a lane count
        if (LOCAL && g < 0) phase(KGeneric{}, std::false_type{}, min(kWave, sTail));
        else if constexpr (!kIsArr<SK>) phase(KStart{}, std::false_type{}, min(kWave, sTail));
        phase(KSteady{}, std::true_type{}, min(sTail, max(0, (n - U) / (2 * U) * (2 * U))));
        phase(KSteady{}, std::false_type{}, sTail);
        phase(KGeneric{}, std::false_type{}, nSteps);
        asm volatile("" ::"v"(vmPad));
    }
    else
    {
        if (LOCAL && g < 0)
            for (; s0 < min(kWave, sTail); s0 += 2 * U)
            {
                body(KGeneric{}, P0{}, std::false_type{}, s0, TA, TB);
                body(KGeneric{}, P1{}, std::false_type{}, s0 + U, TB, TA);
            }
        else if constexpr (!kIsArr<SK>)
            for (; s0 < min(kWave, sTail); s0 += 2 * U)
            {
                body(KStart{}, P0{}, std::false_type{}, s0, TA, TB);
                body(KStart{}, P1{}, std::false_type{}, s0 + U, TB, TA);
            }
        for (; s0 < sTail; s0 += 2 * U)
        {
            body(KSteady{}, P0{}, std::false_type{}, s0, TA, TB);
            body(KSteady{}, P1{}, std::false_type{}, s0 + U, TB, TA);
        }
        for (; s0 < nSteps; s0 += 2 * U)
        {
            body(KGeneric{}, P0{}, std::false_type{}, s0, TA, TB);
            body(KGeneric{}, P1{}, std::false_type{}, s0 + U, TB, TA);
        }
    }
    if (a.timeline && lane == 0)
    {
        uint64_t *tl = a.timeline + kTimelineWords * (size_t)idx;
        tl[0] = tStart;
        tl[1] = tFed;
        tl[2] = now_ticks();
        tl[4] = cFed;  // shader clock (s_memtime): effective frequency = clocks / real time
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
        tl[36] = dbgFeedSlow;
        tl[37] = dbgFeedSpins;
        tl[38] = dbgPubSlow;
        tl[39] = dbgPubSpins;
        tl[40] = dbgFeedSlowSteady;
        tl[41] = dbgFeedSpinsSteady;
#endif
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
// BAND fill (R = 1 int8 text-profile chains): score strips of two rows per lane
// ------------------------------------------------------------------------------------------------
// A chain of 64-row strips hands its bottom row down once per 64 rows, and every hand-off costs the
// 64-step lane skew plus the hand-off latency: at 32768^2 that ramp (511 hand-offs) was two thirds of
// the fill. A BAND is a 128-row score strip: lane k owns rows row0 + 2k and row0 + 2k + 1 and works on
// column s - k + 1 at step s for both, so a band covers twice the rows per lane skew, and the chain of
// bands has half the hand-offs. Its recurrence runs alone (band_steps_asm: 6 VALU per step, 8 local,
// no direction bits, no best-cell keys); its bottom row, published with the same step <-> column map,
// ring tags and granules as a 64-row strip, feeds the next band and, through the granules (drain and
// I/O waves), the 64-row strips of the band below. Those strips (process_strip, the one-wave kernel)
// run in groups of W on the other workgroups: the group's first strip is fed from the band above's
// granules, the rest through the group's LDS rings, and they write the direction planes, the global
// score and the local best cells exactly as the one-wave fill does (the same integer operations on
// the same inputs). Bands exist for every band of a pair but its last (whose bottom row feeds
// nothing) and need no final state; the local recurrence saturates H = X - g at 0 with one clamped
// subtract (g >= 0, X >= 0), so local is banded as well.
template <bool LOCAL, bool HP, bool HN, bool TOUCH, bool ALIGN = false>
__device__ __forceinline__ void process_band(const FillArgs &a, const StripLds &L, lds_int *rings, int idx, int w, int lane)
{
    constexpr int U = 16;
    typedef int i32x4u __attribute__((ext_vector_type(4), aligned(4)));
    idx = uniform(idx);
    StripDesc sd = a.bands[idx];
    sd.pair = uniform(sd.pair);
    sd.row0 = uniform(sd.row0);
    sd.nsteps = uniform(sd.nsteps);
    PairDesc pd = a.pairs[sd.pair];
    pd.text_len = uniform64(pd.text_len);
    pd.pattern_len = uniform64(pd.pattern_len);
    pd.pattern_off = uniform64(pd.pattern_off);
    pd.code_off = uniform64(pd.code_off);
    pd.code_len = uniform64(pd.code_len);
    const int n = (int)pd.text_len, m = (int)pd.pattern_len;
    // the lane's two rows: byte copy k % 4 of each row letter's text profile (process_strip, kArr8)
    uint32_t coff[2];
    sfor<2>([&](auto Rc) {
        constexpr int rho = decltype(Rc)::value;
        const int i = sd.row0 + 2 * lane + rho;
        int c = i <= m ? (int)a.pattern[pd.pattern_off + i - 1] : 0;
        c = min(max(c, 0), a.A - 1);
        if constexpr (ALIGN)
            // kArr8A: copy 0, dword aligned, shifted in registers (process_strip)
            coff[rho] = (uint32_t)((uint64_t)c * 4 * pd.code_len + ((kPad - lane) & ~3) + 4);
        else
            coff[rho] = (uint32_t)(((uint64_t)c * 4 + (lane & 3)) * pd.code_len + kPad - (lane & ~3));
    });
    const __amdgpu_buffer_rsrc_t crsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t *>(a.codes + pd.code_off), 0, 0x7fffffff, kBufRsrcWord3);
    auto load_codes = [&](int s0, int (&dA)[4], int (&dB)[4]) __attribute__((always_inline)) {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_CODES_CONST)
        s0 &= 63;  // timing ablation: cache-resident text codes (results wrong)
#endif
#if defined(SA_EXPERIMENT) && defined(SA_EXP_CODES_POLICY)
        constexpr int kCodePolicy = SA_EXP_CODES_POLICY;  // experiment: cache policy bits of the loads
#else
        constexpr int kCodePolicy = 0;
#endif
        const i32x4u va = __builtin_amdgcn_raw_buffer_load_b128(crsrc, coff[0], s0, kCodePolicy);
        const i32x4u vb = __builtin_amdgcn_raw_buffer_load_b128(crsrc, coff[1], s0, kCodePolicy);
        dA[0] = va.x;
        dA[1] = va.y;
        dA[2] = va.z;
        dA[3] = va.w;
        dB[0] = vb.x;
        dB[1] = vb.y;
        dB[2] = vb.z;
        dB[3] = vb.w;
    };
    lds_int *rin = (lds_int *)(rings + w * kRing);
    lds_int *rout = (lds_int *)(rings + (w + 1) * kRing);
    lds_int *consIn = (lds_int *)&L.cons[w];
    lds_int *consOut = (lds_int *)&L.cons[w + 1];
    lds_int *drainOut = (lds_int *)&L.drain[w + 1];
    lds_int *sink = rings + (L.nwaves + 1) * kRing;
    lds_int *pubBase = lane >= kWave - U ? rout + (lane - (kWave - U)) : sink + lane;
    const uint32_t rinLaneOff = lds_off(rin + lane);
    // the feed protocol of process_strip: read after step BAND_PF_STEP, tags checked at the body end
    int Q = 0, diag = 0, F0 = 0, F1 = 0;  // column-0 boundary
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_MISS)
    // experiment: feed slow-path entries (bodies 0..63 as a mask, all bodies as a count) and polls
    uint64_t missMask = 0;
    uint32_t missCount = 0, spinCount = 0, spin0 = 0;
#endif
    int pfVal = 0;
    bool pfTagged = false;
    uint64_t pfBad = 0;
    auto feed = [&](int base, bool full) __attribute__((always_inline)) {
        if constexpr (!HP)
        {
            asm volatile("v_mov_b32 %0, 0" : "=v"(Q));  // row 0 boundary (opaque: see process_strip)
            return;
        }
        else
        {
            const int tag = ring_tag(base + 1);
            uint64_t need = (1ull << U) - 1;
            if (!full)
            {
                int cnt;
                asm("s_sub_i32 %1, %2, %3\n\ts_max_i32 %1, %1, 0\n\ts_min_i32 %1, %1, %4\n\ts_bfm_b64 %0, %1, 0"
                    : "=s"(need), "=&s"(cnt)
                    : "s"(n), "s"(base), "i"(U)
                    : "scc");
            }
            int x = pfTagged ? pfVal : pfVal ^ tag;
            const uint64_t bad = pfTagged ? pfBad : (ballot(x < 0) & ((1ull << U) - 1));
            pfTagged = false;
            if (__builtin_expect((full ? bad : (bad & need)) != 0, 0))
            {
                uint64_t t0 = 0;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_MISS)
                if (base > 0)
                {
                    ++missCount;
                    if (base / U - 1 < 64) missMask |= 1ull << (base / U - 1);
                }
#endif
                for (uint32_t spin = 1;; ++spin)
                {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_MISS)
                    if (base > 0) ++spinCount;
                    else ++spin0;
#endif
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_WAIT_SLEEP)
                    if (spin > 16) { for (int z = 0; z < SA_EXP_BAND_WAIT_SLEEP; ++z) __builtin_amdgcn_s_sleep(1); }
#else
                    if (spin > 16) __builtin_amdgcn_s_sleep(1);
#endif
                    x = ds_read_sync(rin + lane + ring_slot(base + 1)) ^ tag;
                    if ((ballot(x < 0) & need) == 0) break;
                    if ((spin & 255) == 0)
                    {
                        if (t0 == 0) t0 = now_ticks();
                        else if (!keep_waiting(a, t0, lane)) break;
                    }
                }
            }
            Q = x;
        }
    };
    const uint32_t consAddr = lane == 0 ? lds_off(consIn) : lds_off(sink + lane);
    auto consumed = [&](int upto) __attribute__((always_inline)) {
        if constexpr (HP) asm volatile("ds_write_b32 %0, %1" ::"v"(consAddr), "v"(upto));
    };
    // a ring slot is reused once the drain or I/O wave (drain) and the next band (cons) have read it;
    // a next band of the group that starts another pair's chain reads nothing (the I/O wave, which
    // drains the group's last ring, keeps cons too)
    const bool nextReads = !(w + 1 < L.nwaves && idx + 1 < a.num_bands) || (uniform(a.bands[idx + 1].flags) & kHasPrev);
    int consKnown = 0;
    auto pub_wait = [&](int s0) __attribute__((always_inline)) {
        if constexpr (HN)
        {
            const int cLast = s0 - 64 + U;
            if (__builtin_expect(cLast - kRing > consKnown, 0))
            {
                const uint64_t t0 = now_ticks();
                for (uint32_t spin = 1;; ++spin)
                {
                    consKnown = uniform(lds_ld(drainOut));
                    if (nextReads) consKnown = min(consKnown, uniform(lds_ld(consOut)));
                    if (cLast - kRing <= consKnown) break;
                    __builtin_amdgcn_s_sleep(1);
                    if ((spin & 255) == 0 && !keep_waiting(a, t0, lane)) break;
                }
            }
        }
    };
    int msbv;
    asm volatile("v_mov_b32 %0, 0x80000000" : "=v"(msbv));
    const uint64_t tStart = a.timeline ? now_ticks() : 0;
    int TA0[4], TA1[4], TB0[4], TB1[4], TC0[4], TC1[4], TD0[4], TD1[4];
    const uint32_t ash = (uint32_t)((kPad - lane) & 3);
    int wprev0 = 0, wprev1 = 0;  // kArr8A: the dword before the next body's four, per row
    if constexpr (ALIGN)
    {
        wprev0 = __builtin_amdgcn_raw_buffer_load_b32(crsrc, coff[0] - 4, 0, 0);
        wprev1 = __builtin_amdgcn_raw_buffer_load_b32(crsrc, coff[1] - 4, 0, 0);
    }
    load_codes(0, TA0, TA1);
    // TA's two loads before TB's, as in the steady quads: otherwise the loop's first body waits for
    // one of the previous body's loads in every quad (vmcnt(3) instead of (4))
    __builtin_amdgcn_sched_barrier(0);
    load_codes(U, TB0, TB1);
    if constexpr (HP)
    {
        int c = 1 + lane;
        asm volatile("" : "+v"(c));
        pfVal = lds_ld(rin + ring_slot(c));
    }
    feed(0, false);
    const uint64_t tFed = a.timeline ? now_ticks() : 0;
    const uint64_t cFed = a.timeline ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t quadPf = 0;
    auto set_quad = [&](int s0q) __attribute__((always_inline)) {
        quadPf = 4u * (uint32_t)s0q + 4u * (U + 64);
        asm volatile("" : "+s"(quadPf));
    };
    auto body = [&](auto pos, auto full, int s0, int (&T0)[4], int (&T1)[4], int (&Tn0)[4], int (&Tn1)[4]) __attribute__((always_inline)) {
        constexpr int POS = decltype(pos)::value;
        constexpr bool FULL = decltype(full)::value;
        const int s1 = s0 + U;
        load_codes(s0 + 2 * U, Tn0, Tn1);
        if constexpr (ALIGN)
        {
            auto shift = [&](int(&T)[4], int &wp) __attribute__((always_inline)) {
                const int w4 = T[3];
                T[3] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[3], (uint32_t)T[2], ash);
                T[2] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[2], (uint32_t)T[1], ash);
                T[1] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[1], (uint32_t)T[0], ash);
                T[0] = (int)__builtin_amdgcn_alignbyte((uint32_t)T[0], (uint32_t)wp, ash);
                wp = w4;
            };
            shift(T0, wprev0);
            shift(T1, wprev1);
        }
        BandRegs r;
        r.Q = Q;
        r.diag = diag;
        r.F0 = F0;
        r.F1 = F1;
        sfor<4>([&](auto Wc) {
            constexpr int q = decltype(Wc)::value;
            r.TA[q] = T0[q];
            r.TB[q] = T1[q];
        });
        r.g = a.gap;
        r.pfaddr = HP ? (int)(rinLaneOff + ((quadPf + 4u * U * POS) & (4u * kRingMask))) : 0;
        r.ctag = ring_tag_raw(s1 + 1);
        r.msb = msbv;
        if constexpr (POS == 0) pub_wait(s0 + 3 * U);
        else if constexpr (POS == 2) pub_wait(s0 + U);
        r.pubaddr = (int)lds_off(pubBase + (s0 & kRingMask));
        r.pubtag = ring_tag_raw(s0 - 63);
        band_steps_asm<LOCAL, HN, HP>(r);
        if constexpr (HP)
        {
            pfVal = r.pf;
            pfBad = r.bad;
            pfTagged = true;
        }
        Q = r.Q;
        diag = r.diag;
        F0 = r.F0;
        F1 = r.F1;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_STAMPS)
        // timing: when the band finished bodies 0..15 (words 6..21; the body at 64 publishes the first
        // feed of the band below) and when the next body's feed was in hand (words 22..37)
        if (a.timeline && s0 < 16 * U && lane == 0)
            a.timeline[kTimelineWords * ((size_t)a.num_strips + idx) + 6 + s0 / U] = now_ticks();
        feed(s1, FULL);
        if (a.timeline && s0 < 16 * U && lane == 0)
            a.timeline[kTimelineWords * ((size_t)a.num_strips + idx) + 22 + s0 / U] = now_ticks();
#else
        feed(s1, FULL);
#endif
        if constexpr (POS == 3) consumed(s1 + U);
    };
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    const int nSteps = sd.nsteps;  // a multiple of 2U
    int s0 = 0;
    // L1 touch distance of the text codes (bodies): 32768² global fill -2.5 %, local +4 % at 6 (4 and
    // 8 are slower; same-box A/Bs, profiles/r04/band_touch_v1.log, band_touch_v2.log), so global only,
    // and DNA-sized alphabets only (protein 4096² pays about 4 %): a kernel of its own (TOUCH), since a
    // second copy of the loops inside one kernel lost the gain (profiles/r04/band_touch_v3.log)
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_TOUCH)
    constexpr int kTouch = SA_EXP_BAND_TOUCH;
#else
    constexpr int kTouch = TOUCH && !LOCAL ? 6 : 0;
#endif
    int touchA = 0, touchB = 0;
    // quads of bodies up to `end` (a multiple of 2U), then at most one pair (process_strip's phases)
    auto phase = [&](auto full, auto touch, int end) __attribute__((always_inline)) {
        for (; s0 + 2 * U < end; s0 += 4 * U)
        {
            if constexpr (decltype(touch)::value)
            {
                // one dword per lane of both rows kTouch bodies ahead, so the code loads of that body
                // find their lines in the CU's L1; consumed a quad later, so that no compiler wait
                // stands on it (clamped to the furthest offset the code loads themselves reach)
                asm volatile("" ::"v"(touchA), "v"(touchB));
                touchA = __builtin_amdgcn_raw_buffer_load_b32(crsrc, coff[0], min(s0 + kTouch * U, nSteps + U), 0);
                touchB = __builtin_amdgcn_raw_buffer_load_b32(crsrc, coff[1], min(s0 + kTouch * U, nSteps + U), 0);
            }
            set_quad(s0);
            body(P0{}, full, s0, TA0, TA1, TC0, TC1);
            body(P1{}, full, s0 + U, TB0, TB1, TD0, TD1);
            body(P2{}, full, s0 + 2 * U, TC0, TC1, TA0, TA1);
            body(P3{}, full, s0 + 3 * U, TD0, TD1, TB0, TB1);
        }
        if (s0 < end)
        {
            set_quad(s0 - 2 * U);
            body(P2{}, full, s0, TA0, TA1, TC0, TC1);
            body(P3{}, full, s0 + U, TB0, TB1, TD0, TD1);
            s0 += 2 * U;
            sfor<4>([&](auto Qc) {
                constexpr int q = decltype(Qc)::value;
                TA0[q] = TC0[q];
                TA1[q] = TC1[q];
                TB0[q] = TD0[q];
                TB1[q] = TD1[q];
            });
        }
    };
    // bodies whose next feed lies in columns 1..n (every feed lane needed and delivered), then the rest
    phase(std::true_type{}, std::integral_constant<bool, (kTouch > 0)>{}, min(nSteps, max(0, (n - U) / (2 * U) * (2 * U))));
    phase(std::false_type{}, std::integral_constant<bool, (kTouch > 0)>{}, nSteps);
    if (a.timeline && lane == 0)
    {
        // band records follow the strips' (kTimelineWords words each)
        uint64_t *tl = a.timeline + kTimelineWords * ((size_t)a.num_strips + idx);
        tl[0] = tStart;
        tl[1] = tFed;
        tl[2] = now_ticks();
        tl[4] = cFed;
        tl[5] = __builtin_amdgcn_s_memtime();
        tl[3] = ((uint64_t)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32) |
                (uint32_t)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_MISS)
        tl[38] = missMask;
        tl[39] = missCount;
        tl[40] = spinCount;
        tl[41] = spin0;
#endif
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
//     (s < 8) are rows ρ and ρ+8 of the same step (R >= 16); one v_perm_b32 spreads the four sign
//     bits (both pairs, both slots) over whole bytes (sign-replicating selectors), and one
//     v_bfi_b32 keeps bits 15-s, 7-s, 31-s, 23-s of them: 2 VALU per 4 bits (was 3 with a shift).
//   * At the body's end v_perm_b32 splits the packed words back into each pair's ordinary 32-slot
//     words, so the stored planes, the traceback and the decoders are exactly those of the unpacked
//     kernel.
// About 4.5 VALU per cell instead of 8.2.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as16(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// CHAINS of pair-packed strips (pairs taller than one strip, fill_pair_chain_kernel): one workgroup
// per couple of pairs, one wave per strip of the couple (the same strip of both pairs, packed as
// above); a strip's bottom row goes to the strip below through an LDS array of the whole row (n + a
// wave's skew entries: no wrap, no laps), filled with 0xffffffff at the workgroup's start. Both
// halves of a published value are at most 65534 (plan_create's bound), so that word is never a
// value: the consumer's U feed entries are ready when none of them is 0xffffffff. No global memory
// and no other workgroup is involved, so the chain cannot deadlock whatever the residency. This sizes
// a batch's plan to the GPU when it has few pairs (a shard of the batch on one of N GPUs): strips of
// 8 or 16 rows per lane give the couple 2-4 waves instead of one.
template <int R, bool HP, bool HN>
__device__ __forceinline__ void process_pair(const FillArgs &a, int sA, int sB, int lane, lds_int *feed, lds_int *pub)
{
    // a body is one stored chunk (R = 4: 8 steps, two of the plan's 4-step bodies)
    constexpr int U = Cfg<R>::SB >= 32 ? Cfg<R>::U : 32 / R;
    constexpr int SB = U * R;           // slots per body (per pair)
    constexpr int NP = SB / 16;         // packed words per plane per body
    constexpr int NW = Cfg<R>::NW, LW = Cfg<R>::LW;
    static_assert(R >= 4 && SB == Cfg<R>::CS, "pair kernel: R >= 4, a body is one chunk");
    const StripDesc dA = a.strips[sA], dB = a.strips[sB];
    const PairDesc pA = a.pairs[dA.pair], pB = a.pairs[dB.pair];
    const int n = (int)pA.text_len, m = (int)pA.pattern_len;
    const int g = a.gap;
    const int rowTop = dA.row0 + lane * R;
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
    uint32_t P = 0;  // HN: the bottom row's queue (lane 63 enters a value per step)
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
        if constexpr (HP)
        {
            // lane q < U: the strip above's bottom row at column s0 + 1 + q (lane 0 enters column
            // s0 + 1 + q at step s0 + q); columns past n are never published and never needed
            lds_int *f = feed + (s0 + 1 + kPairFeedOff) + lane;
            const bool need = lane < U && s0 + 1 + lane <= n;
            Q = lds_ld(f);
            while (__builtin_amdgcn_ballot_w64(need && Q == -1) != 0)
            {
                __builtin_amdgcn_s_sleep(1);
                Q = lds_ld(f);
            }
        }
        else asm volatile("v_mov_b32 %0, 0" : "=v"(Q));  // row 0 boundary (opaque zero: see feed())
        uint32_t x0[U * R], x1[U * R];
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
            sfor<R>([&](auto Rc) {
                constexpr int rho = decltype(Rc)::value;
                constexpr int e = q * R + rho;  // the body's slot
                const uint32_t sc = __builtin_amdgcn_perm(colB, colA, rsel[rho]);
                const u16x2 D = as16(diag) + as16(sc);
                const uint32_t left = F[rho];
                const u16x2 M = __builtin_elementwise_max(as16(left), as16(up));
                uint32_t Fn = as32(__builtin_elementwise_max(D, M));
                x0[e] = as32(M - D);                     // DIAG iff sign
                x1[e] = as32(as16(left) - as16(up));     // up > left iff sign
                if constexpr (RAMP) Fn = act ? Fn : left;
                diag = left;
                up = Fn;
                F[rho] = Fn;
                // slots e - 8 and e of a 16-slot group (rows rho - 8 and rho of this step for R >= 16,
                // row rho of the step before and of this one for R = 8): insert as soon as both exist
                // (keeps at most 8 slots of differences live)
                // perm selectors 8..11 replicate the sign bit of a 16-bit half over a whole byte, so
                // the four signs arrive as 0x00 / 0xff bytes and one bit-field insert puts them at
                // 7 - sl of each byte, no shift: 2 VALU per 4 bits. Slot sl = 0 keeps the whole bytes;
                // slots 1..7 overwrite their low bits.
                if constexpr (e % 16 >= 8)
                {
                    constexpr int sl = e % 16 - 8;
                    constexpr int w = e / 16;
                    constexpr uint32_t mask = (0x80808080u >> sl);
                    const uint32_t y0 = __builtin_amdgcn_perm(x0[e - 8], x0[e], 0x0b090a08u);
                    const uint32_t y1 = __builtin_amdgcn_perm(x1[e - 8], x1[e], 0x0b090a08u);
                    if constexpr (sl == 0)
                    {
                        acc[0][w] = y0;
                        acc[1][w] = y1;
                    }
                    else
                    {
                        asm("v_bfi_b32 %0, %1, %2, %0" : "+v"(acc[0][w]) : "v"(mask), "v"(y0));
                        asm("v_bfi_b32 %0, %1, %2, %0" : "+v"(acc[1][w]) : "v"(mask), "v"(y1));
                    }
                }
            });
            // HN: lane 63's bottom row (column s0 + q - 62) enters the publish queue
            if constexpr (HN) P = (uint32_t)__builtin_amdgcn_update_dpp((int)F[R - 1], (int)P, 0x130, 0xf, 0xf, false);
        });
        if constexpr (HN)
        {
            // lanes 64 - U .. 63 hold columns s0 - 62 .. s0 + U - 63 (ramp columns <= 0 land below
            // the entries of column 1 and are never read)
            if (lane >= kWave - U) lds_st(pub + (s0 + lane + U - 126 + kPairFeedOff), (int)P);
        }
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
        if constexpr (LW == 2)
        {
            // (R = 8: a chunk is 32 slots, one word per plane per lane)
            *reinterpret_cast<uint2 *>(dA_) = uint2{vA[0], vA[1]};
            *reinterpret_cast<uint2 *>(dB_) = uint2{vB[0], vB[1]};
        }
        static_assert(LW == 2 || LW % 4 == 0, "chunk store");
        sfor<LW / 4>([&](auto Xc) {
            constexpr int x = decltype(Xc)::value;
            *reinterpret_cast<u32x4 *>(dA_ + 4 * x) = u32x4{vA[4 * x], vA[4 * x + 1], vA[4 * x + 2], vA[4 * x + 3]};
            *reinterpret_cast<u32x4 *>(dB_ + 4 * x) = u32x4{vB[4 * x], vB[4 * x + 1], vB[4 * x + 2], vB[4 * x + 3]};
        });
    };
    // tail pairs of bodies from the first pair holding a body with s1 > n (the global score row is
    // in every strip that holds row m)
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
        // (R = 4: the strip's steps are a multiple of 8, not always of 16)
        if (s0 + U < nSteps) body(std::true_type{}, s0 + U, TB, TA);
    }
    const int rm = m - dA.row0;  // strip-relative row of the last DP row
    if (!HN && rm >= 0 && rm < kWave * R && lane == rm / R)
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
__global__ __launch_bounds__(kWave * kPairWaves, 2) void fill_pair_kernel(FillArgs a)
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
        if (u < units) process_pair<R, false, false>(a, 2 * u, 2 * u + 1, lane, nullptr, nullptr);
    }
}

// Chains: workgroup u = pairs 2u and 2u + 1 (every pair has blockDim / 64 strips), wave w = strip w of
// both; dynamic LDS = (strips - 1) rows of pair_row_entries(n) entries.
template <int R>
__global__ __launch_bounds__(kWave * kPairChainMax) void fill_pair_chain_kernel(FillArgs a)
{
    extern __shared__ int prowRaw[];
    lds_int *prow = (lds_int *)prowRaw;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = uniform((int)(threadIdx.x / kWave));
    const int S = (int)(blockDim.x / kWave);
    const int u = (int)blockIdx.x;
    const PairDesc pA = a.pairs[2 * u], pB = a.pairs[2 * u + 1];
    const int E = pair_row_entries((int)pA.text_len);
    for (int e = threadIdx.x; e < (S - 1) * E; e += blockDim.x) lds_st(prow + e, -1);
    __syncthreads();
    const int sA = uniform(pA.first_strip) + w, sB = uniform(pB.first_strip) + w;
    lds_int *feed = prow + (w - 1) * E, *pub = prow + w * E;
    if (w == 0) process_pair<R, false, true>(a, sA, sB, lane, feed, pub);
    else if (w + 1 < S) process_pair<R, true, true>(a, sA, sB, lane, feed, pub);
    else process_pair<R, true, false>(a, sA, sB, lane, feed, pub);
}

// The I/O wave of a group: global granules of the previous group's last strip -> ring[0], and
// ring[W'] (W' = compute waves with a strip) -> granules for the next group. Only lane 0 polls the
// granules while nothing is there (8 bytes per poll: up to a few hundred waiting groups must not
// load the fabric the running strips use); the bytes move 64 columns per instruction. Ring entries
// carry their lap tags both ways (ring_tag), like the compute waves' own hand-offs.
// (strips: the launch's strips, or its bands in a band workgroup)
__device__ __forceinline__ void io_wave(const FillArgs &a, const StripDesc *strips, int nstrips, int *cons, int *drain,
                                        lds_int *rings, int grp, int W, int lane)
{
    const int first = grp * W;
    const int last = min(first + W, nstrips) - 1;
    const StripDesc sf = strips[first];
    const StripDesc sl = strips[last];
    const int nIn = (sf.flags & kHasPrev) ? (int)a.pairs[sf.pair].text_len : 0;
    const int nOut = (sl.flags & kHasNext) ? (int)a.pairs[sl.pair].text_len : 0;
    const int wl = last - first + 1;  // ring fed by the last strip
    lds_int *r0 = (lds_int *)rings;
    lds_int *cons0 = (lds_int *)&cons[0];
    lds_int *rl = (lds_int *)(rings + wl * kRing);
    lds_int *consL = (lds_int *)&cons[wl];
    const uint64_t *bin = a.bnd + sf.bnd_in;
    uint64_t *bout = a.bnd + sl.bnd_out;
    int copied = 0, drained = 0;
    // slots of columns -63..0 are never copied in: give them their lap-0 tag, or the zeroed entries
    // would pass for lap-1 columns 1985..2048 (a compute-wave producer publishes from column -63)
    if (nIn > 0) lds_st(r0 + ring_slot(lane - 63), ring_tag(lane - 63));
    if (nIn == 0 && nOut == 0) return;
    uint64_t t0 = now_ticks();
    for (uint32_t spin = 1; copied < nIn || drained < nOut; ++spin)
    {
        bool moved = false;
        // 1. issue the granule poll (not waited for yet: the drain below runs under its latency, so
        //    the outgoing bottom row does not wait a global round trip per iteration)
        int want = 0;
        // (kIoWin windows of 64 columns per poll: a round trip with stores in flight takes longer than
        // a fast producer needs for one window)
        uint64_t v[kIoWin];
        if (copied < nIn)
        {
            // ring[0]'s consumer publishes its consumption every kConsEvery columns
            const int room = uniform(lds_ld(cons0)) + kRing - copied;  // free ring slots
            want = min(min(kIoWin * kWave, nIn - copied), room);
            if (want < min(16, nIn - copied)) want = 0;
        }
        // every poll loads whole windows (one round trip from the producer's store to the ring; a
        // lane-0 probe first would add a second): a few KiB per poll per waiting group is nothing
        // next to the fill's own traffic
        sfor<kIoWin>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value;
            v[q] = q * kWave + lane < want ? load_granule(bin + copied + q * kWave + lane) : 0;
        });
        // 2. drain ring[W'] into granules for the next group (up to kIoWin windows)
        for (int rep = 0; rep < kIoWin && drained < nOut; ++rep)
        {
            const int c = drained + lane + 1;
            const int x = lds_ld(rl + ring_slot(c)) ^ ring_tag(c);
            const uint64_t rdy = ballot(x >= 0 && c <= nOut);
            const int upto = drained + (~rdy == 0 ? kWave : (int)__builtin_ctzll(~rdy));
            if (!(upto - drained >= 16 || (upto >= nOut && upto > drained))) break;
            if (c <= upto) store_granule(bout + c - 1, ((uint64_t)a.epoch << 32) | (uint32_t)x);
            const bool full = upto - drained == kWave;
            drained = upto;
            if (lane == 0)
            {
                lds_st(consL, drained);
                lds_st((lds_int *)&drain[wl], drained);  // (bands wait for min(cons, drain))
            }
            moved = true;
            if (!full) break;
        }
        // 3. the poll's result -> ring[0]
        int total = 0;  // ready prefix over the windows
        bool open = want > 0;
        sfor<kIoWin>([&](auto Qc) {
            constexpr int q = decltype(Qc)::value;
            if (!open) return;
            const uint64_t rdy = ballot(q * kWave + lane < want && (uint32_t)(v[q] >> 32) == a.epoch);
            const int cnt = ~rdy == 0 ? kWave : (int)__builtin_ctzll(~rdy);
            const int c = copied + q * kWave + lane + 1;
            if (lane < cnt && (total + cnt >= min(16, nIn - copied))) lds_st(r0 + ring_slot(c), (int)(uint32_t)v[q] | ring_tag(c));
            total += cnt;
            open = cnt == kWave;
        });
        if (want > 0)
        {
            const int cnt = total;
            if (cnt >= min(16, nIn - copied))
            {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_PROGRESS)
                // I/O progress stamps: when ring[0] got column 4096q (timeline words 16..25 of
                // the group's first strip)
                if (a.timeline && lane == 0 && ((copied + cnt) >> 12) != (copied >> 12) && ((copied + cnt) >> 12) < 10)
                    a.timeline[kTimelineWords * (size_t)first + 16 + ((copied + cnt) >> 12)] = now_ticks();
#endif
                copied += cnt;
                moved = true;
            }
        }
        if (moved)
        {
            t0 = now_ticks();
            continue;
        }
        for (int z = 0; z < a.io_sleep; ++z) __builtin_amdgcn_s_sleep(1);
        if ((spin & 127) == 0 && !keep_waiting(a, t0, lane))
        {
            // release the producer so the group drains (the launch reports the abort; ring[0]'s
            // consumer gives up by itself)
            if (lane == 0)
            {
                lds_st(consL, nOut + kRing);
                lds_st((lds_int *)&drain[wl], nOut + kRing);
            }
            return;
        }
    }
}


// BAND fill: the drain wave of a band workgroup copies the in-group rings 1 .. wl-1 (fed by bands
// first .. last-1) to those bands' granules, the feed of the 64-row strips below them; the I/O wave
// still drains the last ring. A wave of its own: its write-through stores would otherwise sit in the
// I/O wave's vmcnt in front of every granule poll (in-order completion) and slow the cross-group
// hand-off.
// With kDrainWaves drain waves, wave d copies the rings r + 1 with r = d (mod kDrainWaves): with three,
// one ring each, and every SIMD of the workgroup holds one band and one helper wave (the I/O wave or a
// drain wave) instead of one SIMD carrying all three rings' copies beside its band, whose pace the
// whole chain then takes.
__device__ __forceinline__ void drain_wave(const FillArgs &a, int *drain, lds_int *rings, int grp, int W, int lane, int d)
{
    const int first = grp * W;
    const int last = min(first + W, a.num_bands) - 1;
    const int wl = last - first + 1;
    int dr[kMaxWaves - 1], drN[kMaxWaves - 1];
    uint64_t *drOut[kMaxWaves - 1];
    bool drPending = false;
    sfor<kMaxWaves - 1>([&](auto Rc) {
        constexpr int r = decltype(Rc)::value;  // ring r + 1, strip first + r
        dr[r] = 0;
        drN[r] = 0;
        drOut[r] = a.bnd;
        if (r + 1 < wl && r % kDrainWaves == d)
        {
            const StripDesc sr = a.bands[first + r];
            if (uniform(sr.flags) & kHasNext)
            {
                drN[r] = (int)uniform64(a.pairs[uniform(sr.pair)].text_len);
                drOut[r] = a.bnd + uniform64(sr.bnd_out);
                drPending = true;
            }
        }
    });
    uint64_t t0 = now_ticks();
    for (uint32_t spin = 1; drPending; ++spin)
    {
        bool moved = false;
        if (drPending)
        {
            drPending = false;
            sfor<kMaxWaves - 1>([&](auto Rc) {
                constexpr int r = decltype(Rc)::value;
                // (up to 4 x 64 columns per pass: the score waves outrun one window per poll round trip)
                for (int rep = 0; rep < 4 && dr[r] < drN[r]; ++rep)
                {
                    const int c = dr[r] + lane + 1;
                    const int x = lds_ld(rings + (r + 1) * kRing + ring_slot(c)) ^ ring_tag(c);
                    const uint64_t rdy = ballot(x >= 0 && c <= drN[r]);
                    const int upto = dr[r] + (~rdy == 0 ? kWave : (int)__builtin_ctzll(~rdy));
                    if (!(upto - dr[r] >= 16 || (upto >= drN[r] && upto > dr[r]))) break;
                    if (c <= upto) store_granule(drOut[r] + c - 1, ((uint64_t)a.epoch << 32) | (uint32_t)x);
                    const bool full = upto - dr[r] == kWave;
                    dr[r] = upto;
                    if (lane == 0) lds_st((lds_int *)&drain[r + 1], upto);
                    moved = true;
                    if (!full) break;
                }
                drPending = drPending || dr[r] < drN[r];
            });
        }
        if (moved)
        {
            t0 = now_ticks();
            continue;
        }
        for (int z = 0; z < a.io_sleep; ++z) __builtin_amdgcn_s_sleep(1);
        if ((spin & 127) == 0 && !keep_waiting(a, t0, lane))
        {
            if (lane == 0)
                for (int r = 1; r < wl; ++r)
                    if ((r - 1) % kDrainWaves == d) lds_st((lds_int *)&drain[r], 1 << 30);  // release the producers
            return;
        }
    }
}

// One workgroup = W compute waves + 1 I/O wave; it takes groups of W consecutive strips from the
// dynamic queue until the queue is empty. The queue order is the strip order, so a strip's
// predecessor has always been handed out before it: progress is guaranteed whatever the residency.
template <int R, bool LOCAL, int SK, bool CHAIN, bool TOUCH = false, bool ALIGN = false>
__global__ __launch_bounds__(kWave * (kMaxWaves + 1 + kDrainWaves)) void fill_kernel(FillArgs a)
{
    extern __shared__ int lds_dyn[];
    GroupHdr &H = *reinterpret_cast<GroupHdr *>(lds_dyn);
    lds_int *rings = (lds_int *)(lds_dyn + sizeof(GroupHdr) / 4);
    const int lane = threadIdx.x & (kWave - 1);
    const int w = uniform((int)(threadIdx.x / kWave));
    // compute waves; with CHAIN wave W is the I/O wave (plans without strip chains have none, and no
    // rings in LDS either: more workgroups fit a CU); band launches have one more wave, the drain
    // wave W + 1 (idle in the strip workgroups)
    const int W = (int)(blockDim.x / kWave) - (CHAIN ? 1 : 0) - (CHAIN && a.num_bands > 0 ? kDrainWaves : 0);
    if constexpr (SK == kTable)
        for (int e = threadIdx.x; e < a.A * a.A; e += blockDim.x) H.S[e] = a.score_tab[e];
    // BAND fill: workgroups [0, band_wgs) take groups of W bands from their own queue, the others
    // groups of W strips; with one workgroup per CU (the launch's LDS request) no CU mixes the two
    constexpr bool kBand = R == 1 && SK == kArr8 && CHAIN;
    const bool bandRole = kBand && a.num_bands > 0 && (int)blockIdx.x < a.band_wgs;
    const StripDesc *strips = bandRole ? a.bands : a.strips;
    const int nstrips = bandRole ? a.num_bands : a.num_strips;
    const int ngroups = bandRole ? a.num_band_groups : a.num_groups;
    uint32_t *qhead = bandRole ? &a.ctrl->band_head : &a.ctrl->queue_head;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_NO_STRIPS)
    if (kBand && a.num_bands > 0 && !bandRole) return;  // timing ablation: the bands alone (results wrong)
#endif
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_XCD)
    bool xcdFirst = true;
#endif
    while (true)
    {
        __syncthreads();  // every wave is done with the previous group's rings
        if (threadIdx.x == 0)
        {
            const bool aborted = __hip_atomic_load(&a.ctrl->abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_BAND_XCD)
            // experiment: band groups placed statically so that consecutive groups share an XCD
            // (workgroup b runs on XCD b % 8): groups x * per .. x * per + per - 1 on XCD x
            if (bandRole && ngroups % 8 == 0 && a.band_wgs == ngroups)
            {
                const int per = ngroups / 8;
                H.group = aborted || !xcdFirst ? ngroups : ((int)blockIdx.x % 8) * per + (int)blockIdx.x / 8;
                xcdFirst = false;
            }
            else
#endif
            H.group = aborted ? ngroups : (int)atomicAdd(qhead, 1u);
            H.nwaves = W;
        }
        if (threadIdx.x <= kMaxWaves) H.cons[threadIdx.x] = H.drain[threadIdx.x] = 0;
        if constexpr (CHAIN)
        {
            // tags: a zeroed ring matches no column (ring_tag)
            typedef int i32x4 __attribute__((ext_vector_type(4)));
            for (int e = 4 * threadIdx.x; e < (W + 1) * kRing; e += 4 * blockDim.x)
                *(__attribute__((address_space(3))) i32x4 *)(rings + e) = i32x4{0, 0, 0, 0};
        }
        __syncthreads();
        const int grp = uniform(H.group);
        if (grp >= ngroups) break;
        if (CHAIN && w == W)
        {
            io_wave(a, strips, nstrips, H.cons, H.drain, rings, grp, W, lane);
        }
        else if (CHAIN && w > W)
        {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_NO_DRAIN)
            // timing ablation: no copies of the in-group rings to granules (the strips starve)
            if (bandRole && lane == 0)
                for (int r = 1; r <= W; ++r) lds_st((lds_int *)&H.drain[r], 1 << 30);
#else
            if (bandRole) drain_wave(a, H.drain, rings, grp, W, lane, w - W - 1);
#endif
        }
        else
        {
            const int idx = grp * W + w;
            if (idx < nstrips)
            {
                // the strip kind is compile-time inside process_strip (branch-free body boundaries)
                // (CHAIN: some pair has several strips; otherwise every strip is alone and only one
                // variant is instantiated, which keeps the register count of the batch kernel down)
                const int f = uniform(strips[idx].flags) & (kHasPrev | kHasNext);
                const StripLds L{H.S, H.cons, H.nwaves, H.drain};
                if constexpr (kBand)
                    if (bandRole)
                    {
                        // the bands issue ahead of the I/O and drain waves sharing their SIMDs (measured
                        // -0.8 % fill for round 3's score waves, profiles/r03/dual_dev/prio_timeline.log)
                        __builtin_amdgcn_s_setprio(2);
                        // (every band publishes its bottom row: kHasNext)
                        if (f & kHasPrev) process_band<LOCAL, true, true, TOUCH, ALIGN>(a, L, rings, idx, w, lane);
                        else process_band<LOCAL, false, true, TOUCH, ALIGN>(a, L, rings, idx, w, lane);
                        __builtin_amdgcn_s_setprio(0);
                        continue;
                    }
                if constexpr (CHAIN)
                {
                    if (f == (kHasPrev | kHasNext)) process_strip<R, LOCAL, SK, true, true, ALIGN>(a, L, rings, idx, w, lane);
                    else if (f == kHasPrev) process_strip<R, LOCAL, SK, true, false, ALIGN>(a, L, rings, idx, w, lane);
                    else if (f == kHasNext) process_strip<R, LOCAL, SK, false, true, ALIGN>(a, L, rings, idx, w, lane);
                    else process_strip<R, LOCAL, SK, false, false, ALIGN>(a, L, rings, idx, w, lane);
                }
                else
                {
                    (void)f;
                    process_strip<R, LOCAL, SK, false, false>(a, L, rings, idx, w, lane);
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
        if constexpr (R == 1 && SK == kArr8 && !LOCAL)
            if (a.num_bands > 0 && a.A <= 4)
            {
                // global band fill of a DNA-sized alphabet: the kernel whose bands touch the codes ahead
                if (lds > 65536)
                    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&fill_kernel<R, LOCAL, SK, true, true>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                hipLaunchKernelGGL((fill_kernel<R, LOCAL, SK, true, true>), dim3(grid), dim3(kWave * (W + 1 + kDrainWaves)), lds, st, a);
                return;
            }
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&fill_kernel<R, LOCAL, SK, true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((fill_kernel<R, LOCAL, SK, true>), dim3(grid), dim3(kWave * (W + 1 + (a.num_bands > 0 ? kDrainWaves : 0))), lds, st, a);
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
        if (sk == kArr8A && chain) launch_fill_align(a, local, grid, W, st);
        else if (sk == kArr8 || sk == kArr8A)
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
        if constexpr (R >= 4)
        {
            if (chain)
            {
                // pair-packed chains: grid = couples, W = strips per pair, one LDS row per strip boundary
                const size_t lds = (size_t)(W - 1) * pair_row_entries(a.pair_text_len) * 4;
                if (lds > 65536)
                    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&fill_pair_chain_kernel<R>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                hipLaunchKernelGGL(fill_pair_chain_kernel<R>, dim3(grid), dim3(kWave * W), lds, st, a);
            }
            else hipLaunchKernelGGL(fill_pair_kernel<R>, dim3(grid), dim3(kWave * W), 0, st, a);
        }
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

#ifdef SA_FILL_ALIGN
// fill_r1a.hip: the kArr8A chain kernels (bands and strips read copy 0 of the text profiles)
void launch_fill_align(const FillArgs &a, bool local, int grid, int W, hipStream_t st)
{
    const size_t lds = std::max(group_lds_bytes(W), (size_t)a.chain_lds);
    const dim3 block(kWave * (W + 1 + (a.num_bands > 0 ? kDrainWaves : 0)));
    auto go = [&](auto kern) {
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3(grid), block, lds, st, a);
    };
#if defined(SA_EXPERIMENT) && defined(SA_EXP_ALIGN_TOUCH)
    // experiment: global bands touch the code lines ahead (the DNA kernel's TOUCH)
    if (!local) return go(&fill_kernel<1, false, kArr8, true, true, true>);
#endif
    if (local) go(&fill_kernel<1, true, kArr8, true, false, true>);
    else go(&fill_kernel<1, false, kArr8, true, false, true>);
}
#else
template void launch_fill_r<SA_FILL_R>(const FillArgs &, bool, int, int, int, bool, hipStream_t);
#endif

}  // namespace sa
