// Traceback for MI355X (gfx950): scalar path walk over the direction planes + parallel letter
// expansion. See sa_walk.h for the record format and DESIGN.md §3.2 for the measurements.
//
// Semantics (bit-exact with the reference CPU path):
//   traceBackNW  alignSequenceCPU.cpp:64-114   start at (m, n); row 0 forces LEFT, column 0 TOP
//   traceBackSW  alignSequenceCPU.cpp:10-62    start at the first maximum, stop at STOP or at the
//                                              border (without the last index update)
//
// A traceback path is a staircase: inside a row it only moves LEFT, inside a column only TOP. The walk
// therefore never steps cell by cell. It takes one scalar "find the first set bit" per ROW (row walk)
// or per COLUMN (column walk), on WINDOWS staged in VGPRs with two bits per cell:
//     bit 2c    the cell ends the run and the next move does not change the walk's free coordinate
//               (row walk: TOP-only; column walk: LEFT)
//     bit 2c+1  the cell ends the run with DIAG (local: DIAG or STOP)
// so for a line (row / column) entered at window position u (even)
//     p = ffs(W0[lane] >> u) = 2 * run + (1 if the leaving move is DIAG),   u += p + (p & 1)
// is the whole line: one v_readlane (issued a line ahead), four SALU and one v_writelane of the record
// p. Lane l of the windows is the l-th line of the current batch of 64 lines, walked from lane 63
// down; window w covers the 16 positions after window w-1 along the free coordinate. When W0 holds
// nothing at or after u the windows rotate (W0 <- W1 ...); after eight the kernel restages. Local
// mode marks a STOP cell by setting both of its bits: the search then finds its even bit, and bit
// p ^ 1 (set only for STOP: an even find is otherwise a run end without DIAG, an odd find has its
// even bit clear) ends the walk. The borders are encoded in the windows (global: column 0 TOP /
// row 0 LEFT; local: STOP), so they need no tests.
//
// ROW WALK (R = 1): lanes = the 64 rows of a strip (lane k = row k), windows = 8 x 16 columns left of
//   the strip's entry column, funnel shifts of the lane's own interleaved plane words (sa_layout.h:
//   R = 1 slot e = j - 1 + k). While a strip is walked, the raw planes of the
//   strip above, around the predicted entry column, are copied to LDS by global_load_lds, so staging
//   reads LDS, not HBM.
// COLUMN WALK (R >= 2, the batch shapes): lanes = 64 consecutive columns (lane l = column J0 - 63 + l),
//   windows = 8 blocks of 16 rows above the current row; a window word of lane l is gathered from the
//   plane words of the block's strip lanes at column J0 - 63 + l (R = 32: one word = 32 rows = two
//   blocks).
// The 64 lines of a batch run unrolled in one asm statement (sa_walk_rows.inc, tools/gen_walk_asm.py);
// partial batches and restages run the same logic as a C++ loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "sa_walk.h"
#include "sa_walk_rows.inc"
#include "sa_wave.h"

namespace sa {

// Plane layout of strip height R (sa_layout.h; the fill's Cfg<R>)
template <int R>
struct Geo {
    static constexpr int U = (16 / R) > 4 ? (16 / R) : 4;
    static constexpr int CS = U * R > 32 ? U * R : 32;  // slots per chunk
    static constexpr int NW = CS / 32;                  // words per plane per lane per chunk
    static constexpr int LW = 2 * NW;                   // dwords per lane per chunk
    static constexpr int RB = kWave * R;                // rows per strip
    static constexpr int FW = R < 16 ? R : 16;          // rows one strip lane gives a 16-row block
    static constexpr int NL = 16 / FW;                  // strip lanes per 16-row block
};

constexpr int kPfChunks = 12;  // R = 1 chunks (32 slots x 64 lanes x 2 planes = 512 B) prefetched per strip
constexpr int kChunkDw = 128;  // dwords per R = 1 chunk
constexpr int kPfDw = kPfChunks * kChunkDw;

__device__ __forceinline__ uint32_t spread16(uint32_t x)  // bit i -> bit 2i (low 16 bits)
{
    x &= 0xffffu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// Window word from 16 cells: E = bits "ends the run, free coordinate unchanged", D = "ends with DIAG
// (local: or STOP)"; the STOP window has STOP at the odd bit.
__device__ __forceinline__ uint32_t window(uint32_t E, uint32_t D) { return spread16(E) | (spread16(D) << 1); }

// ------------------------------------------------------------------------------------------------
// staging
// ------------------------------------------------------------------------------------------------
// Row walk: the eight windows of the calling lane's row (strip row = lane) for origin column jo:
// window w, bit pair c = column jo - 16w - c. The R = 1 planes are interleaved (sa_layout.h): the lane's
// dword stream holds each slot's (plane0, plane1) bits as the (odd, even) bits of a pair, slots
// ascending with the column from bit 31 down, so a window is one funnel shift of two consecutive
// dwords. Raw plane words come from the LDS prefetch when it covers every lane's chunks, else from
// global memory (uniform decision). sb = the strip's first dword.
template <bool LOCAL>
__device__ __forceinline__ void rw_stage(const uint32_t *__restrict__ sb, const uint32_t *pf, int pfclo, int jo,
                                         int lane, uint32_t (&W)[8], uint64_t *dbg = nullptr)
{
    const int etop = jo - 1 + lane;   // slot of column jo in this lane's stream (R = 1: e = j - 1 + k)
    const int c0 = etop >> 5;         // (arithmetic shift: etop may be negative after a restage)
    const bool hi = (etop & 16) != 0;  // slot etop lies in its chunk's second dword
    const int sh = 30 - 2 * (etop & 15);  // its pair down to bits 1:0
    uint32_t L[10];                   // dwords 2c0+1, 2c0, 2c0-1, ..., 2c0-8 of the stream
    const int needLo = max(0, (jo - 1 - 128) >> 5), needHi = (jo + 62) >> 5;
    const bool inPf = pfclo != INT_MIN && needLo >= pfclo && needHi < pfclo + kPfChunks;
    sfor<5>([&](auto Qc) {
        constexpr int q = decltype(Qc)::value;
        const int c = c0 - q;
        const u32x2 v = inPf ? *reinterpret_cast<const u32x2 *>(pf + max(c - pfclo, 0) * kChunkDw + lane * 2)
                             : *reinterpret_cast<const u32x2 *>(sb + (int64_t)max(c, 0) * kChunkDw + lane * 2);
        L[2 * q] = c >= 0 ? v.y : 0u;
        L[2 * q + 1] = c >= 0 ? v.x : 0u;
    });
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
    if (dbg)
    {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+v"(L[0]), "+v"(L[9]));
        dbg[0] += __builtin_amdgcn_s_memtime();  // minus the caller's start stamp
        dbg[1] += inPf ? 0 : 1;
    }
#endif
    uint32_t S[9];  // S[i] = the dword i before slot etop's
    sfor<9>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        S[i] = hi ? L[i] : L[i + 1];
    });
    sfor<8>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        uint32_t x = __builtin_amdgcn_alignbit(S[w + 1], S[w], sh);
        // global: the even bit is raw "up > left"; a run ends with TOP only without DIAG (:78-79).
        // local: plane0 = DIAG|STOP and plane1 = (TOP&~DIAG)|STOP are the window bits as they are
        if constexpr (!LOCAL) x &= ~((x >> 1) & 0x55555555u);
        W[w] = x;
    });
    if (jo < 16 * 8 + 1)
    {
        // the windows reach column 0: columns < 1 are cleared, column 0 is TOP (global, :78-79) or
        // both bits (local: the border ends the walk)
        sfor<8>([&](auto Wc) {
            constexpr int w = decltype(Wc)::value;
            const int z = jo - 16 * w;  // pair of column 0 (uniform)
            const uint32_t vm = z >= 16 ? ~0u : (z <= 0 ? 0u : ((1u << (2 * z)) - 1u));
            const uint32_t c0b = (z >= 0 && z < 16) ? (LOCAL ? 3u : 1u) << (2 * z) : 0u;
            W[w] = (W[w] & vm) | c0b;
        });
    }
}

// Row walk, stager wave: kStageWin windows of the calling lane's row for origin column jo (window w,
// bit pair c = column jo - 16w - c, as rw_stage), from the strip's planes in global memory, into
// dst[w * 64 + lane] (LDS). The walker takes any eight consecutive of them.
constexpr int kStageWin = 24;  // 384 columns: the walker's entry may lie up to 256 columns below the origin
template <bool LOCAL>
__device__ __forceinline__ void rw_stage_far(const uint32_t *__restrict__ sb, int jo, int lane, uint32_t *dst)
{
    const int etop = jo - 1 + lane;
    const int c0 = etop >> 5;
    const bool hi = (etop & 16) != 0;
    const int sh = 30 - 2 * (etop & 15);
    constexpr int NP = (kStageWin + 3) / 2;  // chunk pairs: dwords 2c0+1 .. 2c0 - 2 NP + 2
    uint32_t L[2 * NP];
    sfor<NP>([&](auto Qc) {
        constexpr int q = decltype(Qc)::value;
        const int c = c0 - q;
        const u32x2 v = *reinterpret_cast<const u32x2 *>(sb + (int64_t)max(c, 0) * kChunkDw + lane * 2);
        L[2 * q] = c >= 0 ? v.y : 0u;
        L[2 * q + 1] = c >= 0 ? v.x : 0u;
    });
    sfor<kStageWin>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        const uint32_t lo = hi ? L[w] : L[w + 1], up = hi ? L[w + 1] : L[w + 2];
        uint32_t x = __builtin_amdgcn_alignbit(up, lo, sh);
        if constexpr (!LOCAL) x &= ~((x >> 1) & 0x55555555u);
        const int z = jo - 16 * w;  // pair of column 0 (uniform): columns < 1 cleared, column 0 the border
        if (z < 16)
        {
            const uint32_t vm = z <= 0 ? 0u : ((1u << (2 * z)) - 1u);
            const uint32_t c0b = (z >= 0) ? (LOCAL ? 3u : 1u) << (2 * z) : 0u;
            x = (x & vm) | c0b;
        }
        dst[w * kWave + lane] = x;
    });
}

// Column walk: the eight windows of the calling lane's column j = J0 - 63 + lane for the row blocks
// G0, G0-1, ..., G0-7 (block G = pair rows 16G+1 .. 16G+16; bit pair c = row 16G + 16 - c). Block -1
// is the row-0 border. mb = the pair's first strip's first dword.
template <int R, bool LOCAL>
__device__ __forceinline__ void cw_stage(const uint32_t *__restrict__ mb, int64_t sstride, int J0, int G0, int lane,
                                         uint32_t (&W)[8])
{
    using G_ = Geo<R>;
    const int j = J0 - 63 + lane;
    uint32_t f0[8], f1[8];
    sfor<8>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        const int G = G0 - w;  // uniform
        f0[w] = 0;
        f1[w] = 0;
        if (G >= 0)
        {
            const int r0 = 16 * G;  // first (top) row of the block, 0-based
            const int b = r0 / G_::RB, rs = r0 - b * G_::RB;
            const int k0 = rs / R, rho0 = rs - k0 * R;
            const uint32_t *sb = mb + (int64_t)b * sstride;
            sfor<G_::NL>([&](auto Tc) {
                constexpr int t = decltype(Tc)::value;
                const int k = k0 + t;
                const int s = j - 1 + k;  // the strip lane's step at column j
                const int e = max(s, 0) * R + rho0;
                const int64_t off = (int64_t)(e / G_::CS) * (kWave * G_::LW) + k * G_::LW + (e % G_::CS) / 32;
                const int sh = 32 - G_::FW - (e & 31);
                constexpr uint32_t fm = G_::FW == 32 ? ~0u : ((1u << G_::FW) - 1u);
                const uint32_t x0 = j >= 1 ? (sb[off] >> sh) & fm : 0u;
                const uint32_t x1 = j >= 1 ? (sb[off + G_::NW] >> sh) & fm : 0u;
                f0[w] |= x0 << (G_::FW * (G_::NL - 1 - t));
                f1[w] |= x1 << (G_::FW * (G_::NL - 1 - t));
            });
        }
    });
    sfor<8>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        const int G = G0 - w;
        const uint32_t x0 = f0[w], x1 = f1[w];
        uint32_t E, D;
        if constexpr (!LOCAL)
        {
            D = x0;                                   // DIAG
            E = ~x0 & ~x1 & 0xffffu;                  // LEFT
            if (G == -1) E = 1;                       // row 0: LEFT to column 0 (traceBackNW :80-81)
        }
        else
        {
            D = x0;                                   // DIAG or STOP
            E = ((~x0 & ~x1) | (x0 & x1)) & 0xffffu;  // LEFT, or STOP (both bits)
            if (G == -1) { D = 1; E = 1; }            // row 0: the border ends the walk (STOP)
        }
        if (G < -1) { D = 0; E = 0; }
        W[w] = window(E, D);
    });
}

// Column walk, R = 32, one strip per pair (the batch shapes), staged from an LDS copy of the plane
// sectors the next batch will need: the gathers of cw_stage (16 chunks x one 32-B strip-lane sector
// per window, for 64 columns) were latency-bound with every pair of a batch in flight (255 clk per
// column against 21 alone, tools/tb_batch_phase.py), so they are issued a batch ahead with
// global_load_lds. Buffer layout: [chunk - c_lo][k - k_lo][8 dwords] (a strip lane's segment of a
// chunk: 4 words per plane), kCwChunks x kCwLanes entries.
constexpr int kCwChunks = 20, kCwLanes = 8;  // 64 columns + 8 lanes of skew span <= 19 chunks
constexpr int kCwDw = kCwChunks * kCwLanes * 8;

// The k range [k_lo, k_lo + kCwLanes) that should cover the next batch's windows when the path
// moves `drift` row blocks per batch (rows blocks G0' - 7 .. G0', k = G >> 1).
__device__ __forceinline__ int cw_klo(int G0, int drift) { return max(0, ((G0 - drift - 7) >> 1) - 1); }

// Prefetch for the batch whose lane 63 is column J0n: chunks from the first step it reads.
__device__ __forceinline__ void cw_prefetch(const uint32_t *__restrict__ mb, int nchunks, int J0n, int klo, int lane,
                                            uint32_t *buf, int &clo)
{
    clo = max(0, (J0n - 64 + klo) >> 2);  // step s = j - 1 + k of column J0n - 63 and lane k_lo
    sfor<kCwChunks * kCwLanes * 2 / kWave>([&](auto Ic) {
        constexpr int it = decltype(Ic)::value;
        const int q = it * kWave + lane;        // 16-B piece: (chunk, lane, half)
        const int c = min(clo + (q >> 4), nchunks - 1);
        const int k = min(klo + ((q >> 1) & 7), kWave - 1);
        const uint32_t *src = mb + (int64_t)c * (kWave * 8) + k * 8 + (q & 1) * 4;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(buf + it * kWave * 4), 16, 0, 0);
    });
}

// cw_stage for R = 32 reading the LDS copy (the caller has checked that it covers the windows)
template <bool LOCAL>
__device__ __forceinline__ void cw_stage_lds(const uint32_t *buf, int clo, int klo, int J0, int G0, int lane,
                                             uint32_t (&W)[8])
{
    const int j = J0 - 63 + lane;
    sfor<8>([&](auto Wc) {
        constexpr int w = decltype(Wc)::value;
        const int G = G0 - w;  // uniform
        uint32_t x0 = 0, x1 = 0;
        if (G >= 0)
        {
            const int k = G >> 1, sh = 16 - 16 * (G & 1);  // rho0 = 16 (G & 1)
            const int s = max(j - 1 + k, 0);
            // (lanes left of column 1 compute an index outside the copy: clamped, value unused)
            const int ix = min(max((((s >> 2) - clo) * kCwLanes + (k - klo)) * 8 + (s & 3), 0), kCwDw - 8);
            x0 = j >= 1 ? (buf[ix] >> sh) & 0xffffu : 0u;
            x1 = j >= 1 ? (buf[ix + 4] >> sh) & 0xffffu : 0u;
        }
        uint32_t E, D;
        if constexpr (!LOCAL)
        {
            D = x0;
            E = ~x0 & ~x1 & 0xffffu;
            if (G == -1) E = 1;
        }
        else
        {
            D = x0;
            E = ((~x0 & ~x1) | (x0 & x1)) & 0xffffu;
            if (G == -1) { D = 1; E = 1; }
        }
        if (G < -1) { D = 0; E = 0; }
        W[w] = window(E, D);
    });
}

// ------------------------------------------------------------------------------------------------
// the walk
// ------------------------------------------------------------------------------------------------
// Runs the unrolled 64-line batch (lanes 63..0). Returns st: -1 = batch done, K = windows exhausted
// at lane K, 0x100|K = STOP at lane K; lp = the last record written (or the STOP's p).
template <bool LOCAL>
__device__ __forceinline__ void walk_batch_asm(int &u, int &pa, int &na, int &st, int &lp, uint32_t &vrec,
                                               uint32_t (&W)[8])
{
    if constexpr (!LOCAL)
    {
        asm volatile(SA_WALK_ROWS_GLOBAL
                     : [u] "+s"(u), [pa] "+s"(pa), [na] "+s"(na), [st] "=&s"(st), [lp] "=&s"(lp), [rec] "+v"(vrec),
                       [w0] "+v"(W[0]), [w1] "+v"(W[1]), [w2] "+v"(W[2]), [w3] "+v"(W[3]), [w4] "+v"(W[4]),
                       [w5] "+v"(W[5]), [w6] "+v"(W[6]), [w7] "+v"(W[7])
                     :
                     : "scc", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95",
                       "s96", "s97");
    }
    else
    {
        asm volatile(SA_WALK_ROWS_LOCAL
                     : [u] "+s"(u), [pa] "+s"(pa), [na] "+s"(na), [st] "=&s"(st), [lp] "=&s"(lp), [rec] "+v"(vrec),
                       [w0] "+v"(W[0]), [w1] "+v"(W[1]), [w2] "+v"(W[2]), [w3] "+v"(W[3]), [w4] "+v"(W[4]),
                       [w5] "+v"(W[5]), [w6] "+v"(W[6]), [w7] "+v"(W[7])
                     :
                     : "scc", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95",
                       "s96", "s97");
    }
}

// Line walk state of one batch of 64 lines
struct Lines {
    int u = 0, pa = 0, na = 0;  // window position, positions skipped in this line, rotations
    int kk = 63;                // next lane to walk
    int lastp = 0;              // record of the last finished line
    bool stopped = false;
    int stopLane = 0, stopPos = 0, stopRun = 0;  // local STOP: lane, window position, run
    uint32_t vrec = 0;
};

// The generic loop over lanes kk .. kmin (the asm's logic); `restage` refills exhausted windows.
template <bool LOCAL, typename Restage>
__device__ __forceinline__ void walk_lines(Lines &L, int kmin, uint32_t (&W)[8], Restage &&restage)
{
    while (L.kk >= kmin)
    {
        if (L.na > 7) restage();
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)W[0], L.kk);
        const uint64_t x = (uint64_t)w >> L.u;
        if (x == 0)
        {
            L.pa += 32 - L.u;
            L.u = 0;
            sfor<7>([&](auto Xc) {
                constexpr int q = decltype(Xc)::value;
                W[q] = W[q + 1];
            });
            W[7] = 0;
            ++L.na;
            continue;
        }
        const int pp = (int)__builtin_ctz((uint32_t)x);
        if constexpr (LOCAL)
        {
            if ((x >> (pp ^ 1)) & 1u)  // both bits: STOP
            {
                L.stopped = true;
                L.stopLane = L.kk;
                L.stopPos = L.u + pp;
                L.stopRun = (L.pa + pp) >> 1;
                return;
            }
        }
        L.u += pp + (pp & 1);
        L.vrec = (uint32_t)amdgcn_writelane(L.pa + pp, L.kk, (int)L.vrec);
        L.lastp = L.pa + pp;
        L.pa = 0;
        --L.kk;
    }
}

// The unrolled batch, then the generic loop for whatever it left (a restage or nothing).
template <bool LOCAL, typename Restage>
__device__ __forceinline__ void walk_batch(Lines &L, bool fast, int kmin, uint32_t (&W)[8],
                                           Restage &&restage)
{
    if (fast && L.kk == 63 && kmin == 0)
    {
        int st, lp;
        walk_batch_asm<LOCAL>(L.u, L.pa, L.na, st, lp, L.vrec, W);
        if (st < 0)
        {
            L.kk = -1;
            L.lastp = lp;
        }
        else
        {
            L.kk = st & 0xff;
            if (LOCAL && (st & 0x100))
            {
                L.stopped = true;
                L.stopLane = L.kk;
                L.stopPos = L.u + lp;
                L.stopRun = (L.pa + lp) >> 1;
                return;
            }
        }
    }
    walk_lines<LOCAL>(L, kmin, W, restage);
}

// Start cell and score of pair p; false when there is nothing to walk (head complete).
template <bool LOCAL>
__device__ __forceinline__ bool walk_start(const WalkArgs &a, int p, int n, int m, int first, int nstrips, int lane,
                                           TbHead &h, int &i, int &j)
{
    h.kind = kRecRows;
    h.tail_op = kLeft;
    h.tail = 0;
    h.nrec = 0;
    h.err = 0;
    if constexpr (!LOCAL)
    {
        h.score = nstrips > 0 ? a.pair_score[p] : -a.gap * (n + m);
        i = m;
        j = n;
    }
    else
    {
        uint64_t k = 0;
        for (int s = lane; s < nstrips; s += kWave) k = max(k, a.strip_best[first + s]);
        k = wave_max_u64(k);
        const int rb = a.key_rowbits;
        const uint64_t km = (1ull << rb) - 1;
        const int H = (int)(k >> (2 * rb));
        if (H > 0)
        {
            h.score = H;
            i = (int)(km - ((k >> rb) & km));
            j = (int)(km - (k & km));
        }
        else
        {
            h.score = 0;  // no positive cell: maxIJ stays 0 (alignSequenceCPU.cpp:152)
            i = 0;
            j = 0;
        }
    }
    h.i0 = i;
    h.j0 = j;
    if (i > 0 && j > 0) return true;
    // nothing to walk through: global with an empty sequence (only border moves), or local with no
    // positive cell (empty alignment; starts (uint64)-1 are traceBackSW's initial indices)
    if constexpr (!LOCAL)
    {
        h.tail = i + j;
        h.tail_op = i > 0 ? kTop : kLeft;
        h.start_text = h.start_pattern = (i + j) > 0 ? 0 : -1;
    }
    else
    {
        h.start_text = (int64_t)j - 1;
        h.start_pattern = (int64_t)i - 1;
    }
    return false;
}

// Row walk (R = 1): a walker wave and a stager wave per pair. The walker runs the rows' scalar chain;
// at the start of strip b it asks the stager for strip b-1's windows with origin = strip b's entry
// column (the path only moves left, so strip b-1's entry lies at or left of it), and the stager builds
// kStageWin of them (384 columns) into LDS while the walker walks strip b. When the walker reaches
// strip b-1 and the stager is done and covers the entry column, eight LDS reads replace the staging
// (≈ 20 of the ≈ 85 clocks per row were staging); otherwise the walker stages as before.
// Request words (LDS): [0] sequence number of the last request (-1: quit), [1] strip, [2] origin,
// [3] the last sequence number the stager finished. One wave's LDS operations execute in order, so
// the fields written before [0] / the windows written before [3] are there when it is seen.
template <bool LOCAL>
__device__ void rw_stager(const WalkArgs &a, const uint32_t *mb, int64_t sstride, volatile int *req, uint32_t (*swin)[kStageWin * kWave],
                          int lane)
{
    int seen = 0;
    for (uint32_t spin = 1;; ++spin)
    {
        const int q = uniform(req[0]);
        if (q < 0) return;
        if (q == seen)
        {
            if (spin > 64) __builtin_amdgcn_s_sleep(2);
            continue;
        }
        seen = q;
        spin = 0;
        const int b = uniform(req[1]), O = uniform(req[2]);
        rw_stage_far<LOCAL>(mb + (int64_t)b * sstride, O, lane, swin[q & 1]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the windows before the done word)
        if (lane == 0) req[3] = q;
    }
}

// Where traceBackSW ends in a strip of the local row walk (the rows 64 cb + 1 .. 64 cb + ck + 1, lane l
// = row 64 cb + l + 1, walked from lane ck down; per lane: H at the row's entry He, the row's record
// run / dg, its entry column ce and leaving column lv = ce - run), if it does: the first row in walk
// order where a cell's H is 0 (a STOP, alignSequenceCPU.cpp:18, :189) or a move goes onto row 0 /
// column 0 (:44-46), and the head fields: records (cn0 before the strip), the trailing LEFT run, the
// start indices (Response::startInAlignedText / Pattern). Uniform result.
__device__ __forceinline__ bool local_strip_end(int He, int run, int dg, int ce, int lv, int cb, int ck, int cn0, int gap,
                                                int lane, int &nrec, int &tail, int &st, int &sp0)
{
    const int row = 64 * cb + lane + 1;
    int rz = INT_MAX;  // the first cell r = 0 .. run of the row whose H = He + g r is 0
    if (He == 0) rz = 0;
    else if (gap < 0 && He % (-gap) == 0) rz = He / (-gap);
    const bool e1 = rz <= run && rz < ce;                       // STOP before column 0
    const bool e2 = !e1 && lv <= 0;                              // the LEFT run reaches column 0
    const bool e3 = !e1 && !e2 && (row == 1 || (dg && lv == 1)); // TOP / DIAG onto row 0 / column 0
    const uint64_t ev = ballot(lane <= ck && (e1 || e2 || e3));
    if (ev == 0) return false;
    const int l = 63 - (int)__builtin_clzll(ev);  // the first in walk order (lane k down)
    const int lrow = 64 * cb + l + 1;
    const int lce = __builtin_amdgcn_readlane(ce, l), llv = __builtin_amdgcn_readlane(lv, l);
    const int lrz = __builtin_amdgcn_readlane(rz, l), lrun = __builtin_amdgcn_readlane(run, l);
    const bool l1 = (ballot(e1) >> l) & 1, l2 = (ballot(e2) >> l) & 1;
    nrec = cn0 + (ck - l);
    if (l1)
    {
        tail = lrz;  // the STOP cell (lrow, lce - lrz): every move into it updated the indices
        st = lce - lrz - 1;
        sp0 = lrow - 1;
    }
    else if (l2)
    {
        tail = lrun;  // LEFT moves to column 1, then onto column 0 without an index update
        st = 0;
        sp0 = lrow - 1;
    }
    else
    {
        nrec += 1;  // the row's record is whole; its move lands on the border (no index update)
        tail = 0;
        st = lrow == 1 ? llv - 1 : 0;
        sp0 = lrow == 1 ? 0 : lrow - 1;
    }
    return true;
}

// Local row walk: the stager also runs local_check on every strip the walker posts. The walk runs on
// the global encoding (the R = 1 planes hold no STOP), so where traceBackSW ends -- the first cell
// whose H is 0 (a STOP, alignSequenceCPU.cpp:18, :189) or the first move onto row 0 / column 0
// (:44-46) -- comes from H followed along the path: a row entered at H_e adds g per LEFT cell
// (H(left) = H + g, :176, :185-186), its leaving TOP adds g, its leaving DIAG subtracts S of its cell
// (:178). Per strip (lane l = row 64 b + l + 1, walked from lane k down): the entry columns from a
// prefix sum of the moves, the leaving DIAG cells' letters gathered from the inputs (in flight while
// window requests are served), then a prefix sum of the H steps and one ballot for the first row
// where the walk ends. The walker learns the verdict a strip or two later; the records it wrote past
// it lie past nrec.
__device__ void rw_stager_local(const WalkArgs &a, const PairDesc &sp, const uint32_t *mb, int64_t sstride, volatile int *req,
                                uint32_t (*swin)[kStageWin * kWave], const int *stab, int (*chkBuf)[72], int *chkCtl, int lane)
{
    volatile int *ctl = (volatile int *)chkCtl;
    const int64_t toff = (int64_t)uniform64(sp.text_off), poff = (int64_t)uniform64(sp.pattern_off);
    int seen = 0, cseen = 0;
    bool inflight = false, ended = false;
    int Hc = 0;
    int cb = 0, ck = 0, cn0 = 0;                              // the check in flight: strip, first lane, nrec before
    int run = 0, dg = 0, ce = 0, lv = 0, pl = 0, tl = 0;      // per lane (row)
    for (uint32_t spin = 1;; ++spin)
    {
        const int q = uniform(req[0]);
        if (q < 0) return;
        if (q != seen)
        {
            // window requests first: the walker is waiting for them
            seen = q;
            spin = 0;
            const int b = uniform(req[1]), O = uniform(req[2]);
            rw_stage_far<false>(mb + (int64_t)b * sstride, O, lane, swin[q & 1]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the windows before the done word)
            if (lane == 0) req[3] = q;
            continue;
        }
        if (inflight)
        {
            spin = 0;
            inflight = false;
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(pl), "+v"(tl)::"memory");  // the gathered letters
            const int S = dg ? stab[pl * a.A + tl] : 0;
            const int delta = lane <= ck ? a.gap * run + (dg ? -S : a.gap) : 0;
            const int Pd = wave_prefix_sum(delta);
            const int tot = __builtin_amdgcn_readlane(Pd, ck);
            const int He = Hc + (tot - Pd);  // H at this lane's row entry
            int nrec, tail, st, sp0;
            if (!local_strip_end(He, run, dg, ce, lv, cb, ck, cn0, a.gap, lane, nrec, tail, st, sp0))
            {
                Hc += tot;
                if (lane == 0) ctl[2] = cseen;
                continue;
            }
            if (lane == 0)
            {
                ctl[4] = nrec;
                ctl[5] = tail;
                ctl[6] = st;
                ctl[7] = sp0;
                ctl[2] = cseen;
                ctl[3] = 1;  // (after the fields: one wave's LDS writes execute in order)
            }
            ended = true;
            continue;
        }
        if (!ended && uniform(ctl[0]) > cseen)
        {
            // take the next posted strip: its moves, entry columns, letters (gathers in flight)
            spin = 0;
            ++cseen;
            const int *slot = chkBuf[cseen & 1];
            const int pv = slot[lane];
            cb = uniform(slot[64]);
            ck = uniform(slot[65]);
            const int jc = uniform(slot[66]);
            cn0 = uniform(slot[67]);
            if (cseen == 1) Hc = uniform(slot[68]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) ctl[1] = cseen;  // (the slot is free once read)
            run = lane <= ck ? pv >> 1 : 0;
            dg = lane <= ck ? pv & 1 : 0;
            const int P = wave_prefix_sum(run + dg);
            ce = jc - (__builtin_amdgcn_readlane(P, ck) - P);  // entry column of this lane's row
            lv = ce - run;
            pl = lane <= ck ? (int)a.pattern[poff + 64 * cb + lane] : 0;
            tl = lane <= ck && dg && lv >= 1 ? (int)a.text[toff + lv - 1] : 0;
            inflight = true;
            continue;
        }
        if (spin > 64) __builtin_amdgcn_s_sleep(2);
    }
}

// LDS of the row walk (walk_rw_pair)
template <bool LOCAL>
struct RwLds {
    uint32_t pfbuf[2][kPfDw];
    uint32_t swin[2][kStageWin * kWave];
    int req[4];
    int stab[LOCAL ? 32 * 32 : 1];  // local: the substitution scores S (local_check)
    // local: strips posted for local_check ([2][64 records + b, k, entry column, nrec before, H0]) and
    // the check's control words ([0] posted, [1] taken, [2] done, [3] ended, [4..7] nrec, tail, starts)
    int chkBuf[LOCAL ? 2 : 1][72];
    int chkCtl[8];
};

// The row walk of pair p by a block of two waves (wave 0 the walker, wave 1 the stager); every thread
// of the block calls it (it has a barrier). walk_rw_kernel, and tb_finish_kernel for the pairs the
// table traceback leaves.
template <bool LOCAL>
__device__ __forceinline__ void walk_rw_pair(const WalkArgs &a, const int p, RwLds<LOCAL> &S)
{
    uint32_t(&pfbuf)[2][kPfDw] = S.pfbuf;
    uint32_t(&swin)[2][kStageWin * kWave] = S.swin;
    int *req = S.req;
    int *stab = S.stab;
    int(&chkBuf)[LOCAL ? 2 : 1][72] = S.chkBuf;
    int *chkCtl = S.chkCtl;
    const int lane = threadIdx.x & (kWave - 1);
    if (threadIdx.x < 4) req[threadIdx.x] = 0;
    if (threadIdx.x < 8) chkCtl[threadIdx.x] = 0;
    if constexpr (LOCAL)
        for (int e = threadIdx.x; e < a.A * a.A; e += blockDim.x) stab[e] = a.score_tab[e] - a.gap;  // (the table holds S + g)
    __syncthreads();
    if (threadIdx.x >= 2 * kWave) return;  // (a larger block's other waves: tb_walk_kernel's finish blocks)
    if (threadIdx.x >= kWave)
    {
        // the stager: strips of the pair's chain (R = 1 layout, as the walker computes below)
        const PairDesc sp = a.pairs[p];
        if (uniform(sp.num_strips) > 0 && uniform((int)sp.text_len) > 0)
        {
            const StripDesc s0 = a.strips[uniform(sp.first_strip)];
            if constexpr (LOCAL)
                rw_stager_local(a, sp, a.masks + uniform64(s0.mask_off) * 4, (int64_t)uniform(s0.nsteps) * 4, req, swin,
                                stab, chkBuf, chkCtl, lane);
            else
                rw_stager<false>(a, a.masks + uniform64(s0.mask_off) * 4, (int64_t)uniform(s0.nsteps) * 4, req, swin, lane);
        }
        return;
    }
    PairDesc pd = a.pairs[p];
    const int n = uniform((int)pd.text_len), m = uniform((int)pd.pattern_len);
    const int first = uniform(pd.first_strip), nstrips = uniform(pd.num_strips);
    int32_t *rec = a.rec + uniform64(pd.rec_off);
    const uint64_t tW0 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
    TbHead h;
    int i, j;
    if (walk_start<LOCAL>(a, p, n, m, first, nstrips, lane, h, i, j))
    {
        StripDesc sd = a.strips[first];
        const int nsteps = uniform(sd.nsteps);
        const uint32_t *mb = a.masks + uniform64(sd.mask_off) * 4;  // 16 B per slot
        const int64_t sstride = (int64_t)nsteps * 4;                // dwords per strip
        const int nchunks = nsteps >> 5;
        int b = (i - 1) >> 6, k = (i - 1) & 63, jc = j;
        int nrec = 0;
        int pfb = 0, pfclo = INT_MIN;
        int reqSeq = 0, reqO = 0;  // the last request to the stager
        Lines L;
        // local: the walk runs on the global encoding (the R = 1 planes hold no STOP); after every
        // strip it posts the strip's records to the stager wave, whose local_check finds where
        // traceBackSW ends (rw_stager_local), and it stops once the stager reports the end
        int chkSeq = 0;
        // expected column drift of the path per strip (prefetch placement)
        const int drift = (int)(((int64_t)n * 64 + m / 2) / m);
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
        uint64_t tStage = 0, tBatch = 0;  // shader clocks in staging / in the walk proper
        uint64_t sdbg[2] = {0, 0}, tLoadStart = 0, nStrips = 0, nRestage = 0, nStagerHit = 0;
#endif
        while (b >= 0)
        {
            const uint32_t *sb = mb + (int64_t)b * sstride;
            // this strip's prefetch has landed; the record store of the previous strip (issued
            // after it, the youngest vector-memory operation) may still be in flight
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            uint32_t W[8];
            int jo = jc;
            int u0 = 0;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
            const uint64_t c0 = __builtin_amdgcn_s_memtime();
            tLoadStart += c0;
            ++nStrips;
#endif
            // the stager's windows for this strip: origin reqO, entry jc at window (d >> 4), pair d & 15
            const int d = reqO - jc;
            bool hit;
            if constexpr (LOCAL)
            {
                // the stager's done word first, then its windows speculatively, in one LDS round trip
                // (the wave's LDS reads execute in issue order, so windows read after a done word that
                // matches were complete: the stager writes them before the word); local traceback
                // -2.7 %, but global +2 % (profiles/r04/ab_walkspec_v1.log): global keeps two trips
                const bool near = reqSeq > 0 && d >= 0 && d < 16 * (kStageWin - 8);
                const int sdone = ((volatile int *)req)[3];
                asm volatile("" ::: "memory");
                const uint32_t *src = swin[reqSeq & 1] + (near ? d >> 4 : 0) * kWave + lane;
                uint32_t Ws[8];
                sfor<8>([&](auto Wc) { Ws[decltype(Wc)::value] = src[decltype(Wc)::value * kWave]; });
                hit = near && uniform(sdone) == reqSeq;
                if (hit) sfor<8>([&](auto Wc) { W[decltype(Wc)::value] = Ws[decltype(Wc)::value]; });
            }
            else
            {
                hit = reqSeq > 0 && d >= 0 && d < 16 * (kStageWin - 8) && uniform(((volatile int *)req)[3]) == reqSeq;
                if (hit)
                {
                    const uint32_t *src = swin[reqSeq & 1] + (d >> 4) * kWave + lane;
                    sfor<8>([&](auto Wc) {
                        constexpr int w = decltype(Wc)::value;
                        W[w] = src[w * kWave];
                    });
                }
            }
            if (hit)
            {
                jo = reqO - 16 * (d >> 4);
                u0 = 2 * (d & 15);
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
                ++nStagerHit;
#endif
            }
            else
            {
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
                rw_stage<false>(sb, pfbuf[pfb], pfclo, jo, lane, W, sdbg);
#else
                rw_stage<false>(sb, pfbuf[pfb], pfclo, jo, lane, W);
#endif
            }
            // the next strip's windows: the stager builds them while this strip is walked
            if (b > 0 && a.stager)
            {
                ++reqSeq;
                reqO = jc;
                if (lane == 0)
                {
                    ((volatile int *)req)[1] = b - 1;
                    ((volatile int *)req)[2] = reqO;
                    ((volatile int *)req)[0] = reqSeq;
                }
            }
            // the windows are complete before the prefetch below is issued: otherwise the wait for
            // the staging loads (vmcnt) would also wait for the prefetch
            asm volatile("" : "+v"(W[0]), "+v"(W[1]), "+v"(W[2]), "+v"(W[3]), "+v"(W[4]), "+v"(W[5]), "+v"(W[6]), "+v"(W[7]));
            int pfnext = INT_MIN;
            if (b > 0 && !a.stager)
            {
                // raw planes of the strip above around the predicted entry column -> LDS (without the
                // stager wave; with it, the rare strip it does not cover is staged from global memory)
                const int pred = jc - drift;
                const int clo = max(0, min((pred - 225) >> 5, nchunks - kPfChunks));
                const uint32_t *src = sb - sstride + (int64_t)clo * kChunkDw;
                sfor<kPfChunks / 2>([&](auto Xc) {
                    constexpr int x = decltype(Xc)::value;
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void *)(src + x * 256 + lane * 4),
                        (__attribute__((address_space(3))) void *)(&pfbuf[pfb ^ 1][x * 256]), 16, 0, 0);
                });
                pfnext = clo;
            }
            L.u = u0;
            L.pa = 0;
            L.na = 0;
            L.kk = k;
            L.vrec = 0;
            auto restage = [&]() {
                jo -= 16 * L.na;  // the eight windows are exhausted: the next 128 columns
                L.na = 0;
                L.u = 0;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
                ++nRestage;
#endif
                rw_stage<false>(sb, pfbuf[pfb], INT_MIN, jo, lane, W);
            };
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
            asm volatile("" : "+v"(W[0]));
            const uint64_t c1 = __builtin_amdgcn_s_memtime();
#endif
            walk_batch<false>(L, a.fast != 0, 0, W, restage);
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
            const uint64_t c2 = __builtin_amdgcn_s_memtime();
            tStage += c1 - c0;
            tBatch += c2 - c1;
#endif
            // records of rows k .. kend (record index: rows walked before + k - lane)
            const int kend = L.stopped ? L.stopLane + 1 : 0;
            if (lane >= kend && lane <= k) rec[nrec + k - lane] = (int32_t)L.vrec;
            if constexpr (LOCAL)
            {
                // post this strip to the stager's check (slot chkSeq & 1, free once the stager has
                // taken the check two before); one wave's LDS writes execute in order, so the records
                // and the header are there when the sequence word is
                ++chkSeq;
                // (the stager takes no checks once the walk has ended: stop waiting for the slot then)
                bool over = false, lost = false;
                for (uint32_t spin = 1; uniform(((volatile int *)chkCtl)[1]) < chkSeq - 2; ++spin)
                {
                    if ((over = uniform(((volatile int *)chkCtl)[3]) != 0)) break;
                    if (spin > 16) __builtin_amdgcn_s_sleep(1);
                    // (never: the stager always takes or ends; a bound, not a wait. Exhausted, the slot
                    // is not posted and the pair fails loudly: h.err -> SA_ERR_TIMEOUT)
                    if ((lost = spin > (1u << 26))) break;
                }
                if (lost)
                {
                    h.err = 1;
                    break;
                }
                if (over)
                {
                    nrec += k - kend + 1;
                    break;
                }
                int *slot = chkBuf[chkSeq & 1];
                slot[lane] = (int)L.vrec;
                if (lane == 0)
                {
                    slot[64] = b;
                    slot[65] = k;
                    slot[66] = jc;
                    slot[67] = nrec;
                    slot[68] = h.score;  // (the first check's H at the start cell)
                    ((volatile int *)chkCtl)[0] = chkSeq;
                }
                if (uniform(((volatile int *)chkCtl)[3]) != 0)
                {
                    nrec += k - kend + 1;
                    break;  // the path ended in a strip already checked
                }
            }
            nrec += k - kend + 1;
            if (L.stopped)
            {
                const int iEnd = b * kWave + L.stopLane + 1;  // row of the STOP / border search
                const int f = jo - 16 * L.na - (L.stopPos >> 1);
                h.tail = L.stopRun;
                if (f > 0)
                {
                    h.start_text = f - 1;  // a STOP cell: its indices (the loop exits before moving)
                    h.start_pattern = iEnd - 1;
                }
                else
                {
                    // column 0 reached: the last cell before the border is (iEnd, 1) after a LEFT run,
                    // or (iEnd + 1, 1) when the row was entered at column 0 by a DIAG
                    h.start_text = 0;
                    h.start_pattern = L.stopRun > 0 ? iEnd - 1 : iEnd;
                }
                break;
            }
            jc = jo - 16 * L.na - (L.u >> 1);
            --b;
            k = 63;
            pfb ^= 1;
            pfclo = pfnext;
        }
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
        if (a.timing && lane == 0)
        {
            a.timing[2 * (size_t)gridDim.x + 2 * (size_t)p] = tStage;
            a.timing[2 * (size_t)gridDim.x + 2 * (size_t)p + 1] = tBatch;
            // staging load wait, strips staged from global memory (prefetch missed), strips, restages
            a.timing[4 * (size_t)gridDim.x + 4 * (size_t)p] = sdbg[0] - tLoadStart;
            a.timing[4 * (size_t)gridDim.x + 4 * (size_t)p + 1] = sdbg[1];
            a.timing[4 * (size_t)gridDim.x + 4 * (size_t)p + 2] = nStrips;
            a.timing[4 * (size_t)gridDim.x + 4 * (size_t)p + 3] = nRestage;
            a.timing[8 * (size_t)gridDim.x + (size_t)p] = nStagerHit;
        }
#endif
        if constexpr (!LOCAL)
        {
            h.nrec = nrec;
            if (!L.stopped)
            {
                h.tail = jc;  // row 0: LEFT to column 0 (traceBackNW :80-81)
                h.start_text = 0;
                h.start_pattern = 0;
            }
        }
        else
        {
            // the stager's verdict (the last strip posted is strip 0 at the latest, whose row 1 always
            // ends the walk)
            for (uint32_t spin = 1; h.err == 0 && uniform(((volatile int *)chkCtl)[3]) == 0; ++spin)
            {
                if (spin > 16) __builtin_amdgcn_s_sleep(1);
                // (a bound, never reached: strip 0's check always ends the walk; exhausted, the
                // verdict words were never written and the pair fails loudly instead of reading them)
                if (spin > (1u << 26)) h.err = 1;
            }
            if (h.err == 0)
            {
                h.nrec = ((volatile int *)chkCtl)[4];
                h.tail = ((volatile int *)chkCtl)[5];
                h.start_text = ((volatile int *)chkCtl)[6];
                h.start_pattern = ((volatile int *)chkCtl)[7];
            }
            else
            {
                h.nrec = 0;
                h.tail = 0;
                h.start_text = 0;
                h.start_pattern = 0;
            }
        }
    }
    if (lane == 0)
    {
        ((volatile int *)req)[0] = -1;  // the stager quits (every path of the walker ends here)
        a.heads[p] = h;
        if (a.timing)
        {
            a.timing[2 * (size_t)p] = tW0;
            a.timing[2 * (size_t)p + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

template <bool LOCAL>
__global__ __launch_bounds__(2 * kWave) void walk_rw_kernel(WalkArgs a)
{
    __shared__ RwLds<LOCAL> S;
    const int p = blockIdx.x;
    if (a.tb_pg && uniform(a.tb_pg[p + 1]) > uniform(a.tb_pg[p])) return;  // (the table traceback's pairs)
    walk_rw_pair<LOCAL>(a, p, S);
}

// Column walk (R >= 2): one wave per pair
template <int R, bool LOCAL>
__device__ __forceinline__ void walk_cw_pair(const WalkArgs &a, const int p, uint32_t *cwbuf);

// (np pairs; a grid smaller than np walks them in turn: WalkArgs::cap, the pipelined batch's
// traceback beside the next fill)
template <int R, bool LOCAL>
__global__ __launch_bounds__(64) void walk_cw_kernel(WalkArgs a, int np)
{
    __shared__ uint32_t cwbuf[R == 32 ? 2 * kCwDw : 1];
    for (int p = blockIdx.x; p < np; p += gridDim.x) walk_cw_pair<R, LOCAL>(a, p, cwbuf);
}

template <int R, bool LOCAL>
__device__ __forceinline__ void walk_cw_pair(const WalkArgs &a, const int p, uint32_t *cwbuf)
{
    const int lane = threadIdx.x;
    PairDesc pd = a.pairs[p];
    const int n = uniform((int)pd.text_len), m = uniform((int)pd.pattern_len);
    const int first = uniform(pd.first_strip), nstrips = uniform(pd.num_strips);
    int32_t *rec = a.rec + uniform64(pd.rec_off);
    const uint64_t tW0 = a.timing ? __builtin_amdgcn_s_memrealtime() : 0;
    TbHead h;
    int i, j;
    if (walk_start<LOCAL>(a, p, n, m, first, nstrips, lane, h, i, j))
    {
        h.kind = kRecCols;
        h.tail_op = kTop;
        StripDesc sd = a.strips[first];
        const int nsteps = uniform(sd.nsteps);
        const uint32_t *mb = a.masks + uniform64(sd.mask_off) * 4;
        const int64_t sstride = (int64_t)nsteps * R * 4;  // dwords per strip (nsteps * R slots of 16 B)
        int G0 = (i - 1) >> 4;                            // block of the current row
        int J0 = j;                                       // lane 63 = column J0
        int nrec = 0;
        Lines L;
        L.u = 2 * (16 * G0 + 16 - i);
        // R = 32 single-strip pairs: staging from the LDS copy issued one batch ahead
        const bool useLds = R == 32 && nstrips == 1;
        const int nchunks = (nsteps * R) / Geo<R>::CS;
        const int drift = (int)(((int64_t)m * 64 + n / 2) / max(n, 1) / 16);  // row blocks per batch
        int pfb = 0, pfclo = -1, pfklo = 0, pfJ0 = INT_MIN;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
        uint64_t tStage = 0, tBatch = 0;
#endif
        while (J0 >= 1)
        {
            uint32_t W[8];
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
            const uint64_t c0 = __builtin_amdgcn_s_memtime();
#endif
            bool fromLds = false;
            if constexpr (R == 32)
            {
                // the copy for this batch has landed (the previous batch's record store, issued after
                // it, may still be in flight)
                asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                const int kHi = max(G0, 0) >> 1, kLo = max(G0 - 7, 0) >> 1;
                fromLds = useLds && pfJ0 == J0 && kLo >= pfklo && kHi < pfklo + kCwLanes;
                if (fromLds) cw_stage_lds<LOCAL>(cwbuf + pfb * kCwDw, pfclo, pfklo, J0, G0, lane, W);
            }
            if (!fromLds) cw_stage<R, LOCAL>(mb, sstride, J0, G0, lane, W);
            // the windows are complete before the next prefetch is issued (its wait must not cover them)
            asm volatile("" : "+v"(W[0]), "+v"(W[1]), "+v"(W[2]), "+v"(W[3]), "+v"(W[4]), "+v"(W[5]), "+v"(W[6]), "+v"(W[7]));
            if constexpr (R == 32)
                if (useLds && J0 > 64)
                {
                    pfb ^= 1;
                    pfklo = cw_klo(G0, drift);
                    pfJ0 = J0 - 64;
                    cw_prefetch(mb, nchunks, pfJ0, pfklo, lane, cwbuf + pfb * kCwDw, pfclo);
                }
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
            asm volatile("" : "+v"(W[0]), "+v"(W[7]));
            const uint64_t c1 = __builtin_amdgcn_s_memtime();
#endif
            const int kmin = max(0, 64 - J0);  // lanes of columns >= 1
            L.pa = 0;
            L.na = 0;
            L.kk = 63;
            L.vrec = 0;
            auto restage = [&]() {
                G0 -= L.na;  // the eight blocks are exhausted: the next eight above
                L.na = 0;
                L.u = 0;
                cw_stage<R, LOCAL>(mb, sstride, J0, G0, lane, W);
            };
            walk_batch<LOCAL>(L, a.fast != 0, kmin, W, restage);
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
            const uint64_t c2 = __builtin_amdgcn_s_memtime();
            tStage += c1 - c0;
            tBatch += c2 - c1;
#endif
            const int kend = L.stopped ? L.stopLane + 1 : kmin;
            if (lane >= kend) rec[nrec + 63 - lane] = (int32_t)L.vrec;
            nrec += 64 - kend;
            G0 -= L.na;
            if (L.stopped)
            {
                const int jEnd = J0 - 63 + L.stopLane;           // column of the STOP / border search
                const int f = 16 * G0 + 16 - (L.stopPos >> 1);   // row of the found cell
                h.tail = L.stopRun;
                if (f > 0)
                {
                    h.start_text = jEnd - 1;  // a STOP cell
                    h.start_pattern = f - 1;
                }
                else
                {
                    // row 0 reached: the last cell before the border is (1, jEnd) after a TOP run, or
                    // (1, jEnd + 1) when the column was entered at row 0 by a DIAG
                    h.start_text = L.stopRun > 0 ? jEnd - 1 : jEnd;
                    h.start_pattern = 0;
                }
                break;
            }
            J0 -= 64;
        }
        h.nrec = nrec;
#if defined(SA_EXPERIMENT) && defined(SA_EXP_WALK_TIMING)
        if (a.timing && lane == 0)
        {
            a.timing[2 * (size_t)gridDim.x + 2 * (size_t)p] = tStage;
            a.timing[2 * (size_t)gridDim.x + 2 * (size_t)p + 1] = tBatch;
        }
#endif
        if (!L.stopped)
        {
            const int icur = 16 * G0 + 16 - (L.u >> 1);  // row after the move into column 0 (0: row 0)
            if constexpr (!LOCAL)
            {
                h.tail = icur;  // column 0: TOP to row 0 (traceBackNW :78-79)
                h.start_text = 0;
                h.start_pattern = 0;
            }
            else
            {
                // column 0 reached from column 1, whose leaving cell is row icur + DIAG
                h.start_text = 0;
                h.start_pattern = icur + (L.lastp & 1) - 1;
            }
        }
    }
    if (lane == 0)
    {
        a.heads[p] = h;
        if (a.timing)
        {
            a.timing[2 * (size_t)p] = tW0;
            a.timing[2 * (size_t)p + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// table traceback (R = 1 global; sa_walk.h TbArgs)
// ------------------------------------------------------------------------------------------------
constexpr int kTbMargin = 320;                               // columns staged left of a window
constexpr int kTbChunks = (kTbK + 63 + kTbMargin) / 32 + 2;  // R = 1 chunks (32 slots) staged per strip
constexpr int kTbRow = kTbChunks + 2;                        // LDS dwords per strip row and mask (a zero word first)
constexpr int kTbNz = (kTbChunks + 31) / 32;                 // dwords of a row's nonzero-word mask

typedef __attribute__((address_space(3))) const uint32_t tb_lds_u32;

// 16 slots of a raw word -> 16 bits, slot s at bit s: the even bits 30 - 2s of y
__device__ __forceinline__ uint32_t tb_slots16(uint32_t y)
{
    y &= 0x55555555u;
    y = (y | (y >> 1)) & 0x33333333u;
    y = (y | (y >> 2)) & 0x0F0F0F0Fu;
    y = (y | (y >> 4)) & 0x00FF00FFu;
    y = (y | (y >> 8)) & 0x0000FFFFu;
    return __builtin_bitreverse32(y) >> 16;
}

// One row of traceBackNW (alignSequenceCPU.cpp:64-114) for a chain entering strip row k at column
// x >= 1: LEFT while the cell is LEFT, then TOP or DIAG out of the row; column 0 is TOP (:78-79). The
// staged masks nl / dg hold per strip row one bit per slot (R = 1 slot e = x - 1 + k of column x at bit
// e % 32 of word 1 + e / 32 - clo; word 0 is zero; not LEFT / DIAG); the nearest set nl bit at or
// below the entry's is the cell the row leaves from. The LEFT runs tb_step's probe does not cover: the
// entry's word, then the nearest nonzero word below it from the row's nonzero-word mask nz; -1
// (unknown: the table entry invalid, so a path through it falls back to the sequential walk) when the
// entry or the run leaves the staged chunks.
__device__ __noinline__ int tb_row_slow(int x, int k, tb_lds_u32 *nl, tb_lds_u32 *dg, tb_lds_u32 *nz, int clo, int nch)
{
    const int e = x - 1 + k;
    int i = (e >> 5) - clo;
    if ((unsigned)i >= (unsigned)nch) return -1;
    uint32_t w = nl[k * kTbRow + 1 + i] & (0xffffffffu >> (31 - (e & 31)));
    if (!w)
    {
        // the highest staged word below i with a set bit
        int j = -1;
        for (int q = (i - 1) >> 5; q >= 0 && j < 0 && i > 0; --q)
        {
            uint32_t z = nz[k * kTbNz + q];
            if (q == (i - 1) >> 5) z &= 0xffffffffu >> (31 - ((i - 1) & 31));
            if (z) j = 32 * q + 31 - __builtin_clz(z);
        }
        if (j < 0) return clo * 32 <= k ? 0 : -1;  // none: column 0 if the staged slots reach it
        i = j;
        w = nl[k * kTbRow + 1 + i];
    }
    const int pos = 31 - __builtin_clz(w);
    const int col = (i + clo) * 32 + pos + 1 - k;
    return col <= 0 ? 0 : col - (int)((dg[k * kTbRow + 1 + i] >> pos) & 1u);
}

// One row for a chain at column x (0: column 0, which stays there; -1: unknown, stays unknown). The
// entry's word and the one below it (64 slots as one 64-bit word) cover the 33 .. 64 slots at and left
// of the entry; a longer LEFT run, or an entry outside the staged chunks, goes through tb_row_slow.
__device__ __forceinline__ int tb_step(int x, int k, tb_lds_u32 *nl, tb_lds_u32 *dg, tb_lds_u32 *nz, int clo, int nch)
{
    const int e = x - 1 + k, i = (e >> 5) - clo, bit = e & 31;
    const bool in = x > 0 && (unsigned)i < (unsigned)nch;
    const int a = k * kTbRow + 1 + (in ? i : 0);
    const uint64_t W = ((uint64_t)(nl[a] & (0xffffffffu >> (31 - bit))) << 32) | nl[a - 1];
    const uint64_t G = ((uint64_t)dg[a] << 32) | dg[a - 1];
    const int pos = 63 - __builtin_clzll(W | 1);
    const int col = e - bit - 32 + pos + 1 - k;
    const int d = (int)((G >> pos) & 1u);
    // nothing found: column 0 when the two words reach it (word 0 is real only when clo is 0)
    const bool reach = (i >= 1 || clo == 0) && e - bit - 32 <= k;
    int r = W ? (col <= 0 ? 0 : col - d) : (reach ? 0 : -2);
    if (!in) r = x > 0 ? -2 : x;
    return r != -2 ? r : tb_row_slow(x, k, nl, dg, nz, clo, nch);
}

// Compaction of the distinct chains (tb_table_kernel): chains that met stay equal, and each run of
// equal values in cur[0 .. D) becomes one chain (values of different runs may repeat: they stay apart,
// which costs work, not correctness); map[] (start column -> chain) follows. Thread t holds elements
// E t .. E t + E - 1. Returns the new D.
template <int E>
__device__ __forceinline__ int tb_compact(int *cur, uint16_t *map, uint16_t *tmp, int *wsum, int D)
{
    const int t = threadIdx.x, i0 = E * t;
    int v[E], fl[E];
    int prev = i0 > 0 && i0 < D ? cur[i0 - 1] : 0, f = 0;
    for (int q = 0; q < E; ++q)
    {
        v[q] = i0 + q < D ? cur[i0 + q] : 0;
        fl[q] = i0 + q < D && (i0 + q == 0 || v[q] != prev);
        prev = v[q];
        f += fl[q];
    }
    const int inc = wave_prefix_sum(f);
    const int wv = t / kWave;
    if ((t & (kWave - 1)) == kWave - 1) wsum[wv] = inc;
    __syncthreads();
    int before = 0, total = 0;
    for (int k = 0; k < (int)(blockDim.x / kWave); ++k)
    {
        const int x = wsum[k];
        before += k < wv ? x : 0;
        total += x;
    }
    int nidx[E];
    int c = before + inc - f - 1;  // new chain of the element before i0
    for (int q = 0; q < E; ++q)
    {
        c += fl[q];
        nidx[q] = c;
        if (i0 + q < D) tmp[i0 + q] = (uint16_t)c;
    }
    __syncthreads();  // (every read of cur and wsum is done)
    for (int q = 0; q < E; ++q)
        if (fl[q]) cur[nidx[q]] = v[q];
    for (int e = t; e < kTbK; e += blockDim.x) map[e] = tmp[map[e]];
    __syncthreads();
    return total;
}

// The start cell of pair p (global: (m, n); local: the best cell, from the strips' keys as walk_start)
// and its H, by one wave; false for a local pair without a positive cell (its empty alignment: the
// sequential walk)
__device__ __forceinline__ bool tb_pair_start(const TbArgs &a, int p, const PairDesc &pd, int lane, int &i, int &j, int &H)
{
    i = (int)pd.pattern_len;
    j = (int)pd.text_len;
    if (!a.local)
    {
        H = a.pair_score[p];
        return true;
    }
    const int first = uniform(pd.first_strip), nstrips = uniform(pd.num_strips);
    uint64_t k = 0;
    for (int s = lane; s < nstrips; s += kWave) k = max(k, a.strip_best[first + s]);
    k = wave_max_u64(k);
    const int rb = a.key_rowbits;
    const uint64_t km = (1ull << rb) - 1;
    H = (int)(k >> (2 * rb));
    i = (int)(km - ((k >> rb) & km));
    j = (int)(km - (k & km));
    return H > 0;
}

// Strip tables: block = one strip, 1024 threads, the kTbK start columns of the strip's window; the
// strip's planes around the window staged in LDS as per-row masks (not LEFT, DIAG); rows from the
// strip's last down to its first. Chains that meet stay merged, so after 4 and after 16 rows the
// distinct ones are compacted (2048 -> ~500 -> ~230 at 32768^2 random DNA) and only those walk on.
constexpr int kTbPhases = 3;
// T threads per strip: 512 lets two strips share a CU (plans with more strips than CUs); 1024 when
// every strip has a CU of its own, where a block's serial work is the kernel's time (the first
// phase's 2048 chains at two per thread instead of four, the staging at twice the loads in flight)
template <int T>
__global__ __launch_bounds__(T) void tb_table_kernel(TbArgs a)
{
    __shared__ uint32_t nlm[kWave * kTbRow], dgm[kWave * kTbRow], nzm[kWave * kTbNz];
    __shared__ int cur[kTbK];
    __shared__ uint16_t map[kTbK], tmp[kTbK];
    __shared__ int wsum[16];
    __shared__ int sst[4];
    const int s = blockIdx.x;
    const StripDesc sd = a.strips[s];
    const int p = uniform(sd.pair);
    if (uniform(a.pair_g0[p + 1]) == uniform(a.pair_g0[p])) return;  // (a pair without groups: walk_rw_kernel's)
    const PairDesc pd = a.pairs[p];
    const int n = uniform((int)pd.text_len);
    const int b = s - uniform(pd.first_strip);
    int32_t *st = a.start + kTbStartWords * p;
    int i0, ra, xa, dr, dx;
    if (a.round == 1)
    {
        // every block finds the start cell itself; strip 0's block records it (TbStart), the pair's
        // state (tb_flag 2: pending, 1: the sequential walk) and the local end strip
        if (threadIdx.x < kWave)
        {
            int i, j, H;
            const bool ok = tb_pair_start(a, p, pd, threadIdx.x, i, j, H);
            if (threadIdx.x == 0)
            {
                sst[0] = i;
                sst[1] = j;
                sst[3] = ok;
                if (b == 0)
                {
                    a.tb_flag[p] = ok ? 2 : 1;
                    st[kTbI0] = i;
                    st[kTbJ0] = j;
                    st[kTbH] = H;
                    st[kTbBs] = (i - 1) >> 6;
                    st[kTbRa] = i;  // the first round's line: through (m, n) and (0, 0) / slope 1 from the best cell
                    st[kTbXa] = j;
                    st[kTbDr] = a.local ? 1 : i;
                    st[kTbDx] = a.local ? 1 : j;
                    st[kTbGres] = -1;
                    st[kTbBmin] = 0;
                    a.pend[p] = -1;
                }
            }
        }
        __syncthreads();
        if (!sst[3]) return;
        i0 = ra = sst[0];
        xa = sst[1];
        dr = a.local ? 1 : i0;
        dx = a.local ? 1 : xa;
    }
    else
    {
        if (uniform(a.tb_flag[p]) != 2) return;  // (resolved or fallen back)
        i0 = uniform(st[kTbI0]);
        ra = uniform(st[kTbRa]);
        xa = uniform(st[kTbXa]);
        dr = uniform(st[kTbDr]);
        dx = uniform(st[kTbDx]);
    }
    const int bs = (i0 - 1) >> 6;
    if (b > (ra - 1) >> 6) return;  // (below the anchor: resolved, or below the start cell)
    const int kTop = b == bs ? (i0 - 1) & 63 : 63;
    const int lo = tb_window_lo(b, n, i0, ra, xa, dr, dx);
    if (threadIdx.x == 0) a.win[s] = lo;
    if (a.dbg && threadIdx.x == 0) a.dbg[12 * (size_t)s] = __builtin_amdgcn_s_memrealtime();
    const uint32_t *sb = a.masks + uniform64(sd.mask_off) * 4;
    const int clo = max(0, (lo - 1 - kTbMargin) >> 5);
    const int nch = max(0, min(kTbChunks, (uniform(sd.nsteps) >> 5) - clo));
    if (threadIdx.x < kWave)
    {
        nlm[threadIdx.x * kTbRow] = dgm[threadIdx.x * kTbRow] = 0;
        for (int q = 0; q < kTbNz; ++q) nzm[threadIdx.x * kTbNz + q] = 0;
    }
    __syncthreads();
    constexpr int kStageBatch = 4;  // raw loads in flight per thread
    for (int e0 = threadIdx.x; e0 < nch * kWave; e0 += kStageBatch * blockDim.x)
    {
        u32x2 v[kStageBatch];
        for (int u = 0; u < kStageBatch; ++u)
        {
            const int e = e0 + u * blockDim.x;  // chunk e / 64, strip lane e % 64: its two raw words
            v[u] = e < nch * kWave ? *reinterpret_cast<const u32x2 *>(sb + ((int64_t)clo + e / kWave) * kChunkDw + 2 * (e % kWave))
                                   : u32x2{0u, 0u};
        }
        for (int u = 0; u < kStageBatch; ++u)
        {
            const int e = e0 + u * blockDim.x, q = e / kWave, k = e % kWave;
            if (e >= nch * kWave) break;
            const uint32_t nlw = tb_slots16(v[u].x | (v[u].x >> 1)) | (tb_slots16(v[u].y | (v[u].y >> 1)) << 16);
            nlm[k * kTbRow + 1 + q] = nlw;
            dgm[k * kTbRow + 1 + q] = tb_slots16(v[u].x >> 1) | (tb_slots16(v[u].y >> 1) << 16);
            if (nlw) atomicOr(&nzm[k * kTbNz + (q >> 5)], 1u << (q & 31));
        }
    }
    for (int t = threadIdx.x; t < kTbK; t += blockDim.x)
    {
        cur[t] = lo + t <= n ? lo + t : 0;  // (start columns past n: any chain, masked at the end)
        map[t] = (uint16_t)t;
    }
    __syncthreads();
    tb_lds_u32 *nl = (tb_lds_u32 *)nlm;
    tb_lds_u32 *dg = (tb_lds_u32 *)dgm;
    tb_lds_u32 *nz = (tb_lds_u32 *)nzm;
    uint64_t stamp[12] = {};
    const bool dbg = a.dbg != nullptr;
    if (dbg) stamp[0] = __builtin_amdgcn_s_memrealtime();
    constexpr int kRowsBefore[kTbPhases] = {4, 16, 64};  // rows walked before each compaction
    int D = kTbK, k = kTop;
    for (int ph = 0; ph < kTbPhases; ++ph)
    {
        const int kEnd = max(-1, kTop - kRowsBefore[ph]);
        for (int t = threadIdx.x; t < D; t += blockDim.x)
        {
            int x = cur[t];
            for (int kk = k; kk > kEnd; --kk) x = tb_step(x, kk, nl, dg, nz, clo, nch);
            cur[t] = x;
        }
        k = kEnd;
        __syncthreads();
        if (dbg) stamp[1 + 3 * ph] = __builtin_amdgcn_s_memrealtime();
        if (k < 0) break;
        D = tb_compact<kTbK / T>(cur, map, tmp, wsum, D);
        if (dbg)
        {
            stamp[2 + 3 * ph] = __builtin_amdgcn_s_memrealtime();
            stamp[3 + 3 * ph] = (uint64_t)D;
        }
    }
    // (the pair's first group starts at its first strip: table slots are per pair with groups)
    int32_t *out = a.tbl + (int64_t)(uniform(a.groups[uniform(a.pair_g0[p])].tbl0) + b) * kTbK;
    for (int t = threadIdx.x; t < kTbK; t += blockDim.x) out[t] = lo + t <= n ? cur[map[t]] : -1;
    if (dbg && threadIdx.x == 0)
    {
        stamp[10] = __builtin_amdgcn_s_memrealtime();
        stamp[11] = a.dbg[12 * (size_t)s];  // (the kernel entry stamp, written at the start)
        for (int e = 0; e < 12; ++e) a.dbg[12 * (size_t)s + e] = stamp[e];
    }
}

// Copies tables t0 .. t0 + nt - 1 (kTbK int32 each) of src into LDS (all threads of the block)
__device__ __forceinline__ void tb_stage_tables(int32_t *dst, const int32_t *src, int64_t t0, int nt)
{
    const int4 *s4 = reinterpret_cast<const int4 *>(src + t0 * kTbK);
    int4 *d4 = reinterpret_cast<int4 *>(dst);
    for (int e = threadIdx.x; e < nt * (kTbK / 4); e += blockDim.x) d4[e] = s4[e];
}

// The group's strips walked from the start: s_lo .. min(s_hi, the start cell's strip); false if none
__device__ __forceinline__ bool tb_group_span(const TbArgs &a, const TbGroup &g, const PairDesc &pd, int &sLo, int &sHi)
{
    sLo = uniform(g.s_lo);
    sHi = min(uniform(g.s_hi), uniform(pd.first_strip) + uniform(a.start[kTbStartWords * uniform(g.pair) + kTbBs]));
    return sHi >= sLo;
}

// Group tables: the strip tables of the group (staged in LDS) chained from its first walked strip to
// its last, per start column of the first strip's window (-1 once a column leaves a window)
__global__ __launch_bounds__(1024) void tb_compose_kernel(TbArgs a)
{
    __shared__ int32_t tl[kTbG * kTbK];
    __shared__ int wl[kTbG];
    const TbGroup g = a.groups[blockIdx.x];
    if (uniform(a.tb_flag[uniform(g.pair)]) != 2) return;
    const int gres = uniform(a.start[kTbStartWords * uniform(g.pair) + kTbGres]);
    if (gres >= 0 && (int)blockIdx.x > gres) return;  // (resolved in an earlier round)
    const PairDesc pd = a.pairs[uniform(g.pair)];
    int sLo, sHi;
    if (!tb_group_span(a, g, pd, sLo, sHi)) return;
    const int n = uniform((int)pd.text_len);
    tb_stage_tables(tl, a.tbl, uniform(g.tbl0) + sLo - uniform(g.s_lo), sHi - sLo + 1);
    if (threadIdx.x <= sHi - sLo) wl[threadIdx.x] = a.win[sLo + threadIdx.x];
    __syncthreads();
    const int loHi = wl[sHi - sLo];
    for (int t = threadIdx.x; t < kTbK; t += blockDim.x)
    {
        int x = loHi + t <= n ? loHi + t : -1;
        for (int s = sHi; s >= sLo && x >= 0; --s)
        {
            const int lo = wl[s - sLo];
            x = (x >= lo && x < lo + kTbK) ? tl[(s - sLo) * kTbK + x - lo] : -1;
        }
        a.gtbl[(int64_t)blockIdx.x * kTbK + t] = x;
    }
}

// One block per pair (pending): the group tables chained from the anchor's group upward (staged in LDS
// kTbG at a time) give every group's entry column and the row-0 column; global: the pair's head (the
// trailing LEFT run). A column outside a window at group g: the next round anchors at g's entry
// (TbStart), unless this is the last round or g was the round's first group (no progress): then
// tb_flag = 1 and walk_rw_kernel walks the pair instead.
__global__ __launch_bounds__(1024) void tb_resolve_kernel(TbArgs a)
{
    __shared__ int32_t tl[kTbG * kTbK];
    __shared__ int glo[kTbG];
    __shared__ int xs, gfail, xfail;
    const int p = blockIdx.x;
    // (tb_flag is defined only for pairs with groups: tb_table_kernel writes it)
    if (uniform(a.pair_g0[p + 1]) == uniform(a.pair_g0[p]) || uniform(a.tb_flag[p]) != 2) return;
    const int g0 = uniform(a.pair_g0[p]);
    const PairDesc pd = a.pairs[p];
    const int first = uniform(pd.first_strip);
    int32_t *st = a.start + kTbStartWords * p;
    const int i0 = uniform(st[kTbI0]), bs = uniform(st[kTbBs]);
    // the start cell's group, and the round's first group: the anchor's, or the start cell's
    const int gstart = g0 + bs / kTbG;  // (a pair's groups are its strips kTbG at a time from strip 0)
    const int gs = uniform(st[kTbGres]) >= 0 ? uniform(st[kTbGres]) : gstart;
    if (threadIdx.x == 0)
    {
        xs = st[kTbXa];
        gfail = -1;
    }
    for (int gh = gs + 1; gh > g0; gh -= kTbG)
    {
        const int gl = max(g0, gh - kTbG);
        __syncthreads();  // (the previous chunk's lookups are done)
        if (uniform(gfail) >= 0) break;
        tb_stage_tables(tl, a.gtbl, gl, gh - gl);
        if (threadIdx.x < gh - gl) glo[threadIdx.x] = a.win[min(a.groups[gl + threadIdx.x].s_hi, first + bs)];
        __syncthreads();
        if (threadIdx.x == 0)
        {
            int x = xs;
            for (int g = gh - 1; g >= gl; --g)
            {
                const int lo = glo[g - gl];
                const int y = (x >= lo && x < lo + kTbK) ? tl[(g - gl) * kTbK + x - lo] : -1;
                if (y < 0)
                {
                    gfail = g;  // the path's entry into group g is x; it leaves a window at or in g
                    xfail = x;
                    break;
                }
                a.gent[g] = x;
                x = y;
            }
            xs = x;
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (gfail >= 0)
    {
        if (a.last_round || gfail == gs)
        {
            // local: groups gfail + 1 .. gstart are resolved, and the walk may end in them
            const bool keep = a.local && gfail < gstart;
            a.tb_flag[p] = keep ? 0 : 1;
            if (keep) st[kTbBmin] = a.groups[gfail + 1].s_lo - first;
            return;
        }
        // the next round: anchor at group gfail's entry (its first walked row)
        const int r = min(64 * (min(a.groups[gfail].s_hi, first + bs) - first) + 64, i0);
        st[kTbRa] = r;
        st[kTbXa] = xfail;
        if (a.local)
        {
            st[kTbDr] = i0 - r;  // (> 0: the chain progressed past the start cell's group)
            st[kTbDx] = st[kTbJ0] - xfail;
        }
        else
        {
            st[kTbDr] = r;
            st[kTbDx] = xfail;
        }
        st[kTbGres] = gfail;
        return;
    }
    a.tb_flag[p] = 0;
    if (a.local) return;  // (the head: tb_finish_kernel)
    TbHead h;
    h.kind = kRecRows;
    h.tail_op = kLeft;
    h.tail = xs;  // row 0: LEFT to column 0 (traceBackNW :80-81)
    h.nrec = (int)pd.pattern_len;
    h.err = 0;
    h.score = st[kTbH];
    h.i0 = (int)pd.pattern_len;
    h.j0 = (int)pd.text_len;
    h.start_text = 0;
    h.start_pattern = 0;
    a.heads[p] = h;
}

// One block per group: thread 0 chains the group's strip tables (staged in LDS) from the group's entry
// column (each strip's entry), then wave w walks strip sHi - w from its entry with the row walk's
// staging and unrolled batch and writes its rows' records (record of row i at index i0 - i); local:
// the strip's entry column and the sum of its H steps (local_check's, see rw_stager_local)
// FIN (global): np more blocks after the groups' are tb_finish_kernel<false>'s, block ngroups + p the
// sequential walk of pair p if the tables left it (one launch less: they run beside the walk blocks,
// whose pairs the tables resolved, so they touch none of the same pairs)
template <bool FIN>
__global__ __launch_bounds__(kTbG * kWave) void tb_walk_kernel(TbArgs a, WalkArgs wa)
{
    __shared__ int32_t tl[kTbG * kTbK];
    __shared__ int ent[kTbG], wlo[kTbG];
    if constexpr (FIN)
    {
        static_assert(sizeof(RwLds<false>) <= sizeof(tl), "the finish block's LDS lives in the tables' place");
        if ((int)blockIdx.x >= a.ngroups)
        {
            const int p = (int)blockIdx.x - a.ngroups;
            if (uniform(a.pair_g0[p + 1]) == uniform(a.pair_g0[p])) return;  // (walk_rw_kernel's)
            if (uniform(a.tb_flag[p]) == 0 || a.strict) return;  // (tb_resolve_kernel wrote the head)
            walk_rw_pair<false>(wa, p, *reinterpret_cast<RwLds<false> *>(tl));
            return;
        }
    }
    (void)wa;
    const TbGroup g = a.groups[blockIdx.x];
    const int p = uniform(g.pair);
    if (uniform(a.tb_flag[p]) != 0) return;
    const PairDesc pd = a.pairs[p];
    int sLo, sHi;
    if (!tb_group_span(a, g, pd, sLo, sHi)) return;
    const int first = uniform(pd.first_strip);
    const int i0 = uniform(a.start[kTbStartWords * p + kTbI0]), bs = uniform(a.start[kTbStartWords * p + kTbBs]);
    if (sLo < first + uniform(a.start[kTbStartWords * p + kTbBmin])) return;  // (local: not resolved)
    tb_stage_tables(tl, a.tbl, uniform(g.tbl0) + sLo - uniform(g.s_lo), sHi - sLo + 1);
    if (threadIdx.x <= sHi - sLo) wlo[threadIdx.x] = a.win[sLo + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0)
    {
        int x = a.gent[blockIdx.x];
        for (int s = sHi; s >= sLo; --s)
        {
            ent[sHi - s] = x;
            x = tl[(s - sLo) * kTbK + x - wlo[s - sLo]];
        }
    }
    __syncthreads();
    const int w = uniform((int)(threadIdx.x / kWave)), lane = threadIdx.x & (kWave - 1);
    const int s = sHi - w;
    if (s < sLo) return;
    const int b = s - first;
    const int kTop = b == bs ? (i0 - 1) & 63 : 63;
    const StripDesc sd = a.strips[s];
    const uint32_t *sb = a.masks + uniform64(sd.mask_off) * 4;
    const int jc = uniform(ent[w]);
    int jo = jc;
    uint32_t W[8];
    rw_stage<false>(sb, sb, INT_MIN, jo, lane, W);
    Lines L;
    L.kk = kTop;
    auto restage = [&]() {
        jo -= 16 * L.na;  // the eight windows are exhausted: the next 128 columns
        L.na = 0;
        L.u = 0;
        rw_stage<false>(sb, sb, INT_MIN, jo, lane, W);
    };
    walk_batch<false>(L, a.fast != 0, 0, W, restage);
    if (lane <= kTop) a.rec[uniform64(pd.rec_off) + (i0 - 1 - 64 * b - lane)] = (int32_t)L.vrec;
    if (!a.local) return;
    // the strip's H steps: a row entered at H adds g per LEFT cell, its leaving TOP adds g, its leaving
    // DIAG subtracts S of its cell (the letters gathered from the inputs)
    const int pv = (int)L.vrec;
    const int run = lane <= kTop ? pv >> 1 : 0, dg = lane <= kTop ? pv & 1 : 0;
    const int P = wave_prefix_sum(run + dg);
    const int ce = jc - (__builtin_amdgcn_readlane(P, kTop) - P), lv = ce - run;
    const int pl = lane <= kTop ? (int)a.pattern[pd.pattern_off + 64 * b + lane] : 0;
    const int tl2 = lane <= kTop && dg && lv >= 1 ? (int)a.text[pd.text_off + lv - 1] : 0;
    const int S = dg ? a.score_tab[pl * a.A + tl2] - a.gap : 0;  // (the table holds S + g)
    const int delta = lane <= kTop ? a.gap * run + (dg ? -S : a.gap) : 0;
    const int tot = __builtin_amdgcn_readlane(wave_prefix_sum(delta), kWave - 1);
    if (lane == 0)
    {
        a.sent[s] = jc;
        a.sdelta[s] = tot;
    }
}

// Local, one wave per strip walked: H at the strip's entry (the start cell's H plus the sums of the
// strips walked before it), then local_strip_end on the strip's records (as rw_stager_local); a strip
// where the walk ends writes its head fields and raises the pair's end strip to it
__global__ __launch_bounds__(kWave) void tb_check_kernel(TbArgs a)
{
    const int s = blockIdx.x, lane = threadIdx.x;
    const StripDesc sd = a.strips[s];
    const int p = uniform(sd.pair);
    if (uniform(a.pair_g0[p + 1]) == uniform(a.pair_g0[p]) || uniform(a.tb_flag[p]) != 0) return;
    const PairDesc pd = a.pairs[p];
    const int first = uniform(pd.first_strip);
    const int i0 = uniform(a.start[kTbStartWords * p + kTbI0]), bs = uniform(a.start[kTbStartWords * p + kTbBs]);
    const int b = s - first;
    if (b > bs || b < uniform(a.start[kTbStartWords * p + kTbBmin])) return;  // (not walked / not resolved)
    int hsum = 0;
    for (int q = b + 1 + lane; q <= bs; q += kWave) hsum += a.sdelta[first + q];
    const int Hc = uniform(a.start[kTbStartWords * p + kTbH]) + __builtin_amdgcn_readlane(wave_prefix_sum(hsum), kWave - 1);
    const int kTop = b == bs ? (i0 - 1) & 63 : 63;
    const int jc = uniform(a.sent[s]);
    const int cn0 = i0 - (64 * b + kTop + 1);
    const int pv = lane <= kTop ? a.rec[uniform64(pd.rec_off) + (i0 - 1 - 64 * b - lane)] : 0;
    const int run = lane <= kTop ? pv >> 1 : 0, dg = lane <= kTop ? pv & 1 : 0;
    const int P = wave_prefix_sum(run + dg);
    const int ce = jc - (__builtin_amdgcn_readlane(P, kTop) - P), lv = ce - run;
    const int pl = lane <= kTop ? (int)a.pattern[pd.pattern_off + 64 * b + lane] : 0;
    const int tl2 = lane <= kTop && dg && lv >= 1 ? (int)a.text[pd.text_off + lv - 1] : 0;
    const int S = dg ? a.score_tab[pl * a.A + tl2] - a.gap : 0;
    const int delta = lane <= kTop ? a.gap * run + (dg ? -S : a.gap) : 0;
    const int Pd = wave_prefix_sum(delta);
    const int tot = __builtin_amdgcn_readlane(Pd, kTop);
    const int He = Hc + (tot - Pd);  // H at this lane's row entry
    int nrec, tail, st, sp0;
    if (!local_strip_end(He, run, dg, ce, lv, b, kTop, cn0, a.gap, lane, nrec, tail, st, sp0)) return;
    if (lane != 0) return;
    a.send[4 * s] = nrec;
    a.send[4 * s + 1] = tail;
    a.send[4 * s + 2] = st;
    a.send[4 * s + 3] = sp0;
    atomicMax(&a.pend[p], b);
}

// One block of two waves per pair with groups, last: local, the head from the end strip (the highest
// strip with an end: the first in walk order); then the pairs the tables left (tb_flag 1, or a local
// walk without an end among the resolved strips) are walked sequentially (walk_rw_pair)
template <bool LOCAL>
__global__ __launch_bounds__(2 * kWave) void tb_finish_kernel(TbArgs a, WalkArgs w)
{
    __shared__ RwLds<LOCAL> S;
    const int p = blockIdx.x;
    if (uniform(a.pair_g0[p + 1]) == uniform(a.pair_g0[p])) return;  // (walk_rw_kernel's)
    int flag = uniform(a.tb_flag[p]);
    if (LOCAL && flag == 0)
    {
        const int b = uniform(a.pend[p]);
        if (b >= 0)
        {
            if (threadIdx.x == 0)
            {
                const int s = a.pairs[p].first_strip + b;
                const int32_t *st = a.start + kTbStartWords * p;
                TbHead h;
                h.kind = kRecRows;
                h.tail_op = kLeft;
                h.nrec = a.send[4 * s];
                h.tail = a.send[4 * s + 1];
                h.start_text = a.send[4 * s + 2];
                h.start_pattern = a.send[4 * s + 3];
                h.err = 0;
                h.score = st[kTbH];
                h.i0 = st[kTbI0];
                h.j0 = st[kTbJ0];
                a.heads[p] = h;
            }
            return;
        }
        flag = 1;
    }
    if (flag == 0 || a.strict) return;  // (global: tb_resolve_kernel wrote the head)
    walk_rw_pair<LOCAL>(w, p, S);
}

// ------------------------------------------------------------------------------------------------
// expansion: records -> aligned strings (forward order) and the per-pair result
// ------------------------------------------------------------------------------------------------
// Grid (chunks, pairs): block c of a pair expands records [c * chunk_recs, (c+1) * chunk_recs), so a
// single long pair spreads over up to kMaxChunks CUs (one workgroup took 0.18 ms at 32768^2). Pairs of
// several chunks: expand_sum_kernel first writes each chunk's packed op / letter counts, and a block
// sums those of its pair (the total length L fixes the forward positions) and of the chunks before it
// (its starting position and letter counts); a block holding all of its pair's records (the batch: one
// chunk per pair) takes the totals from its own scan. Each thread expands a run of
// consecutive records; their letters go to an LDS copy of the chunk's slice of both strings when it
// fits (kStage bytes each), which the block then writes out in aligned dwords (per-thread byte runs
// land ~10 bytes apart, one uncoalesced byte store per letter), else straight to HBM. Block 0 also
// writes the trailing run and the sa_result.
constexpr int kExpThreads = 256;
constexpr int kStage = 12288;  // LDS staging bytes per string

// block-wide sums of two 64-bit values (tree in LDS)
__device__ __forceinline__ void block_sum2(int64_t &x, int64_t &y, int64_t *lds)
{
    const int t = threadIdx.x;
    lds[t] = x;
    lds[kExpThreads + t] = y;
    __syncthreads();
    for (int d = kExpThreads / 2; d > 0; d >>= 1)
    {
        if (t < d)
        {
            lds[t] += lds[t + d];
            lds[kExpThreads + t] += lds[kExpThreads + t + d];
        }
        __syncthreads();
    }
    x = lds[0];
    y = lds[kExpThreads];
    __syncthreads();
}

// exclusive block scan: inclusive scan inside each wave by lane shifts, then the waves' totals
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t *lds, int64_t &total)
{
    const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
    int64_t x = v;
    for (int d = 1; d < kWave; d <<= 1)
    {
        const int64_t y = __shfl_up(x, d, kWave);
        if (lane >= d) x += y;
    }
    if (lane == kWave - 1) lds[wv] = x;
    __syncthreads();
    int64_t before = 0;
    total = 0;
    for (int k = 0; k < kExpThreads / kWave; ++k)
    {
        const int64_t s = lds[k];
        before += k < wv ? s : 0;
        total += s;
    }
    __syncthreads();
    return before + x - v;
}

// ops and letters consumed along the free coordinate by record v, packed (each < 2^31 per pair)
__device__ __forceinline__ int64_t rec_counts(int v) { return ((int64_t)((v >> 1) + 1) << 32) | (int64_t)((v >> 1) + (v & 1)); }

// records [lo, hi) of a pair -> put(forward position, text letter, pattern letter)
template <class Put>
__device__ __forceinline__ void expand_records(const TbHead &h, const int32_t *rec, int lo, int hi, int64_t P,
                                               int64_t C0, int64_t L, const int8_t *tx, const int8_t *px,
                                               const char *alpha, char GAP, Put put)
{
    if (h.kind == kRecRows)
    {
        // record q: row i0 - q entered at column j; `run` LEFTs, then DIAG (to column j - run - 1) or TOP
        int64_t i = (int64_t)h.i0 - lo, j = (int64_t)h.j0 - C0;
        for (int q = lo; q < hi; ++q)
        {
            const int v = rec[q];
            const int run = v >> 1, d = v & 1;
            const int64_t flo = L - 1 - P - run;  // forward position of the leaving move
            const int64_t jl = j - run;           // column of the leaving cell
            put(flo, d ? alpha[tx[jl - 1]] : GAP, alpha[px[i - 1]]);
            for (int r = 0; r < run; ++r) put(flo + 1 + r, alpha[tx[jl + r]], GAP);
            P += run + 1;
            j = jl - d;
            i -= 1;
        }
    }
    else
    {
        // record q: column j0 - q entered at row i; `run` TOPs, then DIAG (to row i - run - 1) or LEFT
        int64_t j = (int64_t)h.j0 - lo, i = (int64_t)h.i0 - C0;
        for (int q = lo; q < hi; ++q)
        {
            const int v = rec[q];
            const int run = v >> 1, d = v & 1;
            const int64_t flo = L - 1 - P - run;
            const int64_t il = i - run;  // row of the leaving cell
            put(flo, alpha[tx[j - 1]], d ? alpha[px[il - 1]] : GAP);
            for (int r = 0; r < run; ++r) put(flo + 1 + r, GAP, alpha[px[il + r]]);
            P += run + 1;
            i = il - d;
            j -= 1;
        }
    }
}

__global__ __launch_bounds__(kExpThreads) void expand_kernel(ExpandArgs a)
{
    __shared__ int64_t scan[2 * kExpThreads];
    __shared__ char alpha[40];
    __shared__ __attribute__((aligned(16))) char stT[kStage], stP[kStage];
    const int p = blockIdx.y;
    const int t = threadIdx.x;
    const TbHead h = a.heads[p];
    const int N = h.nrec;
    const int c0 = (int)blockIdx.x * a.chunk_recs;
    if (blockIdx.x > 0 && c0 >= N) return;  // (uniform per block)
    if (t < 33) alpha[t] = a.alphabet[t];
    const PairDesc pd = a.pairs[p];
    const int32_t *rec = a.rec + pd.rec_off;
    const int8_t *tx = a.text + pd.text_off;
    const int8_t *px = a.pattern + pd.pattern_off;
    char *ot = a.out_text + pd.out_off;
    char *op = a.out_pattern + pd.out_off;
    const int cend = min(N, c0 + a.chunk_recs);
    const bool whole = c0 == 0 && cend == N;  // (uniform per block)
    // pass 1: this thread's records of the chunk
    const int per = (cend - c0 + kExpThreads - 1) / kExpThreads;
    const int lo = min(cend, c0 + t * per), hi = min(cend, lo + per);
    int64_t mine = 0;
    for (int q = lo; q < hi; ++q) mine += rec_counts(rec[q]);
    int64_t chunkTot;
    const int64_t exIn = block_exclusive_scan(mine, scan, chunkTot);
    // chunks of a longer pair: every block publishes its chunk's sums, then takes the pair's totals and
    // the prefix before its chunk from all of them. The blocks of one pair wait for each other, so they
    // must all be resident: a pair has at most kMaxChunks blocks, dispatched together in grid order,
    // and every pair before it in the grid completes without waiting for later ones. A published sum
    // carries the fill's epoch in its flag word, (epoch << 32) | ~epoch: no clearing per call (a plan
    // of its own clears the flags once when created; workspace plans' epochs only grow)
    int64_t tot = 0, pre = 0;
    if (!whole)
    {
        const uint64_t tag = ((uint64_t)a.epoch << 32) | (uint32_t)~a.epoch;
        uint64_t *flags = a.chunk_flags + (int64_t)p * kMaxChunks;
        if (t == 0)
        {
            __hip_atomic_store(&a.chunk_sums[(int64_t)p * kMaxChunks + blockIdx.x], chunkTot, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&flags[blockIdx.x], tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        const int nch = (N + a.chunk_recs - 1) / a.chunk_recs;
        for (int c = t; c < nch; c += kExpThreads)
        {
            while (__hip_atomic_load(&flags[c], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != tag)
                __builtin_amdgcn_s_sleep(2);
            const int64_t x = __hip_atomic_load(&a.chunk_sums[(int64_t)p * kMaxChunks + c], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            tot += x;
            pre += c < (int)blockIdx.x ? x : 0;
        }
        block_sum2(tot, pre, scan);
    }
    const int64_t ex = exIn + pre;
    if (whole) tot = chunkTot;
    const int64_t totCnt = tot >> 32, totCons = tot & 0xffffffffll;
    const int64_t P0 = ex >> 32, C0 = ex & 0xffffffffll;
    const int64_t L = totCnt + h.tail;
    const char GAP = alpha[a.A];
    // pass 2: the chunk's forward positions are [L - (pre + chunk ops), L - pre); the LDS copy starts
    // at the dword holding the first one, so LDS and HBM dwords line up
    const int64_t fEnd = L - (pre >> 32);
    const int64_t fBeg = fEnd - (chunkTot >> 32);
    const int64_t sBeg = fBeg - (int64_t)(((uintptr_t)(ot + fBeg)) & 3);
    const bool alignedTP = (((uintptr_t)ot ^ (uintptr_t)op) & 3) == 0;
    if (alignedTP && fEnd - sBeg <= kStage)
    {
        expand_records(h, rec, lo, hi, P0, C0, L, tx, px, alpha, GAP, [&](int64_t f, char ct, char cp) {
            stT[f - sBeg] = ct;
            stP[f - sBeg] = cp;
        });
        __syncthreads();
        // head bytes up to the first whole dword, whole dwords, tail bytes
        const int64_t dBeg = (fBeg + 3 - sBeg) / 4, dEnd = (fEnd - sBeg) / 4;
        const int64_t head = min(fEnd, sBeg + 4 * dBeg) - fBeg;
        if (t < head)
        {
            ot[fBeg + t] = stT[fBeg - sBeg + t];
            op[fBeg + t] = stP[fBeg - sBeg + t];
        }
        for (int64_t d = dBeg + t; d < dEnd; d += kExpThreads)
        {
            *reinterpret_cast<uint32_t *>(ot + sBeg + 4 * d) = *reinterpret_cast<const uint32_t *>(stT + 4 * d);
            *reinterpret_cast<uint32_t *>(op + sBeg + 4 * d) = *reinterpret_cast<const uint32_t *>(stP + 4 * d);
        }
        const int64_t tBeg = max(fBeg + head, sBeg + 4 * dEnd);
        if (tBeg + t < fEnd)
        {
            ot[tBeg + t] = stT[tBeg - sBeg + t];
            op[tBeg + t] = stP[tBeg - sBeg + t];
        }
    }
    else
    {
        expand_records(h, rec, lo, hi, P0, C0, L, tx, px, alpha, GAP, [&](int64_t f, char ct, char cp) {
            ot[f] = ct;
            op[f] = cp;
        });
    }
    if (blockIdx.x != 0) return;
    // the trailing run: forward positions 0 .. tail-1, ending at the walk's last cell
    {
        const int64_t iT = h.kind == kRecRows ? (int64_t)h.i0 - N : (int64_t)h.i0 - totCons;
        const int64_t jT = h.kind == kRecRows ? (int64_t)h.j0 - totCons : (int64_t)h.j0 - N;
        for (int64_t f = t; f < h.tail; f += kExpThreads)
        {
            if (h.tail_op == kLeft)
            {
                ot[f] = alpha[tx[jT - h.tail + f]];
                op[f] = GAP;
            }
            else
            {
                ot[f] = GAP;
                op[f] = alpha[px[iT - h.tail + f]];
            }
        }
    }
    if (t == 0)
    {
        sa_result r;
        r.score = h.score;
        // the control word of this fill: a pair aligned after a hand-off timeout or on bad input carries
        // the error itself, so a device-to-device copy of the results (sa_plan_copy_results, the RCCL
        // gather) keeps it
        r.status = a.ctrl->abort_flag || h.err ? SA_ERR_TIMEOUT : (a.ctrl->bad_input == a.epoch ? SA_ERR_INVALID : SA_OK);
        r.num_alignment_bytes = (uint64_t)L;
        r.start_text = (uint64_t)h.start_text;
        r.start_pattern = (uint64_t)h.start_pattern;
        a.results[p] = r;
    }
}

// ------------------------------------------------------------------------------------------------
// launches
// ------------------------------------------------------------------------------------------------
template <bool LOCAL>
void launch_walk_m(int R, const WalkArgs &a, int np, hipStream_t st)
{
    const int grid = a.cap > 0 ? std::min(np, a.cap) : np;
    switch (R)
    {
    case 1: hipLaunchKernelGGL(walk_rw_kernel<LOCAL>, dim3(np), dim3(2 * kWave), 0, st, a); break;
    case 2: hipLaunchKernelGGL((walk_cw_kernel<2, LOCAL>), dim3(grid), dim3(kWave), 0, st, a, np); break;
    case 4: hipLaunchKernelGGL((walk_cw_kernel<4, LOCAL>), dim3(grid), dim3(kWave), 0, st, a, np); break;
    case 8: hipLaunchKernelGGL((walk_cw_kernel<8, LOCAL>), dim3(grid), dim3(kWave), 0, st, a, np); break;
    case 16: hipLaunchKernelGGL((walk_cw_kernel<16, LOCAL>), dim3(grid), dim3(kWave), 0, st, a, np); break;
    default: hipLaunchKernelGGL((walk_cw_kernel<32, LOCAL>), dim3(grid), dim3(kWave), 0, st, a, np); break;
    }
}

void launch_walk(int R, bool local, const WalkArgs &a, int np, hipStream_t st)
{
    if (local) launch_walk_m<true>(R, a, np, st);
    else launch_walk_m<false>(R, a, np, st);
}

void launch_tb(const TbArgs &args, const WalkArgs &w, int nstrips, int ngroups, int np, int rounds, bool wide, hipStream_t st)
{
    TbArgs a = args;
    for (int r = 1; r <= rounds; ++r)
    {
        a.round = r;
        a.last_round = r == rounds;
        if (wide) hipLaunchKernelGGL(tb_table_kernel<1024>, dim3(nstrips), dim3(1024), 0, st, a);
        else hipLaunchKernelGGL(tb_table_kernel<512>, dim3(nstrips), dim3(512), 0, st, a);
        hipLaunchKernelGGL(tb_compose_kernel, dim3(ngroups), dim3(1024), 0, st, a);
        hipLaunchKernelGGL(tb_resolve_kernel, dim3(np), dim3(1024), 0, st, a);
    }
    a.ngroups = ngroups;
    if (a.local)
    {
        hipLaunchKernelGGL(tb_walk_kernel<false>, dim3(ngroups), dim3(kTbG * kWave), 0, st, a, w);
        hipLaunchKernelGGL(tb_check_kernel, dim3(nstrips), dim3(kWave), 0, st, a);
        hipLaunchKernelGGL(tb_finish_kernel<true>, dim3(np), dim3(2 * kWave), 0, st, a, w);
    }
    else
        hipLaunchKernelGGL(tb_walk_kernel<true>, dim3(ngroups + np), dim3(kTbG * kWave), 0, st, a, w);  // (+ finish)
}

void launch_expand(const ExpandArgs &a, int np, int64_t max_records, hipStream_t st)
{
    ExpandArgs x = a;
    const int64_t recs = std::max<int64_t>(1, max_records);
    const int64_t per = recs <= kChunkRecs ? kChunkRecs : std::max<int64_t>(kMinChunkRecs, (recs + kMaxChunks - 1) / kMaxChunks);
    x.chunk_recs = (int)per;
    const int chunks = (int)((recs + per - 1) / per);
    hipLaunchKernelGGL(expand_kernel, dim3(chunks, np), dim3(kExpThreads), 0, st, x);
}

}  // namespace sa
