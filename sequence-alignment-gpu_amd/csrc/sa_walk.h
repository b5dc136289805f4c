// Traceback kernels (sa_walk.hip): the scalar path walk and the parallel letter expansion.
//
// Replaces the host traceback of the reference's GPU path (alignSequenceGPU.cu:628-649) and follows
// the CPU walks bit-exactly: traceBackNW (alignSequenceCPU.cpp:64-114) and traceBackSW (:10-62).
//
// The walk does not emit one op per step. It writes one RECORD per row (row walk, R = 1) or per
// column (column walk, taller strips): p = 2 * run + diag, where `run` counts the LEFT (row walk) /
// TOP (column walk) moves inside the row / column and `diag` says whether the move that leaves it is
// DIAG (else TOP / LEFT). A header per pair holds the start cell and the trailing run. The expansion
// kernel turns records into the aligned strings with two prefix sums (ops and consumed letters).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sa_hip.h"
#include "sa_layout.h"

namespace sa {

enum { kLeft = 0, kDiag = 1, kTop = 2, kStop = 3 };  // SequenceAlignment.hpp:122
enum { kRecRows = 0, kRecCols = 1 };                 // record kinds

struct TbHead {
    int32_t nrec;     // records, in walk order
    int32_t i0, j0;   // start cell of the walk
    int32_t tail;     // ops after the last record: a run of tail_op
    int32_t kind;     // kRecRows / kRecCols
    int32_t tail_op;  // kLeft / kTop
    int32_t score;
    int32_t err;      // nonzero: the walk gave up on a spin bound (the pair's status becomes SA_ERR_TIMEOUT)
    int64_t start_text, start_pattern;  // Response::startInAlignedText / Pattern
};

struct WalkArgs {
    const StripDesc *strips;
    const PairDesc *pairs;
    const uint32_t *masks;       // direction planes (sa_layout.h)
    const uint64_t *strip_best;  // local: best-cell key per strip
    const int32_t *pair_score;   // global: H[m][n] per pair
    int32_t *rec;                // records
    TbHead *heads;
    uint64_t *timing;            // debug (SA_TB_TIMING): per pair {walk start, walk end}
    int32_t gap, key_rowbits;
    int32_t fast;                // 1: unrolled asm strip walk (0: the generic loop only; tests)
    int32_t stager;              // 1: row walk with the stager wave (0: the walker stages every strip)
    // local row walk (R = 1 planes hold no STOP): H is recomputed along the path (local_check)
    const int8_t *text, *pattern;  // the fill's inputs (alphabet indices)
    const int32_t *score_tab;      // A x A, S + g (the plan's local table)
    int32_t A;
    // table traceback (R = 1, see TbGroup): walk_rw_kernel walks only the pairs without groups
    // (tb_finish_kernel walks those the tables leave)
    const int32_t *tb_pg;          // TbArgs::pair_g0, or null: every pair
    int32_t cap;                   // column walk: at most this many waves, each walking pairs in turn (0: one per pair)
};

// TABLE TRACEBACK (R = 1 plans; sa_walk.hip tb_*_kernel). The sequential walk of a long pair costs
// ~60 clk per row on one wave. Instead every strip b gets a TABLE: for each start column c of a window
// of kTbK columns (tb_window_lo) the column at which the walk entering the strip's last row (the start
// row in the start cell's strip) at c enters the row above the strip (all strips at once, the chains
// that meet merged). Groups of kTbG strips compose their tables; one block per pair chains the group
// tables from the start cell upward, which gives every group's entry column, and each group then
// chains its strips' tables and walks its strips in parallel (one wave each, the row walk's code),
// writing the records by row. A start column outside a window ends the chain: the pair falls back to
// walk_rw_kernel (tb_flag). Local: the walk runs on the raw decisions (the R = 1 planes hold no
// STOP) from the best cell down to row 1; each strip then sums its H steps, and tb_check_kernel finds
// per strip, from H at the strip's entry (the sums of the strips before it), where traceBackSW ends
// in it; the first such strip in walk order gives the pair's head (tb_finish_kernel).
constexpr int kTbK = 2048;       // start columns per strip window
constexpr int kTbG = 16;         // strips per group
constexpr int kTbMinStrips = 8;  // pairs with fewer strips take the sequential walk
// ROUNDS. The windows of a round are centred on a line through an anchor: the start cell, then (a
// round that found the path leaving a window at group g) the path's entry column into group g, which
// is then known. The next round rebuilds the tables of the strips at and above the anchor and resumes
// the chain at group g. Line: global, towards (0, 0) (where the path ends); local, the slope of the
// path from the start cell to the anchor (slope 1 from the start cell in the first round: a local
// alignment's own diagonal; towards (0, 0) measured worse for short ones). Local needs the path only
// down to where traceBackSW ends: a local pair whose chain stops after some groups keeps the groups
// resolved so far, and falls back only when the walk does not end inside them (tb_finish_kernel).
// tb_flag: 0 resolved by the tables, 1 sequential walk, 2 pending (another round).
enum TbStart {
    kTbI0, kTbJ0, kTbH, kTbBs,       // start cell, its H, its strip
    kTbRa, kTbXa, kTbDr, kTbDx,      // anchor row / column, line slope dx / dr (columns per row)
    kTbGres,                         // group the chain resumes at (-1: the start cell's group)
    kTbBmin,                         // local: the lowest strip resolved (the walk may end above it)
    kTbStartWords = 12
};
struct TbGroup {
    int32_t pair, s_lo, s_hi;  // the plan's strip indices, s_lo <= s_hi (one pair's)
    int32_t tbl0;              // strip s_lo's table slot (tables exist only for pairs with groups:
                               // slot of strip s = tbl0 + s - s_lo)
};
struct TbArgs {
    const StripDesc *strips;
    const PairDesc *pairs;
    const uint32_t *masks;
    const TbGroup *groups;
    const int32_t *pair_g0;  // [np + 1]: pair p's groups are pair_g0[p] .. pair_g0[p + 1] - 1
    const int32_t *pair_score;
    const uint64_t *strip_best;  // local: best-cell key per strip
    int32_t *start;          // [pair][kTbStartWords] (tb_start_kernel, tb_resolve_kernel; TbStart)
    int32_t *tbl;            // [strip][kTbK] exit column (-1: start column past n)
    int32_t *win;            // [strip] first column of the strip's window (tb_table_kernel)
    int32_t *gtbl;           // [group][kTbK] exit column of the group (-1: left a window)
    int32_t *gent;           // [group] entry column (tb_resolve_kernel)
    int32_t *tb_flag;        // [pair] 1: walk_rw_kernel walks the pair
    int32_t *rec;
    TbHead *heads;
    // local
    int32_t *sent;           // [strip] entry column of the strip's first walked row (tb_walk_kernel)
    int32_t *sdelta;         // [strip] H change over the strip's walked rows (tb_walk_kernel)
    int32_t *send;           // [strip][4] where the walk ends in the strip: nrec, tail, start text / pattern
    int32_t *pend;           // [pair] the strip of the end (highest strip with an end; tb_check_kernel)
    const int8_t *text, *pattern;
    const int32_t *score_tab;  // A x A, S + g (the plan's local table)
    int32_t A, gap, key_rowbits, local, fast;
    int32_t round, last_round;  // this launch's round of tables (1 ..); the last (a pair still unresolved falls back)
    int32_t strict;             // tests (SA_TB_STRICT): no sequential walk for the pairs the tables leave
    int32_t ngroups;            // the plan's table groups (tb_walk_kernel: finish blocks follow them)
    uint64_t *dbg;             // debug (SA_TB_TABLE_TIMING): per strip 12 words of tb_table_kernel stamps
};

// First column of strip b's window: kTbK columns centred, at the strip's first walked row
// r = min(64 b + 64, i0), on the line x = xa - (ra - r) dx / dr (TbStart), clamped to the pair's columns
__host__ __device__ inline int tb_window_lo(int b, int n, int i0, int ra, int xa, int dr, int dx)
{
    const int64_t r = b * 64 + 64 < i0 ? b * 64 + 64 : i0;
    const int64_t c = xa - (((int64_t)(ra - r) * dx + dr / 2) / dr) - kTbK / 2;
    const int64_t hi = n + 1 - kTbK > 0 ? n + 1 - kTbK : 0;
    return (int)(c < 0 ? 0 : (c > hi ? hi : c));
}
// the table traceback of a plan's pairs with groups; the pairs it leaves are walked by tb_finish_kernel
// with the row walk (w), so walk_rw_kernel need only run for pairs without groups
// wide: 1024 threads per strip table instead of 512 (plans with at most one strip per CU)
void launch_tb(const TbArgs &a, const WalkArgs &w, int nstrips, int ngroups, int np, int rounds, bool wide, hipStream_t st);

struct ExpandArgs {
    const int8_t *text, *pattern;
    const PairDesc *pairs;
    const int32_t *rec;
    const TbHead *heads;
    char *out_text, *out_pattern;
    sa_result *results;
    const Control *ctrl;  // the plan's control word: a fill abort or bad input becomes every pair's status
    int32_t A;
    int32_t chunk_recs;  // records per expansion block (launch_expand sets it)
    int64_t *chunk_sums; // [pair][kMaxChunks] packed op / letter counts per block (pairs of several blocks)
    uint64_t *chunk_flags; // [pair][kMaxChunks] (epoch << 32) | ~epoch once the block's sums are there
    uint32_t epoch;      // the plan's fill epoch (tags chunk_flags)
    char alphabet[33];
};

// one wave per pair: row walk (R = 1) or column walk (R >= 2)
void launch_walk(int R, bool local, const WalkArgs &a, int np, hipStream_t st);
// every plan: records -> aligned strings and sa_result; max_records bounds h.nrec over the pairs
// (pattern rows for the row walk, text columns for the column walk)
constexpr int kChunkRecs = 2048;    // pairs of at most this many records: one expansion block each
constexpr int kMinChunkRecs = 256;  // records per block of a longer pair (at least)
constexpr int kMaxChunks = 256;     // blocks per pair (chunks past a pair's records exit at once)
// chunk_sums and chunk_flags must hold np * kMaxChunks entries when max_records > kChunkRecs
void launch_expand(const ExpandArgs &a, int np, int64_t max_records, hipStream_t st);

}  // namespace sa
