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
    int32_t pad;
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
};

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
    char alphabet[33];
};

// one wave per pair: row walk (R = 1) or column walk (R >= 2)
void launch_walk(int R, bool local, const WalkArgs &a, int np, hipStream_t st);
// every plan: records -> aligned strings and sa_result; max_records bounds h.nrec over the pairs
// (pattern rows for the row walk, text columns for the column walk)
constexpr int kChunkRecs = 2048;  // records per expansion block (at least)
constexpr int kMaxChunks = 64;    // blocks per pair (chunks past a pair's records exit at once)
void launch_expand(const ExpandArgs &a, int np, int64_t max_records, hipStream_t st);

}  // namespace sa
