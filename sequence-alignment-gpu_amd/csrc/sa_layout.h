// Internal data layout shared by the fill and traceback kernels and the host planner.
//
// A pair's DP matrix (pattern rows 1..m, text columns 1..n; row 0 / column 0 are the boundary)
// is cut into horizontal STRIPS of 64*R rows. One wave64 owns a strip: lane k owns the R
// consecutive rows  row0 + k*R + rho  (rho = 0..R-1) and sweeps the text left to right, lane k
// working on column  j = s - k + 1  at step s (a one-column skew per lane, the anti-diagonal
// wavefront). A strip therefore takes n + 63 steps.
//
// DIRECTIONS. Every (step s, row-slot rho) of a strip is a SLOT  e = s*R + rho  holding two bits
// per lane (two planes). Lane k accumulates its own bits in VGPR words and the strip's slots are
// stored in CHUNKS of CS = max(32, U*R) slots (U = steps per unrolled body): chunk c is
// 64 lanes x LW dwords (LW = 2*CS/32), lane k's LW dwords contiguous = {plane0 words, plane1
// words}, each word 32 consecutive slots with the first slot in bit 31. So slot e of lane k is bit
// 31 - e%32 of dword  c*64*LW + k*LW + P*(CS/32) + (e%CS)/32  (c = e/CS, plane P) from the strip's
// base  masks + 16*strip.mask_off  bytes. That is 16 bytes per slot, and a range of slots that
// starts on a chunk boundary is a contiguous byte range. R = 1 (CS = 32, LW = 2) INTERLEAVES the
// planes instead: lane k's two dwords of chunk c are slots 32c .. 32c+15 and 32c+16 .. 32c+31, slot
// e at bits 31 - 2(e%16) (plane0) and 30 - 2(e%16) (plane1) of dword (e%32)/16, so the traceback's
// row windows (two bits per cell) are funnel shifts of the lane's stream. The reference DIRECTION code (LEFT=0,
// DIAG=1, TOP=2, STOP=3; SequenceAlignment.hpp:122) is
//   global: plane0 = DIAG, plane1 = "up > left";  code = plane0 ? DIAG : plane1 ? TOP : LEFT
//   local, R = 1: as global (the raw decision of every cell); STOP is the cell's H == 0, which the
//           row walk recomputes along the path (sa_walk.hip local_check), so no plane holds it
//   local, R > 1: plane0 = DIAG|STOP, plane1 = (TOP&~DIAG)|STOP;  code = plane0 | plane1 << 1
// That is 2 bits per cell written to HBM (the reference writes 1 byte per cell,
// alignSequenceGPU.cu:142); the algorithmic figure used for the roofline stays 1 B/cell.
//
// STRIP HAND-OFF. A strip's bottom row feeds the next strip's first row. Strips are processed in
// groups of W consecutive strips by one workgroup (W compute waves + 1 I/O wave): inside a group
// the row travels through an LDS ring, between groups through a granule array in global memory:
// granule c-1 holds {tag = epoch, value} of column c as one 8-byte write-through store, so the
// consumer needs no flag and no fence (a tag match means the value is there); the per-call epoch
// makes stale granules from earlier calls unreadable.
#pragma once
#include <stdint.h>

namespace sa {

constexpr int kWave = 64;
constexpr int kPad = 64;          // text-code padding before/after each pair

struct StripDesc {
    int32_t pair;       // owning pair
    int32_t row0;       // first DP row (1-based) of the strip
    int32_t flags;      // kHasPrev | kHasNext
    int32_t nsteps;     // steps this strip runs (n + 63 rounded up to the body length)
    uint64_t mask_off;  // first direction slot (16 bytes per slot, see DIRECTIONS)
    uint64_t bnd_in;    // granule index of the predecessor's bottom row (kHasPrev)
    uint64_t bnd_out;   // granule index of this strip's bottom row (kHasNext)
};
enum : int32_t { kHasPrev = 1, kHasNext = 2 };

struct PairDesc {
    uint64_t text_off, text_len, pattern_off, pattern_len;
    uint64_t code_off;     // start of this pair's padded text-code block (R = 1: A text profiles)
    uint64_t code_len;     // dwords per code array: kPad + text_len + 4*kPad
    uint64_t out_off;      // start of this pair's output region (capacity text_len+pattern_len)
    uint64_t rec_off;      // start of this pair's traceback records (int32, capacity max(n, m) + 64)
    int32_t first_strip, num_strips;
};

// Per-launch control block (zeroed by the host before every fill).
struct Control {
    uint32_t queue_head;   // dynamic strip queue
    uint32_t abort_flag;   // set when a hand-off times out
    uint32_t bad_input;    // set by encode_text_kernel: a text or pattern byte outside 0..A-1
    uint32_t band_head;    // band fill: the bands' group queue
};

}  // namespace sa
