/* sa_hip.h — C ABI of the MI355X (gfx950) alignment engine: the drop-in boundary for the
 * reference's GPU path.
 *
 * The reference exposes exactly one GPU entry point,
 *     uint64_t SequenceAlignment::alignSequenceGPU(const Request&, Response*);
 *         (robertszafa/sequence-alignment-gpu: SequenceAlignment.hpp:127, implemented in
 *          alignSequenceGPU.cu:463-653)
 * with C++ linkage and C++ structs. This header is the plain-C layer underneath our C++14
 * re-implementation of that function (sequence-alignment-gpu_amd/csrc/host/align_gpu.cpp):
 * plain pointers and sizes, no torch / HIP types in the signatures, so any FFI (ctypes, cgo,
 * JNI, N-API) can bind it. INTEGRATION.md shows the bindings.
 *
 * Semantics are those of the reference's CPU path (alignSequenceCPU.cpp:10-333), bit-exact:
 * score, aligned text, aligned pattern, start indices — including the local-alignment
 * start-index quirk and the "first maximum in row-major order" rule.
 *
 * Error behaviour mirrors the reference boundary: every entry point returns SA_OK (0) on
 * success and a non-zero code otherwise (the reference returns 1 on failure,
 * alignSequenceGPU.cu:543-545, :590-593); sa_last_error() gives the message.
 */
#ifndef SA_HIP_H
#define SA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_ABI_VERSION 1

/* Request::alignmentType (SequenceAlignment.hpp:78; GLOBAL/LOCAL of programArgs :17). */
enum sa_mode { SA_GLOBAL = 0, SA_LOCAL = 1 };

enum sa_status {
    SA_OK = 0,
    SA_ERR_INVALID = 1,     /* bad argument (sizes, alphabet, score range)                  */
    SA_ERR_NOMEM = 2,       /* device allocation failed (reference: MEM_ERROR, :543)       */
    SA_ERR_HIP = 3,         /* a HIP runtime call failed                                    */
    SA_ERR_UNSUPPORTED = 4, /* input outside the engine's documented limits                 */
    SA_ERR_TIMEOUT = 5      /* an in-kernel hand-off did not complete (engine aborted)      */
};

/* Scoring scheme of a Request (SequenceAlignment.hpp:71-99). */
typedef struct sa_params {
    int32_t mode;                 /* SA_GLOBAL (Needleman-Wunsch) or SA_LOCAL (Smith-Waterman)  */
    int32_t alphabet_size;        /* Request::alphabetSize, 1..32 (4 DNA, 23 protein)           */
    int32_t gap_penalty;          /* Request::gapPenalty (linear gap, subtracted per gap cell)  */
    int32_t rows_per_lane;        /* 0 = automatic; else 1,2,4,8,16,32 (tuning knob)            */
    const int32_t *score_matrix;  /* host, alphabet_size^2 ints, row-major [pattern][text]
                                     (Request::scoreMatrix, indexed as alignSequenceCPU.cpp:172) */
    const char *alphabet;         /* host, alphabet_size letters followed by the gap letter
                                     (Request::alphabet; DNA_ALPHABET / PROTEIN_ALPHABET :56-58) */
} sa_params;

/* One (text, pattern) pair inside device-resident arenas of alphabet indices. */
typedef struct sa_pair {
    uint64_t text_offset;     /* byte offset of the text in the text arena        */
    uint64_t text_len;        /* Request::textNumBytes    (columns of the DP)     */
    uint64_t pattern_offset;  /* byte offset of the pattern in the pattern arena  */
    uint64_t pattern_len;     /* Request::patternNumBytes (rows of the DP)        */
} sa_pair;

/* Per-pair outcome: the scalar fields of Response (SequenceAlignment.hpp:101-120). */
typedef struct sa_result {
    int32_t score;                 /* Response::score                                     */
    int32_t status;                /* SA_OK or an error code for this pair               */
    uint64_t num_alignment_bytes;  /* Response::numAlignmentBytes                         */
    uint64_t start_text;           /* Response::startInAlignedText    (may be (uint64)-1) */
    uint64_t start_pattern;        /* Response::startInAlignedPattern (may be (uint64)-1) */
} sa_result;

typedef struct sa_plan sa_plan;

/* ---- one-shot, host pointers (what alignSequenceGPU needs) ------------------------------ */

/* Align one pair held in host memory (alphabet indices). Synchronous. aligned_text and
 * aligned_pattern receive num_alignment_bytes letters in forward order; cap must be at least
 * text_len + pattern_len. If fill_us is non-NULL it receives the device time of the DP fill in
 * microseconds (the quantity the reference returns under -DBENCHMARK, alignSequenceGPU.cu:613-626). */
int sa_align_pair(const sa_params *params, const char *text, uint64_t text_len,
                  const char *pattern, uint64_t pattern_len, int device, sa_result *out,
                  char *aligned_text, char *aligned_pattern, uint64_t cap, double *fill_us);

/* sa_align_pair keeps, per device, a stream, two events and a grow-only device arena across calls
 * (calls on one device are serialised). This releases them for `device` (-1: every device); they
 * are also released at process exit. */
int sa_release_workspace(int device);

/* ---- many pairs from host memory, sharded over GPUs ------------------------------------ */

/* One pair in host memory (alphabet indices), as a Request holds it (SequenceAlignment.hpp:71-99). */
typedef struct sa_host_pair {
    const char *text;
    uint64_t text_len;
    const char *pattern;
    uint64_t pattern_len;
} sa_host_pair;

/* Align num_pairs independent pairs with one scoring scheme over devices 0..num_gpus-1 of this
 * process (one host thread and one plan per device; the per-pair results are gathered to device 0
 * with RCCL, loaded on first use, communicators kept for the process). Synchronous. results: num_pairs entries. aligned_text / aligned_pattern: NULL (scores only) or
 * num_pairs host buffers, buffer i of at least text_len + pattern_len bytes, receiving pair i's
 * num_alignment_bytes letters in forward order. The pair -> device deal is sa_batch_deal's. If
 * num_gpus exceeds the device count, devices are shared round-robin (no RCCL then).
 * Calls are serialised process-wide (one batch at a time, whatever the devices). Each shard keeps its
 * stream, device arenas, RCCL buffers and plan across calls; a call whose shards have the same pair
 * shapes and scoring parameters as the previous one reuses the plans. */
int sa_align_batch(const sa_params *params, const sa_host_pair *pairs, int64_t num_pairs, int num_gpus,
                   sa_result *results, char *const *aligned_text, char *const *aligned_pattern);

/* The deal sa_align_batch uses (host only, no device calls): shard_of[i] in 0..num_shards-1 for
 * work cells[i] = text_len * pattern_len. Equal work: round-robin (i mod num_shards); otherwise
 * longest-processing-time (largest first to the least-loaded shard, ties to the lower shard). */
int sa_batch_deal(const uint64_t *cells, int64_t num_pairs, int num_shards, int32_t *shard_of);

/* Debug record of the calling thread's last sa_align_batch: shards used, whether the results came
 * through the RCCL gather (1) or straight from each shard (0, shards sharing a device), each shard's
 * wall time from upload to the end of its traceback (shard_ms: up to cap entries) and the gather's
 * wall time (0 without RCCL). */
int sa_batch_last_stats(int32_t *num_shards, int32_t *used_rccl, double *shard_ms, int32_t cap, double *gather_ms);

/* ---- plans: many pairs, device-resident inputs, explicit stream ------------------------- */

/* Build a plan (strip layout, workspace) for num_pairs pairs on `device`. Allocates all device
 * workspace once; the plan can be filled/traced back any number of times. */
int sa_plan_create(const sa_params *params, const sa_pair *pairs, int64_t num_pairs, int device,
                   sa_plan **out);
int sa_plan_destroy(sa_plan *plan);

/* Enqueue the DP fill of every pair on `stream` (a hipStream_t; NULL = the HIP null stream, which is
 * also what torch.cuda's default stream handle 0 denotes).
 * d_text / d_pattern are device arenas of alphabet indices addressed by sa_pair offsets. */
int sa_plan_fill(sa_plan *plan, const void *d_text, const void *d_pattern, void *stream);

/* Enqueue the traceback of every pair (after sa_plan_fill on the same stream). */
int sa_plan_traceback(sa_plan *plan, void *stream);

/* Synchronise `stream` and copy the per-pair results to host (num_pairs entries). Returns
 * SA_ERR_TIMEOUT if the fill aborted. */
int sa_plan_fetch_results(sa_plan *plan, sa_result *out, void *stream);

/* Synchronise `stream` and copy pair `index`'s aligned strings (forward order) to host. */
int sa_plan_fetch_alignment(sa_plan *plan, int64_t index, char *aligned_text, char *aligned_pattern,
                            uint64_t cap, void *stream);

/* Bytes of each of the plan's two aligned-string arenas (text and pattern side). */
uint64_t sa_plan_output_bytes(const sa_plan *plan);

/* Synchronise `stream` and copy every pair's result and both aligned-string arenas to host in one
 * pass (what a batch caller needs: one copy each instead of one per pair). text_buf / pattern_buf
 * hold buf_bytes >= sa_plan_output_bytes(plan) bytes; pair i's aligned text / pattern are the
 * results[i].num_alignment_bytes letters at text_buf + offsets[i] / pattern_buf + offsets[i]
 * (offsets: num_pairs entries). results, text_buf and pattern_buf may each be NULL (not copied).
 * Returns SA_ERR_TIMEOUT if the fill aborted. */
int sa_plan_fetch_all(sa_plan *plan, sa_result *results, char *text_buf, char *pattern_buf, uint64_t buf_bytes,
                      uint64_t *offsets, void *stream);

/* Introspection for benches and tests. */
int sa_plan_info(const sa_plan *plan, int64_t *num_strips, int32_t *rows_per_lane,
                 uint64_t *device_bytes, uint64_t *mask_bytes);
/* Which fill kernel sa_plan_fill launches for the plan (benches and tests). */
enum {
    SA_FILL_STRIPS = 0,      /* one wave per strip (fill_kernel; chains hand rows off in LDS / granules) */
    SA_FILL_BAND = 1,        /* band fill: 128-row score strips feeding the 64-row strips (R = 1) */
    SA_FILL_PAIR = 2,        /* pair-packed lone strips: two pairs per wave (fill_pair_kernel) */
    SA_FILL_PAIR_CHAIN = 3   /* pair-packed chains: a couple of pairs per workgroup, a wave per strip */
};
int sa_plan_fill_kind(const sa_plan *plan);
/* Verification: synchronise `stream` and decode pair `index`'s direction bit-planes into the
 * reference's (pattern_len+1) x (text_len+1) byte DIRECTION matrix (LEFT=0, DIAG=1, TOP=2, STOP=3;
 * row 0 / column 0 as the reference fill sets them, alignSequenceCPU.cpp:145-164, :232-248), so the
 * fill can be compared byte-for-byte with the reference's M. Local plans with one row per lane
 * (rows_per_lane 1) hold no STOP bit in their planes (the raw decisions): STOP is put back wherever
 * the cell's score is 0 (alignSequenceCPU.cpp:188-190), recomputed here on the host from the last
 * fill's inputs, so every plan returns the reference's M. M_out must hold (m+1)*(n+1) bytes. */
int sa_plan_fetch_directions(sa_plan *plan, int64_t index, uint8_t *M_out, void *stream);

/* Device pointer to the per-pair sa_result array written by sa_plan_traceback. */
const void *sa_plan_device_results(const sa_plan *plan);

/* Copies the per-pair sa_result array (num_pairs * sizeof(sa_result) bytes) to device memory d_dst
 * on `stream` (asynchronous, device to device: the batch path's results go to the RCCL gather without
 * a host round trip). The abort / bad-input flags are not checked here (sa_plan_fetch_results does). */
int sa_plan_copy_results(const sa_plan *plan, void *d_dst, void *stream);

/* ---- misc ------------------------------------------------------------------------------ */
int sa_device_count(int *count);
const char *sa_last_error(void);
int sa_abi_version(void);
/* Hash of the sources the library was built from (sequence-alignment-gpu_amd/python/sa_amd/buildid.py):
 * callers compare it with the hash of the sources they ship with and refuse a stale binary. */
const char *sa_build_id(void);
/* Runs the engine's wave-level primitive self-test on `device` (DPP lane shifts, ballots);
 * returns SA_OK when the hardware behaves as the kernels assume. */
int sa_selftest(int device);

#ifdef __cplusplus
}
#endif
#endif /* SA_HIP_H */
