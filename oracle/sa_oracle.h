/* TEST INFRASTRUCTURE ONLY — the CPU oracle. Never linked into, or called by, the product path.
 *
 * A plain-C restatement of the reference CPU path of robertszafa/sequence-alignment-gpu
 * (alignSequenceCPU.cpp), used by tests/ and by bench.py's cpu_baseline leg as the checker.
 * Parity is pinned: tests/golden/ holds fixtures produced by the reference itself
 * (oracle/_ref/ref_align, built from /root/reference by oracle/build_ref.sh) and the
 * reference's own known answers (tests/tests.cu:116-366); tests/test_oracle.py checks this
 * restatement against every one of them.
 */
#ifndef SA_ORACLE_H
#define SA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_LEFT = 0, ORACLE_DIAG = 1, ORACLE_TOP = 2, ORACLE_STOP = 3 }; /* SequenceAlignment.hpp:122 */

/* Global (Needleman-Wunsch) fill — alignSequenceCPU.cpp:203-284. M is (m+1)*(n+1) bytes row-major.
 * Returns H[m][n]. */
int32_t oracle_fill_nw(const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                       const int32_t *S, int32_t A, int32_t gap, uint8_t *M);

/* Local (Smith-Waterman) fill — alignSequenceCPU.cpp:116-201. Returns the max score; *maxIJ is the
 * row-major index of the FIRST cell attaining it (strict '>' scan, initial 0). */
int32_t oracle_fill_sw(const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                       const int32_t *S, int32_t A, int32_t gap, uint8_t *M, uint64_t *maxIJ);

/* Full alignment — alignSequenceCPU.cpp:287-333 with traceBackNW :64-114 / traceBackSW :10-62.
 * mode 0 = global, 1 = local. alphabet has A letters followed by the gap letter.
 * aligned_* must hold at least n+m bytes. Returns 0, or 1 if M could not be allocated. */
int oracle_align(int mode, const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                 const int32_t *S, int32_t A, int32_t gap, const char *alphabet,
                 int32_t *score, uint64_t *num_bytes, uint64_t *start_text, uint64_t *start_pattern,
                 char *aligned_text, char *aligned_pattern);

/* Fill only, timed by the caller (bench cpu_baseline, tests/benchmarks.cu:153-154 convention).
 * mode 2: local with the raw decision of every interior cell (no STOP override, :189), as the
 * engine's rows_per_lane 1 planes hold it. */
int32_t oracle_fill_only(int mode, const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                         const int32_t *S, int32_t A, int32_t gap, uint8_t *M);

#ifdef __cplusplus
}
#endif
#endif
