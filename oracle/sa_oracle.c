/* TEST INFRASTRUCTURE ONLY — CPU oracle (see sa_oracle.h). Plain C99 restatement of the reference's
 * CPU algorithm; every rule below cites the reference line it follows (paths relative to the
 * reference repository root). Nothing in the product links this file.
 */
#include "sa_oracle.h"

#include <stdlib.h>
#include <string.h>

static inline int32_t imax(int32_t a, int32_t b) { return a > b ? a : b; }

/* One DP sweep for both modes. Two rolling int32 rows, as the reference keeps
 * (alignSequenceCPU.cpp:133-134 / :220-221); the direction of every cell goes to M. */
/* raw (local): interior cells keep the decision before the STOP override of :189 (the engine's R = 1
 * direction planes hold exactly that; its STOP cells are the H == 0 ones). */
static int32_t sweep(int local, int raw, const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                     const int32_t *S, int32_t A, int32_t gap, uint8_t *M, uint64_t *maxIJ)
{
    const uint64_t cols = n + 1, rows = m + 1;
    int32_t *prev = (int32_t *)malloc(sizeof(int32_t) * cols);
    int32_t *cur = (int32_t *)malloc(sizeof(int32_t) * cols);
    if (!prev || !cur) { free(prev); free(cur); return 0; }

    /* Row 0. Global: H = -j*g, every cell LEFT, including M[0][0] (:232-236).
     * Local: H = 0, every cell STOP (:145-149). */
    for (uint64_t j = 0; j < cols; ++j)
    {
        cur[j] = local ? 0 : (int32_t)(j * (uint64_t)(-(int64_t)gap));
        M[j] = local ? ORACLE_STOP : ORACLE_LEFT;
    }

    int32_t best = 0;      /* local: running maximum, starts at 0 (:152-153) */
    uint64_t bestIdx = 0;  /* local: row-major index of its first occurrence */
    for (uint64_t i = 1; i < rows; ++i)
    {
        int32_t *t = prev; prev = cur; cur = t;
        uint8_t *Mrow = M + i * cols;
        /* Column 0. Global: H = -i*g, TOP (:247-248). Local: 0, STOP (:163-164). */
        cur[0] = local ? 0 : (int32_t)(i * (uint64_t)(-(int64_t)gap));
        Mrow[0] = local ? ORACLE_STOP : ORACLE_TOP;
        const int32_t *Srow = S + (int32_t)pattern[i - 1] * A;   /* S[pattern*A + text] (:172, :256) */
        for (uint64_t j = 1; j < cols; ++j)
        {
            const int32_t diag = prev[j - 1] + Srow[(int32_t)text[j - 1]];
            const int32_t left = cur[j - 1] - gap;
            const int32_t up = prev[j] - gap;
            const int32_t gapBest = imax(left, up);
            const int32_t h = imax(diag, gapBest);
            /* Tie rule (:181-188, :265-273): DIAG only when strictly better than both gaps,
             * otherwise LEFT when left >= up, otherwise TOP. */
            uint8_t dir = diag > gapBest ? ORACLE_DIAG : (left >= up ? ORACLE_LEFT : ORACLE_TOP);
            if (local)
            {
                /* Non-positive best -> STOP and score 0 (:189-190); first strict max wins (:191-192). */
                if (h <= 0 && !raw) dir = ORACLE_STOP;
                cur[j] = h > 0 ? h : 0;
                if (cur[j] > best) { best = cur[j]; bestIdx = i * cols + j; }
            }
            else
            {
                cur[j] = h;
            }
            Mrow[j] = dir;
        }
    }
    const int32_t last = cur[cols - 1];   /* global score = H[m][n] (:279) */
    free(prev);
    free(cur);
    if (local) { if (maxIJ) *maxIJ = bestIdx; return best; }
    return last;
}

int32_t oracle_fill_nw(const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                       const int32_t *S, int32_t A, int32_t gap, uint8_t *M)
{
    return sweep(0, 0, text, n, pattern, m, S, A, gap, M, NULL);
}

int32_t oracle_fill_sw(const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                       const int32_t *S, int32_t A, int32_t gap, uint8_t *M, uint64_t *maxIJ)
{
    return sweep(1, 0, text, n, pattern, m, S, A, gap, M, maxIJ);
}

int32_t oracle_fill_only(int mode, const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                         const int32_t *S, int32_t A, int32_t gap, uint8_t *M)
{
    uint64_t idx = 0;
    /* mode 2: local with raw decisions (see sweep) */
    return sweep(mode >= 1, mode == 2, text, n, pattern, m, S, A, gap, M, &idx);
}

static void reverse_bytes(char *p, uint64_t len)
{
    for (uint64_t a = 0, b = len; a + 1 < b; ++a, --b) { char t = p[a]; p[a] = p[b - 1]; p[b - 1] = t; }
}

/* Path step in the flat (m+1)x(n+1) matrix: LEFT -1, DIAG -(cols+1), TOP -cols (:40-42, :103-105). */
static inline uint64_t step_back(uint8_t dir, uint64_t cols)
{
    return dir == ORACLE_LEFT ? 1 : (dir == ORACLE_DIAG ? cols + 1 : (dir == ORACLE_TOP ? cols : 0));
}

int oracle_align(int mode, const int8_t *text, uint64_t n, const int8_t *pattern, uint64_t m,
                 const int32_t *S, int32_t A, int32_t gap, const char *alphabet,
                 int32_t *score, uint64_t *num_bytes, uint64_t *start_text, uint64_t *start_pattern,
                 char *at, char *ap)
{
    const uint64_t cols = n + 1, rows = m + 1;
    uint8_t *M = (uint8_t *)malloc(rows * cols);
    if (!M) return 1;
    const char GAP = alphabet[A];
    uint64_t len = 0;
    int ti, pi;
    if (mode == 0)
    {
        *score = oracle_fill_nw(text, n, pattern, m, S, A, gap, M);
        /* traceBackNW (:64-114): walk from the last cell to index 0; row 0 forces LEFT, col 0 TOP;
         * indices decrement per consumed letter and clamp at 0. */
        uint64_t curr = rows * cols - 1;
        ti = (int)n - 1;
        pi = (int)m - 1;
        while (curr > 0)
        {
            uint8_t d = M[curr];
            if (curr % cols == 0) d = ORACLE_TOP;
            else if (curr < cols) d = ORACLE_LEFT;
            const int tt = d == ORACLE_DIAG || d == ORACLE_LEFT;
            const int tp = d == ORACLE_DIAG || d == ORACLE_TOP;
            at[len] = tt ? alphabet[(int)text[ti]] : GAP;
            ap[len] = tp ? alphabet[(int)pattern[pi]] : GAP;
            ++len;
            ti = ti - tt > 0 ? ti - tt : 0;
            pi = pi - tp > 0 ? pi - tp : 0;
            curr -= step_back(d, cols);
        }
    }
    else
    {
        uint64_t start = 0;
        *score = oracle_fill_sw(text, n, pattern, m, S, A, gap, M, &start);
        /* traceBackSW (:10-62): start at the first max cell; stop at STOP; stepping into row 0 or
         * col 0 ends the walk WITHOUT the index decrement, so the reported start is the first aligned
         * index when the walk hits the border and one less when it hits a STOP cell. */
        ti = (int)(start % cols) - 1;
        pi = (int)(start / cols) - 1;
        uint64_t curr = start;
        while (M[curr] != ORACLE_STOP)
        {
            const uint8_t d = M[curr];
            const int tt = d == ORACLE_DIAG || d == ORACLE_LEFT;
            const int tp = d == ORACLE_DIAG || d == ORACLE_TOP;
            at[len] = tt ? alphabet[(int)text[ti]] : GAP;
            ap[len] = tp ? alphabet[(int)pattern[pi]] : GAP;
            ++len;
            curr -= step_back(d, cols);
            if (curr % cols == 0 || curr < cols) break;
            ti = ti - tt > 0 ? ti - tt : 0;
            pi = pi - tp > 0 ? pi - tp : 0;
        }
    }
    free(M);
    /* int -> uint64 with sign extension, as the reference assigns int to uint64_t (:56-57, :108-109). */
    *start_text = (uint64_t)(int64_t)ti;
    *start_pattern = (uint64_t)(int64_t)pi;
    *num_bytes = len;
    reverse_bytes(at, len);
    reverse_bytes(ap, len);
    return 0;
}
