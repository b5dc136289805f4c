// CPU device of the alignSequence CLI (-c / --cpu): what the reference's alignSequenceCPU
// (alignSequenceCPU.cpp:287-333) provides, with the same results. It is a separate user-selected
// device, never a fallback of the GPU path (alignSequenceGPU fails instead of calling it).
//
// Fill: one pass over the (m+1)x(n+1) byte DIRECTION matrix with a single rolling score row;
// the global pass runs in the shifted domain F = H + g*(i+j) (every boundary 0), as the GPU does.
// Tracebacks follow traceBackNW :64-114 and traceBackSW :10-62, start-index quirks included.
#include <algorithm>
#include <iostream>
#include <new>
#include <vector>

#include "SequenceAlignment.hpp"

using SequenceAlignment::DIRECTION;
using SequenceAlignment::Request;
using SequenceAlignment::Response;

namespace
{
// Shared row sweep. LOCAL: H domain with the 0 clamp and STOP; otherwise F domain.
template <bool LOCAL>
std::pair<int, uint64_t> sweep(char *M, uint64_t rows, uint64_t cols, const Request &rq)
{
    const int g = rq.gapPenalty;
    const int A = rq.alphabetSize;
    std::vector<int> row(cols);        // row[j] = value of the current row up to column j-1, previous row after
    for (uint64_t j = 0; j < cols; ++j)
    {
        row[j] = 0;                    // local: H(0,j) = 0;  global: F(0,j) = 0
        M[j] = LOCAL ? DIRECTION::STOP : DIRECTION::LEFT;
    }
    const int diagBonus = LOCAL ? 0 : 2 * g;
    int best = 0;
    uint64_t bestAt = 0;
    for (uint64_t i = 1; i < rows; ++i)
    {
        char *out = M + i * cols;
        out[0] = LOCAL ? DIRECTION::STOP : DIRECTION::TOP;
        const int *sub = rq.scoreMatrix + (int)rq.patternBytes[i - 1] * A;
        int diag = row[0];             // value above-left of the next cell
        int left = 0;                  // column-0 value of this row (local H and global F are 0)
        row[0] = 0;
        for (uint64_t j = 1; j < cols; ++j)
        {
            const int up = row[j];
            const int fromDiag = diag + sub[(int)rq.textBytes[j - 1]] + diagBonus;
            const int fromLeft = LOCAL ? left - g : left;
            const int fromUp = LOCAL ? up - g : up;
            const int gapBest = std::max(fromLeft, fromUp);
            int v = std::max(fromDiag, gapBest);
            char dir = fromDiag > gapBest ? DIRECTION::DIAG : (fromLeft >= fromUp ? DIRECTION::LEFT : DIRECTION::TOP);
            if (LOCAL)
            {
                if (v <= 0) { v = 0; dir = DIRECTION::STOP; }
                if (v > best) { best = v; bestAt = i * cols + j; }
            }
            out[j] = dir;
            diag = up;
            left = v;
            row[j] = v;
        }
    }
    if (LOCAL) return {best, bestAt};
    const uint64_t n = cols - 1, m = rows - 1;
    return {row[cols - 1] - g * (int)(n + m), 0};
}
}  // namespace

int fillMatrixNW(char *M, const uint64_t numRows, const uint64_t numCols, const Request &request)
{
    return sweep<false>(M, numRows, numCols, request).first;
}

std::pair<int, uint64_t> fillMatrixSW(char *M, const uint64_t numRows, const uint64_t numCols, const Request &request)
{
    return sweep<true>(M, numRows, numCols, request);
}

namespace
{
struct Emitter
{
    const Request &rq;
    Response *rs;
    void put(char d, int ti, int pi)
    {
        const bool tt = d == DIRECTION::DIAG || d == DIRECTION::LEFT;
        const bool tp = d == DIRECTION::DIAG || d == DIRECTION::TOP;
        const char gapc = rq.alphabet[rq.alphabetSize];
        rs->alignedTextBytes[rs->numAlignmentBytes] = tt ? rq.alphabet[(int)rq.textBytes[ti]] : gapc;
        rs->alignedPatternBytes[rs->numAlignmentBytes] = tp ? rq.alphabet[(int)rq.patternBytes[pi]] : gapc;
        ++rs->numAlignmentBytes;
    }
    void finish(int ti, int pi)
    {
        rs->startInAlignedText = (uint64_t)(int64_t)ti;
        rs->startInAlignedPattern = (uint64_t)(int64_t)pi;
        std::reverse(rs->alignedTextBytes, rs->alignedTextBytes + rs->numAlignmentBytes);
        std::reverse(rs->alignedPatternBytes, rs->alignedPatternBytes + rs->numAlignmentBytes);
    }
};
}  // namespace

void SequenceAlignment::traceBackNW(const char *M, const uint64_t numRows, const uint64_t numCols,
                                    const Request &request, Response *response)
{
    Emitter em{request, response};
    response->numAlignmentBytes = 0;
    uint64_t i = numRows - 1, j = numCols - 1;
    int ti = (int)request.textNumBytes - 1, pi = (int)request.patternNumBytes - 1;
    while (i > 0 || j > 0)
    {
        const char d = j == 0 ? (char)DIRECTION::TOP : (i == 0 ? (char)DIRECTION::LEFT : M[i * numCols + j]);
        const int tt = d == DIRECTION::DIAG || d == DIRECTION::LEFT;
        const int tp = d == DIRECTION::DIAG || d == DIRECTION::TOP;
        em.put(d, ti, pi);
        ti = std::max(0, ti - tt);
        pi = std::max(0, pi - tp);
        i -= tp;
        j -= tt;
    }
    em.finish(ti, pi);
}

void SequenceAlignment::traceBackSW(const char *M, const uint64_t start, const uint64_t numRows,
                                    const uint64_t numCols, const Request &request, Response *response)
{
    (void)numRows;
    Emitter em{request, response};
    response->numAlignmentBytes = 0;
    uint64_t i = start / numCols, j = start % numCols;
    int ti = (int)j - 1, pi = (int)i - 1;
    while (i > 0 && j > 0 && M[i * numCols + j] != DIRECTION::STOP)
    {
        const char d = M[i * numCols + j];
        const int tt = d == DIRECTION::DIAG || d == DIRECTION::LEFT;
        const int tp = d == DIRECTION::DIAG || d == DIRECTION::TOP;
        em.put(d, ti, pi);
        i -= tp;
        j -= tt;
        if (i == 0 || j == 0) break;  // border reached: no index update (reference :45-46)
        ti = std::max(0, ti - tt);
        pi = std::max(0, pi - tp);
    }
    em.finish(ti, pi);
}

uint64_t SequenceAlignment::alignSequenceCPU(const Request &request, Response *response)
{
    const uint64_t cols = request.textNumBytes + 1, rows = request.patternNumBytes + 1;
    const uint64_t cap = std::max<uint64_t>(1, std::max(2 * request.textNumBytes, request.textNumBytes + request.patternNumBytes));
    std::vector<char> M;
    try
    {
        M.resize(rows * cols);
        delete[] response->alignedTextBytes;
        delete[] response->alignedPatternBytes;
        response->alignedTextBytes = nullptr;
        response->alignedPatternBytes = nullptr;
        response->alignedTextBytes = new char[cap];
        response->alignedPatternBytes = new char[cap];
    }
    catch (const std::bad_alloc &)
    {
        std::cerr << SequenceAlignment::MEM_ERROR;
        return 1;
    }
    if (request.alignmentType == programArgs::GLOBAL)
    {
        response->score = fillMatrixNW(M.data(), rows, cols, request);
        traceBackNW(M.data(), rows, cols, request, response);
    }
    else if (request.alignmentType == programArgs::LOCAL)
    {
        const auto best = fillMatrixSW(M.data(), rows, cols, request);
        response->score = best.first;
        traceBackSW(M.data(), best.second, rows, cols, request, response);
    }
    return 0;
}
