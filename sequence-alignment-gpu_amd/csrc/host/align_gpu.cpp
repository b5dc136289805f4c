// alignSequenceGPU — the drop-in replacement of the reference's GPU entry point
// (SequenceAlignment.hpp:127, alignSequenceGPU.cu:463-653), implemented in C++14 over the C ABI
// of sa_hip.h. Behaviour kept from the reference boundary:
//   * the callee allocates Response::alignedTextBytes / alignedPatternBytes with new[]
//     (alignSequenceGPU.cu:402-403) so the caller's ~Response can delete[] them;
//   * returns 0 on success, 1 on failure with the message on stdout (:543, :590);
//   * under -DBENCHMARK the caller gets alignSequenceGPUFillMicros: DP fill time in microseconds,
//     no traceback (:555-626).
// Differences: buffers are max(2*text, text+pattern) bytes (the reference's 2*text overflows when
// a direct caller passes a pattern longer than the text), previously held Response buffers are
// released instead of leaked, and the device is SA_DEVICE (default 0) instead of always 0.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "SequenceAlignment.hpp"
#include "sa_hip.h"

namespace
{
int deviceFromEnv()
{
    const char *e = std::getenv("SA_DEVICE");
    return e ? std::atoi(e) : 0;
}

bool toParams(const SequenceAlignment::Request &request, sa_params *p)
{
    if (request.alignmentType == SequenceAlignment::programArgs::GLOBAL) p->mode = SA_GLOBAL;
    else if (request.alignmentType == SequenceAlignment::programArgs::LOCAL) p->mode = SA_LOCAL;
    else return false;
    p->alphabet_size = request.alphabetSize;
    p->gap_penalty = request.gapPenalty;
    p->rows_per_lane = 0;
    p->score_matrix = request.scoreMatrix;
    p->alphabet = request.alphabet;
    return true;
}

uint64_t runGPU(const SequenceAlignment::Request &request, SequenceAlignment::Response *response, bool fillOnly)
{
    sa_params params;
    if (!toParams(request, &params))
    {
        std::cout << "error: only --global and --local alignments are implemented\n";
        return 1;
    }
    const uint64_t n = request.textNumBytes, m = request.patternNumBytes;
    const uint64_t cap = std::max<uint64_t>(1, std::max(2 * n, n + m));
    sa_result result;
    double fillMicros = 0.0;
    if (fillOnly)
    {
        // fill-time contract: no strings are produced, Response is left untouched
        if (sa_align_pair(&params, request.textBytes, n, request.patternBytes, m, deviceFromEnv(), &result,
                          nullptr, nullptr, cap, &fillMicros) != SA_OK)
        {
            std::cout << "error: " << sa_last_error() << "\n";
            return 1;
        }
        return std::max<uint64_t>(1, (uint64_t)(fillMicros + 0.5));
    }
    delete[] response->alignedTextBytes;
    delete[] response->alignedPatternBytes;
    response->alignedTextBytes = nullptr;
    response->alignedPatternBytes = nullptr;
    try
    {
        response->alignedTextBytes = new char[cap];
        response->alignedPatternBytes = new char[cap];
    }
    catch (const std::bad_alloc &)
    {
        std::cout << SequenceAlignment::MEM_ERROR;
        return 1;
    }
    const int rc = sa_align_pair(&params, request.textBytes, n, request.patternBytes, m, deviceFromEnv(), &result,
                                 response->alignedTextBytes, response->alignedPatternBytes, cap, nullptr);
    if (rc != SA_OK)
    {
        std::cout << (rc == SA_ERR_NOMEM ? SequenceAlignment::MEM_ERROR : "error: " + std::string(sa_last_error()) + "\n");
        return 1;
    }
    response->score = result.score;
    response->numAlignmentBytes = result.num_alignment_bytes;
    response->startInAlignedText = result.start_text;
    response->startInAlignedPattern = result.start_pattern;
    return 0;
}

bool sameScheme(const sa_params &a, const sa_params &b)
{
    return a.mode == b.mode && a.alphabet_size == b.alphabet_size && a.gap_penalty == b.gap_penalty &&
           a.alphabet == b.alphabet &&
           std::memcmp(a.score_matrix, b.score_matrix, sizeof(int) * a.alphabet_size * a.alphabet_size) == 0;
}
}  // namespace

uint64_t SequenceAlignment::alignSequenceGPUBatch(const Request *requests, Response *responses, uint64_t numRequests,
                                                  int numGpus)
{
    // requests sharing one scoring scheme go to sa_align_batch together (one plan per device)
    std::vector<sa_params> params(numRequests);
    for (uint64_t i = 0; i < numRequests; ++i)
        if (!toParams(requests[i], &params[i]))
        {
            std::cout << "error: only --global and --local alignments are implemented\n";
            return 1;
        }
    std::vector<bool> done(numRequests, false);
    for (uint64_t lead = 0; lead < numRequests; ++lead)
    {
        if (done[lead]) continue;
        std::vector<uint64_t> group;
        for (uint64_t i = lead; i < numRequests; ++i)
            if (!done[i] && sameScheme(params[lead], params[i])) group.push_back(i);
        std::vector<sa_host_pair> pairs(group.size());
        std::vector<char *> at(group.size()), ap(group.size());
        std::vector<sa_result> res(group.size());
        for (size_t q = 0; q < group.size(); ++q)
        {
            const Request &rq = requests[group[q]];
            Response &rs = responses[group[q]];
            pairs[q] = sa_host_pair{rq.textBytes, rq.textNumBytes, rq.patternBytes, rq.patternNumBytes};
            const uint64_t cap = std::max<uint64_t>(1, std::max(2 * rq.textNumBytes, rq.textNumBytes + rq.patternNumBytes));
            delete[] rs.alignedTextBytes;
            delete[] rs.alignedPatternBytes;
            rs.alignedTextBytes = rs.alignedPatternBytes = nullptr;
            try
            {
                rs.alignedTextBytes = new char[cap];
                rs.alignedPatternBytes = new char[cap];
            }
            catch (const std::bad_alloc &)
            {
                std::cout << SequenceAlignment::MEM_ERROR;
                return 1;
            }
            at[q] = rs.alignedTextBytes;
            ap[q] = rs.alignedPatternBytes;
        }
        const int rc = sa_align_batch(&params[lead], pairs.data(), (int64_t)pairs.size(), std::max(1, numGpus),
                                      res.data(), at.data(), ap.data());
        if (rc != SA_OK)
        {
            std::cout << (rc == SA_ERR_NOMEM ? SequenceAlignment::MEM_ERROR : "error: " + std::string(sa_last_error()) + "\n");
            return 1;
        }
        for (size_t q = 0; q < group.size(); ++q)
        {
            Response &rs = responses[group[q]];
            rs.score = res[q].score;
            rs.numAlignmentBytes = res[q].num_alignment_bytes;
            rs.startInAlignedText = res[q].start_text;
            rs.startInAlignedPattern = res[q].start_pattern;
            done[group[q]] = true;
        }
    }
    return 0;
}

uint64_t SequenceAlignment::alignSequenceGPU(const Request &request, Response *response)
{
    return runGPU(request, response, false);
}

uint64_t SequenceAlignment::alignSequenceGPUFillMicros(const Request &request, Response *response)
{
    return runGPU(request, response, true);
}
