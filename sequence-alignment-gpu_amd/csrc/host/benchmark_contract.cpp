// sa_benchmark_contract — a caller written the way the reference's benchmark harness is
// (tests/benchmarks.cu:1-2 defines BENCHMARK before including the API header, then calls
// SequenceAlignment::alignSequenceGPU and reads the returned microseconds, :171-176). With
// BENCHMARK defined, include/SequenceAlignment.hpp maps the name to alignSequenceGPUFillMicros,
// so this file checks that contract: the call returns the DP fill time in microseconds, does no
// traceback (the Response is untouched) and the linked symbol is the fill-only entry point.
//   usage: sa_benchmark_contract <rows> <cols>   -> {"us": ..., "mcups": ..., "response_untouched": ...}
#define BENCHMARK

#include <cstdlib>
#include <cstring>
#include <iostream>

#include "SequenceAlignment.hpp"

int main(int argc, const char *argv[])
{
    const uint64_t numRows = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4097;
    const uint64_t numCols = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 4097;
    static const int blast[16] = {5, -4, -4, -4, -4, 5, -4, -4, -4, -4, 5, -4, -4, -4, -4, 5};
    SequenceAlignment::Request request;
    request.sequenceType = SequenceAlignment::programArgs::DNA;
    request.alignmentType = SequenceAlignment::programArgs::GLOBAL;
    request.alphabet = SequenceAlignment::DNA_ALPHABET;
    request.alphabetSize = SequenceAlignment::NUM_DNA_CHARS;
    request.gapPenalty = 5;
    std::memcpy(request.scoreMatrix, blast, sizeof(blast));
    request.textNumBytes = numCols - 1;
    request.patternNumBytes = numRows - 1;
    request.textBytes = new char[request.textNumBytes];
    request.patternBytes = new char[request.patternNumBytes];
    for (uint64_t i = 0; i < request.textNumBytes; ++i) request.textBytes[i] = (char)(rand() % 4);
    for (uint64_t i = 0; i < request.patternNumBytes; ++i) request.patternBytes[i] = (char)(rand() % 4);
    SequenceAlignment::Response response;
    response.score = -12345;
    const uint64_t us = SequenceAlignment::alignSequenceGPU(request, &response);  // the macro'd name
    const bool untouched = response.alignedTextBytes == nullptr && response.alignedPatternBytes == nullptr &&
                           response.score == -12345;
    std::cout << "{\"us\": " << us << ", \"mcups\": " << (us ? numRows * numCols / us : 0)
              << ", \"response_untouched\": " << (untouched ? "true" : "false") << "}\n";
    return untouched && us > 1 ? 0 : 1;
}
