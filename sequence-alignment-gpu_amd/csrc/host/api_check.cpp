// sa_api_check — a C++14 caller of the batch extension: N DNA Requests of mixed sizes (text at least
// as long as the pattern, as parseArguments guarantees, utilities.cpp:225-230), aligned with one
// SequenceAlignment::alignSequenceGPUBatch call over G GPUs and, one by one, with the reference
// semantics of alignSequenceCPU; every Response field and both strings compared.
//   usage: sa_api_check global|local <requests> <max length> <gpus>
// Prints one JSON line {"requests", "mismatches", "gpu_us", "cpu_us"}; exit status 0 iff all equal.
#include <sys/time.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "SequenceAlignment.hpp"

namespace
{
uint64_t now_us()
{
    timeval t;
    gettimeofday(&t, nullptr);
    return 1000000ull * (uint64_t)t.tv_sec + (uint64_t)t.tv_usec;
}

uint64_t next(uint64_t &s)
{
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return s >> 33;
}
}  // namespace

int main(int argc, const char *argv[])
{
    if (argc < 5)
    {
        std::cerr << "usage: sa_api_check global|local <requests> <max length> <gpus>\n";
        return 2;
    }
    const bool local = std::strcmp(argv[1], "local") == 0;
    const uint64_t count = std::strtoull(argv[2], nullptr, 10), maxLen = std::strtoull(argv[3], nullptr, 10);
    const int gpus = std::atoi(argv[4]);
    static const int blast[16] = {5, -4, -4, -4, -4, 5, -4, -4, -4, -4, 5, -4, -4, -4, -4, 5};
    std::vector<SequenceAlignment::Request> reqs(count);
    uint64_t seed = 12345;
    for (uint64_t i = 0; i < count; ++i)
    {
        SequenceAlignment::Request &r = reqs[i];
        r.deviceType = SequenceAlignment::programArgs::GPU;
        r.sequenceType = SequenceAlignment::programArgs::DNA;
        r.alignmentType = local ? SequenceAlignment::programArgs::LOCAL : SequenceAlignment::programArgs::GLOBAL;
        r.alphabet = SequenceAlignment::DNA_ALPHABET;
        r.alphabetSize = SequenceAlignment::NUM_DNA_CHARS;
        r.gapPenalty = 5;
        std::memcpy(r.scoreMatrix, blast, sizeof(blast));
        r.textNumBytes = 1 + next(seed) % maxLen;
        r.patternNumBytes = 1 + next(seed) % r.textNumBytes;
        r.textBytes = new char[r.textNumBytes];
        r.patternBytes = new char[r.patternNumBytes];
        for (uint64_t x = 0; x < r.textNumBytes; ++x) r.textBytes[x] = (char)(next(seed) % 4);
        // half the patterns are copies of the text with substitutions, so alignments are long
        const bool related = (i & 1) == 0;
        for (uint64_t x = 0; x < r.patternNumBytes; ++x)
            r.patternBytes[x] = related && next(seed) % 8 ? r.textBytes[x] : (char)(next(seed) % 4);
    }
    std::vector<SequenceAlignment::Response> gpu(count), cpu(count);
    const uint64_t t0 = now_us();
    if (SequenceAlignment::alignSequenceGPUBatch(reqs.data(), gpu.data(), count, gpus)) return 1;
    const uint64_t t1 = now_us();
    for (uint64_t i = 0; i < count; ++i)
        if (SequenceAlignment::alignSequenceCPU(reqs[i], &cpu[i])) return 1;
    const uint64_t t2 = now_us();
    uint64_t bad = 0;
    for (uint64_t i = 0; i < count; ++i)
    {
        const SequenceAlignment::Response &g = gpu[i], &c = cpu[i];
        const bool same = g.score == c.score && g.numAlignmentBytes == c.numAlignmentBytes &&
                          g.startInAlignedText == c.startInAlignedText &&
                          g.startInAlignedPattern == c.startInAlignedPattern &&
                          std::memcmp(g.alignedTextBytes, c.alignedTextBytes, c.numAlignmentBytes) == 0 &&
                          std::memcmp(g.alignedPatternBytes, c.alignedPatternBytes, c.numAlignmentBytes) == 0;
        if (!same && bad++ < 3)
            std::cerr << "request " << i << " (" << reqs[i].textNumBytes << "x" << reqs[i].patternNumBytes
                      << "): gpu score " << g.score << " cpu " << c.score << "\n";
    }
    std::cout << "{\"requests\": " << count << ", \"mismatches\": " << bad << ", \"gpu_us\": " << (t1 - t0)
              << ", \"cpu_us\": " << (t2 - t1) << "}\n";
    return bad ? 1 : 0;
}
