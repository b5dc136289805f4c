// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Driver for the *reference's own* CPU path (robertszafa/sequence-alignment-gpu @ /root/reference),
// compiled by oracle/build_ref.sh straight from the reference's source files into oracle/_ref/ref_align.
// This file is ours; it only calls the reference's public CPU functions:
//   parseArguments            utilities.cpp:131
//   prettyAlignmentPrint      utilities.cpp:253
//   alignSequenceCPU          alignSequenceCPU.cpp:287
//   fillMatrixNW / fillMatrixSW  alignSequenceCPU.cpp:203 / :116 (as tests/benchmarks.cu:153-154 does)
//
// Modes
//   ref_align cli <alignSequence args...>   -> exactly what mainDriver.cu:4-27 prints for the CPU device
//   ref_align batch <in.bin> <out.bin>       -> alignSequenceCPU on binary records (format below)
//   ref_align fillbench <global|local> <rows> <cols> <seedT> <seedP> <A> <gap> <matrixfile> <reps> [letters]
//                                            -> best-of-reps fill time in microseconds (benchmarks.cu:102-187);
//                                               letters (default A) = how many letter codes the synthetic
//                                               stream draws from (20 for protein: the standard residues)
//   ref_align parse <alignSequence args...>  -> dumps the Request parseArguments builds (encoded bytes)
//
// batch record (little endian):  int32 mode(0=global,1=local), int32 A, int32 gap, int32 pad,
//   uint64 n(text), uint64 m(pattern), int32 S[A*A], int8 text[n], int8 pattern[m]
// batch result: int32 score, int32 pad, uint64 numAlignmentBytes, uint64 startText, uint64 startPattern,
//   char alignedText[len], char alignedPattern[len]
#include "SequenceAlignment.hpp"   // the build recipe points this at the reference header (GPU include stripped)

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <vector>

using SequenceAlignment::programArgs;

static uint64_t splitmix64(uint64_t &s)
{
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int runCli(int argc, const char *argv[])
{
    SequenceAlignment::Request request;
    SequenceAlignment::Response response;
    if (parseArguments(argc, argv, &request)) return 1;
    if (request.deviceType != programArgs::CPU)
    {
        std::cerr << "ref_align: only the reference CPU device is available here\n";
        return 2;
    }
    if (SequenceAlignment::alignSequenceCPU(request, &response)) return 1;
    prettyAlignmentPrint(response, std::cout);
    return 0;
}

static int runParse(int argc, const char *argv[])
{
    SequenceAlignment::Request request;
    int rc = parseArguments(argc, argv, &request);
    std::cout << "rc " << rc << "\n";
    if (rc) return 0;
    std::cout << "device " << request.deviceType << "\nsequence " << request.sequenceType
              << "\nalignment " << request.alignmentType << "\nalphabetSize " << request.alphabetSize
              << "\ngap " << request.gapPenalty << "\ntext";
    for (uint64_t i = 0; i < request.textNumBytes; ++i) std::cout << " " << int(request.textBytes[i]);
    std::cout << "\npattern";
    for (uint64_t i = 0; i < request.patternNumBytes; ++i) std::cout << " " << int(request.patternBytes[i]);
    std::cout << "\nmatrix";
    for (int i = 0; i < request.alphabetSize * request.alphabetSize; ++i) std::cout << " " << request.scoreMatrix[i];
    std::cout << "\n";
    return 0;
}

static int runBatch(const char *inPath, const char *outPath)
{
    std::ifstream in(inPath, std::ios::binary);
    std::ofstream out(outPath, std::ios::binary);
    if (!in.good() || !out.good()) { std::cerr << "ref_align: cannot open batch files\n"; return 1; }
    while (true)
    {
        int32_t hdr[4];
        if (!in.read(reinterpret_cast<char *>(hdr), sizeof(hdr))) break;
        uint64_t nm[2];
        in.read(reinterpret_cast<char *>(nm), sizeof(nm));
        SequenceAlignment::Request request;
        request.deviceType = programArgs::CPU;
        request.alignmentType = hdr[0] == 0 ? programArgs::GLOBAL : programArgs::LOCAL;
        request.alphabetSize = hdr[1];
        request.sequenceType = hdr[1] == 4 ? programArgs::DNA : programArgs::PROTEIN;
        request.alphabet = hdr[1] == 4 ? SequenceAlignment::DNA_ALPHABET : SequenceAlignment::PROTEIN_ALPHABET;
        request.gapPenalty = hdr[2];
        in.read(reinterpret_cast<char *>(request.scoreMatrix), sizeof(int32_t) * hdr[1] * hdr[1]);
        request.textNumBytes = nm[0];
        request.patternNumBytes = nm[1];
        request.textBytes = new char[nm[0]];
        request.patternBytes = new char[nm[1]];
        in.read(request.textBytes, nm[0]);
        in.read(request.patternBytes, nm[1]);
        SequenceAlignment::Response response;
        if (SequenceAlignment::alignSequenceCPU(request, &response)) return 1;
        int32_t sc[2] = {response.score, 0};
        uint64_t meta[3] = {response.numAlignmentBytes, response.startInAlignedText,
                            response.startInAlignedPattern};
        out.write(reinterpret_cast<char *>(sc), sizeof(sc));
        out.write(reinterpret_cast<char *>(meta), sizeof(meta));
        out.write(response.alignedTextBytes, response.numAlignmentBytes);
        out.write(response.alignedPatternBytes, response.numAlignmentBytes);
    }
    return 0;
}

static int runFillBench(int argc, const char *argv[])
{
    if (argc < 11) { std::cerr << "usage: ref_align fillbench mode rows cols seedT seedP A gap matrix reps\n"; return 1; }
    const bool global = std::strcmp(argv[2], "global") == 0;
    const uint64_t numRows = std::stoull(argv[3]);
    const uint64_t numCols = std::stoull(argv[4]);
    uint64_t seedT = std::stoull(argv[5]), seedP = std::stoull(argv[6]);
    const int A = std::stoi(argv[7]);
    SequenceAlignment::Request request;
    request.alignmentType = global ? programArgs::GLOBAL : programArgs::LOCAL;
    request.alphabetSize = A;
    request.alphabet = A == 4 ? SequenceAlignment::DNA_ALPHABET : SequenceAlignment::PROTEIN_ALPHABET;
    request.gapPenalty = std::stoi(argv[8]);
    parseScoreMatrixFile(argv[9], A, request.scoreMatrix);
    const int reps = std::stoi(argv[10]);
    const int letters = argc > 11 ? std::stoi(argv[11]) : A;
    request.textNumBytes = numCols - 1;
    request.patternNumBytes = numRows - 1;
    request.textBytes = new char[numCols - 1];
    request.patternBytes = new char[numRows - 1];
    for (uint64_t i = 0; i + 1 < numCols; ++i) request.textBytes[i] = char((splitmix64(seedT) >> 33) % letters);
    for (uint64_t i = 0; i + 1 < numRows; ++i) request.patternBytes[i] = char((splitmix64(seedP) >> 33) % letters);
    std::vector<char> M(numRows * numCols);
    double best = 1e300;
    int score = 0;
    for (int r = 0; r < reps; ++r)
    {
        auto t0 = std::chrono::steady_clock::now();
        if (global) score = fillMatrixNW(M.data(), numRows, numCols, request);
        else score = fillMatrixSW(M.data(), numRows, numCols, request).first;
        auto t1 = std::chrono::steady_clock::now();
        best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::cout << "{\"us\": " << best << ", \"score\": " << score << "}\n";
    return 0;
}

int main(int argc, const char *argv[])
{
    if (argc < 2) { std::cerr << "usage: ref_align cli|batch|fillbench|parse ...\n"; return 1; }
    const std::string mode = argv[1];
    if (mode == "cli") { argv[1] = argv[0]; return runCli(argc - 1, argv + 1); }
    if (mode == "parse") { argv[1] = argv[0]; return runParse(argc - 1, argv + 1); }
    if (mode == "batch" && argc == 4) return runBatch(argv[2], argv[3]);
    if (mode == "fillbench") return runFillBench(argc, argv);
    std::cerr << "ref_align: bad mode\n";
    return 1;
}
