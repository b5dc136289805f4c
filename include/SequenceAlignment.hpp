// SequenceAlignment.hpp — the request/response API of robertszafa/sequence-alignment-gpu, re-declared
// for the MI355X build so that existing callers (the alignSequence CLI, tests, benchmarks) compile
// against it unchanged.
//
// Interface parity with the reference header (SequenceAlignment.hpp of the reference):
//   programArgs / argumentMap / USAGE / error strings          :10-50
//   alphabets, sizes, defaults                                  :52-68
//   Request / Response (same members, same order, same owners)  :71-120
//   DIRECTION                                                   :122
//   alignSequenceCPU / alignSequenceGPU / traceBackNW / traceBackSW  :125-131
// Differences: the implementation is compiled into libsequence_alignment.so instead of being
// #included into every translation unit (reference :138-140), so the free functions of
// utilities.cpp are declared here too, and the -DBENCHMARK contract of alignSequenceGPU
// (return fill time in microseconds, skip the traceback; alignSequenceGPU.cu:555-626) is
// selected per caller by the macro below instead of by recompiling the engine.
#pragma once

#include <cstdint>
#include <iostream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace SequenceAlignment
{
enum programArgs
{
    CPU, GPU,                     // device
    DNA, PROTEIN,                 // sequence type
    GLOBAL, LOCAL, SEMI_GLOBAL,   // algorithm (SEMI_GLOBAL is declared by the reference, never implemented)
    SCORE_MATRIX,                 // next argument: score matrix file
    GAP_PENALTY,                  // next argument: gap penalty
};

const std::unordered_map<std::string, programArgs> argumentMap = {
    {"--cpu", programArgs::CPU},          {"-c", programArgs::CPU},
    {"--gpu", programArgs::GPU},          {"-g", programArgs::GPU},
    {"--dna", programArgs::DNA},          {"-d", programArgs::DNA},
    {"--protein", programArgs::PROTEIN},  {"-p", programArgs::PROTEIN},
    {"--global", programArgs::GLOBAL},    {"--local", programArgs::LOCAL},
    {"--score-matrix", programArgs::SCORE_MATRIX}, {"-s", programArgs::SCORE_MATRIX},
    {"--gap-penalty", programArgs::GAP_PENALTY},
};

// User-facing text (byte-identical to the reference: the CLI prints it).
const std::string USAGE =
    "Usage: ./alignSequence [-d|-p] [-c|-g] [--global|--local] [-s <file>] [--gap-penalty <int>] <file> <file>\n"
    "       -d, --dna             - align dna sequences (default)\n"
    "       -p, --protein         - align protein sequence\n"
    "       -c, --cpu             - use cpu device (default)\n"
    "       -g, --gpu             - use gpu device\n"
    "       --global              - use global alignment (default)\n"
    "       --local               - use local alignment\n"
    "       -s, --score-matrix    - next argument is a score matrix file\n"
    "       --gap-penalty         - next argument is a gap open penalty (default 5)\n";
const std::string SEQ_NOT_READ_ERROR = "error: text sequence or pattern sequence not read\n";
const std::string MEM_ERROR = "error: sequence is too long, not enough memory\n";
const std::string SCORE_MATRIX_NOT_READ_ERROR =
    "error: matrix scores not read. Only integer scores accepted (int)\n";
const std::string GAP_PENALTY_NOT_READ_ERROR =
    "error: gap penalty not read. Only integer scores accepted (int)\n";

const unsigned int NUM_DNA_CHARS = 4;
const unsigned int NUM_PROTEIN_CHARS = 23;
// Letter i of a sequence is stored as its index in the alphabet; the entry after the last
// letter is the gap character used in aligned output.
const char DNA_ALPHABET[] = {'A', 'T', 'C', 'G', '-'};
const char PROTEIN_ALPHABET[] = {'A', 'R', 'N', 'D', 'C', 'Q', 'E', 'G', 'H', 'I', 'L', 'K',
                                 'M', 'F', 'P', 'S', 'T', 'W', 'Y', 'V', 'B', 'Z', 'X', '-'};

const programArgs DEFAULT_DEVICE = programArgs::CPU;
const programArgs DEFAULT_SEQUENCE = programArgs::DNA;
const programArgs DEFAULT_ALIGNMENT_TYPE = programArgs::GLOBAL;
static const char *DEFAULT_ALPHABET __attribute__((unused)) = DNA_ALPHABET;
const int DEFAULT_ALPHABET_SIZE = NUM_DNA_CHARS;
const short DEFAULT_GAP_PENALTY = 5;
const std::string DEFAULT_DNA_SCORE_MATRIX_FILE = "scoreMatrices/dna/blast.txt";
const std::string DEFAULT_PROTEIN_SCORE_MATRIX_FILE = "scoreMatrices/protein/blosum50.txt";

struct Request
{
    programArgs deviceType;
    programArgs sequenceType;
    programArgs alignmentType;
    char *textBytes = nullptr;        // alphabet indices, owned (delete[])
    uint64_t textNumBytes;
    char *patternBytes = nullptr;     // alphabet indices, owned (delete[])
    uint64_t patternNumBytes;
    const char *alphabet; int alphabetSize;
    int scoreMatrix[NUM_PROTEIN_CHARS * NUM_PROTEIN_CHARS];  // row-major, stride alphabetSize
    int gapPenalty;

    ~Request()
    {
        delete[] textBytes;
        delete[] patternBytes;
        textBytes = nullptr;
        patternBytes = nullptr;
    }
};

struct Response
{
    char *alignedTextBytes = nullptr;     // letters or '-', forward order, owned (delete[])
    char *alignedPatternBytes = nullptr;
    uint64_t numAlignmentBytes;
    uint64_t startInAlignedText;          // may be (uint64_t)-1 for an empty local alignment
    uint64_t startInAlignedPattern;
    int score;

    ~Response()
    {
        delete[] alignedTextBytes;
        delete[] alignedPatternBytes;
        alignedTextBytes = nullptr;
        alignedPatternBytes = nullptr;
    }
};

enum DIRECTION { LEFT, DIAG, TOP, STOP };

/// CPU device (-c): host implementation in libsequence_alignment.so.
uint64_t alignSequenceCPU(const Request &, Response *);

/// GPU device (-g): the MI355X engine through the C ABI of sa_hip.h. Returns 0 or 1.
uint64_t alignSequenceGPU(const Request &, Response *);

/// -DBENCHMARK contract of the reference: DP fill only, returns its device time in microseconds.
uint64_t alignSequenceGPUFillMicros(const Request &, Response *);

/// Extension (the reference has no multi-GPU path): numRequests independent requests in one call,
/// sharded over devices 0..numGpus-1 (sa_align_batch: one plan per device, RCCL result gather).
/// Fills responses[i] as alignSequenceGPU would. Returns 0, or 1 with the message on stdout.
uint64_t alignSequenceGPUBatch(const Request *requests, Response *responses, uint64_t numRequests, int numGpus);

/// Host tracebacks over a full (m+1)x(n+1) byte DIRECTION matrix (used by the CPU device).
void traceBackNW(const char *, const uint64_t, const uint64_t, const Request &, Response *);
void traceBackSW(const char *, const uint64_t, const uint64_t, const uint64_t, const Request &, Response *);

}  // namespace SequenceAlignment

// Callers compiled with -DBENCHMARK get the reference's benchmark behaviour.
#ifdef BENCHMARK
#define alignSequenceGPU alignSequenceGPUFillMicros
#endif

// Free functions of the reference's utilities.cpp (global namespace there too).
char indexOfLetter(const char letter, const char *alphabet, const int alphabetSize);
int getScore(char char1, char char2, const char *alphabet, const int alphabetSize, const int *scoreMatrix);
int validateAndTransform(std::string &sequence, const char *alphabet, const int alphabetSize);
int readSequenceFile(const std::string fname, SequenceAlignment::Request *request);
int parseScoreMatrixFile(const std::string &fname, const int alphabetSize, int *buffer);
int parseArguments(int argc, const char *argv[], SequenceAlignment::Request *request);
void prettyAlignmentPrint(SequenceAlignment::Response &response, std::ostream &stream);

// CPU fill kernels exposed like the reference (tests/benchmarks.cu:153-154 calls them directly).
int fillMatrixNW(char *M, const uint64_t numRows, const uint64_t numCols, const SequenceAlignment::Request &request);
std::pair<int, uint64_t> fillMatrixSW(char *M, const uint64_t numRows, const uint64_t numCols,
                                      const SequenceAlignment::Request &request);
