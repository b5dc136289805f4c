// Host utilities of the alignSequence CLI: argument parsing, sequence / score-matrix reading and the
// alignment pretty-printer. Behaviour (including messages and order-dependent flag handling) follows
// the reference's utilities.cpp so that the CLI is a drop-in:
//   indexOfLetter :10-15, getScore :19-25, validateAndTransform :31-63, readSequenceFile :65-104,
//   parseScoreMatrixFile :106-129, parseArguments :131-241, prettyAlignmentPrint :253-315.
#include <algorithm>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <iterator>
#include <sstream>
#include <string>

#include "SequenceAlignment.hpp"

using SequenceAlignment::programArgs;

char indexOfLetter(const char letter, const char *alphabet, const int alphabetSize)
{
    for (int k = 0; k < alphabetSize; ++k)
        if (alphabet[k] == letter) return (char)k;
    return -1;
}

int getScore(char char1, char char2, const char *alphabet, const int alphabetSize, const int *scoreMatrix)
{
    const int row = indexOfLetter(char1, alphabet, alphabetSize);
    const int col = indexOfLetter(char2, alphabet, alphabetSize);
    return scoreMatrix[row * alphabetSize + col];
}

// Rewrites `sequence` in place as alphabet indices and returns how many letters it kept:
// FASTA header lines ('>' up to the end of line) are skipped, lower case is folded to upper case,
// anything outside A..Z is dropped; an A..Z letter missing from the alphabet is an error (returns 0).
int validateAndTransform(std::string &sequence, const char *alphabet, const int alphabetSize)
{
    bool inHeader = false;
    unsigned int kept = 0;
    for (size_t pos = 0; pos < sequence.length(); ++pos)
    {
        const char c = sequence[pos];
        if (inHeader)
        {
            if (c != '\n') continue;
            inHeader = false;
        }
        else if (c == '>')
        {
            inHeader = true;
        }
        const char upper = c > 90 ? (char)(c - 32) : c;
        if (upper < 'A' || upper > 'Z') continue;
        const char idx = indexOfLetter(upper, alphabet, alphabetSize);
        if (idx == -1)
        {
            std::cerr << "'" << upper << "'" << " letter not in alphabet." << std::endl;
            return 0;
        }
        sequence[kept++] = idx;
    }
    return (int)kept;
}

int readSequenceFile(const std::string fname, SequenceAlignment::Request *request)
{
    std::ifstream in(fname);
    if (!in.good())
    {
        std::cerr << fname << " file does not exist" << std::endl;
        return -1;
    }
    std::stringstream buf;
    buf << in.rdbuf();
    std::string contents = buf.str();
    const int letters = validateAndTransform(contents, request->alphabet, request->alphabetSize);
    if (letters <= 0) return 0;  // nothing stored; reported later as "not read"
    char **dst = nullptr;
    uint64_t *len = nullptr;
    if (request->textNumBytes == 0) { dst = &request->textBytes; len = &request->textNumBytes; }
    else if (request->patternNumBytes == 0) { dst = &request->patternBytes; len = &request->patternNumBytes; }
    else return 0;  // a third file is ignored
    try
    {
        *dst = new char[letters];
    }
    catch (const std::bad_alloc &)
    {
        std::cerr << SequenceAlignment::MEM_ERROR;
        return -1;
    }
    std::copy(contents.begin(), contents.begin() + letters, *dst);
    *len = (uint64_t)letters;
    return 0;
}

int parseScoreMatrixFile(const std::string &fname, const int alphabetSize, int *buffer)
{
    std::ifstream in(fname);
    if (!in.good())
    {
        // the reference reports the missing file but still returns success (utilities.cpp:123-128)
        std::cerr << fname << " file does not exist" << std::endl;
        return 0;
    }
    for (int k = 0; k < alphabetSize * alphabetSize; ++k)
    {
        int v;
        if (!(in >> v)) return -1;
        buffer[k] = v;
    }
    return 0;
}

int parseArguments(int argc, const char *argv[], SequenceAlignment::Request *request)
{
    if (argc == 1)
    {
        std::cerr << SequenceAlignment::USAGE;
        return 1;
    }
    request->deviceType = SequenceAlignment::DEFAULT_DEVICE;
    request->sequenceType = SequenceAlignment::DEFAULT_SEQUENCE;
    request->alignmentType = SequenceAlignment::DEFAULT_ALIGNMENT_TYPE;
    request->alphabet = SequenceAlignment::DEFAULT_ALPHABET;
    request->alphabetSize = SequenceAlignment::DEFAULT_ALPHABET_SIZE;
    request->gapPenalty = SequenceAlignment::DEFAULT_GAP_PENALTY;
    request->textNumBytes = 0;
    request->patternNumBytes = 0;

    // A value-taking flag arms its slot (again, even after a value was read); the next non-flag
    // argument fills an armed gap penalty first, then an armed score matrix, otherwise it is a
    // sequence file. The alphabet in force for a file is the one selected by the flags before it.
    enum Slot { IDLE, ARMED, FILLED };
    Slot gap = IDLE, matrix = IDLE;
    for (int a = 1; a < argc; ++a)
    {
        auto flag = SequenceAlignment::argumentMap.find(argv[a]);
        if (flag != SequenceAlignment::argumentMap.end())
        {
            switch (flag->second)
            {
            case programArgs::CPU:
            case programArgs::GPU: request->deviceType = flag->second; break;
            case programArgs::DNA:
            case programArgs::PROTEIN: request->sequenceType = flag->second; break;
            case programArgs::GLOBAL:
            case programArgs::LOCAL:
            case programArgs::SEMI_GLOBAL: request->alignmentType = flag->second; break;
            case programArgs::SCORE_MATRIX: matrix = ARMED; break;
            case programArgs::GAP_PENALTY: gap = ARMED; break;
            }
            const bool dna = request->sequenceType == programArgs::DNA;
            request->alphabet = dna ? SequenceAlignment::DNA_ALPHABET : SequenceAlignment::PROTEIN_ALPHABET;
            request->alphabetSize = dna ? SequenceAlignment::NUM_DNA_CHARS : SequenceAlignment::NUM_PROTEIN_CHARS;
            continue;
        }
        if (gap == ARMED)
        {
            try
            {
                request->gapPenalty = std::stoi(argv[a]);
            }
            catch (...)
            {
                std::cerr << SequenceAlignment::GAP_PENALTY_NOT_READ_ERROR;
                return 1;
            }
            gap = FILLED;
        }
        else if (matrix == ARMED)
        {
            if (parseScoreMatrixFile(argv[a], request->alphabetSize, request->scoreMatrix) == -1)
            {
                std::cerr << SequenceAlignment::SCORE_MATRIX_NOT_READ_ERROR;
                return 1;
            }
            matrix = FILLED;
        }
        else if (readSequenceFile(argv[a], request) == -1)
        {
            std::cerr << SequenceAlignment::SEQ_NOT_READ_ERROR;
            return 1;
        }
    }

    if (request->textNumBytes == 0 || request->patternNumBytes == 0)
    {
        std::cerr << SequenceAlignment::SEQ_NOT_READ_ERROR << SequenceAlignment::USAGE;
        return 1;
    }
    if (request->textNumBytes < request->patternNumBytes)
    {
        // the text is the longer sequence (the GPU layout and the response buffers rely on it)
        std::swap(request->textBytes, request->patternBytes);
        std::swap(request->textNumBytes, request->patternNumBytes);
    }
    if (matrix != FILLED)
    {
        const bool dna = request->sequenceType == programArgs::DNA;
        parseScoreMatrixFile(dna ? SequenceAlignment::DEFAULT_DNA_SCORE_MATRIX_FILE
                                 : SequenceAlignment::DEFAULT_PROTEIN_SCORE_MATRIX_FILE,
                             request->alphabetSize, request->scoreMatrix);
    }
    return 0;
}

// Three lines per 50 aligned columns (text, match line, pattern) with 1-based indices, then
// length / identity / gaps / score. Index arithmetic reproduces the reference exactly
// (utilities.cpp:268-306, including the pattern start used on the text line).
void prettyAlignmentPrint(SequenceAlignment::Response &response, std::ostream &stream)
{
    const uint64_t len = response.numAlignmentBytes;
    if (len == 0) return;
    const int perLine = 50;
    int width = 0;
    int widest = (int)(len + std::max(response.startInAlignedText, response.startInAlignedPattern));
    do
    {
        widest /= 10;
        ++width;
    } while (widest != 0);

    int identical = 0, gaps = 0;
    auto label = [&](uint64_t v) { stream << std::setfill(' ') << std::setw(width) << v << " "; };
    for (int lineStart = 0; (uint64_t)lineStart < len; lineStart += perLine)
    {
        const int lineEnd = (int)std::min<uint64_t>(len, (uint64_t)lineStart + perLine);
        label(lineStart + 1 + response.startInAlignedText);
        stream.write(response.alignedTextBytes + lineStart, lineEnd - lineStart);
        stream << "   " << (lineEnd + response.startInAlignedPattern) << " \n";
        stream << std::setfill(' ') << std::setw(width) << " " << " ";
        for (int c = lineStart; c < lineEnd; ++c)
        {
            const char t = response.alignedTextBytes[c], p = response.alignedPatternBytes[c];
            if (t == p) { stream << '|'; ++identical; }
            else if (t == '-' || p == '-') { stream << ' '; ++gaps; }
            else stream << '.';
        }
        stream << "\n";
        label(lineStart + 1);
        stream.write(response.alignedPatternBytes + lineStart, lineEnd - lineStart);
        stream << "   " << lineEnd << "\n\n";
    }
    const double total = len * 1.0;
    stream << "# Length: \t" << len << "\n"
           << "# Identity: \t" << identical << "/" << len << std::setprecision(3) << " ("
           << (identical / total * 100) << "%)\n"
           << "# Gaps: \t" << gaps << "/" << len << std::setprecision(3) << " (" << (gaps / total * 100) << "%)\n"
           << "# Score: \t" << response.score << "\n";
}
