// sa_benchmarks — the reference's benchmark harness modes (tests/benchmarks.cu:102-363), restated
// over this repository's SequenceAlignment API (C++14, links libsequence_alignment.so):
//
//   throughput global|local   DP fill only, best of N (benchmarks.cu:102-187: the -DBENCHMARK
//                             contract, alignSequenceGPUFillMicros here), optional CPU fill
//   latency    global|local   fill + traceback + result strings, end to end (:191-266)
//   batch      N [global|local]  N 8192x8192 requests in sequence, end to end (:269-325); with
//                             --multi G all N in one alignSequenceGPUBatch call over G devices
//   maxlength  global|local   120000^2 and 500000^2, GPU fill only, no repeats (:328-355)
//
// Inputs are the reference's dummy requests (:21-41): protein, gap 5, BLOSUM50 from
// scoreMatrices/protein/blosum50.txt (relative path, as the reference), letters rand() % 22 from
// the unseeded C library generator. MCUPS = numRows * numCols / microseconds with numRows =
// patternNumBytes + 1, the reference's convention (:165). Options:
//   --cpu / --gpu (default: gpu only)   --repeats N (default 5)   --sizes R1xC1,R2xC2,...
//   --json (one JSON line per size besides the human-readable lines)
#include <sys/time.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <utility>
#include <vector>

#include "SequenceAlignment.hpp"

using SequenceAlignment::programArgs;
using Sizes = std::vector<std::pair<uint64_t, uint64_t>>;

namespace
{
struct Options {
    bool cpu = false, gpu = true, json = false;
    int repeats = 5;
    int multi = 0;  // batch: > 0 = one alignSequenceGPUBatch call over this many GPUs
    Sizes sizes;
};

void dummyRequest(SequenceAlignment::Request &r, uint64_t numRows, uint64_t numCols, programArgs type)
{
    r.sequenceType = programArgs::PROTEIN;
    r.alignmentType = type;
    r.alphabet = SequenceAlignment::PROTEIN_ALPHABET;
    r.alphabetSize = SequenceAlignment::NUM_PROTEIN_CHARS;
    r.gapPenalty = 5;
    r.textNumBytes = numCols - 1;
    r.patternNumBytes = numRows - 1;
    r.textBytes = new char[r.textNumBytes];
    r.patternBytes = new char[r.patternNumBytes];
    for (uint64_t i = 0; i < r.textNumBytes; ++i) r.textBytes[i] = (char)(rand() % (r.alphabetSize - 1));
    for (uint64_t i = 0; i < r.patternNumBytes; ++i) r.patternBytes[i] = (char)(rand() % (r.alphabetSize - 1));
    if (parseScoreMatrixFile(SequenceAlignment::DEFAULT_PROTEIN_SCORE_MATRIX_FILE, r.alphabetSize, r.scoreMatrix) != 0)
        std::cerr << "warning: could not parse " << SequenceAlignment::DEFAULT_PROTEIN_SCORE_MATRIX_FILE << "\n";
}

void freeRequest(SequenceAlignment::Request &r)
{
    delete[] r.textBytes;
    delete[] r.patternBytes;
    r.textBytes = r.patternBytes = nullptr;
}

uint64_t micros(const timeval &a, const timeval &b)
{
    return 1000000ull * (uint64_t)(b.tv_sec - a.tv_sec) + (uint64_t)(b.tv_usec - a.tv_usec);
}

uint64_t now_us()
{
    timeval t;
    gettimeofday(&t, nullptr);
    return 1000000ull * (uint64_t)t.tv_sec + (uint64_t)t.tv_usec;
}

const char *typeName(programArgs t) { return t == programArgs::GLOBAL ? "Global" : "Local"; }

void jsonLine(const char *mode, programArgs t, uint64_t rows, uint64_t cols, const char *device, uint64_t us,
              bool cups)
{
    std::printf("{\"mode\": \"%s\", \"type\": \"%s\", \"rows\": %llu, \"cols\": %llu, \"device\": \"%s\", \"us\": %llu",
                mode, typeName(t), (unsigned long long)rows, (unsigned long long)cols, device, (unsigned long long)us);
    if (cups) std::printf(", \"mcups\": %.1f", (double)rows * (double)cols / (double)std::max<uint64_t>(1, us));
    std::printf("}\n");
    std::fflush(stdout);
}

void throughput(const Options &o, programArgs type)
{
    Sizes sizes = o.sizes;
    if (sizes.empty())
    {
        if (type == programArgs::GLOBAL)
            for (uint64_t s = 256; s <= 65536; s *= 2) sizes.push_back({s, s});
        else
            for (uint64_t s = 256; s <= 32768; s *= 2) sizes.push_back({s, 32768});
    }
    std::cout << "\n" << typeName(type) << " alignment benchmark:\n";
    for (const auto &sz : sizes)
    {
        const uint64_t rows = sz.first, cols = sz.second;
        std::cout << "-----  " << rows << " x " << cols << "  -----\n";
        SequenceAlignment::Request req;
        SequenceAlignment::Response resp;
        dummyRequest(req, rows, cols, type);
        uint64_t cpuTime = UINT64_MAX, gpuTime = UINT64_MAX;
        if (o.cpu)
        {
            std::vector<char> M(rows * cols);
            for (int r = 0; r < o.repeats; ++r)
            {
                timeval t1, t2;
                gettimeofday(&t1, nullptr);
                if (type == programArgs::GLOBAL) fillMatrixNW(M.data(), rows, cols, req);
                else fillMatrixSW(M.data(), rows, cols, req);
                gettimeofday(&t2, nullptr);
                cpuTime = std::min(cpuTime, micros(t1, t2));
            }
            cpuTime = std::max<uint64_t>(1, cpuTime);
            std::cout << "CPU = " << cpuTime / 1000 << " ms\nMCUPS: " << rows * cols / cpuTime << "\n\n";
            if (o.json) jsonLine("throughput", type, rows, cols, "cpu", cpuTime, true);
        }
        if (o.gpu)
        {
            for (int r = 0; r < o.repeats; ++r)
                gpuTime = std::min(gpuTime, SequenceAlignment::alignSequenceGPUFillMicros(req, &resp));
            gpuTime = std::max<uint64_t>(1, gpuTime);
            std::cout << "GPU = " << gpuTime / 1000 << " ms\nMCUPS: " << rows * cols / gpuTime << "\n\n";
            if (o.json) jsonLine("throughput", type, rows, cols, "gpu", gpuTime, true);
        }
        if (o.cpu && o.gpu) std::cout << "GPU Speedup = " << (double)cpuTime / (double)gpuTime << "\n";
        freeRequest(req);
    }
}

void latency(const Options &o, programArgs type)
{
    Sizes sizes = o.sizes;
    if (sizes.empty())
    {
        if (type == programArgs::GLOBAL)
            sizes = {{256, 256}, {512, 512}, {1024, 1024}, {4096, 4096}, {8192, 8192}, {16384, 16384},
                     {32768, 32768}, {65536, 65536}};
        else
            for (uint64_t s = 256; s <= 32768; s *= 2) sizes.push_back({s, 32768});
    }
    std::cout << "\n" << typeName(type) << " alignment latency (end-to-end) benchmark:\n";
    for (const auto &sz : sizes)
    {
        const uint64_t rows = sz.first, cols = sz.second;
        std::cout << "-----  " << rows << " x " << cols << "  -----\n";
        SequenceAlignment::Request req;
        SequenceAlignment::Response resp;
        dummyRequest(req, rows, cols, type);
        uint64_t cpuTime = UINT64_MAX, gpuTime = UINT64_MAX;
        if (o.cpu)
        {
            for (int r = 0; r < o.repeats; ++r)
            {
                const uint64_t t0 = now_us();
                SequenceAlignment::alignSequenceCPU(req, &resp);
                cpuTime = std::min(cpuTime, now_us() - t0);
            }
            std::cout << "CPU = " << cpuTime / 1000 << " ms\n";
            if (o.json) jsonLine("latency", type, rows, cols, "cpu", cpuTime, false);
        }
        if (o.gpu)
        {
            for (int r = 0; r < o.repeats; ++r)
            {
                const uint64_t t0 = now_us();
                SequenceAlignment::alignSequenceGPU(req, &resp);
                gpuTime = std::min(gpuTime, now_us() - t0);
            }
            std::cout << "GPU = " << gpuTime / 1000 << " ms\n";
            if (o.json) jsonLine("latency", type, rows, cols, "gpu", gpuTime, false);
        }
        if (o.cpu && o.gpu) std::cout << "GPU Speedup = " << (double)cpuTime / (double)gpuTime << "\n";
        freeRequest(req);
    }
}

void batch(const Options &o, programArgs type, uint64_t nBatches)
{
    Sizes sizes = o.sizes.empty() ? Sizes{{8192, 8192}} : o.sizes;
    std::cout << "\n" << typeName(type) << " alignment batch (" << nBatches << "x) benchmark:\n";
    for (const auto &sz : sizes)
    {
        const uint64_t rows = sz.first, cols = sz.second;
        std::cout << "-----  " << rows << " x " << cols << "  -----\n";
        std::vector<SequenceAlignment::Request> reqs(nBatches);
        std::vector<SequenceAlignment::Response> cpuResp(nBatches), gpuResp(nBatches);
        for (auto &r : reqs) dummyRequest(r, rows, cols, type);
        uint64_t cpuTime = 0, gpuTime = 0;
        if (o.cpu)
        {
            SequenceAlignment::alignSequenceCPU(reqs[0], &cpuResp[0]);  // warmup
            const uint64_t t0 = now_us();
            for (uint64_t i = 0; i < nBatches; ++i) SequenceAlignment::alignSequenceCPU(reqs[i], &cpuResp[i]);
            cpuTime = now_us() - t0;
            std::cout << "CPU = " << cpuTime / 1000 << " ms\n";
            if (o.json) jsonLine("batch", type, rows, cols, "cpu", cpuTime, false);
        }
        if (o.gpu)
        {
            SequenceAlignment::alignSequenceGPU(reqs[0], &gpuResp[0]);  // warmup
            const uint64_t t0 = now_us();
            if (o.multi > 0)
            {
                if (SequenceAlignment::alignSequenceGPUBatch(reqs.data(), gpuResp.data(), nBatches, o.multi))
                    std::exit(1);
            }
            else
                for (uint64_t i = 0; i < nBatches; ++i) SequenceAlignment::alignSequenceGPU(reqs[i], &gpuResp[i]);
            gpuTime = now_us() - t0;
            std::cout << "GPU = " << gpuTime / 1000 << " ms\n";
            if (o.json) jsonLine(o.multi > 0 ? "batch_multi" : "batch", type, rows, cols, "gpu", gpuTime, false);
        }
        if (o.cpu && o.gpu) std::cout << "GPU Speedup = " << (double)cpuTime / (double)gpuTime << "\n";
        for (auto &r : reqs) freeRequest(r);
    }
}

void maxLength(const Options &o, programArgs type)
{
    Sizes sizes = o.sizes.empty() ? Sizes{{120000, 120000}, {500000, 500000}} : o.sizes;
    std::cout << "\n" << typeName(type) << " alignment benchmark:\n";
    for (const auto &sz : sizes)
    {
        const uint64_t rows = sz.first, cols = sz.second;
        std::cout << "-----  " << rows << " x " << cols << "  -----\n";
        SequenceAlignment::Request req;
        SequenceAlignment::Response resp;
        dummyRequest(req, rows, cols, type);
        const uint64_t gpuTime = std::max<uint64_t>(1, SequenceAlignment::alignSequenceGPUFillMicros(req, &resp));
        std::cout << "GPU = " << gpuTime / 1000 << " ms\nMCUPS: " << rows * cols / gpuTime << "\n\n";
        if (o.json) jsonLine("maxlength", type, rows, cols, "gpu", gpuTime, true);
        freeRequest(req);
    }
}

Sizes parseSizes(const char *s)
{
    Sizes out;
    std::string str(s);
    size_t pos = 0;
    while (pos < str.size())
    {
        size_t comma = str.find(',', pos);
        if (comma == std::string::npos) comma = str.size();
        const std::string item = str.substr(pos, comma - pos);
        const size_t x = item.find('x');
        if (x != std::string::npos)
            out.push_back({std::strtoull(item.c_str(), nullptr, 10), std::strtoull(item.c_str() + x + 1, nullptr, 10)});
        pos = comma + 1;
    }
    return out;
}

int usage()
{
    std::cerr << "usage: sa_benchmarks throughput|latency|maxlength global|local [opts]\n"
                 "       sa_benchmarks batch N [global|local] [opts]\n"
                 "opts: --cpu --gpu --no-gpu --repeats N --sizes RxC,RxC --json --multi G (batch: one call over G GPUs)\n";
    return 2;
}
}  // namespace

int main(int argc, const char *argv[])
{
    if (argc < 2) return usage();
    const std::string mode = argv[1];
    Options o;
    programArgs type = programArgs::GLOBAL;
    uint64_t nBatches = 1;
    int i = 2;
    if (mode == "batch")
    {
        if (argc < 3) return usage();
        nBatches = std::strtoull(argv[2], nullptr, 10);
        i = 3;
    }
    for (; i < argc; ++i)
    {
        const std::string a = argv[i];
        if (a == "global") type = programArgs::GLOBAL;
        else if (a == "local") type = programArgs::LOCAL;
        else if (a == "--cpu") o.cpu = true;
        else if (a == "--gpu") o.gpu = true;
        else if (a == "--no-gpu") o.gpu = false;
        else if (a == "--json") o.json = true;
        else if (a == "--repeats" && i + 1 < argc) o.repeats = std::max(1, std::atoi(argv[++i]));
        else if (a == "--sizes" && i + 1 < argc) o.sizes = parseSizes(argv[++i]);
        else if (a == "--multi" && i + 1 < argc) o.multi = std::max(1, std::atoi(argv[++i]));
        else return usage();
    }
    std::cout << "Benchmark on GPU: AMD Instinct MI355X (gfx950) via libsa_hip\n";
    if (mode == "throughput") throughput(o, type);
    else if (mode == "latency") latency(o, type);
    else if (mode == "batch") batch(o, type, nBatches);
    else if (mode == "maxlength") maxLength(o, type);
    else return usage();
    return 0;
}
