// alignSequence — drop-in for the reference CLI (mainDriver.cu:4-27): parse the arguments, run the
// selected device, pretty-print the alignment. `-g` runs the MI355X engine.
#include <iostream>

#include "SequenceAlignment.hpp"

int main(int argc, const char *argv[])
{
    SequenceAlignment::Request request;
    SequenceAlignment::Response response;
    if (parseArguments(argc, argv, &request)) return 1;
    uint64_t err = 0;
    if (request.deviceType == SequenceAlignment::programArgs::GPU)
        err = SequenceAlignment::alignSequenceGPU(request, &response);
    else
        err = SequenceAlignment::alignSequenceCPU(request, &response);
    if (err) return 1;
    prettyAlignmentPrint(response, std::cout);
    return 0;
}
