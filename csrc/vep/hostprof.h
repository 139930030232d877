// In-process sampling profiler of host CPU time (no perf in the image or on the GPU box):
// SIGPROF every `interval_us` of process CPU time records the interrupted user-mode instruction
// address of whichever thread was running. stop() resolves each address to its shared object
// (dladdr) and writes "count object offset symbol" lines; tools/parse_prof_report.py
// symbolises offsets inside the extension with llvm-symbolizer (inlined frames, source lines).
// Used to profile the multi-threaded parse pool in situ (tools/hostprof_parse.py).
#pragma once

#include <string>

namespace vep::hostprof {

void start(int interval_us);
// Stops sampling, writes the histogram to `path`, returns the number of samples.
int stop(const std::string& path);

}  // namespace vep::hostprof
