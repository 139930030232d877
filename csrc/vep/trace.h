// roctx ranges around the data plane's host stages (parse, index, enqueue, wait, publish), so a
// `rocprofv3 --marker-trace` timeline shows them next to the kernels. The roctx library is
// dlopen'ed on first use (no link-time dependency) and only when VEP_ROCTX=1: disabled ranges
// cost one predictable branch. SURVEY.md §5 "Tracing / profiling" (the reference had none).
#pragma once

namespace vep::trace {

bool enabled();
void push(const char* name);
void pop();

class Range {
 public:
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace vep::trace
