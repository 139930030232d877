// roctx loader. See trace.h.
#include "trace.h"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace vep::trace {

namespace {

using PushFn = int (*)(const char*);
using PopFn = int (*)();

struct Roctx {
  bool on = false;
  PushFn push = nullptr;
  PopFn pop = nullptr;
  Roctx() {
    const char* e = std::getenv("VEP_ROCTX");
    if (!e || e[0] != '1') return;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "libroctx64.so.4", "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
      if (push && pop) {
        on = true;
        return;
      }
    }
  }
};

const Roctx& roctx() {
  static Roctx r;
  return r;
}

}  // namespace

bool enabled() { return roctx().on; }
void push(const char* name) { roctx().push(name); }
void pop() { roctx().pop(); }

}  // namespace vep::trace
