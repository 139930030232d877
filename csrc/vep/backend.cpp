// Decoder backend selection. The VCN hardware decoder is reached through rocDecode
// (librocdecode: rocDecCreateDecoder / rocDecDecodeFrame / rocDecGetVideoFrame), which would
// produce NV12 surfaces in HBM per camera that the conversion / letterbox kernels and rings
// consume unchanged (docs/ARCHITECTURE.md §2.3). This image ships no rocDecode, so the probe
// reports false and every camera uses the native subset decoder; the probe result is surfaced
// in bench output and /healthz so a deployment can see which backend would run.
#include <dlfcn.h>

#include "gpu.h"

namespace vep::gpu {

bool rocdecode_available() {
  static const bool ok = [] {
    for (const char* lib : {"librocdecode.so.1", "librocdecode.so.0", "librocdecode.so"}) {
      void* h = dlopen(lib, RTLD_LAZY | RTLD_LOCAL);
      if (!h) continue;
      const bool sym = dlsym(h, "rocDecCreateDecoder") && dlsym(h, "rocDecDecodeFrame") &&
                       dlsym(h, "rocDecGetVideoFrame");
      dlclose(h);
      if (sym) return true;
    }
    return false;
  }();
  return ok;
}

}  // namespace vep::gpu
