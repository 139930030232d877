// VCN hardware decode backend through rocDecode.
//
// The reference decodes every camera with libavcodec on the CPU (python/read_image.py:87,
// `p.decode()`). On MI355X the video core next to the compute dies (VCN) decodes
// H.264 / H.265 into NV12 surfaces in HBM; rocDecode is its user-space API: a bitstream parser
// (rocDecCreateVideoParser / rocDecParseVideoData) calls back with sequence headers, per-picture
// decode parameters and display-order pictures, the decoder (rocDecCreateDecoder /
// rocDecDecodeFrame) runs them on VCN, and rocDecGetVideoFrame maps a decoded surface as HIP
// device pointers.
//
// librocdecode is loaded at run time (dlopen, VEP_ROCDECODE_LIB overrides the search), compiled
// against the official API header that ROCm ships with rocprofiler-sdk; no link-time dependency,
// so builds without the library keep the native decoder. A Session decodes one camera: each
// displayed picture comes back as a Frame that holds its VCN surface until the worker has copied
// it into the camera's NV12 surface (the shared convert / letterbox / ring path then runs
// unchanged, runtime.cpp); dropping the Frame hands the surface back to the parser.
#pragma once

#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "codec.h"

namespace vep::vcn {

// librocdecode loaded and complete (every entry point the backend calls resolved).
bool available();
// Load a specific librocdecode build when none is loaded yet (the default search runs first:
// VEP_ROCDECODE_LIB, then librocdecode.so.{1,0} on the loader path and under /opt/rocm/lib).
bool load(const std::string& path);
// The library the backend loaded ("" when none) and, when none, why.
std::string library();
std::string load_error();

struct Core;  // parser + decoder of one session (vcn.cpp)

// One displayed picture: NV12 planes on the device (pitch in bytes), display-sized.
struct Frame {
  const u8* y = nullptr;
  const u8* uv = nullptr;
  u32 pitch_y = 0, pitch_uv = 0;
  int width = 0, height = 0;
  // the access unit the picture came from
  i64 pts = 0, dts = 0, tag = 0, arrival_ms = 0;
  bool keyframe = false, corrupt = false;
  char type = '?';
  ~Frame();

 private:
  friend class Session;
  friend struct Core;
  std::shared_ptr<Core> core_;
  std::shared_ptr<void> dec_;  // the decoder whose surface this is
  int pic_idx_ = -1;
  u64 generation_ = 0;
};
using FramePtr = std::shared_ptr<Frame>;

struct SessionStats {
  u64 packets = 0, decoded = 0, displayed = 0, sequences = 0, errors = 0;
};

class Session {
 public:
  // device: the HIP device the surfaces live on (rocDecode device_id)
  Session(Codec codec, int device);
  ~Session();
  Session(const Session&) = delete;
  Session& operator=(const Session&) = delete;

  // Feed one access unit; returns the pictures that reached display order, oldest first.
  std::vector<FramePtr> decode(const AccessUnit& au, i64 tag = 0);
  // End of stream: every picture still waiting in the parser's reorder queue. The next AU must
  // start a new coded sequence (parameter sets are re-sent automatically).
  std::vector<FramePtr> flush();
  SessionStats stats() const;
  Codec codec() const { return codec_; }
  int coded_width() const;
  int coded_height() const;

 private:
  void send(const u8* data, size_t n, u32 flags, u64 pts);
  Codec codec_;
  std::shared_ptr<Core> core_;
  std::vector<u8> pkt_;
  // parameter sets of the stream (re-sent ahead of the first picture after a flush)
  std::vector<std::vector<u8>> ps_;
  bool need_ps_ = true;
  u64 next_pts_ = 1;
};

}  // namespace vep::vcn
