// Test double of librocdecode (rocDecode API as declared by ROCm's header) for the VCN backend
// (csrc/vep/vcn.cpp). The image ships no librocdecode and its VCN cannot be reached, so this
// library stands in for it in tests: the parser decodes with the framework's own CPU decoders
// (avc::Decoder + cpu_reconstruct, hevc::Decoder) and replays every output picture through the
// same callback protocol a real parser uses (sequence -> decode_picture -> display_picture in
// display order, pts echoed); the decoder keeps a bounded pool of output surfaces that are only
// reused once the application marks them (rocDecParserMarkFrameForReuse), so a backend that
// leaks surfaces fails here as it would on VCN. Surfaces are HIP device memory, or host memory
// with VEP_ROCDEC_STUB_HOST=1 (CPU backend tests).
//
// Not a decoder product: only the calls the backend makes are implemented.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include <rocprofiler-sdk/rocdecode/details/rocparser.h>

#include "vep/avc.h"
#include "vep/h264.h"
#include "vep/hevc_dec.h"

#define STUB_API extern "C" __attribute__((visibility("default")))

using namespace vep;

namespace {

struct Pending {  // the picture rocDecDecodeFrame stores (set by the parser just before the callback)
  const HostSurface* s = nullptr;
  int crop_left = 0, crop_top = 0, width = 0, height = 0;
};
thread_local Pending g_pending;

struct StubDecoder {
  bool host = false;
  int w = 0, h = 0;  // target (display) size
  u32 pitch = 0;
  std::vector<u8*> y, uv;
  ~StubDecoder() {
    for (size_t i = 0; i < y.size(); ++i) {
      if (host) {
        std::free(y[i]);
        std::free(uv[i]);
      } else {
        (void)hipFree(y[i]);
        (void)hipFree(uv[i]);
      }
    }
  }
};

struct StubParser {
  RocdecParserParams p{};
  std::vector<bool> busy;  // output surface handed to the application, not yet marked for reuse
  int coded_w = 0, coded_h = 0, disp_w = 0, disp_h = 0;
  avc::Decoder avc;
  std::vector<HostSurface> avc_slots;
  hevc::Decoder hevc;
  u64 reuse_marks = 0;
};

bool host_surfaces() {
  const char* e = std::getenv("VEP_ROCDEC_STUB_HOST");
  return e && e[0] == '1';
}

// Feed one picture leaving the decoder's reorder buffer to the application.
rocDecStatus emit(StubParser& sp, const HostSurface& s, int crop_left, int crop_top, int width, int height, u64 pts) {
  if (sp.coded_w != s.coded_w || sp.coded_h != s.coded_h || sp.disp_w != width || sp.disp_h != height) {
    RocdecVideoFormat f{};
    f.codec = sp.p.codec_type;
    f.frame_rate.numerator = 30;
    f.frame_rate.denominator = 1;
    f.progressive_sequence = 1;
    f.min_num_decode_surfaces = 4;
    f.coded_width = u32(s.coded_w);
    f.coded_height = u32(s.coded_h);
    f.display_area.left = crop_left;
    f.display_area.top = crop_top;
    f.display_area.right = crop_left + width;
    f.display_area.bottom = crop_top + height;
    f.chroma_format = rocDecVideoChromaFormat_420;
    const int n = sp.p.pfn_sequence_callback(sp.p.user_data, &f);
    if (n <= 0) return ROCDEC_RUNTIME_ERROR;
    sp.busy.assign(size_t(n), false);
    sp.coded_w = s.coded_w;
    sp.coded_h = s.coded_h;
    sp.disp_w = width;
    sp.disp_h = height;
  }
  int idx = -1;
  for (size_t i = 0; i < sp.busy.size(); ++i)
    if (!sp.busy[i]) {
      idx = int(i);
      break;
    }
  if (idx < 0) return ROCDEC_RUNTIME_ERROR;  // every surface still held by the application
  RocdecPicParams pp{};
  pp.pic_width = s.coded_w;
  pp.pic_height = s.coded_h;
  pp.curr_pic_idx = idx;
  pp.num_slices = 1;
  pp.ref_pic_flag = 1;
  g_pending = Pending{&s, crop_left, crop_top, width, height};
  const int ok = sp.p.pfn_decode_picture(sp.p.user_data, &pp);
  g_pending = Pending{};
  if (!ok) return ROCDEC_RUNTIME_ERROR;
  sp.busy[size_t(idx)] = true;
  RocdecParserDispInfo di{};
  di.picture_index = idx;
  di.progressive_frame = 1;
  di.pts = pts;
  if (!sp.p.pfn_display_picture(sp.p.user_data, &di)) return ROCDEC_RUNTIME_ERROR;
  return ROCDEC_SUCCESS;
}

rocDecStatus emit_avc(StubParser& sp, const std::vector<avc::OutFrame>& outs) {
  for (const avc::OutFrame& o : outs) {
    const rocDecStatus s = emit(sp, sp.avc_slots[size_t(o.slot)], o.info.crop_left, o.info.crop_top, o.info.width,
                                o.info.height, u64(o.au.pts));
    if (s != ROCDEC_SUCCESS) return s;
  }
  return ROCDEC_SUCCESS;
}

rocDecStatus emit_hevc(StubParser& sp, const std::vector<hevc::FramePtr>& outs) {
  for (const hevc::FramePtr& f : outs) {
    const rocDecStatus s = emit(sp, f->s, f->crop_left, f->crop_top, f->width, f->height, u64(f->pts));
    if (s != ROCDEC_SUCCESS) return s;
  }
  return ROCDEC_SUCCESS;
}

}  // namespace

STUB_API rocDecStatus rocDecCreateVideoParser(RocdecVideoParser* h, RocdecParserParams* p) {
  if (!h || !p || !p->pfn_sequence_callback || !p->pfn_decode_picture || !p->pfn_display_picture)
    return ROCDEC_INVALID_PARAMETER;
  if (p->codec_type != rocDecVideoCodec_AVC && p->codec_type != rocDecVideoCodec_HEVC) return ROCDEC_NOT_SUPPORTED;
  auto* sp = new StubParser;
  sp->p = *p;
  *h = sp;
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecParseVideoData(RocdecVideoParser h, RocdecSourceDataPacket* pkt) {
  if (!h || !pkt) return ROCDEC_INVALID_PARAMETER;
  StubParser& sp = *static_cast<StubParser*>(h);
  const bool avc_codec = sp.p.codec_type == rocDecVideoCodec_AVC;
  try {
    if (pkt->flags & ROCDEC_PKT_ENDOFSTREAM) {
      rocDecStatus s = ROCDEC_SUCCESS;
      if (pkt->payload_size == 0) {
        if (avc_codec) s = emit_avc(sp, sp.avc.flush_output());
        else s = emit_hevc(sp, sp.hevc.flush());
      }
      if (sp.p.pfn_display_picture && (pkt->flags & ROCDEC_PKT_NOTIFY_EOS)) sp.p.pfn_display_picture(sp.p.user_data, nullptr);
      return s;
    }
    AccessUnit au;
    au.codec = avc_codec ? Codec::kH264 : Codec::kH265;
    au.pts = i64(pkt->pts);
    for (auto& [o, n] : h264::split_annexb(pkt->payload, pkt->payload_size)) {
      au.add_nal(pkt->payload + o, n);
      const u8 b = pkt->payload[o];
      au.keyframe |= avc_codec ? (b & 0x1F) == 5 : (((b >> 1) & 0x3F) >= 16 && ((b >> 1) & 0x3F) <= 21);
    }
    if (au.nals.empty()) return ROCDEC_SUCCESS;
    if (avc_codec) {
      avc::PicturePtr pic = sp.avc.parse(au);
      if (sp.avc_slots.size() < size_t(pic->dpb_slots)) sp.avc_slots.resize(size_t(pic->dpb_slots));
      for (auto& hs : sp.avc_slots)
        if (hs.coded_w != pic->wmbs * 16 || hs.coded_h != pic->hmbs * 16) hs.alloc(pic->wmbs * 16, pic->hmbs * 16);
      avc::cpu_reconstruct(*pic, sp.avc_slots);
      return emit_avc(sp, pic->outputs);
    }
    return emit_hevc(sp, sp.hevc.decode(au, 0));
  } catch (const std::exception&) {
    return ROCDEC_RUNTIME_ERROR;
  }
}

STUB_API rocDecStatus rocDecParserMarkFrameForReuse(RocdecVideoParser h, int idx) {
  if (!h) return ROCDEC_INVALID_PARAMETER;
  StubParser& sp = *static_cast<StubParser*>(h);
  if (idx < 0 || size_t(idx) >= sp.busy.size()) return ROCDEC_INVALID_PARAMETER;
  sp.busy[size_t(idx)] = false;
  ++sp.reuse_marks;
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecDestroyVideoParser(RocdecVideoParser h) {
  delete static_cast<StubParser*>(h);
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecCreateDecoder(rocDecDecoderHandle* h, RocDecoderCreateInfo* ci) {
  if (!h || !ci || ci->output_format != rocDecVideoSurfaceFormat_NV12 || ci->num_decode_surfaces == 0)
    return ROCDEC_INVALID_PARAMETER;
  auto d = std::make_unique<StubDecoder>();
  d->host = host_surfaces();
  d->w = int(ci->target_width);
  d->h = int(ci->target_height);
  d->pitch = (u32(d->w) + 255u) & ~255u;  // a pitched surface, as VCN output is
  if (!d->host && hipSetDevice(ci->device_id) != hipSuccess) return ROCDEC_DEVICE_INVALID;
  for (u32 i = 0; i < ci->num_decode_surfaces; ++i) {
    u8 *y = nullptr, *uv = nullptr;
    const size_t ny = size_t(d->pitch) * size_t(d->h), nuv = ny / 2;
    if (d->host) {
      y = static_cast<u8*>(std::malloc(ny));
      uv = static_cast<u8*>(std::malloc(nuv));
    } else if (hipMalloc(&y, ny) != hipSuccess || hipMalloc(&uv, nuv) != hipSuccess) {
      return ROCDEC_OUTOF_MEMORY;
    }
    d->y.push_back(y);
    d->uv.push_back(uv);
  }
  *h = d.release();
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecDestroyDecoder(rocDecDecoderHandle h) {
  delete static_cast<StubDecoder*>(h);
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecDecodeFrame(rocDecDecoderHandle h, RocdecPicParams* pp) {
  if (!h || !pp) return ROCDEC_INVALID_PARAMETER;
  StubDecoder& d = *static_cast<StubDecoder*>(h);
  const Pending pe = g_pending;
  if (!pe.s || pp->curr_pic_idx < 0 || size_t(pp->curr_pic_idx) >= d.y.size() || pe.width != d.w || pe.height != d.h)
    return ROCDEC_INVALID_PARAMETER;
  // the display area of the decoded picture into the pitched NV12 output surface
  const HostSurface& s = *pe.s;
  u8* y = d.y[size_t(pp->curr_pic_idx)];
  u8* uv = d.uv[size_t(pp->curr_pic_idx)];
  const u8* sy = s.y.data() + size_t(pe.crop_top) * s.coded_w + pe.crop_left;
  const u8* suv = s.uv.data() + size_t(pe.crop_top / 2) * s.coded_w + (pe.crop_left & ~1);
  if (d.host) {
    for (int r = 0; r < d.h; ++r) std::memcpy(y + size_t(r) * d.pitch, sy + size_t(r) * s.coded_w, size_t(d.w));
    for (int r = 0; r < d.h / 2; ++r) std::memcpy(uv + size_t(r) * d.pitch, suv + size_t(r) * s.coded_w, size_t(d.w));
    return ROCDEC_SUCCESS;
  }
  if (hipMemcpy2D(y, d.pitch, sy, size_t(s.coded_w), size_t(d.w), size_t(d.h), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy2D(uv, d.pitch, suv, size_t(s.coded_w), size_t(d.w), size_t(d.h / 2), hipMemcpyHostToDevice) != hipSuccess)
    return ROCDEC_RUNTIME_ERROR;
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecGetDecodeStatus(rocDecDecoderHandle h, int idx, RocdecDecodeStatus* st) {
  if (!h || !st) return ROCDEC_INVALID_PARAMETER;
  (void)idx;
  st->decode_status = rocDecodeStatus_Success;
  return ROCDEC_SUCCESS;
}

STUB_API rocDecStatus rocDecGetVideoFrame(rocDecDecoderHandle h, int idx, void* ptr[3], u32* pitch,
                                          RocdecProcParams* pp) {
  if (!h || !ptr || !pitch || !pp) return ROCDEC_INVALID_PARAMETER;
  StubDecoder& d = *static_cast<StubDecoder*>(h);
  if (idx < 0 || size_t(idx) >= d.y.size()) return ROCDEC_INVALID_PARAMETER;
  ptr[0] = d.y[size_t(idx)];
  ptr[1] = d.uv[size_t(idx)];
  ptr[2] = nullptr;
  pitch[0] = pitch[1] = d.pitch;
  pitch[2] = 0;
  return ROCDEC_SUCCESS;
}

STUB_API const char* rocDecGetErrorName(rocDecStatus s) {
  switch (s) {
    case ROCDEC_SUCCESS: return "ROCDEC_SUCCESS";
    case ROCDEC_INVALID_PARAMETER: return "ROCDEC_INVALID_PARAMETER";
    case ROCDEC_RUNTIME_ERROR: return "ROCDEC_RUNTIME_ERROR";
    case ROCDEC_OUTOF_MEMORY: return "ROCDEC_OUTOF_MEMORY";
    case ROCDEC_NOT_SUPPORTED: return "ROCDEC_NOT_SUPPORTED";
    case ROCDEC_DEVICE_INVALID: return "ROCDEC_DEVICE_INVALID";
    default: return "ROCDEC_ERROR";
  }
}
