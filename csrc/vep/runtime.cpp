// Data-plane runtime implementation. See runtime.h.
#include "runtime.h"

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <csignal>
#include <cstdio>
#include <map>
#include <thread>

#include "color.h"
#include "trace.h"

namespace vep {

// ------------------------------------------------------------------------------------ Device

Device::Device(int id) : id_(id) {
  if (id_ >= 0) {
    int n = gpu::device_count();
    VEP_CHECK(id_ < n, "GPU " + std::to_string(id_) + " not present (" + std::to_string(n) +
                           " visible)");
    bind();
  }
}
Device::~Device() = default;

void Device::bind() const {
  if (id_ >= 0) VEP_HIP(hipSetDevice(id_));
}

void* Device::alloc(size_t n) {
  n = std::max<size_t>(n, 256);
  if (!gpu()) {
    void* p = std::aligned_alloc(256, (n + 255) & ~size_t(255));
    VEP_CHECK(p, "host alloc failed");
    return p;
  }
  void* p = nullptr;
  VEP_HIP(hipMalloc(&p, n));
  return p;
}
void Device::free(void* p) {
  if (!p) return;
  if (!gpu()) std::free(p);
  else (void)hipFree(p);
}
void* Device::alloc_pinned(size_t n) {
  n = std::max<size_t>(n, 256);
  if (!gpu()) return alloc(n);
  void* p = nullptr;
  VEP_HIP(hipHostMalloc(&p, n, hipHostMallocDefault));
  return p;
}
void Device::free_pinned(void* p) {
  if (!p) return;
  if (!gpu()) std::free(p);
  else (void)hipHostFree(p);
}

// --------------------------------------------------------------------------------- FrameRing

FrameRing::FrameRing(Device& dev, int slots, int width, int height)
    : dev_(dev), w_(width), h_(height) {
  VEP_CHECK(slots >= 1 && slots <= 4096, "ring slots out of range");
  base_ = static_cast<u8*>(dev_.alloc(slot_bytes() * size_t(slots)));
  for (int i = 0; i < slots; ++i) slots_.emplace_back(std::make_unique<Slot>());
}
FrameRing::~FrameRing() { dev_.free(base_); }

int FrameRing::begin_write() {
  std::lock_guard<std::mutex> g(meta_mu_);
  // never overwrite the newest committed frame or a slot an in-flight batch is writing
  const int n = int(slots_.size());
  int s = next_;
  for (int k = 0; k < n; ++k) {
    const int c = (next_ + k) % n;
    if ((n == 1 || c != latest_.load()) && !(slots_[c]->version.load() & 1)) {
      s = c;
      break;
    }
  }
  next_ = (s + 1) % n;
  slots_[s]->version.fetch_add(1, std::memory_order_acq_rel);  // odd: being written
  return s;
}

void FrameRing::commit(int slot, FrameMeta meta) {
  {
    std::lock_guard<std::mutex> g(meta_mu_);
    meta.seq = published_.load() + 1;
    slots_[slot]->meta = meta;
    slots_[slot]->version.fetch_add(1, std::memory_order_acq_rel);  // even: stable
    latest_.store(slot, std::memory_order_release);
    published_.store(meta.seq, std::memory_order_release);
  }
  cv_.notify_all();
}

void FrameRing::abort(int slot) {
  std::lock_guard<std::mutex> g(meta_mu_);
  if (slots_[slot]->version.load() & 1) slots_[slot]->version.fetch_add(1, std::memory_order_acq_rel);
}

bool FrameRing::wait_newer(i64 after, int timeout_ms) const {
  std::unique_lock<std::mutex> g(meta_mu_);
  return cv_.wait_for(g, std::chrono::milliseconds(timeout_ms),
                      [&] { return published_.load() > after; });
}

bool FrameRing::latest(i64 after, FrameMeta* meta, int* slot) const {
  std::lock_guard<std::mutex> g(meta_mu_);
  int s = latest_.load();
  if (s < 0) return false;
  const Slot& sl = *slots_[s];
  if ((sl.version.load() & 1) || sl.meta.seq <= after) return false;
  *meta = sl.meta;
  *slot = s;
  return true;
}

bool FrameRing::still_valid(int slot, i64 seq) const {
  std::lock_guard<std::mutex> g(meta_mu_);
  const Slot& sl = *slots_[slot];
  return !(sl.version.load() & 1) && sl.meta.seq == seq;
}

// ----------------------------------------------------------------------------------- LogRing

void LogRing::add(bool err, std::string line) {
  std::lock_guard<std::mutex> g(mu_);
  auto& q = err ? err_ : out_;
  q.push_back(std::move(line));
  while (q.size() > 1000) q.pop_front();
}

std::string LogRing::dump(bool err, size_t last) const {
  std::lock_guard<std::mutex> g(mu_);
  const auto& q = err ? err_ : out_;
  std::string s;
  size_t start = q.size() > last ? q.size() - last : 0;
  for (size_t i = start; i < q.size(); ++i) {
    s += q[i];
    s += '\n';
  }
  return s;
}

// ------------------------------------------------------------------------------------ Camera

Camera::Camera(Worker& w, int index, std::string name, int ring_slots)
    : ring_slots_cfg(ring_slots), w_(w), index_(index), name_(std::move(name)), use_vcn_(w.vcn()) {
  // Fault injection (tests of per-camera-group containment): VEP_FAULT_CAMERA=<name>[:<n>] makes
  // this camera's n-th access unit (default 1) crash the process inside its parse, as a bug in
  // the bitstream parser hit by a hostile stream would.
  if (const char* f = std::getenv("VEP_FAULT_CAMERA")) {
    const std::string spec(f);
    const size_t colon = spec.rfind(':');
    const std::string who = colon == std::string::npos ? spec : spec.substr(0, colon);
    if (who == name_) fault_after_ = colon == std::string::npos ? 1 : std::max<u64>(1, std::strtoull(f + colon + 1, nullptr, 10));
  }
}

std::vector<AuPtr> Camera::gop_snapshot() {
  std::lock_guard<std::mutex> g(mu_);
  return gop_;
}

// VCN backend: the AUs go to the camera's rocDecode session; the newest picture that reached
// display order is published (older ones of a catch-up run are released at once, as the native
// path collapses them).
bool Camera::build_vcn_job(DecodeJob& job, size_t from, size_t to) {
  job.cam = index_;
  job.refresh = true;  // a complete picture: the surface is rewritten whole
  vcn::FramePtr out;
  try {
    if (!vcn_) {
      const int dev = w_.device().gpu() ? w_.device().id() : 0;
      vcn_ = std::make_unique<vcn::Session>(gop_[from]->codec, dev);
      logs.add(false, std::string("VCN decoder session opened (") + vcn::library() + ")");
    }
    const bool key_only = keyframe_only.load() && to - from == 1 && gop_[from]->keyframe;
    for (size_t i = from; i < to; ++i) {
      std::vector<vcn::FramePtr> fs = vcn_->decode(*gop_[i], i64(i));
      if (!fs.empty()) out = fs.back();
    }
    if (key_only) {  // nothing else of the GOP is decoded: drain the reorder queue
      std::vector<vcn::FramePtr> fs = vcn_->flush();
      if (!fs.empty()) out = fs.back();
    }
  } catch (const std::exception& e) {
    errors.fetch_add(1);
    logs.add(true, std::string("VCN decode failed: ") + e.what());
    decoded_upto_ = gop_.size();  // wait for the next keyframe
    if (vcn_) {
      try {
        vcn_->flush();
      } catch (const std::exception&) {
        vcn_.reset();  // a fresh session at the next keyframe
      }
    }
    return false;
  }
  decoded_upto_ = to;
  if (!out) return false;  // reordering: nothing reached display order yet
  job.ext = out;
  PictureInfo& pi = job.pic;
  pi = PictureInfo{};
  pi.width = out->width;
  pi.height = out->height;
  pi.coded_width = (out->width + 15) & ~15;
  pi.coded_height = (out->height + 15) & ~15;
  pi.pict_type = out->type;
  pi.idr = out->keyframe;
  FrameMeta& m = job.meta;
  m.width = out->width;
  m.height = out->height;
  m.pts = out->pts;
  m.dts = out->dts;
  m.timestamp = out->pts;
  m.packet = out->tag;
  m.keyframe = keyframes_;
  m.is_keyframe = out->keyframe;
  m.is_corrupt = out->corrupt;
  m.frame_type = out->type;
  m.arrival_ms = gop_[to - 1]->arrival_ms;
  return true;
}

bool Camera::build_job(DecodeJob& job, size_t from, size_t to, bool refresh) {
  job.keyframe_only = keyframe_only.load(std::memory_order_relaxed);
  if (use_vcn_) return build_vcn_job(job, from, to);
  job.cam = index_;
  job.refresh = refresh;
  const AccessUnit* last = nullptr;
  try {
    if (!full_ && !hevc_full_) {
      try {
        for (size_t i = from; i < to; ++i) {
          // single-AU jobs may take the header-free I-slice walk: the worker verifies the
          // skipped headers on the GPU (or CPU) before it publishes the frame
          job.pic = parser_.parse(*gop_[i], job.upd, to - from == 1);
          job.upd.keep.push_back(gop_[i]);  // MB samples are referenced in place
          last = gop_[i].get();
        }
      } catch (const UnsupportedStream& e) {
        if (!gop_[0]->keyframe) throw;
        // The stream uses syntax beyond the I_PCM / P_Skip fast path: switch this camera to the
        // general decoder for good and rebuild the job from the GOP's keyframe (the general
        // decoder needs the whole reference history of the GOP).
        const bool h264 = gop_[from]->codec == Codec::kH264;
        (h264 ? full_ : hevc_full_) = true;
        logs.add(false, std::string(h264 ? "general H.264" : "general H.265") + " decoder enabled (" + e.what() + ")");
        job.upd = MbUpdate{};
        from = 0;
        job.refresh = true;
      }
    }
    if (hevc_full_) {
      hevc_.set_gpu_mode(true);
      hevc::FramePtr of;
      const bool key_only = keyframe_only.load() && to - from == 1 && gop_[from]->keyframe;
      for (size_t i = from; i < to; ++i) {
        std::vector<hevc::FramePtr> outs = hevc_.decode(*gop_[i], i64(i));
        if (key_only) {  // nothing else of the GOP is decoded: take the picture out right away
          std::vector<hevc::FramePtr> rest = hevc_.flush();
          outs.insert(outs.end(), rest.begin(), rest.end());
        }
        for (auto& p : hevc_.take_gpu_pictures()) job.hevc.push_back(std::move(p));
        if (!outs.empty()) of = outs.back();
        last = gop_[i].get();
      }
      decoded_upto_ = to;
      if (job.hevc.empty()) return false;
      for (const auto& p : job.hevc)  // (a size change starts a new coded video sequence)
        VEP_CHECK(p->width == job.hevc.back()->width && p->height == job.hevc.back()->height,
                  "HEVC: pictures of different sizes in one decode job");
      job.hevc_slots = hevc_.gpu_slots();
      const hevc::GpuPicture& gp = *job.hevc.back();
      PictureInfo& pi = job.pic;
      pi = PictureInfo{};
      pi.coded_width = (gp.width + 15) & ~15;  // surfaces keep the 16-aligned pitch of the convert kernels
      pi.coded_height = (gp.height + 15) & ~15;
      pi.width = of ? of->width : gp.width;
      pi.height = of ? of->height : gp.height;
      job.out_slot = of ? of->slot : -1;
      job.out_rasl_of = of ? of->rasl_of : -1;
      if (!of) return true;  // reordering: reconstruct only, nothing leaves the DPB yet
      pi.crop_left = of->crop_left;
      pi.crop_top = of->crop_top;
      pi.pict_type = of->type;
      pi.idr = of->keyframe;
      FrameMeta& m = job.meta;
      m.width = of->width;
      m.height = of->height;
      m.pts = of->pts;
      m.dts = of->dts;
      m.timestamp = of->pts;
      m.packet = of->tag;
      m.keyframe = keyframes_;
      m.is_keyframe = of->keyframe;
      m.is_corrupt = false;
      m.frame_type = of->type;
      m.arrival_ms = last->arrival_ms;
      return true;
    }
    if (full_) {
      for (size_t i = from; i < to; ++i) {
        size_t nal = 0;  // (a field pair may come as one access unit: one picture per field)
        do job.avc.push_back(avc_.parse(*gop_[i], i64(i), &nal));
        while (nal < gop_[i]->nals.size());
        last = gop_[i].get();
      }
      job.pic = job.avc.back()->info;
      // the newest picture that left the reorder buffer during this job is the one published
      const avc::OutFrame* of = nullptr;
      for (const auto& p : job.avc)
        if (!p->outputs.empty()) of = &p->outputs.back();
      job.out_slot = of ? of->slot : -1;
      job.out_fields = of && of->fields;
      if (of) {
        job.pic = of->info;
        FrameMeta& m = job.meta;
        m.width = of->info.width;
        m.height = of->info.height;
        m.pts = of->au.pts;
        m.dts = of->au.dts;
        m.timestamp = of->au.pts;
        m.packet = of->au.tag;
        m.keyframe = keyframes_;
        m.is_keyframe = of->au.keyframe;
        m.is_corrupt = of->au.corrupt;
        m.frame_type = of->info.pict_type;
        m.arrival_ms = last->arrival_ms;  // latency: from the packet that completed the output
        decoded_upto_ = to;
        return true;
      }
    }
  } catch (const std::exception& e) {
    errors.fetch_add(1);
    logs.add(true, std::string("failed to decode packet: ") + e.what());
    if (full_) avc_.reset_references();
    decoded_upto_ = gop_.size();  // give up on this GOP; wait for the next keyframe
    return false;
  }
  FrameMeta& m = job.meta;
  m.width = job.pic.width;
  m.height = job.pic.height;
  m.pts = last->pts;
  m.dts = last->dts;
  m.timestamp = last->pts;  // int(frame.time * time_base.denominator) with tb = 1/90000
  m.packet = i64(to - 1);
  m.keyframe = keyframes_;
  m.is_keyframe = last->keyframe;
  m.is_corrupt = last->corrupt;
  m.frame_type = job.pic.pict_type;
  m.arrival_ms = last->arrival_ms;
  decoded_upto_ = to;
  return true;
}

bool Camera::on_access_unit(const AuPtr& au) {
  DecodeJob job;
  {
    std::lock_guard<std::mutex> g(mu_);
    const u64 np = packets.fetch_add(1, std::memory_order_relaxed) + 1;
    if (fault_after_ && np >= fault_after_) {  // (VEP_FAULT_CAMERA, see the constructor)
      std::fprintf(stderr, "vep: injected fault in camera %s's parse (access unit %llu)\n", name_.c_str(),
                   static_cast<unsigned long long>(np));
      std::fflush(stderr);
      std::raise(SIGSEGV);
    }
    bytes_in.fetch_add(au->bytes(), std::memory_order_relaxed);
    last_packet_ms.store(au->arrival_ms ? au->arrival_ms : now_ms());
    if (au->keyframe) {
      gop_.clear();
      decoded_upto_ = 0;
      ++keyframes_;
    }
    if (gop_.empty() && !au->keyframe) {  // rtsp_to_rtmp.py:111-114 "skipping, since not a keyframe"
      skipped.fetch_add(1, std::memory_order_relaxed);
      if (parser_.has_sps() == false) parser_.absorb_parameter_sets(*au);
      return false;
    }
    gop_.push_back(au);
    const i64 lq = last_query_ms.load();
    if (lq == 0) return false;                            // no last_query yet
    if (now_ms() - lq >= idle_cutoff_ms.load()) return false;  // idle > 10 s: stop decoding
    size_t to = gop_.size();
    if (keyframe_only.load()) {
      if (decoded_upto_ > 0) return false;  // keyframe already reconstructed
      to = 1;
    }
    if (decoded_upto_ >= to) return false;
    const size_t from = decoded_upto_;
    if (!build_job(job, from, to, from == 0 && gop_[0]->keyframe)) return false;
  }
  w_.submit(std::move(job));
  return true;
}

void Camera::decode_now(const AuPtr& au) {
  DecodeJob job;
  if (make_job(au, job)) w_.submit(std::move(job));
}

bool Camera::make_job(const AuPtr& au, DecodeJob& job) {
  {
    std::lock_guard<std::mutex> g(mu_);
    packets.fetch_add(1, std::memory_order_relaxed);
    bytes_in.fetch_add(au->bytes(), std::memory_order_relaxed);
    if (au->keyframe) {
      gop_.clear();
      decoded_upto_ = 0;
      ++keyframes_;
    }
    if (gop_.empty() && !au->keyframe) return false;
    gop_.push_back(au);
    size_t from = decoded_upto_, to = gop_.size();
    return build_job(job, from, to, from == 0);
  }
}

// ------------------------------------------------------------------------------------ Worker

// Lanes per GPU worker (WorkerOptions::lanes): lane streams + the serving stream fit the
// default 4 hardware queues per process.
constexpr int kDefaultLanes = 3;
// Batches in flight per lane: one slow batch (a keyframe's intra wavefront) then blocks the
// launching thread only after the other lanes have this many batches queued.
constexpr int kDefaultStages = 3;
// Batches queued per lane launcher thread behind the in-flight ones.
constexpr int kDefaultLaneQueue = 2;
constexpr int kDefaultLaneMergeJobs = 64;  // jobs per merged lane launch (lane launcher threads)
constexpr int kDefaultKfWindowUs = 16000;  // keyframe-only coalescing window (see WorkerOptions)
constexpr int kAllLevels = 1 << 20;        // (a window holding every level of a round)
// H.265 intra transform blocks: one launch per intra level (kernel boundaries order the levels;
// no wave ever polls). kAllLevels (VEP_HEVC_TU_QUEUE=1) = one persistent ticket-queue launch per
// round (waves take blocks in level order and poll their neighbours' edge words), k = windows of
// k levels, -1 = one workgroup per picture. Round 6, GPU-side ceiling of 8 x 4K H.265 (--source
// records, three alternated runs, profiles/r6/hevc_tu/): per-level 2,199 / 2,183 / 2,187
// pictures/s, GPU 91-93 ms per step; queue 2,087 / 2,068 / 2,052, 94-99 ms; per-picture 353-362.
// The queue's ~150x fewer launches do not pay for its polling (84% of its wave-cycles waiting,
// round 5 counters), so per-level launches are the default again.
constexpr int kDefaultTuWindow = 0;

Worker::Worker(const WorkerOptions& o) : opt_(o), dev_(o.device) {
  mock_serve_ = !dev_.gpu() && (opt_.mock_serve || (std::getenv("VEP_MOCK_SERVE") && std::getenv("VEP_MOCK_SERVE")[0] == '1'));
  if (opt_.decoder == kDecoderVcn)
    VEP_CHECK(vcn::available(), "decoder backend 'vcn' requested but rocDecode is unavailable: " + vcn::load_error());
  vcn_ = opt_.decoder == kDecoderVcn || (opt_.decoder == kDecoderAuto && vcn::available());
  if (dev_.gpu()) {
    dev_.bind();
    int nl = opt_.lanes;
    if (nl <= 0) {
      const char* le = std::getenv("VEP_LANES");
      nl = le ? std::atoi(le) : kDefaultLanes;
    }
    nl = std::clamp(nl, 1, 16);
    for (int g = 0; g < nl; ++g) lanes_.push_back(std::make_unique<Lane>());
    // Launcher thread per lane: opt-in (measured no steadier than the single launching thread
    // at the default 3 lanes, whose batches are bound by per-picture wavefront latency).
    const char* lt = std::getenv("VEP_LANE_THREADS");
    threaded_ = nl > 1 && (opt_.lane_threads || (lt && lt[0] == '1'));
    int nq = opt_.queue;
    if (nq <= 0) {
      const char* qe = std::getenv("VEP_LANE_QUEUE");
      nq = qe ? std::atoi(qe) : kDefaultLaneQueue;
    }
    queue_ = std::clamp(nq, 1, 16);
    // lane launchers merge queued batches (merge_queued); VEP_LANE_MERGE = job cap, 0 = off
    const char* me = std::getenv("VEP_LANE_MERGE");
    merge_jobs_ = std::clamp(me ? std::atoi(me) : kDefaultLaneMergeJobs, 0, 4096);
    int kw = opt_.kf_window_us;
    if (kw < 0) {
      const char* ke = std::getenv("VEP_KF_WINDOW_US");
      kw = ke ? std::atoi(ke) : kDefaultKfWindowUs;
    }
    kf_window_us_ = std::clamp(kw, 0, 100000);
    // H.265 intra transform blocks: one launch per level (VEP_HEVC_TU_QUEUE=0), one queue launch
    // per round (=1), or one queue launch per window of k levels (VEP_HEVC_TU_WINDOW=k)
    polite_wait_ = !(std::getenv("VEP_SPIN_WAIT") && std::getenv("VEP_SPIN_WAIT")[0] == '1');
    hevc_tu_window_ = kDefaultTuWindow;
    if (const char* tq = std::getenv("VEP_HEVC_TU_QUEUE")) hevc_tu_window_ = tq[0] == '1' ? kAllLevels : 0;
    if (const char* tw = std::getenv("VEP_HEVC_TU_WINDOW")) hevc_tu_window_ = std::clamp(std::atoi(tw), -1, kAllLevels);
    // (queue waits: longest polling nap, x 256 cycles; 1 = round 4's fixed poll)
    if (const char* tn = std::getenv("VEP_HEVC_TU_NAP")) hevc_tu_nap_ = u32(std::clamp(std::atoi(tn), 1, 256));
    int ns = opt_.stages;
    if (ns <= 0) {
      const char* se = std::getenv("VEP_STAGES");
      ns = se ? std::atoi(se) : kDefaultStages;
    }
    stages_ = std::clamp(ns, 2, 8);
    // Streams map onto the process's few hardware queues (GPU_MAX_HW_QUEUES): create only the
    // ones in use, serving first so its D2H never queues behind a lane's kernels.
    VEP_HIP(hipStreamCreateWithFlags(&serve_stream_, hipStreamNonBlocking));
    VEP_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    if (lanes_.size() == 1) {
      // The copy stream's gather kernel is PCIe-latency bound and must keep its waves resident
      // while the previous batch's decode kernel floods the CUs: give it dispatch priority.
      int prio_lo = 0, prio_hi = 0;
      VEP_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
      VEP_HIP(hipStreamCreateWithPriority(&copy_stream_, hipStreamNonBlocking, prio_hi));
    }
    for (size_t g = 0; g < lanes_.size(); ++g) {
      Lane& ln = *lanes_[g];
      if (g == 0) ln.stream = stream_;
      else VEP_HIP(hipStreamCreateWithFlags(&ln.stream, hipStreamNonBlocking));
      // VEP_LANE_COPY=1 (several lanes): each lane gets its own copy stream, so a batch's MB
      // records / coefficients cross PCIe while the lane's previous batch is still decoding
      // (3 lanes use 7 streams, within the 8 hardware queues bench.py / the package ask for).
      // Otherwise (the default) the copy goes on the lane's own stream: measured faster on
      // 32x1080p (10.7k vs 7.5k fps/GPU, gpurun sweep), cause not yet profiled.
      const char* lc = std::getenv("VEP_LANE_COPY");
      if (lanes_.size() > 1 && lc && std::atoi(lc) == 1)
        VEP_HIP(hipStreamCreateWithFlags(&ln.copy, hipStreamNonBlocking));
      ln.stage.resize(size_t(stages_));
      for (Stage& st : ln.stage) {
        VEP_HIP(hipEventCreateWithFlags(&st.copied, hipEventDisableTiming));
        VEP_HIP(hipEventCreate(&st.e0));
        // waiters sleep instead of spinning: several lane threads wait at once and share the
        // CPUs with the parse threads
        VEP_HIP(hipEventCreateWithFlags(&st.e1, threaded_ ? hipEventBlockingSync : hipEventDefault));
      }
    }
    hostmem::enable_pool();  // AUs finalised from here on are GPU-readable in place
    const char* ap = std::getenv("VEP_AVC_PROF");
    if (ap && ap[0] == '1') {
      avc_prof_ = static_cast<u64*>(dev_.alloc(gpu::kAvcProfSlots * sizeof(u64)));
      VEP_HIP(hipMemset(avc_prof_, 0, gpu::kAvcProfSlots * sizeof(u64)));
    }
    const char* dp = std::getenv("VEP_DBK_PACKED");
    const char* ds = std::getenv("VEP_DBK_SYNC");  // 1: a wave sync after every edge (A/B)
    const char* dg = std::getenv("VEP_DBK_REGS");  // 0: round 4's per-edge LDS lines (A/B)
    dbk_packed_ = ((dp && dp[0] == '0') ? 0 : 1) | ((ds && ds[0] == '1') ? 2 : 0) | ((dg && dg[0] == '0') ? 0 : 4);
    const char* dr = std::getenv("VEP_DIRECT_READS");
    direct_reads_ = opt_.direct_reads && !(dr && dr[0] == '0');
  }
  if (opt_.pack_threads > 0 && !threaded_) pack_pool_ = std::make_unique<ThreadPool>(opt_.pack_threads, domain_thread_init(opt_.domain, nullptr));
  if (!dev_.gpu()) {
    const int n = opt_.domain.cpu_share > 0 ? opt_.domain.cpu_share : std::max(1, int(std::thread::hardware_concurrency()) / 2);
    if (n > 1) cpu_pool_ = std::make_unique<ThreadPool>(n, domain_thread_init(opt_.domain, nullptr));
  }
  if (threaded_)
    for (auto& lp : lanes_) {
      Lane* ln = lp.get();
      ln->th = std::thread([this, ln] {
        name_thread("vep-lane");
        pin_current_thread(opt_.domain.cpus);
        lane_loop(*ln);
      });
    }
  cams_.reserve(size_t(opt_.max_cameras));
  if (opt_.letterbox_size > 0) {
    const size_t S = size_t(opt_.letterbox_size);
    (void)S;
    cons_hwc_ = static_cast<u8*>(dev_.alloc(
        size_t(opt_.max_cameras) * gpu::letterbox_bytes(opt_.letterbox_size, opt_.letterbox_format)));
    size_t es = opt_.chw_dtype == gpu::kChwF32 ? 4 : 2;
    if (opt_.chw_dtype != gpu::kChwNone)
      cons_chw_ = dev_.alloc(size_t(opt_.max_cameras) * 3 * S * S * es);
    cons_rows_ = opt_.max_cameras;
  }
}

void Worker::set_consumer_buffers(u8* hwc, void* chw, int rows) {
  std::lock_guard<std::mutex> lg(launch_mu_);
  VEP_CHECK(opt_.letterbox_size > 0, "worker was built without a letterbox consumer batch");
  if (owns_cons_) {
    if (dev_.gpu()) {
      dev_.bind();
      complete_locked();  // batches in flight still write the worker-owned buffers
    }
    dev_.free(cons_hwc_);
    dev_.free(cons_chw_);
  }
  owns_cons_ = false;
  cons_hwc_ = hwc;
  cons_chw_ = chw;
  cons_rows_ = rows;
}

Worker::~Worker() {
  stop();
  try {
    complete_all();
  } catch (...) {
  }
  std::lock_guard<std::mutex> g(cams_mu_);
  for (auto& c : cams_) {
    if (!c) continue;
    dev_.free(c->surface.y);
    dev_.free(c->surface.uv);
    dev_.free(c->surface.y8);
    dev_.free(c->surface.uv8);
    dev_.free(c->surface.hevc_xg);
    c->set_ring(nullptr);
  }
  if (owns_cons_) {
    dev_.free(cons_hwc_);
    dev_.free(cons_chw_);
  }
  for (auto& lp : lanes_) {
    Lane& ln = *lp;
    {
      std::lock_guard<std::mutex> g(ln.mu);
      ln.stop = true;
    }
    ln.cv.notify_all();
    if (ln.th.joinable()) ln.th.join();
  }
  for (auto& lp : lanes_) {
    Lane& ln = *lp;
    for (Stage& st : ln.stage) {
      dev_.free_pinned(st.err);
      if (st.h) hostmem::unregister_range(st.h);
      dev_.free(st.d);
      dev_.free_pinned(st.h);
      if (st.copied) (void)hipEventDestroy(st.copied);
      if (st.e0) (void)hipEventDestroy(st.e0);
      if (st.e1) (void)hipEventDestroy(st.e1);
    }
    if (ln.stream && ln.stream != stream_) (void)hipStreamDestroy(ln.stream);
    if (ln.copy) (void)hipStreamDestroy(ln.copy);
    if (ln.snap_mark) (void)hipEventDestroy(ln.snap_mark);
  }
  if (snap_ev_) (void)hipEventDestroy(snap_ev_);
  for (auto& b : serve_all_) {
    dev_.free_pinned(b->h);
    for (hipEvent_t e : b->ev)
      if (e) (void)hipEventDestroy(e);
  }
  dev_.free(avc_prof_);
  if (stream_) (void)hipStreamDestroy(stream_);
  if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
  if (serve_stream_) (void)hipStreamDestroy(serve_stream_);
}

int Worker::add_camera(const std::string& name, int ring_slots) {
  std::lock_guard<std::mutex> g(cams_mu_);
  for (auto& c : cams_)
    VEP_CHECK(!c || c->name() != name, "camera already registered: " + name);
  int idx = -1;
  for (size_t i = 0; i < cams_.size(); ++i)
    if (!cams_[i]) { idx = int(i); break; }
  if (idx < 0) {
    VEP_CHECK(int(cams_.size()) < opt_.max_cameras, "worker camera capacity exhausted");
    idx = int(cams_.size());
    cams_.emplace_back();
  }
  // `stages` batches may be in flight on the GPU (+ the lane thread's queue and the batch it is
  // launching): keep one more slot so the newest committed frame stays readable meanwhile
  const int min_slots = dev_.gpu() ? inflight() + (threaded_ ? 2 : 1) : 1;
  cams_[size_t(idx)] = std::make_shared<Camera>(*this, idx, name, std::max(min_slots, ring_slots));
  return idx;
}

void Worker::remove_camera(int idx) {
  flush();
  complete_all();
  std::lock_guard<std::mutex> lg(launch_mu_);
  std::lock_guard<std::mutex> g(cams_mu_);
  VEP_CHECK(idx >= 0 && idx < int(cams_.size()) && cams_[size_t(idx)], "no such camera");
  auto& c = cams_[size_t(idx)];
  dev_.free(c->surface.y);
  dev_.free(c->surface.uv);
  dev_.free(c->surface.y8);
  dev_.free(c->surface.uv8);
  dev_.free(c->surface.hevc_xg);
  c.reset();
}

std::shared_ptr<IngestServices> Worker::ingest_services() {
  std::lock_guard<std::mutex> g(svc_mu_);
  if (auto s = svc_.lock()) return s;
  auto s = opt_.domain.parse_threads > 0 ? std::make_shared<IngestServices>(opt_.domain) : IngestServices::acquire();
  svc_ = s;
  return s;
}

int Worker::ingest_parse_threads() {
  std::lock_guard<std::mutex> g(svc_mu_);
  auto s = svc_.lock();
  return s ? s->parse_threads : 0;
}

std::shared_ptr<Camera> Worker::camera(int idx) {
  std::lock_guard<std::mutex> g(cams_mu_);
  if (idx < 0 || idx >= int(cams_.size())) return nullptr;
  return cams_[size_t(idx)];
}

std::shared_ptr<Camera> Worker::find(const std::string& name) {
  std::lock_guard<std::mutex> g(cams_mu_);
  for (auto& c : cams_)
    if (c && c->name() == name) return c;
  return nullptr;
}

int Worker::num_cameras() const {
  std::lock_guard<std::mutex> g(cams_mu_);
  int n = 0;
  for (auto& c : cams_) n += c ? 1 : 0;
  return n;
}

void Worker::start() {
  std::lock_guard<std::mutex> g(q_mu_);
  if (running_) return;
  running_ = true;
  stop_ = false;
  th_ = std::thread([this] {
    name_thread("vep-worker");
    pin_current_thread(opt_.domain.cpus);
    loop();
  });
}

void Worker::stop() {
  {
    std::lock_guard<std::mutex> g(q_mu_);
    if (!running_) return;
    stop_ = true;
  }
  q_cv_.notify_all();
  taken_cv_.notify_all();
  if (th_.joinable()) th_.join();
  std::lock_guard<std::mutex> g(q_mu_);
  running_ = false;
}

static void fold_update(MbUpdate& into, const MbUpdate& from) {
  VEP_CHECK(into.width_mbs == from.width_mbs && into.height_mbs == from.height_mbs,
            "fold size mismatch");
  for (int mb = 0; mb < from.mbs(); ++mb) {
    int s = from.slot[size_t(mb)];
    if (s < 0) continue;
    into.set_in(mb, from.block(s), u32(into.segs.size()) + from.slot_seg[size_t(s)]);
  }
  into.segs.insert(into.segs.end(), from.segs.begin(), from.segs.end());
  into.keep.insert(into.keep.end(), from.keep.begin(), from.keep.end());
  into.own.insert(into.own.end(), from.own.begin(), from.own.end());
  into.frames += from.frames;
}

// Whether one of the job's own pictures reconstructs its output slot.
static bool reconstructs_output(const DecodeJob& j) {
  for (const auto& p : j.avc)
    if ((p->structure ? p->target / 2 : p->target) == j.out_slot) return true;
  for (const auto& p : j.hevc)
    if (p->target == j.out_slot) return true;
  return false;
}

void merge_job(DecodeJob& p, DecodeJob&& job) {
  VEP_CHECK(p.cam == job.cam, "merge_job: different cameras");
  // collapse into the not-yet-launched job: latest writer wins per macroblock (fast path);
  // general-path pictures are appended (each references the previous ones)
  if (job.general() && p.general() && job.refresh) {
    // A backlog that reaches a keyframe restarts from it (load shedding: the queued pictures are
    // dropped). The keyframe bumps the previous GOP's pictures out of the reorder buffer; when the
    // frame it would publish is one of those, its reconstruction was in the dropped job, so the
    // merged job only reconstructs (the keyframe's picture is published by a later job).
    // (H.265 open GOPs: the RASL pictures of a CRA predict from the previous GOP, whose dropped
    // pictures are never reconstructed; they are not published either)
    std::vector<std::pair<int, i64>> dropped = std::move(p.dropped);
    std::vector<i64> poisoned = std::move(p.poisoned_cra);
    for (const auto& pic : p.avc) dropped.emplace_back(pic->structure ? pic->target / 2 : pic->target, pic->au.pts);
    for (const auto& pic : p.hevc) dropped.emplace_back(pic->target, pic->pts);
    const bool lost = !p.hevc.empty();
    p = std::move(job);
    if (lost)
      for (const auto& pic : p.hevc)
        if (pic->cra) poisoned.push_back(pic->tag);
    p.dropped.insert(p.dropped.begin(), dropped.begin(), dropped.end());
    p.poisoned_cra.insert(p.poisoned_cra.begin(), poisoned.begin(), poisoned.end());
    if (p.out_slot >= 0 && !reconstructs_output(p)) {
      p.out_slot = -1;
      p.out_fields = false;
    }
  } else if (job.general() && p.general()) {
    p.avc.insert(p.avc.end(), job.avc.begin(), job.avc.end());
    p.hevc.insert(p.hevc.end(), job.hevc.begin(), job.hevc.end());
    p.hevc_slots = std::max(p.hevc_slots, job.hevc_slots);
    if (job.out_slot >= 0 || p.out_slot < 0) {  // the newer output wins; none keeps the older
      p.pic = job.pic;
      p.meta = job.meta;
      p.out_slot = job.out_slot;
      p.out_fields = job.out_fields;
      p.out_rasl_of = job.out_rasl_of;
    }
    p.dropped.insert(p.dropped.end(), job.dropped.begin(), job.dropped.end());
    p.poisoned_cra.insert(p.poisoned_cra.end(), job.poisoned_cra.begin(), job.poisoned_cra.end());
  } else if (job.refresh || job.general() != p.general() || p.upd.width_mbs != job.upd.width_mbs ||
             p.upd.height_mbs != job.upd.height_mbs) {
    p = std::move(job);
  } else {
    fold_update(p.upd, job.upd);
    p.pic = job.pic;
    p.meta = job.meta;
  }
}

void Worker::submit(DecodeJob&& job) {
  {
    std::lock_guard<std::mutex> g(q_mu_);
    for (auto& p : pending_) {
      if (p.cam != job.cam) continue;
      merge_job(p, std::move(job));
      q_cv_.notify_one();
      return;
    }
    pending_.push_back(std::move(job));
  }
  q_cv_.notify_one();
}

void Worker::wait_camera_taken(int cam, int timeout_ms) {
  std::unique_lock<std::mutex> g(q_mu_);
  taken_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] {
    if (stop_) return true;
    for (const DecodeJob& p : pending_)
      if (p.cam == cam) return false;
    return true;
  });
}

bool Worker::read_surface(int cam, HostSurface& out, i64* pts) {
  std::shared_ptr<Camera> c;
  int slot;
  {
    std::lock_guard<std::mutex> g(cams_mu_);
    if (cam < 0 || size_t(cam) >= cams_.size() || !cams_[size_t(cam)]) return false;
    c = cams_[size_t(cam)];
    slot = c->out_surface_slot;
    if (pts) *pts = c->out_surface_pts;
  }
  if (slot < 0) return false;
  const Camera::Surface& sf = c->surface;
  if (!dev_.gpu()) {
    if (size_t(slot) >= sf.host.size()) return false;
    out = sf.host[size_t(slot)];
    return true;
  }
  if (!sf.y || slot >= sf.slots) return false;
  out.alloc(sf.wmbs * 16, sf.hmbs * 16, sf.bd, sf.cf);
  void* dy = out.wide() ? static_cast<void*>(out.y16.data()) : static_cast<void*>(out.y.data());
  void* duv = out.wide() ? static_cast<void*>(out.uv16.data()) : static_cast<void*>(out.uv.data());
  VEP_CHECK(sf.slot_y() == size_t(out.coded_w) * size_t(out.coded_h) * size_t(sf.bps), "surface size mismatch");
  dev_.bind();
  VEP_HIP(hipDeviceSynchronize());  // (the picture's reconstruction ran on a lane stream)
  VEP_HIP(hipMemcpy(dy, sf.y + size_t(slot) * sf.slot_y(), sf.slot_y(), hipMemcpyDeviceToHost));
  VEP_HIP(hipMemcpy(duv, sf.uv + size_t(slot) * sf.slot_uv(), sf.slot_uv(), hipMemcpyDeviceToHost));
  return true;
}

void Camera::wait_reconstruction() {
  if (w_.options().backpressure) w_.wait_camera_taken(index_, 2000);
}

void Worker::flush() {
  {
    std::unique_lock<std::mutex> g(q_mu_);
    if (running_) {
      idle_cv_.wait(g, [this] { return pending_.empty() && !busy_; });
      return;
    }
  }
  complete_all();
}

void Worker::loop() {
  dev_.bind();
  std::vector<DecodeJob> batch;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(q_mu_);
      q_cv_.wait(g, [this] { return stop_ || !pending_.empty(); });
      if (stop_ && pending_.empty()) break;
      if (kf_window_us_ > 0) {  // keyframe-only pictures: gather a few per wavefront launch
        auto all_kf = [this] {
          for (const DecodeJob& j : pending_)
            if (!j.keyframe_only) return false;
          return true;
        };
        const size_t enough = 8 * lanes_.size();
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(kf_window_us_);
        while (!stop_ && pending_.size() < enough && all_kf())
          if (q_cv_.wait_until(g, deadline) == std::cv_status::timeout) break;
      }
      batch.swap(pending_);
      busy_ = true;
    }
    taken_cv_.notify_all();
    try {
      launch_async(batch);
    } catch (const std::exception& e) {
      for (auto& j : batch)
        if (auto c = camera(j.cam)) {
          c->errors.fetch_add(1);
          c->logs.add(true, std::string("decode batch failed: ") + e.what());
        }
    }
    batch.clear();
    {
      std::lock_guard<std::mutex> g(q_mu_);
      if (!pending_.empty()) continue;  // keep the pipeline full while work keeps arriving
    }
    try {
      complete_all();
    } catch (const std::exception&) {
    }
    {
      std::lock_guard<std::mutex> g(q_mu_);
      if (pending_.empty()) busy_ = false;
    }
    idle_cv_.notify_all();
  }
  try {
    complete_all();
  } catch (const std::exception&) {
  }
}

void Worker::ensure_surface(Camera& c, const PictureInfo& pi, int slots, int bd, bool weave, int cf) {
  const int bps = bd > 8 ? 2 : 1;
  const int wmbs = pi.coded_width / 16, hmbs = pi.coded_height / 16;
  auto& s = c.surface;
  // the 8-bit frame the conversion reads when the slot is not one (Main10; a woven field pair)
  auto scratch8 = [&] {
    if (!dev_.gpu() || s.y8) return;
    const size_t y8 = size_t(s.wmbs) * 16 * s.hmbs * 16;
    s.y8 = static_cast<u8*>(dev_.alloc(y8));
    s.uv8 = static_cast<u8*>(dev_.alloc(y8 / 2));
  };
  if (s.wmbs == wmbs && s.hmbs == hmbs && s.slots >= slots && s.bd == bd && s.cf == cf && c.ring_ &&
      c.ring_->width() == pi.width && c.ring_->height() == pi.height) {
    if (weave) scratch8();  // (only ever added: no batch in flight reads a missing scratch)
    return;
  }
  dev_.free(s.y);
  dev_.free(s.uv);
  dev_.free(s.y8);
  dev_.free(s.uv8);
  s.y = s.uv = s.y8 = s.uv8 = nullptr;
  s.wmbs = wmbs;
  s.hmbs = hmbs;
  s.slots = std::max(1, slots);
  s.bps = bps;
  s.bd = bd;
  s.cf = cf;
  const size_t ysz = s.slot_y() * size_t(s.slots);
  if (dev_.gpu()) {
    s.y = static_cast<u8*>(dev_.alloc(ysz));
    const size_t uvsz = s.slot_uv() * size_t(s.slots);
    s.uv = static_cast<u8*>(dev_.alloc(uvsz));
    if (bps == 2) {  // Main10 / High 10: u16 samples at the depth's black / grey
      VEP_HIP(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(s.y), u16(16 << (bd - 8)), ysz / 2, stream_));
      VEP_HIP(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(s.uv), u16(128 << (bd - 8)), uvsz / 2, stream_));
      scratch8();
    } else {
      if (weave || cf == 2) scratch8();
      VEP_HIP(hipMemsetAsync(s.y, 16, ysz, stream_));
      VEP_HIP(hipMemsetAsync(s.uv, 128, uvsz, stream_));
    }
    // the camera's lane may be another stream: the fill must land before its first kernel
    if (lanes_.size() > 1) VEP_HIP(hipStreamSynchronize(stream_));
  } else {
    s.host.assign(size_t(s.slots), HostSurface{});
    for (auto& h : s.host) h.alloc(wmbs * 16, hmbs * 16, bd, cf);
  }
  c.set_ring(std::make_shared<FrameRing>(dev_, c.ring_slots_cfg, pi.width, pi.height));
}

static inline size_t al(size_t x, size_t a = 256) { return (x + a - 1) & ~(a - 1); }

// CPU mirror of letterbox_nv12_kernel (same float math, same rounding).
static void cpu_letterbox_nv12(const HostSurface& s, const gpu::LetterboxDesc& d, int S, u8 pad) {
  const u8 pad_y = u8(std::lround(16.0 + pad * 219.0 / 255.0));
  auto axis = [](int o, int p, float r, int src, int& i0, int& i1, float& l) {
    const float v = std::max((float(o - p) + 0.5f) * r - 0.5f, 0.f);
    i0 = int(v);
    i1 = i0 + (i0 < src - 1 ? 1 : 0);
    l = v - float(i0);
  };
  auto lerp = [](const u8* p, int pitch, int step, int x0, int x1, int y0, int y1, float lx, float ly) {
    const float a = p[size_t(y0) * pitch + x0 * step], b = p[size_t(y0) * pitch + x1 * step];
    const float c = p[size_t(y1) * pitch + x0 * step], e = p[size_t(y1) * pitch + x1 * step];
    return (1.f - ly) * ((1.f - lx) * a + lx * b) + ly * ((1.f - lx) * c + lx * e);
  };
  const int pitch = s.coded_w;
  const u8* Y = s.y.data() + size_t(d.crop_top) * pitch + d.crop_left;
  for (int oy = 0; oy < S; ++oy)
    for (int ox = 0; ox < S; ++ox) {
      u8 v = pad_y;
      if (oy >= d.pad_y && oy < d.pad_y + d.nh && ox >= d.pad_x && ox < d.pad_x + d.nw) {
        int x0, x1, y0, y1;
        float lx, ly;
        axis(oy, d.pad_y, d.ry, d.src_h, y0, y1, ly);
        axis(ox, d.pad_x, d.rx, d.src_w, x0, x1, lx);
        v = u8(std::min(lerp(Y, pitch, 1, x0, x1, y0, y1, lx, ly) + 0.5f, 255.f));
      }
      d.out_hwc[size_t(oy) * S + ox] = v;
    }
  const u8* UV = s.uv.data() + size_t(d.crop_top / 2) * pitch + (d.crop_left & ~1);
  const int px = d.pad_x / 2, py = d.pad_y / 2, nwc = d.nw / 2, nhc = d.nh / 2;
  const int sw = (d.src_w + 1) / 2, sh = (d.src_h + 1) / 2;
  u8* out = d.out_hwc + size_t(S) * S;
  for (int cy = 0; cy < S / 2; ++cy)
    for (int cx = 0; cx < S / 2; ++cx) {
      u8 u = 128, w = 128;
      if (cy >= py && cy < py + nhc && cx >= px && cx < px + nwc) {
        int x0, x1, y0, y1;
        float lx, ly;
        axis(cy, py, d.ry, sh, y0, y1, ly);
        axis(cx, px, d.rx, sw, x0, x1, lx);
        u = u8(std::min(lerp(UV, pitch, 2, x0, x1, y0, y1, lx, ly) + 0.5f, 255.f));
        w = u8(std::min(lerp(UV + 1, pitch, 2, x0, x1, y0, y1, lx, ly) + 0.5f, 255.f));
      }
      out[size_t(cy) * S + 2 * cx] = u;
      out[size_t(cy) * S + 2 * cx + 1] = w;
    }
}

static void cpu_letterbox(const HostSurface& s, const gpu::LetterboxDesc& d,
                          const gpu::LetterboxParams& p) {
  const int S = p.size;
  for (int oy = 0; oy < S; ++oy) {
    for (int ox = 0; ox < S; ++ox) {
      float v[3];
      bool in = oy >= d.pad_y && oy < d.pad_y + d.nh && ox >= d.pad_x && ox < d.pad_x + d.nw;
      if (!in) {
        v[0] = v[1] = v[2] = float(p.pad_value);
      } else {
        float sy = std::max((float(oy - d.pad_y) + 0.5f) * d.ry - 0.5f, 0.f);
        float sx = std::max((float(ox - d.pad_x) + 0.5f) * d.rx - 0.5f, 0.f);
        int y0 = int(sy), x0 = int(sx);
        int y1 = y0 + (y0 < d.src_h - 1 ? 1 : 0), x1 = x0 + (x0 < d.src_w - 1 ? 1 : 0);
        float ly = sy - float(y0), lx = sx - float(x0);
        auto px = [&](int x, int y, float* o) {
          x += d.crop_left;
          y += d.crop_top;
          const u8* c = &s.uv[size_t(y >> 1) * s.coded_w + (x & ~1)];
          u8 b, g, r;
          yuv_to_bgr(s.y[size_t(y) * s.coded_w + x], c[0], c[1], &b, &g, &r);
          o[0] = b;
          o[1] = g;
          o[2] = r;
        };
        float a[3], b[3], c[3], e[3];
        px(x0, y0, a);
        px(x1, y0, b);
        px(x0, y1, c);
        px(x1, y1, e);
        float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx),
              w11 = ly * lx;
        for (int k = 0; k < 3; ++k) v[k] = w00 * a[k] + w01 * b[k] + w10 * c[k] + w11 * e[k];
      }
      size_t pix = size_t(oy) * S + ox;
      if (d.out_hwc)
        for (int k = 0; k < 3; ++k)
          d.out_hwc[pix * 3 + k] = u8(std::min(std::max(v[k] + 0.5f, 0.f), 255.f));
      if (d.out_chw && p.chw_dtype == gpu::kChwF32) {
        float* o = static_cast<float*>(d.out_chw);
        const size_t plane = size_t(S) * S;
        for (int k = 0; k < 3; ++k)  // RGB planes from BGR values
          o[k * plane + pix] = (v[2 - k] * (1.f / 255.f) - p.mean[k]) * p.inv_std[k];
      }
    }
  }
}

// Drop jobs of vanished cameras, (re)allocate surfaces/rings, reserve ring slots.
void Worker::prepare(std::vector<DecodeJob>& jobs, std::vector<int>& slots) {
  bool resize = false;
  {
    std::lock_guard<std::mutex> g(cams_mu_);
    jobs.erase(std::remove_if(jobs.begin(), jobs.end(),
                              [&](const DecodeJob& j) {
                                return j.cam < 0 || j.cam >= int(cams_.size()) ||
                                       !cams_[size_t(j.cam)];
                              }),
               jobs.end());
    for (auto& j : jobs) {
      Camera& c = *cams_[size_t(j.cam)];
      const bool have = c.ring_ != nullptr;
      if (have && (c.surface.wmbs * 16 != j.pic.coded_width ||
                   c.surface.hmbs * 16 != j.pic.coded_height || c.ring_->width() != j.pic.width ||
                   c.ring_->height() != j.pic.height || c.surface.slots < j.dpb_slots() ||
                   c.surface.bd != j.bit_depth() || c.surface.cf != j.chroma_format()))
        resize = true;
    }
  }
  if (resize) complete_locked();  // never free a surface an in-flight batch still writes
  std::lock_guard<std::mutex> g(cams_mu_);
  slots.resize(jobs.size());
  for (size_t i = 0; i < jobs.size(); ++i) {
    Camera& c = *cams_[size_t(jobs[i].cam)];
    bool weave = jobs[i].out_fields;
    for (const auto& p : jobs[i].avc) weave |= p->structure != 0;
    ensure_surface(c, jobs[i].pic, jobs[i].dpb_slots(), jobs[i].bit_depth(), weave, jobs[i].chroma_format());
    slots[i] = jobs[i].has_output() ? c.ring_->begin_write() : -1;
  }
}

namespace {

// Coded-MB bitmask + per-word exclusive prefix, and the raster-order list of sample blocks.
// O(coded MBs), not O(picture MBs): a P frame touches a few hundred of 8,160 MBs.
// seg_off[s] = staging byte offset (relative to the job's payload base) of segment s.
void build_index(const MbUpdate& u, const std::vector<size_t>& seg_off, u32* mask, u32* prefix,
                 u32* offsets) {
  const int words = (u.mbs() + 31) / 32;
  std::memset(mask, 0, size_t(words) * sizeof(u32));
  const std::vector<i32>* list = &u.coded;
  std::vector<i32> sorted;
  if (!std::is_sorted(u.coded.begin(), u.coded.end())) {  // GOP collapse re-ordered slots
    sorted = u.coded;
    std::sort(sorted.begin(), sorted.end());
    list = &sorted;
  }
  size_t k = 0;
  for (i32 mb : *list) {
    mask[mb >> 5] |= 1u << (mb & 31);
    const int s = u.slot[size_t(mb)];
    const u32 g = u.slot_seg[size_t(s)];
    offsets[k++] = u32(seg_off[g] + size_t(u.block(s) - u.segs[g].base));
  }
  u32 run = 0;
  for (int w = 0; w < words; ++w) {
    prefix[w] = run;
    run += u32(__builtin_popcount(mask[w]));
  }
}

// Direct mode: per coded MB the device address of its samples inside host memory (pinned AU
// block or staging), instead of an offset into a device-side copy.
void build_index_ptrs(const MbUpdate& u, const std::vector<const u8*>& seg_dev, u32* mask,
                      u32* prefix, u64* ptrs) {
  const int words = (u.mbs() + 31) / 32;
  std::memset(mask, 0, size_t(words) * sizeof(u32));
  const std::vector<i32>* list = &u.coded;
  std::vector<i32> sorted;
  if (!std::is_sorted(u.coded.begin(), u.coded.end())) {
    sorted = u.coded;
    std::sort(sorted.begin(), sorted.end());
    list = &sorted;
  }
  size_t k = 0;
  for (i32 mb : *list) {
    mask[mb >> 5] |= 1u << (mb & 31);
    const int s = u.slot[size_t(mb)];
    const u32 g = u.slot_seg[size_t(s)];
    ptrs[k++] = reinterpret_cast<u64>(seg_dev[g] + (u.block(s) - u.segs[g].base));
  }
  u32 run = 0;
  for (int w = 0; w < words; ++w) {
    prefix[w] = run;
    run += u32(__builtin_popcount(mask[w]));
  }
}

constexpr size_t kPackChunk = size_t(1) << 20;  // bytes per copy task

}  // namespace

void Worker::launch_gpu(Lane& ln, Stage& st) {
  const hipStream_t cs = ln.stream;
  std::vector<DecodeJob>& jobs = st.jobs;
  const int n = int(jobs.size());
  // Slice bytes stay in host memory: pinned AU blocks as received (hostmem.h), or this stage's
  // pinned staging buffer for pageable AUs (one host memcpy). Two ways to the GPU:
  //  * direct (default): decode_convert reads each block straight over PCIe from its host
  //    address (per-MB 64-bit pointer table) — no device copy of the payload at all;
  //  * gather: a gather kernel on the copy stream first pulls the slices into device staging,
  //    and the kernel reads per-MB offsets into that copy.
  // Layout: [descs][letterbox descs][gather chunks][per job: mask, prefix, offsets|ptrs]
  // | [per job: staged payload]. Only the header part is copied by SDMA.
  const bool direct = direct_reads_;
  const size_t off_desc = 0;
  const size_t off_lb = al(sizeof(gpu::DecodeDesc) * size_t(n));
  size_t nchunks = 0;
  auto chunks_of = [](size_t len) { return (len + gpu::kGatherChunk - 1) / gpu::kGatherChunk; };
  if (!direct)
    for (const auto& j : jobs)
      for (const auto& sg : j.upd.segs) nchunks += chunks_of(sg.len);
  // record arrays already in pinned pool memory (hostmem::PinnedAllocator) are gathered by the
  // GPU over PCIe instead of being copied into the staging buffer by the host
  auto pinned = [](const void* p, size_t len) {
    return len > 0 && hostmem::device_address(static_cast<const u8*>(p), len) != nullptr;
  };
  const size_t off_wv = off_lb + al(sizeof(gpu::LetterboxDesc) * size_t(n));  // field-pair weaves
  size_t need = off_wv + al(sizeof(gpu::WeaveDesc) * size_t(n));
  std::vector<size_t> mask_off(static_cast<size_t>(n)), pay_off(static_cast<size_t>(n));
  std::vector<std::vector<size_t>> seg_off(static_cast<size_t>(n));
  auto words_of = [&](int i) { return size_t(jobs[size_t(i)].upd.mbs() + 31) / 32; };
  const size_t ent = direct ? sizeof(u64) : sizeof(u32);
  for (int i = 0; i < n; ++i) {
    mask_off[size_t(i)] = need;
    need += 2 * al(words_of(i) * sizeof(u32), 16) +
            al(size_t(jobs[size_t(i)].upd.nslots) * ent, 16);
  }
  // General H.264 pictures: MB records, coefficient blocks and motion vectors of every picture,
  // plus one AvcDesc array per reconstruction round (round r = r-th picture of each job).
  struct AvcPic {
    const avc::Picture* p;
    int job;
    size_t off_mbs, off_coef, off_mv, off_wp, off_dbk, off_res, off_xg;
  };
  std::vector<AvcPic> apics;
  int rounds = 0;
  for (int i = 0; i < n; ++i) rounds = std::max(rounds, int(jobs[size_t(i)].avc.size()));
  std::vector<size_t> off_round(static_cast<size_t>(rounds));
  std::vector<std::vector<int>> round_pics(static_cast<size_t>(rounds));
  for (int r = 0; r < rounds; ++r) {
    for (int i = 0; i < n; ++i) {
      const auto& v = jobs[size_t(i)].avc;
      if (int(v.size()) <= r) continue;
      const avc::Picture& p = *v[size_t(r)];
      VEP_CHECK(p.hmbs <= gpu::kAvcMaxRows && p.wmbs <= gpu::kAvcMaxCols,
                "picture too large for the wavefront kernels");
      VEP_CHECK(p.wmbs * 16 == jobs[size_t(i)].pic.coded_width &&
                    p.hmbs * 16 * (p.structure ? 2 : 1) == jobs[size_t(i)].pic.coded_height,  // (a field: half)
                "picture size differs from the camera's surfaces");
      AvcPic a{&p, i, 0, 0, 0, 0, 0, 0, 0};
      auto put = [&](const void* src, size_t bytes) {
        const size_t o = need;
        need += al(bytes);
        if (pinned(src, bytes)) nchunks += chunks_of(bytes);
        return o;
      };
      a.off_mbs = put(p.mbs.data(), p.mbs.size() * sizeof(avc::MbRec));
      a.off_coef = put(p.coefs.data(), p.coefs.size() * sizeof(i16));
      a.off_mv = put(p.mvs.data(), p.mvs.size() * sizeof(i16));
      a.off_wp = put(p.wps.data(), p.wps.size() * sizeof(avc::WpEntry));
      round_pics[size_t(r)].push_back(int(apics.size()));
      apics.push_back(a);
    }
    off_round[size_t(r)] = need;
    need += al(round_pics[size_t(r)].size() * sizeof(gpu::AvcDesc));
  }
  // General H.265 pictures: reconstruction records of every picture, one HevcDesc array and one
  // level-range table per round.
  struct HevcPic {
    const hevc::GpuPicture* p;
    int job;
    size_t off_pu, off_tu, off_coef, off_pcm, off_bsv, off_bsh, off_qp, off_pcmmap, off_cslice, off_slices, off_sao;
    size_t off_wp, off_ctile;
  };
  std::vector<HevcPic> hpics;
  int hrounds = 0;
  for (int i = 0; i < n; ++i) hrounds = std::max(hrounds, int(jobs[size_t(i)].hevc.size()));
  std::vector<size_t> off_hround(static_cast<size_t>(hrounds)), off_hranges(static_cast<size_t>(hrounds));
  std::vector<std::vector<int>> hround_pics(static_cast<size_t>(hrounds));
  std::vector<std::vector<gpu::HevcTuRange>> hranges(static_cast<size_t>(hrounds));
  // per round: level-0 ranges, level-0 blocks, intra (queue) ranges, intra blocks
  std::vector<std::array<int, 4>> hwork(static_cast<size_t>(hrounds), std::array<int, 4>{0, 0, 0, 0});
  std::vector<size_t> off_hctr(static_cast<size_t>(hrounds)), off_hpicq(static_cast<size_t>(hrounds));
  // per round, picture mode (hevc_tu_window_ < 0): {desc, first intra block, intra blocks} per picture
  std::vector<std::vector<gpu::HevcTuRange>> hpicq(static_cast<size_t>(hrounds));
  // per round and intra level: first ticket, blocks (the one-launch-per-level mode); per round
  // and queue window: first ticket, blocks (one ticket counter each)
  std::vector<std::vector<std::array<int, 2>>> hlevels(static_cast<size_t>(hrounds));
  std::vector<std::vector<std::array<int, 2>>> hwindows(static_cast<size_t>(hrounds));
  for (int r = 0; r < hrounds; ++r) {
    int maxl = 0;
    for (int i = 0; i < n; ++i) {
      const auto& v = jobs[size_t(i)].hevc;
      if (int(v.size()) <= r) continue;
      const hevc::GpuPicture& p = *v[size_t(r)];
      VEP_CHECK(((p.width + 15) & ~15) == jobs[size_t(i)].pic.coded_width &&
                    ((p.height + 15) & ~15) == jobs[size_t(i)].pic.coded_height,
                "picture size differs from the camera's surfaces");
      HevcPic a{&p, i, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      auto put = [&](size_t bytes) {
        const size_t o = need;
        need += al(std::max<size_t>(bytes, 16));
        return o;
      };
      a.off_pu = put(p.pus.size() * sizeof(hevc::GpuPu));
      a.off_tu = put(p.tus.size() * sizeof(hevc::GpuTu));
      a.off_coef = put(p.coefs.size() * sizeof(i16));
      a.off_pcm = put(p.pcm.size());
      a.off_bsv = put(p.bs_v.size());
      a.off_bsh = put(p.bs_h.size());
      a.off_qp = put(p.qp.size());
      a.off_pcmmap = put(p.pcm_map.size());
      a.off_cslice = put(p.ctb_slice.size() * sizeof(u16));
      a.off_slices = put(p.slices.size() * sizeof(hevc::GpuSlice));
      a.off_sao = put(p.sao_params.size() * sizeof(hevc::GpuSao));
      a.off_wp = put(p.wp.size() * sizeof(hevc::GpuWp));
      a.off_ctile = put(p.ctb_tile.size() * sizeof(u16));
      maxl = std::max(maxl, int(p.level_begin.size()) - 1);
      hround_pics[size_t(r)].push_back(int(hpics.size()));
      hpics.push_back(a);
    }
    off_hround[size_t(r)] = need;
    need += al(hround_pics[size_t(r)].size() * sizeof(gpu::HevcDesc));
    // level 0 (inter residual + PCM, independent blocks): one range per picture, one wide
    // launch. Intra levels >= 1: one ticket queue for the whole round, level-major (a block's
    // producers are at lower levels, so they hold lower tickets).
    int tickets = 0;
    for (int l = 0; l < maxl; ++l) {
      if (l > 0) hlevels[size_t(r)].push_back({tickets, 0});
      for (size_t k = 0; k < hround_pics[size_t(r)].size(); ++k) {
        const hevc::GpuPicture& p = *hpics[size_t(hround_pics[size_t(r)][k])].p;
        if (int(p.level_begin.size()) - 1 <= l) continue;
        const int b = int(p.level_begin[size_t(l)]), e = int(p.level_begin[size_t(l) + 1]);
        if (e <= b) continue;
        if (l == 0) {
          hranges[size_t(r)].push_back({int(k), b, e - b, hwork[size_t(r)][1]});
          hwork[size_t(r)][0] += 1;
          hwork[size_t(r)][1] += e - b;
        } else {
          hranges[size_t(r)].push_back({int(k), b, e - b, tickets});
          hwork[size_t(r)][2] += 1;
          tickets += e - b;
          hlevels[size_t(r)].back()[1] += e - b;
        }
      }
    }
    hwork[size_t(r)][3] = tickets;
    if (hevc_tu_window_ < 0) {  // one workgroup per picture with intra blocks
      for (size_t k = 0; k < hround_pics[size_t(r)].size(); ++k) {
        const hevc::GpuPicture& p = *hpics[size_t(hround_pics[size_t(r)][k])].p;
        if (p.level_begin.size() < 3) continue;  // (levels 0 .. L-1 plus the end: intra needs L >= 2)
        const int b = int(p.level_begin[1]), e = int(p.tus.size());
        if (e > b) hpicq[size_t(r)].push_back({int(k), b, e - b, 0});
      }
    }
    if (hevc_tu_window_ > 0) {  // consecutive levels, hevc_tu_window_ per launch
      const auto& lv = hlevels[size_t(r)];
      for (size_t l = 0; l < lv.size(); l += size_t(hevc_tu_window_)) {
        const size_t e = std::min(lv.size(), l + size_t(hevc_tu_window_));
        const int first = lv[l][0], last = lv[e - 1][0] + lv[e - 1][1];
        if (last > first) hwindows[size_t(r)].push_back({first, last - first});
      }
    }
    off_hranges[size_t(r)] = need;
    need += al(std::max<size_t>(hranges[size_t(r)].size(), 1) * sizeof(gpu::HevcTuRange));
    off_hctr[size_t(r)] = need;  // the queue windows' ticket counters (zero in the upload)
    need += al(std::max<size_t>(hwindows[size_t(r)].size(), 1) * sizeof(u32));
    off_hpicq[size_t(r)] = need;
    need += al(std::max<size_t>(hpicq[size_t(r)].size(), 1) * sizeof(gpu::HevcTuRange));
  }
  const size_t off_gather = need;  // gather chunks: pinned records (+ slices without direct reads)
  need += al(sizeof(gpu::GatherChunk) * std::max<size_t>(nchunks, 1));
  need = al(need);
  const size_t header_bytes = need;
  for (int i = 0; i < n; ++i) {
    pay_off[size_t(i)] = need;
    size_t rel = 0;
    for (const auto& sg : jobs[size_t(i)].upd.segs) {
      seg_off[size_t(i)].push_back(rel);
      rel += al(sg.len, 16);
    }
    need += rel;
  }
  need = al(need);
  for (AvcPic& a : apics) {  // device-only scratch (never copied): per-MB loop-filter inputs,
    a.off_dbk = need;         // intra MBs' residual samples (inter kernel -> intra wavefront)
    need += al(size_t(a.p->nmbs()) * sizeof(gpu::AvcDbkInfo));
    a.off_res = need;
    need += al(size_t(a.p->intra_res) * gpu::kAvcResSamples * sizeof(i16));
    a.off_xg = need;  // deblock exchange between the wavefront's workgroups
    need += al(gpu::avc_xg_bytes(a.p->wmbs, a.p->hmbs));
  }
  need = al(need);
  if (need > st.cap) {
    if (st.h) hostmem::unregister_range(st.h);
    dev_.free(st.d);
    dev_.free_pinned(st.h);
    st.cap = std::max(need + need / 2, size_t(4) << 20);
    st.h = static_cast<u8*>(dev_.alloc_pinned(st.cap));
    st.d = static_cast<u8*>(dev_.alloc(st.cap));
    void* hd_ptr = nullptr;
    if (hipHostGetDevicePointer(&hd_ptr, st.h, 0) != hipSuccess) hd_ptr = st.h;
    hostmem::register_range(st.h, st.cap, static_cast<u8*>(hd_ptr));
  }
  auto mask_ptr = [&](u8* base, int i) { return reinterpret_cast<u32*>(base + mask_off[size_t(i)]); };
  auto prefix_ptr = [&](u8* base, int i) {
    return reinterpret_cast<u32*>(base + mask_off[size_t(i)] + al(words_of(i) * sizeof(u32), 16));
  };
  auto table_ptr = [&](u8* base, int i) {
    return base + mask_off[size_t(i)] + 2 * al(words_of(i) * sizeof(u32), 16);
  };
  // Phase 1: where each segment's bytes are readable by the GPU (staging pageable ones).
  struct CopyTask {
    const u8* src;
    u8* dst;
    size_t len;
  };
  std::vector<CopyTask> tasks;
  auto* gc = reinterpret_cast<gpu::GatherChunk*>(st.h + off_gather);
  size_t ng = 0;
  for (const AvcPic& a : apics) {
    auto add = [&](const void* src, size_t len, size_t off) {
      if (pinned(src, len)) {  // the GPU pulls it (gather kernel after the header copy)
        const u8* dv = hostmem::device_address(static_cast<const u8*>(src), len);
        for (size_t o = 0; o < len; o += gpu::kGatherChunk)
          gc[ng++] = {dv + o, st.d + off + o, u32(std::min<size_t>(gpu::kGatherChunk, len - o)), 0};
        records_gathered_ += u64(len);
        return;
      }
      for (size_t o = 0; o < len; o += kPackChunk)
        tasks.push_back({static_cast<const u8*>(src) + o, st.h + off + o, std::min(kPackChunk, len - o)});
    };
    add(a.p->mbs.data(), a.p->mbs.size() * sizeof(avc::MbRec), a.off_mbs);
    add(a.p->coefs.data(), a.p->coefs.size() * sizeof(i16), a.off_coef);
    add(a.p->mvs.data(), a.p->mvs.size() * sizeof(i16), a.off_mv);
    add(a.p->wps.data(), a.p->wps.size() * sizeof(avc::WpEntry), a.off_wp);
  }
  for (const HevcPic& a : hpics) {
    auto add = [&](const void* src, size_t len, size_t off) {
      for (size_t o = 0; o < len; o += kPackChunk)
        tasks.push_back({static_cast<const u8*>(src) + o, st.h + off + o, std::min(kPackChunk, len - o)});
    };
    const hevc::GpuPicture& p = *a.p;
    add(p.pus.data(), p.pus.size() * sizeof(hevc::GpuPu), a.off_pu);
    add(p.tus.data(), p.tus.size() * sizeof(hevc::GpuTu), a.off_tu);
    add(p.coefs.data(), p.coefs.size() * sizeof(i16), a.off_coef);
    add(p.pcm.data(), p.pcm.size(), a.off_pcm);
    add(p.bs_v.data(), p.bs_v.size(), a.off_bsv);
    add(p.bs_h.data(), p.bs_h.size(), a.off_bsh);
    add(p.qp.data(), p.qp.size(), a.off_qp);
    add(p.pcm_map.data(), p.pcm_map.size(), a.off_pcmmap);
    add(p.ctb_slice.data(), p.ctb_slice.size() * sizeof(u16), a.off_cslice);
    add(p.slices.data(), p.slices.size() * sizeof(hevc::GpuSlice), a.off_slices);
    add(p.sao_params.data(), p.sao_params.size() * sizeof(hevc::GpuSao), a.off_sao);
    add(p.wp.data(), p.wp.size() * sizeof(hevc::GpuWp), a.off_wp);
    add(p.ctb_tile.data(), p.ctb_tile.size() * sizeof(u16), a.off_ctile);
  }
  std::vector<std::vector<const u8*>> seg_dev(static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    const auto& segs = jobs[size_t(i)].upd.segs;
    for (size_t g = 0; g < segs.size(); ++g) {
      const size_t dst_off = pay_off[size_t(i)] + seg_off[size_t(i)][g];
      const u8* src = hostmem::device_address(segs[g].base, segs[g].len);
      if (!src) {  // pageable AU bytes: stage them
        for (size_t o = 0; o < segs[g].len; o += kPackChunk)
          tasks.push_back({segs[g].base + o, st.h + dst_off + o,
                           std::min(kPackChunk, segs[g].len - o)});
        src = hostmem::device_address(st.h + dst_off, segs[g].len);
        VEP_CHECK(src, "staging buffer is not registered");
        pinned_bytes_staged_ += u64(segs[g].len);
      } else {
        pinned_bytes_inplace_ += u64(segs[g].len);
      }
      seg_dev[size_t(i)].push_back(src);
      if (!direct)
        for (size_t o = 0; o < segs[g].len; o += gpu::kGatherChunk)
          gc[ng++] = {src + o, st.d + dst_off + o,
                      u32(std::min<size_t>(gpu::kGatherChunk, segs[g].len - o)), 0};
    }
  }
  VEP_CHECK(ng == nchunks, "gather chunk count mismatch");
  // Phase 2 (per job, pack threads): coded-MB bitmask/prefix + per-MB offsets or pointers.
  auto index = [&](int i) {
    if (direct)
      build_index_ptrs(jobs[size_t(i)].upd, seg_dev[size_t(i)], mask_ptr(st.h, i),
                       prefix_ptr(st.h, i), reinterpret_cast<u64*>(table_ptr(st.h, i)));
    else
      build_index(jobs[size_t(i)].upd, seg_off[size_t(i)], mask_ptr(st.h, i), prefix_ptr(st.h, i),
                  reinterpret_cast<u32*>(table_ptr(st.h, i)));
  };
  const i64 t_index0 = mono_us();
  {
    trace::Range tr("vep.index");
    if (pack_pool_ && n > 1) pack_pool_->parallel_for(n, index);
    else for (int i = 0; i < n; ++i) index(i);
  }
  const i64 t_copy0 = mono_us();
  add_time(&Timers::index, double(t_copy0 - t_index0));
  auto copy = [&](int t) { std::memcpy(tasks[size_t(t)].dst, tasks[size_t(t)].src, tasks[size_t(t)].len); };
  if (pack_pool_ && tasks.size() > 1) pack_pool_->parallel_for(int(tasks.size()), copy);
  else for (int t = 0; t < int(tasks.size()); ++t) copy(t);
  const i64 t_enq0 = mono_us();
  add_time(&Timers::copy, double(t_enq0 - t_copy0));

  if (st.err_cap < size_t(n)) {
    if (st.err) dev_.free_pinned(st.err);
    st.err_cap = std::max<size_t>(size_t(n), 64);
    st.err = static_cast<u32*>(dev_.alloc_pinned(st.err_cap * sizeof(u32)));
    void* ed = nullptr;
    if (hipHostGetDevicePointer(&ed, st.err, 0) != hipSuccess) ed = st.err;
    st.err_dev = static_cast<const u32*>(ed);
  }
  std::memset(st.err, 0, size_t(n) * sizeof(u32));
  auto* hd = reinterpret_cast<gpu::DecodeDesc*>(st.h + off_desc);
  auto* hl = reinterpret_cast<gpu::LetterboxDesc*>(st.h + off_lb);
  auto* hw = reinterpret_cast<gpu::WeaveDesc*>(st.h + off_wv);
  int nweave = 0, weave_pitch = 0, weave_h = 0;
  int tiles = 0;
  // conversion / letterbox descriptors only for jobs that publish a frame (a general-path job
  // whose pictures all wait in the reorder buffer only reconstructs)
  std::vector<int> outs;
  for (int i = 0; i < n; ++i)
    if (jobs[size_t(i)].has_output()) outs.push_back(i);
  const int nout = int(outs.size());
  for (int k = 0; k < nout; ++k) {
    const int i = outs[size_t(k)];
    const DecodeJob& j = jobs[size_t(i)];
    Camera* c = cams_[size_t(j.cam)].get();
    const size_t words = size_t(j.upd.mbs() + 31) / 32;
    gpu::DecodeDesc& d = hd[k];
    const size_t tgt = size_t(j.target());
    if (j.out_fields) {  // field pair: woven into the 8-bit scratch first (launch_weave below)
      const Camera::Surface& sf = c->surface;
      VEP_CHECK(sf.y8 && sf.bps == 1 && sf.hmbs % 2 == 0,
                "field pair output without its weave scratch");
      gpu::WeaveDesc& w = hw[nweave++];
      w.y = sf.y + tgt * sf.slot_y();
      w.uv = sf.uv + tgt * sf.slot_uv();
      w.y8 = sf.y8;
      w.uv8 = sf.uv8;
      w.pitch = sf.wmbs * 16;
      w.height = sf.hmbs * 16;
      weave_pitch = std::max(weave_pitch, w.pitch);
      weave_h = std::max(weave_h, w.height);
    }
    if (c->surface.narrowed() || j.out_fields) {  // Main10 / 4:2:2 / field pair: convert / letterbox the
                                                // 8-bit frame (launch_narrow / launch_weave below)
      d.y = c->surface.y8;
      d.uv = c->surface.uv8;
    } else {
      d.y = c->surface.y + tgt * c->surface.slot_y();
      d.uv = c->surface.uv + tgt * c->surface.slot_uv();
    }
    d.bgr = c->ring_->slot_ptr(st.slots[size_t(i)]);
    (void)words;
    d.mask = mask_ptr(st.d, i);
    d.prefix = prefix_ptr(st.d, i);
    if (direct) {
      d.ptrs = reinterpret_cast<const u64*>(table_ptr(st.d, i));
      d.offsets = nullptr;
      d.payload = nullptr;
    } else {
      d.ptrs = nullptr;
      d.offsets = reinterpret_cast<const u32*>(table_ptr(st.d, i));
      d.payload = st.d + pay_off[size_t(i)];
    }
    const bool whole = j.general() || j.ext;  // the slot already holds the picture
    d.wmbs = whole ? j.pic.coded_width / 16 : j.upd.width_mbs;
    d.hmbs = whole ? j.pic.coded_height / 16 : j.upd.height_mbs;
    if (whole) d.mask = d.prefix = nullptr;  // pure conversion of the reconstructed slot
    d.out_w = j.pic.width;
    d.out_h = j.pic.height;
    d.crop_left = j.pic.crop_left;
    d.crop_top = j.pic.crop_top;
    d.tiles_x = (d.wmbs + gpu::kTileMbW - 1) / gpu::kTileMbW;
    d.tile_begin = tiles;
    d.chk_lo = j.pic.spec_lo;
    d.chk_hi = j.pic.spec_hi;
    d.chk_pat = 0x000Du;  // I_PCM header bytes 0D 00
    d.err = const_cast<u32*>(st.err_dev) + i;
    tiles += gpu::tiles_for(d.wmbs, d.hmbs);
    if (opt_.letterbox_size > 0) {
      gpu::LetterboxDesc& l = hl[k];
      const size_t S = size_t(opt_.letterbox_size);
      l.y = d.y;
      l.uv = d.uv;
      l.pitch = d.wmbs * 16;
      l.src_w = j.pic.width;
      l.src_h = j.pic.height;
      l.crop_left = j.pic.crop_left;
      l.crop_top = j.pic.crop_top;
      VEP_CHECK(j.cam < st.cons_rows, "camera index exceeds consumer batch rows");
      l.out_hwc = st.cons_hwc ? st.cons_hwc + size_t(j.cam) * gpu::letterbox_bytes(int(S), opt_.letterbox_format)
                            : nullptr;
      const size_t es = opt_.chw_dtype == gpu::kChwF32 ? 4 : 2;
      l.out_chw = st.cons_chw ? static_cast<u8*>(st.cons_chw) + size_t(j.cam) * 3 * S * S * es
                            : nullptr;
      gpu::fill_letterbox_geometry(l, opt_.letterbox_size, opt_.letterbox_format == gpu::kLbNV12);
    }
  }
  // AVC descriptors (device addresses known only now)
  for (int r = 0; r < rounds; ++r) {
    auto* ad = reinterpret_cast<gpu::AvcDesc*>(st.h + off_round[size_t(r)]);
    int mbs = 0;
    for (size_t k = 0; k < round_pics[size_t(r)].size(); ++k) {
      const AvcPic& a = apics[size_t(round_pics[size_t(r)][k])];
      const Camera* c = cams_[size_t(jobs[size_t(a.job)].cam)].get();
      gpu::AvcDesc& g = ad[k];
      g.mbs = st.d + a.off_mbs;
      g.coefs = reinterpret_cast<const i16*>(st.d + a.off_coef);
      g.mvs = reinterpret_cast<const i16*>(st.d + a.off_mv);
      g.wps = st.d + a.off_wp;
      g.y = c->surface.y;
      g.uv = c->surface.uv;
      // field pictures address field slots: half a frame slot each (top field rows, then bottom)
      const size_t per = a.p->structure ? 2 : 1;
      g.slot_y = c->surface.slot_y() / per;
      g.slot_uv = c->surface.slot_uv() / per;
      g.wmbs = a.p->wmbs;
      g.hmbs = a.p->hmbs;
      g.target = a.p->target;
      g.constrained = a.p->constrained_intra ? 1 : 0;
      g.mb_begin = mbs;
      g.field = a.p->structure;
      g.err = const_cast<u32*>(st.err_dev) + a.job;
      g.dbk = st.d + a.off_dbk;
      g.res = reinterpret_cast<i16*>(st.d + a.off_res);
      g.xg = reinterpret_cast<u64*>(st.d + a.off_xg);
      g.prof = avc_prof_;
      g.bd = a.p->bd;
      g.qp_bias = a.p->qp_bias;
      g.qpc_bias = a.p->qpc_bias;
      g.cf = a.p->cf;
      g.ncoef = u32(a.p->coefs.size());
      g.nres = u32(a.p->intra_res);
      g.intra_mbs = a.p->intra_mbs;
      g.deblock = a.p->deblock ? 1 : 0;
      VEP_CHECK(c->surface.bd == a.p->bd && c->surface.cf == a.p->cf,
                "H.264: picture bit depth / chroma format differs from the camera's surfaces");
      mbs += a.p->nmbs();
    }
  }
  // HEVC descriptors and level ranges
  std::vector<std::array<int, 2>> hround_work(static_cast<size_t>(hrounds));  // PUs, 4x4 blocks
  for (int r = 0; r < hrounds; ++r) {
    auto* hd2 = reinterpret_cast<gpu::HevcDesc*>(st.h + off_hround[size_t(r)]);
    int pus = 0, blks = 0;
    for (size_t k = 0; k < hround_pics[size_t(r)].size(); ++k) {
      const HevcPic& a = hpics[size_t(hround_pics[size_t(r)][k])];
      const hevc::GpuPicture& p = *a.p;
      const DecodeJob& j = jobs[size_t(a.job)];
      const Camera* c = cams_[size_t(j.cam)].get();
      gpu::HevcDesc& g = hd2[k];
      g = gpu::HevcDesc{};
      g.y = c->surface.y;
      g.uv = c->surface.uv;
      g.slot_y = c->surface.slot_y();
      g.slot_uv = c->surface.slot_uv();
      g.stride = c->surface.wmbs * 16;
      g.width = p.width;
      g.height = p.height;
      g.log2ctb = p.log2ctb;
      g.wctb = p.wctb;
      g.hctb = p.hctb;
      g.target = p.target;
      g.cb_qp_offset = p.cb_qp_offset;
      g.cr_qp_offset = p.cr_qp_offset;
      g.flags = (p.deblock ? 1 : 0) | (p.sao ? 2 : 0) | (p.pcm_nofilter ? 4 : 0) | (p.tiles_block_sao ? 8 : 0) |
                (p.wide() ? gpu::kHevcWide : 0);
      VEP_CHECK(c->surface.bps == (p.wide() ? 2 : 1), "HEVC: picture bit depth differs from the camera's surfaces");
      g.bd_y = p.bd_y;
      g.bd_c = p.bd_c;
      g.pus = st.d + a.off_pu;
      g.tus = st.d + a.off_tu;
      g.coefs = reinterpret_cast<const i16*>(st.d + a.off_coef);
      g.pcm = st.d + a.off_pcm;
      g.bs_v = st.d + a.off_bsv;
      g.bs_h = st.d + a.off_bsh;
      g.qp = reinterpret_cast<const signed char*>(st.d + a.off_qp);
      g.pcm_map = st.d + a.off_pcmmap;
      g.ctb_slice = reinterpret_cast<const u16*>(st.d + a.off_cslice);
      g.slices = st.d + a.off_slices;
      g.sao = st.d + a.off_sao;
      g.wp = st.d + a.off_wp;
      g.ctb_tile = reinterpret_cast<const u16*>(st.d + a.off_ctile);
      const size_t scratch = size_t(j.hevc_slots);  // the extra surface after the DPB slots
      VEP_CHECK(c->surface.slots > j.hevc_slots, "camera surfaces lack the SAO scratch slot");
      g.sao_y = c->surface.y + scratch * c->surface.slot_y();
      g.sao_uv = c->surface.uv + scratch * c->surface.slot_uv();
      g.err = const_cast<u32*>(st.err_dev) + a.job;
      {  // the camera's intra edge exchange (zeroed once: epochs start at 1)
        Camera::Surface& sf = const_cast<Camera*>(c)->surface;
        const size_t words = gpu::hevc_xg_words(g.stride, sf.hmbs * 16);
        if (sf.hevc_xg_words < words) {
          dev_.free(sf.hevc_xg);
          sf.hevc_xg = static_cast<u64*>(dev_.alloc(words * sizeof(u64)));
          VEP_HIP(hipMemset(sf.hevc_xg, 0, words * sizeof(u64)));
          sf.hevc_xg_words = words;
          sf.hevc_epoch = 0;
        }
        if (++sf.hevc_epoch == 0) {  // (after 2^32 rounds) never reuse a tag still in the words
          VEP_HIP(hipMemset(sf.hevc_xg, 0, words * sizeof(u64)));
          sf.hevc_epoch = 1;
        }
        g.xg = hevc_tu_window_ == 0 ? nullptr : sf.hevc_xg;  // (per-level launches read the picture)
        g.xg_h = sf.hmbs * 16;
        g.epoch = sf.hevc_epoch;
        g.nap_max = hevc_tu_nap_;
      }
      g.npu = int(p.pus.size());
      g.pu_begin = pus;
      g.blk_begin = blks;
      pus += g.npu;
      blks += p.w4() * p.h4();
    }
    hround_work[size_t(r)] = {pus, blks};
    auto* hr = reinterpret_cast<gpu::HevcTuRange*>(st.h + off_hranges[size_t(r)]);
    for (size_t k = 0; k < hranges[size_t(r)].size(); ++k) hr[k] = hranges[size_t(r)][k];
    std::memset(st.h + off_hctr[size_t(r)], 0, std::max<size_t>(hwindows[size_t(r)].size(), 1) * sizeof(u32));
    if (!hpicq[size_t(r)].empty())
      std::memcpy(st.h + off_hpicq[size_t(r)], hpicq[size_t(r)].data(), hpicq[size_t(r)].size() * sizeof(gpu::HevcTuRange));
  }
  // H2D on the copy stream overlaps the previous batch's kernels on the compute stream: the
  // small header region by SDMA, the slice payload by the gather kernel (PCIe reads)
  // With several lanes the copy goes on the lane's own stream instead: it then waits for the
  // lane's previous kernels, while the other lanes keep the GPU busy, and no lane ever waits
  // on a queue another lane shares.
  if (ln.copy) {  // the stage's previous batch has completed (launch_on), so st.d is free
    VEP_HIP(hipMemcpyAsync(st.d, st.h, header_bytes, hipMemcpyHostToDevice, ln.copy));
    if (nchunks)
      gpu::launch_gather(reinterpret_cast<const gpu::GatherChunk*>(st.d + off_gather),
                         int(nchunks), ln.copy);
    VEP_HIP(hipEventRecord(st.copied, ln.copy));
    VEP_HIP(hipStreamWaitEvent(cs, st.copied, 0));
    VEP_HIP(hipEventRecord(st.e0, cs));
  } else if (lanes_.size() > 1) {
    VEP_HIP(hipEventRecord(st.e0, cs));
    VEP_HIP(hipMemcpyAsync(st.d, st.h, header_bytes, hipMemcpyHostToDevice, cs));
    if (nchunks)
      gpu::launch_gather(reinterpret_cast<const gpu::GatherChunk*>(st.d + off_gather),
                         int(nchunks), cs);
  } else {
    VEP_HIP(hipMemcpyAsync(st.d, st.h, header_bytes, hipMemcpyHostToDevice, copy_stream_));
    if (nchunks)
      gpu::launch_gather(reinterpret_cast<const gpu::GatherChunk*>(st.d + off_gather),
                         int(nchunks), copy_stream_);
    VEP_HIP(hipEventRecord(st.copied, copy_stream_));
    VEP_HIP(hipStreamWaitEvent(cs, st.copied, 0));
    VEP_HIP(hipEventRecord(st.e0, cs));
  }
  for (int r = 0; r < rounds; ++r) {
    const auto* ad = reinterpret_cast<const gpu::AvcDesc*>(st.d + off_round[size_t(r)]);
    const int np = int(round_pics[size_t(r)].size());
    int mbs = 0;
    bool intra = false, dbk = false, narrow = false;
    int variants = 0;  // High 10 / 4:2:2 pictures by kind (launch_avc_hbd)
    int max_h = 0;
    for (int k : round_pics[size_t(r)]) {
      mbs += apics[size_t(k)].p->nmbs();
      max_h = std::max(max_h, apics[size_t(k)].p->hmbs);
      intra |= apics[size_t(k)].p->intra_mbs > 0;
      dbk |= apics[size_t(k)].p->deblock;
      const avc::Picture& ap = *apics[size_t(k)].p;
      if (ap.bd > 8 || ap.cf == 2) variants |= ap.cf != 2 ? 1 : (ap.bd > 8 ? 4 : 2);
      else narrow = true;
    }
    gpu::launch_avc_inter(ad, np, mbs, cs);
    if (intra && narrow) gpu::launch_avc_intra(ad, np, max_h, cs);
    if (dbk) {
      gpu::launch_avc_bs(ad, np, mbs, cs);
      if (narrow) gpu::launch_avc_deblock(ad, np, max_h, cs, dbk_packed_);
    }
    if (variants) gpu::launch_avc_hbd(ad, np, intra, dbk, variants, cs);  // (High 10 / 4:2:2 pictures)
  }
  for (int r = 0; r < hrounds; ++r) {
    const auto* hd2 = reinterpret_cast<const gpu::HevcDesc*>(st.d + off_hround[size_t(r)]);
    const auto* hr = reinterpret_cast<const gpu::HevcTuRange*>(st.d + off_hranges[size_t(r)]);
    const int np = int(hround_pics[size_t(r)].size());
    bool dbk = false, sao = false;
    for (int k : hround_pics[size_t(r)]) {
      dbk |= hpics[size_t(k)].p->deblock;
      sao |= hpics[size_t(k)].p->sao;
    }
    gpu::launch_hevc_mc(hd2, np, hround_work[size_t(r)][0], cs);
    const auto& hw = hwork[size_t(r)];
    gpu::launch_hevc_tu(hd2, hr, hw[0], 0, hw[1], cs);
    if (hevc_tu_window_ < 0) {  // one workgroup per picture: every dependency wait inside it
      gpu::launch_hevc_tu_pics(hd2, reinterpret_cast<const gpu::HevcTuRange*>(st.d + off_hpicq[size_t(r)]),
                               int(hpicq[size_t(r)].size()), cs);
    } else if (hevc_tu_window_ == 0) {  // one launch per intra level (kernel boundaries order the levels)
      for (const auto& lv : hlevels[size_t(r)]) gpu::launch_hevc_tu(hd2, hr + hw[0], hw[2], lv[0], lv[1], cs);
    } else {  // one queue launch per window of levels, in level order on the stream
      auto* ctr = reinterpret_cast<u32*>(st.d + off_hctr[size_t(r)]);
      // (a window of bounded depth runs one wave per block, each taking its block from the
      // window's ticket counter; the whole round keeps the persistent ticket queue)
      const bool persistent = hevc_tu_window_ >= kAllLevels;
      for (size_t k = 0; k < hwindows[size_t(r)].size(); ++k)
        gpu::launch_hevc_tu_queue(hd2, hr + hw[0], hw[2], hwindows[size_t(r)][k][0], hwindows[size_t(r)][k][1],
                                  ctr + k, persistent, cs);
    }
    if (dbk) {
      gpu::launch_hevc_deblock(hd2, np, hround_work[size_t(r)][1], 0, cs);
      gpu::launch_hevc_deblock(hd2, np, hround_work[size_t(r)][1], 1, cs);
    }
    if (sao) gpu::launch_hevc_sao(hd2, np, hround_work[size_t(r)][1], cs);
  }
  // VCN pictures: the video core's surfaces -> the cameras' NV12 surfaces (device copies on the
  // lane stream, ordered before the conversion; the surfaces return to rocDecode when the batch
  // completes and its jobs are dropped)
  for (int i = 0; i < n; ++i) {
    const DecodeJob& j = jobs[size_t(i)];
    if (!j.ext) continue;
    const Camera* c = cams_[size_t(j.cam)].get();
    const vcn::Frame& f = *j.ext;
    const size_t pitch = size_t(c->surface.wmbs) * 16;
    VEP_CHECK(size_t(f.width) <= pitch && f.height <= c->surface.hmbs * 16, "VCN picture exceeds the camera surface");
    VEP_HIP(hipMemcpy2DAsync(c->surface.y, pitch, f.y, f.pitch_y, size_t(f.width), size_t(f.height),
                             hipMemcpyDefault, cs));
    VEP_HIP(hipMemcpy2DAsync(c->surface.uv, pitch, f.uv, f.pitch_uv, size_t(f.width), size_t(f.height / 2),
                             hipMemcpyDefault, cs));
  }
  gpu::launch_weave(reinterpret_cast<const gpu::WeaveDesc*>(st.d + off_wv), nweave, weave_pitch, weave_h, cs);
  for (int i : outs) {  // Main10 pictures: the published slot's 8-bit NV12 copy
    const DecodeJob& j = jobs[size_t(i)];
    const Camera::Surface& sf = cams_[size_t(j.cam)]->surface;
    const size_t tgt = size_t(j.target());
    if (!sf.narrowed()) continue;
    gpu::launch_narrow(sf.y + tgt * sf.slot_y(), sf.uv + tgt * sf.slot_uv(), sf.y8, sf.uv8, sf.wmbs * 16,
                       sf.hmbs * 16, sf.bd, sf.cf, cs);
  }
  gpu::launch_decode_convert(reinterpret_cast<const gpu::DecodeDesc*>(st.d + off_desc), nout, tiles,
                             cs);
  if (opt_.letterbox_size > 0) {
    gpu::LetterboxParams p{};
    p.size = opt_.letterbox_size;
    p.chw_dtype = opt_.chw_dtype;
    for (int k = 0; k < 3; ++k) {
      p.mean[k] = opt_.mean[k];
      p.inv_std[k] = 1.f / opt_.std[k];
    }
    p.pad_value = 114;
    p.format = opt_.letterbox_format;
    gpu::launch_letterbox(reinterpret_cast<const gpu::LetterboxDesc*>(st.d + off_lb), nout, p,
                          cs);
  }
  VEP_HIP(hipEventRecord(st.e1, cs));
  add_time(&Timers::enqueue, double(mono_us() - t_enq0));
}

void Worker::run_cpu(std::vector<DecodeJob>& jobs, std::vector<int>& slots,
                     std::vector<u32>& err) {
  err.assign(jobs.size(), 0);
  // one task per camera (a camera's jobs stay in order: they share its surfaces)
  std::vector<std::vector<size_t>> groups;
  std::map<int, size_t> of;
  for (size_t i = 0; i < jobs.size(); ++i) {
    auto it = of.find(jobs[i].cam);
    if (it == of.end()) {
      of[jobs[i].cam] = groups.size();
      groups.push_back({i});
    } else {
      groups[it->second].push_back(i);
    }
  }
  auto run = [&](int g) {
    for (size_t i : groups[size_t(g)]) run_cpu_job(jobs, slots, err, i);
  };
  if (cpu_pool_ && groups.size() > 1) cpu_pool_->parallel_for(int(groups.size()), run);
  else
    for (int g = 0; g < int(groups.size()); ++g) run(g);
}

void Worker::run_cpu_job(std::vector<DecodeJob>& jobs, std::vector<int>& slots, std::vector<u32>& err, size_t i) {
  {
    Camera& c = *cams_[size_t(jobs[i].cam)];
    const PictureInfo& pi = jobs[i].pic;
    for (int sl = pi.spec_lo; sl < pi.spec_hi && !err[i]; ++sl) {  // speculative headers
      const u8* b = jobs[i].upd.block(sl);
      err[i] = (b[-2] != 0x0D || b[-1] != 0x00) ? 1u : 0u;
    }
    if (err[i]) return;
    if (jobs[i].ext) {  // VCN picture (host-visible planes on the CPU backend)
      const vcn::Frame& f = *jobs[i].ext;
      HostSurface& hs = c.surface.host[0];
      VEP_CHECK(f.width <= hs.coded_w && f.height <= hs.coded_h, "VCN picture exceeds the camera surface");
      for (int r = 0; r < f.height; ++r)
        std::memcpy(&hs.y[size_t(r) * size_t(hs.coded_w)], f.y + size_t(r) * f.pitch_y, size_t(f.width));
      for (int r = 0; r < f.height / 2; ++r)
        std::memcpy(&hs.uv[size_t(r) * size_t(hs.coded_w)], f.uv + size_t(r) * f.pitch_uv, size_t(f.width));
    } else if (jobs[i].general()) {
      for (const auto& pic : jobs[i].avc) {
        if (!pic->structure) {
          avc::cpu_reconstruct(*pic, c.surface.host);
          continue;
        }
        auto& F = c.surface.fields;  // field slots (half-height surfaces)
        if (F.size() < size_t(pic->dpb_slots)) F.resize(size_t(pic->dpb_slots));
        for (auto& h : F)
          if (h.coded_w != pic->wmbs * 16 || h.coded_h != pic->hmbs * 16 || h.bd != pic->bd || h.cf != pic->cf)
            h.alloc(pic->wmbs * 16, pic->hmbs * 16, pic->bd, pic->cf);
        avc::cpu_reconstruct(*pic, F);
      }
      for (const auto& pic : jobs[i].hevc) hevc::cpu_execute(*pic, c.surface.host);
    } else {
      cpu_apply_update(jobs[i].upd, c.surface.host[0]);
    }
    if (!jobs[i].has_output()) return;
    HostSurface narrow;  // Main10: the 8-bit copy the conversion and the letterbox read
    HostSurface woven;   // a field pair's frame
    if (jobs[i].out_fields) {
      const size_t t = size_t(jobs[i].target());
      VEP_CHECK(2 * t + 1 < c.surface.fields.size(), "field pair output without its fields");
      avc::weave_fields(c.surface.fields[2 * t], c.surface.fields[2 * t + 1], woven);
    }
    const HostSurface& out = jobs[i].out_fields ? woven : c.surface.host[size_t(jobs[i].target())];
    const bool conv = out.wide() || out.cf == 2;
    if (conv) narrow_surface(out, narrow);
    const HostSurface& src = conv ? narrow : out;
    cpu_nv12_to_bgr(src, jobs[i].pic.crop_left, jobs[i].pic.crop_top,
                    jobs[i].pic.width, jobs[i].pic.height, c.ring_->slot_ptr(slots[i]));
    if (opt_.ref_copies) {  // read_image.py:97 tobytes() + :119 SerializeToString()
      const size_t n = size_t(jobs[i].pic.width) * size_t(jobs[i].pic.height) * 3;
      std::vector<u8> bytes(c.ring_->slot_ptr(slots[i]), c.ring_->slot_ptr(slots[i]) + n);
      FrameMeta m{};
      m.width = jobs[i].pic.width;
      m.height = jobs[i].pic.height;
      m.pts = jobs[i].meta.pts;
      const auto pre_suf = encode_video_frame(m, n, c.name());
      std::string msg;
      msg.reserve(pre_suf.first.size() + n + pre_suf.second.size());
      msg += pre_suf.first;
      msg.append(reinterpret_cast<const char*>(bytes.data()), n);
      msg += pre_suf.second;
      ref_copy_bytes_.fetch_add(msg.size(), std::memory_order_relaxed);
    }
    if (opt_.letterbox_size > 0) {
      gpu::LetterboxDesc l{};
      const size_t S = size_t(opt_.letterbox_size);
      l.src_w = jobs[i].pic.width;
      l.src_h = jobs[i].pic.height;
      l.crop_left = jobs[i].pic.crop_left;
      l.crop_top = jobs[i].pic.crop_top;
      const bool nv12 = opt_.letterbox_format == gpu::kLbNV12;
      l.out_hwc = cons_hwc_ ? cons_hwc_ + size_t(jobs[i].cam) *
                                              gpu::letterbox_bytes(int(S), opt_.letterbox_format)
                            : nullptr;
      l.out_chw = (cons_chw_ && opt_.chw_dtype == gpu::kChwF32)
                      ? static_cast<u8*>(cons_chw_) + size_t(jobs[i].cam) * 3 * S * S * 4
                      : nullptr;
      gpu::fill_letterbox_geometry(l, opt_.letterbox_size, nv12);
      if (nv12) {
        cpu_letterbox_nv12(src, l, opt_.letterbox_size, 114);
        return;
      }
      gpu::LetterboxParams p{};
      p.size = opt_.letterbox_size;
      p.chw_dtype = opt_.chw_dtype;
      for (int k = 0; k < 3; ++k) {
        p.mean[k] = opt_.mean[k];
        p.inv_std[k] = 1.f / opt_.std[k];
      }
      p.pad_value = 114;
      cpu_letterbox(src, l, p);
    }
  }
}

// Worker thread, per finished job of a camera: records the job's dropped pictures / poisoned
// CRAs and tells whether its output is one of the recorded stale pictures (each is output once:
// the entry is erased) or a RASL picture of a poisoned CRA.
bool stale_output(Camera& c, const DecodeJob& j, bool check) {
  const u64 now = ++c.jobs_seen_;
  for (const auto& d : j.dropped) c.stale_.push_back({d.first, d.second, now + Camera::kStaleJobs});
  for (i64 tag : j.poisoned_cra) c.bad_cra_.emplace_back(tag, now + Camera::kStaleJobs);
  c.stale_.erase(std::remove_if(c.stale_.begin(), c.stale_.end(), [&](const Camera::StaleOut& s) { return s.until < now; }),
                 c.stale_.end());
  c.bad_cra_.erase(std::remove_if(c.bad_cra_.begin(), c.bad_cra_.end(), [&](const auto& b) { return b.second < now; }),
                   c.bad_cra_.end());
  if (c.stale_.size() > 64) c.stale_.erase(c.stale_.begin(), c.stale_.end() - 64);
  if (!check) return false;
  for (auto it = c.stale_.begin(); it != c.stale_.end(); ++it)
    if (it->slot == j.out_slot && it->pts == j.meta.pts) {
      c.stale_.erase(it);
      return true;
    }
  if (j.out_rasl_of >= 0)
    for (const auto& b : c.bad_cra_)
      if (b.first == j.out_rasl_of) return true;
  return false;
}

void Worker::publish(std::vector<DecodeJob>& jobs, std::vector<int>& slots, const u32* err) {
  trace::Range tr("vep.publish");
  const i64 t = mono_us();
  const i64 wall = now_ms();
  std::lock_guard<std::mutex> g(cams_mu_);
  for (size_t i = 0; i < jobs.size(); ++i) {
    auto& cp = cams_[size_t(jobs[i].cam)];
    const bool out = jobs[i].has_output();
    if (!cp || !cp->ring_) {
      if (out) dropped_.fetch_add(1, std::memory_order_relaxed);
      continue;
    }
    if (!(err && err[i]) && !cp->broken_) {
      // decoded frames (a field pair counts once: its second field)
      u64 np = jobs[i].general() ? jobs[i].hevc.size() : 1;
      for (const auto& p : jobs[i].avc) np += !p->structure || p->second_field;
      pictures_.fetch_add(np, std::memory_order_relaxed);
      cp->pictures.fetch_add(np, std::memory_order_relaxed);
    }
    const bool stale = stale_output(*cp, jobs[i], out && jobs[i].general());
    if (!out) {  // reconstruction only (its pictures wait in the reorder buffer)
      if (err && err[i]) {
        cp->errors.fetch_add(1, std::memory_order_relaxed);
        cp->logs.add(true, "GPU reconstruction wavefront timed out; waiting for the next keyframe");
        cp->broken_ = true;
      } else if (jobs[i].refresh) {
        cp->broken_ = false;  // a keyframe reconstructed (its picture is published later)
      }
      continue;
    }
    if (err && err[i]) {
      dropped_.fetch_add(1, std::memory_order_relaxed);
      cp->errors.fetch_add(1, std::memory_order_relaxed);
      // err bit 0: a speculatively placed I_PCM block failed its header check (decode_convert);
      // bit 1: a reconstruction wavefront timed out waiting for a neighbour (gpu_avc.hip)
      if (err[i] & 2u)
        cp->logs.add(true, "GPU reconstruction wavefront timed out; frame dropped, waiting for the next keyframe");
      if (err[i] & 0xFF00u) {  // (gpu_avc.hip / gpu_avc_hbd.hip bound checks)
        char b[96];
        std::snprintf(b, sizeof b, "GPU reconstruction bound check failed (0x%x); frame dropped", err[i]);
        cp->logs.add(true, b);
        std::fprintf(stderr, "vep: camera %s: %s\n", cp->name().c_str(), b);
      } else if (err[i] & ~2u) {
        cp->logs.add(true, "corrupt keyframe: I_PCM header check failed; waiting for the next keyframe");
      }
      cp->broken_ = true;
      cp->ring_->abort(slots[i]);
      continue;
    }
    if (cp->broken_) {  // surfaces are garbage until a keyframe rewrites every MB
      if (!jobs[i].refresh) {
        cp->ring_->abort(slots[i]);
        dropped_.fetch_add(1, std::memory_order_relaxed);
        continue;
      }
      cp->broken_ = false;
    }
    if (stale) {  // its reconstruction was dropped with a backlog (or predicts from one): a stale surface
      cp->ring_->abort(slots[i]);
      shed_.fetch_add(1, std::memory_order_relaxed);
      cp->shed.fetch_add(1, std::memory_order_relaxed);
      continue;
    }
    jobs[i].meta.decoded_us = t;
    if (jobs[i].meta.arrival_ms > 0) {
      const i64 lat = std::max<i64>(0, wall - jobs[i].meta.arrival_ms);
      int b = 0;
      while (b < Camera::kLatBuckets - 1 && double(lat) > Camera::kLatBucketsMs[b]) ++b;
      cp->lat_hist[b].fetch_add(1, std::memory_order_relaxed);
      cp->lat_sum_ms.fetch_add(u64(lat), std::memory_order_relaxed);
    }
    cp->ring_->commit(slots[i], jobs[i].meta);
    cp->out_surface_slot = jobs[i].general() && !jobs[i].out_fields ? jobs[i].target() : -1;
    cp->out_surface_pts = jobs[i].meta.pts;
    cp->decoded.fetch_add(1, std::memory_order_relaxed);
    frames_.fetch_add(1, std::memory_order_relaxed);
    if (auto hook = std::atomic_load(&publish_hook_)) (*hook)(jobs[i].cam, cp->ring_->published());
  }
  batches_.fetch_add(1);
}

void Worker::set_publish_hook(std::function<void(int, i64)> f) {
  std::shared_ptr<std::function<void(int, i64)>> h;
  if (f) h = std::make_shared<std::function<void(int, i64)>>(std::move(f));
  std::lock_guard<std::mutex> g(cams_mu_);  // (publish holds it: no hook call is in flight after this)
  std::atomic_store(&publish_hook_, h);
}

double Worker::gpu_ms_total() const {
  double m = 0;
  for (const auto& lp : lanes_) m = std::max(m, lp->gpu_ms.load());
  return m;
}

void Worker::add_time(double Timers::*f, double us) {
  std::lock_guard<std::mutex> g(timers_mu_);
  timers.*f += us;
}

// Wait for a batch's completion event without spinning a CPU core. hipEventSynchronize busy-polls
// the HSA completion signal (rdtsc loop in libhsa-runtime64) even for hipEventBlockingSync events
// for a while before it sleeps: in the host profile of the headline that spin was 17% of the
// process's CPU samples, taken from the parse threads. A lane only needs to notice its stage is
// free within a fraction of a batch (~5 ms), so it polls the event and sleeps between polls.
static void wait_event_polite(hipEvent_t e) {
  for (int i = 0;; ++i) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return;
    if (r != hipErrorNotReady) VEP_HIP(r);
    if (i < 2) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(40));
  }
}

void Worker::complete(Lane& ln, Stage& st) {
  if (!st.active) return;
  st.active = false;
  const i64 t0 = mono_us();
  {
    trace::Range tr("vep.wait_gpu");
    if (polite_wait_) wait_event_polite(st.e1);
    else VEP_HIP(hipEventSynchronize(st.e1));
  }
  add_time(&Timers::wait, double(mono_us() - t0));
  float ms = 0;
  if (hipEventElapsedTime(&ms, st.e0, st.e1) == hipSuccess) ln.gpu_ms.store(ln.gpu_ms.load() + ms);
  publish(st.jobs, st.slots, st.err);
  st.jobs.clear();
  st.slots.clear();
  {
    std::lock_guard<std::mutex> g(pub_mu_);
    while (!ln.unpublished.empty() && ln.unpublished.front() >= st.seq && ln.unpublished.front() <= st.seq_last)
      ln.unpublished.pop_front();
  }
  pub_cv_.notify_all();
}

void Worker::launch_on(Lane& ln, Batch&& b) {
  Stage& st = ln.stage[size_t(ln.next)];
  ln.next = (ln.next + 1) % int(ln.stage.size());
  complete(ln, st);  // this lane's oldest batch (`stages` launches ago): its staging is reused
  st.jobs.swap(b.jobs);
  st.slots.swap(b.slots);
  st.seq = b.seq;
  st.seq_last = std::max(b.seq, b.seq_last);
  st.cons_hwc = b.cons_hwc;
  st.cons_chw = b.cons_chw;
  st.cons_rows = b.cons_rows;
  try {
    std::shared_lock<std::shared_mutex> gate(cons_gate_);
    const u64 sg = snap_gen_.load();
    if (ln.snap_seen != sg) {  // this batch's letterbox writes wait for the last snapshot's copy
      VEP_HIP(hipStreamWaitEvent(ln.stream, snap_ev_, 0));
      ln.snap_seen = sg;
    }
    launch_gpu(ln, st);
  } catch (...) {
    // the batch is dropped: give its ring slots back and count it as published
    {
      std::lock_guard<std::mutex> g(cams_mu_);
      for (size_t i = 0; i < st.jobs.size(); ++i) {
        auto& cp = cams_[size_t(st.jobs[i].cam)];
        if (cp && cp->ring_ && st.slots[i] >= 0) cp->ring_->abort(st.slots[i]);
      }
      for (const auto& j : st.jobs) dropped_.fetch_add(j.has_output() ? 1 : 0, std::memory_order_relaxed);
    }
    st.jobs.clear();
    st.slots.clear();
    {
      std::lock_guard<std::mutex> g(pub_mu_);
      while (!ln.unpublished.empty() && ln.unpublished.front() >= st.seq && ln.unpublished.front() <= st.seq_last)
        ln.unpublished.pop_front();
    }
    pub_cv_.notify_all();
    throw;
  }
  st.active = true;
}

// Batches that queued behind this lane's in-flight ones (ln.mu held) join `b`: one launch per
// kernel for all of them. The wavefront kernels (intra, deblock) take about the same time for
// one picture as for many (a picture's latency is its MB-row chain, and a launch of one picture
// fills a few CUs of 256), and the batches would run back to back on the lane's stream anyway,
// so merging turns queueing into parallel work without holding anything back: nothing waits
// for a merge, only what is already waiting is merged. A camera appears at most once per launch
// (its pictures inside one job are rounds; two jobs of one camera in one launch would put
// dependent pictures in the same round), so the merge stops at a batch that repeats a camera,
// at a different consumer batch, or at merge_jobs_ jobs.
void Worker::merge_queued(Lane& ln, Batch& b) {
  if (merge_jobs_ <= 0) return;
  while (!ln.q.empty()) {
    Batch& n = ln.q.front();
    if (n.cons_hwc != b.cons_hwc || n.cons_chw != b.cons_chw || n.cons_rows != b.cons_rows) break;
    if (int(b.jobs.size() + n.jobs.size()) > merge_jobs_) break;
    bool repeat = false;
    for (const DecodeJob& j : n.jobs) {
      for (const DecodeJob& k : b.jobs)
        if (k.cam == j.cam) {
          repeat = true;
          break;
        }
      if (repeat) break;
    }
    if (repeat) break;
    for (size_t i = 0; i < n.jobs.size(); ++i) {
      b.jobs.push_back(std::move(n.jobs[i]));
      b.slots.push_back(n.slots[i]);
    }
    b.seq_last = std::max(n.seq, n.seq_last);
    ln.q.pop_front();
    merged_.fetch_add(1, std::memory_order_relaxed);
  }
}

// Launcher thread of one lane: launches the batches handed over by launch_async, each after
// its staging buffer's previous batch is complete and published, so a lane waiting on a slow
// batch (a keyframe's intra wavefront) never holds back the other lanes.
void Worker::lane_loop(Lane& ln) {
  dev_.bind();
  auto keep_error = [&] {
    std::lock_guard<std::mutex> g(pub_mu_);
    if (!lane_err_) lane_err_ = std::current_exception();
  };
  std::unique_lock<std::mutex> lk(ln.mu);
  for (;;) {
    ln.cv.wait(lk, [&] { return ln.stop || ln.drain || (!ln.q.empty() && !hold_.load()); });
    if (!ln.q.empty() && (!hold_.load() || ln.drain || ln.stop)) {
      Batch b = std::move(ln.q.front());
      ln.q.pop_front();
      merge_queued(ln, b);
      ln.busy = true;
      lk.unlock();
      ln.cv.notify_all();  // room for the next batch
      try {
        launch_on(ln, std::move(b));
      } catch (...) {
        keep_error();
      }
      lk.lock();
      ln.busy = false;
      ln.cv.notify_all();
      continue;
    }
    if (ln.drain) {
      lk.unlock();
      try {
        for (size_t k = 0; k < ln.stage.size(); ++k)
          complete(ln, ln.stage[(size_t(ln.next) + k) % ln.stage.size()]);
      } catch (...) {
        keep_error();
      }
      lk.lock();
      ln.drain = false;
      ln.cv.notify_all();
      continue;
    }
    if (ln.stop) return;
  }
}

void Worker::hold_lanes(bool hold) {
  hold_.store(hold);
  for (auto& lp : lanes_) {
    std::lock_guard<std::mutex> g(lp->mu);  // (a launcher between its predicate check and its wait)
  }
  for (auto& lp : lanes_) lp->cv.notify_all();
}

void Worker::drain_lanes() {
  for (auto& lp : lanes_) {
    std::lock_guard<std::mutex> g(lp->mu);
    lp->drain = true;
  }
  for (auto& lp : lanes_) lp->cv.notify_all();
  for (auto& lp : lanes_) {
    Lane& ln = *lp;
    std::unique_lock<std::mutex> lk(ln.mu);
    ln.cv.wait(lk, [&] { return !ln.drain && ln.q.empty() && !ln.busy; });
  }
  std::exception_ptr e;
  {
    std::lock_guard<std::mutex> g(pub_mu_);
    std::swap(e, lane_err_);
  }
  if (e) std::rethrow_exception(e);
}

void Worker::complete_locked() {
  if (threaded_) {
    drain_lanes();
    return;
  }
  // oldest first: Lane::next names the stage that will be reused next, i.e. the oldest batch
  for (auto& lp : lanes_)
    for (size_t k = 0; k < lp->stage.size(); ++k)
      complete(*lp, lp->stage[(size_t(lp->next) + k) % lp->stage.size()]);
}

void Worker::complete_all() {
  std::lock_guard<std::mutex> lg(launch_mu_);
  if (dev_.gpu()) dev_.bind();
  complete_locked();
}

void Worker::wait_published(u64 seq) {
  std::unique_lock<std::mutex> g(pub_mu_);
  pub_cv_.wait(g, [&] {
    for (const auto& lp : lanes_)
      if (!lp->unpublished.empty() && lp->unpublished.front() <= seq) return false;
    return true;
  });
}

void Worker::launch_async(std::vector<DecodeJob>& jobs) {
  trace::Range tr("vep.launch_async");
  if (jobs.empty()) return;
  std::lock_guard<std::mutex> lg(launch_mu_);
  dev_.bind();
  std::vector<int> slots;
  const i64 t0 = mono_us();
  prepare(jobs, slots);
  add_time(&Timers::prepare, double(mono_us() - t0));
  if (jobs.empty()) return;
  if (!dev_.gpu()) {
    std::vector<u32> err;
    run_cpu(jobs, slots, err);
    publish(jobs, slots, err.data());
    jobs.clear();
    return;
  }
  const size_t nl = lanes_.size();
  std::vector<std::vector<DecodeJob>> lj(nl);
  std::vector<std::vector<int>> ls(nl);
  for (size_t i = 0; i < jobs.size(); ++i) {
    const size_t g = size_t(jobs[i].cam) % nl;  // a camera's surfaces are ordered by its lane
    lj[g].push_back(std::move(jobs[i]));
    ls[g].push_back(slots[i]);
  }
  jobs.clear();
  const u64 seq = ++launch_seq_;
  for (size_t g = 0; g < nl; ++g) {
    if (lj[g].empty()) continue;
    Lane& ln = *lanes_[g];
    {
      std::lock_guard<std::mutex> pg(pub_mu_);
      ln.unpublished.push_back(seq);
    }
    Batch b{std::move(lj[g]), std::move(ls[g]), seq, seq, cons_hwc_, cons_chw_, cons_rows_};
    if (!threaded_) {
      launch_on(ln, std::move(b));
      continue;
    }
    std::unique_lock<std::mutex> lk(ln.mu);
    ln.cv.wait(lk, [&] { return int(ln.q.size()) < queue_; });  // bounded per-lane backlog
    ln.q.push_back(std::move(b));
    lk.unlock();
    ln.cv.notify_all();
  }
  if (threaded_) {
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> g(pub_mu_);
      std::swap(e, lane_err_);
    }
    if (e) std::rethrow_exception(e);
  }
}

std::vector<u64> Worker::avc_profile() {
  std::vector<u64> v(gpu::kAvcProfSlots, 0);
  if (!avc_prof_) return v;
  complete_all();
  VEP_HIP(hipMemcpy(v.data(), avc_prof_, v.size() * sizeof(u64), hipMemcpyDeviceToHost));
  return v;
}

void Worker::run_batch(std::vector<DecodeJob>& jobs) {
  launch_async(jobs);
  complete_all();
}

bool Worker::read_latest(int cam, i64 after, FrameMeta* meta, u8* dst, size_t cap) {
  std::shared_ptr<Camera> c = camera(cam);
  if (!c) return false;
  std::shared_ptr<FrameRing> r = c->ring();
  return r && read_latest(*r, after, meta, dst, cap);
}

Worker::ServeBuf* Worker::acquire_serve(size_t n) {
  ServeBuf* b = nullptr;
  {
    std::unique_lock<std::mutex> g(serve_mu_);
    if (serve_free_.empty() && serve_all_.size() < size_t(kServeBufs)) {
      serve_all_.push_back(std::make_unique<ServeBuf>());
      serve_free_.push_back(serve_all_.back().get());
    }
    serve_cv_.wait(g, [&] { return !serve_free_.empty(); });
    b = serve_free_.back();
    serve_free_.pop_back();
  }
  if (b->cap < n) {  // first use, or a larger ring (resolution change)
    dev_.free_pinned(b->h);
    b->h = static_cast<u8*>(dev_.alloc_pinned(n));
    b->cap = n;
  }
  if (!b->ev[0] && dev_.gpu())
    for (hipEvent_t& e : b->ev)  // waiters sleep: several server threads wait at once
      VEP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync));
  return b;
}

void Worker::release_serve(ServeBuf* b) {
  {
    std::lock_guard<std::mutex> g(serve_mu_);
    serve_free_.push_back(b);
  }
  serve_cv_.notify_one();
}

bool Worker::register_host(void* p, size_t n) {
  if (!dev_.gpu() || !p || !n) return false;
  dev_.bind();
  if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}

void Worker::unregister_host(void* p) {
  if (!dev_.gpu() || !p) return;
  dev_.bind();
  (void)hipHostUnregister(p);
}

bool Worker::read_latest(FrameRing& rg, i64 after, FrameMeta* meta, u8* dst, size_t cap, bool dst_pinned) {
  FrameRing* ring = &rg;
  for (int attempt = 0; attempt < 4; ++attempt) {
    int slot;
    if (!ring->latest(after, meta, &slot)) return false;
    const size_t n = ring->slot_bytes();
    VEP_CHECK(cap >= n, "read_latest destination too small");
    if (dev_.gpu() && dst_pinned) {
      dev_.bind();
      ServeBuf* b = acquire_serve(0);  // only its completion event: the DMA lands in dst
      try {
        VEP_HIP(hipMemcpyAsync(dst, ring->slot_ptr(slot), n, hipMemcpyDeviceToHost, serve_stream_));
        VEP_HIP(hipEventRecord(b->ev[0], serve_stream_));
        VEP_HIP(hipEventSynchronize(b->ev[0]));
      } catch (...) {
        release_serve(b);
        throw;
      }
      release_serve(b);
      if (!ring->still_valid(slot, meta->seq)) continue;
      return true;
    }
    if (dev_.gpu() || mock_serve_) {  // (mock: the same pool and chunking, memcpy for the DMA)
      const bool gpu = dev_.gpu();
      if (gpu) dev_.bind();
      ServeBuf* b = acquire_serve(n);
      const u8* src = ring->slot_ptr(slot);
      const size_t chunk = (n + kServeChunks - 1) / kServeChunks;
      try {
        for (int k = 0; k < kServeChunks; ++k) {
          const size_t off = size_t(k) * chunk;
          if (off >= n) break;
          if (!gpu) {
            std::memcpy(b->h + off, src + off, std::min(chunk, n - off));
            continue;
          }
          VEP_HIP(hipMemcpyAsync(b->h + off, src + off, std::min(chunk, n - off), hipMemcpyDeviceToHost,
                                 serve_stream_));
          VEP_HIP(hipEventRecord(b->ev[k], serve_stream_));
        }
        for (int k = 0; k < kServeChunks; ++k) {
          const size_t off = size_t(k) * chunk;
          if (off >= n) break;
          if (gpu) VEP_HIP(hipEventSynchronize(b->ev[k]));
          std::memcpy(dst + off, b->h + off, std::min(chunk, n - off));
        }
      } catch (...) {
        release_serve(b);
        throw;
      }
      release_serve(b);
      if (!ring->still_valid(slot, meta->seq)) continue;
      return true;
    }
    std::memcpy(dst, ring->slot_ptr(slot), n);
    if (ring->still_valid(slot, meta->seq)) return true;
  }
  return false;
}

size_t Worker::snapshot_consumer(void* dst, size_t cap, int rows, hipStream_t stream) {
  VEP_CHECK(opt_.letterbox_size > 0 && cons_hwc_, "consumer batch disabled (letterbox_size is 0)");
  rows = std::clamp(rows, 0, cons_rows_);
  const size_t n = size_t(rows) * gpu::letterbox_bytes(opt_.letterbox_size, opt_.letterbox_format);
  VEP_CHECK(cap >= n, "snapshot_consumer destination too small");
  if (!n) return 0;
  if (!dev_.gpu()) {  // CPU backend: rows are written by launch_async (under launch_mu_)
    std::lock_guard<std::mutex> g(launch_mu_);
    std::memcpy(dst, cons_hwc_, n);
    snap_gen_.fetch_add(1);
    return n;
  }
  std::unique_lock<std::shared_mutex> gate(cons_gate_);  // no lane enqueues meanwhile
  dev_.bind();
  if (!snap_ev_) {
    VEP_HIP(hipEventCreateWithFlags(&snap_ev_, hipEventDisableTiming));
    for (auto& lp : lanes_) VEP_HIP(hipEventCreateWithFlags(&lp->snap_mark, hipEventDisableTiming));
  }
  const hipStream_t s = stream ? stream : serve_stream_;
  for (auto& lp : lanes_) {  // after every letterbox write enqueued so far
    VEP_HIP(hipEventRecord(lp->snap_mark, lp->stream));
    VEP_HIP(hipStreamWaitEvent(s, lp->snap_mark, 0));
  }
  VEP_HIP(hipMemcpyAsync(dst, cons_hwc_, n, hipMemcpyDeviceToDevice, s));
  VEP_HIP(hipEventRecord(snap_ev_, s));  // ... and before any later one (launch_on waits on it)
  snap_gen_.fetch_add(1);
  if (!stream) VEP_HIP(hipStreamSynchronize(s));
  return n;
}

void Worker::read_latest_many(std::vector<ReadReq>& reqs) {
  if (!dev_.gpu()) {
    for (auto& r : reqs) r.ok = read_latest(*r.ring, r.after, &r.meta, r.dst, r.cap, r.pinned);
    return;
  }
  dev_.bind();
  std::vector<int> slot(reqs.size(), -1);
  bool queued = false;
  for (size_t k = 0; k < reqs.size(); ++k) {
    ReadReq& r = reqs[k];
    r.ok = false;
    if (!r.pinned) {
      r.ok = read_latest(*r.ring, r.after, &r.meta, r.dst, r.cap, false);
      continue;
    }
    if (!r.ring->latest(r.after, &r.meta, &slot[k])) continue;
    VEP_CHECK(r.cap >= r.ring->slot_bytes(), "read_latest_many destination too small");
    VEP_HIP(hipMemcpyAsync(r.dst, r.ring->slot_ptr(slot[k]), r.ring->slot_bytes(), hipMemcpyDeviceToHost,
                           serve_stream_));
    queued = true;
  }
  if (!queued) return;
  ServeBuf* b = acquire_serve(0);  // (its completion event)
  try {
    VEP_HIP(hipEventRecord(b->ev[0], serve_stream_));
    VEP_HIP(hipEventSynchronize(b->ev[0]));
  } catch (...) {
    release_serve(b);
    throw;
  }
  release_serve(b);
  for (size_t k = 0; k < reqs.size(); ++k)  // a slot the writer reused meanwhile is not served
    if (slot[k] >= 0) reqs[k].ok = reqs[k].ring->still_valid(slot[k], reqs[k].meta.seq);
}

// --------------------------------------------------------------------------- proto encoding

static void put_varint(std::string& s, u64 v) {
  while (v >= 0x80) {
    s.push_back(char((v & 0x7f) | 0x80));
    v >>= 7;
  }
  s.push_back(char(v));
}
static void put_tag(std::string& s, int field, int wt) { put_varint(s, u64(field) << 3 | u64(wt)); }
static void put_i64(std::string& s, int field, i64 v) {
  if (v == 0) return;
  put_tag(s, field, 0);
  put_varint(s, u64(v));
}
static void put_bool(std::string& s, int field, bool v) {
  if (!v) return;
  put_tag(s, field, 0);
  s.push_back(1);
}
static void put_str(std::string& s, int field, const std::string& v) {
  if (v.empty()) return;
  put_tag(s, field, 2);
  put_varint(s, v.size());
  s += v;
}

std::pair<std::string, std::string> encode_video_frame(const FrameMeta& m, size_t data_len,
                                                       const std::string& device_id) {
  std::string pre, suf;
  put_i64(pre, 1, m.width);
  put_i64(pre, 2, m.height);
  if (data_len) {
    put_tag(pre, 3, 2);
    put_varint(pre, data_len);
  }
  put_i64(suf, 4, m.timestamp);
  put_bool(suf, 5, m.is_keyframe);
  put_i64(suf, 6, m.pts);
  put_i64(suf, 7, m.dts);
  if (m.frame_type != '?' && m.frame_type != 0) put_str(suf, 8, std::string(1, m.frame_type));
  put_bool(suf, 9, m.is_corrupt);
  if (m.time_base != 0.0) {
    put_tag(suf, 10, 1);
    u64 bits;
    std::memcpy(&bits, &m.time_base, 8);
    for (int i = 0; i < 8; ++i) suf.push_back(char((bits >> (8 * i)) & 0xff));
  }
  if (m.width > 0) {  // ShapeProto{dim: [(H,"0"), (W,"1"), (3,"2")]}
    std::string shape;
    const i64 dims[3] = {m.height, m.width, 3};
    for (int k = 0; k < 3; ++k) {
      std::string dim;
      put_i64(dim, 1, dims[k]);
      put_str(dim, 2, std::string(1, char('0' + k)));
      put_tag(shape, 2, 2);
      put_varint(shape, dim.size());
      shape += dim;
    }
    put_tag(suf, 11, 2);
    put_varint(suf, shape.size());
    suf += shape;
  }
  put_str(suf, 12, device_id);
  put_i64(suf, 13, m.packet);
  put_i64(suf, 14, m.keyframe);
  return {pre, suf};
}

}  // namespace vep
