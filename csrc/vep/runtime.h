// Data-plane runtime: per-camera HBM frame rings, lazy-decode camera state and the per-GPU
// worker that batches every camera's decode into one HIP launch.
//
// Reference parity:
//  * FrameRing replaces the Redis stream `XADD <device> MAXLEN n` / `XREAD` frame cache
//    (python/read_image.py:121, server/grpcapi/grpc_api.go:186-231).
//  * Camera's control atomics replace the Redis keys `last_access_time_<dev>`
//    {last_query, proxy_rtmp} and `is_key_frame_only_<dev>`.
//  * Camera::on_access_unit implements the lazy decode / keyframe-only / GOP catch-up rules of
//    rtsp_to_rtmp.py:94-160 and read_image.py:57-128.
#pragma once

#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>

#include "avc.h"
#include "codec.h"
#include "hevc_dec.h"
#include "hevc_kern.h"
#include "hostplan.h"
#include "ioloop.h"
#include "gpu.h"
#include "pool.h"
#include "vcn.h"

namespace vep {

// VideoFrame metadata (proto/video_streaming.proto VideoFrame; read_image.py:99-117).
struct FrameMeta {
  i64 width = 0, height = 0;
  i64 timestamp = 0, pts = 0, dts = 0;
  i64 packet = 0, keyframe = 0;  // index in GOP, GOP counter
  bool is_keyframe = false, is_corrupt = false;
  char frame_type = '?';
  double time_base = 1.0 / 90000.0;
  i64 seq = 0;            // ring publish counter (per-client cursor, XREAD lastId analog)
  i64 decoded_us = 0;     // monotonic time the frame became readable
  i64 arrival_ms = 0;     // packet arrival wall clock
};

// Device (or host) memory owner. id < 0 selects the CPU backend.
class Device {
 public:
  explicit Device(int id);
  ~Device();
  bool gpu() const { return id_ >= 0; }
  int id() const { return id_; }
  void* alloc(size_t n);
  void free(void* p);
  void* alloc_pinned(size_t n);
  void free_pinned(void* p);
  void bind() const;  // hipSetDevice on the calling thread

 private:
  int id_;
};

// Ring of N decoded BGR24 frames for one camera, seqlock-published.
class FrameRing {
 public:
  FrameRing(Device& dev, int slots, int width, int height);
  ~FrameRing();
  int slots() const { return int(slots_.size()); }
  int width() const { return w_; }
  int height() const { return h_; }
  size_t slot_bytes() const { return size_t(w_) * h_ * 3; }
  u8* slot_ptr(int i) const { return base_ + size_t(i) * slot_bytes(); }
  // writer side (single writer: the worker thread)
  int begin_write();
  void commit(int slot, FrameMeta meta);
  // Release a slot from begin_write() without publishing (frame dropped after a failed check).
  void abort(int slot);
  // reader side: newest committed frame with seq > after (false if none)
  bool latest(i64 after, FrameMeta* meta, int* slot) const;
  // true if `slot` still holds the frame with publish counter `seq`
  bool still_valid(int slot, i64 seq) const;
  i64 published() const { return published_.load(std::memory_order_acquire); }
  // Block until a frame with seq > after is published (XREAD ... BLOCK analog).
  bool wait_newer(i64 after, int timeout_ms) const;

 private:
  mutable std::condition_variable cv_;
  struct Slot {
    std::atomic<u64> version{0};  // odd while being written
    FrameMeta meta;
  };
  Device& dev_;
  int w_, h_;
  u8* base_ = nullptr;
  std::vector<std::unique_ptr<Slot>> slots_;
  mutable std::mutex meta_mu_;
  std::atomic<int> latest_{-1};
  std::atomic<i64> published_{0};
  int next_ = 0;
};

struct DecodeJob {
  int cam = -1;
  MbUpdate upd;                        // PCM / skip fast path (collapsible)
  std::vector<avc::PicturePtr> avc;    // general H.264 path: pictures in decoding order
  std::vector<hevc::GpuPicturePtr> hevc;  // general H.265 path: reconstruction records
  int hevc_slots = 0;                  // DPB surfaces the H.265 pictures use
  PictureInfo pic;                     // the published frame's picture (sizes of the surfaces)
  FrameMeta meta;
  bool refresh = false;  // IDR: every MB is covered
  bool keyframe_only = false;  // from a keyframe-only camera (one picture per GOP)

  // General path: DPB slot of the newest picture that left the reorder buffer in this job (it is
  // converted and published), -1 when every picture of the job is still waiting for output
  // (B-frame reordering): the job then only reconstructs.
  int out_slot = -1;
  bool out_fields = false;  // H.264 field pair: out_slot holds two fields (avc::OutFrame::fields)
  // (slot, pts) of the pictures a keyframe's job dropped from the backlog it replaced
  // (merge_job): the reorder buffer may still output them from later jobs; they are not published
  std::vector<std::pair<int, i64>> dropped;
  // H.265: decode tags of CRA pictures such a job restarted from. Their RASL pictures predict from
  // pictures before the CRA, possibly dropped ones: they are not published either.
  std::vector<i64> poisoned_cra;
  i64 out_rasl_of = -1;  // H.265: the output picture is a RASL picture of the CRA with this tag
  // VCN backend (vcn.h): a picture decoded by the video core; the worker copies its planes into
  // the camera's surface, then converts / letterboxes / publishes it like any other frame.
  vcn::FramePtr ext;
  bool general() const { return !avc.empty() || !hevc.empty(); }
  bool has_output() const { return !general() || out_slot >= 0; }
  // (H.265: the DPB slots plus one scratch surface, the SAO input copy)
  int dpb_slots() const { return !avc.empty() ? avc.back()->dpb_slots : (!hevc.empty() ? hevc_slots + 1 : 1); }
  // bytes per sample of the camera's surfaces: 2 for Main10 pictures (u16 samples), else 1
  // (High 10 H.264 / Main10 H.265: u16 samples at the stream's bit depth)
  int bit_depth() const {
    if (!avc.empty()) return avc.back()->bd;
    if (!hevc.empty()) return std::max(hevc.back()->bd_y, hevc.back()->bd_c);
    return 8;
  }
  int bytes_per_sample() const { return bit_depth() > 8 ? 2 : 1; }
  int chroma_format() const { return !avc.empty() && avc.back()->cf == 2 ? 2 : 1; }
  int target() const { return general() ? out_slot : 0; }
};

// Fold `job` into the not-yet-launched job `p` of the same camera (GOP catch-up collapse).
void merge_job(DecodeJob& p, DecodeJob&& job);

class Worker;

// Bounded log ring (docker json-file analog, rtsp_process_manager.go:72-75; Info returns 100).
class LogRing {
 public:
  void add(bool err, std::string line);
  std::string dump(bool err, size_t last = 100) const;

 private:
  mutable std::mutex mu_;
  std::deque<std::string> out_, err_;
};

// Camera data-plane state (one per registered RTSP process).
class Camera {
 public:
  Camera(Worker& w, int index, std::string name, int ring_slots);
  const std::string& name() const { return name_; }
  int index() const { return index_; }
  // WorkerOptions::backpressure: wait (bounded) until the worker took this camera's queued job
  void wait_reconstruction();

  // --- control (atomics; replaces Redis control keys) ---
  std::atomic<i64> last_query_ms{0};   // 0 = never queried ("no last_query" in the hash)
  std::atomic<bool> keyframe_only{false};
  std::atomic<bool> proxy_rtmp{false};
  std::atomic<i64> idle_cutoff_ms{10000};  // rtsp_to_rtmp.py:144-145

  // --- ingest entry point (called from the camera's network thread) ---
  // Returns true if the AU triggered a decode submission.
  bool on_access_unit(const AuPtr& au);
  // Force-decode (used by bench/tests): parse au and submit regardless of query state.
  void decode_now(const AuPtr& au);
  // Same as decode_now but hands the job back (bench driver batches jobs itself).
  bool make_job(const AuPtr& au, DecodeJob& job);

  // --- stats ---
  // decoded = frames published to the ring; pictures = pictures reconstructed (general path: a
  // picture can be reconstructed in one job and output by a later one)
  std::atomic<u64> packets{0}, decoded{0}, skipped{0}, errors{0}, bytes_in{0}, pictures{0}, shed{0};
  // packet arrival -> frame published (ms) histogram, upper bounds kLatBucketsMs (+inf last)
  static constexpr int kLatBuckets = 12;
  static constexpr double kLatBucketsMs[kLatBuckets - 1] = {1, 2, 5, 10, 20, 35, 50, 100, 250, 500, 1000};
  std::atomic<u64> lat_hist[kLatBuckets] = {};
  std::atomic<u64> lat_sum_ms{0};
  std::atomic<i64> last_packet_ms{0};
  LogRing logs;

  // The ring is replaced on a resolution change: readers hold their own reference.
  std::shared_ptr<FrameRing> ring() const { return std::atomic_load(&ring_); }
  void set_ring(std::shared_ptr<FrameRing> r) { std::atomic_store(&ring_, std::move(r)); }
  StreamParser& parser() { return parser_; }
  // true once the stream left the I_PCM / P_Skip fast path (general H.264 / H.265 decoder in use)
  bool general_decoder() const { return full_ || hevc_full_; }
  // decoder backend serving this camera: "vcn" (rocDecode) or "native" (CPU parse + gfx950)
  const char* backend() const { return use_vcn_ ? "vcn" : "native"; }
  std::mutex& gop_mutex() { return mu_; }
  std::vector<AuPtr> gop_snapshot();   // current GOP packets (for RTMP flush / archive)

  // worker-owned GPU state
  struct Surface {
    int wmbs = 0, hmbs = 0;
    int slots = 1;                 // DPB surfaces (general H.264 path); slot k at y + k * bytes
    int bps = 1;                   // bytes per sample: 2 = u16 samples (HEVC Main10, H.264 High 10)
    int bd = 8;                    // sample bit depth
    int cf = 1;                    // chroma format: 2 = 4:2:2 (NV16: full-height chroma plane)
    u8* y = nullptr;
    u8* uv = nullptr;
    // bps 2 or 4:2:2: the 8-bit NV12 copy of the picture being published (what the BGR
    // conversion and the letterbox read; written by gpu::launch_narrow)
    u8* y8 = nullptr;
    u8* uv8 = nullptr;
    // H.265 intra edge exchange (gpu::hevc_xg_words of the coded picture) and its round epoch
    u64* hevc_xg = nullptr;
    size_t hevc_xg_words = 0;
    u32 hevc_epoch = 0;
    size_t slot_y() const { return size_t(wmbs) * 16 * hmbs * 16 * size_t(bps); }
    size_t slot_uv() const { return cf == 2 ? slot_y() : slot_y() / 2; }
    bool narrowed() const { return bps == 2 || cf == 2; }  // published through y8 / uv8
    std::vector<HostSurface> host;  // CPU backend: one per slot
    std::vector<HostSurface> fields;  // CPU backend, H.264 field pictures: one per field slot
  } surface;
  std::shared_ptr<FrameRing> ring_;  // written by the worker via set_ring(); read via ring()
  // DPB slot and pts of the newest published picture (Worker::read_surface; -1: none / a field
  // pair). Worker thread, under the worker's camera lock.
  int out_surface_slot = -1;
  i64 out_surface_pts = 0;
  int ring_slots_cfg;

 private:
  friend class Worker;
  friend bool stale_output(Camera& c, const DecodeJob& j, bool check);
  bool build_job(DecodeJob& job, size_t from, size_t to, bool refresh);
  bool build_vcn_job(DecodeJob& job, size_t from, size_t to);
  Worker& w_;
  int index_;
  std::string name_;
  std::mutex mu_;
  std::vector<AuPtr> gop_;
  size_t decoded_upto_ = 0;  // gop_[0, decoded_upto_) are reconstructed on the surface
  bool broken_ = false;      // worker thread: a published frame failed its check; drop until IDR
  // Worker thread: DecodeJob::dropped / poisoned_cra of recent jobs. A dropped picture leaves the
  // reorder buffer at most once (its entry is erased when it does); entries also expire after
  // kStaleJobs of the camera's jobs, so a pts that repeats later (looped source, reconnect, wrap)
  // is not suppressed for good.
  static constexpr u64 kStaleJobs = 64;
  struct StaleOut {
    int slot;
    i64 pts;
    u64 until;
  };
  std::vector<StaleOut> stale_;
  std::vector<std::pair<i64, u64>> bad_cra_;  // (CRA tag, expiry)
  u64 jobs_seen_ = 0;
  i64 keyframes_ = 0;
  StreamParser parser_;
  avc::Decoder avc_;
  bool full_ = false;
  // General H.265 path: the CPU parses into reconstruction records (hevc_dec.h records mode);
  // the worker reconstructs them on the GPU (gpu_hevc.hip) or with the CPU mirror.
  bool hevc_full_ = false;
  hevc::Decoder hevc_;
  // VCN backend: one rocDecode session per camera, created on the first keyframe
  bool use_vcn_ = false;
  std::unique_ptr<vcn::Session> vcn_;
  u64 fault_after_ = 0;  // VEP_FAULT_CAMERA: crash on this access unit (0 = never)
};

struct WorkerOptions {
  int device = 0;             // -1 = CPU backend
  int letterbox_size = 0;     // 0 = no consumer batch
  int letterbox_format = 0;   // gpu::LetterboxFormat (BGR HWC or NV12)
  int chw_dtype = 0;          // gpu::ChwDtype for the normalised CHW consumer tensor
  float mean[3] = {0.f, 0.f, 0.f};
  float std[3] = {1.f, 1.f, 1.f};
  int max_cameras = 256;
  int pack_threads = 4;       // host threads packing MB payloads into pinned staging
  bool direct_reads = true;   // decode kernel reads slice bytes from host memory (else gather)
  // Independent GPU pipelines ("lanes"): camera c always runs on lane c % lanes, each lane with
  // its own stream and staging. A keyframe's long intra wavefront then delays only its lane's
  // cameras instead of the whole tick. 0 = VEP_LANES or the default.
  int lanes = 0;
  // Batches in flight per lane (staging buffers): launch_async blocks only when its lane still
  // runs the batch from `stages` launches ago. 0 = VEP_STAGES or the default.
  int stages = 0;
  // Batches a lane's launcher thread may have queued behind its in-flight ones (several lanes):
  // how far the other lanes can run ahead of one held up by a slow batch. 0 = VEP_LANE_QUEUE or
  // the default.
  int queue = 0;
  bool lane_threads = false;  // one launcher thread per lane (also VEP_LANE_THREADS=1)
  // Decoder backend: kDecoderNative (CPU parse + gfx950 reconstruction), kDecoderVcn (rocDecode
  // on the video core; fails when librocdecode is missing) or kDecoderAuto (VCN when present).
  int decoder = 0;
  // Keyframe-only coalescing: while every pending job is a keyframe-only camera's picture, the
  // worker waits up to this long (from the first one) for more before launching, so one
  // latency-bound intra + deblocking wavefront launch serves several pictures. Such cameras
  // show one frame per GOP, so the wait is invisible to their clients. -1 = VEP_KF_WINDOW_US or
  // the default; 0 = off.
  int kf_window_us = -1;
  // CPU backend only (sanitizer runs): serve through the pinned serve-buffer pool with chunked
  // copies, as the GPU path's D2H does, so its concurrency (acquire_serve / release_serve, chunk
  // hand-off) runs under ThreadSanitizer without a GPU. Also VEP_MOCK_SERVE=1.
  bool mock_serve = false;
  // CPU backend: the reference's per-frame copy chain after the BGR24 conversion
  // (read_image.py:97 `img.tobytes()` + :119 `SerializeToString()`): each published frame is
  // copied into a bytes buffer and then into a serialized VideoFrame message. Used by the bench's
  // reference-equivalent CPU run (bench.py), off otherwise.
  bool ref_copies = false;
  // Lossless ingest also waits for reconstruction: a camera's parse strand waits (up to 2 s)
  // until the worker has taken the camera's queued job before parsing its next access unit, so a
  // reconstruction-bound backend back-pressures the socket instead of parsing pictures a GOP
  // catch-up later drops (the reference decodes only what it shows). Used by the bench's
  // reference-equivalent CPU run.
  bool backpressure = false;
  // Host domain (hostplan.h): the CPUs this worker's host threads run on and its ingest pool
  // sizes. parse_threads 0 = none: the worker's threads are not pinned and its cameras share the
  // process-wide ingest services.
  HostDomain domain;
};
enum DecoderBackend : int { kDecoderNative = 0, kDecoderVcn = 1, kDecoderAuto = 2 };

class Worker {
 public:
  explicit Worker(const WorkerOptions& o);
  ~Worker();
  Device& device() { return dev_; }
  const WorkerOptions& options() const { return opt_; }
  const HostDomain& host_domain() const { return opt_.domain; }
  // Ingest services (socket loops, parse strands, fan-out) of this worker's host domain, created
  // with its first IngestSession and released with the last; the process-wide services when the
  // worker has no host domain.
  std::shared_ptr<IngestServices> ingest_services();
  // Parse strands of the live ingest services (0 when none are running).
  int ingest_parse_threads();

  int add_camera(const std::string& name, int ring_slots);
  void remove_camera(int idx);
  // Shared ownership: a reader (gRPC thread) keeps the camera alive across remove_camera().
  std::shared_ptr<Camera> camera(int idx);
  std::shared_ptr<Camera> find(const std::string& name);
  int num_cameras() const;

  // Live mode: a background thread drains submitted jobs in batches.
  void start();
  void stop();
  void submit(DecodeJob&& job);  // merges with a not-yet-launched job of the same camera

  // Synchronous batched decode (bench / tests). Jobs are consumed.
  void run_batch(std::vector<DecodeJob>& jobs);
  // Asynchronous pipeline (per lane `stages()` batches in flight, one staging buffer each; with
  // one lane the H2D runs on a copy stream overlapping the previous batch's kernels).
  // launch_async returns once the batch is enqueued; its frames are published by a later
  // launch_async (when its staging buffer is reused) or by complete_all().
  void launch_async(std::vector<DecodeJob>& jobs);
  void complete_all();
  // Wait until every submitted job is published.
  void flush();

  // Serving: copy the newest frame with seq > after into dst (host). Returns false if none.
  // dst_pinned: dst is page-locked (register_host) -> one DMA straight into it, no staging.
  bool read_latest(int cam, i64 after, FrameMeta* meta, u8* dst, size_t cap);
  bool read_latest(FrameRing& ring, i64 after, FrameMeta* meta, u8* dst, size_t cap, bool dst_pinned = false);
  // Several rings' newest frames at once (the frame bus pump): every copy into page-locked
  // destinations is queued on the serving stream before one wait; others go one by one.
  struct ReadReq {
    FrameRing* ring = nullptr;
    i64 after = 0;
    u8* dst = nullptr;
    size_t cap = 0;
    bool pinned = false;
    FrameMeta meta;  // out
    bool ok = false; // out
  };
  void read_latest_many(std::vector<ReadReq>& reqs);
  // Called after every frame a camera commits to its ring: (camera index, sequence). Runs on the
  // publishing thread with the camera table locked: must be cheap and must not call back in.
  void set_publish_hook(std::function<void(int, i64)> f);
  // Page-lock caller memory (e.g. a shared-memory segment another process maps) for direct
  // D2H. False on the CPU backend or when the driver refuses the range.
  bool register_host(void* p, size_t n);
  void unregister_host(void* p);

  // Consumer batch (letterbox): device pointers of [max_cameras, S, S, 3] u8 and CHW tensor.
  // Point the consumer batch at caller-owned device buffers (e.g. torch tensors that feed an
  // RCCL all-gather); row r belongs to camera index r. Takes effect from the next batch.
  void set_consumer_buffers(u8* hwc, void* chw, int rows);
  u8* consumer_hwc() const { return cons_hwc_; }
  // Consistent copy of consumer rows [0, rows) into dst (device memory on the GPU): ordered after
  // every letterbox write already enqueued on any lane and before any later one, without a host
  // wait. `stream` is the caller's (e.g. torch's current stream, so a collective enqueued next on
  // it reads whole rows: no row is half one frame, half the next); 0 = wait on the host. Reading
  // the live rows instead races the lanes' next letterbox writes. Returns the bytes copied.
  size_t snapshot_consumer(void* dst, size_t cap, int rows, hipStream_t stream);
  u64 snapshots() const { return snap_gen_.load(); }
  void* consumer_chw() const { return cons_chw_; }
  hipStream_t compute_stream() const { return stream_; }  // lane 0
  int lanes() const { return int(lanes_.size()); }
  // batches in flight per lane: a launch publishes the batch from this many launches ago
  int stages() const { return stages_; }
  // batches launch_async may have handed over but not yet published, per lane
  int inflight() const { return stages_ + (threaded_ ? queue_ : 0); }
  // Every launch_async() with work gets a sequence number (launch_seq() after it returns).
  // With several lanes each lane has its own launcher thread, so a batch's frames are published
  // asynchronously: wait_published(s) blocks until every batch with sequence <= s is published.
  u64 launch_seq() const { return launch_seq_.load(); }
  void wait_published(u64 seq);
  u64 batches() const { return batches_.load(); }
  // slice bytes the GPU read in place from pinned AU blocks vs. staged by a host memcpy
  u64 bytes_inplace() const { return pinned_bytes_inplace_.load(); }
  u64 records_gathered() const { return records_gathered_.load(); }  // record bytes the GPU pulled
  int kf_window_us() const { return kf_window_us_; }
  u64 bytes_staged() const { return pinned_bytes_staged_.load(); }
  // frames committed to camera rings (what a client can read) / frames a batch produced but the
  // worker did not publish (GPU check failure, wavefront timeout, camera waiting for a keyframe
  // after an error, camera removed)
  u64 frames() const { return frames_.load(); }
  u64 dropped() const { return dropped_.load(); }
  // outputs not published because their reconstruction was shed with a merged backlog (load
  // shedding at a keyframe, merge_job) or predicts from such a picture (RASL of a shed CRA)
  u64 shed() const { return shed_.load(); }
  u64 merged() const { return merged_.load(); }  // batches merged into an earlier one (lane launchers)
  // Lane launcher threads leave queued batches queued while held (tests: a deterministic queue
  // for merge_queued; a drain still launches them).
  void hold_lanes(bool hold);
  u64 pictures() const { return pictures_.load(); }  // pictures reconstructed
  // GPU time of the batches (first event to last, per lane; the busiest lane's total)
  double gpu_ms_total() const;
  // clock64() phase accumulators of the wavefront kernels (VEP_AVC_PROF=1; gpu::kAvcProfSlots)
  std::vector<u64> avc_profile();

 private:
  struct Stage {  // one pinned + device staging pair and the batch that uses it
    u8* h = nullptr;
    u8* d = nullptr;
    size_t cap = 0;
    hipEvent_t copied = nullptr, e0 = nullptr, e1 = nullptr;
    std::vector<DecodeJob> jobs;
    std::vector<int> slots;
    u64 seq = 0;               // launch sequence of the batch (merged batches: the first ...
    u64 seq_last = 0;          // ... to the last, consecutive in the lane's `unpublished`)
    u8* cons_hwc = nullptr;    // consumer batch at launch time (set_consumer_buffers may move on)
    void* cons_chw = nullptr;
    int cons_rows = 0;
    bool active = false;
    u32* err = nullptr;        // pinned per-job check flags (written by the kernel)
    const u32* err_dev = nullptr;
    size_t err_cap = 0;
  };
  void loop();
  void ensure_surface(Camera& c, const PictureInfo& pi, int slots, int bd = 8, bool weave = false, int cf = 1);
  struct Batch {
    std::vector<DecodeJob> jobs;
    std::vector<int> slots;
    u64 seq = 0, seq_last = 0;
    u8* cons_hwc = nullptr;
    void* cons_chw = nullptr;
    int cons_rows = 0;
  };
  struct Lane {
    hipStream_t stream = nullptr;  // lane 0 uses Worker::stream_
    hipStream_t copy = nullptr;    // H2D of the next batch's MB data while this one decodes
    std::vector<Stage> stage;      // ring of staging buffers (Worker::stages() deep)
    int next = 0;                  // the stage reused next (the oldest in-flight batch)
    std::atomic<double> gpu_ms{0}; // cumulative batch time on this lane
    // launcher thread (several lanes): batches handed over by launch_async
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Batch> q;
    bool busy = false, drain = false, stop = false;
    std::deque<u64> unpublished;   // sequences given to this lane, not yet published (pub_mu_)
    u64 snap_seen = 0;             // consumer snapshots this lane's stream already waits for
    hipEvent_t snap_mark = nullptr;  // recorded by snapshot_consumer: the lane's enqueued work
  };
  void prepare(std::vector<DecodeJob>& jobs, std::vector<int>& slots);
  void launch_gpu(Lane& ln, Stage& st);
  void lane_loop(Lane& ln);
  void merge_queued(Lane& ln, Batch& b);
  void launch_on(Lane& ln, Batch&& b);  // reuse the lane's oldest stage for batch b
  void drain_lanes();
  void run_cpu(std::vector<DecodeJob>& jobs, std::vector<int>& slots, std::vector<u32>& err);
  // err[i] != 0: job i failed its speculative-header check (dropped, camera waits for the
  // next keyframe)
  void publish(std::vector<DecodeJob>& jobs, std::vector<int>& slots, const u32* err = nullptr);
  void complete(Lane& ln, Stage& st);
  void complete_locked();
  WorkerOptions opt_;
  Device dev_;
  hipStream_t stream_ = nullptr, copy_stream_ = nullptr, serve_stream_ = nullptr;
  mutable std::mutex cams_mu_;
  std::vector<std::shared_ptr<Camera>> cams_;
  std::vector<std::unique_ptr<Lane>> lanes_;
  int stages_ = 2;
  bool threaded_ = false;        // one launcher thread per lane
  int queue_ = 0;                // lane queue depth (threaded)
  std::atomic<bool> hold_{false};
  int merge_jobs_ = 0;           // lane launcher: merge queued batches up to this many jobs (0: off)
  std::atomic<u64> launch_seq_{0};
  std::mutex pub_mu_;
  std::condition_variable pub_cv_;
  std::exception_ptr lane_err_;  // first error of a lane thread, rethrown to the launcher
  std::unique_ptr<ThreadPool> pack_pool_;
  // CPU backend: reconstruction + conversion of a batch's cameras in parallel (the reference runs
  // one decoder per camera container); the host domain's CPU share threads
  std::unique_ptr<ThreadPool> cpu_pool_;
  void run_cpu_job(std::vector<DecodeJob>& jobs, std::vector<int>& slots, std::vector<u32>& err, size_t i);

 public:
  // host-side launch path timers (µs, cumulative): where a batch's CPU time goes (summed over
  // lane threads)
  struct Timers_ {
    double prepare = 0, index = 0, copy = 0, enqueue = 0, wait = 0;
  };
  using Timers = Timers_;
  Timers timers;

 private:
  void add_time(double Timers_::*f, double us);
  // Serving: a pool of pinned host buffers, one per in-flight read_latest(), so concurrent
  // requests DMA in parallel instead of queueing on one buffer. Each read streams the slot in
  // kServeChunks pieces: the host copy of chunk k overlaps the DMA of chunk k+1.
  static constexpr int kServeBufs = 8;
  static constexpr int kServeChunks = 4;
  struct ServeBuf {
    u8* h = nullptr;
    size_t cap = 0;
    hipEvent_t ev[kServeChunks] = {};
  };
  ServeBuf* acquire_serve(size_t n);
  void release_serve(ServeBuf* b);
  std::mutex serve_mu_;
  std::condition_variable serve_cv_;
  std::vector<std::unique_ptr<ServeBuf>> serve_all_;
  std::vector<ServeBuf*> serve_free_;
  u8* cons_hwc_ = nullptr;
  void* cons_chw_ = nullptr;
  // consumer snapshots: exclusive while a snapshot is enqueued, shared while a lane enqueues a
  // batch (its letterbox writes must come after the last snapshot's copy)
  std::shared_mutex cons_gate_;
  hipEvent_t snap_ev_ = nullptr;
  std::atomic<u64> snap_gen_{0};
  bool owns_cons_ = true;
  int cons_rows_ = 0;
  // live queue
  std::mutex q_mu_;
  std::condition_variable q_cv_, idle_cv_, taken_cv_;
  std::vector<DecodeJob> pending_;
  int kf_window_us_ = 0;
  // H.265 intra transform blocks: 0 = one launch per dependency level; k > 0 = one queue launch
  // per window of k consecutive levels (kAllLevels: the whole round in one launch)
  int hevc_tu_window_ = 0;
  u32 hevc_tu_nap_ = 16;  // HevcDesc::nap_max (VEP_HEVC_TU_NAP)
  // lanes wait for a stage's batch by polling its event with sleeps (VEP_SPIN_WAIT=1:
  // hipEventSynchronize, which spins a core in the HSA runtime)
  bool polite_wait_ = true;
  bool mock_serve_ = false;  // WorkerOptions::mock_serve

 public:
  u64 ref_copy_bytes() const { return ref_copy_bytes_.load(); }  // WorkerOptions::ref_copies output
  // until no queued (not yet taken) job of camera `cam` or timeout_ms passed
  void wait_camera_taken(int cam, int timeout_ms);
  // Debug / test readback of the DPB surface holding camera `cam`'s newest published picture, at
  // its full sample depth (u16 planes above 8 bits; NV16 chroma for 4:2:2) and coded size: what
  // the reconstruction wrote before the 8-bit narrowing for BGR24. False when none (or a field
  // pair). Call with the camera idle (after decode_now / flush): later jobs reuse the slot.
  bool read_surface(int cam, HostSurface& out, i64* pts);

 private:
  std::atomic<u64> ref_copy_bytes_{0};
  bool running_ = false, stop_ = false, busy_ = false;
  std::thread th_;
  std::mutex svc_mu_;
  std::weak_ptr<IngestServices> svc_;  // ingest_services()
  std::mutex launch_mu_;
  std::shared_ptr<std::function<void(int, i64)>> publish_hook_;  // (atomic_load / atomic_store)
  std::atomic<u64> batches_{0}, frames_{0}, dropped_{0}, pictures_{0}, shed_{0}, merged_{0};
  std::atomic<u64> pinned_bytes_inplace_{0}, pinned_bytes_staged_{0}, records_gathered_{0};
  std::mutex timers_mu_;
  bool direct_reads_ = false;
  u64* avc_prof_ = nullptr;
  int dbk_packed_ = 1;  // VEP_DBK_PACKED=0: the deblocking filter's byte-wise vertical edges (A/B)

 public:
  bool direct_reads() const { return direct_reads_; }
  // cameras decode through rocDecode / VCN (WorkerOptions::decoder)
  bool vcn() const { return vcn_; }

 private:
  bool vcn_ = false;
};

// Protobuf wire encoding of chrys.cloud.videostreaming.v1beta1.VideoFrame
// (field numbers from proto/video_streaming.proto). `data` bytes are supplied separately so
// the payload can be DMA'd straight into the output buffer: returns (prefix, suffix).
std::pair<std::string, std::string> encode_video_frame(const FrameMeta& m, size_t data_len,
                                                       const std::string& device_id);
// Upper bound of the suffix (fields after `data`) encode_video_frame produces for device_id.
inline size_t video_frame_suffix_max(const std::string& device_id) {
  return 7 * 11 + 2 * 2 + 3 + 9 + 48 + 12 + device_id.size();
}

}  // namespace vep
