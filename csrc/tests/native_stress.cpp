// Multi-threaded stress driver for the native data plane, built under ThreadSanitizer by
// `make tsan` (host code only: `-Xarch_host -fsanitize=thread`; the CPU backend runs, so no GPU
// is needed). Exercises every cross-thread hand-off of the runtime:
//   * live Worker (device -1): producer threads feeding cameras (on_access_unit + lazy-decode
//     control atomics) while reader threads poll rings, wait for frames and encode VideoFrames;
//   * ring replacement on a resolution change while readers hold the old ring;
//   * remove_camera while readers still hold the camera;
//   * RTSP server with concurrent clients; IngestSession supervisor start/stop against it.
//   * the general H.264 decoder (Baseline CAVLC and High CABAC IBBP streams) under concurrent
//     producers and readers, with GOP catch-up merges and keyframe-only toggling;
//   * the replay bench driver: parse pool threads + quiesce + step/drain (launch_async,
//     wait_published, complete_all) against readers;
//   * live ingest of a compressed High-profile camera with RTMP pass-through and the archiver;
//   * the frame bus: a pump serving readers in other threads while producers publish, cameras
//     come and go and the serve-buffer pool (mock serve: the GPU path's pool and chunked
//     copies, memcpy for the DMA) is hit by direct readers and consumer snapshots at once;
//   * the fan-out pool: several H.265 decoders parsing multi-slice pictures in parallel at once;
//   * the native gRPC endpoint under hostile HTTP/2 clients (csrc/tests/rpc_stress.cpp).
// Reference: SURVEY.md §5 "Race detection / sanitizers" (the reference had none and real races:
// read_image.py:48,71-74 vs rtsp_to_rtmp.py:147-151; grpc_api.go:181-184).
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "../vep/bench_driver.h"
#include "../vep/bus.h"
#include "../vep/hevc_dec.h"
#include "../vep/ingest.h"
#include "../vep/runtime.h"
#include "../vep/synth.h"

using namespace vep;

#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

// Waits until done(); gives up only when progress() has not changed for stall_ms. A sanitizer
// build runs many times slower than a release one, so no wall-clock budget: a live pipeline that
// keeps making progress is waited for, a stuck one fails.
template <class Done, class Progress, class Tick>
static bool wait_progress(Done done, Progress progress, Tick tick, int stall_ms = 60000) {
  unsigned long long last = progress();
  auto since = std::chrono::steady_clock::now();
  while (!done()) {
    tick();
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const unsigned long long p = progress();
    if (p != last) {
      last = p;
      since = std::chrono::steady_clock::now();
    } else if (std::chrono::steady_clock::now() - since > std::chrono::milliseconds(stall_ms)) {
      return false;
    }
  }
  return true;
}

static void live_worker_stress() {
  WorkerOptions o;
  o.device = -1;
  o.letterbox_size = 64;
  o.max_cameras = 8;
  Worker w(o);
  w.start();
  const int ncam = 4;
  std::vector<int> cams;
  for (int i = 0; i < ncam; ++i) cams.push_back(w.add_camera("c" + std::to_string(i), 3));
  std::atomic<bool> stop{false};
  std::atomic<u64> served{0};
  std::vector<std::thread> th;
  for (int i = 0; i < ncam; ++i) {
    th.emplace_back([&, i] {
      SynthConfig c;
      c.width = (i == 0) ? 96 : 160;
      c.height = (i == 0) ? 64 : 96;
      c.gop = 5;
      c.seed = u64(i + 1);
      c.codec = (i & 1) ? Codec::kH265 : Codec::kH264;
      SynthH264 enc(c);
      auto cam = w.camera(cams[size_t(i)]);
      for (int f = 0; f < 120; ++f) {
        if (i == 0 && f == 60) {  // resolution change mid-stream: the ring is replaced
          c.width = 128;
          c.height = 80;
          enc = SynthH264(c);
        }
        cam->last_query_ms.store(now_ms());
        cam->keyframe_only.store(f % 40 > 30);
        cam->on_access_unit(enc.next());
        if (f % 7 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
      }
    });
  }
  for (int r = 0; r < 3; ++r) {
    th.emplace_back([&, r] {
      std::vector<u8> buf(size_t(160) * 96 * 3);
      i64 cursor[8] = {};
      while (!stop.load()) {
        for (int i = 0; i < ncam; ++i) {
          auto cam = w.camera(cams[size_t(i)]);
          if (!cam) continue;
          auto ring = cam->ring();
          if (!ring) continue;
          if (r == 0) {
            ring->wait_newer(cursor[i], 2);
          }
          FrameMeta m;
          if (ring->slot_bytes() <= buf.size() &&
              w.read_latest(*ring, cursor[i], &m, buf.data(), buf.size())) {
            CHECK(m.seq > cursor[i]);
            cursor[i] = m.seq;
            auto enc = encode_video_frame(m, ring->slot_bytes(), cam->name());
            CHECK(!enc.first.empty());
            served.fetch_add(1);
          }
        }
      }
    });
  }
  for (int i = 0; i < ncam; ++i) th[size_t(i)].join();
  w.flush();
  stop.store(true);
  for (size_t i = ncam; i < th.size(); ++i) th[i].join();
  for (int i = 0; i < ncam; ++i) CHECK(w.camera(cams[size_t(i)])->decoded.load() > 0);
  // remove a camera while a reader still holds it
  auto held = w.camera(cams[1]);
  w.remove_camera(cams[1]);
  CHECK(held->name() == "c1" && !w.camera(cams[1]));
  w.stop();
  std::printf("live worker: served %llu frames\n", (unsigned long long)served.load());
}

static void rtsp_stress() {
  net::RtspServer srv("127.0.0.1", 0);
  net::ServedStream s;
  s.cfg.width = 128;
  s.cfg.height = 96;
  s.cfg.gop = 6;
  s.realtime = false;
  s.cached_frames = 12;
  srv.add_stream("/a", s);
  s.cfg.codec = Codec::kH265;
  srv.add_stream("/b", s);
  srv.start();
  std::vector<std::thread> th;
  std::atomic<int> got{0};
  for (int k = 0; k < 4; ++k) {
    th.emplace_back([&, k] {
      net::RtspClient c("rtsp://127.0.0.1:" + std::to_string(srv.port()) + ((k & 1) ? "/b" : "/a"));
      c.open();
      std::atomic<bool> stop{false};
      int n = 0;
      c.run([&](const AuPtr&) { if (++n >= 30) stop.store(true); }, stop);
      got.fetch_add(n);
    });
  }
  for (auto& t : th) t.join();
  CHECK(got.load() >= 120);

  // supervisor against the farm, with live decode, RTMP pass-through and per-GOP archive
  mux::RtmpSink sink("127.0.0.1", 0);
  sink.start();
  WorkerOptions o;
  o.device = -1;
  Worker w(o);
  w.start();
  int cam = w.add_camera("ingest", 2);
  w.camera(cam)->last_query_ms.store(now_ms());
  IngestConfig ic;
  ic.name = "ingest";
  ic.rtsp_url = "rtsp://127.0.0.1:" + std::to_string(srv.port()) + "/b";
  ic.rtmp_url = "rtmp://127.0.0.1:" + std::to_string(sink.port()) + "/live/stress";
  ic.disk_path = "/tmp/vep_native_stress";
  w.camera(cam)->proxy_rtmp.store(true);
  auto arch = std::make_shared<mux::Archiver>();
  IngestSession sess(w, cam, ic, arch);
  sess.start();
  // the RTMP sender connects and sends on its own thread: also wait for its first messages
  CHECK(wait_progress(
      [&] { return w.camera(cam)->decoded.load() >= 5 && sess.state().rtmp_messages >= 3; },
      [&] { return w.camera(cam)->packets.load() + w.camera(cam)->decoded.load() + sess.state().rtmp_messages; },
      [&] { w.camera(cam)->last_query_ms.store(now_ms()); }));
  sess.stop();
  w.flush();
  CHECK(w.camera(cam)->decoded.load() >= 5);
  arch->flush();
  CHECK(sink.video_messages() > 0);
  w.stop();
  sink.stop();
  srv.stop();
  std::printf("rtsp: %d AUs over 4 clients; ingest decoded %llu\n", got.load(),
              (unsigned long long)w.camera(cam)->decoded.load());
}

static SynthConfig compressed_cfg(const char* profile, u64 seed, int w, int h) {
  SynthConfig c;
  c.width = w;
  c.height = h;
  c.gop = 8;
  c.seed = seed;
  c.compressed = true;
  c.profile = profile;
  c.bframes = 2;
  c.coverage = seed % 2 == 0;  // every MB / sub-MB type on half the cameras
  return c;
}

static void general_decoder_stress() {
  WorkerOptions o;
  o.device = -1;
  o.letterbox_size = 64;
  o.max_cameras = 8;
  Worker w(o);
  w.start();
  const int ncam = 6;  // 2 High, 2 Baseline, 2 H.265 Main (records path + CPU mirror)
  std::vector<int> cams;
  for (int i = 0; i < ncam; ++i) cams.push_back(w.add_camera("g" + std::to_string(i), 3));
  std::atomic<bool> stop{false};
  std::atomic<u64> served{0};
  std::vector<std::thread> th;
  for (int i = 0; i < ncam; ++i) {
    th.emplace_back([&, i] {
      SynthConfig cfg = compressed_cfg(i < 2 ? "high" : "baseline", u64(i + 1), 96 + 16 * (i % 4), 64);
      if (i >= 4) cfg.codec = Codec::kH265;
      SynthH264 enc(cfg);
      auto cam = w.camera(cams[size_t(i)]);
      for (int f = 0; f < 48; ++f) {
        cam->last_query_ms.store(now_ms());
        cam->keyframe_only.store(i == 3 && f % 24 > 16);
        cam->on_access_unit(enc.next());
        if (f % 5 == 0) std::this_thread::sleep_for(std::chrono::microseconds(300));  // catch-up merges
      }
    });
  }
  for (int r = 0; r < 2; ++r) {
    th.emplace_back([&] {
      std::vector<u8> buf(size_t(160) * 64 * 3);
      i64 cursor[8] = {};

      while (!stop.load()) {
        for (int i = 0; i < ncam; ++i) {
          auto cam = w.camera(cams[size_t(i)]);
          auto ring = cam ? cam->ring() : nullptr;
          if (!ring) continue;
          FrameMeta m;
          if (ring->slot_bytes() <= buf.size() && w.read_latest(*ring, cursor[i], &m, buf.data(), buf.size())) {
            CHECK(m.seq > cursor[i]);
            cursor[i] = m.seq;
            served.fetch_add(1);
          }
        }
      }
    });
  }
  for (int i = 0; i < ncam; ++i) th[size_t(i)].join();
  w.flush();
  stop.store(true);
  for (size_t i = ncam; i < th.size(); ++i) th[i].join();
  for (int i = 0; i < ncam; ++i) {
    auto c = w.camera(cams[size_t(i)]);
    if (c->decoded.load() == 0 || c->errors.load() != 0)
      std::printf("camera %d: decoded %llu errors %llu\n%s", i, (unsigned long long)c->decoded.load(),
                  (unsigned long long)c->errors.load(), c->logs.dump(true).c_str());
    CHECK(c->decoded.load() > 0);
    CHECK(c->errors.load() == 0);
  }
  w.stop();
  std::printf("general decoder: served %llu frames, %llu pictures\n", (unsigned long long)served.load(),
              (unsigned long long)w.pictures());
}

static void replay_bench_stress() {
  WorkerOptions o;
  o.device = -1;
  o.letterbox_size = 32;
  o.max_cameras = 6;
  Worker w(o);
  SynthConfig c = compressed_cfg("high", 7, 96, 64);
  c.coverage = false;
  ReplayBench rb(w, 6, c, 16, 3, 2, "rb", 4);
  std::atomic<bool> stop{false};
  std::thread reader([&] {
    std::vector<u8> buf(size_t(96) * 64 * 3);
    i64 cursor = 0;
    while (!stop.load()) {
      auto cam = w.camera(rb.cameras()[0]);
      auto ring = cam ? cam->ring() : nullptr;
      FrameMeta m;
      if (ring && ring->slot_bytes() <= buf.size() && w.read_latest(*ring, cursor, &m, buf.data(), buf.size()))
        cursor = m.seq;
    }
  });
  for (int i = 0; i < 10; ++i) rb.step();
  rb.quiesce();
  const u64 f0 = w.frames();
  for (int i = 0; i < 30; ++i) rb.step();
  rb.drain();
  stop.store(true);
  reader.join();
  CHECK(rb.parse_failures() == 0 && w.dropped() == 0);
  CHECK(w.frames() - f0 >= 30 * 6 - 12);
  std::printf("replay bench: %llu frames published, %llu pictures\n", (unsigned long long)w.frames(),
              (unsigned long long)w.pictures());
}

static void compressed_ingest_stress() {
  net::RtspServer srv("127.0.0.1", 0);
  net::ServedStream s;
  s.cfg = compressed_cfg("high", 11, 160, 96);
  s.cfg.coverage = false;
  s.realtime = false;
  s.cached_frames = 16;
  srv.add_stream("/hi", s);
  srv.start();
  mux::RtmpSink sink("127.0.0.1", 0);
  sink.start();
  WorkerOptions o;
  o.device = -1;
  Worker w(o);
  w.start();
  int cam = w.add_camera("hi", 2);
  w.camera(cam)->last_query_ms.store(now_ms());
  w.camera(cam)->proxy_rtmp.store(true);
  IngestConfig ic;
  ic.name = "hi";
  ic.rtsp_url = "rtsp://127.0.0.1:" + std::to_string(srv.port()) + "/hi";
  ic.rtmp_url = "rtmp://127.0.0.1:" + std::to_string(sink.port()) + "/live/hi";
  ic.disk_path = "/tmp/vep_native_stress_hi";
  auto arch = std::make_shared<mux::Archiver>();
  IngestSession sess(w, cam, ic, arch);
  sess.start();
  CHECK(wait_progress(
      [&] { return w.camera(cam)->decoded.load() >= 20 && sess.state().rtmp_messages >= 3; },
      [&] { return w.camera(cam)->packets.load() + w.camera(cam)->decoded.load() + sess.state().rtmp_messages; },
      [&] { w.camera(cam)->last_query_ms.store(now_ms()); }));
  sess.stop();
  w.flush();
  CHECK(w.camera(cam)->decoded.load() >= 20 && w.camera(cam)->errors.load() == 0);
  arch->flush();
  CHECK(sink.video_messages() > 0);
  w.stop();
  sink.stop();
  srv.stop();
  std::printf("compressed ingest: decoded %llu\n", (unsigned long long)w.camera(cam)->decoded.load());
}

static void bus_stress() {
  WorkerOptions o;
  o.device = -1;
  o.letterbox_size = 32;
  o.max_cameras = 8;
  o.mock_serve = true;
  Worker w(o);
  w.start();
  bus::Owner owner("stress" + std::to_string(::getpid()), 0, 8);
  owner.attach(&w);
  const int ncam = 3;
  std::vector<int> cams;
  for (int i = 0; i < ncam; ++i) {
    cams.push_back(w.add_camera("b" + std::to_string(i), 3));
    owner.add(cams.back(), "b" + std::to_string(i));
  }
  std::atomic<bool> stop{false};
  std::atomic<u64> bus_frames{0}, direct{0}, snaps{0};
  std::vector<std::thread> th;
  for (int i = 0; i < ncam; ++i)
    th.emplace_back([&, i] {
      SynthConfig c;
      c.width = 128;
      c.height = 96;
      c.gop = 6;
      c.seed = u64(40 + i);
      SynthH264 enc(c);
      auto cam = w.camera(cams[size_t(i)]);
      for (int f = 0; f < 90; ++f) {
        cam->last_query_ms.store(now_ms());
        cam->on_access_unit(enc.next());
        std::this_thread::sleep_for(std::chrono::microseconds(300));
      }
    });
  for (int r = 0; r < 4; ++r)  // bus readers (the serving processes' side)
    th.emplace_back([&, r] {
      bus::Reader rd("stress" + std::to_string(::getpid()));
      std::vector<u8> buf;
      i64 cursor[ncam] = {};
      while (!stop.load()) {
        const int i = (r + int(bus_frames.load())) % ncam;
        bus::Reader::Ticket t;
        if (!rd.wait("b" + std::to_string(i), cursor[i], 20, r & 1, &t)) continue;
        buf.resize(t.cap);
        i64 seq = 0;
        const size_t len = rd.copy(t, buf.data(), buf.size(), &seq);
        if (!len) continue;
        CHECK(seq > cursor[size_t(i)] && len > size_t(128) * 96 * 3);
        cursor[size_t(i)] = seq;
        bus_frames.fetch_add(1);
      }
    });
  th.emplace_back([&] {  // direct readers through the serve-buffer pool
    std::vector<u8> buf(size_t(128) * 96 * 3);
    while (!stop.load())
      for (int i = 0; i < ncam; ++i) {
        auto cam = w.camera(cams[size_t(i)]);
        auto ring = cam ? cam->ring() : nullptr;
        FrameMeta m;
        if (ring && w.read_latest(*ring, 0, &m, buf.data(), buf.size())) direct.fetch_add(1);
      }
  });
  th.emplace_back([&] {  // consumer snapshots against the letterbox writes
    std::vector<u8> snap(size_t(ncam) * 32 * 32 * 3);
    while (!stop.load()) {
      w.snapshot_consumer(snap.data(), snap.size(), ncam, nullptr);
      snaps.fetch_add(1);
    }
  });
  for (int i = 0; i < ncam; ++i) th[size_t(i)].join();
  w.flush();
  owner.remove(cams[2]);  // a camera leaves while readers may wait on it
  int extra = w.add_camera("b3", 2);
  owner.add(extra, "b3");
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  stop.store(true);
  for (size_t i = ncam; i < th.size(); ++i) th[i].join();
  owner.stop();
  w.stop();
  CHECK(bus_frames.load() > 0 && direct.load() > 0 && snaps.load() > 0);
  std::printf("frame bus: %llu bus frames, %llu direct reads, %llu snapshots\n",
              (unsigned long long)bus_frames.load(), (unsigned long long)direct.load(),
              (unsigned long long)snaps.load());
}

// Parallel parse units of one picture on the shared fan-out pool, several decoders at once:
// H.265 slices, the tiles of one slice, wavefront rows (per-CTB done flags + per-row contexts)
// and H.264 slices (per-slice neighbour state and records shards).
static void slice_fanout_stress() {
  struct Stream {
    Codec codec;
    int slices, tile_cols, tile_rows;
    bool wpp;
  };
  const Stream streams[] = {{Codec::kH265, 4, 1, 1, false}, {Codec::kH265, 1, 3, 2, false},
                            {Codec::kH265, 2, 1, 1, true}, {Codec::kH264, 4, 1, 1, false}};
  std::atomic<u64> pictures{0};
  for (const Stream& st : streams) {
    SynthConfig c;
    c.width = 320;
    c.height = 192;
    c.gop = 8;
    c.codec = st.codec;
    c.compressed = true;
    c.profile = "high";
    c.slices = st.slices;
    c.tile_cols = st.tile_cols;
    c.tile_rows = st.tile_rows;
    c.wpp = st.wpp;
    c.bframes = 1;
    std::vector<AuPtr> aus;
    {
      SynthH264 enc(c);
      for (int i = 0; i < 12; ++i) aus.push_back(enc.next());
    }
    std::vector<std::thread> th;
    for (int d = 0; d < 3; ++d)
      th.emplace_back([&, d] {
        if (st.codec == Codec::kH264) {
          avc::Decoder dec;
          for (int loop = 0; loop < 3; ++loop) {
            for (const auto& au : aus) (void)dec.parse(*au, 0);
            (void)dec.flush_output();
            dec.reset_references();
            pictures.fetch_add(aus.size());
          }
          return;
        }
        hevc::Decoder dec;
        dec.set_gpu_mode(d != 0);  // records mode (shards merged) and CPU reconstruction
        for (int loop = 0; loop < 3; ++loop) {
          for (const auto& au : aus) dec.decode(*au, 0);
          (void)dec.flush();
          (void)dec.take_gpu_pictures();
          pictures.fetch_add(aus.size());
        }
      });
    for (auto& t : th) t.join();
  }
  std::printf("parallel slices / tiles / wavefront rows: %llu pictures\n", (unsigned long long)pictures.load());
}

void rpc_hostile_stress();  // rpc_stress.cpp

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IONBF, 0);  // progress is visible even if a run is cut short
  if (argc > 1 && std::string(argv[1]) == "rpc") {  // the endpoint part alone
    rpc_hostile_stress();
    std::printf("native_stress ok\n");
    return 0;
  }
  live_worker_stress();
  rtsp_stress();
  general_decoder_stress();
  replay_bench_stress();
  compressed_ingest_stress();
  bus_stress();
  slice_fanout_stress();
  rpc_hostile_stress();
  std::printf("native_stress ok\n");
  return 0;
}
