// Hostile-client stress of the native gRPC endpoint (csrc/vep/rpcsrv.cpp), linked into the
// sanitizer driver (`make asan` / `make tsan`, csrc/tests/native_stress.cpp; `native_stress rpc`
// runs this part alone). A live Worker (CPU backend) publishes frames of three cameras to the
// frame bus while, at once:
//   * legitimate raw HTTP/2 clients request VideoLatestImage frames and check status 0 + data;
//   * CONTINUATION floods, HPACK expansion bombs, oversized frames and bad control frames (each
//     must end its connection with GOAWAY before any large buffering);
//   * stream floods beyond SETTINGS_MAX_CONCURRENT_STREAMS (RST_STREAM REFUSED_STREAM);
//   * HEADERS + DATA + RST_STREAM loops (reset waiters are cancelled; too many resets per second
//     is GOAWAY ENHANCE_YOUR_CALM);
//   * clients with a tiny receive window that never open it, and clients that never read;
//   * a byte-level mutation fuzz of a valid session (flips, insertions, deletions, truncation).
// Pass: no sanitizer report, every legitimate request answered, the limits observed in the
// server's counters. Reference: the grpc-go server the reference relies on for all of this
// (server/main.go:142-153).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../vep/bus.h"
#include "../vep/rpcsrv.h"
#include "../vep/runtime.h"
#include "../vep/synth.h"

using namespace vep;

#define RCHECK(c)                                                                  \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "RCHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

namespace {

enum : u8 { DATA = 0, HEADERS = 1, PRIORITY = 2, RST = 3, SETTINGS = 4, PING = 6, GOAWAY = 7, WINUPD = 8, CONT = 9 };
constexpr u8 END_STREAM = 1, END_HEADERS = 4, PADDED = 8;
const char* kService = "/chrys.cloud.videostreaming.v1beta1.Image/";

std::string frame(u8 type, u8 flags, u32 sid, const std::string& p = std::string()) {
  const u32 n = u32(p.size());
  std::string h = {char(n >> 16), char(n >> 8), char(n), char(type), char(flags),
                   char((sid >> 24) & 0x7F), char(sid >> 16), char(sid >> 8), char(sid)};
  return h + p;
}

std::string be32s(u32 v) { return {char(v >> 24), char(v >> 16), char(v >> 8), char(v)}; }

std::string hp_int(u64 v, int prefix, u8 first) {
  const u32 mask = (1u << prefix) - 1;
  std::string s;
  if (v < mask) return std::string(1, char(first | u8(v)));
  s.push_back(char(first | mask));
  v -= mask;
  while (v >= 128) {
    s.push_back(char(0x80 | (v & 0x7F)));
    v >>= 7;
  }
  s.push_back(char(v));
  return s;
}

std::string hp_lit(const std::string& n, const std::string& v, bool index = false) {
  return std::string(1, char(index ? 0x40 : 0x00)) + hp_int(n.size(), 7, 0) + n + hp_int(v.size(), 7, 0) + v;
}

std::string request_block(const std::string& method = "VideoLatestImage") {
  return hp_lit(":method", "POST") + hp_lit(":scheme", "http") + hp_lit(":path", kService + method) +
         hp_lit(":authority", "x") + hp_lit("content-type", "application/grpc") + hp_lit("te", "trailers");
}

std::string frame_request(const std::string& dev) {
  const std::string body = std::string("\x12") + char(dev.size()) + dev;
  return std::string(1, '\0') + be32s(u32(body.size())) + body;
}

const std::string kPreface = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";

struct Client {
  int fd = -1;
  std::string buf;
  explicit Client(int port, int rcv_timeout_ms = 3000, u32 window = 0) {
    fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(u16(port));
    ::inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
    timeval tv{rcv_timeout_ms / 1000, (rcv_timeout_ms % 1000) * 1000};
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    int on = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &on, sizeof on);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
      ::close(fd);
      fd = -1;
      return;
    }
    std::string st;
    if (window) st = std::string{0, 4} + be32s(window);
    send(kPreface + frame(SETTINGS, 0, 0, st));
  }
  ~Client() {
    if (fd >= 0) ::close(fd);
  }
  bool send(const std::string& s) {
    size_t off = 0;
    while (fd >= 0 && off < s.size()) {
      const ssize_t w = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (w <= 0) return false;
      off += size_t(w);
    }
    return fd >= 0;
  }
  // next frame: type, flags, stream, payload; false on close / timeout
  bool read(u8& type, u8& flags, u32& sid, std::string& p) {
    for (;;) {
      if (buf.size() >= 9) {
        const size_t n = size_t(u8(buf[0])) << 16 | size_t(u8(buf[1])) << 8 | size_t(u8(buf[2]));
        if (buf.size() >= 9 + n) {
          type = u8(buf[3]);
          flags = u8(buf[4]);
          sid = (u32(u8(buf[5])) << 24 | u32(u8(buf[6])) << 16 | u32(u8(buf[7])) << 8 | u32(u8(buf[8]))) & 0x7FFFFFFF;
          p = buf.substr(9, n);
          buf.erase(0, 9 + n);
          return true;
        }
      }
      char tmp[1 << 16];
      const ssize_t r = fd >= 0 ? ::recv(fd, tmp, sizeof tmp, 0) : -1;
      if (r <= 0) return false;
      buf.append(tmp, size_t(r));
    }
  }
  // GOAWAY error code, or -1 when the connection ended / timed out without one
  long goaway() {
    u8 t, f;
    u32 s;
    std::string p;
    while (read(t, f, s, p))
      if (t == GOAWAY && p.size() >= 8) return long(u8(p[4])) << 24 | long(u8(p[5])) << 16 | long(u8(p[6])) << 8 | u8(p[7]);
    return -1;
  }
};

int trailers_status(const std::string& blk) {
  const size_t i = blk.find("grpc-status");
  if (i == std::string::npos || i + 12 >= blk.size()) return -1;
  const size_t n = u8(blk[i + 11]);
  return std::atoi(blk.substr(i + 12, n).c_str());
}

}  // namespace

void rpc_hostile_stress() {
  WorkerOptions o;
  o.device = -1;
  o.letterbox_size = 32;
  o.max_cameras = 8;
  o.mock_serve = true;
  Worker w(o);
  w.start();
  const std::string tag = "rpcs" + std::to_string(::getpid());
  bus::Owner owner(tag, 0, 8);
  owner.attach(&w);
  const int ncam = 3;
  std::vector<int> cams;
  for (int i = 0; i < ncam; ++i) {
    cams.push_back(w.add_camera("r" + std::to_string(i), 3));
    owner.add(cams.back(), "r" + std::to_string(i));
  }
  rpc::ServerOptions so;
  so.host = "127.0.0.1";
  so.port = 0;
  so.bus_tag = tag;
  so.io_threads = 2;
  so.wait_threads = 16;
  so.slow_threads = 2;
  so.reuseport = false;
  so.max_streams = 64;
  so.max_resets_per_s = 400;
  so.stream_deadline_ms = 4000;
  rpc::Server srv(so, [](const std::string& m, const std::string&, const std::string&) {
    rpc::Reply r;
    if (m == "Annotate") throw std::runtime_error(std::string(5000, 'e'));  // long INTERNAL message
    r.msgs.push_back("x");
    return r;
  });
  const int port = srv.port();

  std::atomic<bool> stop{false};
  std::atomic<u64> legit_ok{0}, legit_bad{0}, goaways{0}, refused{0}, fuzzed{0};
  std::vector<std::thread> th;
  for (int i = 0; i < ncam; ++i)  // producers
    th.emplace_back([&, i] {
      SynthConfig c;
      c.width = 128;
      c.height = 96;
      c.gop = 6;
      c.seed = u64(70 + i);
      SynthH264 enc(c);
      auto cam = w.camera(cams[size_t(i)]);
      while (!stop.load()) {
        cam->last_query_ms.store(now_ms());
        cam->on_access_unit(enc.next());
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
    });
  for (int k = 0; k < 3; ++k)  // legitimate clients: one stream per request, as the examples do
    th.emplace_back([&, k] {
      while (!stop.load()) {
        Client c(port, 6000);
        if (c.fd < 0) continue;
        for (u32 sid = 1; sid < 40 && !stop.load(); sid += 2) {
          const std::string dev = "r" + std::to_string((k + int(sid)) % ncam);
          c.send(frame(HEADERS, END_HEADERS, sid, request_block()) + frame(DATA, END_STREAM, sid, frame_request(dev)));
          size_t got = 0;
          int status = -1;
          u8 t, f;
          u32 s;
          std::string p;
          while (status < 0 && c.read(t, f, s, p)) {
            if (t == DATA && s == sid) got += p.size();
            if (t == HEADERS && s == sid && (f & END_STREAM)) status = trailers_status(p);
            if (t == DATA && p.size()) c.send(frame(WINUPD, 0, 0, be32s(u32(p.size()))) + frame(WINUPD, 0, sid, be32s(u32(p.size()))));
          }
          if (status == 0 && got >= 5) legit_ok.fetch_add(1);
          else legit_bad.fetch_add(1);
        }
      }
    });
  th.emplace_back([&] {  // CONTINUATION floods and HPACK bombs
    while (!stop.load()) {
      {
        Client c(port);
        c.send(frame(HEADERS, 0, 1, request_block()));
        const std::string chunk = frame(CONT, 0, 1, std::string(16384, '\0'));
        for (int i = 0; i < 64 && c.send(chunk); ++i) {
        }
        if (c.goaway() == 11) goaways.fetch_add(1);
      }
      {
        Client c(port);
        std::string blk = request_block() + hp_lit("x-big", std::string(4000, 'v'), true) + std::string(4000, char(0x80 | 62));
        c.send(frame(HEADERS, END_HEADERS, 1, blk));
        if (c.goaway() == 11) goaways.fetch_add(1);
      }
      {
        Client c(port);
        c.send(frame(PING, 0, 0, std::string(20000, 'p')));
        if (c.goaway() == 6) goaways.fetch_add(1);
      }
    }
  });
  th.emplace_back([&] {  // stream floods + reset loops
    while (!stop.load()) {
      {
        Client c(port, 1000);
        std::string all;
        for (u32 i = 0; i < 100; ++i) all += frame(HEADERS, END_HEADERS, 1 + 2 * i, request_block());
        c.send(all);
        u8 t, f;
        u32 s;
        std::string p;
        while (c.read(t, f, s, p))
          if (t == RST && p.size() == 4 && p[3] == 7) refused.fetch_add(1);
      }
      {
        Client c(port, 1000);
        std::string all;
        for (u32 i = 0; i < 600; ++i) {
          const u32 sid = 1 + 2 * i;
          all += frame(HEADERS, END_HEADERS, sid, request_block()) + frame(DATA, 0, sid, frame_request("r0")) +
                 frame(RST, 0, sid, be32s(8));
        }
        c.send(all);
        if (c.goaway() == 11) goaways.fetch_add(1);
      }
    }
  });
  th.emplace_back([&] {  // tiny windows never opened, clients that never read, slow-method errors
    while (!stop.load()) {
      std::vector<std::unique_ptr<Client>> cs;
      for (int i = 0; i < 4; ++i) {
        cs.push_back(std::make_unique<Client>(port, 300, i == 0 ? 1 : 0));
        Client& c = *cs.back();
        c.send(frame(HEADERS, END_HEADERS, 1, request_block()) + frame(DATA, END_STREAM, 1, frame_request("r1")));
        c.send(frame(HEADERS, END_HEADERS, 3, request_block("Annotate")) + frame(DATA, END_STREAM, 3, std::string(5, '\0')));
        for (int k = 0; k < 50; ++k) c.send(frame(PING, 0, 0, "12345678"));
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
    }
  });
  th.emplace_back([&] {  // mutation fuzz
    std::mt19937 rng(99);
    std::string base = kPreface + frame(SETTINGS, 0, 0, std::string{0, 4} + be32s(1 << 20)) +
                       frame(PING, 0, 0, "abcdefgh") + frame(WINUPD, 0, 0, be32s(1 << 20));
    for (u32 i = 0; i < 3; ++i) {
      const u32 sid = 1 + 2 * i;
      const std::string blk = request_block(i == 1 ? "ListStreams" : "VideoLatestImage");
      base += frame(HEADERS, 0, sid, blk.substr(0, 20)) + frame(CONT, END_HEADERS, sid, blk.substr(20));
      base += frame(DATA, PADDED, sid, std::string(1, '\3') + frame_request("r2") + std::string(3, '\0'));
      base += frame(PRIORITY, 0, sid, std::string("\0\0\0\0\x10", 5)) + frame(DATA, END_STREAM, sid);
    }
    base += frame(RST, 0, 5, be32s(8)) + frame(GOAWAY, 0, 0, be32s(0) + be32s(0));
    while (!stop.load()) {
      std::string b = base;
      const int nm = 1 + int(rng() % 8);
      for (int m = 0; m < nm && !b.empty(); ++m) {
        const size_t i = rng() % b.size();
        switch (rng() % 4) {
          case 0: b[i] = char(rng()); break;
          case 1: b.insert(i, std::string(1 + rng() % 16, char(rng()))); break;
          case 2: b.erase(i, 1 + rng() % 16); break;
          default: b[i] = char(b[i] ^ (1 << (rng() % 8)));
        }
      }
      if (rng() % 5 == 0) b.resize(rng() % b.size());
      Client c(port, 50);
      c.send(b);
      u8 t, f;
      u32 s;
      std::string p;
      for (int k = 0; k < 4 && c.read(t, f, s, p); ++k) {
      }
      fuzzed.fetch_add(1);
    }
  });
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(8) || legit_ok.load() < 20)
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  stop.store(true);
  for (auto& t : th) t.join();
  const rpc::ServerStats st = srv.stats();
  srv.stop();
  owner.stop();
  w.stop();
  std::printf("rpc hostile: legit ok %llu bad %llu, goaways seen %llu, refused %llu, fuzzed %llu; server: "
              "goaways %llu refused %llu cancelled %llu deadline %llu protocol_errors %llu\n",
              (unsigned long long)legit_ok.load(), (unsigned long long)legit_bad.load(),
              (unsigned long long)goaways.load(), (unsigned long long)refused.load(),
              (unsigned long long)fuzzed.load(), (unsigned long long)st.goaways,
              (unsigned long long)st.refused_streams, (unsigned long long)st.cancelled_waits,
              (unsigned long long)st.deadline_streams, (unsigned long long)st.protocol_errors);
  RCHECK(legit_ok.load() >= 20 && legit_bad.load() * 20 <= legit_ok.load());
  RCHECK(goaways.load() > 0 && refused.load() > 0 && st.refused_streams > 0 && st.goaways > 0);
  RCHECK(fuzzed.load() > 0 && st.protocol_errors > 0);
}
