// Native VideoLatestImage load generator (h2load.h).
#include "h2load.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>

namespace vep::h2load {

namespace {

enum : u8 { kData = 0, kHeaders = 1, kRst = 3, kSettings = 4, kPing = 6, kGoaway = 7, kWinUpd = 8 };
constexpr u8 kEndStream = 1, kAck = 1, kEndHeaders = 4;
constexpr u32 kMaxWindow = 0x7FFFFFFFu;
constexpr u32 kWindowRefill = 8u << 20;  // connection WINDOW_UPDATE every 8 MB received

using Clock = std::chrono::steady_clock;

double now_s() { return std::chrono::duration<double>(Clock::now().time_since_epoch()).count(); }
double wall_s() { return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count(); }

void put_frame(std::string& out, u8 type, u8 flags, u32 sid, const std::string& p) {
  const u32 n = u32(p.size());
  const char h[9] = {char(n >> 16), char(n >> 8), char(n), char(type), char(flags),
                     char((sid >> 24) & 0x7F), char(sid >> 16), char(sid >> 8), char(sid)};
  out.append(h, 9);
  out += p;
}

std::string be32(u32 v) { return {char(v >> 24), char(v >> 16), char(v >> 8), char(v)}; }

// HPACK literal header field without indexing, new name (RFC 7541 §6.2.2), lengths < 127
std::string lit(const std::string& n, const std::string& v) {
  return std::string(1, '\0') + char(n.size()) + n + char(v.size()) + v;
}

struct Conn {
  int fd = -1;
  std::string name;
  std::string out;  // bytes not yet accepted by the socket
  u32 sid = 0;      // stream of the request in flight (0: none)
  u32 next_sid = 1;
  double t0 = 0;
  u64 resp_bytes = 0, unacked = 0;
  // frame parser
  u8 hdr[9] = {};
  int hdr_n = 0;
  u32 left = 0;
  u8 type = 0, flags = 0;
  u32 fsid = 0;
  std::string small;
  bool dead = false;
  bool measured = false;  // the in-flight request was sent inside the measured window
  int done = 0;           // responses completed
};

struct Shared {
  const Options* o;
  std::mutex mu;
  Result r;
};

class Loop {
 public:
  Loop(Shared& sh, std::vector<Conn>& conns) : sh_(sh), cs_(conns) {}

  void run() {
    const Options& o = *sh_.o;
    ep_ = ::epoll_create1(EPOLL_CLOEXEC);
    for (size_t i = 0; i < cs_.size(); ++i) {
      Conn& c = cs_[i];
      if (c.fd < 0) continue;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLET;
      ev.data.u64 = i;
      ::epoll_ctl(ep_, EPOLL_CTL_ADD, c.fd, &ev);
      request(c, false);  // warm-up (the server's cursor for this peer and camera)
    }
    // warm-up: every connection's first response (or its failure)
    const double warm_end = now_s() + o.connect_timeout_s;
    while (now_s() < warm_end && !all([](const Conn& c) { return c.dead || c.done >= 1; })) poll(50);
    // the measured window, on the wall clock shared with the other client processes
    while (wall_s() < o.start_at) std::this_thread::sleep_for(std::chrono::microseconds(500));
    t_end_ = now_s() + o.duration_s;
    measuring_ = true;
    for (Conn& c : cs_)
      if (!c.dead && c.sid == 0) request(c, true);
    while (now_s() < t_end_) poll(20);
    measuring_ = false;
    // responses to requests sent in the window still count; wait for them a while
    const double grace = now_s() + 10.0;
    while (now_s() < grace && !all([](const Conn& c) { return c.dead || c.sid == 0; })) poll(20);
    std::lock_guard<std::mutex> g(sh_.mu);
    sh_.r.lat_ms.insert(sh_.r.lat_ms.end(), lat_.begin(), lat_.end());
    sh_.r.ok += ok_;
    sh_.r.errors += errors_;
    sh_.r.bytes += bytes_;
    if (sh_.r.first_error.empty()) sh_.r.first_error = first_error_;
    ::close(ep_);
  }

 private:
  template <class F>
  bool all(F f) const {
    for (const Conn& c : cs_)
      if (c.fd >= 0 && !f(c)) return false;
    return true;
  }

  void fail(Conn& c, const char* why) {
    if (c.dead) return;
    c.dead = true;
    ++errors_;
    if (first_error_.empty()) first_error_ = why;
    if (c.fd >= 0) ::shutdown(c.fd, SHUT_RDWR);
  }

  void request(Conn& c, bool measured) {
    c.sid = c.next_sid;
    c.next_sid += 2;
    c.resp_bytes = 0;
    c.measured = measured;
    const std::string blk = lit(":method", "POST") + lit(":scheme", "http") +
                            lit(":path", "/chrys.cloud.videostreaming.v1beta1.Image/VideoLatestImage") +
                            lit(":authority", "vep") + lit("content-type", "application/grpc") + lit("te", "trailers");
    std::string body;  // VideoFrameRequest {key_frame_only = 1 (varint), device_id = 2}
    if (sh_.o->key_frame_only) body += std::string("\x08\x01", 2);
    body += char(0x12);
    body += char(c.name.size());
    body += c.name;
    const std::string msg = std::string(1, '\0') + be32(u32(body.size())) + body;
    put_frame(c.out, kHeaders, kEndHeaders, c.sid, blk);
    put_frame(c.out, kData, kEndStream, c.sid, msg);
    c.t0 = now_s();
    flush(c);
  }

  void flush(Conn& c) {
    while (!c.out.empty() && !c.dead) {
      const ssize_t w = ::send(c.fd, c.out.data(), c.out.size(), MSG_NOSIGNAL | MSG_DONTWAIT);
      if (w > 0) {
        c.out.erase(0, size_t(w));
        continue;
      }
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;  // EPOLLOUT resumes it
      if (w < 0 && errno == EINTR) continue;
      fail(c, "send failed");
    }
  }

  void complete(Conn& c, bool good) {
    const double t = now_s();
    if (good && c.resp_bytes > 5) {
      if (c.measured) {
        lat_.push_back((t - c.t0) * 1e3);
        ++ok_;
        bytes_ += c.resp_bytes;
      }
    } else {
      ++errors_;
      if (first_error_.empty()) first_error_ = good ? "empty response" : "stream reset";
    }
    ++c.done;
    c.sid = 0;
    if (measuring_ && t < t_end_) request(c, true);
  }

  void on_frame(Conn& c) {  // a complete non-DATA frame (payload in c.small) or the end of a DATA frame
    switch (c.type) {
      case kData:
        if ((c.flags & kEndStream) && c.fsid == c.sid && c.sid) complete(c, true);
        break;
      case kHeaders:
        if ((c.flags & kEndStream) && c.fsid == c.sid && c.sid) complete(c, true);
        break;
      case kRst:
        if (c.fsid == c.sid && c.sid) complete(c, false);
        break;
      case kSettings:
        if (!(c.flags & kAck)) {
          put_frame(c.out, kSettings, kAck, 0, std::string());
          flush(c);
        }
        break;
      case kPing:
        if (!(c.flags & kAck) && c.small.size() == 8) {
          put_frame(c.out, kPing, kAck, 0, c.small);
          flush(c);
        }
        break;
      case kGoaway:
        fail(c, "GOAWAY from the server");
        break;
      default:
        break;  // WINDOW_UPDATE, PRIORITY, CONTINUATION of a trailer block: nothing to do
    }
  }

  void on_bytes(Conn& c, const u8* p, size_t n) {
    while (n > 0 && !c.dead) {
      if (c.hdr_n < 9) {
        const size_t k = std::min(n, size_t(9 - c.hdr_n));
        std::memcpy(c.hdr + c.hdr_n, p, k);
        c.hdr_n += int(k);
        p += k;
        n -= k;
        if (c.hdr_n < 9) return;
        c.left = u32(c.hdr[0]) << 16 | u32(c.hdr[1]) << 8 | u32(c.hdr[2]);
        c.type = c.hdr[3];
        c.flags = c.hdr[4];
        c.fsid = (u32(c.hdr[5]) << 24 | u32(c.hdr[6]) << 16 | u32(c.hdr[7]) << 8 | u32(c.hdr[8])) & 0x7FFFFFFFu;
        c.small.clear();
        if (c.type != kData && c.left > (1u << 20)) return fail(c, "oversized control frame");
      }
      const size_t k = std::min(n, size_t(c.left));
      if (c.type == kData) {
        if (c.fsid == c.sid) c.resp_bytes += k;
        c.unacked += k;
      } else {
        c.small.append(reinterpret_cast<const char*>(p), k);
      }
      p += k;
      n -= k;
      c.left -= u32(k);
      if (c.left == 0) {
        c.hdr_n = 0;
        on_frame(c);
      }
    }
    if (c.unacked >= kWindowRefill && !c.dead) {  // keep the connection window open
      put_frame(c.out, kWinUpd, 0, 0, be32(u32(c.unacked)));
      c.unacked = 0;
      flush(c);
    }
  }

  void poll(int timeout_ms) {
    epoll_event evs[64];
    const int n = ::epoll_wait(ep_, evs, 64, timeout_ms);
    for (int i = 0; i < n; ++i) {
      Conn& c = cs_[size_t(evs[i].data.u64)];
      if (c.dead) continue;
      if (evs[i].events & EPOLLOUT) flush(c);
      if (evs[i].events & (EPOLLIN | EPOLLERR | EPOLLHUP)) {
        for (;;) {
          const ssize_t r = ::recv(c.fd, buf_, sizeof buf_, MSG_DONTWAIT);
          if (r > 0) {
            on_bytes(c, buf_, size_t(r));
            if (c.dead) break;
            continue;
          }
          if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
          if (r < 0 && errno == EINTR) continue;
          fail(c, "connection closed");
          break;
        }
      }
    }
  }

  Shared& sh_;
  std::vector<Conn>& cs_;
  int ep_ = -1;
  bool measuring_ = false;
  double t_end_ = 0;
  std::vector<double> lat_;
  u64 ok_ = 0, errors_ = 0, bytes_ = 0;
  std::string first_error_;
  u8 buf_[1 << 18];
};

int connect_to(const std::string& host, int port) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  int fd = -1;
  for (addrinfo* a = res; a && fd < 0; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    if (::connect(fd, a->ai_addr, a->ai_addrlen) != 0) {
      ::close(fd);
      fd = -1;
    }
  }
  ::freeaddrinfo(res);
  if (fd < 0) return -1;
  int on = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &on, sizeof on);
  // preface, SETTINGS (largest stream window, 1 MB frames), the connection window opened wide
  std::string out = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
  std::string st;
  st += std::string("\x00\x04", 2) + be32(kMaxWindow);  // SETTINGS_INITIAL_WINDOW_SIZE
  st += std::string("\x00\x05", 2) + be32(1u << 20);    // SETTINGS_MAX_FRAME_SIZE
  put_frame(out, kSettings, 0, 0, st);
  put_frame(out, kWinUpd, 0, 0, be32(kMaxWindow - 65535u));
  size_t off = 0;
  while (off < out.size()) {
    const ssize_t w = ::send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
    if (w <= 0) {
      ::close(fd);
      return -1;
    }
    off += size_t(w);
  }
  return fd;
}

double cpu_seconds() {
  rusage u{};
  ::getrusage(RUSAGE_SELF, &u);
  return double(u.ru_utime.tv_sec + u.ru_stime.tv_sec) + double(u.ru_utime.tv_usec + u.ru_stime.tv_usec) * 1e-6;
}

}  // namespace

Result run(const Options& o) {
  VEP_CHECK(!o.names.empty() && o.clients > 0, "h2load needs cameras and clients");
  Shared sh;
  sh.o = &o;
  const int nt = std::clamp(o.threads, 1, 64);
  std::vector<std::vector<Conn>> parts(static_cast<size_t>(nt));
  u64 refused = 0;
  for (int k = 0; k < o.clients; ++k) {
    Conn c;
    c.name = o.names[size_t(k) % o.names.size()];
    VEP_CHECK(c.name.size() < 120, "camera name too long");
    c.fd = connect_to(o.host, o.port);
    if (c.fd < 0) {
      ++refused;
      continue;
    }
    parts[size_t(k % nt)].push_back(std::move(c));
  }
  std::vector<std::thread> ths;
  for (int t = 0; t < nt; ++t) ths.emplace_back([&, t] { Loop(sh, parts[size_t(t)]).run(); });
  // CPU of the measured window (this process: the client threads and their socket copies)
  while (wall_s() < o.start_at) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  const double c0 = cpu_seconds();
  std::this_thread::sleep_for(std::chrono::duration<double>(o.duration_s));
  const double c1 = cpu_seconds();
  for (auto& th : ths) th.join();
  for (auto& p : parts)
    for (Conn& c : p)
      if (c.fd >= 0) ::close(c.fd);
  sh.r.errors += refused;
  if (refused && sh.r.first_error.empty()) sh.r.first_error = "connect failed";
  sh.r.cpu_s = c1 - c0;
  return std::move(sh.r);
}

}  // namespace vep::h2load
