// RTSP 1.0 (RFC 2326) client and synthetic-camera server over TCP-interleaved RTP.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <limits>
#include <sstream>

#include "md5.h"
#include "net.h"

namespace vep::net {

// ---------------------------------------------------------------------------- socket helpers

static int connect_tcp(const std::string& host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  VEP_CHECK(rc == 0 && res, "cannot resolve host " + host);
  int fd = -1;
  std::string err = "connect failed";
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    rc = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      rc = ::poll(&p, 1, timeout_ms);
      if (rc == 1) {
        int so = 0;
        socklen_t sl = sizeof(so);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl);
        rc = so == 0 ? 0 : -1;
        if (so) err = std::string("connect: ") + strerror(so);
      } else {
        rc = -1;
        err = "connect timeout";
      }
    }
    if (rc == 0) {
      fcntl(fd, F_SETFL, fl);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      break;
    }
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  VEP_CHECK(fd >= 0, err + " (" + host + ":" + std::to_string(port) + ")");
  return fd;
}

static bool send_all(int fd, const u8* p, size_t n, int timeout_ms) {
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (k > 0) {
      p += k;
      n -= size_t(k);
      continue;
    }
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      pollfd q{fd, POLLOUT, 0};
      if (::poll(&q, 1, timeout_ms) != 1) return false;
      continue;
    }
    if (k < 0 && errno == EINTR) continue;
    return false;
  }
  return true;
}

static std::string lower(std::string s) {
  for (auto& c : s) c = char(std::tolower(u8(c)));
  return s;
}
static std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

struct Message {  // parsed RTSP request or response head
  std::string first;
  std::map<std::string, std::string> hdr;  // lower-cased keys
  std::string body;
  int status = 0;
};

static Message parse_head(const std::string& head) {
  Message m;
  std::istringstream is(head);
  std::string line;
  std::getline(is, line);
  m.first = trim(line);
  if (m.first.rfind("RTSP/", 0) == 0) {
    size_t sp = m.first.find(' ');
    if (sp != std::string::npos) m.status = std::atoi(m.first.c_str() + sp + 1);
  }
  while (std::getline(is, line)) {
    line = trim(line);
    if (line.empty()) continue;
    size_t c = line.find(':');
    if (c == std::string::npos) continue;
    m.hdr[lower(trim(line.substr(0, c)))] = trim(line.substr(c + 1));
  }
  return m;
}

// ------------------------------------------------------------------------------ RTSP client

RtspClient::RtspClient(std::string url, RtspClientOptions opt) : url_(std::move(url)), opt_(opt) {
  u_ = parse_url(url_);
  VEP_CHECK(u_.scheme == "rtsp", "RTSP URL expected: " + url_);
}

RtspClient::~RtspClient() { close(); }

void RtspClient::close() {
  if (fd_ >= 0) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  }
}

static std::string clean_url(const Url& u) {
  return "rtsp://" + u.host + ":" + std::to_string(u.port) + u.path;
}

std::string RtspClient::request(const std::string& method, const std::string& uri,
                                const std::string& extra, std::string* body) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    std::string req = method + " " + uri + " RTSP/1.0\r\nCSeq: " + std::to_string(++cseq_) +
                      "\r\nUser-Agent: " + opt_.user_agent + "\r\n";
    if (digest_) {
      std::string ha1 = md5_hex(u_.user + ":" + realm_ + ":" + u_.pass);
      std::string ha2 = md5_hex(method + ":" + uri);
      std::string resp = md5_hex(ha1 + ":" + nonce_ + ":" + ha2);
      req += "Authorization: Digest username=\"" + u_.user + "\", realm=\"" + realm_ +
             "\", nonce=\"" + nonce_ + "\", uri=\"" + uri + "\", response=\"" + resp + "\"\r\n";
    } else if (!auth_.empty()) {
      req += "Authorization: " + auth_ + "\r\n";
    }
    if (!session_.empty()) req += "Session: " + session_ + "\r\n";
    req += extra;
    req += "\r\n";
    VEP_CHECK(send_all(fd_, reinterpret_cast<const u8*>(req.data()), req.size(), opt_.timeout_ms),
              "RTSP send failed");
    // read until a full response (skipping any interleaved frames)
    const i64 deadline = mono_us() + i64(opt_.timeout_ms) * 1000;
    for (;;) {
      // drop interleaved binary frames that precede the response
      while (rpos_ < rbuf_.size() && rbuf_[rpos_] == '$') {
        if (rbuf_.size() - rpos_ < 4) break;
        size_t len = size_t(rbuf_[rpos_ + 2]) << 8 | rbuf_[rpos_ + 3];
        if (rbuf_.size() - rpos_ < 4 + len) break;
        rpos_ += 4 + len;
      }
      std::string view(reinterpret_cast<const char*>(rbuf_.data()) + rpos_, rbuf_.size() - rpos_);
      size_t he = view.find("\r\n\r\n");
      if (!view.empty() && view[0] != '$' && he != std::string::npos) {
        Message m = parse_head(view.substr(0, he + 2));
        size_t cl = m.hdr.count("content-length") ? size_t(std::atol(m.hdr["content-length"].c_str())) : 0;
        if (view.size() >= he + 4 + cl) {
          m.body = view.substr(he + 4, cl);
          rpos_ += he + 4 + cl;
          if (m.status == 401 && attempt == 0 && !u_.user.empty()) {
            std::string wa = m.hdr["www-authenticate"];
            if (lower(wa).rfind("digest", 0) == 0) {
              auto field = [&](const std::string& k) {
                size_t p = wa.find(k + "=\"");
                if (p == std::string::npos) return std::string();
                p += k.size() + 2;
                return wa.substr(p, wa.find('"', p) - p);
              };
              realm_ = field("realm");
              nonce_ = field("nonce");
              digest_ = true;
            } else {
              std::string cred = u_.user + ":" + u_.pass;
              auth_ = "Basic " + base64_encode(reinterpret_cast<const u8*>(cred.data()), cred.size());
            }
            goto retry;
          }
          VEP_CHECK(m.status == 200, method + " failed: " + m.first);
          if (m.hdr.count("session")) {
            std::string s = m.hdr["session"];
            session_ = s.substr(0, s.find(';'));
          }
          if (m.hdr.count("content-base")) base_ = m.hdr["content-base"];
          if (body) *body = m.body;
          if (rpos_ > (1u << 20)) {
            rbuf_.erase(rbuf_.begin(), rbuf_.begin() + long(rpos_));
            rpos_ = 0;
          }
          return m.first;
        }
      }
      i64 left = (deadline - mono_us()) / 1000;
      VEP_CHECK(left > 0, method + " timed out");
      pollfd p{fd_, POLLIN, 0};
      VEP_CHECK(::poll(&p, 1, int(left)) == 1, method + " timed out");
      u8 tmp[65536];
      ssize_t k = ::recv(fd_, tmp, sizeof(tmp), 0);
      VEP_CHECK(k > 0, "connection closed during " + method);
      rbuf_.insert(rbuf_.end(), tmp, tmp + k);
    }
  retry:;
  }
  throw Error(method + ": authentication failed");
}

RtspStreamInfo RtspClient::open() {
  close();
  rbuf_.clear();
  rpos_ = 0;
  session_.clear();
  cseq_ = 0;
  fd_ = connect_tcp(u_.host, u_.port, opt_.timeout_ms);
  last_rx_us_ = last_ka_us_ = mono_us();
  params_sent_ = false;
  const std::string url = clean_url(u_);
  std::string sdp;
  request("OPTIONS", url, "", nullptr);
  request("DESCRIBE", url, "Accept: application/sdp\r\n", &sdp);
  RtspStreamInfo info;
  info.sdp = sdp;
  bool video = false;
  std::istringstream is(sdp);
  std::string line;
  while (std::getline(is, line)) {
    line = trim(line);
    if (line.rfind("m=", 0) == 0) {
      video = line.rfind("m=video", 0) == 0;
      if (video) {
        std::istringstream ms(line.substr(2));
        std::string media, port, proto;
        ms >> media >> port >> proto >> info.payload_type;
      }
      continue;
    }
    if (!video) continue;
    if (line.rfind("a=rtpmap:", 0) == 0) {
      std::string v = lower(line);
      if (v.find("h265") != std::string::npos || v.find("hevc") != std::string::npos)
        info.codec = Codec::kH265;
      size_t sl = v.find('/');
      if (sl != std::string::npos) info.clock_rate = u32(std::atol(v.c_str() + sl + 1));
    } else if (line.rfind("a=fmtp:", 0) == 0) {
      auto grab = [&](const std::string& key) {
        size_t p = line.find(key + "=");
        if (p == std::string::npos) return std::string();
        p += key.size() + 1;
        size_t e = line.find(';', p);
        return trim(line.substr(p, e == std::string::npos ? std::string::npos : e - p));
      };
      std::string sp = grab("sprop-parameter-sets");
      std::stringstream ss(sp);
      std::string item;
      while (std::getline(ss, item, ',')) info.param_sets.push_back(base64_decode(item));
      for (const char* k : {"sprop-vps", "sprop-sps", "sprop-pps"}) {
        std::string v = grab(k);
        if (!v.empty()) info.param_sets.push_back(base64_decode(v));
      }
    } else if (line.rfind("a=control:", 0) == 0) {
      info.control = line.substr(10);
    } else if (line.rfind("a=framerate:", 0) == 0) {
      info.framerate = std::atof(line.c_str() + 12);
    }
  }
  std::string track = url;
  if (!info.control.empty() && info.control != "*") {
    if (info.control.rfind("rtsp://", 0) == 0) track = info.control;
    else {
      std::string base = base_.empty() ? url : base_;
      if (base.back() != '/') base += '/';
      track = base + info.control;
    }
  }
  request("SETUP", track, "Transport: RTP/AVP/TCP;unicast;interleaved=0-1\r\n", nullptr);
  request("PLAY", url, "Range: npt=0.000-\r\n", nullptr);
  info_ = info;
  dep_ = std::make_unique<Depacketizer>(info.codec);
  dep_->set_clock(info.clock_rate);
  return info;
}

// Parse every complete interleaved frame / RTSP message in the receive buffer; access units go
// to `aus`. Returns false (with the reason) on a framing error.
bool RtspClient::parse_buffer(std::vector<AuPtr>& aus, std::string& why) {
  for (;;) {
    size_t avail = rbuf_.size() - rpos_;
    if (avail < 4) break;
    const u8* p = rbuf_.data() + rpos_;
    if (p[0] == '$') {
      size_t len = size_t(p[2]) << 8 | p[3];
      if (avail < 4 + len) break;
      if (p[1] == 0) {
        RtpHeader h;
        const u8* pl;
        size_t pn;
        if (parse_rtp(p + 4, len, h, &pl, &pn) && h.pt == info_.payload_type) dep_->push(h, pl, pn, aus);
      }
      rpos_ += 4 + len;
    } else {
      std::string view(reinterpret_cast<const char*>(p), avail);
      size_t he = view.find("\r\n\r\n");
      if (he == std::string::npos) {
        if (avail > 8192) {
          why = "protocol error: unframed data";
          return false;
        }
        break;
      }
      Message m = parse_head(view.substr(0, he + 2));
      size_t cl = m.hdr.count("content-length") ? size_t(std::atol(m.hdr["content-length"].c_str())) : 0;
      if (avail < he + 4 + cl) break;
      rpos_ += he + 4 + cl;  // keep-alive response or server request: ignore
    }
  }
  if (rpos_ > (1u << 20) || rpos_ == rbuf_.size()) {
    rbuf_.erase(rbuf_.begin(), rbuf_.begin() + long(rpos_));
    rpos_ = 0;
  }
  return true;
}

// Deliver access units; the first keyframe gets the SDP parameter sets prepended when it does
// not carry its own.
void RtspClient::emit(std::vector<AuPtr>& aus, const AuCallback& cb) {
  for (auto& au : aus) {
    if (!params_sent_ && au->keyframe && !info_.param_sets.empty()) {
      bool has_sps = false;
      for (size_t i = 0; i < au->nals.size(); ++i) {
        int t = info_.codec == Codec::kH264 ? (au->nal(i)[0] & 0x1f) : ((au->nal(i)[0] >> 1) & 0x3f);
        has_sps |= (info_.codec == Codec::kH264) ? t == 7 : t == 33;
      }
      params_sent_ = true;
      if (!has_sps) {
        auto a2 = std::make_shared<AccessUnit>();
        a2->codec = au->codec;
        a2->pts = au->pts;
        a2->dts = au->dts;
        a2->duration = au->duration;
        a2->keyframe = au->keyframe;
        a2->corrupt = au->corrupt;
        a2->arrival_ms = au->arrival_ms;
        a2->seq = au->seq;
        for (auto& ps : info_.param_sets) a2->add_nal(ps.data(), ps.size());
        for (size_t i = 0; i < au->nals.size(); ++i) a2->add_nal(au->nal(i), au->nal_size(i));
        a2->pin();
        cb(a2);
        continue;
      }
    }
    cb(au);
  }
  aus.clear();
}

bool RtspClient::maintain(std::string& why) {
  const i64 now = mono_us();
  if (now - last_ka_us_ > 25'000'000) {  // session keep-alive
    std::string ka = "GET_PARAMETER " + clean_url(u_) + " RTSP/1.0\r\nCSeq: " + std::to_string(++cseq_) +
                     "\r\nSession: " + session_ + "\r\n\r\n";
    send_all(fd_, reinterpret_cast<const u8*>(ka.data()), ka.size(), opt_.timeout_ms);
    last_ka_us_ = now;
  }
  if ((now - last_rx_us_) / 1000 >= opt_.timeout_ms) {  // socket stall: nothing for timeout_ms
    why = "timeout";
    return false;
  }
  return true;
}

bool RtspClient::read_available(const AuCallback& cb, std::string& why) {
  VEP_CHECK(fd_ >= 0 && dep_, "RtspClient::read_available before open()");
  std::vector<AuPtr> aus;
  u8 tmp[1 << 16];
  // at most 8 reads per call: a camera that sends faster than we read must not hold the event
  // loop (or a stop() waiting for this callback) forever; the level-triggered loop comes back
  for (int reads = 0; reads < 8; ++reads) {
    ssize_t k = ::recv(fd_, tmp, sizeof(tmp), MSG_DONTWAIT);
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) {
      std::string perr;
      parse_buffer(aus, perr);
      dep_->flush(aus);
      emit(aus, cb);
      why = k == 0 ? "eof" : "recv error";
      return false;
    }
    last_rx_us_ = mono_us();
    bytes_ += u64(k);
    rbuf_.insert(rbuf_.end(), tmp, tmp + k);
    if (!parse_buffer(aus, why)) return false;
    emit(aus, cb);
    if (size_t(k) < sizeof(tmp)) break;  // drained
  }
  return true;
}

std::string RtspClient::run(const AuCallback& cb, const std::atomic<bool>& stop) {
  VEP_CHECK(fd_ >= 0 && dep_, "RtspClient::run before open()");
  last_ka_us_ = mono_us();
  std::string why;
  while (!stop.load()) {
    if (!maintain(why)) return why;
    pollfd p{fd_, POLLIN, 0};
    int pr = ::poll(&p, 1, std::min(opt_.timeout_ms, 200));
    if (pr == 0) continue;
    if (pr < 0) {
      if (errno == EINTR) continue;
      return "poll error";
    }
    if (!read_available(cb, why)) return why;
  }
  return "stopped";
}

// ------------------------------------------------------------------------------ RTSP server

RtspServer::RtspServer(const std::string& bind, int port) : bind_(bind), port_(port) {}

RtspServer::~RtspServer() { stop(); }

void RtspServer::add_stream(const std::string& path, const ServedStream& s) {
  auto st = std::make_shared<Stream>();
  st->cfg = s;
  SynthH264 enc(s.cfg);
  st->sps = enc.sps_nal();
  st->pps = enc.pps_nal();
  st->vps = enc.vps_nal();
  if (s.cached_frames > 0)
    for (int i = 0; i < s.cached_frames; ++i) st->cache.push_back(enc.next());
  const Codec codec = s.cfg.codec;
  for (const AuPtr& au : st->cache) {
    auto& pks = st->cache_pk.emplace_back();
    std::vector<std::vector<u8>> pk;
    for (size_t i = 0; i < au->nals.size(); ++i) {
      pk.clear();
      packetize_nal(codec, au->nal(i), au->nal_size(i), 1400, pk);
      for (size_t j = 0; j < pk.size(); ++j)
        pks.emplace_back(std::move(pk[j]), (i + 1 == au->nals.size()) && (j + 1 == pk.size()));
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  streams_[path.empty() || path[0] != '/' ? "/" + path : path] = st;
}

void RtspServer::inject(const std::string& path, Fault f) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = streams_.find(path.empty() || path[0] != '/' ? "/" + path : path);
  VEP_CHECK(it != streams_.end(), "no such stream " + path);
  it->second->fault.store(int(f));
}

void RtspServer::start() {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  VEP_CHECK(lfd_ >= 0, "socket failed");
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(u16(port_));
  VEP_CHECK(inet_pton(AF_INET, bind_.c_str(), &a.sin_addr) == 1, "bad bind address " + bind_);
  VEP_CHECK(::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0,
            "bind failed on port " + std::to_string(port_));
  VEP_CHECK(::listen(lfd_, 512) == 0, "listen failed");
  socklen_t sl = sizeof(a);
  getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &sl);
  port_ = ntohs(a.sin_port);
  stop_ = false;
  acc_ = std::thread([this] {
    name_thread("vep-farm");
    accept_loop();
  });
}

void RtspServer::stop() {
  if (stop_.exchange(true)) return;
  // wake the accept loop, join it, and only then close: the fd number must not be reused while
  // the loop may still poll it
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
  if (acc_.joinable()) acc_.join();
  if (lfd_ >= 0) {
    ::close(lfd_);
    lfd_ = -1;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  for (int i = 0; i < 200 && live_.load() > 0; ++i)  // sessions are detached; wait for them
    std::this_thread::sleep_for(std::chrono::milliseconds(25));
}

void RtspServer::accept_loop() {
  while (!stop_.load()) {
    pollfd p{lfd_, POLLIN, 0};
    int r = ::poll(&p, 1, 100);
    if (r <= 0) continue;
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(mu_);
    conn_fds_.push_back(fd);
    live_.fetch_add(1);
    std::thread([this, fd] {
      name_thread("vep-farm");
      serve(fd);
    }).detach();
  }
}

void RtspServer::serve(int fd) {
  std::string buf;
  std::shared_ptr<Stream> st;
  std::string session = std::to_string(0x1000 + (std::hash<int>()(fd) & 0xffff)) + "c" + std::to_string(fd);
  bool playing = false;
  auto reply = [&](int code, const std::string& reason, const std::string& cseq,
                   const std::string& extra, const std::string& body) {
    std::string r = "RTSP/1.0 " + std::to_string(code) + " " + reason + "\r\nCSeq: " + cseq +
                    "\r\nServer: vep-synthetic\r\n" + extra;
    if (!body.empty()) r += "Content-Length: " + std::to_string(body.size()) + "\r\n";
    r += "\r\n" + body;
    return send_all(fd, reinterpret_cast<const u8*>(r.data()), r.size(), 5000);
  };
  // ---- request/response phase ----
  while (!stop_.load() && !playing) {
    size_t he;
    while ((he = buf.find("\r\n\r\n")) == std::string::npos) {
      pollfd p{fd, POLLIN, 0};
      int r = ::poll(&p, 1, 200);
      if (stop_.load()) goto done;
      if (r <= 0) continue;
      char tmp[4096];
      ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
      if (k <= 0) goto done;
      buf.append(tmp, size_t(k));
    }
    Message m = parse_head(buf.substr(0, he + 2));
    buf.erase(0, he + 4);
    std::istringstream fl(m.first);
    std::string method, uri;
    fl >> method >> uri;
    std::string cseq = m.hdr["cseq"];
    Url u;
    try { u = parse_url(uri); } catch (...) { u.path = "/"; }
    std::string path = u.path;
    size_t tk = path.find("/trackID=");
    if (tk != std::string::npos) path = path.substr(0, tk);
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = streams_.find(path);
      if (it != streams_.end()) st = it->second;
    }
    if (method == "OPTIONS") {
      reply(200, "OK", cseq, "Public: OPTIONS, DESCRIBE, SETUP, PLAY, TEARDOWN, GET_PARAMETER\r\n", "");
      continue;
    }
    if (!st) {
      reply(404, "Not Found", cseq, "", "");
      goto done;
    }
    if (st->fault.load() == int(Fault::kRefuse)) {
      reply(503, "Service Unavailable", cseq, "", "");
      goto done;
    }
    if (!st->cfg.user.empty()) {
      std::string cred = st->cfg.user + ":" + st->cfg.pass;
      std::string want = "Basic " + base64_encode(reinterpret_cast<const u8*>(cred.data()), cred.size());
      if (m.hdr["authorization"] != want) {
        reply(401, "Unauthorized", cseq, "WWW-Authenticate: Basic realm=\"vep\"\r\n", "");
        continue;
      }
    }
    if (method == "DESCRIBE") {
      std::string sps64 = base64_encode(st->sps.data(), st->sps.size());
      std::string pps64 = base64_encode(st->pps.data(), st->pps.size());
      std::string media;
      if (st->cfg.cfg.codec == Codec::kH265) {  // RFC 7798 §7.1
        std::string vps64 = base64_encode(st->vps.data(), st->vps.size());
        media = "m=video 0 RTP/AVP 96\r\na=rtpmap:96 H265/90000\r\n"
                "a=fmtp:96 sprop-vps=" + vps64 + ";sprop-sps=" + sps64 + ";sprop-pps=" + pps64 + "\r\n";
      } else {  // RFC 6184 §8.1
        char pli[8];
        snprintf(pli, sizeof(pli), "%02X%02X%02X", st->sps[1], st->sps[2], st->sps[3]);
        media = "m=video 0 RTP/AVP 96\r\na=rtpmap:96 H264/90000\r\n"
                "a=fmtp:96 packetization-mode=1;profile-level-id=" + std::string(pli) +
                ";sprop-parameter-sets=" + sps64 + "," + pps64 + "\r\n";
      }
      std::string sdp = "v=0\r\no=- 0 0 IN IP4 " + bind_ + "\r\ns=vep synthetic camera\r\nt=0 0\r\n" +
                        media + "a=control:trackID=0\r\na=framerate:" +
                        std::to_string(st->cfg.cfg.fps) + "\r\n";
      std::string base = "rtsp://" + bind_ + ":" + std::to_string(port_) + path + "/";
      reply(200, "OK", cseq, "Content-Type: application/sdp\r\nContent-Base: " + base + "\r\n", sdp);
    } else if (method == "SETUP") {
      std::string tr = m.hdr["transport"];
      if (tr.find("TCP") == std::string::npos) {
        reply(461, "Unsupported Transport", cseq, "", "");
        continue;
      }
      reply(200, "OK", cseq, "Session: " + session + ";timeout=60\r\nTransport: RTP/AVP/TCP;unicast;interleaved=0-1\r\n", "");
    } else if (method == "PLAY") {
      reply(200, "OK", cseq, "Session: " + session + "\r\nRange: npt=0.000-\r\n", "");
      playing = true;
    } else if (method == "TEARDOWN") {
      reply(200, "OK", cseq, "Session: " + session + "\r\n", "");
      goto done;
    } else {
      reply(200, "OK", cseq, "Session: " + session + "\r\n", "");
    }
  }
  // ---- streaming phase ----
  if (playing && st) {
    std::unique_ptr<SynthH264> enc;
    if (st->cache.empty()) enc = std::make_unique<SynthH264>(st->cfg.cfg);
    const int fps = std::max(1, st->cfg.cfg.fps);
    const Codec codec = st->cfg.cfg.codec;
    RtpHeader h;
    h.ssrc = 0x5ee0000u ^ u32(fd);
    h.seq = u16(fd * 7919);
    i64 frame = 0;
    // capture instants: an access unit with the previous one's pts (the second field of a pair)
    // shares its time slot and RTP timestamp
    i64 tix = -1, prev_pts = std::numeric_limits<i64>::min();
    i64 pace_t0 = -1, pace_f0 = 0;
    std::vector<u8> out;
    std::vector<std::vector<u8>> pk;
    bool skip_gop = false;
    while (!stop_.load()) {
      // handle client requests (TEARDOWN / keep-alive) without blocking
      pollfd p{fd, POLLIN, 0};
      if (::poll(&p, 1, 0) == 1) {
        char tmp[4096];
        ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
        if (k <= 0) break;
        buf.append(tmp, size_t(k));
        size_t he;
        bool bye = false;
        while ((he = buf.find("\r\n\r\n")) != std::string::npos) {
          Message m = parse_head(buf.substr(0, he + 2));
          buf.erase(0, he + 4);
          bye |= m.first.rfind("TEARDOWN", 0) == 0;
          reply(200, "OK", m.hdr["cseq"], "Session: " + session + "\r\n", "");
        }
        if (bye) break;
      }
      int fault = st->fault.exchange(int(Fault::kNone));
      if (fault == int(Fault::kDropConnection) || fault == int(Fault::kRefuse)) {
        if (fault == int(Fault::kRefuse)) st->fault.store(fault);
        break;
      }
      if (fault == int(Fault::kStall)) {
        for (int i = 0; i < 80 && !stop_.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
      }
      AuPtr au = enc ? AuPtr(enc->next()) : st->cache[size_t(frame % i64(st->cache.size()))];
      if (fault == int(Fault::kSkipKeyframe)) skip_gop = true;
      if (skip_gop && au->keyframe) {
        skip_gop = false;
        ++frame;
        continue;
      }
      if (au->pts != prev_pts || tix < 0) ++tix;
      prev_pts = au->pts;
      const int pace = pace_.load();
      if (pace == 1 || (pace < 0 && st->cfg.realtime)) {
        if (pace_t0 < 0) {  // (re)start pacing from this frame on
          pace_t0 = mono_us();
          pace_f0 = tix;
        }
        i64 due = pace_t0 + (tix - pace_f0) * 1000000 / fps;
        i64 now = mono_us();
        if (due > now) std::this_thread::sleep_for(std::chrono::microseconds(due - now));
      } else {
        pace_t0 = -1;
      }
      h.ts = u32(tix * 90000 / fps);
      out.clear();
      const bool cached = !enc && fault != int(Fault::kCorruptNal);
      if (cached) {  // cached AU: payloads packetized once
        for (const auto& [pl, marker] : st->cache_pk[size_t(frame % i64(st->cache.size()))]) {
          h.marker = marker;
          const size_t len = kRtpHeader + pl.size();
          const size_t o = out.size();
          out.resize(o + 4 + len);
          out[o] = '$';
          out[o + 1] = 0;
          out[o + 2] = u8(len >> 8);
          out[o + 3] = u8(len);
          write_rtp_header(&out[o + 4], h);
          std::memcpy(&out[o + 4 + kRtpHeader], pl.data(), pl.size());
          ++h.seq;
        }
      }
      for (size_t i = 0; !cached && i < au->nals.size(); ++i) {
        pk.clear();
        std::vector<u8> nal(au->nal(i), au->nal(i) + au->nal_size(i));
        const bool vcl = codec == Codec::kH264 ? ((nal[0] & 0x1f) == 1 || (nal[0] & 0x1f) == 5)
                                               : ((nal[0] >> 1) & 0x3f) < 32;
        if (fault == int(Fault::kCorruptNal) && vcl && nal.size() > 16) {
          for (size_t j = 4; j < nal.size(); j += 97) nal[j] ^= 0x5a;
          nal[4] = 0x00;  // break the slice header / mb_type
          nal[5] = 0x00;
          nal[6] = 0x01;  // embedded start code: an emulation-prevention violation
        }
        packetize_nal(codec, nal.data(), nal.size(), 1400, pk);
        for (size_t j = 0; j < pk.size(); ++j) {
          h.marker = (i + 1 == au->nals.size()) && (j + 1 == pk.size());
          size_t len = kRtpHeader + pk[j].size();
          size_t o = out.size();
          out.resize(o + 4 + len);
          out[o] = '$';
          out[o + 1] = 0;
          out[o + 2] = u8(len >> 8);
          out[o + 3] = u8(len);
          write_rtp_header(&out[o + 4], h);
          std::memcpy(&out[o + 4 + kRtpHeader], pk[j].data(), pk[j].size());
          ++h.seq;
        }
      }
      // (a lossless reader pauses its socket for seconds while a slow backend drains its backlog)
      if (!send_all(fd, out.data(), out.size(), 30000)) break;
      aus_sent_.fetch_add(1);
      ++frame;
    }
  }
done:
  ::shutdown(fd, SHUT_RDWR);
  {
    std::lock_guard<std::mutex> g(mu_);
    conn_fds_.erase(std::remove(conn_fds_.begin(), conn_fds_.end(), fd), conn_fds_.end());
  }
  ::close(fd);
  live_.fetch_sub(1);
}

}  // namespace vep::net
