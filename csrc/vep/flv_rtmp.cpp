// FLV tags and RTMP (Adobe RTMP 1.0 spec: simple handshake, chunk stream, AMF0 commands).
#include <algorithm>

#include "h264.h"
#include "hevc.h"
#include "mux.h"
#include "net.h"
#include "sock.h"

namespace vep::mux {

// ----------------------------------------------------------------------------------- FLV

std::vector<u8> au_to_avcc(const AccessUnit& au) {
  std::vector<u8> out;
  out.reserve(au.bytes() + 4 * au.nals.size());
  for (size_t i = 0; i < au.nals.size(); ++i) {
    const u8* n = au.nal(i);
    size_t len = au.nal_size(i);
    if (len == 0) continue;
    if (au.codec == Codec::kH264) {
      int t = n[0] & 0x1f;
      if (t == h264::kNalSps || t == h264::kNalPps || t == h264::kNalAud) continue;
    } else {
      int t = (n[0] >> 1) & 0x3f;
      if (t == 32 || t == 33 || t == 34 || t == 35) continue;  // VPS/SPS/PPS/AUD
    }
    out.push_back(u8(len >> 24));
    out.push_back(u8(len >> 16));
    out.push_back(u8(len >> 8));
    out.push_back(u8(len));
    out.insert(out.end(), n, n + len);
  }
  return out;
}

std::vector<u8> flv_avc_sequence_header(const std::vector<u8>& sps, const std::vector<u8>& pps) {
  std::vector<u8> b = {0x17, 0x00, 0x00, 0x00, 0x00};
  std::vector<u8> rec = h264::avcc_record(sps, pps);
  b.insert(b.end(), rec.begin(), rec.end());
  return b;
}

std::vector<u8> flv_avc_nalu(const AccessUnit& au) {
  std::vector<u8> b = {u8(au.keyframe ? 0x17 : 0x27), 0x01, 0x00, 0x00, 0x00};
  std::vector<u8> a = au_to_avcc(au);
  b.insert(b.end(), a.begin(), a.end());
  return b;
}

std::vector<u8> flv_sequence_header(const ParamSets& ps) {
  if (ps.codec == Codec::kH264) return flv_avc_sequence_header(ps.sps, ps.pps);
  // IsExHeader | FrameType 1 (key) | PacketType 0 (SequenceStart), FourCC, hvcC
  std::vector<u8> b = {u8(0x80 | (1 << 4) | 0), 'h', 'v', 'c', '1'};
  std::vector<u8> rec = hevc::hvcc_record(ps.vps, ps.sps, ps.pps);
  b.insert(b.end(), rec.begin(), rec.end());
  return b;
}

std::vector<u8> flv_video(const AccessUnit& au) {
  if (au.codec == Codec::kH264) return flv_avc_nalu(au);
  // PacketType 3 (CodedFramesX: composition time 0 implied), length-prefixed NAL units
  std::vector<u8> b = {u8(0x80 | ((au.keyframe ? 1 : 2) << 4) | 3), 'h', 'v', 'c', '1'};
  std::vector<u8> a = au_to_avcc(au);
  b.insert(b.end(), a.begin(), a.end());
  return b;
}

std::vector<u8> flv_tag(u8 type, u32 ts, const std::vector<u8>& body) {
  std::vector<u8> t;
  t.reserve(body.size() + 15);
  const u32 n = u32(body.size());
  t.push_back(type);
  t.push_back(u8(n >> 16));
  t.push_back(u8(n >> 8));
  t.push_back(u8(n));
  t.push_back(u8(ts >> 16));
  t.push_back(u8(ts >> 8));
  t.push_back(u8(ts));
  t.push_back(u8(ts >> 24));
  t.push_back(0);
  t.push_back(0);
  t.push_back(0);
  t.insert(t.end(), body.begin(), body.end());
  const u32 prev = n + 11;
  t.push_back(u8(prev >> 24));
  t.push_back(u8(prev >> 16));
  t.push_back(u8(prev >> 8));
  t.push_back(u8(prev));
  return t;
}

std::vector<u8> flv_file_header() {
  return {'F', 'L', 'V', 0x01, 0x01, 0x00, 0x00, 0x00, 0x09, 0x00, 0x00, 0x00, 0x00};
}

// ----------------------------------------------------------------------------------- AMF0

namespace {

struct Amf {
  std::vector<u8> b;
  Amf& num(double v) {
    b.push_back(0x00);
    u64 bits;
    std::memcpy(&bits, &v, 8);
    for (int i = 7; i >= 0; --i) b.push_back(u8(bits >> (8 * i)));
    return *this;
  }
  Amf& boolean(bool v) {
    b.push_back(0x01);
    b.push_back(v ? 1 : 0);
    return *this;
  }
  void raw_str(const std::string& s) {
    b.push_back(u8(s.size() >> 8));
    b.push_back(u8(s.size()));
    b.insert(b.end(), s.begin(), s.end());
  }
  Amf& str(const std::string& s) {
    b.push_back(0x02);
    raw_str(s);
    return *this;
  }
  Amf& null() {
    b.push_back(0x05);
    return *this;
  }
  Amf& obj_begin() {
    b.push_back(0x03);
    return *this;
  }
  Amf& key(const std::string& k) {
    raw_str(k);
    return *this;
  }
  Amf& obj_end() {
    b.push_back(0);
    b.push_back(0);
    b.push_back(0x09);
    return *this;
  }
};

struct AmfVal {
  int type = -1;
  double num = 0;
  std::string str;
  std::map<std::string, std::string> obj;  // string-valued properties only
};

bool amf_read(const std::vector<u8>& d, size_t& o, AmfVal& v) {
  if (o >= d.size()) return false;
  v = AmfVal();
  v.type = d[o++];
  auto rs = [&](std::string& s) {
    if (o + 2 > d.size()) return false;
    size_t n = size_t(d[o]) << 8 | d[o + 1];
    o += 2;
    if (o + n > d.size()) return false;
    s.assign(reinterpret_cast<const char*>(&d[o]), n);
    o += n;
    return true;
  };
  switch (v.type) {
    case 0x00: {
      if (o + 8 > d.size()) return false;
      u64 bits = 0;
      for (int i = 0; i < 8; ++i) bits = bits << 8 | d[o + size_t(i)];
      std::memcpy(&v.num, &bits, 8);
      o += 8;
      return true;
    }
    case 0x01:
      if (o + 1 > d.size()) return false;
      v.num = d[o++];
      return true;
    case 0x02:
      return rs(v.str);
    case 0x05:
    case 0x06:
      return true;
    case 0x03:
    case 0x08: {
      if (v.type == 0x08) o += 4;  // ECMA array count
      for (;;) {
        std::string k;
        if (!rs(k)) return false;
        if (k.empty()) {
          if (o < d.size() && d[o] == 0x09) ++o;
          return true;
        }
        AmfVal sub;
        if (!amf_read(d, o, sub)) return false;
        if (sub.type == 0x02) v.obj[k] = sub.str;
        else if (sub.type == 0x00) v.obj[k] = std::to_string(sub.num);
      }
    }
    default:
      return false;
  }
}

std::vector<AmfVal> amf_all(const std::vector<u8>& d) {
  std::vector<AmfVal> out;
  size_t o = 0;
  AmfVal v;
  while (amf_read(d, o, v)) out.push_back(v);
  return out;
}

void put_be(std::vector<u8>& b, u32 v, int n) {
  for (int i = n - 1; i >= 0; --i) b.push_back(u8(v >> (8 * i)));
}

// Chunk a message onto the wire (fmt 0 then fmt 3 continuation chunks).
std::vector<u8> chunk_message(int csid, u8 type, u32 stream, u32 ts, const std::vector<u8>& body,
                              u32 chunk) {
  std::vector<u8> out;
  const bool ext = ts >= 0xFFFFFF;
  out.push_back(u8(csid & 0x3f));
  put_be(out, ext ? 0xFFFFFF : ts, 3);
  put_be(out, u32(body.size()), 3);
  out.push_back(type);
  for (int i = 0; i < 4; ++i) out.push_back(u8(stream >> (8 * i)));  // little endian
  if (ext) put_be(out, ts, 4);
  size_t pos = 0;
  while (pos < body.size()) {
    if (pos) {
      out.push_back(u8(0xC0 | (csid & 0x3f)));
      if (ext) put_be(out, ts, 4);
    }
    size_t n = std::min<size_t>(chunk, body.size() - pos);
    out.insert(out.end(), body.begin() + long(pos), body.begin() + long(pos + n));
    pos += n;
  }
  return out;
}

struct ChunkReader {
  u32 chunk = 128;
  struct St { u32 ts = 0, len = 0, stream = 0, delta = 0; u8 type = 0; bool ext = false; std::vector<u8> data; };
  std::map<int, St> st;
  // Read one complete message (blocking). Returns false on EOF/timeout.
  bool next(int fd, int timeout_ms, u8& type, u32& stream, std::vector<u8>& body) {
    for (;;) {
      u8 b0;
      if (!sock::recv_all(fd, &b0, 1, timeout_ms)) return false;
      int fmt = b0 >> 6, csid = b0 & 0x3f;
      if (csid == 0 || csid == 1) {
        u8 e[2] = {0, 0};
        if (!sock::recv_all(fd, e, csid == 0 ? 1 : 2, timeout_ms)) return false;
        csid = 64 + e[0] + (csid == 1 ? e[1] * 256 : 0);
      }
      St& s = st[csid];
      u8 h[11];
      const int hl = fmt == 0 ? 11 : fmt == 1 ? 7 : fmt == 2 ? 3 : 0;
      if (hl && !sock::recv_all(fd, h, size_t(hl), timeout_ms)) return false;
      u32 t = 0;
      if (hl) t = u32(h[0]) << 16 | u32(h[1]) << 8 | h[2];
      if (fmt <= 1) {
        s.len = u32(h[3]) << 16 | u32(h[4]) << 8 | h[5];
        s.type = h[6];
      }
      if (fmt == 0) s.stream = u32(h[7]) | u32(h[8]) << 8 | u32(h[9]) << 16 | u32(h[10]) << 24;
      if (hl) s.ext = (t == 0xFFFFFF);
      if (s.ext) {
        u8 e[4];
        if (!sock::recv_all(fd, e, 4, timeout_ms)) return false;
        t = u32(e[0]) << 24 | u32(e[1]) << 16 | u32(e[2]) << 8 | e[3];
      }
      if (fmt == 0) s.ts = t;
      else if (hl) s.delta = t;
      size_t want = std::min<size_t>(chunk, s.len - s.data.size());
      size_t o = s.data.size();
      s.data.resize(o + want);
      if (want && !sock::recv_all(fd, s.data.data() + o, want, timeout_ms)) return false;
      if (s.data.size() >= s.len) {
        type = s.type;
        stream = s.stream;
        body.swap(s.data);
        s.data.clear();
        if (type == 1 && body.size() >= 4)
          chunk = (u32(body[0]) << 24 | u32(body[1]) << 16 | u32(body[2]) << 8 | body[3]) & 0x7fffffff;
        return true;
      }
    }
  }
};

bool handshake_client(int fd, int to) {
  std::vector<u8> c(1537, 0);
  c[0] = 3;
  for (size_t i = 9; i < c.size(); ++i) c[i] = u8(i * 131 + 7);
  if (!sock::send_all(fd, c.data(), c.size(), to)) return false;
  std::vector<u8> s(1 + 1536 * 2);
  if (!sock::recv_all(fd, s.data(), s.size(), to)) return false;
  return sock::send_all(fd, s.data() + 1, 1536, to);  // C2 = S1 echo
}

bool handshake_server(int fd, int to) {
  std::vector<u8> c(1537);
  if (!sock::recv_all(fd, c.data(), c.size(), to)) return false;
  std::vector<u8> s(1 + 1536 * 2, 0);
  s[0] = 3;
  std::memcpy(s.data() + 1 + 1536, c.data() + 1, 1536);  // S2 = C1 echo
  if (!sock::send_all(fd, s.data(), s.size(), to)) return false;
  std::vector<u8> c2(1536);
  return sock::recv_all(fd, c2.data(), c2.size(), to);
}

}  // namespace

// ------------------------------------------------------------------------------ publisher

RtmpPublisher::RtmpPublisher(std::string url, int timeout_ms)
    : url_(std::move(url)), timeout_ms_(timeout_ms) {
  net::Url u = net::parse_url(url_);
  VEP_CHECK(u.scheme == "rtmp", "RTMP URL expected: " + url_);
  host_ = u.host;
  port_ = u.port;
  std::string path = u.path.substr(1);
  size_t sl = path.rfind('/');
  VEP_CHECK(sl != std::string::npos && sl + 1 < path.size(), "RTMP URL needs /app/streamkey");
  app_ = path.substr(0, sl);
  key_ = path.substr(sl + 1);
  tc_url_ = "rtmp://" + host_ + ":" + std::to_string(port_) + "/" + app_;
}

RtmpPublisher::~RtmpPublisher() { close(); }

void RtmpPublisher::close() {
  std::lock_guard<std::mutex> g(fd_mu_);
  if (fd_ >= 0) {
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    fd_ = -1;
  }
}

void RtmpPublisher::interrupt() {
  std::lock_guard<std::mutex> g(fd_mu_);
  interrupted_ = true;
  if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
}

void RtmpPublisher::send_message(int csid, u8 type, u32 stream, u32 ts, const std::vector<u8>& body) {
  std::vector<u8> w = chunk_message(csid, type, stream, ts, body, out_chunk_);
  if (!sock::send_all(fd_, w.data(), w.size(), timeout_ms_)) {
    close();
    throw Error("RTMP send failed");
  }
  sent_ += w.size();
  ++msgs_;
}

void RtmpPublisher::connect() {
  close();
  int fd = sock::connect_tcp(host_, port_, timeout_ms_);
  {
    std::lock_guard<std::mutex> g(fd_mu_);
    if (interrupted_) {
      ::close(fd);
      throw Error("RTMP publisher stopped");
    }
    fd_ = fd;
  }
  VEP_CHECK(handshake_client(fd_, timeout_ms_), "RTMP handshake failed");
  ChunkReader rd;
  auto wait_for = [&](const std::string& name, double* stream_out) {
    for (;;) {
      u8 type;
      u32 st;
      std::vector<u8> body;
      VEP_CHECK(rd.next(fd_, timeout_ms_, type, st, body), "RTMP: no reply waiting for " + name);
      if (type != 20) continue;
      auto v = amf_all(body);
      if (v.empty()) continue;
      if (v[0].str == "_error") throw Error("RTMP " + name + " rejected");
      if (name == "onStatus" && v[0].str == "onStatus") {
        for (auto& x : v)
          if (x.obj.count("level") && x.obj["level"] == "error")
            throw Error("RTMP publish rejected: " + x.obj["code"]);
        return;
      }
      if (v[0].str == name) {
        if (stream_out && v.size() >= 4 && v[3].type == 0) *stream_out = v[3].num;
        return;
      }
    }
  };
  // Set Chunk Size 4096
  std::vector<u8> cs;
  put_be(cs, 4096, 4);
  send_message(2, 1, 0, 0, cs);
  out_chunk_ = 4096;
  Amf c;
  c.str("connect").num(1).obj_begin();
  c.key("app").str(app_);
  c.key("type").str("nonprivate");
  c.key("flashVer").str("FMLE/3.0 (compatible; vep)");
  c.key("tcUrl").str(tc_url_);
  c.obj_end();
  send_message(3, 20, 0, 0, c.b);
  wait_for("_result", nullptr);
  Amf r1;
  r1.str("releaseStream").num(2).null().str(key_);
  send_message(3, 20, 0, 0, r1.b);
  Amf r2;
  r2.str("FCPublish").num(3).null().str(key_);
  send_message(3, 20, 0, 0, r2.b);
  Amf cr;
  cr.str("createStream").num(4).null();
  send_message(3, 20, 0, 0, cr.b);
  double sid = 1;
  // skip _result replies to releaseStream/FCPublish until createStream's (which carries a number)
  for (;;) {
    u8 type;
    u32 st;
    std::vector<u8> body;
    VEP_CHECK(rd.next(fd_, timeout_ms_, type, st, body), "RTMP: no createStream reply");
    if (type != 20) continue;
    auto v = amf_all(body);
    if (v.size() >= 4 && v[0].str == "_result" && v[1].num == 4 && v[3].type == 0) {
      sid = v[3].num;
      break;
    }
    if (!v.empty() && v[0].str == "_error" && v.size() > 1 && v[1].num == 4)
      throw Error("RTMP createStream rejected");
  }
  stream_id_ = u32(sid);
  Amf pub;
  pub.str("publish").num(5).null().str(key_).str("live");
  send_message(8, 20, stream_id_, 0, pub.b);
  wait_for("onStatus", nullptr);
}

void RtmpPublisher::send_sequence_header(const ParamSets& ps) {
  send_message(6, 9, stream_id_, 0, flv_sequence_header(ps));
}

void RtmpPublisher::send_au(const AccessUnit& au, u32 ts_ms) {
  send_message(6, 9, stream_id_, ts_ms, flv_video(au));
}

// ---------------------------------------------------------------------------------- sink

RtmpSink::RtmpSink(const std::string& bind, int port) : bind_(bind), port_(port) {}
RtmpSink::~RtmpSink() { stop(); }

void RtmpSink::start() {
  lfd_ = sock::listen_tcp(bind_, port_);
  stop_ = false;
  acc_ = std::thread([this] {
    name_thread("vep-rtmpsink");
    while (!stop_.load()) {
      pollfd p{lfd_, POLLIN, 0};
      if (::poll(&p, 1, 100) <= 0) continue;
      int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (fd < 0) continue;
      live_.fetch_add(1);
      std::thread([this, fd] {
        name_thread("vep-rtmpsink");
        serve(fd);
      }).detach();
    }
  });
}

void RtmpSink::stop() {
  if (stop_.exchange(true)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);  // wake the accept loop; close after the join
  if (acc_.joinable()) acc_.join();
  if (lfd_ >= 0) {
    ::close(lfd_);
    lfd_ = -1;
  }
  for (int i = 0; i < 200 && live_.load() > 0; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(25));
}

std::string RtmpSink::last_stream_key() const {
  std::lock_guard<std::mutex> g(mu_);
  return key_;
}

std::vector<std::vector<u8>> RtmpSink::video_bodies() const {
  std::lock_guard<std::mutex> g(mu_);
  return bodies_;
}

void RtmpSink::serve(int fd) {
  const int to = 1000;
  auto send = [&](int csid, u8 type, u32 stream, const std::vector<u8>& body) {
    std::vector<u8> w = chunk_message(csid, type, stream, 0, body, 128);
    return sock::send_all(fd, w.data(), w.size(), to);
  };
  if (handshake_server(fd, 5000)) {
    ChunkReader rd;
    while (!stop_.load()) {
      u8 type;
      u32 st;
      std::vector<u8> body;
      if (!rd.next(fd, to, type, st, body)) {
        pollfd p{fd, POLLIN | POLLHUP, 0};
        if (stop_.load() || (::poll(&p, 1, 0) == 1 && (p.revents & POLLHUP))) break;
        // idle publisher: keep waiting unless the peer is gone
        char c;
        if (::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT) == 0) break;
        continue;
      }
      if (type == 9) {
        std::lock_guard<std::mutex> g(mu_);
        if (body.size() >= 5 && (body[0] & 0x80)) {  // enhanced RTMP
          const int pkt = body[0] & 0x0f, ftype = (body[0] >> 4) & 7;
          if (std::memcmp(&body[1], "hvc1", 4) == 0) hevc_.fetch_add(1);
          if (pkt == 0) seqhdr_.fetch_add(1);
          else if (pkt == 1 || pkt == 3) {
            video_.fetch_add(1);
            if (ftype == 1) keys_.fetch_add(1);
          }
        } else if (body.size() >= 2) {
          if (body[1] == 0) seqhdr_.fetch_add(1);
          else {
            video_.fetch_add(1);
            if ((body[0] >> 4) == 1) keys_.fetch_add(1);
          }
        }
        bytes_.fetch_add(body.size());
        if (keep_bodies_) bodies_.push_back(std::move(body));
        continue;
      }
      if (type != 20) continue;
      auto v = amf_all(body);
      if (v.size() < 2) continue;
      const std::string& cmd = v[0].str;
      const double txn = v[1].num;
      if (cmd == "connect") {
        std::vector<u8> b;
        put_be(b, 2500000, 4);
        send(2, 5, 0, b);
        b.clear();
        put_be(b, 2500000, 4);
        b.push_back(2);
        send(2, 6, 0, b);
        Amf r;
        r.str("_result").num(txn).obj_begin().key("fmsVer").str("FMS/3,0,1,123").obj_end();
        r.obj_begin().key("level").str("status").key("code").str("NetConnection.Connect.Success").obj_end();
        send(3, 20, 0, r.b);
      } else if (cmd == "createStream") {
        Amf r;
        r.str("_result").num(txn).null().num(1);
        send(3, 20, 0, r.b);
      } else if (cmd == "publish") {
        {
          std::lock_guard<std::mutex> g(mu_);
          key_ = v.size() >= 4 ? v[3].str : "";
        }
        Amf r;
        r.str("onStatus").num(0).null();
        r.obj_begin().key("level").str("status").key("code").str("NetStream.Publish.Start").obj_end();
        send(5, 20, 1, r.b);
      } else if (cmd == "releaseStream" || cmd == "FCPublish") {
        Amf r;
        r.str("_result").num(txn).null();
        send(3, 20, 0, r.b);
      }
    }
  }
  ::shutdown(fd, SHUT_RDWR);
  ::close(fd);
  live_.fetch_sub(1);
}

}  // namespace vep::mux
