// Native gRPC endpoint (HTTP/2 + HPACK). See rpcsrv.h.
#include "rpcsrv.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "bus.h"

namespace vep::rpc {

// ============================================================================ HPACK Huffman

namespace {

// Code length of every symbol (0..255, 256 = EOS), RFC 7541 Appendix B. The code is canonical:
// within a length, codes ascend with the symbol, and each length continues where the shorter one
// ended, so the lengths define it (checked in tests against the RFC's Appendix C examples).
struct HuffTable {
  u8 len[257];
  u32 code[257];
  // decoding: per length L, the first code, the symbol count and where its symbols start in `sym`
  u32 first[31];
  u16 count[31], start[31];
  u16 sym[257];
  HuffTable() {
    auto put = [&](int n, std::initializer_list<int> syms) {
      for (int s : syms) len[s] = u8(n);
    };
    auto put_str = [&](int n, const char* s) {
      for (; *s; ++s) len[u8(*s)] = u8(n);
    };
    std::memset(len, 0, sizeof len);
    put_str(5, "012aceiost");
    put_str(6, " %-./3456789=A_bdfghlmnpru");
    put_str(7, ":BCDEFGHIJKLMNOPQRSTUVWYjkqvwxyz");
    put_str(8, "&*,;XZ");
    put_str(10, "!\"()?");
    put_str(11, "'+|");
    put_str(12, "#>");
    put(13, {0, '$', '@', '[', ']', '~'});
    put_str(14, "^}");
    put_str(15, "<`{");
    put(19, {92, 195, 208});
    put(20, {128, 130, 131, 162, 184, 194, 224, 226});
    put(21, {153, 161, 167, 172, 176, 177, 179, 209, 216, 217, 227, 229, 230});
    put(22, {129, 132, 133, 134, 136, 146, 154, 156, 160, 163, 164, 169, 170, 173, 178, 181, 185, 186, 187, 189,
             190, 196, 198, 228, 232, 233});
    put(23, {1, 135, 137, 138, 139, 140, 141, 143, 147, 149, 150, 151, 152, 155, 157, 158, 165, 166, 168, 174, 175,
             180, 182, 183, 188, 191, 197, 231, 239});
    put(24, {9, 142, 144, 145, 148, 159, 171, 206, 215, 225, 236, 237});
    put(25, {199, 207, 234, 235});
    put(26, {192, 193, 200, 201, 202, 205, 210, 213, 218, 219, 238, 240, 242, 243, 255});
    put(27, {203, 204, 211, 212, 214, 221, 222, 223, 241, 244, 245, 246, 247, 248, 250, 251, 252, 253, 254});
    put(28, {2, 3, 4, 5, 6, 7, 8, 11, 12, 14, 15, 16, 17, 18, 19, 20, 21, 23, 24, 25, 26, 27, 28, 29, 30, 31, 127,
             220, 249});
    put(30, {10, 13, 22, 256});
    // canonical assignment
    std::memset(count, 0, sizeof count);
    for (int s = 0; s < 257; ++s) ++count[len[s]];
    u32 c = 0;
    int idx = 0;
    for (int L = 1; L <= 30; ++L) {
      first[L] = c;
      start[L] = u16(idx);
      for (int s = 0; s < 257; ++s)
        if (len[s] == L) {
          code[s] = c++;
          sym[idx++] = u16(s);
        }
      c <<= 1;
    }
  }
};
const HuffTable& huff() {
  static const HuffTable t;
  return t;
}

}  // namespace

bool huffman_decode(const u8* p, size_t n, std::string& out) {
  const HuffTable& t = huff();
  u32 acc = 0;
  int bits = 0;  // bits in acc (the current code candidate, MSB first)
  int ones = 0;  // trailing run of 1 bits since the last symbol (EOS-prefix padding)
  for (size_t i = 0; i < n; ++i)
    for (int b = 7; b >= 0; --b) {
      const u32 bit = (p[i] >> b) & 1u;
      acc = (acc << 1) | bit;
      ++bits;
      ones = bit ? ones + 1 : 0;
      if (bits >= 5 && t.count[bits] && acc - t.first[bits] < t.count[bits]) {
        const int s = t.sym[t.start[bits] + (acc - t.first[bits])];
        if (s == 256) return false;  // EOS inside the string
        out.push_back(char(s));
        acc = 0;
        bits = 0;
        ones = 0;
      } else if (bits > 30) {
        return false;
      }
    }
  // padding: fewer than 8 bits, all ones (a prefix of EOS)
  return bits < 8 && ones == bits;
}

std::string huffman_encode(const std::string& s) {
  const HuffTable& t = huff();
  std::string out;
  u64 acc = 0;
  int bits = 0;
  for (unsigned char ch : s) {
    acc = (acc << t.len[ch]) | t.code[ch];
    bits += t.len[ch];
    while (bits >= 8) {
      out.push_back(char((acc >> (bits - 8)) & 0xFF));
      bits -= 8;
    }
  }
  if (bits > 0) out.push_back(char(((acc << (8 - bits)) | ((1u << (8 - bits)) - 1)) & 0xFF));
  return out;
}

// ============================================================================ HPACK decoder

namespace {

const char* const kStatic[62][2] = {
    {"", ""},
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""},
    {"cache-control", ""}, {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""},
    {"content-length", ""}, {"content-location", ""}, {"content-range", ""}, {"content-type", ""},
    {"cookie", ""}, {"date", ""}, {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""},
    {"if-match", ""}, {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""},
    {"if-unmodified-since", ""}, {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""},
    {"proxy-authenticate", ""}, {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""},
    {"retry-after", ""}, {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""},
    {"transfer-encoding", ""}, {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""},
};

// HPACK integer with an N-bit prefix (§5.1)
bool read_int(const u8*& p, const u8* end, int prefix, u64& v) {
  if (p >= end) return false;
  const u32 mask = (1u << prefix) - 1;
  v = *p++ & mask;
  if (v < mask) return true;
  int shift = 0;
  for (;;) {
    if (p >= end || shift > 56) return false;
    const u8 b = *p++;
    v += u64(b & 0x7F) << shift;
    shift += 7;
    if (!(b & 0x80)) return true;
  }
}

bool read_str(const u8*& p, const u8* end, std::string& s) {
  if (p >= end) return false;
  const bool h = (*p & 0x80) != 0;
  u64 n;
  if (!read_int(p, end, 7, n) || n > u64(end - p)) return false;
  s.clear();
  if (h) {
    if (!huffman_decode(p, size_t(n), s)) return false;
  } else {
    s.assign(reinterpret_cast<const char*>(p), size_t(n));
  }
  p += n;
  return true;
}

void put_int(std::string& s, int prefix, u8 first_bits, u64 v) {
  const u32 mask = (1u << prefix) - 1;
  if (v < mask) {
    s.push_back(char(first_bits | u8(v)));
    return;
  }
  s.push_back(char(first_bits | mask));
  v -= mask;
  while (v >= 128) {
    s.push_back(char(0x80 | (v & 0x7F)));
    v >>= 7;
  }
  s.push_back(char(v));
}

// literal header field without indexing, new name (§6.2.2), raw strings
void put_literal(std::string& s, const std::string& name, const std::string& value) {
  s.push_back(0);
  put_int(s, 7, 0, name.size());
  s += name;
  put_int(s, 7, 0, value.size());
  s += value;
}

}  // namespace

bool HpackDecoder::entry(size_t idx, std::string& name, std::string& value) const {
  if (idx == 0) return false;
  if (idx <= 61) {
    name = kStatic[idx][0];
    value = kStatic[idx][1];
    return true;
  }
  idx -= 62;
  if (idx >= dyn_.size()) return false;
  name = dyn_[idx].first;
  value = dyn_[idx].second;
  return true;
}

void HpackDecoder::evict() {
  while (size_ > max_ && !dyn_.empty()) {
    size_ -= dyn_.back().first.size() + dyn_.back().second.size() + 32;
    dyn_.pop_back();
  }
}

void HpackDecoder::add(const std::string& name, const std::string& value) {
  const size_t sz = name.size() + value.size() + 32;
  if (sz > max_) {  // (larger than the table: empties it, §4.4)
    dyn_.clear();
    size_ = 0;
    return;
  }
  dyn_.insert(dyn_.begin(), {name, value});
  size_ += sz;
  evict();
}

bool HpackDecoder::decode(const u8* p, size_t n, std::vector<std::pair<std::string, std::string>>& out) {
  const u8* end = p + n;
  std::string name, value;
  size_t list = 0;
  over_ = false;
  auto emit = [&]() {
    list += name.size() + value.size() + 32;
    if (list > max_list_) {
      over_ = true;
      return false;
    }
    out.emplace_back(name, value);
    return true;
  };
  while (p < end) {
    const u8 b = *p;
    u64 idx;
    if (b & 0x80) {  // indexed (§6.1)
      if (!read_int(p, end, 7, idx) || !entry(size_t(idx), name, value)) return false;
      if (!emit()) return false;
    } else if ((b & 0xC0) == 0x40) {  // literal with incremental indexing (§6.2.1)
      if (!read_int(p, end, 6, idx)) return false;
      if (idx) {
        std::string v;
        if (!entry(size_t(idx), name, v)) return false;
      } else if (!read_str(p, end, name)) {
        return false;
      }
      if (!read_str(p, end, value)) return false;
      add(name, value);
      if (!emit()) return false;
    } else if ((b & 0xE0) == 0x20) {  // dynamic table size update (§6.3)
      if (!read_int(p, end, 5, idx) || idx > limit_) return false;
      max_ = size_t(idx);
      evict();
    } else {  // literal without indexing (0000) / never indexed (0001) (§6.2.2-3)
      if (!read_int(p, end, 4, idx)) return false;
      if (idx) {
        std::string v;
        if (!entry(size_t(idx), name, v)) return false;
      } else if (!read_str(p, end, name)) {
        return false;
      }
      if (!read_str(p, end, value)) return false;
      if (!emit()) return false;
    }
  }
  return true;
}

// ============================================================================ server

namespace {

enum : u8 { kData = 0, kHeaders = 1, kPriority = 2, kRst = 3, kSettings = 4, kPush = 5, kPing = 6, kGoaway = 7,
            kWindowUpdate = 8, kContinuation = 9 };
enum : u8 { kEndStream = 1, kAck = 1, kEndHeaders = 4, kPadded = 8, kPriorityFlag = 0x20 };
// error codes (RFC 7540 7)
enum : u32 { kNoError = 0, kProtocolError = 1, kFlowControlError = 3, kFrameSizeError = 6, kRefusedStream = 7,
             kCancel = 8, kCompressionError = 9, kEnhanceYourCalm = 11 };
constexpr u32 kMaxFrame = 16384;  // SETTINGS_MAX_FRAME_SIZE: never raised by this server
constexpr size_t kMaxGrpcMessage = 1024;  // grpc-message bytes before percent-encoding
constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr size_t kPrefaceLen = 24;
constexpr i64 kRecvStreamWindow = 1 << 20;     // advertised per stream (requests are tiny)
constexpr i64 kRecvConnBoost = (16 << 20) - 65535;  // raise the connection window at start

i64 now_ms_mono() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void frame_hdr(std::string& s, u32 len, u8 type, u8 flags, u32 sid) {
  const char h[9] = {char(len >> 16), char(len >> 8), char(len), char(type), char(flags),
                     char((sid >> 24) & 0x7F), char(sid >> 16), char(sid >> 8), char(sid)};
  s.append(h, 9);
}

u32 be32(const u8* p) { return u32(p[0]) << 24 | u32(p[1]) << 16 | u32(p[2]) << 8 | u32(p[3]); }

std::string pct_encode(const std::string& m) {  // grpc-message (gRPC HTTP/2 protocol: percent-encoded)
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : m) {
    if (c >= 0x20 && c <= 0x7E && c != '%') o.push_back(char(c));
    else o += std::string("%") + hex[c >> 4] + hex[c & 15];
  }
  return o;
}

// VideoFrameRequest (proto: key_frame_only = 1 bool, device_id = 2 string)
bool parse_frame_request(const std::string& m, std::string& dev, bool& kfo) {
  const u8* p = reinterpret_cast<const u8*>(m.data());
  const u8* end = p + m.size();
  dev.clear();
  kfo = false;
  auto varint = [&](u64& v) {
    v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (p >= end) return false;
      const u8 b = *p++;
      v |= u64(b & 0x7F) << sh;
      if (!(b & 0x80)) return true;
    }
    return false;
  };
  while (p < end) {
    u64 key, v;
    if (!varint(key)) return false;
    const u32 field = u32(key >> 3), wt = u32(key & 7);
    if (wt == 0) {
      if (!varint(v)) return false;
      if (field == 1) kfo = v != 0;
    } else if (wt == 2) {
      if (!varint(v) || v > u64(end - p)) return false;
      if (field == 2) dev.assign(reinterpret_cast<const char*>(p), size_t(v));
      p += v;
    } else if (wt == 1) {
      if (end - p < 8) return false;
      p += 8;
    } else if (wt == 5) {
      if (end - p < 4) return false;
      p += 4;
    } else {
      return false;
    }
  }
  return true;
}

// A byte range kept alive by `keep`: an output string, or a leased bus slot (lease_ms > 0: the
// bytes live in the frame bus's shared memory, taken then; see bus::Reader::lease).
struct Chunk {
  std::shared_ptr<const void> keep;
  const char* p = nullptr;
  size_t len = 0;
  i64 lease_ms = 0;
};
// One gRPC message (5-byte prefix included) as one or more ranges.
struct Msg {
  std::vector<Chunk> parts;
  size_t size = 0;
  i64 lease_ms = 0;
};
using Buf = std::shared_ptr<const Msg>;

Buf make_msg(std::string s) {
  auto str = std::make_shared<const std::string>(std::move(s));
  auto m = std::make_shared<Msg>();
  m->parts.push_back(Chunk{str, str->data(), str->size(), 0});
  m->size = str->size();
  return m;
}

enum class Kind { kFrame, kSlow, kUnknown };

struct Stream {
  u32 id = 0;
  Kind kind = Kind::kUnknown;
  std::string method;
  std::string rbuf;                  // request bytes not yet framed into messages
  std::deque<std::string> requests;  // complete request messages
  bool remote_closed = false, headers_sent = false, trailers_queued = false, trailers_sent = false;
  bool inflight = false;             // a frame / slow job runs for this stream
  std::shared_ptr<std::atomic<bool>> cancel;  // set when the client resets the stream mid-job
  i64 t0_ms = 0;
  i64 send_win = 65535;
  i64 recv_win = 0;                  // what the client may still send on this stream
  size_t held = 0;                   // received DATA payload bytes not yet credited back
  std::deque<Chunk> pending;         // response messages (5-byte prefix included)
  int status = 0;
  std::string message;
};

struct Conn {
  int fd = -1;
  u64 id = 0;
  std::string peer;
  std::string in;
  size_t in_off = 0;
  bool preface = false, closing = false, epollout = false;
  HpackDecoder hp;
  u32 peer_max_frame = 16384;
  i64 peer_init_win = 65535, conn_send_win = 65535;
  u32 hdr_sid = 0;  // header block in progress (CONTINUATION expected)
  bool hdr_end_stream = false;
  std::string hdr_block;
  u32 last_sid = 0;
  std::map<u32, Stream> streams;
  std::deque<Chunk> out;
  size_t out_bytes = 0;
  bool read_paused = false;      // input paused while the client does not read its output
  i64 recv_win = 0;              // connection receive window left to the client
  u64 credit = 0;                // consumed bytes not yet returned by a connection WINDOW_UPDATE
  i64 rst_window_ms = 0;         // rapid-reset accounting: resets of unanswered streams per second
  u32 rst_count = 0;
};

}  // namespace

struct Server::Impl {
  ServerOptions opt;
  SlowHandler slow;
  bus::Reader reader;
  int listen_fd = -1;
  int port = 0;
  std::atomic<bool> stop_{false};
  std::atomic<u64> next_conn{1};

  struct Loop {
    int ep = -1, wake = -1;
    std::thread th;
    std::mutex mu;
    std::vector<std::function<void()>> tasks;
    std::unordered_map<int, std::shared_ptr<Conn>> conns;  // by fd (loop thread only)
    std::unordered_map<u64, int> fd_of;                    // conn id -> fd (loop thread only)
    i64 last_sweep_ms = 0;
  };
  std::vector<std::unique_ptr<Loop>> loops;
  std::atomic<u32> rr{0};

  // blocking pools
  struct Pool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    bool stop = false;
  };
  Pool waiters, slows;

  // per (peer, camera) cursors (LRU) and per camera newest copied frame
  std::mutex cur_mu;
  std::list<std::string> lru;
  std::unordered_map<std::string, std::pair<i64, std::list<std::string>::iterator>> cursors;
  // one copy out of the bus per frame per process: the first waiter to see a new frame copies it,
  // the others wait for that copy instead of making their own
  struct Cached {
    i64 seq = 0, copying = 0;
    Buf msg;
  };
  std::mutex cache_mu;
  std::condition_variable cache_cv;
  std::unordered_map<std::string, Cached> cache;
  Buf empty_msg = make_msg(std::string(5, '\0'));

  // stats
  std::atomic<u64> n_conn{0}, n_open{0}, n_streams{0}, n_frames{0}, n_empty{0}, n_bytes{0}, n_slow{0}, n_copies{0},
      n_proto{0}, n_goaway{0}, n_refused{0}, n_cancelled{0}, n_deadline{0}, n_leased{0}, n_slow_readers{0};
  mutable std::mutex lat_mu;
  std::vector<float> lat;
  size_t lat_next = 0;

  Impl(const ServerOptions& o, SlowHandler s) : opt(o), slow(std::move(s)), reader(o.bus_tag) {
    const char* z = std::getenv("VEP_RPC_ZERO_COPY");  // 0: copy each new frame (A/B)
    if (z && z[0] == '0') opt.zero_copy = false;
  }

  // ------------------------------------------------------------------ pools
  void pool_start(Pool& p, int n, const char* name) {
    for (int i = 0; i < std::max(1, n); ++i)
      p.th.emplace_back([this, &p, name] {
        name_thread(name);
        std::unique_lock<std::mutex> g(p.mu);
        for (;;) {
          p.cv.wait(g, [&] { return p.stop || !p.q.empty(); });
          if (p.stop && p.q.empty()) return;
          auto fn = std::move(p.q.front());
          p.q.pop_front();
          g.unlock();
          try {
            fn();
          } catch (...) {
          }
          g.lock();
        }
      });
  }
  void pool_post(Pool& p, std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> g(p.mu);
      p.q.push_back(std::move(fn));
    }
    p.cv.notify_one();
  }
  void pool_stop(Pool& p) {
    {
      std::lock_guard<std::mutex> g(p.mu);
      p.stop = true;
    }
    p.cv.notify_all();
    for (auto& t : p.th) t.join();
    p.th.clear();
  }

  // ------------------------------------------------------------------ loops
  void post(Loop& L, std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> g(L.mu);
      L.tasks.push_back(std::move(fn));
    }
    const u64 one = 1;
    (void)!::write(L.wake, &one, sizeof one);
  }

  static constexpr u64 kWakeTag = ~0ull, kListenTag = ~1ull;

  // The listen address: an IPv4 / IPv6 literal or a host name ("localhost", "::", "" = any),
  // resolved with getaddrinfo like grpc's ":port" / "[::]:port" listeners.
  void listen_on() {
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
    addrinfo* res = nullptr;
    const std::string svc = std::to_string(opt.port);
    const int rc = ::getaddrinfo(opt.host.empty() ? nullptr : opt.host.c_str(), svc.c_str(), &hints, &res);
    VEP_CHECK(rc == 0 && res, "rpc: cannot resolve listen host '" + opt.host + "': " + ::gai_strerror(rc));
    std::string err;
    for (addrinfo* ai = res; ai; ai = ai->ai_next) {
      const int fd = ::socket(ai->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      if (fd < 0) continue;
      int on = 1, off = 0;
      ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &on, sizeof on);
      if (opt.reuseport) ::setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &on, sizeof on);
      if (ai->ai_family == AF_INET6) ::setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &off, sizeof off);  // dual stack
      if (::bind(fd, ai->ai_addr, ai->ai_addrlen) == 0 && ::listen(fd, 1024) == 0) {
        listen_fd = fd;
        break;
      }
      err = std::strerror(errno);
      ::close(fd);
    }
    ::freeaddrinfo(res);
    VEP_CHECK(listen_fd >= 0, "rpc: bind to " + opt.host + ":" + std::to_string(opt.port) + " failed: " + err);
    sockaddr_storage a{};
    socklen_t sl = sizeof a;
    ::getsockname(listen_fd, reinterpret_cast<sockaddr*>(&a), &sl);
    port = a.ss_family == AF_INET6 ? ntohs(reinterpret_cast<sockaddr_in6*>(&a)->sin6_port)
                                   : ntohs(reinterpret_cast<sockaddr_in*>(&a)->sin_port);
  }

  void start() {
    listen_on();
    pool_start(waiters, opt.wait_threads, "vep-rpc-wait");
    pool_start(slows, opt.slow_threads, "vep-rpc-slow");
    for (int i = 0; i < std::max(1, opt.io_threads); ++i) {
      auto L = std::make_unique<Loop>();
      L->ep = ::epoll_create1(EPOLL_CLOEXEC);
      L->wake = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
      VEP_CHECK(L->ep >= 0 && L->wake >= 0, "rpc: epoll / eventfd failed");
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = kWakeTag;
      ::epoll_ctl(L->ep, EPOLL_CTL_ADD, L->wake, &ev);
      if (i == 0) {
        ev.data.u64 = kListenTag;
        ::epoll_ctl(L->ep, EPOLL_CTL_ADD, listen_fd, &ev);
      }
      loops.push_back(std::move(L));
    }
    for (auto& L : loops) {
      Loop* lp = L.get();
      L->th = std::thread([this, lp] {
        name_thread("vep-rpc-io");
        run(*lp);
      });
    }
  }

  void shutdown() {
    if (stop_.exchange(true)) return;
    for (auto& L : loops) {
      const u64 one = 1;
      (void)!::write(L->wake, &one, sizeof one);
    }
    for (auto& L : loops)
      if (L->th.joinable()) L->th.join();
    pool_stop(waiters);  // (waits end within a block; results for closed connections are dropped)
    pool_stop(slows);
    for (auto& L : loops) {
      for (auto& [fd, c] : L->conns) ::close(fd);
      L->conns.clear();
      ::close(L->ep);
      ::close(L->wake);
    }
    if (listen_fd >= 0) ::close(listen_fd);
    listen_fd = -1;
  }

  void run(Loop& L) {
    epoll_event evs[64];
    while (!stop_.load()) {
      const int n = ::epoll_wait(L.ep, evs, 64, 250);
      for (int i = 0; i < n; ++i) {
        const u64 tag = evs[i].data.u64;
        if (tag == kWakeTag) {
          u64 v;
          while (::read(L.wake, &v, sizeof v) > 0) {
          }
        } else if (tag == kListenTag) {
          accept_all();
        } else {
          auto it = L.conns.find(int(tag));
          if (it == L.conns.end()) continue;
          std::shared_ptr<Conn> c = it->second;
          if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) on_readable(L, *c);
          if (c->fd >= 0 && (evs[i].events & EPOLLOUT)) flush(L, *c);
        }
      }
      std::vector<std::function<void()>> t;
      {
        std::lock_guard<std::mutex> g(L.mu);
        t.swap(L.tasks);
      }
      for (auto& f : t) f();
      const i64 now = now_ms_mono();
      if (now - L.last_sweep_ms >= 500) {
        L.last_sweep_ms = now;
        sweep(L);
      }
    }
  }

  // grpc's peer strings: "ipv4:1.2.3.4:port", "ipv6:[::1]:port" (a v4-mapped v6 peer as ipv4)
  static std::string peer_name(const sockaddr_storage& a) {
    char ip[INET6_ADDRSTRLEN] = {0};
    if (a.ss_family == AF_INET6) {
      const auto* v6 = reinterpret_cast<const sockaddr_in6*>(&a);
      const int p = ntohs(v6->sin6_port);
      if (IN6_IS_ADDR_V4MAPPED(&v6->sin6_addr)) {
        ::inet_ntop(AF_INET, &v6->sin6_addr.s6_addr[12], ip, sizeof ip);
        return std::string("ipv4:") + ip + ":" + std::to_string(p);
      }
      ::inet_ntop(AF_INET6, &v6->sin6_addr, ip, sizeof ip);
      return std::string("ipv6:[") + ip + "]:" + std::to_string(p);
    }
    const auto* v4 = reinterpret_cast<const sockaddr_in*>(&a);
    ::inet_ntop(AF_INET, &v4->sin_addr, ip, sizeof ip);
    return std::string("ipv4:") + ip + ":" + std::to_string(ntohs(v4->sin_port));
  }

  void accept_all() {
    for (;;) {
      sockaddr_storage a{};
      socklen_t sl = sizeof a;
      const int fd = ::accept4(listen_fd, reinterpret_cast<sockaddr*>(&a), &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int on = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &on, sizeof on);
      int sndbuf = 8 << 20;
      ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof sndbuf);
      auto c = std::make_shared<Conn>();
      c->fd = fd;
      c->id = next_conn.fetch_add(1);
      c->peer = peer_name(a);
      c->hp.set_max_list(opt.max_header_list);
      n_conn.fetch_add(1);
      n_open.fetch_add(1);
      Loop& L = *loops[rr.fetch_add(1) % loops.size()];
      post(L, [this, &L, c] { adopt(L, c); });
    }
  }

  void adopt(Loop& L, const std::shared_ptr<Conn>& c) {
    L.conns[c->fd] = c;
    L.fd_of[c->id] = c->fd;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = u64(c->fd);
    ::epoll_ctl(L.ep, EPOLL_CTL_ADD, c->fd, &ev);
    // server preface: SETTINGS (max concurrent streams, per-stream receive window, max header
    // list size), then a connection window update
    std::string s;
    frame_hdr(s, 18, kSettings, 0, 0);
    const u16 ids[3] = {3, 4, 6};
    const u32 vals[3] = {opt.max_streams, u32(kRecvStreamWindow), opt.max_header_list};
    for (int k = 0; k < 3; ++k) {
      const char e[6] = {char(ids[k] >> 8), char(ids[k]), char(vals[k] >> 24), char(vals[k] >> 16),
                         char(vals[k] >> 8), char(vals[k])};
      s.append(e, 6);
    }
    window_update(s, 0, u32(kRecvConnBoost));
    c->recv_win = 65535 + kRecvConnBoost;
    queue(*c, std::move(s));
    on_readable(L, *c);  // (bytes may already be waiting)
  }

  void close_conn(Loop& L, Conn& c) {
    if (c.fd < 0) return;
    ::epoll_ctl(L.ep, EPOLL_CTL_DEL, c.fd, nullptr);
    ::close(c.fd);
    L.fd_of.erase(c.id);
    const int fd = c.fd;
    c.fd = -1;
    n_open.fetch_sub(1);
    L.conns.erase(fd);  // (c stays alive through the caller's shared_ptr)
  }

  Conn* find(Loop& L, u64 id) {
    auto it = L.fd_of.find(id);
    if (it == L.fd_of.end()) return nullptr;
    auto c = L.conns.find(it->second);
    return c == L.conns.end() ? nullptr : c->second.get();
  }

  // ------------------------------------------------------------------ output
  static void window_update(std::string& s, u32 sid, u32 inc) {
    frame_hdr(s, 4, kWindowUpdate, 0, sid);
    const char v[4] = {char((inc >> 24) & 0x7F), char(inc >> 16), char(inc >> 8), char(inc)};
    s.append(v, 4);
  }

  void queue(Conn& c, std::string s) {
    auto b = std::make_shared<const std::string>(std::move(s));
    c.out_bytes += b->size();
    c.out.push_back(Chunk{b, b->data(), b->size(), 0});
  }

  void flush(Loop& L, Conn& c) {
    while (c.fd >= 0 && !c.out.empty()) {
      iovec iov[256];
      int k = 0;
      for (auto it = c.out.begin(); it != c.out.end() && k < 256; ++it, ++k) {
        iov[k].iov_base = const_cast<char*>(it->p);
        iov[k].iov_len = it->len;
      }
      const ssize_t w = ::writev(c.fd, iov, k);
      if (w < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        if (errno == EINTR) continue;
        close_conn(L, c);
        return;
      }
      n_bytes.fetch_add(u64(w));
      size_t left = size_t(w);
      c.out_bytes -= left;
      while (left > 0) {
        Chunk& f = c.out.front();
        const size_t t = std::min(left, f.len);
        f.p += t;
        f.len -= t;
        left -= t;
        if (f.len == 0) c.out.pop_front();
      }
    }
    if (c.fd < 0) return;
    const bool want = !c.out.empty();
    bool resume = false;
    if (c.read_paused && c.out_bytes <= opt.out_high_water / 2) {
      c.read_paused = false;
      resume = true;
    }
    if (want != c.epollout || resume) {
      set_events(L, c, want);
      c.epollout = want;
    }
    if (c.closing && c.out.empty() && c.streams.empty()) close_conn(L, c);
    if (resume && c.fd >= 0) on_readable(L, c);  // (level-triggered: bytes may be waiting)
  }

  void set_events(Loop& L, Conn& c, bool out) {
    epoll_event ev{};
    ev.events = (c.read_paused ? 0u : u32(EPOLLIN | EPOLLRDHUP)) | (out ? u32(EPOLLOUT) : 0u);
    ev.data.u64 = u64(c.fd);
    ::epoll_ctl(L.ep, EPOLL_CTL_MOD, c.fd, &ev);
  }

  // A header block as HEADERS + CONTINUATION frames no larger than the peer's max frame size.
  void queue_block(Conn& c, const std::string& blk, u32 sid, bool end_stream) {
    const size_t mf = std::max<size_t>(c.peer_max_frame, 16384);
    std::string f;
    size_t off = 0;
    do {
      const size_t n = std::min(mf, blk.size() - off);
      const bool last = off + n == blk.size();
      const u8 type = off == 0 ? kHeaders : kContinuation;
      const u8 flags = u8((last ? kEndHeaders : 0) | (off == 0 && end_stream ? kEndStream : 0));
      frame_hdr(f, u32(n), type, flags, sid);
      f.append(blk, off, n);
      off += n;
    } while (off < blk.size());
    queue(c, std::move(f));
  }

  void send_headers(Conn& c, Stream& s) {
    std::string blk;
    blk.push_back(char(0x88));  // :status 200 (static 8)
    put_int(blk, 4, 0x00, 31);  // content-type (static 31), literal without indexing
    put_int(blk, 7, 0, 16);
    blk += "application/grpc";
    std::string f;
    frame_hdr(f, u32(blk.size()), kHeaders, kEndHeaders, s.id);
    queue(c, f + blk);
    s.headers_sent = true;
  }

  void send_trailers(Conn& c, Stream& s) {
    std::string blk;
    if (!s.headers_sent) {  // trailers-only response
      blk.push_back(char(0x88));
      put_int(blk, 4, 0x00, 31);
      put_int(blk, 7, 0, 16);
      blk += "application/grpc";
    }
    put_literal(blk, "grpc-status", std::to_string(s.status));
    if (!s.message.empty()) put_literal(blk, "grpc-message", pct_encode(s.message.substr(0, kMaxGrpcMessage)));
    queue_block(c, blk, s.id, true);
    s.trailers_sent = true;
  }

  // DATA frames of every stream within the flow-control windows (round robin, one frame per
  // stream per pass), trailers after a stream's last message
  void pump(Loop& L, Conn& c) {
    bool progress = true;
    while (progress) {
      progress = false;
      for (auto it = c.streams.begin(); it != c.streams.end();) {
        Stream& s = it->second;
        if (!s.pending.empty() && c.conn_send_win > 0 && s.send_win > 0) {
          Chunk& m = s.pending.front();
          const size_t n = size_t(std::min<i64>({i64(m.len), i64(c.peer_max_frame), c.conn_send_win, s.send_win}));
          std::string h;
          frame_hdr(h, u32(n), kData, 0, s.id);
          queue(c, std::move(h));
          c.out.push_back(Chunk{m.keep, m.p, n, m.lease_ms});
          c.out_bytes += n;
          m.p += n;
          m.len -= n;
          c.conn_send_win -= i64(n);
          s.send_win -= i64(n);
          if (m.len == 0) s.pending.pop_front();
          progress = true;
        }
        if (s.pending.empty() && s.trailers_queued && !s.trailers_sent) {
          send_trailers(c, s);
          progress = true;
        }
        if (s.trailers_sent) {
          it = erase_stream(c, it);
          continue;
        }
        ++it;
      }
    }
    flush(L, c);
  }

  void respond(Conn& c, Stream& s, const Buf& msg) {
    if (!s.headers_sent) send_headers(c, s);
    for (const Chunk& part : msg->parts) s.pending.push_back(part);
  }

  void finish(Conn& c, Stream& s, int status, const std::string& message) {
    if (s.trailers_queued) return;
    s.trailers_queued = true;
    s.status = status;
    s.message = message;
  }

  void rst(Conn& c, u32 sid, u32 code) {
    std::string f;
    frame_hdr(f, 4, kRst, 0, sid);
    const char v[4] = {char(code >> 24), char(code >> 16), char(code >> 8), char(code)};
    f.append(v, 4);
    queue(c, std::move(f));
  }

  void goaway(Conn& c, u32 code) {
    if (code != kNoError) n_goaway.fetch_add(1);
    std::string f;
    frame_hdr(f, 8, kGoaway, 0, 0);
    const u32 ls = c.last_sid;
    const char v[8] = {char((ls >> 24) & 0x7F), char(ls >> 16), char(ls >> 8), char(ls),
                       char(code >> 24), char(code >> 16), char(code >> 8), char(code)};
    f.append(v, 8);
    queue(c, std::move(f));
    c.closing = true;
  }

  // ------------------------------------------------------------------ input
  // Received DATA bytes of a stream consumed (a request taken, failed or dropped): the client may
  // send that much again. Connection credit goes back in batches; stream credit only to open
  // streams that can still send.
  void release(Conn& c, Stream* s, size_t n) {
    if (n == 0) return;
    if (s) {
      n = std::min(n, s->held);
      s->held -= n;
      if (!s->remote_closed && !s->trailers_queued) {
        std::string w;
        window_update(w, s->id, u32(n));
        s->recv_win += i64(n);
        queue(c, std::move(w));
      }
    }
    c.credit += n;
    if (c.credit >= 16384) {
      std::string w;
      window_update(w, 0, u32(c.credit));
      c.recv_win += i64(c.credit);
      c.credit = 0;
      queue(c, std::move(w));
    }
  }

  std::map<u32, Stream>::iterator erase_stream(Conn& c, std::map<u32, Stream>::iterator it) {
    Stream& s = it->second;
    if (s.cancel) s.cancel->store(true, std::memory_order_release);
    const size_t h = s.held;
    s.held = 0;
    c.credit += h;
    return c.streams.erase(it);
  }

  void on_readable(Loop& L, Conn& c) {
    if (c.out_bytes > opt.out_high_water) {  // the client does not read what it asks for: pause its input
      if (!c.read_paused) {
        c.read_paused = true;
        set_events(L, c, true);
        c.epollout = true;
      }
      return;
    }
    char buf[1 << 16];
    size_t got = 0;
    while (got < opt.read_budget) {  // (level-triggered: what is left comes with the next event)
      const ssize_t r = ::read(c.fd, buf, sizeof buf);
      if (r > 0) {
        c.in.append(buf, size_t(r));
        got += size_t(r);
        if (size_t(r) < sizeof buf) break;
        continue;
      }
      if (r == 0) {
        close_conn(L, c);
        return;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      close_conn(L, c);
      return;
    }
    const u32 err = parse(L, c);
    if (err != kNoError) {
      n_proto.fetch_add(1);
      goaway(c, err);
      c.in.clear();
      c.in_off = 0;
      for (auto it = c.streams.begin(); it != c.streams.end();) it = erase_stream(c, it);
      flush(L, c);
      if (c.fd >= 0) close_conn(L, c);
      return;
    }
    pump(L, c);
  }

  u32 parse(Loop& L, Conn& c) {
    if (!c.preface) {
      if (c.in.size() < kPrefaceLen)
        return std::string(kPreface).compare(0, c.in.size(), c.in) == 0 ? kNoError : kProtocolError;
      if (c.in.compare(0, kPrefaceLen, kPreface) != 0) return kProtocolError;
      c.preface = true;
      c.in_off = kPrefaceLen;
    }
    for (;;) {
      const size_t avail = c.in.size() - c.in_off;
      if (avail < 9) break;
      const u8* h = reinterpret_cast<const u8*>(c.in.data() + c.in_off);
      const u32 len = u32(h[0]) << 16 | u32(h[1]) << 8 | u32(h[2]);
      if (len > kMaxFrame) return kFrameSizeError;  // (checked before buffering the payload)
      if (avail < 9 + size_t(len)) break;
      const u8 type = h[3], flags = h[4];
      const u32 sid = be32(h + 5) & 0x7FFFFFFFu;
      const u32 err = frame(L, c, type, flags, sid, h + 9, len);
      if (err != kNoError) return err;
      c.in_off += 9 + len;
      if (c.fd < 0) return kNoError;
    }
    if (c.in_off > 0 && c.in_off == c.in.size()) {
      c.in.clear();
      c.in_off = 0;
    } else if (c.in_off > 0) {
      c.in.erase(0, c.in_off);  // (at most one partial frame is left: <= 9 + 16384 bytes)
      c.in_off = 0;
    }
    return kNoError;
  }

  // One inbound frame; a non-zero result is a connection error (GOAWAY with that code).
  u32 frame(Loop& L, Conn& c, u8 type, u8 flags, u32 sid, const u8* p, u32 len) {
    if (c.hdr_sid && type != kContinuation) return kProtocolError;  // a header block must be contiguous
    switch (type) {
      case kSettings: {
        if (sid != 0) return kProtocolError;
        if (len % 6) return kFrameSizeError;
        if (flags & kAck) return len ? kFrameSizeError : kNoError;
        for (u32 k = 0; k < len; k += 6) {
          const u16 id = u16(p[k] << 8 | p[k + 1]);
          const u32 v = be32(p + k + 2);
          if (id == 2 && v > 1) return kProtocolError;  // ENABLE_PUSH
          if (id == 4) {  // INITIAL_WINDOW_SIZE: the delta applies to every open stream
            if (v > 0x7FFFFFFFu) return kFlowControlError;
            const i64 d = i64(v) - c.peer_init_win;
            c.peer_init_win = i64(v);
            for (auto& [i, s] : c.streams) s.send_win += d;
          } else if (id == 5) {
            if (v < 16384 || v > 16777215) return kProtocolError;
            c.peer_max_frame = v;
          }
        }
        std::string a;
        frame_hdr(a, 0, kSettings, kAck, 0);
        queue(c, std::move(a));
        return kNoError;
      }
      case kPing: {
        if (sid != 0) return kProtocolError;
        if (len != 8) return kFrameSizeError;
        if (flags & kAck) return kNoError;
        std::string a;
        frame_hdr(a, 8, kPing, kAck, 0);
        a.append(reinterpret_cast<const char*>(p), 8);
        queue(c, std::move(a));
        return kNoError;
      }
      case kWindowUpdate: {
        if (len != 4) return kFrameSizeError;
        const u32 inc = be32(p) & 0x7FFFFFFFu;
        if (sid == 0) {
          if (inc == 0) return kProtocolError;
          c.conn_send_win += inc;
          if (c.conn_send_win > 0x7FFFFFFF) return kFlowControlError;
        } else {
          auto it = c.streams.find(sid);
          if (it != c.streams.end()) {
            if (inc == 0 || it->second.send_win + i64(inc) > 0x7FFFFFFF) {
              rst(c, sid, inc == 0 ? kProtocolError : kFlowControlError);
              erase_stream(c, it);
            } else {
              it->second.send_win += inc;
            }
          }
        }
        return kNoError;
      }
      case kGoaway:
        if (sid != 0) return kProtocolError;
        c.closing = true;
        return kNoError;
      case kRst: {
        if (sid == 0) return kProtocolError;
        if (len != 4) return kFrameSizeError;
        auto it = c.streams.find(sid);
        if (it == c.streams.end()) return kNoError;
        // a reset of a stream that had not been answered: its waiter is released (cancel flag)
        // and the reset counts against the connection (rapid-reset defence)
        if (!it->second.trailers_queued) {
          if (it->second.inflight) n_cancelled.fetch_add(1);
          const i64 now = now_ms_mono();
          if (now - c.rst_window_ms >= 1000) {
            c.rst_window_ms = now;
            c.rst_count = 0;
          }
          if (++c.rst_count > opt.max_resets_per_s) {
            erase_stream(c, it);
            return kEnhanceYourCalm;
          }
        }
        erase_stream(c, it);  // (a job in flight finds no stream)
        return kNoError;
      }
      case kPriority:
        if (sid == 0) return kProtocolError;
        return len == 5 ? kNoError : kFrameSizeError;
      case kHeaders: {
        if (sid == 0 || (sid & 1) == 0) return kProtocolError;
        size_t off = 0, pad = 0;
        if (flags & kPadded) {
          if (len < 1) return kFrameSizeError;
          pad = p[0];
          off = 1;
        }
        if (flags & kPriorityFlag) off += 5;
        if (off + pad > len) return kProtocolError;
        c.hdr_block.assign(reinterpret_cast<const char*>(p + off), len - off - pad);
        c.hdr_sid = sid;
        c.hdr_end_stream = (flags & kEndStream) != 0;
        if (flags & kEndHeaders) return headers_done(L, c);
        return kNoError;
      }
      case kContinuation: {
        if (!c.hdr_sid || sid != c.hdr_sid) return kProtocolError;
        if (c.hdr_block.size() + len > opt.max_header_block) return kEnhanceYourCalm;  // CONTINUATION flood
        c.hdr_block.append(reinterpret_cast<const char*>(p), len);
        if (flags & kEndHeaders) return headers_done(L, c);
        return kNoError;
      }
      case kData: {
        if (sid == 0) return kProtocolError;
        size_t off = 0, pad = 0;
        if (flags & kPadded) {
          if (len < 1) return kFrameSizeError;
          pad = p[0];
          off = 1;
        }
        if (off + pad > len) return kProtocolError;
        // flow control (RFC 7540 6.9): what the client sends counts against the windows this
        // server advertised; the payload is credited back only as its requests are consumed, so
        // a client cannot make the server buffer more than those windows
        c.recv_win -= i64(len);
        if (c.recv_win < 0) return kFlowControlError;
        auto it = c.streams.find(sid);
        const size_t payload = len - off - pad;
        if (it == c.streams.end() || it->second.remote_closed || it->second.trailers_queued) {
          release(c, nullptr, len);  // (reset / finished / half-closed stream: dropped)
          return kNoError;
        }
        Stream& s = it->second;
        s.recv_win -= i64(len);
        if (s.recv_win < 0) {
          rst(c, sid, kFlowControlError);
          erase_stream(c, it);
          release(c, nullptr, len);
          return kNoError;
        }
        if (len > payload) release(c, nullptr, len - payload);  // padding
        s.held += payload;
        s.rbuf.append(reinterpret_cast<const char*>(p + off), payload);
        if (!messages(c, s)) return kNoError;
        if (flags & kEndStream) s.remote_closed = true;
        advance(L, c, s);
        return kNoError;
      }
      default:
        return kNoError;  // PUSH_PROMISE (never from a client), unknown types: ignored
    }
  }

  u32 headers_done(Loop& L, Conn& c) {
    const u32 sid = c.hdr_sid;
    c.hdr_sid = 0;
    std::vector<std::pair<std::string, std::string>> hs;
    const bool ok = c.hp.decode(reinterpret_cast<const u8*>(c.hdr_block.data()), c.hdr_block.size(), hs);
    c.hdr_block.clear();
    c.hdr_block.shrink_to_fit();
    if (!ok) return c.hp.list_too_large() ? kEnhanceYourCalm : kCompressionError;
    auto it = c.streams.find(sid);
    if (it != c.streams.end()) {  // trailers from the client: end of its messages
      if (c.hdr_end_stream) it->second.remote_closed = true;
      advance(L, c, it->second);
      return kNoError;
    }
    if (sid <= c.last_sid) return kNoError;  // (a stream already closed)
    c.last_sid = sid;
    if (c.streams.size() >= opt.max_streams) {  // over SETTINGS_MAX_CONCURRENT_STREAMS
      n_refused.fetch_add(1);
      rst(c, sid, kRefusedStream);
      return kNoError;
    }
    Stream& s = c.streams[sid];
    s.id = sid;
    s.t0_ms = now_ms_mono();
    s.send_win = c.peer_init_win;
    s.recv_win = kRecvStreamWindow;
    n_streams.fetch_add(1);
    std::string path, ctype;
    for (auto& [k, v] : hs) {
      if (k == ":path") path = v;
      else if (k == "content-type") ctype = v;
    }
    const std::string pre = "/" + opt.service + "/";
    if (path.compare(0, pre.size(), pre) == 0) s.method = path.substr(pre.size());
    if (s.method == "VideoLatestImage") s.kind = Kind::kFrame;
    else if (s.method == "ListStreams" || s.method == "Annotate" || s.method == "Proxy" || s.method == "Storage")
      s.kind = Kind::kSlow;
    if (s.kind == Kind::kUnknown || ctype.compare(0, 16, "application/grpc") != 0) {
      finish(c, s, 12, "unknown method " + path.substr(0, 256));  // UNIMPLEMENTED
      return kNoError;
    }
    if (c.hdr_end_stream) s.remote_closed = true;
    advance(L, c, s);
    return kNoError;
  }

  // fail a stream's request side: its buffered requests are dropped (and credited back)
  void fail(Conn& c, Stream& s, int status, const std::string& msg) {
    finish(c, s, status, msg);
    s.rbuf.clear();
    s.requests.clear();
    release(c, &s, s.held);
  }

  // complete gRPC messages of the request bytes; false if the stream was failed
  bool messages(Conn& c, Stream& s) {
    for (;;) {
      if (s.rbuf.size() < 5) return true;
      const u8* b = reinterpret_cast<const u8*>(s.rbuf.data());
      const u32 n = be32(b + 1);
      if (b[0] != 0) {  // compressed: no grpc-encoding is negotiated
        fail(c, s, 12, "compressed requests are not supported");
        return false;
      }
      if (n > (4u << 20)) {
        fail(c, s, 8, "request too large");  // RESOURCE_EXHAUSTED
        return false;
      }
      if (s.rbuf.size() < 5 + size_t(n)) return true;
      if (s.requests.size() >= opt.max_queued_requests) {  // requests faster than they are answered
        fail(c, s, 8, "too many queued requests");
        return false;
      }
      s.requests.push_back(s.rbuf.substr(5, n));
      s.rbuf.erase(0, 5 + size_t(n));
    }
  }

  // start the stream's next job / finish it
  void advance(Loop& L, Conn& c, Stream& s) {
    if (s.trailers_queued || s.inflight) return;
    if (s.kind == Kind::kUnknown) return;
    if (s.kind == Kind::kSlow) {
      if (!s.remote_closed) return;
      std::string req = s.requests.empty() ? std::string() : s.requests.front();
      s.requests.clear();
      release(c, &s, s.held);
      s.inflight = true;
      n_slow.fetch_add(1);
      const u64 cid = c.id;
      const u32 sid = s.id;
      const std::string method = s.method, peer = c.peer;
      pool_post(slows, [this, &L, cid, sid, method, req, peer] {
        Reply r;
        try {
          if (slow) r = slow(method, req, peer);
          else r.status = 12;
        } catch (const std::exception& e) {
          r.status = 13;  // INTERNAL
          r.message = e.what();
        }
        auto rp = std::make_shared<Reply>(std::move(r));
        post(L, [this, &L, cid, sid, rp] {
          Conn* cc = find(L, cid);
          if (!cc) return;
          auto it = cc->streams.find(sid);
          if (it == cc->streams.end()) return;
          Stream& st = it->second;
          st.inflight = false;
          if (rp->status == 0)
            for (auto& m : rp->msgs) {
              std::string w(5, '\0');
              const u32 n = u32(m.size());
              w[1] = char(n >> 24), w[2] = char(n >> 16), w[3] = char(n >> 8), w[4] = char(n);
              respond(*cc, st, make_msg(w + m));
            }
          finish(*cc, st, rp->status, rp->message);
          pump(L, *cc);
        });
      });
      return;
    }
    // VideoLatestImage: one response per request, in order
    if (s.requests.empty()) {
      if (s.remote_closed) finish(c, s, 0, "");
      return;
    }
    if (now_ms_mono() - s.t0_ms > opt.stream_deadline_ms) {
      n_deadline.fetch_add(1);
      fail(c, s, 4, "stream deadline exceeded");  // DEADLINE_EXCEEDED
      return;
    }
    std::string dev;
    bool kfo = false;
    const std::string req = std::move(s.requests.front());
    s.requests.pop_front();
    release(c, &s, req.size() + 5);
    if (!parse_frame_request(req, dev, kfo)) {
      fail(c, s, 13, "bad VideoFrameRequest");
      return;
    }
    s.inflight = true;
    if (!s.cancel) s.cancel = std::make_shared<std::atomic<bool>>(false);
    const u64 cid = c.id;
    const u32 sid = s.id;
    const std::string key = c.peer + '\n' + dev;
    const i64 t0 = now_ms_mono();
    const i64 deadline = s.t0_ms + opt.stream_deadline_ms;
    std::shared_ptr<std::atomic<bool>> cancel = s.cancel;
    pool_post(waiters, [this, &L, cid, sid, dev, kfo, key, t0, deadline, cancel] {
      if (cancel->load(std::memory_order_acquire)) return;  // reset while queued: nothing to answer
      Buf msg = frame_for(dev, kfo, key, deadline, cancel.get());
      if (cancel->load(std::memory_order_acquire)) return;
      record_latency(float(now_ms_mono() - t0));
      post(L, [this, &L, cid, sid, msg] {
        Conn* cc = find(L, cid);
        if (!cc) return;
        auto it = cc->streams.find(sid);
        if (it == cc->streams.end()) return;
        Stream& st = it->second;
        st.inflight = false;
        respond(*cc, st, msg);
        advance(L, *cc, st);
        pump(L, *cc);
      });
    });
  }

  // Output still pointing into a bus slot whose lease is about to lapse (the owner may then rewrite
  // it): the oldest chunks of the connection and of every stream.
  static bool stale_lease(const Conn& c, i64 now) {
    auto old = [&](const Chunk& k) { return k.lease_ms > 0 && now - k.lease_ms > bus::kLeaseSendMs; };
    int n = 0;
    for (auto it = c.out.begin(); it != c.out.end() && n < 8; ++it, ++n)
      if (old(*it)) return true;
    for (const auto& [sid, s] : c.streams)
      if (!s.pending.empty() && old(s.pending.front())) return true;
    return false;
  }

  // Streams past their deadline with no job running end with DEADLINE_EXCEEDED (the reference's
  // 15 s context on the whole stream, grpc_api.go:135-137), whether or not requests arrive.
  void sweep(Loop& L) {
    const i64 now = now_ms_mono();
    std::vector<std::shared_ptr<Conn>> cs;
    cs.reserve(L.conns.size());
    for (auto& [fd, cp] : L.conns) cs.push_back(cp);
    for (auto& cp : cs) {
      Conn& c = *cp;
      if (c.fd < 0) continue;
      if (stale_lease(c, now)) {  // leased bytes unsent for kLeaseSendMs: a client that does not read
        n_slow_readers.fetch_add(1);
        close_conn(L, c);
        continue;
      }
      bool any = false;
      for (auto& [sid, s] : c.streams)
        if (!s.inflight && !s.trailers_queued && now - s.t0_ms > opt.stream_deadline_ms) {
          n_deadline.fetch_add(1);
          fail(c, s, 4, "stream deadline exceeded");
          any = true;
        }
      if (any) pump(L, c);
    }
  }

  // ------------------------------------------------------------------ frames
  i64 cursor(const std::string& key) {
    std::lock_guard<std::mutex> g(cur_mu);
    auto it = cursors.find(key);
    return it == cursors.end() ? 0 : it->second.first;
  }
  void set_cursor(const std::string& key, i64 seq) {
    std::lock_guard<std::mutex> g(cur_mu);
    auto it = cursors.find(key);
    if (it != cursors.end()) {
      it->second.first = seq;
      lru.splice(lru.end(), lru, it->second.second);
      return;
    }
    lru.push_back(key);
    cursors[key] = {seq, std::prev(lru.end())};
    while (cursors.size() > opt.max_cursors) {
      cursors.erase(lru.front());
      lru.pop_front();
    }
  }

  // The newest bus frame of `dev` with seq > the caller's cursor (waiting up to 3 x 1 s), as one
  // gRPC message (5-byte prefix + serialized VideoFrame) shared by every client of the camera;
  // the empty message when none arrives.
  // Ends early (the empty message) when `cancel` is set: the client reset the stream.
  Buf frame_for(const std::string& dev, bool kfo, const std::string& key, i64 deadline_ms,
                const std::atomic<bool>* cancel) {
    const i64 after = cursor(key);
    for (int attempt = 0; attempt < opt.wait_attempts && !stop_.load(); ++attempt) {
      if (cancel->load(std::memory_order_acquire) || now_ms_mono() >= deadline_ms) break;
      bus::Reader::Ticket t;
      const int block = int(std::max<i64>(0, std::min<i64>(opt.wait_block_ms, deadline_ms - now_ms_mono())));
      if (reader.wait(dev, after, block, kfo ? 1 : 0, &t, true, cancel)) {
        const i64 ns = reader.newest_seq(t);
        {
          std::unique_lock<std::mutex> g(cache_mu);
          Cached& e = cache[dev];
          // another waiter is copying this frame: take its copy (bounded: a copy is a memcpy)
          cache_cv.wait_for(g, std::chrono::milliseconds(200), [&] { return e.copying != ns || e.seq >= ns; });
          // (a cached leased frame is reused only well inside its lease)
          const bool fresh = !e.msg || !e.msg->lease_ms || now_ms_mono() - e.msg->lease_ms < bus::kLeaseSendMs / 2;
          if (e.seq >= ns && e.seq > after && e.msg && fresh) {
            const i64 s = e.seq;
            Buf b = e.msg;
            g.unlock();
            set_cursor(key, s);
            n_frames.fetch_add(1);
            return b;
          }
          e.copying = ns;
        }
        i64 seq = 0;
        Buf b;
        if (opt.zero_copy) {  // a lease: DATA frames point into the bus slot, no copy
          if (auto l = reader.lease(t)) {
            const size_t n = l->len;
            auto pre = std::make_shared<const std::string>(
                std::string{'\0', char(n >> 24), char(n >> 16), char(n >> 8), char(n)});
            auto m = std::make_shared<Msg>();
            m->parts.push_back(Chunk{pre, pre->data(), 5, 0});
            m->parts.push_back(Chunk{l, reinterpret_cast<const char*>(l->data), n, l->taken_ms});
            m->size = 5 + n;
            m->lease_ms = l->taken_ms;
            seq = l->seq;
            b = m;
            n_leased.fetch_add(1);
          }
        } else {
          auto m = std::make_shared<std::string>(t.cap + 5, '\0');
          const size_t n = reader.copy(t, reinterpret_cast<u8*>(&(*m)[5]), t.cap, &seq);
          if (n > 0) {
            m->resize(n + 5);
            (*m)[1] = char(n >> 24), (*m)[2] = char(n >> 16), (*m)[3] = char(n >> 8), (*m)[4] = char(n);
            b = make_msg(std::move(*m));
            n_copies.fetch_add(1);
          }
        }
        {
          std::lock_guard<std::mutex> g(cache_mu);
          Cached& e = cache[dev];
          if (e.copying == ns) e.copying = 0;
          if (b && seq >= e.seq) {
            e.seq = seq;
            e.msg = b;
          }
        }
        cache_cv.notify_all();
        if (b) {
          set_cursor(key, seq);
          n_frames.fetch_add(1);
          return b;
        }
      }
      if (!reader.has(dev)) {  // unknown camera / owner restarting: an empty frame (and its copy goes)
        std::lock_guard<std::mutex> g(cache_mu);
        auto it = cache.find(dev);
        if (it != cache.end() && it->second.copying == 0) cache.erase(it);
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(16));
    }
    n_empty.fetch_add(1);
    return empty_msg;
  }

  void record_latency(float ms) {
    std::lock_guard<std::mutex> g(lat_mu);
    if (lat.size() < 8192) lat.push_back(ms);
    else lat[lat_next++ % lat.size()] = ms;
  }
};

Server::Server(const ServerOptions& o, SlowHandler slow) : p_(std::make_unique<Impl>(o, std::move(slow))) {
  p_->start();
}

Server::~Server() { stop(); }

int Server::port() const { return p_->port; }

void Server::stop() { p_->shutdown(); }

std::vector<float> Server::take_latencies() {
  std::lock_guard<std::mutex> g(p_->lat_mu);
  std::vector<float> v;
  v.swap(p_->lat);
  p_->lat_next = 0;
  return v;
}

ServerStats Server::stats() const {
  ServerStats s;
  s.connections = p_->n_conn.load();
  s.connections_open = p_->n_open.load();
  s.streams = p_->n_streams.load();
  s.frames_served = p_->n_frames.load();
  s.empty_frames = p_->n_empty.load();
  s.bytes_sent = p_->n_bytes.load();
  s.slow_calls = p_->n_slow.load();
  s.frame_copies = p_->n_copies.load();
  s.protocol_errors = p_->n_proto.load();
  s.goaways = p_->n_goaway.load();
  s.refused_streams = p_->n_refused.load();
  s.cancelled_waits = p_->n_cancelled.load();
  s.deadline_streams = p_->n_deadline.load();
  s.zero_copy_frames = p_->n_leased.load();
  s.slow_readers = p_->n_slow_readers.load();
  std::vector<float> v;
  {
    std::lock_guard<std::mutex> g(p_->lat_mu);
    v = p_->lat;
  }
  if (!v.empty()) {
    std::sort(v.begin(), v.end());
    s.p50_ms = v[v.size() / 2];
    s.p99_ms = v[std::min(v.size() - 1, v.size() * 99 / 100)];
  }
  return s;
}

}  // namespace vep::rpc
