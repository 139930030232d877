// RTP packetization / depacketization for H.264 (RFC 6184) and H.265 (RFC 7798), base64, URLs.
#include <algorithm>

#include "net.h"

namespace vep::net {

void write_rtp_header(u8* o, const RtpHeader& h) {
  o[0] = 0x80;  // V=2
  o[1] = u8((h.marker ? 0x80 : 0) | (h.pt & 0x7f));
  o[2] = u8(h.seq >> 8);
  o[3] = u8(h.seq);
  o[4] = u8(h.ts >> 24);
  o[5] = u8(h.ts >> 16);
  o[6] = u8(h.ts >> 8);
  o[7] = u8(h.ts);
  o[8] = u8(h.ssrc >> 24);
  o[9] = u8(h.ssrc >> 16);
  o[10] = u8(h.ssrc >> 8);
  o[11] = u8(h.ssrc);
}

bool parse_rtp(const u8* p, size_t n, RtpHeader& h, const u8** payload, size_t* plen) {
  if (n < kRtpHeader || (p[0] >> 6) != 2) return false;
  const int cc = p[0] & 0x0f;
  const bool ext = p[0] & 0x10, pad = p[0] & 0x20;
  h.marker = p[1] & 0x80;
  h.pt = p[1] & 0x7f;
  h.seq = u16(p[2] << 8 | p[3]);
  h.ts = u32(p[4]) << 24 | u32(p[5]) << 16 | u32(p[6]) << 8 | p[7];
  h.ssrc = u32(p[8]) << 24 | u32(p[9]) << 16 | u32(p[10]) << 8 | p[11];
  size_t off = kRtpHeader + size_t(cc) * 4;
  if (off > n) return false;
  if (ext) {
    if (off + 4 > n) return false;
    size_t el = (size_t(p[off + 2]) << 8 | p[off + 3]) * 4;
    off += 4 + el;
    if (off > n) return false;
  }
  size_t end = n;
  if (pad) {
    u8 pl = p[n - 1];
    if (pl == 0 || pl > end - off) return false;
    end -= pl;
  }
  *payload = p + off;
  *plen = end - off;
  return true;
}

void packetize_nal(Codec c, const u8* nal, size_t n, size_t mtu, std::vector<std::vector<u8>>& out) {
  const size_t hdr = (c == Codec::kH264) ? 1 : 2;
  VEP_CHECK(n > hdr && mtu > hdr + 8, "bad NAL / mtu for packetization");
  if (n <= mtu) {
    out.emplace_back(nal, nal + n);
    return;
  }
  const size_t fu_hdr = hdr + 1;  // FU indicator(+payload header) + FU header
  const size_t chunk = mtu - fu_hdr;
  size_t pos = hdr;
  while (pos < n) {
    size_t len = std::min(chunk, n - pos);
    std::vector<u8> pk;
    pk.reserve(len + fu_hdr);
    const bool start = (pos == hdr), end = (pos + len == n);
    if (c == Codec::kH264) {
      pk.push_back(u8((nal[0] & 0xE0) | 28));
      pk.push_back(u8((start ? 0x80 : 0) | (end ? 0x40 : 0) | (nal[0] & 0x1F)));
    } else {
      const int type = (nal[0] >> 1) & 0x3F;
      pk.push_back(u8((nal[0] & 0x81) | (49 << 1)));
      pk.push_back(nal[1]);
      pk.push_back(u8((start ? 0x80 : 0) | (end ? 0x40 : 0) | type));
    }
    pk.insert(pk.end(), nal + pos, nal + pos + len);
    out.push_back(std::move(pk));
    pos += len;
  }
}

std::vector<u8> aggregate_nals(Codec c, const std::vector<std::vector<u8>>& nals) {
  std::vector<u8> pk;
  if (c == Codec::kH264) {
    u8 nri = 0;
    for (auto& n : nals) nri = std::max<u8>(nri, n[0] & 0x60);
    pk.push_back(u8(nri | 24));
  } else {
    pk.push_back(u8(48 << 1));
    pk.push_back(1);  // LayerId 0, TID 1
  }
  for (auto& n : nals) {
    VEP_CHECK(n.size() < 65536, "NAL too large to aggregate");
    pk.push_back(u8(n.size() >> 8));
    pk.push_back(u8(n.size()));
    pk.insert(pk.end(), n.begin(), n.end());
  }
  return pk;
}

bool is_keyframe_nal(Codec c, const u8* nal, size_t n) {
  if (n < 1) return false;
  if (c == Codec::kH264) return (nal[0] & 0x1f) == 5;
  int t = (nal[0] >> 1) & 0x3f;
  return t >= 16 && t <= 23;  // IRAP (BLA/IDR/CRA)
}

void Depacketizer::add_nal(const u8* p, size_t n) {
  if (n == 0) return;
  if (!cur_) cur_ = std::make_shared<AccessUnit>();
  cur_->codec = codec_;
  cur_->add_nal(p, n);
  if (is_keyframe_nal(codec_, p, n)) cur_->keyframe = true;
}

void Depacketizer::finish(std::vector<AuPtr>& out) {
  in_frag_ = false;
  frag_.clear();
  if (!cur_ || cur_->nals.empty()) {
    cur_.reset();
    corrupt_ = false;
    return;
  }
  // extended 90 kHz timestamp relative to the first packet of the session
  if (!have_ts_) {
    ts_base_ = cur_ts_;
    ts_ext_ = 0;
    last_ts_ = cur_ts_;
    have_ts_ = true;
  } else {
    ts_ext_ += i64(i32(cur_ts_ - last_ts_));
    last_ts_ = cur_ts_;
  }
  i64 pts = ts_ext_;
  if (clock_ != 90000) pts = pts * 90000 / i64(clock_);
  cur_->pts = cur_->dts = pts;
  cur_->corrupt = corrupt_;
  cur_->arrival_ms = now_ms();
  cur_->seq = seq_counter_++;
  cur_->pin();  // into device-accessible pinned memory when a GPU worker enabled the pool
  out.push_back(cur_);
  cur_.reset();
  corrupt_ = false;
  ++aus_;
}

void Depacketizer::flush(std::vector<AuPtr>& out) { finish(out); }

void Depacketizer::push(const RtpHeader& h, const u8* p, size_t n, std::vector<AuPtr>& out) {
  if (have_seq_) {
    u16 expect = u16(last_seq_ + 1);
    if (h.seq != expect) {
      u16 gap = u16(h.seq - expect);
      if (gap < 0x8000) {  // forward gap = loss
        lost_ += gap;
        corrupt_ = true;
        if (in_frag_) frag_bad_ = true;
      } else {
        return;  // late / duplicate packet
      }
    }
  }
  have_seq_ = true;
  last_seq_ = h.seq;
  if (cur_ && !cur_->nals.empty() && h.ts != cur_ts_) finish(out);
  cur_ts_ = h.ts;
  if (n == 0) return;
  if (codec_ == Codec::kH264) {
    const int t = p[0] & 0x1f;
    if (t >= 1 && t <= 23) {
      add_nal(p, n);
    } else if (t == 24) {  // STAP-A
      size_t off = 1;
      while (off + 2 <= n) {
        size_t len = size_t(p[off]) << 8 | p[off + 1];
        off += 2;
        if (off + len > n) { corrupt_ = true; break; }
        add_nal(p + off, len);
        off += len;
      }
    } else if (t == 28 && n >= 2) {  // FU-A
      const bool s = p[1] & 0x80, e = p[1] & 0x40;
      if (s) {
        frag_.clear();
        frag_.push_back(u8((p[0] & 0xE0) | (p[1] & 0x1F)));
        in_frag_ = true;
        frag_bad_ = false;
      } else if (!in_frag_) {
        corrupt_ = true;
        return;
      }
      frag_.insert(frag_.end(), p + 2, p + n);
      if (e) {
        if (!frag_bad_) add_nal(frag_.data(), frag_.size());
        in_frag_ = false;
        frag_.clear();
      }
    } else {
      corrupt_ = true;  // STAP-B / MTAP / FU-B are not used by RTSP cameras
    }
  } else {
    if (n < 2) return;
    const int t = (p[0] >> 1) & 0x3f;
    if (t == 48) {  // AP
      size_t off = 2;
      while (off + 2 <= n) {
        size_t len = size_t(p[off]) << 8 | p[off + 1];
        off += 2;
        if (off + len > n) { corrupt_ = true; break; }
        add_nal(p + off, len);
        off += len;
      }
    } else if (t == 49 && n >= 3) {  // FU
      const bool s = p[2] & 0x80, e = p[2] & 0x40;
      if (s) {
        frag_.clear();
        frag_.push_back(u8((p[0] & 0x81) | ((p[2] & 0x3f) << 1)));
        frag_.push_back(p[1]);
        in_frag_ = true;
        frag_bad_ = false;
      } else if (!in_frag_) {
        corrupt_ = true;
        return;
      }
      frag_.insert(frag_.end(), p + 3, p + n);
      if (e) {
        if (!frag_bad_) add_nal(frag_.data(), frag_.size());
        in_frag_ = false;
        frag_.clear();
      }
    } else if (t == 50) {
      // PACI: not used by cameras; ignore
    } else {
      add_nal(p, n);
    }
  }
  if (h.marker) finish(out);
}

// ----------------------------------------------------------------------------------- base64

static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const u8* p, size_t n) {
  std::string s;
  s.reserve((n + 2) / 3 * 4);
  for (size_t i = 0; i < n; i += 3) {
    u32 v = u32(p[i]) << 16 | (i + 1 < n ? u32(p[i + 1]) << 8 : 0) | (i + 2 < n ? p[i + 2] : 0);
    s.push_back(kB64[(v >> 18) & 63]);
    s.push_back(kB64[(v >> 12) & 63]);
    s.push_back(i + 1 < n ? kB64[(v >> 6) & 63] : '=');
    s.push_back(i + 2 < n ? kB64[v & 63] : '=');
  }
  return s;
}

std::vector<u8> base64_decode(const std::string& s) {
  std::vector<u8> out;
  u32 v = 0;
  int bits = 0;
  for (char ch : s) {
    const char* q = std::strchr(kB64, ch);
    if (ch == '=' || !q || ch == 0) continue;
    v = (v << 6) | u32(q - kB64);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back(u8(v >> bits));
    }
  }
  return out;
}

Url parse_url(const std::string& s) {
  Url u;
  size_t p = s.find("://");
  VEP_CHECK(p != std::string::npos, "bad URL (no scheme): " + s);
  u.scheme = s.substr(0, p);
  std::string rest = s.substr(p + 3);
  size_t slash = rest.find('/');
  std::string auth = rest.substr(0, slash);
  u.path = slash == std::string::npos ? "/" : rest.substr(slash);
  size_t at = auth.rfind('@');
  if (at != std::string::npos) {
    std::string cred = auth.substr(0, at);
    auth = auth.substr(at + 1);
    size_t c = cred.find(':');
    u.user = cred.substr(0, c);
    if (c != std::string::npos) u.pass = cred.substr(c + 1);
  }
  size_t colon = auth.rfind(':');
  if (colon != std::string::npos && auth.find(']') == std::string::npos) {
    u.host = auth.substr(0, colon);
    u.port = std::atoi(auth.substr(colon + 1).c_str());
  } else {
    u.host = auth;
  }
  if (u.port == 0) u.port = (u.scheme == "rtmp") ? 1935 : 554;
  return u;
}

}  // namespace vep::net
