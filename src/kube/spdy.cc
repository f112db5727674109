#include "kube/spdy.h"

#include <zlib.h>

#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "core/log.h"
#include "platform/platform.h"

namespace ds {
namespace kube {

// ---------------------------------------------------------------- dictionary

const std::string& spdy_dictionary() {
  // SPDY/3 §2.6.10.1: length-prefixed common header names and values, then common strings.
  static const std::string dict = [] {
    static const char* kNames[] = {
        "options", "head", "post", "put", "delete", "trace", "accept", "accept-charset", "accept-encoding",
        "accept-language", "accept-ranges", "age", "allow", "authorization", "cache-control", "connection",
        "content-base", "content-encoding", "content-language", "content-length", "content-location",
        "content-md5", "content-range", "content-type", "date", "etag", "expect", "expires", "from", "host",
        "if-match", "if-modified-since", "if-none-match", "if-range", "if-unmodified-since", "last-modified",
        "location", "max-forwards", "pragma", "proxy-authenticate", "proxy-authorization", "range", "referer",
        "retry-after", "server", "te", "trailer", "transfer-encoding", "upgrade", "user-agent", "vary", "via",
        "warning", "www-authenticate", "method", "get", "status", "200 OK", "version", "HTTP/1.1", "url",
        "public", "set-cookie", "keep-alive", "origin"};
    std::string d;
    for (const char* n : kNames) d += spdy::u32((uint32_t)std::strlen(n)) + n;
    d += "100101201202205206300302303304305306307402405406407408409410411412413414415416417502504505"
         "203 Non-Authoritative Information204 No Content301 Moved Permanently400 Bad Request401 Unauthorized"
         "403 Forbidden404 Not Found500 Internal Server Error501 Not Implemented503 Service Unavailable"
         "Jan Feb Mar Apr May Jun Jul Aug Sept Oct Nov Dec 00:00:00 Mon, Tue, Wed, Thu, Fri, Sat, Sun, GMT"
         "chunked,text/html,image/png,image/jpg,image/gif,application/xml,application/xhtml+xml,text/plain,"
         "text/javascript,publicprivatemax-age=gzip,deflate,sdchcharset=utf-8charset=iso-8859-1,utf-,*,enq=0.";
    return d;
  }();
  return dict;
}

// ---------------------------------------------------------------- frames

namespace spdy {

std::string u32(uint32_t v) {
  std::string s(4, '\0');
  s[0] = (char)(v >> 24);
  s[1] = (char)(v >> 16);
  s[2] = (char)(v >> 8);
  s[3] = (char)v;
  return s;
}

uint32_t get_u32(const std::string& s, size_t off) {
  const unsigned char* p = (const unsigned char*)s.data() + off;
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

std::string control_frame(uint16_t type, uint8_t flags, const std::string& body) {
  std::string f;
  f.reserve(8 + body.size());
  f += (char)(0x80 | (kVersion >> 8));
  f += (char)(kVersion & 0xff);
  f += (char)(type >> 8);
  f += (char)(type & 0xff);
  uint32_t len = (uint32_t)body.size();
  f += (char)flags;
  f += (char)(len >> 16);
  f += (char)(len >> 8);
  f += (char)len;
  f += body;
  return f;
}

std::string data_frame(uint32_t stream_id, uint8_t flags, const std::string& data) {
  std::string f = u32(stream_id & 0x7fffffff);
  uint32_t len = (uint32_t)data.size();
  f += (char)flags;
  f += (char)(len >> 16);
  f += (char)(len >> 8);
  f += (char)len;
  f += data;
  return f;
}

bool parse(std::string* buf, Frame* f) {
  if (buf->size() < 8) return false;
  const unsigned char* p = (const unsigned char*)buf->data();
  size_t len = ((size_t)p[5] << 16) | ((size_t)p[6] << 8) | p[7];
  if (buf->size() < 8 + len) return false;
  f->control = (p[0] & 0x80) != 0;
  f->flags = p[4];
  if (f->control) {
    f->type = (uint16_t)((p[2] << 8) | p[3]);
    f->stream_id = 0;
  } else {
    f->type = 0;
    f->stream_id = get_u32(*buf, 0) & 0x7fffffff;
  }
  f->body = buf->substr(8, len);
  buf->erase(0, 8 + len);
  return true;
}

}  // namespace spdy

// ---------------------------------------------------------------- header blocks

struct SpdyHeaderCodec::Impl {
  z_stream def{};
  z_stream inf{};
  bool def_ok = false, inf_ok = false;
};

SpdyHeaderCodec::SpdyHeaderCodec() : impl_(std::make_unique<Impl>()) {
  const std::string& d = spdy_dictionary();
  if (deflateInit(&impl_->def, Z_DEFAULT_COMPRESSION) == Z_OK) {
    impl_->def_ok = deflateSetDictionary(&impl_->def, (const Bytef*)d.data(), (uInt)d.size()) == Z_OK;
  }
  impl_->inf_ok = inflateInit(&impl_->inf) == Z_OK;
}

SpdyHeaderCodec::~SpdyHeaderCodec() {
  deflateEnd(&impl_->def);
  inflateEnd(&impl_->inf);
}

std::string SpdyHeaderCodec::compress(const SpdyHeaders& h) {
  std::string raw = spdy::u32((uint32_t)h.size());
  for (auto& kv : h) raw += spdy::u32((uint32_t)kv.first.size()) + kv.first + spdy::u32((uint32_t)kv.second.size()) + kv.second;
  std::string out;
  if (!impl_->def_ok) return out;
  z_stream& z = impl_->def;
  z.next_in = (Bytef*)raw.data();
  z.avail_in = (uInt)raw.size();
  char buf[4096];
  do {
    z.next_out = (Bytef*)buf;
    z.avail_out = sizeof(buf);
    deflate(&z, Z_SYNC_FLUSH);
    out.append(buf, sizeof(buf) - z.avail_out);
  } while (z.avail_out == 0);
  return out;
}

bool SpdyHeaderCodec::decompress(const std::string& block, SpdyHeaders* out) {
  if (!impl_->inf_ok) return false;
  z_stream& z = impl_->inf;
  z.next_in = (Bytef*)block.data();
  z.avail_in = (uInt)block.size();
  std::string raw;
  char buf[4096];
  while (true) {
    z.next_out = (Bytef*)buf;
    z.avail_out = sizeof(buf);
    int r = inflate(&z, Z_SYNC_FLUSH);
    if (r == Z_NEED_DICT) {
      const std::string& d = spdy_dictionary();
      if (inflateSetDictionary(&z, (const Bytef*)d.data(), (uInt)d.size()) != Z_OK) return false;
      continue;
    }
    if (r != Z_OK && r != Z_BUF_ERROR && r != Z_STREAM_END) return false;
    raw.append(buf, sizeof(buf) - z.avail_out);
    if (z.avail_in == 0 && z.avail_out != 0) break;
    if (r == Z_BUF_ERROR && z.avail_in == 0) break;
  }
  out->clear();
  if (raw.size() < 4) return raw.empty();
  uint32_t n = spdy::get_u32(raw, 0);
  size_t off = 4;
  for (uint32_t i = 0; i < n; ++i) {
    if (off + 4 > raw.size()) return false;
    uint32_t nl = spdy::get_u32(raw, off);
    off += 4;
    if (off + nl + 4 > raw.size()) return false;
    std::string name = raw.substr(off, nl);
    off += nl;
    uint32_t vl = spdy::get_u32(raw, off);
    off += 4;
    if (off + vl > raw.size()) return false;
    out->emplace_back(name, raw.substr(off, vl));
    off += vl;
  }
  return true;
}

// ---------------------------------------------------------------- mailbox

namespace {
// a spilled event: end:u8 channel:u32 reset_len:u32 data_len:u32 reset data
constexpr size_t kSpillHeader = 13;

bool pwrite_all(int fd, const char* p, size_t n, uint64_t off) {
  while (n) {
    ssize_t w = ::pwrite(fd, p, n, (off_t)off);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    p += w;
    n -= (size_t)w;
    off += (uint64_t)w;
  }
  return true;
}

bool pread_all(int fd, char* p, size_t n, uint64_t off) {
  while (n) {
    ssize_t r = ::pread(fd, p, n, (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
    off += (uint64_t)r;
  }
  return true;
}
}  // namespace

SpdyMailbox::~SpdyMailbox() {
  if (spill_fd_ >= 0) ::close(spill_fd_);
}

bool SpdyMailbox::spill(const Event& e) {
  if (spill_broken_) return false;
  if (spill_fd_ < 0) {
    std::string dir = spill_dir;
    if (dir.empty()) {
      const char* t = std::getenv("TMPDIR");
      dir = t && *t ? t : "/tmp";
    }
    spill_fd_ = plat::open_unlinked_tmp(dir);
    if (spill_fd_ < 0) {
      spill_broken_ = true;
      return false;
    }
  }
  std::string rec(kSpillHeader, '\0');
  rec[0] = e.end ? 1 : 0;
  auto put = [&](size_t at, uint32_t v) {
    for (int i = 0; i < 4; ++i) rec[at + i] = (char)(v >> (24 - 8 * i));
  };
  put(1, (uint32_t)e.channel);
  put(5, (uint32_t)e.reset.size());
  put(9, (uint32_t)e.data.size());
  rec += e.reset;
  rec += e.data;
  if (!pwrite_all(spill_fd_, rec.data(), rec.size(), spill_w_)) {
    spill_broken_ = spill_events_ == 0;  // (with events on disk the file stays in use)
    return false;
  }
  spill_w_ += rec.size();
  ++spill_events_;
  return true;
}

bool SpdyMailbox::unspill(Event* e) {
  char h[kSpillHeader];
  if (!pread_all(spill_fd_, h, sizeof(h), spill_r_)) return false;
  auto get = [&](size_t at) {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v = (v << 8) | (unsigned char)h[at + i];
    return v;
  };
  e->end = h[0] != 0;
  e->channel = (int)get(1);
  const uint32_t rl = get(5), dl = get(9);
  std::string body(rl + (size_t)dl, '\0');
  if (!body.empty() && !pread_all(spill_fd_, &body[0], body.size(), spill_r_ + kSpillHeader)) return false;
  e->reset = body.substr(0, rl);
  e->data = body.substr(rl);
  spill_r_ += kSpillHeader + body.size();
  if (--spill_events_ == 0) {  // drained: start the file over
    if (::ftruncate(spill_fd_, 0) != 0) spill_broken_ = true;
    spill_r_ = spill_w_ = 0;
  }
  return true;
}

void SpdyMailbox::push(Event e) {
  {
    std::unique_lock<std::mutex> lk(mu);
    if (closed) return;
    while (true) {
      if (closed) return;
      // in memory while there is room and nothing waits on disk (so the order is kept)
      if (spill_events_ == 0 && (e.data.empty() || bytes < cap)) {
        bytes += e.data.size();
        q.push_back(std::move(e));
        break;
      }
      if (spilled() + e.data.size() <= spill_cap && spill(e)) break;
      cv.wait(lk);  // the disk budget is spent, or there is no spill file: wait for the consumer
    }
  }
  cv.notify_all();
}

bool SpdyMailbox::pop(Event* e, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu);
  auto ready = [this] { return !q.empty() || spill_events_ > 0 || closed; };
  if (timeout_ms < 0)
    cv.wait(lk, ready);
  else if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready))
    return false;
  if (closed) return false;
  if (!q.empty()) {
    *e = std::move(q.front());
    q.pop_front();
    bytes -= e->data.size();
  } else if (!unspill(e)) {  // the spill file failed under us: the stream cannot go on
    spill_events_ = 0;
    spill_r_ = spill_w_ = 0;
    spill_broken_ = true;
    *e = Event{0, "", true, "spill"};
  }
  lk.unlock();
  cv.notify_all();  // a push waiting for room
  return true;
}

void SpdyMailbox::close() {
  {
    std::lock_guard<std::mutex> g(mu);
    closed = true;
    q.clear();
    bytes = 0;
    spill_events_ = 0;
    spill_r_ = spill_w_ = 0;
    if (spill_fd_ >= 0) ::close(spill_fd_);
    spill_fd_ = -1;
  }
  cv.notify_all();
}

// ---------------------------------------------------------------- session

SpdySession::SpdySession(std::unique_ptr<net::WebSocket> ws) : ws_(std::move(ws)) {
  reader_ = std::thread([this] { reader(); });
}

SpdySession::~SpdySession() {
  close();
  if (reader_.joinable()) reader_.join();
}

bool SpdySession::usable() const {
  std::lock_guard<std::mutex> g(mu_);
  return !dead_ && !goaway_;
}

bool SpdySession::write_frame(const std::string& frame) {
  // (callers hold wmu_ when header-block order matters)
  if (!ws_->send(frame)) {
    end_all("tunnel closed");
    return false;
  }
  return true;
}

std::shared_ptr<SpdySession::Stream> SpdySession::open(const SpdyHeaders& headers, std::shared_ptr<SpdyMailbox> box,
                                                       int channel, bool fin) {
  auto s = std::make_shared<Stream>();
  s->box = std::move(box);
  s->channel = channel;
  s->local_fin = fin;
  std::lock_guard<std::mutex> w(wmu_);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_ || goaway_) throw net::NetError(dead_ ? "port-forward tunnel closed" : "port-forward tunnel going away");
    s->id = next_id_;
    next_id_ += 2;
    streams_[s->id] = s;
  }
  // SYN_STREAM: stream id, associated stream id, priority (3 bits) + unused + slot, headers
  std::string body = spdy::u32(s->id) + spdy::u32(0) + std::string(2, '\0') + out_codec_.compress(headers);
  if (!write_frame(spdy::control_frame(spdy::SynStream, fin ? spdy::kFlagFin : 0, body)))
    throw net::NetError("port-forward tunnel closed");
  return s;
}

bool SpdySession::send(const std::shared_ptr<Stream>& s, const std::string& data, bool fin) {
  std::lock_guard<std::mutex> w(wmu_);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_) return false;
    if (s->local_fin) return !fin && data.empty();
    if (fin) s->local_fin = true;
  }
  // frames of at most 64 KiB - 1 (the 24-bit length allows more; peers buffer per frame)
  size_t off = 0;
  do {
    size_t n = std::min<size_t>(data.size() - off, 65535);
    bool last = off + n >= data.size();
    if (!write_frame(spdy::data_frame(s->id, last && fin ? spdy::kFlagFin : 0, data.substr(off, n)))) return false;
    off += n;
  } while (off < data.size());
  return true;
}

void SpdySession::consumed(const std::shared_ptr<Stream>& s, size_t n) {
  std::string frames;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_) return;
    s->unacked += n;
    session_unacked_ += n;
    if (s->unacked >= 32768 && !s->remote_end) {
      frames += spdy::control_frame(spdy::WindowUpdate, 0, spdy::u32(s->id) + spdy::u32((uint32_t)s->unacked));
      s->unacked = 0;
    }
    if (session_unacked_ >= 32768) {  // SPDY/3.1 session window: stream id 0
      frames += spdy::control_frame(spdy::WindowUpdate, 0, spdy::u32(0) + spdy::u32((uint32_t)session_unacked_));
      session_unacked_ = 0;
    }
  }
  if (!frames.empty()) {
    std::lock_guard<std::mutex> w(wmu_);
    write_frame(frames);
  }
}

void SpdySession::reset(const std::shared_ptr<Stream>& s, uint32_t status) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_ || !streams_.count(s->id)) return;
    streams_.erase(s->id);
    s->local_fin = true;
  }
  std::lock_guard<std::mutex> w(wmu_);
  write_frame(spdy::control_frame(spdy::RstStream, 0, spdy::u32(s->id) + spdy::u32(status)));
}

void SpdySession::ping() {
  uint32_t id;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_) return;
    id = next_ping_;
    next_ping_ += 2;
    auto now = std::chrono::steady_clock::now();
    // a far end that never answers: what is still unanswered after 5 s will not be, and the map
    // stays small whatever the session's length
    for (auto it = pings_.begin(); it != pings_.end();)
      it = now - it->second > std::chrono::seconds(5) ? pings_.erase(it) : std::next(it);
    pings_[id] = now;
  }
  std::lock_guard<std::mutex> w(wmu_);
  write_frame(spdy::control_frame(spdy::Ping, 0, spdy::u32(id)));
}

size_t SpdySession::pings_in_flight() const {
  std::lock_guard<std::mutex> g(mu_);
  return pings_.size();
}

void SpdySession::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_) return;
  }
  {
    std::lock_guard<std::mutex> w(wmu_);
    uint32_t last = 0;
    ws_->send(spdy::control_frame(spdy::GoAway, 0, spdy::u32(last) + spdy::u32(0)));
  }
  ws_->close();
  end_all("closed");
}

void SpdySession::end_all(const std::string& why) {
  std::vector<std::shared_ptr<Stream>> open;  // streams the peer has not ended
  {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_) return;
    dead_ = true;
    for (auto& kv : streams_)
      if (!kv.second->remote_end) open.push_back(kv.second);
    streams_.clear();
  }
  for (auto& s : open) s->box->push({s->channel, "", true, why});
}

void SpdySession::dispatch_data(uint32_t id, uint8_t flags, std::string data) {
  std::shared_ptr<Stream> s;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = streams_.find(id);
    if (it == streams_.end()) return;  // reset by us, or unknown: dropped
    s = it->second;
    if (flags & spdy::kFlagFin) {
      s->remote_end = true;
      if (s->local_fin) streams_.erase(it);
    }
  }
  if (!data.empty()) s->box->push({s->channel, std::move(data), false, ""});
  if (flags & spdy::kFlagFin) s->box->push({s->channel, "", true, ""});
}

void SpdySession::dispatch_control(uint16_t type, uint8_t flags, const std::string& body) {
  switch (type) {
    case spdy::SynReply:
    case spdy::Headers: {
      SpdyHeaders h;
      in_codec_.decompress(body.size() > 4 ? body.substr(4) : std::string(), &h);  // keeps the zlib stream in step
      if ((flags & spdy::kFlagFin) && body.size() >= 4) dispatch_data(spdy::get_u32(body, 0) & 0x7fffffff, spdy::kFlagFin, "");
      break;
    }
    case spdy::SynStream: {
      // the server opens no streams in port-forward: refuse it (after keeping the zlib state)
      SpdyHeaders h;
      if (body.size() > 10) in_codec_.decompress(body.substr(10), &h);
      if (body.size() >= 4) {
        std::lock_guard<std::mutex> w(wmu_);
        write_frame(spdy::control_frame(spdy::RstStream, 0, spdy::u32(spdy::get_u32(body, 0) & 0x7fffffff) + spdy::u32(3)));
      }
      break;
    }
    case spdy::RstStream: {
      if (body.size() < 8) break;
      uint32_t id = spdy::get_u32(body, 0) & 0x7fffffff;
      uint32_t status = spdy::get_u32(body, 4);
      std::shared_ptr<Stream> s;
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = streams_.find(id);
        if (it == streams_.end()) break;
        s = it->second;
        s->remote_end = true;
        streams_.erase(it);
      }
      s->box->push({s->channel, "", true, "RST_STREAM status " + std::to_string(status)});
      break;
    }
    case spdy::Ping: {
      if (body.size() < 4) break;
      uint32_t id = spdy::get_u32(body, 0);
      if (id & 1) {  // the answer to one of ours (never echoed back: that would loop)
        std::lock_guard<std::mutex> g(mu_);
        auto it = pings_.find(id);
        if (it != pings_.end()) {
          // the smallest seen: a busy peer answers late, the link is never faster than this
          int64_t rtt = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() -
                                                                              it->second).count();
          if (rtt_us_ < 0 || rtt < rtt_us_) rtt_us_ = rtt;
          rtt_samples_++;
          pings_.erase(it);
        }
        break;
      }
      std::lock_guard<std::mutex> w(wmu_);
      write_frame(spdy::control_frame(spdy::Ping, 0, body));
      break;
    }
    case spdy::GoAway: {
      std::lock_guard<std::mutex> g(mu_);
      goaway_ = true;  // streams in flight finish; no new ones
      break;
    }
    default:  // SETTINGS, WINDOW_UPDATE (send windows are not enforced, as in spdystream)
      break;
  }
}

void SpdySession::reader() {
  std::string buf, msg;
  net::WebSocket::Op op;
  while (true) {
    if (!ws_->recv(&msg, &op)) break;
    buf += msg;
    spdy::Frame f;
    while (spdy::parse(&buf, &f)) {
      if (f.control)
        dispatch_control(f.type, f.flags, f.body);
      else
        dispatch_data(f.stream_id, f.flags, std::move(f.body));
    }
  }
  end_all("tunnel closed");
}

}  // namespace kube
}  // namespace ds
