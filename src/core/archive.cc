// gzip + tar streams (sync/tar.go, util/tar/tar.go). Kept free of OpenSSL so the static
// in-container helper (src/helper/helper.cc) can link it with only zlib.
#include <fcntl.h>
#include <stdlib.h>
#include <unistd.h>
#include <zlib.h>

#include <cmath>
#include <cstring>
#include <vector>
#include <map>
#include <memory>
#include <stdexcept>

#include "core/codec.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "platform/platform.h"

namespace ds {

// ------------------------------------------------------------------ gzip

GzipWriter::GzipWriter(Sink sink, int level) : sink_(std::move(sink)) {
  z_stream* z = new z_stream();
  std::memset(z, 0, sizeof(*z));
  if (deflateInit2(z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
    delete z;
    throw std::runtime_error("deflateInit2 failed");
  }
  z_ = z;
}

GzipWriter::~GzipWriter() {
  z_stream* z = (z_stream*)z_;
  deflateEnd(z);
  delete z;
}

bool GzipWriter::pump(int flush) {
  z_stream* z = (z_stream*)z_;
  char out[1 << 16];
  while (true) {
    z->next_out = (Bytef*)out;
    z->avail_out = sizeof(out);
    int r = deflate(z, flush);
    if (r == Z_STREAM_ERROR) return false;
    size_t have = sizeof(out) - z->avail_out;
    if (have && !sink_(out, have)) return false;
    if (flush == Z_FINISH) {
      if (r == Z_STREAM_END) return true;
    } else if (z->avail_in == 0 && z->avail_out != 0) {
      return true;
    }
  }
}

bool GzipWriter::write(const char* d, size_t n) {
  z_stream* z = (z_stream*)z_;
  z->next_in = (Bytef*)d;
  z->avail_in = (uInt)n;
  return pump(Z_NO_FLUSH);
}

bool GzipWriter::finish() {
  if (finished_) return true;
  finished_ = true;
  z_stream* z = (z_stream*)z_;
  z->next_in = nullptr;
  z->avail_in = 0;
  return pump(Z_FINISH);
}

GzipReader::GzipReader(Source src) : src_(std::move(src)), in_(1 << 16) {
  z_stream* z = new z_stream();
  std::memset(z, 0, sizeof(*z));
  if (inflateInit2(z, 15 + 32) != Z_OK) {
    delete z;
    throw std::runtime_error("inflateInit2 failed");
  }
  z_ = z;
}

GzipReader::~GzipReader() {
  z_stream* z = (z_stream*)z_;
  inflateEnd(z);
  delete z;
}

ssize_t GzipReader::read(char* out, size_t n) {
  if (n == 0) return 0;
  z_stream* z = (z_stream*)z_;
  if (single_ && stream_end_) return 0;
  z->next_out = (Bytef*)out;
  z->avail_out = (uInt)n;
  while (z->avail_out == n) {
    if (stream_end_) {
      // multi-member mode: another member may follow the one that just ended
      if (z->avail_in == 0) {
        if (eof_) return 0;
        ssize_t r = src_(in_.data(), in_.size());
        if (r < 0) return -1;
        if (r == 0) {
          eof_ = true;
          return 0;
        }
        z->next_in = (Bytef*)in_.data();
        z->avail_in = (uInt)r;
      }
      inflateReset(z);
      stream_end_ = false;
    }
    if (z->avail_in == 0) {
      if (eof_) return -1;  // the member is truncated
      ssize_t r = src_(in_.data(), in_.size());
      if (r < 0) return -1;
      if (r == 0) {
        eof_ = true;
        return -1;
      }
      z->next_in = (Bytef*)in_.data();
      z->avail_in = (uInt)r;
    }
    int r = inflate(z, Z_NO_FLUSH);
    if (r == Z_STREAM_END) {
      stream_end_ = true;
      if (single_) break;  // never pull the source past the member
      continue;
    }
    if (r != Z_OK && r != Z_BUF_ERROR) return -1;
  }
  return (ssize_t)(n - z->avail_out);
}

std::string GzipReader::leftover() const {
  z_stream* z = (z_stream*)z_;
  if (!stream_end_ || z->avail_in == 0) return "";
  return std::string((const char*)z->next_in, z->avail_in);
}

std::string gzip_compress(const std::string& data, int level) {
  std::string out;
  GzipWriter w(string_sink(&out), level);
  w.write(data);
  w.finish();
  return out;
}

// Order-0 entropy of a sample in bits/byte: already-compressed or random payloads (model
// weights, images, archives) sit near 8 and gain nothing from deflate except its cost.
static double sample_entropy(const unsigned char* p, size_t n) {
  if (n == 0) return 0;
  uint32_t hist[256] = {0};
  for (size_t i = 0; i < n; ++i) hist[p[i]]++;
  double h = 0;
  for (uint32_t c : hist) {
    if (!c) continue;
    double q = (double)c / (double)n;
    h -= q * std::log2(q);
  }
  return h;
}

// deflate at level 1 runs ~20 MB/s on random bytes; stored blocks run at memcpy + CRC speed,
// so a tree of model checkpoints is no longer compression-bound.
static const size_t kAdaptiveChunk = 1 << 20, kEntropySample = 1 << 16;
static const uint64_t kMaxMemberInput = 1ull << 30;

AdaptiveGzipWriter::AdaptiveGzipWriter(Sink sink, int level)
    : sink_(std::move(sink)), level_(level), cur_(level), out_(1 << 17) {
  z_stream* z = new z_stream();
  std::memset(z, 0, sizeof(*z));
  if (deflateInit2(z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
    delete z;
    throw std::runtime_error("deflateInit2 failed");
  }
  z_ = z;
  buf_.reserve(kAdaptiveChunk);
}

AdaptiveGzipWriter::~AdaptiveGzipWriter() {
  z_stream* z = (z_stream*)z_;
  deflateEnd(z);
  delete z;
}

bool AdaptiveGzipWriter::drain(int flush) {
  z_stream* z = (z_stream*)z_;
  int r;
  do {
    z->next_out = (Bytef*)out_.data();
    z->avail_out = (uInt)out_.size();
    r = deflate(z, flush);
    if (r == Z_STREAM_ERROR) return false;
    size_t have = out_.size() - z->avail_out;
    if (have && !sink_(out_.data(), have)) return false;
  } while (z->avail_out == 0 || (flush == Z_FINISH && r != Z_STREAM_END));
  return true;
}

// Ends the current gzip member and starts a fresh deflate stream at `level`. Levels are never
// switched inside one stream (deflateParams after >2 GiB of stored blocks crashes zlib 1.2.11),
// and no member holds more than 1 GiB of input: the output is a series of gzip members, which
// gunzip, `tar xz` (GNU and busybox) and GzipReader all read as one stream.
bool AdaptiveGzipWriter::new_member(int level) {
  z_stream* z = (z_stream*)z_;
  if (member_in_ > 0) {
    z->next_in = nullptr;
    z->avail_in = 0;
    if (!drain(Z_FINISH)) return false;
  }
  deflateEnd(z);
  std::memset(z, 0, sizeof(*z));
  if (deflateInit2(z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  cur_ = level;
  member_in_ = 0;
  return true;
}

bool AdaptiveGzipWriter::deflate_chunk(bool last) {
  z_stream* z = (z_stream*)z_;
  if (!buf_.empty()) {
    const unsigned char* p = (const unsigned char*)buf_.data();
    int want = sample_entropy(p, std::min(buf_.size(), kEntropySample)) > 7.5 ? 0 : level_;
    if ((want != cur_ || member_in_ >= kMaxMemberInput) && !new_member(want)) return false;
  }
  z->next_in = (Bytef*)buf_.data();
  z->avail_in = (uInt)buf_.size();
  member_in_ += buf_.size();
  if (!drain(last ? Z_FINISH : Z_NO_FLUSH)) return false;
  buf_.clear();
  return true;
}

bool AdaptiveGzipWriter::write(const char* d, size_t n) {
  if (finished_) return false;
  while (n > 0) {
    size_t take = std::min(n, kAdaptiveChunk - buf_.size());
    buf_.append(d, take);
    d += take;
    n -= take;
    if (buf_.size() == kAdaptiveChunk && !deflate_chunk(false)) return false;
  }
  return true;
}

bool AdaptiveGzipWriter::finish() {
  if (finished_) return true;
  finished_ = true;
  return deflate_chunk(true);
}

std::string gzip_compress_adaptive(const std::string& data, int level) {
  // one gzip member (any `tar xz` / gunzip reads it) whose level follows each chunk's entropy
  std::string out;
  out.reserve(data.size() / 2 + 1024);
  AdaptiveGzipWriter w(string_sink(&out), level);
  w.write(data);
  w.finish();
  return out;
}

std::string gzip_decompress(const std::string& data) {
  std::string out;
  GzipReader r(string_source(&data));
  char buf[1 << 16];
  while (true) {
    ssize_t n = r.read(buf, sizeof(buf));
    if (n < 0) throw std::runtime_error("gzip: invalid data");
    if (n == 0) break;
    out.append(buf, (size_t)n);
  }
  return out;
}

// ------------------------------------------------------------------ sources / sinks

Source fd_source(int fd) {
  return [fd](char* b, size_t n) -> ssize_t { return read_some(fd, b, n); };
}
Sink fd_sink(int fd) {
  return [fd](const char* d, size_t n) { return write_all(fd, d, n); };
}
Sink string_sink(std::string* out) {
  return [out](const char* d, size_t n) {
    out->append(d, n);
    return true;
  };
}
Source string_source(const std::string* in) {
  auto pos = std::make_shared<size_t>(0);
  return [in, pos](char* b, size_t n) -> ssize_t {
    size_t left = in->size() - *pos;
    size_t c = std::min(left, n);
    std::memcpy(b, in->data() + *pos, c);
    *pos += c;
    return (ssize_t)c;
  };
}

Source prefixed_source(std::string prefix, Source rest) {
  auto pre = std::make_shared<std::string>(std::move(prefix));
  auto pos = std::make_shared<size_t>(0);
  return [pre, pos, rest](char* b, size_t n) -> ssize_t {
    if (*pos < pre->size()) {
      size_t c = std::min(n, pre->size() - *pos);
      std::memcpy(b, pre->data() + *pos, c);
      *pos += c;
      return (ssize_t)c;
    }
    return rest(b, n);
  };
}

Source limited_source(Source inner, uint64_t n) {
  auto left = std::make_shared<uint64_t>(n);
  return [inner, left](char* b, size_t k) -> ssize_t {
    if (*left == 0) return 0;
    ssize_t r = inner(b, (size_t)std::min<uint64_t>(k, *left));
    if (r > 0) *left -= (uint64_t)r;
    if (r == 0) return -1;  // the stream ended before the announced length
    return r;
  };
}

// ------------------------------------------------------------------ spill buffer

SpillBuffer::SpillBuffer(size_t mem_limit, std::string dir) : limit_(mem_limit), dir_(std::move(dir)) {
  if (dir_.empty()) {
    const char* t = getenv("TMPDIR");
    dir_ = t && *t ? t : "/tmp";
  }
}

SpillBuffer::~SpillBuffer() {
  if (fd_ >= 0) ::close(fd_);
}

bool SpillBuffer::flush_stage() {
  if (stage_.empty()) return true;
  if (!write_all(fd_, stage_.data(), stage_.size())) return false;
  stage_.clear();
  if (stage_.capacity() > (2u << 20)) std::string().swap(stage_);
  return true;
}

bool SpillBuffer::append(const char* d, size_t n) {
  size_ += n;
  if (fd_ < 0) {
    if (mem_.size() + n <= limit_) {
      mem_.append(d, n);
      return true;
    }
    // unlinked from the start: nothing is left behind whatever way the process ends
    fd_ = plat::open_unlinked_tmp(dir_);
    if (fd_ < 0) return false;
    stage_.swap(mem_);
    std::string().swap(mem_);
  }
  stage_.append(d, n);
  if (stage_.size() >= (1u << 20)) return flush_stage();
  return true;
}

bool SpillBuffer::replay(const Sink& out) {
  const size_t kBlock = 1 << 20;
  if (fd_ < 0) {
    for (size_t off = 0; off < mem_.size(); off += kBlock)
      if (!out(mem_.data() + off, std::min(kBlock, mem_.size() - off))) return false;
    return true;
  }
  if (!flush_stage()) return false;
  std::vector<char> buf(kBlock);
  uint64_t off = 0;
  while (off < size_) {
    ssize_t r = ::pread(fd_, buf.data(), (size_t)std::min<uint64_t>(kBlock, size_ - off), (off_t)off);
    if (r <= 0) return false;
    if (!out(buf.data(), (size_t)r)) return false;
    off += (uint64_t)r;
  }
  return true;
}

std::string SpillBuffer::head(size_t n) {
  if (fd_ < 0) return mem_.substr(0, n);
  if (!flush_stage()) return "";
  std::string out(std::min<uint64_t>(n, size_), '\0');
  ssize_t r = ::pread(fd_, &out[0], out.size(), 0);
  out.resize(r > 0 ? (size_t)r : 0);
  return out;
}

// ------------------------------------------------------------------ tar

static void put_octal(char* dst, size_t len, uint64_t v) {
  // len includes trailing NUL
  std::string s = strfmt("%0*llo", (int)(len - 1), (unsigned long long)v);
  if (s.size() > len - 1) {
    // base-256 encoding for large values
    std::memset(dst, 0, len);
    dst[0] = (char)0x80;
    for (size_t i = len - 1; i > 0; --i) {
      dst[i] = (char)(v & 0xFF);
      v >>= 8;
    }
    return;
  }
  std::memcpy(dst, s.data(), s.size());
  dst[len - 1] = 0;
}

static uint64_t get_octal(const char* p, size_t len) {
  if ((unsigned char)p[0] & 0x80) {
    uint64_t v = 0;
    for (size_t i = 1; i < len; ++i) v = (v << 8) | (unsigned char)p[i];
    return v;
  }
  uint64_t v = 0;
  size_t i = 0;
  while (i < len && (p[i] == ' ' || p[i] == 0)) ++i;
  for (; i < len && p[i] >= '0' && p[i] <= '7'; ++i) v = v * 8 + (uint64_t)(p[i] - '0');
  return v;
}

bool TarWriter::raw(const char* d, size_t n) { return sink_(d, n); }

static void fill_header(char* h, const std::string& name, const TarEntry& e, char type, int64_t size) {
  std::memset(h, 0, 512);
  std::memcpy(h, name.data(), std::min<size_t>(name.size(), 100));
  put_octal(h + 100, 8, e.mode & 07777);
  put_octal(h + 108, 8, e.uid);
  put_octal(h + 116, 8, e.gid);
  put_octal(h + 124, 12, (uint64_t)size);
  put_octal(h + 136, 12, (uint64_t)(e.mtime < 0 ? 0 : e.mtime));
  h[156] = type;
  if (!e.linkname.empty()) std::memcpy(h + 157, e.linkname.data(), std::min<size_t>(e.linkname.size(), 100));
  std::memcpy(h + 257, "ustar\0", 6);
  std::memcpy(h + 263, "00", 2);
  std::memcpy(h + 265, e.uname.data(), std::min<size_t>(e.uname.size(), 31));
  std::memcpy(h + 297, e.gname.data(), std::min<size_t>(e.gname.size(), 31));
  std::memset(h + 148, ' ', 8);
  unsigned sum = 0;
  for (int i = 0; i < 512; ++i) sum += (unsigned char)h[i];
  std::string cs = strfmt("%06o", sum);
  std::memcpy(h + 148, cs.data(), 6);
  h[154] = 0;
  h[155] = ' ';
}

bool TarWriter::write_header(const TarEntry& e) {
  char h[512];
  bool long_name = e.name.size() > 100;
  bool long_link = e.linkname.size() > 100;
  if (long_name || long_link) {
    std::string rec;
    auto add = [&](const std::string& k, const std::string& v) {
      std::string body = " " + k + "=" + v + "\n";
      size_t len = body.size();
      size_t total = len + std::to_string(len).size();
      if (std::to_string(total).size() != std::to_string(len).size()) total = len + std::to_string(total).size();
      rec += std::to_string(total) + body;
    };
    if (long_name) add("path", e.name);
    if (long_link) add("linkpath", e.linkname);
    TarEntry px;
    px.mode = 0644;
    px.mtime = e.mtime;
    fill_header(h, "PaxHeaders/" + e.name.substr(0, 80), px, 'x', (int64_t)rec.size());
    if (!raw(h, 512)) return false;
    if (!raw(rec.data(), rec.size())) return false;
    size_t pad = (512 - rec.size() % 512) % 512;
    char z[512] = {0};
    if (pad && !raw(z, pad)) return false;
  }
  TarEntry copy = e;
  if (long_link) copy.linkname = e.linkname.substr(0, 100);
  fill_header(h, e.name, copy, e.type, e.type == '0' ? e.size : 0);
  written_in_entry_ = 0;
  return raw(h, 512);
}

bool TarWriter::write_data(const char* d, size_t n) {
  written_in_entry_ += (int64_t)n;
  return raw(d, n);
}

bool TarWriter::end_entry() {
  size_t pad = (size_t)((512 - written_in_entry_ % 512) % 512);
  char z[512] = {0};
  written_in_entry_ = 0;
  return pad == 0 || raw(z, pad);
}

bool TarWriter::add_file(TarEntry e, const std::string& data) {
  e.type = '0';
  e.size = (int64_t)data.size();
  return write_header(e) && write_data(data.data(), data.size()) && end_entry();
}

bool TarWriter::add_file_from_path(TarEntry e, const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  e.type = '0';
  if (!write_header(e)) {
    ::close(fd);
    return false;
  }
  char buf[1 << 16];
  int64_t left = e.size;
  while (left > 0) {
    ssize_t n = ::read(fd, buf, (size_t)std::min<int64_t>(left, (int64_t)sizeof(buf)));
    if (n <= 0) {
      // file shrank: pad with zeros to keep the archive consistent
      std::memset(buf, 0, sizeof(buf));
      while (left > 0) {
        size_t c = (size_t)std::min<int64_t>(left, (int64_t)sizeof(buf));
        if (!write_data(buf, c)) break;
        left -= (int64_t)c;
      }
      break;
    }
    if (!write_data(buf, (size_t)n)) {
      ::close(fd);
      return false;
    }
    left -= n;
  }
  ::close(fd);
  return end_entry();
}

bool TarWriter::add_dir(TarEntry e) {
  e.type = '5';
  e.size = 0;
  if (!e.name.empty() && e.name.back() != '/') e.name += "/";
  return write_header(e) && end_entry();
}

bool TarWriter::finish() {
  char z[1024] = {0};
  return raw(z, sizeof(z));
}

bool TarReader::read_block(char* b) {
  size_t got = 0;
  while (got < 512) {
    ssize_t n = src_(b + got, 512 - got);
    if (n <= 0) return got == 0 ? false : throw std::runtime_error("tar: unexpected EOF");
    got += (size_t)n;
  }
  return true;
}

bool TarReader::skip() {
  char buf[1 << 15];
  while (remaining_ > 0) {
    ssize_t n = read(buf, sizeof(buf));
    if (n <= 0) return false;
  }
  while (pad_ > 0) {
    ssize_t n = src_(buf, (size_t)std::min<int64_t>(pad_, (int64_t)sizeof(buf)));
    if (n <= 0) return false;
    pad_ -= n;
  }
  return true;
}

static std::map<std::string, std::string> parse_pax(const std::string& rec) {
  std::map<std::string, std::string> out;
  size_t p = 0;
  while (p < rec.size()) {
    size_t sp = rec.find(' ', p);
    if (sp == std::string::npos) break;
    size_t len = (size_t)std::strtoull(rec.substr(p, sp - p).c_str(), nullptr, 10);
    if (len == 0 || p + len > rec.size()) break;
    std::string kv = rec.substr(sp + 1, len - (sp + 1 - p) - 1);
    size_t eq = kv.find('=');
    if (eq != std::string::npos) out[kv.substr(0, eq)] = kv.substr(eq + 1);
    p += len;
  }
  return out;
}

bool TarReader::next(TarEntry* e) {
  if (!skip()) return false;
  std::string long_name, long_link;
  std::map<std::string, std::string> pax;
  while (true) {
    char h[512];
    if (!read_block(h)) return false;
    bool zero = true;
    for (int i = 0; i < 512; ++i)
      if (h[i]) {
        zero = false;
        break;
      }
    if (zero) {
      // end-of-archive marker; drain the second block if present
      return false;
    }
    // header checksum (unsigned, or signed as some old tars wrote it): garbage is an error,
    // never a bogus entry
    unsigned sum_u = 0;
    int sum_s = 0;
    for (int i = 0; i < 512; ++i) {
      char c = (i >= 148 && i < 156) ? ' ' : h[i];
      sum_u += (unsigned char)c;
      sum_s += (signed char)c;
    }
    uint64_t stored = get_octal(h + 148, 8);
    if (stored != sum_u && (int64_t)stored != (int64_t)sum_s) throw std::runtime_error("tar: invalid header checksum");
    TarEntry t;
    std::string name(h, strnlen(h, 100));
    std::string prefix;
    if (std::memcmp(h + 257, "ustar", 5) == 0) prefix = std::string(h + 345, strnlen(h + 345, 155));
    if (!prefix.empty()) name = prefix + "/" + name;
    t.name = name;
    t.mode = (uint32_t)get_octal(h + 100, 8);
    t.uid = (uint32_t)get_octal(h + 108, 8);
    t.gid = (uint32_t)get_octal(h + 116, 8);
    t.size = (int64_t)get_octal(h + 124, 12);
    t.mtime = (int64_t)get_octal(h + 136, 12);
    t.type = h[156] ? h[156] : '0';
    t.linkname = std::string(h + 157, strnlen(h + 157, 100));
    t.uname = std::string(h + 265, strnlen(h + 265, 32));
    t.gname = std::string(h + 297, strnlen(h + 297, 32));
    remaining_ = t.size;
    pad_ = (512 - t.size % 512) % 512;
    if (t.type == 'L' || t.type == 'K' || t.type == 'x' || t.type == 'g') {
      std::string data = read_all();
      if (pad_ > 0) skip();
      if (t.type == 'L')
        long_name = std::string(data.c_str());
      else if (t.type == 'K')
        long_link = std::string(data.c_str());
      else if (t.type == 'x')
        pax = parse_pax(data);
      continue;
    }
    if (!long_name.empty()) t.name = long_name;
    if (!long_link.empty()) t.linkname = long_link;
    if (pax.count("path")) t.name = pax["path"];
    if (pax.count("linkpath")) t.linkname = pax["linkpath"];
    if (pax.count("size")) t.size = std::strtoll(pax["size"].c_str(), nullptr, 10);
    if (pax.count("mtime")) t.mtime = (int64_t)std::strtod(pax["mtime"].c_str(), nullptr);
    if (t.type == '5' || t.type == '2' || t.type == '1') {
      remaining_ = t.type == '5' ? 0 : remaining_;
    }
    remaining_ = t.type == '0' || t.type == '7' ? t.size : remaining_;
    pad_ = (512 - remaining_ % 512) % 512;
    *e = t;
    return true;
  }
}

ssize_t TarReader::read(char* out, size_t n) {
  if (remaining_ <= 0) return 0;
  size_t c = (size_t)std::min<int64_t>(remaining_, (int64_t)n);
  ssize_t r = src_(out, c);
  if (r <= 0) throw std::runtime_error("tar: unexpected EOF in entry data");
  remaining_ -= r;
  return r;
}

std::string TarReader::read_all() {
  std::string out;
  char buf[1 << 15];
  while (true) {
    ssize_t n = read(buf, sizeof(buf));
    if (n <= 0) break;
    out.append(buf, (size_t)n);
  }
  return out;
}

}  // namespace ds
