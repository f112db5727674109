// gzip + tar streams (sync/tar.go, util/tar/tar.go). Kept free of OpenSSL so the static
// in-container helper (src/helper/helper.cc) can link it with only zlib.
#include <fcntl.h>
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
  z_stream* z = (z_stream*)z_;
  z->next_out = (Bytef*)out;
  z->avail_out = (uInt)n;
  while (z->avail_out == n) {
    if (z->avail_in == 0) {
      if (eof_) return stream_end_ ? 0 : -1;
      ssize_t r = src_(in_.data(), in_.size());
      if (r < 0) return -1;
      if (r == 0) {
        eof_ = true;
        if (stream_end_) return 0;
        // try to flush what we have
      }
      z->next_in = (Bytef*)in_.data();
      z->avail_in = (uInt)(r > 0 ? r : 0);
      if (r == 0 && !stream_end_) {
        int rr = inflate(z, Z_SYNC_FLUSH);
        if (rr == Z_STREAM_END) stream_end_ = true;
        size_t got = n - z->avail_out;
        return got > 0 ? (ssize_t)got : (stream_end_ ? 0 : -1);
      }
    }
    if (stream_end_) {
      // concatenated member?
      if (z->avail_in > 0) {
        inflateReset(z);
        stream_end_ = false;
      } else {
        continue;
      }
    }
    int r = inflate(z, Z_NO_FLUSH);
    if (r == Z_STREAM_END) {
      stream_end_ = true;
      if (n - z->avail_out > 0) break;
      if (z->avail_in == 0 && eof_) return 0;
      continue;
    }
    if (r != Z_OK && r != Z_BUF_ERROR) return -1;
  }
  return (ssize_t)(n - z->avail_out);
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

std::string gzip_compress_adaptive(const std::string& data, int level) {
  // One gzip member (any `tar xz` / gunzip reads it), compressed in 1 MiB chunks whose level
  // follows their sampled entropy: stored blocks (level 0) for incompressible chunks, `level`
  // otherwise. deflate at level 1 runs ~20 MB/s on random bytes; stored blocks run at memcpy +
  // CRC speed, so a tree of model checkpoints is no longer compression-bound.
  std::string out;
  out.reserve(data.size() / 2 + 1024);
  z_stream z;
  std::memset(&z, 0, sizeof(z));
  if (deflateInit2(&z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    throw std::runtime_error("deflateInit2 failed");
  std::vector<char> buf(1 << 17);
  auto drain = [&](int flush) {
    int r;
    do {
      z.next_out = (Bytef*)buf.data();
      z.avail_out = (uInt)buf.size();
      r = deflate(&z, flush);
      out.append(buf.data(), buf.size() - z.avail_out);
    } while (z.avail_out == 0 || (flush == Z_FINISH && r != Z_STREAM_END));
  };
  const size_t kChunk = 1 << 20, kSample = 1 << 16;
  int cur = level;
  for (size_t off = 0; off < data.size(); off += kChunk) {
    size_t n = std::min(kChunk, data.size() - off);
    const unsigned char* p = (const unsigned char*)data.data() + off;
    int want = sample_entropy(p, std::min(n, kSample)) > 7.5 ? 0 : level;
    if (want != cur) {
      int r;
      do {
        z.next_out = (Bytef*)buf.data();
        z.avail_out = (uInt)buf.size();
        r = deflateParams(&z, want, Z_DEFAULT_STRATEGY);
        out.append(buf.data(), buf.size() - z.avail_out);
      } while (r == Z_BUF_ERROR);
      cur = want;
    }
    z.next_in = (Bytef*)p;
    z.avail_in = (uInt)n;
    drain(Z_NO_FLUSH);
  }
  z.next_in = nullptr;
  z.avail_in = 0;
  drain(Z_FINISH);
  deflateEnd(&z);
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
