#include "sync/frame.h"

#include <zlib.h>

#include <cmath>

namespace ds {
namespace sync {
namespace frame {

namespace {
// order-0 entropy (bits/byte) of up to 64 KiB spread over the chunk
double chunk_entropy(const unsigned char* p, size_t n) {
  if (n == 0) return 0;
  uint32_t hist[256] = {0};
  size_t take = 0;
  const size_t kSlice = 4096;
  size_t stride = n > (64u << 10) ? n / 16 : n;
  for (size_t off = 0; off < n; off += stride) {
    size_t k = std::min(n - off, stride == n ? n : kSlice);
    for (size_t i = 0; i < k; ++i) hist[p[off + i]]++;
    take += k;
  }
  double h = 0;
  for (uint32_t c : hist) {
    if (!c) continue;
    double q = (double)c / (double)take;
    h -= q * std::log2(q);
  }
  return h;
}
}  // namespace

ChunkWriter::ChunkWriter(Sink out, size_t chunk, int level) : out_(std::move(out)), chunk_(chunk), level_(level) {
  if (chunk_ == 0 || chunk_ > kMaxChunk) chunk_ = kMaxChunk;
  buf_.reserve(chunk_);
  if (level_ >= 0) {
    z_stream* z = new z_stream();
    if (deflateInit2(z, level_, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
      delete z;
      throw std::runtime_error("deflateInit2 failed");
    }
    z_ = z;
  }
}

ChunkWriter::~ChunkWriter() {
  if (z_) {
    deflateEnd((z_stream*)z_);
    delete (z_stream*)z_;
  }
}

bool ChunkWriter::write(const char* d, size_t n) {
  if (done_) return false;
  while (n > 0) {
    size_t take = std::min(n, chunk_ - buf_.size());
    buf_.append(d, take);
    d += take;
    n -= take;
    total_ += take;
    if (buf_.size() == chunk_ && !flush()) return false;
  }
  return true;
}

bool ChunkWriter::flush() {
  if (buf_.empty()) return true;
  const char* payload = buf_.data();
  uint32_t n = (uint32_t)buf_.size(), hdr = n;
  if (z_ && chunk_entropy((const unsigned char*)buf_.data(), buf_.size()) < 7.2) {
    z_stream* z = (z_stream*)z_;
    deflateReset(z);
    zbuf_.resize(deflateBound(z, buf_.size()));
    z->next_in = (Bytef*)buf_.data();
    z->avail_in = (uInt)buf_.size();
    z->next_out = (Bytef*)&zbuf_[0];
    z->avail_out = (uInt)zbuf_.size();
    int r = deflate(z, Z_FINISH);
    size_t zn = zbuf_.size() - z->avail_out;
    if (r == Z_STREAM_END && zn < buf_.size()) {
      payload = zbuf_.data();
      n = (uint32_t)zn;
      hdr = n | kDeflatedFlag;
      ++deflated_;
    }
  }
  char h[4] = {(char)(hdr >> 24), (char)(hdr >> 16), (char)(hdr >> 8), (char)hdr};
  bool ok = out_(h, 4) && out_(payload, n);
  wire_ += 4 + n;
  buf_.clear();
  return ok;
}

bool ChunkWriter::finish() {
  if (done_) return true;
  if (!flush()) return false;
  done_ = true;
  char z[4] = {0, 0, 0, 0};
  wire_ += 4;
  return out_(z, 4);
}

ChunkReader::ChunkReader(Source raw) : raw_(std::move(raw)) {}

ChunkReader::~ChunkReader() {
  if (z_) {
    inflateEnd((z_stream*)z_);
    delete (z_stream*)z_;
  }
}

void ChunkReader::read_exact(char* p, size_t n) {
  while (n > 0) {
    ssize_t r = raw_(p, n);
    if (r <= 0) throw std::runtime_error("frame: stream ended inside a chunk");
    p += r;
    n -= (size_t)r;
  }
}

ssize_t ChunkReader::read(char* out, size_t n) {
  if (n == 0) return 0;
  if (dec_pos_ < dec_.size()) {
    size_t c = std::min(n, dec_.size() - dec_pos_);
    std::memcpy(out, dec_.data() + dec_pos_, c);
    dec_pos_ += c;
    total_ += c;
    return (ssize_t)c;
  }
  if (end_) return 0;
  if (left_ == 0) {
    unsigned char h[4];
    read_exact((char*)h, 4);
    uint32_t v = ((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3];
    if (v == 0) {
      end_ = true;
      return 0;
    }
    uint32_t len = v & ~kDeflatedFlag;
    if (len == 0 || len > kMaxChunk + (kMaxChunk >> 4)) throw std::runtime_error("frame: chunk length out of range");
    if (v & kDeflatedFlag) {
      std::string in(len, '\0');
      read_exact(&in[0], len);
      if (!z_) {
        z_stream* z = new z_stream();
        if (inflateInit2(z, -15) != Z_OK) {
          delete z;
          throw std::runtime_error("inflateInit2 failed");
        }
        z_ = z;
      }
      z_stream* z = (z_stream*)z_;
      inflateReset(z);
      dec_.resize(kMaxChunk);
      z->next_in = (Bytef*)in.data();
      z->avail_in = (uInt)in.size();
      z->next_out = (Bytef*)&dec_[0];
      z->avail_out = (uInt)dec_.size();
      int r = inflate(z, Z_FINISH);
      if (r != Z_STREAM_END || z->avail_in != 0) throw std::runtime_error("frame: corrupt deflate chunk");
      dec_.resize(dec_.size() - z->avail_out);
      dec_pos_ = 0;
      return read(out, n);
    }
    left_ = len;
  }
  ssize_t r = raw_(out, std::min<size_t>(n, left_));
  if (r <= 0) throw std::runtime_error("frame: stream ended inside a chunk");
  left_ -= (uint32_t)r;
  total_ += (uint64_t)r;
  return r;
}

void ChunkReader::drain() {
  char buf[1 << 15];
  while (read(buf, sizeof(buf)) > 0) {
  }
}

}  // namespace frame
}  // namespace sync
}  // namespace ds
