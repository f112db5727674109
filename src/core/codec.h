// Hashing, encodings, randomness, gzip and tar streams.
//
// util/hash/hash.go (SHA-256 over path;size;mtime, CRC32 of file contents),
// util/randutil/rand.go, sync/tar.go (tar.gz build/extract), util/tar/tar.go.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace ds {

std::string sha256_hex(const std::string& data);
class Sha256 {
 public:
  Sha256();
  ~Sha256();
  void update(const void* d, size_t n);
  void update(const std::string& s) { update(s.data(), s.size()); }
  std::string hex();
  std::string digest();

 private:
  void* ctx_;
};
uint32_t crc32_bytes(const void* d, size_t n, uint32_t crc = 0);
// CRC32 (IEEE) of a file's contents as 8 lower-case hex chars; "" on error.
std::string crc32_file_hex(const std::string& path);

std::string base64_encode(const std::string& in, bool url = false);
std::string base64_decode(const std::string& in);  // accepts std + url alphabets, padding optional
std::string hex_encode(const std::string& in);

// Random [a-zA-Z0-9] string (util/randutil/rand.go:10).
std::string random_string(size_t n);
std::string random_lower_alnum(size_t n);

using Sink = std::function<bool(const char*, size_t)>;
using Source = std::function<ssize_t(char*, size_t)>;  // 0 = EOF, <0 = error

// Streaming gzip compressor forwarding to a sink.
class GzipWriter {
 public:
  explicit GzipWriter(Sink sink, int level = 6);
  ~GzipWriter();
  bool write(const char* d, size_t n);
  bool write(const std::string& s) { return write(s.data(), s.size()); }
  bool finish();

 private:
  bool pump(int flush);
  Sink sink_;
  void* z_;
  bool finished_ = false;
};

// Streaming gzip whose deflate level adapts per 1 MiB chunk (sampled order-0 entropy): stored
// blocks for incompressible chunks (checkpoints, archives, images), `level` elsewhere. A
// standard gzip stream (a new member at each level change and every 1 GiB); memory is bounded
// by the chunk buffer whatever the stream length.
class AdaptiveGzipWriter {
 public:
  explicit AdaptiveGzipWriter(Sink sink, int level = 1);
  ~AdaptiveGzipWriter();
  AdaptiveGzipWriter(const AdaptiveGzipWriter&) = delete;
  bool write(const char* d, size_t n);
  bool write(const std::string& s) { return write(s.data(), s.size()); }
  bool finish();

 private:
  bool deflate_chunk(bool last);
  bool drain(int flush);
  bool new_member(int level);
  Sink sink_;
  void* z_;
  int level_, cur_;
  uint64_t member_in_ = 0;
  std::string buf_;
  std::vector<char> out_;
  bool finished_ = false;
};

// Streaming gzip decompressor pulling from a source (handles concatenated members).
class GzipReader {
 public:
  explicit GzipReader(Source src);
  ~GzipReader();
  ssize_t read(char* out, size_t n);
  // Single-member mode: stop at the end of the first gzip member and never read the source
  // past it; bytes already pulled beyond the member are available from leftover(). Used when
  // the member is followed by other protocol data on the same stream.
  void set_single_member(bool on) { single_ = on; }
  bool at_end() const { return stream_end_; }
  std::string leftover() const;

 private:
  Source src_;
  void* z_;
  std::vector<char> in_;
  bool eof_ = false;
  bool stream_end_ = false;
  bool single_ = false;
};

// Byte buffer that stays in memory up to `mem_limit` and spills to an unlinked temp file
// beyond it (sync/tar.go:146 writes every archive to a temp file; here only big ones are).
// Lets protocols that must announce a length first (`head -c N`, the reference's fileSize=N
// script) send multi-GB archives with bounded memory.
class SpillBuffer {
 public:
  explicit SpillBuffer(size_t mem_limit = 8u << 20, std::string dir = "");
  ~SpillBuffer();
  SpillBuffer(const SpillBuffer&) = delete;
  bool append(const char* d, size_t n);
  Sink sink() {
    return [this](const char* d, size_t n) { return append(d, n); };
  }
  uint64_t size() const { return size_; }
  bool spilled() const { return fd_ >= 0; }
  // Streams the whole content, from the start, to `out` in blocks of at most 1 MiB.
  bool replay(const Sink& out);
  // First bytes (for format sniffing); up to n.
  std::string head(size_t n);

 private:
  bool flush_stage();
  size_t limit_;
  std::string dir_;
  std::string mem_;    // content while not spilled
  std::string stage_;  // write-behind buffer once spilled
  int fd_ = -1;
  uint64_t size_ = 0;
};

// Source that first returns `prefix`, then reads from `rest` (format sniffing without loss).
Source prefixed_source(std::string prefix, Source rest);
// Source limited to exactly `n` bytes of `inner` (returns 0 after that).
Source limited_source(Source inner, uint64_t n);

std::string gzip_compress(const std::string& data, int level = 6);
// gzip whose deflate level adapts per 1 MiB chunk: stored blocks where the data is already
// incompressible (sampled entropy), `level` elsewhere (see AdaptiveGzipWriter).
std::string gzip_compress_adaptive(const std::string& data, int level = 1);
std::string gzip_decompress(const std::string& data);

struct TarEntry {
  std::string name;  // as stored (no leading "./" normalisation)
  char type = '0';   // '0' file, '5' dir, '2' symlink, '1' hardlink
  uint32_t mode = 0644;
  uint32_t uid = 0, gid = 0;
  int64_t size = 0;
  int64_t mtime = 0;
  std::string linkname;
  std::string uname, gname;
};

class TarWriter {
 public:
  explicit TarWriter(Sink sink) : sink_(std::move(sink)) {}
  bool write_header(const TarEntry& e);
  bool write_data(const char* d, size_t n);  // exactly entry.size bytes in total
  bool end_entry();                          // pads to 512
  bool add_file(TarEntry e, const std::string& data);
  bool add_file_from_path(TarEntry e, const std::string& path);  // streams the file
  bool add_dir(TarEntry e);
  bool finish();  // writes two zero blocks

 private:
  bool raw(const char* d, size_t n);
  Sink sink_;
  int64_t written_in_entry_ = 0;
};

class TarReader {
 public:
  explicit TarReader(Source src) : src_(std::move(src)) {}
  // Returns false at end of archive; throws on corrupt input (bad header checksum, EOF inside
  // an entry).
  bool next(TarEntry* e);
  // Read file data of the current entry; returns 0 when exhausted.
  ssize_t read(char* out, size_t n);
  std::string read_all();
  bool skip();

 private:
  bool read_block(char* b);
  Source src_;
  int64_t remaining_ = 0;
  int64_t pad_ = 0;
};

// Convenience: source that reads from an fd; sink that writes to an fd; string sinks.
Source fd_source(int fd);
Sink fd_sink(int fd);
Sink string_sink(std::string* out);
Source string_source(const std::string* in);

}  // namespace ds
