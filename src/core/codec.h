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

// Streaming gzip decompressor pulling from a source (handles concatenated members).
class GzipReader {
 public:
  explicit GzipReader(Source src);
  ~GzipReader();
  ssize_t read(char* out, size_t n);

 private:
  Source src_;
  void* z_;
  std::vector<char> in_;
  bool eof_ = false;
  bool stream_end_ = false;
};

std::string gzip_compress(const std::string& data, int level = 6);
// gzip whose deflate level adapts per 1 MiB chunk: stored blocks where the data is already
// incompressible (sampled entropy), `level` elsewhere. Output is a standard gzip member.
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
  // Returns false at end of archive; throws on corrupt input.
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
