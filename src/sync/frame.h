// Wire framing of the helper protocol (src/helper/helper.cc <-> src/sync/sync.cc).
//
//   request  := op:u8  len:u64be  payload[len]          (lists of paths, small)
//   stream   := chunk*  end                             (archives of any size)
//   chunk    := n:u32be (1..kMaxChunk)  bytes[n]        (bit 31 of n: raw deflate, see ChunkWriter)
//   end      := 0:u32be
//
// Archives travel as chunk streams, so neither side ever needs the total length up front or
// holds a whole archive in memory: a multi-GB checkpoint moves through a bounded buffer. The
// reference announced every archive's size first and staged it in a temp file on both sides
// (sync/tar.go:146, sync/downstream.go:443).
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "core/codec.h"

namespace ds {
namespace sync {
namespace frame {

constexpr size_t kHeaderSize = 9;
constexpr uint32_t kMaxChunk = 1u << 20;
constexpr uint64_t kMaxListPayload = 1ull << 30;  // request payloads are path lists
constexpr uint32_t kDeflatedFlag = 0x80000000u;

inline std::string header(char op, uint64_t len) {
  std::string h(kHeaderSize, '\0');
  h[0] = op;
  for (int i = 0; i < 8; ++i) h[1 + i] = (char)(len >> (56 - 8 * i));
  return h;
}

inline std::string request(char op, const std::string& payload) { return header(op, payload.size()) + payload; }

inline void parse_header(const unsigned char* h, char* op, uint64_t* len) {
  *op = (char)h[0];
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | h[1 + i];
  *len = v;
}

// Sink -> chunk stream. Buffers up to `chunk` bytes so small writes do not become tiny chunks.
// With level >= 0 each chunk is coded on its own: raw deflate at `level` when its sampled
// entropy says it compresses (source files, logs), stored as-is otherwise (checkpoints,
// archives) — per-chunk, so a tree that mixes both is neither deflate-bound on the
// incompressible part nor uncompressed on the rest, and no gzip CRC pass runs on either side
// (the transport — a pipe, TLS — already guarantees integrity).
//   chunk header n:u32be — bit 31 set: the n & 0x7fffffff payload bytes are raw deflate of at
//   most kMaxChunk decoded bytes.
class ChunkWriter {
 public:
  explicit ChunkWriter(Sink out, size_t chunk = 256u << 10, int level = -1);
  ~ChunkWriter();
  ChunkWriter(const ChunkWriter&) = delete;
  bool write(const char* d, size_t n);
  Sink sink() {
    return [this](const char* d, size_t n) { return write(d, n); };
  }
  bool finish();
  uint64_t bytes() const { return total_; }       // decoded bytes written
  uint64_t wire_bytes() const { return wire_; }   // bytes sent, headers included
  uint64_t deflated_chunks() const { return deflated_; }

 private:
  bool flush();
  Sink out_;
  size_t chunk_;
  int level_;
  void* z_ = nullptr;
  std::string buf_;
  std::string zbuf_;
  uint64_t total_ = 0, wire_ = 0, deflated_ = 0;
  bool done_ = false;
};

// Chunk stream -> Source (0 at the end marker). Throws on a truncated stream, a malformed
// chunk length or bad deflate data; never reads the underlying stream past the end marker.
class ChunkReader {
 public:
  explicit ChunkReader(Source raw);
  ~ChunkReader();
  ChunkReader(const ChunkReader&) = delete;
  ssize_t read(char* out, size_t n);
  Source source() {
    return [this](char* b, size_t n) { return read(b, n); };
  }
  // Consumes the rest of the stream up to and including the end marker.
  void drain();
  bool ended() const { return end_; }
  uint64_t bytes() const { return total_; }

 private:
  void read_exact(char* p, size_t n);
  Source raw_;
  uint32_t left_ = 0;      // raw chunk bytes still unread
  std::string dec_;        // decoded deflate chunk
  size_t dec_pos_ = 0;
  void* z_ = nullptr;
  uint64_t total_ = 0;
  bool end_ = false;
};

}  // namespace frame
}  // namespace sync
}  // namespace ds
