#include "core/codec.h"

#include <fcntl.h>
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <unistd.h>
#include <zlib.h>

#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>

#include "core/proc.h"
#include "core/strutil.h"

namespace ds {

// ------------------------------------------------------------------ hashing

Sha256::Sha256() {
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  EVP_DigestInit_ex(c, EVP_sha256(), nullptr);
  ctx_ = c;
}
Sha256::~Sha256() { EVP_MD_CTX_free((EVP_MD_CTX*)ctx_); }
void Sha256::update(const void* d, size_t n) { EVP_DigestUpdate((EVP_MD_CTX*)ctx_, d, n); }
std::string Sha256::digest() {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_DigestFinal_ex((EVP_MD_CTX*)ctx_, md, &len);
  return std::string((char*)md, len);
}
std::string Sha256::hex() { return hex_encode(digest()); }

std::string sha256_hex(const std::string& data) {
  Sha256 h;
  h.update(data);
  return h.hex();
}

uint32_t crc32_bytes(const void* d, size_t n, uint32_t crc) {
  return (uint32_t)::crc32(crc, (const Bytef*)d, (uInt)n);
}

std::string crc32_file_hex(const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return "";
  uLong crc = ::crc32(0L, Z_NULL, 0);
  char buf[1 << 16];
  while (true) {
    ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0) {
      ::close(fd);
      return "";
    }
    if (n == 0) break;
    crc = ::crc32(crc, (const Bytef*)buf, (uInt)n);
  }
  ::close(fd);
  return strfmt("%08lx", (unsigned long)crc);
}

std::string hex_encode(const std::string& in) {
  static const char* h = "0123456789abcdef";
  std::string out;
  out.reserve(in.size() * 2);
  for (unsigned char c : in) {
    out.push_back(h[c >> 4]);
    out.push_back(h[c & 15]);
  }
  return out;
}

std::string base64_encode(const std::string& in, bool url) {
  static const char* std_tab = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  static const char* url_tab = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
  const char* t = url ? url_tab : std_tab;
  std::string out;
  size_t i = 0;
  while (i + 2 < in.size()) {
    uint32_t v = ((unsigned char)in[i] << 16) | ((unsigned char)in[i + 1] << 8) | (unsigned char)in[i + 2];
    out.push_back(t[(v >> 18) & 63]);
    out.push_back(t[(v >> 12) & 63]);
    out.push_back(t[(v >> 6) & 63]);
    out.push_back(t[v & 63]);
    i += 3;
  }
  if (i + 1 == in.size()) {
    uint32_t v = (unsigned char)in[i] << 16;
    out.push_back(t[(v >> 18) & 63]);
    out.push_back(t[(v >> 12) & 63]);
    out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = ((unsigned char)in[i] << 16) | ((unsigned char)in[i + 1] << 8);
    out.push_back(t[(v >> 18) & 63]);
    out.push_back(t[(v >> 12) & 63]);
    out.push_back(t[(v >> 6) & 63]);
    out.push_back('=');
  }
  return out;
}

std::string base64_decode(const std::string& in) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  std::string out;
  uint32_t acc = 0;
  int bits = 0;
  for (char c : in) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    int v = val(c);
    if (v < 0) throw std::runtime_error("illegal base64 data");
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((char)((acc >> bits) & 0xFF));
    }
  }
  return out;
}

static void rand_bytes(unsigned char* b, size_t n) {
  if (RAND_bytes(b, (int)n) != 1) {
    for (size_t i = 0; i < n; ++i) b[i] = (unsigned char)(rand() & 0xFF);
  }
}

std::string random_string(size_t n) {
  static const char* alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
  std::string out;
  unsigned char b[64];
  while (out.size() < n) {
    rand_bytes(b, sizeof(b));
    for (unsigned char c : b) {
      if (c >= 248) continue;  // 248 = 62*4 for unbiased modulo
      out.push_back(alpha[c % 62]);
      if (out.size() == n) break;
    }
  }
  return out;
}

std::string random_lower_alnum(size_t n) {
  static const char* alpha = "abcdefghijklmnopqrstuvwxyz0123456789";
  std::string out;
  unsigned char b[64];
  while (out.size() < n) {
    rand_bytes(b, sizeof(b));
    for (unsigned char c : b) {
      if (c >= 252) continue;
      out.push_back(alpha[c % 36]);
      if (out.size() == n) break;
    }
  }
  return out;
}

}  // namespace ds
