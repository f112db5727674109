#include "core/net.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstring>

#include "core/codec.h"
#include "core/strutil.h"

namespace ds {
namespace net {

namespace {

int wait_fd(int fd, short ev, int timeout_ms) {
  struct pollfd pf{fd, ev, 0};
  while (true) {
    int r = ::poll(&pf, 1, timeout_ms);
    if (r < 0 && errno == EINTR) continue;
    return r;
  }
}

class PlainConn : public Conn {
 public:
  explicit PlainConn(int fd) : fd_(fd) {}
  ~PlainConn() override {
    if (fd_ >= 0) ::close(fd_);
  }
  ssize_t read(void* buf, size_t n, int timeout_ms) override {
    if (timeout_ms >= 0) {
      int r = wait_fd(fd_, POLLIN, timeout_ms);
      if (r == 0) return -2;
      if (r < 0) return -1;
    }
    while (true) {
      ssize_t g = ::recv(fd_, buf, n, 0);
      if (g < 0 && errno == EINTR) continue;
      return g;
    }
  }
  bool write_all(const void* d, size_t n) override {
    const char* p = (const char*)d;
    while (n) {
      ssize_t w = ::send(fd_, p, n, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      p += w;
      n -= (size_t)w;
    }
    return true;
  }
  void shutdown() override { ::shutdown(fd_, SHUT_RDWR); }
  int fd() const override { return fd_; }

 private:
  int fd_;
};

SSL_CTX* make_ctx(const TlsOptions& t) {
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) throw NetError("SSL_CTX_new failed");
  if (t.insecure) {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_NONE, nullptr);
  } else {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
    if (!t.ca_pem.empty()) {
      X509_STORE* store = SSL_CTX_get_cert_store(ctx);
      BIO* bio = BIO_new_mem_buf(t.ca_pem.data(), (int)t.ca_pem.size());
      while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
        X509_STORE_add_cert(store, x);
        X509_free(x);
      }
      BIO_free(bio);
      ERR_clear_error();
    } else {
      SSL_CTX_set_default_verify_paths(ctx);
    }
  }
  if (!t.cert_pem.empty() && !t.key_pem.empty()) {
    BIO* cb = BIO_new_mem_buf(t.cert_pem.data(), (int)t.cert_pem.size());
    X509* cert = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
    BIO_free(cb);
    BIO* kb = BIO_new_mem_buf(t.key_pem.data(), (int)t.key_pem.size());
    EVP_PKEY* key = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
    BIO_free(kb);
    if (!cert || !key || SSL_CTX_use_certificate(ctx, cert) != 1 || SSL_CTX_use_PrivateKey(ctx, key) != 1) {
      if (cert) X509_free(cert);
      if (key) EVP_PKEY_free(key);
      SSL_CTX_free(ctx);
      throw NetError("invalid client certificate/key");
    }
    X509_free(cert);
    EVP_PKEY_free(key);
  }
  return ctx;
}

class TlsConn : public Conn {
 public:
  TlsConn(int fd, const TlsOptions& t) : fd_(fd) {
    ctx_ = make_ctx(t);
    ssl_ = SSL_new(ctx_);
    SSL_set_fd(ssl_, fd_);
    if (!t.server_name.empty()) {
      SSL_set_tlsext_host_name(ssl_, t.server_name.c_str());
      if (!t.insecure) {
        X509_VERIFY_PARAM* param = SSL_get0_param(ssl_);
        in6_addr a6;
        in_addr a4;
        if (inet_pton(AF_INET, t.server_name.c_str(), &a4) == 1 || inet_pton(AF_INET6, t.server_name.c_str(), &a6) == 1)
          X509_VERIFY_PARAM_set1_ip_asc(param, t.server_name.c_str());
        else
          X509_VERIFY_PARAM_set1_host(param, t.server_name.c_str(), 0);
      }
    }
    if (SSL_connect(ssl_) != 1) {
      unsigned long e = ERR_get_error();
      char buf[256];
      ERR_error_string_n(e, buf, sizeof(buf));
      throw NetError(std::string("tls handshake failed: ") + buf);
    }
  }
  ~TlsConn() override {
    if (ssl_) {
      SSL_shutdown(ssl_);
      SSL_free(ssl_);
    }
    if (ctx_) SSL_CTX_free(ctx_);
    if (fd_ >= 0) ::close(fd_);
  }
  ssize_t read(void* buf, size_t n, int timeout_ms) override {
    std::lock_guard<std::mutex> g(rmu_);
    if (SSL_pending(ssl_) == 0 && timeout_ms >= 0) {
      int r = wait_fd(fd_, POLLIN, timeout_ms);
      if (r == 0) return -2;
      if (r < 0) return -1;
    }
    while (true) {
      int r;
      {
        std::lock_guard<std::mutex> s(ssl_mu_);
        r = SSL_read(ssl_, buf, (int)n);
      }
      if (r > 0) return r;
      int err;
      {
        std::lock_guard<std::mutex> s(ssl_mu_);
        err = SSL_get_error(ssl_, r);
      }
      if (err == SSL_ERROR_ZERO_RETURN) return 0;
      if (err == SSL_ERROR_WANT_READ) {
        if (wait_fd(fd_, POLLIN, timeout_ms < 0 ? 1000 : timeout_ms) <= 0 && timeout_ms >= 0) return -2;
        continue;
      }
      if (err == SSL_ERROR_SYSCALL && r == 0) return 0;
      return -1;
    }
  }
  bool write_all(const void* d, size_t n) override {
    std::lock_guard<std::mutex> g(wmu_);
    const char* p = (const char*)d;
    while (n) {
      int w;
      {
        std::lock_guard<std::mutex> s(ssl_mu_);
        w = SSL_write(ssl_, p, (int)n);
      }
      if (w <= 0) {
        int err;
        {
          std::lock_guard<std::mutex> s(ssl_mu_);
          err = SSL_get_error(ssl_, w);
        }
        if (err == SSL_ERROR_WANT_WRITE || err == SSL_ERROR_WANT_READ) {
          wait_fd(fd_, POLLOUT, 1000);
          continue;
        }
        return false;
      }
      p += w;
      n -= (size_t)w;
    }
    return true;
  }
  void shutdown() override { ::shutdown(fd_, SHUT_RDWR); }
  int fd() const override { return fd_; }

 private:
  int fd_;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  std::mutex rmu_, wmu_, ssl_mu_;
};

}  // namespace

std::unique_ptr<Conn> dial_tcp(const std::string& host, int port, const TlsOptions& tls, int timeout_ms) {
  struct addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  std::string h = host;
  if (h.size() > 2 && h.front() == '[' && h.back() == ']') h = h.substr(1, h.size() - 2);
  int rc = getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res);
  if (rc != 0) throw NetError("dial tcp " + host + ":" + std::to_string(port) + ": " + gai_strerror(rc));
  int fd = -1;
  std::string last_err = "no addresses";
  for (auto* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int r = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (r != 0 && errno == EINPROGRESS) {
      if (wait_fd(fd, POLLOUT, timeout_ms) > 0) {
        int err = 0;
        socklen_t len = sizeof(err);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
        r = err == 0 ? 0 : -1;
        if (err) errno = err;
      } else {
        errno = ETIMEDOUT;
        r = -1;
      }
    }
    if (r == 0) {
      fcntl(fd, F_SETFL, fl);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      break;
    }
    last_err = std::strerror(errno);
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) throw NetError("dial tcp " + host + ":" + std::to_string(port) + ": " + last_err);
  if (tls.enabled) {
    TlsOptions t = tls;
    if (t.server_name.empty()) t.server_name = h;
    return std::make_unique<TlsConn>(fd, t);
  }
  return std::make_unique<PlainConn>(fd);
}

std::unique_ptr<Conn> dial_unix(const std::string& path) {
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw NetError("socket: " + std::string(std::strerror(errno)));
  struct sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  std::strncpy(addr.sun_path, path.c_str(), sizeof(addr.sun_path) - 1);
  if (::connect(fd, (struct sockaddr*)&addr, sizeof(addr)) != 0) {
    std::string e = std::strerror(errno);
    ::close(fd);
    throw NetError("dial unix " + path + ": " + e);
  }
  return std::make_unique<PlainConn>(fd);
}

Url Url::parse(const std::string& s) {
  Url u;
  size_t p = s.find("://");
  if (p == std::string::npos) {
    u.scheme = "https";
    p = 0;
  } else {
    u.scheme = to_lower(s.substr(0, p));
    p += 3;
  }
  if (u.scheme == "unix") {
    u.unix_path = s.substr(p);
    u.path = "/";
    return u;
  }
  size_t slash = s.find('/', p);
  std::string hostport = slash == std::string::npos ? s.substr(p) : s.substr(p, slash - p);
  u.path = slash == std::string::npos ? "" : s.substr(slash);
  size_t at = hostport.rfind('@');
  if (at != std::string::npos) hostport = hostport.substr(at + 1);
  size_t colon = hostport.rfind(':');
  if (colon != std::string::npos && hostport.find(']', colon) == std::string::npos) {
    u.host = hostport.substr(0, colon);
    u.port = std::atoi(hostport.substr(colon + 1).c_str());
  } else {
    u.host = hostport;
    u.port = u.scheme == "https" || u.scheme == "wss" ? 443 : 80;
  }
  if (!u.path.empty() && u.path.back() == '/') u.path.pop_back();
  return u;
}

std::string Response::header(const std::string& k) const {
  auto it = headers.find(to_lower(k));
  return it == headers.end() ? "" : it->second;
}

std::string url_encode(const std::string& s) {
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~')
      out.push_back((char)c);
    else
      out += strfmt("%%%02X", c);
  }
  return out;
}

HttpClient::HttpClient(const std::string& base_url, TlsOptions tls) : url_(Url::parse(base_url)), tls_(std::move(tls)) {
  if (url_.scheme == "https" || url_.scheme == "wss") tls_.enabled = true;
}

std::unique_ptr<Conn> HttpClient::connect() {
  if (!url_.unix_path.empty()) return dial_unix(url_.unix_path);
  return dial_tcp(url_.host, url_.port, tls_);
}

bool read_response_head(Conn& c, Response* r, std::string* rest, int timeout_ms) {
  std::string buf = *rest;
  rest->clear();
  size_t end;
  while ((end = buf.find("\r\n\r\n")) == std::string::npos) {
    char tmp[8192];
    ssize_t n = c.read(tmp, sizeof(tmp), timeout_ms);
    if (n <= 0) return false;
    buf.append(tmp, (size_t)n);
    if (buf.size() > (1 << 20)) return false;
  }
  std::string head = buf.substr(0, end);
  *rest = buf.substr(end + 4);
  auto lines = split(head, "\r\n");
  if (lines.empty()) return false;
  auto sl = split(lines[0], " ");
  if (sl.size() < 2) return false;
  r->status = std::atoi(sl[1].c_str());
  if (sl.size() > 2) {
    std::vector<std::string> reason(sl.begin() + 2, sl.end());
    r->reason = join(reason, " ");
  }
  for (size_t i = 1; i < lines.size(); ++i) {
    size_t colon = lines[i].find(':');
    if (colon == std::string::npos) continue;
    r->headers[to_lower(trim(lines[i].substr(0, colon)))] = trim(lines[i].substr(colon + 1));
  }
  return true;
}

static std::string build_request(const HttpClient& h, const Request& r) {
  std::string base = h.url().path;
  if (!base.empty() && base.back() == '/' && !r.path.empty() && r.path[0] == '/') base.pop_back();
  std::string path = base + r.path;
  if (path.empty()) path = "/";
  std::string host = h.url().unix_path.empty() ? h.url().host : "localhost";
  std::string out = r.method + " " + path + " HTTP/1.1\r\nHost: " + host + "\r\n";
  std::map<std::string, std::string> hdrs;
  for (auto& kv : h.default_headers()) hdrs[kv.first] = kv.second;
  for (auto& kv : r.headers) hdrs[kv.first] = kv.second;
  for (auto& kv : hdrs) out += kv.first + ": " + kv.second + "\r\n";
  if (!hdrs.count("Content-Length") && (!r.body.empty() || r.method == "POST" || r.method == "PUT" || r.method == "PATCH"))
    out += "Content-Length: " + std::to_string(r.body.size()) + "\r\n";
  if (!hdrs.count("Connection")) out += "Connection: close\r\n";
  out += "\r\n";
  return out;
}

Response HttpClient::stream(Request r, const std::function<bool(const std::string&)>& on_data) {
  auto c = connect();
  if (!c->write_all(build_request(*this, r)) || (!r.body.empty() && !c->write_all(r.body)))
    throw NetError("write request failed");
  Response resp;
  std::string rest;
  if (!read_response_head(*c, &resp, &rest, r.timeout_ms)) throw NetError("read response failed: " + r.path);
  bool chunked = to_lower(resp.header("transfer-encoding")).find("chunked") != std::string::npos;
  std::string cl = resp.header("content-length");
  int64_t remaining = cl.empty() ? -1 : std::atoll(cl.c_str());
  if (r.method == "HEAD" || resp.status == 204 || resp.status == 304) return resp;
  auto deliver = [&](const std::string& d) { return d.empty() || on_data(d); };
  char tmp[65536];
  if (chunked) {
    std::string buf = rest;
    while (true) {
      size_t le;
      while ((le = buf.find("\r\n")) == std::string::npos) {
        ssize_t n = c->read(tmp, sizeof(tmp), r.timeout_ms);
        if (n <= 0) return resp;
        buf.append(tmp, (size_t)n);
      }
      size_t sz = std::strtoul(buf.substr(0, le).c_str(), nullptr, 16);
      buf.erase(0, le + 2);
      if (sz == 0) return resp;
      while (buf.size() < sz + 2) {
        ssize_t n = c->read(tmp, sizeof(tmp), r.timeout_ms);
        if (n <= 0) {
          deliver(buf.substr(0, std::min(buf.size(), sz)));
          return resp;
        }
        buf.append(tmp, (size_t)n);
      }
      if (!deliver(buf.substr(0, sz))) return resp;
      buf.erase(0, sz + 2);
    }
  }
  if (!rest.empty()) {
    if (remaining >= 0 && (int64_t)rest.size() > remaining) rest.resize((size_t)remaining);
    if (remaining >= 0) remaining -= (int64_t)rest.size();
    if (!deliver(rest)) return resp;
  }
  while (remaining != 0) {
    size_t want = remaining > 0 ? (size_t)std::min<int64_t>(remaining, (int64_t)sizeof(tmp)) : sizeof(tmp);
    ssize_t n = c->read(tmp, want, r.timeout_ms);
    if (n <= 0) break;
    if (remaining > 0) remaining -= n;
    if (!deliver(std::string(tmp, (size_t)n))) break;
  }
  return resp;
}

Response HttpClient::request(Request r) {
  std::string body;
  Response resp = stream(r, [&](const std::string& d) {
    body += d;
    return true;
  });
  resp.body = std::move(body);
  return resp;
}

// ---------------------------------------------------------------- websocket

std::unique_ptr<WebSocket> WebSocket::connect(HttpClient& http, const std::string& path,
                                              const std::vector<std::string>& protocols, int timeout_ms) {
  auto c = http.connect();
  std::string key = base64_encode(random_string(16));
  Request r;
  r.method = "GET";
  r.path = path;
  r.headers = {{"Connection", "Upgrade"},
               {"Upgrade", "websocket"},
               {"Sec-WebSocket-Version", "13"},
               {"Sec-WebSocket-Key", key}};
  if (!protocols.empty()) r.headers.push_back({"Sec-WebSocket-Protocol", join(protocols, ", ")});
  std::string req = build_request(http, r);
  if (!c->write_all(req)) throw NetError("websocket: write handshake failed");
  Response resp;
  std::string rest;
  if (!read_response_head(*c, &resp, &rest, timeout_ms)) throw NetError("websocket: no handshake response");
  if (resp.status != 101) {
    // read error body for a useful message
    std::string body = rest;
    char tmp[4096];
    while (body.size() < 65536) {
      ssize_t n = c->read(tmp, sizeof(tmp), 2000);
      if (n <= 0) break;
      body.append(tmp, (size_t)n);
    }
    throw NetError("websocket upgrade failed: " + std::to_string(resp.status) + " " + resp.reason + ": " + body);
  }
  Sha256 h;
  (void)h;
  auto ws = std::make_unique<WebSocket>(std::move(c), rest);
  ws->protocol_ = resp.header("sec-websocket-protocol");
  return ws;
}

WebSocket::WebSocket(std::unique_ptr<Conn> c, std::string leftover) : c_(std::move(c)), buf_(std::move(leftover)) {}

WebSocket::~WebSocket() { close(); }

bool WebSocket::send(const std::string& payload, Op op) {
  std::lock_guard<std::mutex> g(wmu_);
  if (closed_) return false;
  std::string f;
  f.push_back((char)(0x80 | op));
  size_t n = payload.size();
  if (n < 126) {
    f.push_back((char)(0x80 | n));
  } else if (n < 65536) {
    f.push_back((char)(0x80 | 126));
    f.push_back((char)(n >> 8));
    f.push_back((char)n);
  } else {
    f.push_back((char)(0x80 | 127));
    for (int i = 7; i >= 0; --i) f.push_back((char)((uint64_t)n >> (8 * i)));
  }
  std::string mask = random_string(4);
  f += mask;
  size_t off = f.size();
  f.resize(off + n);
  for (size_t i = 0; i < n; ++i) f[off + i] = (char)(payload[i] ^ mask[i & 3]);
  return c_->write_all(f);
}

bool WebSocket::read_exact(char* out, size_t n, int timeout_ms) {
  while (buf_.size() < n) {
    char tmp[65536];
    ssize_t r = c_->read(tmp, sizeof(tmp), timeout_ms);
    if (r <= 0) return false;
    buf_.append(tmp, (size_t)r);
  }
  std::memcpy(out, buf_.data(), n);
  buf_.erase(0, n);
  return true;
}

bool WebSocket::recv(std::string* payload, Op* op_out, int timeout_ms) {
  std::string msg;
  Op msg_op = Binary;
  while (true) {
    unsigned char h[2];
    if (!read_exact((char*)h, 2, timeout_ms)) return false;
    bool fin = h[0] & 0x80;
    Op op = (Op)(h[0] & 0x0F);
    bool masked = h[1] & 0x80;
    uint64_t len = h[1] & 0x7F;
    if (len == 126) {
      unsigned char e[2];
      if (!read_exact((char*)e, 2, timeout_ms)) return false;
      len = ((uint64_t)e[0] << 8) | e[1];
    } else if (len == 127) {
      unsigned char e[8];
      if (!read_exact((char*)e, 8, timeout_ms)) return false;
      len = 0;
      for (int i = 0; i < 8; ++i) len = (len << 8) | e[i];
    }
    char mask[4] = {0, 0, 0, 0};
    if (masked && !read_exact(mask, 4, timeout_ms)) return false;
    std::string data(len, '\0');
    if (len && !read_exact(&data[0], len, timeout_ms)) return false;
    if (masked)
      for (size_t i = 0; i < len; ++i) data[i] ^= mask[i & 3];
    if (op == Close) {
      std::lock_guard<std::mutex> g(wmu_);
      closed_ = true;
      return false;
    }
    if (op == Ping) {
      send(data, Pong);
      continue;
    }
    if (op == Pong) continue;
    if (op != Cont) msg_op = op;
    msg += data;
    if (fin) {
      *payload = std::move(msg);
      if (op_out) *op_out = msg_op;
      return true;
    }
  }
}

void WebSocket::close() {
  {
    std::lock_guard<std::mutex> g(wmu_);
    if (closed_ || !c_) return;
  }
  send(std::string("\x03\xe8", 2), Close);
  std::lock_guard<std::mutex> g(wmu_);
  closed_ = true;
  c_->shutdown();
}

void WebSocket::shutdown() {
  if (c_) c_->shutdown();
}

}  // namespace net
}  // namespace ds
