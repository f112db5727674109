#include "core/net.h"

#include "core/compat.h"
#include "core/resolve.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/sha.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <climits>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "core/codec.h"
#include "core/strutil.h"
#include "platform/platform.h"

namespace ds {
namespace net {

Stats& stats() {
  static Stats s;
  return s;
}

namespace {

int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Remaining milliseconds until `deadline` (-1 = no deadline → -1 = wait forever).
int remaining_ms(int64_t deadline) {
  if (deadline < 0) return -1;
  int64_t left = deadline - mono_ms();
  return left < 0 ? 0 : (int)std::min<int64_t>(left, INT_MAX);
}

int wait_fd(int fd, short ev, int timeout_ms) {
  struct pollfd pf{fd, ev, 0};
  while (true) {
    int r = ::poll(&pf, 1, timeout_ms);
    if (r < 0 && errno == EINTR) continue;
    return r;
  }
}

// Waits for `ev` on fd or for a poke of `wake` (drained here). >0 ready, 0 timeout.
int wait_fd_or_wake(int fd, short ev, plat::Waker& wake, int timeout_ms) {
  struct pollfd pf[2] = {{fd, ev, 0}, {wake.fd(), POLLIN, 0}};
  while (true) {
    int r = ::poll(pf, wake.ok() ? 2 : 1, timeout_ms);
    if (r < 0 && errno == EINTR) continue;
    if (r > 0 && wake.ok() && (pf[1].revents & POLLIN)) wake.drain();
    return r;
  }
}

std::string ssl_error_string() {
  std::string out;
  while (unsigned long e = ERR_get_error()) {
    char buf[256];
    ERR_error_string_n(e, buf, sizeof(buf));
    if (!out.empty()) out += "; ";
    out += buf;
  }
  return out;
}

class PlainConn : public Conn {
 public:
  using Conn::write_all;
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
      ssize_t w = plat::send_nosignal(fd_, p, n);
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
  int release() {
    int f = fd_;
    fd_ = -1;
    return f;
  }

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
    // intermediate certificates after the leaf go into the chain
    std::vector<X509*> chain;
    while (cert) {
      X509* extra = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
      if (!extra) break;
      chain.push_back(extra);
    }
    BIO_free(cb);
    ERR_clear_error();
    BIO* kb = BIO_new_mem_buf(t.key_pem.data(), (int)t.key_pem.size());
    EVP_PKEY* key = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
    BIO_free(kb);
    bool ok = cert && key && SSL_CTX_use_certificate(ctx, cert) == 1 && SSL_CTX_use_PrivateKey(ctx, key) == 1;
    for (X509* x : chain) {
      if (ok && SSL_CTX_add_extra_chain_cert(ctx, x) == 1) continue;  // ctx owns x now
      X509_free(x);
    }
    if (cert) X509_free(cert);
    if (key) EVP_PKEY_free(key);
    if (!ok) {
      SSL_CTX_free(ctx);
      throw NetError("invalid client certificate/key");
    }
  }
  return ctx;
}

// Client TLS contexts are shared per credential set (CA, client cert/key, verify mode): the
// PEM parsing happens once, and the context carries a client session cache so a new
// connection to the same API server resumes the last session (TLS 1.3 ticket / 1.2 session
// id) instead of a full handshake with certificate verification on both sides — every
// exec / attach / port-forward stream is a new connection. Off with DEVSPACE_REFERENCE_TIMING
// (client-go configures no session cache).
namespace {
std::mutex g_tls_mu;
// Process-lifetime caches, deliberately never destroyed: OpenSSL's own exit-time cleanup can
// run before static destructors, so freeing contexts there is unsafe. Held through globals,
// they stay reachable at exit (leak checkers do not count them).
std::map<std::string, SSL_CTX*>& g_ctx_cache = *new std::map<std::string, SSL_CTX*>();  // digest -> ctx
std::map<std::string, SSL_SESSION*>& g_sessions = *new std::map<std::string, SSL_SESSION*>();  // digest|peer -> session

int new_session_cb(SSL* ssl, SSL_SESSION* sess) {
  auto* key = static_cast<const std::string*>(SSL_get_app_data(ssl));
  if (!key || !SSL_SESSION_is_resumable(sess)) return 0;
  std::lock_guard<std::mutex> g(g_tls_mu);
  auto it = g_sessions.find(*key);
  if (it != g_sessions.end()) SSL_SESSION_free(it->second);
  g_sessions[*key] = sess;
  return 1;  // we keep the reference
}

// A referenced context for these options (caller frees with SSL_CTX_free) and its cache key.
SSL_CTX* shared_ctx(const TlsOptions& t, std::string* digest) {
  std::string material = std::string(t.insecure ? "1" : "0") + "\n" + t.ca_pem + "\n" + t.cert_pem + "\n" + t.key_pem;
  unsigned char md[SHA256_DIGEST_LENGTH];
  SHA256((const unsigned char*)material.data(), material.size(), md);
  *digest = std::string((const char*)md, sizeof(md));
  std::lock_guard<std::mutex> g(g_tls_mu);
  auto it = g_ctx_cache.find(*digest);
  if (it == g_ctx_cache.end()) {
    SSL_CTX* ctx = make_ctx(t);
    SSL_CTX_set_session_cache_mode(ctx, SSL_SESS_CACHE_CLIENT | SSL_SESS_CACHE_NO_INTERNAL_STORE);
    SSL_CTX_sess_set_new_cb(ctx, new_session_cb);
    if (g_ctx_cache.size() >= 16) {  // bounded: credential sets rarely change within a process
      for (auto& kv : g_ctx_cache) SSL_CTX_free(kv.second);
      g_ctx_cache.clear();
    }
    it = g_ctx_cache.emplace(*digest, ctx).first;
  }
  SSL_CTX_up_ref(it->second);
  return it->second;
}

std::string peer_key(int fd) {
  sockaddr_storage ss{};
  socklen_t len = sizeof(ss);
  if (getpeername(fd, (sockaddr*)&ss, &len) != 0) return "";
  char host[INET6_ADDRSTRLEN] = {0};
  int port = 0;
  if (ss.ss_family == AF_INET) {
    inet_ntop(AF_INET, &((sockaddr_in*)&ss)->sin_addr, host, sizeof(host));
    port = ntohs(((sockaddr_in*)&ss)->sin_port);
  } else if (ss.ss_family == AF_INET6) {
    inet_ntop(AF_INET6, &((sockaddr_in6*)&ss)->sin6_addr, host, sizeof(host));
    port = ntohs(((sockaddr_in6*)&ss)->sin6_port);
  } else {
    return "unix";
  }
  return std::string(host) + ":" + std::to_string(port);
}
}  // namespace

// TLS over a non-blocking socket. SSL_read/SSL_write run under ssl_mu_ only for the duration
// of the call; waiting (poll) happens with no lock held, so a reader blocked on an idle
// stream never holds up a concurrent writer. A writer that makes OpenSSL buffer incoming
// records (TLS 1.2 renegotiation) pokes the waker so the parked reader re-checks.
class TlsConn : public Conn {
 public:
  using Conn::write_all;
  TlsConn(int fd, const TlsOptions& t, int timeout_ms) : fd_(fd) {
    try {
      int fl = fcntl(fd_, F_GETFL);
      fcntl(fd_, F_SETFL, fl | O_NONBLOCK);
      bool resume = !reference_timing();
      std::string digest;
      ctx_ = resume ? shared_ctx(t, &digest) : make_ctx(t);
      ssl_ = SSL_new(ctx_);
      if (!ssl_) throw NetError("SSL_new failed");
      if (resume) {
        session_key_ = digest + "|" + t.server_name + "|" + peer_key(fd_);
        SSL_set_app_data(ssl_, &session_key_);
        std::lock_guard<std::mutex> g(g_tls_mu);
        auto it = g_sessions.find(session_key_);
        if (it != g_sessions.end()) SSL_set_session(ssl_, it->second);
      }
      SSL_set_mode(ssl_, SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
      SSL_set_fd(ssl_, fd_);
      if (!t.server_name.empty()) {
        in6_addr a6;
        in_addr a4;
        bool is_ip = inet_pton(AF_INET, t.server_name.c_str(), &a4) == 1 ||
                     inet_pton(AF_INET6, t.server_name.c_str(), &a6) == 1;
        if (!is_ip) SSL_set_tlsext_host_name(ssl_, t.server_name.c_str());  // SNI must not carry an IP
        if (!t.insecure) {
          X509_VERIFY_PARAM* param = SSL_get0_param(ssl_);
          if (is_ip)
            X509_VERIFY_PARAM_set1_ip_asc(param, t.server_name.c_str());
          else
            X509_VERIFY_PARAM_set1_host(param, t.server_name.c_str(), 0);
        }
      }
      int64_t deadline = timeout_ms < 0 ? -1 : mono_ms() + timeout_ms;
      while (true) {
        ERR_clear_error();
        int r = SSL_connect(ssl_);
        if (r == 1) break;
        int err = SSL_get_error(ssl_, r);
        short ev = err == SSL_ERROR_WANT_READ ? POLLIN : err == SSL_ERROR_WANT_WRITE ? POLLOUT : 0;
        if (!ev) {
          std::string msg = ssl_error_string();
          long vr = SSL_get_verify_result(ssl_);
          if (vr != X509_V_OK) msg += std::string(" (certificate verify: ") + X509_verify_cert_error_string(vr) + ")";
          if (msg.empty()) msg = err == SSL_ERROR_SYSCALL ? "connection closed by peer" : "unknown error";
          throw NetError("tls handshake failed: " + msg);
        }
        int left = remaining_ms(deadline);
        if (left == 0 || wait_fd(fd_, ev, left) == 0) throw NetError("tls handshake timed out");
      }
      stats().tls_handshakes++;
      if (SSL_session_reused(ssl_)) stats().tls_resumed++;
    } catch (...) {
      cleanup();
      throw;
    }
  }
  ~TlsConn() override { cleanup(); }

  ssize_t read(void* buf, size_t n, int timeout_ms) override {
    std::lock_guard<std::mutex> g(rmu_);
    int64_t deadline = timeout_ms < 0 ? -1 : mono_ms() + timeout_ms;
    int want = (int)std::min<size_t>(n, INT_MAX);
    while (true) {
      if (shut_.load()) return 0;
      int r, err = 0;
      unsigned long reason = 0;
      {
        std::lock_guard<std::mutex> s(ssl_mu_);
        ERR_clear_error();
        r = SSL_read(ssl_, buf, want);
        if (r <= 0) {
          err = SSL_get_error(ssl_, r);
          reason = ERR_peek_error();
        }
      }
      if (r > 0) return r;
      short ev;
      if (err == SSL_ERROR_WANT_READ) {
        ev = POLLIN;
      } else if (err == SSL_ERROR_WANT_WRITE) {
        ev = POLLOUT;
      } else if (err == SSL_ERROR_ZERO_RETURN || (err == SSL_ERROR_SYSCALL && reason == 0)) {
        return 0;  // close_notify, or the peer dropped the TCP connection
      } else {
#ifdef SSL_R_UNEXPECTED_EOF_WHILE_READING
        if (ERR_GET_REASON(reason) == SSL_R_UNEXPECTED_EOF_WHILE_READING) return 0;
#endif
        return -1;
      }
      int left = remaining_ms(deadline);
      if (left == 0) return -2;
      int pr = wait_fd_or_wake(fd_, ev, wake_, left);
      if (pr == 0) return -2;
      if (pr < 0) return -1;
    }
  }

  bool write_all(const void* d, size_t n) override {
    std::lock_guard<std::mutex> g(wmu_);
    const char* p = (const char*)d;
    while (n) {
      if (shut_.load()) return false;
      int w, err = 0;
      bool pending;
      {
        std::lock_guard<std::mutex> s(ssl_mu_);
        ERR_clear_error();
        w = SSL_write(ssl_, p, (int)std::min<size_t>(n, 1u << 30));
        if (w <= 0) err = SSL_get_error(ssl_, w);
        pending = SSL_has_pending(ssl_) == 1;
      }
      if (pending) wake_.poke();  // we pulled records the reader has to see
      if (w > 0) {
        p += w;
        n -= (size_t)w;
        continue;
      }
      if (err == SSL_ERROR_WANT_WRITE) {
        if (wait_fd(fd_, POLLOUT, 1000) < 0) return false;
      } else if (err == SSL_ERROR_WANT_READ) {
        // handshake traffic the reader thread may consume first: re-check soon
        if (wait_fd(fd_, POLLIN, 20) < 0) return false;
      } else {
        return false;
      }
    }
    return true;
  }

  void shutdown() override {
    shut_ = true;
    ::shutdown(fd_, SHUT_RDWR);
    wake_.poke();
  }
  int fd() const override { return fd_; }

  bool stale() override {
    struct pollfd pf{fd_, POLLIN, 0};
    int r = ::poll(&pf, 1, 0);
    if (r == 0) return false;
    if (r < 0 || (pf.revents & (POLLERR | POLLHUP | POLLNVAL))) return true;
    // readable: TLS 1.3 session tickets are fine, application data or EOF is not
    std::lock_guard<std::mutex> s(ssl_mu_);
    char c;
    ERR_clear_error();
    int x = SSL_peek(ssl_, &c, 1);
    if (x > 0) return true;
    return SSL_get_error(ssl_, x) != SSL_ERROR_WANT_READ;
  }

 private:
  void cleanup() {
    if (ssl_) {
      SSL_shutdown(ssl_);  // best effort close_notify (non-blocking)
      SSL_free(ssl_);
      ssl_ = nullptr;
    }
    if (ctx_) SSL_CTX_free(ctx_);
    ctx_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  int fd_;
  plat::Waker wake_;
  std::string session_key_;  // SSL app data: where new_session_cb files this peer's tickets
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  std::mutex rmu_, wmu_, ssl_mu_;
  std::atomic<bool> shut_{false};
};

// TCP connect with timeout; returns a blocking fd with TCP_NODELAY. Names resolve through
// core/resolve (no NSS: the release binary is static); getaddrinfo is the last resort.
int dial_fd(const std::string& host, int port, int timeout_ms) {
  std::string rerr;
  std::vector<Address> addrs = resolve(host, port, &rerr);
  if (addrs.empty()) {
    struct addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    struct addrinfo* res = nullptr;
    std::string h = host;
    if (h.size() > 2 && h.front() == '[' && h.back() == ']') h = h.substr(1, h.size() - 2);
    int rc = getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (rc != 0) throw NetError("dial tcp " + host + ":" + std::to_string(port) + ": lookup " + h + ": " + rerr);
    for (auto* ai = res; ai; ai = ai->ai_next) {
      Address a;
      a.family = ai->ai_family;
      std::memcpy(&a.addr, ai->ai_addr, ai->ai_addrlen);
      a.len = ai->ai_addrlen;
      addrs.push_back(a);
    }
    freeaddrinfo(res);
  }
  int fd = -1;
  std::string last_err = "no addresses";
  for (auto& a : addrs) {
    fd = plat::socket_cloexec(a.family, SOCK_STREAM);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int r = ::connect(fd, (struct sockaddr*)&a.addr, a.len);
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
  if (fd < 0) throw NetError("dial tcp " + host + ":" + std::to_string(port) + ": " + last_err);
  stats().tcp_dials++;
  return fd;
}

std::string host_port(const std::string& host, int port) {
  bool v6 = host.find(':') != std::string::npos && host.front() != '[';
  return (v6 ? "[" + host + "]" : host) + ":" + std::to_string(port);
}

// HTTP CONNECT tunnel through an http:// proxy; returns the tunnelled fd.
int connect_via_proxy(const std::string& proxy_url, const std::string& host, int port, int timeout_ms) {
  std::string rest = proxy_url;
  size_t sp = rest.find("://");
  std::string scheme = sp == std::string::npos ? "http" : to_lower(rest.substr(0, sp));
  if (scheme != "http") throw NetError("unsupported proxy scheme " + scheme + " (only http:// proxies)");
  std::string auth_hdr;
  std::string authority = sp == std::string::npos ? rest : rest.substr(sp + 3);
  authority = authority.substr(0, authority.find('/'));
  size_t at = authority.rfind('@');
  if (at != std::string::npos) {
    auth_hdr = "Proxy-Authorization: Basic " + base64_encode(url_decode(authority.substr(0, at))) + "\r\n";
  }
  Url pu = Url::parse(proxy_url);
  if (pu.port == 0 || pu.port == 443) pu.port = sp == std::string::npos || pu.port == 0 ? 80 : pu.port;
  PlainConn pc(dial_fd(pu.host, pu.port, timeout_ms));
  std::string target = host_port(host, port);
  std::string req = "CONNECT " + target + " HTTP/1.1\r\nHost: " + target + "\r\n" + auth_hdr + "\r\n";
  if (!pc.write_all(req)) throw NetError("proxy " + pu.host + ": write CONNECT failed");
  Response resp;
  std::string left;
  if (!read_response_head(pc, &resp, &left, timeout_ms)) throw NetError("proxy " + pu.host + ": no CONNECT response");
  if (resp.status != 200)
    throw NetError("proxy " + pu.host + " refused CONNECT " + target + ": " + std::to_string(resp.status) + " " +
                   resp.reason);
  if (!left.empty()) throw NetError("proxy " + pu.host + ": unexpected bytes after CONNECT response");
  stats().proxied++;
  return pc.release();
}

bool parse_ipv4(const std::string& s, uint32_t* out) {
  in_addr a;
  if (inet_pton(AF_INET, s.c_str(), &a) != 1) return false;
  *out = ntohl(a.s_addr);
  return true;
}

}  // namespace

bool Conn::stale() {
  int f = fd();
  if (f < 0) return true;
  struct pollfd pf{f, POLLIN, 0};
  return ::poll(&pf, 1, 0) != 0;  // EOF, error or unsolicited bytes
}

// ---------------------------------------------------------------- proxy

bool no_proxy_matches(const std::string& no_proxy, const std::string& host_in, int port) {
  std::string host = to_lower(host_in);
  if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  for (std::string e : split(no_proxy, ",")) {
    e = to_lower(trim(e));
    if (e.empty()) continue;
    if (e == "*") return true;
    // optional :port
    int eport = 0;
    size_t colon = e.rfind(':');
    if (colon != std::string::npos && e.find(']') == std::string::npos && e.find(':') == colon &&
        e.find('/') == std::string::npos) {
      eport = std::atoi(e.substr(colon + 1).c_str());
      e = e.substr(0, colon);
    }
    if (eport && eport != port) continue;
    size_t slash = e.find('/');
    if (slash != std::string::npos) {  // IPv4 CIDR
      uint32_t net, ip;
      int bits = std::atoi(e.substr(slash + 1).c_str());
      if (parse_ipv4(e.substr(0, slash), &net) && parse_ipv4(host, &ip) && bits >= 0 && bits <= 32) {
        uint32_t mask = bits == 0 ? 0 : 0xFFFFFFFFu << (32 - bits);
        if ((net & mask) == (ip & mask)) return true;
      }
      continue;
    }
    if (e.front() == '.') e = e.substr(1);
    if (host == e) return true;
    if (host.size() > e.size() && ends_with(host, "." + e)) return true;
  }
  return false;
}

static std::string env_first(std::initializer_list<const char*> names) {
  for (auto* n : names) {
    const char* v = getenv(n);
    if (v && *v) return v;
  }
  return "";
}

ProxyConfig ProxyConfig::from_env() {
  ProxyConfig p;
  p.https_proxy = env_first({"HTTPS_PROXY", "https_proxy", "ALL_PROXY", "all_proxy"});
  p.http_proxy = env_first({"HTTP_PROXY", "http_proxy", "ALL_PROXY", "all_proxy"});
  p.no_proxy = env_first({"NO_PROXY", "no_proxy"});
  return p;
}

std::string ProxyConfig::proxy_for(const std::string& scheme, const std::string& host, int port) const {
  std::string p = scheme == "https" || scheme == "wss" ? https_proxy : http_proxy;
  if (p.empty()) return "";
  if (no_proxy_matches(no_proxy, host, port)) return "";
  return p;
}

std::unique_ptr<Conn> dial_tcp(const std::string& host, int port, const TlsOptions& tls, int timeout_ms,
                               const std::string& proxy_url) {
  int fd = proxy_url.empty() ? dial_fd(host, port, timeout_ms) : connect_via_proxy(proxy_url, host, port, timeout_ms);
  if (tls.enabled) {
    TlsOptions t = tls;
    std::string h = host;
    if (h.size() > 2 && h.front() == '[' && h.back() == ']') h = h.substr(1, h.size() - 2);
    if (t.server_name.empty()) t.server_name = h;
    return std::make_unique<TlsConn>(fd, t, timeout_ms);
  }
  return std::make_unique<PlainConn>(fd);
}

std::unique_ptr<Conn> dial_unix(const std::string& path) {
  int fd = plat::socket_cloexec(AF_UNIX, SOCK_STREAM);
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

// ---------------------------------------------------------------- http client

struct HttpClient::State {
  TlsOptions tls;
  mutable std::mutex mu;
  std::map<std::string, std::string> headers;
  std::vector<std::unique_ptr<Conn>> idle;
  bool keepalive = !reference_timing();  // the reference-equivalent column dials per request
  size_t max_idle = 8;
  ProxyConfig proxy = ProxyConfig::from_env();
  std::function<std::unique_ptr<Conn>()> source;
};

HttpClient::HttpClient() : st_(std::make_shared<State>()) {}

HttpClient::HttpClient(const std::string& base_url, TlsOptions tls)
    : url_(Url::parse(base_url)), st_(std::make_shared<State>()) {
  st_->tls = std::move(tls);
  if (url_.scheme == "https" || url_.scheme == "wss") st_->tls.enabled = true;
}

void HttpClient::set_header(const std::string& k, const std::string& v) {
  std::lock_guard<std::mutex> g(st_->mu);
  st_->headers[k] = v;
}

std::map<std::string, std::string> HttpClient::default_headers() const {
  std::lock_guard<std::mutex> g(st_->mu);
  return st_->headers;
}

void HttpClient::set_tls(TlsOptions tls) {
  std::lock_guard<std::mutex> g(st_->mu);
  bool en = st_->tls.enabled;
  st_->tls = std::move(tls);
  st_->tls.enabled = en;
  st_->idle.clear();
}

void HttpClient::set_keepalive(bool on) {
  std::lock_guard<std::mutex> g(st_->mu);
  st_->keepalive = on;
  if (!on) st_->idle.clear();
}

void HttpClient::set_proxy(ProxyConfig p) {
  std::lock_guard<std::mutex> g(st_->mu);
  st_->proxy = std::move(p);
  st_->idle.clear();
}

size_t HttpClient::idle_connections() const {
  std::lock_guard<std::mutex> g(st_->mu);
  return st_->idle.size();
}

void HttpClient::set_conn_source(std::function<std::unique_ptr<Conn>()> source) {
  std::lock_guard<std::mutex> g(st_->mu);
  st_->source = std::move(source);
}

void HttpClient::close_idle() {
  std::vector<std::unique_ptr<Conn>> drop;
  std::lock_guard<std::mutex> g(st_->mu);
  drop.swap(st_->idle);
}

std::unique_ptr<Conn> HttpClient::connect() {
  if (!url_.unix_path.empty()) {
    auto c = dial_unix(url_.unix_path);
    stats().tcp_dials++;  // counted as a dial for reuse statistics
    return c;
  }
  TlsOptions tls;
  std::string proxy;
  {
    std::lock_guard<std::mutex> g(st_->mu);
    tls = st_->tls;
    proxy = st_->proxy.proxy_for(url_.scheme, url_.host, url_.port);
  }
  return dial_tcp(url_.host, url_.port, tls, 15000, proxy);
}

std::unique_ptr<Conn> HttpClient::take_conn(bool* reused) {
  std::vector<std::unique_ptr<Conn>> dead;
  std::function<std::unique_ptr<Conn>()> source;
  {
    std::lock_guard<std::mutex> g(st_->mu);
    while (!st_->idle.empty()) {
      std::unique_ptr<Conn> c = std::move(st_->idle.back());
      st_->idle.pop_back();
      if (c->stale()) {
        dead.push_back(std::move(c));
        continue;
      }
      *reused = true;
      stats().reused++;
      return c;
    }
    source = st_->source;
  }
  *reused = false;
  if (source)
    if (auto c = source()) return c;  // dialed ahead (counted as a dial then)
  return connect();
}

void HttpClient::put_conn(std::unique_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(st_->mu);
  if (!st_->keepalive || st_->idle.size() >= st_->max_idle) return;
  st_->idle.push_back(std::move(c));
}

namespace {

bool read_head(Conn& c, Response* r, std::string* rest, int timeout_ms, bool* got_any, bool* timed_out = nullptr) {
  std::string buf = *rest;
  rest->clear();
  size_t end;
  while ((end = buf.find("\r\n\r\n")) == std::string::npos) {
    char tmp[8192];
    ssize_t n = c.read(tmp, sizeof(tmp), timeout_ms);
    if (n == -2 && timed_out) *timed_out = true;
    if (n <= 0) return false;
    if (got_any) *got_any = true;
    buf.append(tmp, (size_t)n);
    if (buf.size() > (1 << 20)) return false;
  }
  std::string head = buf.substr(0, end);
  *rest = buf.substr(end + 4);
  auto lines = split(head, "\r\n");
  if (lines.empty()) return false;
  auto sl = split(lines[0], " ");
  if (sl.size() < 2) return false;
  r->version = sl[0];
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

std::string build_request(const Url& url, const std::map<std::string, std::string>& defaults, const Request& r,
                          bool keepalive) {
  std::string base = url.path;
  if (!base.empty() && base.back() == '/' && !r.path.empty() && r.path[0] == '/') base.pop_back();
  std::string path = base + r.path;
  if (path.empty()) path = "/";
  std::string host = url.unix_path.empty() ? url.host : "localhost";
  if (url.unix_path.empty()) {
    bool default_port = (url.port == 443 && (url.scheme == "https" || url.scheme == "wss")) ||
                        (url.port == 80 && (url.scheme == "http" || url.scheme == "ws"));
    if (!default_port && url.port) host = host_port(url.host, url.port);
  }
  std::string out = r.method + " " + path + " HTTP/1.1\r\nHost: " + host + "\r\n";
  std::map<std::string, std::string> hdrs = defaults;
  for (auto& kv : r.headers) hdrs[kv.first] = kv.second;
  for (auto& kv : hdrs) out += kv.first + ": " + kv.second + "\r\n";
  if (r.body_writer) {
    if (!hdrs.count("Transfer-Encoding")) out += "Transfer-Encoding: chunked\r\n";
  } else if (!hdrs.count("Content-Length") &&
             (!r.body.empty() || r.method == "POST" || r.method == "PUT" || r.method == "PATCH")) {
    out += "Content-Length: " + std::to_string(r.body.size()) + "\r\n";
  }
  if (!hdrs.count("Connection") && !keepalive) out += "Connection: close\r\n";
  out += "\r\n";
  return out;
}

}  // namespace

bool read_response_head(Conn& c, Response* r, std::string* rest, int timeout_ms) {
  return read_head(c, r, rest, timeout_ms, nullptr);
}

Response HttpClient::stream(Request r, const std::function<bool(const std::string&)>& on_data) {
  stats().requests++;
  std::map<std::string, std::string> defaults;
  bool keepalive;
  {
    std::lock_guard<std::mutex> g(st_->mu);
    defaults = st_->headers;
    keepalive = st_->keepalive;
  }
  std::string head = build_request(url_, defaults, r, keepalive);
  std::unique_ptr<Conn> c;
  Response resp;
  std::string rest;
  const bool idempotent = r.method == "GET" || r.method == "HEAD" || r.method == "PUT" || r.method == "DELETE" ||
                          r.method == "OPTIONS";
  for (int attempt = 0;; ++attempt) {
    bool reused = false;
    c = take_conn(&reused);
    bool wrote = c->write_all(head);
    if (wrote && r.body_writer) {
      // chunked transfer encoding: the body is produced while it is sent (bounded memory)
      Conn* cp = c.get();
      char hex[32];
      wrote = r.body_writer([&](const char* d, size_t n) {
        if (n == 0) return true;
        int k = std::snprintf(hex, sizeof(hex), "%zx\r\n", n);
        return cp->write_all(std::string(hex, (size_t)k)) && cp->write_all(std::string(d, n)) && cp->write_all("\r\n");
      }) && c->write_all("0\r\n\r\n");
    } else if (wrote && !r.body.empty()) {
      wrote = c->write_all(r.body);
    }
    bool got_any = false, timed_out = false;
    resp = Response();
    rest.clear();
    if (wrote && read_head(*c, &resp, &rest, r.timeout_ms, &got_any, &timed_out)) break;
    // A pooled connection the server closed while it sat idle: retry once on a fresh one —
    // only when the connection was found dead (EOF / reset, never a timeout: a slow server
    // would get the request twice) and the request is safe to repeat or never went out.
    // Streamed bodies cannot be replayed.
    if (reused && !got_any && !timed_out && attempt == 0 && !r.body_writer && (idempotent || !wrote)) continue;
    if (!wrote) throw NetError("write request failed: " + r.method + " " + r.path);
    throw NetError(timed_out ? "timeout waiting for the response: " + r.method + " " + r.path
                             : "read response failed: " + r.path);
  }
  bool reusable = keepalive && resp.version == "HTTP/1.1" &&
                  to_lower(resp.header("connection")).find("close") == std::string::npos;
  if (r.method == "HEAD" || resp.status == 204 || resp.status == 304 || (resp.status >= 100 && resp.status < 200)) {
    if (reusable && rest.empty()) put_conn(std::move(c));
    return resp;
  }
  bool chunked = to_lower(resp.header("transfer-encoding")).find("chunked") != std::string::npos;
  std::string cl = resp.header("content-length");
  int64_t remaining = cl.empty() ? -1 : std::atoll(cl.c_str());
  std::string* err_body = r.errors_to_body && resp.status >= 400 ? &resp.body : nullptr;
  auto deliver = [&](const std::string& d) {
    if (err_body) {
      if (err_body->size() < (1u << 20)) *err_body += d;
      return true;
    }
    return d.empty() || on_data(d);
  };
  char tmp[65536];
  if (chunked) {
    std::string buf = std::move(rest);
    size_t off = 0;  // consumed prefix of buf
    auto need = [&](size_t bytes) {
      while (buf.size() - off < bytes) {
        ssize_t n = c->read(tmp, sizeof(tmp), r.timeout_ms);
        if (n <= 0) return false;
        buf.append(tmp, (size_t)n);
      }
      return true;
    };
    auto line = [&](std::string* out) {
      size_t le;
      while ((le = buf.find("\r\n", off)) == std::string::npos) {
        ssize_t n = c->read(tmp, sizeof(tmp), r.timeout_ms);
        if (n <= 0) return false;
        buf.append(tmp, (size_t)n);
      }
      *out = buf.substr(off, le - off);
      off = le + 2;
      return true;
    };
    while (true) {
      std::string sz_line;
      if (!line(&sz_line)) return resp;
      size_t sz = std::strtoul(sz_line.c_str(), nullptr, 16);
      if (sz == 0) {
        std::string trailer;
        while (line(&trailer) && !trailer.empty()) {
        }
        if (trailer.empty() && off == buf.size() && reusable) put_conn(std::move(c));
        return resp;
      }
      if (!need(sz + 2)) {
        deliver(buf.substr(off, std::min(buf.size() - off, sz)));
        return resp;
      }
      if (!deliver(buf.substr(off, sz))) return resp;
      off += sz + 2;
      if (off > (1 << 20)) {
        buf.erase(0, off);
        off = 0;
      }
    }
  }
  if (!rest.empty()) {
    if (remaining >= 0 && (int64_t)rest.size() > remaining) {
      rest.resize((size_t)remaining);
      reusable = false;
    }
    if (remaining >= 0) remaining -= (int64_t)rest.size();
    if (!deliver(rest)) return resp;
  }
  if (remaining < 0) reusable = false;  // body delimited by EOF
  while (remaining != 0) {
    size_t want = remaining > 0 ? (size_t)std::min<int64_t>(remaining, (int64_t)sizeof(tmp)) : sizeof(tmp);
    ssize_t n = c->read(tmp, want, r.timeout_ms);
    if (n <= 0) {
      reusable = false;
      break;
    }
    if (remaining > 0) remaining -= n;
    if (!deliver(std::string(tmp, (size_t)n))) {
      if (remaining != 0) reusable = false;
      break;
    }
  }
  if (reusable && remaining == 0) put_conn(std::move(c));
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

std::string websocket_accept(const std::string& key) {
  std::string in = key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";
  unsigned char md[SHA_DIGEST_LENGTH];
  SHA1((const unsigned char*)in.data(), in.size(), md);
  return base64_encode(std::string((const char*)md, sizeof(md)));
}

std::unique_ptr<WebSocket> WebSocket::connect(HttpClient& http, const std::string& path,
                                              const std::vector<std::string>& protocols, int timeout_ms,
                                              std::unique_ptr<Conn> conn) {
  auto c = conn && !conn->stale() ? std::move(conn) : http.connect();
  std::string key = base64_encode(random_string(16));
  Request r;
  r.method = "GET";
  r.path = path;
  r.headers = {{"Connection", "Upgrade"},
               {"Upgrade", "websocket"},
               {"Sec-WebSocket-Version", "13"},
               {"Sec-WebSocket-Key", key}};
  if (!protocols.empty()) r.headers.push_back({"Sec-WebSocket-Protocol", join(protocols, ", ")});
  std::string req = build_request(http.url(), http.default_headers(), r, true);
  if (!c->write_all(req)) throw NetError("websocket: write handshake failed");
  Response resp;
  std::string rest;
  if (!read_response_head(*c, &resp, &rest, timeout_ms)) throw NetError("websocket: no handshake response");
  if (resp.status != 101) {
    // read the error body for a useful message: Content-Length bytes when the server sized it
    // (a keep-alive 429 would otherwise hold us for the read timeout), else up to EOF
    std::string body = rest;
    std::string cl = resp.header("content-length");
    size_t want = cl.empty() ? 65536 : std::min<size_t>(65536, (size_t)std::strtoull(cl.c_str(), nullptr, 10));
    char tmp[4096];
    while (body.size() < want) {
      ssize_t n = c->read(tmp, sizeof(tmp), 2000);
      if (n <= 0) break;
      body.append(tmp, (size_t)n);
    }
    throw UpgradeError(resp.status,
                       "websocket upgrade failed: " + std::to_string(resp.status) + " " + resp.reason + ": " + body,
                       resp.header("retry-after"));
  }
  if (resp.header("sec-websocket-accept") != websocket_accept(key))
    throw NetError("websocket upgrade failed: bad Sec-WebSocket-Accept from server");
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
  size_t n = payload.size();
  f.reserve(n + 14);
  f.push_back((char)(0x80 | op));
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
  const unsigned char* m = (const unsigned char*)mask.data();
  const unsigned char* src = (const unsigned char*)payload.data();
  unsigned char* dst = (unsigned char*)&f[off];
  for (size_t i = 0; i < n; ++i) dst[i] = src[i] ^ m[i & 3];
  return c_->write_all(f);
}

bool WebSocket::read_exact(char* out, size_t n, int timeout_ms) {
  while (buf_.size() - buf_off_ < n) {
    if (buf_off_ > 0 && buf_off_ >= buf_.size() / 2) {
      buf_.erase(0, buf_off_);
      buf_off_ = 0;
    }
    char tmp[65536];
    ssize_t r = c_->read(tmp, sizeof(tmp), timeout_ms);
    if (r <= 0) return false;
    buf_.append(tmp, (size_t)r);
  }
  std::memcpy(out, buf_.data() + buf_off_, n);
  buf_off_ += n;
  if (buf_off_ == buf_.size()) {
    buf_.clear();
    buf_off_ = 0;
  }
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
    if (len > kMaxFrame || msg.size() + len > kMaxFrame) {
      // a frame this size is not a Kubernetes stream message: refuse instead of allocating it
      send(std::string("\x03\xf1", 2), Close);  // 1009 message too big
      std::lock_guard<std::mutex> g(wmu_);
      closed_ = true;
      return false;
    }
    char mask[4] = {0, 0, 0, 0};
    if (masked && !read_exact(mask, 4, timeout_ms)) return false;
    std::string data(len, '\0');
    if (len && !read_exact(&data[0], len, timeout_ms)) return false;
    if (masked)
      for (size_t i = 0; i < len; ++i) data[i] ^= mask[i & 3];
    if (op == Close) {
      if (data.size() >= 2) close_code_ = ((unsigned char)data[0] << 8) | (unsigned char)data[1];
      send(data.substr(0, 2), Close);  // echo the close (RFC 6455 §5.5.1)
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
