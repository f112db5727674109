// Network transport: TCP / TLS (OpenSSL) / unix sockets, an HTTP/1.1 client with a keep-alive
// connection pool and CONNECT-proxy support, and an RFC 6455 WebSocket client. Replaces
// client-go's REST + SPDY transports (kubectl/client.go, kubectl/exec.go) and the Docker Engine
// client (docker/client.go) — no third-party HTTP stack is available offline.
//
// Concurrency contract: a Conn may be read by one thread while another writes to it (the exec
// and port-forward pumps do exactly that). TLS connections are non-blocking underneath; the
// OpenSSL object is only ever touched under a short lock and never across a poll(), so a reader
// parked waiting for bytes can not starve a writer (the round-1 wss stdin deadlock).
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace ds {
namespace net {

struct NetError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// A WebSocket upgrade answered with a non-101 status (e.g. 401 → refresh credentials, 429 →
// wait `retry_after` and try again).
struct UpgradeError : NetError {
  int status;
  std::string retry_after;  // the response's Retry-After header ("" if none)
  UpgradeError(int st, const std::string& msg, std::string ra = "")
      : NetError(msg), status(st), retry_after(std::move(ra)) {}
};

struct TlsOptions {
  bool enabled = false;
  bool insecure = false;
  std::string ca_pem, cert_pem, key_pem;
  std::string server_name;
};

// Process-wide transport counters (reported in trace spans; tests assert keep-alive reuse).
struct Stats {
  std::atomic<int64_t> tcp_dials{0};
  std::atomic<int64_t> tls_handshakes{0};
  std::atomic<int64_t> tls_resumed{0};  // of those, abbreviated (session resumption)
  std::atomic<int64_t> requests{0};
  std::atomic<int64_t> reused{0};
  std::atomic<int64_t> proxied{0};
};
Stats& stats();

// A connected byte stream.
class Conn {
 public:
  virtual ~Conn() = default;
  virtual ssize_t read(void* buf, size_t n, int timeout_ms = -1) = 0;  // 0 EOF, -1 err, -2 timeout
  virtual bool write_all(const void* d, size_t n) = 0;
  bool write_all(const std::string& s) { return write_all(s.data(), s.size()); }
  virtual void shutdown() = 0;  // unblock readers (other threads)
  virtual int fd() const = 0;
  // True when the peer has closed or sent unsolicited bytes (an idle pooled conn is stale).
  virtual bool stale();
};

// Proxy selection from HTTPS_PROXY/https_proxy/HTTP_PROXY/http_proxy/ALL_PROXY and
// NO_PROXY/no_proxy ("*", domain suffixes, ".suffix", exact hosts, host:port, IPv4 CIDRs).
struct ProxyConfig {
  std::string https_proxy, http_proxy, no_proxy;
  static ProxyConfig from_env();
  // Proxy URL to use for scheme://host:port, or "" for a direct connection.
  std::string proxy_for(const std::string& scheme, const std::string& host, int port) const;
};
bool no_proxy_matches(const std::string& no_proxy, const std::string& host, int port);

std::unique_ptr<Conn> dial_tcp(const std::string& host, int port, const TlsOptions& tls, int timeout_ms = 15000,
                               const std::string& proxy_url = "");
std::unique_ptr<Conn> dial_unix(const std::string& path);

struct Url {
  std::string scheme, host, path;  // path includes query
  int port = 0;
  std::string unix_path;  // unix:///var/run/docker.sock
  static Url parse(const std::string& s);
};

struct Response {
  int status = 0;
  std::string reason;
  std::string version;  // "HTTP/1.1"
  std::map<std::string, std::string> headers;  // lower-case keys
  std::string body;
  std::string header(const std::string& k) const;
};

struct Request {
  std::string method = "GET";
  std::string path = "/";
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
  // Streamed body (instead of `body`): called once with a sink that sends what it is given as
  // chunked transfer encoding; returns false to abort the request. Never retried.
  std::function<bool(const std::function<bool(const char*, size_t)>&)> body_writer;
  int timeout_ms = 60000;
  // stream(): for status >= 400 collect the body into Response::body instead of on_data
  bool errors_to_body = false;
};

// Endpoint = where to connect + how (base URL, TLS, default headers, proxy). Copies share one
// connection pool and header set (thread-safe).
class HttpClient {
 public:
  HttpClient();
  HttpClient(const std::string& base_url, TlsOptions tls = {});
  void set_header(const std::string& k, const std::string& v);
  void set_tls(TlsOptions tls);  // new client credentials: drops pooled connections
  Response request(Request r);
  Response get(const std::string& path) {
    Request r;
    r.path = path;
    return request(r);
  }
  // Streaming: body chunks delivered to `on_data` (return false to stop). Returns status
  // and headers; the connection goes back to the pool only if the body was fully consumed.
  Response stream(Request r, const std::function<bool(const std::string&)>& on_data);
  // Opens a raw (unpooled) connection to the endpoint (used for upgrades).
  std::unique_ptr<Conn> connect();
  const Url& url() const { return url_; }
  std::map<std::string, std::string> default_headers() const;
  void set_keepalive(bool on);
  void set_proxy(ProxyConfig p);
  size_t idle_connections() const;
  void close_idle();
  // Where a request gets a connection when none is idle, before dialing one: a pool of
  // connections dialed ahead of time (nullptr from it: dial).
  void set_conn_source(std::function<std::unique_ptr<Conn>()> source);

 private:
  struct State;
  std::unique_ptr<Conn> take_conn(bool* reused);
  void put_conn(std::unique_ptr<Conn> c);
  Url url_;
  std::shared_ptr<State> st_;
};

std::string url_encode(const std::string& s);

// Reads an HTTP response head from conn (leftover bytes after the head in *rest).
bool read_response_head(Conn& c, Response* r, std::string* rest, int timeout_ms);

// RFC 6455 §4.2.2: base64(SHA-1(key + GUID)).
std::string websocket_accept(const std::string& key);

class WebSocket {
 public:
  static constexpr uint64_t kMaxFrame = 64ull << 20;  // refuse larger peer frames
  // Performs the client handshake on `path` with the given subprotocols; throws on failure.
  // `conn`: an already dialed (TLS-established) connection to the endpoint to upgrade instead of
  // dialing a new one; ignored when stale.
  static std::unique_ptr<WebSocket> connect(HttpClient& http, const std::string& path,
                                            const std::vector<std::string>& protocols,
                                            int timeout_ms = 30000, std::unique_ptr<Conn> conn = nullptr);
  explicit WebSocket(std::unique_ptr<Conn> c, std::string leftover = "");
  ~WebSocket();
  enum Op { Cont = 0, Text = 1, Binary = 2, Close = 8, Ping = 9, Pong = 10 };
  bool send(const std::string& payload, Op op = Binary);
  // Receives the next data message (control frames handled internally). false on close/EOF.
  bool recv(std::string* payload, Op* op = nullptr, int timeout_ms = -1);
  void close();
  void shutdown();  // unblock a reader thread
  const std::string& protocol() const { return protocol_; }
  std::string protocol_;
  // Close code / reason received from the peer (0 if none).
  int close_code() const { return close_code_; }

 private:
  bool read_exact(char* buf, size_t n, int timeout_ms);
  std::unique_ptr<Conn> c_;
  std::string buf_;
  size_t buf_off_ = 0;
  std::mutex wmu_;
  bool closed_ = false;
  int close_code_ = 0;
};

}  // namespace net
}  // namespace ds
