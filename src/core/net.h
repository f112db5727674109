// Network transport: TCP / TLS (OpenSSL) / unix sockets, an HTTP/1.1 client and an RFC 6455
// WebSocket client. Replaces client-go's REST + SPDY transports (kubectl/client.go,
// kubectl/exec.go) and the Docker Engine client (docker/client.go) — no third-party HTTP stack
// is available offline.
#pragma once

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

struct TlsOptions {
  bool enabled = false;
  bool insecure = false;
  std::string ca_pem, cert_pem, key_pem;
  std::string server_name;
};

// A connected byte stream.
class Conn {
 public:
  virtual ~Conn() = default;
  virtual ssize_t read(void* buf, size_t n, int timeout_ms = -1) = 0;  // 0 EOF, -1 err, -2 timeout
  virtual bool write_all(const void* d, size_t n) = 0;
  bool write_all(const std::string& s) { return write_all(s.data(), s.size()); }
  virtual void shutdown() = 0;  // unblock readers (other threads)
  virtual int fd() const = 0;
};

std::unique_ptr<Conn> dial_tcp(const std::string& host, int port, const TlsOptions& tls, int timeout_ms = 15000);
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
  std::map<std::string, std::string> headers;  // lower-case keys
  std::string body;
  std::string header(const std::string& k) const;
};

struct Request {
  std::string method = "GET";
  std::string path = "/";
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
  int timeout_ms = 60000;
};

// Endpoint = where to connect + how (base URL, TLS, default headers).
class HttpClient {
 public:
  HttpClient() = default;
  HttpClient(const std::string& base_url, TlsOptions tls = {});
  void set_header(const std::string& k, const std::string& v) { default_headers_[k] = v; }
  Response request(Request r);
  Response get(const std::string& path) {
    Request r;
    r.path = path;
    return request(r);
  }
  // Streaming: body chunks delivered to `on_data` (return false to stop). Returns status.
  Response stream(Request r, const std::function<bool(const std::string&)>& on_data);
  // Opens a raw connection to the endpoint (used for upgrades).
  std::unique_ptr<Conn> connect();
  const Url& url() const { return url_; }
  const std::map<std::string, std::string>& default_headers() const { return default_headers_; }

 private:
  Url url_;
  TlsOptions tls_;
  std::map<std::string, std::string> default_headers_;
};

std::string url_encode(const std::string& s);

// Reads an HTTP response head from conn (leftover bytes after the head in *rest).
bool read_response_head(Conn& c, Response* r, std::string* rest, int timeout_ms);

class WebSocket {
 public:
  // Performs the client handshake on `path` with the given subprotocols; throws on failure.
  static std::unique_ptr<WebSocket> connect(HttpClient& http, const std::string& path,
                                            const std::vector<std::string>& protocols,
                                            int timeout_ms = 30000);
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

 private:
  bool read_exact(char* buf, size_t n, int timeout_ms);
  std::unique_ptr<Conn> c_;
  std::string buf_;
  std::mutex wmu_;
  bool closed_ = false;
};

}  // namespace net
}  // namespace ds
