// HTTP client behaviour against scripted local servers (keep-alive retry rules, chunked request
// bodies) and the NSS-free resolver's pieces.
#include <arpa/inet.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <functional>
#include <thread>

#include "core/net.h"
#include "core/resolve.h"
#include "core/fs.h"
#include "core/strutil.h"
#include "deploy/sprig_crypto.h"
#include "kube/client.h"
#include "services/services.h"
#include "testing.h"

using namespace ds;

namespace {

// One-thread TCP server: `serve` gets each accepted connection's fd in turn.
struct ScriptedServer {
  int lfd = -1, port = 0;
  std::thread t;
  std::atomic<bool> stop{false};
  explicit ScriptedServer(std::function<void(int fd, int index)> serve) {
    lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ::bind(lfd, (sockaddr*)&a, sizeof(a));
    socklen_t len = sizeof(a);
    getsockname(lfd, (sockaddr*)&a, &len);
    port = ntohs(a.sin_port);
    ::listen(lfd, 8);
    t = std::thread([this, serve] {
      for (int i = 0; !stop; ++i) {
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) return;
        serve(fd, i);
        ::close(fd);
      }
    });
  }
  ~ScriptedServer() {
    stop = true;
    ::shutdown(lfd, SHUT_RDWR);
    ::close(lfd);
    if (t.joinable()) t.join();
  }
  std::string url() const { return "http://127.0.0.1:" + std::to_string(port); }
};

// Reads one request (head + Content-Length or chunked body); "" on EOF.
std::string read_request(int fd, std::string* body) {
  std::string buf;
  char tmp[65536];
  size_t end;
  while ((end = buf.find("\r\n\r\n")) == std::string::npos) {
    ssize_t n = ::read(fd, tmp, sizeof(tmp));
    if (n <= 0) return "";
    buf.append(tmp, (size_t)n);
  }
  std::string head = buf.substr(0, end);
  std::string rest = buf.substr(end + 4);
  auto more = [&](size_t want) {
    while (rest.size() < want) {
      ssize_t n = ::read(fd, tmp, sizeof(tmp));
      if (n <= 0) return false;
      rest.append(tmp, (size_t)n);
    }
    return true;
  };
  body->clear();
  std::string low = to_lower(head);
  size_t cl = low.find("content-length:");
  if (low.find("transfer-encoding: chunked") != std::string::npos) {
    while (true) {
      size_t le;
      while ((le = rest.find("\r\n")) == std::string::npos)
        if (!more(rest.size() + 1)) return head;
      size_t sz = std::strtoul(rest.substr(0, le).c_str(), nullptr, 16);
      rest.erase(0, le + 2);
      if (!more(sz + 2)) return head;
      body->append(rest.substr(0, sz));
      rest.erase(0, sz + 2);
      if (sz == 0) break;
    }
  } else if (cl != std::string::npos) {
    size_t n = (size_t)std::atoll(low.c_str() + cl + 15);
    more(n);
    *body = rest.substr(0, n);
  }
  return head;
}

void respond(int fd, const std::string& body) {
  std::string r = "HTTP/1.1 200 OK\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
  ::write(fd, r.data(), r.size());
}

void respond_status(int fd, int status, const std::string& retry_after) {
  std::string body = "{\"kind\":\"Status\",\"code\":" + std::to_string(status) + "}";
  std::string r = "HTTP/1.1 " + std::to_string(status) + " X\r\nContent-Type: application/json\r\n" +
                  (retry_after.empty() ? "" : "Retry-After: " + retry_after + "\r\n") +
                  "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
  ::write(fd, r.data(), r.size());
}

// An API server that answers the first `fail` requests with `status` (+ Retry-After), then 200;
// counts requests per method.
struct ThrottlingServer {
  std::atomic<int> seen{0}, posts{0}, gets{0};
  int fail, status;
  std::string retry_after;
  ScriptedServer srv;
  ThrottlingServer(int fail_, int status_, std::string ra)
      : fail(fail_), status(status_), retry_after(std::move(ra)), srv([this](int fd, int) {
          std::string body;
          while (true) {
            std::string head = read_request(fd, &body);
            if (head.empty()) return;
            (starts_with(head, "POST") ? posts : gets)++;
            if (seen++ < fail)
              respond_status(fd, status, retry_after);
            else
              respond(fd, "{\"kind\":\"Pod\"}");
          }
        }) {}
  kube::RestConfig rc() const {
    kube::RestConfig c;
    c.server = srv.url();
    return c;
  }
};

}  // namespace

// a request that outlasts its timeout on a pooled connection must not be sent again
// (a POST creating a pod would be created twice); a connection found dead is retried.
TEST(http_pooled_timeout_is_not_retried) {
  std::atomic<int> posts{0};
  ScriptedServer srv([&](int fd, int) {
    std::string body;
    while (true) {
      std::string head = read_request(fd, &body);
      if (head.empty()) return;
      if (starts_with(head, "POST")) {
        posts++;
        std::this_thread::sleep_for(std::chrono::milliseconds(900));  // slower than the client waits
        return;
      }
      respond(fd, "ok");
    }
  });
  net::HttpClient c(srv.url());
  EXPECT_EQ(c.get("/warm").status, 200);  // leaves a pooled keep-alive connection
  net::Request post;
  post.method = "POST";
  post.path = "/api/v1/namespaces/x/pods";
  post.body = "{}";
  post.timeout_ms = 300;
  EXPECT_THROWS(c.request(post));
  std::this_thread::sleep_for(std::chrono::milliseconds(1200));
  EXPECT_EQ(posts.load(), 1);
}

TEST(http_dead_pooled_connection_is_retried_once) {
  ScriptedServer srv([&](int fd, int) {
    std::string body;
    if (read_request(fd, &body).empty()) return;
    respond(fd, "first");  // then close: the pooled connection is dead before the next use
  });
  net::HttpClient c(srv.url());
  EXPECT_EQ(c.get("/a").body, std::string("first"));
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  net::Response r = c.get("/b");  // written into a dead pooled connection, retried on a new one
  EXPECT_EQ(r.status, 200);
  EXPECT_EQ(r.body, std::string("first"));
}

TEST(http_streamed_request_body_is_chunked) {
  ScriptedServer srv([&](int fd, int) {
    std::string body;
    std::string head = read_request(fd, &body);
    if (head.empty()) return;
    bool chunked = to_lower(head).find("transfer-encoding: chunked") != std::string::npos;
    respond(fd, std::string(chunked ? "chunked:" : "sized:") + std::to_string(body.size()) + ":" +
                    (body.size() > 3 ? body.substr(body.size() - 3) : body));
  });
  net::HttpClient c(srv.url());
  net::Request r;
  r.method = "POST";
  r.path = "/build";
  size_t produced = 0;
  r.body_writer = [&](const std::function<bool(const char*, size_t)>& sink) {
    std::string block(100000, 'x');
    for (int i = 0; i < 50; ++i) {
      if (i == 49) block.replace(block.size() - 3, 3, "end");
      if (!sink(block.data(), block.size())) return false;
      produced += block.size();
    }
    return true;
  };
  net::Response resp = c.request(r);
  EXPECT_EQ(resp.status, 200);
  EXPECT_EQ(resp.body, std::string("chunked:5000000:end"));
  EXPECT_EQ(produced, (size_t)5000000);
}

TEST(resolver_hosts_resolvconf_and_candidates) {
  std::string hosts = "127.0.0.1 localhost\n# comment\n10.1.2.3\tapi.internal  api # alias\n::1 ip6-localhost\n";
  EXPECT_EQ(net::hosts_lookup(hosts, "API").size(), (size_t)1);
  EXPECT_EQ(net::hosts_lookup(hosts, "api.internal.")[0], std::string("10.1.2.3"));
  EXPECT_TRUE(net::hosts_lookup(hosts, "comment").empty());
  net::ResolvConf rc = net::ResolvConf::parse(
      "nameserver 10.96.0.10\nnameserver fe80::1%eth0\nsearch ns1.svc.cluster.local svc.cluster.local cluster.local\n"
      "options ndots:5 timeout:1 attempts:3\n");
  EXPECT_EQ(rc.nameservers.size(), (size_t)2);
  EXPECT_EQ(rc.ndots, 5);
  EXPECT_EQ(rc.timeout_s, 1);
  EXPECT_EQ(rc.attempts, 3);
  auto c = net::dns_candidates("kubernetes.default", rc);  // fewer dots than ndots: search first
  EXPECT_EQ(c.front(), std::string("kubernetes.default.ns1.svc.cluster.local"));
  EXPECT_EQ(c.back(), std::string("kubernetes.default"));
  EXPECT_EQ(net::dns_candidates("example.com.", rc).size(), (size_t)1);
  net::ResolvConf def = net::ResolvConf::parse("");
  EXPECT_EQ(def.nameservers.size(), (size_t)2);
  auto d = net::dns_candidates("a.b", def);  // ndots 1: absolute first
  EXPECT_EQ(d.front(), std::string("a.b"));
  auto lit = net::resolve("127.0.0.1", 80);
  EXPECT_EQ(lit.size(), (size_t)1);
  EXPECT_EQ(net::resolve("[::1]", 80).size(), (size_t)1);
  EXPECT_TRUE(!net::resolve("localhost", 80).empty());
}

TEST(resolver_dns_packets) {
  std::string q = net::dns_query_packet("api.example.com", 1, 0x1234);
  EXPECT_EQ(q.size(), (size_t)(12 + 17 + 4));
  // a response: the question, a CNAME, then two A records (compressed owner names)
  std::string r = q;
  r[2] = (char)0x81;
  r[3] = (char)0x80;
  r[7] = 3;  // ANCOUNT
  auto rr = [&](uint16_t type, const std::string& rdata) {
    std::string x = "\xc0\x0c";
    x.push_back((char)(type >> 8));
    x.push_back((char)type);
    x += std::string("\x00\x01\x00\x00\x00\x3c", 6);
    x.push_back((char)(rdata.size() >> 8));
    x.push_back((char)rdata.size());
    return x + rdata;
  };
  r += rr(5, std::string("\x03" "lb1\xc0\x10", 6));
  r += rr(1, std::string("\x0a\x00\x00\x07", 4));
  r += rr(1, std::string("\x0a\x00\x00\x08", 4));
  std::vector<std::string> addrs;
  bool tc = true;
  EXPECT_TRUE(net::dns_parse_response(r, 0x1234, &addrs, &tc));
  EXPECT_TRUE(!tc);
  EXPECT_EQ(addrs.size(), (size_t)2);
  EXPECT_EQ(addrs[0], std::string("10.0.0.7"));
  std::vector<std::string> none;
  EXPECT_TRUE(!net::dns_parse_response(r, 0x9999, &none, &tc));  // not our id
  std::string nx = q;
  nx[2] = (char)0x81;
  nx[3] = (char)0x83;  // NXDOMAIN
  EXPECT_TRUE(!net::dns_parse_response(nx, 0x1234, &none, &tc));
  EXPECT_TRUE(!net::dns_parse_response(r.substr(0, r.size() - 2), 0x1234, &none, &tc));  // truncated record
}

// port-forward bindAddress "::1" / "::" must not silently become 127.0.0.1.
// Only a request HTTP lets a client repeat is sent on several streams while the app restarts.
TEST(port_forward_hedges_only_repeatable_requests) {
  EXPECT_TRUE(services::hedgeable_request("GET / HTTP/1.1\r\nHost: x\r\n\r\n"));
  EXPECT_TRUE(services::hedgeable_request("HEAD /a HTTP/1.1\r\nHost: x\r\n\r\n"));
  EXPECT_TRUE(!services::hedgeable_request("POST / HTTP/1.1\r\nHost: x\r\nContent-Length: 1\r\n\r\nx"));
  EXPECT_TRUE(!services::hedgeable_request("PUT / HTTP/1.1\r\nHost: x\r\n\r\n"));
  // a GET with a body, a partial head, or a second request after the first: one stream at a time
  EXPECT_TRUE(!services::hedgeable_request("GET / HTTP/1.1\r\nContent-Length: 2\r\n\r\n"));
  EXPECT_TRUE(!services::hedgeable_request("GET / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n"));
  EXPECT_TRUE(!services::hedgeable_request("GET / HTTP/1.1\r\nHost: x\r\n"));
  EXPECT_TRUE(!services::hedgeable_request("GET / HTTP/1.1\r\n\r\nGET /b HTTP/1.1\r\n\r\n"));
  EXPECT_TRUE(!services::hedgeable_request("\x16\x03\x01 tls hello"));
  // a WebSocket handshake opens a session (a dev server's hot-reload socket)
  EXPECT_TRUE(!services::hedgeable_request("GET /ws HTTP/1.1\r\nHost: x\r\nConnection: Upgrade\r\n"
                                           "Upgrade: websocket\r\n\r\n"));
}

TEST(port_forward_listen_addresses) {
  auto d = services::listen_addresses("");
  EXPECT_EQ(d.size(), (size_t)2);
  EXPECT_EQ(d[0].second, std::string("127.0.0.1"));
  EXPECT_EQ(d[1].first, AF_INET6);
  EXPECT_EQ(services::listen_addresses("::1")[0].first, AF_INET6);
  EXPECT_EQ(services::listen_addresses("[::]")[0].second, std::string("::"));
  EXPECT_EQ(services::listen_addresses("0.0.0.0")[0].first, AF_INET);
  EXPECT_EQ(services::listen_addresses("localhost").size(), (size_t)2);
}

// A new connection to the same server resumes the previous TLS session (every exec / attach /
// port-forward stream is a new connection); the handshake count stays, resumed ones are
// counted apart.
TEST(tls_client_resumes_sessions) {
  Value cert = sprig::gen_self_signed_cert("127.0.0.1", {"127.0.0.1"}, {}, 1);
  SSL_CTX* sctx = SSL_CTX_new(TLS_server_method());
  const std::string cert_pem = cert.get("Cert").as_string(), key_pem = cert.get("Key").as_string();
  BIO* cb = BIO_new_mem_buf(cert_pem.data(), (int)cert_pem.size());
  X509* x = PEM_read_bio_X509(cb, nullptr, nullptr, nullptr);
  BIO* kb = BIO_new_mem_buf(key_pem.data(), (int)key_pem.size());
  EVP_PKEY* k = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
  EXPECT_TRUE(SSL_CTX_use_certificate(sctx, x) == 1 && SSL_CTX_use_PrivateKey(sctx, k) == 1);
  ScriptedServer srv([&](int fd, int) {
    SSL* ssl = SSL_new(sctx);
    SSL_set_fd(ssl, fd);
    if (SSL_accept(ssl) == 1) {
      std::string buf;
      char tmp[4096];
      while (buf.find("\r\n\r\n") == std::string::npos) {
        int n = SSL_read(ssl, tmp, sizeof(tmp));
        if (n <= 0) break;
        buf.append(tmp, (size_t)n);
      }
      std::string r = "HTTP/1.1 200 OK\r\nContent-Length: 2\r\nConnection: close\r\n\r\nok";
      SSL_write(ssl, r.data(), (int)r.size());
      SSL_shutdown(ssl);
    }
    SSL_free(ssl);
  });
  net::TlsOptions t;
  t.ca_pem = cert_pem;
  t.server_name = "127.0.0.1";
  net::HttpClient c("https://127.0.0.1:" + std::to_string(srv.port), t);
  c.set_keepalive(false);  // a new connection per request
  int64_t hs0 = net::stats().tls_handshakes.load(), res0 = net::stats().tls_resumed.load();
  for (int i = 0; i < 3; ++i) EXPECT_EQ(c.get("/x").body, std::string("ok"));
  EXPECT_EQ(net::stats().tls_handshakes.load() - hs0, 3);
  EXPECT_EQ(net::stats().tls_resumed.load() - res0, 2);  // all but the first
  X509_free(x);
  EVP_PKEY_free(k);
  BIO_free(cb);
  BIO_free(kb);
  srv.stop = true;
  SSL_CTX_free(sctx);
}

// client-go's retry rule. 429 and 5xx + Retry-After are sent again after the
// header's delay, up to 10 times; a POST is retried on 429 only.
TEST(api_retry_rule_matches_client_go) {
  EXPECT_EQ(kube::retry_wait_ms(429, "1", "POST"), 1000);
  EXPECT_EQ(kube::retry_wait_ms(429, "", "GET"), 1000);
  EXPECT_EQ(kube::retry_wait_ms(429, "0", "PATCH"), 0);
  EXPECT_EQ(kube::retry_wait_ms(429, "3600", "GET"), kube::kMaxRetryAfterS * 1000);
  EXPECT_EQ(kube::retry_wait_ms(429, "Wed, 21 Oct 2015 07:28:00 GMT", "GET"), 1000);
  EXPECT_EQ(kube::retry_wait_ms(503, "2", "GET"), 2000);
  EXPECT_EQ(kube::retry_wait_ms(503, "2", "DELETE"), 2000);
  EXPECT_EQ(kube::retry_wait_ms(503, "2", "POST"), -1);
  EXPECT_EQ(kube::retry_wait_ms(503, "", "GET"), -1);  // a plain 5xx is an error
  EXPECT_EQ(kube::retry_wait_ms(500, "", "PUT"), -1);
  EXPECT_EQ(kube::retry_wait_ms(404, "1", "GET"), -1);
  EXPECT_EQ(kube::retry_wait_ms(200, "1", "GET"), -1);
}

TEST(api_client_retries_throttled_requests) {
  ThrottlingServer ts(3, 429, "0");
  kube::Client c(ts.rc());
  Value v = c.get("/api/v1/namespaces/x/pods/p");
  EXPECT_EQ(v.get("kind").as_string(), std::string("Pod"));
  EXPECT_EQ(ts.gets.load(), 4);
  EXPECT_EQ(c.throttle_retries(), 3);
  // a 429'd POST was not acted on: sent again
  ThrottlingServer tp(2, 429, "0");
  kube::Client cp(tp.rc());
  cp.post("/api/v1/namespaces/x/pods", Value::map());
  EXPECT_EQ(tp.posts.load(), 3);
}

TEST(api_client_never_retries_a_post_on_5xx) {
  ThrottlingServer ts(1, 503, "0");
  kube::Client c(ts.rc());
  bool threw = false;
  try {
    c.post("/api/v1/namespaces/x/pods", Value::map());
  } catch (const kube::ApiError& e) {
    threw = e.code == 503;
  }
  EXPECT_TRUE(threw);
  EXPECT_EQ(ts.posts.load(), 1);
  EXPECT_EQ(c.throttle_retries(), 0);
  // the same 503 + Retry-After on an idempotent verb is retried
  ThrottlingServer tg(1, 503, "0");
  kube::Client cg(tg.rc());
  cg.del("/api/v1/namespaces/x/pods/p");
  EXPECT_EQ(tg.gets.load(), 2);
}

TEST(api_client_gives_up_after_ten_retries) {
  ThrottlingServer ts(1000, 429, "0");
  kube::Client c(ts.rc());
  bool threw = false;
  try {
    c.get("/api/v1/namespaces/x/pods");
  } catch (const kube::ApiError& e) {
    threw = e.code == 429;
  }
  EXPECT_TRUE(threw);
  EXPECT_EQ(ts.gets.load(), 1 + kube::kMaxApiRetries);
}

TEST(api_client_waits_retry_after) {
  ThrottlingServer ts(1, 429, "1");
  kube::Client c(ts.rc());
  auto t0 = std::chrono::steady_clock::now();
  c.get("/api/v1/namespaces/x/pods/p");
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  EXPECT_TRUE(ms >= 950 && ms < 3000);
}

// A tokenFile rotated under running requests (a projected service-account token): the request
// that gets the first 401 reads the file again and is sent again; the others, which also went
// out with the revoked token, are sent again with what it read instead of failing on "nothing
// new in the token file". Only a 401 with the current credentials is final.
TEST(api_client_token_file_rotation_under_concurrent_requests) {
  std::string d = fs::make_temp_dir("tokfile-");
  std::string tf = fs::join(d, "token");
  fs::write_file(tf, "old\n");
  std::atomic<int> unauthorized{0};
  ScriptedServer srv([&](int fd, int) {
    std::string body;
    while (true) {
      std::string head = read_request(fd, &body);
      if (head.empty()) return;
      if (head.find("Authorization: Bearer new") == std::string::npos) {
        unauthorized++;
        respond_status(fd, 401, "");
      } else {
        respond(fd, "{\"kind\":\"Pod\"}");
      }
    }
  });
  kube::RestConfig rc;
  rc.server = srv.url();
  rc.token = "old";
  rc.token_file = tf;
  {
    kube::Client c(rc);
    uint64_t used = c.ensure_fresh_credentials();  // two requests go out with "old"
    fs::write_file(tf, "new\n");                     // the kubelet rotates the token
    EXPECT_TRUE(c.refresh_after_unauthorized(used));  // the first 401: the file has a new token
    EXPECT_TRUE(c.refresh_after_unauthorized(used));  // the second: already replaced, send again
    EXPECT_TRUE(!c.refresh_after_unauthorized(c.ensure_fresh_credentials()));  // current and refused
    EXPECT_EQ(c.get("/api/v1/namespaces/x/pods/p").get("kind").as_string(), std::string("Pod"));
  }  // (the scripted server serves one kept-alive connection at a time)
  // a client that still holds the old token: its first request gets a 401, reads the file, retries
  kube::Client c2(rc);
  int before = unauthorized.load();
  EXPECT_EQ(c2.get("/api/v1/namespaces/x/pods/p").get("kind").as_string(), std::string("Pod"));
  EXPECT_EQ(unauthorized.load(), before + 1);
  fs::remove_all(d);
}

// list + watch against servers that do not play along (client-go's reflector rules): a watch
// that ends in an ERROR event (410 Gone: the resourceVersion is too old) starts over from a
// fresh list; a server that ignores watch=1 and answers with a list is polled instead.
TEST(api_client_list_watch_relists_after_gone_and_polls_without_watch) {
  const std::string pod =
      "{\"metadata\":{\"name\":\"p\",\"namespace\":\"x\",\"resourceVersion\":\"7\","
      "\"creationTimestamp\":\"2026-01-01T00:00:00Z\"},\"status\":{\"phase\":\"Running\"}}";
  {
    std::vector<std::string> heads;
    std::mutex mu;
    int lists = 0;
    ScriptedServer srv([&](int fd, int) {
      std::string body;
      while (true) {
        std::string head = read_request(fd, &body);
        if (head.empty()) return;
        {
          std::lock_guard<std::mutex> g(mu);
          heads.push_back(head.substr(0, head.find("\r\n")));
        }
        if (head.find("watch=1") != std::string::npos)
          respond(fd, "{\"type\":\"ERROR\",\"object\":{\"kind\":\"Status\",\"code\":410,\"reason\":\"Expired\"}}\n");
        else if (lists++ == 0)
          respond(fd, "{\"kind\":\"PodList\",\"metadata\":{\"resourceVersion\":\"5\"},\"items\":[]}");
        else
          respond(fd, "{\"kind\":\"PodList\",\"metadata\":{\"resourceVersion\":\"7\"},\"items\":[" + pod + "]}");
      }
    });
    kube::RestConfig rc;
    rc.server = srv.url();
    kube::Client c(rc);
    bool ok = c.list_watch("/api/v1/namespaces/x/pods", "", 10000,
                           [](const std::vector<Value>& ps) { return !ps.empty(); });
    EXPECT_TRUE(ok);
    std::lock_guard<std::mutex> g(mu);
    EXPECT_EQ(heads.size(), (size_t)3);
    EXPECT_TRUE(heads.size() == 3 && heads[1].find("watch=1") != std::string::npos &&
                heads[1].find("resourceVersion=5") != std::string::npos);
    EXPECT_TRUE(heads.size() == 3 && heads[2].find("watch=1") == std::string::npos);
  }
  {
    std::atomic<int> lists{0}, watches{0};
    ScriptedServer srv([&](int fd, int) {
      std::string body;
      while (true) {
        std::string head = read_request(fd, &body);
        if (head.empty()) return;
        bool w = head.find("watch=1") != std::string::npos;
        (w ? watches : lists)++;
        // an old or odd server: every GET gets the plain list
        bool ready = lists.load() >= 3;
        respond(fd, std::string("{\"kind\":\"PodList\",\"metadata\":{\"resourceVersion\":\"5\"},\"items\":[") +
                        (ready ? pod : "") + "]}");
      }
    });
    kube::RestConfig rc;
    rc.server = srv.url();
    kube::Client c(rc);
    bool ok = c.list_watch("/api/v1/namespaces/x/pods", "", 10000,
                           [](const std::vector<Value>& ps) { return !ps.empty(); });
    EXPECT_TRUE(ok);
    EXPECT_EQ(watches.load(), 1);  // tried once, then polled
    EXPECT_TRUE(lists.load() >= 3);
  }
}
