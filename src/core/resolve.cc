#include "core/resolve.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <time.h>
#include <unistd.h>

#include <cstring>
#include <random>

#include "core/fs.h"
#include "core/strutil.h"
#include "platform/platform.h"

namespace ds {
namespace net {

static bool literal(const std::string& host, int port, Address* out) {
  Address a;
  auto* v4 = (struct sockaddr_in*)&a.addr;
  auto* v6 = (struct sockaddr_in6*)&a.addr;
  if (inet_pton(AF_INET, host.c_str(), &v4->sin_addr) == 1) {
    v4->sin_family = AF_INET;
    v4->sin_port = htons((uint16_t)port);
    a.family = AF_INET;
    a.len = sizeof(*v4);
  } else if (inet_pton(AF_INET6, host.c_str(), &v6->sin6_addr) == 1) {
    v6->sin6_family = AF_INET6;
    v6->sin6_port = htons((uint16_t)port);
    a.family = AF_INET6;
    a.len = sizeof(*v6);
  } else {
    return false;
  }
  a.text = host;
  *out = a;
  return true;
}

ResolvConf ResolvConf::parse(const std::string& text) {
  ResolvConf rc;
  for (auto& raw : split(text, "\n")) {
    std::string line = trim(raw.substr(0, raw.find_first_of("#;")));
    if (line.empty()) continue;
    std::vector<std::string> f;
    for (auto& t : split(replace_all(line, "\t", " "), " "))
      if (!t.empty()) f.push_back(t);
    if (f.empty()) continue;
    if (f[0] == "nameserver" && f.size() > 1) {
      Address a;
      std::string ns = f[1].substr(0, f[1].find('%'));  // drop an IPv6 zone
      if (literal(ns, 53, &a)) rc.nameservers.push_back(ns);
    } else if ((f[0] == "search" || f[0] == "domain") && f.size() > 1) {
      rc.search.assign(f.begin() + 1, f.end());  // the last search/domain line wins
    } else if (f[0] == "options") {
      for (size_t i = 1; i < f.size(); ++i) {
        int64_t v;
        if (starts_with(f[i], "ndots:") && parse_int64(f[i].substr(6), &v)) rc.ndots = (int)std::min<int64_t>(v, 15);
        if (starts_with(f[i], "timeout:") && parse_int64(f[i].substr(8), &v)) rc.timeout_s = (int)std::max<int64_t>(1, v);
        if (starts_with(f[i], "attempts:") && parse_int64(f[i].substr(9), &v))
          rc.attempts = (int)std::max<int64_t>(1, std::min<int64_t>(v, 5));
      }
    }
  }
  if (rc.nameservers.empty()) rc.nameservers = {"127.0.0.1", "::1"};  // resolv.conf(5) default
  return rc;
}

ResolvConf ResolvConf::load(const std::string& path) {
  std::string text;
  fs::read_file(path, &text);
  return parse(text);
}

std::vector<std::string> hosts_lookup(const std::string& text, const std::string& name) {
  std::vector<std::string> out;
  std::string want = to_lower(name);
  if (!want.empty() && want.back() == '.') want.pop_back();
  for (auto& raw : split(text, "\n")) {
    std::string line = trim(raw.substr(0, raw.find('#')));
    std::vector<std::string> f;
    for (auto& t : split(replace_all(line, "\t", " "), " "))
      if (!t.empty()) f.push_back(t);
    if (f.size() < 2) continue;
    for (size_t i = 1; i < f.size(); ++i)
      if (to_lower(f[i]) == want) {
        out.push_back(f[0]);
        break;
      }
  }
  return out;
}

std::string dns_query_packet(const std::string& name, int qtype, uint16_t id) {
  std::string p;
  p.push_back((char)(id >> 8));
  p.push_back((char)id);
  p += std::string("\x01\x00", 2);          // RD
  p += std::string("\x00\x01\x00\x00\x00\x00\x00\x00", 8);  // 1 question
  for (auto& label : split(name, ".")) {
    if (label.empty()) continue;
    p.push_back((char)std::min<size_t>(label.size(), 63));
    p += label.substr(0, 63);
  }
  p.push_back('\0');
  p.push_back((char)(qtype >> 8));
  p.push_back((char)qtype);
  p += std::string("\x00\x01", 2);  // IN
  return p;
}

static bool skip_name(const std::string& p, size_t* off) {
  for (int guard = 0; guard < 128; ++guard) {
    if (*off >= p.size()) return false;
    unsigned char len = (unsigned char)p[*off];
    if (len == 0) {
      *off += 1;
      return true;
    }
    if ((len & 0xc0) == 0xc0) {  // compression pointer ends the name
      *off += 2;
      return *off <= p.size();
    }
    *off += 1 + len;
  }
  return false;
}

bool dns_parse_response(const std::string& p, uint16_t id, std::vector<std::string>* addrs, bool* truncated) {
  if (p.size() < 12) return false;
  auto u16 = [&](size_t o) { return (uint16_t)(((unsigned char)p[o] << 8) | (unsigned char)p[o + 1]); };
  if (u16(0) != id || !(p[2] & 0x80)) return false;  // not our answer
  if (truncated) *truncated = (p[2] & 0x02) != 0;
  int rcode = p[3] & 0x0f;
  if (rcode != 0) return false;
  int qd = u16(4), an = u16(6);
  size_t off = 12;
  for (int i = 0; i < qd; ++i) {
    if (!skip_name(p, &off)) return false;
    off += 4;
  }
  for (int i = 0; i < an; ++i) {
    if (!skip_name(p, &off) || off + 10 > p.size()) return false;
    uint16_t type = u16(off), klass = u16(off + 2), rdlen = u16(off + 8);
    off += 10;
    if (off + rdlen > p.size()) return false;
    char buf[INET6_ADDRSTRLEN] = {0};
    if (klass == 1 && type == 1 && rdlen == 4 && inet_ntop(AF_INET, p.data() + off, buf, sizeof(buf)))
      addrs->push_back(buf);
    if (klass == 1 && type == 28 && rdlen == 16 && inet_ntop(AF_INET6, p.data() + off, buf, sizeof(buf)))
      addrs->push_back(buf);
    off += rdlen;
  }
  return true;
}

std::vector<std::string> dns_candidates(const std::string& name, const ResolvConf& rc) {
  std::vector<std::string> out;
  if (!name.empty() && name.back() == '.') return {name.substr(0, name.size() - 1)};
  int dots = 0;
  for (char c : name) dots += c == '.';
  std::vector<std::string> searched;
  for (auto& s : rc.search) searched.push_back(name + "." + s);
  if (dots >= rc.ndots) {
    out.push_back(name);
    out.insert(out.end(), searched.begin(), searched.end());
  } else {
    out = searched;
    out.push_back(name);
  }
  return out;
}

static std::vector<std::string> dns_lookup(const std::string& fqdn, const ResolvConf& rc) {
  static std::mt19937 rng{(unsigned)time(nullptr) ^ (unsigned)getpid()};
  std::vector<std::string> out;
  for (int qtype : {1, 28}) {
    bool answered = false;
    for (int attempt = 0; attempt < rc.attempts && !answered; ++attempt) {
      for (auto& ns : rc.nameservers) {
        Address a;
        if (!literal(ns, 53, &a)) continue;
        int fd = plat::socket_cloexec(a.family, SOCK_DGRAM);
        if (fd < 0) continue;
        uint16_t id = (uint16_t)rng();
        std::string q = dns_query_packet(fqdn, qtype, id);
        if (::connect(fd, (struct sockaddr*)&a.addr, a.len) != 0 || ::send(fd, q.data(), q.size(), 0) < 0) {
          ::close(fd);
          continue;
        }
        struct pollfd pf{fd, POLLIN, 0};
        char buf[4096];
        ssize_t n = -1;
        if (::poll(&pf, 1, rc.timeout_s * 1000) > 0) n = ::recv(fd, buf, sizeof(buf), 0);
        ::close(fd);
        if (n <= 0) continue;
        std::vector<std::string> got;
        bool tc = false;
        if (dns_parse_response(std::string(buf, (size_t)n), id, &got, &tc)) {
          answered = true;
          out.insert(out.end(), got.begin(), got.end());
          break;
        }
      }
    }
  }
  return out;
}

std::vector<Address> system_resolve(const std::string& host, int port, std::string* err) {
  struct addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
  std::vector<Address> out;
  if (rc != 0) {
    if (err) *err = gai_strerror(rc);
    return out;
  }
  for (int fam : {AF_INET, AF_INET6}) {
    for (auto* ai = res; ai; ai = ai->ai_next) {
      if (ai->ai_family != fam || ai->ai_addrlen > sizeof(sockaddr_storage)) continue;
      Address a;
      a.family = fam;
      std::memcpy(&a.addr, ai->ai_addr, ai->ai_addrlen);
      a.len = ai->ai_addrlen;
      char buf[INET6_ADDRSTRLEN] = {0};
      const void* src = fam == AF_INET ? (const void*)&((struct sockaddr_in*)ai->ai_addr)->sin_addr
                                       : (const void*)&((struct sockaddr_in6*)ai->ai_addr)->sin6_addr;
      inet_ntop(fam, src, buf, sizeof(buf));
      a.text = buf;
      bool dup = false;
      for (auto& o : out) dup = dup || o.text == a.text;
      if (!dup) out.push_back(a);
    }
  }
  freeaddrinfo(res);
  if (out.empty() && err) *err = "no such host";
  return out;
}

std::vector<Address> resolve(const std::string& host_in, int port, std::string* err) {
  std::vector<Address> out;
  std::string host = host_in;
  if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  Address a;
  if (literal(host, port, &a)) return {a};
  if (plat::system_resolver()) return system_resolve(host, port, err);
  std::vector<std::string> ips;
  std::string hosts;
  if (fs::read_file("/etc/hosts", &hosts)) ips = hosts_lookup(hosts, host);
  if (ips.empty() && to_lower(host) == "localhost") ips = {"127.0.0.1", "::1"};
  if (ips.empty()) {
    ResolvConf rc = ResolvConf::load();
    for (auto& fqdn : dns_candidates(host, rc)) {
      ips = dns_lookup(fqdn, rc);
      if (!ips.empty()) break;
    }
  }
  // IPv4 first: clusters and daemons listen there more often than not
  for (int fam : {AF_INET, AF_INET6})
    for (auto& ip : ips)
      if (literal(ip, port, &a) && a.family == fam) out.push_back(a);
  if (out.empty() && err) *err = "no such host";
  return out;
}

}  // namespace net
}  // namespace ds
