// Host name resolution without glibc's NSS (the release binary is fully static, like the
// reference's CGO_ENABLED=0 Go build — scripts/build-all.bash:44-50 — whose net package carries
// its own resolver too). Order: IP literal, /etc/hosts, then DNS over UDP to the nameservers of
// /etc/resolv.conf with its search list and ndots (Kubernetes in-cluster names need both).
#pragma once

#include <sys/socket.h>

#include <string>
#include <vector>

namespace ds {
namespace net {

struct Address {
  int family = 0;
  struct sockaddr_storage addr {};
  socklen_t len = 0;
  std::string text;  // printable address
};

struct ResolvConf {
  std::vector<std::string> nameservers;  // IPv4/IPv6 literals
  std::vector<std::string> search;
  int ndots = 1;
  int timeout_s = 2;
  int attempts = 2;
  static ResolvConf parse(const std::string& text);
  static ResolvConf load(const std::string& path = "/etc/resolv.conf");
};

// Addresses for host:port (IPv4 first, then IPv6). Empty with *err set when nothing resolves.
std::vector<Address> resolve(const std::string& host, int port, std::string* err = nullptr);

// getaddrinfo (NSS, the OS's own DNS configuration); what resolve() uses when
// plat::system_resolver() says so (the portable build).
std::vector<Address> system_resolve(const std::string& host, int port, std::string* err = nullptr);

// Pieces, exposed for tests.
std::vector<std::string> hosts_lookup(const std::string& hosts_text, const std::string& name);
std::string dns_query_packet(const std::string& name, int qtype, uint16_t id);
// Parses a DNS response: A/AAAA record addresses (printable) of the answer section, any owner
// (a CNAME chain comes with its final records). false when malformed, an error rcode or the id
// differs.
bool dns_parse_response(const std::string& pkt, uint16_t id, std::vector<std::string>* addrs, bool* truncated);
// Candidate FQDNs for a name under the resolv.conf search rules.
std::vector<std::string> dns_candidates(const std::string& name, const ResolvConf& rc);

}  // namespace net
}  // namespace ds
