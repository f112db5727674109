// Port-forward through the in-container helper (`devspace-helper forward`, src/helper/forward.cc
// <-> src/services/portforward.cc HelperLink): the connections of one forward multiplexed over
// one exec stream, with the hold of a connection the app refuses done *in the pod*.
//
// Why: a request sent while the app restarts (hot reload) is refused by the pod; through the
// kubelet's port-forward each retry costs a round trip to the cluster, so on a remote cluster
// the request reaches the new server up to a round trip after it listens (the WAN loop was
// 82 ms or 113 ms depending on that phase). The helper retries the pod-local connect every few
// milliseconds instead and connects once: the request is delivered exactly once, within ms of
// the app listening, whatever the link.
//
// Frames use the helper framing (src/sync/frame.h): op:u8 len:u64be payload, payload starting
// with the connection id (u32be).
//   client -> helper   'O' id port:u16be hold_ms:u32be   open: connect to localhost:port, retrying
//                                                        a refused connect for up to hold_ms
//                      'D' id bytes                      data (kept until connected)
//                      'F' id                            client half-close (after its data)
//                      'K' id                            abort
//                      'A' id n:u32be                    n more bytes of the app's data written
//                                                        to the local connection
//   helper -> client   'C' id                            connected
//                      'D' id bytes                      data from the app
//                      'F' id                            the app closed its side
//                      'E' id message                    failed ("connection refused" after the
//                                                        hold) or reset; the id is gone
//                      'A' id n:u32be                    n more bytes of the client's data written
//                                                        to the app
//
// Flow control: each side keeps at most kWindow bytes of one connection's data unacknowledged
// ('A'), so a slow reader at either end holds back that connection only, and neither side
// buffers more than kWindow per connection (a multi-GB download through the forward to a slow
// local reader, or an upload to an app that reads slowly, cannot grow either process).
#pragma once

#include <cstdint>
#include <string>

#include "sync/frame.h"

namespace ds {
namespace sync {
namespace fwd {

inline std::string u32be(uint32_t v) {
  std::string s(4, '\0');
  for (int i = 0; i < 4; ++i) s[i] = (char)(v >> (24 - 8 * i));
  return s;
}

inline uint32_t get_u32be(const std::string& s, size_t at) {
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) v = (v << 8) | (unsigned char)s[at + i];
  return v;
}

inline std::string frame(char op, uint32_t id, const std::string& body = "") {
  return frame::request(op, u32be(id) + body);
}

inline std::string open_frame(uint32_t id, int port, uint32_t hold_ms) {
  std::string b(2, '\0');
  b[0] = (char)((port >> 8) & 0xff);
  b[1] = (char)(port & 0xff);
  return frame('O', id, b + u32be(hold_ms));
}

constexpr uint64_t kMaxFramePayload = (1u << 20) + 16;
constexpr uint64_t kWindow = 4u << 20;      // unacknowledged bytes per connection and direction
constexpr uint64_t kAckEvery = 256u << 10;  // a reader acknowledges at least this often

inline std::string ack_frame(uint32_t id, uint64_t n) { return frame('A', id, u32be((uint32_t)n)); }

}  // namespace fwd
}  // namespace sync
}  // namespace ds
