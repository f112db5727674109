// SPDY/3.1 sessions tunneled over a WebSocket: Kubernetes' multiplexed port-forward.
//
// The reference forwards with client-go's SPDY dialer: one SPDY connection per pod and a pair of
// streams (error + data) per local connection (/root/reference/pkg/devspace/kubectl/client.go:356-380,
// portforward.NewOnAddresses). SPDY upgrades are deprecated upstream; since Kubernetes 1.30 the API
// server also accepts a WebSocket upgrade with subprotocol "SPDY/3.1+portforward.k8s.io" whose
// binary messages carry the SPDY byte stream (KEP-4006). One such tunnel serves every local
// connection of a forward: a new connection costs a SYN_STREAM pair written into the open tunnel
// (its bytes follow at once, no round trip), instead of a TCP + TLS + WebSocket upgrade per
// connection — the difference a developer on a laptop pays per request to a remote MI355X node.
//
// Implemented from the SPDY/3.1 framing (control frames: SYN_STREAM, SYN_REPLY, RST_STREAM,
// SETTINGS, PING, GOAWAY, HEADERS, WINDOW_UPDATE; data frames with FIN) and its zlib header-block
// compression with the protocol's fixed dictionary. Like the Go spdystream the API servers use,
// send windows are not enforced (the peer's WINDOW_UPDATEs are read and ignored) while received
// data is acknowledged with WINDOW_UPDATE frames.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "core/net.h"

namespace ds {
namespace kube {

using SpdyHeaders = std::vector<std::pair<std::string, std::string>>;

// The SPDY/3 header-compression dictionary (1423 bytes, zlib dictionary id 0xe3c6a7c2).
const std::string& spdy_dictionary();

// Header blocks: a zlib stream per direction and session, primed with the dictionary; each
// block ends with a sync flush.
class SpdyHeaderCodec {
 public:
  SpdyHeaderCodec();
  ~SpdyHeaderCodec();
  SpdyHeaderCodec(const SpdyHeaderCodec&) = delete;
  SpdyHeaderCodec& operator=(const SpdyHeaderCodec&) = delete;
  std::string compress(const SpdyHeaders& h);
  // false on a corrupt block
  bool decompress(const std::string& block, SpdyHeaders* out);

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// Everything a consumer of streams waits on: (channel, bytes) events of the streams registered
// to it, plus their ends.
// Kubelets do not enforce SPDY windows (spdystream), so a fast download to a slow local client
// arrives whatever the client announces. The session's reader must not wait for one slow
// consumer: that would stall every other connection of the pod's tunnel, and its PINGs, as a Go
// spdystream frame loop does. So: up to `cap` unread bytes in memory, then events spill, in
// order, to a nameless temporary file (plat::open_unlinked_tmp), up to `spill_cap` bytes. Only
// past that (or without a usable temp directory) does push() wait for the consumer.
struct SpdyMailbox {
  struct Event {
    int channel;      // what the stream was registered as (port-forward: 0 data, 1 error)
    std::string data;
    bool end = false;  // FIN or RST from the peer, or the session ended
    std::string reset;  // RST_STREAM status, "" otherwise
  };
  SpdyMailbox() = default;
  SpdyMailbox(const SpdyMailbox&) = delete;
  SpdyMailbox& operator=(const SpdyMailbox&) = delete;
  ~SpdyMailbox();
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Event> q;
  size_t bytes = 0;         // data bytes queued in memory
  size_t cap = 4u << 20;
  uint64_t spill_cap = 1ull << 30;  // DEVSPACE_PORTFORWARD_SPILL_MB
  std::string spill_dir;            // "" = $TMPDIR or /tmp
  bool closed = false;      // the consumer is gone: data is dropped, nothing blocks
  void push(Event e);
  // false on timeout, or once closed
  bool pop(Event* e, int timeout_ms = -1);
  // the consumer is done: queued data is dropped, pushes stop blocking, pop() returns false
  void close();
  uint64_t spilled() const { return spill_w_ - spill_r_; }  // bytes waiting on disk (under mu)

 private:
  bool spill(const Event& e);  // under mu; false if the spill file cannot be used
  bool unspill(Event* e);      // under mu; the oldest spilled event
  int spill_fd_ = -1;
  bool spill_broken_ = false;
  uint64_t spill_w_ = 0, spill_r_ = 0;
  size_t spill_events_ = 0;
};

class SpdySession {
 public:
  struct Stream {
    uint32_t id = 0;
    int channel = 0;
    std::shared_ptr<SpdyMailbox> box;
    bool local_fin = false;
    bool remote_end = false;
    uint64_t unacked = 0;  // received bytes not yet announced in a WINDOW_UPDATE
  };

  // Takes the upgraded WebSocket (its subprotocol already checked) and starts the reader.
  explicit SpdySession(std::unique_ptr<net::WebSocket> ws);
  ~SpdySession();
  SpdySession(const SpdySession&) = delete;
  SpdySession& operator=(const SpdySession&) = delete;

  // Opens a client stream (odd id). `fin`: no data will be sent on it. Throws NetError when the
  // session is gone or the peer said GOAWAY.
  std::shared_ptr<Stream> open(const SpdyHeaders& headers, std::shared_ptr<SpdyMailbox> box, int channel,
                               bool fin = false);
  // Data on a stream; `fin` half-closes it. false when the session is gone.
  bool send(const std::shared_ptr<Stream>& s, const std::string& data, bool fin = false);
  // The consumer took `n` bytes of this stream: acknowledged once 32 KiB accumulate.
  void consumed(const std::shared_ptr<Stream>& s, size_t n);
  void reset(const std::shared_ptr<Stream>& s, uint32_t status = 5 /* CANCEL */);
  // false once the tunnel closed or the peer sent GOAWAY (no new streams).
  bool usable() const;
  void close();
  uint64_t streams_opened() const { return next_id_ / 2; }
  // Sends a PING; its answer measures the round trip to the far end of the tunnel (the kubelet),
  // without the pod. rtt_us(): the smallest round trip measured, -1 before an answer came.
  void ping();
  int64_t rtt_us() const { return rtt_us_.load(); }
  int rtt_samples() const { return rtt_samples_.load(); }  // PINGs answered
  // PINGs sent in the last 5 s and not answered yet
  size_t pings_in_flight() const;

 private:
  void reader();
  void end_all(const std::string& why);
  bool write_frame(const std::string& frame);
  void dispatch_control(uint16_t type, uint8_t flags, const std::string& body);
  void dispatch_data(uint32_t id, uint8_t flags, std::string data);

  std::unique_ptr<net::WebSocket> ws_;
  std::mutex wmu_;  // frame order on the wire = compression order of header blocks
  SpdyHeaderCodec out_codec_;
  SpdyHeaderCodec in_codec_;  // the reader thread's
  mutable std::mutex mu_;
  std::map<uint32_t, std::shared_ptr<Stream>> streams_;
  uint32_t next_id_ = 1;
  bool dead_ = false;
  bool goaway_ = false;
  uint64_t session_unacked_ = 0;
  uint32_t next_ping_ = 1;  // client PING ids are odd
  std::map<uint32_t, std::chrono::steady_clock::time_point> pings_;  // in flight (under mu_)
  std::atomic<int64_t> rtt_us_{-1};
  std::atomic<int> rtt_samples_{0};
  std::thread reader_;
};

// Frame builders and a parser, exposed for tests (and the session).
namespace spdy {
constexpr uint16_t kVersion = 3;
enum ControlType : uint16_t {
  SynStream = 1, SynReply = 2, RstStream = 3, Settings = 4, Ping = 6, GoAway = 7, Headers = 8, WindowUpdate = 9
};
constexpr uint8_t kFlagFin = 0x01;
std::string control_frame(uint16_t type, uint8_t flags, const std::string& body);
std::string data_frame(uint32_t stream_id, uint8_t flags, const std::string& data);
std::string u32(uint32_t v);
uint32_t get_u32(const std::string& s, size_t off);
// Parses one frame at the front of `buf` (consumed on success). false: incomplete.
struct Frame {
  bool control = false;
  uint16_t type = 0;      // control
  uint32_t stream_id = 0;  // data
  uint8_t flags = 0;
  std::string body;
};
bool parse(std::string* buf, Frame* f);
}  // namespace spdy

}  // namespace kube
}  // namespace ds
