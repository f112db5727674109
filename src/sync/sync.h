// Bidirectional local <-> container file sync (the reference's hot path, sync/*.go).
//
// Same decision rules as the reference (Appendix A of SURVEY.md: sync/evaluater.go,
// sync/tar.go untar rules, sync/file_index.go bookkeeping) with three wire protocols:
//   Mode::Compat — byte-for-byte the reference's POSIX scripts and timing constants
//                  (600 ms upload window, 1300 ms downstream poll + stability rule,
//                  `sleep 0.1` receive polling). Used as the reference-equivalent baseline.
//   Mode::Fast   — POSIX-only but streamed: the platform's tree watcher (platform/watch.h:
//                  inotify on Linux, the stat-scan watcher in the portable build) + ~15 ms
//                  coalescing, `head -c N | tar x`
//                  (no temp files / polling), newline acks; downstream `find -cnewer` change
//                  probes every 250 ms after activity, backing off to 1.3 s when idle.
//   Mode::Helper — uploads a static helper (src/helper) into the container that speaks a
//                  framed binary protocol (64-bit lengths, chunk-streamed archives) and pushes
//                  the pod's inotify events for event-driven downstream; falls back to Fast when it
//                  cannot run.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/match.h"
#include "core/watch.h"
#include "sync/transport.h"

namespace ds {
namespace sync {

enum class Mode { Compat, Fast, Helper };
Mode parse_mode(const std::string& s);

// Shell snippet that picks where the in-container helper lives: the first of `dirs` that already
// holds an executable `<dir>/<file>` ("HAVE <dir>"), else the first that is writable and lets a
// file in it execute ("NEED <dir>"; hardened pods mount /tmp noexec), else "NOHELPER" (also on a
// non-x86_64 container: the helper is a static x86_64 binary). `when_present`: shell run right
// after "HAVE <dir>" with $dsd set to that directory (starting the helper in the same round trip).
std::string helper_probe_script(const std::string& file, const std::vector<std::string>& dirs,
                                const std::string& when_present = "");
// Where the helper is looked for in a container, in order.
const std::vector<std::string>& helper_dirs();  // compat|fast|helper (default fast); env DEVSPACE_SYNC_MODE
const char* mode_name(Mode m);

struct FileInfo {
  std::string name;  // relative to the sync root, with leading "/" ("" = root)
  int64_t size = 0;
  int64_t mtime = 0;  // seconds (rounded for local files); 0 marks a remove change
  bool is_dir = false;
  bool is_symlink = false;
  int64_t remote_mode = 0;
  int remote_uid = 0, remote_gid = 0;
  bool has_remote_attrs = false;
  // Local nanosecond mtime at the last upload/download (non-compat modes only): detects two
  // same-size edits within one second, which the reference's rounded mtimes miss.
  int64_t local_mtime_ns = 0;
  // The container's side of the same (helper listings only; 0 = unknown): in a listing, the
  // file's nanosecond mtime; in the index, the stamp of the version last downloaded or uploaded.
  // A pod process rewriting a file at the same size within one second (a metrics file, a log
  // line) moves it, where seconds and size do not.
  int64_t remote_mtime_ns = 0;
  // The listing saw the file within a second of being written (a coarse filesystem clock can
  // give the next write the same stamp): once it is still, its content is checked (CRC-32)
  // against the local copy instead of trusting the stamp.
  bool remote_unsettled = false;
};

// Parses one `stat -c "%n///%s,%Y,%f,%a,%u,%g"` line (sync/file_information.go:62), or the
// helper's form with a seventh field, the nanoseconds of the mtime.
// Returns nullopt for the dest path itself; throws on malformed lines.
std::optional<FileInfo> parse_file_line(const std::string& line, const std::string& dest_path);

// Shared index of known files (sync/file_index.go). Ordered so subtree removal is
// O(log n + k) instead of the reference's O(n) scan.
class FileIndex {
 public:
  std::mutex mu;
  std::map<std::string, FileInfo> files;
  FileInfo* find(const std::string& name) {
    auto it = files.find(name);
    return it == files.end() ? nullptr : &it->second;
  }
  // Adds every ancestor directory of dirpath (lock held by caller).
  void create_dir(const std::string& dirpath);
  // Removes dirpath and its subtree (lock held by caller).
  void remove_dir(const std::string& dirpath);
};

struct Options {
  std::string watch_path;      // local directory
  std::string dest_path;       // container path (logical, e.g. /app)
  std::string pod_name;        // for log context
  std::vector<std::string> exclude_paths, download_exclude_paths, upload_exclude_paths;
  int64_t upstream_limit = 0;    // bytes/s
  int64_t downstream_limit = 0;  // bytes/s
  bool verbose = false;
  bool silent = false;  // no sync.log entries (CopyToContainer)
  Mode mode = Mode::Fast;
  std::string helper_path;  // static helper binary (Mode::Helper)
  // Timing knobs (defaults depend on mode; <0 = mode default)
  int upstream_window_ms = -1;
  int downstream_poll_ms = -1;
  // Fast mode: probe for changes (`find -newer`) between full listings (false = always list)
  bool downstream_probe = true;
  // Reconnect: when set, a dead stream triggers a transport refresh (e.g. pick the newest
  // running pod again) instead of a fatal stop (the reference log.Fatalf's, sync_config.go:481).
  std::function<std::shared_ptr<Transport>()> reconnect;
  int max_reconnects = 10;
  // A stream that delivers no byte for this long is dead (replaces fixed per-transfer
  // deadlines: a multi-GB transfer may take minutes, a stalled one is cut after this).
  int idle_timeout_ms = 120000;
  // Files at least this big get a one-time warning suggesting an exclude (<0: the default,
  // 1 GiB, or $DEVSPACE_SYNC_WARN_FILE_MB).
  int64_t large_file_warn_bytes = -1;
  std::function<void(const std::string&)> on_error;
  std::function<void()> on_initial_sync_done;
  std::string sync_log_name = "sync";
};

struct Stats {
  uint64_t upstream_batches = 0, upstream_changes = 0;
  uint64_t downstream_batches = 0, downstream_changes = 0;
  uint64_t reconnects = 0;
  double last_upload_ms = 0;  // first event -> remote ack
  uint64_t bytes_up = 0, bytes_down = 0;
  // downstream scanning (non-helper modes): full `find | stat` listings, cheap change probes
  // (fast mode: `find -newer stamp`, one line at most) and the listing bytes read
  uint64_t full_scans = 0, probes = 0, probe_hits = 0, scan_bytes = 0;
  int probe_interval_ms = 0;  // fast mode: the adaptive interval last waited (250 .. 1300)
};

class Session {
 public:
  Session(Options opts, std::shared_ptr<Transport> transport);
  ~Session();
  Session(const Session&) = delete;

  void start();  // setup + shells + watcher + threads (initial sync runs asynchronously)
  void stop(const std::string& fatal_error = "");
  bool wait_initial_sync(int timeout_ms);
  bool running() const { return running_; }
  std::string error();
  Stats stats();
  const Options& options() const { return o_; }
  std::string pod_name();  // current pod (changes when a reconnect picks a new one)
  Mode effective_mode() const { return mode_; }

  // Decision rules (sync/evaluater.go) — index lock held by the caller.
  // Public so the property tests (tests/test_sync_rules_fuzz.py) can drive them directly.
  bool should_remove_remote(const std::string& rel);
  bool should_upload(const std::string& rel, const fs::StatInfo& st, bool initial);
  bool should_download(const FileInfo& f);
  bool should_remove_local(const std::string& abs, const FileInfo& f);

  // --- pieces exposed for tests (the reference tests drive setup/initialSync directly)
  void setup();
  void open_shells();
  void start_watcher();
  void initial_sync();
  void start_loops(bool upstream, bool downstream);
  FileIndex& index() { return index_; }
  // Extracts a downstream tar.gz (as received from the container) into the local folder.
  void apply_downstream_archive(const std::string& archive) { untar_stream(string_source(&archive), nullptr); }

  // One-shot upload of a local folder/file (sync/util.go:21 CopyToContainer).
  static void copy_to_container(std::shared_ptr<Transport> t, const std::string& local_path,
                                const std::string& container_path, std::vector<std::string> excludes,
                                Mode mode = Mode::Fast);

 private:
  struct UpEvent {
    std::string abs_path;
    bool has_info = false;
    FileInfo info;
    long t_us = 0;
    bool settled = false;
  };

  // logging
  void logf(const std::string& msg);
  void log_error(const std::string& msg);


  // upstream
  void push_event(UpEvent e);
  void upstream_loop();
  std::optional<FileInfo> evaluate_change(const std::string& rel, const std::string& abs);
  void apply_upstream(std::vector<FileInfo>& changes, long first_event_us, bool bulk = false);
  void apply_removes(const std::vector<FileInfo>& removes);
  void apply_creates(const std::vector<FileInfo>& creates, bool bulk = false);
  // Streams a tar of `files` (recursively) to the container. Runs without the index lock (it
  // takes it per lookup): the downstream loop keeps working during a multi-GB upload, and skips
  // the paths in flight. `bulk`: the helper's bulk lane (yields to interactive uploads frame by
  // frame). Returns the wire bytes sent; throws on a broken stream.
  uint64_t stream_upload(const std::vector<FileInfo>& files, std::map<std::string, FileInfo>* written, bool bulk);
  void recursive_tar(const std::string& rel, std::map<std::string, FileInfo>* written, TarWriter* tw, int depth);
  bool wait_ack(LineReader& r, const std::string& keyword, bool partial, std::string* before = nullptr,
                int timeout_ms = 120000);
  void stop_loops();
  // Bulk write to a shell's stdin with an idle timeout (SyncError when stuck or closed).
  void send(int fd, const char* d, size_t n);
  void send(int fd, const std::string& s) { send(fd, s.data(), s.size()); }
  // Blocking reads with an idle timeout (no byte for idle_ms -> SyncError), honouring stop().
  std::string read_line_idle(LineReader& r, int idle_ms, const char* what);
  Source reader_source(LineReader& r, int idle_ms, const char* what);

  // Helper-mode upstream lanes (src/helper/helper.cc): uploads run concurrently, interleaved frame
  // by frame on the one upstream helper; replies "@lane ..." are read by the waiters (up_wait). A batch with
  // large files goes to the bulk lane (bulk_thread_), so an edit made meanwhile is uploaded at
  // once on its own lane instead of behind the archive; an edit of a path the bulk upload carries
  // waits for it (deferred_) so the older bytes can never land last.
  void dispatch_upstream(std::vector<FileInfo>& changes, long first_event_us);
  void bulk_loop();
  // one frame (header + optional data) written atomically to the upstream helper's stdin
  void up_frame(const std::string& head, const char* d, size_t n);
  void wait_no_priority();  // bulk frames wait while an interactive upload is sending
  std::string up_wait(int lane, int idle_ms, const char* what);
  void start_up_reader();
  std::mutex up_wmu_, up_pmu_;
  std::condition_variable up_pcv_;
  std::atomic<int> up_prio_{0};
  std::mutex up_rmu_;
  std::condition_variable up_rcv_;
  std::map<int, std::string> up_replies_;  // up_rmu_
  bool up_reader_eof_ = false;             // up_rmu_
  bool up_reading_ = false;                // up_rmu_: a waiter is reading up_out_
  std::thread bulk_thread_;
  std::deque<std::vector<FileInfo>> bulk_q_;  // q_mu_
  bool bulk_busy_ = false;                    // q_mu_
  std::vector<std::string> deferred_;         // q_mu_: abs paths re-evaluated after the bulk upload
  // Paths being uploaded or removed (downstream leaves them alone until the index has them).
  std::mutex inflight_mu_;
  std::map<std::string, int> inflight_;
  std::map<std::string, int> inflight_bulk_;
  void mark_inflight(const std::vector<FileInfo>& files, bool bulk, bool on);
  bool in_flight(const std::string& rel, bool bulk_only);
  void warn_large(const std::string& rel, int64_t size);  // index lock held
  struct Progress;
  void send_changes_to_upstream(std::vector<FileInfo> changes);
  void diff_server_client(const std::string& abs, std::vector<FileInfo>* send,
                          std::map<std::string, FileInfo>* download, bool dont_send);

  // downstream
  void downstream_loop();
  std::vector<FileInfo> collect_changes(std::map<std::string, FileInfo>* removes);
  // Helper mode: files downloaded while their stamp was fresh and still since, checked by CRC-32
  // on both sides; the ones whose content differs are added to *creates (down shell held).
  void verify_unsettled(const std::vector<FileInfo>& files, std::vector<FileInfo>* creates);
  bool probe_changes();  // fast mode: did anything under dest change since the last probes?
  std::string probe_id_;
  bool up_has_head_ = true;  // fast mode: container has `head -c` for streamed uploads
  long probe_seq_ = 0;
  void apply_downstream(const std::vector<FileInfo>& creates, std::map<std::string, FileInfo>& removes);
  // Streams the files from the container straight into the local tree (no archive in memory).
  // bulk: on the bulk download channel (its own exec session and helper), so pod-side changes
  // keep flowing on the main channel while a multi-GB file comes down.
  void download_and_apply(const std::vector<FileInfo>& files, bool bulk = false);
  // Helper mode: files >= 4 MiB found by a scan are downloaded by bulk_down_loop on a second
  // channel; the paths stay in downloading_ (skipped by later scans) until they are in.
  void bulk_down_loop();
  bool open_bulk_down_shell();
  bool downloading(const std::string& rel);
  void wait_bulk_down_idle();
  std::unique_ptr<Shell> bulk_down_shell_;
  LineReader bulk_down_out_;
  std::mutex bulk_down_mu_;      // the bulk download channel (held across a download)
  std::mutex bulk_down_ptr_mu_;  // bulk_down_shell_ itself (set, terminated, reset)
  std::thread bulk_down_thread_;
  std::atomic<bool> bulk_down_on_{false};  // bulk_down_thread_ runs: big downloads may go there
  std::deque<std::vector<FileInfo>> bulk_down_q_;  // q_mu_
  bool bulk_down_busy_ = false;                    // q_mu_
  std::set<std::string> downloading_;              // inflight_mu_
  // Extracts a tar / tar.gz stream into the local folder, each file through a temp name and a
  // rename. leftover != nullptr: the stream continues after the archive (fast protocol) — a gzip
  // member is read exactly to its end and any bytes pulled past it are returned there.
  void untar_stream(Source raw, std::string* leftover);
  void remove_files_and_folders(std::map<std::string, FileInfo>& removes);
  void delete_safe_recursive(const std::string& rel, std::map<std::string, FileInfo>& removes);
  void create_folders(const std::vector<FileInfo>& dirs);
  std::map<std::string, FileInfo> clone_index();

  // symlinks (sync/symlink.go)
  std::optional<fs::StatInfo> add_symlink(const std::string& rel, const std::string& abs);
  void remove_symlinks(const std::string& abs);

  // shells / modes
  std::string remote(const std::string& container_path) const;  // apply transport prefix
  // `opened`: the shell, already opened (open_shells keeps the order of the opens)
  void open_up_shell(std::unique_ptr<Shell> opened = nullptr);
  void open_down_shell();
  // starts the container-side change watch in the helper that reports it
  void request_watch();
  // role: kUploader uploads a missing helper and says when it is there, kWaiter (a shell opened
  // at the same time) waits for that instead of uploading the same bytes again, kAlone does both
  enum HelperRole { kAlone, kUploader, kWaiter };
  bool start_helper(std::unique_ptr<Shell>& sh, LineReader& out, HelperRole role = kAlone);
  std::mutex helper_mu_;
  std::condition_variable helper_cv_;
  int helper_state_ = 0;  // the uploader's helper: 0 not known yet, 1 in the container, 2 failed
  bool concurrent_open_ = false;  // open_shells is opening both shells (written before its thread starts)
  void fail(const std::string& err);  // stream failure -> reconnect or stop
  void supervise();

  Options o_;
  std::shared_ptr<Transport> transport_;
  Mode mode_;
  std::string dest_;  // shell-visible dest path
  int window_ms_ = 15, poll_ms_ = 250;
  FileIndex index_;
  GitIgnore ignore_, download_ignore_, upload_ignore_;
  bool has_ignore_ = false, has_download_ignore_ = false, has_upload_ignore_ = false;
  std::shared_ptr<log::FileLogger> log_;

  std::unique_ptr<Shell> up_shell_, down_shell_;
  LineReader up_out_, down_out_, down_err_;
  LineReader up_err_;  // change events of the upstream helper (it runs the watch: own-echo filter)
  bool up_helper_ = false, down_helper_ = false;
  std::mutex up_shell_mu_, down_shell_mu_;

  std::unique_ptr<TreeWatcher> watcher_;
  std::map<std::string, std::unique_ptr<PollWatcher>> symlinks_;  // abs symlink path -> target watcher
  std::map<std::string, std::string> symlink_targets_;
  std::mutex symlink_mu_;

  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<UpEvent> queue_;
  bool up_busy_ = false;  // guarded by q_mu_
  void wait_upstream_idle();
  void drop_identical_copies(std::vector<FileInfo>& changes);

  std::thread up_thread_, down_thread_, supervisor_;
  // Stop diagnostics: one bit per loop thread that has not returned yet, and the step stop() is
  // at. A stop that takes longer than DEVSPACE_SYNC_STOP_WARN_MS (20 s) logs both, every period,
  // to sync.log and stderr, so a stop that never ends names the loop and the step it waits on.
  enum LoopBit : unsigned { kUpLoop = 1, kBulkLoop = 2, kBulkDownLoop = 4, kDownLoop = 8, kSupervisor = 16 };
  std::atomic<unsigned> live_loops_{0};
  std::atomic<const char*> stop_step_{""};
  std::thread spawn_loop(LoopBit bit, std::function<void()> body);
  std::string describe_stop_state();
  std::atomic<bool> running_{false}, stopping_{false};
  std::atomic<bool> failed_{false};
  std::mutex pod_mu_;
  std::mutex state_mu_;
  std::condition_variable state_cv_;
  bool initial_done_ = false;
  std::string error_;
  Stats stats_;
  std::mutex stats_mu_;
  // Paths whose upload was cut off by a broken stream (index lock): re-sent after a reconnect
  // even though the container may now hold a newer-looking partial copy.
  std::set<std::string> force_up_;
  std::set<std::string> warned_large_;  // index lock
  int64_t large_warn_bytes_ = 1ll << 30;
  std::string pending_failure_;
  int reconnects_ = 0;
};

// True when a relative path has a ".." segment (archive entries from the container that
// would land outside the synced folder are skipped).
bool has_dotdot_segment(const std::string& rel);

}  // namespace sync
}  // namespace ds
