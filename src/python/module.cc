// Python bindings for the native engine (devspace_amd._native).
// Used by the workload-side hot-reload runner (inotify watcher), the benchmark harness
// (sync sessions driven in-process) and the pytest suite.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <condition_variable>
#include <deque>
#include <mutex>

#include "config/config.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/match.h"
#include "core/value.h"
#include "core/watch.h"
#include "sync/frame.h"
#include "sync/sync.h"

namespace py = pybind11;
using namespace ds;

static py::object to_py(const Value& v) {
  switch (v.type()) {
    case Value::Type::Null: return py::none();
    case Value::Type::Bool: return py::bool_(v.as_bool());
    case Value::Type::Int: return py::int_(v.as_int());
    case Value::Type::Float: return py::float_(v.as_double());
    case Value::Type::String: return py::str(v.str());
    case Value::Type::Seq: {
      py::list l;
      for (auto& it : v.items()) l.append(to_py(it));
      return l;
    }
    case Value::Type::Map: {
      py::dict d;
      for (auto& e : v.entries()) d[py::str(e.first)] = to_py(e.second);
      return d;
    }
  }
  return py::none();
}

static Value from_py(const py::handle& o) {
  if (o.is_none()) return Value();
  if (py::isinstance<py::bool_>(o)) return Value(o.cast<bool>());
  if (py::isinstance<py::int_>(o)) return Value((int64_t)o.cast<long long>());
  if (py::isinstance<py::float_>(o)) return Value(o.cast<double>());
  if (py::isinstance<py::str>(o)) return Value(o.cast<std::string>());
  if (py::isinstance<py::dict>(o)) {
    Value m = Value::map();
    for (auto item : o.cast<py::dict>()) m[py::str(item.first).cast<std::string>()] = from_py(item.second);
    return m;
  }
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    Value s = Value::seq();
    for (auto item : o) s.push(from_py(item));
    return s;
  }
  return Value(py::str(o).cast<std::string>());
}

// Inotify watcher with a queue drained from Python (no callbacks across threads).
class PyWatcher {
 public:
  // settled_only: report a path only once its write finished (close-after-write, rename into
  // place, delete), not on every IN_MODIFY of a file still being written.
  explicit PyWatcher(const std::string& root, bool settled_only = false) {
    std::string err;
    if (!w_->start(
            root,
            [this, settled_only](const std::string& p, bool settled) {
              if (settled_only && !settled) return;
              {
                std::lock_guard<std::mutex> g(mu_);
                q_.push_back(p);
              }
              cv_.notify_all();
            },
            &err))
      throw std::runtime_error(err);
  }
  std::vector<std::string> poll(int timeout_ms) {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [this] { return !q_.empty(); });
    std::vector<std::string> out(q_.begin(), q_.end());
    q_.clear();
    return out;
  }
  void close() { w_->stop(); }

 private:
  std::unique_ptr<TreeWatcher> w_ = make_tree_watcher();
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> q_;
};

class PySync {
 public:
  PySync(const std::string& watch_path, const std::string& dest_path, const std::string& mode,
         std::vector<std::string> exclude, std::vector<std::string> download_exclude,
         std::vector<std::string> upload_exclude, const std::string& helper_path, const std::string& log_dir,
         const std::string& pod_name) {
    sync::Options o;
    o.watch_path = watch_path;
    o.dest_path = dest_path;
    o.mode = sync::parse_mode(mode);
    o.exclude_paths = std::move(exclude);
    o.download_exclude_paths = std::move(download_exclude);
    o.upload_exclude_paths = std::move(upload_exclude);
    o.helper_path = helper_path;
    o.pod_name = pod_name;
    if (!log_dir.empty()) log::logdir() = log_dir;
    o.reconnect = [] { return std::make_shared<sync::LocalShellTransport>(); };
    s_ = std::make_unique<sync::Session>(o, std::make_shared<sync::LocalShellTransport>());
  }
  void start() {
    py::gil_scoped_release nogil;
    s_->start();
  }
  bool wait_initial_sync(int ms) {
    py::gil_scoped_release nogil;
    return s_->wait_initial_sync(ms);
  }
  void stop() {
    py::gil_scoped_release nogil;
    s_->stop();
  }
  bool running() { return s_->running(); }
  std::string error() { return s_->error(); }
  std::string mode() { return sync::mode_name(s_->effective_mode()); }
  py::dict stats() {
    auto st = s_->stats();
    py::dict d;
    d["upstream_batches"] = st.upstream_batches;
    d["upstream_changes"] = st.upstream_changes;
    d["downstream_batches"] = st.downstream_batches;
    d["downstream_changes"] = st.downstream_changes;
    d["reconnects"] = st.reconnects;
    d["last_upload_ms"] = st.last_upload_ms;
    d["bytes_up"] = st.bytes_up;
    d["bytes_down"] = st.bytes_down;
    d["full_scans"] = st.full_scans;
    d["probes"] = st.probes;
    d["probe_hits"] = st.probe_hits;
    d["probe_interval_ms"] = st.probe_interval_ms;
    d["scan_bytes"] = st.scan_bytes;
    return d;
  }

 private:
  std::unique_ptr<sync::Session> s_;
};

// The sync decision rules on an unstarted session, for property tests:
// the caller sets up the index and asks shouldUpload / shouldDownload / shouldRemove*.
class PyRules {
 public:
  PyRules(const std::string& watch_path, const std::string& mode, std::vector<std::string> exclude,
          std::vector<std::string> download_exclude, std::vector<std::string> upload_exclude) {
    sync::Options o;
    o.watch_path = watch_path;
    o.dest_path = "/app";
    o.mode = sync::parse_mode(mode);
    o.exclude_paths = std::move(exclude);
    o.download_exclude_paths = std::move(download_exclude);
    o.upload_exclude_paths = std::move(upload_exclude);
    o.silent = true;
    s_ = std::make_unique<sync::Session>(o, std::make_shared<sync::LocalShellTransport>());
    s_->setup();
  }
  void put(const std::string& name, int64_t size, int64_t mtime, bool is_dir, bool is_symlink, int64_t local_mtime_ns) {
    sync::FileInfo f;
    f.name = name;
    f.size = size;
    f.mtime = mtime;
    f.is_dir = is_dir;
    f.is_symlink = is_symlink;
    f.local_mtime_ns = local_mtime_ns;
    std::lock_guard<std::mutex> g(s_->index().mu);
    s_->index().files[name] = f;
  }
  void create_dir(const std::string& d) {
    std::lock_guard<std::mutex> g(s_->index().mu);
    s_->index().create_dir(d);
  }
  void remove_dir(const std::string& d) {
    std::lock_guard<std::mutex> g(s_->index().mu);
    s_->index().remove_dir(d);
  }
  py::object get(const std::string& name) {
    std::lock_guard<std::mutex> g(s_->index().mu);
    sync::FileInfo* f = s_->index().find(name);
    if (!f) return py::none();
    py::dict d;
    d["size"] = f->size;
    d["mtime"] = f->mtime;
    d["is_dir"] = f->is_dir;
    d["is_symlink"] = f->is_symlink;
    return d;
  }
  std::vector<std::string> names() {
    std::lock_guard<std::mutex> g(s_->index().mu);
    std::vector<std::string> out;
    for (auto& kv : s_->index().files) out.push_back(kv.first);
    return out;
  }
  bool should_upload(const std::string& rel, bool exists, bool is_dir, bool is_symlink, int64_t mtime_sec,
                     int64_t mtime_nsec, int64_t size, bool initial) {
    fs::StatInfo st;
    st.exists = exists;
    st.is_dir = is_dir;
    st.is_reg = exists && !is_dir && !is_symlink;
    st.is_symlink = is_symlink;
    st.mtime_sec = mtime_sec;
    st.mtime_nsec = mtime_nsec;
    st.size = size;
    std::lock_guard<std::mutex> g(s_->index().mu);
    return s_->should_upload(rel, st, initial);
  }
  bool should_download(const std::string& name, int64_t size, int64_t mtime, bool is_dir, bool is_symlink) {
    sync::FileInfo f;
    f.name = name;
    f.size = size;
    f.mtime = mtime;
    f.is_dir = is_dir;
    f.is_symlink = is_symlink;
    std::lock_guard<std::mutex> g(s_->index().mu);
    return s_->should_download(f);
  }
  bool should_remove_remote(const std::string& rel) {
    std::lock_guard<std::mutex> g(s_->index().mu);
    return s_->should_remove_remote(rel);
  }
  bool should_remove_local(const std::string& abs, const std::string& name, int64_t size, int64_t mtime, bool is_dir) {
    sync::FileInfo f;
    f.name = name;
    f.size = size;
    f.mtime = mtime;
    f.is_dir = is_dir;
    std::lock_guard<std::mutex> g(s_->index().mu);
    return s_->should_remove_local(abs, f);
  }
  void apply_archive(py::bytes data) {
    std::string a(data);
    py::gil_scoped_release nogil;
    s_->apply_downstream_archive(a);
  }

 private:
  std::unique_ptr<sync::Session> s_;
};

// The strict config schema as nested dicts (docs generator: docs/reference/configuration.md).
py::object schema_to_py(const config::Schema& s) {
  static const char* kinds[] = {"string", "integer", "boolean", "any", "struct", "list", "map"};
  py::dict d;
  d["kind"] = kinds[s.kind];
  if (!s.type_name.empty()) d["type"] = s.type_name;
  if (s.kind == config::Schema::Struct) {
    py::list fields;
    for (auto& f : s.fields) fields.append(py::make_tuple(f.first, schema_to_py(*f.second)));
    d["fields"] = fields;
  }
  if (s.elem) d["elem"] = schema_to_py(*s.elem);
  return std::move(d);
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "devspace native engine (C++17) bindings";
  log::set_fatal_throws(true);
  m.def("yaml_parse", [](const std::string& s) { return to_py(yaml_parse(s)); });
  m.def("yaml_parse_all", [](const std::string& s) {
    py::list l;
    for (auto& d : yaml_parse_all(s)) l.append(to_py(d));
    return l;
  });
  m.def("yaml_dump", [](py::object o) { return yaml_dump(from_py(o)); });
  m.def("json_dump", [](py::object o) { return json_dump(from_py(o)); });
  m.def("sha256_hex", [](py::bytes b) { return sha256_hex(std::string(b)); });
  m.def("gitignore_match", [](std::vector<std::string> pats, const std::string& path) {
    return GitIgnore(pats).matches(path);
  });
  m.def("dockerignore_match", [](std::vector<std::string> pats, const std::string& path) {
    return DockerIgnore(pats).matches(path);
  });
  m.def("glob_match", &glob_match);
  m.def("frame_header", [](const std::string& op, uint64_t len) {
    return py::bytes(sync::frame::header(op.empty() ? '\0' : op[0], len));
  });
  m.def("frame_parse", [](py::bytes b) {
    std::string h(b);
    if (h.size() != sync::frame::kHeaderSize) throw std::invalid_argument("frame header must be 9 bytes");
    char op;
    uint64_t len;
    sync::frame::parse_header((const unsigned char*)h.data(), &op, &len);
    return py::make_tuple(std::string(1, op), len);
  });
  m.def("parse_config", [](py::object data) { return to_py(config::parse_versioned(from_py(data))); });
  m.def("config_schema", [](const std::string& which) {
    if (which == "latest") return schema_to_py(config::schema_latest());
    if (which == "v1alpha1") return schema_to_py(config::schema_v1alpha1());
    if (which == "configs") return schema_to_py(config::schema_configs());
    if (which == "vars") return schema_to_py(config::schema_vars());
    throw std::invalid_argument("unknown schema " + which + " (latest|v1alpha1|configs|vars)");
  });
  m.def("copy_to_container",
        [](const std::string& local, const std::string& container, std::vector<std::string> excludes,
           const std::string& mode) {
          py::gil_scoped_release nogil;
          sync::Session::copy_to_container(std::make_shared<sync::LocalShellTransport>(), local, container,
                                           excludes, sync::parse_mode(mode));
        },
        py::arg("local"), py::arg("container"), py::arg("excludes") = std::vector<std::string>{},
        py::arg("mode") = "fast");
  py::class_<PyWatcher>(m, "Watcher")
      .def(py::init<const std::string&, bool>(), py::arg("root"), py::arg("settled_only") = false)
      .def("poll", &PyWatcher::poll, py::arg("timeout_ms") = 1000)
      .def("close", &PyWatcher::close);
  py::class_<PySync>(m, "SyncSession")
      .def(py::init<const std::string&, const std::string&, const std::string&, std::vector<std::string>,
                    std::vector<std::string>, std::vector<std::string>, const std::string&, const std::string&,
                    const std::string&>(),
           py::arg("watch_path"), py::arg("dest_path"), py::arg("mode") = "fast",
           py::arg("exclude") = std::vector<std::string>{}, py::arg("download_exclude") = std::vector<std::string>{},
           py::arg("upload_exclude") = std::vector<std::string>{}, py::arg("helper_path") = "",
           py::arg("log_dir") = "", py::arg("pod_name") = "")
      .def("start", &PySync::start)
      .def("wait_initial_sync", &PySync::wait_initial_sync, py::arg("timeout_ms") = 30000)
      .def("stop", &PySync::stop)
      .def("running", &PySync::running)
      .def("error", &PySync::error)
      .def("mode", &PySync::mode)
      .def("stats", &PySync::stats);
  py::class_<PyRules>(m, "SyncRules")
      .def(py::init<const std::string&, const std::string&, std::vector<std::string>, std::vector<std::string>,
                    std::vector<std::string>>(),
           py::arg("watch_path"), py::arg("mode") = "fast", py::arg("exclude") = std::vector<std::string>{},
           py::arg("download_exclude") = std::vector<std::string>{},
           py::arg("upload_exclude") = std::vector<std::string>{})
      .def("put", &PyRules::put, py::arg("name"), py::arg("size") = 0, py::arg("mtime") = 0, py::arg("is_dir") = false,
           py::arg("is_symlink") = false, py::arg("local_mtime_ns") = 0)
      .def("create_dir", &PyRules::create_dir)
      .def("remove_dir", &PyRules::remove_dir)
      .def("get", &PyRules::get)
      .def("names", &PyRules::names)
      .def("should_upload", &PyRules::should_upload, py::arg("rel"), py::arg("exists"), py::arg("is_dir"),
           py::arg("is_symlink"), py::arg("mtime_sec"), py::arg("mtime_nsec"), py::arg("size"), py::arg("initial"))
      .def("should_download", &PyRules::should_download, py::arg("name"), py::arg("size"), py::arg("mtime"),
           py::arg("is_dir") = false, py::arg("is_symlink") = false)
      .def("should_remove_remote", &PyRules::should_remove_remote)
      .def("should_remove_local", &PyRules::should_remove_local, py::arg("abs"), py::arg("name"), py::arg("size"),
           py::arg("mtime"), py::arg("is_dir") = false)
      .def("apply_archive", &PyRules::apply_archive);
}
