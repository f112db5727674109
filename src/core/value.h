// Dynamic document tree used for YAML / JSON / config / manifests.
//
// The reference unmarshals YAML into typed Go structs (config/versions/latest/schema.go:23)
// and walks map[interface{}]interface{} trees for vars and manifests
// (deploy/kubectl/walk/walk.go:10). Here a single ordered tree type serves both roles;
// typed access and strict validation are provided by config/schema.
#pragma once

#include <cstdint>
#include <functional>
#include <initializer_list>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ds {

class Value {
 public:
  enum class Type { Null, Bool, Int, Float, String, Seq, Map };
  using SeqT = std::vector<Value>;
  using MapT = std::vector<std::pair<std::string, Value>>;

  Value() = default;
  Value(std::nullptr_t) {}
  Value(bool b) : type_(Type::Bool), b_(b) {}
  Value(int i) : type_(Type::Int), i_(i) {}
  Value(int64_t i) : type_(Type::Int), i_(i) {}
  Value(uint64_t i) : type_(Type::Int), i_((int64_t)i) {}
  Value(double d) : type_(Type::Float), d_(d) {}
  Value(const char* s) : type_(Type::String), s_(s) {}
  Value(std::string s) : type_(Type::String), s_(std::move(s)) {}

  static Value seq() {
    Value v;
    v.type_ = Type::Seq;
    return v;
  }
  static Value map() {
    Value v;
    v.type_ = Type::Map;
    return v;
  }
  static Value seq_of(std::initializer_list<Value> items) {
    Value v = seq();
    for (auto& it : items) v.seq_.push_back(it);
    return v;
  }
  static Value strings(const std::vector<std::string>& items) {
    Value v = seq();
    for (auto& it : items) v.seq_.emplace_back(it);
    return v;
  }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_int() const { return type_ == Type::Int; }
  bool is_float() const { return type_ == Type::Float; }
  bool is_number() const { return type_ == Type::Int || type_ == Type::Float; }
  bool is_string() const { return type_ == Type::String; }
  bool is_seq() const { return type_ == Type::Seq; }
  bool is_map() const { return type_ == Type::Map; }
  bool is_scalar() const { return !is_seq() && !is_map(); }

  // YAML-level: the scalar was written with quotes (so "123" stays a string).
  bool quoted() const { return quoted_; }
  void set_quoted(bool q) { quoted_ = q; }

  bool as_bool(bool def = false) const;
  int64_t as_int(int64_t def = 0) const;
  double as_double(double def = 0) const;
  // Scalar rendered as text (ints/bools formatted, null -> "").
  std::string as_string(const std::string& def = "") const;
  const std::string& str() const { return s_; }

  // Sequence access
  const SeqT& items() const { return seq_; }
  SeqT& items() { return seq_; }
  void push(Value v) {
    if (type_ == Type::Null) type_ = Type::Seq;
    seq_.push_back(std::move(v));
  }
  size_t size() const { return is_seq() ? seq_.size() : is_map() ? map_.size() : 0; }
  const Value& operator[](size_t i) const { return seq_.at(i); }
  Value& operator[](size_t i) { return seq_.at(i); }
  const Value& operator[](int i) const { return seq_.at((size_t)i); }
  Value& operator[](int i) { return seq_.at((size_t)i); }

  // Map access
  const MapT& entries() const { return map_; }
  MapT& entries() { return map_; }
  bool has(const std::string& k) const;
  const Value* find(const std::string& k) const;
  Value* find(const std::string& k);
  // Returns a null Value when absent (never throws).
  const Value& get(const std::string& k) const;
  // Creates the key when absent (turns Null into Map).
  Value& operator[](const std::string& k);
  Value& operator[](const char* k) { return (*this)[std::string(k)]; }
  void set(const std::string& k, Value v) { (*this)[k] = std::move(v); }
  bool erase(const std::string& k);
  std::vector<std::string> keys() const;

  // Dotted path helpers: "dev.sync" -> nested lookup (no creation).
  const Value& at_path(const std::string& dotted) const;
  Value& ensure_path(const std::string& dotted);

  bool operator==(const Value& o) const;
  bool operator!=(const Value& o) const { return !(*this == o); }

  // Empty == null, or empty map/seq/string (mirrors reflect isZero in the reference's Split).
  bool empty_like() const;

  static const Value& null_value();

 private:
  Type type_ = Type::Null;
  bool quoted_ = false;
  bool b_ = false;
  int64_t i_ = 0;
  double d_ = 0;
  std::string s_;
  SeqT seq_;
  MapT map_;
};

const char* type_name(Value::Type t);

// Deep merge (config/configutil/merge.go:17 semantics): maps merge recursively,
// sequences and scalars in `over` replace those in `base`; null in `over` is ignored.
void merge_into(Value& base, const Value& over);

// Remove null entries and empty maps/seqs recursively (used before saving).
Value prune_empty(const Value& v);

// Generic tree walk: calls fn on each string scalar; fn may replace it.
// (deploy/kubectl/walk/walk.go:10)
void walk_strings(Value& v, const std::function<bool(const std::string& key, Value& val)>& fn,
                  const std::string& key = "");

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// YAML
Value yaml_parse(const std::string& text);                  // first document
std::vector<Value> yaml_parse_all(const std::string& text);  // all documents
std::string yaml_dump(const Value& v);
Value yaml_load_file(const std::string& path);

// JSON
Value json_parse(const std::string& text);
std::string json_dump(const Value& v, int indent = -1);
std::string json_escape(const std::string& s);

}  // namespace ds
