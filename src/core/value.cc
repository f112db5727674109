#include "core/value.h"

#include <cmath>
#include <cstdarg>
#include <cstdio>

#include "core/strutil.h"

namespace ds {

std::string strfmt(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  char buf[1024];
  va_list ap2;
  va_copy(ap2, ap);
  int n = vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n < (int)sizeof(buf)) {
    va_end(ap2);
    return std::string(buf, n < 0 ? 0 : n);
  }
  std::string out(n + 1, '\0');
  vsnprintf(&out[0], n + 1, fmt, ap2);
  va_end(ap2);
  out.resize(n);
  return out;
}

const char* type_name(Value::Type t) {
  switch (t) {
    case Value::Type::Null: return "null";
    case Value::Type::Bool: return "bool";
    case Value::Type::Int: return "int";
    case Value::Type::Float: return "float";
    case Value::Type::String: return "string";
    case Value::Type::Seq: return "sequence";
    case Value::Type::Map: return "map";
  }
  return "?";
}

const Value& Value::null_value() {
  static const Value n;
  return n;
}

bool Value::as_bool(bool def) const {
  switch (type_) {
    case Type::Bool: return b_;
    case Type::Int: return i_ != 0;
    case Type::String: {
      std::string l = to_lower(s_);
      if (l == "true" || l == "yes" || l == "on" || l == "1") return true;
      if (l == "false" || l == "no" || l == "off" || l == "0") return false;
      return def;
    }
    default: return def;
  }
}

int64_t Value::as_int(int64_t def) const {
  switch (type_) {
    case Type::Int: return i_;
    case Type::Float: return (int64_t)d_;
    case Type::Bool: return b_ ? 1 : 0;
    case Type::String: {
      int64_t v;
      if (parse_int64(trim(s_), &v)) return v;
      return def;
    }
    default: return def;
  }
}

double Value::as_double(double def) const {
  switch (type_) {
    case Type::Int: return (double)i_;
    case Type::Float: return d_;
    case Type::String: {
      double v;
      if (parse_double(trim(s_), &v)) return v;
      return def;
    }
    default: return def;
  }
}

static std::string format_double(double d) {
  if (std::isinf(d)) return d > 0 ? ".inf" : "-.inf";
  if (std::isnan(d)) return ".nan";
  if (d == std::floor(d) && std::fabs(d) < 1e15) {
    return strfmt("%.1f", d);
  }
  std::string s = strfmt("%.17g", d);
  // shortest round-trip representation
  for (int prec = 1; prec <= 17; ++prec) {
    std::string t = strfmt("%.*g", prec, d);
    if (std::strtod(t.c_str(), nullptr) == d) return t;
  }
  return s;
}

std::string Value::as_string(const std::string& def) const {
  switch (type_) {
    case Type::String: return s_;
    case Type::Int: return std::to_string(i_);
    case Type::Float: return format_double(d_);
    case Type::Bool: return b_ ? "true" : "false";
    case Type::Null: return def;
    default: return def;
  }
}

bool Value::has(const std::string& k) const { return find(k) != nullptr; }

const Value* Value::find(const std::string& k) const {
  if (type_ != Type::Map) return nullptr;
  for (auto& e : map_)
    if (e.first == k) return &e.second;
  return nullptr;
}

Value* Value::find(const std::string& k) {
  if (type_ != Type::Map) return nullptr;
  for (auto& e : map_)
    if (e.first == k) return &e.second;
  return nullptr;
}

const Value& Value::get(const std::string& k) const {
  const Value* v = find(k);
  return v ? *v : null_value();
}

Value& Value::operator[](const std::string& k) {
  if (type_ == Type::Null) type_ = Type::Map;
  if (type_ != Type::Map) throw std::runtime_error("value is not a map (key " + k + ")");
  for (auto& e : map_)
    if (e.first == k) return e.second;
  map_.emplace_back(k, Value());
  return map_.back().second;
}

bool Value::erase(const std::string& k) {
  if (type_ != Type::Map) return false;
  for (auto it = map_.begin(); it != map_.end(); ++it) {
    if (it->first == k) {
      map_.erase(it);
      return true;
    }
  }
  return false;
}

std::vector<std::string> Value::keys() const {
  std::vector<std::string> out;
  for (auto& e : map_) out.push_back(e.first);
  return out;
}

const Value& Value::at_path(const std::string& dotted) const {
  const Value* cur = this;
  for (auto& part : split(dotted, ".")) {
    if (part.empty()) continue;
    cur = cur->find(part);
    if (!cur) return null_value();
  }
  return *cur;
}

Value& Value::ensure_path(const std::string& dotted) {
  Value* cur = this;
  for (auto& part : split(dotted, ".")) {
    if (part.empty()) continue;
    cur = &(*cur)[part];
  }
  return *cur;
}

bool Value::operator==(const Value& o) const {
  if (type_ != o.type_) {
    if (is_number() && o.is_number()) return as_double() == o.as_double();
    return false;
  }
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return b_ == o.b_;
    case Type::Int: return i_ == o.i_;
    case Type::Float: return d_ == o.d_;
    case Type::String: return s_ == o.s_;
    case Type::Seq: return seq_ == o.seq_;
    case Type::Map: {
      if (map_.size() != o.map_.size()) return false;
      for (auto& e : map_) {
        const Value* ov = o.find(e.first);
        if (!ov || !(*ov == e.second)) return false;
      }
      return true;
    }
  }
  return false;
}

bool Value::empty_like() const {
  switch (type_) {
    case Type::Null: return true;
    case Type::Seq: return seq_.empty();
    case Type::Map: return map_.empty();
    default: return false;
  }
}

void merge_into(Value& base, const Value& over) {
  if (over.is_null()) return;
  if (over.is_map() && base.is_map()) {
    for (auto& e : over.entries()) {
      Value* b = base.find(e.first);
      if (b && b->is_map() && e.second.is_map()) {
        merge_into(*b, e.second);
      } else if (!e.second.is_null()) {
        base[e.first] = e.second;
      }
    }
    return;
  }
  base = over;
}

Value prune_empty(const Value& v) {
  if (v.is_map()) {
    Value out = Value::map();
    for (auto& e : v.entries()) {
      Value c = prune_empty(e.second);
      if (c.is_null()) continue;
      if ((c.is_map() || c.is_seq()) && c.size() == 0) continue;
      out[e.first] = std::move(c);
    }
    return out;
  }
  if (v.is_seq()) {
    Value out = Value::seq();
    for (auto& it : v.items()) {
      if (it.is_null()) continue;
      out.push(prune_empty(it));
    }
    return out;
  }
  return v;
}

void walk_strings(Value& v, const std::function<bool(const std::string&, Value&)>& fn, const std::string& key) {
  if (v.is_map()) {
    for (auto& e : v.entries()) walk_strings(e.second, fn, e.first);
  } else if (v.is_seq()) {
    for (auto& it : v.items()) walk_strings(it, fn, key);
  } else if (v.is_string()) {
    fn(key, v);
  }
}

}  // namespace ds
