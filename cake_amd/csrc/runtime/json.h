// Minimal JSON value, parser and serializer for the host runtime.
//
// Needed by the safetensors header / model.safetensors.index.json handling
// (reference: cake-core/src/utils/mod.rs:42-104 via serde_json, and
// cake-split-model/src/main.rs:15-25,105-139) and by the C++/Python boundary.
// Objects keep insertion order (the safetensors header is rewritten in the
// order it was read), numbers are kept as double plus an exact int64 when
// integral (tensor offsets exceed 2^53 only for >8 PiB files).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace cake {

class Json {
 public:
  enum Type { Null, Bool, Number, String, Array, Object };

  Json() : type_(Null) {}
  static Json boolean(bool b) { Json j; j.type_ = Bool; j.b_ = b; return j; }
  static Json number(double d) { Json j; j.type_ = Number; j.d_ = d; j.i_ = (int64_t)d; j.is_int_ = false; return j; }
  static Json integer(int64_t i) { Json j; j.type_ = Number; j.d_ = (double)i; j.i_ = i; j.is_int_ = true; return j; }
  static Json string(std::string s) { Json j; j.type_ = String; j.s_ = std::move(s); return j; }
  static Json array() { Json j; j.type_ = Array; return j; }
  static Json object() { Json j; j.type_ = Object; return j; }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Null; }
  bool is_object() const { return type_ == Object; }
  bool is_array() const { return type_ == Array; }
  bool is_string() const { return type_ == String; }
  bool is_number() const { return type_ == Number; }

  bool as_bool() const { check(Bool); return b_; }
  double as_double() const { check(Number); return d_; }
  int64_t as_int() const { check(Number); return is_int_ ? i_ : (int64_t)d_; }
  const std::string& as_string() const { check(String); return s_; }

  // arrays
  size_t size() const { return type_ == Array ? arr_.size() : (type_ == Object ? obj_.size() : 0); }
  const Json& at(size_t i) const { check(Array); return arr_.at(i); }
  void push(Json v) { check(Array); arr_.push_back(std::move(v)); }
  const std::vector<Json>& items() const { check(Array); return arr_; }

  // objects (ordered)
  bool has(const std::string& k) const;
  const Json& get(const std::string& k) const;
  void set(const std::string& k, Json v);
  const std::vector<std::pair<std::string, Json>>& members() const { check(Object); return obj_; }

  static Json parse(const std::string& text);
  std::string dump(int indent = -1) const;

 private:
  void check(Type t) const {
    if (type_ != t) throw std::runtime_error("json: wrong type access");
  }
  void dump_to(std::string& out, int indent, int depth) const;

  Type type_;
  bool b_ = false;
  double d_ = 0;
  int64_t i_ = 0;
  bool is_int_ = false;
  std::string s_;
  std::vector<Json> arr_;
  std::vector<std::pair<std::string, Json>> obj_;
  std::map<std::string, size_t> index_;
};

}  // namespace cake
