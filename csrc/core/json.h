// Minimal JSON value + streaming parser/serializer for the control plane.
//
// The reference frames every control message as a concatenated JSON value on a
// TCP stream (Go json.Decoder, distributor/transport.go:97-124) and marshals map
// keys as sorted strings (Go encoding/json). This codec reproduces that framing:
// `parse_prefix` consumes exactly one JSON value from the front of a buffer and
// reports how many bytes it used, or "incomplete" when more bytes are needed.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace dissem {

class Json {
 public:
  enum class Kind : uint8_t { Null, Bool, Int, Float, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::map<std::string, Json>;  // sorted keys == Go marshal order

  Json() : kind_(Kind::Null) {}
  Json(std::nullptr_t) : kind_(Kind::Null) {}
  Json(bool b) : kind_(Kind::Bool), b_(b) {}
  Json(int v) : kind_(Kind::Int), neg_(v < 0), mag_(v < 0 ? uint64_t(-(int64_t)v) : uint64_t(v)) {}
  Json(int64_t v) : kind_(Kind::Int), neg_(v < 0), mag_(v < 0 ? uint64_t(0) - uint64_t(v) : uint64_t(v)) {}
  Json(uint64_t v) : kind_(Kind::Int), neg_(false), mag_(v) {}
  Json(unsigned v) : kind_(Kind::Int), neg_(false), mag_(v) {}
  Json(double d) : kind_(Kind::Float), d_(d) {}
  Json(const char* s) : kind_(Kind::String), s_(std::make_shared<std::string>(s)) {}
  Json(std::string s) : kind_(Kind::String), s_(std::make_shared<std::string>(std::move(s))) {}
  Json(Array a) : kind_(Kind::Array), a_(std::make_shared<Array>(std::move(a))) {}
  Json(Object o) : kind_(Kind::Object), o_(std::make_shared<Object>(std::move(o))) {}

  static Json object() { return Json(Object{}); }
  static Json array() { return Json(Array{}); }

  Kind kind() const { return kind_; }
  bool is_null() const { return kind_ == Kind::Null; }
  bool is_object() const { return kind_ == Kind::Object; }
  bool is_array() const { return kind_ == Kind::Array; }
  bool is_string() const { return kind_ == Kind::String; }
  bool is_number() const { return kind_ == Kind::Int || kind_ == Kind::Float; }

  int64_t as_i64() const;
  uint64_t as_u64() const;
  double as_f64() const;
  bool as_bool() const;
  const std::string& as_str() const;
  const Array& as_array() const;
  Array& as_array();
  const Object& as_object() const;
  Object& as_object();

  // Object access. `operator[]` on a non-const value converts Null to Object.
  Json& operator[](const std::string& key);
  const Json* find(const std::string& key) const;  // case-insensitive fallback like Go
  bool has(const std::string& key) const { return find(key) != nullptr; }
  int64_t get_i64(const std::string& key, int64_t dflt = 0) const;
  uint64_t get_u64(const std::string& key, uint64_t dflt = 0) const;
  std::string get_str(const std::string& key, const std::string& dflt = "") const;
  bool get_bool(const std::string& key, bool dflt = false) const;
  void push_back(Json v);

  std::string dump() const;
  void dump_to(std::string& out) const;

  // Parse exactly one value; throws on malformed input or trailing garbage.
  static Json parse(const std::string& text);
  // Parse one value from buf[0..len). Returns bytes consumed (>0), 0 if the
  // value is incomplete (need more bytes), throws on malformed input. Leading
  // whitespace is skipped and counted.
  static size_t parse_prefix(const char* buf, size_t len, Json& out);
  // The extent of one value at the front of buf[0..len) without building it:
  // bytes it spans (leading whitespace included), 0 if incomplete. Checks
  // nesting and string syntax only (the decoder validates the rest); lets a
  // stream reader find a message's end once instead of re-parsing a large
  // message on every partial read.
  static size_t scan_prefix(const char* buf, size_t len);

 private:
  Kind kind_;
  bool b_ = false;
  bool neg_ = false;
  uint64_t mag_ = 0;
  double d_ = 0;
  // Value semantics: copies are deep (control messages are small).
  std::shared_ptr<std::string> s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
  void detach();  // copy-on-write before mutation

 public:
  Json(const Json&) = default;
  Json(Json&&) noexcept = default;
  Json& operator=(const Json&) = default;
  Json& operator=(Json&&) noexcept = default;
};

struct JsonIncomplete : std::runtime_error {
  JsonIncomplete() : std::runtime_error("incomplete json") {}
};

}  // namespace dissem
