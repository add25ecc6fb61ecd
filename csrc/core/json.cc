#include "core/json.h"

#include <cctype>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <strings.h>

namespace dissem {

namespace {
[[noreturn]] void type_error(const char* want) {
  throw std::runtime_error(std::string("json: value is not ") + want);
}
}  // namespace

void Json::detach() {
  if (s_ && s_.use_count() > 1) s_ = std::make_shared<std::string>(*s_);
  if (a_ && a_.use_count() > 1) a_ = std::make_shared<Array>(*a_);
  if (o_ && o_.use_count() > 1) o_ = std::make_shared<Object>(*o_);
}

int64_t Json::as_i64() const {
  if (kind_ == Kind::Int) return int64_t(neg_ ? uint64_t(0) - mag_ : mag_);  // two's complement, no signed overflow
  if (kind_ == Kind::Float) return int64_t(d_);
  if (kind_ == Kind::Bool) return b_ ? 1 : 0;
  type_error("a number");
}
uint64_t Json::as_u64() const {
  if (kind_ == Kind::Int) return neg_ ? uint64_t(0) - mag_ : mag_;
  if (kind_ == Kind::Float) return d_ < 0 ? 0 : uint64_t(d_);
  if (kind_ == Kind::Bool) return b_ ? 1 : 0;
  type_error("a number");
}
double Json::as_f64() const {
  if (kind_ == Kind::Int) return neg_ ? -double(mag_) : double(mag_);
  if (kind_ == Kind::Float) return d_;
  type_error("a number");
}
bool Json::as_bool() const {
  if (kind_ == Kind::Bool) return b_;
  type_error("a bool");
}
const std::string& Json::as_str() const {
  if (kind_ != Kind::String) type_error("a string");
  return *s_;
}
const Json::Array& Json::as_array() const {
  if (kind_ != Kind::Array) type_error("an array");
  return *a_;
}
Json::Array& Json::as_array() {
  if (kind_ != Kind::Array) type_error("an array");
  detach();
  return *a_;
}
const Json::Object& Json::as_object() const {
  if (kind_ != Kind::Object) type_error("an object");
  return *o_;
}
Json::Object& Json::as_object() {
  if (kind_ != Kind::Object) type_error("an object");
  detach();
  return *o_;
}

Json& Json::operator[](const std::string& key) {
  if (kind_ == Kind::Null) {
    kind_ = Kind::Object;
    o_ = std::make_shared<Object>();
  }
  return as_object()[key];
}

const Json* Json::find(const std::string& key) const {
  if (kind_ != Kind::Object) return nullptr;
  auto it = o_->find(key);
  if (it != o_->end()) return &it->second;
  // Go's encoding/json matches field names case-insensitively ("Id" == "ID").
  for (auto& kv : *o_)
    if (kv.first.size() == key.size() && strcasecmp(kv.first.c_str(), key.c_str()) == 0)
      return &kv.second;
  return nullptr;
}
int64_t Json::get_i64(const std::string& key, int64_t dflt) const {
  auto* v = find(key);
  return (v && v->is_number()) ? v->as_i64() : dflt;
}
uint64_t Json::get_u64(const std::string& key, uint64_t dflt) const {
  auto* v = find(key);
  return (v && v->is_number()) ? v->as_u64() : dflt;
}
std::string Json::get_str(const std::string& key, const std::string& dflt) const {
  auto* v = find(key);
  return (v && v->is_string()) ? v->as_str() : dflt;
}
bool Json::get_bool(const std::string& key, bool dflt) const {
  auto* v = find(key);
  return (v && v->kind() == Kind::Bool) ? v->as_bool() : dflt;
}
void Json::push_back(Json v) {
  if (kind_ == Kind::Null) {
    kind_ = Kind::Array;
    a_ = std::make_shared<Array>();
  }
  as_array().push_back(std::move(v));
}

// ---------------------------------------------------------------- serialize
static void dump_string(const std::string& s, std::string& out) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(char(c));
        }
    }
  }
  out.push_back('"');
}

void Json::dump_to(std::string& out) const {
  switch (kind_) {
    case Kind::Null: out += "null"; break;
    case Kind::Bool: out += b_ ? "true" : "false"; break;
    case Kind::Int: {
      char buf[24];
      char* e = buf;
      if (neg_) *e++ = '-';
      e = std::to_chars(e, buf + sizeof buf, mag_).ptr;
      out.append(buf, size_t(e - buf));
      break;
    }
    case Kind::Float: {
      if (!std::isfinite(d_)) { out += "null"; break; }
      char buf[40];
      snprintf(buf, sizeof buf, "%.17g", d_);
      out += buf;
      break;
    }
    case Kind::String: dump_string(*s_, out); break;
    case Kind::Array: {
      out.push_back('[');
      bool first = true;
      for (auto& v : *a_) {
        if (!first) out.push_back(',');
        first = false;
        v.dump_to(out);
      }
      out.push_back(']');
      break;
    }
    case Kind::Object: {
      out.push_back('{');
      bool first = true;
      for (auto& kv : *o_) {
        if (!first) out.push_back(',');
        first = false;
        dump_string(kv.first, out);
        out.push_back(':');
        kv.second.dump_to(out);
      }
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump() const {
  std::string out;
  dump_to(out);
  return out;
}

// -------------------------------------------------------------------- parse
namespace {
struct Parser {
  const char* p;
  const char* end;
  int depth = 0;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json parse error: ") + what);
  }
  void need(size_t n) {
    if (size_t(end - p) < n) throw JsonIncomplete();
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  char peek() {
    need(1);
    return *p;
  }
  void expect_lit(const char* lit) {
    size_t n = strlen(lit);
    for (size_t i = 0; i < n; ++i) {
      need(i + 1);
      if (p[i] != lit[i]) fail("bad literal");
    }
    p += n;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out.push_back(char(cp));
    } else if (cp < 0x800) {
      out.push_back(char(0xC0 | (cp >> 6)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(char(0xE0 | (cp >> 12)));
      out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(char(0xF0 | (cp >> 18)));
      out.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    need(4);
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = p[i];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad \\u escape");
    }
    p += 4;
    return v;
  }
  std::string str() {
    if (peek() != '"') fail("expected string");
    ++p;
    std::string out;
    for (;;) {
      need(1);
      char c = *p++;
      if (c == '"') return out;
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      need(1);
      char e = *p++;
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00) {
            need(2);
            if (p[0] == '\\' && p[1] == 'u') {
              p += 2;
              uint32_t lo = hex4();
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }
  Json number() {
    const char* s = p;
    bool neg = false;
    if (*p == '-') { neg = true; ++p; }
    bool is_float = false;
    // A number at the very end of the buffer may be truncated mid-stream.
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' ||
                       *p == '+' || *p == '-')) {
      if (*p == '.' || *p == 'e' || *p == 'E') is_float = true;
      ++p;
    }
    if (p == end) throw JsonIncomplete();
    const char* digits = s + (neg ? 1 : 0);
    if (digits == p) fail("bad number");
    if (!is_float) {
      // in place: no token copy (control-plane batches carry thousands of integers)
      uint64_t mag = 0;
      auto r = std::from_chars(digits, p, mag);
      if (r.ec == std::errc::result_out_of_range) return Json(strtod(std::string(s, p).c_str(), nullptr));
      if (r.ec != std::errc() || r.ptr != p) fail("bad integer");
      if (neg) {
        if (mag > (1ull << 63)) return Json(-double(mag));
        return Json(int64_t(uint64_t(0) - uint64_t(mag)));
      }
      return Json(mag);
    }
    std::string tok(s, p);
    char* ep = nullptr;
    double d = strtod(tok.c_str(), &ep);
    if (*ep != 0) fail("bad float");
    return Json(d);
  }
  Json value() {
    if (++depth > 256) fail("nesting too deep");
    ws();
    char c = peek();
    Json out;
    if (c == '{') {
      ++p;
      Json::Object obj;
      ws();
      if (peek() == '}') {
        ++p;
      } else {
        for (;;) {
          ws();
          std::string k = str();
          ws();
          if (peek() != ':') fail("expected ':'");
          ++p;
          obj.insert_or_assign(std::move(k), value());
          ws();
          char d = peek();
          ++p;
          if (d == '}') break;
          if (d != ',') fail("expected ',' or '}'");
        }
      }
      out = Json(std::move(obj));
    } else if (c == '[') {
      ++p;
      Json::Array arr;
      ws();
      if (peek() == ']') {
        ++p;
      } else {
        for (;;) {
          arr.push_back(value());
          ws();
          char d = peek();
          ++p;
          if (d == ']') break;
          if (d != ',') fail("expected ',' or ']'");
        }
      }
      out = Json(std::move(arr));
    } else if (c == '"') {
      out = Json(str());
    } else if (c == 't') {
      expect_lit("true");
      out = Json(true);
    } else if (c == 'f') {
      expect_lit("false");
      out = Json(false);
    } else if (c == 'n') {
      expect_lit("null");
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      out = number();
    } else {
      fail("unexpected character");
    }
    --depth;
    return out;
  }
};
}  // namespace

size_t Json::parse_prefix(const char* buf, size_t len, Json& out) {
  Parser ps{buf, buf + len};
  ps.ws();
  if (ps.p == ps.end) return 0;
  try {
    out = ps.value();
  } catch (const JsonIncomplete&) {
    return 0;
  }
  return size_t(ps.p - buf);
}

size_t Json::scan_prefix(const char* buf, size_t len) {
  const char* p = buf;
  const char* end = buf + len;
  auto ws = [&] {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  };
  ws();
  if (p == end) return 0;
  int depth = 0;
  for (;;) {
    if (p == end) return 0;
    const char c = *p;
    if (c == '"') {
      ++p;
      for (;;) {
        if (p == end) return 0;
        if (*p == '\\') {
          if (end - p < 2) return 0;
          p += 2;
          continue;
        }
        if (*p++ == '"') break;
      }
    } else if (c == '{' || c == '[') {
      if (++depth > 256) throw std::runtime_error("json parse error: nesting too deep");
      ++p;
    } else if (c == '}' || c == ']') {
      if (--depth < 0) throw std::runtime_error("json parse error: unbalanced");
      ++p;
    } else if (c == ',' || c == ':' || c == ' ' || c == '\n' || c == '\r' || c == '\t') {
      if (depth == 0) throw std::runtime_error("json parse error: unexpected separator");
      ++p;
    } else {
      // a scalar (number or literal): complete once a delimiter follows it
      while (p < end && *p != ',' && *p != ']' && *p != '}' && *p != ' ' && *p != '\n' && *p != '\r' &&
             *p != '\t' && *p != ':')
        ++p;
      if (p == end) return 0;
    }
    if (depth == 0) return size_t(p - buf);
  }
}

Json Json::parse(const std::string& text) {
  // Terminal numbers are only "complete" once followed by a delimiter, so pad.
  std::string padded = text + " ";
  Parser ps{padded.data(), padded.data() + padded.size()};
  Json out;
  try {
    out = ps.value();
  } catch (const JsonIncomplete&) {
    throw std::runtime_error("json parse error: truncated input");
  }
  ps.ws();
  if (ps.p != ps.end) throw std::runtime_error("json parse error: trailing characters");
  return out;
}

}  // namespace dissem
