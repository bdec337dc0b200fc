#include "json.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

namespace cake {

bool Json::has(const std::string& k) const {
  return type_ == Object && index_.count(k) != 0;
}

const Json& Json::get(const std::string& k) const {
  check(Object);
  auto it = index_.find(k);
  if (it == index_.end()) throw std::runtime_error("json: missing key '" + k + "'");
  return obj_[it->second].second;
}

void Json::set(const std::string& k, Json v) {
  check(Object);
  auto it = index_.find(k);
  if (it != index_.end()) {
    obj_[it->second].second = std::move(v);
  } else {
    index_[k] = obj_.size();
    obj_.emplace_back(k, std::move(v));
  }
}

namespace {

struct Parser {
  const char* p;
  const char* end;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json parse error: ") + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if ((size_t)(end - p) >= n && std::memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static void utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F));
      o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (end - p < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string str() {
    if (p >= end || *p != '"') fail("expected string");
    ++p;
    std::string o;
    while (true) {
      if (p >= end) fail("unterminated string");
      char c = *p++;
      if (c == '"') break;
      if (c != '\\') { o += c; continue; }
      if (p >= end) fail("bad escape");
      char e = *p++;
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(o, cp);
          break;
        }
        default: fail("unknown escape");
      }
    }
    return o;
  }
  Json num() {
    const char* s = p;
    bool integral = true;
    if (p < end && (*p == '-' || *p == '+')) ++p;
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' ||
                       *p == '-' || *p == '+')) {
      if (*p == '.' || *p == 'e' || *p == 'E') integral = false;
      ++p;
    }
    std::string t(s, p);
    if (t.empty()) fail("expected number");
    if (integral) {
      errno = 0;
      long long v = std::strtoll(t.c_str(), nullptr, 10);
      if (errno == 0) return Json::integer(v);
    }
    return Json::number(std::strtod(t.c_str(), nullptr));
  }
  Json value(int depth) {
    if (depth > 256) fail("nesting too deep");
    ws();
    if (p >= end) fail("unexpected end");
    char c = *p;
    if (c == '{') {
      ++p;
      Json o = Json::object();
      ws();
      if (p < end && *p == '}') { ++p; return o; }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (p >= end || *p != ':') fail("expected ':'");
        ++p;
        o.set(k, value(depth + 1));
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '}') { ++p; break; }
        fail("expected ',' or '}'");
      }
      return o;
    }
    if (c == '[') {
      ++p;
      Json a = Json::array();
      ws();
      if (p < end && *p == ']') { ++p; return a; }
      while (true) {
        a.push(value(depth + 1));
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == ']') { ++p; break; }
        fail("expected ',' or ']'");
      }
      return a;
    }
    if (c == '"') return Json::string(str());
    if (lit("true")) return Json::boolean(true);
    if (lit("false")) return Json::boolean(false);
    if (lit("null")) return Json();
    return num();
  }
};

void escape(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          out += b;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

}  // namespace

Json Json::parse(const std::string& text) {
  Parser ps{text.data(), text.data() + text.size()};
  Json v = ps.value(0);
  ps.ws();
  if (ps.p != ps.end) ps.fail("trailing characters");
  return v;
}

void Json::dump_to(std::string& out, int indent, int depth) const {
  auto nl = [&](int d) {
    if (indent < 0) return;
    out += '\n';
    out.append((size_t)(indent * d), ' ');
  };
  switch (type_) {
    case Null: out += "null"; break;
    case Bool: out += b_ ? "true" : "false"; break;
    case Number: {
      if (is_int_) {
        out += std::to_string(i_);
      } else if (std::isfinite(d_) && d_ == std::floor(d_) && std::fabs(d_) < 9e15) {
        out += std::to_string((long long)d_);
      } else {
        char b[32];
        std::snprintf(b, sizeof b, "%.17g", d_);
        out += b;
      }
      break;
    }
    case String: escape(out, s_); break;
    case Array: {
      out += '[';
      for (size_t i = 0; i < arr_.size(); ++i) {
        if (i) out += ',';
        nl(depth + 1);
        arr_[i].dump_to(out, indent, depth + 1);
      }
      if (!arr_.empty()) nl(depth);
      out += ']';
      break;
    }
    case Object: {
      out += '{';
      for (size_t i = 0; i < obj_.size(); ++i) {
        if (i) out += ',';
        nl(depth + 1);
        escape(out, obj_[i].first);
        out += indent >= 0 ? ": " : ":";
        obj_[i].second.dump_to(out, indent, depth + 1);
      }
      if (!obj_.empty()) nl(depth);
      out += '}';
      break;
    }
  }
}

std::string Json::dump(int indent) const {
  std::string out;
  dump_to(out, indent, 0);
  return out;
}

}  // namespace cake
