// json.h — a small JSON DOM (objects keep their members in document order, a duplicated key reads
// as its last value, like Python's json.load) shared by the dataset reader (dataset.cpp) and the
// model-description lowering (plan_json.cpp).
#pragma once
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ign {
namespace json {

struct JVal {
  enum Type { Null, Bool, Num, Str, Arr, Obj } t = Null;
  double num = 0;
  std::string str;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;   // document order
  const JVal* get(const std::string& k) const {
    const JVal* r = nullptr;
    for (auto& kv : obj)
      if (kv.first == k) r = &kv.second;    // a duplicated key keeps the last value, as json.load
    return r;
  }
};

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Parser {
 public:
  // what: the document's name in error messages
  Parser(const char* b, const char* e, const char* what = "data.json") : p_(b), e_(e), what_(what) {}
  JVal parse() {
    JVal v = value();
    ws();
    if (p_ != e_) throw JsonError(std::string("trailing characters in ") + what_);
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  const char* what_;
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  [[noreturn]] void bad(const char* what) { throw JsonError(std::string("malformed ") + what_ + ": " + what); }
  JVal value() {
    ws();
    if (p_ >= e_) bad("unexpected end");
    JVal v;
    switch (*p_) {
      case '{': {
        v.t = JVal::Obj;
        ++p_;
        ws();
        if (p_ < e_ && *p_ == '}') { ++p_; return v; }
        for (;;) {
          ws();
          if (p_ >= e_ || *p_ != '"') bad("expected a key");
          std::string k = string();
          ws();
          if (p_ >= e_ || *p_ != ':') bad("expected ':'");
          ++p_;
          v.obj.emplace_back(std::move(k), value());
          ws();
          if (p_ < e_ && *p_ == ',') { ++p_; continue; }
          if (p_ < e_ && *p_ == '}') { ++p_; return v; }
          bad("expected ',' or '}'");
        }
      }
      case '[': {
        v.t = JVal::Arr;
        ++p_;
        ws();
        if (p_ < e_ && *p_ == ']') { ++p_; return v; }
        for (;;) {
          v.arr.push_back(value());
          ws();
          if (p_ < e_ && *p_ == ',') { ++p_; continue; }
          if (p_ < e_ && *p_ == ']') { ++p_; return v; }
          bad("expected ',' or ']'");
        }
      }
      case '"':
        v.t = JVal::Str;
        v.str = string();
        return v;
      case 't':
        if (e_ - p_ >= 4 && !strncmp(p_, "true", 4)) { p_ += 4; v.t = JVal::Bool; v.num = 1; return v; }
        bad("literal");
      case 'f':
        if (e_ - p_ >= 5 && !strncmp(p_, "false", 5)) { p_ += 5; v.t = JVal::Bool; v.num = 0; return v; }
        bad("literal");
      case 'n':
        if (e_ - p_ >= 4 && !strncmp(p_, "null", 4)) { p_ += 4; return v; }
        bad("literal");
      default: {
        char* q = nullptr;
        v.num = strtod(p_, &q);
        if (q == p_) bad("number");
        if (q > e_) bad("number past the end");
        p_ = q;
        v.t = JVal::Num;
        return v;
      }
    }
  }
  static void utf8(std::string& s, unsigned cp) {
    if (cp < 0x80) s += (char)cp;
    else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
    } else {
      s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 0x3F));
      s += (char)(0x80 | ((cp >> 6) & 0x3F)); s += (char)(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4() {
    if (e_ - p_ < 4) bad("\\u escape");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else bad("\\u escape");
    }
    return v;
  }
  std::string string() {
    ++p_;   // opening quote
    std::string s;
    while (p_ < e_ && *p_ != '"') {
      if (*p_ != '\\') { s += *p_++; continue; }
      ++p_;
      if (p_ >= e_) bad("escape");
      char c = *p_++;
      switch (c) {
        case '"': s += '"'; break;
        case '\\': s += '\\'; break;
        case '/': s += '/'; break;
        case 'b': s += '\b'; break;
        case 'f': s += '\f'; break;
        case 'n': s += '\n'; break;
        case 'r': s += '\r'; break;
        case 't': s += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(s, cp);
          break;
        }
        default: bad("escape");
      }
    }
    if (p_ >= e_) bad("unterminated string");
    ++p_;
    return s;
  }
};

}  // namespace json
}  // namespace ign
