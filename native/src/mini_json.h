// mini_json.h — small recursive-descent JSON reader used by the mock amdsmi library.
// Header-only; supports objects, arrays, strings (with \" \\ \n \t \uXXXX→'?'), numbers,
// true/false/null. Enough for test fixtures; not a general-purpose parser.
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace gmjson {

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0;
  std::string str;
  std::vector<Value> arr;
  std::map<std::string, Value> obj;

  const Value* get(const std::string& k) const {
    if (kind != Object) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
  }
  double num_or(const std::string& k, double d) const {
    const Value* v = get(k);
    return (v && v->kind == Number) ? v->num : d;
  }
  std::string str_or(const std::string& k, const std::string& d) const {
    const Value* v = get(k);
    return (v && v->kind == String) ? v->str : d;
  }
};

class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}
  bool parse(Value& out) {
    ws();
    if (!value(out)) return false;
    ws();
    return i_ == s_.size();
  }

 private:
  const std::string& s_;
  size_t i_ = 0;

  void ws() {
    while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r'))
      ++i_;
  }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) ++n;
    if (s_.compare(i_, n, w) != 0) return false;
    i_ += n;
    return true;
  }
  bool value(Value& v) {
    if (i_ >= s_.size()) return false;
    char c = s_[i_];
    if (c == '{') return object(v);
    if (c == '[') return array(v);
    if (c == '"') {
      v.kind = Value::String;
      return string(v.str);
    }
    if (c == 't') {
      v.kind = Value::Bool;
      v.b = true;
      return lit("true");
    }
    if (c == 'f') {
      v.kind = Value::Bool;
      v.b = false;
      return lit("false");
    }
    if (c == 'n') {
      v.kind = Value::Null;
      return lit("null");
    }
    return number(v);
  }
  bool number(Value& v) {
    const char* start = s_.c_str() + i_;
    char* end = nullptr;
    // accept hex integers too (0x950) — handy for gfx versions in fixtures
    if (s_.compare(i_, 2, "0x") == 0)
      v.num = (double)strtoull(start, &end, 16);
    else
      v.num = strtod(start, &end);
    if (end == start) return false;
    i_ += (size_t)(end - start);
    v.kind = Value::Number;
    return true;
  }
  bool string(std::string& out) {
    if (s_[i_] != '"') return false;
    ++i_;
    out.clear();
    while (i_ < s_.size()) {
      char c = s_[i_++];
      if (c == '"') return true;
      if (c == '\\') {
        if (i_ >= s_.size()) return false;
        char e = s_[i_++];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'u':
            if (i_ + 4 > s_.size()) return false;
            i_ += 4;
            out.push_back('?');
            break;
          default: out.push_back(e);
        }
      } else {
        out.push_back(c);
      }
    }
    return false;
  }
  bool array(Value& v) {
    v.kind = Value::Array;
    ++i_;
    ws();
    if (i_ < s_.size() && s_[i_] == ']') {
      ++i_;
      return true;
    }
    while (true) {
      Value e;
      ws();
      if (!value(e)) return false;
      v.arr.push_back(std::move(e));
      ws();
      if (i_ >= s_.size()) return false;
      if (s_[i_] == ',') {
        ++i_;
        continue;
      }
      if (s_[i_] == ']') {
        ++i_;
        return true;
      }
      return false;
    }
  }
  bool object(Value& v) {
    v.kind = Value::Object;
    ++i_;
    ws();
    if (i_ < s_.size() && s_[i_] == '}') {
      ++i_;
      return true;
    }
    while (true) {
      ws();
      std::string k;
      if (i_ >= s_.size() || !string(k)) return false;
      ws();
      if (i_ >= s_.size() || s_[i_] != ':') return false;
      ++i_;
      ws();
      Value e;
      if (!value(e)) return false;
      v.obj[k] = std::move(e);
      ws();
      if (i_ >= s_.size()) return false;
      if (s_[i_] == ',') {
        ++i_;
        continue;
      }
      if (s_[i_] == '}') {
        ++i_;
        return true;
      }
      return false;
    }
  }
};

inline bool parse(const std::string& text, Value& out) {
  Parser p(text);
  return p.parse(out);
}

}  // namespace gmjson
