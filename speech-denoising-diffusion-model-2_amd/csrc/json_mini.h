// Minimal JSON reader for the config blocks handed to sddm_configure (config_unet.json etc.).
// Supports objects, arrays, numbers, strings (basic escapes), true/false/null.
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>
#include <cstdlib>

namespace sddm {

struct Json {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;

  bool has(const std::string& k) const { return kind == OBJ && obj.count(k); }
  const Json& at(const std::string& k) const {
    static const Json null_json;
    auto it = obj.find(k);
    return (kind == OBJ && it != obj.end()) ? it->second : null_json;
  }
  double number(const std::string& k, double dflt) const {
    const Json& v = at(k);
    if (v.kind == NUM) return v.num;
    if (v.kind == BOOL) return v.b ? 1.0 : 0.0;
    return dflt;
  }
  std::string string(const std::string& k, const std::string& dflt) const {
    const Json& v = at(k);
    return v.kind == STR ? v.str : dflt;
  }
  std::vector<int> ints(const std::string& k, std::vector<int> dflt) const {
    const Json& v = at(k);
    if (v.kind != ARR) return dflt;
    std::vector<int> r;
    for (const auto& e : v.arr) r.push_back((int)e.num);
    return r;
  }

  static Json parse(const std::string& s) {
    size_t i = 0;
    Json j = parse_value(s, i);
    skip(s, i);
    if (i != s.size()) throw std::runtime_error("trailing characters in JSON");
    return j;
  }

 private:
  static void skip(const std::string& s, size_t& i) {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
  }
  static Json parse_value(const std::string& s, size_t& i) {
    skip(s, i);
    if (i >= s.size()) throw std::runtime_error("unexpected end of JSON");
    Json j;
    const char c = s[i];
    if (c == '{') {
      j.kind = OBJ;
      ++i;
      skip(s, i);
      if (i < s.size() && s[i] == '}') { ++i; return j; }
      while (true) {
        skip(s, i);
        Json key = parse_value(s, i);
        if (key.kind != STR) throw std::runtime_error("JSON object key must be a string");
        skip(s, i);
        if (i >= s.size() || s[i] != ':') throw std::runtime_error("expected ':' in JSON");
        ++i;
        j.obj[key.str] = parse_value(s, i);
        skip(s, i);
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; break; }
        throw std::runtime_error("expected ',' or '}' in JSON");
      }
    } else if (c == '[') {
      j.kind = ARR;
      ++i;
      skip(s, i);
      if (i < s.size() && s[i] == ']') { ++i; return j; }
      while (true) {
        j.arr.push_back(parse_value(s, i));
        skip(s, i);
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; break; }
        throw std::runtime_error("expected ',' or ']' in JSON");
      }
    } else if (c == '"') {
      j.kind = STR;
      ++i;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\' && i + 1 < s.size()) {
          const char e = s[i + 1];
          j.str += (e == 'n') ? '\n' : (e == 't') ? '\t' : e;
          i += 2;
        } else {
          j.str += s[i++];
        }
      }
      if (i >= s.size()) throw std::runtime_error("unterminated JSON string");
      ++i;
    } else if (s.compare(i, 4, "true") == 0) {
      j.kind = BOOL; j.b = true; i += 4;
    } else if (s.compare(i, 5, "false") == 0) {
      j.kind = BOOL; j.b = false; i += 5;
    } else if (s.compare(i, 4, "null") == 0) {
      j.kind = NUL; i += 4;
    } else {
      char* end = nullptr;
      j.kind = NUM;
      j.num = std::strtod(s.c_str() + i, &end);
      if (end == s.c_str() + i) throw std::runtime_error("bad JSON value");
      i = (size_t)(end - s.c_str());
    }
    return j;
  }
};

}  // namespace sddm
