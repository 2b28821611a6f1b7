// json.hpp — minimal JSON value + parser for scene files (the reference links jsoncpp,
// Graphics.h:3 / GUI.h:120-149; it is not available here, and only this subset is needed).
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rmr {
namespace json {

struct Value {
    enum Kind { Null, Bool, Int, Real, String, Array, Object } kind = Null;
    bool b = false;
    long long i = 0;
    double d = 0.0;
    std::string s;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;  // insertion order kept

    bool is_null() const { return kind == Null; }
    bool is_int() const { return kind == Int; }
    bool is_number() const { return kind == Int || kind == Real; }
    bool is_string() const { return kind == String; }
    bool is_array() const { return kind == Array; }
    bool is_object() const { return kind == Object; }
    double as_double() const { return kind == Int ? (double)i : (kind == Real ? d : 0.0); }
    size_t size() const { return kind == Array ? arr.size() : (kind == Object ? obj.size() : 0); }
    const Value& operator[](size_t k) const {
        static const Value null;
        return (kind == Array && k < arr.size()) ? arr[k] : null;
    }
    const Value& get(const std::string& key) const {
        static const Value null;
        if (kind != Object) return null;
        for (const auto& kv : obj)
            if (kv.first == key) return kv.second;
        return null;
    }
    bool has(const std::string& key) const { return !get(key).is_null(); }
};

class Parser {
public:
    explicit Parser(const std::string& t) : s_(t), p_(0) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t p_;
    [[noreturn]] void fail(const char* m) {
        throw std::runtime_error(std::string("JSON parse error at offset ") + std::to_string(p_) + ": " + m);
    }
    void ws() {
        while (p_ < s_.size()) {
            char c = s_[p_];
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') { p_++; continue; }
            if (c == '/' && p_ + 1 < s_.size() && s_[p_ + 1] == '/') {  // jsoncpp allows comments
                while (p_ < s_.size() && s_[p_] != '\n') p_++;
                continue;
            }
            if (c == '/' && p_ + 1 < s_.size() && s_[p_ + 1] == '*') {
                size_t e = s_.find("*/", p_ + 2);
                if (e == std::string::npos) fail("unterminated comment");
                p_ = e + 2;
                continue;
            }
            break;
        }
    }
    Value value() {
        ws();
        if (p_ >= s_.size()) fail("unexpected end");
        char c = s_[p_];
        if (c == '{') return object();
        if (c == '[') return array();
        if (c == '"') { Value v; v.kind = Value::String; v.s = str(); return v; }
        if (s_.compare(p_, 4, "true") == 0) { p_ += 4; Value v; v.kind = Value::Bool; v.b = true; return v; }
        if (s_.compare(p_, 5, "false") == 0) { p_ += 5; Value v; v.kind = Value::Bool; return v; }
        if (s_.compare(p_, 4, "null") == 0) { p_ += 4; return Value(); }
        return number();
    }
    Value object() {
        Value v;
        v.kind = Value::Object;
        p_++;
        ws();
        if (p_ < s_.size() && s_[p_] == '}') { p_++; return v; }
        for (;;) {
            ws();
            if (p_ >= s_.size() || s_[p_] != '"') fail("expected key");
            std::string k = str();
            ws();
            if (p_ >= s_.size() || s_[p_] != ':') fail("expected ':'");
            p_++;
            Value x = value();
            v.obj.emplace_back(k, std::move(x));
            ws();
            if (p_ < s_.size() && s_[p_] == ',') { p_++; ws(); if (p_ < s_.size() && s_[p_] == '}') { p_++; return v; } continue; }
            if (p_ < s_.size() && s_[p_] == '}') { p_++; return v; }
            fail("expected ',' or '}'");
        }
    }
    Value array() {
        Value v;
        v.kind = Value::Array;
        p_++;
        ws();
        if (p_ < s_.size() && s_[p_] == ']') { p_++; return v; }
        for (;;) {
            v.arr.push_back(value());
            ws();
            if (p_ < s_.size() && s_[p_] == ',') { p_++; ws(); if (p_ < s_.size() && s_[p_] == ']') { p_++; return v; } continue; }
            if (p_ < s_.size() && s_[p_] == ']') { p_++; return v; }
            fail("expected ',' or ']'");
        }
    }
    std::string str() {
        std::string r;
        p_++;
        while (p_ < s_.size() && s_[p_] != '"') {
            char c = s_[p_++];
            if (c == '\\') {
                if (p_ >= s_.size()) fail("bad escape");
                char e = s_[p_++];
                switch (e) {
                case 'n': r += '\n'; break;
                case 't': r += '\t'; break;
                case 'r': r += '\r'; break;
                case 'b': r += '\b'; break;
                case 'f': r += '\f'; break;
                case 'u': {
                    if (p_ + 4 > s_.size()) fail("bad \\u");
                    unsigned cp = (unsigned)std::strtoul(s_.substr(p_, 4).c_str(), nullptr, 16);
                    p_ += 4;
                    if (cp < 0x80) r += (char)cp;
                    else if (cp < 0x800) { r += (char)(0xC0 | (cp >> 6)); r += (char)(0x80 | (cp & 0x3F)); }
                    else { r += (char)(0xE0 | (cp >> 12)); r += (char)(0x80 | ((cp >> 6) & 0x3F)); r += (char)(0x80 | (cp & 0x3F)); }
                    break;
                }
                default: r += e; break;
                }
            } else {
                r += c;
            }
        }
        if (p_ >= s_.size()) fail("unterminated string");
        p_++;
        return r;
    }
    Value number() {
        size_t st = p_;
        if (p_ < s_.size() && (s_[p_] == '-' || s_[p_] == '+')) p_++;
        bool real = false;
        while (p_ < s_.size()) {
            char c = s_[p_];
            if (c >= '0' && c <= '9') { p_++; continue; }
            if (c == '.' || c == 'e' || c == 'E' || ((c == '-' || c == '+') && (s_[p_ - 1] == 'e' || s_[p_ - 1] == 'E'))) {
                real = true; p_++; continue;
            }
            break;
        }
        if (st == p_) fail("unexpected character");
        std::string t = s_.substr(st, p_ - st);
        Value v;
        if (!real) {
            v.kind = Value::Int;
            v.i = std::strtoll(t.c_str(), nullptr, 10);
        } else {
            v.kind = Value::Real;
            v.d = std::strtod(t.c_str(), nullptr);
        }
        return v;
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace json
}  // namespace rmr
