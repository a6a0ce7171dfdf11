// Minimal JSON reader with the value semantics nart's scene loader relies on
// (nlohmann::json 3.11.3 as used in src/core/scene.cpp and src/core/render.cpp:327-414):
//  * numbers keep their integer/float kind; floats are parsed with strtod (double) and
//    narrowed by the caller (nlohmann get<float>() = static_cast<float>(double));
//  * integers are parsed as int64/uint64 and cast by get<T>();
//  * object key lookup of a missing key yields null (nlohmann operator[] inserts null).
#pragma once

#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace nartjson {

struct Value {
    enum Kind { Null, Bool, Int, Uint, Float, String, Array, Object } kind = Null;
    bool b = false;
    int64_t i = 0;
    uint64_t u = 0;
    double d = 0.0;
    std::string s;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;  // nlohmann default object_t is std::map

    bool is_null() const { return kind == Null; }
    bool is_object() const { return kind == Object; }
    bool is_array() const { return kind == Array; }
    bool is_number() const { return kind == Int || kind == Uint || kind == Float; }
    bool is_string() const { return kind == String; }
    bool contains(const std::string& k) const { return kind == Object && obj.count(k) != 0; }

    const Value& operator[](const std::string& k) const {
        static const Value null_value;
        if (kind != Object) return null_value;
        auto it = obj.find(k);
        return it == obj.end() ? null_value : it->second;
    }
    size_t size() const {
        if (kind == Array) return arr.size();
        if (kind == Object) return obj.size();
        if (kind == Null) return 0;
        return 1;
    }

    // nlohmann get<float>() / get<uint32_t>() etc: static_cast from the stored kind.
    template <typename T>
    T num() const {
        switch (kind) {
            case Int: return static_cast<T>(i);
            case Uint: return static_cast<T>(u);
            case Float: return static_cast<T>(d);
            case Bool: return static_cast<T>(b);
            default: throw std::runtime_error("type_error: value is not a number");
        }
    }
    std::string str() const {
        if (kind != String) throw std::runtime_error("type_error: value is not a string");
        return s;
    }
    std::vector<float> floats() const {
        if (kind != Array) throw std::runtime_error("type_error: value is not an array");
        std::vector<float> v;
        for (const Value& e : arr) v.push_back(e.num<float>());
        return v;
    }
};

class Parser {
public:
    explicit Parser(const std::string& text) : t_(text), p_(0) {}
    Value parse() {
        Value v = value();
        ws();
        if (p_ != t_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& t_;
    size_t p_;

    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("parse_error at byte ") + std::to_string(p_) + ": " + what);
    }
    void ws() {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t' || t_[p_] == '\n' || t_[p_] == '\r')) ++p_;
    }
    bool lit(const char* s) {
        size_t n = std::strlen(s);
        if (t_.compare(p_, n, s) == 0) {
            p_ += n;
            return true;
        }
        return false;
    }
    Value value() {
        ws();
        if (p_ >= t_.size()) fail("unexpected end");
        char c = t_[p_];
        Value v;
        if (c == '{') {
            ++p_;
            v.kind = Value::Object;
            ws();
            if (p_ < t_.size() && t_[p_] == '}') {
                ++p_;
                return v;
            }
            for (;;) {
                ws();
                if (p_ >= t_.size() || t_[p_] != '"') fail("expected key");
                std::string k = string();
                ws();
                if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
                ++p_;
                v.obj[k] = value();  // duplicate keys: last wins (std::map assignment)
                ws();
                if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
                if (p_ < t_.size() && t_[p_] == '}') { ++p_; break; }
                fail("expected ',' or '}'");
            }
            return v;
        }
        if (c == '[') {
            ++p_;
            v.kind = Value::Array;
            ws();
            if (p_ < t_.size() && t_[p_] == ']') {
                ++p_;
                return v;
            }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
                if (p_ < t_.size() && t_[p_] == ']') { ++p_; break; }
                fail("expected ',' or ']'");
            }
            return v;
        }
        if (c == '"') {
            v.kind = Value::String;
            v.s = string();
            return v;
        }
        if (lit("true")) { v.kind = Value::Bool; v.b = true; return v; }
        if (lit("false")) { v.kind = Value::Bool; v.b = false; return v; }
        if (lit("null")) return v;
        return number();
    }
    std::string string() {
        ++p_;  // opening quote
        std::string out;
        while (p_ < t_.size() && t_[p_] != '"') {
            char c = t_[p_++];
            if (c == '\\') {
                if (p_ >= t_.size()) fail("bad escape");
                char e = t_[p_++];
                switch (e) {
                    case '"': out += '"'; break;
                    case '\\': out += '\\'; break;
                    case '/': out += '/'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 't': out += '\t'; break;
                    case 'u': {
                        if (p_ + 4 > t_.size()) fail("bad \\u escape");
                        unsigned cp = std::strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
                        p_ += 4;
                        if (cp < 0x80) out += char(cp);
                        else if (cp < 0x800) { out += char(0xC0 | (cp >> 6)); out += char(0x80 | (cp & 0x3F)); }
                        else { out += char(0xE0 | (cp >> 12)); out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: fail("bad escape");
                }
            } else {
                out += c;
            }
        }
        if (p_ >= t_.size()) fail("unterminated string");
        ++p_;
        return out;
    }
    Value number() {
        size_t start = p_;
        bool is_float = false;
        if (t_[p_] == '-') ++p_;
        if (p_ >= t_.size() || !(t_[p_] >= '0' && t_[p_] <= '9')) fail("invalid literal");
        while (p_ < t_.size() && t_[p_] >= '0' && t_[p_] <= '9') ++p_;
        if (p_ < t_.size() && t_[p_] == '.') {
            is_float = true;
            ++p_;
            while (p_ < t_.size() && t_[p_] >= '0' && t_[p_] <= '9') ++p_;
        }
        if (p_ < t_.size() && (t_[p_] == 'e' || t_[p_] == 'E')) {
            is_float = true;
            ++p_;
            if (p_ < t_.size() && (t_[p_] == '+' || t_[p_] == '-')) ++p_;
            while (p_ < t_.size() && t_[p_] >= '0' && t_[p_] <= '9') ++p_;
        }
        std::string tok = t_.substr(start, p_ - start);
        Value v;
        if (!is_float) {
            errno = 0;
            if (tok[0] == '-') {
                long long x = std::strtoll(tok.c_str(), nullptr, 10);
                if (errno == 0) { v.kind = Value::Int; v.i = x; return v; }
            } else {
                unsigned long long x = std::strtoull(tok.c_str(), nullptr, 10);
                if (errno == 0) { v.kind = Value::Uint; v.u = x; return v; }
            }
        }
        v.kind = Value::Float;
        v.d = std::strtod(tok.c_str(), nullptr);
        return v;
    }
};

}  // namespace nartjson
