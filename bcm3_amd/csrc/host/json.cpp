// json.cpp -- see json.h
#include "json.h"

#include <cctype>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <limits>
#include <sstream>

namespace bcm3 {

const Json* Json::find(const std::string& k) const
{
    if (type != Object) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
}

double Json::as_double() const
{
    if (type == Number) return num;
    if (type == Bool) return b ? 1.0 : 0.0;
    if (type == Null) return std::numeric_limits<double>::quiet_NaN();
    if (type == String) {
        if (str == "NaN" || str == "nan") return std::numeric_limits<double>::quiet_NaN();
        return std::strtod(str.c_str(), nullptr);
    }
    throw JsonError{"value is not a number"};
}

namespace {

struct P {
    const std::string& s;
    size_t i = 0;
    explicit P(const std::string& x) : s(x) {}
    [[noreturn]] void fail(const std::string& m) { throw JsonError{"JSON parse error at " + std::to_string(i) + ": " + m}; }
    void ws()
    {
        while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
    }
    bool lit(const char* w)
    {
        size_t n = std::char_traits<char>::length(w);
        if (s.compare(i, n, w) == 0) {
            i += n;
            return true;
        }
        return false;
    }
    std::string string()
    {
        if (s[i] != '"') fail("expected string");
        i++;
        std::string o;
        while (i < s.size() && s[i] != '"') {
            char c = s[i++];
            if (c == '\\') {
                if (i >= s.size()) fail("bad escape");
                char e = s[i++];
                switch (e) {
                case 'n': o += '\n'; break;
                case 't': o += '\t'; break;
                case 'r': o += '\r'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'u': {
                    unsigned v = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
                    i += 4;
                    if (v < 0x80) o += (char)v;
                    else if (v < 0x800) {
                        o += (char)(0xC0 | (v >> 6));
                        o += (char)(0x80 | (v & 0x3F));
                    } else {
                        o += (char)(0xE0 | (v >> 12));
                        o += (char)(0x80 | ((v >> 6) & 0x3F));
                        o += (char)(0x80 | (v & 0x3F));
                    }
                    break;
                }
                default: o += e;
                }
            } else {
                o += c;
            }
        }
        if (i >= s.size()) fail("unterminated string");
        i++;
        return o;
    }
    Json value()
    {
        ws();
        if (i >= s.size()) fail("unexpected end");
        Json v;
        char c = s[i];
        if (c == '{') {
            i++;
            v.type = Json::Object;
            ws();
            if (s[i] == '}') {
                i++;
                return v;
            }
            for (;;) {
                ws();
                std::string k = string();
                ws();
                if (s[i] != ':') fail("expected ':'");
                i++;
                v.obj[k] = value();
                ws();
                if (s[i] == ',') {
                    i++;
                    continue;
                }
                if (s[i] == '}') {
                    i++;
                    return v;
                }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            i++;
            v.type = Json::Array;
            ws();
            if (s[i] == ']') {
                i++;
                return v;
            }
            for (;;) {
                v.arr.push_back(value());
                ws();
                if (s[i] == ',') {
                    i++;
                    continue;
                }
                if (s[i] == ']') {
                    i++;
                    return v;
                }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.type = Json::String;
            v.str = string();
            return v;
        }
        if (lit("null")) return v;
        if (lit("true")) {
            v.type = Json::Bool;
            v.b = true;
            return v;
        }
        if (lit("false")) {
            v.type = Json::Bool;
            return v;
        }
        if (lit("NaN")) {
            v.type = Json::Number;
            v.num = std::numeric_limits<double>::quiet_NaN();
            return v;
        }
        if (lit("Infinity")) {
            v.type = Json::Number;
            v.num = std::numeric_limits<double>::infinity();
            return v;
        }
        if (lit("-Infinity")) {
            v.type = Json::Number;
            v.num = -std::numeric_limits<double>::infinity();
            return v;
        }
        char* e = nullptr;
        v.num = std::strtod(s.c_str() + i, &e);
        if (e == s.c_str() + i) fail("unexpected character");
        i = (size_t)(e - s.c_str());
        v.type = Json::Number;
        return v;
    }
};

}  // namespace

Json json_parse(const std::string& text)
{
    P p(text);
    Json v = p.value();
    p.ws();
    if (p.i != text.size()) p.fail("trailing characters");
    return v;
}

Json json_load(const std::string& filename)
{
    std::ifstream f(filename);
    if (!f) throw JsonError{"cannot open " + filename};
    std::stringstream ss;
    ss << f.rdbuf();
    return json_parse(ss.str());
}

namespace {
void dump_to(const Json& j, std::string& o)
{
    switch (j.type) {
    case Json::Null: o += "null"; break;
    case Json::Bool: o += j.b ? "true" : "false"; break;
    case Json::Number:
        if (!std::isfinite(j.num)) {
            o += "null";
        } else {
            char buf[32];
            snprintf(buf, sizeof buf, "%.17g", j.num);
            o += buf;
        }
        break;
    case Json::String:
        o += '"';
        for (char c : j.str) {
            if (c == '"' || c == '\\') {
                o += '\\';
                o += c;
            } else if ((unsigned char)c < 0x20) {
                char buf[8];
                snprintf(buf, sizeof buf, "\\u%04x", (unsigned char)c);
                o += buf;
            } else {
                o += c;
            }
        }
        o += '"';
        break;
    case Json::Array:
        o += '[';
        for (size_t i = 0; i < j.arr.size(); i++) {
            if (i) o += ',';
            dump_to(j.arr[i], o);
        }
        o += ']';
        break;
    case Json::Object: {
        o += '{';
        bool first = true;
        for (auto& kv : j.obj) {
            if (!first) o += ',';
            first = false;
            Json k;
            k.type = Json::String;
            k.str = kv.first;
            dump_to(k, o);
            o += ':';
            dump_to(kv.second, o);
        }
        o += '}';
        break;
    }
    }
}
}  // namespace

std::string json_dump(const Json& j)
{
    std::string o;
    dump_to(j, o);
    return o;
}

}  // namespace bcm3
