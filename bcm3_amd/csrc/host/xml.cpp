// xml.cpp -- see xml.h
#include "xml.h"

#include <cctype>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace bcm3 {

const XmlNode* XmlNode::child(const std::string& n) const
{
    for (auto& c : children)
        if (c->name == n) return c.get();
    return nullptr;
}

std::vector<const XmlNode*> XmlNode::children_named(const std::string& n) const
{
    std::vector<const XmlNode*> out;
    for (auto& c : children)
        if (c->name == n) out.push_back(c.get());
    return out;
}

const std::string& XmlNode::get(const std::string& k) const
{
    auto it = attr.find(k);
    if (it == attr.end()) throw XmlError{"No such node (<xmlattr>." + k + ") in <" + name + ">"};
    return it->second;
}

static bool parse_double_strict(const std::string& s, double& v)
{
    // Boost's lexical conversion: the whole string (modulo surrounding spaces) must be a number
    const char* b = s.c_str();
    while (*b && std::isspace((unsigned char)*b)) b++;
    if (!*b) return false;
    char* e = nullptr;
    v = std::strtod(b, &e);
    if (e == b) return false;
    while (*e && std::isspace((unsigned char)*e)) e++;
    return *e == 0;
}

double XmlNode::get_double(const std::string& k, double def) const
{
    auto it = attr.find(k);
    if (it == attr.end()) return def;
    double v;
    return parse_double_strict(it->second, v) ? v : def;
}

double XmlNode::get_double(const std::string& k) const
{
    double v;
    if (!parse_double_strict(get(k), v)) throw XmlError{"conversion of data to type \"double\" failed: " + k};
    return v;
}

long XmlNode::get_long(const std::string& k, long def) const
{
    auto it = attr.find(k);
    if (it == attr.end()) return def;
    char* e = nullptr;
    long v = std::strtol(it->second.c_str(), &e, 10);
    return (e && *e == 0 && !it->second.empty()) ? v : def;
}

bool XmlNode::get_bool(const std::string& k, bool def) const
{
    auto it = attr.find(k);
    if (it == attr.end()) return def;
    const std::string& s = it->second;
    if (s == "true" || s == "1") return true;
    if (s == "false" || s == "0") return false;
    return def;
}

namespace {

struct Parser {
    const std::string& s;
    size_t i = 0;
    explicit Parser(const std::string& src) : s(src) {}

    [[noreturn]] void fail(const std::string& m) { throw XmlError{"XML parse error at offset " + std::to_string(i) + ": " + m}; }
    bool starts(const char* p) const { return s.compare(i, std::char_traits<char>::length(p), p) == 0; }
    void skip_ws()
    {
        while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
    }
    void skip_until(const char* end)
    {
        size_t p = s.find(end, i);
        if (p == std::string::npos) fail(std::string("unterminated, expected ") + end);
        i = p + std::char_traits<char>::length(end);
    }
    std::string name()
    {
        size_t b = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == ':' ||
                                s[i] == '.'))
            i++;
        if (b == i) fail("expected a name");
        return s.substr(b, i - b);
    }
    static std::string unescape(const std::string& v)
    {
        std::string o;
        for (size_t k = 0; k < v.size(); k++) {
            if (v[k] == '&') {
                size_t e = v.find(';', k);
                if (e != std::string::npos) {
                    std::string ent = v.substr(k + 1, e - k - 1);
                    if (ent == "lt") o += '<';
                    else if (ent == "gt") o += '>';
                    else if (ent == "amp") o += '&';
                    else if (ent == "quot") o += '"';
                    else if (ent == "apos") o += '\'';
                    else o += v.substr(k, e - k + 1);
                    k = e;
                    continue;
                }
            }
            o += v[k];
        }
        return o;
    }
    void misc()
    {
        for (;;) {
            skip_ws();
            if (starts("<?")) skip_until("?>");
            else if (starts("<!--")) skip_until("-->");
            else if (starts("<!")) skip_until(">");
            else break;
        }
    }
    std::unique_ptr<XmlNode> element()
    {
        if (i >= s.size() || s[i] != '<') fail("expected '<'");
        i++;
        auto n = std::make_unique<XmlNode>();
        n->name = name();
        for (;;) {
            skip_ws();
            if (starts("/>")) {
                i += 2;
                return n;
            }
            if (i < s.size() && s[i] == '>') {
                i++;
                break;
            }
            std::string k = name();
            skip_ws();
            if (i >= s.size() || s[i] != '=') fail("expected '='");
            i++;
            skip_ws();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) fail("expected quote");
            char q = s[i++];
            size_t e = s.find(q, i);
            if (e == std::string::npos) fail("unterminated attribute");
            n->attr[k] = unescape(s.substr(i, e - i));
            i = e + 1;
        }
        for (;;) {
            size_t b = i;
            while (i < s.size() && s[i] != '<') i++;
            n->text += unescape(s.substr(b, i - b));
            if (i >= s.size()) fail("unterminated element <" + n->name + ">");
            if (starts("</")) {
                i += 2;
                std::string en = name();
                if (en != n->name) fail("mismatched </" + en + "> for <" + n->name + ">");
                skip_ws();
                if (i >= s.size() || s[i] != '>') fail("expected '>'");
                i++;
                return n;
            }
            if (starts("<!--")) {
                skip_until("-->");
                continue;
            }
            if (starts("<?")) {
                skip_until("?>");
                continue;
            }
            n->children.push_back(element());
        }
    }
};

}  // namespace

std::unique_ptr<XmlNode> xml_parse(const std::string& text)
{
    Parser p(text);
    auto root = std::make_unique<XmlNode>();
    p.misc();
    while (p.i < text.size()) {
        root->children.push_back(p.element());
        p.misc();
    }
    return root;
}

std::unique_ptr<XmlNode> xml_load(const std::string& filename)
{
    std::ifstream f(filename);
    if (!f) throw XmlError{"cannot open " + filename};
    std::stringstream ss;
    ss << f.rdbuf();
    return xml_parse(ss.str());
}

}  // namespace bcm3
