// mpcg_yaml.cpp — reader for the YAML subset of include/mpc_planner_solver/mpcg_yaml.h.
#include "mpc_planner_solver/mpcg_yaml.h"

#include <cerrno>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace mpcg {

YamlNode YamlNode::scalar(std::string s) {
    YamlNode n;
    n.kind_ = Kind::Scalar;
    n.text_ = std::move(s);
    return n;
}

YamlNode YamlNode::null() {
    YamlNode n;
    n.kind_ = Kind::Null;
    return n;
}

YamlNode YamlNode::sequence() {
    YamlNode n;
    n.kind_ = Kind::Sequence;
    n.seq_ = std::make_shared<std::vector<YamlNode>>();
    return n;
}

YamlNode YamlNode::map() {
    YamlNode n;
    n.kind_ = Kind::Map;
    n.map_ = std::make_shared<std::vector<Entry>>();
    n.index_ = std::make_shared<std::unordered_map<std::string, std::size_t>>();
    return n;
}

std::size_t YamlNode::size() const {
    if (kind_ == Kind::Sequence) return seq_->size();
    if (kind_ == Kind::Map) return map_->size();
    return 0;
}

static const YamlNode& undefined_node() {
    static const YamlNode u;
    return u;
}

const YamlNode& YamlNode::operator[](const std::string& key) const {
    if (kind_ != Kind::Map) return undefined_node();
    auto it = index_->find(key);
    return it == index_->end() ? undefined_node() : (*map_)[it->second].second;
}

const YamlNode& YamlNode::operator[](std::size_t i) const {
    if (kind_ != Kind::Sequence || i >= seq_->size()) return undefined_node();
    return (*seq_)[i];
}

static const std::vector<YamlNode::Entry>& empty_entries() {
    static const std::vector<YamlNode::Entry> e;
    return e;
}

YamlNode::const_iterator YamlNode::begin() const { return kind_ == Kind::Map ? map_->cbegin() : empty_entries().cbegin(); }
YamlNode::const_iterator YamlNode::end() const { return kind_ == Kind::Map ? map_->cend() : empty_entries().cend(); }

void YamlNode::push_back(YamlNode v) {
    if (kind_ != Kind::Sequence) throw std::runtime_error("yaml: push_back on a non-sequence");
    seq_->push_back(std::move(v));
}

void YamlNode::set(const std::string& key, YamlNode v) {
    if (kind_ != Kind::Map) throw std::runtime_error("yaml: set on a non-map");
    auto it = index_->find(key);
    if (it != index_->end()) {
        (*map_)[it->second].second = std::move(v);
        return;
    }
    (*index_)[key] = map_->size();
    map_->emplace_back(scalar(key), std::move(v));
}

const std::string& YamlNode::require_scalar(const char* what) const {
    if (kind_ != Kind::Scalar) throw std::runtime_error(std::string("yaml: node is not a scalar (as<") + what + ">)");
    return text_;
}

template <>
long YamlNode::as<long>() const {
    const std::string& s = require_scalar("long");
    char* end = nullptr;
    errno = 0;
    long v = std::strtol(s.c_str(), &end, 10);
    if (errno || end == s.c_str() || *end) throw std::runtime_error("yaml: bad integer '" + s + "'");
    return v;
}

template <>
int YamlNode::as<int>() const { return static_cast<int>(as<long>()); }

template <>
unsigned int YamlNode::as<unsigned int>() const {
    long v = as<long>();
    if (v < 0) throw std::runtime_error("yaml: negative value for unsigned");
    return static_cast<unsigned int>(v);
}

template <>
double YamlNode::as<double>() const {
    const std::string& s = require_scalar("double");
    if (s == ".inf" || s == ".Inf" || s == "inf") return 1.0 / 0.0;
    if (s == "-.inf" || s == "-.Inf" || s == "-inf") return -1.0 / 0.0;
    char* end = nullptr;
    double v = std::strtod(s.c_str(), &end);
    if (end == s.c_str() || *end) throw std::runtime_error("yaml: bad number '" + s + "'");
    return v;
}

template <>
bool YamlNode::as<bool>() const {
    const std::string& s = require_scalar("bool");
    if (s == "true" || s == "True" || s == "TRUE" || s == "yes" || s == "on") return true;
    if (s == "false" || s == "False" || s == "FALSE" || s == "no" || s == "off") return false;
    throw std::runtime_error("yaml: bad boolean '" + s + "'");
}

template <>
std::string YamlNode::as<std::string>() const { return require_scalar("string"); }

// ---------------------------------------------------------------- parser
namespace {

struct Line {
    int indent;
    std::string body;
    int number;
};

std::string strip_comment(const std::string& s) {
    char quote = 0;
    for (std::size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if (quote) {
            if (c == quote) quote = 0;
        } else if (c == '"' || c == '\'') {
            quote = c;
        } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
            return s.substr(0, i);
        }
    }
    return s;
}

std::string trim(const std::string& s) {
    std::size_t a = s.find_first_not_of(" \t\r");
    if (a == std::string::npos) return "";
    std::size_t b = s.find_last_not_of(" \t\r");
    return s.substr(a, b - a + 1);
}

[[noreturn]] void fail(int line, const std::string& msg) {
    throw std::runtime_error("yaml line " + std::to_string(line) + ": " + msg);
}

YamlNode parse_scalar(const std::string& raw, int line) {
    std::string s = trim(raw);
    if (s.empty() || s == "~" || s == "null") return YamlNode::null();
    if (s.front() == '"' || s.front() == '\'') {
        if (s.size() < 2 || s.back() != s.front()) fail(line, "unterminated quoted scalar");
        return YamlNode::scalar(s.substr(1, s.size() - 2));
    }
    if (s.front() == '[') {
        if (s.back() != ']') fail(line, "flow sequence must close on the same line");
        YamlNode seq = YamlNode::sequence();
        std::string inner = trim(s.substr(1, s.size() - 2));
        if (inner.empty()) return seq;
        std::size_t start = 0;
        char quote = 0;
        for (std::size_t i = 0; i <= inner.size(); ++i) {
            char c = i < inner.size() ? inner[i] : ',';
            if (quote) {
                if (c == quote) quote = 0;
                continue;
            }
            if (c == '"' || c == '\'') quote = c;
            else if (c == ',') {
                seq.push_back(parse_scalar(inner.substr(start, i - start), line));
                start = i + 1;
            }
        }
        return seq;
    }
    if (s.front() == '{') fail(line, "flow maps are outside the supported subset");
    return YamlNode::scalar(s);
}

// position of the key/value separator ': ' (or a trailing ':') outside quotes
std::size_t key_sep(const std::string& s) {
    char quote = 0;
    for (std::size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if (quote) {
            if (c == quote) quote = 0;
            continue;
        }
        if (c == '"' || c == '\'') quote = c;
        else if (c == ':' && (i + 1 == s.size() || s[i + 1] == ' ')) return i;
    }
    return std::string::npos;
}

bool is_item(const std::string& b) { return b == "-" || (b.size() >= 2 && b[0] == '-' && b[1] == ' '); }

YamlNode parse_block(const std::vector<Line>& L, std::size_t& i, int indent);

YamlNode parse_sequence(const std::vector<Line>& L, std::size_t& i, int indent) {
    YamlNode seq = YamlNode::sequence();
    while (i < L.size() && L[i].indent == indent && is_item(L[i].body)) {
        std::string rest = L[i].body.size() > 1 ? trim(L[i].body.substr(2)) : "";
        int ln = L[i].number;
        ++i;
        if (rest.empty()) {
            if (i < L.size() && L[i].indent > indent) seq.push_back(parse_block(L, i, L[i].indent));
            else seq.push_back(YamlNode::null());
        } else if (key_sep(rest) != std::string::npos && rest.front() != '"' && rest.front() != '\'') {
            fail(ln, "maps inside sequence items are outside the supported subset");
        } else {
            seq.push_back(parse_scalar(rest, ln));
        }
    }
    return seq;
}

YamlNode parse_map(const std::vector<Line>& L, std::size_t& i, int indent) {
    YamlNode map = YamlNode::map();
    while (i < L.size() && L[i].indent == indent && !is_item(L[i].body)) {
        const std::string& b = L[i].body;
        int ln = L[i].number;
        std::size_t c = key_sep(b);
        if (c == std::string::npos) fail(ln, "expected 'key: value'");
        std::string key = trim(b.substr(0, c));
        if (key.size() >= 2 && (key.front() == '"' || key.front() == '\'') && key.back() == key.front())
            key = key.substr(1, key.size() - 2);
        std::string val = trim(b.substr(c + 1));
        ++i;
        if (!val.empty()) {
            map.set(key, parse_scalar(val, ln));
        } else if (i < L.size() && L[i].indent > indent) {
            map.set(key, parse_block(L, i, L[i].indent));
        } else if (i < L.size() && L[i].indent == indent && is_item(L[i].body)) {
            map.set(key, parse_sequence(L, i, indent));  // PyYAML: "key:\n- a\n- b"
        } else {
            map.set(key, YamlNode::null());
        }
    }
    return map;
}

YamlNode parse_block(const std::vector<Line>& L, std::size_t& i, int indent) {
    return is_item(L[i].body) ? parse_sequence(L, i, indent) : parse_map(L, i, indent);
}

}  // namespace

YamlNode yaml_parse(const std::string& text) {
    std::vector<Line> L;
    std::istringstream in(text);
    std::string raw;
    int number = 0;
    while (std::getline(in, raw)) {
        ++number;
        if (raw.rfind("---", 0) == 0 || raw.rfind("...", 0) == 0) continue;
        std::string s = strip_comment(raw);
        if (trim(s).empty()) continue;
        if (s.find('\t') != std::string::npos && s.find_first_not_of(" \t") > s.find('\t'))
            fail(number, "tab indentation");
        int ind = static_cast<int>(s.find_first_not_of(' '));
        L.push_back({ind, trim(s), number});
    }
    if (L.empty()) return YamlNode::null();
    std::size_t i = 0;
    YamlNode root = parse_block(L, i, L[0].indent);
    if (i != L.size()) fail(L[i].number, "unexpected indentation");
    return root;
}

YamlNode yaml_load_file(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("yaml: cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return yaml_parse(ss.str());
}

}  // namespace mpcg
