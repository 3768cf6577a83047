// sc_model.cpp -- libconfig-subset reader/writer + strict cascade loading.
// See sc_model.hpp for the reference interfaces mirrored here.
#include "sc_model.hpp"

#include <cctype>
#include <cerrno>
#include <clocale>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "surfcascade.h"

namespace sc {

const CfgValue *CfgValue::find(const std::string &key) const {
    for (const CfgValue &v : items)
        if (v.name == key) return &v;
    return nullptr;
}

int Cascade::total_weak() const {
    int n = 0;
    for (const Stage &s : stages) n += (int)s.weak.size();
    return n;
}

// ---------------------------------------------------------------------------
// reader
// ---------------------------------------------------------------------------
namespace {

// Nesting bound of groups / arrays / lists: libconfig's bison parser fails a
// too-deep file with a parse error when its stack (YYMAXDEPTH 10000 states)
// runs out; this recursive-descent reader fails it at 1000 levels (a model
// nests 4 deep) instead of overflowing the thread's stack.
constexpr int kMaxDepth = 1000;

struct Parser {
    const std::string &s;
    size_t i = 0;
    int line = 1;
    int depth = 0;

    [[noreturn]] void fail(const std::string &what) {
        throw Error{SC_ERR_PARSE, "model.cfg:" + std::to_string(line) + ": " + what};
    }

    void skip() {  // whitespace and the three comment forms
        for (;;) {
            if (i >= s.size()) return;
            char c = s[i];
            if (c == '\n') { line++; i++; continue; }
            if (std::isspace((unsigned char)c)) { i++; continue; }
            if (c == '#' || (c == '/' && i + 1 < s.size() && s[i + 1] == '/')) {
                while (i < s.size() && s[i] != '\n') i++;
                continue;
            }
            if (c == '/' && i + 1 < s.size() && s[i + 1] == '*') {
                size_t e = s.find("*/", i + 2);
                if (e == std::string::npos) fail("unterminated comment");
                for (size_t k = i; k < e; k++) line += s[k] == '\n';
                i = e + 2;
                continue;
            }
            return;
        }
    }

    bool peek(char c) {
        skip();
        return i < s.size() && s[i] == c;
    }

    static bool name_start(char c) { return std::isalpha((unsigned char)c) || c == '*'; }
    static bool name_char(char c) {
        return std::isalnum((unsigned char)c) || c == '-' || c == '_' || c == '*';
    }

    std::string name() {
        skip();
        if (i >= s.size() || !name_start(s[i])) fail("setting name expected");
        size_t b = i;
        while (i < s.size() && name_char(s[i])) i++;
        return s.substr(b, i - b);
    }

    // number token: float / int / int64 / hex (scanner.c:1146-1172 semantics)
    bool number(CfgValue &v) {
        size_t b = i, k = i;
        if (k < s.size() && (s[k] == '+' || s[k] == '-')) k++;
        if (k + 1 < s.size() && s[k] == '0' && (s[k + 1] == 'x' || s[k + 1] == 'X')) {
            size_t h = k + 2;
            while (h < s.size() && std::isxdigit((unsigned char)s[h])) h++;
            if (h == k + 2) fail("bad hex literal");
            std::string t = s.substr(b, h - b);
            bool is64 = h < s.size() && s[h] == 'L';
            while (h < s.size() && s[h] == 'L') h++;
            v.type = is64 ? CfgValue::Int64 : CfgValue::Int;
            v.ival = (int64_t)std::strtoull(t.c_str() + (k - b) + 2, nullptr, 16);
            if (!is64) v.ival = (int32_t)(uint32_t)v.ival;
            i = h;
            return true;
        }
        size_t d0 = k;
        while (k < s.size() && std::isdigit((unsigned char)s[k])) k++;
        bool digits = k > d0, dot = false, expo = false;
        if (k < s.size() && s[k] == '.') {
            dot = true;
            k++;
            while (k < s.size() && std::isdigit((unsigned char)s[k])) k++;
        }
        if (k < s.size() && (s[k] == 'e' || s[k] == 'E')) {
            size_t e = k + 1;
            if (e < s.size() && (s[e] == '+' || s[e] == '-')) e++;
            size_t e0 = e;
            while (e < s.size() && std::isdigit((unsigned char)s[e])) e++;
            if (e > e0) { expo = true; k = e; }
        }
        if (!digits && !dot) return false;
        std::string t = s.substr(b, k - b);
        if (dot || expo) {
            if (!dot && !digits) fail("bad float literal");
            v.type = CfgValue::Float;
            v.fval = std::strtod(t.c_str(), nullptr);  // atof (scanner.c:1146)
            i = k;
            return true;
        }
        bool is64 = k < s.size() && s[k] == 'L';
        errno = 0;
        long long x = std::strtoll(t.c_str(), nullptr, 10);
        if (errno == ERANGE) fail("integer out of range");
        if (is64) {
            while (k < s.size() && s[k] == 'L') k++;
            v.type = CfgValue::Int64;
        } else {
            if (x < INT32_MIN || x > INT32_MAX) fail("integer out of range");
            v.type = CfgValue::Int;
        }
        v.ival = x;
        i = k;
        return true;
    }

    std::string string_lit() {
        std::string out;
        for (;;) {  // adjacent literals concatenate
            i++;     // opening quote
            while (i < s.size() && s[i] != '"') {
                char c = s[i++];
                if (c == '\n') line++;
                if (c != '\\') { out += c; continue; }
                if (i >= s.size()) fail("bad escape");
                char e = s[i++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 'f': out += '\f'; break;
                    case 't': out += '\t'; break;
                    case 'x': {
                        if (i + 2 > s.size()) fail("bad \\x escape");
                        out += (char)std::strtol(s.substr(i, 2).c_str(), nullptr, 16);
                        i += 2;
                        break;
                    }
                    default: out += e;
                }
            }
            if (i >= s.size()) fail("unterminated string");
            i++;
            if (!peek('"')) return out;
        }
    }

    CfgValue value() {
        skip();
        if (i >= s.size()) fail("value expected");
        CfgValue v;
        char c = s[i];
        if ((c == '{' || c == '[' || c == '(') && depth >= kMaxDepth) fail("nested too deeply");
        struct Nest {  // depth of the aggregate being read (restored on throw too)
            int &d;
            explicit Nest(int &x) : d(++x) {}
            ~Nest() { d--; }
        };
        if (c == '{') {
            Nest nest(depth);
            i++;
            v.type = CfgValue::Group;
            settings(v, '}');
            return v;
        }
        if (c == '[' || c == '(') {
            Nest nest(depth);
            char close = c == '[' ? ']' : ')';
            v.type = c == '[' ? CfgValue::Array : CfgValue::List;
            i++;
            if (!peek(close)) {
                for (;;) {
                    CfgValue e = value();
                    if (v.type == CfgValue::Array) {
                        if (e.type == CfgValue::Group || e.type == CfgValue::List ||
                            e.type == CfgValue::Array)
                            fail("array elements must be scalar");
                        if (!v.items.empty() && v.items[0].type != e.type)
                            fail("array elements must share one type");
                    }
                    v.items.push_back(std::move(e));
                    if (peek(',')) { i++; continue; }
                    break;
                }
            }
            if (!peek(close)) fail(std::string("'") + close + "' expected");
            i++;
            return v;
        }
        if (c == '"') {
            v.type = CfgValue::String;
            v.sval = string_lit();
            return v;
        }
        if (number(v)) return v;
        if (name_start(c)) {
            std::string t = name();
            std::string lo;
            for (char ch : t) lo += (char)std::tolower((unsigned char)ch);
            if (lo == "true" || lo == "false") {
                v.type = CfgValue::Bool;
                v.ival = lo == "true";
                return v;
            }
            fail("unexpected identifier '" + t + "'");
        }
        fail(std::string("unexpected character '") + c + "'");
    }

    void settings(CfgValue &grp, char close) {
        for (;;) {
            skip();
            if (i >= s.size()) {
                if (close) fail("unexpected end of file");
                return;
            }
            if (close && s[i] == close) { i++; return; }
            std::string n = name();
            skip();
            if (i >= s.size() || (s[i] != '=' && s[i] != ':')) fail("'=' or ':' expected");
            i++;
            if (grp.find(n)) fail("duplicate setting '" + n + "'");
            CfgValue v = value();
            v.name = n;
            grp.items.push_back(std::move(v));
            if (peek(';') || peek(',')) i++;
        }
    }
};

}  // namespace

// libconfig's include directive (scanner.l: `^[ \t]*@include[ \t]+"file"`):
// the named file's text replaces the line.  Model::Load sets no include
// directory, so relative paths resolve against the working directory.
std::string expand_includes(const std::string &text, int depth) {
    if (text.find("@include") == std::string::npos) return text;
    if (depth >= 10)  // libconfig's MAX_INCLUDE_DEPTH
        throw Error{SC_ERR_PARSE, "@include nested too deeply"};
    std::string out;
    size_t pos = 0;
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size();
        const std::string ln = text.substr(pos, eol - pos);
        size_t k = 0;
        while (k < ln.size() && (ln[k] == ' ' || ln[k] == '\t')) k++;
        if (ln.compare(k, 8, "@include") == 0) {
            size_t q0 = ln.find('"', k + 8), q1 = q0 == std::string::npos ? q0 : ln.find('"', q0 + 1);
            if (q1 == std::string::npos) throw Error{SC_ERR_PARSE, "bad @include line"};
            const std::string path = ln.substr(q0 + 1, q1 - q0 - 1);
            std::FILE *f = std::fopen(path.c_str(), "rb");
            if (!f) throw Error{SC_ERR_PARSE, "cannot open include file '" + path + "'"};
            std::string inc;
            char buf[4096];
            size_t n;
            while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) inc.append(buf, n);
            std::fclose(f);
            out += expand_includes(inc, depth + 1);
            out += ln.substr(q1 + 1);
        } else {
            out += ln;
        }
        if (eol < text.size()) out += '\n';
        pos = eol + 1;
    }
    return out;
}

CfgValue cfg_parse(const std::string &text_in) {
    const std::string text = expand_includes(text_in, 0);
    Parser p{text};
    CfgValue root;
    root.type = CfgValue::Group;
    p.settings(root, 0);
    return root;
}

// ---------------------------------------------------------------------------
// writer (libconfig.c:168-243, 631-653; tab width 2)
// ---------------------------------------------------------------------------

std::string cfg_format_float(double v) {
    char buf[64];
    std::snprintf(buf, sizeof(buf) - 3, "%.*g", 10, v);
    if (!std::strchr(buf, 'e')) {
        if (!std::strchr(buf, '.')) {
            std::strcat(buf, ".0");
        } else {
            for (char *p = buf + std::strlen(buf) - 1; p > buf; --p)
                if (*p != '0') { *(++p) = '\0'; break; }
        }
    }
    return buf;
}

namespace {
void indent(std::string &o, int depth) {
    if (depth > 1) o.append((size_t)(depth - 1) * 2, ' ');
}
void write_setting(std::string &o, const CfgValue &v, int depth);

void write_value(std::string &o, const CfgValue &v, int depth) {
    char buf[64];
    switch (v.type) {
        case CfgValue::Bool: o += v.ival ? "true" : "false"; break;
        case CfgValue::Int: std::snprintf(buf, sizeof buf, "%d", (int)v.ival); o += buf; break;
        case CfgValue::Int64: std::snprintf(buf, sizeof buf, "%lldL", (long long)v.ival); o += buf; break;
        case CfgValue::Float: o += cfg_format_float(v.fval); break;
        case CfgValue::String: {
            o += '"';
            for (unsigned char c : v.sval) {
                if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
                else if (c == '\n') o += "\\n";
                else if (c == '\r') o += "\\r";
                else if (c == '\f') o += "\\f";
                else if (c == '\t') o += "\\t";
                else if (c >= ' ') o += (char)c;
                else { std::snprintf(buf, sizeof buf, "\\x%02X", c); o += buf; }
            }
            o += '"';
            break;
        }
        case CfgValue::List:
        case CfgValue::Array: {
            o += v.type == CfgValue::List ? "( " : "[ ";
            for (size_t k = 0; k < v.items.size(); k++) {
                write_value(o, v.items[k], depth + 1);
                if (k + 1 < v.items.size()) o += ',';
                o += ' ';
            }
            o += v.type == CfgValue::List ? ')' : ']';
            break;
        }
        case CfgValue::Group: {
            if (depth > 0) {
                o += '\n';
                indent(o, depth);
                o += "{\n";
            }
            for (const CfgValue &c : v.items) write_setting(o, c, depth + 1);
            indent(o, depth);
            if (depth > 0) o += '}';
            break;
        }
    }
}

void write_setting(std::string &o, const CfgValue &v, int depth) {
    indent(o, depth);
    if (!v.name.empty()) {
        o += v.name;
        o += v.type == CfgValue::Group ? " : " : " = ";
    }
    write_value(o, v, depth);
    if (depth > 0) o += ";\n";
}
}  // namespace

std::string cfg_write(const CfgValue &root) {
    std::string o;
    write_value(o, root, 0);
    return o;
}

// ---------------------------------------------------------------------------
// typed access (libconfigcpp.c++:700-716 operators, :1137-1145 assertType;
// auto-convert off) -- strict: missing key => SC_ERR_MODEL
// ---------------------------------------------------------------------------
namespace {
const CfgValue &get(const CfgValue &g, const char *key, const std::string &where) {
    const CfgValue *v = g.find(key);
    if (!v) throw Error{SC_ERR_MODEL, where + ": missing setting '" + key + "'"};
    return *v;
}
[[noreturn]] void type_err(const CfgValue &v, const std::string &where, const char *want) {
    throw Error{SC_ERR_MODEL, where + ": setting '" + v.name + "' is not " + want};
}
double as_double(const CfgValue &v, const std::string &where) {
    if (v.type != CfgValue::Float) type_err(v, where, "a float");
    return v.fval;
}
float as_float(const CfgValue &v, const std::string &where) {
    return static_cast<float>(as_double(v, where));  // libconfigcpp.c++:710-716
}
int as_int(const CfgValue &v, const std::string &where) {
    if (v.type != CfgValue::Int) type_err(v, where, "an int");
    return (int)v.ival;
}
const CfgValue &as_seq(const CfgValue &v, CfgValue::Type t, const std::string &where) {
    if (v.type != t) type_err(v, where, t == CfgValue::List ? "a list" : "an array");
    return v;
}
CfgValue mk(const char *name, CfgValue::Type t) {
    CfgValue v;
    v.name = name ? name : "";
    v.type = t;
    return v;
}
CfgValue mkf(const char *name, double x) { CfgValue v = mk(name, CfgValue::Float); v.fval = x; return v; }
CfgValue mki(const char *name, int64_t x) { CfgValue v = mk(name, CfgValue::Int); v.ival = x; return v; }
}  // namespace

// Model::Load, Model.cpp:120-186.
Cascade cascade_from_cfg(const CfgValue &root) {
    Cascade c;
    const CfgValue &cg = get(root, "cascade_classifier", "root");
    if (cg.type != CfgValue::Group) type_err(cg, "root", "a group");
    const std::string W0 = "cascade_classifier";
    c.max_stages_num = as_int(get(cg, "max_stages_num", W0), W0);
    c.FPR_target = as_float(get(cg, "FPR_target", W0), W0);
    c.TPR_min_perstage = as_float(get(cg, "TPR_min_perstage", W0), W0);
    c.FPR = as_float(get(cg, "FPR", W0), W0);
    c.TPR = as_float(get(cg, "TPR", W0), W0);
    const CfgValue &sl = as_seq(get(cg, "stage_classifiers", W0), CfgValue::List, W0);
    for (size_t i = 0; i < sl.items.size(); i++) {
        const CfgValue &sg = sl.items[i];
        std::string W1 = "stage_classifiers[" + std::to_string(i) + "]";
        if (sg.type != CfgValue::Group) throw Error{SC_ERR_MODEL, W1 + ": not a group"};
        Stage st;
        st.search_step = as_float(get(sg, "search_step", W1), W1);
        st.auc_step = as_float(get(sg, "auc_step", W1), W1);
        st.TPR_min = as_float(get(sg, "TPR_min", W1), W1);
        st.n_total = as_int(get(sg, "n_total", W1), W1);
        st.n_pos = as_int(get(sg, "n_pos", W1), W1);
        st.n_neg = as_int(get(sg, "n_neg", W1), W1);
        st.FPR = as_float(get(sg, "FPR", W1), W1);
        st.TPR = as_float(get(sg, "TPR", W1), W1);
        st.theta = as_float(get(sg, "theta", W1), W1);
        st.total_AUC_score = as_float(get(sg, "total_AUC_score", W1), W1);
        st.sample_num = as_int(get(sg, "sample_num", W1), W1);
        st.max_iters = as_int(get(sg, "max_iters", W1), W1);
        const CfgValue &wl = as_seq(get(sg, "weak_classifiers", W1), CfgValue::List, W1);
        for (size_t j = 0; j < wl.items.size(); j++) {
            const CfgValue &wg = wl.items[j];
            std::string W2 = W1 + ".weak_classifiers[" + std::to_string(j) + "]";
            if (wg.type != CfgValue::Group) throw Error{SC_ERR_MODEL, W2 + ": not a group"};
            WeakLR wk;
            wk.patch_index = as_int(get(wg, "patch_index", W2), W2);
            wk.eps = as_double(get(wg, "eps", W2), W2);
            wk.C = as_double(get(wg, "C", W2), W2);
            wk.nr_class = as_int(get(wg, "nr_class", W2), W2);
            wk.nr_feature = as_int(get(wg, "nr_feature", W2), W2);
            wk.bias = as_double(get(wg, "bias", W2), W2);
            const CfgValue &wa = as_seq(get(wg, "w", W2), CfgValue::Array, W2);
            for (const CfgValue &e : wa.items) wk.w.push_back(as_float(e, W2 + ".w"));
            const CfgValue &la = as_seq(get(wg, "label", W2), CfgValue::Array, W2);
            if (la.items.size() < 2) throw Error{SC_ERR_MODEL, W2 + ": label needs 2 entries"};
            wk.label[0] = as_int(la.items[0], W2 + ".label");
            wk.label[1] = as_int(la.items[1], W2 + ".label");
            st.weak.push_back(std::move(wk));
        }
        c.stages.push_back(std::move(st));
    }
    return c;
}

// Model::Save, Model.cpp:24-83 (same keys, same order, same types).
CfgValue cascade_to_cfg(const Cascade &c) {
    CfgValue root = mk(nullptr, CfgValue::Group);
    CfgValue cg = mk("cascade_classifier", CfgValue::Group);
    cg.items.push_back(mki("max_stages_num", c.max_stages_num));
    cg.items.push_back(mkf("FPR_target", c.FPR_target));
    cg.items.push_back(mkf("TPR_min_perstage", c.TPR_min_perstage));
    cg.items.push_back(mkf("FPR", c.FPR));
    cg.items.push_back(mkf("TPR", c.TPR));
    CfgValue sl = mk("stage_classifiers", CfgValue::List);
    for (const Stage &st : c.stages) {
        CfgValue sg = mk(nullptr, CfgValue::Group);
        sg.items.push_back(mkf("search_step", st.search_step));
        sg.items.push_back(mkf("auc_step", st.auc_step));
        sg.items.push_back(mkf("TPR_min", st.TPR_min));
        sg.items.push_back(mki("n_total", st.n_total));
        sg.items.push_back(mki("n_pos", st.n_pos));
        sg.items.push_back(mki("n_neg", st.n_neg));
        sg.items.push_back(mkf("FPR", st.FPR));
        sg.items.push_back(mkf("TPR", st.TPR));
        sg.items.push_back(mkf("theta", st.theta));
        sg.items.push_back(mkf("total_AUC_score", st.total_AUC_score));
        sg.items.push_back(mki("sample_num", st.sample_num));
        sg.items.push_back(mki("max_iters", st.max_iters));
        CfgValue wl = mk("weak_classifiers", CfgValue::List);
        for (const WeakLR &wk : st.weak) {
            CfgValue wg = mk(nullptr, CfgValue::Group);
            wg.items.push_back(mki("patch_index", wk.patch_index));
            wg.items.push_back(mkf("eps", wk.eps));
            wg.items.push_back(mkf("C", wk.C));
            wg.items.push_back(mki("nr_class", wk.nr_class));
            wg.items.push_back(mki("nr_feature", wk.nr_feature));
            wg.items.push_back(mkf("bias", wk.bias));
            CfgValue wa = mk("w", CfgValue::Array);
            for (float x : wk.w) wa.items.push_back(mkf(nullptr, x));
            wg.items.push_back(std::move(wa));
            CfgValue la = mk("label", CfgValue::Array);
            la.items.push_back(mki(nullptr, wk.label[0]));
            la.items.push_back(mki(nullptr, wk.label[1]));
            wg.items.push_back(std::move(la));
            wl.items.push_back(std::move(wg));
        }
        sg.items.push_back(std::move(wl));
        sl.items.push_back(std::move(sg));
    }
    cg.items.push_back(std::move(sl));
    root.items.push_back(std::move(cg));
    return root;
}

// What the detect path needs beyond a successful Load.
void validate_for_detect(const Cascade &c, int n_patches) {
    if (c.stages.empty()) throw Error{SC_ERR_MODEL, "cascade has no stages"};
    for (size_t i = 0; i < c.stages.size(); i++) {
        const Stage &st = c.stages[i];
        if (st.weak.empty())
            throw Error{SC_ERR_MODEL, "stage " + std::to_string(i) + " has no weak classifiers"};
        for (size_t j = 0; j < st.weak.size(); j++) {
            const WeakLR &wk = st.weak[j];
            std::string where = "stage " + std::to_string(i) + " weak " + std::to_string(j);
            if (wk.w.size() != 33)
                throw Error{SC_ERR_MODEL, where + ": w must have 33 entries (32 + bias weight)"};
            if (wk.patch_index < 0 || wk.patch_index >= n_patches)
                throw Error{SC_ERR_MODEL, where + ": patch_index " + std::to_string(wk.patch_index) +
                                              " outside the template's " + std::to_string(n_patches) +
                                              " patches"};
        }
    }
}

// DenseSURFFeatureExtractor::ExtractPatches, DenseSURFFeatureExtractor.cpp:49-63
// (shapes .cpp:21; min cell edge 6 and stride 4, .h:34-35).
std::vector<int32_t> extract_patches(int tw, int th) {
    static const int shp[3][2] = {{2, 2}, {1, 4}, {4, 1}};
    std::vector<int32_t> r;
    for (auto &sh : shp)
        for (int c = 6; c <= tw / 2; c++) {
            int pw = sh[0] * c, ph = sh[1] * c;
            for (int y = 0; y + ph <= th; y += 4)
                for (int x = 0; x + pw <= tw; x += 4) {
                    r.push_back(x);
                    r.push_back(y);
                    r.push_back(pw);
                    r.push_back(ph);
                }
        }
    return r;
}

}  // namespace sc
