// Go front-end: project-level package analysis with the go-analyzer JSON contract.
//
// Parity target: tools/go-analyzer/pkg/analysis/{analyzer.go,types.go} (the
// reference's only native component, run as a subprocess by
// GoSourceParser.java:339-454).  This is an in-process C++ replacement that
// emits the same ProjectAnalysis document (types.go:10-175):
//   * module path from go.mod                                   analyzer.go:51-66
//   * lexical directory walk, excluded dirs / test / generated  :69-118, :735-751
//   * per package: internal imports, structs (fields, embedded),
//     interfaces, funcs (receiver, params, returns, doc, panic)  :140-404
//   * methods bound to structs by receiver name                 :481-502
//   * entry point (main.main or HTTP registration calls)        :505-534, :651-681
//   * HTTP handler params -> ("GET", "")                        :685-706
//   * class type by handler presence, then dir-name keywords    :537-623
// Divergences (docs/PARITY.md): ParamInfo.package is the resolved internal
// import path (the reference returns only the alias, analyzer.go:461-478, so
// parameter links almost never matched); generic receivers bind to their base
// type; `implements` is populated from method-name sets within the module; the
// walk never skips the project root itself even if its name starts with '.';
// literal route registrations (gin/echo/chi/fiber verbs, Group prefixes,
// Go 1.22 "METHOD /path" mux patterns) give handlers a real verb + path, so Go
// handlers become HTTP endpoints (the reference never reports a path).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <dirent.h>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "srcscan.hpp"

namespace srcscan {
namespace {

struct GoParam {
    std::string name, type, package;
    bool is_pointer = false, is_slice = false, is_variadic = false;
};
struct GoField {
    std::string name, type, package, tag;
    bool exported = false;
};
struct GoFunc {
    std::string name, file, receiver, http_method, http_path, doc;
    int line = 0;
    std::vector<GoParam> params;
    std::vector<std::string> returns;
    bool has_panic = false;
    bool has_http_registration = false;
};
struct GoStruct {
    std::string name, file;
    int line = 0;
    std::vector<GoField> fields;
    std::vector<std::string> embedded;
    std::vector<GoFunc> methods;
    std::vector<std::string> implements;
};
struct GoIfaceMethod {
    std::string name;
    std::vector<GoParam> params;
};
struct GoInterface {
    std::string name, file;
    int line = 0;
    std::vector<GoIfaceMethod> methods;
    std::vector<std::string> embedded;
};
// A literal route registration `recv.VERB("/path", ..., qual.Handler)`.
// (Addition: the reference's analyzer only reports ("GET", "") for handlers,
// which the Java side then treats as "not an endpoint".)
struct GoRoute {
    std::string recv, method, path, qualifier, handler;
};
struct GoGroup {
    std::string var, parent, prefix;
};
struct GoPackage {
    std::string path, dir, pkg_name, class_type = "OTHER";
    std::vector<std::string> files, imports;
    std::vector<GoStruct> structs;
    std::vector<GoInterface> interfaces;
    std::vector<GoFunc> functions;
    std::vector<GoRoute> routes;  // group prefixes already applied
    bool entry_point = false;
    bool ok = false;
};

const std::unordered_set<std::string_view> kHttpRegistration = {
    "GET", "POST", "PUT", "DELETE", "PATCH", "HEAD", "OPTIONS", "Get", "Post", "Put",
    "Delete", "Patch", "Handle", "HandleFunc", "Group", "Route", "Any"};

bool excluded_dir(const std::string& name) {
    static const std::unordered_set<std::string> ex = {"vendor", "testdata", ".git", "node_modules",
                                                       "third_party", "tools", ".idea", ".vscode"};
    return ex.count(name) > 0 || (!name.empty() && name[0] == '.');
}

bool generated_file(const std::string& name) {
    return ends_with(name, ".pb.go") || ends_with(name, "_generated.go") || ends_with(name, "_gen.go") ||
           name == "wire_gen.go" || name == "mock_gen.go";
}

bool eligible_go_file(const std::string& name) {
    return ends_with(name, ".go") && !ends_with(name, "_test.go") && !generated_file(name);
}

bool is_exported_name(std::string_view s) {
    return !s.empty() && s[0] >= 'A' && s[0] <= 'Z';
}

// Per-file parse state
struct FileParse {
    std::string file;            // basename
    std::string pkg_name;
    std::map<std::string, std::string> alias_to_path;  // import alias -> path
    std::vector<std::string> import_paths;
    std::vector<GoStruct> structs;
    std::vector<GoInterface> interfaces;
    std::vector<GoFunc> funcs;
    std::vector<GoRoute> routes;
    std::vector<GoGroup> groups;
    bool has_http_registration = false;
};

const std::unordered_map<std::string_view, const char*> kRouteVerbs = {
    {"GET", "GET"},       {"POST", "POST"},   {"PUT", "PUT"},     {"DELETE", "DELETE"}, {"PATCH", "PATCH"},
    {"HEAD", "HEAD"},     {"OPTIONS", "OPTIONS"}, {"Get", "GET"}, {"Post", "POST"},     {"Put", "PUT"},
    {"Delete", "DELETE"}, {"Patch", "PATCH"}, {"Head", "HEAD"},   {"Options", "OPTIONS"}, {"Any", "GET"},
    {"Handle", "GET"},    {"HandleFunc", "GET"}};

std::string join_route(const std::string& prefix, const std::string& path) {
    if (prefix.empty()) return path;
    if (path.empty()) return prefix;
    bool a = prefix.back() == '/', b = path.front() == '/';
    if (a && b) return prefix + path.substr(1);
    if (!a && !b) return prefix + "/" + path;
    return prefix + path;
}

class GoFileParser {
public:
    GoFileParser(std::string_view src, const std::vector<Token>& toks, const std::string& module, FileParse& fp)
        : src_(src), t(toks), n((int)toks.size()), module_(module), fp_(fp) {
        // line starts for doc-comment lookup
        line_starts_.push_back(0);
        for (size_t i = 0; i < src.size(); ++i)
            if (src[i] == '\n') line_starts_.push_back(i + 1);
    }

    void run() {
        int i = 0;
        while (i < n) {
            const Token& k = t[i];
            if (k.kind == Tok::Semi || k.is(';')) { ++i; continue; }
            if (k.ident("package") && i + 1 < n && t[i + 1].ident()) {
                fp_.pkg_name = std::string(t[i + 1].text);
                i += 2;
                continue;
            }
            if (k.ident("import")) { i = parse_import(i + 1); continue; }
            if (k.ident("type")) { i = parse_type_decl(i + 1); continue; }
            if (k.ident("func")) { i = parse_func(i); continue; }
            if ((k.ident("var") || k.ident("const")) ) { i = skip_decl(i + 1); continue; }
            i = next(i);
        }
    }

private:
    std::string_view src_;
    const std::vector<Token>& t;
    int n;
    const std::string& module_;
    FileParse& fp_;
    std::vector<size_t> line_starts_;

    bool P(int i, char c) const { return i >= 0 && i < n && t[i].is(c); }
    bool I(int i) const { return i >= 0 && i < n && t[i].ident(); }
    bool S(int i) const { return i >= 0 && i < n && (t[i].kind == Tok::Semi || t[i].is(';')); }
    int next(int i) const { return (i < n && t[i].match > i) ? t[i].match + 1 : i + 1; }

    int skip_decl(int i) {
        if (P(i, '(')) return next(i);
        while (i < n && !S(i)) i = next(i);
        return i;
    }

    int parse_import(int i) {
        auto one = [&](int k, int end) {
            std::string alias;
            if (k < end && (I(k) || P(k, '.') || P(k, '_'))) {
                alias = std::string(t[k].text);
                ++k;
            }
            if (k < end && t[k].kind == Tok::String) {
                std::string path(unquote(t[k].text));
                fp_.import_paths.push_back(path);
                if (alias.empty()) {
                    size_t s = path.rfind('/');
                    alias = s == std::string::npos ? path : path.substr(s + 1);
                }
                if (alias != "_" && alias != ".") fp_.alias_to_path[alias] = path;
            }
        };
        if (P(i, '(') && t[i].match > i) {
            int end = t[i].match;
            int k = i + 1;
            while (k < end) {
                int se = k;
                while (se < end && !S(se)) ++se;
                if (se > k) one(k, se);
                k = se + 1;
            }
            return end + 1;
        }
        int se = i;
        while (se < n && !S(se)) ++se;
        one(i, se);
        return se;
    }

    // exprToString (analyzer.go:710-733) over the token range of a type.
    std::string type_string(int b, int e) const {
        if (b >= e) return "";
        const Token& k = t[b];
        if (k.is('*')) return "*" + type_string(b + 1, e);
        if (k.is("...")) return "..." + type_string(b + 1, e);
        if (k.is('[')) {
            int close = k.match;
            if (close < 0 || close >= e) return "*ast.BadExpr";
            return "[]" + type_string(close + 1, e);
        }
        if (k.is('(') && k.match == e - 1) return "*ast.ParenExpr";
        if (k.ident("map") && P(b + 1, '[') && t[b + 1].match > 0) {
            int close = t[b + 1].match;
            return "map[" + type_string(b + 2, close) + "]" + type_string(close + 1, e);
        }
        if (k.ident("chan")) {
            int s = b + 1;
            if (s < n && t[s].is(std::string_view("<-"))) ++s;
            return "chan " + type_string(s, e);
        }
        if (k.is("<-") && I(b + 1) && t[b + 1].text == "chan") return "chan " + type_string(b + 2, e);
        if (k.ident("interface")) return "interface{}";
        if (k.ident("func")) return "func()";
        if (k.ident("struct")) return "*ast.StructType";
        if (k.ident()) {
            if (P(b + 1, '.') && I(b + 2)) {
                if (b + 3 == e) return std::string(k.text) + "." + std::string(t[b + 2].text);
                if (P(b + 3, '[')) return "*ast.IndexExpr";
                return std::string(k.text) + "." + std::string(t[b + 2].text);
            }
            if (b + 1 == e) return std::string(k.text);
            if (P(b + 1, '[')) return "*ast.IndexExpr";
            return std::string(k.text);
        }
        return "*ast.BadExpr";
    }

    // resolveTypePackage, with the alias resolved to an internal import path.
    std::string type_package(int b, int e) const {
        while (b < e && (t[b].is('*') || t[b].is("..."))) ++b;
        if (b < e && t[b].is('[') && t[b].match > b) return type_package(t[b].match + 1, e);
        if (I(b) && P(b + 1, '.') && I(b + 2)) {
            auto it = fp_.alias_to_path.find(std::string(t[b].text));
            if (it != fp_.alias_to_path.end() && starts_with(it->second, module_)) return it->second;
        }
        return "";
    }

    // Splits [b, e) on top-level commas.
    std::vector<std::pair<int, int>> split(int b, int e) const {
        std::vector<std::pair<int, int>> out;
        int seg = b;
        for (int i = b; i < e; ++i) {
            if (t[i].kind == Tok::Semi) continue;
            if ((t[i].is('(') || t[i].is('[') || t[i].is('{')) && t[i].match > i) { i = t[i].match; continue; }
            if (t[i].is(',')) { out.emplace_back(seg, i); seg = i + 1; }
        }
        if (seg < e) out.emplace_back(seg, e);
        // drop virtual semicolons at the edges
        for (auto& p : out) {
            while (p.first < p.second && t[p.first].kind == Tok::Semi) ++p.first;
            while (p.second > p.first && t[p.second - 1].kind == Tok::Semi) --p.second;
        }
        return out;
    }

    // Whether an entry `X ...` names a parameter (vs being a bare type).
    bool entry_is_named(int b, int e) const {
        if (!I(b) || e - b < 2) return false;
        const Token& k = t[b + 1];
        if (k.is('.')) return false;  // pkg.Type
        if (k.is('[')) {
            // `a []int` / `a [4]int` named; `List[int]` generic type
            if (P(b + 2, ']')) return true;
            if (b + 2 < e && (t[b + 2].kind == Tok::Number || t[b + 2].is("..."))) return true;
            return false;
        }
        return true;
    }

    // Go field list semantics (IdentifierList Type | Type), one ParamInfo per name.
    std::vector<GoParam> param_list(int b, int e) const {
        std::vector<GoParam> out;
        auto entries = split(b, e);
        bool any_named = false;
        for (auto& en : entries)
            if (entry_is_named(en.first, en.second)) { any_named = true; break; }
        std::vector<std::string> pending_names;
        for (auto& en : entries) {
            if (en.first >= en.second) continue;
            if (!any_named) {
                GoParam p;
                fill_param(p, en.first, en.second);
                out.push_back(p);
                continue;
            }
            if (entry_is_named(en.first, en.second)) {
                pending_names.emplace_back(t[en.first].text);
                int tb = en.first + 1;
                for (auto& nm : pending_names) {
                    GoParam p;
                    p.name = nm;
                    fill_param(p, tb, en.second);
                    out.push_back(p);
                }
                pending_names.clear();
            } else {
                pending_names.emplace_back(t[en.first].text);  // shares the next type
            }
        }
        return out;
    }

    void fill_param(GoParam& p, int b, int e) const {
        p.type = type_string(b, e);
        p.is_pointer = t[b].is('*');
        p.is_slice = t[b].is('[');
        p.is_variadic = t[b].is("...");
        p.package = type_package(b, e);
    }

    // Result types: one entry per field group (analyzer.go:373-377).
    std::vector<std::string> results(int b, int e) const {
        std::vector<std::string> out;
        if (b >= e) return out;
        if (P(b, '(') && t[b].match == e - 1) {
            auto entries = split(b + 1, e - 1);
            bool any_named = false;
            for (auto& en : entries)
                if (entry_is_named(en.first, en.second)) { any_named = true; break; }
            for (auto& en : entries) {
                if (en.first >= en.second) continue;
                if (!any_named) out.push_back(type_string(en.first, en.second));
                else if (entry_is_named(en.first, en.second)) out.push_back(type_string(en.first + 1, en.second));
            }
            return out;
        }
        out.push_back(type_string(b, e));
        return out;
    }

    // [begin, end) byte range of 1-based line `ln`, trimmed of surrounding blanks.
    bool line_span(int ln, size_t& b, size_t& e) const {
        if (ln < 1 || ln > (int)line_starts_.size()) return false;
        b = line_starts_[ln - 1];
        e = ln < (int)line_starts_.size() ? line_starts_[ln] - 1 : src_.size();
        while (b < e && (src_[b] == ' ' || src_[b] == '\t')) ++b;
        while (e > b && (src_[e - 1] == ' ' || src_[e - 1] == '\t' || src_[e - 1] == '\r')) --e;
        return true;
    }

    // Doc.List[0].Text of the comment group ending on the line above `line`.
    std::string doc_for_line(int line) const {
        size_t b, e;
        int l = line - 1;
        if (!line_span(l, b, e) || b == e) return "";
        std::string_view cur = src_.substr(b, e - b);
        if (starts_with(cur, "//")) {
            int first = l;
            size_t pb, pe;
            while (first - 1 >= 1 && line_span(first - 1, pb, pe) && starts_with(src_.substr(pb, pe - pb), "//")) --first;
            line_span(first, pb, pe);
            std::string_view s = src_.substr(pb, pe - pb);
            if (starts_with(s, "// ")) s.remove_prefix(3);
            return std::string(s);
        }
        if (ends_with(cur, "*/")) {
            size_t open = src_.rfind("/*", e);
            if (open == std::string_view::npos) return "";
            return std::string(src_.substr(open, e - open));
        }
        return "";
    }

    int parse_type_decl(int i) {
        if (P(i, '(') && t[i].match > i) {
            int end = t[i].match;
            int k = i + 1;
            while (k < end) {
                while (k < end && S(k)) ++k;
                if (k >= end) break;
                k = parse_type_spec(k, end);
            }
            return end + 1;
        }
        return parse_type_spec(i, n);
    }

    // Name [TypeParams] [=] Type
    int parse_type_spec(int i, int end) {
        if (!I(i)) {
            while (i < end && !S(i)) i = next(i);
            return i;
        }
        int name_tok = i;
        ++i;
        if (P(i, '[') && t[i].match > i) {
            // type parameters vs array type: `T [N]int` has a Number / `]` next
            if (!(P(i + 1, ']') || (i + 1 < n && t[i + 1].kind == Tok::Number))) i = t[i].match + 1;
        }
        if (P(i, '=')) ++i;
        if (I(i) && t[i].text == "struct" && P(i + 1, '{') && t[i + 1].match > i + 1) {
            GoStruct st;
            st.name = std::string(t[name_tok].text);
            st.file = fp_.file;
            st.line = t[name_tok].line;
            parse_struct_fields(i + 2, t[i + 1].match, st);
            fp_.structs.push_back(std::move(st));
            i = t[i + 1].match + 1;
        } else if (I(i) && t[i].text == "interface" && P(i + 1, '{') && t[i + 1].match > i + 1) {
            GoInterface it;
            it.name = std::string(t[name_tok].text);
            it.file = fp_.file;
            it.line = t[name_tok].line;
            parse_interface(i + 2, t[i + 1].match, it);
            fp_.interfaces.push_back(std::move(it));
            i = t[i + 1].match + 1;
        }
        while (i < end && !S(i)) i = next(i);
        return i;
    }

    void parse_struct_fields(int b, int e, GoStruct& st) {
        int k = b;
        while (k < e) {
            while (k < e && S(k)) ++k;
            if (k >= e) break;
            int le = k;
            while (le < e && !S(le)) le = next(le);
            // trailing tag
            int te = le;
            std::string tag;
            if (te - 1 >= k && t[te - 1].kind == Tok::String) {
                tag = std::string(t[te - 1].text);
                --te;
            }
            bool embedded = P(k, '*') || (I(k) && (te - k == 1 || P(k + 1, '.')));
            if (embedded) {
                GoField f;
                f.type = type_string(k, te);
                f.exported = is_exported_name([&]() {
                    std::string c = f.type;
                    size_t s = c.find_first_not_of("*[]");
                    c = s == std::string::npos ? "" : c.substr(s);
                    size_t d = c.rfind('.');
                    return d == std::string::npos ? c : c.substr(d + 1);
                }());
                f.tag = tag;
                f.package = type_package(k, te);
                st.embedded.push_back(f.type);
                st.fields.push_back(f);
            } else {
                // IdentifierList Type
                std::vector<std::string> names;
                int j = k;
                while (I(j)) {
                    names.emplace_back(t[j].text);
                    if (P(j + 1, ',')) { j += 2; continue; }
                    ++j;
                    break;
                }
                std::string ty = type_string(j, te);
                std::string pkg = type_package(j, te);
                for (auto& nm : names) {
                    GoField f;
                    f.name = nm;
                    f.type = ty;
                    f.exported = is_exported_name(nm);
                    f.tag = tag;
                    f.package = pkg;
                    st.fields.push_back(f);
                }
            }
            k = le;
        }
    }

    void parse_interface(int b, int e, GoInterface& it) {
        int k = b;
        while (k < e) {
            while (k < e && S(k)) ++k;
            if (k >= e) break;
            int le = k;
            while (le < e && !S(le)) le = next(le);
            if (I(k) && P(k + 1, '(') && t[k + 1].match > k + 1) {
                GoIfaceMethod m;
                m.name = std::string(t[k].text);
                m.params = param_list(k + 2, t[k + 1].match);
                it.methods.push_back(m);
            } else if (I(k) && le - k == 1) {
                it.embedded.emplace_back(t[k].text);
            } else if (I(k) && P(k + 1, '.') && I(k + 2) && le - k == 3) {
                it.embedded.push_back(std::string(t[k].text) + "." + std::string(t[k + 2].text));
            }
            k = le;
        }
    }

    void scan_body(int b, int e, GoFunc& f) {
        for (int k = b; k < e; ++k) {
            const Token& tk = t[k];
            if (tk.ident("panic") && P(k + 1, '(') && !(k > 0 && P(k - 1, '.'))) f.has_panic = true;
            if (tk.is('.') && I(k + 1) && P(k + 2, '(') && kHttpRegistration.count(t[k + 1].text)) {
                f.has_http_registration = true;
                route_call(k);
            }
        }
    }

    // `recv.VERB("path", ..., handler)` / `v := recv.Group("prefix")`
    void route_call(int dot) {
        int open = dot + 2, close = t[open].match;
        if (close < 0 || !(open + 1 < close) || t[open + 1].kind != Tok::String) return;
        std::string recv = (dot > 0 && I(dot - 1)) ? std::string(t[dot - 1].text) : "";
        std::string_view verb = t[dot + 1].text;
        std::string path(unquote(t[open + 1].text));
        if (verb == "Group" || verb == "Route") {
            // v := r.Group("/api")  (Route with a closure is not followed)
            if (verb == "Group" && dot >= 3 && (t[dot - 2].is(":=") || t[dot - 2].is('=')) && I(dot - 3))
                fp_.groups.push_back({std::string(t[dot - 3].text), recv, path});
            return;
        }
        auto vit = kRouteVerbs.find(verb);
        if (vit == kRouteVerbs.end()) return;
        std::string method = vit->second;
        if (verb == "Handle" || verb == "HandleFunc") {
            // Go 1.22 ServeMux patterns: "POST /items/{id}"
            size_t sp = path.find(' ');
            if (sp != std::string::npos && sp > 0 && path[0] != '/') {
                method = path.substr(0, sp);
                path = path.substr(sp + 1);
            }
        }
        // last top-level argument = the handler
        int last = -1;
        for (int k = open + 1; k < close; k = next(k))
            if (t[k].is(',')) last = k;
        if (last < 0) return;
        int hb = last + 1, he = close;
        std::string qualifier, handler;
        for (int k = hb; k < he; ++k) {
            if (P(k, '(') || P(k, '{')) return;  // call / closure: no named handler
            if (I(k)) {
                if (k + 1 < he && t[k + 1].is('.')) qualifier = std::string(t[k].text);
                else handler = std::string(t[k].text);
            }
        }
        if (handler.empty() || handler == "func") return;
        fp_.routes.push_back({recv, method, path, qualifier, handler});
    }

    int parse_func(int i) {
        int start = i;
        ++i;  // func
        GoFunc f;
        f.file = fp_.file;
        f.line = t[start].line;
        if (P(i, '(') && t[i].match > i) {  // receiver
            int rb = i + 1, re = t[i].match;
            auto ps = param_list(rb, re);
            if (!ps.empty()) {
                std::string r = ps[0].type;
                if (r == "*ast.IndexExpr" || r == "**ast.IndexExpr") {
                    // generic receiver: bind to the base type name (divergence)
                    int k = rb;
                    if (entry_is_named(rb, re)) ++k;
                    std::string base;
                    bool ptr = false;
                    while (k < re && t[k].is('*')) { ptr = true; ++k; }
                    if (I(k)) base = std::string(t[k].text);
                    r = (ptr ? "*" : "") + base;
                }
                f.receiver = r;
            }
            i = t[i].match + 1;
        }
        if (!I(i)) {  // not a declaration we understand
            while (i < n && !S(i)) i = next(i);
            return i;
        }
        f.name = std::string(t[i].text);
        ++i;
        if (P(i, '[') && t[i].match > i) i = t[i].match + 1;  // type parameters
        if (!P(i, '(') || t[i].match < 0) return i;
        f.params = param_list(i + 1, t[i].match);
        i = t[i].match + 1;
        int rb = i;
        while (i < n && !P(i, '{') && !S(i)) i = next(i);
        f.returns = results(rb, i);
        if (P(i, '{') && t[i].match > i) {
            scan_body(i + 1, t[i].match, f);
            i = t[i].match + 1;
        }
        f.doc = doc_for_line(f.line);
        // detectHTTPHandler (analyzer.go:685-706)
        for (auto& p : f.params) {
            const std::string& ty = p.type;
            if (contains(ty, "http.ResponseWriter") || contains(ty, "http.Request") || contains(ty, "gin.Context") ||
                contains(ty, "echo.Context") || contains(ty, "fiber.Ctx")) {
                f.http_method = "GET";
                break;
            }
        }
        if (f.has_http_registration) fp_.has_http_registration = true;
        fp_.funcs.push_back(std::move(f));
        return i;
    }
};

std::string read_module_path(const std::string& root) {
    std::string data;
    if (!read_file(join_path(root, "go.mod"), data)) return "";
    size_t i = 0;
    while (i < data.size()) {
        size_t e = data.find('\n', i);
        if (e == std::string::npos) e = data.size();
        std::string_view line(data.data() + i, e - i);
        while (!line.empty() && (line.front() == ' ' || line.front() == '\t')) line.remove_prefix(1);
        while (!line.empty() && (line.back() == ' ' || line.back() == '\r' || line.back() == '\t')) line.remove_suffix(1);
        if (starts_with(line, "module ")) {
            line.remove_prefix(7);
            while (!line.empty() && line.front() == ' ') line.remove_prefix(1);
            std::string m(line);
            if (m.size() >= 2 && m.front() == '"' && m.back() == '"') m = m.substr(1, m.size() - 2);
            return m;
        }
        i = e + 1;
    }
    return "";
}

struct DirEntry {
    std::string name;
    bool is_dir;
};

std::vector<DirEntry> go_list_dir(const std::string& dir) {
    std::vector<std::pair<std::string, bool>> raw;
    std::vector<DirEntry> out;
    if (!list_dir(dir, raw)) return out;  // sorted; symlinks are not followed as dirs
    out.reserve(raw.size());
    for (auto& e : raw) out.push_back({std::move(e.first), e.second});
    return out;
}

// filepath.Walk order: a directory's package is discovered when its first
// eligible file is reached; entries are visited in lexical order.
void walk_packages(const std::string& dir, const std::string& rel, std::vector<std::pair<std::string, std::string>>& out,
                   bool is_root) {
    bool recorded = false;
    for (auto& e : go_list_dir(dir)) {
        if (e.is_dir) {
            if (excluded_dir(e.name)) continue;
            walk_packages(join_path(dir, e.name), rel.empty() ? e.name : rel + "/" + e.name, out, false);
        } else if (!recorded && eligible_go_file(e.name)) {
            out.emplace_back(dir, rel);
            recorded = true;
        }
    }
    (void)is_root;
}

void infer_class_type(GoPackage& pa) {
    for (auto& f : pa.functions)
        if (!f.http_method.empty()) { pa.class_type = "CONTROLLER"; return; }
    for (auto& s : pa.structs)
        for (auto& m : s.methods)
            if (!m.http_method.empty()) { pa.class_type = "CONTROLLER"; return; }
    std::string base = pa.dir;
    size_t sl = base.rfind('/');
    if (sl != std::string::npos) base = base.substr(sl + 1);
    std::string dn = to_lower(base);
    struct Row { std::vector<const char*> keys; const char* type; };
    static const Row rows[] = {
        {{"handler", "controller", "api", "transport", "http", "rest", "grpc", "endpoint"}, "CONTROLLER"},
        {{"service", "usecase", "application"}, "SERVICE"},
        {{"repository", "repo", "store", "storage", "dao", "persistence", "database"}, "REPOSITORY"},
        {{"model", "entity", "domain"}, "ENTITY"},
        {{"dto", "request", "response", "payload", "schema"}, "DTO"},
        {{"config", "cfg", "configuration"}, "CONFIGURATION"},
        {{"listener", "consumer", "subscriber", "worker", "queue"}, "LISTENER"},
        {{"util", "utils", "helper", "helpers", "middleware", "interceptor", "pkg"}, "UTILITY"}};
    for (auto& r : rows)
        for (auto* k : r.keys)
            if (dn.find(k) != std::string::npos) { pa.class_type = r.type; return; }
    pa.class_type = "OTHER";
}

void analyze_package(const std::string& root, const std::string& dir, const std::string& rel, const std::string& module,
                     GoPackage& pa) {
    pa.dir = rel;
    pa.path = rel.empty() ? module : module + "/" + rel;
    std::vector<FileParse> parses;
    std::vector<std::string> sources;
    for (auto& e : go_list_dir(dir)) {
        if (e.is_dir || !eligible_go_file(e.name)) continue;
        std::string src;
        if (!read_file(join_path(dir, e.name), src)) continue;
        sources.push_back(std::move(src));
        FileParse fp;
        fp.file = e.name;
        CLexOptions opt;
        opt.go = true;
        std::vector<Token> toks = lex_c_family(sources.back(), opt);
        GoFileParser(sources.back(), toks, module, fp).run();
        parses.push_back(std::move(fp));
    }
    (void)root;
    if (parses.empty()) return;
    // First package wins (the reference takes an arbitrary map entry).
    pa.pkg_name = parses[0].pkg_name;
    std::set<std::string> imports;
    std::vector<GoFunc> all_funcs;
    bool http_reg = false;
    for (auto& fp : parses) {
        if (fp.pkg_name != pa.pkg_name) continue;
        pa.files.push_back(fp.file);
        for (auto& p : fp.import_paths)
            if (!module.empty() && starts_with(p, module)) imports.insert(p);
        for (auto& s : fp.structs) pa.structs.push_back(std::move(s));
        for (auto& it : fp.interfaces) pa.interfaces.push_back(std::move(it));
        for (auto& f : fp.funcs) all_funcs.push_back(std::move(f));
        http_reg = http_reg || fp.has_http_registration;
        // group prefixes are file-local variables: v1 := r.Group("/v1"); v1.GET(...)
        std::unordered_map<std::string, const GoGroup*> groups;
        for (auto& g : fp.groups) groups[g.var] = &g;
        for (auto& r : fp.routes) {
            GoRoute rr = r;
            std::string var = r.recv;
            for (int depth = 0; depth < 16; ++depth) {
                auto it = groups.find(var);
                if (it == groups.end()) break;
                rr.path = join_route(it->second->prefix, rr.path);
                if (it->second->parent == var) break;
                var = it->second->parent;
            }
            pa.routes.push_back(std::move(rr));
        }
    }
    pa.imports.assign(imports.begin(), imports.end());
    // bindMethodsToStructs
    std::unordered_map<std::string, size_t> by_name;
    for (size_t k = 0; k < pa.structs.size(); ++k) by_name[pa.structs[k].name] = k;
    for (auto& f : all_funcs) {
        if (!f.receiver.empty()) {
            std::string r = f.receiver;
            if (!r.empty() && r[0] == '*') r = r.substr(1);
            auto it = by_name.find(r);
            if (it != by_name.end()) {
                pa.structs[it->second].methods.push_back(f);
                continue;
            }
        }
        pa.functions.push_back(f);
    }
    // detectEntryPoint
    if (pa.pkg_name == "main")
        for (auto& f : pa.functions)
            if (f.name == "main" && f.receiver.empty()) pa.entry_point = true;
    if (http_reg) pa.entry_point = true;
    infer_class_type(pa);
    pa.ok = true;
}

void write_param(JsonWriter& w, const GoParam& p) {
    w.begin_obj();
    w.kv("name", p.name);
    w.kv("type", p.type);
    if (!p.package.empty()) w.kv("package", p.package);
    if (p.is_pointer) w.kv("isPointer", true);
    if (p.is_slice) w.kv("isSlice", true);
    if (p.is_variadic) w.kv("isVariadic", true);
    w.end_obj();
}

void write_params(JsonWriter& w, const char* key, const std::vector<GoParam>& ps) {
    w.key(key);
    if (ps.empty()) { w.value_null(); return; }
    w.begin_arr();
    for (auto& p : ps) write_param(w, p);
    w.end_arr();
}

void write_strs(JsonWriter& w, const char* key, const std::vector<std::string>& v) {
    w.key(key);
    if (v.empty()) { w.value_null(); return; }
    w.begin_arr();
    for (auto& s : v) w.value_str(s);
    w.end_arr();
}

void write_func(JsonWriter& w, const GoFunc& f) {
    w.begin_obj();
    w.kv("name", f.name);
    w.kv("file", f.file);
    w.kv_int("line", f.line);
    if (!f.receiver.empty()) w.kv("receiver", f.receiver);
    write_params(w, "params", f.params);
    write_strs(w, "returns", f.returns);
    if (!f.http_method.empty()) w.kv("httpMethod", f.http_method);
    if (!f.http_path.empty()) w.kv("httpPath", f.http_path);
    if (f.has_panic) w.kv("hasPanic", true);
    if (!f.doc.empty()) w.kv("doc", f.doc);
    w.end_obj();
}

// Every struct's implemented interfaces (those whose whole method set it
// has), in the order the reference lists them (packages, then interfaces in
// declaration order).  Candidates come from an index of each interface's
// smallest method name -- an interface whose methods a struct all has has
// that one too -- instead of testing every (struct, interface) pair: at 1,000
// packages of similar services that product was ~10^6 set comparisons on one
// thread, most of the Go scan.  Structs are then matched in parallel.
void compute_implements(std::vector<GoPackage>& pkgs, int threads) {
    struct IfaceRef { std::string qname; std::set<std::string> methods; std::string pkg; };
    std::vector<IfaceRef> ifaces;
    for (auto& p : pkgs)
        for (auto& it : p.interfaces) {
            if (it.methods.empty()) continue;
            IfaceRef r;
            r.pkg = p.path;
            r.qname = it.name;
            for (auto& m : it.methods) r.methods.insert(m.name);
            ifaces.push_back(std::move(r));
        }
    std::unordered_map<std::string, std::vector<size_t>> by_first;
    for (size_t k = 0; k < ifaces.size(); ++k) by_first[*ifaces[k].methods.begin()].push_back(k);
    parallel_for(pkgs.size(), threads, [&](size_t pi) {
        GoPackage& p = pkgs[pi];
        for (auto& s : p.structs) {
            std::set<std::string> have;
            for (auto& m : s.methods) have.insert(m.name);
            std::vector<size_t> cand;
            for (auto& name : have) {
                auto it = by_first.find(name);
                if (it == by_first.end()) continue;
                for (size_t k : it->second)
                    if (std::includes(have.begin(), have.end(), ifaces[k].methods.begin(), ifaces[k].methods.end()))
                        cand.push_back(k);
            }
            std::sort(cand.begin(), cand.end());
            for (size_t k : cand) {
                const IfaceRef& r = ifaces[k];
                s.implements.push_back(r.pkg == p.path ? r.qname : r.pkg + "." + r.qname);
            }
        }
    });
}

}  // namespace

// Analyzes a Go module and renders the go-analyzer ProjectAnalysis JSON.
struct GoProject {
    std::string module;
    std::vector<GoPackage> packages;
};

// Gives detected handlers (functions with a ResponseWriter / gin.Context /
// echo.Context / fiber.Ctx parameter) the verb and literal path of the route
// that registers them.  Candidates are matched by handler name; when several
// routes share a name, the qualifier (`handler.List`, `userHandler.List`) must
// match the package name or the receiver type.  Ambiguous handlers keep the
// reference's ("GET", no path).
static void bind_routes(std::vector<GoPackage>& pkgs) {
    std::unordered_map<std::string, std::vector<const GoRoute*>> by_name;
    for (auto& p : pkgs)
        for (auto& r : p.routes) by_name[r.handler].push_back(&r);
    if (by_name.empty()) return;
    auto bind = [&](GoFunc& f, const GoPackage& p) {
        if (f.http_method.empty()) return;
        auto it = by_name.find(f.name);
        if (it == by_name.end()) return;
        std::string recv = to_lower(!f.receiver.empty() && f.receiver[0] == '*' ? f.receiver.substr(1) : f.receiver);
        std::vector<const GoRoute*> c = it->second;
        if (c.size() > 1) {
            std::vector<const GoRoute*> keep;
            for (auto* r : c) {
                std::string q = to_lower(r->qualifier);
                if (q.empty()) continue;
                if (q == to_lower(p.pkg_name) || (!recv.empty() && (q == recv || recv.find(q) != std::string::npos ||
                                                                    q.find(recv) != std::string::npos)))
                    keep.push_back(r);
            }
            c.swap(keep);
        }
        if (c.empty()) return;
        for (auto* r : c)  // all candidates must agree
            if (r->method != c[0]->method || r->path != c[0]->path) return;
        f.http_method = c[0]->method;
        f.http_path = c[0]->path;
    };
    for (auto& p : pkgs) {
        for (auto& f : p.functions) bind(f, p);
        for (auto& s : p.structs)
            for (auto& m : s.methods) bind(m, p);
    }
}

static GoProject analyze_go(const std::string& root, int threads) {
    using clk = std::chrono::steady_clock;
    static const bool timing = std::getenv("DMCP_GO_TIMING") != nullptr;
    const auto t0 = clk::now();
    GoProject gp;
    gp.module = read_module_path(root);
    std::vector<std::pair<std::string, std::string>> dirs;
    walk_packages(root, "", dirs, true);
    const auto t1 = clk::now();
    std::vector<GoPackage> pkgs(dirs.size());
    parallel_for(dirs.size(), threads, [&](size_t k) {
        analyze_package(root, dirs[k].first, dirs[k].second, gp.module, pkgs[k]);
    });
    const auto t2 = clk::now();
    for (auto& p : pkgs)
        if (p.ok) gp.packages.push_back(std::move(p));
    compute_implements(gp.packages, threads);
    const auto t3 = clk::now();
    bind_routes(gp.packages);
    const auto t4 = clk::now();
    if (timing) {
        auto us = [](clk::time_point a, clk::time_point b) {
            return (long long)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
        };
        std::fprintf(stderr, "go: walk %lld us, packages %lld us, implements %lld us, routes %lld us\n", us(t0, t1),
                     us(t1, t2), us(t2, t3), us(t3, t4));
    }
    return gp;
}

static void write_go_project(JsonWriter& w, const GoProject& gp) {
    w.begin_obj();
    w.kv("module", gp.module);
    w.key("packages");
    if (gp.packages.empty()) {
        w.value_null();
    } else {
        w.begin_arr();
        for (auto& p : gp.packages) {
            w.begin_obj();
            w.kv("path", p.path);
            w.kv("dir", p.dir);
            write_strs(w, "files", p.files);
            write_strs(w, "imports", p.imports);
            w.key("structs");
            if (p.structs.empty()) w.value_null();
            else {
                w.begin_arr();
                for (auto& s : p.structs) {
                    w.begin_obj();
                    w.kv("name", s.name);
                    w.kv("file", s.file);
                    w.kv_int("line", s.line);
                    w.key("fields");
                    if (s.fields.empty()) w.value_null();
                    else {
                        w.begin_arr();
                        for (auto& f : s.fields) {
                            w.begin_obj();
                            w.kv("name", f.name);
                            w.kv("type", f.type);
                            if (!f.package.empty()) w.kv("package", f.package);
                            w.kv("isExported", f.exported);
                            if (!f.tag.empty()) w.kv("tag", f.tag);
                            w.end_obj();
                        }
                        w.end_arr();
                    }
                    w.key("methods");
                    if (s.methods.empty()) w.value_null();
                    else {
                        w.begin_arr();
                        for (auto& m : s.methods) write_func(w, m);
                        w.end_arr();
                    }
                    write_strs(w, "embeddedTypes", s.embedded);
                    write_strs(w, "implements", s.implements);
                    w.end_obj();
                }
                w.end_arr();
            }
            w.key("interfaces");
            if (p.interfaces.empty()) w.value_null();
            else {
                w.begin_arr();
                for (auto& it : p.interfaces) {
                    w.begin_obj();
                    w.kv("name", it.name);
                    w.kv("file", it.file);
                    w.kv_int("line", it.line);
                    w.key("methods");
                    if (it.methods.empty()) w.value_null();
                    else {
                        w.begin_arr();
                        for (auto& m : it.methods) {
                            w.begin_obj();
                            w.kv("name", m.name);
                            write_params(w, "params", m.params);
                            w.end_obj();
                        }
                        w.end_arr();
                    }
                    write_strs(w, "embeddedInterfaces", it.embedded);
                    w.end_obj();
                }
                w.end_arr();
            }
            w.key("functions");
            if (p.functions.empty()) w.value_null();
            else {
                w.begin_arr();
                for (auto& f : p.functions) write_func(w, f);
                w.end_arr();
            }
            w.kv("isEntryPoint", p.entry_point);
            w.kv("classType", p.class_type);
            w.end_obj();
        }
        w.end_arr();
    }
    w.end_obj();
}

std::string analyze_go_project_json(const std::string& root, int threads) {
    GoProject gp = analyze_go(root, threads);
    JsonWriter w;
    write_go_project(w, gp);
    return w.out;
}

// Converts the package view into per-file records (GoSourceParser.java parity:
// identifier = package path, methods named Receiver.Method, panic -> "panic").
void go_project_files(const std::string& root, int threads, std::string& module, std::vector<FileRec>& files,
                      std::string* go_json) {
    GoProject gp = analyze_go(root, threads);
    module = gp.module;
    if (go_json) {
        const auto t = std::chrono::steady_clock::now();
        JsonWriter w;
        write_go_project(w, gp);
        *go_json = std::move(w.out);
        if (std::getenv("DMCP_GO_TIMING"))
            std::fprintf(stderr, "go: json %lld us\n",
                         (long long)std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::steady_clock::now() - t).count());
    }
    std::unordered_set<std::string> known;
    for (auto& p : gp.packages) known.insert(p.path);
    for (auto& p : gp.packages) {
        for (auto& fname : p.files) {
            FileRec fr;
            fr.rel_path = p.dir.empty() ? fname : p.dir + "/" + fname;
            fr.abs_path = join_path(root, fr.rel_path);
            fr.identifier = p.path;
            fr.class_type = p.class_type;
            fr.entry_point = p.entry_point;
            fr.package_name = p.pkg_name;
            fr.parsed = true;
            for (auto& imp : p.imports)
                if (known.count(imp) && imp != p.path) fr.deps.push_back(imp);
            auto add = [&](const GoFunc& f) {
                if (f.file != fname) return;
                MethodRec m;
                std::string recv = f.receiver;
                if (!recv.empty() && recv[0] == '*') recv = recv.substr(1);
                m.name = recv.empty() ? f.name : recv + "." + f.name;
                m.line = f.line;
                if (!f.http_method.empty()) { m.has_http_method = true; m.http_method = f.http_method; }
                if (!f.http_path.empty()) { m.has_http_path = true; m.http_path = f.http_path; }
                if (f.has_panic) m.exceptions.push_back("panic");
                std::vector<std::string> matched;
                for (auto& prm : f.params)
                    if (!prm.package.empty() && known.count(prm.package)) matched.push_back(prm.package);
                if (!matched.empty()) {
                    bool replaced = false;
                    for (auto& kv : fr.params)
                        if (kv.first == m.name) { kv.second = matched; replaced = true; }
                    if (!replaced) fr.params.emplace_back(m.name, matched);
                }
                fr.methods.push_back(std::move(m));
            };
            for (auto& f : p.functions) add(f);
            for (auto& s : p.structs)
                for (auto& m : s.methods) add(m);
            files.push_back(std::move(fr));
        }
    }
    std::sort(files.begin(), files.end(), [](const FileRec& a, const FileRec& b) { return a.rel_path < b.rel_path; });
}

}  // namespace srcscan
