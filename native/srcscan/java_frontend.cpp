// Java front-end: one lex + one structural pass per compilation unit.
//
// Parity target: analysis/domain/java/JavaSourceParser.java
//   * package / non-wildcard imports, static imports reduced to their class  (:173-189, :539-564)
//   * top-level types only (cu.getTypes()); constructors of classes and records,
//     then the type's own methods, begin line = first annotation/modifier  (:277-371)
//   * entry point: type- or method-level annotation in ENTRY_POINT_ANNOTATIONS (:68-75, :199-223)
//   * class type: first mapped type annotation, else method Kafka/EventListener (:78-88, :236-263)
//   * HTTP verb/path from @Get/Post/Put/Delete/PatchMapping or @RequestMapping (:91-97, :573-611)
//   * parameter type names with generics / varargs / array suffix stripped (:480-500);
//     constructors of records are not parameter-scanned (:415-425)
// Divergences (documented in docs/PARITY.md): annotations are matched on their
// simple name (a fully-qualified @org...RestController also counts), array-valued
// mapping paths take their first element, and a syntax error degrades to a
// best-effort result instead of failing the whole analysis (SourceParser.java:171-179).
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "srcscan.hpp"

namespace srcscan {
namespace {

const std::unordered_set<std::string_view> kEntryPointAnns = {
    "RestController", "Controller", "KafkaListener", "Scheduled", "EventListener", "SpringBootApplication"};

const std::unordered_map<std::string_view, std::string_view> kAnnClassType = {
    {"RestController", "CONTROLLER"}, {"Controller", "CONTROLLER"}, {"Service", "SERVICE"},
    {"Repository", "REPOSITORY"},     {"Configuration", "CONFIGURATION"}, {"Entity", "ENTITY"},
    {"KafkaListener", "LISTENER"},    {"EventListener", "LISTENER"}};

const std::unordered_map<std::string_view, std::string_view> kHttpAnn = {
    {"GetMapping", "GET"}, {"PostMapping", "POST"}, {"PutMapping", "PUT"},
    {"DeleteMapping", "DELETE"}, {"PatchMapping", "PATCH"}};

const std::unordered_set<std::string_view> kModifiers = {
    "public", "protected", "private", "static", "final", "abstract", "synchronized", "native",
    "transient", "volatile", "strictfp", "default", "sealed"};

struct Annotation {
    std::string_view simple;  // last segment of the name
    int lparen = -1, rparen = -1;
};

struct Parser {
    const std::vector<Token>& t;
    int n;
    explicit Parser(const std::vector<Token>& toks) : t(toks), n((int)toks.size()) {}

    bool at(int i, char c) const { return i < n && t[i].is(c); }
    bool ident_at(int i) const { return i < n && t[i].ident(); }
    int after(int i) const {  // index after a bracketed group starting at i (or i+1)
        if (i < n && t[i].match > i) return t[i].match + 1;
        return i + 1;
    }

    // '@' Name(.Name)* [ '(' ... ')' ] -> returns index after the annotation.
    int parse_annotation(int i, Annotation& a) const {
        ++i;  // '@'
        if (!ident_at(i)) return i;
        a.simple = t[i].text;
        ++i;
        while (at(i, '.') && ident_at(i + 1)) {
            a.simple = t[i + 1].text;
            i += 2;
        }
        if (at(i, '(') && t[i].match > i) {
            a.lparen = i;
            a.rparen = t[i].match;
            i = t[i].match + 1;
        }
        return i;
    }

    // Skips a <...> group starting at '<'; returns index after the closing '>'.
    int skip_angles(int i) const {
        int depth = 0;
        for (; i < n; ++i) {
            const Token& k = t[i];
            if (k.is('<')) ++depth;
            else if (k.is('>')) { if (--depth <= 0) return i + 1; }
            else if (k.is('(') || k.is('[') || k.is('{')) { if (k.match > i) i = k.match; }
            else if (k.is(';')) return i;
        }
        return i;
    }

    // Text of tokens [b, e) in a compact, JavaParser-like form.
    std::string text(int b, int e) const {
        std::string s;
        for (int i = b; i < e; ++i) {
            const Token& k = t[i];
            if (!s.empty()) {
                char prev = s.back();
                bool word = k.kind == Tok::Ident || k.kind == Tok::Number || k.kind == Tok::String || k.kind == Tok::Char;
                bool prev_word = is_ident_char((unsigned char)prev) || prev == '"' || prev == '\'';
                if ((word && prev_word) || k.is('+') || prev == '+' || k.is('-') || k.is('*') ||
                    k.is("==") || k.is("!=") || k.is("&&") || k.is("||") || prev == ',' ||
                    (k.is('?') ) || prev == '?' || k.is(':') || prev == ':')
                    s += ' ';
            }
            s.append(k.text.data(), k.text.size());
        }
        return s;
    }

    // Annotation member value -> string as the reference reports it.
    std::string value_string(int b, int e) const {
        if (e - b == 1 && t[b].kind == Tok::String) return std::string(unquote(t[b].text));
        if (e - b >= 2 && t[b].is('{') && t[b].match == e - 1) {
            // array initializer: first element (divergence: reference prints the array)
            int inner_b = b + 1, inner_e = e - 1;
            int k = inner_b;
            while (k < inner_e && !t[k].is(',')) k = after(k);
            if (k > inner_b) return value_string(inner_b, k);
            return std::string();
        }
        return text(b, e);
    }

    // Finds `name = value` in annotation args; returns value range via out params.
    bool ann_pair(const Annotation& a, std::string_view name, int& vb, int& ve) const {
        if (a.lparen < 0) return false;
        int i = a.lparen + 1, end = a.rparen;
        while (i < end) {
            int seg_b = i;
            while (i < end && !t[i].is(',')) i = after(i);
            int seg_e = i;
            if (seg_e - seg_b >= 3 && t[seg_b].ident() && t[seg_b + 1].is('=')) {
                if (t[seg_b].text == name) { vb = seg_b + 2; ve = seg_e; return true; }
            }
            ++i;
        }
        return false;
    }

    bool ann_is_normal(const Annotation& a) const {
        if (a.lparen < 0) return false;
        int b = a.lparen + 1;
        return a.rparen - b >= 2 && t[b].ident() && t[b + 1].is('=');
    }

    // extractAnnotationPath (:573-588)
    bool ann_path(const Annotation& a, std::string& out) const {
        if (a.lparen < 0) return false;  // marker annotation
        if (a.rparen == a.lparen + 1) return false;
        if (!ann_is_normal(a)) {
            out = value_string(a.lparen + 1, a.rparen);
            return true;
        }
        int vb, ve;
        // first pair named value or path, in source order
        int i = a.lparen + 1, end = a.rparen;
        while (i < end) {
            int seg_b = i;
            while (i < end && !t[i].is(',')) i = after(i);
            int seg_e = i;
            if (seg_e - seg_b >= 3 && t[seg_b].ident() && t[seg_b + 1].is('=') &&
                (t[seg_b].text == "value" || t[seg_b].text == "path")) {
                vb = seg_b + 2;
                ve = seg_e;
                out = value_string(vb, ve);
                return true;
            }
            ++i;
        }
        return false;
    }

    // extractRequestMappingMethod (:596-611)
    std::string request_mapping_method(const Annotation& a) const {
        if (!ann_is_normal(a)) return "GET";
        int vb, ve;
        if (!ann_pair(a, "method", vb, ve)) return "GET";
        if (ve - vb >= 2 && t[vb].is('{') && t[vb].match == ve - 1) {
            // array: first element
            int k = vb + 1;
            while (k < ve - 1 && !t[k].is(',')) k = after(k);
            vb = vb + 1;
            ve = k;
        }
        // last identifier segment
        for (int k = ve - 1; k >= vb; --k)
            if (t[k].ident()) return std::string(t[k].text);
        return "GET";
    }

    // Splits [b, e) on top-level commas honouring <> nesting.
    std::vector<std::pair<int, int>> split_params(int b, int e) const {
        std::vector<std::pair<int, int>> out;
        int depth = 0, seg = b;
        for (int i = b; i < e; ++i) {
            const Token& k = t[i];
            if (k.is('<')) ++depth;
            else if (k.is('>')) { if (depth > 0) --depth; }
            else if ((k.is('(') || k.is('[') || k.is('{')) && k.match > i) { i = k.match; continue; }
            else if (k.is(',') && depth == 0) { out.emplace_back(seg, i); seg = i + 1; }
        }
        if (seg < e) out.emplace_back(seg, e);
        return out;
    }

    // One parameter declaration -> its type as written (JavaParser getTypeAsString-ish).
    std::string param_type(int b, int e) const {
        int i = b;
        while (i < e) {
            if (t[i].is('@')) { Annotation a; i = parse_annotation(i, a); continue; }
            if (t[i].ident("final")) { ++i; continue; }
            break;
        }
        // trailing name (and optional C-style dims after it)
        int end = e;
        while (end - 2 >= i && t[end - 1].is(']') && t[end - 2].is('[')) end -= 2;
        if (end - 1 > i && t[end - 1].ident()) --end;  // the parameter name
        std::string s;
        for (int k = i; k < end; ++k) {
            if (t[k].is('@')) { Annotation a; k = parse_annotation(k, a) - 1; continue; }
            if (!s.empty() && t[k].ident() && (is_ident_char((unsigned char)s.back()))) s += ' ';
            s.append(t[k].text.data(), t[k].text.size());
        }
        return s;
    }

    static std::string simple_type_name(std::string s) {
        size_t g = s.find('<');
        if (g != std::string::npos && g > 0) s = s.substr(0, g);
        if (ends_with(s, "...")) s = s.substr(0, s.size() - 3);
        if (ends_with(s, "[]")) s = s.substr(0, s.size() - 2);
        // trim
        while (!s.empty() && s.back() == ' ') s.pop_back();
        return s;
    }

    // Throws list [b, e) -> type strings
    std::vector<std::string> throws_list(int b, int e) const {
        std::vector<std::string> out;
        for (auto& seg : split_params(b, e)) {
            std::string s;
            for (int k = seg.first; k < seg.second; ++k) {
                if (t[k].is('@')) { Annotation a; k = parse_annotation(k, a) - 1; continue; }
                if (t[k].is(',')) s += ", ";
                else s.append(t[k].text.data(), t[k].text.size());
            }
            if (!s.empty()) out.push_back(s);
        }
        return out;
    }

    struct TypeDecl {
        std::string_view kind;  // class | interface | enum | record | annotation
        std::string_view name;
        std::vector<Annotation> anns;
        int body_b = -1, body_e = -1;
        int end = -1;  // index after the declaration
    };

    // Parses a type declaration whose kind keyword is at i (annotations already collected).
    bool parse_type_header(int i, TypeDecl& d) {
        if (at(i, '@') && i + 1 < n && t[i + 1].ident("interface")) {
            d.kind = "annotation";
            i += 2;
        } else if (ident_at(i) && (t[i].text == "class" || t[i].text == "interface" ||
                                   t[i].text == "enum" || t[i].text == "record")) {
            d.kind = t[i].text;
            ++i;
        } else {
            return false;
        }
        if (!ident_at(i)) return false;
        d.name = t[i].text;
        ++i;
        // header until body: skip <...>, (...) record components, extends/implements lists
        while (i < n && !t[i].is('{')) {
            if (t[i].is('<')) { i = skip_angles(i); continue; }
            if ((t[i].is('(') || t[i].is('[')) && t[i].match > i) { i = t[i].match + 1; continue; }
            if (t[i].is(';')) return false;
            ++i;
        }
        if (i >= n || t[i].match < 0) return false;
        d.body_b = i + 1;
        d.body_e = t[i].match;
        d.end = t[i].match + 1;
        return true;
    }

    bool is_type_keyword_at(int i) const {
        if (at(i, '@') && i + 1 < n && t[i + 1].ident("interface")) return true;
        if (!ident_at(i)) return false;
        std::string_view s = t[i].text;
        if (s == "class" || s == "interface" || s == "enum") return true;
        // 'record' is contextual: record Name ( ...
        if (s == "record" && ident_at(i + 1) && (at(i + 2, '(') || at(i + 2, '<'))) return true;
        return false;
    }

    // Member scan of a top-level type body.
    void parse_members(const TypeDecl& d, FileRec& out, bool& listener_method, bool& entry_method) {
        int i = d.body_b, end = d.body_e;
        if (d.kind == "enum") {
            // skip the constant list up to the first top-level ';'
            while (i < end && !t[i].is(';')) i = after(i);
            if (i < end) ++i;
        }
        while (i < end) {
            if (t[i].is(';')) { ++i; continue; }
            int start = i;
            std::vector<Annotation> anns;
            for (;;) {
                if (at(i, '@') && !(i + 1 < n && t[i + 1].ident("interface"))) {
                    Annotation a;
                    i = parse_annotation(i, a);
                    anns.push_back(a);
                    continue;
                }
                if (ident_at(i) && kModifiers.count(t[i].text)) { ++i; continue; }
                if (ident_at(i) && t[i].text == "non" && at(i + 1, '-') && i + 2 < n && t[i + 2].ident("sealed")) {
                    i += 3;
                    continue;
                }
                break;
            }
            if (i >= end) break;
            if (t[i].is('{')) { i = after(i); continue; }  // initializer block
            if (is_type_keyword_at(i)) {                 // nested type: skipped
                TypeDecl nested;
                if (parse_type_header(i, nested)) { i = nested.end; continue; }
                ++i;
                continue;
            }
            if (t[i].is('<')) i = skip_angles(i);  // generic method type parameters
            // find '(' | '=' | ';' | '{' at angle depth 0
            int k = i, depth = 0, found = -1;
            char what = 0;
            while (k < end) {
                const Token& tk = t[k];
                if (tk.is('<')) { ++depth; ++k; continue; }
                if (tk.is('>')) { if (depth > 0) --depth; ++k; continue; }
                if (depth == 0 && (tk.is('(') || tk.is('=') || tk.is(';') || tk.is('{'))) {
                    found = k;
                    what = tk.text[0];
                    break;
                }
                if (tk.is('@')) { Annotation a; k = parse_annotation(k, a); continue; }
                if ((tk.is('[') || tk.is('(')) && tk.match > k) { k = tk.match + 1; continue; }
                ++k;
            }
            if (found < 0) break;
            if (what == '(' && found - 1 >= i && t[found - 1].ident()) {
                bool is_ctor = (found - 1 == i) && t[found - 1].text == d.name;
                int pb = found + 1, pe = t[found].match;
                if (pe < 0) break;
                int j = pe + 1;
                while (at(j, '[') && at(j + 1, ']')) j += 2;
                std::vector<std::string> exceptions;
                if (ident_at(j) && t[j].text == "throws") {
                    int tb = j + 1, te = tb;
                    while (te < end && !t[te].is('{') && !t[te].is(';')) te = after(te);
                    exceptions = throws_list(tb, te);
                    j = te;
                }
                if (ident_at(j) && t[j].text == "default") {  // annotation member default
                    while (j < end && !t[j].is(';')) j = after(j);
                }
                if (at(j, '{')) j = after(j);
                else if (at(j, ';')) ++j;
                bool record_it = d.kind != "annotation" &&
                                 (!is_ctor || d.kind == "class" || d.kind == "record");
                if (is_ctor && d.kind == "interface") record_it = false;
                if (record_it) {
                    MethodRec m;
                    m.name = std::string(t[found - 1].text);
                    m.line = t[start].line;
                    m.is_ctor = is_ctor;
                    m.params_eligible = !(is_ctor && d.kind == "record");
                    m.exceptions = std::move(exceptions);
                    if (!is_ctor) {
                        for (auto& a : anns) {
                            auto it = kHttpAnn.find(a.simple);
                            if (it != kHttpAnn.end()) {
                                m.has_http_method = true;
                                m.http_method = std::string(it->second);
                                m.has_http_path = ann_path(a, m.http_path);
                                break;
                            }
                            if (a.simple == "RequestMapping") {
                                m.has_http_method = true;
                                m.http_method = request_mapping_method(a);
                                m.has_http_path = ann_path(a, m.http_path);
                                break;
                            }
                        }
                        for (auto& a : anns) {
                            if (kEntryPointAnns.count(a.simple)) entry_method = true;
                            if (a.simple == "KafkaListener" || a.simple == "EventListener") listener_method = true;
                        }
                    }
                    for (auto& seg : split_params(pb, pe)) {
                        std::string ty = simple_type_name(param_type(seg.first, seg.second));
                        m.param_types.push_back(ty);
                    }
                    out.methods.push_back(std::move(m));
                }
                i = j;
                continue;
            }
            // field (or something we do not model): skip to the end of the declaration
            if (what == '{') { i = after(found); continue; }
            k = found;
            while (k < end && !t[k].is(';')) k = after(k);
            i = k + 1;
        }
    }
};

}  // namespace

void analyze_java(std::string_view src, FileRec& out) {
    CLexOptions opt;
    opt.java = true;
    std::vector<Token> toks = lex_c_family(src, opt);
    Parser p(toks);
    int i = 0, n = (int)toks.size();
    bool seen_type = false;
    bool class_type_set = false;
    while (i < n) {
        const Token& tk = toks[i];
        if (tk.is(';')) { ++i; continue; }
        if (!seen_type && tk.ident("package")) {
            int j = i + 1;
            std::string name;
            while (j < n && !toks[j].is(';')) { name.append(toks[j].text.data(), toks[j].text.size()); ++j; }
            out.package_name = name;
            i = j + 1;
            continue;
        }
        if (!seen_type && tk.ident("import")) {
            int j = i + 1;
            ImportRec imp;
            if (j < n && toks[j].ident("static")) { imp.is_static = true; ++j; }
            std::string name;
            while (j < n && !toks[j].is(';')) {
                if (toks[j].is('*')) imp.is_asterisk = true;
                else name.append(toks[j].text.data(), toks[j].text.size());
                ++j;
            }
            if (imp.is_asterisk && !name.empty() && name.back() == '.') name.pop_back();
            imp.imported = name;
            out.imports.push_back(std::move(imp));
            i = j + 1;
            continue;
        }
        // top-level type with annotations / modifiers
        int j = i;
        std::vector<Annotation> anns;
        for (;;) {
            if (p.at(j, '@') && !(j + 1 < n && toks[j + 1].ident("interface"))) {
                Annotation a;
                j = p.parse_annotation(j, a);
                anns.push_back(a);
                continue;
            }
            if (p.ident_at(j) && kModifiers.count(toks[j].text)) { ++j; continue; }
            if (p.ident_at(j) && toks[j].text == "non" && p.at(j + 1, '-')) { j += 3; continue; }
            break;
        }
        Parser::TypeDecl d;
        if (p.is_type_keyword_at(j) && p.parse_type_header(j, d)) {
            seen_type = true;
            d.anns = anns;
            bool listener_method = false, entry_method = false;
            p.parse_members(d, out, listener_method, entry_method);
            for (auto& a : anns)
                if (kEntryPointAnns.count(a.simple)) out.entry_point = true;
            if (entry_method) out.entry_point = true;
            if (!class_type_set) {
                for (auto& a : anns) {
                    auto it = kAnnClassType.find(a.simple);
                    if (it != kAnnClassType.end()) {
                        out.class_type = std::string(it->second);
                        class_type_set = true;
                        break;
                    }
                }
                if (!class_type_set && listener_method) {
                    out.class_type = "LISTENER";
                    class_type_set = true;
                }
            }
            i = d.end;
            continue;
        }
        i = j > i ? j : i + 1;
    }
    out.parsed = true;
}

}  // namespace srcscan
