// TypeScript / JavaScript front-end.
//
// Parity target: src/main/resources/js/analyzer/src/extractor.ts (Babel visitors)
// and detector.ts.  The reference runs Babel inside GraalJS once per file
// (NodeJsGraalParser.java:150-174); here a context-aware lexer (regex vs
// division, template literals, JSX) feeds a structural scanner that emits the
// same facts the Babel visitors collect:
//   ImportDeclaration specifiers (named / default / namespace)      extractor.ts:67-93
//   ClassDeclaration decorators -> class type / entry point, class
//     methods and arrow-valued class properties (no constructors)    :96-127, :339-394
//   FunctionDeclaration (any depth)                                   :130-150
//   exported `const x = () => ...` / function expressions            :153-190
//   non-exported variable declarators incl. wrapper calls             :197-229, :471-493
//   object-literal arrow properties and shorthand methods             :233-271
//   Express `app|router.<verb>(` registrations                        :274-298
//   NestJS @Get/@Post/... only for framework 'nestjs'                 :361-366, :396-431
//   Next.js App Router route handlers                                 :495-520
//   parameter types = TSTypeReference identifiers only                :433-460
//   filename class-type table / well-known entry files                :522-553
// Methods are emitted in Babel pre-order (a class's members at class entry).
#include <algorithm>
#include <string>
#include <unordered_set>

#include "srcscan.hpp"

namespace srcscan {
namespace {

// ===================================================================== lexer
const char* kTsPunct[] = {">>>=", "...", "===", "!==", "**=", "<<=", ">>=", "&&=", "||=", "??=",
                          "=>",   "?.",  "??",  "==",  "!=",  "<=",  ">=",  "&&",  "||",  "++",
                          "--",   "+=",  "-=",  "*=",  "/=",  "%=",  "&=",  "|=",  "^=",  "**",
                          "<<",   nullptr};

const std::unordered_set<std::string_view> kExprKeywords = {
    "return", "typeof", "instanceof", "in", "of", "new", "delete", "void", "throw", "case",
    "do", "else", "yield", "await", "extends", "default", "export"};

class TsLexer {
public:
    TsLexer(std::string_view s, bool jsx) : src(s), n(s.size()), jsx_(jsx) {}
    std::vector<Token> toks;

    void run() {
        if (n >= 2 && src[0] == '#' && src[1] == '!')
            while (i < n && src[i] != '\n') ++i;
        lex_js(false);
        match_brackets(toks);
    }

private:
    std::string_view src;
    size_t n, i = 0;
    int line = 1;
    bool nl = false;
    bool jsx_;

    void push(Tok k, size_t b, size_t e, int ln) {
        Token t{k, src.substr(b, e - b), ln};
        t.nl_before = nl;
        nl = false;
        toks.push_back(t);
    }

    // Is the next token in expression-start position (regex / JSX allowed)?
    bool expr_start() const {
        if (toks.empty()) return true;
        const Token& p = toks.back();
        switch (p.kind) {
            case Tok::Ident: return kExprKeywords.count(p.text) > 0;
            case Tok::Number:
            case Tok::String:
            case Tok::Template:
            case Tok::Regex: return false;
            case Tok::JsxText: return false;
            case Tok::Punct: return !(p.text == ")" || p.text == "]" || p.text == "}");
            default: return true;
        }
    }

    void skip_ws_comments() {
        while (i < n) {
            char c = src[i];
            if (c == '\n') { ++line; nl = true; ++i; continue; }
            if (c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v') { ++i; continue; }
            if (c == '/' && i + 1 < n && src[i + 1] == '/') {
                while (i < n && src[i] != '\n') ++i;
                continue;
            }
            if (c == '/' && i + 1 < n && src[i + 1] == '*') {
                i += 2;
                while (i < n && !(src[i] == '*' && i + 1 < n && src[i + 1] == '/')) {
                    if (src[i] == '\n') { ++line; nl = true; }
                    ++i;
                }
                i = std::min(n, i + 2);
                continue;
            }
            break;
        }
    }

    void lex_string(char q) {
        size_t b = i++;
        int ln = line;
        while (i < n && src[i] != q) {
            if (src[i] == '\\' && i + 1 < n) {
                if (src[i + 1] == '\n') ++line;
                ++i;
            } else if (src[i] == '\n') {
                break;  // unterminated
            }
            ++i;
        }
        if (i < n && src[i] == q) ++i;
        push(Tok::String, b, i, ln);
    }

    // Template literal starting at a backtick; substitutions are lexed as JS.
    void lex_template() {
        size_t b = i++;
        int ln = line;
        for (;;) {
            while (i < n && src[i] != '`' && !(src[i] == '$' && i + 1 < n && src[i + 1] == '{')) {
                if (src[i] == '\\' && i + 1 < n) ++i;
                if (src[i] == '\n') ++line;
                ++i;
            }
            if (i >= n) { push(Tok::Template, b, i, ln); return; }
            if (src[i] == '`') { ++i; push(Tok::Template, b, i, ln); return; }
            // ${
            push(Tok::Template, b, i, ln);
            ++i;  // '$'
            push(Tok::Punct, i, i + 1, line);  // '{'
            ++i;
            lex_js(true);
            b = i;
            ln = line;
        }
    }

    bool lex_regex() {
        size_t b = i++;
        bool in_class = false;
        while (i < n) {
            char c = src[i];
            if (c == '\n') { i = b; return false; }
            if (c == '\\') { i += 2; continue; }
            if (c == '[') in_class = true;
            else if (c == ']') in_class = false;
            else if (c == '/' && !in_class) break;
            ++i;
        }
        if (i >= n) { i = b; return false; }
        ++i;
        while (i < n && is_ident_char((unsigned char)src[i])) ++i;
        push(Tok::Regex, b, i, line);
        return true;
    }

    // JSX element at '<' (expression position). Attribute values and
    // children expressions are lexed as JS; text and tags become JsxText.
    void lex_jsx_element() {
        size_t b = i;
        int ln = line;
        ++i;  // '<'
        auto tag_chars = [&]() {
            while (i < n && (is_ident_char((unsigned char)src[i]) || src[i] == '.' || src[i] == ':' || src[i] == '-')) ++i;
        };
        tag_chars();
        // attributes
        for (;;) {
            while (i < n && (src[i] == ' ' || src[i] == '\t' || src[i] == '\r' || src[i] == '\n')) {
                if (src[i] == '\n') ++line;
                ++i;
            }
            if (i >= n) return;
            char c = src[i];
            if (c == '/' && i + 1 < n && src[i + 1] == '>') {
                i += 2;
                push(Tok::JsxText, b, i, ln);
                return;
            }
            if (c == '>') { ++i; break; }
            if (c == '{') {
                push(Tok::JsxText, b, i, ln);
                push(Tok::Punct, i, i + 1, line);
                ++i;
                lex_js(true);
                b = i;
                ln = line;
                continue;
            }
            if (c == '"' || c == '\'') {
                char q = c;
                ++i;
                while (i < n && src[i] != q) { if (src[i] == '\n') ++line; ++i; }
                if (i < n) ++i;
                continue;
            }
            if (c == '/' && i + 1 < n && (src[i + 1] == '/' || src[i + 1] == '*')) {
                push(Tok::JsxText, b, i, ln);
                skip_ws_comments();
                b = i;
                ln = line;
                continue;
            }
            ++i;  // attribute name chars, '='
        }
        push(Tok::JsxText, b, i, ln);
        // children
        b = i;
        ln = line;
        for (;;) {
            while (i < n && src[i] != '<' && src[i] != '{') {
                if (src[i] == '\n') ++line;
                ++i;
            }
            if (i >= n) { push(Tok::JsxText, b, i, ln); return; }
            if (src[i] == '{') {
                push(Tok::JsxText, b, i, ln);
                push(Tok::Punct, i, i + 1, line);
                ++i;
                lex_js(true);
                b = i;
                ln = line;
                continue;
            }
            // '<'
            if (i + 1 < n && src[i + 1] == '/') {  // closing tag
                while (i < n && src[i] != '>') { if (src[i] == '\n') ++line; ++i; }
                if (i < n) ++i;
                push(Tok::JsxText, b, i, ln);
                return;
            }
            push(Tok::JsxText, b, i, ln);
            lex_jsx_element();
            b = i;
            ln = line;
        }
    }

    // Lexes JS tokens; with stop_on_close, returns after the '}' that closes
    // the enclosing substitution / expression container.
    void lex_js(bool stop_on_close) {
        int depth = 0;
        while (true) {
            skip_ws_comments();
            if (i >= n) return;
            unsigned char c = src[i];
            int ln = line;
            if (c == '"' || c == '\'') { lex_string((char)c); continue; }
            if (c == '`') { lex_template(); continue; }
            if (is_ident_start(c) || c == '#' || c == '\\') {
                size_t b = i++;
                while (i < n && (is_ident_char((unsigned char)src[i]) || src[i] == '\\')) ++i;
                push(Tok::Ident, b, i, ln);
                continue;
            }
            if ((c >= '0' && c <= '9') || (c == '.' && i + 1 < n && src[i + 1] >= '0' && src[i + 1] <= '9')) {
                size_t b = i++;
                while (i < n) {
                    char d = src[i];
                    if (is_ident_char((unsigned char)d) || d == '.') { ++i; continue; }
                    if ((d == '+' || d == '-') && (src[i - 1] == 'e' || src[i - 1] == 'E') &&
                        !(src[b] == '0' && b + 1 < n && (src[b + 1] == 'x' || src[b + 1] == 'X'))) {
                        ++i;
                        continue;
                    }
                    break;
                }
                push(Tok::Number, b, i, ln);
                continue;
            }
            if (c == '/' && expr_start()) {
                if (lex_regex()) continue;
            }
            if (c == '<' && jsx_ && expr_start() && i + 1 < n &&
                (is_ident_start((unsigned char)src[i + 1]) || src[i + 1] == '>')) {
                lex_jsx_element();
                continue;
            }
            if (c == '{') { ++depth; push(Tok::Punct, i, i + 1, ln); ++i; continue; }
            if (c == '}') {
                push(Tok::Punct, i, i + 1, ln);
                ++i;
                if (depth == 0 && stop_on_close) return;
                if (depth > 0) --depth;
                continue;
            }
            if (c == '?' && i + 1 < n && src[i + 1] == '.' && i + 2 < n && src[i + 2] >= '0' && src[i + 2] <= '9') {
                push(Tok::Punct, i, i + 1, ln);
                ++i;
                continue;
            }
            bool matched = false;
            for (const char** p = kTsPunct; *p; ++p) {
                size_t len = std::strlen(*p);
                if (i + len <= n && src.compare(i, len, *p) == 0) {
                    push(Tok::Punct, i, i + len, ln);
                    i += len;
                    matched = true;
                    break;
                }
            }
            if (matched) continue;
            push(Tok::Punct, i, i + 1, ln);
            ++i;
        }
    }
};

// =================================================================== scanner
const std::unordered_set<std::string_view> kTsKeywordTypes = {
    "string", "number", "boolean", "any", "void", "unknown", "never", "object", "undefined",
    "null", "bigint", "symbol", "this", "true", "false"};

const std::unordered_set<std::string_view> kStmtKeywords = {
    "const", "let", "var", "function", "class", "if", "for", "while", "do", "return", "switch",
    "try", "throw", "break", "continue", "import", "export", "interface", "type", "enum",
    "namespace", "module", "declare", "abstract", "async"};

const std::unordered_set<std::string_view> kMemberModifiers = {
    "public", "private", "protected", "static", "readonly", "abstract", "declare", "override",
    "accessor"};

const std::unordered_set<std::string_view> kNextMethods = {"GET", "POST", "PUT", "DELETE",
                                                           "PATCH", "HEAD", "OPTIONS"};

struct Decorator {
    std::string_view name;  // empty when the callee is not a plain identifier
    bool is_call = false;
    int lparen = -1, rparen = -1;
    int line = 0;
};

struct FuncShape {
    int params_b = -1, params_e = -1;  // parameter token range (exclusive of parens)
    int body_b = -1, body_e = -1;      // body range ('{' .. '}' exclusive) or expression range
    bool block = false;
    int end = -1;                      // index after the function expression
};

class TsScanner {
public:
    TsScanner(const std::vector<Token>& toks, const std::string& rel_path, const std::string& framework,
              FileRec& out)
        : t(toks), n((int)toks.size()), path(rel_path), fw(framework), out(out) {}

    void run() {
        scan(0, n, true);
        if (class_type == "OTHER") class_type = class_type_from_filename();
        if (!entry) entry = well_known_entry();
        out.class_type = class_type;
        out.entry_point = entry;
        out.parsed = true;
    }

private:
    const std::vector<Token>& t;
    int n;
    const std::string& path;
    const std::string& fw;
    FileRec& out;
    std::string class_type = "OTHER";
    bool entry = false;
    int guard = 0;

    // ---------------------------------------------------------------- utils
    bool P(int i, char c) const { return i >= 0 && i < n && t[i].is(c); }
    bool P(int i, std::string_view s) const { return i >= 0 && i < n && t[i].kind == Tok::Punct && t[i].text == s; }
    bool I(int i) const { return i >= 0 && i < n && t[i].kind == Tok::Ident; }
    bool I(int i, std::string_view s) const { return i >= 0 && i < n && t[i].kind == Tok::Ident && t[i].text == s; }
    int after_group(int i) const { return (i < n && t[i].match > i) ? t[i].match + 1 : i + 1; }

    // Does a token at i (given the previous token) start an expression?
    bool expression_context(int i) const {
        if (i <= 0) return false;
        const Token& p = t[i - 1];
        if (p.kind == Tok::Ident) {
            static const std::unordered_set<std::string_view> kw = {
                "return", "yield", "await", "typeof", "void", "delete", "new", "case", "in",
                "of", "instanceof", "throw", "extends"};
            return kw.count(p.text) > 0;
        }
        if (p.kind == Tok::Punct) {
            if (p.text == ")" || p.text == "]" || p.text == "}" || p.text == ";") return false;
            return true;  // operators, '(', '[', ',', '=', ':', '?', '{'...
        }
        if (p.kind == Tok::JsxText) return true;
        return false;
    }

    // Skips a TS type starting at i; stops before a depth-0 token for which
    // stop(i) is true. `brace_ends` makes a '{' that follows a complete type
    // terminate it (function bodies after return types).
    template <class Stop>
    int skip_type(int i, int end, Stop stop, bool brace_ends) const {
        int angle = 0;
        bool expect_type = true;  // at a position where a type may start
        while (i < end) {
            const Token& k = t[i];
            if (angle == 0 && stop(i)) return i;
            if (k.kind == Tok::Punct) {
                std::string_view s = k.text;
                if (s == "<") { ++angle; expect_type = true; ++i; continue; }
                if (s == ">" ) { if (angle > 0) --angle; expect_type = false; ++i; continue; }
                if (s == ">=") { if (angle > 0) { --angle; ++i; continue; } return i; }
                if (s == "{") {
                    if (angle == 0 && brace_ends && !expect_type) return i;
                    i = after_group(i);
                    expect_type = false;
                    continue;
                }
                if (s == "(" || s == "[") { i = after_group(i); expect_type = false; continue; }
                if (s == ";" && angle == 0) return i;
                if (s == ")" || s == "]" || s == "}") return i;  // closing of an enclosing group
                expect_type = (s == "|" || s == "&" || s == "," || s == "=>" || s == ":" || s == "?" ||
                               s == "." || s == "...");
                ++i;
                continue;
            }
            if (k.kind == Tok::Ident) {
                if (angle == 0 && k.nl_before && !expect_type) return i;  // ASI
                expect_type = (k.text == "keyof" || k.text == "typeof" || k.text == "readonly" ||
                               k.text == "infer" || k.text == "extends" || k.text == "is" ||
                               k.text == "asserts" || k.text == "unique" || k.text == "new");
                ++i;
                continue;
            }
            expect_type = false;
            ++i;
        }
        return i;
    }

    // Returns the index of the token after the end of an expression that
    // starts at i (stops at ',' ';' or an ASI boundary at depth 0).
    int expr_end(int i, int end) const {
        int start = i;
        while (i < end) {
            const Token& k = t[i];
            if (k.kind == Tok::Punct) {
                if (k.text == "," || k.text == ";") return i;
                if (k.text == ")" || k.text == "]" || k.text == "}") return i;
                if ((k.text == "(" || k.text == "[" || k.text == "{") && k.match > i) {
                    i = k.match + 1;
                    continue;
                }
            }
            if (i > start && k.nl_before && asi_break(i)) return i;
            ++i;
        }
        return i;
    }

    bool asi_break(int i) const {
        const Token& prev = t[i - 1];
        const Token& k = t[i];
        if (prev.kind == Tok::Punct) {
            std::string_view s = prev.text;
            if (!(s == ")" || s == "]" || s == "}" || s == "++" || s == "--")) return false;
        }
        if (prev.kind == Tok::Ident && kExprKeywords.count(prev.text)) return false;
        if (k.kind == Tok::Punct) {
            std::string_view s = k.text;
            // a continuation operator keeps the expression going
            if (s == "." || s == "?." || s == "?" || s == ":" || s == "=>" || s == "=" || s == "+" ||
                s == "-" || s == "*" || s == "/" || s == "%" || s == "&&" || s == "||" || s == "??" ||
                s == "|" || s == "&" || s == "==" || s == "===" || s == "!=" || s == "!==" ||
                s == "<" || s == ">" || s == "<=" || s == ">=" || s == "," || s == ")" || s == "]" ||
                s == "}" || s == "(" || s == "[" || s == "**" || s == "<<" || s == "+=" || s == "-=")
                return false;
            return true;
        }
        if (k.kind == Tok::Ident && (k.text == "as" || k.text == "satisfies" || k.text == "in" ||
                                     k.text == "instanceof"))
            return false;
        return true;
    }

    // Arrow function at i? (optional async, optional <T>, params, ': type', '=>')
    bool arrow_at(int i, int end, FuncShape& f) const {
        int k = i;
        if (I(k, "async") && k + 1 < end && !t[k + 1].nl_before &&
            (P(k + 1, '(') || I(k + 1) || P(k + 1, '<')))
            ++k;
        if (P(k, '<')) {  // generic arrow
            int a = 0;
            int j = k;
            for (; j < end; ++j) {
                if (P(j, '<')) ++a;
                else if (P(j, '>')) { if (--a == 0) break; }
                else if (P(j, ';') || P(j, '{')) return false;
            }
            if (j >= end) return false;
            k = j + 1;
        }
        if (P(k, '(') && t[k].match > k) {
            int rp = t[k].match;
            int j = rp + 1;
            if (P(j, ':')) {
                j = skip_type(j + 1, end, [&](int x) { return P(x, "=>") || P(x, ';') || P(x, ','); }, false);
            }
            if (!P(j, "=>")) return false;
            f.params_b = k + 1;
            f.params_e = rp;
            return arrow_body(j + 1, end, f);
        }
        if (I(k) && P(k + 1, "=>") && !(I(k, "async") && k == i && false)) {
            f.params_b = f.params_e = -1;  // single untyped param
            return arrow_body(k + 2, end, f);
        }
        return false;
    }

    bool arrow_body(int j, int end, FuncShape& f) const {
        if (P(j, '{') && t[j].match > j) {
            f.block = true;
            f.body_b = j + 1;
            f.body_e = t[j].match;
            f.end = t[j].match + 1;
        } else {
            f.block = false;
            f.body_b = j;
            f.body_e = expr_end(j, end);
            f.end = f.body_e;
        }
        return true;
    }

    // Function expression at i? ([async] function [*] [name] [<T>] (params) [: T] { body })
    bool function_expr_at(int i, int end, FuncShape& f) const {
        int k = i;
        if (I(k, "async") && I(k + 1, "function")) ++k;
        if (!I(k, "function")) return false;
        ++k;
        if (P(k, '*')) ++k;
        if (I(k) && !P(k, '(')) ++k;
        if (P(k, '<')) {
            int a = 0;
            for (; k < end; ++k) {
                if (P(k, '<')) ++a;
                else if (P(k, '>')) { if (--a == 0) { ++k; break; } }
            }
        }
        if (!P(k, '(') || t[k].match < 0) return false;
        f.params_b = k + 1;
        f.params_e = t[k].match;
        int j = t[k].match + 1;
        if (P(j, ':')) j = skip_type(j + 1, end, [&](int x) { return P(x, '{') || P(x, ';'); }, true);
        if (!P(j, '{') || t[j].match < 0) return false;
        f.block = true;
        f.body_b = j + 1;
        f.body_e = t[j].match;
        f.end = t[j].match + 1;
        return true;
    }

    bool func_value_at(int i, int end, FuncShape& f) const {
        return arrow_at(i, end, f) || function_expr_at(i, end, f);
    }

    // extractParameterTypes (extractor.ts:433-460)
    std::vector<std::string> param_types(int b, int e) const {
        std::vector<std::string> types;
        if (b < 0) return types;
        int seg = b, angle = 0;
        auto handle = [&](int sb, int se) {
            int k = sb;
            while (k < se && P(k, '@')) {  // parameter decorators
                ++k;
                while (k < se && (I(k) || P(k, '.'))) ++k;
                if (P(k, '(')) k = after_group(k);
            }
            bool prop = false;
            while (k < se && I(k) && kMemberModifiers.count(t[k].text) && I(k + 1)) { ++k; prop = true; }
            (void)prop;
            if (!I(k)) return;  // pattern / rest element
            ++k;
            if (P(k, '?')) ++k;
            if (!P(k, ':')) return;
            ++k;
            if (!I(k) || kTsKeywordTypes.count(t[k].text)) return;
            std::string_view name = t[k].text;
            int j = k + 1;
            if (P(j, '<')) {
                int a = 0;
                for (; j < se; ++j) {
                    if (P(j, '<')) ++a;
                    else if (P(j, '>')) { if (--a == 0) { ++j; break; } }
                    else if (P(j, ">=")) { if (--a == 0) { break; } }
                }
            }
            // the annotation must end here (or at a default value)
            if (j < se && !P(j, '=') && !P(j, ">=")) return;
            types.emplace_back(name);
        };
        for (int i = b; i < e; ++i) {
            const Token& k = t[i];
            if (k.is('<')) ++angle;
            else if (k.is('>')) { if (angle > 0) --angle; }
            else if ((k.is('(') || k.is('[') || k.is('{')) && k.match > i) { i = k.match; continue; }
            else if (k.is(',') && angle == 0) { handle(seg, i); seg = i + 1; }
        }
        if (seg < e) handle(seg, e);
        return types;
    }

    void add_method(std::string_view name, int line, int pb, int pe,
                    const std::string* http_method = nullptr, const std::string* http_path = nullptr) {
        MethodRec m;
        m.name = std::string(name);
        m.line = line;
        m.param_types = param_types(pb, pe);
        if (http_method) { m.has_http_method = true; m.http_method = *http_method; }
        if (http_path) { m.has_http_path = true; m.http_path = *http_path; }
        out.methods.push_back(std::move(m));
    }

    // Next.js App Router (extractor.ts:495-520)
    bool next_http(std::string_view name, std::string& method, std::string& route, bool& has_route) const {
        if (fw != "nextjs") return false;
        if (path.find("route.") == std::string::npos) return false;
        if (!kNextMethods.count(name)) return false;
        method = std::string(name);
        has_route = false;
        size_t app = path.find("app/");
        if (app == std::string::npos) return true;
        std::string after = path.substr(app + 4);
        size_t r = after.rfind("/route.");
        if (r == std::string::npos) return true;
        std::string rp = "/" + after.substr(0, r);
        std::string outp;
        for (size_t k = 0; k < rp.size(); ++k) {
            if (rp[k] == '[') {
                size_t close = rp.find(']', k);
                if (close != std::string::npos && close > k + 1) {
                    outp += ':';
                    outp += rp.substr(k + 1, close - k - 1);
                    k = close;
                    continue;
                }
            }
            outp += rp[k];
        }
        route = outp;
        has_route = true;
        return true;
    }

    void add_function_like(std::string_view name, int line, int pb, int pe) {
        std::string hm, hp;
        bool has_route = false;
        if (next_http(name, hm, hp, has_route)) {
            add_method(name, line, pb, pe, &hm, has_route ? &hp : nullptr);
            entry = true;
        } else {
            add_method(name, line, pb, pe);
        }
    }

    // @Name(...) decorator list starting at i
    int parse_decorators(int i, int end, std::vector<Decorator>& decs) const {
        while (i < end && P(i, '@')) {
            Decorator d;
            d.line = t[i].line;
            ++i;
            if (P(i, '(')) {  // @(expr)
                i = after_group(i);
                decs.push_back(d);
                continue;
            }
            int name_b = i;
            bool dotted = false;
            while (i < end && (I(i) || (P(i, '.') && I(i + 1)))) {
                if (P(i, '.')) dotted = true;
                ++i;
            }
            if (!dotted && name_b < i) d.name = t[name_b].text;
            if (P(i, '<')) {  // type arguments
                int a = 0;
                for (; i < end; ++i) {
                    if (P(i, '<')) ++a;
                    else if (P(i, '>')) { if (--a == 0) { ++i; break; } }
                }
            }
            if (P(i, '(') && t[i].match > i) {
                d.is_call = true;
                d.lparen = i;
                d.rparen = t[i].match;
                i = t[i].match + 1;
            }
            decs.push_back(d);
        }
        return i;
    }

    // extractNestJsHttpInfo (extractor.ts:396-431)
    bool nest_http(const std::vector<Decorator>& decs, std::string& method, std::string& p, bool& has_path) const {
        if (fw != "nestjs") return false;
        for (auto& d : decs) {
            if (!d.is_call || d.name.empty()) continue;
            std::string_view m;
            if (d.name == "Get") m = "GET";
            else if (d.name == "Post") m = "POST";
            else if (d.name == "Put") m = "PUT";
            else if (d.name == "Delete") m = "DELETE";
            else if (d.name == "Patch") m = "PATCH";
            else continue;
            method = std::string(m);
            has_path = false;
            int a = d.lparen + 1;
            if (a == d.rparen) {
                // `@Post()` routes the controller root.  Divergence: the
                // reference leaves the path null, so such handlers were never
                // reported as HTTP endpoints.
                p = "/";
                has_path = true;
            } else if (t[a].kind == Tok::String) {
                int a_end = a + 1;
                if (a_end == d.rparen || P(a_end, ',')) {
                    p = std::string(unquote(t[a].text));
                    has_path = true;
                }
            }
            return true;
        }
        return false;
    }

    // ------------------------------------------------------------- classes
    // i at 'class'; decs = decorators attached to the declaration.
    int parse_class(int i, int end, const std::vector<Decorator>& decs, bool declaration) {
        int k = i + 1;
        while (k < end && !P(k, '{')) {
            if ((P(k, '(') || P(k, '[')) && t[k].match > k) { k = t[k].match + 1; continue; }
            if (P(k, ';')) return k;
            ++k;
        }
        if (k >= end || t[k].match < 0) return k;
        int body_b = k + 1, body_e = t[k].match;
        if (!declaration) {
            scan(body_b, body_e, true);
            return body_e + 1;
        }
        for (auto& d : decs) {
            if (d.name.empty()) continue;
            if (d.name == "Controller") { class_type = "CONTROLLER"; entry = true; }
            else if (d.name == "Injectable" && class_type == "OTHER") class_type = "SERVICE";
            else if (d.name == "Component" || d.name == "Directive" || d.name == "Pipe") class_type = "UTILITY";
            else if (d.name == "NgModule") class_type = "CONFIGURATION";
        }
        struct Pending { int b, e; bool block; };
        std::vector<Pending> nested;
        int m = body_b;
        while (m < body_e) {
            if (P(m, ';') || P(m, ',')) { ++m; continue; }
            int start = m;
            std::vector<Decorator> mdecs;
            m = parse_decorators(m, body_e, mdecs);
            int mod_start = m;
            (void)mod_start;
            // static block
            if (I(m, "static") && P(m + 1, '{')) {
                nested.push_back({m + 2, t[m + 1].match, true});
                m = after_group(m + 1);
                continue;
            }
            // modifiers (a modifier followed by '(' or '=' or ':' is the member name)
            while (I(m) && (kMemberModifiers.count(t[m].text) || t[m].text == "async" ||
                            t[m].text == "get" || t[m].text == "set") &&
                   m + 1 < body_e && !P(m + 1, '(') && !P(m + 1, '=') && !P(m + 1, ':') &&
                   !P(m + 1, ';') && !P(m + 1, '?') && !P(m + 1, '!') && !P(m + 1, '<') && !t[m + 1].nl_before)
                ++m;
            if (P(m, '*')) ++m;
            // key
            bool ident_key = false;
            std::string_view key;
            if (I(m)) {
                key = t[m].text;
                ident_key = key[0] != '#';
                ++m;
            } else if (P(m, '[') && t[m].match > m) {
                m = t[m].match + 1;  // computed key or index signature
            } else if (m < body_e && (t[m].kind == Tok::String || t[m].kind == Tok::Number)) {
                ++m;
            } else {
                ++m;
                continue;
            }
            if (P(m, '?') || P(m, '!')) ++m;
            if (P(m, '<')) {  // method type parameters
                int a = 0;
                for (; m < body_e; ++m) {
                    if (P(m, '<')) ++a;
                    else if (P(m, '>')) { if (--a == 0) { ++m; break; } }
                }
            }
            int line = t[start].line;
            if (P(m, '(') && t[m].match > m) {  // method
                int pb = m + 1, pe = t[m].match;
                int j = pe + 1;
                if (P(j, ':')) j = skip_type(j + 1, body_e, [&](int x) { return P(x, '{') || P(x, ';'); }, true);
                if (P(j, '{') && t[j].match > j) {
                    if (ident_key && key != "constructor") {
                        std::string hm, hp;
                        bool has_path = false;
                        if (nest_http(mdecs, hm, hp, has_path)) {
                            add_method(key, line, pb, pe, &hm, has_path ? &hp : nullptr);
                            entry = true;
                        } else {
                            add_method(key, line, pb, pe);
                        }
                    }
                    nested.push_back({j + 1, t[j].match, true});
                    m = t[j].match + 1;
                } else {
                    m = j;  // abstract method / overload signature (TSDeclareMethod)
                    while (m < body_e && !P(m, ';') && !t[m].nl_before) m = after_group(m);
                }
                continue;
            }
            // property: [: type] [= init]
            if (P(m, ':')) m = skip_type(m + 1, body_e, [&](int x) { return P(x, '=') || P(x, ';') || P(x, '}'); }, false);
            if (P(m, '=')) {
                int ib = m + 1;
                FuncShape f;
                if (ident_key && func_value_at(ib, body_e, f)) {
                    std::string hm, hp;
                    bool has_path = false;
                    if (nest_http(mdecs, hm, hp, has_path)) {
                        add_method(key, line, f.params_b, f.params_e, &hm, has_path ? &hp : nullptr);
                        entry = true;
                    } else {
                        add_method(key, line, f.params_b, f.params_e);
                    }
                }
                int ie = expr_end(ib, body_e);
                nested.push_back({ib, ie, false});
                m = ie;
            }
        }
        for (auto& p : nested) scan(p.b, p.e, p.block);
        return body_e + 1;
    }

    // --------------------------------------------------------- declarations
    // i at const/let/var; exported = inside `export`.
    int parse_var_decl(int i, int end, bool exported) {
        int k = i + 1;
        for (;;) {
            if (k >= end) return k;
            int id_tok = -1;
            if (I(k)) {
                id_tok = k;
                ++k;
            } else if ((P(k, '{') || P(k, '[')) && t[k].match > k) {
                k = t[k].match + 1;  // destructuring pattern
            } else {
                return k;
            }
            if (P(k, '!')) ++k;
            if (P(k, ':'))
                k = skip_type(k + 1, end, [&](int x) { return P(x, '=') || P(x, ',') || P(x, ';'); }, false);
            if (!P(k, '=')) {
                if (P(k, ',')) { ++k; continue; }
                return k;
            }
            int ib = k + 1;
            int ie = expr_end(ib, end);
            if (id_tok >= 0) {
                FuncShape f;
                bool direct = func_value_at(ib, ie, f);
                if (direct) {
                    add_function_like(t[id_tok].text, t[id_tok].line, f.params_b, f.params_e);
                } else if (!exported) {
                    // wrapped: callee(...) whose first argument is a function (extractor.ts:471-493)
                    int c = ib;
                    while (c < ie && (I(c) || P(c, '.') || P(c, "?."))) ++c;
                    if (P(c, '<')) {
                        int a = 0;
                        for (; c < ie; ++c) {
                            if (P(c, '<')) ++a;
                            else if (P(c, '>')) { if (--a == 0) { ++c; break; } }
                        }
                    }
                    if (c > ib && P(c, '(') && t[c].match > c) {
                        FuncShape g;
                        if (func_value_at(c + 1, t[c].match, g)) {
                            int ge = g.end;
                            if (ge == t[c].match || P(ge, ','))
                                add_function_like(t[id_tok].text, t[id_tok].line, g.params_b, g.params_e);
                        }
                    }
                }
            }
            scan(ib, ie, false);
            k = ie;
            if (P(k, ',')) { ++k; continue; }
            return k;
        }
    }

    // i at 'function' or 'async' (function declaration in statement position)
    int parse_function_decl(int i, int end) {
        int start = i;
        int k = i;
        if (I(k, "async")) ++k;
        ++k;  // 'function'
        if (P(k, '*')) ++k;
        int name_tok = -1;
        if (I(k)) { name_tok = k; ++k; }
        if (P(k, '<')) {
            int a = 0;
            for (; k < end; ++k) {
                if (P(k, '<')) ++a;
                else if (P(k, '>')) { if (--a == 0) { ++k; break; } }
            }
        }
        if (!P(k, '(') || t[k].match < 0) return k;
        int pb = k + 1, pe = t[k].match;
        int j = pe + 1;
        if (P(j, ':')) j = skip_type(j + 1, end, [&](int x) { return P(x, '{') || P(x, ';'); }, true);
        if (!P(j, '{') || t[j].match < 0) return j;  // TSDeclareFunction / overload
        if (name_tok >= 0) add_function_like(t[name_tok].text, t[start].line, pb, pe);
        scan(j + 1, t[j].match, true);
        return t[j].match + 1;
    }

    // ------------------------------------------------------------- objects
    // '{' at i in expression position: object literal.
    void parse_object(int i) {
        int b = i + 1, e = t[i].match;
        int seg = b;
        for (int k = b; k <= e; ++k) {
            if (k == e || P(k, ',')) {
                if (seg < k) property(seg, k);
                seg = k + 1;
                continue;
            }
            if ((P(k, '(') || P(k, '[') || P(k, '{')) && t[k].match > k) k = t[k].match;
        }
    }

    void property(int b, int e) {
        int k = b;
        if (P(k, "...")) { scan(k + 1, e, false); return; }
        int start = k;
        // object method: [async] [get|set] [*] key ( ... ) { ... }
        int m = k;
        while (I(m) && (t[m].text == "async" || t[m].text == "get" || t[m].text == "set") && m + 1 < e &&
               !P(m + 1, '(') && !P(m + 1, ':') && !P(m + 1, ','))
            ++m;
        if (P(m, '*')) ++m;
        bool ident_key = I(m);
        int key_tok = m;
        if (I(m) || (m < e && (t[m].kind == Tok::String || t[m].kind == Tok::Number))) ++m;
        else if (P(m, '[') && t[m].match > m) m = t[m].match + 1;
        if (P(m, '<')) {
            int a = 0;
            for (; m < e; ++m) {
                if (P(m, '<')) ++a;
                else if (P(m, '>')) { if (--a == 0) { ++m; break; } }
            }
        }
        if (P(m, '(') && t[m].match > m) {
            int pb = m + 1, pe = t[m].match;
            int j = pe + 1;
            if (P(j, ':')) j = skip_type(j + 1, e, [&](int x) { return P(x, '{'); }, true);
            if (P(j, '{') && t[j].match > j) {
                if (ident_key) add_method(t[key_tok].text, t[start].line, pb, pe);
                scan(j + 1, t[j].match, true);
                if (t[j].match + 1 < e) scan(t[j].match + 1, e, false);
                return;
            }
        }
        // key: value
        k = start;
        bool simple_key = I(k) && P(k + 1, ':');
        int colon = -1;
        if (simple_key) colon = k + 1;
        else if (k < e && (t[k].kind == Tok::String || t[k].kind == Tok::Number) && P(k + 1, ':')) colon = k + 1;
        else if (P(k, '[') && t[k].match > k && P(t[k].match + 1, ':')) colon = t[k].match + 1;
        if (colon >= 0) {
            int vb = colon + 1;
            FuncShape f;
            if (simple_key && func_value_at(vb, e, f)) add_method(t[k].text, t[k].line, f.params_b, f.params_e);
            scan(vb, e, false);
            return;
        }
        scan(b, e, false);  // shorthand, spread or something we do not model
    }

    // --------------------------------------------------------------- scan
    // Generic scan of [b, e). `stmt` = statement list (blocks) vs expression.
    void scan(int b, int e, bool stmt) {
        if (guard >= 400) return;  // pathological nesting guard
        struct Depth { int& d; explicit Depth(int& x) : d(x) { ++d; } ~Depth() { --d; } } depth_guard(guard);
        int i = b;
        std::vector<Decorator> pending;
        while (i < e) {
            const Token& k = t[i];
            if (k.kind == Tok::Punct) {
                if (k.text == "@" ) {
                    pending.clear();
                    i = parse_decorators(i, e, pending);
                    continue;
                }
                if (k.text == "{" && k.match > i) {
                    bool obj = !stmt_start(i, stmt) && expression_context(i) && !P(i - 1, "=>");
                    if (obj) {
                        parse_object(i);
                    } else {
                        scan(i + 1, k.match, true);
                    }
                    i = k.match + 1;
                    continue;
                }
                if (k.text == "(" && k.match > i) {
                    // arrow parameters: skip their types, scan default values only
                    FuncShape f;
                    if (arrow_at(i, e, f)) {
                        scan_params(f.params_b, f.params_e);
                        if (f.block) scan(f.body_b, f.body_e, true);
                        else scan(f.body_b, f.body_e, false);
                        i = f.end;
                        continue;
                    }
                    scan(i + 1, k.match, false);
                    i = k.match + 1;
                    continue;
                }
                ++i;
                continue;
            }
            if (k.kind != Tok::Ident) { ++i; continue; }
            std::string_view w = k.text;
            bool at_stmt = stmt_start(i, stmt);
            // property access `x.class` etc. are not keywords
            if (i > b && (P(i - 1, '.') || P(i - 1, "?."))) { ++i; continue; }
            // CommonJS `require('./x')` and dynamic `import('./x')` with a literal
            // specifier (the legacy NodeJsSourceParser resolved require(); the
            // Babel extractor only sees ES imports)
            if ((w == "require" || w == "import") && P(i + 1, '(') && i + 3 < e &&
                t[i + 2].kind == Tok::String && P(i + 3, ')')) {
                ImportRec r;
                r.imported = w == "require" ? "require" : "import()";
                r.source = std::string(unquote(t[i + 2].text));
                out.imports.push_back(r);
                i += 4;
                continue;
            }
            if (w == "import" && !P(i + 1, '(') && !P(i + 1, '.')) { i = parse_import(i, e); continue; }
            if (w == "export") { i = parse_export(i, e, pending); pending.clear(); continue; }
            if (w == "class" || (w == "abstract" && I(i + 1, "class"))) {
                int ci = w == "class" ? i : i + 1;
                bool decl = at_stmt || !pending.empty() || (i > b && I(i - 1, "declare"));
                i = parse_class(ci, e, pending, decl);
                pending.clear();
                continue;
            }
            if ((w == "function" || (w == "async" && I(i + 1, "function") && !t[i + 1].nl_before))) {
                if (at_stmt) { i = parse_function_decl(i, e); continue; }
                FuncShape f;
                if (function_expr_at(i, e, f)) {
                    scan_params(f.params_b, f.params_e);
                    scan(f.body_b, f.body_e, true);
                    i = f.end;
                    continue;
                }
                ++i;
                continue;
            }
            if ((w == "const" || w == "let" || w == "var") && (I(i + 1) || P(i + 1, '{') || P(i + 1, '['))) {
                if (w == "const" && I(i + 1, "enum")) { i = skip_ts_decl(i + 1, e); continue; }
                i = parse_var_decl(i, e, false);
                continue;
            }
            if (at_stmt && (w == "interface" ) && I(i + 1)) { i = skip_ts_decl(i, e); continue; }
            if (at_stmt && w == "type" && I(i + 1) && (P(i + 2, '=') || P(i + 2, '<'))) { i = skip_ts_decl(i, e); continue; }
            if (at_stmt && w == "enum" && I(i + 1)) { i = skip_ts_decl(i, e); continue; }
            if (at_stmt && w == "declare") {
                if (I(i + 1, "module") || I(i + 1, "namespace") || I(i + 1, "global")) { ++i; continue; }
                if (I(i + 1, "const") || I(i + 1, "let") || I(i + 1, "var") || I(i + 1, "function")) {
                    i = skip_declare(i, e);
                    continue;
                }
                ++i;
                continue;
            }
            if ((w == "as" || w == "satisfies") && i > b && !at_stmt) {
                i = skip_type(i + 1, e, [&](int x) {
                    return P(x, ')') || P(x, ',') || P(x, ';') || P(x, ']') || P(x, '}') || P(x, '=') ||
                           P(x, "&&") || P(x, "||") || P(x, "??") || P(x, '?') || P(x, ':');
                }, true);
                continue;
            }
            // Express registrations (extractor.ts:274-298)
            if ((w == "app" || w == "router") && P(i + 1, '.') && I(i + 2) && P(i + 3, '(')) {
                std::string_view verb = t[i + 2].text;
                if (verb == "get" || verb == "post" || verb == "put" || verb == "delete" || verb == "patch" ||
                    verb == "all" || verb == "use") {
                    entry = true;
                    if (class_type == "OTHER") class_type = "CONTROLLER";
                }
            }
            // arrow with a single identifier parameter: x => ...
            if (P(i + 1, "=>")) {
                FuncShape f;
                if (arrow_at(i, e, f)) {
                    if (f.block) scan(f.body_b, f.body_e, true);
                    else scan(f.body_b, f.body_e, false);
                    i = f.end;
                    continue;
                }
            }
            if (w == "async") {
                FuncShape f;
                if (arrow_at(i, e, f)) {
                    scan_params(f.params_b, f.params_e);
                    if (f.block) scan(f.body_b, f.body_e, true);
                    else scan(f.body_b, f.body_e, false);
                    i = f.end;
                    continue;
                }
            }
            ++i;
        }
    }

    // Arrow/function parameter list: only default values can hold nested code.
    void scan_params(int b, int e) {
        if (b < 0) return;
        int angle = 0, seg = b;
        auto handle = [&](int sb, int se) {
            for (int k = sb; k < se; ++k) {
                if ((P(k, '(') || P(k, '[') || P(k, '{')) && t[k].match > k) { k = t[k].match; continue; }
                if (P(k, '<')) {
                    int a = 0;
                    for (; k < se; ++k) {
                        if (P(k, '<')) ++a;
                        else if (P(k, '>')) { if (--a == 0) break; }
                    }
                    continue;
                }
                if (P(k, '=')) { scan(k + 1, se, false); return; }
            }
        };
        for (int i = b; i < e; ++i) {
            if (P(i, '<')) ++angle;
            else if (P(i, '>')) { if (angle > 0) --angle; }
            else if ((P(i, '(') || P(i, '[') || P(i, '{')) && t[i].match > i) { i = t[i].match; continue; }
            else if (P(i, ',') && angle == 0) { handle(seg, i); seg = i + 1; }
        }
        if (seg < e) handle(seg, e);
    }

    bool stmt_start(int i, bool stmt) const {
        if (!stmt) return false;
        if (i <= 0) return true;
        const Token& p = t[i - 1];
        if (p.kind == Tok::Punct) {
            if (p.text == ";" || p.text == "{" || p.text == "}") return true;
            if (p.text == ")") {
                // `if (...) stmt` etc.: a statement follows unless this ')' closes an expression
                int open = p.match;
                if (open > 0 && t[open - 1].kind == Tok::Ident) {
                    std::string_view s = t[open - 1].text;
                    if (s == "if" || s == "for" || s == "while" || s == "with") return true;
                }
                return t[i].nl_before;
            }
            if (p.text == ":" ) return false;
            return false;
        }
        if (p.kind == Tok::Ident) {
            if (p.text == "else" || p.text == "do") return true;
            if (p.text == "default" && i >= 2 && I(i - 2, "export")) return true;
            if (t[i].nl_before && !kExprKeywords.count(p.text)) return true;
            return false;
        }
        if (t[i].nl_before) return true;
        return false;
    }

    int skip_ts_decl(int i, int e) {
        // interface X<..> extends .. { } | type X<..> = T; | enum X { }
        int k = i + 1;
        if (I(i, "type")) {
            while (k < e && !P(k, '=')) {
                if (P(k, '<')) {
                    int a = 0;
                    for (; k < e; ++k) {
                        if (P(k, '<')) ++a;
                        else if (P(k, '>')) { if (--a == 0) break; }
                    }
                }
                ++k;
            }
            if (k < e) k = skip_type(k + 1, e, [&](int x) { return P(x, ';'); }, false);
            return k;
        }
        while (k < e && !P(k, '{')) {
            if (P(k, ';')) return k + 1;
            if ((P(k, '(') || P(k, '[')) && t[k].match > k) { k = t[k].match + 1; continue; }
            ++k;
        }
        return after_group(k);
    }

    int skip_declare(int i, int e) {
        int k = i + 1;
        while (k < e && !P(k, ';') && !(k > i + 2 && t[k].nl_before && asi_break(k))) k = after_group(k);
        return k;
    }

    // import declarations (extractor.ts:67-93)
    int parse_import(int i, int e) {
        int k = i + 1;
        if (k < e && t[k].kind == Tok::String) return k + 1;  // side-effect import: no specifiers
        bool type_only = false;
        if (I(k, "type") && !P(k + 1, ',') && !I(k + 1, "from")) { type_only = true; ++k; }
        (void)type_only;
        std::vector<ImportRec> specs;
        while (k < e) {
            if (I(k, "from")) break;
            if (I(k) && !I(k, "from")) {  // default
                ImportRec r;
                r.imported = "default";
                r.local = std::string(t[k].text);
                specs.push_back(r);
                ++k;
                continue;
            }
            if (P(k, '*') && I(k + 1, "as") && I(k + 2)) {
                ImportRec r;
                r.imported = "*";
                r.local = std::string(t[k + 2].text);
                specs.push_back(r);
                k += 3;
                continue;
            }
            if (P(k, '{') && t[k].match > k) {
                int end = t[k].match;
                int s = k + 1;
                while (s < end) {
                    int se = s;
                    while (se < end && !P(se, ',')) ++se;
                    int a = s;
                    if (I(a, "type") && se - a >= 2 && !P(a + 1, ',')) ++a;  // inline type modifier
                    if (a < se) {
                        ImportRec r;
                        std::string_view imported = t[a].kind == Tok::String ? unquote(t[a].text) : t[a].text;
                        r.imported = std::string(imported);
                        r.local = r.imported;
                        if (a + 2 < se + 1 && I(a + 1, "as") && a + 2 < se) r.local = std::string(t[a + 2].text);
                        specs.push_back(r);
                    }
                    s = se + 1;
                }
                k = end + 1;
                continue;
            }
            if (P(k, ',')) { ++k; continue; }
            break;
        }
        if (!I(k, "from") || k + 1 >= e || t[k + 1].kind != Tok::String) return k + 1;
        std::string source(unquote(t[k + 1].text));
        for (auto& r : specs) {
            r.source = source;
            out.imports.push_back(r);
        }
        k += 2;
        // import attributes: with { type: 'json' } / assert { ... }
        if ((I(k, "with") || I(k, "assert")) && P(k + 1, '{')) k = after_group(k + 1);
        return k;
    }

    int parse_export(int i, int e, const std::vector<Decorator>& pending) {
        int k = i + 1;
        if (I(k, "default")) {
            ++k;
            std::vector<Decorator> decs = pending;
            if (P(k, '@')) k = parse_decorators(k, e, decs);
            if (I(k, "abstract") && I(k + 1, "class")) ++k;
            if (I(k, "class")) return parse_class(k, e, decs, true);
            if (I(k, "function") || (I(k, "async") && I(k + 1, "function"))) return parse_function_decl(k, e);
            int ee = expr_end(k, e);
            scan(k, ee, false);
            return ee;
        }
        if (I(k, "declare")) return skip_declare(k, e);
        std::vector<Decorator> decs = pending;
        if (P(k, '@')) k = parse_decorators(k, e, decs);
        if (I(k, "abstract") && I(k + 1, "class")) ++k;
        if (I(k, "class")) return parse_class(k, e, decs, true);
        if (I(k, "function") || (I(k, "async") && I(k + 1, "function"))) return parse_function_decl(k, e);
        if (I(k, "const") && I(k + 1, "enum")) return skip_ts_decl(k + 1, e);
        if (I(k, "const") || I(k, "let") || I(k, "var")) return parse_var_decl(k, e, true);
        if (I(k, "interface") || I(k, "enum")) return skip_ts_decl(k, e);
        if (I(k, "type") && !P(k + 1, '{') && !P(k + 1, '*')) return skip_ts_decl(k, e);
        if (I(k, "namespace") || I(k, "module")) return k;  // body scanned as a block by the caller
        // export { a, b } [from '...'] / export * from '...' / export = x
        int ee = k;
        while (ee < e && !P(ee, ';') && !(ee > k && t[ee].nl_before && asi_break(ee))) ee = after_group(ee);
        return ee;
    }

    std::string class_type_from_filename() const {
        size_t slash = path.rfind('/');
        std::string fn = to_lower(slash == std::string::npos ? path : path.substr(slash + 1));
        struct { const char* k; const char* v; } table[] = {
            {".controller.", "CONTROLLER"}, {".service.", "SERVICE"}, {".repository.", "REPOSITORY"},
            {".entity.", "ENTITY"}, {".dto.", "DTO"}, {".config.", "CONFIGURATION"},
            {".middleware.", "UTILITY"}, {".guard.", "UTILITY"}, {".interceptor.", "UTILITY"},
            {".pipe.", "UTILITY"}, {".filter.", "UTILITY"}, {".exception.", "EXCEPTION"},
            {".listener.", "LISTENER"}, {".module.", "CONFIGURATION"}};
        for (auto& r : table)
            if (fn.find(r.k) != std::string::npos) return r.v;
        return "OTHER";
    }

    bool well_known_entry() const {
        size_t slash = path.rfind('/');
        std::string fn = slash == std::string::npos ? path : path.substr(slash + 1);
        static const std::unordered_set<std::string> names = {"main.ts", "main.js", "index.ts", "index.js",
                                                              "app.ts", "app.js", "server.ts", "server.js"};
        return names.count(fn) > 0;
    }
};

}  // namespace

void analyze_ts(std::string_view src, const std::string& rel_path, const std::string& framework, bool jsx,
                FileRec& out) {
    TsLexer lx(src, jsx);
    lx.run();
    TsScanner sc(lx.toks, rel_path, framework, out);
    sc.run();
}

// detector.ts:11-85
FrameworkInfo detect_framework(std::string_view package_json) {
    FrameworkInfo fi;
    JsonValue root;
    if (!parse_json(package_json, root) || root.kind != JsonValue::Obj) return fi;
    auto has = [&](std::string_view dep) {
        for (const char* sec : {"dependencies", "devDependencies"}) {
            const JsonValue* d = root.get(sec);
            if (d && d->kind == JsonValue::Obj && d->get(dep)) {
                const JsonValue* v = d->get(dep);
                // JS truthiness of the version string: "" is falsy
                if (v->kind == JsonValue::Str && v->s.empty()) continue;
                if (v->kind == JsonValue::Null || (v->kind == JsonValue::Bool && !v->b)) continue;
                return true;
            }
        }
        return false;
    };
    if (has("typescript")) fi.features.emplace_back("typescript", "true");
    auto ret = [&](const char* name, const char* root_dir) {
        fi.name = name;
        fi.source_root = root_dir;
        return fi;
    };
    if (has("@nestjs/core")) { fi.features.emplace_back("decorators", "true"); return ret("nestjs", "src"); }
    if (has("next")) { fi.features.emplace_back("router", "unknown"); return ret("nextjs", "src"); }
    if (has("nuxt") || has("nuxt3")) return ret("nuxt", "src");
    if (has("@angular/core")) { fi.features.emplace_back("decorators", "true"); return ret("angular", "src"); }
    if (has("vue")) return ret("vue", "src");
    if (has("@remix-run/node") || has("@remix-run/react")) return ret("remix", "app");
    if (has("@sveltejs/kit")) return ret("sveltekit", "src");
    if (has("astro")) return ret("astro", "src");
    if (has("fastify")) return ret("fastify", "src");
    if (has("express")) return ret("express", "src");
    return fi;
}

}  // namespace srcscan
