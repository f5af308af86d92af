// srcscan -- native source front-ends for the dmcp indexer.
//
// Shared infrastructure: token model, a C-family lexer (Java / Go flavours),
// bracket matching, a tiny JSON writer/reader and a fixed thread pool.
//
// The reference parses Java with JavaParser (JavaSourceParser.java:61-64),
// TS/JS with Babel inside GraalJS (GraalJsAnalyzerEngine.java:73-164) and Go
// with a separate go/ast binary (tools/go-analyzer).  None of those exist on
// this host, so all three front-ends are hand-written C++17 over one token
// model, and every file is lexed exactly once (the reference re-parses each
// Java file ~5 times, JavaSourceParser.java:631-643).
#pragma once

#include <atomic>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <string_view>
#include <thread>
#include <utility>
#include <vector>

namespace srcscan {

enum class Tok : uint8_t {
    Ident,
    Number,
    String,    // "..." / '...' (JS) / `...` (Go raw) / """...""" (Java text block)
    Char,      // Java/Go character literal
    Template,  // JS template literal chunk (whole literal when no substitutions)
    Regex,     // JS regular-expression literal
    Punct,
    JsxText,   // opaque JSX text / tag chunk (TS front-end only)
    Semi,      // Go automatic semicolon (virtual)
    End
};

struct Token {
    Tok kind;
    std::string_view text;
    int line;         // 1-based line of the first character
    int match = -1;   // index of the matching bracket for ( [ { ) ] }
    bool nl_before = false;  // a newline separates this token from the previous one

    bool is(char c) const { return kind == Tok::Punct && text.size() == 1 && text[0] == c; }
    bool is(std::string_view s) const { return (kind == Tok::Punct || kind == Tok::Ident) && text == s; }
    bool ident() const { return kind == Tok::Ident; }
    bool ident(std::string_view s) const { return kind == Tok::Ident && text == s; }
};

inline bool is_ident_start(unsigned char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' || c == '$' || c >= 0x80;
}
inline bool is_ident_char(unsigned char c) {
    return is_ident_start(c) || (c >= '0' && c <= '9');
}

// Links every bracket token to its partner; unbalanced brackets keep match=-1.
void match_brackets(std::vector<Token>& toks);

// ---------------------------------------------------------------- C lexer
struct CLexOptions {
    bool go = false;    // backtick raw strings, automatic semicolons, no text blocks
    bool java = false;  // """ text blocks
};
std::vector<Token> lex_c_family(std::string_view src, const CLexOptions& opt);

// Strips the quotes of a string literal token (no escape processing: the
// reference's annotation values are compared/printed as written).
std::string_view unquote(std::string_view lit);

// ---------------------------------------------------------------- JSON out
class JsonWriter {
public:
    std::string out;
    void raw(std::string_view s) { out.append(s.data(), s.size()); }
    void str(std::string_view s);
    void null() { out += "null"; }
    void boolean(bool b) { out += b ? "true" : "false"; }
    void integer(long long v) { out += std::to_string(v); }
    void key(std::string_view k) { comma(); str(k); out += ':'; need_comma_ = false; }
    void begin_obj() { comma(); out += '{'; need_comma_ = false; }
    void end_obj() { out += '}'; need_comma_ = true; }
    void begin_arr() { comma(); out += '['; need_comma_ = false; }
    void end_arr() { out += ']'; need_comma_ = true; }
    void value_str(std::string_view s) { comma(); str(s); need_comma_ = true; }
    void value_null() { comma(); null(); need_comma_ = true; }
    void value_bool(bool b) { comma(); boolean(b); need_comma_ = true; }
    void value_int(long long v) { comma(); integer(v); need_comma_ = true; }
    void kv(std::string_view k, std::string_view v) { key(k); value_str(v); }
    void kv_opt(std::string_view k, const std::string* v) { key(k); if (v) value_str(*v); else value_null(); }
    void kv(std::string_view k, bool v) { key(k); value_bool(v); }
    void kv_int(std::string_view k, long long v) { key(k); value_int(v); }
    void str_array(std::string_view k, const std::vector<std::string>& v) {
        key(k); begin_arr(); for (auto& s : v) value_str(s); end_arr();
    }
private:
    bool need_comma_ = false;
    void comma() { if (need_comma_) out += ','; }
};

// Minimal JSON reader sufficient for package.json dependency maps.
struct JsonValue {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    std::string s;
    bool b = false;
    std::vector<JsonValue> arr;
    std::vector<std::pair<std::string, JsonValue>> obj;
    const JsonValue* get(std::string_view k) const {
        for (auto& kv : obj) if (kv.first == k) return &kv.second;
        return nullptr;
    }
};
bool parse_json(std::string_view text, JsonValue& out);

// --------------------------------------------------------------- threading
// Runs fn(i) for i in [0, n) on `threads` workers (0 = hardware concurrency).
void parallel_for(size_t n, int threads, const std::function<void(size_t)>& fn);

// ------------------------------------------------------------------- files
// Every filesystem access of the front-ends goes through these helpers, which
// also serve *mounted in-memory trees*: paths under a root returned by
// vfs_mount() ("/__vfs__/<n>") resolve against that tree, so a project can be
// scanned straight from git objects without a checkout on disk.
bool read_file(const std::string& path, std::string& out, size_t max_bytes = 0);
bool file_exists(const std::string& path);
bool dir_exists(const std::string& path);
// Sorted (name, is_dir) children of a directory (real or mounted).
bool list_dir(const std::string& dir, std::vector<std::pair<std::string, bool>>& out);
// Mounts files given as (relative path, content); returns the virtual root.
std::string vfs_mount(std::vector<std::pair<std::string, std::string>>&& files);
// The same without copying: the contents must outlive vfs_unmount().
std::string vfs_mount_views(const std::vector<std::pair<std::string, std::string_view>>& files);
void vfs_unmount(const std::string& root);
std::string join_path(const std::string& a, const std::string& b);
std::string normalize_path(const std::string& p);  // resolves . and .. lexically

// Lowercases ASCII.
std::string to_lower(std::string_view s);
bool starts_with(std::string_view s, std::string_view p);
bool ends_with(std::string_view s, std::string_view p);
bool contains(std::string_view s, std::string_view p);

}  // namespace srcscan
