#include "common.hpp"

#include "gitobj.hpp"

#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <cstdlib>
#include <dirent.h>
#include <memory>
#include <mutex>
#include <sys/stat.h>
#include <unordered_map>

namespace srcscan {

void match_brackets(std::vector<Token>& toks) {
    std::vector<int> stack;
    stack.reserve(64);
    for (int i = 0; i < (int)toks.size(); ++i) {
        Token& t = toks[i];
        if (t.kind != Tok::Punct || t.text.size() != 1) continue;
        char c = t.text[0];
        if (c == '(' || c == '[' || c == '{') {
            stack.push_back(i);
        } else if (c == ')' || c == ']' || c == '}') {
            char want = c == ')' ? '(' : (c == ']' ? '[' : '{');
            // Tolerate unbalanced input: pop to the nearest matching opener.
            int j = (int)stack.size() - 1;
            while (j >= 0 && toks[stack[j]].text[0] != want) --j;
            if (j < 0) continue;
            int open = stack[j];
            stack.resize(j);
            toks[open].match = i;
            t.match = open;
        }
    }
}

static const char* kMultiPunct[] = {
    "...", "::", "->", ":=", "<-", "==", "!=", "&&", "||", "++", "--",
    "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<=", ">=", nullptr};

std::vector<Token> lex_c_family(std::string_view src, const CLexOptions& opt) {
    std::vector<Token> toks;
    toks.reserve(src.size() / 4 + 16);
    size_t i = 0, n = src.size();
    int line = 1;
    bool nl = false;
    auto go_semi_ok = [&]() {
        if (!opt.go || toks.empty()) return false;
        const Token& t = toks.back();
        switch (t.kind) {
            case Tok::Ident:
            case Tok::Number:
            case Tok::String:
            case Tok::Char:
                return true;
            case Tok::Punct:
                return t.text == ")" || t.text == "]" || t.text == "}" || t.text == "++" || t.text == "--";
            default:
                return false;
        }
    };
    auto newline = [&]() {
        if (go_semi_ok()) {
            Token s{Tok::Semi, std::string_view(), line};
            toks.push_back(s);
        }
        ++line;
        nl = true;
    };
    auto push = [&](Tok k, size_t b, size_t e, int ln) {
        Token t{k, src.substr(b, e - b), ln};
        t.nl_before = nl;
        nl = false;
        toks.push_back(t);
    };
    while (i < n) {
        unsigned char c = src[i];
        if (c == '\n') { newline(); ++i; continue; }
        if (c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v') { ++i; continue; }
        if (c == '/' && i + 1 < n && src[i + 1] == '/') {
            while (i < n && src[i] != '\n') ++i;
            continue;
        }
        if (c == '/' && i + 1 < n && src[i + 1] == '*') {
            i += 2;
            bool had_nl = false;
            while (i < n && !(src[i] == '*' && i + 1 < n && src[i + 1] == '/')) {
                if (src[i] == '\n') { ++line; had_nl = true; }
                ++i;
            }
            i = std::min(n, i + 2);
            if (had_nl) {  // a multi-line comment acts like a newline (Go spec)
                if (go_semi_ok()) toks.push_back(Token{Tok::Semi, std::string_view(), line});
                nl = true;
            }
            continue;
        }
        int ln = line;
        if (opt.java && c == '"' && i + 2 < n && src[i + 1] == '"' && src[i + 2] == '"') {
            size_t b = i;
            i += 3;
            while (i < n && !(src[i] == '"' && i + 2 < n && src[i + 1] == '"' && src[i + 2] == '"' && src[i - 1] != '\\')) {
                if (src[i] == '\n') ++line;
                ++i;
            }
            i = std::min(n, i + 3);
            push(Tok::String, b, i, ln);
            continue;
        }
        if (c == '"') {
            size_t b = i++;
            while (i < n && src[i] != '"' && src[i] != '\n') {
                if (src[i] == '\\' && i + 1 < n) ++i;
                ++i;
            }
            if (i < n && src[i] == '"') ++i;
            push(Tok::String, b, i, ln);
            continue;
        }
        if (c == '\'') {
            size_t b = i++;
            while (i < n && src[i] != '\'' && src[i] != '\n') {
                if (src[i] == '\\' && i + 1 < n) ++i;
                ++i;
            }
            if (i < n && src[i] == '\'') ++i;
            push(Tok::Char, b, i, ln);
            continue;
        }
        if (opt.go && c == '`') {
            size_t b = i++;
            while (i < n && src[i] != '`') {
                if (src[i] == '\n') ++line;
                ++i;
            }
            if (i < n) ++i;
            push(Tok::String, b, i, ln);
            continue;
        }
        if ((c >= '0' && c <= '9') || (c == '.' && i + 1 < n && src[i + 1] >= '0' && src[i + 1] <= '9')) {
            size_t b = i++;
            while (i < n) {
                unsigned char d = src[i];
                if (is_ident_char(d) || d == '.') { ++i; continue; }
                if ((d == '+' || d == '-') && (src[i - 1] == 'e' || src[i - 1] == 'E' || src[i - 1] == 'p' || src[i - 1] == 'P')) {
                    ++i;
                    continue;
                }
                break;
            }
            push(Tok::Number, b, i, ln);
            continue;
        }
        if (is_ident_start(c)) {
            size_t b = i++;
            while (i < n && is_ident_char((unsigned char)src[i])) ++i;
            push(Tok::Ident, b, i, ln);
            continue;
        }
        // punctuation
        bool matched = false;
        for (const char** p = kMultiPunct; *p; ++p) {
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
    if (go_semi_ok()) toks.push_back(Token{Tok::Semi, std::string_view(), line});
    match_brackets(toks);
    return toks;
}

std::string_view unquote(std::string_view lit) {
    if (lit.size() >= 6 && starts_with(lit, "\"\"\"") && ends_with(lit, "\"\"\"")) return lit.substr(3, lit.size() - 6);
    if (lit.size() >= 2) {
        char a = lit.front(), b = lit.back();
        if ((a == '"' || a == '\'' || a == '`') && a == b) return lit.substr(1, lit.size() - 2);
    }
    return lit;
}

// ------------------------------------------------------------------ JSON
namespace {
// Length of the well-formed UTF-8 sequence at s[i] (RFC 3629: no overlongs,
// no surrogates, nothing past U+10FFFF), 0 when it is not one.
size_t utf8_seq(std::string_view s, size_t i) {
    const unsigned char c = (unsigned char)s[i];
    size_t n;
    unsigned lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) n = 2;
    else if (c >= 0xE0 && c <= 0xEF) {
        n = 3;
        if (c == 0xE0) lo = 0xA0;
        if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
        n = 4;
        if (c == 0xF0) lo = 0x90;
        if (c == 0xF4) hi = 0x8F;
    } else
        return 0;
    if (i + n > s.size()) return 0;
    const unsigned char c1 = (unsigned char)s[i + 1];
    if (c1 < lo || c1 > hi) return 0;
    for (size_t k = 2; k < n; ++k)
        if (((unsigned char)s[i + k] & 0xC0) != 0x80) return 0;
    return n;
}
}  // namespace

void JsonWriter::str(std::string_view s) {
    out += '"';
    for (size_t i = 0; i < s.size(); ++i) {
        const unsigned char c = (unsigned char)s[i];
        if (c >= 0x80) {
            // source files are not always UTF-8 (Latin-1 comments, binary
            // junk): an invalid byte becomes U+FFFD, so the document is
            // always valid JSON text
            const size_t n = utf8_seq(s, i);
            if (n == 0) {
                out += "\xEF\xBF\xBD";
            } else {
                out.append(s.data() + i, n);
                i += n - 1;
            }
            continue;
        }
        switch (c) {
            case '"': out += "\\\""; break;
            case '\\': out += "\\\\"; break;
            case '\n': out += "\\n"; break;
            case '\r': out += "\\r"; break;
            case '\t': out += "\\t"; break;
            case '\b': out += "\\b"; break;
            case '\f': out += "\\f"; break;
            default:
                if (c < 0x20) {
                    char buf[8];
                    std::snprintf(buf, sizeof buf, "\\u%04x", c);
                    out += buf;
                } else {
                    out += (char)c;
                }
        }
    }
    out += '"';
}

namespace {
struct JsonParser {
    std::string_view t;
    size_t i = 0;
    int depth = 0;
    void ws() { while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\r' || t[i] == '\t')) ++i; }
    bool lit(const char* s) {
        size_t n = std::strlen(s);
        if (t.compare(i, n, s) == 0) { i += n; return true; }
        return false;
    }
    bool string(std::string& out) {
        if (i >= t.size() || t[i] != '"') return false;
        ++i;
        while (i < t.size() && t[i] != '"') {
            char c = t[i++];
            if (c == '\\' && i < t.size()) {
                char e = t[i++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (i + 4 > t.size()) return false;
                        unsigned cp = (unsigned)std::stoul(std::string(t.substr(i, 4)), nullptr, 16);
                        i += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (i >= t.size()) return false;
        ++i;
        return true;
    }
    bool value(JsonValue& v) {
        if (++depth > 256) return false;
        ws();
        if (i >= t.size()) return false;
        char c = t[i];
        bool ok = true;
        if (c == '{') {
            v.kind = JsonValue::Obj;
            ++i;
            ws();
            if (i < t.size() && t[i] == '}') { ++i; --depth; return true; }
            while (ok) {
                ws();
                std::string k;
                if (!string(k)) return false;
                ws();
                if (i >= t.size() || t[i] != ':') return false;
                ++i;
                JsonValue child;
                if (!value(child)) return false;
                v.obj.emplace_back(std::move(k), std::move(child));
                ws();
                if (i < t.size() && t[i] == ',') { ++i; continue; }
                if (i < t.size() && t[i] == '}') { ++i; break; }
                return false;
            }
        } else if (c == '[') {
            v.kind = JsonValue::Arr;
            ++i;
            ws();
            if (i < t.size() && t[i] == ']') { ++i; --depth; return true; }
            while (true) {
                JsonValue child;
                if (!value(child)) return false;
                v.arr.push_back(std::move(child));
                ws();
                if (i < t.size() && t[i] == ',') { ++i; continue; }
                if (i < t.size() && t[i] == ']') { ++i; break; }
                return false;
            }
        } else if (c == '"') {
            v.kind = JsonValue::Str;
            ok = string(v.s);
        } else if (lit("true")) {
            v.kind = JsonValue::Bool; v.b = true;
        } else if (lit("false")) {
            v.kind = JsonValue::Bool; v.b = false;
        } else if (lit("null")) {
            v.kind = JsonValue::Null;
        } else {
            v.kind = JsonValue::Num;
            size_t b = i;
            while (i < t.size() && (std::strchr("+-0123456789.eE", t[i]) != nullptr)) ++i;
            if (b == i) return false;
            v.s = std::string(t.substr(b, i - b));
        }
        --depth;
        return ok;
    }
};
}  // namespace

bool parse_json(std::string_view text, JsonValue& out) {
    JsonParser p{text};
    if (!p.value(out)) return false;
    p.ws();
    return p.i == text.size();
}

// ------------------------------------------------------------- threading
namespace {

// Persistent workers for parallel_for: an analysis runs three or four
// parallel phases of ~1 ms (blob inflation, per-file analysis, resolution)
// and spawning 16 threads per phase cost about as much as the resolution
// itself.  One job at a time (a concurrent caller falls back to its own
// threads); the caller works too.  A forked child (multiprocessing) starts a
// fresh pool: the parent's threads do not exist there.
class WorkerPool {
public:
    static WorkerPool& get() {
        static std::mutex mu;
        static WorkerPool* pool = nullptr;
        std::lock_guard<std::mutex> lk(mu);
        if (pool == nullptr || pool->pid_ != ::getpid()) pool = new WorkerPool();  // a stale one is leaked, never touched
        return *pool;
    }

    // fn(i) for i < n on `want` threads (caller included); false when busy
    bool run(size_t n, int want, const std::function<void(size_t)>& fn) {
        std::unique_lock<std::mutex> job(busy_, std::try_to_lock);
        if (!job.owns_lock()) return false;
        const int helpers = want - 1;
        {
            std::lock_guard<std::mutex> lk(mu_);
            while ((int)threads_.size() < helpers) {
                const int idx = (int)threads_.size();
                threads_.emplace_back([this, idx] { worker(idx); });
                threads_.back().detach();
            }
            fn_ = &fn;
            n_ = n;
            next_.store(0, std::memory_order_relaxed);
            active_ = helpers;
            remaining_ = helpers;
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return remaining_ == 0; });
        fn_ = nullptr;
        return true;
    }

private:
    WorkerPool() : pid_(::getpid()) {}

    void drain() {
        for (;;) {
            const size_t i = next_.fetch_add(1, std::memory_order_relaxed);
            if (i >= n_) break;
            (*fn_)(i);
        }
    }

    void worker(int idx) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (idx >= active_) continue;  // not needed for this job
            }
            drain();
            std::lock_guard<std::mutex> lk(mu_);
            if (--remaining_ == 0) done_.notify_one();
        }
    }

    const pid_t pid_;
    std::mutex busy_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> threads_;
    uint64_t gen_ = 0;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0;
    int active_ = 0, remaining_ = 0;
    std::atomic<size_t> next_{0};
};

}  // namespace

void parallel_for(size_t n, int threads, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    int hw = (int)std::thread::hardware_concurrency();
    if (hw <= 0) hw = 4;
    // default: the machine's threads, at most 32 (a 256-thread host shares
    // its CPUs among one process per GPU; ~2,000-file phases gain nothing past that)
    int t = threads > 0 ? threads : std::min(hw, 32);
    if ((size_t)t > n) t = (int)n;
    if (t <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    if (t <= 64 && WorkerPool::get().run(n, t, fn)) return;
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    pool.reserve(t);
    for (int w = 0; w < t; ++w) {
        pool.emplace_back([&]() {
            for (;;) {
                size_t i = next.fetch_add(1, std::memory_order_relaxed);
                if (i >= n) break;
                fn(i);
            }
        });
    }
    for (auto& th : pool) th.join();
}

// ----------------------------------------------------------------- files
namespace {

constexpr std::string_view kVfsPrefix = "/__vfs__/";

// A mounted file: a view of its content.
struct VEntry {
    std::string_view data;
};

struct VirtualTree {
    std::vector<std::string> owned;        // contents copied in (vfs_mount)
    std::deque<VEntry> entries;            // mount order; stable addresses
    std::unordered_map<std::string, VEntry*> files;  // rel path -> entry
    std::unordered_map<std::string, std::vector<std::pair<std::string, bool>>> dirs;  // rel dir -> children
};

std::mutex g_vfs_mu;
std::unordered_map<std::string, std::shared_ptr<const VirtualTree>> g_vfs;  // root -> tree
long long g_vfs_next = 0;

// Resolves a mounted path: returns the tree and sets rel ("" for the root).
std::shared_ptr<const VirtualTree> vfs_resolve(const std::string& path, std::string& rel) {
    if (path.compare(0, kVfsPrefix.size(), kVfsPrefix) != 0) return nullptr;
    size_t slash = path.find('/', kVfsPrefix.size());
    std::string root = path.substr(0, slash);
    rel = slash == std::string::npos ? std::string() : path.substr(slash + 1);
    while (!rel.empty() && rel.back() == '/') rel.pop_back();
    std::lock_guard<std::mutex> lk(g_vfs_mu);
    auto it = g_vfs.find(root);
    return it == g_vfs.end() ? nullptr : it->second;
}

}  // namespace

namespace {

// files: (path, content)
std::string mount_tree(std::shared_ptr<VirtualTree> tree, const std::vector<std::pair<std::string, std::string_view>>& files) {
    std::unordered_map<std::string, std::unordered_map<std::string, bool>> kids;  // dir -> name -> is_dir
    kids[""];
    tree->files.reserve(files.size());
    // consecutive files mostly share their directory (tree order): its
    // ancestors are registered once per run of siblings
    std::string last_dir = "\x01";
    std::unordered_map<std::string, bool>* siblings = nullptr;
    for (auto& kv : files) {
        std::string_view rel = kv.first;
        while (!rel.empty() && rel.front() == '/') rel.remove_prefix(1);
        if (rel.empty()) continue;
        const size_t slash = rel.rfind('/');
        const std::string_view dir = slash == std::string_view::npos ? std::string_view() : rel.substr(0, slash);
        if (!siblings || dir != last_dir) {
            std::string parent;
            size_t pos = 0;
            while (pos < dir.size()) {
                size_t s2 = dir.find('/', pos);
                if (s2 == std::string_view::npos) s2 = dir.size();
                std::string name(dir.substr(pos, s2 - pos));
                kids[parent].emplace(name, true);
                parent = parent.empty() ? name : parent + "/" + name;
                pos = s2 + 1;
            }
            last_dir.assign(dir);
            siblings = &kids[last_dir];  // node-based map: stays valid across inserts
        }
        siblings->emplace(std::string(rel.substr(slash == std::string_view::npos ? 0 : slash + 1)), false);
        VEntry& e = tree->entries.emplace_back();
        e.data = kv.second;
        tree->files[std::string(rel)] = &e;
    }
    for (auto& d : kids) {
        auto& v = tree->dirs[d.first];
        v.assign(d.second.begin(), d.second.end());
        std::sort(v.begin(), v.end(), [](const std::pair<std::string, bool>& a, const std::pair<std::string, bool>& b) {
            return a.first < b.first;
        });
    }
    std::lock_guard<std::mutex> lk(g_vfs_mu);
    std::string root = std::string(kVfsPrefix) + std::to_string(++g_vfs_next);
    g_vfs[root] = std::move(tree);
    return root;
}

}  // namespace

std::string vfs_mount(std::vector<std::pair<std::string, std::string>>&& files) {
    auto tree = std::make_shared<VirtualTree>();
    tree->owned.reserve(files.size());
    std::vector<std::pair<std::string, std::string_view>> views;
    views.reserve(files.size());
    for (auto& kv : files) {
        tree->owned.push_back(std::move(kv.second));
        views.emplace_back(std::move(kv.first), tree->owned.back());
    }
    return mount_tree(std::move(tree), views);
}

std::string vfs_mount_views(const std::vector<std::pair<std::string, std::string_view>>& files) {
    return mount_tree(std::make_shared<VirtualTree>(), files);
}

void vfs_unmount(const std::string& root) {
    std::lock_guard<std::mutex> lk(g_vfs_mu);
    g_vfs.erase(root);
}

bool list_dir(const std::string& dir, std::vector<std::pair<std::string, bool>>& out) {
    out.clear();
    std::string rel;
    if (auto t = vfs_resolve(dir, rel)) {
        auto it = t->dirs.find(rel);
        if (it == t->dirs.end()) return false;
        out = it->second;
        return true;
    }
    DIR* d = opendir(dir.c_str());
    if (!d) return false;
    while (dirent* e = readdir(d)) {
        std::string name = e->d_name;
        if (name == "." || name == "..") continue;
        bool is_dir = e->d_type == DT_DIR;
        if (e->d_type == DT_UNKNOWN) is_dir = dir_exists(join_path(dir, name));
        out.emplace_back(std::move(name), is_dir);
    }
    closedir(d);
    std::sort(out.begin(), out.end(),
              [](const std::pair<std::string, bool>& a, const std::pair<std::string, bool>& b) {
                  return a.first < b.first;
              });
    return true;
}

bool read_file(const std::string& path, std::string& out, size_t max_bytes) {
    std::string rel;
    if (auto t = vfs_resolve(path, rel)) {
        auto it = t->files.find(rel);
        if (it == t->files.end()) return false;
        const std::string_view* d = &it->second->data;
        if (max_bytes && d->size() > max_bytes) return false;
        out.assign(d->data(), d->size());
        return true;
    }
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (sz < 0 || (max_bytes && (size_t)sz > max_bytes)) { std::fclose(f); return false; }
    out.resize((size_t)sz);
    size_t got = sz ? std::fread(&out[0], 1, (size_t)sz, f) : 0;
    std::fclose(f);
    out.resize(got);
    return true;
}

bool file_exists(const std::string& path) {
    std::string rel;
    if (auto t = vfs_resolve(path, rel)) return t->files.count(rel) > 0;
    struct stat st;
    return ::stat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

bool dir_exists(const std::string& path) {
    std::string rel;
    if (auto t = vfs_resolve(path, rel)) return t->dirs.count(rel) > 0;
    struct stat st;
    return ::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::string join_path(const std::string& a, const std::string& b) {
    if (a.empty()) return b;
    if (b.empty()) return a;
    if (a.back() == '/') return a + b;
    return a + "/" + b;
}

std::string normalize_path(const std::string& p) {
    bool abs = !p.empty() && p[0] == '/';
    std::vector<std::string> parts;
    size_t i = 0;
    while (i <= p.size()) {
        size_t j = p.find('/', i);
        if (j == std::string::npos) j = p.size();
        std::string seg = p.substr(i, j - i);
        if (seg.empty() || seg == ".") {
        } else if (seg == "..") {
            if (!parts.empty() && parts.back() != "..") parts.pop_back();
            else if (!abs) parts.push_back("..");
        } else {
            parts.push_back(seg);
        }
        i = j + 1;
    }
    std::string out = abs ? "/" : "";
    for (size_t k = 0; k < parts.size(); ++k) {
        if (k) out += '/';
        out += parts[k];
    }
    return out;
}

std::string to_lower(std::string_view s) {
    std::string r(s);
    for (auto& c : r) if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
    return r;
}
bool starts_with(std::string_view s, std::string_view p) { return s.size() >= p.size() && s.compare(0, p.size(), p) == 0; }
bool ends_with(std::string_view s, std::string_view p) { return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0; }
bool contains(std::string_view s, std::string_view p) { return s.find(p) != std::string_view::npos; }

}  // namespace srcscan
