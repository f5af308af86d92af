// Loose git object reader: inflates `objects/xx/yyyy…` files on a thread pool,
// and resolves a ref + lists a commit's tree from loose objects (what
// `git rev-parse <ref>^{commit}` and `git ls-tree -r` report, without the two
// processes).  Anything packed or unusual makes these return false and the
// caller asks git.
//
// An in-memory snapshot (dmcp/index/source.py) needs the content of every
// source blob at one commit.  `git cat-file --batch` inflates them serially
// per process; a freshly committed repository keeps its objects loose (one
// zlib stream per file), which makes that read CPU-bound.  Here each worker
// opens, inflates and header-checks whole objects independently; objects that
// are not loose (packed) come back empty and the caller reads those through
// git, which owns the pack/delta machinery.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "gitobj.hpp"
#include "common.hpp"

namespace gitobj {

namespace {

bool slurp(const std::string& path, std::string& out) {
    int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    struct stat st;
    if (::fstat(fd, &st) != 0) {
        ::close(fd);
        return false;
    }
    out.resize(static_cast<size_t>(st.st_size));
    size_t got = 0;
    while (got < out.size()) {
        ssize_t r = ::read(fd, &out[got], out.size() - got);
        if (r <= 0) break;
        got += static_cast<size_t>(r);
    }
    ::close(fd);
    out.resize(got);
    return got > 0;
}

// "<type> <size>\0<content>" -> content (type checked against `want`, or
// returned through `type` when want is null); false on anything else
bool inflate_object(const std::string& z, std::string& out, const char* want, std::string* type = nullptr) {
    z_stream s;
    std::memset(&s, 0, sizeof(s));
    if (inflateInit(&s) != Z_OK) return false;
    s.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(z.data()));
    s.avail_in = static_cast<uInt>(z.size());
    // header first (at most "blob " + 20 digits + NUL)
    char head[32];
    s.next_out = reinterpret_cast<Bytef*>(head);
    s.avail_out = sizeof(head);
    int rc = inflate(&s, Z_SYNC_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
        inflateEnd(&s);
        return false;
    }
    size_t have = sizeof(head) - s.avail_out;
    const char* nul = static_cast<const char*>(std::memchr(head, 0, have));
    const char* sp = nul ? static_cast<const char*>(std::memchr(head, ' ', static_cast<size_t>(nul - head))) : nullptr;
    if (!sp || sp == head || sp + 1 >= nul ||
        (want && (std::strlen(want) != static_cast<size_t>(sp - head) || std::memcmp(head, want, sp - head) != 0))) {
        inflateEnd(&s);
        return false;
    }
    if (type) type->assign(head, static_cast<size_t>(sp - head));
    size_t size = 0;
    for (const char* p = sp + 1; p < nul; ++p) {
        if (*p < '0' || *p > '9') {
            inflateEnd(&s);
            return false;
        }
        size = size * 10 + static_cast<size_t>(*p - '0');
    }
    size_t body_have = have - static_cast<size_t>(nul + 1 - head);
    out.resize(size);
    if (body_have > size) {
        inflateEnd(&s);
        return false;
    }
    std::memcpy(&out[0], nul + 1, body_have);
    if (rc != Z_STREAM_END && body_have < size) {
        s.next_out = reinterpret_cast<Bytef*>(&out[body_have]);
        s.avail_out = static_cast<uInt>(size - body_have);
        rc = inflate(&s, Z_FINISH);
        body_have = size - s.avail_out;
    }
    inflateEnd(&s);
    return (rc == Z_STREAM_END || rc == Z_OK || rc == Z_BUF_ERROR) && body_have == size;
}

bool read_loose(const std::vector<std::string>& object_dirs, const std::string& sha, std::string& body,
                const char* want, std::string* type = nullptr) {
    if (sha.size() != 40) return false;
    std::string z;
    for (const std::string& d : object_dirs) {
        if (slurp(d + "/" + sha.substr(0, 2) + "/" + sha.substr(2), z)) break;
        z.clear();
    }
    return !z.empty() && inflate_object(z, body, want, type);
}

bool is_hex40(std::string_view s) {
    if (s.size() != 40) return false;
    for (char c : s)
        if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
    return true;
}

std::string trim(std::string s) {
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r' || s.back() == ' ')) s.pop_back();
    return s;
}

// git check-ref-format's rules, as far as a path on disk is concerned: a name
// git would refuse (and so never resolve) must not be read as a file here
// either -- "../../x" would otherwise leave refs/ and follow whatever "ref: "
// line it finds.  Refused names return false, so git answers instead.
bool ref_name_ok(const std::string& ref) {
    if (ref.empty() || ref.front() == '/' || ref.back() == '/' || ref.back() == '.') return false;
    if (ref.size() >= 5 && ref.compare(ref.size() - 5, 5, ".lock") == 0) return false;
    if (ref.find("..") != std::string::npos || ref.find("@{") != std::string::npos ||
        ref.find("//") != std::string::npos || ref == "@")
        return false;
    for (unsigned char c : ref) {
        if (c < 0x20 || c == 0x7f || c == ' ' || c == '~' || c == '^' || c == ':' || c == '?' || c == '*' ||
            c == '[' || c == '\\')
            return false;
    }
    size_t start = 0;  // no component may start with '.' or end with ".lock"
    while (start <= ref.size()) {
        size_t end = ref.find('/', start);
        if (end == std::string::npos) end = ref.size();
        if (end == start || ref[start] == '.') return false;
        if (end - start >= 5 && ref.compare(end - 5, 5, ".lock") == 0) return false;
        start = end + 1;
    }
    return true;
}

// a ref's target: loose ref file (symbolic refs followed), else packed-refs
bool ref_target(const std::string& git_dir, const std::string& ref, std::string& sha, int depth = 0) {
    if (depth > 5 || !ref_name_ok(ref)) return false;
    std::string text;
    if (slurp(git_dir + "/" + ref, text)) {
        text = trim(text);
        if (text.rfind("ref: ", 0) == 0) return ref_target(git_dir, text.substr(5), sha, depth + 1);
        if (!is_hex40(text)) return false;
        sha = text;
        return true;
    }
    if (ref == "HEAD" || !slurp(git_dir + "/packed-refs", text)) return false;
    size_t pos = 0;
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size();
        std::string_view line(text.data() + pos, eol - pos);
        if (line.size() > 41 && line[40] == ' ' && line.substr(41) == ref && is_hex40(line.substr(0, 40))) {
            sha.assign(line.substr(0, 40));
            return true;
        }
        pos = eol + 1;
    }
    return false;
}

void hex20(const unsigned char* b, std::string& out) {
    static const char* hx = "0123456789abcdef";
    out.resize(40);
    for (int i = 0; i < 20; ++i) {
        out[2 * i] = hx[b[i] >> 4];
        out[2 * i + 1] = hx[b[i] & 15];
    }
}

// ls-tree -r order: entries in tree order, subtrees expanded in place
bool walk_tree(const std::vector<std::string>& object_dirs, const std::string& tree_sha, const std::string& prefix,
               std::vector<std::pair<std::string, std::string>>& out, int depth) {
    if (depth > 256) return false;
    std::string body;
    if (!read_loose(object_dirs, tree_sha, body, "tree")) return false;
    size_t p = 0;
    std::string sha;
    while (p < body.size()) {
        size_t sp = body.find(' ', p);
        if (sp == std::string::npos) return false;
        size_t nul = body.find('\0', sp);
        if (nul == std::string::npos || nul + 21 > body.size()) return false;
        std::string_view mode(body.data() + p, sp - p);
        std::string name = prefix + body.substr(sp + 1, nul - sp - 1);
        hex20(reinterpret_cast<const unsigned char*>(body.data() + nul + 1), sha);
        p = nul + 21;
        if (mode == "40000") {
            if (!walk_tree(object_dirs, sha, name + "/", out, depth + 1)) return false;
        } else if (mode == "100644" || mode == "100755" || mode == "100664") {
            out.emplace_back(std::move(name), sha);
        } else if (mode != "120000" && mode != "160000") {
            return false;  // unknown mode: let git decide
        }
    }
    return true;
}

}  // namespace

bool read_loose_blob(const std::vector<std::string>& object_dirs, const std::string& sha, std::string& out) {
    return read_loose(object_dirs, sha, out, "blob");
}

bool resolve_commit(const std::string& git_dir, const std::vector<std::string>& refs, std::string& commit) {
    std::vector<std::string> object_dirs{git_dir + "/objects"};
    std::string alt;
    if (slurp(git_dir + "/objects/info/alternates", alt)) {
        size_t pos = 0;
        while (pos < alt.size()) {
            size_t eol = alt.find('\n', pos);
            if (eol == std::string::npos) eol = alt.size();
            std::string line = trim(alt.substr(pos, eol - pos));
            if (!line.empty() && line[0] != '#') object_dirs.push_back(line);
            pos = eol + 1;
        }
    }
    for (const std::string& ref : refs) {
        std::string sha;
        if (!ref_target(git_dir, ref, sha)) continue;
        // peel annotated tags down to the commit (`<ref>^{commit}`)
        for (int hop = 0; hop < 8; ++hop) {
            std::string body, type;
            if (!read_loose(object_dirs, sha, body, nullptr, &type)) return false;  // packed: git decides
            if (type == "commit") {
                commit = sha;
                return true;
            }
            if (type != "tag" || body.rfind("object ", 0) != 0 || body.size() < 47) break;
            sha = body.substr(7, 40);
            if (!is_hex40(sha)) break;
        }
        return false;  // the ref exists but does not name a commit: git's error path
    }
    return false;
}

bool list_tree(const std::vector<std::string>& object_dirs, const std::string& commit,
               std::vector<std::pair<std::string, std::string>>& out) {
    std::string body;
    if (!read_loose(object_dirs, commit, body, "commit")) return false;
    if (body.rfind("tree ", 0) != 0 || body.size() < 45) return false;
    const std::string tree = body.substr(5, 40);
    if (!is_hex40(tree)) return false;
    out.clear();
    return walk_tree(object_dirs, tree, "", out, 0);
}

LooseResult read_loose_blobs(const std::vector<std::string>& object_dirs, const std::vector<std::string>& shas,
                             int threads, uint64_t max_bytes) {
    LooseResult r;
    r.data.resize(shas.size());
    r.found.assign(shas.size(), 0);
    std::atomic<uint64_t> total{0};
    std::atomic<bool> exceeded{false};
    srcscan::parallel_for(shas.size(), threads, [&](size_t i) {
        if (exceeded.load(std::memory_order_relaxed)) return;
        const std::string& sha = shas[i];
        if (sha.size() < 4) return;
        std::string z;
        for (const std::string& d : object_dirs) {
            if (slurp(d + "/" + sha.substr(0, 2) + "/" + sha.substr(2), z)) break;
            z.clear();
        }
        if (z.empty()) return;
        std::string body;
        if (!inflate_object(z, body, "blob")) return;
        uint64_t t = total.fetch_add(body.size(), std::memory_order_relaxed) + body.size();
        if (max_bytes && t > max_bytes) exceeded.store(true, std::memory_order_relaxed);
        r.data[i] = std::move(body);
        r.found[i] = 1;
    });
    r.total_bytes = total.load();
    r.exceeded = exceeded.load();
    return r;
}

}  // namespace gitobj
