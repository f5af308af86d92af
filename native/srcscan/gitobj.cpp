// Loose git object reader: inflates `objects/xx/yyyy…` files on a thread pool.
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

// "blob <size>\0<content>" -> content; false on anything else
bool inflate_blob(const std::string& z, std::string& out) {
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
    if (!nul || have < 6 || std::memcmp(head, "blob ", 5) != 0) {
        inflateEnd(&s);
        return false;
    }
    size_t size = 0;
    for (const char* p = head + 5; p < nul; ++p) {
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

}  // namespace

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
        if (!inflate_blob(z, body)) return;
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
