// Binary wire form of a ScanResult (see wire.hpp).
#include "wire.hpp"

#include <cstdint>
#include <atomic>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace srcscan {

namespace {

struct Out {
    std::string s;
    void u8(uint8_t v) { s.push_back(static_cast<char>(v)); }
    void u32(uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
    void i64(int64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }
    void str(const std::string& v) {
        u32(static_cast<uint32_t>(v.size()));
        s.append(v);
    }
    void strs(const std::vector<std::string>& v) {
        u32(static_cast<uint32_t>(v.size()));
        for (const auto& x : v) str(x);
    }
};

struct Bad : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct In {
    const char* p;
    size_t n;
    void need(size_t k) const {
        if (k > n) throw Bad("truncated scan result");
    }
    uint8_t u8() {
        need(1);
        const uint8_t v = static_cast<uint8_t>(*p);
        ++p, --n;
        return v;
    }
    uint32_t u32() {
        need(4);
        uint32_t v;
        std::memcpy(&v, p, 4);
        p += 4, n -= 4;
        return v;
    }
    int64_t i64() {
        need(8);
        int64_t v;
        std::memcpy(&v, p, 8);
        p += 8, n -= 8;
        return v;
    }
    // a count of elements of at least `min_bytes` each: bounded by what is left
    uint32_t count(size_t min_bytes) {
        const uint32_t c = u32();
        if ((uint64_t)c * min_bytes > n) throw Bad("scan result count exceeds its payload");
        return c;
    }
    std::string str() {
        const uint32_t k = u32();
        need(k);
        std::string v(p, k);
        p += k, n -= k;
        return v;
    }
    void strs(std::vector<std::string>& v) {
        const uint32_t c = count(4);
        v.clear();
        v.reserve(c);
        for (uint32_t i = 0; i < c; ++i) v.push_back(str());
    }
};

// slim: without what only the scan's own resolution pass reads (the absolute
// path, imports, per-method parameter type names) -- the parent builds its
// objects and rows from the resolved fields alone
void put_file(Out& o, const FileRec& f, bool slim) {
    static const std::string empty;
    static const std::vector<std::string> none;
    o.str(slim ? empty : f.abs_path);
    o.str(f.rel_path);
    o.str(f.identifier);
    o.str(f.class_type);
    o.u8(static_cast<uint8_t>((f.entry_point ? 1 : 0) | (f.parsed ? 2 : 0)));
    o.str(f.package_name);
    o.u32(static_cast<uint32_t>(f.methods.size()));
    for (const MethodRec& m : f.methods) {
        o.str(m.name);
        o.u32(static_cast<uint32_t>(m.line));
        o.u8(static_cast<uint8_t>((m.has_http_method ? 1 : 0) | (m.has_http_path ? 2 : 0) | (m.is_ctor ? 4 : 0) |
                                  (m.params_eligible ? 8 : 0)));
        o.str(m.http_method);
        o.str(m.http_path);
        o.strs(m.exceptions);
        o.strs(slim ? none : m.param_types);
    }
    o.u32(static_cast<uint32_t>(slim ? 0 : f.imports.size()));
    for (const ImportRec& im : f.imports) {
        if (slim) break;
        o.str(im.imported);
        o.str(im.local);
        o.str(im.source);
        o.u8(static_cast<uint8_t>((im.is_static ? 1 : 0) | (im.is_asterisk ? 2 : 0)));
    }
    o.strs(f.deps);
    o.u32(static_cast<uint32_t>(f.params.size()));
    for (const auto& pm : f.params) {
        o.str(pm.first);
        o.strs(pm.second);
    }
}

void get_file(In& d, FileRec& f) {
    f.abs_path = d.str();
    f.rel_path = d.str();
    f.identifier = d.str();
    f.class_type = d.str();
    const uint8_t fl = d.u8();
    f.entry_point = fl & 1;
    f.parsed = (fl & 2) != 0;
    f.package_name = d.str();
    const uint32_t nm = d.count(25);
    f.methods.resize(nm);
    for (uint32_t j = 0; j < nm; ++j) {
        MethodRec& m = f.methods[j];
        m.name = d.str();
        m.line = static_cast<int>(d.u32());
        const uint8_t mf = d.u8();
        m.has_http_method = mf & 1;
        m.has_http_path = (mf & 2) != 0;
        m.is_ctor = (mf & 4) != 0;
        m.params_eligible = (mf & 8) != 0;
        m.http_method = d.str();
        m.http_path = d.str();
        d.strs(m.exceptions);
        d.strs(m.param_types);
    }
    const uint32_t ni = d.count(13);
    f.imports.resize(ni);
    for (uint32_t j = 0; j < ni; ++j) {
        ImportRec& im = f.imports[j];
        im.imported = d.str();
        im.local = d.str();
        im.source = d.str();
        const uint8_t imf = d.u8();
        im.is_static = imf & 1;
        im.is_asterisk = (imf & 2) != 0;
    }
    d.strs(f.deps);
    const uint32_t np = d.count(8);
    f.params.resize(np);
    for (uint32_t j = 0; j < np; ++j) {
        f.params[j].first = d.str();
        d.strs(f.params[j].second);
    }
}

}  // namespace

std::string encode_result(const ScanResult& r, bool slim) {
    Out o;
    o.s.reserve(64 + r.files.size() * 512 + r.go_json.size());
    o.s.append("SSW2", 4);
    o.str(r.language);
    o.str(r.source_root);
    o.u8(r.has_framework);
    o.str(r.framework.name);
    o.str(r.framework.source_root);
    o.u32(static_cast<uint32_t>(r.framework.features.size()));
    for (const auto& kv : r.framework.features) {
        o.str(kv.first);
        o.str(kv.second);
    }
    o.str(r.module);
    o.str(r.go_json);
    // the file records, encoded in parallel, behind a table of their byte
    // lengths (so the decoder splits them over threads too)
    const size_t nfiles = r.files.size();
    std::vector<std::string> recs(nfiles);
    parallel_for(nfiles, 0, [&](size_t k) {
        Out fo;
        fo.s.reserve(512);
        put_file(fo, r.files[k], slim);
        recs[k] = std::move(fo.s);
    });
    size_t total = 0;
    for (const std::string& x : recs) total += x.size();
    o.s.reserve(o.s.size() + 4 * (nfiles + 1) + total + 64);
    o.u32(static_cast<uint32_t>(nfiles));
    for (const std::string& x : recs) o.u32(static_cast<uint32_t>(x.size()));
    for (const std::string& x : recs) o.s.append(x);
    o.u32(static_cast<uint32_t>(r.skipped));
    o.i64(r.elapsed_us);
    o.i64(r.walk_us);
    o.i64(r.analyze_us);
    o.i64(r.resolve_us);
    o.i64(r.mount_us);
    return std::move(o.s);
}

bool decode_result(std::string_view in, ScanResult& r, std::string& err) {
    try {
        In d{in.data(), in.size()};
        d.need(4);
        if (std::memcmp(d.p, "SSW2", 4) != 0) throw Bad("not a scan result (bad magic)");
        d.p += 4, d.n -= 4;
        r.language = d.str();
        r.source_root = d.str();
        r.has_framework = d.u8() != 0;
        r.framework.name = d.str();
        r.framework.source_root = d.str();
        const uint32_t nf = d.count(8);
        r.framework.features.clear();
        for (uint32_t i = 0; i < nf; ++i) {
            std::string k = d.str();
            r.framework.features.emplace_back(std::move(k), d.str());
        }
        r.module = d.str();
        r.go_json = d.str();
        // the length table, checked against the bytes left, then every record
        // decoded on its own slice (in parallel) and required to fill it exactly
        const uint32_t nfiles = d.count(4 + 33);  // a length + the fixed-size part of a record
        std::vector<size_t> off(static_cast<size_t>(nfiles) + 1, 0);
        for (uint32_t k = 0; k < nfiles; ++k) {
            const uint32_t len = d.u32();
            if (len < 33) throw Bad("scan result file record too short");
            off[k + 1] = off[k] + len;
        }
        d.need(off[nfiles]);
        r.files.clear();
        r.files.resize(nfiles);
        std::atomic<bool> bad{false};
        std::string why;
        std::mutex why_mu;
        const char* base = d.p;
        parallel_for(nfiles, 0, [&](size_t k) {
            if (bad.load(std::memory_order_relaxed)) return;
            try {
                In fd{base + off[k], off[k + 1] - off[k]};
                get_file(fd, r.files[k]);
                if (fd.n != 0) throw Bad("scan result file record has trailing bytes");
            } catch (const std::exception& e) {  // Bad, or bad_alloc from a hostile length
                std::lock_guard<std::mutex> g(why_mu);
                if (!bad.exchange(true)) why = e.what();
            }
        });
        if (bad) throw Bad(why);
        d.p += off[nfiles], d.n -= off[nfiles];
        r.skipped = static_cast<int>(d.u32());
        r.elapsed_us = d.i64();
        r.walk_us = d.i64();
        r.analyze_us = d.i64();
        r.resolve_us = d.i64();
        r.mount_us = d.i64();
        if (d.n != 0) throw Bad("trailing bytes after the scan result");
        return true;
    } catch (const Bad& e) {
        err = e.what();
        return false;
    } catch (const std::bad_alloc&) {
        err = "scan result too large";
        return false;
    }
}

}  // namespace srcscan
