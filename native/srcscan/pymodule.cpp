// Python binding: dmcp._srcscan (pybind11, host C++ only).
// The GIL is released during scanning so REST/MCP threads keep serving.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/random.h>

#include <cctype>
#include <chrono>
#include <cstring>
#include <deque>
#include <memory>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bulkwriter.hpp"
#include "gitobj.hpp"
#include "graphjson.hpp"
#include "srcscan.hpp"
#include "wire.hpp"

namespace py = pybind11;

namespace {

// sequence (list / tuple) of equal-length tuples of None / int / float / str
// -> one flattened batch (CPython API directly, GIL held).  Text values are
// views into the str objects' UTF-8 buffers: the caller keeps ``rows`` alive
// (and unmodified) until the writer is done with them.
dbw::Batch to_batch(const std::string& sql, py::handle rows) {
    dbw::Batch b;
    b.sql = sql;
    PyObject* seq = PySequence_Fast(rows.ptr(), "rows must be a sequence");
    if (!seq) throw py::error_already_set();
    py::object keep = py::reinterpret_steal<py::object>(seq);
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n == 0) return b;
    PyObject** items = PySequence_Fast_ITEMS(seq);
    PyObject* first = items[0];
    if (!PyTuple_Check(first)) throw py::type_error("rows must be tuples");
    b.ncols = static_cast<int>(PyTuple_GET_SIZE(first));
    b.values.resize(static_cast<size_t>(n) * b.ncols);
    for (Py_ssize_t r = 0; r < n; ++r) {
        PyObject* row = items[r];
        if (!PyTuple_Check(row) || PyTuple_GET_SIZE(row) != b.ncols) throw py::type_error("ragged rows");
        for (int c = 0; c < b.ncols; ++c) {
            PyObject* o = PyTuple_GET_ITEM(row, c);
            dbw::Value& v = b.values[static_cast<size_t>(r) * b.ncols + c];
            if (o == Py_None) {
                v.kind = dbw::Value::Null;
            } else if (PyUnicode_Check(o)) {
                Py_ssize_t len = 0;
                const char* s = PyUnicode_AsUTF8AndSize(o, &len);
                if (!s) throw py::error_already_set();
                v.kind = dbw::Value::Text;
                v.p = s;
                v.n = static_cast<int32_t>(len);
            } else if (PyBool_Check(o) || PyLong_Check(o)) {
                v.kind = dbw::Value::Int;
                v.i = PyLong_AsLongLong(o);
                if (v.i == -1 && PyErr_Occurred()) throw py::error_already_set();
            } else if (PyFloat_Check(o)) {
                v.kind = dbw::Value::Real;
                v.d = PyFloat_AS_DOUBLE(o);
            } else {
                throw py::type_error("unsupported column value type");
            }
        }
    }
    return b;
}

// (relative path, bytes) pairs -> scan of the mounted in-memory tree (GIL released)
srcscan::ScanResult scan_mounted(py::list files, const std::string& language, int threads,
                                 const std::string& framework, bool go_doc = true) {
    const auto t = std::chrono::steady_clock::now();
    // contents are viewed in place: the (path, bytes) tuples are held
    // (immutable bytes) until the scan is done
    std::vector<py::object> hold;
    hold.reserve(files.size());
    std::vector<std::pair<std::string, std::string_view>> tree;
    tree.reserve(files.size());
    for (auto item : files) {
        auto tup = item.cast<py::tuple>();
        if (tup.size() != 2) throw py::type_error("files: (path, bytes) pairs expected");
        PyObject* content = tup[1].ptr();
        char* data = nullptr;
        Py_ssize_t n = 0;
        if (!PyBytes_Check(content) || PyBytes_AsStringAndSize(content, &data, &n) < 0)
            throw py::type_error("files: content must be bytes");
        tree.emplace_back(tup[0].cast<std::string>(), std::string_view(data, static_cast<size_t>(n)));
        hold.push_back(std::move(tup));
    }
    py::gil_scoped_release release;
    std::string root = srcscan::vfs_mount_views(tree);
    const long long mount_us =
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t).count();
    srcscan::ScanOptions opt;
    opt.language = language;
    opt.threads = threads;
    opt.framework = framework;
    opt.go_doc = go_doc;
    try {
        srcscan::ScanResult r = srcscan::scan_project(root, opt);
        r.mount_us = mount_us;
        srcscan::vfs_unmount(root);
        return r;
    } catch (...) {
        srcscan::vfs_unmount(root);
        throw;
    }
}

py::str pystr(const std::string& s) {
    PyObject* o = PyUnicode_DecodeUTF8(s.data(), static_cast<Py_ssize_t>(s.size()), "replace");
    if (!o) throw py::error_already_set();
    return py::reinterpret_steal<py::str>(o);
}

// ------------------------------------------------------------- Phase 1 rows
// json.dumps(list_of_str) with the default separators and ensure_ascii=True,
// byte for byte ('["A", "B"]', non-ASCII as \uXXXX / surrogate pairs).
void json_str_list_ascii(PyObject* seq, std::string& out) {
    static const char* hex = "0123456789abcdef";
    out.push_back('[');
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (i) out.append(", ");
        PyObject* o = items[i];
        if (!PyUnicode_Check(o)) throw py::type_error("exception names must be str");
        out.push_back('"');
        const Py_ssize_t len = PyUnicode_GET_LENGTH(o);
        const int kind = PyUnicode_KIND(o);
        const void* data = PyUnicode_DATA(o);
        for (Py_ssize_t k = 0; k < len; ++k) {
            const Py_UCS4 c = PyUnicode_READ(kind, data, k);
            auto u4 = [&](unsigned v) {
                out.append("\\u");
                for (int sh = 12; sh >= 0; sh -= 4) out.push_back(hex[(v >> sh) & 15]);
            };
            switch (c) {
                case '"': out.append("\\\""); break;
                case '\\': out.append("\\\\"); break;
                case '\n': out.append("\\n"); break;
                case '\r': out.append("\\r"); break;
                case '\t': out.append("\\t"); break;
                case '\b': out.append("\\b"); break;
                case '\f': out.append("\\f"); break;
                default:
                    if (c < 0x20 || (c >= 0x7f && c < 0x10000)) {  // outside ' '..'~'
                        u4(c);
                    } else if (c >= 0x10000) {
                        const unsigned v = c - 0x10000;
                        u4(0xd800 | (v >> 10));
                        u4(0xdc00 | (v & 0x3ff));
                    } else {
                        out.push_back((char)c);
                    }
            }
        }
        out.push_back('"');
    }
    out.push_back(']');
}

struct RowBuilder {
    dbw::Batch b;
    explicit RowBuilder(const std::string& sql, int ncols) {
        b.sql = sql;
        b.ncols = ncols;
    }
    void null() { b.values.emplace_back(); }
    void text(const char* p, Py_ssize_t n) {
        dbw::Value v;
        v.kind = dbw::Value::Text;
        v.p = p;
        v.n = static_cast<int32_t>(n);
        b.values.push_back(v);
    }
    void str(PyObject* o) {  // a str the caller keeps alive, or None
        if (o == Py_None) return null();
        Py_ssize_t n = 0;
        const char* p = PyUnicode_AsUTF8AndSize(o, &n);
        if (!p) throw py::error_already_set();
        text(p, n);
    }
    void owned(std::string&& s) {
        b.owned.push_back(std::move(s));
        text(b.owned.back().data(), (Py_ssize_t)b.owned.back().size());
    }
    void integer_or_null(PyObject* o) {
        if (o == Py_None) return null();
        dbw::Value v;
        v.kind = dbw::Value::Int;
        v.i = PyLong_AsLongLong(o);
        if (v.i == -1 && PyErr_Occurred()) throw py::error_already_set();
        b.values.push_back(v);
    }
    void integer(long long i) {
        dbw::Value v;
        v.kind = dbw::Value::Int;
        v.i = i;
        b.values.push_back(v);
    }
    bool empty() const { return b.values.empty(); }
};

PyObject* getattr_borrowed(PyObject* o, const char* name, std::vector<py::object>& hold) {
    PyObject* a = PyObject_GetAttrString(o, name);
    if (!a) throw py::error_already_set();
    hold.emplace_back(py::reinterpret_steal<py::object>(a));
    return a;
}

// One Python str per distinct value (new references handed out).
// Invalid UTF-8 in a source (Latin-1 identifiers, junk bytes) becomes U+FFFD
// instead of failing the whole project's scan with a UnicodeDecodeError.
struct StrCache {
    std::unordered_map<std::string_view, PyObject*> map;
    std::deque<std::string> owned;  // keys of values whose bytes were not valid UTF-8
    ~StrCache() {
        for (auto& kv : map) Py_DECREF(kv.second);
    }
    PyObject* get(const std::string& v) {
        auto it = map.find(std::string_view(v));
        if (it == map.end()) {
            PyObject* o = PyUnicode_DecodeUTF8(v.data(), static_cast<Py_ssize_t>(v.size()), "replace");
            if (!o) throw py::error_already_set();
            // the key views the str's own UTF-8 buffer (alive while cached) --
            // or a copy of the raw bytes when replacement changed them
            Py_ssize_t n = 0;
            const char* u = PyUnicode_AsUTF8AndSize(o, &n);
            if (!u) {
                Py_DECREF(o);
                throw py::error_already_set();
            }
            std::string_view key(u, static_cast<size_t>(n));
            if (key != std::string_view(v)) {
                owned.emplace_back(v);
                key = owned.back();
            }
            it = map.emplace(key, o).first;
        }
        return Py_NewRef(it->second);
    }
};

py::list str_list(const std::vector<std::string>& v) {
    py::list out(v.size());
    for (size_t i = 0; i < v.size(); ++i) out[i] = pystr(v[i]);
    return out;
}

// ScanResult -> Python objects without a JSON round trip: the document's
// top-level keys, "files" as tuples (path, identifier, classType, entryPoint,
// package, deps, params [(method, [ids])], methods), each method an instance
// of ``method_cls`` (a tuple subclass: StaticMethodInfo) built like
// tuple.__new__(method_cls, (name, line, httpMethod, httpPath, exceptions)).
py::dict scan_result_objects(const srcscan::ScanResult& r, py::handle method_cls) {
    if (!PyType_Check(method_cls.ptr()) || !PyType_IsSubtype((PyTypeObject*)method_cls.ptr(), &PyTuple_Type))
        throw py::type_error("method_cls must be a tuple subclass");
    auto* mtype = (PyTypeObject*)method_cls.ptr();
    py::dict d;
    d["language"] = pystr(r.language);
    d["sourceRoot"] = pystr(r.source_root);
    if (r.has_framework) {
        py::dict fw, features;
        fw["name"] = pystr(r.framework.name);
        fw["sourceRoot"] = pystr(r.framework.source_root);
        for (auto& kv : r.framework.features) features[pystr(kv.first)] = pystr(kv.second);
        fw["features"] = features;
        d["framework"] = fw;
    } else {
        d["framework"] = py::none();
    }
    if (r.language == "go") d["module"] = pystr(r.module);
    py::dict stats;
    stats["discovered"] = (long long)r.files.size() + r.skipped;
    stats["analyzed"] = (long long)r.files.size();
    stats["skipped"] = r.skipped;
    stats["elapsedUs"] = r.elapsed_us;
    py::dict phase;
    phase["mount"] = r.mount_us;
    phase["walk"] = r.walk_us;
    phase["analyze"] = r.analyze_us;
    phase["resolve"] = r.resolve_us;
    stats["phaseUs"] = phase;
    d["stats"] = stats;
    // Raw C API (no pybind temporaries): ~5x10^4 objects for a 2,000-class
    // project.  Values that repeat across files (class types, packages, HTTP
    // verbs, dependency / parameter targets, exception names) share one str.
    StrCache shared;
    auto fresh = [](const std::string& v) {
        PyObject* o = PyUnicode_DecodeUTF8(v.data(), static_cast<Py_ssize_t>(v.size()), "replace");
        if (!o) throw py::error_already_set();
        return o;
    };
    auto shared_list = [&](const std::vector<std::string>& v) {
        PyObject* l = PyList_New(static_cast<Py_ssize_t>(v.size()));
        if (!l) throw py::error_already_set();
        for (size_t i = 0; i < v.size(); ++i) PyList_SET_ITEM(l, i, shared.get(v[i]));
        return l;
    };
    py::list files(r.files.size());
    for (size_t k = 0; k < r.files.size(); ++k) {
        const srcscan::FileRec& f = r.files[k];
        PyObject* params = PyList_New(static_cast<Py_ssize_t>(f.params.size()));
        if (!params) throw py::error_already_set();
        for (size_t i = 0; i < f.params.size(); ++i) {
            PyObject* pair = PyTuple_New(2);
            if (!pair) throw py::error_already_set();
            PyTuple_SET_ITEM(pair, 0, fresh(f.params[i].first));
            PyTuple_SET_ITEM(pair, 1, shared_list(f.params[i].second));
            PyList_SET_ITEM(params, i, pair);
        }
        PyObject* methods = PyList_New(static_cast<Py_ssize_t>(f.methods.size()));
        if (!methods) throw py::error_already_set();
        for (size_t i = 0; i < f.methods.size(); ++i) {
            const srcscan::MethodRec& m = f.methods[i];
            PyObject* exc = PyTuple_New(static_cast<Py_ssize_t>(m.exceptions.size()));
            if (!exc) throw py::error_already_set();
            for (size_t j = 0; j < m.exceptions.size(); ++j) PyTuple_SET_ITEM(exc, j, shared.get(m.exceptions[j]));
            // what tuple.__new__(method_cls, fields) builds (tuple_subtype_new)
            PyObject* obj = mtype->tp_alloc(mtype, 5);
            if (!obj) throw py::error_already_set();
            PyTuple_SET_ITEM(obj, 0, fresh(m.name));
            PyTuple_SET_ITEM(obj, 1, PyLong_FromLong(m.line));
            PyTuple_SET_ITEM(obj, 2, m.has_http_method ? shared.get(m.http_method) : Py_NewRef(Py_None));
            PyTuple_SET_ITEM(obj, 3, m.has_http_path ? fresh(m.http_path) : Py_NewRef(Py_None));
            PyTuple_SET_ITEM(obj, 4, exc);
            PyList_SET_ITEM(methods, i, obj);
        }
        PyObject* rec = PyTuple_New(8);
        if (!rec) throw py::error_already_set();
        PyTuple_SET_ITEM(rec, 0, fresh(f.rel_path));
        PyTuple_SET_ITEM(rec, 1, fresh(f.identifier));
        PyTuple_SET_ITEM(rec, 2, shared.get(f.class_type));
        PyTuple_SET_ITEM(rec, 3, PyBool_FromLong(f.entry_point));
        PyTuple_SET_ITEM(rec, 4, shared.get(f.package_name));
        PyTuple_SET_ITEM(rec, 5, shared_list(f.deps));
        PyTuple_SET_ITEM(rec, 6, params);
        PyTuple_SET_ITEM(rec, 7, methods);
        PyList_SET_ITEM(files.ptr(), k, rec);
    }
    d["files"] = files;
    d["go"] = r.go_json.empty() ? py::object(py::none()) : py::object(pystr(r.go_json));
    return d;
}

// Phase 1 of the indexing pipeline (dmcp/index/pipeline.py::_phase1_static):
// class / method / parameter rows straight from the parsed units into the
// bulk writer (no per-row Python tuples), plus the graph metadata the caller
// publishes.  Same ids in the same order as the Python loop (ids[] consumed
// class, its methods, ..., then parameter links) and the same values.
// The caller keeps ``order``, ``units``, ``ids`` and the scalar strings alive
// until the writer has finished (text values are views into them).
// Time-ordered version-7 UUID strings (RFC 9562): 48-bit ms timestamp, then
// a 74-bit counter started at a random point (rand_a + rand_b), so a batch is
// strictly increasing and bulk inserts append to the primary-key B-trees.
struct Uuid7Gen {
    unsigned long long ms = 0, hi = 0, lo = 0;
    Uuid7Gen() {
        unsigned char seed[10];
        if (getrandom(seed, sizeof(seed), 0) != (ssize_t)sizeof(seed)) throw std::runtime_error("getrandom failed");
        ms = (unsigned long long)std::chrono::duration_cast<std::chrono::milliseconds>(
                 std::chrono::system_clock::now().time_since_epoch())
                 .count();
        // counter: 12 bits (rand_a) + 62 bits (rand_b); start in the lower half to avoid overflow
        hi = ((unsigned long long)(seed[0] & 0x07) << 8) | seed[1];  // 11 bits
        for (int j = 2; j < 10; ++j) lo = (lo << 8) | seed[j];
        lo &= 0x1FFFFFFFFFFFFFFFull;  // 61 bits
    }
    void next(char* s) {  // 36 chars
        static const char* hex = "0123456789abcdef";
        unsigned char b[16];
        for (int j = 0; j < 6; ++j) b[j] = (unsigned char)(ms >> (8 * (5 - j)));
        b[6] = (unsigned char)(0x70 | ((hi >> 8) & 0x0F));
        b[7] = (unsigned char)(hi & 0xFF);
        b[8] = (unsigned char)(0x80 | ((lo >> 56) & 0x3F));
        for (int j = 9; j < 16; ++j) b[j] = (unsigned char)(lo >> (8 * (15 - j)));
        if (++lo >> 62) {
            lo = 0;
            ++hi;
        }
        int k = 0;
        for (int j = 0; j < 16; ++j) {
            if (j == 4 || j == 6 || j == 8 || j == 10) s[k++] = '-';
            s[k++] = hex[b[j] >> 4];
            s[k++] = hex[b[j] & 15];
        }
    }
};

// json.dumps(list_of_str) (default separators, ensure_ascii) of UTF-8 strings
void json_ascii_list(const std::vector<std::string>& v, std::string& out) {
    static const char* hex = "0123456789abcdef";
    auto u4 = [&](unsigned c) {
        out += "\\u";
        for (int sh = 12; sh >= 0; sh -= 4) out += hex[(c >> sh) & 15];
    };
    out = "[";
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) out += ", ";
        out += '"';
        const std::string& s = v[i];
        for (size_t k = 0; k < s.size();) {
            unsigned char c = (unsigned char)s[k];
            unsigned cp = c;
            size_t len = 1;
            if (c >= 0xF0 && k + 3 < s.size() + 0) { cp = ((c & 7u) << 18) | ((s[k + 1] & 63u) << 12) | ((s[k + 2] & 63u) << 6) | (s[k + 3] & 63u); len = 4; }
            else if (c >= 0xE0 && k + 2 < s.size()) { cp = ((c & 15u) << 12) | ((s[k + 1] & 63u) << 6) | (s[k + 2] & 63u); len = 3; }
            else if (c >= 0xC0 && k + 1 < s.size()) { cp = ((c & 31u) << 6) | (s[k + 1] & 63u); len = 2; }
            k += len;
            if (cp == '"') out += "\\\"";
            else if (cp == '\\') out += "\\\\";
            else if (cp == '\n') out += "\\n";
            else if (cp == '\r') out += "\\r";
            else if (cp == '\t') out += "\\t";
            else if (cp == '\b') out += "\\b";
            else if (cp == '\f') out += "\\f";
            else if (cp < 0x20 || (cp >= 0x7f && cp < 0x10000)) u4(cp);
            else if (cp >= 0x10000) {
                cp -= 0x10000;
                u4(0xD800 + (cp >> 10));
                u4(0xDC00 + (cp & 0x3FF));
            } else out += (char)cp;
        }
        out += '"';
    }
    out += "]";
}

// Class and method rows of a finished scan handed to the bulk writer at once
// (before any Python object exists), so the inserts start while the caller
// still builds the graph; Phase 1 then only binds the ids (phase1_rows with
// pre_ids) and writes the parameter rows.  Java / TypeScript units (a later
// file with the same identifier replaces the earlier one, as
// parsers/base.py::_add_unit does); Go merges files per package: not here.
// The rows view the ScanResult's strings and one id buffer, which the
// batches keep alive (freed on the writer thread after the inserts).
struct StaticRowsSpec {
    dbw::BulkWriter* writer = nullptr;
    std::string pid, now, commit, cls_sql, meth_sql;
    bool commit_null = false;
};

struct StaticRowsKeep {
    std::shared_ptr<const srcscan::ScanResult> r;
    StaticRowsSpec spec;
    std::string ids;                  // 36 chars per id: per emitted file its class id, then its method ids
    std::vector<size_t> first;        // per file: offset of its class id in `ids` (npos: replaced file)
    std::deque<std::string> strings;  // JSON exception lists
};

const std::string& normalize_class_type(const std::string& t) {
    static const std::string kTypes[] = {"CONTROLLER", "SERVICE", "REPOSITORY", "ENTITY", "DTO",
                                         "CONFIGURATION", "LISTENER", "UTILITY", "EXCEPTION", "OTHER"};
    for (const std::string& k : kTypes) {
        if (k.size() != t.size()) continue;
        bool eq = true;
        for (size_t i = 0; i < t.size() && eq; ++i) eq = std::toupper((unsigned char)t[i]) == k[i];
        if (eq) return k;
    }
    return kTypes[9];  // ClassType.from_string: OTHER
}

// GIL not needed: reads the (const) ScanResult, which a concurrent Python
// object build may read too
void emit_static_rows(const std::shared_ptr<StaticRowsKeep>& keep) {
    const srcscan::ScanResult& r = *keep->r;
    const StaticRowsSpec& spec = keep->spec;
    std::unordered_map<std::string_view, size_t> last;
    last.reserve(r.files.size() * 2);
    size_t n_ids = 0;
    for (size_t k = 0; k < r.files.size(); ++k) last[r.files[k].identifier] = k;
    for (size_t k = 0; k < r.files.size(); ++k)
        if (last[r.files[k].identifier] == k) n_ids += 1 + r.files[k].methods.size();
    keep->ids.resize(36 * n_ids);  // never reallocated below: rows view it
    keep->first.assign(r.files.size(), std::string::npos);
    Uuid7Gen gen;
    size_t at = 0;
    const int chunk = 256;
    RowBuilder cls(spec.cls_sql, 10), meth(spec.meth_sql, 10);
    int pending = 0;
    auto flush = [&]() {
        cls.b.keep = keep;
        meth.b.keep = keep;
        if (!cls.empty()) spec.writer->put(std::move(cls.b));
        if (!meth.empty()) spec.writer->put(std::move(meth.b));
        cls = RowBuilder(spec.cls_sql, 10);
        meth = RowBuilder(spec.meth_sql, 10);
        pending = 0;
    };
    auto sv = [](RowBuilder& b, const std::string& s) { b.text(s.data(), (Py_ssize_t)s.size()); };
    for (size_t k = 0; k < r.files.size(); ++k) {
        const srcscan::FileRec& f = r.files[k];
        if (last[f.identifier] != k) continue;
        if (pending == chunk) flush();
        ++pending;
        keep->first[k] = at;
        const char* cid = &keep->ids[at];
        gen.next(&keep->ids[at]);
        at += 36;
        const std::string& ident = f.identifier;
        const size_t dot = ident.rfind('.');
        cls.text(cid, 36);
        sv(cls, spec.pid);
        sv(cls, ident);
        if (dot != std::string::npos) cls.text(ident.data() + dot + 1, (Py_ssize_t)(ident.size() - dot - 1));
        else sv(cls, ident);
        if (dot != std::string::npos) cls.text(ident.data(), (Py_ssize_t)dot); else cls.null();
        sv(cls, normalize_class_type(f.class_type));
        cls.null();
        sv(cls, f.rel_path);
        sv(cls, spec.now);
        if (spec.commit_null) cls.null(); else sv(cls, spec.commit);
        for (const srcscan::MethodRec& m : f.methods) {
            gen.next(&keep->ids[at]);
            meth.text(&keep->ids[at], 36);
            at += 36;
            meth.text(cid, 36);
            sv(meth, m.name);
            meth.null();
            meth.text("[]", 2);
            if (m.exceptions.empty()) {
                meth.text("[]", 2);
            } else {
                keep->strings.emplace_back();
                json_ascii_list(m.exceptions, keep->strings.back());
                sv(meth, keep->strings.back());
            }
            if (m.has_http_method) sv(meth, m.http_method); else meth.null();
            if (m.has_http_path) sv(meth, m.http_path); else meth.null();
            meth.integer(m.line);
            sv(meth, spec.now);
        }
    }
    flush();
}

py::tuple phase1_rows(dbw::BulkWriter& writer, py::list order, py::dict units, py::object ids, py::str pid,
                      py::str now, py::handle commit_hash, const std::string& cls_sql, const std::string& meth_sql,
                      const std::string& param_sql, py::handle method_info_cls, int chunk, py::object graph_targets,
                      py::object pre_ids) {
    if (!PyType_Check(method_info_cls.ptr()) ||
        !PyType_IsSubtype((PyTypeObject*)method_info_cls.ptr(), &PyTuple_Type))
        throw py::type_error("method_info_cls must be a tuple subclass");
    auto* mi_type = (PyTypeObject*)method_info_cls.ptr();
    // ids: a caller list consumed in order, or None = fresh UUIDv7s (kept
    // alive by ``generated``, returned to the caller with the metadata)
    const bool given = !ids.is_none();
    if (given && !PyList_Check(ids.ptr())) throw py::type_error("ids must be a list or None");
    // pre_ids: ident -> (class id, [method ids]) of rows already written by
    // scan_sources_objects(rows=...): only the ids are bound here, the
    // class / method rows are not written again
    const bool pre = !pre_ids.is_none();
    if (pre && (given || !PyDict_Check(pre_ids.ptr()))) throw py::type_error("pre_ids must be a dict (and ids None)");
    const Py_ssize_t n_ids = given ? PyList_GET_SIZE(ids.ptr()) : 0;
    Py_ssize_t next_id = 0;
    py::list generated;
    Uuid7Gen gen;
    auto nid = [&]() -> PyObject* {
        if (given) {
            if (next_id >= n_ids) throw py::value_error("phase1_rows: ran out of ids");
            return PyList_GET_ITEM(ids.ptr(), next_id++);
        }
        char buf[36];
        gen.next(buf);
        PyObject* o = PyUnicode_FromStringAndSize(buf, 36);
        if (!o || PyList_Append(generated.ptr(), o) < 0) {
            Py_XDECREF(o);
            throw py::error_already_set();
        }
        Py_DECREF(o);  // the list holds it
        return o;
    };
    static const std::string empty_list = "[]";
    py::dict class_ids, class_types, method_infos, methods_by_ident, links;
    // graph_targets = (class_ids, node_info, method_info, mparams, nodes,
    // NodeInfo, MethodParameterLink) of the ProjectGraph being built: filled
    // in place, as ProjectGraph.load_static_metadata would from the returned
    // dicts (which then stay empty, class_ids aside)
    const bool direct = !graph_targets.is_none();
    py::dict g_node_info, g_method_info, g_mparams, g_nodes;
    PyTypeObject *ni_type = nullptr, *mpl_type = nullptr;
    if (direct) {
        py::tuple gt = graph_targets.cast<py::tuple>();
        if (gt.size() != 7) throw py::value_error("graph_targets must have 7 items");
        class_ids = gt[0].cast<py::dict>();
        g_node_info = gt[1].cast<py::dict>();
        g_method_info = gt[2].cast<py::dict>();
        g_mparams = gt[3].cast<py::dict>();
        g_nodes = gt[4].cast<py::dict>();
        for (int k : {5, 6})
            if (!PyType_Check(gt[k].ptr()) || !PyType_IsSubtype((PyTypeObject*)gt[k].ptr(), &PyTuple_Type))
                throw py::type_error("graph_targets record types must be tuple subclasses");
        ni_type = (PyTypeObject*)gt[5].ptr();
        mpl_type = (PyTypeObject*)gt[6].ptr();
    }
    auto make_record = [](PyTypeObject* type, PyObject* fields) -> PyObject* {
        py::tuple args = py::make_tuple(py::reinterpret_borrow<py::object>(fields));
        PyObject* r = PyTuple_Type.tp_new(type, args.ptr(), nullptr);
        if (!r) throw py::error_already_set();
        return r;
    };
    std::vector<py::object> hold;  // attribute values fetched from the units
    long long n_cls = 0, n_meth = 0, n_par = 0;
    RowBuilder cls(cls_sql, 10), meth(meth_sql, 10);
    int pending = 0;
    auto flush = [&]() {
        if (!cls.empty()) writer.put(std::move(cls.b));
        if (!meth.empty()) writer.put(std::move(meth.b));
        cls = RowBuilder(cls_sql, 10);
        meth = RowBuilder(meth_sql, 10);
        pending = 0;
    };
    PyObject* none_tuple = PyTuple_New(0);
    py::object keep_empty = py::reinterpret_steal<py::object>(none_tuple);
    const Py_ssize_t n_order = PyList_GET_SIZE(order.ptr());
    for (Py_ssize_t oi = 0; oi < n_order; ++oi) {
        PyObject* ident = PyList_GET_ITEM(order.ptr(), oi);
        PyObject* unit = PyDict_GetItemWithError(units.ptr(), ident);
        if (!unit) {
            if (PyErr_Occurred()) throw py::error_already_set();
            continue;
        }
        if (pending == chunk) flush();
        ++pending;
        PyObject* pre_mids = nullptr;
        PyObject* cid;
        if (pre) {
            PyObject* rec = PyDict_GetItemWithError(pre_ids.ptr(), ident);
            if (!rec) {
                if (PyErr_Occurred()) throw py::error_already_set();
                throw py::value_error("phase1_rows: a unit has no pre-written row");
            }
            if (!PyTuple_Check(rec) || PyTuple_GET_SIZE(rec) != 2 || !PyList_Check(PyTuple_GET_ITEM(rec, 1)))
                throw py::type_error("pre_ids values must be (class id, [method ids])");
            cid = PyTuple_GET_ITEM(rec, 0);
            pre_mids = PyTuple_GET_ITEM(rec, 1);
        } else {
            cid = nid();
        }
        if (PyDict_SetItem(class_ids.ptr(), ident, cid) < 0) throw py::error_already_set();
        PyObject* ct_enum = getattr_borrowed(unit, "class_type", hold);
        PyObject* ct = getattr_borrowed(ct_enum, "value", hold);
        PyObject* src = getattr_borrowed(unit, "source_file", hold);
        // simple / package name: views into the identifier's UTF-8 bytes
        Py_ssize_t ilen = 0;
        const char* is = PyUnicode_AsUTF8AndSize(ident, &ilen);
        if (!is) throw py::error_already_set();
        Py_ssize_t dot = -1;
        for (Py_ssize_t k = ilen - 1; k >= 0; --k)
            if (is[k] == '.') {
                dot = k;
                break;
            }
        if (!pre) {
            cls.str(cid);
            cls.str(pid.ptr());
            cls.text(is, ilen);
            if (dot >= 0) cls.text(is + dot + 1, ilen - dot - 1); else cls.text(is, ilen);
            if (dot >= 0) cls.text(is, dot); else cls.null();
            cls.str(ct);
            cls.null();
            cls.str(src);
            cls.str(now.ptr());
            cls.str(commit_hash.ptr());
        }
        ++n_cls;
        if (direct) {
            PyObject* f = PyTuple_Pack(2, ct, Py_None);
            if (!f) throw py::error_already_set();
            py::object keep_f = py::reinterpret_steal<py::object>(f);
            py::object ni = py::reinterpret_steal<py::object>(make_record(ni_type, f));
            if (PyDict_SetItem(g_node_info.ptr(), ident, ni.ptr()) < 0) throw py::error_already_set();
        } else if (PyDict_SetItem(class_types.ptr(), ident, ct) < 0) {
            throw py::error_already_set();
        }
        PyObject* methods = getattr_borrowed(unit, "methods", hold);
        PyObject* mseq = PySequence_Fast(methods, "unit.methods must be a sequence");
        if (!mseq) throw py::error_already_set();
        py::object keep_mseq = py::reinterpret_steal<py::object>(mseq);
        const Py_ssize_t nm = PySequence_Fast_GET_SIZE(mseq);
        if (pre && PyList_GET_SIZE(pre_mids) != nm) throw py::value_error("phase1_rows: method ids do not match");
        py::list infos(nm), mids(nm);
        for (Py_ssize_t k = 0; k < nm; ++k) {
            PyObject* m = PySequence_Fast_GET_ITEM(mseq, k);
            if (!PyTuple_Check(m) || PyTuple_GET_SIZE(m) < 5) throw py::type_error("methods must be StaticMethodInfo");
            PyObject* name = PyTuple_GET_ITEM(m, 0);
            PyObject* line = PyTuple_GET_ITEM(m, 1);
            PyObject* hm = PyTuple_GET_ITEM(m, 2);
            PyObject* hp = PyTuple_GET_ITEM(m, 3);
            PyObject* exc = PyTuple_GET_ITEM(m, 4);
            PyObject* mid = pre ? PyList_GET_ITEM(pre_mids, k) : nid();
            if (!pre) {
                meth.str(mid);
                meth.str(cid);
                meth.str(name);
                meth.null();
                meth.text(empty_list.data(), 2);
                PyObject* eseq = PySequence_Fast(exc, "exceptions must be a sequence");
                if (!eseq) throw py::error_already_set();
                py::object keep_e = py::reinterpret_steal<py::object>(eseq);
                if (PySequence_Fast_GET_SIZE(eseq) == 0) {
                    meth.text(empty_list.data(), 2);
                } else {
                    std::string js;
                    json_str_list_ascii(eseq, js);
                    meth.owned(std::move(js));
                }
                meth.str(hm);
                meth.str(hp);
                meth.integer_or_null(line);
                meth.str(now.ptr());
            }
            ++n_meth;
            // MethodInfo(name, None, (), exc, http_method, http_path, line)
            PyObject* args = PyTuple_Pack(7, name, Py_None, none_tuple, exc, hm, hp, line);
            if (!args) throw py::error_already_set();
            py::object keep_args = py::reinterpret_steal<py::object>(args);
            PyObject* info = PyTuple_Type.tp_new(mi_type, py::make_tuple(keep_args).ptr(), nullptr);
            if (!info) throw py::error_already_set();
            PyList_SET_ITEM(infos.ptr(), k, info);
            PyObject* pair = PyTuple_Pack(2, name, mid);
            if (!pair) throw py::error_already_set();
            PyList_SET_ITEM(mids.ptr(), k, pair);
        }
        if (PyDict_SetItem((direct ? g_method_info : method_infos).ptr(), ident, infos.ptr()) < 0 ||
            PyDict_SetItem(methods_by_ident.ptr(), ident, mids.ptr()) < 0)
            throw py::error_already_set();
    }
    flush();
    // parameter links (CodeContextService.java:274-291, 805-856): the first
    // method of each name that has resolved parameter types
    RowBuilder par(param_sql, 5);
    PyObject *key, *mids;
    Py_ssize_t pos = 0;
    while (PyDict_Next(methods_by_ident.ptr(), &pos, &key, &mids)) {
        PyObject* unit = PyDict_GetItemWithError(units.ptr(), key);
        if (!unit) {
            if (PyErr_Occurred()) throw py::error_already_set();
            continue;
        }
        PyObject* params = getattr_borrowed(unit, "params", hold);
        if (!PyDict_Check(params) || PyDict_GET_SIZE(params) == 0 || PyList_GET_SIZE(mids) == 0) continue;
        py::dict per;
        const Py_ssize_t nm = PyList_GET_SIZE(mids);
        for (Py_ssize_t k = 0; k < nm; ++k) {
            PyObject* pair = PyList_GET_ITEM(mids, k);
            PyObject* mname = PyTuple_GET_ITEM(pair, 0);
            PyObject* mid = PyTuple_GET_ITEM(pair, 1);
            PyObject* targets = PyDict_GetItemWithError(params, mname);
            if (!targets) {
                if (PyErr_Occurred()) throw py::error_already_set();
                continue;
            }
            const int t = PyObject_IsTrue(targets);
            if (t < 0) throw py::error_already_set();
            if (!t) continue;
            const int has = PyDict_Contains(per.ptr(), mname);
            if (has < 0) throw py::error_already_set();
            if (!has && PyDict_SetItem(per.ptr(), mname, targets) < 0) throw py::error_already_set();
            PyObject* tseq = PySequence_Fast(targets, "parameter targets must be a sequence");
            if (!tseq) throw py::error_already_set();
            py::object keep_t = py::reinterpret_steal<py::object>(tseq);
            const Py_ssize_t nt = PySequence_Fast_GET_SIZE(tseq);
            for (Py_ssize_t p = 0; p < nt; ++p) {
                PyObject* tcid = PyDict_GetItemWithError(class_ids.ptr(), PySequence_Fast_GET_ITEM(tseq, p));
                if (!tcid) {
                    if (PyErr_Occurred()) throw py::error_already_set();
                    continue;
                }
                par.str(nid());
                par.str(mid);
                par.integer(p);
                par.str(tcid);
                par.str(now.ptr());
                ++n_par;
            }
        }
        if (!PyDict_GET_SIZE(per.ptr())) continue;
        if (!direct) {
            if (PyDict_SetItem(links.ptr(), key, per.ptr()) < 0) throw py::error_already_set();
            continue;
        }
        // ProjectGraph.load_static_metadata's link pass: targets that are
        // graph nodes, as MethodParameterLink(position, target)
        const int is_node = PyDict_Contains(g_nodes.ptr(), key);
        if (is_node < 0) throw py::error_already_set();
        if (!is_node) continue;
        PyObject* gper = nullptr;
        PyObject *mname, *targets;
        Py_ssize_t ppos = 0;
        while (PyDict_Next(per.ptr(), &ppos, &mname, &targets)) {
            PyObject* tseq = PySequence_Fast(targets, "parameter targets must be a sequence");
            if (!tseq) throw py::error_already_set();
            py::object keep_t = py::reinterpret_steal<py::object>(tseq);
            py::list lks;
            const Py_ssize_t nt = PySequence_Fast_GET_SIZE(tseq);
            for (Py_ssize_t p = 0; p < nt; ++p) {
                PyObject* t = PySequence_Fast_GET_ITEM(tseq, p);
                const int in = PyDict_Contains(g_nodes.ptr(), t);
                if (in < 0) throw py::error_already_set();
                if (!in) continue;
                py::object posn = py::int_(p);
                PyObject* f = PyTuple_Pack(2, posn.ptr(), t);
                if (!f) throw py::error_already_set();
                py::object keep_f = py::reinterpret_steal<py::object>(f);
                py::object link = py::reinterpret_steal<py::object>(make_record(mpl_type, f));
                lks.append(link);
            }
            if (lks.empty()) continue;
            if (!gper) {
                gper = PyDict_GetItemWithError(g_mparams.ptr(), key);
                if (!gper) {
                    if (PyErr_Occurred()) throw py::error_already_set();
                    py::dict fresh;
                    if (PyDict_SetItem(g_mparams.ptr(), key, fresh.ptr()) < 0) throw py::error_already_set();
                    gper = fresh.ptr();  // now owned by g_mparams
                }
            }
            PyObject* lst = PyDict_GetItemWithError(gper, mname);
            if (!lst) {
                if (PyErr_Occurred()) throw py::error_already_set();
                if (PyDict_SetItem(gper, mname, lks.ptr()) < 0) throw py::error_already_set();
            } else if (PyList_SetSlice(lst, PY_SSIZE_T_MAX, PY_SSIZE_T_MAX, lks.ptr()) < 0) {  // extend
                throw py::error_already_set();
            }
        }
    }
    if (!par.empty()) writer.put(std::move(par.b));
    return py::make_tuple(n_cls, n_meth, n_par, class_ids, class_types, method_infos, methods_by_ident, links,
                          generated);
}

}  // namespace

// The Python objects of a scan (scan_result_objects) and, with rows =
// (BulkWriter, project id, now, commit hash | None, class INSERT, method
// INSERT), its class / method rows streamed to the writer from a helper thread
// while this one builds the objects (row ids in d["rowIds"]).  Shared by the
// in-process scan and the isolated child's binary result.
py::dict objects_and_rows(std::shared_ptr<const srcscan::ScanResult> shared, py::handle method_cls, py::object rows) {
    std::shared_ptr<StaticRowsKeep> keep;
    std::thread emitter;
    std::atomic<long long> emit_us{0};
    if (!rows.is_none() && shared->language != "go") {
        py::tuple rt = rows.cast<py::tuple>();
        if (rt.size() != 6) throw py::value_error("rows must have 6 items");
        keep = std::make_shared<StaticRowsKeep>();
        keep->r = shared;
        StaticRowsSpec& spec = keep->spec;
        spec.writer = &rt[0].cast<dbw::BulkWriter&>();
        spec.pid = rt[1].cast<std::string>();
        spec.now = rt[2].cast<std::string>();
        spec.commit_null = rt[3].is_none();
        if (!spec.commit_null) spec.commit = rt[3].cast<std::string>();
        spec.cls_sql = rt[4].cast<std::string>();
        spec.meth_sql = rt[5].cast<std::string>();
        emitter = std::thread([keep, &emit_us] {
            const auto t = std::chrono::steady_clock::now();
            emit_static_rows(keep);
            emit_us = std::chrono::duration_cast<std::chrono::microseconds>(
                          std::chrono::steady_clock::now() - t).count();
        });
    }
    py::dict d;
    try {
        const auto t = std::chrono::steady_clock::now();
        d = scan_result_objects(*shared, method_cls);
        py::dict(d["stats"])["phaseUs"].cast<py::dict>()["objects"] =
            std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t)
                .count();
    } catch (...) {
        if (emitter.joinable()) {
            py::gil_scoped_release release;
            emitter.join();
        }
        throw;
    }
    if (emitter.joinable()) {
        {
            py::gil_scoped_release release;
            emitter.join();
        }
        py::dict(d["stats"])["phaseUs"].cast<py::dict>()["rows"] = emit_us.load();
        py::dict row_ids;
        for (size_t k = 0; k < shared->files.size(); ++k) {
            const size_t at = keep->first[k];
            if (at == std::string::npos) continue;  // a file replaced by a later one
            const size_t nm = shared->files[k].methods.size();
            py::list mids(nm);
            for (size_t j = 0; j < nm; ++j) mids[j] = py::str(&keep->ids[at + 36 * (j + 1)], 36);
            row_ids[pystr(shared->files[k].identifier)] = py::make_tuple(py::str(&keep->ids[at], 36), mids);
        }
        d["rowIds"] = row_ids;
    }
    // the rest of the ScanResult is freed off this thread (by the
    // writer after its inserts, or here by a helper)
    keep.reset();
    std::thread([](std::shared_ptr<const srcscan::ScanResult>) {}, std::move(shared)).detach();
    return d;
}

PYBIND11_MODULE(_srcscan, m) {
    m.doc() = "Native Java / TypeScript / Go source front-ends for dmcp";
    m.def(
        "scan_project",
        [](const std::string& root, const std::string& language, int threads, const std::string& framework) {
            std::string out;
            {
                py::gil_scoped_release release;
                srcscan::ScanOptions opt;
                opt.language = language;
                opt.threads = threads;
                opt.framework = framework;
                out = srcscan::scan_project_json(root, opt);
            }
            return py::bytes(out);
        },
        py::arg("root"), py::arg("language") = "auto", py::arg("threads") = 0, py::arg("framework") = "");
    m.def(
        "scan_sources",
        [](py::list files, const std::string& language, int threads, const std::string& framework) {
            // (relative path, bytes) pairs -> a mounted in-memory tree -> the same
            // document scan_project produces for a checkout of those files
            std::vector<std::pair<std::string, std::string>> tree;
            tree.reserve(files.size());
            for (auto item : files) {
                auto tup = item.cast<py::tuple>();
                tree.emplace_back(tup[0].cast<std::string>(), tup[1].cast<std::string>());
            }
            std::string out;
            {
                py::gil_scoped_release release;
                std::string root = srcscan::vfs_mount(std::move(tree));
                srcscan::ScanOptions opt;
                opt.language = language;
                opt.threads = threads;
                opt.framework = framework;
                try {
                    out = srcscan::scan_project_json(root, opt);
                } catch (...) {
                    srcscan::vfs_unmount(root);
                    throw;
                }
                srcscan::vfs_unmount(root);
            }
            return py::bytes(out);
        },
        py::arg("files"), py::arg("language") = "auto", py::arg("threads") = 0, py::arg("framework") = "");
    m.def(
        "scan_sources_objects",
        [](py::list files, const std::string& language, int threads, const std::string& framework,
           py::handle method_cls, py::object rows, bool go_doc) {
            auto r = std::make_unique<srcscan::ScanResult>(scan_mounted(files, language, threads, framework,
                                                                        go_doc));
            return objects_and_rows(std::shared_ptr<const srcscan::ScanResult>(std::move(r)), method_cls, rows);
        },
        py::arg("files"), py::arg("language"), py::arg("threads"), py::arg("framework"), py::arg("method_cls"),
        py::arg("rows") = py::none(), py::arg("go_doc") = true,
        "scan_sources as Python objects (files as tuples, methods as method_cls) -- no JSON round trip; "
        "with rows, the class / method rows are written first (ids in 'rowIds'); go_doc=False: no "
        "go-analyzer package document (Go)");
    m.def(
        "result_objects",
        [](py::bytes blob, py::handle method_cls, py::object rows) {
            // the isolated scan child's binary ScanResult (wire.hpp) -> the
            // scan_sources_objects result, rows to the writer included
            auto r = std::make_unique<srcscan::ScanResult>();
            std::string err;
            bool ok;
            {
                char* data = nullptr;
                Py_ssize_t n = 0;
                if (PyBytes_AsStringAndSize(blob.ptr(), &data, &n) < 0) throw py::error_already_set();
                py::gil_scoped_release release;
                ok = srcscan::decode_result(std::string_view(data, static_cast<size_t>(n)), *r, err);
            }
            if (!ok) throw py::value_error("scan result: " + err);
            return objects_and_rows(std::shared_ptr<const srcscan::ScanResult>(std::move(r)), method_cls, rows);
        },
        py::arg("blob"), py::arg("method_cls"), py::arg("rows") = py::none(),
        "the binary ScanResult of `srcscan serve` as scan_sources_objects returns it (untrusted bytes: every "
        "length checked)");
    m.def(
        "encode_scan",
        [](py::list files, const std::string& language, int threads, const std::string& framework, bool go_doc) {
            // the serve child's reply, computed in process (tests)
            srcscan::ScanResult r = scan_mounted(files, language, threads, framework, go_doc);
            std::string out;
            {
                py::gil_scoped_release release;
                out = srcscan::encode_result(r, /*slim=*/true);
            }
            return py::bytes(out);
        },
        py::arg("files"), py::arg("language"), py::arg("threads"), py::arg("framework"), py::arg("go_doc") = true);
    m.def(
        "scan_file",
        [](const std::string& path, const std::string& language, const std::string& rel, const std::string& fw) {
            std::string out;
            {
                py::gil_scoped_release release;
                out = srcscan::scan_file_json(path, language, rel, fw);
            }
            return py::bytes(out);
        },
        py::arg("path"), py::arg("language"), py::arg("rel") = "", py::arg("framework") = "");
    m.def(
        "graph_json",
        [](long version, py::handle nodes, py::handle class_ids, py::handle out, py::handle entry,
           py::handle mparams, py::handle node_info, py::handle method_info) {
            graphjson::Writer w;
            try {
                graphjson::write_graph(w, version, nodes.ptr(), class_ids.ptr(), out.ptr(), entry.ptr(),
                                       mparams.ptr(), node_info.ptr(), method_info.ptr());
            } catch (const graphjson::TypeError& e) {
                throw py::type_error(e.what());
            }
            PyObject* r = PyUnicode_DecodeUTF8(w.s.data(), static_cast<Py_ssize_t>(w.s.size()), "strict");
            if (!r) throw py::error_already_set();
            return py::reinterpret_steal<py::object>(r);
        },
        "ProjectGraph JSON from its containers (byte-identical to the json.dumps path)");
    m.def(
        "analyze_source",
        [](const std::string& content, const std::string& language, const std::string& file_path,
           const std::string& fw) {
            std::string out;
            {
                py::gil_scoped_release release;
                out = srcscan::analyze_source_json(content, language, file_path, fw);
            }
            return py::bytes(out);
        },
        py::arg("content"), py::arg("language"), py::arg("file_path"), py::arg("framework") = "unknown",
        "analyse one in-memory source file (GraalJsAnalyzerEngine.analyzeFile parity)");
    m.def(
        "analyze_go",
        [](const std::string& root, int threads) {
            std::string out;
            {
                py::gil_scoped_release release;
                out = srcscan::analyze_go_project_json(root, threads);
            }
            return py::bytes(out);
        },
        py::arg("root"), py::arg("threads") = 0);
    m.def("detect_framework", [](const std::string& pkg) {
        auto fi = srcscan::detect_framework(pkg);
        py::dict features;
        for (auto& kv : fi.features) features[py::str(kv.first)] = kv.second;
        py::dict d;
        d["name"] = fi.name;
        d["sourceRoot"] = fi.source_root;
        d["features"] = features;
        return d;
    });
    m.def("detect_language", &srcscan::detect_language);
    // RFC 4122 version-4 UUID strings in bulk (the indexer needs one per class,
    // method and parameter row; uuid.uuid4() costs ~6 us each in CPython).
    m.def(
        "uuid4_batch",
        [](size_t n) {
            std::vector<unsigned char> buf(n * 16);
            size_t got = 0;
            while (got < buf.size()) {
                ssize_t r = getrandom(buf.data() + got, buf.size() - got, 0);
                if (r <= 0) throw std::runtime_error("getrandom failed");
                got += (size_t)r;
            }
            static const char* hex = "0123456789abcdef";
            py::list out(n);
            char s[36];
            for (size_t i = 0; i < n; ++i) {
                unsigned char* b = &buf[i * 16];
                b[6] = (unsigned char)((b[6] & 0x0F) | 0x40);
                b[8] = (unsigned char)((b[8] & 0x3F) | 0x80);
                int k = 0;
                for (int j = 0; j < 16; ++j) {
                    if (j == 4 || j == 6 || j == 8 || j == 10) s[k++] = '-';
                    s[k++] = hex[b[j] >> 4];
                    s[k++] = hex[b[j] & 15];
                }
                out[i] = py::str(s, 36);
            }
            return out;
        },
        py::arg("n"));
    // RFC 9562 version-7 UUIDs: 48-bit Unix-ms timestamp, then a 74-bit counter
    // seeded randomly per batch, so ids of one batch sort in generation order.
    // Row keys that arrive in key order append to the B-trees instead of
    // splitting random pages (measured ~20% cheaper inserts/deletes in SQLite).
    m.def(
        "uuid7_batch",
        [](size_t n) {
            Uuid7Gen gen;
            py::list out(n);
            char s[36];
            for (size_t i = 0; i < n; ++i) {
                gen.next(s);
                out[i] = py::str(s, 36);
            }
            return out;
        },
        py::arg("n"));

    m.def(
        "read_loose_blobs",
        [](const std::vector<std::string>& object_dirs, const std::vector<std::string>& shas, int threads,
           uint64_t max_bytes) {
            gitobj::LooseResult r;
            {
                py::gil_scoped_release release;
                r = gitobj::read_loose_blobs(object_dirs, shas, threads, max_bytes);
            }
            py::list out(shas.size());
            for (size_t i = 0; i < shas.size(); ++i) {
                if (r.found[i])
                    out[i] = py::bytes(r.data[i]);
                else
                    out[i] = py::none();
                std::string().swap(r.data[i]);
            }
            return py::make_tuple(out, r.exceeded);
        },
        py::arg("object_dirs"), py::arg("shas"), py::arg("threads") = 0, py::arg("max_bytes") = 0,
        "Loose-object blob contents (None where an object is not loose) and whether max_bytes was exceeded.");

    m.def(
        "resolve_ref",
        [](const std::string& git_dir, const std::vector<std::string>& refs) -> py::object {
            std::string commit;
            bool ok;
            {
                py::gil_scoped_release release;
                ok = gitobj::resolve_commit(git_dir, refs, commit);
            }
            if (!ok) return py::none();
            return pystr(commit);
        },
        py::arg("git_dir"), py::arg("refs"),
        "Commit id of the first resolvable ref (tags peeled) from loose refs/objects; None = ask git.");
    m.def(
        "list_tree_loose",
        [](const std::vector<std::string>& object_dirs, const std::string& commit) -> py::object {
            std::vector<std::pair<std::string, std::string>> entries;
            bool ok;
            {
                py::gil_scoped_release release;
                ok = gitobj::list_tree(object_dirs, commit, entries);
            }
            if (!ok) return py::none();
            py::list out(entries.size());
            for (size_t i = 0; i < entries.size(); ++i) {
                PyObject* path = PyUnicode_DecodeUTF8(entries[i].first.data(),
                                                      static_cast<Py_ssize_t>(entries[i].first.size()), "strict");
                if (!path) {  // not UTF-8: git's own listing decides how to present it
                    PyErr_Clear();
                    return py::none();
                }
                out[i] = py::make_tuple(py::reinterpret_steal<py::str>(path), pystr(entries[i].second));
            }
            return out;
        },
        py::arg("object_dirs"), py::arg("commit"),
        "(path, blob id) of the commit's regular files in ls-tree -r order, or None unless all trees are loose.");

    py::class_<dbw::BulkWriter>(m, "BulkWriter",
                                "One SQLite write transaction on a worker thread (see bulkwriter.hpp).")
        .def(py::init([](const std::string& path, int busy_timeout_ms, py::list setup) {
                 std::vector<dbw::Batch> stmts;
                 for (auto item : setup) {  // (sql, rows): the caller keeps ``setup`` alive
                     auto tup = item.cast<py::tuple>();
                     stmts.push_back(to_batch(tup[0].cast<std::string>(), tup[1]));
                 }
                 return new dbw::BulkWriter(path, busy_timeout_ms, std::move(stmts));
             }),
             py::arg("path"), py::arg("busy_timeout_ms"), py::arg("setup"))
        .def(
            "put", [](dbw::BulkWriter& w, const std::string& sql, py::handle rows) { w.put(to_batch(sql, rows)); },
            py::arg("sql"), py::arg("rows"))
        .def("commit", &dbw::BulkWriter::commit)
        .def("abort", &dbw::BulkWriter::abort, py::call_guard<py::gil_scoped_release>())
        .def(
            "wait",
            [](dbw::BulkWriter& w) {
                std::string err;
                {
                    py::gil_scoped_release release;
                    err = w.wait();
                }
                if (!err.empty()) throw std::runtime_error("bulk write failed: " + err);
                return w.rows_written();
            })
        .def("phase1_rows", &phase1_rows, py::arg("order"), py::arg("units"), py::arg("ids"), py::arg("pid"),
             py::arg("now"), py::arg("commit_hash"), py::arg("class_sql"), py::arg("method_sql"),
             py::arg("param_sql"), py::arg("method_info_cls"), py::arg("chunk") = 256,
             py::arg("graph_targets") = py::none(), py::arg("pre_ids") = py::none(),
             "Phase 1 rows of the parsed units straight into this writer (see phase1_rows in pymodule.cpp)")
        .def_property_readonly("rows_written", &dbw::BulkWriter::rows_written)
        .def("timings", [](const dbw::BulkWriter& w) {
            py::dict d;
            d["setup_ms"] = w.setup_ms();
            d["rows_ms"] = w.rows_ms();
            d["commit_ms"] = w.commit_ms();
            d["idle_ms"] = w.idle_ms();
            d["free_ms"] = w.free_ms();
            d["open_ms"] = w.open_ms();
            d["t_start_s"] = w.t_start();
            d["t_setup_s"] = w.t_setup();
            d["t_commit_s"] = w.t_commit();
            d["t_end_s"] = w.t_end();
            return d;
        });
    m.attr("ABI_VERSION") = 6;  // 6: scan_sources_objects(..., go_doc=)
}
