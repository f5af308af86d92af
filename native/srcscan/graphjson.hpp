// ProjectGraph JSON serialisation straight from the Python containers.
//
// ``ProjectGraph.to_json`` (dmcp/graph/project_graph.py) builds a dict tree
// and hands it to ``json.dumps``: ~3x the work of the encoding itself for a
// 2,000-class graph (1.3 MB of JSON, ~10^5 small objects).  This walks the
// graph's own dicts / NamedTuples with the CPython API (GIL held) and writes
// byte-identical output -- same key order, same omission of absent fields,
// same escaping as ``json.dumps(..., separators=(",", ":"), ensure_ascii=False)``.
// Anything of an unexpected type raises TypeError and the caller falls back
// to the Python encoder.
//
// Wire format parity: ProjectGraph.java toJson (:634-750) plus "version".
#pragma once

#include <Python.h>

#include <charconv>
#include <stdexcept>
#include <string>

namespace graphjson {

struct TypeError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Writer {
public:
    std::string s;

    void lit(const char* p) { s.append(p); }
    void ch(char c) { s.push_back(c); }

    void str(PyObject* o) {
        if (!PyUnicode_Check(o)) throw TypeError("expected str");
        Py_ssize_t n = 0;
        const char* p = PyUnicode_AsUTF8AndSize(o, &n);
        if (!p) throw TypeError("unencodable str");
        s.push_back('"');
        const char* run = p;
        const char* end = p + n;
        for (const char* q = p; q < end; ++q) {
            const unsigned char c = static_cast<unsigned char>(*q);
            if (c >= 0x20 && c != '"' && c != '\\') continue;
            s.append(run, q - run);
            run = q + 1;
            switch (c) {
                case '"': s.append("\\\""); break;
                case '\\': s.append("\\\\"); break;
                case '\n': s.append("\\n"); break;
                case '\r': s.append("\\r"); break;
                case '\t': s.append("\\t"); break;
                case '\b': s.append("\\b"); break;
                case '\f': s.append("\\f"); break;
                default: {
                    static const char hex[] = "0123456789abcdef";
                    char buf[6] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15]};
                    s.append(buf, 6);
                }
            }
        }
        s.append(run, end - run);
        s.push_back('"');
    }

    void integer(PyObject* o) {
        if (!PyLong_Check(o) || PyBool_Check(o)) throw TypeError("expected int");
        long long v = PyLong_AsLongLong(o);
        if (v == -1 && PyErr_Occurred()) {
            PyErr_Clear();
            throw TypeError("int out of range");
        }
        char buf[24];
        auto r = std::to_chars(buf, buf + sizeof buf, v);
        s.append(buf, r.ptr - buf);
    }

    // "key": before a value
    void key(const char* k, bool& first) {
        if (!first) s.push_back(',');
        first = false;
        s.push_back('"');
        s.append(k);
        s.append("\":");
    }
    void key(PyObject* k, bool& first) {
        if (!first) s.push_back(',');
        first = false;
        str(k);
        s.push_back(':');
    }

    // JSON array of str from any sequence
    void str_seq(PyObject* seq) {
        PyObject* fast = PySequence_Fast(seq, "expected a sequence");
        if (!fast) {
            PyErr_Clear();
            throw TypeError("expected a sequence");
        }
        const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
        PyObject** it = PySequence_Fast_ITEMS(fast);
        s.push_back('[');
        try {
            for (Py_ssize_t i = 0; i < n; ++i) {
                if (i) s.push_back(',');
                str(it[i]);
            }
        } catch (...) {
            Py_DECREF(fast);
            throw;
        }
        Py_DECREF(fast);
        s.push_back(']');
    }

    // JSON array of the keys of a dict (used as an ordered set)
    void key_list(PyObject* d) {
        if (!PyDict_Check(d)) throw TypeError("expected dict");
        s.push_back('[');
        Py_ssize_t pos = 0;
        PyObject *k, *v;
        bool first = true;
        while (PyDict_Next(d, &pos, &k, &v)) {
            if (!first) s.push_back(',');
            first = false;
            str(k);
        }
        s.push_back(']');
    }
};

inline PyObject* tuple_item(PyObject* t, Py_ssize_t i) {
    if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) <= i) throw TypeError("expected a record tuple");
    return PyTuple_GET_ITEM(t, i);
}

inline bool truthy_seq(PyObject* o) {
    if (o == Py_None) return false;
    Py_ssize_t n = PyObject_Length(o);
    if (n < 0) {
        PyErr_Clear();
        throw TypeError("expected a sized sequence");
    }
    return n > 0;
}

// nodes: {id: sourceFile}, class_ids: {id: classId}, out: {id: {dep: None}},
// entry: {id: None}, mparams: {cls: {method: [(position, target)]}},
// node_info: {id: (classType, description)}, method_info: {id: [MethodInfo]}
inline void write_graph(Writer& w, long version, PyObject* nodes, PyObject* class_ids, PyObject* out,
                        PyObject* entry, PyObject* mparams, PyObject* node_info, PyObject* method_info) {
    for (PyObject* d : {nodes, class_ids, out, entry, mparams, node_info, method_info})
        if (!PyDict_Check(d)) throw TypeError("graph containers must be dicts");
    w.s.reserve(static_cast<size_t>(PyDict_GET_SIZE(nodes)) * 640 + 256);
    w.lit("{\"version\":");
    {
        char buf[24];
        auto r = std::to_chars(buf, buf + sizeof buf, version);
        w.s.append(buf, r.ptr - buf);
    }
    Py_ssize_t pos;
    PyObject *k, *v;

    w.lit(",\"nodes\":{");
    pos = 0;
    bool first = true;
    while (PyDict_Next(nodes, &pos, &k, &v)) {
        w.key(k, first);
        w.lit("{\"sourceFile\":");
        w.str(v);
        PyObject* cid = PyDict_GetItemWithError(class_ids, k);
        if (cid) {
            w.lit(",\"classId\":");
            w.str(cid);
        } else if (PyErr_Occurred()) {
            PyErr_Clear();
            throw TypeError("bad class id key");
        }
        w.ch('}');
    }

    w.lit("},\"edges\":{");
    pos = 0;
    first = true;
    while (PyDict_Next(out, &pos, &k, &v)) {
        w.key(k, first);
        w.key_list(v);
    }

    w.lit("},\"entryPoints\":");
    w.key_list(entry);

    w.lit(",\"methodParameters\":{");
    pos = 0;
    first = true;
    while (PyDict_Next(mparams, &pos, &k, &v)) {
        w.key(k, first);
        if (!PyDict_Check(v)) throw TypeError("method parameters must be dicts");
        w.ch('{');
        Py_ssize_t p2 = 0;
        PyObject *mk, *links;
        bool f2 = true;
        while (PyDict_Next(v, &p2, &mk, &links)) {
            w.key(mk, f2);
            PyObject* fast = PySequence_Fast(links, "links");
            if (!fast) {
                PyErr_Clear();
                throw TypeError("links must be a sequence");
            }
            const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
            PyObject** it = PySequence_Fast_ITEMS(fast);
            w.ch('[');
            try {
                for (Py_ssize_t i = 0; i < n; ++i) {
                    if (i) w.ch(',');
                    w.lit("{\"position\":");
                    w.integer(tuple_item(it[i], 0));
                    w.lit(",\"target\":");
                    w.str(tuple_item(it[i], 1));
                    w.ch('}');
                }
            } catch (...) {
                Py_DECREF(fast);
                throw;
            }
            Py_DECREF(fast);
            w.ch(']');
        }
        w.ch('}');
    }

    w.lit("},\"nodeInfo\":{");
    pos = 0;
    first = true;
    while (PyDict_Next(node_info, &pos, &k, &v)) {
        w.key(k, first);
        w.ch('{');
        bool f2 = true;
        PyObject* ct = tuple_item(v, 0);
        PyObject* desc = tuple_item(v, 1);
        if (ct != Py_None) {
            w.key("classType", f2);
            w.str(ct);
        }
        if (desc != Py_None) {
            w.key("description", f2);
            w.str(desc);
        }
        w.ch('}');
    }

    w.lit("},\"methodInfo\":{");
    pos = 0;
    first = true;
    while (PyDict_Next(method_info, &pos, &k, &v)) {
        w.key(k, first);
        PyObject* fast = PySequence_Fast(v, "methods");
        if (!fast) {
            PyErr_Clear();
            throw TypeError("methods must be a sequence");
        }
        const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
        PyObject** it = PySequence_Fast_ITEMS(fast);
        w.ch('[');
        try {
            for (Py_ssize_t i = 0; i < n; ++i) {
                PyObject* m = it[i];
                if (i) w.ch(',');
                w.lit("{\"methodName\":");
                w.str(tuple_item(m, 0));
                bool f2 = false;
                PyObject* desc = tuple_item(m, 1);
                if (desc != Py_None) {
                    w.key("description", f2);
                    w.str(desc);
                }
                PyObject* logic = tuple_item(m, 2);
                if (truthy_seq(logic)) {
                    w.key("businessLogic", f2);
                    w.str_seq(logic);
                }
                PyObject* exc = tuple_item(m, 3);
                if (truthy_seq(exc)) {
                    w.key("exceptions", f2);
                    w.str_seq(exc);
                }
                PyObject* verb = tuple_item(m, 4);
                if (verb != Py_None) {
                    w.key("httpMethod", f2);
                    w.str(verb);
                }
                PyObject* path = tuple_item(m, 5);
                if (path != Py_None) {
                    w.key("httpPath", f2);
                    w.str(path);
                }
                PyObject* line = tuple_item(m, 6);
                if (line != Py_None) {
                    w.key("lineNumber", f2);
                    w.integer(line);
                }
                w.ch('}');
            }
        } catch (...) {
            Py_DECREF(fast);
            throw;
        }
        Py_DECREF(fast);
        w.ch(']');
    }
    w.lit("}}");
}

}  // namespace graphjson
