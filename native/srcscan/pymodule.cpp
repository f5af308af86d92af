// Python binding: dmcp._srcscan (pybind11, host C++ only).
// The GIL is released during scanning so REST/MCP threads keep serving.
#include <pybind11/pybind11.h>
#include <sys/random.h>

#include <cstring>
#include <vector>

#include "srcscan.hpp"

namespace py = pybind11;

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
    m.attr("ABI_VERSION") = 1;
}
