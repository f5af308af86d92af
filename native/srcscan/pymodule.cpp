// Python binding: dmcp._srcscan (pybind11, host C++ only).
// The GIL is released during scanning so REST/MCP threads keep serving.
#include <pybind11/pybind11.h>

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
    m.attr("ABI_VERSION") = 1;
}
