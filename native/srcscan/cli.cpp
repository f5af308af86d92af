// srcscan CLI -- the native analyzer as a standalone binary.
//
//   srcscan [-o out.json] [--lang auto|java|typescript|go] [--threads N]
//           [--framework NAME] <project-root>
//   srcscan go [-o out.json] <project-root>      go-analyzer compatible ProjectAnalysis
//   srcscan file --lang java|typescript [--rel REL] [--framework F] <file>
//
// Mirrors tools/go-analyzer/cmd/analyzer/main.go:20-59: JSON on stdout or to
// the -o file; exit status 1 on usage / I/O errors.
#include <cstdio>
#include <cstring>
#include <string>

#include "srcscan.hpp"

static int usage() {
    std::fprintf(stderr,
                 "usage: srcscan [-o out.json] [--lang L] [--threads N] [--framework F] <project-root>\n"
                 "       srcscan go [-o out.json] <project-root>\n"
                 "       srcscan file --lang java|typescript [--rel REL] [--framework F] <file>\n");
    return 1;
}

int main(int argc, char** argv) {
    std::string mode = "project", out, lang = "auto", framework, rel, target;
    int threads = 0;
    int i = 1;
    if (i < argc && (std::strcmp(argv[i], "go") == 0 || std::strcmp(argv[i], "file") == 0)) mode = argv[i++];
    for (; i < argc; ++i) {
        std::string a = argv[i];
        auto need = [&](std::string& dst) {
            if (i + 1 >= argc) return false;
            dst = argv[++i];
            return true;
        };
        if (a == "-o") { if (!need(out)) return usage(); }
        else if (a == "--lang") { if (!need(lang)) return usage(); }
        else if (a == "--framework") { if (!need(framework)) return usage(); }
        else if (a == "--rel") { if (!need(rel)) return usage(); }
        else if (a == "--threads") { std::string v; if (!need(v)) return usage(); threads = std::atoi(v.c_str()); }
        else if (a == "-h" || a == "--help") return usage();
        else if (target.empty()) target = a;
        else return usage();
    }
    if (target.empty()) return usage();
    std::string json;
    if (mode == "go") {
        if (!srcscan::file_exists(srcscan::join_path(target, "go.mod"))) {
            std::fprintf(stderr, "error: reading go.mod: %s/go.mod not found\n", target.c_str());
            return 1;
        }
        json = srcscan::analyze_go_project_json(target, threads);
    } else if (mode == "file") {
        json = srcscan::scan_file_json(target, lang, rel, framework);
    } else {
        if (!srcscan::dir_exists(target)) {
            std::fprintf(stderr, "error: %s is not a directory\n", target.c_str());
            return 1;
        }
        srcscan::ScanOptions opt;
        opt.language = lang;
        opt.threads = threads;
        opt.framework = framework;
        json = srcscan::scan_project_json(target, opt);
    }
    if (out.empty()) {
        std::fwrite(json.data(), 1, json.size(), stdout);
        std::fputc('\n', stdout);
        return 0;
    }
    FILE* f = std::fopen(out.c_str(), "wb");
    if (!f) {
        std::fprintf(stderr, "error: cannot write %s\n", out.c_str());
        return 1;
    }
    std::fwrite(json.data(), 1, json.size(), f);
    std::fclose(f);
    return 0;
}
