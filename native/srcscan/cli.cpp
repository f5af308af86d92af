// srcscan CLI -- the native analyzer as a standalone binary.
//
//   srcscan [-o out.json] [--lang auto|java|typescript|go] [--threads N]
//           [--framework NAME] <project-root>
//   srcscan go [-o out.json] <project-root>      go-analyzer compatible ProjectAnalysis
//   srcscan file --lang java|typescript [--rel REL] [--framework F] <file>
//   srcscan stdin [--lang L] [--threads N] [--framework F]
//           a project streamed on stdin (u64 LE file count, then per file a
//           u64 LE length + relative path and a u64 LE length + contents) --
//           the isolated scan of an in-memory snapshot (dmcp/parsers/isolated.py):
//           the untrusted parse runs in this short-lived process, which starts
//           in milliseconds (the Python child took ~100 ms to import)
//   srcscan serve
//           the persistent isolated scan child: per request on stdin a u64 LE
//           length + header text ("language\nthreads\nframework\ngo_doc"), the
//           project stream of `stdin`; per request on stdout a u8 status (0 ok,
//           1 error) + u64 LE length + the binary ScanResult (wire.hpp) or the
//           error message.  Exits 0 at end of input, 3 on a truncated request.
//
// Mirrors tools/go-analyzer/cmd/analyzer/main.go:20-59: JSON on stdout or to
// the -o file; exit status 1 on usage / I/O errors.
#include <chrono>
#include <csignal>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "common.hpp"
#include "srcscan.hpp"
#include "wire.hpp"

static bool read_exact(void* dst, size_t n) {
    return n == 0 || std::fread(dst, 1, n, stdin) == n;
}

static bool read_blob(std::string& out) {
    uint64_t n = 0;
    if (!read_exact(&n, sizeof n) || n > (uint64_t(1) << 34)) return false;
    out.resize((size_t)n);
    return read_exact(out.data(), (size_t)n);
}

// fault injection for the isolation tests (DMCP_SCAN_CHILD_FAULT=hang|crash)
static void injected_fault() {
    const char* f = std::getenv("DMCP_SCAN_CHILD_FAULT");
    if (!f) return;
    if (std::strcmp(f, "hang") == 0) std::this_thread::sleep_for(std::chrono::hours(1));
    if (std::strcmp(f, "crash") == 0) std::raise(SIGSEGV);  // as a front-end fault would
}

static int scan_stdin(const srcscan::ScanOptions& opt, std::string& json) {
    uint64_t nfiles = 0;
    if (!read_exact(&nfiles, sizeof nfiles)) return 3;
    std::vector<std::pair<std::string, std::string>> tree;
    tree.reserve((size_t)nfiles);
    for (uint64_t k = 0; k < nfiles; ++k) {
        std::string rel, data;
        if (!read_blob(rel) || !read_blob(data)) return 3;
        tree.emplace_back(std::move(rel), std::move(data));
    }
    injected_fault();
    std::string root = srcscan::vfs_mount(std::move(tree));
    json = srcscan::scan_project_json(root, opt);
    srcscan::vfs_unmount(root);
    return 0;
}

static bool write_exact(const void* src, size_t n) { return n == 0 || std::fwrite(src, 1, n, stdout) == n; }

// one request of `serve` after its header: the tree, the scan, the framed reply
static int serve_one(const std::string& header) {
    srcscan::ScanOptions opt;
    {
        std::vector<std::string> f;
        size_t a = 0;
        for (;;) {
            const size_t b = header.find('\n', a);
            f.push_back(header.substr(a, b == std::string::npos ? std::string::npos : b - a));
            if (b == std::string::npos) break;
            a = b + 1;
        }
        if (f.size() != 4) return 3;
        opt.language = f[0].empty() ? "auto" : f[0];
        opt.threads = std::atoi(f[1].c_str());
        opt.framework = f[2];
        opt.go_doc = f[3] != "0";
    }
    uint64_t nfiles = 0;
    if (!read_exact(&nfiles, sizeof nfiles) || nfiles > (uint64_t(1) << 24)) return 3;
    std::vector<std::pair<std::string, std::string>> tree;
    tree.reserve((size_t)nfiles);
    for (uint64_t k = 0; k < nfiles; ++k) {
        std::string rel, data;
        if (!read_blob(rel) || !read_blob(data)) return 3;
        tree.emplace_back(std::move(rel), std::move(data));
    }
    injected_fault();
    uint8_t status = 0;
    std::string payload;
    std::string root = srcscan::vfs_mount(std::move(tree));
    srcscan::ScanResult res;  // freed after the reply is out (~160k strings at 2,000 files)
    try {
        srcscan::scan_project_into(root, opt, res);
        payload = srcscan::encode_result(res, /*slim=*/true);
    } catch (const std::exception& e) {
        status = 1;
        payload = e.what();
    }
    const uint64_t n = payload.size();
    const bool ok = write_exact(&status, 1) && write_exact(&n, sizeof n) &&
                    write_exact(payload.data(), payload.size()) && std::fflush(stdout) == 0;
    srcscan::vfs_unmount(root);  // the tree too
    return ok ? 0 : 1;
}

static int serve() {
    for (;;) {
        uint64_t hn = 0;
        const size_t got = std::fread(&hn, 1, sizeof hn, stdin);
        if (got == 0) return 0;  // end of input: the parent is done with this child
        if (got != sizeof hn || hn > 4096) return 3;
        std::string header((size_t)hn, '\0');
        if (!read_exact(header.data(), header.size())) return 3;
        const int rc = serve_one(header);
        if (rc != 0) return rc;
    }
}

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
    if (i < argc && std::strcmp(argv[i], "serve") == 0) return serve();
    if (i < argc && (std::strcmp(argv[i], "go") == 0 || std::strcmp(argv[i], "file") == 0 ||
                     std::strcmp(argv[i], "stdin") == 0))
        mode = argv[i++];
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
    if (target.empty() && mode != "stdin") return usage();
    std::string json;
    if (mode == "stdin") {
        srcscan::ScanOptions opt;
        opt.language = lang;
        opt.threads = threads;
        opt.framework = framework;
        int rc = scan_stdin(opt, json);
        if (rc != 0) {
            std::fprintf(stderr, "error: truncated project stream on stdin\n");
            return rc;
        }
    } else if (mode == "go") {
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
