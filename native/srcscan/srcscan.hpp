// srcscan public data model and entry points.
#pragma once

#include <string>
#include <vector>

#include "common.hpp"

namespace srcscan {

// One statically extracted method (mirrors StaticMethodInfo.java:23-29 plus
// raw parameter type names for the later cross-file resolution).
struct MethodRec {
    std::string name;
    int line = 0;
    bool has_http_method = false, has_http_path = false;
    std::string http_method, http_path;
    std::vector<std::string> exceptions;
    std::vector<std::string> param_types;  // raw names as written (language-specific)
    bool is_ctor = false;                  // Java constructor (params only for class ctors)
    bool params_eligible = true;           // Java: record ctors are not param-scanned
};

// An import as the front-end saw it.
struct ImportRec {
    std::string imported;  // Java: FQCN as written; TS: imported name / 'default' / '*'
    std::string local;     // TS local binding
    std::string source;    // TS module specifier
    bool is_static = false;
    bool is_asterisk = false;
};

// Per-file front-end result.
struct FileRec {
    std::string abs_path;
    std::string rel_path;      // relative to the project root, '/' separated
    std::string identifier;    // FQCN / dotted module path / Go package path
    std::string class_type = "OTHER";
    bool entry_point = false;
    bool parsed = false;       // false: unreadable / too large / skipped
    std::string package_name;  // Java package; Go package clause name
    std::vector<MethodRec> methods;
    std::vector<ImportRec> imports;
    // resolved by the project pass
    std::vector<std::string> deps;
    std::vector<std::pair<std::string, std::vector<std::string>>> params;  // method -> known ids
};

// ------------------------------------------------------------- front-ends
// Java (JavaSourceParser.java parity): fills package, imports, class type,
// entry point flag and methods of one compilation unit.
void analyze_java(std::string_view src, FileRec& out);

// TS/JS (analyzer-bundle extractor.ts parity).
void analyze_ts(std::string_view src, const std::string& rel_path, const std::string& framework,
                bool jsx, FileRec& out);

// Framework detection from package.json text (detector.ts parity).
struct FrameworkInfo {
    std::string name = "unknown";
    std::string source_root = "src";
    std::vector<std::pair<std::string, std::string>> features;
};
FrameworkInfo detect_framework(std::string_view package_json);

// Go: see go_frontend.cpp (project-level analysis with the types.go contract).
struct GoProject;
std::string analyze_go_project_json(const std::string& root, int threads);

// ------------------------------------------------------------- project API
struct ScanOptions {
    std::string language = "auto";  // auto | java | typescript | go
    int threads = 0;
    std::string framework;          // TS only: override detection
    size_t max_file_bytes = 5u * 1024u * 1024u;  // NodeJsGraalParser.java:57
    bool go_doc = true;             // Go only: also render the go-analyzer package document
};

// Result of a project scan (what the JSON document of project.cpp holds).
struct ScanResult {
    std::string language;
    std::string source_root = ".";
    bool has_framework = false;
    FrameworkInfo framework;
    std::string module;    // go only
    std::string go_json;   // go only: ProjectAnalysis document
    std::vector<FileRec> files;
    int skipped = 0;
    long long elapsed_us = 0;
    // wall time of the scan's phases (file discovery, per-file analysis,
    // cross-file resolution); mount_us is set by callers that mount a tree
    long long walk_us = 0, analyze_us = 0, resolve_us = 0, mount_us = 0;
};

// Scans a project root (a directory or a mounted in-memory tree).
ScanResult scan_project(const std::string& root, const ScanOptions& opt);
// The same into ``r`` (a caller that decides when the result is freed).
void scan_project_into(const std::string& root, const ScanOptions& opt, ScanResult& r);

// The same scan as a JSON document (see docs in project.cpp).
std::string scan_project_json(const std::string& root, const ScanOptions& opt);
std::string scan_result_json(const ScanResult& r);

// Single-file analysis (tests / debugging); returns the FileRec as JSON.
std::string scan_file_json(const std::string& path, const std::string& language,
                           const std::string& rel_path, const std::string& framework);
// One in-memory source (no file read): ``file_path`` names the unit.
std::string analyze_source_json(const std::string& content, const std::string& language, const std::string& file_path,
                                const std::string& framework);

std::string detect_language(const std::string& root);

}  // namespace srcscan
