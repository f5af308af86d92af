// Project-level orchestration: discovery, parallel per-file analysis and the
// cross-file resolution pass (dependencies, entry points, parameter links).
//
// This is the native counterpart of SourceParser.parse (SourceParser.java:146-194)
// plus the language hooks of JavaSourceParser / NodeJsGraalParser /
// GoSourceParser.  Every file is read and analysed once, in parallel; the
// reference re-parses Java files in every pass.
//
// Output JSON document:
// {
//   "language": "java" | "typescript" | "go",
//   "sourceRoot": "src/main/java" | "src" | "app" | ".",
//   "framework": {"name", "sourceRoot", "features": {..}} | null,
//   "module": "<go module>" (go only),
//   "stats": {"discovered", "analyzed", "skipped", "elapsedMs"},
//   "files": [{ "path", "identifier", "classType", "entryPoint", "package",
//               "deps": [...], "params": {method: [ids]},
//               "methods": [{"name", "line", "httpMethod", "httpPath", "exceptions"}] }],
//   "go": { ProjectAnalysis } (go only, when requested)
// }
#include <algorithm>
#include <chrono>
#include <dirent.h>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "srcscan.hpp"

namespace srcscan {

void go_project_files(const std::string& root, int threads, std::string& module, std::vector<FileRec>& files,
                      std::string* go_json);

namespace {

struct Entry {
    std::string name;
    bool is_dir;
};

std::vector<Entry> entries(const std::string& dir) {
    std::vector<std::pair<std::string, bool>> raw;
    std::vector<Entry> out;
    if (!list_dir(dir, raw)) return out;  // sorted by name; real or mounted tree
    out.reserve(raw.size());
    for (auto& e : raw) out.push_back({std::move(e.first), e.second});
    return out;
}

// Recursive walk collecting relative paths of files accepted by `keep`;
// directories rejected by `skip_dir` are pruned.
template <class Keep, class SkipDir>
void walk(const std::string& abs, const std::string& rel, Keep keep, SkipDir skip_dir, std::vector<std::string>& out,
          int depth = 0) {
    if (depth > 64) return;
    for (auto& e : entries(abs)) {
        std::string r = rel.empty() ? e.name : rel + "/" + e.name;
        if (e.is_dir) {
            if (skip_dir(e.name)) continue;
            walk(join_path(abs, e.name), r, keep, skip_dir, out, depth + 1);
        } else if (keep(e.name)) {
            out.push_back(r);
        }
    }
}

long long us_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t).count();
}

std::string strip_ext(const std::string& rel, const std::string& ext) {
    return ends_with(rel, ext) ? rel.substr(0, rel.size() - ext.size()) : rel;
}

std::string dotted(std::string s) {
    for (auto& c : s) if (c == '/' || c == '\\') c = '.';
    return s;
}

void write_file(JsonWriter& w, const FileRec& f) {
    w.begin_obj();
    w.kv("path", f.rel_path);
    w.kv("identifier", f.identifier);
    w.kv("classType", f.class_type);
    w.kv("entryPoint", f.entry_point);
    w.kv("package", f.package_name);
    w.kv("parsed", f.parsed);
    w.str_array("deps", f.deps);
    w.key("params");
    w.begin_obj();
    for (auto& kv : f.params) w.str_array(kv.first, kv.second);
    w.end_obj();
    w.key("methods");
    w.begin_arr();
    for (auto& m : f.methods) {
        w.begin_obj();
        w.kv("name", m.name);
        w.kv_int("line", m.line);
        w.kv_opt("httpMethod", m.has_http_method ? &m.http_method : nullptr);
        w.kv_opt("httpPath", m.has_http_path ? &m.http_path : nullptr);
        w.str_array("exceptions", m.exceptions);
        w.end_obj();
    }
    w.end_arr();
    w.end_obj();
}

// ------------------------------------------------------------------- Java
void scan_java(const std::string& root, const ScanOptions& opt, ScanResult& res) {
    std::vector<FileRec>& files = res.files;
    const std::string src_root = "src/main/java";
    std::string abs_src = join_path(root, src_root);
    if (!dir_exists(abs_src)) return;
    std::vector<std::string> rels;
    auto t = std::chrono::steady_clock::now();
    walk(abs_src, "", [](const std::string& n) { return ends_with(n, ".java"); },
         [](const std::string&) { return false; }, rels);
    res.walk_us = us_since(t);
    t = std::chrono::steady_clock::now();
    files.resize(rels.size());
    std::vector<std::string> sources(rels.size());
    parallel_for(rels.size(), opt.threads, [&](size_t k) {
        FileRec& f = files[k];
        f.rel_path = src_root + "/" + rels[k];
        f.abs_path = join_path(root, f.rel_path);
        f.identifier = dotted(strip_ext(rels[k], ".java"));
        std::string src;
        if (!read_file(f.abs_path, src)) return;
        analyze_java(src, f);
    });
    for (auto& f : files) if (!f.parsed) ++res.skipped;
    res.analyze_us = us_since(t);
    t = std::chrono::steady_clock::now();
    // resolution pass
    std::unordered_set<std::string> known;
    known.reserve(files.size() * 2);
    for (auto& f : files) known.insert(f.identifier);
    parallel_for(files.size(), opt.threads, [&](size_t k) {
        FileRec& f = files[k];
        std::unordered_set<std::string> seen;
        std::unordered_map<std::string, std::string> import_map;
        for (auto& imp : f.imports) {
            if (imp.is_asterisk) continue;
            std::string fq = imp.imported;
            if (imp.is_static) {
                size_t d = fq.rfind('.');
                fq = (d != std::string::npos && d > 0) ? fq.substr(0, d) : std::string();
            }
            if (fq.empty()) continue;
            size_t d = fq.rfind('.');
            if (d != std::string::npos && d > 0) import_map[fq.substr(d + 1)] = fq;
            if (known.count(fq) && seen.insert(fq).second) f.deps.push_back(fq);
        }
        // extractMethodParameters: constructors then methods; last overload wins
        for (auto& m : f.methods) {
            if (!m.params_eligible || m.param_types.empty()) continue;
            std::vector<std::string> matched;
            for (auto& ty : m.param_types) {
                if (ty.empty()) continue;
                if (known.count(ty)) { matched.push_back(ty); continue; }
                auto it = import_map.find(ty);
                if (it != import_map.end() && known.count(it->second)) { matched.push_back(it->second); continue; }
                if (!f.package_name.empty()) {
                    std::string same = f.package_name + "." + ty;
                    if (known.count(same)) matched.push_back(same);
                }
            }
            if (matched.empty()) continue;
            bool replaced = false;
            for (auto& kv : f.params)
                if (kv.first == m.name) { kv.second = matched; replaced = true; break; }
            if (!replaced) f.params.emplace_back(m.name, matched);
        }
    });
    res.resolve_us = us_since(t);
}

// ------------------------------------------------------------- TypeScript
const std::unordered_set<std::string> kTsExcludedDirs = {"node_modules", "dist", ".next", "build",
                                                         "coverage", "__tests__", "__mocks__"};

bool ts_source_file(const std::string& name) {
    if (!(ends_with(name, ".ts") || ends_with(name, ".tsx") || ends_with(name, ".js") || ends_with(name, ".jsx")))
        return false;
    if (contains(name, ".spec.") || contains(name, ".test.")) return false;
    if (ends_with(name, ".d.ts")) return false;
    return true;
}

void scan_ts(const std::string& root, const ScanOptions& opt, std::vector<FileRec>& files, int& skipped,
             FrameworkInfo& fw, std::string& source_root) {
    std::string pkg;
    if (!read_file(join_path(root, "package.json"), pkg)) pkg = "{}";
    fw = detect_framework(pkg);
    if (!opt.framework.empty()) fw.name = opt.framework;
    source_root = dir_exists(join_path(root, fw.source_root)) ? fw.source_root : "src";
    std::string abs_src = join_path(root, source_root);
    std::vector<std::string> rels;
    if (dir_exists(abs_src))
        walk(abs_src, "", ts_source_file, [](const std::string& n) { return kTsExcludedDirs.count(n) > 0; }, rels);
    files.resize(rels.size());
    std::string fw_name = fw.name;
    parallel_for(rels.size(), opt.threads, [&](size_t k) {
        FileRec& f = files[k];
        f.rel_path = source_root + "/" + rels[k];
        f.abs_path = join_path(root, f.rel_path);
        // identifier: strip the last extension, '/' -> '.' (NodeJsGraalParser.java:193-203)
        std::string r = rels[k];
        size_t dot = r.rfind('.');
        size_t slash = r.rfind('/');
        if (dot != std::string::npos && dot > 0 && (slash == std::string::npos || dot > slash + 1 || dot > slash))
            r = r.substr(0, dot);
        f.identifier = dotted(r);
        std::string src;
        if (!read_file(f.abs_path, src, opt.max_file_bytes)) return;  // > 5 MB or unreadable: skipped
        bool jsx = !ends_with(f.rel_path, ".ts");
        analyze_ts(src, f.rel_path, fw_name, jsx, f);
    });
    // drop skipped files entirely (they never become graph nodes)
    std::vector<FileRec> kept;
    kept.reserve(files.size());
    for (auto& f : files) {
        if (f.parsed) kept.push_back(std::move(f));
        else ++skipped;
    }
    files.swap(kept);
    std::unordered_set<std::string> known;
    for (auto& f : files) known.insert(f.identifier);
    const std::string abs_root_norm = normalize_path(abs_src);
    auto resolve = [&](const std::string& import_path, const std::string& file_rel) -> std::string {
        // resolve against the importing file's directory (NodeJsGraalParser.java:371-401),
        // anchored at the detected source root of *this* project.
        std::string dir = file_rel;
        size_t s = dir.rfind('/');
        dir = s == std::string::npos ? std::string() : dir.substr(0, s);
        std::string full = normalize_path(join_path(join_path(root, dir), import_path));
        std::string prefix = abs_root_norm + "/";
        if (!starts_with(full, prefix)) return std::string();
        std::string cand = dotted(full.substr(prefix.size()));
        if (known.count(cand)) return cand;
        std::string idx = cand + ".index";
        if (known.count(idx)) return idx;
        return std::string();
    };
    parallel_for(files.size(), opt.threads, [&](size_t k) {
        FileRec& f = files[k];
        std::unordered_set<std::string> seen;
        std::unordered_map<std::string, std::string> type_map;
        for (auto& imp : f.imports) {
            if (!starts_with(imp.source, ".")) continue;
            std::string r = resolve(imp.source, f.rel_path);
            if (r.empty()) continue;
            if (seen.insert(r).second) f.deps.push_back(r);
            type_map[imp.local] = r;
        }
        for (auto& m : f.methods) {
            std::vector<std::string> matched;
            for (auto& ty : m.param_types) {
                auto it = type_map.find(ty);
                if (it != type_map.end() && known.count(it->second)) matched.push_back(it->second);
            }
            if (matched.empty()) continue;
            bool replaced = false;
            for (auto& kv : f.params)
                if (kv.first == m.name) { kv.second = matched; replaced = true; break; }
            if (!replaced) f.params.emplace_back(m.name, matched);
        }
    });
}

}  // namespace

std::string detect_language(const std::string& root) {
    // CodeContextService.detectParser (:1628-1642)
    if (file_exists(join_path(root, "go.mod"))) return "go";
    if (file_exists(join_path(root, "package.json")) && !file_exists(join_path(root, "pom.xml")) &&
        !file_exists(join_path(root, "build.gradle")) && !file_exists(join_path(root, "build.gradle.kts")))
        return "typescript";
    return "java";
}

ScanResult scan_project(const std::string& root, const ScanOptions& opt) {
    ScanResult r;
    scan_project_into(root, opt, r);
    return r;
}

void scan_project_into(const std::string& root, const ScanOptions& opt, ScanResult& r) {
    auto t0 = std::chrono::steady_clock::now();
    std::string lang = opt.language;
    if (lang == "auto" || lang.empty()) lang = detect_language(root);
    if (lang == "ts" || lang == "js" || lang == "javascript" || lang == "node") lang = "typescript";
    if (lang == "typescript") {
        scan_ts(root, opt, r.files, r.skipped, r.framework, r.source_root);
        r.has_framework = true;
    } else if (lang == "go") {
        go_project_files(root, opt.threads, r.module, r.files, opt.go_doc ? &r.go_json : nullptr);
    } else {
        lang = "java";
        r.source_root = "src/main/java";
        scan_java(root, opt, r);
    }
    r.language = lang;
    r.elapsed_us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
}

std::string scan_result_json(const ScanResult& r) {
    JsonWriter w;
    w.begin_obj();
    w.kv("language", r.language);
    w.kv("sourceRoot", r.source_root);
    w.key("framework");
    if (r.has_framework) {
        w.begin_obj();
        w.kv("name", r.framework.name);
        w.kv("sourceRoot", r.framework.source_root);
        w.key("features");
        w.begin_obj();
        for (auto& kv : r.framework.features) w.kv(kv.first, kv.second);
        w.end_obj();
        w.end_obj();
    } else {
        w.value_null();
    }
    if (r.language == "go") w.kv("module", r.module);
    w.key("stats");
    w.begin_obj();
    w.kv_int("discovered", (long long)r.files.size() + r.skipped);
    w.kv_int("analyzed", (long long)r.files.size());
    w.kv_int("skipped", r.skipped);
    w.kv_int("elapsedUs", r.elapsed_us);
    w.key("phaseUs");
    w.begin_obj();
    w.kv_int("mount", r.mount_us);
    w.kv_int("walk", r.walk_us);
    w.kv_int("analyze", r.analyze_us);
    w.kv_int("resolve", r.resolve_us);
    w.end_obj();
    w.end_obj();
    w.key("files");
    w.begin_arr();
    for (auto& f : r.files) write_file(w, f);
    w.end_arr();
    if (!r.go_json.empty()) {
        w.key("go");
        w.raw(r.go_json);
    }
    w.end_obj();
    return w.out;
}

std::string scan_project_json(const std::string& root, const ScanOptions& opt) {
    return scan_result_json(scan_project(root, opt));
}

namespace {
std::string analyze_one_json(const std::string& path, const std::string* content, const std::string& language,
                             const std::string& rel_path, const std::string& framework) {
    FileRec f;
    f.abs_path = path;
    f.rel_path = rel_path.empty() ? path : rel_path;
    // ``rel_path`` is relative to the source root: it names the unit
    if (!rel_path.empty()) {
        std::string r = rel_path;
        size_t dot = r.rfind('.'), slash = r.rfind('/');
        if (dot != std::string::npos && dot > 0 && (slash == std::string::npos || dot > slash + 1)) r = r.substr(0, dot);
        f.identifier = dotted(r);
    }
    std::string src;
    const bool have = content != nullptr || read_file(path, src);
    if (have) {
        const std::string& text = content != nullptr ? *content : src;
        if (language == "java") analyze_java(text, f);
        else analyze_ts(text, f.rel_path, framework.empty() ? "unknown" : framework, !ends_with(path, ".ts"), f);
    }
    JsonWriter w;
    write_file(w, f);
    // raw imports / param types are useful for tests of the per-file hooks
    std::string out = w.out;
    out.pop_back();  // remove '}'
    JsonWriter x;
    x.key("imports");
    x.begin_arr();
    for (auto& imp : f.imports) {
        x.begin_obj();
        x.kv("importedName", imp.imported);
        x.kv("localName", imp.local);
        x.kv("source", imp.source);
        x.kv("isStatic", imp.is_static);
        x.kv("isAsterisk", imp.is_asterisk);
        x.end_obj();
    }
    x.end_arr();
    x.key("rawParams");
    x.begin_arr();
    for (auto& m : f.methods) {
        x.begin_obj();
        x.kv("name", m.name);
        x.str_array("types", m.param_types);
        x.kv("eligible", m.params_eligible);
        x.end_obj();
    }
    x.end_arr();
    out += ",";
    out += x.out;
    out += "}";
    return out;
}
}  // namespace

std::string scan_file_json(const std::string& path, const std::string& language, const std::string& rel_path,
                           const std::string& framework) {
    return analyze_one_json(path, nullptr, language, rel_path, framework);
}

std::string analyze_source_json(const std::string& content, const std::string& language, const std::string& file_path,
                                const std::string& framework) {
    // GraalJsAnalyzerEngine.analyzeFile(content, filePath, framework) parity:
    // the path only names the unit (class-type filename table, Next.js routes)
    return analyze_one_json(file_path, &content, language, file_path, framework);
}

}  // namespace srcscan
