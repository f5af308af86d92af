// Loose git object reader (see gitobj.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace gitobj {

struct LooseResult {
    std::vector<std::string> data;  // blob contents (valid where found[i])
    std::vector<uint8_t> found;     // 0: not a loose blob in any object dir
    uint64_t total_bytes = 0;
    bool exceeded = false;          // more than max_bytes of content read
};

// Reads `shas` (40-hex object ids) from the first of `object_dirs` holding
// each as a loose object, on `threads` workers (0 = hardware concurrency).
LooseResult read_loose_blobs(const std::vector<std::string>& object_dirs, const std::vector<std::string>& shas,
                             int threads, uint64_t max_bytes);

// One loose blob's content; false when it is not a loose blob in any dir.
bool read_loose_blob(const std::vector<std::string>& object_dirs, const std::string& sha, std::string& out);

// The commit the first resolvable ref of `refs` ("HEAD", "refs/heads/x",
// "refs/tags/x") names, annotated tags peeled.  false when git must answer
// (ref storage or objects not readable here, or the ref is not a commit).
bool resolve_commit(const std::string& git_dir, const std::vector<std::string>& refs, std::string& commit);

// (path, blob id) of every regular file at `commit`, in `git ls-tree -r`
// order (symlinks and submodules skipped); false unless every tree is loose.
bool list_tree(const std::vector<std::string>& object_dirs, const std::string& commit,
               std::vector<std::pair<std::string, std::string>>& out);

}  // namespace gitobj
