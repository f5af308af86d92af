"""Git access through the ``git`` CLI (the reference uses JGit).

Parity: clone (``CodeContextService.java:1653-1683`` shallow ``depth=1`` of the
branch; ``ProjectSyncService.java:754-777`` full clone for diffing), HEAD hash,
and diff classification (``ProjectSyncService.java:497-542``: ADD/MODIFY/COPY
-> changed, DELETE -> deleted, RENAME -> both; missing old commit or no
previous hash -> full resync).  ``git.ssh-key-path`` and
``git.timeout-seconds`` -- declared but unused in the reference -- are honoured
here (``GIT_SSH_COMMAND`` and a per-command timeout).
"""
from __future__ import annotations

import logging
import os
import shlex
import shutil
import subprocess
import time
from dataclasses import dataclass
from typing import List, Optional, Tuple

from ..models.domain import GitDiffResult, RepositoryUrl

LOG = logging.getLogger(__name__)


class GitError(RuntimeError):
    pass


@dataclass
class CloneResult:
    directory: str
    commit_hash: str


class GitClient:
    def __init__(self, clone_base_path: str = "/tmp/domain-mcp-repos",
                 ssh_key_path: Optional[str] = None, timeout_seconds: int = 300) -> None:
        self.clone_base_path = clone_base_path
        self.ssh_key_path = ssh_key_path
        self.timeout = timeout_seconds
        self.read_local_in_place = True  # snapshot(): local repositories without a private clone
        self.native_objects = True  # snapshot(): ref + tree read from loose objects natively when possible

    def _env(self) -> dict:
        env = dict(os.environ)
        env["GIT_TERMINAL_PROMPT"] = "0"
        if self.ssh_key_path:
            # git runs GIT_SSH_COMMAND through a shell: the key path is quoted
            env["GIT_SSH_COMMAND"] = (f"ssh -i {shlex.quote(self.ssh_key_path)} -o IdentitiesOnly=yes "
                                      "-o StrictHostKeyChecking=accept-new")
        return env

    def _git(self, args: List[str], cwd: Optional[str] = None, check: bool = True) -> Tuple[int, str, str]:
        try:
            r = subprocess.run(["git", *args], cwd=cwd, env=self._env(), stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, text=True, timeout=self.timeout)
        except subprocess.TimeoutExpired as e:
            raise GitError(f"git {' '.join(args[:2])} timed out after {self.timeout}s") from e
        if check and r.returncode != 0:
            raise GitError(f"git {' '.join(args[:2])} failed: {r.stderr.strip() or r.stdout.strip()}")
        return r.returncode, r.stdout, r.stderr

    @staticmethod
    def _source(url: RepositoryUrl) -> str:
        local = url.local_path()
        if local is not None:
            return "file://" + os.path.abspath(local)  # file:// so --depth is honoured
        return url.value

    def new_clone_dir(self, name: str, suffix: str = "") -> str:
        os.makedirs(self.clone_base_path, exist_ok=True)
        return os.path.join(self.clone_base_path, f"{name}{suffix}-{int(time.time() * 1000)}")

    def clone(self, url: RepositoryUrl, branch: Optional[str], shallow: bool = True,
              directory: Optional[str] = None) -> CloneResult:
        dest = directory or self.new_clone_dir(url.repository_name())
        os.makedirs(os.path.dirname(dest) or ".", exist_ok=True)
        args = ["clone", "--quiet", "--no-tags"]
        local = url.local_path()
        if local is not None:
            # Local repository: share its object store (alternates) instead of
            # re-packing through upload-pack -- 5-10x faster than a file://
            # shallow clone, full history available for diffing.
            args += ["--shared", "--single-branch"]
            source = os.path.abspath(local)
        else:
            if shallow:
                args += ["--depth", "1", "--single-branch"]
            source = url.value
        if branch:
            args += ["--branch", branch]
        args += [source, dest]
        LOG.info("Cloning %s (branch: %s) to %s", url, branch, dest)
        try:
            self._git(args)
        except GitError as e:
            shutil.rmtree(dest, ignore_errors=True)
            raise GitError(f"Failed to clone repository: {e}") from e
        return CloneResult(dest, self.head(dest))

    def snapshot(self, url: RepositoryUrl, branch: Optional[str], shallow: bool = True,
                 max_bytes: int = 1 << 30):
        """The branch head as a :class:`~dmcp.index.source.SourceTree` without a
        working-tree checkout (bare clone + ``cat-file --batch``); falls back to
        a checkout when the candidate sources exceed ``max_bytes``."""
        from .source import CheckoutTree, MemoryTree, list_tree, native_commit_tree, read_blobs, wanted
        local = url.local_path()
        if local is not None and self.read_local_in_place:
            return self._local_snapshot(url, os.path.abspath(local), branch, shallow, max_bytes)
        dest = self.new_clone_dir(url.repository_name(), "-bare")
        args = ["clone", "--quiet", "--no-tags", "--bare"]
        if local is not None:
            args += ["--shared", "--single-branch"]
            source = os.path.abspath(local)
        else:
            if shallow:
                args += ["--depth", "1"]
            args += ["--single-branch"]
            source = url.value
        if branch:
            args += ["--branch", branch]
        args += [source, dest]
        LOG.info("Fetching %s (branch: %s) into %s", url, branch, dest)
        try:
            self._git(args)
            # the clone's refs + tree read natively when its objects are loose
            # (a --shared local clone: alternates into a loose store) -- two
            # git processes fewer; a packed clone falls back to git
            fast = native_commit_tree(dest, self.branch_refs(branch)) if self.native_objects else None
            if fast is not None:
                commit, listing = fast
            else:
                commit = self.head(dest)
                listing = list_tree(self, dest, commit)
            entries = [e for e in listing if wanted(e[0])]
            blobs = read_blobs(self, dest, [e[1] for e in entries], max_bytes)
            if blobs is None:
                LOG.info("%s: sources exceed the %d MiB in-memory limit, using a checkout", url, max_bytes >> 20)
                shutil.rmtree(dest, ignore_errors=True)
                c = self.clone(url, branch, shallow=shallow)
                return CheckoutTree(c.directory, c.commit_hash)
        except GitError as e:
            shutil.rmtree(dest, ignore_errors=True)
            raise GitError(f"Failed to clone repository: {e}") from e
        except Exception:
            shutil.rmtree(dest, ignore_errors=True)
            raise
        return MemoryTree(dest, commit, {e[0]: b for e, b in zip(entries, blobs)})

    def resolve_commit(self, repo_dir: str, branch: Optional[str]) -> str:
        """The commit ``git clone --branch <branch>`` would check out: the
        branch head, else the tag of that name; HEAD when no branch is given."""
        for ref in self.branch_refs(branch):
            rc, out, _ = self._git(["rev-parse", "--verify", "--quiet", f"{ref}^{{commit}}"], cwd=repo_dir,
                                   check=False)
            if rc == 0 and out.strip():
                return out.strip()
        raise GitError(f"Remote branch {branch} not found in upstream origin" if branch
                       else "repository has no HEAD commit")

    @staticmethod
    def branch_refs(branch: Optional[str]) -> List[str]:
        return [f"refs/heads/{branch}", f"refs/tags/{branch}"] if branch else ["HEAD"]

    def _local_snapshot(self, url: RepositoryUrl, source: str, branch: Optional[str], shallow: bool,
                        max_bytes: int):
        """A local repository's objects are read in place: content-addressed
        objects never change, so a private clone adds nothing but a process
        and a ref copy.  The tree does not own (and never deletes) ``source``."""
        from .source import CheckoutTree, MemoryTree, list_tree, native_commit_tree, read_blobs, wanted
        LOG.info("Reading %s (branch: %s) in place", url, branch)
        try:
            fast = native_commit_tree(source, self.branch_refs(branch)) if self.native_objects else None
            if fast is not None:
                commit, listing = fast
            else:
                commit = self.resolve_commit(source, branch)
                listing = list_tree(self, source, commit)
            entries = [e for e in listing if wanted(e[0])]
            blobs = read_blobs(self, source, [e[1] for e in entries], max_bytes)
        except GitError as e:
            raise GitError(f"Failed to clone repository: {e}") from e
        if blobs is None:
            LOG.info("%s: sources exceed the %d MiB in-memory limit, using a checkout", url, max_bytes >> 20)
            c = self.clone(url, branch, shallow=shallow)
            return CheckoutTree(c.directory, c.commit_hash)
        return MemoryTree(source, commit, {e[0]: b for e, b in zip(entries, blobs)}, owned=False)

    def head(self, repo_dir: str) -> str:
        return self._git(["rev-parse", "HEAD"], cwd=repo_dir)[1].strip()

    def commit_exists(self, repo_dir: str, commit: str) -> bool:
        rc, _, _ = self._git(["cat-file", "-e", f"{commit}^{{commit}}"], cwd=repo_dir, check=False)
        return rc == 0

    def diff(self, repo_dir: str, old_commit: Optional[str], new_commit: str) -> GitDiffResult:
        if not old_commit or not old_commit.strip():
            LOG.info("No previous commit hash, treating as full resync")
            return GitDiffResult.full_resync(new_commit)
        if not self.commit_exists(repo_dir, old_commit):
            LOG.warning("Old commit %s not found (force push?), treating as full resync", old_commit)
            return GitDiffResult.full_resync(new_commit)
        # -z: NUL-separated records with raw paths.  Without it git quotes
        # any path with a non-ASCII byte ("src/acm\303\251/A.java"), which
        # then matches no parsed file and the class is wrongly "unchanged"
        out = self._git(["diff", "-z", "--name-status", "-M", "-C", "--no-color", old_commit, new_commit],
                        cwd=repo_dir)[1]
        return parse_name_status_z(out, new_commit)

    @staticmethod
    def cleanup(directory: Optional[str]) -> None:
        if directory and os.path.isdir(directory):
            shutil.rmtree(directory, ignore_errors=True)


def parse_name_status_z(text: str, new_commit: str) -> GitDiffResult:
    """``git diff -z --name-status -M -C`` output: a status token, then one
    path (A/M/T/D/U) or two (R<score>/C<score>: source, destination), each
    NUL-terminated -- the JGit ``DiffEntry`` classification of
    ``ProjectSyncService.computeDiff`` (:497-542): ADD/MODIFY/COPY -> changed,
    DELETE -> deleted, RENAME -> both."""
    changed, deleted = set(), set()
    tok = text.split("\0")
    i, n = 0, len(tok)
    while i < n:
        status = tok[i].strip()
        if not status:
            i += 1
            continue
        kind = status[:1]
        if kind in ("R", "C"):
            if i + 2 >= n:
                break
            src, dst = tok[i + 1], tok[i + 2]
            if kind == "R":
                deleted.add(src)
            changed.add(dst)
            i += 3
            continue
        if i + 1 >= n:
            break
        path = tok[i + 1]
        if kind == "D":
            deleted.add(path)
        elif kind in ("A", "M", "T", "U"):
            changed.add(path)
        i += 2
    return GitDiffResult.of(new_commit, changed, deleted)


def parse_name_status(text: str, new_commit: str) -> GitDiffResult:
    """Line form (no ``-z``; ASCII paths only) -- kept for callers that
    already hold such output."""
    changed, deleted = set(), set()
    for line in text.splitlines():
        if not line.strip():
            continue
        parts = line.split("\t")
        status = parts[0][:1]
        if status in ("A", "M", "T") and len(parts) >= 2:
            changed.add(parts[1])
        elif status == "D" and len(parts) >= 2:
            deleted.add(parts[1])
        elif status == "R" and len(parts) >= 3:
            deleted.add(parts[1])
            changed.add(parts[2])
        elif status == "C" and len(parts) >= 3:
            changed.add(parts[2])
    return GitDiffResult.of(new_commit, changed, deleted)


def read_readme(repo_dir: str, max_length: int = 10_000) -> Optional[str]:
    """README.md, truncated to ``max_length`` + marker (CodeContextService.java:1688-1712)."""
    path = os.path.join(repo_dir, "README.md")
    if not os.path.isfile(path):
        return None
    try:
        with open(path, "r", encoding="utf-8", errors="replace") as f:
            content = f.read()
    except OSError as e:
        LOG.warning("Failed to read README.md: %s", e)
        return None
    if not content.strip():
        return None
    if len(content) > max_length:
        return content[:max_length] + "\n...(truncated)"
    return content
