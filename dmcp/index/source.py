"""Source trees: the files of one commit, either checked out on disk or held
in memory straight from git objects.

The reference clones every repository to a temp directory with JGit, walks
the checkout, and deletes it afterwards (``CodeContextService.java:1653-1683``,
``:465``).  Writing thousands of files only to read them once and unlink them
was the largest single cost of an analysis here (≈ 35 % of a 2,000-class
index on MI355X hosts).  :class:`MemoryTree` instead clones **bare**
(``--shared`` for local repositories, ``--depth 1`` for remote analyses), lists
the commit with ``git ls-tree`` and streams the blobs the front-ends need
through one ``git cat-file --batch`` process; the native scanner then parses a
mounted in-memory tree (``srcscan.scan_sources``) and enrichment reads source
text from the same map.  Every byte of every source file at HEAD is still
read and parsed; nothing is cached across analyses.  Repositories larger than
``max_bytes`` of candidate sources fall back to a regular checkout
(:class:`CheckoutTree`).
"""
from __future__ import annotations

import logging
import os
import shutil
import subprocess
from typing import Dict, Iterable, List, Optional, Tuple

LOG = logging.getLogger(__name__)

# files the front-ends read (sources + the manifests language/framework
# detection looks at + README.md for the project description)
SOURCE_EXTENSIONS = (".java", ".ts", ".tsx", ".js", ".jsx", ".go")
MANIFESTS = {"README.md", "package.json", "go.mod", "pom.xml", "build.gradle", "build.gradle.kts"}


def wanted(path: str) -> bool:
    if path.endswith(SOURCE_EXTENSIONS):
        # vendored npm trees are excluded by every front-end (TS and Go walks)
        return not (path.startswith("node_modules/") or "/node_modules/" in path)
    return path in MANIFESTS  # repository root only


def detect_language_from(paths: Iterable[str]) -> str:
    """CodeContextService.detectParser (:1628-1642) over a path set."""
    s = set(paths)
    if "go.mod" in s:
        return "go"
    if "package.json" in s and not ({"pom.xml", "build.gradle", "build.gradle.kts"} & s):
        return "typescript"
    return "java"


class SourceTree:
    """One commit's files.  ``directory`` is the checkout (or bare repository)
    on disk that must be removed by :meth:`cleanup`."""

    commit_hash: str
    directory: Optional[str]
    git_dir: Optional[str]

    def read_bytes(self, rel: str) -> Optional[bytes]:
        raise NotImplementedError

    def read_text(self, rel: str) -> Optional[str]:
        b = self.read_bytes(rel)
        return None if b is None else b.decode("utf-8", "replace")

    def detect_language(self) -> str:
        raise NotImplementedError

    def scan(self, language: str, threads: int, framework: str = "") -> bytes:
        """Raw native scan document (JSON bytes)."""
        raise NotImplementedError

    def readme(self, max_length: int = 10_000) -> Optional[str]:
        """README.md truncated to ``max_length`` + marker (CodeContextService.java:1688-1712)."""
        content = self.read_text("README.md")
        if content is None or not content.strip():
            return None
        if len(content) > max_length:
            return content[:max_length] + "\n...(truncated)"
        return content

    def cleanup(self) -> None:
        if self.directory and os.path.isdir(self.directory):
            shutil.rmtree(self.directory, ignore_errors=True)


class CheckoutTree(SourceTree):
    def __init__(self, directory: str, commit_hash: str) -> None:
        self.directory = directory
        self.git_dir = directory
        self.commit_hash = commit_hash

    def read_bytes(self, rel: str) -> Optional[bytes]:
        try:
            with open(os.path.join(self.directory, rel), "rb") as f:
                return f.read()
        except OSError:
            return None

    def detect_language(self) -> str:
        from ..parsers.base import detect_language
        return detect_language(self.directory)

    def scan(self, language: str, threads: int, framework: str = "") -> bytes:
        from ..parsers.base import native
        return native().scan_project(self.directory, language, threads, framework)


class MemoryTree(SourceTree):
    def __init__(self, git_dir: str, commit_hash: str, files: Dict[str, bytes]) -> None:
        self.directory = git_dir
        self.git_dir = git_dir
        self.commit_hash = commit_hash
        self.files = files

    def read_bytes(self, rel: str) -> Optional[bytes]:
        return self.files.get(rel.replace(os.sep, "/"))

    def detect_language(self) -> str:
        return detect_language_from(self.files)

    def scan(self, language: str, threads: int, framework: str = "") -> bytes:
        from ..parsers.base import native
        return native().scan_sources(list(self.files.items()), language, threads, framework)


def list_tree(git, git_dir: str, rev: str = "HEAD") -> List[Tuple[str, str]]:
    """(path, blob sha) of every regular file blob at ``rev`` (no sizes: ``-l``
    would inflate every loose object just to report its length)."""
    out = git._git(["ls-tree", "-r", "-z", "--full-tree", rev], cwd=git_dir)[1]
    entries = []
    for rec in out.split("\0"):
        if not rec:
            continue
        meta, path = rec.split("\t", 1)
        mode, typ, sha = meta.split()
        if typ != "blob" or mode == "120000":  # submodules (commit) and symlinks skipped
            continue
        entries.append((path, sha))
    return entries


def read_blobs(git, git_dir: str, shas: List[str], max_bytes: int = 0) -> Optional[List[bytes]]:
    """Contents of ``shas`` streamed through one ``git cat-file --batch``
    process; None as soon as more than ``max_bytes`` (if > 0) have arrived."""
    if not shas:
        return []
    import threading
    p = subprocess.Popen(["git", "cat-file", "--batch"], cwd=git_dir, env=git._env(), stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.DEVNULL)

    def feed():
        try:
            p.stdin.write(("\n".join(shas) + "\n").encode())
            p.stdin.close()
        except (BrokenPipeError, OSError):
            pass

    writer = threading.Thread(target=feed, daemon=True)
    writer.start()
    blobs: List[bytes] = []
    total = 0
    try:
        rd = p.stdout
        for sha in shas:
            header = rd.readline().split()
            if len(header) < 3 or header[1] == b"missing":
                raise RuntimeError(f"git cat-file: object {sha} missing")
            size = int(header[2])
            total += size
            if max_bytes and total > max_bytes:
                return None
            blobs.append(rd.read(size))
            rd.read(1)  # trailing LF
        return blobs
    finally:
        if p.poll() is None:
            p.kill()
        p.wait()
        writer.join(timeout=5)
