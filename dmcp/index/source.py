"""Source trees: the files of one commit, either checked out on disk or held
in memory straight from git objects.

The reference clones every repository to a temp directory with JGit, walks
the checkout, and deletes it afterwards (``CodeContextService.java:1653-1683``,
``:465``).  Writing thousands of files only to read them once and unlink them
was the largest single cost of an analysis here (≈ 35 % of a 2,000-class
index on MI355X hosts).  :class:`MemoryTree` instead reads git objects: a
remote repository is cloned **bare** (``--depth 1``), a local one is read in
place (its objects are content-addressed and immutable).  The commit is listed
with ``git ls-tree``; loose blobs are inflated natively on a thread pool
(``native/srcscan/gitobj.cpp``) and packed ones streamed through ``git
cat-file --batch``.  The native scanner then parses a mounted in-memory tree
(``srcscan.scan_sources``) and enrichment reads source text from the same map.  Every byte of every source file at HEAD is still
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

    def scan_objects(self, language: str, threads: int, framework: str = "", rows=None) -> Optional[dict]:
        """The scan document as Python objects built natively (no JSON round
        trip), or None when this tree only offers :meth:`scan`.  ``rows``: see
        ``SourceParser.scan_tree`` (trees that cannot write rows ignore it)."""
        return None

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
    """``owned``: ``git_dir`` is a private bare clone removed by :meth:`cleanup`
    (False when a local repository's object store is read in place)."""

    def __init__(self, git_dir: str, commit_hash: str, files: Dict[str, bytes], owned: bool = True) -> None:
        self.directory = git_dir if owned else None
        self.git_dir = git_dir
        self.commit_hash = commit_hash
        self._files = files

    @property
    def files(self) -> Dict[str, bytes]:
        return self._files

    @files.setter
    def files(self, value: Dict[str, bytes]) -> None:
        self._files = value

    def read_bytes(self, rel: str) -> Optional[bytes]:
        return self.files.get(rel.replace(os.sep, "/"))

    def detect_language(self) -> str:
        return detect_language_from(self.files)

    def scan(self, language: str, threads: int, framework: str = "") -> bytes:
        from ..parsers.base import native
        return native().scan_sources(list(self.files.items()), language, threads, framework)

    def scan_objects(self, language: str, threads: int, framework: str = "", rows=None) -> Optional[dict]:
        from ..models.domain import StaticMethodInfo
        from ..parsers.base import native
        fn = getattr(native(), "scan_sources_objects", None)
        if fn is None:
            return None
        if rows is not None:
            # the indexing pipeline (rows given) never reads the Go analyzer's
            # package document (3.6 MB of JSON for a 1,000-file repository,
            # rendered on one thread): not built on that path
            # the call form from the module's ABI, never by retrying a call
            # that may already have streamed rows to the writer
            if getattr(native(), "ABI_VERSION", 0) >= 6:
                return fn(list(self.files.items()), language, threads, framework, StaticMethodInfo, rows,
                          go_doc=False)
            return fn(list(self.files.items()), language, threads, framework, StaticMethodInfo, rows)
        return fn(list(self.files.items()), language, threads, framework, StaticMethodInfo)


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


class _Budget:
    """Byte budget shared by concurrent readers."""

    def __init__(self, limit: int) -> None:
        import threading
        self.limit = limit
        self.used = 0
        self.exceeded = False
        self._lock = threading.Lock()

    def take(self, n: int) -> bool:
        with self._lock:
            self.used += n
            if self.limit and self.used > self.limit:
                self.exceeded = True
            return not self.exceeded


def _object_dirs(git_dir: str) -> List[str]:
    own = os.path.join(git_dir, "objects")
    if not os.path.isdir(own):
        own = os.path.join(git_dir, ".git", "objects")
    dirs = [own]
    try:
        with open(os.path.join(own, "info", "alternates")) as f:
            dirs += [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]
    except OSError:
        pass
    return dirs


def git_dir_of(path: str) -> Optional[str]:
    """The git directory of a work tree (``<path>/.git``) or bare repository
    (``path`` itself); None for anything else (e.g. a ``.git`` file of a linked
    work tree), which is left to git."""
    dot = os.path.join(path, ".git")
    if os.path.isdir(dot):
        return dot
    if os.path.isfile(os.path.join(path, "HEAD")) and os.path.isdir(os.path.join(path, "objects")):
        return path
    return None


def native_commit_tree(repo: str, refs: List[str]) -> Optional[Tuple[str, List[Tuple[str, str]]]]:
    """(commit, ls-tree entries) read straight from a loose object store
    (``native/srcscan/gitobj.cpp``): what ``git rev-parse --verify
    <ref>^{commit}`` over ``refs`` and ``git ls-tree -r`` report, without the
    two processes.  None whenever git has to answer (packed objects or refs the
    reader does not handle, no native extension)."""
    try:
        from .. import _srcscan  # type: ignore
    except ImportError:
        return None
    resolve = getattr(_srcscan, "resolve_ref", None)
    gd = git_dir_of(repo)
    if resolve is None or gd is None or not mostly_loose(repo):
        return None
    commit = resolve(gd, refs)
    if commit is None:
        return None
    entries = _srcscan.list_tree_loose(_object_dirs(repo), commit)
    if entries is None:
        return None
    return commit, entries


def mostly_loose(git_dir: str) -> bool:
    """True when the repository's objects (alternates included) are mostly
    loose: git creates a fan-out directory per object-id prefix on demand and
    ``gc`` prunes the emptied ones, so ≥ 16 of them means a loose store."""
    n = 0
    for d in _object_dirs(git_dir):
        try:
            with os.scandir(d) as it:
                n += sum(1 for e in it if len(e.name) == 2 and e.is_dir())
        except OSError:
            continue
    return n >= 16


def default_procs(git_dir: str, n_blobs: int) -> int:
    """Reader processes for ``n_blobs``.  Measured on an MI355X host
    (``scripts/catfile_sweep.py``, 2,003 blobs): zlib-inflating loose objects
    is CPU-bound and scales (1/2/4/8 processes: 39.7/27.5/18.0/14.6 ms), a
    packed store is bound by each process mapping the pack index (6.4/5.1/
    5.6/10.5 ms)."""
    cpus = os.cpu_count() or 1
    if mostly_loose(git_dir):
        return max(1, min(8, n_blobs // 256, cpus))
    return 2 if n_blobs >= 1024 and cpus > 1 else 1


def _native_loose_reader():
    try:
        from .. import _srcscan  # type: ignore
    except ImportError:
        return None
    return getattr(_srcscan, "read_loose_blobs", None)


def read_blobs(git, git_dir: str, shas: List[str], max_bytes: int = 0, procs: int = 0,
               threads: int = 0) -> Optional[List[bytes]]:
    """Contents of ``shas``; None as soon as more than ``max_bytes`` (if > 0)
    of blob data has arrived in total.

    A mostly-loose store is inflated natively on ``threads`` workers
    (``native/srcscan/gitobj.cpp``; 0 = up to 16), and only the objects that are
    not loose go through git; otherwise ``procs`` concurrent ``git cat-file
    --batch`` processes read everything (0 = :func:`default_procs`)."""
    if not shas:
        return []
    reader = _native_loose_reader()
    if reader is not None and mostly_loose(git_dir):
        nthreads = threads or max(1, min(16, os.cpu_count() or 1, len(shas) // 64 or 1))
        blobs, exceeded = reader(_object_dirs(git_dir), shas, nthreads, max_bytes)
        if exceeded:
            return None
        missing = [i for i, b in enumerate(blobs) if b is None]
        if missing:
            have = sum(len(b) for b in blobs if b is not None)
            if max_bytes and have > max_bytes:
                return None
            rest = _read_via_git(git, git_dir, [shas[i] for i in missing], max_bytes - have if max_bytes else 0,
                                 procs)
            if rest is None:
                return None
            for i, b in zip(missing, rest):
                blobs[i] = b
        return blobs
    return _read_via_git(git, git_dir, shas, max_bytes, procs)


def _read_via_git(git, git_dir: str, shas: List[str], max_bytes: int, procs: int) -> Optional[List[bytes]]:
    if not shas:
        return []
    if procs <= 0:
        procs = default_procs(git_dir, len(shas))
    budget = _Budget(max_bytes)
    if procs == 1:
        return _read_blobs_one(git, git_dir, shas, budget)
    from concurrent.futures import ThreadPoolExecutor
    step = -(-len(shas) // procs)
    parts = [shas[i:i + step] for i in range(0, len(shas), step)]
    with ThreadPoolExecutor(max_workers=len(parts)) as ex:
        results = list(ex.map(lambda part: _read_blobs_one(git, git_dir, part, budget), parts))
    if budget.exceeded or any(r is None for r in results):
        return None
    out: List[bytes] = []
    for r in results:
        out.extend(r)
    return out


def _read_blobs_one(git, git_dir: str, shas: List[str], budget: "_Budget") -> Optional[List[bytes]]:
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
    try:
        rd = p.stdout
        for sha in shas:
            header = rd.readline().split()
            if len(header) < 3 or header[1] == b"missing":
                raise RuntimeError(f"git cat-file: object {sha} missing")
            size = int(header[2])
            if not budget.take(size):
                return None
            blobs.append(rd.read(size))
            rd.read(1)  # trailing LF
        return blobs
    finally:
        if p.poll() is None:
            p.kill()
        p.wait()
        writer.join(timeout=5)
