"""Source scan in a fresh child process with a time limit.

The reference runs its one native analyzer (Go) as a subprocess: 120 s
timeout, ``destroyForcibly`` on expiry, and a non-zero exit logged and
treated as a failure (``GoSourceParser.java:62, 339-418``).  dmcp's
front-ends are in-process C++ for speed; for untrusted (remote) repositories
the indexer can run the same scan here instead: the child gets the tree (a
checkout directory, or the snapshot's files over its stdin), runs the native
scan and writes the JSON document to its stdout.  A crash (signal, abort) or
a hang past ``timeout_s`` kills the child only -- the server process never
executes the untrusted parse -- and surfaces as :class:`ScanFailed`, which
the pipeline turns into ``ANALYSIS_FAILED``.

The child is the native analyzer binary (``bin/srcscan stdin`` / ``srcscan
<root>``, built with the module) when it is present -- it starts in
milliseconds -- else a Python child running the same native scan.
"""
from __future__ import annotations

import json
import logging
import os
import struct
import subprocess
import time
import sys
from typing import Optional

LOG = logging.getLogger(__name__)
_HDR = struct.Struct("<Q")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class ScanFailed(RuntimeError):
    pass


def _write_blob(stream, data) -> None:
    """``data``: bytes or a byte memoryview (written without a copy)."""
    stream.write(_HDR.pack(data.nbytes if isinstance(data, memoryview) else len(data)))
    stream.write(data)


def _read_blob(stream) -> Optional[bytes]:
    hdr = stream.read(_HDR.size)
    if len(hdr) < _HDR.size:
        return None
    n = _HDR.unpack(hdr)[0]
    data = stream.read(n)
    return data if len(data) == n else None


def native_cli() -> Optional[str]:
    """The built ``bin/srcscan`` analyzer, or None."""
    path = os.path.join(ROOT, "bin", "srcscan")
    return path if os.access(path, os.X_OK) else None


def scan_in_child(tree, language: str, threads: int, framework: str = "", timeout_s: float = 120.0,
                  env_extra: Optional[dict] = None, native: Optional[bool] = None) -> dict:
    """The scan document of ``tree`` (a :class:`dmcp.index.source.SourceTree`),
    computed by a child process; raises :class:`ScanFailed` on a crash, a
    non-zero exit, unreadable output or a timeout."""
    from ..index.source import CheckoutTree
    files = None if isinstance(tree, CheckoutTree) else tree.files
    header = {"language": language, "threads": threads, "framework": framework}
    if files is None:
        header["root"] = tree.directory
    else:
        header["nfiles"] = len(files)
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.update(env_extra or {})
    cli = native_cli() if native is not False else None
    if cli is not None:
        argv = [cli] + (["stdin"] if files is not None else []) + ["--lang", language or "auto",
                                                                   "--threads", str(int(threads or 0))]
        if framework:
            argv += ["--framework", framework]
        if files is None:
            argv.append(tree.directory)
    else:
        argv = [sys.executable, "-m", "dmcp.parsers.isolated"]
    proc = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env,
                            cwd=ROOT)
    # the tree is STREAMED to the child from a writer thread (no serialised
    # copy of an up-to-1-GiB snapshot in this process) while two reader
    # threads drain its stdout / stderr (a full pipe would block either side)
    import threading

    def feed() -> None:
        try:
            if cli is not None:  # the binary: u64 file count, then (path, contents) blobs
                if files is not None:
                    proc.stdin.write(_HDR.pack(len(files)))
            else:
                _write_blob(proc.stdin, json.dumps(header).encode())
            if files is not None:
                for rel, data in files.items():
                    _write_blob(proc.stdin, rel.encode("utf-8", "surrogateescape"))
                    _write_blob(proc.stdin, memoryview(data).cast("B"))
        except (BrokenPipeError, OSError, ValueError):
            pass  # the child died (reported by its exit status) or was killed
        finally:
            try:
                proc.stdin.close()
            except OSError:
                pass
    got = {}

    def drain(name, stream) -> None:
        got[name] = stream.read()
    threads = [threading.Thread(target=feed, name="scan-feed", daemon=True),
               threading.Thread(target=drain, args=("out", proc.stdout), name="scan-out", daemon=True),
               threading.Thread(target=drain, args=("err", proc.stderr), name="scan-err", daemon=True)]
    for t in threads:
        t.start()
    try:
        proc.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        proc.kill()
        proc.wait()
        for t in threads:
            t.join(10)
        raise ScanFailed(f"source scan did not finish in {timeout_s:.0f} s (child killed)")
    for t in threads:
        t.join(30)
    out, err = got.get("out", b""), got.get("err", b"")
    if proc.returncode != 0:
        tail = (err or b"").decode("utf-8", "replace").strip().splitlines()[-3:]
        how = f"signal {-proc.returncode}" if proc.returncode < 0 else f"exit code {proc.returncode}"
        raise ScanFailed(f"source scan process failed ({how}): {' | '.join(tail)}")
    try:
        return json.loads(out)
    except ValueError as e:
        raise ScanFailed(f"source scan produced unreadable output: {e}") from e


# ---------------------------------------------------------------- persistent
class _ServeChild:
    """One ``srcscan serve`` process: requests in, binary ScanResults out
    (native/srcscan/wire.hpp); its stderr tail is kept for error messages."""

    def __init__(self, cli: str, env: dict) -> None:
        import threading
        self.proc = subprocess.Popen([cli, "serve"], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                     stderr=subprocess.PIPE, env=env, cwd=ROOT)
        self.err = bytearray()
        self.uses = 0

        def drain() -> None:
            for chunk in iter(lambda: self.proc.stderr.read1(4096), b""):
                self.err += chunk
                del self.err[:-4096]
        threading.Thread(target=drain, name="scan-child-err", daemon=True).start()

    def alive(self) -> bool:
        return self.proc.poll() is None

    def kill(self) -> None:
        try:
            self.proc.kill()
        except OSError:
            pass
        try:
            self.proc.wait(10)
        except subprocess.TimeoutExpired:
            pass

    def close(self) -> None:
        try:
            self.proc.stdin.close()
            self.proc.wait(5)
        except (OSError, subprocess.TimeoutExpired):
            self.kill()

    def request(self, files, language: str, threads: int, framework: str, go_doc: bool) -> bytes:
        """One scan; raises OSError / EOFError if the child dies, ScanFailed
        on a reported error."""
        w, r = self.proc.stdin, self.proc.stdout
        head = f"{language or 'auto'}\n{int(threads or 0)}\n{framework or ''}\n{1 if go_doc else 0}".encode()
        # the files go out in ~4 MiB writes (one write per path / content cost
        # ~1 ms of interpreter time per 2,000 files)
        parts = [_HDR.pack(len(head)), head, _HDR.pack(len(files))]
        size = 0
        for rel, data in files.items():
            rb = rel.encode("utf-8", "surrogateescape")
            parts += (_HDR.pack(len(rb)), rb, _HDR.pack(len(data)), data)
            size += len(rb) + len(data)
            if size >= 1 << 22:
                w.write(b"".join(parts))
                parts, size = [], 0
        w.write(b"".join(parts))
        w.flush()
        status = r.read(1)
        hdr = r.read(_HDR.size)
        if len(status) != 1 or len(hdr) != _HDR.size:
            raise EOFError("scan child closed its output")
        n = _HDR.unpack(hdr)[0]
        payload = r.read(n)
        if len(payload) != n:
            raise EOFError("scan child reply truncated")
        self.uses += 1
        if status != b"\x00":
            raise ScanFailed("source scan failed: " + payload.decode("utf-8", "replace")[:500])
        return payload


class ScanChildPool:
    """Persistent isolated scan children (``srcscan serve``) shared by the
    analyses of this process: the untrusted parse still runs outside the
    service process with a time limit, and a crash or hang still kills only
    the child (which is then discarded), but a scan no longer pays a process
    start, and its result crosses the pipe as a binary ScanResult that the
    parent decodes natively into the same objects -- and database rows -- as
    an in-process scan (no JSON document, round-5 verdict item 7).

    A child is reused for at most ``max_uses`` scans (``SCAN_CHILD_MAX_USES``,
    default 64; 1 = a fresh child per scan, the reference's one process per
    analysis, GoSourceParser.java:339-418)."""

    def __init__(self, max_idle: int = 4, max_uses: Optional[int] = None) -> None:
        import threading
        self.max_idle = max_idle
        self.max_uses = max_uses if max_uses is not None else int(os.environ.get("SCAN_CHILD_MAX_USES", "64"))
        self._idle: list = []
        self._lock = threading.Lock()
        self.spawned = 0

    def _env(self, env_extra: Optional[dict]) -> dict:
        env = dict(os.environ)
        env.update(env_extra or {})
        return env

    def scan(self, tree, language: str, threads: int, framework: str = "", timeout_s: float = 120.0,
             go_doc: bool = True, env_extra: Optional[dict] = None) -> bytes:
        """The binary ScanResult of ``tree`` (in-memory snapshot files)."""
        import threading
        cli = native_cli()
        if cli is None:
            raise ScanFailed("the native analyzer binary (bin/srcscan) is missing")
        fault = os.environ.get("DMCP_SCAN_CHILD_FAULT")
        if fault:  # fault injection (tests): a dedicated child that sees it
            env_extra = dict(env_extra or {}, DMCP_SCAN_CHILD_FAULT=fault)
        child = None
        if not env_extra:
            with self._lock:
                while self._idle and child is None:
                    c = self._idle.pop()
                    child = c if c.alive() else None
        if child is None:
            child = _ServeChild(cli, self._env(env_extra))
            self.spawned += 1
        box: dict = {}

        def run() -> None:
            try:
                box["out"] = child.request(tree.files, language, threads, framework, go_doc)
            except BaseException as e:  # noqa: BLE001 -- reported below
                box["err"] = e
        t = threading.Thread(target=run, name="scan-child-io", daemon=True)
        t.start()
        t.join(timeout_s)
        if t.is_alive():
            child.kill()
            t.join(10)
            raise ScanFailed(f"source scan did not finish in {timeout_s:.0f} s (child killed)")
        err = box.get("err")
        if err is not None:
            if isinstance(err, ScanFailed) and child.alive():
                self._release(child, env_extra)  # a reported error: the child itself is fine
                raise err
            child.kill()
            rc = child.proc.returncode
            how = (f"signal {-rc}" if rc is not None and rc < 0 else f"exit code {rc}")
            tail = bytes(child.err).decode("utf-8", "replace").strip().splitlines()[-3:]
            raise ScanFailed(f"source scan process failed ({how}): {' | '.join(tail) or err}") from err
        self._release(child, env_extra)
        return box["out"]

    def _release(self, child: _ServeChild, env_extra: Optional[dict]) -> None:
        if env_extra or child.uses >= self.max_uses or not child.alive():
            child.close()
            return
        with self._lock:
            if len(self._idle) < self.max_idle:
                self._idle.append(child)
                return
        child.close()

    def close(self) -> None:
        with self._lock:
            idle, self._idle = self._idle, []
        for c in idle:
            c.close()


_POOL: Optional[ScanChildPool] = None


def child_pool() -> ScanChildPool:
    global _POOL
    if _POOL is None:
        _POOL = ScanChildPool()
        import atexit
        atexit.register(_POOL.close)
    return _POOL


def objects_supported() -> bool:
    """The persistent binary child path is available: the analyzer binary and
    a module that decodes its result."""
    if native_cli() is None:
        return False
    from .base import native
    return hasattr(native(), "result_objects")


def scan_objects_in_child(tree, language: str, threads: int, framework: str = "", timeout_s: float = 120.0,
                          rows=None, go_doc: bool = True, env_extra: Optional[dict] = None,
                          timing: Optional[dict] = None) -> dict:
    """:meth:`SourceTree.scan_objects` with the parse in a persistent child:
    the same document (objects, ``rowIds`` with ``rows``), the class / method
    rows streamed to the writer by the parent as the result is decoded."""
    from ..models.domain import StaticMethodInfo
    from .base import native
    t0 = time.perf_counter()
    blob = child_pool().scan(tree, language, threads, framework, timeout_s, go_doc=go_doc, env_extra=env_extra)
    t1 = time.perf_counter()
    try:
        doc = native().result_objects(blob, StaticMethodInfo, rows)
    except ValueError as e:
        raise ScanFailed(f"source scan produced an unreadable result: {e}") from e
    if timing is not None:
        # where an isolated scan's time goes: the child round trip (files out,
        # scan, binary result back) and the parent's decode into objects + rows
        timing.update(child_ms=(t1 - t0) * 1e3, decode_ms=(time.perf_counter() - t1) * 1e3)
    return doc


def child_main() -> int:
    rx, tx = sys.stdin.buffer, sys.stdout.buffer
    head = _read_blob(rx)
    if head is None:
        return 2
    h = json.loads(head)
    from .base import native
    if os.environ.get("DMCP_SCAN_CHILD_FAULT") == "hang":  # fault injection for tests
        import time
        time.sleep(3600)
    if os.environ.get("DMCP_SCAN_CHILD_FAULT") == "crash":
        import ctypes
        ctypes.string_at(0)  # SIGSEGV, as a native front-end fault would
    if "root" in h:
        out = native().scan_project(h["root"], h["language"], h["threads"], h["framework"])
    else:
        files = []
        for _ in range(int(h["nfiles"])):
            rel, data = _read_blob(rx), _read_blob(rx)
            if rel is None or data is None:
                return 3
            files.append((rel.decode("utf-8", "surrogateescape"), data))
        out = native().scan_sources(files, h["language"], h["threads"], h["framework"])
    tx.write(out)
    tx.flush()
    return 0


if __name__ == "__main__":
    raise SystemExit(child_main())
