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
