"""In-tree native build driver (no pip install, no JIT cache).

Builds, into the source tree so the artefacts travel with the repo snapshot:

* ``dmcp/_srcscan<ext>``  -- pybind11 module over ``native/srcscan`` (host C++17)
* ``bin/srcscan``         -- the standalone analyzer CLI (go-analyzer replacement)
* ``bin/srcscan-asan``    -- optional ASan/UBSan build of the CLI (``--sanitize``)
* ``build/asan/_srcscan<ext>`` -- optional ASan/UBSan build of the Python
  module (``--sanitize``); ``DMCP_SRCSCAN_SO=<path>`` makes ``dmcp`` load it,
  under ``LD_PRELOAD=$(gcc -print-file-name=libasan.so)`` (scripts/asan_tests.sh)
* ``dmcp/ops/_hipops<ext>`` -- HIP kernels for gfx950 (see :mod:`dmcp.ops.build`)
* ``dmcp/enrich/_grammar<ext>`` -- the local engine's native grammar / step
  builder (``native/grammar/engine.cpp``, host C++17 + pybind11)

Usage: ``python -m dmcp.buildtools [--sanitize] [--no-hip] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from typing import List, Sequence

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "native", "srcscan")
BUILD = os.path.join(ROOT, "build", "native")
BIN = os.path.join(ROOT, "bin")

CORE_SOURCES = ["common.cpp", "java_frontend.cpp", "ts_frontend.cpp", "go_frontend.cpp", "project.cpp", "gitobj.cpp",
                "wire.cpp"]
MODULE_SOURCES = ["bulkwriter.cpp"]
CXX = os.environ.get("CXX", "g++")
CXXFLAGS = ["-std=c++17", "-O3", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread"]


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def srcscan_module_path() -> str:
    return os.path.join(ROOT, "dmcp", "_srcscan" + ext_suffix())


def _digest(paths: Sequence[str], extra: str = "") -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def _compile_objects(flags: List[str], tag: str, jobs: int) -> List[str]:
    os.makedirs(BUILD, exist_ok=True)
    headers = [os.path.join(NATIVE, h) for h in os.listdir(NATIVE) if h.endswith(".hpp")]

    def one(src: str) -> str:
        s = os.path.join(NATIVE, src)
        key = _digest([s] + headers, " ".join(flags))
        obj = os.path.join(BUILD, f"{src[:-4]}.{tag}.{key}.o")
        if not os.path.exists(obj):
            _run([CXX, *flags, "-c", s, "-o", obj])
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        return list(ex.map(one, CORE_SOURCES))


def build_srcscan(force: bool = False, sanitize: bool = False, jobs: int = 0) -> str:
    jobs = jobs or min(8, os.cpu_count() or 4)
    sources = [os.path.join(NATIVE, s) for s in os.listdir(NATIVE) if s.endswith((".cpp", ".hpp"))]
    stamp = os.path.join(BUILD, "srcscan.stamp")
    key = _digest(sources, " ".join(CXXFLAGS) + sys.version)
    target = srcscan_module_path()
    cli = os.path.join(BIN, "srcscan")
    if (not force and os.path.exists(target) and os.path.exists(cli) and os.path.exists(stamp)
            and open(stamp).read().strip() == key):
        if not sanitize or os.path.exists(os.path.join(BIN, "srcscan-asan")):
            return target
    objs = _compile_objects(CXXFLAGS, "rel", jobs)
    import pybind11  # noqa: WPS433 (build-time only)
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{NATIVE}"]
    py_obj = os.path.join(BUILD, f"pymodule.{_digest([os.path.join(NATIVE, 'pymodule.cpp')])}.o")
    _run([CXX, *CXXFLAGS, *inc, "-fvisibility=hidden", "-c", os.path.join(NATIVE, "pymodule.cpp"), "-o", py_obj])
    # module-only sources (the CLI does not write the database): the bulk row
    # writer links the system libsqlite3 runtime (the library Python's sqlite3
    # uses); the loose-object reader (core: the VFS inflates lazily) links zlib
    mod_objs = []
    for src in MODULE_SOURCES:
        obj = os.path.join(BUILD, src[:-4] + ".o")
        _run([CXX, *CXXFLAGS, f"-I{NATIVE}", "-c", os.path.join(NATIVE, src), "-o", obj])
        mod_objs.append(obj)
    tmp = target + ".tmp"
    _run([CXX, "-shared", "-pthread", "-o", tmp, py_obj, *mod_objs, *objs, "-l:libsqlite3.so.0", "-lz"])
    os.replace(tmp, target)
    os.makedirs(BIN, exist_ok=True)
    _run([CXX, *CXXFLAGS, "-o", cli, os.path.join(NATIVE, "cli.cpp"), *objs, "-lz"])
    if sanitize:
        san = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
               "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
        sobjs = _compile_objects(san, "asan", jobs)
        _run([CXX, *san, "-o", os.path.join(BIN, "srcscan-asan"), os.path.join(NATIVE, "cli.cpp"), *sobjs, "-lz"])
    with open(stamp, "w") as f:
        f.write(key)
    return target


GRAMMAR_SRC = os.path.join(ROOT, "native", "grammar", "engine.cpp")


def grammar_module_path() -> str:
    return os.path.join(ROOT, "dmcp", "enrich", "_grammar" + ext_suffix())


def build_grammar(force: bool = False) -> str:
    """``dmcp/enrich/_grammar<ext>`` (rebuilt when its source changes)."""
    target = grammar_module_path()
    stamp = os.path.join(BUILD, "grammar.stamp")
    key = _digest([GRAMMAR_SRC], " ".join(CXXFLAGS) + sys.version)
    if not force and os.path.exists(target) and os.path.exists(stamp) and open(stamp).read().strip() == key:
        return target
    import pybind11  # noqa: WPS433 (build-time only)
    os.makedirs(BUILD, exist_ok=True)
    tmp = target + ".tmp"
    _run([CXX, *CXXFLAGS, "-shared", "-fvisibility=hidden", f"-I{pybind11.get_include()}",
          f"-I{sysconfig.get_paths()['include']}", "-o", tmp, GRAMMAR_SRC])
    os.replace(tmp, target)
    with open(stamp, "w") as f:
        f.write(key)
    return target


SAN_FLAGS = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fPIC", "-pthread",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]


def asan_module_path() -> str:
    return os.path.join(ROOT, "build", "asan", "_srcscan" + ext_suffix())


def build_srcscan_asan(jobs: int = 0) -> str:
    """The Python module with AddressSanitizer + UBSan (host code only):
    every native path the server runs -- lexers, front-ends, in-memory tree,
    loose-object inflater, bulk row writer, row builders -- instrumented."""
    jobs = jobs or min(8, os.cpu_count() or 4)
    target = asan_module_path()
    sources = [os.path.join(NATIVE, s) for s in os.listdir(NATIVE) if s.endswith((".cpp", ".hpp"))]
    key = _digest(sources, " ".join(SAN_FLAGS) + sys.version)
    stamp = target + ".stamp"
    if os.path.exists(target) and os.path.exists(stamp) and open(stamp).read().strip() == key:
        return target
    objs = _compile_objects(SAN_FLAGS, "asan", jobs)
    import pybind11  # noqa: WPS433 (build-time only)
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{NATIVE}"]
    os.makedirs(os.path.dirname(target), exist_ok=True)
    extra = []
    for src in ["pymodule.cpp", *MODULE_SOURCES]:
        obj = os.path.join(BUILD, src[:-4] + ".asan.o")
        _run([CXX, *SAN_FLAGS, *inc, "-fvisibility=hidden", "-c", os.path.join(NATIVE, src), "-o", obj])
        extra.append(obj)
    tmp = target + ".tmp"
    _run([CXX, *SAN_FLAGS, "-shared", "-o", tmp, *extra, *objs, "-l:libsqlite3.so.0", "-lz"])
    os.replace(tmp, target)
    with open(stamp, "w") as f:
        f.write(key)
    return target


def grammar_asan_module_path() -> str:
    return os.path.join(ROOT, "build", "asan", "_grammar" + ext_suffix())


def build_grammar_asan() -> str:
    """The native grammar engine with AddressSanitizer + UBSan (host code):
    loaded instead of ``dmcp/enrich/_grammar`` when ``DMCP_GRAMMAR_SO`` names
    it (scripts/asan_tests.sh, tests/test_grammar_fuzz.py)."""
    target = grammar_asan_module_path()
    key = _digest([GRAMMAR_SRC], " ".join(SAN_FLAGS) + sys.version)
    stamp = target + ".stamp"
    if os.path.exists(target) and os.path.exists(stamp) and open(stamp).read().strip() == key:
        return target
    import pybind11  # noqa: WPS433 (build-time only)
    os.makedirs(os.path.dirname(target), exist_ok=True)
    tmp = target + ".tmp"
    _run([CXX, *SAN_FLAGS, "-shared", "-fvisibility=hidden", f"-I{pybind11.get_include()}",
          f"-I{sysconfig.get_paths()['include']}", "-o", tmp, GRAMMAR_SRC])
    os.replace(tmp, target)
    with open(stamp, "w") as f:
        f.write(key)
    return target


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="also build bin/srcscan-asan")
    ap.add_argument("--no-hip", action="store_true", help="skip the gfx950 HIP kernels")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(argv)
    print(build_srcscan(force=a.force, sanitize=a.sanitize, jobs=a.jobs))
    print(build_grammar(force=a.force))
    if a.sanitize:
        print(build_srcscan_asan(jobs=a.jobs))
        print(build_grammar_asan())
    if not a.no_hip:
        try:
            from dmcp.ops import build as hipbuild
        except ImportError:
            hipbuild = None
        if hipbuild is not None:
            print(hipbuild.build(force=a.force))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
