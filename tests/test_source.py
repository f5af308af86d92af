"""Source trees: in-memory git snapshots (bare clone + cat-file, native scan of
a mounted tree) must index exactly what a checkout does; size-capped fallback
to a checkout; the native VFS mount."""
import json
import os
import subprocess

import pytest

from conftest import make_app
from dmcp.index.git import GitClient
from dmcp.index.source import CheckoutTree, MemoryTree, detect_language_from, wanted
from dmcp.models.domain import RepositoryUrl
from dmcp.parsers.base import native
from dmcp.utils import synth


def _git(root, *args):
    subprocess.run(["git", "-C", str(root), *args], check=True, capture_output=True)


def test_wanted_and_language_detection():
    assert wanted("src/main/java/A.java") and wanted("web/x.tsx") and wanted("README.md")
    assert not wanted("docs/README.md") and not wanted("node_modules/x/index.js")
    assert not wanted("web/node_modules/y.ts") and not wanted("img.png")
    assert detect_language_from(["go.mod", "main.go"]) == "go"
    assert detect_language_from(["package.json", "src/a.ts"]) == "typescript"
    assert detect_language_from(["package.json", "pom.xml"]) == "java"


@pytest.mark.parametrize("kind", ["java", "nest", "go"])
def test_snapshot_equals_checkout(tmp_path, kind):
    repo = tmp_path / "r"
    if kind == "java":
        synth.java_spring_repo(str(repo), 24)
    elif kind == "nest":
        synth.nestjs_repo(str(repo), 4)
    else:
        synth.go_gin_repo(str(repo), 3)
    g = GitClient(str(tmp_path / "clones"))
    url = RepositoryUrl.of(str(repo))
    mem = g.snapshot(url, "main")
    # a local repository is read in place: nothing to own, nothing deleted
    assert isinstance(mem, MemoryTree) and mem.directory is None and mem.git_dir == str(repo)
    g.read_local_in_place = False  # the private bare-clone path (remote repositories)
    bare = g.snapshot(url, "main")
    assert isinstance(bare, MemoryTree) and not os.path.exists(os.path.join(bare.directory, "README.md"))
    assert bare.files == mem.files and bare.commit_hash == mem.commit_hash
    bare.cleanup()
    c = g.clone(url, "main")
    disk = CheckoutTree(c.directory, c.commit_hash)
    assert mem.commit_hash == disk.commit_hash and mem.detect_language() == disk.detect_language()
    lang = disk.detect_language()
    a, b = json.loads(mem.scan(lang, 4)), json.loads(disk.scan(lang, 4))
    a["stats"] = b["stats"] = None
    assert a == b and a["files"]
    assert mem.readme() == disk.readme()
    some = a["files"][0]["path"]
    assert mem.read_text(some) == disk.read_text(some)
    mem.cleanup()
    disk.cleanup()
    assert not os.listdir(tmp_path / "clones")
    assert os.path.isdir(repo / ".git") and len(os.listdir(repo)) > 1  # source repository untouched


def test_snapshot_fallback_to_checkout_and_errors(tmp_path):
    repo = tmp_path / "r"
    synth.java_spring_repo(str(repo), 8)
    g = GitClient(str(tmp_path / "clones"))
    t = g.snapshot(RepositoryUrl.of(str(repo)), "main", max_bytes=100)
    assert isinstance(t, CheckoutTree) and os.path.isfile(os.path.join(t.directory, "README.md"))
    assert json.loads(t.scan("java", 2))["files"]
    t.cleanup()
    assert not os.path.exists(t.directory)
    with pytest.raises(Exception):
        g.snapshot(RepositoryUrl.of(str(tmp_path / "missing")), "main")
    with pytest.raises(Exception):
        g.snapshot(RepositoryUrl.of(str(repo)), "no-such-branch")
    assert not os.listdir(tmp_path / "clones")


def test_symlinks_and_submodule_entries_skipped(tmp_path):
    repo = tmp_path / "r"
    synth.java_spring_repo(str(repo), 8)
    os.symlink("README.md", repo / "LINK.java")
    _git(repo, "add", "-A")
    _git(repo, "-c", "user.email=a@b", "-c", "user.name=n", "commit", "-qm", "link")
    t = GitClient(str(tmp_path / "c")).snapshot(RepositoryUrl.of(str(repo)), "main")
    assert "LINK.java" not in t.files and "README.md" in t.files
    t.cleanup()


def test_in_memory_and_checkout_pipelines_agree(tmp_path):
    synth.java_spring_repo(str(tmp_path / "shop"), 16)
    results = {}
    for mode in (True, False):
        app = make_app(tmp_path / f"m{mode}", git_in_memory=mode)
        r = app.indexer.analyze_project(str(tmp_path / "shop"))
        g = app.cache.get_graph(r.project_id)
        results[mode] = (r.classes_analyzed, r.endpoints_found, sorted(g.identifiers()),
                         {i: g.dependencies(i) for i in g.identifiers()},
                         sorted(c.description for c in app.repos.classes.find_by_project_id(r.project_id)))
        s = app.indexer.sync_project(app.repos.projects.find_by_id(r.project_id))
        assert s.success
        app.close()
    assert results[True] == results[False]


def test_vfs_mount_listing_and_isolation(tmp_path):
    n = native()
    files = [("src/main/java/a/A.java", b"package a;\nimport b.B;\n@Service public class A {}"),
             ("src/main/java/b/B.java", b"package b;\npublic class B {}")]
    doc = json.loads(n.scan_sources(files, "auto", 2, ""))
    assert doc["language"] == "java" and [f["identifier"] for f in doc["files"]] == ["a.A", "b.B"]
    assert doc["files"][0]["deps"] == ["b.B"] and doc["files"][0]["classType"] == "SERVICE"
    assert json.loads(n.scan_sources([], "java", 1, ""))["files"] == []
    ts = json.loads(n.scan_sources([("package.json", b'{"dependencies":{"express":"4"}}'),
                                    ("src/r.ts", b"router.get('/x', h);\n")], "auto", 1, ""))
    assert ts["language"] == "typescript" and ts["framework"]["name"] == "express" and ts["files"][0]["entryPoint"]


def test_default_procs_tracks_object_store(tmp_path):
    """Loose stores get several readers, packed stores at most two."""
    import subprocess
    from dmcp.index.source import default_procs, mostly_loose
    from dmcp.utils import synth
    src = tmp_path / "src"
    synth.java_spring_repo(str(src), 300)
    bare = tmp_path / "b"
    subprocess.run(["git", "clone", "-q", "--bare", "--shared", str(src), str(bare)], check=True)
    assert mostly_loose(str(bare))
    assert default_procs(str(bare), 2000) >= 1
    subprocess.run(["git", "-C", str(src), "gc", "-q", "--prune=now"], check=True)
    assert not mostly_loose(str(bare))
    assert default_procs(str(bare), 2000) <= 2
    assert default_procs(str(bare), 10) == 1


def test_native_loose_reader_matches_git_with_mixed_store(tmp_path):
    """Loose objects come from the native inflater, packed ones from git; the
    result equals cat-file's for every blob (empty and binary ones included)."""
    import subprocess
    from dmcp.index.git import GitClient
    from dmcp.index.source import _native_loose_reader, _read_via_git, list_tree, read_blobs
    assert _native_loose_reader() is not None, "dmcp._srcscan.read_loose_blobs missing"
    src = tmp_path / "src"
    src.mkdir()

    def git(*a):
        subprocess.run(["git", "-C", str(src), *a], check=True, capture_output=True)
    git("init", "-q")
    git("config", "user.email", "t@t")
    git("config", "user.name", "t")
    for i in range(40):
        (src / f"A{i}.java").write_text(f"package a; class A{i} {{}}\n" * (i + 1))
    git("add", ".")
    git("commit", "-qm", "one")
    git("gc", "-q", "--prune=now")  # first generation packed
    (src / "Empty.java").write_bytes(b"")
    (src / "Bin.java").write_bytes(bytes(range(256)) * 50)
    for i in range(40, 80):
        (src / f"A{i}.java").write_text(f"package a; class A{i} {{ int x = {i}; }}\n" * 30)
    git("add", ".")
    git("commit", "-qm", "two")  # second generation loose
    g = GitClient(str(tmp_path / "c"))
    shas = [s for _, s in list_tree(g, str(src), "HEAD")]
    # force the native path regardless of the loose/packed heuristic
    import dmcp.index.source as S
    orig = S.mostly_loose
    S.mostly_loose = lambda d: True
    try:
        got = read_blobs(g, str(src), shas)
        assert read_blobs(g, str(src), shas, max_bytes=1000) is None
    finally:
        S.mostly_loose = orig
    assert got == _read_via_git(g, str(src), shas, 0, 1)
    assert b"" in got and bytes(range(256)) * 50 in got


@pytest.mark.parametrize("kind", ["java", "nest", "go"])
def test_scan_objects_equal_json_document(tmp_path, kind):
    """The direct-object scan (no JSON round trip) parses to exactly what the
    JSON document parses to."""
    import json as _json
    from dmcp.parsers.base import to_parsed_project
    repo = tmp_path / "r"
    {"java": lambda: synth.java_spring_repo(str(repo), 30),
     "nest": lambda: synth.nestjs_repo(str(repo), 5),
     "go": lambda: synth.go_gin_repo(str(repo), 4)}[kind]()
    t = GitClient(str(tmp_path / "c")).snapshot(RepositoryUrl.of(str(repo)), "main")
    lang = t.detect_language()
    a = to_parsed_project(t.scan_objects(lang, 4))
    b = to_parsed_project(_json.loads(t.scan(lang, 4)))
    a.stats = b.stats = None
    if isinstance(a.go_analysis, str):  # kept as JSON text until asked for (GoSourceParser.go_analysis)
        a.go_analysis = _json.loads(a.go_analysis)
    assert a.units and a == b
    assert all(type(m).__name__ == "StaticMethodInfo" for u in a.units.values() for m in u.methods)


def test_native_ref_and_tree_match_git(tmp_path):
    """resolve_ref / list_tree_loose report what rev-parse <ref>^{commit} and
    ls-tree -r do (nested trees, executables, symlinks, a gitlink, branches,
    lightweight and annotated tags, packed refs), and give up (None) on
    packed objects so git answers."""
    from dmcp import _srcscan
    from dmcp.index.source import _object_dirs, git_dir_of, list_tree, native_commit_tree
    src = tmp_path / "src"
    src.mkdir()

    def git(*a):
        return subprocess.run(["git", "-C", str(src), *a], check=True, capture_output=True, text=True).stdout
    git("init", "-q", "-b", "main")
    git("config", "user.email", "t@t")
    git("config", "user.name", "t")
    for rel in ("a/b/c/D.java", "a/B.java", "z.ts", "a/b/E.go", "ü/Ñ.java"):
        p = src / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(f"// {rel}\n")
    (src / "run.sh").write_text("#!/bin/sh\n")
    os.chmod(src / "run.sh", 0o755)
    os.symlink("z.ts", src / "link.ts")
    git("add", "-A")
    git("update-index", "--add", "--cacheinfo", "160000," + "1" * 40 + ",sub")  # a submodule entry
    git("commit", "-qm", "one")
    git("tag", "light")
    git("checkout", "-qb", "dev")
    (src / "a" / "New.java").write_text("class New {}\n")
    git("add", "-A")
    git("commit", "-qm", "two")
    git("tag", "-a", "rel", "-m", "annotated")
    git("checkout", "-q", "main")
    g = GitClient(str(tmp_path / "c"))
    gd, dirs = git_dir_of(str(src)), _object_dirs(str(src))
    assert gd == str(src / ".git")

    def check():
        for branch in (None, "main", "dev", "light", "rel"):
            refs = g.branch_refs(branch)
            commit = _srcscan.resolve_ref(gd, refs)
            assert commit == g.resolve_commit(str(src), branch), branch
            assert _srcscan.list_tree_loose(dirs, commit) == list_tree(g, str(src), commit)
        assert _srcscan.resolve_ref(gd, g.branch_refs("nope")) is None
    check()
    listing = _srcscan.list_tree_loose(dirs, g.resolve_commit(str(src), "dev"))
    paths = [p for p, _ in listing]
    assert "a/b/c/D.java" in paths and "run.sh" in paths and "ü/Ñ.java" in paths
    assert "link.ts" not in paths and "sub" not in paths
    git("pack-refs", "--all")  # refs now only in packed-refs
    assert not (src / ".git" / "refs" / "tags" / "rel").exists()
    check()
    import dmcp.index.source as S
    orig = S.mostly_loose
    S.mostly_loose = lambda d: True
    try:
        assert native_commit_tree(str(src), ["HEAD"])[0] == g.resolve_commit(str(src), None)
        git("gc", "-q", "--prune=now")  # objects packed: the native reader declines
        assert native_commit_tree(str(src), ["HEAD"]) is None
    finally:
        S.mostly_loose = orig
    snap = g.snapshot(RepositoryUrl.of(str(src)), "dev")  # git path after the fallback
    assert "a/New.java" in snap.files


def _scan_in_child(q):
    from dmcp.parsers.base import native as _native
    files = [(f"src/main/java/a/A{i}.java", f"package a;\npublic class A{i} {{}}".encode()) for i in range(64)]
    q.put(len(json.loads(_native().scan_sources(files, "java", 8, ""))["files"]))


def test_worker_pool_survives_fork():
    """parallel_for's persistent workers: a forked child (multiprocessing)
    scans with a fresh pool instead of waiting on the parent's threads, and
    concurrent scans from several Python threads all complete."""
    import multiprocessing as mp
    import threading
    n = native()
    files = [(f"src/main/java/a/A{i}.java", f"package a;\npublic class A{i} {{}}".encode()) for i in range(64)]
    assert len(json.loads(n.scan_sources(files, "java", 8, ""))["files"]) == 64  # pool started here
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_scan_in_child, args=(q,))
    p.start()
    p.join(60)
    assert p.exitcode == 0 and q.get(timeout=5) == 64
    out = []
    ts = [threading.Thread(target=lambda: out.append(len(json.loads(n.scan_sources(files, "java", 8, ""))["files"])))
          for _ in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert out == [64] * 6


def test_native_ref_reader_refuses_names_git_refuses(tmp_path):
    """A branch name such as '../../x' must not make the native reader open a
    file outside refs/ (git check-ref-format refuses it; the native reader
    returns None so git answers, and git errors)."""
    import subprocess
    from dmcp import _srcscan
    from dmcp.index.source import git_dir_of
    from dmcp.utils import synth
    repo = tmp_path / "r"
    synth.java_spring_repo(str(repo), 4)
    gd = git_dir_of(str(repo))
    head = subprocess.run(["git", "-C", str(repo), "rev-parse", "HEAD"], capture_output=True, text=True).stdout.strip()
    (tmp_path / "evil").write_text(head + "\n")  # a file outside the repository
    branch = subprocess.run(["git", "-C", str(repo), "branch", "--show-current"], capture_output=True,
                            text=True).stdout.strip()
    assert _srcscan.resolve_ref(gd, [f"refs/heads/{branch}"]) == head
    for bad in ["refs/heads/../../../evil", "../../evil", "/etc/passwd", "refs/heads/a.lock", "refs/heads/x@{1}",
                "refs/heads/.hidden", "refs/heads/a b", "refs/heads//x", "refs/heads/x."]:
        assert _srcscan.resolve_ref(gd, [bad]) is None, bad


def test_isolated_scan_matches_in_process_and_survives_faults(tmp_path):
    """The child-process scan (remote repositories) returns the in-process
    document; a crashing or hanging child becomes ScanFailed, and through
    analyze_project an ANALYSIS_FAILED project while this process lives on
    (GoSourceParser.java:62, 339-418: 120 s kill of the native analyzer)."""
    import pytest
    from conftest import make_app
    from dmcp.index.git import GitClient
    from dmcp.models.domain import ProjectStatus, RepositoryUrl
    from dmcp.parsers.base import parser_for
    from dmcp.parsers.isolated import ScanFailed, scan_in_child
    from dmcp.utils import synth
    from dmcp.utils.errors import DomainError
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 24)
    tree = GitClient(str(tmp_path / "c")).snapshot(RepositoryUrl.of(str(repo)), None)
    inproc = parser_for("java").scan_tree(tree)
    iso = parser_for("java").scan_tree(tree, isolate_timeout_s=60)
    assert set(iso.units) == set(inproc.units) and len(iso.units) == 25
    a, b = inproc.units["co.acme.shop.order.OrderController"], iso.units["co.acme.shop.order.OrderController"]
    assert a.methods == b.methods and a.params == b.params and a.class_type == b.class_type
    from dmcp.parsers.isolated import native_cli
    assert native_cli() is not None  # built with the module: the default child
    for native in (True, False):  # bin/srcscan stdin, and the Python child
        doc = scan_in_child(tree, "java", 1, "", 60, native=native)
        assert len(doc["files"] if "files" in doc else doc.get("units", doc)) > 0
        with pytest.raises(ScanFailed, match="signal"):
            scan_in_child(tree, "java", 1, "", 60, env_extra={"DMCP_SCAN_CHILD_FAULT": "crash"}, native=native)
        with pytest.raises(ScanFailed, match="did not finish"):
            scan_in_child(tree, "java", 1, "", 2, env_extra={"DMCP_SCAN_CHILD_FAULT": "hang"}, native=native)
    docs = [scan_in_child(tree, "java", 1, "", 60, native=n) for n in (True, False)]
    for d in docs:
        d.pop("stats", None)  # timings
    assert docs[0] == docs[1]
    app = make_app(tmp_path, scan_isolation="process", scan_timeout_seconds=2.0)
    assert app.indexer.analyze_project(str(repo)).success  # isolated, healthy
    import os
    os.environ["DMCP_SCAN_CHILD_FAULT"] = "hang"
    try:
        with pytest.raises(DomainError) as e:
            app.indexer.analyze_project(str(repo))
    finally:
        del os.environ["DMCP_SCAN_CHILD_FAULT"]
    assert e.value.error_code == "ANALYSIS_FAILED" and "did not finish" in str(e.value)
    p = app.repos.projects.find_by_name("shop")
    assert p.status is ProjectStatus.ERROR
    assert app.repos.classes.count_by_project()[p.id] == 25  # the previous analysis' rows survive
    assert app.indexer.analyze_project(str(repo)).success  # and the server carries on
    app.close()


def test_go_document_on_demand(tmp_path):
    """The Go analyzer's package document: parsed only when asked for
    (GoSourceParser.go_analysis), and not rendered at all on the indexing
    pipeline's path (go_doc=False) -- the units are the same either way."""
    from dmcp.models.domain import StaticMethodInfo
    from dmcp.parsers.base import GoSourceParser, native, to_parsed_project
    repo = tmp_path / "r"
    synth.go_gin_repo(str(repo), 3)
    t = GitClient(str(tmp_path / "c")).snapshot(RepositoryUrl.of(str(repo)), "main")
    p = GoSourceParser(2)
    p.scan_tree(t)
    assert isinstance(p.project.go_analysis, str)
    doc = p.go_analysis()
    assert isinstance(doc, dict) and doc["packages"] and p.go_analysis() is doc
    fn = native().scan_sources_objects
    with_doc = fn(list(t.files.items()), "go", 2, "", StaticMethodInfo)
    without = fn(list(t.files.items()), "go", 2, "", StaticMethodInfo, None, go_doc=False)
    assert with_doc["go"] and without["go"] is None
    a, b = to_parsed_project(with_doc), to_parsed_project(without)
    assert a.units == b.units and a.file_to_identifier == b.file_to_identifier
