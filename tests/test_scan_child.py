"""The persistent isolated scan child (round 6, verdict item 7): ``srcscan
serve`` parses remote (untrusted) repositories out of the service process
and returns a binary ScanResult (native/srcscan/wire.cpp) that the parent
decodes natively into the same objects -- and database rows -- as an
in-process scan.  Covers: equality with the in-process scan for the three
front-ends, child reuse and replacement after a crash or a hang, the
one-child-per-scan mode, and a decoder that never trusts its input (the
child parsed an untrusted repository): truncated / corrupted results raise,
never crash (``GoSourceParser.java:339-418``: the reference's analyzer
subprocess, 120 s limit, failure = ANALYSIS_FAILED)."""
import os
import random

import pytest

from dmcp.index.git import GitClient
from dmcp.models.domain import RepositoryUrl, StaticMethodInfo
from dmcp.parsers import isolated
from dmcp.parsers.base import native
from dmcp.utils import synth


def _tree(tmp_path, kind):
    root = tmp_path / kind
    if kind == "java":
        synth.java_spring_repo(str(root), 30)
    elif kind == "ts":
        synth.nestjs_repo(str(root), n_modules=6)
    else:
        synth.go_service_repo(str(root), n_packages=6)
    return GitClient(str(tmp_path / f"c{kind}")).snapshot(RepositoryUrl.of(str(root)), None)


def _strip(doc):
    doc = dict(doc)
    doc.pop("stats", None)
    return doc


@pytest.mark.parametrize("kind", ["java", "ts", "go"])
def test_child_result_equals_the_in_process_scan(tmp_path, kind):
    tree = _tree(tmp_path, kind)
    lang = {"java": "java", "ts": "typescript", "go": "go"}[kind]
    inproc = native().scan_sources_objects(list(tree.files.items()), lang, 2, "", StaticMethodInfo)
    child = isolated.scan_objects_in_child(tree, lang, 2, "", 60)
    assert _strip(child) == _strip(inproc)
    assert len(child["files"]) > 0


def test_children_are_reused_and_replaced(tmp_path):
    tree = _tree(tmp_path, "java")
    pool = isolated.ScanChildPool(max_uses=3)
    try:
        blobs = [pool.scan(tree, "java", 1, "", 60) for _ in range(3)]
        assert pool.spawned == 1  # one process for three scans
        assert all(len(b) == len(blobs[0]) for b in blobs)
        pool.scan(tree, "java", 1, "", 60)
        assert pool.spawned == 2  # max_uses reached: a fresh child
        # a child that died while idle is not handed out again
        pool._idle[0].kill()
        pool.scan(tree, "java", 1, "", 60)
        assert pool.spawned == 3
        # faults: the faulty child is discarded, the next scan gets a fresh one
        with pytest.raises(isolated.ScanFailed, match="signal"):
            pool.scan(tree, "java", 1, "", 60, env_extra={"DMCP_SCAN_CHILD_FAULT": "crash"})
        with pytest.raises(isolated.ScanFailed, match="did not finish"):
            pool.scan(tree, "java", 1, "", 2, env_extra={"DMCP_SCAN_CHILD_FAULT": "hang"})
        assert len(pool.scan(tree, "java", 1, "", 60)) == len(blobs[0])
    finally:
        pool.close()
    one = isolated.ScanChildPool(max_uses=1)  # the reference's one analyzer process per analysis
    try:
        for _ in range(3):
            one.scan(tree, "java", 1, "", 60)
        assert one.spawned == 3 and one._idle == []
    finally:
        one.close()


def test_decoder_rejects_corrupt_results(tmp_path):
    """Every truncation and a few thousand random corruptions of a real
    result: ValueError or a well-formed result, never a crash."""
    tree = _tree(tmp_path, "java")
    blob = native().encode_scan(list(tree.files.items()), "java", 1, "", True)
    ok = native().result_objects(blob, StaticMethodInfo)
    assert len(ok["files"]) == 31
    rng = random.Random(7)
    cuts = sorted({0, 1, 3, 4, 5, len(blob) - 1} | {rng.randrange(len(blob)) for _ in range(300)})
    for n in cuts:
        with pytest.raises(ValueError):
            native().result_objects(blob[:n], StaticMethodInfo)
    with pytest.raises(ValueError):
        native().result_objects(blob + b"\0", StaticMethodInfo)  # trailing bytes
    for _ in range(2000):
        b = bytearray(blob)
        for _ in range(rng.randint(1, 8)):
            b[rng.randrange(4, len(b))] = rng.randrange(256)
        try:
            native().result_objects(bytes(b), StaticMethodInfo)
        except (ValueError, UnicodeDecodeError):
            pass
    # huge counts / lengths are refused before any allocation
    import struct
    evil = b"SSW2" + struct.pack("<I", 0xFFFFFFF0)
    with pytest.raises(ValueError):
        native().result_objects(evil, StaticMethodInfo)


def test_remote_analysis_streams_rows_from_the_child(tmp_path):
    """A remote-path analysis (scan isolated in the child) hands the class /
    method rows to the native writer as the local path does, and indexes the
    same rows."""
    from conftest import make_app
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 24)
    app = make_app(tmp_path, scan_isolation="process", require_enrichment_for_analyze=False)
    r = app.indexer.analyze_project(str(repo))
    assert r.success and r.classes_analyzed == 25
    ids = {c.full_class_name: c.id for c in app.repos.classes.find_by_project_id(r.project_id)}
    app.close()
    app2 = make_app(tmp_path / "b", scan_isolation="inline", require_enrichment_for_analyze=False)
    os.makedirs(tmp_path / "b", exist_ok=True)
    r2 = app2.indexer.analyze_project(str(repo))
    names2 = {c.full_class_name for c in app2.repos.classes.find_by_project_id(r2.project_id)}
    assert set(ids) == names2
    app2.close()
