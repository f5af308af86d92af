"""The reference's ``IndexAnalysisTest.analyzeAllQueries`` on SQLite.

``src/test/java/co/fanki/domainmcp/analysis/IndexAnalysisTest.java`` loads
``src/test/resources/index-analysis-data.sql`` (50 projects / 850 classes /
2,250 methods) statement by statement (``:156-186``) and prints ``EXPLAIN
(ANALYZE, BUFFERS)`` for every repository SQL constant (``:191-356``).  Here the
same data file -- plain ``INSERT`` SQL, read as text from the read-only
reference checkout when it is present, otherwise the case is skipped -- is
loaded into the SQLite schema and every statement's ``EXPLAIN QUERY PLAN`` is
checked for index use (the reference only prints; its findings became
migration V4).  ``tests/test_store.py::test_query_plans_use_indexes`` covers the
same shape with generated data, so nothing depends on the reference file.
"""
import os
import time

import pytest

from dmcp.store.db import Database
from dmcp.store.repositories import Repositories, SourceClassRepository, SourceMethodRepository

FIXTURE = "/root/reference/src/test/resources/index-analysis-data.sql"
TEST_PROJECT_ID = "5677b1e8-da1b-4dda-a5a5-71668d09f5f4"      # IndexAnalysisTest.java:125
TEST_CLASS_ID = "b8b003b3-ebfe-9846-fc8e-8c66696648fa"        # :126
TEST_CLASS_NAME = "co.fanki.project0.controller.Api0Controller"  # :127


def load_statements(db, path):
    """``loadTestData`` (:156-186): skip comments/blank lines, execute at ';'."""
    stmt = []
    n = 0
    with db.transaction() as c:
        with open(path, encoding="utf-8") as f:
            for line in f:
                if line.startswith("--") or not line.strip():
                    continue
                stmt.append(line)
                if line.rstrip().endswith(";"):
                    sql = "".join(stmt).strip()
                    stmt = []
                    if sql:
                        c.execute(sql)
                        n += 1
    return n


@pytest.mark.skipif(not os.path.isfile(FIXTURE), reason="reference checkout not mounted")
def test_analyze_all_queries(tmp_path):
    db = Database(str(tmp_path / "index.db"))
    repos = Repositories(db)
    t0 = time.perf_counter()
    load_statements(db, FIXTURE)
    load_ms = (time.perf_counter() - t0) * 1e3
    counts = {t: db.query(f"SELECT COUNT(*) FROM {t}")[0][0] for t in ("projects", "source_classes",
                                                                       "source_methods")}
    assert counts == {"projects": 50, "source_classes": 850, "source_methods": 2250}
    cases = {
        # the SQLite statements (graph JSON joined from project_graphs)
        "ProjectRepository.FIND_BY_ID": (repos.projects.FIND_BY_ID, (TEST_PROJECT_ID,)),
        "ProjectRepository.FIND_BY_REPOSITORY_URL": (repos.projects.FIND_BY_REPOSITORY_URL,
                                                     ("https://github.com/test/project-0.git",)),
        "SourceClassRepository.FIND_BY_ID": (SourceClassRepository.FIND_BY_ID, (TEST_CLASS_ID,)),
        "SourceClassRepository.FIND_BY_PROJECT_ID": (SourceClassRepository.FIND_BY_PROJECT_ID, (TEST_PROJECT_ID,)),
        "SourceClassRepository.FIND_BY_FULL_CLASS_NAME": (SourceClassRepository.FIND_BY_FULL_CLASS_NAME,
                                                          (TEST_CLASS_NAME,)),
        "SourceClassRepository.FIND_BY_PROJECT_ID_AND_FULL_CLASS_NAME": (
            SourceClassRepository.FIND_BY_PROJECT_ID_AND_FULL_CLASS_NAME, (TEST_PROJECT_ID, TEST_CLASS_NAME)),
        "SourceClassRepository.FIND_BY_PACKAGE_PREFIX": (
            SourceClassRepository.FIND_BY_PACKAGE_PREFIX,
            ("co.fanki.project0", "co.fanki.project0.", "co.fanki.project0/")),
        "SourceClassRepository.COUNT_BY_PROJECT_ID": (SourceClassRepository.COUNT_BY_PROJECT_ID, (TEST_PROJECT_ID,)),
        "SourceMethodRepository.FIND_BY_CLASS_ID": (SourceMethodRepository.FIND_BY_CLASS_ID, (TEST_CLASS_ID,)),
        "SourceMethodRepository.FIND_BY_CLASS_NAME": (SourceMethodRepository.FIND_BY_CLASS_NAME, (TEST_CLASS_NAME,)),
        "SourceMethodRepository.FIND_BY_CLASS_ID_AND_METHOD_NAME": (
            SourceMethodRepository.FIND_BY_CLASS_ID_AND_METHOD_NAME, (TEST_CLASS_ID, "getAll")),
        "SourceMethodRepository.FIND_HTTP_ENDPOINTS_BY_PROJECT_ID": (
            SourceMethodRepository.FIND_HTTP_ENDPOINTS_BY_PROJECT_ID, (TEST_PROJECT_ID,)),
        "SourceMethodRepository.COUNT_ENDPOINTS_BY_PROJECT_ID": (
            SourceMethodRepository.COUNT_ENDPOINTS_BY_PROJECT_ID, (TEST_PROJECT_ID,)),
    }
    report = [f"SQLITE QUERY PLAN ANALYSIS (fixture loaded in {load_ms:.1f} ms; {counts})"]
    for name, (sql, params) in cases.items():
        plan = " | ".join(r[3] for r in db.query("EXPLAIN QUERY PLAN " + sql, params))
        q0 = time.perf_counter()
        rows = db.query(sql, params)
        ms = (time.perf_counter() - q0) * 1e3
        report.append(f"{name}: {len(rows)} rows in {ms:.3f} ms :: {plan}")
        # no full-table scan of the big tables; every filter is an index search
        for table in ("source_classes", "source_methods", "projects"):
            assert f"SCAN {table}" not in plan.replace(f"SCAN {table} USING", "SEARCH"), (name, plan)
        assert ms < 50, (name, ms)  # V4 target for the endpoint query was "~50 ms" at 1 M classes
    print("\n".join(report))
    # sanity against the fixture: Project0 has 5 controllers with endpoints
    assert repos.methods.count_endpoints_by_project_id(TEST_PROJECT_ID) > 0
    assert repos.classes.find_by_full_class_name(TEST_CLASS_NAME).id == TEST_CLASS_ID
    db.close()
