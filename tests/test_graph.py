"""ProjectGraph behaviours (ProjectGraphTest in the reference) + cache."""
import json

import pytest

from dmcp.graph.cache import GraphCache
from dmcp.graph.project_graph import (FrozenGraphError, MethodEnrichmentData, MethodInfo, ProjectGraph)


def chain():
    g = ProjectGraph()
    for n in "ABCD":
        g.add_node(f"co.{n}", f"src/{n}.java")
    g.add_dependency("co.A", "co.B")
    g.add_dependency("co.B", "co.C")
    g.mark_as_entry_point("co.A")
    return g


def test_nodes_and_overwrite():
    g = ProjectGraph()
    g.add_node("a", "x.java")
    g.add_node("b", "y.java")
    g.add_node("a", "z.java")
    assert g.node_count() == 2 and g.source_file("a") == "z.java"
    for bad in ((None, "f"), ("", "f"), ("a", None), ("a", "  ")):
        with pytest.raises(ValueError):
            g.add_node(*bad)


def test_dependencies_require_known_nodes():
    g = chain()
    g.add_dependency("co.A", "co.Unknown")
    g.add_dependency("co.Unknown", "co.A")
    g.add_dependency("co.A", "co.B")  # duplicate
    assert g.dependencies("co.A") == ("co.B",)
    assert g.dependencies("co.D") == () and g.dependencies("nope") == () and g.dependencies(None) == ()
    with pytest.raises(ValueError):
        g.add_dependency(None, "co.A")
    with pytest.raises(ValueError):
        g.add_dependency("co.A", " ")


def test_dependents_reverse_index():
    g = chain()
    g.add_node("co.E", "E.java")
    g.add_dependency("co.E", "co.C")
    assert g.dependents("co.C") == ("co.B", "co.E")
    assert g.dependents("co.A") == () and g.dependents(None) == () and g.dependents("x") == ()
    assert isinstance(g.dependents("co.C"), tuple)  # immutable view


def test_entry_points():
    g = chain()
    g.mark_as_entry_point("co.Unknown")
    g.mark_as_entry_point("co.A")
    assert g.entry_point_count() == 1 and g.is_entry_point("co.A") and not g.is_entry_point("co.B")
    assert not g.is_entry_point(None)
    with pytest.raises(ValueError):
        g.mark_as_entry_point("")


def test_resolve_both_directions_cycles_and_self():
    g = chain()
    assert set(g.resolve("co.B")) == {"co.A", "co.C"}
    assert g.resolve("co.C") == ("co.B",)
    assert g.resolve("co.D") == () and g.resolve(None) == () and g.resolve("x") == ()
    g.add_dependency("co.C", "co.A")
    assert set(g.resolve("co.A")) == {"co.B", "co.C"}
    g.add_dependency("co.D", "co.D")
    assert g.resolve("co.D") == ("co.D",)


def test_analysis_order_bfs_then_orphans():
    g = ProjectGraph()
    for n in ["ctl", "svc", "repo", "ent", "orphan", "ctl2", "dto"]:
        g.add_node(n, n + ".java")
    g.add_dependency("ctl", "svc")
    g.add_dependency("svc", "repo")
    g.add_dependency("repo", "ent")
    g.add_dependency("ctl2", "dto")
    g.add_dependency("ctl2", "svc")
    g.mark_as_entry_point("ctl")
    g.mark_as_entry_point("ctl2")
    order = g.analysis_order()
    assert order[:2] == ["ctl", "ctl2"]
    assert order.index("svc") < order.index("repo") < order.index("ent")
    assert order[-1] == "orphan" and len(order) == len(set(order)) == 7
    assert ProjectGraph().analysis_order() == []


def test_analysis_order_cycle_terminates():
    g = chain()
    g.add_dependency("co.C", "co.A")
    assert g.analysis_order() == ["co.A", "co.B", "co.C", "co.D"]


def test_class_ids():
    g = chain()
    g.bind_class_id("co.A", "id1")
    g.bind_class_id("co.A", "id2")
    assert g.class_id("co.A") == "id2" and g.class_id("co.B") is None and g.class_id("zz") is None
    with pytest.raises(ValueError):
        g.bind_class_id("co.A", " ")


def test_method_parameters():
    g = chain()
    g.add_method_parameter("co.A", "create", 0, "co.B")
    g.add_method_parameter("co.A", "create", 1, "co.C")
    g.add_method_parameter("co.A", "find", 0, "co.C")
    g.add_method_parameter("co.A", "x", 0, "co.Nope")
    g.add_method_parameter("co.Nope", "x", 0, "co.A")
    mp = g.method_parameters("co.A")
    assert [(l.position, l.target_identifier) for l in mp["create"]] == [(0, "co.B"), (1, "co.C")]
    assert set(mp) == {"create", "find"}
    assert g.method_parameter_targets("co.A") == ("co.B", "co.C")
    assert g.method_parameters("co.B") == {} and g.method_parameter_targets("co.B") == ()
    with pytest.raises(ValueError):
        g.add_method_parameter("co.A", "m", -1, "co.B")
    with pytest.raises(ValueError):
        g.add_method_parameter("co.A", None, 0, "co.B")


def test_metadata_endpoints_and_enrichment():
    g = chain()
    g.set_node_info("co.A", "CONTROLLER", None)
    g.add_method_info("co.A", MethodInfo("list", None, (), (), "GET", "/a", 5))
    g.add_method_info("co.A", MethodInfo("helper", None, (), ("IOException",), None, None, 9))
    g.add_method_info("co.B", MethodInfo("run", None, (), (), "GET", None, 3))
    eps = g.all_endpoints()
    assert [(i, m.method_name) for i, m in eps] == [("co.A", "list")]
    assert eps[0][1].http_endpoint() == "GET /a" and g.methods("co.B")[0].http_endpoint() is None
    assert g.methods("nope") == ()
    g.apply_enrichment("co.A", "CONTROLLER", "Lists things", {"list": MethodEnrichmentData("Lists", ("a", "b"))})
    assert g.node_info("co.A").description == "Lists things"
    lst = g.methods("co.A")[0]
    assert lst.description == "Lists" and lst.business_logic == ("a", "b") and lst.http_path == "/a"
    assert g.methods("co.A")[1].exceptions == ("IOException",)
    assert g.has_metadata() and not ProjectGraph().has_metadata()


def test_json_round_trip():
    g = chain()
    g.bind_class_id("co.A", "c1")
    g.add_method_parameter("co.A", "m", 0, "co.B")
    g.set_node_info("co.A", "CONTROLLER", "desc")
    g.set_node_info("co.B", None, None)
    g.add_method_info("co.A", MethodInfo("m", "d", ("s1",), ("E",), "POST", "/x", 7))
    g.add_method_info("co.A", MethodInfo("n"))
    r = ProjectGraph.from_json(g.to_json())
    assert r.identifiers() == g.identifiers() and r.dependencies("co.A") == ("co.B",)
    assert r.dependents("co.B") == ("co.A",) and r.entry_points() == ("co.A",)
    assert r.class_id("co.A") == "c1" and r.source_file("co.D") == "src/D.java"
    assert r.method_parameters("co.A") == g.method_parameters("co.A")
    assert r.node_info("co.A") == g.node_info("co.A") and r.node_info("co.B").class_type is None
    assert r.methods("co.A") == g.methods("co.A")
    assert r.analysis_order() == g.analysis_order()
    doc = json.loads(g.to_json())
    assert set(doc) >= {"nodes", "edges", "entryPoints", "methodParameters", "nodeInfo", "methodInfo"}
    assert doc["nodes"]["co.A"] == {"sourceFile": "src/A.java", "classId": "c1"}
    assert ProjectGraph.from_json(ProjectGraph().to_json()).node_count() == 0


def test_old_format_and_bad_json():
    old = '{"nodes":{"co.fanki.A":{"sourceFile":"src/A.java"}},"edges":{},"entryPoints":[]}'
    r = ProjectGraph.from_json(old)
    assert r.node_count() == 1 and r.method_parameters("co.fanki.A") == {} and not r.has_metadata()
    for bad in (None, "  "):
        with pytest.raises(ValueError):
            ProjectGraph.from_json(bad)
    with pytest.raises(ValueError):
        ProjectGraph.from_json("{invalid-json")


def test_freeze_and_copy():
    g = chain().freeze()
    with pytest.raises(FrozenGraphError):
        g.add_node("x", "y")
    c = g.copy()
    c.add_node("x", "y")
    assert c.contains("x") and not g.contains("x") and not c.frozen


def test_cache_put_rename_and_load(tmp_db):
    from dmcp.models.domain import Project, RepositoryUrl
    from dmcp.store.repositories import Repositories
    repos = Repositories(tmp_db)
    cache = GraphCache(repos.projects)
    g = chain()
    cache.put("p1", "shop", g)
    assert g.frozen and cache.get_graph_by_project_name("shop") is g and cache.get_project_id_by_name("shop") == "p1"
    cache.put("p1", "shop2", chain())
    assert cache.get_graph_by_project_name("shop") is None and cache.get_graph("p1").contains("co.A")
    assert cache.get_graph(None) is None and cache.get_graph_by_project_name(None) is None
    # load_all: one corrupt graph does not block the others
    good = Project.create("good", RepositoryUrl.of("https://github.com/a/good.git"))
    good.graph_data = chain().to_json()
    bad = Project.create("bad", RepositoryUrl.of("https://github.com/a/bad.git"))
    bad.graph_data = "{not json"
    repos.projects.save(good)
    repos.projects.save(bad)
    fresh = GraphCache(repos.projects)
    assert fresh.load_all() == 1 and fresh.get_graph_by_project_name("good") is not None
    assert fresh.reload(good.id) and not fresh.reload(bad.id) and not fresh.reload("missing")
    fresh.evict(good.id)
    assert fresh.get_graph(good.id) is None


def test_load_static_metadata_equals_per_call_api():
    """The Phase 1 bulk loader builds exactly the graph the per-element
    setters build (link positions kept when a target is not a node)."""
    from dmcp.graph.project_graph import MethodInfo, ProjectGraph

    def base():
        g = ProjectGraph()
        for n in ("a.A", "a.B", "a.C"):
            g.add_node(n, n.replace(".", "/") + ".java")
        g.add_dependency("a.A", "a.B")
        return g
    infos = {"a.A": [MethodInfo("run", None, (), ("E",), "GET", "/x", 3)], "a.B": [], "a.C": []}
    params = {"a.A": {"run": ["a.B", "x.Missing", "a.C"], "stop": ["a.C"]}, "zz.NotANode": {"m": ["a.A"]}}
    g1 = base()
    for ident, cid in (("a.A", "1"), ("a.B", "2"), ("a.C", "3")):
        g1.bind_class_id(ident, cid)
        g1.set_node_info(ident, "SERVICE", None)
        g1.set_method_infos(ident, infos[ident])
    for ident, per in params.items():
        for m, targets in per.items():
            for pos, t in enumerate(targets):
                g1.add_method_parameter(ident, m, pos, t)
    g2 = base()
    g2.load_static_metadata({"a.A": "1", "a.B": "2", "a.C": "3"}, {k: "SERVICE" for k in ("a.A", "a.B", "a.C")},
                            infos, params)
    assert g1.to_dict() == g2.to_dict()
    assert [(l.position, l.target_identifier) for l in g2.method_parameters("a.A")["run"]] == [(0, "a.B"), (2, "a.C")]


def test_native_json_encoder_is_byte_identical_to_json_dumps():
    """``_srcscan.graph_json`` (native/srcscan/graphjson.hpp) vs the dict + json.dumps path,
    including escapes, non-ASCII, empty strings and absent optional fields."""
    from dmcp.graph import project_graph as pg
    assert pg._native_encoder() is not None, "native encoder must be built"
    g = ProjectGraph()
    odd = 'a"\\\n\x01é  '
    g.add_node(odd, "f\t.java")
    g.add_node("b", "b.java")
    g.add_node("c", "c.java")
    g.add_dependency(odd, "b")
    g.add_dependency("b", "c")
    g.mark_as_entry_point("b")
    g.bind_class_id("b", "cid")
    g.add_method_parameter("b", "m", 0, odd)
    g.add_method_parameter("b", "m", 3, "c")
    g.set_node_info("b", None, "d\x1f")
    g.set_node_info(odd, "SERVICE", None)
    g.add_method_info("b", MethodInfo("m", "", ("x", "y\"z"), (), "GET", "/p", 0))
    g.add_method_info("b", MethodInfo("n", None, [], ["E"], None, None, None))
    for graph in (g, ProjectGraph()):
        assert graph.to_json() == json.dumps(graph.to_dict(), separators=(",", ":"), ensure_ascii=False)
        assert ProjectGraph.from_json(graph.to_json()).to_dict() == graph.to_dict()


def test_native_json_encoder_falls_back_on_unexpected_types():
    g = ProjectGraph()
    g.add_node("a", "a.java")
    g.add_method_info("a", MethodInfo("m", line_number=3.5))  # float line: not an int
    assert json.loads(g.to_json())["methodInfo"]["a"][0]["lineNumber"] == 3.5
