"""Graph query DSL (GraphQueryTest / GraphQueryServiceTest) and the context
read operations (CodeContextServiceTest) against an analyzed synthetic repo."""
import pytest

from dmcp.query.context import candidate_class_names, candidate_method_names
from dmcp.query.dsl import GraphQuery, TokenType
from dmcp.utils.errors import DomainError

O = "co.acme.shop.order"
U = "co.acme.shop.user"


# ------------------------------------------------------------------ lexer
def test_parse_basic_and_tokens():
    q = GraphQuery.parse("  shop:OrderService:methods:+logic:?create ")
    assert q.project == "shop" and q.raw == "shop:OrderService:methods:+logic:?create"
    assert [(t.type, t.value) for t in q.tokens] == [
        (TokenType.NAVIGATE, "OrderService"), (TokenType.NAVIGATE, "methods"),
        (TokenType.INCLUDE, "logic"), (TokenType.CHECK, "create")]
    assert q.first_navigation() == "OrderService" and q.navigations_from(1) == ["methods"]
    assert q.navigations_from(5) == [] and q.has_include("LOGIC") and q.has_check()
    assert q.check_value() == "create" and [str(t) for t in q.tokens][2:] == ["+logic", "?create"]


def test_parse_trailing_and_empty_segments():
    q = GraphQuery.parse("shop:endpoints::")  # Java split drops trailing empties
    assert [t.value for t in q.tokens] == ["endpoints"]
    q = GraphQuery.parse("shop:A::methods")
    assert [t.value for t in q.tokens] == ["A", "methods"]


@pytest.mark.parametrize("bad,msg", [
    (None, "required"), ("   ", "required"), ("shop", "at least project:target"),
    ("shop:", "at least project:target"), (" :X", "Project name"), ("shop:+logic", "navigation target"),
    ("shop:?x", "navigation target"), ("shop:X:+", "requires a value"), ("shop:X:?", "requires a value"),
    ("shop: : ", "at least one target")])
def test_parse_errors(bad, msg):
    with pytest.raises(DomainError) as e:
        GraphQuery.parse(bad)
    assert e.value.error_code == "INVALID_QUERY" and msg in e.value.message


# --------------------------------------------------------------- executor
def test_endpoints_and_logic(java_app):
    r = java_app.graph_query.query("shop:endpoints").to_dict()
    assert r["resultType"] == "endpoints" and r["project"] == "shop" and r["count"] == 10
    first = r["results"][0]
    assert set(first) == {"className", "classType", "methodName", "httpMethod", "httpPath", "description"}
    assert first["classType"] == "CONTROLLER" and first["description"].startswith("Performs")
    r2 = java_app.graph_query.query("shop:ENDPOINTS:+logic").to_dict()
    assert r2["results"][0]["businessLogic"] and r2["count"] == 10


def test_classes_with_includes(java_app):
    r = java_app.graph_query.query("shop:classes:+dependencies:+dependents:+methods").to_dict()
    assert r["count"] == 17
    svc = next(x for x in r["results"] if x["className"] == f"{O}.OrderService")
    assert f"{U}.UserService" in svc["dependencies"] and svc["classType"] == "SERVICE"
    assert "dependents" in svc and svc["methods"] and not svc["entryPoint"]
    plain = java_app.graph_query.query("shop:classes").to_dict()["results"][0]
    assert "dependencies" not in plain and "methods" not in plain


def test_entrypoints(java_app):
    r = java_app.graph_query.query("shop:entrypoints:+logic").to_dict()
    names = {x["className"] for x in r["results"]}
    assert {f"{O}.OrderController", f"{U}.UserController", "co.acme.shop.Application"} <= names
    ctl = next(x for x in r["results"] if x["className"] == f"{O}.OrderController")
    assert len(ctl["endpoints"]) == 5 and "businessLogic" in ctl["endpoints"][0]
    assert ctl["endpoints"][0]["httpEndpoint"] == "GET /"


def test_vertex_resolution_order(java_app):
    g = java_app.cache.get_graph_by_project_name("shop")
    rs = java_app.graph_query.resolve_class_name
    assert rs(f"{O}.Order", g) == f"{O}.Order"
    assert rs("orderservice", g) == f"{O}.OrderService"   # simple name, case-insensitive
    assert rs("UserRepo", g) == f"{U}.UserRepository"      # substring
    assert rs("NoSuchThing", g) is None


def test_vertex_overview_methods_deps(java_app):
    gq = java_app.graph_query
    ov = gq.query("shop:OrderService").to_dict()
    assert ov["resultType"] == "class" and ov["count"] == 1
    item = ov["results"][0]
    assert item["className"] == f"{O}.OrderService" and "businessLogic" not in item["methods"][0]
    assert gq.query("shop:OrderService:+logic").to_dict()["results"][0]["methods"][0]["businessLogic"]
    ms = gq.query("shop:OrderService:methods").to_dict()
    assert ms["resultType"] == "methods" and all("lineNumber" in m for m in ms["results"])
    deps = gq.query("shop:OrderService:dependencies").to_dict()
    assert deps["resultType"] == "dependencies" and f"{U}.UserService" in [d["className"] for d in deps["results"]]
    dents = gq.query("shop:UserService:dependents").to_dict()
    assert f"{O}.OrderService" in [d["className"] for d in dents["results"]]
    assert gq.query("shop:OrderService:whatever").to_dict()["resultType"] == "class"


def test_single_method_and_check(java_app):
    gq = java_app.graph_query
    m = gq.query("shop:OrderController:method:LIST").to_dict()
    assert m["resultType"] == "method" and m["results"][0]["httpMethod"] == "GET"
    c = gq.query("shop:OrderController:methods:?list").to_dict()  # check beats sub-navigation
    assert c["resultType"] == "check" and c["results"][0]["exists"] and c["results"][0]["httpEndpoint"] == "GET /"
    c2 = gq.query("shop:OrderController:?nope").to_dict()["results"][0]
    assert c2 == {"className": f"{O}.OrderController", "check": "nope", "exists": False}
    with pytest.raises(DomainError) as e:
        gq.query("shop:OrderController:method")
    assert e.value.error_code == "INVALID_QUERY"
    with pytest.raises(DomainError) as e:
        gq.query("shop:OrderController:method:nope")
    assert e.value.error_code == "METHOD_NOT_FOUND"


def test_not_found_errors(java_app):
    with pytest.raises(DomainError) as e:
        java_app.graph_query.query("nosuch:endpoints")
    assert e.value.error_code == "PROJECT_NOT_FOUND"
    with pytest.raises(DomainError) as e:
        java_app.graph_query.query("shop:Zzzz")
    assert e.value.error_code == "CLASS_NOT_FOUND"


# ---------------------------------------------------------------- context
def test_list_and_search(java_app):
    ps = java_app.context.list_projects()
    assert len(ps) == 1 and ps[0]["name"] == "shop" and ps[0]["basePackage"] == "co.acme.shop"
    assert ps[0]["classCount"] == 17 and ps[0]["endpointCount"] == 10 and ps[0]["status"] == "ANALYZED"
    s = java_app.context.search_project("shop", "order")
    assert s["found"] and s["totalClassesInProject"] == 17 and len(s["matches"]) == 8
    assert all(m["description"] for m in s["matches"])
    miss = java_app.context.search_project("nope", "x")
    assert not miss["found"] and "list_projects" in miss["message"]


def test_class_context(java_app):
    c = java_app.context.get_class_context(f"{O}.OrderService")
    assert c["found"] and c["classType"] == "SERVICE" and c["projectUrl"].endswith("shop")
    assert c["graphInfo"]["dependencies"] and c["methods"][0]["businessLogic"]
    assert list(c) == ["found", "className", "classType", "description", "projectDescription", "methods",
                       "projectUrl", "message", "knownProjects", "graphInfo"]
    scoped = java_app.context.get_class_context(f"{O}.OrderService", "shop")
    assert scoped["found"]
    miss = java_app.context.get_class_context("com.x.Nope")
    assert not miss["found"] and miss["knownProjects"][0]["basePackage"] == "co.acme.shop"
    assert not java_app.context.get_class_context(f"{O}.OrderService", "other")["found"]


def test_method_context(java_app):
    m = java_app.context.get_method_context(f"{O}.OrderController", "search")
    assert m["found"] and m["httpEndpoint"] == "POST /search/{id}" and m["lineNumber"]
    assert [p["typeName"] for p in m["parameterTypes"]] == [f"{O}.OrderRequest"]
    nm = java_app.context.get_method_context(f"{O}.OrderController", "nope")
    assert not nm["found"] and nm["message"] == "Class found but method not indexed" and nm["knownProjects"] == []
    nc = java_app.context.get_method_context("x.Y", "z")
    assert not nc["found"] and nc["knownProjects"]


def test_stack_trace_context(java_app):
    frames = [
        {"className": f"{O}.OrderController", "methodName": "search", "lineNumber": 22},
        {"className": f"{O}.OrderService$$SpringCGLIB$$0", "methodName": "lambda$list$0", "lineNumber": 5},
        {"className": f"{O}.OrderService", "methodName": "nonexistent", "lineNumber": 1},
        {"className": "java.lang.Thread", "methodName": "run", "lineNumber": 1},
    ]
    r = java_app.context.get_stack_trace_context(frames)
    path = r["executionPath"]
    assert [e["order"] for e in path] == [1, 2, 3, 4]
    assert path[0]["found"] and path[0]["httpEndpoint"] == "POST /search/{id}"
    assert path[1]["found"] and path[1]["className"] == f"{O}.OrderService" and path[1]["methodName"] == "list"
    assert not path[2]["found"] and path[2]["classType"] == "SERVICE"
    assert not path[3]["found"] and path[3]["classType"] is None
    assert len(r["missingContext"]) == 2 and r["projectUrl"].endswith("shop")
    rel = {e["className"] for e in r["relatedDependencies"]}
    assert f"{U}.UserService" in rel and f"{O}.OrderController" not in rel
    assert java_app.context.get_stack_trace_context([])["executionPath"] == []


def test_candidate_names():
    assert candidate_class_names("a.B$C") == ["a.B$C", "a.B"]
    assert candidate_method_names("lambda$doIt$3") == ["lambda$doIt$3", "doIt"]
    assert candidate_method_names("<init>") == ["<init>", None]
    assert candidate_method_names(None) == [None]


def test_class_dependencies(java_app):
    d = java_app.context.get_class_dependencies(f"{O}.OrderController")
    assert d["found"] and d["entryPoint"]
    mp = {x["methodName"]: x["parameterTypes"] for x in d["methodParameterTypes"]}
    assert mp["search"][0]["className"] == f"{O}.OrderRequest" and mp["search"][0]["classType"] == "OTHER"
    assert not java_app.context.get_class_dependencies("x.Y")["found"]
    p = java_app.context.get_class_dependencies("x.Y", "shop")
    assert not p["found"] and p["message"] == "Class not found in project shop"
    assert "list_projects" in java_app.context.get_class_dependencies("x.Y", "nope")["message"]


def test_overview_and_service_api(java_app):
    o = java_app.context.get_project_overview("shop")
    assert o["found"] and o["totalClasses"] == 17 and o["classTypeBreakdown"]["CONTROLLER"] == 2
    ctl = next(e for e in o["entryPoints"] if e["className"] == f"{O}.OrderController")
    assert "GET /" in ctl["httpEndpoints"]
    api = java_app.context.get_service_api("shop")
    assert api["found"] and len(api["controllers"]) == 2
    ep = next(e for e in api["controllers"][0]["endpoints"] if e["methodName"] != "list")
    assert ep["parameters"] and ep["parameters"][0]["position"] >= 0
    assert not java_app.context.get_project_overview("nope")["found"]
    assert not java_app.context.get_service_api("nope")["found"]
