"""One test per case of the reference's ``GraphQueryTest`` (24) and
``GraphQueryServiceTest`` (22).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/application/GraphQueryTest.java``
and ``GraphQueryServiceTest.java``.  The reference mocks ``GraphService`` with
Mockito; here a real :class:`GraphCache` holds the same hand-built graph
(``buildTestGraph``, ``GraphQueryServiceTest.java:40-95``).  Every
``DomainException`` assertion also checks the error code.
"""
import pytest

from dmcp.graph.cache import GraphCache
from dmcp.graph.project_graph import MethodInfo, ProjectGraph
from dmcp.query.dsl import GraphQuery, GraphQueryService, Token, TokenType
from dmcp.utils.errors import DomainError


def parse_error(q, code="INVALID_QUERY"):
    with pytest.raises(DomainError) as ei:
        GraphQuery.parse(q)
    assert ei.value.error_code == code


# =========================== GraphQueryTest ===================================
def test_when_parsing_given_project_and_target_should_tokenize():
    q = GraphQuery.parse("stadium-service:endpoints")
    assert q.project == "stadium-service" and q.first_navigation() == "endpoints"
    assert len(q.tokens) == 1 and q.tokens[0].type is TokenType.NAVIGATE


def test_when_parsing_given_multiple_navigations_should_tokenize_all():
    q = GraphQuery.parse("proj:UserService:methods")
    assert q.project == "proj"
    assert [t.value for t in q.navigations()] == ["UserService", "methods"]


def test_when_parsing_given_class_with_method_navigation_should_capture_all():
    assert GraphQuery.parse("proj:UserService:method:createUser").navigations_from(0) == [
        "UserService", "method", "createUser"]


def test_when_parsing_given_include_token_should_recognize():
    q = GraphQuery.parse("proj:endpoints:+logic")
    assert len(q.navigations()) == 1 and q.first_navigation() == "endpoints"
    assert [t.value for t in q.includes()] == ["logic"] and q.has_include("logic")


def test_when_parsing_given_multiple_includes_should_capture_all():
    q = GraphQuery.parse("proj:classes:+dependencies:+dependents")
    assert len(q.navigations()) == 1 and len(q.includes()) == 2
    assert q.has_include("dependencies") and q.has_include("dependents")


def test_when_parsing_given_include_mixed_with_navigation_should_separate():
    q = GraphQuery.parse("proj:UserService:methods:+logic")
    assert [t.value for t in q.navigations()] == ["UserService", "methods"]
    assert len(q.includes()) == 1 and q.has_include("logic")


def test_has_include_given_case_insensitive_should_match():
    q = GraphQuery.parse("proj:endpoints:+Logic")
    assert q.has_include("logic") and q.has_include("LOGIC")


def test_when_parsing_given_check_token_should_recognize():
    q = GraphQuery.parse("proj:UserService:?createUser")
    assert len(q.navigations()) == 1 and q.first_navigation() == "UserService"
    assert q.has_check() and q.check_value() == "createUser"


def test_when_parsing_given_no_check_should_not_have_check():
    q = GraphQuery.parse("proj:UserService:methods")
    assert not q.has_check() and q.check_value() is None


def test_when_parsing_given_check_and_include_should_capture_both():
    q = GraphQuery.parse("proj:UserService:+logic:?createUser")
    assert q.has_include("logic") and q.has_check() and q.check_value() == "createUser"


def test_navigations_from_given_valid_index_should_return_sublist():
    assert GraphQuery.parse("proj:UserService:method:createUser").navigations_from(1) == ["method", "createUser"]


def test_navigations_from_given_out_of_bounds_should_return_empty():
    assert GraphQuery.parse("proj:endpoints").navigations_from(1) == []


def test_first_navigation_given_entrypoints_should_return():
    assert GraphQuery.parse("proj:entrypoints").first_navigation() == "entrypoints"


def test_first_navigation_given_classes_should_return():
    assert GraphQuery.parse("proj:classes").first_navigation() == "classes"


def test_token_to_string_should_format_with_prefix():
    assert str(Token(TokenType.NAVIGATE, "foo")) == "foo"
    assert str(Token(TokenType.INCLUDE, "logic")) == "+logic"
    assert str(Token(TokenType.CHECK, "create")) == "?create"


def test_raw_should_return_original_query():
    assert GraphQuery.parse("proj:endpoints:+logic").raw == "proj:endpoints:+logic"


def test_when_parsing_given_null_query_should_throw():
    parse_error(None)


def test_when_parsing_given_blank_query_should_throw():
    parse_error("   ")


def test_when_parsing_given_only_project_should_throw():
    parse_error("stadium-service")


def test_when_parsing_given_empty_project_should_throw():
    parse_error(":endpoints")


def test_when_parsing_given_empty_include_value_should_throw():
    parse_error("proj:endpoints:+")


def test_when_parsing_given_empty_check_value_should_throw():
    parse_error("proj:UserService:?")


def test_when_parsing_given_include_as_first_token_should_throw():
    parse_error("proj:+logic")


def test_when_parsing_given_check_as_first_token_should_throw():
    parse_error("proj:?foo")


# ======================== GraphQueryServiceTest ===============================
def build_test_graph() -> ProjectGraph:
    g = ProjectGraph()
    for n in ("UserController", "UserService", "UserRepository", "UserDto"):
        g.add_node(f"co.fanki.{n}", f"src/{n}.java")
    g.add_dependency("co.fanki.UserController", "co.fanki.UserService")
    g.add_dependency("co.fanki.UserService", "co.fanki.UserRepository")
    g.mark_as_entry_point("co.fanki.UserController")
    g.set_node_info("co.fanki.UserController", "CONTROLLER", "Handles user HTTP requests")
    g.set_node_info("co.fanki.UserService", "SERVICE", "User business logic")
    g.set_node_info("co.fanki.UserRepository", "REPOSITORY", "User data access")
    g.set_node_info("co.fanki.UserDto", "DTO", "User data transfer object")
    g.add_method_info("co.fanki.UserController", MethodInfo(
        "getUsers", "Lists all users", ("Query users", "Map to DTOs"), (), "GET", "/api/users", 25))
    g.add_method_info("co.fanki.UserController", MethodInfo(
        "createUser", "Creates a new user", ("Validate input", "Save user"), ("ValidationException",),
        "POST", "/api/users", 40))
    g.add_method_info("co.fanki.UserService", MethodInfo(
        "findAll", "Finds all users", ("Delegate to repository",), (), None, None, 15))
    g.add_method_info("co.fanki.UserService", MethodInfo(
        "create", "Creates a user", ("Validate", "Persist"), ("DuplicateUserException",), None, None, 30))
    return g


@pytest.fixture
def svc():
    cache = GraphCache()
    cache.put("pid-1", "my-project", build_test_graph())
    return GraphQueryService(cache)


def run(svc, q):
    return svc.execute(GraphQuery.parse(q))


def by_class(result, name):
    return next(m for m in result.results if m["className"] == name)


def test_when_executing_given_unknown_project_should_throw(svc):
    with pytest.raises(DomainError) as ei:
        run(svc, "unknown:endpoints")
    assert ei.value.error_code == "PROJECT_NOT_FOUND"


def test_when_querying_endpoints_should_return_all_http_methods(svc):
    r = run(svc, "my-project:endpoints")
    assert (r.result_type, r.project, r.count) == ("endpoints", "my-project", 2)
    assert r.results[0]["httpMethod"] is not None and r.results[0]["httpPath"] is not None


def test_when_querying_endpoints_given_include_logic_should_include_it(svc):
    r = run(svc, "my-project:endpoints:+logic")
    assert r.count == 2 and "businessLogic" in r.results[0]


def test_when_querying_endpoints_given_no_include_should_omit_logic(svc):
    assert "businessLogic" not in run(svc, "my-project:endpoints").results[0]


def test_when_querying_classes_should_return_all_nodes(svc):
    r = run(svc, "my-project:classes")
    assert (r.result_type, r.count) == ("classes", 4)


def test_when_querying_classes_given_include_dependencies_should_include(svc):
    ctrl = by_class(run(svc, "my-project:classes:+dependencies"), "co.fanki.UserController")
    assert "co.fanki.UserService" in ctrl["dependencies"]


def test_when_querying_classes_given_include_methods_should_include(svc):
    assert "methods" in by_class(run(svc, "my-project:classes:+methods"), "co.fanki.UserController")


def test_when_querying_entrypoints_should_return_only_entry_points(svc):
    r = run(svc, "my-project:entrypoints")
    assert (r.result_type, r.count) == ("entrypoints", 1)
    assert r.results[0]["className"] == "co.fanki.UserController"


def test_when_querying_entrypoints_given_include_logic_should_include(svc):
    assert "businessLogic" in run(svc, "my-project:entrypoints:+logic").results[0]["endpoints"][0]


def test_when_querying_vertex_given_simple_name_should_resolve(svc):
    r = run(svc, "my-project:UserService")
    assert (r.result_type, r.count) == ("class", 1)
    assert r.results[0]["className"] == "co.fanki.UserService"


def test_when_querying_vertex_given_full_name_should_resolve(svc):
    assert run(svc, "my-project:co.fanki.UserService").results[0]["className"] == "co.fanki.UserService"


def test_when_querying_vertex_given_unknown_class_should_throw(svc):
    with pytest.raises(DomainError) as ei:
        run(svc, "my-project:Unknown")
    assert ei.value.error_code == "CLASS_NOT_FOUND"


def test_when_querying_vertex_methods_should_return_all(svc):
    r = run(svc, "my-project:UserService:methods")
    assert (r.result_type, r.count) == ("methods", 2)


def test_when_querying_vertex_methods_given_include_logic_should_include(svc):
    assert "businessLogic" in run(svc, "my-project:UserService:methods:+logic").results[0]


def test_when_querying_vertex_dependencies_should_return_outgoing(svc):
    r = run(svc, "my-project:UserController:dependencies")
    assert (r.result_type, r.count) == ("dependencies", 1)
    assert r.results[0]["className"] == "co.fanki.UserService"


def test_when_querying_vertex_dependents_should_return_incoming(svc):
    r = run(svc, "my-project:UserService:dependents")
    assert (r.result_type, r.count) == ("dependents", 1)
    assert r.results[0]["className"] == "co.fanki.UserController"


def test_when_querying_single_method_should_return_detail(svc):
    r = run(svc, "my-project:UserController:method:createUser")
    assert (r.result_type, r.count) == ("method", 1)
    assert r.results[0]["methodName"] == "createUser" and r.results[0]["httpMethod"] == "POST"


def test_when_querying_single_method_given_unknown_should_throw(svc):
    with pytest.raises(DomainError) as ei:
        run(svc, "my-project:UserController:method:unknown")
    assert ei.value.error_code == "METHOD_NOT_FOUND"


def test_when_querying_vertex_overview_should_include_method_summaries(svc):
    info = run(svc, "my-project:UserController").results[0]
    assert len(info["methods"]) == 2


def test_when_checking_given_existing_method_should_return_true(svc):
    r = run(svc, "my-project:UserController:?createUser")
    assert (r.result_type, r.count) == ("check", 1)
    assert r.results[0]["exists"] is True and r.results[0]["methodName"] == "createUser"


def test_when_checking_given_non_existing_method_should_return_false(svc):
    r = run(svc, "my-project:UserController:?deleteUser")
    assert r.result_type == "check" and r.results[0]["exists"] is False


def test_when_checking_given_existing_method_should_include_details(svc):
    item = run(svc, "my-project:UserController:?getUsers").results[0]
    assert item["exists"] is True and item["methodName"] == "getUsers"
    assert item["description"] == "Lists all users" and item["httpEndpoint"] == "GET /api/users"
