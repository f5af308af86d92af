"""One test per case of the reference's ``CodeContextServiceTest`` (20 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/application/CodeContextServiceTest.java``.
The reference stubs four repositories and ``GraphService`` with EasyMock;
here the same rows live in a real SQLite store and the same hand-built graphs
in a real :class:`GraphCache`, so each case also exercises the SQL.
"""
import pytest

from dmcp.graph.cache import GraphCache
from dmcp.graph.project_graph import ProjectGraph
from dmcp.models.domain import ClassType, Project, RepositoryUrl, SourceClass, SourceMethod
from dmcp.query.context import ContextService
from dmcp.store.db import Database
from dmcp.store.repositories import Repositories


class World:
    def __init__(self, path):
        self.db = Database(path)
        self.repos = Repositories(self.db)
        self.cache = GraphCache()
        self.svc = ContextService(self.repos, self.cache)

    def project(self, name, url, description=None):
        p = Project.create(name, RepositoryUrl.of(url), "main")
        if description:
            p.update_description(description)
        self.repos.projects.save(p)
        return p

    def cls(self, project, fqcn, ct, desc, sf):
        sc = SourceClass.create(project.id, fqcn, ct, desc, sf, "abc123")
        self.repos.classes.save(sc)
        return sc

    def method(self, sc, name, desc, logic, exc, verb, path, line):
        m = SourceMethod.create(sc.id, name, desc, logic, exc, verb, path, line)
        self.repos.methods.save(m)
        return m

    def graph(self, project, g):
        self.cache.put(project.id, project.name, g)
        return g


@pytest.fixture
def w(tmp_path):
    world = World(str(tmp_path / "ctx.db"))
    yield world
    world.db.close()


def nodes(*pairs):
    g = ProjectGraph()
    for ident, sf in pairs:
        g.add_node(ident, sf)
    return g


def test_when_getting_class_context_given_existing_class_should_return_full_context(w):
    p = w.project("user-service", "https://github.com/fanki/user-svc.git")
    sc = w.cls(p, "co.fanki.user.UserService", ClassType.SERVICE, "User management", "UserService.java")
    w.method(sc, "findById", "Finds user by ID", ["Query DB"], [], None, None, 30)
    w.method(sc, "createUser", "Creates a new user", ["Validate", "Save"], ["DuplicateEmailException"],
             "POST", "/api/users", 55)
    g = nodes(("co.fanki.user.UserService", "UserService.java"), ("co.fanki.user.UserRepository", "UserRepo.java"),
              ("co.fanki.user.UserController", "UserCtrl.java"))
    g.add_dependency("co.fanki.user.UserService", "co.fanki.user.UserRepository")
    g.add_dependency("co.fanki.user.UserController", "co.fanki.user.UserService")
    g.mark_as_entry_point("co.fanki.user.UserController")
    w.graph(p, g)
    c = w.svc.get_class_context("co.fanki.user.UserService")
    assert c["found"] and c["className"] == "co.fanki.user.UserService" and c["classType"] == "SERVICE"
    assert [m["name"] for m in c["methods"]] == ["findById", "createUser"]
    gi = c["graphInfo"]
    assert gi["dependencies"] == ["co.fanki.user.UserRepository"]
    assert gi["dependents"] == ["co.fanki.user.UserController"] and gi["entryPoint"] is False


def test_when_getting_class_context_given_unknown_class_should_return_not_found(w):
    c = w.svc.get_class_context("com.unknown.Foo")
    assert not c["found"] and c["className"] == "com.unknown.Foo" and c["message"]


def test_when_getting_method_context_given_existing_method_should_return_context(w):
    p = w.project("order-service", "https://github.com/fanki/orders.git")
    sc = w.cls(p, "co.fanki.order.OrderService", ClassType.SERVICE, "Order processing", "OrderService.java")
    w.method(sc, "placeOrder", "Places a new order for a customer",
             ["Validate items", "Calculate total", "Save order"], ["InsufficientStockException"],
             "POST", "/api/orders", 85)
    g = nodes(("co.fanki.order.OrderService", "OrderService.java"), ("co.fanki.order.OrderDto", "OrderDto.java"))
    g.add_method_parameter("co.fanki.order.OrderService", "placeOrder", 0, "co.fanki.order.OrderDto")
    w.graph(p, g)
    c = w.svc.get_method_context("co.fanki.order.OrderService", "placeOrder")
    assert c["found"] and c["className"] == "co.fanki.order.OrderService" and c["methodName"] == "placeOrder"
    assert c["httpEndpoint"] == "POST /api/orders" and len(c["businessLogic"]) == 3
    assert c["parameterTypes"] == [{"position": 0, "typeName": "co.fanki.order.OrderDto"}]


def test_when_getting_method_context_given_unknown_class_should_return_not_found(w):
    c = w.svc.get_method_context("com.unknown.Foo", "bar")
    assert not c["found"] and c["message"]


def test_when_getting_method_context_given_class_found_but_method_missing_should_return_partial_context(w):
    p = w.project("order-service", "https://github.com/fanki/orders.git")
    w.cls(p, "co.fanki.order.OrderService", ClassType.SERVICE, "Order processing", "OrderService.java")
    c = w.svc.get_method_context("co.fanki.order.OrderService", "unknownMethod")
    assert not c["found"] and c["message"] == "Class found but method not indexed"


def test_when_getting_stack_trace_context_given_mixed_frames_should_return_found_and_missing(w):
    p = w.project("payment-service", "https://github.com/fanki/payment.git")
    sc = w.cls(p, "co.fanki.payment.PaymentService", ClassType.SERVICE, "Payment processing",
               "PaymentService.java")
    w.method(sc, "processPayment", "Processes a payment", ["Validate", "Charge", "Save"],
             ["PaymentDeclinedException"], None, None, 42)
    ctx = w.svc.get_stack_trace_context([
        {"className": "co.fanki.payment.PaymentService", "methodName": "processPayment", "lineNumber": 42},
        {"className": "org.springframework.web.servlet.DispatcherServlet", "methodName": "doDispatch",
         "lineNumber": 1067}])
    path = ctx["executionPath"]
    assert len(path) == 2 and len(ctx["missingContext"]) == 1
    assert path[0]["found"] and path[0]["className"] == "co.fanki.payment.PaymentService"
    assert path[0]["methodName"] == "processPayment" and path[0]["classType"] == "SERVICE"
    assert len(path[0]["businessLogic"]) == 3
    assert not path[1]["found"] and path[1]["className"] == "org.springframework.web.servlet.DispatcherServlet"
    assert ctx["projectUrl"] == "https://github.com/fanki/payment.git"


def test_when_getting_stack_trace_context_given_graph_with_neighbors_should_include_related_dependencies(w):
    p = w.project("order-service", "https://github.com/fanki/orders.git")
    ctrl = w.cls(p, "co.fanki.order.OrderController", ClassType.CONTROLLER, "Order REST controller",
                 "OrderController.java")
    w.method(ctrl, "createOrder", "Creates a new order", ["Validates input", "Delegates to service"], [],
             "POST", "/api/orders", 30)
    svc = w.cls(p, "co.fanki.order.OrderService", ClassType.SERVICE, "Order processing service", "OrderService.java")
    w.method(svc, "processOrder", "Processes the order", ["Calculate total", "Save"], [], None, None, 50)
    g = nodes(("co.fanki.order.OrderController", "OrderController.java"),
              ("co.fanki.order.OrderService", "OrderService.java"))
    g.add_dependency("co.fanki.order.OrderController", "co.fanki.order.OrderService")
    w.graph(p, g)
    ctx = w.svc.get_stack_trace_context([{"className": "co.fanki.order.OrderController",
                                          "methodName": "createOrder", "lineNumber": 30}])
    assert len(ctx["executionPath"]) == 1 and not ctx["missingContext"]
    n = ctx["relatedDependencies"][0]
    assert (n["className"], n["methodName"], n["found"]) == ("co.fanki.order.OrderService", "processOrder", True)


def test_when_getting_stack_trace_context_given_all_frames_missing_should_return_empty_neighbors(w):
    ctx = w.svc.get_stack_trace_context([{"className": "com.unknown.FooService", "methodName": "doStuff",
                                          "lineNumber": 10}])
    assert len(ctx["executionPath"]) == 1 and not ctx["executionPath"][0]["found"]
    assert len(ctx["missingContext"]) == 1 and ctx["relatedDependencies"] == []


def test_when_getting_class_dependencies_given_existing_class_should_return_full_graph(w):
    p = w.project("order-service", "https://github.com/fanki/orders.git")
    w.cls(p, "co.fanki.order.OrderService", ClassType.SERVICE, "Order processing", "OrderService.java")
    w.cls(p, "co.fanki.order.OrderRepository", ClassType.REPOSITORY, "Order persistence", "OrderRepository.java")
    w.cls(p, "co.fanki.order.OrderController", ClassType.CONTROLLER, "Order REST API", "OrderController.java")
    g = nodes(("co.fanki.order.OrderService", "OrderService.java"),
              ("co.fanki.order.OrderRepository", "OrderRepository.java"),
              ("co.fanki.order.OrderController", "OrderController.java"), ("co.fanki.order.OrderDto", "OrderDto.java"))
    g.add_dependency("co.fanki.order.OrderService", "co.fanki.order.OrderRepository")
    g.add_dependency("co.fanki.order.OrderController", "co.fanki.order.OrderService")
    g.add_method_parameter("co.fanki.order.OrderService", "placeOrder", 0, "co.fanki.order.OrderDto")
    g.mark_as_entry_point("co.fanki.order.OrderController")
    w.graph(p, g)
    r = w.svc.get_class_dependencies("co.fanki.order.OrderService")
    assert r["found"] and r["entryPoint"] is False
    assert [(d["className"], d["classType"]) for d in r["dependencies"]] == [
        ("co.fanki.order.OrderRepository", "REPOSITORY")]
    assert [(d["className"], d["classType"]) for d in r["dependents"]] == [
        ("co.fanki.order.OrderController", "CONTROLLER")]
    assert [m["methodName"] for m in r["methodParameterTypes"]] == ["placeOrder"]


def test_when_getting_class_dependencies_given_unknown_class_should_return_not_found(w):
    r = w.svc.get_class_dependencies("com.unknown.Foo")
    assert not r["found"] and r["message"]


def test_when_getting_project_overview_given_existing_project_should_return_overview(w):
    p = w.project("order-service", "https://github.com/fanki/orders.git", "Order management system")
    ctrl = w.cls(p, "co.fanki.order.OrderController", ClassType.CONTROLLER, "Order REST controller",
                 "OrderController.java")
    w.cls(p, "co.fanki.order.OrderService", ClassType.SERVICE, "Order processing", "OrderService.java")
    w.method(ctrl, "createOrder", "Creates order", [], [], "POST", "/api/orders", 30)
    g = nodes(("co.fanki.order.OrderController", "OrderController.java"),
              ("co.fanki.order.OrderService", "OrderService.java"))
    g.mark_as_entry_point("co.fanki.order.OrderController")
    w.graph(p, g)
    o = w.svc.get_project_overview("order-service")
    assert o["found"] and o["projectName"] == "order-service"
    assert o["totalClasses"] == 2 and o["totalEntryPoints"] == 1
    assert {"CONTROLLER", "SERVICE"} <= set(o["classTypeBreakdown"])
    assert o["entryPoints"][0]["className"] == "co.fanki.order.OrderController"
    assert o["entryPoints"][0]["httpEndpoints"] == ["POST /api/orders"]


def test_when_getting_project_overview_given_unknown_project_should_return_not_found(w):
    o = w.svc.get_project_overview("unknown-project")
    assert not o["found"] and o["message"]


def test_when_getting_service_api_given_existing_project_should_return_endpoints_with_params(w):
    p = w.project("order-service", "https://github.com/fanki/orders.git", "Order management system")
    ctrl = w.cls(p, "co.fanki.order.OrderController", ClassType.CONTROLLER, "Order REST controller",
                 "OrderController.java")
    w.cls(p, "co.fanki.order.OrderDto", ClassType.DTO, "Order data transfer object", "OrderDto.java")
    w.method(ctrl, "createOrder", "Creates a new order", ["Validate input", "Delegate to service"],
             ["InvalidOrderException"], "POST", "/api/orders", 30)
    w.method(ctrl, "getOrder", "Gets an order by ID", ["Query DB"], ["OrderNotFoundException"],
             "GET", "/api/orders/{id}", 50)
    g = nodes(("co.fanki.order.OrderController", "OrderController.java"), ("co.fanki.order.OrderDto", "OrderDto.java"))
    g.mark_as_entry_point("co.fanki.order.OrderController")
    g.add_method_parameter("co.fanki.order.OrderController", "createOrder", 0, "co.fanki.order.OrderDto")
    w.graph(p, g)
    r = w.svc.get_service_api("order-service")
    assert r["found"] and r["projectName"] == "order-service" and len(r["controllers"]) == 1
    ctrl_out = r["controllers"][0]
    assert ctrl_out["className"] == "co.fanki.order.OrderController" and len(ctrl_out["endpoints"]) == 2
    post = next(e for e in ctrl_out["endpoints"] if e["httpMethod"] == "POST")
    assert (post["methodName"], post["httpPath"]) == ("createOrder", "/api/orders")
    assert [(x["className"], x["classType"]) for x in post["parameters"]] == [("co.fanki.order.OrderDto", "DTO")]
    get = next(e for e in ctrl_out["endpoints"] if e["httpMethod"] == "GET")
    assert get["methodName"] == "getOrder" and get["parameters"] == []


def test_when_getting_service_api_given_unknown_project_should_return_not_found(w):
    r = w.svc.get_service_api("unknown-service")
    assert not r["found"] and r["message"]


def test_when_getting_service_api_given_project_with_no_graph_should_return_not_found(w):
    w.project("orphan-service", "https://github.com/fanki/orphan.git")
    r = w.svc.get_service_api("orphan-service")
    assert not r["found"] and r["message"] and r["controllers"] == []


def search_world(w):
    p = w.project("my-project", "https://github.com/example/my-project.git")
    g = nodes(("com.example.OrderService", "OrderService.java"),
              ("com.example.OrderController", "OrderController.java"), ("com.example.UserService", "UserService.java"))
    g.mark_as_entry_point("com.example.OrderController")
    w.cls(p, "com.example.OrderService", ClassType.SERVICE, "Order processing", "OrderService.java")
    w.cls(p, "com.example.OrderController", ClassType.CONTROLLER, "Order REST API", "OrderController.java")
    w.graph(p, g)
    return p


def test_when_searching_project_given_existing_project_and_matching_query_should_return_matches(w):
    search_world(w)
    r = w.svc.search_project("my-project", "Order")
    assert r["found"] and r["projectName"] == "my-project" and r["query"] == "Order"
    assert len(r["matches"]) == 2 and r["totalClassesInProject"] == 3
    by = {m["className"]: m for m in r["matches"]}
    assert by["com.example.OrderController"]["entryPoint"] is True
    assert by["com.example.OrderService"]["classType"] == "SERVICE"


def test_when_searching_project_given_unknown_project_should_return_not_found(w):
    r = w.svc.search_project("unknown", "Order")
    assert not r["found"] and r["message"]


def test_when_searching_project_given_no_matching_query_should_return_empty_matches(w):
    p = w.project("my-project", "https://github.com/example/my-project.git")
    w.graph(p, nodes(("com.example.OrderService", "OrderService.java")))
    r = w.svc.search_project("my-project", "ZzzNotExist")
    assert r["found"] and r["matches"] == [] and r["totalClassesInProject"] == 1


def test_when_getting_class_context_given_project_name_should_scope_to_project(w):
    p = w.project("my-project", "https://github.com/fanki/orders.git")
    sc = w.cls(p, "com.example.OrderService", ClassType.SERVICE, "Order processing", "OrderService.java")
    w.method(sc, "findById", "Finds order by ID", ["Query DB"], [], None, None, 30)
    g = nodes(("com.example.OrderService", "OrderService.java"), ("com.example.OrderRepository", "OrderRepository.java"))
    g.add_dependency("com.example.OrderService", "com.example.OrderRepository")
    w.graph(p, g)
    # a same-named class in another project must not be picked
    other = w.project("other", "https://github.com/fanki/other.git")
    w.cls(other, "com.example.OrderService", ClassType.UTILITY, "Other", "OrderService.java")
    c = w.svc.get_class_context("com.example.OrderService", "my-project")
    assert c["found"] and c["className"] == "com.example.OrderService" and c["classType"] == "SERVICE"
    assert len(c["methods"]) == 1 and c["graphInfo"]["dependencies"] == ["com.example.OrderRepository"]


def test_when_getting_class_context_given_project_name_and_class_not_in_graph_should_return_not_found(w):
    p = w.project("my-project", "https://github.com/example/my-project.git")
    w.graph(p, nodes(("com.example.UserService", "UserService.java")))
    c = w.svc.get_class_context("com.example.OrderService", "my-project")
    assert not c["found"] and c["className"] == "com.example.OrderService"
