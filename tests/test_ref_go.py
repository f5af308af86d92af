"""One test per case of the reference's Go analyzer tests (12) and
``GoAnalysisResultTest`` (5).

* ``tools/go-analyzer/pkg/analysis/analyzer_test.go`` -- the same
  ``createTestProject`` tree (``:11-160``) analysed by the native C++ Go
  front-end through :func:`dmcp.parsers.goresult.analyze_go`.
* ``src/test/java/co/fanki/domainmcp/analysis/domain/golang/GoAnalysisResultTest.java``
  -- the JSON contract mapped onto :class:`GoAnalysisResult` records.
"""
import json
import os
import textwrap

import pytest

from dmcp.parsers.goresult import GoAnalysisResult, analyze_go

MOD = "github.com/test/myapp"


def write(root, rel, body):
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(textwrap.dedent(body).lstrip("\n"))


@pytest.fixture
def project(tmp_path):
    d = str(tmp_path)
    write(d, "go.mod", f"module {MOD}\n\ngo 1.22\n")
    write(d, "main.go", """
        package main

        import (
        	"fmt"
        	"github.com/test/myapp/internal/handler"
        )

        func main() {
        	h := handler.NewOrderHandler()
        	fmt.Println(h)
        }
        """)
    write(d, "internal/handler/order_handler.go", """
        package handler

        import (
        	"net/http"
        	"github.com/test/myapp/internal/service"
        )

        // OrderHandler handles HTTP requests for orders.
        type OrderHandler struct {
        	svc *service.OrderService
        }

        // NewOrderHandler creates a new OrderHandler.
        func NewOrderHandler() *OrderHandler {
        	return &OrderHandler{}
        }

        // Create handles order creation via HTTP POST.
        func (h *OrderHandler) Create(w http.ResponseWriter, r *http.Request) {
        	panic("not implemented")
        }

        // List returns all orders.
        func (h *OrderHandler) List(w http.ResponseWriter, r *http.Request) {
        	// no panic here
        }
        """)
    write(d, "internal/service/order_service.go", """
        package service

        import "github.com/test/myapp/internal/repository"

        // OrderService contains business logic for orders.
        type OrderService struct {
        	repo *repository.OrderRepository
        }

        // CreateOrder creates a new order.
        func (s *OrderService) CreateOrder(name string) error {
        	return nil
        }

        // FindByID finds an order by its ID.
        func (s *OrderService) FindByID(id string) (string, error) {
        	return "", nil
        }
        """)
    write(d, "internal/repository/order_repository.go", """
        package repository

        // OrderRepository handles persistence for orders.
        type OrderRepository struct {
        	db interface{}
        }

        // Save persists an order to the database.
        func (r *OrderRepository) Save(name string) error {
        	return nil
        }

        // FindByID finds an order by ID.
        func (r *OrderRepository) FindByID(id string) (string, error) {
        	return "", nil
        }
        """)
    write(d, "internal/model/order.go", """
        package model

        // Order represents a business order.
        type Order struct {
        	ID    string
        	Name  string
        	Total float64
        }

        // OrderStatus is the status of an order.
        type OrderStatus string

        const (
        	OrderStatusPending  OrderStatus = "pending"
        	OrderStatusComplete OrderStatus = "complete"
        )
        """)
    write(d, "internal/model/customer.go", """
        package model

        // Customer represents a customer.
        type Customer struct {
        	ID   string
        	Name string
        }
        """)
    write(d, "internal/config/config.go", """
        package config

        // Config holds application configuration.
        type Config struct {
        	Port     int
        	DBHost   string
        	DBPort   int
        }

        // NewConfig creates a default configuration.
        func NewConfig() *Config {
        	return &Config{Port: 8080}
        }
        """)
    return d


def pkg(result, sub):
    p = result.package(MOD + ("/" + sub if sub else ""))
    assert p is not None, sub
    return p


# ============================ analyzer_test.go ================================
def test_analyzer_full_project(project):
    r = analyze_go(project)
    assert r.module == MOD and len(r.packages) >= 5
    assert json.dumps(r._asdict(), default=lambda o: o._asdict() if hasattr(o, "_asdict") else str(o))


def test_analyzer_package_discovery(project):
    paths = {p.path for p in analyze_go(project).packages}
    for sub in ("", "/internal/handler", "/internal/service", "/internal/repository", "/internal/model",
                "/internal/config"):
        assert MOD + sub in paths


def test_analyzer_struct_extraction(project):
    h = pkg(analyze_go(project), "internal/handler")
    assert len(h.structs) == 1
    s = h.structs[0]
    assert s.name == "OrderHandler" and len(s.methods) == 2
    assert [f.name for f in s.fields] == ["svc"]


def test_analyzer_function_extraction(project):
    h = pkg(analyze_go(project), "internal/handler")
    assert len(h.functions) == 1
    fn = h.functions[0]
    assert fn.name == "NewOrderHandler" and fn.receiver == ""
    assert fn.doc == "NewOrderHandler creates a new OrderHandler."


def test_analyzer_panic_detection(project):
    ms = {m.name: m for m in pkg(analyze_go(project), "internal/handler").structs[0].methods}
    assert ms["Create"].has_panic and not ms["List"].has_panic


def test_analyzer_import_extraction(project):
    imports = pkg(analyze_go(project), "internal/handler").imports
    assert MOD + "/internal/service" in imports and "net/http" not in imports


def test_analyzer_entry_point_detection(project):
    r = analyze_go(project)
    assert pkg(r, "").is_entry_point and not pkg(r, "internal/config").is_entry_point


def test_analyzer_class_type_inference(project):
    r = analyze_go(project)
    expected = {"internal/handler": "CONTROLLER", "internal/service": "SERVICE",
                "internal/repository": "REPOSITORY", "internal/model": "ENTITY",
                "internal/config": "CONFIGURATION"}
    assert {k: pkg(r, k).class_type for k in expected} == expected


def test_analyzer_model_package(project):
    m = pkg(analyze_go(project), "internal/model")
    assert len(m.files) == 2 and {s.name for s in m.structs} == {"Order", "Customer"}


def test_analyzer_http_handler_detection(project):
    ms = {m.name: m for m in pkg(analyze_go(project), "internal/handler").structs[0].methods}
    assert ms["Create"].http_method != ""


def test_analyzer_excludes_test_files(project):
    write(project, "internal/service/order_service_test.go", """
        package service

        import "testing"

        func TestCreateOrder(t *testing.T) {
        	// test
        }
        """)
    assert "order_service_test.go" not in pkg(analyze_go(project), "internal/service").files


def test_analyzer_excludes_generated_files(project):
    write(project, "internal/model/order.pb.go", """
        package model

        // Code generated by protoc-gen-go. DO NOT EDIT.
        type OrderProto struct {}
        """)
    m = pkg(analyze_go(project), "internal/model")
    assert "order.pb.go" not in m.files and "OrderProto" not in {s.name for s in m.structs}


# ========================= GoAnalysisResultTest ===============================
FULL = {
    "module": "github.com/user/myapp",
    "packages": [{
        "path": "github.com/user/myapp/internal/handler", "dir": "internal/handler",
        "files": ["order_handler.go"], "imports": ["github.com/user/myapp/internal/service"],
        "structs": [{
            "name": "OrderHandler", "file": "order_handler.go", "line": 15,
            "fields": [{"name": "service", "type": "*service.OrderService",
                        "package": "github.com/user/myapp/internal/service", "isExported": False, "tag": ""}],
            "methods": [{"name": "Create", "file": "order_handler.go", "line": 25, "receiver": "*OrderHandler",
                         "params": [{"name": "c", "type": "*gin.Context", "package": "", "isPointer": True,
                                     "isSlice": False, "isVariadic": False}],
                         "returns": [], "httpMethod": "GET", "httpPath": "", "hasPanic": False,
                         "doc": "Create handles order creation."}],
            "embeddedTypes": [], "implements": ["Handler"]}],
        "interfaces": [{"name": "Handler", "file": "order_handler.go", "line": 10,
                        "methods": [{"name": "Create", "params": [{"name": "c", "type": "*gin.Context",
                                                                   "package": "", "isPointer": True,
                                                                   "isSlice": False, "isVariadic": False}]}],
                        "embeddedInterfaces": []}],
        "functions": [{"name": "NewOrderHandler", "file": "order_handler.go", "line": 20, "receiver": "",
                       "params": [{"name": "svc", "type": "*service.OrderService",
                                   "package": "github.com/user/myapp/internal/service", "isPointer": True,
                                   "isSlice": False, "isVariadic": False}],
                       "returns": ["*OrderHandler"], "httpMethod": "", "httpPath": "", "hasPanic": False,
                       "doc": "NewOrderHandler creates a new handler."}],
        "isEntryPoint": True, "classType": "CONTROLLER"}]}


def test_when_deserializing_given_full_project_json_should_map_all_fields():
    r = GoAnalysisResult.from_json(json.dumps(FULL))
    assert r.module == "github.com/user/myapp" and len(r.packages) == 1
    p = r.packages[0]
    assert (p.path, p.dir, p.files, p.is_entry_point, p.class_type) == (
        "github.com/user/myapp/internal/handler", "internal/handler", ("order_handler.go",), True, "CONTROLLER")
    assert p.imports == ("github.com/user/myapp/internal/service",)
    (s,) = p.structs
    assert (s.name, s.line, len(s.fields), len(s.methods), s.implements) == ("OrderHandler", 15, 1, 1, ("Handler",))
    f = s.fields[0]
    assert (f.name, f.type_name, f.package_path, f.is_exported) == (
        "service", "*service.OrderService", "github.com/user/myapp/internal/service", False)
    m = s.methods[0]
    assert (m.name, m.receiver, m.line, m.http_method, m.doc) == (
        "Create", "*OrderHandler", 25, "GET", "Create handles order creation.")
    (prm,) = m.params
    assert (prm.name, prm.type_name, prm.is_pointer) == ("c", "*gin.Context", True)
    (iface,) = p.interfaces
    assert iface.name == "Handler" and [sig.name for sig in iface.methods] == ["Create"]
    (fn,) = p.functions
    assert (fn.name, fn.receiver, fn.has_panic) == ("NewOrderHandler", "", False)


def test_when_deserializing_given_minimal_json_should_handle_nulls():
    r = GoAnalysisResult.from_json(json.dumps({"module": "example.com/minimal", "packages": [{
        "path": "example.com/minimal", "dir": "", "files": ["main.go"], "imports": [], "structs": [],
        "interfaces": [], "functions": [{"name": "main", "file": "main.go", "line": 5, "receiver": "",
                                         "params": [], "returns": [], "httpMethod": "", "httpPath": "",
                                         "hasPanic": False, "doc": ""}],
        "isEntryPoint": True, "classType": "OTHER"}]}))
    p = r.packages[0]
    assert r.module == "example.com/minimal" and not p.structs and not p.interfaces
    assert [f.name for f in p.functions] == ["main"] and p.is_entry_point
    # null collections map to empty tuples as well
    q = GoAnalysisResult.from_dict({"module": "m", "packages": [{"path": "m", "structs": None,
                                                                  "functions": None}]}).packages[0]
    assert q.structs == () and q.functions == () and q.files == ()


def test_when_deserializing_given_unknown_fields_should_ignore_them():
    r = GoAnalysisResult.from_json('{"module": "example.com/test", "packages": [], '
                                   '"unknownField": "should be ignored", "anotherUnknown": 42}')
    assert r.module == "example.com/test" and r.packages == ()


def test_when_deserializing_given_struct_with_embedded_types_should_parse_them():
    r = GoAnalysisResult.from_dict({"module": "example.com/embedded", "packages": [{
        "path": "example.com/embedded", "dir": "", "files": ["model.go"], "imports": [],
        "structs": [{"name": "Admin", "file": "model.go", "line": 10, "fields": [], "methods": [],
                     "embeddedTypes": ["User", "sync.Mutex"], "implements": []}],
        "interfaces": [], "functions": [], "isEntryPoint": False, "classType": "ENTITY"}]})
    s = r.packages[0].structs[0]
    assert s.name == "Admin" and set(s.embedded_types) == {"User", "sync.Mutex"} and len(s.embedded_types) == 2


def test_when_deserializing_given_function_with_panic_should_set_flag():
    r = GoAnalysisResult.from_dict({"module": "example.com/panic", "packages": [{
        "path": "example.com/panic", "dir": "", "files": ["validator.go"], "imports": [], "structs": [],
        "interfaces": [], "functions": [{"name": "MustParse", "file": "validator.go", "line": 8, "receiver": "",
                                         "params": [{"name": "input", "type": "string", "package": "",
                                                     "isPointer": False, "isSlice": False, "isVariadic": False}],
                                         "returns": ["Config"], "httpMethod": "", "httpPath": "",
                                         "hasPanic": True, "doc": "MustParse panics if input is invalid."}],
        "isEntryPoint": False, "classType": "UTILITY"}]})
    fn = r.packages[0].functions[0]
    assert fn.name == "MustParse" and fn.has_panic and len(fn.params) == 1 and not fn.params[0].is_pointer


def test_native_analyzer_output_maps_onto_the_contract(project):
    """The native document round-trips through the records (every key known)."""
    raw = json.loads(__import__("dmcp.parsers.base", fromlist=["native"]).native().analyze_go(project, 0))
    r = GoAnalysisResult.from_dict(raw)
    assert r.module == raw["module"] and len(r.packages) == len(raw["packages"])
