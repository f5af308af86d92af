"""Go front-end (tools/go-analyzer analyzer_test.go + GoAnalysisResultTest in
the reference): package discovery, structs / interfaces / functions,
receivers, panic detection, internal imports, entry points, class types,
exclusions, the go-analyzer JSON contract, and (addition) route binding."""
import json
import os
import textwrap

import pytest

from dmcp.parsers.base import GoSourceParser, native


def write(root, rel, body):
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(textwrap.dedent(body).lstrip("\n"))


@pytest.fixture
def project(tmp_path):
    r = str(tmp_path)
    write(r, "go.mod", "module example.com/shop\n\ngo 1.22\n")
    write(r, "main.go", """
        package main

        import (
            "fmt"
            "example.com/shop/internal/api"
        )

        func main() {
            fmt.Println(api.NewInvoiceAPI())
        }
        """)
    write(r, "internal/api/invoice_api.go", """
        package api

        import (
            "net/http"
            "example.com/shop/internal/billing"
        )

        // InvoiceAPI serves invoices over HTTP.
        type InvoiceAPI struct {
            svc *billing.InvoiceService
        }

        // NewInvoiceAPI builds the API.
        func NewInvoiceAPI() *InvoiceAPI { return &InvoiceAPI{} }

        // Issue issues an invoice.
        func (a *InvoiceAPI) Issue(w http.ResponseWriter, r *http.Request) {
            panic("todo")
        }

        // Show renders one invoice.
        func (a *InvoiceAPI) Show(w http.ResponseWriter, r *http.Request) {
        }

        func Routes(mux *http.ServeMux, a *InvoiceAPI) {
            mux.HandleFunc("POST /invoices", a.Issue)
            mux.HandleFunc("GET /invoices/{id}", a.Show)
        }
        """)
    write(r, "internal/billing/invoice_service.go", """
        package billing

        import "example.com/shop/internal/store"

        // InvoiceService holds billing rules.
        type InvoiceService struct {
            repo *store.InvoiceStore
            Logger
        }

        type Logger interface {
            Log(msg string)
        }

        // Issue creates an invoice.
        func (s *InvoiceService) Issue(customer string, cents int64) error { return nil }

        func (s InvoiceService) Total(ids []string, extra ...int) (int64, error) { return 0, nil }
        """)
    write(r, "internal/store/invoice_store.go", """
        package store

        type InvoiceStore struct{ db interface{} }

        func (s *InvoiceStore) Save(id string) error { return nil }
        """)
    write(r, "internal/store/invoice_store_test.go", "package store\n\nfunc TestX() {}\n")
    write(r, "internal/store/zz_generated.go", "package store\n\ntype Generated struct{}\n")
    write(r, "internal/model/invoice.go", "package model\n\ntype Invoice struct {\n    ID string `json:\"id\"`\n}\n")
    write(r, "internal/config/config.go", "package config\n\ntype Config struct{ Port int }\n")
    write(r, "vendor/x/x.go", "package x\n\ntype V struct{}\n")
    write(r, "testdata/t.go", "package t\n")
    write(r, ".hidden/h.go", "package h\n")
    return r


def test_packages_and_identifiers(project):
    p = GoSourceParser()
    g = p.parse(project)
    assert set(g.identifiers()) == {"example.com/shop", "example.com/shop/internal/api",
                                    "example.com/shop/internal/billing", "example.com/shop/internal/store",
                                    "example.com/shop/internal/model", "example.com/shop/internal/config"}
    assert g.dependencies("example.com/shop") == ("example.com/shop/internal/api",)
    assert g.dependencies("example.com/shop/internal/api") == ("example.com/shop/internal/billing",)
    assert g.is_entry_point("example.com/shop") and g.is_entry_point("example.com/shop/internal/api")
    assert not g.is_entry_point("example.com/shop/internal/billing")
    assert p.project.module == "example.com/shop"


def test_class_types_and_methods(project):
    p = GoSourceParser()
    proj = p.scan(project)
    u = proj.units
    assert u["example.com/shop/internal/api"].class_type.value == "CONTROLLER"
    assert u["example.com/shop/internal/billing"].class_type.value == "OTHER"
    assert u["example.com/shop/internal/store"].class_type.value == "REPOSITORY"
    assert u["example.com/shop/internal/model"].class_type.value == "ENTITY"
    assert u["example.com/shop/internal/config"].class_type.value == "CONFIGURATION"
    api = {m.method_name: m for m in u["example.com/shop/internal/api"].methods}
    assert set(api) == {"NewInvoiceAPI", "Routes", "InvoiceAPI.Issue", "InvoiceAPI.Show"}
    assert api["InvoiceAPI.Issue"].exceptions == ("panic",) and api["InvoiceAPI.Show"].exceptions == ()
    # route binding (addition): Go 1.22 mux patterns give verb + path
    assert (api["InvoiceAPI.Issue"].http_method, api["InvoiceAPI.Issue"].http_path) == ("POST", "/invoices")
    assert (api["InvoiceAPI.Show"].http_method, api["InvoiceAPI.Show"].http_path) == ("GET", "/invoices/{id}")
    assert api["NewInvoiceAPI"].http_method is None
    billing = {m.method_name for m in u["example.com/shop/internal/billing"].methods}
    assert billing == {"InvoiceService.Issue", "InvoiceService.Total"}


def test_analyze_go_contract(project):
    doc = json.loads(native().analyze_go(project, 2))
    assert doc["module"] == "example.com/shop"
    pk = {p["path"]: p for p in doc["packages"]}
    assert "example.com/shop/internal/store" in pk
    store = pk["example.com/shop/internal/store"]
    assert store["files"] == ["invoice_store.go"]  # _test.go and *_generated.go excluded
    assert [s["name"] for s in store["structs"]] == ["InvoiceStore"]
    billing = pk["example.com/shop/internal/billing"]
    svc = billing["structs"][0]
    assert svc["name"] == "InvoiceService" and svc["embeddedTypes"] == ["Logger"]
    # an embedded type is also listed as a nameless field (extractFields parity)
    assert [f["name"] for f in svc["fields"]] == ["repo", ""]
    assert billing["interfaces"][0]["name"] == "Logger"
    total = next(m for m in svc["methods"] if m["name"] == "Total")
    assert total["receiver"] == "InvoiceService"
    assert [p["name"] for p in total["params"]] == ["ids", "extra"] and total["params"][1]["isVariadic"]
    assert total["returns"] == ["int64", "error"]
    issue = next(m for m in pk["example.com/shop/internal/api"]["structs"][0]["methods"] if m["name"] == "Issue")
    assert issue["hasPanic"] and issue["httpMethod"] == "POST" and issue["doc"].startswith("Issue issues")
    assert billing["imports"] == ["example.com/shop/internal/store"]
    model = pk["example.com/shop/internal/model"]["structs"][0]["fields"][0]
    assert model["tag"] == '`json:"id"`' or model["tag"] == 'json:"id"'
    assert not any(p.startswith("example.com/shop/vendor") or "testdata" in p for p in pk)


def test_gin_groups_and_ambiguous_names(tmp_path):
    r = str(tmp_path)
    write(r, "go.mod", "module m\n")
    write(r, "handlers/users.go", """
        package handlers
        import "github.com/gin-gonic/gin"
        type UserHandler struct{}
        func (h *UserHandler) List(c *gin.Context) {}
        type OrderHandler struct{}
        func (h *OrderHandler) List(c *gin.Context) {}
        func Health(c *gin.Context) {}
        """)
    write(r, "server/router.go", """
        package server
        import (
            "github.com/gin-gonic/gin"
            "m/handlers"
        )
        func Setup(r *gin.Engine, userHandler *handlers.UserHandler, orderHandler *handlers.OrderHandler) {
            v1 := r.Group("/api/v1")
            users := v1.Group("/users")
            users.GET("", userHandler.List)
            v1.GET("/orders", orderHandler.List)
            r.GET("/health", handlers.Health)
        }
        """)
    u = GoSourceParser().scan(r).units["m/handlers"]
    ms = {m.method_name: (m.http_method, m.http_path) for m in u.methods}
    assert ms["UserHandler.List"] == ("GET", "/api/v1/users")
    assert ms["OrderHandler.List"] == ("GET", "/api/v1/orders")
    assert ms["Health"] == ("GET", "/health")


def test_no_go_mod_and_empty(tmp_path):
    assert GoSourceParser().parse(str(tmp_path)).node_count() == 0
    write(str(tmp_path), "a/a.go", "package a\nfunc A() {}\n")
    g = GoSourceParser().parse(str(tmp_path))
    assert g.identifiers() == ["a"] or g.node_count() == 1
