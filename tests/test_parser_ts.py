"""TypeScript / JavaScript front-end (NodeJsGraalParserTest, NodeJsSourceParserTest
and GraalJsAnalyzerEngineTest in the reference)."""
import json
import os
import textwrap

import pytest

from dmcp.models.domain import ClassType
from dmcp.parsers.base import NodeJsSourceParser, native


def write(root, rel, body):
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(textwrap.dedent(body).lstrip("\n"))
    return p


def analyze(src, rel="src/x.ts", fw="unknown"):
    p = "/tmp/_dmcp_ts_probe_" + os.path.basename(rel)
    with open(p, "w") as f:
        f.write(textwrap.dedent(src).lstrip("\n"))
    try:
        return json.loads(native().scan_file(p, "typescript", rel, fw))
    finally:
        os.unlink(p)


@pytest.fixture
def parser():
    return NodeJsSourceParser()


def test_language_and_graph(tmp_path, parser):
    r = str(tmp_path)
    write(r, "package.json", '{"dependencies": {"@nestjs/core": "10"}}')
    write(r, "src/main.ts", "import { AppModule } from './app.module';\nasync function bootstrap() {}\nbootstrap();\n")
    write(r, "src/app.module.ts", "import { UsersController } from './users/users.controller';\nexport class AppModule {}\n")
    write(r, "src/users/users.controller.ts", """
        import { Controller, Get } from '@nestjs/common';
        import { UsersService } from './users.service';
        @Controller('users')
        export class UsersController {
          constructor(private readonly svc: UsersService) {}
          @Get()
          list() { return this.svc.all(); }
        }
        """)
    write(r, "src/users/users.service.ts", """
        import { Injectable } from '@nestjs/common';
        import { User } from '../entities/user.entity';
        @Injectable()
        export class UsersService { all(): User[] { return []; } }
        """)
    write(r, "src/entities/user.entity.ts", "export class User { id: string; }\n")
    assert parser.language() == "typescript"
    g = parser.parse(r)
    assert parser.framework()["name"] == "nestjs" and parser.source_root() == "src"
    assert set(g.identifiers()) == {"main", "app.module", "users.users.controller", "users.users.service",
                                    "entities.user.entity"}
    assert g.dependencies("users.users.controller") == ("users.users.service",)
    assert g.dependencies("users.users.service") == ("entities.user.entity",)
    assert g.is_entry_point("main") and g.is_entry_point("users.users.controller")
    assert not g.is_entry_point("users.users.service")
    assert g.source_file("users.users.service") == "src/users/users.service.ts"
    order = g.analysis_order()
    assert order.index("users.users.controller") < order.index("users.users.service") < order.index(
        "entities.user.entity")


def test_discovery_rules(tmp_path, parser):
    r = str(tmp_path)
    write(r, "src/a.ts", "export const a = 1;\n")
    write(r, "src/b.js", "module.exports = {};\n")
    write(r, "src/c.tsx", "export default function C() { return null; }\n")
    write(r, "src/d.jsx", "export function D() {}\n")
    write(r, "src/a.test.ts", "test('x', () => {});\n")
    write(r, "src/a.spec.ts", "describe('x', () => {});\n")
    write(r, "src/types.d.ts", "declare const X: number;\n")
    for d in ("node_modules", "dist", ".next", "build", "coverage", "__tests__", "__mocks__"):
        write(r, f"src/{d}/x.ts", "export const x = 1;\n")
    write(r, "src/readme.md", "# no")
    write(r, "src/deep/nested/path/thing.ts", "export const t = 1;\n")
    g = parser.parse(r)
    assert set(g.identifiers()) == {"a", "b", "c", "d", "deep.nested.path.thing"}


def test_empty_missing_and_null(tmp_path, parser):
    os.makedirs(tmp_path / "src")
    assert parser.parse(str(tmp_path)).node_count() == 0
    assert NodeJsSourceParser().parse(str(tmp_path / "none")).node_count() == 0
    with pytest.raises(ValueError):
        parser.parse(None)


def test_import_resolution(tmp_path, parser):
    r = str(tmp_path)
    write(r, "src/services/user.service.ts", "export class UserService {}\n")
    write(r, "src/utils/index.ts", "export const u = 1;\n")
    write(r, "src/lib/helper.js", "module.exports = {};\n")
    write(r, "src/controllers/user.controller.ts", """
        import { UserService } from '../services/user.service';
        import * as utils from '../utils';
        import express from 'express';
        import { x } from '@scope/pkg';
        const helper = require('../lib/helper');
        export class UserController {}
        """)
    g = parser.parse(r)
    assert set(g.dependencies("controllers.user.controller")) == {"services.user.service", "utils.index",
                                                                  "lib.helper"}


@pytest.mark.parametrize("rel,src,entry", [
    ("src/main.ts", "console.log(1);\n", True), ("src/index.js", "x();\n", True),
    ("src/app.ts", "export const app = 1;\n", True), ("src/server.js", "listen();\n", True),
    ("src/routes/users.ts", "router.get('/users', (req, res) => res.send([]));\n", True),
    ("src/api.ts", "app.use('/api', router);\n", True),
    ("src/plain.service.ts", "export class PlainService { run() {} }\n", False)])
def test_entry_points(rel, src, entry):
    assert analyze(src, rel)["entryPoint"] is entry


@pytest.mark.parametrize("rel,src,fw,ctype", [
    ("src/u.ts", "@Controller('u')\nexport class U {}\n", "nestjs", "CONTROLLER"),
    ("src/s.ts", "@Injectable()\nexport class S {}\n", "nestjs", "SERVICE"),
    ("src/r.ts", "router.get('/x', h);\n", "express", "CONTROLLER"),
    ("src/users.controller.ts", "export class A {}\n", "unknown", "CONTROLLER"),
    ("src/users.service.ts", "export class A {}\n", "unknown", "SERVICE"),
    ("src/users.repository.ts", "export class A {}\n", "unknown", "REPOSITORY"),
    ("src/user.entity.ts", "export class A {}\n", "unknown", "ENTITY"),
    ("src/plain.ts", "export class A {}\n", "unknown", "OTHER")])
def test_class_types(rel, src, fw, ctype):
    assert analyze(src, rel, fw)["classType"] == ctype


def test_methods_and_nest_http():
    d = analyze("""
        import { Controller, Get, Post, Put, Delete, Patch, Body } from '@nestjs/common';
        @Controller('users')
        export class UsersController {
          constructor(private readonly s: UsersService) {}

          @Get(':id')
          findOne(id: string) { return 1; }

          @Post()
          async create(@Body() dto: CreateUserDto) {}

          @Put('a') put() {}
          @Delete('b') del() {}
          @Patch('c') patch() {}
          private helper() {}
        }
        """, "src/users/users.controller.ts", "nestjs")
    ms = [(m["name"], m.get("httpMethod"), m.get("httpPath")) for m in d["methods"]]
    assert ("findOne", "GET", ":id") in ms and ("create", "POST", "/") in ms
    assert ("put", "PUT", "a") in ms and ("del", "DELETE", "b") in ms and ("patch", "PATCH", "c") in ms
    assert ("helper", None, None) in ms
    line = {m["name"]: m["line"] for m in d["methods"]}
    assert line["findOne"] == 6  # Babel: a decorated member starts at its first decorator


def test_functions_arrows_objects_hooks():
    d = analyze("""
        import { useCallback, useMemo } from 'react';
        export const validations = {
            email: (value: string) => value.includes('@'),
            password(value: string) { return value.length >= 8; },
        };
        export async function load(id: string) {}
        export const save = async (u: User) => {};
        const legacy = function (x) { return x; };
        export default function Form() {
            const isOk = (s: Section) => true;
            const onLogin = useCallback(async (v: LoginValues) => {}, []);
            const total = useMemo(() => 1, []);
            return null;
        }
        if (x) { while (y) {} }
        """, "src/form.tsx")
    names = [m["name"] for m in d["methods"]]
    for n in ("email", "password", "load", "save", "legacy", "Form", "isOk", "onLogin", "total"):
        assert n in names, (n, names)
    for kw in ("if", "while", "return", "function"):
        assert kw not in names


def test_nextjs_route_handlers():
    d = analyze("""
        export async function GET(request: Request) { return Response.json([]); }
        export async function POST(request: Request) { return Response.json({}); }
        """, "src/app/api/users/route.ts", "nextjs")
    assert d["entryPoint"]
    ms = {m["name"]: (m.get("httpMethod"), m.get("httpPath")) for m in d["methods"]}
    assert ms["GET"] == ("GET", "/api/users") and ms["POST"] == ("POST", "/api/users")


def test_parameter_types(tmp_path, parser):
    r = str(tmp_path)
    write(r, "src/dto/create-user.dto.ts", "export class CreateUserDto {}\n")
    write(r, "src/models/user.ts", "export interface User { id: string }\n")
    f = write(r, "src/users.service.ts", """
        import { CreateUserDto } from './dto/create-user.dto';
        import { User } from './models/user';
        export class UsersService {
          create(dto: CreateUserDto, actor: User, note: string) {}
          async find(id: string, count: number) {}
          untyped(a, b) {}
          list(users: User[], opts?: Partial<CreateUserDto>) {}
        }
        """)
    parser.scan(r)
    p = parser.extract_method_parameters(f)
    assert p["create"] == ["dto.create-user.dto", "models.user"]
    assert "find" not in p and "untyped" not in p


def test_invalid_syntax_does_not_crash():
    d = analyze("export class { ((( ]]] function ( => {{{ `${ unterminated", "src/bad.ts")
    assert d["parsed"] in (True, False)


def test_framework_detection():
    fw = native().detect_framework
    assert fw('{"dependencies": {"@nestjs/core": "10"}}')["name"] == "nestjs"
    assert fw('{"dependencies": {"next": "14"}}')["name"] == "nextjs"
    assert fw('{"dependencies": {"express": "4"}}')["name"] == "express"
    assert fw('{"dependencies": {"vue": "3"}}')["name"] == "vue"
    assert fw('{"dependencies": {"@angular/core": "17"}}')["name"] == "angular"
    assert fw("{}")["name"] == "unknown" and fw("not json")["name"] == "unknown"
