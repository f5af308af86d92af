"""One test per case of the reference's ``GraalJsAnalyzerEngineTest`` (25 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/domain/nodejs/GraalJsAnalyzerEngineTest.java``:
``detectFramework(packageJson)`` and ``analyzeFile(content, filePath,
framework)`` on in-memory sources, answered by :class:`AnalyzerEngine` over
the native TS/JS front-end instead of GraalJS + Babel.
"""
import textwrap

import pytest

from dmcp.parsers.tsengine import AnalyzerEngine


@pytest.fixture
def engine():
    e = AnalyzerEngine()
    yield e
    e.close()


def src(s):
    return textwrap.dedent(s).lstrip("\n")


def names(result):
    return [m.name for m in result.methods]


def test_when_creating_should_load_bundle_successfully(engine):
    assert engine is not None


def test_when_detecting_given_nest_js_project_should_detect_framework(engine):
    fw = engine.detect_framework('{ "dependencies": { "@nestjs/core": "10.0.0" } }')
    assert fw.name == "nestjs" and fw.source_root == "src"


def test_when_detecting_given_next_js_project_should_detect_framework(engine):
    assert engine.detect_framework('{ "dependencies": { "next": "14.0.0" } }').name == "nextjs"


def test_when_detecting_given_express_project_should_detect_framework(engine):
    assert engine.detect_framework('{ "dependencies": { "express": "4.18.0" } }').name == "express"


def test_when_detecting_given_vue_project_should_detect_framework(engine):
    assert engine.detect_framework('{ "dependencies": { "vue": "3.0.0" } }').name == "vue"


def test_when_detecting_given_angular_project_should_detect_framework(engine):
    assert engine.detect_framework('{ "dependencies": { "@angular/core": "17.0.0" } }').name == "angular"


def test_when_analyzing_file_given_class_with_methods_should_extract_all_methods(engine):
    r = engine.analyze_file(src("""
        export class UserService {
            findById(id: string) {
                return null;
            }

            createUser(name: string) {
                return { name };
            }
        }
        """), "src/services/user.service.ts", "unknown")
    assert names(r) == ["findById", "createUser"]


def test_when_analyzing_file_given_nest_js_controller_should_extract_http_info(engine):
    r = engine.analyze_file(src("""
        import { Controller, Get, Post } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get('/all')
            findAll() { return []; }

            @Post('/create')
            create(body: any) { return body; }
        }
        """), "src/user.controller.ts", "nestjs")
    assert r.class_type == "CONTROLLER" and r.entry_point
    assert [(m.http_method, m.http_path) for m in r.methods] == [("GET", "/all"), ("POST", "/create")]


def test_when_analyzing_file_given_injectable_service_should_infer_service_type(engine):
    r = engine.analyze_file(src("""
        import { Injectable } from '@nestjs/common';

        @Injectable()
        export class UserService {
            findAll() { return []; }
        }
        """), "src/user.service.ts", "nestjs")
    assert r.class_type == "SERVICE"


def test_when_analyzing_file_given_service_filename_should_infer_service_type(engine):
    r = engine.analyze_file("export class OrderService {\n    findAll() { return []; }\n}\n",
                            "src/order.service.ts", "unknown")
    assert r.class_type == "SERVICE"


def test_when_analyzing_file_given_relative_imports_should_extract_raw_imports(engine):
    r = engine.analyze_file(src("""
        import { UserService } from '../services/user.service';
        import { Config } from './config';
        import axios from 'axios';

        export class UserController {
            constructor(private userService: UserService) {}
        }
        """), "src/controllers/user.controller.ts", "unknown")
    assert len(r.raw_imports) == 3
    by_src = {i.source: i for i in r.raw_imports}
    assert (by_src["../services/user.service"].imported_name, by_src["../services/user.service"].local_name) == (
        "UserService", "UserService")
    assert by_src["./config"].imported_name == "Config"
    assert (by_src["axios"].imported_name, by_src["axios"].local_name) == ("default", "axios")


def test_when_analyzing_file_given_typed_params_should_extract_parameter_types(engine):
    r = engine.analyze_file(src("""
        import { UserRepository } from './user.repository';

        export class UserService {
            findUser(repo: UserRepository) {
                return repo.find();
            }
        }
        """), "src/services/user.service.ts", "unknown")
    assert names(r) == ["findUser"] and "UserRepository" in r.methods[0].parameter_types


def test_when_analyzing_file_given_main_file_should_detect_entry_point(engine):
    assert engine.analyze_file("async function bootstrap() {}\nbootstrap();\n", "src/main.ts", "unknown").entry_point


def test_when_analyzing_file_given_express_routes_should_detect_entry_point(engine):
    r = engine.analyze_file(src("""
        import { Router } from 'express';

        const router = Router();

        router.get('/users', (req, res) => res.json([]));

        export default router;
        """), "src/routes/users.ts", "unknown")
    assert r.entry_point and r.class_type == "CONTROLLER"


def test_when_analyzing_file_given_top_level_arrow_function_should_extract_method(engine):
    r = engine.analyze_file(src("""
        import { NextApiRequest, NextApiResponse } from 'next';

        const eventHandler = async (
            req: NextApiRequest,
            res: NextApiResponse
        ) => {
            res.json({ ok: true });
        };

        export default eventHandler;
        """), "pages/api/event/check/index.ts", "nextjs")
    m = next(m for m in r.methods if m.name == "eventHandler")
    assert "NextApiRequest" in m.parameter_types and "NextApiResponse" in m.parameter_types


def test_when_analyzing_file_given_multiple_top_level_arrow_functions_should_extract_all(engine):
    r = engine.analyze_file(src("""
        const handler = async (req: Request) => {
            return Response.json({});
        };

        const helper = (data: string) => {
            return data.toUpperCase();
        };

        export default handler;
        """), "src/api/handler.ts", "unknown")
    assert len(r.methods) == 2 and set(names(r)) == {"handler", "helper"}


def test_when_analyzing_file_given_object_with_arrow_functions_should_extract_methods(engine):
    r = engine.analyze_file(src("""
        export const validations = {
            email: (value: string) => {
                return value.includes('@');
            },
            password: (value: string) => {
                return value.length >= 8;
            },
        };
        """), "src/auth/validations.ts", "unknown")
    assert {"email", "password"} <= set(names(r))


def test_when_analyzing_file_given_object_shorthand_methods_should_extract_methods(engine):
    r = engine.analyze_file(src("""
        const api = {
            fetchUsers() {
                return fetch('/users');
            },
            createUser(data: UserDto) {
                return fetch('/users', { method: 'POST' });
            },
        };

        export default api;
        """), "src/lib/api.ts", "unknown")
    assert {"fetchUsers", "createUser"} <= set(names(r))


def test_when_analyzing_file_given_nested_arrow_functions_should_extract_them(engine):
    r = engine.analyze_file(src("""
        export default function FormEditShape() {
            const isSectionSeletable = (section: Section) => {
                return section.type === 'selectable';
            };

            const getOptionsByFieldName = (fieldName: string) => {
                return options[fieldName] || [];
            };

            return null;
        }
        """), "src/components/FormEditShape/index.tsx", "unknown")
    assert {"FormEditShape", "isSectionSeletable", "getOptionsByFieldName"} <= set(names(r))


def test_when_analyzing_file_given_use_callback_wrapped_should_extract_method(engine):
    r = engine.analyze_file(src("""
        import { useCallback } from 'react';

        export default function LoginContainer() {
            const handleLogin = useCallback(async (values: LoginValues) => {
                await loginApi(values);
            }, [loginApi]);

            const handleForgotPassword = useCallback(() => {
                navigate('/forgot-password');
            }, [navigate]);

            return null;
        }
        """), "src/components/LoginContainer.tsx", "unknown")
    assert {"handleLogin", "handleForgotPassword"} <= set(names(r))


def test_when_analyzing_file_given_use_memo_wrapped_should_extract_method(engine):
    r = engine.analyze_file(src("""
        import { useMemo } from 'react';

        export default function Component() {
            const computeTotal = useMemo(() => {
                return items.reduce((sum, i) => sum + i.price, 0);
            }, [items]);

            return null;
        }
        """), "src/components/Component.tsx", "unknown")
    assert "computeTotal" in names(r)


def test_when_analyzing_file_given_invalid_syntax_should_not_crash(engine):
    r = engine.analyze_file("this is not {{ valid syntax !!!", "src/broken.ts", "unknown")
    assert r is not None and r.methods == ()


def test_when_analyzing_multiple_files_should_reuse_engine(engine):
    s = engine.analyze_file("export class UserService {\n    findAll() { return []; }\n}\n",
                            "src/user.service.ts", "unknown")
    c = engine.analyze_file("export class UserController {\n    index() { return []; }\n}\n",
                            "src/user.controller.ts", "unknown")
    assert (s.class_type, len(s.methods)) == ("SERVICE", 1)
    assert (c.class_type, len(c.methods)) == ("CONTROLLER", 1)


def test_when_analyzing_file_given_standalone_functions_should_extract_them(engine):
    r = engine.analyze_file(src("""
        export function processOrder(orderId: string) {
            return orderId;
        }

        function internalHelper(data: any) {
            return data;
        }
        """), "src/lib/orders.ts", "unknown")
    assert names(r) == ["processOrder", "internalHelper"]


def test_when_analyzing_file_given_next_js_route_handler_should_extract_http_info(engine):
    r = engine.analyze_file(src("""
        export async function GET(request: Request) {
            return Response.json({ users: [] });
        }

        export async function POST(request: Request) {
            return Response.json({ created: true });
        }
        """), "src/app/api/users/route.ts", "nextjs")
    assert r.entry_point and r.methods
    get = next(m for m in r.methods if m.name == "GET")
    post = next(m for m in r.methods if m.name == "POST")
    assert (get.http_method, get.http_path) == ("GET", "/api/users") and post.http_method == "POST"
