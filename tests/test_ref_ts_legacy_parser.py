"""One test per case of the reference's ``NodeJsSourceParserTest`` (47 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/domain/nodejs/NodeJsSourceParserTest.java``
-- the regex-based parser that the reference keeps but never wires into
production.  Here it is :class:`LegacyNodeJsSourceParser`,
a mode of the native TS/JS front-end (see its docstring).  As in the
reference, the trees have no ``package.json`` and the per-file hooks are
called without a prior ``parse``.
"""
import os
import textwrap

import pytest

from dmcp.models.domain import ClassType
from dmcp.parsers.base import LegacyNodeJsSourceParser


@pytest.fixture
def parser():
    return LegacyNodeJsSourceParser()


def source_root(tmp_path):
    sr = os.path.join(str(tmp_path), "src")
    os.makedirs(sr, exist_ok=True)
    return sr


def write(sr, sub, name, content):
    d = os.path.join(sr, sub) if sub else sr
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, name)
    with open(p, "w") as f:
        f.write(textwrap.dedent(content).lstrip("\n"))
    return p


def graph(tmp_path, parser, files):
    sr = source_root(tmp_path)
    for sub, name, body in files:
        write(sr, sub, name, body)
    return parser.parse(str(tmp_path))


def test_when_getting_language_should_return_typescript(parser):
    assert parser.language() == "typescript"


def test_when_parsing_given_project_with_multiple_files_should_build_correct_graph(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("controllers", "user.controller.ts", """
            import { UserService } from '../services/user.service';

            @Controller('/users')
            export class UserController {
                constructor(private userService: UserService) {}
            }
            """),
        ("services", "user.service.ts", """
            import { UserRepository } from '../repositories/user.repository';

            export class UserService {
                constructor(private userRepo: UserRepository) {}
            }
            """),
        ("repositories", "user.repository.ts", """
            export class UserRepository {
                findById(id: string) { return null; }
            }
            """),
        ("", "main.ts", """
            import { NestFactory } from '@nestjs/core';
            import { AppModule } from './app.module';

            async function bootstrap() {
                const app = await NestFactory.create(AppModule);
                await app.listen(3000);
            }
            bootstrap();
            """)])
    assert g.node_count() == 4
    for i in ("controllers.user.controller", "services.user.service", "repositories.user.repository", "main"):
        assert g.contains(i)


def test_when_parsing_given_ts_and_js_files_should_discover_all(tmp_path, parser):
    g = graph(tmp_path, parser, [("", "app.ts", "export const a = 1;"), ("", "utils.js", "module.exports = {};"),
                                 ("", "Component.tsx", "export default () => <div/>;"),
                                 ("", "Legacy.jsx", "module.exports = () => <div/>;")])
    assert g.node_count() == 4 and all(g.contains(i) for i in ("app", "utils", "Component", "Legacy"))


def test_when_parsing_given_test_files_should_exclude_them(tmp_path, parser):
    g = graph(tmp_path, parser, [("", "service.ts", "export class Service {}"),
                                 ("", "service.spec.ts", "describe('Service', () => {});"),
                                 ("", "service.test.ts", "test('service', () => {});")])
    assert g.node_count() == 1 and g.contains("service")


def test_when_parsing_given_declaration_files_should_exclude_them(tmp_path, parser):
    g = graph(tmp_path, parser, [("", "service.ts", "export class Service {}"),
                                 ("", "types.d.ts", "declare module 'foo';")])
    assert g.node_count() == 1 and g.contains("service")


def test_when_parsing_given_excluded_directories_should_exclude_them(tmp_path, parser):
    g = graph(tmp_path, parser, [("", "app.ts", "export const app = true;"),
                                 ("node_modules/lodash", "index.ts", "export default {};"),
                                 ("dist", "bundle.js", "var x = 1;"),
                                 ("__tests__", "app.test.ts", "test('app', () => {});"),
                                 ("__mocks__", "mock.ts", "export default {};")])
    assert g.node_count() == 1 and g.contains("app")


def test_when_parsing_given_empty_source_directory_should_return_empty_graph(tmp_path, parser):
    g = graph(tmp_path, parser, [])
    assert g.node_count() == 0 and g.entry_point_count() == 0 and not g.identifiers()


def test_when_parsing_given_no_source_root_directory_should_return_empty_graph(tmp_path, parser):
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 0 and g.entry_point_count() == 0


def test_when_parsing_given_null_project_root_should_throw_exception(parser):
    with pytest.raises(ValueError):
        parser.parse(None)


def test_when_parsing_given_nested_path_should_produce_dotted_identifier(tmp_path, parser):
    assert graph(tmp_path, parser, [("services/user", "user.service.ts", "export class UserService {}")]
                 ).contains("services.user.user.service")


def test_when_parsing_given_root_file_should_produce_simple_identifier(tmp_path, parser):
    assert graph(tmp_path, parser, [("", "config.ts", "export const config = {};")]).contains("config")


def test_when_parsing_given_tsx_file_should_strip_extension(tmp_path, parser):
    assert graph(tmp_path, parser, [("components", "Button.tsx", "export const Button = () => <button/>;")]
                 ).contains("components.Button")


def test_when_parsing_given_source_file_paths_should_store_relative_paths(tmp_path, parser):
    g = graph(tmp_path, parser, [("services", "auth.service.ts", "export class AuthService {}")])
    assert g.source_file("services.auth.service") == "src/services/auth.service.ts"


def test_when_parsing_given_es6_relative_import_should_resolve_dependency(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("services", "order.service.ts", """
            import { OrderRepository } from './order.repository';

            export class OrderService {
                constructor(private repo: OrderRepository) {}
            }
            """),
        ("services", "order.repository.ts", "export class OrderRepository {}\n")])
    assert "services.order.repository" in g.resolve("services.order.service")


def test_when_parsing_given_es6_parent_dir_import_should_resolve_dependency(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("controllers", "order.controller.ts",
         "import { OrderService } from '../services/order.service';\n\nexport class OrderController {}\n"),
        ("services", "order.service.ts", "export class OrderService {}\n")])
    assert "services.order.service" in g.resolve("controllers.order.controller")


def test_when_parsing_given_es6_index_import_should_resolve_dependency(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("utils", "index.ts", "export function helper() {}\n"),
        ("services", "my.service.ts", """
            import { helper } from '../utils';

            export class MyService {
                run() { helper(); }
            }
            """)])
    assert "utils.index" in g.resolve("services.my.service")


def test_when_parsing_given_external_imports_should_filter_them_out(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("services", "api.service.ts", """
            import axios from 'axios';
            import { Injectable } from '@nestjs/common';
            import { Config } from './config';

            export class ApiService {}
            """),
        ("services", "config.ts", "export const Config = {};\n")])
    assert list(g.resolve("services.api.service")) == ["services.config"]


def test_when_parsing_given_require_relative_import_should_resolve_dependency(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("lib", "processor.js", """
            const helper = require('./helper');

            module.exports = { process: () => helper.run() };
            """),
        ("lib", "helper.js", "module.exports = { run: () => {} };\n")])
    assert "lib.helper" in g.resolve("lib.processor")


def entries(tmp_path, parser, sub, name, body):
    return graph(tmp_path, parser, [(sub, name, body)]).entry_point_count()


def test_when_parsing_given_main_ts_file_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "", "main.ts", "async function bootstrap() {}\nbootstrap();\n") == 1


def test_when_parsing_given_index_js_file_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "", "index.js", "const app = require('express')();\napp.listen(3000);\n") == 1


def test_when_parsing_given_app_ts_file_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "", "app.ts", "export class App {}\n") == 1


def test_when_parsing_given_server_js_file_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "", "server.js",
                   "const http = require('http');\n\nhttp.createServer().listen(3000);\n") == 1


def test_when_parsing_given_nest_js_controller_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "controllers", "user.controller.ts", """
        import { Controller, Get } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get()
            findAll() { return []; }
        }
        """) == 1


def test_when_parsing_given_express_routes_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "routes", "users.ts", """
        import { Router } from 'express';

        const router = Router();

        router.get('/users', (req, res) => {
            res.json([]);
        });

        router.post('/users', (req, res) => {
            res.status(201).json({});
        });

        export default router;
        """) == 1


def test_when_parsing_given_app_use_route_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "middleware", "logger.ts", """
        const express = require('express');
        const app = express();

        app.use('/api', (req, res, next) => {
            console.log('Request:', req.method, req.url);
            next();
        });
        """) == 1


def test_when_parsing_given_plain_service_should_not_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "services", "plain.service.ts", """
        export class PlainService {
            doSomething() { return 42; }
        }
        """) == 0


def test_when_getting_analysis_order_given_entry_point_with_deps_should_bfs_order(tmp_path, parser):
    g = graph(tmp_path, parser, [
        ("controllers", "order.controller.ts", """
            import { OrderService } from '../services/order.service';

            @Controller('/orders')
            export class OrderController {}
            """),
        ("services", "order.service.ts",
         "import { OrderRepo } from '../repositories/order.repo';\n\nexport class OrderService {}\n"),
        ("repositories", "order.repo.ts", "export class OrderRepo {}\n")])
    order = g.analysis_order()
    assert len(order) == 3 and order[0] == "controllers.order.controller"
    assert order.index("services.order.service") < order.index("repositories.order.repo")


def test_when_parsing_given_non_source_files_should_ignore_them(tmp_path, parser):
    g = graph(tmp_path, parser, [("", "valid.ts", "export const x = 1;"), ("", "config.json", "{}"),
                                 ("", "README.md", "# Hello")])
    assert g.node_count() == 1 and g.contains("valid")


def test_when_parsing_given_nested_identifier_should_work_with_source_class(tmp_path, parser):
    from dmcp.models.domain import package_name_of, simple_name_of
    ident = "services.user.user.service"
    assert graph(tmp_path, parser, [("services/user", "user.service.ts", "export class UserService {}")]
                 ).contains(ident)
    assert simple_name_of(ident) == "service" and package_name_of(ident) == "services.user.user"


# -- extractMethodParameters (no prior parse) ----------------------------------
def params(parser, sr, rel, known):
    return parser.extract_method_parameters(os.path.join(sr, rel), sr, set(known))


def test_when_extracting_params_given_typed_ts_param_should_return_it(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "services", "user.service.ts", """
        import { UserRepository } from './user.repository';

        export class UserService {
            findUser(repo: UserRepository) {
                return repo.find();
            }
        }
        """)
    write(sr, "services", "user.repository.ts", "export class UserRepository {\n    find() { return null; }\n}\n")
    r = params(parser, sr, "services/user.service.ts", {"services.user.service", "services.user.repository"})
    assert r["findUser"] == ["services.user.repository"]


def test_when_extracting_params_given_multiple_typed_params_should_return_all(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "services", "order.service.ts", """
        import { OrderRepo } from './order.repo';
        import { Customer } from './customer';

        export class OrderService {
            placeOrder(repo: OrderRepo, customer: Customer, note: string) {
            }
        }
        """)
    write(sr, "services", "order.repo.ts", "export class OrderRepo {}\n")
    write(sr, "services", "customer.ts", "export class Customer {}\n")
    p = params(parser, sr, "services/order.service.ts",
               {"services.order.service", "services.order.repo", "services.customer"})["placeOrder"]
    assert len(p) == 2 and set(p) == {"services.order.repo", "services.customer"}


def test_when_extracting_params_given_no_type_annotations_should_return_empty(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "lib", "processor.js", """
        module.exports = {
            process(data, count) {
                return data;
            }
        };
        """)
    assert params(parser, sr, "lib/processor.js", {"lib.processor"}) == {}


def test_when_extracting_params_given_only_primitive_types_should_return_empty(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "services", "calc.ts", """
        export class Calculator {
            add(a: number, b: number): number {
                return a + b;
            }
        }
        """)
    assert params(parser, sr, "services/calc.ts", {"services.calc"}) == {}


def test_when_extracting_params_given_async_function_should_extract_params(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "services", "api.service.ts", """
        import { HttpClient } from './http.client';

        export class ApiService {
            async fetchData(client: HttpClient) {
                return client.get('/data');
            }
        }
        """)
    write(sr, "services", "http.client.ts", "export class HttpClient {\n    get(url: string) { return null; }\n}\n")
    r = params(parser, sr, "services/api.service.ts", {"services.api.service", "services.http.client"})
    assert r["fetchData"] == ["services.http.client"]


# -- inferClassType (no prior parse) -------------------------------------------
def class_type(tmp_path, parser, sub, name, body):
    return parser.infer_class_type(write(source_root(tmp_path), sub, name, body))


def test_when_inferring_class_type_given_nest_js_controller_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "controllers", "user.controller.ts", """
        import { Controller, Get } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get()
            findAll() { return []; }
        }
        """) is ClassType.CONTROLLER


def test_when_inferring_class_type_given_nest_js_injectable_should_return_service(tmp_path, parser):
    assert class_type(tmp_path, parser, "services", "user.service.ts", """
        import { Injectable } from '@nestjs/common';

        @Injectable()
        export class UserService {
            findAll() { return []; }
        }
        """) is ClassType.SERVICE


def test_when_inferring_class_type_given_express_routes_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "routes", "users.ts", """
        import { Router } from 'express';

        const router = Router();

        router.get('/users', (req, res) => res.json([]));

        export default router;
        """) is ClassType.CONTROLLER


def test_when_inferring_class_type_given_controller_filename_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.controller.ts",
                      "export class OrderController {\n    create() { return {}; }\n}\n") is ClassType.CONTROLLER


def test_when_inferring_class_type_given_service_filename_should_return_service(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.service.ts",
                      "export class OrderService {\n    findAll() { return []; }\n}\n") is ClassType.SERVICE


def test_when_inferring_class_type_given_repository_filename_should_return_repository(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.repository.ts",
                      "export class OrderRepository {\n    findAll() { return []; }\n}\n") is ClassType.REPOSITORY


def test_when_inferring_class_type_given_entity_filename_should_return_entity(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.entity.ts",
                      "export class Order {\n    id: string;\n    total: number;\n}\n") is ClassType.ENTITY


def test_when_inferring_class_type_given_plain_file_should_return_other(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "utils.ts",
                      "export function helper() {\n    return 42;\n}\n") is ClassType.OTHER


# -- extractMethods (no prior parse) -------------------------------------------
def methods(tmp_path, parser, name, body):
    return parser.extract_methods(write(source_root(tmp_path), "", name, body))


def test_when_extracting_methods_given_simple_functions_should_return_with_line_numbers(tmp_path, parser):
    ms = methods(tmp_path, parser, "service.ts", """
        export class UserService {
            findById(id: string) {
                return null;
            }

            createUser(name: string) {
                return { name };
            }
        }
        """)
    assert [(m.method_name, m.line_number) for m in ms] == [("findById", 2), ("createUser", 6)]


def test_when_extracting_methods_given_nest_js_decorators_should_extract_http_info(tmp_path, parser):
    ms = methods(tmp_path, parser, "user.controller.ts", """
        import { Controller, Get, Post } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get('/all')
            findAll() { return []; }

            @Post('/create')
            create(body: any) { return body; }
        }
        """)
    assert [(m.method_name, m.http_method, m.http_path) for m in ms] == [
        ("findAll", "GET", "/all"), ("create", "POST", "/create")]


def test_when_extracting_methods_given_async_function_should_extract_it(tmp_path, parser):
    (m,) = methods(tmp_path, parser, "api.service.ts", """
        export class ApiService {
            async fetchData(url: string) {
                return fetch(url);
            }
        }
        """)
    assert m.method_name == "fetchData" and m.http_method is None and not m.exceptions


def test_when_extracting_methods_given_keywords_should_exclude_them(tmp_path, parser):
    ms = methods(tmp_path, parser, "processor.ts", """
        export class Processor {
            process(data: string) {
                if (data) {
                    for (const item of []) {
                        while (true) {
                            break;
                        }
                    }
                }
            }
        }
        """)
    assert [m.method_name for m in ms] == ["process"]


def test_when_extracting_methods_given_no_methods_should_return_empty(tmp_path, parser):
    assert methods(tmp_path, parser, "constants.ts",
                   "export const API_URL = 'https://api.example.com';\nexport const MAX_RETRIES = 3;\n") == []
