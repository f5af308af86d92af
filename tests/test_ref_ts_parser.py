"""One test per case of the reference's ``NodeJsGraalParserTest`` (40 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/domain/nodejs/NodeJsGraalParserTest.java``
(GraalJS + Babel bundle there; the native C++ TS/JS front-end here) with the
same ``@TempDir`` trees (``createSourceRoot`` / ``writePackageJson`` /
``writeSourceFile``, ``:983-1006``).
"""
import os
import textwrap

import pytest

from dmcp.models.domain import ClassType
from dmcp.parsers.base import NodeJsSourceParser

NEST = '{"dependencies":{"@nestjs/core":"10.0.0"}}'


@pytest.fixture
def parser():
    return NodeJsSourceParser()


def project(tmp_path, pkg="{}"):
    sr = os.path.join(str(tmp_path), "src")
    os.makedirs(sr, exist_ok=True)
    with open(os.path.join(str(tmp_path), "package.json"), "w") as f:
        f.write(pkg)
    return sr


def write(sr, sub, name, content):
    d = os.path.join(sr, sub) if sub else sr
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, name)
    with open(p, "w") as f:
        f.write(textwrap.dedent(content).lstrip("\n"))
    return p


def test_when_getting_language_should_return_typescript(parser):
    assert parser.language() == "typescript"


def test_when_parsing_given_project_with_multiple_files_should_build_correct_graph(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "controllers", "user.controller.ts", """
        import { UserService } from '../services/user.service';

        @Controller('/users')
        export class UserController {
            constructor(private userService: UserService) {}
        }
        """)
    write(sr, "services", "user.service.ts", """
        import { UserRepository } from '../repositories/user.repository';

        export class UserService {
            constructor(private userRepo: UserRepository) {}
        }
        """)
    write(sr, "repositories", "user.repository.ts", """
        export class UserRepository {
            findById(id: string) { return null; }
        }
        """)
    write(sr, "", "main.ts", """
        import { NestFactory } from '@nestjs/core';
        import { AppModule } from './app.module';

        async function bootstrap() {
            const app = await NestFactory.create(AppModule);
            await app.listen(3000);
        }
        bootstrap();
        """)
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 4
    for i in ("controllers.user.controller", "services.user.service", "repositories.user.repository", "main"):
        assert g.contains(i)


def test_when_parsing_given_ts_and_js_files_should_discover_all(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "", "app.ts", "export const a = 1;")
    write(sr, "", "utils.js", "module.exports = {};")
    write(sr, "", "Component.tsx", "export default function Comp() { return null; }")
    write(sr, "", "Legacy.jsx", "module.exports = function() { return null; };")
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 4 and all(g.contains(i) for i in ("app", "utils", "Component", "Legacy"))


def test_when_parsing_given_test_files_should_exclude_them(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "", "service.ts", "export class Service {}")
    write(sr, "", "service.spec.ts", "describe('Service', () => {});")
    write(sr, "", "service.test.ts", "test('service', () => {});")
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 1 and g.contains("service")


def test_when_parsing_given_declaration_files_should_exclude_them(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "", "service.ts", "export class Service {}")
    write(sr, "", "types.d.ts", "declare module 'foo';")
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 1 and g.contains("service")


def test_when_parsing_given_excluded_directories_should_exclude_them(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "", "app.ts", "export const app = true;")
    write(sr, "node_modules/lodash", "index.ts", "export default {};")
    write(sr, "dist", "bundle.js", "var x = 1;")
    write(sr, "__tests__", "app.test.ts", "test('app', () => {});")
    write(sr, "__mocks__", "mock.ts", "export default {};")
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 1 and g.contains("app")


def test_when_parsing_given_empty_source_directory_should_return_empty_graph(tmp_path, parser):
    project(tmp_path)
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 0 and g.entry_point_count() == 0 and not g.identifiers()


def test_when_parsing_given_null_project_root_should_throw_exception(parser):
    with pytest.raises(ValueError):
        parser.parse(None)


def test_when_parsing_given_nested_path_should_produce_dotted_identifier(tmp_path, parser):
    write(project(tmp_path), "services/user", "user.service.ts", "export class UserService {}")
    assert parser.parse(str(tmp_path)).contains("services.user.user.service")


def test_when_parsing_given_root_file_should_produce_simple_identifier(tmp_path, parser):
    write(project(tmp_path), "", "config.ts", "export const config = {};")
    assert parser.parse(str(tmp_path)).contains("config")


def test_when_parsing_given_tsx_file_should_strip_extension(tmp_path, parser):
    write(project(tmp_path), "components", "Button.tsx", "export default function Button() { return null; }")
    assert parser.parse(str(tmp_path)).contains("components.Button")


def test_when_parsing_given_source_file_paths_should_store_relative_paths(tmp_path, parser):
    write(project(tmp_path), "services", "auth.service.ts", "export class AuthService {}")
    assert parser.parse(str(tmp_path)).source_file("services.auth.service") == "src/services/auth.service.ts"


def test_when_parsing_given_es6_relative_import_should_resolve_dependency(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "services", "order.service.ts", """
        import { OrderRepository } from './order.repository';

        export class OrderService {
            constructor(private repo: OrderRepository) {}
        }
        """)
    write(sr, "services", "order.repository.ts", "export class OrderRepository {}\n")
    assert "services.order.repository" in parser.parse(str(tmp_path)).resolve("services.order.service")


def test_when_parsing_given_es6_parent_dir_import_should_resolve_dependency(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "controllers", "order.controller.ts", """
        import { OrderService } from '../services/order.service';

        export class OrderController {}
        """)
    write(sr, "services", "order.service.ts", "export class OrderService {}\n")
    assert "services.order.service" in parser.parse(str(tmp_path)).resolve("controllers.order.controller")


def test_when_parsing_given_es6_index_import_should_resolve_dependency(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "utils", "index.ts", "export function helper() {}\n")
    write(sr, "services", "my.service.ts", """
        import { helper } from '../utils';

        export class MyService {
            run() { helper(); }
        }
        """)
    assert "utils.index" in parser.parse(str(tmp_path)).resolve("services.my.service")


def test_when_parsing_given_external_imports_should_filter_them_out(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "services", "api.service.ts", """
        import axios from 'axios';
        import { Injectable } from '@nestjs/common';
        import { Config } from './config';

        export class ApiService {}
        """)
    write(sr, "services", "config.ts", "export const Config = {};\n")
    assert list(parser.parse(str(tmp_path)).resolve("services.api.service")) == ["services.config"]


def entries(tmp_path, parser, sub, name, body, pkg="{}"):
    write(project(tmp_path, pkg), sub, name, body)
    return parser.parse(str(tmp_path)).entry_point_count()


def test_when_parsing_given_main_ts_file_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "", "main.ts", "async function bootstrap() {}\nbootstrap();\n") == 1


def test_when_parsing_given_index_js_file_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "", "index.js",
                   "const app = require('express')();\napp.listen(3000);\n") == 1


def test_when_parsing_given_nest_js_controller_should_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "controllers", "user.controller.ts", """
        import { Controller, Get } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get()
            findAll() { return []; }
        }
        """, NEST) == 1


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


def test_when_parsing_given_plain_service_should_not_detect_entry_point(tmp_path, parser):
    assert entries(tmp_path, parser, "services", "plain.service.ts", """
        export class PlainService {
            doSomething() { return 42; }
        }
        """) == 0


def test_when_getting_analysis_order_given_entry_point_with_deps_should_bfs_order(tmp_path, parser):
    sr = project(tmp_path, NEST)
    write(sr, "controllers", "order.controller.ts", """
        import { OrderService } from '../services/order.service';

        @Controller('/orders')
        export class OrderController {}
        """)
    write(sr, "services", "order.service.ts", """
        import { OrderRepo } from '../repositories/order.repo';

        export class OrderService {}
        """)
    write(sr, "repositories", "order.repo.ts", "export class OrderRepo {}\n")
    order = parser.parse(str(tmp_path)).analysis_order()
    assert len(order) == 3 and order[0] == "controllers.order.controller"
    assert order.index("services.order.service") < order.index("repositories.order.repo")


def test_when_parsing_given_non_source_files_should_ignore_them(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "", "valid.ts", "export const x = 1;")
    write(sr, "", "config.json", "{}")
    write(sr, "", "README.md", "# Hello")
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 1 and g.contains("valid")


# -- extractMethodParameters ---------------------------------------------------
def test_when_extracting_params_given_typed_ts_param_should_return_it(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "services", "user.service.ts", """
        import { UserRepository } from './user.repository';

        export class UserService {
            findUser(repo: UserRepository) {
                return repo.find();
            }
        }
        """)
    write(sr, "services", "user.repository.ts", """
        export class UserRepository {
            find() { return null; }
        }
        """)
    parser.parse(str(tmp_path))
    r = parser.extract_method_parameters(os.path.join(sr, "services/user.service.ts"), sr,
                                         {"services.user.service", "services.user.repository"})
    assert r["findUser"] == ["services.user.repository"]


def test_when_extracting_params_given_multiple_typed_params_should_return_all(tmp_path, parser):
    sr = project(tmp_path)
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
    parser.parse(str(tmp_path))
    p = parser.extract_method_parameters(os.path.join(sr, "services/order.service.ts"), sr,
                                         {"services.order.service", "services.order.repo", "services.customer"})
    assert len(p["placeOrder"]) == 2 and set(p["placeOrder"]) == {"services.order.repo", "services.customer"}


def test_when_extracting_params_given_no_type_annotations_should_return_empty(tmp_path, parser):
    sr = project(tmp_path)
    write(sr, "lib", "processor.js", """
        module.exports = {
            process(data, count) {
                return data;
            }
        };
        """)
    parser.parse(str(tmp_path))
    assert parser.extract_method_parameters(os.path.join(sr, "lib/processor.js"), sr, {"lib.processor"}) == {}


# -- inferClassType ------------------------------------------------------------
def class_type(tmp_path, parser, sub, name, body, pkg="{}"):
    f = write(project(tmp_path, pkg), sub, name, body)
    parser.parse(str(tmp_path))
    return parser.infer_class_type(f)


def test_when_inferring_class_type_given_nest_js_controller_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "controllers", "user.controller.ts", """
        import { Controller, Get } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get()
            findAll() { return []; }
        }
        """, NEST) is ClassType.CONTROLLER


def test_when_inferring_class_type_given_nest_js_injectable_should_return_service(tmp_path, parser):
    assert class_type(tmp_path, parser, "services", "user.service.ts", """
        import { Injectable } from '@nestjs/common';

        @Injectable()
        export class UserService {
            findAll() { return []; }
        }
        """, NEST) is ClassType.SERVICE


def test_when_inferring_class_type_given_express_routes_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "routes", "users.ts", """
        import { Router } from 'express';

        const router = Router();

        router.get('/users', (req, res) => res.json([]));

        export default router;
        """) is ClassType.CONTROLLER


def test_when_inferring_class_type_given_controller_filename_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.controller.ts", """
        export class OrderController {
            create() { return {}; }
        }
        """) is ClassType.CONTROLLER


def test_when_inferring_class_type_given_service_filename_should_return_service(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.service.ts", """
        export class OrderService {
            findAll() { return []; }
        }
        """) is ClassType.SERVICE


def test_when_inferring_class_type_given_repository_filename_should_return_repository(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.repository.ts", """
        export class OrderRepository {
            findAll() { return []; }
        }
        """) is ClassType.REPOSITORY


def test_when_inferring_class_type_given_entity_filename_should_return_entity(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "order.entity.ts", """
        export class Order {
            id: string;
            total: number;
        }
        """) is ClassType.ENTITY


def test_when_inferring_class_type_given_plain_file_should_return_other(tmp_path, parser):
    assert class_type(tmp_path, parser, "", "utils.ts", """
        export function helper() {
            return 42;
        }
        """) is ClassType.OTHER


# -- extractMethods ------------------------------------------------------------
def methods(tmp_path, parser, sub, name, body, pkg="{}"):
    f = write(project(tmp_path, pkg), sub, name, body)
    parser.parse(str(tmp_path))
    return parser.extract_methods(f)


def test_when_extracting_methods_given_simple_functions_should_return_with_line_numbers(tmp_path, parser):
    ms = methods(tmp_path, parser, "", "service.ts", """
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
    ms = methods(tmp_path, parser, "", "user.controller.ts", """
        import { Controller, Get, Post } from '@nestjs/common';

        @Controller('/users')
        export class UserController {
            @Get('/all')
            findAll() { return []; }

            @Post('/create')
            create(body: any) { return body; }
        }
        """, NEST)
    assert [(m.method_name, m.http_method, m.http_path) for m in ms] == [
        ("findAll", "GET", "/all"), ("create", "POST", "/create")]


def test_when_extracting_methods_given_async_function_should_extract_it(tmp_path, parser):
    (m,) = methods(tmp_path, parser, "", "api.service.ts", """
        export class ApiService {
            async fetchData(url: string) {
                return fetch(url);
            }
        }
        """)
    assert m.method_name == "fetchData" and m.http_method is None and not m.exceptions


def test_when_extracting_methods_given_no_methods_should_return_empty(tmp_path, parser):
    assert methods(tmp_path, parser, "", "constants.ts", """
        export const API_URL = 'https://api.example.com';
        export const MAX_RETRIES = 3;
        """) == []


def test_when_extracting_methods_given_top_level_arrow_function_should_extract_it(tmp_path, parser):
    ms = methods(tmp_path, parser, "api", "handler.ts", """
        const eventHandler = async (req: Request, res: Response) => {
            res.json({ ok: true });
        };

        export default eventHandler;
        """)
    assert [m.method_name for m in ms] == ["eventHandler"]


def test_when_extracting_methods_given_function_expression_variable_should_extract_it(tmp_path, parser):
    ms = methods(tmp_path, parser, "api", "process.ts", """
        const processData = function(input: string) {
            return input.trim();
        };

        export default processData;
        """)
    assert [m.method_name for m in ms] == ["processData"]
