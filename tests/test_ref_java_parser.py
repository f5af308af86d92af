"""One test per case of the reference's ``JavaSourceParserTest`` (45 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/domain/java/JavaSourceParserTest.java``:
the same ``@TempDir`` source trees (``createSourceRoot`` / ``writeJavaFile``
helpers, ``:1237-1262``) parsed by the native C++ Java front-end.  The
per-file hooks (``infer_class_type`` / ``extract_methods`` /
``extract_method_parameters``) are called stand-alone, without a prior
project parse, as the reference does.
"""
import os
import textwrap

import pytest

from dmcp.models.domain import ClassType
from dmcp.parsers.base import JavaSourceParser


@pytest.fixture
def parser():
    return JavaSourceParser()


def source_root(root):
    sr = os.path.join(str(root), "src", "main", "java")
    os.makedirs(sr, exist_ok=True)
    return sr


def write(sr, pkg_path, name, content):
    d = os.path.join(sr, pkg_path) if pkg_path else sr
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, name)
    with open(p, "w") as f:
        f.write(textwrap.dedent(content).lstrip("\n"))
    return p


def test_when_parsing_given_project_with_multiple_files_should_build_correct_graph(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Application.java", """
        package co.fanki.app;
        import org.springframework.boot.SpringApplication;
        @SpringBootApplication
        public class Application {
            public static void main(String[] args) {
                SpringApplication.run(Application.class, args);
            }
        }
        """)
    write(sr, "co/fanki/app/controller", "UserController.java", """
        package co.fanki.app.controller;
        import co.fanki.app.service.UserService;
        import org.springframework.web.bind.annotation.GetMapping;
        @RestController
        public class UserController {
            private final UserService userService;
        }
        """)
    write(sr, "co/fanki/app/service", "UserService.java", """
        package co.fanki.app.service;
        import co.fanki.app.domain.User;
        public class UserService {
            public User findById(String id) { return null; }
        }
        """)
    write(sr, "co/fanki/app/domain", "User.java", """
        package co.fanki.app.domain;
        public class User {
            private String id;
            private String name;
        }
        """)
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 4
    for ident in ("co.fanki.app.Application", "co.fanki.app.controller.UserController",
                  "co.fanki.app.service.UserService", "co.fanki.app.domain.User"):
        assert g.contains(ident)


def test_when_parsing_given_dependencies_between_files_should_resolve_edges(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "OrderService.java", """
        package co.fanki.app;
        import co.fanki.app.OrderRepository;
        public class OrderService {
            private final OrderRepository repo;
        }
        """)
    write(sr, "co/fanki/app", "OrderRepository.java", "package co.fanki.app;\npublic class OrderRepository {\n}\n")
    g = parser.parse(str(tmp_path))
    assert "co.fanki.app.OrderRepository" in g.resolve("co.fanki.app.OrderService")


def test_when_parsing_given_entry_point_annotations_should_mark_entry_points(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "ApiController.java", "package co.fanki.app;\n@RestController\npublic class ApiController {\n}\n")
    write(sr, "co/fanki/app", "PlainService.java", "package co.fanki.app;\npublic class PlainService {\n}\n")
    g = parser.parse(str(tmp_path))
    assert g.entry_point_count() == 1
    assert g.analysis_order()[0] == "co.fanki.app.ApiController"


def test_when_parsing_given_empty_source_directory_should_return_empty_graph(tmp_path, parser):
    source_root(tmp_path)
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 0 and g.entry_point_count() == 0 and not g.identifiers()


def test_when_parsing_given_no_source_root_directory_should_return_empty_graph(tmp_path, parser):
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 0 and g.entry_point_count() == 0


def test_when_parsing_given_null_project_root_should_throw_exception(parser):
    with pytest.raises(ValueError):
        parser.parse(None)


def test_when_parsing_given_source_file_paths_should_store_relative_paths(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Config.java", "package co.fanki.app;\npublic class Config {\n}\n")
    g = parser.parse(str(tmp_path))
    assert g.source_file("co.fanki.app.Config") == "src/main/java/co/fanki/app/Config.java"


def test_when_parsing_given_external_imports_should_filter_to_internal_only(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "MyService.java", """
        package co.fanki.app;
        import java.util.List;
        import org.springframework.stereotype.Service;
        import co.fanki.app.MyRepository;
        @Service
        public class MyService {
        }
        """)
    write(sr, "co/fanki/app", "MyRepository.java", "package co.fanki.app;\npublic class MyRepository {\n}\n")
    deps = parser.parse(str(tmp_path)).resolve("co.fanki.app.MyService")
    assert list(deps) == ["co.fanki.app.MyRepository"]


def test_when_parsing_given_static_import_of_internal_class_should_resolve_dependency(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Constants.java", """
        package co.fanki.app;
        public class Constants {
            public static final String NAME = "fanki";
        }
        """)
    write(sr, "co/fanki/app", "Printer.java", """
        package co.fanki.app;
        import static co.fanki.app.Constants.NAME;
        public class Printer {
        }
        """)
    assert "co.fanki.app.Constants" in parser.parse(str(tmp_path)).resolve("co.fanki.app.Printer")


def test_when_parsing_given_imports_after_class_declaration_should_ignore_them(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Ignored.java", "package co.fanki.app;\npublic class Ignored {\n}\n")
    write(sr, "co/fanki/app", "Weird.java", "package co.fanki.app;\npublic class Weird {\n}\n")
    assert "co.fanki.app.Ignored" not in parser.parse(str(tmp_path)).resolve("co.fanki.app.Weird")


def entry_count(tmp_path, parser, name, body):
    write(source_root(tmp_path), "co/fanki/app", name, body)
    return parser.parse(str(tmp_path)).entry_point_count()


def test_when_parsing_given_controller_annotation_should_detect_entry_point(tmp_path, parser):
    assert entry_count(tmp_path, parser, "WebController.java",
                       "package co.fanki.app;\n@Controller\npublic class WebController {\n}\n") == 1


def test_when_parsing_given_kafka_listener_annotation_should_detect_entry_point(tmp_path, parser):
    assert entry_count(tmp_path, parser, "EventConsumer.java", """
        package co.fanki.app;
        public class EventConsumer {
            @KafkaListener(topics = "orders")
            public void consume(String message) {
            }
        }
        """) == 1


def test_when_parsing_given_scheduled_annotation_should_detect_entry_point(tmp_path, parser):
    assert entry_count(tmp_path, parser, "CronJob.java", """
        package co.fanki.app;
        public class CronJob {
            @Scheduled(fixedRate = 5000)
            public void run() {
            }
        }
        """) == 1


def test_when_parsing_given_event_listener_annotation_should_detect_entry_point(tmp_path, parser):
    assert entry_count(tmp_path, parser, "DomainListener.java", """
        package co.fanki.app;
        public class DomainListener {
            @EventListener
            public void onEvent(Object event) {
            }
        }
        """) == 1


def test_when_parsing_given_spring_boot_application_annotation_should_detect_entry_point(tmp_path, parser):
    assert entry_count(tmp_path, parser, "App.java", """
        package co.fanki.app;
        @SpringBootApplication
        public class App {
            public static void main(String[] args) {}
        }
        """) == 1


def test_when_parsing_given_no_annotations_should_not_detect_entry_point(tmp_path, parser):
    assert entry_count(tmp_path, parser, "PlainPojo.java", """
        package co.fanki.app;
        public class PlainPojo {
            private String name;
        }
        """) == 0


def test_when_extracting_fqcn_given_nested_package_should_produce_dotted_name(tmp_path, parser):
    write(source_root(tmp_path), "co/fanki/checkout/domain", "Cart.java",
          "package co.fanki.checkout.domain;\npublic class Cart {\n}\n")
    assert parser.parse(str(tmp_path)).contains("co.fanki.checkout.domain.Cart")


def test_when_extracting_fqcn_given_root_package_file_should_produce_simple_name(tmp_path, parser):
    write(source_root(tmp_path), "", "Main.java", "public class Main {\n}\n")
    assert parser.parse(str(tmp_path)).contains("Main")


def test_when_getting_analysis_order_given_entry_points_with_deps_should_bfs_order(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Controller.java",
          "package co.fanki.app;\nimport co.fanki.app.Service;\n@RestController\npublic class Controller {\n}\n")
    write(sr, "co/fanki/app", "Service.java",
          "package co.fanki.app;\nimport co.fanki.app.Repository;\npublic class Service {\n}\n")
    write(sr, "co/fanki/app", "Repository.java", "package co.fanki.app;\npublic class Repository {\n}\n")
    order = parser.parse(str(tmp_path)).analysis_order()
    assert len(order) == 3 and order[0] == "co.fanki.app.Controller"
    assert order.index("co.fanki.app.Service") < order.index("co.fanki.app.Repository")


def test_when_parsing_given_non_java_files_should_ignore_them(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Valid.java", "package co.fanki.app;\npublic class Valid {\n}\n")
    write(sr, "co/fanki/app", "notes.txt", "This is not a Java file.")
    write(sr, "co/fanki/app", "config.xml", "<config/>")
    g = parser.parse(str(tmp_path))
    assert g.node_count() == 1 and g.contains("co.fanki.app.Valid")


# -- extractMethodParameters ---------------------------------------------------
def params_of(parser, sr, rel, known):
    return parser.extract_method_parameters(os.path.join(sr, rel), sr, set(known))


def test_when_extracting_params_given_single_internal_param_should_return_it(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "UserService.java", """
        package co.fanki.app;
        import co.fanki.app.UserRepository;
        public class UserService {
            public void findUser(UserRepository repo) {
            }
        }
        """)
    write(sr, "co/fanki/app", "UserRepository.java", "package co.fanki.app;\npublic class UserRepository {\n}\n")
    r = params_of(parser, sr, "co/fanki/app/UserService.java",
                  {"co.fanki.app.UserService", "co.fanki.app.UserRepository"})
    assert r["findUser"] == ["co.fanki.app.UserRepository"]


def order_customer(tmp_path, signature):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "OrderService.java", f"""
package co.fanki.app;
import co.fanki.app.Order;
import co.fanki.app.Customer;
public class OrderService {{
    {signature} {{
    }}
}}
""")
    write(sr, "co/fanki/app", "Order.java", "package co.fanki.app;\npublic class Order {}\n")
    write(sr, "co/fanki/app", "Customer.java", "package co.fanki.app;\npublic class Customer {}\n")
    return sr


KNOWN_OC = {"co.fanki.app.OrderService", "co.fanki.app.Order", "co.fanki.app.Customer"}


def test_when_extracting_params_given_multiple_params_should_return_all_matched(tmp_path, parser):
    sr = order_customer(tmp_path, "public void placeOrder(Order order, Customer customer, String note)")
    p = params_of(parser, sr, "co/fanki/app/OrderService.java", KNOWN_OC)["placeOrder"]
    assert len(p) == 2 and set(p) == {"co.fanki.app.Order", "co.fanki.app.Customer"}


def test_when_extracting_params_given_multiline_signature_should_resolve_params(tmp_path, parser):
    sr = order_customer(tmp_path, "public void placeOrder(\n            final Order order,\n"
                                  "            final Customer customer,\n            final String note)")
    p = params_of(parser, sr, "co/fanki/app/OrderService.java", KNOWN_OC)["placeOrder"]
    assert len(p) == 2 and set(p) == {"co.fanki.app.Order", "co.fanki.app.Customer"}


def test_when_extracting_params_given_only_external_types_should_return_empty(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Printer.java", """
        package co.fanki.app;
        public class Printer {
            public void print(String message, int count) {
            }
        }
        """)
    assert params_of(parser, sr, "co/fanki/app/Printer.java", {"co.fanki.app.Printer"}) == {}


def test_when_extracting_params_given_same_package_type_should_resolve_it(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Handler.java", """
        package co.fanki.app;
        public class Handler {
            public void handle(Event event) {
            }
        }
        """)
    write(sr, "co/fanki/app", "Event.java", "package co.fanki.app;\npublic class Event {}\n")
    r = params_of(parser, sr, "co/fanki/app/Handler.java", {"co.fanki.app.Handler", "co.fanki.app.Event"})
    assert r["handle"] == ["co.fanki.app.Event"]


def test_when_extracting_params_given_final_annotated_param_should_still_match(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Processor.java", """
        package co.fanki.app;
        import co.fanki.app.Task;
        public class Processor {
            public void process(final Task task) {
            }
        }
        """)
    write(sr, "co/fanki/app", "Task.java", "package co.fanki.app;\npublic class Task {}\n")
    r = params_of(parser, sr, "co/fanki/app/Processor.java", {"co.fanki.app.Processor", "co.fanki.app.Task"})
    assert r["process"] == ["co.fanki.app.Task"]


def test_when_extracting_params_given_method_with_no_params_should_skip_it(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "Runner.java", """
        package co.fanki.app;
        public class Runner {
            public void run() {
            }
        }
        """)
    assert params_of(parser, sr, "co/fanki/app/Runner.java", {"co.fanki.app.Runner"}) == {}


# -- inferClassType ------------------------------------------------------------
def class_type(tmp_path, parser, name, body):
    return parser.infer_class_type(write(source_root(tmp_path), "co/fanki/app", name, body))


def test_when_inferring_class_type_given_rest_controller_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "UserController.java", """
        package co.fanki.app;
        @RestController
        @RequestMapping("/api/users")
        public class UserController {
        }
        """) is ClassType.CONTROLLER


def test_when_inferring_class_type_given_controller_should_return_controller(tmp_path, parser):
    assert class_type(tmp_path, parser, "WebController.java",
                      "package co.fanki.app;\n@Controller\npublic class WebController {\n}\n") is ClassType.CONTROLLER


def test_when_inferring_class_type_given_service_annotation_should_return_service(tmp_path, parser):
    assert class_type(tmp_path, parser, "UserService.java",
                      "package co.fanki.app;\n@Service\npublic class UserService {\n}\n") is ClassType.SERVICE


def test_when_inferring_class_type_given_repository_annotation_should_return_repository(tmp_path, parser):
    assert class_type(tmp_path, parser, "UserRepository.java",
                      "package co.fanki.app;\n@Repository\npublic class UserRepository {\n}\n") is ClassType.REPOSITORY


def test_when_inferring_class_type_given_configuration_annotation_should_return_configuration(tmp_path, parser):
    assert class_type(tmp_path, parser, "AppConfig.java",
                      "package co.fanki.app;\n@Configuration\npublic class AppConfig {\n}\n") is ClassType.CONFIGURATION


def test_when_inferring_class_type_given_entity_annotation_should_return_entity(tmp_path, parser):
    assert class_type(tmp_path, parser, "User.java", """
        package co.fanki.app;
        @Entity
        public class User {
            private String id;
        }
        """) is ClassType.ENTITY


def test_when_inferring_class_type_given_kafka_listener_should_return_listener(tmp_path, parser):
    assert class_type(tmp_path, parser, "EventConsumer.java", """
        package co.fanki.app;
        public class EventConsumer {
            @KafkaListener(topics = "orders")
            public void consume(String msg) {}
        }
        """) is ClassType.LISTENER


def test_when_inferring_class_type_given_no_annotations_should_return_other(tmp_path, parser):
    assert class_type(tmp_path, parser, "PlainPojo.java", """
        package co.fanki.app;
        public class PlainPojo {
            private String name;
        }
        """) is ClassType.OTHER


# -- extractMethods ------------------------------------------------------------
def methods(tmp_path, parser, name, body):
    return parser.extract_methods(write(source_root(tmp_path), "co/fanki/app", name, body))


def test_when_extracting_methods_given_simple_class_should_return_methods_with_line_numbers(tmp_path, parser):
    ms = methods(tmp_path, parser, "UserService.java", """
        package co.fanki.app;

        public class UserService {

            public void findById(String id) {
                // implementation
            }

            public void createUser(String name) {
                // implementation
            }
        }
        """)
    assert [(m.method_name, m.line_number) for m in ms] == [("findById", 5), ("createUser", 9)]


def test_when_extracting_methods_given_get_mapping_should_extract_http_info(tmp_path, parser):
    ms = methods(tmp_path, parser, "UserController.java", """
        package co.fanki.app;

        @RestController
        public class UserController {

            @GetMapping("/users")
            public void listUsers() {
            }

            @PostMapping("/users")
            public void createUser(String name) {
            }

            @PutMapping("/users/{id}")
            public void updateUser(String id) {
            }

            @DeleteMapping("/users/{id}")
            public void deleteUser(String id) {
            }

            @PatchMapping("/users/{id}")
            public void patchUser(String id) {
            }
        }
        """)
    assert [(m.method_name, m.http_method, m.http_path) for m in ms] == [
        ("listUsers", "GET", "/users"), ("createUser", "POST", "/users"), ("updateUser", "PUT", "/users/{id}"),
        ("deleteUser", "DELETE", "/users/{id}"), ("patchUser", "PATCH", "/users/{id}")]


def test_when_extracting_methods_given_throws_clause_should_extract_exceptions(tmp_path, parser):
    ms = methods(tmp_path, parser, "OrderService.java", """
        package co.fanki.app;

        public class OrderService {

            public void placeOrder(String id) throws IllegalArgumentException, IOException {
                // implementation
            }
        }
        """)
    assert len(ms) == 1 and ms[0].method_name == "placeOrder"
    assert list(ms[0].exceptions) == ["IllegalArgumentException", "IOException"]


def test_when_extracting_methods_given_no_methods_should_return_empty(tmp_path, parser):
    assert methods(tmp_path, parser, "Constants.java", """
        package co.fanki.app;

        public class Constants {
            public static final String NAME = "fanki";
        }
        """) == []


def test_when_extracting_methods_given_method_with_no_http_annotation_should_have_null_http(tmp_path, parser):
    (m,) = methods(tmp_path, parser, "Service.java", """
        package co.fanki.app;

        public class Service {
            public void doWork() {
            }
        }
        """)
    assert m.http_method is None and m.http_path is None and not m.exceptions


def test_when_extracting_methods_given_request_mapping_should_extract_http_info(tmp_path, parser):
    (m,) = methods(tmp_path, parser, "LegacyController.java", """
        package co.fanki.app;

        @RestController
        public class LegacyController {

            @RequestMapping(value = "/api/legacy", method = RequestMethod.POST)
            public void legacyEndpoint() {
            }
        }
        """)
    assert (m.http_method, m.http_path) == ("POST", "/api/legacy")


def test_when_extracting_methods_given_multiline_throws_should_extract_exceptions(tmp_path, parser):
    (m,) = methods(tmp_path, parser, "Processor.java", """
        package co.fanki.app;

        public class Processor {

            public void process(
                    final String input)
                    throws IllegalStateException {
                // implementation
            }
        }
        """)
    assert m.method_name == "process" and list(m.exceptions) == ["IllegalStateException"]


def test_when_extracting_methods_given_generic_return_types_should_extract_correctly(tmp_path, parser):
    ms = methods(tmp_path, parser, "EventService.java", """
        package co.fanki.app;

        import java.util.List;
        import java.util.Map;
        import java.util.Optional;

        public class EventService {

            public Map<String, List<String>> getByCode(String code) {
                return null;
            }

            public Optional<Map<String, Object>> findDetails(String id) {
                return Optional.empty();
            }

            public List<String> findAll() {
                return List.of();
            }

            public void save(String name) {
            }
        }
        """)
    assert [m.method_name for m in ms] == ["getByCode", "findDetails", "findAll", "save"]


def test_when_extracting_methods_given_constructor_and_method_should_extract_both(tmp_path, parser):
    ms = methods(tmp_path, parser, "MyService.java", """
        package co.fanki.app;

        public class MyService {

            public MyService(String dependency) {
            }

            public void doWork() {
            }
        }
        """)
    assert [m.method_name for m in ms] == ["MyService", "doWork"]


def test_when_extracting_params_given_generic_return_type_should_extract_params(tmp_path, parser):
    sr = source_root(tmp_path)
    write(sr, "co/fanki/app", "OrderService.java", """
        package co.fanki.app;

        import java.util.Map;
        import java.util.List;
        import co.fanki.app.Order;

        public class OrderService {
            public Map<String, List<Order>> findOrders(Order filter) {
                return null;
            }
        }
        """)
    write(sr, "co/fanki/app", "Order.java", "package co.fanki.app;\npublic class Order {}\n")
    r = params_of(parser, sr, "co/fanki/app/OrderService.java", {"co.fanki.app.OrderService", "co.fanki.app.Order"})
    assert r["findOrders"] == ["co.fanki.app.Order"]
