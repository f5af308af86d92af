"""Java front-end (JavaSourceParserTest in the reference): identifiers,
import dependencies, entry points, class types, methods / HTTP mappings /
throws / line numbers and method-parameter resolution."""
import os
import textwrap

import pytest

from dmcp.models.domain import ClassType
from dmcp.parsers.base import JavaSourceParser, native

SRC = "src/main/java"


def write(root, pkg, name, body):
    d = os.path.join(root, SRC, *pkg.split(".")) if pkg else os.path.join(root, SRC)
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, name)
    with open(p, "w") as f:
        f.write(textwrap.dedent(body).lstrip("\n"))
    return p


@pytest.fixture
def parser():
    return JavaSourceParser()


def test_multi_file_graph(tmp_path, parser):
    r = str(tmp_path)
    write(r, "co.fanki.app", "Application.java", """
        package co.fanki.app;
        @SpringBootApplication
        public class Application { public static void main(String[] args) {} }
        """)
    write(r, "co.fanki.app.controller", "UserController.java", """
        package co.fanki.app.controller;
        import co.fanki.app.service.UserService;
        @RestController
        public class UserController { private final UserService s; }
        """)
    write(r, "co.fanki.app.service", "UserService.java", """
        package co.fanki.app.service;
        import co.fanki.app.domain.User;
        import java.util.List;
        @Service
        public class UserService { List<User> all() { return null; } }
        """)
    write(r, "co.fanki.app.domain", "User.java", "package co.fanki.app.domain;\npublic class User {}\n")
    g = parser.parse(r)
    assert g.node_count() == 4 and g.entry_point_count() == 2
    assert g.dependencies("co.fanki.app.controller.UserController") == ("co.fanki.app.service.UserService",)
    assert g.dependencies("co.fanki.app.service.UserService") == ("co.fanki.app.domain.User",)
    assert g.source_file("co.fanki.app.domain.User") == "src/main/java/co/fanki/app/domain/User.java"
    order = g.analysis_order()
    assert order.index("co.fanki.app.service.UserService") < order.index("co.fanki.app.domain.User")


def test_empty_and_missing_roots(tmp_path, parser):
    os.makedirs(tmp_path / SRC)
    assert parser.parse(str(tmp_path)).node_count() == 0
    assert JavaSourceParser().parse(str(tmp_path / "nope")).node_count() == 0
    with pytest.raises(ValueError):
        parser.parse(None)


def test_imports_internal_static_and_after_class(tmp_path, parser):
    r = str(tmp_path)
    write(r, "co.fanki.app", "MyRepository.java", "package co.fanki.app;\npublic class MyRepository {}\n")
    write(r, "co.fanki.app", "Constants.java", "package co.fanki.app;\npublic class Constants { "
                                                 "public static final int MAX = 1; }\n")
    write(r, "co.fanki.app", "Ignored.java", "package co.fanki.app;\npublic class Ignored {}\n")
    write(r, "co.fanki.app.svc", "Svc.java", """
        package co.fanki.app.svc;
        import co.fanki.app.MyRepository;
        import static co.fanki.app.Constants.MAX;
        import java.util.List;
        import org.springframework.stereotype.Service;
        import co.fanki.app.*;
        public class Svc {
            String s = "import co.fanki.app.Ignored;";
        }
        // import co.fanki.app.Ignored;
        """)
    g = parser.parse(r)
    assert set(g.dependencies("co.fanki.app.svc.Svc")) == {"co.fanki.app.MyRepository", "co.fanki.app.Constants"}


@pytest.mark.parametrize("annotation,entry,ctype", [
    ("@RestController", True, ClassType.CONTROLLER), ("@Controller", True, ClassType.CONTROLLER),
    ("@Service", False, ClassType.SERVICE), ("@Repository", False, ClassType.REPOSITORY),
    ("@Configuration", False, ClassType.CONFIGURATION), ("@Entity", False, ClassType.ENTITY),
    ("@SpringBootApplication", True, ClassType.OTHER), ("", False, ClassType.OTHER),
    ("@org.springframework.web.bind.annotation.RestController", True, ClassType.CONTROLLER)])
def test_class_annotations(tmp_path, parser, annotation, entry, ctype):
    f = write(str(tmp_path), "co.fanki.app", "X.java", f"package co.fanki.app;\n{annotation}\npublic class X {{}}\n")
    parser.scan(str(tmp_path))
    assert parser.is_entry_point(f) == entry and parser.infer_class_type(f) is ctype


@pytest.mark.parametrize("method_annotation", ["@KafkaListener(topics = \"t\")", "@EventListener", "@Scheduled(cron = \"0 * * * * *\")"])
def test_method_level_entry_points(tmp_path, parser, method_annotation):
    f = write(str(tmp_path), "co.fanki.app", "L.java", f"""
        package co.fanki.app;
        public class L {{
            {method_annotation}
            public void consume(String message) {{}}
        }}
        """)
    parser.scan(str(tmp_path))
    assert parser.is_entry_point(f)
    expected = ClassType.OTHER if "Scheduled" in method_annotation else ClassType.LISTENER
    assert parser.infer_class_type(f) is expected


def test_fqcn_nested_and_root_package(tmp_path, parser):
    write(str(tmp_path), "co.fanki.checkout.domain", "Cart.java", "package co.fanki.checkout.domain;\nclass Cart {}\n")
    write(str(tmp_path), "", "Main.java", "public class Main {}\n")
    (tmp_path / SRC / "notes.txt").write_text("not java")
    g = parser.parse(str(tmp_path))
    assert g.contains("co.fanki.checkout.domain.Cart") and g.contains("Main") and g.node_count() == 2


def test_methods_lines_http_throws(tmp_path, parser):
    f = write(str(tmp_path), "co.fanki.app", "UserController.java", """
        package co.fanki.app;

        @RestController
        public class UserController {

            public UserController(String dep) {
            }

            @GetMapping("/users")
            public void listUsers() {
            }

            @PostMapping(value = "/users")
            public void createUser(String name) throws IllegalArgumentException, java.io.IOException {
            }

            @PutMapping(path = "/users/{id}")
            public void updateUser(String id) {
            }

            @DeleteMapping("/users/{id}")
            public void deleteUser(String id) {
            }

            @PatchMapping("/users/{id}")
            public void patchUser(String id) {
            }

            @RequestMapping(value = "/api/legacy", method = RequestMethod.POST)
            public void legacy() {
            }

            @RequestMapping("/default")
            public java.util.Map<String, java.util.List<String>> byCode(
                    final String code)
                    throws IllegalStateException {
                return null;
            }

            private void helper() {}
        }
        """)
    parser.scan(str(tmp_path))
    ms = parser.extract_methods(f)
    got = [(m.method_name, m.http_method, m.http_path, list(m.exceptions)) for m in ms]
    assert got == [
        ("UserController", None, None, []),
        ("listUsers", "GET", "/users", []),
        ("createUser", "POST", "/users", ["IllegalArgumentException", "java.io.IOException"]),
        ("updateUser", "PUT", "/users/{id}", []),
        ("deleteUser", "DELETE", "/users/{id}", []),
        ("patchUser", "PATCH", "/users/{id}", []),
        ("legacy", "POST", "/api/legacy", []),
        ("byCode", "GET", "/default", ["IllegalStateException"]),
        ("helper", None, None, []),
    ]
    # JavaParser's node range starts at the first annotation
    assert [m.line_number for m in ms[:3]] == [6, 9, 13]


def test_records_and_interfaces(tmp_path, parser):
    f = write(str(tmp_path), "co.fanki.app", "Money.java", """
        package co.fanki.app;
        public record Money(long cents, String currency) {
            public Money {
                if (cents < 0) throw new IllegalArgumentException();
            }
            public Money plus(Money other) { return new Money(cents + other.cents, currency); }
        }
        """)
    g = write(str(tmp_path), "co.fanki.app", "Point.java", """
        package co.fanki.app;
        public record Point(int x, int y) {
            public Point(int x, int y) { this.x = x; this.y = y; }
            public int sum() { return x + y; }
            class Nested { void hidden() {} }
        }
        """)
    parser.scan(str(tmp_path))
    # compact canonical constructors are not ConstructorDeclarations in
    # JavaParser (reference: recordDecl.getConstructors()); explicit ones are
    assert [m.method_name for m in parser.extract_methods(f)] == ["plus"]
    assert [m.method_name for m in parser.extract_methods(g)] == ["Point", "sum"]
    assert parser.extract_method_parameters(f) == {"plus": ["co.fanki.app.Money"]}


def test_method_parameters(tmp_path, parser):
    r = str(tmp_path)
    for n in ("UserRepository", "Order", "Customer", "Task"):
        write(r, "co.fanki.app", f"{n}.java", f"package co.fanki.app;\npublic class {n} {{}}\n")
    write(r, "co.fanki.app.events", "Event.java", "package co.fanki.app.events;\npublic class Event {}\n")
    f = write(r, "co.fanki.app", "Svc.java", """
        package co.fanki.app;
        import co.fanki.app.events.Event;
        import java.util.List;
        public class Svc {
            public void findUser(UserRepository repo) {}
            public void placeOrder(
                    Order order,
                    Customer customer, String note) {}
            public void print(String message, int count) {}
            public void handle(Event event) {}
            public void process(final @Valid Task task) {}
            public List<Order> batch(List<Order> orders, Task... tasks) { return orders; }
            public void run() {}
        }
        """)
    parser.scan(r)
    params = parser.extract_method_parameters(f)
    assert params["findUser"] == ["co.fanki.app.UserRepository"]
    assert params["placeOrder"] == ["co.fanki.app.Order", "co.fanki.app.Customer"]
    assert params["handle"] == ["co.fanki.app.events.Event"]
    assert params["process"] == ["co.fanki.app.Task"]
    # generics are stripped to the raw type (List -> unknown), varargs to the element type
    assert params["batch"] == ["co.fanki.app.Task"]
    assert "print" not in params and "run" not in params
    known = {"co.fanki.app.Order"}
    assert parser.extract_method_parameters(f, known_identifiers=known) == {
        "placeOrder": ["co.fanki.app.Order"]}


def test_tricky_syntax_does_not_confuse_the_lexer(tmp_path, parser):
    f = write(str(tmp_path), "co.fanki.app", "Tricky.java", '''
        package co.fanki.app;
        /* public void commented() {} */
        public class Tricky {
            String block = """
                public void inTextBlock() {}
                """;
            char c = '{';
            String s = "}{ \\" public void inString() {}";
            @GetMapping({"/a", "/b"})
            public <T extends Comparable<T>> T max(T a, T b) { return a; }
            class Inner { void innerMethod() {} }
            public void after() { Runnable r = () -> { }; }
        }
        ''')
    parser.scan(str(tmp_path))
    names = [m.method_name for m in parser.extract_methods(f)]
    assert "commented" not in names and "inTextBlock" not in names and "inString" not in names
    assert "max" in names and "after" in names


def test_native_scan_file_and_stats(tmp_path):
    write(str(tmp_path), "co.x", "A.java", "package co.x;\n@Service\npublic class A { void a() {} }\n")
    import json
    doc = json.loads(native().scan_project(str(tmp_path), "java", 2, ""))
    assert doc["language"] == "java" and doc["sourceRoot"] == "src/main/java"
    assert doc["stats"]["discovered"] == 1 and doc["stats"]["analyzed"] == 1
    one = json.loads(native().scan_file(str(tmp_path / SRC / "co/x/A.java"), "java", "co/x/A.java"))
    assert one["identifier"] == "co.x.A" and one["classType"] == "SERVICE"
