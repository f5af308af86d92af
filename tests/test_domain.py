"""Domain model behaviours (PreconditionsTest, RepositoryUrlTest, ProjectTest,
ProjectStateMachineTest, ClassTypeTest, SourceClassTest, SourceMethodTest,
MethodParameterTest in the reference)."""
import pytest

from dmcp.models.domain import (ClassType, GitDiffResult, MethodParameter, Project, ProjectStatus, RepositoryUrl,
                                SourceClass, SourceMethod, StaticMethodInfo, allowed_transitions, transition)
from dmcp.utils.errors import (DomainError, require, require_domain, require_non_blank, require_non_negative,
                               require_non_null, require_positive)


# ------------------------------------------------------------------ guards
def test_preconditions():
    assert require_non_null("x", "m") == "x"
    with pytest.raises(ValueError, match="boom"):
        require_non_null(None, "boom")
    assert require_non_blank(" a ", "m") == " a "
    for bad in (None, "", "   "):
        with pytest.raises(ValueError):
            require_non_blank(bad, "m")
    require(True, "m")
    with pytest.raises(ValueError):
        require(False, "m")
    with pytest.raises(DomainError) as e:
        require_domain(False, "rule")
    assert e.value.error_code == "DOMAIN_ERROR"
    assert require_positive(1, "m") == 1
    with pytest.raises(ValueError):
        require_positive(0, "m")
    assert require_non_negative(0, "m") == 0
    with pytest.raises(ValueError):
        require_non_negative(-1, "m")


def test_domain_error_code():
    e = DomainError("msg", "CODE")
    assert str(e) == "msg" and e.error_code == "CODE"
    assert DomainError("m").error_code == "DOMAIN_ERROR"


# ----------------------------------------------------------- RepositoryUrl
def test_repository_url_https_and_ssh():
    u = RepositoryUrl.of("https://github.com/example/repo.git")
    assert u.value == "https://github.com/example/repo.git" and u.is_https() and not u.is_ssh()
    s = RepositoryUrl.of("git@github.com:example/my-project.git")
    assert s.is_ssh() and not s.is_https()
    assert s.repository_name() == "my-project"
    assert RepositoryUrl.of("https://github.com/example/my-project.git").repository_name() == "my-project"


def test_repository_url_invalid():
    for bad in ("not-a-valid-url", "  ", "http://github.com/x/y.git", "https://github.com/x/y"):
        with pytest.raises(ValueError):
            RepositoryUrl.of(bad)


def test_repository_url_equality_and_local():
    a = RepositoryUrl.of("https://github.com/example/repo.git")
    assert a == RepositoryUrl.of("https://github.com/example/repo.git") and hash(a) == hash(RepositoryUrl.of(a.value))
    loc = RepositoryUrl.of("/srv/git/shop")
    assert loc.is_local() and loc.local_path() == "/srv/git/shop" and loc.repository_name() == "shop"
    f = RepositoryUrl.of("file:///srv/git/orders.git")
    assert f.local_path() == "/srv/git/orders.git" and f.repository_name() == "orders"


# ------------------------------------------------------------ state machine
@pytest.mark.parametrize("frm,to,ok", [
    ("PENDING", "ANALYZING", True), ("PENDING", "ANALYZED", False), ("PENDING", "SYNCING", False),
    ("ANALYZING", "ANALYZED", True), ("ANALYZING", "ERROR", True), ("ANALYZING", "ANALYZING", False),
    ("ANALYZED", "ANALYZING", True), ("ANALYZED", "SYNCING", True), ("ANALYZED", "ERROR", False),
    ("SYNCING", "ANALYZED", True), ("SYNCING", "ERROR", True), ("SYNCING", "PENDING", False),
    ("ERROR", "ANALYZING", True), ("ERROR", "SYNCING", True), ("ERROR", "ANALYZED", False)])
def test_transitions(frm, to, ok):
    f, t = ProjectStatus(frm), ProjectStatus(to)
    if ok:
        assert transition(f, t) is t
    else:
        with pytest.raises(DomainError) as e:
            transition(f, t)
        assert e.value.error_code == "PROJECT_INVALID_TRANSITION"
    assert (t in allowed_transitions(f)) == ok


def test_is_processing():
    assert ProjectStatus.ANALYZING.is_processing() and ProjectStatus.SYNCING.is_processing()
    assert not ProjectStatus.ANALYZED.is_processing()


# ------------------------------------------------------------------ Project
def test_project_lifecycle():
    p = Project.create("shop", RepositoryUrl.of("https://github.com/a/shop.git"))
    assert p.status is ProjectStatus.PENDING and p.default_branch == "main" and p.last_analyzed_at is None
    p.start_analysis()
    assert p.status is ProjectStatus.ANALYZING
    p.analysis_completed("abc123")
    assert p.status is ProjectStatus.ANALYZED and p.last_commit_hash == "abc123" and p.last_analyzed_at
    p.start_sync()
    p.sync_completed("def456")
    assert p.last_commit_hash == "def456" and p.status is ProjectStatus.ANALYZED
    with pytest.raises(ValueError):
        p.start_analysis() or p.analysis_completed("  ")


def test_project_error_and_recovery():
    p = Project.create("x", RepositoryUrl.of("https://github.com/a/x.git"), "develop")
    assert p.default_branch == "develop"
    p.start_analysis()
    assert p.recover_stuck() and p.status is ProjectStatus.ERROR
    p.start_sync()
    p.mark_error()
    p.start_analysis()
    with pytest.raises(DomainError):
        Project.create("y", RepositoryUrl.of("https://github.com/a/y.git")).mark_error()


def test_project_mutators():
    p = Project.create("x", RepositoryUrl.of("https://github.com/a/x.git"))
    p.update_description("desc")
    p.update_graph_data("{}")
    p.rename("z")
    assert (p.description, p.graph_data, p.name) == ("desc", "{}", "z")
    with pytest.raises(ValueError):
        p.rename(" ")


# -------------------------------------------------------------- ClassType
def test_class_type_from_string():
    assert ClassType.from_string("controller") is ClassType.CONTROLLER
    assert ClassType.from_string(" Service ") is ClassType.SERVICE
    for bad in (None, "", "  ", "nonsense"):
        assert ClassType.from_string(bad) is ClassType.OTHER
    assert ClassType.CONTROLLER.is_request_handler() and ClassType.LISTENER.is_request_handler()
    assert ClassType.SERVICE.contains_business_logic() and not ClassType.DTO.contains_business_logic()
    assert ClassType.DTO.description == "Data Transfer Object"
    assert len(ClassType) == 10


# ------------------------------------------------------- class / method rows
def test_source_class():
    c = SourceClass.create("p1", "co.fanki.user.UserService", ClassType.SERVICE, None, "src/x.java", "h")
    assert c.simple_name == "UserService" and c.package_name == "co.fanki.user"
    assert c.belongs_to_package("co.fanki") and c.belongs_to_package("co.fanki.user")
    assert not c.belongs_to_package("co.fank") and not c.belongs_to_package(None)
    d = SourceClass.create("p1", "Main", ClassType.OTHER, None, None, None)
    assert d.simple_name == "Main" and d.package_name is None
    with pytest.raises(ValueError):
        SourceClass.create("p1", " ", ClassType.OTHER, None, None, None)


def test_source_method_endpoint():
    m = SourceMethod.create("c1", "createUser", None, None, ["E"], "POST", "/users", 10)
    assert m.is_http_endpoint() and m.http_endpoint() == "POST /users"
    assert m.business_logic == () and m.exceptions == ("E",)
    n = SourceMethod.create("c1", "x", None, None, None, "GET", None, None)
    assert not n.is_http_endpoint() and n.http_endpoint() is None
    with pytest.raises(ValueError):
        SourceMethod.create("c1", "", None, None, None, None, None, None)


def test_method_parameter():
    p = MethodParameter.create("m1", 0, "c1")
    assert p.position == 0 and p.id
    with pytest.raises(ValueError):
        MethodParameter.create("m1", -1, "c1")
    with pytest.raises(ValueError):
        MethodParameter.create("m1", 0, "")


def test_static_method_info_and_diff():
    s = StaticMethodInfo.simple("run", 3)
    assert s.http_method is None and s.exceptions == ()
    full = GitDiffResult.full_resync("h")
    assert full.is_affected("anything")
    d = GitDiffResult.of("h", {"a.java"}, {"b.java"})
    assert d.is_affected("a.java") and d.is_affected("b.java") and not d.is_affected("c.java")
