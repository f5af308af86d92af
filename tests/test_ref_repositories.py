"""One test per case of the reference's repository integration tests.

Mirrors ``project/domain/ProjectRepositoryIntegrationTest.java`` (9),
``analysis/domain/SourceClassRepositoryIntegrationTest.java`` (9) and
``analysis/domain/SourceMethodRepositoryIntegrationTest.java`` (11) (under
``src/test/java/co/fanki/domainmcp/``).  The reference runs them against a
Testcontainers ``postgres:14`` with Flyway V1-V8; here every case runs twice:
on a fresh SQLite file with the same final schema (``dmcp/store/db.py``) and
on the PostgreSQL store (``dmcp/store/pg.py``) over the wire protocol, served
by ``tests/pgfake.py``.  Unlike the reference's (CI-excluded) integration
tests, these run on every CPU pass.
"""
import pytest

from dmcp.models.domain import ClassType, Project, ProjectStatus, RepositoryUrl, SourceClass, SourceMethod
from dmcp.store.db import Database
from dmcp.store.repositories import Repositories


@pytest.fixture(params=["sqlite", "postgres"])
def repos(request, tmp_path):
    if request.param == "sqlite":
        db = Database(str(tmp_path / "repo.db"))
        yield Repositories(db)
        db.close()
        return
    from dmcp.store.pg import PgDatabase
    from tests.pgfake import FakePgServer
    with FakePgServer(str(tmp_path / "pg.sqlite"), auth="md5") as srv:
        db = PgDatabase.from_url(srv.url())
        yield Repositories(db)
        db.close()


def new_project(name="Test Project", url="https://github.com/test/repo.git"):
    return Project.create(name, RepositoryUrl.of(url))


# ====================== ProjectRepositoryIntegrationTest =======================
def test_when_saving_project_given_valid_project_should_persist(repos):
    p = new_project()
    repos.projects.save(p)
    found = repos.projects.find_by_id(p.id)
    assert found is not None and found.name == p.name


def test_when_finding_by_url_given_existing_url_should_return_project(repos):
    p = new_project()
    repos.projects.save(p)
    assert repos.projects.find_by_repository_url(p.repository_url).id == p.id


def test_when_finding_by_url_given_non_existing_url_should_return_empty(repos):
    assert repos.projects.find_by_repository_url(RepositoryUrl.of("https://github.com/nonexistent/repo.git")) is None


def test_when_updating_project_given_existing_project_should_update_fields(repos):
    p = new_project()
    repos.projects.save(p)
    p.start_analysis()
    p.analysis_completed("abc123")
    repos.projects.update(p)
    found = repos.projects.find_by_id(p.id)
    assert found.status is ProjectStatus.ANALYZED and found.last_analyzed_at is not None
    assert found.last_commit_hash == "abc123"


def test_when_finding_all_given_multiple_projects_should_return_all(repos):
    repos.projects.save(new_project())
    repos.projects.save(new_project("Project 2", "https://github.com/test/repo2.git"))
    assert len(repos.projects.find_all()) == 2


def test_when_finding_by_status_given_matching_status_should_return_filtered(repos):
    pending = new_project()
    repos.projects.save(pending)
    analyzed = new_project("Analyzed", "https://github.com/test/analyzed.git")
    analyzed.start_analysis()
    analyzed.analysis_completed("def456")
    repos.projects.save(analyzed)
    assert [p.id for p in repos.projects.find_by_status(ProjectStatus.PENDING)] == [pending.id]


def test_when_deleting_project_given_existing_project_should_remove(repos):
    p = new_project()
    repos.projects.save(p)
    repos.projects.delete(p.id)
    assert repos.projects.find_by_id(p.id) is None


def test_when_checking_exists_given_existing_url_should_return_true(repos):
    p = new_project()
    repos.projects.save(p)
    assert repos.projects.exists_by_repository_url(p.repository_url)


def test_when_checking_exists_given_non_existing_url_should_return_false(repos):
    assert not repos.projects.exists_by_repository_url(RepositoryUrl.of("https://github.com/nonexistent/repo.git"))


# =================== SourceClassRepositoryIntegrationTest =====================
@pytest.fixture
def project(repos):
    p = new_project()
    repos.projects.save(p)
    return p


def new_class(project, fqcn):
    return SourceClass.create(project.id, fqcn, ClassType.SERVICE, "Test class description",
                              "src/main/java/" + fqcn.replace(".", "/") + ".java", "abc123")


def test_when_saving_class_given_valid_class_should_persist(repos, project):
    sc = new_class(project, "co.fanki.user.UserService")
    repos.classes.save(sc)
    found = repos.classes.find_by_id(sc.id)
    assert found.full_class_name == sc.full_class_name and found.class_type is ClassType.SERVICE


def test_when_finding_by_full_class_name_given_existing_class_should_return(repos, project):
    sc = new_class(project, "co.fanki.user.UserService")
    repos.classes.save(sc)
    assert repos.classes.find_by_full_class_name("co.fanki.user.UserService").id == sc.id


def test_when_finding_by_full_class_name_given_non_existing_should_return_empty(repos, project):
    assert repos.classes.find_by_full_class_name("co.fanki.nonexistent.Class") is None


def test_when_finding_by_project_id_given_project_with_classes_should_return_all(repos, project):
    for n in ("co.fanki.user.UserService", "co.fanki.user.UserController", "co.fanki.order.OrderService"):
        repos.classes.save(new_class(project, n))
    assert len(repos.classes.find_by_project_id(project.id)) == 3


def test_when_finding_by_package_prefix_given_matching_package_should_return_filtered(repos, project):
    for n in ("co.fanki.user.UserService", "co.fanki.user.UserController", "co.fanki.order.OrderService"):
        repos.classes.save(new_class(project, n))
    assert len(repos.classes.find_by_package_prefix("co.fanki.user")) == 2


def test_when_counting_by_project_id_given_classes_exist_should_return_count(repos, project):
    repos.classes.save(new_class(project, "co.fanki.user.UserService"))
    repos.classes.save(new_class(project, "co.fanki.user.UserController"))
    assert repos.classes.count_by_project_id(project.id) == 2


def test_when_saving_all_given_multiple_classes_should_persist_all(repos, project):
    repos.classes.save_all([new_class(project, n) for n in (
        "co.fanki.user.UserService", "co.fanki.user.UserController", "co.fanki.order.OrderService")])
    assert repos.classes.count_by_project_id(project.id) == 3


def test_when_deleting_by_project_id_given_classes_exist_should_remove_all(repos, project):
    repos.classes.save(new_class(project, "co.fanki.user.UserService"))
    repos.classes.save(new_class(project, "co.fanki.user.UserController"))
    repos.classes.delete_by_project_id(project.id)
    assert repos.classes.count_by_project_id(project.id) == 0


def test_when_deleting_given_existing_class_should_remove(repos, project):
    sc = new_class(project, "co.fanki.user.UserService")
    repos.classes.save(sc)
    repos.classes.delete(sc.id)
    assert repos.classes.find_by_id(sc.id) is None


# ================== SourceMethodRepositoryIntegrationTest =====================
@pytest.fixture
def cls(repos, project):
    sc = SourceClass.create(project.id, "co.fanki.user.UserService", ClassType.SERVICE, "User service",
                            "src/main/java/co/fanki/user/UserService.java", "abc123")
    repos.classes.save(sc)
    return sc


def method(cls, name, verb=None, path=None, desc="Test method description"):
    return SourceMethod.create(cls.id, name, desc if verb is None else "HTTP endpoint", None, None, verb, path, None)


def test_when_saving_method_given_valid_method_should_persist(repos, cls):
    m = method(cls, "createUser")
    repos.methods.save(m)
    assert repos.methods.find_by_id(m.id).method_name == "createUser"


def test_when_saving_method_given_business_logic_list_should_persist_and_retrieve(repos, cls):
    m = SourceMethod.create(cls.id, "createUser", "Creates a new user",
                            ["Validates input", "Saves to DB", "Publishes event"], ["ValidationException"],
                            "POST", "/api/users", 45)
    repos.methods.save(m)
    found = repos.methods.find_by_id(m.id)
    assert len(found.business_logic) == 3 and found.business_logic[0] == "Validates input"
    assert len(found.exceptions) == 1


def test_when_finding_by_class_id_given_methods_exist_should_return_all(repos, cls):
    for n in ("createUser", "updateUser", "deleteUser"):
        repos.methods.save(method(cls, n))
    assert len(repos.methods.find_by_class_id(cls.id)) == 3


def test_when_finding_by_class_name_given_methods_exist_should_return_all(repos, cls):
    repos.methods.save(method(cls, "createUser"))
    repos.methods.save(method(cls, "updateUser"))
    assert len(repos.methods.find_by_class_name("co.fanki.user.UserService")) == 2


def test_when_finding_by_class_name_and_method_name_given_exists_should_return(repos, cls):
    repos.methods.save(method(cls, "createUser"))
    found = repos.methods.find_by_class_name_and_method_name("co.fanki.user.UserService", "createUser")
    assert found is not None and found.method_name == "createUser"


def test_when_finding_by_class_name_and_method_name_given_not_exists_should_return_empty(repos, cls):
    assert repos.methods.find_by_class_name_and_method_name("co.fanki.user.UserService", "nonExistent") is None


def test_when_finding_http_endpoints_given_endpoints_exist_should_return_filtered(repos, project, cls):
    repos.methods.save(method(cls, "create", "POST", "/api/users"))
    repos.methods.save(method(cls, "list", "GET", "/api/users"))
    repos.methods.save(method(cls, "helper"))
    assert len(repos.methods.find_http_endpoints_by_project_id(project.id)) == 2


def test_when_counting_endpoints_given_endpoints_exist_should_return_count(repos, project, cls):
    repos.methods.save(method(cls, "create", "POST", "/api/users"))
    repos.methods.save(method(cls, "list", "GET", "/api/users"))
    repos.methods.save(method(cls, "helper"))
    assert repos.methods.count_endpoints_by_project_id(project.id) == 2


def test_when_saving_all_given_multiple_methods_should_persist_all(repos, cls):
    repos.methods.save_all([method(cls, n) for n in ("createUser", "updateUser", "deleteUser")])
    assert len(repos.methods.find_by_class_id(cls.id)) == 3


def test_when_deleting_given_existing_method_should_remove(repos, cls):
    m = method(cls, "createUser")
    repos.methods.save(m)
    repos.methods.delete(m.id)
    assert repos.methods.find_by_id(m.id) is None


def test_when_deleting_by_class_id_given_methods_exist_should_remove_all(repos, cls):
    repos.methods.save(method(cls, "createUser"))
    repos.methods.save(method(cls, "updateUser"))
    repos.methods.delete_by_class_id(cls.id)
    assert repos.methods.find_by_class_id(cls.id) == []


def test_deleting_a_class_cascades_to_its_methods(repos, cls):
    """FK ``ON DELETE CASCADE`` (``V1__initial_schema.sql:168-184``)."""
    m = method(cls, "createUser")
    repos.methods.save(m)
    repos.classes.delete(cls.id)
    assert repos.methods.find_by_id(m.id) is None
