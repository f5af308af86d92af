"""Incremental sync: the diff classification of every path shape and language.

Reference: ``ProjectSyncService.computeDiff`` (``:497-542``; JGit DiffEntry:
ADD/MODIFY/COPY -> changed, DELETE -> deleted, RENAME -> both) and
``syncProject`` (``:140-486``).  The reference has no sync tests at all
(SURVEY §4 coverage gaps) and no Go branch in sync (``:782-790``).
"""
import subprocess

import pytest

from conftest import make_app
from dmcp.enrich.backend import FakeBackend
from dmcp.index.git import parse_name_status_z
from dmcp.models.domain import ProjectStatus
from dmcp.utils import synth

O = "co.acme.shop.order"
U = "co.acme.shop.user"


def _git(root, *args):
    return subprocess.run(["git", "-C", str(root), *args], check=True, capture_output=True, text=True).stdout


def _commit(root, msg="change"):
    _git(root, "add", "-A")
    _git(root, "-c", "user.email=a@b", "-c", "user.name=t", "commit", "-qm", msg)


def _analyze(tmp_path, repo):
    fake = FakeBackend()
    app = make_app(tmp_path, backend=fake)
    r = app.indexer.analyze_project(str(repo))
    assert r.success
    return app, fake, r.project_id


def _sync(app, pid):
    s = app.indexer.sync_project(app.repos.projects.find_by_id(pid))
    assert s.success, s.error_message
    p = app.repos.projects.find_by_id(pid)
    assert p.status is ProjectStatus.ANALYZED and p.last_commit_hash == s.commit_hash
    return s


def test_parse_name_status_z_records():
    out = ("M\0src/a.java\0A\0src/acmé/Ñ.java\0D\0old.java\0R100\0from.java\0to.java\0"
           "R087\0x/p.java\0y/q.java\0C075\0orig.java\0copy.java\0T\0t.java\0")
    d = parse_name_status_z(out, "h")
    assert d.changed_files == {"src/a.java", "src/acmé/Ñ.java", "to.java", "y/q.java", "copy.java", "t.java"}
    assert d.deleted_files == {"old.java", "from.java", "x/p.java"}
    assert parse_name_status_z("", "h").changed_files == set()
    # a path containing a tab or newline is one token with -z
    d = parse_name_status_z("M\0we\tird\nname.java\0", "h")
    assert d.changed_files == {"we\tird\nname.java"}


def test_git_diff_reports_raw_non_ascii_paths(tmp_path):
    repo = tmp_path / "r"
    synth.java_spring_repo(str(repo), 8)
    from dmcp.index.git import GitClient
    old = _git(repo, "rev-parse", "HEAD").strip()
    d = repo / "src/main/java/co/acme/shop/acmé"
    d.mkdir(parents=True)
    (d / "Ünïcode.java").write_text("package co.acme.shop.acmé;\npublic class Ünïcode {}\n")
    _commit(repo)
    new = _git(repo, "rev-parse", "HEAD").strip()
    diff = GitClient(str(tmp_path / "c")).diff(str(repo), old, new)
    assert diff.changed_files == {"src/main/java/co/acme/shop/acmé/Ünïcode.java"}


def test_sync_modified_class_in_non_ascii_directory(tmp_path):
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 16)
    d = repo / "src/main/java/co/acme/shop/façade"
    d.mkdir(parents=True)
    (d / "Façade.java").write_text("package co.acme.shop.façade;\n\n@org.springframework.stereotype.Service\n"
                                   "public class Façade {\n    public void one() {}\n}\n")
    _commit(repo)
    app, fake, pid = _analyze(tmp_path, repo)
    (d / "Façade.java").write_text("package co.acme.shop.façade;\n\n@org.springframework.stereotype.Service\n"
                                   "public class Façade {\n    public void one() {}\n    public void two() {}\n}\n")
    _commit(repo)
    fake.calls.clear()
    s = _sync(app, pid)
    assert (s.added_classes, s.updated_classes, s.deleted_classes) == (0, 1, 0)
    assert fake.calls == ["co.acme.shop.façade.Façade"]
    names = [m.method_name for m in app.repos.methods.find_by_class_name("co.acme.shop.façade.Façade")]
    assert names == ["one", "two"]
    g = app.cache.get_graph(pid)
    assert [m.method_name for m in g.methods("co.acme.shop.façade.Façade")] == ["one", "two"]
    app.close()


def test_sync_pure_rename_R100(tmp_path):
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 16)
    app, fake, pid = _analyze(tmp_path, repo)
    base = repo / "src/main/java/co/acme/shop"
    (base / "audit").mkdir()
    # a moved file keeps its content byte for byte except the package line ->
    # git reports a high-similarity rename; the class gets a new FQCN
    src = (base / "order/OrderConfig.java").read_text()
    (base / "order/OrderConfig.java").unlink()
    (base / "audit/OrderConfig.java").write_text(src.replace("package co.acme.shop.order;",
                                                             "package co.acme.shop.audit;"))
    _commit(repo)
    assert _git(repo, "diff", "--name-status", "-M", "HEAD~1", "HEAD").startswith("R")
    fake.calls.clear()
    s = _sync(app, pid)
    assert (s.added_classes, s.updated_classes, s.deleted_classes, s.unchanged_classes) == (1, 0, 1, 16)
    assert fake.calls == ["co.acme.shop.audit.OrderConfig"]
    assert app.repos.classes.find_by_full_class_name(f"{O}.OrderConfig") is None
    assert app.repos.classes.find_by_full_class_name("co.acme.shop.audit.OrderConfig") is not None
    g = app.cache.get_graph(pid)
    assert g.contains("co.acme.shop.audit.OrderConfig") and not g.contains(f"{O}.OrderConfig")
    app.close()


def test_sync_partial_rename_same_class_name(tmp_path):
    """Rename with edits where the FQCN does not change (file moved between
    source roots would change it; here only the file name changes) -- the
    class is an update, not a delete + add: it keeps its id."""
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 16)
    app, fake, pid = _analyze(tmp_path, repo)
    base = repo / "src/main/java/co/acme/shop/user"
    old_id = app.repos.classes.find_by_full_class_name(f"{U}.UserService").id
    text = (base / "UserService.java").read_text()
    _git(repo, "mv", "src/main/java/co/acme/shop/user/UserService.java",
         "src/main/java/co/acme/shop/user/UserServiceImpl.java")
    (base / "UserServiceImpl.java").write_text(
        text.replace("public class UserService {", "public class UserServiceImpl {\n    public void extra() {}\n"))
    _commit(repo)
    fake.calls.clear()
    s = _sync(app, pid)
    # the Java identifier follows the file path: UserService -> UserServiceImpl
    assert s.added_classes == 1 and s.deleted_classes == 1
    assert fake.calls == [f"{U}.UserServiceImpl"]
    assert app.repos.classes.find_by_id(old_id) is None
    ids = app.repos.classes.find_by_full_class_name(f"{U}.UserServiceImpl")
    assert "extra" in [m.method_name for m in app.repos.methods.find_by_class_id(ids.id)]
    app.close()


def test_sync_deleted_class_that_is_a_parameter_type_of_an_unchanged_class(tmp_path):
    repo = tmp_path / "shop"
    synth.java_spring_repo(str(repo), 16)
    base = repo / "src/main/java/co/acme/shop/order"
    (base / "Coupon.java").write_text("package co.acme.shop.order;\n\npublic class Coupon {\n}\n")
    (base / "Pricing.java").write_text(
        "package co.acme.shop.order;\n\n@org.springframework.stereotype.Service\npublic class Pricing {\n"
        "    public long price(Coupon c, OrderRequest r) { return 0; }\n}\n")
    _commit(repo)
    app, fake, pid = _analyze(tmp_path, repo)
    ctx = app.context.get_method_context(f"{O}.Pricing", "price")
    assert [p["typeName"] for p in ctx["parameterTypes"]] == [f"{O}.Coupon", f"{O}.OrderRequest"]
    (base / "Coupon.java").unlink()  # Pricing.java itself does not change
    _commit(repo)
    s = _sync(app, pid)
    assert s.deleted_classes == 1 and s.updated_classes == 0
    # the link to the deleted class is gone from the DB and from the graph; the other stays
    ctx = app.context.get_method_context(f"{O}.Pricing", "price")
    assert [p["typeName"] for p in ctx["parameterTypes"]] == [f"{O}.OrderRequest"]
    g = app.cache.get_graph(pid)
    assert f"{O}.Coupon" not in [t for ts in g.method_parameters(f"{O}.Pricing").values() for t in ts]
    n = app.db.query_one("SELECT COUNT(*) FROM method_parameters mp JOIN source_classes c ON c.id = mp.class_id "
                         "WHERE c.full_class_name = ?", (f"{O}.Coupon",))[0]
    assert n == 0
    app.close()


def test_sync_typescript_project(tmp_path):
    repo = tmp_path / "svc"
    synth.nestjs_repo(str(repo), n_modules=4)
    app, fake, pid = _analyze(tmp_path, repo)
    before = app.repos.classes.count_by_project()[pid]
    svc = repo / "src/order/order.service.ts"
    svc.write_text(svc.read_text().replace("  findAll = async", "  async cancel(id: string): Promise<void> {}\n\n"
                                                                 "  findAll = async"))
    (repo / "src/user/user.entity.ts").unlink()
    (repo / "src/audit.ts").write_text("export function audit(x: string) { return x; }\n")
    _commit(repo)
    fake.calls.clear()
    s = _sync(app, pid)
    assert (s.added_classes, s.updated_classes, s.deleted_classes) == (1, 1, 1), s.to_dict()
    assert sorted(fake.calls) == ["audit", "order.order.service"]
    assert app.repos.classes.count_by_project()[pid] == before
    names = [m.method_name for m in app.repos.methods.find_by_class_name("order.order.service")]
    assert "cancel" in names
    g = app.cache.get_graph(pid)
    assert g.contains("audit") and not g.contains("user.user.entity")
    app.close()


def test_sync_go_project(tmp_path):
    repo = tmp_path / "gosvc"
    mod = "github.com/acme/gosvc"
    synth.go_gin_repo(str(repo), n_packages=3, module=mod)
    app, fake, pid = _analyze(tmp_path, repo)
    svc = repo / "internal/orderservice/service.go"
    svc.write_text(svc.read_text() + "\n// Cancel drops one order.\nfunc (s *Service) Cancel(id string) {}\n")
    (repo / "internal/audit").mkdir()
    (repo / "internal/audit/audit.go").write_text("package audit\n\n// Record logs.\nfunc Record(x string) {}\n")
    _commit(repo)
    fake.calls.clear()
    s = _sync(app, pid)
    # a Go identifier is the package: the changed file updates its package
    assert (s.added_classes, s.updated_classes, s.deleted_classes) == (1, 1, 0), s.to_dict()
    assert sorted(fake.calls) == [f"{mod}/internal/audit", f"{mod}/internal/orderservice"]
    names = [m.method_name for m in app.repos.methods.find_by_class_name(f"{mod}/internal/orderservice")]
    assert "Service.Cancel" in names
    # deleting a whole package deletes its node
    subprocess.run(["rm", "-r", str(repo / "internal/audit")], check=True)
    _commit(repo)
    s = _sync(app, pid)
    assert s.deleted_classes == 1 and not app.cache.get_graph(pid).contains(f"{mod}/internal/audit")
    app.close()
