"""One test per case of the reference's domain unit tests (95 cases).

Mirrors, case by case:
``shared/PreconditionsTest.java`` (13), ``project/domain/RepositoryUrlTest.java`` (7),
``project/domain/ProjectTest.java`` (14), ``project/domain/ProjectStateMachineTest.java`` (16),
``analysis/domain/ClassTypeTest.java`` (12), ``SourceClassTest.java`` (11),
``SourceMethodTest.java`` (12), ``MethodParameterTest.java`` (10)
(all under ``src/test/java/co/fanki/domainmcp/``).  ``IllegalArgumentException``
maps to ``ValueError``; ``DomainException`` to :class:`DomainError`.
"""
from datetime import datetime, timedelta, timezone

import pytest

from dmcp.models.domain import (ClassType, MethodParameter, Project, ProjectStatus, RepositoryUrl,
                                SourceClass, SourceMethod, new_id, transition)
from dmcp.utils.errors import (DomainError, require, require_domain, require_non_blank, require_non_negative,
                               require_non_null, require_positive)

S = ProjectStatus


# =========================== PreconditionsTest ================================
def test_when_require_non_null_given_non_null_value_should_return_value():
    assert require_non_null("test", "message") == "test"


def test_when_require_non_null_given_null_value_should_throw_exception():
    with pytest.raises(ValueError, match="Value is null"):
        require_non_null(None, "Value is null")


def test_when_require_non_blank_given_non_blank_string_should_return_string():
    assert require_non_blank("test", "message") == "test"


def test_when_require_non_blank_given_blank_string_should_throw_exception():
    with pytest.raises(ValueError):
        require_non_blank("  ", "String is blank")


def test_when_require_non_blank_given_null_string_should_throw_exception():
    with pytest.raises(ValueError):
        require_non_blank(None, "String is null")


def test_when_require_given_true_condition_should_not_throw():
    require(True, "Should not throw")


def test_when_require_given_false_condition_should_throw_exception():
    with pytest.raises(ValueError, match="Condition is false"):
        require(False, "Condition is false")


def test_when_require_domain_given_false_condition_should_throw_domain_exception():
    with pytest.raises(DomainError) as ei:
        require_domain(False, "Domain error")
    assert ei.value.error_code == "DOMAIN_ERROR" and str(ei.value) == "Domain error"


def test_when_require_positive_given_positive_value_should_return_value():
    assert require_positive(5, "message") == 5


def test_when_require_positive_given_zero_should_throw_exception():
    with pytest.raises(ValueError):
        require_positive(0, "Not positive")


def test_when_require_positive_given_negative_should_throw_exception():
    with pytest.raises(ValueError):
        require_positive(-1, "Not positive")


def test_when_require_non_negative_given_zero_should_return_zero():
    assert require_non_negative(0, "message") == 0


def test_when_require_non_negative_given_negative_should_throw_exception():
    with pytest.raises(ValueError):
        require_non_negative(-1, "Negative")


# =========================== RepositoryUrlTest ================================
def test_when_creating_url_given_valid_https_url_should_create():
    url = RepositoryUrl.of("https://github.com/example/repo.git")
    assert url.value == "https://github.com/example/repo.git"
    assert url.is_https() and not url.is_ssh()


def test_when_creating_url_given_valid_ssh_url_should_create():
    url = RepositoryUrl.of("git@github.com:example/repo.git")
    assert url.value == "git@github.com:example/repo.git"
    assert url.is_ssh() and not url.is_https()


def test_when_creating_url_given_invalid_url_should_throw_exception():
    with pytest.raises(ValueError):
        RepositoryUrl.of("not-a-valid-url")


def test_when_creating_url_given_blank_url_should_throw_exception():
    with pytest.raises(ValueError):
        RepositoryUrl.of("  ")


def test_when_extracting_repo_name_given_https_url_should_return_name():
    assert RepositoryUrl.of("https://github.com/example/my-project.git").repository_name() == "my-project"


def test_when_extracting_repo_name_given_ssh_url_should_return_name():
    assert RepositoryUrl.of("git@github.com:example/my-project.git").repository_name() == "my-project"


def test_when_comparing_urls_given_same_value_should_be_equal():
    a = RepositoryUrl.of("https://github.com/example/repo.git")
    b = RepositoryUrl.of("https://github.com/example/repo.git")
    assert a == b and hash(a) == hash(b)


# ============================== ProjectTest ===================================
def new_project() -> Project:
    return Project.create("Test", RepositoryUrl.of("https://github.com/test/repo.git"))



def analyzed_project() -> Project:
    p = new_project()
    p.start_analysis()
    p.analysis_completed("abc123")
    return p


def test_when_creating_project_given_valid_data_should_create_with_pending_status():
    url = RepositoryUrl.of("https://github.com/example/repo.git")
    p = Project.create("Test Project", url)
    assert p.id and p.name == "Test Project" and p.repository_url == url
    assert p.default_branch == "main" and p.status is S.PENDING and p.created_at is not None


def test_when_creating_project_given_custom_branch_should_use_custom_branch():
    p = Project.create("Test Project", RepositoryUrl.of("https://github.com/example/repo.git"), "develop")
    assert p.default_branch == "develop"


def test_when_starting_analysis_given_pending_status_should_transition_to_analyzing():
    p = new_project()
    p.start_analysis()
    assert p.status is S.ANALYZING


def test_when_starting_analysis_given_analyzing_status_should_throw_exception():
    p = new_project()
    p.start_analysis()
    with pytest.raises(DomainError):
        p.start_analysis()


def test_when_completing_analysis_given_analyzing_status_should_transition_to_analyzed():
    p = new_project()
    p.start_analysis()
    p.analysis_completed("abc123")
    assert p.status is S.ANALYZED and p.last_commit_hash == "abc123" and p.last_analyzed_at is not None


def test_when_starting_analysis_given_analyzed_status_should_transition_to_analyzing():
    p = analyzed_project()
    p.start_analysis()
    assert p.status is S.ANALYZING


def test_when_starting_analysis_given_error_status_should_transition_to_analyzing():
    p = new_project()
    p.start_analysis()
    p.mark_error()
    p.start_analysis()
    assert p.status is S.ANALYZING


def test_when_marking_error_given_analyzing_status_should_transition_to_error():
    p = new_project()
    p.start_analysis()
    p.mark_error()
    assert p.status is S.ERROR


def test_when_starting_sync_given_analyzing_status_should_throw_domain_exception():
    p = new_project()
    p.start_analysis()
    with pytest.raises(DomainError):
        p.start_sync()


def test_when_starting_sync_given_analyzed_status_should_transition_to_syncing():
    p = analyzed_project()
    p.start_sync()
    assert p.status is S.SYNCING


def test_when_completing_sync_given_syncing_status_should_transition_to_analyzed():
    p = analyzed_project()
    p.start_sync()
    p.sync_completed("def456")
    assert p.status is S.ANALYZED and p.last_commit_hash == "def456" and p.last_analyzed_at is not None


def test_when_marking_error_given_syncing_status_should_transition_to_error():
    p = analyzed_project()
    p.start_sync()
    p.mark_error()
    assert p.status is S.ERROR


def test_when_renaming_given_valid_name_should_update_name():
    p = new_project()
    p.rename("New Name")
    assert p.name == "New Name"


def test_when_renaming_given_blank_name_should_throw_exception():
    with pytest.raises(ValueError):
        new_project().rename("  ")


# ========================= ProjectStateMachineTest ============================
@pytest.mark.parametrize("src,dst", [
    (S.PENDING, S.ANALYZING),    # whenTransitioning_givenPendingToAnalyzing_shouldReturnAnalyzing
    (S.ANALYZING, S.ANALYZED),   # ..._givenAnalyzingToAnalyzed_shouldReturnAnalyzed
    (S.ANALYZING, S.ERROR),      # ..._givenAnalyzingToError_shouldReturnError
    (S.ANALYZED, S.ANALYZING),   # ..._givenAnalyzedToAnalyzing_shouldReturnAnalyzing
    (S.ANALYZED, S.SYNCING),     # ..._givenAnalyzedToSyncing_shouldReturnSyncing
    (S.SYNCING, S.ANALYZED),     # ..._givenSyncingToAnalyzed_shouldReturnAnalyzed
    (S.SYNCING, S.ERROR),        # ..._givenSyncingToError_shouldReturnError
    (S.ERROR, S.ANALYZING),      # ..._givenErrorToAnalyzing_shouldReturnAnalyzing
    (S.ERROR, S.SYNCING),        # ..._givenErrorToSyncing_shouldReturnSyncing
])
def test_when_transitioning_given_allowed_move_should_return_target(src, dst):
    assert transition(src, dst) is dst


@pytest.mark.parametrize("src,dst", [
    (S.PENDING, S.ANALYZED),     # whenTransitioning_givenPendingToAnalyzed_shouldThrowDomainException
    (S.ANALYZED, S.ERROR),       # ..._givenAnalyzedToError_shouldThrowDomainException
    (S.ERROR, S.ANALYZED),       # ..._givenErrorToAnalyzed_shouldThrowDomainException
    (S.PENDING, S.SYNCING),      # ..._givenPendingToSyncing_shouldThrowDomainException
    (S.SYNCING, S.ANALYZING),    # ..._givenSyncingToAnalyzing_shouldThrowDomainException
])
def test_when_transitioning_given_illegal_move_should_throw_domain_exception(src, dst):
    with pytest.raises(DomainError) as ei:
        transition(src, dst)
    assert ei.value.error_code == "PROJECT_INVALID_TRANSITION"


def test_when_transitioning_given_null_from_should_throw_illegal_argument_exception():
    with pytest.raises(ValueError):
        transition(None, S.ANALYZING)


def test_when_transitioning_given_null_to_should_throw_illegal_argument_exception():
    with pytest.raises(ValueError):
        transition(S.PENDING, None)


# ============================== ClassTypeTest =================================
def test_when_parsing_string_given_valid_type_should_return_correct_enum():
    for name in ("CONTROLLER", "SERVICE", "REPOSITORY", "ENTITY", "DTO"):
        assert ClassType.from_string(name) is ClassType[name]


def test_when_parsing_string_given_lowercase_type_should_return_correct_enum():
    assert ClassType.from_string("controller") is ClassType.CONTROLLER
    assert ClassType.from_string("service") is ClassType.SERVICE


def test_when_parsing_string_given_mixed_case_type_should_return_correct_enum():
    assert ClassType.from_string("Controller") is ClassType.CONTROLLER
    assert ClassType.from_string("Service") is ClassType.SERVICE


def test_when_parsing_string_given_invalid_type_should_return_other():
    for v in ("INVALID", "unknown", "xyz"):
        assert ClassType.from_string(v) is ClassType.OTHER


def test_when_parsing_string_given_null_or_blank_should_return_other():
    for v in (None, "", "  "):
        assert ClassType.from_string(v) is ClassType.OTHER


def test_when_checking_request_handler_given_controller_should_return_true():
    assert ClassType.CONTROLLER.is_request_handler()


def test_when_checking_request_handler_given_listener_should_return_true():
    assert ClassType.LISTENER.is_request_handler()


def test_when_checking_request_handler_given_service_should_return_false():
    assert not ClassType.SERVICE.is_request_handler()


def test_when_checking_business_logic_given_service_should_return_true():
    assert ClassType.SERVICE.contains_business_logic()


def test_when_checking_business_logic_given_entity_should_return_true():
    assert ClassType.ENTITY.contains_business_logic()


def test_when_checking_business_logic_given_controller_should_return_false():
    assert not ClassType.CONTROLLER.contains_business_logic()


def test_when_getting_description_given_any_type_should_return_non_null_description():
    for t in ClassType:
        assert t.description and t.description.strip(), t


# ============================= SourceClassTest ================================
def source_class(fqcn):
    return SourceClass.create(new_id(), fqcn, ClassType.SERVICE, "Test class", None, None)


def test_when_creating_class_given_valid_data_should_create_with_correct_values():
    pid = new_id()
    c = SourceClass.create(pid, "co.fanki.user.UserService", ClassType.SERVICE, "Manages user operations",
                           "src/main/java/co/fanki/user/UserService.java", "abc123def")
    assert c.id and c.project_id == pid and c.full_class_name == "co.fanki.user.UserService"
    assert c.simple_name == "UserService" and c.package_name == "co.fanki.user"
    assert c.class_type is ClassType.SERVICE and c.description == "Manages user operations"
    assert c.commit_hash == "abc123def" and c.created_at is not None


def test_when_creating_class_given_no_package_should_handle_simple_name():
    c = SourceClass.create(new_id(), "UserService", ClassType.SERVICE, "Manages user operations",
                           "UserService.java", None)
    assert (c.full_class_name, c.simple_name, c.package_name) == ("UserService", "UserService", None)


def test_when_creating_class_given_null_project_id_should_throw_exception():
    with pytest.raises(ValueError):
        SourceClass.create(None, "co.fanki.Test", ClassType.OTHER, None, None, None)


def test_when_creating_class_given_blank_class_name_should_throw_exception():
    with pytest.raises(ValueError):
        SourceClass.create(new_id(), "  ", ClassType.OTHER, None, None, None)


def test_when_creating_class_given_null_class_type_should_throw_exception():
    with pytest.raises(ValueError):
        SourceClass.create(new_id(), "co.fanki.Test", None, None, None, None)


def test_when_checking_package_given_exact_match_should_return_true():
    assert source_class("co.fanki.user.UserService").belongs_to_package("co.fanki.user")


def test_when_checking_package_given_subpackage_should_return_true():
    c = source_class("co.fanki.user.domain.User")
    assert c.belongs_to_package("co.fanki.user") and c.belongs_to_package("co.fanki") and c.belongs_to_package("co")


def test_when_checking_package_given_different_package_should_return_false():
    c = source_class("co.fanki.user.UserService")
    assert not c.belongs_to_package("co.fanki.order") and not c.belongs_to_package("com.example")


def test_when_checking_package_given_partial_match_should_return_false():
    assert not source_class("co.fanki.user.UserService").belongs_to_package("co.fanki.use")


def test_when_checking_package_given_null_package_should_return_false():
    assert not source_class("co.fanki.user.UserService").belongs_to_package(None)


def test_source_class_when_reconstituting_given_all_fields_should_recreate_exactly():
    cid, pid = new_id(), new_id()
    created = datetime.now(timezone.utc) - timedelta(hours=1)
    c = SourceClass.reconstitute(cid, pid, "co.fanki.user.UserService", "UserService", "co.fanki.user",
                                 ClassType.SERVICE, "Manages user operations",
                                 "src/main/java/co/fanki/user/UserService.java", "abc123def", created)
    assert (c.id, c.project_id, c.full_class_name, c.simple_name, c.package_name) == (
        cid, pid, "co.fanki.user.UserService", "UserService", "co.fanki.user")
    assert c.class_type is ClassType.SERVICE and c.description == "Manages user operations"
    assert c.commit_hash == "abc123def" and c.created_at == created


# ============================= SourceMethodTest ===============================
def http_method(verb, path):
    return SourceMethod.create(new_id(), "testMethod", "Test description", None, None, verb, path, None)


def test_when_creating_method_given_valid_data_should_create_with_correct_values():
    cid = new_id()
    m = SourceMethod.create(cid, "createUser", "Creates a new user", ["Validates input", "Saves to DB"],
                            ["ValidationException"], "POST", "/api/users", 45)
    assert m.id and m.class_id == cid and m.method_name == "createUser"
    assert m.description == "Creates a new user"
    assert list(m.business_logic) == ["Validates input", "Saves to DB"]
    assert list(m.exceptions) == ["ValidationException"]
    assert (m.http_method, m.http_path, m.line_number) == ("POST", "/api/users", 45)
    assert m.created_at is not None


def test_when_creating_method_given_null_class_id_should_throw_exception():
    with pytest.raises(ValueError):
        SourceMethod.create(None, "test", None, None, None, None, None, None)


def test_when_creating_method_given_blank_method_name_should_throw_exception():
    with pytest.raises(ValueError):
        SourceMethod.create(new_id(), "  ", None, None, None, None, None, None)


def test_when_creating_method_given_null_lists_should_return_empty_lists():
    m = SourceMethod.create(new_id(), "test", None, None, None, None, None, None)
    assert len(m.business_logic) == 0 and len(m.exceptions) == 0


def test_when_checking_http_endpoint_given_both_method_and_path_should_return_true():
    assert http_method("GET", "/api/users").is_http_endpoint()


def test_when_checking_http_endpoint_given_only_method_should_return_false():
    assert not http_method("GET", None).is_http_endpoint()


def test_when_checking_http_endpoint_given_only_path_should_return_false():
    assert not http_method(None, "/api/users").is_http_endpoint()


def test_when_checking_http_endpoint_given_neither_method_nor_path_should_return_false():
    assert not http_method(None, None).is_http_endpoint()


def test_when_getting_http_endpoint_given_valid_endpoint_should_return_combined():
    assert http_method("POST", "/api/users").http_endpoint() == "POST /api/users"


def test_when_getting_http_endpoint_given_non_endpoint_should_return_null():
    assert http_method(None, None).http_endpoint() is None


def test_source_method_when_reconstituting_given_all_fields_should_recreate_exactly():
    mid, cid = new_id(), new_id()
    created = datetime.now(timezone.utc) - timedelta(hours=1)
    m = SourceMethod.reconstitute(mid, cid, "testMethod", "Test description", ["Step 1", "Step 2"], ["Ex1"],
                                  "PUT", "/api/test", 100, created)
    assert (m.id, m.class_id, m.method_name, m.description) == (mid, cid, "testMethod", "Test description")
    assert list(m.business_logic) == ["Step 1", "Step 2"] and list(m.exceptions) == ["Ex1"]
    assert (m.http_method, m.http_path, m.line_number, m.created_at) == ("PUT", "/api/test", 100, created)


def test_when_creating_method_given_lists_should_return_immutable_copies():
    original = ["Step 1"]
    m = SourceMethod.create(new_id(), "test", None, original, None, None, None, None)
    original.append("Step 2")
    assert len(m.business_logic) == 1
    with pytest.raises(AttributeError):
        m.business_logic.append("Step 3")


# =========================== MethodParameterTest ==============================
def test_when_creating_given_valid_inputs_should_create_instance():
    p = MethodParameter.create("method-1", 0, "class-1")
    assert p.id and (p.method_id, p.position, p.class_id) == ("method-1", 0, "class-1")
    assert p.created_at is not None


def test_when_creating_given_position_greater_than_zero_should_create_instance():
    assert MethodParameter.create("method-1", 3, "class-1").position == 3


def test_method_parameter_when_reconstituting_given_all_fields_should_preserve_values():
    created = datetime(2025, 1, 15, 10, 30, tzinfo=timezone.utc)
    p = MethodParameter.reconstitute("param-id", "method-id", 2, "class-id", created)
    assert (p.id, p.method_id, p.position, p.class_id, p.created_at) == (
        "param-id", "method-id", 2, "class-id", created)


def test_when_creating_given_null_method_id_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.create(None, 0, "class-1")


def test_when_creating_given_blank_method_id_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.create("  ", 0, "class-1")


def test_when_creating_given_null_class_id_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.create("method-1", 0, None)


def test_when_creating_given_blank_class_id_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.create("method-1", 0, "")


def test_when_creating_given_negative_position_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.create("method-1", -1, "class-1")


def test_when_reconstituting_given_null_id_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.reconstitute(None, "method-1", 0, "class-1", datetime.now(timezone.utc))


def test_when_reconstituting_given_blank_id_should_throw_exception():
    with pytest.raises(ValueError):
        MethodParameter.reconstitute("", "method-1", 0, "class-1", datetime.now(timezone.utc))
