"""One test per case of the reference's ``ProjectGraphTest`` (98 cases).

Mirrors ``src/test/java/co/fanki/domainmcp/analysis/domain/ProjectGraphTest.java``
case by case; test names are the reference's ``when…_given…_should…`` names in
snake case.  Java's ``IllegalArgumentException`` maps to ``ValueError`` and the
reference's unmodifiable ``Set``/``List`` views map to tuples (immutable).
"""
import json

import pytest

from dmcp.graph.project_graph import (MethodEnrichmentData, MethodInfo, ProjectGraph)


def chain():
    """Controller -> Service -> Repository (``buildSimpleChainGraph``, ``:630-638``)."""
    g = ProjectGraph()
    g.add_node("co.fanki.Controller", "src/Controller.java")
    g.add_node("co.fanki.Service", "src/Service.java")
    g.add_node("co.fanki.Repository", "src/Repository.java")
    g.add_dependency("co.fanki.Controller", "co.fanki.Service")
    g.add_dependency("co.fanki.Service", "co.fanki.Repository")
    return g


def nodes(*names):
    g = ProjectGraph()
    for n in names:
        g.add_node(f"co.fanki.{n}", f"src/{n}.java")
    return g


def immutable(view):
    with pytest.raises((AttributeError, TypeError)):
        view.add("co.fanki.Hack")  # tuples have no add / item assignment
    with pytest.raises(TypeError):
        view[0] = "co.fanki.Hack"


# -- addNode -------------------------------------------------------------------
def test_when_adding_node_given_valid_identifier_and_file_should_increase_node_count():
    g = nodes("UserService")
    assert g.node_count() == 1 and g.contains("co.fanki.UserService")


def test_when_adding_node_given_multiple_distinct_nodes_should_track_all():
    g = nodes("UserService", "OrderService", "User")
    assert g.node_count() == 3
    assert set(g.identifiers()) == {"co.fanki.UserService", "co.fanki.OrderService", "co.fanki.User"}


def test_when_adding_node_given_duplicate_identifier_should_overwrite_source_file():
    g = ProjectGraph()
    g.add_node("co.fanki.UserService", "src/old/UserService.java")
    g.add_node("co.fanki.UserService", "src/new/UserService.java")
    assert g.node_count() == 1
    assert g.source_file("co.fanki.UserService") == "src/new/UserService.java"


def test_when_adding_node_given_null_identifier_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().add_node(None, "src/Test.java")


def test_when_adding_node_given_blank_identifier_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().add_node("  ", "src/Test.java")


def test_when_adding_node_given_null_source_file_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().add_node("co.fanki.Test", None)


def test_when_adding_node_given_blank_source_file_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().add_node("co.fanki.Test", "")


# -- addDependency -------------------------------------------------------------
def test_when_adding_dependency_given_both_nodes_exist_should_create_edge():
    g = nodes("Controller", "Service")
    g.add_dependency("co.fanki.Controller", "co.fanki.Service")
    assert "co.fanki.Service" in g.resolve("co.fanki.Controller")


def test_when_adding_dependency_given_from_node_unknown_should_ignore_silently():
    g = nodes("Service")
    g.add_dependency("co.fanki.Unknown", "co.fanki.Service")
    assert g.resolve("co.fanki.Service") == ()


def test_when_adding_dependency_given_to_node_unknown_should_ignore_silently():
    g = nodes("Controller")
    g.add_dependency("co.fanki.Controller", "co.fanki.Unknown")
    assert g.resolve("co.fanki.Controller") == ()


def test_when_adding_dependency_given_both_nodes_unknown_should_ignore_silently():
    g = ProjectGraph()
    g.add_dependency("co.fanki.A", "co.fanki.B")
    assert g.node_count() == 0 and g.edge_count() == 0


def test_when_adding_dependency_given_null_from_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().add_dependency(None, "co.fanki.B")


def test_when_adding_dependency_given_blank_to_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().add_dependency("co.fanki.A", "  ")


def test_when_adding_dependency_given_duplicate_should_not_create_multiple_edges():
    g = nodes("A", "B")
    g.add_dependency("co.fanki.A", "co.fanki.B")
    g.add_dependency("co.fanki.A", "co.fanki.B")
    assert len(g.resolve("co.fanki.A")) == 1 and g.edge_count() == 1


# -- markAsEntryPoint ----------------------------------------------------------
def test_when_marking_entry_point_given_known_node_should_increase_entry_point_count():
    g = nodes("Controller")
    g.mark_as_entry_point("co.fanki.Controller")
    assert g.entry_point_count() == 1


def test_when_marking_entry_point_given_unknown_node_should_ignore_silently():
    g = ProjectGraph()
    g.mark_as_entry_point("co.fanki.Unknown")
    assert g.entry_point_count() == 0


def test_when_marking_entry_point_given_null_identifier_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().mark_as_entry_point(None)


def test_when_marking_entry_point_given_blank_identifier_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().mark_as_entry_point("")


def test_when_marking_entry_point_given_already_marked_should_not_duplicate():
    g = nodes("Controller")
    g.mark_as_entry_point("co.fanki.Controller")
    g.mark_as_entry_point("co.fanki.Controller")
    assert g.entry_point_count() == 1


# -- dependencies --------------------------------------------------------------
def test_when_querying_dependencies_given_node_with_outgoing_should_return_direct_deps():
    assert set(chain().dependencies("co.fanki.Controller")) == {"co.fanki.Service"}


def test_when_querying_dependencies_given_leaf_node_should_return_empty_set():
    assert not chain().dependencies("co.fanki.Repository")


def test_when_querying_dependencies_given_unknown_node_should_return_empty_set():
    assert not chain().dependencies("co.fanki.Unknown")


def test_when_querying_dependencies_given_null_should_return_empty_set():
    assert not chain().dependencies(None)


def test_when_querying_dependencies_should_be_unmodifiable():
    g = chain()
    immutable(g.dependencies("co.fanki.Controller"))
    assert g.dependencies("co.fanki.Controller") == ("co.fanki.Service",)


# -- dependents ----------------------------------------------------------------
def test_when_querying_dependents_given_node_with_incoming_should_return_reverse_deps():
    assert set(chain().dependents("co.fanki.Service")) == {"co.fanki.Controller"}


def test_when_querying_dependents_given_root_node_should_return_empty_set():
    assert not chain().dependents("co.fanki.Controller")


def test_when_querying_dependents_given_leaf_node_should_return_incoming():
    assert set(chain().dependents("co.fanki.Repository")) == {"co.fanki.Service"}


def test_when_querying_dependents_given_unknown_node_should_return_empty_set():
    assert not chain().dependents("co.fanki.Unknown")


def test_when_querying_dependents_given_null_should_return_empty_set():
    assert not chain().dependents(None)


def test_when_querying_dependents_should_be_unmodifiable():
    g = chain()
    immutable(g.dependents("co.fanki.Service"))
    assert g.dependents("co.fanki.Service") == ("co.fanki.Controller",)


# -- isEntryPoint / entryPoints ------------------------------------------------
def test_when_checking_is_entry_point_given_marked_node_should_return_true():
    g = nodes("Controller")
    g.mark_as_entry_point("co.fanki.Controller")
    assert g.is_entry_point("co.fanki.Controller")


def test_when_checking_is_entry_point_given_unmarked_node_should_return_false():
    assert not nodes("Service").is_entry_point("co.fanki.Service")


def test_when_checking_is_entry_point_given_null_should_return_false():
    assert not ProjectGraph().is_entry_point(None)


def test_when_getting_entry_points_given_marked_nodes_should_return_all():
    g = nodes("A", "B", "C")
    g.mark_as_entry_point("co.fanki.A")
    g.mark_as_entry_point("co.fanki.B")
    assert set(g.entry_points()) == {"co.fanki.A", "co.fanki.B"}


def test_when_getting_entry_points_given_no_entry_points_should_return_empty_set():
    assert not nodes("A").entry_points()


def test_when_getting_entry_points_should_be_unmodifiable():
    g = nodes("A")
    g.mark_as_entry_point("co.fanki.A")
    immutable(g.entry_points())
    assert g.entry_point_count() == 1


# -- resolve -------------------------------------------------------------------
def test_when_resolving_given_direct_dependency_should_return_target():
    assert "co.fanki.Service" in chain().resolve("co.fanki.Controller")


def test_when_resolving_given_reverse_dependency_should_return_source():
    n = chain().resolve("co.fanki.Service")
    assert "co.fanki.Controller" in n and "co.fanki.Repository" in n


def test_when_resolving_given_both_directions_should_return_all():
    assert set(chain().resolve("co.fanki.Service")) == {"co.fanki.Controller", "co.fanki.Repository"}


def test_when_resolving_given_leaf_node_should_return_only_incoming():
    assert set(chain().resolve("co.fanki.Repository")) == {"co.fanki.Service"}


def test_when_resolving_given_null_identifier_should_return_empty_set():
    assert not chain().resolve(None)


def test_when_resolving_given_unknown_identifier_should_return_empty_set():
    assert not chain().resolve("co.fanki.Unknown")


def test_when_resolving_given_isolated_node_should_return_empty_set():
    assert not nodes("Isolated").resolve("co.fanki.Isolated")


# -- analysisOrder -------------------------------------------------------------
def test_when_computing_analysis_order_given_entry_point_chain_should_start_from_entry_point():
    g = chain()
    g.mark_as_entry_point("co.fanki.Controller")
    order = g.analysis_order()
    assert order.index("co.fanki.Controller") == 0
    assert order.index("co.fanki.Service") < order.index("co.fanki.Repository")


def test_when_computing_analysis_order_given_multiple_entry_points_should_visit_all_reachable():
    g = nodes("ControllerA", "ControllerB", "ServiceA", "ServiceB")
    g.add_dependency("co.fanki.ControllerA", "co.fanki.ServiceA")
    g.add_dependency("co.fanki.ControllerB", "co.fanki.ServiceB")
    g.mark_as_entry_point("co.fanki.ControllerA")
    g.mark_as_entry_point("co.fanki.ControllerB")
    order = g.analysis_order()
    assert len(order) == 4
    assert order.index("co.fanki.ControllerA") < order.index("co.fanki.ServiceA")
    assert order.index("co.fanki.ControllerB") < order.index("co.fanki.ServiceB")


def test_when_computing_analysis_order_given_orphans_should_append_at_end():
    g = nodes("Controller", "Service", "Orphan")
    g.add_dependency("co.fanki.Controller", "co.fanki.Service")
    g.mark_as_entry_point("co.fanki.Controller")
    order = g.analysis_order()
    assert len(order) == 3 and order[-1] == "co.fanki.Orphan"


def test_when_computing_analysis_order_given_no_entry_points_should_return_all_as_orphans():
    order = nodes("A", "B").analysis_order()
    assert len(order) == 2 and set(order) == {"co.fanki.A", "co.fanki.B"}


def test_when_computing_analysis_order_given_empty_graph_should_return_empty_list():
    assert ProjectGraph().analysis_order() == []


def test_when_computing_analysis_order_given_diamond_dependency_should_visit_each_node_once():
    g = nodes("Root", "Left", "Right", "Leaf")
    g.add_dependency("co.fanki.Root", "co.fanki.Left")
    g.add_dependency("co.fanki.Root", "co.fanki.Right")
    g.add_dependency("co.fanki.Left", "co.fanki.Leaf")
    g.add_dependency("co.fanki.Right", "co.fanki.Leaf")
    g.mark_as_entry_point("co.fanki.Root")
    order = g.analysis_order()
    assert len(order) == 4 and len(set(order)) == 4 and order.index("co.fanki.Root") == 0


# -- bindClassId / classId -----------------------------------------------------
def test_when_binding_class_id_given_valid_data_should_be_retrievable():
    g = nodes("User")
    g.bind_class_id("co.fanki.User", "class-uuid-123")
    assert g.class_id("co.fanki.User") == "class-uuid-123"


def test_when_retrieving_class_id_given_unbound_identifier_should_return_null():
    assert nodes("User").class_id("co.fanki.User") is None


def test_when_retrieving_class_id_given_unknown_identifier_should_return_null():
    assert ProjectGraph().class_id("co.fanki.Unknown") is None


def test_when_binding_class_id_given_null_identifier_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().bind_class_id(None, "id-123")


def test_when_binding_class_id_given_blank_class_id_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph().bind_class_id("co.fanki.User", "")


def test_when_binding_class_id_given_overwrite_should_replace_old_value():
    g = nodes("User")
    g.bind_class_id("co.fanki.User", "old-id")
    g.bind_class_id("co.fanki.User", "new-id")
    assert g.class_id("co.fanki.User") == "new-id"


# -- sourceFile / contains -----------------------------------------------------
def test_when_retrieving_source_file_given_known_node_should_return_file_path():
    g = ProjectGraph()
    g.add_node("co.fanki.User", "src/main/java/User.java")
    assert g.source_file("co.fanki.User") == "src/main/java/User.java"


def test_when_retrieving_source_file_given_unknown_node_should_return_null():
    assert ProjectGraph().source_file("co.fanki.Unknown") is None


def test_when_checking_contains_given_existing_node_should_return_true():
    assert nodes("User").contains("co.fanki.User")


def test_when_checking_contains_given_absent_node_should_return_false():
    assert not ProjectGraph().contains("co.fanki.Unknown")


def test_when_checking_contains_given_null_should_return_false():
    assert not ProjectGraph().contains(None)


# -- toJson / fromJson ---------------------------------------------------------
def test_when_serializing_to_json_given_populated_graph_should_round_trip():
    g = chain()
    g.mark_as_entry_point("co.fanki.Controller")
    g.bind_class_id("co.fanki.Controller", "id-ctrl")
    g.bind_class_id("co.fanki.Service", "id-svc")
    r = ProjectGraph.from_json(g.to_json())
    assert r.node_count() == g.node_count() and r.entry_point_count() == g.entry_point_count()
    for n in ("Controller", "Service", "Repository"):
        assert r.source_file(f"co.fanki.{n}") == g.source_file(f"co.fanki.{n}")
    assert r.class_id("co.fanki.Controller") == "id-ctrl"
    assert r.class_id("co.fanki.Service") == "id-svc"
    assert r.class_id("co.fanki.Repository") is None


def test_when_serializing_to_json_given_edges_should_preserve_dependencies():
    g = chain()
    g.mark_as_entry_point("co.fanki.Controller")
    r = ProjectGraph.from_json(g.to_json())
    assert set(r.resolve("co.fanki.Service")) == set(g.resolve("co.fanki.Service"))


def test_when_serializing_to_json_given_empty_graph_should_round_trip():
    r = ProjectGraph.from_json(ProjectGraph().to_json())
    assert r.node_count() == 0 and r.entry_point_count() == 0


def test_when_serializing_to_json_given_entry_points_should_preserve_them():
    g = nodes("A", "B")
    g.mark_as_entry_point("co.fanki.A")
    g.mark_as_entry_point("co.fanki.B")
    assert ProjectGraph.from_json(g.to_json()).entry_point_count() == 2


def test_when_serializing_to_json_given_analysis_order_should_be_preserved():
    g = chain()
    g.mark_as_entry_point("co.fanki.Controller")
    assert ProjectGraph.from_json(g.to_json()).analysis_order() == g.analysis_order()


def test_when_deserializing_from_json_given_null_json_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph.from_json(None)


def test_when_deserializing_from_json_given_blank_json_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph.from_json("  ")


def test_when_deserializing_from_json_given_malformed_json_should_throw_exception():
    with pytest.raises(ValueError):
        ProjectGraph.from_json("{invalid-json")


# -- identifiers / counts ------------------------------------------------------
def test_when_getting_identifiers_given_populated_graph_should_return_all_keys():
    assert set(nodes("A", "B").identifiers()) == {"co.fanki.A", "co.fanki.B"}


def test_when_getting_identifiers_given_empty_graph_should_return_empty_set():
    assert not ProjectGraph().identifiers()


def test_when_getting_identifiers_should_be_unmodifiable():
    g = nodes("A")
    immutable(g.identifiers())
    with pytest.raises(AttributeError):
        g.identifier_set().add("co.fanki.B")  # the live view is read-only too
    assert g.node_count() == 1


def test_when_getting_node_count_given_empty_graph_should_return_zero():
    assert ProjectGraph().node_count() == 0


def test_when_getting_entry_point_count_given_no_entry_points_should_return_zero():
    assert nodes("A").entry_point_count() == 0


# -- complex scenarios ---------------------------------------------------------
def cyclic():
    g = nodes("A", "B")
    g.add_dependency("co.fanki.A", "co.fanki.B")
    g.add_dependency("co.fanki.B", "co.fanki.A")
    return g


def test_when_resolving_given_cyclic_dependency_should_return_correct_neighbors():
    g = cyclic()
    assert set(g.resolve("co.fanki.A")) == {"co.fanki.B"}
    assert set(g.resolve("co.fanki.B")) == {"co.fanki.A"}


def test_when_computing_analysis_order_given_cyclic_dependency_should_not_loop():
    g = cyclic()
    g.mark_as_entry_point("co.fanki.A")
    assert g.analysis_order() == ["co.fanki.A", "co.fanki.B"]


def test_when_serializing_to_json_given_cyclic_graph_should_round_trip():
    g = cyclic()
    g.mark_as_entry_point("co.fanki.A")
    r = ProjectGraph.from_json(g.to_json())
    assert set(r.resolve("co.fanki.A")) == set(g.resolve("co.fanki.A"))
    assert set(r.resolve("co.fanki.B")) == set(g.resolve("co.fanki.B"))
    assert r.analysis_order() == g.analysis_order()


def test_when_resolving_given_self_dependency_should_include_self():
    g = nodes("A")
    g.add_dependency("co.fanki.A", "co.fanki.A")
    assert set(g.resolve("co.fanki.A")) == {"co.fanki.A"}


def test_when_serializing_to_json_should_produce_valid_json_string():
    g = nodes("User")
    text = g.to_json()
    assert text is not None
    for frag in ('"nodes"', '"edges"', '"entryPoints"', "co.fanki.User", "src/User.java"):
        assert frag in text
    json.loads(text)


# -- addMethodParameter --------------------------------------------------------
def test_when_adding_method_parameter_given_both_nodes_exist_should_be_retrievable():
    g = nodes("Controller", "UserDto")
    g.add_method_parameter("co.fanki.Controller", "createUser", 0, "co.fanki.UserDto")
    params = g.method_parameters("co.fanki.Controller")
    assert list(params) == ["createUser"]
    (link,) = params["createUser"]
    assert link.position == 0 and link.target_identifier == "co.fanki.UserDto"


def test_when_adding_method_parameter_given_unknown_owner_should_ignore_silently():
    g = nodes("UserDto")
    g.add_method_parameter("co.fanki.Unknown", "create", 0, "co.fanki.UserDto")
    assert not g.method_parameters("co.fanki.Unknown")


def test_when_adding_method_parameter_given_unknown_target_should_ignore_silently():
    g = nodes("Controller")
    g.add_method_parameter("co.fanki.Controller", "create", 0, "co.fanki.Unknown")
    assert not g.method_parameters("co.fanki.Controller")


def test_when_adding_method_parameter_given_null_method_name_should_throw_exception():
    g = nodes("Controller", "UserDto")
    with pytest.raises(ValueError):
        g.add_method_parameter("co.fanki.Controller", None, 0, "co.fanki.UserDto")


def test_when_adding_method_parameter_given_negative_position_should_throw_exception():
    g = nodes("Controller", "UserDto")
    with pytest.raises(ValueError):
        g.add_method_parameter("co.fanki.Controller", "create", -1, "co.fanki.UserDto")


def test_when_querying_method_parameter_targets_given_class_with_params_should_return_target_set():
    g = nodes("Controller", "UserDto", "OrderDto")
    g.add_method_parameter("co.fanki.Controller", "create", 0, "co.fanki.UserDto")
    g.add_method_parameter("co.fanki.Controller", "order", 0, "co.fanki.OrderDto")
    assert set(g.method_parameter_targets("co.fanki.Controller")) == {"co.fanki.UserDto", "co.fanki.OrderDto"}


def test_when_querying_method_parameter_targets_given_class_with_no_params_should_return_empty_set():
    assert not nodes("Controller").method_parameter_targets("co.fanki.Controller")


def test_when_serializing_to_json_given_method_parameters_should_round_trip():
    g = nodes("Controller", "UserDto")
    g.add_method_parameter("co.fanki.Controller", "createUser", 0, "co.fanki.UserDto")
    params = ProjectGraph.from_json(g.to_json()).method_parameters("co.fanki.Controller")
    assert len(params) == 1
    (link,) = params["createUser"]
    assert (link.position, link.target_identifier) == (0, "co.fanki.UserDto")


OLD_FORMAT = '{"nodes":{"co.fanki.A":{"sourceFile":"src/A.java"}},"edges":{},"entryPoints":[]}'


def test_when_deserializing_from_json_given_old_format_without_method_parameters_should_load_with_empty_params():
    r = ProjectGraph.from_json(OLD_FORMAT)
    assert r.node_count() == 1 and not r.method_parameters("co.fanki.A")


def test_when_adding_method_parameter_given_multiple_methods_and_positions_should_track_all_correctly():
    g = nodes("Service", "UserDto", "OrderDto")
    g.add_method_parameter("co.fanki.Service", "process", 0, "co.fanki.UserDto")
    g.add_method_parameter("co.fanki.Service", "process", 1, "co.fanki.OrderDto")
    g.add_method_parameter("co.fanki.Service", "validate", 0, "co.fanki.UserDto")
    params = g.method_parameters("co.fanki.Service")
    assert len(params) == 2
    assert [(l.position, l.target_identifier) for l in params["process"]] == [
        (0, "co.fanki.UserDto"), (1, "co.fanki.OrderDto")]
    assert [(l.position, l.target_identifier) for l in params["validate"]] == [(0, "co.fanki.UserDto")]


# -- NodeInfo and MethodInfo ---------------------------------------------------
def test_when_setting_node_info_should_be_retrievable():
    g = nodes("UserService")
    g.set_node_info("co.fanki.UserService", "SERVICE", "Handles user logic")
    info = g.node_info("co.fanki.UserService")
    assert info is not None and info.class_type == "SERVICE" and info.description == "Handles user logic"


def test_when_adding_method_info_should_be_retrievable():
    g = nodes("Controller")
    g.add_method_info("co.fanki.Controller", MethodInfo("getUsers", "Lists users", ("Query DB", "Map DTOs"),
                                                        ("NotFoundException",), "GET", "/api/users", 25))
    (mi,) = g.methods("co.fanki.Controller")
    assert mi.method_name == "getUsers" and mi.description == "Lists users"
    assert list(mi.business_logic) == ["Query DB", "Map DTOs"]
    assert list(mi.exceptions) == ["NotFoundException"]
    assert mi.is_http_endpoint() and mi.http_endpoint() == "GET /api/users" and mi.line_number == 25


def test_when_querying_methods_for_unknown_node_should_return_empty_list():
    assert not ProjectGraph().methods("co.fanki.Unknown")


def test_when_method_info_is_not_endpoint_should_report_not_endpoint():
    mi = MethodInfo("process", "Processes", (), (), None, None, 10)
    assert not mi.is_http_endpoint() and mi.http_endpoint() is None


def test_when_querying_all_endpoints_should_return_only_http_methods():
    g = nodes("Controller", "Service")
    g.add_method_info("co.fanki.Controller", MethodInfo("getUsers", None, (), (), "GET", "/api/users", 10))
    g.add_method_info("co.fanki.Service", MethodInfo("findAll", None, (), (), None, None, 20))
    eps = g.all_endpoints()
    assert len(eps) == 1
    assert eps[0][0] == "co.fanki.Controller" and eps[0][1].method_name == "getUsers"


def test_when_applying_enrichment_should_update_descriptions_and_logic():
    g = nodes("Service")
    g.set_node_info("co.fanki.Service", "SERVICE", None)
    g.add_method_info("co.fanki.Service", MethodInfo("process", None, (), (), None, None, 10))
    g.apply_enrichment("co.fanki.Service", "SERVICE", "Business processing service",
                       {"process": MethodEnrichmentData("Processes incoming data",
                                                        ("Validate", "Transform", "Persist"))})
    assert g.node_info("co.fanki.Service").description == "Business processing service"
    mi = g.methods("co.fanki.Service")[0]
    assert mi.description == "Processes incoming data"
    assert list(mi.business_logic) == ["Validate", "Transform", "Persist"]


def test_when_serializing_metadata_should_round_trip():
    g = nodes("Controller")
    g.set_node_info("co.fanki.Controller", "CONTROLLER", "HTTP handler")
    g.add_method_info("co.fanki.Controller", MethodInfo("create", "Creates something", ("Validate", "Save"),
                                                        ("BadRequest",), "POST", "/api/items", 30))
    r = ProjectGraph.from_json(g.to_json())
    ni = r.node_info("co.fanki.Controller")
    assert ni is not None and (ni.class_type, ni.description) == ("CONTROLLER", "HTTP handler")
    (mi,) = r.methods("co.fanki.Controller")
    assert (mi.method_name, mi.description) == ("create", "Creates something")
    assert list(mi.business_logic) == ["Validate", "Save"] and list(mi.exceptions) == ["BadRequest"]
    assert (mi.http_method, mi.http_path, mi.line_number) == ("POST", "/api/items", 30)


def test_when_deserializing_old_format_should_have_no_metadata():
    r = ProjectGraph.from_json(OLD_FORMAT)
    assert not r.has_metadata() and r.node_info("co.fanki.A") is None and not r.methods("co.fanki.A")


def test_when_graph_has_metadata_has_metadata_should_return_true():
    g = nodes("A")
    g.set_node_info("co.fanki.A", "SERVICE", "desc")
    assert g.has_metadata()


def test_when_graph_has_no_metadata_has_metadata_should_return_false():
    assert not nodes("A").has_metadata()
