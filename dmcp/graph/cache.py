"""Process-wide cache of published project graphs.

Parity: ``analysis/domain/GraphService.java`` -- ``loadAll`` at start-up
(``:55-76``; one corrupt graph never blocks the others), ``getGraph``
(``:84``), ``reload`` (``:93-109``), ``put`` (``:118-122``),
``getGraphByProjectName`` (``:130-136``), ``getProjectIdByName`` (``:144``).

Graphs are frozen on ``put`` so readers can never observe a mutation
(copy-on-publish).  A rename removes the stale name entry
(the reference keeps it forever).
"""
from __future__ import annotations

import logging
import threading
from typing import Dict, Optional

from .project_graph import ProjectGraph

LOG = logging.getLogger(__name__)


class GraphCache:
    def __init__(self, project_repository=None) -> None:
        self._graphs: Dict[str, ProjectGraph] = {}
        self._name_to_id: Dict[str, str] = {}
        self._id_to_name: Dict[str, str] = {}
        self._lock = threading.Lock()
        self._projects = project_repository

    def load_all(self) -> int:
        """Deserializes every persisted graph; returns how many were loaded."""
        if self._projects is None:
            return 0
        loaded = 0
        for project in self._projects.find_all_with_graph():
            try:
                graph = ProjectGraph.from_json(project.graph_data)
                self.put(project.id, project.name, graph)
                loaded += 1
            except Exception as e:  # corrupt graph: log and skip (GraphService.java:69-72)
                LOG.warning("Failed to load graph for project %s: %s", project.id, e)
        LOG.info("Loaded %d project graphs into cache", loaded)
        return loaded

    def reload(self, project_id: str) -> bool:
        if self._projects is None:
            return False
        project = self._projects.find_by_id(project_id)
        if project is None or project.graph_data is None:
            return False
        try:
            self.put(project.id, project.name, ProjectGraph.from_json(project.graph_data))
            return True
        except Exception as e:
            LOG.warning("Failed to reload graph for project %s: %s", project_id, e)
            return False

    def put(self, project_id: str, project_name: str, graph: ProjectGraph) -> None:
        graph.freeze()
        with self._lock:
            self._graphs[project_id] = graph
            old = self._id_to_name.get(project_id)
            if old is not None and old != project_name and self._name_to_id.get(old) == project_id:
                del self._name_to_id[old]
            self._name_to_id[project_name] = project_id
            self._id_to_name[project_id] = project_name

    def evict(self, project_id: str) -> None:
        with self._lock:
            self._graphs.pop(project_id, None)
            name = self._id_to_name.pop(project_id, None)
            if name is not None and self._name_to_id.get(name) == project_id:
                del self._name_to_id[name]

    def get_graph(self, project_id: Optional[str]) -> Optional[ProjectGraph]:
        if project_id is None:
            return None
        return self._graphs.get(project_id)

    def get_graph_by_project_name(self, project_name: Optional[str]) -> Optional[ProjectGraph]:
        pid = self._name_to_id.get(project_name) if project_name is not None else None
        return self._graphs.get(pid) if pid is not None else None

    def get_project_id_by_name(self, project_name: Optional[str]) -> Optional[str]:
        return self._name_to_id.get(project_name) if project_name is not None else None

    def project_names(self):
        return list(self._name_to_id)

    def __len__(self) -> int:
        return len(self._graphs)
