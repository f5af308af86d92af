"""Process-wide cache of published project graphs.

Parity: ``analysis/domain/GraphService.java`` -- ``loadAll`` at start-up
(``:55-76``; one corrupt graph never blocks the others), ``getGraph``
(``:84``), ``reload`` (``:93-109``), ``put`` (``:118-122``),
``getGraphByProjectName`` (``:130-136``), ``getProjectIdByName`` (``:144``).

Graphs are frozen on ``put`` so readers can never observe a mutation
(copy-on-publish).  A rename removes the stale name entry
(the reference keeps it forever).

Cross-process freshness (the reference's two deployment modes share one
database, SURVEY §1, yet its MCP process loads graphs once at start-up and
never sees a re-analysis done by the analysis service): with
``refresh_s`` set, a lookup at most every ``refresh_s`` seconds reads every
project's ``graph_version`` (a small query, no graph JSON) and reloads the
graphs whose version moved, loads new projects and drops deleted ones.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Dict, Optional

from .project_graph import ProjectGraph

LOG = logging.getLogger(__name__)


class GraphCache:
    def __init__(self, project_repository=None, refresh_s: Optional[float] = None) -> None:
        self._graphs: Dict[str, ProjectGraph] = {}
        self._name_to_id: Dict[str, str] = {}
        self._id_to_name: Dict[str, str] = {}
        self._versions: Dict[str, int] = {}  # graph_version of each graph as loaded / written here
        self._bad: Dict[str, int] = {}       # versions that failed to load (not retried)
        self._lock = threading.Lock()
        self._refresh_lock = threading.Lock()
        self._projects = project_repository
        self.refresh_s = refresh_s
        self._checked = time.monotonic()
        self.reloads = 0

    # ------------------------------------------------------------ freshness
    def refresh(self, force: bool = False) -> int:
        """Reloads graphs another process re-wrote; returns how many changed."""
        if self._projects is None or (self.refresh_s is None and not force):
            return 0
        now = time.monotonic()
        if not force and now - self._checked < self.refresh_s:
            return 0
        if not self._refresh_lock.acquire(blocking=force):
            return 0  # another reader is refreshing; serve what is cached
        try:
            self._checked = now
            try:
                versions = self._projects.graph_versions()
            except Exception as e:
                LOG.warning("Graph cache refresh failed: %s", e)
                return 0
            changed = 0
            for pid, (name, version) in versions.items():
                if self._bad.get(pid) == version:
                    continue  # that version does not deserialize; wait for the next one
                if self._versions.get(pid) != version or pid not in self._graphs:
                    if self.reload(pid):
                        changed += 1
                    else:
                        self._bad[pid] = version
                elif self._id_to_name.get(pid) != name:
                    self.put(pid, name, self._graphs[pid], version)
            for pid in [p for p in self._versions if p not in versions]:
                self.evict(pid)  # deleted (or graph cleared) by another process
                changed += 1
            self.reloads += changed
            return changed
        finally:
            self._refresh_lock.release()

    def load_all(self) -> int:
        """Deserializes every persisted graph; returns how many were loaded."""
        if self._projects is None:
            return 0
        loaded = 0
        # versions read BEFORE the graphs: a graph written in between is then
        # newer than its recorded version and refresh() reloads it (the other
        # order would record a newer version next to an older graph for ever)
        try:
            versions = self._projects.graph_versions()
        except Exception:
            versions = {}
        for project in self._projects.find_all_with_graph():
            try:
                graph = ProjectGraph.from_json(project.graph_data)
                v = versions.get(project.id)
                self.put(project.id, project.name, graph, v[1] if v is not None else -1)
                loaded += 1
            except Exception as e:  # corrupt graph: log and skip (GraphService.java:69-72)
                LOG.warning("Failed to load graph for project %s: %s", project.id, e)
        LOG.info("Loaded %d project graphs into cache", loaded)
        return loaded

    def reload(self, project_id: str) -> bool:
        if self._projects is None:
            return False
        version = self._projects.graph_version(project_id)  # read before the graph: never newer than it
        project = self._projects.find_by_id(project_id)
        if project is None or project.graph_data is None:
            return False
        try:
            self.put(project.id, project.name, ProjectGraph.from_json(project.graph_data), version)
            return True
        except Exception as e:
            LOG.warning("Failed to reload graph for project %s: %s", project_id, e)
            return False

    def put(self, project_id: str, project_name: str, graph: ProjectGraph, version: Optional[int] = None) -> None:
        """``version``: the row's ``graph_version`` this graph corresponds to
        (read from the database when omitted -- call after the commit, by the
        lease holder, the project's only writer)."""
        graph.freeze()
        if version is None and self._projects is not None:
            try:
                version = self._projects.graph_version(project_id)
            except Exception:
                version = None
        with self._lock:
            if version is not None:
                self._versions[project_id] = version
            self._graphs[project_id] = graph
            old = self._id_to_name.get(project_id)
            if old is not None and old != project_name and self._name_to_id.get(old) == project_id:
                del self._name_to_id[old]
            self._name_to_id[project_name] = project_id
            self._id_to_name[project_id] = project_name

    def evict(self, project_id: str) -> None:
        with self._lock:
            self._graphs.pop(project_id, None)
            self._versions.pop(project_id, None)
            name = self._id_to_name.pop(project_id, None)
            if name is not None and self._name_to_id.get(name) == project_id:
                del self._name_to_id[name]

    def get_graph(self, project_id: Optional[str]) -> Optional[ProjectGraph]:
        if project_id is None:
            return None
        if self.refresh_s is not None:
            self.refresh()
        return self._graphs.get(project_id)

    def get_graph_by_project_name(self, project_name: Optional[str]) -> Optional[ProjectGraph]:
        if self.refresh_s is not None:
            self.refresh()
        pid = self._name_to_id.get(project_name) if project_name is not None else None
        return self._graphs.get(pid) if pid is not None else None

    def get_project_id_by_name(self, project_name: Optional[str]) -> Optional[str]:
        if self.refresh_s is not None:
            self.refresh()
        return self._name_to_id.get(project_name) if project_name is not None else None

    def project_names(self):
        if self.refresh_s is not None:
            self.refresh()
        return list(self._name_to_id)

    def __len__(self) -> int:
        return len(self._graphs)
