"""Project registry operations.

Parity: ``analysis/application/ProjectService.java`` -- ``registerProject``
(``:46-68``, code ``PROJECT_ALREADY_EXISTS``), ``findById`` / ``getById``
(``:76-92``, ``PROJECT_NOT_FOUND``), ``findByRepositoryUrl``, ``listProjects``,
``listByStatus``, ``markAnalysisStarted`` / ``markAnalysisCompleted`` /
``markError`` (``:129-160``) and ``deleteProject`` (``:167-170``).  The
reference never calls this service; here it backs project deletion over REST
and the CLI, and keeps the graph cache consistent (a deleted project's graph
is evicted, which the reference had no path for).
"""
from __future__ import annotations

import logging
from typing import List, Optional

from ..graph.cache import GraphCache
from ..models.domain import Project, ProjectStatus, RepositoryUrl
from ..store.repositories import Repositories
from ..utils.errors import DomainError

LOG = logging.getLogger(__name__)


class ProjectService:
    def __init__(self, repos: Repositories, cache: Optional[GraphCache] = None) -> None:
        self.repos = repos
        self.cache = cache

    def register_project(self, name: str, repository_url: str, default_branch: Optional[str] = None) -> Project:
        LOG.info("Registering project: %s with repository: %s", name, repository_url)
        url = RepositoryUrl.of(repository_url)
        if self.repos.projects.exists_by_repository_url(url):
            raise DomainError("A project with this repository URL already exists", "PROJECT_ALREADY_EXISTS")
        project = Project.create(name, url, default_branch) if default_branch else Project.create(name, url)
        self.repos.projects.save(project)
        return project

    def find_by_id(self, project_id: str) -> Optional[Project]:
        return self.repos.projects.find_by_id(project_id)

    def get_by_id(self, project_id: str) -> Project:
        p = self.find_by_id(project_id)
        if p is None:
            raise DomainError(f"Project not found: {project_id}", "PROJECT_NOT_FOUND")
        return p

    def find_by_repository_url(self, repository_url: str) -> Optional[Project]:
        return self.repos.projects.find_by_repository_url(RepositoryUrl.of(repository_url))

    def list_projects(self) -> List[Project]:
        return self.repos.projects.find_all()

    def list_by_status(self, status: ProjectStatus) -> List[Project]:
        return self.repos.projects.find_by_status(status)

    def mark_analysis_started(self, project_id: str) -> None:
        p = self.get_by_id(project_id)
        p.start_analysis()
        self.repos.projects.update_status(p)

    def mark_analysis_completed(self, project_id: str, commit_hash: str) -> None:
        p = self.get_by_id(project_id)
        p.analysis_completed(commit_hash)
        self.repos.projects.update_status(p)
        LOG.info("Project %s analysis completed for commit: %s", project_id, commit_hash)

    def mark_error(self, project_id: str) -> None:
        p = self.get_by_id(project_id)
        p.mark_error()
        self.repos.projects.update_status(p)
        LOG.warning("Project %s marked as error", project_id)

    def delete_project(self, project_id: str) -> bool:
        """Deletes the project and (FK cascade) its classes, methods and
        parameter links; evicts its graph.  Returns False if it did not exist."""
        p = self.find_by_id(project_id)
        if p is None:
            return False
        if p.status.is_processing():
            raise DomainError(f"Project {p.name} is being processed ({p.status.value})", "PROJECT_BUSY")
        with self.repos.db.transaction():
            self.repos.params.delete_by_project_id(project_id)
            self.repos.methods.delete_by_project_id(project_id)
            self.repos.classes.delete_by_project_id(project_id)
            self.repos.projects.delete(project_id)
        if self.cache is not None:
            self.cache.evict(project_id)
        LOG.info("Project %s (%s) deleted", project_id, p.name)
        return True
