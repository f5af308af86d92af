"""Domain model: projects, classes, methods, parameters and their value objects.

Parity map (reference paths relative to ``src/main/java/co/fanki/domainmcp``):

* :class:`ClassType`           -- ``analysis/domain/ClassType.java:16-93``
* :class:`ProjectStatus` FSM   -- ``project/domain/ProjectStatus.java:13-42``,
  ``project/domain/ProjectStateMachine.java:34-70``
* :class:`RepositoryUrl`       -- ``project/domain/RepositoryUrl.java:19-87``
  (extended: ``file://`` URLs and absolute local paths are accepted so an
  offline host can index local git repositories)
* :class:`Project`             -- ``project/domain/Project.java:50-205``
* :class:`SourceClass`         -- ``analysis/domain/SourceClass.java:68-161``
* :class:`SourceMethod`        -- ``analysis/domain/SourceMethod.java:74-147``
* :class:`MethodParameter`     -- ``analysis/domain/MethodParameter.java:52-62``
* :class:`StaticMethodInfo`    -- ``analysis/domain/StaticMethodInfo.java:23-42``
* :class:`GitDiffResult`       -- ``analysis/domain/GitDiffResult.java:38-72``
"""
from __future__ import annotations

import enum
import re
import uuid
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import FrozenSet, Iterable, List, NamedTuple, Optional, Tuple

from ..utils.errors import (DomainError, require, require_non_blank,
                            require_non_negative, require_non_null)


def new_id() -> str:
    return str(uuid.uuid4())


def new_ids(n: int) -> List[str]:
    """``n`` UUID strings for a batch of new rows.  The native generator emits
    time-ordered version-7 UUIDs (ordered within the batch) so bulk inserts
    append to the primary-key B-trees; the reference used random UUID4s."""
    if n <= 0:
        return []
    try:
        from .. import _srcscan  # type: ignore
        return _srcscan.uuid7_batch(n)
    except (ImportError, AttributeError):
        return [str(uuid.uuid4()) for _ in range(n)]


def utc_now() -> datetime:
    return datetime.now(timezone.utc)


# --------------------------------------------------------------------------
# ClassType
# --------------------------------------------------------------------------
class ClassType(str, enum.Enum):
    CONTROLLER = "CONTROLLER"
    SERVICE = "SERVICE"
    REPOSITORY = "REPOSITORY"
    ENTITY = "ENTITY"
    DTO = "DTO"
    CONFIGURATION = "CONFIGURATION"
    LISTENER = "LISTENER"
    UTILITY = "UTILITY"
    EXCEPTION = "EXCEPTION"
    OTHER = "OTHER"

    @property
    def description(self) -> str:
        return _CLASS_TYPE_DESCRIPTIONS[self]

    @classmethod
    def from_string(cls, value: Optional[str]) -> "ClassType":
        """Case-insensitive lookup that falls back to OTHER (never raises)."""
        if value is None or not str(value).strip():
            return cls.OTHER
        try:
            return cls[str(value).strip().upper()]
        except KeyError:
            return cls.OTHER

    def is_request_handler(self) -> bool:
        return self in (ClassType.CONTROLLER, ClassType.LISTENER)

    def contains_business_logic(self) -> bool:
        return self in (ClassType.SERVICE, ClassType.ENTITY)

    def __str__(self) -> str:
        return self.value


_CLASS_TYPE_DESCRIPTIONS = {
    ClassType.CONTROLLER: "Controller handling HTTP requests",
    ClassType.SERVICE: "Service containing business logic",
    ClassType.REPOSITORY: "Repository for data persistence",
    ClassType.ENTITY: "Domain entity",
    ClassType.DTO: "Data Transfer Object",
    ClassType.CONFIGURATION: "Configuration class",
    ClassType.LISTENER: "Message listener/consumer",
    ClassType.UTILITY: "Utility/helper class",
    ClassType.EXCEPTION: "Exception class",
    ClassType.OTHER: "Other/unclassified",
}


# --------------------------------------------------------------------------
# Project status + state machine
# --------------------------------------------------------------------------
class ProjectStatus(str, enum.Enum):
    PENDING = "PENDING"
    ANALYZING = "ANALYZING"
    ANALYZED = "ANALYZED"
    ERROR = "ERROR"
    SYNCING = "SYNCING"

    def is_processing(self) -> bool:
        return self in (ProjectStatus.ANALYZING, ProjectStatus.SYNCING)

    def __str__(self) -> str:
        return self.value


_TRANSITIONS = {
    ProjectStatus.PENDING: frozenset({ProjectStatus.ANALYZING}),
    ProjectStatus.ANALYZING: frozenset({ProjectStatus.ANALYZED, ProjectStatus.ERROR}),
    ProjectStatus.ANALYZED: frozenset({ProjectStatus.ANALYZING, ProjectStatus.SYNCING}),
    ProjectStatus.SYNCING: frozenset({ProjectStatus.ANALYZED, ProjectStatus.ERROR}),
    ProjectStatus.ERROR: frozenset({ProjectStatus.ANALYZING, ProjectStatus.SYNCING}),
}


def allowed_transitions(from_status: ProjectStatus) -> FrozenSet[ProjectStatus]:
    return _TRANSITIONS.get(from_status, frozenset())


def transition(from_status: ProjectStatus, to_status: ProjectStatus) -> ProjectStatus:
    """Validates a status move; raises ``PROJECT_INVALID_TRANSITION``."""
    require_non_null(from_status, "from status is required")
    require_non_null(to_status, "to status is required")
    if to_status not in allowed_transitions(from_status):
        raise DomainError(f"Invalid transition: {from_status.value} → {to_status.value}",
                          "PROJECT_INVALID_TRANSITION")
    return to_status


# --------------------------------------------------------------------------
# RepositoryUrl
# --------------------------------------------------------------------------
_HTTPS_RE = re.compile(r"^https://[\w.-]+(/[\w.-]+)+\.git$")
_SSH_RE = re.compile(r"^git@[\w.-]+:[\w.-]+(/[\w.-]+)*\.git$")
_FILE_RE = re.compile(r"^file://(/[^\x00]+)$")


class RepositoryUrl:
    """Validated git repository location (value object, hashable)."""

    __slots__ = ("_value",)

    def __init__(self, value: str) -> None:
        require_non_blank(value, "Repository URL cannot be null or blank")
        require(self.is_valid(value), f"Invalid repository URL format: {value}")
        self._value = value

    @classmethod
    def of(cls, url: str) -> "RepositoryUrl":
        return cls(url)

    @staticmethod
    def is_valid(url: str) -> bool:
        if _HTTPS_RE.match(url) or _SSH_RE.match(url):
            return True
        # Offline extension: local repositories by file:// URL or absolute path.
        if _FILE_RE.match(url):
            return True
        return url.startswith("/") and len(url) > 1 and "\x00" not in url

    @property
    def value(self) -> str:
        return self._value

    def is_ssh(self) -> bool:
        return bool(_SSH_RE.match(self._value))

    def is_https(self) -> bool:
        return bool(_HTTPS_RE.match(self._value))

    def is_local(self) -> bool:
        return not (self.is_ssh() or self.is_https())

    def local_path(self) -> Optional[str]:
        if self._value.startswith("file://"):
            return self._value[len("file://"):]
        if self._value.startswith("/"):
            return self._value
        return None

    def repository_name(self) -> str:
        v = self._value.rstrip("/")
        start = max(v.rfind("/"), v.rfind(":"))
        name = v[start + 1:]
        if name.endswith(".git"):
            name = name[:-4]
        return name

    def __eq__(self, other: object) -> bool:
        return isinstance(other, RepositoryUrl) and other._value == self._value

    def __hash__(self) -> int:
        return hash(self._value)

    def __repr__(self) -> str:
        return f"RepositoryUrl({self._value!r})"

    def __str__(self) -> str:
        return self._value


# --------------------------------------------------------------------------
# Project aggregate
# --------------------------------------------------------------------------
class Project:
    """The repository being indexed; status moves only through the FSM."""

    def __init__(self, id: str, name: str, repository_url: RepositoryUrl,
                 default_branch: Optional[str] = "main",
                 created_at: Optional[datetime] = None) -> None:
        self.id = require_non_blank(id, "Project ID is required")
        self.name = require_non_blank(name, "Project name is required")
        self.repository_url = require_non_null(repository_url, "Repository URL is required")
        self.default_branch = default_branch if default_branch is not None else "main"
        self.description: Optional[str] = None
        self.status = ProjectStatus.PENDING
        self.last_analyzed_at: Optional[datetime] = None
        self.last_commit_hash: Optional[str] = None
        self.graph_data: Optional[str] = None
        self.base_package: Optional[str] = None
        self.created_at = created_at or utc_now()
        self.updated_at = self.created_at

    @classmethod
    def create(cls, name: str, repository_url: RepositoryUrl,
               default_branch: Optional[str] = "main") -> "Project":
        return cls(new_id(), name, repository_url, default_branch, utc_now())

    @classmethod
    def reconstitute(cls, id: str, name: str, repository_url: RepositoryUrl,
                     default_branch: Optional[str], description: Optional[str],
                     status: ProjectStatus, last_analyzed_at: Optional[datetime],
                     last_commit_hash: Optional[str], graph_data: Optional[str],
                     created_at: Optional[datetime], updated_at: Optional[datetime],
                     base_package: Optional[str] = None) -> "Project":
        p = cls(id, name, repository_url, default_branch, created_at)
        p.description = description
        p.status = require_non_null(status, "Project status is required")
        p.last_analyzed_at = last_analyzed_at
        p.last_commit_hash = last_commit_hash
        p.graph_data = graph_data
        p.updated_at = updated_at
        p.base_package = base_package
        return p

    def _touch(self) -> None:
        self.updated_at = utc_now()

    def start_analysis(self) -> None:
        self.status = transition(self.status, ProjectStatus.ANALYZING)
        self._touch()

    def analysis_completed(self, commit_hash: str) -> None:
        require_non_blank(commit_hash, "Commit hash is required")
        self.status = transition(self.status, ProjectStatus.ANALYZED)
        now = utc_now()
        self.last_analyzed_at = now
        self.last_commit_hash = commit_hash
        self.updated_at = now

    def start_sync(self) -> None:
        self.status = transition(self.status, ProjectStatus.SYNCING)
        self._touch()

    def sync_completed(self, commit_hash: str) -> None:
        require_non_blank(commit_hash, "Commit hash is required")
        self.status = transition(self.status, ProjectStatus.ANALYZED)
        now = utc_now()
        self.last_analyzed_at = now
        self.last_commit_hash = commit_hash
        self.updated_at = now

    def update_description(self, description: Optional[str]) -> None:
        self.description = description
        self._touch()

    def update_graph_data(self, graph_data: Optional[str]) -> None:
        self.graph_data = graph_data
        self._touch()

    def mark_error(self) -> None:
        self.status = transition(self.status, ProjectStatus.ERROR)
        self._touch()

    def recover_stuck(self) -> bool:
        """Crash recovery (not in the reference): a project left in
        ANALYZING/SYNCING by a dead process is moved to ERROR so it can be
        re-analyzed or synced. Returns True when a move happened."""
        if self.status.is_processing():
            self.mark_error()
            return True
        return False

    def rename(self, new_name: str) -> None:
        self.name = require_non_blank(new_name, "Project name is required")
        self._touch()

    def __repr__(self) -> str:
        return f"Project(id={self.id!r}, name={self.name!r}, status={self.status.value})"


# --------------------------------------------------------------------------
# SourceClass / SourceMethod / MethodParameter
# --------------------------------------------------------------------------
def simple_name_of(full_class_name: str) -> str:
    i = full_class_name.rfind(".")
    return full_class_name if i < 0 else full_class_name[i + 1:]


def package_name_of(full_class_name: str) -> Optional[str]:
    i = full_class_name.rfind(".")
    return None if i < 0 else full_class_name[:i]


@dataclass(slots=True)
class SourceClass:
    id: str
    project_id: str
    full_class_name: str
    simple_name: str
    package_name: Optional[str]
    class_type: ClassType
    description: Optional[str] = None
    source_file: Optional[str] = None
    commit_hash: Optional[str] = None
    created_at: Optional[datetime] = None

    def __post_init__(self) -> None:
        require_non_blank(self.id, "Class ID is required")
        require_non_blank(self.project_id, "Project ID is required")
        require_non_blank(self.full_class_name, "Full class name is required")
        require_non_blank(self.simple_name, "Simple name is required")
        require_non_null(self.class_type, "Class type is required")
        if self.created_at is None:
            self.created_at = utc_now()

    @classmethod
    def create(cls, project_id: str, full_class_name: str, class_type: ClassType,
               description: Optional[str], source_file: Optional[str],
               commit_hash: Optional[str]) -> "SourceClass":
        require_non_blank(full_class_name, "Full class name is required")
        return cls(new_id(), project_id, full_class_name, simple_name_of(full_class_name),
                   package_name_of(full_class_name), class_type, description,
                   source_file, commit_hash, utc_now())

    @classmethod
    def reconstitute(cls, id: str, project_id: str, full_class_name: str, simple_name: str,
                     package_name: Optional[str], class_type: ClassType, description: Optional[str],
                     source_file: Optional[str], commit_hash: Optional[str],
                     created_at: Optional[datetime]) -> "SourceClass":
        return cls(id, project_id, full_class_name, simple_name, package_name, class_type,
                   description, source_file, commit_hash, created_at)

    def belongs_to_package(self, pkg: Optional[str]) -> bool:
        if self.package_name is None or pkg is None:
            return False
        return self.package_name == pkg or self.package_name.startswith(pkg + ".")


@dataclass(slots=True)
class SourceMethod:
    id: str
    class_id: str
    method_name: str
    description: Optional[str] = None
    business_logic: Tuple[str, ...] = ()
    exceptions: Tuple[str, ...] = ()
    http_method: Optional[str] = None
    http_path: Optional[str] = None
    line_number: Optional[int] = None
    created_at: Optional[datetime] = None

    def __post_init__(self) -> None:
        require_non_blank(self.id, "Method ID is required")
        require_non_blank(self.class_id, "Class ID is required")
        require_non_blank(self.method_name, "Method name is required")
        # immutable copies (SourceMethod.java keeps List.copyOf views)
        self.business_logic = tuple(self.business_logic) if self.business_logic else ()
        self.exceptions = tuple(self.exceptions) if self.exceptions else ()
        if self.created_at is None:
            self.created_at = utc_now()

    @classmethod
    def create(cls, class_id: str, method_name: str, description: Optional[str],
               business_logic: Optional[Iterable[str]], exceptions: Optional[Iterable[str]],
               http_method: Optional[str], http_path: Optional[str],
               line_number: Optional[int]) -> "SourceMethod":
        return cls(new_id(), class_id, method_name, description,
                   tuple(business_logic or ()), tuple(exceptions or ()),
                   http_method, http_path, line_number, utc_now())

    @classmethod
    def reconstitute(cls, id: str, class_id: str, method_name: str, description: Optional[str],
                     business_logic: Optional[Iterable[str]], exceptions: Optional[Iterable[str]],
                     http_method: Optional[str], http_path: Optional[str],
                     line_number: Optional[int], created_at: Optional[datetime]) -> "SourceMethod":
        return cls(id, class_id, method_name, description, tuple(business_logic or ()),
                   tuple(exceptions or ()), http_method, http_path, line_number, created_at)

    def is_http_endpoint(self) -> bool:
        return self.http_method is not None and self.http_path is not None

    def http_endpoint(self) -> Optional[str]:
        if not self.is_http_endpoint():
            return None
        return f"{self.http_method} {self.http_path}"


@dataclass(slots=True)
class MethodParameter:
    id: str
    method_id: str
    position: int
    class_id: str
    created_at: Optional[datetime] = None

    def __post_init__(self) -> None:
        require_non_blank(self.id, "Parameter ID is required")
        require_non_blank(self.method_id, "Method ID is required")
        require_non_negative(self.position, "Position must be non-negative")
        require_non_blank(self.class_id, "Class ID is required")
        if self.created_at is None:
            self.created_at = utc_now()

    @classmethod
    def create(cls, method_id: str, position: int, class_id: str) -> "MethodParameter":
        return cls(new_id(), method_id, position, class_id, utc_now())

    @classmethod
    def reconstitute(cls, id: str, method_id: str, position: int, class_id: str,
                     created_at: Optional[datetime]) -> "MethodParameter":
        return cls(id, method_id, position, class_id, created_at)


class StaticMethodInfo(NamedTuple):
    """Parser -> pipeline DTO: one statically extracted method."""

    method_name: str
    line_number: Optional[int]
    http_method: Optional[str] = None
    http_path: Optional[str] = None
    exceptions: tuple = ()

    @classmethod
    def simple(cls, method_name: str, line_number: Optional[int]) -> "StaticMethodInfo":
        return cls(method_name, line_number, None, None, ())


@dataclass(frozen=True, slots=True)
class GitDiffResult:
    new_commit_hash: str
    changed_files: FrozenSet[str]
    deleted_files: FrozenSet[str]
    full_resync_required: bool

    @classmethod
    def full_resync(cls, new_commit_hash: str) -> "GitDiffResult":
        return cls(new_commit_hash, frozenset(), frozenset(), True)

    @classmethod
    def of(cls, new_commit_hash: str, changed: Iterable[str], deleted: Iterable[str]) -> "GitDiffResult":
        return cls(new_commit_hash, frozenset(changed), frozenset(deleted), False)

    def is_affected(self, source_file: str) -> bool:
        return (self.full_resync_required or source_file in self.changed_files
                or source_file in self.deleted_files)
