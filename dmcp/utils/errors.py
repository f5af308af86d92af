"""Error types and argument guards (the shared kernel).

Parity: ``shared/DomainException.java:11-69`` (message + error code, default
``DOMAIN_ERROR``) and ``shared/Preconditions.java:26-104`` (guards raising
``IllegalArgumentException`` -> here :class:`ValueError`).
"""
from __future__ import annotations

from typing import Optional, TypeVar

T = TypeVar("T")

DEFAULT_ERROR_CODE = "DOMAIN_ERROR"


class DomainError(Exception):
    """A business-rule failure carrying a machine-readable ``error_code``.

    REST maps it to HTTP 400/500 bodies ``{error, errorCode}``; MCP maps it to
    ``isError=true`` with ``"Error: <message>"`` text.
    """

    def __init__(self, message: str, error_code: str = DEFAULT_ERROR_CODE,
                 cause: Optional[BaseException] = None) -> None:
        super().__init__(message)
        self.message = message
        self.error_code = error_code or DEFAULT_ERROR_CODE
        if cause is not None:
            self.__cause__ = cause

    def __str__(self) -> str:  # keeps "Error: <msg>" formatting identical
        return self.message


def require_non_null(value: Optional[T], message: str) -> T:
    if value is None:
        raise ValueError(message)
    return value


def require_non_blank(value: Optional[str], message: str) -> str:
    if value is None or not isinstance(value, str) or not value.strip():
        raise ValueError(message)
    return value


def require(condition: bool, message: str) -> None:
    if not condition:
        raise ValueError(message)


def require_domain(condition: bool, message: str) -> None:
    if not condition:
        raise DomainError(message)


def require_positive(value: int, message: str) -> int:
    if value <= 0:
        raise ValueError(message)
    return value


def require_non_negative(value: int, message: str) -> int:
    if value < 0:
        raise ValueError(message)
    return value
