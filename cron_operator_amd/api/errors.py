"""Kubernetes API errors (``metav1.Status`` + ``apierrors`` predicates).

Shared by the fake apiserver (raises them), both client transports (map HTTP
responses / in-memory raises onto them) and the reconciler (which tests
``is_not_found``/``is_already_exists`` exactly where the reference calls
``apierrors.IsNotFound``/``IsAlreadyExists``, ``cron_controller.go:98,215,230``).
"""
from __future__ import annotations

from typing import Any, Dict, Optional


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str, details: Optional[Dict[str, Any]] = None,
                 retry_after: Optional[int] = None):
        super().__init__(message)
        self.code = code
        self.reason = reason
        self.message = message
        self.details = details or {}
        # seconds from a Retry-After header / details.retryAfterSeconds (429s, overloaded apiserver)
        self.retry_after = retry_after

    def status(self) -> Dict[str, Any]:
        st: Dict[str, Any] = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                              "message": self.message, "reason": self.reason, "code": self.code}
        details = dict(self.details)
        if self.retry_after is not None:
            details["retryAfterSeconds"] = self.retry_after
        if details:
            st["details"] = details
        return st

    @staticmethod
    def from_status(code: int, body: Any) -> "ApiError":
        if isinstance(body, dict) and body.get("kind") == "Status":
            det = body.get("details") or {}
            ra = det.get("retryAfterSeconds") if isinstance(det, dict) else None
            return ApiError(int(body.get("code") or code), body.get("reason") or _reason_for(code),
                            body.get("message") or "", body.get("details"), ra if isinstance(ra, int) else None)
        text = body if isinstance(body, str) else str(body)
        return ApiError(code, _reason_for(code), text or f"HTTP {code}")

    def __repr__(self) -> str:
        return f"ApiError({self.code}, {self.reason!r}, {self.message!r})"


def _reason_for(code: int) -> str:
    return {400: "BadRequest", 401: "Unauthorized", 403: "Forbidden", 404: "NotFound",
            405: "MethodNotAllowed", 406: "NotAcceptable", 409: "Conflict", 410: "Expired",
            415: "UnsupportedMediaType", 422: "Invalid", 429: "TooManyRequests",
            500: "InternalError", 503: "ServiceUnavailable", 504: "Timeout"}.get(code, "Unknown")


def _qualified(resource: str, group: str) -> str:
    return f"{resource}.{group}" if group else resource


def not_found(resource: str, group: str, name: str) -> ApiError:
    return ApiError(404, "NotFound", f'{_qualified(resource, group)} "{name}" not found',
                    {"name": name, "group": group, "kind": resource})


def already_exists(resource: str, group: str, name: str) -> ApiError:
    return ApiError(409, "AlreadyExists", f'{_qualified(resource, group)} "{name}" already exists',
                    {"name": name, "group": group, "kind": resource})


def conflict(resource: str, group: str, name: str, why: str) -> ApiError:
    return ApiError(409, "Conflict", f'Operation cannot be fulfilled on {_qualified(resource, group)} "{name}": '
                                     f"{why}", {"name": name, "group": group, "kind": resource})


def invalid(kind: str, group: str, name: str, causes: list) -> ApiError:
    msg = "; ".join(f"{c.get('field')}: {c.get('message')}" for c in causes)
    return ApiError(422, "Invalid", f'{kind}.{group} "{name}" is invalid: {msg}' if group else
                    f'{kind} "{name}" is invalid: {msg}',
                    {"name": name, "group": group, "kind": kind, "causes": causes})


def bad_request(msg: str) -> ApiError:
    return ApiError(400, "BadRequest", msg)


def gone(msg: str) -> ApiError:
    return ApiError(410, "Expired", msg)


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, ApiError) and (e.reason == "NotFound" or (e.code == 404 and e.reason in ("", "Unknown")))


def is_already_exists(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "AlreadyExists"


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "Conflict"


def is_gone(e: BaseException) -> bool:
    return isinstance(e, ApiError) and (e.code == 410 or e.reason in ("Expired", "Gone"))


def is_invalid(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "Invalid"


def ignore_not_found(e: Optional[BaseException]) -> Optional[BaseException]:
    return None if e is None or is_not_found(e) else e
