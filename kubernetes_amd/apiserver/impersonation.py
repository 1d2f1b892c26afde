"""User impersonation: `Impersonate-User`, `Impersonate-Group`, `Impersonate-Extra-<key>`.

Parity: `staging/src/k8s.io/apiserver/pkg/endpoints/filters/impersonation.go` WithImpersonation.
Every impersonated attribute is authorized for the requesting user with verb `impersonate`:
users (`users`, core group), groups (`groups`), service accounts (`serviceaccounts` in the
account's namespace, when the user name is `system:serviceaccount:<ns>:<name>`) and extra
values (`userextras/<key>` in authentication.k8s.io). The request then runs as the new user.
When Impersonate-Group headers are sent they are the COMPLETE group list (each one authorized
above); only when none are sent does a service account gain `system:serviceaccounts` and
`system:serviceaccounts:<ns>` and every impersonated user except `system:anonymous` join
`system:authenticated` (`impersonation.go:66-124`, `groupsSpecified`). Group or extra headers
without Impersonate-User are rejected.
"""
from __future__ import annotations

from .auth import User

SA_PREFIX = "system:serviceaccount:"


class ImpersonationError(Exception):
    def __init__(self, code, message):
        super().__init__(message)
        self.code, self.message = code, message


def _values(headers, name):
    v = headers.get(name)
    if v is None:
        return []
    return [x.strip() for x in (v if isinstance(v, list) else str(v).split(",")) if x.strip()]


def requested(headers) -> bool:
    return any(k.lower().startswith("impersonate-") for k in headers)


def impersonate(headers, user, authorize):
    """-> the user the request runs as. `authorize(user, verb, ns, resource, sub, name, group)`
    raises on denial."""
    name = headers.get("impersonate-user")
    groups = _values(headers, "impersonate-group")
    extras = {k.lower()[len("impersonate-extra-"):]: _values(headers, k) for k in headers
              if k.lower().startswith("impersonate-extra-")}
    if not name:
        if groups or extras:
            raise ImpersonationError(400, "requested impersonation of groups or extra fields without a user")
        return user
    groups_specified = bool(groups)
    new_groups = []
    if name.startswith(SA_PREFIX) and name.count(":") == 3:
        _, _, ns, sa = name.split(":")
        authorize(user, "impersonate", ns, "serviceaccounts", "", sa, "")
        if not groups_specified:
            new_groups = ["system:serviceaccounts", f"system:serviceaccounts:{ns}"]
    else:
        authorize(user, "impersonate", None, "users", "", name, "")
    for g in groups:
        authorize(user, "impersonate", None, "groups", "", g, "")
        if g not in new_groups:
            new_groups.append(g)
    for key, vals in extras.items():
        for v in vals:
            authorize(user, "impersonate", None, "userextras", key, v, "authentication.k8s.io")
    if not groups_specified and name != "system:anonymous" and "system:authenticated" not in new_groups:
        new_groups.append("system:authenticated")
    out = User(name, "", new_groups, impersonated_by=user)
    if extras:
        out.extra = extras          # carried for SubjectAccessReview-style consumers
    return out
