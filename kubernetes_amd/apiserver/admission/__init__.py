"""Admission framework: ordered chains of mutating then validating plugins.

Parity: `staging/src/k8s.io/apiserver/pkg/admission` (`Interface`, `MutationInterface`,
`ValidationInterface`, `Attributes`, plugin registry by name) and the
`--admission-control` ordered list (`cmd/kube-apiserver/app/options/plugins.go:51,82`).
"""
from __future__ import annotations

CREATE, UPDATE, DELETE, CONNECT = "CREATE", "UPDATE", "DELETE", "CONNECT"


class AdmissionError(Exception):
    def __init__(self, message, code=403, reason="Forbidden"):
        super().__init__(message)
        self.code = code
        self.reason = reason


class Attributes:
    __slots__ = ("operation", "resource", "subresource", "namespace", "name", "obj", "old", "user", "kind", "options",
                 "prefetched")

    def __init__(self, operation, resource, subresource, namespace, name, obj, old=None, user=None, kind="", options=None):
        self.operation = operation
        self.resource = resource
        self.subresource = subresource
        self.namespace = namespace
        self.name = name
        self.obj = obj
        self.old = old
        self.user = user
        self.kind = kind
        self.options = options
        self.prefetched = None   # objects the server read ahead for plugins (uncached resources)


class Plugin:
    name = ""
    operations = (CREATE, UPDATE, DELETE, CONNECT)

    def __init__(self, server=None, config=None):
        self.server = server
        self.config = config or {}

    def handles(self, op):
        return op in self.operations

    # Mutating plugins override admit(); validating plugins override validate().
    def admit(self, a: Attributes):
        return None

    def validate(self, a: Attributes):
        return None


REGISTRY: dict[str, type] = {}


def register(cls):
    REGISTRY[cls.name] = cls
    return cls


class Chain:
    def __init__(self, plugins):
        self.plugins = plugins
        self._mut = [p for p in plugins if type(p).admit is not Plugin.admit]
        self._val = [p for p in plugins if type(p).validate is not Plugin.validate]
        self._charge = [p for p in plugins if hasattr(p, "charge")]
        self._prepare = [p for p in plugins if hasattr(p, "prepare")]
        self.names = {getattr(p, "name", "") for p in plugins}

    async def prepare(self, a: Attributes):
        """Mutating plugins that need an API round trip before the rest of the chain
        (NamespaceAutoProvision creates the namespace)."""
        for p in self._prepare:
            if p.handles(a.operation):
                await p.prepare(a)

    def admit(self, a: Attributes):
        for p in self._mut:
            if p.handles(a.operation):
                p.admit(a)

    def validate(self, a: Attributes):
        for p in self._val:
            if p.handles(a.operation):
                p.validate(a)

    async def charge(self, a: Attributes):
        """Validating plugins whose decision needs an API round trip (ResourceQuota writes the
        charged usage to the quota object); the last step before the object is committed."""
        for p in self._charge:
            if p.handles(a.operation):
                await p.charge(a)


DEFAULT_PLUGINS = [
    "NamespaceLifecycle", "LimitRanger", "ServiceAccount", "DefaultTolerationSeconds",
    "Priority", "ResourceV2", "ExtendedResourceToleration", "DefaultStorageClass", "NodeRestriction",
    "MutatingAdmissionWebhook", "ValidatingAdmissionWebhook", "ResourceQuota",
]


def new_chain(names, server=None, configs=None):
    from . import estimation, limitranger, plugins, security  # noqa: F401 - registers built-ins
    configs = configs or {}
    out = []
    for n in names:
        if n not in REGISTRY:
            raise ValueError(f"unknown admission plugin {n!r}")
        out.append(REGISTRY[n](server, configs.get(n)))
    return Chain(out)
