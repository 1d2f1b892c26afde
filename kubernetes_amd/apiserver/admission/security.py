"""Security and policy admission plugins.

  * PodSecurityPolicy — `plugin/pkg/admission/security/podsecuritypolicy/admission.go` +
    `pkg/security/podsecuritypolicy`: the pod must validate against at least one PSP the
    requesting user (or the pod's service account) may `use`; the first policy (by name) that
    validates without mutation wins, else the first that validates after defaulting
    (runAsUser MustRunAs range default, default add-capabilities, read-only root fs default);
    the chosen policy is recorded in annotation `kubernetes.io/psp`. Checked fields: privileged,
    hostNetwork / hostPID / hostIPC, hostPorts ranges, volume types (`*` allowed),
    allowedHostPaths prefixes, allowed / required-drop capabilities, runAsUser
    (MustRunAs ranges / MustRunAsNonRoot / RunAsAny), readOnlyRootFilesystem,
    allowPrivilegeEscalation. MI355X: a PSP can forbid device access by volume type (hostPath
    `/dev`) — GPU devices themselves are injected by the kubelet only for allocated IDs.
  * PodPreset — `plugin/pkg/admission/podpreset/admission.go`: presets whose selector matches
    the pod's labels merge env / envFrom / volumes / volumeMounts into every container (conflicts
    reject the preset), annotation `podpreset.admission.kubernetes.io/podpreset-<name>: <rv>`;
    opt-out annotation `podpreset.admission.kubernetes.io/exclude: "true"`.
  * EventRateLimit — `plugin/pkg/admission/eventratelimit`: token buckets on event writes per
    Server / Namespace / User / SourceAndObject (qps, burst, LRU cacheSize); over the limit -> 429.
  * PodTolerationRestriction — `plugin/pkg/admission/podtolerationrestriction`: namespace (or
    cluster-config) default tolerations are merged in (conflicts refuse the pod), non-BestEffort
    pods tolerate memory pressure, and the tolerations whitelist is enforced in both phases.
  * DenyEscalatingExec / DenyExecOnPrivileged — `plugin/pkg/admission/exec`: no exec/attach into
    privileged or host-namespace pods.
  * SecurityContextDeny — `plugin/pkg/admission/securitycontext/scdeny`: rejects pods setting
    SELinux options / runAsUser / supplementalGroups / fsGroup.
  * OwnerReferencesPermissionEnforcement — `plugin/pkg/admission/gc`: setting
    `blockOwnerDeletion` requires `update` on the owner's `finalizers` subresource.
  * ImagePolicyWebhook — `plugin/pkg/admission/imagepolicy`: an ImageReview is POSTed to a
    kubeconfig-named backend, answers cached per allow/deny TTL, transient failures retried;
    default-deny on backend failure unless `defaultAllow` (failed-open annotation).
"""
from __future__ import annotations

import json
import time

from ...api.labels import label_selector_as_selector
from . import CONNECT, CREATE, UPDATE, AdmissionError, Plugin, register

PSP_ANN = "kubernetes.io/psp"


def _sc(c):
    return c.get("securityContext") or {}


def _containers(spec):
    return list(spec.get("initContainers") or []) + list(spec.get("containers") or [])


def _in_ranges(v, ranges):
    return any(int(r.get("min", 0)) <= v <= int(r.get("max", 0)) for r in ranges or ())


def _only_gc_fields_changed(new, old):
    """rbacregistry.IsOnlyMutatingGCFields: an update touching only ownerReferences / finalizers."""
    if old is None:
        return False

    def strip(o):
        o = dict(o)
        md = dict(o.get("metadata") or {})
        for k in ("ownerReferences", "finalizers", "resourceVersion", "generation"):
            md.pop(k, None)
        o["metadata"] = md
        return o
    return strip(new) == strip(old)


@register
class PodSecurityPolicy(Plugin):
    """`plugin/pkg/admission/security/podsecuritypolicy/admission.go`.

    Policies are taken in name order and each is tried on a copy of the pod (`psp.Provider`:
    default, then validate). Admit (CREATE) keeps the first policy that validates the pod without
    changing it, else the first that validates it after defaulting, among the policies the
    requesting user — or the pod's service account — may `use` (RBAC verb `use` on
    `podsecuritypolicies` in the pod's namespace); the winner is recorded in annotation
    `kubernetes.io/psp`. Validate (CREATE and UPDATE, after every mutating plugin) requires a
    usable policy that accepts the pod unchanged, so a later plugin cannot smuggle in what the
    policy forbids. Updates touching only ownerReferences / finalizers are ignored. With no
    policy at all the pod is refused (failOnNoPolicies, the default; config
    `{"failOnNoPolicies": false}` admits instead). Refusals aggregate the errors of the usable
    policies only.
    """
    name = "PodSecurityPolicy"
    operations = (CREATE, UPDATE)

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        self.fail_on_no_policies = (config or {}).get("failOnNoPolicies", True) is not False

    def _can_use(self, user, name, ns, sa_name):
        from ..auth import AttributesRecord, User
        az = getattr(self.server, "authz", None)
        if az is None:
            return True
        subjects = []
        if sa_name:
            subjects.append(User(f"system:serviceaccount:{ns}:{sa_name}", "",
                                 ["system:serviceaccounts", f"system:serviceaccounts:{ns}", "system:authenticated"]))
        if user is not None:
            subjects.append(user)
        # 1.9 checks the `extensions` group; `policy` (where later releases moved PSPs) is honoured too
        for u in subjects:
            for group in ("extensions", "policy"):
                ok, _ = az.authorize(AttributesRecord(u, "use", ns, "podsecuritypolicies", "", name, group, "", True))
                if ok:
                    return True
        return False

    @staticmethod
    def _ignore(a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return True
        return a.operation == UPDATE and _only_gc_fields_changed(a.obj, a.old)

    def _compute(self, a, mutation_allowed):
        """computeSecurityContext: (allowed pod | None, policy name, errors, fatal message)."""
        import copy
        from .psp import Provider, ProviderError
        pod = a.obj
        policies = sorted(self.server.list_objects("podsecuritypolicies") if self.server else (),
                          key=lambda p: p["metadata"]["name"])
        if not policies and not self.fail_on_no_policies:
            return pod, "", [], None
        providers = []
        for p in policies:
            try:
                providers.append(Provider(p))
            except ProviderError:
                continue
        if not providers:
            return None, "", [], "no providers available to validate pod request"
        sa = (pod.get("spec") or {}).get("serviceAccountName")
        mutated_pod, mutated_name, errors = None, "", {}
        for prov in providers:
            cp = copy.deepcopy(pod)
            errs = prov.assign(cp)
            if errs:
                errors[prov.name] = errs
                continue
            mutated = cp != pod
            if mutated and not mutation_allowed:
                continue
            if not self._can_use(a.user, prov.name, a.namespace, sa):
                continue
            if not mutated:
                return cp, prov.name, [], None
            if mutated_pod is None:
                mutated_pod, mutated_name = cp, prov.name
        if mutated_pod is not None:
            return mutated_pod, mutated_name, [], None
        agg = [f"provider {n}: {e}" for n, errs in errors.items() if self._can_use(a.user, n, a.namespace, sa)
               for e in errs]
        return None, "", agg, None

    def _forbid(self, a, msg):
        md = a.obj.get("metadata") or {}
        raise AdmissionError(f'pods "{md.get("name") or md.get("generateName") or a.name}" is forbidden: {msg}')

    def admit(self, a):
        if self._ignore(a) or a.operation != CREATE:
            return
        allowed, name, errs, fatal = self._compute(a, True)
        if fatal:
            self._forbid(a, fatal)
        if allowed is None:
            self._forbid(a, f"unable to validate against any pod security policy: [{', '.join(errs)}]")
        if allowed is not a.obj:
            a.obj.clear()
            a.obj.update(allowed)
        if name:
            md = a.obj.setdefault("metadata", {})
            md["annotations"] = dict(md.get("annotations") or {}, **{PSP_ANN: name})

    def validate(self, a):
        if self._ignore(a):
            return
        allowed, _, errs, fatal = self._compute(a, False)
        if fatal:
            self._forbid(a, fatal)
        if allowed is None or allowed != a.obj:
            self._forbid(a, f"unable to validate against any pod security policy: [{', '.join(errs)}]")


class PresetConflict(ValueError):
    pass


def _merge_by_name(orig, presets, field, what):
    """mergeEnv / mergeVolumes: keep `orig`, append each preset item whose name is new; an
    item whose name is taken by a different value is a conflict (all conflicts aggregated)."""
    seen = {x["name"]: x for x in orig or ()}
    out, errs = list(orig or ()), []
    for pp in presets:
        for v in (pp.get("spec") or {}).get(field) or ():
            found = seen.get(v["name"])
            if found is None:
                seen[v["name"]] = v
                out.append(v)
            elif found != v:
                errs.append(f"merging {what} for {pp['metadata'].get('name', '')} has a conflict on {v['name']}")
    if errs:
        raise PresetConflict("; ".join(errs))
    return out


def merge_env(env, presets):
    return _merge_by_name(env, presets, "env", "env")


def merge_volumes(volumes, presets):
    out = _merge_by_name(volumes, presets, "volumes", "volumes")
    return out or None


def merge_env_from(env_from, presets):
    out = list(env_from or ())
    for pp in presets:
        out.extend((pp.get("spec") or {}).get("envFrom") or ())
    return out


def merge_volume_mounts(mounts, presets):
    """mergeVolumeMounts: conflicts on the mount name or on the mount path."""
    by_name = {m["name"]: m for m in mounts or ()}
    by_path = {m["mountPath"]: m for m in mounts or ()}
    out, errs = list(mounts or ()), []
    for pp in presets:
        name = pp["metadata"].get("name", "")
        for m in (pp.get("spec") or {}).get("volumeMounts") or ():
            found = by_name.get(m["name"])
            if found is None:
                by_name[m["name"]] = m
                out.append(m)
            elif found != m:
                errs.append(f"merging volume mounts for {name} has a conflict on {m['name']}")
            found = by_path.get(m["mountPath"])
            if found is None:
                by_path[m["mountPath"]] = m
            elif found != m:
                errs.append(f"merging volume mounts for {name} has a conflict on mount path {m['mountPath']}")
    if errs:
        raise PresetConflict("; ".join(errs))
    return out


@register
class PodPreset(Plugin):
    """`plugin/pkg/admission/podpreset/admission.go` (CREATE of pods, not mirror pods, not pods
    annotated `podpreset.admission.kubernetes.io/exclude: "true"`): every PodPreset of the
    namespace whose selector matches the pod's labels is applied — volumes to the pod; env,
    envFrom and volumeMounts to each (regular) container — and recorded as annotation
    `podpreset.admission.kubernetes.io/podpreset-<name>: <resourceVersion>`. The presets are
    applied all together or not at all: any conflict (an env var, volume or mount of the same name
    with a different value, or two mounts on one path — between the pod and a preset or between
    presets) leaves the pod unchanged and admitted, with a warning event like the reference."""
    name = "PodPreset"
    operations = (CREATE,)
    EXCLUDE = "podpreset.admission.kubernetes.io/exclude"
    PREFIX = "podpreset.admission.kubernetes.io"

    def admit(self, a):
        if a.resource != "pods" or a.subresource or a.operation != CREATE or not isinstance(a.obj, dict):
            return
        pod = a.obj
        md = pod.setdefault("metadata", {})
        anns = md.get("annotations") or {}
        if "kubernetes.io/config.mirror" in anns or anns.get(self.EXCLUDE) == "true":
            return
        presets = [pp for pp in sorted(self.server.list_objects("podpresets", a.namespace) if self.server else (),
                                       key=lambda p: p["metadata"]["name"])
                   if label_selector_as_selector((pp.get("spec") or {}).get("selector")).matches(md.get("labels") or {})]
        if not presets:
            return
        self.apply(pod, presets)

    @classmethod
    def apply(cls, pod, presets) -> bool:
        """safeToApplyPodPresetsOnPod + applyPodPresetsOnPod; False (pod untouched) on conflict."""
        spec = pod.setdefault("spec", {})
        try:
            volumes = merge_volumes(spec.get("volumes"), presets)
            merged = [(merge_env(c.get("env"), presets), merge_volume_mounts(c.get("volumeMounts"), presets),
                       merge_env_from(c.get("envFrom"), presets)) for c in spec.get("containers") or ()]
        except PresetConflict as e:
            import logging
            logging.getLogger("admission.podpreset").warning(
                "conflict occurred while applying podpresets: %s on pod: %s err: %s",
                ",".join(p["metadata"]["name"] for p in presets), (pod.get("metadata") or {}).get("name"), e)
            return False
        if volumes is not None:
            spec["volumes"] = volumes
        for c, (env, mounts, env_from) in zip(spec.get("containers") or (), merged):
            for k, v in (("env", env), ("volumeMounts", mounts), ("envFrom", env_from)):
                if v:
                    c[k] = v
        md = pod.setdefault("metadata", {})
        md["annotations"] = dict(md.get("annotations") or {})
        for pp in presets:
            md["annotations"][f"{cls.PREFIX}/podpreset-{pp['metadata']['name']}"] = \
                pp["metadata"].get("resourceVersion", "")
        return True


class _Bucket:
    """flowcontrol token bucket (qps refill, `burst` capacity, starts full)."""

    def __init__(self, qps, burst, clock=time.monotonic):
        self.qps, self.burst, self.clock = float(qps), float(burst), clock
        self.tokens, self.t = float(burst), clock()

    def take(self):
        now = self.clock()
        self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
        self.t = now
        if self.tokens >= 1:
            self.tokens -= 1
            return True
        return False


EVENT_LIMIT_TYPES = ("Server", "Namespace", "User", "SourceAndObject")
DEFAULT_EVENT_CACHE_SIZE = 4096


def validate_event_rate_limit_config(cfg) -> list[str]:
    """eventratelimit/apis/eventratelimit/validation ValidateConfiguration."""
    errs = []
    limits = (cfg or {}).get("limits") or []
    if not limits:
        errs.append("limits: Invalid value: must not be empty")
    for i, lim in enumerate(limits):
        t = lim.get("type")
        if t not in EVENT_LIMIT_TYPES:
            errs.append(f"limits[{i}].type: Unsupported value: {t!r}: supported values: "
                        + ", ".join(f'"{x}"' for x in EVENT_LIMIT_TYPES))
        if int(lim.get("burst") or 0) <= 0:
            errs.append(f"limits[{i}].burst: Invalid value: {lim.get('burst')}: must be positive")
        if float(lim.get("qps") or 0) <= 0:     # int32 in the reference; fractions allowed here
            errs.append(f"limits[{i}].qps: Invalid value: {lim.get('qps')}: must be positive")
        if t != "Server" and int(lim.get("cacheSize") or 0) < 0:
            errs.append(f"limits[{i}].cacheSize: Invalid value: {lim.get('cacheSize')}: must not be negative")
    return errs


def _source_and_object_key(a):
    ev = a.obj if isinstance(a.obj, dict) else {}
    src, io = ev.get("source") or {}, ev.get("involvedObject") or {}
    return "".join(str(x or "") for x in (src.get("component"), src.get("host"), io.get("kind"), io.get("namespace"),
                                           io.get("name"), io.get("uid"), io.get("apiVersion")))


class _LimitEnforcer:
    """eventratelimit/limitenforcer.go: one bucket (Server) or an LRU of per-key buckets."""

    KEYS = {"Server": lambda a: "", "Namespace": lambda a: a.namespace or "",
            "User": lambda a: getattr(a.user, "name", "") if a.user is not None else "",
            "SourceAndObject": _source_and_object_key}

    def __init__(self, lim, clock):
        from collections import OrderedDict
        self.type = lim["type"]
        self.qps, self.burst, self.clock = lim["qps"], lim["burst"], clock
        self.key = self.KEYS[self.type]
        self.size = int(lim.get("cacheSize") or 0) or DEFAULT_EVENT_CACHE_SIZE
        self.single = _Bucket(self.qps, self.burst, clock) if self.type == "Server" else None
        self.cache: OrderedDict = OrderedDict()

    def accept(self, a):
        k = self.key(a)
        b = self.single
        if b is None:
            b = self.cache.get(k)
            if b is None:
                b = self.cache[k] = _Bucket(self.qps, self.burst, self.clock)
                if len(self.cache) > self.size:
                    self.cache.popitem(last=False)
            else:
                self.cache.move_to_end(k)
        if not b.take():
            return f"limit reached on type {self.type} for key {k}"
        return None


@register
class EventRateLimit(Plugin):
    """`plugin/pkg/admission/eventratelimit`: events (CREATE and UPDATE) pass one token bucket
    per configured limit — Server, per Namespace, per User or per SourceAndObject (the event's
    source component + host and involved object kind / namespace / name / uid / apiVersion),
    the per-key buckets held in an LRU of `cacheSize` (default 4096). Every limit is charged
    even when an earlier one refuses; any refusal is a 429. The config is validated like the
    reference (at least one limit, known types, positive qps / burst, non-negative cacheSize)."""
    name = "EventRateLimit"
    operations = (CREATE, UPDATE)

    def __init__(self, server=None, config=None, clock=time.monotonic):
        super().__init__(server, config)
        errs = validate_event_rate_limit_config(config)
        if errs:
            raise ValueError("EventRateLimit: " + "; ".join(errs))
        self.enforcers = [_LimitEnforcer(lim, clock) for lim in config["limits"]]

    def validate(self, a):
        if a.resource != "events" or a.subresource:
            return
        err = None
        for e in self.enforcers:
            err = e.accept(a) or err
        if err:
            raise AdmissionError(err, 429, "TooManyRequests")


MEMORY_PRESSURE_TAINT = "node.kubernetes.io/memory-pressure"


def _tol_key(t):
    return (t.get("key", ""), t.get("effect", ""))


def _tol_equal(a, b):
    """pkg/util/tolerations AreEqual: key, operator, value, effect and tolerationSeconds."""
    return (a.get("key", ""), a.get("operator", "") or "", a.get("value", ""), a.get("effect", ""),
            a.get("tolerationSeconds")) == (b.get("key", ""), b.get("operator", "") or "", b.get("value", ""),
                                            b.get("effect", ""), b.get("tolerationSeconds"))


def tolerations_conflict(first, second) -> bool:
    """IsConflict: a (key, effect) present in both with different tolerations."""
    sm = {_tol_key(t): t for t in second}
    return any(_tol_key(t) in sm and not _tol_equal(t, sm[_tol_key(t)]) for t in first)


def merge_tolerations(first, second) -> list:
    """MergeTolerations: `second`, plus the (key, effect) entries of `first` it lacks."""
    have = {_tol_key(t) for t in second}
    out = list(second)
    for k, t in {_tol_key(t): t for t in first}.items():
        if k not in have:
            out.append(t)
    return out


def verify_against_whitelist(tolerations, whitelist) -> bool:
    """VerifyAgainstWhitelist: every (key, effect) of the pod is whitelisted with an equal toleration."""
    if not whitelist:
        return True
    w = {_tol_key(t): t for t in whitelist}
    return all(_tol_key(t) in w and _tol_equal(t, w[_tol_key(t)]) for t in tolerations)


@register
class PodTolerationRestriction(Plugin):
    """`plugin/pkg/admission/podtolerationrestriction/admission.go`.

    Admit (CREATE, or UPDATE of a pod whose initializers are pending): the namespace's
    `scheduler.alpha.kubernetes.io/defaultTolerations` — or, when the annotation is absent, the
    cluster `default` from the plugin config (an empty annotation overrides it) — is merged into
    the pod's tolerations; a (key, effect) both define differently refuses the pod ("namespace
    tolerations and pod tolerations conflict"). Non-BestEffort pods also tolerate
    `node.kubernetes.io/memory-pressure:NoSchedule`. Validate (CREATE and UPDATE): the pod's
    tolerations must be in the namespace's `tolerationsWhitelist` (cluster `whitelist` when the
    annotation is absent; an empty list allows everything). Config (`--admission-control-config-
    file`): `{"default": [...], "whitelist": [...]}`.
    """
    name = "PodTolerationRestriction"
    operations = (CREATE, UPDATE)
    DEFAULT = "scheduler.alpha.kubernetes.io/defaultTolerations"
    WHITELIST = "scheduler.alpha.kubernetes.io/tolerationsWhitelist"

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        cfg = config or {}
        self.cluster_default = list(cfg.get("default") or ())
        self.cluster_whitelist = list(cfg.get("whitelist") or ())

    @staticmethod
    def _ignore(a):
        return a.resource != "pods" or a.subresource or not isinstance(a.obj, dict)

    def _namespace(self, name):
        ns = self.server.get_object("namespaces", None, name) if self.server else None
        if ns is None and self.server is not None:
            raise AdmissionError(f'namespaces "{name}" not found', 404, "NotFound")
        return ns or {}

    def _ns_tolerations(self, ns, key):
        """extractNSTolerations: None when unset, [] when empty, else the parsed list."""
        ann = (ns.get("metadata") or {}).get("annotations") or {}
        if key not in ann:
            return None
        if not ann[key]:
            return []
        try:
            ts = json.loads(ann[key])
        except ValueError as e:
            raise AdmissionError(f"invalid {key} annotation: {e}", 500, "InternalError")
        if not isinstance(ts, list):
            raise AdmissionError(f"invalid {key} annotation: not a list", 500, "InternalError")
        return ts

    def admit(self, a):
        if self._ignore(a):
            return
        spec = a.obj.setdefault("spec", {})
        final = list(spec.get("tolerations") or ())
        updating_uninit = a.operation == UPDATE and a.old is not None and \
            ((a.old.get("metadata") or {}).get("initializers") or {}).get("pending")
        if a.operation == CREATE or updating_uninit:
            ts = self._ns_tolerations(self._namespace(a.namespace), self.DEFAULT)
            if ts is None:
                ts = self.cluster_default
            if ts:
                if final:
                    if tolerations_conflict(ts, final):
                        raise AdmissionError("namespace tolerations and pod tolerations conflict")
                    final = merge_tolerations(ts, final)
                else:
                    final = list(ts)
        from ..registry import qos_class
        if qos_class(a.obj) != "BestEffort":
            final = merge_tolerations(final, [{"key": MEMORY_PRESSURE_TAINT, "operator": "Exists",
                                               "effect": "NoSchedule"}])
        if final or "tolerations" in spec:
            spec["tolerations"] = final
        self.validate(a)

    def validate(self, a):
        if self._ignore(a):
            return
        tols = (a.obj.get("spec") or {}).get("tolerations") or ()
        if not tols:
            return
        wl = self._ns_tolerations(self._namespace(a.namespace), self.WHITELIST)
        if wl is None:
            wl = self.cluster_whitelist
        if wl and not verify_against_whitelist(tols, wl):
            raise AdmissionError("pod tolerations (possibly merged with namespace default tolerations) conflict "
                                 "with its namespace whitelist")


@register
class DenyEscalatingExec(Plugin):
    name = "DenyEscalatingExec"
    operations = (CONNECT, CREATE)

    def validate(self, a):
        if a.resource != "pods" or a.subresource not in ("exec", "attach"):
            return
        pod = a.old if a.old is not None else (self.server.get_object("pods", a.namespace, a.name) if self.server else None)
        if pod is None:
            return
        spec = pod.get("spec") or {}
        if spec.get("hostPID") or spec.get("hostIPC"):
            raise AdmissionError("cannot exec into or attach to a container using host pid or ipc")
        if any(_sc(c).get("privileged") for c in _containers(spec)):
            raise AdmissionError("cannot exec into or attach to a privileged container")


@register
class DenyExecOnPrivileged(DenyEscalatingExec):
    """`plugin/pkg/admission/exec` NewDenyExecOnPrivileged (deprecated): only privileged
    containers are protected, host-namespace pods are not."""
    name = "DenyExecOnPrivileged"

    def validate(self, a):
        if a.resource != "pods" or a.subresource not in ("exec", "attach"):
            return
        pod = a.old if a.old is not None else (self.server.get_object("pods", a.namespace, a.name) if self.server else None)
        if pod is not None and any(_sc(c).get("privileged") for c in _containers(pod.get("spec") or {})):
            raise AdmissionError("cannot exec into or attach to a privileged container")


@register
class SecurityContextDeny(Plugin):
    name = "SecurityContextDeny"
    operations = (CREATE, UPDATE)

    def validate(self, a):
        if a.resource != "pods" or a.subresource or a.obj is None:
            return
        spec = a.obj.get("spec") or {}
        psc = spec.get("securityContext") or {}
        for f in ("supplementalGroups", "seLinuxOptions", "runAsUser", "fsGroup"):
            if f in psc:
                raise AdmissionError(f"pod.Spec.SecurityContext.{f} is forbidden")
        for c in _containers(spec):
            for f in ("seLinuxOptions", "runAsUser"):
                if f in _sc(c):
                    raise AdmissionError(f"SecurityContext.{f} is forbidden")


@register
class OwnerReferencesPermissionEnforcement(Plugin):
    name = "OwnerReferencesPermissionEnforcement"
    operations = (CREATE, UPDATE)

    def validate(self, a):
        if a.obj is None or a.subresource:
            return
        new = [r for r in (a.obj.get("metadata") or {}).get("ownerReferences") or () if r.get("blockOwnerDeletion")]
        old = {r.get("uid") for r in ((a.old or {}).get("metadata") or {}).get("ownerReferences") or () if r.get("blockOwnerDeletion")}
        added = [r for r in new if r.get("uid") not in old]
        if not added:
            return
        from ...api import meta as m
        from ..auth import AttributesRecord
        for r in added:
            ri = m.BY_KIND.get(r.get("kind"))
            if ri is None:
                continue
            ok, _ = self.server.authz.authorize(AttributesRecord(a.user, "update", a.namespace if ri.namespaced else "",
                                                                 ri.plural, "finalizers", r.get("name", ""), ri.group, "", True))
            if not ok:
                raise AdmissionError(f"cannot set blockOwnerDeletion if an ownerReference refers to a resource you can't set "
                                     f"finalizers on: User \"{getattr(a.user, 'name', '')}\" cannot update {ri.plural}/finalizers")


# ImagePolicyWebhook config bounds, seconds (imagepolicy/config.go:27-41)
DEFAULT_RETRY_BACKOFF, MIN_RETRY_BACKOFF, MAX_RETRY_BACKOFF = 0.5, 1e-9, 300.0
DEFAULT_ALLOW_TTL, MIN_ALLOW_TTL, MAX_ALLOW_TTL = 300.0, 1.0, 1800.0
DEFAULT_DENY_TTL, MIN_DENY_TTL, MAX_DENY_TTL = 30.0, 1.0, 1800.0
IMAGE_POLICY_FAILED_OPEN = "alpha.image-policy.k8s.io/failed-open"


def normalize_config_duration(name, scale, value, lo, hi, default):
    """config.go normalizeConfigDuration: -1 disables (0), 0 takes the default, otherwise the
    number is in units of `scale` seconds and must land in [lo, hi]."""
    value = int(value or 0)
    if value == -1:
        return 0.0
    if value == 0:
        return default
    v = value * scale
    if v < lo or v > hi:
        raise ValueError(f"image policy webhook {name}: valid value is between {lo}s and {hi}s, got {v}s")
    return v


def normalize_image_policy_config(cfg: dict) -> dict:
    """config.go normalizeWebhookConfig: retryBackoff in ms, allowTTL / denyTTL in seconds."""
    out = dict(cfg)
    out["retryBackoff"] = normalize_config_duration("backoff", 1e-3, cfg.get("retryBackoff"), MIN_RETRY_BACKOFF,
                                                    MAX_RETRY_BACKOFF, DEFAULT_RETRY_BACKOFF)
    out["allowTTL"] = normalize_config_duration("allow cache", 1.0, cfg.get("allowTTL"), MIN_ALLOW_TTL,
                                                MAX_ALLOW_TTL, DEFAULT_ALLOW_TTL)
    out["denyTTL"] = normalize_config_duration("deny cache", 1.0, cfg.get("denyTTL"), MIN_DENY_TTL,
                                               MAX_DENY_TTL, DEFAULT_DENY_TTL)
    return out


class _WebhookFailure(Exception):
    def __init__(self, message, transient=False):
        super().__init__(message)
        self.transient = transient


@register
class ImagePolicyWebhook(Plugin):
    """`plugin/pkg/admission/imagepolicy/admission.go`.

    Config (`--admission-control-config-file`, :190-260): `{"imagePolicy": {kubeConfigFile,
    allowTTL, denyTTL, retryBackoff, defaultAllow}}`; the kubeconfig names the backend and its TLS
    material, resolved like a webhook kubeconfig (the current context, or the unnamed cluster and
    user when there is none). For each pod CREATE / UPDATE an ImageReview (containers then init
    containers, annotations filtered to `*.image-policy.k8s.io/*`, namespace) is POSTed; answers
    are cached in a 1024-entry LRU keyed by the review spec for allowTTL / denyTTL; transport
    errors, 5xx and 429 are retried with exponential backoff (`util/webhook` factor 1.5, 5
    steps); a non-2xx answer is an error. On backend failure the pod is refused, unless
    `defaultAllow`, which admits it annotated `alpha.image-policy.k8s.io/failed-open: "true"`.

    The backend call runs in the async `charge` step (off the event loop, like the reference's
    per-request goroutine), so a slow backend never stalls other requests; list the plugin before
    ResourceQuota so a refused pod is not charged. A flat `{"url": ...}` config is accepted for
    plain-HTTP test backends.
    """
    name = "ImagePolicyWebhook"
    operations = (CREATE, UPDATE)

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        if config is None:
            raise ValueError("ImagePolicyWebhook: no config specified")
        cfg = normalize_image_policy_config(config.get("imagePolicy", config))
        self.ssl = None
        self.url = cfg.get("url")
        if cfg.get("kubeConfigFile"):
            from ...client import clientcmd
            r = clientcmd.resolve_webhook(cfg["kubeConfigFile"])
            self.url, self.ssl = r.server, r.ssl_context
        if not self.url:
            raise ValueError("ImagePolicyWebhook: no backend (kubeConfigFile) configured")
        self.allow_ttl, self.deny_ttl = cfg["allowTTL"], cfg["denyTTL"]
        self.retry_backoff = cfg["retryBackoff"]
        self.default_allow = bool(cfg.get("defaultAllow", False))
        self.timeout = float(cfg.get("timeout", 30.0))
        from collections import OrderedDict
        self.cache: OrderedDict[str, tuple] = OrderedDict()
        self.cache_size = 1024

    def _review(self, a):
        pod = a.obj
        spec = pod.get("spec") or {}
        ctrs = list(spec.get("containers") or ()) + list(spec.get("initContainers") or ())
        anns = (pod.get("metadata") or {}).get("annotations") or {}
        return {"containers": [{"image": c.get("image", "")} for c in ctrs],
                "annotations": {k: v for k, v in anns.items() if ".image-policy.k8s.io/" in k},
                "namespace": a.namespace or ""}

    def _cached(self, key):
        hit = self.cache.get(key)
        if hit is None:
            return None
        status, expires = hit
        if time.monotonic() >= expires:
            del self.cache[key]
            return None
        self.cache.move_to_end(key)
        return status

    def _remember(self, key, status):
        ttl = self.allow_ttl if status.get("allowed") else self.deny_ttl
        if ttl <= 0:
            return
        self.cache[key] = (status, time.monotonic() + ttl)
        self.cache.move_to_end(key)
        while len(self.cache) > self.cache_size:
            self.cache.popitem(last=False)

    def _post(self, body: bytes) -> dict:
        import urllib.error
        import urllib.request
        req = urllib.request.Request(self.url, body, {"Content-Type": "application/json",
                                                      "Accept": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout, context=self.ssl) as r:
                data = r.read()
        except urllib.error.HTTPError as e:
            raise _WebhookFailure(f"Error contacting webhook: {e.code}",
                                  transient=e.code >= 500 or e.code == 429 or bool(e.headers.get("Retry-After")))
        except (OSError, ValueError) as e:
            raise _WebhookFailure(f"error contacting webhook: {e}", transient=True)
        try:
            return json.loads(data).get("status") or {}
        except (ValueError, AttributeError) as e:
            raise _WebhookFailure(f"bad webhook response: {e}")

    def _post_with_backoff(self, body: bytes) -> dict:
        """util/webhook WithExponentialBackoff: transient failures are retried."""
        import random
        delay = self.retry_backoff
        for step in range(5):
            try:
                return self._post(body)
            except _WebhookFailure as e:
                if not e.transient or step == 4:
                    raise
            time.sleep(delay * (1 + 0.2 * random.random()))
            delay *= 1.5
        raise AssertionError("unreachable")

    async def charge(self, a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return
        spec = self._review(a)
        key = json.dumps(spec, sort_keys=True)
        status = self._cached(key)
        if status is None:
            body = json.dumps({"apiVersion": "imagepolicy.k8s.io/v1alpha1", "kind": "ImageReview",
                               "spec": spec}).encode()
            import asyncio
            try:
                status = await asyncio.get_running_loop().run_in_executor(None, self._post_with_backoff, body)
            except _WebhookFailure as e:
                if self.default_allow:
                    md = a.obj.setdefault("metadata", {})
                    md["annotations"] = dict(md.get("annotations") or {}, **{IMAGE_POLICY_FAILED_OPEN: "true"})
                    return
                raise AdmissionError(f'pods "{_pod_name(a)}" is forbidden: {e}')
            self._remember(key, status)
        if not status.get("allowed"):
            why = (f"image policy webhook backend denied one or more images: {status['reason']}"
                   if status.get("reason") else "one or more images rejected by webhook backend")
            raise AdmissionError(f'pods "{_pod_name(a)}" is forbidden: {why}')


def _pod_name(a):
    md = a.obj.get("metadata") or {}
    return md.get("name") or md.get("generateName") or a.name or ""
