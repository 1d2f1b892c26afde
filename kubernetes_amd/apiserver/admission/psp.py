"""PodSecurityPolicy providers: per-policy strategies that default and validate a pod.

Parity: `pkg/security/podsecuritypolicy` — `provider.go` (CreatePodSecurityContext,
CreateContainerSecurityContext, ValidatePodSecurityContext, ValidateContainerSecurityContext),
`factory.go` (strategy selection) and the strategies:

  * user (`user/{mustrunas,nonroot,runasany}.go`): MustRunAs defaults to the first range's
    min and requires a UID in a range; MustRunAsNonRoot requires runAsNonRoot or a non-zero
    UID (and defaults runAsNonRoot: true when neither is set); RunAsAny;
  * group (`group/{mustrunas,runasany}.go`) for fsGroup and supplementalGroups;
  * selinux (`selinux/{mustrunas,runasany}.go`): MustRunAs defaults and pins user/role/type/level;
  * capabilities (`capabilities/mustrunas.go`): default-add minus the container's drops, union
    the required drops; adds must be default or allowed (`*` allows all); required drops must be
    dropped;
  * apparmor / seccomp (`apparmor/strategy.go`, `seccomp/strategy.go`): default and allowed
    profile annotations on the policy, profiles in pod annotations;
  * sysctl (`sysctl/mustmatchpatterns.go`): the policy annotation
    `security.alpha.kubernetes.io/sysctls` lists allowed patterns (`*` suffix = prefix match;
    absent = all allowed, empty = none);
  * volumes (`util/util.go`): allowed volume types (`*` = all), allowedHostPaths prefixes
    (path-segment aware), allowedFlexVolumes drivers; host ports, host namespaces, privileged,
    readOnlyRootFilesystem, allowPrivilegeEscalation / defaultAllowPrivilegeEscalation.

Pods are plain v1 dicts: host namespaces live in `spec`, the pod security context in
`spec.securityContext`, and a container's effective runAsUser / runAsNonRoot / seLinuxOptions
fall back to the pod's. A provider never adds an empty securityContext, so a pod that needs no
defaulting compares equal to its original (the admission plugin's "not mutated" test).
"""
from __future__ import annotations

import copy
import json

SECCOMP_POD = "seccomp.security.alpha.kubernetes.io/pod"
SECCOMP_CONTAINER_PREFIX = "container.seccomp.security.alpha.kubernetes.io/"
SECCOMP_DEFAULT = "seccomp.security.alpha.kubernetes.io/defaultProfileName"
SECCOMP_ALLOWED = "seccomp.security.alpha.kubernetes.io/allowedProfileNames"
APPARMOR_CONTAINER_PREFIX = "container.apparmor.security.beta.kubernetes.io/"
APPARMOR_DEFAULT = "apparmor.security.beta.kubernetes.io/defaultProfileName"
APPARMOR_ALLOWED = "apparmor.security.beta.kubernetes.io/allowedProfileNames"
PSP_SYSCTLS = "security.alpha.kubernetes.io/sysctls"
POD_SYSCTLS = "security.alpha.kubernetes.io/sysctls"
POD_UNSAFE_SYSCTLS = "security.alpha.kubernetes.io/unsafe-sysctls"

# every volume source a pod may use (`util.GetVolumeFSType`), by its v1 JSON field name
VOLUME_TYPES = ("hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "secret", "nfs",
                "iscsi", "glusterfs", "persistentVolumeClaim", "rbd", "flexVolume", "cinder", "cephfs", "flocker",
                "downwardAPI", "fc", "azureFile", "configMap", "vsphereVolume", "quobyte", "azureDisk",
                "photonPersistentDisk", "storageos", "projected", "portworxVolume", "scaleIO", "csi")


class ProviderError(ValueError):
    """A policy whose strategies cannot be built (factory.go CreateStrategies)."""


def _fmt(v):
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, str):
        return json.dumps(v)
    return str(v)


def invalid(path, value, detail):
    return f"{path}: Invalid value: {_fmt(value)}: {detail}"


def required(path, detail=""):
    return f"{path}: Required value" + (f": {detail}" if detail else "")


def forbidden(path, detail):
    return f"{path}: Forbidden: {detail}"


def _in_ranges(v, ranges):
    return any(int(r.get("min", 0)) <= int(v) <= int(r.get("max", 0)) for r in ranges or ())


def has_path_prefix(path, prefix):
    """util.hasPathPrefix: `/foo` allows `/foo` and `/foo/bar`, not `/foobar`."""
    path, prefix = path.rstrip("/"), prefix.rstrip("/")
    if not path.startswith(prefix):
        return False
    return len(path) == len(prefix) or path[len(prefix)] == "/"


def volume_type(v):
    return next((k for k in VOLUME_TYPES if v.get(k) is not None), None)


class _User:
    def __init__(self, opts):
        self.rule = (opts or {}).get("rule", "RunAsAny")
        self.ranges = (opts or {}).get("ranges") or []
        if self.rule == "MustRunAs" and not self.ranges:
            raise ProviderError("MustRunAsRange requires at least one range")
        if self.rule not in ("MustRunAs", "MustRunAsNonRoot", "RunAsAny"):
            raise ProviderError(f"Unrecognized RunAsUser strategy type {self.rule}")

    def generate(self):
        return int(self.ranges[0]["min"]) if self.rule == "MustRunAs" else None

    def validate(self, path, non_root, uid):
        if self.rule == "MustRunAs":
            if uid is None:
                return [required(f"{path}.runAsUser")]
            if not _in_ranges(uid, self.ranges):
                return [invalid(f"{path}.runAsUser", uid, f"must be in the ranges: {self._ranges()}")]
        elif self.rule == "MustRunAsNonRoot":
            if non_root is None and uid is None:
                return [required(f"{path}.runAsNonRoot", "must be true")]
            if non_root is False:
                return [invalid(f"{path}.runAsNonRoot", False, "must be true")]
            if uid == 0:
                return [invalid(f"{path}.runAsUser", 0, "running with the root UID is forbidden")]
        return []

    def _ranges(self):
        return "[" + " ".join(f"{{{r.get('min')} {r.get('max')}}}" for r in self.ranges) + "]"


class _Group:
    def __init__(self, opts, field):
        self.rule = (opts or {}).get("rule", "RunAsAny")
        self.ranges = (opts or {}).get("ranges") or []
        self.field = field
        if self.rule == "MustRunAs" and not self.ranges:
            raise ProviderError("ranges must be supplied for MustRunAs")
        if self.rule not in ("MustRunAs", "RunAsAny"):
            raise ProviderError(f"Unrecognized {field} strategy type {self.rule}")

    def generate(self):
        return [int(self.ranges[0]["min"])] if self.rule == "MustRunAs" else None

    def generate_single(self):
        return int(self.ranges[0]["min"]) if self.rule == "MustRunAs" else None

    def validate(self, groups):
        if self.rule != "MustRunAs":
            return []
        errs = []
        if not groups:
            errs.append(invalid(self.field, groups or [], "unable to validate empty groups against required ranges"))
        for g in groups or ():
            if not _in_ranges(g, self.ranges):
                errs.append(invalid(self.field, groups, f"{g} is not an allowed group"))
        return errs


class _SELinux:
    def __init__(self, opts):
        self.rule = (opts or {}).get("rule", "RunAsAny")
        self.options = (opts or {}).get("seLinuxOptions")
        if self.rule == "MustRunAs" and self.options is None:
            raise ProviderError("MustRunAs requires SELinuxOptions")
        if self.rule not in ("MustRunAs", "RunAsAny"):
            raise ProviderError(f"Unrecognized SELinuxContext strategy type {self.rule}")

    def generate(self):
        return copy.deepcopy(self.options) if self.rule == "MustRunAs" else None

    def validate(self, path, se):
        if self.rule != "MustRunAs":
            return []
        if se is None:
            return [required(path)]
        errs = []
        for k in ("level", "role", "type", "user"):
            want = self.options.get(k, "")
            if se.get(k, "") != want:
                errs.append(invalid(f"{path}.{k}", se.get(k, ""), f"must be {want}"))
        return errs


class _Capabilities:
    def __init__(self, default_add, required_drop, allowed):
        self.default_add = list(default_add or ())
        self.required_drop = list(required_drop or ())
        self.allowed = list(allowed or ())

    def generate(self, container):
        caps = (container.get("securityContext") or {}).get("capabilities")
        c_add = set((caps or {}).get("add") or ())
        c_drop = set((caps or {}).get("drop") or ())
        add = (set(self.default_add) - c_drop) | c_add
        drop = set(self.required_drop) | c_drop
        if len(add) == len(c_add) and len(drop) == len(c_drop):
            return caps
        out = {}
        if add:
            out["add"] = sorted(add)
        if drop:
            out["drop"] = sorted(drop)
        return out

    def validate(self, path, caps):
        if caps is None:
            if not self.default_add and not self.required_drop:
                return []
            return [invalid(f"{path}.capabilities", None, "required capabilities are not set on the securityContext")]
        if "*" in self.allowed:
            return []
        errs = []
        for cap in caps.get("add") or ():
            if cap not in self.default_add and cap not in self.allowed:
                errs.append(invalid(f"{path}.capabilities.add", cap, "capability may not be added"))
        drops = set(caps.get("drop") or ())
        for d in self.required_drop:
            if d not in drops:
                errs.append(invalid(f"{path}.capabilities.drop", list(caps.get("drop") or []),
                                    f"{d} is required to be dropped but was not found"))
        return errs


class _Profiles:
    """apparmor / seccomp: a default profile and an allow-list, both from policy annotations."""

    def __init__(self, anns, default_key, allowed_key, any_token=None):
        self.default = anns.get(default_key, "")
        self.allowed_string = anns.get(allowed_key, "")
        self.allowed = None
        self.allow_any = False
        if allowed_key in anns:
            self.allowed = set()
            for p in anns[allowed_key].split(","):
                if any_token is not None and p == any_token:
                    self.allow_any = True
                else:
                    self.allowed.add(p)


class Provider:
    """One PodSecurityPolicy's strategies (`provider.go` simpleProvider)."""

    def __init__(self, psp):
        self.psp = psp
        self.name = psp["metadata"]["name"]
        sp = self.sp = psp.get("spec") or {}
        anns = (psp.get("metadata") or {}).get("annotations") or {}
        errs = []
        for attr, build in (("user", lambda: _User(sp.get("runAsUser"))),
                            ("selinux", lambda: _SELinux(sp.get("seLinux"))),
                            ("fs_group", lambda: _Group(sp.get("fsGroup"), "fsGroup")),
                            ("sup_groups", lambda: _Group(sp.get("supplementalGroups"), "supplementalGroups"))):
            try:
                setattr(self, attr, build())
            except ProviderError as e:
                errs.append(str(e))
        if errs:
            raise ProviderError(f"error creating provider for PSP {self.name}: " + "; ".join(errs))
        self.caps = _Capabilities(sp.get("defaultAddCapabilities"), sp.get("requiredDropCapabilities"),
                                  sp.get("allowedCapabilities"))
        self.apparmor = _Profiles(anns, APPARMOR_DEFAULT, APPARMOR_ALLOWED)
        self.seccomp = _Profiles(anns, SECCOMP_DEFAULT, SECCOMP_ALLOWED, any_token="*")
        self.sysctl_patterns = None if PSP_SYSCTLS not in anns else \
            ([] if not anns[PSP_SYSCTLS] else anns[PSP_SYSCTLS].split(","))
        # extensions/v1beta1 defaulting: allowPrivilegeEscalation defaults to true
        self.allow_escalation = sp.get("allowPrivilegeEscalation", True) is not False
        self.default_allow_escalation = sp.get("defaultAllowPrivilegeEscalation")

    # -- defaulting ------------------------------------------------------------------------------

    def create_pod_security_context(self, pod):
        spec = pod["spec"]
        sc = dict(spec.get("securityContext") or {})
        anns = dict((pod.get("metadata") or {}).get("annotations") or {})
        if sc.get("supplementalGroups") is None:
            g = self.sup_groups.generate()
            if g is not None:
                sc["supplementalGroups"] = g
        if sc.get("fsGroup") is None:
            g = self.fs_group.generate_single()
            if g is not None:
                sc["fsGroup"] = g
        if sc.get("seLinuxOptions") is None:
            se = self.selinux.generate()
            if se is not None:
                sc["seLinuxOptions"] = se
        profile = anns.get(SECCOMP_POD) or self.seccomp.default
        if profile:
            anns[SECCOMP_POD] = profile
        return sc, anns

    def create_container_security_context(self, pod, container):
        psc = pod["spec"].get("securityContext") or {}
        sc = dict(container.get("securityContext") or {})
        anns = dict((pod.get("metadata") or {}).get("annotations") or {})
        eff_uid = sc.get("runAsUser", psc.get("runAsUser"))
        if eff_uid is None:
            uid = self.user.generate()
            if uid is not None:
                sc["runAsUser"] = eff_uid = uid
        if sc.get("seLinuxOptions", psc.get("seLinuxOptions")) is None:
            se = self.selinux.generate()
            if se is not None:
                sc["seLinuxOptions"] = se
        key = APPARMOR_CONTAINER_PREFIX + container.get("name", "")
        if not anns.get(key) and self.apparmor.default:
            anns[key] = self.apparmor.default
        if sc.get("runAsNonRoot", psc.get("runAsNonRoot")) is None and eff_uid is None and \
                self.user.rule == "MustRunAsNonRoot":
            sc["runAsNonRoot"] = True
        caps = self.caps.generate({"securityContext": sc})
        if caps is not None:
            sc["capabilities"] = caps
        elif "capabilities" in sc:
            sc.pop("capabilities")
        if self.sp.get("readOnlyRootFilesystem") and sc.get("readOnlyRootFilesystem") is None:
            sc["readOnlyRootFilesystem"] = True
        if self.default_allow_escalation is not None and sc.get("allowPrivilegeEscalation") is None:
            sc["allowPrivilegeEscalation"] = bool(self.default_allow_escalation)
        if not self.allow_escalation and sc.get("allowPrivilegeEscalation") is None:
            sc["allowPrivilegeEscalation"] = False
        return sc, anns

    # -- validation ------------------------------------------------------------------------------

    def validate_pod_security_context(self, pod, path="spec.securityContext"):
        spec = pod["spec"]
        sc = spec.get("securityContext") or {}
        anns = (pod.get("metadata") or {}).get("annotations") or {}
        errs = []
        errs += self.fs_group.validate([sc["fsGroup"]] if sc.get("fsGroup") is not None else [])
        errs += self.sup_groups.validate(sc.get("supplementalGroups") or [])
        errs += self._validate_seccomp(anns.get(SECCOMP_POD, ""), f"pod.metadata.annotations[{SECCOMP_POD}]")
        errs += self.selinux.validate(f"{path}.seLinuxOptions", sc.get("seLinuxOptions"))
        for f, what in (("hostNetwork", "Host network"), ("hostPID", "Host PID"), ("hostIPC", "Host IPC")):
            if spec.get(f) and not self.sp.get(f):
                errs.append(invalid(f"{path}.{f}", True, f"{what} is not allowed to be used"))
        errs += self._validate_sysctls(anns)
        vols = self.sp.get("volumes") or []
        for i, v in enumerate(spec.get("volumes") or ()):
            fs = volume_type(v)
            vpath = f"spec.volumes[{i}]"
            if fs is None:
                errs.append(invalid(vpath, "", f"unknown volume type for volume: {v.get('name', '')}"))
                continue
            if "*" not in vols and fs not in vols:
                errs.append(invalid(vpath, fs, f"{fs} volumes are not allowed to be used"))
                continue
            if fs == "hostPath":
                allowed = self.sp.get("allowedHostPaths") or []
                hp = (v.get("hostPath") or {}).get("path", "")
                if allowed and not any(has_path_prefix(hp, a.get("pathPrefix", "")) for a in allowed):
                    errs.append(invalid(f"{vpath}.hostPath.pathPrefix", hp, "is not allowed to be used"))
            if fs == "flexVolume" and self.sp.get("allowedFlexVolumes"):
                drv = (v.get("flexVolume") or {}).get("driver", "")
                if drv not in {f.get("driver") for f in self.sp["allowedFlexVolumes"]}:
                    errs.append(invalid(f"{path}.volumes[{i}].driver", drv, "Flexvolume driver is not allowed to be used"))
        return errs

    def validate_container_security_context(self, pod, container, path):
        spec = pod["spec"]
        psc = spec.get("securityContext") or {}
        sc = container.get("securityContext") or {}
        anns = (pod.get("metadata") or {}).get("annotations") or {}
        name = container.get("name", "")
        errs = []
        errs += self.user.validate(path, sc.get("runAsNonRoot", psc.get("runAsNonRoot")),
                                   sc.get("runAsUser", psc.get("runAsUser")))
        errs += self.selinux.validate(f"{path}.seLinuxOptions", sc.get("seLinuxOptions", psc.get("seLinuxOptions")))
        errs += self._validate_apparmor(anns, name)
        cprofile = anns.get(SECCOMP_CONTAINER_PREFIX + name, anns.get(SECCOMP_POD, ""))
        errs += self._validate_seccomp(cprofile, f"pod.metadata.annotations[{SECCOMP_CONTAINER_PREFIX + name}]")
        if sc.get("privileged") and not self.sp.get("privileged"):
            errs.append(invalid(f"{path}.privileged", True, "Privileged containers are not allowed"))
        errs += self.caps.validate(path, sc.get("capabilities"))
        if spec.get("hostNetwork") and not self.sp.get("hostNetwork"):
            errs.append(invalid(f"{path}.hostNetwork", True, "Host network is not allowed to be used"))
        for kind in ("containers", "initContainers"):
            for idx, c in enumerate(spec.get(kind) or ()):
                for port in c.get("ports") or ():
                    hp = int(port.get("hostPort") or 0)
                    if hp > 0 and not _in_ranges(hp, self.sp.get("hostPorts")):
                        errs.append(invalid(f"{path}.{kind}[{idx}].hostPort", hp,
                                            f"Host port {hp} is not allowed to be used. Allowed ports: "
                                            f"[{self._host_port_ranges()}]"))
        if spec.get("hostPID") and not self.sp.get("hostPID"):
            errs.append(invalid(f"{path}.hostPID", True, "Host PID is not allowed to be used"))
        if spec.get("hostIPC") and not self.sp.get("hostIPC"):
            errs.append(invalid(f"{path}.hostIPC", True, "Host IPC is not allowed to be used"))
        if self.sp.get("readOnlyRootFilesystem"):
            ro = sc.get("readOnlyRootFilesystem")
            if ro is None:
                errs.append(invalid(f"{path}.readOnlyRootFilesystem", None,
                                    "ReadOnlyRootFilesystem may not be nil and must be set to true"))
            elif not ro:
                errs.append(invalid(f"{path}.readOnlyRootFilesystem", False, "ReadOnlyRootFilesystem must be set to true"))
        esc = sc.get("allowPrivilegeEscalation")
        if not self.allow_escalation and (esc is None or esc):
            errs.append(invalid(f"{path}.allowPrivilegeEscalation", esc,
                                "Allowing privilege escalation for containers is not allowed"))
        return errs

    def _host_port_ranges(self):
        return ",".join(str(r.get("min")) if r.get("min") == r.get("max") else f"{r.get('min')}-{r.get('max')}"
                        for r in self.sp.get("hostPorts") or ())

    def _validate_seccomp(self, profile, path):
        s = self.seccomp
        if not s.allow_any and not s.allowed and profile:
            return [forbidden(path, "seccomp may not be set")]
        allowed = (not s.allowed and not profile) or s.allow_any or profile in (s.allowed or ())
        if not allowed:
            return [forbidden(path, f"{profile} is not an allowed seccomp profile. Valid values are {s.allowed_string}")]
        return []

    def _validate_apparmor(self, anns, name):
        a = self.apparmor
        if a.allowed is None:
            return []
        path = f"pod.metadata.annotations[{APPARMOR_CONTAINER_PREFIX + name}]"
        profile = anns.get(APPARMOR_CONTAINER_PREFIX + name, "")
        if not profile:
            return [forbidden(path, "AppArmor profile must be set")] if a.allowed else []
        if profile not in a.allowed:
            return [forbidden(path, f"{profile} is not an allowed profile. Allowed values: {json.dumps(a.allowed_string)}")]
        return []

    def _validate_sysctls(self, anns):
        patterns = ["*"] if self.sysctl_patterns is None else self.sysctl_patterns
        errs = []
        for key in (POD_SYSCTLS, POD_UNSAFE_SYSCTLS):
            raw = anns.get(key, "")
            path = f"pod.metadata.annotations[{key}]"
            names = []
            for kv in filter(None, raw.split(",")):
                if "=" not in kv:
                    errs.append(invalid(path, raw, f"sysctl {json.dumps(kv)} not of the format sysctl_name=value"))
                    continue
                names.append(kv.split("=", 1)[0])
            if names and not patterns:
                errs.append(invalid(path, raw, "sysctls are not allowed"))
                continue
            for i, n in enumerate(names):
                if not any((p.endswith("*") and n.startswith(p[:-1])) or n == p for p in patterns):
                    errs.append(forbidden(f"{path}[{i}]", f"sysctl {json.dumps(n)} is not allowed"))
        return errs

    # -- admission.go assignSecurityContext ------------------------------------------------------

    def assign(self, pod) -> list[str]:
        """Default then validate `pod` in place; the list of errors (empty = admitted)."""
        errs = []
        spec = pod.setdefault("spec", {})
        md = pod.setdefault("metadata", {})
        psc, anns = self.create_pod_security_context(pod)
        _set_or_drop(spec, "securityContext", psc)
        _set_or_drop(md, "annotations", anns)
        errs += self.validate_pod_security_context(pod)
        for kind in ("initContainers", "containers"):
            for i, c in enumerate(spec.get(kind) or ()):
                sc, anns = self.create_container_security_context(pod, c)
                _set_or_drop(c, "securityContext", sc)
                _set_or_drop(md, "annotations", anns)
                errs += self.validate_container_security_context(pod, c, f"spec.{kind}[{i}].securityContext")
        return errs


def _set_or_drop(d, key, value):
    """Never turn an absent field into an empty one (keeps unmutated pods equal); the create_*
    helpers only add to a copy of the original, so an empty value means the original was empty."""
    if value:
        d[key] = value


__all__ = ["Provider", "ProviderError", "VOLUME_TYPES", "has_path_prefix", "volume_type"]
