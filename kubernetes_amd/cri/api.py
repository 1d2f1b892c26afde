"""CRI v1alpha1 RuntimeService / ImageService — wire-compatible message classes.

Field numbers follow `pkg/kubelet/apis/cri/v1alpha1/runtime/api.proto` exactly (enums are
carried as int32 varints, which is the same encoding on the wire), so a real CRI runtime or
`crictl` speaking v1alpha1 could talk to the server in `server.py`, and the kubelet client in
`remote.py` could talk to a real runtime. Services: `runtime.RuntimeService` (:17-87) and
`runtime.ImageService` (:90-105).
"""
from __future__ import annotations

from ..utils.protodesc import build

S, B, I32, I64, U32, U64, BY, M = "string", "bool", "int32", "int64", "uint32", "uint64", "bytes", "message"


def f(name, num, typ, label="opt", tname=None):
    return (name, num, typ, label, tname)


# enums (api.proto:136-160, 356-359, 689-694)
TCP, UDP = 0, 1
SANDBOX_READY, SANDBOX_NOTREADY = 0, 1
CONTAINER_CREATED, CONTAINER_RUNNING, CONTAINER_EXITED, CONTAINER_UNKNOWN = 0, 1, 2, 3
STATE_NAMES = {0: "CONTAINER_CREATED", 1: "CONTAINER_RUNNING", 2: "CONTAINER_EXITED", 3: "CONTAINER_UNKNOWN"}
STATE_VALUES = {v: k for k, v in STATE_NAMES.items()}

SCHEMA = {
    "VersionRequest": [f("version", 1, S)],
    "VersionResponse": [f("version", 1, S), f("runtime_name", 2, S), f("runtime_version", 3, S),
                        f("runtime_api_version", 4, S)],
    "DNSConfig": [f("servers", 1, S, "rep"), f("searches", 2, S, "rep"), f("options", 3, S, "rep")],
    "PortMapping": [f("protocol", 1, I32), f("container_port", 2, I32), f("host_port", 3, I32), f("host_ip", 4, S)],
    "Mount": [f("container_path", 1, S), f("host_path", 2, S), f("readonly", 3, B), f("selinux_relabel", 4, B),
              f("propagation", 5, I32)],
    "NamespaceOption": [f("host_network", 1, B), f("host_pid", 2, B), f("host_ipc", 3, B)],
    "Int64Value": [f("value", 1, I64)],
    "SELinuxOption": [f("user", 1, S), f("role", 2, S), f("type", 3, S), f("level", 4, S)],
    "LinuxSandboxSecurityContext": [f("namespace_options", 1, M, "opt", "NamespaceOption"),
                                    f("selinux_options", 2, M, "opt", "SELinuxOption"),
                                    f("run_as_user", 3, M, "opt", "Int64Value"), f("readonly_rootfs", 4, B),
                                    f("supplemental_groups", 5, I64, "rep"), f("privileged", 6, B),
                                    f("seccomp_profile_path", 7, S)],
    "LinuxPodSandboxConfig": [f("cgroup_parent", 1, S),
                              f("security_context", 2, M, "opt", "LinuxSandboxSecurityContext"),
                              f("sysctls", 3, S, "map")],
    "PodSandboxMetadata": [f("name", 1, S), f("uid", 2, S), f("namespace", 3, S), f("attempt", 4, U32)],
    "PodSandboxConfig": [f("metadata", 1, M, "opt", "PodSandboxMetadata"), f("hostname", 2, S),
                         f("log_directory", 3, S), f("dns_config", 4, M, "opt", "DNSConfig"),
                         f("port_mappings", 5, M, "rep", "PortMapping"), f("labels", 6, S, "map"),
                         f("annotations", 7, S, "map"), f("linux", 8, M, "opt", "LinuxPodSandboxConfig")],
    "RunPodSandboxRequest": [f("config", 1, M, "opt", "PodSandboxConfig")],
    "RunPodSandboxResponse": [f("pod_sandbox_id", 1, S)],
    "StopPodSandboxRequest": [f("pod_sandbox_id", 1, S)],
    "StopPodSandboxResponse": [],
    "RemovePodSandboxRequest": [f("pod_sandbox_id", 1, S)],
    "RemovePodSandboxResponse": [],
    "PodSandboxStatusRequest": [f("pod_sandbox_id", 1, S), f("verbose", 2, B)],
    "PodSandboxNetworkStatus": [f("ip", 1, S)],
    "Namespace": [f("options", 2, M, "opt", "NamespaceOption")],
    "LinuxPodSandboxStatus": [f("namespaces", 1, M, "opt", "Namespace")],
    "PodSandboxStatus": [f("id", 1, S), f("metadata", 2, M, "opt", "PodSandboxMetadata"), f("state", 3, I32),
                         f("created_at", 4, I64), f("network", 5, M, "opt", "PodSandboxNetworkStatus"),
                         f("linux", 6, M, "opt", "LinuxPodSandboxStatus"), f("labels", 7, S, "map"),
                         f("annotations", 8, S, "map")],
    "PodSandboxStatusResponse": [f("status", 1, M, "opt", "PodSandboxStatus"), f("info", 2, S, "map")],
    "PodSandboxStateValue": [f("state", 1, I32)],
    "PodSandboxFilter": [f("id", 1, S), f("state", 2, M, "opt", "PodSandboxStateValue"), f("label_selector", 3, S, "map")],
    "ListPodSandboxRequest": [f("filter", 1, M, "opt", "PodSandboxFilter")],
    "PodSandbox": [f("id", 1, S), f("metadata", 2, M, "opt", "PodSandboxMetadata"), f("state", 3, I32),
                   f("created_at", 4, I64), f("labels", 5, S, "map"), f("annotations", 6, S, "map")],
    "ListPodSandboxResponse": [f("items", 1, M, "rep", "PodSandbox")],
    "ImageSpec": [f("image", 1, S)],
    "KeyValue": [f("key", 1, S), f("value", 2, S)],
    "LinuxContainerResources": [f("cpu_period", 1, I64), f("cpu_quota", 2, I64), f("cpu_shares", 3, I64),
                                f("memory_limit_in_bytes", 4, I64), f("oom_score_adj", 5, I64),
                                f("cpuset_cpus", 6, S), f("cpuset_mems", 7, S)],
    "Capability": [f("add_capabilities", 1, S, "rep"), f("drop_capabilities", 2, S, "rep")],
    "LinuxContainerSecurityContext": [f("capabilities", 1, M, "opt", "Capability"), f("privileged", 2, B),
                                      f("namespace_options", 3, M, "opt", "NamespaceOption"),
                                      f("selinux_options", 4, M, "opt", "SELinuxOption"),
                                      f("run_as_user", 5, M, "opt", "Int64Value"), f("run_as_username", 6, S),
                                      f("readonly_rootfs", 7, B), f("supplemental_groups", 8, I64, "rep"),
                                      f("apparmor_profile", 9, S), f("seccomp_profile_path", 10, S),
                                      f("no_new_privs", 11, B)],
    "LinuxContainerConfig": [f("resources", 1, M, "opt", "LinuxContainerResources"),
                             f("security_context", 2, M, "opt", "LinuxContainerSecurityContext")],
    "ContainerMetadata": [f("name", 1, S), f("attempt", 2, U32)],
    "Device": [f("container_path", 1, S), f("host_path", 2, S), f("permissions", 3, S)],
    "ContainerConfig": [f("metadata", 1, M, "opt", "ContainerMetadata"), f("image", 2, M, "opt", "ImageSpec"),
                        f("command", 3, S, "rep"), f("args", 4, S, "rep"), f("working_dir", 5, S),
                        f("envs", 6, M, "rep", "KeyValue"), f("mounts", 7, M, "rep", "Mount"),
                        f("devices", 8, M, "rep", "Device"), f("labels", 9, S, "map"), f("annotations", 10, S, "map"),
                        f("log_path", 11, S), f("stdin", 12, B), f("stdin_once", 13, B), f("tty", 14, B),
                        f("linux", 15, M, "opt", "LinuxContainerConfig")],
    "CreateContainerRequest": [f("pod_sandbox_id", 1, S), f("config", 2, M, "opt", "ContainerConfig"),
                               f("sandbox_config", 3, M, "opt", "PodSandboxConfig")],
    "CreateContainerResponse": [f("container_id", 1, S)],
    "StartContainerRequest": [f("container_id", 1, S)],
    "StartContainerResponse": [],
    "StopContainerRequest": [f("container_id", 1, S), f("timeout", 2, I64)],
    "StopContainerResponse": [],
    "RemoveContainerRequest": [f("container_id", 1, S)],
    "RemoveContainerResponse": [],
    "ContainerStateValue": [f("state", 1, I32)],
    "ContainerFilter": [f("id", 1, S), f("state", 2, M, "opt", "ContainerStateValue"), f("pod_sandbox_id", 3, S),
                        f("label_selector", 4, S, "map")],
    "ListContainersRequest": [f("filter", 1, M, "opt", "ContainerFilter")],
    "Container": [f("id", 1, S), f("pod_sandbox_id", 2, S), f("metadata", 3, M, "opt", "ContainerMetadata"),
                  f("image", 4, M, "opt", "ImageSpec"), f("image_ref", 5, S), f("state", 6, I32),
                  f("created_at", 7, I64), f("labels", 8, S, "map"), f("annotations", 9, S, "map")],
    "ListContainersResponse": [f("containers", 1, M, "rep", "Container")],
    "ContainerStatusRequest": [f("container_id", 1, S), f("verbose", 2, B)],
    "ContainerStatus": [f("id", 1, S), f("metadata", 2, M, "opt", "ContainerMetadata"), f("state", 3, I32),
                        f("created_at", 4, I64), f("started_at", 5, I64), f("finished_at", 6, I64),
                        f("exit_code", 7, I32), f("image", 8, M, "opt", "ImageSpec"), f("image_ref", 9, S),
                        f("reason", 10, S), f("message", 11, S), f("labels", 12, S, "map"),
                        f("annotations", 13, S, "map"), f("mounts", 14, M, "rep", "Mount"), f("log_path", 15, S)],
    "ContainerStatusResponse": [f("status", 1, M, "opt", "ContainerStatus"), f("info", 2, S, "map")],
    "UpdateContainerResourcesRequest": [f("container_id", 1, S), f("linux", 2, M, "opt", "LinuxContainerResources")],
    "UpdateContainerResourcesResponse": [],
    "ExecSyncRequest": [f("container_id", 1, S), f("cmd", 2, S, "rep"), f("timeout", 3, I64)],
    "ExecSyncResponse": [f("stdout", 1, BY), f("stderr", 2, BY), f("exit_code", 3, I32)],
    "ExecRequest": [f("container_id", 1, S), f("cmd", 2, S, "rep"), f("tty", 3, B), f("stdin", 4, B),
                    f("stdout", 5, B), f("stderr", 6, B)],
    "ExecResponse": [f("url", 1, S)],
    "AttachRequest": [f("container_id", 1, S), f("stdin", 2, B), f("tty", 3, B), f("stdout", 4, B), f("stderr", 5, B)],
    "AttachResponse": [f("url", 1, S)],
    "PortForwardRequest": [f("pod_sandbox_id", 1, S), f("port", 2, I32, "rep")],
    "PortForwardResponse": [f("url", 1, S)],
    "ImageFilter": [f("image", 1, M, "opt", "ImageSpec")],
    "ListImagesRequest": [f("filter", 1, M, "opt", "ImageFilter")],
    "Image": [f("id", 1, S), f("repo_tags", 2, S, "rep"), f("repo_digests", 3, S, "rep"), f("size", 4, U64),
              f("uid", 5, M, "opt", "Int64Value"), f("username", 6, S)],
    "ListImagesResponse": [f("images", 1, M, "rep", "Image")],
    "ImageStatusRequest": [f("image", 1, M, "opt", "ImageSpec"), f("verbose", 2, B)],
    "ImageStatusResponse": [f("image", 1, M, "opt", "Image"), f("info", 2, S, "map")],
    "AuthConfig": [f("username", 1, S), f("password", 2, S), f("auth", 3, S), f("server_address", 4, S),
                   f("identity_token", 5, S), f("registry_token", 6, S)],
    "PullImageRequest": [f("image", 1, M, "opt", "ImageSpec"), f("auth", 2, M, "opt", "AuthConfig"),
                         f("sandbox_config", 3, M, "opt", "PodSandboxConfig")],
    "PullImageResponse": [f("image_ref", 1, S)],
    "RemoveImageRequest": [f("image", 1, M, "opt", "ImageSpec")],
    "RemoveImageResponse": [],
    "NetworkConfig": [f("pod_cidr", 1, S)],
    "RuntimeConfig": [f("network_config", 1, M, "opt", "NetworkConfig")],
    "UpdateRuntimeConfigRequest": [f("runtime_config", 1, M, "opt", "RuntimeConfig")],
    "UpdateRuntimeConfigResponse": [],
    "RuntimeCondition": [f("type", 1, S), f("status", 2, B), f("reason", 3, S), f("message", 4, S)],
    "RuntimeStatus": [f("conditions", 1, M, "rep", "RuntimeCondition")],
    "StatusRequest": [f("verbose", 1, B)],
    "StatusResponse": [f("status", 1, M, "opt", "RuntimeStatus"), f("info", 2, S, "map")],
    "ImageFsInfoRequest": [],
    "UInt64Value": [f("value", 1, U64)],
    "StorageIdentifier": [f("uuid", 1, S)],
    "FilesystemUsage": [f("timestamp", 1, I64), f("storage_id", 2, M, "opt", "StorageIdentifier"),
                        f("used_bytes", 3, M, "opt", "UInt64Value"), f("inodes_used", 4, M, "opt", "UInt64Value")],
    "ImageFsInfoResponse": [f("image_filesystems", 1, M, "rep", "FilesystemUsage")],
    "ContainerStatsRequest": [f("container_id", 1, S)],
    "ContainerAttributes": [f("id", 1, S), f("metadata", 2, M, "opt", "ContainerMetadata"), f("labels", 3, S, "map"),
                            f("annotations", 4, S, "map")],
    "CpuUsage": [f("timestamp", 1, I64), f("usage_core_nano_seconds", 2, M, "opt", "UInt64Value")],
    "MemoryUsage": [f("timestamp", 1, I64), f("working_set_bytes", 2, M, "opt", "UInt64Value")],
    "ContainerStats": [f("attributes", 1, M, "opt", "ContainerAttributes"), f("cpu", 2, M, "opt", "CpuUsage"),
                       f("memory", 3, M, "opt", "MemoryUsage"), f("writable_layer", 4, M, "opt", "FilesystemUsage")],
    "ContainerStatsResponse": [f("stats", 1, M, "opt", "ContainerStats")],
    "ContainerStatsFilter": [f("id", 1, S), f("pod_sandbox_id", 2, S), f("label_selector", 3, S, "map")],
    "ListContainerStatsRequest": [f("filter", 1, M, "opt", "ContainerStatsFilter")],
    "ListContainerStatsResponse": [f("stats", 1, M, "rep", "ContainerStats")],
}

MSG = build("runtime", "runtime/v1alpha1/api.proto", SCHEMA)

RUNTIME_SERVICE = "runtime.RuntimeService"
IMAGE_SERVICE = "runtime.ImageService"


def _m(name):
    return (MSG[name + "Request"], MSG[name + "Response"], False)


RUNTIME_METHODS = {n: _m(n) for n in (
    "Version", "RunPodSandbox", "StopPodSandbox", "RemovePodSandbox", "PodSandboxStatus", "ListPodSandbox",
    "CreateContainer", "StartContainer", "StopContainer", "RemoveContainer", "ListContainers", "ContainerStatus",
    "UpdateContainerResources", "ExecSync", "Exec", "Attach", "PortForward", "ContainerStats",
    "ListContainerStats", "UpdateRuntimeConfig", "Status")}
IMAGE_METHODS = {n: _m(n) for n in ("ListImages", "ImageStatus", "PullImage", "RemoveImage", "ImageFsInfo")}

# labels the kubelet puts on sandboxes/containers (`pkg/kubelet/kuberuntime/labels.go`)
POD_NAME = "io.kubernetes.pod.name"
POD_NAMESPACE = "io.kubernetes.pod.namespace"
POD_UID = "io.kubernetes.pod.uid"
CONTAINER_NAME = "io.kubernetes.container.name"
# the original pod / container specs ride along as annotations so a backend runtime behind the
# CRI server sees exactly what the kubelet would have passed it in-process
POD_SPEC_ANNOTATION = "kubernetes-amd.io/pod"
CONTAINER_SPEC_ANNOTATION = "kubernetes-amd.io/container"
CGROUP_PARENT_ANNOTATION = "kubernetes-amd.io/cgroup-parent"   # pod cgroup (runtime joins it)
# CRI v1alpha1 has no runAsGroup (added in later CRI versions): carried as an annotation
RUN_AS_GROUP_ANNOTATION = "kamd.io/run-as-group"
# RuntimeStatus condition: whether containers get a private /dev + device cgroup
DEVICE_ISOLATION_CONDITION = "DeviceIsolation"
