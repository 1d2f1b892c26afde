"""Device plugin API v1alpha ("v1alpha2") and plugin registration API v1beta — wire-compatible
message classes and gRPC service bindings.

Parity:
  * `pkg/kubelet/apis/deviceplugin/v1alpha/api.proto:17-154` — service DevicePlugin
    {GetPluginInfo, ListAndWatch(stream), AdmitPod, InitContainer}; field numbers identical.
    `GetPluginInfoResponse.labels` (field 2) is included: it exists in the reference's
    generated `api.pb.go:81-86` but not its .proto — one canonical schema.
  * `pkg/kubelet/apis/pluginregistration/v1beta/api.proto:16-54` — service Identity
    {GetSupportedVersions, GetPluginIdentity, PluginRegistrationStatus}, served on the SAME
    unix socket as DevicePlugin (the kubelet dials the plugin).
  * constants `pkg/kubelet/apis/deviceplugin/v1alpha/constants.go:19-36`.
"""
from __future__ import annotations

import grpc

from ..utils.protodesc import build

VERSION = "v1alpha2"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"
DEVICE_MANAGER_PATH = "/var/lib/kubelet/device-plugin"
DEVICE_PLUGINS_PATH = DEVICE_MANAGER_PATH + "/plugins"

DP = build("deviceplugin", "deviceplugin/v1alpha/api.proto", {
    "GetPluginInfoRequest": [],
    "GetPluginInfoResponse": [("init_timeout", 1, "int64", "opt", None), ("labels", 2, "string", "map", None)],
    "ListAndWatchRequest": [],
    "Device": [("ID", 1, "string", "opt", None), ("health", 2, "string", "opt", None),
               ("Attributes", 3, "string", "map", None)],
    "ListAndWatchResponse": [("devices", 1, "message", "rep", "Device")],
    "Container": [("name", 1, "string", "opt", None), ("devices", 2, "string", "rep", None)],
    "AdmitPodRequest": [("pod_name", 1, "string", "opt", None),
                        ("init_containers", 2, "message", "map", "Container"),
                        ("containers", 3, "message", "map", "Container")],
    "PodSpec": [("annotations", 1, "string", "map", None)],
    "AdmitPodResponse": [("pod", 1, "message", "opt", "PodSpec")],
    "InitContainerRequest": [("container", 1, "message", "opt", "Container")],
    "Mount": [("container_path", 1, "string", "opt", None), ("host_path", 2, "string", "opt", None),
              ("read_only", 3, "bool", "opt", None)],
    "DeviceSpec": [("container_path", 1, "string", "opt", None), ("host_path", 2, "string", "opt", None),
                   ("permissions", 3, "string", "opt", None)],
    "ContainerSpec": [("envs", 1, "string", "map", None), ("mounts", 2, "message", "rep", "Mount"),
                      ("devices", 3, "message", "rep", "DeviceSpec"), ("annotations", 4, "string", "map", None)],
    "InitContainerResponse": [("spec", 1, "message", "opt", "ContainerSpec")],
})

PR = build("pluginregistration", "pluginregistration/v1beta/api.proto", {
    "Empty": [],
    "GetSupportedVersionsRequest": [],
    "GetSupportedVersionsResponse": [("supported_versions", 1, "string", "rep", None)],
    "GetPluginIdentityRequest": [("version", 1, "string", "opt", None)],
    "GetPluginIdentityResponse": [("resource_name", 1, "string", "opt", None)],
    "RegistrationStatus": [("success", 1, "bool", "opt", None), ("error", 2, "string", "opt", None)],
})

DP_SERVICE = "deviceplugin.DevicePlugin"
ID_SERVICE = "pluginregistration.Identity"

# method -> (request class, response class, streaming response?)
DP_METHODS = {
    "GetPluginInfo": (DP["GetPluginInfoRequest"], DP["GetPluginInfoResponse"], False),
    "ListAndWatch": (DP["ListAndWatchRequest"], DP["ListAndWatchResponse"], True),
    "AdmitPod": (DP["AdmitPodRequest"], DP["AdmitPodResponse"], False),
    "InitContainer": (DP["InitContainerRequest"], DP["InitContainerResponse"], False),
}
ID_METHODS = {
    "GetSupportedVersions": (PR["GetSupportedVersionsRequest"], PR["GetSupportedVersionsResponse"], False),
    "GetPluginIdentity": (PR["GetPluginIdentityRequest"], PR["GetPluginIdentityResponse"], False),
    "PluginRegistrationStatus": (PR["RegistrationStatus"], PR["Empty"], False),
}


def generic_handler(service: str, methods: dict, impl) -> grpc.GenericRpcHandler:
    """Bind `impl.<Method>(request, context)` coroutines as a grpc.aio service."""
    handlers = {}
    for name, (req, resp, stream) in methods.items():
        fn = getattr(impl, name)
        if stream:
            handlers[name] = grpc.unary_stream_rpc_method_handler(
                fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
        else:
            handlers[name] = grpc.unary_unary_rpc_method_handler(
                fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
    return grpc.method_handlers_generic_handler(service, handlers)


class _Stub:
    def __init__(self, channel, service, methods):
        for name, (req, resp, stream) in methods.items():
            path = f"/{service}/{name}"
            if stream:
                m = channel.unary_stream(path, request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
            else:
                m = channel.unary_unary(path, request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
            setattr(self, name, m)


def device_plugin_stub(channel):
    return _Stub(channel, DP_SERVICE, DP_METHODS)


def identity_stub(channel):
    return _Stub(channel, ID_SERVICE, ID_METHODS)
