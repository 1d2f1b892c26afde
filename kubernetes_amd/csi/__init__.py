"""Container Storage Interface (CSI v0.1, alpha in the reference): wire API, a host-path
driver, the external attacher, and the kubelet / attach-detach integration."""
