"""Container images: references, the node-local OCI store (blobs, tags, unpacked root
filesystems), the Registry v2 pull client with pull-secret keyrings, and a small read-only
registry server (add-on / tests)."""
