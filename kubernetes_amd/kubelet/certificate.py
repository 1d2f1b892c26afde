"""Kubelet TLS bootstrap and client-certificate rotation.

Parity: `pkg/kubelet/certificate/bootstrap/bootstrap.go` (`LoadClientCert`: with only a bootstrap
kubeconfig, generate a key, submit a CSR for `CN=system:node:<node>, O=system:nodes` with usages
{digital signature, key encipherment, client auth}, wait for the signed certificate, write a
kubeconfig using it) and `pkg/kubelet/certificate/kubelet.go` / `client-go/util/certificate`
(rotate when 70-90 % of the validity has elapsed).
"""
from __future__ import annotations

import asyncio
import base64
import os
import time

from ..client import clientcmd
from ..native import crypto

USAGES = ["digital signature", "key encipherment", "client auth"]


async def request_certificate(client, node_name, key_pem, timeout=300.0, name=None):
    csr_pem = crypto.make_csr(key_pem, f"system:node:{node_name}", ["system:nodes"])
    name = name or f"node-csr-{node_name}-{int(time.time() * 1000) % 10**8}"
    await client.create("certificatesigningrequests", {"metadata": {"name": name}, "spec": {
        "request": base64.b64encode(csr_pem.encode()).decode(), "usages": USAGES}})
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        c = await client.get("certificatesigningrequests", name)
        st = c.get("status") or {}
        if any(x.get("type") == "Denied" for x in st.get("conditions") or ()):
            raise PermissionError(f"certificate signing request {name} was denied")
        if st.get("certificate"):
            return base64.b64decode(st["certificate"]).decode()
        await asyncio.sleep(0.2)
    raise TimeoutError(f"timed out waiting for CSR {name} to be signed")


async def bootstrap_client_certificate(bootstrap_kubeconfig, kubeconfig, node_name, pki_dir, timeout=300.0):
    """Write `kubeconfig` with a freshly issued node client certificate."""
    cfg, path = clientcmd.load(bootstrap_kubeconfig)
    r = clientcmd.resolve(cfg, None, os.path.dirname(os.path.abspath(path)))
    client = clientcmd.client_from(bootstrap_kubeconfig)
    try:
        key = crypto.generate_key()
        cert = await request_certificate(client, node_name, key, timeout)
    finally:
        await client.close()
    os.makedirs(pki_dir, exist_ok=True)
    for fn, data in (("kubelet-client.crt", cert), ("kubelet-client.key", key)):
        p = os.path.join(pki_dir, fn)
        with open(os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600), "w") as f:
            f.write(data)
    out = clientcmd.build("default-cluster", r.server, f"system:node:{node_name}", ca_pem=r.ca_pem,
                          client_cert_pem=cert, client_key_pem=key)
    clientcmd.save(out, kubeconfig)
    return cert


def needs_rotation(cert_pem, now=None, fraction=0.7):
    now = now or time.time()
    not_after = crypto.cert_not_after(cert_pem)
    # validity start is not exposed; issued certificates are one year unless the signer says otherwise
    lifetime = 365 * 86400
    return now >= not_after - lifetime * (1 - fraction)
