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


def rotation_deadline(cert_pem, jitter=None):
    """`certificate_manager.go nextRotationDeadline`: a uniformly random point between 70 % and
    90 % of the certificate's validity."""
    import random
    nb, na = crypto.cert_not_before(cert_pem), crypto.cert_not_after(cert_pem)
    j = random.uniform(0.7, 0.9) if jitter is None else jitter
    return nb + (na - nb) * j


def needs_rotation(cert_pem, now=None, fraction=0.7):
    now = time.time() if now is None else now
    return now >= rotation_deadline(cert_pem, fraction)


class CertificateRotator:
    """Client-certificate rotation for the kubelet (`--rotate-certificates`): when the deadline
    passes, request a new certificate over the CURRENT credential (the CSR is then a
    `selfnodeclient` request the approver accepts), rewrite the kubeconfig atomically and swap
    the live client's TLS context so new connections present the new certificate."""

    def __init__(self, kubeconfig, node_name, pki_dir, client=None, check_interval=60.0):
        self.kubeconfig, self.node, self.pki = kubeconfig, node_name, pki_dir
        self.client = client
        self.interval = check_interval
        self.deadline = None
        self.rotations = 0

    def _current(self):
        cfg, p = clientcmd.load(self.kubeconfig)
        users = cfg.get("users") or [{}]
        data = (users[0].get("user") or {}).get("client-certificate-data")
        return base64.b64decode(data).decode() if data else None

    async def maybe_rotate(self, now=None):
        cert = self._current()
        if cert is None:
            return False
        if self.deadline is None:
            self.deadline = rotation_deadline(cert)
        now = time.time() if now is None else now
        if now < self.deadline:
            return False
        cfg, p = clientcmd.load(self.kubeconfig)
        r = clientcmd.resolve(cfg, None, os.path.dirname(os.path.abspath(p)))
        client = clientcmd.client_from(self.kubeconfig)
        try:
            key = crypto.generate_key()
            new = await request_certificate(client, self.node, key, name=f"node-csr-{self.node}-rot{int(now) % 10**8}")
        finally:
            await client.close()
        for fn, data in (("kubelet-client.crt", new), ("kubelet-client.key", key)):
            fp = os.path.join(self.pki, fn)
            os.makedirs(self.pki, exist_ok=True)
            with open(os.open(fp + ".tmp", os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600), "w") as f:
                f.write(data)
            os.replace(fp + ".tmp", fp)
        clientcmd.save(clientcmd.build("default-cluster", r.server, f"system:node:{self.node}", ca_pem=r.ca_pem,
                                       client_cert_pem=new, client_key_pem=key), self.kubeconfig)
        if self.client is not None:
            fresh = clientcmd.resolve(clientcmd.load(self.kubeconfig)[0], None, os.path.dirname(os.path.abspath(p)))
            self.client.http.set_ssl_context(fresh.ssl_context)
        self.deadline = rotation_deadline(new)
        self.rotations += 1
        return True

    async def run(self):
        while True:
            try:
                await self.maybe_rotate()
            except Exception as e:  # noqa: BLE001 - retried on the next tick, like the reference's backoff
                import logging
                logging.getLogger("kubelet.certificate").warning("certificate rotation failed: %s", e)
            await asyncio.sleep(self.interval)
