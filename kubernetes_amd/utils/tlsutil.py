"""TLS contexts and the kubelet's self-signed serving certificate.

Parity:
* `k8s.io/client-go/util/cert` GenerateSelfSignedCertKey — what the kubelet serves when no
  `--tls-cert-file` is given (`cmd/kubelet/app/server.go` InitializeTLS): a one-off CA
  `<host>-ca@<unix time>` and a serving certificate `<host>@<unix time>` signed by it for the
  host name, `localhost`, `127.0.0.1` and the node's addresses, written to
  `<cert-dir>/kubelet.crt` (certificate followed by the CA) and `kubelet.key`, reused across
  restarts;
* server contexts with optional x509 client authentication (`--client-ca-file`: a client
  certificate is verified when presented, anonymous / token requests still reach the
  authenticator chain);
* client contexts: verify against a CA when one is configured; without one, the peer is not
  verified — the reference's API server talks to kubelets with InsecureSkipVerify unless
  `--kubelet-certificate-authority` is set.
"""
from __future__ import annotations

import os
import ssl
import time


def server_context(cert_file: str, key_file: str, client_ca_file: str | None = None) -> ssl.SSLContext:
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(cert_file, key_file)
    if client_ca_file:
        ctx.verify_mode = ssl.CERT_OPTIONAL
        ctx.load_verify_locations(client_ca_file)
    return ctx


def client_context(ca_file: str | None = None, cert_file: str | None = None, key_file: str | None = None) -> ssl.SSLContext:
    if ca_file:
        ctx = ssl.create_default_context(cafile=ca_file)
        # kubelets and pods are reached by IP as often as by name; the chain is still verified
        ctx.check_hostname = False
    else:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    if cert_file:
        ctx.load_cert_chain(cert_file, key_file or cert_file)
    return ctx


def unverified_client_context() -> ssl.SSLContext:
    return client_context()


def self_signed_serving_cert(cert_dir: str, host: str, addresses=(), basename="kubelet") -> tuple[str, str]:
    """-> (cert path, key path), generating them on first use (`<basename>.crt/.key`; the API
    server's `--cert-dir` pair is `apiserver.crt/.key`)."""
    from ..native import crypto
    cert_path, key_path = os.path.join(cert_dir, basename + ".crt"), os.path.join(cert_dir, basename + ".key")
    if os.path.exists(cert_path) and os.path.exists(key_path):
        return cert_path, key_path
    os.makedirs(cert_dir, exist_ok=True)
    now = int(time.time())
    ca, ca_key = crypto.self_signed_ca(f"{host}-ca@{now}")
    key = crypto.generate_key()
    sans = [f"DNS:{host}", "DNS:localhost", "IP:127.0.0.1"]
    for a in addresses:
        if a and a not in ("127.0.0.1", host):
            sans.append(f"IP:{a}" if a.replace(".", "").isdigit() or ":" in a else f"DNS:{a}")
    cert = crypto.issue_cert(key_pem=key, cn=f"{host}@{now}", ca_cert=ca, ca_key=ca_key, usage="server", sans=tuple(sans))
    fd = os.open(key_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        f.write(key)
    with open(cert_path, "w") as f:
        f.write(cert if cert.endswith("\n") else cert + "\n")
        f.write(ca)
    return cert_path, key_path
