"""Request authenticators beyond the token file.

Parity (`staging/src/k8s.io/apiserver/pkg/authentication`, `pkg/kubeapiserver/authenticator/config.go`):
  * x509 client certificates — `request/x509/x509.go`: CommonName = user, Organization = groups,
    chain verified against `--client-ca-file` (the TLS layer does the verification);
  * bootstrap tokens — `plugin/pkg/auth/authenticator/token/bootstrap/bootstrap.go`: `<id>.<secret>`
    looked up in `kube-system/bootstrap-token-<id>` (type `bootstrap.kubernetes.io/token`,
    `usage-bootstrap-authentication: "true"`, not expired), user `system:bootstrap:<id>`, groups
    `system:bootstrappers` + `auth-extra-groups`;
  * service-account JWTs — `pkg/serviceaccount/jwt.go`: RS256 / ES256 signed with
    `--service-account-key-file`, issuer `kubernetes/serviceaccount`, the referenced secret and
    service account must still exist (`--service-account-lookup`), user
    `system:serviceaccount:<ns>:<name>`, groups `system:serviceaccounts[:<ns>]`;
  * webhook token review — `plugin/pkg/authenticator/token/webhook`: POST a TokenReview to a
    remote service, results cached for `--authentication-token-webhook-cache-ttl` (2 min);
  * union with anonymous fallback — `request/union`, `--anonymous-auth`.
JWT signatures are computed by the native crypto library (OpenSSL EVP).
"""
from __future__ import annotations

import base64
import hmac
import json
import re
import time

from ..api.meta import parse_rfc3339
from ..native import crypto
from .auth import ANONYMOUS, User

SA_ISSUER = "kubernetes/serviceaccount"
BOOTSTRAP_RE = re.compile(r"^([a-z0-9]{6})\.([a-z0-9]{16})$")


def b64url(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def b64url_decode(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def _der_to_raw(sig: bytes, n=32) -> bytes:
    """DER ECDSA signature -> JOSE r||s."""
    i = 2 if sig[1] < 0x80 else 2 + (sig[1] & 0x7F)
    rl = sig[i + 1]
    r = int.from_bytes(sig[i + 2:i + 2 + rl], "big")
    j = i + 2 + rl
    sl = sig[j + 1]
    s = int.from_bytes(sig[j + 2:j + 2 + sl], "big")
    return r.to_bytes(n, "big") + s.to_bytes(n, "big")


def _raw_to_der(raw: bytes) -> bytes:
    def integer(v):
        b = v.to_bytes((v.bit_length() + 8) // 8 or 1, "big")
        return b"\x02" + bytes([len(b)]) + b
    h = len(raw) // 2
    body = integer(int.from_bytes(raw[:h], "big")) + integer(int.from_bytes(raw[h:], "big"))
    return b"\x30" + bytes([len(body)]) + body


def jwt_sign(key_pem: str, claims: dict) -> str:
    alg = "ES256" if "EC PRIVATE" in key_pem or _is_ec(key_pem) else "RS256"
    head = b64url(json.dumps({"alg": alg, "typ": "JWT"}, separators=(",", ":")).encode())
    body = b64url(json.dumps(claims, separators=(",", ":")).encode())
    sig = crypto.sign(key_pem, f"{head}.{body}".encode())
    if alg == "ES256":
        sig = _der_to_raw(sig)
    return f"{head}.{body}.{b64url(sig)}"


def _is_ec(key_pem):
    try:
        return "BEGIN PUBLIC KEY" in crypto.public_key(key_pem) and len(crypto.public_key(key_pem)) < 300
    except crypto.CryptoError:
        return False


def jwt_verify(pub_pems, token: str):
    """Returns the claims if the signature verifies against one of the keys, else None."""
    try:
        h, b, s = token.split(".")
        head = json.loads(b64url_decode(h))
        claims = json.loads(b64url_decode(b))
        sig = b64url_decode(s)
    except (ValueError, json.JSONDecodeError):
        return None
    if head.get("alg") not in ("RS256", "ES256"):
        return None
    if head["alg"] == "ES256":
        sig = _raw_to_der(sig)
    data = f"{h}.{b}".encode()
    for k in pub_pems:
        if crypto.verify(k, data, sig):
            return claims
    return None


def _peer_pem(req):
    t = getattr(req, "transport", None)
    so = t.get_extra_info("ssl_object") if t is not None else None
    der = so.getpeercert(binary_form=True) if so is not None else None
    if not der:
        return None
    import ssl as _ssl
    return _ssl.DER_cert_to_PEM_cert(der)


def _cn(cert):
    for rdn in cert.get("subject") or ():
        for k, v in rdn:
            if k == "commonName":
                return v
    return ""


class X509Authenticator:
    """`--client-ca-file`. With `ca_pem` the peer certificate must chain to that CA (the TLS
    listener also trusts the front-proxy CA, whose certificates are not user credentials)."""

    def __init__(self, ca_pem=None):
        self.ca_pem = ca_pem

    def authenticate_request(self, req):
        t = getattr(req, "transport", None)
        cert = t.get_extra_info("peercert") if t is not None else None
        if not cert:
            return None
        if self.ca_pem:
            pem = _peer_pem(req)
            if pem is None or not crypto.verify_cert(pem, self.ca_pem)[0]:
                return None
        cn, orgs = "", []
        for rdn in cert.get("subject") or ():
            for k, v in rdn:
                if k == "commonName":
                    cn = v
                elif k == "organizationName":
                    orgs.append(v)
        if not cn:
            return None
        return User(cn, "", orgs + ["system:authenticated"])


class RequestHeaderAuthenticator:
    """Front-proxy authentication (`--requestheader-*`, `authenticatorfactory/requestheader.go`):
    a client certificate signed by `--requestheader-client-ca-file` (with a CN in
    `--requestheader-allowed-names`, when given) vouches for the user named in the first
    non-empty `--requestheader-username-headers` header (X-Remote-User), its groups
    (X-Remote-Group, repeatable) and extras (X-Remote-Extra-<key>)."""

    def __init__(self, ca_pem, allowed_names=(), username_headers=("X-Remote-User",),
                 group_headers=("X-Remote-Group",), extra_prefixes=("X-Remote-Extra-",)):
        self.ca_pem = ca_pem
        self.allowed = set(allowed_names or ())
        self.user_h = [h.lower() for h in username_headers]
        self.group_h = [h.lower() for h in group_headers]
        self.extra_p = [h.lower() for h in extra_prefixes]

    def authenticate_request(self, req):
        t = getattr(req, "transport", None)
        cert = t.get_extra_info("peercert") if t is not None else None
        if not cert:
            return None
        name = next((req.headers.get(h) for h in self.user_h if req.headers.get(h)), None)
        if not name:
            return None
        pem = _peer_pem(req)
        if pem is None or not crypto.verify_cert(pem, self.ca_pem)[0]:
            return None
        if self.allowed and _cn(cert) not in self.allowed:
            return None
        groups = []
        for h in self.group_h:
            v = req.headers.get(h)
            if v:
                groups += [g.strip() for g in v.split(",") if g.strip()]   # repeated headers arrive joined
        return User(name, "", groups + ["system:authenticated"])


class BasicAuthenticator:
    """`--basic-auth-file`: CSV password,user,uid[,"group1,group2"]; `Authorization: Basic`."""

    def __init__(self, path):
        import csv
        self.users = {}
        with open(path) as f:
            for row in csv.reader(f):
                if len(row) < 3 or row[0].startswith("#"):
                    continue
                groups = [g for g in (row[3].split(",") if len(row) > 3 else []) if g]
                self.users[row[1]] = (row[0], User(row[1], row[2], groups + ["system:authenticated"]))

    def authenticate_request(self, req):
        h = req.headers.get("authorization", "")
        if not h.lower().startswith("basic "):
            return None
        try:
            user, _, pw = base64.b64decode(h[6:].strip()).decode().partition(":")
        except (ValueError, UnicodeDecodeError):
            return False
        rec = self.users.get(user)
        if rec is None or not hmac.compare_digest(rec[0], pw):
            return False
        return rec[1]


def _secret_data(sec, key):
    v = (sec.get("data") or {}).get(key)
    if v is not None:
        try:
            return base64.b64decode(v).decode()
        except Exception:
            return None
    return (sec.get("stringData") or {}).get(key)


class BootstrapTokenAuthenticator:
    def __init__(self, server):
        self.server = server

    def authenticate_token(self, token):
        mt = BOOTSTRAP_RE.match(token)
        if not mt:
            return None
        tid, tsecret = mt.groups()
        sec = self.server.get_object("secrets", "kube-system", f"bootstrap-token-{tid}")
        if sec is None or sec.get("type") != "bootstrap.kubernetes.io/token":
            return False
        if _secret_data(sec, "token-id") != tid or not hmac.compare_digest(_secret_data(sec, "token-secret") or "", tsecret):
            return False
        if (_secret_data(sec, "usage-bootstrap-authentication") or "") != "true":
            return False
        exp = _secret_data(sec, "expiration")
        if exp and (parse_rfc3339(exp) or 0) < time.time():
            return False
        groups = ["system:bootstrappers"] + [g for g in (_secret_data(sec, "auth-extra-groups") or "").split(",") if g]
        return User(f"system:bootstrap:{tid}", "", groups + ["system:authenticated"])


class ServiceAccountAuthenticator:
    def __init__(self, public_keys, server=None, lookup=True):
        self.keys = list(public_keys)
        self.server = server
        self.lookup = lookup

    def authenticate_token(self, token):
        if token.count(".") != 2:
            return None
        claims = jwt_verify(self.keys, token)
        if claims is None or claims.get("iss") != SA_ISSUER:
            return None if claims is None else False
        ns = claims.get("kubernetes.io/serviceaccount/namespace")
        name = claims.get("kubernetes.io/serviceaccount/service-account.name")
        uid = claims.get("kubernetes.io/serviceaccount/service-account.uid", "")
        secret = claims.get("kubernetes.io/serviceaccount/secret.name")
        if not ns or not name:
            return False
        if self.lookup and self.server is not None:
            sa = self.server.get_object("serviceaccounts", ns, name)
            if sa is None or (uid and sa["metadata"].get("uid") != uid):
                return False
            if secret and self.server.get_object("secrets", ns, secret) is None:
                return False
        return User(f"system:serviceaccount:{ns}:{name}", uid,
                    ["system:serviceaccounts", f"system:serviceaccounts:{ns}", "system:authenticated"])


def service_account_token(key_pem, sa, secret_name):
    md = sa["metadata"]
    return jwt_sign(key_pem, {"iss": SA_ISSUER, "sub": f"system:serviceaccount:{md['namespace']}:{md['name']}",
                              "kubernetes.io/serviceaccount/namespace": md["namespace"],
                              "kubernetes.io/serviceaccount/secret.name": secret_name,
                              "kubernetes.io/serviceaccount/service-account.name": md["name"],
                              "kubernetes.io/serviceaccount/service-account.uid": md.get("uid", "")})


class WebhookTokenAuthenticator:
    def __init__(self, url, ttl=120.0, ssl_context=None):
        self.url = url
        self.ttl = ttl
        self.ssl = ssl_context
        self.cache: dict = {}

    def authenticate_token(self, token):
        hit = self.cache.get(token)
        now = time.monotonic()
        if hit is not None and now - hit[1] < self.ttl:
            return hit[0]
        import urllib.request
        body = json.dumps({"apiVersion": "authentication.k8s.io/v1", "kind": "TokenReview",
                           "spec": {"token": token}}).encode()
        req = urllib.request.Request(self.url, body, {"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=10, context=self.ssl) as r:
                st = (json.loads(r.read()).get("status") or {})
        except OSError:
            return None
        u = None
        if st.get("authenticated"):
            us = st.get("user") or {}
            u = User(us.get("username", ""), us.get("uid", ""), list(us.get("groups") or []) + ["system:authenticated"])
        self.cache[token] = (u if u else False, now)
        return u if u else False


class UnionAuthenticator:
    """Tries request authenticators (x509), then bearer-token authenticators in order.
    A token rejected by every authenticator -> 401; no credentials -> anonymous (if allowed)."""

    def __init__(self, request_authenticators=(), token_authenticators=(), anonymous=True):
        self.req_auth = list(request_authenticators)
        self.tok_auth = list(token_authenticators)
        self.anonymous = anonymous

    def authenticate_request(self, req):
        for a in self.req_auth:
            u = a.authenticate_request(req)
            if u is False:
                return None          # credentials presented and rejected (basic auth): 401
            if u is not None:
                return u
        return self.authenticate(req.headers)

    def authenticate(self, headers):
        h = headers.get("authorization", "")
        if h.lower().startswith("bearer "):
            tok = h[7:].strip()
            for a in self.tok_auth:
                u = a.authenticate_token(tok) if hasattr(a, "authenticate_token") else a.tokens.get(tok)
                if u:
                    return u
            return None
        return ANONYMOUS if self.anonymous else None


# ------------------------------------------------------------------------------------ JWK <-> PEM
def _der_len(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def _tlv(tag, body):
    return bytes([tag]) + _der_len(len(body)) + body


def _der_int(v):
    b = v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big")
    if b[0] & 0x80:
        b = b"\x00" + b
    return _tlv(0x02, b)


_RSA_ALG = _tlv(0x30, bytes.fromhex("06092a864886f70d010101") + b"\x05\x00")
_EC_ALG = _tlv(0x30, bytes.fromhex("06072a8648ce3d0201") + bytes.fromhex("06082a8648ce3d030107"))


def _pem(der):
    b = base64.b64encode(der).decode()
    return "-----BEGIN PUBLIC KEY-----\n" + "\n".join(b[i:i + 64] for i in range(0, len(b), 64)) + "\n-----END PUBLIC KEY-----\n"


def jwk_to_pem(jwk: dict) -> str:
    """RSA (`n`, `e`) or P-256 EC (`x`, `y`) JWK → SubjectPublicKeyInfo PEM."""
    if jwk.get("kty") == "RSA":
        n = int.from_bytes(b64url_decode(jwk["n"]), "big")
        e = int.from_bytes(b64url_decode(jwk["e"]), "big")
        key = _tlv(0x30, _der_int(n) + _der_int(e))
        return _pem(_tlv(0x30, _RSA_ALG + _tlv(0x03, b"\x00" + key)))
    if jwk.get("kty") == "EC" and jwk.get("crv", "P-256") == "P-256":
        pt = b"\x04" + b64url_decode(jwk["x"]).rjust(32, b"\x00") + b64url_decode(jwk["y"]).rjust(32, b"\x00")
        return _pem(_tlv(0x30, _EC_ALG + _tlv(0x03, b"\x00" + pt)))
    raise ValueError(f"unsupported JWK kty={jwk.get('kty')} crv={jwk.get('crv')}")


def _read_tlv(b, i):
    tag = b[i]
    ln = b[i + 1]
    i += 2
    if ln & 0x80:
        k = ln & 0x7F
        ln = int.from_bytes(b[i:i + k], "big")
        i += k
    return tag, b[i:i + ln], i + ln


def pem_to_jwk(pem: str, kid: str = "") -> dict:
    """Inverse of `jwk_to_pem` (used to publish keys in a JWKS document)."""
    pub = crypto.public_key(pem)
    der = base64.b64decode("".join(l for l in pub.splitlines() if not l.startswith("-----")))
    _, spki, _ = _read_tlv(der, 0)
    _, alg, j = _read_tlv(spki, 0)
    _, bits, _ = _read_tlv(spki, j)
    key = bits[1:]
    out = {"kid": kid, "use": "sig"}
    if alg.startswith(bytes.fromhex("06092a864886f70d010101")):
        _, seq, _ = _read_tlv(key, 0)
        _, n, k = _read_tlv(seq, 0)
        _, e, _ = _read_tlv(seq, k)
        out.update(kty="RSA", alg="RS256", n=b64url(n.lstrip(b"\x00")), e=b64url(e))
    else:
        out.update(kty="EC", alg="ES256", crv="P-256", x=b64url(key[1:33]), y=b64url(key[33:65]))
    return out


class OIDCAuthenticator:
    """OpenID Connect ID-token authenticator.

    Parity: `staging/src/k8s.io/apiserver/plugin/pkg/authenticator/token/oidc/oidc.go` (1.9):
    keys from the issuer's discovery document (`/.well-known/openid-configuration` →
    `jwks_uri`, refreshed on an unknown `kid`), `iss` must equal the issuer URL, `aud` must
    contain the client id, `exp` in the future, `email_verified` required when the username
    claim is `email`; usernames from any other claim are prefixed with `<issuer>#` unless a
    prefix is configured (`--oidc-username-prefix`, `-` disables); groups from
    `--oidc-groups-claim` (string or list) with `--oidc-groups-prefix`; `--oidc-required-claim`.
    `keys` may be given directly (air-gapped clusters without a reachable issuer).
    """

    def __init__(self, issuer_url, client_id, username_claim="sub", username_prefix=None, groups_claim=None,
                 groups_prefix="", ca_file=None, required_claims=None, keys=None, refresh_interval=10.0):
        self.issuer = issuer_url.rstrip("/")
        self.client_id = client_id
        self.username_claim = username_claim
        if username_prefix is None:
            username_prefix = "" if username_claim == "email" else self.issuer + "#"
        self.username_prefix = "" if username_prefix == "-" else username_prefix
        self.groups_claim = groups_claim
        self.groups_prefix = groups_prefix or ""
        self.ca_file = ca_file
        self.required = dict(required_claims or {})
        self.keys = dict(keys or {})       # kid -> PEM
        self.refresh_interval = refresh_interval
        self._last_fetch = 0.0
        self._fetching = None
        if not self.keys:
            self.refresh()

    def refresh(self):
        """Fetch the issuer's keys on a background thread (the request path never blocks on
        the network; tokens are rejected until keys are known, as in the reference)."""
        import threading
        if self._fetching is not None and self._fetching.is_alive():
            return self._fetching
        self._fetching = threading.Thread(target=self._fetch, name="oidc-keys", daemon=True)
        self._fetching.start()
        return self._fetching

    def _fetch(self):
        import ssl
        import urllib.request
        now = time.monotonic()
        if now - self._last_fetch < self.refresh_interval:
            return
        self._last_fetch = now
        ctx = ssl.create_default_context(cafile=self.ca_file) if self.issuer.startswith("https") else None
        try:
            with urllib.request.urlopen(self.issuer + "/.well-known/openid-configuration", timeout=5, context=ctx) as r:
                disc = json.loads(r.read())
            with urllib.request.urlopen(disc["jwks_uri"], timeout=5, context=ctx) as r:
                jwks = json.loads(r.read())
        except (OSError, ValueError, KeyError):
            return
        keys = {}
        for k in jwks.get("keys") or ():
            try:
                keys[k.get("kid", "")] = jwk_to_pem(k)
            except (ValueError, KeyError):
                continue
        if keys:
            self.keys = keys

    def authenticate_token(self, token):
        if token.count(".") != 2:
            return None
        try:
            head = json.loads(b64url_decode(token.split(".")[0]))
        except (ValueError, json.JSONDecodeError):
            return None
        kid = head.get("kid", "")
        if not self.keys or (kid and kid not in self.keys):
            self.refresh()
        cands = [self.keys[kid]] if kid in self.keys else list(self.keys.values())
        claims = jwt_verify(cands, token) if cands else None
        if claims is None:
            return None
        if claims.get("iss") != self.issuer:
            return None
        aud = claims.get("aud")
        if self.client_id not in (aud if isinstance(aud, list) else [aud]):
            return None
        if claims.get("exp") is None or claims["exp"] < time.time():
            return None
        for k, v in self.required.items():
            if claims.get(k) != v:
                return None
        name = claims.get(self.username_claim)
        if not isinstance(name, str) or not name:
            return None
        if self.username_claim == "email" and claims.get("email_verified") is False:
            return None
        groups = []
        if self.groups_claim:
            g = claims.get(self.groups_claim)
            groups = [g] if isinstance(g, str) else list(g or [])
        return User(self.username_prefix + name, "", [self.groups_prefix + x for x in groups] + ["system:authenticated"])
