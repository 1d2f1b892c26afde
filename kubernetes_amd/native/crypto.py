"""ctypes binding for libkamd_crypto.so (native/crypto/kamd_crypto.cc).

Symmetric primitives for encryption at rest (AES-CBC, AES-GCM, NaCl secretbox) and x509
helpers (key generation, CSR, issuing, subject parsing, chain verification) used by kubeadm's
certs phase, the CSR signing controller and the x509 client-certificate authenticator.
"""
from __future__ import annotations

import ctypes
import os

from . import LIB_DIR

_lib = None
_c = ctypes.c_char_p
_b = ctypes.c_void_p
_l = ctypes.c_long
_i = ctypes.c_int


class CryptoError(Exception):
    pass


def lib_path():
    return os.path.join(LIB_DIR, "libkamd_crypto.so")


def _L():
    global _lib
    if _lib is None:
        p = lib_path()
        if not os.path.exists(p):
            raise CryptoError(f"{p} not built: run `python -m kubernetes_amd.native.build`")
        L = ctypes.CDLL(p)
        L.kc_random.argtypes = [_b, _i]
        for f in (L.kc_aes_cbc_encrypt, L.kc_aes_cbc_decrypt):
            f.argtypes = [_c, _i, _c, _c, _l, _b]
            f.restype = _l
        for f in (L.kc_aes_gcm_seal, L.kc_aes_gcm_open):
            f.argtypes = [_c, _i, _c, _c, _l, _c, _l, _b]
            f.restype = _l
        for f in (L.kc_secretbox_seal, L.kc_secretbox_open):
            f.argtypes = [_c, _c, _c, _l, _b]
            f.restype = _l
        L.kc_genkey.argtypes = [_c, _i, _b, _l]
        L.kc_genkey.restype = _l
        L.kc_issue_cert.argtypes = [_c, _c, _c, _c, _c, _l, _c, _c, _l, _b, _l]
        L.kc_issue_cert.restype = _l
        L.kc_make_csr.argtypes = [_c, _c, _b, _l]
        L.kc_make_csr.restype = _l
        L.kc_subject.argtypes = [_c, _i, _b, _l]
        L.kc_subject.restype = _l
        L.kc_verify_cert.argtypes = [_c, _c, _b, _l]
        L.kc_verify_cert.restype = _l
        L.kc_cert_not_after.argtypes = [_c]
        L.kc_cert_not_after.restype = _l
        L.kc_cert_not_before.argtypes = [_c]
        L.kc_cert_not_before.restype = _l
        L.kc_sign.argtypes = [_c, _c, _l, _b, _l]
        L.kc_sign.restype = _l
        L.kc_public_key.argtypes = [_c, _b, _l]
        L.kc_public_key.restype = _l
        L.kc_verify.argtypes = [_c, _c, _l, _c, _l]
        L.kc_verify.restype = _l
        _lib = L
    return _lib


def random_bytes(n: int) -> bytes:
    buf = ctypes.create_string_buffer(n)
    if _L().kc_random(buf, n) != 0:
        raise CryptoError("RAND_bytes failed")
    return buf.raw


def _check_key(key, sizes=(16, 24, 32)):
    if len(key) not in sizes:
        raise CryptoError(f"invalid key size {len(key)}")


def aes_cbc_encrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    _check_key(key)
    out = ctypes.create_string_buffer(len(data) + 16)
    n = _L().kc_aes_cbc_encrypt(key, len(key), iv, data, len(data), out)
    if n < 0:
        raise CryptoError("aes-cbc encrypt failed")
    return out.raw[:n]


def aes_cbc_decrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    _check_key(key)
    if not data or len(data) % 16:
        raise CryptoError("the stored data is not a multiple of the block size")
    out = ctypes.create_string_buffer(len(data))
    n = _L().kc_aes_cbc_decrypt(key, len(key), iv, data, len(data), out)
    if n < 0:
        raise CryptoError("invalid padding on input")
    return out.raw[:n]


def aes_gcm_seal(key: bytes, nonce: bytes, data: bytes, aad: bytes = b"") -> bytes:
    _check_key(key)
    out = ctypes.create_string_buffer(len(data) + 16)
    n = _L().kc_aes_gcm_seal(key, len(key), nonce, aad, len(aad), data, len(data), out)
    if n < 0:
        raise CryptoError("aes-gcm seal failed")
    return out.raw[:n]


def aes_gcm_open(key: bytes, nonce: bytes, data: bytes, aad: bytes = b"") -> bytes:
    _check_key(key)
    out = ctypes.create_string_buffer(max(1, len(data)))
    n = _L().kc_aes_gcm_open(key, len(key), nonce, aad, len(aad), data, len(data), out)
    if n < 0:
        raise CryptoError("cipher: message authentication failed")
    return out.raw[:n]


def secretbox_seal(key: bytes, nonce: bytes, data: bytes) -> bytes:
    _check_key(key, (32,))
    if len(nonce) != 24:
        raise CryptoError("secretbox nonce must be 24 bytes")
    out = ctypes.create_string_buffer(len(data) + 16)
    n = _L().kc_secretbox_seal(key, nonce, data, len(data), out)
    if n < 0:
        raise CryptoError("secretbox seal failed")
    return out.raw[:n]


def secretbox_open(key: bytes, nonce: bytes, data: bytes) -> bytes:
    _check_key(key, (32,))
    out = ctypes.create_string_buffer(max(1, len(data)))
    n = _L().kc_secretbox_open(key, nonce, data, len(data), out)
    if n < 0:
        raise CryptoError("output array too small / decryption failed")
    return out.raw[:n]


# ---------------------------------------------------------------- x509
_CAP = 1 << 16


def _text(fn, *args) -> str:
    out = ctypes.create_string_buffer(_CAP)
    n = fn(*args, out, _CAP)
    if n < 0:
        raise CryptoError(out.value.decode(errors="replace"))
    return out.value.decode()


def _e(s):
    return s.encode() if isinstance(s, str) else (s or b"")


def subject_string(cn: str, orgs=()) -> str:
    return ";".join([f"CN={cn}"] + [f"O={o}" for o in orgs])


def parse_subject(s: str) -> tuple[str, list]:
    cn, orgs = "", []
    for part in s.split(";"):
        k, _, v = part.partition("=")
        if k == "CN":
            cn = v
        elif k == "O":
            orgs.append(v)
    return cn, orgs


def generate_key(kind: str = "ec", bits: int = 2048) -> str:
    return _text(_L().kc_genkey, _e(kind), bits)


def issue_cert(key_pem="", csr_pem="", cn="", orgs=(), ca_cert="", ca_key="", days=365, usage="both",
               sans=(), serial=0) -> str:
    subj = subject_string(cn, orgs) if cn else ""
    if not serial:
        serial = int.from_bytes(random_bytes(7), "big") | 1
    return _text(_L().kc_issue_cert, _e(key_pem), _e(csr_pem), _e(subj), _e(ca_cert), _e(ca_key), days,
                 _e(usage), _e(",".join(sans)), serial)


def self_signed_ca(cn: str, days: int = 3650, kind: str = "ec") -> tuple[str, str]:
    key = generate_key(kind)
    return issue_cert(key_pem=key, cn=cn, days=days, usage="ca"), key


def make_csr(key_pem: str, cn: str, orgs=()) -> str:
    return _text(_L().kc_make_csr, _e(key_pem), _e(subject_string(cn, orgs)))


def cert_subject(pem: str) -> tuple[str, list]:
    return parse_subject(_text(_L().kc_subject, _e(pem), 0))


def csr_subject(pem: str) -> tuple[str, list]:
    return parse_subject(_text(_L().kc_subject, _e(pem), 1))


def verify_cert(cert_pem: str, ca_pem: str) -> tuple[bool, str]:
    out = ctypes.create_string_buffer(1024)
    rc = _L().kc_verify_cert(_e(cert_pem), _e(ca_pem), out, 1024)
    return rc == 0, out.value.decode(errors="replace")


def cert_not_before(pem: str) -> int:
    return _L().kc_cert_not_before(_e(pem))


def cert_not_after(pem: str) -> int:
    return _L().kc_cert_not_after(_e(pem))


def sign(key_pem: str, data: bytes) -> bytes:
    """RS256 (RSA key) or DER ECDSA-SHA256 (EC key) signature."""
    out = ctypes.create_string_buffer(1024)
    n = _L().kc_sign(_e(key_pem), data, len(data), out, 1024)
    if n < 0:
        raise CryptoError("signing failed")
    return out.raw[:n]


def public_key(pem: str) -> str:
    return _text(_L().kc_public_key, _e(pem))


def verify(pub_pem: str, data: bytes, sig: bytes) -> bool:
    return _L().kc_verify(_e(pub_pem), data, len(data), sig, len(sig)) == 1
