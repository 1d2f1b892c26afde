// kamd_crypto — native crypto for the control plane (C ABI, loaded with ctypes).
//
// Replaces the Go crypto the reference links in:
//   * storage value transformers (encryption at rest):
//       aescbc    staging/src/k8s.io/apiserver/pkg/storage/value/encrypt/aes/aes.go:93-150
//                 (16-byte random IV || AES-CBC(PKCS#7))
//       aesgcm    .../encrypt/aes/aes.go:51-83 (12-byte nonce || AES-GCM seal, AAD = etcd key)
//       secretbox .../encrypt/secretbox/secretbox.go:36-68 (24-byte nonce || NaCl secretbox =
//                 XSalsa20 + Poly1305, tag first)
//   * x509 for kubeadm's certs phase, the CSR signing controller and client-cert authn
//     (cmd/kubeadm/app/phases/certs, pkg/controller/certificates/signer).
// AES and Poly1305 come from OpenSSL's EVP layer (AES-NI); XSalsa20 is implemented here
// because OpenSSL has no Salsa20.
#include <openssl/evp.h>
#include <openssl/rand.h>
#include <openssl/pem.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>
#include <openssl/ec.h>
#include <openssl/err.h>
#include <openssl/core_names.h>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

extern "C" {

int kc_random(uint8_t* out, int n) { return RAND_bytes(out, n) == 1 ? 0 : -1; }

static const EVP_CIPHER* cbc_for(int keylen) {
  switch (keylen) {
    case 16: return EVP_aes_128_cbc();
    case 24: return EVP_aes_192_cbc();
    case 32: return EVP_aes_256_cbc();
  }
  return nullptr;
}
static const EVP_CIPHER* gcm_for(int keylen) {
  switch (keylen) {
    case 16: return EVP_aes_128_gcm();
    case 24: return EVP_aes_192_gcm();
    case 32: return EVP_aes_256_gcm();
  }
  return nullptr;
}

// out must hold n + 16 bytes. Returns ciphertext length (PKCS#7 padded) or -1.
long kc_aes_cbc_encrypt(const uint8_t* key, int keylen, const uint8_t* iv, const uint8_t* in, long n, uint8_t* out) {
  const EVP_CIPHER* c = cbc_for(keylen);
  if (!c) return -1;
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  int l1 = 0, l2 = 0;
  long r = -1;
  if (EVP_EncryptInit_ex(ctx, c, nullptr, key, iv) == 1 &&
      EVP_EncryptUpdate(ctx, out, &l1, in, (int)n) == 1 && EVP_EncryptFinal_ex(ctx, out + l1, &l2) == 1)
    r = l1 + l2;
  EVP_CIPHER_CTX_free(ctx);
  return r;
}

// Returns plaintext length, -1 on bad key / block size, -2 on bad padding.
long kc_aes_cbc_decrypt(const uint8_t* key, int keylen, const uint8_t* iv, const uint8_t* in, long n, uint8_t* out) {
  const EVP_CIPHER* c = cbc_for(keylen);
  if (!c || n <= 0 || n % 16) return -1;
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  int l1 = 0, l2 = 0;
  long r = -2;
  if (EVP_DecryptInit_ex(ctx, c, nullptr, key, iv) == 1 && EVP_DecryptUpdate(ctx, out, &l1, in, (int)n) == 1 &&
      EVP_DecryptFinal_ex(ctx, out + l1, &l2) == 1)
    r = l1 + l2;
  EVP_CIPHER_CTX_free(ctx);
  return r;
}

// out must hold n + 16 (ciphertext || tag, as Go's cipher.AEAD.Seal). Returns n + 16 or -1.
long kc_aes_gcm_seal(const uint8_t* key, int keylen, const uint8_t* nonce, const uint8_t* aad, long aadlen,
                     const uint8_t* in, long n, uint8_t* out) {
  const EVP_CIPHER* c = gcm_for(keylen);
  if (!c) return -1;
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  int l = 0, lf = 0;
  long r = -1;
  if (EVP_EncryptInit_ex(ctx, c, nullptr, nullptr, nullptr) == 1 &&
      EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) == 1 &&
      EVP_EncryptInit_ex(ctx, nullptr, nullptr, key, nonce) == 1 &&
      (aadlen == 0 || EVP_EncryptUpdate(ctx, nullptr, &l, aad, (int)aadlen) == 1) &&
      EVP_EncryptUpdate(ctx, out, &l, in, (int)n) == 1 && EVP_EncryptFinal_ex(ctx, out + l, &lf) == 1 &&
      EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_GET_TAG, 16, out + n) == 1)
    r = n + 16;
  EVP_CIPHER_CTX_free(ctx);
  return r;
}

// in = ciphertext || tag (n bytes). Returns n - 16, or -1 (bad key) / -2 (authentication failed).
long kc_aes_gcm_open(const uint8_t* key, int keylen, const uint8_t* nonce, const uint8_t* aad, long aadlen,
                     const uint8_t* in, long n, uint8_t* out) {
  const EVP_CIPHER* c = gcm_for(keylen);
  if (!c || n < 16) return -1;
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  int l = 0, lf = 0;
  long r = -2;
  long m = n - 16;
  if (EVP_DecryptInit_ex(ctx, c, nullptr, nullptr, nullptr) == 1 &&
      EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, 12, nullptr) == 1 &&
      EVP_DecryptInit_ex(ctx, nullptr, nullptr, key, nonce) == 1 &&
      (aadlen == 0 || EVP_DecryptUpdate(ctx, nullptr, &l, aad, (int)aadlen) == 1) &&
      EVP_DecryptUpdate(ctx, out, &l, in, (int)m) == 1 &&
      EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_TAG, 16, (void*)(in + m)) == 1 &&
      EVP_DecryptFinal_ex(ctx, out + l, &lf) == 1)
    r = m;
  EVP_CIPHER_CTX_free(ctx);
  return r;
}

// ---------------------------------------------------------------- XSalsa20 + Poly1305 (NaCl secretbox)
static inline uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
static inline uint32_t ld32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
static inline void st32(uint8_t* p, uint32_t v) { p[0] = v; p[1] = v >> 8; p[2] = v >> 16; p[3] = v >> 24; }
static const uint8_t SIGMA[16] = {'e', 'x', 'p', 'a', 'n', 'd', ' ', '3', '2', '-', 'b', 'y', 't', 'e', ' ', 'k'};

// 20-round Salsa20 core over state x (in place), returning the un-added words in y.
static void salsa_rounds(uint32_t* x) {
  for (int i = 0; i < 20; i += 2) {
    x[4] ^= rotl(x[0] + x[12], 7);  x[8] ^= rotl(x[4] + x[0], 9);
    x[12] ^= rotl(x[8] + x[4], 13); x[0] ^= rotl(x[12] + x[8], 18);
    x[9] ^= rotl(x[5] + x[1], 7);   x[13] ^= rotl(x[9] + x[5], 9);
    x[1] ^= rotl(x[13] + x[9], 13); x[5] ^= rotl(x[1] + x[13], 18);
    x[14] ^= rotl(x[10] + x[6], 7); x[2] ^= rotl(x[14] + x[10], 9);
    x[6] ^= rotl(x[2] + x[14], 13); x[10] ^= rotl(x[6] + x[2], 18);
    x[3] ^= rotl(x[15] + x[11], 7); x[7] ^= rotl(x[3] + x[15], 9);
    x[11] ^= rotl(x[7] + x[3], 13); x[15] ^= rotl(x[11] + x[7], 18);
    x[1] ^= rotl(x[0] + x[3], 7);   x[2] ^= rotl(x[1] + x[0], 9);
    x[3] ^= rotl(x[2] + x[1], 13);  x[0] ^= rotl(x[3] + x[2], 18);
    x[6] ^= rotl(x[5] + x[4], 7);   x[7] ^= rotl(x[6] + x[5], 9);
    x[4] ^= rotl(x[7] + x[6], 13);  x[5] ^= rotl(x[4] + x[7], 18);
    x[11] ^= rotl(x[10] + x[9], 7); x[8] ^= rotl(x[11] + x[10], 9);
    x[9] ^= rotl(x[8] + x[11], 13); x[10] ^= rotl(x[9] + x[8], 18);
    x[12] ^= rotl(x[15] + x[14], 7); x[13] ^= rotl(x[12] + x[15], 9);
    x[14] ^= rotl(x[13] + x[12], 13); x[15] ^= rotl(x[14] + x[13], 18);
  }
}

static void salsa_init(uint32_t* s, const uint8_t* k, const uint8_t* in16) {
  s[0] = ld32(SIGMA); s[5] = ld32(SIGMA + 4); s[10] = ld32(SIGMA + 8); s[15] = ld32(SIGMA + 12);
  for (int i = 0; i < 4; i++) { s[1 + i] = ld32(k + 4 * i); s[11 + i] = ld32(k + 16 + 4 * i); }
  for (int i = 0; i < 4; i++) s[6 + i] = ld32(in16 + 4 * i);
}

// HSalsa20: derive the XSalsa20 subkey from key and the first 16 nonce bytes.
static void hsalsa20(uint8_t* out32, const uint8_t* k, const uint8_t* n16) {
  uint32_t x[16];
  salsa_init(x, k, n16);
  salsa_rounds(x);
  const int idx[8] = {0, 5, 10, 15, 6, 7, 8, 9};
  for (int i = 0; i < 8; i++) st32(out32 + 4 * i, x[idx[i]]);
}

// XOR n bytes of Salsa20(key, nonce8) keystream starting at block 0 into out.
static void salsa20_xor(uint8_t* out, const uint8_t* in, long n, const uint8_t* n8, const uint8_t* k) {
  uint8_t inb[16];
  memcpy(inb, n8, 8);
  uint64_t ctr = 0;
  uint8_t block[64];
  for (long off = 0; off < n; off += 64, ctr++) {
    for (int i = 0; i < 8; i++) inb[8 + i] = (uint8_t)(ctr >> (8 * i));
    uint32_t s[16], x[16];
    salsa_init(s, k, inb);
    memcpy(x, s, sizeof x);
    salsa_rounds(x);
    for (int i = 0; i < 16; i++) st32(block + 4 * i, x[i] + s[i]);
    long m = n - off < 64 ? n - off : 64;
    for (long i = 0; i < m; i++) out[off + i] = (in ? in[off + i] : 0) ^ block[i];
  }
}

static int poly1305(uint8_t* tag, const uint8_t* key32, const uint8_t* msg, long n) {
  EVP_MAC* mac = EVP_MAC_fetch(nullptr, "POLY1305", nullptr);
  if (!mac) return -1;
  EVP_MAC_CTX* ctx = EVP_MAC_CTX_new(mac);
  size_t outl = 0;
  int ok = ctx && EVP_MAC_init(ctx, key32, 32, nullptr) == 1 && EVP_MAC_update(ctx, msg, (size_t)n) == 1 &&
           EVP_MAC_final(ctx, tag, &outl, 16) == 1 && outl == 16;
  EVP_MAC_CTX_free(ctx);
  EVP_MAC_free(mac);
  return ok ? 0 : -1;
}

// NaCl crypto_secretbox (as golang.org/x/crypto/nacl/secretbox.Seal): out = tag(16) || ciphertext(n).
long kc_secretbox_seal(const uint8_t* key32, const uint8_t* nonce24, const uint8_t* in, long n, uint8_t* out) {
  uint8_t sub[32];
  hsalsa20(sub, key32, nonce24);
  std::vector<uint8_t> buf(32 + n);
  std::vector<uint8_t> zin(32 + n, 0);
  memcpy(zin.data() + 32, in, n);
  salsa20_xor(buf.data(), zin.data(), 32 + n, nonce24 + 16, sub);   // buf[0:32] = poly key
  memcpy(out + 16, buf.data() + 32, n);
  int rc = poly1305(out, buf.data(), out + 16, n);
  OPENSSL_cleanse(sub, sizeof sub);
  OPENSSL_cleanse(buf.data(), 32);
  return rc == 0 ? n + 16 : -1;
}

// in = tag || ciphertext (n bytes). Returns n - 16 or -2 if authentication fails.
long kc_secretbox_open(const uint8_t* key32, const uint8_t* nonce24, const uint8_t* in, long n, uint8_t* out) {
  if (n < 16) return -2;
  uint8_t sub[32], pk[32], tag[16];
  hsalsa20(sub, key32, nonce24);
  salsa20_xor(pk, nullptr, 32, nonce24 + 16, sub);
  if (poly1305(tag, pk, in + 16, n - 16) != 0) return -1;
  if (CRYPTO_memcmp(tag, in, 16) != 0) return -2;
  std::vector<uint8_t> zin(n - 16 + 32, 0), ks(n - 16 + 32);
  memcpy(zin.data() + 32, in + 16, n - 16);
  salsa20_xor(ks.data(), zin.data(), (long)zin.size(), nonce24 + 16, sub);
  memcpy(out, ks.data() + 32, n - 16);
  OPENSSL_cleanse(sub, sizeof sub);
  return n - 16;
}

// ---------------------------------------------------------------- x509
// All x509 entry points write NUL-terminated PEM/text into (out, cap) and return its length,
// or -1 on error (message in out).
static long put(char* out, long cap, const std::string& s) {
  if ((long)s.size() + 1 > cap) return -1;
  memcpy(out, s.c_str(), s.size() + 1);
  return (long)s.size();
}
static long fail(char* out, long cap, const char* what) {
  std::string m = what;
  unsigned long e = ERR_get_error();
  if (e) { char b[256]; ERR_error_string_n(e, b, sizeof b); m += ": "; m += b; }
  if (cap > 0) { strncpy(out, m.c_str(), cap - 1); out[cap - 1] = 0; }
  return -1;
}
static std::string bio_str(BIO* b) {
  char* p = nullptr;
  long n = BIO_get_mem_data(b, &p);
  return std::string(p, n);
}
static EVP_PKEY* load_key(const char* pem) {
  BIO* b = BIO_new_mem_buf(pem, -1);
  EVP_PKEY* k = PEM_read_bio_PrivateKey(b, nullptr, nullptr, nullptr);
  BIO_free(b);
  return k;
}
static X509* load_cert(const char* pem) {
  BIO* b = BIO_new_mem_buf(pem, -1);
  X509* c = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
  BIO_free(b);
  return c;
}

// New private key: kind "ec" (P-256) or "rsa" (bits). PKCS#8 PEM.
long kc_genkey(const char* kind, int bits, char* out, long cap) {
  EVP_PKEY* k = nullptr;
  if (strcmp(kind, "rsa") == 0) k = EVP_RSA_gen(bits > 0 ? bits : 2048);
  else k = EVP_EC_gen("P-256");
  if (!k) return fail(out, cap, "keygen");
  BIO* b = BIO_new(BIO_s_mem());
  PEM_write_bio_PrivateKey(b, k, nullptr, nullptr, 0, nullptr, nullptr);
  long r = put(out, cap, bio_str(b));
  BIO_free(b);
  EVP_PKEY_free(k);
  return r;
}

// Subject "CN=name;O=group1;O=group2" -> X509_NAME
static X509_NAME* make_name(const char* subj) {
  X509_NAME* n = X509_NAME_new();
  std::string s = subj;
  size_t pos = 0;
  while (pos <= s.size()) {
    size_t e = s.find(';', pos);
    std::string part = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
    size_t eq = part.find('=');
    if (eq != std::string::npos)
      X509_NAME_add_entry_by_txt(n, part.substr(0, eq).c_str(), MBSTRING_UTF8,
                                 (const unsigned char*)part.c_str() + eq + 1, -1, -1, 0);
    if (e == std::string::npos) break;
    pos = e + 1;
  }
  return n;
}

static void add_ext(X509* c, X509* issuer, int nid, const char* value) {
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, issuer, c, nullptr, nullptr, 0);
  X509_EXTENSION* ex = X509V3_EXT_conf_nid(nullptr, &ctx, nid, value);
  if (ex) { X509_add_ext(c, ex, -1); X509_EXTENSION_free(ex); }
}

// Issue a certificate for public key `pub_from_key_pem` (a private key PEM) or `csr_pem`.
// ca_cert/ca_key NULL -> self-signed CA. usage: "ca" | "server" | "client" | "both".
// sans: comma-separated "DNS:x,IP:1.2.3.4" (may be empty). subj: "CN=..;O=.." (ignored for a CSR
// unless non-empty).
long kc_issue_cert(const char* key_pem, const char* csr_pem, const char* subj, const char* ca_cert_pem,
                   const char* ca_key_pem, long days, const char* usage, const char* sans, long serial,
                   char* out, long cap) {
  EVP_PKEY* pub = nullptr;
  X509_REQ* req = nullptr;
  X509_NAME* name = nullptr;
  if (csr_pem && *csr_pem) {
    BIO* b = BIO_new_mem_buf(csr_pem, -1);
    req = PEM_read_bio_X509_REQ(b, nullptr, nullptr, nullptr);
    BIO_free(b);
    if (!req) return fail(out, cap, "bad CSR");
    pub = X509_REQ_get_pubkey(req);
    if (!pub || X509_REQ_verify(req, pub) != 1) { X509_REQ_free(req); EVP_PKEY_free(pub); return fail(out, cap, "CSR signature"); }
    name = (subj && *subj) ? make_name(subj) : X509_NAME_dup(X509_REQ_get_subject_name(req));
  } else {
    pub = load_key(key_pem);
    if (!pub) return fail(out, cap, "bad key");
    name = make_name(subj);
  }
  EVP_PKEY* signer = nullptr;
  X509* ca = nullptr;
  if (ca_cert_pem && *ca_cert_pem) {
    ca = load_cert(ca_cert_pem);
    signer = load_key(ca_key_pem);
    if (!ca || !signer) { EVP_PKEY_free(pub); X509_NAME_free(name); X509_REQ_free(req); X509_free(ca); EVP_PKEY_free(signer);
      return fail(out, cap, "bad CA"); }
  } else {
    signer = pub;
    EVP_PKEY_up_ref(signer);
  }
  X509* c = X509_new();
  X509_set_version(c, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(c), serial > 0 ? serial : 1);
  X509_gmtime_adj(X509_getm_notBefore(c), -300);
  X509_gmtime_adj(X509_getm_notAfter(c), days * 86400L);
  X509_set_pubkey(c, pub);
  X509_set_subject_name(c, name);
  X509_set_issuer_name(c, ca ? X509_get_subject_name(ca) : name);
  X509* issuer = ca ? ca : c;
  std::string u = usage ? usage : "both";
  if (u == "ca") {
    add_ext(c, issuer, NID_basic_constraints, "critical,CA:TRUE");
    add_ext(c, issuer, NID_key_usage, "critical,digitalSignature,keyEncipherment,keyCertSign");
  } else {
    add_ext(c, issuer, NID_basic_constraints, "critical,CA:FALSE");
    add_ext(c, issuer, NID_key_usage, "critical,digitalSignature,keyEncipherment");
    const char* eku = u == "server" ? "serverAuth" : u == "client" ? "clientAuth" : "serverAuth,clientAuth";
    add_ext(c, issuer, NID_ext_key_usage, eku);
  }
  add_ext(c, issuer, NID_subject_key_identifier, "hash");
  if (sans && *sans) add_ext(c, issuer, NID_subject_alt_name, sans);
  long r;
  if (X509_sign(c, signer, EVP_sha256()) <= 0) {
    r = fail(out, cap, "sign");
  } else {
    BIO* b = BIO_new(BIO_s_mem());
    PEM_write_bio_X509(b, c);
    r = put(out, cap, bio_str(b));
    BIO_free(b);
  }
  X509_free(c); X509_free(ca); EVP_PKEY_free(signer); EVP_PKEY_free(pub); X509_NAME_free(name); X509_REQ_free(req);
  return r;
}

// PKCS#10 CSR for key_pem with subject subj ("CN=..;O=..").
long kc_make_csr(const char* key_pem, const char* subj, char* out, long cap) {
  EVP_PKEY* k = load_key(key_pem);
  if (!k) return fail(out, cap, "bad key");
  X509_REQ* r = X509_REQ_new();
  X509_NAME* n = make_name(subj);
  X509_REQ_set_subject_name(r, n);
  X509_REQ_set_pubkey(r, k);
  long rc;
  if (X509_REQ_sign(r, k, EVP_sha256()) <= 0) rc = fail(out, cap, "csr sign");
  else {
    BIO* b = BIO_new(BIO_s_mem());
    PEM_write_bio_X509_REQ(b, r);
    rc = put(out, cap, bio_str(b));
    BIO_free(b);
  }
  X509_NAME_free(n); X509_REQ_free(r); EVP_PKEY_free(k);
  return rc;
}

static std::string name_text(X509_NAME* n) {
  // "CN=x;O=a;O=b" in entry order
  std::string s;
  for (int i = 0; i < X509_NAME_entry_count(n); i++) {
    X509_NAME_ENTRY* e = X509_NAME_get_entry(n, i);
    int nid = OBJ_obj2nid(X509_NAME_ENTRY_get_object(e));
    unsigned char* u = nullptr;
    int l = ASN1_STRING_to_UTF8(&u, X509_NAME_ENTRY_get_data(e));
    if (l < 0) continue;
    if (!s.empty()) s += ";";
    s += OBJ_nid2sn(nid);
    s += "=";
    s.append((char*)u, l);
    OPENSSL_free(u);
  }
  return s;
}

// Subject of a certificate (kind 0) or CSR (kind 1) as "CN=..;O=..".
long kc_subject(const char* pem, int kind, char* out, long cap) {
  if (kind == 0) {
    X509* c = load_cert(pem);
    if (!c) return fail(out, cap, "bad cert");
    long r = put(out, cap, name_text(X509_get_subject_name(c)));
    X509_free(c);
    return r;
  }
  BIO* b = BIO_new_mem_buf(pem, -1);
  X509_REQ* q = PEM_read_bio_X509_REQ(b, nullptr, nullptr, nullptr);
  BIO_free(b);
  if (!q) return fail(out, cap, "bad CSR");
  long r = put(out, cap, name_text(X509_REQ_get_subject_name(q)));
  X509_REQ_free(q);
  return r;
}

// Verify cert_pem was issued by ca_pem and is currently valid. 0 = ok, else -1 (reason in out).
long kc_verify_cert(const char* cert_pem, const char* ca_pem, char* out, long cap) {
  X509* c = load_cert(cert_pem);
  X509* ca = load_cert(ca_pem);
  long r = -1;
  if (c && ca) {
    X509_STORE* st = X509_STORE_new();
    X509_STORE_add_cert(st, ca);
    X509_STORE_CTX* ctx = X509_STORE_CTX_new();
    X509_STORE_CTX_init(ctx, st, c, nullptr);
    if (X509_verify_cert(ctx) == 1) r = put(out, cap, "ok") >= 0 ? 0 : -1;
    else fail(out, cap, X509_verify_cert_error_string(X509_STORE_CTX_get_error(ctx)));
    X509_STORE_CTX_free(ctx);
    X509_STORE_free(st);
  } else {
    fail(out, cap, "bad cert");
  }
  X509_free(c);
  X509_free(ca);
  return r;
}

// notAfter as seconds since the epoch (or -1).
long kc_cert_not_after(const char* pem) {
  X509* c = load_cert(pem);
  if (!c) return -1;
  struct tm t;
  long r = -1;
  if (ASN1_TIME_to_tm(X509_get0_notAfter(c), &t) == 1) r = (long)timegm(&t);
  X509_free(c);
  return r;
}

long kc_cert_not_before(const char* pem) {
  X509* c = load_cert(pem);
  if (!c) return -1;
  struct tm t;
  long r = -1;
  if (ASN1_TIME_to_tm(X509_get0_notBefore(c), &t) == 1) r = (long)timegm(&t);
  X509_free(c);
  return r;
}

// ---------------------------------------------------------------- signatures (JWT RS256 / ES256)
// Sign `data` with the private key (RSA: PKCS#1 v1.5 SHA-256; EC: ECDSA SHA-256, DER). Returns the
// signature length written to out, or -1.
long kc_sign(const char* key_pem, const uint8_t* data, long n, uint8_t* out, long cap) {
  EVP_PKEY* k = load_key(key_pem);
  if (!k) return -1;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  size_t sl = 0;
  long r = -1;
  if (EVP_DigestSignInit(ctx, nullptr, EVP_sha256(), nullptr, k) == 1 &&
      EVP_DigestSign(ctx, nullptr, &sl, data, (size_t)n) == 1 && (long)sl <= cap &&
      EVP_DigestSign(ctx, out, &sl, data, (size_t)n) == 1)
    r = (long)sl;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(k);
  return r;
}

// PEM of the public key of a private key / certificate / public key.
long kc_public_key(const char* pem, char* out, long cap) {
  EVP_PKEY* k = load_key(pem);
  if (!k) {
    X509* c = load_cert(pem);
    if (c) { k = X509_get_pubkey(c); X509_free(c); }
  }
  if (!k) {
    BIO* b = BIO_new_mem_buf(pem, -1);
    k = PEM_read_bio_PUBKEY(b, nullptr, nullptr, nullptr);
    BIO_free(b);
  }
  if (!k) return fail(out, cap, "no key");
  BIO* b = BIO_new(BIO_s_mem());
  PEM_write_bio_PUBKEY(b, k);
  long r = put(out, cap, bio_str(b));
  BIO_free(b);
  EVP_PKEY_free(k);
  return r;
}

// 1 = valid, 0 = invalid signature, -1 = bad key.
long kc_verify(const char* pub_pem, const uint8_t* data, long n, const uint8_t* sig, long sl) {
  BIO* b = BIO_new_mem_buf(pub_pem, -1);
  EVP_PKEY* k = PEM_read_bio_PUBKEY(b, nullptr, nullptr, nullptr);
  BIO_free(b);
  if (!k) return -1;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  long r = 0;
  if (EVP_DigestVerifyInit(ctx, nullptr, EVP_sha256(), nullptr, k) == 1 &&
      EVP_DigestVerify(ctx, sig, (size_t)sl, data, (size_t)n) == 1)
    r = 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(k);
  ERR_clear_error();
  return r;
}

}  // extern "C"
