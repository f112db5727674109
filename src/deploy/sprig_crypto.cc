#include "deploy/sprig_crypto.h"

#include <crypt.h>
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rand.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <stdexcept>

#include "core/codec.h"

namespace ds {
namespace sprig {

namespace {

struct PkeyDel {
  void operator()(EVP_PKEY* p) const { EVP_PKEY_free(p); }
};
struct X509Del {
  void operator()(X509* p) const { X509_free(p); }
};
struct BioDel {
  void operator()(BIO* p) const { BIO_free(p); }
};
using Pkey = std::unique_ptr<EVP_PKEY, PkeyDel>;
using Cert = std::unique_ptr<X509, X509Del>;
using Bio = std::unique_ptr<BIO, BioDel>;

[[noreturn]] void fail(const std::string& what) { throw std::runtime_error("sprig crypto: " + what); }

Pkey keygen(const std::string& type) {
  EVP_PKEY* k = nullptr;
  if (type == "rsa")
    k = EVP_PKEY_Q_keygen(nullptr, nullptr, "RSA", (size_t)2048);
  else if (type == "ecdsa")
    k = EVP_PKEY_Q_keygen(nullptr, nullptr, "EC", "P-256");
  else if (type == "ed25519")
    k = EVP_PKEY_Q_keygen(nullptr, nullptr, "ED25519");
  else
    fail("unknown key type " + type + " (rsa, ecdsa, ed25519)");
  if (!k) fail("key generation failed");
  return Pkey(k);
}

std::string bio_string(BIO* b) {
  char* data = nullptr;
  long n = BIO_get_mem_data(b, &data);
  return std::string(data, n > 0 ? (size_t)n : 0);
}

std::string key_pem(EVP_PKEY* k) {
  Bio b(BIO_new(BIO_s_mem()));
  int ok;
  if (EVP_PKEY_get_base_id(k) == EVP_PKEY_ED25519)
    ok = PEM_write_bio_PrivateKey(b.get(), k, nullptr, nullptr, 0, nullptr, nullptr);
  else  // traditional "RSA PRIVATE KEY" / "EC PRIVATE KEY" blocks, as Go's x509.Marshal{PKCS1,EC}PrivateKey
    ok = PEM_write_bio_PrivateKey_traditional(b.get(), k, nullptr, nullptr, 0, nullptr, nullptr);
  if (!ok) fail("PEM encoding of the key failed");
  return bio_string(b.get());
}

std::string cert_pem(X509* c) {
  Bio b(BIO_new(BIO_s_mem()));
  if (!PEM_write_bio_X509(b.get(), c)) fail("PEM encoding of the certificate failed");
  return bio_string(b.get());
}

void add_ext(X509* cert, X509* issuer, int nid, const std::string& value) {
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, issuer, cert, nullptr, nullptr, 0);
  X509_EXTENSION* ex = X509V3_EXT_conf_nid(nullptr, &ctx, nid, value.c_str());
  if (!ex) fail("bad certificate extension " + value);
  X509_add_ext(cert, ex, -1);
  X509_EXTENSION_free(ex);
}

// issuer == nullptr: self-signed with `key`.
Cert make_cert(const std::string& cn, const std::vector<std::string>& ips, const std::vector<std::string>& dns,
               int days, bool is_ca, EVP_PKEY* key, X509* issuer, EVP_PKEY* issuer_key) {
  Cert c(X509_new());
  X509_set_version(c.get(), 2);
  // 128-bit random serial, as crypto/x509 templates in Sprig
  unsigned char raw[16];
  RAND_bytes(raw, sizeof(raw));
  raw[0] &= 0x7f;
  BIGNUM* bn = BN_bin2bn(raw, sizeof(raw), nullptr);
  BN_to_ASN1_INTEGER(bn, X509_get_serialNumber(c.get()));
  BN_free(bn);
  X509_gmtime_adj(X509_getm_notBefore(c.get()), 0);
  X509_gmtime_adj(X509_getm_notAfter(c.get()), (long)days * 24 * 3600);
  X509_set_pubkey(c.get(), key);
  X509_NAME* name = X509_get_subject_name(c.get());
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_UTF8, (const unsigned char*)cn.c_str(), -1, -1, 0);
  X509_set_issuer_name(c.get(), issuer ? X509_get_subject_name(issuer) : name);
  X509* iss = issuer ? issuer : c.get();
  if (is_ca) {
    add_ext(c.get(), iss, NID_basic_constraints, "critical,CA:TRUE");
    add_ext(c.get(), iss, NID_key_usage, "critical,digitalSignature,keyEncipherment,keyCertSign");
  } else {
    add_ext(c.get(), iss, NID_basic_constraints, "critical,CA:FALSE");
    add_ext(c.get(), iss, NID_key_usage, "critical,digitalSignature,keyEncipherment");
  }
  add_ext(c.get(), iss, NID_ext_key_usage, "serverAuth,clientAuth");
  std::string san;
  for (auto& ip : ips) san += (san.empty() ? "" : ",") + std::string("IP:") + ip;
  for (auto& d : dns) san += (san.empty() ? "" : ",") + std::string("DNS:") + d;
  if (!san.empty()) add_ext(c.get(), iss, NID_subject_alt_name, san);
  EVP_PKEY* signer = issuer_key ? issuer_key : key;
  const EVP_MD* md = EVP_PKEY_get_base_id(signer) == EVP_PKEY_ED25519 ? nullptr : EVP_sha256();
  if (!X509_sign(c.get(), signer, md)) fail("signing the certificate failed");
  return c;
}

Value pair(X509* c, EVP_PKEY* k) {
  Value v = Value::map();
  v["Cert"] = cert_pem(c);
  v["Key"] = key_pem(k);
  return v;
}

}  // namespace

std::string gen_private_key(const std::string& type) { return key_pem(keygen(type).get()); }

Value gen_ca(const std::string& cn, int days) {
  Pkey k = keygen("rsa");
  Cert c = make_cert(cn, {}, {}, days, true, k.get(), nullptr, nullptr);
  return pair(c.get(), k.get());
}

Value gen_self_signed_cert(const std::string& cn, const std::vector<std::string>& ips,
                           const std::vector<std::string>& dns, int days) {
  Pkey k = keygen("rsa");
  Cert c = make_cert(cn, ips, dns, days, false, k.get(), nullptr, nullptr);
  return pair(c.get(), k.get());
}

Value gen_signed_cert(const std::string& cn, const std::vector<std::string>& ips, const std::vector<std::string>& dns,
                      int days, const Value& ca) {
  std::string cert_s = ca.get("Cert").as_string(), key_s = ca.get("Key").as_string();
  Bio cb(BIO_new_mem_buf(cert_s.data(), (int)cert_s.size()));
  Cert ca_cert(PEM_read_bio_X509(cb.get(), nullptr, nullptr, nullptr));
  Bio kb(BIO_new_mem_buf(key_s.data(), (int)key_s.size()));
  Pkey ca_key(PEM_read_bio_PrivateKey(kb.get(), nullptr, nullptr, nullptr));
  if (!ca_cert || !ca_key) fail("genSignedCert: the CA is not a {Cert, Key} pair of PEM blocks");
  Pkey k = keygen("rsa");
  Cert c = make_cert(cn, ips, dns, days, false, k.get(), ca_cert.get(), ca_key.get());
  return pair(c.get(), k.get());
}

std::string encrypt_aes(const std::string& password, const std::string& plaintext) {
  unsigned char key[32] = {0};
  std::memcpy(key, password.data(), std::min<size_t>(32, password.size()));
  unsigned char iv[16];
  RAND_bytes(iv, sizeof(iv));
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  std::string out((const char*)iv, sizeof(iv));
  out.resize(sizeof(iv) + plaintext.size() + 16);
  int n1 = 0, n2 = 0;
  bool ok = EVP_EncryptInit_ex(ctx, EVP_aes_256_cbc(), nullptr, key, iv) &&
            EVP_EncryptUpdate(ctx, (unsigned char*)&out[16], &n1, (const unsigned char*)plaintext.data(),
                              (int)plaintext.size()) &&
            EVP_EncryptFinal_ex(ctx, (unsigned char*)&out[16 + n1], &n2);
  EVP_CIPHER_CTX_free(ctx);
  if (!ok) fail("encryptAES failed");
  out.resize(16 + (size_t)n1 + (size_t)n2);
  return base64_encode(out);
}

std::string decrypt_aes(const std::string& password, const std::string& b64) {
  std::string raw = base64_decode(b64);
  if (raw.size() < 16 || (raw.size() - 16) % 16 != 0) fail("decryptAES: ciphertext is not a multiple of the block size");
  unsigned char key[32] = {0};
  std::memcpy(key, password.data(), std::min<size_t>(32, password.size()));
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  std::string out(raw.size(), '\0');
  int n1 = 0, n2 = 0;
  bool ok = EVP_DecryptInit_ex(ctx, EVP_aes_256_cbc(), nullptr, key, (const unsigned char*)raw.data()) &&
            EVP_DecryptUpdate(ctx, (unsigned char*)&out[0], &n1, (const unsigned char*)raw.data() + 16,
                              (int)raw.size() - 16) &&
            EVP_DecryptFinal_ex(ctx, (unsigned char*)&out[n1], &n2);
  EVP_CIPHER_CTX_free(ctx);
  if (!ok) fail("decryptAES: bad key or corrupt ciphertext");
  out.resize((size_t)n1 + (size_t)n2);
  return out;
}

std::string htpasswd(const std::string& user, const std::string& password) {
  if (user.find(':') != std::string::npos) return "invalid username: " + user;  // sprig's text
  unsigned char rnd[16];
  RAND_bytes(rnd, sizeof(rnd));
  char setting[CRYPT_GENSALT_OUTPUT_SIZE];
  // bcrypt with Go's bcrypt.DefaultCost (10) and its "$2a$" prefix, via libxcrypt
  if (!crypt_gensalt_rn("$2a$", 10, (const char*)rnd, (int)sizeof(rnd), setting, (int)sizeof(setting)))
    fail("htpasswd: bcrypt salt generation failed");
  struct crypt_data data;
  std::memset(&data, 0, sizeof(data));
  const char* h = crypt_r(password.c_str(), setting, &data);
  if (!h || h[0] == '*') fail("htpasswd: bcrypt failed");
  return user + ":" + h;
}

}  // namespace sprig
}  // namespace ds
