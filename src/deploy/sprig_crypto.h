// Sprig's certificate and encryption functions for chart templates (genPrivateKey, genCA,
// genSelfSignedCert, genSignedCert, encryptAES, decryptAES), on OpenSSL. Charts that ship
// admission webhooks or TLS endpoints generate their certificates with these at install time.
#pragma once

#include <string>
#include <vector>

#include "core/value.h"

namespace ds {
namespace sprig {

// PEM private key: "rsa" (2048 bit, PKCS#1 "RSA PRIVATE KEY"), "ecdsa" (P-256, "EC PRIVATE
// KEY"), "ed25519" (PKCS#8 "PRIVATE KEY"), as Sprig's genPrivateKey.
std::string gen_private_key(const std::string& type);
// {Cert, Key} PEM strings. CA: RSA-2048 key, CA basic constraints, certSign usage.
Value gen_ca(const std::string& cn, int days);
Value gen_self_signed_cert(const std::string& cn, const std::vector<std::string>& ips,
                           const std::vector<std::string>& dns, int days);
// Signed by `ca` ({Cert, Key} as genCA returns).
Value gen_signed_cert(const std::string& cn, const std::vector<std::string>& ips, const std::vector<std::string>& dns,
                      int days, const Value& ca);
// AES-256-CBC, key = password bytes zero-padded/truncated to 32, random IV, PKCS#7 padding,
// base64(iv || ciphertext) — Sprig's format, so values round-trip with charts rendered by Helm.
std::string encrypt_aes(const std::string& password, const std::string& plaintext);
std::string decrypt_aes(const std::string& password, const std::string& b64);
// "user:$2a$10$..." (bcrypt, cost 10), the htpasswd line docker-registry style charts render.
std::string htpasswd(const std::string& user, const std::string& password);

}  // namespace sprig
}  // namespace ds
