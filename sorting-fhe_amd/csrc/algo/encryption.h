// Encryption front end: public surface of the reference's src/encryption.h
// (Encryption :57-79, DebugEncryption :81-94, PRINT_PT :34-46).
#pragma once

#include <cassert>
#include <cmath>
#include <fstream>
#include <sstream>
#include <vector>

#include "ciphertext-fwd.h"
#include "key/keypair.h"
#include "lattice/hal/lat-backend.h"
#include "openfhe.h"

using namespace lbcrypto;

// Debug print of a ciphertext's decryption (compiled in when ENABLE_PRINT_PT
// is defined, as the reference's default build does: CMakeLists.txt:63-66).
#ifdef ENABLE_PRINT_PT
// (one decryption serves both the values and the precision estimate)
#define PRINT_PT(enc, ct)                                                              \
    do {                                                                               \
        if (dynamic_cast<const DebugEncryption*>((enc).get()) != nullptr) {            \
            const Plaintext _dp = (enc)->getDecrypt((ct));                             \
            std::cout << DebugEncryption::realValues(_dp) << ": " << #ct << " Level: "  \
                      << (ct)->GetLevel() << ", LogPrecision: " << _dp->GetLogPrecision() \
                      << "\n";                                                         \
        }                                                                              \
    } while (0)
#else
#define PRINT_PT(enc, ct)
#endif

class Encryption {
  public:
    Encryption(CryptoContext<DCRTPoly> cc, PublicKey<DCRTPoly> pk) : m_cc(cc), m_PublicKey(pk) {}
    virtual ~Encryption() = default;

    // Encrypts `input` packed with the context's batch size (asserts it fits
    // in n/2 slots, as encryption.cpp:5-12).
    Ciphertext<DCRTPoly> encryptInput(std::vector<double> input);

    virtual std::vector<double> getPlaintext(const Ciphertext<DCRTPoly>&,
                                             double threshold = 1e-10) const {
        (void)threshold;
        throw std::runtime_error("Decryption not available in base Encryption class");
    }
    virtual Plaintext getDecrypt(const Ciphertext<DCRTPoly>&) const {
        throw std::runtime_error("Decryption not available in base Encryption class");
    }

    CryptoContext<DCRTPoly> m_cc;
    PublicKey<DCRTPoly> m_PublicKey;
};

class DebugEncryption : public Encryption {
  public:
    DebugEncryption(CryptoContext<DCRTPoly> cc, KeyPair<DCRTPoly> kp)
        : Encryption(cc, kp.publicKey), m_PrivateKey(kp.secretKey) {}
    ~DebugEncryption() override = default;

    [[nodiscard]] std::vector<double> getPlaintext(const Ciphertext<DCRTPoly>& ct,
                                                   double threshold = 1e-10) const override;
    Plaintext getDecrypt(const Ciphertext<DCRTPoly>& ct) const override;
    // a decryption's real slot values, |x| < threshold shown as 0 (getPlaintext's form)
    static std::vector<double> realValues(const Plaintext& pt, double threshold = 1e-10);

  private:
    PrivateKey<DCRTPoly> m_PrivateKey;
};
