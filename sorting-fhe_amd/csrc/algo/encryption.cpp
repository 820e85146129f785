// Reference: src/encryption.cpp:5-33.
#include "encryption.h"

Ciphertext<DCRTPoly> Encryption::encryptInput(std::vector<double> input) {
    if (input.size() > m_cc->GetRingDimension() / 2)
        throw OpenFHEException("encryptInput: input larger than the maximum batch size (n/2)");
    return m_cc->Encrypt(m_PublicKey, m_cc->MakeCKKSPackedPlaintext(input));
}

std::vector<double> DebugEncryption::realValues(const Plaintext& pt, double threshold) {
    std::vector<double> v = pt->GetRealPackedValue();
    for (double& x : v)
        if (std::fabs(x) < threshold) x = 0.0;
    return v;
}

std::vector<double> DebugEncryption::getPlaintext(const Ciphertext<DCRTPoly>& ct,
                                                  double threshold) const {
    Plaintext pt;
    m_cc->Decrypt(m_PrivateKey, ct, &pt);
    return realValues(pt, threshold);
}

Plaintext DebugEncryption::getDecrypt(const Ciphertext<DCRTPoly>& ct) const {
    Plaintext pt;
    m_cc->Decrypt(m_PrivateKey, ct, &pt);
    return pt;
}
