// k-way sorting network: evaluation helpers (public surface of the
// reference's src/k-way/EvalUtils.h:1-96).  Rotations by arbitrary amounts
// are chains of the power-of-two keys KWayAdapter generates; level checks
// bootstrap lazily (EvalBootstrap, core/bootstrap.cpp).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "ciphertext-fwd.h"
#include "encryption.h"
#include "openfhe.h"
#include "sign.h"

using namespace lbcrypto;

namespace kwaySort {

// little-endian binary digits of n (EvalUtils.cpp:9-16)
std::vector<int> binary(int n);

class EvalUtils {
  public:
    EvalUtils() = default;
    EvalUtils(CryptoContext<DCRTPoly> cc) : m_cc(cc) {}
    EvalUtils(CryptoContext<DCRTPoly> cc, std::shared_ptr<Encryption> enc, const PublicKey<DCRTPoly>& publicKey,
              const PrivateKey<DCRTPoly>& privateKey)
        : m_cc(cc), m_publicKey(publicKey), m_privateKey(privateKey), m_enc(enc) {}

    // ctxt_out = coeff * ctxt by doublings and additions (no level)
    void multByInt(Ciphertext<DCRTPoly>& ctxt, long coeff, Ciphertext<DCRTPoly>& ctxt_out);

    // products; CKKS here carries no separate imaginary cleanup
    void multAndKillImage(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt2, Ciphertext<DCRTPoly>& ctxt_out);
    void squareAndKillImage(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt_out);

    // bootstrap ctxt when fewer than level + 1 levels remain of multDepth
    void checkLevelAndBoot(Ciphertext<DCRTPoly>& ctxt, int level, int multDepth, bool verbose = true);
    void checkLevelAndBoot2(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt2, long depth, long po2bit,
                            bool verbose = true);

    // 1 - ctxt, or mask - ctxt
    void flipCtxt(Ciphertext<DCRTPoly>& ctxt);
    void flipCtxt(Ciphertext<DCRTPoly>& ctxt, Plaintext& mask);

    // declared by the reference, never defined there (EvalUtils.h:53-67)
    void evalPoly(Ciphertext<DCRTPoly>& ctxt, const std::vector<long>& coeff, long logDivByPo2,
                  Ciphertext<DCRTPoly>& ctxt_out);
    void evalF(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_out);
    void evalG(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_out);
    void approxComp(Ciphertext<DCRTPoly>& a, Ciphertext<DCRTPoly>& b, int multDepth, long d_f, long d_g);
    void approxComp2(Ciphertext<DCRTPoly>& a, Ciphertext<DCRTPoly>& b, Ciphertext<DCRTPoly>& c,
                     Ciphertext<DCRTPoly>& d, int multDepth, long d_f, long d_g);

    // rotation by r >= 0 slots as a chain of power-of-two rotations
    void leftRotate(Ciphertext<DCRTPoly>& ctxt, long r, Ciphertext<DCRTPoly>& ctxt_out);
    void rightRotate(Ciphertext<DCRTPoly>& ctxt, long r, Ciphertext<DCRTPoly>& ctxt_out);

    void debugWithSk(Ciphertext<DCRTPoly>& ctxt, long length, const std::string& str);

    void setPrivateKey(const PrivateKey<DCRTPoly>& privateKey) { m_privateKey = privateKey; }
    void setPublicKey(const PublicKey<DCRTPoly>& publicKey) { m_publicKey = publicKey; }

  protected:
    // the power-of-two chain of a rotation by `sign * r`
    void rotateChain(Ciphertext<DCRTPoly>& ctxt, long r, int sign, Ciphertext<DCRTPoly>& ctxt_out);

    CryptoContext<DCRTPoly> m_cc;
    PublicKey<DCRTPoly> m_publicKey;
    PrivateKey<DCRTPoly> m_privateKey;
    std::shared_ptr<Encryption> m_enc;
};

}  // namespace kwaySort
