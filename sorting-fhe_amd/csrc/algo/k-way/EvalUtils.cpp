// k-way evaluation helpers (reference src/k-way/EvalUtils.cpp).
#include "EvalUtils.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <iostream>

namespace kwaySort {

std::vector<int> binary(int n) {
    std::vector<int> bits;
    for (; n > 0; n >>= 1) bits.push_back(n & 1);
    return bits;
}

// Horner over the binary digits of |coeff|, most significant first
void EvalUtils::multByInt(Ciphertext<DCRTPoly>& ctxt, long coeff, Ciphertext<DCRTPoly>& ctxt_out) {
    const Ciphertext<DCRTPoly> unit = coeff < 0 ? m_cc->EvalNegate(ctxt) : ctxt;
    const unsigned long c = (unsigned long)std::labs(coeff);
    ctxt_out = unit;
    if (c == 0) return;  // as the reference: the input itself (no digits to fold)
    int top = 63;
    while (!((c >> top) & 1)) --top;
    for (int b = top - 1; b >= 0; --b) {
        ctxt_out = m_cc->EvalAdd(ctxt_out, ctxt_out);
        if ((c >> b) & 1) ctxt_out = m_cc->EvalAdd(ctxt_out, unit);
    }
}

void EvalUtils::multAndKillImage(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt2,
                                 Ciphertext<DCRTPoly>& ctxt_out) {
    ctxt_out = m_cc->EvalMult(ctxt1, ctxt2);
}

void EvalUtils::squareAndKillImage(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt_out) {
    ctxt_out = m_cc->EvalSquare(ctxt1);
}

void EvalUtils::checkLevelAndBoot(Ciphertext<DCRTPoly>& ctxt, int level, int multDepth, bool verbose) {
    const int left = multDepth - (int)ctxt->GetLevel();
    if (left >= level + 1) return;  // a ciphertext at level == depth cannot be bootstrapped: keep one spare
    static const bool debug = std::getenv("SFHE_KWAY_DEBUG") != nullptr;
    verbose = verbose || (debug && m_privateKey);
    if (verbose) {
        std::cout << "Starting bootstrap at level " << ctxt->GetLevel() << " (MultDepth : " << multDepth
                  << ", Required level: " << level << ")" << std::endl;
        if (m_privateKey) debugWithSk(ctxt, 5, "before boot");
    }
    ctxt = m_cc->EvalBootstrap(ctxt);
    if (verbose) {
        std::cout << "Finished bootstrapping at level " << ctxt->GetLevel() << std::endl;
        if (m_privateKey) debugWithSk(ctxt, 5, "after boot");
    }
}

void EvalUtils::checkLevelAndBoot2(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt2, long level,
                                   long multDepth, bool verbose) {
    checkLevelAndBoot(ctxt, (int)level, (int)multDepth, verbose);
    checkLevelAndBoot(ctxt2, (int)level, (int)multDepth, verbose);
}

void EvalUtils::flipCtxt(Ciphertext<DCRTPoly>& ctxt) {
    m_cc->EvalNegateInPlace(ctxt);
    m_cc->EvalAddInPlace(ctxt, 1.0);
}

void EvalUtils::flipCtxt(Ciphertext<DCRTPoly>& ctxt, Plaintext& mask) {
    m_cc->EvalNegateInPlace(ctxt);
    m_cc->EvalAddInPlace(ctxt, mask);
}

void EvalUtils::rotateChain(Ciphertext<DCRTPoly>& ctxt, long r, int sign, Ciphertext<DCRTPoly>& ctxt_out) {
    Ciphertext<DCRTPoly> cur = ctxt;
    for (long bit = 1; bit <= r; bit <<= 1)
        if (r & bit) cur = m_cc->EvalRotate(cur, (int32_t)(sign * bit));
    ctxt_out = cur;
}

void EvalUtils::leftRotate(Ciphertext<DCRTPoly>& ctxt, long r, Ciphertext<DCRTPoly>& ctxt_out) {
    rotateChain(ctxt, r, +1, ctxt_out);
}

void EvalUtils::rightRotate(Ciphertext<DCRTPoly>& ctxt, long r, Ciphertext<DCRTPoly>& ctxt_out) {
    rotateChain(ctxt, r, -1, ctxt_out);
}

void EvalUtils::debugWithSk(Ciphertext<DCRTPoly>& ctxt, long length, const std::string& str) {
    if (!str.empty()) std::cout << "check " + str << std::endl;
    Plaintext pt;
    m_cc->Decrypt(m_privateKey, ctxt, &pt);
    const std::vector<double> v = pt->GetRealPackedValue();
    for (long i = 0; i < std::min<long>(20, length); ++i) std::cout << "(" << i << ", " << v[i] << "), ";
    for (size_t i = v.size() > 20 ? v.size() - 20 : 0; i < v.size(); ++i) std::cout << "(" << i << ", " << v[i] << "), ";
    size_t at = 0;
    double mx = 0;
    for (size_t i = 0; i < v.size(); ++i)
        if (std::fabs(v[i]) > mx) mx = std::fabs(v[i]), at = i;
    std::cout << str << " max val = " << at << ", " << mx << std::endl;
}

}  // namespace kwaySort
