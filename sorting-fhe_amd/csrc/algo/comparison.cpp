// Reference: src/comparison.cpp:4-22 (compare), :24-40 (indicator).
#include "comparison.h"

Ciphertext<DCRTPoly> Comparison::compare(const CryptoContext<DCRTPoly>& cc,
                                         const Ciphertext<DCRTPoly>& a,
                                         const Ciphertext<DCRTPoly>& b, SignFunc SignFunc,
                                         SignConfig& Cfg) {
    auto s = sign(cc->EvalSub(a, b), cc, SignFunc, Cfg);
    return cc->EvalMult(cc->EvalAdd(s, 1.0), 0.5);
}

Ciphertext<DCRTPoly> Comparison::indicator(const CryptoContext<DCRTPoly>& cc,
                                           const Ciphertext<DCRTPoly>& x, const double c,
                                           SignFunc SignFunc, SignConfig& Cfg) {
    // step(x + c) * (1 - step(x - c))
    auto step = [&](const Ciphertext<DCRTPoly>& v) {
        return cc->EvalMult(cc->EvalAdd(sign(v, cc, SignFunc, Cfg), 1.0), 0.5);
    };
    auto lower = step(cc->EvalAdd(x, c));
    auto upper = step(cc->EvalSub(x, c));
    return cc->EvalMultAndRelinearize(lower, cc->EvalSub(1.0, upper));
}
