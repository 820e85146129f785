// MEHP24 helpers used by DirectSort::sort_hybrid1 (reference
// src/mehp24/mehp24_utils.cpp; see mehp24_utils.h).
#include "mehp24/mehp24_utils.h"

using namespace lbcrypto;

namespace mehp24 {
namespace utils {

Ciphertext<DCRTPoly> signAdv(Ciphertext<DCRTPoly>& c, const size_t dg, const size_t df) {
    // g3 / f3 in the power basis (reference :248-253; sign.cpp:17-21, :40-44)
    static const std::vector<double> g3 = {0, 4589.0 / 1024.0, 0, -16577.0 / 1024.0,
                                           0, 25614.0 / 1024.0, 0, -12860.0 / 1024.0};
    static const std::vector<double> f3 = {0, 35.0 / 16.0, 0, -35.0 / 16.0, 0, 21.0 / 16.0, 0, -5.0 / 16.0};
    static const std::vector<double> f3Final = {0.5, 35.0 / 32.0, 0, -35.0 / 32.0, 0, 21.0 / 32.0, 0, -5.0 / 32.0};
    auto cc = c->GetCryptoContext();
    for (size_t d = 0; d < dg; ++d) c = cc->EvalPolyLinear(c, g3);
    for (size_t d = 0; d + 1 < df; ++d) c = cc->EvalPolyLinear(c, f3);
    c = cc->EvalPolyLinear(c, f3Final);
    return c;
}

Ciphertext<DCRTPoly> indicatorAdv(const Ciphertext<DCRTPoly>& c, const double b, const size_t dg,
                                  const size_t df) {
    auto cc = c->GetCryptoContext();
    auto tmp = cc->EvalMult(c, 1.0 / b);   // (1.0 / b) * c
    auto c1 = cc->EvalAdd(tmp, 0.5 / b);   // tmp + 0.5 / b
    auto c2 = cc->EvalSub(tmp, 0.5 / b);   // tmp - 0.5 / b
    c1 = signAdv(c1, dg, df);
    c2 = signAdv(c2, dg, df);
    return cc->EvalMult(c1, cc->EvalSub(1.0, c2));  // c1 * (1 - c2)
}

uint32_t depth2degree(const uint32_t depth) {
    // the largest Chebyshev degree EvalChebyshevSeriesPS evaluates in
    // `depth` levels, shifted by one (reference :215-244)
    static const uint32_t t[] = {2, 5, 13, 27, 59, 119, 247, 495, 1007, 2031, 4031, 8127};
    return depth >= 3 && depth <= 14 ? t[depth - 3] : (uint32_t)-1;
}

std::vector<int32_t> getRotationIndices(const size_t matrixSize) {
    size_t sz = matrixSize;
    std::vector<int32_t> idx;
    if (matrixSize > 256) {
        for (size_t i = 0; i < matrixSize / 256; ++i) {
            idx.push_back((int32_t)(i * 256));
            idx.push_back(-(int32_t)(i * 256));
        }
        sz = 256;
    }
    for (size_t i = 0; i < LOG2(sz); ++i) {
        idx.push_back(1 << i);
        idx.push_back(-(1 << i));
        idx.push_back(-(1 << (LOG2(sz) + i)));
        const int32_t t = (int32_t)(sz * (sz - 1) / ((size_t)1 << (i + 1)));
        idx.push_back(t);
        idx.push_back(-t);
    }
    return idx;
}

}  // namespace utils
}  // namespace mehp24
