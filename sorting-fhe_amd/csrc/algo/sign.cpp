// Composite sign polynomials on the device engine.
//
// Reference: src/sign.cpp:9-60 (CompositeSign<3>), :62-158
// (CompositeSign<4>), :160-185 (composition with lazy bootstrap),
// :635-651 (dispatcher).  The polynomials are the published ones
// (Cheon-Kim-Kim 2019); the evaluation order keeps the reference's depth:
// every odd polynomial of degree 2^k - 1 costs exactly k levels because the
// coefficient multiplications happen at depth 1.
#include "sign.h"

#include <cmath>
#include <map>
#include <vector>

using namespace lbcrypto;

namespace {

using Ct = Ciphertext<DCRTPoly>;

// sum_{i} c[i] x^(2i+1) for c.size() == 2^(k-1) odd coefficients, depth k:
//   P(x) = A(x) + B(x) * x^(2^(k-1)),  A,B of half the degree.
// pw[j] holds x^(2^(j+1)) (x^2, x^4, x^8, ...).
//
// Every term lands directly at the level its sum works at, so no partial sum
// is level-adjusted: B is formed at the level just above the product's, A at
// the product's level, and a coefficient times x at whatever level it is
// wanted, as one weighted sum that folds the scale into its integer weight
// (one rescale, like EvalMult(x, c), but at any level below x's).  Only a
// power x^(2^j) may need aligning, once per level (memo).  Degree 7: 10
// rescales instead of 12 (4 coefficient products, 5 ciphertext products, x^2
// aligned once); same depth and polynomial.
struct OddPoly {
    const CryptoContext<DCRTPoly>& cc;
    const Ct& x;
    const std::vector<Ct>& pw;
    std::map<std::pair<size_t, uint32_t>, Ct> aligned;

    // c x at level `at` (> x's level)
    Ct constAt(double c, uint32_t at) {
        const uint64_t *r0, *r1;
        std::vector<DeviceBufferPtr> keep;
        cc->RowsAt(x, at - 1, &r0, &r1, keep);  // settled (and gathered into a replicated tail)
        const std::vector<const uint64_t*> i0{r0}, i1{r1};
        const std::vector<double> w{c}, sc{x->scale};
        return cc->LinearWSumRescale(i0, i1, w, at - 1, x->GetSlots(), &sc);
    }
    const Ct& power(size_t j, uint32_t level) {
        if (pw[j]->GetLevel() >= level) return pw[j];
        auto key = std::make_pair(j, level);
        auto it = aligned.find(key);
        if (it != aligned.end()) return it->second;
        return aligned[key] = cc->AdjustLevel(pw[j], level);
    }
    static size_t powIndex(size_t half) {
        size_t j = 0;
        while ((size_t)2 << j < 2 * half) ++j;  // x^(2*half) = pw[j]
        return j;
    }
    // level eval(c, cnt, 0) reaches
    uint32_t natural(size_t cnt) const {
        if (cnt == 1) return x->GetLevel() + 1;
        const size_t half = cnt / 2;
        return std::max(natural(half), pw[powIndex(half)]->GetLevel()) + 1;
    }
    Ct eval(const double* c, size_t cnt, uint32_t want) {
        if (cnt == 1) return constAt(c[0], std::max(x->GetLevel() + 1, want));
        const size_t half = cnt / 2, j = powIndex(half);
        const uint32_t Lp = std::max(std::max(natural(half), pw[j]->GetLevel()) + 1, want);
        Ct hi = eval(c + half, half, Lp - 1);
        Ct prod = cc->EvalMult(hi, power(j, Lp - 1));
        Ct lo = eval(c, half, Lp);
        return cc->EvalAdd(lo, prod);
    }
};

Ct oddPolyFull(const CryptoContext<DCRTPoly>& cc, const Ct& x, const std::vector<double>& c) {
    // even powers x^2, x^4, ... up to x^(cnt)
    std::vector<Ct> pw;
    pw.push_back(cc->EvalSquare(x));
    for (size_t p = 4; p < 2 * c.size(); p *= 2) pw.push_back(cc->EvalSquare(pw.back()));
    OddPoly op{cc, x, pw, {}};
    return op.eval(c.data(), c.size(), 0);
}

template <int n>
struct CompositePolys;

// g_3(x) = (4589x - 16577x^3 + 25614x^5 - 12860x^7) / 2^10
// f_3(x) = (35x - 35x^3 + 21x^5 - 5x^7) / 2^4
template <>
struct CompositePolys<3> {
    static constexpr int g_depth = 3, f_depth = 3;
    static Ct g(const Ct& x, const CryptoContext<DCRTPoly>& cc) {
        static const std::vector<double> c = {4589.0 / 1024, -16577.0 / 1024, 25614.0 / 1024,
                                              -12860.0 / 1024};
        return oddPolyFull(cc, x, c);
    }
    static Ct f(const Ct& x, const CryptoContext<DCRTPoly>& cc) {
        static const std::vector<double> c = {35.0 / 16, -35.0 / 16, 21.0 / 16, -5.0 / 16};
        return oddPolyFull(cc, x, c);
    }
};

// g_4: degree-27 Chebyshev series (depth 5); f_4: odd degree-15 (depth 4).
template <>
struct CompositePolys<4> {
    static constexpr int g_depth = 4, f_depth = 4;
    static Ct g(const Ct& x, const CryptoContext<DCRTPoly>& cc) {
        static const std::vector<double> cheb = {
            0.0, 1.077117252745569,    0.0, -0.36166113998402755,
            0.0, 0.2137420717859748,   0.0, -0.15635204788780485,
            0.0, 0.11749645501187332,  0.0, -0.10074154666447852,
            0.0, 0.08002086947825496,  0.0, -0.07533558758484624,
            0.0, 0.059514472116534836, 0.0, -0.06146663712787884,
            0.0, 0.04570084927999001,  0.0, -0.05403683682999072,
            0.0, 0.03364293851188723,  0.0, -0.054459493266273494};
        return cc->EvalChebyshevSeriesPS(x, cheb, -1, 1);
    }
    static Ct f(const Ct& x, const CryptoContext<DCRTPoly>& cc) {
        static const std::vector<double> c = {3.14208984375,  -7.33154296875, 13.19677734375,
                                              -15.71044921875, 12.21923828125, -5.99853515625,
                                              1.69189453125,  -0.20947265625};
        return oddPolyFull(cc, x, c);
    }
};

}  // namespace

template <int n>
Ciphertext<DCRTPoly> compositeSign(Ciphertext<DCRTPoly> x, CryptoContext<DCRTPoly> cc,
                                   const SignConfig& Cfg) {
    // Bootstrap before a polynomial that would not fit the remaining budget
    // (never triggers at the default multDepth = 100).
    auto refresh = [&](Ct& c, int need) {
        if (Cfg.multDepth - (int)c->GetLevel() < need + 2) c = cc->EvalBootstrap(c);
    };
    // g is applied max(dg, 1) times: the reference applies it once before
    // its loop over i = 1 .. dg-1 (src/sign.cpp:173-178), so dg = 0 still
    // evaluates g once (SignTest's CompositeSignTest relies on it).
    Ct y = x;
    const int gCount = Cfg.compos.dg > 1 ? Cfg.compos.dg : 1;
    for (int i = 0; i < gCount; ++i) {
        refresh(y, CompositePolys<n>::g_depth);
        y = CompositePolys<n>::g(y, cc);
    }
    for (int i = 0; i < Cfg.compos.df; ++i) {
        refresh(y, CompositePolys<n>::f_depth);
        y = CompositePolys<n>::f(y, cc);
    }
    return y;
}

template Ciphertext<DCRTPoly> compositeSign<3>(Ciphertext<DCRTPoly>, CryptoContext<DCRTPoly>,
                                               const SignConfig&);
template Ciphertext<DCRTPoly> compositeSign<4>(Ciphertext<DCRTPoly>, CryptoContext<DCRTPoly>,
                                               const SignConfig&);

Ciphertext<DCRTPoly> sign(Ciphertext<DCRTPoly> x, CryptoContext<DCRTPoly> cc, SignFunc func,
                          const SignConfig& Cfg) {
    if (func == SignFunc::CompositeSign) {
        if (Cfg.compos.n == 3) return compositeSign<3>(x, cc, Cfg);
        if (Cfg.compos.n == 4) return compositeSign<4>(x, cc, Cfg);
    }
    // SignumPolycircuit / Tanh / NaiveDiscrete (and the reference's
    // fall-through for other n, sign.cpp:638-645) are outside the hot path.
    throw OpenFHEException("sign: only SignFunc::CompositeSign with n in {3,4} is implemented");
}
