// Homomorphic comparison: public surface of the reference's src/comparison.h
// (Sinc<N> :11-79, Comparison :81-101); compare/indicator in comparison.cpp.
#pragma once

#include <cmath>
#include <memory>

#include "encryption.h"
#include "openfhe.h"
#include "sign.h"

using namespace lbcrypto;

// Sinc-type indicator functions interpolated by the Chebyshev generators
// (coefficients.h).  N is the period parameter; the sort uses Sinc<2N>.
template <int N>
struct Sinc {
    static constexpr double kEps = 1e-10;

    static double simple_sinc(double x) { return std::fabs(x) < 0.5 ? 1.0 : 0.0; }

    // (kept as the reference defines it: sin(pi x) / pi * x)
    static double sinc(double x) { return std::fabs(x) < kEps ? 1.0 : std::sin(M_PI * x) / M_PI * x; }

    // sin(pi N x) / (pi N x): 1 at x = 0, 0 at nonzero multiples of 1/N
    static double scaled_sinc(double x) {
        if (std::fabs(x) < kEps) return 1.0;
        const double t = M_PI * N * x;
        return std::sin(t) / t;
    }

    static double scaled_sinc_j(double x, int j) {
        auto term = [](double t) { return std::fabs(t) < kEps ? 1.0 : std::sin(t) / t; };
        const double a = N * M_PI * x - j * M_PI;
        return term(a) + term(a + N * M_PI);
    }

    // S(x) + S(x + 1/2): 1 at x in {0, -1/2} (mod the 1/N lattice), else 0;
    // used by rotationIndexCheckN on z = (i - rank - c) / (2N) in (-1, 1/2).
    static double doubled_sinc(double x) { return scaled_sinc(x) + scaled_sinc(x + 0.5); }
};

class Comparison {
  public:
    Comparison(std::shared_ptr<Encryption> enc) : m_enc(enc) {}
    Comparison() : m_enc(nullptr) {}

    // (sign(a - b) + 1) / 2: 1 if a > b, 0 if a < b, 1/2 if equal.
    Ciphertext<DCRTPoly> compare(const CryptoContext<DCRTPoly>& cc, const Ciphertext<DCRTPoly>& a,
                                 const Ciphertext<DCRTPoly>& b, SignFunc SignFunc,
                                 SignConfig& Cfg);

    // MEHP24-style: 1 if |x| < c else 0 (used by the hybrid sorts).
    Ciphertext<DCRTPoly> indicator(const CryptoContext<DCRTPoly>& cc, const Ciphertext<DCRTPoly>& x,
                                   const double c, SignFunc SignFunc, SignConfig& Cfg);

  private:
    std::shared_ptr<Encryption> m_enc;
};
