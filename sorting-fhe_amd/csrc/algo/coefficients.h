// Chebyshev coefficient tables for the sinc indicators.
//
// The reference generates these at build time (utils/generate_cheb_doubled_
// coeffs.cpp:14-49, utils/generate_cheb_coeffs.cpp:14-64) by interpolating
// at degree 13011 with OpenFHE's EvalChebyshevCoefficients, thresholding,
// trimming trailing small terms and printing with the default 6-significant-
// digit ostream format.  This engine computes the same tables once per
// process (lbcrypto::EvalChebyshevCoefficients in core/chebyshev.cpp) and
// applies the same threshold / trim / %g rounding.
#pragma once
#include <cstddef>
#include <vector>

namespace sfhe {
constexpr int kSincInterpolationDegree = 13011;
// doubled sinc of Sinc<2N> on [-1,1]: |c| < 1e-8 -> 0, trailing trimmed
const std::vector<double>& doubledSincCoefficients(int N);
// scaled sinc of Sinc<2N>: odd terms zeroed, even |c| < 1e-6 -> 0
const std::vector<double>& scaledSincCoefficients(int N);
}  // namespace sfhe

template <std::size_t N>
const std::vector<double>& selectDoubledSincCoefficients() {
    return sfhe::doubledSincCoefficients((int)N);
}
template <std::size_t N>
const std::vector<double>& selectCoefficients() {
    return sfhe::scaledSincCoefficients((int)N);
}
