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

// The same polynomial p(z) = c0/2 + sum c_k T_k(z) re-expanded on the
// sub-interval z in [lo, hi] (within [-1, 1]):  p(z) = d0/2 + sum d_k T_k(y),
// y = (2z - lo - hi) / (hi - lo).  Restricting a Chebyshev series to a
// sub-interval is well conditioned (|d| <= ~|c|); terms below 1e-12 max|d|
// are dropped (|change| < 1e-12 at every point).  Used by the placement
// (DESIGN.md §2 "precision"): the reference's z = (r - rank - c)/2N only
// takes values in (-1, 1/2), and its hits z = 0 sit where every
// T_{2^i}(z) = +-1, the points where noise injected into the PS giant steps
// (T_2M = 2 T_M^2 - 1) grows 4x per doubling; at y = 1/3 it grows ~2x.
const std::vector<double>& rebasedChebyshev(const std::vector<double>& c, double lo, double hi);
}  // namespace sfhe

template <std::size_t N>
const std::vector<double>& selectDoubledSincCoefficients() {
    return sfhe::doubledSincCoefficients((int)N);
}
template <std::size_t N>
const std::vector<double>& selectCoefficients() {
    return sfhe::scaledSincCoefficients((int)N);
}
