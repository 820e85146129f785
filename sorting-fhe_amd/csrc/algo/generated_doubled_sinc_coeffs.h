// Forwarding header: the reference generates generated_doubled_sinc_coeffs.h at build time
// (utils/generate_cheb_*coeffs.cpp); this engine computes the same tables
// (coefficients.h: selectDoubledSincCoefficients<N>, selectCoefficients<N>).
#pragma once
#include "coefficients.h"
