#include "coefficients.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>

#include "comparison.h"

namespace sfhe {
namespace {

// value as printed by `std::ostream << double` with default precision (%g, 6 digits)
double round6g(double x) {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%g", x);
    return std::strtod(buf, nullptr);
}

double doubledSinc2N(int N, double x) {
    // Sinc<2N>::doubled_sinc, with the period parameter at run time
    auto S = [N](double t) {
        if (std::fabs(t) < 1e-10) return 1.0;
        const double a = M_PI * (2.0 * N) * t;
        return std::sin(a) / a;
    };
    return S(x) + S(x + 0.5);
}

double scaledSinc2N(int N, double x) {
    if (std::fabs(x) < 1e-10) return 1.0;
    const double a = M_PI * (2.0 * N) * x;
    return std::sin(a) / a;
}

std::vector<double> build(int N, bool doubled) {
    auto c = lbcrypto::EvalChebyshevCoefficients(
        [N, doubled](double x) { return doubled ? doubledSinc2N(N, x) : scaledSinc2N(N, x); },
        -1.0, 1.0, kSincInterpolationDegree);
    for (size_t i = 0; i < c.size(); ++i) {
        if (doubled) {
            if (std::fabs(c[i]) < 1e-8) c[i] = 0.0;
        } else {
            if (i % 2 == 1 || std::fabs(c[i]) < 1e-6) c[i] = 0.0;
        }
    }
    const double trim = doubled ? 1e-8 : 1e-15;
    while (!c.empty() && std::fabs(c.back()) < trim) c.pop_back();
    for (double& v : c) v = round6g(v);
    return c;
}

const std::vector<double>& cached(int N, bool doubled) {
    static std::mutex mu;
    static std::map<std::pair<int, bool>, std::unique_ptr<std::vector<double>>> tab;
    std::lock_guard<std::mutex> g(mu);
    auto& p = tab[{N, doubled}];
    if (!p) p.reset(new std::vector<double>(build(N, doubled)));
    return *p;
}

}  // namespace

const std::vector<double>& doubledSincCoefficients(int N) { return cached(N, true); }
const std::vector<double>& scaledSincCoefficients(int N) { return cached(N, false); }

}  // namespace sfhe
