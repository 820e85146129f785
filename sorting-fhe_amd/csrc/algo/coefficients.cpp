#include "coefficients.h"

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <tuple>
#include <memory>
#include <mutex>
#include <thread>

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

std::vector<double> rebase(const std::vector<double>& c, double lo, double hi) {
    const size_t D = c.size() - 1;
    // p at the D+1 Chebyshev nodes of y (Clenshaw in long double), then the
    // discrete Chebyshev transform: exact for a degree-D polynomial.  O(D^2)
    // in long double: over the host's cores (the cold sort paid it serially)
    std::vector<long double> pv(D + 1);
    lbcrypto::ParallelFor(D + 1, [&](size_t j) {
        const long double y = std::cos((long double)M_PI * ((long double)j + 0.5L) / (long double)(D + 1));
        const long double z = (long double)lo + (y + 1.0L) * ((long double)hi - (long double)lo) / 2.0L;
        long double b1 = 0, b2 = 0;
        for (size_t k = D; k >= 1; --k) {
            const long double b0 = 2.0L * z * b1 - b2 + (long double)c[k];
            b2 = b1;
            b1 = b0;
        }
        pv[j] = z * b1 - b2 + 0.5L * (long double)c[0];
    });
    // cos(pi k (2j+1) / (2(D+1))) depends on k(2j+1) mod 4(D+1)
    const size_t P = 4 * (D + 1);
    std::vector<long double> ctab(P);
    for (size_t m = 0; m < P; ++m) ctab[m] = std::cos((long double)M_PI * (long double)m / (2.0L * (D + 1)));
    std::vector<double> d(D + 1);
    lbcrypto::ParallelFor(D + 1, [&](size_t k) {
        long double acc = 0;
        size_t idx = k % P;
        const size_t step = (2 * k) % P;
        for (size_t j = 0; j <= D; ++j) {
            acc += pv[j] * ctab[idx];
            idx += step;
            if (idx >= P) idx -= P;
        }
        d[k] = (double)(acc * 2.0L / (long double)(D + 1));
    });
    double mx = 0;
    for (double v : d) mx = std::max(mx, std::fabs(v));
    for (double& v : d)
        if (std::fabs(v) < 1e-12 * mx) v = 0.0;
    while (d.size() > 1 && d.back() == 0.0) d.pop_back();
    return d;
}

}  // namespace

const std::vector<double>& rebasedChebyshev(const std::vector<double>& c, double lo, double hi) {
    static std::mutex mu;
    static std::map<std::tuple<uint64_t, size_t, double, double>, std::unique_ptr<std::vector<double>>> tab;
    uint64_t h = 1469598103934665603ull;  // content key (FNV-1a over the bits)
    for (double v : c) {
        uint64_t b;
        std::memcpy(&b, &v, 8);
        h = (h ^ b) * 1099511628211ull;
    }
    std::lock_guard<std::mutex> g(mu);
    auto& p = tab[std::make_tuple(h, c.size(), lo, hi)];
    if (!p) p.reset(new std::vector<double>(c.empty() ? c : rebase(c, lo, hi)));
    return *p;
}

const std::vector<double>& doubledSincCoefficients(int N) { return cached(N, true); }
const std::vector<double>& scaledSincCoefficients(int N) { return cached(N, false); }

}  // namespace sfhe
