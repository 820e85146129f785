// CKKS canonical-embedding encoder (host).
//
// Slot j of a plaintext m(X) is m(zeta^(5^j)), zeta = exp(i*pi/n), so the
// automorphism X -> X^(5^r) is a left rotation by r (OpenFHE convention,
// SURVEY.md §8(a) a-12(ii)).  A vector of `slots` < n/2 values is packed
// sparsely: m(X) = sum_t u_t X^(t*gap), gap = n/(2*slots), which replicates
// the vector with period `slots` across all n/2 slots (a-12(i)).
// The transform is the standard O(S log S) "special FFT" over the rotation
// group <5> mod 2n (Cheon-Kim-Kim-Song).
#include <algorithm>
#include <cmath>
#include <complex>
#include <vector>

#include "state.h"

namespace lbcrypto {

namespace {

struct FFTTables {
    uint32_t n = 0;
    std::vector<uint64_t> rot;                  // 5^j mod 2n, j < n/2
    std::vector<std::complex<double>> ksi;      // exp(2 pi i k / 2n), k <= 2n
};

const FFTTables& tables(uint32_t n) {
    static std::mutex mu;
    static std::map<uint32_t, std::unique_ptr<FFTTables>> cache;
    std::lock_guard<std::mutex> g(mu);
    auto& t = cache[n];
    if (!t) {
        t.reset(new FFTTables);
        t->n = n;
        const uint64_t M = 2ull * n;
        t->rot.resize(n / 2);
        uint64_t g5 = 1;
        for (uint32_t j = 0; j < n / 2; ++j) {
            t->rot[j] = g5;
            g5 = (g5 * 5) % M;
        }
        t->ksi.resize(M + 1);
        for (uint64_t k = 0; k <= M; ++k) {
            double a = 2.0 * M_PI * (double)k / (double)M;
            t->ksi[k] = std::complex<double>(std::cos(a), std::sin(a));
        }
    }
    return *t;
}

void bitReverse(std::complex<double>* v, uint32_t size) {
    for (uint32_t i = 1, j = 0; i < size; ++i) {
        uint32_t bit = size >> 1;
        for (; j >= bit; bit >>= 1) j -= bit;
        j += bit;
        if (i < j) std::swap(v[i], v[j]);
    }
}

// slots -> coefficient pairs
void fftSpecialInv(std::complex<double>* v, uint32_t size, const FFTTables& t) {
    const uint64_t M = 2ull * t.n;
    for (uint32_t len = size; len >= 1; len >>= 1) {
        for (uint32_t i = 0; i < size; i += len) {
            uint32_t lenh = len >> 1;
            uint64_t lenq = (uint64_t)len << 2;
            const uint64_t step = M / lenq;  // lenq divides M: the divisions are masks and a product
            for (uint32_t j = 0; j < lenh; ++j) {
                uint64_t idx = (lenq - (t.rot[j] & (lenq - 1))) * step;
                std::complex<double> u = v[i + j] + v[i + j + lenh];
                std::complex<double> w = (v[i + j] - v[i + j + lenh]) * t.ksi[idx];
                v[i + j] = u;
                v[i + j + lenh] = w;
            }
        }
    }
    bitReverse(v, size);
    for (uint32_t i = 0; i < size; ++i) v[i] /= (double)size;
}

// coefficient pairs -> slots
void fftSpecial(std::complex<double>* v, uint32_t size, const FFTTables& t) {
    const uint64_t M = 2ull * t.n;
    bitReverse(v, size);
    // butterflies j0 <= j < j1 of every block of stage `len` in [lo, hi)
    auto stage = [&](uint32_t len, uint32_t lo, uint32_t hi, uint32_t j0, uint32_t j1) {
        const uint32_t lenh = len >> 1;
        const uint64_t lenq = (uint64_t)len << 2;
        const uint64_t step = M / lenq;  // as fftSpecialInv
        for (uint32_t i = lo; i < hi; i += len)
            for (uint32_t j = j0; j < j1; ++j) {
                uint64_t idx = (t.rot[j] & (lenq - 1)) * step;
                std::complex<double> u = v[i + j];
                std::complex<double> w = v[i + j + lenh] * t.ksi[idx];
                v[i + j] = u + w;
                v[i + j + lenh] = u - w;
            }
    };
    // Large decodes (the debug prints' 32 768-slot decryptions) on 16 host
    // threads: the stages inside blocks of size/16 run per block, the last
    // four stages split each block's butterflies.  Every butterfly computes
    // what the sequential loop computes, so the values are identical.
    const uint32_t T = size >= 8192 ? 16 : 1, B = size / T;
    if (T > 1) {
        ParallelFor(T, [&](size_t b) {
            for (uint32_t len = 2; len <= B; len <<= 1) stage(len, (uint32_t)b * B, (uint32_t)(b + 1) * B, 0, len >> 1);
        }, 1);
        for (uint32_t len = 2 * B; len <= size; len <<= 1) {
            const uint32_t lenh = len >> 1, part = lenh / T;
            ParallelFor(T, [&](size_t p) { stage(len, 0, size, (uint32_t)p * part, (uint32_t)(p + 1) * part); }, 1);
        }
        return;
    }
    for (uint32_t len = 2; len <= size; len <<= 1) stage(len, 0, size, 0, len >> 1);
}

}  // namespace

void ckks_encoder_tables(uint32_t n, const uint64_t** rot, const double** ksi) {
    const FFTTables& t = tables(n);
    *rot = t.rot.data();
    *ksi = reinterpret_cast<const double*>(t.ksi.data());  // (re, im) pairs: std::complex layout
}

int ckks_encode(const std::vector<std::complex<double>>& vals, uint32_t slots, uint32_t n,
                double scale, std::vector<int64_t>& coeffs) {
    const FFTTables& t = tables(n);
    std::vector<std::complex<double>> u(slots, 0.0);
    for (size_t i = 0; i < vals.size() && i < slots; ++i) u[i] = vals[i];
    fftSpecialInv(u.data(), slots, t);
    coeffs.assign(n, 0);
    const uint32_t gap = (n / 2) / slots;
    // Coefficients beyond 62 bits (large values at a large scale, e.g.
    // RotationTest's [0, 255) at scale 2^59): like OpenFHE's CKKS encoder,
    // encode value * scale / 2^shift and let the caller multiply every
    // residue by 2^shift (the low `shift` bits are below double precision
    // anyway: a double carries 53 significant bits).
    double mx = 0.0;
    for (uint32_t i = 0; i < slots; ++i)
        mx = std::max(mx, std::max(std::fabs(u[i].real()), std::fabs(u[i].imag())) * scale);
    if (!std::isfinite(mx)) SFHE_THROW("encoded value is not finite");
    int shift = 0;
    while (mx >= 4.0e18) {  // < 2^62 after the shift
        mx *= 0.5;
        ++shift;
    }
    if (shift > 60) SFHE_THROW("encoded value exceeds the supported range (|value * scale| >= 2^122)");
    const double sc = std::ldexp(scale, -shift);
    for (uint32_t i = 0; i < slots; ++i) {
        coeffs[(size_t)i * gap] = (int64_t)std::nearbyint(u[i].real() * sc);
        coeffs[(size_t)n / 2 + (size_t)i * gap] = (int64_t)std::nearbyint(u[i].imag() * sc);
    }
    return shift;
}

void ckks_decode(const std::vector<double>& c, uint32_t slots, uint32_t n,
                 std::vector<std::complex<double>>& out) {
    const FFTTables& t = tables(n);
    const uint32_t gap = (n / 2) / slots;
    out.assign(slots, 0.0);
    for (uint32_t i = 0; i < slots; ++i)
        out[i] = std::complex<double>(c[(size_t)i * gap], c[(size_t)n / 2 + (size_t)i * gap]);
    fftSpecial(out.data(), slots, t);
}

}  // namespace lbcrypto
