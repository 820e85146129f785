// Bootstrapping precision probe (developer tool, not a test): where the error
// of one EvalBootstrap comes from (core/bootstrap.cpp steps 1-7).
//
//   boot_probe logn S b0 b1 [seed]
//
// The engine's stage tap (SetBootstrapTap) hands over every stage's
// ciphertext and, for the linear stages, the slot map it applied.  Each tap
// is decrypted; the noise a stage ADDS is its decryption minus the stage's
// exact function (in double) of the previous stage's decryption, and that
// noise is carried to the output through the remaining stages' exact
// functions.  The chain from the traced (ModRaised) input is also replayed
// exactly three ways -- EvalMod as the true modular reduction 2 pi frac(x),
// as sin(2 pi x), and as the engine's polynomial (Chebyshev series + double
// angles) -- which separates the sine's nonlinearity and the polynomial's
// approximation error from the CKKS noise.  (Decrypting a tap settles a
// lazily rescaled ciphertext, so the tapped run's noise is that of the
// settled form.)
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "openfhe.h"

using namespace lbcrypto;
using cd = std::complex<double>;
using CV = std::vector<cd>;
using SlotMap = CryptoContextImpl<DCRTPoly>::BootstrapSlotMap;

namespace {

struct Tap {
    std::string stage;
    CV v;
    SlotMap map;
    bool linear = false;
    uint32_t level = 0;
};

CV applyMap(const SlotMap& m, const CV& in) {
    const size_t S = in.size();
    CV out(S, 0.0);
    for (const auto& [k, d] : m)
        for (size_t p = 0; p < S; ++p) out[p] += d[p] * in[(p + k) % S];
    return out;
}

double log2max(const std::vector<double>& e) {
    double m = 0;
    for (double x : e) m = std::max(m, std::fabs(x));
    return m > 0 ? std::log2(m) : -1e9;
}
double log2rms(const std::vector<double>& e) {
    double s = 0;
    for (double x : e) s += x * x;
    s = std::sqrt(s / (double)e.size());
    return s > 0 ? std::log2(s) : -1e9;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: boot_probe logn S b0 b1 [seed]\n");
        return 2;
    }
    const uint32_t logn = std::atoi(argv[1]), S = std::atoi(argv[2]);
    const uint32_t b0 = std::atoi(argv[3]), b1 = std::atoi(argv[4]);
    const uint64_t seed = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 1;
    // the k-way configuration (kway_adapter.h:41-64): scale 2^59, first modulus 60 bits
    CCParams<CryptoContextCKKSRNS> p;
    p.SetRingDim(1u << logn);
    p.SetBatchSize(S);
    p.SetScalingModSize(59);
    p.SetFirstModSize(60);
    p.SetSecurityLevel(HEStd_NotSet);
    {  // depth: the bootstrap's levels + 3 levels used before it (tests/test_bootstrap.py)
        auto tmp = GenCryptoContext([&] {
            auto q = p;
            q.SetMultiplicativeDepth(30);
            return q;
        }());
        p.SetMultiplicativeDepth(tmp->GetBootstrapDepth({b0, b1}, S) + 3);
    }
    auto cc = GenCryptoContext(p);
    cc->Enable(PKE);
    cc->Enable(KEYSWITCH);
    cc->Enable(LEVELEDSHE);
    cc->Enable(ADVANCEDSHE);
    cc->Enable(FHE);
    cc->EvalBootstrapSetup({b0, b1}, {0, 0}, S);
    auto kp = cc->KeyGen();
    cc->EvalMultKeyGen(kp.secretKey);
    cc->EvalBootstrapKeyGen(kp.secretKey, S);
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<double> x(S);
    for (auto& v : x) v = U(rng);
    auto ct = cc->Encrypt(kp.publicKey, cc->MakeCKKSPackedPlaintext(x, 1, 0, nullptr, S));
    for (int i = 0; i < 3; ++i) ct = cc->EvalMult(ct, 1.0);

    std::vector<Tap> taps;
    cc->SetBootstrapTap([&](const char* stage, const Ciphertext<DCRTPoly>& c, const SlotMap* m) {
        Plaintext pt;
        cc->Decrypt(kp.secretKey, c, &pt);
        Tap t;
        t.stage = stage;
        t.v = pt->GetCKKSPackedValue();
        t.v.resize(S);
        t.level = c->GetLevel();
        if (m) {
            t.map = *m;
            t.linear = true;
        }
        taps.push_back(std::move(t));
    });
    auto out = cc->EvalBootstrap(ct);
    cc->SetBootstrapTap(nullptr);
    Plaintext pout;
    cc->Decrypt(kp.secretKey, out, &pout);
    std::vector<double> got(S);
    for (uint32_t i = 0; i < S; ++i) got[i] = pout->GetCKKSPackedValue()[i].real();

    // the stage list: traced, c2s..., yre, yim, wre, wim, s2c...
    size_t it = 0;
    while (it < taps.size() && taps[it].stage != "traced") ++it;
    if (it == taps.size()) {
        std::fprintf(stderr, "no traced tap\n");
        return 1;
    }
    const CV traced = taps[it].v;
    std::vector<const Tap*> c2s, s2c;
    const Tap *yre = nullptr, *yim = nullptr, *wre = nullptr, *wim = nullptr;
    for (size_t i = it + 1; i < taps.size(); ++i) {
        const Tap& t = taps[i];
        if (t.stage == "c2s") c2s.push_back(&t);
        else if (t.stage == "s2c") s2c.push_back(&t);
        else if (t.stage == "yre") yre = &t;
        else if (t.stage == "yim") yim = &t;
        else if (t.stage == "wre") wre = &t;
        else if (t.stage == "wim") wim = &t;
    }
    if (!yre || !yim || !wre || !wim || c2s.empty() || s2c.empty()) {
        std::fprintf(stderr, "missing taps\n");
        return 1;
    }
    const double Kb = CryptoContextImpl<DCRTPoly>::BootstrapOverflowBound();
    const uint32_t R = CryptoContextImpl<DCRTPoly>::BootstrapDoubleAngles();
    const auto cheb = EvalChebyshevCoefficients(
        [&](double v) { return std::cos(2.0 * M_PI * (v - 0.25) / (double)(1u << R)); }, -Kb, Kb,
        CryptoContextImpl<DCRTPoly>::BootstrapChebDegree() + 1);
    // EvalMod variants on y = x / Kb, over complex y: the slots' imaginary
    // noise goes through the polynomial too (P(y + i e) ~ P(y) + i e P'(y))
    enum Mod { kTrueMod, kSin, kPoly };
    auto evalMod = [&](cd y, Mod m) -> cd {
        const cd xx = y * Kb;
        if (m == kTrueMod) return 2.0 * M_PI * (xx.real() - std::nearbyint(xx.real()));
        if (m == kSin) return std::sin(2.0 * M_PI * xx);
        // Chebyshev series on [-1, 1] (Clenshaw; c_0 halved, OpenFHE's convention)
        cd b1c = 0, b2c = 0;
        for (size_t k = cheb.size(); k-- > 1;) {
            const cd t = 2.0 * y * b1c - b2c + cheb[k];
            b2c = b1c;
            b1c = t;
        }
        cd c = y * b1c - b2c + 0.5 * cheb[0];
        for (uint32_t i = 0; i < R; ++i) c = 2.0 * c * c - 1.0;
        return c;
    };
    auto realOnly = [&](const CV& v) {
        CV r(S);
        for (uint32_t i = 0; i < S; ++i) r[i] = v[i].real();
        return r;
    };
    // continuations to the (real) output
    auto fromW = [&](const CV& wr, const CV& wi, size_t s2cFrom) {
        CV v(S);
        for (uint32_t i = 0; i < S; ++i) v[i] = wr[i] + cd(0.0, 1.0) * wi[i];
        for (size_t g = s2cFrom; g < s2c.size(); ++g) v = applyMap(s2c[g]->map, v);
        std::vector<double> r(S);
        for (uint32_t i = 0; i < S; ++i) r[i] = v[i].real();
        return r;
    };
    auto fromY = [&](const CV& yr, const CV& yi, Mod m) {
        CV wr(S), wi(S);
        for (uint32_t i = 0; i < S; ++i) {
            wr[i] = evalMod(yr[i], m);
            wi[i] = evalMod(yi[i], m);
        }
        return fromW(wr, wi, 0);
    };
    // re = h + conj(h), i im = h - conj(h); yre = re / Kb, yim = i im (-i / Kb)
    // (slot-wise conjugation: exact for the noise-free h, and what the
    // ciphertexts compute for a noisy one)
    auto yOf = [&](const CV& h, CV& yr, CV& yi) {
        yr.assign(S, 0.0);
        yi.assign(S, 0.0);
        for (uint32_t i = 0; i < S; ++i) {
            yr[i] = (h[i] + std::conj(h[i])) / Kb;
            yi[i] = (h[i] - std::conj(h[i])) * cd(0.0, -1.0 / Kb);
        }
    };
    auto fromC2S = [&](CV h, size_t from, Mod m) {
        for (size_t g = from; g < c2s.size(); ++g) h = applyMap(c2s[g]->map, h);
        CV yr, yi;
        yOf(h, yr, yi);
        return fromY(yr, yi, m);
    };
    auto diff = [&](const std::vector<double>& a, const std::vector<double>& b) {
        std::vector<double> d(S);
        for (uint32_t i = 0; i < S; ++i) d[i] = a[i] - b[i];
        return d;
    };
    auto line = [&](const char* what, const std::vector<double>& e) {
        std::printf("  %-52s max 2^%6.1f  rms 2^%6.1f\n", what, log2max(e), log2rms(e));
    };
    std::printf("boot_probe: ring 2^%u, S = %u, level budget {%u, %u}, scale 2^59, K + 1 = %.0f, "
                "Chebyshev degree %u + %u double angles\n",
                logn, S, b0, b1, Kb, CryptoContextImpl<DCRTPoly>::BootstrapChebDegree(), R);
    std::vector<double> xv(x.begin(), x.end());
    line("TOTAL: output - input", diff(got, xv));
    std::printf(" exact replays from the traced (ModRaised) input:\n");
    const auto outMod = fromC2S(traced, 0, kTrueMod);
    const auto outSin = fromC2S(traced, 0, kSin);
    const auto outPoly = fromC2S(traced, 0, kPoly);
    line("input side (adjust / raise / trace): mod - x", diff(outMod, xv));
    line("EvalMod nonlinearity: sin - mod", diff(outSin, outMod));
    line("EvalMod polynomial: poly - sin", diff(outPoly, outSin));
    std::printf(" CKKS noise added by each stage, carried to the output through the exact\n"
                " remaining stages (EvalMod as its polynomial, over complex slots):\n");
    CV prev = traced;
    for (size_t g = 0; g < c2s.size(); ++g) {
        const CV pred = applyMap(c2s[g]->map, prev);
        char nm[64];
        std::snprintf(nm, sizeof nm, "CoeffsToSlots group %zu", g);
        line(nm, diff(fromC2S(c2s[g]->v, g + 1, kPoly), fromC2S(pred, g + 1, kPoly)));
        prev = c2s[g]->v;
    }
    {
        CV yr, yi;
        yOf(prev, yr, yi);
        line("conjugation split + 1/(K+1)", diff(fromY(yre->v, yim->v, kPoly), fromY(yr, yi, kPoly)));
        // how much of the y stages' noise is imaginary (removed by taking real parts)
        line("  of which the imaginary parts of y",
             diff(fromY(yre->v, yim->v, kPoly), fromY(realOnly(yre->v), realOnly(yim->v), kPoly)));
    }
    {
        CV pr(S), pi(S);
        for (uint32_t i = 0; i < S; ++i) {
            pr[i] = evalMod(yre->v[i], kPoly);
            pi[i] = evalMod(yim->v[i], kPoly);
        }
        line("EvalMod evaluation (vs its polynomial)", diff(fromW(wre->v, wim->v, 0), fromW(pr, pi, 0)));
        line("  of which the imaginary parts of w",
             diff(fromW(wre->v, wim->v, 0), fromW(realOnly(wre->v), realOnly(wim->v), 0)));
    }
    {
        CV v(S);
        for (uint32_t i = 0; i < S; ++i) v[i] = wre->v[i] + cd(0.0, 1.0) * wim->v[i];
        for (size_t g = 0; g < s2c.size(); ++g) {
            const CV pred = applyMap(s2c[g]->map, v);
            CV a = s2c[g]->v, b = pred;
            for (size_t h = g + 1; h < s2c.size(); ++h) {
                a = applyMap(s2c[h]->map, a);
                b = applyMap(s2c[h]->map, b);
            }
            std::vector<double> e(S);
            for (uint32_t i = 0; i < S; ++i) e[i] = a[i].real() - b[i].real();
            char nm[64];
            std::snprintf(nm, sizeof nm, "SlotsToCoeffs group %zu", g);
            line(nm, e);
            v = s2c[g]->v;
        }
    }
    // the EvalMod input range actually seen (|frac(x)| drives the nonlinearity)
    double fmax = 0;
    for (uint32_t i = 0; i < S; ++i)
        for (double y : {yre->v[i].real(), yim->v[i].real()}) {
            const double xx = y * Kb;  // (real parts)
            fmax = std::max(fmax, std::fabs(xx - std::nearbyint(xx)));
        }
    std::printf(" max |frac(x)| at EvalMod's input: 2^%.1f\n", std::log2(fmax));
    {  // EvalMod's own noise in w units: the bootstrap's run, then the same
       // evaluation on a fresh encryption of yre's values at yre's level
        auto absLine = [&](const char* what, const CV& a, const std::vector<cd>& b) {
            double mx = 0;
            for (uint32_t i = 0; i < S; ++i) mx = std::max(mx, std::abs(a[i] - b[i]));
            std::printf("  %-52s max 2^%6.1f\n", what, std::log2(mx));
        };
        std::printf(" EvalMod noise at its output (w units, |w| <= 1):\n");
        CV pr(S);
        for (uint32_t i = 0; i < S; ++i) pr[i] = evalMod(yre->v[i], kPoly);
        absLine("in the bootstrap (wre vs P(yre))", wre->v, pr);
        std::vector<double> yv(S);
        for (uint32_t i = 0; i < S; ++i) yv[i] = yre->v[i].real();
        auto c = cc->Encrypt(kp.publicKey, cc->MakeCKKSPackedPlaintext(yv, 1, yre->level, nullptr, S));
        c = cc->EvalChebyshevSeriesPS(c, cheb, -1.0, 1.0);
        std::vector<cd> ser(S);
        for (uint32_t i = 0; i < S; ++i) {  // the series alone (before the double angles)
            double b1c = 0, b2c = 0;
            for (size_t k = cheb.size(); k-- > 1;) {
                const double t = 2.0 * yv[i] * b1c - b2c + cheb[k];
                b2c = b1c;
                b1c = t;
            }
            ser[i] = yv[i] * b1c - b2c + 0.5 * cheb[0];
        }
        auto dec = [&](const Ciphertext<DCRTPoly>& ct) {
            Plaintext pt;
            cc->Decrypt(kp.secretKey, ct, &pt);
            CV v = pt->GetCKKSPackedValue();
            v.resize(S);
            return v;
        };
        char nm[80];
        std::snprintf(nm, sizeof nm, "fresh input: Chebyshev PS (degree %u, level %u -> %u)",
                      CryptoContextImpl<DCRTPoly>::BootstrapChebDegree(), yre->level, c->GetLevel());
        absLine(nm, dec(c), ser);
        for (uint32_t r = 0; r < R; ++r) {
            c = cc->EvalAdd(cc->EvalMult(cc->EvalAdd(c, c), c), -1.0);
            for (auto& v : ser) v = 2.0 * v * v - 1.0;
            std::snprintf(nm, sizeof nm, "fresh input: + double angle %u", r + 1);
            absLine(nm, dec(c), ser);
        }
    }
    return 0;
}
