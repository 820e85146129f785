// Precision probe (developer tool, not a test): per-stage CKKS error of
// sort_hybrid1 / DirectSort::sort against the exact slot values, and the
// noise each stage ADDS (decrypted output minus the stage's exact slot
// function applied to the decrypted input).
//
//   prec_probe h1 N logn [secure] [seed]     hybrid1 (reference sort_algo.h:1067-1229), with taps
//   prec_probe ds N logn [secure] [seed]     DirectSort (sort_algo.h:752-774), rank + placement
//   prec_probe h|h2 N logn [secure] [seed]   sort_hybrid / sort_hybrid2 (:894-1062, :1233-1389)
//   prec_probe h1x N logn [secure] [seed]    sort_hybrid1 without taps (decrypting a tap settles
//                                            a lazily rescaled ciphertext, so taps change the noise)
//   prec_probe h2s N logn [secure] [seed]    hybrid II's scaled-sinc stage: input noise vs the
//                                            noise the series adds, binned by |x|
//   prec_probe sinc N logn [0] [seed]        SincTest's encrypted doubled-sinc series alone
//
// Engine knobs under test are read from the environment by the library.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "sort_algo.h"

namespace {

using Vec = std::vector<double>;

struct Probe {
    CryptoContext<DCRTPoly> cc;
    PrivateKey<DCRTPoly> sk;
    Vec dec(const Ciphertext<DCRTPoly>& ct) {
        Plaintext pt;
        cc->Decrypt(sk, ct, &pt);
        Vec v = pt->GetRealPackedValue();
        v.resize(ct->GetSlots());
        return v;
    }
    // err of d against e on the slots where pick(s) holds
    template <class F>
    static void stat(const Vec& d, const Vec& e, F pick, double& mx, double& rms) {
        mx = 0;
        double s2 = 0;
        size_t k = 0;
        for (size_t i = 0; i < d.size(); ++i) {
            if (!pick(i)) continue;
            double x = std::fabs(d[i] - e[i % e.size()]);
            mx = std::max(mx, x);
            s2 += x * x;
            ++k;
        }
        rms = k ? std::sqrt(s2 / k) : 0;
    }
    void report(const char* what, const Ciphertext<DCRTPoly>& ct, const Vec& d, const Vec& exact, const Vec* local) {
        auto all = [](size_t) { return true; };
        double m1, r1, m2 = 0, r2 = 0;
        stat(d, exact, all, m1, r1);
        if (local) stat(d, *local, all, m2, r2);
        std::printf("%-34s L%-3u slots %-6zu  vs exact max %.3e rms %.3e (log2 %6.2f)", what, ct->GetLevel(), d.size(),
                    m1, r1, std::log2(std::max(m1, 1e-300)));
        if (local) std::printf("  | added: max %.3e rms %.3e", m2, r2);
        std::printf("\n");
        std::fflush(stdout);
    }
};

Vec rotL(const Vec& v, long r) {
    const long n = (long)v.size();
    Vec o(v.size());
    long s = ((r % n) + n) % n;
    for (long i = 0; i < n; ++i) o[i] = v[(i + s) % n];
    return o;
}
Vec tile(const Vec& v, size_t S) {
    Vec o(S);
    for (size_t i = 0; i < S; ++i) o[i] = v[i % v.size()];
    return o;
}
double odd7(const double* c, double x) {
    double x2 = x * x;
    return x * (c[0] + x2 * (c[1] + x2 * (c[2] + x2 * c[3])));
}
const double G3[4] = {4589.0 / 1024, -16577.0 / 1024, 25614.0 / 1024, -12860.0 / 1024};
const double F3[4] = {35.0 / 16, -35.0 / 16, 21.0 / 16, -5.0 / 16};
double signAdvExact(double x, int dg, int df) {
    for (int i = 0; i < dg; ++i) x = odd7(G3, x);
    for (int i = 0; i + 1 < df; ++i) x = odd7(F3, x);
    return 0.5 + 0.5 * odd7(F3, x);
}
Vec mapv(const Vec& v, double (*f)(double, int, int), int a, int b) {
    Vec o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = f(v[i], a, b);
    return o;
}

std::vector<double> inputVector(int N, unsigned seed) {
    std::vector<int> p(N);
    std::iota(p.begin(), p.end(), 0);
    std::shuffle(p.begin(), p.end(), std::mt19937(seed));
    std::vector<double> x(N);
    for (int i = 0; i < N; ++i) x[i] = p[i] / (double)N;
    return x;
}

// f = c0/2 + sum_k c_k T_k(x) (the Chebyshev-series convention of EvalChebyshevSeriesPS), Clenshaw
double chebEval(const std::vector<double>& c, double x) {
    long double b1 = 0, b2 = 0;
    for (size_t k = c.size() - 1; k >= 1; --k) {
        long double b0 = c[k] + 2.0L * x * b1 - b2;
        b2 = b1;
        b1 = b0;
    }
    return (double)(c[0] / 2.0L + x * b1 - b2);
}

// hybrid II's series stage for batch 0, rotation 0 (reference sort_algo.h:1249-1308):
// d = i/N - rank_j/N on the N x N matrix, then the scaled-sinc series.  Its
// error splits into what the input noise explains (p(decrypted d) - p(exact d))
// and what the series adds (decrypted output - p(decrypted d)); the same series
// on a fresh encryption of the exact d at the same level isolates the series'
// own noise from the rank's.
template <int N>
int seriesStage(Probe& P, CryptoContext<DCRTPoly>& cc, KeyPair<DCRTPoly>& kp, DirectSort<N>& ds,
                std::shared_ptr<Encryption>& enc, Ciphertext<DCRTPoly> rank, Ciphertext<DCRTPoly> ct,
                const Vec& rankExact, const Vec& sorted) {
    const size_t S = (size_t)N * N;
    const auto& co = selectCoefficients<N>();
    std::printf("    series degree %zu\n", co.size() - 1);
    auto rk = rank->Clone();
    rk->SetSlots((uint32_t)S);
    auto r = cc->EvalMult(rk, 1.0 / N);
    Vec sub(S), dE(S);
    for (size_t i = 0; i < (size_t)N; ++i)
        for (size_t j = 0; j < (size_t)N; ++j) sub[i * N + j] = (double)i / N;
    for (size_t s = 0; s < S; ++s) dE[s] = sub[s] - rankExact[s % N] / N;
    auto d = cc->EvalSub(cc->MakeCKKSPackedPlaintext(sub, 1, r->GetLevel(), nullptr, (uint32_t)S), r);
    Vec dD = P.dec(d);
    P.report("d = i/N - rank/N", d, dD, dE, nullptr);
    auto series = [&](const Ciphertext<DCRTPoly>& in, const Vec& inD, const char* name) {
        auto o = cc->EvalChebyshevSeriesPS(in, co, -1, 1);
        Vec oE(S), oL(S);
        for (size_t s = 0; s < S; ++s) {
            oE[s] = chebEval(co, dE[s]);
            oL[s] = chebEval(co, inD[s]);
        }
        Vec oD = P.dec(o);
        P.report(name, o, oD, oE, &oL);
        const double edges[] = {0.0, 0.25, 0.5, 0.75, 0.9, 0.97, 1.01};
        for (int bI = 0; bI + 1 < 7; ++bI) {
            double mAdd = 0, mIn = 0;
            for (size_t s = 0; s < S; ++s) {
                const double a = std::fabs(dE[s]);
                if (a < edges[bI] || a >= edges[bI + 1]) continue;
                mAdd = std::max(mAdd, std::fabs(oD[s] - oL[s]));
                mIn = std::max(mIn, std::fabs(oL[s] - oE[s]));
            }
            std::printf("      |x| in [%.2f, %.2f): added max %.3e   input-explained max %.3e\n", edges[bI],
                        edges[bI + 1], mAdd, mIn);
        }
    };
    series(d, dD, "sinc series on d");
    auto fresh = cc->Encrypt(kp.publicKey, cc->MakeCKKSPackedPlaintext(dE, 1, d->GetLevel(), nullptr, (uint32_t)S));
    series(fresh, P.dec(fresh), "sinc series on fresh exact d");
    auto out = ds.rotationIndexCheckHybrid2(rank, ct, kp.secretKey);
    Vec oD = P.dec(out);
    oD.resize(N);
    P.report("rotationIndexCheckHybrid2", out, oD, sorted, nullptr);
    return 0;
}

template <int N>
int run(const std::string& mode, int logn, bool secure, unsigned seed) {
    CCParams<CryptoContextCKKSRNS> params;
    std::vector<int> rots;
    uint32_t depth;
    if (mode == "h1" || mode == "h1x" || mode == "h" || mode == "h2" || mode == "h2s") {
        const sfhe::SizeParams* hp = mode == "h" ? sfhe::hybridParams(N, 0)
                                     : (mode == "h2" || mode == "h2s") ? sfhe::hybridParams(N, 2)
                                                                       : sfhe::hybrid1Params(N);
        depth = hp->multDepth;
        rots = hp->rotations;
        params.SetBatchSize(N);
        params.SetScalingModSize(40);
    } else {
        DirectSort<N>::getSizeParameters(params, rots);
        depth = params.GetMultiplicativeDepth();
    }
    params.SetMultiplicativeDepth(depth);
    params.SetRingDim(1u << logn);
    params.SetSecurityLevel(secure ? HEStd_128_classic : HEStd_NotSet);
    if (const char* d = std::getenv("PROBE_DNUM")) params.SetNumLargeDigits((uint32_t)std::atoi(d));
    if (const char* d = std::getenv("PROBE_SCALE")) params.SetScalingModSize((uint32_t)std::atoi(d));
    params.SetSeed(seed);
    auto cc = GenCryptoContext(params);
    cc->Enable(PKE);
    cc->Enable(KEYSWITCH);
    cc->Enable(LEVELEDSHE);
    cc->Enable(ADVANCEDSHE);
    auto kp = cc->KeyGen();
    cc->EvalMultKeyGen(kp.secretKey);
    cc->EvalRotateKeyGen(kp.secretKey, rots);
    Probe P{cc, kp.secretKey};
    auto enc = std::make_shared<Encryption>(cc, kp.publicKey);
    DirectSort<N> ds(cc, kp.publicKey, rots, enc);
    std::printf("== %s N=%d ring 2^%d depth %u secure %d seed %u\n", mode.c_str(), N, logn, depth, secure, seed);

    Vec x = inputVector(N, seed);
    Vec rankExact(N);
    {
        std::vector<int> idx(N);
        std::iota(idx.begin(), idx.end(), 0);
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return x[a] < x[b]; });
        for (int r = 0; r < N; ++r) rankExact[idx[r]] = r;
    }
    Vec sorted = x;
    std::sort(sorted.begin(), sorted.end());
    auto ct = enc->encryptInput(x);
    P.report("input", ct, P.dec(ct), x, nullptr);

    SignConfig cfg(CompositeSignConfig(3, N <= 16 ? 2 : N <= 128 ? 3 : N <= 512 ? 4 : 5, 2));
    if (mode == "h1x" || mode == "h" || mode == "h2") {
        for (int t = 0; t < 2; ++t) {
            auto c2 = enc->encryptInput(x);
            auto o = mode == "h" ? ds.sort_hybrid(c2, SignFunc::CompositeSign, cfg, kp.secretKey)
                     : mode == "h2" ? ds.sort_hybrid2(c2, SignFunc::CompositeSign, cfg, kp.secretKey)
                                    : ds.sort_hybrid1(c2, SignFunc::CompositeSign, cfg, kp.secretKey);
            Vec d = P.dec(o);
            d.resize(N);
            P.report(mode == "h" ? "sort_hybrid" : mode == "h2" ? "sort_hybrid2" : "sort_hybrid1", o, d, sorted,
                     nullptr);
            if (o->GetLevel() != depth) std::printf("    LEVEL MISMATCH: %u vs depth %u\n", o->GetLevel(), depth);
        }
        return 0;
    }
    Ciphertext<DCRTPoly> rank;
    if (std::getenv("PROBE_EXACT_RANK")) {  // isolate placement noise: a fresh encryption of the exact ranks
        auto r0 = ds.constructRank(ct, SignFunc::CompositeSign, cfg);
        auto pt = cc->MakeCKKSPackedPlaintext(rankExact, 1, r0->GetLevel(), nullptr, N);
        rank = cc->Encrypt(kp.publicKey, pt);
    } else {
        rank = ds.constructRank(ct, SignFunc::CompositeSign, cfg);
    }
    Vec rankD = P.dec(rank);
    P.report("rank", rank, rankD, rankExact, nullptr);

    if (mode == "ds") {
        // constructRank's stages for batch 0 (reference sort_algo.h:368-506):
        // the shifted copy vecRotsOpt builds and the comparison of it
        const sfhe::RankLayout L(N, (int)cc->GetRingDimension() / 2);
        RotationComposer<N> rc(cc, enc, rots);
        std::vector<int> am(L.npRank);
        std::iota(am.begin(), am.end(), 0);
        auto pre = rc.rotateMany(ct, am);
        for (auto& p : pre) p->SetSlots(L.S);
        Vec xS = tile(x, L.S);
        for (int b = 0; b < std::min(L.B, 2); ++b) {
            auto shifted = ds.vecRotsOpt(pre, L.P, L.S, L.npRank, b);
            Vec shE(L.S);
            for (int s = 0; s < L.S; ++s) shE[s] = x[(s % N + b * L.P + s / N) % N];
            Vec shD = P.dec(shifted);
            P.report(b ? "vecRotsOpt shifted (batch 1)" : "vecRotsOpt shifted (batch 0)", shifted, shD, shE, nullptr);
            auto dup = ct->Clone();
            dup->SetSlots(L.S);
            Comparison comp(enc);
            auto cmpo = comp.compare(cc, dup, shifted, SignFunc::CompositeSign, cfg);
            Vec cE(L.S), cL(L.S);
            for (int s = 0; s < L.S; ++s) {
                const double dexact = xS[s] - shE[s], dloc = xS[s] - shD[s];
                auto stepf = [&](double dd) {
                    double y = dd;
                    for (int i = 0; i < std::max(cfg.compos.dg, 1); ++i) y = odd7(G3, y);
                    for (int i = 0; i < cfg.compos.df; ++i) y = odd7(F3, y);
                    return (y + 1) / 2;
                };
                cE[s] = stepf(dexact);
                cL[s] = stepf(dloc);
            }
            P.report("compare(dup, shifted)", cmpo, P.dec(cmpo), cE, &cL);
        }
        auto out = ds.rotationIndexCheckN(rank, ct);
        P.report("sort (placement)", out, P.dec(out), sorted, nullptr);
        return 0;
    }

    if (mode == "h2s") return seriesStage<N>(P, cc, kp, ds, enc, rank, ct, rankExact, sorted);

    // ---- rotationIndexCheckHybrid1 with taps (N <= 256: one batch, M = N) ----
    const size_t M = N, S = (size_t)N * N;
    rank->SetSlots((uint32_t)S);
    ct->SetSlots((uint32_t)S);
    const uint32_t dg = (uint32_t)((std::log2((double)N) + 1) / 2), df = 2;
    Vec sub(S);
    for (size_t i = 0; i < M; ++i)
        for (size_t j = 0; j < M; ++j) sub[i * M + j] = (double)i;
    auto subPt = cc->MakeCKKSPackedPlaintext(sub, 1, rank->GetLevel(), nullptr, (uint32_t)S);
    auto rm = cc->EvalSub(subPt, rank);
    Vec rmExact(S), rmLocal(S);
    for (size_t s = 0; s < S; ++s) {
        rmExact[s] = sub[s] - rankExact[s % N];
        rmLocal[s] = sub[s] - rankD[s % N];
    }
    Vec rmD = P.dec(rm);
    P.report("subMask - rank", rm, rmD, rmExact, &rmLocal);

    // indicatorAdv(c, N, dg, 2) with taps
    auto tmp = cc->EvalMult(rm, 1.0 / N);
    auto c1 = cc->EvalAdd(tmp, 0.5 / N);
    auto c2 = cc->EvalSub(tmp, 0.5 / N);
    Vec c1E(S), c2E(S), c1L(S);
    for (size_t s = 0; s < S; ++s) {
        c1E[s] = rmExact[s] / N + 0.5 / N;
        c2E[s] = rmExact[s] / N - 0.5 / N;
        c1L[s] = rmD[s] / N + 0.5 / N;
    }
    Vec c1D = P.dec(c1);
    P.report("c1 = c/N + 1/2N", c1, c1D, c1E, &c1L);
    static const std::vector<double> g3 = {0, G3[0], 0, G3[1], 0, G3[2], 0, G3[3]};
    static const std::vector<double> f3 = {0, F3[0], 0, F3[1], 0, F3[2], 0, F3[3]};
    static const std::vector<double> f3F = {0.5, F3[0] / 2, 0, F3[1] / 2, 0, F3[2] / 2, 0, F3[3] / 2};
    auto stage = [&](Ciphertext<DCRTPoly> c, Vec& exact, Vec dIn, const std::vector<double>& p, bool tap,
                     const char* name) {
        auto o = cc->EvalPolyLinear(c, p);
        auto f = [&](double v) {
            double r = p[0], pw = 1;
            for (size_t k = 1; k < p.size(); ++k) {
                pw *= v;
                r += p[k] * pw;
            }
            return r;
        };
        Vec loc(dIn.size());
        for (size_t s = 0; s < exact.size(); ++s) exact[s] = f(exact[s]);
        for (size_t s = 0; s < dIn.size(); ++s) loc[s] = f(dIn[s]);
        Vec d = P.dec(o);
        if (tap) P.report(name, o, d, exact, &loc);
        return std::make_pair(o, d);
    };
    auto signTap = [&](Ciphertext<DCRTPoly> c, Vec exact, Vec dIn, bool tap, const char* tag) {
        char nm[64];
        for (uint32_t i = 0; i < dg; ++i) {
            std::snprintf(nm, sizeof nm, "%s g3 #%u", tag, i + 1);
            auto r = stage(c, exact, dIn, g3, tap, nm);
            c = r.first;
            dIn = r.second;
        }
        for (uint32_t i = 0; i + 1 < df; ++i) {
            std::snprintf(nm, sizeof nm, "%s f3 #%u", tag, i + 1);
            auto r = stage(c, exact, dIn, f3, tap, nm);
            c = r.first;
            dIn = r.second;
        }
        std::snprintf(nm, sizeof nm, "%s f3final", tag);
        auto r = stage(c, exact, dIn, f3F, tap, nm);
        return std::make_tuple(r.first, exact, r.second);
    };
    auto [s1, s1E, s1D] = signTap(c1, c1E, c1D, true, "sign(c1)");
    Vec c2D = P.dec(c2);
    auto [s2, s2E, s2D] = signTap(c2, c2E, c2D, false, "sign(c2)");
    auto one = cc->EvalSub(1.0, s2);
    auto ind = cc->EvalMult(s1, one);
    Vec indE(S), indL(S);
    for (size_t s = 0; s < S; ++s) {
        indE[s] = s1E[s] * (1 - s2E[s]);
        indL[s] = s1D[s] * (1 - s2D[s]);
    }
    Vec indD = P.dec(ind);
    P.report("indicator", ind, indD, indE, &indL);
    // entries that should be 1 vs 0
    {
        double m1 = 0, m0 = 0;
        for (size_t s = 0; s < S; ++s) {
            double e = std::fabs(indD[s] - (rmExact[s] == 0 ? 1.0 : 0.0));
            (rmExact[s] == 0 ? m1 : m0) = std::max(rmExact[s] == 0 ? m1 : m0, e);
        }
        std::printf("    indicator vs 0/1: max err on hits %.3e, off hits %.3e\n", m1, m0);
    }
    auto z = ds.getZero()->Clone();
    z->SetSlots((uint32_t)S);
    auto prod = cc->EvalMult(ct, ind);
    Vec xs = tile(x, S), prodE(S), prodL(S);
    Vec xsD = P.dec(ct);
    for (size_t s = 0; s < S; ++s) {
        prodE[s] = xs[s] * indE[s];
        prodL[s] = xsD[s % xsD.size()] * indD[s];
    }
    Vec prodD = P.dec(prod);
    P.report("x * indicator", prod, prodD, prodE, &prodL);
    auto acc = cc->EvalAdd(z, prod);
    Vec accD = P.dec(acc);
    P.report("zero + product", acc, accD, prodE, &prodD);
    // sumColumnsToTarget(acc, M, 0, mask) without and with the mask
    auto sumEx = [&](Vec v) {
        size_t step = M >> 1;
        for (size_t i = 0; i < (size_t)std::log2((double)M); ++i, step >>= 1) {
            Vec r = rotL(v, (long)step);
            for (size_t s = 0; s < v.size(); ++s) v[s] += r[s];
        }
        return v;
    };
    auto sc = ds.sumColumnsToTarget(acc, M, 0, false);
    Vec scE = sumEx(prodE), scL = sumEx(accD), scD = P.dec(sc);
    P.report("sumColumns (rotations only)", sc, scD, scE, &scL);
    auto colMask = [&](Vec v) {
        for (size_t s = 0; s < v.size(); ++s)
            if (s % M != 0) v[s] = 0;
        return v;
    };
    std::vector<double> cm(S, 0.0);
    for (size_t i = 0; i < M; ++i) cm[M * i] = 1.0;
    auto sm = cc->EvalMult(sc, cc->MakeCKKSPackedPlaintext(cm, 1, sc->GetLevel(), nullptr, (uint32_t)S));
    Vec smE = colMask(scE), smL = colMask(scD), smD = P.dec(sm);
    P.report("sumColumns masked", sm, smD, smE, &smL);
    auto trEx = [&](Vec v) {
        size_t step = M * (M - 1) / 2;
        for (size_t i = 0; i < (size_t)std::log2((double)M); ++i, step >>= 1) {
            Vec r = rotL(v, (long)step);
            for (size_t s = 0; s < v.size(); ++s) v[s] += r[s];
        }
        return v;
    };
    auto tr = ds.transposeColumnTarget(sm, M, 0, false);
    Vec trE = trEx(smE), trL = trEx(smD), trD = P.dec(tr);
    P.report("transpose (rotations only)", tr, trD, trE, &trL);
    std::vector<double> rmk(S, 0.0);
    for (size_t i = 0; i < M; ++i) rmk[i] = 1.0;
    auto fin = cc->EvalMult(tr, cc->MakeCKKSPackedPlaintext(rmk, 1, tr->GetLevel(), nullptr, (uint32_t)S));
    Vec finD = P.dec(fin);
    finD.resize(N);
    Vec trLN(trD.begin(), trD.begin() + N);
    P.report("final (first N slots)", fin, finD, sorted, &trLN);
    // the library's own sort_hybrid1 on the same input
    auto ref = ds.sort_hybrid1(ct, SignFunc::CompositeSign, cfg, kp.secretKey);
    Vec refD = P.dec(ref);
    refD.resize(N);
    P.report("sort_hybrid1 (library)", ref, refD, sorted, nullptr);
    return 0;
}

// tests/SincTest.cpp's encrypted experiment (depth 15, default scales, a
// uniform grid on [-1, 1] over every slot): the doubled-sinc series' error,
// split at |x| < 1/(2N) (the hit, an extremum of every giant step)
template <int N>
int sincSeries(int logn, unsigned seed) {
    CCParams<CryptoContextCKKSRNS> params;
    params.SetSecurityLevel(HEStd_NotSet);
    params.SetRingDim(1u << logn);
    params.SetMultiplicativeDepth(15);
    params.SetSeed(seed);
    auto cc = GenCryptoContext(params);
    cc->Enable(PKE);
    cc->Enable(KEYSWITCH);
    cc->Enable(LEVELEDSHE);
    cc->Enable(ADVANCEDSHE);
    auto kp = cc->KeyGen();
    cc->EvalMultKeyGen(kp.secretKey);
    Probe P{cc, kp.secretKey};
    const auto& coeffs = selectDoubledSincCoefficients<N>();
    const size_t slots = (1u << logn) / 2;
    Vec x(slots), f(slots);
    for (size_t i = 0; i < slots; ++i) {
        x[i] = -1.0 + 2.0 * (double)i / (double)(slots - 1);
        f[i] = Sinc<2 * N>::doubled_sinc(x[i]);
    }
    auto pt = cc->MakeCKKSPackedPlaintext(x);
    auto ct = cc->Encrypt(kp.publicKey, pt);
    auto out = cc->EvalChebyshevSeriesPS(ct, coeffs, -1.0, 1.0);
    Vec d = P.dec(out);
    double m0, r0, m1, r1;
    P.stat(d, f, [&](size_t i) { return std::fabs(x[i]) < 0.5 / N; }, m0, r0);
    P.stat(d, f, [&](size_t i) { return std::fabs(x[i]) >= 0.5 / N; }, m1, r1);
    std::printf("sinc N=%d degree %zu ring 2^%d level %u | hit max %.3e rms %.3e | rest max %.3e rms %.3e\n", N,
                coeffs.size() - 1, logn, out->GetLevel(), m0, r0, m1, r1);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s h1|ds N logn [secure] [seed]\n", argv[0]);
        return 2;
    }
    std::string mode = argv[1];
    int N = std::atoi(argv[2]), logn = std::atoi(argv[3]);
    bool secure = argc > 4 && std::atoi(argv[4]);
    unsigned seed = argc > 5 ? (unsigned)std::atoi(argv[5]) : 20251205u + N;
    std::cout.setstate(std::ios::failbit);  // the sort's progress prints
    if (mode == "sinc") switch (N) {
            case 32: return sincSeries<32>(logn, seed);
            case 64: return sincSeries<64>(logn, seed);
            case 128: return sincSeries<128>(logn, seed);
            case 256: return sincSeries<256>(logn, seed);
            default: std::fprintf(stderr, "sinc: N in {32, 64, 128, 256}\n"); return 2;
        }
    switch (N) {
        case 8: return run<8>(mode, logn, secure, seed);
        case 64: return run<64>(mode, logn, secure, seed);
        case 128: return run<128>(mode, logn, secure, seed);
        case 256: return run<256>(mode, logn, secure, seed);
        default: std::fprintf(stderr, "N in {8, 64, 128, 256}\n"); return 2;
    }
}
