// Prim-level microbenchmark of the HIP backend (links libsfhe.so).
//   make -C tools microbench && tools/build/microbench [logn]
// Times sfp_ntt (forward / inverse) over a range of limb counts, and the
// fused key-switch / rescale prims at the metric context's top level.
// Reports average wall time per call (stream-synchronised batches) and the
// algorithmic bandwidth (prims.h byte model).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "openfhe.h"
#include "prims.h"
#include "state.h"

using namespace lbcrypto;

extern "C" int sfp_ntt_trace(sfp_dev* d, unsigned long long* out32);

// per-block phase clocks of the last measured NTTs (SFHE_NTT_TRACE builds)
static void printTrace(sfp_dev* d) {
    unsigned long long t[32];
    if (sfp_ntt_trace(d, t) != 0) return;
    static const char* names[4] = {"fwd ROW", "fwd COL", "inv ROW", "inv COL"};
    for (int v = 0; v < 4; ++v) {
        const unsigned long long nb = t[v * 8 + 7];
        if (!nb) continue;
        std::printf("    %s blocks=%llu clk/block:", names[v], nb);
        for (int p = 0; p < 6; ++p) std::printf(" %7.0f", (double)t[v * 8 + p] / nb);
        std::printf("\n");
    }
}

template <class F>
static double timeIt(sfp_dev* d, int iters, F&& f) {
    // MB_REPS caps the repetitions (PMC passes serialise every dispatch)
    static const int cap = std::getenv("MB_REPS") ? std::atoi(std::getenv("MB_REPS")) : 0;
    if (cap > 0 && iters > cap) iters = cap;
    f();
    sfp_sync(d);
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < iters; ++i) f();
    sfp_sync(d);
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
}

int main(int argc, char** argv) {
    const int logn = argc > 1 ? std::atoi(argv[1]) : 16;
    CCParams<CryptoContextCKKSRNS> p;
    p.SetMultiplicativeDepth(34);
    p.SetScalingModSize(40);
    p.SetRingDim(1u << logn);
    p.SetBatchSize(256);
    p.SetSecurityLevel(HEStd_NotSet);
    auto cc = GenCryptoContext(p);
    SfheContextState* s = cc->state();
    sfp_dev* d = s->dev;
    const uint32_t n = s->n;
    const size_t maxRows = 160;
    auto* buf = (uint64_t*)sfp_alloc(d, maxRows * n * 8);
    const uint32_t NP = s->Lq + s->K;  // valid prime indices: [0, NP)
    for (size_t r0 = 0; r0 < maxRows; r0 += NP) {
        const uint32_t c = (uint32_t)std::min<size_t>(NP, maxRows - r0);
        sfp_sample_uniform(d, buf + r0 * n, sfp_limbs{c, c, 0, 0}, 7 + r0);
    }
    setvbuf(stdout, nullptr, _IONBF, 0);
    std::printf("n=2^%d Lq=%u K=%u dnum=%u alpha=%u\n", logn, s->Lq, s->K, s->dnum, s->alpha);
    std::printf("%-10s %6s %10s %10s %10s %10s\n", "op", "rows", "fwd us", "fwd GB/s", "inv us",
                "inv GB/s");
    for (uint32_t rows : {1u, 2u, 4u, 8u, 16u, 24u, 35u, 44u, 70u, 96u, 140u}) {
        static const uint32_t base = std::getenv("MB_BASE") ? std::atoi(std::getenv("MB_BASE")) : 0;
        if (rows > maxRows || (rows <= NP && rows + base > NP)) continue;
        // beyond NP rows the map wraps: rows [NP, rows) reuse primes 0.. (batched launches)
        const sfp_limbs m = rows <= NP ? sfp_limbs{rows, rows, base, 0} : sfp_limbs{rows, NP, 0, 0};
        if (rows > 2 * NP) continue;
        unsigned long long scratch[32];
        sfp_ntt_trace(d, scratch);
        const double f = timeIt(d, 50, [&] { sfp_ntt(d, buf, m, 0); });
        const double i = timeIt(d, 50, [&] { sfp_ntt(d, buf, m, 1); });
        const double bytes = 32.0 * rows * n;  // two passes x 16 B per coefficient
        std::printf("%-10s %6u %10.2f %10.1f %10.2f %10.1f\n", "ntt", rows, f, bytes / f / 1e3, i,
                    bytes / i / 1e3);
        printTrace(d);
    }
    // Lane concurrency: K forward NTTs on lane 0 alone, then K on each of
    // lanes 0 and 1 (independent buffers, issued alternately).  ratio = the
    // two-lane time / the one-lane time: 1.0 = the lanes overlap fully, 2.0 =
    // they serialise (the sort's two batches are such lanes).
    if (sfp_lanes(d) >= 2) {
        std::printf("%-10s %6s %10s %10s %8s\n", "lanes", "rows", "1 lane us", "2 lanes us", "ratio");
        for (uint32_t rows : {1u, 4u, 8u, 16u, 35u}) {
            if (rows > NP || 2 * rows > maxRows) continue;
            const sfp_limbs m{rows, rows, 0, 0};
            uint64_t* b1 = buf + (size_t)(maxRows / 2) * n;
            const double one = timeIt(d, 50, [&] {
                sfp_set_lane(d, 0);
                sfp_ntt(d, buf, m, 0);
            });
            const double two = timeIt(d, 50, [&] {
                sfp_set_lane(d, 0);
                sfp_ntt(d, buf, m, 0);
                sfp_set_lane(d, 1);
                sfp_ntt(d, b1, m, 0);
            });
            sfp_set_lane(d, 0);
            std::printf("%-10s %6u %10.2f %10.2f %8.2f\n", "ntt", rows, one, two, two / one);
        }
    }
    // key switch pieces at the top level (ell = Lq)
    const uint32_t ell = s->Lq, K = s->K, beta = (ell + s->alpha - 1) / s->alpha;
    const size_t stride = (size_t)(ell + K) * n;
    auto* ext = (uint64_t*)sfp_alloc(d, stride * beta * 8);
    auto* scr = (uint64_t*)sfp_alloc(d, (size_t)2 * ell * n * 8);
    auto* acc = (uint64_t*)sfp_alloc(d, 2 * stride * 8);
    auto* out = (uint64_t*)sfp_alloc(d, (size_t)2 * ell * n * 8);
    sfp_sample_uniform(d, acc, sfp_limbs{ell + K, ell, s->Lq, 0}, 9);
    sfp_sample_uniform(d, acc + stride, sfp_limbs{ell + K, ell, s->Lq, 0}, 10);
    // conversion tables as the engine builds them
    std::vector<sfp_conv*> convs;
    {
        auto ct = cc->Encrypt(cc->KeyGen().publicKey, cc->MakeCKKSPackedPlaintext(std::vector<double>(256, 0.5)));
        cc->EvalMultKeyGen(cc->KeyGen().secretKey);
        auto sq = cc->EvalMult(ct, ct);  // builds the modup tables of the top level
        cc->Settle(sq);                  // (a lazy product relinearises when settled)
        (void)sq;
        convs = s->modupConv.at(ell);
    }
    // the conversion family's algorithmic bytes from here on (tools/pmc_traffic.py
    // pairs them with the last CONV_ALGO launches of the PMC passes)
    sfp_prof_set(d, SFP_FAM_CONV, 1);
    const double mu = timeIt(d, 30, [&] {
        sfp_modup(d, ext, buf, ell, K, s->Lq, s->alpha, convs.data(), scr);
    });
    for (uint32_t j = 0; j < beta; ++j) {
        // source rows: the digit's own primes (rows lo.. of buf hold residues mod those)
        const uint64_t* src = buf + (size_t)j * s->alpha * n;
        const double cv = timeIt(d, 30, [&] { sfp_conv_apply(d, ext, src, convs[j]); });
        std::printf("conv digit %u          : %8.2f us\n", j, cv);
    }
    const double ki = timeIt(d, 30, [&] {
        sfp_ks_inner(d, acc, acc + stride, ext, stride, s->relinKey->ptr, beta, ell, K, s->Lq);
    });
    const double md = timeIt(d, 30, [&] {
        sfp_moddown2(d, out, out + (size_t)ell * n, acc, stride, ell, K, s->Lq, s->moddownConv,
                     s->pInvModQ.data(), 1, 1, scr, 0);
    });
    const double rs = timeIt(d, 30, [&] {
        sfp_rescale(d, out, buf, ell, s->qInvTable[ell].data(), 2, (size_t)ell * n, (size_t)(ell - 1) * n);
    });
    // the fused key-switch chains (ModUp + inner product in one pass family;
    // tensor + relinearisation + rescale without the tensor in HBM)
    const double mi = timeIt(d, 30, [&] {
        sfp_modup_inner(d, acc, acc + stride, buf, ell, K, s->Lq, s->alpha, convs.data(), s->relinKey->ptr,
                        nullptr, nullptr, 0, 0, ~0u, ext, scr);
    });
    const size_t pw = (size_t)ell * n;
    // four canonical operand polynomials (residues of each row's own prime)
    auto* ops = (uint64_t*)sfp_alloc(d, 4 * pw * 8);
    for (int k = 0; k < 4; ++k) sfp_sample_uniform(d, ops + k * pw, sfp_limbs{ell, ell, 0, 0}, 21 + k);
    const double mr = timeIt(d, 30, [&] {
        sfp_mult_relin_rescale(d, out, out + pw, ops, ops + pw, ops + 2 * pw, ops + 3 * pw, ell, K, s->Lq,
                               s->alpha, convs.data(), s->relinKey->ptr, s->moddownConv, s->pInvModQ.data(),
                               s->pModQ.data(), s->qInvTable[ell].data(), acc, ext, scr);
    });
    const double B = 8.0 * n;
    std::printf("modup   ell=%u beta=%u: %8.2f us  (%.1f GB/s on ell + beta(ell+K) rows)\n", ell, beta,
                mu, (ell + beta * (ell + K)) * B / mu / 1e3);
    std::printf("ks_inner            : %8.2f us  (%.1f GB/s)\n", ki, (3.0 * beta + 2) * (ell + K) * B / ki / 1e3);
    std::printf("moddown2            : %8.2f us  (%.1f GB/s on 2(ell+K) + 2 ell rows)\n", md,
                (2.0 * (ell + K) + 2.0 * ell) * B / md / 1e3);
    std::printf("rescale x2 polys    : %8.2f us  (%.1f GB/s on 4 ell rows)\n", rs, 4.0 * ell * B / rs / 1e3);
    std::printf("modup_inner (fused) : %8.2f us  (modup + ks_inner: %.2f us)\n", mi, mu + ki);
    std::printf("mult_relin_rescale  : %8.2f us\n", mr);
    {
        uint64_t launches = 0, timed = 0;
        double ms = 0, bytes = 0;
        sfp_prof_read(d, SFP_FAM_CONV, &launches, &timed, &ms, &bytes);
        sfp_prof_set(d, SFP_FAM_CONV, 0);
        std::printf("CONV_ALGO launches=%llu bytes=%.0f ms=%.3f\n", (unsigned long long)launches, bytes, ms);
    }
    const char* e = sfp_last_error(d);
    if (e) std::printf("ERROR: %s\n", e);
    return e ? 1 : 0;
}
