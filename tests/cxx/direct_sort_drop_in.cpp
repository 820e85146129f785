// Drop-in check: the call sequence of the reference's DirectSortTest
// (tests/DirectSortTest.cpp:29-54 SetUp, :96-198 SortTest) written against
// this engine's reference-compatible headers only (sort_algo.h, openfhe.h),
// linked to libsfhe.so (HIP) or libsfhe_oracle.so (CPU oracle).
//   usage: direct_sort_drop_in N logRingDim secure(0/1)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <random>
#include <vector>

#include "encryption.h"
#include "openfhe.h"
#include "sort_algo.h"

using namespace lbcrypto;

template <size_t N>
int run(int logRing, bool secure) {
    CCParams<CryptoContextCKKSRNS> parameters;
    std::vector<int> rotations;
    DirectSort<N>::getSizeParameters(parameters, rotations);
    parameters.SetSecurityLevel(secure ? HEStd_128_classic : HEStd_NotSet);
    parameters.SetRingDim(1 << logRing);
    auto cc = GenCryptoContext(parameters);
    cc->Enable(PKE);
    cc->Enable(KEYSWITCH);
    cc->Enable(LEVELEDSHE);
    cc->Enable(ADVANCEDSHE);
    auto keys = cc->KeyGen();
    cc->EvalMultKeyGen(keys.secretKey);
    cc->EvalRotateKeyGen(keys.secretKey, rotations);
    const int multDepth = (int)parameters.GetMultiplicativeDepth();
    auto enc = std::make_shared<DebugEncryption>(cc, keys);

    // distinct k/N in random order (tests/utils.h getVectorWithMinDiff semantics)
    std::vector<double> input(N);
    for (size_t i = 0; i < N; ++i) input[i] = (double)i / N;
    std::mt19937 gen(20251205 + N);
    std::shuffle(input.begin(), input.end(), gen);

    auto ctxt = enc->encryptInput(input);
    auto directSort = std::make_unique<DirectSort<N>>(cc, keys.publicKey, rotations, enc);
    SignConfig Cfg;
    if (N <= 16)
        Cfg = SignConfig(CompositeSignConfig(3, 2, 2));
    else if (N <= 128)
        Cfg = SignConfig(CompositeSignConfig(3, 3, 2));
    else
        Cfg = SignConfig(CompositeSignConfig(3, 4, 2));

    auto t0 = std::chrono::high_resolution_clock::now();
    Ciphertext<DCRTPoly> out = directSort->sort(ctxt, SignFunc::CompositeSign, Cfg);
    auto t1 = std::chrono::high_resolution_clock::now();

    Plaintext pt;
    cc->Decrypt(keys.secretKey, out, &pt);
    pt->SetLength(N);
    auto got = pt->GetRealPackedValue();
    std::vector<double> want = input;
    std::sort(want.begin(), want.end());
    double maxErr = 0;
    for (size_t i = 0; i < N; ++i) maxErr = std::max(maxErr, std::fabs(got[i] - want[i]));
    std::cout << "DROPIN N=" << N << " level=" << out->GetLevel() << " depth=" << multDepth
              << " maxErr=" << maxErr << " ms="
              << std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count() << std::endl;
    return (out->GetLevel() == (uint32_t)multDepth && maxErr < 0.01) ? 0 : 1;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 8;
    const int logRing = argc > 2 ? std::atoi(argv[2]) : 12;
    const bool secure = argc > 3 && std::atoi(argv[3]) != 0;
    switch (N) {
        case 4: return run<4>(logRing, secure);
        case 8: return run<8>(logRing, secure);
        case 16: return run<16>(logRing, secure);
        case 256: return run<256>(logRing, secure);
        default: std::cerr << "unsupported N\n"; return 2;
    }
}
