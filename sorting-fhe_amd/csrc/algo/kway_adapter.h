// k-way sort behind the SortBase<N> interface (public surface of the
// reference's src/kway_adapter.h:1-75; SURVEY §8(f) row 2, BASELINE config 4:
// N = 1024 = 2^10 at ring 2^17, depth 40, scale 59, levelBudget {5,5}).
#pragma once

#include <cassert>
#include <cmath>
#include <memory>

#include "k-way/Sorter.h"
#include "key/privatekey-fwd.h"
#include "sort_algo.h"

constexpr int next_power_of_two(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return n <= 0 ? 1 : p;
}

template <int N>
class KWayAdapter : public SortBase<N> {
  public:
    KWayAdapter(CryptoContext<DCRTPoly> cc, PublicKey<DCRTPoly> publicKey, PrivateKey<DCRTPoly> privateKey,
                std::shared_ptr<Encryption> enc, int k, int M)
        : SortBase<N>(enc), m_cc(cc), m_PublicKey(publicKey), m_enc(enc) {
        assert(std::pow(k, M) == N && "k^M should be equal to input length N");
        m_sorter = std::make_unique<kwaySort::Sorter>(cc, enc, N, k, M, privateKey, publicKey);
    }

    // batch = next power of two >= N, q0 60 bits, scale 59, depth 40, the
    // +-2^i rotation keys; bootstrapping level budget {4,4} up to N = 128,
    // {5,5} above (kway_adapter.h:41-64)
    static void getSizeParameters(CCParams<CryptoContextCKKSRNS>& parameters, std::vector<int>& rotations,
                                  std::vector<uint32_t>& levelBudget) {
        parameters.SetBatchSize(next_power_of_two(N));
        parameters.SetFirstModSize(60);
        parameters.SetScalingModSize(59);
        for (int i = 1; i < N; i *= 2) {
            rotations.push_back(i);
            rotations.push_back(-i);
        }
        levelBudget = N <= 128 ? std::vector<uint32_t>{4, 4} : std::vector<uint32_t>{5, 5};
        parameters.SetMultiplicativeDepth(40);
    }

    // (Not graph-captured, unlike DirectSort::sort: a captured graph pins
    // every buffer it touches for its lifetime.  One hipGraph per stage was
    // tried at N = 1024 @ 2^17: each stage is ~4.1 k nodes, and the capture
    // of stage 17 failed on a host synchronisation -- the pool, whose blocks
    // 16 captured stages now pinned, had to grow.)
    Ciphertext<DCRTPoly> sort(const Ciphertext<DCRTPoly>& input_array, SignFunc, SignConfig& Cfg) override {
        return sortEager(input_array, Cfg);
    }

  private:
    Ciphertext<DCRTPoly> sortEager(const Ciphertext<DCRTPoly>& input_array, SignConfig& Cfg) {
        Ciphertext<DCRTPoly> in = input_array->Clone(), out;
        m_sorter->sorter(in, out, Cfg);
        return out;
    }

    CryptoContext<DCRTPoly> m_cc;
    PublicKey<DCRTPoly> m_PublicKey;
    std::shared_ptr<Encryption> m_enc;
    std::unique_ptr<kwaySort::Sorter> m_sorter;
};
