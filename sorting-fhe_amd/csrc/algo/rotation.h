// Slot rotations by composition of available rotation keys.
// Public surface of the reference's src/rotation.h: Step :12-18,
// DecomposeAlgo :28, Decomposer<N> :30-166, RotationComposer<N> :193-238,
// RotationTree<N> :240-358.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <iostream>
#include <map>
#include <memory>
#include <set>
#include <vector>

#include "ciphertext-fwd.h"
#include "encryption.h"
#include "lattice/hal/lat-backend.h"
#include "openfhe.h"

using namespace lbcrypto;

struct Step {
    int8_t value;  // digit: -1/0/1 (NAF, BNAF) or 1 (binary / greedy)
    int stepSize;  // signed rotation amount of this step
    Step(int8_t v, int s) : value(v), stepSize(s) {}
    Step(int s) : value(1), stepSize(s) {}
};

inline void dump(std::vector<Step> steps) {
    std::cout << "Decomposed steps: [";
    for (const auto& s : steps) std::cout << "(" << (int)s.value << ", " << s.stepSize << "), ";
    std::cout << " ]" << std::endl;
}

enum class DecomposeAlgo { NAF, BNAF, BINARY };

// Splits a rotation amount into steps that have keys: whole multiples of
// the largest key first, then the largest keys below the amount until it is
// within the "doubling chain" range, then a signed-digit / binary expansion.
template <int N>
class Decomposer {
  public:
    explicit Decomposer(std::vector<int> rot) : keys(std::move(rot)) {
        std::sort(keys.begin(), keys.end());
        // reach of the doubling chain 1,2,4,...: sum of every key that is
        // exactly twice its predecessor in sorted order
        int prev = 1;
        for (int k : keys) {
            if (k / 2 == prev) chainReach += k;
            prev = k;
        }
    }

    std::vector<int> getRotIndices() { return keys; }

    std::vector<Step> decompose(int rotation, int wrapN, DecomposeAlgo algo) {
        std::vector<Step> out;
        const int top = keys.back();
        for (; rotation >= top; rotation -= top) out.emplace_back(top);
        if (rotation == 0) return out;
        while (rotation > chainReach) {
            int below = *(std::lower_bound(keys.begin(), keys.end(), rotation) - 1);
            out.emplace_back(below);
            rotation -= below;
        }
        if (rotation == 0) return out;
        std::vector<Step> tail = algo == DecomposeAlgo::NAF    ? naf(rotation)
                                 : algo == DecomposeAlgo::BNAF ? bnaf(rotation)
                                                               : binary(rotation);
        out.insert(out.end(), tail.begin(), tail.end());
        // a step that is a whole number of periods is the identity
        out.erase(std::remove_if(out.begin(), out.end(),
                                 [wrapN](const Step& s) { return s.stepSize % wrapN == 0; }),
                  out.end());
        return out;
    }

  private:
    std::vector<Step> binary(int r) const {
        std::vector<Step> s;
        for (int b = 31; b >= 0; --b) {
            const int w = 1 << b;
            if (w < N && (r & w)) s.emplace_back((int8_t)1, w);
        }
        return s;
    }

    // non-adjacent form, most significant step first; -N/2 folds to +N/2
    std::vector<Step> naf(int r) const {
        std::vector<Step> s;
        for (int b = 0; r != 0; ++b, r >>= 1) {
            if (!(r & 1)) continue;
            const int z = (r & 2) ? -1 : 1;
            const int w = z * (1 << b);
            if (w == -N / 2)
                s.emplace_back((int8_t)-z, -w);
            else
                s.emplace_back((int8_t)z, w);
            r -= z;
        }
        std::reverse(s.begin(), s.end());
        return s;
    }

    // balanced base-2 signed digits (ties rounded toward the next digit)
    std::vector<Step> bnaf(int r) const {
        std::vector<int> dig;
        for (int K = r; K != 0;) {
            int d = K % 2;
            K = (K - d) / 2;
            if (d > 1 || (d == 1 && (K % 2) >= 1)) {
                d -= 2;
                K += 1;
            }
            dig.push_back(d);
        }
        std::vector<Step> s;
        for (size_t b = 0; b < dig.size(); ++b)
            if (dig[b]) s.emplace_back((int8_t)dig[b], (int)(dig[b] * (int64_t(1) << b)));
        std::reverse(s.begin(), s.end());
        return s;
    }

    std::vector<int> keys;
    int chainReach = 0;
};

template <int N>
class RotationComposer {
  public:
    RotationComposer(CryptoContext<DCRTPoly> cc, std::shared_ptr<Encryption> enc,
                     std::vector<int> rotIndices, DecomposeAlgo algo = DecomposeAlgo::BINARY)
        : m_cc(cc), m_enc(enc), m_decomposer(rotIndices), m_algo(algo),
          m_keys(rotIndices.begin(), rotIndices.end()) {}

    // Left rotation by `rotation` slots (period = the ciphertext's slots).
    Ciphertext<DCRTPoly> rotate(const Ciphertext<DCRTPoly>& in, int rotation) {
        if (rotation % (int)in->GetSlots() == 0) return in->Clone();
        if (m_keys.count(rotation)) return m_cc->EvalRotate(in, rotation);
        Ciphertext<DCRTPoly> r = in;
        for (const auto& s : m_decomposer.decompose(rotation, in->GetSlots(), m_algo))
            r = m_cc->EvalRotate(r, s.stepSize);
        return r == in ? in->Clone() : r;
    }

    // Engine extension: several rotations of ONE ciphertext sharing a single
    // key-switch ModUp (hoisting).  Same results as rotate() up to noise.
    std::vector<Ciphertext<DCRTPoly>> rotateMany(const Ciphertext<DCRTPoly>& in,
                                                 const std::vector<int>& amounts) {
        std::vector<Ciphertext<DCRTPoly>> out(amounts.size());
        static const bool noHoist = std::getenv("SFHE_NO_HOIST") != nullptr;
        bool hoist = !noHoist;
        for (int a : amounts)
            if (a % (int)in->GetSlots() != 0 && !m_keys.count(a)) hoist = false;
        if (!hoist) {
            for (size_t i = 0; i < amounts.size(); ++i) out[i] = rotate(in, amounts[i]);
            return out;
        }
        std::shared_ptr<FastRotationPrecomp> pre;
        for (int a : amounts)
            if (a % (int)in->GetSlots() != 0) {
                pre = m_cc->EvalFastRotationPrecompute(in);
                break;
            }
        // the rotations are independent: batches of them run as merged
        // launches (BatchScope; same values, one op per virtual lane)
        const size_t w = m_cc->BatchWidth();
        for (size_t b0 = 0; b0 < amounts.size(); b0 += w) {
            const size_t b1 = std::min(amounts.size(), b0 + w);
            BatchScope bs(m_cc.get(), (uint32_t)(b1 - b0));
            for (size_t i = b0; i < b1; ++i) {
                bs.lane((uint32_t)(i - b0));
                if (amounts[i] % (int)in->GetSlots() == 0)
                    out[i] = in->Clone();
                else
                    out[i] = m_cc->EvalFastRotation(in, amounts[i], m_cc->GetCyclotomicOrder(), pre);
            }
        }
        return out;
    }

    // sum_k rotate(in_k, rotations_k), the value of EvalAddMany over rotate():
    // each term's steps but the last are applied as rotate() would, and the
    // last steps of all terms share one ModDown (EvalRotateSum).
    Ciphertext<DCRTPoly> rotateSum(const std::vector<Ciphertext<DCRTPoly>>& in,
                                   const std::vector<int>& rotations) {
        std::vector<Ciphertext<DCRTPoly>> pre;
        std::vector<int32_t> last;
        for (size_t k = 0; k < in.size(); ++k) {
            const int r = rotations[k], slots = (int)in[k]->GetSlots();
            if (r % slots == 0 || m_keys.count(r)) {
                pre.push_back(in[k]);
                last.push_back(r % slots == 0 ? 0 : r);
                continue;
            }
            const auto steps = m_decomposer.decompose(r, slots, m_algo);
            Ciphertext<DCRTPoly> x = in[k];
            for (size_t i = 0; i + 1 < steps.size(); ++i) x = m_cc->EvalRotate(x, steps[i].stepSize);
            pre.push_back(x);
            last.push_back(steps.empty() ? 0 : steps.back().stepSize);
        }
        return m_cc->EvalRotateSum(pre, last);
    }

    const std::set<int>& getRotationCalls() const { return rotation_calls; }
    void clearRotationCalls() { rotation_calls.clear(); }

  private:
    CryptoContext<DCRTPoly> m_cc;
    std::shared_ptr<Encryption> m_enc;
    Decomposer<N> m_decomposer;
    DecomposeAlgo m_algo;
    std::set<int> m_keys;
    std::set<int> rotation_calls;
};

// Rotation with a cache of composed step results (reference :240-358; used
// only by its RotationTest / RotationBenchmark).  Steps are applied with
// hoisted key switching from the input.
template <int N>
class RotationTree {
  public:
    RotationTree(CryptoContext<DCRTPoly> cc, const std::vector<int>& rotIndices,
                 DecomposeAlgo algo = DecomposeAlgo::NAF)
        : m_cc(cc), m_decomposer(rotIndices), m_algo(algo) {}

    void buildTree(int, int) {}

    Ciphertext<DCRTPoly> treeRotate(const Ciphertext<DCRTPoly>& input, int rotation) {
        auto steps = m_decomposer.decompose(rotation, input->GetSlots(), m_algo);
        Ciphertext<DCRTPoly> r = input;
        int acc = 0;
        for (const auto& s : steps) {
            acc += s.stepSize;
            auto it = m_cache.find(acc);
            if (it != m_cache.end() && m_src == input.get()) {
                r = it->second;
                continue;
            }
            r = m_cc->EvalRotate(r, s.stepSize);
            if (m_src != input.get()) {
                m_cache.clear();
                m_src = input.get();
            }
            m_cache[acc] = r;
        }
        return r == input ? input->Clone() : r;
    }

  private:
    CryptoContext<DCRTPoly> m_cc;
    Decomposer<N> m_decomposer;
    DecomposeAlgo m_algo;
    const void* m_src = nullptr;
    std::map<int, Ciphertext<DCRTPoly>> m_cache;
};
