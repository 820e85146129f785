// k-way sorting network: comparator networks and slot matching (public
// surface of the reference's src/k-way/SortUtils.h:1-122).
//
// Sub-sorters take their inputs as ciphertexts aligned slot for slot plus the
// pairwise comparison bits c(x, y) = [x > y] (CKKS values in {0, 1}) and
// return the sorted order using only the select form
//   max = c (x - y) + y,   min = x + y - max
// (one level per select).  slotMatching* line a stage's sub-sorter members
// and comparison bits up in the same slots; slotAssemble puts the sorted
// members back.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "EvalUtils.h"
#include "Masking.h"
#include "encryption.h"
#include "openfhe.h"

using namespace lbcrypto;

namespace kwaySort {

class SortUtils : public EvalUtils {
  public:
    SortUtils() = default;
    SortUtils(CryptoContext<DCRTPoly> cc, std::shared_ptr<Encryption> enc, long numSlots, long k, long M)
        : EvalUtils(cc), m_numSlots(numSlots), m_k(k), m_M(M), m_enc(enc) {
        initializeLevels();
    }
    SortUtils(CryptoContext<DCRTPoly> cc, std::shared_ptr<Encryption> enc, long numSlots, long k, long M,
              const PrivateKey<DCRTPoly>& privateKey, const PublicKey<DCRTPoly>& publicKey)
        : EvalUtils(cc, enc, publicKey, privateKey), m_numSlots(numSlots), m_k(k), m_M(M), m_enc(enc) {
        initializeLevels();
    }

    // comp (a - b) + b: a where comp = 1, b where comp = 0
    void fcnL(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt2, Ciphertext<DCRTPoly>& comp,
              Ciphertext<DCRTPoly>& ctxt_out);
    void compareMax(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt2, Ciphertext<DCRTPoly>& comp,
                    Ciphertext<DCRTPoly>& ctxt_out);
    void compareMin(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt2, Ciphertext<DCRTPoly>& comp,
                    Ciphertext<DCRTPoly>& ctxt_out);

    // [a, b], [a > b] -> [min, max]
    void twoSorter(Ciphertext<DCRTPoly>* ctxt, Ciphertext<DCRTPoly>& comp, Ciphertext<DCRTPoly>* ctxt_out);
    void twoSorter(Ciphertext<DCRTPoly>& ctxt1, Ciphertext<DCRTPoly>& ctxt2, Ciphertext<DCRTPoly>& comp,
                   Ciphertext<DCRTPoly>* ctxt_out);
    // [a, b, c], [a>b, a>c, b>c]
    void threeSorter(Ciphertext<DCRTPoly>* ctxt, Ciphertext<DCRTPoly>* comp, Ciphertext<DCRTPoly>* ctxt_out);
    // [a, b, c, d], [a>b, a>c, a>d, b>c, b>d, c>d]
    void fourSorter(Ciphertext<DCRTPoly>* ctxt, Ciphertext<DCRTPoly>* comp, Ciphertext<DCRTPoly>* ctxt_out);
    // [a .. e], [a>b a>c a>d a>e b>c b>d b>e c>d c>e d>e]
    void fiveSorter(Ciphertext<DCRTPoly>* ctxt, Ciphertext<DCRTPoly>* comp, Ciphertext<DCRTPoly>* ctxt_out);

    void slotMatching2(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_comp,
                       std::vector<std::vector<int>>& indices, long shift, Ciphertext<DCRTPoly>* ctxt_out,
                       Ciphertext<DCRTPoly>& ctxt_comp_out);
    void slotMatching3(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_comp,
                       std::vector<std::vector<int>>& indices, long shift, Ciphertext<DCRTPoly>* ctxt_out,
                       Ciphertext<DCRTPoly>* ctxt_comp_out);
    void slotMatching4(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_comp1,
                       Ciphertext<DCRTPoly>& ctxt_comp2, std::vector<std::vector<int>>& indices, long shift,
                       Ciphertext<DCRTPoly>* ctxt_out, Ciphertext<DCRTPoly>* ctxt_comp_out);
    void slotMatching5(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_comp1,
                       Ciphertext<DCRTPoly>& ctxt_comp2, std::vector<std::vector<int>>& indices, long shift,
                       Ciphertext<DCRTPoly>* ctxt_out, Ciphertext<DCRTPoly>* ctxt_comp_out);
    void slotMatching2345(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_comp1,
                          Ciphertext<DCRTPoly>& ctxt_comp2, std::vector<std::vector<int>>& indices, long shift,
                          Ciphertext<DCRTPoly>* ctxt_out, Ciphertext<DCRTPoly>* ctxt_comp_out);
    // declared by the reference, never defined there (SortUtils.h:95-99)
    void slotMatching23(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_comp,
                        std::vector<std::vector<int>>& indices, long shift, Ciphertext<DCRTPoly>* ctxt_out,
                        Ciphertext<DCRTPoly>* ctxt_comp_out);

    // ctxt_out = sum_i RotR(ctxt_sort[i], i shift)
    void slotAssemble(Ciphertext<DCRTPoly>* ctxt_sort, long num, long shift, Ciphertext<DCRTPoly>& ctxt_out);

  protected:
    void initializeLevels() { m_level = {0, 0, 2, 3, 4, 6}; }

    // 0/1 mask of the slots labelled (size, pos) in `indices`, as a plaintext
    Plaintext labelMask(const std::vector<std::vector<int>>& indices, std::initializer_list<int> sizes, int pos);

    long m_numSlots = 0;
    long m_k = 0;
    long m_M = 0;
    std::vector<int> m_level;
    std::shared_ptr<Encryption> m_enc;
};

}  // namespace kwaySort
