// k-way sorting network driver (public surface of the reference's
// src/k-way/Sorter.h:1-100): the stage loop of HKC+21's k-way network over
// k^M slots, each stage = one comparison ciphertext (two for k = 5), slot
// matching, the 2/3/4/5-sorters and reassembly, with lazy bootstrapping.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "SortUtils.h"
#include "comparison.h"
#include "openfhe.h"
#include "sign.h"

namespace kwaySort {

class Sorter : public SortUtils {
  public:
    Sorter() = default;
    Sorter(CryptoContext<DCRTPoly> cc, std::shared_ptr<Encryption> enc, long numSlots, long k, long M)
        : SortUtils(cc, enc, numSlots, k, M) {
        initLevels();
    }
    Sorter(CryptoContext<DCRTPoly> cc, std::shared_ptr<Encryption> enc, long numSlots, long k, long M,
           const PrivateKey<DCRTPoly>& privateKey, const PublicKey<DCRTPoly>& publicKey)
        : SortUtils(cc, enc, numSlots, k, M, privateKey, publicKey) {
        initLevels();
    }

    // one stage's sub-sorters of size 2 / 3 / 4 / 5 / mixed 2..5: sort the
    // matched members, keep each sub-sorter's head slots, reassemble
    void runTwoSorter(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long shift,
                      Ciphertext<DCRTPoly>& ctxt_comp, Ciphertext<DCRTPoly>& ctxt_out);
    void runThreeSorter(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long shift,
                        Ciphertext<DCRTPoly>& ctxt_comp, Ciphertext<DCRTPoly>& ctxt_out);
    void runFourSorter(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long shift,
                       Ciphertext<DCRTPoly>& ctxt_comp1, Ciphertext<DCRTPoly>& ctxt_comp2,
                       Ciphertext<DCRTPoly>& ctxt_out);
    void runFiveSorter(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long shift,
                       Ciphertext<DCRTPoly>& ctxt_comp1, Ciphertext<DCRTPoly>& ctxt_comp2,
                       Ciphertext<DCRTPoly>& ctxt_out);
    void run2345Sorter(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long shift,
                       Ciphertext<DCRTPoly>& ctxt_comp1, Ciphertext<DCRTPoly>& ctxt_comp2,
                       Ciphertext<DCRTPoly>& ctxt_out);

    // every member moved onto the slot of the member `rot` before it
    // (ctxt_rot); ctxt_fix = the slots no sub-sorter of the stage touches
    void rightRotateForSort(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long logDist,
                            long slope, Ciphertext<DCRTPoly>& ctxt_rot, Ciphertext<DCRTPoly>& ctxt_fix);
    // ctxt_comp = [ctxt > ctxt_rot] (and [ctxt > ctxt_rot_rot] for k = 5)
    void comparisonForSort(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long logDist,
                           long slope, Ciphertext<DCRTPoly>& ctxt_comp, Ciphertext<DCRTPoly>& ctxt_fix,
                           SignConfig& Cfg);
    void comparisonForSort2(Ciphertext<DCRTPoly>& ctxt, std::vector<std::vector<int>>& indices, long logDist,
                            long slope, Ciphertext<DCRTPoly>& ctxt_comp1, Ciphertext<DCRTPoly>& ctxt_comp2,
                            Ciphertext<DCRTPoly>& ctxt_fix, SignConfig& Cfg);

    // the whole network (Sorter.cpp:284-404)
    void sorter(Ciphertext<DCRTPoly>& ctxt, Ciphertext<DCRTPoly>& ctxt_out, SignConfig& Cfg);
    // engine extension: the network's stages [first, last) on ctxt (in place;
    // false: no stage schedule for this k) -- the pieces KWayAdapter captures
    int stageCount() const;
    bool runStages(Ciphertext<DCRTPoly>& ctxt, int first, int last, SignConfig& Cfg);

  protected:
    // levels a stage of each sub-sorter size needs after its comparison
    void initLevels() { m_level = {0, 1, 3, 5, 6, 7}; }

    Comparison comp;
};

}  // namespace kwaySort
