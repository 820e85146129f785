// k-way sorting network driver (reference src/k-way/Sorter.cpp).
#include "Sorter.h"

#include <cassert>
#include <cstdlib>
#include <string>
#include <iostream>

#include "encryption.h"

namespace kwaySort {

using Ct = Ciphertext<DCRTPoly>;

void Sorter::runTwoSorter(Ct& ctxt, std::vector<std::vector<int>>& indices, long shift, Ct& ctxt_comp,
                          Ct& ctxt_out) {
    Plaintext head = labelMask(indices, {2}, 1);
    Ct members[2], bit, sorted[2];
    slotMatching2(ctxt, ctxt_comp, indices, shift, members, bit);
    twoSorter(members, bit, sorted);
    for (Ct& s : sorted) s = m_cc->EvalMult(s, head);
    Ct back;
    rightRotate(sorted[1], shift, back);
    ctxt_out = m_cc->EvalAdd(sorted[0], back);
}

void Sorter::runThreeSorter(Ct& ctxt, std::vector<std::vector<int>>& indices, long shift, Ct& ctxt_comp,
                            Ct& ctxt_out) {
    Plaintext head = labelMask(indices, {3}, 1);
    Ct members[3], bits[3], sorted[3];
    slotMatching3(ctxt, ctxt_comp, indices, shift, members, bits);
    threeSorter(members, bits, sorted);
    for (Ct& s : sorted) s = m_cc->EvalMult(s, head);
    slotAssemble(sorted, 3, shift, ctxt_out);
}

void Sorter::runFourSorter(Ct& ctxt, std::vector<std::vector<int>>& indices, long shift, Ct& ctxt_comp1,
                           Ct& ctxt_comp2, Ct& ctxt_out) {
    Ct members[4], bits[6], sorted[4];  // members come masked to the heads already
    slotMatching4(ctxt, ctxt_comp1, ctxt_comp2, indices, shift, members, bits);
    fourSorter(members, bits, sorted);
    slotAssemble(sorted, 4, shift, ctxt_out);
}

void Sorter::runFiveSorter(Ct& ctxt, std::vector<std::vector<int>>& indices, long shift, Ct& ctxt_comp1,
                           Ct& ctxt_comp2, Ct& ctxt_out) {
    Plaintext head = labelMask(indices, {5}, 1);
    Ct members[5], bits[10], sorted[5];
    slotMatching5(ctxt, ctxt_comp1, ctxt_comp2, indices, shift, members, bits);
    fiveSorter(members, bits, sorted);
    for (Ct& s : sorted) s = m_cc->EvalMult(s, head);
    slotAssemble(sorted, 5, shift, ctxt_out);
}

// sub-sorters of sizes 2..5 run as 5-sorters; output i is kept on the heads of
// the sub-sorters that have a member i
void Sorter::run2345Sorter(Ct& ctxt, std::vector<std::vector<int>>& indices, long shift, Ct& ctxt_comp1,
                           Ct& ctxt_comp2, Ct& ctxt_out) {
    Ct members[5], bits[10], sorted[5];
    slotMatching2345(ctxt, ctxt_comp1, ctxt_comp2, indices, shift, members, bits);
    fiveSorter(members, bits, sorted);
    Plaintext keep[5] = {labelMask(indices, {2, 3, 4, 5}, 1), labelMask(indices, {2, 3, 4, 5}, 1),
                         labelMask(indices, {3, 4, 5}, 1), labelMask(indices, {4, 5}, 1), labelMask(indices, {5}, 1)};
    for (int i = 0; i < 5; ++i) sorted[i] = m_cc->EvalMult(sorted[i], keep[i]);
    slotAssemble(sorted, 5, shift, ctxt_out);
}

// Members other than a sub-sorter's last move `rot` slots right (onto the
// next member); the last members of the sizes that wrap move back left to the
// head.  Slope 0: only k-sorters; the middle slope: (k-1)-sorters; otherwise
// every size, and the 1-member "sorters" stay in ctxt_fix.
void Sorter::rightRotateForSort(Ct& ctxt, std::vector<std::vector<int>>& indices, long logDist, long slope,
                                Ct& ctxt_rot, Ct& ctxt_fix) {
    std::vector<double> notLast(m_numSlots, 0.0);
    std::vector<std::vector<double>> lastOf(m_k, std::vector<double>(m_numSlots, 0.0));
    for (long i = 0; i < m_numSlots; ++i) {
        const int size = indices[0][i], pos = indices[1][i];
        if (pos < size) notLast[i] = 1.0;
        if (size > 0 && size == pos) lastOf[size - 1][i] = 1.0;
    }
    const long rot = getRotateDistance(m_k, logDist, slope);
    Ct left = m_cc->EvalMult(ctxt, m_cc->MakeCKKSPackedPlaintext(notLast));
    rightRotate(left, rot, ctxt_rot);
    auto wrap = [&](long size) {  // last members of `size`-sorters, moved to their heads
        Ct last = m_cc->EvalMult(ctxt, m_cc->MakeCKKSPackedPlaintext(lastOf[size - 1]));
        Ct moved;
        leftRotate(last, (size - 1) * rot, moved);
        ctxt_rot = m_cc->EvalAdd(ctxt_rot, moved);
        return last;
    };
    if (slope == 0) {
        wrap(m_k);
        return;
    }
    if (slope == m_k / 2 + 1) {
        Ct last = wrap(m_k - 1);
        ctxt_fix = m_cc->EvalSub(m_cc->EvalSub(ctxt, left), last);
        return;
    }
    ctxt_fix = m_cc->EvalSub(ctxt, left);
    ctxt_fix = m_cc->EvalSub(ctxt_fix, m_cc->EvalMult(ctxt, m_cc->MakeCKKSPackedPlaintext(lastOf[0])));
    for (long size = 2; size <= m_k; ++size) ctxt_fix = m_cc->EvalSub(ctxt_fix, wrap(size));
}

void Sorter::comparisonForSort(Ct& ctxt, std::vector<std::vector<int>>& indices, long logDist, long slope,
                               Ct& ctxt_comp, Ct& ctxt_fix, SignConfig& Cfg) {
    Ct prev;
    rightRotateForSort(ctxt, indices, logDist, slope, prev, ctxt_fix);
    ctxt_comp = comp.compare(m_cc, ctxt, prev, SignFunc::CompositeSign, Cfg);
}

void Sorter::comparisonForSort2(Ct& ctxt, std::vector<std::vector<int>>& indices, long logDist, long slope,
                                Ct& ctxt_comp1, Ct& ctxt_comp2, Ct& ctxt_fix, SignConfig& Cfg) {
    Ct prev1, prev2, unused;
    rightRotateForSort(ctxt, indices, logDist, slope, prev1, ctxt_fix);
    rightRotateForSort(prev1, indices, logDist, slope, prev2, unused);
    ctxt_comp1 = comp.compare(m_cc, ctxt, prev1, SignFunc::CompositeSign, Cfg);
    ctxt_comp2 = comp.compare(m_cc, ctxt, prev2, SignFunc::CompositeSign, Cfg);
}

int Sorter::stageCount() const { return (int)(m_M + m_M * (m_M - 1) / 2 * ((m_k + 1) / 2)); }

void Sorter::sorter(Ct& ctxt, Ct& ctxt_out, SignConfig& Cfg) {
    assert((m_k == 2 || m_k == 3 || m_k == 5) && "Only k=2,3,5 is supported");
    if (!runStages(ctxt, 0, stageCount(), Cfg)) return;
    ctxt_out = ctxt;
    std::cout << "Level of output: " << ctxt->GetLevel() << std::endl;
    PRINT_PT(m_enc, ctxt_out);
}

bool Sorter::runStages(Ct& ctxt, int first, int last, SignConfig& Cfg) {
    constexpr bool verbose = false;
    const int depth = Cfg.multDepth;
    const long k = m_k;
    Ct fix, c1, c2;
    for (int stage = first; stage < last; ++stage) {
        std::cout << " == stage " << stage << " == " << std::endl;
        const auto [m, logDist, slope] = sortType((int)m_k, (int)m_M, stage);
        const long shift = getRotateDistance(m_k, logDist, slope);
        std::cout << m_k << " " << m_M << " " << m << " " << logDist << " " << slope << std::endl;
        std::cout << "Level " << m_level[m_k] << "\n";
        auto idx = genIndices(m_numSlots, m_k, m_M, m, logDist, slope);
        auto boot = [&](Ct& c, int lvl) { checkLevelAndBoot(c, lvl, depth, verbose); };
        if (slope == 0) {  // merge stage: k-sorters
            boot(ctxt, m_level[k]);
            if (k == 5) {
                comparisonForSort2(ctxt, idx, logDist, slope, c1, c2, fix, Cfg);
                checkLevelAndBoot2(c1, c2, m_level[k], depth, verbose);
                runFiveSorter(ctxt, idx, shift, c1, c2, ctxt);
            } else {
                comparisonForSort(ctxt, idx, logDist, slope, c1, fix, Cfg);
                boot(c1, m_level[k]);
                if (k == 2)
                    runTwoSorter(ctxt, idx, shift, c1, ctxt);
                else
                    runThreeSorter(ctxt, idx, shift, c1, ctxt);
            }
        } else if (slope == k / 2 + 1) {  // middle stage of odd k: (k-1)-sorters
            boot(ctxt, m_level[k - 1]);
            if (k == 3) {
                comparisonForSort(ctxt, idx, logDist, slope, c1, fix, Cfg);
                boot(c1, m_level[k - 1]);
                runTwoSorter(ctxt, idx, shift, c1, ctxt);
            } else {
                comparisonForSort2(ctxt, idx, logDist, slope, c1, c2, fix, Cfg);
                boot(ctxt, m_level[k - 1]);
                checkLevelAndBoot2(c1, c2, m_level[k - 1], depth, verbose);
                runFourSorter(ctxt, idx, shift, c1, c2, ctxt);
            }
            ctxt = m_cc->EvalAdd(ctxt, fix);
        } else if (k == 5 && slope == 1) {
            boot(ctxt, m_level[5]);
            comparisonForSort2(ctxt, idx, logDist, slope, c1, c2, fix, Cfg);
            checkLevelAndBoot2(c1, c2, m_level[5], depth, verbose);
            run2345Sorter(ctxt, idx, shift, c1, c2, ctxt);
            ctxt = m_cc->EvalAdd(ctxt, fix);
        } else if ((k == 5 && slope == 2) || (k == 3 && slope == 1)) {  // 2- and 3-sorters
            Ct two, three;
            boot(ctxt, m_level[3]);
            comparisonForSort(ctxt, idx, logDist, slope, c1, fix, Cfg);
            boot(c1, m_level[2]);
            runTwoSorter(ctxt, idx, shift, c1, two);
            boot(c1, m_level[3]);
            runThreeSorter(ctxt, idx, shift, c1, three);
            ctxt = m_cc->EvalAdd(m_cc->EvalAdd(two, fix), three);
        } else if (k == 2 && slope == 1) {
            Ct two;
            boot(ctxt, m_level[2]);
            comparisonForSort(ctxt, idx, logDist, slope, c1, fix, Cfg);
            boot(c1, m_level[2]);
            runTwoSorter(ctxt, idx, shift, c1, two);
            ctxt = m_cc->EvalAdd(two, fix);
        } else {
            std::cout << "[Sorter::Sorter] ERROR : no matching k & slope" << std::endl;
            return false;
        }
        std::cout << " == End stage " << stage << " == " << std::endl;
        if (std::getenv("SFHE_KWAY_DEBUG") && m_privateKey) debugWithSk(ctxt, 8, "stage " + std::to_string(stage));
    }
    return true;
}

}  // namespace kwaySort
