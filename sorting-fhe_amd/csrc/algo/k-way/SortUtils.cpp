// k-way comparator networks and slot matching (reference
// src/k-way/SortUtils.cpp).
#include "SortUtils.h"

namespace kwaySort {

using Ct = Ciphertext<DCRTPoly>;

Plaintext SortUtils::labelMask(const std::vector<std::vector<int>>& indices, std::initializer_list<int> sizes,
                               int pos) {
    std::vector<double> m(m_numSlots, 0.0);
    for (long i = 0; i < m_numSlots; ++i)
        if (indices[1][i] == pos)
            for (int s : sizes)
                if (indices[0][i] == s) m[i] = 1.0;
    return m_cc->MakeCKKSPackedPlaintext(m);
}

void SortUtils::fcnL(Ct& ctxt1, Ct& ctxt2, Ct& comp, Ct& ctxt_out) {
    ctxt_out = m_cc->EvalAdd(m_cc->EvalMult(m_cc->EvalSub(ctxt1, ctxt2), comp), ctxt2);
}

void SortUtils::compareMax(Ct& ctxt1, Ct& ctxt2, Ct& comp, Ct& ctxt_out) { fcnL(ctxt1, ctxt2, comp, ctxt_out); }

void SortUtils::compareMin(Ct& ctxt1, Ct& ctxt2, Ct& comp, Ct& ctxt_out) { fcnL(ctxt2, ctxt1, comp, ctxt_out); }

void SortUtils::twoSorter(Ct* ctxt, Ct& comp, Ct* ctxt_out) { twoSorter(ctxt[0], ctxt[1], comp, ctxt_out); }

void SortUtils::twoSorter(Ct& ctxt0, Ct& ctxt1, Ct& comp, Ct* ctxt_out) {
    fcnL(ctxt0, ctxt1, comp, ctxt_out[1]);  // max
    ctxt_out[0] = m_cc->EvalSub(m_cc->EvalAdd(ctxt0, ctxt1), ctxt_out[1]);
}

// min / max of {a, b} against c: the bits [min(a,b) > c, max(a,b) > c] are
// the 2-sorted [a>c, b>c] under the a>b bit
void SortUtils::threeSorter(Ct* x, Ct* c, Ct* out) {
    Ct ab[2], abVsC[2];
    twoSorter(x[0], x[1], c[0], ab);
    twoSorter(c[1], c[2], c[0], abVsC);
    compareMax(ab[1], x[2], abVsC[1], out[2]);
    compareMin(ab[0], x[2], abVsC[0], out[0]);
    out[1] = m_cc->EvalSub(m_cc->EvalSub(m_cc->EvalAdd(m_cc->EvalAdd(x[0], x[1]), x[2]), out[0]), out[2]);
}

// two 2-sorted pairs (m1, M1), (m2, M2) merged; the cross bits come from
// re-sorting the raw bits with the pairs' own comparison bits
void SortUtils::fourSorter(Ct* x, Ct* c, Ct* out) {
    // c = [a>b, a>c, a>d, b>c, b>d, c>d]
    Ct p1[2], p2[2];
    twoSorter(x[0], x[1], c[0], p1);
    twoSorter(x[2], x[3], c[5], p2);
    Ct p1VsC[2], p1VsD[2];
    twoSorter(c[1], c[3], c[0], p1VsC);  // [m1 > c, M1 > c]
    twoSorter(c[2], c[4], c[0], p1VsD);  // [m1 > d, M1 > d]
    Ct bigVs2[2], smallVs2[2];
    twoSorter(p1VsC[1], p1VsD[1], c[5], bigVs2);    // [M1 > m2, M1 > M2]
    twoSorter(p1VsC[0], p1VsD[0], c[5], smallVs2);  // [m1 > m2, m1 > M2]
    compareMax(p1[1], p2[1], bigVs2[1], out[3]);
    Ct ifBig1, ifBig2;
    compareMax(p1[0], p2[1], smallVs2[1], ifBig1);  // second largest when M1 is the largest
    compareMax(p1[1], p2[0], bigVs2[0], ifBig2);    // ... when M2 is
    compareMax(ifBig1, ifBig2, bigVs2[1], out[2]);
    compareMin(p1[0], p2[0], smallVs2[0], out[0]);
    Ct rest = m_cc->EvalAdd(m_cc->EvalAdd(x[0], x[1]), m_cc->EvalAdd(x[2], x[3]));
    out[1] = m_cc->EvalSub(m_cc->EvalSub(m_cc->EvalSub(rest, out[0]), out[2]), out[3]);
}

// a 3-sorted triple (m, mid, M) and a 2-sorted pair (m', M') merged
void SortUtils::fiveSorter(Ct* x, Ct* c, Ct* out) {
    // c = [a>b a>c a>d a>e b>c b>d b>e c>d c>e d>e]
    Ct tri[3] = {x[0], x[1], x[2]};
    Ct triBits[3] = {c[0], c[1], c[4]};
    Ct t[3];
    threeSorter(tri, triBits, t);
    Ct pr[2];
    twoSorter(x[3], x[4], c[9], pr);
    Ct vsD[3] = {c[2], c[5], c[7]}, vsE[3] = {c[3], c[6], c[8]};
    Ct tVsD[3], tVsE[3];  // [m > d, mid > d, M > d], the same against e
    threeSorter(vsD, triBits, tVsD);
    threeSorter(vsE, triBits, tVsE);
    Ct hiVs[2], midVs[2], loVs[2];  // each: [x > m', x > M']
    twoSorter(tVsD[2], tVsE[2], c[9], hiVs);
    twoSorter(tVsD[1], tVsE[1], c[9], midVs);
    twoSorter(tVsD[0], tVsE[0], c[9], loVs);
    compareMax(t[2], pr[1], hiVs[1], out[4]);
    compareMin(t[0], pr[0], loVs[0], out[0]);
    Ct a, b;
    compareMax(t[1], pr[1], midVs[1], a);  // fourth when M is the largest
    compareMax(t[2], pr[0], hiVs[0], b);   // fourth when M' is
    compareMax(a, b, hiVs[1], out[3]);
    compareMin(t[1], pr[0], midVs[0], a);  // second when m' is the smallest
    compareMin(t[0], pr[1], loVs[1], b);   // second when m is
    compareMin(a, b, loVs[0], out[1]);
    Ct sum = m_cc->EvalAdd(m_cc->EvalAdd(m_cc->EvalAdd(x[0], x[1]), m_cc->EvalAdd(x[2], x[3])), x[4]);
    for (int i : {0, 1, 3, 4}) sum = m_cc->EvalSub(sum, out[i]);
    out[2] = sum;
}

void SortUtils::slotMatching2(Ct& ctxt, Ct& ctxt_comp, std::vector<std::vector<int>>&, long shift, Ct* ctxt_out,
                              Ct& ctxt_comp_out) {
    ctxt_out[0] = ctxt;
    leftRotate(ctxt, shift, ctxt_out[1]);
    ctxt_comp_out = ctxt_comp;
}

// The stage's comparison ciphertext holds, in each member's slot, that member
// against the member `shift` slots before it; the other pairs are rotations of
// it, flipped (1 - c) where the pair is seen from the other side.
void SortUtils::slotMatching3(Ct& ctxt, Ct& ctxt_comp, std::vector<std::vector<int>>& indices, long shift,
                              Ct* ctxt_out, Ct* ctxt_comp_out) {
    Plaintext head = labelMask(indices, {3}, 1);
    for (int i = 0; i < 3; ++i) leftRotate(ctxt, i * shift, ctxt_out[i]);
    ctxt_comp_out[1] = ctxt_comp;
    leftRotate(ctxt_comp, shift, ctxt_comp_out[0]);
    leftRotate(ctxt_comp, 2 * shift, ctxt_comp_out[2]);
    flipCtxt(ctxt_comp_out[0], head);
    flipCtxt(ctxt_comp_out[2], head);
}

void SortUtils::slotMatching4(Ct& ctxt, Ct& ctxt_comp1, Ct& ctxt_comp2, std::vector<std::vector<int>>& indices,
                              long shift, Ct* ctxt_arr, Ct* ctxt_comp_arr) {
    // (the reference also masks the comparison ciphertexts with all four
    // position masks and then overwrites the products: not repeated here)
    Plaintext head = labelMask(indices, {4}, 1);
    ctxt_comp_arr[2] = ctxt_comp1;
    leftRotate(ctxt_comp1, shift, ctxt_comp_arr[0]);
    leftRotate(ctxt_comp1, 2 * shift, ctxt_comp_arr[3]);
    leftRotate(ctxt_comp1, 3 * shift, ctxt_comp_arr[5]);
    ctxt_comp_arr[1] = ctxt_comp2;
    leftRotate(ctxt_comp2, shift, ctxt_comp_arr[4]);
    for (int i : {0, 3, 5}) flipCtxt(ctxt_comp_arr[i], head);
    for (int i = 0; i < 4; ++i) {
        leftRotate(ctxt, i * shift, ctxt_arr[i]);
        ctxt_arr[i] = m_cc->EvalMult(ctxt_arr[i], head);
    }
}

void SortUtils::slotMatching5(Ct& ctxt, Ct& ctxt_comp1, Ct& ctxt_comp2, std::vector<std::vector<int>>& indices,
                              long shift, Ct* ctxt_arr, Ct* ctxt_comp_arr) {
    Plaintext head = labelMask(indices, {5}, 1);
    for (int i = 0; i < 5; ++i) leftRotate(ctxt, i * shift, ctxt_arr[i]);
    // comp1 rotated by 0..4 shifts: a>e, a>b, b>c, c>d, d>e; comp2: a>d, b>e, a>c, b>d, c>e
    const int from1[5] = {3, 0, 4, 7, 9}, from2[5] = {2, 6, 1, 5, 8};
    for (int i = 0; i < 5; ++i) {
        leftRotate(ctxt_comp1, i * shift, ctxt_comp_arr[from1[i]]);
        leftRotate(ctxt_comp2, i * shift, ctxt_comp_arr[from2[i]]);
    }
    for (int i : {0, 1, 4, 5, 7, 8, 9}) flipCtxt(ctxt_comp_arr[i], head);
}

// sub-sorters of sizes 2..5 side by side (k = 5, slope 1): each pair's bit is
// assembled from whichever comparison ciphertext holds it for that size
void SortUtils::slotMatching2345(Ct& ctxt, Ct& ctxt_comp1, Ct& ctxt_comp2, std::vector<std::vector<int>>& indices,
                                 long shift, Ct* ctxt_arr, Ct* ctxt_comp_arr) {
    for (int i = 0; i < 5; ++i) leftRotate(ctxt, i * shift, ctxt_arr[i]);
    Plaintext m2345 = labelMask(indices, {2, 3, 4, 5}, 1), m345 = labelMask(indices, {3, 4, 5}, 1),
              m45 = labelMask(indices, {4, 5}, 1), m3 = labelMask(indices, {3}, 1), m4 = labelMask(indices, {4}, 1),
              m5 = labelMask(indices, {5}, 1);
    // rotate `src` by `r` shifts, keep `keep`, optionally flip there
    auto part = [&](Ct& src, long r, Plaintext& keep, bool flip) {
        Ct t;
        leftRotate(src, r * shift, t);
        t = m_cc->EvalMult(t, keep);
        if (flip) flipCtxt(t, keep);
        return t;
    };
    leftRotate(ctxt_comp1, shift, ctxt_comp_arr[0]);  // a>b
    flipCtxt(ctxt_comp_arr[0], m2345);
    ctxt_comp_arr[1] = m_cc->EvalAdd(m_cc->EvalMult(ctxt_comp1, m3), part(ctxt_comp2, 2, m45, true));  // a>c
    ctxt_comp_arr[2] = m_cc->EvalAdd(m_cc->EvalMult(ctxt_comp1, m4), m_cc->EvalMult(ctxt_comp2, m5));  // a>d
    ctxt_comp_arr[3] = m_cc->EvalMult(ctxt_comp1, m5);                                                  // a>e
    ctxt_comp_arr[4] = part(ctxt_comp1, 2, m345, true);                                                 // b>c
    ctxt_comp_arr[5] = part(ctxt_comp2, 3, m45, true);                                                  // b>d
    ctxt_comp_arr[6] = part(ctxt_comp2, 1, m5, false);                                                  // b>e
    ctxt_comp_arr[7] = part(ctxt_comp1, 3, m45, true);                                                  // c>d
    ctxt_comp_arr[8] = part(ctxt_comp2, 4, m5, true);                                                   // c>e
    ctxt_comp_arr[9] = part(ctxt_comp1, 4, m5, true);                                                   // d>e
}

void SortUtils::slotAssemble(Ct* ctxt_sort, long num, long shift, Ct& ctxt_out) {
    ctxt_out = ctxt_sort[0];
    for (long i = 1; i < num; ++i) {
        Ct r;
        rightRotate(ctxt_sort[i], i * shift, r);
        ctxt_out = m_cc->EvalAdd(ctxt_out, r);
    }
}

}  // namespace kwaySort
