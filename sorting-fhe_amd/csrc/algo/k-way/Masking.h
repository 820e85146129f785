// k-way sorting network: stage schedule and slot labelling (public surface of
// the reference's src/k-way/Masking.h:1-32; HKC+21 k-way network).
//
// A stage of the network over k^M slots is described by (m, logDist, slope)
// (sortType); genIndices labels every slot with the size of the sub-sorter it
// belongs to in that stage and its 1-based position inside it; masks select
// the slots with a given (size, position) label.
#pragma once

#include <algorithm>
#include <cmath>
#include <tuple>
#include <vector>

#include "openfhe.h"

using namespace lbcrypto;

namespace kwaySort {

void printMask(const std::vector<double>& mask, long start = 0, long end = -1);
void printVector(const std::vector<int>& mask, long start = 0, long end = -1);

// (m, logDist, slope) of network stage `stage` (Masking.cpp:26-47)
std::tuple<int, int, int> sortType(int k, int M, int stage);

// labels[0][slot] = sub-sorter size, labels[1][slot] = position (1-based);
// 0 / 0 for slots no sub-sorter touches (Masking.cpp:49-144)
std::vector<std::vector<int>> genIndices(long numSlots, long k, long M, long m, long dist, long slope);

// mask[slot] = 1 where the label is (index0, index1); other entries are left
// as they are (Masking.cpp:146-156)
void genMask(const std::vector<std::vector<int>>& indices, long index0, long index1, std::vector<double>& mask);

// slot distance between consecutive members of a stage's sub-sorters
// (Masking.cpp:158-167)
long getRotateDistance(long k, long logDist, long slope);

}  // namespace kwaySort
