// k-way network schedule and slot labelling (reference src/k-way/Masking.cpp).
#include "Masking.h"

#include <cstdint>
#include <iostream>

namespace kwaySort {

namespace {

long ipow(long b, long e) {
    long r = 1;
    while (e-- > 0) r *= b;
    return r;
}

}  // namespace

void printMask(const std::vector<double>& mask, long start, long end) {
    if (end == -1) end = (long)mask.size();
    for (long i = start; i < end; ++i) std::cout << mask[i] << " ";
    std::cout << std::endl;
}

void printVector(const std::vector<int>& mask, long start, long end) {
    if (end == -1) end = (long)mask.size();
    for (long i = start; i < end; ++i) std::cout << mask[i] << " ";
    std::cout << std::endl;
}

// Stages come in rounds r = 0, 1, ...: round r is one "slope 0" merge stage
// followed by r * ceil(k/2) cleanup stages; f(r) = r + r(r-1)/2 ceil(k/2)
// stages precede round r.  Inside the round, cleanup stage n >= 1 works at
// level m = ceil(n / ceil(k/2)) with slope 1 + (n - 1) mod ceil(k/2).
std::tuple<int, int, int> sortType(int k, int /*M*/, int stage) {
    const int half = (k + 1) / 2;
    auto first = [half](int r) { return r + r * (r - 1) / 2 * half; };
    int r = 0;
    while (first(r + 1) <= stage) ++r;
    const int n = stage - first(r);
    const int m = (n + half - 1) / half;
    const int slope = n == 0 ? 0 : (n - 1) % half + 1;
    return {m, r - m, slope};
}

// Every block of dist * k^(m+1) slots is a k^m x k grid of dist-wide cells,
// cell (row, col) at slots start + dist (row + k^m col) for slope 0 and
// start + dist (col + k row) otherwise.
//  * slope 0: each grid row is one k-sorter, position = col + 1;
//  * slope > k/2 (odd k, the middle stage): (k-1)-sorters over the runs of
//    k-1 cells that start at col k - k/2 of each of the first k^m - 1 rows;
//  * otherwise: sorters along the diagonals (row, col) -> (row + 1,
//    col - slope) that start on row 0 at col >= slope or on a middle row at
//    col >= k - slope; a diagonal of L cells is an L-sorter, position = the
//    cell's rank along it.  (No two diagonals meet: a start on row s > 0 would
//    need an earlier one from col >= k.)
std::vector<std::vector<int>> genIndices(long numSlots, long k, long M, long m, long logDist, long slope) {
    std::vector<std::vector<int>> lab(2, std::vector<int>(numSlots, 0));
    const long rows = ipow(k, m), dist = ipow(k, logDist), total = ipow(k, M);
    auto mark = [&](long slot0, int size, int pos) {
        for (long d = 0; d < dist; ++d) {
            lab[0][slot0 + d] = size;
            lab[1][slot0 + d] = pos;
        }
    };
    for (long start = 0; start < total; start += dist * rows * k) {
        if (slope == 0) {
            for (long row = 0; row < rows; ++row)
                for (long col = 0; col < k; ++col) mark(start + dist * (row + rows * col), (int)k, (int)col + 1);
            continue;
        }
        if (slope > k / 2) {
            for (long row = 0; row + 1 < rows; ++row)
                for (long p = 1; p < k; ++p) mark(start + dist * ((k - k / 2) + k * row + p - 1), (int)k - 1, (int)p);
            continue;
        }
        auto diagonal = [&](long row, long col) {
            std::vector<long> cells;
            for (; row < rows && col >= 0; ++row, col -= slope) cells.push_back(start + dist * (col + k * row));
            for (size_t j = 0; j < cells.size(); ++j) mark(cells[j], (int)cells.size(), (int)j + 1);
        };
        for (long col = slope; col < k; ++col) diagonal(0, col);
        for (long row = 1; row + 1 < rows; ++row)
            for (long col = k - slope; col < k; ++col) diagonal(row, col);
    }
    return lab;
}

void genMask(const std::vector<std::vector<int>>& indices, long index0, long index1, std::vector<double>& mask) {
    const size_t n = indices[0].size();
    mask.resize(n, 0.0);
    for (size_t i = 0; i < n; ++i)
        if (indices[0][i] == index0 && indices[1][i] == index1) mask[i] = 1.0;
}

long getRotateDistance(long k, long logDist, long slope) {
    const long dist = ipow(k, logDist);
    return (slope == 0 || slope == k / 2 + 1) ? dist : dist * (k - slope);
}

}  // namespace kwaySort
