// k-way schedule / slot-label dump (test infrastructure).  Built twice by
// oracle/Makefile `ref`: against the REFERENCE's src/k-way/Masking.cpp
// (compiled where it lies) and against the engine's algo/k-way/Masking.cpp;
// tests/test_kway.py requires identical output.  For k in {2,3,5} and every
// stage of every k^M <= 1024 network: sortType, getRotateDistance and the
// genIndices labels of all k^M slots, plus genMask of every (size, pos) label.
#include <cstdio>
#include <vector>

#include "Masking.h"

int main() {
    for (int k : {2, 3, 5}) {
        int total = 1;
        for (int M = 1; total * k <= 1024; ++M) {
            total *= k;
            const int stages = M + M * (M - 1) / 2 * ((k + 1) / 2);
            for (int stage = 0; stage < stages; ++stage) {
                auto [m, logDist, slope] = kwaySort::sortType(k, M, stage);
                std::printf("k=%d M=%d stage=%d m=%d logDist=%d slope=%d rot=%ld\n", k, M, stage, m, logDist, slope,
                            kwaySort::getRotateDistance(k, logDist, slope));
                auto idx = kwaySort::genIndices(total, k, M, m, logDist, slope);
                for (int row = 0; row < 2; ++row) {
                    for (int v : idx[row]) std::printf("%d ", v);
                    std::printf("\n");
                }
                for (int size = 1; size <= k; ++size)
                    for (int pos = 1; pos <= size; ++pos) {
                        std::vector<double> mask;
                        kwaySort::genMask(idx, size, pos, mask);
                        int ones = 0;
                        for (double x : mask) ones += x != 0.0;
                        std::printf("mask %d %d %d\n", size, pos, ones);
                    }
            }
        }
    }
    return 0;
}
